# r6p: where the C2 shadow query's time goes now (ablation bits, wrong
# images): 32 no occlusion query at all, 512 no convex-solid test, 1024 no
# other-light test, 1536 neither, 1 no shadow ray at all
set -o pipefail
mkdir -p gpurun_out
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_DEBUG=32" "MRT_DEBUG=512" "MRT_DEBUG=1024" "MRT_DEBUG=1536" "MRT_DEBUG=1" "MRT_DEBUG=0" "MRT_DEBUG=512" > gpurun_out/r6p_ablation.log 2>&1
rc=$?; cat gpurun_out/r6p_ablation.log; exit $rc
