# r6s: shadow-query cost split at the current library (ablation bits, wrong
# images) and C4's sensitivity to LDS-resident top nodes (MRT_LDS_NODES caps
# the staged BFS prefix: 0 / 5 / 21 vs the default, which fits ~45 nodes)
set -o pipefail
mkdir -p gpurun_out
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_DEBUG=32" "MRT_DEBUG=512" "MRT_DEBUG=4096" "MRT_DEBUG=1024" "MRT_DEBUG=0" "MRT_DEBUG=4096" > gpurun_out/r6s_ablation.log 2>&1 || exit $?
cat gpurun_out/r6s_ablation.log
bash tools/env_sweep.sh "--config c4 --steps 10 --warmup 2 --sustain 0 --no-image-check" "MRT_DEBUG=0" "MRT_LDS_NODES=0" "MRT_LDS_NODES=5" "MRT_LDS_NODES=21" "MRT_DEBUG=0" "MRT_LDS_NODES=21" > gpurun_out/r6s_c4_lds.log 2>&1
rc=$?; cat gpurun_out/r6s_c4_lds.log; exit $rc
