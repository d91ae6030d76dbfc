# r6i: convex occluders with the exhaustive per-solid fallback (no occluder-tree
# walk on the convex path): C2 A/B alternating, then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
bash tools/env_sweep.sh "--sustain 0" "MRT_CONVEX=1" "MRT_CONVEX=0" "MRT_CONVEX=1" "MRT_CONVEX=0" > gpurun_out/r6i_ab.log 2>&1; cat gpurun_out/r6i_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6i_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6i_gpu_tests.log; exit $rc
