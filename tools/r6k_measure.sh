# r6k: last-bounce occlusion query through the convex solids (origin primitive
# in queue plane 1 .w): A/B against the previous library, then the GPU suite
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_prev.so libmrt.so libmrt_prev.so > gpurun_out/r6k_ab.log 2>&1; cat gpurun_out/r6k_ab.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6k_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6k_gpu_tests.log; exit $rc
