# r6o: lights_occlude over the lights other than the target (one light test
# per C2 shadow ray instead of two) + the spill-trimmed stream kernel: GPU
# suite, then C2 / L=5 / C4 alternating against HEAD's library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6o_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6o_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_head.so libmrt.so libmrt_head.so libmrt.so libmrt_head.so > gpurun_out/r6o_ab.log 2>&1
rc=$?; cat gpurun_out/r6o_ab.log; exit $rc
