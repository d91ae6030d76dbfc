# r6q: the own-face skip by the face's own normal (d . n >= 1e-3 instead of
# the slab axis >= 0.01): GPU suite, then C2 / L=5 alternating against HEAD's
# library (f57d6cf's predecessor, libmrt_head.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6q_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6q_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_head.so libmrt.so libmrt_head.so libmrt.so libmrt_head.so > gpurun_out/r6q_ab.log 2>&1
rc=$?; cat gpurun_out/r6q_ab.log; exit $rc
