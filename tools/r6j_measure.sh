# r6j: the whole GPU suite after the zero-slot divisor fix
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6j_gpu_tests.log 2>&1
rc=$?; tail -8 gpurun_out/r6j_gpu_tests.log; exit $rc
