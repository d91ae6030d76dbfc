# r6 final: the GPU suite and every configuration's bench line at the final
# library (tools/run_configs.sh -> gpurun_out/r6_configs/cfg_<config>.json)
set -o pipefail
mkdir -p gpurun_out
md5sum metal-renderer_amd/lib/libmrt.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6f_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6f_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/run_configs.sh gpurun_out/r6_configs
