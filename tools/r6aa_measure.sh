# r6aa: 8-bit quantised global nodes in the path kernel (libmrt_qn.so,
# MRT_QNODES=1) against the fp32 nodes: C4 / C3 / C5 share alternating, then
# the configuration parity tests (precise full-size C4 / C5 / C3 bitwise
# against the oracle) on the variant
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--sustain 0 --steps 12 --warmup 2 --no-image-check" c4 -- libmrt.so libmrt_qn.so libmrt.so libmrt_qn.so > gpurun_out/r6aa_ab.log 2>&1 || exit $?
cat gpurun_out/r6aa_ab.log
bash tools/lib_sweep.sh "--sustain 0 --steps 4 --warmup 1 --shard-of 8" c5 -- libmrt.so libmrt_qn.so >> gpurun_out/r6aa_ab.log 2>&1 || exit $?
bash tools/lib_sweep.sh "--sustain 0 --steps 4 --warmup 1" c3 -- libmrt.so libmrt_qn.so >> gpurun_out/r6aa_ab.log 2>&1 || exit $?
tail -4 gpurun_out/r6aa_ab.log
MRT_LIB=metal-renderer_amd/lib/libmrt_qn.so timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scale.py -q -x --timeout 600 --timeout-method thread > gpurun_out/r6aa_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6aa_tests.log; exit $rc
