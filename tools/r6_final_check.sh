# r6 final check at HEAD: the GPU suite, smoke() and the driver's default line
set -o pipefail
mkdir -p gpurun_out
md5sum metal-renderer_amd/lib/libmrt.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6_final_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r6_final_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6_final_bench.json 2> gpurun_out/r6_final_bench.log
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r6_final_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('same_library'))"; exit $rc
