# r6ad: 8-rank rehearsals on one GPU at the final library (host transport:
# RCCL refuses two ranks on one device), each rank's tiles gathered to rank 0
# and its image checked bitwise against a 1-GPU render: C2 fast / precise, C5
# fast; then the driver's default line on this box
set -o pipefail
mkdir -p gpurun_out/r6_multirank
md5sum metal-renderer_amd/lib/libmrt.so
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py --gpus 8 --exchange-backend host --check-image --no-cpu-baseline "$@" > gpurun_out/r6_multirank/$name.json 2> gpurun_out/r6_multirank/$name.log; local rc=$?; python3 -c "import json,sys; d=json.loads(open('gpurun_out/r6_multirank/$name.json').read().strip().splitlines()[-1] if open('gpurun_out/r6_multirank/$name.json').read().strip().startswith('{') and '\n' not in open('gpurun_out/r6_multirank/$name.json').read().strip() else open('gpurun_out/r6_multirank/$name.json').read()); print('$name', d['value'], d.get('image_check'))" 2>/dev/null || tail -3 gpurun_out/r6_multirank/$name.log; return $rc; }
run n8 --steps 3 --warmup 1 || exit $?
run n8p --steps 2 --warmup 1 --precise || exit $?
run n8c5 --config c5 --steps 1 --warmup 1 || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6ad_bench_default.json 2> gpurun_out/r6ad_bench_default.log
rc=$?; python3 -c "import json; d=json.loads(open('gpurun_out/r6ad_bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'])"; exit $rc
