# r6ae: 5-minute sustained C2 window and a 2-minute C4 window at the final
# library (progress lines to the .err files every 30 s)
set -o pipefail
mkdir -p gpurun_out
md5sum metal-renderer_amd/lib/libmrt.so
timeout -k 10 420 python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --sustain 300 > gpurun_out/r6ae_c2_5min.json 2> gpurun_out/r6ae_c2_5min.err || exit $?
timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c4 --steps 30 --warmup 2 --sustain 120 > gpurun_out/r6ae_c4_2min.json 2> gpurun_out/r6ae_c4_2min.err
rc=$?; for f in gpurun_out/r6ae_c2_5min.json gpurun_out/r6ae_c4_2min.json; do python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['sustained'])"; done; exit $rc
