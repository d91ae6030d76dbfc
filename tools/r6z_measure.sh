# r6z: smoke(), the c2i line with the corrected counters, and the headline
# default bench line (the driver's command) on this box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6z_smoke.log 2>&1 || { cat gpurun_out/r6z_smoke.log; exit 1; }
tail -1 gpurun_out/r6z_smoke.log
timeout -k 10 300 python3 bench.py --config c2i --steps 80 --warmup 5 > gpurun_out/r6z_cfg_c2i.json 2> gpurun_out/r6z_cfg_c2i.log || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6z_bench_default.json 2> gpurun_out/r6z_bench_default.log
rc=$?; tail -c 300 gpurun_out/r6z_bench_default.json; exit $rc
