# r3: full GPU suite at the current library; bench lines c2 / c4 / 1/8 share; 2-rank host rehearsal
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh "p_tests:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "p_c2:100:$B --config c2" "p_s8:100:$B --config c2 --shard-of 8" "p_c4:150:$B --config c4" \
 "p_g2:200:python3 bench.py --gpus 2 --exchange-backend host --check-image --steps 4 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "p_c2_noshadow:100:MRT_DEBUG=1 $B --config c2" "p_c2b:100:$B --config c2"
PASSES="valu sq1" timeout -k 10 300 bash tools/pmc_probe.sh r3p c4 > gpurun_out/probe_r3p_c4.txt 2>&1; tail -25 gpurun_out/probe_r3p_c4.txt
