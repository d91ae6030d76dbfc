# r3: path slack 12 + pipelined tile shares: full GPU suite, then A/B benches
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
 "i_tests:900:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "i_s8:100:$B --config c2 --shard-of 8" "i_s8_inf1:100:MRT_INFLIGHT=1 $B --config c2 --shard-of 8" \
 "i_s8b:100:$B --config c2 --shard-of 8" "i_s8_inf1b:100:MRT_INFLIGHT=1 $B --config c2 --shard-of 8" \
 "i_s4:100:$B --config c2 --shard-of 4" "i_s2:100:$B --config c2 --shard-of 2" \
 "i_c2:100:$B --config c2" "i_c4:150:$B --config c4" "i_c3:300:python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --config c3" \
 "i_g2:200:python3 bench.py --gpus 2 --exchange-backend host --check-image --steps 2 --warmup 1 --no-cpu-baseline"
