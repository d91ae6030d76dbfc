# r3: pinned asynchronous read-back; pipelined share vs one stream, alternating; leaf slack 8 default
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --config c2 --shard-of 8"
tools/gpu_run.sh "l_a1:100:$B" "l_c1:100:MRT_INFLIGHT=1 $B" "l_a2:100:$B" "l_c2:100:MRT_INFLIGHT=1 $B" \
 "l_a3:100:$B" "l_c3:100:MRT_INFLIGHT=1 $B" \
 "l_full:100:python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --config c2" \
 "l_c4:150:python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --config c4" \
 "l_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
