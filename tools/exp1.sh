export TMPDIR=/tmp
B="python3 bench.py --config c2 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh "fulltrace:200:rocprofv3 --kernel-trace -d gpurun_out/full -o run -f csv -- $B --steps 2" \
 "s8_ev_a:100:$B --steps 10 --shard-of 8" "s8_noev_a:100:$B --steps 10 --shard-of 8 --no-kernel-timing" \
 "s8_ev_b:100:$B --steps 10 --shard-of 8" "s8_noev_b:100:$B --steps 10 --shard-of 8 --no-kernel-timing" \
 "full_noev:100:$B --steps 5 --no-kernel-timing" "full_ev:100:$B --steps 5"
