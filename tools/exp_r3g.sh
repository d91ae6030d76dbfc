# r3: traversal slack (interior loop ends with <= K lanes still seeking a leaf)
# and the 1/8-share loss vs shard count / launch size
export TMPDIR=/tmp
B="python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
 "g_sweep:900:bash tools/lib_sweep.sh '--steps 5 --warmup 1' c2 c4 c3 -- libmrt.so libmrt_sl2.so libmrt_sl4.so libmrt_sl8.so libmrt_sl16.so libmrt.so libmrt_sl4.so libmrt_sl8.so" \
 "g_s2:100:$B --shard-of 2" "g_s4:100:$B --shard-of 4" "g_s8:100:$B --shard-of 8" "g_s16:100:$B --shard-of 16" \
 "g_s8b16:100:MRT_BATCH=16 $B --shard-of 8" "g_full:100:$B"
