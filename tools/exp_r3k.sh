# r3: pipelined 1/8 share regression hunt (spans on/off, one stream), alternating
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --config c2 --shard-of 8"
tools/gpu_run.sh "k_a1:100:$B" "k_b1:100:MRT_SPANS=0 $B" "k_c1:100:MRT_INFLIGHT=1 $B" \
 "k_a2:100:$B" "k_b2:100:MRT_SPANS=0 $B" "k_c2:100:MRT_INFLIGHT=1 $B" \
 "k_a3:100:$B --steps 40" "k_b3:100:MRT_SPANS=0 $B --steps 40"
tools/gpu_run.sh "k_sweep:900:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 -- libmrt_lf8.so libmrt_lf12.so libmrt_lf16.so libmrt_lf24.so libmrt_lf32.so libmrt_lf8.so libmrt_lf16.so"
