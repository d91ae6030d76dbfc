# r3: shadow-query share of C4 (ablation), NT radiance for the stream kernel (C2)
B4="python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline"
B2="python3 bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline"
B3="python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh \
 "d_c4:120:$B4" "d_c4_noshadow:120:MRT_DEBUG=1 $B4" \
 "d_c3:120:$B3" "d_c3_noshadow:120:MRT_DEBUG=1 $B3" \
 "d_c2:120:$B2" "d_c2_ntw:120:MRT_LIB=metal-renderer_amd/lib/libmrt_ntw.so $B2" \
 "d_c2b:120:$B2" "d_c2_ntwb:120:MRT_LIB=metal-renderer_amd/lib/libmrt_ntw.so $B2" \
 "d_s8:120:$B2 --shard-of 8" "d_s8_ntw:120:MRT_LIB=metal-renderer_amd/lib/libmrt_ntw.so $B2 --shard-of 8"
