# r3 C4 path-kernel A/B: 12-word path state, 6 waves/SIMD, branch-free pushes
B="python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline"
tools/gpu_run.sh \
 "b_base:120:$B" \
 "b_push3:120:MRT_LIB=metal-renderer_amd/lib/libmrt_push3.so $B" \
 "b_w6:120:MRT_LIB=metal-renderer_amd/lib/libmrt_w6.so $B" \
 "b_w6push3:120:MRT_LIB=metal-renderer_amd/lib/libmrt_w6push3.so $B" \
 "b_base2:120:$B" \
 "b_push3_2:120:MRT_LIB=metal-renderer_amd/lib/libmrt_push3.so $B" \
 "b_w6_2:120:MRT_LIB=metal-renderer_amd/lib/libmrt_w6.so $B" \
 "b_w6push3_2:120:MRT_LIB=metal-renderer_amd/lib/libmrt_w6push3.so $B" \
 "b_c3:120:python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline" \
 "b_c3_w6:120:MRT_LIB=metal-renderer_amd/lib/libmrt_w6.so python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline" \
 "c4cpu:300:python3 bench.py --config c4 --steps 2 --warmup 1" \
 "tests:600:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -k 'configs or parity'"
