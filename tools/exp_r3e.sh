# r3: dual-query path kernel (path2) A/B on C4 and C3, and its parity tests
B4="python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline"
B3="python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline"
T="python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread"
tools/gpu_run.sh \
 "tests_p2:600:$T -k 'configs or parity or scale'" \
 "tests_p2_g:600:MRT_MODE=0 $T tests/test_gpu_configs.py tests/test_gpu_scale.py" \
 "e_p1:120:MRT_PATH2=0 $B4" "e_p2:120:$B4" "e_p2g:120:MRT_MODE=0 $B4" "e_p1g:120:MRT_PATH2=0 MRT_MODE=0 $B4" \
 "e_p1b:120:MRT_PATH2=0 $B4" "e_p2b:120:$B4" "e_p2gb:120:MRT_MODE=0 $B4" \
 "e3_p1:120:MRT_PATH2=0 $B3" "e3_p2:120:$B3" "e3_p2g:120:MRT_MODE=0 $B3"
