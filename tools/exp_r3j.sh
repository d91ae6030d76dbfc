# r3: device spans; leaf-loop slack and service threshold with path slack 12;
# the path kernel on C2 with slack
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
 "j_tests:300:python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'spans or pipelined or in_flight'" \
 "j_sweep:900:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 -- libmrt.so libmrt_lf2.so libmrt_lf4.so libmrt_lf8.so libmrt_sv16.so libmrt_sv32.so libmrt.so libmrt_lf4.so" \
 "j_c2path:100:MRT_KERNEL=path $B --config c2" "j_c2:100:$B --config c2" "j_s8:100:$B --config c2 --shard-of 8"
