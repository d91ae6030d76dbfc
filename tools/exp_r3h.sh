# r3: path-kernel traversal slack sweep (MRT_PATH_SLACK)
export TMPDIR=/tmp
tools/gpu_run.sh \
 "h_sweep:900:bash tools/lib_sweep.sh '--steps 3 --warmup 1' c4 c3 c3g -- libmrt_ps8.so libmrt_ps12.so libmrt_ps16.so libmrt_ps24.so libmrt_ps32.so libmrt_ps48.so libmrt_ps16.so libmrt_ps24.so" \
 "h_c5:600:bash tools/lib_sweep.sh '--steps 1 --warmup 1 --shard-of 8' c5 -- libmrt.so libmrt_ps16.so libmrt_ps24.so libmrt_ps32.so"
