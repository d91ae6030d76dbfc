# r6r: nearest queries from inside the room without a walk (room_nearest):
# GPU suite, then C2 / L=5 alternating against the r6q library (libmrt_head.so
# = 57c87b6) and with room_nearest off (MRT_DEBUG=2048)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r6r_gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r6r_gpu_tests.log
bash tools/lib_sweep.sh "--sustain 0" c2 c2l5 -- libmrt.so libmrt_head.so libmrt.so libmrt_head.so > gpurun_out/r6r_ab.log 2>&1
cat gpurun_out/r6r_ab.log
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_DEBUG=2048" "MRT_DEBUG=0" "MRT_DEBUG=2048" > gpurun_out/r6r_env.log 2>&1
cat gpurun_out/r6r_env.log; exit $rc
