# r6u: per-frame cadence (c2i) with the accumulates on the render streams
# (chained by events, MRT_ACC_RENDER=1) at 2 and 3 render streams, against
# the main-stream accumulate (default); batched C2 beside it
set -o pipefail
mkdir -p gpurun_out
bash tools/env_sweep.sh "--config c2i --steps 20 --no-image-check" "MRT_DEBUG=0" "MRT_ACC_RENDER=1" "MRT_ACC_RENDER=1 MRT_INFLIGHT=3" "MRT_INFLIGHT=3" "MRT_DEBUG=0" "MRT_ACC_RENDER=1" "MRT_ACC_RENDER=1 MRT_INFLIGHT=3" > gpurun_out/r6u_c2i.log 2>&1 || exit $?
cat gpurun_out/r6u_c2i.log
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_ACC_RENDER=1" "MRT_ACC_RENDER=1 MRT_INFLIGHT=3" > gpurun_out/r6u_c2.log 2>&1
rc=$?; cat gpurun_out/r6u_c2.log
timeout -k 10 300 env MRT_DIAG=1 MRT_ACC_RENDER=1 MRT_INFLIGHT=3 python -u -m pytest tests/test_gpu_cadence.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1
rc2=$?; tail -3 gpurun_out/r6u_tests.log; exit $((rc | rc2))
