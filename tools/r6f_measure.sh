# r6f: convex occluders A/B on C2 (alternating, MRT_CONVEX=0 turns them off), then the parity suites that cover the stream kernel
set -o pipefail
bash tools/env_sweep.sh "--sustain 0" "MRT_CONVEX=1" "MRT_CONVEX=0" "MRT_CONVEX=1" "MRT_CONVEX=0" > gpurun_out/r6f_ab.log 2>&1 && cat gpurun_out/r6f_ab.log && \
timeout -k 10 900 python3 -u -m pytest -m gpu -x -q --timeout 600 --timeout-method thread tests/test_gpu_configs.py -k "c2_full_size or frames_in_flight" tests/test_gpu_stream.py tests/test_occluders.py tests/test_gpu_parity.py tests/test_gpu_primary.py > gpurun_out/r6f_tests.log 2>&1; tail -5 gpurun_out/r6f_tests.log
