set -o pipefail
timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/r6b_c2.json 2> gpurun_out/r6b_c2.err && \
timeout -k 10 200 python3 bench.py --no-cpu-baseline --config c4 --steps 30 --warmup 3 --sustain 0 > gpurun_out/r6b_c4.json 2> gpurun_out/r6b_c4.err && \
timeout -k 10 240 python3 tools/hbm_activity.py gpurun_out/r6b_hbm_c2.json -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --sustain 15 > gpurun_out/r6b_hbm.log 2>&1
