# r6e: occlusion-walk ablation bound on C2 (MRT_DEBUG 32: no occlusion walk of
# the light samples; 96: nor of the last bounce's light hit; wrong images, the
# path work unchanged), alternating, then the DRAM-side activity of C2 and C4
set -o pipefail
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_DEBUG=32" "MRT_DEBUG=96" "MRT_DEBUG=0" "MRT_DEBUG=32" "MRT_DEBUG=96" > gpurun_out/r6e_ablation.log 2>&1 && cat gpurun_out/r6e_ablation.log && \
timeout -k 10 240 python3 tools/hbm_activity.py gpurun_out/r6e_hbm_c2.json -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --sustain 15 > gpurun_out/r6e_hbm_c2.log 2>&1 && \
timeout -k 10 240 python3 tools/hbm_activity.py gpurun_out/r6e_hbm_c4.json -- python3 bench.py --no-cpu-baseline --config c4 --steps 30 --warmup 2 --sustain 15 --no-image-check > gpurun_out/r6e_hbm_c4.log 2>&1; grep -v "calibration copy" gpurun_out/r6e_hbm_c2.log | head -40; grep -v "calibration copy" gpurun_out/r6e_hbm_c4.log | head -40
