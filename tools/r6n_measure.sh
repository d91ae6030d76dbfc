# r6n: session restart: GPU suite on the spill-trimmed build (mbcnt lane
# prefix, host-computed cos_min^2), A/B against HEAD's library, C4 line, the
# occlusion-walk ablation with convex occluders, the DRAM-side activity of C2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r6n_gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r6n_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/lib_sweep.sh "--sustain 0" c2 c4 -- libmrt.so libmrt_head.so libmrt.so libmrt_head.so > gpurun_out/r6n_ab.log 2>&1 || exit $?
cat gpurun_out/r6n_ab.log
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_DEBUG=32" "MRT_DEBUG=96" > gpurun_out/r6n_ablation.log 2>&1 || exit $?
bash tools/env_sweep.sh "--config c2i --steps 20 --no-image-check" "MRT_DEBUG=0" "MRT_DEBUG=256" "MRT_DEBUG=0" "MRT_DEBUG=256" >> gpurun_out/r6n_ablation.log 2>&1 || exit $?
cat gpurun_out/r6n_ablation.log
timeout -k 10 240 python3 tools/hbm_activity.py gpurun_out/r6n_hbm_c2.json -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --sustain 15 > gpurun_out/r6n_hbm_c2.log 2>&1
rc=$?; grep -v "calibration copy" gpurun_out/r6n_hbm_c2.log | tail -30; exit $rc
