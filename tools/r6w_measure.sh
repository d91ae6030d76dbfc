# r6w: DRAM-side traffic of C2 and C4 at the final library (memory-controller
# activity, tools/hbm_activity.py), merged into profiles/pmc_<cfg>.json by
# tools/dram_merge.py on the CPU
set -o pipefail
mkdir -p gpurun_out
md5sum metal-renderer_amd/lib/libmrt.so
timeout -k 10 240 python3 tools/hbm_activity.py gpurun_out/r6w_hbm_c2.json -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --sustain 15 > gpurun_out/r6w_hbm_c2.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/hbm_activity.py gpurun_out/r6w_hbm_c4.json -- python3 bench.py --no-cpu-baseline --config c4 --steps 30 --warmup 2 --sustain 15 > gpurun_out/r6w_hbm_c4.log 2>&1
rc=$?; grep -h workload_HBM gpurun_out/r6w_hbm_c*.json; exit $rc
