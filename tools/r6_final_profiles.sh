# r6 final: rocprofv3 trace + PMC passes of every configuration at the final
# library (tools/profile.sh; summarised here by tools/prof_summary.py into
# profiles/pmc_<config>.json and profiles/r6a_<config>_*), then the C2 lane
# statistics (MRT_LANESTATS variant library)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r6a}
bash tools/profile.sh $T c2 || exit $?
LPS=64 STEPS=6 bash tools/profile.sh $T c2i --no-image-check || exit $?   # (the image check's 64-frame launches would join the per-frame ones)
bash tools/profile.sh $T c2l5 || exit $?
NAME=c2s8 STEPS=40 WARM=4 bash tools/profile.sh $T c2 --shard-of 8 || exit $?
STEPS=6 WARM=1 bash tools/profile.sh $T c3 || exit $?
STEPS=6 WARM=1 bash tools/profile.sh $T c3g || exit $?
bash tools/profile.sh $T c4 || exit $?
NAME=c5s8 STEPS=8 WARM=1 bash tools/profile.sh $T c5 --shard-of 8 || exit $?
if [ -f metal-renderer_amd/lib/libmrt_lanes.so ]; then
  MRT_DIAG=1 MRT_LIB=metal-renderer_amd/lib/libmrt_lanes.so timeout -k 10 300 python3 tools/lane_stats.py c2 8 > gpurun_out/${T}_lanes_c2.log 2>&1 || exit $?
  grep '^{' gpurun_out/${T}_lanes_c2.log > gpurun_out/${T}_lanes_c2.json; tail -5 gpurun_out/${T}_lanes_c2.log
fi
