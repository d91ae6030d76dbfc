# r6ab: ablation (wrong images): the convex test without its exhaustive
# fallback (libmrt_fnofb.so) against the product, C2 alternating
set -o pipefail
mkdir -p gpurun_out
bash tools/lib_sweep.sh "--sustain 0" c2 -- libmrt.so libmrt_fnofb.so libmrt.so libmrt_fnofb.so > gpurun_out/r6ab_ab.log 2>&1
rc=$?; cat gpurun_out/r6ab_ab.log; exit $rc
