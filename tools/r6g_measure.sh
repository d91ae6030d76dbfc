# r6g: convex occluders (unrolled face slots) A/B on C2, alternating
set -o pipefail
bash tools/env_sweep.sh "--sustain 0" "MRT_CONVEX=1" "MRT_CONVEX=0" "MRT_CONVEX=1" "MRT_CONVEX=0" > gpurun_out/r6g_ab.log 2>&1; cat gpurun_out/r6g_ab.log
