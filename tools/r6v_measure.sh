# r6v: the main tree's shape for C2 at the r6 library (host SAH: leaf size
# MRT_LEAF 1 / 2 (default) / 3 / 4, traversal cost MRT_CTRAV 0.5 / 2), then
# the final configuration lines with the r6a counters (same library)
set -o pipefail
mkdir -p gpurun_out
bash tools/env_sweep.sh "--sustain 0" "MRT_DEBUG=0" "MRT_LEAF=1" "MRT_LEAF=3" "MRT_LEAF=4" "MRT_CTRAV=0.5" "MRT_CTRAV=2" "MRT_DEBUG=0" "MRT_LEAF=1" > gpurun_out/r6v_tree.log 2>&1 || exit $?
cat gpurun_out/r6v_tree.log
bash tools/run_configs.sh gpurun_out/r6_configs2
