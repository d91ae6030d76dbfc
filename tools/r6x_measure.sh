# r6x: r6v (tree shape sweep + final configuration lines) and r6w (DRAM-side
# traffic of C2 / C4) in one call
set -o pipefail
bash tools/r6w_measure.sh || exit $?
bash tools/r6v_measure.sh
