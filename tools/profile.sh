#!/bin/bash
# rocprofv3 passes for one bench config (run on the GPU box from the repo root).
# usage: tools/profile.sh <tag> <config> [extra bench args]
# pass 1: kernel trace + stats; passes 2-6: PMC counters, each in its own run
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
TAG=${1:-r1}; CFG=${2:-c2}; shift 2
export TMPDIR=/tmp
# one render stream: the renderer's default two frame batches in flight
# overlap consecutive launches, which stretches each launch's trace span
# (the bench times them by device spans instead); counters per launch are
# the same either way
INF=${MRT_INFLIGHT:-1}
export MRT_DIAG=1 MRT_INFLIGHT=$INF
# NAME: the output's config name (default the bench config; e.g. c5s8 for
# --config c5 --shard-of 8 -> profiles/pmc_c5s8.json via prof_summary.py)
NAME=${NAME:-$CFG}
OUT=gpurun_out/prof_${TAG}_${NAME}
mkdir -p $OUT
# the library these passes measure (bench.py compares it with the one it loads)
md5sum metal-renderer_amd/lib/libmrt.so | cut -d' ' -f1 > $OUT/lib.md5
# >= 10 timed launches after warm-up: the trace pass's average over the timed
# launches (prof_summary.py drops the WARM warm-up launches) is the kernel's
# time per launch on one render stream
STEPS=${STEPS:-12}; WARM=${WARM:-2}
# LPS: hot-kernel launches per step (64 for c2i: one per drawn frame)
LPS=${LPS:-1}
echo "$STEPS $WARM $LPS" > $OUT/steps
BENCH="python3 bench.py --config $CFG --steps $STEPS --warmup $WARM --no-cpu-baseline --sustain 0 $*"
set -o pipefail
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1; local rc=$?; tail -n 3 $OUT/$name.log; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step trace 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -f csv -- $BENCH
# the same run at the renderer's default two render streams: the trace's
# period per launch (first start to last end of the timed launches / count)
# is the kernel's share of the step the bench times
export MRT_DIAG=1 MRT_INFLIGHT=2
step trace2 300 rocprofv3 --kernel-trace -d $OUT/trace2 -o run -f csv -- $BENCH
export MRT_DIAG=1 MRT_INFLIGHT=$INF
step fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT/fetch -o run -f csv -- $BENCH
step write 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT/write -o run -f csv -- $BENCH
step sq 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT/sq -o run -f csv -- $BENCH
step lanes 400 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT/lanes -o run -f csv -- $BENCH
step clk 400 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT/clk -o run -f csv -- $BENCH
