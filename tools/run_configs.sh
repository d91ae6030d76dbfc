#!/bin/bash
# Every BASELINE configuration's bench line (GPU box, repo root): default bench
# (CPU oracle baseline + image parity, fast and precise) for c1..c4 and c2l5
# (C2 at MAX_PATH_LENGTH 5: the primary ray + 4 bounces), and one GPU's 1/8
# tile share for c2 and c5 (the 8-GPU configuration's per-GPU work).  Timed
# regions of >= ~1 s (a short one carries the pipeline's fill and drain:
# C4 at 5 steps read 1.5 % below its 10-s sustained rate).
# usage: tools/run_configs.sh <outdir>
OUT=${1:-gpurun_out/configs}
mkdir -p $OUT
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 $secs python3 bench.py "$@" > $OUT/cfg_$name.json 2> $OUT/cfg_$name.log; local rc=$?; tail -c 300 $OUT/cfg_$name.json; echo; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run c1 300 --config c1 --steps 50 --warmup 5
run c2 400 --config c2 --steps 100 --warmup 5
run c2l5 400 --config c2l5 --steps 100 --warmup 5
run c2s8 200 --config c2 --steps 400 --warmup 10 --shard-of 8 --no-cpu-baseline --pmc profiles/pmc_c2s8.json
run c3 400 --config c3 --steps 6 --warmup 1
run c2i 300 --config c2i --steps 80 --warmup 5
run c3g 400 --config c3g --steps 6 --warmup 1
run c4 400 --config c4 --steps 30 --warmup 2
run c5s8 300 --config c5 --steps 10 --warmup 1 --shard-of 8 --no-cpu-baseline --pmc profiles/pmc_c5s8.json
