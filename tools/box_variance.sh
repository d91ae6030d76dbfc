#!/bin/bash
# One box's sample for the cross-box spread of the headline lines (run it in
# several gpurun calls: each call gets a fresh box).  usage: tools/box_variance.sh <outdir>
OUT=${1:-gpurun_out/var}
mkdir -p $OUT
ID=$(hostname)-$(date +%s)
D=$OUT/$ID
mkdir -p $D
(rocm-smi --showuniqueid --showclocks 2>/dev/null || true) > $D/smi.txt
run() { local name=$1 secs=$2; shift 2; timeout -k 10 $secs python3 bench.py "$@" > $D/$name.json 2> $D/$name.log; local rc=$?; echo "$ID $name rc=$rc $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); s=d.get("sustained") or {}; print(d["value"], s.get("value"))' $D/$name.json 2>/dev/null)"; [ $rc -eq 0 ] || exit $rc; }
run c2 400 --no-cpu-baseline
run c4 300 --config c4 --steps 30 --warmup 2 --no-cpu-baseline --no-image-check
run c5s8 300 --config c5 --shard-of 8 --steps 10 --warmup 1 --no-cpu-baseline --no-image-check
run c2i 300 --config c2i --steps 80 --warmup 5 --no-cpu-baseline --no-image-check
