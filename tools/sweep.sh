#!/bin/bash
# Sweep bench.py over env settings on the GPU box; one JSON line per setting.
# usage: tools/sweep.sh <tag> "<bench args>" "ENV1=a ENV2=b" "ENV1=c" ...
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out
OUT=gpurun_out/sweep_$TAG.log
: > $OUT
for envs in "$@"; do
  line=$(timeout -k 10 120 env $envs python3 bench.py --no-cpu-baseline $ARGS 2>/dev/null | grep '^{')
  rc=$?
  echo "$envs | rc=$rc | $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["frac"], r["frac_job"], r["avg_launch_ms"])' "$line" 2>/dev/null)" | tee -a $OUT
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
