#!/bin/bash
# bench.py under env settings on the GPU box; one line per setting.
# usage: tools/env_sweep.sh "<bench args>" "ENV1=a ENV2=b" "ENV1=c" ...
ARGS=$1; shift
mkdir -p gpurun_out
for envs in "$@"; do
  line=$(env MRT_DIAG=1 $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline $ARGS 2>/dev/null | grep '^{')
  rc=$?
  echo "[$envs] rc=$rc $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["frac"], r["avg_launch_ms"])' "$line" 2>/dev/null)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
