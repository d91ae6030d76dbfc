#!/bin/bash
# Run bench.py with alternative libmrt builds (MRT_LIB) on the GPU box; one line per (lib, config).
# usage: tools/lib_sweep.sh "<bench args>" <config list> -- lib1 lib2 ...
ARGS=$1; shift
CFGS=()
while [ "$1" != "--" ]; do CFGS+=("$1"); shift; done; shift
mkdir -p gpurun_out
for lib in "$@"; do
  for cfg in "${CFGS[@]}"; do
    line=$(MRT_LIB=metal-renderer_amd/lib/$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --config $cfg $ARGS 2>/dev/null | grep '^{')
    rc=$?
    echo "$lib $cfg rc=$rc $(python3 -c 'import json,sys; d=json.loads(sys.argv[1]); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["frac"], r["avg_launch_ms"])' "$line" 2>/dev/null)"
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done
