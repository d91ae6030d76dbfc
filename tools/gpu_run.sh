#!/bin/bash
# Run GPU steps on the gpurun box, each under its own time limit; stop at the
# first step that ends by a signal / fault / timeout (anything but 0 or 1).
# usage: tools/gpu_run.sh "name:seconds:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== fatal rc=$rc, stopping"; exit $rc; fi
done
