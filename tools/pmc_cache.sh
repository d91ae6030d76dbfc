#!/bin/bash
# cache-hierarchy counter pass for the bounce kernel (one pass: 2 TCC + 2 TCP counters)
# usage: tools/pmc_cache.sh <config> [extra bench args]
export TMPDIR=/tmp
CFG=${1:-c4}; shift
OUT=gpurun_out/pmc_cache_$CFG
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT -o run -f csv -- python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline "$@" > $OUT/log.txt 2>&1
rc=$?
tail -2 $OUT/log.txt
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("bounce_", "path_kernel", "stream_kernel")):
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print(f"{k:32s} {agg[k]/n[k]:.4g}")
h, m = agg.get("TCC_HIT_sum", 0), agg.get("TCC_MISS_sum", 0)
if h + m: print(f"L2 hit rate {h / (h + m):.3f}")
a, rq = agg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), agg.get("TCP_TCC_READ_REQ_sum", 0)
if a: print(f"L1 -> L2 read requests per L1 access {rq / a:.3f}")
PY
exit $rc
