#!/bin/bash
# Counter passes for one bench config (GPU box, repo root), one rocprofv3 run
# per pass (gfx950 per-block limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD).
# usage: [PASSES="valu sq1 ..."] tools/pmc_probe.sh <tag> <config> [extra bench args]
# prints per-launch averages of the hot kernel's counters
export TMPDIR=/tmp
TAG=${1:-probe}; CFG=${2:-c4}; shift 2
OUT=gpurun_out/pmc_${TAG}_$CFG
mkdir -p $OUT
BENCH="python3 bench.py --config $CFG --steps 1 --warmup 1 --no-cpu-baseline $*"
K='bounce_|path_kernel|stream_kernel'
pass() { local name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d $OUT/$name -o run -f csv -- $BENCH > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -3 $OUT/$name.log; exit 1; }; }
for P in ${PASSES:-valu sq1 sq2 tcp1 tcp2 tcc}; do case $P in
valu) pass valu SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU ;;
sq1) pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR ;;
sq2) pass sq2 SQ_WAVE_CYCLES SQ_IFETCH SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT ;;
tcp1) pass tcp1 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum ;;
tcp2) pass tcp2 TCP_TCP_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum ;;
tcc) pass tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE ;;
esac; done
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("bounce_", "path_kernel", "stream_kernel")):
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
v = {k: agg[k] / n[k] for k in agg}
for k in sorted(v): print(f"{k:36s} {v[k]:.5g}")
wc = v.get("SQ_WAVE_CYCLES", 0)
def r(a, b, label):
    if v.get(a) is not None and v.get(b): print(f"  {label:40s} {v[a] / v[b]:.4g}")
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_INST_LEVEL_VMEM",
          "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_INST_CYCLES_VMEM_RD"):
    r(k, "SQ_WAVE_CYCLES", k + "/WAVE_CYCLES")
if v.get("SQ_ACTIVE_INST_VALU"):
    print(f"  {'VALU lane utilisation (active lanes/64)':40s} {v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_ACTIVE_INST_VALU']):.4g}")
r("TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum", "L1->L2 read latency (cycles/req)")
r("TCP_TCP_LATENCY_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP latency (cycles/access)")
r("TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_TRANSLATION_HIT_sum", "UTCL1 miss/hit")
r("TCC_HIT_sum", "TCC_REQ_sum", "L2 hit rate")
r("TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "L1 miss (L2 req) per L1 access")
PY
