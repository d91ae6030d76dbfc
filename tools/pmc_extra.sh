#!/bin/bash
# extra SQ counter pass for the hot kernel (one pass): LDS array occupancy, bank conflicts, LDS waits
export TMPDIR=/tmp
OUT=gpurun_out/pmc_extra_${1:-c2}
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-include-regex 'bounce_|path_kernel|stream_kernel' -d $OUT -o run -f csv -- python3 bench.py --config ${1:-c2} --steps 2 --warmup 1 --no-cpu-baseline > $OUT/log.txt 2>&1
rc=$?
tail -3 $OUT/log.txt
python3 - "$OUT" <<'PY'
import csv, sys, collections, glob
agg = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("bounce_", "path_kernel", "stream_kernel")):
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print(f"{k:24s} {agg[k]/n[k]:.4g}")
wc = agg["SQ_WAVE_CYCLES"]
for k in sorted(agg):
    if k != "SQ_WAVE_CYCLES" and wc: print(f"  {k}/WAVE_CYCLES = {agg[k]/wc:.3f}")
# LDS array busy share: SQ_LDS_IDX_ACTIVE (LDS-array cycles, summed over CUs) / (256 CUs x kernel cycles);
# GRBM_GUI_ACTIVE sums 8 XCDs' GPU-busy cycles
if agg["GRBM_GUI_ACTIVE"]:
    cyc = agg["GRBM_GUI_ACTIVE"] / n["GRBM_GUI_ACTIVE"] / 8
    print(f"  LDS array busy share = SQ_LDS_IDX_ACTIVE / (256 x {cyc:.4g}) = {agg['SQ_LDS_IDX_ACTIVE'] / n['SQ_LDS_IDX_ACTIVE'] / (256 * cyc):.3f}")
    print(f"  bank-conflict share of LDS cycles = {agg['SQ_LDS_BANK_CONFLICT'] / max(agg['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
PY
exit $rc
