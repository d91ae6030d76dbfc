#!/usr/bin/env python3
"""Add the DRAM-side traffic estimate of a tools/hbm_activity.py run to the
configuration's counter file (profiles/pmc_<config>.json, key "dram_side").

rocprofv3's FETCH_SIZE / WRITE_SIZE count the L2's fabric requests, Infinity
Cache hits included; hbm_activity.py samples the memory controllers' activity
(amd-smi UMC %) behind the Infinity Cache and calibrates it with a device copy
whose HBM bytes are known.  Bytes per launch = the estimated HBM rate over the
busy samples x the workload's step time (one hot-kernel launch per step).
usage: tools/dram_merge.py <hbm_activity json> <config>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, cfg = sys.argv[1], sys.argv[2]
h = json.load(open(src))
line = json.loads([l for l in h["workload_stdout_tail"].splitlines() if l.startswith("{")][-1])
gbps = h["estimate"]["workload_HBM_GBps_busy"]
ms = line["ms_per_step"]
path = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")
p = json.load(open(path))
p["dram_side"] = {
    "GBps": round(gbps, 1),
    "frac_of_8TBps": round(gbps / 8000.0, 4),
    "bytes_per_launch": int(gbps * 1e9 * ms * 1e-3),
    "l2_side_bytes_per_launch": p.get("hbm_bytes_per_launch"),
    "umc_activity_pct": round(h["workload"]["umc_mean_busy"], 2),
    "GBps_per_umc_pct": round(h["estimate"]["GBps_per_umc_pct"], 2),
    "calibration_copy_GBps": round(h["calibration"]["copy_GBps"], 1),
    "ms_per_step": ms,
    "method": "amd-smi UMC activity sampled over the workload, calibrated by a 4-GiB device copy (tools/hbm_activity.py)",
    "source": os.path.relpath(src, ROOT),
}
json.dump(p, open(path, "w"), indent=1)
print(cfg, p["dram_side"])
