#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>_<cfg>) into profiles/.

Writes:
  profiles/<tag>_<cfg>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_<cfg>_summary.md         per-kernel timing + PMC-derived HBM traffic and SQ ratios
  profiles/pmc_<cfg>.json                 HBM bytes per bounce launch (read by bench.py -> roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KB;
on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads,
so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH and WRITE collected in
separate passes).
"""
import collections
import csv
import json
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


HOT = ("bounce_", "path_kernel", "stream_kernel")   # the hot kernel: wavefront kernels or the path megakernel


def counters(path):
    agg, n = collections.defaultdict(float), collections.Counter()
    meta = {}
    for r in csv.DictReader(open(path)):
        if not any(k in r["Kernel_Name"] for k in HOT):
            continue
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
        meta = {k: r[k] for k in ("VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Grid_Size", "Workgroup_Size")}
    return {k: agg[k] / n[k] for k in agg}, meta


def main(tag="r1", cfg="c2"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_{cfg}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats_csv = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copyfile(stats_csv, os.path.join(out, f"{tag}_{cfg}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats_csv)))
    fetch, meta = counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write, _ = counters(os.path.join(src, "write", "run_counter_collection.csv"))
    sq, _ = counters(os.path.join(src, "sq", "run_counter_collection.csv"))
    clk, _ = counters(os.path.join(src, "clk", "run_counter_collection.csv"))
    lanes_csv = os.path.join(src, "lanes", "run_counter_collection.csv")
    lanes = counters(lanes_csv)[0] if os.path.exists(lanes_csv) else {}
    # VALUUtilization (rocprofiler-sdk counter_defs.yaml): active lanes per
    # issued VALU instruction / 64 — the share of issued lane-slots doing work
    lane_util = (lanes["SQ_THREAD_CYCLES_VALU"] / (64.0 * lanes["SQ_ACTIVE_INST_VALU"])
                 if lanes.get("SQ_ACTIVE_INST_VALU") else None)
    bounce = next(r for r in rows if any(k in r["Name"] for k in HOT))
    avg_ns = float(bounce["AverageNs"])
    # the timed launches alone: the trace's per-dispatch records of the hot
    # kernel minus the warm-up launches (profile.sh STEPS / WARM; one launch
    # per step on C1-C5), so the average is comparable with ms_per_step
    timed_ns, timed_n = None, None
    trace_csv = os.path.join(src, "trace", "run_kernel_trace.csv")
    steps_file = os.path.join(src, "steps")
    def steps_lps():
        f = [int(x) for x in open(steps_file).read().split()]
        return f[0] * (f[2] if len(f) > 2 else 1), f[1] * (f[2] if len(f) > 2 else 1)   # launches: timed, warm-up

    if os.path.exists(trace_csv) and os.path.exists(steps_file):
        steps, warm = steps_lps()
        durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in
                sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
                if r["Kernel_Name"] == bounce["Name"]]
        if len(durs) >= steps + warm:
            tail = durs[-steps:]
            timed_ns, timed_n = sum(tail) / len(tail), len(tail)
    # the two-stream run: period per launch over the timed launches
    period_ns = None
    trace2_csv = os.path.join(src, "trace2", "run_kernel_trace.csv")
    if os.path.exists(trace2_csv) and os.path.exists(steps_file):
        steps, warm = steps_lps()
        ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace2_csv))
              if r["Kernel_Name"] == bounce["Name"]]
        ev.sort()
        if len(ev) >= steps + warm:
            tail = ev[-steps:]
            # from the end of the last warm-up launch to the end of the last
            # timed one: each timed launch's share of the (overlapped) stream
            t0 = ev[-steps - 1][1]
            period_ns = (max(e for _, e in tail) - t0) / steps
    hbm = (2.0 * fetch["FETCH_SIZE"] + write["WRITE_SIZE"]) * 1024.0
    lines = [f"# rocprofv3 summary — {tag} / {cfg}", "",
             "`tools/profile.sh` → kernel trace + stats pass, then separate PMC passes "
             "(FETCH_SIZE; WRITE_SIZE; SQ; VALU lanes; GRBM), one render stream (MRT_INFLIGHT=1).", "",
             (f"Hot kernel over the {timed_n} timed launches (warm-up excluded): **{timed_ns / 1e6:.3f} ms per launch** "
              f"(the stats table below averages every launch, warm-up included)." if timed_ns else
              "Timed-launch average unavailable (no per-dispatch trace)."), "",
             (f"At the renderer's default two render streams (overlapping launches) the hot kernel's period "
              f"over the same timed launches is **{period_ns / 1e6:.3f} ms per launch** (end of the last warm-up "
              f"launch to the end of the last timed one, / launches)." if period_ns else ""), "",
             "| kernel | calls | avg µs | total ms | % |", "|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |")
    lines += ["", f"## {bounce['Name'][:60]} PMC (per launch, averaged)", "",
              f"* FETCH_SIZE {fetch['FETCH_SIZE']:.0f} KB (×2 gfx950 correction), WRITE_SIZE {write['WRITE_SIZE']:.0f} KB "
              f"→ **HBM traffic {hbm / 1e6:.1f} MB per launch**, {hbm / (avg_ns * 1e-9) / 1e9:.0f} GB/s over the "
              f"average launch ({avg_ns / 1e3:.1f} µs)",
              f"* SQ: VALU insts {sq.get('SQ_INSTS_VALU', 0):.3g}, SALU {sq.get('SQ_INSTS_SALU', 0):.3g}, "
              f"LDS {sq.get('SQ_INSTS_LDS', 0):.3g}, VMEM rd {sq.get('SQ_INSTS_VMEM_RD', 0):.3g}; "
              f"WAIT_ANY / WAVE_CYCLES = {sq.get('SQ_WAIT_ANY', 0) / max(1, sq.get('SQ_WAVE_CYCLES', 1)):.2f}, "
              f"ACTIVE_INST_VALU / WAVE_CYCLES = {sq.get('SQ_ACTIVE_INST_VALU', 0) / max(1, sq.get('SQ_WAVE_CYCLES', 1)):.2f}",
              f"* effective clock ≈ GRBM_GUI_ACTIVE / 8 / launch = "
              f"{clk.get('GRBM_GUI_ACTIVE', 0) / 8 / (avg_ns * 1e-9) / 1e9:.2f} GHz (reads high on overlapping dispatches)",
              f"* dispatch: {meta}"]
    # VALU issue share: a wave64 VALU instruction occupies its SIMD's issue for
    # 2 cycles (MI355X_MICROARCH.md); capacity = 256 CUs x 4 SIMDs x clock x t
    clk_hz = clk.get("GRBM_GUI_ACTIVE", 0) / 8 / (avg_ns * 1e-9)   # (PMC passes time every launch alike)
    valu_frac = (2.0 * sq.get("SQ_INSTS_VALU", 0) / (1024 * clk_hz * avg_ns * 1e-9)) if clk_hz else None
    wave_cycles = max(1.0, sq.get("SQ_WAVE_CYCLES", 1.0))
    try:
        commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                                text=True).stdout.strip() or None
    except OSError:
        commit = None
    lines.append(f"* VALU issue share = 2 x VALU insts / (1024 SIMDs x clock x launch) = "
                 f"{valu_frac if valu_frac is None else round(valu_frac, 3)}")
    if lane_util is not None:
        lines.append(f"* VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU) = {lane_util:.3f} "
                     f"(share of issued lane-slots with an active lane)")
    md5_path = os.path.join(src, "lib.md5")
    lib_md5 = open(md5_path).read().strip() if os.path.exists(md5_path) else None
    m = re.search(r"(bounce_\w*kernel|path_kernel|stream_kernel)<[^>]*>", bounce["Name"])
    kernel = m.group(0) if m else bounce["Name"][:60]
    lines.append(f"* measured library: lib/libmrt.so md5 {lib_md5}, repository commit {commit}")
    with open(os.path.join(out, f"{tag}_{cfg}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    with open(os.path.join(out, f"pmc_{cfg}.json"), "w") as f:
        json.dump({"tag": tag, "config": cfg, "kernel": kernel, "commit": commit, "lib_md5": lib_md5,
                   "hbm_bytes_per_launch": round(hbm),
                   "fetch_size_kb": fetch["FETCH_SIZE"], "write_size_kb": write["WRITE_SIZE"],
                   "avg_launch_ns_rocprof": avg_ns, "avg_launch_ns_rocprof_timed": timed_ns,
                   "timed_launches_rocprof": timed_n, "period_ns_rocprof_2streams": period_ns,
                   "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024",
                   "sq": sq, "clock_ghz": round(clk_hz / 1e9, 3),
                   "valu_issue_frac": None if valu_frac is None else round(valu_frac, 4),
                   "wait_any_frac": round(sq.get("SQ_WAIT_ANY", 0) / wave_cycles, 4),
                   "valu_active_frac": round(sq.get("SQ_ACTIVE_INST_VALU", 0) / wave_cycles, 4),
                   "valu_lane_util": None if lane_util is None else round(lane_util, 4), "lanes": lanes},
                  f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(*sys.argv[1:])
