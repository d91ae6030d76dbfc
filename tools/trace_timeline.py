#!/usr/bin/env python3
"""Print the tail of a rocprofv3 kernel trace as a timeline (start, duration,
gap to the previous kernel) — used to see launch gaps, ramps and drains.
usage: tools/trace_timeline.py <run_kernel_trace.csv> [last_n]"""
import csv
import sys


def main(path, last=40):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    t0, prev = int(rows[0]["Start_Timestamp"]), None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev else 0.0
        print(f"{(s - t0) / 1000:9.1f} us  dur {(e - s) / 1000:8.1f}  gap {gap:6.1f}  {r['Kernel_Name'][:70]}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
