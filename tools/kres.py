#!/usr/bin/env python3
"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output: one line per
kernel (VGPRs, spills, SGPRs, LDS), filtered by a substring of the mangled name.
usage: tools/kres.py <remarks.txt> [substring]"""
import re
import sys


def main(path, sub=""):
    cur, out = None, {}
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/block\])?: (\d+)", line)
        if cur and m:
            out[cur][m.group(1).strip()] = int(m.group(2))
    for k, v in out.items():
        if sub in k:
            print(f"{k[28:90]:62s} VGPR {v.get('VGPRs', '?'):>3} spill {v.get('VGPRs Spill', '?'):>3} "
                  f"SGPR {v.get('SGPRs', '?'):>3} sspill {v.get('SGPRs Spill', '?'):>3} LDS {v.get('LDS Size', '?')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
