#!/usr/bin/env python3
"""Where a kernel's scratch (spill) accesses sit relative to its loops.

Disassembles one kernel of a gfx950 code object (llvm-objdump), finds the
loops as the ranges spanned by backward branches, and prints every scratch
instruction with the loops that contain it (innermost first: start, end and
length in instructions) and whether that loop reads BVH nodes from LDS
(ds_read_b96 / b128: a traversal loop).
usage: tools/scratch_sites.py <code object> <kernel symbol substring>
(extract the code object from a build/*.hipfb with clang-offload-bundler
--unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950)"""
import re
import subprocess
import sys

co, pat = sys.argv[1], sys.argv[2]
txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                     text=True, check=True).stdout
labels, ins, cur = {}, [], None
for line in txt.split("\n"):
    m = re.match(r"^([0-9a-f]+) <(.*)>:", line)
    if m:
        labels[m.group(2)] = int(m.group(1), 16)
        cur = m.group(2)
        continue
    m = re.search(r"//\s*([0-9A-F]{12}):", line)
    if m and cur and pat in cur:
        ins.append((int(m.group(1), 16), line.split("//")[0].strip(), line))
if not ins:
    sys.exit(f"no kernel matching {pat}")
base = ins[0][0]
loops = []
for a, t, full in ins:
    m = re.match(r"s_(cbranch_\w+|branch)\s", t)
    tgt = re.search(r"<([^>]*)\+0x([0-9a-f]+)>", full)
    if m and tgt and tgt.group(1) in labels:
        ta = labels[tgt.group(1)] + int(tgt.group(2), 16)
        if ta <= a:
            loops.append((ta, a))
print(f"{len(ins)} instructions, {len(loops)} backward branches")
for a, t, _ in ins:
    if "scratch_" not in t:
        continue
    inside = sorted((lo, hi) for lo, hi in loops if lo <= a <= hi)
    inside.sort(key=lambda x: x[1] - x[0])
    desc = []
    for lo, hi in inside[:2]:
        body = [x for y, x, _ in ins if lo <= y <= hi]
        trav = sum(1 for x in body if x.startswith(("ds_read_b96", "ds_read_b128")))
        desc.append(f"[{lo - base:#x}..{hi - base:#x}] {len(body)} instr, {trav} node reads")
    print(f"{a - base:#7x} {t[:48]:48s} in {len(inside)} loops; innermost: {'; '.join(desc) or '-'}")

# the traversal loops: backward branches spanning node reads, and the scratch
# accesses inside any of them
trav = []
for lo, hi in loops:
    body = [(y, x) for y, x, _ in ins if lo <= y <= hi]
    if len(body) < 400 and any(x.startswith(("ds_read_b96", "ds_read_b128")) for _, x in body):
        trav.append((lo, hi, len(body), sum(1 for _, x in body if "scratch_" in x)))
print(f"{len(trav)} traversal-sized loops (< 400 instructions with node / triangle reads); "
      f"scratch accesses inside them: {sum(t[3] for t in trav)}")
for lo, hi, n, k in sorted(trav):
    print(f"  [{lo - base:#x}..{hi - base:#x}] {n} instr, scratch {k}")
