#!/usr/bin/env python3
"""Per-kernel resource usage from a gfx950 code object's AMDGPU metadata
note (llvm-readelf --notes): VGPRs, SGPR/VGPR spills, scratch bytes.
usage: tools/kres_co.py <code object> [kernel-name substring ...]"""
import re
import subprocess
import sys


def kernels(co):
    txt = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True,
                         text=True, check=True).stdout
    body = txt.split("amdhsa.kernels:", 1)[1]
    out = []
    for item in re.split(r"\n\s{2,6}- \.", body)[1:]:
        f = dict(re.findall(r"\.?([a-z_]+):\s+([^\s]+)", "." + item))
        if "name" in f:
            out.append(f)
    return out


if __name__ == "__main__":
    co, pats = sys.argv[1], sys.argv[2:]
    for k in kernels(co):
        if pats and not any(p in k["name"] for p in pats):
            continue
        print(f'{k["name"][:70]:70s} vgpr {k.get("vgpr_count")} vspill {k.get("vgpr_spill_count")} '
              f'sspill {k.get("sgpr_spill_count")} scratch {k.get("private_segment_fixed_size")}')
