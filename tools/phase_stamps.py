#!/usr/bin/env python3
"""Phase shares of the bounce kernel from the diagnostic stamp build
(make -C metal-renderer_amd stamps; run with MRT_LIB=.../libmrt_stamps.so).
usage: tools/phase_stamps.py [config] [frames]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metal-renderer_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)
import mrt  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
scene = mrt.Scene(cfg["scene"], bench.resolve_mtl(cfg), procedural_triangles=cfg["procedural"], device=0)
r = mrt.Renderer(scene, cfg["width"], cfg["height"], cfg["L"])
r.draw(8)
r.sync()
mrt.debug_stamps(reset=True)
r.draw(frames)
r.sync()
st = mrt.debug_stamps(reset=True)
names = ["load/raygen", "nearest trace", "shade", "compact+write", "shadow trace+write"]
tot = float(sum(st[:5]))
print(f"{cfg['workload']}: {frames} frames, {int(st[5])} wave-iterations")
for k, n in enumerate(names):
    print(f"  {n:20s} {100.0 * st[k] / tot:6.2f} %   {st[k] / max(1, st[5]):10.1f} cyc/wave-iter")
r.close()
