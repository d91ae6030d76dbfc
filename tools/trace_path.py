#!/usr/bin/env python3
"""Print one path's queries (GPU box) from a diagnostic library built with
  make -C metal-renderer_amd vfast VNAME=trace VFLAGS="-DMRT_TRACE_PX=1 -DMRT_TRACE_X=<x> -DMRT_TRACE_Y=<y> \\
       -DMRT_TRACE_F=<frame> -DMRT_TRACE_B=<bounce>"
and loaded with MRT_LIB=metal-renderer_amd/lib/libmrt_ftrace.so: each run renders frames 0..F of the
C5 frame with a fresh renderer; the kernel printf()s the traced path's nearest / shadow queries (float
bits) and, for bounce B, every traversal step, so runs can be diffed.
usage: tools/trace_path.py <frames> <runs>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metal-renderer_amd"))
import mrt  # noqa: E402

frames, runs = int(sys.argv[1]), int(sys.argv[2])
sc = mrt.Scene("cornellbox", procedural_triangles=1 << 20, device=0)
for run in range(runs):
    print(f"=== run {run}", flush=True)
    r = mrt.Renderer(sc, 3840, 2160, 8)
    r.draw(frames)
    r.sync()
    r.close()
    sys.stdout.flush()
