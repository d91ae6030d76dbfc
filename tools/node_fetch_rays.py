#!/usr/bin/env python3
"""Query records for tools/node_fetch_stats.cpp: the oracle's own rays of one
C4 frame (renderer/Shaders.metal stages: every bounce's path rays as nearest
queries, every valid shadow ray as an any-hit query below its target's t),
written as float32 (origin, tmin, direction, tmax, kind).
usage: tools/node_fetch_rays.py W H L out.bin"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("metal-renderer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import mrt  # noqa: E402
import oracle  # noqa: E402
from helpers import SEED  # noqa: E402

W, H, L, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
sc = mrt.Scene("cornellbox", procedural_triangles=1 << 20, device=-1)
e = sc.export()
osc = oracle.OracleScene.from_arrays(e["vertices"], e["references"], e["materials"])
V, R = e["vertices"]["v"], e["references"]["tri"]
f = 0
rays = oracle.raygen(W, H, oracle.noise_table(SEED, f))
recs = []
for i in range(L):
    noise = oracle.noise_table(SEED, oracle.noise_frame_for(f, i))
    live = rays["maxDistance"] >= 0
    r = np.zeros((int(live.sum()), 9), np.float32)
    r[:, 0:3] = rays["origin"][live]
    r[:, 3] = rays["minDistance"][live]
    r[:, 4:7] = rays["direction"][live]
    r[:, 7] = np.inf
    recs.append(r)
    isect = osc.intersect_bvh(rays, threads=8)
    srays = np.zeros(len(rays), oracle.SRAY_DTYPE)
    osc.shade(W, H, f, L, noise, isect, rays, srays)
    ok = srays["maxDistance"] >= 0
    s = srays[ok]
    tri = R[s["targetIndex"]]
    v0, v1, v2 = V[tri[:, 0]], V[tri[:, 1]], V[tri[:, 2]]
    n = np.cross(v1 - v0, v2 - v0)
    tT = ((v0 - s["origin"]) * n).sum(1) / (s["direction"] * n).sum(1)
    q = np.zeros((len(s), 9), np.float32)
    q[:, 0:3] = s["origin"]
    q[:, 4:7] = s["direction"]
    q[:, 7] = tT
    q[:, 8] = 1.0
    recs.append(q)
    sis = osc.intersect_bvh(srays, threads=8)
    oracle.resolve(sis, rays, srays)
a = np.concatenate(recs)
a.tofile(out)
print(f"{len(a)} queries ({int((a[:, 8] == 0).sum())} nearest, {int((a[:, 8] == 1).sum())} any-hit) -> {out}")
