#!/usr/bin/env python3
"""Measure the culling slack the kernels' traversal needs.

The kernels cull a BVH child only when its slab entry lies beyond the current
hit's t by more than 2^-11 of it (kernels.hip kCullScale).  A hit is safe from
every visiting order iff each box on the path from the root to its leaf is
entered no later than t_hit * (1 + 2^-11).  This tool traces the oracle's own
rays of one full-size frame through the oracle's stages (renderer/Shaders.metal
rayGenerator / intersectionHandler / lightSamplingHandler), finds each ray's
nearest hit with the oracle's CPU BVH WITHOUT culling by the current hit (the
brute force over every box the ray enters), and asks libmrt's host-only test
entry mrt_debug_box_margin for (t_entry - t_hit) / t_hit over the kernels' own
BVH4 boxes on that hit's path, in both builds' slab arithmetic.

usage: tools/box_margin.py [W H L frame procedural_triangles threads out.json]
       (default: the C4 frame 1920 1080 4 0 1048576 8)
Runs on the CPU (no device): the scene is built host-only.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("metal-renderer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import mrt  # noqa: E402
import oracle  # noqa: E402
from helpers import SEED  # noqa: E402


def main():
    a = sys.argv[1:]
    W, H, L, frame = (int(a[0]), int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else (1920, 1080, 4, 0)
    proc = int(a[4]) if len(a) > 4 else 1 << 20
    threads = int(a[5]) if len(a) > 5 else 8
    out_path = a[6] if len(a) > 6 else None
    t0 = time.time()
    sc = mrt.Scene("cornellbox", procedural_triangles=proc, device=-1)
    e = sc.export()
    osc = oracle.OracleScene.from_arrays(e["vertices"], e["references"], e["materials"])
    print(f"scene {sc.info['triangles']} triangles, BVH4 {sc.info['bvh_nodes']} nodes ({time.time() - t0:.1f} s)",
          flush=True)
    rays = oracle.raygen(W, H, oracle.noise_table(SEED, frame))
    kinds = {"path": [], "shadow": []}   # rows: (hit precise, hit fast, near ties precise, near ties fast)
    stats = {}
    for i in range(L):
        noise = oracle.noise_table(SEED, oracle.noise_frame_for(frame, i))
        t1 = time.time()
        isect = osc.intersect_bvh(rays, threads=threads, nocull=True)
        if i >= 1:
            live = (rays["maxDistance"] >= 0) & (isect["distance"] >= 0)
            kinds["path"].append(sc.box_margin(rays[live], isect[live]))
        srays = np.zeros(len(rays), oracle.SRAY_DTYPE)
        osc.shade(W, H, frame, L, noise, isect, rays, srays)
        sis = osc.intersect_bvh(srays, threads=threads, nocull=True)
        live = (srays["maxDistance"] >= 0) & (sis["distance"] >= 0)
        kinds["shadow"].append(sc.box_margin(srays[live], sis[live]))
        oracle.resolve(sis, rays, srays)
        print(f"bounce {i}: {int((rays['maxDistance'] >= 0).sum())} rays alive after shading "
              f"({time.time() - t1:.1f} s)", flush=True)
    for k, parts in kinds.items():
        m = np.concatenate(parts) if parts else np.zeros((0, 4), np.float32)
        row = {"hits": int(len(m)), "with_near_ties": int(np.isfinite(m[:, 2]).sum() + np.isinf(m[:, 2]).sum()
                                                          - (m[:, 2] == -np.inf).sum())}
        for col, name in ((0, "precise"), (1, "fast"), (2, "near_ties_precise"), (3, "near_ties_fast")):
            v = m[:, col].astype(np.float64)
            row[name] = {
                "max": float(v.max()) if len(v) and v.max() > -np.inf else None,
                "max_over_2^-11": float(v.max() / 2.0 ** -11) if len(v) and v.max() > -np.inf else None,
                "missed_boxes": int((v == np.inf).sum()),
                "positive": int((v > 0).sum()),
                "above_2^-20": int((v > 2.0 ** -20).sum()),
                "above_2^-16": int((v > 2.0 ** -16).sum()),
                "above_2^-11": int((v > 2.0 ** -11).sum()),
            }
            if len(v):
                j = int(np.argmax(v))
                row[name]["argmax"] = j
        stats[k] = row
        print(k, json.dumps(row), flush=True)
    result = {"scene": f"cornellbox + {proc} procedural triangles", "W": W, "H": H, "L": L, "frame": frame,
              "seed": SEED, "kernel_slack": 2.0 ** -11, "margins": stats, "seconds": round(time.time() - t0, 1)}
    if out_path:
        with open(out_path, "w") as f:
            json.dump(result, f, indent=1)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
