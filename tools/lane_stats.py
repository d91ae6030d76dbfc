#!/usr/bin/env python3
"""Where idle SIMD lanes come from, per loop of the hot kernel, from the
diagnostic lane-statistics library (make -C metal-renderer_amd variant
VNAME=lanes VFLAGS=-DMRT_LANESTATS=1; run on the GPU box with
MRT_LIB=metal-renderer_amd/lib/libmrt_lanes.so).

For every traversal loop the library counts the wave iterations and the
active lanes in them; lane utilisation of a loop = lanes / (64 x iterations)
(the share of the loop's issued lane-slots that do work; a wave64 VALU
instruction costs its SIMD the same issue whatever its exec mask).

usage: tools/lane_stats.py [config] [frames]   -> one JSON line + a table
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metal-renderer_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)
import mrt  # noqa: E402

NAMES = ["near_lanes", "near_calls", "near_int_iters", "near_int_lanes", "near_leaf_iters", "near_leaf_lanes",
         "occ_lanes", "occ_calls", "occ_int_iters", "occ_int_lanes", "occ_leaf_iters", "occ_leaf_lanes",
         "shade_calls", "shade_lanes", "wave_calls", "wave_active", "shadow_rays", "shadow_calls",
         "list_calls", "list_lanes", "svc_rounds", "svc_lanes", "trav_rounds", "trav_lanes", "refill_lanes",
         "outer_iters", "stream_camera_iters", "stream_level_iters", "stream_queue_wait_cycles",
         "stream_queue_waits"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    cfg = bench.CONFIGS[name]
    scene = mrt.Scene(cfg["scene"], bench.resolve_mtl(cfg), procedural_triangles=cfg["procedural"], device=0)
    r = mrt.Renderer(scene, cfg["width"], cfg["height"], cfg["L"])
    r.draw(2)
    r.sync()
    mrt.debug_lanes(reset=True)
    r.draw(frames)
    r.sync()
    v = [int(x) for x in mrt.debug_lanes(reset=False)]
    st = r.stats()
    r.close()
    c = dict(zip(NAMES, v))
    if not any(v):
        raise SystemExit("all counters zero: run with MRT_LIB=metal-renderer_amd/lib/libmrt_lanes.so")

    def util(lanes, iters):
        return round(lanes / (64.0 * iters), 4) if iters else None

    path = st["kernel"] == 1
    out = {"config": name, "frames": frames, "kernel": {0: "bounce", 1: "path", 2: "stream"}[st["kernel"]],
           "counters": c}
    if path:
        # the path kernel's rounds mix nearest and occlusion lanes in one loop
        out["interior_util"] = util(c["near_int_lanes"] + c["occ_int_lanes"], c["near_int_iters"])
        out["leaf_util"] = util(c["near_leaf_lanes"] + c["occ_leaf_lanes"], c["near_leaf_iters"])
        out["interior_steps"] = {"nearest": c["near_int_lanes"], "occlusion": c["occ_int_lanes"],
                                 "wave_iters": c["near_int_iters"]}
        out["leaf_steps"] = {"nearest": c["near_leaf_lanes"], "occlusion": c["occ_leaf_lanes"],
                             "wave_iters": c["near_leaf_iters"]}
        out["service_util"] = util(c["svc_lanes"], c["svc_rounds"])
        out["shade_lanes_per_service"] = round(c["shade_lanes"] / max(1, c["svc_rounds"]), 2)
        out["round_util"] = util(c["trav_lanes"], c["trav_rounds"])
    else:
        for q in ("near", "occ"):
            out[f"{q}_interior_util"] = util(c[f"{q}_int_lanes"], c[f"{q}_int_iters"])
            out[f"{q}_leaf_util"] = util(c[f"{q}_leaf_lanes"], c[f"{q}_leaf_iters"])
            out[f"{q}_entry_util"] = util(c[f"{q}_lanes"], c[f"{q}_calls"])
            out[f"{q}_int_steps_per_ray"] = round(c[f"{q}_int_lanes"] / max(1, c[f"{q}_lanes"]), 3)
            out[f"{q}_leaf_steps_per_ray"] = round(c[f"{q}_leaf_lanes"] / max(1, c[f"{q}_lanes"]), 3)
            out[f"{q}_int_iters_per_call"] = round(c[f"{q}_int_iters"] / max(1, c[f"{q}_calls"]), 3)
            out[f"{q}_leaf_iters_per_call"] = round(c[f"{q}_leaf_iters"] / max(1, c[f"{q}_calls"]), 3)
        out["wave_entry_util"] = util(c["wave_active"], c["wave_calls"])
        out["shade_util"] = util(c["shade_lanes"], c["shade_calls"])
        out["shadow_phase_util"] = util(c["shadow_rays"], c["shadow_calls"])
        out["list_util"] = util(c["list_lanes"], c["list_calls"])
        if c.get("stream_queue_waits"):
            # shader-clock cycles (s_memtime) a wave spends in the queue
            # iteration's wait for its own stores, per level iteration
            out["queue_wait_cycles_per_iter"] = round(c["stream_queue_wait_cycles"] / c["stream_queue_waits"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
