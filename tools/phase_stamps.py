#!/usr/bin/env python3
"""Phase shares of the bounce kernel from the diagnostic stamp build
(make -C metal-renderer_amd stamps; run with MRT_LIB=.../libmrt_stamps.so).
usage: tools/phase_stamps.py [config] [frames] [shard_count]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metal-renderer_amd"))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS)
import mrt  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c2"]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 16
shards = int(sys.argv[3]) if len(sys.argv) > 3 else 1
scene = mrt.Scene(cfg["scene"], bench.resolve_mtl(cfg), procedural_triangles=cfg["procedural"], device=0)
r = mrt.Renderer(scene, cfg["width"], cfg["height"], cfg["L"], shard_rank=0, shard_count=shards)
r.draw(8)
r.sync()
mrt.debug_stamps(reset=True)
r.draw(frames)
r.sync()
st = mrt.debug_stamps(reset=False)
names = ["load/raygen", "nearest trace", "shade", "compact+write", "shadow trace+write"]
tot = float(sum(st[:5]))
print(f"{cfg['workload']}: {frames} frames, {int(st[5])} wave-iterations")
for k, n in enumerate(names):
    print(f"  {n:20s} {100.0 * st[k] / tot:6.2f} %   {st[k] / max(1, st[5]):10.1f} cyc/wave-iter")
r.close()

# launch-boundary timeline of the last launch of each bounce (ramp / drain)
import numpy as np  # noqa: E402
wt = mrt.debug_wave_times().astype(np.int64)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.save(os.path.join(ROOT, "gpurun_out", f"wave_times_{sys.argv[1] if len(sys.argv) > 1 else 'c2'}_s{shards}.npy"), wt)
why = wt[..., 2] >> 32
wt[..., 2] &= 0xFFFFFFFF
for b in range(min(4, cfg["L"])):
    e = wt[b][wt[b][:, 2] > 0]
    if len(e) == 0:
        continue
    t0, t1 = e[:, 0].min(), e[:, 1].max()
    span = (t1 - t0) / 100.0   # us
    starts = np.sort((e[:, 0] - t0) / 100.0)
    ends = np.sort((e[:, 1] - t0) / 100.0)
    busy = ((e[:, 1] - e[:, 0]) / 100.0).sum() / (len(e) * span)
    print(f"  bounce {b}: {len(e)} waves, span {span:8.1f} us, waves busy {100 * busy:5.1f} % of span; "
          f"start p50/p99/max {np.percentile(starts, 50):6.1f}/{np.percentile(starts, 99):6.1f}/{starts[-1]:6.1f} us; "
          f"exit min/p10/p50 {ends[0]:8.1f}/{np.percentile(ends, 10):8.1f}/{np.percentile(ends, 50):8.1f} us "
          f"(drain = span - p50 exit {span - np.percentile(ends, 50):6.1f} us); iterations/wave "
          f"min/mean/max {e[:, 2].min()}/{e[:, 2].mean():.1f}/{e[:, 2].max()}; "
          f"exits by full segment {(why[b][wt[b][:, 2] > 0] == 2).sum()}")
for b in range(min(4, cfg["L"])):
    e = wt[b][wt[b][:, 2] > 0]
    if len(e) == 0:
        continue
    t0 = e[:, 0].min()
    lg, lw, ex = (e[:, 3] - t0) / 100.0, (e[:, 4] - t0) / 100.0, (e[:, 1] - t0) / 100.0
    grabs = np.maximum(1, (e[:, 2] & 0xFFFFFFFF) // 2)
    print(f"  bounce {b}: last grab p50 {np.median(lg):.0f} us; its work p50/max {np.median(lw - lg):.0f}/{(lw - lg).max():.0f} us; "
          f"exit after work p50/max {np.median(ex - lw):.0f}/{(ex - lw).max():.0f} us; grab latency mean "
          f"{(e[:, 5] / grabs).mean() / 100:.1f} us, max p50 {np.median(e[:, 6]) / 100:.1f} us, last grab's p50/max "
          f"{np.median(e[:, 7]) / 100:.1f}/{e[:, 7].max() / 100:.1f} us")
