#!/usr/bin/env python3
"""DRAM-side view of a workload: the memory controllers' activity (amd-smi
metric --usage, UMC activity %) sampled while it runs, calibrated against a
copy whose HBM bytes are known.

rocprofv3's FETCH_SIZE / WRITE_SIZE count the L2's fabric requests, Infinity
Cache hits included (MI355X_MICROARCH.md, FETCH_SIZE note), and gfx950 exposes
no Infinity-Cache / data-fabric counter through rocprofv3 (none among the 4,012
counters `rocprofv3 --list-avail` prints).  The UMC activity is measured at the
memory controllers, behind the Infinity Cache.  Calibration: a device-to-device
copy of 4 GiB buffers (16x the Infinity Cache, so every byte goes to HBM),
timed, gives GB/s per % of UMC activity; the workload's HBM rate is its mean
activity times that ratio (an estimate: activity is a busy-time share, not a
byte count).

usage (GPU box): tools/hbm_activity.py <out.json> -- <workload command ...>
"""
import json
import subprocess
import sys
import threading
import time


def sample_umc():
    """One amd-smi reading of GPU 0: (gfx activity %, umc activity %)."""
    r = subprocess.run(["amd-smi", "metric", "-g", "0", "-u", "--json"], capture_output=True, text=True, timeout=20)
    d = json.loads(r.stdout)
    if isinstance(d, dict) and "gpu_data" in d:   # {"gpu_data": [{"gpu": 0, "usage": {...}}]}
        d = d["gpu_data"]
    if isinstance(d, list):
        d = d[0]
    u = d.get("usage", d)

    def val(k):
        v = u.get(k)
        if isinstance(v, dict):
            v = v.get("value")
        try:
            return float(v)
        except (TypeError, ValueError):
            return None
    return val("gfx_activity"), val("umc_activity"), u


class Sampler:
    def __init__(self):
        self.rows, self._stop = [], False
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self._stop:
            try:
                g, m, _ = sample_umc()
                self.rows.append((time.time(), g, m))
            except Exception as e:   # keep sampling; report the failure
                self.rows.append((time.time(), None, None))
                print("amd-smi:", e, flush=True)
            time.sleep(0.2)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self._stop = True
        self.t.join()


def mean_active(rows, t0, t1):
    """Mean UMC activity over [t0, t1], and over the samples whose gfx
    activity shows the GPU busy."""
    sel = [r for r in rows if t0 <= r[0] <= t1 and r[2] is not None]
    busy = [r for r in sel if (r[1] or 0) >= 50]
    m = lambda xs: sum(x[2] for x in xs) / len(xs) if xs else None   # noqa: E731
    return {"samples": len(sel), "umc_mean": m(sel), "busy_samples": len(busy), "umc_mean_busy": m(busy)}


def calibrate(seconds=12.0):
    import torch
    n = 1 << 30   # 4 GiB of float32 per buffer
    x = torch.empty(n, dtype=torch.float32, device="cuda").uniform_()
    y = torch.empty_like(x)
    y.copy_(x)
    torch.cuda.synchronize()
    t0 = time.time()
    k = 0
    while time.time() - t0 < seconds:
        y.copy_(x)
        k += 1
        if k % 8 == 0:
            torch.cuda.synchronize()
            print(f"calibration copy: {k} copies", flush=True)
    torch.cuda.synchronize()
    dt = time.time() - t0
    gbs = 2.0 * n * 4 * k / dt / 1e9   # read + write
    del x, y
    torch.cuda.empty_cache()
    return t0, t0 + dt, gbs


def main():
    out = sys.argv[1]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    res = {"command": cmd}
    with Sampler() as s:
        time.sleep(2.0)
        i0 = time.time()
        idle = (i0 - 2.0, i0)
        c0, c1, gbs = calibrate()
        res["calibration"] = {"copy_GBps": gbs, **mean_active(s.rows, c0 + 1.0, c1)}
        time.sleep(2.0)
        w0 = time.time()
        p = subprocess.run(cmd, capture_output=True, text=True)
        w1 = time.time()
        res["workload_rc"] = p.returncode
        res["workload_stdout_tail"] = p.stdout[-4000:]
        res["workload"] = mean_active(s.rows, w0, w1)
        res["idle"] = mean_active(s.rows, *idle)
    cal = res["calibration"]
    if cal["umc_mean_busy"] and res["workload"]["umc_mean_busy"] is not None:
        per = cal["copy_GBps"] / cal["umc_mean_busy"]
        res["estimate"] = {"GBps_per_umc_pct": per,
                           "workload_HBM_GBps_busy": per * res["workload"]["umc_mean_busy"]}
    res["samples"] = s.rows
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("samples", "workload_stdout_tail")}, indent=1))


if __name__ == "__main__":
    main()
