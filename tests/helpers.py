"""Test helpers: device buffers (torch as plumbing), image metrics, golden data."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
SEED = 0x6D6574616C2D7274


def to_dev(arr: np.ndarray):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()).cuda()


def from_dev(t, dtype, count=None) -> np.ndarray:
    import torch
    torch.cuda.synchronize()
    a = t.cpu().numpy().view(dtype)
    return a if count is None else a[:count]


def dev_ptr(t) -> int:
    return int(t.data_ptr())


def pixel_metrics(gpu_img: np.ndarray, ref_img: np.ndarray):
    """Per-pixel relative L2 (||g-c|| / (||c|| + 1e-3)) over RGB,
    NaN-aware (a pixel NaN in both counts as matching).  Returns
    (rel_l2 per pixel, whole-image relative RMSE, bit-identical fraction)."""
    g = gpu_img[..., :3].astype(np.float64)
    c = ref_img[..., :3].astype(np.float64)
    both_nan = np.isnan(g).any(-1) & np.isnan(c).any(-1)
    g = np.where(np.isnan(g), 0.0, g)
    c = np.where(np.isnan(c), 0.0, c)
    d = np.sqrt(((g - c) ** 2).sum(-1))
    rel = d / (np.sqrt((c ** 2).sum(-1)) + 1e-3)
    rel = np.where(both_nan, 0.0, rel)
    rmse = np.sqrt(((g - c) ** 2).mean()) / (np.sqrt((c ** 2).mean()) + 1e-12)
    same = (gpu_img[..., :3].view(np.uint32) == ref_img[..., :3].view(np.uint32)).all(-1) | both_nan
    return rel, rmse, same.mean()


def golden_stats():
    with open(os.path.join(GOLDEN, "golden_stats.json")) as f:
        return json.load(f)


def golden_blocks(name: str) -> np.ndarray:
    with np.load(os.path.join(GOLDEN, "goldens.npz")) as z:
        return z[name]


def banner_mask(h: int, w: int) -> np.ndarray:
    m = np.ones((h, w), bool)
    m[int(585 * h / 600):, int(680 * w / 800):] = False
    return m


def compare_to_golden(img_bottom_up: np.ndarray, name: str):
    """Banner-masked mean RGB ratio and 40x30 block relative MAE of a render
    (our row 0 = bottom) against a Mitsuba golden (renderer/Media/reference)."""
    H, W = img_bottom_up.shape[:2]
    ours = img_bottom_up[::-1, :, :3].astype(np.float64)
    m = banner_mask(H, W)
    mean_ours = ours[m].mean(0)
    st = golden_stats()[name]
    mean_gold = np.array(st["mean_rgb"])
    bh, bw = H // 30, W // 40
    blocks = np.where(m[..., None], ours, 0.0)[: 30 * bh, : 40 * bw].reshape(30, bh, 40, bw, 3).mean((1, 3))
    gold = golden_blocks(name).astype(np.float64)
    block_rel_mae = np.abs(blocks - gold).mean() / gold.mean()
    return mean_ours / mean_gold, block_rel_mae


def host_threads(cap: int = 16) -> int:
    """Oracle threads: the CPUs this process may run on, at most `cap` (the
    GPU box's CPU share for one GPU is 16; os.cpu_count() there reports the
    whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(cap, n))
