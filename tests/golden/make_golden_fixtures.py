"""Generate tests/golden/goldens.npz + golden_stats.json from the reference's
Mitsuba goldens (renderer/Media/reference/*.exr).  Runs only where
/root/reference exists (this container); the outputs are committed so the GPU
box never reads the reference.

Fixture contents (data only: inputs/expected outputs):
  * per golden: banner-masked mean linear RGB, peak, and a 40x30 block-mean
    image (20x20-pixel blocks of the 800x600 image, row 0 = TOP, banner
    masked to 0 — the same mask is applied to our renders before comparing).
  * white-box-2.exr: one golden copied unchanged (data; the smallest, 428 KB)
    as the fixture of libmrt's own EXR reader (tests/test_host.py);
  * the scene OBJ/MTL data files the reference ships (renderer/Media/*.obj,
    *.mtl) are copied unchanged into metal-renderer_amd/scenes/: they are the
    product's input data ("scenes in renderer/Media render unchanged"), not
    source code.
"""
from __future__ import annotations

import glob
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import exr  # noqa: E402

REF = "/root/reference/renderer/Media"
BANNER_ROW, BANNER_COL = 585, 680  # Mitsuba banner at rows 590-594, cols 687-794


def banner_mask(h=600, w=800):
    m = np.ones((h, w), bool)
    m[int(BANNER_ROW * h / 600):, int(BANNER_COL * w / 800):] = False
    return m


def block_means(img, bh=20, bw=20):
    H, W, C = img.shape
    return img[: H // bh * bh, : W // bw * bw].reshape(H // bh, bh, W // bw, bw, C).mean((1, 3))


def main():
    stats, blocks = {}, {}
    m = banner_mask()
    for p in sorted(glob.glob(os.path.join(REF, "reference", "*.exr"))):
        name = os.path.basename(p)[:-4]
        im = exr.read_rgb(p)
        stats[name] = {
            "mean_rgb": [float(v) for v in im[m].mean(0)],
            "peak": float(im[m].max()),
            "shape": list(im.shape),
        }
        blocks[name] = block_means(np.where(m[..., None], im, 0.0)).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "goldens.npz"), **blocks)
    with open(os.path.join(HERE, "golden_stats.json"), "w") as f:
        json.dump(stats, f, indent=1, sort_keys=True)
    # scene data files the reference ships (inputs, not source code)
    sdir = os.path.join(os.path.dirname(os.path.dirname(HERE)), "metal-renderer_amd", "scenes")
    os.makedirs(sdir, exist_ok=True)
    for fn in ("cornellbox.obj", "cornellbox.mtl", "white-box.obj", "CornellBox-Water-plastic.obj",
               "CornellBox-Water-plastic.mtl", "CornellBox-Water-mirror.obj", "CornellBox-Water-mirror.mtl",
               "CornellBox-Water.obj", "CornellBox-Water.mtl"):
        shutil.copyfile(os.path.join(REF, fn), os.path.join(sdir, fn))
    shutil.copyfile(os.path.join(REF, "reference", "white-box-2.exr"), os.path.join(HERE, "white-box-2.exr"))
    print(json.dumps(stats, indent=1))


if __name__ == "__main__":
    main()
