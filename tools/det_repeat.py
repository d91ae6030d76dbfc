#!/usr/bin/env python3
"""Repeatability check (GPU box): render the same frame several times with
fresh renderers and count the pixels that differ from the first render.
usage: tools/det_repeat.py [--config c5|c4|c3|c2] [--runs N] [--precise]
(how the path kernel's order-dependent pixel was found)"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "metal-renderer_amd"))
import mrt  # noqa: E402

CASES = {"c2": ("cornellbox", 0, 1920, 1080, 4, 64), "c3": ("CornellBox-Water-plastic", 0, 1920, 1080, 8, 256),
         "c4": ("cornellbox", 1 << 20, 1920, 1080, 4, 64), "c5": ("cornellbox", 1 << 20, 3840, 2160, 8, 256)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="c5", choices=sorted(CASES))
    p.add_argument("--runs", type=int, default=4)
    p.add_argument("--precise", action="store_true")
    a = p.parse_args()
    scene, proc, W, H, L, F = CASES[a.config]
    sc = mrt.Scene(scene, procedural_triangles=proc, device=0)
    imgs = []
    for _ in range(a.runs):
        r = mrt.Renderer(sc, W, H, L, precise=a.precise)
        r.draw(F)
        imgs.append(r.read_image())
        r.close()
    for i, b in enumerate(imgs[1:], 1):
        d = (b[..., :3] != imgs[0][..., :3]).any(-1)
        print(f"{a.config} {'precise' if a.precise else 'fast'} run {i}: {int(d.sum())} pixels differ",
              list(zip(*np.nonzero(d)))[:3], flush=True)


if __name__ == "__main__":
    main()
