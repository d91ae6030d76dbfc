"""CPU check of the camera-ray candidate lists (csrc/primary.cpp): for every
pixel and many noise jitters (the extremes included) the brute-force nearest
triangle of the camera ray — formed and tested with the kernels' float
arithmetic, IEEE (precise build) and with the fast build's FMA contraction and
approximate reciprocals — is in its 8x8 block's list (tools/primary_check.cpp).  The GPU
side (bitwise equality with the traversal) is tests/test_gpu_primary.py."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "metal-renderer_amd", "csrc")
SCENES = os.path.join(ROOT, "metal-renderer_amd", "scenes")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("primary") / "primary_check")
    srcs = [os.path.join(ROOT, "tools", "primary_check.cpp")] + [os.path.join(CSRC, f + ".cpp")
                                                                   for f in ("scene", "bvh", "primary")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, "-o", exe] + srcs, check=True)
    return exe


@pytest.mark.parametrize("scene,W,H,jitters,cap,fast", [
    ("cornellbox", 320, 180, 8, 12, 0),
    ("cornellbox", 97, 61, 32, 12, 0),      # partial blocks at the right and top edges
    ("cornellbox", 1920, 1080, 0, 12, 0),   # the C2 frame: the nine jitter extremes per pixel
    ("cornellbox", 2, 2, 64, 40, 0),       # one block: the whole image plane
    ("CornellBox-Water-plastic", 160, 90, 2, 40, 0),
    # the fast build's arithmetic (FMA contraction, approximate rcp / rsq: ~9x
    # slower to emulate, so smaller frames)
    ("cornellbox", 320, 180, 8, 12, 1),
    ("cornellbox", 97, 61, 32, 12, 1),
    ("cornellbox", 480, 270, 0, 12, 1),     # a quarter of the C2 frame's pixels, jitter extremes
    ("cornellbox", 2, 2, 64, 40, 1),
    ("CornellBox-Water-plastic", 64, 36, 2, 40, 1),
])
def test_lists_are_conservative(checker, scene, W, H, jitters, cap, fast):
    out = subprocess.run([checker, os.path.join(SCENES, scene + ".obj"), str(W), str(H), str(jitters), "0", str(cap),
                          str(fast)], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    words = out.stdout.split()
    assert words[0] == "violations" and words[1] == "0", out.stdout
    listed = int(words[words.index("listed") + 1])
    assert listed > 0, out.stdout


def test_lists_skip_dense_scenes(checker):
    """A 1M-triangle scene (C4) is too dense for lists: none are built and
    every block traverses."""
    out = subprocess.run([checker, os.path.join(SCENES, "cornellbox.obj"), "320", "180", "1", "1048576", "12"],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "lists not built" in out.stdout
