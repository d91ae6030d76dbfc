"""Camera-ray candidate lists (csrc/primary.cpp): bounce 0 of the wavefront
kernels tests the 8x8 pixel block's list of triangles instead of traversing
the BVH.  The nearest hit is the (t, primitive) minimum over every triangle a
ray hits, and a list holds every triangle a camera ray of its block can hit,
so the image and the active-ray count must be bit-identical to the traversal's
(MRT_PRIMARY=0) — precise build and fast build alike (the same tri_pair code
runs in both paths)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render(mrt_mod, monkeypatch, scene, W, H, L, frames, primary, precise, stream=True, shard=(0, 1)):
    monkeypatch.setenv("MRT_PRIMARY", "1" if primary else "0")
    monkeypatch.setenv("MRT_BATCH", "2")
    if stream:
        monkeypatch.delenv("MRT_STREAM", raising=False)
    else:
        monkeypatch.setenv("MRT_STREAM", "0")
    r = mrt_mod.Renderer(scene, W, H, L, precise=precise, shard_rank=shard[0], shard_count=shard[1])
    r.draw(frames)
    img, st = r.read_image(), r.stats()
    r.close()
    return img, st


@pytest.mark.parametrize("build", ["precise", "fast"])
@pytest.mark.parametrize("W,H", [(256, 144), (97, 61), (640, 360)])
def test_primary_lists_bitwise(gpu, mrt_mod, monkeypatch, build, W, H):
    sc = mrt_mod.Scene("cornellbox")
    a, sa = _render(mrt_mod, monkeypatch, sc, W, H, 4, 5, True, build == "precise")
    b, sb = _render(mrt_mod, monkeypatch, sc, W, H, 4, 5, False, build == "precise")
    assert sa["primary_blocks"] > 0 and sb["primary_blocks"] == 0, (sa["primary_blocks"], sb["primary_blocks"])
    assert sa["kernel"] == 2
    assert np.isfinite(a).all() and a[..., :3].max() > 0
    if build == "precise":
        assert sa["active_ray_bounces"] == sb["active_ray_bounces"]
        assert a.tobytes() == b.tobytes()
    else:   # fast: FMA contraction may differ between the two code paths
        assert abs(sa["active_ray_bounces"] - sb["active_ray_bounces"]) <= sb["active_ray_bounces"] // 1000
        rel = np.abs(a - b).max(-1) / (np.abs(b).max(-1) + 1e-3)
        assert np.mean(rel <= 1e-2) >= 0.999


@pytest.mark.parametrize("L", [1, 2, 5])
def test_primary_lists_bounce_kernel_and_lengths(gpu, mrt_mod, monkeypatch, L):
    """The per-bounce wavefront (MRT_STREAM=0) uses the lists at bounce 0
    too; L = 1 is camera rays only (emission), the C1 configuration."""
    sc = mrt_mod.Scene("cornellbox")
    for stream in (True, False):
        a, sa = _render(mrt_mod, monkeypatch, sc, 200, 120, L, 3, True, True, stream=stream)
        b, sb = _render(mrt_mod, monkeypatch, sc, 200, 120, L, 3, False, True, stream=stream)
        assert sa["primary_blocks"] > 0
        assert sa["active_ray_bounces"] == sb["active_ray_bounces"]
        assert a.tobytes() == b.tobytes(), (L, stream)


def test_primary_lists_tile_share(gpu, mrt_mod, monkeypatch):
    """Blocks are global pixel blocks: a tile share (rank 1 of 3) reads the
    same lists and renders its tiles exactly as with traversal."""
    sc = mrt_mod.Scene("cornellbox")
    a, sa = _render(mrt_mod, monkeypatch, sc, 300, 200, 4, 4, True, True, shard=(1, 3))
    b, sb = _render(mrt_mod, monkeypatch, sc, 300, 200, 4, 4, False, True, shard=(1, 3))
    assert sa["primary_blocks"] > 0
    assert sa["active_ray_bounces"] == sb["active_ray_bounces"]
    assert a.tobytes() == b.tobytes()


def test_primary_lists_match_oracle(gpu, mrt_mod, oracle_mod, monkeypatch):
    """With the lists on (the default), the precise render is the oracle's
    brute-force render, bit for bit."""
    W, H, L, frames = 120, 90, 4, 3
    sc = mrt_mod.Scene("cornellbox")
    img, st = _render(mrt_mod, monkeypatch, sc, W, H, L, frames, True, True)
    assert st["primary_blocks"] > 0
    ref, A = oracle_mod.OracleScene(mrt_mod.scene_path("cornellbox")).render(W, H, L, mrt_mod.DEFAULT_SEED, frames,
                                                                               threads=4)
    assert st["active_ray_bounces"] == A
    assert img[..., :3].tobytes() == np.ascontiguousarray(ref[..., :3]).tobytes()



@pytest.mark.parametrize("scene", ["CornellBox-Water-plastic", "cornellbox"])
def test_path_kernel_builds_no_lists(gpu, mrt_mod, monkeypatch, scene):
    """The path megakernel refills lanes one at a time; lists there measured
    slower (C3 -4.8 %), so renderers on it build none."""
    monkeypatch.setenv("MRT_KERNEL", "path")
    _, st = _render(mrt_mod, monkeypatch, mrt_mod.Scene(scene), 160, 90, 4, 1, True, True)
    assert st["kernel"] == 1 and st["primary_blocks"] == 0


@pytest.mark.parametrize("scene", ["CornellBox-Water-plastic", "CornellBox-Water-mirror"])
def test_primary_lists_wavefront_specular_scenes(gpu, mrt_mod, monkeypatch, scene):
    """The specular scenes on the per-bounce wavefront (MRT_KERNEL=wave):
    lists at bounce 0, traversal after, bit-identical to traversal only."""
    monkeypatch.setenv("MRT_KERNEL", "wave")
    sc = mrt_mod.Scene(scene)
    a, sa = _render(mrt_mod, monkeypatch, sc, 320, 180, 8, 3, True, True)
    b, sb = _render(mrt_mod, monkeypatch, sc, 320, 180, 8, 3, False, True)
    assert sa["kernel"] == 0 and sa["primary_blocks"] > 0 and sb["primary_blocks"] == 0
    assert sa["active_ray_bounces"] == sb["active_ray_bounces"]
    assert a.tobytes() == b.tobytes()
