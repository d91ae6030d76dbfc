"""GPU: the wave-local streaming wavefront (kernels.hip::stream_kernel) —
every bounce of a frame batch in one launch, each wave running 64 rays of one
bounce at a time from its own per-level queues — renders exactly what one
launch per bounce (bounce_kernel, MRT_STREAM=0) renders.

Rays carry their pixel slot, so the order in which a wave runs them never
changes a path: images and active-ray counts must be bitwise equal, in both
builds, for every path length, ragged frame, tile shard and batch size
(renderer/Renderer.mm:500-585 is the per-bounce loop both restate)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _render(mrt_mod, monkeypatch, scene, W, H, L, frames, chain, precise, shard=(0, 1), batch=None, draws=1):
    monkeypatch.setenv("MRT_STREAM", "1" if chain else "0")
    if batch:
        monkeypatch.setenv("MRT_BATCH", str(batch))
    else:
        monkeypatch.delenv("MRT_BATCH", raising=False)
    r = mrt_mod.Renderer(scene, W, H, L, precise=precise, shard_rank=shard[0], shard_count=shard[1])
    for _ in range(draws):
        r.draw(frames)
    img, st = r.read_image(), r.stats()
    r.close()
    return img, st


@pytest.fixture(scope="module")
def boxes(mrt_mod):
    return {name: mrt_mod.Scene(name) for name in ("cornellbox", "white-box")}


@pytest.mark.parametrize("precise", [True, False])
@pytest.mark.parametrize("scene,W,H,L", [("cornellbox", 64, 48, 4), ("cornellbox", 333, 97, 7),
                                         ("white-box", 200, 120, 2), ("cornellbox", 96, 64, 1)])
def test_stream_equals_per_bounce_launches(gpu, mrt_mod, monkeypatch, boxes, precise, scene, W, H, L):
    a, sa = _render(mrt_mod, monkeypatch, boxes[scene], W, H, L, 3, True, precise)
    b, sb = _render(mrt_mod, monkeypatch, boxes[scene], W, H, L, 3, False, precise)
    assert sa["kernel"] == 2 and sb["kernel"] == 0
    assert np.isfinite(a).all() and a[..., :3].max() > 0
    assert a.tobytes() == b.tobytes()
    assert sa["active_ray_bounces"] == sb["active_ray_bounces"]
    assert sa["kernel_launches"] == 1 and sb["kernel_launches"] == L


@pytest.mark.parametrize("shard", [(0, 3), (2, 3), (5, 8)])
def test_stream_tile_shards(gpu, mrt_mod, monkeypatch, boxes, shard):
    """Small shares are what the single launch is for (one GPU's 1/8 of a
    frame): each rank's tiles render bitwise as with per-bounce launches."""
    a, sa = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 520, 300, 4, 4, True, True, shard=shard)
    b, sb = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 520, 300, 4, 4, False, True, shard=shard)
    assert a.tobytes() == b.tobytes() and sa["active_ray_bounces"] == sb["active_ray_bounces"]


def test_stream_batches_and_draws(gpu, mrt_mod, monkeypatch, boxes):
    """Several batches per draw (one launch each, the per-wave queues reused)
    and consecutive draws: bitwise as per-bounce."""
    a, sa = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 160, 96, 5, 7, True, False, batch=3, draws=2)
    b, sb = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 160, 96, 5, 7, False, False, batch=3, draws=2)
    assert sa["kernel_launches"] == 2 * 3 and sb["kernel_launches"] == 2 * 3 * 5
    assert a.tobytes() == b.tobytes() and sa["active_ray_bounces"] == sb["active_ray_bounces"]


def test_stream_with_frames_in_flight(gpu, mrt_mod, monkeypatch, boxes):
    """Waves never wait for each other, so launches of different frame
    batches may share the GPU: frames in flight stay bitwise."""
    a, sa = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 200, 120, 4, 7, True, False, batch=2, draws=2)
    monkeypatch.setenv("MRT_INFLIGHT", "3")
    b, sb = _render(mrt_mod, monkeypatch, boxes["cornellbox"], 200, 120, 4, 7, True, False, batch=2, draws=2)
    assert sa["kernel"] == 2 and sb["kernel"] == 2
    assert a.tobytes() == b.tobytes() and sa["active_ray_bounces"] == sb["active_ray_bounces"]


def test_stray_kernel_env_ignored_without_mrt_diag(gpu, mrt_mod, monkeypatch):
    """A stray MRT_KERNEL / MRT_INFLIGHT / MRT_BATCH in the environment does not
    change the product's kernel choice or streams unless MRT_DIAG=1."""
    sc = mrt_mod.Scene("cornellbox")
    monkeypatch.delenv("MRT_DIAG", raising=False)
    monkeypatch.delenv("MRT_KERNEL", raising=False)
    monkeypatch.delenv("MRT_INFLIGHT", raising=False)
    r = mrt_mod.Renderer(sc, 96, 64, 4)
    want = (r.stats()["kernel"], r.stats()["inflight"])
    r.draw(2)
    img = r.read_image()
    r.close()
    assert want[0] == 2   # the streaming wavefront for an all-in-LDS scene
    monkeypatch.setenv("MRT_KERNEL", "wave")
    monkeypatch.setenv("MRT_INFLIGHT", "3")
    monkeypatch.setenv("MRT_BATCH", "1")
    r = mrt_mod.Renderer(sc, 96, 64, 4)
    assert (r.stats()["kernel"], r.stats()["inflight"]) == want
    r.draw(2)
    assert r.read_image().tobytes() == img.tobytes()
    r.close()
    monkeypatch.setenv("MRT_DIAG", "1")   # now they apply (MRT_STREAM=0 would select kernel 0 as well)
    monkeypatch.setenv("MRT_STREAM", "0")
    r = mrt_mod.Renderer(sc, 96, 64, 4)
    assert (r.stats()["kernel"], r.stats()["inflight"]) == (0, 3)
    r.close()
