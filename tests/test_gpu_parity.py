"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Precise build (MRT_FLAG_PRECISE): IEEE binary32, no FMA contraction, sin/cos
correctly rounded — expected to match the oracle bit for bit; the gate is the
BASELINE.md parity criterion (per-pixel relative L2 <= 1e-4 on >= 99.9 % of
pixels, whole-image relative RMSE <= 1e-3), stage buffers byte-identical on
>= 99.9 % of records.  Fast build: per-pixel relative L2 <= 1e-2 on >= 99 %.
"""
import numpy as np
import pytest

from helpers import SEED, dev_ptr, from_dev, pixel_metrics, to_dev

pytestmark = pytest.mark.gpu


def _scene(mrt_mod, name, cache={}):
    if name not in cache:
        cache[name] = mrt_mod.Scene(name)
    return cache[name]


def _oscene(oracle_mod, mrt_mod, name, cache={}):
    if name not in cache:
        cache[name] = oracle_mod.OracleScene(mrt_mod.scene_path(name))
    return cache[name]


@pytest.mark.parametrize("W,H", [(64, 48), (257, 131)])
def test_raygen_bitexact(gpu, mrt_mod, oracle_mod, W, H):
    sc = _scene(mrt_mod, "cornellbox")
    noise = oracle_mod.noise_table(SEED, 3)
    ref = oracle_mod.raygen(W, H, noise)
    d_noise = to_dev(noise)
    d_rays = to_dev(np.zeros(W * H, oracle_mod.RAY_DTYPE))
    mrt_mod.raygen(sc, W, H, dev_ptr(d_noise), dev_ptr(d_rays), precise=True)
    got = from_dev(d_rays, oracle_mod.RAY_DTYPE)
    assert got.tobytes() == ref.tobytes()


def _random_rays(oracle_mod, n, rng):
    r = np.zeros(n, oracle_mod.RAY_DTYPE)
    r["origin"] = rng.uniform([-0.95, 0.05, -0.95], [0.95, 1.95, 2.3], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r["direction"] = d.astype(np.float32)
    r["maxDistance"] = np.float32(np.inf)
    r["maxDistance"][::17] = -1.0                       # disabled rays
    r["maxDistance"][5::23] = rng.uniform(0.01, 1.0, size=len(r["maxDistance"][5::23]))
    # axis-aligned directions (zero components) and rays starting on surfaces
    r["direction"][1::31] = np.array([0.0, 1.0, 0.0], np.float32)
    r["direction"][2::31] = np.array([0.0, 0.0, -1.0], np.float32)
    r["origin"][3::37, 1] = 0.0
    return r


@pytest.mark.parametrize("scene", ["cornellbox", "white-box", "CornellBox-Water-plastic"])
@pytest.mark.parametrize("precise", [True, False])
def test_intersect_matches_bruteforce(gpu, mrt_mod, oracle_mod, scene, precise):
    """BVH4 traversal == brute-force MPS nearest-hit semantics (t, primitive,
    u, v)."""
    sc, osc = _scene(mrt_mod, scene), _oscene(oracle_mod, mrt_mod, scene)
    rng = np.random.default_rng(7)
    # NumPy 2 repacks padded structured dtypes in concatenate: restore the 80-B layout
    rays = np.concatenate([_random_rays(oracle_mod, 6000, rng),
                           oracle_mod.raygen(80, 60, oracle_mod.noise_table(SEED, 0))]).astype(oracle_mod.RAY_DTYPE)
    assert rays.dtype.itemsize == 80
    ref = osc.intersect(rays)
    d_rays = to_dev(rays)
    d_out = to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
    mrt_mod.intersect(sc, dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=precise)
    got = from_dev(d_out, oracle_mod.ISECT_DTYPE)
    hit_ref, hit_got = ref["distance"] >= 0, got["distance"] >= 0
    if precise:
        diff = np.nonzero((got.view(np.uint32).reshape(-1, 4) != ref.view(np.uint32).reshape(-1, 4)).any(1))[0]
        assert len(diff) == 0, f"{len(diff)} mismatching intersections, first {diff[:10]}"
    else:
        agree = (hit_ref == hit_got) & (~hit_ref | (got["triangleIndex"] == ref["triangleIndex"]))
        assert agree.mean() >= 0.999
        both = hit_ref & hit_got & agree
        np.testing.assert_allclose(got["distance"][both], ref["distance"][both], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("scene,L", [("cornellbox", 8), ("cornellbox", 2), ("CornellBox-Water-plastic", 8)])
def test_stage_pipeline_bitexact(gpu, mrt_mod, oracle_mod, scene, L):
    """One frame through the stage ABI (raygen, L x {intersect, shade, intersect,
    resolve}, accumulate) in lockstep with the oracle's stages — the
    reference's own dispatch order (renderer/Renderer.mm:500-585)."""
    W, H = 48, 40
    sc, osc = _scene(mrt_mod, scene), _oscene(oracle_mod, mrt_mod, scene)
    f = 4
    n_rg = oracle_mod.noise_table(SEED, f)
    rays = oracle_mod.raygen(W, H, n_rg)
    srays = np.zeros(W * H, oracle_mod.SRAY_DTYPE)
    img = np.zeros((H, W, 4), np.float32)
    d_rays = to_dev(rays)
    d_srays = to_dev(srays)
    d_isect = to_dev(np.zeros(W * H, oracle_mod.ISECT_DTYPE))
    d_img = to_dev(img)
    for i in range(L):
        noise = oracle_mod.noise_table(SEED, oracle_mod.noise_frame_for(f, i))
        d_noise = to_dev(noise)
        is_ref = osc.intersect(rays)
        mrt_mod.intersect(sc, dev_ptr(d_rays), 80, W * H, dev_ptr(d_isect))
        assert from_dev(d_isect, oracle_mod.ISECT_DTYPE).tobytes() == is_ref.tobytes(), f"path intersect {i}"
        osc.shade(W, H, f, L, noise, is_ref, rays, srays)
        mrt_mod.shade(sc, W, H, f, L, dev_ptr(d_noise), dev_ptr(d_isect), dev_ptr(d_rays), dev_ptr(d_srays))
        g_rays, g_srays = from_dev(d_rays, oracle_mod.RAY_DTYPE), from_dev(d_srays, oracle_mod.SRAY_DTYPE)
        rec_same = (g_rays.view(np.uint8).reshape(-1, 80) == rays.view(np.uint8).reshape(-1, 80)).all(1)
        assert rec_same.mean() >= 0.999, f"shade {i}: {np.count_nonzero(~rec_same)} ray records differ"
        assert g_srays.tobytes() == srays.tobytes() or \
            (g_srays.view(np.uint8).reshape(-1, 48) == srays.view(np.uint8).reshape(-1, 48)).all(1).mean() >= 0.999
        # continue from the oracle's state so a rare flip cannot cascade
        d_rays.copy_(to_dev(rays))
        d_srays.copy_(to_dev(srays))
        is2 = osc.intersect(srays)
        mrt_mod.intersect(sc, dev_ptr(d_srays), 48, W * H, dev_ptr(d_isect))
        assert from_dev(d_isect, oracle_mod.ISECT_DTYPE).tobytes() == is2.tobytes(), f"shadow intersect {i}"
        oracle_mod.resolve(is2, rays, srays)
        mrt_mod.resolve_shadow(sc, W * H, dev_ptr(d_isect), dev_ptr(d_rays), dev_ptr(d_srays))
        assert from_dev(d_rays, oracle_mod.RAY_DTYPE).tobytes() == rays.tobytes(), f"resolve {i}"
    oracle_mod.accumulate(0, rays, img)
    mrt_mod.accumulate(sc, W, H, 0, dev_ptr(d_rays), dev_ptr(d_img))
    assert from_dev(d_img, np.float32).tobytes() == img.tobytes()


def _render_gpu(mrt_mod, sc, W, H, L, frames, precise, shard=(0, 1), seed=SEED):
    r = mrt_mod.Renderer(sc, W, H, L, seed=seed, precise=precise, shard_rank=shard[0], shard_count=shard[1])
    r.draw(frames)
    img = r.read_image()
    st = r.stats()
    r.close()
    return img, st


@pytest.mark.parametrize("scene,W,H,L,frames", [
    ("cornellbox", 64, 64, 1, 2),
    ("cornellbox", 64, 64, 2, 3),
    ("cornellbox", 100, 70, 4, 3),
    ("cornellbox", 96, 80, 8, 4),
    ("white-box", 80, 60, 8, 2),
    ("CornellBox-Water-plastic", 48, 36, 8, 2),
    ("CornellBox-Water-mirror", 40, 30, 3, 2),
])
def test_render_parity_precise(gpu, mrt_mod, oracle_mod, scene, W, H, L, frames):
    sc, osc = _scene(mrt_mod, scene), _oscene(oracle_mod, mrt_mod, scene)
    ref, A_ref = osc.render(W, H, L, SEED, frames, threads=8)
    img, st = _render_gpu(mrt_mod, sc, W, H, L, frames, precise=True)
    rel, rmse, same = pixel_metrics(img, ref)
    print(f"{scene} {W}x{H} L={L} f={frames}: bit-identical {same:.5f}, rel<=1e-4 {np.mean(rel <= 1e-4):.5f}, "
          f"rmse {rmse:.2e}, A gpu {st['active_ray_bounces']} oracle {A_ref}")
    assert np.mean(rel <= 1e-4) >= 0.999
    assert rmse <= 1e-3
    assert abs(st["active_ray_bounces"] - A_ref) <= max(2, A_ref // 1000)
    assert st["paths"] == W * H * frames


@pytest.mark.parametrize("W,H,L,frames", [(2, 2, 4, 3), (7, 3, 8, 2), (2, 130, 4, 2), (130, 2, 4, 2),
                                          (65, 65, 1, 2), (63, 129, 8, 1)])
def test_render_parity_tiny_and_ragged(gpu, mrt_mod, oracle_mod, W, H, L, frames):
    """Edge shapes: the smallest image (2x2: rayGenerator divides by W - 1 and
    H - 1, Shaders.metal:75-103, so 1-pixel sizes are rejected with
    MRT_ERR_INVALID, test_host), two-pixel rows / columns, sizes one off a
    64x64 tile and an 8x8 candidate-list block (partial tiles, partial
    waves, the last tile of a row and of the image): the precise build meets
    test_render_parity_precise's gates against the oracle (the bit-identical
    share is printed), every pixel is rendered exactly once per frame, and
    the image's alpha is 1 everywhere."""
    sc, osc = _scene(mrt_mod, "cornellbox"), _oscene(oracle_mod, mrt_mod, "cornellbox")
    ref, A_ref = osc.render(W, H, L, SEED, frames, threads=8)
    img, st = _render_gpu(mrt_mod, sc, W, H, L, frames, precise=True)
    assert img.shape[:2] == (H, W)
    rel, rmse, same = pixel_metrics(img, ref)
    print(f"{W}x{H} L={L} f={frames}: bit-identical {same:.5f}, A gpu {st['active_ray_bounces']} oracle {A_ref}")
    assert np.mean(rel <= 1e-4) >= 0.999 and rmse <= 1e-3   # the gates of test_render_parity_precise
    assert abs(st["active_ray_bounces"] - A_ref) <= max(2, A_ref // 1000)
    assert st["paths"] == W * H * frames
    assert np.all(img[..., 3] == 1.0)


@pytest.mark.parametrize("W,H,shards", [(2, 2, 8), (70, 10, 4), (64, 64, 3)])
def test_shards_with_no_tile(gpu, mrt_mod, W, H, shards):
    """Tile shares of an image with fewer 64x64 tiles than ranks: a rank that
    owns no tile draws (no-op kernels, no error) and renders no path; the
    shares still sum to the 1-GPU image bitwise."""
    sc = _scene(mrt_mod, "cornellbox")
    full, _ = _render_gpu(mrt_mod, sc, W, H, 4, 2, precise=True)
    acc = np.zeros_like(full)
    paths, empty = 0, 0
    for k in range(shards):
        part, st = _render_gpu(mrt_mod, sc, W, H, 4, 2, precise=True, shard=(k, shards))
        acc += part
        paths += st["paths"]
        empty += st["paths"] == 0
    assert paths == W * H * 2
    tiles = ((W + 63) // 64) * ((H + 63) // 64)   # round-robin: ranks >= tiles own none
    assert empty == max(0, shards - tiles)
    assert np.array_equal(acc[..., :3], full[..., :3])


@pytest.mark.parametrize("W,H", [(1, 1), (1, 64), (64, 1), (0, 8)])
def test_one_pixel_sizes_rejected(gpu, mrt_mod, W, H):
    """rayGenerator divides by (W - 1) and (H - 1) (Shaders.metal:75-103): a
    renderer (and a resize) below 2x2 is refused with an error, not rendered
    as NaN directions."""
    sc = _scene(mrt_mod, "cornellbox")
    with pytest.raises(mrt_mod.MrtError):
        mrt_mod.Renderer(sc, W, H, 4)
    r = mrt_mod.Renderer(sc, 8, 8, 4)
    with pytest.raises(mrt_mod.MrtError):
        r.resize(W, H)
    r.draw(1)   # still usable at its old size
    r.close()


def test_zero_frame_draw_is_a_noop(gpu, mrt_mod):
    """draw(0) enqueues nothing: the image, frame index and statistics are
    unchanged (mrt_renderer_draw_n with n = 0, as a MAX_FRAMES-capped draw)."""
    sc = _scene(mrt_mod, "cornellbox")
    r = mrt_mod.Renderer(sc, 48, 32, 4, seed=SEED, precise=True)
    r.draw(2)
    a, sa = r.read_image(), r.stats()
    r.draw(0)
    b, sb = r.read_image(), r.stats()
    r.close()
    assert a.tobytes() == b.tobytes()
    assert sa["frame_index"] == sb["frame_index"] and sa["paths"] == sb["paths"]


@pytest.mark.parametrize("scene,L", [("cornellbox", 4), ("CornellBox-Water-plastic", 8)])
def test_render_parity_fast(gpu, mrt_mod, oracle_mod, scene, L):
    W, H, frames = 64, 48, 3
    sc, osc = _scene(mrt_mod, scene), _oscene(oracle_mod, mrt_mod, scene)
    ref, _ = osc.render(W, H, L, SEED, frames, threads=8)
    img, _ = _render_gpu(mrt_mod, sc, W, H, L, frames, precise=False)
    rel, rmse, same = pixel_metrics(img, ref)
    print(f"fast {scene}: bit-identical {same:.4f}, rel<=1e-2 {np.mean(rel <= 1e-2):.5f}, rmse {rmse:.2e}")
    assert np.mean(rel <= 1e-2) >= 0.99


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_shard_invariance(gpu, mrt_mod, shards):
    """Tile-sharded renders summed == the 1-GPU image, bitwise."""
    sc = _scene(mrt_mod, "cornellbox")
    W, H, L, frames = 200, 150, 4, 2
    full, st_full = _render_gpu(mrt_mod, sc, W, H, L, frames, precise=False)
    acc = np.zeros_like(full)
    paths = 0
    for k in range(shards):
        part, st = _render_gpu(mrt_mod, sc, W, H, L, frames, precise=False, shard=(k, shards))
        acc[..., :3] += part[..., :3]
        acc[..., 3] += part[..., 3]
        paths += st["paths"]
    assert paths == W * H * frames
    assert np.array_equal(acc[..., :3], full[..., :3])
    assert np.all(acc[..., 3] == 1.0)


@pytest.mark.parametrize("scene", ["cornellbox", "CornellBox-Water-plastic"])
def test_frame_batching_invariance(gpu, mrt_mod, monkeypatch, scene):
    """Frames per launch (MRT_BATCH) and the split of frames across draw calls
    change the launch structure, not the image: bitwise equal, same A."""
    sc = _scene(mrt_mod, scene)
    W, H, L = 136, 72, 5
    out = {}
    for batch, draws in [(1, (7,)), (3, (7,)), (8, (7,)), (64, (7,)), (3, (4, 3)), (2, (1, 5, 1))]:
        monkeypatch.setenv("MRT_BATCH", str(batch))
        r = mrt_mod.Renderer(sc, W, H, L, shard_rank=1, shard_count=2)
        for d in draws:
            r.draw(d)
        out[(batch, draws)] = (r.read_image(), r.stats()["active_ray_bounces"])
        r.close()
    ref_img, ref_a = out[(1, (7,))]
    assert np.isfinite(ref_img).all() and ref_img[..., :3].max() > 0
    for key, (img, a) in out.items():
        assert img.tobytes() == ref_img.tobytes(), key
        assert a == ref_a, key


def test_deterministic_and_reset(gpu, mrt_mod):
    sc = _scene(mrt_mod, "cornellbox")
    r = mrt_mod.Renderer(sc, 320, 240, 4)
    r.draw(3)
    a = r.read_image()
    r.reset()
    r.draw(3)
    b = r.read_image()
    r.resize(160, 120)
    r.draw(1)
    c = r.read_image()
    st = r.stats()
    r.close()
    assert a.tobytes() == b.tobytes()
    assert c.shape == (120, 160, 4) and st["frame_index"] == 1 and np.isfinite(c).all()


def test_save_image_roundtrip(gpu, mrt_mod, tmp_path):
    import exr
    sc = _scene(mrt_mod, "cornellbox")
    r = mrt_mod.Renderer(sc, 64, 48, 2)
    r.draw(2)
    img = r.read_image()
    r.save_current_image(str(tmp_path / "out.exr"))
    r.save_current_image(str(tmp_path / "out.pfm"))
    r.close()
    back = exr.read_rgb(str(tmp_path / "out.exr"))[::-1]   # EXR is top-down
    assert np.array_equal(back, img[..., :3])
    with open(tmp_path / "out.pfm", "rb") as f:
        header = f.readline() + f.readline() + f.readline()
        data = np.frombuffer(f.read(), "<f4").reshape(48, 64, 3)
    assert header.startswith(b"PF") and np.array_equal(data, img[..., :3])


@pytest.mark.parametrize("W,H,count", [(200, 150, 3), (1920, 1080, 8), (64, 64, 1)])
def test_tiles_pack_unpack(gpu, mrt_mod, W, H, count):
    """Device tile pack (multi-GPU exchange) == its numpy restatement; unpacking
    every shard's packed tiles rebuilds the image bitwise."""
    rng = np.random.default_rng(W + count)
    img = rng.standard_normal((H, W, 4)).astype(np.float32)
    d_img = to_dev(img)
    d_out = to_dev(np.zeros_like(img))
    for k in range(count):
        n = mrt_mod.tiles_packed_floats(W, H, k, count)
        d_p = to_dev(np.zeros(n, np.float32))
        mrt_mod.tiles_pack(dev_ptr(d_img), W, H, k, count, dev_ptr(d_p))
        got = from_dev(d_p, np.float32)
        assert got.tobytes() == mrt_mod.tiles_pack_host(img, k, count).tobytes()
        mrt_mod.tiles_unpack(dev_ptr(d_p), W, H, k, count, dev_ptr(d_out))
    assert from_dev(d_out, np.float32).tobytes() == img.tobytes()


@pytest.mark.parametrize("flags", [0, 1, 2, 3, 1 << 8, (2 << 8) | 2, (3 << 8) | 1, (4 << 8) | 3])
def test_display_blit(gpu, mrt_mod, oracle_mod, flags):
    """blitFragment (Shaders.metal:33-70) against its numpy restatement:
    tone map, sRGB, and the four golden-comparison modes."""
    rng = np.random.default_rng(flags)
    H, W = 37, 53
    img = (rng.standard_normal((H, W, 4)) * 2).astype(np.float32)
    ref = np.abs(rng.standard_normal((H, W, 4))).astype(np.float32)
    d_img, d_ref, d_out = to_dev(img), to_dev(ref), to_dev(np.zeros_like(img))
    mrt_mod.display(dev_ptr(d_img), dev_ptr(d_out), W, H, flags, reference_ptr=dev_ptr(d_ref) if flags >> 8 else None)
    got = from_dev(d_out, np.float32).reshape(H, W, 4)
    want = oracle_mod.display(img, ref, flags, 10.0)
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=2e-5)


def test_max_frames(gpu, mrt_mod):
    """MAX_FRAMES (Renderer.mm:589-590): draws past the limit change nothing."""
    sc = _scene(mrt_mod, "cornellbox")
    r = mrt_mod.Renderer(sc, 64, 48, 2)
    r.set_max_frames(3)
    r.draw(2)
    r.draw(5)
    a = r.read_image()
    st = r.stats()
    r.draw(1)
    b = r.read_image()
    r.close()
    r2 = mrt_mod.Renderer(sc, 64, 48, 2)
    r2.draw(3)
    c = r2.read_image()
    r2.close()
    assert st["frame_index"] == 3 and a.tobytes() == b.tobytes() == c.tobytes()


def test_pack_on_renderer_stream(gpu, mrt_mod):
    """The overlapped exchange's pattern (bench.py): a shard renderer's owned
    tiles packed on the renderer's stream behind its draw, completion observed
    through a libmrt event, equal to the packed tiles of the synchronised image."""
    W, H, count = 200, 130, 3
    scene = _scene(mrt_mod, "cornellbox")
    d_img = to_dev(np.zeros((H, W, 4), np.float32))
    r = mrt_mod.Renderer(scene, W, H, 2, shard_rank=1, shard_count=count, image_ptr=dev_ptr(d_img))
    n = mrt_mod.tiles_packed_floats(W, H, 1, count)
    d_p = to_dev(np.zeros(n, np.float32))
    ev = mrt_mod.Event()
    r.draw(3)
    mrt_mod.tiles_pack(dev_ptr(d_img), W, H, 1, count, dev_ptr(d_p), stream=r.stream(), sync=False)
    ev.record(r.stream())
    ev.synchronize()
    got = from_dev(d_p, np.float32)
    r.sync()
    img = from_dev(d_img, np.float32).reshape(H, W, 4)
    ev.close()
    r.close()
    assert np.any(img != 0)
    assert got.tobytes() == mrt_mod.tiles_pack_host(img, 1, count).tobytes()


def test_golden_compare_display(gpu, mrt_mod, oracle_mod):
    """COMPARISON_MODE end to end from the C ABI (Renderer.mm:162-253 +
    Shaders.metal:53-66): load the reference's white-box-2 golden with
    libmrt's EXR reader into the renderer, blit each compare mode to host
    memory, equal to the numpy restatement of blitFragment on the same
    images."""
    import os
    golden_path = os.path.join(os.path.dirname(__file__), "golden", "white-box-2.exr")
    sc = _scene(mrt_mod, "white-box")
    r = mrt_mod.Renderer(sc, 800, 600, 2)
    r.draw(4)
    img = r.read_image()
    r.load_reference(golden_path)
    gold = mrt_mod.load_exr(golden_path)
    for flags in (0, 1, 3, (1 << 8), (2 << 8) | 1, (3 << 8) | 2, (4 << 8) | 3):
        got = r.display(flags, 10.0)
        want = oracle_mod.display(img, gold, flags, 10.0)
        # the blit runs in the fast build (native exp / pow), the restatement
        # in numpy float32: agreement to ~1e-5 of the displayed value
        np.testing.assert_allclose(got, want, rtol=2e-5, atol=1e-4)
    with pytest.raises(mrt_mod.MrtError, match="reference image"):
        r2 = mrt_mod.Renderer(sc, 64, 48, 2)
        try:
            r2.load_reference(golden_path)
        finally:
            r2.close()
    r.close()


@pytest.mark.parametrize("switch", ["static_noise", "no_accumulate", "debug_material", "all"])
@pytest.mark.parametrize("scene,L", [("cornellbox", 4), ("CornellBox-Water-plastic", 8)])
def test_compile_time_switches_match_oracle(gpu, mrt_mod, oracle_mod, switch, scene, L):
    """The reference's compile-time switches as runtime flags, precise build
    vs the oracle bitwise: ANIMATE_NOISE 0 (Raytracing.h:20, Renderer.mm:
    485-497), ACCUMULATE_IMAGE false (Raytracing.h:14, Shaders.metal:241),
    DEBUG_MATERIAL 1 (Shaders.metal:7,142-147) — over two draws so the
    running mean, frame batches and noise window all take part."""
    W, H, frames = 72, 40, (3, 2)
    on = {k: switch in (k, "all") for k in ("static_noise", "no_accumulate", "debug_material")}
    oflags = ((oracle_mod.STATIC_NOISE if on["static_noise"] else 0) |
              (oracle_mod.NO_ACCUMULATE if on["no_accumulate"] else 0) |
              (oracle_mod.DEBUG_MATERIAL if on["debug_material"] else 0))
    sc, osc = _scene(mrt_mod, scene), _oscene(oracle_mod, mrt_mod, scene)
    ref, A = osc.render(W, H, L, SEED, sum(frames), threads=8, flags=oflags)
    r = mrt_mod.Renderer(sc, W, H, L, precise=True, animate_noise=not on["static_noise"],
                         accumulate_image=not on["no_accumulate"], debug_material=on["debug_material"])
    for n in frames:
        r.draw(n)
    img, st = r.read_image(), r.stats()
    r.close()
    plain, _ = osc.render(W, H, L, SEED, sum(frames), threads=8)
    assert img.tobytes() != plain.tobytes()          # the switch changes the image
    rel, rmse, same = pixel_metrics(img, ref)
    print(f"{switch} {scene}: bit-identical {same:.5f}")
    assert np.mean(rel <= 1e-4) >= 0.999 and rmse <= 1e-3
    assert st["active_ray_bounces"] == A


def test_debug_material_stage_and_no_accumulate_stage(gpu, mrt_mod, oracle_mod):
    """mrt_shade with MRT_FLAG_DEBUG_MATERIAL and mrt_accumulate with
    MRT_FLAG_NO_ACCUMULATE (the stage ABI, B-2) equal the oracle's stages."""
    W, H, L, f = 40, 30, 4, 5
    sc, osc = _scene(mrt_mod, "CornellBox-Water-plastic"), _oscene(oracle_mod, mrt_mod, "CornellBox-Water-plastic")
    rays = oracle_mod.raygen(W, H, oracle_mod.noise_table(SEED, f))
    noise = oracle_mod.noise_table(SEED, oracle_mod.noise_frame_for(f, 0))
    isect = osc.intersect(rays)
    srays = np.zeros(W * H, oracle_mod.SRAY_DTYPE)
    d_rays, d_srays, d_isect, d_noise = to_dev(rays), to_dev(srays), to_dev(isect), to_dev(noise)
    osc.shade(W, H, f, L, noise, isect, rays, srays, oracle_mod.DEBUG_MATERIAL)
    mrt_mod.shade(sc, W, H, f, L, dev_ptr(d_noise), dev_ptr(d_isect), dev_ptr(d_rays), dev_ptr(d_srays),
                  debug_material=True)
    assert from_dev(d_rays, oracle_mod.RAY_DTYPE).tobytes() == rays.tobytes()
    img = np.full((H, W, 4), 0.25, np.float32)
    d_img = to_dev(img)
    oracle_mod.accumulate(7, rays, img, oracle_mod.NO_ACCUMULATE)
    mrt_mod.accumulate(sc, W, H, 7, dev_ptr(d_rays), dev_ptr(d_img), accumulate_image=False)
    assert from_dev(d_img, np.float32).tobytes() == img.tobytes()


def test_c_cli_matches_oracle(gpu, mrt_mod, oracle_mod, tmp_path):
    """The C host (metal-renderer_amd/cli/render.c: includes include/mrt.h,
    links libmrt.so, built by build()) renders cornellbox 64x48, L = 4,
    2 frames, precise, to a PFM that matches the oracle at the BASELINE.md
    gate (the reference's app shell: macos/GameViewController.m:25-27 +
    Renderer.h:3-8)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(mrt_mod.LIB_PATH), "..", "bin", "mrt_render")
    out = tmp_path / "cli.pfm"
    p = subprocess.run([exe, "--scene", "cornellbox", "--w", "64", "--h", "48", "--spp", "2", "--L", "4",
                        "--precise", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    with open(out, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        assert float(f.readline()) < 0   # little endian
        img = np.frombuffer(f.read(), "<f4").reshape(h, w, 3)   # bottom-up rows == ours
    ref, A = _oscene(oracle_mod, mrt_mod, "cornellbox").render(64, 48, 4, SEED, 2, threads=8)
    rel, rmse, same = pixel_metrics(np.concatenate([img, np.ones((h, w, 1), np.float32)], -1), ref)
    assert (w, h) == (64, 48)
    assert np.mean(rel <= 1e-4) >= 0.999 and rmse <= 1e-3
    import json
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["frames"] == 2 and line["active_ray_bounces_rank0"] == A


def test_c_cli_two_ranks_host_exchange(gpu, mrt_mod, tmp_path):
    """mrt_render --gpus 2 --exchange host: two forked ranks (one GPU here;
    RCCL needs one device per rank) render their tiles and rank 0 assembles
    the frame through host memory: equal to the single-rank render bitwise."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(mrt_mod.LIB_PATH), "..", "bin", "mrt_render")
    args = ["--scene", "cornellbox", "--w", "200", "--h", "130", "--spp", "3", "--L", "4"]
    imgs = []
    for extra, name in ((["--gpus", "1"], "a.pfm"), (["--gpus", "2", "--exchange", "host"], "b.pfm")):
        p = subprocess.run([exe] + args + extra + ["--out", str(tmp_path / name)], capture_output=True, text=True,
                           timeout=120)
        assert p.returncode == 0, p.stderr
        imgs.append((tmp_path / name).read_bytes())
    assert imgs[0] == imgs[1]


def test_display_ring_frames_in_flight(gpu, mrt_mod):
    """The facade's frame loop (integration/objc/Renderer.mm): draw, enqueue
    the blit of frame n into slot n % 3, map the slot of frame n - 2 — the
    reference's 3 frames in flight.  Each mapped slot equals the synchronous
    blit of the same frame, bitwise; misuse fails loudly."""
    sc = _scene(mrt_mod, "cornellbox")
    flags = 3   # tone map + sRGB
    want = []
    r = mrt_mod.Renderer(sc, 160, 120, 4)
    for n in range(6):
        r.draw()
        want.append(r.display(flags, 10.0))
    r.close()
    r = mrt_mod.Renderer(sc, 160, 120, 4)
    got = {}
    for n in range(6):
        r.draw()
        r.display_enqueue(n % 3, flags, 10.0)
        if n >= 2:
            got[n - 2] = r.display_map((n - 2) % 3)
    got[4], got[5] = r.display_map(4 % 3), r.display_map(5 % 3)
    for n in range(6):
        assert got[n].tobytes() == want[n].tobytes(), n
    with pytest.raises(mrt_mod.MrtError, match="slot"):
        r.display_enqueue(3)
    r.resize(80, 64)
    with pytest.raises(mrt_mod.MrtError, match="not enqueued"):
        r.display_map(0)
    r.close()

