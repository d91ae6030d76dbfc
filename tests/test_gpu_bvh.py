"""GPU: the device BVH builders (LBVH and PLOC) and the MPS-shaped
acceleration-structure ABI over raw device buffers (mrt_accel_*), the
replacement for MPSTriangleAccelerationStructure + MPSRayIntersector
(renderer/Renderer.mm:456-469).

Parity anchor: MPS semantics are restated by the oracle's brute-force
nearest hit (cull none, ties -> lowest primitive, distance = -1 on miss or
maxDistance < 0).  A traversal over any conservative BVH must return exactly
that answer, so every comparison here is bitwise (precise build)."""
import numpy as np
import pytest

from helpers import SEED, dev_ptr, from_dev, pixel_metrics, to_dev

pytestmark = pytest.mark.gpu


def _rays(oracle_mod, n, rng, lo=(-0.95, 0.05, -0.95), hi=(0.95, 1.95, 2.3)):
    r = np.zeros(n, oracle_mod.RAY_DTYPE)
    r["origin"] = rng.uniform(lo, hi, size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r["direction"] = d.astype(np.float32)
    r["maxDistance"] = np.float32(np.inf)
    r["maxDistance"][::17] = -1.0
    r["maxDistance"][5::23] = rng.uniform(0.01, 1.0, size=len(r["maxDistance"][5::23]))
    r["direction"][1::31] = np.array([0.0, 1.0, 0.0], np.float32)
    r["origin"][3::37, 1] = 0.0
    return r


def _isect_bits(a):
    return a.view(np.uint32).reshape(-1, 4)


DEVICE_BUILDERS = [2, 3]   # MRT_BVH_DEVICE_LBVH, MRT_BVH_DEVICE_PLOC


@pytest.mark.parametrize("scene,proc", [("cornellbox", 0), ("CornellBox-Water-plastic", 0), ("cornellbox", 65536)])
@pytest.mark.parametrize("leaf", [1, 4])
@pytest.mark.parametrize("builder", DEVICE_BUILDERS)
def test_device_bvh_structure(gpu, mrt_mod, scene, proc, leaf, builder):
    s = mrt_mod.Scene(scene, procedural_triangles=proc, max_leaf_size=leaf, bvh_builder=builder)
    s.check_bvh()   # every primitive in exactly one leaf, boxes contain triangles, stack bound
    i = s.info
    assert i["bvh_width"] == 4 and i["triangles"] >= proc
    assert 0 < i["bvh_nodes"] <= i["triangles"] and i["bvh_max_stack"] <= 256
    assert i["bvh_lds_nodes"] <= i["bvh_nodes"] and i["build_ms"] > 0
    s.close()


@pytest.mark.parametrize("scene", ["cornellbox", "white-box", "CornellBox-Water-plastic"])
@pytest.mark.parametrize("builder", DEVICE_BUILDERS)
def test_device_bvh_intersect_bitexact(gpu, mrt_mod, oracle_mod, scene, builder):
    s = mrt_mod.Scene(scene, bvh_builder=builder)
    osc = oracle_mod.OracleScene(mrt_mod.scene_path(scene))
    rays = np.concatenate([_rays(oracle_mod, 6000, np.random.default_rng(11)),
                           oracle_mod.raygen(80, 60, oracle_mod.noise_table(SEED, 0))]).astype(oracle_mod.RAY_DTYPE)
    ref = osc.intersect(rays)
    d_rays, d_out = to_dev(rays), to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
    mrt_mod.intersect(s, dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=True)
    got = from_dev(d_out, oracle_mod.ISECT_DTYPE)
    bad = np.nonzero((_isect_bits(got) != _isect_bits(ref)).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:8]}"
    s.close()


@pytest.mark.parametrize("scene,L", [("cornellbox", 4), ("CornellBox-Water-plastic", 8)])
def test_render_device_bvh_equals_sah(gpu, mrt_mod, oracle_mod, scene, L):
    """The image does not depend on the BVH: precise renders over the device
    LBVH / PLOC trees and the host SAH BVH are bit-identical, and match the oracle."""
    W, H, frames = 96, 64, 3
    imgs = []
    for builder in (mrt_mod.BVH_HOST_SAH, mrt_mod.BVH_DEVICE_LBVH, mrt_mod.BVH_DEVICE_PLOC):
        s = mrt_mod.Scene(scene, bvh_builder=builder)
        r = mrt_mod.Renderer(s, W, H, L, precise=True)
        r.draw(frames)
        imgs.append((r.read_image(), r.stats()["active_ray_bounces"]))
        r.close()
        s.close()
    for img, a in imgs[1:]:
        assert img.tobytes() == imgs[0][0].tobytes() and a == imgs[0][1]
    ref, A = oracle_mod.OracleScene(mrt_mod.scene_path(scene)).render(W, H, L, SEED, frames, threads=8)
    rel, rmse, _ = pixel_metrics(imgs[1][0], ref)
    assert np.mean(rel <= 1e-4) >= 0.999 and rmse <= 1e-3


def _export_dev(mrt_mod, scene, proc=0):
    s = mrt_mod.Scene(scene, procedural_triangles=proc, device=-1)
    e = s.export()
    s.close()
    return e


@pytest.mark.parametrize("builder", [1, 2, 3])
def test_accel_raw_buffers_bitexact(gpu, mrt_mod, oracle_mod, builder):
    """mrt_accel_* over the reference's own Vertex (24 B) / uint32 index buffers."""
    scene = "CornellBox-Water-plastic"
    e = _export_dev(mrt_mod, scene)
    d_v, d_i = to_dev(e["vertices"]), to_dev(e["indices"])
    T = len(e["indices"]) // 3
    acc = mrt_mod.Accel(dev_ptr(d_v), 24, dev_ptr(d_i), T, builder=builder)
    info = acc.info()
    assert info["triangles"] == T and info["builder"] == builder and info["bvh_nodes"] > 0
    osc = oracle_mod.OracleScene(mrt_mod.scene_path(scene))
    rays = _rays(oracle_mod, 8000, np.random.default_rng(3))
    ref = osc.intersect(rays)
    d_rays, d_out = to_dev(rays), to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
    acc.intersect(dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=True)
    got = from_dev(d_out, oracle_mod.ISECT_DTYPE)
    assert (_isect_bits(got) == _isect_bits(ref)).all()
    # 48-B LightSamplingRay records through the same call (stride contract)
    sr = np.zeros(len(rays), oracle_mod.SRAY_DTYPE)
    for k in ("origin", "minDistance", "direction", "maxDistance"):
        sr[k] = rays[k]
    d_sr = to_dev(sr)
    acc.intersect(dev_ptr(d_sr), 48, len(sr), dev_ptr(d_out), precise=True)
    assert (_isect_bits(from_dev(d_out, oracle_mod.ISECT_DTYPE)) == _isect_bits(ref)).all()
    acc.close()


def test_accel_rebuild_after_vertex_update(gpu, mrt_mod, oracle_mod):
    """MPS `rebuild` re-reads the buffers: move the geometry, rebuild, and the
    device LBVH answers exactly like a host-SAH structure over the new data."""
    e = _export_dev(mrt_mod, "cornellbox", proc=20000)
    T = len(e["indices"]) // 3
    d_v, d_i = to_dev(e["vertices"]), to_dev(e["indices"])
    lb = mrt_mod.Accel(dev_ptr(d_v), 24, dev_ptr(d_i), T)   # default builder: device PLOC
    assert lb.info()["builder"] == mrt_mod.BVH_DEVICE_PLOC
    v2 = e["vertices"].copy()
    v2["v"] = v2["v"] * np.float32(0.9) + np.float32(0.05)
    d_v.copy_(to_dev(v2))
    lb.rebuild()
    sah = mrt_mod.Accel(dev_ptr(d_v), 24, dev_ptr(d_i), T, builder=mrt_mod.BVH_HOST_SAH)
    rays = _rays(oracle_mod, 20000, np.random.default_rng(5))
    d_rays = to_dev(rays)
    outs = []
    for acc in (lb, sah):
        d_out = to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
        acc.intersect(dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=True)
        outs.append(from_dev(d_out, oracle_mod.ISECT_DTYPE))
    assert (outs[0]["distance"] >= 0).mean() > 0.5
    assert (_isect_bits(outs[0]) == _isect_bits(outs[1])).all()
    lb.close()
    sah.close()


@pytest.mark.parametrize("T", [0, 1, 3, 5, 17])
def test_accel_tiny_and_empty(gpu, mrt_mod, oracle_mod, T):
    """Edge sizes: empty structure (every ray misses), a single leaf at the
    root (T <= max leaf size), one level of nodes — the device LBVH answers
    bitwise like the host-SAH structure over the same buffers."""
    e = _export_dev(mrt_mod, "cornellbox")
    idx = e["indices"][: 3 * T].copy()
    d_v, d_i = to_dev(e["vertices"]), to_dev(idx if T else np.zeros(3, np.uint32))
    rays = _rays(oracle_mod, 4000, np.random.default_rng(T))
    d_rays = to_dev(rays)
    outs = []
    for builder in ([mrt_mod.BVH_DEVICE_PLOC, mrt_mod.BVH_DEVICE_LBVH] + ([mrt_mod.BVH_HOST_SAH] if T else [])):
        acc = mrt_mod.Accel(dev_ptr(d_v), 24, dev_ptr(d_i), T, builder=builder)
        d_out = to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
        acc.intersect(dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=True)
        outs.append(from_dev(d_out, oracle_mod.ISECT_DTYPE))
        acc.close()
    if T == 0:
        for o in outs:
            assert (o["distance"] == -1.0).all() and (o["triangleIndex"] == 0xFFFFFFFF).all()
    else:
        assert (outs[0]["distance"] >= 0).any()
        for o in outs[1:]:
            assert (_isect_bits(o) == _isect_bits(outs[0])).all()


@pytest.mark.parametrize("builder", DEVICE_BUILDERS)
def test_device_bvh_deep_scene_matches_sah(gpu, mrt_mod, oracle_mod, builder):
    """1M-triangle procedural scene (BASELINE C4): the device trees are deeper
    than the stage kernel's LDS stack (spill variant), and still answer every
    ray bitwise like the host-SAH tree; a short render agrees bitwise too."""
    proc = 1 << 20
    scenes = [mrt_mod.Scene("cornellbox", procedural_triangles=proc, bvh_builder=b)
              for b in (mrt_mod.BVH_HOST_SAH, builder)]
    scenes[1].check_bvh()
    rays = _rays(oracle_mod, 50000, np.random.default_rng(17))
    d_rays = to_dev(rays)
    outs = []
    for sc in scenes:
        d_out = to_dev(np.zeros(len(rays), oracle_mod.ISECT_DTYPE))
        mrt_mod.intersect(sc, dev_ptr(d_rays), 80, len(rays), dev_ptr(d_out), precise=True)
        outs.append(from_dev(d_out, oracle_mod.ISECT_DTYPE))
    assert (outs[0]["distance"] >= 0).mean() > 0.5
    assert (_isect_bits(outs[0]) == _isect_bits(outs[1])).all()
    imgs = []
    for sc in scenes:
        r = mrt_mod.Renderer(sc, 128, 96, 4, precise=True)
        r.draw(2)
        imgs.append(r.read_image())
        r.close()
    assert imgs[0].tobytes() == imgs[1].tobytes()
    print(f"builder {builder}: max_stack {scenes[1].info['bvh_max_stack']}, build {scenes[1].info['build_ms']:.1f} ms")
    for sc in scenes:
        sc.close()
