"""CPU: the shadow-ray occluder tree (metal-renderer_amd/csrc/occluders.h).

lightSamplingHandler (renderer/Shaders.metal:214-231) counts a light sample
iff the shadow ray's nearest hit (renderer/Renderer.mm:545-553) is the target
light triangle.  The product leaves the triangles of culled supporting planes
(walls, floor, ceiling) out of a second BVH that shadow rays from origins
inside those planes traverse.  These tests restate the plane choice and check
the claim it rests on with the kernels' own float32 ray-triangle arithmetic
(kernels.hip tri_bary, with and without FMA contraction): from an origin
inside every culled plane by the margin, no culled triangle reports a hit in
[0, t_light] — including origins at the margin and shadow rays grazing the
ceiling the light hangs under.  (The GPU tests check the renders: precise
build bit-identical to the oracle, which has no occluder tree, and fast
build bitwise equal with the tree on and off.)
"""
import os

import numpy as np
import pytest

from helpers import SEED


def _supporting_planes(V, I, light_pts):
    """Restatement of occluders.cpp's choice: planes of triangles with every
    scene vertex on one side, every light vertex strictly inside."""
    P = V[I.reshape(-1, 3)].astype(np.float64)
    planes = []
    culled = np.zeros(len(P), bool)
    for t, (v0, v1, v2) in enumerate(P):
        n = np.cross(v1 - v0, v2 - v0)
        n /= np.linalg.norm(n)
        w = n @ v0
        s = V.astype(np.float64) @ n - w
        tol = 1e-6
        if (s > tol).any() and (s < -tol).any():
            continue
        if (s > tol).any():
            n, w = -n, -w
        if (light_pts @ n - w > -1e-4).any():
            continue
        culled[t] = True
        if not any(np.allclose(n, q[:3]) and abs(w - q[3]) < 1e-6 for q in planes):
            planes.append(np.array([*n, w]))
    return np.array(planes), culled


def _fma(a, b, c):
    return (a.astype(np.float64) * b + c).astype(np.float32)


def _tri_t(o, d, v0, e1, e2, fma):
    """kernels.hip tri_bary in float32: (t, inside)."""
    f32 = np.float32

    def cross(a, b):
        if fma:
            return np.stack([_fma(a[..., 1], b[..., 2], -(a[..., 2] * b[..., 1])),
                             _fma(a[..., 2], b[..., 0], -(a[..., 0] * b[..., 2])),
                             _fma(a[..., 0], b[..., 1], -(a[..., 1] * b[..., 0]))], -1)
        return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                         a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                         a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], -1)

    def dot(a, b):
        if fma:
            return _fma(a[..., 2], b[..., 2], _fma(a[..., 1], b[..., 1], a[..., 0] * b[..., 0]))
        return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]

    p = cross(d, e2)
    det = dot(e1, p)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = f32(1.0) / det
        s = o - v0
        b1 = dot(s, p) * inv
        q = cross(s, e1)
        b2 = dot(d, q) * inv
        t = dot(e2, q) * inv
        ok = (det != 0) & (b1 >= 0) & (b1 <= 1) & (b2 >= 0) & (b1 + b2 <= 1)
    return t, ok


@pytest.mark.parametrize("scene", ["cornellbox", "white-box"])
@pytest.mark.parametrize("lights_out", ["1", "0"])
def test_occluder_tree_with_and_without_lights_checks(mrt_mod, monkeypatch, scene, lights_out):
    """The occluder tree with the light triangles left out (the default; the
    kernels test them in lights_occlude) or kept (MRT_OCC_LIGHTS=0) passes
    the host tree check: exactly the kept primitives, boxes containing them,
    its stack bound.  white-box keeps only its two light triangles, so with
    them out there is no tree at all (occ_root = kEmptyChild)."""
    monkeypatch.setenv("MRT_OCC_LIGHTS", lights_out)
    s = mrt_mod.Scene(scene, device=-1)
    assert s.info["occluder_planes"] == 5
    s.check_bvh()
    if scene == "white-box":
        assert s.info["occluder_culled"] == 10 and s.info["occluder_nodes"] == 0
    s.close()


def test_occluder_planes_of_the_shipped_scenes(mrt_mod):
    s = mrt_mod.Scene("cornellbox", device=-1)
    assert s.info["occluder_planes"] == 5          # floor, ceiling, back, left, right walls
    assert s.info["occluder_culled"] == 14         # their 10 triangles + the two boxes' bottoms
    assert s.info["occluder_nodes"] >= 1
    assert 0 < s.info["occluder_margin"] < 1e-4    # below DISTANCE_EPSILON: origins on the walls qualify
    # ABI 8 exports the planes: unit outward normals, every vertex inside
    P = np.array(s.info["occluder_plane"][:5], np.float64)
    assert np.allclose(np.linalg.norm(P[:, :3], axis=1), 1.0, atol=1e-6)
    V = s.export()["vertices"]["v"].astype(np.float64)
    assert (V @ P[:, :3].T - P[:, 3] <= 1e-5).all()
    off = mrt_mod.Scene("cornellbox", device=-1, occluder_tree=False)
    assert off.info["occluder_planes"] == 0 and off.info["occluder_culled"] == 0
    # Water scenes: the walls are < 1/8 of 7 K triangles: no second tree
    w = mrt_mod.Scene("CornellBox-Water-plastic", device=-1)
    assert w.info["occluder_planes"] == 0


@pytest.mark.parametrize("fma", [False, True])
def test_culled_triangles_never_occlude(mrt_mod, fma):
    s = mrt_mod.Scene("cornellbox", device=-1)
    e = s.export()
    V = e["vertices"]["v"]
    I = e["indices"]
    L = e["lights"][:-1]
    light_pts = np.concatenate([L["v1"]["v"], L["v2"]["v"], L["v3"]["v"]]).astype(np.float64)
    planes, culled = _supporting_planes(V, I, light_pts)
    assert culled.sum() == s.info["occluder_culled"] and len(planes) == s.info["occluder_planes"]
    margin = np.float32(s.info["occluder_margin"])

    rng = np.random.default_rng(SEED)
    n = 120_000
    lo, hi = V.min(0), V.max(0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    # adversarial origins: at 1-2 margins from a random culled plane
    k = n // 2
    pl = planes[rng.integers(0, len(planes), k)]
    dist = margin * rng.uniform(1.0, 2.0, k)
    foot = o[:k] - ((o[:k].astype(np.float64) * pl[:, :3]).sum(1) - pl[:, 3])[:, None] * pl[:, :3]
    o[:k] = (foot - dist[:, None] * pl[:, :3]).astype(np.float32)
    # origins near the ceiling (shadow rays grazing the plane the light hangs under)
    g = n // 8
    o[k:k + g, 1] = np.float32(2.0) - margin * rng.uniform(1.0, 30.0, g).astype(np.float32)
    # the kernel's selection: inside every culled plane by the margin (float32)
    inside = np.ones(n, bool)
    for p in planes.astype(np.float32):
        inside &= (_fma(p[0], o[:, 0], _fma(p[1], o[:, 1], _fma(p[2], o[:, 2], -p[3]))) <= -margin)
    o = o[inside]
    assert len(o) > n // 2
    # the light point and the shadow direction (as shade_hit: normalize(q - p))
    li = rng.integers(0, len(L), len(o))
    r1 = np.sqrt(rng.uniform(0, 1, len(o))).astype(np.float32)
    r2 = rng.uniform(0, 1, len(o)).astype(np.float32)
    bu, bv, bw = 1 - r1, r1 * (1 - r2), r1 * r2
    q = (L["v1"]["v"][li] * bu[:, None] + L["v2"]["v"][li] * bv[:, None] + L["v3"]["v"][li] * bw[:, None])
    q = q.astype(np.float32)
    d = q - o
    d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
    # t of the target light triangle
    tgt = L["index"][li]
    Pv = V[I.reshape(-1, 3)]
    tv0 = Pv[tgt, 0]
    tT, ok = _tri_t(o, d, tv0, Pv[tgt, 1] - tv0, Pv[tgt, 2] - tv0, fma)
    o, d, tT = o[ok], d[ok], tT[ok]
    assert len(o) > n // 3
    for t in np.nonzero(culled)[0]:
        v0 = Pv[t, 0]
        tt, hit = _tri_t(o, d, v0[None], (Pv[t, 1] - v0)[None], (Pv[t, 2] - v0)[None], fma)
        bad = hit & (tt >= 0) & (tt <= tT)
        assert not bad.any(), (t, o[bad][:3], d[bad][:3], tt[bad][:3], tT[bad][:3])


def _sliver_room(path):
    """A 2 x 2 x 2 room (floor, ceiling, back and side walls; open front, as
    the cornellbox), a box in it, and a SLIVER light 0.01 from the left wall,
    nearly parallel to it: shadow rays toward it graze its plane at every
    angle, and its triangle's c = |e1||e2| / |e1 x e2| is large."""
    V, N, F = [], [], []

    def quad(a, b, c, d, n, mtl):
        k = len(V)
        V.extend([a, b, c, d])
        N.append(n)
        F.append((mtl, [(k + 1, k + 2, k + 3, len(N)), (k + 3, k + 4, k + 1, len(N))]))

    quad((-1, 0, 1), (1, 0, 1), (1, 0, -1), (-1, 0, -1), (0, 1, 0), "white")      # floor
    quad((-1, 2, -1), (1, 2, -1), (1, 2, 1), (-1, 2, 1), (0, -1, 0), "white")     # ceiling
    quad((1, 0, -1), (1, 2, -1), (-1, 2, -1), (-1, 0, -1), (0, 0, 1), "white")    # back wall
    quad((-1, 0, -1), (-1, 2, -1), (-1, 2, 1), (-1, 0, 1), (1, 0, 0), "white")    # left wall
    quad((1, 0, 1), (1, 2, 1), (1, 2, -1), (1, 0, -1), (-1, 0, 0), "white")      # right wall
    b = [(-0.3, 0.0, -0.3), (0.3, 0.0, -0.3), (0.3, 0.0, 0.3), (-0.3, 0.0, 0.3)]
    t = [(x, 0.7, z) for x, _, z in b]
    quad(t[0], t[3], t[2], t[1], (0, 1, 0), "white")                               # box top
    for i in range(4):                                                             # box sides
        j = (i + 1) % 4
        n = np.cross(np.subtract(t[i], b[i]), np.subtract(b[j], b[i]))
        quad(b[i], t[i], t[j], b[j], tuple(-n / np.linalg.norm(n)), "white")
    # the sliver light: long (1.7) and thin (0.02 at its base, c ~ 120 at its tip), 0.01 inside the left wall
    k = len(V)
    V.extend([(-0.99, 0.6, -0.6), (-0.99, 1.8, 0.6), (-0.99, 0.6, -0.58)])
    N.append((1, 0, 0))
    F.append(("light", [(k + 1, k + 3, k + 2, len(N))]))
    with open(path, "w") as f:
        f.write("mtllib sliver.mtl\n")
        for v in V:
            f.write("v %.6f %.6f %.6f\n" % v)
        for n in N:
            f.write("vn %.6f %.6f %.6f\n" % tuple(n))
        for mtl, tris in F:
            f.write(f"usemtl {mtl}\n")
            for a, b_, c, n in tris:
                f.write(f"f {a}//{n} {b_}//{n} {c}//{n}\n")
    with open(os.path.join(os.path.dirname(path), "sliver.mtl"), "w") as f:
        f.write("newmtl white\nKd 0.8 0.8 0.8\nKs 1.0 0.0 0.0\n\nnewmtl light\nKd 1 1 1\nKs 1.0 0.0 0.0\nKa 20 20 20\n")


@pytest.mark.parametrize("fma", [False, True])
def test_sliver_light_grazing_rays_never_culled_hits(mrt_mod, tmp_path, fma):
    """the light's own computed t has an error of about
    10 u S c_L / |cos_L|, unbounded for rays grazing the light's plane, which
    the culled triangles' margin does not cover.  The library therefore sends
    shadow rays with cos_L < occluder_cos_min (= 20 u S c_L / D_L + normal
    deviation) through the main tree.  With a sliver light 0.01 from a culled
    wall and rays at every angle to it — many within a few degrees of its
    plane — no culled triangle reports a hit in [0, t_light] for any ray the
    guard lets through, in the kernels' float32 arithmetic."""
    path = str(tmp_path / "sliver.obj")
    _sliver_room(path)
    s = mrt_mod.Scene(path, device=-1)
    info = s.info
    assert info["occluder_planes"] >= 4 and info["occluder_culled"] >= 10
    cos_min = np.float32(info["occluder_cos_min"])
    assert 0.01 < cos_min < 0.2   # c_L ~ 120: rays within ~3 degrees of the light's plane are guarded
    e = s.export()
    V = e["vertices"]["v"]
    I = e["indices"]
    L = e["lights"][:-1]
    light_pts = np.concatenate([L["v1"]["v"], L["v2"]["v"], L["v3"]["v"]]).astype(np.float64)
    planes, culled = _supporting_planes(V, I, light_pts)
    assert culled.sum() == info["occluder_culled"]
    margin = np.float32(info["occluder_margin"])
    rng = np.random.default_rng(SEED + 7)
    n = 200_000
    lo, hi = V.min(0), V.max(0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    # a third of the origins near the light's plane (x = -0.99): grazing rays
    g = n // 3
    o[:g, 0] = (np.float32(-0.99) + rng.uniform(-2e-3, 2e-3, g)).astype(np.float32)
    inside = np.ones(n, bool)
    for p in planes.astype(np.float32):
        inside &= (_fma(p[0], o[:, 0], _fma(p[1], o[:, 1], _fma(p[2], o[:, 2], -p[3]))) <= -margin)
    o = o[inside]
    li = np.zeros(len(o), np.int64)
    r1 = np.sqrt(rng.uniform(0, 1, len(o))).astype(np.float32)
    r2 = rng.uniform(0, 1, len(o)).astype(np.float32)
    bu, bv, bw = 1 - r1, r1 * (1 - r2), r1 * r2
    q = (L["v1"]["v"][li] * bu[:, None] + L["v2"]["v"][li] * bv[:, None] + L["v3"]["v"][li] * bw[:, None])
    q = q.astype(np.float32)
    d = q - o
    d = (d / np.sqrt((d * d).sum(1, keepdims=True))).astype(np.float32)
    # the kernels' cosine to the (interpolated, here constant) light normal
    ln = (L["v1"]["n"][li] * bu[:, None] + L["v2"]["n"][li] * bv[:, None] + L["v3"]["n"][li] * bw[:, None])
    ln = (ln / np.sqrt((ln * ln).sum(1, keepdims=True))).astype(np.float32)
    cosL = -(d * ln).sum(1).astype(np.float32)
    tgt = L["index"][li]
    Pv = V[I.reshape(-1, 3)]
    tv0 = Pv[tgt, 0]
    tT, ok = _tri_t(o, d, tv0, Pv[tgt, 1] - tv0, Pv[tgt, 2] - tv0, fma)
    valid = ok & (tT >= np.float32(1e-4)) & (cosL >= np.float32(3.807693583e-05))
    guarded = valid & (cosL >= cos_min)
    assert guarded.sum() > 20_000
    assert (valid & (cosL < cos_min)).sum() > 1_000   # the grazing population the guard sends to the main tree
    o, d, tT = o[guarded], d[guarded], tT[guarded]
    for t in np.nonzero(culled)[0]:
        v0 = Pv[t, 0]
        tt, hit = _tri_t(o, d, v0[None], (Pv[t, 1] - v0)[None], (Pv[t, 2] - v0)[None], fma)
        bad = hit & (tt >= 0) & (tt <= tT)
        assert not bad.any(), (t, o[bad][:3], d[bad][:3], tt[bad][:3], tT[bad][:3])


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["stream", "bounce", "path"])
@pytest.mark.parametrize("precise", [True, False])
@pytest.mark.parametrize("scene,W,H,L", [("cornellbox", 96, 64, 4), ("white-box", 80, 48, 5),
                                         ("cornellbox", 130, 70, 8)])
def test_gpu_occluder_tree_renders_bitwise(gpu, mrt_mod, monkeypatch, kernel, precise, scene, W, H, L):
    """Shadow rays through the occluder tree give the same answers as through
    the whole scene: images and ray counts bitwise equal with the tree on and
    off, in every kernel (stream, per-bounce, path) and both builds — and with
    the light triangles left out of the tree (tested in lights_occlude, the
    default) or kept in it (MRT_OCC_LIGHTS=0), and with the convex-occluder
    test (cornellbox's two blocks, the default there) on and off (MRT_CONVEX=0)."""
    monkeypatch.setenv("MRT_STREAM", "0" if kernel == "bounce" else "1")
    if kernel == "path":
        monkeypatch.setenv("MRT_KERNEL", "path")
    out = []
    for tree, lights_out, convex in ((True, True, True), (True, True, False), (True, False, False),
                                     (False, True, False)):
        monkeypatch.setenv("MRT_OCC_LIGHTS", "1" if lights_out else "0")
        monkeypatch.setenv("MRT_CONVEX", "1" if convex else "0")
        s = mrt_mod.Scene(scene, occluder_tree=tree)
        assert (s.info["occluder_planes"] > 0) == tree
        assert s.info["convex_solids"] == (2 if convex and scene == "cornellbox" else 0)
        r = mrt_mod.Renderer(s, W, H, L, precise=precise)
        r.draw(3)
        out.append((r.read_image(), r.stats()["active_ray_bounces"]))
        r.close()
        s.close()
    (a, na) = out[0]
    assert np.isfinite(a).all() and a[..., :3].max() > 0
    for b, nb in out[1:]:
        assert a.tobytes() == b.tobytes() and na == nb
