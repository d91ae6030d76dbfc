"""CPU: the exit bound of nearest queries (kernels.hip exit_bound,
occluders.cpp header).

MPS answers the nearest hit of a path ray (renderer/Renderer.mm:519-523).
Every scene vertex lies inside each culled supporting plane (walls, floor,
ceiling), so a ray leaving the room through the first plane it crosses
outward cannot hit any triangle beyond that crossing; the kernels therefore
skip every BVH box the ray first enters beyond
  min over planes with n.d > 0 of (w - n.o + exit_margin) / (n.d)  (x 1.0001).
The leaf tests are unchanged (h.t is not clamped), so the answer is the
brute-force nearest hit exactly when no box holding that hit is skipped.
This test checks that claim with the kernels' float32 arithmetic (tri_bary
with and without FMA contraction, the slab test on the triangle's padded
box, which every box above it contains): for 300 K rays — bounce-ray origins
on every triangle offset by +-DISTANCE_EPSILON (Shaders.metal:171, 205),
origins in the room, near its corners and at the margins, directions over the
sphere, grazing every culled plane and aimed at the corners — the padded box
of the brute-force answer is always entered before the bound.  (The GPU
tests check the renders: the precise build bit-identical to the oracle,
which has no bound.)
"""
import numpy as np
import pytest

from helpers import SEED
from test_occluders import _fma, _tri_t


def _exit_bound(planes, margin, o, d):
    """kernels.hip exit_bound in float32 (explicit fmaf in both builds)."""
    f32 = np.float32
    tb = np.full(len(o), np.inf, f32)
    for p in planes:
        c = _fma(p[0], d[:, 0], _fma(p[1], d[:, 1], (p[2] * d[:, 2]).astype(f32)))
        num = (f32(p[3]) + f32(margin)) - _fma(p[0], o[:, 0], _fma(p[1], o[:, 1], (p[2] * o[:, 2]).astype(f32)))
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            t = (num / c).astype(f32)
        tb = np.where(c > 0, np.minimum(tb, t), tb)
    return (tb * f32(1.0001)).astype(f32)


def _box_entry(lo, hi, o, d):
    """The slab test's entry distance (kernels.hip make_raybox / slab, float32),
    clamped at tmin = 0."""
    f32 = np.float32
    dd = np.where(np.abs(d) > 1e-20, d, np.copysign(f32(1e-20), d)).astype(f32)
    inv = (f32(1.0) / dd).astype(f32)
    a = ((lo - o) * inv).astype(f32)
    b = ((hi - o) * inv).astype(f32)
    return np.maximum(np.minimum(a, b).max(1), f32(0.0))


def _rays(V, I, planes, n, rng):
    f32 = np.float32
    P = V[I.reshape(-1, 3)].astype(np.float64)
    T = len(P)
    lo, hi = V.min(0).astype(np.float64), V.max(0).astype(np.float64)
    o = np.empty((n, 3))
    # bounce origins: a point of a random triangle + its normal x (+-1e-4)
    k = n // 2
    ti = rng.integers(0, T, k)
    r1 = np.sqrt(rng.uniform(0, 1, k))
    r2 = rng.uniform(0, 1, k)
    pt = P[ti, 0] * (1 - r1)[:, None] + P[ti, 1] * (r1 * (1 - r2))[:, None] + P[ti, 2] * (r1 * r2)[:, None]
    nr = np.cross(P[ti, 1] - P[ti, 0], P[ti, 2] - P[ti, 0])
    nr /= np.linalg.norm(nr, axis=1, keepdims=True)
    o[:k] = pt + nr * (1e-4 * rng.choice([-1.0, 1.0], k))[:, None]
    # room points, and points near the room's corners and edges
    m = n // 4
    o[k:k + m] = rng.uniform(lo, hi, (m, 3))
    c = rng.integers(0, 2, (n - k - m, 3))
    o[k + m:] = np.where(c, hi, lo) + rng.normal(0, 1e-3, (n - k - m, 3)) * (hi - lo)
    # directions: sphere; a quarter grazing a random culled plane; an eighth at a corner
    d = rng.normal(size=(n, 3))
    g = n // 4
    pl = planes[rng.integers(0, len(planes), g), :3].astype(np.float64)
    tang = np.cross(pl, rng.normal(size=(g, 3)))
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    eps = 10.0 ** rng.uniform(-7, -2, g) * rng.choice([-1.0, 1.0], g)
    d[:g] = tang + eps[:, None] * pl
    q = n // 8
    corner = np.where(rng.integers(0, 2, (q, 3)), hi, lo)
    d[g:g + q] = corner - o[g:g + q]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o.astype(f32), d.astype(f32)


@pytest.mark.parametrize("fma", [False, True])
@pytest.mark.parametrize("scene", ["cornellbox"])
def test_exit_bound_never_skips_the_nearest_hit(mrt_mod, scene, fma):
    s = mrt_mod.Scene(scene, device=-1)
    info = s.info
    npl = info["occluder_planes"]
    assert npl == 5 and 0 < info["occluder_exit_margin"] < 1e-3
    planes = np.array(info["occluder_plane"][:npl], np.float32)
    e = s.export()
    V = e["vertices"]["v"].astype(np.float32)
    I = e["indices"]
    P = V[I.reshape(-1, 3)]
    T = len(P)
    rng = np.random.default_rng(SEED)
    n = 300_000
    o, d = _rays(V, I, planes, n, rng)
    tb = _exit_bound(planes, info["occluder_exit_margin"], o, d)
    # brute-force nearest hit, the kernels' tie rule (lowest primitive)
    best_t = np.full(n, np.inf, np.float32)
    best_k = np.full(n, -1)
    for k in range(T):
        v0 = P[k, 0]
        t, ok = _tri_t(o, d, v0[None], (P[k, 1] - v0)[None], (P[k, 2] - v0)[None], fma)
        hit = ok & (t >= 0) & (t < best_t)   # (t, k) order: an equal t keeps the lower k
        best_t = np.where(hit, t, best_t)
        best_k = np.where(hit, k, best_k)
    found = best_k >= 0
    assert found.mean() > 0.5
    # the answer's padded box (bvh.cpp padded_box) is entered before the bound
    tri = P[best_k[found]]
    lo, hi = tri.min(1), tri.max(1)
    mag = np.maximum(np.abs(lo), np.abs(hi))
    pad = (np.float32(1e-5) * mag + np.float32(1e-6)).astype(np.float32)
    entry = _box_entry((lo - pad).astype(np.float32), (hi + pad).astype(np.float32), o[found], d[found])
    bad = ~(entry <= tb[found])
    assert not bad.any(), (o[found][bad][:3], d[found][bad][:3], entry[bad][:3], tb[found][bad][:3])
    # the bound does skip: most rays leave the room well before +inf
    assert np.isfinite(tb).mean() > 0.8
