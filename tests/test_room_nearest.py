"""CPU: nearest queries from inside the room without a tree walk (kernels.hip
room_nearest, mrt_scene_info ABI 10) against the brute-force nearest hit, in
float32.

On C2's scene every triangle is a light, a wall triangle of one culled plane
or on one of the two convex solids (the blocks, bottoms included).  A path
ray whose origin is inside every culled plane is answered from a candidate
set: per solid the faces whose padded region (the face's own reach along its
axis, padded by delta, times the other axes' padded slabs) the ray crosses
inside the padded solid, no later than h.t (1 + 2^-11) — the face it enters
first, then the others; the walls whose padded crossing starts before the
ray is delta outside an approached plane (or which it approaches at
|cos| < room_graze); every light triangle.  Each candidate is tested with
the leaf test's arithmetic and tie rule, so the answer is the brute force's
whenever the candidate set holds every triangle the leaf test accepts at
t <= the answer.  That is checked here over >= 1 M rays — origins on every
surface (offset 1e-4 along the interpolated normal, as shade_hit), cosine-
and uniformly distributed directions, rays aimed at the blocks' edges and
corners and at the room's edges, and rays grazing the walls and the blocks'
faces at 1e-2 ... 1e-7 — in IEEE arithmetic and with one FMA contraction
pattern: (t, prim, u, v) equal the brute force's bit for bit."""
import numpy as np
import pytest

from helpers import SEED
from test_convex_occluders import F, _cross, _dot, _face_normals, _fma, _solid_faces


def _bary(o, d, v0, v1, v2, fma):
    """kernels.hip tri_bary: (ok, t, u, v), float32."""
    e1, e2 = (v1 - v0).astype(F), (v2 - v0).astype(F)
    p = _cross(d, e2, fma)
    det = _dot(e1, p, fma)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = (F(1) / det).astype(F)
        s = (o - v0).astype(F)
        b1 = (_dot(s, p, fma) * inv).astype(F)
        q = _cross(s, e1, fma)
        b2 = (_dot(d, q, fma) * inv).astype(F)
        t = (_dot(e2, q, fma) * inv).astype(F)
        u = ((F(1) - b1).astype(F) - b2).astype(F)
        ok = (det != 0) & (b1 >= 0) & (b1 <= 1) & (b2 >= 0) & ((b1 + b2).astype(F) <= 1)
    return ok, t, u, b1


class _Hit:
    def __init__(self, n):
        self.t = np.full(n, np.inf, F)
        self.u = np.zeros(n, F)
        self.v = np.zeros(n, F)
        self.prim = np.full(n, 0xFFFFFFFF, np.int64)
        self.found = np.zeros(n, bool)

    def update(self, mask, prim, ok, t, u, v):
        hit = mask & ok & (t >= 0) & (t <= self.t)
        take = hit & (~self.found | (t < self.t) | (prim < self.prim))
        self.found |= take
        self.t = np.where(take, t, self.t)
        self.u = np.where(take, u, self.u)
        self.v = np.where(take, v, self.v)
        self.prim = np.where(take, prim, self.prim)


def _pair(h, o, d, pair, mask, prims, fma):
    for j in range(2):
        prim = (pair.astype(np.int64) >> (16 * j)) & 0xFFFF
        valid = mask & (prim != 0xFFFF)
        pi = np.where(valid, prim, 0)
        ok, t, u, v = _bary(o, d, prims[pi, 0], prims[pi, 1], prims[pi, 2], fma)
        h.update(valid, pi, ok, t, u, v)


CULL = F(1) + F(2.0 ** -11)


def room_nearest(o, d, origin, info, prims, own_face, own_normal, lights, fma):
    """kernels.hip room_nearest, float32 (the precise build's 1 / x)."""
    n = len(o)
    h = _Hit(n)
    own = np.where(origin < len(prims), own_face[np.minimum(origin, len(prims) - 1)], 0).astype(np.int64)
    own_n = own_normal[np.minimum(origin, len(prims) - 1)]
    own_skip = np.where((own != 0) & (_dot(d, own_n, fma) >= F(1e-3)), (own - 1) >> 3, -1)
    obb = np.array(info["convex_obb"], F)
    inner = np.array(info["convex_inner"], F)
    near = np.array(info["convex_near_tris"], np.uint32)
    for c in range(info["convex_solids"]):
        B, I = obb[c], inner[c]
        T0 = np.zeros(n, F)
        T1 = (h.t * CULL).astype(F)
        e0, e1, x0, x1, neg = [], [], [], [], []
        for a in range(3):
            nv = np.broadcast_to(B[3 * a:3 * a + 3], d.shape)
            nd, no = _dot(nv, d, fma), _dot(nv, o, fma)
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                inv = (F(1) / nd).astype(F)
                tl, th = ((B[9 + 2 * a] - no) * inv).astype(F), ((B[10 + 2 * a] - no) * inv).astype(F)
                til, tih = ((I[2 * a] - no) * inv).astype(F), ((I[2 * a + 1] - no) * inv).astype(F)
            pos = ~np.signbit(nd)
            neg.append(~pos)
            e0.append(np.where(pos, tl, th)), e1.append(np.where(pos, til, tih))
            x0.append(np.where(pos, tih, til)), x1.append(np.where(pos, th, tl))
            T0 = np.fmax(T0, e0[a])
            T1 = np.fmin(T1, x1[a])
        box = (T0 <= T1) & (own_skip != c)
        cand = np.zeros((n, 6), bool)
        first = np.full(n, 8)
        first_t = np.full(n, np.inf, F)
        for a in range(3):
            es, xs = np.fmax(e0[a], T0), np.fmax(x0[a], T0)
            ce = box & (es <= np.fmin(e1[a], T1))
            cl = box & (xs <= np.fmin(x1[a], T1))
            eb = 2 * a + neg[a].astype(np.int64)
            lb = eb ^ 1
            cand[np.arange(n), eb] |= ce
            cand[np.arange(n), lb] |= cl
            take = ce & (es < first_t)
            first_t, first = np.where(take, es, first_t), np.where(take, eb, first)
            take = cl & (xs < first_t)
            first_t, first = np.where(take, xs, first_t), np.where(take, lb, first)
        has = first < 8
        pr = np.where(has, near[c][np.minimum(first, 5)], 0xFFFFFFFF).astype(np.uint32)
        _pair(h, o, d, pr, has, prims, fma)
        cand[np.arange(n)[has], first[has]] = False
        for a in range(3):
            eb = 2 * a + neg[a].astype(np.int64)
            lb = eb ^ 1
            m = cand[np.arange(n), eb] & (np.fmax(e0[a], T0) <= (h.t * CULL).astype(F))
            _pair(h, o, d, near[c][eb], m, prims, fma)
            m = cand[np.arange(n), lb] & (np.fmax(x0[a], T0) <= (h.t * CULL).astype(F))
            _pair(h, o, d, near[c][lb], m, prims, fma)
    # walls
    planes = np.array(info["occluder_plane"][:info["occluder_planes"]], F)
    walls = np.array(info["wall_pairs"], np.uint32)
    delta, graze = F(info["convex_delta"]), F(info["room_graze"])
    te = (h.t * CULL).astype(F)
    tlo = np.full((n, len(planes)), np.inf, F)
    gz = np.zeros((n, len(planes)), bool)
    for k, P in enumerate(planes):
        nv = np.broadcast_to(P[:3], d.shape)
        nd = _dot(nv, d, fma)
        dist = (P[3] - _dot(nv, o, fma)).astype(F)
        ap = nd > 0
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            inv = (F(1) / nd).astype(F)
            lo_, hi_ = ((dist - delta) * inv).astype(F), ((dist + delta) * inv).astype(F)
        tlo[:, k] = np.where(ap, lo_, np.inf)
        te = np.where(ap, np.fmin(te, hi_), te)
        gz[:, k] = ap & (nd < graze)
    for k in range(len(planes)):
        m = gz[:, k] | ((tlo[:, k] < np.inf) & (tlo[:, k] <= te))
        _pair(h, o, d, np.full(n, walls[k][0], np.uint32), m, prims, fma)
        _pair(h, o, d, np.full(n, walls[k][1], np.uint32), m & (walls[k][1] != 0xFFFFFFFF), prims, fma)
    for p in lights:
        ok, t, u, v = _bary(o, d, prims[p, 0], prims[p, 1], prims[p, 2], fma)
        h.update(np.ones(n, bool), np.full(n, p), ok, t, u, v)
    return h


def brute(o, d, prims, fma):
    h = _Hit(len(o))
    for p in range(len(prims)):
        ok, t, u, v = _bary(o, d, prims[p, 0], prims[p, 1], prims[p, 2], fma)
        h.update(np.ones(len(o), bool), np.full(len(o), p), ok, t, u, v)
    return h


@pytest.fixture(scope="module")
def room(mrt_mod):
    s = mrt_mod.Scene("cornellbox", device=-1)
    e = s.export()
    info = dict(s.info)
    s.close()
    V = e["vertices"]["v"].astype(F)
    N = e["vertices"]["n"].astype(F)
    tri = e["references"]["tri"]
    return info, V, N, tri, e


def test_room_data_classifies_every_triangle(room):
    info, V, N, tri, e = room
    assert info["room_nearest"] == 1 and info["convex_solids"] == 2
    seen = []
    for c in range(2):
        for w in info["convex_near_tris"][c]:
            seen += [p for p in ((w & 0xFFFF), (w >> 16)) if p != 0xFFFF]
    for k in range(info["occluder_planes"]):
        for w in info["wall_pairs"][k]:
            seen += [p for p in ((w & 0xFFFF), (w >> 16)) if p != 0xFFFF]
    lights = np.nonzero(e["references"]["lightTriangleIndex"] != 0xFFFFFFFF)[0].tolist()
    assert sorted(seen + lights) == list(range(len(tri)))   # each triangle exactly once
    assert len(seen) == 34                                  # 24 block (bottoms included) + 10 wall triangles


def _rays(info, V, N, tri, e, rng, n):
    T = len(tri)
    ot = rng.integers(0, T, n)
    r1, r2 = rng.random(n).astype(F), rng.random(n).astype(F)
    edge = rng.random(n) < 0.3
    r1 = np.where(edge, F(1) - rng.random(n).astype(F) * F(10.0) ** -rng.uniform(1, 6, n).astype(F), r1)
    sq = np.sqrt(r1).astype(F)
    w = np.stack([F(1) - sq, sq * (F(1) - r2), sq * r2], 1).astype(F)
    w = np.take_along_axis(w, rng.permuted(np.tile(np.arange(3), (n, 1)), axis=1), 1)
    v, nv = V[tri[ot]], N[tri[ot]]
    hv = (v[:, 0] * w[:, :1] + v[:, 1] * w[:, 1:2] + v[:, 2] * w[:, 2:]).astype(F)
    hn = (nv[:, 0] * w[:, :1] + nv[:, 1] * w[:, 1:2] + nv[:, 2] * w[:, 2:]).astype(F)
    hn = (hn / np.sqrt((hn * hn).sum(1, keepdims=True))).astype(F)
    o = (hv + hn * F(1e-4)).astype(F)
    kind = rng.integers(0, 4, n)
    # 0: cosine-weighted about the normal; 1: uniform sphere; 2: aimed at a
    # point near a triangle edge / corner (blocks' and walls'); 3: grazing a
    # random scene plane (tangent + tilt 1e-2 ... 1e-7)
    u1, u2 = rng.random(n), rng.random(n)
    ref = np.where(np.abs(hn[:, 0:1]) < 0.9, np.array([[1.0, 0, 0]]), np.array([[0, 1.0, 0]]))
    b1 = np.cross(hn, ref)
    b1 /= np.linalg.norm(b1, axis=1, keepdims=True)
    b2 = np.cross(hn, b1)
    r = np.sqrt(u1)[:, None]
    phi = (2 * np.pi * u2)[:, None]
    dc = b1 * (r * np.cos(phi)) + b2 * (r * np.sin(phi)) + hn * np.sqrt(1 - u1)[:, None]
    du = rng.standard_normal((n, 3))
    tt = rng.integers(0, T, n)
    k = rng.integers(0, 3, n)
    tv = V[tri[tt]].astype(np.float64)
    a0, a1 = tv[np.arange(n), k], tv[np.arange(n), (k + 1) % 3]
    pt = a0 + (a1 - a0) * rng.random(n)[:, None]
    pt += rng.standard_normal((n, 3)) * (10.0 ** -rng.uniform(3, 8, n))[:, None]
    da = pt - o
    pn = np.cross(tv[:, 1] - tv[:, 0], tv[:, 2] - tv[:, 0])
    pn /= np.linalg.norm(pn, axis=1, keepdims=True)
    tg = rng.standard_normal((n, 3))
    tg -= (tg * pn).sum(1, keepdims=True) * pn
    tg /= np.linalg.norm(tg, axis=1, keepdims=True)
    dg = tg + (rng.choice([-1.0, 1.0], n) * 10.0 ** -rng.uniform(2, 7, n))[:, None] * pn
    d = np.select([kind[:, None] == 0, kind[:, None] == 1, kind[:, None] == 2], [dc, du, da], dg)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(F)
    return o, d, ot


@pytest.mark.parametrize("fma", [False, True], ids=["ieee", "fma"])
def test_room_nearest_equals_brute_force(room, fma):
    info, V, N, tri, e = room
    prims = V[tri]
    own_map, _ = _solid_faces(info)
    own_face = np.zeros(len(tri), np.uint32)
    for p, f in own_map.items():
        own_face[p] = f
    # the bottoms (culled, on the floor) carry no face code: they never start a shadow or path ray
    own_normal = _face_normals(info, V, tri)
    lights = np.nonzero(e["references"]["lightTriangleIndex"] != 0xFFFFFFFF)[0]
    planes = np.array(info["occluder_plane"][:info["occluder_planes"]], F)
    margin = F(info["occluder_margin"])
    rng = np.random.default_rng(SEED + 11 + int(fma))
    checked = 0
    for _ in range(6):
        n = 200_000
        o, d, ot = _rays(info, V, N, tri, e, rng, n)
        inside = np.ones(n, bool)
        for P in planes:
            inside &= (_dot(np.broadcast_to(P[:3], o.shape), o, fma) - P[3]) <= -margin
        o, d, ot = o[inside], d[inside], ot[inside]
        got = room_nearest(o, d, ot.astype(np.int64), info, prims, own_face, own_normal, lights, fma)
        ref = brute(o, d, prims, fma)
        for name in ("found", "prim", "t", "u", "v"):
            a, b = getattr(got, name), getattr(ref, name)
            same = (a == b) | (~ref.found & ~got.found) if name != "found" else (a == b)
            bad = np.nonzero(~same)[0]
            assert len(bad) == 0, (name, len(bad), o[bad[:2]], d[bad[:2]], ot[bad[:2]], a[bad[:2]], b[bad[:2]])
        checked += len(o)
    assert checked >= 1_000_000
