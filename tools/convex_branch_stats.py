import os, sys
import numpy as np
ROOT = "/root/repo"
for sub in ("metal-renderer_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, sub))
import mrt, oracle
from helpers import SEED
import test_convex_occluders as T
F = np.float32
W, H, L = 480, 272, 4
sc = mrt.Scene("cornellbox", device=-1)
info = dict(sc.info); e = sc.export()
osc = oracle.OracleScene.from_arrays(e["vertices"], e["references"], e["materials"])
V = e["vertices"]["v"].astype(F); R = e["references"]["tri"]
prims = V[R]
own_map, solid = T._solid_faces(info)
own_face = np.zeros(len(R), np.uint32)
for p, f in own_map.items(): own_face[p] = f
f = 0
rays = oracle.raygen(W, H, oracle.noise_table(SEED, f))
recs = []
pix = np.arange(W * H)
for i in range(L):
    noise = oracle.noise_table(SEED, oracle.noise_frame_for(f, i))
    isect = osc.intersect_bvh(rays, threads=8)
    srays = np.zeros(len(rays), oracle.SRAY_DTYPE)
    osc.shade(W, H, f, L, noise, isect, rays, srays)
    ok = srays["maxDistance"] >= 0
    s = srays[ok]
    recs.append((i, pix[ok], s["origin"].astype(F), s["direction"].astype(F), s["targetIndex"], isect["triangleIndex"][ok]))
    sis = osc.intersect_bvh(srays, threads=8)
    oracle.resolve(sis, rays, srays)
planes = np.array(info["occluder_plane"][:info["occluder_planes"]], F); margin = F(info["occluder_margin"])
obb = np.array(info["convex_obb"], F); pairs = np.array(info["convex_face_tris"], np.uint32)
for (b, px, o, d, lt, org) in recs:
    n = len(o)
    okT, tT = T._tri_bary(o, d, prims[lt, 0], prims[lt, 1], prims[lt, 2], False)
    inside = np.ones(n, bool)
    for P in planes:
        inside &= (T._dot(np.broadcast_to(P[:3], o.shape), o, False) - P[3]) <= -margin
    q = okT & (tT >= F(1e-4)) & inside
    own = own_face[org]
    stats = {}
    lane = {}
    for c in range(info["convex_solids"]):
        B = obb[c]; t0 = np.zeros(n, F); t1 = tT.copy(); fin = np.full(n, 8); fout = np.full(n, 8); own_nd = np.zeros(n, F)
        for a in range(3):
            nv = np.broadcast_to(B[3*a:3*a+3], d.shape)
            nd = T._dot(nv, d, False); no = T._dot(nv, o, False)
            with np.errstate(all="ignore"):
                inv = (F(1)/nd).astype(F); tlo = ((B[9+2*a]-no)*inv).astype(F); thi = ((B[10+2*a]-no)*inv).astype(F)
            pos = ~np.signbit(nd); tn, tf = np.where(pos, tlo, thi), np.where(pos, thi, tlo)
            with np.errstate(invalid="ignore"):
                i_, o_ = tn > t0, tf < t1
            t0 = np.where(i_, tn, t0); fin = np.where(i_, np.where(pos, 2*a, 2*a+1), fin)
            t1 = np.where(o_, tf, t1); fout = np.where(o_, np.where(pos, 2*a+1, 2*a), fout)
            f0 = c*8+2*a; own_nd = np.where(own == f0+1, -nd, np.where(own == f0+2, nd, own_nd))
        leaves_own = (own > c*8) & (own <= c*8+6) & (own_nd >= F(0.01))
        cand = q & (t0 <= t1) & ~leaves_own
        pp = np.concatenate([pairs[c], np.full(1, 0xFFFFFFFF, np.uint32)])
        pin = np.where(fin < 6, pp[np.minimum(fin, 8)], 0xFFFFFFFF).astype(np.uint32)
        pout = np.where(fout < 6, pp[np.minimum(fout, 8)], 0xFFFFFFFF).astype(np.uint32)
        def face(pair):
            hit = np.zeros(n, bool)
            for j in range(2):
                prim = (pair >> (16*j)) & 0xFFFF; valid = prim != 0xFFFF; pi = np.where(valid, prim, 0)
                ok, t = T._tri_bary(o, d, prims[pi, 0], prims[pi, 1], prims[pi, 2], False)
                hit |= valid & ok & (t >= 0) & (t <= tT)
            return hit
        h1 = face(np.where(pin != 0xFFFFFFFF, pin, pout))
        need2 = cand & ~h1 & (pin != 0xFFFFFFFF)
        h2 = face(pout)
        hit = h1 | (need2 & h2)
        needfb = cand & ~hit
        lane[c] = dict(cand=cand, need2=need2, fb=needfb, leaves=q & leaves_own, slab_empty=q & ~(t0 <= t1))
    # waves: group by bounce and 8x8 pixel block (coherent) / random 64
    x, y = px % W, px // W
    blk = (y // 8) * (W // 8) + (x // 8)
    order = np.argsort(blk, kind="stable")
    def wave_frac(mask, grouping):
        m = mask[grouping]
        nw = (len(m) + 63) // 64
        mm = np.zeros(nw * 64, bool); mm[:len(m)] = m
        return mm.reshape(nw, 64).any(1).mean()
    rnd = np.random.default_rng(1).permutation(n)
    out = [f"bounce {b}: shadow rays {n}, queried via convex {int(q.sum())}"]
    for c in lane:
        L_ = lane[c]
        out.append(f"  solid {c}: lanes cand {L_['cand'][q].mean():.3f} need2 {L_['need2'][q].mean():.4f} fallback {L_['fb'][q].mean():.4f} leaves_own {L_['leaves'][q].mean():.3f} slab-empty {L_['slab_empty'][q].mean():.3f}"
                   f" | waves(blocks) cand {wave_frac(L_['cand'], order):.2f} need2 {wave_frac(L_['need2'], order):.2f} fb {wave_frac(L_['fb'], order):.2f}"
                   f" | waves(random) cand {wave_frac(L_['cand'], rnd):.2f} need2 {wave_frac(L_['need2'], rnd):.2f} fb {wave_frac(L_['fb'], rnd):.2f}")
    print("\n".join(out))
