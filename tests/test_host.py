"""CPU: the product's host side (libmrt.so without a device).

* the C-ABI library loads and exports every symbol include/mrt.h declares;
* scene import + flattening (renderer/Renderer.mm:255-454) is byte-identical
  to the oracle's independent restatement on every shipped scene;
* the BVH builder's output passes its structural check (every primitive in
  exactly one leaf, boxes contain their triangles, depth within the stack);
* noise tables and the shard mask agree with the oracle / the tiling rule;
* errors come back as status codes with a message, never as crashes.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from helpers import SEED

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = ["cornellbox", "white-box", "CornellBox-Water-plastic", "CornellBox-Water-mirror", "CornellBox-Water"]


def test_library_exports_every_declared_symbol(mrt_mod):
    header = open(os.path.join(ROOT, "include", "mrt.h")).read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(mrt_\w+)\s*\(", header, re.M))
    assert len(declared) >= 25
    lib = ctypes.CDLL(mrt_mod.LIB_PATH)
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    assert set(mrt_mod.EXPORTED) == declared
    assert mrt_mod.lib().mrt_abi_version() == 9


def test_objc_facade_binds_only_declared_symbols(mrt_mod):
    """integration/objc/Renderer.mm (the drop-in Renderer, not compilable
    here) calls only functions and flags the C ABI declares, and covers every
    selector of renderer/Renderer.h:3-8 plus the MTKViewDelegate methods."""
    src = open(os.path.join(ROOT, "integration", "objc", "Renderer.mm")).read()
    header = open(os.path.join(ROOT, "include", "mrt.h")).read()
    called = set(re.findall(r"\b(mrt_\w+)\s*\(", src))
    assert {"mrt_scene_create", "mrt_renderer_create", "mrt_renderer_resize", "mrt_renderer_draw",
            "mrt_renderer_display_enqueue", "mrt_renderer_display_map", "mrt_renderer_load_reference",
            "mrt_renderer_save_image"} <= called
    assert "mrt_renderer_display(" not in src   # no per-frame host wait (3 frames in flight)
    assert called <= set(mrt_mod.EXPORTED), called - set(mrt_mod.EXPORTED)
    for macro in set(re.findall(r"\b(MRT_[A-Z_]+)\b", src)):
        assert re.search(r"(#define\s+" + macro + r"|^\s*" + macro + r"\s*=)", header, re.M), macro
    for sel in ("initWithMetalKitView:", "saveCurrentImage", "drawInMTKView:", "drawableSizeWillChange:"):
        assert sel in src, sel


def test_device_count_never_fails(mrt_mod):
    assert mrt_mod.device_count() >= 0


@pytest.mark.parametrize("scene", SCENES)
def test_flatten_matches_oracle(mrt_mod, oracle_mod, scene):
    s = mrt_mod.Scene(scene, device=-1)
    e = s.export()
    o = oracle_mod.OracleScene(mrt_mod.scene_path(scene))
    for k, ov in [("vertices", o.vertices), ("indices", o.indices), ("materials", o.materials),
                  ("references", o.references), ("lights", o.lights)]:
        assert e[k].tobytes() == ov.tobytes(), k
    assert s.info["triangles"] == o.n_triangles and s.info["light_triangles"] == o.n_lights


@pytest.mark.parametrize("scene", SCENES)
@pytest.mark.parametrize("leaf", [1, 4, 16])
def test_bvh_structure(mrt_mod, scene, leaf):
    s = mrt_mod.Scene(scene, device=-1, max_leaf_size=leaf)
    s.check_bvh()   # containment, every primitive once, stack bound
    i = s.info
    assert i["bvh_width"] == 4 and i["bvh_depth"] < 32
    assert i["bvh_lds_nodes"] <= i["bvh_nodes"]
    assert i["bvh_max_stack"] <= 48


def test_bvh_width_default_and_invalid(mrt_mod):
    assert mrt_mod.Scene("cornellbox", device=-1).info["bvh_width"] == 4
    assert mrt_mod.Scene("CornellBox-Water-plastic", device=-1).info["bvh_width"] == 4
    for w in (2, 3, 8):   # BVH4 is the one layout the kernels traverse
        with pytest.raises(mrt_mod.MrtError, match="bvh_width"):
            mrt_mod.Scene("cornellbox", device=-1, bvh_width=w)


def test_bvh_procedural_mesh(mrt_mod):
    s = mrt_mod.Scene("cornellbox", device=-1, procedural_triangles=1 << 16, procedural_seed=3, bvh_width=4)
    assert s.info["triangles"] == 36 + (1 << 16)
    s.check_bvh()
    assert s.info["bvh_depth"] < s.info["bvh_max_stack"] <= 48
    e = s.export()
    v = e["vertices"]["v"][72:]
    assert v[:, 1].min() > 0.2 and v[:, 1].max() < 1.6 and np.abs(v[:, [0, 2]]).max() < 0.8
    n = np.linalg.norm(e["vertices"]["n"][72:], axis=1)
    np.testing.assert_allclose(n, 1.0, rtol=1e-5)
    # deterministic for a seed
    e2 = mrt_mod.Scene("cornellbox", device=-1, procedural_triangles=1 << 16, procedural_seed=3).export()
    assert e["vertices"].tobytes() == e2["vertices"].tobytes()


def test_full_sweep_sah_builder(mrt_mod, monkeypatch):
    """Scenes of >= 64 K triangles use the presorted full-sweep SAH builder
    (bvh.cpp build_full): a valid tree (every primitive in one leaf, boxes
    contain their triangles, depth within the stack) of lower SAH cost than the
    binned builder (MRT_FULL_SWEEP=0) on the same mesh; deterministic."""
    costs = {}
    for full in ("1", "0"):
        monkeypatch.setenv("MRT_FULL_SWEEP", full)
        s = mrt_mod.Scene("cornellbox", device=-1, procedural_triangles=1 << 16, procedural_seed=5)
        s.check_bvh()
        costs[full] = (s.info["bvh_sah_cost"], s.info["bvh_nodes"], s.info["bvh_max_stack"])
        s.close()
    assert costs["1"][0] < costs["0"][0]
    monkeypatch.setenv("MRT_FULL_SWEEP", "1")
    s = mrt_mod.Scene("cornellbox", device=-1, procedural_triangles=1 << 16, procedural_seed=5)
    assert (s.info["bvh_sah_cost"], s.info["bvh_nodes"], s.info["bvh_max_stack"]) == costs["1"]
    s.close()


@pytest.mark.parametrize("scene,proc", [("cornellbox", 0), ("CornellBox-Water-plastic", 0), ("cornellbox", 1 << 15)])
def test_area_optimal_collapse(mrt_mod, monkeypatch, scene, proc):
    """The BVH4 collapse by dynamic programming (bvh.cpp, MRT_COLLAPSE=1; the
    default below 64 K triangles) keeps the binary tree's leaves and picks the
    wide interior nodes of least summed area: a valid tree (containment, every
    primitive once, stack bound) whose SAH cost is below the greedy
    largest-area collapse's (MRT_COLLAPSE=0), with no more nodes."""
    got = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("MRT_COLLAPSE", mode)
        s = mrt_mod.Scene(scene, device=-1, procedural_triangles=proc)
        s.check_bvh()
        got[mode] = (s.info["bvh_sah_cost"], s.info["bvh_nodes"], s.info["bvh_leaves"])
        s.close()
    (c0, n0, l0), (c1, n1, l1) = got["0"], got["1"]
    assert l1 == l0                   # the same binary leaves
    assert c1 < c0 and n1 <= n0


def test_mtl_override_glass_variant(mrt_mod, tmp_path):
    """BASELINE C3 glass variant: Ks 0 0 +1.5 instantiates MATERIAL_SMOOTH_DIELECTRIC."""
    src = open(mrt_mod.scene_path("CornellBox-Water-plastic")[:-4] + ".mtl").read()
    glass = src.replace("Ks 0.0 0.0 -1.5", "Ks 0.0 0.0 1.5")
    p = tmp_path / "glass.mtl"
    p.write_text(glass)
    m = mrt_mod.Scene("CornellBox-Water-plastic", str(p), device=-1).export()["materials"]
    assert m["materialType"][0] == 3 and m["ior"][0] == np.float32(1.5)


@pytest.mark.parametrize("frame", [-1, 0, 1, 77])
def test_noise_matches_oracle(mrt_mod, oracle_mod, frame):
    assert mrt_mod.noise_table(SEED, frame).tobytes() == oracle_mod.noise_table(SEED, frame).tobytes()


@pytest.mark.parametrize("W,H,S", [(1920, 1080, 8), (100, 70, 3), (64, 64, 2), (257, 131, 5)])
def test_shard_masks_partition_the_frame(mrt_mod, W, H, S):
    total = np.zeros((H, W), np.int32)
    owned_sum = 0
    for r in range(S):
        m, n = mrt_mod.shard_mask(W, H, r, S)
        assert n == int(m.sum())
        total += m
        owned_sum += n
    assert np.all(total == 1) and owned_sum == W * H
    # tiles are 64x64 and round-robin
    m0, _ = mrt_mod.shard_mask(W, H, 0, S)
    assert m0[0, 0] == 1 and (W <= 64 or m0[0, 64] == (1 if S == 1 else 0))


def test_errors_are_status_codes(mrt_mod):
    with pytest.raises(mrt_mod.MrtError, match="cannot open"):
        mrt_mod.Scene("/nonexistent/scene.obj", device=-1)
    L = mrt_mod.lib()
    assert L.mrt_renderer_create(None, None) == -1
    assert b"null" in L.mrt_last_error()
    with pytest.raises(mrt_mod.MrtError, match="shard_rank"):
        mrt_mod.shard_mask(64, 64, 3, 2)


def test_accel_argument_errors(mrt_mod):
    """mrt_accel_* validate their arguments before touching a device."""
    import ctypes
    L = mrt_mod.lib()
    h = ctypes.c_void_p()
    assert L.mrt_accel_create(None, ctypes.byref(h)) == -1
    d = mrt_mod.AccelDesc(None, 24, None, 12, 0, 0, 0, None)   # triangles but no buffers
    assert L.mrt_accel_create(ctypes.byref(d), ctypes.byref(h)) == -1 and b"null buffer" in L.mrt_last_error()
    d = mrt_mod.AccelDesc(1, 8, 1, 12, 0, 0, 0, None)           # stride below one position
    assert L.mrt_accel_create(ctypes.byref(d), ctypes.byref(h)) == -1 and b"vertex_stride" in L.mrt_last_error()
    d = mrt_mod.AccelDesc(1, 24, 1, 12, 0, 7, 0, None)          # unknown builder
    assert L.mrt_accel_create(ctypes.byref(d), ctypes.byref(h)) == -1 and b"builder" in L.mrt_last_error()
    assert L.mrt_accel_intersect(None, None, 80, 0, None, 0, None) == -1
    with pytest.raises(mrt_mod.MrtError, match="needs a device"):
        mrt_mod.Scene("cornellbox", device=-1, bvh_builder=mrt_mod.BVH_DEVICE_LBVH)


def test_comm_argument_errors_without_device(mrt_mod):
    """The exchange ABI rejects bad arguments with a status code (no device needed)."""
    import ctypes
    L = mrt_mod.lib()
    h = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(128)
    assert L.mrt_comm_create(uid, 0, 0, 0, ctypes.byref(h)) == -1     # no ranks
    assert L.mrt_comm_create(uid, 2, 2, 0, ctypes.byref(h)) == -1     # rank out of range
    assert L.mrt_comm_create(None, 1, 0, 0, ctypes.byref(h)) == -1
    assert L.mrt_comm_unique_id(uid, 16) == -1                          # buffer too small
    assert L.mrt_renderer_exchange(None, None, 1) == -1
    assert L.mrt_renderer_exchange_flush(None) == -1
    assert L.mrt_renderer_tiles_read(None, None, 0) == -1
    assert L.mrt_comm_destroy(None) == 0
    assert b"bad argument" in L.mrt_last_error() or b"null" in L.mrt_last_error()


def _write_exr(path, rgb, comp, ptype):
    """Tiny scanline EXR writer (test-only): comp 0 NONE / 2 ZIPS, ptype 1 HALF / 2 FLOAT, B G R channels."""
    import struct
    import zlib
    H, W, _ = rgb.shape
    out = bytearray(struct.pack("<II", 20000630, 2))

    def attr(name, typ, val):
        out.extend(name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(val)) + val)
    ch = b"".join(c.encode() + b"\0" + struct.pack("<iBBBBii", ptype, 0, 0, 0, 0, 1, 1) for c in "BGR") + b"\0"
    attr("channels", "chlist", ch)
    attr("compression", "compression", bytes([comp]))
    attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, W - 1, H - 1))
    attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, W - 1, H - 1))
    attr("lineOrder", "lineOrder", b"\0")
    out.extend(b"\0")
    table = len(out)
    out.extend(b"\0" * 8 * H)
    dt = "<f2" if ptype == 1 else "<f4"
    for y in range(H):
        raw = b"".join(rgb[y, :, c].astype(dt).tobytes() for c in (2, 1, 0))
        data = raw
        if comp == 2:
            a = np.frombuffer(raw, np.uint8)
            t = np.concatenate([a[0::2], a[1::2]]).astype(np.int32)
            d = t.copy()
            d[1:] = (t[1:] - t[:-1] + 128) & 0xFF
            z = zlib.compress(d.astype(np.uint8).tobytes())
            data = z if len(z) < len(raw) else raw
        struct.pack_into("<Q", out, table + 8 * y, len(out))
        out.extend(struct.pack("<ii", y, len(data)) + data)
    open(path, "wb").write(bytes(out))


def test_exr_reader_matches_golden_decoder(mrt_mod):
    """libmrt's EXR reader (mrt_image_load_exr, the loadReferenceImage
    replacement, renderer/Renderer.mm:162-253) decodes the reference's own
    Mitsuba golden (ZIP, half RGB, 800x600) bit for bit like the test
    decoder tests/exr.py, flipped to row 0 = bottom, A = 1."""
    import exr
    path = os.path.join(ROOT, "tests", "golden", "white-box-2.exr")
    got = mrt_mod.load_exr(path)
    want = exr.read_rgb(path)[::-1]
    assert got.shape == (600, 800, 4)
    assert got[..., :3].tobytes() == np.ascontiguousarray(want).tobytes()
    assert np.all(got[..., 3] == 1.0)


@pytest.mark.parametrize("comp,ptype", [(0, 2), (0, 1), (2, 1), (2, 2)])
def test_exr_reader_formats(mrt_mod, tmp_path, comp, ptype):
    """NONE / ZIPS compression, HALF / FLOAT channels, odd sizes."""
    import exr
    rng = np.random.default_rng(comp * 7 + ptype)
    rgb = (rng.standard_normal((13, 37, 3)) * 4).astype(np.float16 if ptype == 1 else np.float32).astype(np.float32)
    rgb[0, 0] = [0.0, 65504.0 if ptype == 1 else 1e30, -2.5e-7]   # zero, max half / huge float, subnormal-ish
    rgb = rgb.astype(np.float16).astype(np.float32) if ptype == 1 else rgb
    p = str(tmp_path / "t.exr")
    _write_exr(p, rgb, comp, ptype)
    got = mrt_mod.load_exr(p)
    assert np.array_equal(got[::-1, :, :3], rgb) and np.array_equal(got[..., :3], exr.read_rgb(p)[::-1])
    with pytest.raises(mrt_mod.MrtError, match="OpenEXR|open"):
        mrt_mod.load_exr(str(tmp_path / "missing.exr"))


@pytest.mark.parametrize("L", [2, 4, 8])
def test_stream_kernel_level_bound(L):
    """kernels.hip::stream_kernel keeps a wave's queue per bounce level in
    kStreamCap = 128 slots.  Its schedule — run the deepest level holding
    >= 64 rays, else up to 64 camera rays, else (camera rays exhausted) the
    deepest non-empty level; survivors append to the next level — must never
    hold more than 127 rays in a level, for any survivor pattern.  A
    restatement of the schedule driven by random and adversarial survivor
    counts (every ray survives, none do, bursts) checks the bound and that
    every ray is run exactly once per bounce it reaches."""
    rng = np.random.default_rng(L)
    for trial in range(200):
        cam = int(rng.integers(1, 3000))
        mode = trial % 4
        cnt = [0] * L
        pend = cam
        runs = [0] * L   # rays run per bounce
        alive = [0] * L  # survivors of bounce b
        while True:
            lvl = next((k for k in range(L - 1, 0, -1) if cnt[k] >= 64), 0)
            if lvl == 0 and pend > 0:
                n = min(64, pend)
                pend -= n
            else:
                if lvl == 0:
                    lvl = next((k for k in range(L - 1, 0, -1) if cnt[k] > 0), 0)
                    if lvl == 0:
                        break
                n = min(64, cnt[lvl])
                cnt[lvl] -= n
            runs[lvl] += n
            if lvl + 1 < L:
                s = n if mode == 0 else 0 if mode == 1 else (n if rng.random() < 0.5 else 0) if mode == 2 \
                    else int(rng.integers(0, n + 1))
                cnt[lvl + 1] += s
                alive[lvl] += s
                assert cnt[lvl + 1] <= 127, (L, trial, cnt)
        assert runs[0] == cam
        assert all(runs[b + 1] == alive[b] for b in range(L - 1))


def test_bench_launcher_fails_loudly_without_device():
    """bench.py --gpus 2 without a launcher starts two ranks itself; when a rank
    fails (here: no HIP device in this container) the job exits non-zero and
    prints no result line — it never falls back to one rank."""
    import json as _json
    import subprocess
    import sys as _sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    p = subprocess.run([_sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--config", "c1",
                        "--steps", "1", "--warmup", "0", "--exchange-backend", "host"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert "rank" in p.stderr


def test_bench_child_argv():
    import importlib.util
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    saved = sys.argv
    try:
        sys.argv = ["bench.py", "--config", "c5", "--sweep-gpus", "1,2,4,8", "--gpus=3", "--steps", "2"]
        argv = bench._child_argv(4)
    finally:
        sys.argv = saved
    assert argv[2:] == ["--config", "c5", "--steps", "2", "--gpus", "4"]


def test_stray_diagnostic_env_ignored_without_mrt_diag(mrt_mod, monkeypatch):
    """The library reads its diagnostic MRT_* overrides only under MRT_DIAG=1
    (csrc/diag_env.h): a host that integrates libmrt with stray variables set
    gets the product configuration.  Host-only scenes (no device): the BVH
    builder's and the occluder tree's overrides."""
    def info():
        s = mrt_mod.Scene("cornellbox", device=-1)
        i = dict(s.info)
        s.close()
        for k in ("build_ms",):
            i.pop(k)
        return i
    monkeypatch.delenv("MRT_DIAG", raising=False)
    default = info()
    assert default["occluder_planes"] > 0
    for k, v in (("MRT_OCCLUDERS", "0"), ("MRT_LEAF", "8"), ("MRT_COLLAPSE", "0"), ("MRT_BINS", "4"),
                 ("MRT_KERNEL", "wave"), ("MRT_BATCH", "2"), ("MRT_INFLIGHT", "3")):
        monkeypatch.setenv(k, v)
    assert info() == default
    monkeypatch.setenv("MRT_DIAG", "1")   # the same variables take effect only now
    diag = info()
    assert diag["occluder_planes"] == 0 and diag != default
