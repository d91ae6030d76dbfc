"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
import this module — as the checker, never as the thing measured or shipped.
The restated algorithm lives in ``oracle/mrt_oracle.cpp`` (each function cites
the reference file:line it follows).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "liboracle.so")

# numpy views of the reference AoS records (renderer/Raytracing.h:47-123)
RAY_DTYPE = np.dtype({
    "names": ["origin", "minDistance", "direction", "maxDistance", "throughput", "radiance", "params"],
    "formats": [("<f4", 3), "<f4", ("<f4", 3), "<f4", ("<f4", 3), ("<f4", 3), ("<f4", 4)],
    "offsets": [0, 12, 16, 28, 32, 44, 64],
    "itemsize": 80,
})
SRAY_DTYPE = np.dtype({
    "names": ["origin", "minDistance", "direction", "maxDistance", "throughput", "targetIndex"],
    "formats": [("<f4", 3), "<f4", ("<f4", 3), "<f4", ("<f4", 3), "<u4"],
    "offsets": [0, 12, 16, 28, 32, 44],
    "itemsize": 48,
})
ISECT_DTYPE = np.dtype({
    "names": ["distance", "triangleIndex", "coordinates"],
    "formats": ["<f4", "<u4", ("<f4", 2)],
    "offsets": [0, 4, 8],
    "itemsize": 16,
})
VERTEX_DTYPE = np.dtype({"names": ["v", "n"], "formats": [("<f4", 3), ("<f4", 3)], "offsets": [0, 12], "itemsize": 24})
MATERIAL_DTYPE = np.dtype({
    "names": ["diffuse", "emissive", "ior", "materialType"],
    "formats": [("<f4", 3), ("<f4", 3), "<f4", "<u4"],
    "offsets": [0, 12, 24, 28], "itemsize": 32,
})
TRIREF_DTYPE = np.dtype({
    "names": ["tri", "materialIndex", "lightTriangleIndex"],
    "formats": [("<u4", 3), "<u4", "<u4"], "offsets": [0, 12, 16], "itemsize": 20,
})
LIGHT_DTYPE = np.dtype({
    "names": ["emissive", "v1", "v2", "v3", "area", "pdf", "cdf", "index"],
    "formats": [("<f4", 3), VERTEX_DTYPE, VERTEX_DTYPE, VERTEX_DTYPE, "<f4", "<f4", "<f4", "<u4"],
    "offsets": [0, 12, 36, 60, 84, 88, 92, 96], "itemsize": 100,
})

_lib = None

# orc_render / orc_shade / orc_accumulate flags: the reference's compile-time
# switches (renderer/Raytracing.h:14,20; renderer/Shaders.metal:7) and the
# traversal the CPU baseline times
STATIC_NOISE = 1      # ANIMATE_NOISE 0
NO_ACCUMULATE = 2     # ACCUMULATE_IMAGE false
DEBUG_MATERIAL = 4    # DEBUG_MATERIAL 1
BVH = 8               # nearest hits through the CPU BVH (same answers as brute force); boxes are
                      # culled only beyond the current hit's t * (1 + 2^-6), far wider than the
                      # kernels' 2^-11 slack, so the two do not share an error mode
BVH_NOCULL = 16       # with BVH: no culling by the current hit at all (every box the ray's
                      # [tmin, tmax] slab interval enters)


def build() -> None:
    """Compile the oracle with its committed Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u32, u64, i64 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64
        L.orc_scene_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(vp)]
        L.orc_scene_from_arrays.argtypes = [vp, u32, vp, u32, vp, u32, ctypes.POINTER(vp)]
        L.orc_scene_free.argtypes = [vp]
        L.orc_scene_counts.argtypes = [vp, vp]
        for n in ("vertices", "indices", "materials", "references", "lights"):
            f = getattr(L, "orc_scene_" + n)
            f.argtypes = [vp]
            f.restype = vp
        L.orc_noise_table.argtypes = [u64, i64, vp]
        L.orc_noise_frame_for.argtypes = [i64, u32]
        L.orc_noise_frame_for.restype = i64
        L.orc_raygen.argtypes = [u32, u32, vp, vp]
        L.orc_intersect.argtypes = [vp, vp, u32, u32, vp]
        L.orc_intersect_bvh.argtypes = [vp, vp, u32, u32, vp]
        L.orc_intersect_bvh_mt.argtypes = [vp, vp, u32, u32, vp, u32, u32]
        L.orc_shade.argtypes = [vp, u32, u32, u32, u32, vp, vp, vp, vp, u32]
        L.orc_resolve.argtypes = [u32, vp, vp, vp]
        L.orc_accumulate.argtypes = [u32, u32, vp, vp, u32]
        L.orc_render.argtypes = [vp, u32, u32, u32, u64, u32, u32, u32, vp, vp, vp, u32]
        L.orc_set_packet_threshold.argtypes = [u64]
        _lib = L
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


class OracleScene:
    """Flattened scene exactly as initRaytracing builds it (Renderer.mm:255-454)."""

    def __init__(self, obj_path: str | None = None, mtl_override: str | None = None, *, _handle=None):
        L = lib()
        if _handle is not None:
            self.h = _handle
        else:
            h = ctypes.c_void_p()
            rc = L.orc_scene_load(obj_path.encode(), (mtl_override or "").encode(), ctypes.byref(h))
            if rc != 0:
                raise RuntimeError(f"oracle failed to load {obj_path}")
            self.h = h
        c = np.zeros(5, np.uint32)
        L.orc_scene_counts(self.h, _p(c))
        self.n_vertices, self.n_triangles, self.n_materials, self.n_lights, n_light_entries = map(int, c)

        def view(fn, dtype, n):
            ptr = fn(self.h)
            buf = (ctypes.c_uint8 * (dtype.itemsize * n)).from_address(ptr) if n else bytearray()
            return np.frombuffer(buf, dtype=dtype, count=n).copy()

        self.vertices = view(L.orc_scene_vertices, VERTEX_DTYPE, self.n_vertices)
        self.indices = view(L.orc_scene_indices, np.dtype("<u4"), 3 * self.n_triangles)
        self.materials = view(L.orc_scene_materials, MATERIAL_DTYPE, self.n_materials)
        self.references = view(L.orc_scene_references, TRIREF_DTYPE, self.n_triangles)
        self.lights = view(L.orc_scene_lights, LIGHT_DTYPE, n_light_entries)

    @classmethod
    def from_arrays(cls, vertices: np.ndarray, references: np.ndarray, materials: np.ndarray) -> "OracleScene":
        vertices = np.ascontiguousarray(vertices, VERTEX_DTYPE)
        references = np.ascontiguousarray(references, TRIREF_DTYPE)
        materials = np.ascontiguousarray(materials, MATERIAL_DTYPE)
        h = ctypes.c_void_p()
        lib().orc_scene_from_arrays(_p(vertices), len(vertices), _p(references), len(references),
                                    _p(materials), len(materials), ctypes.byref(h))
        return cls(_handle=h)

    def __del__(self):
        try:
            lib().orc_scene_free(self.h)
        except Exception:
            pass

    # ---- stages (renderer/Shaders.metal) ----
    def intersect(self, rays: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays)
        if rays.dtype.itemsize not in (RAY_DTYPE.itemsize, SRAY_DTYPE.itemsize):
            raise ValueError(f"ray records must be Ray (80 B) or LightSamplingRay (48 B), got {rays.dtype.itemsize} B")
        out = np.zeros(len(rays), ISECT_DTYPE)
        lib().orc_intersect(self.h, _p(rays), rays.dtype.itemsize, len(rays), _p(out))
        return out

    def intersect_bvh(self, rays: np.ndarray, threads: int = 1, nocull: bool = False) -> np.ndarray:
        """intersect() through the CPU baseline's BVH (identical answers);
        nocull: no culling by the current hit (see BVH_NOCULL)."""
        rays = np.ascontiguousarray(rays)
        out = np.zeros(len(rays), ISECT_DTYPE)
        if threads == 1 and not nocull:
            lib().orc_intersect_bvh(self.h, _p(rays), rays.dtype.itemsize, len(rays), _p(out))
        else:
            lib().orc_intersect_bvh_mt(self.h, _p(rays), rays.dtype.itemsize, len(rays), _p(out), threads,
                                       1 if nocull else 0)
        return out

    def shade(self, W, H, frame_index, max_path_length, noise, isect, rays, srays, flags=0):
        lib().orc_shade(self.h, W, H, frame_index, max_path_length, _p(noise), _p(isect), _p(rays), _p(srays), flags)

    def render(self, W, H, L, seed, frames, frame_begin=0, threads=1, image=None, pixel_mask=None, flags=0):
        """Returns (image[H,W,4] float32, active ray-bounces A); flags: STATIC_NOISE,
        NO_ACCUMULATE, DEBUG_MATERIAL, BVH, BVH_NOCULL."""
        if image is None:
            image = np.zeros((H, W, 4), np.float32)
        active = np.zeros(1, np.uint64)
        mask_p = _p(pixel_mask) if pixel_mask is not None else None
        rc = lib().orc_render(self.h, W, H, L, seed, frame_begin, frame_begin + frames, threads, mask_p,
                              _p(image), _p(active), flags)
        if rc != 0:
            raise RuntimeError("orc_render failed")
        return image, int(active[0])


PACKET_THRESHOLD = 4096   # orc_render / orc_intersect default (triangles)


def set_packet_threshold(triangles: int) -> None:
    """Scenes with at least this many triangles are brute-forced in ray
    packets over SoA triangle blocks (same answers, far faster on 1M
    triangles); tests move it to check both forms agree."""
    lib().orc_set_packet_threshold(triangles)


def noise_table(seed: int, frame: int) -> np.ndarray:
    out = np.zeros(64 * 64 * 4, np.float32)
    lib().orc_noise_table(seed, frame, _p(out))
    return out


def noise_frame_for(frame: int, iteration: int) -> int:
    return int(lib().orc_noise_frame_for(frame, iteration))


def raygen(W: int, H: int, noise: np.ndarray) -> np.ndarray:
    rays = np.zeros(W * H, RAY_DTYPE)
    lib().orc_raygen(W, H, _p(np.ascontiguousarray(noise, np.float32)), _p(rays))
    return rays


def resolve(isect, rays, srays):
    lib().orc_resolve(len(rays), _p(isect), _p(rays), _p(srays))


def accumulate(frame_index, rays, image, flags=0):
    lib().orc_accumulate(len(rays), frame_index, _p(rays), _p(image), flags)


def to_srgb(v: np.ndarray) -> np.ndarray:
    """toSRGB — renderer/Raytracing.h:130-135 (float32)."""
    v = v.astype(np.float32)
    lin = np.float32(12.92) * v
    gam = np.float32(1.055) * np.power(np.maximum(v, np.float32(0)), np.float32(1.0 / 2.4)) - np.float32(0.055)
    out = np.where(v < np.float32(0.0031308), lin, gam)
    return np.where(v <= 0, np.float32(0), np.where(v >= 1, np.float32(1), out)).astype(np.float32)


def display(image: np.ndarray, reference: np.ndarray | None, flags: int, scale: float) -> np.ndarray:
    """blitFragment — renderer/Shaders.metal:33-70 (ENABLE_TONE_MAPPING = flags & 1,
    MANUAL_SRGB = flags & 2, COMPARISON_MODE = flags >> 8, COMPARISON_SCALE = scale)."""
    def blit(c):
        c = c.astype(np.float32)
        if flags & 1:
            c = (np.float32(1) - np.exp(-c)).astype(np.float32)          # Shaders.metal:44-46
        if flags & 2:
            c = c.copy()
            c[..., :3] = to_srgb(c[..., :3])                               # Shaders.metal:48-52
        return c
    c = blit(image)
    mode = (flags >> 8) & 0xFF
    if mode == 0:
        return c
    r = blit(reference)
    if mode == 1:
        o = np.abs(c - r)                                                  # :54-56
    elif mode == 2:
        o = np.maximum(0, r - c)                                           # :57-59
    elif mode == 3:
        o = np.maximum(0, c - r)                                           # :60-62
    else:
        k = np.float32(1.0 / 3.0)                                          # :63-67
        lc = (c[..., 0] * k + c[..., 1] * k) + c[..., 2] * k
        lr = (r[..., 0] * k + r[..., 1] * k) + r[..., 2] * k
        o = np.stack([np.maximum(0, lc - lr), np.maximum(0, lr - lc), np.zeros_like(lc), np.ones_like(lc)], -1)
    return (o * np.float32(scale)).astype(np.float32)
