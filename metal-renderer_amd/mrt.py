"""Python mirror of the reference's Renderer interface over libmrt.so (C ABI).

The reference API (renderer/Renderer.h:3-8, Renderer.mm) maps to:

    -initWithMetalKitView:            -> Renderer(scene, width, height, ...)
    -mtkView:drawableSizeWillChange:  -> Renderer.resize(width, height)
    -drawInMTKView:                   -> Renderer.draw()          (1 spp frame)
    -saveCurrentImage                 -> Renderer.save_current_image(path)
    title-bar "Mrays/s, ms/frame"     -> Renderer.stats()

and the per-stage dispatches of performRaytracing: (Renderer.mm:500-585) map to
the module functions raygen / intersect / shade / resolve_shadow / accumulate,
which take device pointers (ints) to reference-layout AoS buffers.

This module only binds the native library: every call runs the HIP kernels in
libmrt.so.  There is no CPU fallback; if the library is missing the import
fails loudly.

Interop note: PyTorch-ROCm wheels bundle their own HIP runtime, HSA runtime
and RCCL under the same sonames as ROCm's (libamdhip64.so.7, librccl.so.1), so
a process holds ONE copy of each — whichever was loaded first (checked in
/proc/self/maps: with torch imported first, libmrt binds to torch/lib's
copies).  Device pointers (torch tensors) can therefore be handed to libmrt;
the tests import torch first (the order that is exercised), and synchronise
libmrt's work with Renderer.sync() / synchronize() rather than torch streams.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MRT_LIB") or os.path.join(HERE, "lib", "libmrt.so")   # MRT_LIB: diagnostic builds
INCLUDE_H = os.path.join(os.path.dirname(HERE), "include", "mrt.h")
SCENES_DIR = os.path.join(HERE, "scenes")   # renderer/Media scene data, rendered unchanged

FLAG_PRECISE = 1
FLAG_PROFILE = 2
# the reference's compile-time switches (renderer/Raytracing.h:14,20; Shaders.metal:7)
FLAG_STATIC_NOISE = 4       # ANIMATE_NOISE 0
FLAG_NO_ACCUMULATE = 8      # ACCUMULATE_IMAGE false
FLAG_DEBUG_MATERIAL = 16    # DEBUG_MATERIAL 1
COMM_ID_BYTES = 128
EXCHANGE_GATHER, EXCHANGE_REDUCE, EXCHANGE_OVERLAP = 1, 2, 0x100
DEFAULT_SEED = 0x6D6574616C2D7274  # "metal-rt"

RAY_BYTES, SHADOW_RAY_BYTES, ISECT_BYTES = 80, 48, 16


class MrtError(RuntimeError):
    pass


ERR_COMM = -6   # MRT_ERR_COMM: a collective failed or timed out; the communicator is aborted


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("obj_path", ctypes.c_char_p),
        ("mtl_override", ctypes.c_char_p),
        ("procedural_triangles", ctypes.c_uint32),
        ("procedural_seed", ctypes.c_uint64),
        ("max_leaf_size", ctypes.c_uint32),
        ("lds_nodes", ctypes.c_uint32),
        ("device", ctypes.c_int),
        ("bvh_width", ctypes.c_uint32),
        ("bvh_builder", ctypes.c_uint32),
        ("no_occluder_tree", ctypes.c_uint32),
    ]


BVH_HOST_SAH, BVH_DEVICE_LBVH, BVH_DEVICE_PLOC = 1, 2, 3


class AccelDesc(ctypes.Structure):
    _fields_ = [
        ("vertices", ctypes.c_void_p), ("vertex_stride", ctypes.c_uint32),
        ("indices", ctypes.c_void_p), ("triangle_count", ctypes.c_uint32),
        ("device", ctypes.c_int), ("builder", ctypes.c_uint32), ("max_leaf_size", ctypes.c_uint32),
        ("stream", ctypes.c_void_p),
    ]


class AccelInfo(ctypes.Structure):
    _fields_ = [
        ("triangles", ctypes.c_uint32), ("bvh_nodes", ctypes.c_uint32), ("bvh_leaves", ctypes.c_uint32),
        ("bvh_levels", ctypes.c_uint32), ("bvh_max_stack", ctypes.c_uint32), ("builder", ctypes.c_uint32),
        ("build_ms", ctypes.c_double), ("device_bytes", ctypes.c_uint64),
    ]


class SceneInfo(ctypes.Structure):
    _fields_ = [
        ("vertices", ctypes.c_uint32), ("triangles", ctypes.c_uint32), ("materials", ctypes.c_uint32),
        ("light_triangles", ctypes.c_uint32), ("bvh_nodes", ctypes.c_uint32), ("bvh_leaves", ctypes.c_uint32),
        ("bvh_depth", ctypes.c_uint32), ("bvh_lds_nodes", ctypes.c_uint32), ("bvh_width", ctypes.c_uint32),
        ("bvh_max_stack", ctypes.c_uint32), ("bvh_sah_cost", ctypes.c_double),
        ("build_ms", ctypes.c_double), ("device_bytes", ctypes.c_uint64),
        ("occluder_planes", ctypes.c_uint32), ("occluder_culled", ctypes.c_uint32),
        ("occluder_nodes", ctypes.c_uint32), ("occluder_margin", ctypes.c_float),
        ("occluder_max_stack", ctypes.c_uint32), ("occluder_cos_min", ctypes.c_float),
        ("occluder_plane", (ctypes.c_float * 4) * 8),
        ("convex_solids", ctypes.c_uint32), ("convex_delta", ctypes.c_float),
        ("convex_obb", (ctypes.c_float * 16) * 4), ("convex_face_tris", (ctypes.c_uint32 * 8) * 4),
    ]


def _plain(v):
    """ctypes arrays (nested) to lists; scalars unchanged."""
    return [_plain(x) for x in v] if isinstance(v, ctypes.Array) else v


class RendererDesc(ctypes.Structure):
    _fields_ = [
        ("scene", ctypes.c_void_p),
        ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
        ("max_path_length", ctypes.c_uint32),
        ("seed", ctypes.c_uint64),
        ("shard_rank", ctypes.c_uint32), ("shard_count", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("stream", ctypes.c_void_p),
        ("image", ctypes.c_void_p),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("frame_index", ctypes.c_uint64), ("paths", ctypes.c_uint64), ("active_ray_bounces", ctypes.c_uint64),
        ("last_draw_ms", ctypes.c_double), ("mpaths_per_s", ctypes.c_double),
        ("kernel_launches", ctypes.c_uint64), ("kernel_ms", ctypes.c_double), ("owned_pixels", ctypes.c_uint64),
        ("timed_launches", ctypes.c_uint64), ("kernel", ctypes.c_uint32), ("inflight", ctypes.c_uint32),
        ("span_ms", ctypes.c_double), ("spans", ctypes.c_uint64),
        ("primary_blocks", ctypes.c_uint32), ("primary_mean", ctypes.c_float),
        ("noise_ms", ctypes.c_double), ("noise_tables", ctypes.c_uint64),
        ("draws", ctypes.c_uint64), ("draws_overlapped", ctypes.c_uint64), ("inflight_waits", ctypes.c_uint64),
        ("noise_waits", ctypes.c_uint64), ("noise_prefetched", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTED = [
    "mrt_scene_create", "mrt_scene_info_get", "mrt_scene_export", "mrt_scene_destroy", "mrt_scene_check_bvh",
    "mrt_raygen", "mrt_intersect", "mrt_shade", "mrt_resolve_shadow", "mrt_accumulate",
    "mrt_renderer_create", "mrt_renderer_resize", "mrt_renderer_reset", "mrt_renderer_prepare",
    "mrt_renderer_draw", "mrt_renderer_draw_n", "mrt_renderer_sync", "mrt_renderer_image", "mrt_renderer_stream",
    "mrt_renderer_read_image", "mrt_renderer_save_image", "mrt_renderer_stats", "mrt_renderer_destroy",
    "mrt_last_error", "mrt_abi_version", "mrt_noise_table", "mrt_device_count", "mrt_synchronize",
    "mrt_event_record", "mrt_event_synchronize", "mrt_event_destroy",
    "mrt_debug_stamps", "mrt_debug_wave_times", "mrt_shard_mask",
    "mrt_tiles_packed_floats", "mrt_tiles_pack", "mrt_tiles_unpack", "mrt_display", "mrt_renderer_set_max_frames",
    "mrt_accel_create", "mrt_accel_rebuild", "mrt_accel_intersect", "mrt_accel_info_get", "mrt_accel_destroy",
    "mrt_comm_unique_id", "mrt_comm_create", "mrt_comm_destroy", "mrt_renderer_exchange",
    "mrt_renderer_exchange_flush", "mrt_renderer_tiles_read", "mrt_renderer_tiles_write",
    "mrt_image_load_exr", "mrt_renderer_load_reference", "mrt_renderer_display",
    "mrt_renderer_display_enqueue", "mrt_renderer_display_map",
    "mrt_debug_lanes", "mrt_debug_exchange_unpack", "mrt_debug_box_margin",
    "mrt_debug_magic_div", "mrt_comm_set_timeout", "mrt_comm_check", "mrt_debug_comm_fail",
]

_lib = None


def build(jobs: int = 4) -> None:
    """Compile libmrt.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MrtError(f"native library missing: {LIB_PATH} (run __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i64, c_int = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
    sig = {
        "mrt_scene_create": [ctypes.POINTER(SceneDesc), ctypes.POINTER(vp)],
        "mrt_scene_info_get": [vp, ctypes.POINTER(SceneInfo)],
        "mrt_scene_export": [vp, vp, vp, vp, vp, vp],
        "mrt_scene_destroy": [vp],
        "mrt_scene_check_bvh": [vp],
        "mrt_raygen": [vp, u32, u32, vp, vp, u32, vp],
        "mrt_intersect": [vp, vp, u32, u32, vp, u32, vp],
        "mrt_shade": [vp, u32, u32, u32, u32, vp, vp, vp, vp, u32, vp],
        "mrt_resolve_shadow": [vp, u32, vp, vp, vp, u32, vp],
        "mrt_accumulate": [vp, u32, u32, u32, vp, vp, u32, vp],
        "mrt_renderer_create": [ctypes.POINTER(RendererDesc), ctypes.POINTER(vp)],
        "mrt_renderer_resize": [vp, u32, u32],
        "mrt_renderer_reset": [vp],
        "mrt_renderer_prepare": [vp, u32],
        "mrt_renderer_draw": [vp],
        "mrt_renderer_draw_n": [vp, u32],
        "mrt_renderer_sync": [vp],
        "mrt_renderer_image": [vp, ctypes.POINTER(vp)],
        "mrt_renderer_stream": [vp, ctypes.POINTER(vp)],
        "mrt_renderer_read_image": [vp, vp, ctypes.c_size_t],
        "mrt_renderer_save_image": [vp, ctypes.c_char_p],
        "mrt_renderer_stats": [vp, ctypes.POINTER(Stats)],
        "mrt_renderer_destroy": [vp],
        "mrt_last_error": [],
        "mrt_abi_version": [],
        "mrt_noise_table": [u64, i64, vp],
        "mrt_device_count": [],
        "mrt_synchronize": [vp],
        "mrt_event_record": [vp, ctypes.POINTER(vp)],
        "mrt_event_synchronize": [vp],
        "mrt_event_destroy": [vp],
        "mrt_debug_stamps": [vp, c_int],
        "mrt_debug_wave_times": [vp, ctypes.c_size_t],
        "mrt_debug_lanes": [vp, ctypes.c_size_t, c_int],
        "mrt_debug_exchange_unpack": [vp, u32, vp, ctypes.c_size_t],
        "mrt_debug_box_margin": [vp, vp, u32, u32, vp, vp],
        "mrt_debug_magic_div": [u32, vp, u32, vp],
        "mrt_comm_set_timeout": [vp, u32],
        "mrt_comm_check": [vp],
        "mrt_debug_comm_fail": [vp, u32],
        "mrt_shard_mask": [u32, u32, u32, u32, vp, vp],
        "mrt_tiles_packed_floats": [u32, u32, u32, u32, ctypes.POINTER(u64)],
        "mrt_display": [vp, vp, vp, u32, u32, u32, ctypes.c_float, vp],
        "mrt_renderer_set_max_frames": [vp, u32],
        "mrt_tiles_pack": [vp, u32, u32, u32, u32, vp, vp],
        "mrt_tiles_unpack": [vp, u32, u32, u32, u32, vp, vp],
        "mrt_accel_create": [ctypes.POINTER(AccelDesc), ctypes.POINTER(vp)],
        "mrt_accel_rebuild": [vp],
        "mrt_accel_intersect": [vp, vp, u32, u32, vp, u32, vp],
        "mrt_accel_info_get": [vp, ctypes.POINTER(AccelInfo)],
        "mrt_accel_destroy": [vp],
        "mrt_comm_unique_id": [vp, ctypes.c_size_t],
        "mrt_comm_create": [vp, u32, u32, c_int, ctypes.POINTER(vp)],
        "mrt_comm_destroy": [vp],
        "mrt_renderer_exchange": [vp, vp, u32],
        "mrt_renderer_exchange_flush": [vp],
        "mrt_renderer_tiles_read": [vp, vp, ctypes.c_size_t],
        "mrt_renderer_tiles_write": [vp, u32, vp, ctypes.c_size_t],
        "mrt_image_load_exr": [ctypes.c_char_p, vp, ctypes.c_size_t, ctypes.POINTER(u32), ctypes.POINTER(u32)],
        "mrt_renderer_load_reference": [vp, ctypes.c_char_p],
        "mrt_renderer_display": [vp, u32, ctypes.c_float, vp, ctypes.c_size_t],
        "mrt_renderer_display_enqueue": [vp, u32, ctypes.c_float, u32],
        "mrt_renderer_display_map": [vp, u32, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)],
    }
    for name, args in sig.items():
        fn = getattr(L, name, None)
        if fn is None and os.environ.get("MRT_LIB"):   # an older diagnostic build (A/B): entries it lacks
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = c_int
    L.mrt_last_error.restype = ctypes.c_char_p
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        e = MrtError(f"{what} failed ({rc}): {lib().mrt_last_error().decode()}")
        e.status = rc
        raise e


def scene_path(name: str) -> str:
    """Path of a scene shipped with the package (metal-renderer_amd/scenes: the
    reference's renderer/Media OBJ/MTL data files, unchanged)."""
    return name if os.path.sep in name else os.path.join(SCENES_DIR, name if name.endswith(".obj") else name + ".obj")


class Scene:
    """Flattened scene + BVH on the device (initRaytracing, Renderer.mm:255-470)."""

    def __init__(self, obj: str, mtl_override: str | None = None, *, procedural_triangles: int = 0,
                 procedural_seed: int = 1, max_leaf_size: int = 0, lds_nodes: int = 0, device: int = 0,
                 bvh_width: int = 0, bvh_builder: int = 0, occluder_tree: bool = True):
        self._h = None
        d = SceneDesc(scene_path(obj).encode(), (mtl_override or "").encode(), procedural_triangles,
                      procedural_seed, max_leaf_size, lds_nodes, device, bvh_width, bvh_builder,
                      0 if occluder_tree else 1)
        h = ctypes.c_void_p()
        _check(lib().mrt_scene_create(ctypes.byref(d), ctypes.byref(h)), "mrt_scene_create")
        self._h = h
        info = SceneInfo()
        _check(lib().mrt_scene_info_get(h, ctypes.byref(info)), "mrt_scene_info_get")
        self.info = {k: _plain(getattr(info, k)) for k, _ in SceneInfo._fields_}

    @property
    def handle(self):
        return self._h

    def export(self):
        """Flattened reference-layout buffers as numpy structured arrays."""
        import numpy as np
        n = self.info
        vt = np.dtype({"names": ["v", "n"], "formats": [("<f4", 3), ("<f4", 3)], "offsets": [0, 12], "itemsize": 24})
        mt = np.dtype({"names": ["diffuse", "emissive", "ior", "materialType"],
                       "formats": [("<f4", 3), ("<f4", 3), "<f4", "<u4"], "offsets": [0, 12, 24, 28], "itemsize": 32})
        rt = np.dtype({"names": ["tri", "materialIndex", "lightTriangleIndex"],
                       "formats": [("<u4", 3), "<u4", "<u4"], "offsets": [0, 12, 16], "itemsize": 20})
        lt = np.dtype({"names": ["emissive", "v1", "v2", "v3", "area", "pdf", "cdf", "index"],
                       "formats": [("<f4", 3), vt, vt, vt, "<f4", "<f4", "<f4", "<u4"],
                       "offsets": [0, 12, 36, 60, 84, 88, 92, 96], "itemsize": 100})
        V = np.zeros(n["vertices"], vt)
        I = np.zeros(3 * n["triangles"], np.uint32)
        M = np.zeros(n["materials"], mt)
        R = np.zeros(n["triangles"], rt)
        Lt = np.zeros(n["light_triangles"] + 1, lt)
        p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        _check(lib().mrt_scene_export(self._h, p(V), p(I), p(M), p(R), p(Lt)), "mrt_scene_export")
        return {"vertices": V, "indices": I, "materials": M, "references": R, "lights": Lt}

    def check_bvh(self) -> None:
        _check(lib().mrt_scene_check_bvh(self._h), "mrt_scene_check_bvh")

    def box_margin(self, rays, intersections):
        """Host-only test entry mrt_debug_box_margin: per ray (numpy records,
        reference layout) and its nearest hit, the culling slack the hit needs
        in the main tree, as (precise, fast) slab arithmetic, then the same for
        the hit's near ties (mrt.h): float32 [n, 4]."""
        import numpy as np
        rays = np.ascontiguousarray(rays)
        intersections = np.ascontiguousarray(intersections)
        assert len(rays) == len(intersections) and intersections.dtype.itemsize == 16
        out = np.zeros((len(rays), 4), np.float32)
        p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        _check(lib().mrt_debug_box_margin(self._h, p(rays), rays.dtype.itemsize, len(rays), p(intersections), p(out)),
               "mrt_debug_box_margin")
        return out

    def close(self):
        if self._h:
            lib().mrt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Accel:
    """MPSTriangleAccelerationStructure + MPSRayIntersector over caller-owned
    device buffers (renderer/Renderer.mm:456-469): positions at `vertex_stride`
    (24 = sizeof(Vertex)), uint32 indices, nearest-hit queries."""

    def __init__(self, vertices_ptr: int, vertex_stride: int, indices_ptr: int, triangle_count: int, *,
                 device: int = 0, builder: int = 0, max_leaf_size: int = 0, stream: int | None = None):
        self._h = None
        d = AccelDesc(vertices_ptr, vertex_stride, indices_ptr, triangle_count, device, builder, max_leaf_size,
                      stream)
        h = ctypes.c_void_p()
        _check(lib().mrt_accel_create(ctypes.byref(d), ctypes.byref(h)), "mrt_accel_create")
        self._h = h

    def rebuild(self) -> None:
        _check(lib().mrt_accel_rebuild(self._h), "mrt_accel_rebuild")

    def info(self) -> dict:
        i = AccelInfo()
        _check(lib().mrt_accel_info_get(self._h, ctypes.byref(i)), "mrt_accel_info_get")
        return {k: getattr(i, k) for k, _ in AccelInfo._fields_}

    def intersect(self, rays_ptr: int, stride: int, count: int, isect_ptr: int, precise=True, stream=None,
                  sync=True) -> None:
        _check(lib().mrt_accel_intersect(self._h, rays_ptr, stride, count, isect_ptr, _flags(precise), stream),
               "mrt_accel_intersect")
        if sync:
            synchronize(stream)

    def close(self):
        if self._h:
            lib().mrt_accel_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """One accumulating renderer on one device (the reference's `Renderer`)."""

    def __init__(self, scene: Scene, width: int, height: int, max_path_length: int = 8, *,
                 seed: int = DEFAULT_SEED, shard_rank: int = 0, shard_count: int = 1, precise: bool = False,
                 profile: bool = False, stream: int | None = None, image_ptr: int | None = None,
                 animate_noise: bool = True, accumulate_image: bool = True, debug_material: bool = False):
        """animate_noise / accumulate_image / debug_material: the reference's
        ANIMATE_NOISE, ACCUMULATE_IMAGE and DEBUG_MATERIAL switches (defaults =
        the reference's defaults)."""
        self._h = None
        self.scene = scene  # keep alive
        flags = ((FLAG_PRECISE if precise else 0) | (FLAG_PROFILE if profile else 0) |
                 (0 if animate_noise else FLAG_STATIC_NOISE) | (0 if accumulate_image else FLAG_NO_ACCUMULATE) |
                 (FLAG_DEBUG_MATERIAL if debug_material else 0))
        d = RendererDesc(scene.handle, width, height, max_path_length, seed, shard_rank, shard_count, flags,
                         stream, image_ptr)
        h = ctypes.c_void_p()
        _check(lib().mrt_renderer_create(ctypes.byref(d), ctypes.byref(h)), "mrt_renderer_create")
        self._h = h
        self.width, self.height = width, height

    # -mtkView:drawableSizeWillChange:
    def resize(self, width: int, height: int) -> None:
        _check(lib().mrt_renderer_resize(self._h, width, height), "mrt_renderer_resize")
        self.width, self.height = width, height

    def reset(self) -> None:
        _check(lib().mrt_renderer_reset(self._h), "mrt_renderer_reset")

    def prepare(self, frames: int) -> None:
        _check(lib().mrt_renderer_prepare(self._h, frames), "mrt_renderer_prepare")

    # -drawInMTKView:
    def draw(self, frames: int = 1) -> None:
        _check(lib().mrt_renderer_draw_n(self._h, frames), "mrt_renderer_draw_n")

    def draw_frame(self) -> None:
        """One drawInMTKView: frame (mrt_renderer_draw, 1 spp): enqueued
        without waiting for the GPU (at most 3 draws in flight, the
        reference's MaxBuffersInFlight)."""
        _check(lib().mrt_renderer_draw(self._h), "mrt_renderer_draw")

    def set_max_frames(self, n: int) -> None:
        """MAX_FRAMES (Renderer.mm:589-590): draws past frame n are no-ops (0 = unlimited)."""
        _check(lib().mrt_renderer_set_max_frames(self._h, n), "mrt_renderer_set_max_frames")

    def sync(self) -> None:
        _check(lib().mrt_renderer_sync(self._h), "mrt_renderer_sync")

    def image_ptr(self) -> int:
        p = ctypes.c_void_p()
        _check(lib().mrt_renderer_image(self._h, ctypes.byref(p)), "mrt_renderer_image")
        return p.value

    def stream(self) -> int:
        """The renderer's main stream (libmrt's HIP runtime)."""
        p = ctypes.c_void_p()
        _check(lib().mrt_renderer_stream(self._h, ctypes.byref(p)), "mrt_renderer_stream")
        return p.value

    def read_image(self):
        """[H, W, 4] float32, row 0 = bottom (the reference texture orientation)."""
        import numpy as np
        img = np.zeros((self.height, self.width, 4), np.float32)
        _check(lib().mrt_renderer_read_image(self._h, ctypes.c_void_p(img.ctypes.data), img.size),
               "mrt_renderer_read_image")
        return img

    # -saveCurrentImage
    def save_current_image(self, path: str) -> None:
        _check(lib().mrt_renderer_save_image(self._h, path.encode()), "mrt_renderer_save_image")

    # ---- multi-GPU exchange (include/mrt.h: mrt_renderer_exchange) ----
    def exchange(self, comm: "Comm", mode: int = EXCHANGE_GATHER) -> None:
        """Enqueue the image exchange of this shard renderer on its stream:
        RCCL gather of the packed owned tiles to rank 0 (or SUM reduce)."""
        _check(lib().mrt_renderer_exchange(self._h, comm.handle, mode), "mrt_renderer_exchange")

    def exchange_flush(self) -> None:
        _check(lib().mrt_renderer_exchange_flush(self._h), "mrt_renderer_exchange_flush")

    def tiles_read(self, rank: int, count: int):
        """This shard's owned tiles packed into host memory (float32)."""
        import numpy as np
        out = np.zeros(tiles_packed_floats(self.width, self.height, rank, count), np.float32)
        _check(lib().mrt_renderer_tiles_read(self._h, ctypes.c_void_p(out.ctypes.data), out.size),
               "mrt_renderer_tiles_read")
        return out

    def tiles_write(self, shard_rank: int, packed) -> None:
        """Write another shard's packed tiles (host float32) into the image."""
        import numpy as np
        packed = np.ascontiguousarray(packed, np.float32)
        _check(lib().mrt_renderer_tiles_write(self._h, shard_rank, ctypes.c_void_p(packed.ctypes.data), packed.size),
               "mrt_renderer_tiles_write")

    def debug_exchange_unpack(self, nranks: int, gathered) -> None:
        """Test entry: rank 0's unpack of an nranks-way gather whose received
        buffer is `gathered` (host float32, nranks slabs of
        tiles_packed_floats(W, H, 0, nranks) floats) — the RCCL path's unpack
        of slabs 1..N-1 without a communicator."""
        import numpy as np
        g = np.ascontiguousarray(gathered, np.float32)
        _check(lib().mrt_debug_exchange_unpack(self._h, nranks, ctypes.c_void_p(g.ctypes.data), g.size),
               "mrt_debug_exchange_unpack")

    # ---- golden comparison (loadReferenceImage + blitFragment) ----
    def load_reference(self, path: str) -> None:
        _check(lib().mrt_renderer_load_reference(self._h, path.encode()), "mrt_renderer_load_reference")

    def display(self, flags: int = 0, compare_scale: float = 10.0):
        """[H, W, 4] float32 blit of the image (row 0 = bottom)."""
        import numpy as np
        img = np.zeros((self.height, self.width, 4), np.float32)
        _check(lib().mrt_renderer_display(self._h, flags, compare_scale, ctypes.c_void_p(img.ctypes.data), img.size),
               "mrt_renderer_display")
        return img

    def display_enqueue(self, slot: int, flags: int = 0, compare_scale: float = 10.0) -> None:
        """Queue the blit of the image into display slot `slot` (no host wait)."""
        _check(lib().mrt_renderer_display_enqueue(self._h, flags, compare_scale, slot), "mrt_renderer_display_enqueue")

    def display_map(self, slot: int):
        """[H, W, 4] float32 copy of display slot `slot` (waits for its blit)."""
        import numpy as np
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        _check(lib().mrt_renderer_display_map(self._h, slot, ctypes.byref(p), ctypes.byref(n)),
               "mrt_renderer_display_map")
        buf = (ctypes.c_float * n.value).from_address(p.value)
        return np.frombuffer(buf, np.float32).reshape(self.height, self.width, 4).copy()

    def stats(self) -> dict:
        s = Stats()
        _check(lib().mrt_renderer_stats(self._h, ctypes.byref(s)), "mrt_renderer_stats")
        return s.as_dict()

    def close(self):
        if self._h:
            lib().mrt_renderer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- stage-level ABI (device pointers, reference AoS layouts) -------------
# Each call launches on `stream` (None = libmrt's default stream) and, unless
# sync=False, waits for it with mrt_synchronize (torch.cuda.synchronize() does
# not see libmrt's runtime copy).
def synchronize(stream=None) -> None:
    _check(lib().mrt_synchronize(stream), "mrt_synchronize")


def _flags(precise):
    return FLAG_PRECISE if precise else 0


def raygen(scene: Scene, width: int, height: int, noise_ptr: int, rays_ptr: int, precise=True, stream=None,
           sync=True):
    _check(lib().mrt_raygen(scene.handle, width, height, noise_ptr, rays_ptr, _flags(precise), stream), "mrt_raygen")
    if sync:
        synchronize(stream)


def intersect(scene: Scene, rays_ptr: int, stride: int, count: int, isect_ptr: int, precise=True, stream=None,
              sync=True):
    _check(lib().mrt_intersect(scene.handle, rays_ptr, stride, count, isect_ptr, _flags(precise), stream),
           "mrt_intersect")
    if sync:
        synchronize(stream)


def shade(scene: Scene, width, height, frame_index, max_path_length, noise_ptr, isect_ptr, rays_ptr, srays_ptr,
          precise=True, stream=None, sync=True, debug_material=False):
    flags = _flags(precise) | (FLAG_DEBUG_MATERIAL if debug_material else 0)
    _check(lib().mrt_shade(scene.handle, width, height, frame_index, max_path_length, noise_ptr, isect_ptr, rays_ptr,
                           srays_ptr, flags, stream), "mrt_shade")
    if sync:
        synchronize(stream)


def resolve_shadow(scene: Scene, count, isect_ptr, rays_ptr, srays_ptr, precise=True, stream=None, sync=True):
    _check(lib().mrt_resolve_shadow(scene.handle, count, isect_ptr, rays_ptr, srays_ptr, _flags(precise), stream),
           "mrt_resolve_shadow")
    if sync:
        synchronize(stream)


def accumulate(scene: Scene, width, height, frame_index, rays_ptr, image_ptr, precise=True, stream=None, sync=True,
               accumulate_image=True):
    flags = _flags(precise) | (0 if accumulate_image else FLAG_NO_ACCUMULATE)
    _check(lib().mrt_accumulate(scene.handle, width, height, frame_index, rays_ptr, image_ptr, flags,
                                stream), "mrt_accumulate")
    if sync:
        synchronize(stream)


def noise_table(seed: int, frame: int):
    import numpy as np
    out = np.zeros(64 * 64 * 4, np.float32)
    _check(lib().mrt_noise_table(seed, frame, ctypes.c_void_p(out.ctypes.data)), "mrt_noise_table")
    return out


def shard_mask(width: int, height: int, rank: int, count: int):
    """[H, W] uint8 ownership mask of a shard (row 0 = bottom) and its pixel count."""
    import numpy as np
    m = np.zeros((height, width), np.uint8)
    n = np.zeros(1, np.uint64)
    _check(lib().mrt_shard_mask(width, height, rank, count, ctypes.c_void_p(m.ctypes.data),
                                ctypes.c_void_p(n.ctypes.data)), "mrt_shard_mask")
    return m, int(n[0])


DISPLAY_TONEMAP, DISPLAY_SRGB = 1, 2


def display_compare(mode: int) -> int:
    return mode << 8


def display(image_ptr: int, out_ptr: int, width: int, height: int, flags: int = 0, reference_ptr: int | None = None,
            compare_scale: float = 10.0, stream=None, sync=True) -> None:
    """blitFragment (Shaders.metal:33-70): tone map / sRGB / golden comparison on the device."""
    _check(lib().mrt_display(image_ptr, reference_ptr, out_ptr, width, height, flags, compare_scale, stream),
           "mrt_display")
    if sync:
        synchronize(stream)


def tiles_packed_floats(width: int, height: int, rank: int, count: int) -> int:
    n = ctypes.c_uint64()
    _check(lib().mrt_tiles_packed_floats(width, height, rank, count, ctypes.byref(n)), "mrt_tiles_packed_floats")
    return n.value


def tiles_pack(image_ptr: int, width: int, height: int, rank: int, count: int, packed_ptr: int, stream=None,
               sync=True) -> None:
    """A shard's owned tiles of a device image -> dense [tile][64*64] RGBA32F (multi-GPU exchange)."""
    _check(lib().mrt_tiles_pack(image_ptr, width, height, rank, count, packed_ptr, stream), "mrt_tiles_pack")
    if sync:
        synchronize(stream)


def tiles_unpack(packed_ptr: int, width: int, height: int, rank: int, count: int, image_ptr: int, stream=None,
                 sync=True) -> None:
    _check(lib().mrt_tiles_unpack(packed_ptr, width, height, rank, count, image_ptr, stream), "mrt_tiles_unpack")
    if sync:
        synchronize(stream)


def tiles_pack_host(image, rank: int, count: int):
    """numpy restatement of mrt_tiles_pack (host rehearsal of the exchange; image is H x W x 4)."""
    import numpy as np
    H, W = image.shape[:2]
    tx_n, ty_n = (W + 63) // 64, (H + 63) // 64
    tiles = list(range(rank, tx_n * ty_n, count))
    out = np.zeros((len(tiles), 64, 64, 4), np.float32)
    for k, t in enumerate(tiles):
        ty, tx = divmod(t, tx_n)
        blk = image[ty * 64:(ty + 1) * 64, tx * 64:(tx + 1) * 64]
        out[k, :blk.shape[0], :blk.shape[1]] = blk
    return out


def tiles_unpack_host(packed, image, rank: int, count: int) -> None:
    H, W = image.shape[:2]
    tx_n, ty_n = (W + 63) // 64, (H + 63) // 64
    for k, t in enumerate(range(rank, tx_n * ty_n, count)):
        ty, tx = divmod(t, tx_n)
        h, w = min(64, H - ty * 64), min(64, W - tx * 64)
        image[ty * 64:ty * 64 + h, tx * 64:tx * 64 + w] = packed[k, :h, :w]


def debug_magic_div(d: int, n):
    """n // d through libmrt's exact launch-divisor division (test entry)."""
    import numpy as np
    n = np.ascontiguousarray(n, np.uint32)
    q = np.zeros(len(n), np.uint32)
    _check(lib().mrt_debug_magic_div(d, ctypes.c_void_p(n.ctypes.data), len(n), ctypes.c_void_p(q.ctypes.data)),
           "mrt_debug_magic_div")
    return q


def debug_stamps(reset: bool = True):
    import numpy as np
    out = np.zeros(8, np.uint64)
    _check(lib().mrt_debug_stamps(ctypes.c_void_p(out.ctypes.data), int(reset)), "mrt_debug_stamps")
    return out


def debug_lanes(reset: bool = True):
    """Lane-occupancy counters of the lane-statistics library (zeros in the
    product library); tools/lane_stats.py names the slots."""
    import numpy as np
    out = np.zeros(64, np.uint64)
    _check(lib().mrt_debug_lanes(ctypes.c_void_p(out.ctypes.data), out.size, int(reset)), "mrt_debug_lanes")
    return out


def debug_wave_times():
    """Per-wave timeline of the last launch of each bounce index % 4 (stamp
    library only), shape (4, 8192, 16), 100 MHz ticks: {start, exit,
    iterations | exit reason << 32, last grab, end of the last grab's work,
    summed grab latency, max grab latency, last grab's latency, phase
    cycles 0..4, 0, 0, 0}."""
    import numpy as np
    out = np.zeros((4, 8192, 16), np.uint64)
    _check(lib().mrt_debug_wave_times(ctypes.c_void_p(out.ctypes.data), out.size), "mrt_debug_wave_times")
    return out


class Event:
    """A completion marker on a libmrt stream (host-side ordering against
    another runtime's work, e.g. torch/RCCL in the multi-GPU exchange)."""

    def __init__(self):
        self._e = ctypes.c_void_p()

    def record(self, stream=None) -> None:
        _check(lib().mrt_event_record(stream, ctypes.byref(self._e)), "mrt_event_record")

    def synchronize(self) -> None:
        _check(lib().mrt_event_synchronize(self._e), "mrt_event_synchronize")

    def close(self) -> None:
        if self._e.value:
            _check(lib().mrt_event_destroy(self._e), "mrt_event_destroy")
            self._e = ctypes.c_void_p()


def load_exr(path: str):
    """Decode a scanline OpenEXR file (libmrt's reader): [H, W, 4] float32,
    row 0 = BOTTOM."""
    import numpy as np
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib().mrt_image_load_exr(path.encode(), None, 0, ctypes.byref(w), ctypes.byref(h)), "mrt_image_load_exr")
    img = np.zeros((h.value, w.value, 4), np.float32)
    _check(lib().mrt_image_load_exr(path.encode(), ctypes.c_void_p(img.ctypes.data), img.size, ctypes.byref(w),
                                    ctypes.byref(h)), "mrt_image_load_exr")
    return img


def comm_unique_id() -> bytes:
    """ncclGetUniqueId on rank 0; distribute the bytes to every rank."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check(lib().mrt_comm_unique_id(buf, COMM_ID_BYTES), "mrt_comm_unique_id")
    return buf.raw


class Comm:
    """RCCL communicator of one rank (one process per GPU)."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int = 0):
        self._h = None
        if len(unique_id) != COMM_ID_BYTES:
            raise MrtError("unique id must be 128 bytes")
        h = ctypes.c_void_p()
        _check(lib().mrt_comm_create(ctypes.create_string_buffer(unique_id, COMM_ID_BYTES), nranks, rank, device,
                                     ctypes.byref(h)), "mrt_comm_create")
        self._h = h
        self.nranks, self.rank = nranks, rank

    @property
    def handle(self):
        return self._h

    def set_timeout(self, ms: int) -> None:
        """Bound of the renderer's waits for this communicator's collectives (0 = 120 s)."""
        _check(lib().mrt_comm_set_timeout(self._h, ms), "mrt_comm_set_timeout")

    def check(self) -> None:
        """Non-blocking health check: raises MrtError once the communicator is aborted."""
        _check(lib().mrt_comm_check(self._h), "mrt_comm_check")

    def debug_fail(self, mode: int) -> None:
        """Test entry: 1 = report an asynchronous error, 2 = collectives never complete."""
        _check(lib().mrt_debug_comm_fail(self._h, mode), "mrt_debug_comm_fail")

    def close(self):
        if self._h:
            lib().mrt_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    return int(lib().mrt_device_count())
