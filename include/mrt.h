/*
 * mrt.h — C ABI of the MI355X-native path tracer (libmrt.so).
 *
 * This is the drop-in boundary for the hot path of serhii-rieznik/metal-renderer.
 * The reference exposes the path through two boundaries, both reproduced here:
 *
 *   B-1  App <-> renderer:  the Objective-C `Renderer` (renderer/Renderer.h:3-8)
 *        -initWithMetalKitView:            -> mrt_renderer_create
 *        -mtkView:drawableSizeWillChange:  -> mrt_renderer_resize   (Renderer.mm:640-657)
 *        -drawInMTKView:                   -> mrt_renderer_draw     (Renderer.mm:587-638)
 *        -saveCurrentImage                 -> mrt_renderer_save_image (Renderer.mm:659-662;
 *                                             a working save, the reference's is a stub)
 *        window-title stats                -> mrt_renderer_stats    (Renderer.mm:631-637)
 *   B-2  Renderer <-> GPU:  the per-stage dispatches of performRaytracing:
 *        (renderer/Renderer.mm:500-585) over the reference AoS records
 *        (renderer/Raytracing.h:47-123):
 *        rayGenerator        (Shaders.metal:75-103)   -> mrt_raygen
 *        MPS nearest-hit     (Renderer.mm:519-523,545-553; config :464-469)
 *                                                     -> mrt_intersect
 *        MPS rebuild         (Renderer.mm:456-462)    -> mrt_scene_create (BVH build)
 *   MPS itself, over raw vertex/index buffers (Renderer.mm:456-469):
 *        MPSTriangleAccelerationStructure + rebuild -> mrt_accel_create / mrt_accel_rebuild
 *        MPSRayIntersector encodeIntersection (Nearest)  -> mrt_accel_intersect
 *        intersectionHandler (Shaders.metal:105-212)  -> mrt_shade
 *        lightSamplingHandler(Shaders.metal:214-231)  -> mrt_resolve_shadow
 *        accumulateImage     (Shaders.metal:233-249)  -> mrt_accumulate
 *
 * Conventions: every function returns 0 on success and a negative mrt_status
 * on failure; mrt_last_error() returns a thread-local message.  No exception
 * crosses the ABI.  Handles are opaque.  A handle is externally synchronised
 * (one caller thread at a time, like the MTKView main thread).  Device
 * pointers are HIP device memory on the handle's device; `stream` arguments
 * are hipStream_t (NULL = the handle's own stream).
 * Image layout: RGBA32F, W*H*4 floats, row 0 = BOTTOM of the view (the
 * reference's texture orientation, Shaders.metal:81,94).
 */
#ifndef MRT_H_
#define MRT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRT_ABI_VERSION 9

typedef enum mrt_status {
  MRT_OK = 0,
  MRT_ERR_INVALID = -1,   /* bad argument */
  MRT_ERR_IO = -2,        /* scene / image file error */
  MRT_ERR_HIP = -3,       /* HIP runtime error (no device, launch failure, ...) */
  MRT_ERR_NOMEM = -4,
  MRT_ERR_STATE = -5,     /* call not valid in the handle's current state */
  MRT_ERR_COMM = -6       /* ABI 9: an RCCL collective reported an asynchronous error or did not complete
                             within the communicator's timeout; the communicator is aborted and every
                             later use of it fails with this status (renderers stay usable) */
} mrt_status;

/* flags */
#define MRT_FLAG_PRECISE 1u   /* parity kernels: IEEE div/sqrt, no FMA contraction, CR sin/cos */
#define MRT_FLAG_PROFILE 2u   /* time the bounce launches of every 8th frame with HIP events (mrt_stats.kernel_ms);
                                 timing events serialise a stream's launches, so only a sample is timed */
/* The reference's compile-time switches as runtime flags (renderer/Raytracing.h:11-33,
 * renderer/Shaders.metal:7); the defaults (flag clear) are the reference's defaults. */
#define MRT_FLAG_STATIC_NOISE 4u      /* ANIMATE_NOISE 0 (Raytracing.h:20): every frame reads the initial noise
                                         table (Renderer.mm:109-129; :485-497 skipped).  Renderer flag. */
#define MRT_FLAG_NO_ACCUMULATE 8u     /* ACCUMULATE_IMAGE false (Raytracing.h:14, Shaders.metal:241): the image
                                         holds the last frame's radiance alone.  Renderer and mrt_accumulate. */
#define MRT_FLAG_DEBUG_MATERIAL 16u   /* DEBUG_MATERIAL 1 (Shaders.metal:7,142-147): at each hit the path radiance
                                         is set to fresnel(n, -wI, 1.0, 1.5) before emission and NEE add to it.
                                         Renderer and mrt_shade. */

typedef struct mrt_scene mrt_scene;
typedef struct mrt_renderer mrt_renderer;

/* ---- scene (initRaytracing: Renderer.mm:255-470) ------------------------ */
typedef struct mrt_scene_desc {
  const char* obj_path;            /* OBJ scene (renderer/Media/<name>.obj) */
  const char* mtl_override;        /* optional .mtl used instead of the OBJ's mtllib (NULL/"" = none) */
  uint32_t procedural_triangles;   /* >0: append a seeded displaced sphere of this many triangles */
  uint64_t procedural_seed;
  uint32_t max_leaf_size;          /* BVH leaf size, 0 = default (2) */
  uint32_t lds_nodes;              /* top BVH nodes staged in LDS, 0 = default; UINT32_MAX = none */
  int device;                      /* HIP device ordinal; -1 = host only (import + BVH, no upload) */
  uint32_t bvh_width;              /* 4 = BVH4 (the binary SAH tree collapsed), 0 = default (4); other widths are rejected */
  uint32_t bvh_builder;            /* MRT_BVH_*; 0 = default (host binned SAH) */
  uint32_t no_occluder_tree;       /* 1: shadow rays always traverse the main tree (no occluder tree, see
                                      mrt_scene_info.occluder_planes); 0 = default (built for host-SAH
                                      scenes of <= 16384 triangles with culled supporting planes) */
} mrt_scene_desc;

/* BVH builders */
#define MRT_BVH_HOST_SAH 1u      /* host binned-SAH BVH2, collapsed to BVH4 (best traversal quality) */
#define MRT_BVH_DEVICE_LBVH 2u   /* device linear BVH (Morton sort + radix tree, collapsed to BVH4
                                    on the GPU; BVH4 only) — fastest build, weakest tree */
#define MRT_BVH_DEVICE_PLOC 3u   /* device PLOC (Morton sort + nearest-neighbour clustering, collapsed
                                    to BVH4 on the GPU) — near-SAH tree; builds from device buffers */

typedef struct mrt_scene_info {
  uint32_t vertices, triangles, materials, light_triangles;
  uint32_t bvh_nodes, bvh_leaves, bvh_depth, bvh_lds_nodes;
  uint32_t bvh_width, bvh_max_stack;   /* node width; traversal stack entries a ray can need */
  double bvh_sah_cost;
  double build_ms;                 /* host BVH build time */
  uint64_t device_bytes;           /* scene + BVH bytes resident on the device */
  /* shadow-ray occluder tree: triangles in supporting planes with every light
   * strictly inside (walls, floor, ceiling) cannot occlude a shadow ray from
   * an origin inside those planes; such rays traverse a second BVH over the
   * other triangles (same answers).  0 planes = no occluder tree. */
  uint32_t occluder_planes, occluder_culled, occluder_nodes;
  float occluder_margin;
  uint32_t occluder_max_stack;     /* traversal stack entries the occluder tree can need (<= bvh_max_stack:
                                      a deeper occluder tree is not built); renderers size their stack by
                                      the deeper tree.  ABI 7. */
  float occluder_cos_min;          /* shadow rays whose cosine to the target light's normal is below this
                                      traverse the main tree (bound on the light's own t error). ABI 7. */
  /* ABI 8: the culled planes (n, w; outward unit normal n, inside
   * n.x - w <= -occluder_margin), occluder_planes of them */
  float occluder_plane[8][4];
  /* ABI 9: convex occluders — every triangle of the (light-free) occluder
   * tree lies on one of convex_solids parallelepiped solids (e.g. the Cornell
   * box's blocks): shadow rays through that tree are decided per solid by a
   * segment test against its three slabs pushed out by convex_delta, and the
   * leaf test of the face the segment enters, before any walk (kernels.hip
   * convex_occlusion).  convex_obb[c] = three unit axis normals (9 floats),
   * then each axis's padded slab (lo, hi); convex_face_tris[c][2a + side]
   * (side 0: the lo face, 1: the hi face) = its two primitive ids, 16 bits
   * each, 0xFFFF = none. */
  uint32_t convex_solids;
  float convex_delta;
  float convex_obb[4][16];
  uint32_t convex_face_tris[4][8];
} mrt_scene_info;

int mrt_scene_create(const mrt_scene_desc* desc, mrt_scene** out);
int mrt_scene_info_get(const mrt_scene* scene, mrt_scene_info* info);
/* Copy the flattened reference-layout buffers to host memory (any pointer may
 * be NULL): Vertex[24 B], uint32 indices, Material[32 B], TriangleReference[20 B],
 * LightTriangle[100 B] (light_triangles + 1 entries, the sentinel last). */
int mrt_scene_export(const mrt_scene* scene, void* vertices, void* indices, void* materials,
                     void* references, void* lights);
int mrt_scene_destroy(mrt_scene* scene);
/* Structural check of the built BVH (host): every primitive in exactly one
 * leaf, every child box contains its subtree's triangles, depth within the
 * traversal stack.  0 = valid. */
int mrt_scene_check_bvh(const mrt_scene* scene);

/* ---- acceleration structure over raw buffers (the MPS interface) --------
 * MPSTriangleAccelerationStructure (Renderer.mm:456-462): vertexBuffer with
 * vertexStride = sizeof(Vertex) = 24, uint32 indexBuffer, triangleCount =
 * indices / 3, `rebuild` once; MPSRayIntersector (Renderer.mm:464-469):
 * nearest hit, cull none, ray records (origin, minDistance, direction,
 * maxDistance) at rayStride, intersections (distance, primitiveIndex, (u,v)). */
typedef struct mrt_accel mrt_accel;
typedef struct mrt_accel_desc {
  const void* vertices;            /* device pointer: 3 floats (position) at the start of every vertex */
  uint32_t vertex_stride;          /* bytes between vertices (>= 12, multiple of 4) */
  const uint32_t* indices;         /* device pointer: 3 uint32 per triangle */
  uint32_t triangle_count;
  int device;                      /* HIP device of the buffers */
  uint32_t builder;                /* MRT_BVH_*; 0 = default (MRT_BVH_DEVICE_PLOC) */
  uint32_t max_leaf_size;          /* 0 = default (2) */
  void* stream;                    /* hipStream_t of libmrt's runtime, NULL = own stream */
} mrt_accel_desc;
typedef struct mrt_accel_info {
  uint32_t triangles, bvh_nodes, bvh_leaves, bvh_levels, bvh_max_stack, builder;
  double build_ms;                 /* device time (LBVH) or host time (SAH) of the last (re)build */
  uint64_t device_bytes;
} mrt_accel_info;
/* Build the structure (the buffers must stay valid until the next rebuild). */
int mrt_accel_create(const mrt_accel_desc* desc, mrt_accel** out);
/* Rebuild from the same buffers (their contents may have changed). */
int mrt_accel_rebuild(mrt_accel* accel);
/* Nearest hit of `count` ray records of `stride` bytes (contract of mrt_intersect). */
int mrt_accel_intersect(const mrt_accel* accel, const void* rays, uint32_t stride, uint32_t count,
                        void* intersections, uint32_t flags, void* stream);
int mrt_accel_info_get(const mrt_accel* accel, mrt_accel_info* info);
int mrt_accel_destroy(mrt_accel* accel);

/* ---- stage-level ABI (B-2), reference AoS layouts, device pointers ------- */
/* rayGenerator over a W x H grid: noise = 64*64 float4 (one noise slot). */
int mrt_raygen(const mrt_scene* scene, uint32_t width, uint32_t height, const float* noise,
               void* rays /* Ray[W*H], 80 B */, uint32_t flags, void* stream);
/* MPS nearest-hit: records of `stride` bytes whose first 32 B are
 * (origin, minDistance, direction, maxDistance); cull none; distance = -1 on
 * miss or maxDistance < 0; ties -> lowest primitive index. */
int mrt_intersect(const mrt_scene* scene, const void* rays, uint32_t stride, uint32_t count,
                  void* intersections /* Intersection[count], 16 B */, uint32_t flags, void* stream);
/* intersectionHandler for iteration with SharedData.frameIndex = frame_index
 * and MAX_PATH_LENGTH = max_path_length; noise = the slot bound at index 8. */
int mrt_shade(const mrt_scene* scene, uint32_t width, uint32_t height, uint32_t frame_index,
              uint32_t max_path_length, const float* noise, const void* intersections, void* rays,
              void* shadow_rays /* LightSamplingRay[W*H], 48 B */, uint32_t flags, void* stream);
int mrt_resolve_shadow(const mrt_scene* scene, uint32_t count, const void* intersections, void* rays,
                       const void* shadow_rays, uint32_t flags, void* stream);
int mrt_accumulate(const mrt_scene* scene, uint32_t width, uint32_t height, uint32_t frame_index,
                   const void* rays, float* image_rgba, uint32_t flags, void* stream);

/* ---- renderer (B-1) ------------------------------------------------------ */
typedef struct mrt_renderer_desc {
  const mrt_scene* scene;          /* not owned; must outlive the renderer */
  uint32_t width, height;          /* the reference's W,H = CONTENT_SCALE * drawable */
  uint32_t max_path_length;        /* MAX_PATH_LENGTH (Raytracing.h:23), 1..64 */
  uint64_t seed;                   /* replaces the clock seed (Renderer.mm:109,486) */
  uint32_t shard_rank;             /* 64x64 tile t is rendered iff t % shard_count == shard_rank */
  uint32_t shard_count;            /* 0 or 1 = the whole frame */
  uint32_t flags;                  /* MRT_FLAG_* */
  void* stream;                    /* optional external hipStream_t of the SAME HIP runtime as
                                      libmrt (NULL = own stream).  Never pass a stream created
                                      by another runtime copy (e.g. PyTorch's bundled HIP). */
  float* image;                    /* optional external device image (W*H*4 floats), else owned */
} mrt_renderer_desc;

typedef struct mrt_stats {         /* counters are cumulative since create/resize */
  uint64_t frame_index;            /* frames accumulated since create/resize/reset */
  uint64_t paths;                  /* pixel paths traced by this renderer (owned pixels x frames) */
  uint64_t active_ray_bounces;     /* A: rays alive at the start of each bounce, summed */
  double last_draw_ms;             /* GPU time of the last draw/draw_n (HIP events) */
  double mpaths_per_s;             /* paths of the last draw / last_draw_ms */
  uint64_t kernel_launches;        /* bounce-kernel launches issued */
  double kernel_ms;                /* summed durations of the timed launches (MRT_FLAG_PROFILE) */
  uint64_t owned_pixels;
  uint64_t timed_launches;         /* launches behind kernel_ms (every 8th frame's) */
  uint32_t kernel;                 /* the hot kernel: 0 = wavefront of per-bounce launches, 1 = path megakernel,
                                      2 = streaming wavefront (all bounces of a frame batch in one launch) */
  uint32_t inflight;               /* frame batches in flight (render streams); > 1: launches overlap */
  double span_ms;                  /* summed device-measured spans of the frame batches' render launches
                                      (earliest block start to latest wave end, chip wall clock) */
  uint64_t spans;                  /* frame batches behind span_ms (every batch) */
  uint32_t primary_blocks;         /* 8x8 pixel blocks whose camera rays test a candidate list instead of
                                      traversing the BVH (0 = lists off; MRT_PRIMARY=0 disables) */
  float primary_mean;              /* mean candidate-list length over those blocks */
  /* ABI 7: host cost of the noise schedule (the reference regenerates one
   * table per frame on the CPU before the frame's commit, Renderer.mm:486-496;
   * here mrt_renderer_prepare / draw_n generate a window of tables on the host
   * threads and upload it once) */
  double noise_ms;                 /* host wall time generating noise tables (ABI 8: on the schedule's worker
                                      thread, overlapped with rendering; uploads are asynchronous) */
  uint64_t noise_tables;           /* per-frame tables generated (noise_ms / noise_tables = cost per frame) */
  /* ABI 8: the per-frame cadence (drawInMTKView:, Renderer.mm:587-600).  A
   * draw enqueues its launches without waiting for the GPU: noise tables come
   * from device chunks of 64 frames generated ahead on a worker thread and
   * uploaded on their own stream; the one host wait a draw can reach is the
   * reference's in-flight bound (MaxBuffersInFlight = 3 draws, :16, :593). */
  uint64_t draws;                  /* draw / draw_n calls that enqueued frames */
  uint64_t draws_overlapped;       /* draws enqueued while the previous draw was still executing on the GPU */
  uint64_t inflight_waits;         /* draws that waited for the draw 3 back to finish (the in-flight bound) */
  uint64_t noise_waits;            /* draws (and prepares) that waited for a chunk's host generation */
  uint64_t noise_prefetched;       /* chunks the worker generated ahead and a draw found ready */
} mrt_stats;

int mrt_renderer_create(const mrt_renderer_desc* desc, mrt_renderer** out);
/* drawableSizeWillChange: reallocate, frameIndex = 0 (Renderer.mm:640-657) */
int mrt_renderer_resize(mrt_renderer* r, uint32_t width, uint32_t height);
/* frameIndex = 0 without reallocating: the next frame overwrites every pixel
 * the renderer owns (until then the image keeps its content; pixels written
 * by an exchange or mrt_renderer_tiles_write, and an external image, are
 * cleared here); the cumulative counters of mrt_stats are kept. */
int mrt_renderer_reset(mrt_renderer* r);
/* Generate the noise tables for frames [frame_index, frame_index+n) ahead
 * of time and enqueue their upload (the reference regenerates one slot per
 * frame on the CPU, Renderer.mm:486-496).  Blocks on host generation only.
 * draw_n does the same itself when a chunk is missing, and asks the worker
 * thread for the next chunk of 64 frames while these render. */
int mrt_renderer_prepare(mrt_renderer* r, uint32_t n);
/* One frame: 1 spp, MAX_PATH_LENGTH bounces, running-mean accumulation. */
int mrt_renderer_draw(mrt_renderer* r);
int mrt_renderer_draw_n(mrt_renderer* r, uint32_t n);
/* Wait for all queued work of the renderer. */
int mrt_renderer_sync(mrt_renderer* r);
/* Device pointer of the accumulation image (for an RCCL reduce). */
int mrt_renderer_image(mrt_renderer* r, float** device_image);
/* The renderer's main HIP stream (libmrt's runtime): work queued on it, e.g.
 * mrt_tiles_pack of the image, runs after the renderer's draws without a
 * host round trip. */
int mrt_renderer_stream(mrt_renderer* r, void** stream);
/* Synchronise and copy the image to host memory (rgba must hold W*H*4 floats). */
int mrt_renderer_read_image(mrt_renderer* r, float* rgba, size_t count);
/* MAX_FRAMES (Raytracing.h:28, Renderer.mm:589-590): once frame_index reaches
 * max_frames, draws are no-ops (0 = unlimited, the reference's default). */
int mrt_renderer_set_max_frames(mrt_renderer* r, uint32_t max_frames);
/* Save the image top-down as .pfm (float RGB) or .exr (float RGBA, uncompressed). */
int mrt_renderer_save_image(mrt_renderer* r, const char* path);
int mrt_renderer_stats(const mrt_renderer* r, mrt_stats* stats);
int mrt_renderer_destroy(mrt_renderer* r);

/* ---- misc ----------------------------------------------------------------- */
const char* mrt_last_error(void);
int mrt_abi_version(void);
/* The deterministic noise table of SURVEY.md A.3 for frame `frame` (-1 = the
 * initial table), 64*64*4 floats, host memory. */
int mrt_noise_table(uint64_t seed, int64_t frame, float* out16384);
/* Host helper (no device needed): the pixels a shard owns under the 64x64
 * tile round-robin (tile t -> shard t % shard_count), as a W*H byte mask
 * (row 0 = bottom); returns the number of owned pixels via *owned. */
int mrt_shard_mask(uint32_t width, uint32_t height, uint32_t shard_rank, uint32_t shard_count, uint8_t* mask,
                   uint64_t* owned);
/* Display (blitFragment, Shaders.metal:33-70): the reference's compile-time
 * blit switches as flags — tone map 1 - exp(-c) (ENABLE_TONE_MAPPING),
 * toSRGB (MANUAL_SRGB, Raytracing.h:130-135), and COMPARISON_MODE 1..4
 * against a reference image (e.g. a Mitsuba golden, Renderer.mm:162-253)
 * scaled by compare_scale (COMPARISON_SCALE = 10).  Device pointers, W*H
 * RGBA32F in and out; `reference` may be NULL when no compare mode is set. */
#define MRT_DISPLAY_TONEMAP 1u
#define MRT_DISPLAY_SRGB 2u
#define MRT_DISPLAY_COMPARE(mode) ((uint32_t)(mode) << 8)   /* 1 abs, 2 ref-to-color, 3 color-to-ref, 4 luminance */
int mrt_display(const float* image, const float* reference, float* out, uint32_t width, uint32_t height,
                uint32_t flags, float compare_scale, void* stream);

/* Golden images: loadReferenceImage (renderer/Renderer.mm:162-253) reads
 * Media/reference/<scene>-<L>.exr (Mitsuba goldens: ZIP-compressed half RGB)
 * and flips it into the comparison texture.  mrt_image_load_exr decodes a
 * scanline OpenEXR file (NONE / ZIPS / ZIP compression, HALF / FLOAT / UINT
 * channels; R, G, B, A by name, A = 1 if absent) into host RGBA32F with
 * row 0 = BOTTOM; call with rgba = NULL to get the size first.  No device. */
int mrt_image_load_exr(const char* path, float* rgba, size_t capacity_floats, uint32_t* width, uint32_t* height);
/* The renderer's comparison image (COMPARISON_MODE != 0): the golden at
 * `path`, which must have the renderer's W x H, uploaded to the device. */
int mrt_renderer_load_reference(mrt_renderer* r, const char* path);
/* blitFragment for a host without its own GPU code: mrt_display of the
 * accumulation image (tone map / sRGB / compare mode against the loaded
 * reference) into host memory (rgba: W*H*4 floats, row 0 = bottom). */
int mrt_renderer_display(mrt_renderer* r, uint32_t flags, float compare_scale, float* rgba, size_t count);
/* The same blit without a host wait, for a frame loop that keeps frames in
 * flight as the reference does (MaxBuffersInFlight = 3, its semaphore:
 * renderer/Renderer.mm:16,593-600).  _enqueue queues the blit of the image
 * as of the draws queued so far, and its copy into display slot `slot`
 * (< MRT_DISPLAY_SLOTS; pinned host memory owned by the renderer), on the
 * renderer's stream, and returns at once.  _map waits for that slot's copy
 * and returns its pixels (W*H*4 floats, row 0 = bottom), valid until the
 * slot is enqueued again or the renderer is resized or destroyed.  Typical
 * loop: draw; enqueue(frame % 3); present map((frame - 2) % 3). */
#define MRT_DISPLAY_SLOTS 3u
int mrt_renderer_display_enqueue(mrt_renderer* r, uint32_t flags, float compare_scale, uint32_t slot);
int mrt_renderer_display_map(mrt_renderer* r, uint32_t slot, const float** rgba, size_t* count);

/* Multi-GPU exchange of the accumulation image: a shard's
 * owned 64x64 tiles packed densely, [k][64*64] RGBA32F for its k-th owned
 * tile (tile t = shard_rank + k*shard_count, row-major tiles; zeros outside
 * the image).  Device pointers; pack reads `image`, unpack writes only the
 * shard's pixels of `image`.  Bitwise moves.  mrt_tiles_packed_floats gives
 * the packed size (host, no device). */
int mrt_tiles_packed_floats(uint32_t width, uint32_t height, uint32_t shard_rank, uint32_t shard_count,
                            uint64_t* floats);
int mrt_tiles_pack(const float* image, uint32_t width, uint32_t height, uint32_t shard_rank,
                   uint32_t shard_count, float* packed, void* stream);
int mrt_tiles_unpack(const float* packed, uint32_t width, uint32_t height, uint32_t shard_rank,
                     uint32_t shard_count, float* image, void* stream);
/* ---- multi-GPU exchange through RCCL --------------------
 * One process per GPU.  Rank 0 makes a unique id, the host distributes its
 * MRT_COMM_ID_BYTES bytes to every rank (any control channel: MPI, a socket,
 * torch.distributed gloo), each rank creates its communicator on its device,
 * and a renderer created with shard_rank = rank, shard_count = nranks
 * exchanges its accumulation image with one collective, enqueued on the
 * renderer's stream (no host round trip):
 *   MRT_EXCHANGE_GATHER — pack the rank's owned 64x64 tiles densely
 *     (mrt_tiles_pack), one ncclGather of the packed tiles to rank 0
 *     (1/N of the image per rank; on xGMI rank 0 receives the N-1 slabs
 *     over N-1 links at once), rank 0 unpacks them into its image;
 *   MRT_EXCHANGE_REDUCE — one in-place ncclReduce(sum) of the RGBA32F image
 *     to rank 0 (non-owned pixels are 0, so the sum is the 1-GPU image).
 * Either way rank 0's image is bitwise the single-device render.
 * MRT_EXCHANGE_OVERLAP (gather only): the collective runs on the
 * communicator's own stream after the pack, and rank 0's unpack is deferred
 * to the next exchange (or mrt_renderer_exchange_flush), so the transfer
 * overlaps the renderer's next draw; the packed tiles are double-buffered.
 * The reference has no multi-GPU path (a single Metal device). */
#define MRT_COMM_ID_BYTES 128
#define MRT_EXCHANGE_GATHER 1u
#define MRT_EXCHANGE_REDUCE 2u
#define MRT_EXCHANGE_OVERLAP 0x100u
typedef struct mrt_comm mrt_comm;
int mrt_comm_unique_id(void* id, size_t bytes);   /* ncclGetUniqueId: bytes >= MRT_COMM_ID_BYTES */
int mrt_comm_create(const void* id, uint32_t nranks, uint32_t rank, int device, mrt_comm** out);
int mrt_comm_destroy(mrt_comm* comm);
int mrt_renderer_exchange(mrt_renderer* r, mrt_comm* comm, uint32_t mode);
/* Complete a deferred (MRT_EXCHANGE_OVERLAP) exchange on the renderer's stream
 * and wait, bounded by the communicator's timeout, for the collective to
 * complete on the device (ABI 9; mrt_renderer_sync / _read_image wait the same
 * way).  Meanwhile the communicator's asynchronous error is polled
 * (ncclCommGetAsyncError); on an error or at the timeout it is aborted
 * (ncclCommAbort) and MRT_ERR_COMM is returned with mrt_last_error() set. */
int mrt_renderer_exchange_flush(mrt_renderer* r);
/* ABI 9: the bound of those waits (0 = the default, 120000 ms), and a
 * non-blocking health check (MRT_OK, or MRT_ERR_COMM once aborted or when an
 * asynchronous error is pending — which aborts it). */
int mrt_comm_set_timeout(mrt_comm* comm, uint32_t timeout_ms);
int mrt_comm_check(mrt_comm* comm);
/* Test entry (ABI 9): inject a failure into the communicator's health checks
 * — 1: an asynchronous error is reported; 2: its collectives never complete
 * (the bounded wait reaches the timeout); 0: none.  The abort that follows is
 * the real one (ncclCommAbort). */
int mrt_debug_comm_fail(mrt_comm* comm, uint32_t mode);
/* Host-side exchange for hosts with their own transport (MPI, gloo, ...):
 * the renderer's owned tiles packed to host memory (mrt_tiles_packed_floats
 * floats for its shard), and another shard's packed tiles written into the
 * image.  Both synchronise the renderer. */
int mrt_renderer_tiles_read(mrt_renderer* r, float* host_packed, size_t floats);
int mrt_renderer_tiles_write(mrt_renderer* r, uint32_t shard_rank, const float* host_packed, size_t floats);

/* Wait for work queued by libmrt on `stream` (NULL = everything on the device
 * libmrt's runtime has queued). */
int mrt_synchronize(void* stream);
/* Stream-ordered completion markers in libmrt's runtime (the host-side
 * ordering between libmrt's work and another runtime's, e.g. the multi-GPU
 * exchange): record an event on `stream` (NULL = the default stream),
 * creating it first when *event is NULL; wait for it; destroy it. */
int mrt_event_record(void* stream, void** event);
int mrt_event_synchronize(void* event);
int mrt_event_destroy(void* event);
/* Diagnostics: cycles spent per phase of the bounce loop, summed over the
 * waves of the last launch of each bounce index % 4 (out[0..4] = load, trace, shade, shadow, finish; out[5] = wave iterations).
 * Non-zero only in the separately built stamp library (make stamps). */
int mrt_debug_stamps(uint64_t* out8, int reset);
/* Diagnostics: per-wave timeline of the last bounce launch of each bounce
 * index % 4: out[((b % 4) * 8192 + wave) * 16 + k], k = {first iteration,
 * exit, iterations | exit reason << 32 (1 input exhausted, 2 output segment
 * full), last grab, end of the last grab's work, summed grab latency, max
 * grab latency, last grab's latency, phase cycles 0..4} in 100 MHz real-time ticks; n = number
 * of uint64 to copy (at most 4 * 8192 * 16).  Zeros outside the stamp library. */
int mrt_debug_wave_times(uint64_t* out, size_t n);
/* Diagnostics (ABI 7): lane-occupancy counters of the separately built
 * lane-statistics library (make variant VNAME=lanes VFLAGS=-DMRT_LANESTATS=1):
 * out[k] for k < n (at most 64), summed over every wave of every launch since
 * the last reset — per traversal loop the wave iterations and the active
 * lanes in them (tools/lane_stats.py names the slots).  Zeros otherwise. */
int mrt_debug_lanes(uint64_t* out, size_t n, int reset);
/* Test entry (ABI 7): rank 0's unpack of an N-rank gather without a
 * communicator.  `gathered` (host) holds nranks slabs of
 * mrt_tiles_packed_floats(W, H, 0, nranks) floats, rank k's at slab k, as the
 * gather of MRT_EXCHANGE_GATHER delivers them; the renderer (shard_rank 0,
 * shard_count nranks) unpacks slabs 1..N-1 into its image with the RCCL
 * path's own unpack.  Synchronises the renderer. */
int mrt_debug_exchange_unpack(mrt_renderer* r, uint32_t nranks, const float* gathered, size_t floats);
/* Test entry (ABI 9, host only, no device): the traversal culling slack each
 * ray's nearest hit needs in the scene's main tree.  For ray record i
 * (origin, minDistance, direction, maxDistance at `stride` bytes) and its
 * brute-force nearest hit intersections[i] (reference layout, distance < 0 =
 * miss): out[4i + 0..1] = the largest (t_entry - t_hit) / t_hit over the child
 * boxes on the path from the root to the hit primitive's leaf, with the slab
 * test in the precise build's arithmetic ((p - o) * inv) and the fast build's
 * (fma(p, inv, -o * inv)); out[4i + 2..3] = the same for the near ties — the
 * triangles sharing a vertex position with the hit whose triangle test passes
 * within first-order rounding bounds (4u per operation chain), each at the
 * smallest t those bounds allow, within 2^-10 of t_hit (what a differently
 * rounding triangle test may report instead).  +inf if the ray
 * misses one of those boxes altogether, -inf for none.  The kernels cull a
 * child only when its entry lies beyond h.t * (1 + 2^-11) (kernels.hip
 * kCullScale): every value below 2^-11 is a hit no visiting order can lose
 * (DESIGN.md §3.1). */
int mrt_debug_box_margin(const mrt_scene* scene, const void* rays, uint32_t stride, uint32_t count,
                         const void* intersections, float* out);
/* Test entry (ABI 9, host only): q[i] = n[i] / d through the kernels' exact
 * division by a launch divisor (kernels.h magic_div: the multiplier the
 * renderer passes, applied as the kernels' mulhi + shift), n[i] < 2^31. */
int mrt_debug_magic_div(uint32_t d, const uint32_t* n, uint32_t count, uint32_t* q);
/* Number of HIP devices visible (0 when none; never fails). */
int mrt_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* MRT_H_ */
