// renderer.cpp — host orchestration + the C ABI of include/mrt.h.
//
// mrt_renderer_draw_n mirrors performRaytracing: (renderer/Renderer.mm:500-585)
// frame by frame, restructured for MI355X as a wavefront of fused bounce
// launches (kernels.hip::bounce_kernel):
//   reference per frame: rayGenerator, L x {MPS intersect, intersectionHandler,
//                        MPS intersect (shadow), lightSamplingHandler},
//                        accumulateImage                       = 2 + 4L passes
//   here per frame:      L bounce launches over a compacted SoA ray queue
//                        (raygen fused into bounce 0, shadow resolve and
//                        accumulation fused into the bounce where the path
//                        ends)                                 = L launches
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mrt.h"
#include "bvh.h"
#include "bvh_gpu.h"
#include "image.h"
#include "kernels.h"
#include "noise.h"
#include "noise_schedule.h"
#include "occluders.h"
#include "primary.h"
#include "scene.h"
#include "diag_env.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return fail(MRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                \
  } while (0)

inline float bitsf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  ~DevBuf() { if (p) (void)hipFree(p); }
  hipError_t alloc(size_t n) {
    if (p) { (void)hipFree(p); p = nullptr; }
    bytes = n;
    return n ? hipMalloc(&p, n) : hipSuccess;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// traversal-stack spill of the stage intersect kernel (trees deeper than its
// kMaxStack-entry LDS stack): (need - 32) entries x its persistent grid
hipError_t alloc_isect_spill(DevBuf& b, uint32_t max_stack) {
  if (max_stack <= (uint32_t)mrt::kMaxStack) return b.alloc(0);
  return b.alloc((size_t)(max_stack - 32) * mrt::kIntersectSpillGrid * 256 * 4);
}

#define NCCL_TRY(expr)                                                                            \
  do {                                                                                            \
    ncclResult_t e_ = (expr);                                                                     \
    if (e_ != ncclSuccess)                                                                        \
      return fail(MRT_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(e_));               \
  } while (0)

hipError_t upload(DevBuf& b, const void* src, size_t n) {
  hipError_t e = b.alloc(std::max<size_t>(n, 16));
  if (e != hipSuccess) return e;
  return n ? hipMemcpy(b.p, src, n, hipMemcpyHostToDevice) : hipSuccess;
}

}  // namespace

// MPS-shaped acceleration structure over caller-owned device buffers
struct mrt_accel {
  mrt_accel_desc desc{};
  DevBuf nodes, tris;
  DevBuf isect_spill;       // stage intersect stack spill for trees deeper than kMaxStack
  mrt::DeviceScene dev{};
  mrt_accel_info info{};
};

struct mrt_scene {
  int device = 0;
  DevBuf isect_spill;       // stage intersect stack spill for trees deeper than kMaxStack
  mrt::HostScene host;
  mrt::BvhResult bvh;
  // the shadow-ray occluder tree (occluders.h) as uploaded after the main
  // tree: node refs rebased by bvh.num_nodes, leaf records by the triangle
  // count, leaf primitive ids = scene primitives (host copy for check_bvh)
  std::vector<float> occ_nodes, occ_tris;
  std::vector<uint32_t> occ_keep;   // primitives the occluder tree holds
  int32_t occ_root = 0;
  uint32_t occ_node_base = 0, occ_max_stack = 0;
  DevBuf nodes, tris, prims, materials, lights;
  mrt::DeviceScene dev{};
  mrt_scene_info info{};
};

// bookkeeping of one draw_n call whose statistics are not read back yet
struct DrawRecord {
  DevBuf counters;                          // per (batch, bounce) survivor totals, then the launches' grab
                                            // counters (one buffer: one memset per draw)
  hipEvent_t start = nullptr, stop = nullptr;
  hipEvent_t cleared = nullptr;             // the counters' memset (other render streams of the draw wait on it)
  hipEvent_t copied = nullptr;              // the counters' copy to `host` (read-back stream) is done
  void* host = nullptr;                     // pinned (device-mapped) copy of `counters`, written behind the draw
  void* host_dev = nullptr;                 // its device address
  size_t host_bytes = 0;
  std::vector<hipEvent_t> kernel_events;    // MRT_FLAG_PROFILE: 2 per timed bounce launch
  uint32_t frames = 0;
  uint32_t launches = 0;                    // batches (bounce launches = batches * L)
  size_t span_off = 0;                      // byte offset of the batches' [2] u64 spans in `counters`
  size_t counter_bytes = 0;                 // bytes of `counters` this draw uses
  size_t events = 0;
  bool pending = false;
  // the counters are all zero once this entry's last draw enqueued its
  // folding accumulate (which zeroes them behind the draw); a draw that
  // returned early after its first launch leaves them dirty
  bool clean = false;
};
constexpr int kDrawRing = 3;

// One in-flight frame: its queues, segment counts, per-pixel path radiance and
// the stream its render launches run on.  Batches b and b+1 run on different
// slots concurrently (the reference keeps up to 3 frames in flight,
// renderer/Renderer.mm:16,593-600); their accumulations run in order on the
// main stream because the running mean is order-dependent.
struct FrameSlot {
  hipStream_t stream = nullptr;
  bool own_stream = false;
  DevBuf queue[2][mrt::kQueuePlanes];   // ray queues (the streaming wavefront: queue[0] holds the per-wave queues)
  DevBuf segments;          // 2 queues x 2 classes x grid per-block survivor counts + 2 chunk words
  DevBuf radiance;          // W*H float4, written once per owned pixel per frame
  DevBuf spill;             // traversal stack entries beyond the LDS capacity (deep BVHs)
  hipEvent_t acc_done = nullptr;      // on the main stream: the accumulate that last read `radiance`
  hipEvent_t kernel_done = nullptr;   // on `stream`: its last render launch
  bool acc_recorded = false;
};

// Failure state of one RCCL communicator, shared by the communicator and the
// renderers that enqueued collectives on it (a renderer may outlive it: a
// deferred unpack after mrt_comm_destroy).  A collective that reports an
// asynchronous error (ncclCommGetAsyncError) or does not complete within the
// timeout aborts the communicator (ncclCommAbort: its pending kernels exit);
// every later use of it fails with MRT_ERR_COMM.  The reference has no
// collective (one Metal device, renderer/Renderer.mm:595) and ignores its
// command-buffer errors (:131,141,145); this is the exchange's own contract.
struct CommHealth {
  std::mutex m;
  ncclComm_t comm = nullptr;   // null once destroyed or aborted
  bool aborted = false;
  std::string error;           // why it was aborted
  double timeout_ms = 120000.0;
  uint32_t inject = 0;         // test entry mrt_debug_comm_fail: 1 async error, 2 collectives never complete
};

// RCCL communicator of one rank (one process per GPU) and the stream its
// overlapped collectives run on
struct mrt_comm {
  ncclComm_t comm = nullptr;
  uint32_t nranks = 0, rank = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  std::shared_ptr<CommHealth> health = std::make_shared<CommHealth>();
};

// Image exchange state of a renderer (mrt_renderer_exchange): the packed
// owned tiles, double-buffered so an overlapped gather of step k can still be
// reading buffer k % 2 while step k + 1 packs into the other, and on rank 0
// the gathered slabs of every rank.
struct Exchange {
  DevBuf packed[2], gathered, staging;
  hipEvent_t pack_done[2] = {nullptr, nullptr}, gather_done[2] = {nullptr, nullptr};
  bool gather_recorded[2] = {false, false};
  uint64_t slab_floats = 0;   // packed floats per rank (rank 0 owns the most tiles)
  int pending = -1;           // buffer whose gather awaits rank 0's unpack (overlap mode)
  uint32_t next = 0;
  const mrt_comm* comm = nullptr;
  // the communicator's shape, copied at each exchange: a deferred unpack
  // never dereferences `comm` (it may be destroyed before the flush)
  uint32_t rank = 0, nranks = 1;
  uint32_t width = 0, height = 0;   // image size the pending gather was packed at
  // the last collective enqueued (on whichever stream it ran) and the health
  // of its communicator: mrt_renderer_sync / _exchange_flush wait for it with
  // a bound instead of blocking on a stream a stuck peer never releases
  hipEvent_t coll_done = nullptr;
  bool coll_pending = false;
  std::shared_ptr<CommHealth> health;
};

struct mrt_renderer {
  const mrt_scene* scene = nullptr;
  mrt_renderer_desc desc{};
  hipStream_t stream = nullptr;   // main stream (external or own); slot 0 runs on it
  bool own_stream = false;
  float* image = nullptr;
  bool own_image = false;
  uint32_t tiles_x = 0, tiles_y = 0, owned_tiles = 0;
  uint64_t owned_pixels = 0;
  std::vector<FrameSlot> slots;
  uint32_t max_frames = 0;   // MAX_FRAMES (0 = unlimited)
  // Frame batches in flight (MRT_INFLIGHT; default 1 for a whole frame, 2 for a
  // tile share).  With k >= 2 every slot renders on its own stream and the
  // accumulates run on the main stream, so batch b + 1 (of this draw or the
  // next) only waits for the accumulate that last read its slot's radiance:
  // its persistent blocks take the CUs as batch b's drain (~0.2 ms per
  // launch, whatever its length) frees them.  One GPU's 1/8 tile share of C2
  // launches 2.1-ms kernels, where that drain is 10 %.
  uint32_t inflight = 1;
  uint32_t slot_next = 0;   // slot of the next batch (rotates across draws)
  double wall_khz = 0.0;    // device wall clock (span timestamps; 0 = spans off, MRT_SPANS=0)
  bool image_foreign = false;   // the image holds pixels this renderer did not render (exchange / tiles_write)
  uint32_t grid = 0;        // persistent grid of the bounce kernel
  // noise tables in device chunks of 64 frames, generated ahead on a worker
  // thread and uploaded on their own stream (noise_schedule.h)
  std::unique_ptr<mrt::NoiseSchedule> noise;
  mrt::NoiseSchedule::Counters noise_base;   // the schedule's counters at the last stats reset
  uint64_t draw_seq = 0;     // draws enqueued (pins the noise chunks a draw reads)
  uint64_t frame_index = 0;
  // Draws in flight: each draw records its survivor counters and events in
  // its own ring entry, and its statistics are read back lazily (when the
  // entry is reused, or on stats / sync / read), so consecutive draws queue
  // back to back without a host round trip between them.
  DrawRecord draws[kDrawRing];
  uint32_t draw_next = 0;   // ring entry of the next draw (= the oldest pending one)
  uint32_t profile_every = 8;   // time the launches of every n-th batch (MRT_PROFILE_EVERY)
  uint32_t batch = 1;           // frames per bounce launch (frame batching)
  bool counter_fold = true;     // draw statistics copied + cleared by the last accumulate (MRT_COUNTER_FOLD)
  mrt_stats stats{};
  uint32_t stack_entries = 32;
  bool stream_allowed = false;  // streaming wavefront possible for this scene / configuration
  bool stream_mode = false; // wavefront as one launch per frame batch with per-wave queues (stream_kernel)
  bool path_mode = true;   // one path-megakernel launch per frame batch (else L bounce launches, MRT_KERNEL=wave)
  uint32_t debug = 0;   // MRT_DEBUG ablation bits (profiling only)
  // camera-ray candidate lists per 8x8 pixel block (primary.h), rebuilt for
  // every frame size; bounce 0 of the wavefront kernels (a wave = one block)
  // tests the block's list instead of traversing: C2 +4.6 % (alternating
  // A/B).  The path kernel refills lanes one by one, so its lists would be
  // per-lane dependent global loads at refill: C3 -4.8 %, not used there.
  // MRT_PRIMARY=0: off; MRT_PRIMARY_CAP: longest list (12)
  bool primary_allowed = true;
  uint32_t primary_cap = 12;
  DevBuf primary;
  uint32_t primary_bx = 0;
  Exchange x;
  DevBuf reference, display;   // comparison image (mrt_renderer_load_reference) and blit output
  struct DisplaySlot {          // mrt_renderer_display_enqueue / _map: pinned copies of the blit
    float* host = nullptr;
    size_t floats = 0;
    hipEvent_t done = nullptr;
    bool queued = false;
  } shown[MRT_DISPLAY_SLOTS];
};

namespace {

int finalize_draw(mrt_renderer* r, DrawRecord& d) {
  if (!d.pending) return MRT_OK;
  HIP_TRY(hipEventSynchronize(d.stop));
  float ms = 0.0f;
  HIP_TRY(hipEventElapsedTime(&ms, d.start, d.stop));
  const uint32_t L = r->desc.max_path_length;
  // the whole counter buffer (survivor counts, grab counters, spans) was
  // copied to pinned memory on the main stream behind the draw: no
  // synchronous copy, so the host never waits for work queued after it
  HIP_TRY(hipEventSynchronize(d.copied));
  const uint32_t* cnt = static_cast<const uint32_t*>(d.host);
  uint64_t active = r->owned_pixels * d.frames;   // bounce 0: every owned pixel's camera ray
  for (uint32_t k = 0; k < d.launches; ++k)
    for (uint32_t b = 0; b + 1 < L; ++b) active += cnt[(size_t)k * L + b];
  r->stats.active_ray_bounces += active;
  r->stats.last_draw_ms = ms;
  const uint64_t paths = r->owned_pixels * d.frames;
  r->stats.mpaths_per_s = ms > 0.0f ? (double)paths / (ms * 1e-3) / 1e6 : 0.0;
  r->stats.kernel_launches += (uint64_t)d.launches * (r->path_mode || r->stream_mode ? 1u : L);
  {
    std::vector<unsigned long long> sp((size_t)2 * d.launches);
    std::memcpy(sp.data(), static_cast<const char*>(d.host) + d.span_off, sp.size() * 8);
    for (uint32_t k = 0; k < d.launches; ++k) {
      const unsigned long long t0 = ~sp[2 * k], t1 = sp[2 * k + 1];
      if (sp[2 * k] && t1 >= t0 && r->wall_khz > 0.0) {
        r->stats.span_ms += (double)(t1 - t0) / r->wall_khz;
        r->stats.spans += 1;
      }
    }
  }
  if (r->desc.flags & MRT_FLAG_PROFILE) {
    for (size_t k = 0; k + 1 < d.events; k += 2) {
      float ms_k = 0.0f;
      HIP_TRY(hipEventElapsedTime(&ms_k, d.kernel_events[k], d.kernel_events[k + 1]));
      r->stats.kernel_ms += ms_k;
      r->stats.timed_launches += 1;
    }
  }
  d.pending = false;
  return MRT_OK;
}

// read back every pending draw, oldest first
int finalize_pending(mrt_renderer* r) {
  for (int i = 0; i < kDrawRing; ++i) {
    const int rc = finalize_draw(r, r->draws[(r->draw_next + i) % kDrawRing]);
    if (rc) return rc;
  }
  return MRT_OK;
}

// the noise chunks of frames [f0, f0 + n): generated (host threads, unless
// the worker already has) and uploaded asynchronously; never waits for the GPU
int acquire_noise(mrt_renderer* r, int64_t f0, uint32_t n, std::vector<mrt::NoiseSchedule::Chunk*>* out) {
  using NS = mrt::NoiseSchedule;
  const int64_t k0 = NS::chunk_of(f0), k1 = NS::chunk_of(f0 + (int64_t)n - 1);
  HIP_TRY(r->noise->poll(k0, k1));   // (never evicts a chunk this draw reads)
  const uint64_t waits = r->noise->counters().waits;
  for (int64_t k = k0; k <= k1; ++k) {
    NS::Chunk* c = nullptr;
    HIP_TRY(r->noise->acquire(k, r->draw_seq, &c));
    if (out) out->push_back(c);
  }
  if (r->noise->counters().waits != waits) r->stats.noise_waits += 1;
  // the next chunk's tables are generated while these frames render
  r->noise->prefetch(k1 + 1);
  return MRT_OK;
}

int alloc_frame_buffers(mrt_renderer* r) {
  const uint32_t W = r->desc.width, H = r->desc.height;
  const uint32_t S = std::max<uint32_t>(1, r->desc.shard_count);
  r->tiles_x = (W + mrt::kTile - 1) / mrt::kTile;
  r->tiles_y = (H + mrt::kTile - 1) / mrt::kTile;
  const uint32_t T = r->tiles_x * r->tiles_y;
  r->owned_tiles = r->desc.shard_rank < T ? (T - r->desc.shard_rank + S - 1) / S : 0;
  r->owned_pixels = 0;
  for (uint32_t t = r->desc.shard_rank; t < T; t += S) {
    const uint32_t tx = t % r->tiles_x, ty = t / r->tiles_x;
    const uint64_t w = std::min<uint32_t>(mrt::kTile, W - tx * mrt::kTile);
    const uint64_t h = std::min<uint32_t>(mrt::kTile, H - ty * mrt::kTile);
    r->owned_pixels += w * h;
  }
  // frames per launch: about 2^27 rays per launch (64 frames at 1080p, up
  // to kMaxBatch), so the launch-boundary drain (the last grabs finishing at
  // falling occupancy, ~20-40 us) is a small share of each launch: C2 at
  // 2^24 rays per launch (8 frames) 5210, 2^25 5431, 2^26 5551, 2^27 5617
  // Mpaths/s.  Memory: 64 B per queued ray x 2 queues + 16 B radiance
  // (~19.5 GB at 2^27 rays, of 288 GB).
  const size_t owned_slots = std::max<size_t>(1, (size_t)r->owned_tiles * 4096);
  r->batch = (uint32_t)std::min<size_t>(mrt::kMaxBatch, std::max<size_t>(1, ((size_t)1 << 27) / owned_slots));
  if (const char* v = mrt::diag_env("MRT_BATCH"))
    r->batch = std::max<uint32_t>(1, std::min<uint32_t>(mrt::kMaxBatch, (uint32_t)std::strtoul(v, nullptr, 0)));
  // a ray's tag holds batch * owned slots in 31 bits
  while (r->batch > 1 && owned_slots * r->batch >= ((size_t)1 << 31)) --r->batch;
  if (owned_slots >= ((size_t)1 << 31)) return fail(MRT_ERR_INVALID, "frame too large");
  // queue capacity: every owned slot of the batch + per-block rounding and
  // slack of the segments (kernels.h)
  const size_t slots = owned_slots * r->batch + (size_t)r->grid * (256 + mrt::kSegSlack);
  r->stream_mode = r->stream_allowed;
  for (FrameSlot& fs : r->slots) {
    HIP_TRY(fs.segments.alloc(((size_t)4 * r->grid + 2) * 4));   // 2 queues x 2 classes x grid + 2 chunk words
    HIP_TRY(hipMemsetAsync(fs.segments.p, 0, fs.segments.bytes, r->stream));
    // the path kernel keeps the path state in LDS: no ray queues; the
    // streaming wavefront needs only its per-wave queues
    const size_t qslots = r->stream_mode ? mrt::stream_slots(r->desc.max_path_length, r->grid) : slots;
    for (int q = 0; q < 2; ++q)
      for (int p = 0; p < mrt::kQueuePlanes; ++p)
        HIP_TRY(fs.queue[q][p].alloc(r->path_mode || (r->stream_mode && q == 1) ? 0 : qslots * 16));
    HIP_TRY(fs.radiance.alloc(owned_slots * r->batch * 16));
    const uint32_t need = r->scene->dev.max_stack;
    // spill rows of max_stack words per lane (kernels.hip LdsCtx::spill_lane)
    if (need > r->stack_entries && !fs.spill.p) HIP_TRY(fs.spill.alloc((size_t)need * r->grid * 256 * 4));
  }
  if (r->own_image) {
    if (r->image) (void)hipFree(r->image);
    r->image = nullptr;
    HIP_TRY(hipMalloc(&r->image, (size_t)W * H * 16));
  }
  HIP_TRY(hipMemsetAsync(r->image, 0, (size_t)W * H * 16, r->stream));
  r->image_foreign = false;
  r->frame_index = 0;
  r->stats = mrt_stats{};
  r->noise_base = r->noise->counters();
  r->stats.owned_pixels = r->owned_pixels;
  r->stats.kernel = r->path_mode ? 1u : (r->stream_mode ? 2u : 0u);
  r->stats.inflight = r->inflight;
  {
    mrt::PrimaryLists pl;
    const mrt::BvhResult& b = r->scene->bvh;
    HIP_TRY(r->primary.alloc(0));
    r->primary_bx = 0;
    if (r->primary_allowed && !r->path_mode &&
        mrt::build_primary_lists(b.tris.data(), (uint32_t)(b.tris.size() / 12), W, H, r->primary_cap, pl)) {
      HIP_TRY(upload(r->primary, pl.words.data(), pl.words.size() * 4));
      r->primary_bx = pl.blocks_x;
      r->stats.primary_blocks = pl.listed_blocks;
      r->stats.primary_mean = (float)pl.mean_count;
    }
  }
  // the render streams do not wait on the main stream: its memsets above
  // (segments, image) complete before any batch is queued
  HIP_TRY(hipStreamSynchronize(r->stream));
  return MRT_OK;
}

inline hipError_t launch_bounce(const mrt_renderer* r, const mrt::BounceArgs& a, hipStream_t s) {
  if (r->desc.flags & MRT_FLAG_PRECISE) return mrt::precise::launch_bounce(r->scene->dev, a, r->stack_entries, r->grid, s);
  return mrt::fast::launch_bounce(r->scene->dev, a, r->stack_entries, r->grid, s);
}

inline hipError_t launch_stream(const mrt_renderer* r, const mrt::BounceArgs& a, hipStream_t s) {
  if (r->desc.flags & MRT_FLAG_PRECISE) return mrt::precise::launch_stream(r->scene->dev, a, r->stack_entries, r->grid, s);
  return mrt::fast::launch_stream(r->scene->dev, a, r->stack_entries, r->grid, s);
}

inline hipError_t launch_paths(const mrt_renderer* r, const mrt::BounceArgs& a, hipStream_t s) {
  if (r->desc.flags & MRT_FLAG_PRECISE) return mrt::precise::launch_paths(r->scene->dev, a, r->stack_entries, r->grid, s);
  return mrt::fast::launch_paths(r->scene->dev, a, r->stack_entries, r->grid, s);
}

inline hipError_t launch_accumulate_frame(const mrt_renderer* r, const mrt::AccumArgs& a, hipStream_t s) {
  if (r->desc.flags & MRT_FLAG_PRECISE) return mrt::precise::launch_accumulate_frame(a, s);
  return mrt::fast::launch_accumulate_frame(a, s);
}

bool precise(uint32_t flags) { return (flags & MRT_FLAG_PRECISE) != 0; }

int write_pfm(const char* path, const std::vector<float>& rgba, uint32_t W, uint32_t H) {
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(MRT_ERR_IO, std::string("cannot write ") + path);
  std::fprintf(f, "PF\n%u %u\n-1.0\n", W, H);
  std::vector<float> row(3 * (size_t)W);
  for (uint32_t y = 0; y < H; ++y) {   // PFM scanlines are bottom-to-top == our row order
    for (uint32_t x = 0; x < W; ++x)
      for (int c = 0; c < 3; ++c) row[3 * x + c] = rgba[4 * ((size_t)y * W + x) + c];
    std::fwrite(row.data(), 4, row.size(), f);
  }
  std::fclose(f);
  return MRT_OK;
}

// Uncompressed scanline OpenEXR, FLOAT A,B,G,R channels, top-down.
int write_exr(const char* path, const std::vector<float>& rgba, uint32_t W, uint32_t H) {
  std::vector<uint8_t> out;
  auto put = [&](const void* p, size_t n) { const uint8_t* b = (const uint8_t*)p; out.insert(out.end(), b, b + n); };
  auto put_i32 = [&](int32_t v) { put(&v, 4); };
  auto put_str = [&](const char* s) { put(s, std::strlen(s) + 1); };
  auto attr = [&](const char* name, const char* type, const std::vector<uint8_t>& v) {
    put_str(name); put_str(type); put_i32((int32_t)v.size()); put(v.data(), v.size());
  };
  const uint32_t magic = 20000630u, version = 2u;
  put(&magic, 4); put(&version, 4);
  std::vector<uint8_t> ch;
  for (const char* c : {"A", "B", "G", "R"}) {
    ch.insert(ch.end(), c, c + 2);
    const int32_t pt = 2;  // FLOAT
    const uint8_t plin[4] = {0, 0, 0, 0};
    const int32_t xs = 1, ys = 1;
    ch.insert(ch.end(), (const uint8_t*)&pt, (const uint8_t*)&pt + 4);
    ch.insert(ch.end(), plin, plin + 4);
    ch.insert(ch.end(), (const uint8_t*)&xs, (const uint8_t*)&xs + 4);
    ch.insert(ch.end(), (const uint8_t*)&ys, (const uint8_t*)&ys + 4);
  }
  ch.push_back(0);
  attr("channels", "chlist", ch);
  attr("compression", "compression", {0});
  const int32_t box[4] = {0, 0, (int32_t)W - 1, (int32_t)H - 1};
  std::vector<uint8_t> bx((const uint8_t*)box, (const uint8_t*)box + 16);
  attr("dataWindow", "box2i", bx);
  attr("displayWindow", "box2i", bx);
  attr("lineOrder", "lineOrder", {0});
  const float par = 1.0f, ssw = 1.0f, swc[2] = {0.0f, 0.0f};
  attr("pixelAspectRatio", "float", std::vector<uint8_t>((const uint8_t*)&par, (const uint8_t*)&par + 4));
  attr("screenWindowCenter", "v2f", std::vector<uint8_t>((const uint8_t*)swc, (const uint8_t*)swc + 8));
  attr("screenWindowWidth", "float", std::vector<uint8_t>((const uint8_t*)&ssw, (const uint8_t*)&ssw + 4));
  out.push_back(0);
  const size_t line_bytes = (size_t)W * 4 * 4;
  uint64_t off = out.size() + 8ull * H;
  for (uint32_t y = 0; y < H; ++y) { put(&off, 8); off += 8 + line_bytes; }
  std::vector<float> line(4 * (size_t)W);
  for (uint32_t y = 0; y < H; ++y) {
    const uint32_t src = H - 1 - y;   // EXR is top-down; our row 0 is the bottom
    for (int c = 0; c < 4; ++c) {      // A, B, G, R
      const int comp = 3 - c;
      for (uint32_t x = 0; x < W; ++x) line[(size_t)c * W + x] = rgba[4 * ((size_t)src * W + x) + comp];
    }
    put_i32((int32_t)y);
    put_i32((int32_t)line_bytes);
    put(line.data(), line_bytes);
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) return fail(MRT_ERR_IO, std::string("cannot write ") + path);
  std::fwrite(out.data(), 1, out.size(), f);
  std::fclose(f);
  return MRT_OK;
}

}  // namespace

namespace {

int exchange_buffers(mrt_renderer* r, const mrt_comm* c) {
  Exchange& x = r->x;
  uint64_t floats = 0;
  if (mrt_tiles_packed_floats(r->desc.width, r->desc.height, 0, c->nranks, &floats)) return MRT_ERR_INVALID;
  if (x.slab_floats == floats && x.packed[0].p) return MRT_OK;
  HIP_TRY(hipStreamSynchronize(r->stream));
  x.slab_floats = floats;
  for (int i = 0; i < 2; ++i) {
    HIP_TRY(x.packed[i].alloc(floats * 4));
    HIP_TRY(hipMemsetAsync(x.packed[i].p, 0, floats * 4, r->stream));   // ranks with fewer tiles send zero padding
    if (!x.pack_done[i]) HIP_TRY(hipEventCreateWithFlags(&x.pack_done[i], hipEventDisableTiming));
    if (!x.gather_done[i]) HIP_TRY(hipEventCreateWithFlags(&x.gather_done[i], hipEventDisableTiming));
    x.gather_recorded[i] = false;
  }
  if (c->rank == 0) HIP_TRY(x.gathered.alloc(floats * 4 * c->nranks));
  return MRT_OK;
}

// rank 0: unpack every other rank's slab of gather buffer `i` into the image
// (on the renderer's stream, after the gather); other ranks: order the
// renderer's stream after the gather so sync/read see it complete
int exchange_unpack(mrt_renderer* r, int i) {
  Exchange& x = r->x;
  HIP_TRY(hipStreamWaitEvent(r->stream, x.gather_done[i], 0));
  if (x.rank == 0)
    for (uint32_t k = 1; k < x.nranks; ++k)
      HIP_TRY(mrt::fast::launch_tiles_move(x.gathered.as<float4>() + (size_t)k * (x.slab_floats / 4),
                                           reinterpret_cast<float4*>(r->image), x.width, x.height, k,
                                           x.nranks, false, r->stream));
  return MRT_OK;
}

// Forget a deferred (overlapped) gather without unpacking it — its tiles
// belong to an image that resize / reset discards.  The gather itself may
// still be writing the receive buffer: `wait` (resize, which may reallocate
// the exchange buffers) waits for it; reset need not (the next gather into
// the same buffer runs after it on the communicator's stream, and nothing
// else reads the buffer), so the overlap of the gather with the next draw
// is kept.
int exchange_wait(mrt_renderer* r);

int exchange_drop(mrt_renderer* r, bool wait) {
  Exchange& x = r->x;
  if (x.pending < 0) return MRT_OK;
  x.pending = -1;
  if (wait) return exchange_wait(r);   // (the pending gather is the last collective)
  return MRT_OK;
}

// Abort a communicator (lock held): its pending collectives are cancelled
// and every later use fails.  Returns the MRT_ERR_COMM status.
int comm_abort_locked(CommHealth& h, const std::string& why) {
  if (!h.aborted) {
    if (h.comm) (void)ncclCommAbort(h.comm);
    h.comm = nullptr;
    h.aborted = true;
    h.error = why;
  }
  return fail(MRT_ERR_COMM, "RCCL communicator aborted: " + h.error);
}

// Non-blocking health check of a communicator (lock held).
int comm_check_locked(CommHealth& h) {
  if (h.aborted) return fail(MRT_ERR_COMM, "RCCL communicator aborted: " + h.error);
  if (!h.comm) return MRT_OK;   // destroyed: nothing can fail any more
  ncclResult_t e = ncclSuccess;
  if (h.inject == 1) e = ncclSystemError;
  else if (ncclCommGetAsyncError(h.comm, &e) != ncclSuccess) e = ncclInternalError;
  if (e != ncclSuccess && e != ncclInProgress)
    return comm_abort_locked(h, std::string("asynchronous error: ") + ncclGetErrorString(e));
  return MRT_OK;
}

// The renderer's exchange state after its communicator failed: nothing is
// left to unpack or wait for (the image keeps the renderer's own tiles).
void exchange_forget(mrt_renderer* r) {
  r->x.pending = -1;
  r->x.coll_pending = false;
  r->x.comm = nullptr;
}

// Wait, with the communicator's timeout as the bound, for the renderer's last
// collective to complete on the device; poll its asynchronous error meanwhile.
int exchange_wait(mrt_renderer* r) {
  Exchange& x = r->x;
  if (!x.coll_pending) return MRT_OK;
  std::shared_ptr<CommHealth> h = x.health;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0;; ++spin) {
    double timeout_ms;
    {
      std::lock_guard<std::mutex> lk(h->m);
      if (h->inject != 2) {
        const hipError_t q = hipEventQuery(x.coll_done);
        if (q == hipSuccess) { x.coll_pending = false; return MRT_OK; }
        if (q != hipErrorNotReady) {
          exchange_forget(r);
          return fail(MRT_ERR_HIP, std::string("exchange: ") + hipGetErrorString(q));
        }
      }
      if (int rc = comm_check_locked(*h)) { exchange_forget(r); return rc; }
      timeout_ms = h->timeout_ms;
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (ms > timeout_ms) {
        const int rc = comm_abort_locked(*h, "collective did not complete within " + std::to_string((long)timeout_ms) +
                                                  " ms (a peer stopped or the link failed)");
        exchange_forget(r);
        return rc;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(spin < 100 ? 20 : 500));
  }
}

int exchange_flush(mrt_renderer* r) {
  if (r->x.coll_pending && r->x.health) {   // a failed communicator surfaces at the next exchange call
    std::lock_guard<std::mutex> lk(r->x.health->m);
    if (int rc = comm_check_locked(*r->x.health)) { exchange_forget(r); return rc; }
  }
  if (r->x.pending < 0) return MRT_OK;
  const int i = r->x.pending;
  r->x.pending = -1;
  return exchange_unpack(r, i);
}

}  // namespace

extern "C" {

const char* mrt_last_error(void) { return g_last_error.c_str(); }
int mrt_abi_version(void) { return MRT_ABI_VERSION; }

int mrt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int mrt_shard_mask(uint32_t W, uint32_t H, uint32_t rank, uint32_t count, uint8_t* mask, uint64_t* owned) {
  if (W == 0 || H == 0) return fail(MRT_ERR_INVALID, "empty image");
  const uint32_t S = count ? count : 1;
  if (rank >= S) return fail(MRT_ERR_INVALID, "shard_rank >= shard_count");
  const uint32_t tx_n = (W + mrt::kTile - 1) / mrt::kTile, ty_n = (H + mrt::kTile - 1) / mrt::kTile;
  uint64_t n = 0;
  for (uint32_t y = 0; y < H; ++y)
    for (uint32_t x = 0; x < W; ++x) {
      const uint32_t t = (y / mrt::kTile) * tx_n + x / mrt::kTile;
      const bool mine = (t % S) == rank;
      if (mask) mask[(size_t)y * W + x] = mine ? 1 : 0;
      n += mine;
    }
  (void)ty_n;
  if (owned) *owned = n;
  return MRT_OK;
}

int mrt_display(const float* image, const float* reference, float* out, uint32_t W, uint32_t H, uint32_t flags,
                float compare_scale, void* stream) {
  const uint32_t mode = (flags >> 8) & 0xFFu;
  if (!image || !out || W == 0 || H == 0 || mode > 4 || (mode && !reference) || (flags & ~0xFF03u))
    return fail(MRT_ERR_INVALID, "mrt_display: bad argument");
  HIP_TRY(mrt::fast::launch_display(reinterpret_cast<const float4*>(image), reinterpret_cast<const float4*>(reference),
                                    reinterpret_cast<float4*>(out), W * H, flags, compare_scale, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_tiles_packed_floats(uint32_t W, uint32_t H, uint32_t rank, uint32_t count, uint64_t* floats) {
  const uint32_t S = count ? count : 1;
  if (!floats || W == 0 || H == 0 || rank >= S) return fail(MRT_ERR_INVALID, "mrt_tiles_packed_floats: bad argument");
  const uint32_t T = ((W + mrt::kTile - 1) / mrt::kTile) * ((H + mrt::kTile - 1) / mrt::kTile);
  const uint64_t owned = rank < T ? (T - rank + S - 1) / S : 0;
  *floats = owned * mrt::kTile * mrt::kTile * 4;
  return MRT_OK;
}

int mrt_tiles_pack(const float* image, uint32_t W, uint32_t H, uint32_t rank, uint32_t count, float* packed,
                   void* stream) {
  const uint32_t S = count ? count : 1;
  if (!image || !packed || W == 0 || H == 0 || rank >= S) return fail(MRT_ERR_INVALID, "mrt_tiles_pack: bad argument");
  HIP_TRY(mrt::fast::launch_tiles_move(reinterpret_cast<const float4*>(image), reinterpret_cast<float4*>(packed), W, H,
                                       rank, S, true, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_tiles_unpack(const float* packed, uint32_t W, uint32_t H, uint32_t rank, uint32_t count, float* image,
                     void* stream) {
  const uint32_t S = count ? count : 1;
  if (!image || !packed || W == 0 || H == 0 || rank >= S) return fail(MRT_ERR_INVALID, "mrt_tiles_unpack: bad argument");
  HIP_TRY(mrt::fast::launch_tiles_move(reinterpret_cast<const float4*>(packed), reinterpret_cast<float4*>(image), W, H,
                                       rank, S, false, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_synchronize(void* stream) {
  if (stream) HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  else HIP_TRY(hipDeviceSynchronize());
  return MRT_OK;
}

int mrt_event_record(void* stream, void** event) {
  if (!event) return fail(MRT_ERR_INVALID, "null event");
  if (!*event) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *event = (void*)e;
  }
  HIP_TRY(hipEventRecord((hipEvent_t)*event, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_event_synchronize(void* event) {
  if (!event) return fail(MRT_ERR_INVALID, "null event");
  HIP_TRY(hipEventSynchronize((hipEvent_t)event));
  return MRT_OK;
}

int mrt_event_destroy(void* event) {
  if (event) HIP_TRY(hipEventDestroy((hipEvent_t)event));
  return MRT_OK;
}

int mrt_debug_stamps(uint64_t* out8, int reset) {
  if (!out8) return fail(MRT_ERR_INVALID, "null output");
  HIP_TRY(mrt::fast::read_stamps(reinterpret_cast<unsigned long long*>(out8), reset != 0));
  return MRT_OK;
}

int mrt_debug_wave_times(uint64_t* out, size_t n) {
  if (!out) return fail(MRT_ERR_INVALID, "null output");
  HIP_TRY(mrt::fast::read_wave_times(reinterpret_cast<unsigned long long*>(out), n));
  return MRT_OK;
}

int mrt_debug_lanes(uint64_t* out, size_t n, int reset) {
  if (!out) return fail(MRT_ERR_INVALID, "null output");
  HIP_TRY(mrt::fast::read_lane_stats(reinterpret_cast<unsigned long long*>(out), n, reset != 0));
  return MRT_OK;
}

int mrt_noise_table(uint64_t seed, int64_t frame, float* out) {
  if (!out) return fail(MRT_ERR_INVALID, "null output");
  mrt::make_noise_table(seed, frame, out);
  return MRT_OK;
}

// ---------------------------------------------------------------------------
// scene
// ---------------------------------------------------------------------------
int mrt_scene_create(const mrt_scene_desc* desc, mrt_scene** out) {
  if (!desc || !out || !desc->obj_path) return fail(MRT_ERR_INVALID, "mrt_scene_create: null argument");
  *out = nullptr;
  std::unique_ptr<mrt_scene> s(new mrt_scene());
  s->device = desc->device;
  std::string err;
  if (!mrt::import_obj(desc->obj_path, desc->mtl_override ? desc->mtl_override : "", s->host, err))
    return fail(MRT_ERR_IO, err);
  if (desc->procedural_triangles) mrt::append_procedural_mesh(s->host, desc->procedural_triangles, desc->procedural_seed);
  mrt::flatten(s->host);
  const mrt::HostScene& h = s->host;
  const uint32_t T = (uint32_t)h.references.size();

  mrt::BvhBuildOptions opt;
  if (desc->max_leaf_size) opt.max_leaf_size = desc->max_leaf_size;
  if (desc->lds_nodes == UINT32_MAX) opt.lds_node_budget = 0;
  else if (desc->lds_nodes) opt.lds_node_budget = desc->lds_nodes;
  else opt.lds_node_budget = 256;   // BFS prefix; the launcher stages what fits (fit_lds_nodes)
  if (const char* v = mrt::diag_env("MRT_LDS_NODES"); v && !desc->lds_nodes) opt.lds_node_budget = (uint32_t)std::strtoul(v, nullptr, 0);
  // large scenes (traversed from global memory): a finer SAH — 64 bins, and
  // the exact sweep for ranges below 64 K triangles: C4 1822 -> 1925-1935
  // Mpaths/s (+5.7 %, SAH cost 22.3 -> 20.5), C3 / C3g (7 K triangles) unchanged
  // (tools/env_sweep.sh, r2).  The presorted full sweep at every node
  // (MRT_FULL_SWEEP=1: SAH cost 19.0, the fastest build) measured C4 -1.1 %,
  // C5 share -1.0 %, C2 -2.5 % against it, so it is opt-in.
  if (T >= 65536) {
    opt.bins = 64;
    opt.exact_sah_below = 65536;
  }
  if (const char* v = mrt::diag_env("MRT_FULL_SWEEP")) opt.full_sweep = std::atoi(v) != 0;
  // tuning overrides (profiling): MRT_LEAF = max leaf size, MRT_CTRAV = SAH node cost
  if (const char* v = mrt::diag_env("MRT_LEAF")) opt.max_leaf_size = (uint32_t)std::strtoul(v, nullptr, 0);
  if (const char* v = mrt::diag_env("MRT_CTRAV")) opt.traversal_cost = std::strtof(v, nullptr);
  if (const char* v = mrt::diag_env("MRT_BINS")) opt.bins = (uint32_t)std::strtoul(v, nullptr, 0);
  if (const char* v = mrt::diag_env("MRT_EXACT_SAH")) opt.exact_sah_below = (uint32_t)std::strtoul(v, nullptr, 0);
  // BVH4 collapse: opt.collapse_dp's size policy (bvh.h), the same for every
  // build path — the area-optimal collapse below 64 K triangles: C2 +0.8 %,
  // C3 +1.9 %, C3g +0.5 %; the 1M-triangle C4 tree (21 % fewer, fuller
  // nodes: more children pushed per step) -1.2 %, so greedy there (r4)
  const uint32_t builder = desc->bvh_builder ? desc->bvh_builder : MRT_BVH_HOST_SAH;
  // BVH4 is the one layout the kernels traverse (BVH2 measured -24 %, a
  // compressed BVH8 -33 % and a quantised BVH4 -10 % on C4 in r2)
  opt.width = desc->bvh_width ? desc->bvh_width : 4;
  if (opt.width != 4) return fail(MRT_ERR_INVALID, "bvh_width must be 4 (or 0 = default)");
  if (builder != MRT_BVH_HOST_SAH && builder != MRT_BVH_DEVICE_LBVH && builder != MRT_BVH_DEVICE_PLOC)
    return fail(MRT_ERR_INVALID, "unknown bvh_builder");
  if (builder != MRT_BVH_HOST_SAH && desc->device < 0) return fail(MRT_ERR_INVALID, "device BVH build needs a device");
  double build_ms = 0.0;
  if (builder == MRT_BVH_HOST_SAH) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!mrt::build_bvh(h.vertices.data()->v, sizeof(mrt::RefVertex), h.indices.data(), T, opt, s->bvh, err))
      return fail(MRT_ERR_INVALID, "BVH build failed: " + err);
    build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  } else {
    // MPS-style: the vertex and index buffers go to the device first and the
    // structure is built there (MPSTriangleAccelerationStructure.rebuild)
    HIP_TRY(hipSetDevice(desc->device));
    DevBuf dv, di;
    HIP_TRY(upload(dv, h.vertices.data(), h.vertices.size() * sizeof(mrt::RefVertex)));
    HIP_TRY(upload(di, h.indices.data(), h.indices.size() * 4));
    mrt::GpuBvhResult g;
    if (mrt::build_bvh_gpu(dv.as<float>(), sizeof(mrt::RefVertex), di.as<uint32_t>(), T, opt.max_leaf_size,
                           builder == MRT_BVH_DEVICE_PLOC ? mrt::GpuBvhAlgo::kPloc : mrt::GpuBvhAlgo::kLbvh, nullptr, g,
                           err) != hipSuccess)
      return fail(MRT_ERR_HIP, "device BVH build failed: " + err);
    s->nodes.p = g.nodes; s->nodes.bytes = g.nodes_bytes;
    s->tris.p = g.tris; s->tris.bytes = g.tris_bytes;
    build_ms = g.build_ms;
    // host copy of the tree for mrt_scene_check_bvh / info
    mrt::BvhResult& b = s->bvh;
    b.nodes.resize(g.nodes_bytes / 4);
    b.tris.resize(g.tris_bytes / 4);
    HIP_TRY(hipMemcpy(b.nodes.data(), g.nodes, g.nodes_bytes, hipMemcpyDeviceToHost));
    if (g.tris_bytes) HIP_TRY(hipMemcpy(b.tris.data(), g.tris, g.tris_bytes, hipMemcpyDeviceToHost));
    b.root = g.root;
    b.num_nodes = g.num_nodes;
    b.num_leaves = g.num_leaves;
    b.max_depth = g.levels;
    b.wide_depth = g.levels;
    b.width = 4;
    b.max_stack = g.max_stack;
    b.lds_nodes = std::min<uint32_t>(opt.lds_node_budget, g.num_nodes);   // BFS order: any prefix is the top
    b.sah_cost = 0.0;
  }
  if (s->bvh.max_stack > (uint32_t)mrt::kMaxTraversalStack)
    return fail(MRT_ERR_INVALID, "BVH needs a deeper traversal stack (" + std::to_string(s->bvh.max_stack) + " entries, " +
                                     std::to_string(s->bvh.wide_depth) + " levels)");

  // per-primitive shading records (primitive order)
  std::vector<float> prims((size_t)T * 24);
  for (uint32_t t = 0; t < T; ++t) {
    const mrt::RefTriangleReference& r = h.references[t];
    float* o = &prims[(size_t)t * 24];
    for (int k = 0; k < 3; ++k) {
      const mrt::RefVertex& v = h.vertices[r.tri[k]];
      o[4 * k + 0] = v.v[0]; o[4 * k + 1] = v.v[1]; o[4 * k + 2] = v.v[2]; o[4 * k + 3] = 0.0f;
      o[12 + 4 * k + 0] = v.n[0]; o[12 + 4 * k + 1] = v.n[1]; o[12 + 4 * k + 2] = v.n[2]; o[12 + 4 * k + 3] = 0.0f;
    }
    o[3] = bitsf(r.materialIndex);
    o[7] = bitsf(r.lightTriangleIndex);
  }
  std::vector<float> mats(h.materials.size() * 8);
  for (size_t m = 0; m < h.materials.size(); ++m) {
    const mrt::RefMaterial& M = h.materials[m];
    float* o = &mats[m * 8];
    o[0] = M.diffuse[0]; o[1] = M.diffuse[1]; o[2] = M.diffuse[2]; o[3] = M.ior;
    o[4] = M.emissive[0]; o[5] = M.emissive[1]; o[6] = M.emissive[2]; o[7] = bitsf(M.materialType);
  }
  std::vector<float> lights(h.lights.size() * 28, 0.0f);
  for (size_t l = 0; l < h.lights.size(); ++l) {
    const mrt::RefLightTriangle& L = h.lights[l];
    float* o = &lights[l * 28];
    o[0] = L.emissive[0]; o[1] = L.emissive[1]; o[2] = L.emissive[2]; o[3] = L.area;
    const mrt::RefVertex* v[3] = {&L.v1, &L.v2, &L.v3};
    for (int k = 0; k < 3; ++k) {
      for (int c = 0; c < 3; ++c) { o[4 + 8 * k + c] = v[k]->v[c]; o[8 + 8 * k + c] = v[k]->n[c]; }
    }
    o[7] = L.pdf;
    o[11] = L.cdf;
    o[15] = bitsf(L.index);
  }
  // shadow-ray occluder tree (occluders.h): a second BVH4 over the triangles
  // outside the culled supporting planes, appended to the main tree's node
  // and leaf-triangle arrays (refs rebased); host-SAH scenes only
  std::vector<float> up_nodes = s->bvh.nodes, up_tris = s->bvh.tris;
  mrt::OccluderSet occ;
  mrt::BvhResult ob;
  bool occ_on = builder == MRT_BVH_HOST_SAH && !desc->no_occluder_tree;
  if (const char* v = mrt::diag_env("MRT_OCCLUDERS")) occ_on = occ_on && std::atoi(v) != 0;
  if (occ_on) {
    std::vector<float> lv, ln;
    for (uint32_t l = 0; l < h.light_count; ++l)
      for (const mrt::RefVertex* v : {&h.lights[l].v1, &h.lights[l].v2, &h.lights[l].v3}) {
        lv.insert(lv.end(), {v->v[0], v->v[1], v->v[2]});
        ln.insert(ln.end(), {v->n[0], v->n[1], v->n[2]});
      }
    occ_on = mrt::find_occluders(h.vertices.data()->v, sizeof(mrt::RefVertex), (uint32_t)h.vertices.size(),
                                 h.indices.data(), T, lv.data(), ln.data(), h.light_count, occ);
  }
  // with few light triangles the occluder tree leaves them out: every shadow
  // ray enters the light's own leaf box, and the kernels test the other
  // light triangles in one wave-uniform loop instead (kernels.hip
  // lights_occlude; MRT_OCC_LIGHTS=0 keeps them in the tree)
  bool occ_lights = occ_on && h.light_count <= mrt::kOccLightsMax;
  if (const char* v = mrt::diag_env("MRT_OCC_LIGHTS")) occ_lights = occ_lights && std::atoi(v) != 0;
  if (occ_lights) {
    std::vector<uint8_t> is_light(T, 0);
    for (uint32_t l = 0; l < h.light_count; ++l)
      if (h.lights[l].index < T) is_light[h.lights[l].index] = 1;
    occ.keep.erase(std::remove_if(occ.keep.begin(), occ.keep.end(), [&](uint32_t t) { return is_light[t] != 0; }),
                   occ.keep.end());
  }
  const uint32_t node_base = (uint32_t)(s->bvh.nodes.size() / 32), tri_base = T;
  int32_t occ_root = mrt::kEmptyChild;
  if (occ_on && !occ.keep.empty()) {
    std::vector<uint32_t> sub;
    sub.reserve(occ.keep.size() * 3);
    for (uint32_t t : occ.keep) sub.insert(sub.end(), {h.indices[3 * t], h.indices[3 * t + 1], h.indices[3 * t + 2]});
    mrt::BvhBuildOptions oo = opt;
    oo.lds_node_budget = 0;
    if (const char* v = mrt::diag_env("MRT_OCC_LEAF"))
      oo.max_leaf_size = std::max(1u, std::min<uint32_t>(mrt::kMaxLeafSize, (uint32_t)std::strtoul(v, nullptr, 0)));
    if (const char* v = mrt::diag_env("MRT_OCC_TCOST")) oo.traversal_cost = std::strtof(v, nullptr);
    if (!mrt::build_bvh(h.vertices.data()->v, sizeof(mrt::RefVertex), sub.data(), (uint32_t)occ.keep.size(), oo, ob, err))
      return fail(MRT_ERR_INVALID, "occluder BVH build failed: " + err);
    auto rebase = [&](int32_t r) -> int32_t {
      if (r == mrt::kEmptyChild) return r;
      if (r >= 0) return r + (int32_t)node_base;
      const uint32_t lr = ~(uint32_t)r;
      return mrt::leaf_ref((lr >> mrt::kLeafCountBits) + tri_base, (lr & (mrt::kMaxLeafSize - 1)) + 1);
    };
    for (uint32_t k = 0; k < ob.num_nodes; ++k)
      for (int c = 0; c < 4; ++c) {
        float& f = ob.nodes[32 * (size_t)k + 24 + c];
        f = bitsf((uint32_t)rebase((int32_t)fbits(f)));
      }
    for (size_t i = 0; i < occ.keep.size(); ++i) {   // leaf prim ids: subset position -> primitive
      float& f = ob.tris[12 * i + 3];
      f = bitsf(occ.keep[fbits(f)]);
    }
    occ_root = rebase(ob.root);
    // the renderer sizes its LDS stack by the deeper of the two trees
    // (dev.max_stack): an occluder tree deeper than the traversal stack
    // allows, or deeper than the main tree (it holds a subset of its
    // triangles, so it would only cost the main tree's stack variant), is
    // dropped and shadow rays traverse the main tree
    if (ob.max_stack > (uint32_t)mrt::kMaxTraversalStack || ob.max_stack > s->bvh.max_stack) {
      occ_on = false;
      occ_root = mrt::kEmptyChild;
    } else {
      if (ob.num_nodes) up_nodes.insert(up_nodes.end(), ob.nodes.begin(), ob.nodes.begin() + 32 * (size_t)ob.num_nodes);
      up_tris.insert(up_tris.end(), ob.tris.begin(), ob.tris.end());
      s->occ_nodes.assign(ob.nodes.begin(), ob.nodes.begin() + 32 * (size_t)ob.num_nodes);
      s->occ_tris = ob.tris;
      s->occ_keep = occ.keep;
      s->occ_root = occ_root;
      s->occ_node_base = node_base;
      s->occ_max_stack = ob.max_stack;
    }
  }
  // convex occluders (occluders.h): every triangle of the light-free
  // occluder tree on a convex solid; the solids' faces go to the kernels and
  // each solid triangle's face index into its shading record (p2.w)
  mrt::ConvexSet conv;
  bool conv_on = occ_on && occ_lights && occ_root != mrt::kEmptyChild;
  if (const char* v = mrt::diag_env("MRT_CONVEX")) conv_on = conv_on && std::atoi(v) != 0;
  if (conv_on)
    conv_on = mrt::find_convex_occluders(h.vertices.data()->v, sizeof(mrt::RefVertex), (uint32_t)h.vertices.size(),
                                         h.indices.data(), T, occ.keep, occ, conv);
  if (conv_on)
    for (uint32_t t = 0; t < T; ++t) {
      const uint32_t code = conv.prim_face[t];   // c * 8 + face + 1, 0: not on a solid
      prims[(size_t)t * 24 + 11] = bitsf(code);
      // the face's outward unit normal in n0.w, n1.w, n2.w (kernels.hip convex_occlusion's own-face test)
      if (code)
        for (int c = 0; c < 3; ++c) prims[(size_t)t * 24 + 15 + 4 * c] = conv.face_normal[(code - 1) / 8][3 * ((code - 1) % 8) + c];
    }
  mrt_scene_info& in = s->info;
  if (conv_on) {
    in.convex_solids = conv.count;
    in.convex_delta = conv.delta;
    for (uint32_t c = 0; c < conv.count; ++c) {
      for (int i = 0; i < 16; ++i) in.convex_obb[c][i] = conv.obb[c][i];
      for (int k = 0; k < 8; ++k) in.convex_face_tris[c][k] = conv.face_tris[c][k];
    }
  }
  if (occ_on) {
    in.occluder_planes = (uint32_t)occ.planes.size();
    in.occluder_culled = occ.culled;
    in.occluder_nodes = ob.num_nodes;
    in.occluder_margin = occ.margin;
    in.occluder_max_stack = ob.max_stack;
    in.occluder_cos_min = occ.cos_min;
    for (size_t k = 0; k < occ.planes.size() && k < 8; ++k)
      for (int c = 0; c < 4; ++c) in.occluder_plane[k][c] = occ.planes[k][c];
  }
  in.vertices = (uint32_t)h.vertices.size();
  in.triangles = T;
  in.materials = (uint32_t)h.materials.size();
  in.light_triangles = h.light_count;
  in.bvh_nodes = s->bvh.num_nodes;
  in.bvh_leaves = s->bvh.num_leaves;
  in.bvh_depth = s->bvh.max_depth;
  in.bvh_lds_nodes = s->bvh.lds_nodes;
  in.bvh_width = s->bvh.width;
  in.bvh_max_stack = s->bvh.max_stack;
  in.bvh_sah_cost = s->bvh.sah_cost;
  in.build_ms = build_ms;
  if (desc->device < 0) {   // host-only scene (CPU tests of import + BVH)
    *out = s.release();
    return MRT_OK;
  }
  // the kernels address nodes and leaf triangles with 32-bit buffer offsets
  // (kernels.hip buf_ld4): each array below 4 GiB (~33 M nodes, ~89 M
  // triangles; a scene beyond that needs the flat-address build)
  if ((uint64_t)up_nodes.size() * 4 >= (1ull << 32) || (uint64_t)up_tris.size() * 4 >= (1ull << 32) ||
      (uint64_t)s->bvh.nodes.size() * 4 >= (1ull << 32) || (uint64_t)T * 48 >= (1ull << 32))
    return fail(MRT_ERR_INVALID, "scene too large: BVH nodes or leaf triangles exceed 4 GiB");
  HIP_TRY(hipSetDevice(desc->device));
  if (builder == MRT_BVH_HOST_SAH) {
    HIP_TRY(upload(s->nodes, up_nodes.data(), up_nodes.size() * 4));
    HIP_TRY(upload(s->tris, up_tris.data(), up_tris.size() * 4));
  }
  HIP_TRY(upload(s->prims, prims.data(), prims.size() * 4));
  HIP_TRY(upload(s->materials, mats.data(), mats.size() * 4));
  HIP_TRY(upload(s->lights, lights.data(), lights.size() * 4));
  mrt::DeviceScene& d = s->dev;
  d.nodes = s->nodes.as<float>();
  d.tris = s->tris.as<float>();
  d.prims = s->prims.as<float>();
  d.materials = s->materials.as<float>();
  d.lights = s->lights.as<float>();
  d.root = s->bvh.root;
  d.num_nodes = s->bvh.num_nodes;
  d.num_triangles = T;
  d.num_materials = (uint32_t)h.materials.size();
  d.num_lights = h.light_count;
  d.lds_nodes = s->bvh.lds_nodes;
  d.width = s->bvh.width;
  d.max_stack = s->bvh.max_stack;
  d.origin_test = T >= mrt::kOriginTestTriangles ? 1u : 0u;   // (global-memory trees)
  if (const char* v = mrt::diag_env("MRT_ORIGIN_TEST")) d.origin_test = std::atoi(v) != 0;
  d.region_grabs = T >= mrt::kRegionGrabTriangles ? 1u : 0u;
  if (const char* v = mrt::diag_env("MRT_REGIONS")) d.region_grabs = std::atoi(v) != 0;
  d.light_shortcut = h.light_count <= mrt::kLightShortcutMax ? 1u : 0u;
  if (const char* v = mrt::diag_env("MRT_LAST_LIGHT")) d.light_shortcut = d.light_shortcut && std::atoi(v) != 0;
  d.occ_root = occ_root;
  d.occ_planes = 0;
  d.occ_lights = 0;
  if (occ_on) {
    d.occ_lights = occ_lights ? 1u : 0u;
    d.occ_nodes = (uint32_t)(up_nodes.size() / 32) - s->bvh.num_nodes;   // (a leaf-root main tree keeps one dummy node)
    d.occ_tris = (uint32_t)occ.keep.size();
    d.occ_planes = (uint32_t)occ.planes.size();
    d.occ_margin = occ.margin;
    d.occ_cos_min = occ.cos_min;
    d.occ_cos_min2 = occ.cos_min * occ.cos_min;
    for (uint32_t k = 0; k < d.occ_planes; ++k)
      for (int c = 0; c < 4; ++c) d.occ_plane[k][c] = occ.planes[k][c];
    d.max_stack = std::max(d.max_stack, ob.max_stack);
  }
  d.conv_count = in.convex_solids;
  std::memcpy(d.conv_obb, in.convex_obb, sizeof(d.conv_obb));
  std::memcpy(d.conv_face_tris, in.convex_face_tris, sizeof(d.conv_face_tris));
  HIP_TRY(alloc_isect_spill(s->isect_spill, d.max_stack));
  in.device_bytes = s->nodes.bytes + s->tris.bytes + s->prims.bytes + s->materials.bytes + s->lights.bytes;
  *out = s.release();
  return MRT_OK;
}

int mrt_scene_info_get(const mrt_scene* scene, mrt_scene_info* info) {
  if (!scene || !info) return fail(MRT_ERR_INVALID, "null argument");
  *info = scene->info;
  return MRT_OK;
}

int mrt_scene_export(const mrt_scene* scene, void* vertices, void* indices, void* materials, void* references,
                     void* lights) {
  if (!scene) return fail(MRT_ERR_INVALID, "null scene");
  const mrt::HostScene& h = scene->host;
  if (vertices) std::memcpy(vertices, h.vertices.data(), h.vertices.size() * sizeof(mrt::RefVertex));
  if (indices) std::memcpy(indices, h.indices.data(), h.indices.size() * 4);
  if (materials) std::memcpy(materials, h.materials.data(), h.materials.size() * sizeof(mrt::RefMaterial));
  if (references) std::memcpy(references, h.references.data(), h.references.size() * sizeof(mrt::RefTriangleReference));
  if (lights) std::memcpy(lights, h.lights.data(), h.lights.size() * sizeof(mrt::RefLightTriangle));
  return MRT_OK;
}

extern "C++" {
namespace {
// Structural check of one BVH4 over the scene's primitives: every primitive
// in `want` in exactly one leaf (and no other), every child box contains its
// subtree's triangles, leaf records match the vertices, the stack bound
// holds.  node(ref) / tri(k) map the tree's (possibly rebased) references to
// host records; nodes [node_lo, node_lo + num_nodes) must all be reachable.
template <class NodeFn, class TriFn>
int check_tree(const mrt::HostScene& h, int32_t root, uint32_t node_lo, uint32_t num_nodes, uint32_t tri_lo,
               uint32_t tri_count, uint32_t max_stack, const std::vector<uint8_t>& want, NodeFn node, TriFn tri,
               const char* what) {
  const uint32_t T = (uint32_t)h.references.size();
  std::vector<uint8_t> seen(T, 0);
  auto fbits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
  auto bad = [&](const char* m) { return fail(MRT_ERR_STATE, std::string(what) + ": " + m); };
  // pend = stack entries pushed by the ancestors (bounded by max_stack)
  struct Item { int32_t ref; float lo[3], hi[3]; uint32_t depth, pend; };
  std::vector<Item> stack;
  stack.push_back(Item{root, {-1e30f, -1e30f, -1e30f}, {1e30f, 1e30f, 1e30f}, 0, 0});
  uint32_t nodes_seen = 0;
  while (!stack.empty()) {
    Item it = stack.back();
    stack.pop_back();
    if (it.depth >= (uint32_t)mrt::kMaxTraversalStack) return bad("BVH too deep");
    if (it.ref >= 0) {
      if ((uint32_t)it.ref < node_lo || (uint32_t)it.ref - node_lo >= num_nodes) return bad("BVH node index out of range");
      ++nodes_seen;
      Item ch[4];
      uint32_t nc = 0;
      {
        const float* n = node((uint32_t)it.ref);
        for (int c = 0; c < 4; ++c) {
          const int32_t ref = (int32_t)fbits(n[24 + c]);
          if (ref == mrt::kEmptyChild) continue;
          if (nc != (uint32_t)c) return bad("BVH4 empty slot before a used one");
          ch[nc++] = Item{ref, {n[c], n[8 + c], n[16 + c]}, {n[4 + c], n[12 + c], n[20 + c]}, it.depth + 1, 0};
        }
        if (nc < 2) return bad("BVH4 node with fewer than two children");
      }
      for (uint32_t c = 0; c < nc; ++c) {
        for (int k = 0; k < 3; ++k)
          if (!(ch[c].lo[k] <= ch[c].hi[k])) return bad("BVH empty child box");
        ch[c].pend = it.pend + nc - 1;
        if (ch[c].pend > max_stack) return bad("BVH stack bound too small");
        stack.push_back(ch[c]);
      }
    } else {
      const uint32_t leaf = ~(uint32_t)it.ref;
      const uint32_t first = leaf >> mrt::kLeafCountBits, cnt = (leaf & (mrt::kMaxLeafSize - 1)) + 1;
      if (first < tri_lo || first - tri_lo + cnt > tri_count) return bad("BVH leaf range out of bounds");
      for (uint32_t k = first; k < first + cnt; ++k) {
        const float* t = tri(k);
        const uint32_t prim = fbits(t[3]);
        if (prim >= T || !want[prim] || seen[prim]) return bad("BVH primitive missing, foreign or duplicated");
        seen[prim] = 1;
        for (int c = 0; c < 3; ++c) {
          const float* p = h.vertices[h.references[prim].tri[c]].v;
          for (int a = 0; a < 3; ++a)
            if (!(p[a] >= it.lo[a] && p[a] <= it.hi[a])) return bad("BVH box does not contain its triangle");
        }
        // leaf record = (v0, prim), (v1 - v0), (v2 - v0)
        const float* v0 = h.vertices[h.references[prim].tri[0]].v;
        const float* v1 = h.vertices[h.references[prim].tri[1]].v;
        const float* v2 = h.vertices[h.references[prim].tri[2]].v;
        for (int a = 0; a < 3; ++a)
          if (t[a] != v0[a] || t[4 + a] != v1[a] - v0[a] || t[8 + a] != v2[a] - v0[a])
            return bad("BVH leaf triangle record mismatch");
      }
    }
  }
  for (uint32_t t = 0; t < T; ++t)
    if (want[t] && !seen[t]) return bad("BVH primitive not referenced");
  if (nodes_seen != num_nodes) return bad("BVH has unreachable nodes");
  return MRT_OK;
}
}  // namespace
}  // extern "C++"

int mrt_scene_check_bvh(const mrt_scene* scene) {
  if (!scene) return fail(MRT_ERR_INVALID, "null scene");
  const mrt::BvhResult& b = scene->bvh;
  const mrt::HostScene& h = scene->host;
  const uint32_t T = (uint32_t)h.references.size();
  std::vector<uint8_t> all(T, 1);
  if (const char* dn = mrt::diag_env("MRT_DUMP_NODE")) {   // diagnostic: one node's rows and its leaf triangles
    const uint32_t k = (uint32_t)std::strtoul(dn, nullptr, 0);
    if (k < b.num_nodes) {
      const float* n = &b.nodes[32 * (size_t)k];
      for (int i = 0; i < 32; ++i) std::fprintf(stderr, "NODE %u %d %08x %.9g\n", k, i, fbits(n[i]), n[i]);
      for (int c = 0; c < 4; ++c) {
        const int32_t r = (int32_t)fbits(n[24 + c]);
        if (r >= 0 || r == mrt::kEmptyChild) continue;
        const uint32_t lr = ~(uint32_t)r, first = lr >> mrt::kLeafCountBits, cnt = (lr & (mrt::kMaxLeafSize - 1)) + 1;
        for (uint32_t t = first; t < first + cnt; ++t)
          for (int i = 0; i < 12; ++i)
            std::fprintf(stderr, "TRI %d %u %d %08x\n", c, t, i, fbits(b.tris[12 * (size_t)t + i]));
      }
    }
  }
  int rc = check_tree(
      h, b.root, 0, b.num_nodes, 0, T, b.max_stack, all, [&](uint32_t r) { return &b.nodes[32 * (size_t)r]; },
      [&](uint32_t k) { return &b.tris[12 * (size_t)k]; }, "main tree");
  if (rc || scene->occ_keep.empty()) return rc;
  // the occluder tree: exactly the kept primitives, its own stack bound, which
  // the renderer's stack (sized by the deeper tree) covers
  std::vector<uint8_t> kept(T, 0);
  for (uint32_t p : scene->occ_keep) kept[p] = 1;
  const uint32_t occ_nodes = (uint32_t)(scene->occ_nodes.size() / 32);
  if (scene->occ_max_stack > b.max_stack) return fail(MRT_ERR_STATE, "occluder tree: deeper than the main tree");
  return check_tree(
      h, scene->occ_root, scene->occ_node_base, occ_nodes, T, (uint32_t)scene->occ_keep.size(), scene->occ_max_stack,
      kept, [&](uint32_t r) { return &scene->occ_nodes[32 * (size_t)(r - scene->occ_node_base)]; },
      [&](uint32_t k) { return &scene->occ_tris[12 * (size_t)(k - T)]; }, "occluder tree");
}

int mrt_debug_magic_div(uint32_t d, const uint32_t* n, uint32_t count, uint32_t* q) {
  if (d == 0 || (count && (!n || !q))) return fail(MRT_ERR_INVALID, "mrt_debug_magic_div: bad argument");
  const mrt::MagicDiv m = mrt::magic_div(d);
  for (uint32_t i = 0; i < count; ++i) q[i] = mrt::mdiv_host(n[i], m);
  return MRT_OK;
}

int mrt_debug_box_margin(const mrt_scene* scene, const void* rays, uint32_t stride, uint32_t count,
                         const void* intersections, float* out) {
  if (!scene || (count && (!rays || !intersections || !out))) return fail(MRT_ERR_INVALID, "null argument");
  if (stride < 32 || stride % 4) return fail(MRT_ERR_INVALID, "ray stride must be >= 32 and a multiple of 4");
  const mrt::BvhResult& b = scene->bvh;
  const mrt::HostScene& h = scene->host;
  const uint32_t T = (uint32_t)h.references.size();
  // (parent node, child slot) of every interior node and of every primitive's leaf
  struct Up { uint32_t node, slot; };
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  std::vector<Up> node_up(b.num_nodes, Up{kNone, 0}), prim_up(T, Up{kNone, 0});
  if (b.root >= 0)
    for (uint32_t n = 0; n < b.num_nodes; ++n)
      for (uint32_t c = 0; c < 4; ++c) {
        const int32_t ref = (int32_t)fbits(b.nodes[32 * (size_t)n + 24 + c]);
        if (ref == mrt::kEmptyChild) continue;
        if (ref >= 0) { node_up[ref] = Up{n, c}; continue; }
        const uint32_t lr = ~(uint32_t)ref, first = lr >> mrt::kLeafCountBits, cnt = (lr & (mrt::kMaxLeafSize - 1)) + 1;
        for (uint32_t k = first; k < first + cnt; ++k) prim_up[fbits(b.tris[12 * (size_t)k + 3])] = Up{n, c};
      }
  // triangles around each vertex position (vertex records are per (position,
  // normal), so corners are matched by their position bits)
  std::vector<std::pair<uint64_t, uint32_t>> corner;   // (hash of position, triangle)
  corner.reserve(3 * (size_t)T);
  auto pos_key = [&](uint32_t vi) {
    const float* v = h.vertices[vi].v;
    return ((uint64_t)fbits(v[0]) * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)fbits(v[1]) * 0xC2B2AE3D27D4EB4Full) ^
           ((uint64_t)fbits(v[2]) * 0x165667B19E3779F9ull);
  };
  for (uint32_t t = 0; t < T; ++t)
    for (int c = 0; c < 3; ++c) corner.emplace_back(pos_key(h.references[t].tri[c]), t);
  std::sort(corner.begin(), corner.end());
  const uint8_t* rp = static_cast<const uint8_t*>(rays);
  const mrt::RefIntersection* is = static_cast<const mrt::RefIntersection*>(intersections);
  for (uint32_t i = 0; i < count; ++i) {
    const float* f = reinterpret_cast<const float*>(rp + (size_t)i * stride);
    float* o4 = out + 4 * (size_t)i;
    o4[0] = o4[1] = o4[2] = o4[3] = -INFINITY;   // a miss, or a leaf-root tree (no box above the triangle)
    if (!(is[i].distance >= 0.0f) || is[i].triangleIndex >= T || prim_up[is[i].triangleIndex].node == kNone) continue;
    const float tmin = f[3];
    float inv[3], oinv[3];
    for (int a = 0; a < 3; ++a) {   // kernels.hip make_raybox (the fast build's reciprocal correctly rounded here)
      const float d = f[4 + a], dd = std::fabs(d) > 1e-20f ? d : std::copysign(1e-20f, d);
      inv[a] = 1.0f / dd;
      oinv[a] = f[a] * inv[a];
    }
    // the worst (t_entry - t) / t over the boxes above primitive k's leaf
    auto margin = [&](uint32_t k, float t, float* worst) {
      for (Up u = prim_up[k]; u.node != kNone; u = node_up[u.node]) {
        const float* n = &b.nodes[32 * (size_t)u.node];
        for (int form = 0; form < 2; ++form) {   // 0: precise (p - o) * inv, 1: fast fma(p, inv, -o * inv)
          float tn = tmin, tf = INFINITY;
          for (int a = 0; a < 3; ++a) {
            const float lo = n[8 * a + u.slot], hi = n[8 * a + 4 + u.slot];
            const float x0 = form ? std::fma(lo, inv[a], -oinv[a]) : (lo - f[a]) * inv[a];
            const float x1 = form ? std::fma(hi, inv[a], -oinv[a]) : (hi - f[a]) * inv[a];
            tn = std::fmax(tn, std::fmin(x0, x1));
            tf = std::fmin(tf, std::fmax(x0, x1));
          }
          // a box the ray's slab interval misses altogether: no culling slack finds the triangle
          worst[form] = std::fmax(worst[form], tn <= tf ? (tn - t) / t : INFINITY);
        }
      }
    };
    const uint32_t hit = is[i].triangleIndex;
    const float t_hit = is[i].distance;
    margin(hit, t_hit, o4);
    // near ties: triangles sharing a vertex position with the hit whose
    // Moller-Trumbore test some rounding of its float operations could pass
    // (a build that rounds differently — FMA contraction, an approximate
    // reciprocal — may report one of them instead, at its own t: DESIGN.md
    // §3.1's ray).  b1, b2 and t are evaluated exactly (double, on the float
    // inputs) with first-order error bounds of 4u per operation chain; a
    // neighbour counts when every test passes within its bound, and its slack
    // is taken at the smallest t the bound allows.
    const double o[3] = {f[0], f[1], f[2]}, d[3] = {f[4], f[5], f[6]};
    std::vector<uint32_t> ring;
    for (int c = 0; c < 3; ++c) {
      const uint64_t key = pos_key(h.references[hit].tri[c]);
      for (auto it = std::lower_bound(corner.begin(), corner.end(), std::make_pair(key, 0u));
           it != corner.end() && it->first == key; ++it)
        if (it->second != hit) ring.push_back(it->second);
    }
    std::sort(ring.begin(), ring.end());
    ring.erase(std::unique(ring.begin(), ring.end()), ring.end());
    auto norm = [](const double* x) { return std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]); };
    for (uint32_t k : ring) {
      const float* v0 = h.vertices[h.references[k].tri[0]].v;
      const float* v1 = h.vertices[h.references[k].tri[1]].v;
      const float* v2 = h.vertices[h.references[k].tri[2]].v;
      double e1[3], e2[3], sv[3];   // e1, e2 as the kernels' float records hold them
      for (int a = 0; a < 3; ++a) {
        e1[a] = (double)(v1[a] - v0[a]);
        e2[a] = (double)(v2[a] - v0[a]);
        sv[a] = o[a] - (double)v0[a];
      }
      const double p[3] = {d[1] * e2[2] - d[2] * e2[1], d[2] * e2[0] - d[0] * e2[2], d[0] * e2[1] - d[1] * e2[0]};
      const double q[3] = {sv[1] * e1[2] - sv[2] * e1[1], sv[2] * e1[0] - sv[0] * e1[2], sv[0] * e1[1] - sv[1] * e1[0]};
      const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
      if (det == 0.0) continue;
      const double b1 = (sv[0] * p[0] + sv[1] * p[1] + sv[2] * p[2]) / det;
      const double b2 = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) / det;
      const double t = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) / det;
      constexpr double u4 = 4.0 * 0x1p-24;
      const double np = norm(p), nq = norm(sv) * norm(e1) + norm(q), ad = std::fabs(det);
      const double eb1 = u4 * (norm(sv) * np + std::fabs(b1) * norm(e1) * np) / ad;
      const double eb2 = u4 * (norm(d) * nq + std::fabs(b2) * norm(e1) * np) / ad;
      const double et = u4 * (norm(e2) * nq + std::fabs(t) * norm(e1) * np) / ad;
      if (!(b1 >= -eb1 && b2 >= -eb2 && b1 + b2 <= 1.0 + eb1 + eb2 && t + et >= tmin && t - et > 0.0)) continue;
      if (!(std::fabs(t - t_hit) <= 0x1p-10 * t_hit + et)) continue;
      margin(k, (float)(t - et), o4 + 2);
    }
  }
  return MRT_OK;
}

int mrt_scene_destroy(mrt_scene* scene) {
  delete scene;
  return MRT_OK;
}

// ---------------------------------------------------------------------------
// acceleration structure over raw buffers (MPSTriangleAccelerationStructure +
// MPSRayIntersector, renderer/Renderer.mm:456-469)
// ---------------------------------------------------------------------------
namespace {
int accel_build(mrt_accel* a) {
  const mrt_accel_desc& d = a->desc;
  const uint32_t T = d.triangle_count;
  const uint32_t leaf = d.max_leaf_size ? d.max_leaf_size : 2;
  HIP_TRY(hipSetDevice(d.device));
  hipStream_t s = (hipStream_t)d.stream;
  std::string err;
  if (a->info.builder != MRT_BVH_HOST_SAH) {
    mrt::GpuBvhResult g;
    if (mrt::build_bvh_gpu(reinterpret_cast<const float*>(d.vertices), d.vertex_stride, d.indices, T, leaf,
                           a->info.builder == MRT_BVH_DEVICE_PLOC ? mrt::GpuBvhAlgo::kPloc : mrt::GpuBvhAlgo::kLbvh,
                           s, g, err) != hipSuccess)
      return fail(MRT_ERR_HIP, "device BVH build failed: " + err);
    (void)a->nodes.alloc(0);
    (void)a->tris.alloc(0);
    a->nodes.p = g.nodes; a->nodes.bytes = g.nodes_bytes;
    a->tris.p = g.tris; a->tris.bytes = g.tris_bytes;
    a->dev.root = g.root;
    a->dev.num_nodes = g.num_nodes;
    a->dev.max_stack = g.max_stack;
    a->info.bvh_nodes = g.num_nodes;
    a->info.bvh_leaves = g.num_leaves;
    a->info.bvh_levels = g.levels;
    a->info.bvh_max_stack = g.max_stack;
    a->info.build_ms = g.build_ms;
  } else {
    // host binned SAH: read the buffers back (the reference's own data path
    // never does this; kept for quality comparison and as a fallback-free
    // alternative for small scenes)
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t nv = 0;
    std::vector<uint32_t> idx((size_t)T * 3);
    if (T) HIP_TRY(hipMemcpy(idx.data(), d.indices, idx.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t v : idx) nv = std::max(nv, v + 1);
    std::vector<uint8_t> verts((size_t)nv * d.vertex_stride);
    if (nv) HIP_TRY(hipMemcpy(verts.data(), d.vertices, verts.size(), hipMemcpyDeviceToHost));
    mrt::BvhBuildOptions opt;
    opt.max_leaf_size = leaf;
    opt.width = 4;
    opt.lds_node_budget = 0;
    mrt::BvhResult b;
    const auto t0 = std::chrono::steady_clock::now();
    if (T == 0) return fail(MRT_ERR_INVALID, "host SAH build of an empty structure (use the device builder)");
    if (!mrt::build_bvh(reinterpret_cast<const float*>(verts.data()), d.vertex_stride, idx.data(), T, opt, b, err))
      return fail(MRT_ERR_INVALID, "BVH build failed: " + err);
    a->info.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    HIP_TRY(upload(a->nodes, b.nodes.data(), b.nodes.size() * 4));
    HIP_TRY(upload(a->tris, b.tris.data(), b.tris.size() * 4));
    a->dev.root = b.root;
    a->dev.num_nodes = b.num_nodes;
    a->dev.max_stack = b.max_stack;
    a->info.bvh_nodes = b.num_nodes;
    a->info.bvh_leaves = b.num_leaves;
    a->info.bvh_levels = b.wide_depth;
    a->info.bvh_max_stack = b.max_stack;
  }
  if (a->dev.max_stack > (uint32_t)mrt::kMaxTraversalStack) return fail(MRT_ERR_INVALID, "BVH needs a deeper traversal stack");
  if ((uint64_t)a->nodes.bytes >= (1ull << 32) || (uint64_t)a->tris.bytes >= (1ull << 32))   // 32-bit buffer offsets
    return fail(MRT_ERR_INVALID, "acceleration structure too large: nodes or leaf triangles exceed 4 GiB");
  HIP_TRY(alloc_isect_spill(a->isect_spill, a->dev.max_stack));
  a->dev.nodes = a->nodes.as<float>();
  a->dev.tris = a->tris.as<float>();
  a->dev.num_triangles = T;
  a->dev.width = 4;
  a->dev.lds_nodes = 0;
  a->info.triangles = T;
  a->info.device_bytes = a->nodes.bytes + a->tris.bytes;
  return MRT_OK;
}
}  // namespace

int mrt_accel_create(const mrt_accel_desc* desc, mrt_accel** out) {
  if (!desc || !out) return fail(MRT_ERR_INVALID, "mrt_accel_create: null argument");
  *out = nullptr;
  if (desc->triangle_count && (!desc->vertices || !desc->indices))
    return fail(MRT_ERR_INVALID, "mrt_accel_create: null buffer");
  if (desc->vertex_stride < 12 || desc->vertex_stride % 4) return fail(MRT_ERR_INVALID, "mrt_accel_create: bad vertex_stride");
  if (desc->max_leaf_size > (uint32_t)mrt::kMaxLeafSize) return fail(MRT_ERR_INVALID, "mrt_accel_create: max_leaf_size > 16");
  const uint32_t builder = desc->builder ? desc->builder : MRT_BVH_DEVICE_PLOC;
  if (builder != MRT_BVH_HOST_SAH && builder != MRT_BVH_DEVICE_LBVH && builder != MRT_BVH_DEVICE_PLOC)
    return fail(MRT_ERR_INVALID, "unknown builder");
  std::unique_ptr<mrt_accel> a(new mrt_accel());
  a->desc = *desc;
  a->info.builder = builder;
  const int rc = accel_build(a.get());
  if (rc) return rc;
  *out = a.release();
  return MRT_OK;
}

int mrt_accel_rebuild(mrt_accel* accel) {
  if (!accel) return fail(MRT_ERR_INVALID, "null accel");
  return accel_build(accel);
}

int mrt_accel_intersect(const mrt_accel* accel, const void* rays, uint32_t stride, uint32_t count, void* isect,
                        uint32_t flags, void* stream) {
  if (!accel || (!rays && count) || (!isect && count) || stride < 32 || (stride % 4))
    return fail(MRT_ERR_INVALID, "mrt_accel_intersect: bad argument");
  HIP_TRY(hipSetDevice(accel->desc.device));
  if (precise(flags))
    HIP_TRY(mrt::precise::launch_intersect(accel->dev, rays, stride, count, (mrt::RefIntersection*)isect,
                                           accel->isect_spill.as<uint32_t>(), (hipStream_t)stream));
  else
    HIP_TRY(mrt::fast::launch_intersect(accel->dev, rays, stride, count, (mrt::RefIntersection*)isect,
                                        accel->isect_spill.as<uint32_t>(), (hipStream_t)stream));
  return MRT_OK;
}

int mrt_accel_info_get(const mrt_accel* accel, mrt_accel_info* info) {
  if (!accel || !info) return fail(MRT_ERR_INVALID, "null argument");
  *info = accel->info;
  return MRT_OK;
}

int mrt_accel_destroy(mrt_accel* accel) {
  delete accel;
  return MRT_OK;
}

// ---------------------------------------------------------------------------
// stage-level ABI
// ---------------------------------------------------------------------------
#define STAGE_CALL(call) \
  HIP_TRY(precise(flags) ? mrt::precise::call : mrt::fast::call)

int mrt_raygen(const mrt_scene* scene, uint32_t W, uint32_t H, const float* noise, void* rays, uint32_t flags,
               void* stream) {
  if (!scene || !noise || !rays || W < 2 || H < 2) return fail(MRT_ERR_INVALID, "mrt_raygen: bad argument");
  STAGE_CALL(launch_raygen(W, H, noise, (mrt::RefRay*)rays, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_intersect(const mrt_scene* scene, const void* rays, uint32_t stride, uint32_t count, void* isect,
                  uint32_t flags, void* stream) {
  if (!scene || (!rays && count) || (!isect && count) || stride < 32 || (stride % 4))
    return fail(MRT_ERR_INVALID, "mrt_intersect: bad argument");
  STAGE_CALL(launch_intersect(scene->dev, rays, stride, count, (mrt::RefIntersection*)isect,
                              scene->isect_spill.as<uint32_t>(), (hipStream_t)stream));
  return MRT_OK;
}

int mrt_shade(const mrt_scene* scene, uint32_t W, uint32_t H, uint32_t frame_index, uint32_t L, const float* noise,
              const void* isect, void* rays, void* srays, uint32_t flags, void* stream) {
  if (!scene || !noise || !isect || !rays || !srays || W == 0 || H == 0 || L == 0)
    return fail(MRT_ERR_INVALID, "mrt_shade: bad argument");
  STAGE_CALL(launch_shade(scene->dev, W, H, frame_index, L, noise, (const mrt::RefIntersection*)isect,
                          (mrt::RefRay*)rays, (mrt::RefShadowRay*)srays,
                          (flags & MRT_FLAG_DEBUG_MATERIAL) ? mrt::kShadeDebugMaterial : 0u, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_resolve_shadow(const mrt_scene* scene, uint32_t count, const void* isect, void* rays, const void* srays,
                       uint32_t flags, void* stream) {
  if (!scene || (count && (!isect || !rays || !srays))) return fail(MRT_ERR_INVALID, "mrt_resolve_shadow: bad argument");
  STAGE_CALL(launch_resolve(count, (const mrt::RefIntersection*)isect, (mrt::RefRay*)rays,
                            (const mrt::RefShadowRay*)srays, (hipStream_t)stream));
  return MRT_OK;
}

int mrt_accumulate(const mrt_scene* scene, uint32_t W, uint32_t H, uint32_t frame_index, const void* rays,
                   float* image, uint32_t flags, void* stream) {
  if (!scene || !rays || !image || W == 0 || H == 0) return fail(MRT_ERR_INVALID, "mrt_accumulate: bad argument");
  STAGE_CALL(launch_accumulate(W, H, frame_index, (const mrt::RefRay*)rays, image, !(flags & MRT_FLAG_NO_ACCUMULATE),
                               (hipStream_t)stream));
  return MRT_OK;
}

// ---------------------------------------------------------------------------
// renderer
// ---------------------------------------------------------------------------
int mrt_renderer_create(const mrt_renderer_desc* desc, mrt_renderer** out) {
  if (!desc || !out || !desc->scene) return fail(MRT_ERR_INVALID, "mrt_renderer_create: null argument");
  *out = nullptr;
  if (desc->width < 2 || desc->height < 2 || desc->width > 32768 || desc->height > 32768)
    return fail(MRT_ERR_INVALID, "image size must be in [2, 32768]");
  if ((uint64_t)desc->width * desc->height >= (1ull << 31)) return fail(MRT_ERR_INVALID, "image too large");
  if (desc->max_path_length == 0 || desc->max_path_length > 64)
    return fail(MRT_ERR_INVALID, "max_path_length must be in [1, 64]");
  const uint32_t S = std::max<uint32_t>(1, desc->shard_count);
  if (desc->shard_rank >= S) return fail(MRT_ERR_INVALID, "shard_rank >= shard_count");
  constexpr uint32_t kKnownFlags = MRT_FLAG_PRECISE | MRT_FLAG_PROFILE | MRT_FLAG_STATIC_NOISE |
                                   MRT_FLAG_NO_ACCUMULATE | MRT_FLAG_DEBUG_MATERIAL;
  if (desc->flags & ~kKnownFlags) return fail(MRT_ERR_INVALID, "unknown renderer flags");
  std::unique_ptr<mrt_renderer> r(new mrt_renderer());
  r->scene = desc->scene;
  r->desc = *desc;
  r->desc.shard_count = S;
  HIP_TRY(hipSetDevice(desc->scene->device));
  if (desc->stream) {
    r->stream = (hipStream_t)desc->stream;
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking));
    r->own_stream = true;
  }
  r->own_image = desc->image == nullptr;
  r->image = desc->image;
  r->noise = std::make_unique<mrt::NoiseSchedule>(desc->seed, (desc->flags & MRT_FLAG_STATIC_NOISE) != 0);
  for (DrawRecord& d : r->draws) {
    HIP_TRY(hipEventCreate(&d.start));
    HIP_TRY(hipEventCreate(&d.stop));
    HIP_TRY(hipEventCreateWithFlags(&d.cleared, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&d.copied, hipEventDisableTiming));
  }
  // LDS stack capacity: the BVH's bound rounded up to 8/16 entries when it is
  // <= 16; deeper BVHs keep 8 entries in LDS and spill the rest to global
  // memory (MRT_STACK overrides the cap).  LDS per block bounds the resident
  // blocks per CU, and for global-memory traversal occupancy wins: C4 with
  // 8 LDS entries + spill ran 1.5x faster than with a 32-entry LDS stack.
  // r3, with traversal slack: trees deeper than 32 entries (the 1M-triangle
  // scenes, 48) keep 12 in LDS — C4 +1.9 %; C3 (26) is best at 8 (12: -0.4 %,
  // C3g -0.9 %), and 16 entries lose everywhere (C4 -0.4 %, C3g -2.4 %)
  // the deeper of the main and the occluder tree (dev.max_stack): shadow rays
  // may traverse either
  const uint32_t need = desc->scene->dev.max_stack;
  uint32_t cap = need <= 16 ? 16 : (need > 32 ? 12 : 8);
  if (const char* v = mrt::diag_env("MRT_STACK")) cap = std::max<uint32_t>(8, (uint32_t)std::strtoul(v, nullptr, 0));
  const uint32_t want = std::min(need, cap);
  r->stack_entries = want <= 8 ? 8 : want <= 12 ? 12 : want <= 16 ? 16 : want <= 24 ? 24 : 32;
  if (need > r->stack_entries)   // spill variants: 8 / 12 (path kernel; the wavefront runs 16) / 16 / 32
    r->stack_entries = r->stack_entries <= 8 ? 8 : r->stack_entries <= 12 ? 12 : r->stack_entries <= 16 ? 16 : 32;
  if (const char* dbg = mrt::diag_env("MRT_DEBUG")) r->debug = (uint32_t)std::strtoul(dbg, nullptr, 0);
  if (const char* v = mrt::diag_env("MRT_COUNTER_FOLD")) r->counter_fold = std::atoi(v) != 0;
  if (const char* v = mrt::diag_env("MRT_PROFILE_EVERY"))
    r->profile_every = std::max<uint32_t>(1, (uint32_t)std::strtoul(v, nullptr, 0));
  {
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, desc->scene->device) == hipSuccess)
      r->wall_khz = (double)khz;
  }
  if (const char* v = mrt::diag_env("MRT_SPANS"))
    if (std::atoi(v) == 0) r->wall_khz = 0.0;
  // two frame batches in flight on their own streams (one launch's drain
  // overlaps the next launch's start): a tile share +5 % (r3.3), a whole C2
  // frame +0.9 % (9598 / 9596 / 9600 vs 9521 / 9479 / 9521 Mpaths/s,
  // alternating in one call)
  r->inflight = 2u;
  if (const char* v = mrt::diag_env("MRT_INFLIGHT")) r->inflight = (uint32_t)std::strtoul(v, nullptr, 0);
  r->inflight = std::max<uint32_t>(1, std::min<uint32_t>(8, r->inflight));
  r->slots.resize(r->inflight);
  for (uint32_t k = 0; k < r->inflight; ++k) {
    FrameSlot& fs = r->slots[k];
    if (r->inflight == 1) {   // one slot: everything in order on the main stream
      fs.stream = r->stream;
    } else {
      HIP_TRY(hipStreamCreateWithFlags(&fs.stream, hipStreamNonBlocking));
      fs.own_stream = true;
    }
    HIP_TRY(hipEventCreateWithFlags(&fs.acc_done, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&fs.kernel_done, hipEventDisableTiming));
  }
  // kernel: scenes traversed from global memory run the path megakernel (all
  // bounces of a frame batch in one launch: C3 +15 %, C4 +1.5 % over the
  // wavefront), scenes staged whole in LDS the wavefront of per-bounce
  // launches (C2: the path kernel is 24 % slower); MRT_KERNEL=path|wave
  // overrides.
  if (const char* v = mrt::diag_env("MRT_PRIMARY")) r->primary_allowed = std::atoi(v) != 0;
  if (const char* v = mrt::diag_env("MRT_PRIMARY_CAP"))
    r->primary_cap = std::max<uint32_t>(1, std::min<uint32_t>(mrt::kPrimaryFallback - 1, (uint32_t)std::strtoul(v, nullptr, 0)));
  r->path_mode = mrt::fast::path_preferred(desc->scene->dev);
  if (const char* k = mrt::diag_env("MRT_KERNEL")) r->path_mode = std::strcmp(k, "path") == 0;
  // streaming wavefront (one launch per frame batch, per-wave ray queues)
  // for whole-scene-in-LDS scenes; MRT_STREAM=0 keeps one launch per bounce
  {
    const char* c = mrt::diag_env("MRT_STREAM");
    const bool want = !c || std::atoi(c) != 0;
    r->stream_allowed = want && !r->path_mode && desc->max_path_length <= mrt::kStreamMaxL &&
                        mrt::fast::stream_supported(desc->scene->dev, r->stack_entries);
  }
  // persistent grid of the kernel this renderer launches: the stream kernel
  // sizes it by its own LDS (the per-bounce kernel's segment scratch grows
  // with the grid: sized for that, a 24-KB scene image + stack left C2 at 4
  // instead of 5 blocks per CU)
  const bool precise = (desc->flags & MRT_FLAG_PRECISE) != 0;
  if (r->path_mode)
    HIP_TRY(precise ? mrt::precise::path_grid(r->scene->dev, r->stack_entries, &r->grid)
                    : mrt::fast::path_grid(r->scene->dev, r->stack_entries, &r->grid));
  else if (r->stream_allowed)
    HIP_TRY(precise ? mrt::precise::stream_grid(r->scene->dev, r->stack_entries, &r->grid)
                    : mrt::fast::stream_grid(r->scene->dev, r->stack_entries, &r->grid));
  else
    HIP_TRY(precise ? mrt::precise::bounce_grid(desc->scene->dev, r->stack_entries, 0u, &r->grid)
                    : mrt::fast::bounce_grid(desc->scene->dev, r->stack_entries, 0u, &r->grid));
  if (const char* g = mrt::diag_env("MRT_GRID")) r->grid = std::max<uint32_t>(1, (uint32_t)std::strtoul(g, nullptr, 0));
  // the noise schedule's upload stream, staging buffers and worker on the
  // renderer's device.  Created after the render streams: a process has 4
  // hardware queues and streams share them round-robin in creation order, so
  // a stream created before the render streams pushed a render stream onto a
  // queue another stream's work serialises with (C2 -10 %, C4 -7 %, measured r6)
  HIP_TRY(r->noise->init());
  int rc = alloc_frame_buffers(r.get());
  if (rc) return rc;
  *out = r.release();
  return MRT_OK;
}

int mrt_renderer_resize(mrt_renderer* r, uint32_t width, uint32_t height) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  if (width < 2 || height < 2 || width > 32768 || height > 32768) return fail(MRT_ERR_INVALID, "bad size");
  if (!r->own_image) return fail(MRT_ERR_STATE, "cannot resize an externally owned image");
  int rc = finalize_pending(r);
  if (rc) return rc;
  rc = exchange_drop(r, true);   // a pending gather was packed for the old size: never unpack it into the new image
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(r->stream));
  r->desc.width = width;
  r->desc.height = height;
  r->x.slab_floats = 0;    // the exchange buffers are re-sized for the new image at the next exchange
  return alloc_frame_buffers(r);
}

int mrt_renderer_reset(mrt_renderer* r) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  int rc = exchange_drop(r, false);   // the pre-reset frame's deferred tiles must not land in the cleared image
  if (rc) return rc;
  // The next frame (f = 0) overwrites every pixel this renderer owns, and
  // pixels it does not own stay 0 — unless an exchange wrote other ranks'
  // tiles into the image: only then is it cleared (stream-ordered after
  // the pending draws).  An external image is always cleared.
  if (r->image_foreign || !r->own_image) {
    HIP_TRY(hipMemsetAsync(r->image, 0, (size_t)r->desc.width * r->desc.height * 16, r->stream));
    r->image_foreign = false;
  }
  r->frame_index = 0;
  r->stats.frame_index = 0;   // cumulative counters (paths, A, kernel time) persist
  return MRT_OK;
}

int mrt_renderer_prepare(mrt_renderer* r, uint32_t n) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  return acquire_noise(r, (int64_t)r->frame_index, std::max<uint32_t>(1, n), nullptr);
}

int mrt_renderer_draw_n(mrt_renderer* r, uint32_t n) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  if (r->max_frames)   // MAX_FRAMES: renderer/Renderer.mm:589-590
    n = r->frame_index >= r->max_frames ? 0u : (uint32_t)std::min<uint64_t>(n, r->max_frames - r->frame_index);
  if (n == 0) return MRT_OK;
  DrawRecord& d = r->draws[r->draw_next];
  // at most kDrawRing (3) draws in flight: the ring entry's previous draw must
  // have finished — the reference's MaxBuffersInFlight semaphore
  // (renderer/Renderer.mm:16, :593-600), the only host wait of a draw
  if (d.pending && hipEventQuery(d.copied) == hipErrorNotReady) r->stats.inflight_waits += 1;
  int rc = finalize_draw(r, d);
  if (rc) return rc;
  r->draw_seq += 1;
  std::vector<mrt::NoiseSchedule::Chunk*> chunks;
  rc = acquire_noise(r, (int64_t)r->frame_index, n, &chunks);
  if (rc) return rc;
  const uint32_t L = r->desc.max_path_length;
  const uint32_t B = r->batch;
  // frame batches of up to B frames, none crossing a noise chunk (64 frames,
  // a multiple of B): a 64-frame draw from a multiple of 64 is one batch
  struct Batch { uint64_t f; uint32_t frames; mrt::NoiseSchedule::Chunk* noise; };
  std::vector<Batch> batches;
  for (uint64_t f = r->frame_index, end = r->frame_index + n; f < end;) {
    const int64_t k = mrt::NoiseSchedule::chunk_of((int64_t)f);
    const uint64_t chunk_end = (uint64_t)(k + 1) * mrt::NoiseSchedule::kChunkFrames;
    const uint32_t b = (uint32_t)std::min<uint64_t>({(uint64_t)B, end - f, chunk_end - f});
    batches.push_back({f, b, chunks[(size_t)(k - mrt::NoiseSchedule::chunk_of((int64_t)r->frame_index))]});
    f += b;
  }
  const uint32_t nb = (uint32_t)batches.size();
  // survivor counters [nb * L] and, 128-B aligned after them, the grab
  // counters of every launch of the draw: zeroed by ONE memset
  const size_t grab_words = (size_t)mrt::kGrabRanges * mrt::kGrabStride;
  const size_t grab_off = ((size_t)nb * L + 31) / 32 * 32;   // words
  const size_t span_off = (grab_off + (size_t)nb * L * grab_words + 1) / 2 * 8;   // bytes, 8-B aligned
  const size_t counter_bytes = span_off + (size_t)nb * 16;
  bool fresh = false;
  if (d.counters.bytes < counter_bytes) {
    HIP_TRY(d.counters.alloc(counter_bytes));
    fresh = true;
  }
  if (d.host_bytes < counter_bytes) {
    if (d.host) HIP_TRY(hipHostFree(d.host));
    d.host = d.host_dev = nullptr;
    d.host_bytes = 0;
    HIP_TRY(hipHostMalloc(&d.host, counter_bytes, hipHostMallocMapped));
    HIP_TRY(hipHostGetDevicePointer(&d.host_dev, d.host, 0));
    d.host_bytes = counter_bytes;
  }
  const uint32_t launches_per_batch = r->path_mode || r->stream_mode ? 1u : L;
  const bool profile = (r->desc.flags & MRT_FLAG_PROFILE) != 0;
  if (profile) {
    const size_t need = (size_t)2 * nb * launches_per_batch;   // at most every batch is timed
    while (d.kernel_events.size() < need) {
      hipEvent_t e;
      HIP_TRY(hipEventCreate(&e));
      d.kernel_events.push_back(e);
    }
  }
  HIP_TRY(hipEventRecord(d.start, r->stream));
  // The render launches never wait on the main stream (it only carries
  // accumulates and image work; a noise chunk's upload is waited for through
  // its own event): the counters are cleared on the first batch's render
  // stream and the draw's other render streams wait for that.
  // The draw's last accumulate copies its statistics to the pinned host copy
  // and zeroes the counters for the ring entry's next draw (whose host side
  // has waited for that accumulate in finalize_draw): a fresh buffer, or one
  // whose last draw stopped before its folding accumulate, is the only one to
  // clear here.  MRT_COUNTER_FOLD=0: memset + copy per draw.
  const uint32_t s0 = r->slot_next;
  const bool clear = fresh || !d.clean || !r->counter_fold;
  d.clean = false;   // set again once this draw's folding accumulate is enqueued
  if (clear) HIP_TRY(hipMemsetAsync(d.counters.p, 0, d.counters.bytes, r->slots[s0].stream));
  if (clear && r->inflight > 1 && nb > 1) {
    HIP_TRY(hipEventRecord(d.cleared, r->slots[s0].stream));
    for (uint32_t j = 1; j < std::min(nb, r->inflight); ++j)
      HIP_TRY(hipStreamWaitEvent(r->slots[(s0 + j) % r->inflight].stream, d.cleared, 0));
  }
  uint32_t* cnt = d.counters.as<uint32_t>();
  size_t ev = 0;
  for (uint32_t k = 0; k < nb; ++k) {
    const uint64_t f = batches[k].f;
    const uint32_t batch = batches[k].frames;
    mrt::NoiseSchedule::Chunk* nc = batches[k].noise;
    const uint32_t slot = (s0 + k) % r->inflight;
    FrameSlot& fs = r->slots[slot];
    const bool own = fs.stream != r->stream;
    // the slot's radiance is free once the accumulate that last read it ran.
    // (Rotating batch-sized regions of it instead, so that a single-frame
    // draw waits only once per 64 frames, measured -1.1 % on the per-frame
    // cadence: the next kernel then competes with the accumulates for CUs.)
    if (own && fs.acc_recorded) HIP_TRY(hipStreamWaitEvent(fs.stream, fs.acc_done, 0));
    float4* radiance = fs.radiance.as<float4>();
    // the noise chunk's upload (once per chunk upload and render stream)
    if (!(nc->waited_streams & (1u << slot))) {
      HIP_TRY(hipStreamWaitEvent(fs.stream, nc->ready, 0));
      nc->waited_streams |= 1u << slot;
    }
    uint32_t* seg = fs.segments.as<uint32_t>();
    uint32_t* meta = seg + 4 * (size_t)r->grid;
    for (uint32_t b = 0; b < launches_per_batch; ++b) {
      mrt::BounceArgs a{};
      a.width = r->desc.width;
      a.height = r->desc.height;
      a.frame_index = (uint32_t)f;
      a.batch = batch;
      a.bounce = b;
      a.max_path_length = L;
      a.shard_rank = r->desc.shard_rank;
      a.shard_count = r->desc.shard_count;
      a.tiles_x = r->tiles_x;
      a.num_slots = r->owned_tiles * 4096u;
      a.div_tiles = mrt::magic_div(a.tiles_x);
      a.div_slots = mrt::magic_div(a.num_slots);
      a.div_batch = mrt::magic_div(batch);
      // (a rank that owns no tile has num_slots 0: its lanes all exit at the
      // idx < num_slots * batch bound before any quotient by it)
      if (!mrt::magic_ok(a.div_tiles, a.tiles_x) ||
          (a.num_slots && !mrt::magic_ok(a.div_slots, a.num_slots)) ||
          !mrt::magic_ok(a.div_batch, batch))
        return fail(MRT_ERR_STATE, "draw: a launch divisor's magic multiplier does not divide exactly");
      a.debug = r->debug;
      a.flags = (r->desc.flags & MRT_FLAG_DEBUG_MATERIAL) ? mrt::kShadeDebugMaterial : 0u;
      a.in_segments = 2 * r->grid;   // two material classes per block
      a.in_seg_count = seg + (size_t)((b + 1) & 1) * 2 * r->grid;
      a.in_chunk = meta + ((b + 1) & 1);
      a.out_seg_count = seg + (size_t)(b & 1) * 2 * r->grid;
      a.out_chunk = meta + (b & 1);
      a.out_total = cnt + (size_t)k * L + b;
      a.grab = d.counters.as<uint32_t>() + grab_off + ((size_t)k * L + b) * grab_words;
      for (int p = 0; p < mrt::kQueuePlanes; ++p) {
        a.in_q.plane[p] = fs.queue[b & 1][p].as<float4>();
        a.out_q.plane[p] = fs.queue[(b + 1) & 1][p].as<float4>();
      }
      a.noise_window = static_cast<const float4*>(nc->dev);
      a.noise_offset = (uint32_t)((int64_t)f - mrt::NoiseSchedule::first_frame(mrt::NoiseSchedule::chunk_of((int64_t)f)));
      a.radiance = radiance;
      a.stack_spill = fs.spill.as<uint32_t>();
      a.bounce_counts = cnt + (size_t)k * L;
      a.primary = r->primary.as<uint32_t>();
      a.primary_bx = r->primary_bx;
      a.span = r->wall_khz > 0.0
                   ? reinterpret_cast<unsigned long long*>(static_cast<char*>(d.counters.p) + span_off) + 2 * k
                   : nullptr;
      // every batch holding a frame f with f % profile_every == 0: every
      // batch of a batched draw, every 8th single-frame draw
      const bool timed = profile && ((f % r->profile_every) == 0 || (f % r->profile_every) + batch > r->profile_every);
      if (timed) HIP_TRY(hipEventRecord(d.kernel_events[ev++], fs.stream));
      if (r->path_mode) HIP_TRY(launch_paths(r, a, fs.stream));
      else if (r->stream_mode) HIP_TRY(launch_stream(r, a, fs.stream));
      else HIP_TRY(launch_bounce(r, a, fs.stream));
      if (timed) HIP_TRY(hipEventRecord(d.kernel_events[ev++], fs.stream));
    }
    // accumulateImage for frames f .. f+batch-1 on the main stream, in batch
    // order (the running mean's order), behind this batch's render launch
    if (own) {
      HIP_TRY(hipEventRecord(fs.kernel_done, fs.stream));
      HIP_TRY(hipStreamWaitEvent(r->stream, fs.kernel_done, 0));
    }
    mrt::AccumArgs acc{};
    acc.width = r->desc.width;
    acc.height = r->desc.height;
    acc.frame_index = (uint32_t)f;
    acc.batch = batch;
    acc.shard_rank = r->desc.shard_rank;
    acc.shard_count = r->desc.shard_count;
    acc.tiles_x = r->tiles_x;
    // (MRT_DEBUG bit 256, ablation: the accumulate launches but touches no
    // pixel — its statistics fold alone; a wrong image)
    acc.num_slots = (r->debug & 256u) ? 0u : r->owned_tiles * 4096u;
    acc.radiance = radiance;
    acc.image = reinterpret_cast<float4*>(r->image);
    acc.accumulate = (r->desc.flags & MRT_FLAG_NO_ACCUMULATE) ? 0u : 1u;
    if (k + 1 == nb && r->counter_fold) {
      acc.counters = d.counters.as<uint32_t>();
      acc.host_counters = static_cast<uint32_t*>(d.host_dev);
      acc.copy_words = nb * L;
      acc.span_word = (uint32_t)(span_off / 4);
      acc.span_words = nb * 4;
      acc.zero_words = (uint32_t)(d.counters.bytes / 4);
    }
    HIP_TRY(launch_accumulate_frame(r, acc, r->stream));
    HIP_TRY(hipEventRecord(fs.acc_done, r->stream));
    fs.acc_recorded = true;
    if (k + 1 == nb && r->counter_fold) d.clean = true;
  }
  r->slot_next = (s0 + nb) % r->inflight;
  HIP_TRY(hipEventRecord(d.stop, r->stream));
  // the chunks' buffers are reusable once this draw's accumulates (which
  // follow every render launch of the draw) have run
  for (mrt::NoiseSchedule::Chunk* c : chunks) {
    HIP_TRY(hipEventRecord(c->last_use, r->stream));
    c->used = true;
  }
  {   // enqueued while the previous draw is still rendering (frames in flight)
    const DrawRecord& prev = r->draws[(r->draw_next + kDrawRing - 1) % kDrawRing];
    if (prev.pending && hipEventQuery(prev.stop) == hipErrorNotReady) r->stats.draws_overlapped += 1;
  }
  r->stats.draws += 1;
  // (no stream of its own: a process has few hardware queues — 4 by
  // default — and two streams sharing one serialise their launches)
  if (!r->counter_fold)
    HIP_TRY(hipMemcpyAsync(d.host, d.counters.p, counter_bytes, hipMemcpyDeviceToHost, r->stream));
  HIP_TRY(hipEventRecord(d.copied, r->stream));
  d.pending = true;
  d.frames = n;
  d.launches = nb;
  d.span_off = span_off;
  d.counter_bytes = counter_bytes;
  d.events = ev;
  r->draw_next = (r->draw_next + 1) % kDrawRing;
  r->frame_index += n;
  r->stats.frame_index = r->frame_index;
  r->stats.paths += r->owned_pixels * n;
  return MRT_OK;
}

int mrt_renderer_draw(mrt_renderer* r) { return mrt_renderer_draw_n(r, 1); }

int mrt_renderer_set_max_frames(mrt_renderer* r, uint32_t max_frames) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  r->max_frames = max_frames;
  return MRT_OK;
}

int mrt_renderer_sync(mrt_renderer* r) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  // the last collective first, with a bound: a stream blocked by a stuck
  // peer's collective would otherwise hold this host wait forever
  int rc = exchange_wait(r);
  if (rc) return rc;
  rc = finalize_pending(r);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(r->stream));
  return MRT_OK;
}

int mrt_renderer_image(mrt_renderer* r, float** device_image) {
  if (!r || !device_image) return fail(MRT_ERR_INVALID, "null argument");
  *device_image = r->image;
  return MRT_OK;
}

int mrt_renderer_stream(mrt_renderer* r, void** stream) {
  if (!r || !stream) return fail(MRT_ERR_INVALID, "null argument");
  *stream = (void*)r->stream;
  return MRT_OK;
}

int mrt_renderer_read_image(mrt_renderer* r, float* rgba, size_t count) {
  if (!r || !rgba) return fail(MRT_ERR_INVALID, "null argument");
  const size_t need = (size_t)r->desc.width * r->desc.height * 4;
  if (count < need) return fail(MRT_ERR_INVALID, "output buffer too small");
  int rc = exchange_flush(r);   // a deferred (overlapped) exchange lands first
  if (rc) return rc;
  rc = mrt_renderer_sync(r);
  if (rc) return rc;
  HIP_TRY(hipMemcpy(rgba, r->image, need * 4, hipMemcpyDeviceToHost));
  return MRT_OK;
}

int mrt_renderer_save_image(mrt_renderer* r, const char* path) {
  if (!r || !path) return fail(MRT_ERR_INVALID, "null argument");
  const uint32_t W = r->desc.width, H = r->desc.height;
  std::vector<float> img((size_t)W * H * 4);
  int rc = mrt_renderer_read_image(r, img.data(), img.size());
  if (rc) return rc;
  const std::string p(path);
  auto ends = [&](const char* s) { const size_t n = std::strlen(s); return p.size() >= n && p.compare(p.size() - n, n, s) == 0; };
  if (ends(".pfm")) return write_pfm(path, img, W, H);
  if (ends(".exr")) return write_exr(path, img, W, H);
  return fail(MRT_ERR_INVALID, "unsupported image extension (use .pfm or .exr)");
}

int mrt_image_load_exr(const char* path, float* rgba, size_t capacity, uint32_t* width, uint32_t* height) {
  if (!path || !width || !height) return fail(MRT_ERR_INVALID, "mrt_image_load_exr: null argument");
  std::vector<float> img;
  uint32_t W = 0, H = 0;
  std::string err;
  if (!mrt::load_exr(path, img, W, H, err)) return fail(MRT_ERR_IO, err);
  *width = W;
  *height = H;
  if (!rgba) return MRT_OK;
  if (capacity < img.size()) return fail(MRT_ERR_INVALID, "mrt_image_load_exr: buffer too small");
  std::memcpy(rgba, img.data(), img.size() * 4);
  return MRT_OK;
}

int mrt_renderer_load_reference(mrt_renderer* r, const char* path) {
  if (!r || !path) return fail(MRT_ERR_INVALID, "null argument");
  std::vector<float> img;
  uint32_t W = 0, H = 0;
  std::string err;
  if (!mrt::load_exr(path, img, W, H, err)) return fail(MRT_ERR_IO, err);
  if (W != r->desc.width || H != r->desc.height)
    return fail(MRT_ERR_INVALID, "reference image is " + std::to_string(W) + "x" + std::to_string(H) + ", renderer " +
                                     std::to_string(r->desc.width) + "x" + std::to_string(r->desc.height));
  HIP_TRY(hipSetDevice(r->scene->device));
  HIP_TRY(hipStreamSynchronize(r->stream));
  HIP_TRY(upload(r->reference, img.data(), img.size() * 4));
  return MRT_OK;
}

int mrt_renderer_display(mrt_renderer* r, uint32_t flags, float compare_scale, float* rgba, size_t count) {
  if (!r || !rgba) return fail(MRT_ERR_INVALID, "null argument");
  const size_t need = (size_t)r->desc.width * r->desc.height * 4;
  if (count < need) return fail(MRT_ERR_INVALID, "output buffer too small");
  if (((flags >> 8) & 0xFFu) && !r->reference.p) return fail(MRT_ERR_STATE, "compare mode without a loaded reference");
  int rc = exchange_flush(r);
  if (rc) return rc;
  if (r->display.bytes < need * 4) HIP_TRY(r->display.alloc(need * 4));
  rc = mrt_display(r->image, r->reference.as<float>(), r->display.as<float>(), r->desc.width, r->desc.height, flags,
                   compare_scale, r->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(rgba, r->display.p, need * 4, hipMemcpyDeviceToHost, r->stream));
  return mrt_renderer_sync(r);
}

int mrt_renderer_display_enqueue(mrt_renderer* r, uint32_t flags, float compare_scale, uint32_t slot) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  if (slot >= MRT_DISPLAY_SLOTS) return fail(MRT_ERR_INVALID, "display slot >= MRT_DISPLAY_SLOTS");
  if (((flags >> 8) & 0xFFu) && !r->reference.p) return fail(MRT_ERR_STATE, "compare mode without a loaded reference");
  const size_t need = (size_t)r->desc.width * r->desc.height * 4;
  auto& ds = r->shown[slot];
  if (ds.queued) HIP_TRY(hipEventSynchronize(ds.done));   // its previous copy may still be landing
  if (ds.floats != need) {
    if (ds.host) HIP_TRY(hipHostFree(ds.host));
    ds.host = nullptr;
    ds.floats = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ds.host), need * 4, hipHostMallocDefault));
    ds.floats = need;
  }
  if (!ds.done) HIP_TRY(hipEventCreateWithFlags(&ds.done, hipEventDisableTiming));
  int rc = exchange_flush(r);
  if (rc) return rc;
  // one device blit buffer: the next blit is queued behind this copy
  if (r->display.bytes < need * 4) HIP_TRY(r->display.alloc(need * 4));
  rc = mrt_display(r->image, r->reference.as<float>(), r->display.as<float>(), r->desc.width, r->desc.height, flags,
                   compare_scale, r->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(ds.host, r->display.p, need * 4, hipMemcpyDeviceToHost, r->stream));
  HIP_TRY(hipEventRecord(ds.done, r->stream));
  ds.queued = true;
  return MRT_OK;
}

int mrt_renderer_display_map(mrt_renderer* r, uint32_t slot, const float** rgba, size_t* count) {
  if (!r || !rgba) return fail(MRT_ERR_INVALID, "null argument");
  if (slot >= MRT_DISPLAY_SLOTS) return fail(MRT_ERR_INVALID, "display slot >= MRT_DISPLAY_SLOTS");
  auto& ds = r->shown[slot];
  if (!ds.queued || ds.floats != (size_t)r->desc.width * r->desc.height * 4)
    return fail(MRT_ERR_STATE, "display slot not enqueued at the current size");
  HIP_TRY(hipEventSynchronize(ds.done));
  *rgba = ds.host;
  if (count) *count = ds.floats;
  return MRT_OK;
}

int mrt_renderer_stats(const mrt_renderer* r, mrt_stats* stats) {
  if (!r || !stats) return fail(MRT_ERR_INVALID, "null argument");
  int rc = finalize_pending(const_cast<mrt_renderer*>(r));
  if (rc) return rc;
  *stats = r->stats;
  const mrt::NoiseSchedule::Counters& c = r->noise->counters();
  stats->noise_ms = c.gen_ms - r->noise_base.gen_ms;
  stats->noise_tables = c.tables - r->noise_base.tables;
  stats->noise_prefetched = c.prefetched - r->noise_base.prefetched;
  return MRT_OK;
}

int mrt_renderer_destroy(mrt_renderer* r) {
  if (!r) return MRT_OK;
  (void)exchange_wait(r);   // bounded: a failed communicator is aborted, not waited for
  (void)finalize_pending(r);
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  for (int i = 0; i < 2; ++i) {   // an overlapped gather may still read the packed tiles
    if (r->x.gather_recorded[i]) (void)hipEventSynchronize(r->x.gather_done[i]);
    if (r->x.pack_done[i]) (void)hipEventDestroy(r->x.pack_done[i]);
    if (r->x.gather_done[i]) (void)hipEventDestroy(r->x.gather_done[i]);
  }
  if (r->x.coll_done) (void)hipEventDestroy(r->x.coll_done);
  if (r->own_image && r->image) (void)hipFree(r->image);
  for (auto& ds : r->shown) {
    if (ds.done) (void)hipEventDestroy(ds.done);
    if (ds.host) (void)hipHostFree(ds.host);
  }
  for (FrameSlot& fs : r->slots) {
    if (fs.acc_done) (void)hipEventDestroy(fs.acc_done);
    if (fs.kernel_done) (void)hipEventDestroy(fs.kernel_done);
    if (fs.own_stream) (void)hipStreamDestroy(fs.stream);
  }
  r->slots.clear();
  for (DrawRecord& d : r->draws) {
    for (hipEvent_t e : d.kernel_events) (void)hipEventDestroy(e);
    if (d.start) (void)hipEventDestroy(d.start);
    if (d.stop) (void)hipEventDestroy(d.stop);
    if (d.cleared) (void)hipEventDestroy(d.cleared);
    if (d.copied) (void)hipEventDestroy(d.copied);
    if (d.host) (void)hipHostFree(d.host);
  }
  r->noise.reset();   // joins the worker; the draws reading its chunks have finished (stream synchronised above)
  if (r->own_stream) (void)hipStreamDestroy(r->stream);
  delete r;
  return MRT_OK;
}

// ---------------------------------------------------------------------------
// multi-GPU exchange (RCCL), SURVEY.md §8(e)
// ---------------------------------------------------------------------------
int mrt_comm_unique_id(void* id, size_t bytes) {
  if (!id || bytes < sizeof(ncclUniqueId)) return fail(MRT_ERR_INVALID, "mrt_comm_unique_id: need 128 bytes");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return MRT_OK;
}

int mrt_comm_create(const void* id, uint32_t nranks, uint32_t rank, int device, mrt_comm** out) {
  if (!id || !out || nranks == 0 || rank >= nranks || device < 0)
    return fail(MRT_ERR_INVALID, "mrt_comm_create: bad argument");
  *out = nullptr;
  std::unique_ptr<mrt_comm> c(new mrt_comm());
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t e = ncclCommInitRank(&c->comm, (int)nranks, u, (int)rank);
  if (e != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    return fail(MRT_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(e));
  }
  c->health->comm = c->comm;
  *out = c.release();
  return MRT_OK;
}

int mrt_comm_destroy(mrt_comm* c) {
  if (!c) return MRT_OK;
  (void)hipSetDevice(c->device);
  {
    std::lock_guard<std::mutex> lk(c->health->m);
    if (c->health->aborted) c->comm = nullptr;   // ncclCommAbort already freed it
    c->health->comm = nullptr;                   // renderers holding the health no longer touch it
  }
  if (c->stream && c->comm) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MRT_OK;
}

int mrt_comm_set_timeout(mrt_comm* c, uint32_t timeout_ms) {
  if (!c) return fail(MRT_ERR_INVALID, "null communicator");
  std::lock_guard<std::mutex> lk(c->health->m);
  c->health->timeout_ms = timeout_ms ? (double)timeout_ms : 120000.0;
  return MRT_OK;
}

int mrt_comm_check(mrt_comm* c) {
  if (!c) return fail(MRT_ERR_INVALID, "null communicator");
  std::lock_guard<std::mutex> lk(c->health->m);
  return comm_check_locked(*c->health);
}

int mrt_debug_comm_fail(mrt_comm* c, uint32_t mode) {
  if (!c || mode > 2) return fail(MRT_ERR_INVALID, "mrt_debug_comm_fail: bad argument");
  std::lock_guard<std::mutex> lk(c->health->m);
  c->health->inject = mode;
  return MRT_OK;
}


int mrt_renderer_exchange(mrt_renderer* r, mrt_comm* c, uint32_t mode) {
  if (!r || !c) return fail(MRT_ERR_INVALID, "mrt_renderer_exchange: null argument");
  const uint32_t kind = mode & 0xFFu;
  const bool overlap = (mode & MRT_EXCHANGE_OVERLAP) != 0;
  if ((kind != MRT_EXCHANGE_GATHER && kind != MRT_EXCHANGE_REDUCE) || (mode & ~0x1FFu) ||
      (overlap && kind != MRT_EXCHANGE_GATHER))
    return fail(MRT_ERR_INVALID, "mrt_renderer_exchange: bad mode");
  if (c->nranks != r->desc.shard_count || c->rank != r->desc.shard_rank)
    return fail(MRT_ERR_INVALID, "mrt_renderer_exchange: the renderer's shard (rank, count) must be the comm's");
  if (c->device != r->scene->device) return fail(MRT_ERR_INVALID, "mrt_renderer_exchange: comm on another device");
  {
    std::lock_guard<std::mutex> lk(c->health->m);
    if (int rc = comm_check_locked(*c->health)) return rc;
  }
  HIP_TRY(hipSetDevice(c->device));
  if (r->x.comm && r->x.comm != c) { int rc = exchange_flush(r); if (rc) return rc; }
  r->x.comm = c;
  int rc = exchange_flush(r);   // the previous overlapped gather's unpack (rank 0)
  if (rc) return rc;
  const uint32_t W = r->desc.width, H = r->desc.height;
  if (c->rank == 0 && c->nranks > 1) r->image_foreign = true;   // other ranks' tiles land in rank 0's image
  if (!r->x.coll_done) HIP_TRY(hipEventCreateWithFlags(&r->x.coll_done, hipEventDisableTiming));
  r->x.health = c->health;
  if (kind == MRT_EXCHANGE_REDUCE) {   // one in-place SUM reduce of the RGBA32F image to rank 0
    NCCL_TRY(ncclReduce(r->image, r->image, (size_t)W * H * 4, ncclFloat, ncclSum, 0, c->comm, r->stream));
    HIP_TRY(hipEventRecord(r->x.coll_done, r->stream));
    r->x.coll_pending = true;
    return MRT_OK;
  }
  rc = exchange_buffers(r, c);
  if (rc) return rc;
  Exchange& x = r->x;
  x.rank = c->rank;
  x.nranks = c->nranks;
  x.width = W;
  x.height = H;
  const int i = overlap ? (int)x.next : 0;
  x.next ^= 1u;
  // the gather two exchanges ago may still be reading packed[i]
  if (x.gather_recorded[i]) HIP_TRY(hipStreamWaitEvent(r->stream, x.gather_done[i], 0));
  HIP_TRY(mrt::fast::launch_tiles_move(reinterpret_cast<const float4*>(r->image), x.packed[i].as<float4>(), W, H,
                                       c->rank, c->nranks, true, r->stream));
  float* recv = c->rank == 0 ? x.gathered.as<float>() : x.packed[i].as<float>();
  if (overlap) {
    // the collective waits for the pack (and, on rank 0, for the previous
    // unpack, which precedes the pack on the renderer's stream) and runs on
    // the communicator's stream while the renderer's next draw proceeds.  A
    // renderer with frame batches on two render streams (a tile share) never
    // makes a render launch wait on its main stream, so there the collective
    // stays on the main stream: a process has 4 hardware queues by default,
    // and a stream sharing one with a render stream would hold that stream's
    // launches behind the collective.
    hipStream_t gs = r->inflight > 1 ? r->stream : c->stream;
    if (gs != r->stream) {
      HIP_TRY(hipEventRecord(x.pack_done[i], r->stream));
      HIP_TRY(hipStreamWaitEvent(gs, x.pack_done[i], 0));
    }
    NCCL_TRY(ncclGather(x.packed[i].p, recv, x.slab_floats, ncclFloat, 0, c->comm, gs));
    HIP_TRY(hipEventRecord(x.gather_done[i], gs));
    HIP_TRY(hipEventRecord(x.coll_done, gs));
    x.coll_pending = true;
    x.gather_recorded[i] = true;
    x.pending = i;
    return MRT_OK;
  }
  NCCL_TRY(ncclGather(x.packed[i].p, recv, x.slab_floats, ncclFloat, 0, c->comm, r->stream));
  HIP_TRY(hipEventRecord(x.gather_done[i], r->stream));
  HIP_TRY(hipEventRecord(x.coll_done, r->stream));
  x.coll_pending = true;
  x.gather_recorded[i] = true;
  return exchange_unpack(r, i);
}

// Test entry (include/mrt.h): rank 0's half of the gather exchange without
// a communicator — `gathered` (host, nranks slabs of slab_floats packed
// floats, rank k's at k * slab_floats, as ncclGather delivers them) is copied
// into the receive buffer and unpacked by the same exchange_unpack the RCCL
// path runs, so slabs k >= 1 of an N-rank gather are exercised on one device.
int mrt_debug_exchange_unpack(mrt_renderer* r, uint32_t nranks, const float* gathered, size_t floats) {
  if (!r || !gathered) return fail(MRT_ERR_INVALID, "mrt_debug_exchange_unpack: null argument");
  if (nranks < 2 || r->desc.shard_count != nranks || r->desc.shard_rank != 0)
    return fail(MRT_ERR_INVALID, "mrt_debug_exchange_unpack: the renderer must be rank 0 of nranks >= 2");
  HIP_TRY(hipSetDevice(r->scene->device));
  int rc = exchange_flush(r);
  if (rc) return rc;
  mrt_comm c;   // shape only: exchange_buffers reads rank / nranks
  c.nranks = nranks;
  c.rank = 0;
  c.device = r->scene->device;
  rc = exchange_buffers(r, &c);
  if (rc) return rc;
  Exchange& x = r->x;
  if (floats != x.slab_floats * nranks) return fail(MRT_ERR_INVALID, "mrt_debug_exchange_unpack: need nranks * slab floats");
  x.rank = 0;
  x.nranks = nranks;
  x.width = r->desc.width;
  x.height = r->desc.height;
  r->image_foreign = true;
  HIP_TRY(hipMemcpyAsync(x.gathered.p, gathered, floats * 4, hipMemcpyHostToDevice, r->stream));
  HIP_TRY(hipEventRecord(x.gather_done[0], r->stream));   // "the gather is done"
  x.gather_recorded[0] = true;
  rc = exchange_unpack(r, 0);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(r->stream));
  return MRT_OK;
}

int mrt_renderer_exchange_flush(mrt_renderer* r) {
  if (!r) return fail(MRT_ERR_INVALID, "null renderer");
  int rc = exchange_flush(r);
  if (rc) return rc;
  return exchange_wait(r);   // the collective done on the device, or the communicator aborted
}

int mrt_renderer_tiles_read(mrt_renderer* r, float* host, size_t floats) {
  if (!r || !host) return fail(MRT_ERR_INVALID, "null argument");
  uint64_t n = 0;
  int rc = mrt_tiles_packed_floats(r->desc.width, r->desc.height, r->desc.shard_rank, r->desc.shard_count, &n);
  if (rc) return rc;
  if (floats < n) return fail(MRT_ERR_INVALID, "mrt_renderer_tiles_read: buffer too small");
  rc = exchange_flush(r);
  if (rc) return rc;
  if (r->x.staging.bytes < n * 4) HIP_TRY(r->x.staging.alloc(n * 4));
  HIP_TRY(mrt::fast::launch_tiles_move(reinterpret_cast<const float4*>(r->image), r->x.staging.as<float4>(),
                                       r->desc.width, r->desc.height, r->desc.shard_rank, r->desc.shard_count, true,
                                       r->stream));
  HIP_TRY(hipMemcpyAsync(host, r->x.staging.p, n * 4, hipMemcpyDeviceToHost, r->stream));
  return mrt_renderer_sync(r);
}

int mrt_renderer_tiles_write(mrt_renderer* r, uint32_t shard_rank, const float* host, size_t floats) {
  if (!r || !host) return fail(MRT_ERR_INVALID, "null argument");
  if (shard_rank >= r->desc.shard_count) return fail(MRT_ERR_INVALID, "mrt_renderer_tiles_write: shard_rank >= shard_count");
  uint64_t n = 0;
  int rc = mrt_tiles_packed_floats(r->desc.width, r->desc.height, shard_rank, r->desc.shard_count, &n);
  if (rc) return rc;
  if (floats < n) return fail(MRT_ERR_INVALID, "mrt_renderer_tiles_write: buffer too small");
  rc = exchange_flush(r);
  if (rc) return rc;
  r->image_foreign = true;
  HIP_TRY(hipStreamSynchronize(r->stream));   // the staging buffer may still feed a queued copy
  if (r->x.staging.bytes < n * 4) HIP_TRY(r->x.staging.alloc(n * 4));
  HIP_TRY(hipMemcpyAsync(r->x.staging.p, host, n * 4, hipMemcpyHostToDevice, r->stream));
  HIP_TRY(mrt::fast::launch_tiles_move(r->x.staging.as<float4>(), reinterpret_cast<float4*>(r->image), r->desc.width,
                                       r->desc.height, shard_rank, r->desc.shard_count, false, r->stream));
  return mrt_renderer_sync(r);
}

}  // extern "C"

