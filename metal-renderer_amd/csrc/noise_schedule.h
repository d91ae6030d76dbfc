// noise_schedule.h — the per-frame noise tables of a renderer, generated
// ahead of the frames that read them and uploaded without a host wait on the
// GPU.
//
// The reference regenerates one 64x64 float4 table per frame on the CPU in
// updateSharedData, right before the frame's command buffer is committed
// (renderer/Renderer.mm:472-498), into the slot of that frame's in-flight
// buffer (MaxBuffersInFlight = 3, :16, :593-600).  A frame's kernels read
// T_f, T_{f-1} and T_{f-2} (noise.h).  Here the tables live in device CHUNKS:
// chunk k holds the tables of frames [64k - 2, 64k + 64) (frames < 0 = the
// initial table), so any launch whose frames lie inside one chunk addresses
// all three tables of each of its frames contiguously.  A chunk is generated
// on the host (mt19937_64, noise.h) into pinned staging, copied with
// hipMemcpyAsync on the schedule's own stream and published by an event that
// render streams wait on (hipStreamWaitEvent, a device-side wait).  A worker
// thread generates chunk k + 1 while the frames of chunk k render, so a
// progressive render that draws one frame per call (the reference's
// drawInMTKView: cadence) never waits for noise and never drains a stream.
// Chunks stay cached on the device (4.2 MB each) and a buffer is reused only
// once the events of its last readers and its upload have completed
// (hipEventQuery: no host wait) — a reset back to frame 0 finds chunk 0
// still resident.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace mrt {

class NoiseSchedule {
 public:
  static constexpr int64_t kChunkFrames = 64;          // = kMaxBatch: an aligned 64-frame batch is one chunk
  static constexpr int64_t kChunkTables = kChunkFrames + 2;

  struct Chunk {
    int64_t index = -1;                   // chunk k: frames [64k - 2, 64k + 64); -1 = empty
    void* dev = nullptr;                  // kChunkTables x kNoiseFloats floats
    hipEvent_t ready = nullptr;           // upload complete (recorded on the schedule's stream)
    hipEvent_t last_use = nullptr;        // recorded on the renderer's main stream after each draw that read it
    bool uploaded = false, used = false;
    uint32_t waited_streams = 0;          // render slots whose stream already waits on `ready` (bit per slot)
    uint64_t lru = 0;
    uint64_t pin = 0;                     // draw sequence number that holds it (not reusable during that draw)
  };

  struct Counters {
    double gen_ms = 0.0;           // host wall time generating tables (worker or caller)
    uint64_t tables = 0;           // tables generated
    uint64_t waits = 0;            // acquisitions that waited for a chunk's generation (host CPU work only)
    uint64_t prefetched = 0;       // chunks generated ahead by the worker and found ready when needed
    uint64_t uploads = 0;          // chunk uploads enqueued
  };

  NoiseSchedule(uint64_t seed, bool static_noise) : seed_(seed), static_(static_noise) {}
  ~NoiseSchedule();
  NoiseSchedule(const NoiseSchedule&) = delete;
  NoiseSchedule& operator=(const NoiseSchedule&) = delete;

  static int64_t chunk_of(int64_t frame) { return frame / kChunkFrames; }
  static int64_t first_frame(int64_t chunk) { return chunk * kChunkFrames - 2; }

  // The device chunk k, uploaded (or its upload enqueued) and pinned for draw
  // `seq`.  Blocks only while the host generates the chunk (if the worker has
  // not already); never waits for the GPU.
  hipError_t acquire(int64_t k, uint64_t seq, Chunk** out);
  // Ask the worker to generate chunk k ahead (no-op if it is resident or
  // being generated, or the worker is busy with another chunk).
  void prefetch(int64_t k);
  // Upload a chunk the worker finished since the last call (async).  Chunks
  // [keep_lo, keep_hi] (the ones the caller's draw is about to read) are not
  // evicted to make room for it.
  hipError_t poll(int64_t keep_lo = -1, int64_t keep_hi = -2);
  // Create the upload stream, staging buffers and worker on the current
  // device (the renderer calls it after hipSetDevice; acquire() otherwise).
  hipError_t init();
  const Counters& counters() const { return c_; }

 private:
  enum JobState { kIdle, kQueued, kRunning, kDone };
  struct Stage {
    float* host = nullptr;                // pinned, kChunkTables x kNoiseFloats
    hipEvent_t copied = nullptr;          // the last upload from it
    bool copy_recorded = false;
  };
  void worker_main();
  void generate(int64_t k, float* out);   // kChunkTables tables on up to 8 host threads
  Chunk* find(int64_t k);
  hipError_t slot_for(int64_t k, uint64_t seq, Chunk** out, int64_t keep_lo = -1, int64_t keep_hi = -2);
  // job_ is kDone: copy its stage into a chunk (lock held)
  hipError_t upload_done_job(Chunk** out, uint64_t seq, int64_t keep_lo = -1, int64_t keep_hi = -2);

  uint64_t seed_;
  bool static_;
  bool inited_ = false;
  hipStream_t stream_ = nullptr;
  std::vector<std::unique_ptr<Chunk>> chunks_;   // stable addresses: a draw holds Chunk pointers
  uint64_t tick_ = 0;
  Stage stage_[2];
  // worker: one job at a time (chunk job_chunk_ into stage_[job_stage_])
  std::thread worker_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
  JobState job_ = kIdle;
  int64_t job_chunk_ = -1;
  int job_stage_ = 0;
  bool job_prefetch_ = false;
  double job_ms_ = 0.0;
  uint32_t jobs_ = 0;
  Counters c_;
};

}  // namespace mrt
