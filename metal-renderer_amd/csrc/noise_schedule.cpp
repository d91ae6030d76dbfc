// noise_schedule.cpp — see noise_schedule.h.
#include "noise_schedule.h"

#include <algorithm>
#include <chrono>

#include "noise.h"

namespace mrt {

namespace {
constexpr size_t kChunkBytes = (size_t)NoiseSchedule::kChunkTables * kNoiseFloats * sizeof(float);
}

NoiseSchedule::~NoiseSchedule() {
  {
    std::lock_guard<std::mutex> lk(m_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
  if (stream_) (void)hipStreamSynchronize(stream_);   // pending uploads read the pinned stages
  for (auto& c : chunks_) {
    if (c->dev) (void)hipFree(c->dev);
    if (c->ready) (void)hipEventDestroy(c->ready);
    if (c->last_use) (void)hipEventDestroy(c->last_use);
  }
  for (Stage& s : stage_) {
    if (s.host) (void)hipHostFree(s.host);
    if (s.copied) (void)hipEventDestroy(s.copied);
  }
  if (stream_) (void)hipStreamDestroy(stream_);
}

hipError_t NoiseSchedule::init() {
  if (inited_) return hipSuccess;
  // the uploads' own stream: a render stream waits for a chunk's `ready`
  // event only, never for the copy queue as a whole
  hipError_t e = hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking);
  for (Stage& s : stage_) {
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&s.host), kChunkBytes, hipHostMallocDefault);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.copied, hipEventDisableTiming);
  }
  if (e != hipSuccess) return e;
  worker_ = std::thread([this] { worker_main(); });
  inited_ = true;
  return hipSuccess;
}

void NoiseSchedule::generate(int64_t k, float* out) {
  const int64_t f0 = first_frame(k);
  const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=] {
      for (int64_t j = t; j < kChunkTables; j += nt) {
        const int64_t f = f0 + j;   // frames < 0: the initial table (noise.h); ANIMATE_NOISE 0: always
        make_noise_table(seed_, f < 0 || static_ ? -1 : f, out + (size_t)j * kNoiseFloats);
      }
    });
  for (auto& x : th) x.join();
}

void NoiseSchedule::worker_main() {
  std::unique_lock<std::mutex> lk(m_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || job_ == kQueued; });
    if (stop_) return;
    job_ = kRunning;
    const int64_t k = job_chunk_;
    Stage& s = stage_[job_stage_];
    const bool wait_copy = s.copy_recorded;
    lk.unlock();
    // the stage's previous upload (two jobs back) must have left it: a host
    // wait on the copy engine, on this thread only
    if (wait_copy) (void)hipEventSynchronize(s.copied);
    const auto t0 = std::chrono::steady_clock::now();
    generate(k, s.host);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    lk.lock();
    job_ms_ = ms;
    job_ = kDone;
    cv_.notify_all();
  }
}

NoiseSchedule::Chunk* NoiseSchedule::find(int64_t k) {
  for (auto& c : chunks_)
    if (c->index == k && c->uploaded) return c.get();
  return nullptr;
}

hipError_t NoiseSchedule::slot_for(int64_t k, uint64_t seq, Chunk** out, int64_t keep_lo, int64_t keep_hi) {
  (void)k;
  Chunk* best = nullptr;
  for (auto& up : chunks_) {
    Chunk* c = up.get();
    if (!c->uploaded) { best = c; break; }
    if (seq && c->pin == seq) continue;   // read by the draw being enqueued
    if (c->index >= keep_lo && c->index <= keep_hi) continue;   // about to be read by the caller's draw
    if (c->used && hipEventQuery(c->last_use) != hipSuccess) continue;   // a queued draw still reads it
    if (hipEventQuery(c->ready) != hipSuccess) continue;                 // its upload is still landing
    if (!best || c->lru < best->lru) best = c;
  }
  if (!best) {
    auto c = std::make_unique<Chunk>();
    hipError_t e = hipMalloc(&c->dev, kChunkBytes);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->last_use, hipEventDisableTiming);
    if (e != hipSuccess) {
      if (c->dev) (void)hipFree(c->dev);
      if (c->ready) (void)hipEventDestroy(c->ready);
      return e;
    }
    best = c.get();
    chunks_.push_back(std::move(c));
  }
  best->index = -1;
  best->uploaded = false;
  best->used = false;
  best->waited_streams = 0;
  *out = best;
  return hipSuccess;
}

hipError_t NoiseSchedule::upload_done_job(Chunk** out, uint64_t seq, int64_t keep_lo, int64_t keep_hi) {
  Chunk* c = nullptr;
  hipError_t e = slot_for(job_chunk_, seq, &c, keep_lo, keep_hi);
  if (e != hipSuccess) return e;
  Stage& s = stage_[job_stage_];
  e = hipMemcpyAsync(c->dev, s.host, kChunkBytes, hipMemcpyHostToDevice, stream_);
  if (e == hipSuccess) e = hipEventRecord(s.copied, stream_);
  if (e == hipSuccess) e = hipEventRecord(c->ready, stream_);
  if (e != hipSuccess) return e;
  s.copy_recorded = true;
  c->index = job_chunk_;
  c->uploaded = true;
  c->lru = ++tick_;
  c_.gen_ms += job_ms_;
  c_.tables += (uint64_t)kChunkTables;
  c_.uploads += 1;
  if (job_prefetch_) c_.prefetched += 1;
  job_ = kIdle;
  *out = c;
  return hipSuccess;
}

hipError_t NoiseSchedule::poll(int64_t keep_lo, int64_t keep_hi) {
  if (!inited_) return hipSuccess;
  std::lock_guard<std::mutex> lk(m_);
  if (job_ != kDone) return hipSuccess;
  Chunk* c = nullptr;
  return upload_done_job(&c, 0, keep_lo, keep_hi);
}

void NoiseSchedule::prefetch(int64_t k) {
  if (k < 0 || !inited_ || find(k)) return;
  {
    std::lock_guard<std::mutex> lk(m_);
    if (job_ != kIdle) return;   // the worker holds another chunk (it is uploaded at the next poll)
    job_chunk_ = k;
    job_stage_ = (int)(jobs_++ & 1u);
    job_prefetch_ = true;
    job_ = kQueued;
  }
  cv_.notify_all();
}

hipError_t NoiseSchedule::acquire(int64_t k, uint64_t seq, Chunk** out) {
  hipError_t e = init();
  if (e != hipSuccess) return e;
  if (Chunk* c = find(k)) {
    c->lru = ++tick_;
    c->pin = seq;
    *out = c;
    return hipSuccess;
  }
  std::unique_lock<std::mutex> lk(m_);
  bool waited = false;
  for (;;) {
    if (job_ == kDone) {
      const bool mine = job_chunk_ == k;
      Chunk* c = nullptr;
      e = upload_done_job(&c, seq);
      if (e != hipSuccess) return e;
      if (mine) {
        if (waited) c_.waits += 1;
        c->pin = seq;
        *out = c;
        return hipSuccess;
      }
      continue;   // a prefetch of another chunk: uploaded and cached, now ours
    }
    if (job_ == kIdle) {
      job_chunk_ = k;
      job_stage_ = (int)(jobs_++ & 1u);
      job_prefetch_ = false;
      job_ = kQueued;
      cv_.notify_all();
    }
    waited = true;
    cv_.wait(lk, [&] { return job_ == kDone; });
  }
}

}  // namespace mrt
