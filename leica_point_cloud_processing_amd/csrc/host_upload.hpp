// host_upload.hpp -- host side of the cloud upload: a small persistent worker pool and a
// pipelined, pinned-staging copy of strided xyz records into HBM.
//
// A PointXYZRGB record is 32 bytes of which the engine needs 12 (x, y, z).  hipMemcpy from
// pageable memory moves all 32 through the runtime's own bounce buffer (13.5 GB/s measured for
// 2 x 5M records, profiles/r01/bench_C4_final.json ms_upload).  Here the host workers pack xyz
// straight into a ring of pinned slots while the DMA engine drains the previous slots, so PCIe
// carries 12 B per point and packing overlaps the transfer.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mgicp {

class HostPool {
 public:
  explicit HostPool(int nthreads) {
    for (int t = 1; t < nthreads; ++t) th_.emplace_back([this] { worker(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return static_cast<int>(th_.size()) + 1; }

  // f(i) for every i in [0, n), spread over the workers and the calling thread
  void parallel_for(size_t n, const std::function<void(size_t)>& f) {
    if (th_.empty() || n <= 1) {
      for (size_t i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      n_ = n;
      next_.store(0);
      active_ = th_.size();
      ++gen_;
    }
    cv_.notify_all();
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
    job_ = nullptr;
  }

 private:
  void worker() {
    unsigned long long seen = 0;
    for (;;) {
      const std::function<void(size_t)>* job;
      size_t n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        job = job_;
        n = n_;
      }
      for (size_t i; (i = next_.fetch_add(1)) < n;) (*job)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_one();
    }
  }

  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  size_t active_ = 0;
  unsigned long long gen_ = 0;
  bool stop_ = false;
};

// Ring of pinned host slots, each with the event of its last DMA.
struct PinnedRing {
  static constexpr int kSlots = 4;
  static constexpr size_t kSlotBytes = size_t(8) << 20;
  unsigned char* buf[kSlots] = {};
  hipEvent_t ev[kSlots] = {};
  bool ready = false;

  hipError_t init() {
    if (ready) return hipSuccess;
    for (int i = 0; i < kSlots; ++i) {
      hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&buf[i]), kSlotBytes, hipHostMallocDefault);
      if (e != hipSuccess) return e;
      e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    ready = true;
    return hipSuccess;
  }
  void release() {
    for (int i = 0; i < kSlots; ++i) {
      if (ev[i]) (void)hipEventSynchronize(ev[i]), (void)hipEventDestroy(ev[i]);
      if (buf[i]) (void)hipHostFree(buf[i]);
      ev[i] = nullptr;
      buf[i] = nullptr;
    }
    ready = false;
  }
};

// Process-wide packing workers and pinned ring, shared by every context of the process and
// created once (the pinned allocation and the threads cost milliseconds).  Never destroyed:
// tearing them down from a static destructor would race the HIP runtime's own teardown.
struct HostUploader {
  std::mutex mu;  // one upload at a time owns the ring
  HostPool* pool = nullptr;
  PinnedRing ring;
  static HostUploader& instance() {
    static HostUploader* u = new HostUploader();
    return *u;
  }
  hipError_t init(int threads) {
    std::lock_guard<std::mutex> lk(mu);
    if (!pool) pool = new HostPool(threads);
    return ring.init();
  }
};

// Copy the xyz of n strided host records into d_xyz (3n packed floats) on `s`.  Returns after
// the last DMA is queued; the caller synchronises the stream.
inline hipError_t upload_xyz(HostPool& pool, PinnedRing& ring, const void* host, size_t n,
                             size_t stride, float* d_xyz, hipStream_t s) {
  hipError_t e = ring.init();
  if (e != hipSuccess) return e;
  const size_t per = PinnedRing::kSlotBytes / 12;  // points per slot
  const unsigned char* src = static_cast<const unsigned char*>(host);
  const size_t parts = static_cast<size_t>(pool.size()) * 4;
  for (size_t c = 0, k = 0; c < n; c += per, ++k) {
    const int slot = static_cast<int>(k % PinnedRing::kSlots);
    // the slot's previous DMA (this upload's, or an earlier one's on any stream) has drained;
    // an event never recorded completes at once
    e = hipEventSynchronize(ring.ev[slot]);
    if (e != hipSuccess) return e;
    const size_t cnt = std::min(per, n - c);
    float* dst = reinterpret_cast<float*>(ring.buf[slot]);
    const unsigned char* base = src + c * stride;
    pool.parallel_for(parts, [&](size_t part) {
      const size_t i0 = cnt * part / parts, i1 = cnt * (part + 1) / parts;
      if (stride == 12) {
        std::memcpy(dst + 3 * i0, base + 12 * i0, 12 * (i1 - i0));
        return;
      }
      for (size_t i = i0; i < i1; ++i) std::memcpy(dst + 3 * i, base + i * stride, 12);
    });
    e = hipMemcpyAsync(d_xyz + 3 * c, dst, cnt * 12, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ring.ev[slot], s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Copy one 4-byte field (at byte `offset` of each strided host record) of n records into d_out
// on `s`, through the same pinned ring (the colour word of PointXYZRGB for VoxelGrid).
inline hipError_t upload_u32_field(HostPool& pool, PinnedRing& ring, const void* host, size_t n,
                                   size_t stride, size_t offset, uint32_t* d_out, hipStream_t s) {
  hipError_t e = ring.init();
  if (e != hipSuccess) return e;
  const size_t per = PinnedRing::kSlotBytes / 4;
  const unsigned char* src = static_cast<const unsigned char*>(host) + offset;
  const size_t parts = static_cast<size_t>(pool.size()) * 4;
  for (size_t c = 0, k = 0; c < n; c += per, ++k) {
    const int slot = static_cast<int>(k % PinnedRing::kSlots);
    e = hipEventSynchronize(ring.ev[slot]);
    if (e != hipSuccess) return e;
    const size_t cnt = std::min(per, n - c);
    uint32_t* dst = reinterpret_cast<uint32_t*>(ring.buf[slot]);
    const unsigned char* base = src + c * stride;
    pool.parallel_for(parts, [&](size_t part) {
      const size_t i0 = cnt * part / parts, i1 = cnt * (part + 1) / parts;
      for (size_t i = i0; i < i1; ++i) std::memcpy(dst + i, base + i * stride, 4);
    });
    e = hipMemcpyAsync(d_out + c, dst, cnt * 4, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ring.ev[slot], s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace mgicp
