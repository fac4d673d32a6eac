// shm_rows.hpp -- node-wide transport of the sharded sums (host-only C++, POSIX; no HIP).
//
// One process per GPU on one node.  Every per-pass / per-iteration sum of the engine
// is a fixed reduction tree whose leaves are "supers" (32768 grid-sorted source positions; rank r
// owns supers [S r / N, S (r + 1) / N)).  Instead of an RCCL all-gather per BFGS pass, every rank's
// GPU writes its super partials straight into ONE POSIX shared-memory segment mapped (and
// hipHostRegister'ed) by every rank, at their GLOBAL super index, and every rank's host waits for
// all rows and takes the same fixed-order total -- bitwise the single-GPU result, no collective on
// the pass path.
//
// Segment layout (bytes):
//   [0, 4096)                  header (magic, geometry, creator's ready flag, attach counter)
//   [4096, 4096 + 64 x 64)     gather flags, one 64-byte line per rank
//   rows   2 x max_sup x 256   pass rows: 32 words per super, word (stamp << 32 | 32-bit half);
//                              the pass with row stamp s writes buffer s & 1
//   gath   2 x max_sup x 640   generic gathers (<= 80 doubles per super); gather g uses buffer g & 1
//   ipc    64 x 128            r05: per rank a 64-byte hipIpcMemHandle_t of its xGMI row-exchange buffer
//                              and a 64-bit publication flag (mgicp_comm_attach_xgmi)
//
// Why two buffers make reuse safe: a rank writes pass s + 2 into the buffer of pass s only after
// its host saw every row of pass s + 1, i.e. after every rank's host published s + 1's command,
// i.e. after every rank's host finished reading pass s.  The same argument holds for gathers.
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>

namespace mgicp {
namespace shm {

constexpr uint64_t kMagic = 0x31574f5250434947ull;  // "GICPROW1"
constexpr int kMaxRanks = 64;
constexpr size_t kHeader = 4096;
constexpr size_t kFlagLine = 64;
constexpr size_t kRowWords = 32;   // 16 doubles as stamped halves
constexpr int kGathVals = 80;      // largest nv of a generic gather (Gauss-Newton moments)
constexpr size_t kIpcLine = 128;   // r05: IPC handle (64 B) + flag (8 B) per rank

struct Header {
  uint64_t magic;
  uint64_t bytes;
  uint64_t max_sup;
  uint32_t nranks;
  uint32_t pad;
  std::atomic<uint32_t> ready;     // creator: geometry written
  std::atomic<uint32_t> attached;  // ranks that mapped the segment
};

inline size_t segment_bytes(long long max_sup) {
  return kHeader + kMaxRanks * kFlagLine + 2 * static_cast<size_t>(max_sup) * kRowWords * 8 +
         2 * static_cast<size_t>(max_sup) * kGathVals * 8 + kMaxRanks * kIpcLine;
}

struct Segment {
  void* base = nullptr;
  size_t bytes = 0;
  long long max_sup = 0;
  int nranks = 1, rank = 0;
  Header* hdr() const { return static_cast<Header*>(base); }
  std::atomic<uint64_t>* flag(int r) const {
    return reinterpret_cast<std::atomic<uint64_t>*>(static_cast<char*>(base) + kHeader + r * kFlagLine);
  }
  // pass rows, parity buffer p (host view)
  uint64_t* rows(int p) const {
    return reinterpret_cast<uint64_t*>(static_cast<char*>(base) + kHeader + kMaxRanks * kFlagLine) +
           static_cast<size_t>(p) * max_sup * kRowWords;
  }
  size_t rows_offset_bytes() const { return kHeader + kMaxRanks * kFlagLine; }
  size_t rows_stride_words() const { return static_cast<size_t>(max_sup) * kRowWords; }
  // r05: rank r's IPC handle slot (64 bytes) and its publication flag
  unsigned char* ipc_handle(int r) const {
    return static_cast<unsigned char*>(base) + kHeader + kMaxRanks * kFlagLine +
           2 * static_cast<size_t>(max_sup) * kRowWords * 8 + 2 * static_cast<size_t>(max_sup) * kGathVals * 8 +
           static_cast<size_t>(r) * kIpcLine;
  }
  std::atomic<uint64_t>* ipc_flag(int r) const {
    return reinterpret_cast<std::atomic<uint64_t>*>(ipc_handle(r) + 64);
  }
  double* gath(int p) const {
    return reinterpret_cast<double*>(static_cast<char*>(base) + kHeader + kMaxRanks * kFlagLine +
                                     2 * static_cast<size_t>(max_sup) * kRowWords * 8) +
           static_cast<size_t>(p) * max_sup * kGathVals;
  }
};

inline double elapsed_s(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Map the segment `name` (every rank passes the same name, nranks and max_sup) and wait until all
// nranks ranks have mapped it; the name is unlinked afterwards (the mappings keep the segment), so
// nothing is left in /dev/shm even if a rank dies later.  The creator (first shm_open with O_EXCL)
// sizes the object -- fresh pages are zero, so no stale stamp can match -- and writes the geometry.
inline bool attach(Segment& s, const char* name, int nranks, int rank, long long max_sup, double timeout_s,
                   std::string& err) {
  if (!name || name[0] != '/' || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks || max_sup < 1) {
    err = "shm attach: invalid arguments (name must start with '/', 1 <= nranks <= 64)";
    return false;
  }
  const size_t bytes = segment_bytes(max_sup);
  const auto t0 = std::chrono::steady_clock::now();
  bool creator = false;
  int fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd >= 0) {
    creator = true;
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      err = std::string("shm attach: ftruncate: ") + std::strerror(errno);
      close(fd);
      shm_unlink(name);
      return false;
    }
  } else if (errno == EEXIST) {
    for (;;) {  // the creator may not have sized it yet
      fd = shm_open(name, O_RDWR, 0600);
      struct stat st;
      if (fd >= 0 && fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) == bytes) break;
      if (fd >= 0 && fstat(fd, &st) == 0 && st.st_size != 0 && static_cast<size_t>(st.st_size) != bytes) {
        err = "shm attach: segment exists with another geometry (max_source_points differs between ranks?)";
        close(fd);
        return false;
      }
      if (fd >= 0) close(fd);
      if (elapsed_s(t0) > timeout_s) {
        err = "shm attach: timed out waiting for the creator to size the segment";
        return false;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  } else {
    err = std::string("shm attach: shm_open: ") + std::strerror(errno);
    return false;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    err = std::string("shm attach: mmap: ") + std::strerror(errno);
    if (creator) shm_unlink(name);
    return false;
  }
  s.base = p;
  s.bytes = bytes;
  s.max_sup = max_sup;
  s.nranks = nranks;
  s.rank = rank;
  Header* h = s.hdr();
  if (creator) {
    h->magic = kMagic;
    h->bytes = bytes;
    h->max_sup = static_cast<uint64_t>(max_sup);
    h->nranks = static_cast<uint32_t>(nranks);
    h->ready.store(1, std::memory_order_release);
  } else {
    while (h->ready.load(std::memory_order_acquire) != 1) {
      if (elapsed_s(t0) > timeout_s) {
        err = "shm attach: timed out waiting for the creator's header";
        munmap(p, bytes);
        s.base = nullptr;
        return false;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    if (h->magic != kMagic || h->bytes != bytes || h->max_sup != static_cast<uint64_t>(max_sup) ||
        h->nranks != static_cast<uint32_t>(nranks)) {
      err = "shm attach: segment geometry differs between ranks";
      munmap(p, bytes);
      s.base = nullptr;
      return false;
    }
  }
  const uint32_t joined = h->attached.fetch_add(1, std::memory_order_acq_rel) + 1;
  while (joined < static_cast<uint32_t>(nranks) && h->attached.load(std::memory_order_acquire) < static_cast<uint32_t>(nranks)) {
    if (elapsed_s(t0) > timeout_s) {
      err = "shm attach: timed out waiting for every rank to map the segment";
      munmap(p, bytes);
      s.base = nullptr;
      shm_unlink(name);  // the job is broken: leave nothing in /dev/shm
      return false;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  shm_unlink(name);  // every rank holds a mapping now; ENOENT after the first unlink is fine
  return true;
}

inline void detach(Segment& s) {
  if (s.base) munmap(s.base, s.bytes);
  s.base = nullptr;
  s.bytes = 0;
}

// A stamped row is complete when all 32 words carry `stamp` in their high halves.
inline bool row_complete(const uint64_t* row, uint32_t stamp) {
  for (size_t w = 0; w < kRowWords; ++w)
    if (static_cast<uint32_t>(__atomic_load_n(row + w, __ATOMIC_ACQUIRE) >> 32) != stamp) return false;
  return true;
}

// The 16 doubles of a complete row.
inline void row_decode(const uint64_t* row, double out[16]) {
  for (int v = 0; v < 16; ++v) {
    const uint64_t lo = __atomic_load_n(row + 2 * v, __ATOMIC_ACQUIRE) & 0xffffffffull;
    const uint64_t hi = __atomic_load_n(row + 2 * v + 1, __ATOMIC_ACQUIRE) & 0xffffffffull;
    const uint64_t bits = (hi << 32) | lo;
    std::memcpy(&out[v], &bits, sizeof(double));
  }
}

// The fixed-order total over nsup supers of nv values (rows[s * nv + v]) exactly as the device's
// wave_total computes it on one wave: lane l sums supers l, l + 64, ... in order from 0.0, then the
// shuffle tree lanes[i] += lanes[i + off] for off = 32 ... 1; lane 0 holds the total.
inline void fixed_total(const double* rows, long long nsup, int nv, double* out) {
  for (int v = 0; v < nv; ++v) {
    double lanes[64];
    for (int l = 0; l < 64; ++l) {
      double a = 0.0;
      for (long long sg = l; sg < nsup; sg += 64) a += rows[static_cast<size_t>(sg) * nv + v];
      lanes[l] = a;
    }
    for (int off = 32; off > 0; off >>= 1)
      for (int i = 0; i < off; ++i) lanes[i] = lanes[i] + lanes[i + off];
    out[v] = lanes[0];
  }
}

// Generic gather, step 2: after this rank's rows of gather g are in gath(g & 1) (caller), publish g
// and wait until every rank has published g.  false on timeout.
inline bool gather_publish_wait(const Segment& s, uint64_t g, double timeout_s) {
  s.flag(s.rank)->store(g, std::memory_order_release);
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < s.nranks; ++r) {
    for (unsigned spins = 0; s.flag(r)->load(std::memory_order_acquire) < g; ++spins) {
      if ((spins & 1023u) == 1023u && elapsed_s(t0) > timeout_s) return false;
    }
  }
  return true;
}

}  // namespace shm
}  // namespace mgicp
