// Test harness (CPU only, g++): drives the node-wide row transport of libmgicp.so
// (leica_point_cloud_processing_amd/csrc/shm_rows.hpp) from several processes without a GPU.  Each
// process plays one rank: it writes its supers' stamped rows the way fdf_server_kernel's finishing
// waves do (32 words per super, (stamp << 32) | 32-bit half, parity buffer stamp & 1) and waits for
// every rank's rows / gathers exactly as mgicp_engine.hip's wait_rows / combine_to_host do.
#include "../leica_point_cloud_processing_amd/csrc/shm_rows.hpp"

#include <cstring>
#include <vector>

using namespace mgicp;

static shm::Segment g_seg;
static std::string g_err;

extern "C" {

int h_attach(const char* name, int nranks, int rank, long long max_sup, double timeout_s) {
  return shm::attach(g_seg, name, nranks, rank, max_sup, timeout_s, g_err) ? 0 : -1;
}

const char* h_error() { return g_err.c_str(); }

void h_detach() { shm::detach(g_seg); }

// rows of supers [first, first + n) of the pass stamped `stamp` (vals: n x 16 doubles)
void h_write_rows(unsigned int stamp, long long first, long long n, const double* vals) {
  uint64_t* buf = g_seg.rows(static_cast<int>(stamp & 1u));
  for (long long s = 0; s < n; ++s) {
    uint64_t* row = buf + static_cast<size_t>(first + s) * shm::kRowWords;
    for (int v = 0; v < 16; ++v) {
      uint64_t bits;
      std::memcpy(&bits, &vals[s * 16 + v], sizeof(bits));
      const uint64_t hi = static_cast<uint64_t>(stamp) << 32;
      __atomic_store_n(row + 2 * v, hi | (bits & 0xffffffffull), __ATOMIC_RELEASE);
      __atomic_store_n(row + 2 * v + 1, hi | (bits >> 32), __ATOMIC_RELEASE);
    }
  }
}

// every row of the pass stamped `stamp`, then the fixed-order total; -1 on timeout
int h_wait_total(unsigned int stamp, long long ntot, double* out16, double timeout_s) {
  const uint64_t* buf = g_seg.rows(static_cast<int>(stamp & 1u));
  std::vector<double> rows(static_cast<size_t>(ntot) * 16);
  const auto t0 = std::chrono::steady_clock::now();
  for (long long r = 0; r < ntot; ++r) {
    const uint64_t* row = buf + static_cast<size_t>(r) * shm::kRowWords;
    while (!shm::row_complete(row, stamp))
      if (shm::elapsed_s(t0) > timeout_s) return -1;
    shm::row_decode(row, &rows[static_cast<size_t>(r) * 16]);
  }
  shm::fixed_total(rows.data(), ntot, 16, out16);
  return 0;
}

// generic gather g: this rank's nloc supers (nv values each) at their global rows, publish, wait,
// fixed-order total over ntot supers
int h_gather(unsigned long long g, long long first, long long nloc, long long ntot, int nv, const double* mine,
             double* out, double timeout_s) {
  double* buf = g_seg.gath(static_cast<int>(g & 1));
  std::memcpy(buf + static_cast<size_t>(first) * nv, mine, static_cast<size_t>(nloc) * nv * sizeof(double));
  if (!shm::gather_publish_wait(g_seg, g, timeout_s)) return -1;
  shm::fixed_total(buf, ntot, nv, out);
  return 0;
}

}  // extern "C"
