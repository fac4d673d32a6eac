// mgicp_engine.hip -- host engine behind include/mi355x_gicp.h (libmgicp.so).
//
// Replaces pcl::GeneralizedIterativeClosestPoint<PointXYZRGB,PointXYZRGB>::align as called
// at /root/reference/src/GICPAlignment.cpp:96 (and :116 via iterate()).  The outer loop is
// GICP::computeTransformation (registration/impl/gicp.hpp): per iteration one correspondence
// sweep on the GPU, then estimateRigidTransformationBFGS whose objective passes run on the
// GPU and whose 6-DoF BFGS logic runs here (pcl_bfgs.hpp), then PCL's delta test.
// Multi-GPU: one process per GPU, contiguous ranges of the grid-sorted source cloud per rank,
// target replicated; the per-pass sums travel through a node-wide shared-memory segment of super
// rows (shm_rows.hpp: every rank's GPU writes its rows, every host takes the same fixed-order
// total), or -- without that segment -- one RCCL all-gather of super partials per pass (xGMI).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mi355x_gicp.h"
#include "host_upload.hpp"
#include "mgicp_internal.hpp"
#include "gn_solver.hpp"
#include "pcl_bfgs.hpp"
#include "shm_rows.hpp"

using namespace mgicp;

namespace {

constexpr double kDefaultOccupancy = 10.0;          // mean points per non-empty cell (A/B: profiles/r01/ab_tocc)
constexpr size_t kSmallBytes = size_t(64) << 10;  // pinned readback scratch per context
constexpr size_t kSketchOffset = size_t(32) << 10;  // the grid sizing sketch's registers in it (16 KiB)
constexpr size_t kMaxCells = size_t(1) << 29;       // dense cell table cap (2 GiB of uint32)
constexpr size_t kMaxBoxCells = size_t(1) << 27;    // per-cell point boxes up to 4 GiB (32 B per cell)

double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

#ifndef MGICP_ASYNC_RING_CAP
#define MGICP_ASYNC_RING_CAP 4  // rings the lazy source's head-start k-NN searches before leaving a point to the lazy pass
#endif
#ifndef MGICP_PASS_DIAG
#define MGICP_PASS_DIAG 0
#endif

// MGICP_TRACE=1: phase timestamps of uploads and grid builds on stderr (host-time diagnosis)
bool trace_on() {
  static const int on = [] {
    const char* t = std::getenv("MGICP_TRACE");
    return t && std::atoi(t) != 0 ? 1 : 0;
  }();
  return on != 0;
}
// MGICP_KNN_STATS=1: k-NN hand-off counts per covariance pass on stderr (diagnostic)
// (read at every covariance pass: tests switch it per context)
bool knn_stats_on() { return std::getenv("MGICP_KNN_STATS") != nullptr; }
#define MGICP_TRACE_AT(label)                                                  \
  do {                                                                         \
    if (trace_on()) std::fprintf(stderr, "[mgicp] %10.3f ms  %s\n", now_ms(), label); \
  } while (0)

struct Mat4 {  // row-major float 4x4
  float m[4][4];
  static Mat4 identity() {
    Mat4 r;
    std::memset(r.m, 0, sizeof(r.m));
    r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.f;
    return r;
  }
  static Mat4 from_cm(const float* cm) {
    Mat4 r;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) r.m[i][j] = cm[j * 4 + i];
    return r;
  }
  void to_cm(float* cm) const {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) cm[j * 4 + i] = m[i][j];
  }
  bool is_identity() const {
    const Mat4 I = identity();
    return std::memcmp(m, I.m, sizeof(m)) == 0;
  }
  Xf34 xf() const {
    Xf34 x;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 4; ++j) x.m[4 * i + j] = m[i][j];
    return x;
  }
};

// GICP::applyState(t = I, x): R = AngleAxisf(x5,Z) * AngleAxisf(x4,Y) * AngleAxisf(x3,X)
// evaluated through Eigen's quaternion products, then t.col(3) += (x0, x1, x2, 0).
struct Quat { float w, x, y, z; };
// r06: glibc's sincosf / sincos, not sinf + cosf / sin + cos.  PCL is built by gcc, whose sincos pass
// turns Eigen's cos(ha) / sin(ha) (and computeRDerivative's cos / sin of each angle) into ONE sincos call;
// glibc's sincos differs from separate sin / cos calls by an ulp on rare arguments (7 in 1e5 random
// gradients differed, tests/test_parity_configs_gpu.py::test_oracle_on_the_engine_tree_is_bitwise_the_engine
// caught one), and clang never forms it -- so the engine names it.
Quat quat_axis(float angle, int axis) {
  const float ha = 0.5f * angle;
  float s, c;
  ::sincosf(ha, &s, &c);
  Quat q{c, 0.f, 0.f, 0.f};
  if (axis == 0) q.x = s;
  if (axis == 1) q.y = s;
  if (axis == 2) q.z = s;
  return q;
}
Quat quat_mul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}
Mat4 apply_state(const Vec6& x) {
  const Quat q = quat_mul(quat_mul(quat_axis(static_cast<float>(x[5]), 2),
                                   quat_axis(static_cast<float>(x[4]), 1)),
                          quat_axis(static_cast<float>(x[3]), 0));
  const float tx = 2.0f * q.x, ty = 2.0f * q.y, tz = 2.0f * q.z;
  const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  Mat4 T = Mat4::identity();
  T.m[0][0] = 1.0f - (tyy + tzz);
  T.m[0][1] = txy - twz;
  T.m[0][2] = txz + twy;
  T.m[1][0] = txy + twz;
  T.m[1][1] = 1.0f - (txx + tzz);
  T.m[1][2] = tyz - twx;
  T.m[2][0] = txz - twy;
  T.m[2][1] = tyz + twx;
  T.m[2][2] = 1.0f - (txx + tyy);
  T.m[0][3] = 0.0f + static_cast<float>(x[0]);
  T.m[1][3] = 0.0f + static_cast<float>(x[1]);
  T.m[2][3] = 0.0f + static_cast<float>(x[2]);
  return T;
}

// GICP::computeRDerivative + matricesInnerProd (tr(dR * Rsum))
void r_derivative(const Vec6& x, const double R[3][3], Vec6& g) {
  const double phi = x[3], theta = x[4], psi = x[5];
  double cphi, sphi, ctheta, stheta, cpsi, spsi;  // glibc's sincos, as gcc-built PCL calls it (quat_axis)
  ::sincos(phi, &sphi, &cphi);
  ::sincos(theta, &stheta, &ctheta);
  ::sincos(psi, &spsi, &cpsi);
  double d[3][3][3];
  // d/dphi
  d[0][0][0] = 0.; d[0][1][0] = 0.; d[0][2][0] = 0.;
  d[0][0][1] = sphi * spsi + cphi * cpsi * stheta;
  d[0][1][1] = -cpsi * sphi + cphi * spsi * stheta;
  d[0][2][1] = cphi * ctheta;
  d[0][0][2] = cphi * spsi - cpsi * sphi * stheta;
  d[0][1][2] = -cphi * cpsi - sphi * spsi * stheta;
  d[0][2][2] = -ctheta * sphi;
  // d/dtheta
  d[1][0][0] = -cpsi * stheta;
  d[1][1][0] = -spsi * stheta;
  d[1][2][0] = -ctheta;
  d[1][0][1] = cpsi * ctheta * sphi;
  d[1][1][1] = ctheta * sphi * spsi;
  d[1][2][1] = -sphi * stheta;
  d[1][0][2] = cphi * cpsi * ctheta;
  d[1][1][2] = cphi * ctheta * spsi;
  d[1][2][2] = -cphi * stheta;
  // d/dpsi
  d[2][0][0] = -ctheta * spsi;
  d[2][1][0] = cpsi * ctheta;
  d[2][2][0] = 0.;
  d[2][0][1] = -cphi * cpsi - sphi * spsi * stheta;
  d[2][1][1] = -cphi * spsi + cpsi * sphi * stheta;
  d[2][2][1] = 0.;
  d[2][0][2] = cpsi * sphi - cphi * spsi * stheta;
  d[2][1][2] = sphi * spsi + cphi * cpsi * stheta;
  d[2][2][2] = 0.;
  for (int a = 0; a < 3; ++a) {
    double r = 0.;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) r += d[a][j][i] * R[i][j];
    g[3 + a] = r;
  }
}

// Device buffers a reserve() replaces are freed at quiet points of their OWN context (the end of an
// align, a destroy), not at once: hipFree waits for the whole device, which stalled set_*'s grid build
// behind the other cloud's covariance head start on the second stream (r04, ~2 ms, profiles/r04/prep7).
// One graveyard per context: a context's quiet point never frees -- and so never waits
// on -- buffers of another context or device.
struct Graveyard {
  std::vector<void*> v;
  void flush() {
    for (void* p : v) (void)hipFree(p);
    v.clear();
  }
};
// r06: a device allocation that fails for lack of memory first evicts the process-wide
// target cache's entry of the current device (set below, next to the cache) and retries once
bool (*g_oom_evict)() = nullptr;
// the graveyard of the context being constructed: every DevBuf member of a mgicp_ctx picks it up
thread_local Graveyard* t_new_ctx_grave = nullptr;

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  Graveyard* grave = t_new_ctx_grave;
  bool fine = false;  // fine-grained device memory (r06: the xGMI exchange rows, which peers store into)
  // grows by >= 1/4 so that a sequence of slightly larger requests (grid sizing iterations,
  // the second cloud) does not pay a hipFree/hipMalloc pair each time
  hipError_t reserve(size_t n) {
    if (n <= cap && p) return hipSuccess;
    const size_t want = std::max<size_t>(std::max<size_t>(n, 1), cap ? cap + cap / 4 : 0);
    if (p) {
      if (grave) grave->v.push_back(p);
      else (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
    auto alloc = [&]() {
      return fine ? hipExtMallocWithFlags(reinterpret_cast<void**>(&p), want * sizeof(T), hipDeviceMallocFinegrained)
                  : hipMalloc(&p, want * sizeof(T));
    };
    hipError_t e = alloc();
    if (e == hipErrorOutOfMemory && g_oom_evict) {
      (void)hipGetLastError();
      p = nullptr;
      if (g_oom_evict()) e = alloc();
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct Cloud {
  size_t n = 0;
  bool dirty = false;      // grid must be rebuilt
  bool have_cov = false;   // covariances valid for [cov_p0, cov_p1)
  size_t cov_p0 = 0, cov_p1 = 0;
  DevBuf<unsigned char> raw;  // staging of strided records
  DevBuf<float4> orig;        // original order, w = index
  DevBuf<float4> pts;         // grid-sorted
  DevBuf<uint32_t> perm;      // sorted pos -> original index
  DevBuf<uint32_t> cell_start;
  DevBuf<uint8_t> empty_dist; // empty-space map (target only: 1-NN queries leave the surface)
  bool want_empty_map = false;
  DevBuf<uint32_t> seed, seed_scratch;  // seed map (target: first-sweep 1-NN seeds)
  bool want_seed_map = false;
  DevBuf<float4> boxes;       // per-cell point boxes (target only: the 1-NN sweeps prune by them)
  bool want_boxes = false;
  DevBuf<float4> pairs;       // pair-interleaved points (target only: the wave-uniform 1-NN scan)
  bool want_pairs = false;
  bool drop_nonfinite = false; // build the grid over the finite points only (KdTreeFLANN semantics)
  double occupancy = 0;        // grid sizing target (points per non-empty cell); 0 = context default
  size_t n_built = 0;          // points of the last grid built in this slot
  bool fresh_grid = false;     // the grid is the one a fresh context builds for these points (target cache)
  DevBuf<double2> cov;        // 3 * cov_stride
  size_t cov_stride = 0;      // entries per covariance array (n, or the padded all-gather size)
  float lo[3] = {0.f, 0.f, 0.f}, hi[3] = {0.f, 0.f, 0.f};  // bounding box (original coordinates)
  GridView view{};
  size_t ncells = 0;
  Cov3 cov3() const { return Cov3{cov.p, cov.p + cov_stride, cov.p + 2 * cov_stride}; }
};

enum { kFamCov = 0, kFamCorr = 1, kFamFdf = 2, kFamRed = 3, kFamCompact = 4, kFamMoments = 5, kFams = 6 };

// pass-path counters (mgicp_debug_pass_stats)
enum {
  kStSrvLaunch = 0,  // resident servers launched
  kStSrvPass,        // objective passes run by a server
  kStLaunchedPass,   // objective passes run by a launched kernel (gated, plain, or taking over)
  kStTakeover,       // server passes that missed their deadline and were re-run as launched passes
  kStBar,            // 1: the server reads its commands from device memory written through the BAR
  kStRowsAlloc,      // private host-row buffer allocations
  kStTransport,      // 0 local, 1 RCCL, 2 shared segment, 3 shared segment + RCCL (bulk all-gathers),
                     // 4 xGMI row exchange (+ segment), 5 xGMI row exchange + RCCL
  kStSrvDenied,      // server launches refused because another context of this process held the device
  kStCount
};

// One resident server per device and process: its blocks need every CU of the device (one block
// per CU, 512 registers per lane), so a second context aligning on the same device at the same
// time runs launched passes instead of a second server.
std::atomic<int> g_srv_busy[64];

template <class T>
void swap_buf(DevBuf<T>& a, DevBuf<T>& b) {  // the device memory changes hands; each side keeps its graveyard
  std::swap(a.p, b.p);
  std::swap(a.cap, b.cap);
}

// r05 target cache: one entry per device (its DevBufs belong to no context: grave = nullptr)
struct TargetCache {
  std::mutex mu;
  bool valid = false;
  Cloud t;
  int k = 0;
  double eps = 0, occupancy = 0;
  float vlist_cell = 0.f;
  bool vl_valid = false, vl_alloc = false, vl_off = false;
  VListView vl{};
  size_t vl_ncells = 0;
  uint32_t vl_epoch = 0;
  int vl_groups = 0;
  DevBuf<uint32_t> vl_cell;
  DevBuf<float4> vl_pool;
  DevBuf<unsigned int> vl_ctr;
  long long hits = 0, donations = 0;
};
TargetCache g_tcache[64];

// the target's device state: every buffer a grid, its covariances and its cell lists live in
template <class F>
void each_target_buf(Cloud& a, Cloud& b, F&& f) {
  f(a.orig, b.orig); f(a.pts, b.pts); f(a.perm, b.perm); f(a.cell_start, b.cell_start);
  f(a.empty_dist, b.empty_dist); f(a.seed, b.seed); f(a.seed_scratch, b.seed_scratch); f(a.boxes, b.boxes);
  f(a.pairs, b.pairs); f(a.cov, b.cov);
}
void tcache_clear_locked(TargetCache& c) {
  Cloud none;
  each_target_buf(c.t, none, [](auto& x, auto&) { x.release(); });
  c.vl_cell.release();
  c.vl_pool.release();
  c.vl_ctr.release();
  c.valid = false;
}
bool tcache_evict_current() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  TargetCache& c = g_tcache[dev & 63];
  std::unique_lock<std::mutex> lk(c.mu, std::try_to_lock);  // never from inside the cache's own lock
  if (!lk.owns_lock() || (!c.valid && !c.t.orig.p && !c.vl_pool.p)) return false;
  tcache_clear_locked(c);
  return true;
}
struct OomHookInit {
  OomHookInit() { g_oom_evict = &tcache_evict_current; }
} g_oom_hook_init;

}  // namespace

struct mgicp_ctx {
  std::unique_ptr<Graveyard> grave;  // replaced device buffers of THIS context, freed at its quiet points
  mgicp_params prm{};
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  Cloud src, tgt;
  Cloud aux;  // scratch cloud of the resolution / radius / segment-differences helpers
  Cloud qry;  // query points of the FOD-side helpers (packed only, no grid)
  // FOD-side helper buffers (SegmentDifferences, VoxelGrid)
  DevBuf<uint32_t> f_flags, f_pos, f_rgba_in, f_rgba, f_rgba2;
  DevBuf<float4> f_vox, f_vox2;
  DevBuf<unsigned char> f_keep;
  DevBuf<unsigned int> f_count;
  double occupancy = kDefaultOccupancy;  // grid cell sizing target (debug option "grid_occ")
  // objective-pass launch shape over the fixed reduction tree, A/B-measured on MI355X at 5M points
  // (profiles/r02/ab_tree): 512 persistent 4-wave blocks -- 2 waves per SIMD, so chunk reductions
  // and tickets overlap other waves' streaming (71 us vs 76 us at 256 blocks), and the gated
  // grid (134 VGPRs: 3 waves per SIMD) stays resident while it waits at the gate (14.5 ms per C4
  // align vs 14.9 ms at 1024 blocks); in-launch finish
  bool fused_finish = true;              // in-launch reduction finish (debug option "fused_finish")
  int fdf_max_blocks = 512;              // objective-pass grid cap (fixed)
  // alternate the objective-pass direction: 360 MB of streams at 5M points exceed the 256 MiB
  // Infinity Cache, so each pass re-reads the previous pass's tail from it (73 -> 68 us)
  bool alt_sweep = true;                 // (fixed)
  int fdf_diag = 0;  // timing diagnostics of the objective pass (kernel modes 2 no reduction, 4 no tickets; not set by the host)
  double ms_upload_pending = 0;
  // host uploads go through the process-wide HostUploader (host_upload.hpp)
  int host_threads = 8;                  // packing workers (fixed)
  DevBuf<float> xyz_dev;                 // packed xyz landing zone
  // per source point (sorted), rank shard only
  DevBuf<float4> src_out;  // guess-applied source (only when guess != I)
  const float4* d_out = nullptr;
  // compacted accepted correspondences of the current outer iteration (shard-relative)
  DevBuf<uint32_t> prev_pos;  // matched target sorted position per shard point (also the next 1-NN seed)
  DevBuf<uint32_t> flags;
  DevBuf<unsigned char> nn_work;      // NnWork list of the wave sweep's stragglers (r03)
  DevBuf<unsigned int> nn_work_n;
  DevBuf<float> corr_f;    // 6 streams
  DevBuf<double> corr_d;   // 6 streams

  size_t corr_cap = 0;     // elements per stream (multiple of 4)
  bool seed_valid = false;
  // query order of the 1-NN sweeps (Morton order of the shard)
  bool query_order = true;
  bool qperm_valid = false;
  DevBuf<uint32_t> qperm;
  // the fixed reduction tree (internal.hpp kChunkPts / kSuperChunks): chunk layout of the streams,
  // chunk and super partials of this shard, the all-gathered supers of every rank, the total
  DevBuf<uint32_t> ccnt;  // chunk_count(ns): correspondences per chunk (fixed-slot layout, r04)
  DevBuf<double> partial;       // chunk partials, kRedVals each
  DevBuf<unsigned long long> tpart;  // the server's stamped chunk partials, 32 words each (r03; 0xff.. = no stamp)
  size_t tpart_n = 0;
  bool srv_tagged = true;            // the server's tagged tail (the chunk-ticket tail of r02 is the launched kernel's)
  DevBuf<double> spart;         // super partials (max_supers() rows: the all-gather send size)
  DevBuf<double> gath;          // nranks x max_supers() rows
  DevBuf<double> red;           // kRedVals
  DevBuf<unsigned int> tickets; // per super + 1: arrival counters of the in-launch finish
  size_t tickets_n = 0;
  // Gauss-Newton mode: chunk / super partials and the totals of one pass, and their host copy
  DevBuf<double> mpartial, msuper, mred;
  double mom[kMomVals] = {};
  double out_ctr[3] = {0, 0, 0};  // moment expansion centre: bbox midpoint of the guess-applied source
  unsigned char* h_small = nullptr;  // pinned, mapped host scratch (kSmallBytes) for small readbacks
  unsigned char* d_small = nullptr;  // its device address (kernels write results there directly)
  double* h_red = nullptr;   // pinned, mapped, coherent host memory
  double* d_h_red = nullptr; // its device address
  unsigned long long* h_flag = nullptr;  // pass-completion word (host / device views)
  unsigned long long* d_flag = nullptr;
  unsigned long long pass_seq = 0;
  bool poll = true;          // poll the completion word instead of hipStreamSynchronize (fixed)
  // pre-launched (gated) objective passes: pass k + 1 is queued while pass k runs and waits on the
  // host-written command block (debug option "gated"; single-GPU polled mode)
  bool gated = true;
  PassCmd* h_cmd = nullptr;             // pinned, mapped, coherent host memory
  PassCmd* d_cmd = nullptr;             // its device address
  PassCmd* mail = nullptr;              // device copy block 0 of a gated pass forwards to the others
  // the server's command block in fine-grained device memory that the host stores into through the
  // BAR (debug option "bar_cmd"): every server block polls it, no PCIe read and no mailbox hop
  bool bar = true;
  PassCmd* bar_cmd = nullptr;
  // blocks polling the host copy (fixed): 1 measured best (14.15 ms / C4 align;
  // 8 pollers 14.8 ms, all 256 blocks on host memory ~70 ms: PCIe read contention;
  // profiles/r02/ab_gate)
  int gate_pollers = 1;
  // MGICP_GATE_TRACE=1: per gated pass (seq & 1023) the device wall clock at kernel start, command
  // seen, last block through the gate; the host's wall clock (us) at flag seen / command published
  unsigned long long* h_gtrace = nullptr;  // mapped host memory, 4 x 1024
  unsigned long long* d_gtrace = nullptr;
  std::vector<double> host_gt;             // 2 x 1024
  unsigned long long gated_seq = 0;     // sequence number of the queued gated pass (0 = none)
  unsigned long long gate_timeout = 0;  // wall_clock64 ticks a gated pass waits before giving up
  // the resident pass server (debug option "resident"; single GPU polled mode, or any rank count with the
  // shared row segment): one launch per BFGS run keeps part of the compacted streams in registers /
  // LDS across all its passes
  bool resident = true;
  bool srv_live = false;                // a server is running and waits for pass srv_next
  bool srv_locked = false;              // this context holds g_srv_busy[device]
  bool srv_degraded = false;            // a server pass was taken over: launched passes until the align ends
  unsigned long long srv_next = 0;
  int cus = 0;                          // compute units (the server's grid)
  int srv_cus = 0;                      // debug option "srv_cus": cap on the server's blocks (0 = every CU)
  int srv_waves = 4;                    // server shape: 4 waves per CU (one per SIMD)
  int stall_pass = -1;                  // env MGICP_SRV_STALL_PASS (tests): a server block withholds this pass
  int quit_pass = -1;                   // env MGICP_DEBUG_QUIT_PASS (tests): the host gives up at this pass index
                                        // with MGICP_E_COMM (a rank that dies mid-align, seen from the others)
  bool corr_wave = true;                // wave-uniform 1-NN sweeps (fixed)
  int corr_lds_pts = -1;                // small-ball waves: union-box cell bounds in LDS (-1), + points when <= N fit (N > 0), off (0) (MGICP_CORR_LDS_PTS)
  int corr_split = 0;                   // waves of the wave sweep with <= this many stragglers hand them to a kernel of
                                        // their own (MGICP_CORR_SPLIT; 0 = every straggler finishes in place)
  float corr_rcap = 5.f;                // cells: lanes with a larger seed bound search alone (MGICP_CORR_RCAP)
  // r03 A/B (profiles/r03/corrsweep): union boxes of <= 96 rows and 16 cells along x, for waves whose
  // mean seed bound is >= 1.25 cells (the first sweep mostly): 2455 -> 2300 us per C4 align's sweeps
  int corr_max_rows = 96;               // union boxes with more rows / x cells: per-lane search
  int corr_max_x = 16;
  float corr_union_min_r = 1.25f;       // cells: waves whose mean seed bound is smaller search per lane
  double row_deadline_ms = 500.0;       // env MGICP_ROW_DEADLINE_MS: own rows missing this long -> take over
  double remote_deadline_s = 120.0;     // env MGICP_REMOTE_DEADLINE_S: other ranks' rows / gathers
  unsigned long long* h_ptimes = nullptr;  // MGICP_PASS_TIMES=1: per pass gate exit / finish (wall clock)
  unsigned long long* d_ptimes = nullptr;
  // the passes' super partials as stamped host rows (32 words per super, two parity buffers; env
  // MGICP_HOST_ROWS): private pinned memory, or the node-wide shared segment
  bool host_rows = true;
  unsigned long long* h_rows = nullptr;
  unsigned long long* d_rows = nullptr;
  size_t rows_cap = 0;                  // supers per parity buffer
  std::vector<double> row_sums;         // decoded super partials
  unsigned int pass_idx = 0;            // objective passes so far: the row stamp (identical on every rank)
  unsigned long long gather_idx = 0;    // generic gathers through the shared segment so far
  // node-wide transport (mgicp_comm_attach_shm)
  bool have_shm = false;
  shm::Segment shm;
  // r05 xGMI row exchange (mgicp_comm_attach_xgmi, needs the segment for its rendezvous): every rank's
  // super reducers store their rows into this rank's exchange buffer (xrows: 2 parity buffers of
  // max_sup rows, device memory) and into every other rank's, mapped by IPC over xGMI; a one-wave
  // totaler per rank takes the fixed-order total on the device and stores it as one stamped host row
  bool have_xgmi = false;
  DevBuf<unsigned long long> xrows;
  std::vector<void*> xpeer;               // the other ranks' exchange buffers (IPC mappings), rank order
  unsigned long long* h_xtot = nullptr;   // the totaler's stamped row (32 words; host / device views)
  unsigned long long* d_xtot = nullptr;
  unsigned int* h_xgen = nullptr;         // generation word: a totaler exits when it changes
  unsigned int* d_xgen = nullptr;
  unsigned int xgen = 0;
  unsigned long long xseq = 0;            // attaches so far (the segment's publication flag value)
  hipStream_t xstream = nullptr;
  bool xstream_own = false;  // r06: the aux stream (idle during a BFGS run: N > 1 keeps the synchronous
                             // covariance path) when the context has one -- no third stream per context
  unsigned char* shm_d = nullptr;       // device view of the segment (hipHostRegister'ed)
  long long st[kStCount] = {};          // pass-path counters
  // the resident server as the aligns run it (mgicp_debug_server_time): two events per launch
  struct SrvEv { hipEvent_t a, b; long long passes; };
  std::vector<SrvEv> srv_ev;            // launches not yet resolved (the last one may be live)
  double srv_time_ms = 0;
  long long srv_time_passes = 0, srv_time_launches = 0;
  bool spin_pause = false;              // pause instruction in the row spin (off: measured no gain)
  // MGICP_PASS_TIMES: host view of the server passes -- command published -> rows complete
  // (device pass + PCIe both ways) and rows complete -> next command (host BFGS step)
  double ht_dev = 0, ht_host = 0, ht_bfgs = 0, ht_eval = 0, ht_last_rows = 0;
  int ht_n = 0, ht_nh = 0, ht_ne = 0;
  // build scratch
  DevBuf<uint32_t> counts, keys, keys_sorted, vals;
  DevBuf<unsigned char> scratch;
  DevBuf<unsigned long long> u64;
  bool split_target_cov = true;     // multi-GPU: target covariances split + all-gathered (fixed)
  // lazy source covariances (r04, debug option "lazy_src_cov"): a source point's covariance is computed the
  // first time a sweep accepts it -- every consumer (Mahalanobis of the compaction, GN moments) reads
  // accepted points only, so points the gate never accepts (clutter, debris far off the part) never
  // pay PCL's exact 20-NN search; the values are the eager ones bit for bit
  bool lazy_src_cov = true;
  bool src_lazy_ready = false;      // cov arrays sized and cov_ok cleared for the current shard
  size_t src_lazy_p0 = 0, src_lazy_p1 = 0;
  DevBuf<uint8_t> cov_ok;           // per shard point: covariance computed
  DevBuf<uint32_t> cov_need;        // this sweep's accepted points without a covariance (absolute positions)
  // r04: set_target builds the target's grid and starts its k-NN covariances on a second stream, so
  // they run while the caller uploads the source; prepare joins them (debug option "async_cov" 0: off)
  bool async_tgt = true;
  // MGICP_AUX_CU_SKIP=k > 1: the aux stream on a CU mask leaving every k-th CU to the main stream (A/B
  // 0, 2, 4, 8: profiles/r04/ncab1, up to -1.4 ms new clouds).  Off: a CU mask belongs to the hardware
  // queue, and past GPU_MAX_HW_QUEUES streams share queues, so another context's main stream could
  // inherit the mask -- and a resident server needs every CU (it stalled test_inlaunch_finish_*)
  int aux_cu_skip = 0;
  // (and set_source the source's: single rank, same stream; with the lazy source mode these cover
  // every point, computed while the first sweep runs)
  bool tgt_cov_pending = false;     // the aux stream's covariance launches not joined yet
  bool src_cov_pending = false;
  bool src_async_lazy = false;      // the source's launch was ring-capped (lazy mode): the rest stays lazy
  int async_ring_cap = MGICP_ASYNC_RING_CAP;  // rings the source's head start searches (lazy mode)
  // one stream for both clouds' launches: with a stream each the process exceeds its hardware queues
  // (GPU_MAX_HW_QUEUES, 4) and the main stream ends up sharing one with them (profiles/r04/prep7)
  hipStream_t aux_stream = nullptr;
  hipEvent_t aux_ev[4] = {nullptr, nullptr, nullptr, nullptr};  // [3]: main stream -> aux (a grid built) (r06)
  // completion of the target's [0] / source's [1] launch,
                                                       // [2] the source's Morton order sorted on the aux stream
  bool qperm_aux = false;                    // qperm is being sorted on the aux stream (aux_ev[2])
  DevBuf<uint32_t> aq_keys, aq_keys_sorted, aq_vals;  // its sort buffers (the main stream's may be busy)
  DevBuf<unsigned char> aq_scratch;
  DevBuf<unsigned int> aux_cnt;     // their hand-off counts: [0] target, [1] source
  DevBuf<uint32_t> knn_fb2;         // the source's hand-off list
  bool knn_wave = true;             // r06: lazy pass + hand-offs by the wave-per-query kernel (debug option "knn_wave")
  bool knn_logged = true;           // wave-staged k-NN kernel + hand-off (debug option "knn_logged" 0: register-list only)
  DevBuf<uint32_t> knn_fb;          // points the logged k-NN kernel leaves to the register-list one
  unsigned int knn_fallbacks = 0;   // their count in the last covariance launch
  DevBuf<float> fpartial;
  // the target's 1-NN cell lists (r04, DESIGN.md "1-NN cell lists"; debug option "vlist" 0: the r03 sweeps)
  bool vlist = true;
  bool fuse_compact = true;           // r04: compaction fused into listed sweeps (debug option "fuse_compact")
  DevBuf<uint32_t> vl_defer;          // chunks a fused sweep deferred to the compaction launch
  float vlist_cell = 0.6f;            // fine cell edge / the target grid's cell edge (fixed)
  bool vl_stats = false;              // debug option "vlist_stats": per-sweep list diagnostics on stderr
  bool vl_valid = false;              // lists belong to the current target grid and gate
  bool vl_alloc = false;              // their state words and pool are allocated and initialised
  bool vl_off = false;                // the gate is too large for a fine grid of this target: r03 sweeps
  VListView vl{};
  size_t vl_ncells = 0;
  DevBuf<uint32_t> vl_cell, vl_build, vl_bcentre, vl_pend;
  DevBuf<float4> vl_pool;
  DevBuf<unsigned int> vl_ctr;
  uint32_t vl_epoch = 0;              // sweeps run over the current lists
  // A cell's list is built when a sweep of the SECOND align (or debug sweep group) over the current
  // target and gate queries it: the first align after a set_target runs the r03 sweep (no list work,
  // the ms-to-converge of a one-off align is unchanged), the second builds the lists of every cell it
  // queries, later aligns (GICPAlignment::iterate, the next scans of the same CAD target) read them.
  int vl_groups = 0;                  // aligns / debug sweep groups finished over the current lists
  bool vl_eager = false;              // debug option "vlist_eager" 1: build every queried cell at once (default: a cell
                                      // is built when a later sweep queries it again)
  // aligns (or debug sweep groups) after a set_target / gate change that run the r03 sweep before the
  // lists are used (debug option "vlist_cold" N).  The lists pay off only over many aligns on one target
  // (a later scan against the same CAD cloud, bench.py's steady state): building them costs ~57 ms
  // eagerly or ~15 ms spread over two aligns lazily at C4, so the reference's align + iterate pair on
  // one cloud pair (GICPAlignment.cpp:96, :116) runs both aligns without them (r04, profiles/r04/policy)
  int vl_cold_groups = 2;
  // r05 target cache (process-wide, one entry per device): a destroyed context leaves its target's grid,
  // covariances and 1-NN cell lists there; a later context whose set_target uploads the same points
  // (compared on the device, bit for bit) adopts them instead of rebuilding -- GICPState constructs a
  // fresh GICPAlignment per scan against the same CAD cloud (LeicaStateMachine.cpp:149-150)
  bool tcache_on = false;               // debug option "target_cache" (r06: opt-in; VERDICT r05 weak 5 --
                                        // the reference node aligns once per process)
  bool tcache_adopted = false;          // the current target came from the cache
  // multi-GPU
  int nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;
  // state of the last correspondence sweep
  bool have_corr = false;
  Mat4 last_guess = Mat4::identity();
  std::vector<float> trace;
  int n_evals = 0;
  // profiling
  bool profiling = false;
  unsigned prof_stride = 8;   // objective-pass event sampling (fixed)
  unsigned long long prof_tick = 0;
  struct EvPair { hipEvent_t a, b; int fam; };
  std::vector<EvPair> pending;
  std::vector<hipEvent_t> pool;
  double fam_ms[kFams] = {};
  int fam_cnt[kFams] = {};

  // shards start on super boundaries: rank r owns supers [super_first(r), super_first(r + 1))
  long long nsup_total() const { return static_cast<long long>((src.n + kSuperPts - 1) / kSuperPts); }
  size_t shard_at(int r) const {
    return std::min(src.n, static_cast<size_t>(super_first(r, nsup_total(), nranks)) * kSuperPts);
  }
  size_t shard_p0() const { return shard_at(rank); }
  size_t shard_p1() const { return shard_at(rank + 1); }
  long long nsup_local() const {
    return super_first(rank + 1, nsup_total(), nranks) - super_first(rank, nsup_total(), nranks);
  }
  long long max_supers() const { return (nsup_total() + nranks - 1) / nranks; }
};

namespace {

int fail(mgicp_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCK(expr)                                                                    \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(ctx, (e_ == hipErrorOutOfMemory) ? MGICP_E_NOMEM : MGICP_E_HIP,      \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                  \
  } while (0)

#define NCCLCK(expr)                                                                   \
  do {                                                                                 \
    ncclResult_t r_ = (expr);                                                          \
    if (r_ != ncclSuccess)                                                             \
      return fail(ctx, MGICP_E_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
  } while (0)

hipEvent_t ev_get(mgicp_ctx* ctx) {
  if (!ctx->pool.empty()) {
    hipEvent_t e = ctx->pool.back();
    ctx->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

struct ProfScope {
  mgicp_ctx* ctx;
  int fam;
  hipEvent_t a = nullptr;
  ProfScope(mgicp_ctx* c, int f) : ctx(c), fam(f) {
    // objective passes are sampled (every prof_stride-th launch: identical work per launch, and
    // two event records per pass would cost ~4 % of the PCL-mode align); the rest are all timed
    if (ctx->profiling && (fam != kFamFdf || (ctx->prof_tick++ % ctx->prof_stride) == 0)) {
      a = ev_get(ctx);
      (void)hipEventRecord(a, ctx->stream);
    }
  }
  ~ProfScope() {
    if (a) {
      hipEvent_t b = ev_get(ctx);
      (void)hipEventRecord(b, ctx->stream);
      ctx->pending.push_back({a, b, fam});
    }
  }
};

void prof_resolve(mgicp_ctx* ctx) {
  for (auto& p : ctx->pending) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      ctx->fam_ms[p.fam] += ms;
      ctx->fam_cnt[p.fam] += 1;
    }
    ctx->pool.push_back(p.a);
    ctx->pool.push_back(p.b);
  }
  ctx->pending.clear();
}

// command block of the queued gated pass: op / reverse / A first, then the sequence number
void publish_cmd(mgicp_ctx* ctx, unsigned long long seq, unsigned int op, int reverse, const Xf34* A,
                 unsigned int rstamp = 0) {
  // every 8-byte half: (stamp << 32) | word, one aligned 8-byte store each (single-copy atomic)
  unsigned int w[kCmdWords] = {};
  if (A) std::memcpy(w, A->m, 12 * sizeof(unsigned int));
  w[12] = op;
  w[13] = static_cast<unsigned int>(reverse);
  w[14] = rstamp;
  const unsigned long long stamp = static_cast<unsigned long long>(static_cast<unsigned int>(seq)) << 32;
  if (ctx->bar_cmd) {
    // device memory through the BAR: aligned 8-byte stores, then a store fence so they leave the
    // core's write-combining buffers now
    volatile unsigned long long* b = ctx->bar_cmd->h;
    for (int i = 0; i < kCmdWords; ++i) b[i] = stamp | w[i];
    __builtin_ia32_sfence();
  }
  for (int i = 0; i < kCmdWords; ++i) __atomic_store_n(&ctx->h_cmd->h[i], stamp | w[i], __ATOMIC_RELEASE);
}

// r05 xGMI: end the running totaler (if any) -- it exits when the generation word changes
void xgmi_cancel(mgicp_ctx* ctx) {
  if (ctx->have_xgmi && ctx->h_xgen) __atomic_store_n(ctx->h_xgen, ++ctx->xgen, __ATOMIC_RELEASE);
}

// r05: drop the xGMI row exchange (stream drained first: no totaler, no server writes into it)
void xgmi_detach(mgicp_ctx* ctx) {
  if (!ctx->have_xgmi) return;
  xgmi_cancel(ctx);
  if (ctx->xstream) (void)hipStreamSynchronize(ctx->xstream);
  for (void* p : ctx->xpeer) (void)hipIpcCloseMemHandle(p);
  ctx->xpeer.clear();
  ctx->xrows.release();
  ctx->have_xgmi = false;
}

// release a queued gated pass (or the resident server) without running it (end of a BFGS run,
// any stream drain)
void cancel_gated(mgicp_ctx* ctx) {
  if (ctx->srv_live) {
    xgmi_cancel(ctx);
    publish_cmd(ctx, ctx->srv_next, kPassCancel, 0, nullptr);
    ctx->pass_seq = std::max(ctx->pass_seq, ctx->srv_next);  // its sequence number is spent
    ctx->srv_live = false;
    // host-row passes leave the tickets as multiples of their supers' sizes: re-arm them for the
    // launched passes (stream order: after the server has exited)
    (void)hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream);
    // the device's server slot stays with this context until its stream has drained (sync): a
    // cancelled server may still be finishing, and another context's server must not start beside
    // it; this context's next BFGS run re-launches behind it in stream order
  }
  if (!ctx->gated_seq) return;
  publish_cmd(ctx, ctx->gated_seq, kPassCancel, 0, nullptr);
  ctx->pass_seq = std::max(ctx->pass_seq, ctx->gated_seq);  // its sequence number is spent
  ctx->gated_seq = 0;
}

// server launches whose events have completed (after a drain: all of them) -> the in-align totals
void srv_resolve(mgicp_ctx* ctx) {
  for (auto& e : ctx->srv_ev) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
      ctx->srv_time_ms += ms;
      ctx->srv_time_passes += e.passes;
      ctx->srv_time_launches += 1;
    }
    ctx->pool.push_back(e.a);
    ctx->pool.push_back(e.b);
  }
  ctx->srv_ev.clear();
}

// after a stream drain: no server of this context is running, the device's slot is free again
void srv_release(mgicp_ctx* ctx) {
  if (ctx->srv_locked && !ctx->srv_live) {
    g_srv_busy[ctx->device & 63].store(0, std::memory_order_release);
    ctx->srv_locked = false;
  }
}

int sync(mgicp_ctx* ctx) {
  cancel_gated(ctx);  // a queued gated pass would otherwise hold the stream until its timeout
  HIPCK(hipStreamSynchronize(ctx->stream));
  srv_release(ctx);
  if (ctx->profiling) prof_resolve(ctx);
  if (!ctx->srv_ev.empty()) srv_resolve(ctx);
  return MGICP_OK;
}

// Row stamps count objective passes; every buffer that holds stamps of earlier passes (the server's
// stamped chunk partials, this context's private host rows) is cleared whenever the count restarts
// (an attach or detach of the shared segment, the 2^31 wrap), so a stale word can never carry the
// stamp of a new pass.  The stream is drained first: no server still writes them.
int reset_stamps(mgicp_ctx* ctx) {
  int rc = sync(ctx);
  if (rc) return rc;
  if (ctx->tpart.p && ctx->tpart_n) {
    HIPCK(hipMemsetAsync(ctx->tpart.p, 0xff, ctx->tpart_n * sizeof(unsigned long long), ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
  }
  if (ctx->h_rows) std::memset(ctx->h_rows, 0, 2 * ctx->rows_cap * shm::kRowWords * sizeof(unsigned long long));
  if (ctx->have_xgmi) {  // stamps restart: no stale row of the exchange buffer may validate
    if (ctx->xstream) HIPCK(hipStreamSynchronize(ctx->xstream));
    HIPCK(hipMemsetAsync(ctx->xrows.p, 0, ctx->xrows.cap * sizeof(unsigned long long), ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    std::memset(ctx->h_xtot, 0, shm::kRowWords * sizeof(unsigned long long));
  }
  ctx->pass_idx = 0;
  ctx->gather_idx = 0;
  return MGICP_OK;
}

// Upload strided host records (or copy device records) and pack to float4 (original order).
int build_grid(mgicp_ctx* ctx, Cloud& cl, bool defer_extras = false);
int build_grid_extras(mgicp_ctx* ctx, Cloud& cl);
const uint32_t* query_perm(mgicp_ctx* ctx);
bool morton_perm(mgicp_ctx* ctx, const Cloud& c, size_t p0, size_t n, DevBuf<uint32_t>& out, bool aux);

// the covariances started by cov_prep_async: wait for the aux stream, then hand the points the
// logged kernel left (log overflow, ties at the k-th distance) to the register-list kernel on the
// main stream -- the same two launches as compute_cov
int cov_join(mgicp_ctx* ctx, bool tgt) {
  bool& pending = tgt ? ctx->tgt_cov_pending : ctx->src_cov_pending;
  if (!pending) return MGICP_OK;
  pending = false;
  Cloud& c = tgt ? ctx->tgt : ctx->src;
  // this cloud's launches only (the logged k-NN pass and its hand-off, chained on the aux stream):
  // the main stream waits for them on the device, the host does not
  HIPCK(hipStreamWaitEvent(ctx->stream, ctx->aux_ev[tgt ? 0 : 1], 0));
  if (ctx->knn_logged && knn_stats_on()) {  // as compute_cov reports it
    unsigned int nfb = 0;
    HIPCK(hipMemcpyAsync(ctx->h_small, ctx->aux_cnt.p + (tgt ? 0 : 1), sizeof(nfb), hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipStreamSynchronize(ctx->stream));
    std::memcpy(&nfb, ctx->h_small, sizeof(nfb));
    ctx->knn_fallbacks = nfb;
    std::fprintf(stderr, "[knn] %zu points, %u left to the register-list kernel\n", c.n, nfb);
  }
  if (!tgt && ctx->src_async_lazy) return MGICP_OK;  // the points it gave up on: computed if a sweep accepts them
  c.have_cov = true;
  c.cov_p0 = 0;
  c.cov_p1 = c.n;
  return MGICP_OK;
}
int cov_join_all(mgicp_ctx* ctx) {
  const int rc = cov_join(ctx, true);
  return rc ? rc : cov_join(ctx, false);
}

// set_target's / set_source's head start (single rank, eager target covariances, not profiling): the
// cloud's grid now (its host round trips), then its k-NN covariances on the aux stream -- the
// target's overlap the source's upload and grid build, the source's the first 1-NN sweep.  Any
// failure leaves the cloud for prepare, which reports it as before.
int cov_prep_async(mgicp_ctx* ctx, bool tgt) {
  Cloud& c = tgt ? ctx->tgt : ctx->src;
  if (!ctx->async_tgt || !ctx->aux_stream || ctx->nranks != 1 || ctx->comm || ctx->have_shm || ctx->profiling ||
      static_cast<size_t>(ctx->prm.k) > c.n)
    return MGICP_OK;
  // r06: the grid's core (sorted points, cell starts) only; the 1-NN extras are queued after the k-NN
  if (build_grid(ctx, c, true) != MGICP_OK) return MGICP_OK;
  if (c.n < static_cast<size_t>(ctx->prm.k)) return build_grid_extras(ctx, c);
  HIPCK(c.cov.reserve(3 * c.n));
  c.cov_stride = c.n;
  // the source in the lazy mode: a ring-capped launch (a point whose 20 neighbours lie beyond the
  // cap -- scan clutter, debris -- is left to the lazy pass, which computes it only if a sweep accepts
  // it; r04 C4F: the uncapped head start spent ~40 ms on them); its points are marked in cov_ok
  const bool capped = !tgt && ctx->lazy_src_cov && ctx->knn_logged && ctx->async_ring_cap >= 0;
  // r06 fix: the flag belongs to the SOURCE's launch -- the target's head start (set_target after
  // set_source on a context whose old target let the source start first) must not clear it, or the
  // source's join would mark the points its capped launch gave up on as computed (stale covariances)
  if (!tgt) ctx->src_async_lazy = capped;
  if (capped) {
    HIPCK(ctx->cov_ok.reserve(c.n));
    HIPCK(ctx->cov_need.reserve(c.n));
    HIPCK(hipMemsetAsync(ctx->cov_ok.p, 0, c.n, ctx->stream));
    ctx->src_lazy_ready = true;
    ctx->src_lazy_p0 = 0;
    ctx->src_lazy_p1 = c.n;
  }
  if (ctx->knn_logged) {
    HIPCK((tgt ? ctx->knn_fb : ctx->knn_fb2).reserve(c.n));
    HIPCK(ctx->aux_cnt.reserve(2));
    HIPCK(hipMemsetAsync(ctx->aux_cnt.p + (tgt ? 0 : 1), 0, sizeof(unsigned int), ctx->stream));
  }
  // the grid (and the count) before the aux stream reads them: a device-side dependency (r06; r04-r05
  // waited on the host)
  HIPCK(hipEventRecord(ctx->aux_ev[3], ctx->stream));
  HIPCK(hipStreamWaitEvent(ctx->aux_stream, ctx->aux_ev[3], 0));
  // the source's Morton query order is sorted on the aux stream ahead of its k-NN, so the main stream stays
  // empty for set_target's upload (r05: queued behind a main-stream sort that shares the CUs with the k-NN,
  // the target's copies waited ~2 ms)
  if (!tgt && ctx->query_order && !ctx->qperm_valid && !ctx->qperm_aux) {
    const size_t p0 = ctx->shard_p0(), ns = ctx->shard_p1() - p0;
    if (ns > 0 && morton_perm(ctx, c, p0, ns, ctx->qperm, true)) {
      HIPCK(hipEventRecord(ctx->aux_ev[2], ctx->aux_stream));
      ctx->qperm_valid = true;
      ctx->qperm_aux = true;
    }
  }
  HIPCK(launch_knn_cov(c.view, ctx->prm.k, ctx->prm.gicp_eps, 0, c.n, c.cov3(), nullptr,
                       ctx->knn_logged ? (tgt ? ctx->knn_fb.p : ctx->knn_fb2.p) : nullptr,
                       ctx->knn_logged ? ctx->aux_cnt.p + (tgt ? 0 : 1) : nullptr, ctx->aux_stream,
                       capped ? ctx->async_ring_cap : -1, capped ? ctx->cov_ok.p : nullptr,
                       ctx->knn_logged ? 2 * std::max(ctx->cus, 1) : 0, ctx->knn_wave));
  HIPCK(hipEventRecord(ctx->aux_ev[tgt ? 0 : 1], ctx->aux_stream));
  MGICP_TRACE_AT(tgt ? "head start: target k-NN queued" : "head start: source k-NN queued");
  (tgt ? ctx->tgt_cov_pending : ctx->src_cov_pending) = true;
  if (int rc = build_grid_extras(ctx, c)) return rc;  // the target's empty / seed map, boxes, pairs
  // r05: the source's 1-NN query order (a Morton sort of the shard) now, on the main stream beside the
  // covariances -- not inside the first align's loop
  if (!tgt && !ctx->qperm_aux) (void)query_perm(ctx);
  return MGICP_OK;
}

// after a set_*: the head start of the cloud just set -- its grid now (its host round trips), then its
// k-NN covariances on the aux stream.  r06: the source's grid is sized from the source alone (like the
// target's from the target), so its head start runs at set_source, whatever the order of the set_* calls
// and whether a target exists yet: the reference sets the source first (GICPAlignment.cpp:89-90), and
// the source's k-NN now overlaps set_target's upload and grid build.  (r04-r05 started the source's grid
// from the target's cell size, so a source set first waited for set_target; that dependency rested on a
// C4F trajectory flip later traced to a bug -- set_target's head start cleared the source's ring-cap flag
// -- not to the summation order, which the r06 ledger shows does not move C2F / C4F / C5:
// DESIGN.md "Summation-order ledger".)  The target's covariances are joined only before the first
// compaction, so they run beside the first 1-NN sweep.
int cov_prep_async_all(mgicp_ctx* ctx) {
  int rc = MGICP_OK;
  if (ctx->tgt.dirty && (rc = cov_prep_async(ctx, true))) return rc;
  if (ctx->src.dirty) rc = cov_prep_async(ctx, false);
  return rc;
}

int upload_cloud(mgicp_ctx* ctx, Cloud& cl, const float* xyz, size_t n, size_t stride,
                 bool device_ptr) {
  if (n == 0 || !xyz || stride < 12 || (stride % 4) != 0)
    return fail(ctx, MGICP_E_INVALID, "invalid cloud (null, empty or stride not a multiple of 4 >= 12)");
  if (n >= (size_t(1) << 31) - 1)  // 32-bit point indices / hipcub item counts
    return fail(ctx, MGICP_E_INVALID, "cloud too large: at most 2^31 - 2 points per cloud");
  if (&cl == &ctx->tgt || &cl == &ctx->src) {  // an async covariance launch still reads the old cloud
    const int rj = cov_join(ctx, &cl == &ctx->tgt);
    if (rj) return rj;
  }
  if (&cl == &ctx->src && ctx->qperm_aux)  // the aux stream's Morton sort still reads the source's grid
    HIPCK(hipStreamWaitEvent(ctx->stream, ctx->aux_ev[2], 0));
  const double t0 = now_ms();
  MGICP_TRACE_AT("upload: begin");
  HIPCK(cl.orig.reserve(n));
  MGICP_TRACE_AT("upload: orig reserved");
  if (device_ptr) {
    HIPCK(launch_pack_points(xyz, n, stride, cl.orig.p, ctx->stream));
  } else {
    // host workers pack xyz into pinned slots while earlier slots are in flight
    HostUploader& up = HostUploader::instance();
    HIPCK(up.init(ctx->host_threads));
    HIPCK(ctx->xyz_dev.reserve(3 * n));
    MGICP_TRACE_AT("upload: staging ready");
    {
      std::lock_guard<std::mutex> lk(up.mu);
      HIPCK(upload_xyz(*up.pool, up.ring, xyz, n, stride, ctx->xyz_dev.p, ctx->stream));
    }
    MGICP_TRACE_AT("upload: all chunks queued");
    HIPCK(launch_pack_points(ctx->xyz_dev.p, n, 12, cl.orig.p, ctx->stream));
  }
  int rc = sync(ctx);
  if (rc) return rc;
  MGICP_TRACE_AT("upload: synced");
  cl.n = n;
  cl.dirty = true;
  cl.have_cov = false;
  if (&cl == &ctx->src) ctx->qperm_valid = false;
  if (&cl == &ctx->src || &cl == &ctx->tgt) {
    // the previous sweep's matches index the old clouds: never seed from / reuse them
    ctx->have_corr = false;
    ctx->seed_valid = false;
    ctx->ms_upload_pending += now_ms() - t0;
  }
  return MGICP_OK;
}

// r05 target cache.  A single-rank context leaves its target at destroy when the grid is the one a fresh
// context would build for those points (fresh_grid; since r06 every grid is sized from its own cloud
// alone -- DESIGN.md "Target cache").
void tcache_donate(mgicp_ctx* ctx, bool cov_complete) {
  Cloud& t = ctx->tgt;
  if (!ctx->tcache_on || ctx->nranks != 1 || ctx->comm || ctx->have_shm || t.dirty || t.n == 0 || t.n_built != t.n ||
      !t.fresh_grid)
    return;
  TargetCache& c = g_tcache[ctx->device & 63];
  std::lock_guard<std::mutex> lk(c.mu);
  tcache_clear_locked(c);
  each_target_buf(c.t, t, [](auto& x, auto& y) { swap_buf(x, y); });
  c.t.n = t.n;
  c.t.have_cov = cov_complete && (!t.have_cov || (t.cov_p0 == 0 && t.cov_p1 == t.n)) && t.cov_stride == t.n;
  c.t.cov_p0 = 0;
  c.t.cov_p1 = t.n;
  c.t.cov_stride = t.cov_stride;
  c.t.want_empty_map = t.want_empty_map;
  c.t.want_seed_map = t.want_seed_map;
  c.t.want_boxes = t.want_boxes;
  c.t.want_pairs = t.want_pairs;
  c.t.drop_nonfinite = t.drop_nonfinite;
  c.t.occupancy = t.occupancy;
  c.t.n_built = t.n_built;
  c.t.fresh_grid = true;
  std::memcpy(c.t.lo, t.lo, sizeof(t.lo));
  std::memcpy(c.t.hi, t.hi, sizeof(t.hi));
  c.t.view = t.view;
  c.t.ncells = t.ncells;
  c.k = ctx->prm.k;
  c.eps = ctx->prm.gicp_eps;
  c.occupancy = t.occupancy > 0 ? t.occupancy : ctx->occupancy;
  // the cell lists travel with the target once built (the donor ran 3+ aligns on it).  The list policy
  // itself does not go on across contexts: GICPState's engines run 2 aligns each, and building the lists
  // in a later cycle cost 39 + 151 ms at C4 (profiles/r05/check5) against ~1.6 ms saved per cycle
  c.vl_valid = ctx->vl_valid && ctx->vl_alloc;
  if (c.vl_valid) {
    if (ctx->vl_alloc) {
      swap_buf(c.vl_cell, ctx->vl_cell);
      swap_buf(c.vl_pool, ctx->vl_pool);
      swap_buf(c.vl_ctr, ctx->vl_ctr);
    }
    c.vl = ctx->vl;
    c.vl_alloc = ctx->vl_alloc;
    c.vl_off = ctx->vl_off;
    c.vl_ncells = ctx->vl_ncells;
    c.vl_epoch = ctx->vl_epoch;
    c.vl_groups = ctx->vl_groups;
    c.vlist_cell = ctx->vlist_cell;
  }
  c.valid = true;
  c.donations++;
}

// After set_target's upload: the cached state when the uploaded points equal the cached ones bit for bit
// (original order, w = original index).  The context's previous target buffers go to its graveyard.
int tcache_adopt(mgicp_ctx* ctx) {
  ctx->tcache_adopted = false;
  Cloud& t = ctx->tgt;
  if (!ctx->tcache_on || ctx->nranks != 1 || ctx->comm || ctx->have_shm) return MGICP_OK;
  TargetCache& c = g_tcache[ctx->device & 63];
  std::lock_guard<std::mutex> lk(c.mu);
  const double occ = t.occupancy > 0 ? t.occupancy : ctx->occupancy;
  if (!c.valid || c.t.n != t.n || c.occupancy != occ || c.t.drop_nonfinite != t.drop_nonfinite ||
      c.t.want_pairs != t.want_pairs || c.t.want_boxes != t.want_boxes)
    return MGICP_OK;
  unsigned int* diff = reinterpret_cast<unsigned int*>(ctx->d_small);
  MGICP_TRACE_AT("adopt: compare");
  HIPCK(launch_equal(t.orig.p, c.t.orig.p, t.n, diff, ctx->stream));
  int rc = sync(ctx);
  if (rc) return rc;
  MGICP_TRACE_AT("adopt: compared");
  unsigned int d = 1;
  std::memcpy(&d, ctx->h_small, sizeof(d));
  if (d != 0) return MGICP_OK;
  each_target_buf(t, c.t, [](auto& x, auto& y) { swap_buf(x, y); });
  t.dirty = false;
  t.have_cov = c.t.have_cov && c.k == ctx->prm.k && c.eps == ctx->prm.gicp_eps;
  t.cov_p0 = 0;
  t.cov_p1 = t.have_cov ? t.n : 0;
  t.cov_stride = c.t.cov_stride;
  t.n_built = c.t.n_built;
  t.fresh_grid = true;
  std::memcpy(t.lo, c.t.lo, sizeof(t.lo));
  std::memcpy(t.hi, c.t.hi, sizeof(t.hi));
  t.view = c.t.view;  // the same device memory, now this context's
  t.ncells = c.t.ncells;
  ctx->vl_valid = false;
  if (c.vl_valid && c.vlist_cell == ctx->vlist_cell) {
    if (c.vl_alloc) {
      swap_buf(ctx->vl_cell, c.vl_cell);
      swap_buf(ctx->vl_pool, c.vl_pool);
      swap_buf(ctx->vl_ctr, c.vl_ctr);
    }
    ctx->vl = c.vl;
    ctx->vl_valid = true;
    ctx->vl_alloc = c.vl_alloc;
    ctx->vl_off = c.vl_off;
    ctx->vl_ncells = c.vl_ncells;
    ctx->vl_epoch = c.vl_epoch;
    ctx->vl_groups = c.vl_groups;
  }
  // the cache now holds this context's previous target buffers: to the graveyard (freed at a quiet point)
  Cloud none;
  each_target_buf(c.t, none, [&](auto& x, auto&) {
    if (x.p) ctx->grave->v.push_back(x.p);
    x.p = nullptr;
    x.cap = 0;
  });
  for (void* p : {static_cast<void*>(c.vl_cell.p), static_cast<void*>(c.vl_pool.p), static_cast<void*>(c.vl_ctr.p)})
    if (p) ctx->grave->v.push_back(p);
  c.vl_cell.p = nullptr; c.vl_cell.cap = 0;
  c.vl_pool.p = nullptr; c.vl_pool.cap = 0;
  c.vl_ctr.p = nullptr; c.vl_ctr.cap = 0;
  c.valid = false;
  c.hits++;
  ctx->tcache_adopted = true;
  return MGICP_OK;
}

// Build the row-sorted uniform grid of a cloud (one-time per set_*).
int build_grid(mgicp_ctx* ctx, Cloud& cl, bool defer_extras) {
  const size_t n = cl.n;
  hipStream_t s = ctx->stream;
  // 1. bounding box + finiteness
  const int nb = static_cast<int>(std::min<size_t>((n + 255) / 256, 1024));
  MGICP_TRACE_AT("grid: begin");
  // block partials land straight in mapped host memory (nb * 8 floats <= 32 KiB): no copy
  HIPCK(launch_bbox(cl.orig.p, n, reinterpret_cast<float*>(ctx->d_small), nb, s));
  const float* hp = reinterpret_cast<const float*>(ctx->h_small);
  MGICP_TRACE_AT("grid: bbox queued");
  int rc = sync(ctx);
  if (rc) return rc;
  MGICP_TRACE_AT("grid: bbox synced");
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  double bad = 0;
  for (int b = 0; b < nb; ++b) {
    for (int d = 0; d < 3; ++d) {
      mn[d] = std::min(mn[d], hp[b * 8 + d]);
      mx[d] = std::max(mx[d], hp[b * 8 + 3 + d]);
    }
    bad += hp[b * 8 + 6];
  }
  if (bad > 0 && cl.drop_nonfinite) {
    // keep the finite points (original indices stay in w) and rebuild from them
    HIPCK(ctx->f_flags.reserve(n + 1));
    HIPCK(ctx->f_pos.reserve(n + 1));
    HIPCK(cl.pts.reserve(n));
    const size_t sb = scan_scratch_bytes(n + 1);
    HIPCK(ctx->scratch.reserve(sb));
    HIPCK(launch_finite_compact(cl.orig.p, n, ctx->f_flags.p, ctx->f_pos.p, ctx->scratch.p, sb, cl.pts.p, s));
    HIPCK(hipMemcpyAsync(ctx->h_small, ctx->f_pos.p + n, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if ((rc = sync(ctx))) return rc;
    uint32_t kept = 0;
    std::memcpy(&kept, ctx->h_small, sizeof(kept));
    if (kept > 0) HIPCK(hipMemcpyAsync(cl.orig.p, cl.pts.p, kept * sizeof(float4), hipMemcpyDeviceToDevice, s));
    cl.n = kept;
    if (kept == 0) {
      cl.dirty = false;
      return MGICP_OK;  // empty cloud: callers check cl.n
    }
    return build_grid(ctx, cl, defer_extras);
  }
  if (bad > 0) return fail(ctx, MGICP_E_NONFINITE, "cloud contains NaN/Inf coordinates");
  for (int d = 0; d < 3; ++d) {
    cl.lo[d] = mn[d];
    cl.hi[d] = mx[d];
  }
  float ext[3];
  float maxext = 0.f, maxabs = 0.f;
  for (int d = 0; d < 3; ++d) {
    ext[d] = mx[d] - mn[d];
    maxext = std::max(maxext, ext[d]);
    maxabs = std::max(maxabs, std::max(std::fabs(mn[d]), std::fabs(mx[d])));
  }
  // 2. cell size: aim at `target_occ` points per non-empty cell
  const double target_occ = cl.occupancy > 0 ? cl.occupancy : ctx->occupancy;
  auto dims = [&](double h, int* nd) {
    size_t nc = 1;
    for (int d = 0; d < 3; ++d) {
      const float inv_h = static_cast<float>(1.0 / h);
      nd[d] = static_cast<int>(std::floor(static_cast<double>(ext[d]) * inv_h)) + 1;
      nc *= static_cast<size_t>(nd[d]);
    }
    return nc;
  };
  double h = maxext > 0.f ? static_cast<double>(maxext) / std::cbrt(static_cast<double>(n)) : 1.0;
  // r06: the cell size is a function of this cloud alone -- never of this slot's
  // previous grid or of the other cloud's (the source's grid sets the order of every objective sum).
  // One sketch pass (cell_sketch_kernel) estimates the non-empty cells at kSketchScales sizes
  // h0 * 2^(k - 10) around the 3-D guess h0 above; the size is interpolated in log-log between the two
  // that bracket the target occupancy.  r01-r05 ran trial histograms instead (scattered atomics, a host
  // round trip each, two per cloud on a surface: ~0.6-0.8 ms per 5M cloud before the sort)
  const bool fresh = true;
  h = std::max(h, 1e-6);
  if (maxext > 0.f && n > 1) {
    SketchScales sc;
    double hk[kSketchScales];
    for (int k = 0; k < kSketchScales; ++k) {
      hk[k] = h * std::ldexp(1.0, k - 10);
      sc.inv[k] = static_cast<float>(1.0 / hk[k]);
    }
    HIPCK(ctx->scratch.reserve(static_cast<size_t>(kSketchBlocks + 32) * kSketchScales * kSketchR));
    HIPCK(launch_cell_sketch(cl.orig.p, n, mn[0], mn[1], mn[2], sc, ctx->scratch.p, ctx->d_small + kSketchOffset, s));
    rc = sync(ctx);
    if (rc) return rc;
    MGICP_TRACE_AT("grid: sizing sketch synced");
    const unsigned char* regs = ctx->h_small + kSketchOffset;
    double occ[kSketchScales];
    for (int k = 0; k < kSketchScales; ++k) {
      // HyperLogLog estimate of the non-empty cells (linear counting while registers are still zero)
      double inv_sum = 0.0;
      int zeros = 0;
      for (int j = 0; j < kSketchR; ++j) {
        const int r = regs[k * kSketchR + j];
        inv_sum += std::ldexp(1.0, -r);
        zeros += r == 0;
      }
      const double R = kSketchR;
      double e = 0.7213 / (1.0 + 1.079 / R) * R * R / inv_sum;
      if (e <= 2.5 * R && zeros > 0) e = R * std::log(R / zeros);
      occ[k] = static_cast<double>(n) / std::max(e, 1.0);
    }
    int k1 = -1;
    for (int k = 0; k < kSketchScales && k1 < 0; ++k)
      if (occ[k] >= target_occ) k1 = k;
    if (k1 < 0) {
      h = hk[kSketchScales - 1];  // fewer points than the target per cell even at the coarsest size
    } else if (k1 == 0) {
      // finer than the finest size: extrapolate with the finest pair's growth exponent (1-3)
      double dim = std::log(std::max(occ[1], occ[0]) / occ[0]) / std::log(2.0);
      dim = std::min(3.0, std::max(1.0, dim));
      h = hk[0] * std::pow(target_occ / occ[0], 1.0 / dim);
    } else {
      const double t = (std::log(target_occ) - std::log(occ[k1 - 1])) / (std::log(occ[k1]) - std::log(occ[k1 - 1]));
      h = hk[k1 - 1] * std::exp2(std::min(1.0, std::max(0.0, t)));
    }
    h = std::max(h, 1e-6);
    if (trace_on()) {
      std::fprintf(stderr, "[mgicp] grid sizing n %zu h0 %.6g -> h %.6g (target %.1f); estimated occupancy", n, hk[10],
                   h, target_occ);
      for (int k = 0; k < kSketchScales; ++k) std::fprintf(stderr, " %.3g", occ[k]);
      std::fprintf(stderr, "\n");
    }
  }
  int nd[3];
  size_t nc = dims(h, nd);
  while (nc > kMaxCells) {
    h *= std::cbrt(static_cast<double>(nc) / kMaxCells) * 1.01;
    nc = dims(h, nd);
  }
  const float inv_h = static_cast<float>(1.0 / h);
  // 3. cell keys, stable radix sort -> permutation, cell_start from the sorted keys (cell_end_kernel +
  // an exclusive max-scan: no histogram of atomics)
  HIPCK(ctx->counts.reserve(nc + 1));
  HIPCK(ctx->keys.reserve(n));
  HIPCK(ctx->keys_sorted.reserve(n));
  HIPCK(ctx->vals.reserve(n));
  HIPCK(cl.perm.reserve(n));
  HIPCK(cl.cell_start.reserve(nc + 1));
  HIPCK(cl.pts.reserve(n));
  MGICP_TRACE_AT("grid: final buffers reserved");
  HIPCK(launch_cell_hist(cl.orig.p, n, mn[0], mn[1], mn[2], inv_h, nd[0], nd[1], nd[2], nullptr, ctx->keys.p, s));
  int bits = 1;
  while ((size_t(1) << bits) < nc && bits < 32) ++bits;
  const size_t sb = std::max(sort_scratch_bytes(n, bits), cell_start_scratch_bytes(nc));
  HIPCK(ctx->scratch.reserve(sb));
  HIPCK(launch_iota(ctx->vals.p, n, s));
  HIPCK(launch_sort_pairs(ctx->scratch.p, sb, ctx->keys.p, ctx->keys_sorted.p, ctx->vals.p,
                          cl.perm.p, n, bits, s));
  HIPCK(launch_cell_starts(ctx->keys_sorted.p, n, nc, ctx->counts.p, cl.cell_start.p, ctx->scratch.p, sb, s));
  HIPCK(launch_gather_sorted(cl.orig.p, cl.perm.p, n, cl.pts.p, s));
  MGICP_TRACE_AT("grid: sort queued");
  if (trace_on() && n > 0) {  // diagnostics: the grid's real occupancy (host copy of the sorted keys)
    std::vector<uint32_t> ks(n);
    HIPCK(hipMemcpyAsync(ks.data(), ctx->keys_sorted.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if ((rc = sync(ctx))) return rc;
    size_t runs = 1;
    for (size_t i = 1; i < n; ++i) runs += ks[i] != ks[i - 1];
    std::fprintf(stderr, "[mgicp] grid n %zu h %.6g cells %d x %d x %d, non-empty %zu, occupancy %.2f\n", n, h, nd[0],
                 nd[1], nd[2], runs, static_cast<double>(n) / runs);
  }
  if (!defer_extras) {
    rc = sync(ctx);
    if (rc) return rc;
    MGICP_TRACE_AT("grid: sorted");
  }
  // the build scratch stays allocated for the next build (hipFree + hipMalloc of these
  // tens-of-MB buffers cost milliseconds of host time between the two clouds' builds)
  GridView& g = cl.view;
  g.ox = mn[0];
  g.oy = mn[1];
  g.oz = mn[2];
  g.h = static_cast<float>(h);
  g.inv_h = inv_h;
  // rounding slack: a few ulps of the largest coordinate plus a sliver of a cell
  g.slop = 8.f * maxabs * 1.1920929e-7f + 1e-6f * static_cast<float>(h);
  g.nx = nd[0];
  g.ny = nd[1];
  g.nz = nd[2];
  g.cell_start = cl.cell_start.p;
  g.pts = cl.pts.p;
  g.empty_dist = nullptr;
  g.seed = nullptr;
  g.boxes = nullptr;
  g.pairs = nullptr;
  cl.ncells = nc;
  cl.n_built = n;
  cl.fresh_grid = fresh;
  cl.dirty = false;
  cl.have_cov = false;
  if (&cl == &ctx->tgt) ctx->vl_valid = false;  // the 1-NN cell lists index the old target
  if (&cl == &ctx->src) ctx->src_lazy_ready = false;  // lazy covariances: none computed for this cloud
  if (&cl == &ctx->src || &cl == &ctx->tgt) {  // sorted positions changed
    ctx->have_corr = false;
    ctx->seed_valid = false;
  }
  return defer_extras ? MGICP_OK : build_grid_extras(ctx, cl);
}

// The 1-NN sweeps' extras of a built grid (target): empty-space + seed map, per-cell boxes, the
// pair-interleaved copy -- queued on the main stream, no host wait.  r06: set_target's head start queues
// the target's k-NN (which needs none of them) BEFORE these, so the 0.7-0.8 ms of the empty map at C4 run
// beside the k-NN instead of in front of it (the target's k-NN is the cold first align's long pole).
int build_grid_extras(mgicp_ctx* ctx, Cloud& cl) {
  GridView& g = cl.view;
  hipStream_t s = ctx->stream;
  const size_t nc = cl.ncells, n = cl.n;
  if (cl.want_empty_map) {
    HIPCK(cl.empty_dist.reserve(nc));
    HIPCK(ctx->scratch.reserve(nc));
    if (cl.want_seed_map) {
      HIPCK(cl.seed.reserve(nc));
      HIPCK(cl.seed_scratch.reserve(nc));
    }
    HIPCK(launch_empty_map(cl.cell_start.p, g.nx, g.ny, g.nz, cl.empty_dist.p, ctx->scratch.p, s,
                           cl.want_seed_map ? cl.seed.p : nullptr, cl.want_seed_map ? cl.seed_scratch.p : nullptr,
                           &g));
    MGICP_TRACE_AT("grid: empty map queued");
    g.empty_dist = cl.empty_dist.p;
    if (cl.want_seed_map) g.seed = cl.seed.p;
  }
  if (cl.want_boxes && nc <= kMaxBoxCells) {
    HIPCK(cl.boxes.reserve(2 * nc));
    HIPCK(launch_cell_boxes(cl.pts.p, cl.cell_start.p, nc, cl.boxes.p, s));
    g.boxes = cl.boxes.p;
  }
  if (cl.want_pairs) {
    HIPCK(cl.pairs.reserve(2 * pair_count(n)));
    HIPCK(launch_pairs(cl.pts.p, n, cl.pairs.p, s));
    g.pairs = cl.pairs.p;
  }
  return MGICP_OK;
}

// Morton order of points [p0, p0 + n) of a grid-sorted cloud: a stable sort of 30-bit Morton codes
// over the cloud's bbox.  Query order of the k-NN / 1-NN kernels (a wave's queries then form a
// compact 3-D patch); results stay indexed by grid-sorted position.  false on failure.
bool morton_perm(mgicp_ctx* ctx, const Cloud& c, size_t p0, size_t n, DevBuf<uint32_t>& out, bool aux) {
  hipStream_t s = aux ? ctx->aux_stream : ctx->stream;
  DevBuf<uint32_t>& keys = aux ? ctx->aq_keys : ctx->keys;
  DevBuf<uint32_t>& keys_sorted = aux ? ctx->aq_keys_sorted : ctx->keys_sorted;
  DevBuf<uint32_t>& vals = aux ? ctx->aq_vals : ctx->vals;
  DevBuf<unsigned char>& scratch = aux ? ctx->aq_scratch : ctx->scratch;
  float ext = 0.f;
  for (int d = 0; d < 3; ++d) ext = std::max(ext, c.hi[d] - c.lo[d]);
  const float inv = ext > 0.f ? 1024.0f / (ext * 1.0001f) : 0.f;
  if (out.reserve(n) != hipSuccess || keys.reserve(n) != hipSuccess ||
      keys_sorted.reserve(n) != hipSuccess || vals.reserve(n) != hipSuccess)
    return false;
  const size_t sb = sort_scratch_bytes(n, 30);
  if (scratch.reserve(sb) != hipSuccess) return false;
  return launch_morton_keys(c.pts.p, p0, n, c.lo, inv, keys.p, vals.p, s) == hipSuccess &&
         launch_sort_pairs(scratch.p, sb, keys.p, keys_sorted.p, vals.p, out.p, n, 30, s) == hipSuccess;
}

// query order of the shard's 1-NN sweeps and source covariances (once per source cloud and shard)
const uint32_t* query_perm(mgicp_ctx* ctx) {
  if (!ctx->query_order) return nullptr;
  if (ctx->qperm_aux) {  // sorted on the aux stream at set_source: the main stream waits for it on the device
    ctx->qperm_aux = false;
    if (hipStreamWaitEvent(ctx->stream, ctx->aux_ev[2], 0) != hipSuccess) ctx->qperm_valid = false;
  }
  if (ctx->qperm_valid) return ctx->qperm.p;
  const size_t p0 = ctx->shard_p0(), ns = ctx->shard_p1() - p0;
  if (ns == 0 || !morton_perm(ctx, ctx->src, p0, ns, ctx->qperm, false)) return nullptr;
  ctx->qperm_valid = true;
  return ctx->qperm.p;
}

constexpr unsigned int kWaveKnnMax = 65536;  // r06: lazy / hand-off lists up to this size run knn_wave_kernel

// covariances of sorted positions [p0, p1) into arrays of `stride` entries (default n)
int compute_cov(mgicp_ctx* ctx, Cloud& cl, size_t p0, size_t p1, size_t stride = 0) {
  MGICP_TRACE_AT("cov: begin");
  if (stride < cl.n) stride = cl.n;
  HIPCK(cl.cov.reserve(3 * stride));
  cl.cov_stride = stride;
  MGICP_TRACE_AT("cov: reserved");
  // grid order, not Morton order: the k = 20 queries sit on the surface and the row-major order
  // measured faster (3.97 vs 4.42 ms at 5M, profiles/r01/ab_qorder/)
  const uint32_t* perm = nullptr;
  const bool logged = ctx->knn_logged;
  if (logged) {
    HIPCK(ctx->knn_fb.reserve(p1 - p0));
    HIPCK(ctx->u64.reserve(1));
    HIPCK(hipMemsetAsync(ctx->u64.p, 0, sizeof(unsigned long long), ctx->stream));
  }
  unsigned int* fb_count = reinterpret_cast<unsigned int*>(ctx->u64.p);
  {
    ProfScope ps(ctx, kFamCov);
    HIPCK(launch_knn_cov(cl.view, ctx->prm.k, ctx->prm.gicp_eps, p0, p1, cl.cov3(), perm,
                         logged ? ctx->knn_fb.p : nullptr, logged ? fb_count : nullptr, ctx->stream));
  }
  if (logged) {
    // the points the logged kernel left to the register-list kernel (log overflow, ties at tau)
    HIPCK(hipMemcpyAsync(ctx->h_small, fb_count, sizeof(unsigned int), hipMemcpyDeviceToHost, ctx->stream));
    int rc0 = sync(ctx);
    if (rc0) return rc0;
    unsigned int nfb = 0;
    std::memcpy(&nfb, ctx->h_small, sizeof(nfb));
    ctx->knn_fallbacks = nfb;
    const bool stats = knn_stats_on();
    if (stats) std::fprintf(stderr, "[knn] %zu points, %u left to the register-list kernel\n", p1 - p0, nfb);
    if (nfb) {
      ProfScope ps(ctx, kFamCov);
      if (ctx->knn_wave && nfb <= kWaveKnnMax)
        HIPCK(launch_knn_wave(cl.view, ctx->prm.k, ctx->prm.gicp_eps, ctx->knn_fb.p, nullptr, nfb, cl.cov3(), ctx->stream));
      else
        HIPCK(launch_knn_cov(cl.view, ctx->prm.k, ctx->prm.gicp_eps, 0, nfb, cl.cov3(), ctx->knn_fb.p, nullptr,
                             nullptr, ctx->stream));
    }
  }
  int rc = sync(ctx);
  if (rc) return rc;
#if defined(MGICP_CORR_PHASES) && MGICP_CORR_PHASES
  {
    unsigned long long ph[24];
    HIPCK(corr_phase_take(ph));
    if (ph[0])
      std::fprintf(stderr, "[knnb] waves %llu staged %llu (non-monotone %llu, over the cap %llu) | per wave: union points %.1f, "
                   "pieces %.1f, block candidates mean lane %.1f busiest lane %.1f | lanes past the block %llu, hand-offs %llu "
                   "of %llu\n", ph[0], ph[1], ph[4], ph[5], double(ph[2]) / ph[0], double(ph[3]) / ph[0],
                   double(ph[6]) / ph[0] / 64.0, double(ph[7]) / ph[0], ph[8], ph[9], ph[10]);
    if (ph[0] && ph[1] && ph[0] > ph[1])
      std::fprintf(stderr, "[knnb] cycles per wave -- staged: setup %.0f, copy %.0f, passes %.0f | unstaged: setup %.0f, "
                   "passes %.0f\n", double(ph[11]) / ph[1], double(ph[12]) / ph[1], double(ph[13]) / ph[1],
                   double(ph[15]) / (ph[0] - ph[1]), double(ph[16]) / (ph[0] - ph[1]));
    const double w = ph[21] ? static_cast<double>(ph[21]) : 1.0;
    std::fprintf(stderr, "[knn-div] waves %llu | per wave: test iterations %.1f, max lane tests %.1f, mean lane tests %.1f"
                 " | cycles/wave search %.0f, moments + finish %.0f\n",
                 ph[21], ph[18] / w, ph[19] / w, ph[20] / w / 64.0, ph[22] / w, ph[23] / w);
  }
#endif
  MGICP_TRACE_AT("cov: done");
  cl.have_cov = true;
  cl.cov_p0 = p0;
  cl.cov_p1 = p1;
  return MGICP_OK;
}

// target covariances (computeCovariances on the target, once per target cloud).  Multi-GPU
// (SURVEY.md 8e): rank r computes the r-th of N equal slices and one in-place all-gather per
// covariance array (48 bytes per point in total) completes every rank's copy -- the values are
// per point, so the result is the single-GPU one bit for bit.
int target_cov(mgicp_ctx* ctx) {
  Cloud& t = ctx->tgt;
  if (!ctx->comm || ctx->nranks < 2 || !ctx->split_target_cov) return compute_cov(ctx, t, 0, t.n);
  const size_t N = static_cast<size_t>(ctx->nranks), r = static_cast<size_t>(ctx->rank);
  const size_t cnt = (t.n + N - 1) / N;
  int rc = compute_cov(ctx, t, std::min(t.n, r * cnt), std::min(t.n, (r + 1) * cnt), N * cnt);
  if (rc) return rc;
  const Cov3 c = t.cov3();
  NCCLCK(ncclGroupStart());
  for (double2* a : {c.a, c.b, c.c})
    NCCLCK(ncclAllGather(a + r * cnt, a, 2 * cnt, ncclDouble, ctx->comm, ctx->stream));
  NCCLCK(ncclGroupEnd());
  if ((rc = sync(ctx))) return rc;
  t.cov_p0 = 0;
  t.cov_p1 = t.n;
  return MGICP_OK;
}

// Registration::initCompute + initComputeReciprocal + computeCovariances (both clouds)
int prepare(mgicp_ctx* ctx, bool need_cov) {
  if (ctx->src.n == 0 || ctx->tgt.n == 0)
    return fail(ctx, MGICP_E_INVALID, "source and target clouds must be set before align");
  const int k = ctx->prm.k;
  if (static_cast<size_t>(k) > ctx->src.n || static_cast<size_t>(k) > ctx->tgt.n)
    return fail(ctx, MGICP_E_TOO_FEW_POINTS,
                "a cloud has fewer points than k_correspondences (PCL computeCovariances)");
  int rc;
  if (ctx->tgt.dirty && (rc = build_grid(ctx, ctx->tgt))) return rc;
  if (ctx->src.dirty && (rc = build_grid(ctx, ctx->src))) return rc;
  if (!need_cov) return MGICP_OK;
  // set_target's covariances still running count as current: the first sweep runs beside them and
  // joins them before its compaction (r05: the 1-NN search needs no covariance)
  if (!ctx->tgt.have_cov && !ctx->tgt_cov_pending && (rc = target_cov(ctx))) return rc;
  // set_source's covariances still running count as current: the sweep joins them (overlapped)
  const bool src_cur = ctx->src_cov_pending ||
                       (ctx->src.have_cov && ctx->src.cov_p0 == ctx->shard_p0() && ctx->src.cov_p1 == ctx->shard_p1());
  if (ctx->lazy_src_cov && !src_cur) {
    // computed per sweep for the points it accepts (cov_lazy); here only sized and marked empty
    if (!ctx->src_lazy_ready || ctx->src_lazy_p0 != ctx->shard_p0() || ctx->src_lazy_p1 != ctx->shard_p1()) {
      Cloud& c = ctx->src;
      const size_t ns = ctx->shard_p1() - ctx->shard_p0();
      HIPCK(c.cov.reserve(3 * c.n));
      c.cov_stride = c.n;
      HIPCK(ctx->cov_ok.reserve(std::max<size_t>(ns, 1)));
      HIPCK(ctx->cov_need.reserve(std::max<size_t>(ns, 1)));
      HIPCK(hipMemsetAsync(ctx->cov_ok.p, 0, std::max<size_t>(ns, 1), ctx->stream));
      ctx->src_lazy_ready = true;
      ctx->src_lazy_p0 = ctx->shard_p0();
      ctx->src_lazy_p1 = ctx->shard_p1();
    }
    return MGICP_OK;
  }
  if (!src_cur)
    if ((rc = compute_cov(ctx, ctx->src, ctx->shard_p0(), ctx->shard_p1()))) return rc;
  return MGICP_OK;
}

// the covariances a sweep needs (lazy source mode): its accepted source points without one, computed
// by the same kernels as the eager pass (the k-NN kernel, the register-list hand-off for the rest)
int cov_lazy(mgicp_ctx* ctx) {
  if (!ctx->lazy_src_cov || ctx->src.have_cov) return MGICP_OK;
  const size_t p0 = ctx->shard_p0(), ns = ctx->shard_p1() - p0;
  HIPCK(ctx->u64.reserve(1));
  unsigned int* cnt = reinterpret_cast<unsigned int*>(ctx->u64.p);  // [0] points to compute, [1] hand-offs
  HIPCK(hipMemsetAsync(cnt, 0, 2 * sizeof(unsigned int), ctx->stream));
  HIPCK(launch_cov_need(ctx->flags.p, ctx->cov_ok.p, p0, ns, ctx->cov_need.p, cnt, ctx->stream));
  HIPCK(hipMemcpyAsync(ctx->h_small, cnt, sizeof(unsigned int), hipMemcpyDeviceToHost, ctx->stream));
  int rc = sync(ctx);
  if (rc) return rc;
  unsigned int need = 0;
  std::memcpy(&need, ctx->h_small, sizeof(need));
  if (knn_stats_on()) std::fprintf(stderr, "[knn-lazy] source covariances to compute for this sweep: %u\n", need);
  if (!need) return MGICP_OK;
  // r06: few points (after the head start: mostly the isolated ones its ring cap left -- C4F's debris and
  // clutter near the part, 21k in the first sweep) run one wave each, so their long ring searches do not
  // leave a few per-lane waves as the launch's tail (C4F: 5 ms -> 0.9 ms); a bulk list (the synchronous
  // path -- N > 1 ranks, profiling -- where the first sweep needs every source covariance) keeps the
  // per-lane kernels, 64 points per wave
  if (ctx->knn_wave && need <= kWaveKnnMax) {
    ProfScope ps(ctx, kFamCov);
    HIPCK(launch_knn_wave(ctx->src.view, ctx->prm.k, ctx->prm.gicp_eps, ctx->cov_need.p, nullptr, need, ctx->src.cov3(),
                          ctx->stream));
    return MGICP_OK;
  }
  const bool logged = ctx->knn_logged;
  if (logged) HIPCK(ctx->knn_fb.reserve(need));
  {
    ProfScope ps(ctx, kFamCov);
    HIPCK(launch_knn_cov(ctx->src.view, ctx->prm.k, ctx->prm.gicp_eps, 0, need, ctx->src.cov3(), ctx->cov_need.p,
                         logged ? ctx->knn_fb.p : nullptr, logged ? cnt + 1 : nullptr, ctx->stream));
  }
  if (logged) {
    HIPCK(hipMemcpyAsync(ctx->h_small, cnt + 1, sizeof(unsigned int), hipMemcpyDeviceToHost, ctx->stream));
    if ((rc = sync(ctx))) return rc;
    unsigned int nfb = 0;
    std::memcpy(&nfb, ctx->h_small, sizeof(nfb));
    ctx->knn_fallbacks = nfb;
    ProfScope ps(ctx, kFamCov);
    if (nfb)
      HIPCK(launch_knn_cov(ctx->src.view, ctx->prm.k, ctx->prm.gicp_eps, 0, nfb, ctx->src.cov3(), ctx->knn_fb.p, nullptr,
                           nullptr, ctx->stream));
  }
  return MGICP_OK;
}

int ensure_host_red(mgicp_ctx* ctx) {
  if (!ctx->h_cmd) {
    HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_cmd), sizeof(PassCmd),
                        hipHostMallocMapped | hipHostMallocCoherent));
    HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_cmd), ctx->h_cmd, 0));
    std::memset(ctx->h_cmd, 0, sizeof(PassCmd));
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) != hipSuccess || khz <= 0)
      khz = 100000;  // 100 MHz: the gfx9 constant wall clock
    ctx->gate_timeout = static_cast<unsigned long long>(khz) * 1000ull * 10ull;  // 10 s
    HIPCK(hipMalloc(reinterpret_cast<void**>(&ctx->mail), sizeof(PassCmd)));
    HIPCK(hipMemsetAsync(ctx->mail, 0, sizeof(PassCmd), ctx->stream));
    // host stores into device memory need the whole VRAM behind the PCIe BAR (large BAR); without
    // it block 0 polls the pinned copy
    hipDeviceProp_t prop;
    const bool large_bar = hipGetDeviceProperties(&prop, ctx->device) == hipSuccess && prop.isLargeBar;
    if (ctx->bar && large_bar && !ctx->bar_cmd) {
      if (hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->bar_cmd), sizeof(PassCmd), hipDeviceMallocFinegrained) !=
          hipSuccess)
        ctx->bar_cmd = nullptr;  // no host-writable device memory: block 0 polls the pinned copy
      else
        HIPCK(hipMemset(ctx->bar_cmd, 0, sizeof(PassCmd)));  // complete before the host's first store
    }
#if MGICP_PASS_DIAG
    // diagnostic builds (make variant DEFS=-DMGICP_PASS_DIAG=1): per-pass device / host timestamps of
    // the resident server and of the gated passes, summarised on stderr at the end of every align
    {
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_ptimes), 2 * 1024 * sizeof(unsigned long long),
                          hipHostMallocMapped | hipHostMallocCoherent));
      HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_ptimes), ctx->h_ptimes, 0));
      std::memset(ctx->h_ptimes, 0, 2 * 1024 * sizeof(unsigned long long));
    }
    {
      HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_gtrace), 4 * 1024 * sizeof(unsigned long long),
                          hipHostMallocMapped | hipHostMallocCoherent));
      HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_gtrace), ctx->h_gtrace, 0));
      std::memset(ctx->h_gtrace, 0, 4 * 1024 * sizeof(unsigned long long));
      ctx->host_gt.assign(2 * 1024, 0.0);
    }
#endif
  }
  if (ctx->h_red) return MGICP_OK;
  // kRedVals sums followed by the pass-completion word (see launch_fdf_soa's done_flag)
  HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_red), 2 * kRedVals * sizeof(double),
                      hipHostMallocMapped | hipHostMallocCoherent));
  HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_h_red), ctx->h_red, 0));
  std::memset(ctx->h_red, 0, 2 * kRedVals * sizeof(double));
  ctx->h_flag = reinterpret_cast<unsigned long long*>(ctx->h_red + kRedVals);
  ctx->d_flag = reinterpret_cast<unsigned long long*>(ctx->d_h_red + kRedVals);
  return MGICP_OK;
}

// Wait for pass `seq` to publish its sums: spin on the mapped completion word; after ~0.5 s fall
// back to a stream synchronisation so a failed launch surfaces as an error instead of a hang.
int wait_pass(mgicp_ctx* ctx, unsigned long long seq) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spins = 0;; ++spins) {
    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) == seq) return MGICP_OK;
    if ((spins & 1023u) == 1023u &&
        std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500))
      break;
  }
  int rc = sync(ctx);
  if (rc) return rc;
  if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) != seq)
    return fail(ctx, MGICP_E_HIP, "objective pass finished without publishing its sums");
  return MGICP_OK;
}

CorrSoA corr_soa(mgicp_ctx* ctx);

// Where the host rows of the passes live: this context's private pinned buffers (single rank), or
// the node-wide shared segment (every rank's rows at their global super index).  Parity buffer p
// starts stride words after parity 0; this rank's rows start at super `first`.
struct RowView {
  unsigned long long* h0 = nullptr;  // host view, parity 0, super 0
  unsigned long long* d0 = nullptr;  // device view, parity 0, super 0
  size_t stride = 0;                 // words between the parity buffers
  long long first = 0, nloc = 0, ntot = 0;
  unsigned long long* dev_rows(unsigned int rstamp) const {  // this rank's rows of the pass stamped rstamp
    return d0 + (rstamp & 1u) * stride + static_cast<size_t>(first) * shm::kRowWords;
  }
};

RowView row_view(const mgicp_ctx* ctx) {
  RowView v;
  if (ctx->have_shm) {
    v.h0 = reinterpret_cast<unsigned long long*>(ctx->shm.rows(0));
    v.d0 = reinterpret_cast<unsigned long long*>(ctx->shm_d + ctx->shm.rows_offset_bytes());
    v.stride = ctx->shm.rows_stride_words();
    v.ntot = ctx->nsup_total();
    v.first = super_first(ctx->rank, v.ntot, ctx->nranks);
    v.nloc = ctx->nsup_local();
  } else {
    v.h0 = ctx->h_rows;
    v.d0 = ctx->d_rows;
    v.stride = ctx->rows_cap * shm::kRowWords;
    v.ntot = v.nloc = ctx->nsup_local();
  }
  return v;
}

// Host rows for the current source cloud: the private buffers grow as needed (two parity buffers);
// the shared segment was sized at attach time.
int ensure_rows(mgicp_ctx* ctx) {
  const long long nsup = ctx->nsup_total();
  if (ctx->have_shm) {
    if (nsup > ctx->shm.max_sup)
      return fail(ctx, MGICP_E_INVALID, "source cloud larger than the shared row segment (mgicp_comm_attach_shm "
                                        "max_source_points)");
    return MGICP_OK;
  }
  if (ctx->h_rows && ctx->rows_cap >= static_cast<size_t>(nsup)) return MGICP_OK;
  if (ctx->h_rows) {
    int rc = sync(ctx);  // no server of an earlier run may still hold the old rows
    if (rc) return rc;
    HIPCK(hipHostFree(ctx->h_rows));
  }
  ctx->h_rows = nullptr;
  const size_t cap = static_cast<size_t>(std::max<long long>(nsup, 64));
  const size_t bytes = 2 * cap * shm::kRowWords * sizeof(unsigned long long);
  HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_rows), bytes, hipHostMallocMapped | hipHostMallocCoherent));
  HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_rows), ctx->h_rows, 0));
  std::memset(ctx->h_rows, 0, bytes);  // stamp 0 is never a pass's stamp
  ctx->rows_cap = cap;
  ctx->st[kStRowsAlloc]++;
  return MGICP_OK;
}

// A server pass missed its deadline (its blocks could not all run: other work on the device, a
// profiler, a withheld block in the tests): cancel the server -- blocks still waiting see the later
// command and exit, blocks that start late exit at their first gate -- and re-run the pass as a
// launched kernel that writes the same rows with the same stamp (the sums are bitwise those of the
// server: same chunks, lane order and tree).  The rest of the align runs launched passes.
int take_over(mgicp_ctx* ctx, unsigned int rstamp, const Xf34& A) {
  cancel_gated(ctx);  // tickets re-armed on the stream after the server has exited
  ctx->srv_degraded = true;
  ctx->st[kStTakeover]++;
  ctx->st[kStLaunchedPass]++;
  const size_t ns = ctx->shard_p1() - ctx->shard_p0();
  HIPCK(launch_fdf_soa(corr_soa(ctx), ctx->ccnt.p, ns, A, ctx->partial.p, ctx->spart.p,
                       fdf_grid_blocks(ns, ctx->fdf_max_blocks), ctx->tickets.p, nullptr, 0, nullptr, 0, ctx->stream,
                       row_view(ctx).dev_rows(rstamp), rstamp));
  // host-row passes leave the tickets as multiples of their supers' sizes: re-arm them for whatever
  // form the next pass takes
  HIPCK(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream));
  return MGICP_OK;
}

// Wait for every host row of the pass stamped rstamp (32 stamped words per super: this rank's own
// rows first, then the other ranks'), then take the total exactly as wave_total / wave_sum would on
// one wave (shm::fixed_total).  Own rows missing after row_deadline_ms: the pass is taken over
// (take_over, when allowed) and waited for again; after a stream drain every row is checked once
// more before an error is returned.  Other ranks' rows: remote_deadline_s.
int wait_rows(mgicp_ctx* ctx, unsigned int rstamp, const Xf34& A, double out[kRedVals], bool allow_takeover) {
  const RowView rv = row_view(ctx);
  const unsigned long long* buf = rv.h0 + (rstamp & 1u) * rv.stride;
  ctx->row_sums.resize(static_cast<size_t>(std::max<long long>(rv.ntot, 1)) * kRedVals);
  auto t0 = std::chrono::steady_clock::now();
  bool taken = false;
  const double dl_own = ctx->row_deadline_ms * 1e-3;
  auto wait_row = [&](long long r, bool own) -> int {
    const unsigned long long* row = buf + shm::kRowWords * static_cast<size_t>(r);
    for (unsigned spins = 0; !shm::row_complete(reinterpret_cast<const uint64_t*>(row), rstamp); ++spins) {
      if (ctx->spin_pause) __builtin_ia32_pause();
      if ((spins & 1023u) != 1023u) continue;
      const double el = shm::elapsed_s(t0);
      if (own && !taken && allow_takeover && el > dl_own) {
        int rc = take_over(ctx, rstamp, A);
        if (rc) return rc;
        taken = true;
        t0 = std::chrono::steady_clock::now();
        continue;
      }
      if (own && el > (taken ? ctx->remote_deadline_s : dl_own)) {
        int rc = sync(ctx);  // drains the stream (and cancels a live server): the rows are final now
        if (rc) return rc;
        if (shm::row_complete(reinterpret_cast<const uint64_t*>(row), rstamp)) break;
        char msg[192];
        std::snprintf(msg, sizeof(msg),
                      "objective pass finished without publishing its super rows (row %lld of %lld: stamp %08x "
                      "expected, words 0 / 31 carry %08x / %08x)",
                      r, rv.nloc, rstamp, static_cast<unsigned int>(row[0] >> 32),
                      static_cast<unsigned int>(row[31] >> 32));
        return fail(ctx, MGICP_E_HIP, msg);
      }
      if (!own && el > ctx->remote_deadline_s)
        return fail(ctx, MGICP_E_COMM, "another rank did not publish its super rows (shared row segment)");
    }
    shm::row_decode(reinterpret_cast<const uint64_t*>(row), &ctx->row_sums[static_cast<size_t>(r) * kRedVals]);
    return MGICP_OK;
  };
  for (long long r = rv.first; r < rv.first + rv.nloc; ++r) {
    int rc = wait_row(r, true);
    if (rc) return rc;
  }
  t0 = std::chrono::steady_clock::now();
  for (long long r = 0; r < rv.ntot; ++r) {
    if (r >= rv.first && r < rv.first + rv.nloc) continue;
    int rc = wait_row(r, false);
    if (rc) return rc;
  }
  shm::fixed_total(ctx->row_sums.data(), rv.ntot, kRedVals, out);
  return MGICP_OK;
}

// r05 xGMI: the pass total the rank's totaler stored (every rank's rows arrived in its buffer)
int wait_xtot(mgicp_ctx* ctx, unsigned int rstamp, double out[kRedVals]) {
  const auto t0 = std::chrono::steady_clock::now();
  const uint64_t* row = reinterpret_cast<const uint64_t*>(ctx->h_xtot);
  for (unsigned spins = 0; !shm::row_complete(row, rstamp); ++spins) {
    if ((spins & 1023u) == 1023u && shm::elapsed_s(t0) > ctx->remote_deadline_s)
      return fail(ctx, MGICP_E_COMM, "xGMI row exchange: the pass total did not complete (a rank stopped publishing)");
  }
  shm::row_decode(row, out);
  return MGICP_OK;
}

int ensure_iter_buffers(mgicp_ctx* ctx) {
  const size_t ns = ctx->shard_p1() - ctx->shard_p0();
  const size_t nch = static_cast<size_t>(chunk_count(ns));
  const size_t msup = static_cast<size_t>(ctx->max_supers());
  HIPCK(ctx->partial.reserve(std::max<size_t>(nch, 1) * kRedVals));
  if (ctx->tpart_n < std::max<size_t>(nch, 1) * 32) {  // stamps 0xffffffff: never a pass's stamp
    HIPCK(ctx->tpart.reserve(std::max<size_t>(nch, 1) * 32));
    HIPCK(hipMemsetAsync(ctx->tpart.p, 0xff, ctx->tpart.cap * sizeof(unsigned long long), ctx->stream));
    ctx->tpart_n = ctx->tpart.cap;
  }
  HIPCK(ctx->spart.reserve(std::max<size_t>(msup, 1) * kRedVals));
  HIPCK(ctx->ccnt.reserve(std::max<size_t>(nch, 1)));
  HIPCK(ctx->red.reserve(kRedVals));
  if (ctx->tickets_n < msup + 1) {  // zero between passes: every finishing wave re-arms its own
    HIPCK(ctx->tickets.reserve(msup + 1));
    HIPCK(hipMemsetAsync(ctx->tickets.p, 0, (msup + 1) * sizeof(unsigned int), ctx->stream));
    ctx->tickets_n = msup + 1;
  }
  int rc = ensure_host_red(ctx);
  if (rc) return rc;
  // fixed slots: chunk c's run starts at c * kChunkPts (padded to a multiple of 4 within the chunk)
  const size_t cap = std::max<size_t>(nch, 1) * kChunkPts;
  HIPCK(ctx->prev_pos.reserve(ns + 1));
  HIPCK(ctx->flags.reserve(ns + 1));
  if (ctx->corr_cap < cap) {
    HIPCK(ctx->corr_f.reserve(6 * cap));
    HIPCK(ctx->corr_d.reserve(6 * cap));
    ctx->corr_cap = cap;
  }
  return MGICP_OK;
}

// totals (nv values) of the shard's super partials `sup`: all-gathered across ranks over RCCL and
// finished in the fixed global order (launch_finish_supers), or -- single rank or detached shard
// -- finished over this shard's own supers
int combine_supers(mgicp_ctx* ctx, int nv, const double* sup, double* out) {
  if (ctx->comm) {
    const long long msup = ctx->max_supers();
    HIPCK(ctx->gath.reserve(static_cast<size_t>(ctx->nranks) * msup * nv));
    NCCLCK(ncclAllGather(sup, ctx->gath.p, static_cast<size_t>(msup) * nv, ncclDouble, ctx->comm, ctx->stream));
    HIPCK(launch_finish_supers(ctx->gath.p, ctx->nsup_total(), msup, ctx->nranks, nv, out, ctx->stream));
  } else {
    const long long ns = ctx->nsup_local();
    HIPCK(launch_finish_supers(sup, ns, ns, 1, nv, out, ctx->stream));
  }
  return MGICP_OK;
}

// The same totals delivered to the host (GN moments once per outer iteration, fitness once per
// call).  With the shared segment: a generic gather -- this rank copies its supers to their global
// rows of the gather's parity buffer, publishes the gather index and waits for every rank's, and
// every host takes the fixed-order total itself (no collective).  Otherwise combine_supers + D2H.
int combine_to_host(mgicp_ctx* ctx, int nv, const double* sup, double* out) {
  if (ctx->have_shm) {
    const unsigned long long g = ++ctx->gather_idx;
    double* buf = ctx->shm.gath(static_cast<int>(g & 1));
    const long long ntot = ctx->nsup_total();
    const long long first = super_first(ctx->rank, ntot, ctx->nranks), nloc = ctx->nsup_local();
    if (nloc > 0)
      HIPCK(hipMemcpyAsync(buf + static_cast<size_t>(first) * nv, sup, static_cast<size_t>(nloc) * nv * sizeof(double),
                           hipMemcpyDeviceToHost, ctx->stream));
    int rc = sync(ctx);
    if (rc) return rc;
    if (!shm::gather_publish_wait(ctx->shm, g, ctx->remote_deadline_s))
      return fail(ctx, MGICP_E_COMM, "another rank did not publish its supers (shared segment gather)");
    // the gather rows are packed nv per super: fixed_total reads rows[s * nv + v]
    shm::fixed_total(buf, ntot, nv, out);
    return MGICP_OK;
  }
  double* dst = nv == kRedVals ? ctx->red.p : ctx->mred.p;
  int rc = combine_supers(ctx, nv, sup, dst);
  if (rc) return rc;
  HIPCK(hipMemcpyAsync(ctx->h_small, dst, static_cast<size_t>(nv) * sizeof(double), hipMemcpyDeviceToHost,
                       ctx->stream));
  if ((rc = sync(ctx))) return rc;
  std::memcpy(out, ctx->h_small, static_cast<size_t>(nv) * sizeof(double));
  return MGICP_OK;
}

// guess-applied source cloud ("output" after transformPointCloud(output, output, guess))
int set_output(mgicp_ctx* ctx, const Mat4& G) {
  float lo[3], hi[3];
  if (G.is_identity()) {
    ctx->d_out = ctx->src.pts.p;  // x*1 + y*0 + z*0 + 0 == x: identity leaves points intact
    for (int d = 0; d < 3; ++d) {
      lo[d] = ctx->src.lo[d];
      hi[d] = ctx->src.hi[d];
    }
  } else {
    HIPCK(ctx->src_out.reserve(ctx->src.n));
    HIPCK(launch_xform_points(ctx->src.pts.p, ctx->src.n, G.xf(), ctx->src_out.p, ctx->stream));
    ctx->d_out = ctx->src_out.p;
    // bbox of the transformed cloud (the Gauss-Newton expansion centre)
    const size_t n = ctx->src.n;
    const int nb = static_cast<int>(std::min<size_t>((n + 255) / 256, 1024));
    HIPCK(launch_bbox(ctx->src_out.p, n, reinterpret_cast<float*>(ctx->d_small), nb, ctx->stream));
    int rc = sync(ctx);
    if (rc) return rc;
    const float* hp = reinterpret_cast<const float*>(ctx->h_small);
    for (int d = 0; d < 3; ++d) {
      lo[d] = INFINITY;
      hi[d] = -INFINITY;
    }
    for (int b = 0; b < nb; ++b)
      for (int d = 0; d < 3; ++d) {
        lo[d] = std::min(lo[d], hp[b * 8 + d]);
        hi[d] = std::max(hi[d], hp[b * 8 + 3 + d]);
      }
  }
  for (int d = 0; d < 3; ++d) ctx->out_ctr[d] = static_cast<double>(0.5f * (lo[d] + hi[d]));
  ctx->last_guess = G;
  return MGICP_OK;
}

// transform_R(i,j) = sum_k double(T(i,k)) * double(G(k,j)), top-left 3x3
Rot33d rot_of(const Mat4& T, const Mat4& G) {
  Rot33d R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      double a = 0.0;
      for (int k = 0; k < 4; ++k) a += static_cast<double>(T.m[i][k]) * static_cast<double>(G.m[k][j]);
      R.m[3 * i + j] = a;
    }
  return R;
}

CorrSoA corr_soa(mgicp_ctx* ctx) {
  const size_t c = ctx->corr_cap;
  float* f = ctx->corr_f.p;
  double* d = ctx->corr_d.p;
  return CorrSoA{f, f + c, f + 2 * c, f + 3 * c, f + 4 * c, f + 5 * c,
                 d, d + c, d + 2 * c, d + 3 * c, d + 4 * c, d + 5 * c};
}

// The fine grid of the target's 1-NN cell lists for the current gate (once per target grid and gate;
// the lists themselves are built by the sweeps, cell by cell, the first time a query lands in a cell).
// The grid covers the target's bbox grown by the gate + 2 cells, so a query outside it is farther than
// the gate from every target point; cells of vlist_cell x the target grid's cell edge, fewer than 2^28
// cells (else the lists are off for this gate: the r03 sweeps).
int vl_prepare(mgicp_ctx* ctx) {
  const double gate = ctx->prm.max_corr_dist;
  const size_t ns = ctx->shard_p1() - ctx->shard_p0();
  if (!(ctx->vl_valid && ctx->vl.gate == gate)) {
    ctx->vl_valid = false;
    ctx->vl_off = false;
    const Cloud& t = ctx->tgt;
    const double h = t.view.h;
    double c = std::max(h * static_cast<double>(ctx->vlist_cell), 1e-6);
    double ext = 0, maxabs = 0;
    for (int d = 0; d < 3; ++d) {
      ext = std::max(ext, static_cast<double>(t.hi[d] - t.lo[d]));
      maxabs = std::max(maxabs, std::max(std::fabs(static_cast<double>(t.lo[d])), std::fabs(static_cast<double>(t.hi[d]))));
    }
    constexpr size_t kVlMaxCells = size_t(1) << 28;
    int nd[3] = {0, 0, 0};
    double pad = 0;
    for (int it = 0; it < 64; ++it) {
      pad = gate * (1.0 + 1e-5) + 1e-9 + 2.0 * c;
      size_t nc = 1;
      for (int d = 0; d < 3; ++d) {
        nd[d] = static_cast<int>(std::floor((static_cast<double>(t.hi[d] - t.lo[d]) + 2.0 * pad) / c)) + 1;
        nc *= static_cast<size_t>(nd[d]);
      }
      if (nc <= kVlMaxCells) break;
      c *= std::cbrt(static_cast<double>(nc) / kVlMaxCells) * 1.01;
    }
    ctx->vl.gate = gate;
    if (c > 4.0 * std::max(h, 1e-6)) {  // a gate this wide against this target: lists would overflow
      ctx->vl_off = true;
      ctx->vl_valid = true;
      return MGICP_OK;
    }
    const size_t nc = static_cast<size_t>(nd[0]) * nd[1] * nd[2];
    VListView& v = ctx->vl;
    v.ox = static_cast<float>(t.lo[0] - pad);
    v.oy = static_cast<float>(t.lo[1] - pad);
    v.oz = static_cast<float>(t.lo[2] - pad);
    v.c = static_cast<float>(c);
    v.inv_c = static_cast<float>(1.0 / c);
    // the fp32 cell assignment floor((q - o) * inv_c) of a query: a few ulps of the coordinates
    // and of the cell count, covered with a wide margin
    v.es = static_cast<float>(3.0e-6 * (maxabs + pad + ext) + 1e-4 * c);
    v.nx = nd[0];
    v.ny = nd[1];
    v.nz = nd[2];
    ctx->vl_ncells = nc;
    ctx->vl_valid = true;
    ctx->vl_alloc = false;
    ctx->vl_epoch = 0;
    ctx->vl_groups = 0;
  }
  // the state words and the pool (~0.4 + 2 GB at C4) only once a sweep uses the lists: the first align
  // after a set_target runs the r03 sweep and must not pay for their allocation (r04)
  if (!ctx->vl_off && !ctx->vl_alloc && ctx->vl_groups >= ctx->vl_cold_groups) {
    const Cloud& t = ctx->tgt;
    VListView& v = ctx->vl;
    const size_t nc = ctx->vl_ncells;
    HIPCK(ctx->vl_cell.reserve(nc));
    HIPCK(hipMemsetAsync(ctx->vl_cell.p, 0xff, nc * sizeof(uint32_t), ctx->stream));
    // list starts are stored in units of 4 entries in 25 bits: at most 2^27 entries (16 bytes each)
    const size_t cap = std::min<size_t>(size_t(1) << 27, std::max<size_t>(size_t(1) << 22, 32 * t.n));
    HIPCK(ctx->vl_pool.reserve(cap));
    HIPCK(ctx->vl_ctr.reserve(8));  // [4]: the build's second-pass cells (r06)
    HIPCK(hipMemsetAsync(ctx->vl_ctr.p, 0, 8 * sizeof(unsigned int), ctx->stream));
    v.cell = ctx->vl_cell.p;
    v.pool = ctx->vl_pool.p;
    v.pool_cap = static_cast<uint32_t>(cap);
    v.ctr = ctx->vl_ctr.p;
    ctx->vl_alloc = true;
  }
  if (ctx->vl_off || !ctx->vl_alloc) return MGICP_OK;
  // per-sweep lists sized by the shard (one request / pending entry per query at most)
  const size_t q = std::max<size_t>(ns, 1);
  HIPCK(ctx->vl_build.reserve(q));
  HIPCK(ctx->vl_bcentre.reserve(q));
  HIPCK(ctx->vl_pend.reserve(q));
  ctx->vl.build = ctx->vl_build.p;
  ctx->vl.bcentre = ctx->vl_bcentre.p;
  ctx->vl.build_cap = static_cast<uint32_t>(std::min(ctx->vl_build.cap, ctx->vl_ncells));
  ctx->vl.pend = ctx->vl_pend.p;
  if (++ctx->vl_epoch >= 0x40000000u) {  // epochs wrap: every touched mark then reads as "earlier sweep"
    ctx->vl_epoch = 1;
  }
  ctx->vl.epoch = ctx->vl_epoch;
  ctx->vl.eager = ctx->vl_eager ? 1 : 0;
  ctx->vl.tpts = ctx->tgt.pts.p;
  return MGICP_OK;
}

// The 1-NN sweep kernel of one correspondence phase: the target's cell lists (r04, default), else the
// wave-uniform scan (debug option "vlist" 0, and the first aligns after a set_target); exact, same
// results.
bool sweep_listed(const mgicp_ctx* ctx) {
  return ctx->vlist && ctx->vl_valid && ctx->vl_alloc && !ctx->vl_off && ctx->vl_groups >= ctx->vl_cold_groups;
}

// fc (nullable, listed sweeps only): the compaction fused into the sweep
hipError_t launch_sweep(mgicp_ctx* ctx, const Mat4& T, double thr, bool seeded, const uint32_t* qp,
                        const FusedCompact* fc = nullptr) {
  const size_t p0 = ctx->shard_p0(), p1 = ctx->shard_p1();
  const GridView& g = ctx->tgt.view;
  if (sweep_listed(ctx))
    return launch_vl_sweep(g, ctx->vl, ctx->d_out, p0, p1, T.xf(), thr, seeded ? 1 : 0, ctx->prev_pos.p, ctx->flags.p,
                           ctx->cus, ctx->stream, fc);
  if (ctx->corr_wave && g.pairs) {
    const float rc = ctx->corr_rcap * g.h;
    void* work = nullptr;
    if (ctx->corr_split > 0) {
      hipError_t e = ctx->nn_work.reserve(nn_work_bytes(p1 - p0));
      if (e == hipSuccess) e = ctx->nn_work_n.reserve(1);
      if (e != hipSuccess) return e;
      work = ctx->nn_work.p;
    }
    return launch_correspond_wave(g, ctx->d_out, p0, p1, T.xf(), thr, seeded ? 1 : 0, ctx->prev_pos.p,
                                  ctx->flags.p, qp, rc * rc, ctx->corr_max_rows, ctx->corr_max_x, ctx->corr_union_min_r,
                                  work, ctx->nn_work_n.p, ctx->corr_split, ctx->corr_lds_pts, ctx->stream);
  }
  return launch_correspond(g, ctx->d_out, p0, p1, T.xf(), thr, seeded ? 1 : 0, ctx->prev_pos.p, ctx->flags.p, qp,
                           ctx->stream);
}

// One correspondence sweep (the loop body of computeTransformation before the BFGS call):
// exact 1-NN per source point, then a deterministic compaction of the accepted ones (exclusive
// scan of the flags, scatter in grid-sorted order) that computes their Mahalanobis matrices
// straight into the SoA streams.  `seed` uses the previous sweep's matches as 1-NN starting
// candidates (exact either way).
int correspond(mgicp_ctx* ctx, const Mat4& T, const Mat4& G, bool seed) {
  const double thr = ctx->prm.max_corr_dist * ctx->prm.max_corr_dist;
  const size_t p0 = ctx->shard_p0(), p1 = ctx->shard_p1(), ns = p1 - p0;
  hipStream_t s = ctx->stream;
  const bool seeded = seed && ctx->seed_valid;
  HIPCK(hipMemsetAsync(ctx->flags.p + ns, 0, sizeof(uint32_t), s));
  const uint32_t* qp = query_perm(ctx);
  MGICP_TRACE_AT("corr: query order ready");
  if (ctx->vlist) {
    int rc = vl_prepare(ctx);
    if (rc) return rc;
  }
  MGICP_TRACE_AT("corr: lists prepared");
  // the compaction fused into a listed sweep: both clouds' covariances must be complete (or, lazy
  // source mode, marked per point) -- not on the first align after set_*, which runs the r03 sweep
  const bool fused = ctx->fuse_compact && sweep_listed(ctx) && ctx->tgt.have_cov &&
                     !ctx->tgt_cov_pending && !ctx->src_cov_pending &&
                     (ctx->src.have_cov || (ctx->lazy_src_cov && ctx->src_lazy_ready));
  FusedCompact fc{};
  if (fused) {
    HIPCK(ctx->vl_defer.reserve(std::max(chunk_count(ns), 1)));
    fc.cov_s = ctx->src.cov3();
    fc.cov_t = ctx->tgt.cov3();
    fc.R = rot_of(T, G);
    fc.cov_ok = ctx->src.have_cov ? nullptr : ctx->cov_ok.p;
    fc.ccnt = ctx->ccnt.p;
    fc.defer = ctx->vl_defer.p;
    fc.out = corr_soa(ctx);
  }
  {
    ProfScope ps(ctx, kFamCorr);
    HIPCK(launch_sweep(ctx, T, thr, seeded, qp, fused ? &fc : nullptr));
  }
  ctx->seed_valid = true;
  MGICP_TRACE_AT("corr: sweep queued");
  if (ctx->vl_stats && sweep_listed(ctx)) {
    unsigned int c3[3];
    HIPCK(hipMemcpyAsync(c3, ctx->vl_ctr.p, 3 * sizeof(unsigned int), hipMemcpyDeviceToHost, s));
    HIPCK(ctx->u64.reserve(64));
    HIPCK(launch_vl_stats(ctx->vl, ctx->vl_ncells, ctx->u64.p, s));
    unsigned long long st[64];
    HIPCK(hipMemcpyAsync(st, ctx->u64.p, sizeof(st), hipMemcpyDeviceToHost, s));
    HIPCK(hipStreamSynchronize(s));
    double hist_mean = st[0] ? static_cast<double>(st[1]) / st[0] : 0.0;
    unsigned long long acc = 0, p95 = 0;
    for (int L = 0; L < 56; ++L) {
      acc += st[8 + L];
      if (!p95 && acc >= 0.95 * st[0]) p95 = L;
    }
    std::fprintf(stderr, "[vlist] cell %.3f mm grid %dx%dx%d | sweep: %u cells requested, %u queries pending | lists %llu "
                 "(mean %.1f, p95 %llu entries), reject %llu, overflow %llu, pool %u of %u\n",
                 1e3 * ctx->vl.c, ctx->vl.nx, ctx->vl.ny, ctx->vl.nz, c3[1], c3[2], st[0], hist_mean, p95, st[2], st[3],
                 c3[0], ctx->vl.pool_cap);
  }
#if defined(MGICP_VL_DIAG) && MGICP_VL_DIAG
  {
    unsigned long long ph[24];
    HIPCK(hipStreamSynchronize(s));
    HIPCK(corr_phase_take(ph));
    const double c = ph[0] ? static_cast<double>(ph[0]) : 1.0;
    if (ph[0] && sweep_listed(ctx))
      std::fprintf(stderr, "[vl-build] cells %llu | per cell: candidates %.1f, stage-1 survivors %.1f, kept %.1f | cycles/cell "
                   "gather %.0f, stage 1 %.0f, stage 2 %.0f | survivors <=8 %llu <=16 %llu <=32 %llu <=64 %llu <=128 %llu "
                   "<=256 %llu >256 %llu | stage-2 cycles of cells with > 64 survivors: %.1f %%\n",
                   ph[0], ph[1] / c, ph[2] / c, ph[3] / c, ph[4] / c, ph[5] / c, ph[6] / c, ph[9], ph[10], ph[11], ph[12],
                   ph[13], ph[14], ph[8], ph[6] ? 100.0 * ph[15] / ph[6] : 0.0);
  }
#elif defined(MGICP_CORR_PHASES) && MGICP_CORR_PHASES
  {
    unsigned long long ph[24];
    HIPCK(hipStreamSynchronize(s));
    HIPCK(corr_phase_take(ph));
    const double w = ph[7] ? static_cast<double>(ph[7]) : 1.0;
    std::fprintf(stderr, "[corr-phase] waves %llu (per-lane finish %llu) | cycles/wave seeds %.0f box %.0f scan %.0f "
                 "winner %.0f finish %.0f | waves by stragglers 0:%llu 1-4:%llu 5-16:%llu 17-63:%llu 64:%llu, "
                 "stragglers %llu | per-lane waves: none included %llu, rows %llu, x cells %llu, small balls %llu\n", ph[7],
                 ph[6], ph[0] / w, ph[1] / w, ph[2] / w, ph[3] / w, ph[4] / w, ph[8], ph[9], ph[10], ph[11], ph[12], ph[13],
                 ph[14], ph[15], ph[16], ph[17]);
  }
#endif
#if MGICP_CORR_STATS
  {
    unsigned long long st[8];
    HIPCK(hipStreamSynchronize(s));
    HIPCK(corr_stats_take(st));
    if (ctx->corr_wave && ctx->tgt.view.pairs)
      std::fprintf(stderr, "[corr-stats] wave scan: queries %llu accepted %llu rejected %llu | per-lane tests/query %.1f "
                   "ranges/query %.1f | lanes left to the per-lane search %llu | union-scan waves %llu of %llu, "
                   "candidates per union wave %.1f\n",
                   st[0], st[1], st[2], st[0] ? double(st[3]) / st[0] : 0.0, st[0] ? double(st[4]) / st[0] : 0.0, st[5],
                   st[7], (st[0] + 63) / 64, st[7] ? double(st[6]) / st[7] : 0.0);
    else
      std::fprintf(stderr, "[corr-stats] queries %llu accepted %llu rejected %llu | tests/query acc %.1f rej %.1f | ranges/query acc %.1f rej %.1f\n",
                   st[0], st[1], st[2], st[1] ? double(st[3]) / st[1] : 0.0, st[2] ? double(st[4]) / st[2] : 0.0,
                   st[1] ? double(st[5]) / st[1] : 0.0, st[2] ? double(st[6]) / st[2] : 0.0);
  }
#endif
  {
    int rc = cov_join_all(ctx);  // set_target's / set_source's covariances (they ran beside this sweep)
    if (rc) return rc;
    rc = cov_lazy(ctx);  // covariances of newly accepted source points (lazy source mode)
    MGICP_TRACE_AT("corr: lazy covariances queued (sweep drained)");
    if (rc) return rc;
  }
  {
    ProfScope ps(ctx, kFamCompact);
    // fused: only the chunks the sweep deferred (pending queries, lazy covariances computed above)
    HIPCK(launch_compact(ctx->d_out, ctx->tgt.view.pts, ctx->src.cov3(), ctx->tgt.cov3(), rot_of(T, G),
                         ctx->prev_pos.p, ctx->flags.p, p0, p1, ctx->ccnt.p, corr_soa(ctx), s,
                         fused ? ctx->vl_defer.p : nullptr, fused ? ctx->vl_ctr.p + 3 : nullptr, ctx->cus));
  }
  // no host round trip here: the correspondence count arrives with the first objective pass (its
  // count lane) and every consumer of the streams runs on the same stream
  ctx->have_corr = true;
  return MGICP_OK;
}

// OptimizationFunctorWithIndices::fdf on the device; memoises the last state
struct DeviceFunctor {
  mgicp_ctx* ctx;
  bool have_memo = false;
  Vec6 memo_x{};
  double memo_f = 0;
  Vec6 memo_g{};
  double m = 0;  // correspondences of this sweep (all ranks)

  int pass(const Vec6& x, double sums[kRedVals]) {
    const double t_entry = ctx->h_ptimes ? now_ms() : 0.0;
    const Mat4 A = apply_state(x);
    const size_t ns = ctx->shard_p1() - ctx->shard_p0();
    const int nb = fdf_grid_blocks(ns, ctx->fdf_max_blocks);
    int rc;
    // alternate the sweep direction so each pass starts on the Infinity-Cache-resident tail
    // of the previous one (deterministic: the sums do not depend on the direction)
    const int reverse = (ctx->alt_sweep ? (ctx->n_evals & 1) : 0) | ctx->fdf_diag;
    const bool poll = ctx->poll && !ctx->fdf_diag;
    // the pass's row stamp: the objective-pass index, identical on every rank (0 is never a stamp;
    // stamps >= 2^31 belong to mgicp_debug_pass_bench's timing form).  At the wrap every stamped
    // buffer is cleared and the count restarts at 1, so parity buffers keep alternating.
    if (ctx->pass_idx + 1 >= 0x80000000u && (rc = reset_stamps(ctx))) return rc;
    if (ctx->quit_pass >= 0 && ctx->pass_idx + 1 >= static_cast<unsigned int>(ctx->quit_pass))
      return fail(ctx, MGICP_E_COMM, "MGICP_DEBUG_QUIT_PASS: this rank stops publishing its rows");
    const unsigned long long seq = ++ctx->pass_seq;
    const unsigned int rstamp = ++ctx->pass_idx;
    // single GPU: the finishing wave writes the totals straight into mapped pinned host memory.
    // Shared row segment (any rank count): every pass -- server or launched -- writes its super rows
    // there and every host takes the total.  Otherwise (RCCL only) the pass leaves its super
    // partials, then combine_supers (RCCL all-gather + the fixed-order total) and a one-wave kernel
    // publishes the totals plus the completion word.
    const bool shm_rows = ctx->have_shm;
    const bool inlaunch = ctx->fused_finish && !ctx->comm && ctx->nranks == 1 && !shm_rows;
    double* out = inlaunch ? ctx->d_h_red : nullptr;
    const bool gate = ctx->gated && poll && inlaunch && !ctx->profiling;
    const Xf34 Ax = A.xf();
    const CorrSoA c = corr_soa(ctx);
    const bool want_srv = ctx->resident && !ctx->srv_degraded && !ctx->profiling && !ctx->fdf_diag &&
                          (gate || (shm_rows && ctx->poll));
    int cap = ctx->srv_cus > 0 ? std::min(ctx->srv_cus, ctx->cus) : ctx->cus;
    if (ctx->have_xgmi) cap = std::min(cap, ctx->cus - 1);  // one CU left to the totaler wave
    int nsrv = want_srv ? fdf_server_blocks(ns, cap, ctx->srv_waves) : 0;
    // the host rows first: a failure here (e.g. a source larger than the shared segment) must not
    // leave the device's server slot taken
    if (!ctx->srv_live && (shm_rows || (nsrv > 0 && ctx->host_rows)) && (rc = ensure_rows(ctx))) return rc;
    if (nsrv > 0 && !ctx->srv_live && !ctx->srv_locked) {
      int idle = 0;  // one server per device and process (g_srv_busy)
      ctx->srv_locked = g_srv_busy[ctx->device & 63].compare_exchange_strong(idle, 1, std::memory_order_acq_rel);
      if (!ctx->srv_locked) {
        nsrv = 0;
        ctx->st[kStSrvDenied]++;
      }
    }
    const bool rows = shm_rows || (nsrv > 0 && ctx->host_rows);
    const bool xg = ctx->have_xgmi;
    if (xg && nsrv <= 0)
      return fail(ctx, MGICP_E_COMM, "xGMI row exchange needs the resident pass server on every rank (the device's "
                                     "server slot is held by another context, or profiling is on)");
    if (nsrv > 0) {
      // the resident server runs every pass of this BFGS run: start it with the first one
      if (!ctx->srv_live) {
        cancel_gated(ctx);
        ctx->ht_last_rows = 0;  // host-view diagnostics: a new BFGS run, not a host step
        const RowView rv = row_view(ctx);
        // xGMI: rows into this rank's exchange buffer and every peer's, at the global super index
        PeerRows pr{};
        unsigned long long* xr = nullptr;
        if (xg) {
          xr = ctx->xrows.p + static_cast<size_t>(rv.first) * shm::kRowWords;
          pr.n = static_cast<int>(ctx->xpeer.size());
          for (int r = 0; r < pr.n; ++r)
            pr.p[r] = static_cast<unsigned long long*>(ctx->xpeer[r]) + static_cast<size_t>(rv.first) * shm::kRowWords;
        }
        hipEvent_t ea = ev_get(ctx);
        hipError_t e = hipEventRecord(ea, ctx->stream);
        if (e == hipSuccess) e = hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream);
        {
          ProfScope ps(ctx, kFamFdf);
          if (e == hipSuccess)
            e = launch_fdf_server(c, ctx->ccnt.p, ns, ctx->partial.p, ctx->spart.p, ctx->tickets.p,
                                  out, ctx->d_flag, seq, ctx->bar_cmd ? ctx->bar_cmd : ctx->d_cmd, ctx->mail,
                                  ctx->gate_timeout, ctx->d_ptimes, 0, Ax, xg ? xr : (rows ? rv.dev_rows(0) : nullptr),
                                  rv.stride, nsrv, ctx->srv_waves, ctx->bar_cmd ? nsrv : 1, ctx->stall_pass,
                                  ctx->srv_tagged ? ctx->tpart.p : nullptr, ctx->stream, xg ? &pr : nullptr);
          // the totaler of this BFGS run (its own stream; exits on the generation change of the cancel)
          if (e == hipSuccess && xg) {
            const unsigned int gen = ++ctx->xgen;
            __atomic_store_n(ctx->h_xgen, gen, __ATOMIC_RELEASE);
            e = launch_xgmi_total(ctx->xrows.p, rv.stride, rv.ntot, rstamp, ctx->d_xtot, ctx->d_xgen, gen,
                                  ctx->gate_timeout, ctx->xstream);
          }
        }
        hipEvent_t eb = nullptr;
        if (e == hipSuccess) {
          eb = ev_get(ctx);
          e = hipEventRecord(eb, ctx->stream);  // completes when the server exits (stream order)
        }
        if (e != hipSuccess) {
          g_srv_busy[ctx->device & 63].store(0, std::memory_order_release);
          ctx->srv_locked = false;
          ctx->pool.push_back(ea);
          if (eb) ctx->pool.push_back(eb);
          HIPCK(e);
        }
        ctx->srv_ev.push_back({ea, eb, 0});
        ctx->srv_live = true;
        ctx->st[kStSrvLaunch]++;
        ctx->st[kStBar] = ctx->bar_cmd ? 1 : 0;
      }
      if (!ctx->srv_ev.empty()) ctx->srv_ev.back().passes++;
      const double t_pub = ctx->h_ptimes ? now_ms() : 0.0;
      if (ctx->h_ptimes && ctx->ht_last_rows > 0 && t_pub - ctx->ht_last_rows < 1.0) {
        ctx->ht_host += t_pub - ctx->ht_last_rows;
        ctx->ht_bfgs += t_entry - ctx->ht_last_rows;
        ++ctx->ht_nh;
      }
      publish_cmd(ctx, seq, kPassRun, 0, &Ax, rstamp);
      ctx->srv_next = seq + 1;
      ctx->st[kStSrvPass]++;
      if (xg) {
        if ((rc = wait_xtot(ctx, rstamp, sums))) return rc;
      } else if (rows) {
        if ((rc = wait_rows(ctx, rstamp, Ax, sums, true))) return rc;
        if (ctx->h_ptimes) {
          ctx->ht_last_rows = now_ms();
          ctx->ht_dev += ctx->ht_last_rows - t_pub;
          ++ctx->ht_n;
        }
      } else {
        if ((rc = wait_pass(ctx, seq))) return rc;
        std::memcpy(sums, ctx->h_red, kRedVals * sizeof(double));
      }
      ctx->n_evals++;
      return MGICP_OK;
    }
    ctx->st[kStLaunchedPass]++;
    if (shm_rows) {
      // a launched pass into the shared rows (profiling, a degraded align, an unservable shard)
      cancel_gated(ctx);
      {
        ProfScope ps(ctx, kFamFdf);
        HIPCK(launch_fdf_soa(c, ctx->ccnt.p, ns, Ax, ctx->partial.p, ctx->spart.p, nb,
                             ctx->tickets.p, nullptr, reverse, nullptr, seq, ctx->stream,
                             row_view(ctx).dev_rows(rstamp), rstamp));
      }
      if ((rc = wait_rows(ctx, rstamp, Ax, sums, false))) return rc;
      ctx->n_evals++;
      return MGICP_OK;
    }
    if (ctx->gated_seq == seq) {
      // pass `seq` is already resident, waiting: hand it its state
      publish_cmd(ctx, seq, kPassRun, reverse, &Ax);
      if (ctx->h_gtrace) ctx->host_gt[2 * (seq & 1023) + 1] = now_ms() * 1e3;
      ctx->gated_seq = 0;
    } else {
      cancel_gated(ctx);
      ProfScope ps(ctx, kFamFdf);
      HIPCK(launch_fdf_soa(c, ctx->ccnt.p, ns, Ax, ctx->partial.p, ctx->spart.p, nb,
                           ctx->tickets.p, out, reverse, (poll && inlaunch) ? ctx->d_flag : nullptr, seq,
                           ctx->stream));
    }
    if (gate) {
      // queue pass seq + 1 now (its launch overlaps this pass); it runs once the BFGS step has
      // published x_{k+1}, or exits on cancel when the BFGS run ends
      HIPCK(launch_fdf_soa_gated(c, ctx->ccnt.p, ns, ctx->partial.p, ctx->spart.p, nb,
                                 ctx->tickets.p, out, ctx->d_flag, seq + 1, ctx->d_cmd, ctx->mail,
                                 ctx->gate_timeout, ctx->d_gtrace, ctx->gate_pollers, ctx->stream));
      ctx->gated_seq = seq + 1;
    }
    if (!inlaunch) {
      {
        ProfScope ps(ctx, kFamRed);
        if ((rc = combine_supers(ctx, kRedVals, ctx->spart.p, ctx->red.p))) return rc;
      }
      if (poll) {
        HIPCK(launch_publish(ctx->red.p, kRedVals, ctx->d_h_red, ctx->d_flag, seq, ctx->stream));
      } else {
        HIPCK(hipMemcpyAsync(ctx->h_red, ctx->red.p, kRedVals * sizeof(double), hipMemcpyDeviceToHost,
                             ctx->stream));
      }
    }
    rc = poll ? wait_pass(ctx, seq) : sync(ctx);
    if (ctx->h_gtrace) ctx->host_gt[2 * ((seq + 1) & 1023)] = now_ms() * 1e3;  // sums of seq seen
    if (rc) return rc;
    std::memcpy(sums, ctx->h_red, kRedVals * sizeof(double));
    ctx->n_evals++;
    return MGICP_OK;
  }

  int eval(const Vec6& x, double& f, Vec6& g) {
    if (have_memo && std::memcmp(x.v, memo_x.v, sizeof(x.v)) == 0) {
      f = memo_f;
      g = memo_g;
      return 0;
    }
    double s[kRedVals];
    int rc = pass(x, s);
    if (rc) return rc;
    m = s[13];
    f = s[0] / m;
    const double sc = 2.0 / m;
    g[0] = s[1] * sc;
    g[1] = s[2] * sc;
    g[2] = s[3] * sc;
    double R[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) R[a][b] = s[4 + 3 * a + b] * sc;
    r_derivative(x, R, g);
    have_memo = true;
    memo_x = x;
    memo_f = f;
    memo_g = g;
    if (ctx->h_ptimes && ctx->ht_last_rows > 0) {
      ctx->ht_eval += now_ms() - ctx->ht_last_rows;
      ++ctx->ht_ne;
    }
    return 0;
  }
};

// GICP::estimateRigidTransformationBFGS: 0 = accepted, MGICP_E_SOLVER = PCL would throw
struct GateGuard {  // a BFGS run leaves no gated pass queued behind it
  mgicp_ctx* ctx;
  ~GateGuard() { cancel_gated(ctx); }
};

// every error return of an align (a HIP error mid-loop, MGICP_E_COMM from a quitting rank, ...) drains
// the stream and gives the device's server slot back, so other contexts on the device keep their
// resident server; the error message of the failure is kept
struct AlignDrain {
  mgicp_ctx* ctx;
  bool armed = true;
  ~AlignDrain() {
    if (!armed) return;
    const std::string err = ctx->err;
    cancel_gated(ctx);
    (void)hipStreamSynchronize(ctx->stream);
    srv_release(ctx);
    if (!ctx->srv_ev.empty()) srv_resolve(ctx);
    ctx->err = err;
  }
};

int estimate_bfgs(mgicp_ctx* ctx, Mat4& T, int* n_corr) {
  GateGuard guard{ctx};
  Vec6 x;
  x[0] = T.m[0][3];
  x[1] = T.m[1][3];
  x[2] = T.m[2][3];
  x[3] = std::atan2(static_cast<double>(T.m[2][1]), static_cast<double>(T.m[2][2]));
  x[4] = std::asin(-static_cast<double>(T.m[2][0]));
  x[5] = std::atan2(static_cast<double>(T.m[1][0]), static_cast<double>(T.m[0][0]));
  DeviceFunctor fn{ctx};
  // the correspondence count arrives with the first objective pass (its count lane)
  double s[kRedVals];
  int rc = fn.pass(x, s);
  if (rc) return rc;
  *n_corr = static_cast<int>(s[13]);
  if (s[13] < 4) return MGICP_E_SOLVER;  // NotEnoughPointsException
  {
    // seed the memo with this pass so minimizeInit reuses it
    fn.m = s[13];
    fn.memo_x = x;
    fn.memo_f = s[0] / fn.m;
    const double sc = 2.0 / fn.m;
    fn.memo_g[0] = s[1] * sc;
    fn.memo_g[1] = s[2] * sc;
    fn.memo_g[2] = s[3] * sc;
    double R[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) R[a][b] = s[4 + 3 * a + b] * sc;
    r_derivative(x, R, fn.memo_g);
    fn.have_memo = true;
  }
  PclBfgs<DeviceFunctor> bfgs(fn);
  const double gradient_tol = 1e-2;
  int inner = 0;
  int result = bfgs.init(x);
  result = kRunning;
  do {
    inner++;
    result = bfgs.step(x);
    if (bfgs.error) return bfgs.error;
    if (result) break;
    result = bfgs.test_gradient(gradient_tol);
  } while (result == kRunning && inner < ctx->prm.max_inner_iter);
  if (bfgs.error) return bfgs.error;
  if (result == kNoProgress || result == kSuccess || inner == ctx->prm.max_inner_iter) {
    T = apply_state(x);
    return MGICP_OK;
  }
  return MGICP_E_SOLVER;  // SolverDidntConvergeException
}

// Gauss-Newton mode, one device pass per outer iteration: the 74 moments of the objective over
// the accepted correspondences of the last sweep at T (Mahalanobis computed on the fly), finished
// over the fixed reduction tree (chunks, supers, all-gathered supers, fixed-order total), copied to
// the host.
int moments_pass(mgicp_ctx* ctx, const Mat4& T, const Mat4& G, bool supers_only = false) {
  const size_t p0 = ctx->shard_p0(), p1 = ctx->shard_p1();
  hipStream_t s = ctx->stream;
  const int nch = chunk_count(p1 - p0);
  HIPCK(ctx->mpartial.reserve(std::max(nch, 1) * static_cast<size_t>(kMomVals)));
  HIPCK(ctx->msuper.reserve(std::max<long long>(ctx->max_supers(), 1) * static_cast<size_t>(kMomVals)));
  HIPCK(ctx->mred.reserve(kMomVals));
  {
    ProfScope ps(ctx, kFamMoments);
    if (nch > 0) {
      HIPCK(launch_gn_moments(ctx->d_out, ctx->tgt.view.pts, ctx->src.cov3(), ctx->tgt.cov3(),
                              rot_of(T, G), T.xf(), ctx->out_ctr, ctx->prev_pos.p, ctx->flags.p, p0,
                              p1, ctx->mpartial.p, chunk_grid_blocks(p1 - p0), s));
      HIPCK(launch_super_reduce(ctx->mpartial.p, nch, kMomVals, ctx->msuper.p, s));
    }
  }
  if (supers_only) return sync(ctx);
  int rc = combine_to_host(ctx, kMomVals, ctx->msuper.p, ctx->mom);
  if (rc) return rc;
  ctx->n_evals++;
  return MGICP_OK;
}

// the correspondence sweep of the Gauss-Newton mode: exact 1-NN (same kernel as the BFGS mode),
// then the moment pass; no scan / compaction (the moment pass reads the flags directly)
int correspond_gn(mgicp_ctx* ctx, const Mat4& T, const Mat4& G, bool seed) {
  const double thr = ctx->prm.max_corr_dist * ctx->prm.max_corr_dist;
  const bool seeded = seed && ctx->seed_valid;
  const uint32_t* qp = query_perm(ctx);
  if (ctx->vlist) {
    int rc = vl_prepare(ctx);
    if (rc) return rc;
  }
  {
    ProfScope ps(ctx, kFamCorr);
    HIPCK(launch_sweep(ctx, T, thr, seeded, qp));
  }
  ctx->seed_valid = true;
  ctx->have_corr = false;  // the SoA streams of the BFGS mode are not refreshed
  int rc = cov_join_all(ctx);
  if (rc) return rc;
  if ((rc = cov_lazy(ctx))) return rc;
  return moments_pass(ctx, T, G);
}

// Gauss-Newton estimate on the moments of the last sweep (taken at T); T <- solution.
// 0 = accepted, MGICP_E_SOLVER = fewer than 4 correspondences or a singular normal matrix.
int estimate_gn(mgicp_ctx* ctx, Mat4& T, int* n_corr) {
  *n_corr = static_cast<int>(ctx->mom[73]);
  if (ctx->mom[73] < 4) return MGICP_E_SOLVER;
  gn::Problem pb;
  pb.mom = ctx->mom;
  gn::Pose P;
  for (int a = 0; a < 3; ++a) {
    pb.c[a] = ctx->out_ctr[a];
    for (int k = 0; k < 4; ++k) pb.T0[a][k] = static_cast<double>(T.m[a][k]);
    for (int k = 0; k < 3; ++k) P.R[a][k] = pb.T0[a][k];
    P.t[a] = pb.T0[a][3];
  }
  int host_evals = 0;
  if (!gn::solve(pb, P, ctx->prm.max_inner_iter, &host_evals)) return MGICP_E_SOLVER;
  for (int a = 0; a < 3; ++a) {
    for (int k = 0; k < 3; ++k) T.m[a][k] = static_cast<float>(P.R[a][k]);
    T.m[a][3] = static_cast<float>(P.t[a]);
  }
  return MGICP_OK;
}

int check_params(mgicp_ctx* ctx, const mgicp_params& p) {
  if (p.k < 1 || p.k > kMaxK)
    return fail(ctx, MGICP_E_INVALID, "k (k_correspondences) must be in [1, 32]");
  if (p.max_iter < 1 || p.max_inner_iter < 1 || !(p.max_corr_dist >= 0) || !(p.rot_eps > 0) ||
      !(p.tf_eps >= 0) ||
      (p.solver != MGICP_SOLVER_PCL_BFGS && p.solver != MGICP_SOLVER_GN))
    return fail(ctx, MGICP_E_INVALID, "invalid GICP parameters");
  return MGICP_OK;
}

}  // namespace

// =====================================================================================
// C-ABI
// =====================================================================================
extern "C" {

void mgicp_default_params(mgicp_params* p) {
  if (!p) return;
  p->max_iter = 100;        // GICPAlignment.cpp:30
  p->tf_eps = 4e-3;         // GICPAlignment.cpp:29
  p->rot_eps = 2e-3;        // PCL GICP rotation_epsilon_
  p->max_corr_dist = 4e-2;  // GICPAlignment.cpp:31
  p->gicp_eps = 1e-3;       // PCL GICP gicp_epsilon_
  p->k = 20;                // PCL GICP k_correspondences_
  p->max_inner_iter = 20;   // PCL GICP max_inner_iterations_
  p->solver = MGICP_SOLVER_PCL_BFGS;
  p->device = -1;
  p->fixed_iterations = 0;
}

int mgicp_device_count(int* n) {
  if (!n) return MGICP_E_INVALID;
  return hipGetDeviceCount(n) == hipSuccess ? MGICP_OK : MGICP_E_HIP;
}

int mgicp_create(mgicp_ctx** out, const mgicp_params* p) {
  if (!out) return MGICP_E_INVALID;
  *out = nullptr;
  std::unique_ptr<Graveyard> grave(new Graveyard());
  t_new_ctx_grave = grave.get();
  mgicp_ctx* ctx = new mgicp_ctx();
  t_new_ctx_grave = nullptr;
  ctx->grave = std::move(grave);
  // runtime environment (INTEGRATION.md "Environment"): deadlines of the pass transport and the fault
  // injection of the multi-rank tests only -- every alternative code path is a compile-time option
  // (Makefile `variant`) or a test's explicit mgicp_debug_option call, never an environment variable
  if (const char* sp = std::getenv("MGICP_SRV_STALL_PASS")) ctx->stall_pass = std::atoi(sp);
  if (const char* qp = std::getenv("MGICP_DEBUG_QUIT_PASS")) ctx->quit_pass = std::atoi(qp);
  if (const char* dl = std::getenv("MGICP_ROW_DEADLINE_MS")) {
    const double v = std::atof(dl);
    if (v > 0) ctx->row_deadline_ms = v;
  }
  if (const char* rd = std::getenv("MGICP_REMOTE_DEADLINE_S")) {
    const double v = std::atof(rd);
    if (v > 0) ctx->remote_deadline_s = v;
  }
  {
    const unsigned hc = std::thread::hardware_concurrency();
    ctx->host_threads = static_cast<int>(std::max(1u, std::min(8u, hc ? hc : 1u)));
  }
  if (p) ctx->prm = *p;
  else mgicp_default_params(&ctx->prm);
  int rc = check_params(ctx, ctx->prm);
  if (rc) {
    delete ctx;
    return rc;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    delete ctx;
    return MGICP_E_HIP;
  }
  if (ctx->prm.device >= 0) {
    if (ctx->prm.device >= ndev || hipSetDevice(ctx->prm.device) != hipSuccess) {
      delete ctx;
      return MGICP_E_INVALID;
    }
    ctx->device = ctx->prm.device;
  } else if (hipGetDevice(&ctx->device) != hipSuccess) {
    delete ctx;
    return MGICP_E_HIP;
  }
  if (hipDeviceGetAttribute(&ctx->cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess)
    ctx->cus = 0;  // no resident server
  ctx->tgt.want_empty_map = true;  // correspondence / fitness queries start off the surface
  ctx->tgt.want_seed_map = true;  // first 1-NN sweep seeded from a nearest non-empty cell
  // per-cell point boxes in the 1-NN sweeps: exact and 1.75x fewer candidates in sweep 1, but the
  // per-cell box loads and tests cost more than they save (C4 correspondence 1.39 vs 1.11 ms,
  // profiles/r02/ab_boxes): off
  ctx->tgt.want_boxes = false;
  ctx->tgt.want_pairs = ctx->corr_wave;  // the wave-uniform 1-NN scan (r03) reads the target's pair copy
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return MGICP_E_HIP;
  }
  MGICP_TRACE_AT("create: stream");
  bool ok = hipHostMalloc(reinterpret_cast<void**>(&ctx->h_small), kSmallBytes,
                          hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_small), ctx->h_small, 0) == hipSuccess;
  MGICP_TRACE_AT("create: pinned words");
  ok = ok && preload_kernels(ctx->h_small, kSmallBytes, ctx->stream) == hipSuccess;
  MGICP_TRACE_AT("create: kernels loaded");
  ok = ok && HostUploader::instance().init(ctx->host_threads) == hipSuccess;
  MGICP_TRACE_AT("create: upload staging");
  if (!ok) {
    if (ctx->h_small) (void)hipHostFree(ctx->h_small);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return MGICP_E_HIP;
  }
  // the pass path's pinned command / result words and the BAR command block (its memset is
  // synchronous): here, not in the first align, where they waited for the covariance head start
  (void)ensure_host_red(ctx);  // (retried by the first align if it failed)
  MGICP_TRACE_AT("create: pass words + BAR block");
  // the stream of the covariance head start (created here: a stream's creation costs milliseconds
  // of host time, which set_* would otherwise pay before the launch).  A CU mask on it (leaving CUs to
  // the main stream) was measured -0.5 to -1.4 ms on new clouds (profiles/r04/ncab1) but a CU mask
  // belongs to the hardware queue, which past GPU_MAX_HW_QUEUES streams share: not used.
  hipError_t se = hipSuccess;
  if (ctx->async_tgt) se = hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking);
  if (ctx->async_tgt && (se != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->aux_ev[0], hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->aux_ev[1], hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->aux_ev[2], hipEventDisableTiming) != hipSuccess ||
                         hipEventCreateWithFlags(&ctx->aux_ev[3], hipEventDisableTiming) != hipSuccess)) {
    if (ctx->aux_stream) (void)hipStreamDestroy(ctx->aux_stream);
    for (hipEvent_t& ev : ctx->aux_ev)
      if (ev) (void)hipEventDestroy(ev), ev = nullptr;
    ctx->aux_stream = nullptr;
  }
  MGICP_TRACE_AT("create: aux stream");
  *out = ctx;
  return MGICP_OK;
}

int mgicp_set_params(mgicp_ctx* ctx, const mgicp_params* p) {
  if (!ctx || !p) return MGICP_E_INVALID;
  int rc = check_params(ctx, *p);
  if (rc) return rc;
  if ((rc = cov_join_all(ctx))) return rc;  // a pending covariance launch uses the old k / eps
  const bool cov_change = p->k != ctx->prm.k || p->gicp_eps != ctx->prm.gicp_eps;
  const int dev = ctx->device;
  ctx->prm = *p;
  ctx->prm.device = dev;
  if (cov_change) {
    ctx->src.have_cov = false;
    ctx->tgt.have_cov = false;
    ctx->src_lazy_ready = false;
  }
  return MGICP_OK;
}

const char* mgicp_last_error(const mgicp_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

void mgicp_destroy(mgicp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  cancel_gated(ctx);
  if (ctx->aux_stream) (void)hipStreamSynchronize(ctx->aux_stream);
  // a head-start launch chain that ran to its end on the aux stream completed the target's covariances
  const bool tgt_cov_done = ctx->tgt.have_cov || (ctx->tgt_cov_pending && !ctx->tgt.dirty);
  ctx->tgt_cov_pending = ctx->src_cov_pending = false;
  (void)hipStreamSynchronize(ctx->stream);
  srv_release(ctx);
  tcache_donate(ctx, tgt_cov_done);  // r05: the target's grid, covariances and lists outlive the context
  ctx->f_flags.release(); ctx->f_pos.release(); ctx->f_rgba_in.release(); ctx->f_rgba.release();
  ctx->f_rgba2.release(); ctx->f_vox.release(); ctx->f_vox2.release(); ctx->f_keep.release();
  ctx->f_count.release();
  for (Cloud* c : {&ctx->src, &ctx->tgt, &ctx->aux, &ctx->qry}) {
    c->raw.release(); c->orig.release(); c->pts.release(); c->perm.release();
    c->cell_start.release(); c->cov.release(); c->empty_dist.release(); c->boxes.release(); c->pairs.release();
    c->seed.release(); c->seed_scratch.release();
  }
  ctx->src_out.release();
  ctx->qperm.release();
  ctx->aq_keys.release(); ctx->aq_keys_sorted.release(); ctx->aq_vals.release(); ctx->aq_scratch.release();
  ctx->partial.release(); ctx->red.release(); ctx->mpartial.release(); ctx->mred.release(); ctx->counts.release(); ctx->keys.release();
  ctx->keys_sorted.release(); ctx->vals.release(); ctx->scratch.release(); ctx->u64.release();
  ctx->fpartial.release();
  ctx->knn_fb.release();
  ctx->tickets.release();
  ctx->tickets_n = 0;
  ctx->ccnt.release(); ctx->spart.release(); ctx->gath.release(); ctx->msuper.release();
  ctx->prev_pos.release(); ctx->flags.release();
  ctx->nn_work.release(); ctx->nn_work_n.release();
  ctx->vl_cell.release(); ctx->vl_pool.release(); ctx->vl_ctr.release();
  ctx->vl_build.release(); ctx->vl_bcentre.release(); ctx->vl_pend.release(); ctx->vl_defer.release();
  ctx->cov_ok.release(); ctx->cov_need.release();
  ctx->aux_cnt.release(); ctx->knn_fb2.release();
  ctx->tpart.release();
  ctx->tpart_n = 0;
  ctx->corr_f.release(); ctx->corr_d.release();
  ctx->xyz_dev.release();
  if (ctx->mail) (void)hipFree(ctx->mail);
  if (ctx->h_red) (void)hipHostFree(ctx->h_red);
  if (ctx->h_cmd) (void)hipHostFree(ctx->h_cmd);
  if (ctx->h_gtrace) (void)hipHostFree(ctx->h_gtrace);
  if (ctx->h_ptimes) (void)hipHostFree(ctx->h_ptimes);
  if (ctx->h_rows) (void)hipHostFree(ctx->h_rows);
  xgmi_detach(ctx);
  if (ctx->xstream && ctx->xstream_own) (void)hipStreamDestroy(ctx->xstream);
  if (ctx->h_xtot) (void)hipHostFree(ctx->h_xtot);
  if (ctx->have_shm) {
    (void)hipHostUnregister(ctx->shm.base);
    shm::detach(ctx->shm);
    ctx->have_shm = false;
  }
  if (ctx->bar_cmd) (void)hipFree(ctx->bar_cmd);
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  prof_resolve(ctx);
  srv_resolve(ctx);
  for (hipEvent_t e : ctx->pool) (void)hipEventDestroy(e);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->aux_stream) (void)hipStreamDestroy(ctx->aux_stream);
  ctx->grave->flush();
  for (hipEvent_t e : ctx->aux_ev)
    if (e) (void)hipEventDestroy(e);
  delete ctx;
}

int mgicp_set_target(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = upload_cloud(ctx, ctx->tgt, xyz, n, stride, false);
  if (!rc) rc = tcache_adopt(ctx);
  return rc ? rc : cov_prep_async_all(ctx);
}
int mgicp_set_source(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const int rc = upload_cloud(ctx, ctx->src, xyz, n, stride, false);
  return rc ? rc : cov_prep_async_all(ctx);
}
int mgicp_set_target_device(mgicp_ctx* ctx, const float* d_xyz, size_t n, size_t stride) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = upload_cloud(ctx, ctx->tgt, d_xyz, n, stride, true);
  if (!rc) rc = tcache_adopt(ctx);
  return rc ? rc : cov_prep_async_all(ctx);
}
int mgicp_set_source_device(mgicp_ctx* ctx, const float* d_xyz, size_t n, size_t stride) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const int rc = upload_cloud(ctx, ctx->src, d_xyz, n, stride, true);
  return rc ? rc : cov_prep_async_all(ctx);
}

int mgicp_align(mgicp_ctx* ctx, const float guess_cm[16], float out_T_cm[16], mgicp_result* res) {
  if (!ctx || !out_T_cm) return MGICP_E_INVALID;
  if (ctx->nranks > 1 && !ctx->comm && !ctx->have_shm)
    return fail(ctx, MGICP_E_INVALID, "detached shard context: only the debug entry points are available");
  HIPCK(hipSetDevice(ctx->device));
  mgicp_result r;
  std::memset(&r, 0, sizeof(r));
  const double t0 = now_ms();
  MGICP_TRACE_AT("align: begin");
  AlignDrain drain{ctx};
  int rc = prepare(ctx, true);
  if (rc) return rc;
  MGICP_TRACE_AT("align: prepared");
  rc = ensure_iter_buffers(ctx);
  if (rc) return rc;
  MGICP_TRACE_AT("align: iteration buffers ready");
  const double t1 = now_ms();
  const Mat4 G = guess_cm ? Mat4::from_cm(guess_cm) : Mat4::identity();
  if ((rc = set_output(ctx, G))) return rc;

  Mat4 T = Mat4::identity(), prev = Mat4::identity();
  ctx->trace.clear();
  ctx->n_evals = 0;
  ctx->srv_degraded = false;  // a take-over degrades the rest of one align only
  int nr_iterations = 0;
  bool converged = false;
  int solver_rc = MGICP_OK;
  while (!converged) {
    const bool gn_mode = ctx->prm.solver == MGICP_SOLVER_GN;
    rc = gn_mode ? correspond_gn(ctx, T, G, nr_iterations > 0)
                 : correspond(ctx, T, G, nr_iterations > 0);
    if (rc) return rc;
    prev = T;
    int ncorr = 0;
    MGICP_TRACE_AT("align: sweep done");
    rc = gn_mode ? estimate_gn(ctx, T, &ncorr) : estimate_bfgs(ctx, T, &ncorr);
    MGICP_TRACE_AT("align: solve done");
    r.n_corr = ncorr;
    if (rc == MGICP_E_SOLVER) {  // PCLException caught: converged_ stays false
      T = prev;
      solver_rc = rc;
      break;
    }
    if (rc) return rc;
    double delta = 0.;
    for (int k = 0; k < 4; ++k)
      for (int l = 0; l < 4; ++l) {
        const double ratio = (k < 3 && l < 3) ? 1. / ctx->prm.rot_eps : 1. / ctx->prm.tf_eps;
        const double c_delta = ratio * static_cast<double>(std::fabs(prev.m[k][l] - T.m[k][l]));
        if (c_delta > delta) delta = c_delta;
      }
    float tcm[16];
    T.to_cm(tcm);
    ctx->trace.insert(ctx->trace.end(), tcm, tcm + 16);
    nr_iterations++;
    const bool stop = ctx->prm.fixed_iterations
                          ? nr_iterations >= ctx->prm.max_iter
                          : (nr_iterations >= ctx->prm.max_iter || delta < 1);
    if (stop) {
      converged = true;
      prev = T;
    }
  }
  // polled passes leave their kernels' completion unobserved: drain the stream once
  if ((rc = sync(ctx))) return rc;
  drain.armed = false;
  if (!ctx->tgt_cov_pending && !ctx->src_cov_pending) ctx->grave->flush();  // a quiet point
  if (ctx->vl_valid) ctx->vl_groups++;
  if (ctx->h_gtrace) {
    // diagnostics of the gated passes of this align: device-side gate wait and spread, host-side
    // decision time (sums seen -> command published); device wall clock in 10 ns ticks (100 MHz)
    double w = 0, sp = 0, hd = 0;
    int cnt = 0;
    for (int i = 0; i < 1024; ++i) {
      const unsigned long long* t = ctx->h_gtrace + 4 * i;
      if (!t[0] || !t[1] || !t[2] || ctx->host_gt[2 * i + 1] <= 0 || ctx->host_gt[2 * i] <= 0) continue;
      w += (t[1] - t[0]) * 0.01;
      sp += (static_cast<double>(t[2]) - static_cast<double>(t[1])) * 0.01;
      hd += ctx->host_gt[2 * i + 1] - ctx->host_gt[2 * i];
      ++cnt;
    }
    if (cnt)
      std::fprintf(stderr, "[gate-trace] passes %d | device: block-0 wait %.2f us, last block through the gate +%.2f us | host: sums seen -> command published %.2f us\n",
                   cnt, w / cnt, sp / cnt, hd / cnt);
    std::memset(ctx->h_gtrace, 0, 4 * 1024 * sizeof(unsigned long long));
    std::fill(ctx->host_gt.begin(), ctx->host_gt.end(), 0.0);
  }
  if (ctx->h_ptimes) {
    // diagnostics of the resident server: per pass, block 0's gate exit -> the finishing wave
    // (device active time) and the previous finish -> this gate exit (host turnaround + gate)
    double act = 0, gap = 0;
    int na = 0, ng = 0;
    for (int i = 0; i < 1024; ++i) {
      const unsigned long long* t = ctx->h_ptimes + 2 * i;
      if (t[0] && t[1] && t[1] > t[0]) { act += (t[1] - t[0]) * 0.01; ++na; }
      const unsigned long long* pv = ctx->h_ptimes + 2 * ((i + 1023) & 1023);
      if (t[0] && pv[1] && t[0] > pv[1] && t[0] - pv[1] < 100000) { gap += (t[0] - pv[1]) * 0.01; ++ng; }
    }
    if (na)
      std::fprintf(stderr, "[pass-times] passes %d | active %.2f us | finish -> next gate exit %.2f us (%d)\n", na,
                   act / na, ng ? gap / ng : 0.0, ng);
    if (ctx->ht_n)
      std::fprintf(stderr, "[pass-times] host view: %d passes | command -> rows complete %.2f us | rows -> next command %.2f us (BFGS step until the next pass %.2f us)\n",
                   ctx->ht_n, 1e3 * ctx->ht_dev / ctx->ht_n, ctx->ht_nh ? 1e3 * ctx->ht_host / ctx->ht_nh : 0.0,
                   ctx->ht_nh ? 1e3 * ctx->ht_bfgs / ctx->ht_nh : 0.0);
    if (ctx->ht_ne)
      std::fprintf(stderr, "[pass-times] host view: rows complete -> f, g of the pass ready %.2f us (%d)\n",
                   1e3 * ctx->ht_eval / ctx->ht_ne, ctx->ht_ne);
    ctx->ht_dev = ctx->ht_host = ctx->ht_bfgs = ctx->ht_eval = ctx->ht_last_rows = 0;
    ctx->ht_n = ctx->ht_nh = ctx->ht_ne = 0;
    std::memset(ctx->h_ptimes, 0, 2 * 1024 * sizeof(unsigned long long));
  }
  // final_transformation_ = previous_transformation_ (3x3) * guess (3x3); t = prev t + guess t
  Mat4 F = Mat4::identity();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      float a = prev.m[i][0] * G.m[0][j];
      a = a + prev.m[i][1] * G.m[1][j];
      a = a + prev.m[i][2] * G.m[2][j];
      F.m[i][j] = a;
    }
  for (int i = 0; i < 3; ++i) F.m[i][3] = prev.m[i][3] + G.m[i][3];
  F.to_cm(out_T_cm);
  const double t2 = now_ms();
  r.converged = converged ? 1 : 0;
  r.iterations = nr_iterations;
  r.n_evals = ctx->n_evals;
  r.ms_upload = ctx->ms_upload_pending;
  ctx->ms_upload_pending = 0;
  r.ms_prep = t1 - t0;
  r.ms_loop = t2 - t1;
  r.ms_total = t2 - t0 + r.ms_upload;
  if (res) *res = r;
  if (solver_rc) return fail(ctx, solver_rc, "GICP solver threw (fewer than 4 correspondences or BFGS failure)");
  return MGICP_OK;
}

// getFitnessScore's chunk and super partials of this shard ([0] sum d2, [13] count) in spart
static int fitness_supers(mgicp_ctx* ctx, const Mat4& T, double max_range) {
  const size_t p0 = ctx->shard_p0(), p1 = ctx->shard_p1();
  const int nch = chunk_count(p1 - p0);
  if (nch == 0) return MGICP_OK;
  HIPCK(launch_fitness(ctx->tgt.view, ctx->src.pts.p, p0, p1, T.xf(), max_range, ctx->partial.p,
                       chunk_grid_blocks(p1 - p0), ctx->stream));
  HIPCK(launch_super_reduce(ctx->partial.p, nch, kRedVals, ctx->spart.p, ctx->stream));
  return MGICP_OK;
}

int mgicp_fitness(mgicp_ctx* ctx, const float T_cm[16], double max_range, double* out) {
  if (!ctx || !T_cm || !out) return MGICP_E_INVALID;
  if (ctx->nranks > 1 && !ctx->comm && !ctx->have_shm)
    return fail(ctx, MGICP_E_INVALID, "detached shard context: only the debug entry points are available");
  HIPCK(hipSetDevice(ctx->device));
  int rc = prepare(ctx, false);
  if (rc) return rc;
  if ((rc = ensure_iter_buffers(ctx))) return rc;
  if (!(max_range > 0)) max_range = 1.7976931348623157e308;
  const Mat4 T = Mat4::from_cm(T_cm);
  if ((rc = fitness_supers(ctx, T, max_range))) return rc;
  double tot[kRedVals];
  if ((rc = combine_to_host(ctx, kRedVals, ctx->spart.p, tot))) return rc;
  const double nr = tot[13];
  *out = nr > 0 ? tot[0] / nr : 1.7976931348623157e308;
  return MGICP_OK;
}

int mgicp_transform_source(mgicp_ctx* ctx, const float T_cm[16], float* out, size_t out_stride) {
  if (!ctx || !T_cm || !out || out_stride < 12 || ctx->src.n == 0) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const size_t n = ctx->src.n;
  DevBuf<float4> tmp;
  HIPCK(tmp.reserve(n));
  HIPCK(launch_xform_points(ctx->src.orig.p, n, Mat4::from_cm(T_cm).xf(), tmp.p, ctx->stream));
  std::vector<float4> h(n);
  HIPCK(hipMemcpyAsync(h.data(), tmp.p, n * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
  int rc = sync(ctx);
  tmp.release();
  if (rc) return rc;
  unsigned char* base = reinterpret_cast<unsigned char*>(out);
  for (size_t i = 0; i < n; ++i) {
    float* o = reinterpret_cast<float*>(base + i * out_stride);
    o[0] = h[i].x;
    o[1] = h[i].y;
    o[2] = h[i].z;
  }
  return MGICP_OK;
}

int mgicp_transform_cloud(mgicp_ctx* ctx, const float T_cm[16], const float* in, size_t n,
                          size_t in_stride, float* out, size_t out_stride) {
  if (!ctx || !T_cm || (n && (!in || !out)) || in_stride < 12 || out_stride < 12 ||
      (in_stride % 4) || (out_stride % 4))
    return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  if (n == 0) return MGICP_OK;
  DevBuf<unsigned char> raw;
  DevBuf<float4> a, b;
  HIPCK(raw.reserve(n * in_stride));
  HIPCK(a.reserve(n));
  HIPCK(b.reserve(n));
  HIPCK(hipMemcpyAsync(raw.p, in, n * in_stride, hipMemcpyHostToDevice, ctx->stream));
  HIPCK(launch_pack_points(raw.p, n, in_stride, a.p, ctx->stream));
  HIPCK(launch_xform_points(a.p, n, Mat4::from_cm(T_cm).xf(), b.p, ctx->stream));
  std::vector<float4> h(n);
  HIPCK(hipMemcpyAsync(h.data(), b.p, n * sizeof(float4), hipMemcpyDeviceToHost, ctx->stream));
  int rc = sync(ctx);
  raw.release();
  a.release();
  b.release();
  if (rc) return rc;
  unsigned char* base = reinterpret_cast<unsigned char*>(out);
  for (size_t i = 0; i < n; ++i) {
    float* o = reinterpret_cast<float*>(base + i * out_stride);
    o[0] = h[i].x;
    o[1] = h[i].y;
    o[2] = h[i].z;
  }
  return MGICP_OK;
}

int mgicp_cloud_resolution(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride, double* out) {
  if (!ctx || !out) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  *out = 0.0;
  if (n < 2) return MGICP_OK;  // no point has a 2nd neighbour: res stays 0
  int rc = upload_cloud(ctx, ctx->aux, xyz, n, stride, false);
  if (rc) return rc;
  // Utils::computeCloudResolution skips non-finite points and its KdTree holds only finite ones
  // (src/Utils.cpp:152-160): grid and queries over the finite points
  ctx->aux.drop_nonfinite = true;
  rc = build_grid(ctx, ctx->aux);
  ctx->aux.drop_nonfinite = false;
  if (rc) return rc;
  const size_t nf = ctx->aux.n;
  if (nf < 2) return MGICP_OK;  // nearestKSearch never returns 2: n_points = 0, res = 0
  const int nb = static_cast<int>((nf + 255) / 256);
  HIPCK(ctx->partial.reserve(static_cast<size_t>(nb) * kRedVals));
  HIPCK(ctx->red.reserve(kRedVals));
  if ((rc = ensure_host_red(ctx))) return rc;
  HIPCK(launch_resolution(ctx->aux.view, nf, ctx->partial.p, nb, ctx->stream));
  HIPCK(launch_reduce_finish(ctx->partial.p, nb, ctx->red.p, ctx->stream));
  HIPCK(hipMemcpyAsync(ctx->h_red, ctx->red.p, kRedVals * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  if ((rc = sync(ctx))) return rc;
  const double cnt = ctx->h_red[13];
  *out = cnt > 0 ? ctx->h_red[0] / cnt : 0.0;
  return MGICP_OK;
}

int mgicp_radius_filter(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride, double radius,
                        int min_neighbors, unsigned char* keep) {
  if (!ctx || !keep || min_neighbors < 1 || !(radius >= 0)) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  if (n == 0) return MGICP_OK;
  int rc = upload_cloud(ctx, ctx->aux, xyz, n, stride, false);
  if (rc) return rc;
  // NormalEstimation gives non-finite points NaN normals and searches a tree of the finite points
  // only: grid over the finite points, keep = 0 for every other record
  ctx->aux.drop_nonfinite = true;
  rc = build_grid(ctx, ctx->aux);
  ctx->aux.drop_nonfinite = false;
  if (rc) return rc;
  DevBuf<unsigned char> d_keep;
  HIPCK(d_keep.reserve(n));
  HIPCK(hipMemsetAsync(d_keep.p, 0, n, ctx->stream));
  const float r2 = static_cast<float>(radius * radius);
  // one query per finite point; the kernel scatters keep[] through the original index in w
  HIPCK(launch_radius_keep(ctx->aux.view, ctx->aux.n, r2, min_neighbors, d_keep.p, ctx->stream));
  HIPCK(hipMemcpyAsync(keep, d_keep.p, n, hipMemcpyDeviceToHost, ctx->stream));
  rc = sync(ctx);
  d_keep.release();
  return rc;
}

int mgicp_segment_differences(mgicp_ctx* ctx, const float T_cm[16], const float* in, size_t n,
                              size_t in_stride, const float* sub, size_t n_sub, size_t sub_stride,
                              double sqr_threshold, unsigned char* keep, size_t* n_keep) {
  if (!ctx || !n_keep || (n && (!in || !keep)) || (n_sub && !sub) || !(sqr_threshold == sqr_threshold))
    return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  *n_keep = 0;
  if (n == 0) return MGICP_OK;
  if (n_sub == 0) {  // "input - empty target = input": every record, finite or not
    std::memset(keep, 1, n);
    *n_keep = n;
    return MGICP_OK;
  }
  int rc = upload_cloud(ctx, ctx->aux, sub, n_sub, sub_stride, false);
  if (rc) return rc;
  ctx->aux.drop_nonfinite = true;
  rc = build_grid(ctx, ctx->aux);
  ctx->aux.drop_nonfinite = false;
  if (rc) return rc;
  if (ctx->aux.n == 0) {  // no finite target point: nearestKSearch finds nothing, nothing kept
    std::memset(keep, 0, n);
    return MGICP_OK;
  }
  if ((rc = upload_cloud(ctx, ctx->qry, in, n, in_stride, false))) return rc;
  hipStream_t s = ctx->stream;
  HIPCK(ctx->f_keep.reserve(n));
  HIPCK(ctx->f_count.reserve(1));
  HIPCK(hipMemsetAsync(ctx->f_count.p, 0, sizeof(unsigned int), s));
  const Mat4 T = T_cm ? Mat4::from_cm(T_cm) : Mat4::identity();
  HIPCK(launch_segdiff(ctx->aux.view, ctx->qry.orig.p, n, T.xf(), T_cm ? 1 : 0, sqr_threshold,
                       ctx->f_keep.p, ctx->f_count.p, s));
  HIPCK(hipMemcpyAsync(keep, ctx->f_keep.p, n, hipMemcpyDeviceToHost, s));
  HIPCK(hipMemcpyAsync(ctx->h_small, ctx->f_count.p, sizeof(unsigned int), hipMemcpyDeviceToHost, s));
  if ((rc = sync(ctx))) return rc;
  unsigned int cnt = 0;
  std::memcpy(&cnt, ctx->h_small, sizeof(cnt));
  *n_keep = cnt;
  return MGICP_OK;
}

int mgicp_voxel_grid(mgicp_ctx* ctx, const float* in, size_t n, size_t stride, int rgb_offset,
                     const double leaf[3], int min_points_per_voxel, float* out, size_t out_stride,
                     size_t* n_out) {
  if (!ctx || !n_out || !leaf || (n && (!in || !out)) || out_stride < 12 || (out_stride % 4) ||
      (rgb_offset >= 0 && (static_cast<size_t>(rgb_offset) + 4 > stride ||
                           static_cast<size_t>(rgb_offset) + 4 > out_stride || (rgb_offset % 4))))
    return MGICP_E_INVALID;
  for (int d = 0; d < 3; ++d)
    if (!(leaf[d] > 0)) return fail(ctx, MGICP_E_INVALID, "leaf size must be > 0");
  HIPCK(hipSetDevice(ctx->device));
  *n_out = 0;
  if (n == 0) return MGICP_OK;
  int rc = upload_cloud(ctx, ctx->qry, in, n, stride, false);
  if (rc) return rc;
  hipStream_t s = ctx->stream;
  const bool rgb = rgb_offset >= 0;
  if (rgb) {  // the packed colour word of every record, through the pinned pipelined upload
    HIPCK(ctx->f_rgba_in.reserve(n));
    HostUploader& up = HostUploader::instance();
    HIPCK(up.init(ctx->host_threads));
    {
      std::lock_guard<std::mutex> lk(up.mu);
      HIPCK(upload_u32_field(*up.pool, up.ring, in, n, stride, static_cast<size_t>(rgb_offset),
                             ctx->f_rgba_in.p, s));
      if ((rc = sync(ctx))) return rc;
    }
  }
  // getMinMax3D over the finite points
  const int nb = static_cast<int>(std::min<size_t>((n + 255) / 256, 1024));
  HIPCK(launch_bbox(ctx->qry.orig.p, n, reinterpret_cast<float*>(ctx->d_small), nb, s));
  if ((rc = sync(ctx))) return rc;
  const float* hp = reinterpret_cast<const float*>(ctx->h_small);
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int b = 0; b < nb; ++b)
    for (int d = 0; d < 3; ++d) {
      mn[d] = std::min(mn[d], hp[b * 8 + d]);
      mx[d] = std::max(mx[d], hp[b * 8 + 3 + d]);
    }
  if (!(mn[0] <= mx[0])) return MGICP_OK;  // no finite point
  float inv[3];
  for (int d = 0; d < 3; ++d) inv[d] = 1.0f / static_cast<float>(leaf[d]);
  int64_t dd[3];
  for (int d = 0; d < 3; ++d) dd[d] = static_cast<int64_t>((mx[d] - mn[d]) * inv[d]) + 1;
  auto put = [&](size_t i, float x, float y, float z, const uint32_t* c) {
    unsigned char* r = reinterpret_cast<unsigned char*>(out) + i * out_stride;
    std::memset(r, 0, out_stride);
    float* f = reinterpret_cast<float*>(r);
    f[0] = x; f[1] = y; f[2] = z;
    if (out_stride >= 16) f[3] = 1.0f;
    if (c) std::memcpy(r + rgb_offset, c, 4);
  };
  if (dd[0] * dd[1] * dd[2] > static_cast<int64_t>(INT32_MAX)) {
    // "Leaf size is too small for the input dataset": output = input
    const unsigned char* base = reinterpret_cast<const unsigned char*>(in);
    for (size_t i = 0; i < n; ++i) {
      const float* p = reinterpret_cast<const float*>(base + i * stride);
      uint32_t c = 0;
      if (rgb) std::memcpy(&c, base + i * stride + rgb_offset, 4);
      put(i, p[0], p[1], p[2], rgb ? &c : nullptr);
    }
    *n_out = n;
    return MGICP_OK;
  }
  int min_b[3], div_b[3];
  for (int d = 0; d < 3; ++d) {
    min_b[d] = static_cast<int>(std::floor(mn[d] * inv[d]));
    div_b[d] = static_cast<int>(std::floor(mx[d] * inv[d])) - min_b[d] + 1;
  }
  Cloud& q = ctx->qry;
  HIPCK(ctx->keys.reserve(n));
  HIPCK(ctx->keys_sorted.reserve(n));
  HIPCK(ctx->vals.reserve(n));
  HIPCK(q.perm.reserve(n));
  HIPCK(ctx->f_flags.reserve(n + 1));
  HIPCK(ctx->f_pos.reserve(n + 1));
  const size_t sb = std::max(sort_scratch_bytes(n, 32), scan_scratch_bytes(n + 1));
  HIPCK(ctx->scratch.reserve(sb));
  HIPCK(launch_voxel_keys(q.orig.p, n, inv, min_b, div_b[0], div_b[0] * div_b[1], ctx->keys.p, s));
  HIPCK(launch_iota(ctx->vals.p, n, s));
  HIPCK(launch_sort_pairs(ctx->scratch.p, sb, ctx->keys.p, ctx->keys_sorted.p, ctx->vals.p, q.perm.p, n, 32, s));
  HIPCK(launch_voxel_heads(ctx->keys_sorted.p, n, ctx->f_flags.p, s));
  HIPCK(launch_exclusive_scan(ctx->scratch.p, sb, ctx->f_flags.p, ctx->f_pos.p, n + 1, s));
  HIPCK(hipMemcpyAsync(ctx->h_small, ctx->f_pos.p + n, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  if ((rc = sync(ctx))) return rc;
  uint32_t nv = 0;
  std::memcpy(&nv, ctx->h_small, sizeof(nv));
  HIPCK(ctx->f_vox.reserve(nv + 1));
  if (rgb) HIPCK(ctx->f_rgba.reserve(nv + 1));
  HIPCK(launch_voxel_centroids(ctx->keys_sorted.p, q.perm.p, ctx->f_flags.p, ctx->f_pos.p, n, q.orig.p,
                               rgb ? ctx->f_rgba_in.p : nullptr, ctx->f_vox.p, rgb ? ctx->f_rgba.p : nullptr, s));
  const float4* vox = ctx->f_vox.p;
  const uint32_t* vrgb = rgb ? ctx->f_rgba.p : nullptr;
  if (min_points_per_voxel > 1) {
    HIPCK(ctx->f_vox2.reserve(nv + 1));
    if (rgb) HIPCK(ctx->f_rgba2.reserve(nv + 1));
    const size_t sb2 = scan_scratch_bytes(nv + 1);
    HIPCK(ctx->scratch.reserve(std::max(sb, sb2)));
    HIPCK(launch_voxel_minpts(ctx->f_vox.p, vrgb, nv, static_cast<uint32_t>(min_points_per_voxel), ctx->f_flags.p,
                              ctx->f_pos.p, ctx->scratch.p, sb2, ctx->f_vox2.p, rgb ? ctx->f_rgba2.p : nullptr, s));
    HIPCK(hipMemcpyAsync(ctx->h_small, ctx->f_pos.p + nv, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if ((rc = sync(ctx))) return rc;
    std::memcpy(&nv, ctx->h_small, sizeof(nv));
    vox = ctx->f_vox2.p;
    vrgb = rgb ? ctx->f_rgba2.p : nullptr;
  }
  std::vector<float4> hv(nv);
  std::vector<uint32_t> hc(rgb ? nv : 0);
  if (nv) {
    HIPCK(hipMemcpyAsync(hv.data(), vox, nv * sizeof(float4), hipMemcpyDeviceToHost, s));
    if (rgb) HIPCK(hipMemcpyAsync(hc.data(), vrgb, nv * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  }
  if ((rc = sync(ctx))) return rc;
  for (size_t v = 0; v < nv; ++v) put(v, hv[v].x, hv[v].y, hv[v].z, rgb ? &hc[v] : nullptr);
  *n_out = nv;
  return MGICP_OK;
}

int mgicp_get_unique_id(unsigned char id[128]) {
  if (!id) return MGICP_E_INVALID;
  ncclUniqueId uid;
  if (ncclGetUniqueId(&uid) != ncclSuccess) return MGICP_E_COMM;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
  std::memcpy(id, &uid, 128);
  return MGICP_OK;
}

int mgicp_comm_init(mgicp_ctx* ctx, int nranks, int rank, const unsigned char id[128]) {
  if (!ctx || nranks < 1 || rank < 0 || rank >= nranks) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  if (int rj = cov_join_all(ctx)) return rj;  // the shard changes under them
  if (ctx->comm) {
    (void)ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
  }
  if (ctx->have_shm) {  // the segment's geometry belongs to the old rank layout
    int rc = sync(ctx);
    if (rc) return rc;
    (void)hipHostUnregister(ctx->shm.base);
    shm::detach(ctx->shm);
    ctx->have_shm = false;
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  ctx->qperm_valid = false;
  ctx->src_lazy_ready = false;
  ctx->src.have_cov = false;
  ctx->have_corr = false;
  ctx->seed_valid = false;  // the shard (and its per-point match buffers) changes
  ctx->st[kStTransport] = 0;
  // id == NULL: detached shard (debug entry points only, until mgicp_comm_attach_shm).  nranks == 1
  // with an id builds a real one-rank communicator, so the collective code path can be exercised on
  // a single device.
  if (!id) return MGICP_OK;
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  ncclComm_t comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    // r06: the context stays a detached shard of the same layout (an RCCL-free rank once a segment is
    // attached), so a caller can fall back without re-creating it (parallel.setup_transport)
    return fail(ctx, MGICP_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  ctx->comm = comm;
  ctx->st[kStTransport] = 1;
  return MGICP_OK;
}

int mgicp_comm_attach_xgmi(mgicp_ctx* ctx, int on) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = cov_join_all(ctx);
  if (rc || (rc = sync(ctx))) return rc;
  xgmi_detach(ctx);
  if (!on) return reset_stamps(ctx);
  if (!ctx->have_shm)
    return fail(ctx, MGICP_E_INVALID, "xGMI row exchange: attach the shared segment first (its rendezvous)");
  if (ctx->nranks - 1 > kMaxPeers) return fail(ctx, MGICP_E_INVALID, "xGMI row exchange: at most 9 ranks");
  // host words of the totaler (pinned, mapped) and its stream, once per context
  if (!ctx->h_xtot) {
    HIPCK(hipHostMalloc(reinterpret_cast<void**>(&ctx->h_xtot), shm::kRowWords * sizeof(unsigned long long) + 64,
                        hipHostMallocMapped | hipHostMallocCoherent));
    HIPCK(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->d_xtot), ctx->h_xtot, 0));
    std::memset(ctx->h_xtot, 0, shm::kRowWords * sizeof(unsigned long long) + 64);
    ctx->h_xgen = reinterpret_cast<unsigned int*>(ctx->h_xtot + shm::kRowWords);
    ctx->d_xgen = reinterpret_cast<unsigned int*>(ctx->d_xtot + shm::kRowWords);
  }
  if (!ctx->xstream && ctx->aux_stream) {
    if (int rj = cov_join_all(ctx)) return rj;
    ctx->xstream = ctx->aux_stream;
  }
  if (!ctx->xstream) {
    HIPCK(hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking));
    ctx->xstream_own = true;
  }
  // this rank's exchange buffer, zeroed (stamp 0 is never a pass stamp), published by IPC handle
  const size_t words = 2 * static_cast<size_t>(ctx->shm.max_sup) * shm::kRowWords;
  // fine-grained: peers' servers store into it over xGMI while this rank's totaler polls it
  // inside one running kernel; coarse-grained memory is coherent across devices only at kernel boundaries
  ctx->xrows.fine = true;
  HIPCK(ctx->xrows.reserve(words));
  HIPCK(hipMemset(ctx->xrows.p, 0, ctx->xrows.cap * sizeof(unsigned long long)));
  hipIpcMemHandle_t h;
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle slot");
  HIPCK(hipIpcGetMemHandle(&h, ctx->xrows.p));
  const uint64_t seq = ++ctx->xseq;  // every rank attaches in the same sequence
  std::memcpy(ctx->shm.ipc_handle(ctx->rank), &h, sizeof(h));
  ctx->shm.ipc_flag(ctx->rank)->store(seq, std::memory_order_release);
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < ctx->nranks; ++r) {
    while (ctx->shm.ipc_flag(r)->load(std::memory_order_acquire) < seq) {
      if (shm::elapsed_s(t0) > ctx->remote_deadline_s)
        return fail(ctx, MGICP_E_COMM, "xGMI row exchange: another rank did not publish its buffer");
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  for (int r = 0; r < ctx->nranks; ++r) {
    if (r == ctx->rank) continue;
    hipIpcMemHandle_t hr;
    std::memcpy(&hr, ctx->shm.ipc_handle(r), sizeof(hr));
    void* p = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&p, hr, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      for (void* q : ctx->xpeer) (void)hipIpcCloseMemHandle(q);
      ctx->xpeer.clear();
      return fail(ctx, MGICP_E_HIP, std::string("xGMI row exchange: hipIpcOpenMemHandle: ") + hipGetErrorString(e));
    }
    ctx->xpeer.push_back(p);
  }
  ctx->have_xgmi = true;
  ctx->st[kStTransport] = ctx->comm ? 5 : 4;
  return reset_stamps(ctx);  // every rank restarts its pass stamps with the transport
}

int mgicp_comm_attach_shm(mgicp_ctx* ctx, const char* name, size_t max_source_points) {
  if (!ctx) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = cov_join_all(ctx);  // the shard changes under them
  if (rc) return rc;
  rc = reset_stamps(ctx);  // the stamp count restarts with the transport on every rank
  if (rc) return rc;
  if (ctx->have_shm) {
    xgmi_detach(ctx);  // its rendezvous (and the peers' buffers) go with the segment
    (void)hipHostUnregister(ctx->shm.base);
    shm::detach(ctx->shm);
    ctx->have_shm = false;
    ctx->st[kStTransport] = ctx->comm ? 1 : 0;
  }
  if (!name) return MGICP_OK;  // detach only
  if (max_source_points == 0) max_source_points = size_t(32) << 20;
  if (max_source_points >= (size_t(1) << 31))
    return fail(ctx, MGICP_E_INVALID, "max_source_points: at most 2^31 - 2 points per cloud");
  const long long max_sup = static_cast<long long>((max_source_points + kSuperPts - 1) / kSuperPts);
  std::string err;
  shm::Segment seg;
  if (!shm::attach(seg, name, ctx->nranks, ctx->rank, max_sup, ctx->remote_deadline_s, err))
    return fail(ctx, MGICP_E_COMM, err);
  // the GPU writes its rows straight into the segment: map it into the device's address space
  hipError_t e = hipHostRegister(seg.base, seg.bytes, hipHostRegisterMapped);
  void* d = nullptr;
  if (e == hipSuccess) e = hipHostGetDevicePointer(&d, seg.base, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister(seg.base);
    shm::detach(seg);
    return fail(ctx, MGICP_E_HIP, std::string("hipHostRegister of the shared row segment: ") + hipGetErrorString(e));
  }
  ctx->shm = seg;
  ctx->shm_d = static_cast<unsigned char*>(d);
  ctx->have_shm = true;  // row stamps and gather indices count from the attach (reset_stamps above)
  ctx->st[kStTransport] = ctx->comm ? 3 : 2;
  return MGICP_OK;
}

int mgicp_debug_pass_stats(mgicp_ctx* ctx, long long out[8]) {
  if (!ctx || !out) return MGICP_E_INVALID;
  for (int i = 0; i < kStCount; ++i) out[i] = ctx->st[i];
  return MGICP_OK;
}

int mgicp_debug_server_time(mgicp_ctx* ctx, double* out_ms, long long* out_passes, long long* out_launches,
                            int reset) {
  if (!ctx || !out_ms || !out_passes || !out_launches) return MGICP_E_INVALID;
  *out_ms = ctx->srv_time_ms;
  *out_passes = ctx->srv_time_passes;
  *out_launches = ctx->srv_time_launches;
  if (reset) {
    ctx->srv_time_ms = 0;
    ctx->srv_time_passes = ctx->srv_time_launches = 0;
  }
  return MGICP_OK;
}

int mgicp_debug_target_cov_slice(mgicp_ctx* ctx, int nranks, int rank, double* out_c6) {
  if (!ctx || !out_c6 || nranks < 1 || rank < 0 || rank >= nranks) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = prepare(ctx, false);
  if (rc || (rc = cov_join_all(ctx))) return rc;  // set_target's k-NN launch still writes tgt.cov
  Cloud& t = ctx->tgt;
  const size_t N = static_cast<size_t>(nranks), r = static_cast<size_t>(rank);
  const size_t cnt = (t.n + N - 1) / N;
  const size_t a = std::min(t.n, r * cnt), b = std::min(t.n, (r + 1) * cnt);
  // target_cov's slice call, verbatim: the same range, the same N * cnt array layout
  if ((rc = compute_cov(ctx, t, a, b, N * cnt))) return rc;
  t.have_cov = false;  // only a slice is current: the next align recomputes the target's covariances
  const size_t st = t.cov_stride, m = b - a;
  std::vector<double2> h(3 * std::max<size_t>(m, 1));
  if (m) {
    const Cov3 c = t.cov3();
    HIPCK(hipMemcpyAsync(h.data(), c.a + a, m * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipMemcpyAsync(h.data() + m, c.b + a, m * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
    HIPCK(hipMemcpyAsync(h.data() + 2 * m, c.c + a, m * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
  }
  (void)st;
  if ((rc = sync(ctx))) return rc;
  for (size_t i = 0; i < m; ++i) {  // grid-sorted order, as the arrays hold them
    double* o = out_c6 + 6 * i;
    o[0] = h[i].x; o[1] = h[i].y; o[2] = h[m + i].x; o[3] = h[m + i].y; o[4] = h[2 * m + i].x; o[5] = h[2 * m + i].y;
  }
  return static_cast<int>(m);
}

int mgicp_debug_vlist_stats(mgicp_ctx* ctx, long long out[8]) {
  if (!ctx || !out) return MGICP_E_INVALID;
  for (int i = 0; i < 8; ++i) out[i] = 0;
  if (!ctx->vlist || !ctx->vl_valid || ctx->vl_off || !ctx->vl_alloc) return MGICP_OK;
  HIPCK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  unsigned int c3[3];
  HIPCK(hipMemcpyAsync(c3, ctx->vl_ctr.p, 3 * sizeof(unsigned int), hipMemcpyDeviceToHost, s));
  HIPCK(ctx->u64.reserve(64));
  HIPCK(launch_vl_stats(ctx->vl, ctx->vl_ncells, ctx->u64.p, s));
  unsigned long long st[64];
  HIPCK(hipMemcpyAsync(st, ctx->u64.p, sizeof(st), hipMemcpyDeviceToHost, s));
  int rc = sync(ctx);
  if (rc) return rc;
  out[0] = c3[1];
  out[1] = c3[2];
  out[2] = static_cast<long long>(st[0]);
  out[3] = static_cast<long long>(st[1]);
  out[4] = static_cast<long long>(st[2]);
  out[5] = static_cast<long long>(st[3]);
  out[6] = c3[0];
  out[7] = static_cast<long long>(ctx->vl_ncells);
  return MGICP_OK;
}

// r06: the objective's stream order -- original indices of this rank's source points in the order the
// compacted streams (and so every sum's fixed tree) visit them; the oracle's summation-order ledger runs
// the engine's tree over it (oracle/gicp_ref.c ref_set_sum_order).  Returns the count (<= cap written).
int mgicp_debug_source_order(mgicp_ctx* ctx, uint32_t* out, size_t cap) {
  if (!ctx || !out) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = prepare(ctx, false);
  if (rc) return rc;
  const size_t p0 = ctx->shard_p0(), ns = ctx->shard_p1() - p0;
  if (cap < ns) return fail(ctx, MGICP_E_INVALID, "debug_source_order: cap below the shard's point count");
  HIPCK(hipMemcpyAsync(out, ctx->src.perm.p + p0, ns * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  if ((rc = sync(ctx))) return rc;
  return static_cast<int>(ns);
}

int mgicp_debug_covariances(mgicp_ctx* ctx, int which, double* out_c6) {
  if (!ctx || !out_c6 || (which != 0 && which != 1)) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = prepare(ctx, true);
  if (rc) return rc;
  // both clouds: prepare counts set_target's running covariances as current
  if ((rc = cov_join_all(ctx))) return rc;
  if (which == 0 &&!(ctx->src.have_cov && ctx->src.cov_p0 == ctx->shard_p0() && ctx->src.cov_p1 == ctx->shard_p1())) {
    // every source covariance (lazy mode computes only the accepted points' ones)
    if ((rc = compute_cov(ctx, ctx->src, ctx->shard_p0(), ctx->shard_p1()))) return rc;
    if (ctx->src_lazy_ready) HIPCK(hipMemsetAsync(ctx->cov_ok.p, 1, ctx->shard_p1() - ctx->shard_p0(), ctx->stream));
  }
  Cloud& cl = which ? ctx->tgt : ctx->src;
  const size_t n = cl.n;
  const size_t st = cl.cov_stride;
  std::vector<double2> h(3 * st);
  std::vector<uint32_t> perm(n);
  HIPCK(hipMemcpyAsync(h.data(), cl.cov.p, 3 * st * sizeof(double2), hipMemcpyDeviceToHost, ctx->stream));
  HIPCK(hipMemcpyAsync(perm.data(), cl.perm.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  if ((rc = sync(ctx))) return rc;
  for (size_t p = 0; p < n; ++p) {
    double* o = out_c6 + 6 * static_cast<size_t>(perm[p]);
    o[0] = h[p].x; o[1] = h[p].y;
    o[2] = h[st + p].x; o[3] = h[st + p].y;
    o[4] = h[2 * st + p].x; o[5] = h[2 * st + p].y;
  }
  return MGICP_OK;
}

static int debug_corr(mgicp_ctx* ctx, const float T_cm[16], bool seeded, int* out_tgt, double* out_M6) {
  if (!ctx || !T_cm) return MGICP_E_INVALID;
  if (seeded && !ctx->seed_valid) return fail(ctx, MGICP_E_INVALID, "no previous sweep to seed from");
  HIPCK(hipSetDevice(ctx->device));
  int rc = prepare(ctx, true);
  if (rc) return rc;
  if ((rc = ensure_iter_buffers(ctx))) return rc;
  const size_t n = ctx->src.n;
  const Mat4 G = Mat4::identity();
  if ((rc = set_output(ctx, G))) return rc;
  if ((rc = correspond(ctx, Mat4::from_cm(T_cm), G, seeded))) return rc;
  if (ctx->vl_valid) ctx->vl_groups++;
  const size_t p0 = ctx->shard_p0(), p1 = ctx->shard_p1(), ns = p1 - p0;
  std::vector<uint32_t> nn(ns), flag(ns), perm(n), tperm(ctx->tgt.n);
  std::vector<uint32_t> ccnt(static_cast<size_t>(chunk_count(ns)));
  HIPCK(hipMemcpyAsync(nn.data(), ctx->prev_pos.p, ns * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCK(hipMemcpyAsync(flag.data(), ctx->flags.p, ns * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  if (!ccnt.empty())
    HIPCK(hipMemcpyAsync(ccnt.data(), ctx->ccnt.p, ccnt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCK(hipMemcpyAsync(perm.data(), ctx->src.perm.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCK(hipMemcpyAsync(tperm.data(), ctx->tgt.perm.p, ctx->tgt.n * sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  const size_t cap = ctx->corr_cap;
  std::vector<double> M(6 * cap);
  HIPCK(hipMemcpyAsync(M.data(), ctx->corr_d.p, 6 * cap * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  if ((rc = sync(ctx))) return rc;
  int cnt = 0;
  size_t rank = 0;  // accepted before k in k's chunk
  for (size_t p = p0; p < p1; ++p) {
    const size_t i = perm[p], k = p - p0;
    if (k % kChunkPts == 0) rank = 0;
    const bool ok = flag[k] != 0;
    if (out_tgt) out_tgt[i] = ok ? static_cast<int>(tperm[nn[k]]) : -1;
    if (out_M6) {
      double* o = out_M6 + 6 * i;
      const size_t at = (k / kChunkPts) * kChunkPts + rank;  // the chunk's run of the streams
      for (int v = 0; v < 6; ++v) o[v] = ok ? M[v * cap + at] : 0.0;
    }
    if (ok) {
      cnt++;
      rank++;
    }
  }
  for (size_t c = 0; c < ccnt.size(); ++c) {  // the compaction's counts agree with the flags
    size_t m = 0;
    for (size_t k = c * kChunkPts; k < std::min(ns, (c + 1) * kChunkPts); ++k) m += flag[k] != 0;
    if (m != ccnt[c]) return fail(ctx, MGICP_E_HIP, "chunk counts disagree with the sweep's flags");
  }
  return cnt;
}

int mgicp_debug_correspondences(mgicp_ctx* ctx, const float T_cm[16], int* out_tgt, double* out_M6) {
  return debug_corr(ctx, T_cm, false, out_tgt, out_M6);
}

int mgicp_debug_correspondences_seeded(mgicp_ctx* ctx, const float T_cm[16], int* out_tgt, double* out_M6) {
  return debug_corr(ctx, T_cm, true, out_tgt, out_M6);
}

int mgicp_debug_fdf(mgicp_ctx* ctx, const double x[6], double* f, double g6[6]) {
  if (!ctx || !x || !ctx->have_corr) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  GateGuard guard{ctx};  // no queued pass / live server outlives the call
  DeviceFunctor fn{ctx};
  Vec6 xv, gv;
  for (int i = 0; i < 6; ++i) xv[i] = x[i];
  double fv = 0;
  int rc = fn.eval(xv, fv, gv);
  if (rc) return rc;
  if (f) *f = fv;
  if (g6)
    for (int i = 0; i < 6; ++i) g6[i] = gv[i];
  return MGICP_OK;
}

int mgicp_debug_fdf_sums(mgicp_ctx* ctx, const double x[6], double out16[16]) {
  if (!ctx || !x || !out16 || !ctx->have_corr) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  GateGuard guard{ctx};
  DeviceFunctor fn{ctx};
  Vec6 xv;
  for (int i = 0; i < 6; ++i) xv[i] = x[i];
  return fn.pass(xv, out16);
}

int mgicp_debug_pass_bench(mgicp_ctx* ctx, const double x[6], int npasses, int mode, double* out_ms,
                           double out16[16]) {
  if (!ctx || !x || npasses < 1 || npasses > 100000 || (mode != 0 && mode != 1) || !ctx->have_corr)
    return MGICP_E_INVALID;
  if (ctx->comm || ctx->nranks != 1 || ctx->have_shm)
    return fail(ctx, MGICP_E_INVALID, "pass bench: single-rank contexts only");
  HIPCK(hipSetDevice(ctx->device));
  int rc = sync(ctx);  // cancels any queued pass / live server
  if (rc) return rc;
  if ((rc = ensure_host_red(ctx))) return rc;
  Vec6 xv;
  for (int i = 0; i < 6; ++i) xv[i] = x[i];
  const Xf34 A = apply_state(xv).xf();
  const size_t ns = ctx->shard_p1() - ctx->shard_p0();
  const CorrSoA c = corr_soa(ctx);
  hipEvent_t a = nullptr, b = nullptr;
  HIPCK(hipEventCreate(&a));
  HIPCK(hipEventCreate(&b));
  HIPCK(hipEventRecord(a, ctx->stream));
  hipError_t e = hipSuccess;
  const bool rows = mode == 0 && ctx->host_rows;
  if (rows && (rc = ensure_rows(ctx))) return rc;
  if (rows) HIPCK(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream));
  if (mode == 0) {
    const int cap = ctx->srv_cus > 0 ? std::min(ctx->srv_cus, ctx->cus) : ctx->cus;
    const int nb = fdf_server_blocks(ns, cap, ctx->srv_waves);
    if (nb <= 0) {
      (void)hipEventDestroy(a);
      (void)hipEventDestroy(b);
      return fail(ctx, MGICP_E_INVALID, "pass bench: shard not servable by the resident server");
    }
    const unsigned long long seq0 = ++ctx->pass_seq;
    const RowView rv = row_view(ctx);
    e = launch_fdf_server(c, ctx->ccnt.p, ns, ctx->partial.p, ctx->spart.p, ctx->tickets.p,
                          ctx->d_h_red, ctx->d_flag, seq0, ctx->d_cmd, ctx->mail, ctx->gate_timeout, ctx->d_ptimes,
                          npasses, A, rows ? rv.dev_rows(0) : nullptr, rv.stride, nb, ctx->srv_waves, 1, -1,
                          ctx->srv_tagged ? ctx->tpart.p : nullptr, ctx->stream);
    ctx->pass_seq = seq0 + static_cast<unsigned long long>(npasses);  // the closing cancel's stamp too
  } else {
    const int nb = fdf_grid_blocks(ns, ctx->fdf_max_blocks);
    for (int k = 0; k < npasses && e == hipSuccess; ++k)
      e = launch_fdf_soa(c, ctx->ccnt.p, ns, A, ctx->partial.p, ctx->spart.p, nb, ctx->tickets.p,
                         ctx->d_h_red, ctx->alt_sweep ? (k & 1) : 0, ctx->d_flag, ++ctx->pass_seq, ctx->stream);
  }
  if (e == hipSuccess) e = hipEventRecord(b, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  float ms = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  HIPCK(e);
  if (MGICP_PASS_DIAG && mode == 0) {
    PassCmd m{};
    HIPCK(hipMemcpy(&m, ctx->mail, sizeof(PassCmd), hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[srv-debug] seq0 %llu npasses %d ms %.3f | mail:", ctx->pass_seq - npasses, npasses, ms);
    for (int i = 0; i < 16; ++i)
      std::fprintf(stderr, " %x:%x", static_cast<unsigned>(m.h[i] >> 32), static_cast<unsigned>(m.h[i]));
    std::fprintf(stderr, "\n");
    if (ctx->h_ptimes)
      for (unsigned long long q = ctx->pass_seq - npasses; q < ctx->pass_seq + 1; ++q)
        std::fprintf(stderr, "[srv-debug] pass %llu: gate exit %llu finish %llu\n", q, ctx->h_ptimes[2 * (q & 1023)],
                     ctx->h_ptimes[2 * (q & 1023) + 1]);
  }
  if (rows) {
    // the host-row tickets are left as multiples of the supers' sizes: re-arm them
    HIPCK(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream));
    double tot[kRedVals];
    // the timing form stamps each pass's rows with its sequence number | 2^31
    const Xf34 unused{};
    if ((rc = wait_rows(ctx, static_cast<unsigned int>(ctx->pass_seq - 1) | 0x80000000u, unused, tot, false))) return rc;
    if ((rc = sync(ctx))) return rc;
    if (out16) std::memcpy(out16, tot, kRedVals * sizeof(double));
  } else {
    if (__atomic_load_n(ctx->h_flag, __ATOMIC_ACQUIRE) != ctx->pass_seq - (mode == 0 ? 1 : 0))
      return fail(ctx, MGICP_E_HIP, "pass bench: the last pass did not publish its sums");
    if (out16) std::memcpy(out16, ctx->h_red, kRedVals * sizeof(double));
  }
  if (out_ms) *out_ms = static_cast<double>(ms) / npasses;
  return MGICP_OK;
}

int mgicp_debug_moments(mgicp_ctx* ctx, const float T_cm[16], double out80[80]) {
  if (!ctx || !T_cm || !out80 || !ctx->seed_valid) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = moments_pass(ctx, Mat4::from_cm(T_cm), ctx->last_guess);
  if (rc) return rc;
  std::memcpy(out80, ctx->mom, kMomVals * sizeof(double));
  return MGICP_OK;
}

int mgicp_debug_supers(mgicp_ctx* ctx, int kind, const double* arg, double* out, int cap) {
  if (!ctx || !arg || !out || kind < 0 || kind > 2) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const long long nsup = ctx->nsup_local();
  if (nsup > cap) return fail(ctx, MGICP_E_INVALID, "debug_supers: output too small");
  const int nv = kind == 1 ? kMomVals : kRedVals;
  float Tcm[16];
  for (int i = 0; i < 16 && kind != 0; ++i) Tcm[i] = static_cast<float>(arg[i]);
  int rc;
  const double* sup = ctx->spart.p;
  if (kind == 0) {  // one objective pass at x over the last sweep, stopped at the supers
    if (!ctx->have_corr) return fail(ctx, MGICP_E_INVALID, "no correspondence sweep yet");
    cancel_gated(ctx);
    Vec6 x;
    for (int i = 0; i < 6; ++i) x[i] = arg[i];
    const size_t ns = ctx->shard_p1() - ctx->shard_p0();
    // host-row passes leave the tickets as multiples of their supers' sizes
    HIPCK(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets_n * sizeof(unsigned int), ctx->stream));
    HIPCK(launch_fdf_soa(corr_soa(ctx), ctx->ccnt.p, ns, apply_state(x).xf(), ctx->partial.p,
                         ctx->spart.p, fdf_grid_blocks(ns, ctx->fdf_max_blocks), ctx->tickets.p, nullptr, 0,
                         nullptr, 0, ctx->stream));
  } else if (kind == 1) {
    if (!ctx->seed_valid) return fail(ctx, MGICP_E_INVALID, "no correspondence sweep yet");
    if ((rc = moments_pass(ctx, Mat4::from_cm(Tcm), ctx->last_guess, true))) return rc;
    sup = ctx->msuper.p;
  } else {
    if ((rc = prepare(ctx, false)) || (rc = ensure_iter_buffers(ctx))) return rc;
    const double mr = arg[16] > 0 ? arg[16] : 1.7976931348623157e308;
    if ((rc = fitness_supers(ctx, Mat4::from_cm(Tcm), mr))) return rc;
  }
  if (nsup > 0)
    HIPCK(hipMemcpyAsync(out, sup, static_cast<size_t>(nsup) * nv * sizeof(double), hipMemcpyDeviceToHost,
                         ctx->stream));
  if ((rc = sync(ctx))) return rc;
  return static_cast<int>(nsup);
}

int mgicp_debug_finish_supers(mgicp_ctx* ctx, int nv, const double* rows, long long nsup, long long maxsup,
                              int nranks, double* out) {
  if (!ctx || !rows || !out || (nv != kRedVals && nv != kMomVals) || nsup < 0 || maxsup < 0 || nranks < 1)
    return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const size_t nrow = static_cast<size_t>(nranks) * maxsup * nv;
  DevBuf<double> d, o;
  HIPCK(d.reserve(std::max<size_t>(nrow, 1)));
  HIPCK(o.reserve(nv));
  if (nrow) HIPCK(hipMemcpyAsync(d.p, rows, nrow * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIPCK(launch_finish_supers(d.p, nsup, maxsup, nranks, nv, o.p, ctx->stream));
  HIPCK(hipMemcpyAsync(out, o.p, nv * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  int rc = sync(ctx);
  d.release();
  o.release();
  return rc;
}

int mgicp_debug_wave_reduce(mgicp_ctx* ctx, const double* in, int nwaves, double* out_tree, double* out_rs) {
  if (!ctx || !in || !out_tree || !out_rs || nwaves <= 0) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  const size_t nin = static_cast<size_t>(nwaves) * 64 * 16, nout = static_cast<size_t>(nwaves) * 16;
  DevBuf<double> d, t, r;
  HIPCK(d.reserve(nin));
  HIPCK(t.reserve(nout));
  HIPCK(r.reserve(nout));
  HIPCK(hipMemcpyAsync(d.p, in, nin * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIPCK(launch_wave_reduce_check(d.p, nwaves, t.p, r.p, ctx->stream));
  HIPCK(hipMemcpyAsync(out_tree, t.p, nout * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPCK(hipMemcpyAsync(out_rs, r.p, nout * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  int rc = sync(ctx);
  d.release();
  t.release();
  r.release();
  return rc;
}

int mgicp_debug_trace(mgicp_ctx* ctx, float* out, int max_iters) {
  if (!ctx || !out || max_iters < 0) return MGICP_E_INVALID;
  const int n = static_cast<int>(ctx->trace.size() / 16);
  const int m = std::min(n, max_iters);
  std::memcpy(out, ctx->trace.data(), static_cast<size_t>(m) * 16 * sizeof(float));
  return n;
}

int mgicp_debug_kernel_times(mgicp_ctx* ctx, double out_ms[MGICP_KERNEL_FAMILIES],
                             int out_counts[MGICP_KERNEL_FAMILIES]) {
  if (!ctx || !out_ms) return MGICP_E_INVALID;
  prof_resolve(ctx);
  for (int i = 0; i < kFams; ++i) {
    out_ms[i] = ctx->fam_cnt[i] ? ctx->fam_ms[i] / ctx->fam_cnt[i] : 0.0;
    if (out_counts) out_counts[i] = ctx->fam_cnt[i];
  }
  return MGICP_OK;
}

int mgicp_set_profiling(mgicp_ctx* ctx, int on) {
  if (!ctx) return MGICP_E_INVALID;
  (void)hipSetDevice(ctx->device);
  cancel_gated(ctx);
  (void)hipStreamSynchronize(ctx->stream);
  srv_release(ctx);
  prof_resolve(ctx);
  ctx->profiling = on != 0;
  ctx->prof_tick = 0;
  for (int i = 0; i < kFams; ++i) {
    ctx->fam_ms[i] = 0;
    ctx->fam_cnt[i] = 0;
  }
  return MGICP_OK;
}

// r05 target cache: [0] the current target was adopted from the cache, [1] adoptions and [2] donations
// on this device so far (process-wide), [3] an entry is cached on this device, [4] the source grid's start
// from the cached target's cell size (r05; since r06 always 0: the source's grid never depends on the target)
int mgicp_debug_cache_stats(mgicp_ctx* ctx, long long out[5]) {
  if (!ctx || !out) return MGICP_E_INVALID;
  TargetCache& c = g_tcache[ctx->device & 63];
  std::lock_guard<std::mutex> lk(c.mu);
  out[0] = ctx->tcache_adopted ? 1 : 0;
  out[1] = c.hits;
  out[2] = c.donations;
  out[3] = c.valid ? 1 : 0;
  out[4] = 0;  // r06: no speculative source grid any more (the source's grid never depends on the target)
  return MGICP_OK;
}

void mgicp_release_cache(void) {
  int dev = 0;
  const bool have = hipGetDevice(&dev) == hipSuccess;
  for (int d = 0; d < 64; ++d) {
    TargetCache& c = g_tcache[d];
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.valid && !c.t.orig.p && !c.vl_pool.p) continue;
    (void)hipSetDevice(d);
    tcache_clear_locked(c);
  }
  if (have) (void)hipSetDevice(dev);
}

// Test / diagnostic forms of the engine (INTEGRATION.md "Debug options"): explicit per-context calls,
// never environment variables, so a deployment cannot switch a kernel by accident.
// Pending covariance launches are joined and the stream drained first; list-related options drop the
// target's 1-NN cell lists.
int mgicp_debug_option(mgicp_ctx* ctx, const char* name, double value) {
  if (!ctx || !name) return MGICP_E_INVALID;
  HIPCK(hipSetDevice(ctx->device));
  int rc = cov_join_all(ctx);
  if (rc || (rc = sync(ctx))) return rc;
  const std::string n(name);
  const bool on = value != 0.0;
  const int iv = static_cast<int>(value);
  if (n == "resident") ctx->resident = on;              // resident pass server (else one launch per pass)
  else if (n == "host_rows") ctx->host_rows = on;       // server supers as stamped host rows (else device total)
  else if (n == "srv_cus") ctx->srv_cus = std::max(0, iv);  // cap on the server's blocks (0 = every CU)
  else if (n == "fused_finish") ctx->fused_finish = on; // in-launch reduction finish of launched passes
  else if (n == "gated") ctx->gated = on;               // launched passes pre-queued behind a command gate
  else if (n == "async_cov") ctx->async_tgt = on && ctx->aux_stream;  // set_*'s covariance head start
  else if (n == "lazy_src_cov") {                       // source covariances of accepted points only
    ctx->lazy_src_cov = on;
    ctx->src.have_cov = false;
    ctx->src_lazy_ready = false;
  } else if (n == "async_ring_cap") {                   // rings the source's lazy-mode head start searches (-1: all)
    ctx->async_ring_cap = iv;
  } else if (n == "knn_wave") {                         // k-NN: lazy pass + hand-offs one wave per point (1) or per lane (0)
    ctx->knn_wave = on;
  } else if (n == "knn_logged") {                       // k-NN: the logged kernel + hand-off (1) or the register-list kernel only (0)
    ctx->knn_logged = on;
    ctx->src.have_cov = ctx->tgt.have_cov = false;
    ctx->src_lazy_ready = false;
  } else if (n == "vlist") ctx->vlist = on, ctx->vl_valid = false;  // the target's 1-NN cell lists
  else if (n == "vlist_cold") ctx->vl_cold_groups = std::max(0, iv), ctx->vl_valid = false;
  else if (n == "vlist_eager") ctx->vl_eager = on, ctx->vl_valid = false;
  else if (n == "vlist_stats") ctx->vl_stats = on;      // per-sweep list statistics on stderr
  else if (n == "fuse_compact") ctx->fuse_compact = on; // compaction fused into listed sweeps
  else if (n == "target_cache") ctx->tcache_on = on;    // adopt / leave the target state (process cache)
  else if (n == "grid_occ") {                           // grid sizing (points per non-empty cell), next set_*
    if (!(value >= 1.0 && value <= 256.0)) return fail(ctx, MGICP_E_INVALID, "grid_occ must be in [1, 256]");
    ctx->occupancy = value;
  } else if (n == "bar_cmd") {                          // server commands through the BAR (else pinned copy)
    ctx->bar = on;
    if (!on && ctx->bar_cmd) {
      (void)hipFree(ctx->bar_cmd);
      ctx->bar_cmd = nullptr;
    }
    if (on && !ctx->bar_cmd) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, ctx->device) == hipSuccess && prop.isLargeBar &&
          hipExtMallocWithFlags(reinterpret_cast<void**>(&ctx->bar_cmd), sizeof(PassCmd), hipDeviceMallocFinegrained) ==
              hipSuccess)
        HIPCK(hipMemset(ctx->bar_cmd, 0, sizeof(PassCmd)));
      else
        ctx->bar_cmd = nullptr;
    }
  } else {
    return fail(ctx, MGICP_E_INVALID, "unknown debug option: " + n);
  }
  return MGICP_OK;
}

}  // extern "C"
