// mgicp_internal.hpp -- shared device-side layouts and kernel launchers of libmgicp.so.
//
// HBM layout (DESIGN.md "Data layout"): every cloud lives in a uniform grid sorted by
// linear cell index (z-major, then y, then x; stable in the original point index), so a
// row of cells is one contiguous range of the point array:
//   pts        float4[n]      (x, y, z, bit_cast<float>(original index))
//   cell_start uint32[nc + 1] exclusive prefix of per-cell counts (dense over the bbox)
//   cov        3 x double2[n] symmetric covariance {c00,c01},{c02,c11},{c12,c22}
// Per source point of the shard (sorted order), rewritten every outer iteration:
//   nn_pos     uint32[n]      matched target sorted position (UINT32_MAX = rejected)
//   flags/pos  uint32[n+1]    acceptance and its exclusive scan (compacted slot)
// Accepted correspondences: CorrSoA (below), 72 bytes each.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace mgicp {

struct GridView {
  float ox, oy, oz;   // grid origin (bbox min)
  float h, inv_h;     // cell edge and its reciprocal
  float slop;         // absolute rounding slack for ring lower bounds (metres)
  int nx, ny, nz;
  const uint32_t* cell_start;  // nx*ny*nz + 1
  const float4* pts;           // sorted points
  // optional empty-space map: per cell, the Chebyshev distance (in cells) to the nearest
  // non-empty cell, capped at kEmptyCap + 1; rings closer than it hold no point
  const uint8_t* empty_dist;
  // optional seed map (with empty_dist): per cell within the cap, the sorted position of a point in
  // a Chebyshev-nearest non-empty cell -- a real candidate that seeds an unseeded 1-NN search
  const uint32_t* seed;
  // optional per-cell point boxes (2 float4 per cell: min xyz | bits(start), max xyz | bits(end));
  // 1-NN searches skip cells whose point box lies beyond their bound
  const float4* boxes;
  // optional pair-interleaved copy of pts for the wave-uniform 1-NN scan (2 float4 per pair of
  // points: x0 x1 y0 y1 | z0 z1 w0 w1; pair_count(n) pairs, far sentinels past n)
  const float4* pairs;
};

#ifndef MGICP_EMPTY_CAP
#define MGICP_EMPTY_CAP 15
#endif
constexpr int kEmptyCap = MGICP_EMPTY_CAP;

struct Cov3 {  // SoA triple of double2 arrays
  double2* a;  // {m00, m01}
  double2* b;  // {m02, m11}
  double2* c;  // {m12, m22}
};

// Accepted correspondences of one outer iteration, compacted in grid-sorted source order and
// stored as 12 streams (each padded to a multiple of 4 elements) so that an objective pass reads
// 72 bytes per correspondence with 16-byte loads and no branch.
struct CorrSoA {
  float *sx, *sy, *sz, *qx, *qy, *qz;
  double *m00, *m01, *m02, *m11, *m12, *m22;
};

// Number of values reduced per objective pass:
//   [0] f-sum  [1..3] g_t sum  [4..12] Rsum (row-major)  [13] count  [14..15] pad
constexpr int kRedVals = 16;
constexpr int kMaxK = 32;  // largest k_correspondences_ the covariance kernel serves
constexpr int kRedThreads = 256;
// Number of values reduced per Gauss-Newton moment pass (MGICP_SOLVER_GN):
//   [0] sum r0'M r0  [1..12] sum (M r0) w'  [13..72] sum M_p (w w')_q  [73] count  [74..79] pad
constexpr int kMomVals = 80;

// The fixed global reduction tree of every sharded sum (objective passes, Gauss-Newton moments,
// fitness): chunks of kChunkPts grid-sorted source positions (one wave each), supers of
// kSuperChunks chunks, then the total over supers.  Shards start on super boundaries (rank r owns
// supers [nsup * r / N, nsup * (r + 1) / N)), so every N reproduces the N = 1 sums bit for bit.
constexpr int kChunkPts = 1024;
constexpr int kSuperChunks = 32;
constexpr size_t kSuperPts = static_cast<size_t>(kChunkPts) * kSuperChunks;
inline int chunk_count(size_t n) { return static_cast<int>((n + kChunkPts - 1) / kChunkPts); }
__host__ __device__ inline long long super_first(int r, long long nsup, int nranks) {
  return nsup * r / nranks;
}
__host__ __device__ inline int super_owner(long long s, long long nsup, int nranks) {
  int r = static_cast<int>(s * nranks / (nsup > 0 ? nsup : 1));
  if (r > nranks - 1) r = nranks - 1;
  while (r > 0 && s < super_first(r, nsup, nranks)) --r;
  while (r < nranks - 1 && s >= super_first(r + 1, nsup, nranks)) ++r;
  return r;
}

// Xform as 3x4 row-major float (the top three rows of an Eigen::Matrix4f).
struct Xf34 { float m[12]; };

// Command block of a pre-launched (gated) objective pass, in pinned mapped host memory (and its
// device-memory forward).  Self-validating without fences: every 8-byte half carries one payload
// word (low 32 bits) and the low 32 bits of the pass's sequence number (high 32 bits); aligned
// 8-byte stores and loads are single-copy atomic on both sides, so a reader that finds the stamp
// in all kCmdWords halves holds a complete command of that pass -- in the same PCIe round trip
// that detects it.  Words: [0..11] A (Xf34 bit patterns), [12] op, [13] sweep direction, [14] the
// pass's row stamp (host-row passes: the objective-pass index, identical on every rank, that stamps
// the super rows and selects their parity buffer).  A waiting block that finds a complete command
// with a LATER sequence number was left behind by a cancel and exits.
constexpr unsigned int kPassRun = 1;
constexpr unsigned int kPassCancel = 2;
constexpr int kCmdWords = 15;
struct alignas(128) PassCmd {
  unsigned long long h[16];
};
struct Rot33d { double m[9]; };

// ---- launchers (mgicp_kernels.hip); all asynchronous on `s` ----
hipError_t launch_pack_points(const void* raw, size_t n, size_t stride, float4* out,
                              hipStream_t s);
hipError_t launch_bbox(const float4* pts, size_t n, float* partial /*nb*8*/, int nb,
                       hipStream_t s);
hipError_t launch_cell_hist(const float4* pts, size_t n, float ox, float oy, float oz,
                            float inv_h, int nx, int ny, int nz, uint32_t* counts,
                            uint32_t* keys /*nullable*/, hipStream_t s);
// r06: the grid's sizing sketch (cell_sketch_kernel): kSketchR one-byte HyperLogLog registers of the
// occupied cells at each of kSketchScales cell sizes (1 / inv[k]) over origin (ox, oy, oz), in one pass;
// `partial` holds (kSketchBlocks + 32) * kSketchScales * kSketchR bytes, the merged registers land in `out`
constexpr int kSketchScales = 16;
constexpr int kSketchLog2R = 7;  // 128 registers per size (~9 % error): 8 KiB of LDS, so a sketch block
                                  // fits beside the source's k-NN (12 KiB per wave, 12 waves per CU)
constexpr int kSketchR = 1 << kSketchLog2R;
constexpr int kSketchBlocks = 1024;  // of 256 threads (4 per CU: the per-scale LDS read-check is latency-bound)
struct SketchScales { float inv[kSketchScales]; };
hipError_t launch_cell_sketch(const float4* pts, size_t n, float ox, float oy, float oz, const SketchScales& sc,
                              uint8_t* partial, uint8_t* out, hipStream_t s);
// r06: cell_start[0..nc] of a grid from its sorted keys (no histogram): `ends` (nc + 1 words) is
// zeroed and receives each non-empty cell's end, then an exclusive max-scan gives the starts
size_t cell_start_scratch_bytes(size_t nc);
hipError_t launch_cell_starts(const uint32_t* keys_sorted, size_t n, size_t nc, uint32_t* ends, uint32_t* cell_start,
                              void* scratch, size_t scratch_bytes, hipStream_t s);
hipError_t launch_gather_sorted(const float4* pts, const uint32_t* perm, size_t n,
                                float4* out, hipStream_t s);
hipError_t launch_xform_points(const float4* in, size_t n, Xf34 T, float4* out,
                               hipStream_t s);
// k-NN covariances of [p0, p1).  fb / fb_count (nullable): the logged-threshold kernel, which lists
// in fb (count in *fb_count, device, zeroed by the caller) the points it leaves to the register-list
// kernel; run that list with perm = fb, p0 = 0, p1 = count, fb = nullptr.
// ring_cap >= 0 (logged kernel only): a query whose search passes that ring gives up -- no
// covariance, not listed in fb, ok[p] stays 0; every other query sets ok[p] = 1 (ok nullable)
// r06: exact k-NN covariances with one wave per query (the lazy pass, the hand-off), queries list[i] for
// i < *count (count non-null, device-side) or n; blocks <= 0: one wave per query
hipError_t launch_knn_wave(const GridView& g, int k, double eps, const uint32_t* list, const unsigned int* count,
                           size_t n, Cov3 cov, hipStream_t s, int blocks = 0);
hipError_t launch_knn_cov(const GridView& g, int k, double eps, size_t p0, size_t p1,
                          Cov3 cov, const uint32_t* perm /*nullable: query order*/, uint32_t* fb,
                          unsigned int* fb_count, hipStream_t s, int ring_cap = -1, uint8_t* ok = nullptr,
                          int chain = 0 /*> 0: the hand-off launch follows on s, that many blocks, device count*/,
                          bool wave_handoff = true /*r06: the chained hand-off by knn_wave_kernel*/);
// nn_pos: per source point (shard-relative) the matched target sorted position, UINT32_MAX when
// rejected; with `seeded` its previous contents seed the exact 1-NN search.  flags: 1 if accepted.
hipError_t launch_correspond(const GridView& tgt, const float4* src, size_t p0, size_t p1, Xf34 T,
                             double thr, int seeded, uint32_t* nn_pos, uint32_t* flags,
                             const uint32_t* qperm /*nullable: query order*/, hipStream_t s);
// the wave-uniform form (needs tgt.pairs): lanes whose seed bound exceeds sqrt(rcap2), or waves whose
// union box exceeds max_rows rows or max_xcells cells along x, or whose mean seed bound is below
// union_min_r cells, finish with the per-lane search
hipError_t launch_correspond_wave(const GridView& tgt, const float4* src, size_t p0, size_t p1, Xf34 T,
                                  double thr, int seeded, uint32_t* nn_pos, uint32_t* flags, const uint32_t* qperm,
                                  float rcap2, int max_rows, int max_xcells, float union_min_r,
                                  void* work /*nullable: NnWork list of stragglers, nn_work_bytes(p1 - p0)*/,
                                  unsigned int* work_n, int split_max /*waves with at most this many stragglers hand them on*/,
                                  int lds_cap /*small-ball waves: union box staged in LDS when it has <= lds_cap points*/,
                                  hipStream_t s);
size_t nn_work_bytes(size_t n);

// ---- the target's 1-NN cell lists (r04; DESIGN.md "1-NN cell lists") ----
// A fine uniform grid over the target's bbox grown by the gate.  Per cell: the target points that can
// be the exact 1-NN (fp32 FLANN d2, original-index tie-break) of some query in the cell whose d2 is
// below the gate -- a superset, pruned by the affine dominance test against 9 anchor points -- or
// "reject" (no target point within the gate of the cell).  Lists are built the first time a sweep
// queries the cell and persist until the target or the gate changes.
constexpr uint32_t kVlNotBuilt = 0xFFFFFFFFu;  // never queried
constexpr uint32_t kVlRequested = 0xFFFFFFFEu; // queued for this sweep's build
constexpr uint32_t kVlOverflow = 0xFFFFFFFDu;  // more than kVlMaxList entries / candidates / pool full
constexpr uint32_t kVlReject = 0xFFFFFFFCu;    // no target point within the gate of the cell
constexpr uint32_t kVlTouched = 0x80000000u;   // | epoch: first queried in sweep `epoch` (built when queried
                                               // again in a later sweep); values below: (off4 << 6) | count
constexpr int kVlLong = 63;                    // count field 63: a long list -- its true count in the x bits of a
                                               // header entry at off, its entries from off + 4
                                               // (lists padded to a multiple of 4 with far sentinels; off4 = list
                                               // start / 4, < 2^25)
struct VListView {
  float ox, oy, oz;      // fine grid origin
  float c, inv_c;        // fine cell edge and its float reciprocal
  float es;              // box growth covering the fp32 cell assignment of queries
  int nx, ny, nz;
  double gate;           // max correspondence distance the lists are built for
  uint32_t* cell;        // nx * ny * nz states / (off << 6 | count)
  float4* pool;          // list entries {x, y, z, bits(sorted target position)}
  const float4* tpts;    // the target's sorted points (w = original index: exact-distance ties only)
  uint32_t pool_cap;     // entries (< 2^26)
  unsigned int* ctr;     // [0] pool head (persistent), [1] cells requested, [2] queries pending, [3] deferred
                         // chunks, [4] cells left to the build's second pass (per sweep)
  uint32_t* build;       // requested cells of this sweep
  uint32_t* bcentre;     // per requested cell: sorted position of the cell centre's 1-NN (or none)
  uint32_t build_cap;
  uint32_t* pend;        // shard-relative positions of this sweep's queries without a list
  uint32_t epoch;        // this sweep's number (1 .. 2^30 - 1)
  int eager;             // 1: build a cell's list at its first query (else at its first query in a later sweep)
};
// one sweep over the lists: listed queries answered at once, reject cells rejected, the others
// queued (pend) and their cells requested; then the requested cells' lists are built and the
// pending queries answered by the exact per-lane search (seeded like correspond_kernel)
// the compaction fused into a listed sweep (vl_query_compact_kernel): its inputs; chunks it cannot
// finish (a pending query, a lazy source covariance not computed yet) are listed in `defer`, count
// in VListView::ctr[3], for launch_compact(..., defer, ctr + 3)
struct FusedCompact {
  Cov3 cov_s, cov_t;
  Rot33d R;
  const uint8_t* cov_ok;  // lazy source mode: per shard point, covariance computed (nullptr: all are)
  uint32_t* ccnt;
  uint32_t* defer;
  CorrSoA out;
};
hipError_t launch_vl_sweep(const GridView& tgt, const VListView& vl, const float4* src, size_t p0, size_t p1,
                           Xf34 T, double thr, int seeded, uint32_t* nn_pos, uint32_t* flags, int cus,
                           hipStream_t s, const FusedCompact* fc = nullptr);
// lazy source covariances (r04): shard positions k with flags[k] && !cov_ok[k] -> list (absolute
// positions p0 + k, *count of them), cov_ok[k] = 1
hipError_t launch_cov_need(const uint32_t* flags, uint8_t* cov_ok, size_t p0, size_t n, uint32_t* list,
                           unsigned int* count, hipStream_t s);
// diagnostics (mgicp_debug_option "vlist_stats"): per built cell list lengths histogram etc. into out[64]
hipError_t launch_vl_stats(const VListView& vl, size_t ncells, unsigned long long* out /*device, 64*/, hipStream_t s);
size_t     pair_count(size_t n);
hipError_t launch_pairs(const float4* pts, size_t n, float4* out, hipStream_t s);
// Morton keys (30 bit, bbox lo, 1024 / extent = inv) of points [p0, p0 + n) and values 0..n-1
hipError_t launch_morton_keys(const float4* pts, size_t p0, size_t n, const float lo[3], float inv,
                              uint32_t* keys, uint32_t* vals, hipStream_t s);
// accepted correspondences -> their chunk's run of the streams (fixed slots: chunk c at c *
// kChunkPts, ccnt[c] of them, pads to a multiple of 4 zeroed), computing the Mahalanobis matrices
// on the way
// defer (nullable): only the chunks a fused listed sweep deferred (list + device count)
hipError_t launch_compact(const float4* src, const float4* tpts, const Cov3& cov_s,
                          const Cov3& cov_t, Rot33d R, const uint32_t* nn_pos,
                          const uint32_t* flags, size_t p0, size_t p1, uint32_t* ccnt, CorrSoA out, hipStream_t s,
                          const uint32_t* defer = nullptr, const unsigned int* defer_count = nullptr, int cus = 0);
// objective pass over the shard's chunks (ns source positions): chunk partials (partial,
// chunk_count(ns) x kRedVals), super partials (spart), and with `out` the total (in-launch).
// tickets: one per super + one, zero between passes.  done_flag (nullable, mapped host memory):
// the finishing wave stores `seq` there with a system-scope release after `out`, so the host can
// poll instead of synchronising the stream
// host_rows (nullable): super partials as stamped host rows (stamp rstamp, this pass's parity buffer
// at the rank's first super; tickets counted modulo the supers' sizes) instead of spart / out
hipError_t launch_fdf_soa(const CorrSoA& c, const uint32_t* ccnt, size_t ns, Xf34 A,
                          double* partial, double* spart, int nb, unsigned int* tickets, double* out, int reverse,
                          unsigned long long* done_flag, unsigned long long seq, hipStream_t s,
                          unsigned long long* host_rows = nullptr, unsigned int rstamp = 0);
// the same pass pre-launched before its state is known: block 0 waits for cmd->seq == seq (or for
// `timeout_ticks` of wall_clock64) and forwards the command to `mail` (device memory) for the other
// blocks; then every block runs with its A / reverse, or exits on a cancel
hipError_t launch_fdf_soa_gated(const CorrSoA& c, const uint32_t* ccnt, size_t ns,
                                double* partial, double* spart, int nb, unsigned int* tickets, double* out,
                                unsigned long long* done_flag, unsigned long long seq, const PassCmd* cmd,
                                PassCmd* mail, unsigned long long timeout_ticks,
                                unsigned long long* gtrace /*nullable: diagnostics*/,
                                int host_pollers /*blocks [0, host_pollers) poll the host copy*/, hipStream_t s);
int        fdf_grid_blocks(size_t ns, int max_blocks = 2048);
// the resident pass server (one launch per BFGS run, see mgicp_kernels.hip): passes seq0, seq0 + 1,
// ... each run on the command with that stamp, until a cancel (or a later command); bench_passes > 0
// (timing): that many passes of A back to back without commands.  fdf_server_blocks: its grid for a
// shard of ns positions on `cus` CUs (0: not servable, use the launched passes)
int        fdf_server_blocks(size_t ns, int cus, int waves /*4 per CU*/);
// r05, N > 1 over xGMI: the other ranks' exchange buffers (IPC-mapped device memory), at this rank's
// first super; a super's reducer stores its row into its own buffer (host_rows) and into every one of
// these, so each rank's buffer receives every rank's rows
constexpr int kMaxPeers = 8;
struct PeerRows {
  unsigned long long* p[kMaxPeers];
  int n;
};
hipError_t launch_fdf_server(const CorrSoA& c, const uint32_t* ccnt, size_t ns, double* partial,
                             double* spart, unsigned int* tickets, double* out, unsigned long long* done_flag,
                             unsigned long long seq0, const PassCmd* cmd, PassCmd* mail,
                             unsigned long long timeout_ticks, unsigned long long* ptimes /*nullable*/,
                             int bench_passes, Xf34 A,
                             unsigned long long* host_rows /*nullable: super rows to the host, parity 0*/,
                             size_t rows_stride /*words from the parity-0 to the parity-1 row buffer*/, int nb,
                             int waves, int pollers /*blocks reading cmd themselves (1 or nb)*/,
                             int stall_pass /*tests: -1, or the pass the last block withholds*/,
                             unsigned long long* tpart /*nullable: stamped chunk partials, 32 words per chunk (r03)*/,
                             hipStream_t s, const PeerRows* peers = nullptr);
// r05 xGMI totaler (one wave, persistent for a BFGS run): for passes stamp0, stamp0 + 1, ... waits until
// all nsup rows of the pass in this rank's exchange buffer (rows0, parity buffers `stride` words apart)
// carry the pass's stamp, takes the fixed-order total (shm::fixed_total's tree) and stores it as one
// stamped 32-word row at `out` (mapped host memory); exits when *gen_word != gen or after
// `timeout_ticks` without a complete pass
hipError_t launch_xgmi_total(const unsigned long long* rows0, size_t stride, long long nsup, unsigned int stamp0,
                             unsigned long long* out, const unsigned int* gen_word, unsigned int gen,
                             unsigned long long timeout_ticks, hipStream_t s);

// super partials of nch chunk partials of nv (kRedVals or kMomVals) values
hipError_t launch_super_reduce(const double* chunk, int nch, int nv, double* sup, hipStream_t s);
// totals of nsup supers held as nranks rows of maxsup (row r: rank r's supers, from super_first(r))
// tests: wave_sum x 16 vs wave_sum16 on in[w][lane][16] (mgicp_debug_wave_reduce)
hipError_t launch_wave_reduce_check(const double* in, int nwaves, double* out_tree, double* out_rs, hipStream_t s);
hipError_t launch_finish_supers(const double* sup, long long nsup, long long maxsup, int nranks, int nv,
                                double* out, hipStream_t s);
// Gauss-Newton moments of the accepted correspondences of [p0, p1) at T0 (R = rot(T0 * guess),
// ctr = expansion centre): chunk partials of kMomVals doubles (grid: chunk_grid_blocks)
int        chunk_grid_blocks(size_t ns);
hipError_t launch_gn_moments(const float4* src, const float4* tpts, const Cov3& cov_s,
                             const Cov3& cov_t, Rot33d R, Xf34 T0, const double ctr[3],
                             const uint32_t* nn_pos, const uint32_t* flags, size_t p0, size_t p1,
                             double* partial, int nb, hipStream_t s);
// n (<= 64) doubles -> mapped host memory, then seq -> the host-polled completion word
hipError_t launch_publish(const double* in, int n, double* host_out, unsigned long long* flag,
                          unsigned long long seq, hipStream_t s);
// fitness chunk partials ([0] sum d2, [13] count) of [p0, p1) (grid: chunk_grid_blocks)
hipError_t launch_fitness(const GridView& tgt, const float4* src, size_t p0, size_t p1,
                          Xf34 T, double max_range, double* partial, int nb, hipStream_t s);
hipError_t launch_reduce_finish(const double* partial, int nb, double* out, hipStream_t s);
hipError_t launch_resolution(const GridView& g, size_t n, double* partial, int nb, hipStream_t s);
hipError_t launch_radius_keep(const GridView& g, size_t n, float r2, int need, unsigned char* keep,
                              hipStream_t s);

// ---- FOD-side callers ----
// finite points of `in` -> out (order kept, w = original index kept); flags/pos: n + 1 each,
// scratch: scan_scratch_bytes(n + 1); the count is pos[n]
hipError_t launch_finite_compact(const float4* in, size_t n, uint32_t* flags, uint32_t* pos,
                                 void* scratch, size_t scratch_bytes, float4* out, hipStream_t s);
// SegmentDifferences: keep[i] = finite(T in_i) && 1-NN float d2 > thr; *count += kept
hipError_t launch_segdiff(const GridView& g, const float4* in, size_t n, Xf34 T, int has_T, double thr,
                          unsigned char* keep, unsigned int* count, hipStream_t s);
// VoxelGrid: leaf keys (non-finite -> 0xffffffff), run heads of the sorted keys (n + 1 flags),
// per-leaf centroids at the scanned head positions, min_points_per_voxel compaction
hipError_t launch_voxel_keys(const float4* pts, size_t n, const float inv[3], const int min_b[3],
                             int mul1, int mul2, uint32_t* keys, hipStream_t s);
hipError_t launch_voxel_heads(const uint32_t* keys_sorted, size_t n, uint32_t* flags, hipStream_t s);
hipError_t launch_voxel_centroids(const uint32_t* keys_sorted, const uint32_t* perm, const uint32_t* flags,
                                  const uint32_t* pos, size_t n, const float4* pts, const uint32_t* rgba,
                                  float4* out, uint32_t* out_rgba, hipStream_t s);
hipError_t launch_voxel_minpts(const float4* vox, const uint32_t* vox_rgba, size_t nv, uint32_t need,
                               uint32_t* flags, uint32_t* pos, void* scratch, size_t scratch_bytes,
                               float4* out, uint32_t* out_rgba, hipStream_t s);

#if defined(MGICP_CORR_PHASES) && MGICP_CORR_PHASES
hipError_t corr_phase_take(unsigned long long out[24]);  // diagnostic builds: read and reset
#endif
#if defined(MGICP_CORR_STATS) && MGICP_CORR_STATS
hipError_t corr_stats_take(unsigned long long out[8]);  // diagnostic builds: read and reset
#endif

// radix sort / scan scratch (hipcub)
size_t sort_scratch_bytes(size_t n, int bits);
hipError_t launch_sort_pairs(void* scratch, size_t scratch_bytes, const uint32_t* keys_in,
                             uint32_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                             size_t n, int bits, hipStream_t s);
size_t scan_scratch_bytes(size_t n);
hipError_t launch_exclusive_scan(void* scratch, size_t scratch_bytes, const uint32_t* in,
                                 uint32_t* out, size_t n, hipStream_t s);
hipError_t launch_iota(uint32_t* v, size_t n, hipStream_t s);
// r05 target cache: *diff = 1 when a[0..n) and b[0..n) differ in any bit (else 0)
hipError_t launch_equal(const float4* a, const float4* b, size_t n, unsigned int* diff, hipStream_t s);
// resolve all kernels once (moves the code-object loading cost into mgicp_create)
// and exercise both copy directions once, small and large (pinned: pinned host scratch)
hipError_t preload_kernels(void* pinned, size_t pinned_bytes, hipStream_t s);
// per-cell point boxes of a built grid (GridView::boxes), 2 * nc float4
hipError_t launch_cell_boxes(const float4* pts, const uint32_t* cell_start, size_t nc, float4* boxes,
                             hipStream_t s);
// empty-space distance map of a grid (3 separable capped min-max passes); scratch: nc bytes
hipError_t launch_empty_map(const uint32_t* cell_start, int nx, int ny, int nz, uint8_t* out,
                            uint8_t* scratch, hipStream_t s,
                            uint32_t* seed = nullptr /*nullable: nc entries*/, uint32_t* seed_scratch = nullptr,
                            const GridView* g = nullptr /*with seed: each cell's point nearest its centre*/);

}  // namespace mgicp
