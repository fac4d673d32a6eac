// mgicp_kernels.hip -- hand-written CDNA4 (gfx950, wave64) kernels of the GICP engine.
//
// Kernel families (DESIGN.md "Kernels"):
//   knn_cov      exact k-NN (k = 20) over the Morton-free row-sorted uniform grid + PCL's
//                raw-moment covariance + fp64 Jacobi SVD regularisation
//                (PCL GICP::computeCovariances, registration/impl/gicp.hpp)
//   correspond   T * p, radius-bounded exact 1-NN, Mahalanobis (R Cs R' + Ct)^-1
//                (the correspondence loop of GICP::computeTransformation)
//   fdf          one objective pass of OptimizationFunctorWithIndices::fdf:
//                f, grad_t and Rsum in fp64, 64-lane __shfl_down + LDS block reduction,
//                deterministic fixed-order finish
//   fitness      Registration::getFitnessScore 1-NN mean d^2
//
// Numerics: the file is compiled with -ffp-contract=off (and the pragma below) so every fp32
// expression rounds exactly like PCL's non-FMA SSE2 Eigen code and like oracle/gicp_ref.c.
#pragma clang fp contract(off)

#define MGICP_NN_UNROLL 4  // candidate gathers in flight per lane in the 1-NN scans
#define MGICP_CORR_WAVES 8  // resident waves per SIMD requested for the 1-NN kernel (64 VGPRs; A/B profiles/r01/ab_w8)
#define MGICP_COV_WAVES 1  // resident waves per SIMD requested for the k-NN covariance kernel
#ifndef MGICP_KNN_DIV
#define MGICP_KNN_DIV 0  // 1 (with MGICP_CORR_PHASES): k-NN candidate tests per lane vs per wave (diagnostic)
#endif
#ifndef MGICP_CORR_STATS
#define MGICP_CORR_STATS 0  // 1: count 1-NN work per sweep (diagnostic builds only)
#endif
#define MGICP_SRV_STAGGER 2  // resident pass server: 2 = wave wid computes its resident chunks after wid/4 of its streamed ones, 1 = odd waves last, 0 = all first
#ifndef MGICP_VL_DIAG
#define MGICP_VL_DIAG 0  // 1 (with MGICP_CORR_PHASES): per-stage counters and shader clocks of vl_build_kernel
#endif
#ifndef MGICP_CORR_PHASES
#define MGICP_CORR_PHASES 0  // 1: per-phase shader-clock totals of the wave 1-NN sweep (diagnostic builds only)
#endif
constexpr bool kSeedBox = true;  // seeded 1-NN queries search the cube of their seed's ball (box_search)
constexpr int kRegListBatch = 8;  // register-list k-NN rows in guarded batches of this many points

#include "mgicp_internal.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace mgicp {

// ------------------------------------------------------------------------------------
// common device helpers
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float dist2(float qx, float qy, float qz, const float4& p) {
  // FLANN L2_Simple: ((0 + dx^2) + dy^2) + dz^2 in float, dx = query - point
  const float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  float r = dx * dx;
  r = r + dy * dy;
  r = r + dz * dz;
  return r;
}

// (d2, original index) packed so that one u64 compare is the lexicographic order
__device__ __forceinline__ unsigned long long mkkey(float d2, float w) {
  return (static_cast<unsigned long long>(__float_as_uint(d2)) << 32) |
         static_cast<unsigned long long>(__float_as_uint(w));
}

// Eigen Matrix4f * Vector4f (w = 1): ((c0 x + c1 y) + c2 z) + c3
__device__ __forceinline__ void xform(const Xf34& T, float x, float y, float z, float& ox,
                                      float& oy, float& oz) {
  float a = T.m[0] * x;
  a = a + T.m[1] * y;
  a = a + T.m[2] * z;
  ox = a + T.m[3];
  float b = T.m[4] * x;
  b = b + T.m[5] * y;
  b = b + T.m[6] * z;
  oy = b + T.m[7];
  float c = T.m[8] * x;
  c = c + T.m[9] * y;
  c = c + T.m[10] * z;
  oz = c + T.m[11];
}

__device__ __forceinline__ int qcell(float v, float o, float inv_h) {
  float f = floorf((v - o) * inv_h);
  f = fminf(fmaxf(f, -1048576.f), 1048576.f);
  return static_cast<int>(f);
}

__device__ __forceinline__ int bcell(float v, float o, float inv_h, int n) {
  int c = qcell(v, o, inv_h);
  return c < 0 ? 0 : (c > n - 1 ? n - 1 : c);
}

// distance from q to the nearest face of the cell box [c-r, c+r] beyond which grid cells
// remain unvisited along this axis (INF when none remain)
__device__ __forceinline__ float axis_bound(float q, float o, float h, int c, int r, int n) {
  const float dlo = (c - r > 0) ? q - (o + static_cast<float>(c - r) * h) : INFINITY;
  const float dhi = (c + r < n - 1) ? (o + static_cast<float>(c + r + 1) * h) - q : INFINITY;
  return fminf(dlo, dhi);
}

// lower bound of the distance from q to cell c's slab [o + c h, o + (c+1) h) along one axis
__device__ __forceinline__ float cell_gap(float q, float o, float h, int c, float slop) {
  const float lo = o + static_cast<float>(c) * h;
  const float hi = o + static_cast<float>(c + 1) * h;
  const float d = fmaxf(lo - q, q - hi);
  return fmaxf(d - slop, 0.f);
}

__device__ __forceinline__ int dist_out(int c, int n) {
  return c < 0 ? -c : (c > n - 1 ? c - (n - 1) : 0);
}

// +1 when q lies in the upper half of its cell along an axis (the +1 neighbour is nearer), else -1
__device__ __forceinline__ int near_side(float q, float o, float h, int c) {
  return (q - (o + static_cast<float>(c) * h)) * 2.f >= h ? 1 : -1;
}

// Visit grid rings (Chebyshev shells of cells) around q in increasing order until the
// visitor proves that no unvisited point can enter its result.  A ring's rows of cells
// are contiguous ranges of the sorted point array.
// r_from > 0: rings below r_from were visited already (the staged block of knn_blk_kernel)
template <class V>
__device__ __forceinline__ void ring_search(const GridView& g, float qx, float qy, float qz,
                                            V& vis, int r_from = 0) {
  const int cx = qcell(qx, g.ox, g.inv_h), cy = qcell(qy, g.oy, g.inv_h),
            cz = qcell(qz, g.oz, g.inv_h);
  int rmin = max(max(dist_out(cx, g.nx), dist_out(cy, g.ny)), dist_out(cz, g.nz));
  if (rmin == 0 && g.empty_dist) {
    // rings nearer than the closest non-empty cell hold no point: start there (exact)
    rmin = g.empty_dist[static_cast<size_t>(cx) +
                        static_cast<size_t>(g.nx) * (static_cast<size_t>(cy) + static_cast<size_t>(g.ny) * cz)];
  }
  for (int r = max(rmin, r_from); r < (1 << 22); ++r) {
    if constexpr (V::kRingCap) {
      if (r > vis.ring_cap) {
        vis.gave_up = true;
        return;
      }
    }
    if (r > 0) {
      const float L = fminf(fminf(axis_bound(qx, g.ox, g.h, cx, r - 1, g.nx),
                                  axis_bound(qy, g.oy, g.h, cy, r - 1, g.ny)),
                            axis_bound(qz, g.oz, g.h, cz, r - 1, g.nz));
      if (L == INFINITY) return;  // every cell visited
      const float Ls = L * 0.99999f - g.slop;
      if (vis.done(Ls)) return;
    }
    const int x0 = cx - r, x1 = cx + r, y0 = cy - r, y1 = cy + r, z0 = cz - r, z1 = cz + r;
    const int xlo = max(x0, 0), xhi = min(x1, g.nx - 1);
    const int ylo = max(y0, 0), yhi = min(y1, g.ny - 1);
    const int zlo = max(z0, 0), zhi = min(z1, g.nz - 1);
    // V::kNearFirst: rows nearest to q first (the visitor's bound shrinks sooner, so more rows
    // are pruned; measured faster for the k-NN covariances, slower for the 1-NN sweeps), else
    // plain z / y order.  The order of visits does not change the result.
    const int zc = V::kNearFirst ? min(max(cz, zlo), zhi) : zlo;
    const int yc = V::kNearFirst ? min(max(cy, ylo), yhi) : ylo;
    const int zspan = V::kNearFirst ? 2 * max(zc - zlo, zhi - zc) : zhi - zlo;
    const int yspan = V::kNearFirst ? 2 * max(yc - ylo, yhi - yc) : yhi - ylo;
    const int zdn = near_side(qz, g.oz, g.h, cz), ydn = near_side(qy, g.oy, g.h, cy);
    for (int mz = 0; mz <= zspan; ++mz) {
      const int z = V::kNearFirst ? zc + ((mz & 1) ? zdn : -zdn) * ((mz + 1) >> 1) : zlo + mz;
      if (V::kNearFirst && (z < zlo || z > zhi)) continue;
      const bool zf = (z == z0) || (z == z1);
      const float gz = cell_gap(qz, g.oz, g.h, z, g.slop);
      for (int my = 0; my <= yspan; ++my) {
        const int y = V::kNearFirst ? yc + ((my & 1) ? ydn : -ydn) * ((my + 1) >> 1) : ylo + my;
        if (V::kNearFirst && (y < ylo || y > yhi)) continue;
        // ball-cell pruning: skip rows / cells whose box lies beyond the visitor's current
        // worst distance (margin 1e-5 relative + slop keeps the search exact, ties included)
        const float w = vis.prune2() * 1.00001f;
        const float gy = cell_gap(qy, g.oy, g.h, y, g.slop);
        const float gyz = gy * gy + gz * gz;
        if (gyz > w) continue;
        const uint32_t* row = g.cell_start + (static_cast<size_t>(z) * g.ny + y) * g.nx;
        if (zf || y == y0 || y == y1) {
          const float rx = sqrtf(w - gyz) + g.slop;
          const int xa = max(xlo, qcell(qx - rx, g.ox, g.inv_h));
          const int xb = min(xhi, qcell(qx + rx, g.ox, g.inv_h));
          if (xa <= xb) vis.range(g, row[xa], row[xb + 1]);
        } else {
          if (x0 >= 0) {
            const float gx = cell_gap(qx, g.ox, g.h, x0, g.slop);
            if (gx * gx + gyz <= w) vis.range(g, row[x0], row[x0 + 1]);
          }
          if (x1 < g.nx) {
            const float gx = cell_gap(qx, g.ox, g.h, x1, g.slop);
            if (gx * gx + gyz <= vis.prune2() * 1.00001f) vis.range(g, row[x1], row[x1 + 1]);
          }
        }
      }
    }
  }
}

// r05: true when the grid's empty-space map proves that no point lies within sqrt(thr) of q -- the bound
// ring_search checks first (rings closer than the nearest non-empty cell hold no point; L = the distance
// to the faces of that empty box, shrunk by the same margins), so a query the gate must reject (scan
// clutter centimetres off the part) skips its seeds and the gate-sized ball search of the 1-NN sweeps
__device__ __forceinline__ bool empty_reject(const GridView& g, float qx, float qy, float qz, double thr) {
  if (!g.empty_dist) return false;
  const int cx = qcell(qx, g.ox, g.inv_h), cy = qcell(qy, g.oy, g.inv_h), cz = qcell(qz, g.oz, g.inv_h);
  int r = max(max(dist_out(cx, g.nx), dist_out(cy, g.ny)), dist_out(cz, g.nz));
  if (r == 0)
    r = g.empty_dist[static_cast<size_t>(cx) +
                     static_cast<size_t>(g.nx) * (static_cast<size_t>(cy) + static_cast<size_t>(g.ny) * cz)];
  if (r <= 0) return false;
  const float L = fminf(fminf(axis_bound(qx, g.ox, g.h, cx, r - 1, g.nx), axis_bound(qy, g.oy, g.h, cy, r - 1, g.ny)),
                        axis_bound(qz, g.oz, g.h, cz, r - 1, g.nz));
  if (L == INFINITY) return true;  // every cell lies in the empty box: the grid holds no point at all
  const float Ls = L * 0.99999f - g.slop;
  return Ls > 0.f && static_cast<double>(Ls) * static_cast<double>(Ls) >= thr;
}

// lower bound of the distance from q to a point box [lo, hi] (component-wise, each gap shrunk by
// the rounding slop); an empty cell's sentinel box (lo = +INF, hi = -INF) gives +INF
__device__ __forceinline__ float box_gap2(float qx, float qy, float qz, const float4& lo, const float4& hi,
                                          float slop) {
  const float gx = fmaxf(fmaxf(lo.x - qx, qx - hi.x) - slop, 0.f);
  const float gy = fmaxf(fmaxf(lo.y - qy, qy - hi.y) - slop, 0.f);
  const float gz = fmaxf(fmaxf(lo.z - qz, qz - hi.z) - slop, 0.f);
  return gx * gx + gy * gy + gz * gz;
}

// Cells [xa, xb] of one grid row with their TIGHT point boxes (GridView::boxes): only the span
// from the first to the last cell whose box can still hold a winner is scanned.  A query off a
// surface (the 1-NN sweeps: 2-35 mm above the target) sees a whole slab of surface cells inside
// its ball when cells are bounded by their grid boxes; by their point boxes only the cells next
// to the foot of the query survive.  Exact: a skipped cell's every point lies beyond the bound.
template <class V>
__device__ __forceinline__ void visit_row_boxed(const GridView& g, size_t row, int xa, int xb, float w,
                                                V& vis) {
  uint32_t s = 0xffffffffu, e = 0u;
  for (int x = xa; x <= xb; ++x) {
    const float4 lo = g.boxes[2 * (row + x)], hi = g.boxes[2 * (row + x) + 1];
    if (box_gap2(vis.qx, vis.qy, vis.qz, lo, hi, g.slop) <= w) {
      s = min(s, __float_as_uint(lo.w));
      e = max(e, __float_as_uint(hi.w));
    }
  }
  if (s < e) vis.range(g, s, e);
}

// ring_search with per-cell point boxes (targets of the 1-NN sweeps): identical ring order,
// termination and row pruning; inside a row the cell boxes decide which points are scanned
template <class V>
__device__ __forceinline__ void ring_search_boxed(const GridView& g, float qx, float qy, float qz,
                                                  V& vis) {
  const int cx = qcell(qx, g.ox, g.inv_h), cy = qcell(qy, g.oy, g.inv_h),
            cz = qcell(qz, g.oz, g.inv_h);
  int rmin = max(max(dist_out(cx, g.nx), dist_out(cy, g.ny)), dist_out(cz, g.nz));
  if (rmin == 0 && g.empty_dist)
    rmin = g.empty_dist[static_cast<size_t>(cx) +
                        static_cast<size_t>(g.nx) * (static_cast<size_t>(cy) + static_cast<size_t>(g.ny) * cz)];
  for (int r = rmin; r < (1 << 22); ++r) {
    if (r > 0) {
      const float L = fminf(fminf(axis_bound(qx, g.ox, g.h, cx, r - 1, g.nx),
                                  axis_bound(qy, g.oy, g.h, cy, r - 1, g.ny)),
                            axis_bound(qz, g.oz, g.h, cz, r - 1, g.nz));
      if (L == INFINITY) return;
      const float Ls = L * 0.99999f - g.slop;
      if (vis.done(Ls)) return;
    }
    const int x0 = cx - r, x1 = cx + r, y0 = cy - r, y1 = cy + r, z0 = cz - r, z1 = cz + r;
    const int xlo = max(x0, 0), xhi = min(x1, g.nx - 1);
    const int ylo = max(y0, 0), yhi = min(y1, g.ny - 1);
    const int zlo = max(z0, 0), zhi = min(z1, g.nz - 1);
    for (int z = zlo; z <= zhi; ++z) {
      const bool zf = (z == z0) || (z == z1);
      const float gz = cell_gap(qz, g.oz, g.h, z, g.slop);
      for (int y = ylo; y <= yhi; ++y) {
        const float w = vis.prune2() * 1.00001f;
        const float gy = cell_gap(qy, g.oy, g.h, y, g.slop);
        const float gyz = gy * gy + gz * gz;
        if (gyz > w) continue;
        const size_t row = (static_cast<size_t>(z) * g.ny + y) * g.nx;
        if (zf || y == y0 || y == y1) {
          const float rx = sqrtf(w - gyz) + g.slop;
          const int xa = max(xlo, qcell(qx - rx, g.ox, g.inv_h));
          const int xb = min(xhi, qcell(qx + rx, g.ox, g.inv_h));
          if (xa <= xb) visit_row_boxed(g, row, xa, xb, w, vis);
        } else {
          if (x0 >= 0) visit_row_boxed(g, row, x0, x0, w, vis);
          if (x1 < g.nx) visit_row_boxed(g, row, x1, x1, vis.prune2() * 1.00001f, vis);
        }
      }
    }
  }
}

// exact k-NN visitor: register-resident sorted list of (d2, index) keys.  A runtime k < K is
// served by the K-slot list with its first K - k slots pre-filled with the sentinel key 0: every
// real key is >= 0 and an insert never moves in front of an equal key, so the sentinels stay in
// front and slots [K - k, K) hold the k nearest in (d2, index) order.
template <int K>
struct KnnVisitor {
  static constexpr bool kNearFirst = true;
  static constexpr bool kRingCap = false;
  float qx, qy, qz;
  unsigned long long key[K];
  uint32_t pos[K];

  __device__ __forceinline__ void init(float x, float y, float z, int nsent = 0) {
    qx = x; qy = y; qz = z;
#pragma unroll
    for (int k = 0; k < K; ++k) { key[k] = k < nsent ? 0ull : ~0ull; pos[k] = 0u; }
  }
  __device__ __forceinline__ bool done(float Ls) const {
    if (key[K - 1] == ~0ull || !(Ls > 0.f)) return false;
    return __uint_as_float(static_cast<uint32_t>(key[K - 1] >> 32)) < Ls * Ls;
  }
  // squared radius beyond which no point can enter the result
  __device__ __forceinline__ float prune2() const {
    return key[K - 1] == ~0ull ? INFINITY : __uint_as_float(static_cast<uint32_t>(key[K - 1] >> 32));
  }
  __device__ __forceinline__ void insert(unsigned long long c, uint32_t cp) {
#pragma unroll
    for (int k = K - 1; k > 0; --k) {
      const bool sh = c < key[k - 1];
      const bool here = !sh && c < key[k];
      const unsigned long long nk = sh ? key[k - 1] : (here ? c : key[k]);
      const uint32_t np = sh ? pos[k - 1] : (here ? cp : pos[k]);
      key[k] = nk;
      pos[k] = np;
    }
    if (c < key[0]) { key[0] = c; pos[0] = cp; }
  }
  __device__ __forceinline__ void test(const float4& p, uint32_t j) {
    const unsigned long long c = mkkey(dist2(qx, qy, qz, p), p.w);
    if (c < key[K - 1]) insert(c, j);
  }
  __device__ __forceinline__ void range(const GridView& g, uint32_t a, uint32_t b) {
    uint32_t j = a;
    // guarded batches (r03): every load of a batch in flight at once, the row's tail included
    for (; j < b; j += kRegListBatch) {
      float4 pb[kRegListBatch];
#pragma unroll
      for (int u = 0; u < kRegListBatch; ++u) pb[u] = g.pts[min(j + u, b - 1)];
#pragma unroll
      for (int u = 0; u < kRegListBatch; ++u)
        if (j + u < b) test(pb[u], j + u);
    }
  }
};

#if MGICP_CORR_PHASES
// [0] seeds [1] union box + row table [2] union scan [3] winner [4] per-lane finish [5] stores,
// shader-clock cycles summed over waves; [6] waves with a per-lane finish, [7] waves
__device__ unsigned long long g_corr_phase[24];  // [8..12] waves by straggler count 0, 1-4, 5-16, 17-63, 64; [13] stragglers
#define MGICP_PH(k)                                                                         \
  do {                                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                             \
    if (lane == 0) atomicAdd(&g_corr_phase[k], t_ - ph_t);                                  \
    ph_t = t_;                                                                              \
  } while (0)
#else
#define MGICP_PH(k) do {} while (0)
#endif
#if MGICP_CORR_STATS
// [0] queries [1] accepted [2] rejected [3] candidates tested (accepted) [4] (rejected)
// [5] cell ranges scanned (accepted) [6] (rejected)
__device__ unsigned long long g_corr_stats[8];
#endif

// exact 1-NN visitor, optionally bounded by an acceptance threshold thr on d2
struct NnVisitor {
  static constexpr bool kNearFirst = false;
  static constexpr bool kRingCap = false;
  float qx, qy, qz;
  double thr;
  float thr_f;  // float upper bound of thr (pruning radius cap)
  unsigned long long best;
  uint32_t pos;
#if MGICP_CORR_STATS
  uint32_t ntest = 0, nrange = 0, nring = 0;
#endif

  __device__ __forceinline__ void init(float x, float y, float z, double t) {
    qx = x; qy = y; qz = z; thr = t; best = ~0ull; pos = 0u;
    thr_f = (t >= 3.0e38) ? INFINITY : __double2float_ru(t);
  }
  __device__ __forceinline__ float prune2() const {
    const float b = best == ~0ull ? INFINITY : __uint_as_float(static_cast<uint32_t>(best >> 32));
    return fminf(b, thr_f);
  }
  __device__ __forceinline__ bool done(float Ls) const {
    if (!(Ls > 0.f)) return false;
    if (static_cast<double>(Ls) * static_cast<double>(Ls) >= thr) return true;
    if (best == ~0ull) return false;
    return __uint_as_float(static_cast<uint32_t>(best >> 32)) < Ls * Ls;
  }
  __device__ __forceinline__ void test(const float4& p, uint32_t j) {
    const unsigned long long c = mkkey(dist2(qx, qy, qz, p), p.w);
    if (c < best) { best = c; pos = j; }
  }
  __device__ __forceinline__ void range(const GridView& g, uint32_t a, uint32_t b) {
    uint32_t j = a;
#if MGICP_CORR_STATS
    ntest += b - a;
    nrange += 1;
#endif
    // a moving pointer: the four loads of a step share one 64-bit address (immediate offsets);
    // indexing g.pts[j + u] with a 32-bit j recomputed a 64-bit address per candidate (the
    // sweep is VALU-bound: SQ_INSTS_VALU x 4 cycles = the kernel time)
    const float4* q = g.pts + a;
    const uint32_t n4 = (b - a) >> 2;
    for (uint32_t i = 0; i < n4; ++i, q += 4, j += 4) {
      const float4 p0 = q[0], p1 = q[1], p2 = q[2], p3 = q[3];
      test(p0, j);
      test(p1, j + 1);
      test(p2, j + 2);
      test(p3, j + 3);
    }
    for (; j < b; ++j, ++q) test(*q, j);
  }
};

// Exact search of the cube [q - R, q + R] of cells, R = the visitor's current bound (a real seed
// candidate, so the nearest point lies inside): rows nearest to q first, each row's x-range and
// each row itself pruned by the shrinking bound exactly as in ring_search.  For a seeded query
// it visits the rows of the seed's ball once, without ring_search's per-ring face bounds and the
// rows of whole Chebyshev shells (sweeps >= 2 of the correspondence loop).
template <class V>
__device__ __forceinline__ void box_search(const GridView& g, float qx, float qy, float qz, V& vis) {
  const float R = sqrtf(vis.prune2() * 1.00001f) + g.slop;
  const int za = max(qcell(qz - R, g.oz, g.inv_h), 0), zb = min(qcell(qz + R, g.oz, g.inv_h), g.nz - 1);
  const int ya = max(qcell(qy - R, g.oy, g.inv_h), 0), yb = min(qcell(qy + R, g.oy, g.inv_h), g.ny - 1);
  const int zc = min(max(qcell(qz, g.oz, g.inv_h), za), zb), yc = min(max(qcell(qy, g.oy, g.inv_h), ya), yb);
  const int zdn = near_side(qz, g.oz, g.h, zc), ydn = near_side(qy, g.oy, g.h, yc);
  const int zspan = 2 * max(zc - za, zb - zc), yspan = 2 * max(yc - ya, yb - yc);
  for (int mz = 0; mz <= zspan; ++mz) {
    const int z = zc + ((mz & 1) ? zdn : -zdn) * ((mz + 1) >> 1);
    if (z < za || z > zb) continue;
    const float gz = cell_gap(qz, g.oz, g.h, z, g.slop);
    const float gz2 = gz * gz;
    if (gz2 > vis.prune2() * 1.00001f) continue;
    const uint32_t* zrow = g.cell_start + static_cast<size_t>(z) * g.ny * g.nx;
    for (int my = 0; my <= yspan; ++my) {
      const int y = yc + ((my & 1) ? ydn : -ydn) * ((my + 1) >> 1);
      if (y < ya || y > yb) continue;
      const float w = vis.prune2() * 1.00001f;
      const float gy = cell_gap(qy, g.oy, g.h, y, g.slop);
      const float gyz = gy * gy + gz2;
      if (gyz > w) continue;
      const float rx = sqrtf(w - gyz) + g.slop;
      const int xa = max(qcell(qx - rx, g.ox, g.inv_h), 0);
      const int xb = min(qcell(qx + rx, g.ox, g.inv_h), g.nx - 1);
      if (xa > xb) continue;
      const uint32_t* row = zrow + static_cast<uint32_t>(y) * static_cast<uint32_t>(g.nx);
      vis.range(g, row[xa], row[xb + 1]);
    }
  }
}

// LDS written by some lanes of a wave and read by others: LDS executes one wave's instructions in
// order, so only the compiler must not move the reads above the writes
__device__ __forceinline__ void lds_wave_sync() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// box_search over a wave's union box staged in LDS (r03, correspond_wave_kernel's small-ball
// waves): the same rows, x-ranges, pruning and candidate keys as box_search -- so the same result --
// with the cell bounds and the points read from the wave's LDS copy instead of dependent global
// gathers.  Row s = (z - Z0) * nyb + (y - Y0) of the box holds its cells' starts for x = X0 .. X1 + 1
// at lb[s * (nxb + 1) ..] (global sorted positions) and its points from lp[loff[s]] on; the
// lane's ball (radius from its current best) lies inside the box by construction.
template <class V>
__device__ __forceinline__ void box_search_lds(const GridView& g, float qx, float qy, float qz, V& vis, int Z0,
                                               int Y0, int X0, int nyb, int nxb, const uint32_t* lb,
                                               const uint32_t* loff, const float4* lp) {
  const float R = sqrtf(vis.prune2() * 1.00001f) + g.slop;
  const int za = max(qcell(qz - R, g.oz, g.inv_h), 0), zb = min(qcell(qz + R, g.oz, g.inv_h), g.nz - 1);
  const int ya = max(qcell(qy - R, g.oy, g.inv_h), 0), yb = min(qcell(qy + R, g.oy, g.inv_h), g.ny - 1);
  const int zc = min(max(qcell(qz, g.oz, g.inv_h), za), zb), yc = min(max(qcell(qy, g.oy, g.inv_h), ya), yb);
  const int zdn = near_side(qz, g.oz, g.h, zc), ydn = near_side(qy, g.oy, g.h, yc);
  const int zspan = 2 * max(zc - za, zb - zc), yspan = 2 * max(yc - ya, yb - yc);
  const int nb = nxb + 1;
  for (int mz = 0; mz <= zspan; ++mz) {
    const int z = zc + ((mz & 1) ? zdn : -zdn) * ((mz + 1) >> 1);
    if (z < za || z > zb) continue;
    const float gz = cell_gap(qz, g.oz, g.h, z, g.slop);
    const float gz2 = gz * gz;
    if (gz2 > vis.prune2() * 1.00001f) continue;
    for (int my = 0; my <= yspan; ++my) {
      const int y = yc + ((my & 1) ? ydn : -ydn) * ((my + 1) >> 1);
      if (y < ya || y > yb) continue;
      const float w = vis.prune2() * 1.00001f;
      const float gy = cell_gap(qy, g.oy, g.h, y, g.slop);
      const float gyz = gy * gy + gz2;
      if (gyz > w) continue;
      const float rx = sqrtf(w - gyz) + g.slop;
      const int xa = max(qcell(qx - rx, g.ox, g.inv_h), 0);
      const int xb = min(qcell(qx + rx, g.ox, g.inv_h), g.nx - 1);
      if (xa > xb) continue;
      const int sr = (z - Z0) * nyb + (y - Y0);
      const uint32_t* b = lb + sr * nb;
      const uint32_t a0 = b[0], ja = b[xa - X0], jb = b[xb + 1 - X0];
      if (lp) {
        const float4* q = lp + loff[sr] + (ja - a0);
        for (uint32_t j = ja; j < jb; ++j, ++q) vis.test(*q, j);
      } else {
        vis.range(g, ja, jb);  // bounds from LDS, candidates from the global sorted points
      }
    }
  }
}

// radius-count visitor: counts points with float d2 < r2 (FLANN RadiusResultSet: dist < radius),
// stopping as soon as `need` are found
struct RadiusCountVisitor {
  static constexpr bool kNearFirst = false;
  static constexpr bool kRingCap = false;
  float qx, qy, qz;
  float r2;
  int need, count;

  __device__ __forceinline__ bool done(float Ls) const {
    if (count >= need) return true;
    return Ls > 0.f && Ls * Ls >= r2;
  }
  __device__ __forceinline__ float prune2() const { return count >= need ? 0.f : r2; }
  __device__ __forceinline__ void range(const GridView& g, uint32_t a, uint32_t b) {
    for (uint32_t j = a; j < b && count < need; ++j) {
      if (dist2(qx, qy, qz, g.pts[j]) < r2) ++count;
    }
  }
};

// ------------------------------------------------------------------------------------
// grid build
// ------------------------------------------------------------------------------------
__global__ void pack_points_kernel(const unsigned char* raw, size_t n, size_t stride,
                                   float4* out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* p = reinterpret_cast<const float*>(raw + i * stride);
  out[i] = make_float4(p[0], p[1], p[2], __uint_as_float(static_cast<uint32_t>(i)));
}

__global__ __launch_bounds__(256) void bbox_kernel(const float4* pts, size_t n, float* partial) {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  float bad = 0.f;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const float4 p = pts[i];
    if (!isfinite(p.x) || !isfinite(p.y) || !isfinite(p.z)) { bad += 1.f; continue; }
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  __shared__ float sm[7][256];
  for (int d = 0; d < 3; ++d) { sm[d][threadIdx.x] = mn[d]; sm[3 + d][threadIdx.x] = mx[d]; }
  sm[6][threadIdx.x] = bad;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      for (int d = 0; d < 3; ++d) {
        sm[d][threadIdx.x] = fminf(sm[d][threadIdx.x], sm[d][threadIdx.x + s]);
        sm[3 + d][threadIdx.x] = fmaxf(sm[3 + d][threadIdx.x], sm[3 + d][threadIdx.x + s]);
      }
      sm[6][threadIdx.x] += sm[6][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x < 7) partial[blockIdx.x * 8 + threadIdx.x] = sm[threadIdx.x][0];
}

__global__ void cell_hist_kernel(const float4* pts, size_t n, float ox, float oy, float oz,
                                 float inv_h, int nx, int ny, int nz, uint32_t* counts,
                                 uint32_t* keys) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool live = i < n;
  uint32_t lin = 0xffffffffu;
  if (live) {
    const float4 p = pts[i];
    const uint32_t cx = bcell(p.x, ox, inv_h, nx), cy = bcell(p.y, oy, inv_h, ny),
                   cz = bcell(p.z, oz, inv_h, nz);
    lin = cx + static_cast<uint32_t>(nx) * (cy + static_cast<uint32_t>(ny) * cz);
    if (keys) keys[i] = lin;
  }
  if (!counts) return;  // r06: keys only (the grid's counts come from the sorted keys, cell_end_kernel)
  // r03: scan-ordered clouds (a scanner's line order) put runs of consecutive points into one cell;
  // the run's first lane adds the run length, one atomic per run instead of one per point.  The
  // synthetic bench clouds are in random order (no runs): there the kernel stays bound by the
  // memory-side atomics (~260 us per 5M points, profiles/r03/prep)
  const int lane = threadIdx.x & 63;
  const uint32_t prev = __shfl_up(lin, 1, 64);
  const bool head = live && (lane == 0 || prev != lin);
  const unsigned long long hm = __builtin_amdgcn_ballot_w64(head);
  const unsigned long long lm = __builtin_amdgcn_ballot_w64(live);
  if (head) {
    const unsigned long long above = hm & ~((2ull << lane) - 1ull);  // heads after this lane
    const int next = above ? __builtin_ctzll(above) : 64 - __builtin_clzll(lm);  // run end (exclusive)
    atomicAdd(&counts[lin], static_cast<uint32_t>(next - lane));
  }
}

// r06: the grid's sizing sketch.  build_grid aims at ~10 points per non-empty cell; r01-r05 found the cell
// size by trial histograms (an atomic per point into the counts -- scattered atomics, ~250 us per 5M
// points -- then a count of the non-empty cells and a host round trip, twice per cloud on surfaces).
// Here ONE pass estimates the number of non-empty cells at kSketchScales cell sizes at once: per size a
// HyperLogLog sketch of the occupied cells (kSketchR one-byte registers, LDS atomicMax, a fixed 32-bit
// hash of the cell coordinates), block sketches written to `partial` and max-merged by
// sketch_merge_kernel.  The estimate only picks the cell size (every grid is exact); max is
// order-independent, so the size is a function of the cloud alone.
__device__ __forceinline__ unsigned int fmix32(unsigned int h) {  // MurmurHash3's finaliser
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

__device__ __forceinline__ unsigned int sketch_cell(float v, float inv) {
  return static_cast<unsigned int>(static_cast<int>(fminf(fmaxf(floorf(v * inv), -1.0e9f), 1.0e9f)));
}

__global__ __launch_bounds__(256) void cell_sketch_kernel(const float4* __restrict__ pts, size_t n, float ox, float oy,
                                                          float oz, SketchScales sc, uint8_t* __restrict__ partial) {
  constexpr int R = kSketchR, S = kSketchScales;
  __shared__ unsigned int reg[S * R];
  for (int t = threadIdx.x; t < S * R; t += blockDim.x) reg[t] = 0u;
  __syncthreads();
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const float4 p = pts[i];
    const float fx = p.x - ox, fy = p.y - oy, fz = p.z - oz;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const float inv = sc.inv[k];
      const unsigned int key = fmix32(sketch_cell(fx, inv) * 0x9e3779b1u ^ sketch_cell(fy, inv) * 0x85ebca77u ^
                                      sketch_cell(fz, inv) * 0xc2b2ae3du);
      const unsigned int idx = key >> (32 - kSketchLog2R);
      const unsigned int rank = static_cast<unsigned int>(__builtin_clz((key << kSketchLog2R) | (1u << (kSketchLog2R - 1)))) + 1u;
      // most updates change nothing once the registers fill up: a plain read first (same-address reads
      // broadcast) keeps the LDS atomics -- serialised per address, many lanes share a cell at coarse
      // sizes -- to the few that raise a register
      if (rank > reg[k * R + idx]) atomicMax(&reg[k * R + idx], rank);
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < S * R; t += blockDim.x)
    partial[static_cast<size_t>(blockIdx.x) * (S * R) + t] = static_cast<uint8_t>(reg[t]);
}

// max-merge of the block sketches: blockIdx.y takes blocks [y nblocks / ny, (y + 1) nblocks / ny) into
// partial row nblocks + y (ny rows after the block rows), then the ny rows into `out` (ny == 1)
__global__ __launch_bounds__(256) void sketch_merge_kernel(uint8_t* __restrict__ partial, int b0, int nblocks,
                                                           uint8_t* __restrict__ out) {
  constexpr int SR = kSketchScales * kSketchR;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= SR) return;
  const int ny = gridDim.y, y = blockIdx.y;
  const int lo = b0 + y * nblocks / ny, hi = b0 + (y + 1) * nblocks / ny;
  unsigned int m = 0;
#pragma unroll 8
  for (int b = lo; b < hi; ++b) m = max(m, static_cast<unsigned int>(partial[static_cast<size_t>(b) * SR + t]));
  if (out) out[t] = static_cast<uint8_t>(m);
  else partial[static_cast<size_t>(b0 + nblocks + y) * SR + t] = static_cast<uint8_t>(m);
}

// r06: cell_start from the sorted keys: the last point of each non-empty cell stores the cell's end
// (its position + 1) into `ends` (zeroed), and an exclusive max-scan over the nc + 1 entries then gives
// every cell's start (the end of the nearest non-empty cell before it) -- the exclusive prefix sum of the
// per-cell counts, without a histogram of atomics
__global__ void cell_end_kernel(const uint32_t* __restrict__ keys_sorted, size_t n, uint32_t* __restrict__ ends) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = keys_sorted[i];
  if (i + 1 == n || keys_sorted[i + 1] != k) ends[k] = static_cast<uint32_t>(i + 1);
}

__global__ void gather_sorted_kernel(const float4* pts, const uint32_t* perm, size_t n,
                                     float4* out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = pts[perm[i]];
}

__global__ void xform_points_kernel(const float4* in, size_t n, Xf34 T, float4* out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  float x, y, z;
  xform(T, p.x, p.y, p.z, x, y, z);
  out[i] = make_float4(x, y, z, p.w);
}

// empty-space map, pass 0: 0 for non-empty cells, 255 for empty ones; with `seed`, a non-empty
// cell's seed is its first sorted position (an empty cell's is undefined until a pass sets it)
__global__ void empty_init_kernel(const uint32_t* __restrict__ cs, size_t nc, uint8_t* __restrict__ e,
                                  uint32_t* __restrict__ seed, const float4* __restrict__ pts, int nx, int ny,
                                  float ox, float oy, float oz, float h) {
  const size_t c = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const uint32_t a = cs[c], b = cs[c + 1];
  const bool full = b > a;
  e[c] = full ? 0 : 255;
  if (!seed) return;
  uint32_t best = full ? a : 0xffffffffu;
  if (full && pts) {
    // the cell's point nearest to the cell centre: a better seed than an arbitrary one for every
    // query that lands in or near the cell
    const int x = static_cast<int>(c % static_cast<size_t>(nx));
    const int y = static_cast<int>((c / static_cast<size_t>(nx)) % static_cast<size_t>(ny));
    const int z = static_cast<int>(c / (static_cast<size_t>(nx) * ny));
    const float cx = ox + (static_cast<float>(x) + 0.5f) * h, cy = oy + (static_cast<float>(y) + 0.5f) * h,
                cz = oz + (static_cast<float>(z) + 0.5f) * h;
    float bd = INFINITY;
    // r06: 4 loads in flight per round (a wave's few non-empty cells otherwise walk their points one
    // dependent load at a time); the clamped duplicates of a short tail are skipped
    for (uint32_t j0 = a; j0 < b; j0 += 4) {
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) p[u] = pts[min(j0 + u, b - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float d = dist2(cx, cy, cz, p[u]);
        if (j0 + u < b && d < bd) { bd = d; best = j0 + u; }
      }
    }
  }
  seed[c] = best;
}

// one separable pass of the Chebyshev (L-inf) distance transform along an axis of extent n and
// element stride `stride`: out(c) = min_{|d| <= kEmptyCap} max(|d|, in(c + d*stride)), capped at
// kEmptyCap + 1.  With seeds, the seed of the winning cell travels along (first winner in |d|, minus
// side first), so the final seed lies in a Chebyshev-nearest non-empty cell.  r04: all 2 kEmptyCap
// neighbours are loaded up front (out-of-line slots read as empty) and the candidates are then taken
// in the original order from registers.  r06: a thread takes 4 consecutive cells of one line, so the
// 2 kEmptyCap + 4 loaded bytes serve all four (r04: 2 kEmptyCap + 1 byte loads per cell, ~170 us
// per pass at C4's 14-20M target cells); consecutive threads take neighbouring lines (y / z passes)
// or neighbouring groups of a row (x pass), so every load instruction stays coalesced.
constexpr int kEmptyGroup = 4;
__global__ __launch_bounds__(256) void empty_pass_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                         size_t nlines, int n, size_t stride,
                                                         const uint32_t* __restrict__ sin,
                                                         uint32_t* __restrict__ sout) {
  constexpr int cap = kEmptyCap, G = kEmptyGroup, W = 2 * cap + G;
  const size_t ng = static_cast<size_t>((n + G - 1) / G);
  const size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= nlines * ng) return;
  size_t L, g;
  if (stride == 1) { L = t / ng; g = t % ng; }
  else { L = t % nlines; g = t / nlines; }
  // line L's first cell: lines are indexed by the cell's coordinates off this axis
  const size_t base = (L % stride) + (L / stride) * stride * static_cast<size_t>(n);
  const int i0 = static_cast<int>(g) * G;
  int win[W];  // in() of cells i0 - cap .. i0 + G - 1 + cap of the line (255 outside it)
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int i = i0 - cap + w;
    const int ic = min(max(i, 0), n - 1);  // clamped: an in-line address
    const int v = in[base + static_cast<size_t>(ic) * stride];
    win[w] = (i == ic) ? v : 255;
  }
#pragma unroll
  for (int u = 0; u < G; ++u) {
    if (i0 + u >= n) break;
    const size_t c = base + static_cast<size_t>(i0 + u) * stride;
    int best = min(win[cap + u], cap + 1);
    int dbest = 0;  // signed offset of the winner
#pragma unroll
    for (int d = 1; d <= cap; ++d) {
      if (d < best) {
        const int v = max(d, win[cap + u - d]);
        if (v < best) { best = v; dbest = -d; }
        const int w = max(d, win[cap + u + d]);
        if (w < best) { best = w; dbest = d; }
      }
    }
    out[c] = static_cast<uint8_t>(min(best, cap + 1));
    if (sout) {
      const size_t arg = dbest < 0 ? c - static_cast<size_t>(-dbest) * stride : c + static_cast<size_t>(dbest) * stride;
      sout[c] = best <= cap ? sin[arg] : 0xffffffffu;
    }
  }
}

// per-cell point boxes: boxes[2c] = (min x, min y, min z, bits(start)), boxes[2c + 1] =
// (max x, max y, max z, bits(end)); an empty cell gets the sentinel (+INF / -INF) box
__global__ void cell_box_kernel(const float4* __restrict__ pts, const uint32_t* __restrict__ cs, size_t nc,
                                float4* __restrict__ boxes) {
  const size_t c = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  const uint32_t a = cs[c], b = cs[c + 1];
  float lx = INFINITY, ly = INFINITY, lz = INFINITY, hx = -INFINITY, hy = -INFINITY, hz = -INFINITY;
  for (uint32_t j = a; j < b; ++j) {
    const float4 p = pts[j];
    lx = fminf(lx, p.x); ly = fminf(ly, p.y); lz = fminf(lz, p.z);
    hx = fmaxf(hx, p.x); hy = fmaxf(hy, p.y); hz = fmaxf(hz, p.z);
  }
  boxes[2 * c] = make_float4(lx, ly, lz, __uint_as_float(a));
  boxes[2 * c + 1] = make_float4(hx, hy, hz, __uint_as_float(b));
}

__global__ void iota_kernel(uint32_t* v, size_t n) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) v[i] = static_cast<uint32_t>(i);
}

// ------------------------------------------------------------------------------------
// covariance: exact kNN + PCL raw moments + fp64 Jacobi (bit-identical to the oracle)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void jacobi3(double a[3][3], double v[3][3]) {
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) v[r][c] = (r == c) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 50; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int p = (e == 2) ? 1 : 0, q = (e == 0) ? 1 : 2, o = 3 - p - q;
      const double apq = a[p][q];
      const double app = a[p][p], aqq = a[q][q];
      if (fabs(apq) <= 1e-18 * (fabs(app) + fabs(aqq))) {
        a[p][q] = a[q][p] = 0.0;
        continue;
      }
      rotated = true;
      const double theta = (aqq - app) / (2.0 * apq);
      double t;
      if (fabs(theta) > 1e150) t = 0.5 / theta;
      else t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0);
      const double s = t * c;
      a[p][p] = app - t * apq;
      a[q][q] = aqq + t * apq;
      a[p][q] = a[q][p] = 0.0;
      const double aop = a[o][p], aoq = a[o][q];
      a[o][p] = a[p][o] = c * aop - s * aoq;
      a[o][q] = a[q][o] = s * aop + c * aoq;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const double vp = v[r][p], vq = v[r][q];
        v[r][p] = c * vp - s * vq;
        v[r][q] = s * vp + c * vq;
      }
    }
    if (!rotated) break;
  }
}

__device__ __forceinline__ double sel3(int i, double a, double b, double c) {
  return i == 0 ? a : (i == 1 ? b : c);
}

// ---- two-phase k-NN selection (knn_cov2_kernel) ----------------------------------------------
// Phase 1 finds the EXACT k-th smallest float d2 (tau) with a branch-free network over a register
// list of float keys: key[j] = max(key[j-1], min(d2, key[j])) = med3(key[j-1], d2, key[j]) (the
// list is ascending; d2 is finite) inserts d2 in ONE v_med3_f32 per slot (the (d2, index) insert
// with 64-bit keys and positions costs ~8 per slot, and in SIMT every lane pays it whenever ANY
// lane inserts: knn_cov was VALU-bound at 25k instructions per wave).
// Every candidate whose d2 does not exceed the CURRENT k-th is appended to the
// lane's LDS log as its sorted position (the (d2, original index) key is recomputed from the point,
// bit-identically, when the log is read): thresholds only fall, so the log holds every member of the
// final k-NN set (ties at the final k-th included) -- no second search.
#define MGICP_KNN_LOG_BATCH 8  // log entries read per batch (compaction, moments): loads in flight together
constexpr int kLogBatch = MGICP_KNN_LOG_BATCH;
#define MGICP_KNN_RANGE_BATCH 8  // candidates per guarded batch of the logged k-NN rows (0: 4-wide + tail)

template <int K>
struct KthVisitor {
  static constexpr bool kNearFirst = true;
  static constexpr bool kRingCap = true;
  int ring_cap = 1 << 30;  // rings past this one: give up (the point's covariance is left for later)
  bool gave_up = false;
  float qx, qy, qz;
  float key[K];  // ascending; the first nsent slots hold the sentinel -1 (always in front)
  uint32_t* lpos;  // lane-strided LDS log of sorted positions, cap entries
  int cnt, cap;
#if MGICP_KNN_DIV
  unsigned ntest = 0, witer = 0;  // this lane's tests; wave iterations counted by the first active lane
#endif
  __device__ __forceinline__ void init(float x, float y, float z, int nsent) {
    qx = x; qy = y; qz = z;
    cnt = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) key[k] = k < nsent ? -1.f : INFINITY;
  }
  __device__ __forceinline__ bool done(float Ls) const { return Ls > 0.f && key[K - 1] < Ls * Ls; }
  __device__ __forceinline__ float prune2() const { return key[K - 1]; }
  const float4* pts;
  // a full log drops the entries the threshold has since passed (d2 recomputed from the point)
  // (entries in batches of kLogBatch: all loads of a batch in flight at once; writes only reach
  // entries already read)
  __device__ __forceinline__ void compact() {
    int m = 0;
    for (int i0 = 0; i0 < cnt; i0 += kLogBatch) {
      uint32_t j[kLogBatch];
      float4 pt[kLogBatch];
#pragma unroll
      for (int u = 0; u < kLogBatch; ++u) j[u] = lpos[min(i0 + u, cnt - 1) * 64];
#pragma unroll
      for (int u = 0; u < kLogBatch; ++u) pt[u] = pts[j[u]];
#pragma unroll
      for (int u = 0; u < kLogBatch; ++u)
        if (i0 + u < cnt && dist2(qx, qy, qz, pt[u]) <= key[K - 1]) lpos[(m++) * 64] = j[u];
    }
    cnt = m;
  }
  __device__ __forceinline__ void test(float d, float w, uint32_t j) {
#if MGICP_KNN_DIV
    ++ntest;
    if (static_cast<unsigned>(__lane_id()) == static_cast<unsigned>(__builtin_ctzll(__builtin_amdgcn_read_exec()))) ++witer;
#endif
    if (d <= key[K - 1]) {
      if (cnt == cap) compact();
      if (cnt < cap) lpos[cnt * 64] = j;
      ++cnt;
    }
    if (d < key[K - 1]) {  // (a value equal to the k-th leaves the multiset of the k smallest as is)
#pragma unroll
      for (int k = K - 1; k > 0; --k) key[k] = __builtin_amdgcn_fmed3f(key[k - 1], d, key[k]);
      key[0] = fminf(d, key[0]);
    }
  }
  __device__ __forceinline__ void range(const GridView& g, uint32_t a, uint32_t b) {
#if MGICP_KNN_RANGE_BATCH
    // guarded batches: every load of a batch in flight at once, a row's tail included (the
    // clamped duplicate loads hit the same lines; their tests are skipped)
    for (uint32_t j0 = a; j0 < b; j0 += MGICP_KNN_RANGE_BATCH) {
      float4 pb[MGICP_KNN_RANGE_BATCH];
#pragma unroll
      for (int u = 0; u < MGICP_KNN_RANGE_BATCH; ++u) pb[u] = g.pts[min(j0 + u, b - 1)];
#pragma unroll
      for (int u = 0; u < MGICP_KNN_RANGE_BATCH; ++u)
        if (j0 + u < b) test(dist2(qx, qy, qz, pb[u]), pb[u].w, j0 + u);
    }
#else
    const float4* q = g.pts + a;
    uint32_t j = a;
    for (; j + 4 <= b; j += 4, q += 4) {
      const float4 p0 = q[0], p1 = q[1], p2 = q[2], p3 = q[3];
      test(dist2(qx, qy, qz, p0), p0.w, j);
      test(dist2(qx, qy, qz, p1), p1.w, j + 1);
      test(dist2(qx, qy, qz, p2), p2.w, j + 2);
      test(dist2(qx, qy, qz, p3), p3.w, j + 3);
    }
    for (; j < b; ++j, ++q) test(dist2(qx, qy, qz, *q), q->w, j);
#endif
  }
};

// PCL's covariance of the k = K - nsent neighbours at sorted positions pos[nsent..K) (in (d2,
// index) order), regularised and stored at p (shared by both k-NN kernels)
template <int K>
__device__ __forceinline__ void cov_from_sorted(const GridView& g, double eps, const uint32_t (&pos)[K],
                                                int nsent, Cov3 cov, size_t p);

// `perm` (optional): query order over [p0, p1) (Morton order: compact 3-D patch per wave)
// k = K - nsent neighbours (nsent > 0 only on the generic rounded-up instantiations)
// dcount (nullable): the number of queries is *dcount (the logged kernel's hand-off count, read on
// the device so the hand-off can follow it in stream order); the grid strides over them
template <int K>
__global__ __launch_bounds__(256, MGICP_COV_WAVES) void knn_cov_kernel(GridView g, double eps, size_t p0,
                                                      size_t p1, Cov3 cov,
                                                      const uint32_t* __restrict__ perm, int nsent,
                                                      const unsigned int* __restrict__ dcount) {
  const size_t n = dcount ? static_cast<size_t>(*dcount) : p1 - p0;
  for (size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const size_t p = p0 + (perm ? perm[t] : t);
    const float4 q = g.pts[p];
    KnnVisitor<K> vis;
    vis.init(q.x, q.y, q.z, nsent);
    ring_search(g, q.x, q.y, q.z, vis);
    cov_from_sorted<K>(g, eps, vis.pos, nsent, cov, p);
  }
}

// PCL's covariance from the raw moments of the k neighbours (sums in the oracle's order or proven
// order-independent), regularised and stored at p
__device__ __forceinline__ void cov_finish(double m0, double m1, double m2, double (&a)[3][3], double kd,
                                           double eps, Cov3 cov, size_t p) {
  double mean[3] = {m0 / kd, m1 / kd, m2 / kd};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      a[i][j] /= kd;
      a[i][j] -= mean[i] * mean[j];
      a[j][i] = a[i][j];
    }
  double v[3][3];
  jacobi3(a, v);
  const double sv0 = fabs(a[0][0]), sv1 = fabs(a[1][1]), sv2 = fabs(a[2][2]);
  int ord[3] = {0, 1, 2};
  // descending selection sort, no swap on ties (identical to the oracle)
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = i + 1; j < 3; ++j) {
      const double sj = sel3(ord[j], sv0, sv1, sv2), si = sel3(ord[i], sv0, sv1, sv2);
      if (sj > si) { const int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    }
  double C00 = 0.0, C01 = 0.0, C02 = 0.0, C11 = 0.0, C12 = 0.0, C22 = 0.0;
#pragma unroll
  for (int kk = 0; kk < 3; ++kk) {
    const int col = ord[kk];
    const double w = (kk == 2) ? eps : 1.0;
    const double v0 = sel3(col, v[0][0], v[0][1], v[0][2]);
    const double v1 = sel3(col, v[1][0], v[1][1], v[1][2]);
    const double v2 = sel3(col, v[2][0], v[2][1], v[2][2]);
    const double u0 = w * v0, u1 = w * v1, u2 = w * v2;
    C00 += u0 * v0;
    C01 += u0 * v1;
    C02 += u0 * v2;
    C11 += u1 * v1;
    C12 += u1 * v2;
    C22 += u2 * v2;
  }
  cov.a[p] = make_double2(C00, C01);
  cov.b[p] = make_double2(C02, C11);
  cov.c[p] = make_double2(C12, C22);
}

template <int K>
__device__ __forceinline__ void cov_from_sorted(const GridView& g, double eps, const uint32_t (&pos)[K],
                                                int nsent, Cov3 cov, size_t p) {
  double m0 = 0.0, m1 = 0.0, m2 = 0.0;
  double a[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (k < nsent) continue;
    const float4 pt = g.pts[pos[k]];
    m0 += pt.x;
    m1 += pt.y;
    m2 += pt.z;
    a[0][0] += static_cast<double>(pt.x * pt.x);
    a[1][0] += static_cast<double>(pt.y * pt.x);
    a[1][1] += static_cast<double>(pt.y * pt.y);
    a[2][0] += static_cast<double>(pt.z * pt.x);
    a[2][1] += static_cast<double>(pt.z * pt.y);
    a[2][2] += static_cast<double>(pt.z * pt.z);
  }
  cov_finish(m0, m1, m2, a, static_cast<double>(K - nsent), eps, cov, p);
}

// ---- r06: one WAVE per query (the lazy pass and the hand-off) ----------------------------------
// The per-lane ring search (KnnVisitor / KthVisitor) walks a query's rings row by row on one lane; a
// point whose k neighbours lie many rings out -- scan clutter and debris the gate accepts (C4F: 21k of them
// in the first sweep, their 20-NN 2-3 cm away, 6-8 rings of 3.6 mm cells) -- then chains hundreds of
// dependent row loads, and the few waves of the lazy pass ran ~5 ms at C4F for that tail.  Here the 64
// lanes of a wave share ONE query: ring by ring, lane l takes rows l, l + 64, ... of the shell, keeping its
// own K smallest (d2 bits, original index) keys; a row is skipped when it lies beyond min(the lane's own
// K-th, the wave's smallest K-th at the ring start) -- each is an upper bound of the true K-th distance,
// the subset argument, with ring_search's 1e-5 margin and slop.  After ring r - 1 the search stops when
// k keys of the whole wave lie strictly inside L, the distance to the unvisited cells (ring_search's
// bound and margins).  A k-round wave merge (64-bit min, the winning lane pops its front) yields the k
// keys in ascending (d2, index) order; the moments are summed in that order and finished by cov_finish --
// cov_from_sorted's sums of KnnVisitor's set, bit for bit.
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned int lo = __shfl_xor(static_cast<unsigned int>(v), o, 64);
    const unsigned int hi = __shfl_xor(static_cast<unsigned int>(v >> 32), o, 64);
    const unsigned long long w = (static_cast<unsigned long long>(hi) << 32) | lo;
    v = w < v ? w : v;
  }
  return v;
}

template <int K>
struct WaveKnnLane {
  unsigned long long key[K];
  uint32_t pos[K];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int i = 0; i < K; ++i) { key[i] = ~0ull; pos[i] = 0u; }
  }
  __device__ __forceinline__ float kth2() const {
    return key[K - 1] == ~0ull ? INFINITY : __uint_as_float(static_cast<uint32_t>(key[K - 1] >> 32));
  }
  __device__ __forceinline__ void insert(unsigned long long c, uint32_t cp) {
#pragma unroll
    for (int i = K - 1; i > 0; --i) {
      const bool sh = c < key[i - 1];
      const bool here = !sh && c < key[i];
      key[i] = sh ? key[i - 1] : (here ? c : key[i]);
      pos[i] = sh ? pos[i - 1] : (here ? cp : pos[i]);
    }
    if (c < key[0]) { key[0] = c; pos[0] = cp; }
  }
  __device__ __forceinline__ void range(const GridView& g, float qx, float qy, float qz, uint32_t a, uint32_t b) {
    for (uint32_t j0 = a; j0 < b; j0 += 4) {
      float4 pb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) pb[u] = g.pts[min(j0 + u, b - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (j0 + u >= b) continue;
        const unsigned long long c = mkkey(dist2(qx, qy, qz, pb[u]), pb[u].w);
        if (c < key[K - 1]) insert(c, j0 + u);
      }
    }
  }
  // entries with d2 strictly below Ls^2 (the list is ascending)
  __device__ __forceinline__ int below(float Ls2) const {
    int n = 0;
#pragma unroll
    for (int i = 0; i < K; ++i)
      n += (key[i] != ~0ull && __uint_as_float(static_cast<uint32_t>(key[i] >> 32)) < Ls2) ? 1 : 0;
    return n;
  }
};

// queries: list[i] (sorted positions of the cloud) for i < *count (device count) or n; one wave each,
// grid-striding.  k <= K neighbours (K: the instantiation).
template <int K>
__global__ __launch_bounds__(256) void knn_wave_kernel(GridView g, double eps, const uint32_t* __restrict__ list,
                                                       const unsigned int* __restrict__ count, size_t n, int k,
                                                       Cov3 cov) {
  const int lane = threadIdx.x & 63;
  const size_t nq = count ? static_cast<size_t>(*count) : n;
  const size_t nw = static_cast<size_t>(gridDim.x) * (blockDim.x >> 6);
  for (size_t wq = static_cast<size_t>(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); wq < nq; wq += nw) {
    const size_t p = list ? list[wq] : wq;
    const float4 q = g.pts[p];
    const float qx = q.x, qy = q.y, qz = q.z;
    WaveKnnLane<K> L;
    L.init();
    const int cx = qcell(qx, g.ox, g.inv_h), cy = qcell(qy, g.oy, g.inv_h), cz = qcell(qz, g.oz, g.inv_h);
    int rmin = max(max(dist_out(cx, g.nx), dist_out(cy, g.ny)), dist_out(cz, g.nz));
    if (rmin == 0 && g.empty_dist)
      rmin = g.empty_dist[static_cast<size_t>(cx) +
                          static_cast<size_t>(g.nx) * (static_cast<size_t>(cy) + static_cast<size_t>(g.ny) * cz)];
    for (int r = rmin; r < (1 << 22); ++r) {
      if (r > 0) {
        const float Lb = fminf(fminf(axis_bound(qx, g.ox, g.h, cx, r - 1, g.nx), axis_bound(qy, g.oy, g.h, cy, r - 1, g.ny)),
                               axis_bound(qz, g.oz, g.h, cz, r - 1, g.nz));
        if (Lb == INFINITY) break;  // every cell visited
        const float Ls = Lb * 0.99999f - g.slop;
        int nb = Ls > 0.f ? L.below(Ls * Ls) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) nb += __shfl_xor(nb, o, 64);
        if (nb >= k) break;
      }
      // the wave's tightest upper bound of the k-th distance at the ring start
      float wb = L.kth2();
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wb = fminf(wb, __shfl_xor(wb, o, 64));
      const int x0 = cx - r, x1 = cx + r, y0 = cy - r, y1 = cy + r, z0 = cz - r, z1 = cz + r;
      const int xlo = max(x0, 0), xhi = min(x1, g.nx - 1);
      const int ylo = max(y0, 0), yhi = min(y1, g.ny - 1);
      const int zlo = max(z0, 0), zhi = min(z1, g.nz - 1);
      if (xlo > xhi || ylo > yhi || zlo > zhi) continue;
      const int ny_r = yhi - ylo + 1;
      const int nrows = (zhi - zlo + 1) * ny_r;
      // rows in batches of 64 (one per lane): each lane forms its row's candidate ranges (pruned against
      // the wave's bound), then the batch's points are flattened over the wave -- lane l tests points l,
      // l + 64, ... of the concatenated ranges -- so a row crossing a dense surface does not leave one lane
      // to scan it while 63 wait (the hand-off's points: dense clusters, duplicates)
      for (int t0 = 0; t0 < nrows; t0 += 64) {
        uint32_t a1 = 0, b1 = 0, a2 = 0, b2 = 0;
        const int t = t0 + lane;
        float wbb = L.kth2();
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) wbb = fminf(wbb, __shfl_xor(wbb, o, 64));
        const float w = fminf(wbb, wb) * 1.00001f;
        if (t < nrows) {
          const int z = zlo + t / ny_r, y = ylo + t % ny_r;
          const bool zf = (z == z0) || (z == z1);
          const float gz = cell_gap(qz, g.oz, g.h, z, g.slop);
          const float gy = cell_gap(qy, g.oy, g.h, y, g.slop);
          const float gyz = gy * gy + gz * gz;
          if (gyz <= w) {
            const uint32_t* row = g.cell_start + (static_cast<size_t>(z) * g.ny + y) * g.nx;
            if (zf || y == y0 || y == y1) {
              const float rx = sqrtf(w - gyz) + g.slop;
              const int xa = max(xlo, qcell(qx - rx, g.ox, g.inv_h));
              const int xb = min(xhi, qcell(qx + rx, g.ox, g.inv_h));
              if (xa <= xb) { a1 = row[xa]; b1 = row[xb + 1]; }
            } else {
              if (x0 >= 0) {
                const float gx = cell_gap(qx, g.ox, g.h, x0, g.slop);
                if (gx * gx + gyz <= w) { a1 = row[x0]; b1 = row[x0 + 1]; }
              }
              if (x1 < g.nx) {
                const float gx = cell_gap(qx, g.ox, g.h, x1, g.slop);
                if (gx * gx + gyz <= w) { a2 = row[x1]; b2 = row[x1 + 1]; }
              }
            }
          }
        }
        const uint32_t n1 = b1 - a1, cnt = n1 + (b2 - a2);
        uint32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_up(inc, o, 64);
          if (lane >= o) inc += u;
        }
        const uint32_t off = inc - cnt;
        const uint32_t tot = __builtin_amdgcn_readlane(inc, 63);
        for (uint32_t f0 = 0; f0 < tot; f0 += 64) {
          const uint32_t f = f0 + static_cast<uint32_t>(lane);
          // the owner: the last lane whose range starts at or before f (binary search over the offsets)
          int lo = 0;
#pragma unroll
          for (int step = 32; step > 0; step >>= 1) {
            const uint32_t om = __shfl(off, lo + step, 64);
            if (lo + step < 64 && om <= f) lo += step;
          }
          const uint32_t o_off = __shfl(off, lo, 64), o_a1 = __shfl(a1, lo, 64), o_n1 = __shfl(n1, lo, 64);
          const uint32_t o_a2 = __shfl(a2, lo, 64);
          if (f < tot) {
            const uint32_t i = f - o_off;
            const uint32_t j = i < o_n1 ? o_a1 + i : o_a2 + (i - o_n1);
            const float4 pt = g.pts[j];
            const unsigned long long c = mkkey(dist2(qx, qy, qz, pt), pt.w);
            if (c < L.key[K - 1]) L.insert(c, j);
          }
        }
      }
    }
    // k-round merge in ascending key order; the moments in that order (cov_from_sorted's)
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    double a[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
    for (int i = 0; i < k; ++i) {
      const unsigned long long m = wave_min_u64(L.key[0]);
      const unsigned long long win = __builtin_amdgcn_ballot_w64(L.key[0] == m);
      const int wl = win ? static_cast<int>(__builtin_ctzll(win)) : 0;
      const uint32_t wp = __builtin_amdgcn_readlane(L.pos[0], wl);
      if (lane == wl) {
#pragma unroll
        for (int j = 0; j < K - 1; ++j) { L.key[j] = L.key[j + 1]; L.pos[j] = L.pos[j + 1]; }
        L.key[K - 1] = ~0ull;
      }
      const float4 pt = g.pts[wp];
      m0 += pt.x;
      m1 += pt.y;
      m2 += pt.z;
      a[0][0] += static_cast<double>(pt.x * pt.x);
      a[1][0] += static_cast<double>(pt.y * pt.x);
      a[1][1] += static_cast<double>(pt.y * pt.y);
      a[2][0] += static_cast<double>(pt.z * pt.x);
      a[2][1] += static_cast<double>(pt.z * pt.y);
      a[2][2] += static_cast<double>(pt.z * pt.z);
    }
    if (lane == 0) cov_finish(m0, m1, m2, a, static_cast<double>(k), eps, cov, p);
  }
}

// Order-independence certificate for a double sum of n <= 32 floats: if every nonzero term is a
// normal float with |f| in [2^Emin, 2^(Emax+1)) and Emax - Emin <= 24, every term is a multiple of
// 2^(Emin-23) and every partial sum, in ANY order, is bounded by 32 * 2^(Emax+1) <= 2^(Emin-23+53):
// all partial sums are exact doubles, so the result equals the oracle's sorted-order sum bit for
// bit.  All-zero sums are trivially exact; a sum mixing zeros (or denormals) with nonzero terms is
// not certified (the lane goes to the sorted kernel).
struct SumCert {
  float lo = INFINITY, hi = 0.f;
  __device__ __forceinline__ void add(float f) {
    lo = fminf(lo, fabsf(f));
    hi = fmaxf(hi, fabsf(f));
  }
  __device__ __forceinline__ bool ok() const {
    if (hi == 0.f) return true;
    const int elo = static_cast<int>(__float_as_uint(lo) >> 23), ehi = static_cast<int>(__float_as_uint(hi) >> 23);
    return elo > 0 && ehi - elo <= 24;
  }
};

// Logged-threshold k-NN covariance (default): ONE near-first ring search finds the exact k-th float
// d2 (tau) with KthVisitor's med3 network while logging every candidate that was within the
// threshold of its time into the lane's LDS log (compacted to the entries within the current
// threshold whenever it fills); at the end the log entries with d2 <= tau are the k-NN set.  With
// exactly k of them (no ties at tau) and the nine moment sums certified order-independent
// (SumCert), the moments are summed in log order -- bit-identical to the oracle's (d2, index)
// order without sorting.  Any other lane (log overflow, ties at tau, uncertified sums) is listed in
// fb for the register-list kernel.  64-thread blocks, cap x 4 bytes of dynamic LDS per lane.

#define MGICP_KNN_MINW 1  // resident waves per SIMD requested for the logged k-NN kernel (VGPR cap)

template <int K>
__global__ __launch_bounds__(64, MGICP_KNN_MINW) void knn_cov2_kernel(GridView g, double eps, size_t p0, size_t p1, Cov3 cov,
                                                      const uint32_t* __restrict__ perm, int nsent, int cap,
                                                      uint32_t* __restrict__ fb, unsigned int* __restrict__ fb_count,
                                                      int ring_cap, uint8_t* __restrict__ ok_out) {
  extern __shared__ uint32_t s_pos[];
  const size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p1 - p0) return;
  const size_t p = p0 + (perm ? perm[t] : t);
  const float4 q = g.pts[p];
#if MGICP_KNN_DIV
  unsigned long long kt0 = __builtin_amdgcn_s_memtime();
#endif
  KthVisitor<K> v1;
  v1.init(q.x, q.y, q.z, nsent);
  v1.lpos = s_pos + threadIdx.x;
  v1.pts = g.pts;
  v1.cap = cap;
  if (ring_cap >= 0) v1.ring_cap = ring_cap;
  ring_search(g, q.x, q.y, q.z, v1);
  // ring_cap (the source's head start, lazy mode): a point whose k-NN lie farther out (clutter, debris)
  // is left to the lazy pass, which computes it only if a sweep accepts it (ok_out stays 0)
  if (v1.gave_up) return;
#if MGICP_KNN_DIV
  {  // [18] wave iterations of test() [19] max over lanes of the lane's tests [20] lane tests [21] waves
    // [22] search cycles [23] moments + finish cycles (shader clock, summed over waves)
    const unsigned long long kt1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(&g_corr_phase[22], kt1 - kt0);
    kt0 = kt1;
    unsigned long long it = v1.witer, c = v1.ntest, cm = v1.ntest;
    for (int o = 32; o; o >>= 1) {
      it += __shfl_xor(it, o);
      c += __shfl_xor(c, o);
      cm = max(cm, __shfl_xor(cm, o));
    }
    if (threadIdx.x == 0) {
      atomicAdd(&g_corr_phase[18], it);
      atomicAdd(&g_corr_phase[19], cm);
      atomicAdd(&g_corr_phase[20], c);
      atomicAdd(&g_corr_phase[21], 1ull);
    }
  }
#endif
  const int kreal = K - nsent;
  bool ok = v1.cnt <= cap;
  if (ok) {
    const float tau = v1.key[K - 1];
    double m0 = 0.0, m1 = 0.0, m2 = 0.0;
    double a[3][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}};
    SumCert c0, c1, c2, c00, c10, c11, c20, c21, c22;
    int m = 0;
    for (int i0 = 0; i0 < v1.cnt; i0 += kLogBatch) {
     float4 pb[kLogBatch];
#pragma unroll
     for (int u = 0; u < kLogBatch; ++u) pb[u] = g.pts[s_pos[min(i0 + u, v1.cnt - 1) * 64 + threadIdx.x]];
#pragma unroll
     for (int u = 0; u < kLogBatch; ++u) {
      const float4 pt = pb[u];
      if (i0 + u >= v1.cnt || dist2(q.x, q.y, q.z, pt) > tau) continue;
      ++m;
      const float xx = pt.x * pt.x, yx = pt.y * pt.x, yy = pt.y * pt.y;
      const float zx = pt.z * pt.x, zy = pt.z * pt.y, zz = pt.z * pt.z;
      m0 += pt.x;
      m1 += pt.y;
      m2 += pt.z;
      a[0][0] += static_cast<double>(xx);
      a[1][0] += static_cast<double>(yx);
      a[1][1] += static_cast<double>(yy);
      a[2][0] += static_cast<double>(zx);
      a[2][1] += static_cast<double>(zy);
      a[2][2] += static_cast<double>(zz);
      c0.add(pt.x);
      c1.add(pt.y);
      c2.add(pt.z);
      c00.add(xx);
      c10.add(yx);
      c11.add(yy);
      c20.add(zx);
      c21.add(zy);
      c22.add(zz);
     }
    }
    ok = m == kreal && c0.ok() && c1.ok() && c2.ok() && c00.ok() && c10.ok() && c11.ok() && c20.ok() &&
         c21.ok() && c22.ok();
    if (ok) cov_finish(m0, m1, m2, a, static_cast<double>(kreal), eps, cov, p);
  }
#if MGICP_KNN_DIV
  if (threadIdx.x == 0) atomicAdd(&g_corr_phase[23], __builtin_amdgcn_s_memtime() - kt0);
#endif
  // log overflow, ties at tau or an uncertified sum: KnnVisitor's sorted (d2, index) list finishes
  // this point in a follow-up launch over the list (knn_cov_kernel with perm = fb)
  if (!ok) fb[atomicAdd(fb_count, 1u)] = static_cast<uint32_t>(p);
  if (ok_out) ok_out[p] = 1;  // computed here or by the hand-off launch
}


// ------------------------------------------------------------------------------------
// correspondence + Mahalanobis
// ------------------------------------------------------------------------------------
__device__ __forceinline__ void load_cov(const Cov3& c, size_t i, double M[3][3]) {
  const double2 a = c.a[i], b = c.b[i], d = c.c[i];
  M[0][0] = a.x; M[0][1] = a.y; M[0][2] = b.x;
  M[1][0] = a.y; M[1][1] = b.y; M[1][2] = d.x;
  M[2][0] = b.x; M[2][1] = d.x; M[2][2] = d.y;
}

// Exact radius-gated 1-NN of T*s for every source point of the shard.  The search is
// latency-bound on dependent candidate gathers, so this kernel does nothing else: it keeps a
// small register footprint (occupancy) and leaves the fp64 Mahalanobis work to the compaction.
// `qperm` (optional): the shard's query order -- thread t handles shard point qperm[t], a
// Morton order of the source, so that a wave's queries form a compact 3-D patch.
// The starting candidates of a 1-NN query (real points, so any of them keeps the search exact):
// last sweep's match, and the seed map's points of the query's cell (and, in the first sweep, of
// its 6 face neighbours)
__device__ __forceinline__ void seed_query(const GridView& tg, int seeded, uint32_t prev, float qx, float qy, float qz,
                                           NnVisitor& vis) {
  // r03: every seed index first, then every seed point -- two dependent round trips for up to 8
  // seeds instead of one per seed (a branch per seed serialised them: ~90k cycles per wave in
  // the first sweep).  Loads are unconditional from valid addresses, results masked; the
  // visitor's minimum does not depend on the order of the candidates.
  constexpr uint32_t kNone = 0xffffffffu;
  uint32_t sp[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sp[k] = kNone;
  if (seeded) sp[7] = prev;  // last iteration's match
  if (tg.seed) {  // seeded sweeps also test the seed map's candidate (the nearer one wins)
    // the seed map: a point of a Chebyshev-nearest non-empty cell of the query's cell (and, in the
    // first sweep, of its 6 face neighbours)
    const int cx = qcell(qx, tg.ox, tg.inv_h), cy = qcell(qy, tg.oy, tg.inv_h), cz = qcell(qz, tg.oz, tg.inv_h);
    const bool seven = !seeded;  // the first sweep tests the seeds of the query's cell and its 6 face neighbours
    const int dd[7][3] = {{0, 0, 0}, {-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k > 0 && !seven) break;
      const int x = cx + dd[k][0], y = cy + dd[k][1], z = cz + dd[k][2];
      const bool in = x >= 0 && x < tg.nx && y >= 0 && y < tg.ny && z >= 0 && z < tg.nz;
      const size_t ci = in ? static_cast<size_t>(x) + static_cast<size_t>(tg.nx) *
                                                          (static_cast<size_t>(y) + static_cast<size_t>(tg.ny) * z)
                           : 0;
      const uint32_t v = tg.seed[ci];
      sp[k] = in ? v : kNone;
    }
  }
  float4 pt[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) pt[k] = tg.pts[sp[k] != kNone ? sp[k] : 0u];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (sp[k] != kNone) vis.test(pt[k], sp[k]);
}

// ---- wave-uniform 1-NN sweep (r03) ----------------------------------------------------------
// The per-lane search (correspond_kernel) issues one 16-byte gather per candidate and lane; its 64
// lanes touch ~18 cache lines per load, and the texture addresser was busy 87-88 % of every sweep
// (TA_TA_BUSY, profiles/r03/corrdiag): the sweeps were bound by vector-memory ADDRESS throughput,
// not by bytes or arithmetic.  Here the 64 Morton-ordered queries of a wave scan the rows of their
// UNION box together: every row and candidate is wave-uniform, so cell bounds and points arrive
// through the scalar cache (s_load, one 64-byte load per 4 candidates for the whole wave) and
// every lane tests every candidate with packed fp32 arithmetic on a pair-interleaved copy of the
// target (GridView::pairs: x0 x1 y0 y1 z0 z1 w0 w1 per pair) -- bit-identical distances (the FLANN
// order, no contraction).  A 4-candidate block costs 8 packed + 3 VALU per lane; the exact
// (d2, index) key compare runs only when some lane's block minimum reaches its bound.
// Exactness: every lane starts from real seed candidates (bound R); the union box covers every
// included lane's ball; a row is skipped only when no lane's CURRENT bound reaches it; testing
// points outside a lane's ball never changes its exact minimum.  Lanes whose bound exceeds rcap
// (no seed nearby, rejected queries), or waves whose union box is too large, finish with the
// per-lane search from their best.
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// r03: lanes the union scan does not settle are handed to correspond_finish_kernel through a work
// list instead of finishing in place -- in place, a wave waited for its slowest straggler with the
// other lanes idle (62 % of the first sweep's waves had one; 66 % of its wave time)
struct NnWork {
  uint32_t q;     // shard-relative source position
  uint32_t pos;   // the visitor's best so far (sorted target position)
  unsigned long long best;  // its (d2 bits << 32 | index) key, ~0 = none
};

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return __builtin_amdgcn_readfirstlane(v);
}

// squared distances (FLANN L2_Simple per element: ((dx^2) + dy^2) + dz^2, dx = query - point) of this
// lane's query to the 4 candidates of two staged pairs (a0 a1 | b0 b1)
__device__ __forceinline__ void pair_d2(float qx, float qy, float qz, const f4v& a0, const f4v& a1, const f4v& b0,
                                        const f4v& b1, f2v& ra, f2v& rb) {
  const f2v qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
  f2v dx = qx2 - f2v{a0.x, a0.y}, dy = qy2 - f2v{a0.z, a0.w}, dz = qz2 - f2v{a1.x, a1.y};
  ra = dx * dx;
  ra = ra + dy * dy;
  ra = ra + dz * dz;
  dx = qx2 - f2v{b0.x, b0.y};
  dy = qy2 - f2v{b0.z, b0.w};
  dz = qz2 - f2v{b1.x, b1.y};
  rb = dx * dx;
  rb = rb + dy * dy;
  rb = rb + dz * dz;
}

constexpr int kStagePairs = 64;     // pairs staged per wave and chunk (128 candidates, 2 KiB of LDS)
constexpr int kCorrRowSlots = 256;  // union-box rows whose cell bounds a wave keeps in registers (4 per lane)
constexpr int kLdsRows = 64;        // small-ball LDS path: rows of the union box (one per lane in the scan)
constexpr int kLdsBounds = 256;     // cell starts of the box kept in LDS (rows x (x cells + 1))
constexpr int kLdsMeta = (kLdsBounds + kLdsRows) / 4;  // float4 slots of the bounds + row offsets
constexpr int kLdsMaxPts = 512;     // largest lds_cap the kernel is built for (points per wave)

__global__ __launch_bounds__(256, MGICP_CORR_WAVES) void correspond_wave_kernel(
    GridView tg, const float4* __restrict__ src, size_t p0, size_t p1, Xf34 T, double thr, int seeded,
    uint32_t* __restrict__ nn_pos, uint32_t* __restrict__ flags, const uint32_t* __restrict__ qperm, float rcap2,
    int max_rows, int max_xcells, float union_min_r, NnWork* __restrict__ work, unsigned int* __restrict__ work_n,
    int split_max, int lds_cap) {
  __shared__ f4v stage[4][2 * kStagePairs];
  // small-ball waves: the union box's cell bounds, row offsets and points (dynamic LDS, lds_cap
  // points per wave; 0 = off)
  extern __shared__ float4 s_lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool live = t < p1 - p0;  // no early exit: every lane of the wave takes part in the union scan
#if MGICP_CORR_PHASES
  unsigned long long ph_t = __builtin_amdgcn_s_memtime();
#endif
  const size_t p = p0 + (live ? (qperm ? qperm[t] : t) : 0);
  float qx = 0.f, qy = 0.f, qz = 0.f;
  NnVisitor vis;
  if (live) {
    const float4 s = src[p];
    xform(T, s.x, s.y, s.z, qx, qy, qz);
  }
  vis.init(qx, qy, qz, thr);
  const bool rej = live && empty_reject(tg, qx, qy, qz, thr);  // no candidate, no union box, no finish
  if (live && !rej) seed_query(tg, seeded, seeded ? nn_pos[p - p0] : 0xffffffffu, qx, qy, qz, vis);
  MGICP_PH(0);
  // ---- the union box of the included lanes' seed balls
  const float bd0 = vis.prune2();
  bool incl = live && !rej && bd0 <= rcap2;
  int zl = INT_MAX, zh = INT_MIN, yl = INT_MAX, yh = INT_MIN, xl = INT_MAX, xh = INT_MIN;
  float rsum = 0.f;
  if (incl) {
    const float R = sqrtf(bd0 * 1.00001f) + tg.slop;
    rsum = R;
    zl = max(qcell(qz - R, tg.oz, tg.inv_h), 0);
    zh = min(qcell(qz + R, tg.oz, tg.inv_h), tg.nz - 1);
    yl = max(qcell(qy - R, tg.oy, tg.inv_h), 0);
    yh = min(qcell(qy + R, tg.oy, tg.inv_h), tg.ny - 1);
    xl = max(qcell(qx - R, tg.ox, tg.inv_h), 0);
    xh = min(qcell(qx + R, tg.ox, tg.inv_h), tg.nx - 1);
  }
  const int Z0 = wave_min_i(zl), Z1 = wave_max_i(zh), Y0 = wave_min_i(yl), Y1 = wave_max_i(yh);
  const int X0 = wave_min_i(xl), X1 = wave_max_i(xh);
  // small balls (later sweeps: queries near their match) are cheaper per lane: mean bound in cells
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) rsum += __shfl_xor(rsum, o, 64);
  const float nincl = static_cast<float>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(incl)));
  const bool box_ok = Z0 <= Z1 && Y0 <= Y1 && X0 <= X1 &&
                      static_cast<long long>(Z1 - Z0 + 1) * (Y1 - Y0 + 1) <= min(max_rows, kCorrRowSlots) &&
                      X1 - X0 + 1 <= max_xcells &&
                      __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(rsum))) >= union_min_r * tg.h * nincl;
#if MGICP_CORR_PHASES
  // why a wave is left to the per-lane search: [14] no lane included, [15] rows, [16] x cells,
  // [17] mean seed bound below union_min_r (first failing test counted)
  if (lane == 0 && !box_ok) {
    const bool c0 = Z0 <= Z1 && Y0 <= Y1 && X0 <= X1;
    const bool c1 = c0 && static_cast<long long>(Z1 - Z0 + 1) * (Y1 - Y0 + 1) <= min(max_rows, kCorrRowSlots);
    const bool c2 = c1 && X1 - X0 + 1 <= max_xcells;
    atomicAdd(&g_corr_phase[!c0 ? 14 : !c1 ? 15 : !c2 ? 16 : 17], 1ull);
  }
#endif
  const bool incl0 = incl;
  if (!box_ok) incl = false;
  bool tie = false;
  if (box_ok) {
    const f4v* pairs = reinterpret_cast<const f4v*>(tg.pairs);
    f4v* st = stage[wid];
#if MGICP_CORR_STATS
    unsigned long long ncand = 0;
#endif
    // the box's row table: cell bounds [cell_start(row, X0), cell_start(row, X1 + 1)) of slot
    // s = (z - Z0) * nyb + (y - Y0) in lane s & 63 of ra[s >> 6] / rb[s >> 6] -- one gather for every
    // row instead of a dependent load per row
    const int nyb = Y1 - Y0 + 1, nrows = (Z1 - Z0 + 1) * nyb;
    uint32_t ra[kCorrRowSlots / 64], rb[kCorrRowSlots / 64];
#pragma unroll
    for (int k = 0; k < kCorrRowSlots / 64; ++k) {
      const int sl = lane + 64 * k;
      ra[k] = rb[k] = 0;
      if (sl < nrows) {
        const uint32_t row = (static_cast<uint32_t>(Z0 + sl / nyb) * tg.ny + static_cast<uint32_t>(Y0 + sl % nyb)) * tg.nx;
        ra[k] = tg.cell_start[row + X0];
        rb[k] = tg.cell_start[row + X1 + 1];
      }
    }
    // the union scan keeps, per lane, the smallest d2 seen (bcur) and the pair index of the block
    // holding it (bpi); a later block reaching exactly bcur is a tie between two distinct points
    // (every position is tested once: out-of-row positions of a row's edge blocks are masked), left
    // to the per-lane search.  The winner inside the block is resolved exactly after the scan.
    float bcur = INFINITY;
    uint32_t bpi = 0;
    MGICP_PH(1);
    // rows nearest the box centre first (the bounds shrink sooner; the order changes no result)
    const int zc = (Z0 + Z1) >> 1, yc = (Y0 + Y1) >> 1;
    const int zspan = 2 * max(zc - Z0, Z1 - zc), yspan = 2 * max(yc - Y0, Y1 - yc);
    for (int mz = 0; mz <= zspan; ++mz) {
      const int z = zc + ((mz & 1) ? 1 : -1) * ((mz + 1) >> 1);
      if (z < Z0 || z > Z1) continue;
      const float gz = cell_gap(qz, tg.oz, tg.h, z, tg.slop);
      const float gz2 = gz * gz;
      if (!__builtin_amdgcn_ballot_w64(incl && gz2 <= fminf(bd0, bcur) * 1.00001f)) continue;
      for (int my = 0; my <= yspan; ++my) {
        const int y = yc + ((my & 1) ? 1 : -1) * ((my + 1) >> 1);
        if (y < Y0 || y > Y1) continue;
        const float gy = cell_gap(qy, tg.oy, tg.h, y, tg.slop);
        if (!__builtin_amdgcn_ballot_w64(incl && gy * gy + gz2 <= fminf(bd0, bcur) * 1.00001f)) continue;
        const int sl = (z - Z0) * nyb + (y - Y0);
        uint32_t a = 0, b = 0;
#pragma unroll
        for (int k = 0; k < kCorrRowSlots / 64; ++k)
          if ((sl >> 6) == k) {
            a = __builtin_amdgcn_readlane(ra[k], sl & 63);
            b = __builtin_amdgcn_readlane(rb[k], sl & 63);
          }
#if MGICP_CORR_STATS
        ncand += b - a;
#endif
        // stage the row's pairs [a / 2, ceil(b / 2)) in chunks (coalesced: lane l loads float4 l)
        const uint32_t pe = (b + 1) >> 1;
        for (uint32_t c0 = a >> 1; c0 < pe; c0 += kStagePairs) {
          const uint32_t np = min(static_cast<uint32_t>(kStagePairs), pe - c0);
          // always a whole chunk (pair_count pads kStagePairs + 2 far pairs past the cloud): both
          // loads in flight at once; pairs past the row are staged but not scanned
          const f4v v0 = pairs[2 * c0 + lane], v1 = pairs[2 * c0 + 64 + lane];
          st[lane] = v0;
          st[lane + 64] = v1;
          for (uint32_t k = 0; k < np; k += 2) {
            const uint32_t pi = c0 + k, j = 2 * pi;
            f2v r0, r1;
            pair_d2(qx, qy, qz, st[2 * k], st[2 * k + 1], st[2 * k + 2], st[2 * k + 3], r0, r1);
            if (j < a || j + 3 >= b) {  // a row's edge block: positions outside [a, b) are another row's
              if (j < a) r0.x = INFINITY;
              if (j + 1 < a || j + 1 >= b) r0.y = INFINITY;
              if (j + 2 >= b) r1.x = INFINITY;
              if (j + 3 >= b) r1.y = INFINITY;
            }
            const float m = fminf(fminf(r0.x, r0.y), fminf(r1.x, r1.y));
            const bool lt = m < bcur;
            tie = lt ? false : (tie || m == bcur);
            bcur = lt ? m : bcur;
            bpi = lt ? pi : bpi;
          }
        }
      }
    }
    MGICP_PH(2);
    // the winner of the lane's best block: exact (d2, index) keys of its 4 candidates, masked like
    // the scan (a position outside the block's row cannot hold bcur: it was masked there, and it is
    // a real point tested in its own row -- taking it is still exact, the keys decide)
    if (bcur < INFINITY) {
      const f4v a0 = pairs[2 * bpi], a1 = pairs[2 * bpi + 1], b0 = pairs[2 * bpi + 2], b1 = pairs[2 * bpi + 3];
      f2v r0, r1;
      pair_d2(qx, qy, qz, a0, a1, b0, b1, r0, r1);
      const uint32_t j = 2 * bpi;
      const unsigned long long k0 = (static_cast<unsigned long long>(__float_as_uint(r0.x)) << 32) | __float_as_uint(a1.z);
      const unsigned long long k1 = (static_cast<unsigned long long>(__float_as_uint(r0.y)) << 32) | __float_as_uint(a1.w);
      const unsigned long long k2 = (static_cast<unsigned long long>(__float_as_uint(r1.x)) << 32) | __float_as_uint(b1.z);
      const unsigned long long k3 = (static_cast<unsigned long long>(__float_as_uint(r1.y)) << 32) | __float_as_uint(b1.w);
      if (k0 < vis.best) { vis.best = k0; vis.pos = j; }
      if (k1 < vis.best) { vis.best = k1; vis.pos = j + 1; }
      if (k2 < vis.best) { vis.best = k2; vis.pos = j + 2; }
      if (k3 < vis.best) { vis.best = k3; vis.pos = j + 3; }
    }
#if MGICP_CORR_STATS
    if (lane == 0) {
      atomicAdd(&g_corr_stats[6], ncand);
      atomicAdd(&g_corr_stats[7], 1ull);
    }
#endif
  }
  // ---- small-ball waves (union scan not worth it): stage the union box once per wave in LDS, then
  // every included lane runs the exact box search from its seed bound on the LDS copy
  if (!box_ok && lds_cap != 0 && Z0 <= Z1 && Y0 <= Y1 && X0 <= X1) {
    const int nyb = Y1 - Y0 + 1, nxb = X1 - X0 + 1, nrows = (Z1 - Z0 + 1) * nyb, nb = nxb + 1;
    if (nrows <= kLdsRows && nrows * nb <= kLdsBounds) {
      const int cap = max(lds_cap, 0);  // lds_cap < 0: cell bounds only, candidates stay global gathers
      uint32_t* lb = reinterpret_cast<uint32_t*>(s_lds + static_cast<size_t>(wid) * (cap + kLdsMeta));
      uint32_t* loff = lb + kLdsBounds;
      float4* lp = s_lds + static_cast<size_t>(wid) * (cap + kLdsMeta) + kLdsMeta;
      // cell starts of every row of the box for x = X0 .. X1 + 1 (independent loads)
      uint32_t cb[kLdsBounds / 64];
#pragma unroll
      for (int k = 0; k < kLdsBounds / 64; ++k) {
        const int tt = lane + 64 * k;
        const int sr = tt / nb, x = tt - sr * nb;
        const uint32_t row = (static_cast<uint32_t>(Z0 + sr / nyb) * tg.ny + static_cast<uint32_t>(Y0 + sr % nyb)) * tg.nx;
        cb[k] = tt < nrows * nb ? tg.cell_start[row + X0 + x] : 0u;
      }
#pragma unroll
      for (int k = 0; k < kLdsBounds / 64; ++k)
        if (lane + 64 * k < nrows * nb) lb[lane + 64 * k] = cb[k];
      lds_wave_sync();
      // row s (lane s) holds lb[s][nxb] - lb[s][0] points: exclusive scan over the rows
      const uint32_t cnt = lane < nrows ? lb[lane * nb + nxb] - lb[lane * nb] : 0u;
      uint32_t inc = cnt;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(inc, off, 64);
        if (lane >= off) inc += u;
      }
      const uint32_t npts = __builtin_amdgcn_readlane(inc, 63);
      if (lane < nrows) loff[lane] = inc - cnt;
      lds_wave_sync();
      if (lds_cap < 0) {
        if (incl0) box_search_lds(tg, qx, qy, qz, vis, Z0, Y0, X0, nyb, nxb, lb, loff, static_cast<const float4*>(nullptr));
        incl = incl0;
        tie = false;
      } else if (npts <= static_cast<uint32_t>(cap)) {
        // the points, in box order: slot t belongs to the last row whose offset is <= t
        for (uint32_t k0 = 0; k0 < npts; k0 += 256) {  // 4 loads per lane in flight per round
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t tt = k0 + static_cast<uint32_t>(lane + 64 * k);
          uint32_t gp = 0;
          if (tt < npts) {
            int lo = 0, hi = nrows - 1;
            while (lo < hi) {
              const int mid = (lo + hi + 1) >> 1;
              if (loff[mid] <= tt) lo = mid; else hi = mid - 1;
            }
            gp = lb[lo * nb] + (tt - loff[lo]);
          }
          v[k] = tg.pts[gp];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (k0 + static_cast<uint32_t>(lane + 64 * k) < npts) lp[k0 + lane + 64 * k] = v[k];
        }
        lds_wave_sync();
        if (incl0) box_search_lds(tg, qx, qy, qz, vis, Z0, Y0, X0, nyb, nxb, lb, loff, lp);
        incl = incl0;  // settled exactly (keys decide ties): only lanes without a seed ball remain
        tie = false;
      }
    }
  }
  MGICP_PH(3);
  // ---- lanes the union scan did not settle (not included, or a tie between two distinct points
  // at the scan minimum): the per-lane exact search from their best
  const bool fin = live && !rej && (!incl || tie);
#if MGICP_CORR_PHASES
  {
    const int nf = __builtin_popcountll(__builtin_amdgcn_ballot_w64(fin));
    if (lane == 0) {
      if (nf) atomicAdd(&g_corr_phase[6], 1ull);
      atomicAdd(&g_corr_phase[7], 1ull);
      atomicAdd(&g_corr_phase[nf == 0 ? 8 : nf <= 4 ? 9 : nf <= 16 ? 10 : nf < 64 ? 11 : 12], 1ull);
      atomicAdd(&g_corr_phase[13], static_cast<unsigned long long>(nf));
    }
  }
#endif
  const unsigned long long fm = __builtin_amdgcn_ballot_w64(fin);
  if (work && __builtin_popcountll(fm) <= split_max) {
    // hand the stragglers on: one atomic per wave, slots in lane order
    const unsigned long long m = fm;
    if (m) {
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(work_n, static_cast<unsigned int>(__builtin_popcountll(m)));
      base = __builtin_amdgcn_readfirstlane(base);
      const unsigned int off = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u));
      if (fin) work[base + off] = NnWork{static_cast<uint32_t>(p - p0), vis.pos, vis.best};
    }
    MGICP_PH(4);
    if (!live || fin) return;
  } else {
    if (fin) {
      if (vis.best != ~0ull) box_search(tg, qx, qy, qz, vis);
      else ring_search(tg, qx, qy, qz, vis);
    }
    MGICP_PH(4);
  }
  if (!live) return;
  const bool ok = vis.best != ~0ull &&
                  static_cast<double>(__uint_as_float(static_cast<uint32_t>(vis.best >> 32))) < thr;
  nn_pos[p - p0] = ok ? vis.pos : 0xffffffffu;
  flags[p - p0] = ok ? 1u : 0u;
#if MGICP_CORR_STATS
  // [0] queries [1] accepted [2] rejected [3] per-lane tests (seeds + fallback) [4] per-lane ranges
  // [5] lanes left to the per-lane search [6] union candidates (per wave) [7] union-scan waves
  atomicAdd(&g_corr_stats[0], 1ull);
  atomicAdd(&g_corr_stats[ok ? 1 : 2], 1ull);
  atomicAdd(&g_corr_stats[3], static_cast<unsigned long long>(vis.ntest));
  atomicAdd(&g_corr_stats[4], static_cast<unsigned long long>(vis.nrange));
  if (!incl || tie) atomicAdd(&g_corr_stats[5], 1ull);
#endif
}

// The stragglers of correspond_wave_kernel: the per-lane exact search from the visitor state the
// union scan left (a real candidate and its key, or none), 64 of them per wave.  Grid-stride over
// the device-side count.
__global__ __launch_bounds__(256, MGICP_CORR_WAVES) void correspond_finish_kernel(
    GridView tg, const float4* __restrict__ src, size_t p0, Xf34 T, double thr, const NnWork* __restrict__ work,
    const unsigned int* __restrict__ work_n, uint32_t* __restrict__ nn_pos, uint32_t* __restrict__ flags) {
  const unsigned int n = *work_n;
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const NnWork w = work[i];
    const float4 s = src[p0 + w.q];
    float qx, qy, qz;
    xform(T, s.x, s.y, s.z, qx, qy, qz);
    NnVisitor vis;
    vis.init(qx, qy, qz, thr);
    vis.best = w.best;
    vis.pos = w.pos;
    if (vis.best != ~0ull) box_search(tg, qx, qy, qz, vis);
    else ring_search(tg, qx, qy, qz, vis);
    const bool ok = vis.best != ~0ull &&
                    static_cast<double>(__uint_as_float(static_cast<uint32_t>(vis.best >> 32))) < thr;
    nn_pos[w.q] = ok ? vis.pos : 0xffffffffu;
    flags[w.q] = ok ? 1u : 0u;
  }
}

// pair-interleaved copy of the sorted points (GridView::pairs): pair i = {x_2i, x_2i+1, y.., y..,
// z.., z.., bits(w_2i), bits(w_2i+1)}; positions past n are far sentinels (d2 = +inf, w = ~0)
__global__ void pairs_kernel(const float4* __restrict__ pts, size_t n, size_t npairs, float4* __restrict__ out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  const float far = 3.0e38f;
  const float4 s = make_float4(far, far, far, __uint_as_float(0xffffffffu));
  const float4 a = 2 * i < n ? pts[2 * i] : s, b = 2 * i + 1 < n ? pts[2 * i + 1] : s;
  out[2 * i] = make_float4(a.x, b.x, a.y, b.y);
  out[2 * i + 1] = make_float4(a.z, b.z, a.w, b.w);
}

__global__ __launch_bounds__(256, MGICP_CORR_WAVES) void correspond_kernel(GridView tg, const float4* __restrict__ src,
                                                         size_t p0, size_t p1, Xf34 T, double thr,
                                                         int seeded, uint32_t* __restrict__ nn_pos,
                                                         uint32_t* __restrict__ flags,
                                                         const uint32_t* __restrict__ qperm) {
  const size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= p1 - p0) return;
  const size_t p = p0 + (qperm ? qperm[t] : t);
  const float4 s = src[p];
  float qx, qy, qz;
  xform(T, s.x, s.y, s.z, qx, qy, qz);
  NnVisitor vis;
  vis.init(qx, qy, qz, thr);
  if (seeded) {
    // seed with last iteration's match: a real candidate, so the exact search only tightens it,
    // and the ball-cell pruning starts from a near-final radius
    const uint32_t pp = nn_pos[p - p0];
    if (pp != 0xffffffffu) vis.range(tg, pp, pp + 1);
  }
  if (tg.seed) {  // seeded sweeps also test the seed map's candidate (the nearer one wins)
    if (!seeded) {
      // the first sweep: the seeds of the query's cell and its 6 face neighbours, the nearest wins
      const int cx = qcell(qx, tg.ox, tg.inv_h), cy = qcell(qy, tg.oy, tg.inv_h), cz = qcell(qz, tg.oz, tg.inv_h);
      const int dd[7][3] = {{0, 0, 0}, {-1, 0, 0}, {1, 0, 0}, {0, -1, 0}, {0, 1, 0}, {0, 0, -1}, {0, 0, 1}};
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int x = cx + dd[k][0], y = cy + dd[k][1], z = cz + dd[k][2];
        if (x >= 0 && x < tg.nx && y >= 0 && y < tg.ny && z >= 0 && z < tg.nz) {
          const uint32_t pp = tg.seed[static_cast<size_t>(x) +
                                      static_cast<size_t>(tg.nx) * (static_cast<size_t>(y) + static_cast<size_t>(tg.ny) * z)];
          if (pp != 0xffffffffu) vis.range(tg, pp, pp + 1);
        }
      }
    } else
    {
      // a point of a Chebyshev-nearest non-empty cell (seed map): the first sweep's seed, and in
      // later sweeps a second candidate beside the last match (queries move by up to centimetres
      // after the first BFGS run) -- any real candidate keeps the search exact and lets box_search
      // prune from its first row
      const int cx = qcell(qx, tg.ox, tg.inv_h), cy = qcell(qy, tg.oy, tg.inv_h), cz = qcell(qz, tg.oz, tg.inv_h);
      if (cx >= 0 && cx < tg.nx && cy >= 0 && cy < tg.ny && cz >= 0 && cz < tg.nz) {
        const uint32_t pp = tg.seed[static_cast<size_t>(cx) +
                                    static_cast<size_t>(tg.nx) * (static_cast<size_t>(cy) + static_cast<size_t>(tg.ny) * cz)];
        if (pp != 0xffffffffu) vis.range(tg, pp, pp + 1);
      }
    }
  }
  if (tg.boxes) ring_search_boxed(tg, qx, qy, qz, vis);
  else if (kSeedBox && vis.best != ~0ull) box_search(tg, qx, qy, qz, vis);
  else ring_search(tg, qx, qy, qz, vis);
  const bool ok = vis.best != ~0ull &&
                  static_cast<double>(__uint_as_float(static_cast<uint32_t>(vis.best >> 32))) < thr;
  nn_pos[p - p0] = ok ? vis.pos : 0xffffffffu;
  flags[p - p0] = ok ? 1u : 0u;
#if MGICP_CORR_STATS
  atomicAdd(&g_corr_stats[0], 1ull);
  atomicAdd(&g_corr_stats[ok ? 1 : 2], 1ull);
  atomicAdd(&g_corr_stats[ok ? 3 : 4], static_cast<unsigned long long>(vis.ntest));
  atomicAdd(&g_corr_stats[ok ? 5 : 6], static_cast<unsigned long long>(vis.nrange));
#endif
}

// ---- 1-NN cell lists (r04): DESIGN.md "1-NN cell lists" ---------------------------------------------
// Exactness (every claim on real numbers, every fp32 d2 within a relative 2.4e-7 of its real value):
// a query q counted in fine cell C lies in C's box grown by es (the fp32 cell assignment).  Its fp32
// 1-NN key winner t* -- when accepted (d2 < thr) -- lies within D(1 + 1e-5) of q, and within
// |q - t_c| <= U of q (t_c: the cell centre's 1-NN, U: its largest distance to a box corner), so the
// gathered set S = {t : boxdist(t, box) <= min(U, D)(1 + 1e-5)} holds it.  A point t is dropped from
// S only when some real target point a is closer to EVERY point of the box by more than 1e-5 of t's
// largest squared distance to the box: |q - t|^2 - |q - a|^2 is affine in q, so its minimum over the
// box is taken at a corner and computed in closed form; then d2_f32(q, a) < d2_f32(q, t) for every
// q in the box and t is never the winner.  So the list's minimum key is the exact winner for
// accepted queries, and a rejected query's list minimum is >= thr as well (every listed point is a
// real point, no closer than the true 1-NN).  Queries outside the fine grid, or in a cell with no
// target point within D(1 + 1e-5) + its half diagonal of the centre, are rejected.
constexpr int kVlCand = 1024;  // candidates a build wave keeps in LDS (more: the cell stays a fallback cell)
#define MGICP_VLIST_BATCH 4  // list entries a query loads per round (a multiple of 4)
constexpr int kVlBatch = MGICP_VLIST_BATCH;

__device__ __forceinline__ void vl_cell_xyz(const VListView& v, uint32_t ci, uint32_t& ix, uint32_t& iy, uint32_t& iz) {
  const uint32_t nx = static_cast<uint32_t>(v.nx), ny = static_cast<uint32_t>(v.ny);
  ix = ci % nx;
  iy = (ci / nx) % ny;
  iz = ci / (nx * ny);
}

// (defined with the compaction below)
__device__ __forceinline__ void mahalanobis(const Rot33d& R, const double (&C1)[3][3],
                                            const double (&C2)[3][3], double (&m6)[6]);

// the minimum (fp32 d2, original-index tie-break) over the built list of state `st` (< kVlTouched):
// its d2 (inf: none), winner position bp and entry w (bp / w untouched when the list holds no point)
__device__ __forceinline__ float vl_list_min(const VListView& v, uint32_t st, float qx, float qy, float qz,
                                             uint32_t& bp, float4& w) {
  float bd = INFINITY;
  uint32_t off = (st >> 6) << 2, cnt = st & 63u;
  if (cnt == static_cast<uint32_t>(kVlLong)) {  // a long list: count in the header entry
    cnt = __float_as_uint(v.pool[off].x);
    off += 4;
  }
  // lists are padded to a multiple of 4 with far sentinels (d2 = inf): kVlBatch entries per round in
  // flight (groups of 4 past the list's end are not loaded)
  const float4* e = v.pool + off;
  for (uint32_t j = 0; j < cnt; j += kVlBatch) {
    float4 a[kVlBatch];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = e[j + u];
#pragma unroll
    for (int u = 4; u < kVlBatch; ++u)
      a[u] = j + (u & ~3) < cnt ? e[j + u] : make_float4(3.0e38f, 3.0e38f, 3.0e38f, 0.f);
#pragma unroll
    for (int u = 0; u < kVlBatch; ++u) {
      const float d = dist2(qx, qy, qz, a[u]);
      const uint32_t pu = __float_as_uint(a[u].w);
      if (d < bd) {
        bd = d;
        bp = pu;
        w = a[u];
      } else if (d == bd && d < INFINITY && pu != bp) {
        // an exact-distance tie (measure zero on scans, lattices have them): the lower original
        // index wins, as the (d2, index) key of every other 1-NN search
        if (__float_as_uint(v.tpts[pu].w) < __float_as_uint(v.tpts[bp].w)) {
          bp = pu;
          w = a[u];
        }
      }
    }
  }
  return bd;
}

// One query of a listed sweep (every lane of the wave calls it: the request / pending lists take one
// atomic per wave).  Returns 1 accepted (nn / winner coordinates in bp / w), 0 rejected or not live,
// 2 pending (the cell has no list yet: vl_fallback_kernel answers it); s = the source point.
__device__ __forceinline__ int vl_query_point(const VListView& v, const float4* __restrict__ src, size_t p0, size_t n,
                                              const Xf34& T, double thr, size_t t, int lane, float4& s, uint32_t& bp,
                                              float4& w) {
  const bool live = t < n;
  const uint32_t k = static_cast<uint32_t>(t);
  float qx = 0.f, qy = 0.f, qz = 0.f;
  s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (live) {
    s = src[p0 + t];
    xform(T, s.x, s.y, s.z, qx, qy, qz);
  }
  const int ix = qcell(qx, v.ox, v.inv_c), iy = qcell(qy, v.oy, v.inv_c), iz = qcell(qz, v.oz, v.inv_c);
  const bool inside = live && ix >= 0 && ix < v.nx && iy >= 0 && iy < v.ny && iz >= 0 && iz < v.nz;
  const uint32_t ci = inside ? static_cast<uint32_t>(ix) +
                                   static_cast<uint32_t>(v.nx) * (static_cast<uint32_t>(iy) +
                                                                  static_cast<uint32_t>(v.ny) * static_cast<uint32_t>(iz))
                             : 0u;
  const uint32_t st = inside ? v.cell[ci] : kVlReject;
  const bool pending = live && st >= kVlTouched && st != kVlReject;
  // a cell's list is built when it is queried in a sweep after the one that first queried it (or at
  // once, eager): cells a single sweep passes through cost one state word, not a build
  bool req = false;
  const uint32_t mine = kVlTouched | v.epoch;
  if (pending && st == kVlNotBuilt) {
    if (v.eager) req = atomicCAS(&v.cell[ci], kVlNotBuilt, kVlRequested) == kVlNotBuilt;
    else atomicCAS(&v.cell[ci], kVlNotBuilt, mine);
  } else if (pending && st < kVlReject && st != mine) {  // touched in an earlier sweep
    req = atomicCAS(&v.cell[ci], st, kVlRequested) == st;
  }
  // the cell's build request and the query's place in the pending list: one atomic per wave each
  const unsigned long long rm = __builtin_amdgcn_ballot_w64(req);
  if (rm) {
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(&v.ctr[1], static_cast<unsigned int>(__builtin_popcountll(rm)));
    base = __builtin_amdgcn_readfirstlane(base);
    const unsigned int o = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(rm >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(rm), 0u));
    if (req) {
      if (base + o < v.build_cap) v.build[base + o] = ci;
      else atomicExch(&v.cell[ci], kVlNotBuilt);  // no room this sweep: requested again later
    }
  }
  const unsigned long long pm = __builtin_amdgcn_ballot_w64(pending);
  if (pm) {
    unsigned int base = 0;
    if (lane == 0) base = atomicAdd(&v.ctr[2], static_cast<unsigned int>(__builtin_popcountll(pm)));
    base = __builtin_amdgcn_readfirstlane(base);
    const unsigned int o = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(pm >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(pm), 0u));
    if (pending) v.pend[base + o] = k;
  }
  bp = 0xffffffffu;
  w = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!live) return 0;
  if (pending) return 2;
  const float bd = st < kVlTouched ? vl_list_min(v, st, qx, qy, qz, bp, w) : INFINITY;
  const bool ok = bp != 0xffffffffu && static_cast<double>(bd) < thr;
  if (!ok) bp = 0xffffffffu;
  return ok ? 1 : 0;
}

__global__ __launch_bounds__(256) void vl_query_kernel(VListView v, const float4* __restrict__ src, size_t p0,
                                                       size_t n, Xf34 T, double thr, uint32_t* __restrict__ nn_pos,
                                                       uint32_t* __restrict__ flags) {
  // grid order (shard positions): the source reads and the nn_pos / flags writes are coalesced, and
  // neighbouring lanes query neighbouring cells (shared table lines and lists)
  const size_t t = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  float4 s, w;
  uint32_t bp;
  const int r = vl_query_point(v, src, p0, n, T, thr, t, threadIdx.x & 63, s, bp, w);
  if (t >= n || r == 2) return;
  nn_pos[t] = bp;
  flags[t] = r == 1 ? 1u : 0u;
}

// r04: the listed sweep with the compaction fused in (DESIGN.md "Fixed-slot compaction").  One
// 256-thread block per chunk takes its 1024 points in 4 rounds of 256 (grid order); after each
// round's queries a block scan ranks the accepted ones and they go straight into the chunk's fixed
// slots with their Mahalanobis matrices -- the winner's coordinates come from its list entry, the
// source point from the query, so the compaction re-reads neither.  A chunk with a pending query
// (its cell had no list) or, in the lazy source mode, an accepted point without a covariance yet is
// DEFERRED: listed in `defer` (count in v.ctr[3]) and compacted whole by chunk_compact_list_kernel
// once the fallback and the covariances are done.  Results are those of vl_query_kernel +
// chunk_compact_kernel bit for bit (same per-point arithmetic, same slots).
__global__ __launch_bounds__(256, 6) void vl_query_compact_kernel(VListView v, const float4* __restrict__ src, size_t p0,
                                                               size_t n, Xf34 T, double thr,
                                                               uint32_t* __restrict__ nn_pos,
                                                               uint32_t* __restrict__ flags, Cov3 cov_s, Cov3 cov_t,
                                                               Rot33d R, const uint8_t* __restrict__ cov_ok,
                                                               uint32_t* __restrict__ ccnt, uint32_t* __restrict__ defer,
                                                               CorrSoA o) {
  __shared__ uint32_t s_w[2][4];
  __shared__ uint32_t s_defer[2];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t k0 = static_cast<size_t>(blockIdx.x) * kChunkPts;
  uint32_t run = 0;
  bool deferred = false;
#pragma unroll 1
  for (int u = 0; u < kChunkPts / 256; ++u) {
    const size_t t = k0 + static_cast<size_t>(u) * 256 + threadIdx.x;
    float4 s, w;
    uint32_t bp;
    const int r = vl_query_point(v, src, p0, n, T, thr, t, lane, s, bp, w);
    if (t < n && r != 2) {
      nn_pos[t] = bp;
      flags[t] = r == 1 ? 1u : 0u;
    }
    const bool acc = r == 1;
    const bool hold = r == 2 || (acc && cov_ok && !cov_ok[t]);
    const unsigned long long m = __builtin_amdgcn_ballot_w64(acc);
    const unsigned long long hm = __builtin_amdgcn_ballot_w64(hold);
    if (lane == 0) {
      s_w[u & 1][wid] = static_cast<uint32_t>(__builtin_popcountll(m));
      s_defer[u & 1] = 0u;  // (every wave stores 0 before the barrier, then the holders set it)
    }
    __syncthreads();
    if (lane == 0 && hm) s_defer[u & 1] = 1u;
    __syncthreads();
    deferred = deferred || s_defer[u & 1] != 0u;
    uint32_t before = run;
    for (int q = 0; q < wid; ++q) before += s_w[u & 1][q];
    run += s_w[u & 1][0] + s_w[u & 1][1] + s_w[u & 1][2] + s_w[u & 1][3];
    if (acc && !deferred) {
      const uint32_t rk = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u));
      const size_t i = k0 + before + rk;
      double C1[3][3], C2[3][3], m6[6];
      load_cov(cov_s, p0 + t, C1);
      load_cov(cov_t, bp, C2);
      mahalanobis(R, C1, C2, m6);
      o.m00[i] = m6[0]; o.m01[i] = m6[1]; o.m02[i] = m6[2];
      o.m11[i] = m6[3]; o.m12[i] = m6[4]; o.m22[i] = m6[5];
      o.sx[i] = s.x; o.sy[i] = s.y; o.sz[i] = s.z;
      o.qx[i] = w.x; o.qy[i] = w.y; o.qz[i] = w.z;
    }
  }
  if (deferred) {
    if (threadIdx.x == 0) defer[atomicAdd(&v.ctr[3], 1u)] = blockIdx.x;
    return;
  }
  if (threadIdx.x == 0) ccnt[blockIdx.x] = run;
  const uint32_t pad = ((run + 3u) & ~3u) - run;
  if (threadIdx.x < pad) {
    const size_t i = k0 + run + threadIdx.x;
    o.sx[i] = 0.f; o.sy[i] = 0.f; o.sz[i] = 0.f; o.qx[i] = 0.f; o.qy[i] = 0.f; o.qz[i] = 0.f;
    o.m00[i] = 0.0; o.m01[i] = 0.0; o.m02[i] = 0.0; o.m11[i] = 0.0; o.m12[i] = 0.0; o.m22[i] = 0.0;
  }
}

// the requested cells' centres: exact 1-NN within sqrt(thr_c) (none: every point is farther than the
// gate from the whole cell -> reject)
__global__ __launch_bounds__(256) void vl_centre_kernel(GridView tg, VListView v, double thr_c) {
  const unsigned int n = min(v.ctr[1], v.build_cap);
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    uint32_t ix, iy, iz;
    vl_cell_xyz(v, v.build[i], ix, iy, iz);
    const float cx = v.ox + (static_cast<float>(ix) + 0.5f) * v.c;
    const float cy = v.oy + (static_cast<float>(iy) + 0.5f) * v.c;
    const float cz = v.oz + (static_cast<float>(iz) + 0.5f) * v.c;
    NnVisitor vis;
    vis.init(cx, cy, cz, thr_c);
    seed_query(tg, 0, 0xffffffffu, cx, cy, cz, vis);
    if (vis.best != ~0ull) box_search(tg, cx, cy, cz, vis);
    else ring_search(tg, cx, cy, cz, vis);
    const bool ok = vis.best != ~0ull &&
                    static_cast<double>(__uint_as_float(static_cast<uint32_t>(vis.best >> 32))) < thr_c;
    v.bcentre[i] = ok ? vis.pos : 0xffffffffu;
  }
}

// affine dominance over the grown box (closed form of the minimum over its corners): does a (box-centred
// a3, |a|^2 = a2) beat t (t3, |t|^2 = tt, largest squared distance to the box M2) at every point of the box?
__device__ __forceinline__ bool vl_dominates(const double (&a3)[3], double a2, const double (&t3)[3], double tt,
                                             double margin, const double (&hx)[3]) {
  const double fmin = tt - a2 - 2.0 * (hx[0] * fabs(a3[0] - t3[0]) + hx[1] * fabs(a3[1] - t3[1]) +
                                       hx[2] * fabs(a3[2] - t3[2]));
  return fmin > margin;
}

// One wave per requested cell: gather S from the target grid (rows of the box grown by R, one round
// trip for up to 64 rows' bounds, then the points), pick the anchors (the centre's 1-NN and each grown
// corner's nearest candidate), drop every candidate an anchor dominates, then every survivor another
// survivor dominates (dominance is transitive, so the order of the drops does not matter), append the
// rest to the pool padded to a multiple of 4 entries with far sentinels.
// r06: two passes.  The first (vl_build_kernel) keeps at most kVlCandS candidates per wave in LDS (16 B
// each: the sorted position rides in w) and the anchors in LDS instead of registers, so that more build
// waves share a SIMD (r05: 174 VGPRs and 20 KB of LDS per wave, 1.5 waves per SIMD, latency-bound); a
// cell with more candidates stays requested and the second pass (vl_build_large_kernel, kVlCand
// candidates) builds it.  Both run the same per-cell body: the lists are those of the r05 kernel.
constexpr int kVlWaves = 2;    // waves per block of the large pass (LDS: kVlCand x 16 bytes per wave)
constexpr int kVlCandS = 512;  // candidates a first-pass wave keeps (8 KB of LDS: 4 waves per SIMD, as the VGPRs allow)
constexpr int kVlWavesS = 4;   // waves per first-pass block
constexpr int kVlGU = 2;       // candidate loads per lane in flight per gather round (r05: 4; registers)

template <int kCand, bool kLast>
__device__ __forceinline__ void vl_build_cell(const GridView& tg, const VListView& v, uint32_t sl, uint32_t ci, uint32_t tc,
                                              int lane, float4* __restrict__ cand, uint32_t* __restrict__ rowa,
                                              uint32_t* __restrict__ rowp, double* __restrict__ anc,
                                              unsigned int& pk_off, unsigned int& pk_left, unsigned int pk_chunk) {
  {
    if (tc == 0xffffffffu) {
      if (lane == 0) v.cell[ci] = kVlReject;
      return;
    }
#if MGICP_VL_DIAG
    unsigned long long vt0 = __builtin_amdgcn_s_memtime();
#endif
    uint32_t ix, iy, iz;
    vl_cell_xyz(v, ci, ix, iy, iz);
    const uint32_t ii[3] = {ix, iy, iz};
    const float o3[3] = {v.ox, v.oy, v.oz};
    double lo[3], hi[3], ctr[3], hx[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      lo[d] = static_cast<double>(o3[d]) + static_cast<double>(ii[d]) * static_cast<double>(v.c) - v.es;
      hi[d] = lo[d] + static_cast<double>(v.c) + 2.0 * v.es;
      ctr[d] = 0.5 * (lo[d] + hi[d]);
      hx[d] = 0.5 * (hi[d] - lo[d]);
    }
    const float4 pc = tg.pts[tc];
    const double pc3[3] = {pc.x, pc.y, pc.z};
    double U2 = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const double m = fmax(fabs(lo[d] - pc3[d]), fabs(hi[d] - pc3[d]));
      U2 += m * m;
    }
    const double Dp = v.gate * (1.0 + 1e-5) + 1e-9;
    const double R = fmin(sqrt(U2) * (1.0 + 1e-5) + 1e-9, Dp);
    const float R2f = static_cast<float>(R * R) * 1.0001f + 1e-12f;
    const float lof[3] = {static_cast<float>(lo[0]), static_cast<float>(lo[1]), static_cast<float>(lo[2])};
    const float hif[3] = {static_cast<float>(hi[0]), static_cast<float>(hi[1]), static_cast<float>(hi[2])};
    const float Rf = static_cast<float>(R) * 1.0001f;
    const int x0 = max(qcell(lof[0] - Rf, tg.ox, tg.inv_h), 0), x1 = min(qcell(hif[0] + Rf, tg.ox, tg.inv_h), tg.nx - 1);
    const int y0 = max(qcell(lof[1] - Rf, tg.oy, tg.inv_h), 0), y1 = min(qcell(hif[1] + Rf, tg.oy, tg.inv_h), tg.ny - 1);
    const int z0 = max(qcell(lof[2] - Rf, tg.oz, tg.inv_h), 0), z1 = min(qcell(hif[2] + Rf, tg.oz, tg.inv_h), tg.nz - 1);
    int nc = 0;
    bool ovf = false;
    if (x0 <= x1 && y0 <= y1 && z0 <= z1) {
      const int nyr = y1 - y0 + 1, nrows = (z1 - z0 + 1) * nyr;
      for (int r0 = 0; r0 < nrows && !ovf; r0 += 64) {
        const int r = r0 + lane;
        uint32_t a = 0, cnt = 0;
        if (r < nrows) {
          const int z = z0 + r / nyr, y = y0 + r % nyr;
          const float zl = tg.oz + static_cast<float>(z) * tg.h, yl = tg.oy + static_cast<float>(y) * tg.h;
          const float gz = fmaxf(fmaxf(lof[2] - (zl + tg.h), zl - hif[2]) - tg.slop, 0.f);
          const float gy = fmaxf(fmaxf(lof[1] - (yl + tg.h), yl - hif[1]) - tg.slop, 0.f);
          const float gyz = gy * gy + gz * gz;
          if (gyz <= R2f) {
            // r06: only the row's chord of the grown ball (the box grown by R is a cube of up to 2 x 40 mm
            // around an off-surface cell, its rows' full x spans held ~70x the ball's candidates).  A kept
            // point has gx^2 <= R2f - gyz up to the fp32 rounding of both sums (< 1e-6 R2f); slop covers the
            // coordinates' own rounding, qcell is monotone: every point of S is in [xa, xb]
            const float rx = sqrtf(fmaxf(R2f - gyz, 0.f) + 1e-6f * R2f) * 1.0001f + tg.slop;
            const int xa = max(x0, qcell(lof[0] - rx, tg.ox, tg.inv_h));
            const int xb = min(x1, qcell(hif[0] + rx, tg.ox, tg.inv_h));
            if (xa <= xb) {
              const uint32_t row = (static_cast<uint32_t>(z) * static_cast<uint32_t>(tg.ny) + static_cast<uint32_t>(y)) *
                                   static_cast<uint32_t>(tg.nx);
              a = tg.cell_start[row + xa];
              cnt = tg.cell_start[row + xb + 1] - a;
            }
          }
        }
        uint32_t inc = cnt;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t u = __shfl_up(inc, off, 64);
          if (lane >= off) inc += u;
        }
        const uint32_t tot = __builtin_amdgcn_readlane(inc, 63);
        rowa[lane] = a;
        rowp[lane] = inc - cnt;
        lds_wave_sync();
        for (uint32_t t0 = 0; t0 < tot && !ovf; t0 += 64 * kVlGU) {
          float4 pt[kVlGU];
          uint32_t pj[kVlGU];
#pragma unroll
          for (int u = 0; u < kVlGU; ++u) {
            const uint32_t tt = t0 + static_cast<uint32_t>(lane + 64 * u);
            uint32_t j = 0;
            if (tt < tot) {
              int lo_r = 0, hi_r = 63;  // the last row whose exclusive prefix is <= tt
              while (lo_r < hi_r) {
                const int mid = (lo_r + hi_r + 1) >> 1;
                if (rowp[mid] <= tt) lo_r = mid; else hi_r = mid - 1;
              }
              j = rowa[lo_r] + (tt - rowp[lo_r]);
            }
            pj[u] = j;
            pt[u] = tg.pts[j];
          }
#pragma unroll
          for (int u = 0; u < kVlGU; ++u) {
            const uint32_t tt = t0 + static_cast<uint32_t>(lane + 64 * u);
            const float gx = fmaxf(fmaxf(lof[0] - pt[u].x, pt[u].x - hif[0]), 0.f);
            const float gy = fmaxf(fmaxf(lof[1] - pt[u].y, pt[u].y - hif[1]), 0.f);
            const float gz = fmaxf(fmaxf(lof[2] - pt[u].z, pt[u].z - hif[2]), 0.f);
            const bool keep = tt < tot && gx * gx + gy * gy + gz * gz <= R2f;
            const unsigned long long m = __builtin_amdgcn_ballot_w64(keep);
            const int o = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u)));
            if (keep && nc + o < kCand) cand[nc + o] = make_float4(pt[u].x, pt[u].y, pt[u].z, __uint_as_float(pj[u]));
            nc += __builtin_popcountll(m);
          }
          if (nc > kCand) ovf = true;
        }
        lds_wave_sync();  // rowa / rowp are rewritten by the next batch of rows
      }
    }
    if (ovf && !kLast) {  // stays requested: the large pass builds it (listed at the free end of `build`)
      if (lane == 0) {
        const unsigned int r = atomicAdd(&v.ctr[4], 1u);
        const unsigned int n = min(v.ctr[1], v.build_cap);
        if (r < v.build_cap - n) v.build[v.build_cap - 1u - r] = sl;
      }
      return;
    }
    if (ovf || nc == 0) {
      if (lane == 0) v.cell[ci] = ovf ? kVlOverflow : kVlReject;
      return;
    }
    lds_wave_sync();
#if MGICP_VL_DIAG
    // [0] cells [1] candidates [2] stage-1 survivors [3] kept [4..7] cycles gather / stage 1 / stage 2 /
    // write [8] survivors > 256 [9..14] survivors <= 8, 16, 32, 64, 128, 256 [15] stage-2 cycles of cells
    // with > 64 survivors [16] rows scanned
    unsigned long long vt1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      atomicAdd(&g_corr_phase[0], 1ull);
      atomicAdd(&g_corr_phase[1], static_cast<unsigned long long>(nc));
      atomicAdd(&g_corr_phase[4], vt1 - vt0);
    }
#endif
    // anchors: the nearest candidate of each grown corner (box-centred float coordinates suffice:
    // any real point is a valid anchor) and the centre's 1-NN
    unsigned long long ak[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) ak[c] = ~0ull;
    const float cf[3] = {static_cast<float>(ctr[0]), static_cast<float>(ctr[1]), static_cast<float>(ctr[2])};
    const float hf[3] = {static_cast<float>(hx[0]), static_cast<float>(hx[1]), static_cast<float>(hx[2])};
    for (int kq = lane; kq < nc; kq += 64) {
      const float4 tp = cand[kq];
      const float tx = tp.x - cf[0], ty = tp.y - cf[1], tz = tp.z - cf[2];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float dx = ((c & 1) ? hf[0] : -hf[0]) - tx, dy = ((c & 2) ? hf[1] : -hf[1]) - ty,
                    dz = ((c & 4) ? hf[2] : -hf[2]) - tz;
        const float d2 = dx * dx + dy * dy + dz * dz;
        const unsigned long long key = (static_cast<unsigned long long>(__float_as_uint(d2)) << 32) |
                                       static_cast<unsigned int>(kq);
        ak[c] = key < ak[c] ? key : ak[c];
      }
    }
    // the anchors (wave-uniform) go straight to LDS: {x, y, z, |a|^2} relative to the box centre, the
    // centre's 1-NN first (not 72 VGPRs held through stage 1)
    {
      const double a0 = pc3[0] - ctr[0], a1 = pc3[1] - ctr[1], a2 = pc3[2] - ctr[2];
      if (lane == 0) {
        anc[0] = a0;
        anc[1] = a1;
        anc[2] = a2;
        anc[3] = a0 * a0 + a1 * a1 + a2 * a2;
      }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const unsigned long long m = wave_min_u64(ak[c]);
      const int kq = static_cast<int>(static_cast<unsigned int>(m));
      const float4 ap = cand[kq];
      const double a0 = static_cast<double>(ap.x) - ctr[0], a1 = static_cast<double>(ap.y) - ctr[1],
                   a2 = static_cast<double>(ap.z) - ctr[2];
      if (lane == 0) {
        anc[4 * (1 + c) + 0] = a0;
        anc[4 * (1 + c) + 1] = a1;
        anc[4 * (1 + c) + 2] = a2;
        anc[4 * (1 + c) + 3] = a0 * a0 + a1 * a1 + a2 * a2;
      }
    }
    lds_wave_sync();
    // stage 1: the anchors' dominance, survivors compacted to the front of cand (in order: a batch is
    // read whole before its survivors are written, and they land at or before their own slots)
    int ns = 0;
    for (int i0 = 0; i0 < nc; i0 += 64) {
      const int kq = i0 + lane;
      bool keep = false;
      float4 tp = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kq < nc) {
        tp = cand[kq];
        const double t3[3] = {static_cast<double>(tp.x) - ctr[0], static_cast<double>(tp.y) - ctr[1],
                              static_cast<double>(tp.z) - ctr[2]};
        double M2 = 0.0, tt = 0.0;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const double e = fabs(t3[d]) + hx[d];
          M2 += e * e;
          tt += t3[d] * t3[d];
        }
        const double margin = 1e-5 * M2 + 1e-15;
        bool dom = false;
#pragma unroll
        for (int a = 0; a < 9; ++a) {
          const double a3[3] = {anc[4 * a + 0], anc[4 * a + 1], anc[4 * a + 2]};
          dom = dom || vl_dominates(a3, anc[4 * a + 3], t3, tt, margin, hx);
        }
        keep = !dom;
      }
      lds_wave_sync();
      const unsigned long long m = __builtin_amdgcn_ballot_w64(keep);
      const int o = static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                              __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u)));
      if (keep) cand[ns + o] = tp;
      ns += __builtin_popcountll(m);
      lds_wave_sync();
    }
#if MGICP_VL_DIAG
    unsigned long long vt2 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      atomicAdd(&g_corr_phase[2], static_cast<unsigned long long>(ns));
      atomicAdd(&g_corr_phase[5], vt2 - vt1);
      const int b = ns <= 8 ? 9 : ns <= 16 ? 10 : ns <= 32 ? 11 : ns <= 64 ? 12 : ns <= 128 ? 13 : ns <= 256 ? 14 : 8;
      atomicAdd(&g_corr_phase[b], 1ull);
    }
#endif
    // stage 2: survivors against each other (up to 256 survivors; more are kept as they are, in a
    // long list)
    const bool pair = ns <= 256;
    uint32_t keepm = 0;
    for (int i = 0; i < kCand / 64; ++i) {
      const int kq = lane + 64 * i;
      if (kq >= ns) break;
      if (!pair) {
        keepm |= 1u << i;
        continue;
      }
      const float4 tp = cand[kq];
      const double t3[3] = {static_cast<double>(tp.x) - ctr[0], static_cast<double>(tp.y) - ctr[1],
                            static_cast<double>(tp.z) - ctr[2]};
      double M2 = 0.0, tt = 0.0;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const double e = fabs(t3[d]) + hx[d];
        M2 += e * e;
        tt += t3[d] * t3[d];
      }
      const double margin = 1e-5 * M2 + 1e-15;
      bool dom = false;
      for (int j = 0; j < ns && !dom; ++j) {
        if (j == kq) continue;
        const float4 ap = cand[j];
        const double a3[3] = {static_cast<double>(ap.x) - ctr[0], static_cast<double>(ap.y) - ctr[1],
                              static_cast<double>(ap.z) - ctr[2]};
        const double a2 = a3[0] * a3[0] + a3[1] * a3[1] + a3[2] * a3[2];
        dom = vl_dominates(a3, a2, t3, tt, margin, hx);
      }
      if (!dom) keepm |= 1u << i;
    }
    unsigned int cntl = static_cast<unsigned int>(__builtin_popcount(keepm));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cntl += __shfl_xor(cntl, o, 64);
    cntl = __builtin_amdgcn_readfirstlane(cntl);
#if MGICP_VL_DIAG
    unsigned long long vt3 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      atomicAdd(&g_corr_phase[3], static_cast<unsigned long long>(cntl));
      atomicAdd(&g_corr_phase[6], vt3 - vt2);
      if (ns > 64) atomicAdd(&g_corr_phase[15], vt3 - vt2);
    }
#endif
    const bool lng = cntl >= static_cast<unsigned int>(kVlLong);
    const unsigned int cnt4 = ((cntl + 3u) & ~3u) + (lng ? 4u : 0u);
    // the list's place in the pool: r06, from the wave's own pool chunk (pk_chunk entries reserved at a
    // time) -- one returning atomic on the pool head per CELL serialised the whole build on that one L2
    // line (r05: ~34 ns per cell, 143 ms for C4's 4.19M cells).  Pool head: no reservation once the head
    // has passed the cap, so the head exceeds the cap by at most the reservations of the waves in flight
    // (never wraps); the fit test cannot overflow.  Where a list lands changes no result.
    unsigned int off = 0xffffffffu;
    if (cnt4 <= pk_left) {
      off = pk_off;
      pk_off += cnt4;
      pk_left -= cnt4;
    } else {
      const unsigned int r = max(cnt4, pk_chunk);
      if (lane == 0 && __hip_atomic_load(&v.ctr[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v.pool_cap)
        off = atomicAdd(&v.ctr[0], r);
      off = __builtin_amdgcn_readfirstlane(off);
      if (off >= v.pool_cap || r > v.pool_cap - off) {
        if (lane == 0) v.cell[ci] = kVlOverflow;
        return;
      }
      pk_off = off + cnt4;
      pk_left = r - cnt4;
    }
    const unsigned int e0 = off + (lng ? 4u : 0u);
    if (lng && lane < 4) v.pool[off + lane] = make_float4(__uint_as_float(cntl), 0.f, 0.f, 0.f);
    unsigned int run = 0;
    for (int i = 0; i < kCand / 64; ++i) {
      const bool b = (keepm >> i) & 1u;
      const unsigned long long m = __builtin_amdgcn_ballot_w64(b);
      if (b) {
        const unsigned int o = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u));
        const float4 c4 = cand[lane + 64 * i];
        v.pool[e0 + run + o] = c4;
      }
      run += static_cast<unsigned int>(__builtin_popcountll(m));
    }
    const unsigned int npad = ((cntl + 3u) & ~3u) - cntl;
    if (static_cast<unsigned int>(lane) < npad)  // far sentinels (d2 = inf) up to the multiple of 4
      v.pool[e0 + cntl + lane] = make_float4(3.0e38f, 3.0e38f, 3.0e38f, 0.f);
    if (lane == 0) v.cell[ci] = ((off >> 2) << 6) | (lng ? static_cast<unsigned int>(kVlLong) : cntl);
    lds_wave_sync();  // cand is rewritten for the wave's next cell
  }
}

// a build wave's pool chunk: 512 entries, fewer when the pool is small (the chunks every wave of a launch
// may leave unfilled stay below 1/16 of the pool); a multiple of 4
__device__ __forceinline__ unsigned int vl_pool_chunk(const VListView& v, unsigned int nwaves) {
  const unsigned int c = v.pool_cap / (16u * max(nwaves, 1u));
  return max(16u, min(512u, c)) & ~3u;
}

// first pass: one wave per requested cell, at most kVlCandS candidates
__global__ __launch_bounds__(64 * kVlWavesS) void vl_build_kernel(GridView tg, VListView v) {
  __shared__ float4 cand[kVlWavesS][kVlCandS];
  __shared__ uint32_t rowa[kVlWavesS][64], rowp[kVlWavesS][64];
  __shared__ double anc[kVlWavesS][36];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned int n = min(v.ctr[1], v.build_cap);
  const unsigned int nwv = gridDim.x * static_cast<unsigned int>(kVlWavesS);
  unsigned int pk_off = 0, pk_left = 0;
  const unsigned int pk_chunk = vl_pool_chunk(v, nwv);
  for (unsigned int sl = blockIdx.x * kVlWavesS + static_cast<unsigned int>(wid); sl < n; sl += nwv)
    vl_build_cell<kVlCandS, false>(tg, v, sl, v.build[sl], v.bcentre[sl], lane, cand[wid], rowa[wid], rowp[wid], anc[wid],
                                   pk_off, pk_left, pk_chunk);
}

// second pass: the cells the first left requested (more than kVlCandS candidates); each wave checks 64
// slots per round (one load of the slots and their states), then builds its requested cells in turn
__global__ __launch_bounds__(64 * kVlWaves) void vl_build_large_kernel(GridView tg, VListView v) {
  __shared__ float4 cand[kVlWaves][kVlCand];
  __shared__ uint32_t rowa[kVlWaves][64], rowp[kVlWaves][64];
  __shared__ double anc[kVlWaves][36];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned int n = min(v.ctr[1], v.build_cap);
  const unsigned int nwv = gridDim.x * static_cast<unsigned int>(kVlWaves);
  unsigned int pk_off = 0, pk_left = 0;
  const unsigned int pk_chunk = vl_pool_chunk(v, nwv);
  // the first pass listed its cells at the free end of `build` (all of them when they fit): one wave each
  const unsigned int nr = v.ctr[4];
  if (nr <= v.build_cap - n) {
    for (unsigned int i = blockIdx.x * kVlWaves + static_cast<unsigned int>(wid); i < nr; i += nwv) {
      const unsigned int sl = v.build[v.build_cap - 1u - i];
      vl_build_cell<kVlCand, true>(tg, v, sl, v.build[sl], v.bcentre[sl], lane, cand[wid], rowa[wid], rowp[wid],
                                   anc[wid], pk_off, pk_left, pk_chunk);
    }
    return;
  }
  // (no room for the list: every slot's state checked, 64 per wave and round)
  for (unsigned int s0 = (blockIdx.x * kVlWaves + static_cast<unsigned int>(wid)) * 64u; s0 < n; s0 += nwv * 64u) {
    const unsigned int sl = s0 + static_cast<unsigned int>(lane);
    uint32_t ci = 0;
    bool todo = false;
    if (sl < n) {
      ci = v.build[sl];
      todo = v.cell[ci] == kVlRequested;
    }
    unsigned long long m = __builtin_amdgcn_ballot_w64(todo);
    while (m) {
      const int l = static_cast<int>(__builtin_ctzll(m));
      m &= m - 1;
      const uint32_t c = __builtin_amdgcn_readlane(ci, l);
      vl_build_cell<kVlCand, true>(tg, v, s0 + static_cast<unsigned int>(l), c, v.bcentre[s0 + static_cast<unsigned int>(l)], lane, cand[wid], rowa[wid],
                                   rowp[wid], anc[wid], pk_off, pk_left, pk_chunk);
    }
  }
}

// the sweep's queries without a list: the exact per-lane search, seeded as in correspond_kernel
__global__ __launch_bounds__(256) void vl_fallback_kernel(GridView tg, VListView v, const float4* __restrict__ src,
                                                          size_t p0, Xf34 T, double thr, int seeded,
                                                          uint32_t* __restrict__ nn_pos, uint32_t* __restrict__ flags) {
  const unsigned int n = v.ctr[2];
  for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t k = v.pend[i];
    const float4 s = src[p0 + k];
    float qx, qy, qz;
    xform(T, s.x, s.y, s.z, qx, qy, qz);
    // r06: a query whose cell this sweep's build just listed (or rejected) reads the list -- the listed
    // sweep's exact answer -- instead of the per-lane grid search (the build runs before this kernel)
    const int ix = qcell(qx, v.ox, v.inv_c), iy = qcell(qy, v.oy, v.inv_c), iz = qcell(qz, v.oz, v.inv_c);
    const bool inside = ix >= 0 && ix < v.nx && iy >= 0 && iy < v.ny && iz >= 0 && iz < v.nz;
    const uint32_t st = inside ? v.cell[static_cast<uint32_t>(ix) +
                                        static_cast<uint32_t>(v.nx) * (static_cast<uint32_t>(iy) +
                                                                       static_cast<uint32_t>(v.ny) * static_cast<uint32_t>(iz))]
                               : kVlReject;
    if (st < kVlTouched || st == kVlReject) {
      uint32_t bp = 0xffffffffu;
      float4 w;
      const float bd = st < kVlTouched ? vl_list_min(v, st, qx, qy, qz, bp, w) : INFINITY;
      const bool ok = bp != 0xffffffffu && static_cast<double>(bd) < thr;
      nn_pos[k] = ok ? bp : 0xffffffffu;
      flags[k] = ok ? 1u : 0u;
      continue;
    }
    NnVisitor vis;
    vis.init(qx, qy, qz, thr);
    if (!empty_reject(tg, qx, qy, qz, thr)) {  // r05: no point within the gate: rejected without a search
      seed_query(tg, seeded, seeded ? nn_pos[k] : 0xffffffffu, qx, qy, qz, vis);
      if (vis.best != ~0ull) box_search(tg, qx, qy, qz, vis);
      else ring_search(tg, qx, qy, qz, vis);
    }
    const bool ok = vis.best != ~0ull &&
                    static_cast<double>(__uint_as_float(static_cast<uint32_t>(vis.best >> 32))) < thr;
    nn_pos[k] = ok ? vis.pos : 0xffffffffu;
    flags[k] = ok ? 1u : 0u;
  }
}

// diagnostics: [0] cells listed [1] list entries [2] reject [3] overflow [4] requested [5] not built,
// [8 + L] cells with list length L (L < 56)
__global__ __launch_bounds__(256) void vl_stats_kernel(const uint32_t* __restrict__ cell, size_t n,
                                                       unsigned long long* out) {
  // r06: per-block LDS counts, one atomic per block and counter (r05: one global atomic per listed cell on
  // 64 shared addresses, 23 ms per call at C4)
  __shared__ unsigned int cnt[64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0u;
  __syncthreads();
  unsigned int entries = 0;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint32_t c = cell[i];
    if (c == kVlNotBuilt) continue;  // the common case: no atomics
    if (c < kVlTouched) {
      atomicAdd(&cnt[0], 1u);
      entries += c & 63u;
      atomicAdd(&cnt[8 + min(c & 63u, 55u)], 1u);
    } else {
      atomicAdd(&cnt[c == kVlReject ? 2 : c == kVlOverflow ? 3 : c == kVlRequested ? 4 : 5], 1u);
    }
  }
  atomicAdd(&cnt[1], entries);
  __syncthreads();
  if (threadIdx.x < 64 && cnt[threadIdx.x] != 0u)
    atomicAdd(&out[threadIdx.x], static_cast<unsigned long long>(cnt[threadIdx.x]));
}

#if MGICP_CORR_PHASES
hipError_t corr_phase_take(unsigned long long out[24]) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_corr_phase), 24 * sizeof(unsigned long long));
  unsigned long long z[24] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_corr_phase), z, sizeof(z));
  return e;
}
#endif
#if MGICP_CORR_STATS
hipError_t corr_stats_take(unsigned long long out[8]) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_corr_stats), 8 * sizeof(unsigned long long));
  unsigned long long z[8] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_corr_stats), z, sizeof(z));
  return e;
}
#endif

// 10-bit spread for 3-D Morton codes
__device__ __forceinline__ uint32_t spread3(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000ffu;
  v = (v | (v << 8)) & 0x0300f00fu;
  v = (v | (v << 4)) & 0x030c30c3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// 30-bit Morton code of each shard point over the cloud's bbox (1024 steps per axis), value =
// shard-relative position; a stable sort of (key, value) gives the query order of the 1-NN sweeps
__global__ void morton_key_kernel(const float4* __restrict__ pts, size_t p0, size_t n, float ox, float oy,
                                  float oz, float inv, uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 q = pts[p0 + i];
  const int ix = min(max(static_cast<int>((q.x - ox) * inv), 0), 1023);
  const int iy = min(max(static_cast<int>((q.y - oy) * inv), 0), 1023);
  const int iz = min(max(static_cast<int>((q.z - oz) * inv), 0), 1023);
  keys[i] = spread3(ix) | (spread3(iy) << 1) | (spread3(iz) << 2);
  vals[i] = static_cast<uint32_t>(i);
}

// M = (R Cs R' + Ct)^-1 in fp64 with Eigen's 3x3 cofactor inverse (gicp.hpp
// computeTransformation): the upper triangle {m00, m01, m02, m11, m12, m22}.
__device__ __forceinline__ void mahalanobis(const Rot33d& R, const double (&C1)[3][3],
                                            const double (&C2)[3][3], double (&m6)[6]) {
  double RC[3][3], tm[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double a = R.m[3 * r + 0] * C1[0][c];
      a = a + R.m[3 * r + 1] * C1[1][c];
      a = a + R.m[3 * r + 2] * C1[2][c];
      RC[r][c] = a;
    }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double a = RC[r][0] * R.m[3 * c + 0];
      a = a + RC[r][1] * R.m[3 * c + 1];
      a = a + RC[r][2] * R.m[3 * c + 2];
      tm[r][c] = a + C2[r][c];
    }
#define COF(i, j) (tm[((i) + 1) % 3][((j) + 1) % 3] * tm[((i) + 2) % 3][((j) + 2) % 3] - \
                   tm[((i) + 1) % 3][((j) + 2) % 3] * tm[((i) + 2) % 3][((j) + 1) % 3])
  const double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
  double det = c00 * tm[0][0];
  det = det + c10 * tm[1][0];
  det = det + c20 * tm[2][0];
  const double inv = 1.0 / det;
  // Eigen: result(i, j) = cofactor(j, i) / det; keep the upper triangle
  m6[0] = c00 * inv;
  m6[1] = c10 * inv;
  m6[2] = c20 * inv;
  m6[3] = COF(1, 1) * inv;
  m6[4] = COF(2, 1) * inv;
  m6[5] = COF(2, 2) * inv;
#undef COF
}

// Fixed-slot chunk layout of the compacted streams (r04): chunk c of the shard (source positions
// [c * kChunkPts, (c + 1) * kChunkPts) of the shard, a fixed global partition -- shards start on
// super boundaries) keeps its cnt_c accepted correspondences, in grid-sorted order, at slots
// [c * kChunkPts, c * kChunkPts + cnt_c) and zeroes the <= 3 pad slots up to a multiple of 4 (M = 0:
// they add signed zeros only); ccnt[c] = cnt_c.  Slots past a chunk's run are never read.  One
// 256-thread block per chunk takes its points in 4 rounds of 256 (coalesced, in order): a block
// scan of the round's flags ranks them, so no global scan and no chunk-base pass (r01-r03: an
// exclusive scan of the ns flags, chunk_base_kernel, then the scatter).  The matched target point and
// the Mahalanobis matrix of every accepted correspondence go straight into the SoA streams.
__device__ __forceinline__ void chunk_compact_body(int c, const float4* __restrict__ src,
                                                   const float4* __restrict__ tpts, const Cov3& cov_s,
                                                   const Cov3& cov_t, const Rot33d& R,
                                                   const uint32_t* __restrict__ nn_pos,
                                                   const uint32_t* __restrict__ flags, size_t p0, size_t p1,
                                                   uint32_t* __restrict__ ccnt, const CorrSoA& o) {
  __shared__ uint32_t s_w[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t k0 = static_cast<size_t>(c) * kChunkPts;
  const size_t ns = p1 - p0;
  uint32_t run = 0;  // accepted in the earlier rounds
#pragma unroll 1
  for (int u = 0; u < kChunkPts / 256; ++u) {
    const size_t k = k0 + static_cast<size_t>(u) * 256 + threadIdx.x;
    const bool acc = k < ns && flags[k] != 0u;
    const unsigned long long m = __builtin_amdgcn_ballot_w64(acc);
    if (lane == 0) s_w[u & 1][wid] = static_cast<uint32_t>(__builtin_popcountll(m));
    __syncthreads();  // (double-buffered counts: the next round writes the other half)
    uint32_t before = run;
    for (int w = 0; w < wid; ++w) before += s_w[u & 1][w];
    run += s_w[u & 1][0] + s_w[u & 1][1] + s_w[u & 1][2] + s_w[u & 1][3];
    if (acc) {
      const uint32_t r = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m), 0u));
      const size_t i = k0 + before + r;
      const size_t p = p0 + k;
      const uint32_t j = nn_pos[k];
      const float4 s = src[p], t = tpts[j];
      double C1[3][3], C2[3][3], m6[6];
      load_cov(cov_s, p, C1);
      load_cov(cov_t, j, C2);
      mahalanobis(R, C1, C2, m6);
      o.m00[i] = m6[0]; o.m01[i] = m6[1]; o.m02[i] = m6[2];
      o.m11[i] = m6[3]; o.m12[i] = m6[4]; o.m22[i] = m6[5];
      o.sx[i] = s.x; o.sy[i] = s.y; o.sz[i] = s.z;
      o.qx[i] = t.x; o.qy[i] = t.y; o.qz[i] = t.z;
    }
  }
  if (threadIdx.x == 0) ccnt[c] = run;
  const uint32_t pad = ((run + 3u) & ~3u) - run;
  if (threadIdx.x < pad) {
    const size_t i = k0 + run + threadIdx.x;
    o.sx[i] = 0.f; o.sy[i] = 0.f; o.sz[i] = 0.f; o.qx[i] = 0.f; o.qy[i] = 0.f; o.qz[i] = 0.f;
    o.m00[i] = 0.0; o.m01[i] = 0.0; o.m02[i] = 0.0; o.m11[i] = 0.0; o.m12[i] = 0.0; o.m22[i] = 0.0;
  }
}

__global__ __launch_bounds__(256, 6) void chunk_compact_kernel(const float4* __restrict__ src,
                                                            const float4* __restrict__ tpts, Cov3 cov_s,
                                                            Cov3 cov_t, Rot33d R,
                                                            const uint32_t* __restrict__ nn_pos,
                                                            const uint32_t* __restrict__ flags, size_t p0,
                                                            size_t p1, uint32_t* __restrict__ ccnt, CorrSoA o) {
  chunk_compact_body(static_cast<int>(blockIdx.x), src, tpts, cov_s, cov_t, R, nn_pos, flags, p0, p1, ccnt, o);
}

// the chunks a fused listed sweep deferred (list `defer`, *count of them): compacted whole
__global__ __launch_bounds__(256, 6) void chunk_compact_list_kernel(const float4* __restrict__ src,
                                                                 const float4* __restrict__ tpts, Cov3 cov_s,
                                                                 Cov3 cov_t, Rot33d R,
                                                                 const uint32_t* __restrict__ nn_pos,
                                                                 const uint32_t* __restrict__ flags, size_t p0,
                                                                 size_t p1, uint32_t* __restrict__ ccnt,
                                                                 const uint32_t* __restrict__ defer,
                                                                 const unsigned int* __restrict__ count, CorrSoA o) {
  const unsigned int nd = *count;
  for (unsigned int i = blockIdx.x; i < nd; i += gridDim.x) {
    chunk_compact_body(static_cast<int>(defer[i]), src, tpts, cov_s, cov_t, R, nn_pos, flags, p0, p1, ccnt, o);
    __syncthreads();  // the next chunk reuses the block's LDS counts
  }
}

// chunk j's groups of 4 slots in the fixed-slot layout: [chunk_g0(j), chunk_g1(ccnt, j))
__device__ __forceinline__ uint32_t chunk_g0(int j) { return static_cast<uint32_t>(j) * (kChunkPts / 4); }
__device__ __forceinline__ uint32_t chunk_g1(const uint32_t* __restrict__ ccnt, int j) {
  return chunk_g0(j) + ((ccnt[j] + 3u) >> 2);
}

// ------------------------------------------------------------------------------------
// objective pass (fdf) and reductions
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// ---- 16 values at once: wave_sum's tree as a reduce-scatter in registers (r03) -----------------
// wave_sum pairs lanes (l, l + d) for d = 32, 16, 8, 4, 2, 1 -- the same pairs as l ^ d on the
// lanes that carry the result -- so any scheme that adds exactly those pairs at every level gives
// lane 0's sums bit for bit (fp64 addition is commutative).  Here, instead of 16 x 6 shuffles
// through the LDS crossbar (192 ds_bpermute and ~60 exposed lgkmcnt waits per chunk at one wave per
// SIMD), each level halves the values a lane keeps and exchanges only those: d = 32 and 16 by
// gfx950's v_permlane32_swap / v_permlane16_swap, d = 8 by DPP row_ror:8, the last three levels on
// two values by row_ror:12 and quad_perm (row_ror:n makes lane l read lane (l - n) mod 16 of its row;
// the pairs needed are those of the lanes with bit 2 clear, where row_ror:12 reads lane l + 4 = l ^ 4).
// About 70 VALU instructions, no LDS traffic.
// Afterwards lane 8k (k = 0..7) holds values 2k and 2k + 1 (lane bits 5, 4, 3 = value bits 3, 2, 1).
__device__ __forceinline__ unsigned int lo32(double v) {
  return static_cast<unsigned int>(__double_as_longlong(v));
}
__device__ __forceinline__ unsigned int hi32(double v) {
  return static_cast<unsigned int>(static_cast<unsigned long long>(__double_as_longlong(v)) >> 32);
}
__device__ __forceinline__ double mk64(unsigned int lo, unsigned int hi) {
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
template <int kCtrl>
__device__ __forceinline__ double dpp64(double v) {
  return mk64(static_cast<unsigned int>(__builtin_amdgcn_mov_dpp(static_cast<int>(lo32(v)), kCtrl, 0xF, 0xF, false)),
              static_cast<unsigned int>(__builtin_amdgcn_mov_dpp(static_cast<int>(hi32(v)), kCtrl, 0xF, 0xF, false)));
}
// lanes with bit log2(kD) clear: a[l] + a[l ^ kD]; set: b[l] + b[l ^ kD]   (kD = 32 or 16)
template <int kD>
__device__ __forceinline__ double swap_add(double a, double b) {
  unsigned int alo = lo32(a), ahi = hi32(a), blo = lo32(b), bhi = hi32(b);
  if constexpr (kD == 32) {
    const auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    alo = l[0]; blo = l[1]; ahi = h[0]; bhi = h[1];
  }
  return mk64(alo, ahi) + mk64(blo, bhi);
}
__device__ __forceinline__ void wave_sum16(double (&v)[16], int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = swap_add<32>(v[i], v[i + 8]);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = swap_add<16>(v[i], v[i + 4]);
  const bool b3 = (lane & 8) != 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double x = b3 ? v[i + 2] : v[i], y = b3 ? v[i] : v[i + 2];
    v[i] = x + dpp64<0x128>(y);  // row_ror:8 = lane l ^ 8
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) v[i] = v[i] + dpp64<0x12C>(v[i]);  // row_ror:12 reads lane l + 4 = l ^ 4 where bit 2 is clear
#pragma unroll
  for (int i = 0; i < 2; ++i) v[i] = v[i] + dpp64<0x4E>(v[i]);   // quad_perm [2,3,0,1] = l ^ 2
#pragma unroll
  for (int i = 0; i < 2; ++i) v[i] = v[i] + dpp64<0xB1>(v[i]);   // quad_perm [1,0,3,2] = l ^ 1
}

// reduce kRedVals doubles across a 256-thread block; thread 0 writes dst[0..15]
__device__ __forceinline__ void block_reduce_store(double (&acc)[kRedVals], double* dst) {
  __shared__ double sm[4][kRedVals];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();  // sm may still be read by a previous call in this block
#pragma unroll
  for (int v = 0; v < kRedVals; ++v) {
    const double w = wave_sum(acc[v]);
    if (lane == 0) sm[wid][v] = w;
  }
  __syncthreads();
  if (threadIdx.x < kRedVals) {
    const int v = threadIdx.x;
    double s = sm[0][v];
    s = s + sm[1][v];
    s = s + sm[2][v];
    s = s + sm[3][v];
    dst[v] = s;
  }
}

// ---- the fixed global reduction tree (identical for every rank count) ----------------------
//   chunk  (kChunkPts source positions of the grid-sorted cloud): one wave; lane l accumulates
//          its elements in order, then wave_sum's shuffle tree          -> partial[c][v]
//   super  (kSuperChunks consecutive chunks): partial[c0][v] + partial[c0+1][v] + ... in order
//   total  lane l sums supers l, l + 64, ... in order, then wave_sum    -> out[v]
// Shards start on super boundaries, so a rank's supers are exactly the N = 1 run's supers with
// the same indices; a multi-GPU pass all-gathers the supers and runs the same total.
// In-launch finish, fence-free form of cdna_hip_programming.md Guideline 16 (MI355X_MICROARCH.md
// "Valid forms", first table row): partials are stored write-through (sc1, relaxed agent-scope
// atomic stores) and drained (s_waitcnt vmcnt(0)) before an agent-scope ticket is taken; the wave
// drawing the last ticket reads them with sc1 loads.  No buffer_wbl2 / buffer_inv (a release
// fence per block cost ~25 us per launch at 1024 blocks).
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
      const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(p)), __ATOMIC_RELAXED,
      __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one wave: values [v0, v0 + 16) of the total over nsup supers of NV values each, held as
// nranks rows of maxsup supers (row r = the supers of rank r, super_first(r) onwards); lane 0
// writes out[v0 + v]
template <int NV, bool kSc1>
__device__ __forceinline__ void wave_total(const double* sup, long long nsup, long long maxsup, int nranks, int v0,
                                           double* out) {
  const int lane = threadIdx.x & 63;
  double acc[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.0;
  for (long long sg = lane; sg < nsup; sg += 64) {
    size_t at = static_cast<size_t>(sg);
    if (nranks > 1) {
      const int r = super_owner(sg, nsup, nranks);
      at = static_cast<size_t>(r) * maxsup + (sg - super_first(r, nsup, nranks));
    }
    const double* row = sup + at * NV + v0;
#pragma unroll
    for (int v = 0; v < 16; ++v)
      if (v0 + v < NV) acc[v] += kSc1 ? ld_sc1(row + v) : row[v];
  }
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = wave_sum(acc[v]);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < 16; ++v)
      if (v0 + v < NV) out[v0 + v] = acc[v];
  }
}

// super partials of nch chunk partials (NV values each): block s, thread v < NV
template <int NV>
__global__ void super_reduce_kernel(const double* __restrict__ chunk, int nch, double* __restrict__ sup) {
  const int v = threadIdx.x, sj = blockIdx.x;
  if (v >= NV) return;
  const int c0 = sj * kSuperChunks, nin = min(kSuperChunks, nch - c0);
  double a = chunk[static_cast<size_t>(c0) * NV + v];
  for (int q = 1; q < nin; ++q) a = a + chunk[static_cast<size_t>(c0 + q) * NV + v];
  sup[static_cast<size_t>(sj) * NV + v] = a;
}

// totals of all supers (one wave per 16 values); rows of maxsup supers per rank
template <int NV>
__global__ __launch_bounds__(64) void finish_supers_kernel(const double* __restrict__ sup, long long nsup,
                                                           long long maxsup, int nranks, double* __restrict__ out) {
  wave_total<NV, false>(sup, nsup, maxsup, nranks, 16 * blockIdx.x, out);
}

// the 8 x 16 bytes of a command block: system-coherent loads of the host's pinned copy
// (sc0 sc1: no GPU cache holds them) or agent-coherent loads of the device mailbox (sc1)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool kHost>
__device__ __forceinline__ void read_cmd(const PassCmd* c, unsigned long long (&v)[16]) {
  u32x4 r[8];
  const u32x4* p = reinterpret_cast<const u32x4*>(c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (kHost) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(r[i]) : "v"(p + i) : "memory");
    else asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r[i]) : "v"(p + i) : "memory");
  }
  // the wait names the loads' destination registers as operands: the compiler does not know that an
  // asm load's output is only valid after s_waitcnt, and a wait with no operands let it move the
  // stamp compares above it (they then read the address registers -- r03: a server that never saw
  // its next command)
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])
               :
               : "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[2 * i] = (static_cast<unsigned long long>(r[i].y) << 32) | r[i].x;
    v[2 * i + 1] = (static_cast<unsigned long long>(r[i].w) << 32) | r[i].z;
  }
}

// block 0's forward of a validated command to the device mailbox (agent-coherent vector stores)
__device__ __forceinline__ void write_mail(PassCmd* c, const unsigned long long (&v)[16]) {
  u32x4* p = reinterpret_cast<u32x4*>(c);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    u32x4 w;
    w.x = static_cast<unsigned int>(v[2 * i]); w.y = static_cast<unsigned int>(v[2 * i] >> 32);
    w.z = static_cast<unsigned int>(v[2 * i + 1]); w.w = static_cast<unsigned int>(v[2 * i + 1] >> 32);
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p + i), "v"(w) : "memory");
  }
}

// one correspondence of OptimizationFunctorWithIndices::fdf: pp = A s (fp32, Eigen order),
// r = fp32(pp - q) widened to fp64, t = M r, accumulate r't, t and s t'
__device__ __forceinline__ void fdf_point(const Xf34& A, float sx, float sy, float sz, float qx,
                                          float qy, float qz, double m00, double m01, double m02,
                                          double m11, double m12, double m22,
                                          double (&acc)[kRedVals]) {
  float px, py, pz;
  xform(A, sx, sy, sz, px, py, pz);
  const double r0 = static_cast<double>(px - qx);
  const double r1 = static_cast<double>(py - qy);
  const double r2 = static_cast<double>(pz - qz);
  double t0 = m00 * r0; t0 = t0 + m01 * r1; t0 = t0 + m02 * r2;
  double t1 = m01 * r0; t1 = t1 + m11 * r1; t1 = t1 + m12 * r2;
  double t2 = m02 * r0; t2 = t2 + m12 * r1; t2 = t2 + m22 * r2;
  double d = r0 * t0; d = d + r1 * t1; d = d + r2 * t2;
  const double dx = sx, dy = sy, dz = sz;
  acc[0] += d;
  acc[1] += t0; acc[2] += t1; acc[3] += t2;
  acc[4] += dx * t0; acc[5] += dx * t1; acc[6] += dx * t2;
  acc[7] += dy * t0; acc[8] += dy * t1; acc[9] += dy * t2;
  acc[10] += dz * t0; acc[11] += dz * t1; acc[12] += dz * t2;
}

// the fp64 part of fdf_point for a residual r = fp32(A s - q) already widened to fp64
__device__ __forceinline__ void fdf_point_r(double r0, double r1, double r2, float sx, float sy, float sz,
                                            double m00, double m01, double m02, double m11, double m12,
                                            double m22, double (&acc)[kRedVals]) {
  double t0 = m00 * r0; t0 = t0 + m01 * r1; t0 = t0 + m02 * r2;
  double t1 = m01 * r0; t1 = t1 + m11 * r1; t1 = t1 + m12 * r2;
  double t2 = m02 * r0; t2 = t2 + m12 * r1; t2 = t2 + m22 * r2;
  double d = r0 * t0; d = d + r1 * t1; d = d + r2 * t2;
  const double dx = sx, dy = sy, dz = sz;
  acc[0] += d;
  acc[1] += t0; acc[2] += t1; acc[3] += t2;
  acc[4] += dx * t0; acc[5] += dx * t1; acc[6] += dx * t2;
  acc[7] += dy * t0; acc[8] += dy * t1; acc[9] += dy * t2;
  acc[10] += dz * t0; acc[11] += dz * t1; acc[12] += dz * t2;
}

// Eigen's Matrix4f * Vector4f for two points at once (packed fp32, v_pk_mul_f32 / v_pk_add_f32):
// element-wise the same roundings as xform, half the fp32 instructions
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void resid2(const Xf34& T, pf2 x, pf2 y, pf2 z, pf2 qx, pf2 qy, pf2 qz, pf2& rx,
                                       pf2& ry, pf2& rz) {
  pf2 a = T.m[0] * x;
  a = a + T.m[1] * y;
  a = a + T.m[2] * z;
  rx = (a + T.m[3]) - qx;
  pf2 b = T.m[4] * x;
  b = b + T.m[5] * y;
  b = b + T.m[6] * z;
  ry = (b + T.m[7]) - qy;
  pf2 c = T.m[8] * x;
  c = c + T.m[9] * y;
  c = c + T.m[10] * z;
  rz = (c + T.m[11]) - qz;
}

// 4 consecutive correspondences of the compacted streams (one 16-byte load per stream and lane):
// f = sx sy sz qx qy qz (float4 of 4 coordinates), d = m00 m00' m01 m01' m02 m02' m11 m11' m12 m12'
// m22 m22' (double2 of 2 matrix entries) -- 72 dwords
struct CorrGroup {
  float4 f[6];
  double2 d[12];
};

__device__ __forceinline__ void load_group(const CorrSoA& c, uint32_t i, CorrGroup& g) {
  g.f[0] = reinterpret_cast<const float4*>(c.sx)[i];
  g.f[1] = reinterpret_cast<const float4*>(c.sy)[i];
  g.f[2] = reinterpret_cast<const float4*>(c.sz)[i];
  g.f[3] = reinterpret_cast<const float4*>(c.qx)[i];
  g.f[4] = reinterpret_cast<const float4*>(c.qy)[i];
  g.f[5] = reinterpret_cast<const float4*>(c.qz)[i];
  const size_t i2 = 2 * static_cast<size_t>(i);
  const double* const m[6] = {c.m00, c.m01, c.m02, c.m11, c.m12, c.m22};
#pragma unroll
  for (int e = 0; e < 6; ++e) {
    const double2* M = reinterpret_cast<const double2*>(m[e]) + i2;
    g.d[2 * e] = M[0];
    g.d[2 * e + 1] = M[1];
  }
}

// the group's 4 correspondences in stream order (residuals two at a time in packed fp32)
__device__ __forceinline__ void fdf_group(const Xf34& A, const CorrGroup& g, double (&acc)[kRedVals]) {
  fdf_point(A, g.f[0].x, g.f[1].x, g.f[2].x, g.f[3].x, g.f[4].x, g.f[5].x, g.d[0].x, g.d[2].x, g.d[4].x,
            g.d[6].x, g.d[8].x, g.d[10].x, acc);
  fdf_point(A, g.f[0].y, g.f[1].y, g.f[2].y, g.f[3].y, g.f[4].y, g.f[5].y, g.d[0].y, g.d[2].y, g.d[4].y,
            g.d[6].y, g.d[8].y, g.d[10].y, acc);
  fdf_point(A, g.f[0].z, g.f[1].z, g.f[2].z, g.f[3].z, g.f[4].z, g.f[5].z, g.d[1].x, g.d[3].x, g.d[5].x,
            g.d[7].x, g.d[9].x, g.d[11].x, acc);
  fdf_point(A, g.f[0].w, g.f[1].w, g.f[2].w, g.f[3].w, g.f[4].w, g.f[5].w, g.d[1].y, g.d[3].y, g.d[5].y,
            g.d[7].y, g.d[9].y, g.d[11].y, acc);
}

// The gate of a pass whose state is not known at launch (pre-launched gated passes and the
// resident pass server).  Every block's thread 0 polls a command block until it carries this
// pass's sequence number: blocks [0, host_pollers) the host-written copy (pinned, mapped,
// system-coherent loads, or device memory the host stores into through the BAR), the others the
// device mailbox block 0 forwards it to.  Returns false on a cancel command, on a complete command
// with a LATER sequence number (this block was left behind by a cancel: a server whose blocks could
// not all be resident when the host gave up on a pass), or after `timeout` wall-clock ticks -- every
// wave reaches an exit.  rstamp: the command's row stamp (word 14).
__device__ __forceinline__ bool pass_gate(unsigned long long seq, const PassCmd* cmd, PassCmd* mail,
                                          unsigned long long timeout, unsigned long long* gtrace,
                                          int host_pollers, Xf34& A, int& reverse, unsigned int& rstamp) {
  __shared__ unsigned int sw[kCmdWords];
  __shared__ int sok;
  __syncthreads();  // sw / sok of the previous gate of this block are consumed
  if (threadIdx.x == 0) {
    // block 0 alone polls the host's command block over PCIe (256 pollers of host memory were
    // measured to delay the command by ~320 us) and forwards it to the device mailbox the
    // other blocks poll; both blocks are read whole (8 x 16 B per poll) and validated by stamp
    const bool host_poller = blockIdx.x < host_pollers;
    const unsigned int stamp = static_cast<unsigned int>(seq);
    const unsigned long long t0 = wall_clock64();
    unsigned long long v[16];
    bool got = false, later = false;
    for (;;) {
      if (host_poller) read_cmd<true>(cmd, v);
      else read_cmd<false>(mail, v);
      const unsigned int st0 = static_cast<unsigned int>(v[0] >> 32);
      bool same = true;
#pragma unroll
      for (int i = 1; i < kCmdWords; ++i) same = same && static_cast<unsigned int>(v[i] >> 32) == st0;
      if (same && st0 == stamp) { got = true; break; }
      // a complete, newer command: the host has moved past this pass (signed 32-bit distance)
      if (same && static_cast<int>(st0 - stamp) > 0) { later = true; break; }
      if (wall_clock64() - t0 > timeout) break;  // no command: give up as if cancelled
      __builtin_amdgcn_s_sleep(1);
    }
    if (gtrace && host_poller) {  // diagnostics: kernel start and command seen (wall clock)
      gtrace[4 * (seq & 1023)] = t0;
      gtrace[4 * (seq & 1023) + 1] = wall_clock64();
    }
    if (!got) {
      // a timeout or a later command forwards a cancel (stamped with the later sequence number
      // when there is one), so every block still waiting for this pass exits promptly
      const unsigned long long st = later ? (v[0] >> 32) : static_cast<unsigned long long>(stamp);
#pragma unroll
      for (int i = 0; i < kCmdWords; ++i) v[i] = (st << 32) | (i == 12 ? kPassCancel : 0u);
    }
#pragma unroll
    for (int i = 0; i < kCmdWords; ++i) sw[i] = static_cast<unsigned int>(v[i]);
    if (blockIdx.x == 0 && host_pollers > 0 && host_pollers < static_cast<int>(gridDim.x)) write_mail(mail, v);
    sok = got ? 1 : 0;
  }
  __syncthreads();
  if (gtrace && threadIdx.x == 0)  // diagnostics: the latest block to pass the gate
    atomicMax(&gtrace[4 * (seq & 1023) + 2], wall_clock64());
  if (!sok || sw[12] != kPassRun) return false;
#pragma unroll
  for (int i = 0; i < 12; ++i) A.m[i] = __uint_as_float(sw[i]);
  reverse = static_cast<int>(sw[13]);
  rstamp = sw[14];
  return true;
}

// chunk j's partial (wave_sum's shuffle tree of the lanes' in-order sums) and its exact count
// (ccnt: pad slots are not counted), stored write-through (sc1)
__device__ __forceinline__ void chunk_store(int j, double (&acc)[kRedVals], const uint32_t* __restrict__ ccnt,
                                            double* __restrict__ partial, int lane) {
  const double cnt = static_cast<double>(ccnt[j]);
  double* pj = partial + static_cast<size_t>(j) * kRedVals;
  // acc[13..15] are never accumulated (+0.0), so value 13 -- the count -- is replaced after the
  // tree and 14, 15 come out +0.0 as the r02 form stored them
  wave_sum16(acc, lane);
  if ((lane & 7) == 0) {
    const double v1 = lane == 48 ? cnt : acc[1];
    u32x4 w;
    w.x = lo32(acc[0]); w.y = hi32(acc[0]); w.z = lo32(v1); w.w = hi32(v1);
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(pj + (lane >> 2)), "v"(w) : "memory");
  }
}

// ---- the tagged tail of the resident server (r03) ------------------------------------------------
// A chunk partial as 32 stamped words, value v in words 2v (low half) and 2v + 1 (high half), each
// (rstamp << 32) | half and written whole by one write-through store (the 8-byte {data, tag}
// granule of MI355X_MICROARCH "Valid forms"): a reader needs no ticket, drain or fence -- a word is
// current when it carries this pass's stamp.
__device__ __forceinline__ void chunk_store_tagged(int j, double (&acc)[kRedVals], const uint32_t* __restrict__ ccnt,
                                                   unsigned long long* __restrict__ tpart, int lane,
                                                   unsigned int rstamp) {
  const double cnt = static_cast<double>(ccnt[j]);
  wave_sum16(acc, lane);
  if ((lane & 7) == 0) {  // lane 8k: values 2k, 2k + 1 -> words 4k .. 4k + 3
    const double v1 = lane == 48 ? cnt : acc[1];
    unsigned long long* pj = tpart + static_cast<size_t>(j) * 32 + (lane >> 1);
    u32x4 w0, w1;
    w0.x = lo32(acc[0]); w0.y = rstamp; w0.z = hi32(acc[0]); w0.w = rstamp;
    w1.x = lo32(v1); w1.y = rstamp; w1.z = hi32(v1); w1.w = rstamp;
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(pj), "v"(w0) : "memory");
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(pj + 2), "v"(w1) : "memory");
  }
}

__device__ __forceinline__ unsigned long long ld_sc1_u64(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The designated reducer of super sj (wave sj): its 16 sums -- lane v < 16 returns value v, the
// chunks summed in chunk order exactly as wave_tickets does -- once every chunk of the super carries
// this pass's stamp.  false (no row) when the host has moved on: a newer stamp in the command block
// than the current pass `cur` in the command block (`cmd`, device memory the host writes through the
// BAR; nullptr: not checked) or `limit`
// wall-clock ticks without the super completing.
// lane l reads chunks 8 (l >> 4) .. 8 (l >> 4) + 7 of value l & 15 (one round of 16 loads per lane);
// the chunk-order chain then runs in lanes 0..15, the other quarters brought over by permlane swaps
__device__ __forceinline__ double lane_from(double x, int q) {  // lane v < 16: x of lane v + 16 q
  unsigned int l = lo32(x), h = hi32(x);
  if (q & 2) {
    l = __builtin_amdgcn_permlane32_swap(l, l, false, false)[1];
    h = __builtin_amdgcn_permlane32_swap(h, h, false, false)[1];
  }
  if (q & 1) {
    l = __builtin_amdgcn_permlane16_swap(l, l, false, false)[1];
    h = __builtin_amdgcn_permlane16_swap(h, h, false, false)[1];
  }
  return mk64(l, h);
}

__device__ __forceinline__ bool super_sum_tagged(const unsigned long long* __restrict__ tpart, int sj, int nch,
                                                 int lane, unsigned int rstamp, const PassCmd* cmd, unsigned int cur,
                                                 unsigned long long limit, double& a, bool cmd_host = true) {
  const int c0 = sj * kSuperChunks, nin = min(kSuperChunks, nch - c0);
  const int v = lane & 15, qb = 8 * (lane >> 4);
  const unsigned long long t0 = wall_clock64();
  double t[8];
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const unsigned long long* w = tpart + static_cast<size_t>(c0 + min(qb + q, nin - 1)) * 32 + 2 * v;
      const unsigned long long lo = ld_sc1_u64(w), hi = ld_sc1_u64(w + 1);
      ok = ok && static_cast<unsigned int>(lo >> 32) == rstamp && static_cast<unsigned int>(hi >> 32) == rstamp;
      t[q] = mk64(static_cast<unsigned int>(lo), static_cast<unsigned int>(hi));
    }
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
    if (cmd) {
      unsigned long long c[16];
      if (cmd_host) read_cmd<true>(cmd, c);
      else read_cmd<false>(cmd, c);
      const unsigned int st = __builtin_amdgcn_readfirstlane(static_cast<unsigned int>(c[0] >> 32));
      if (static_cast<int>(st - cur) > 0) return false;  // a newer command: the host took the pass over
    }
    if (wall_clock64() - t0 > limit) return false;
    __builtin_amdgcn_s_sleep(4);
  }
  // chunk order: a = t_0 + t_1 + ... + t_(nin-1), chunks 8k .. 8k + 7 from lane v + 16 k
  a = t[0];
#pragma unroll
  for (int q = 1; q < 8; ++q)
    if (q < nin) a = a + t[q];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double x = lane_from(t[q], k);
      if (8 * k + q < nin) a = a + x;
    }
  }
  return true;
}

// After a wave stored all its chunk partials (chunks w0, w0 + nw, ...; reverse & 1: counted from
// the back): tickets, the supers it completes, and -- for the wave completing the last super -- the
// total into `out` and `seq` into done_flag.  Returns true on that finishing wave.
// host_rows (nullable, mapped host memory -- private, or a node-wide shared segment at this rank's
// first super -- 32 words per super, already offset to this pass's parity buffer): each super
// partial goes straight to the host as one 256-byte store of stamped halves ((rstamp << 32) |
// 32-bit half, value v in words 2v (low) and 2v + 1 (high)); the host takes the total in
// wave_total's order, so there is no global ticket, device total or completion flag on the pass's
// critical path (returns false).  chain (timing form only): after its row, each super wave also
// takes a global ticket (modulo the super count) and the wave completing the last super returns
// true, to forward the next command.
__device__ __forceinline__ bool wave_tickets(int w0, int nw, int nch, int reverse, unsigned int* __restrict__ tickets,
                                             const double* __restrict__ partial, double* __restrict__ spart,
                                             double* __restrict__ out, unsigned long long* done_flag,
                                             unsigned long long seq, int lane,
                                             unsigned long long* host_rows = nullptr, bool chain = false,
                                             unsigned int rstamp = 0) {
  const int nsup = (nch + kSuperChunks - 1) / kSuperChunks;
  // tickets, once per wave after all of its chunks (a per-chunk drain + atomic round trip cost
  // ~60 us per pass at 256 blocks): lane k takes the super of the wave's k-th chunk
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int nmine = (nch - w0 + nw - 1) / nw;  // <= 64: the grid has >= nch / 64 waves
  int last = 0;
  if (lane < nmine) {
    const int w = w0 + lane * nw;
    const int j = (reverse & 1) ? nch - 1 - w : w;
    const int sj = j / kSuperChunks, nin = min(kSuperChunks, nch - sj * kSuperChunks);
    const unsigned old = __hip_atomic_fetch_add(tickets + sj, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // host-row mode never re-arms a ticket (a reset racing the host's next command is avoided by
    // construction): every pass adds exactly nin to each super's counter, zeroed at server launch
    last = (host_rows ? old % static_cast<unsigned>(nin) : old) == static_cast<unsigned>(nin - 1) ? 1 : 0;
  }
  unsigned long long done = __ballot(last);
  bool fin = false;
  while (done) {
    // this wave completed super sj: its partial (chunk order), then the global ticket
    const int k = __builtin_ctzll(done);
    done &= done - 1;
    const int w = w0 + k * nw;
    const int j = (reverse & 1) ? nch - 1 - w : w;
    const int sj = j / kSuperChunks, cfirst = sj * kSuperChunks, nin = min(kSuperChunks, nch - cfirst);
    double a = 0.0;
    if (lane < kRedVals) {
      // all kSuperChunks loads in flight at once (a runtime-bounded loop issued them one round
      // trip at a time), then the chunk-order sum
      double t[kSuperChunks];
#pragma unroll
      for (int q = 0; q < kSuperChunks; ++q)
        t[q] = ld_sc1(partial + static_cast<size_t>(cfirst + min(q, nin - 1)) * kRedVals + lane);
      a = t[0];
#pragma unroll
      for (int q = 1; q < kSuperChunks; ++q)
        if (q < nin) a = a + t[q];
      if (!host_rows) st_sc1(spart + static_cast<size_t>(sj) * kRedVals + lane, a);
    }
    if (host_rows) {
      // lane l < 32: half l & 1 of value l >> 1, stamped; one 256-byte store per super
      const long long bits = __double_as_longlong(__shfl(a, lane >> 1, 64));
      const unsigned int half = static_cast<unsigned int>((lane & 1) ? (bits >> 32) : bits);
      // system-coherent write-through (sc0 sc1): a plain store to mapped host memory may sit in the
      // L2 until something releases it; the 32 lanes' 8-byte words leave as one 256-byte burst
      if (lane < 32) {
        const unsigned long long w = (static_cast<unsigned long long>(rstamp) << 32) | half;
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(host_rows + static_cast<size_t>(sj) * 32 + lane),
                     "v"(w)
                     : "memory");
      }
      if (chain) {
        int lastc = 0;
        if (lane == 0)
          lastc = __hip_atomic_fetch_add(tickets + nsup, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) %
                          static_cast<unsigned>(nsup) == static_cast<unsigned>(nsup - 1) ? 1 : 0;
        if (__shfl(lastc, 0, 64)) fin = true;
      }
      continue;
    }
    int lastg = 0;
    if (lane == 0) {
      __hip_atomic_store(tickets + sj, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lastg = __hip_atomic_fetch_add(tickets + nsup, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                      static_cast<unsigned>(nsup - 1) ? 1 : 0;
    }
    if (!__shfl(lastg, 0, 64)) continue;
    // every super is stored: the total (single rank; with out == nullptr the supers are the result)
    if (out) wave_total<kRedVals, true>(spart, nsup, nsup, 1, 0, out);
    fin = true;
    if (lane == 0) {
      __hip_atomic_store(tickets + nsup, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (done_flag && out) {
        // lane 0 wrote every out[v]; once they are drained, publish the pass number to the host
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(done_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  return fin;
}

// Objective pass over the compacted streams: 4 correspondences per thread-iteration, every load
// 16 bytes per lane (float4 of 4 coordinates, double2 of 2 matrix entries).
// kGated (fdf_soa_gated_kernel): the pass is launched BEFORE the host knows its state.  Every
// block's thread 0 polls the host-written command block (pinned, mapped, system-scope acquire)
// until it carries this pass's sequence number, then the block takes A / direction from it -- or
// returns at once on a cancel command (or after `timeout` wall-clock ticks: every wave reaches
// an exit).  The host pre-launches pass k + 1 while pass k runs, so the next pass is resident
// when the host's BFGS step publishes x_{k+1}: no launch latency between consecutive passes.
// host_rows (nullable): the launched pass writes its super partials as stamped host rows (stamp
// rstamp, tickets counted modulo the supers' sizes) instead of a device total -- the form of the
// server's passes, used when a server pass is taken over (missed deadline) or cannot run.
template <bool kGated>
__device__ __forceinline__ void fdf_soa_body(CorrSoA c, const uint32_t* __restrict__ ccnt, int nch, Xf34 A,
                                             double* __restrict__ partial, double* __restrict__ spart,
                                             unsigned int* __restrict__ tickets, double* __restrict__ out,
                                             int reverse, unsigned long long* done_flag,
                                             unsigned long long seq, const PassCmd* cmd, PassCmd* mail,
                                             unsigned long long timeout, unsigned long long* gtrace,
                                             int host_pollers, unsigned long long* host_rows, unsigned int rstamp) {
  if constexpr (kGated) {
    if (!pass_gate(seq, cmd, mail, timeout, gtrace, host_pollers, A, reverse, rstamp)) return;
  }
  // persistent waves over the shard's chunks (reverse: back to front, so the tail of the previous
  // pass, still in the 256 MiB Infinity Cache, is consumed first)
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * (blockDim.x >> 6);
  const int w0 = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
  for (int w = w0; w < nch; w += nw) {
    const int j = (reverse & 1) ? nch - 1 - w : w;
    double acc[kRedVals];
#pragma unroll
    for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
    const uint32_t g1 = chunk_g1(ccnt, j);
    for (uint32_t i = chunk_g0(j) + lane; i < g1; i += 64) {
      CorrGroup g;
      load_group(c, i, g);
      fdf_group(A, g, acc);
    }
    if (reverse & 2) {  // timing diagnostics only (MGICP_FDF_DIAG): stream, no reduction
      if (acc[0] == 12345.0) partial[j] = acc[1];
      continue;
    }
    if (reverse & 4) {  // timing diagnostics only: chunk partials, no tickets
#pragma unroll
      for (int v = 0; v < 13; ++v) acc[v] = wave_sum(acc[v]);
      if (lane == 0)
        for (int v = 0; v < 13; ++v) partial[static_cast<size_t>(j) * kRedVals + v] = acc[v];
      continue;
    }
    chunk_store(j, acc, ccnt, partial, lane);
  }
  if (w0 >= nch || (reverse & 6)) return;
  wave_tickets(w0, nw, nch, reverse, tickets, partial, spart, out, done_flag, seq, lane, host_rows, false, rstamp);
}

// ---- the resident pass server --------------------------------------------------------------
// All objective passes of one BFGS run read the SAME compacted streams (72 B per correspondence,
// 360 MB at C4).  The server is ONE launch per BFGS run with one 4-wave block per CU (1 wave per
// SIMD, up to 512 VGPR+AGPR per lane; a plain launch after an occupancy check -- its blocks wait on
// the host's commands, not on each other, and a block that is not resident when the host gives up
// on a pass exits at its first gate, see pass_gate): each wave keeps its first chunk (4 groups per
// lane, 288 dwords) in registers and half of its second chunk (2 groups per lane, 36 KiB per wave,
// 144 KiB per CU) in LDS for the whole run, and streams only the rest from HBM / Infinity Cache.
// Between passes every block waits at the gate for the host's next command (pass_gate); the
// chunk -> wave assignment, the lanes' element order and the reduction tree are those of
// fdf_soa_body with reverse = 0, so every pass gives bit-identical sums.  bench_passes > 0 (timing
// only): run that many passes of state A back to back, the finishing wave forwarding the next
// command itself.  ptimes (nullable): per pass, block 0's gate exit and the finish (wall clock).
// A/B (profiles/r02/ab_server): the 31 % of the bytes this keeps on chip buy less than expected,
// because one wave per SIMD keeps few loads in flight; software-pipelining the streamed groups in
// registers (2-3 resident groups, spills) or through an LDS-DMA ring (3 resident groups) measured
// 67-77 us per pass against ~65 us for this form and ~66-70 us for launched passes.
// Two shapes (env MGICP_SRV_WAVES): 4 waves per CU (1 per SIMD, 512 VGPR+AGPR) holding a whole chunk
// in registers + 2 groups in LDS (31 % of C4's bytes on chip), or 8 waves per CU (2 per SIMD, 256
// registers) holding 1 group in registers + 1 in LDS each (21 %) with two waves per SIMD to
// overlap the streamed loads.
template <int kWaves>
struct SrvShape;
template <>
struct SrvShape<4> {
  static constexpr int kReg = 4, kLds = 2;  // kReg = 4: the LDS groups are chunk 1's first kLds
};
template <>
struct SrvShape<8> {
  static constexpr int kReg = 1, kLds = 1;  // kReg < 4: the LDS groups follow in chunk 0
};

// kBench: the timing instantiation (bench_passes > 0) -- a symbol of its own, so a rocprofv3 kernel
// trace separates it from the servers of the aligns (its duration / bench_passes = one pass)
// host_rows: parity-0 row buffer at this rank's first super, rows_stride words to the parity-1
// buffer (a pass writes into buffer rstamp & 1).  stall_pass >= 0 (tests only): the last block skips
// that pass (relative to seq0) entirely, so the host must take it over.
template <bool kBench, int kWaves>
__global__ __launch_bounds__(64 * kWaves, 1) void fdf_server_kernel(
    CorrSoA c, const uint32_t* __restrict__ ccnt, int nch, double* __restrict__ partial, double* __restrict__ spart, unsigned int* __restrict__ tickets,
    double* __restrict__ out, unsigned long long* done_flag, unsigned long long seq0, const PassCmd* cmd,
    PassCmd* mail, unsigned long long timeout, unsigned long long* ptimes, int bench_passes, Xf34 Abench,
    unsigned long long* host_rows, size_t rows_stride, int pollers, int stall_pass,
    unsigned long long* __restrict__ tpart, PeerRows peers) {
  constexpr int kR = SrvShape<kWaves>::kReg, kL = SrvShape<kWaves>::kLds;
  static_assert(kR <= 4 && (kR == 4 || kR + kL <= 4), "resident groups: chunk 0, then chunk 1 only after a full chunk 0");
  __shared__ float4 lf[kWaves][kL][6][64];
  __shared__ double2 ld[kWaves][kL][12][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = gridDim.x * kWaves;
  const int w0 = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x * kWaves + wid));
  // resident data: groups [0, kR) of chunk w0 in registers; kLds groups in LDS -- chunk w1's first
  // ones when chunk w0 is whole in registers, else chunk w0's next ones (each lane reads back only
  // its own slots, so no barrier is needed)
  const int w1 = w0 + nw;
  CorrGroup R[kR];
  uint32_t rb = 0, re = 0, lb = 0, le = 0;
  if (w0 < nch) {
    rb = chunk_g0(w0);
    re = chunk_g1(ccnt, w0);
  }
  if (kR == 4 && w1 < nch) {
    lb = chunk_g0(w1);
    le = chunk_g1(ccnt, w1);
  } else if (kR < 4) {
    lb = rb + 64 * kR;
    le = re;
  }
#pragma unroll
  for (int k = 0; k < kR; ++k)
    if (rb + lane + 64 * k < re) load_group(c, rb + lane + 64 * k, R[k]);
#pragma unroll
  for (int k = 0; k < kL; ++k) {
    if (lb + lane + 64 * k < le) {
      CorrGroup g;
      load_group(c, lb + lane + 64 * k, g);
#pragma unroll
      for (int q = 0; q < 6; ++q) lf[wid][k][q][lane] = g.f[q];
#pragma unroll
      for (int q = 0; q < 12; ++q) ld[wid][k][q][lane] = g.d[q];
    }
  }
  auto lds_group = [&](int k, const Xf34& A, double (&acc)[kRedVals]) {
    CorrGroup g;
#pragma unroll
    for (int q = 0; q < 6; ++q) g.f[q] = lf[wid][k][q][lane];
#pragma unroll
    for (int q = 0; q < 12; ++q) g.d[q] = ld[wid][k][q][lane];
    fdf_group(A, g, acc);
  };
  // pollers: blocks [0, pollers) read the command block themselves (system-coherent loads); the
  // others poll the mailbox block 0 forwards to.  1 = the host's pinned copy (PCIe reads by one
  // block); gridDim = a command block the host stores straight into device memory (BAR)
  const int host_pollers = kBench ? 0 : pollers;
  for (unsigned long long seq = seq0;; ++seq) {
    Xf34 A = Abench;
    int rev = 0;
    // the timing form stamps rows with seq | 2^31 (align passes stamp their pass index, < 2^31)
    unsigned int rstamp = static_cast<unsigned int>(seq) | 0x80000000u;
    if (!(kBench && seq == seq0) && !pass_gate(seq, cmd, mail, timeout, nullptr, host_pollers, A, rev, rstamp))
      return;
    if (stall_pass >= 0 && seq - seq0 == static_cast<unsigned long long>(stall_pass) &&
        blockIdx.x == gridDim.x - 1)
      continue;  // tests: withhold this block's share of the pass
    unsigned long long* rows = host_rows ? host_rows + (rstamp & 1u) * rows_stride : nullptr;
    if (ptimes && blockIdx.x == 0 && threadIdx.x == 0) ptimes[2 * (seq & 1023)] = wall_clock64();
    // r03: with host rows (and at most one super per wave) the chunk partials are stamped words and
    // wave s reduces super s once all its chunks carry this pass's stamp: no chunk tickets, no drain
    const int nsup = (nch + kSuperChunks - 1) / kSuperChunks;
    const bool tagged = tpart != nullptr && rows != nullptr && nsup <= nw;
    auto store = [&](int j, double (&acc)[kRedVals]) {
      if (tagged) chunk_store_tagged(j, acc, ccnt, tpart, lane, rstamp);
      else chunk_store(j, acc, ccnt, partial, lane);
    };
    // odd waves take their streamed chunks first and their resident ones last, even waves the
    // reverse: the CU's memory pipe is never left idle while all its waves compute resident data
    // (the order of a wave's chunks does not change any sum)
    // the wave's streamed chunks [c0, c1) (chunks w1 + nw, w1 + 2 nw, ...)
    auto stream_chunks = [&](int c0, int c1) {
      for (int w = w1 + nw * (1 + c0); w < nch && c0 < c1; w += nw, ++c0) {
        double acc[kRedVals];
#pragma unroll
        for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
        const uint32_t g1 = chunk_g1(ccnt, w);
        for (uint32_t i = chunk_g0(w) + lane; i < g1; i += 64) {
          CorrGroup g;
          load_group(c, i, g);
          fdf_group(A, g, acc);
        }
        store(w, acc);
      }
    };
    // stagger: wave wid computes its resident chunks after split(wid) of its streamed ones, so the
    // CU's memory pipe is never left idle while all its waves compute resident data (the order of
    // a wave's chunks does not change any sum).  MGICP_SRV_STAGGER 1: odd waves last, 2: quarters
    const int nst = w1 + nw < nch ? (nch - w1 - 1) / nw : 0;
    const int split = MGICP_SRV_STAGGER == 2 ? (wid * nst + kWaves / 2) / kWaves
                                             : (MGICP_SRV_STAGGER == 1 && (wid & 1) ? nst : 0);
    stream_chunks(0, split);
    if (w0 < nch) {
      double acc[kRedVals];
#pragma unroll
      for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
#pragma unroll
      for (int k = 0; k < kR; ++k)
        if (rb + lane + 64 * k < re) fdf_group(A, R[k], acc);
      if (kR < 4) {
#pragma unroll
        for (int k = 0; k < kL; ++k)
          if (lb + lane + 64 * k < le) lds_group(k, A, acc);
        for (uint32_t i = rb + lane + 64 * (kR + kL); i < re; i += 64) {
          CorrGroup g;
          load_group(c, i, g);
          fdf_group(A, g, acc);
        }
      }
      store(w0, acc);
    }
    if (w1 < nch) {
      double acc[kRedVals];
#pragma unroll
      for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
      uint32_t i0 = chunk_g0(w1) + lane;
      if (kR == 4) {
#pragma unroll
        for (int k = 0; k < kL; ++k)
          if (lb + lane + 64 * k < le) lds_group(k, A, acc);
        i0 = lb + lane + 64 * kL;
      }
      const uint32_t g1 = chunk_g1(ccnt, w1);
      for (uint32_t i = i0; i < g1; i += 64) {
        CorrGroup g;
        load_group(c, i, g);
        fdf_group(A, g, acc);
      }
      store(w1, acc);
    }
    stream_chunks(split, nst);
    if (w0 >= nch) continue;
    // the timing form writes host rows too when given them (chained on the device by a global
    // ticket), so it times the pass the aligns run
    bool fin = false;
    if (tagged) {
      if (w0 < nsup) {
        double a = 0.0;
        // a newer command means the host took this pass over: with the BAR command block every block
        // polls it; otherwise the mailbox block 0 forwards the host's commands to (without
        // a watch the reducers of a cancelled server spun until their timeout)
        const bool bar_cmd = host_pollers >= static_cast<int>(gridDim.x);
        const PassCmd* watch = kBench ? nullptr : (bar_cmd ? cmd : mail);
        if (super_sum_tagged(tpart, w0, nch, lane, rstamp, watch, static_cast<unsigned int>(seq), timeout >> 3, a,
                             bar_cmd)) {
          // the super's row, as wave_tickets writes it: lane l < 32 stores half l & 1 of value l >> 1
          const long long bits = __double_as_longlong(__shfl(a, lane >> 1, 64));
          const unsigned int half = static_cast<unsigned int>((lane & 1) ? (bits >> 32) : bits);
          if (lane < 32) {
            const unsigned long long w = (static_cast<unsigned long long>(rstamp) << 32) | half;
            asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(rows + static_cast<size_t>(w0) * 32 + lane),
                         "v"(w)
                         : "memory");
            // r05 xGMI: the same row into every other rank's exchange buffer (peer device memory)
            for (int r = 0; r < peers.n; ++r) {
              unsigned long long* pr = peers.p[r] + (rstamp & 1u) * rows_stride + static_cast<size_t>(w0) * 32 + lane;
              asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(pr), "v"(w) : "memory");
            }
          }
          if (kBench) {  // timing form: the reducer of the last super forwards the next command
            int lastc = 0;
            if (lane == 0)
              lastc = __hip_atomic_fetch_add(tickets + nsup, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) %
                              static_cast<unsigned>(nsup) == static_cast<unsigned>(nsup - 1) ? 1 : 0;
            fin = __shfl(lastc, 0, 64) != 0;
          }
        }
      }
    } else {
      fin = wave_tickets(w0, nw, nch, 0, tickets, partial, spart, out, done_flag, seq, lane, rows, kBench && rows,
                         rstamp);
    }
    if (fin && lane == 0) {
      if (ptimes) ptimes[2 * (seq & 1023) + 1] = wall_clock64();
      if (kBench) {
        // the next bench pass (or a cancel after the last), forwarded like block 0 forwards the host's
        unsigned long long v[16] = {};
        const bool more = seq + 1 < seq0 + static_cast<unsigned long long>(bench_passes);
        const unsigned int s1 = static_cast<unsigned int>(seq + 1);
        const unsigned long long st = static_cast<unsigned long long>(s1) << 32;
#pragma unroll
        for (int i = 0; i < kCmdWords; ++i)
          v[i] = st | (i < 12 ? (more ? __float_as_uint(Abench.m[i]) : 0u)
                              : (i == 12 ? (more ? kPassRun : kPassCancel) : (i == 14 ? (s1 | 0x80000000u) : 0u)));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        write_mail(mail, v);
      }
    }
  }
}

__global__ __launch_bounds__(256) void fdf_soa_kernel(CorrSoA c, const uint32_t* __restrict__ ccnt, int nch, Xf34 A,
                                                      double* __restrict__ partial, double* __restrict__ spart,
                                                      unsigned int* __restrict__ tickets, double* __restrict__ out,
                                                      int reverse, unsigned long long* done_flag,
                                                      unsigned long long seq, unsigned long long* host_rows,
                                                      unsigned int rstamp) {
  fdf_soa_body<false>(c, ccnt, nch, A, partial, spart, tickets, out, reverse, done_flag, seq, nullptr,
                      nullptr, 0, nullptr, 0, host_rows, rstamp);
}

__global__ __launch_bounds__(256) void fdf_soa_gated_kernel(CorrSoA c, const uint32_t* __restrict__ ccnt, int nch,
                                                            double* __restrict__ partial, double* __restrict__ spart,
                                                            unsigned int* __restrict__ tickets,
                                                            double* __restrict__ out, unsigned long long* done_flag,
                                                            unsigned long long seq, const PassCmd* cmd,
                                                            PassCmd* mail, unsigned long long timeout,
                                                            unsigned long long* gtrace, int host_pollers) {
  fdf_soa_body<true>(c, ccnt, nch, Xf34{}, partial, spart, tickets, out, 0, done_flag, seq, cmd, mail,
                     timeout, gtrace, host_pollers, nullptr, 0);
}

// ------------------------------------------------------------------------------------
// Gauss-Newton moment pass (MGICP_SOLVER_GN)
// ------------------------------------------------------------------------------------
// For a fixed correspondence set the GICP objective is an exact quadratic in A = [R | t]
// (DESIGN.md "The moment form"), so ONE pass per outer iteration collects everything the host
// Gauss-Newton solve needs: with the correspondence transform T0, r0 = fl(fl(T0 s) - q) and
// w = (s - c, 1),
//   [0] sum r0' M r0   [1 + 4a + k] sum (M r0)_a w_k   [13 + 10p + q] sum M_p (w w')_q   [73] count
// (p over the 6 upper-triangle entries of M, q over the 10 of w w').  The Mahalanobis matrix is
// computed on the fly (no compaction, no SoA streams): 136 B read per source point of the shard.
// One wave per chunk of the shard (chunk partials of the fixed reduction tree); lane l takes the
// chunk's positions l, l + 64, ... in order.
__global__ __launch_bounds__(256) void gn_moments_kernel(
    const float4* __restrict__ src, const float4* __restrict__ tpts, Cov3 cov_s, Cov3 cov_t,
    Rot33d R, Xf34 T0, double cx, double cy, double cz, const uint32_t* __restrict__ nn_pos,
    const uint32_t* __restrict__ flags, size_t p0, size_t p1, double* __restrict__ partial) {
  const size_t ch = (static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const size_t c0 = p0 + ch * kChunkPts;
  if (c0 >= p1) return;
  const size_t c1 = min(c0 + kChunkPts, p1);
  double acc[kMomVals];
#pragma unroll
  for (int v = 0; v < kMomVals; ++v) acc[v] = 0.0;
  for (size_t p = c0 + (threadIdx.x & 63); p < c1; p += 64) {
    if (!flags[p - p0]) continue;
    const uint32_t j = nn_pos[p - p0];
    const float4 s = src[p], t = tpts[j];
    double C1[3][3], C2[3][3], m6[6];
    load_cov(cov_s, p, C1);
    load_cov(cov_t, j, C2);
    mahalanobis(R, C1, C2, m6);
    float px, py, pz;
    xform(T0, s.x, s.y, s.z, px, py, pz);
    const double r0 = static_cast<double>(px - t.x);
    const double r1 = static_cast<double>(py - t.y);
    const double r2 = static_cast<double>(pz - t.z);
    double mr[3];
    mr[0] = m6[0] * r0; mr[0] = mr[0] + m6[1] * r1; mr[0] = mr[0] + m6[2] * r2;
    mr[1] = m6[1] * r0; mr[1] = mr[1] + m6[3] * r1; mr[1] = mr[1] + m6[4] * r2;
    mr[2] = m6[2] * r0; mr[2] = mr[2] + m6[4] * r1; mr[2] = mr[2] + m6[5] * r2;
    double d = r0 * mr[0]; d = d + r1 * mr[1]; d = d + r2 * mr[2];
    acc[0] += d;
    const double w[4] = {static_cast<double>(s.x) - cx, static_cast<double>(s.y) - cy,
                         static_cast<double>(s.z) - cz, 1.0};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[1 + 4 * a + k] += mr[a] * w[k];
    const double ww[10] = {w[0] * w[0], w[0] * w[1], w[0] * w[2], w[0],        w[1] * w[1],
                           w[1] * w[2], w[1],        w[2] * w[2], w[2],        1.0};
#pragma unroll
    for (int pp = 0; pp < 6; ++pp)
#pragma unroll
      for (int q = 0; q < 10; ++q) acc[13 + 10 * pp + q] += m6[pp] * ww[q];
    acc[73] += 1.0;
  }
#pragma unroll
  for (int v = 0; v < kMomVals; ++v) acc[v] = wave_sum(acc[v]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int v = 0; v < kMomVals; ++v) partial[ch * kMomVals + v] = acc[v];
  }
}

// n doubles of device memory -> mapped host memory, then `seq` into the host-polled completion
// word with a system-scope release (multi-GPU passes: runs after the RCCL all-reduce)
__global__ void publish_kernel(const double* __restrict__ in, int n, double* out,
                               unsigned long long* flag, unsigned long long seq) {
  if (threadIdx.x < n) out[threadIdx.x] = in[threadIdx.x];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave per chunk of the shard, like gn_moments_kernel: chunk partials [0] sum d2, [13] count
__global__ __launch_bounds__(256) void fitness_kernel(GridView tg, const float4* __restrict__ src,
                                                      size_t p0, size_t p1, Xf34 T,
                                                      double max_range,
                                                      double* __restrict__ partial) {
  const size_t ch = (static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const size_t c0 = p0 + ch * kChunkPts;
  if (c0 >= p1) return;
  const size_t c1 = min(c0 + kChunkPts, p1);
  double acc[kRedVals];
#pragma unroll
  for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
  for (size_t p = c0 + (threadIdx.x & 63); p < c1; p += 64) {
    const float4 s = src[p];
    float qx, qy, qz;
    xform(T, s.x, s.y, s.z, qx, qy, qz);
    NnVisitor vis;
    vis.init(qx, qy, qz, INFINITY);
    if (tg.boxes) ring_search_boxed(tg, qx, qy, qz, vis);
    else ring_search(tg, qx, qy, qz, vis);
    if (vis.best != ~0ull) {
      const float d2 = __uint_as_float(static_cast<uint32_t>(vis.best >> 32));
      if (static_cast<double>(d2) <= max_range) {
        acc[0] += d2;
        acc[13] += 1.0;
      }
    }
  }
  acc[0] = wave_sum(acc[0]);
  acc[13] = wave_sum(acc[13]);
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int v = 0; v < kRedVals; ++v) partial[ch * kRedVals + v] = acc[v];
  }
}

// Utils::computeCloudResolution: sqrt of the 2nd-nearest (self is 1st) float d2, summed in fp64
__global__ __launch_bounds__(256) void resolution_kernel(GridView g, size_t n,
                                                         double* __restrict__ partial) {
  double acc[kRedVals];
#pragma unroll
  for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
  const size_t p = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p < n && n >= 2) {
    const float4 q = g.pts[p];
    KnnVisitor<2> vis;
    vis.init(q.x, q.y, q.z);
    ring_search(g, q.x, q.y, q.z, vis);
    const float d2 = __uint_as_float(static_cast<uint32_t>(vis.key[1] >> 32));
    acc[0] = static_cast<double>(sqrtf(d2));
    acc[13] = 1.0;
  }
  block_reduce_store(acc, partial + static_cast<size_t>(blockIdx.x) * kRedVals);
}

// NormalEstimation's NaN-normal test: fewer than `need` radius neighbours (self included)
__global__ void radius_keep_kernel(GridView g, size_t n, float r2, int need,
                                   unsigned char* __restrict__ keep_orig) {
  const size_t p = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float4 q = g.pts[p];
  RadiusCountVisitor vis{q.x, q.y, q.z, r2, need, 0};
  ring_search(g, q.x, q.y, q.z, vis);
  keep_orig[__float_as_uint(q.w)] = vis.count >= need ? 1 : 0;
}

__global__ __launch_bounds__(256) void reduce_finish_kernel(const double* __restrict__ partial,
                                                            int nb, double* __restrict__ out) {
  double acc[kRedVals];
#pragma unroll
  for (int v = 0; v < kRedVals; ++v) acc[v] = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
#pragma unroll
    for (int v = 0; v < kRedVals; ++v) acc[v] += partial[static_cast<size_t>(b) * kRedVals + v];
  }
  block_reduce_store(acc, out);
}

// ------------------------------------------------------------------------------------
// FOD-side callers of the GICP path
// ------------------------------------------------------------------------------------
// 1 for finite points (cloud compaction before a grid build: KdTreeFLANN skips NaN points)
__global__ void finite_flags_kernel(const float4* __restrict__ p, size_t n, uint32_t* __restrict__ flags) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i > n) return;
  flags[i] = (i < n && isfinite(p[i].x) && isfinite(p[i].y) && isfinite(p[i].z)) ? 1u : 0u;
}

__global__ void scatter_flagged_kernel(const float4* __restrict__ in, const uint32_t* __restrict__ flags,
                                       const uint32_t* __restrict__ pos, size_t n, float4* __restrict__ out) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && flags[i]) out[pos[i]] = in[i];
}

// "is there a point with float d2 <= thr?" -- stops at the first one (exact: the ring bound
// proves absence before giving up)
struct WithinVisitor {
  static constexpr bool kNearFirst = false;
  static constexpr bool kRingCap = false;
  float qx, qy, qz;
  double thr;
  float thr_f;  // float upper bound of thr (pruning radius)
  bool found;
  __device__ __forceinline__ bool done(float Ls) const {
    if (found) return true;
    return Ls > 0.f && static_cast<double>(Ls) * static_cast<double>(Ls) > thr;
  }
  __device__ __forceinline__ float prune2() const { return found ? -1.f : thr_f; }
  __device__ __forceinline__ void range(const GridView& g, uint32_t a, uint32_t b) {
    for (uint32_t j = a; j < b && !found; ++j)
      if (static_cast<double>(dist2(qx, qy, qz, g.pts[j])) <= thr) found = true;
  }
};

// pcl::getPointCloudDifference: keep[i] = 1 iff input point i, transformed by T, is finite and
// its nearest neighbour in the grid has float d2 > thr (src/Filter.cpp:176-189); counts kept points
__global__ __launch_bounds__(256) void segdiff_kernel(GridView g, const float4* __restrict__ in,
                                                      size_t n, Xf34 T, int has_T, double thr,
                                                      unsigned char* __restrict__ keep,
                                                      unsigned int* __restrict__ count) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  bool k = false;
  if (i < n) {
    const float4 p = in[i];
    float qx = p.x, qy = p.y, qz = p.z;
    if (has_T) xform(T, p.x, p.y, p.z, qx, qy, qz);
    if (isfinite(qx) && isfinite(qy) && isfinite(qz)) {
      WithinVisitor vis{qx, qy, qz, thr, thr >= 3.0e38 ? INFINITY : __double2float_ru(thr), false};
      ring_search(g, qx, qy, qz, vis);
      k = !vis.found;
    }
    keep[i] = k ? 1 : 0;
  }
  // one integer atomic per wave (order-independent: the count is exact)
  const unsigned long long ballot = __ballot(k);
  if ((threadIdx.x & 63) == 0 && ballot) atomicAdd(count, static_cast<unsigned int>(__popcll(ballot)));
}

// VoxelGrid leaf index of every point (voxel_grid.hpp applyFilter, first pass); non-finite
// points get the sentinel 0xffffffff and sort behind every leaf
__global__ void voxel_key_kernel(const float4* __restrict__ p, size_t n, float ix, float iy, float iz,
                                 int bx, int by, int bz, int mul1, int mul2, uint32_t* __restrict__ keys) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 q = p[i];
  if (!isfinite(q.x) || !isfinite(q.y) || !isfinite(q.z)) {
    keys[i] = 0xffffffffu;
    return;
  }
  const int i0 = static_cast<int>(floorf(q.x * ix) - static_cast<float>(bx));
  const int i1 = static_cast<int>(floorf(q.y * iy) - static_cast<float>(by));
  const int i2 = static_cast<int>(floorf(q.z * iz) - static_cast<float>(bz));
  keys[i] = static_cast<uint32_t>(i0 + i1 * mul1 + i2 * mul2);
}

// run heads of the sorted leaf keys (sentinel excluded); flags[n] = 0 closes the scan
__global__ void voxel_head_kernel(const uint32_t* __restrict__ keys, size_t n, uint32_t* __restrict__ flags) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    flags[n] = 0;
    return;
  }
  const uint32_t k = keys[i];
  flags[i] = (k != 0xffffffffu && (i == 0 || keys[i - 1] != k)) ? 1u : 0u;
}

// CentroidPoint<PointXYZRGB> of one leaf per head thread, summed sequentially in the sorted
// order (stable in the input index): xyz fp32 sums / float(count); r, g, b, a float sums,
// truncated after the division.  out[v] = (cx, cy, cz, bit_cast(count)).
__global__ void voxel_centroid_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ perm,
                                      const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos,
                                      size_t n, const float4* __restrict__ pts, const uint32_t* __restrict__ rgba,
                                      float4* __restrict__ out, uint32_t* __restrict__ out_rgba) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n || !flags[i]) return;
  const uint32_t k = keys[i];
  float sx = 0.f, sy = 0.f, sz = 0.f, r = 0.f, g = 0.f, b = 0.f, a = 0.f;
  size_t l = i;
  for (; l < n && keys[l] == k; ++l) {
    const uint32_t j = perm[l];
    const float4 q = pts[j];
    sx = sx + q.x;
    sy = sy + q.y;
    sz = sz + q.z;
    if (rgba) {
      const uint32_t c = rgba[j];
      b = b + static_cast<float>(c & 0xffu);
      g = g + static_cast<float>((c >> 8) & 0xffu);
      r = r + static_cast<float>((c >> 16) & 0xffu);
      a = a + static_cast<float>(c >> 24);
    }
  }
  const uint32_t cnt = static_cast<uint32_t>(l - i);
  const float fc = static_cast<float>(cnt);
  const uint32_t v = pos[i];
  out[v] = make_float4(sx / fc, sy / fc, sz / fc, __uint_as_float(cnt));
  if (rgba)
    out_rgba[v] = (static_cast<uint32_t>(a / fc) << 24) | (static_cast<uint32_t>(r / fc) << 16) |
                  (static_cast<uint32_t>(g / fc) << 8) | static_cast<uint32_t>(b / fc);
}

// min_points_per_voxel: 1 for leaves with at least `need` points (flags[nv] = 0)
__global__ void voxel_minpts_kernel(const float4* __restrict__ vox, size_t nv, uint32_t need,
                                    uint32_t* __restrict__ flags) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i > nv) return;
  flags[i] = (i < nv && __float_as_uint(vox[i].w) >= need) ? 1u : 0u;
}

__global__ void scatter_voxels_kernel(const float4* __restrict__ in, const uint32_t* __restrict__ in_rgba,
                                      const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos,
                                      size_t nv, float4* __restrict__ out, uint32_t* __restrict__ out_rgba) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= nv || !flags[i]) return;
  out[pos[i]] = in[i];
  if (in_rgba) out_rgba[pos[i]] = in_rgba[i];
}

// ------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------
static inline unsigned nblk(size_t n, unsigned t = 256) {
  return static_cast<unsigned>((n + t - 1) / t);
}

hipError_t launch_pack_points(const void* raw, size_t n, size_t stride, float4* out,
                              hipStream_t s) {
  if (!n) return hipSuccess;
  pack_points_kernel<<<nblk(n), 256, 0, s>>>(static_cast<const unsigned char*>(raw), n, stride,
                                             out);
  return hipGetLastError();
}

hipError_t launch_bbox(const float4* pts, size_t n, float* partial, int nb, hipStream_t s) {
  bbox_kernel<<<nb, 256, 0, s>>>(pts, n, partial);
  return hipGetLastError();
}

hipError_t launch_cell_hist(const float4* pts, size_t n, float ox, float oy, float oz,
                            float inv_h, int nx, int ny, int nz, uint32_t* counts,
                            uint32_t* keys, hipStream_t s) {
  if (!n) return hipSuccess;
  cell_hist_kernel<<<nblk(n), 256, 0, s>>>(pts, n, ox, oy, oz, inv_h, nx, ny, nz, counts, keys);
  return hipGetLastError();
}

hipError_t launch_cell_sketch(const float4* pts, size_t n, float ox, float oy, float oz, const SketchScales& sc,
                              uint8_t* partial, uint8_t* out, hipStream_t s) {
  constexpr int SR = kSketchScales * kSketchR, kSlices = 32;
  cell_sketch_kernel<<<kSketchBlocks, 256, 0, s>>>(pts, n, ox, oy, oz, sc, partial);
  sketch_merge_kernel<<<dim3((SR + 255) / 256, kSlices), 256, 0, s>>>(partial, 0, kSketchBlocks, nullptr);
  sketch_merge_kernel<<<dim3((SR + 255) / 256, 1), 256, 0, s>>>(partial, kSketchBlocks, kSlices, out);
  return hipGetLastError();
}

size_t cell_start_scratch_bytes(size_t nc) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveScan(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                          static_cast<uint32_t*>(nullptr), hipcub::Max(), 0u,
                                          static_cast<int>(nc + 1));
  return bytes;
}

hipError_t launch_cell_starts(const uint32_t* keys_sorted, size_t n, size_t nc, uint32_t* ends, uint32_t* cell_start,
                              void* scratch, size_t scratch_bytes, hipStream_t s) {
  hipError_t e = hipMemsetAsync(ends, 0, (nc + 1) * sizeof(uint32_t), s);
  if (e != hipSuccess) return e;
  if (n) cell_end_kernel<<<nblk(n), 256, 0, s>>>(keys_sorted, n, ends);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  return hipcub::DeviceScan::ExclusiveScan(scratch, scratch_bytes, static_cast<const uint32_t*>(ends), cell_start,
                                           hipcub::Max(), 0u, static_cast<int>(nc + 1), s);
}

hipError_t launch_gather_sorted(const float4* pts, const uint32_t* perm, size_t n, float4* out,
                                hipStream_t s) {
  if (!n) return hipSuccess;
  gather_sorted_kernel<<<nblk(n), 256, 0, s>>>(pts, perm, n, out);
  return hipGetLastError();
}

hipError_t launch_xform_points(const float4* in, size_t n, Xf34 T, float4* out, hipStream_t s) {
  if (!n) return hipSuccess;
  xform_points_kernel<<<nblk(n), 256, 0, s>>>(in, n, T, out);
  return hipGetLastError();
}

hipError_t launch_empty_map(const uint32_t* cell_start, int nx, int ny, int nz, uint8_t* out,
                            uint8_t* scratch, hipStream_t s, uint32_t* seed, uint32_t* seed_scratch,
                            const GridView* g) {
  const size_t nc = static_cast<size_t>(nx) * ny * nz;
  if (!nc) return hipSuccess;
  uint32_t* s2 = seed ? seed_scratch : nullptr;
  // init -> scratch, then x: scratch -> out, y: out -> scratch, z: scratch -> out (r06: the result lands
  // in `out` / `seed` without the copies of r01-r05)
  empty_init_kernel<<<nblk(nc), 256, 0, s>>>(cell_start, nc, scratch, s2, g ? g->pts : nullptr, nx, ny,
                                             g ? g->ox : 0.f, g ? g->oy : 0.f, g ? g->oz : 0.f, g ? g->h : 0.f);
  auto pass = [&](const uint8_t* in, uint8_t* o, int n, size_t stride, const uint32_t* si, uint32_t* so) {
    const size_t nlines = nc / static_cast<size_t>(n);
    const size_t nt = nlines * static_cast<size_t>((n + kEmptyGroup - 1) / kEmptyGroup);
    empty_pass_kernel<<<nblk(nt), 256, 0, s>>>(in, o, nlines, n, stride, si, so);
  };
  pass(scratch, out, nx, 1, s2, seed);
  pass(out, scratch, ny, static_cast<size_t>(nx), seed, s2);
  pass(scratch, out, nz, static_cast<size_t>(nx) * ny, s2, seed);
  return hipGetLastError();
}

hipError_t launch_cell_boxes(const float4* pts, const uint32_t* cell_start, size_t nc, float4* boxes,
                             hipStream_t s) {
  if (!nc) return hipSuccess;
  cell_box_kernel<<<nblk(nc), 256, 0, s>>>(pts, cell_start, nc, boxes);
  return hipGetLastError();
}

// r05 target cache: *diff |= 1 when the two arrays differ in any bit
__global__ __launch_bounds__(256) void equal_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b, size_t n,
                                                    unsigned int* __restrict__ diff) {
  bool d = false;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const uint4 x = a[i], y = b[i];
    d = d || x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
  }
  if (__builtin_amdgcn_ballot_w64(d) != 0ull && (threadIdx.x & 63) == 0) atomicOr(diff, 1u);
}

hipError_t launch_equal(const float4* a, const float4* b, size_t n, unsigned int* diff, hipStream_t s) {
  hipError_t e = hipMemsetAsync(diff, 0, sizeof(unsigned int), s);
  if (e != hipSuccess || n == 0) return e;
  equal_kernel<<<2048, 256, 0, s>>>(reinterpret_cast<const uint4*>(a), reinterpret_cast<const uint4*>(b), n, diff);
  return hipGetLastError();
}

hipError_t launch_iota(uint32_t* v, size_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  iota_kernel<<<nblk(n), 256, 0, s>>>(v, n);
  return hipGetLastError();
}

// log capacity (entries per lane) of the logged k-NN kernel: K + 28
static int knn_log_cap(int K) { return std::min(K + 28, 128); }

template <int K>
static hipError_t knn_cov_k(const GridView& g, double eps, size_t p0, size_t p1, Cov3 cov,
                            const uint32_t* perm, int k, uint32_t* fb, unsigned int* fb_count, hipStream_t s,
                            int ring_cap, uint8_t* ok, int chain, bool wave_handoff) {
  if (fb) {
    const int cap = knn_log_cap(K);
    knn_cov2_kernel<K><<<nblk(p1 - p0, 64), 64, cap * 64 * sizeof(uint32_t), s>>>(g, eps, p0, p1, cov, perm,
                                                                                 K - k, cap, fb, fb_count, ring_cap,
                                                                                 ok);
    // chain: the hand-off follows at once in stream order, its count read on the device (a grid of
    // `chain` blocks striding over the list)
    if (chain > 0 && wave_handoff) knn_wave_kernel<K><<<chain, 256, 0, s>>>(g, eps, fb, fb_count, 0, k, cov);
    else if (chain > 0) knn_cov_kernel<K><<<chain, 256, 0, s>>>(g, eps, 0, 0, cov, fb, K - k, fb_count);
  } else {
    knn_cov_kernel<K><<<nblk(p1 - p0), 256, 0, s>>>(g, eps, p0, p1, cov, perm, K - k, nullptr);
  }
  return hipGetLastError();
}

// r06: the wave-per-query k-NN over a list (device count, or n), k <= K
template <int K>
static hipError_t knn_wave_k(const GridView& g, double eps, const uint32_t* list, const unsigned int* count, size_t n,
                             int k, Cov3 cov, hipStream_t s, int blocks) {
  if (blocks <= 0) blocks = static_cast<int>(std::min<size_t>((n + 3) / 4, 65535));
  if (blocks <= 0) return hipSuccess;
  knn_wave_kernel<K><<<blocks, 256, 0, s>>>(g, eps, list, count, n, k, cov);
  return hipGetLastError();
}

hipError_t launch_knn_wave(const GridView& g, int k, double eps, const uint32_t* list, const unsigned int* count,
                           size_t n, Cov3 cov, hipStream_t s, int blocks) {
  if (!count && n == 0) return hipSuccess;
  if (k <= 8) return knn_wave_k<8>(g, eps, list, count, n, k, cov, s, blocks);
  if (k <= 16) return knn_wave_k<16>(g, eps, list, count, n, k, cov, s, blocks);
  if (k <= 20) return knn_wave_k<20>(g, eps, list, count, n, k, cov, s, blocks);
  if (k <= 24) return knn_wave_k<24>(g, eps, list, count, n, k, cov, s, blocks);
  return knn_wave_k<32>(g, eps, list, count, n, k, cov, s, blocks);
}

// exact instantiations for PCL's default (20) and its round neighbours; any other k in
// [1, kMaxK] runs on the next multiple of 8 with K - k sentinel slots.  With fb / fb_count the
// logged kernel (knn_cov2_kernel) runs and lists the points it leaves to KnnVisitor; without, (or for that
// list: perm = fb, p0 = 0, p1 = count) the register-list kernel runs.
hipError_t launch_knn_cov(const GridView& g, int k, double eps, size_t p0, size_t p1, Cov3 cov,
                          const uint32_t* perm, uint32_t* fb, unsigned int* fb_count, hipStream_t s, int ring_cap,
                          uint8_t* ok, int chain, bool wave_handoff) {
  if (p1 <= p0) return hipSuccess;
  switch (k) {
    case 5: return knn_cov_k<5>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    case 10: return knn_cov_k<10>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    case 15: return knn_cov_k<15>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    case 20: return knn_cov_k<20>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    case 25: return knn_cov_k<25>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    case 30: return knn_cov_k<30>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
    default: break;
  }
  if (k < 1 || k > kMaxK) return hipErrorInvalidValue;
  if (k <= 8) return knn_cov_k<8>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
  if (k <= 16) return knn_cov_k<16>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
  if (k <= 24) return knn_cov_k<24>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
  return knn_cov_k<32>(g, eps, p0, p1, cov, perm, k, fb, fb_count, s, ring_cap, ok, chain, wave_handoff);
}


hipError_t launch_vl_sweep(const GridView& tgt, const VListView& vl, const float4* src, size_t p0, size_t p1,
                           Xf34 T, double thr, int seeded, uint32_t* nn_pos, uint32_t* flags, int cus,
                           hipStream_t s, const FusedCompact* fc) {
  if (p1 <= p0) return hipSuccess;
  hipError_t e = hipMemsetAsync(vl.ctr + 1, 0, 4 * sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  if (fc)
    vl_query_compact_kernel<<<chunk_count(p1 - p0), 256, 0, s>>>(vl, src, p0, p1 - p0, T, thr, nn_pos, flags, fc->cov_s,
                                                                  fc->cov_t, fc->R, fc->cov_ok, fc->ccnt, fc->defer,
                                                                  fc->out);
  else
    vl_query_kernel<<<nblk(p1 - p0), 256, 0, s>>>(vl, src, p0, p1 - p0, T, thr, nn_pos, flags);
  // requested cells: the centre's 1-NN within the gate + the grown cell's half diagonal, then the lists
  const double hd = std::sqrt(3.0) * (0.5 * static_cast<double>(vl.c) + static_cast<double>(vl.es));
  const double rc = vl.gate * (1.0 + 1e-5) + 1e-9 + hd;
  const unsigned g = static_cast<unsigned>(std::max(cus, 1));
  vl_centre_kernel<<<4 * g, 256, 0, s>>>(tgt, vl, rc * rc * (1.0 + 1e-5));
  vl_build_kernel<<<8 * g, 64 * kVlWavesS, 0, s>>>(tgt, vl);
  vl_build_large_kernel<<<4 * g, 64 * kVlWaves, 0, s>>>(tgt, vl);
  vl_fallback_kernel<<<8 * g, 256, 0, s>>>(tgt, vl, src, p0, T, thr, seeded, nn_pos, flags);
  return hipGetLastError();
}

// lazy source covariances: the accepted points of a sweep whose covariance was never computed
// the accepted points of a sweep without a covariance, listed (any order) and marked.  One block of
// 256 threads takes kCovNeedPer consecutive points per thread round, counts its points, and takes its
// list slots with ONE atomic (one per wave saturated the counter's memory-side atomics in the first
// sweep of a cloud: ~0.3 ms at 5M, profiles/r04/prep4)
constexpr int kCovNeedPer = 16;
// flags == nullptr (lazy target covariances): the points marked 2 by cov_mark_kernel, or (rest) every
// point not marked 1
__global__ __launch_bounds__(256) void cov_need_kernel(const uint32_t* __restrict__ flags, uint8_t* __restrict__ cov_ok,
                                                       size_t p0, size_t n, uint32_t* __restrict__ list,
                                                       unsigned int* __restrict__ count, int rest) {
  __shared__ unsigned int s_w[4];
  __shared__ unsigned int s_base;
  const size_t k0 = static_cast<size_t>(blockIdx.x) * (256 * kCovNeedPer);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long m[kCovNeedPer];
  unsigned int mine = 0;
#pragma unroll
  for (int u = 0; u < kCovNeedPer; ++u) {
    const size_t k = k0 + static_cast<size_t>(u) * 256 + threadIdx.x;
    bool need = false;
    if (k < n) {
      if (flags) need = flags[k] && !cov_ok[k];
      else need = rest ? cov_ok[k] != 1 : cov_ok[k] == 2;
    }
    m[u] = __builtin_amdgcn_ballot_w64(need);
    mine += static_cast<unsigned int>(__builtin_popcountll(m[u]));
  }
  if (lane == 0) s_w[wid] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    s_base = tot ? atomicAdd(count, tot) : 0u;
  }
  __syncthreads();
  unsigned int o = s_base;
  for (int w = 0; w < wid; ++w) o += s_w[w];
#pragma unroll
  for (int u = 0; u < kCovNeedPer; ++u) {
    const size_t k = k0 + static_cast<size_t>(u) * 256 + threadIdx.x;
    if ((m[u] >> lane) & 1ull) {
      const unsigned int r = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned int>(m[u] >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<unsigned int>(m[u]), 0u));
      list[o + r] = static_cast<uint32_t>(p0 + k);
      cov_ok[k] = 1;
    }
    o += static_cast<unsigned int>(__builtin_popcountll(m[u]));
  }
}

hipError_t launch_cov_need(const uint32_t* flags, uint8_t* cov_ok, size_t p0, size_t n, uint32_t* list,
                           unsigned int* count, hipStream_t s) {
  hipError_t e = hipMemsetAsync(count, 0, sizeof(unsigned int), s);
  if (e != hipSuccess || n == 0) return e;
  cov_need_kernel<<<nblk(n, 256 * kCovNeedPer), 256, 0, s>>>(flags, cov_ok, p0, n, list, count, 0);
  return hipGetLastError();
}

hipError_t launch_vl_stats(const VListView& vl, size_t ncells, unsigned long long* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, 64 * sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  vl_stats_kernel<<<2048, 256, 0, s>>>(vl.cell, ncells, out);
  return hipGetLastError();
}

hipError_t launch_correspond(const GridView& tgt, const float4* src, size_t p0, size_t p1, Xf34 T,
                             double thr, int seeded, uint32_t* nn_pos, uint32_t* flags,
                             const uint32_t* qperm, hipStream_t s) {
  if (p1 <= p0) return hipSuccess;
  correspond_kernel<<<nblk(p1 - p0), 256, 0, s>>>(tgt, src, p0, p1, T, thr, seeded, nn_pos, flags, qperm);
  return hipGetLastError();
}

hipError_t launch_correspond_wave(const GridView& tgt, const float4* src, size_t p0, size_t p1, Xf34 T,
                                  double thr, int seeded, uint32_t* nn_pos, uint32_t* flags, const uint32_t* qperm,
                                  float rcap2, int max_rows, int max_xcells, float union_min_r, void* work,
                                  unsigned int* work_n, int split_max, int lds_cap, hipStream_t s) {
  if (p1 <= p0) return hipSuccess;
  if (!tgt.pairs || (work && !work_n)) return hipErrorInvalidValue;
  NnWork* w = static_cast<NnWork*>(work);
  if (w) {
    hipError_t e = hipMemsetAsync(work_n, 0, sizeof(unsigned int), s);
    if (e != hipSuccess) return e;
  }
  if (lds_cap > 0) lds_cap = std::min(lds_cap, kLdsMaxPts) & ~63;
  const size_t shm = lds_cap ? 4 * static_cast<size_t>(std::max(lds_cap, 0) + kLdsMeta) * sizeof(float4) : 0;
  correspond_wave_kernel<<<nblk(p1 - p0), 256, shm, s>>>(tgt, src, p0, p1, T, thr, seeded, nn_pos, flags, qperm,
                                                         rcap2, max_rows, max_xcells, union_min_r, w, work_n,
                                                         split_max, lds_cap);
  if (w) {
    // grid-stride over the stragglers: 8 blocks of 4 waves per CU (the count is known on the device only)
    const unsigned int nb = static_cast<unsigned int>(std::min<size_t>(nblk(p1 - p0), 2048));
    correspond_finish_kernel<<<nb, 256, 0, s>>>(tgt, src, p0, T, thr, w, work_n, nn_pos, flags);
  }
  return hipGetLastError();
}

size_t nn_work_bytes(size_t n) { return n * sizeof(NnWork); }

size_t pair_count(size_t n) { return (n + 1) / 2 + kStagePairs + 2; }

hipError_t launch_pairs(const float4* pts, size_t n, float4* out, hipStream_t s) {
  const size_t np = pair_count(n);
  pairs_kernel<<<nblk(np), 256, 0, s>>>(pts, n, np, out);
  return hipGetLastError();
}

hipError_t launch_morton_keys(const float4* pts, size_t p0, size_t n, const float lo[3], float inv,
                              uint32_t* keys, uint32_t* vals, hipStream_t s) {
  if (!n) return hipSuccess;
  morton_key_kernel<<<nblk(n), 256, 0, s>>>(pts, p0, n, lo[0], lo[1], lo[2], inv, keys, vals);
  return hipGetLastError();
}

hipError_t launch_compact(const float4* src, const float4* tpts, const Cov3& cov_s,
                          const Cov3& cov_t, Rot33d R, const uint32_t* nn_pos,
                          const uint32_t* flags, size_t p0, size_t p1, uint32_t* ccnt, CorrSoA out, hipStream_t s,
                          const uint32_t* defer, const unsigned int* defer_count, int cus) {
  const int nch = chunk_count(p1 - p0);
  if (nch == 0) return hipSuccess;
  if (defer)
    chunk_compact_list_kernel<<<std::min(nch, 2 * std::max(cus, 1)), 256, 0, s>>>(
        src, tpts, cov_s, cov_t, R, nn_pos, flags, p0, p1, ccnt, defer, defer_count, out);
  else
    chunk_compact_kernel<<<nch, 256, 0, s>>>(src, tpts, cov_s, cov_t, R, nn_pos, flags, p0, p1, ccnt, out);
  return hipGetLastError();
}

hipError_t launch_fdf_soa(const CorrSoA& c, const uint32_t* ccnt, size_t ns, Xf34 A,
                          double* partial, double* spart, int nb, unsigned int* tickets, double* out, int reverse,
                          unsigned long long* done_flag, unsigned long long seq, hipStream_t s,
                          unsigned long long* host_rows, unsigned int rstamp) {
  const int nch = chunk_count(ns);
  if (nch == 0) return hipSuccess;
  fdf_soa_kernel<<<nb, 256, 0, s>>>(c, ccnt, nch, A, partial, spart, tickets, out, reverse, done_flag,
                                    seq, host_rows, rstamp);
  return hipGetLastError();
}

hipError_t launch_fdf_soa_gated(const CorrSoA& c, const uint32_t* ccnt, size_t ns,
                                double* partial, double* spart, int nb, unsigned int* tickets, double* out,
                                unsigned long long* done_flag, unsigned long long seq, const PassCmd* cmd,
                                PassCmd* mail, unsigned long long timeout_ticks, unsigned long long* gtrace,
                                int host_pollers, hipStream_t s) {
  const int nch = chunk_count(ns);
  if (nch == 0) return hipSuccess;
  fdf_soa_gated_kernel<<<nb, 256, 0, s>>>(c, ccnt, nch, partial, spart, tickets, out, done_flag, seq,
                                          cmd, mail, timeout_ticks, gtrace, host_pollers);
  return hipGetLastError();
}

int fdf_server_blocks(size_t ns, int cus, int waves) {
  // one block of `waves` waves per CU, fewer when the shard has fewer chunks; 0 when a wave would
  // hold more than 64 chunks (its lanes draw the tickets of all its chunks at once)
  const int nch = chunk_count(ns);
  if (nch == 0 || cus <= 0 || (waves != 4 && waves != 8)) return 0;
  const int nb = std::min(cus, (nch + waves - 1) / waves);
  if (nch > 64 * waves * nb) return 0;
  return nb;
}

hipError_t launch_fdf_server(const CorrSoA& c, const uint32_t* ccnt, size_t ns, double* partial,
                             double* spart, unsigned int* tickets, double* out, unsigned long long* done_flag,
                             unsigned long long seq0, const PassCmd* cmd, PassCmd* mail,
                             unsigned long long timeout_ticks, unsigned long long* ptimes, int bench_passes,
                             Xf34 A, unsigned long long* host_rows, size_t rows_stride, int nb, int waves,
                             int pollers, int stall_pass, unsigned long long* tpart, hipStream_t s,
                             const PeerRows* peers) {
  int nch = chunk_count(ns);
  if (peers && (peers->n < 0 || peers->n > kMaxPeers || (peers->n > 0 && (!host_rows || !tpart))))
    return hipErrorInvalidValue;  // peer rows go with the tagged tail's host rows only
  // one shape: 4 waves per CU (the 8-wave shape, 2 waves per SIMD with less residency, measured
  // 57.7-58.0 vs 50.2-50.3 us per pass, profiles/r03/srv8, is not built)
  if (nch == 0 || nb <= 0 || waves != 4) return hipErrorInvalidValue;
  // a pass completes only when every block has run it, so refuse a grid the device cannot hold at
  // once (one block per CU, at most one per CU by its LDS and registers).  That check is all a
  // cooperative launch adds; the blocks do not synchronise with each other (only with the host's
  // commands), and a server whose blocks cannot all be resident (other work on the device) is
  // cancelled by the host after its deadline -- blocks that start late see the later command at
  // their first gate and exit (pass_gate) -- and the pass re-runs as a launched pass.
  const bool b = bench_passes > 0;
  const void* fn = b ? reinterpret_cast<const void*>(fdf_server_kernel<true, 4>)
                     : reinterpret_cast<const void*>(fdf_server_kernel<false, 4>);
  int per_cu = 0, dev = 0, cus = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * waves, 0);
  if (e == hipSuccess) e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  if (per_cu < 1 || static_cast<long long>(per_cu) * cus < nb) return hipErrorCooperativeLaunchTooLarge;
  PeerRows pr{};
  if (peers) pr = *peers;
#define MGICP_SRV_LAUNCH(B, W)                                                                                  \
  fdf_server_kernel<B, W><<<nb, 64 * (W), 0, s>>>(c, ccnt, nch, partial, spart, tickets, out, done_flag, \
                                                  seq0, cmd, mail, timeout_ticks, ptimes, bench_passes, A, host_rows, \
                                                  rows_stride, pollers, stall_pass, tpart, pr)
  if (b) MGICP_SRV_LAUNCH(true, 4);
  else MGICP_SRV_LAUNCH(false, 4);
#undef MGICP_SRV_LAUNCH
  return hipGetLastError();
}

// system-scope load (bypasses the caches): rows other GPUs store into this GPU's memory over xGMI
__device__ __forceinline__ unsigned long long ld_sys_u64(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// r05 xGMI totaler: one wave per rank for a BFGS run (see launch_xgmi_total in mgicp_internal.hpp).
// Rows are stamped halves (word 2v, 2v + 1 of a row = value v's low / high half, high 32 bits of each
// word = the pass stamp), written by every rank's super reducers into this rank's buffer over xGMI.
// The total is shm::fixed_total's: lane l sums supers l, l + 64, ... from 0.0, then wave_sum's tree.
__global__ __launch_bounds__(64) void xgmi_total_kernel(const unsigned long long* __restrict__ rows0, size_t stride,
                                                         long long nsup, unsigned int stamp0,
                                                         unsigned long long* __restrict__ out,
                                                         const unsigned int* __restrict__ gen_word, unsigned int gen,
                                                         unsigned long long timeout) {
  const int lane = threadIdx.x;
  for (unsigned int st = stamp0;; ++st) {
    const unsigned long long* buf = rows0 + (st & 1u) * stride;
    const unsigned long long t0 = wall_clock64();
    double acc[16];
    // one pass over the rows both checks the stamps and sums the values (lane l: supers l, l + 64, ...
    // in order from 0.0); any stale word and the poll starts over
    for (;;) {
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[v] = 0.0;
      bool ok = true;
      for (long long sg = lane; sg < nsup; sg += 64) {
        const unsigned long long* row = buf + static_cast<size_t>(sg) * 32;
        unsigned long long w[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) w[k] = ld_sys_u64(row + k);
#pragma unroll
        for (int k = 0; k < 32; ++k) ok = ok && static_cast<unsigned int>(w[k] >> 32) == st;
#pragma unroll
        for (int v = 0; v < 16; ++v)
          acc[v] += mk64(static_cast<unsigned int>(w[2 * v]), static_cast<unsigned int>(w[2 * v + 1]));
      }
      if (__builtin_amdgcn_ballot_w64(!ok) == 0ull) break;
      const unsigned int g = __hip_atomic_load(const_cast<unsigned int*>(gen_word), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
      if (g != gen || wall_clock64() - t0 > timeout) return;  // cancelled (BFGS run over) or nothing arrives
      __builtin_amdgcn_s_sleep(1);
    }
    double tot = 0.0;  // lane v < 16: total v
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const double t = __shfl(wave_sum(acc[v]), 0, 64);
      if ((lane >> 1) == v) tot = t;
    }
    if (lane < 32) {
      const long long bits = __double_as_longlong(tot);
      const unsigned int half = static_cast<unsigned int>((lane & 1) ? (bits >> 32) : bits);
      const unsigned long long w = (static_cast<unsigned long long>(st) << 32) | half;
      asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(out + lane), "v"(w) : "memory");
    }
  }
}

hipError_t launch_xgmi_total(const unsigned long long* rows0, size_t stride, long long nsup, unsigned int stamp0,
                             unsigned long long* out, const unsigned int* gen_word, unsigned int gen,
                             unsigned long long timeout_ticks, hipStream_t s) {
  if (!rows0 || !out || !gen_word || nsup < 1) return hipErrorInvalidValue;
  xgmi_total_kernel<<<1, 64, 0, s>>>(rows0, stride, nsup, stamp0, out, gen_word, gen, timeout_ticks);
  return hipGetLastError();
}

hipError_t launch_super_reduce(const double* chunk, int nch, int nv, double* sup, hipStream_t s) {
  if (nch <= 0) return hipSuccess;
  const int nsup = (nch + kSuperChunks - 1) / kSuperChunks;
  if (nv == kRedVals) super_reduce_kernel<kRedVals><<<nsup, 64, 0, s>>>(chunk, nch, sup);
  else if (nv == kMomVals) super_reduce_kernel<kMomVals><<<nsup, 128, 0, s>>>(chunk, nch, sup);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// one wave per block: the 16 shuffle trees (lane 0) and the register reduce-scatter (lanes 8k)
__global__ __launch_bounds__(64) void wave_reduce_check_kernel(const double* __restrict__ in, double* __restrict__ out_tree,
                                                               double* __restrict__ out_rs) {
  const int lane = threadIdx.x;
  const double* row = in + (static_cast<size_t>(blockIdx.x) * 64 + lane) * 16;
  double a[16], b[16];
#pragma unroll
  for (int v = 0; v < 16; ++v) a[v] = b[v] = row[v];
#pragma unroll
  for (int v = 0; v < 16; ++v) a[v] = wave_sum(a[v]);
  if (lane == 0)
    for (int v = 0; v < 16; ++v) out_tree[static_cast<size_t>(blockIdx.x) * 16 + v] = a[v];
  wave_sum16(b, lane);
  if ((lane & 7) == 0) {
    out_rs[static_cast<size_t>(blockIdx.x) * 16 + (lane >> 2)] = b[0];
    out_rs[static_cast<size_t>(blockIdx.x) * 16 + (lane >> 2) + 1] = b[1];
  }
}

hipError_t launch_wave_reduce_check(const double* in, int nwaves, double* out_tree, double* out_rs, hipStream_t s) {
  if (nwaves <= 0) return hipErrorInvalidValue;
  wave_reduce_check_kernel<<<nwaves, 64, 0, s>>>(in, out_tree, out_rs);
  return hipGetLastError();
}

hipError_t launch_finish_supers(const double* sup, long long nsup, long long maxsup, int nranks, int nv,
                                double* out, hipStream_t s) {
  if (nv == kRedVals) finish_supers_kernel<kRedVals><<<1, 64, 0, s>>>(sup, nsup, maxsup, nranks, out);
  else if (nv == kMomVals) finish_supers_kernel<kMomVals><<<kMomVals / 16, 64, 0, s>>>(sup, nsup, maxsup, nranks, out);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_publish(const double* in, int n, double* host_out, unsigned long long* flag,
                          unsigned long long seq, hipStream_t s) {
  publish_kernel<<<1, 64, 0, s>>>(in, n, host_out, flag, seq);
  return hipGetLastError();
}

int chunk_grid_blocks(size_t ns) {  // one wave per chunk, 4 waves per block
  return static_cast<int>(std::max<size_t>(1, (static_cast<size_t>(chunk_count(ns)) + 3) / 4));
}

hipError_t launch_gn_moments(const float4* src, const float4* tpts, const Cov3& cov_s,
                             const Cov3& cov_t, Rot33d R, Xf34 T0, const double ctr[3],
                             const uint32_t* nn_pos, const uint32_t* flags, size_t p0, size_t p1,
                             double* partial, int nb, hipStream_t s) {
  gn_moments_kernel<<<nb, 256, 0, s>>>(src, tpts, cov_s, cov_t, R, T0, ctr[0], ctr[1], ctr[2],
                                       nn_pos, flags, p0, p1, partial);
  return hipGetLastError();
}


int fdf_grid_blocks(size_t ns, int max_blocks) {
  // persistent 4-wave blocks over the chunks; a wave takes at most 64 chunks (its lanes draw the
  // tickets of its chunks at once)
  const size_t nch = static_cast<size_t>(chunk_count(ns));
  const size_t want = std::min<size_t>((nch + 3) / 4, static_cast<size_t>(std::max(max_blocks, 1)));
  return static_cast<int>(std::max<size_t>({want, (nch + 255) / 256, 1}));
}

hipError_t launch_fitness(const GridView& tgt, const float4* src, size_t p0, size_t p1, Xf34 T,
                          double max_range, double* partial, int nb, hipStream_t s) {
  fitness_kernel<<<nb, 256, 0, s>>>(tgt, src, p0, p1, T, max_range, partial);
  return hipGetLastError();
}

hipError_t launch_resolution(const GridView& g, size_t n, double* partial, int nb, hipStream_t s) {
  resolution_kernel<<<nb, 256, 0, s>>>(g, n, partial);
  return hipGetLastError();
}

hipError_t launch_radius_keep(const GridView& g, size_t n, float r2, int need, unsigned char* keep,
                              hipStream_t s) {
  if (!n) return hipSuccess;
  radius_keep_kernel<<<nblk(n), 256, 0, s>>>(g, n, r2, need, keep);
  return hipGetLastError();
}

hipError_t launch_reduce_finish(const double* partial, int nb, double* out, hipStream_t s) {
  reduce_finish_kernel<<<1, kRedThreads, 0, s>>>(partial, nb, out);
  return hipGetLastError();
}

hipError_t launch_finite_compact(const float4* in, size_t n, uint32_t* flags, uint32_t* pos,
                                 void* scratch, size_t scratch_bytes, float4* out, hipStream_t s) {
  finite_flags_kernel<<<nblk(n + 1), 256, 0, s>>>(in, n, flags);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = launch_exclusive_scan(scratch, scratch_bytes, flags, pos, n + 1, s)) != hipSuccess) return e;
  scatter_flagged_kernel<<<nblk(n), 256, 0, s>>>(in, flags, pos, n, out);
  return hipGetLastError();
}

hipError_t launch_segdiff(const GridView& g, const float4* in, size_t n, Xf34 T, int has_T, double thr,
                          unsigned char* keep, unsigned int* count, hipStream_t s) {
  if (!n) return hipSuccess;
  segdiff_kernel<<<nblk(n), 256, 0, s>>>(g, in, n, T, has_T, thr, keep, count);
  return hipGetLastError();
}

hipError_t launch_voxel_keys(const float4* pts, size_t n, const float inv[3], const int min_b[3],
                             int mul1, int mul2, uint32_t* keys, hipStream_t s) {
  if (!n) return hipSuccess;
  voxel_key_kernel<<<nblk(n), 256, 0, s>>>(pts, n, inv[0], inv[1], inv[2], min_b[0], min_b[1], min_b[2],
                                           mul1, mul2, keys);
  return hipGetLastError();
}

hipError_t launch_voxel_heads(const uint32_t* keys_sorted, size_t n, uint32_t* flags, hipStream_t s) {
  voxel_head_kernel<<<nblk(n + 1), 256, 0, s>>>(keys_sorted, n, flags);
  return hipGetLastError();
}

hipError_t launch_voxel_centroids(const uint32_t* keys_sorted, const uint32_t* perm, const uint32_t* flags,
                                  const uint32_t* pos, size_t n, const float4* pts, const uint32_t* rgba,
                                  float4* out, uint32_t* out_rgba, hipStream_t s) {
  if (!n) return hipSuccess;
  voxel_centroid_kernel<<<nblk(n), 256, 0, s>>>(keys_sorted, perm, flags, pos, n, pts, rgba, out, out_rgba);
  return hipGetLastError();
}

hipError_t launch_voxel_minpts(const float4* vox, const uint32_t* vox_rgba, size_t nv, uint32_t need,
                               uint32_t* flags, uint32_t* pos, void* scratch, size_t scratch_bytes,
                               float4* out, uint32_t* out_rgba, hipStream_t s) {
  voxel_minpts_kernel<<<nblk(nv + 1), 256, 0, s>>>(vox, nv, need, flags);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = launch_exclusive_scan(scratch, scratch_bytes, flags, pos, nv + 1, s)) != hipSuccess) return e;
  if (!nv) return hipSuccess;
  scatter_voxels_kernel<<<nblk(nv), 256, 0, s>>>(vox, vox_rgba, flags, pos, nv, out, out_rgba);
  return hipGetLastError();
}

size_t sort_scratch_bytes(size_t n, int bits) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr),
                                     static_cast<const uint32_t*>(nullptr),
                                     static_cast<uint32_t*>(nullptr), static_cast<int>(n), 0, bits);
  return bytes;
}

hipError_t launch_sort_pairs(void* scratch, size_t scratch_bytes, const uint32_t* keys_in,
                             uint32_t* keys_out, const uint32_t* vals_in, uint32_t* vals_out,
                             size_t n, int bits, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(scratch, scratch_bytes, keys_in, keys_out, vals_in,
                                            vals_out, static_cast<int>(n), 0, bits, s);
}

size_t scan_scratch_bytes(size_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                   static_cast<uint32_t*>(nullptr), static_cast<int>(n));
  return bytes;
}

hipError_t launch_exclusive_scan(void* scratch, size_t scratch_bytes, const uint32_t* in,
                                 uint32_t* out, size_t n, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(scratch, scratch_bytes, in, out, static_cast<int>(n), s);
}

// Resolve every kernel of the code object (and run hipcub's sort / scan once on a few
// elements) so that the one-time loading cost lands in mgicp_create, not in the first align.
hipError_t preload_kernels(void* pinned, size_t pinned_bytes, hipStream_t s) {
  const void* fns[] = {
      reinterpret_cast<const void*>(&pack_points_kernel),
      reinterpret_cast<const void*>(&bbox_kernel),
      reinterpret_cast<const void*>(&cell_hist_kernel),
      reinterpret_cast<const void*>(&cell_sketch_kernel),
      reinterpret_cast<const void*>(&sketch_merge_kernel),
      reinterpret_cast<const void*>(&cell_end_kernel),
      reinterpret_cast<const void*>(&gather_sorted_kernel),
      reinterpret_cast<const void*>(&xform_points_kernel),
      reinterpret_cast<const void*>(&empty_init_kernel),
      reinterpret_cast<const void*>(&empty_pass_kernel),
      reinterpret_cast<const void*>(&iota_kernel),
      reinterpret_cast<const void*>(&cell_box_kernel),
      reinterpret_cast<const void*>(&knn_cov_kernel<5>),
      reinterpret_cast<const void*>(&knn_cov_kernel<10>),
      reinterpret_cast<const void*>(&knn_cov_kernel<15>),
      reinterpret_cast<const void*>(&knn_cov_kernel<20>),
      reinterpret_cast<const void*>(&knn_cov_kernel<25>),
      reinterpret_cast<const void*>(&knn_cov_kernel<30>),
      reinterpret_cast<const void*>(&knn_cov_kernel<8>),
      reinterpret_cast<const void*>(&knn_cov_kernel<16>),
      reinterpret_cast<const void*>(&knn_cov_kernel<24>),
      reinterpret_cast<const void*>(&knn_cov_kernel<32>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<5>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<10>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<15>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<20>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<25>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<30>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<8>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<16>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<24>),
      reinterpret_cast<const void*>(&knn_cov2_kernel<32>),
      reinterpret_cast<const void*>(&correspond_kernel),
      reinterpret_cast<const void*>(&morton_key_kernel),
      reinterpret_cast<const void*>(&chunk_compact_kernel),
      reinterpret_cast<const void*>(&chunk_compact_list_kernel),
      reinterpret_cast<const void*>(&vl_query_compact_kernel),
      reinterpret_cast<const void*>(&fdf_soa_kernel),
      reinterpret_cast<const void*>(&fdf_soa_gated_kernel),
      reinterpret_cast<const void*>(&fdf_server_kernel<false, 4>),
      reinterpret_cast<const void*>(&fdf_server_kernel<true, 4>),
      reinterpret_cast<const void*>(&fdf_server_kernel<false, 8>),
      reinterpret_cast<const void*>(&fdf_server_kernel<true, 8>),
      reinterpret_cast<const void*>(&fitness_kernel),
      reinterpret_cast<const void*>(&resolution_kernel),
      reinterpret_cast<const void*>(&radius_keep_kernel),
      reinterpret_cast<const void*>(&reduce_finish_kernel),
      reinterpret_cast<const void*>(&gn_moments_kernel),
      reinterpret_cast<const void*>(&publish_kernel),
      reinterpret_cast<const void*>(&super_reduce_kernel<kRedVals>),
      reinterpret_cast<const void*>(&super_reduce_kernel<kMomVals>),
      reinterpret_cast<const void*>(&finish_supers_kernel<kRedVals>),
      reinterpret_cast<const void*>(&finish_supers_kernel<kMomVals>),
      reinterpret_cast<const void*>(&finite_flags_kernel),
      reinterpret_cast<const void*>(&scatter_flagged_kernel),
      reinterpret_cast<const void*>(&segdiff_kernel),
      reinterpret_cast<const void*>(&voxel_key_kernel),
      reinterpret_cast<const void*>(&voxel_head_kernel),
      reinterpret_cast<const void*>(&voxel_centroid_kernel),
      reinterpret_cast<const void*>(&voxel_minpts_kernel),
      reinterpret_cast<const void*>(&scatter_voxels_kernel),
  };
  for (const void* f : fns) {
    hipFuncAttributes attr;
    hipError_t e = hipFuncGetAttributes(&attr, f);
    if (e != hipSuccess) return e;
  }
  constexpr size_t n = 64;
  uint32_t* buf = nullptr;
  void* big = nullptr;
  hipError_t e = hipMalloc(&buf, 4 * n * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&big, pinned_bytes);
  if (e != hipSuccess) return e;
  if (e != hipSuccess) return e;
  const size_t sb = std::max(sort_scratch_bytes(n, 8), scan_scratch_bytes(n));
  void* scratch = nullptr;
  e = hipMalloc(&scratch, sb);
  if (e == hipSuccess) e = hipMemsetAsync(buf, 0, 4 * n * sizeof(uint32_t), s);
  if (e == hipSuccess) e = launch_iota(buf + n, n, s);
  if (e == hipSuccess) e = launch_sort_pairs(scratch, sb, buf, buf + 2 * n, buf + n, buf + 3 * n, n, 8, s);
  if (e == hipSuccess) e = launch_exclusive_scan(scratch, sb, buf + n, buf + 2 * n, n, s);
  // one small copy each way, from pinned and from pageable memory: the runtime brings up its
  // copy engines / bounce buffers on first use (measured 8-10 ms per direction), which would
  // otherwise land in the first upload and the first grid build's readback
  uint32_t host[4] = {0, 0, 0, 0};
  // (small copies and large ones take different paths: exercise both sizes)
  if (e == hipSuccess) e = hipMemcpyAsync(buf, pinned, 16, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(pinned, buf + 2 * n, 16, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(big, pinned, pinned_bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = launch_iota(static_cast<uint32_t*>(big), pinned_bytes / 4, s);
  if (e == hipSuccess) e = hipMemcpyAsync(pinned, big, pinned_bytes, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = launch_iota(static_cast<uint32_t*>(big), pinned_bytes / 8, s);
  if (e == hipSuccess) e = hipMemcpyAsync(pinned, big, pinned_bytes / 2, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipMemcpyAsync(buf, host, sizeof(host), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(host, buf + 2 * n, sizeof(host), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(scratch);
  (void)hipFree(buf);
  (void)hipFree(big);
  return e;
}

}  // namespace mgicp
