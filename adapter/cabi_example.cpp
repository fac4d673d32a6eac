// adapter/cabi_example.cpp -- C++ host code driving the C-ABI exactly as the GICPAlignment
// adapter does (set inputs with a 32-byte PointXYZRGB stride, align, fitness, transform),
// without PCL.  Built by `make adapter-example`; run it on a GPU box:
//     ./adapter/cabi_example            -> prints T and checks it against the known rotation
#include <mi355x_gicp.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace {
struct PointXYZRGB {  // pcl::PointXYZRGB memory layout
  float x, y, z, pad;
  unsigned rgba;
  unsigned pad2[3];
};
static_assert(sizeof(PointXYZRGB) == 32, "layout");

void sample_box(std::vector<PointXYZRGB>& out, size_t n, unsigned seed) {
  std::mt19937 rng(seed);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::uniform_int_distribution<int> face(0, 5);
  out.resize(n);
  for (auto& p : out) {
    float v[3] = {u(rng), 0.5f * u(rng), 0.25f * u(rng)};
    const int f = face(rng);
    const float ext[3] = {1.f, 0.5f, 0.25f};
    v[f / 2] = (f % 2) ? ext[f / 2] : -ext[f / 2];
    p = PointXYZRGB{v[0], v[1], v[2], 1.f, 0u, {0u, 0u, 0u}};
  }
}
}  // namespace

int main() {
  std::vector<PointXYZRGB> src, tgt;
  sample_box(src, 20000, 1);
  const float a = 0.05f, c = std::cos(a), s = std::sin(a);
  tgt = src;
  for (auto& p : tgt) {  // target = Rz(a) * source + (0.01, 0, 0)
    const float x = p.x, y = p.y;
    p.x = c * x - s * y + 0.01f;
    p.y = s * x + c * y;
  }
  mgicp_params prm;
  mgicp_default_params(&prm);
  mgicp_ctx* ctx = nullptr;
  int rc = mgicp_create(&ctx, &prm);
  if (rc != MGICP_OK) {
    std::printf("mgicp_create failed: %d (no GPU?)\n", rc);
    return 2;
  }
  rc = mgicp_set_source(ctx, &src[0].x, src.size(), sizeof(PointXYZRGB));
  rc |= mgicp_set_target(ctx, &tgt[0].x, tgt.size(), sizeof(PointXYZRGB));
  float T[16];
  mgicp_result res;
  rc |= mgicp_align(ctx, nullptr, T, &res);
  double fitness = 0.0;
  mgicp_fitness(ctx, T, 0.0, &fitness);
  std::printf("rc=%d converged=%d iterations=%d n_corr=%d passes=%d ms_total=%.3f fitness=%.3e\n", rc,
              res.converged, res.iterations, res.n_corr, res.n_evals, res.ms_total, fitness);
  for (int r = 0; r < 4; ++r)
    std::printf("  [% .6f % .6f % .6f % .6f]\n", T[r], T[4 + r], T[8 + r], T[12 + r]);
  const double err = std::fabs(T[0] - c) + std::fabs(T[1] - s) + std::fabs(T[4] + s) + std::fabs(T[12] - 0.01f);
  bool ok = rc == MGICP_OK && res.converged && err < 1e-3;

  // the opt-in Gauss-Newton mode (one moment pass per outer iteration), same clouds
  prm.solver = MGICP_SOLVER_GN;
  rc = mgicp_set_params(ctx, &prm);
  float Tg[16];
  rc |= mgicp_align(ctx, nullptr, Tg, &res);
  const double err_gn = std::fabs(Tg[0] - c) + std::fabs(Tg[1] - s) + std::fabs(Tg[4] + s) + std::fabs(Tg[12] - 0.01f);
  std::printf("GN: rc=%d converged=%d iterations=%d passes=%d err=%.2e\n", rc, res.converged, res.iterations,
              res.n_evals, err_gn);
  ok = ok && rc == MGICP_OK && res.converged && res.n_evals == res.iterations && err_gn < 1e-3;

  // Filter::downsampleCloud (VoxelGrid, 5 cm leaves) and Filter::removeFromCloud
  // (SegmentDifferences of the aligned source against the target) on PointXYZRGB records
  std::vector<PointXYZRGB> vox(src.size());
  size_t n_vox = 0;
  const double leaf[3] = {0.05, 0.05, 0.05};
  rc = mgicp_voxel_grid(ctx, &src[0].x, src.size(), sizeof(PointXYZRGB), 16, leaf, 0, &vox[0].x,
                        sizeof(PointXYZRGB), &n_vox);
  std::vector<unsigned char> keep(src.size());
  size_t n_keep = 0;
  rc |= mgicp_segment_differences(ctx, Tg, &src[0].x, src.size(), sizeof(PointXYZRGB), &tgt[0].x, tgt.size(),
                                  sizeof(PointXYZRGB), 1e-4, keep.data(), &n_keep);
  std::printf("VoxelGrid: %zu -> %zu leaves; SegmentDifferences(aligned, 1 cm): %zu of %zu kept; rc=%d\n",
              src.size(), n_vox, n_keep, src.size(), rc);
  ok = ok && rc == MGICP_OK && n_vox > 0 && n_vox < src.size() && n_keep < src.size() / 100;
  mgicp_destroy(ctx);
  std::printf("%s\n", ok ? "cabi_example: OK" : "cabi_example: FAILED");
  return ok ? 0 : 1;
}
