/*
 * gicp_ref.c -- TEST INFRASTRUCTURE ONLY: the parity oracle and the timed CPU baseline.
 *
 * CPU restatement of PCL 1.8.1 GeneralizedIterativeClosestPoint<PointXYZRGB,PointXYZRGB>
 * as used by the reference (include/GICPAlignment.h:153, src/GICPAlignment.cpp:86-109).
 * PCL is an un-vendored third-party dependency (PCL 1.8.1, pinned by .travis.yml:11 and
 * README.md:82-89); its algorithm is restated from the published sources per SURVEY.md
 * Appendix A:
 *   - Registration::align                    registration/impl/registration.hpp
 *   - GICP::computeCovariances               registration/impl/gicp.hpp
 *   - GICP::computeTransformation            registration/impl/gicp.hpp
 *   - GICP::estimateRigidTransformationBFGS  registration/impl/gicp.hpp
 *   - OptimizationFunctorWithIndices::{f,df,fdf}, computeRDerivative, applyState
 *   - BFGS (GSL vector_bfgs2 port)           registration/bfgs.h
 *   - Registration::getFitnessScore          registration/impl/registration.hpp
 *   - KdTreeFLANN exact (eps = 0) k-NN        kdtree/impl/kdtree_flann.hpp (leaf size 15)
 *
 * Exactness contract shared with the HIP engine (DESIGN.md "Numerics"):
 *   * compiled with -ffp-contract=off (no FMA contraction) so fp32 expressions round like
 *     PCL's SSE2 (non-FMA) Eigen code;
 *   * squared distances are float ((dx*dx + dy*dy) + dz*dz) like FLANN L2_Simple;
 *   * k-NN ties are broken by the lower point index (FLANN's order is traversal dependent;
 *     exact float ties have measure zero on continuous data -- documented);
 *   * covariance = fp32 products summed in fp64 (PCL's pt.x*pt.x into Matrix3d);
 *   * the 3x3 symmetric SVD is a cyclic Jacobi in fp64 (any exact eigensolver gives PCL's
 *     C = u1u1' + u2u2' + eps*u3u3' up to fp64 rounding).
 */
#define _POSIX_C_SOURCE 200809L
#define _GNU_SOURCE 1 /* sincos / sincosf (glibc) */
#include "gicp_ref.h"

#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------ */
/* small helpers                                                                         */
/* ------------------------------------------------------------------------------------ */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* float squared distance, FLANN L2_Simple order: ((0 + dx^2) + dy^2) + dz^2 */
static inline float d2f(const float* a, const float* b) {
    float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    float r = dx * dx;
    r = r + dy * dy;
    r = r + dz * dz;
    return r;
}

/* Eigen Matrix4f * Vector4f (w = 1) with SSE2 packet order: ((c0*x + c1*y) + c2*z) + c3;
 * identical to pcl::transformPointCloud's scalar expression.  T is row-major here. */
static inline void xform(const float T[4][4], const float p[3], float o[3]) {
    for (int r = 0; r < 3; ++r) {
        float a = T[r][0] * p[0];
        a = a + T[r][1] * p[1];
        a = a + T[r][2] * p[2];
        o[r] = a + T[r][3];
    }
}

static void cm_to_rm(const float cm[16], float T[4][4]) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) T[r][c] = cm[c * 4 + r];
}
static void rm_to_cm(const float T[4][4], float cm[16]) {
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) cm[c * 4 + r] = T[r][c];
}
static void identity4(float T[4][4]) {
    memset(T, 0, 16 * sizeof(float));
    T[0][0] = T[1][1] = T[2][2] = T[3][3] = 1.0f;
}

/* ------------------------------------------------------------------------------------ */
/* kd-tree (exact search; leaf size 15 like PCL's KDTreeSingleIndexParams(15))            */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int left, right; /* children; -1 => leaf */
    int start, end;  /* leaf range into perm */
    int dim;
    float split;
} kd_node;

typedef struct {
    const float* pts; /* n x 3, owned by caller */
    int n;
    int* perm;
    kd_node* nodes;
    int nnodes, cap;
} kdtree;

static int kd_new_node(kdtree* t) {
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 1024;
        t->nodes = (kd_node*)realloc(t->nodes, (size_t)t->cap * sizeof(kd_node));
    }
    return t->nnodes++;
}

/* quickselect: place the k-th smallest (by coordinate dim) of perm[lo,hi) at position k */
static void kd_select(const float* pts, int* perm, int lo, int hi, int k, int dim) {
    while (hi - lo > 1) {
        int mid = lo + (hi - lo) / 2;
        float pv = pts[3 * perm[mid] + dim];
        int i = lo, j = hi - 1;
        while (i <= j) {
            while (pts[3 * perm[i] + dim] < pv) ++i;
            while (pts[3 * perm[j] + dim] > pv) --j;
            if (i <= j) {
                int tmp = perm[i]; perm[i] = perm[j]; perm[j] = tmp;
                ++i; --j;
            }
        }
        if (k <= j) hi = j + 1;
        else if (k >= i) lo = i;
        else return;
    }
}

static int kd_build_rec(kdtree* t, int start, int end) {
    int id = kd_new_node(t);
    kd_node nd;
    nd.start = start; nd.end = end; nd.left = nd.right = -1; nd.dim = 0; nd.split = 0.f;
    if (end - start > 15) {
        float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int i = start; i < end; ++i) {
            const float* p = t->pts + 3 * t->perm[i];
            for (int d = 0; d < 3; ++d) {
                if (p[d] < lo[d]) lo[d] = p[d];
                if (p[d] > hi[d]) hi[d] = p[d];
            }
        }
        int dim = 0;
        float ext = hi[0] - lo[0];
        for (int d = 1; d < 3; ++d)
            if (hi[d] - lo[d] > ext) { ext = hi[d] - lo[d]; dim = d; }
        if (ext > 0.f) {
            int mid = start + (end - start) / 2;
            kd_select(t->pts, t->perm, start, end, mid, dim);
            nd.dim = dim;
            nd.split = t->pts[3 * t->perm[mid] + dim];
            /* left = [start, mid) all <= split ; right = [mid, end) all >= split */
            t->nodes[id] = nd;
            int l = kd_build_rec(t, start, mid);
            int r = kd_build_rec(t, mid, end);
            t->nodes[id].left = l;
            t->nodes[id].right = r;
            return id;
        }
        /* all points identical: one big leaf */
    }
    t->nodes[id] = nd;
    return id;
}

static void kd_build(kdtree* t, const float* pts, int n) {
    memset(t, 0, sizeof(*t));
    t->pts = pts;
    t->n = n;
    t->perm = (int*)malloc((size_t)(n > 0 ? n : 1) * sizeof(int));
    for (int i = 0; i < n; ++i) t->perm[i] = i;
    if (n > 0) kd_build_rec(t, 0, n);
}

static void kd_free(kdtree* t) {
    free(t->perm);
    free(t->nodes);
    memset(t, 0, sizeof(*t));
}

/* k-best result set ordered by (d2, index) */
typedef struct {
    int k, count;
    float* d2;
    int* idx;
} knn_set;

static inline int knn_better(float da, int ia, float db, int ib) {
    return da < db || (da == db && ia < ib);
}
static inline float knn_worst(const knn_set* s) {
    return s->count < s->k ? FLT_MAX : s->d2[s->k - 1];
}
static inline void knn_add(knn_set* s, float d2, int idx) {
    if (s->count == s->k && !knn_better(d2, idx, s->d2[s->k - 1], s->idx[s->k - 1])) return;
    int i = s->count < s->k ? s->count++ : s->k - 1;
    while (i > 0 && knn_better(d2, idx, s->d2[i - 1], s->idx[i - 1])) {
        s->d2[i] = s->d2[i - 1];
        s->idx[i] = s->idx[i - 1];
        --i;
    }
    s->d2[i] = d2;
    s->idx[i] = idx;
}

static void kd_search(const kdtree* t, int node, const float* q, knn_set* s) {
    const kd_node* nd = &t->nodes[node];
    if (nd->left < 0) {
        for (int i = nd->start; i < nd->end; ++i) {
            int j = t->perm[i];
            knn_add(s, d2f(q, t->pts + 3 * j), j);
        }
        return;
    }
    float diff = q[nd->dim] - nd->split;
    int first = diff < 0.f ? nd->left : nd->right;
    int second = diff < 0.f ? nd->right : nd->left;
    kd_search(t, first, q, s);
    /* far side holds points whose float d2 >= diff^2 (monotone rounding); <= keeps ties */
    if (diff * diff <= knn_worst(s)) kd_search(t, second, q, s);
}

static void kd_knn(const kdtree* t, const float* q, int k, int* idx, float* d2) {
    knn_set s;
    s.k = k; s.count = 0; s.d2 = d2; s.idx = idx;
    if (t->n > 0) kd_search(t, 0, q, &s);
    for (int i = s.count; i < k; ++i) { idx[i] = -1; d2[i] = FLT_MAX; }
}

/* ------------------------------------------------------------------------------------ */
/* covariances (GICP::computeCovariances)                                                */
/* ------------------------------------------------------------------------------------ */

/* cyclic Jacobi on a symmetric 3x3 (fp64).  Returns eigenvalues on the diagonal of a and
 * eigenvectors in the columns of v.  Shared bit-for-bit with the HIP kernel. */
static void jacobi3(double a[3][3], double v[3][3]) {
    static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) v[r][c] = (r == c) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; ++sweep) {
        int rotated = 0;
        for (int e = 0; e < 3; ++e) {
            int p = P[e], q = Q[e], o = 3 - p - q;
            double apq = a[p][q];
            double app = a[p][p], aqq = a[q][q];
            if (fabs(apq) <= 1e-18 * (fabs(app) + fabs(aqq))) {
                a[p][q] = a[q][p] = 0.0;
                continue;
            }
            rotated = 1;
            double theta = (aqq - app) / (2.0 * apq);
            double t;
            if (fabs(theta) > 1e150) t = 0.5 / theta;
            else t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            double c = 1.0 / sqrt(t * t + 1.0);
            double s = t * c;
            a[p][p] = app - t * apq;
            a[q][q] = aqq + t * apq;
            a[p][q] = a[q][p] = 0.0;
            double aop = a[o][p], aoq = a[o][q];
            a[o][p] = a[p][o] = c * aop - s * aoq;
            a[o][q] = a[q][o] = s * aop + c * aoq;
            for (int r = 0; r < 3; ++r) {
                double vp = v[r][p], vq = v[r][q];
                v[r][p] = c * vp - s * vq;
                v[r][q] = s * vp + c * vq;
            }
        }
        if (!rotated) break;
    }
}

/* The per-point covariance of PCL computeCovariances from k neighbour coordinates given in
 * (d2, index) order, regularised to u1u1' + u2u2' + eps*u3u3' (u sorted by singular value). */
static void cov_from_neighbours(const float* pts, const int* nn, int k, double eps, double c6[6]) {
    double mean[3] = {0, 0, 0};
    double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int j = 0; j < k; ++j) {
        const float* pt = pts + 3 * nn[j];
        mean[0] += pt[0];
        mean[1] += pt[1];
        mean[2] += pt[2];
        cov[0][0] += (double)(pt[0] * pt[0]);
        cov[1][0] += (double)(pt[1] * pt[0]);
        cov[1][1] += (double)(pt[1] * pt[1]);
        cov[2][0] += (double)(pt[2] * pt[0]);
        cov[2][1] += (double)(pt[2] * pt[1]);
        cov[2][2] += (double)(pt[2] * pt[2]);
    }
    double kd = (double)k;
    mean[0] /= kd; mean[1] /= kd; mean[2] /= kd;
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b <= a; ++b) {
            cov[a][b] /= kd;
            cov[a][b] -= mean[a] * mean[b];
            cov[b][a] = cov[a][b];
        }
    double v[3][3];
    jacobi3(cov, v);
    /* singular values = |eigenvalues|; order descending, ties by lower column index */
    double sv[3] = {fabs(cov[0][0]), fabs(cov[1][1]), fabs(cov[2][2])};
    int ord[3] = {0, 1, 2};
    for (int i = 0; i < 3; ++i)
        for (int j = i + 1; j < 3; ++j)
            if (sv[ord[j]] > sv[ord[i]]) { int t = ord[i]; ord[i] = ord[j]; ord[j] = t; }
    /* cov = sum_k w_k * col_k col_k', k in SVD order, w = (1, 1, eps) */
    double C[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int kk = 0; kk < 3; ++kk) {
        int col = ord[kk];
        double w = (kk == 2) ? eps : 1.0;
        double u0 = w * v[0][col], u1 = w * v[1][col], u2 = w * v[2][col];
        C[0][0] += u0 * v[0][col];
        C[0][1] += u0 * v[1][col];
        C[0][2] += u0 * v[2][col];
        C[1][1] += u1 * v[1][col];
        C[1][2] += u1 * v[2][col];
        C[2][2] += u2 * v[2][col];
    }
    c6[0] = C[0][0]; c6[1] = C[0][1]; c6[2] = C[0][2];
    c6[3] = C[1][1]; c6[4] = C[1][2]; c6[5] = C[2][2];
}

static void compute_covariances(const kdtree* t, int k, double eps, int threads, double* c6) {
    int n = t->n;
    (void)threads;
#pragma omp parallel num_threads(threads > 1 ? threads : 1) if (threads > 1)
    {
        int* nn = (int*)malloc((size_t)k * sizeof(int));
        float* d2 = (float*)malloc((size_t)k * sizeof(float));
#pragma omp for schedule(dynamic, 1024)
        for (int i = 0; i < n; ++i) {
            kd_knn(t, t->pts + 3 * i, k, nn, d2);
            cov_from_neighbours(t->pts, nn, k, eps, c6 + 6 * (size_t)i);
        }
        free(nn);
        free(d2);
    }
}

/* ------------------------------------------------------------------------------------ */
/* GICP state                                                                            */
/* ------------------------------------------------------------------------------------ */
/* moment layout: [0] S0 = sum r0'M r0; [1..12] B[a][i] = sum (M r0)_a w_i; [13..72]
 * Q[ab][ij] = sum M_ab w_i w_j (ab over 00,01,02,11,12,22; ij over the upper pairs of 4);
 * [73] count; w = (s - ctr, 1), r0 = fl(fl(T0 s) - q) */
#define MOM_VALS 74
struct ref_gicp {
    ref_params prm;
    float* src; int ns; int src_dirty;
    float* tgt; int nt; int tgt_dirty;
    kdtree tree_src, tree_tgt;
    double* cov_src; double* cov_tgt; /* 6 per point */
    /* per-align scratch */
    float* out;       /* output cloud (guess applied), ns x 3 */
    double* mahal;    /* ns x 9 row-major */
    int* corr_src; int* corr_tgt; int m;
    int n_evals;
    /* moment-form objective (prm.objective == 1): taken at the correspondence transform T0 */
    double mom[MOM_VALS];
    float T0[4][4];
    double ctr[3];
    /* summation-order ledger (r06, ref_set_sum_order): 0 the order above, 1 the engine's fixed tree over
     * sum_perm, 2 reversed sequential, 3 sequential over sum_perm */
    int sum_mode;
    int mahal_upper;    /* 1: the Mahalanobis matrix's upper triangle mirrored (the engine's 6-entry storage) */
    uint32_t* sum_perm; /* ns entries: stream position -> source index */
    int* sum_tj;        /* per source index: its correspondence slot, -1 = rejected (scratch) */
};

void ref_default_params(ref_params* p) {
    p->max_iterations = 100;
    p->transformation_epsilon = 4e-3;
    p->rotation_epsilon = 2e-3;
    p->max_corr_dist = 4e-2;
    p->gicp_epsilon = 1e-3;
    p->k_correspondences = 20;
    p->max_inner_iterations = 20;
    p->fixed_iterations = 0;
    p->threads = 1;
    p->objective = 0;
    p->solver = 0;
    p->variant = 0;
}

ref_gicp* ref_create(const ref_params* p) {
    ref_gicp* g = (ref_gicp*)calloc(1, sizeof(ref_gicp));
    if (p) g->prm = *p;
    else ref_default_params(&g->prm);
    return g;
}

int ref_set_params(ref_gicp* g, const ref_params* p) {
    if (!g || !p) return REF_E_INVALID;
    g->prm = *p;
    return REF_OK;
}

static void free_sum_order(ref_gicp* g) {
    free(g->sum_perm); free(g->sum_tj);
    g->sum_perm = NULL; g->sum_tj = NULL; g->sum_mode = 0;
}

static void free_scratch(ref_gicp* g) {
    free(g->out); free(g->mahal); free(g->corr_src); free(g->corr_tgt);
    g->out = NULL; g->mahal = NULL; g->corr_src = g->corr_tgt = NULL; g->m = 0;
}

void ref_destroy(ref_gicp* g) {
    if (!g) return;
    kd_free(&g->tree_src); kd_free(&g->tree_tgt);
    free(g->src); free(g->tgt); free(g->cov_src); free(g->cov_tgt);
    free_scratch(g);
    free_sum_order(g);
    free(g);
}

static float* copy_xyz(const float* xyz, size_t n, size_t stride, int* bad) {
    float* o = (float*)malloc((n ? n : 1) * 3 * sizeof(float));
    const char* base = (const char*)xyz;
    *bad = 0;
    for (size_t i = 0; i < n; ++i) {
        const float* p = (const float*)(base + i * stride);
        o[3 * i] = p[0]; o[3 * i + 1] = p[1]; o[3 * i + 2] = p[2];
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) *bad = 1;
    }
    return o;
}

int ref_set_source(ref_gicp* g, const float* xyz, size_t n, size_t stride) {
    free_sum_order(g);  /* a stream order belongs to one source cloud */
    if (!g || (!xyz && n) || stride < 12) return REF_E_INVALID;
    int bad;
    free(g->src);
    g->src = copy_xyz(xyz, n, stride, &bad);
    g->ns = (int)n;
    g->src_dirty = 1;
    free(g->cov_src); g->cov_src = NULL; /* setInputSource resets input_covariances_ */
    return bad ? REF_E_NONFINITE : REF_OK;
}

int ref_set_target(ref_gicp* g, const float* xyz, size_t n, size_t stride) {
    if (!g || (!xyz && n) || stride < 12) return REF_E_INVALID;
    int bad;
    free(g->tgt);
    g->tgt = copy_xyz(xyz, n, stride, &bad);
    g->nt = (int)n;
    g->tgt_dirty = 1;
    free(g->cov_tgt); g->cov_tgt = NULL; /* setInputTarget resets target_covariances_ */
    return bad ? REF_E_NONFINITE : REF_OK;
}

/* Registration::initCompute / ICP::initComputeReciprocal + computeCovariances x2 */
static int prepare(ref_gicp* g) {
    int k = g->prm.k_correspondences;
    if (g->ns <= 0 || g->nt <= 0) return REF_E_INVALID;
    if (k > g->ns || k > g->nt) return REF_E_TOO_FEW_POINTS;
    if (g->tgt_dirty) {
        kd_free(&g->tree_tgt);
        kd_build(&g->tree_tgt, g->tgt, g->nt);
        g->tgt_dirty = 0;
    }
    if (g->src_dirty) {
        kd_free(&g->tree_src);
        kd_build(&g->tree_src, g->src, g->ns);
        g->src_dirty = 0;
    }
    if (!g->cov_tgt) {
        g->cov_tgt = (double*)malloc((size_t)g->nt * 6 * sizeof(double));
        compute_covariances(&g->tree_tgt, k, g->prm.gicp_epsilon, g->prm.threads, g->cov_tgt);
    }
    if (!g->cov_src) {
        g->cov_src = (double*)malloc((size_t)g->ns * 6 * sizeof(double));
        compute_covariances(&g->tree_src, k, g->prm.gicp_epsilon, g->prm.threads, g->cov_src);
    }
    return REF_OK;
}

/* ------------------------------------------------------------------------------------ */
/* applyState / computeRDerivative / functor                                             */
/* ------------------------------------------------------------------------------------ */
typedef struct { float w, x, y, z; } quatf;

static quatf quat_axis(float angle, int axis) {
    quatf q;
    float ha = 0.5f * angle;
    /* glibc sincosf: gcc-built PCL / Eigen get cos(ha), sin(ha) from one sincosf call (gcc's sincos pass);
     * named explicitly so the oracle does not depend on its own compiler forming it */
    float s, cw;
    sincosf(ha, &s, &cw);
    q.w = cw;
    q.x = axis == 0 ? s : 0.f;
    q.y = axis == 1 ? s : 0.f;
    q.z = axis == 2 ? s : 0.f;
    /* Eigen: vec() = sin(ha) * axis -> s * 0 = 0, s * 1 = s */
    return q;
}

static quatf quat_mul(quatf a, quatf b) {
    quatf r;
    r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
    r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
    r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
    r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
    return r;
}

/* applyState(t = I, x): R = AngleAxisf(x5,Z)*AngleAxisf(x4,Y)*AngleAxisf(x3,X) */
static void apply_state(const double x[6], float T[4][4]) {
    quatf q = quat_mul(quat_mul(quat_axis((float)x[5], 2), quat_axis((float)x[4], 1)),
                       quat_axis((float)x[3], 0));
    float tx = 2.0f * q.x, ty = 2.0f * q.y, tz = 2.0f * q.z;
    float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    identity4(T);
    T[0][0] = 1.0f - (tyy + tzz);
    T[0][1] = txy - twz;
    T[0][2] = txz + twy;
    T[1][0] = txy + twz;
    T[1][1] = 1.0f - (txx + tzz);
    T[1][2] = tyz - twx;
    T[2][0] = txz - twy;
    T[2][1] = tyz + twx;
    T[2][2] = 1.0f - (txx + tyy);
    /* t.col(3) += (x0, x1, x2, 0) on t = I */
    T[0][3] = 0.0f + (float)x[0];
    T[1][3] = 0.0f + (float)x[1];
    T[2][3] = 0.0f + (float)x[2];
}

void ref_apply_state(const double x[6], float out_cm[16]) {
    float T[4][4];
    apply_state(x, T);
    rm_to_cm(T, out_cm);
}

/* matricesInnerProd(dR, Rsum) = sum_ij dR(j,i) * Rsum(i,j) */
static double inner_prod(const double a[3][3], const double b[3][3]) {
    double r = 0.;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r += a[j][i] * b[i][j];
    return r;
}

static void r_derivative(const double x[6], const double R[3][3], double g[6]) {
    double phi = x[3], theta = x[4], psi = x[5];
    double cphi, sphi, ctheta, stheta, cpsi, spsi; /* glibc sincos, as gcc-built PCL calls it */
    sincos(phi, &sphi, &cphi);
    sincos(theta, &stheta, &ctheta);
    sincos(psi, &spsi, &cpsi);
    double dphi[3][3], dtheta[3][3], dpsi[3][3];
    dphi[0][0] = 0.; dphi[1][0] = 0.; dphi[2][0] = 0.;
    dphi[0][1] = sphi * spsi + cphi * cpsi * stheta;
    dphi[1][1] = -cpsi * sphi + cphi * spsi * stheta;
    dphi[2][1] = cphi * ctheta;
    dphi[0][2] = cphi * spsi - cpsi * sphi * stheta;
    dphi[1][2] = -cphi * cpsi - sphi * spsi * stheta;
    dphi[2][2] = -ctheta * sphi;

    dtheta[0][0] = -cpsi * stheta;
    dtheta[1][0] = -spsi * stheta;
    dtheta[2][0] = -ctheta;
    dtheta[0][1] = cpsi * ctheta * sphi;
    dtheta[1][1] = ctheta * sphi * spsi;
    dtheta[2][1] = -sphi * stheta;
    dtheta[0][2] = cphi * cpsi * ctheta;
    dtheta[1][2] = cphi * ctheta * spsi;
    dtheta[2][2] = -cphi * stheta;

    dpsi[0][0] = -ctheta * spsi;
    dpsi[1][0] = cpsi * ctheta;
    dpsi[2][0] = 0.;
    dpsi[0][1] = -cphi * cpsi - sphi * spsi * stheta;
    dpsi[1][1] = -cphi * spsi + cpsi * sphi * stheta;
    dpsi[2][1] = 0.;
    dpsi[0][2] = cpsi * sphi - cphi * spsi * stheta;
    dpsi[1][2] = sphi * spsi + cphi * cpsi * stheta;
    dpsi[2][2] = 0.;

    g[3] = inner_prod(dphi, R);
    g[4] = inner_prod(dtheta, R);
    g[5] = inner_prod(dpsi, R);
}

/* One pass over the correspondences: want_f / want_g select the functor flavour
 * (operator(), df, fdf).  Sums run sequentially in correspondence order (threads <= 1). */
typedef struct { double f; double gt[3]; double R[3][3]; } fdf_acc;

static void fdf_range(const ref_gicp* g, const float A[4][4], int c0, int c1, fdf_acc* acc) {
    memset(acc, 0, sizeof(*acc));
    for (int c = c0; c < c1; ++c) {
        int i = g->corr_src[c], j = g->corr_tgt[c];
        const float* ps = g->out + 3 * (size_t)i;
        const float* pt = g->tgt + 3 * (size_t)j;
        float pp[3];
        xform(A, ps, pp);
        double res[3] = {(double)(pp[0] - pt[0]), (double)(pp[1] - pt[1]), (double)(pp[2] - pt[2])};
        const double* M = g->mahal + 9 * (size_t)i;
        double tmp[3];
        for (int r = 0; r < 3; ++r) {
            double a = M[3 * r + 0] * res[0];
            a = a + M[3 * r + 1] * res[1];
            a = a + M[3 * r + 2] * res[2];
            tmp[r] = a;
        }
        double d = res[0] * tmp[0];
        d = d + res[1] * tmp[1];
        d = d + res[2] * tmp[2];
        acc->f += d;
        acc->gt[0] += tmp[0]; acc->gt[1] += tmp[1]; acc->gt[2] += tmp[2];
        /* base_transformation_ = I, so pp = p_src exactly */
        double s3[3] = {ps[0], ps[1], ps[2]};
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) acc->R[a][b] += s3[a] * tmp[b];
    }
}

static const int kSymA[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
static const int kSymW[10][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {1, 1}, {1, 2}, {1, 3}, {2, 2}, {2, 3}, {3, 3}};
static int sym_a(int a, int b) { static const int t[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}}; return t[a][b]; }
static int sym_w(int i, int j) {
    static const int t[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
    return t[i][j];
}

/* One pass over correspondences [c0, c1) at T0: the 74 moments of the quadratic objective
 * (a contiguous range is one rank's share in the N > 1 decomposition). */
static void moments_build_range(ref_gicp* g, const float T0[4][4], int c0, int c1) {
    memcpy(g->T0, T0, sizeof(g->T0));
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < g->ns; ++i)
        for (int a = 0; a < 3; ++a) {
            float v = g->out[3 * (size_t)i + a];
            if (v < lo[a]) lo[a] = v;
            if (v > hi[a]) hi[a] = v;
        }
    for (int a = 0; a < 3; ++a) g->ctr[a] = (double)(0.5f * (lo[a] + hi[a]));
    double* mo = g->mom;
    memset(mo, 0, sizeof(g->mom));
    for (int c = c0; c < c1; ++c) {
        int i = g->corr_src[c], j = g->corr_tgt[c];
        const float* ps = g->out + 3 * (size_t)i;
        const float* pt = g->tgt + 3 * (size_t)j;
        float pp[3];
        xform(T0, ps, pp);
        double r0[3] = {(double)(pp[0] - pt[0]), (double)(pp[1] - pt[1]), (double)(pp[2] - pt[2])};
        const double* M = g->mahal + 9 * (size_t)i;
        double w[4] = {(double)ps[0] - g->ctr[0], (double)ps[1] - g->ctr[1], (double)ps[2] - g->ctr[2], 1.0};
        double Mr[3];
        for (int a = 0; a < 3; ++a) Mr[a] = M[3 * a] * r0[0] + M[3 * a + 1] * r0[1] + M[3 * a + 2] * r0[2];
        mo[0] += r0[0] * Mr[0] + r0[1] * Mr[1] + r0[2] * Mr[2];
        for (int a = 0; a < 3; ++a)
            for (int k = 0; k < 4; ++k) mo[1 + 4 * a + k] += Mr[a] * w[k];
        for (int p = 0; p < 6; ++p) {
            double mab = M[3 * kSymA[p][0] + kSymA[p][1]];
            for (int q = 0; q < 10; ++q) mo[13 + 10 * p + q] += mab * (w[kSymW[q][0]] * w[kSymW[q][1]]);
        }
        mo[73] += 1.0;
    }
}

static void moments_build(ref_gicp* g, const float T0[4][4]) { moments_build_range(g, T0, 0, g->m); }

/* f / grad at x from the moments: r(x) = r0 + Y w, Y = [dR | dR ctr + dt], dA = A(x) - T0 */
static void moments_eval(ref_gicp* g, const double x[6], double* f, double grad[6]) {
    float A[4][4];
    apply_state(x, A);
    const double* mo = g->mom;
    double Y[3][4];
    for (int a = 0; a < 3; ++a) {
        double u = (double)A[a][3] - (double)g->T0[a][3];
        for (int k = 0; k < 3; ++k) {
            Y[a][k] = (double)A[a][k] - (double)g->T0[a][k];
            u += Y[a][k] * g->ctr[k];
        }
        Y[a][3] = u;
    }
    /* G[b][i] = sum w_i (M r)_b = B[b][i] + sum_{c,j} Y[c][j] Q[bc][ij] */
    double G[3][4];
    for (int b = 0; b < 3; ++b)
        for (int i = 0; i < 4; ++i) {
            double acc = 0.0;
            for (int c = 0; c < 3; ++c)
                for (int j = 0; j < 4; ++j) acc += Y[c][j] * mo[13 + 10 * sym_a(b, c) + sym_w(i, j)];
            G[b][i] = mo[1 + 4 * b + i] + acc;
        }
    double m = mo[73];
    g->n_evals++;
    if (f) {
        double corr = 0.0;
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 4; ++i) corr += Y[a][i] * (mo[1 + 4 * a + i] + G[a][i]);
        *f = (mo[0] + corr) / m;
    }
    if (grad) {
        double s = 2.0 / m;
        double R[3][3];
        for (int b = 0; b < 3; ++b) grad[b] = G[b][3] * s;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) R[a][b] = (G[b][a] + g->ctr[a] * G[b][3]) * s;
        r_derivative(x, R, grad);
    }
}

/* ------------------------------------------------------------------------------------ */
/* Gauss-Newton solver on the moment form (ref_params.solver = 1): checker for the engine's  */
/* MGICP_SOLVER_GN.  Not a PCL 1.8.1 algorithm: PCL only has the BFGS solver; GN is the      */
/* north-star's "6x6 J'WJ / J'Wr" solve, held to PCL by SURVEY 8c's fixed-point protocol.    */
/* Pose update about the centre c: p^ = T s - c, r = p^ + c - q, T <- [Exp(w) | v] * T,      */
/* J_i = [-[p^_i]x | I].  J'MJ and J'Mr at any pose are linear in the 74 moments.            */
/* ------------------------------------------------------------------------------------ */
static void gn_pose_from_float(const float T[4][4], double R[3][3], double t[3]) {
    for (int a = 0; a < 3; ++a) {
        for (int k = 0; k < 3; ++k) R[a][k] = (double)T[a][k];
        t[a] = (double)T[a][3];
    }
}

/* f*m, and (when H != NULL) H = sum J'MJ, gv = sum J'Mr (half gradient) at pose (R, t) */
static double gn_eval(const ref_gicp* g, const double R[3][3], const double t[3], double H[6][6],
                      double gv[6]) {
    const double* mo = g->mom;
    const double* c = g->ctr;
    double Y[3][4], E[3][4];
    for (int a = 0; a < 3; ++a) {
        double u = t[a] - (double)g->T0[a][3];
        double e = t[a] - c[a];
        for (int k = 0; k < 3; ++k) {
            Y[a][k] = R[a][k] - (double)g->T0[a][k];
            u += Y[a][k] * c[k];
            E[a][k] = R[a][k];
            e += R[a][k] * c[k];
        }
        Y[a][3] = u;
        E[a][3] = e;
    }
    double G[3][4]; /* sum (M r)_b w_i */
    for (int b = 0; b < 3; ++b)
        for (int i = 0; i < 4; ++i) {
            double acc = mo[1 + 4 * b + i];
            for (int cc = 0; cc < 3; ++cc)
                for (int j = 0; j < 4; ++j) acc += Y[cc][j] * mo[13 + 10 * sym_a(b, cc) + sym_w(i, j)];
            G[b][i] = acc;
        }
    double fm = mo[0];
    for (int a = 0; a < 3; ++a)
        for (int i = 0; i < 4; ++i) fm += Y[a][i] * (mo[1 + 4 * a + i] + G[a][i]);
    if (!H) return fm;
    /* Z[e][a] = sum p^_e (M r)_a ; N[e][a][b] = sum p^_e M_ab ; K[e][f][a][b] = sum p^_e p^_f M_ab */
    double Z[3][3], N[3][3][3], K[3][3][3][3];
    for (int e = 0; e < 3; ++e)
        for (int a = 0; a < 3; ++a) {
            double z = 0.0;
            for (int i = 0; i < 4; ++i) z += E[e][i] * G[a][i];
            Z[e][a] = z;
        }
    for (int e = 0; e < 3; ++e)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                double s = 0.0;
                for (int i = 0; i < 4; ++i) s += E[e][i] * mo[13 + 10 * sym_a(a, b) + sym_w(i, 3)];
                N[e][a][b] = s;
            }
    for (int e = 0; e < 3; ++e)
        for (int f = 0; f < 3; ++f)
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double s = 0.0;
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j < 4; ++j)
                            s += E[e][i] * E[f][j] * mo[13 + 10 * sym_a(a, b) + sym_w(i, j)];
                    K[e][f][a][b] = s;
                }
    static const int eps[3][3][3] = {{{0, 0, 0}, {0, 0, 1}, {0, -1, 0}},
                                     {{0, 0, -1}, {0, 0, 0}, {1, 0, 0}},
                                     {{0, 1, 0}, {-1, 0, 0}, {0, 0, 0}}};
    /* rotation rows: J_w = -[p^]x, so J_w' M r = p^ x (M r), J_w' M J_v = [p^]x M,
     * J_w' M J_w = -[p^]x M [p^]x */
    for (int i = 0; i < 3; ++i) {
        double s = 0.0;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) s += eps[i][j][k] * Z[j][k];
        gv[i] = s;
        gv[3 + i] = G[i][3];
    }
    for (int i = 0; i < 3; ++i)
        for (int l = 0; l < 3; ++l) {
            double wv = 0.0, ww = 0.0;
            for (int j = 0; j < 3; ++j)
                for (int k = 0; k < 3; ++k) {
                    if (!eps[i][j][k]) continue;
                    wv += eps[i][j][k] * N[j][k][l];
                    for (int mm = 0; mm < 3; ++mm)
                        for (int n = 0; n < 3; ++n)
                            if (eps[mm][n][l]) ww -= eps[i][j][k] * eps[mm][n][l] * K[j][n][k][mm];
                }
            H[i][3 + l] = wv;
            H[3 + l][i] = wv;
            H[i][l] = ww;
            H[3 + i][3 + l] = mo[13 + 10 * sym_a(i, l) + 9];
        }
    return fm;
}

/* Cholesky solve of H x = -b; 0 on success */
static int gn_chol_solve(double H[6][6], const double b[6], double x[6]) {
    double L[6][6];
    memset(L, 0, sizeof(L));
    for (int j = 0; j < 6; ++j) {
        double d = H[j][j];
        for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
        if (!(d > 0.0)) return -1;
        L[j][j] = sqrt(d);
        for (int i = j + 1; i < 6; ++i) {
            double s = H[i][j];
            for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
            L[i][j] = s / L[j][j];
        }
    }
    double y[6];
    for (int i = 0; i < 6; ++i) {
        double s = -b[i];
        for (int k = 0; k < i; ++k) s -= L[i][k] * y[k];
        y[i] = s / L[i][i];
    }
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s -= L[k][i] * x[k];
        x[i] = s / L[i][i];
    }
    return 0;
}

/* Exp of a rotation vector (Rodrigues) */
static void gn_exp(const double w[3], double Rx[3][3]) {
    double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    double th = sqrt(th2);
    double a, b;
    if (th < 1e-8) {
        a = 1.0 - th2 / 6.0;
        b = 0.5 - th2 / 24.0;
    } else {
        double sth, cth;
        sincos(th, &sth, &cth);
        a = sth / th;
        b = (1.0 - cth) / th2;
    }
    double W[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double w2 = W[i][0] * W[0][j] + W[i][1] * W[1][j] + W[i][2] * W[2][j];
            Rx[i][j] = (i == j ? 1.0 : 0.0) + a * W[i][j] + b * w2;
        }
}

static void gn_apply(const double R[3][3], const double t[3], const double c[3], const double xi[6],
                     double s, double R2[3][3], double t2[3]) {
    double w[3] = {s * xi[0], s * xi[1], s * xi[2]};
    double Rx[3][3];
    gn_exp(w, Rx);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) R2[i][j] = Rx[i][0] * R[0][j] + Rx[i][1] * R[1][j] + Rx[i][2] * R[2][j];
        t2[i] = Rx[i][0] * (t[0] - c[0]) + Rx[i][1] * (t[1] - c[1]) + Rx[i][2] * (t[2] - c[2]) + c[i] + s * xi[3 + i];
    }
}

/* Inner GN solve on the correspondence set of the moments (taken at T = T0); T <- solution.
 * 0 = accepted, -1 = too few correspondences / singular normal matrix (PCL would throw). */
static int estimate_gn(ref_gicp* g, float T[4][4]) {
    if (g->mom[73] < 4) return -1;
    double R[3][3], t[3];
    gn_pose_from_float(T, R, t);
    double H[6][6], gv[6];
    double fm = gn_eval(g, R, t, H, gv);
    g->n_evals++;
    for (int it = 0; it < g->prm.max_inner_iterations; ++it) {
        double xi[6];
        if (gn_chol_solve(H, gv, xi)) return -1;
        double R2[3][3], t2[3], f2 = 0.0, s = 1.0;
        int ok = 0;
        for (int h = 0; h < 8; ++h, s *= 0.5) {
            gn_apply(R, t, g->ctr, xi, s, R2, t2);
            f2 = gn_eval(g, R2, t2, NULL, NULL);
            if (f2 <= fm) { ok = 1; break; }
        }
        if (!ok) break; /* no descent along the GN direction: at the minimum to rounding */
        memcpy(R, R2, sizeof(R));
        memcpy(t, t2, sizeof(t));
        double step = 0.0;
        for (int k = 0; k < 6; ++k) step = fmax(step, fabs(s * xi[k]));
        if (step < 1e-12) break;
        fm = gn_eval(g, R, t, H, gv);
        g->n_evals++;
    }
    for (int a = 0; a < 3; ++a) {
        for (int k = 0; k < 3; ++k) T[a][k] = (float)R[a][k];
        T[a][3] = (float)t[a];
    }
    return 0;
}

/* ---- summation-order ledger (r06) ------------------------------------------
 * The engine sums a pass over a FIXED tree keyed to its source stream order (mgicp_kernels.hip
 * fdf_soa_body / chunk_store / wave_tickets / wave_total): chunks of 1024 stream positions; in a chunk
 * the accepted correspondences are compacted in stream order into groups of 4, lane l of the wave takes
 * groups l, l + 64, ... and accumulates their terms in order; the 64 lane sums meet in the shuffle tree
 * (pairs l, l + d for d = 32 ... 1); a super = 32 consecutive chunks, summed in chunk order from the
 * first; the total: lane l sums supers l, l + 64, ... from 0.0, then the same shuffle tree.  Restated
 * here over any stream order (sum_perm), so the oracle can run the BFGS on the engine's sums, on
 * another order's, or on a reversed sequential sum -- the spread of iterations and T over orders. */
static void acc_add(fdf_acc* a, const fdf_acc* b) {
    a->f = a->f + b->f;
    for (int k = 0; k < 3; ++k) a->gt[k] = a->gt[k] + b->gt[k];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a->R[r][c] = a->R[r][c] + b->R[r][c];
}
static void lane_tree(fdf_acc* lanes) { /* lanes[0] = the 64-lane shuffle tree */
    for (int off = 32; off > 0; off >>= 1)
        for (int i = 0; i < off; ++i) acc_add(&lanes[i], &lanes[i + off]);
}
static void fdf_tree(ref_gicp* g, const float A[4][4], fdf_acc* tot) {
    const int ns = g->ns, nch = (ns + 1023) / 1024, nsup = (nch + 31) / 32;
    fdf_acc* chunk = (fdf_acc*)calloc((size_t)nch, sizeof(fdf_acc));
    fdf_acc lanes[64], one;
    int* list = (int*)malloc(1024 * sizeof(int));
    for (int j = 0; j < nch; ++j) {
        int cnt = 0;
        for (int p = 1024 * j; p < ns && p < 1024 * (j + 1); ++p) {
            const int slot = g->sum_tj[g->sum_perm[p]];
            if (slot >= 0) list[cnt++] = slot;
        }
        memset(lanes, 0, sizeof(lanes));
        for (int k = 0; k < cnt; ++k) {
            const int lane = (k / 4) % 64;
            fdf_range(g, A, list[k], list[k] + 1, &one);
            acc_add(&lanes[lane], &one);
        }
        lane_tree(lanes);
        chunk[j] = lanes[0];
    }
    memset(lanes, 0, sizeof(lanes));
    for (int sj = 0; sj < nsup; ++sj) {
        fdf_acc a = chunk[32 * sj];
        for (int q = 1; q < 32 && 32 * sj + q < nch; ++q) acc_add(&a, &chunk[32 * sj + q]);
        acc_add(&lanes[sj % 64], &a);
    }
    lane_tree(lanes);
    *tot = lanes[0];
    free(list);
    free(chunk);
}

int ref_set_mahalanobis_upper(ref_gicp* g, int on) {
    if (!g) return REF_E_INVALID;
    g->mahal_upper = on != 0;
    return REF_OK;
}

int ref_set_sum_order(ref_gicp* g, int mode, const uint32_t* perm, size_t n) {
    if (!g || mode < 0 || mode > 3) return REF_E_INVALID;
    free_sum_order(g);
    if (mode == 1 || mode == 3) {
        if (!perm || n != (size_t)g->ns) return REF_E_INVALID;
        g->sum_perm = (uint32_t*)malloc(n * sizeof(uint32_t));
        g->sum_tj = (int*)malloc(n * sizeof(int));
        char* seen = (char*)calloc(n, 1);
        for (size_t p = 0; p < n; ++p) {
            if (perm[p] >= n || seen[perm[p]]) { free(seen); free_sum_order(g); return REF_E_INVALID; }
            seen[perm[p]] = 1;
            g->sum_perm[p] = perm[p];
        }
        free(seen);
    }
    g->sum_mode = mode;
    return REF_OK;
}

/* the raw 13 sums of one pass in the current summation mode (ledger checks against the engine's
 * mgicp_debug_fdf_sums): f, grad_t[3], Rsum[3][3] row-major, then the count */
int ref_fdf_mode_sums(ref_gicp* g, const double x[6], double out14[14]);

static void functor_eval(ref_gicp* g, const double x[6], double* f, double grad[6]) {
    if (g->prm.objective == 1) {
        moments_eval(g, x, f, grad);
        return;
    }
    float A[4][4];
    apply_state(x, A);
    int m = g->m;
    int nt = g->prm.threads > 1 ? g->prm.threads : 1;
    fdf_acc tot;
    if (g->sum_mode) {
        if (g->sum_mode == 2) {  /* reversed sequential */
            fdf_acc one;
            memset(&tot, 0, sizeof(tot));
            for (int c = m - 1; c >= 0; --c) { fdf_range(g, A, c, c + 1, &one); acc_add(&tot, &one); }
        } else {
            for (int i = 0; i < g->ns; ++i) g->sum_tj[i] = -1;
            for (int c = 0; c < m; ++c) g->sum_tj[g->corr_src[c]] = c;
            if (g->sum_mode == 1) {
                fdf_tree(g, A, &tot);
            } else {  /* sequential over sum_perm */
                fdf_acc one;
                memset(&tot, 0, sizeof(tot));
                for (int p = 0; p < g->ns; ++p) {
                    const int c = g->sum_tj[g->sum_perm[p]];
                    if (c >= 0) { fdf_range(g, A, c, c + 1, &one); acc_add(&tot, &one); }
                }
            }
        }
    } else if (nt == 1) {
        fdf_range(g, A, 0, m, &tot);
    } else {
        fdf_acc* parts = (fdf_acc*)calloc((size_t)nt, sizeof(fdf_acc));
#pragma omp parallel for num_threads(nt) schedule(static, 1)
        for (int t = 0; t < nt; ++t) {
            int c0 = (int)((long long)m * t / nt), c1 = (int)((long long)m * (t + 1) / nt);
            fdf_range(g, A, c0, c1, &parts[t]);
        }
        tot = parts[0];
        for (int t = 1; t < nt; ++t) {
            tot.f += parts[t].f;
            for (int a = 0; a < 3; ++a) {
                tot.gt[a] += parts[t].gt[a];
                for (int b = 0; b < 3; ++b) tot.R[a][b] += parts[t].R[a][b];
            }
        }
        free(parts);
    }
    g->n_evals++;
    if (f) *f = tot.f / m;
    if (grad) {
        double s = 2.0 / m;
        grad[0] = tot.gt[0] * s; grad[1] = tot.gt[1] * s; grad[2] = tot.gt[2] * s;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) tot.R[a][b] *= s;
        r_derivative(x, tot.R, grad);
    }
}

int ref_fdf_mode_sums(ref_gicp* g, const double x[6], double out14[14]) {
    if (!g || !out14 || g->m <= 0) return REF_E_INVALID;
    float A[4][4];
    apply_state(x, A);
    fdf_acc tot;
    if (g->sum_mode == 1 || g->sum_mode == 3) {
        for (int i = 0; i < g->ns; ++i) g->sum_tj[i] = -1;
        for (int c = 0; c < g->m; ++c) g->sum_tj[g->corr_src[c]] = c;
    }
    if (g->sum_mode == 1) {
        fdf_tree(g, A, &tot);
    } else {
        fdf_range(g, A, 0, g->m, &tot);
    }
    out14[0] = tot.f;
    for (int a = 0; a < 3; ++a) {
        out14[1 + a] = tot.gt[a];
        for (int b = 0; b < 3; ++b) out14[4 + 3 * a + b] = tot.R[a][b];
    }
    out14[13] = (double)g->m;
    return REF_OK;
}

int ref_fdf_sums(ref_gicp* g, const double x[6], int c0, int c1, double out14[14]) {
    if (!g || !out14 || c0 < 0 || c1 > g->m || c0 > c1) return REF_E_INVALID;
    float A[4][4];
    apply_state(x, A);
    fdf_acc acc;
    fdf_range(g, A, c0, c1, &acc);
    out14[0] = acc.f;
    for (int a = 0; a < 3; ++a) {
        out14[1 + a] = acc.gt[a];
        for (int b = 0; b < 3; ++b) out14[4 + 3 * a + b] = acc.R[a][b];
    }
    out14[13] = (double)(c1 - c0);
    return REF_OK;
}

int ref_moments(ref_gicp* g, const float T0_cm[16], double out74[74]) {
    if (!g || !g->out || g->m <= 0) return REF_E_INVALID;
    float T0[4][4];
    cm_to_rm(T0_cm, T0);
    moments_build(g, T0);
    if (out74) memcpy(out74, g->mom, sizeof(g->mom));
    return REF_OK;
}

int ref_moments_range(ref_gicp* g, const float T0_cm[16], int c0, int c1, double out74[74]) {
    if (!g || !g->out || g->m <= 0 || c0 < 0 || c1 < c0 || c1 > g->m || !out74) return REF_E_INVALID;
    float T0[4][4];
    cm_to_rm(T0_cm, T0);
    moments_build_range(g, T0, c0, c1);
    memcpy(out74, g->mom, sizeof(g->mom));
    return REF_OK;
}

int ref_fdf(ref_gicp* g, const double x[6], double* f, double g6[6]) {
    if (!g || g->m <= 0) return REF_E_INVALID;
    functor_eval(g, x, f, g6);
    return REF_OK;
}

/* ------------------------------------------------------------------------------------ */
/* BFGS (registration/bfgs.h, GSL vector_bfgs2 port) -- Scalar = double, N = 6           */
/* ------------------------------------------------------------------------------------ */
enum { BFGS_NEG_EPS = -3, BFGS_NOT_STARTED = -2, BFGS_RUNNING = -1, BFGS_SUCCESS = 0, BFGS_NO_PROGRESS = 1 };

typedef struct {
    ref_gicp* g;
    double rho, sigma, tau1, tau2, tau3, step_size;
    int order, bracket_iters, section_iters;
    double f, gradient[6];
    double delta_f, fp0;
    double x0[6], dx0[6], dg0[6], g0[6], dx[6], p[6];
    double pnorm, g0norm;
    double f_alpha, df_alpha, x_alpha[6], g_alpha[6];
    double f_cache_key, df_cache_key, x_cache_key, g_cache_key;
} bfgs_t;

static double dot6(const double* a, const double* b) {
    double r = 0;
    for (int i = 0; i < 6; ++i) r += a[i] * b[i];
    return r;
}
static double norm6(const double* a) { return sqrt(dot6(a, a)); }

static void b_move_to(bfgs_t* b, double alpha) {
    for (int i = 0; i < 6; ++i) b->x_alpha[i] = b->x0[i] + alpha * b->p[i];
    b->x_cache_key = alpha;
}
static double b_slope(bfgs_t* b) { return dot6(b->g_alpha, b->p); }

static double b_apply_f(bfgs_t* b, double alpha) {
    if (alpha == b->f_cache_key) return b->f_alpha;
    b_move_to(b, alpha);
    functor_eval(b->g, b->x_alpha, &b->f_alpha, NULL);
    b->f_cache_key = alpha;
    return b->f_alpha;
}
static double b_apply_df(bfgs_t* b, double alpha) {
    if (alpha == b->df_cache_key) return b->df_alpha;
    b_move_to(b, alpha);
    if (alpha != b->g_cache_key) {
        functor_eval(b->g, b->x_alpha, NULL, b->g_alpha);
        b->g_cache_key = alpha;
    }
    b->df_alpha = b_slope(b);
    b->df_cache_key = alpha;
    return b->df_alpha;
}
static void b_apply_fdf(bfgs_t* b, double alpha, double* f, double* df) {
    if (alpha == b->f_cache_key && alpha == b->df_cache_key) {
        *f = b->f_alpha; *df = b->df_alpha;
        return;
    }
    if (alpha == b->f_cache_key || alpha == b->df_cache_key) {
        *f = b_apply_f(b, alpha);
        *df = b_apply_df(b, alpha);
        return;
    }
    b_move_to(b, alpha);
    functor_eval(b->g, b->x_alpha, &b->f_alpha, b->g_alpha);
    b->f_cache_key = alpha;
    b->g_cache_key = alpha;
    b->df_alpha = b_slope(b);
    b->df_cache_key = alpha;
    *f = b->f_alpha; *df = b->df_alpha;
}
static void b_update_position(bfgs_t* b, double alpha, double* x, double* f, double* g) {
    double fa, dfa;
    b_apply_fdf(b, alpha, &fa, &dfa);
    *f = b->f_alpha;
    memcpy(x, b->x_alpha, sizeof(double) * 6);
    memcpy(g, b->g_alpha, sizeof(double) * 6);
}
static void b_change_direction(bfgs_t* b) {
    memcpy(b->x_alpha, b->x0, sizeof(double) * 6);
    b->x_cache_key = 0.0;
    b->f_cache_key = 0.0;
    memcpy(b->g_alpha, b->g0, sizeof(double) * 6);
    b->g_cache_key = 0.0;
    b->df_alpha = b_slope(b);
    b->df_cache_key = 0.0;
}

static double poly3(const double c[4], double x) { /* Eigen::poly_eval (Horner) */
    double v = c[3];
    v = v * x + c[2];
    v = v * x + c[1];
    v = v * x + c[0];
    return v;
}
static void check_extremum(const double c[4], double x, double* xmin, double* fmin) {
    double y = poly3(c, x);
    if (y < *fmin) { *xmin = x; *fmin = y; }
}

static double b_interpolate(double a, double fa, double fpa, double b, double fb, double fpb,
                            double xmin, double xmax, int order, int variant) {
    double y, alpha, ymin, ymax, fmin;
    ymin = (xmin - a) / (b - a);
    ymax = (xmax - a) / (b - a);
    if (ymin > ymax) { double t = ymin; ymin = ymax; ymax = t; }
    /* PCL 1.8.1 tests !(fpb != fpa) here (GSL: GSL_IS_REAL(fpb)); restated as published */
    const int cubic = (variant & 2) ? isfinite(fpb) : (!(fpb != fpa) && fpb != INFINITY);
    if (order > 2 && cubic) {
        fpa = fpa * (b - a);
        fpb = fpb * (b - a);
        double eta = 3 * (fb - fa) - 2 * fpa - fpb;
        double xi = fpa + fpb - 2 * (fb - fa);
        double c[4] = {fa, fpa, eta, xi};
        y = ymin;
        fmin = poly3(c, ymin);
        check_extremum(c, ymax, &y, &fmin);
        /* real roots of c1 + 2 c2 y + 3 c3 y^2 */
        double qa = 3 * xi, qb = 2 * eta, qc = fpa;
        if (qa != 0.0) {
            double disc = qb * qb - 4 * qa * qc;
            if (disc >= 0.0) {
                double sq = sqrt(disc);
                double y0 = (-qb - sq) / (2 * qa), y1 = (-qb + sq) / (2 * qa);
                if (y0 > y1) { double t = y0; y0 = y1; y1 = t; }
                if (y0 > ymin && y0 < ymax) check_extremum(c, y0, &y, &fmin);
                if (y1 > ymin && y1 < ymax) check_extremum(c, y1, &y, &fmin);
            }
        } else if (qb != 0.0) {
            double y0 = -qc / qb;
            if (y0 > ymin && y0 < ymax) check_extremum(c, y0, &y, &fmin);
        }
    } else {
        fpa = fpa * (b - a);
        double fl = fa + ymin * (fpa + ymin * (fb - fa - fpa));
        double fh = fa + ymax * (fpa + ymax * (fb - fa - fpa));
        double c = 2 * (fb - fa - fpa); /* curvature */
        y = ymin;
        fmin = fl;
        if (fh < fmin) { y = ymax; fmin = fh; }
        if ((variant & 4) ? c > 0 : c > a) { /* PCL 1.8.1 compares against a (GSL: c > 0); restated as published */
            double z = -fpa / c;
            if (z > ymin && z < ymax) {
                double f = fa + z * (fpa + z * (fb - fa - fpa));
                if (f < fmin) { y = z; fmin = f; }
            }
        }
    }
    alpha = a + y * (b - a);
    return alpha;
}

static int b_line_search(bfgs_t* b, double rho, double sigma, double tau1, double tau2, double tau3,
                         int order, double alpha1, double* alpha_new) {
    double f0, fp0, falpha, falpha_prev, fpalpha, fpalpha_prev, delta, alpha_next;
    double alpha = alpha1, alpha_prev = 0.0;
    double a, bb, fa, fb, fpa, fpb;
    int i = 0;
    b_apply_fdf(b, 0.0, &f0, &fp0);
    falpha_prev = f0;
    fpalpha_prev = fp0;
    a = 0.0; bb = alpha;
    fa = f0; fb = 0.0;
    fpa = fp0; fpb = 0.0;
    while (i++ < b->bracket_iters) {
        falpha = b_apply_f(b, alpha);
        if (falpha > f0 + alpha * rho * fp0 || falpha >= falpha_prev) {
            a = alpha_prev; fa = falpha_prev; fpa = fpalpha_prev;
            bb = alpha; fb = falpha; fpb = NAN;
            break;
        }
        fpalpha = b_apply_df(b, alpha);
        if (fabs(fpalpha) <= -sigma * fp0) {
            *alpha_new = alpha;
            return BFGS_SUCCESS;
        }
        if (fpalpha >= 0) {
            a = alpha; fa = falpha; fpa = fpalpha;
            bb = alpha_prev; fb = falpha_prev; fpb = fpalpha_prev;
            break;
        }
        delta = alpha - alpha_prev;
        {
            double lower = alpha + delta;
            double upper = alpha + tau1 * delta;
            alpha_next = b_interpolate(alpha_prev, falpha_prev, fpalpha_prev, alpha, falpha,
                                       fpalpha, lower, upper, order, b->g->prm.variant);
        }
        alpha_prev = alpha;
        falpha_prev = falpha;
        fpalpha_prev = fpalpha;
        alpha = alpha_next;
    }
    while (i++ < b->section_iters) {
        delta = bb - a;
        {
            double lower = a + tau2 * delta;
            double upper = bb - tau3 * delta;
            alpha = b_interpolate(a, fa, fpa, bb, fb, fpb, lower, upper, order, b->g->prm.variant);
        }
        falpha = b_apply_f(b, alpha);
        if ((a - alpha) * fpa <= ((b->g->prm.variant & 32) ? 0.0 : DBL_EPSILON)) return BFGS_NO_PROGRESS;
        if (falpha > f0 + rho * alpha * fp0 || falpha >= fa) {
            bb = alpha; fb = falpha; fpb = NAN;
        } else {
            fpalpha = b_apply_df(b, alpha);
            if (fabs(fpalpha) <= -sigma * fp0) {
                *alpha_new = alpha;
                return BFGS_SUCCESS;
            }
            if (((bb - a) >= 0 && fpalpha >= 0) || ((bb - a) <= 0 && fpalpha <= 0)) {
                bb = a; fb = fa; fpb = fpa;
                a = alpha; fa = falpha; fpa = fpalpha;
            } else {
                a = alpha; fa = falpha; fpa = fpalpha;
            }
        }
    }
    return BFGS_SUCCESS;
}

static int b_minimize_init(bfgs_t* b, double* x) {
    b->delta_f = 0;
    memset(b->dx, 0, sizeof(b->dx));
    functor_eval(b->g, x, &b->f, b->gradient);
    memcpy(b->x0, x, sizeof(double) * 6);
    memcpy(b->g0, b->gradient, sizeof(double) * 6);
    b->g0norm = norm6(b->g0);
    for (int i = 0; i < 6; ++i) b->p[i] = b->gradient[i] * -1 / b->g0norm;
    b->pnorm = norm6(b->p);
    b->fp0 = -b->g0norm;
    memcpy(b->x_alpha, b->x0, sizeof(double) * 6);
    b->x_cache_key = 0;
    b->f_alpha = b->f;
    b->f_cache_key = 0;
    memcpy(b->g_alpha, b->g0, sizeof(double) * 6);
    b->g_cache_key = 0;
    b->df_alpha = b_slope(b);
    b->df_cache_key = 0;
    return BFGS_NOT_STARTED;
}

static int b_minimize_one_step(bfgs_t* b, double* x) {
    double alpha = 0.0, alpha1;
    double f0 = b->f;
    if (b->pnorm == 0.0 || b->g0norm == 0.0 || b->fp0 == 0) {
        memset(b->dx, 0, sizeof(b->dx));
        return BFGS_NO_PROGRESS;
    }
    if (b->delta_f < 0) {
        double del = fmax(-b->delta_f, 10 * DBL_EPSILON * fabs(f0));
        alpha1 = fmin(1.0, 2.0 * del / (-b->fp0));
    } else {
        alpha1 = fabs(b->step_size);
    }
    int status = b_line_search(b, b->rho, b->sigma, b->tau1, b->tau2, b->tau3, b->order, alpha1, &alpha);
    if (status != BFGS_SUCCESS) return status;
    b_update_position(b, alpha, x, &b->f, b->gradient);
    b->delta_f = b->f - f0;
    {
        double dxg, dgg, dxdg, dgnorm, A, B;
        for (int i = 0; i < 6; ++i) {
            b->dx0[i] = x[i] - b->x0[i];
            b->dx[i] = b->dx0[i];
            b->dg0[i] = b->gradient[i] - b->g0[i];
        }
        dxg = dot6(b->dx0, b->gradient);
        dgg = dot6(b->dg0, b->gradient);
        dxdg = dot6(b->dx0, b->dg0);
        dgnorm = norm6(b->dg0);
        if (dxdg != 0) {
            B = dxg / dxdg;
            A = -(1.0 + dgnorm * dgnorm / dxdg) * B + dgg / dxdg;
        } else {
            B = 0;
            A = 0;
        }
        for (int i = 0; i < 6; ++i) {
            b->p[i] = -A * b->dx0[i];
            b->p[i] += -B * b->dg0[i];
            b->p[i] += b->gradient[i];
        }
    }
    memcpy(b->g0, b->gradient, sizeof(double) * 6);
    memcpy(b->x0, x, sizeof(double) * 6);
    b->g0norm = norm6(b->g0);
    b->pnorm = norm6(b->p);
    double dir = (dot6(b->p, b->gradient) > 0) ? -1.0 : 1.0;
    for (int i = 0; i < 6; ++i) b->p[i] *= dir / b->pnorm;
    b->pnorm = norm6(b->p);
    b->fp0 = dot6(b->p, b->g0);
    b_change_direction(b);
    return BFGS_SUCCESS;
}

/* estimateRigidTransformationBFGS: returns 0 on acceptance, -1 if PCL would throw */
static int estimate_bfgs(ref_gicp* g, float T[4][4]) {
    if (g->m < 4) return -1; /* NotEnoughPointsException */
    double x[6];
    x[0] = T[0][3];
    x[1] = T[1][3];
    x[2] = T[2][3];
    x[3] = atan2((double)T[2][1], (double)T[2][2]);
    x[4] = asin(-(double)T[2][0]);
    x[5] = atan2((double)T[1][0], (double)T[0][0]);
    bfgs_t b;
    memset(&b, 0, sizeof(b));
    b.g = g;
    b.sigma = 0.01; b.rho = 0.01; b.tau1 = 9; b.tau2 = 0.05; b.tau3 = 0.5; b.order = 3;
    b.step_size = (g->prm.variant & 16) ? 0.1 : 1;
    b.bracket_iters = (g->prm.variant & 8) ? 20 : 100;
    b.section_iters = (g->prm.variant & 8) ? 20 : 100;
    const double gradient_tol = (g->prm.variant & 1) ? g->prm.gicp_epsilon : 1e-2;
    int inner = 0;
    int result = b_minimize_init(&b, x);
    result = BFGS_RUNNING;
    do {
        inner++;
        result = b_minimize_one_step(&b, x);
        if (result) break;
        result = (norm6(b.gradient) < gradient_tol) ? BFGS_SUCCESS : BFGS_RUNNING;
    } while (result == BFGS_RUNNING && inner < g->prm.max_inner_iterations);
    if (result == BFGS_NO_PROGRESS || result == BFGS_SUCCESS || inner == g->prm.max_inner_iterations) {
        apply_state(x, T);
        return 0;
    }
    return -1; /* SolverDidntConvergeException */
}

/* ------------------------------------------------------------------------------------ */
/* correspondences + Mahalanobis (one outer iteration of computeTransformation)          */
/* ------------------------------------------------------------------------------------ */
static void full3(const double* c6, double C[3][3]) {
    C[0][0] = c6[0]; C[0][1] = c6[1]; C[0][2] = c6[2];
    C[1][0] = c6[1]; C[1][1] = c6[3]; C[1][2] = c6[4];
    C[2][0] = c6[2]; C[2][1] = c6[4]; C[2][2] = c6[5];
}

/* M = (R C1 R' + C2)^-1 with Eigen's 3x3 cofactor inverse */
static void mahalanobis(const double R[3][3], const double* c1, const double* c2, double* M9) {
    double C1[3][3], C2[3][3], RC[3][3], t[3][3];
    full3(c1, C1);
    full3(c2, C2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = R[i][0] * C1[0][j];
            a = a + R[i][1] * C1[1][j];
            a = a + R[i][2] * C1[2][j];
            RC[i][j] = a;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = RC[i][0] * R[j][0];
            a = a + RC[i][1] * R[j][1];
            a = a + RC[i][2] * R[j][2];
            t[i][j] = a + C2[i][j];
        }
#define COF(i, j) (t[((i) + 1) % 3][((j) + 1) % 3] * t[((i) + 2) % 3][((j) + 2) % 3] - \
                   t[((i) + 1) % 3][((j) + 2) % 3] * t[((i) + 2) % 3][((j) + 1) % 3])
    double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    double det = c00 * t[0][0];
    det = det + c10 * t[1][0];
    det = det + c20 * t[2][0];
    double inv = 1.0 / det;
    M9[0] = c00 * inv; M9[1] = c10 * inv; M9[2] = c20 * inv;
    M9[3] = COF(0, 1) * inv; M9[4] = COF(1, 1) * inv; M9[5] = COF(2, 1) * inv;
    M9[6] = COF(0, 2) * inv; M9[7] = COF(1, 2) * inv; M9[8] = COF(2, 2) * inv;
#undef COF
}

/* R = (T * guess) top-left 3x3 in fp64 (transform_R loop of computeTransformation) */
static void rot_of(const float T[4][4], const float G[4][4], double R[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double a = 0.0;
            for (int k = 0; k < 4; ++k) a += (double)T[i][k] * (double)G[k][j];
            R[i][j] = a;
        }
}

/* fills g->corr_* and g->mahal; returns count; nn_tgt/nn_d2 optional full outputs */
static int correspondence_sweep(ref_gicp* g, const float T[4][4], const float G[4][4], int* nn_tgt,
                                float* nn_d2) {
    double R[3][3];
    rot_of(T, G, R);
    double thr = g->prm.max_corr_dist * g->prm.max_corr_dist;
    int n = g->ns;
    int* tj = (int*)malloc((size_t)n * sizeof(int));
    int nt = g->prm.threads > 1 ? g->prm.threads : 1;
    (void)nt;
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1024) if (nt > 1)
    for (int i = 0; i < n; ++i) {
        float q[3];
        xform(T, g->out + 3 * (size_t)i, q);
        int j;
        float d2;
        kd_knn(&g->tree_tgt, q, 1, &j, &d2);
        if (nn_tgt) nn_tgt[i] = ((double)d2 < thr) ? j : -1;
        if (nn_d2) nn_d2[i] = d2;
        if ((double)d2 < thr) {
            double* M9 = g->mahal + 9 * (size_t)i;
            mahalanobis(R, g->cov_src + 6 * (size_t)i, g->cov_tgt + 6 * (size_t)j, M9);
            if (g->mahal_upper) { M9[3] = M9[1]; M9[6] = M9[2]; M9[7] = M9[5]; }
            tj[i] = j;
        } else {
            tj[i] = -1;
        }
    }
    int cnt = 0;
    for (int i = 0; i < n; ++i)
        if (tj[i] >= 0) {
            g->corr_src[cnt] = i;
            g->corr_tgt[cnt] = tj[i];
            cnt++;
        }
    free(tj);
    g->m = cnt;
    return cnt;
}

static void alloc_scratch(ref_gicp* g) {
    free_scratch(g);
    size_t n = (size_t)g->ns;
    g->out = (float*)malloc(n * 3 * sizeof(float));
    g->mahal = (double*)malloc(n * 9 * sizeof(double));
    g->corr_src = (int*)malloc(n * sizeof(int));
    g->corr_tgt = (int*)malloc(n * sizeof(int));
    for (size_t i = 0; i < n; ++i) {
        double* M = g->mahal + 9 * i;
        memset(M, 0, 9 * sizeof(double));
        M[0] = M[4] = M[8] = 1.0;
    }
}

int ref_correspondences(ref_gicp* g, const float T_cm[16], const float guess_cm[16], int* out_tgt,
                        float* out_d2, double* out_M9) {
    if (!g) return REF_E_INVALID;
    int rc = prepare(g);
    if (rc) return rc;
    float T[4][4], G[4][4];
    cm_to_rm(T_cm, T);
    cm_to_rm(guess_cm, G);
    if (!g->out) alloc_scratch(g);
    for (int i = 0; i < g->ns; ++i) xform(G, g->src + 3 * (size_t)i, g->out + 3 * (size_t)i);
    int m = correspondence_sweep(g, T, G, out_tgt, out_d2);
    if (out_M9) memcpy(out_M9, g->mahal, (size_t)g->ns * 9 * sizeof(double));
    return m;
}

/* ------------------------------------------------------------------------------------ */
/* align (Registration::align -> GICP::computeTransformation)                            */
/* ------------------------------------------------------------------------------------ */
int ref_align(ref_gicp* g, const float guess_cm[16], float out_T_cm[16], ref_result* res,
              float* trace) {
    if (!g) return REF_E_INVALID;
    ref_result r;
    memset(&r, 0, sizeof(r));
    double t0 = now_s();
    int rc = prepare(g);
    if (rc) return rc;
    double t1 = now_s();
    r.t_cov_s = t1 - t0;

    float G[4][4], T[4][4], prev[4][4];
    if (guess_cm) cm_to_rm(guess_cm, G);
    else identity4(G);
    identity4(T);
    identity4(prev);
    alloc_scratch(g);
    g->n_evals = 0;
    /* output = input (w = 1); transformPointCloud(output, output, guess) */
    for (int i = 0; i < g->ns; ++i) xform(G, g->src + 3 * (size_t)i, g->out + 3 * (size_t)i);

    int nr_iterations = 0, converged = 0;
    while (!converged) {
        correspondence_sweep(g, T, G, NULL, NULL);
        r.n_corr_last = g->m;
        if (g->prm.objective == 1 || g->prm.solver == 1) moments_build(g, T);
        memcpy(prev, T, sizeof(T));
        if ((g->prm.solver == 1 ? estimate_gn(g, T) : estimate_bfgs(g, T)) != 0)
            break; /* PCLException: converged_ stays false */
        double delta = 0.;
        for (int k = 0; k < 4; ++k)
            for (int l = 0; l < 4; ++l) {
                double ratio = (k < 3 && l < 3) ? 1. / g->prm.rotation_epsilon
                                                : 1. / g->prm.transformation_epsilon;
                double c_delta = ratio * (double)fabsf(prev[k][l] - T[k][l]);
                if (c_delta > delta) delta = c_delta;
            }
        if (trace) rm_to_cm(T, trace + 16 * nr_iterations);
        nr_iterations++;
        int stop = g->prm.fixed_iterations ? (nr_iterations >= g->prm.max_iterations)
                                           : (nr_iterations >= g->prm.max_iterations || delta < 1);
        if (stop) {
            converged = 1;
            memcpy(prev, T, sizeof(T));
        }
    }
    /* final_transformation_ = prev (3x3) * guess (3x3), translation prev + guess */
    float F[4][4];
    identity4(F);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            float a = prev[i][0] * G[0][j];
            a = a + prev[i][1] * G[1][j];
            a = a + prev[i][2] * G[2][j];
            F[i][j] = a;
        }
    for (int i = 0; i < 3; ++i) F[i][3] = prev[i][3] + G[i][3];
    rm_to_cm(F, out_T_cm);
    double t2 = now_s();
    r.converged = converged;
    r.iterations = nr_iterations;
    r.n_evals = g->n_evals;
    r.t_loop_s = t2 - t1;
    r.t_total_s = t2 - t0;
    if (res) *res = r;
    return REF_OK;
}

int ref_fitness(ref_gicp* g, const float T_cm[16], double max_range, double* out) {
    if (!g || !out) return REF_E_INVALID;
    if (g->tgt_dirty || !g->tree_tgt.nodes) {
        kd_free(&g->tree_tgt);
        kd_build(&g->tree_tgt, g->tgt, g->nt);
        g->tgt_dirty = 0;
    }
    float T[4][4];
    cm_to_rm(T_cm, T);
    double fitness = 0.0;
    int nr = 0;
    for (int i = 0; i < g->ns; ++i) {
        float q[3];
        xform(T, g->src + 3 * (size_t)i, q);
        int j;
        float d2;
        kd_knn(&g->tree_tgt, q, 1, &j, &d2);
        if (d2 <= max_range) {
            fitness += d2;
            nr++;
        }
    }
    *out = nr > 0 ? fitness / nr : DBL_MAX;
    return REF_OK;
}

/* ------------------------------------------------------------------------------------ */
int ref_covariances(const float* xyz, size_t n, size_t stride, int k, double eps, int threads,
                    double* out_c6) {
    if (!xyz || !out_c6 || stride < 12) return REF_E_INVALID;
    if ((size_t)k > n) return REF_E_TOO_FEW_POINTS;
    int bad;
    float* pts = copy_xyz(xyz, n, stride, &bad);
    if (bad) { free(pts); return REF_E_NONFINITE; }
    kdtree t;
    kd_build(&t, pts, (int)n);
    compute_covariances(&t, k, eps, threads, out_c6);
    kd_free(&t);
    free(pts);
    return REF_OK;
}

int ref_knn(const float* xyz, size_t n, size_t stride, const float* queries, size_t nq, int k,
            int* out_idx, float* out_d2) {
    if (!xyz || !queries || stride < 12) return REF_E_INVALID;
    int bad;
    float* pts = copy_xyz(xyz, n, stride, &bad);
    kdtree t;
    kd_build(&t, pts, (int)n);
    for (size_t i = 0; i < nq; ++i) kd_knn(&t, queries + 3 * i, k, out_idx + (size_t)k * i, out_d2 + (size_t)k * i);
    kd_free(&t);
    free(pts);
    return REF_OK;
}

/* ------------------------------------------------------------------------------------ */
/* The FOD-side callers either side of the GICP path          */
/* ------------------------------------------------------------------------------------ */

/* pcl::SegmentDifferences<PointXYZRGB>::segment -> pcl::getPointCloudDifference (PCL 1.8.1
 * segmentation/impl/segment_differences.hpp), as called by Filter::removeFromCloud
 * (src/Filter.cpp:176-189) with threshold = 4e-3 * voxelize_factor
 * (src/LeicaStateMachine.cpp:186-187).  setDistanceThreshold stores the value compared
 * against the SQUARED nearest-neighbour distance: input point i is kept iff it is finite and
 * its float 1-NN d^2 in `sub` is > sqr_threshold.  An empty `sub` returns the input unchanged
 * (every point kept, finite or not).  Non-finite `sub` points never enter the search tree
 * (KdTreeFLANN::setInputCloud skips them). */
int ref_segment_differences(const float* in, size_t n, size_t in_stride, const float* sub,
                            size_t ns, size_t sub_stride, double sqr_threshold,
                            unsigned char* keep, size_t* n_keep) {
    if ((!in && n) || (!sub && ns) || (!keep && n) || !n_keep || in_stride < 12 || sub_stride < 12)
        return REF_E_INVALID;
    *n_keep = 0;
    if (ns == 0) {
        for (size_t i = 0; i < n; ++i) keep[i] = 1;
        *n_keep = n;
        return REF_OK;
    }
    float* pts = (float*)malloc(ns * 3 * sizeof(float));
    size_t m = 0;
    for (size_t j = 0; j < ns; ++j) {
        const float* p = (const float*)((const char*)sub + j * sub_stride);
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) continue;
        pts[3 * m] = p[0]; pts[3 * m + 1] = p[1]; pts[3 * m + 2] = p[2];
        ++m;
    }
    kdtree t;
    kd_build(&t, pts, (int)m);
    size_t cnt = 0;
    for (size_t i = 0; i < n; ++i) {
        const float* p = (const float*)((const char*)in + i * in_stride);
        keep[i] = 0;
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) continue;
        if (m == 0) continue; /* nearestKSearch finds nothing: PCL warns and skips the point */
        int j;
        float d2;
        kd_knn(&t, p, 1, &j, &d2);
        if ((double)d2 > sqr_threshold) {
            keep[i] = 1;
            ++cnt;
        }
    }
    kd_free(&t);
    free(pts);
    *n_keep = cnt;
    return REF_OK;
}

typedef struct { uint32_t idx, pt; } vg_entry;
static int vg_cmp(const void* a, const void* b) {
    const vg_entry* x = (const vg_entry*)a;
    const vg_entry* y = (const vg_entry*)b;
    if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
    return x->pt < y->pt ? -1 : (x->pt > y->pt ? 1 : 0);
}

/* pcl::VoxelGrid<PointXYZRGB>::applyFilter (PCL 1.8.1 filters/impl/voxel_grid.hpp) with the
 * defaults Filter::downsampleCloud uses (src/Filter.cpp:91-105): no filter field,
 * downsample_all_data = true (CentroidPoint: xyz summed in fp32 and divided by float(n);
 * r, g, b, a summed as floats and truncated after the division), min_points_per_voxel as given.
 *   inverse_leaf = 1.0f / leaf (float);  min_b = (int)floor(min_p * inv);  div = max_b - min_b + 1;
 *   ijk = (int)(floor(p * inv) - (float)min_b);  idx = i + j div_x + k div_x div_y;
 *   points sorted by idx; output = one centroid per voxel in ascending idx.
 * PCL sorts with std::sort (not stable), so the fp32 summation order inside a voxel is
 * unspecified there; this restatement sums in ascending input index (the engine does the
 * same, so the two agree bit for bit; against PCL itself centroids agree to fp32 rounding).
 * Non-finite points are skipped (is_dense = false path).  Returns REF_OK with *overflow = 1
 * and the input copied when div_x*div_y*div_z exceeds INT32_MAX (PCL's "leaf size too small"
 * path: output = input).  out_xyz: 3 * n floats; out_rgba (optional): n uint32. */
int ref_voxel_grid(const float* in, size_t n, size_t stride, int rgb_offset, const float leaf[3],
                   int min_points, float* out_xyz, uint32_t* out_rgba, size_t* n_out, int* overflow) {
    if ((!in && n) || !leaf || !n_out || !overflow || stride < 12 || (n && !out_xyz)) return REF_E_INVALID;
    *n_out = 0;
    *overflow = 0;
    float inv[3];
    for (int d = 0; d < 3; ++d) inv[d] = 1.0f / leaf[d];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    size_t nf = 0;
    for (size_t i = 0; i < n; ++i) {
        const float* p = (const float*)((const char*)in + i * stride);
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) continue;
        for (int d = 0; d < 3; ++d) {
            if (p[d] < mn[d]) mn[d] = p[d];
            if (p[d] > mx[d]) mx[d] = p[d];
        }
        ++nf;
    }
    if (nf == 0) return REF_OK;
    int64_t dd[3];
    for (int d = 0; d < 3; ++d) dd[d] = (int64_t)((mx[d] - mn[d]) * inv[d]) + 1;
    if (dd[0] * dd[1] * dd[2] > (int64_t)INT32_MAX) {
        *overflow = 1;
        for (size_t i = 0; i < n; ++i) {
            const char* rec = (const char*)in + i * stride;
            memcpy(out_xyz + 3 * i, rec, 3 * sizeof(float));
            if (out_rgba && rgb_offset >= 0) memcpy(out_rgba + i, rec + rgb_offset, sizeof(uint32_t));
        }
        *n_out = n;
        return REF_OK;
    }
    int min_b[3], max_b[3], div_b[3];
    for (int d = 0; d < 3; ++d) {
        min_b[d] = (int)floorf(mn[d] * inv[d]);
        max_b[d] = (int)floorf(mx[d] * inv[d]);
        div_b[d] = max_b[d] - min_b[d] + 1;
    }
    const int mul[3] = {1, div_b[0], div_b[0] * div_b[1]};
    vg_entry* iv = (vg_entry*)malloc((nf ? nf : 1) * sizeof(vg_entry));
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) {
        const float* p = (const float*)((const char*)in + i * stride);
        if (!isfinite(p[0]) || !isfinite(p[1]) || !isfinite(p[2])) continue;
        int idx = 0;
        for (int d = 0; d < 3; ++d) {
            int ijk = (int)(floorf(p[d] * inv[d]) - (float)min_b[d]);
            idx += ijk * mul[d];
        }
        iv[k].idx = (uint32_t)idx;
        iv[k].pt = (uint32_t)i;
        ++k;
    }
    qsort(iv, k, sizeof(vg_entry), vg_cmp);
    size_t out = 0;
    for (size_t a = 0; a < k;) {
        size_t b = a + 1;
        while (b < k && iv[b].idx == iv[a].idx) ++b;
        if (b - a >= (size_t)(min_points > 0 ? min_points : 0)) {
            float sx = 0.f, sy = 0.f, sz = 0.f, r = 0.f, g = 0.f, bl = 0.f, al = 0.f;
            for (size_t l = a; l < b; ++l) {
                const char* rec = (const char*)in + (size_t)iv[l].pt * stride;
                const float* p = (const float*)rec;
                sx += p[0]; sy += p[1]; sz += p[2];
                if (rgb_offset >= 0) {
                    uint32_t c;
                    memcpy(&c, rec + rgb_offset, sizeof(c));
                    bl += (float)(c & 0xffu);
                    g += (float)((c >> 8) & 0xffu);
                    r += (float)((c >> 16) & 0xffu);
                    al += (float)(c >> 24);
                }
            }
            const float cnt = (float)(b - a);
            out_xyz[3 * out] = sx / cnt;
            out_xyz[3 * out + 1] = sy / cnt;
            out_xyz[3 * out + 2] = sz / cnt;
            if (out_rgba && rgb_offset >= 0)
                out_rgba[out] = ((uint32_t)(al / cnt) << 24) | ((uint32_t)(r / cnt) << 16) |
                                ((uint32_t)(g / cnt) << 8) | (uint32_t)(bl / cnt);
            ++out;
        }
        a = b;
    }
    free(iv);
    *n_out = out;
    return REF_OK;
}
