/*
 * gicp_ref.h -- TEST INFRASTRUCTURE ONLY (the parity oracle / CPU baseline).
 *
 * A plain-C CPU restatement of PCL 1.8.1 pcl::GeneralizedIterativeClosestPoint
 * as instantiated by the reference at include/GICPAlignment.h:153 and driven by
 * GICPAlignment::fineAlignment (src/GICPAlignment.cpp:86-109).  PCL is not
 * vendored under /root/reference and is not installed here, so this file
 * restates the published PCL 1.8.1 algorithm (registration/impl/gicp.hpp,
 * registration/bfgs.h, registration/impl/registration.hpp) -- see SURVEY.md
 * Appendix A and DESIGN.md "Oracle".
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / the timed CPU path.  The product
 * (leica_point_cloud_processing_amd/) never links or calls it.
 *
 * Conventions: 4x4 matrices crossing this header are COLUMN-MAJOR (Eigen's
 * default storage), like include/mi355x_gicp.h.
 */
#ifndef GICP_REF_H
#define GICP_REF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int    max_iterations;         /* max_iterations_       (src/GICPAlignment.cpp:30 -> 100) */
    double transformation_epsilon; /* transformation_epsilon_ (src/GICPAlignment.cpp:29 -> 4e-3) */
    double rotation_epsilon;       /* rotation_epsilon_     (PCL GICP default 2e-3) */
    double max_corr_dist;          /* corr_dist_threshold_  (src/GICPAlignment.cpp:31 -> 0.04), squared before use */
    double gicp_epsilon;           /* gicp_epsilon_         (PCL GICP default 1e-3) */
    int    k_correspondences;      /* k_correspondences_    (PCL GICP default 20) */
    int    max_inner_iterations;   /* max_inner_iterations_ (PCL GICP default 20) */
    int    fixed_iterations;       /* test hook: 1 => ignore the delta test, run exactly max_iterations */
    int    threads;                /* <=1: single thread (PCL 1.8.1 GICP is single-threaded); >1: OpenMP */
    int    objective;              /* 0: PCL per-point functor passes (default, PCL 1.8.1 itself);
                                      1: moment form -- the same quadratic objective evaluated from
                                      74 fp64 moments taken once per outer iteration (checker for the
                                      engine's MGICP_OBJ_MOMENTS mode) */
    int    solver;                 /* 0: PCL BFGS (default); 1: Gauss-Newton on the moment form
                                      (checker for the engine's MGICP_SOLVER_GN; not in PCL) */
    int    variant;                /* 0 (default): the restatement as published.  Bits select one
                                      plausible alternative reading of a bfgs.h / gicp.hpp choice that
                                      was restated without its source (DESIGN.md "Oracle uncertainty
                                      ledger"): 1 inner gradient test at gicp_epsilon_ (1e-3) instead of
                                      1e-2; 2 cubic branch taken on a finite fpb (GSL GSL_IS_REAL) instead
                                      of !(fpb != fpa); 4 quadratic curvature test c > 0 (GSL) instead of
                                      c > a; 8 bracket / section caps 20 instead of 100; 16 first trial
                                      step 0.1 instead of 1; 32 line-search no-progress test against 0
                                      instead of DBL_EPSILON */
} ref_params;

typedef struct {
    int    converged;      /* PCL hasConverged() */
    int    iterations;     /* nr_iterations_ */
    int    n_corr_last;    /* correspondences in the last outer iteration */
    int    n_evals;        /* BFGS functor passes over the correspondences (f, df or fdf) */
    double t_cov_s;        /* trees + covariances (one-time phase) */
    double t_loop_s;       /* outer GICP loop (correspondences + BFGS) */
    double t_total_s;
} ref_result;

/* status codes (mirror include/mi355x_gicp.h) */
#define REF_OK               0
#define REF_E_INVALID       -1
#define REF_E_TOO_FEW_POINTS -2
#define REF_E_NONFINITE     -4

typedef struct ref_gicp ref_gicp;

void      ref_default_params(ref_params* p);
ref_gicp* ref_create(const ref_params* p);
void      ref_destroy(ref_gicp* g);
int       ref_set_params(ref_gicp* g, const ref_params* p);
/* Copies the clouds (xyz at byte offset 0, 4, 8 of each record) and marks them dirty. */
int       ref_set_source(ref_gicp* g, const float* xyz, size_t n, size_t stride_bytes);
int       ref_set_target(ref_gicp* g, const float* xyz, size_t n, size_t stride_bytes);
/* Registration::align(output, guess).  trace (optional, max_iterations*16 floats) receives
 * transformation_ after every outer iteration (column-major). */
int       ref_align(ref_gicp* g, const float guess_cm[16], float out_T_cm[16], ref_result* res,
                    float* trace);
/* Registration::getFitnessScore(max_range) for the final transform T. */
int       ref_fitness(ref_gicp* g, const float T_cm[16], double max_range, double* out);

/* ---- component hooks used by the parity tests ---- */
/* GICP::computeCovariances: out_c6 = n x {c00,c01,c02,c11,c12,c22} (fp64). */
int ref_covariances(const float* xyz, size_t n, size_t stride_bytes, int k, double eps,
                    int threads, double* out_c6);
/* Exact kNN (k nearest by (float d^2, index) order, self included). */
int ref_knn(const float* xyz, size_t n, size_t stride_bytes, const float* queries, size_t nq,
            int k, int* out_idx, float* out_d2);
/* One outer-iteration correspondence sweep at transformation T (col-major) with R = (T*guess)3x3.
 * out_tgt[i] = target index or -1 if rejected; out_M9 (optional) = row-major Mahalanobis. */
int ref_correspondences(ref_gicp* g, const float T_cm[16], const float guess_cm[16],
                        int* out_tgt, float* out_d2, double* out_M9);
/* Moment-form objective (ref_params.objective = 1): build the 74 moments of the last
 * correspondence set at transform T0 (col-major); out74 optional. */
int ref_moments(ref_gicp* g, const float T0_cm[16], double out74[74]);
int ref_moments_range(ref_gicp* g, const float T0_cm[16], int c0, int c1, double out74[74]);
/* OptimizationFunctorWithIndices::fdf at state x for the last correspondence set. */
int ref_fdf(ref_gicp* g, const double x[6], double* f, double g6[6]);
/* raw sums of the functor over correspondences [c0, c1): f, g_t[3], Rsum[9] row-major, count
 * (the per-shard partials of the multi-GPU decomposition) */
int ref_fdf_sums(ref_gicp* g, const double x[6], int c0, int c1, double out14[14]);
/* r06 summation-order ledger: every later objective pass sums in mode 0 (the default: sequential in
 * correspondence order, or the OpenMP parts), 1 (the engine's fixed chunk -> super -> total tree over
 * the stream order perm[0..n), n = source points), 2 (reversed sequential) or 3 (sequential over perm) */
int ref_set_sum_order(ref_gicp* g, int mode, const uint32_t* perm, size_t n);
/* the raw sums of one pass at x in the current mode (0: sequential, 1: the engine tree) */
int ref_fdf_mode_sums(ref_gicp* g, const double x[6], double out14[14]);
/* r06: 1 = use the Mahalanobis matrix's upper triangle mirrored, as the engine stores it (6 fp64 per
 * correspondence); 0 (default) = PCL's full Eigen inverse of (R C1 R' + C2), whose off-diagonal pairs
 * differ by an ulp when R != I (R C1 R' is not exactly symmetric in fp64).  Applies from the next sweep. */
int ref_set_mahalanobis_upper(ref_gicp* g, int on);
/* applyState(I, x): column-major float 4x4. */
void ref_apply_state(const double x[6], float out_cm[16]);

/* FOD-side callers around the GICP path; see gicp_ref.c */
int ref_segment_differences(const float* in, size_t n, size_t in_stride, const float* sub,
                            size_t ns, size_t sub_stride, double sqr_threshold,
                            unsigned char* keep, size_t* n_keep);
int ref_voxel_grid(const float* in, size_t n, size_t stride, int rgb_offset, const float leaf[3],
                   int min_points, float* out_xyz, uint32_t* out_rgba, size_t* n_out, int* overflow);

#ifdef __cplusplus
}
#endif
#endif
