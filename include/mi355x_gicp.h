/*
 * mi355x_gicp.h -- C-ABI of the MI355X-native GICP fine-alignment engine (libmgicp.so).
 *
 * This is the drop-in boundary for the reference's hot path
 *     GICPAlignment::fineAlignment()  ->  gicp_.align(*aligned_cloud)
 *     (/root/reference/src/GICPAlignment.cpp:86-109, the align call at :96, and the
 *      second align in iterateFineAlignment at :116)
 * i.e. it replaces pcl::GeneralizedIterativeClosestPoint<PointXYZRGB,PointXYZRGB>
 * (/root/reference/include/GICPAlignment.h:153) under the unchanged GICPAlignment class.
 * Plain pointers and sizes only; no PCL, Eigen, HIP or torch types cross this header.
 *
 * Matrices are 4x4 float, COLUMN-MAJOR (Eigen::Matrix4f storage order).
 * Point clouds are passed as xyz at byte offsets 0/4/8 of records of `stride_bytes`
 * (32 for pcl::PointXYZRGB, 16 for pcl::PointXYZ, 12 for packed xyz).
 *
 * Threading: one context per host thread; every call blocks until its result is on the
 * host.  Several contexts may align on one device at once: one of them at a time runs the
 * resident pass server (it needs every CU), the others run launched passes.  Status codes: 0 = OK,
 * negative = error (mgicp_last_error() has the message).
 */
#ifndef MI355X_GICP_H
#define MI355X_GICP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGICP_OK                0
#define MGICP_E_INVALID        -1  /* bad argument / state */
#define MGICP_E_TOO_FEW_POINTS -2  /* a cloud has fewer than k points (PCL logs and leaves
                                      its covariances empty, gicp.hpp computeCovariances) */
#define MGICP_E_SOLVER         -3  /* < 4 correspondences or BFGS failure: PCL's
                                      estimateRigidTransformationBFGS throws; align() returns
                                      this with converged = 0 and T = last good transform */
#define MGICP_E_NONFINITE      -4  /* NaN/Inf coordinates in an input cloud */
#define MGICP_E_HIP            -5  /* HIP runtime error */
#define MGICP_E_COMM           -6  /* RCCL error */
#define MGICP_E_NOMEM          -7  /* device allocation failed / grid too large */

#define MGICP_SOLVER_PCL_BFGS   0  /* PCL 1.8.1 BFGS trajectory (parity mode, default) */
#define MGICP_SOLVER_GN         1  /* opt-in fast mode (SURVEY.md 8b "solver"): one device pass
                                      per outer iteration collects the 74 moments of the
                                      quadratic objective, Gauss-Newton on SE(3) runs on the host;
                                      multi-GPU: one 80-double all-reduce per outer iteration.
                                      Not in PCL 1.8.1: reported against the fixed-point protocol
                                      and the oracle's GN restatement, not the BFGS trajectory */

typedef struct {
    int    max_iter;        /* Registration::setMaximumIterations  (GICPAlignment.cpp:50; default 100) */
    double tf_eps;          /* setTransformationEpsilon             (GICPAlignment.cpp:52; default 4e-3) */
    double rot_eps;         /* GICP rotation_epsilon_                (PCL default 2e-3) */
    double max_corr_dist;   /* setMaxCorrespondenceDistance          (GICPAlignment.cpp:51; default 0.04) */
    double gicp_eps;        /* GICP gicp_epsilon_                    (PCL default 1e-3) */
    int    k;               /* GICP k_correspondences_               (PCL default 20; any k in [1, 32]) */
    int    max_inner_iter;  /* GICP max_inner_iterations_            (PCL default 20) */
    int    solver;          /* MGICP_SOLVER_* */
    int    device;          /* HIP device ordinal; -1 = current device */
    int    fixed_iterations;/* 1 = ignore the delta test and run exactly max_iter iterations
                               (matched-iteration parity protocol) */
} mgicp_params;

typedef struct {
    int    converged;       /* Registration::hasConverged() */
    int    iterations;      /* GICP nr_iterations_ */
    int    n_corr;          /* correspondences in the last outer iteration (all ranks) */
    int    n_evals;         /* BFGS objective passes over the correspondences */
    double ms_total;        /* host call -> transform on host */
    double ms_upload;       /* host -> HBM copies of dirty clouds */
    double ms_prep;         /* grid build + kNN covariances (one-time per set_*) */
    double ms_loop;         /* outer GICP loop (correspondences + BFGS) */
} mgicp_result;

typedef struct mgicp_ctx mgicp_ctx;

/* ---- lifecycle ---- */
void        mgicp_default_params(mgicp_params* p);
int         mgicp_create(mgicp_ctx** ctx, const mgicp_params* p);
int         mgicp_set_params(mgicp_ctx* ctx, const mgicp_params* p);
const char* mgicp_last_error(const mgicp_ctx* ctx);
void        mgicp_destroy(mgicp_ctx* ctx);
/* r05 target cache (r06: OPT-IN per context, debug option "target_cache" 1; off by default because the
 * reference node aligns once per process): mgicp_destroy leaves such a single-rank context's target state
 * (grid, covariances, 1-NN cell lists; ~0.5-3 GB at 5M points) in a process-wide cache, one entry per
 * device; a later opted-in set_target whose points equal the cached ones bit for bit (compared on the
 * device) adopts it instead of rebuilding -- results are those of a rebuild bit for bit.  A device
 * allocation that runs out of memory evicts the device's entry and retries once.  This frees every
 * cached entry. */
void        mgicp_release_cache(void);
int         mgicp_device_count(int* n);

/* ---- inputs (Registration::setInputTarget / setInputSource) ----
 * At most 2^31 - 2 points per cloud (32-bit point indices); larger clouds return MGICP_E_INVALID.
 * Host buffers are copied at call time; the cloud is marked dirty so the next align()
 * rebuilds its grid and covariances (PCL resets its trees/covariances the same way).
 * The *_device variants take a device pointer already resident in HBM on this context's
 * device (no H2D copy). */
int mgicp_set_target(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
int mgicp_set_source(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes);
int mgicp_set_target_device(mgicp_ctx* ctx, const float* d_xyz, size_t n, size_t stride_bytes);
int mgicp_set_source_device(mgicp_ctx* ctx, const float* d_xyz, size_t n, size_t stride_bytes);

/* ---- the hot path: Registration::align(output, guess) ----
 * guess may be NULL (identity, as GICPAlignment calls align()).  out_T receives
 * getFinalTransformation().  Returns MGICP_E_SOLVER when PCL would report !hasConverged()
 * because the solver threw. */
int mgicp_align(mgicp_ctx* ctx, const float guess_cm[16], float out_T_cm[16], mgicp_result* res);

/* Registration::getFitnessScore(max_range) for transform T over the source cloud
 * (GICPAlignment.cpp:103,123).  max_range <= 0 means DBL_MAX (PCL default). */
int mgicp_fitness(mgicp_ctx* ctx, const float T_cm[16], double max_range, double* out);

/* pcl::transformPointCloud(source, out, T) for the xyz fields (GICPAlignment.cpp:144-147):
 * writes n transformed xyz triples into out (record stride out_stride_bytes), leaving the
 * other bytes of each record untouched. */
int mgicp_transform_source(mgicp_ctx* ctx, const float T_cm[16], float* out, size_t out_stride_bytes);

/* pcl::transformPointCloud(in, out, T) for any cloud (GICPAlignment::applyTFtoCloud,
 * src/GICPAlignment.cpp:144-147): xyz of n records of `in` are transformed on the GPU and
 * written into `out` (other bytes of the out records untouched; in == out allowed). */
int mgicp_transform_cloud(mgicp_ctx* ctx, const float T_cm[16], const float* in, size_t n,
                          size_t in_stride_bytes, float* out, size_t out_stride_bytes);

/* ---- helpers of GICPAlignment(use_covariances = true) ----
 * Utils::computeCloudResolution (src/Utils.cpp:145-174): mean distance from each point to its
 * nearest other point (the 2nd of a 2-NN query), fp64 sum of float sqrt.  Non-finite records are
 * skipped as queries and as neighbours (0 when fewer than 2 finite points remain). */
int mgicp_cloud_resolution(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes,
                           double* out);
/* The NaN-normal removal of GICPAlignment::getCovariances (src/GICPAlignment.cpp:56-71):
 * pcl::NormalEstimation yields a NaN normal when fewer than 3 points (self included) lie
 * within the search radius (KdTreeFLANN::radiusSearch: float d^2 < float(radius^2)).
 * keep[i] = 1 iff record i is finite and at least min_neighbors finite points (itself included)
 * lie within the radius; non-finite records always get keep[i] = 0 (NaN normal). */
int mgicp_radius_filter(mgicp_ctx* ctx, const float* xyz, size_t n, size_t stride_bytes,
                        double radius, int min_neighbors, unsigned char* keep);

/* ---- the FOD-side callers either side of the GICP path ----
 * pcl::SegmentDifferences<PointXYZRGB>::segment as called by Filter::removeFromCloud
 * (src/Filter.cpp:176-189) on the cloud the FSM just transformed with
 * pcl::transformPointCloud (src/LeicaStateMachine.cpp:182; pass that transform as T_cm, or NULL
 * for an already-transformed input).  keep[i] = 1 iff input record i (after T) is finite and
 * its nearest neighbour among the finite points of `sub` has float d^2 > sqr_threshold (PCL's
 * setDistanceThreshold value is compared with the SQUARED distance).  An empty `sub` keeps every
 * record (PCL: output = input).  *n_keep = number of kept records; output order = input order. */
int mgicp_segment_differences(mgicp_ctx* ctx, const float T_cm[16], const float* in, size_t n,
                              size_t in_stride, const float* sub, size_t n_sub, size_t sub_stride,
                              double sqr_threshold, unsigned char* keep, size_t* n_keep);
/* pcl::VoxelGrid<PointXYZRGB>::filter as called by Filter::downsampleCloud (src/Filter.cpp:91-105):
 * one centroid record per occupied leaf (leaf sizes in metres), in ascending leaf index
 * (i + j div_x + k div_x div_y over floor(p / leaf) - floor(min / leaf)).  xyz = fp32 mean
 * (summed in input order), r/g/b/a of the packed colour word at rgb_offset (-1: none) averaged
 * as floats and truncated (CentroidPoint); leaves with fewer than min_points_per_voxel points are
 * dropped; non-finite records skipped.  `out` holds up to n records of out_stride bytes: x, y, z
 * at 0/4/8, 1.0f at 12 (out_stride >= 16), the colour word at rgb_offset, other bytes zero.  When
 * div_x*div_y*div_z exceeds INT32_MAX PCL warns and returns the input: so does this call. */
int mgicp_voxel_grid(mgicp_ctx* ctx, const float* in, size_t n, size_t stride, int rgb_offset,
                     const double leaf[3], int min_points_per_voxel, float* out, size_t out_stride,
                     size_t* n_out);

/* ---- multi-GPU: one process per GPU, point-range shards of the source cloud ----
 * Rank 0 calls mgicp_get_unique_id and broadcasts the 128 bytes out of band (bench.py uses
 * the TCP rendezvous of leica_point_cloud_processing_amd/parallel.py); every rank then calls
 * mgicp_comm_init before set_* / align.  Every objective pass then all-gathers the ranks' super
 * partials (16 doubles per 32768 source points; GN mode: 80 per super, once per outer iteration)
 * and sums them in a fixed order, so every N gives the single-GPU result bit for bit (see
 * mgicp_debug_supers); the target covariances are computed in N slices and all-gathered.  nranks = 1 with an id builds a
 * one-rank communicator (the collective path on a single device); id = NULL makes a "detached"
 * shard for the debug entry points (or an RCCL-free rank, once mgicp_comm_attach_shm succeeds). */
int mgicp_get_unique_id(unsigned char id[128]);
int mgicp_comm_init(mgicp_ctx* ctx, int nranks, int rank, const unsigned char id[128]);
/* Node-local transport of the per-pass sums (all ranks on one node), called by EVERY rank after
 * mgicp_comm_init with the same POSIX shared-memory name ("/..."; unique per job, e.g. chosen by
 * rank 0 and broadcast) and the same max_source_points (0 = 32M; the largest source cloud any
 * later set_source may hold).  It blocks until every rank has mapped the segment, then unlinks the
 * name.  From then on every objective pass writes each rank's super partials straight from its GPU
 * into the segment (resident pass server on every rank, no collective per pass) and every rank's
 * host takes the same fixed-order total; GN moments and fitness gather through it too.  Results
 * stay bitwise those of one GPU.  RCCL (if initialised) is then used only for the one-time
 * all-gather of the target covariances; without it every rank computes them all.  Every rank must
 * run the same sequence of align / fitness calls.  MGICP_E_COMM: segment or peers unavailable (the
 * context keeps its previous transport).  name = NULL detaches (back to RCCL / local). */
int mgicp_comm_attach_shm(mgicp_ctx* ctx, const char* name, size_t max_source_points);
/* r05: per-pass super rows over xGMI instead of host memory (needs mgicp_comm_attach_shm first: the
 * segment carries the IPC rendezvous; every rank calls this in the same sequence).  on = 1: this rank
 * allocates a device exchange buffer, publishes its IPC handle and opens every other rank's; from then
 * on the resident server's super reducers store each row into every rank's buffer (peer device memory,
 * xGMI) and a one-wave totaler per rank takes the fixed-order total on the device -- the host reads one
 * 32-word row per pass instead of every rank's rows.  Sums, iterations and T stay bitwise those of one
 * GPU.  The server leaves one CU to the totaler; a pass that cannot run on the server (another context
 * holds the device's server slot, profiling) returns MGICP_E_COMM.  on = 0 detaches. */
int mgicp_comm_attach_xgmi(mgicp_ctx* ctx, int on);

/* ---- introspection for parity tests (original point order) ---- */
/* covariances of the source (which = 0) or target (which = 1): n x {c00,c01,c02,c11,c12,c22} */
int mgicp_debug_covariances(mgicp_ctx* ctx, int which, double* out_c6);
/* r06: the original indices of this rank's source points in the order the objective's compacted streams
 * -- and so every pass's fixed reduction tree -- visit them (the grid-sorted order); returns the count.
 * The oracle's summation-order ledger runs the engine's tree over it (oracle/gicp_ref.h ref_set_sum_order). */
int mgicp_debug_source_order(mgicp_ctx* ctx, uint32_t* out, size_t cap);
/* one correspondence sweep at T (col-major); out_tgt[i] = target index or -1;
 * out_M6 (optional) = n x {m00,m01,m02,m11,m12,m22}; returns the count or < 0 */
int mgicp_debug_correspondences(mgicp_ctx* ctx, const float T_cm[16], int* out_tgt, double* out_M6);
/* the same sweep SEEDED with the previous sweep's matches, as the outer iterations after the first
 * run it; same outputs */
int mgicp_debug_correspondences_seeded(mgicp_ctx* ctx, const float T_cm[16], int* out_tgt, double* out_M6);
/* OptimizationFunctorWithIndices::fdf at x over the last correspondence sweep */
int mgicp_debug_fdf(mgicp_ctx* ctx, const double x[6], double* f, double g6[6]);
/* the raw reduced sums of one objective pass at x: [0] sum r'Mr, [1..3] sum Mr,
 * [4..12] sum s (Mr)' row-major, [13] correspondence count.  With mgicp_comm_init(ctx, n, r,
 * NULL) (a "detached" shard, no RCCL) they cover rank r's source range only, so sharding can
 * be verified on one device; align/fitness refuse to run in that mode. */
int mgicp_debug_fdf_sums(mgicp_ctx* ctx, const double x[6], double out16[16]);
/* Objective-pass timing (bench.py's roofline leg): npasses passes at state x over the last
 * correspondence sweep, back to back on the device, bracketed by HIP events on the context's
 * stream.  mode 0: the resident pass server (one launch running all passes; the pass
 * the aligns use on one GPU), mode 1: one fdf_soa_kernel launch per pass.  out_ms: average per
 * pass; out16: the sums of the last pass (as mgicp_debug_fdf_sums).  Single-rank contexts only. */
int mgicp_debug_pass_bench(mgicp_ctx* ctx, const double x[6], int npasses, int mode, double* out_ms,
                           double out16[16]);
/* MGICP_SOLVER_GN's moment pass at T (col-major) over the last correspondence sweep
 * (mgicp_debug_correspondences or an align): out80[0] sum r'Mr, [1..12] sum (Mr) w' (row-major
 * 3x4), [13..72] sum M_p (w w')_q (p: m00 m01 m02 m11 m12 m22; q: upper triangle of the 4x4
 * w w'), [73] count, with r = fl(fl(T s) - q), w = (s - c, 1), c = bbox midpoint of the source */
int mgicp_debug_moments(mgicp_ctx* ctx, const float T_cm[16], double out80[80]);
/* The fixed reduction tree behind every sharded sum (objective passes, GN moments, fitness):
 * chunks of 1024 grid-sorted source positions, supers of 32 chunks, then a fixed-order total over
 * the supers; rank r of N owns supers [nsup * r / N, nsup * (r + 1) / N), so its super partials are
 * the single-GPU run's, bit for bit.  mgicp_debug_supers writes this shard's super partials of one
 * pass -- kind 0: objective pass at x = arg[0..5] (16 values per super, as mgicp_debug_fdf_sums);
 * kind 1: the GN moment pass at the col-major T = arg[0..15] (80 per super, as
 * mgicp_debug_moments); kind 2: getFitnessScore at T = arg[0..15], max_range = arg[16] (16 per
 * super: [0] sum d2, [13] count) -- and returns how many (<= cap) or < 0. */
int mgicp_debug_supers(mgicp_ctx* ctx, int kind, const double* arg, double* out, int cap);
/* the multi-GPU finish itself: the fixed-order total of nsup supers of nv (16 or 80) values held as
 * nranks rows of maxsup supers (row r = rank r's supers; padding rows are never read) */
int mgicp_debug_finish_supers(mgicp_ctx* ctx, int nv, const double* rows, long long nsup, long long maxsup,
                              int nranks, double* out);
/* the chunk reduction of every pass (one wave, 16 values per lane): for each of nwaves waves of
 * in[w][lane][16], out_tree[w][16] = 16 wave_sum shuffle trees (lane 0's sums) and out_rs[w][16] =
 * the register reduce-scatter the passes use (permlane swaps + DPP); the two must agree bit for bit */
int mgicp_debug_wave_reduce(mgicp_ctx* ctx, const double* in, int nwaves, double* out_tree, double* out_rs);
/* per-iteration transformation_ of the last align (col-major, iterations x 16) */
int mgicp_debug_trace(mgicp_ctx* ctx, float* out, int max_iters);
/* average device time (ms) of each kernel family while profiling is on, for roofline
 * reporting: [0] covariance kNN, [1] correspondence 1-NN, [2] BFGS objective pass,
 * [3] separate reduction finish, [4] compaction + Mahalanobis, [5] Gauss-Newton moment pass (+ its
 * finish); counts in out_counts (optional) */
#define MGICP_KERNEL_FAMILIES 6
int mgicp_debug_kernel_times(mgicp_ctx* ctx, double out_ms[MGICP_KERNEL_FAMILIES],
                             int out_counts[MGICP_KERNEL_FAMILIES]);
/* objective-pass path counters since mgicp_create: [0] resident servers launched, [1] passes run
 * by a server, [2] passes run by launched kernels, [3] server passes that missed their deadline
 * (env MGICP_ROW_DEADLINE_MS, default 500) and were taken over by a launched pass (bitwise the
 * same sums; the rest of that align runs launched passes), [4] 1 if the server reads its commands
 * from device memory the host writes through the BAR, [5] private host-row buffer allocations,
 * [6] transport (0 local, 1 RCCL, 2 shared segment, 3 shared segment + RCCL), [7] server launches
 * refused because another context of this process ran a server on the same device */
int mgicp_debug_pass_stats(mgicp_ctx* ctx, long long out[8]);
/* the resident pass server as the aligns run it (always on, two HIP events per server launch on the
 * engine's stream, resolved when an align drains): *out_ms = summed device duration of the server
 * launches (first command .. cancel, host round trips between passes included), *out_passes = the
 * passes those launches ran, *out_launches = the launches; reset = 1 zeroes the counters after the
 * read.  out_ms / out_passes = the in-align time of one objective pass. */
int mgicp_debug_server_time(mgicp_ctx* ctx, double* out_ms, long long* out_passes, long long* out_launches,
                            int reset);
/* the r-th of N target-covariance slices exactly as rank r of an N-rank context computes it before
 * the all-gather (points [r cnt, min(n, (r + 1) cnt)), cnt = ceil(n / N), arrays of N cnt entries):
 * 6 values per point of the slice, in grid-sorted order, into out_c6 (c00 c01 c02 c11 c12 c22);
 * returns the slice's point count.  Assembled in rank order the N slices are the all-gathered arrays (tests; the cached target
 * covariances are recomputed by the next align). */
int mgicp_debug_target_cov_slice(mgicp_ctx* ctx, int nranks, int rank, double* out_c6);
/* the target's 1-NN cell lists (DESIGN.md "1-NN cell lists"): out[0] cells requested and out[1]
 * queries left to the exact per-lane search by the last sweep, out[2] cells with a list, out[3] list
 * entries, out[4] reject cells, out[5] overflow cells, out[6] pool entries used, out[7] fine-grid
 * cells (0 when the lists are off: debug option "vlist" 0 or a gate too wide for a fine grid) */
int mgicp_debug_vlist_stats(mgicp_ctx* ctx, long long out[8]);
/* enable (1) / disable (0) per-launch HIP event timing (off by default); objective passes
 * ([2]) are sampled every 8th launch, every other family is timed on every launch */
int mgicp_set_profiling(mgicp_ctx* ctx, int on);
/* test / diagnostic forms of the engine, set explicitly on one context (never through the
 * environment): "resident", "host_rows", "srv_cus", "fused_finish", "gated", "bar_cmd" (the
 * objective-pass path), "async_cov", "lazy_src_cov", "knn_logged", "knn_wave" (covariances), "vlist",
 * "vlist_cold", "vlist_eager", "vlist_stats", "fuse_compact" (1-NN cell lists),
 * "target_cache", "grid_occ" (grid
 * sizing of the next set_*).  Every form gives the default path's results bit for bit (the GPU tests
 * that pin each one: INTEGRATION.md "Debug options"); MGICP_E_INVALID for an unknown name. */
int mgicp_debug_option(mgicp_ctx* ctx, const char* name, double value);
/* target cache (mgicp_release_cache): out[0] the current target was adopted from the cache, out[1]
 * adoptions and out[2] donations on this device so far, out[3] an entry is cached on this device,
 * out[4] 0 (r05: the source grid's start from a cached target; since r06 a grid depends on its own cloud
 * alone).
 * Debug option "target_cache" 1: this context adopts and leaves targets (default 0: neither). */
int mgicp_debug_cache_stats(mgicp_ctx* ctx, long long out[5]);

#ifdef __cplusplus
}
#endif
#endif
