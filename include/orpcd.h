/*
 * orpcd.h — C-ABI of liborpcd_hip.so, the MI355X-native implementation of
 * OR-PCD's inner registration loop (dpolimeni/Multi-scale-pointcloud-
 * registration, `or-pcd` 0.0.1-BETA.7).
 *
 * Plain pointers and sizes only: no torch, no HIP types in the signatures.
 * The caller owns every host buffer; a context owns all device memory.
 * One context per (thread, device); a context is not re-entrant.  No C++
 * exception crosses this boundary: every entry point returns an orpcd_status
 * and orpcd_last_error() holds the message of the last failure.
 *
 * Reference interfaces each entry point replaces (file:line under
 * /root/reference/src/or_pcd/):
 *   orpcd_set_target / orpcd_set_source / orpcd_gicp_batch
 *       GeneralizedICP.optimize            Optimizer/generalizedICP.py:47-83
 *       -> o3d registration_generalized_icp Optimizer/generalizedICP.py:59-70
 *       batched over the multistart loop   Aligner/Aligner.py:178-202
 *   orpcd_set_targets / orpcd_gicp_batch_targets
 *       the multistarts of one compass iteration's six candidates
 *                                          Aligner/Aligner.py:206-226, 263-298
 *   orpcd_set_source_rows / orpcd_gicp_shard_*
 *       one GeneralizedICP.optimize with the source rows split over GPUs
 *                                          Optimizer/generalizedICP.py:59-70
 *   orpcd_set_source_points / orpcd_icp_p2p_batch
 *       Aligner.refine_registration(PointToPoint) Aligner/Aligner.py:319-364
 *       -> o3d registration_icp             Aligner/Aligner.py:352-359
 *   orpcd_sor / orpcd_voxel_down_sample / orpcd_farthest_downsample
 *       SOR.process                        Preprocessor/Outliers/sor.py:51-79
 *       VoxelDownsampler.process           Preprocessor/Downsamplers/voxelDownsampler.py:77-126
 *       FarthestDownsampler.process        Preprocessor/Downsamplers/farthestDownsampler.py:26-54
 *   orpcd_estimate_normals
 *       o3d EstimateNormals(KNN 20) inside registration_generalized_icp, and
 *       source_copy.estimate_normals(Hybrid) Optimizer/fastGlobalOptimizer.py:118-127
 *   orpcd_nn1_radius
 *       o3d GetRegistrationResultAndCorrespondences (SearchHybrid(r, 1)),
 *       the correspondence step of every ICP iteration (generalizedICP.py:60)
 *   orpcd_fpfh
 *       o3d compute_fpfh_feature           Optimizer/fastGlobalOptimizer.py:130-142
 *   orpcd_fpfh_from_normals
 *       o3d compute_fpfh_feature on a cloud with normals (o3d Feature.cpp)
 *   orpcd_fgr
 *       o3d registration_fgr_based_on_feature_matching
 *                                          Optimizer/fastGlobalOptimizer.py:158-174
 *   orpcd_feature_nn
 *       the feature matching inside registration_fgr_based_on_feature_matching
 *   orpcd_fgr_optimize
 *       FastGlobalOptimizer.optimize       Optimizer/fastGlobalOptimizer.py:146-190
 *   orpcd_comm_*, orpcd_gicp_shard_run
 *       the same call over several GPUs, its per-pass all-reduce on device
 *                                          generalizedICP.py:59-70 (C5)
 *   orpcd_set_target_rows, orpcd_target_cov_rows, orpcd_set_target_cov
 *       the target's KNN-20 covariances (generalizedICP.py:59-70) split by
 *       rows over the same GPUs, one all-gather
 *   orpcd_fgr_optimize_batch
 *       the B optimize() calls of one multistart (or of several scale
 *       candidates)                        Aligner/Aligner.py:178-202, 263-298
 *   orpcd_rng_draw_attempts
 *       the np.random draws of initialize_rotation, attempt after attempt
 *                                          Aligner/Aligner.py:125-162, 178-186
 *   orpcd_rigid_residual
 *       recognising the posed copy source @ R0 + t0 of a cached cloud
 *                                          Aligner/Aligner.py:183-190
 */
#ifndef ORPCD_H
#define ORPCD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORPCD_ABI_VERSION 1

typedef enum {
    ORPCD_OK = 0,
    ORPCD_EINVAL = 1,  /* invalid argument (maps to the reference's validation) */
    ORPCD_ENOCORR = 2, /* no correspondences (Python: ValueError / Warning)     */
    ORPCD_EDEVICE = 3  /* HIP runtime / kernel failure                          */
} orpcd_status;

typedef struct orpcd_ctx orpcd_ctx;

int orpcd_abi_version(void);
/* sha256 (16 hex) of the sources the library was built from, and the extra
 * compile flags of an instrumented variant ("" for the product build); the
 * Python binding refuses a library whose id differs from the sources beside it */
const char* orpcd_build_id(void);
const char* orpcd_build_flags(void);
int orpcd_device_count(int* count);
int orpcd_ctx_create(int device, orpcd_ctx** out);
int orpcd_ctx_destroy(orpcd_ctx* ctx);
const char* orpcd_last_error(const orpcd_ctx* ctx);

/* ------------------------------------------------------------------ clouds
 * Target: uploaded once per scale candidate (Aligner.compass_step scales the
 * target, Aligner.py:221-222).  Builds the fp32 search copy and the per-point
 * GICP covariances C_t = R_{e1->n} diag(eps,1,1) R^T from KNN-20 normals.   */
int orpcd_set_target(orpcd_ctx* ctx, const double* xyz, int64_t m, double epsilon);
/* Source: uploaded once per align() (the preprocessed source, unposed).
 * KNN-20 neighbourhood covariances are computed once; each start's posed
 * covariances are derived from them (rigid equivariance).     */
int orpcd_set_source(orpcd_ctx* ctx, const double* xyz, int64_t n);

typedef struct {
    double max_correspondence_distance; /* generalizedICP.py:15-19, default 0.5  */
    int32_t max_iteration;              /* ICPConvergenceCriteria(max_iteration)  */
    double relative_fitness;            /* Open3D default 1e-6                    */
    double relative_rmse;               /* Open3D default 1e-6                    */
    double epsilon;                     /* GICP covariance epsilon, default 1e-3  */
} orpcd_gicp_params;

/* GICP from identity for B starts of the current source posed as
 *     source_initialized = source @ R0[b] + t0[b]      (Aligner.py:183-185)
 * against the current target.  Outputs per start b:
 *   T_out[16*b]   Open3D's column-convention transformation (row-major 4x4),
 *                 i.e. what registration_generalized_icp returns BEFORE the
 *                 plugin transposes R (generalizedICP.py:72-74);
 *   rmse_out[b]   inlier RMSE, fitness_out[b] = |corr| / N,
 *   iters_out[b]  ICP iterations executed, ncorr_out[b] = |corr|.
 * Any of the output pointers except T_out/rmse_out may be NULL.             */
int orpcd_gicp_batch(orpcd_ctx* ctx, const double* R0, const double* t0, int32_t B,
                     const orpcd_gicp_params* params, double* T_out, double* rmse_out,
                     double* fitness_out, int32_t* iters_out, int64_t* ncorr_out);

/* Several targets per batch: the six scale candidates of one compass
 * iteration (Aligner.py:263-298, each compass_step scaling the target,
 * :221-222) as ONE device batch instead of six.  orpcd_set_targets uploads
 * ntargets (<= 16) clouds, xyz = their rows concatenated, m[k] rows each;
 * orpcd_gicp_batch_targets runs start b against target target_of_start[b]
 * (outputs in start order, as orpcd_gicp_batch).  orpcd_set_target is the
 * one-target case; orpcd_gicp_batch = every start against target 0.         */
int orpcd_set_targets(orpcd_ctx* ctx, const double* xyz, const int64_t* m, int32_t ntargets, double epsilon);
int orpcd_gicp_batch_targets(orpcd_ctx* ctx, const double* R0, const double* t0, const int32_t* target_of_start,
                             int32_t B, const orpcd_gicp_params* params, double* T_out, double* rmse_out,
                             double* fitness_out, int32_t* iters_out, int64_t* ncorr_out);

/* orpcd_gicp_batch_targets over passes [pass_begin, pass_end) only: a window
 * of the same loop.  state_in (B x 18 doubles, caller order: T row-major 4x4
 * as the solve keeps it, then the previous pass's fitness and rmse) is where
 * the starts stand at pass_begin (NULL at pass_begin 0).  After the window,
 * done_out[b] = 1 for the starts that finished (their outputs are set) and
 * state_out holds the others' state at pass_end; resuming them from it, in
 * any batch and on any context with the same source and targets, continues
 * them bit for bit (the multi-GPU re-deal of running starts).  */
int orpcd_gicp_batch_window(orpcd_ctx* ctx, const double* R0, const double* t0, const int32_t* target_of_start,
                            int32_t B, const orpcd_gicp_params* params, int32_t pass_begin, int32_t pass_end,
                            const double* state_in, double* state_out, int32_t* done_out, double* T_out,
                            double* rmse_out, double* fitness_out, int32_t* iters_out, int64_t* ncorr_out);

/* A target's device state -- Morton layout, tile / quarter / super-tile
 * boxes, seed grid and GICP covariances -- as one device buffer, and its
 * adoption by another context (on this or another GPU): the multi-GPU
 * re-deal of running starts moves target layouts between
 * ranks (an RCCL all-gather of these buffers) instead of building them again.
 * orpcd_target_layout_bytes: the buffer size for target k (< the targets set);
 * orpcd_get_target_layout: writes it to device memory dev_out (>= that size,
 * on this context's device, 256-byte aligned);
 * orpcd_set_target_layouts: makes ntargets (<= 16) such buffers the targets
 * 0..ntargets-1 of ctx, as orpcd_set_targets would have made them from the
 * same clouds and epsilon (bit for bit: batches on them return the same
 * results).  Replaces orpcd_set_targets.                                    */
int64_t orpcd_target_layout_bytes(orpcd_ctx* ctx, int32_t k);
/* device memory on ctx's device for such buffers, for callers without an
 * allocator of their own (256-byte aligned); freed by orpcd_device_free.    */
int orpcd_device_alloc(orpcd_ctx* ctx, int64_t bytes, void** dev_out);
int orpcd_device_free(orpcd_ctx* ctx, void* dev);
int orpcd_get_target_layout(orpcd_ctx* ctx, int32_t k, void* dev_out, int64_t bytes);
int orpcd_set_target_layouts(orpcd_ctx* ctx, const void* const* dev_in, int32_t ntargets);

/* ------------------------------------ source KNN-20 boundary ties (per pose)
 * Open3D recomputes the source's KNN-20 covariances on every posed copy
 * source_initialized = source @ R0 + t0 (Aligner.py:183-185; the PointCloud
 * rebuilt in generalizedICP.py:54-70).  The batch rotates the unposed cloud's
 * covariances, equal up to rounding except at points whose 20th and 21st
 * neighbours are within the posing rounding of each other ("ties"):
 * orpcd_set_source / orpcd_set_source_rows list them with every candidate
 * neighbour, and each batch re-decides them per start from the posed
 * coordinates numpy forms, np.dot(source, R0) + t0 (fma(a2, b2, fma(a1, b1,
 * a0 * b0)) + t per coordinate).
 * orpcd_source_ties: *n_ties listed points, *n_rows the input indices of
 *   every point involved (ties and candidates, increasing; rows_out, nullable,
 *   n_rows capacity), *complete 0 when more ties existed than were listed.
 * orpcd_set_posed_tie_rows: the posed coordinates of those rows for each of
 *   the next batch's B starts (B x n_rows x 3, caller order; a start whose
 *   block begins with NaN uses numpy's product); consumed by that batch, which
 *   must have B starts.  B <= 0 clears.  The drop-in path passes the rows of
 *   the cloud it was actually given.
 * orpcd_tie_sets: every tie's 20 neighbours (input indices, (d^2, index)
 *   order; n_ties x 20): from posed_rows (n_rows x 3) when not NULL, else
 *   those start b of the last batch used.                                   */
int orpcd_source_ties(orpcd_ctx* ctx, int64_t* n_ties, int64_t* n_rows, int32_t* complete, int64_t* rows_out);
int orpcd_set_posed_tie_rows(orpcd_ctx* ctx, int32_t B, const double* xyz);
int orpcd_tie_sets(orpcd_ctx* ctx, int32_t b, const double* posed_rows, int32_t* sets_out);
/* The posing the batch applies: out[i] = xyz[idx[i]] @ R + t (R row-major,
 * idx NULL = rows 0..n-1) as numpy's np.dot + broadcast add forms it.  Host
 * code only.                                                                */
int orpcd_pose_rows(const double* xyz, const int64_t* idx, int64_t n, const double* R, const double* t, double* out);

/* --------------------------------------- PointToPoint ICP refinement (§8f)
 * Aligner.refine_registration (Aligner.py:319-364, icp_type="PointToPoint")
 * -> o3d registration_icp(source, target, distance_threshold, init,
 *    TransformationEstimationPointToPoint(), ICPConvergenceCriteria(max_iter)).
 * orpcd_set_source_points: the source's search layout only (no covariances;
 * a later orpcd_gicp_batch needs orpcd_set_source again).  The target comes
 * from orpcd_set_target (epsilon < 0 skips its covariances).
 * orpcd_icp_p2p_batch: B independent refinements, init[16*b] a 4x4 applied
 * as Open3D applies `init` (column convention: p' = R p + t, row-major
 * storage); T_out[16*b] = Open3D's result.transformation (init included).
 * params->epsilon is ignored.                                               */
int orpcd_set_source_points(orpcd_ctx* ctx, const double* xyz, int64_t n);
int orpcd_icp_p2p_batch(orpcd_ctx* ctx, const double* init, int32_t B, const orpcd_gicp_params* params,
                        double* T_out, double* rmse_out, double* fitness_out, int32_t* iters_out,
                        int64_t* ncorr_out);

/* ------------------------------------------------ preprocessing (§8f)
 * orpcd_sor: SOR.process (Preprocessor/Outliers/sor.py:51-79) -> o3d
 *   remove_statistical_outlier(nb_neighbors, std_ratio): kept input indices
 *   (increasing) in idx_out (n capacity), their count in *n_out; avg_out (n,
 *   nullable) the per-point mean KNN distance.  nb_neighbors <= 1024.
 * orpcd_voxel_down_sample: VoxelDownsampler (Downsamplers/voxelDownsampler.py:
 *   77-126) -> o3d voxel_down_sample(voxel_size): averaged points (n*3
 *   capacity, nullable = count only), voxels in lexicographic (ix, iy, iz)
 *   order (Open3D: unordered_map order); at most 2^21 voxels per axis.
 * orpcd_farthest_downsample: FarthestDownsampler.process (Downsamplers/
 *   farthestDownsampler.py:26-54): sample_size indices starting at `first`
 *   (the caller's np.random.randint draw).                                  */
int orpcd_sor(orpcd_ctx* ctx, const double* xyz, int64_t n, int32_t nb_neighbors, double std_ratio,
              int64_t* idx_out, int64_t* n_out, double* avg_out);
int orpcd_voxel_down_sample(orpcd_ctx* ctx, const double* xyz, int64_t n, double voxel_size, double* out_xyz,
                            int64_t* n_out);
int orpcd_farthest_downsample(orpcd_ctx* ctx, const double* xyz, int64_t n, int32_t sample_size, int64_t first,
                              int64_t* idx_out);

/* ------------------------------------------------------- kernel-level entry
 * Radius-bounded exact 1-NN (d^2 < r^2 strictly, fp64 re-checked);
 * idx = -1 when no target lies within radius.                               */
int orpcd_nn1_radius(orpcd_ctx* ctx, const double* q, int64_t nq, const double* t, int64_t m,
                     double radius, int32_t* idx_out, double* d2_out);
/* EstimateNormals: knn neighbours (radius <= 0: pure KNN; > 0: hybrid).
 * normals (n*3), raw neighbourhood covariance (n*9), GICP covariance (n*9,
 * only when epsilon >= 0).  Any output may be NULL.                         */
int orpcd_estimate_normals(orpcd_ctx* ctx, const double* xyz, int64_t n, int32_t knn, double radius,
                           double epsilon, double* normals_out, double* rawcov_out, double* gicpcov_out);

/* FPFH (33 bins, Open3D layout transposed to n x 33) after Hybrid normals.  */
int orpcd_fpfh(orpcd_ctx* ctx, const double* xyz, int64_t n, double normal_radius, int32_t normal_knn,
               double fpfh_radius, int32_t fpfh_knn, double* normals_out, double* feat_out);

/* compute_fpfh_feature on a cloud that already carries normals (n x 3). */
int orpcd_fpfh_from_normals(orpcd_ctx* ctx, const double* xyz, const double* normals, int64_t n,
                            double fpfh_radius, int32_t fpfh_knn, double* feat_out);

typedef struct {
    double division_factor;                 /* 1.4  fastGlobalOptimizer.py:25 */
    double tuple_scale;                     /* 0.9                            */
    double maximum_correspondence_distance; /* 0.5                            */
    int32_t iteration_number;               /* 100                            */
    int32_t decrease_mu;                    /* 1                              */
    int32_t maximum_tuple_count;            /* Open3D default 1000            */
    uint64_t seed;                          /* tuple-test RNG (mt19937)       */
} orpcd_fgr_params;

/* FGR on given features (n x 33 and m x 33, row-major).  T_out: Open3D's
 * column-convention transformation; n_mutual_out[2] = {mutual matches,
 * tuple correspondences}.                                                   */
int orpcd_fgr(orpcd_ctx* ctx, const double* src, int64_t n, const double* tgt, int64_t m,
              const double* src_feat, const double* tgt_feat, const orpcd_fgr_params* params,
              double* T_out, double* fitness_out, double* rmse_out, int64_t* ncorr_out,
              int64_t* n_mutual_out);

/* ------------------------------------------- one start, rows over ranks (C5)
 * A single GICP whose SOURCE rows are split over ranks; the target is
 * replicated.  Per pass every rank computes its local normal-equation sums
 * (29 doubles: JTJ upper 21, JTr 6, sum d^2, count), the caller all-reduces
 * them (RCCL), and every rank applies the same update.  The reference runs
 * this as one registration_generalized_icp call (generalizedICP.py:59-70).
 *
 * orpcd_set_source_rows: covariances from the FULL cloud's neighbourhoods,
 * device rows [row_begin, row_end) only.                                    */
int orpcd_set_source_rows(orpcd_ctx* ctx, const double* xyz, int64_t n, int64_t row_begin, int64_t row_end);
int orpcd_gicp_shard_begin(orpcd_ctx* ctx, const double* R0, const double* t0, const orpcd_gicp_params* params,
                           int64_t n_total);
/* local sums of the current pass; *active = 0 once the start has finished */
int orpcd_gicp_shard_pass(orpcd_ctx* ctx, double* sums_out, int32_t* active);
/* global (all-reduced) sums -> convergence test, solve, next queries */
int orpcd_gicp_shard_update(orpcd_ctx* ctx, const double* sums_in, int32_t* done_out);
int orpcd_gicp_shard_result(orpcd_ctx* ctx, double* T_out, double* rmse_out, double* fitness_out,
                            int32_t* iters_out, int64_t* ncorr_out);

/* The same start with the collective on the device (RCCL over xGMI, librccl
 * loaded at run time).  orpcd_comm_unique_id makes a 128-byte RCCL id on one
 * rank; the caller hands it to the others over any host channel; every rank's
 * context joins with orpcd_comm_init(nranks, rank, id).  orpcd_gicp_shard_run
 * then runs every pass after orpcd_gicp_shard_begin: local sums, their
 * all-reduce and the solve are queued on the library's stream (no host round
 * trip per pass; the done flag is read every "sync_every" passes);
 * orpcd_gicp_shard_result reads the answer.  One rank: bit-identical to
 * orpcd_gicp_batch with one start.                                          */
int orpcd_comm_unique_id(uint8_t* id_out);
int orpcd_comm_init(orpcd_ctx* ctx, int32_t nranks, int32_t rank, const uint8_t* id);
int orpcd_comm_destroy(orpcd_ctx* ctx);
int orpcd_gicp_shard_run(orpcd_ctx* ctx, int32_t* passes_out);

/* The target side of the same split: every rank builds the whole target's
 * search layout and seed grid (the search needs them) but runs the KNN-20
 * covariance pass only over its slice of Morton rows [row_begin, row_end)
 * (ceil(m / nranks) rounded up to whole 64-point tiles).  With a communicator
 * of nranks ranks (orpcd_comm_init) one RCCL all-gather on the library's
 * stream completes the covariances and the target is set as by
 * orpcd_set_target (bit for bit).  Without one (or nranks == 1 trivially
 * complete), the caller completes it: orpcd_target_cov_rows reads this rank's
 * rows (orpcd_target_cov_width() doubles per row, Morton order), and
 * orpcd_set_target_cov takes the concatenation of every rank's rows (m rows).
 * The GICP calls refuse an incomplete target.                               */
int orpcd_set_target_rows(orpcd_ctx* ctx, const double* xyz, int64_t m, double epsilon, int32_t rank,
                          int32_t nranks, int64_t* row_begin, int64_t* row_end);
int32_t orpcd_target_cov_width(void);
int orpcd_target_cov_rows(orpcd_ctx* ctx, int64_t row_begin, int64_t row_end, double* out);
int orpcd_set_target_cov(orpcd_ctx* ctx, const double* cov);

/* Nearest feature row (squared Euclidean, ties -> lowest index) of every
 * query row: the KDTreeFlann SearchKNN(feature, 1) calls of Open3D's
 * AdvancedMatching (FastGlobalRegistration.cpp), on the fp64 matrix cores.
 * q: nq x dim, t: nt x dim (row-major), dim <= 36.                          */
int orpcd_feature_nn(orpcd_ctx* ctx, const double* q, int64_t nq, const double* t, int64_t nt, int32_t dim,
                     int32_t* idx_out);

/* FastGlobalOptimizer.optimize in one call (fastGlobalOptimizer.py:146-190):
 * FPFH of both clouds on device (Hybrid normal / FPFH neighbourhoods), then
 * FGR as orpcd_fgr.  target_features_from_source = 1 reproduces the
 * reference's use of the SOURCE features for the target (:137-142); it
 * requires m <= n (the reference would read past the features otherwise). */
int orpcd_fgr_optimize(orpcd_ctx* ctx, const double* src, int64_t n, const double* tgt, int64_t m,
                       double normal_radius, int32_t normal_knn, double fpfh_radius, int32_t fpfh_knn,
                       int32_t target_features_from_source, const orpcd_fgr_params* params,
                       double* T_out, double* fitness_out, double* rmse_out, int64_t* ncorr_out,
                       int64_t* n_mutual_out);

/* FastGlobalOptimizer.optimize for B posed copies of one source as ONE call
 * (the multistart of Aligner.py:178-202 and the speculative compass's
 * candidates, replacing B calls of orpcd_fgr_optimize): start b is
 * optimize(src @ R0[b] + t0[b], target[target_of_start[b]]) (R0 row-major,
 * posed as numpy rounds np.dot(src, R0) + t0), bit for bit what
 * orpcd_fgr_optimize returns for that posed copy.  Up to 16 targets,
 * concatenated in tgts (m[k] points each); target_of_start may be NULL
 * (every start against target 0).  Per start: T_out[16 b] (column
 * convention), fitness / rmse / ncorr [b], n_mutual_out[2 b .. 2 b + 1].
 * The per-start normals, FPFH, normalisation and evaluation run queued on the
 * device; the tuple tests run on host threads; the B IRLS problems run in one
 * launch.                                                                   */
int orpcd_fgr_optimize_batch(orpcd_ctx* ctx, const double* src, int64_t n, const double* tgts, const int64_t* m,
                             int32_t ntgt, const double* R0, const double* t0, const int32_t* target_of_start,
                             int32_t B, double normal_radius, int32_t normal_knn, double fpfh_radius,
                             int32_t fpfh_knn, int32_t target_features_from_source, const orpcd_fgr_params* params,
                             double* T_out, double* fitness_out, double* rmse_out, int64_t* ncorr_out,
                             int64_t* n_mutual_out);

/* Tuning knobs (defaults are the measured best on MI355X):
 *   "search_waves"  split a start's tiles over waves until ~this many run
 *   "sync_every"    passes between host checks of the per-start done flags
 *   "super_cull"    0/1: first culling level over 64-tile super-tiles
 *   "reseed"        0/1: representative seeding for queries that found no
 *                   target within radius in the previous pass
 *   "small_batch"   at most this many running starts: half the search_waves
 *                   target
 *   "sched"         0/1: search waves dispatched heaviest first by the
 *                   previous pass's measured cost (ordered dispatch)
 *   "sched_items", "sched_min_starts"  its split granularity, and the batch
 *                   size from which it is used
 *   "sched_xcd"     0 (default) / 1: ordered dispatch, each XCD takes one
 *                   contiguous chunk of a cost class's items (measured: no
 *                   gain)
 *   "sched_cap_us"  ordered dispatch: plan no split longer than this many us
 *                   of the previous pass's measured cost (0: no cap)
 *   "seed_grid"     1 (default) / 0: every query's search bound is also
 *                   seeded by the target nearest its cell of the target's
 *                   48^3 seed grid (built at set_target / set_targets)
 *   "seed_reps"     pass-0 search bound without the seed grid: nearest of
 *                   ~this many tile representatives per query
 *   "exact_blocks", "exact_fused"  the fp64 re-search's grid in exact mode:
 *                   at most exact_blocks blocks, exact_fused per running
 *                   start inside the accumulation launch (0: a launch of
 *                   its own before the accumulation)
 *   "count_tiles"   1 (default) / 0: while profiling (orpcd_profiling), the
 *                   search also counts the quarters it scans (stats [2], [5]);
 *                   0 keeps only the hipEvent timing (the counters' atomics
 *                   cost 7-14% of a multistart)
 *   "exact_nn"      1 (default): every correspondence is the fp64 nearest
 *                   target (the oracle's lexicographic (d^2, input index)
 *                   minimum, i.e. Open3D's KD-tree answer); 0: the fp32
 *                   search's answer (candidates within 2^-17 relative in d^2
 *                   resolved by Morton position)
 * Apart from exact_nn, every knob returns bit-identical results; only the
 * speed differs.
 * An unknown key or a value out of range returns ORPCD_EINVAL.            */
int orpcd_set_option(orpcd_ctx* ctx, const char* key, double value);

/* Test entry: n 6x6 systems (per system 27 doubles: the JTJ upper triangle
 * row-major (21), then JTr (6)) solved as the GICP update is (det check,
 * LDLT, TransformVector6dToMatrix4d) by the single-lane and by the
 * wave-parallel device code; per system 23 doubles each: det, x (6), the 4x4
 * update (16).  The two must agree bit for bit.                            */
int orpcd_test_solve6(orpcd_ctx* ctx, const double* sums27, int32_t n, double* out_serial, double* out_wave);

/* Test entry: the correspondences of the last pass of each start of the last
 * batch (orpcd_gicp_batch / orpcd_gicp_batch_targets / orpcd_icp_p2p_batch;
 * for a multi-target batch, b indexes the starts in the caller's order):
 * idx_out[b * N + i] = input index of the nearest target of source point i
 * (input order) in start b's final pass, -1 when none lay inside the search
 * radius (before the strict fp64 d^2 < r^2 test of the accumulation).  With
 * option "exact_nn" these are the oracle's KD-tree answers
 * (oracle/orpcd_oracle.cpp KDTree::nn1: lexicographic (d^2, index) minimum). */
int orpcd_gicp_correspondences(orpcd_ctx* ctx, int32_t B, int32_t* idx_out);

/* --------------------------------------------------------- host RNG replay
 * n consecutive Aligner.initialize_rotation() draws (Aligner.py:129-131,160)
 * from numpy's legacy MT19937 RandomState, bit for bit: per attempt three
 * uniform(low, high) (theta, n x 3) then randn(3) (normal, n x 3).  The
 * state is numpy's get_state() tuple: key (624 words), pos, has_gauss,
 * cached gaussian; it is advanced in place.  Host code only (no device).   */
int orpcd_rng_draw_attempts(uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss, int64_t n,
                            double low, double high, double* theta, double* normal);

/* ------------------------------------------------- drop-in rigid-image check
 * out[0] = max |src - (base R + t)| over the n points and 3 axes (row
 * vectors: src_i = base_i R + t, R row-major), out[1] = max |src|.  The
 * drop-in GeneralizedICP.optimize (the reference's Aligner passing
 * source @ R0 + t0 per attempt, Aligner.py:183-190) runs a call on its cached
 * cloud only when out[0] <= 1e-12 (1 + out[1]).  Host code only.            */
int orpcd_rigid_residual(const double* base, const double* src, int64_t n, const double* R, const double* t,
                         double* out);

/* ------------------------------------------------------------ measurement
 * Live kernel timing (hipEvents on the context's stream).  When enabled,
 * every launch of the dominant correspondence kernel is bracketed.
 * stats[0] = launches, [1] = total ms, [2] = query-target pairs evaluated
 * by the culled scan, [3] = GICP iterations completed, [4] = correspondence
 * passes (start x pass), [5] = 64-point target tiles scanned, [6] = total
 * ms of the fp64 accumulation kernel, [7] = how many of the timed launches
 * ran the ordered-dispatch search (nn_search_sched_kernel; the rest ran
 * nn_search_kernel), [8] = queries re-searched in fp64 (exact_nn), [9] =
 * queries searched while exact_nn was on.  [1] times the search kernel (and,
 * in exact mode, the fp64 re-search that follows it) only.
 * Always counted (host wall-clock, whether profiling or not): [10] ms inside
 * GICP batch calls (set-up to outputs), [11] ms of it in the pass launch
 * calls, [12] ms of it waiting for the device (the every-sync_every-passes
 * synchronisation), [13] GICP batches.
 * Feature nearest neighbour (orpcd_feature_nn, orpcd_fgr*; while profiling,
 * hipEvents around each pass): [14] pass-1 ms, [15] pass-2 (exact
 * re-measure) ms, [16] pass-1 query-target pairs (queries x distinct target
 * rows), [17] pass-2 pairs (flagged queries x distinct rows), [18] calls.
 * Always counted: [19] GICP starts whose source KNN-20 boundary ties may not
 * all have been re-decided from their posed copy (tie table overflowed, or
 * the posed coordinates beyond the size the tie band was set for).          */
int orpcd_profiling(orpcd_ctx* ctx, int32_t enable);
int orpcd_stats(orpcd_ctx* ctx, double* stats_out, int32_t n);
int orpcd_reset_stats(orpcd_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* ORPCD_H */
