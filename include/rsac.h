/*
 * rsac.h -- C ABI of the MI355X RANSAC engine (librsac.so).
 *
 * Drop-in boundary for the reference's RANSAC hot path.  The reference calls
 * OpenCV through the cv2 Python binding:
 *
 *   cv2.solvePnPRansac(objectPoints, imagePoints, K, dist, iterationsCount,
 *                      reprojectionError, confidence) -> retval, rvec, tvec, inliers
 *        main_v1.py:497-502, testpro-K.py:72-75, testpro.py:536-541, test_pro.py:515-520
 *   cv2.findHomography(src, dst, cv2.RANSAC, ransacReprojThreshold) -> H, mask
 *        main_v1.py:312, process.py:200, test02.py:263, testpro.py:350, test_pro.py:351
 *   Python loop of findHomography over candidate locations
 *        main_v1.py:274-284 (find_homographies), process.py:147-185
 *   K sweep of solvePnPRansac over 27 intrinsics
 *        testpro-K.py:58-75 (estimate_camera_orientation)
 *
 * Each entry point below replaces one of those.  Plain pointers and sizes
 * only; the Python layer (rsac/, ctypes) mirrors the cv2 signatures on top.
 *
 * Conventions
 *   - returns RSAC_OK (model found), RSAC_NO_MODEL (retval=False in cv2
 *     terms), or a negative RSAC_E* code; rsac_last_error() gives the text
 *     (thread-local).
 *   - host inputs: float64, array-of-structs exactly as numpy holds them
 *     (points3d N x 3, points2d N x 2), converted to float32 like OpenCV does.
 *     With RSAC_F_DEVICE_IN the same layout lives in device memory.
 *     With RSAC_F_DEVICE_SOA the inputs are already device float32
 *     structure-of-arrays: pts3d = X[N] Y[N] Z[N], pts2d = U[N] V[N].
 *   - inlier masks are RANSAC-phase masks (uint8, one per point), as OpenCV
 *     returns them; host memory unless RSAC_F_DEVICE_OUT.
 *   - work is enqueued on `stream` (hipStream_t; NULL = the context stream, a blocking stream
 *     ordered with the device null stream, i.e. with torch's default stream);
 *     calls on one context are serialised; contexts are independent.
 */
#ifndef RSAC_H
#define RSAC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RSAC_ABI_VERSION 2  /* 2: rsac_set_score_variant removed; rsac_pnp_hypotheses subset width follows RSAC_F_MINIMAL_EPNP5 */

#if defined(__GNUC__)
#define RSAC_EXPORT __attribute__((visibility("default")))
#else
#define RSAC_EXPORT
#endif

/* status codes */
#define RSAC_OK 0
#define RSAC_NO_MODEL 1
#define RSAC_MORE 2 /* rsac_pnp_ransac_first_round: the first round did not end the scan */
#define RSAC_EINVAL (-1)
#define RSAC_ETOOFEW (-2) /* fewer than 4 correspondences (cv2 raises) */
#define RSAC_EHIP (-3)
#define RSAC_ENOMEM (-4)
#define RSAC_ENODEV (-5)

/* flags */
#define RSAC_F_SAMPLER_OPENCV (1u << 0) /* OpenCV MWC getSubset sequence (host-generated) instead of Philox */
#define RSAC_F_ADAPTIVE (1u << 1)       /* RANSACUpdateNumIters early termination, evaluated in rounds */
#define RSAC_F_REFINE (1u << 2)         /* non-minimal refit on the inliers (LM) -> R,t / H */
#define RSAC_F_DEVICE_IN (1u << 3)      /* inputs are device pointers (float64 AoS) */
#define RSAC_F_DEVICE_SOA (1u << 4)     /* inputs are device float32 SoA (implies device) */
#define RSAC_F_DEVICE_OUT (1u << 5)     /* inlier mask output is a device pointer */
#define RSAC_F_EXACT_ONLY (1u << 6)     /* disable the float32 pre-filter in scoring (A/B and tests) */
#define RSAC_F_ASYNC (1u << 8)          /* rsac_pnp_evaluate_range: device outputs, no host wait (see there) */
#define RSAC_F_EPNP (1u << 9)           /* PnP: EPnP on the inliers as the final solve (what solvePnPRansac
                                           runs after a SOLVEPNP_P3P minimal kernel); with RSAC_F_REFINE,
                                           LM from the EPnP pose */
#define RSAC_F_MINIMAL_EPNP5 (1u << 10) /* PnP: 5-point samples solved by EPnP -- solvePnPRansac's default
                                           SOLVEPNP_ITERATIVE kernel, the one every reference call runs
                                           (main_v1.py:497, testpro-K.py:72 pass no flags;
                                           model_points = 5, also in
                                           RANSACUpdateNumIters); explicit subsets are then n x 5 */
#define RSAC_F_LO (1u << 7)             /* LO-RANSAC (PnP, one problem): local optimisation at every new best,
                                           BASELINE.json configs[4]; see DESIGN.md "LO-RANSAC" */
#define RSAC_F_RVEC_ROUNDTRIP (1u << 11) /* PnP: every minimal model's rotation goes through
                                           R' = Rodrigues(Rodrigues(R)) before it is scored, as
                                           OpenCV's PnPRansacCallback keeps (rvec, tvec) and
                                           computeError projects through Rodrigues(rvec)
                                           (main_v1.py:497, testpro-K.py:72); the deterministic
                                           Rodrigues of rsac_rodrigues_* */

typedef struct rsac_ctx rsac_ctx;

/* per-call diagnostics (all optional; without them no HIP timing events are recorded) */
typedef struct rsac_stats {
    int64_t best_hyp;      /* index of the winning hypothesis (-1 none) */
    int64_t iters;         /* RANSAC iterations consumed (OpenCV `iter` at exit) */
    int64_t hyps_scored;   /* hypotheses evaluated on the GPU (>= iters) */
    int32_t n_inliers;     /* RANSAC-phase inlier count of the winner */
    int32_t rounds;        /* launches of the solve+score pair */
    double gpu_ms;         /* device time of solve+score (events), summed over rounds */
    double solve_ms;       /* ... of which the sample+minimal-solve kernel */
    double score_ms;       /* ... of which the scoring kernel */
    int32_t lo_improvements; /* LO-RANSAC: refits that raised the best count */
    int32_t reserved;
} rsac_stats;

/* Timing of any PnP call on the context (batched ones included, which take no stats argument):
 * with rsac_set_timing(ctx, 1) every call records HIP events around its solve and scoring
 * launches on the call's stream, and rsac_last_stats returns the last call's rsac_stats
 * (gpu_ms / solve_ms / score_ms summed over its rounds).  Off by default (no events). */
RSAC_EXPORT int rsac_set_timing(rsac_ctx *ctx, int32_t on);
RSAC_EXPORT int rsac_last_stats(rsac_ctx *ctx, rsac_stats *out);

RSAC_EXPORT int rsac_create(int device, rsac_ctx **out);
RSAC_EXPORT void rsac_destroy(rsac_ctx *ctx);
RSAC_EXPORT const char *rsac_last_error(void);
RSAC_EXPORT int rsac_abi_version(void);
RSAC_EXPORT int rsac_device_count(void);
RSAC_EXPORT int rsac_set_round_size(rsac_ctx *ctx, int64_t hyps_per_round); /* adaptive round length (default 4096) */

/* The pose refit (solvePnPRefineLM, main_v1.py:508-509) of a problem above 4096 points runs
 * on several cooperating blocks that must be resident at once.  rsac_refit_blocks reports, for
 * an n-point problem, the ranges of its summation order (lm_blocks) and the blocks that share
 * them on this device (the co-resident limit; fewer blocks walk more ranges each, same order,
 * same bits).  The blocks wait on each other's sums (about 1 s at most): when other work keeps
 * some of them from being resident that long, the call is redone with one block per refit (no
 * co-residency needed, the same bits), so the caller always gets the refined pose. */
RSAC_EXPORT int rsac_refit_blocks(rsac_ctx *ctx, int32_t n, int32_t *ranges, int32_t *blocks);
/* Test hooks, not for production use.  RSAC_DBG_REFIT_MAX_BLOCKS: cap the refit's
 * cooperating blocks (0 = the device limit).  RSAC_DBG_REFIT_DROP_BLOCK (nonzero): launch one
 * block fewer than the ranges' stride, so one range's sums never arrive. */
#define RSAC_DBG_REFIT_MAX_BLOCKS 1
#define RSAC_DBG_REFIT_DROP_BLOCK 2
#define RSAC_DBG_MF_CELL_PTS 5 /* > 0: the MFMA scorer runs every tile by cells of this many points */
/* RSAC_DBG_SPEC_OVERFLOW (nonzero): the host's replay of a speculative first round treats it as
 * having more improvements than the device records (the restart-from-hypothesis-0 branch) */
#define RSAC_DBG_SPEC_OVERFLOW 6
/* RSAC_DBG_F64_SELFTEST: rsac_debug_set(ctx, RSAC_DBG_F64_SELFTEST, n) runs the fast f64 root /
 * division cores (rsac_math.h dsqrt_fast / ddiv_fast) and the Jacobi rotation's fast form against
 * the IEEE operators on the device, over n random operand sets inside their stated ranges plus the
 * range ends; rsac_debug_get(ctx, RSAC_DBG_F64_SELFTEST, &m) then gives the number of results that
 * differ in any bit (0 expected). */
#define RSAC_DBG_F64_SELFTEST 7
RSAC_EXPORT int rsac_debug_set(rsac_ctx *ctx, int32_t key, int64_t value);
/* RSAC_DBG_SPEC_FINISHES / RSAC_DBG_SPEC_REDOS (read only): rsac_pnp_ransac(_batched) calls whose
 * finish was enqueued behind the device's own pick of the winners, and those of them the host's
 * replay rejected (the finish then ran again on the host's winners). */
#define RSAC_DBG_SPEC_FINISHES 3
#define RSAC_DBG_SPEC_REDOS 4
RSAC_EXPORT int rsac_debug_get(rsac_ctx *ctx, int32_t key, int64_t *value);

/* cv2.solvePnPRansac (main_v1.py:497).  K: 3x3 row-major f64.  Minimal
 * solver: P3P (Lambda Twist) on 4 points.  n_iters = iterationsCount cap,
 * reproj_thresh in px, confidence as in OpenCV.  Outputs R (3x3 row-major),
 * t (3), mask (n). */
RSAC_EXPORT int rsac_pnp_ransac(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                    int32_t n_iters, double reproj_thresh, double confidence, uint64_t seed, uint32_t flags,
                    double R_out[9], double t_out[3], uint8_t *inlier_mask_out, rsac_stats *stats, void *stream);

/* Batched PnP: P independent problems, problem p owns points
 * [offsets[p], offsets[p+1]) and intrinsics K[9p..9p+8] (the K sweep of
 * testpro-K.py:58 is P problems sharing points; pass repeated rows).
 * Outputs per problem: R (9), t (3), status (RSAC_OK/RSAC_NO_MODEL),
 * n_inliers, mask (total points). */
RSAC_EXPORT int rsac_pnp_ransac_batched(rsac_ctx *ctx, const void *pts3d, const void *pts2d, const int64_t *offsets,
                            int32_t n_problems, const double *K, int32_t n_iters, double reproj_thresh,
                            double confidence, uint64_t seed, uint32_t flags, double *R_out, double *t_out,
                            int32_t *status_out, int32_t *n_inliers_out, uint8_t *inlier_mask_out, void *stream);

/* rsac_pnp_ransac_batched with the per-problem results written as f64 rows (ok 0/1, n_inliers,
 * R 9 row-major, t 3) into rows_out, a DEVICE buffer of n_problems x 14 doubles, by a kernel
 * reading the winners' records where they already are: the rows of a rank's problem chunk go to
 * the multi-GPU all-gather without passing through host arrays (rsac/parallel.py
 * pnp_batched_rows).  Returns with the stream synchronised. */
RSAC_EXPORT int rsac_pnp_ransac_batched_rows(rsac_ctx *ctx, const void *pts3d, const void *pts2d,
                                             const int64_t *offsets, int32_t n_problems, const double *K,
                                             int32_t n_iters, double reproj_thresh, double confidence, uint64_t seed,
                                             uint32_t flags, double *rows_out, uint8_t *inlier_mask_out,
                                             void *stream);

/* cv2.findHomography(src, dst, cv2.RANSAC, thr) (main_v1.py:312):
 * src, dst N x 2.  Defaults of OpenCV: max_iters 2000, confidence 0.995. */
RSAC_EXPORT int rsac_homography_ransac(rsac_ctx *ctx, const void *src, const void *dst, int32_t n, int32_t max_iters,
                           double thresh, double confidence, uint64_t seed, uint32_t flags, double H_out[9],
                           uint8_t *mask_out, rsac_stats *stats, void *stream);

/* The location-search loop of find_homographies (main_v1.py:274-284) as one
 * call: P problems with point ranges given by offsets. */
RSAC_EXPORT int rsac_homography_ransac_batched(rsac_ctx *ctx, const void *src, const void *dst, const int64_t *offsets,
                                   int32_t n_problems, int32_t max_iters, double thresh, double confidence,
                                   uint64_t seed, uint32_t flags, double *H_out, int32_t *status_out,
                                   int32_t *n_inliers_out, uint8_t *mask_out, void *stream);

/* The camera-location search of find_homographies / find_homography
 * (main_v1.py:254-348, 419; driver main_v1.py:862-866) as one call.
 * For every candidate location l (locations: L x 3 f64) and every feature i
 * noted on the image (pixels[i] != (0,0), main_v1.py:304):
 *   pos2 = (dz/dx, dy/dx) of pos3d[i] - loc[l]              (main_v1.py:305-308)
 *   H, mask = findHomography(pos2, pixels, RANSAC, thr)     (main_v1.py:312)
 *   err1 = sum_{mask} |pixel - H pos2|,  err2 = sum_{mask} |pos2 - H^-1 pixel|
 *          + (#outliers) * thr                              (main_v1.py:332-348, 419)
 * Host f64 arrays (pos3d n x 3, pixels n x 2).  Outputs: err_out L x 2
 * (err1, err2; (0, 0) where no model, which the driver maps to 1e6), and
 * optionally H_out L x 9 (findHomography's H = inv(M) of main_v1.py:314),
 * status_out L, n_inliers_out L, mask_out L x n_good (RANSAC-phase),
 * n_good_out.  flags: as rsac_homography_ransac (OpenCV sampler + adaptive +
 * refine reproduce cv2.findHomography). */
RSAC_EXPORT int rsac_location_search(rsac_ctx *ctx, const double *pos3d, const double *pixels, int32_t n,
                                     const double *locations, int32_t n_locations, double thresh, int32_t max_iters,
                                     double confidence, uint32_t flags, double *H_out, double *err_out,
                                     int32_t *status_out, int32_t *n_inliers_out, uint8_t *mask_out,
                                     int32_t *n_good_out, void *stream);

/* Fundamental-matrix RANSAC (BASELINE.json configs[3]; the reference has no
 * implementation -- SURVEY.md §8d -- so DESIGN.md "Fundamental matrix" defines it):
 * 8-point samples (Philox), normalised 8-point DLT + rank 2, Sampson test
 * r^2 <= thr^2 (a^2 + b^2 + a'^2 + b'^2) in f64, adaptive RANSACUpdateNumIters with
 * 8 model points.  pts1, pts2: N x 2 (x2^T F x1 = 0).  Flags: ADAPTIVE, DEVICE_IN,
 * DEVICE_SOA, DEVICE_OUT, EXACT_ONLY. */
RSAC_EXPORT int rsac_fundamental_ransac(rsac_ctx *ctx, const void *pts1, const void *pts2, int32_t n, int32_t max_iters,
                                        double thresh, double confidence, uint64_t seed, uint32_t flags,
                                        double F_out[9], uint8_t *mask_out, rsac_stats *stats, void *stream);
/* per-hypothesis probe (status, counts, models) of the fundamental-matrix path */
RSAC_EXPORT int rsac_fundamental_hypotheses(rsac_ctx *ctx, const void *pts1, const void *pts2, int32_t n,
                                            int64_t hyp_begin, int32_t n_hyps, double thresh, uint64_t seed,
                                            uint32_t flags, int32_t *counts_out, int8_t *status_out,
                                            double *models_out, void *stream);

/* The winner of a sharded run, re-derived on every rank without a host round trip
 * ("the winning model is re-derivable from hyp_idx on every rank"):
 * key = device pointer to the all-reduced packed key (count << 32 | ~index; 0 = none);
 * pts3d / pts2d = device f64 AoS; writes the hypothesis' R 9, t 3 to model_out
 * (device, 12 doubles; zeros for key 0) and its RANSAC-test mask to mask_out (device,
 * n bytes, optional).  Asynchronous on `stream`. */
RSAC_EXPORT int rsac_pnp_winner(rsac_ctx *ctx, const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                                double thresh, uint64_t seed, const int64_t *key, double *model_out,
                                uint8_t *mask_out, void *stream);

/* GeoCoordTransformer (main_v1.py:36-57, pyproj EPSG:4326 <-> EPSG:326zz/327zz):
 * inverse != 0: (easting, northing) -> (lon, lat) degrees; inverse == 0: the reverse.
 * in, out: n x 2 f64 (host, or device with RSAC_F_DEVICE_IN: enqueued on `stream`, no wait).
 * Krueger's series to 6th order (DESIGN.md "DEM ray march"). */
RSAC_EXPORT int rsac_utm_convert(rsac_ctx *ctx, int inverse, const double *in, int64_t n, int32_t zone, int32_t south,
                                 uint32_t flags, double *out, void *stream);

/* ray_intersect_dem (main_v1.py:635-656) for n_rays rays at once: from origins[i] (UTM
 * easting, northing, height) march along dirs[i] in `step` m steps, int(max_search_dist /
 * step) times; a ray hits at the first position, from step index min_steps (150 in the
 * reference) on, not above the DEM.  The DEM is the reference's RegularGridInterpolator over
 * (lat, lon): dem ny x nx f64 row-major, lat_i = i * dy + y0, lon_j = j * dx + x0 (GDAL
 * geotransform: y0 = gt[3], dy = gt[5], x0 = gt[0], dx = gt[1]); each step's UTM position is
 * converted with the zone's inverse projection.  Outputs: hits_out n x 3 (NaN without a hit), status_out n:
 * 0 hit, 1 no hit within the distance (None), 2 left the DEM (the reference's caught
 * interpolation error, None).  Host arrays, or device with RSAC_F_DEVICE_IN (all of them; the
 * call then only enqueues on `stream` and returns without waiting). */
RSAC_EXPORT int rsac_dem_ray_intersect(rsac_ctx *ctx, const double *origins, const double *dirs, int32_t n_rays,
                                       const double *dem, int32_t ny, int32_t nx, double y0, double dy, double x0,
                                       double dx, int32_t zone, int32_t south, double max_search_dist, double step,
                                       int32_t min_steps, uint32_t flags, double *hits_out, int8_t *status_out,
                                       void *stream);

/* Minimal slice: inlier counts of given poses (H x [R 9, t 3] f64, host)
 * under the reprojection test of PnPRansacCallback::computeError. */
RSAC_EXPORT int rsac_score_poses(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                     const double *poses, int32_t n_poses, double reproj_thresh, uint32_t flags, int32_t *counts_out,
                     void *stream);

/* Hypothesis-range evaluation for sharding one problem over ranks
 * (SURVEY.md §8e): evaluates hypotheses [hyp_begin, hyp_begin + n_hyps) of
 * the Philox stream and returns the packed key
 * (count << 32) | (0xFFFFFFFF - low32(global index)) of the best one (lowest
 * index among ties), that hypothesis' model (R, t) and, if mask_out is
 * given, its RANSAC-phase mask (device pointer with RSAC_F_DEVICE_OUT).
 * Ranks all-reduce(MAX) the key.
 * RSAC_F_ASYNC: key_out (one int64, the raw packed key, 0 = no model) and model_out
 * (12 doubles) are DEVICE pointers, mask_out must be a device pointer too; the call only
 * enqueues work on `stream` and returns RSAC_OK without waiting (no stats). */
RSAC_EXPORT int rsac_pnp_evaluate_range(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                            int64_t hyp_begin, int64_t n_hyps, double reproj_thresh, uint64_t seed, uint32_t flags,
                            int64_t *key_out, double model_out[12], uint8_t *mask_out, rsac_stats *stats,
                            void *stream);

/* Raw hot-path outputs for hypotheses [hyp_begin, hyp_begin + n_hyps) of
 * one problem: per-hypothesis status (1 model, 0 solver failed, -1 no
 * subset), inlier count and model (16 f64: R 9, t 3 | H 9; then valid.  PnP
 * records leave valid to the status byte on the device: host outputs get it
 * filled in, RSAC_F_DEVICE_OUT outputs carry an unspecified slot 12).
 * subsets (host int32 n_hyps x 4, or x 5 with RSAC_F_MINIMAL_EPNP5; optional) replaces the Philox draw, e.g.
 * with OpenCV's MWC sequence.  This is what the parity tests compare with
 * the CPU restatement hypothesis by hypothesis. */
RSAC_EXPORT int rsac_pnp_hypotheses(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                                    int64_t hyp_begin, int32_t n_hyps, double reproj_thresh, uint64_t seed,
                                    uint32_t flags, const int32_t *subsets, int32_t *counts_out, int8_t *status_out,
                                    double *models_out, void *stream);
RSAC_EXPORT int rsac_homography_hypotheses(rsac_ctx *ctx, const void *src, const void *dst, int32_t n,
                                           int64_t hyp_begin, int32_t n_hyps, double thresh, uint64_t seed,
                                           uint32_t flags, const int32_t *subsets, int32_t *counts_out,
                                           int8_t *status_out, double *models_out, void *stream);

/* Mask of a given pose under the RANSAC test (used after a sharded run). */
RSAC_EXPORT int rsac_pnp_mask(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                  const double model[12], double reproj_thresh, uint32_t flags, uint8_t *mask_out,
                  int32_t *count_out, void *stream);

/* cv2.solvePnP(..., flags=SOLVEPNP_EPNP) on the masked points (mask NULL = all), the
 * final solve cv2.solvePnPRansac runs on its inliers when the minimal solver is P3P
 * (flags=SOLVEPNP_P3P).  Host arrays; the same computation as the device
 * pass of RSAC_F_EPNP, bit for bit.  Returns RSAC_NO_MODEL for < 4 points or a degenerate
 * (planar) cloud. */
RSAC_EXPORT int rsac_pnp_epnp(const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                              const uint8_t *mask, double R_out[9], double t_out[3]);

/* The minimal solver of cv2.solvePnPRansac's default flags on one 5-point sample, on the host
 * (no GPU needed): solvePnP(..., SOLVEPNP_EPNP) in OpenCV's operation sequence (undistortPoints
 * to f32 normalised points, epnp.cpp with lapack.cpp's JacobiSVD; rsac_cvepnp.h, the source the
 * k_cvepnp5_* kernels run, the 12 x 12 JacobiSVD there on six lanes).  pts3d 5 x 3 and pts2d
 * 5 x 2 f64 AoS, rounded to f32 like solvePnPRansac's CV_32F copies (main_v1.py:497,
 * testpro-K.py:72).  Always RSAC_OK (OpenCV's EPnP reports a pose for any sample; a degenerate
 * one gives NaN). */
RSAC_EXPORT int rsac_pnp_epnp_minimal(const double *pts3d, const double *pts2d, const double K[9], double R_out[9],
                                      double t_out[3]);

/* Host-side non-minimal fits (no GPU needed), f64 AoS host inputs rounded
 * to f32 like the RANSAC path.  mask may be NULL (= all points).
 * rsac_pnp_refine: LM on (R, t) in place, cv2.solvePnPRefineLM
 *   (main_v1.py:508, testpro-K.py:122); returns iterations used.
 * rsac_homography_fit: normalised least-squares DLT + 10 LM iterations,
 *   findHomography's method-0 / final polish (main_v1.py:312). */
RSAC_EXPORT int rsac_pnp_refine(const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                                const uint8_t *mask, double R[9], double t[3], int32_t max_iter);
RSAC_EXPORT int rsac_homography_fit(const double *src, const double *dst, int32_t n, const uint8_t *mask,
                                    double H_out[9]);

/* cv2.solvePnPRefineLM (main_v1.py:508-509, testpro-K.py:122-125) on the device: LM on (R, t)
 * in place from the given start over the masked points (mask NULL = all); host f64 AoS inputs,
 * rounded to f32 like the RANSAC path.  The same bits as rsac_pnp_refine (host). */
RSAC_EXPORT int rsac_pnp_refine_lm(rsac_ctx *ctx, const double *pts3d, const double *pts2d, int32_t n,
                                   const double K[9], const uint8_t *mask, double R[9], double t[3], void *stream);

/* compute_reprojection_error (testpro-K.py:32-36) = cv2.projectPoints (testpro-K.py:33, zero
 * distortion) + the per-point L2 norm of the pixel residual, in f64 on the f64 inputs:
 * proj_out n x 2 (optional), err_out n (optional).  Host arrays, or (RSAC_F_DEVICE_IN) device
 * arrays for inputs and outputs alike, then only enqueued on `stream`. */
RSAC_EXPORT int rsac_pnp_reprojection_errors(rsac_ctx *ctx, const double *pts3d, const double *pts2d, int32_t n,
                                             const double K[9], const double R[9], const double t[3],
                                             uint32_t flags, double *proj_out, double *err_out, void *stream);

/* estimate_camera_orientation (testpro-K.py:39-125) in one call: solvePnPRansac of the points
 * under each of the n_k intrinsics Ks (n_k x 9, the loop of :58-75, one batched launch
 * sequence; flags as rsac_pnp_ransac_batched: the final solve is RSAC_F_REFINE / RSAC_F_EPNP),
 * the gate "success and >= min_inliers inliers" (:77, 6 in the reference), the mean inlier
 * reprojection error of every K on the device (:80-82, through the pose's rvec as projectPoints
 * sees it), the first K with the strictly smallest mean (:90-97), then solvePnPRefineLM of that
 * K's pose on its inliers (:122-125).  Host f64 arrays.  Outputs: *best_out (-1: every K failed,
 * RSAC_NO_MODEL), and optionally per K mean_err_out (NaN where gated), models_out (R 9, t 3 of
 * solvePnPRansac), status_out (RSAC_OK = passed the gate), n_inliers_out, masks_out (n_k x n);
 * R_out / t_out the refined pose of the winner. */
RSAC_EXPORT int rsac_pnp_orientation_sweep(rsac_ctx *ctx, const double *pts3d, const double *pts2d, int32_t n,
                                           const double *Ks, int32_t n_k, int32_t n_iters, double reproj_thresh,
                                           double confidence, uint64_t seed, uint32_t flags, int32_t min_inliers,
                                           int32_t *best_out, double *mean_err_out, double *models_out,
                                           int32_t *status_out, int32_t *n_inliers_out, uint8_t *masks_out,
                                           double R_out[9], double t_out[3], void *stream);

/* Rodrigues (cv2.Rodrigues, main_v1.py:895): vector <-> matrix in cvRodrigues2's operation
 * sequence (range check, R = U V^T through lapack.cpp's JacobiSVD, the theta ~ pi branch;
 * c I + c1 r r^T + s [r]x element by element); acos / sin / cos are series polynomials (~1 ulp),
 * so the bits are the device's and the oracle's, not libm's. */
RSAC_EXPORT void rsac_rodrigues_v2m(const double r[3], double R[9]);
RSAC_EXPORT void rsac_rodrigues_m2v(const double R[9], double r[3]);

/* RANSACUpdateNumIters (OpenCV ptsetreg.cpp) */
RSAC_EXPORT int rsac_update_num_iters(double p, double ep, int model_points, int max_iters);

/* The sequential best-model scan of OpenCV's RANSAC loop (ptsetreg.cpp run(): "count >
 * max(maxGoodCount, modelPoints - 1)" replaces the best, then RANSACUpdateNumIters), over
 * per-hypothesis (status, count) in hypothesis order.  rsac_pnp_ransac runs it internally;
 * it is exported for drivers that produce the counts elsewhere, e.g. the multi-GPU loop of
 * rsac/parallel.py, which gathers each round's counts from every rank and scans them
 * identically everywhere.  Host-only, no device work. */
typedef struct rsac_scan_state {
    int64_t niters;   /* current iteration budget (starts at max_iters) */
    int64_t best;     /* index of the best hypothesis so far, -1 = none */
    int64_t iter;     /* hypotheses consumed */
    int32_t max_good; /* inliers of the best */
    int32_t done;     /* budget reached or sampler exhausted */
} rsac_scan_state;
RSAC_EXPORT void rsac_scan_init(rsac_scan_state *st, int32_t max_iters);
/* consume hypotheses [st->iter, st->iter + count); status < 0 = sampler gave up (ends the scan) */
RSAC_EXPORT int rsac_scan(rsac_scan_state *st, const int32_t *counts, const int8_t *status, int64_t count, int32_t n,
                          int32_t model_points, double confidence);
/* LO-RANSAC drivers: as rsac_scan, but return right after a new best (*improved = 1,
 * st->iter = its index + 1) so that it can be optimised locally before the scan goes on */
RSAC_EXPORT int rsac_scan_until_best(rsac_scan_state *st, const int32_t *counts, const int8_t *status, int64_t count,
                                     int32_t n, int32_t model_points, double confidence, int32_t *improved);
/* apply a locally optimised inlier count: raises max_good and lowers the iteration bound */
RSAC_EXPORT int rsac_scan_raise(rsac_scan_state *st, int32_t count, int32_t n, int32_t model_points, double confidence);

/* The multi-GPU adaptive loop's exchange format and scan (rsac/parallel.py):
 * rsac_pnp_hypothesis_rows evaluates Philox hypotheses [hyp_begin, hyp_begin + n_hyps) of one
 * problem and writes {status, count} int32 pairs into rows_out (DEVICE, n_hyps x 2), enqueued on
 * `stream` without waiting; ranks all-gather their rows into one device buffer (RCCL).
 * rsac_scan_device consumes such rows (device, count x 2) as rsac_scan / rsac_scan_until_best
 * would (stop_on_improve: return after a new best, *improved = 1): the improvements are listed on
 * the device and only they reach the host, where the iteration bound is applied. */
/* The sharded adaptive loop's first round (rsac/parallel.py sharded_ransac):
 * rsac_pnp_ransac of one problem (RSAC_F_ADAPTIVE, Philox sampler; RSAC_F_LO allowed) capped at
 * its first round, the 256 hypotheses rsac_pnp_ransac starts with.  Every rank runs it
 * redundantly, with no collective: most scans end inside that round (C2, C5).
 *   - The round ended the scan: the call IS rsac_pnp_ransac (R, t, mask, refit as there; the
 *     device's speculative finish, one synchronisation) and returns RSAC_OK / RSAC_NO_MODEL,
 *     with *st_out the final scan state (done = 1).
 *   - Otherwise it returns RSAC_MORE: *st_out is the scan state after the round (iter = its
 *     length, done = 0), R_out / t_out the best model so far (LO: the locally optimised one),
 *     mask_out undefined; the caller continues the scan from st_out->iter (sharded rounds).
 * stats (optional) as rsac_pnp_ransac. */
RSAC_EXPORT int rsac_pnp_ransac_first_round(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n,
                                            const double K[9], int32_t n_iters, double reproj_thresh,
                                            double confidence, uint64_t seed, uint32_t flags, double R_out[9],
                                            double t_out[3], uint8_t *mask_out, rsac_scan_state *st_out,
                                            rsac_stats *stats, void *stream);
RSAC_EXPORT int rsac_pnp_hypothesis_rows(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n,
                                         const double K[9], int64_t hyp_begin, int32_t n_hyps, double reproj_thresh,
                                         uint64_t seed, uint32_t flags, int32_t *rows_out, void *stream);
RSAC_EXPORT int rsac_scan_device(rsac_ctx *ctx, rsac_scan_state *st, const int32_t *rows, int64_t count, int32_t n,
                                 int32_t model_points, double confidence, int32_t stop_on_improve,
                                 int32_t *improved, void *stream);

/* One LO-RANSAC local optimisation (RSAC_F_LO's step) of a pose on the device: up to 4
 * rounds of LM refit on the current RANSAC inliers + recount, kept while the count rises.
 * model_in / model_out: R 9 row-major, t 3.  *count_out = the final inlier count (>= the
 * model's own count), *steps_out = refits that raised it.  flags: RSAC_F_DEVICE_IN. */
RSAC_EXPORT int rsac_pnp_local_opt(rsac_ctx *ctx, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                                   const double model_in[12], double thresh, uint32_t flags, double model_out[12],
                                   int32_t *count_out, int32_t *steps_out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* RSAC_H */
