// rsac_internal.h -- kernel argument blocks and launchers shared by the
// kernels (rsac_kernels.hip) and the host driver (rsac_api.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstddef>

namespace rsac {

struct EpnpStage1;
struct EpnpStage2;

// PnP problem set on the device.  Problem p owns points [offsets[p],
// offsets[p+1]) of the SoA arrays; its hypothesis records live at
// [p * hyp_stride, p * hyp_stride + H).
// Hypothesis h of problem p (h counted from the start of the call) is record
// p * hyp_stride + h; its Philox counter is (rng_base + h, stream), so a
// shard of one problem's hypothesis space is selected by rng_base.  Every
// problem of a batch uses the same stream (0): a batched call equals the loop
// of single calls it replaces, as each cv2 call restarts OpenCV's RNG.
struct PnpArgs {
    const float *X, *Y, *Z, *U, *V;
    const int64_t *offsets;  // P + 1
    const double *cams;      // P x (fx, fy, cx, cy)
    const float *thr2;       // P
    double *models;          // P x hyp_stride x 16
    int8_t *status;          // P x hyp_stride
    const int32_t *subsets;  // optional P x hyp_stride x 4 (OpenCV sampler)
    const int8_t *sub_status;
    int64_t hyp_stride;
    int64_t rng_base;
    uint64_t seed;
    // float32 pre-filter (DESIGN.md "Scoring"): per-problem frame / constants (the points are
    // centred on frame[0..2] where they are used), per-hypothesis float32 records.  fmodels ==
    // nullptr (or exact_only) selects the all-f64 scoring kernel.
    const double *frame;  // P x kFrameStride: c0 c1 c2 B rho cmax wmax 0 | write_fmodel_mx's terms (8..15)
    const float *fconst;  // P x kFconstStride
    float *fmodels;       // P x hyp_stride x kFModelStride
    // set when the solve kernel precedes the scoring launch: the solve zeroes these counts, so a
    // split scoring launch (atomic count accumulation) needs no memset
    int32_t *counts_out;
    int exact_only;
    // optional fused reduction (single problem): max over the scored hypotheses of
    // (count << 32) | (0xFFFFFFFF - low32(rng_base + h)), atomically into *best_key
    unsigned long long *best_key;
    int *queue;  // counters of the f32 scoring kernels, words 0..3 (reset by the frame and solve kernels)
    int32_t max_n;  // largest problem (points); small problems score one lane per hypothesis
    int fform = 2;  // f32 record form: 1 the scaled form of k_pnp_score_sc (small rounds), 2 the MFMA
                    // form of k_pnp_score_mf (form 1 for problems outside its operand range)
    // MFMA scoring operands per point (fform 2; written with the centred coordinates): PF = two
    // uint4 per point, f16 {hi XC, hi YC, hi ZC, 1, lo XC, lo YC, lo ZC, 0} and the same x 2^-11
    // (the B operand of the lanes that hold the hypotheses' lo parts x 2^11);
    // UV = (u - cx, v - cy) / sqrt(T)
    uint4 *PF = nullptr;
    float2 *UV = nullptr;
    // sample size and minimal solver: 4 = P3P (SOLVEPNP_P3P), 5 = EPnP on 5 points (the
    // default SOLVEPNP_ITERATIVE kernel, RSAC_F_MINIMAL_EPNP5); subsets then hold sample_k indices
    int32_t sample_k = 4;
    // EPnP-5 minimal solve in three launches (k_cvepnp5_*): kEpnpRec doubles of M^T M, its sorted
    // rows and the frame per hypothesis of one launch (P x H, launch-local positions); required when
    // sample_k == 5
    double *epnp = nullptr;
    // RSAC_F_RVEC_ROUNDTRIP: the solve kernels replace each minimal model's R by
    // Rodrigues(Rodrigues(R)) (rsac_math.h rodrigues_roundtrip) before writing its records
    int32_t rvec_rt = 0;
    // 1: the scaled-form scorer builds this round's form-1 records from the f64 models itself
    // (write_fmodel_sc at its unit staging): the round's solve ran beside the problem's set-up
    // (k_pnp_setup_solve4), before the frame existed, and wrote no records
    int32_t fm_inline = 0;
    // test hook (RSAC_DBG_MF_CELL_PTS): > 0 splits every tile of the MFMA scorer into cells of
    // this many points (the unit-size sweep of scripts/mf_units.py); 0 = the launcher's policy
    int32_t dbg_cell_pts = 0;
};

// EPnP-5 solve scratch per hypothesis of one launch (doubles): rsac_kernels.hip k_cvepnp5_* layout
constexpr int kEpnpRec = 192;

constexpr int kFrameStride = 16;
constexpr int kFconstStride = 16;
constexpr int kFModelStride = 16;

struct HomArgs {
    const float *SX, *SY, *DX, *DY;
    const int64_t *offsets;
    const float *thr2;
    double *models;
    int8_t *status;
    const int32_t *subsets;
    const int8_t *sub_status;
    int64_t hyp_stride;
    int64_t rng_base;
    uint64_t seed;
    int32_t max_n;  // largest problem (points)
    // fundamental matrix only: float32 Sampson pre-filter (kernels k_fm_bounds / k_fm_score_f32),
    // per-hypothesis records (kFModelStride floats) and per-problem coordinate bounds
    // (min / max of x1 y1 x2 y2, ordered ints, k_fm_bounds); nullptr: the all-f64 kernel
    float *fmodels;
    const int *fbounds;
    int *fm_queue = nullptr;  // work-queue counter of k_fm_score_q (zeroed before each launch)
};

// problems with at most this many points are scored one lane per hypothesis
// (all points staged in LDS) instead of the points-across-lanes tiles
constexpr int kLanePts = 256;

// mask of the hypothesis a packed key names (problem 0, records at hyp 0..)
hipError_t launch_pnp_mask_key(const PnpArgs &a, int32_t n, const unsigned long long *key, uint8_t *mask,
                               hipStream_t s);
// evaluate_range's epilogue in one launch: record named by the key -> rec16 (+ model12, the raw
// key -> key_out, when non-null) and its mask (when non-null); problem 0
hipError_t launch_pnp_key_finish(const PnpArgs &a, int32_t n, const unsigned long long *key, uint8_t *mask,
                                 double *rec16, double *model12, int64_t *key_out, hipStream_t s);
// record of the hypothesis a packed key names -> out[16] (zeros when key == 0)
hipError_t launch_key_model(const double *models, const unsigned long long *key, int64_t rng_base, double *out,
                            hipStream_t s);

// Single-round scan support (non-adaptive runs without LO): the scan's improvements are the
// strict prefix maxima of the counts of valid hypotheses (status > 0) above model_points - 1,
// up to the first status < 0.  k_scan_records lists them per problem, so the host runs the
// exact scan (RANSACUpdateNumIters with the host's libm) on a few records instead of copying
// every count.  nrec = -1: more than kScanRecs records (the caller falls back to all counts).
constexpr int kScanRecs = 14;
struct ScanRecords {
    int32_t nrec, first_neg;  // first_neg = H when no status < 0
    int32_t idx[kScanRecs], cnt[kScanRecs];
    int32_t dev_best, dev_done;  // the device's replay (ScanDecide), for the host to verify
};
// optional device replay of the first round (scan_records with the device's libm), so the final
// mask and refit can be enqueued before the host has seen the records; the host's own replay
// decides, and redoes the finish if it picked another winner (a last-ulp difference in
// RANSACUpdateNumIters):
//   fixed = 0 (adaptive, one problem): problem 0's replay; its best hypothesis -> best_out[0];
//   fixed = 1 (the round is every problem's whole budget): every problem's replay (its point
//   count from offsets); record index prob * stride + best -> best_out[prob] (-1: no model)
struct ScanDecide {
    int64_t *best_out = nullptr;
    int32_t n = 0;                      // points (fixed = 0)
    const int64_t *offsets = nullptr;   // device problem offsets (fixed = 1)
    int64_t max_iters = 0;
    double confidence = 0;
    int32_t fixed = 0;
};
// a speculative PnP round's scan, left to the finish's mask launch (k_scan_mask)
struct ScanFuse {
    bool pending = false;
    const int32_t *counts = nullptr;
    const int8_t *status = nullptr;
    int64_t stride = 0;
    int32_t H = 0;
    int model_points = 0;
    ScanRecords *out = nullptr;
    ScanDecide dec;
};
hipError_t launch_scan_records(const int32_t *counts, const int8_t *status, int64_t stride, int32_t P, int32_t H,
                               int model_points, ScanRecords *out, hipStream_t s, ScanDecide dec = ScanDecide());

// the multi-GPU adaptive scan (rsac_scan_device): records of a gathered round of {status, count}
// rows above floor0 -> *out (pinned host memory); rows of one problem's (status, counts)
hipError_t launch_scan_rows(const int32_t *rows, int32_t count, int32_t floor0, ScanRecords *out, hipStream_t s);
hipError_t launch_pack_rows(const int8_t *status, const int32_t *counts, int32_t H, int32_t *rows, hipStream_t s);

// best packed key of counts[0, H) (+ its model record -> model_out[16]);
// key = 0 when no hypothesis has a model with >= 1 inlier
hipError_t launch_best_key(const int32_t *counts, const int8_t *status, int32_t H, int64_t hyp_begin,
                           unsigned long long *key, const double *models, double *model_out, hipStream_t s);

// copy model records rec[p] (<0: zero) into out[p][16]
// rec (device, P entries) or, with rec == nullptr, rec0 for the one problem
hipError_t launch_gather_models(const double *models, const int64_t *rec, int32_t P, double *out, hipStream_t s,
                                int64_t rec0 = -1);

// OpenCV's count == model_points branch: per problem with kind[p] = 4 / 5 the record p of rec4 /
// rec5 (the minimal model of its points in input order) -> out[p] (+ host_out[p], pinned), and its
// mask rows all 1 (model) or all 0 (none); kind[p] = 0: untouched.  kind, offsets on the device.
hipError_t launch_direct_finish(const double *rec4, const double *rec5, const int8_t *st4, const int8_t *st5,
                                const int8_t *kind, const int64_t *offsets, int32_t P, double *out, double *host_out,
                                uint8_t *mask, hipStream_t s);

// the problems' result rows (ok, n_inliers, R 9, t 3; f64, P x 14) on the device: info = P x
// {record index (< 0: no model), n_inliers} int64 (host-pinned), models = the winners' records
hipError_t launch_pnp_rows(const int64_t *info, const double *models, int32_t P, double *rows, hipStream_t s);

// frame of every problem (centre, bounds, f32 constants) + centred coords;
// also resets a.best_key (if set) and a.queue.  bounds_ws: P x 10 ints.
// prep: a deferred device f64 -> f32 conversion of one problem (<= 65536 points) to fuse into
// the frame launch (k_pnp_setup1); X .. V the staging SoA it fills
struct PnpPrepare {
    const double *p3 = nullptr, *p2 = nullptr;
    float *X = nullptr, *Y = nullptr, *Z = nullptr, *U = nullptr, *V = nullptr;
    // k_pnp_setup_fc's scratch: per-block bounds (kSetupMaxBlocks x 10 floats) and its ticket
    // (zero on allocation, reset by the kernel)
    float *part = nullptr;
    int *ticket = nullptr;
};
constexpr int kSetupMaxBlocks = 256;
// batches whose problems all have at most this many points set up in one launch (k_pnp_setup_b)
constexpr int kSetupBatchMaxN = 8192;
hipError_t launch_pnp_frame(const PnpArgs &a, int32_t P, int32_t max_n, int32_t *bounds_ws, float *XC, float *YC,
                            float *ZC, double *frame, float *fconst, hipStream_t s,
                            const PnpPrepare *prep = nullptr);
// f32 records for H given f64 models (rsac_score_poses / rsac_pnp_mask)
hipError_t launch_pnp_fmodels(const PnpArgs &a, int32_t P, int32_t H, hipStream_t s);
hipError_t launch_pnp_prepare(const double *p3, const double *p2, int64_t n, float *X, float *Y, float *Z, float *U,
                              float *V, hipStream_t s);
hipError_t launch_hom_prepare(const double *src, const double *dst, int64_t n, float *SX, float *SY, float *DX,
                              float *DY, hipStream_t s);
// solve / score hypotheses [hyp_begin, hyp_begin + H) of every problem
// a one-problem set-up deferred by pnp_args into the first P3P solve (k_pnp_setup_solve4)
struct PnpSetupFuse {
    PnpPrepare prep;
    int32_t max_n;
    int32_t *ws;
    double *frame;
    float *fconst;
};
hipError_t launch_pnp_solve(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s,
                            const PnpSetupFuse *fuse = nullptr);
// whether a one-problem round of H P3P hypotheses can take its set-up into the solve launch: the
// 4-lane solve, then the scaled-form scorer building the round's records itself (fm_inline)
bool pnp_setup_fusable(const PnpArgs &a, int32_t H);
// RSAC_DBG_F64_SELFTEST: fast f64 cores vs IEEE on n random operand sets; mismatches added to *bad
hipError_t launch_f64_selftest(int64_t n, int *bad, hipStream_t s);
hipError_t launch_pnp_score(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s);
// the packed best key of counts [hyp_begin, hyp_begin + H) of one problem into *a.best_key (no-op
// without it); launch_pnp_score does this itself when a.best_key is set
hipError_t launch_pnp_best_key(const PnpArgs &a, int64_t hyp_begin, int32_t H, const int32_t *counts, hipStream_t s);
bool scan_mask_fusable(int32_t H);
hipError_t launch_scan_mask(const ScanFuse &f, const PnpArgs &a, int32_t P, int32_t max_n, uint8_t *mask,
                            double *model_out, double *host_model_out, hipStream_t s);
hipError_t launch_pnp_mask(const PnpArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s, int64_t best0 = -1, double *model_out = nullptr,
                           double *host_model_out = nullptr);
hipError_t launch_hom_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s);
hipError_t launch_hom_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s);
hipError_t launch_hom_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s, int64_t best0 = -1);

// fundamental matrix (8-point + Sampson) on the homography argument block
hipError_t launch_fm_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s);
// coordinate bounds of every problem for the f32 Sampson pre-filter (ws: P x 8 ints)
hipError_t launch_fm_bounds(const HomArgs &a, int32_t P, int32_t max_n, int *ws, hipStream_t s);
hipError_t launch_fm_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts, hipStream_t s);
hipError_t launch_fm_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                          hipStream_t s, int64_t best0 = -1);

// LM refit of every problem's model record (models: P x kModelStride, R 9, t 3, valid)
// on the inliers of mask (concatenated points), one block per problem
hipError_t launch_pnp_epnp_s1(const PnpArgs &a, int32_t P, const uint8_t *mask, const double *models,
                              EpnpStage1 *st1, hipStream_t s);
hipError_t launch_pnp_epnp_s3(const PnpArgs &a, int32_t P, const uint8_t *mask, const EpnpStage1 *st1,
                              const EpnpStage2 *st2, double *models, hipStream_t s);
// multi-block refit scratch (problems > 4096 points): the tagged block-sum granules, two buffers
// of [64 blocks][28 terms][2] u64, zeroed on allocation and whenever launch wraps;
// launch: the per-context launch counter of the tags.  host_off: the problems' offsets (P + 1)
constexpr size_t kLmGranuleBytes = 2ull * 64 * 28 * 2 * 8;
struct LmScratch {
    unsigned long long *gran = nullptr;
    unsigned launch = 0;
    int max_blocks = 0;        // blocks of one problem that can run at once (pnp_refine_coresident)
    int drop_block = 0;        // test hook RSAC_DBG_REFIT_DROP_BLOCK
    int32_t *fail = nullptr;   // pinned host word: a refit's range sums never arrived
    int coop = 0;              // RSAC_REFIT_COOP=1: multi-block refits through hipLaunchCooperativeKernel
                               // (co-residency guaranteed or the launch refused, then one block);
                               // off by default: +25 us on C2 ms-to-best, +0.3 ms on C5
};
// co-resident k_pnp_refine blocks on `device` (occupancy x CUs, capped at kLmMaxBlocks; >= 1)
int pnp_refine_coresident(int device);
hipError_t launch_pnp_refine(const PnpArgs &a, int32_t P, const uint8_t *mask, double *models, int32_t *iters,
                             hipStream_t s, LmScratch *scratch, const int64_t *host_off,
                             double *host_models = nullptr,  // pinned: R, t also written there
                             const double *src = nullptr,    // start records (else models)
                             const int32_t *stop = nullptr); // nonzero: no-op (an ended LO chain)
// device state of an LO-RANSAC chain (k_pnp_lo_count)
struct LoState {
    int32_t cur, stopped, best_buf, improvements;
    alignas(8) int32_t count;  // count and ticket: one 64-bit atomic (k_pnp_lo_count)
    int32_t ticket, last_total, pad;
};
static_assert(offsetof(LoState, ticket) == offsetof(LoState, count) + 4, "count, ticket adjacent");
hipError_t launch_pnp_lo_count(const PnpArgs &a, int32_t n, double *model, uint8_t *mask, LoState *st, int step,
                               int32_t init_cur, double *best_out, LoState *host_st, hipStream_t s);

// mask + inlier count (atomically into *count, zeroed by the caller) of one model record, problem 0
hipError_t launch_pnp_model_count(const PnpArgs &a, int32_t n, const double *model, uint8_t *mask, int32_t *count,
                                  hipStream_t s);

// re-solve the hypothesis named by a device packed key (+ its mask); cam = fx fy cx cy thr2
hipError_t launch_pnp_winner(const double *p3, const double *p2, int32_t n, const double *cam, uint64_t seed,
                             const int64_t *key, double *rec, double *model_out, uint8_t *mask, hipStream_t s);

// compute_reprojection_error (testpro-K.py:32-36): one pose's projections / errors over f64
// AoS device points, and the mean inlier error of P poses over one shared point set
struct PoseCam {
    double R[9], t[3], cam[4];
};
hipError_t launch_pnp_reproj(const double *p3, const double *p2, int32_t n, const PoseCam &pc, double *proj,
                             double *err, hipStream_t s);
hipError_t launch_pnp_reproj_mean(const double *p3, const double *p2, int32_t n, int32_t P, const double *poses,
                                  const double *cams, const uint8_t *masks, double *out, hipStream_t s);

// UTM <-> WGS84 (lon, lat degrees / easting, northing), and the DEM ray march (rsac_geo.h)
hipError_t launch_utm(bool inverse, const double *in, int64_t n, int zone, bool south, double *out, hipStream_t s);
hipError_t launch_dem_march(const double *o, const double *d, int32_t n, const double *dem, int32_t ny, int32_t nx,
                            double y0, double dy, double x0, double dx, int zone, bool south, int32_t n_steps,
                            double step, int32_t min_steps, double *hits, int8_t *status, hipStream_t s);

// camera-location search (main_v1.py:254-348): pos2 of every (location, feature) pair, then
// err1 / err2 of every location's homography
hipError_t launch_loc_pos2(const double *p3, const double *px, int32_t n, const double *locs, int32_t L, double *src,
                           double *dst, hipStream_t s);
hipError_t launch_loc_score(const double *src, const double *dst, const uint8_t *mask, const double *H,
                            const int32_t *ok, int32_t L, int32_t n, double thr, double *err, hipStream_t s);

}  // namespace rsac
