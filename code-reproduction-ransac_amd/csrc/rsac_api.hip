// rsac_api.hip -- the C ABI of include/rsac.h: context, input staging,
// round loop (solve + score on the GPU, sequential scan on the host),
// masks and refits.
//
// One call == one cv2.solvePnPRansac / cv2.findHomography of the reference
// (main_v1.py:497 / main_v1.py:312), or the whole Python loop around it for
// the batched entry points (main_v1.py:274-284, testpro-K.py:58-75).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rsac.h"
#include "rsac_host.h"
#include "rsac_internal.h"
#include "rsac_math.h"

using namespace rsac;

static thread_local std::string g_err;

static int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return fail(RSAC_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

namespace {

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return (T *)p; }
};

constexpr size_t kMaxModelBytes = size_t(32) << 30;  // hypothesis records kept resident per call
// OpenCV-sampler rounds up to this many bytes of subsets + statuses are read by the solve kernels
// from pinned host memory instead of being copied (run_loop)
constexpr int64_t kSubsetZeroCopyBytes = 64 << 10;

// hipMemcpy2DAsync, as one linear copy when the rows are contiguous (one problem): the 2-D path
// costs tens of microseconds more per call on this runtime (measured in the adaptive loop)
hipError_t copy_rows(void *dst, size_t dpitch, const void *src, size_t spitch, size_t width, size_t height,
                     hipMemcpyKind kind, hipStream_t s) {
    if (height == 1 || (dpitch == width && spitch == width))
        return hipMemcpyAsync(dst, src, width * height, kind, s);
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, kind, s);
}

}  // namespace

struct rsac_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // the last async copy out of h_pts / h_small: the host waits on it before rewriting the
    // buffer (calls may return before their copies ran, RSAC_F_ASYNC)
    hipEvent_t ev_pts = nullptr, ev_small = nullptr;
    int64_t round_size = 4096;
    // rsac_set_timing: every PnP call records HIP events around its solve and score launches and
    // leaves its statistics in last_stats (rsac_last_stats)
    bool timing = false;
    rsac_stats last_stats{};
    // device scratch
    DevBuf pts, tables, models, status, counts, subsets, substatus, best, bestmodels, mask;
    int64_t *d_off = nullptr;  // views into `tables`: offsets (P+1), cams (P x 4), thr2 (P)
    double *d_cams = nullptr;
    float *d_thr2 = nullptr;
    DevBuf bounds_ws, frame, fconst, fmodels, queue;  // float32 pre-filter state (PnP)
    DevBuf mxpts;                                              // MFMA point operands (PF, UV: 40 B / point)
    DevBuf epnp5;                                              // EPnP-5 minimal solve: kEpnpRec doubles / hypothesis of a launch
    DevBuf direct;                                             // count == model_points problems (direct_solve)
    PinBuf h_direct;
    DevBuf loc;                                                // location search: inputs, pos2, H, err
    DevBuf lo;                                                 // LO-RANSAC: 2 model records, chain state, 2 masks
    const void *lo_state_base = nullptr;                       // the lo allocation whose LoState is zeroed
    PinBuf h_lo;                                               // LO chain state, written by the device
    PinBuf h_lmfail;                                           // multi-block refit failure word (device-written)
    int dbg_refit_max_blocks = 0;                              // RSAC_DBG_REFIT_MAX_BLOCKS (0: device limit)
    int64_t spec_finishes = 0, spec_redos = 0;                 // RSAC_DBG_SPEC_FINISHES / _REDOS
    int32_t scanrec_copy = 0;  // problems whose device scan records still go to h_scanrec (issue_scanrec_copy)
    int32_t dbg_cell_pts = 0;                                  // RSAC_DBG_MF_CELL_PTS
    bool dbg_spec_overflow = false;                            // RSAC_DBG_SPEC_OVERFLOW
    int64_t dbg_f64_selftest = -1;                             // RSAC_DBG_F64_SELFTEST's last mismatch count
    DevBuf win;                                                // rsac_pnp_winner: the re-derived record
    DevBuf reproj;                                             // reprojection errors / the K sweep's inputs
    DevBuf geo;                                                // geodesy / DEM: staged host inputs and outputs
    DevBuf epnp;                                               // EPnP stage records (P x (stage 1 + stage 2))
    DevBuf lmscr;                                              // multi-block LM refit: tagged wave sums
    DevBuf setup_scr;                                          // k_pnp_setup_fc: ticket + per-block bounds
    // a one-problem set-up pnp_args deferred into the first P3P solve (run_loop launches it with
    // the solve as k_pnp_setup_solve4; flush_setup launches it alone where nothing fuses)
    PnpSetupFuse pending_setup{};
    bool pending_on = false;
    LmScratch lm;                                              // ... and its launch counter
    std::vector<char> last_tables;                             // the tables last uploaded (stage_tables)
    void *last_tables_dev = nullptr;
    // pinned host staging
    DevBuf scanrec;                                            // first-round improvement records (P > 1)
    PinBuf h_scanrec;
    PinBuf h_pts, h_small, h_counts, h_status, h_subsets, h_substatus, h_best, h_bestmodels, h_mask, h_epnp;
    PinBuf h_rowinfo;  // rsac_pnp_ransac_batched_rows: {record, n_inliers} per problem
};

// ---------------------------------------------------------------------------
// problem staging
// ---------------------------------------------------------------------------
namespace {

struct Staged {
    int P = 0;
    int64_t total = 0;
    std::vector<int64_t> off;
    int32_t max_n() const {
        int64_t m = 0;
        for (size_t p = 0; p + 1 < off.size(); ++p) m = std::max(m, off[p + 1] - off[p]);
        return (int32_t)m;
    }
    const float *d[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // device SoA
    std::vector<float> hbuf;                                            // host SoA copy (refits, MWC check)
    const float *h[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    bool host_ready = false;
    PnpPrepare prep;  // stage_points(defer): the conversion pnp_args fuses into its frame launch
};

// ncomp3 = 3 for PnP (pts3d N x 3, pts2d N x 2 -> X Y Z U V), 2 for 2D-2D (src, dst -> SX SY DX DY)
// defer: one device-input PnP problem of <= 65536 points, or a batch of problems of at most
// kSetupBatchMaxN points each, is converted by pnp_args' frame launch (the caller must call
// pnp_args next)
int stage_points(rsac_ctx *c, const void *a, const void *b, int ncomp_a, const int64_t *offsets, int32_t P, int32_t n,
                 uint32_t flags, hipStream_t s, Staged &st, bool defer = false) {
    st.P = P;
    st.off.resize(P + 1);
    if (offsets) {
        for (int p = 0; p <= P; ++p) st.off[p] = offsets[p];
        if (st.off[0] != 0) return fail(RSAC_EINVAL, "offsets[0] must be 0");
        for (int p = 0; p < P; ++p)
            if (st.off[p + 1] < st.off[p]) return fail(RSAC_EINVAL, "offsets must be non-decreasing");
    } else {
        st.off[0] = 0;
        st.off[1] = n;
    }
    const int64_t N = st.off[P];
    st.total = N;
    const int nc = ncomp_a + 2;
    if (flags & RSAC_F_DEVICE_SOA) {
        const float *A = (const float *)a, *B = (const float *)b;
        for (int k = 0; k < ncomp_a; ++k) st.d[k] = A + k * N;
        st.d[ncomp_a] = B;
        st.d[ncomp_a + 1] = B + N;
        return RSAC_OK;
    }
    HIPCHK(c->pts.ensure(sizeof(float) * nc * std::max<int64_t>(N, 1)));
    float *D = c->pts.as<float>();
    for (int k = 0; k < nc; ++k) st.d[k] = D + k * N;
    if (flags & RSAC_F_DEVICE_IN) {
        int64_t max_n = 0;
        for (int p = 0; p < P; ++p) max_n = std::max<int64_t>(max_n, st.off[p + 1] - st.off[p]);
        if (ncomp_a == 3 && defer && N > 0 && (P == 1 ? N <= 65536 : max_n <= kSetupBatchMaxN)) {
            st.prep = PnpPrepare{(const double *)a, (const double *)b, D, D + N, D + 2 * N, D + 3 * N, D + 4 * N};
            return RSAC_OK;
        }
        if (ncomp_a == 3)
            HIPCHK(launch_pnp_prepare((const double *)a, (const double *)b, N, D, D + N, D + 2 * N, D + 3 * N,
                                      D + 4 * N, s));
        else
            HIPCHK(launch_hom_prepare((const double *)a, (const double *)b, N, D, D + N, D + 2 * N, D + 3 * N, s));
        return RSAC_OK;
    }
    // host float64 AoS -> float32 SoA (the CV_32F conversion of OpenCV), pinned, one H2D copy
    HIPCHK(hipEventSynchronize(c->ev_pts));
    HIPCHK(c->h_pts.ensure(sizeof(float) * nc * std::max<int64_t>(N, 1)));
    float *H = c->h_pts.as<float>();
    const double *A = (const double *)a, *B = (const double *)b;
    auto convert = [&](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            for (int k = 0; k < ncomp_a; ++k) H[k * N + i] = (float)A[ncomp_a * i + k];
            H[ncomp_a * N + i] = (float)B[2 * i];
            H[(ncomp_a + 1) * N + i] = (float)B[2 * i + 1];
        }
    };
    // large batches (C3 handed over as host arrays: 2M points) convert in chunks on the host pool
    // (converting and copying in slices, the copies overlapping the conversion, measured no
    // faster within the host's run-to-run spread: DESIGN.md §6)
    constexpr int64_t kChunk = 16384;
    if (N > 4 * kChunk)
        parallel_for((int)((N + kChunk - 1) / kChunk),
                     [&](int ch) { convert(ch * kChunk, std::min<int64_t>(N, (int64_t)(ch + 1) * kChunk)); });
    else
        convert(0, N);
    HIPCHK(hipMemcpyAsync(D, H, sizeof(float) * nc * N, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(c->ev_pts, s));
    for (int k = 0; k < nc; ++k) st.h[k] = H + k * N;
    st.host_ready = true;
    return RSAC_OK;
}

// host copy of the staged SoA (needed by refits / the MWC homography check)
int ensure_host_points(Staged &st, int nc, hipStream_t s) {
    if (st.host_ready) return RSAC_OK;
    const int64_t N = st.total;
    st.hbuf.resize(std::max<int64_t>(nc * N, 1));
    for (int k = 0; k < nc; ++k) {
        HIPCHK(hipMemcpyAsync(st.hbuf.data() + k * N, st.d[k], sizeof(float) * N, hipMemcpyDeviceToHost, s));
        st.h[k] = st.hbuf.data() + k * N;
    }
    HIPCHK(hipStreamSynchronize(s));
    st.host_ready = true;
    return RSAC_OK;
}

// small per-problem tables, one H2D copy: offsets (int64 P+1), cams (P x fx fy cx cy, f64),
// thr2 (f32, findInliers' float t = (float)(thresh*thresh))
int stage_tables(rsac_ctx *c, const Staged &st, const double *K, double thresh, hipStream_t s) {
    const int P = st.P;
    auto al = [](size_t b) { return (b + 15) & ~size_t(15); };
    const size_t off_b = al(sizeof(int64_t) * (P + 1)), cam_b = al(sizeof(double) * 4 * P), thr_b = al(sizeof(float) * P);
    const size_t tot = off_b + cam_b + thr_b;
    HIPCHK(c->tables.ensure(tot));
    // the same tables as the previous call (a bench or a multi-GPU driver step): no upload
    std::vector<char> &prev = c->last_tables;
    const bool same_buf = c->last_tables_dev == c->tables.p && prev.size() == tot;
    HIPCHK(hipEventSynchronize(c->ev_small));
    HIPCHK(c->h_small.ensure(tot));
    char *hs = c->h_small.as<char>();
    memcpy(hs, st.off.data(), sizeof(int64_t) * (P + 1));
    double *hc = (double *)(hs + off_b);
    for (int p = 0; p < P; ++p) {
        if (K) {
            const double *k = K + 9 * p;
            hc[4 * p] = k[0]; hc[4 * p + 1] = k[4]; hc[4 * p + 2] = k[2]; hc[4 * p + 3] = k[5];
        } else {
            hc[4 * p] = hc[4 * p + 1] = 1.0; hc[4 * p + 2] = hc[4 * p + 3] = 0.0;
        }
    }
    float *ht = (float *)(hs + off_b + cam_b);
    const float t2 = (float)(thresh * thresh);
    for (int p = 0; p < P; ++p) ht[p] = t2;
    char *d = c->tables.as<char>();
    if (!(same_buf && memcmp(prev.data(), hs, tot) == 0)) {
        HIPCHK(hipMemcpyAsync(d, hs, tot, hipMemcpyHostToDevice, s));
        HIPCHK(hipEventRecord(c->ev_small, s));
        prev.assign(hs, hs + tot);
        c->last_tables_dev = c->tables.p;
    }
    c->d_off = (int64_t *)d;
    c->d_cams = (double *)(d + off_b);
    c->d_thr2 = (float *)(d + off_b + cam_b);
    return RSAC_OK;
}

int ensure_hyp_buffers(rsac_ctx *c, int P, int64_t stride, bool subsets) {
    const size_t recs = (size_t)P * (size_t)stride;
    if (recs * kModelStride * sizeof(double) > kMaxModelBytes)
        return fail(RSAC_ENOMEM, "%lld hypothesis records exceed the resident budget", (long long)recs);
    HIPCHK(c->models.ensure(recs * kModelStride * sizeof(double)));
    HIPCHK(c->fmodels.ensure(recs * kFModelStride * sizeof(float)));
    HIPCHK(c->status.ensure(recs));
    HIPCHK(c->counts.ensure(recs * sizeof(int32_t)));
    HIPCHK(c->best.ensure(sizeof(int64_t) * P));
    HIPCHK(c->bestmodels.ensure(sizeof(double) * kModelStride * P));
    HIPCHK(c->h_best.ensure(sizeof(int64_t) * P));
    HIPCHK(c->h_bestmodels.ensure(sizeof(double) * kModelStride * P));
    if (subsets) {
        HIPCHK(c->subsets.ensure(recs * 5 * sizeof(int32_t)));  // up to 5 indices per sample
        HIPCHK(c->substatus.ensure(recs));
        HIPCHK(c->h_subsets.ensure(recs * 5 * sizeof(int32_t)));
        HIPCHK(c->h_substatus.ensure(recs));
    }
    return RSAC_OK;
}

hipStream_t pick_stream(rsac_ctx *c, void *stream) { return stream ? (hipStream_t)stream : c->stream; }

// PnpArgs for a staged problem set, with the float32 pre-filter frame built
// on the device (unless RSAC_F_EXACT_ONLY).  Call after stage_tables and
// ensure_hyp_buffers.
// defer_setup: a one-problem P3P call's set-up (converted device inputs, k_pnp_setup_fc) is left to
// the first solve launch (c->pending_setup), which runs it beside the solve (k_pnp_setup_solve4);
// the caller launches nothing that reads the points, the frame or the queue before that solve, or
// calls flush_setup.
int pnp_args(rsac_ctx *c, const Staged &st, uint32_t flags, uint64_t seed, int64_t stride, int64_t rng_base,
             hipStream_t s, PnpArgs &a, unsigned long long *best_key = nullptr, bool defer_setup = false) {
    c->pending_on = false;
    a = PnpArgs{};
    a.X = st.d[0]; a.Y = st.d[1]; a.Z = st.d[2]; a.U = st.d[3]; a.V = st.d[4];
    a.offsets = c->d_off;
    a.max_n = st.max_n();
    a.cams = c->d_cams;
    a.thr2 = c->d_thr2;
    a.models = c->models.as<double>();
    a.status = c->status.as<int8_t>();
    a.hyp_stride = stride;
    a.rng_base = rng_base;
    a.seed = seed;
    a.best_key = best_key;
    const int P = st.P;
    const int64_t N = st.total;
    HIPCHK(c->queue.ensure(4096));  // kQWords ints (rsac_kernels.hip)
    HIPCHK(c->bounds_ws.ensure(sizeof(int32_t) * 10 * P));
    HIPCHK(c->frame.ensure(sizeof(double) * kFrameStride * P));
    HIPCHK(c->fconst.ensure(sizeof(float) * kFconstStride * P));
    a.queue = c->queue.as<int>();
    a.exact_only = (flags & RSAC_F_EXACT_ONLY) ? 1 : 0;
    a.sample_k = (flags & RSAC_F_MINIMAL_EPNP5) ? 5 : 4;  // EPnP-5: ensure_epnp5 before each solve
    a.rvec_rt = (flags & RSAC_F_RVEC_ROUNDTRIP) ? 1 : 0;
    a.dbg_cell_pts = c->dbg_cell_pts;
    int32_t max_n = 0;
    for (int p = 0; p < P; ++p) max_n = std::max<int32_t>(max_n, (int32_t)(st.off[p + 1] - st.off[p]));
    // resets best_key and the queue, then builds the frame (also in exact mode: cheap)
    // one problem: k_pnp_setup_fc's scratch (its ticket starts at 0; the kernel resets it)
    if (!a.exact_only) {  // the MFMA scorer's point operands, written with the centring
        HIPCHK(c->mxpts.ensure(40 * std::max<int64_t>(N, 1)));
        a.PF = c->mxpts.as<uint4>();
        a.UV = reinterpret_cast<float2 *>(c->mxpts.as<char>() + 32 * std::max<int64_t>(N, 1));
    }
    PnpPrepare prep = st.prep;
    if (P == 1) {
        if (!c->setup_scr.p) {
            HIPCHK(c->setup_scr.ensure(64 + sizeof(float) * 10 * kSetupMaxBlocks));
            HIPCHK(hipMemsetAsync(c->setup_scr.p, 0, 64, s));
        }
        prep.ticket = c->setup_scr.as<int>();
        prep.part = (float *)(c->setup_scr.as<char>() + 64);
    }
    if (defer_setup && P == 1 && a.sample_k == 4 && !a.exact_only && !(flags & RSAC_F_LO) && prep.p3 && prep.part &&
        prep.ticket && max_n <= 65536) {
        c->pending_setup = PnpSetupFuse{prep, max_n, c->bounds_ws.as<int32_t>(), c->frame.as<double>(),
                                        c->fconst.as<float>()};
        c->pending_on = true;
    } else {
        HIPCHK(launch_pnp_frame(a, P, max_n, c->bounds_ws.as<int32_t>(), nullptr, nullptr, nullptr,
                                c->frame.as<double>(), c->fconst.as<float>(), s, &prep));
    }
    if (!a.exact_only) {
        a.counts_out = c->counts.as<int32_t>();
        a.frame = c->frame.as<double>();
        a.fconst = c->fconst.as<float>();
        a.fmodels = c->fmodels.as<float>();
        a.fform = 2;  // MFMA records (form 1 for small rounds and out-of-f16-range problems)
    }
    return RSAC_OK;
}

// the deferred set-up alone (a path that does not start with a fusable P3P solve)
int flush_setup(rsac_ctx *c, const PnpArgs &a, hipStream_t s) {
    if (!c->pending_on) return RSAC_OK;
    c->pending_on = false;
    const PnpSetupFuse &f = c->pending_setup;
    HIPCHK(launch_pnp_frame(a, 1, f.max_n, f.ws, nullptr, nullptr, nullptr, f.frame, f.fconst, s, &f.prep));
    return RSAC_OK;
}

// the EPnP-5 solve's scratch for launches of up to P x H hypotheses (kEpnpRec doubles each, at
// launch-local positions: one round's worth, not one per hypothesis record), within the resident
// budget; a no-op for P3P
int ensure_epnp5(rsac_ctx *c, PnpArgs &a, int32_t P, int64_t H) {
    if (a.sample_k != 5) return RSAC_OK;
    const size_t bytes = (size_t)std::max(P, 1) * (size_t)std::max<int64_t>(H, 1) * kEpnpRec * sizeof(double);
    if (bytes > kMaxModelBytes)
        return fail(RSAC_ENOMEM, "EPnP-5 scratch for %lld hypotheses exceeds the resident budget",
                    (long long)P * (long long)H);
    HIPCHK(c->epnp5.ensure(bytes));
    a.epnp = c->epnp5.as<double>();
    return RSAC_OK;
}

// fundamental matrix: the f32 Sampson pre-filter's records and coordinate bounds (unless
// RSAC_F_EXACT_ONLY, which keeps the all-f64 scoring kernel).  Call after ensure_hyp_buffers.
int fm_prefilter(rsac_ctx *c, HomArgs &a, int32_t P, uint32_t flags, hipStream_t s) {
    if (flags & RSAC_F_EXACT_ONLY) return RSAC_OK;
    HIPCHK(c->bounds_ws.ensure(sizeof(int32_t) * 10 * P));  // >= 8 per problem
    a.fmodels = c->fmodels.as<float>();
    a.fbounds = c->bounds_ws.as<int>();
    HIPCHK(c->queue.ensure(4096));  // kQWords ints (rsac_kernels.hip)
    a.fm_queue = c->queue.as<int>() + 8;  // its own counter (the PnP kernels use word 0)
    HIPCHK(launch_fm_bounds(a, P, a.max_n, c->bounds_ws.as<int>(), s));
    return RSAC_OK;
}

enum class Model { PnP, Hom, Fm };  // Fm: fundamental matrix on the HomArgs block

// The RANSAC loop of RANSACPointSetRegistrator::run for P problems at once:
// rounds of `round` hypotheses are solved + scored on the GPU, then every
// unfinished problem's scan consumes them in index order.
struct LoopOut {
    std::vector<ScanState> scan;
    int rounds = 0;
    int64_t scored = 0;
    double gpu_ms = 0, solve_ms = 0, score_ms = 0;
    int32_t lo_improvements = 0;
    // speculative first round (run_loop with a ScanDecide): the records are on their way to
    // the host and the device has picked the winner; spec_resolve replays and verifies
    bool spec_pending = false;
    ScanFuse fuse;  // a pending speculative PnP scan: the finish's mask launch runs it (k_scan_mask)
    int64_t spec_H = 0;
    bool timing = true;  // HIP events around solve / score (the caller wants rsac_stats)
    // OpenCV's sampler: one MWC state per problem, carried across rounds and across the resume of a
    // speculative first round
    std::vector<Mwc> rngs;
};

// LO-RANSAC local optimisation of the new best of problem 0 (DESIGN.md "LO-RANSAC";
// the oracle's orc_pnp_ransac_lo): up to 4 rounds of LM refit on the current inliers +
// recount, kept while the count rises.  An improved model replaces the best
// hypothesis' record, so the final mask / gather / refit see it.
constexpr int kLoSteps = 4;

// the multi-block LM refit's scratch (rsac_internal.h LmScratch; granules zeroed once here),
// the device's co-resident block limit for it, and the pinned failure word
LmScratch *lm_scratch(rsac_ctx *c, hipStream_t s) {
    if (!c->lmscr.p) {
        if (c->lmscr.ensure(kLmGranuleBytes) != hipSuccess) return nullptr;
        if (hipMemsetAsync(c->lmscr.p, 0, kLmGranuleBytes, s) != hipSuccess) return nullptr;
        if (c->h_lmfail.ensure(sizeof(int32_t)) != hipSuccess) return nullptr;
        *c->h_lmfail.as<int32_t>() = 0;
        c->lm.gran = (unsigned long long *)c->lmscr.p;
        c->lm.fail = c->h_lmfail.as<int32_t>();
        c->lm.launch = 0;
        int coop = 0;
        const char *ev = getenv("RSAC_REFIT_COOP");
        if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, c->device) == hipSuccess)
            c->lm.coop = coop && ev && ev[0] == '1';  // opt-in: +25 us on C2 ms-to-best (scripts/refit_coop_ab.py)
    }
    if (c->lm.max_blocks == 0) {
        c->lm.max_blocks = pnp_refine_coresident(c->device);
        if (c->dbg_refit_max_blocks > 0) c->lm.max_blocks = std::min(c->lm.max_blocks, c->dbg_refit_max_blocks);
    }
    return &c->lm;
}

// after the synchronisation that follows refits: a multi-block refit whose range sums never
// all arrived (its blocks were not all co-resident: other work held the CUs for longer than the
// kernel's ~1 s wait) kept the start pose and set the failure word.  The caller then redoes the
// call with one block per refit (with_one_refit_block), which needs no co-residency and gives
// the same bits.
constexpr int kRetryOneBlock = -1000;  // internal: not an RSAC_* code, never returned to callers
int lm_check(rsac_ctx *c) {
    int32_t *f = c->h_lmfail.as<int32_t>();
    if (f && __atomic_load_n(f, __ATOMIC_ACQUIRE)) {
        *f = 0;
        if (c->lm.max_blocks > 1) return kRetryOneBlock;
        return fail(RSAC_EHIP, "pose refit: a single-block LM refit lost its own range sums");
    }
    return RSAC_OK;
}

// run `call` (an API body); when one of its multi-block refits failed for lack of co-residency,
// run it again with every refit on one block
template <class F>
int with_one_refit_block(rsac_ctx *c, F call) {
    int r = call();
    if (r != kRetryOneBlock) return r;
    const int saved = c->lm.max_blocks;
    c->lm.max_blocks = 1;
    c->lo_state_base = nullptr;  // an LO chain's device state starts from zero again
    r = call();
    c->lm.max_blocks = saved;
    return r == kRetryOneBlock ? fail(RSAC_EHIP, "pose refit failed with one block") : r;
}

// The kLoSteps steps are enqueued at once and decided on the device (k_pnp_lo_count): step k
// refits record src_k on mask k into rec[(k + 1) % 2], recounts it, and either makes it the best
// (copied over the best hypothesis' record) or ends the chain, after which the remaining
// launches are no-ops.  One synchronisation per LO call; the state comes back in pinned memory.
int local_opt(rsac_ctx *c, const PnpArgs &a, int32_t n, ScanState &sc, double confidence, hipStream_t s,
              int32_t &improvements) {
    const size_t rec_bytes = sizeof(double) * kModelStride;
    HIPCHK(c->lo.ensure(2 * rec_bytes + 64 + 2 * (size_t)std::max(n, 1)));
    HIPCHK(c->h_lo.ensure(sizeof(LoState)));
    double *rec[2] = {c->lo.as<double>(), c->lo.as<double>() + kModelStride};
    LoState *st = (LoState *)(rec[1] + kModelStride);
    uint8_t *mk[2] = {(uint8_t *)st + 64, (uint8_t *)st + 64 + std::max(n, 1)};
    if (c->lo_state_base != c->lo.p) {  // count and ticket must start at 0 (then self-resetting)
        HIPCHK(hipMemsetAsync(st, 0, sizeof(LoState), s));
        c->lo_state_base = c->lo.p;
    }
    LoState *hst = c->h_lo.as<LoState>();
    double *best_rec = a.models + sc.best * kModelStride;  // problem 0: record index = hypothesis
    HIPCHK(launch_pnp_lo_count(a, n, best_rec, mk[0], st, -1, sc.max_good, nullptr, hst, s));
    for (int step = 0; step < kLoSteps; ++step) {
        const double *src = step == 0 ? best_rec : rec[step & 1];
        double *dst = rec[(step + 1) & 1];
        HIPCHK(launch_pnp_refine(a, 1, mk[step & 1], dst, nullptr, s, lm_scratch(c, s), nullptr, nullptr, src,
                                 &st->stopped));
        HIPCHK(launch_pnp_lo_count(a, n, dst, mk[(step + 1) & 1], st, step, 0, best_rec, hst, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (int r = lm_check(c)) return r;
    improvements += hst->improvements;
    if (hst->improvements > 0 && hst->cur > sc.max_good) {
        sc.max_good = hst->cur;
        sc.niters = update_num_iters(confidence, (double)(n - hst->cur) / n, a.sample_k, (int)sc.niters);
        if (sc.iter >= sc.niters) sc.done = true;
    }
    return RSAC_OK;
}

void add_times(rsac_ctx *c, double &gpu, double &solve, double &score) {
    float a = 0, b = 0;
    if (hipEventElapsedTime(&a, c->ev0, c->ev1) == hipSuccess) solve += a;
    if (hipEventElapsedTime(&b, c->ev1, c->ev2) == hipSuccess) score += b;
    gpu += (double)a + (double)b;
}

int run_loop(rsac_ctx *c, Model model, const Staged &st, void *args, int32_t max_iters, double confidence,
             uint32_t flags, hipStream_t s, LoopOut &out, const ScanDecide *spec = nullptr, bool resume = false,
             int max_rounds = 0) {
    const int P = st.P;
    const int64_t H = std::max(max_iters, 1);
    const bool adaptive = (flags & RSAC_F_ADAPTIVE) != 0;
    const bool lo = (flags & RSAC_F_LO) != 0 && model == Model::PnP && P == 1;
    const int64_t round = adaptive ? std::min<int64_t>(std::max<int64_t>(c->round_size, 64), H) : H;
    const int64_t stride = H;
    int r = ensure_hyp_buffers(c, P, stride, (flags & RSAC_F_SAMPLER_OPENCV) != 0);
    if (r) return r;
    HIPCHK(c->h_counts.ensure(sizeof(int32_t) * P * round));
    HIPCHK(c->h_status.ensure((size_t)P * round));

    PnpArgs *pa = model == Model::PnP ? (PnpArgs *)args : nullptr;
    HomArgs *ha = model != Model::PnP ? (HomArgs *)args : nullptr;
    if (pa) {  // a round is at most `round` hypotheses of each problem
        r = ensure_epnp5(c, *pa, P, round);
        if (r) return r;
    }
    // RANSACUpdateNumIters' model_points = the sample size (5 for the EPnP-5 minimal solver)
    const int model_points = model == Model::Fm ? 8 : pa ? pa->sample_k : 4;
    const int sk = model_points;  // indices per drawn subset
#define SETARG(field, val) \
    do {                   \
        if (pa) pa->field = (val); else ha->field = (val); \
    } while (0)
    SETARG(models, c->models.as<double>());
    SETARG(status, c->status.as<int8_t>());
    SETARG(hyp_stride, stride);
    SETARG(subsets, (const int32_t *)nullptr);
    SETARG(sub_status, (const int8_t *)nullptr);

    // OpenCV's subset sequence is sequential in one MWC state per problem and call: the
    // states persist across rounds, each round's slice is drawn on the host (problems in
    // parallel) and uploaded before its solve
    const bool opencv = (flags & RSAC_F_SAMPLER_OPENCV) != 0;
    std::vector<Mwc> &rngs = out.rngs;
    if (opencv) {
        if (!resume) rngs.assign(P, Mwc());
        SETARG(subsets, c->subsets.as<int32_t>());
        SETARG(sub_status, c->substatus.as<int8_t>());
    }
#undef SETARG

    // adaptive: the first round is short (most runs stop within it), later ones double
    int64_t cur = adaptive ? std::min<int64_t>(round, 256) : round;
    int64_t hb0 = 0;
    if (resume) {  // after a verified speculative first round (OpenCV's sampler: out.rngs carries on)
        hb0 = out.spec_H;
        cur = std::min<int64_t>(cur * 2, round);
    } else {
        out.scan.assign(P, ScanState());
        for (auto &sc : out.scan) sc.reset((int)H);
    }
    for (int64_t hb = hb0, Hr = 0; hb < H; hb += Hr) {
        if (max_rounds > 0 && out.rounds >= max_rounds) break;  // the caller goes on (first-round mode)
        Hr = std::min<int64_t>(cur, H - hb);
        cur = std::min<int64_t>(cur * 2, round);
        if (opencv) {
            int32_t *hs = c->h_subsets.as<int32_t>();
            int8_t *hss = c->h_substatus.as<int8_t>();
            parallel_for(P, [&](int p) {
                int8_t *os = hss + (size_t)p * stride + hb;
                const int np = (int)(st.off[p + 1] - st.off[p]);
                if (np < sk || out.scan[p].done) {  // nothing to draw: the solve skips status < 0
                    memset(os, -1, Hr);
                    return;
                }
                const float *hom[4];
                if (model == Model::Hom)
                    for (int k = 0; k < 4; ++k) hom[k] = st.h[k] + st.off[p];
                mwc_subsets(rngs[p], np, Hr, model == Model::Hom ? hom : nullptr, hs + ((size_t)p * stride + hb) * sk,
                            os, sk);
            });
            // a small round's subsets are read by the solve straight from the pinned host rows (no
            // copy launches in the latency path: an adaptive run's first round); larger rounds go
            // to the device in two copies.  Either way the host rewrites the rows only after the
            // round's synchronisation.
            const bool zero_copy = (int64_t)P * Hr * (4 * sk + 1) <= kSubsetZeroCopyBytes;
            const int32_t *sub = zero_copy ? hs : c->subsets.as<int32_t>();
            const int8_t *sst = zero_copy ? hss : c->substatus.as<int8_t>();
            if (!zero_copy) {
                HIPCHK(copy_rows(c->subsets.as<int32_t>() + hb * sk, sizeof(int32_t) * sk * stride, hs + hb * sk,
                                 sizeof(int32_t) * sk * stride, sizeof(int32_t) * sk * Hr, P, hipMemcpyHostToDevice,
                                 s));
                HIPCHK(copy_rows(c->substatus.as<int8_t>() + hb, stride, hss + hb, stride, Hr, P,
                                 hipMemcpyHostToDevice, s));
            }
            if (pa) {
                pa->subsets = sub;
                pa->sub_status = sst;
            } else {
                ha->subsets = sub;
                ha->sub_status = sst;
            }
        }
        if (out.timing) HIPCHK(hipEventRecord(c->ev0, s));
        if (pa) {
            // the deferred set-up beside the round's solve; the scorer then builds the records
            const bool fused = c->pending_on && P == 1 && pnp_setup_fusable(*pa, (int32_t)Hr);
            if (fused) {
                c->pending_on = false;
                HIPCHK(launch_pnp_solve(*pa, P, hb, Hr, s, &c->pending_setup));
            } else {
                r = flush_setup(c, *pa, s);
                if (r) return r;
                HIPCHK(launch_pnp_solve(*pa, P, hb, Hr, s));
            }
            if (out.timing) HIPCHK(hipEventRecord(c->ev1, s));
            pa->fm_inline = fused ? 1 : 0;
            const hipError_t se = launch_pnp_score(*pa, P, hb, Hr, c->counts.as<int32_t>(), s);
            pa->fm_inline = 0;
            HIPCHK(se);
        } else if (model == Model::Fm) {
            HIPCHK(launch_fm_solve(*ha, P, hb, Hr, s));
            if (out.timing) HIPCHK(hipEventRecord(c->ev1, s));
            HIPCHK(launch_fm_score(*ha, P, hb, Hr, c->counts.as<int32_t>(), s));
        } else {
            HIPCHK(launch_hom_solve(*ha, P, hb, Hr, s));
            if (out.timing) HIPCHK(hipEventRecord(c->ev1, s));
            HIPCHK(launch_hom_score(*ha, P, hb, Hr, c->counts.as<int32_t>(), s));
        }
        if (out.timing) HIPCHK(hipEventRecord(c->ev2, s));
        // the first round without LO: the device lists each problem's scan improvements
        // (prefix-maximum records) and the host replays the exact scan on them; later rounds (and
        // LO) copy every count
        std::vector<int> full;  // problems scanned from their full count / status rows
        if (!lo && hb == 0) {
            HIPCHK(c->h_scanrec.ensure(sizeof(ScanRecords) * P));
            // a speculative one-problem PnP round: the finish's mask launch replays the scan itself
            // (k_scan_mask), one launch fewer in front of the refit.  (Batches keep the two launches:
            // every mask block of every problem replaying its problem's scan made C3's scan + masks
            // 39 us against 21, r05.)
            const bool fuse = spec && P == 1 && model == Model::PnP && scan_mask_fusable((int32_t)Hr);
            if (fuse) {
                out.fuse = ScanFuse{true, c->counts.as<int32_t>(), c->status.as<int8_t>(), stride, (int32_t)Hr,
                                    model_points, c->h_scanrec.as<ScanRecords>(), *spec};
            } else if (P == 1) {
                // one problem: the kernel writes its record straight into pinned host memory (no
                // copy launch); many problems: device records and one copy (thousands of scattered
                // 4-byte writes over PCIe cost more than the copy)
                HIPCHK(launch_scan_records(c->counts.as<int32_t>(), c->status.as<int8_t>(), stride, P, (int32_t)Hr,
                                           model_points, c->h_scanrec.as<ScanRecords>(), s,
                                           spec ? *spec : ScanDecide()));
            } else {
                HIPCHK(c->scanrec.ensure(sizeof(ScanRecords) * P));
                HIPCHK(launch_scan_records(c->counts.as<int32_t>(), c->status.as<int8_t>(), stride, P, (int32_t)Hr,
                                           model_points, c->scanrec.as<ScanRecords>(), s,
                                           spec ? *spec : ScanDecide()));
                // a speculative finish: copied behind the finish's mask kernel (issue_scanrec_copy),
                // which would otherwise wait for the copy
                if (spec)
                    c->scanrec_copy = P;
                else
                    HIPCHK(hipMemcpyAsync(c->h_scanrec.p, c->scanrec.p, sizeof(ScanRecords) * P,
                                          hipMemcpyDeviceToHost, s));
            }
            if (spec) {  // no synchronisation: the caller enqueues the finish, then spec_resolve
                out.spec_pending = true;
                out.spec_H = Hr;
                return RSAC_OK;
            }
            HIPCHK(hipStreamSynchronize(s));
            const ScanRecords *rec = c->h_scanrec.as<ScanRecords>();
            for (int p = 0; p < P; ++p) {
                if (rec[p].nrec < 0) {
                    full.push_back(p);
                    continue;
                }
                const int np = (int)(st.off[p + 1] - st.off[p]);
                scan_records(out.scan[p], rec[p].idx, rec[p].cnt, rec[p].nrec, rec[p].first_neg, (int64_t)Hr, np,
                             model_points, confidence);  // the first round: the scan starts at 0
            }
            if (!full.empty()) {
                HIPCHK(copy_rows(c->h_counts.p, sizeof(int32_t) * Hr, c->counts.as<int32_t>() + hb,
                                 sizeof(int32_t) * stride, sizeof(int32_t) * Hr, P, hipMemcpyDeviceToHost, s));
                HIPCHK(copy_rows(c->h_status.p, Hr, c->status.as<int8_t>() + hb, stride, Hr, P, hipMemcpyDeviceToHost,
                                 s));
                HIPCHK(hipStreamSynchronize(s));
                for (int p : full) {
                    const int np = (int)(st.off[p + 1] - st.off[p]);
                    scan_step(out.scan[p], c->h_counts.as<int32_t>() + (size_t)p * Hr,
                              c->h_status.as<int8_t>() + (size_t)p * Hr, Hr, np, model_points, confidence);
                }
            }
            if (out.timing) add_times(c, out.gpu_ms, out.solve_ms, out.score_ms);
            out.rounds++;
            out.scored += (int64_t)Hr;
            bool all_done = true;
            for (int p = 0; p < P; ++p) all_done = all_done && out.scan[p].done;
            if (all_done) break;
            continue;  // later rounds copy their counts
        }
        HIPCHK(copy_rows(c->h_counts.p, sizeof(int32_t) * Hr, c->counts.as<int32_t>() + hb,
                                sizeof(int32_t) * stride, sizeof(int32_t) * Hr, P, hipMemcpyDeviceToHost, s));
        HIPCHK(copy_rows(c->h_status.p, Hr, c->status.as<int8_t>() + hb, stride, Hr, P,
                                hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (out.timing) add_times(c, out.gpu_ms, out.solve_ms, out.score_ms);
        out.rounds++;
        out.scored += (int64_t)Hr;
        bool all_done = true;
        for (int p = 0; p < P; ++p) {
            ScanState &sc = out.scan[p];
            const int np = (int)(st.off[p + 1] - st.off[p]);
            const int32_t *cr = c->h_counts.as<int32_t>() + (size_t)p * Hr;
            const int8_t *sr = c->h_status.as<int8_t>() + (size_t)p * Hr;
            if (lo) {
                // stop at every new best, optimise it locally, continue with the raised floor
                while (!sc.done && sc.iter < hb + Hr) {
                    scan_step(sc, cr + (sc.iter - hb), sr + (sc.iter - hb), hb + Hr - sc.iter, np, model_points,
                              confidence, true);
                    if (sc.improved) {
                        sc.improved = false;
                        int rr = local_opt(c, *pa, np, sc, confidence, s, out.lo_improvements);
                        if (rr) return rr;
                    }
                }
            } else if (!sc.done) {
                scan_step(sc, cr, sr, Hr, np, model_points, confidence);
            }
            all_done = all_done && sc.done;
        }
        if (all_done) break;
    }
    return RSAC_OK;
}

// the deferred copy of a speculative round's device scan records to the host (run_loop)
hipError_t issue_scanrec_copy(rsac_ctx *c, hipStream_t s) {
    if (!c->scanrec_copy) return hipSuccess;
    const size_t bytes = sizeof(ScanRecords) * c->scanrec_copy;
    c->scanrec_copy = 0;
    return hipMemcpyAsync(c->h_scanrec.p, c->scanrec.p, bytes, hipMemcpyDeviceToHost, s);
}

// after the stream synchronised: the host's replay of a speculative first round (one problem).
// ok: it ended the scan with the winner the device picked (the finish enqueued on the device's
// pick is the result); otherwise the caller starts over without speculation.
int spec_resolve(rsac_ctx *c, const Staged &st, LoopOut &out, int model_points, double confidence, bool &ok,
                 bool fixed, int64_t stride, hipStream_t s) {
    const int P = fixed ? st.P : 1;
    if (c->scanrec_copy) {  // not yet issued by a finish: copy and wait here
        HIPCHK(issue_scanrec_copy(c, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    const ScanRecords *recs = c->h_scanrec.as<ScanRecords>();
    out.spec_pending = false;
    ok = false;
    if (!fixed && (recs[0].nrec < 0 || c->dbg_spec_overflow)) {  // more improvements than records: the caller runs the loop afresh
        out.scan[0].reset((int)out.scan[0].niters);
        out.spec_H = 0;
        return RSAC_OK;
    }
    std::vector<int> full;  // problems with more improvements than records: their full rows
    for (int p = 0; p < P; ++p) {
        const ScanRecords &rec = recs[p];
        if (rec.nrec < 0) {
            full.push_back(p);
            continue;
        }
        const int np = (int)(st.off[p + 1] - st.off[p]);
        scan_records(out.scan[p], rec.idx, rec.cnt, rec.nrec, rec.first_neg, out.spec_H, np, model_points,
                     confidence);
    }
    if (!full.empty()) {
        const int64_t Hr = out.spec_H;
        HIPCHK(c->h_counts.ensure(sizeof(int32_t) * P * Hr));
        HIPCHK(c->h_status.ensure((size_t)P * Hr));
        HIPCHK(copy_rows(c->h_counts.p, sizeof(int32_t) * Hr, c->counts.as<int32_t>(), sizeof(int32_t) * stride,
                         sizeof(int32_t) * Hr, P, hipMemcpyDeviceToHost, s));
        HIPCHK(copy_rows(c->h_status.p, Hr, c->status.as<int8_t>(), stride, Hr, P, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int p : full) {
            const int np = (int)(st.off[p + 1] - st.off[p]);
            scan_step(out.scan[p], c->h_counts.as<int32_t>() + (size_t)p * Hr,
                      c->h_status.as<int8_t>() + (size_t)p * Hr, Hr, np, model_points, confidence);
        }
    }
    if (out.timing) add_times(c, out.gpu_ms, out.solve_ms, out.score_ms);
    out.rounds = 1;
    out.scored = out.spec_H;
    ok = true;
    for (int p = 0; p < P; ++p) {
        const ScanRecords &rec = recs[p];
        // (fixed budget: the round was the whole budget, whether or not the scan flagged it done)
        ok = ok && (fixed || out.scan[p].done) && rec.dev_done && out.scan[p].best == (int64_t)rec.dev_best;
    }
    return RSAC_OK;
}

// masks + winning models of every problem; records of winners -> c->best
// defer_sync: leave the stream running (the caller enqueues more work, synchronises, then
// calls finish_masks_host to copy a host mask out)
// dev_best: the winners' record indices are already on the device (c->best, a speculative
// first round), not in lo
int finish_masks(rsac_ctx *c, Model model, const Staged &st, void *args, const LoopOut &lo, int64_t stride,
                 uint8_t *mask_out, uint32_t flags, hipStream_t s, bool defer_sync = false, bool dev_best = false) {
    const int P = st.P;
    int64_t *hb = c->h_best.as<int64_t>();
    for (int p = 0; p < P; ++p) hb[p] = lo.scan[p].best >= 0 ? (int64_t)p * stride + lo.scan[p].best : -1;
    // one problem: the record index goes as a kernel argument (no upload)
    const int64_t *dbest = P == 1 && !dev_best ? nullptr : c->best.as<int64_t>();
    if (P > 1 && !dev_best)
        HIPCHK(hipMemcpyAsync(c->best.p, hb, sizeof(int64_t) * P, hipMemcpyHostToDevice, s));
    const int64_t N = st.total;
    // PnP: the mask kernel also gathers the winners' records (one launch fewer)
    const bool fused_gather = model == Model::PnP && N > 0;
    if (!fused_gather)
        HIPCHK(launch_gather_models(c->models.as<double>(), dbest, P, c->bestmodels.as<double>(), s, hb[0]));
    int32_t max_n = 0;
    for (int p = 0; p < P; ++p) max_n = std::max<int32_t>(max_n, (int32_t)(st.off[p + 1] - st.off[p]));
    uint8_t *dmask;
    if (flags & RSAC_F_DEVICE_OUT) {
        dmask = mask_out;
    } else {
        HIPCHK(c->mask.ensure(std::max<int64_t>(N, 1)));
        dmask = c->mask.as<uint8_t>();
    }
    if (N > 0) {
        // without a refit the winners also go straight to the pinned host records
        double *hmodels = defer_sync ? nullptr : c->h_bestmodels.as<double>();
        if (model == Model::PnP && dev_best && lo.fuse.pending)  // the speculative round's scan, then the masks
            HIPCHK(launch_scan_mask(lo.fuse, *(PnpArgs *)args, P, max_n, dmask, c->bestmodels.as<double>(), hmodels,
                                    s));
        else if (model == Model::PnP)
            HIPCHK(launch_pnp_mask(*(PnpArgs *)args, P, max_n, dbest, dmask, s, hb[0], c->bestmodels.as<double>(),
                                   hmodels));
        else if (model == Model::Fm)
            HIPCHK(launch_fm_mask(*(HomArgs *)args, P, max_n, dbest, dmask, s, hb[0]));
        else
            HIPCHK(launch_hom_mask(*(HomArgs *)args, P, max_n, dbest, dmask, s, hb[0]));
    }
    HIPCHK(issue_scanrec_copy(c, s));
    // the winners' records for the host (a refit copies the refined ones instead)
    if (!defer_sync && !(model == Model::PnP && N > 0))
        HIPCHK(hipMemcpyAsync(c->h_bestmodels.p, c->bestmodels.p, sizeof(double) * kModelStride * P,
                              hipMemcpyDeviceToHost, s));
    if (!(flags & RSAC_F_DEVICE_OUT) && mask_out && N > 0) {
        HIPCHK(c->h_mask.ensure(N));
        HIPCHK(hipMemcpyAsync(c->h_mask.p, dmask, N, hipMemcpyDeviceToHost, s));
        if (defer_sync) return RSAC_OK;
        HIPCHK(hipStreamSynchronize(s));
        memcpy(mask_out, c->h_mask.p, N);
    } else if (!defer_sync) {
        HIPCHK(hipStreamSynchronize(s));
    }
    return RSAC_OK;
}

// after a deferred finish_masks and a stream synchronisation: the host mask copy-out
void finish_masks_host(rsac_ctx *c, const Staged &st, uint8_t *mask_out, uint32_t flags) {
    if (!(flags & RSAC_F_DEVICE_OUT) && mask_out && st.total > 0) memcpy(mask_out, c->h_mask.p, st.total);
}

int check_device(rsac_ctx *c) {
    if (!c) return fail(RSAC_EINVAL, "null context");
    HIPCHK(hipSetDevice(c->device));
    return RSAC_OK;
}

// mask for refits when the caller wanted the mask on the device (or not at all)
int host_mask(rsac_ctx *c, const Staged &st, uint8_t *mask_out, uint32_t flags, hipStream_t s,
              std::vector<uint8_t> &tmp, const uint8_t **hm) {
    if (mask_out && !(flags & RSAC_F_DEVICE_OUT)) {
        *hm = mask_out;
        return RSAC_OK;
    }
    tmp.resize(std::max<int64_t>(st.total, 1));
    const uint8_t *src = (flags & RSAC_F_DEVICE_OUT) && mask_out ? mask_out : c->mask.as<uint8_t>();
    HIPCHK(hipMemcpyAsync(tmp.data(), src, st.total, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *hm = tmp.data();
    return RSAC_OK;
}

// the winners' masks, then the final solve on the device, one block per problem, on the
// RANSAC-phase inliers: EPnP (solvePnPRansac with SOLVEPNP_P3P), then / or LM
// (solvePnPRefineLM); returns with the stream synchronised and c->h_bestmodels filled.
// dev_best: the winners come from the device's speculative replay (c->best)
int pnp_finish(rsac_ctx *c, const Staged &st, const PnpArgs &a, const LoopOut &lo, int64_t stride, const double *K,
               uint8_t *mask_out, uint32_t flags, hipStream_t s, bool refit, bool dev_best) {
    const int P = st.P;
    int r = finish_masks(c, Model::PnP, st, (void *)&a, lo, stride, mask_out, flags, s, refit, dev_best);
    if (r || !refit) return r;
    const uint8_t *dmask = (flags & RSAC_F_DEVICE_OUT) && mask_out ? mask_out : c->mask.as<uint8_t>();
    if (flags & RSAC_F_EPNP) {
        // stage 1 (sums) on the device, stage 2 (12 x 12 eigenvectors + betas, O(1)) on the
        // host, stage 3 (pose candidates) on the device
        const size_t b1 = sizeof(EpnpStage1) * P, b2 = sizeof(EpnpStage2) * P;
        HIPCHK(c->epnp.ensure(b1 + b2));
        HIPCHK(c->h_epnp.ensure(b1 + b2));
        EpnpStage1 *d1 = c->epnp.as<EpnpStage1>(), *h1 = c->h_epnp.as<EpnpStage1>();
        EpnpStage2 *d2 = (EpnpStage2 *)(d1 + P), *h2 = (EpnpStage2 *)(h1 + P);
        HIPCHK(launch_pnp_epnp_s1(a, P, dmask, c->bestmodels.as<double>(), d1, s));
        HIPCHK(hipMemcpyAsync(h1, d1, b1, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        parallel_for(P, [&](int p) {
            const double *Kp = K + 9 * p;
            if (h1[p].ok != 0.0) epnp_stage2(h1[p], Cam{Kp[0], Kp[4], Kp[2], Kp[5]}, h2[p]);
            else memset(&h2[p], 0, sizeof(EpnpStage2));
        });
        HIPCHK(hipMemcpyAsync(d2, h2, b2, hipMemcpyHostToDevice, s));
        HIPCHK(launch_pnp_epnp_s3(a, P, dmask, d1, d2, c->bestmodels.as<double>(), s));
    }
    if (flags & RSAC_F_REFINE)  // the refit also writes R, t into the pinned host records
        HIPCHK(launch_pnp_refine(a, P, dmask, c->bestmodels.as<double>(), nullptr, s, lm_scratch(c, s),
                                 st.off.data(), c->h_bestmodels.as<double>()));
    else
        HIPCHK(hipMemcpyAsync(c->h_bestmodels.p, c->bestmodels.p, sizeof(double) * kModelStride * P,
                              hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (flags & RSAC_F_REFINE)
        if (int r = lm_check(c)) return r;
    finish_masks_host(c, st, mask_out, flags);
    return RSAC_OK;
}

// OpenCV's `count == model_points` branches ([OpenCV, unvendored] solvepnp.cpp solvePnPRansac,
// fundam.cpp findHomography; reached from main_v1.py:497-502, testpro-K.py:72-75, main_v1.py:312):
// no RANSAC.  The minimal kernel runs once on all the points in input order (no subset check), the
// result is its model with every index an inlier, and there is no final solve (no LM / EPnP refit,
// no homography LM).  PnP: 4 points -> P3P whatever the flags (model_points is 4 for
// SOLVEPNP_P3P / AP3P and for npoints == 4), 5 points under the default flags -> EPnP
// (model_points 5; RSAC_F_MINIMAL_EPNP5).  Homography: 4 points -> runKernel, method 0's path.
// A failed solve -> no model and no inliers.  kind[p] = the direct sample size of problem p, 0 for
// a RANSAC problem.
std::vector<int8_t> direct_kinds(const Staged &st, Model model, int sample_k, int &count) {
    std::vector<int8_t> kind(st.P, 0);
    count = 0;
    for (int p = 0; p < st.P; ++p) {
        const int64_t np = st.off[p + 1] - st.off[p];
        int8_t k = 0;
        if (model == Model::PnP)
            k = np == 4 ? 4 : (np == 5 && sample_k == 5) ? 5 : 0;
        else if (model == Model::Hom)
            k = np == 4 ? 4 : 0;
        kind[p] = k;
        count += k != 0;
    }
    return kind;
}

// the direct problems' minimal solves (one record per problem and kind, sample = 0 .. k-1 with
// status 1, every other problem status -1 so the kernels skip it), then k_direct_finish: their
// records -> c->bestmodels / the pinned c->h_bestmodels and their mask rows (dmask, device) set
// to 1 (model) or 0.  The caller synchronises, then reads the outcome with direct_apply.
int direct_solve(rsac_ctx *c, Model model, const Staged &st, const void *args, const std::vector<int8_t> &kind,
                 uint8_t *dmask, hipStream_t s) {
    const int P = st.P;
    // device layout: rec4, rec5 (P x kModelStride f64 each) | sub4 (P x 4), sub5 (P x 5) i32 |
    // sst4, sst5, st4, st5, kind (P i8 each)
    const size_t recb = sizeof(double) * kModelStride * P, subb = sizeof(int32_t) * 9 * P;
    const size_t bytes = 2 * recb + subb + 5 * (size_t)P;
    HIPCHK(c->direct.ensure(bytes));
    HIPCHK(c->h_direct.ensure(subb + 5 * (size_t)P));
    char *d = c->direct.as<char>();
    double *rec4 = (double *)d, *rec5 = rec4 + (size_t)kModelStride * P;
    int32_t *dsub4 = (int32_t *)(d + 2 * recb), *dsub5 = dsub4 + 4 * (size_t)P;
    int8_t *dsst4 = (int8_t *)(d + 2 * recb + subb), *dsst5 = dsst4 + P, *dst4 = dsst5 + P, *dst5 = dst4 + P,
           *dkind = dst5 + P;
    char *h = c->h_direct.as<char>();
    int32_t *hsub4 = (int32_t *)h, *hsub5 = hsub4 + 4 * (size_t)P;
    int8_t *hsst4 = (int8_t *)(h + subb), *hsst5 = hsst4 + P, *hkind = hsst5 + 3 * (size_t)P;
    bool any5 = false;
    for (int p = 0; p < P; ++p) {
        for (int j = 0; j < 4; ++j) hsub4[4 * p + j] = j;
        for (int j = 0; j < 5; ++j) hsub5[5 * p + j] = j;
        hsst4[p] = kind[p] == 4 ? 1 : -1;
        hsst5[p] = kind[p] == 5 ? 1 : -1;
        hkind[p] = kind[p];
        any5 = any5 || kind[p] == 5;
    }
    HIPCHK(hipMemcpyAsync(dsub4, h, subb + 2 * (size_t)P, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dkind, hkind, P, hipMemcpyHostToDevice, s));
    if (model == Model::PnP) {
        for (int k = 4; k <= 5; ++k) {
            if (k == 5 && !any5) break;
            PnpArgs ad = *(const PnpArgs *)args;
            ad.models = k == 4 ? rec4 : rec5;
            ad.status = k == 4 ? dst4 : dst5;
            ad.hyp_stride = 1;
            ad.subsets = k == 4 ? dsub4 : dsub5;
            ad.sub_status = k == 4 ? dsst4 : dsst5;
            ad.sample_k = k;
            ad.counts_out = nullptr;
            ad.fmodels = nullptr;
            ad.queue = nullptr;
            ad.best_key = nullptr;
            int r = ensure_epnp5(c, ad, P, 1);
            if (r) return r;
            HIPCHK(launch_pnp_solve(ad, P, 0, 1, s));
        }
    } else {
        HomArgs ad = *(const HomArgs *)args;
        ad.models = rec4;
        ad.status = dst4;
        ad.hyp_stride = 1;
        ad.subsets = dsub4;
        ad.sub_status = dsst4;
        HIPCHK(launch_hom_solve(ad, P, 0, 1, s));
    }
    HIPCHK(c->bestmodels.ensure(sizeof(double) * kModelStride * P));
    HIPCHK(c->h_bestmodels.ensure(sizeof(double) * kModelStride * P));
    HIPCHK(launch_direct_finish(rec4, rec5, dst4, dst5, dkind, c->d_off, P, c->bestmodels.as<double>(),
                                c->h_bestmodels.as<double>(), dmask, s));
    return RSAC_OK;
}

// after the synchronisation that follows direct_solve: the direct problems' scan states (best 0 or
// -1, every point or none an inlier, no iterations) and their rows of a host mask
void direct_apply(rsac_ctx *c, const Staged &st, const std::vector<int8_t> &kind, std::vector<ScanState> &scan,
                  uint8_t *host_mask) {
    const double *bm = c->h_bestmodels.as<double>();
    for (int p = 0; p < st.P; ++p) {
        if (!kind[p]) continue;
        const int np = (int)(st.off[p + 1] - st.off[p]);
        const bool ok = bm[(size_t)kModelStride * p + kValidSlot] != 0.0;
        ScanState &sc = scan[p];
        sc.best = ok ? 0 : -1;
        sc.max_good = ok ? np : 0;
        sc.iter = 0;
        sc.done = true;
        if (host_mask) memset(host_mask + st.off[p], ok ? 1 : 0, np);
    }
}

int pnp_core(rsac_ctx *c, const void *pts3d, const void *pts2d, const int64_t *offsets, int32_t P, int32_t n,
             const double *K, int32_t n_iters, double thr, double conf, uint64_t seed, uint32_t flags, double *R_out,
             double *t_out, int32_t *status_out, int32_t *ninl_out, uint8_t *mask_out, rsac_stats *stats,
             hipStream_t s, rsac_scan_state *first_round = nullptr, double *rows_dev = nullptr) {
    // RSAC_DBG_PHASES=1: the host-side phases of every call on stderr (microseconds; a diagnostic)
    static const bool dbg_phases = [] {
        const char *e = getenv("RSAC_DBG_PHASES");
        return e && e[0] == '1';
    }();
    using dbg_clock = std::chrono::steady_clock;
    dbg_clock::time_point tp[6];
    auto mark = [&](int i) {
        if (dbg_phases) tp[i] = dbg_clock::now();
    };
    mark(0);
    int r = check_device(c);
    if (r) return r;
    if (P <= 0 || !K) return fail(RSAC_EINVAL, "bad problem count or K");
    // (first-round mode continues in the caller with model_points 4: P3P only)
    if (first_round &&
        (P != 1 || !(flags & RSAC_F_ADAPTIVE) || (flags & (RSAC_F_SAMPLER_OPENCV | RSAC_F_MINIMAL_EPNP5))))
        return fail(RSAC_EINVAL, "first-round mode: one problem, adaptive, Philox sampler, P3P");
    Staged st;
    r = stage_points(c, pts3d, pts2d, 3, offsets, P, n, flags, s, st, true);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    const int64_t stride = std::max(n_iters, 1);
    r = ensure_hyp_buffers(c, P, stride, (flags & RSAC_F_SAMPLER_OPENCV) != 0);
    if (r) return r;
    PnpArgs a;
    // one P3P problem: the set-up runs inside the first solve launch (k_pnp_setup_solve4)
    r = pnp_args(c, st, flags, seed, stride, 0, s, a, nullptr, true);
    if (r) return r;
    int n_direct = 0;  // problems of OpenCV's count == model_points branch (direct_kinds)
    const std::vector<int8_t> dkind = direct_kinds(st, Model::PnP, a.sample_k, n_direct);
    const bool all_direct = n_direct == P;
    if (all_direct || n_direct > 0) {  // the direct branch solves without run_loop
        r = flush_setup(c, a, s);
        if (r) return r;
    }
    // one adaptive problem: the device replays the first round's scan itself and the final mask
    // and refit are enqueued behind it, so the call synchronises once; the host verifies the
    // device's pick afterwards and redoes the call without speculation on a mismatch (a libm
    // ulp in RANSACUpdateNumIters) or when the first round did not end the scan
    // fixed budget (adaptive off, any number of problems): the one round covers every problem's
    // budget and the device replays every problem's scan, so the finish is enqueued behind the
    // scan the same way, with no host round trip in between
    const bool adaptive = (flags & RSAC_F_ADAPTIVE) != 0;
    const bool spec_fixed = !adaptive && !(flags & RSAC_F_LO) && st.total > 0;
    // (OpenCV's sampler too: its MWC state after the first round is kept in lo.rngs for the resume)
    const bool spec = spec_fixed || (P == 1 && adaptive && !(flags & RSAC_F_LO) && st.total > 0);
    ScanDecide dec;
    if (spec) {
        dec.best_out = c->best.as<int64_t>();
        dec.n = (int32_t)st.total;
        dec.max_iters = std::max(n_iters, 1);
        dec.confidence = conf;
        dec.fixed = spec_fixed ? 1 : 0;
        dec.offsets = spec_fixed ? c->d_off : nullptr;
    }
    LoopOut lo;
    lo.timing = stats != nullptr || c->timing;
    mark(1);
    // first-round mode (rsac_pnp_ransac_first_round): the loop stops after its first round when
    // that round did not end the scan; the caller continues from the exported scan state
    auto fill_stats = [&](rsac_stats &o) {
        o = rsac_stats{};
        o.best_hyp = lo.scan[0].best;
        o.iters = lo.scan[0].iter;
        o.hyps_scored = lo.scored;
        o.n_inliers = lo.scan[0].max_good;
        o.rounds = lo.rounds;
        o.gpu_ms = lo.gpu_ms;
        o.solve_ms = lo.solve_ms;
        o.score_ms = lo.score_ms;
        o.lo_improvements = lo.lo_improvements;
    };
    auto more = [&]() -> int {
        const ScanState &sc = lo.scan[0];
        *first_round = rsac_scan_state{sc.niters, sc.best, sc.iter, sc.max_good, sc.done ? 1 : 0};
        if (sc.best >= 0 && (R_out || t_out)) {  // the best record so far (LO: the optimised model)
            double m[kModelStride];
            HIPCHK(hipMemcpyAsync(m, c->models.as<double>() + (size_t)kModelStride * sc.best,
                                  sizeof(double) * kModelStride, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (R_out) memcpy(R_out, m, 9 * sizeof(double));
            if (t_out) memcpy(t_out, m + 9, 3 * sizeof(double));
        }
        if (ninl_out) ninl_out[0] = sc.max_good;
        if (stats) fill_stats(*stats);  // the first round's figures (timing fields included)
        if (c->timing) fill_stats(c->last_stats);
        return RSAC_MORE;
    };
    if (all_direct) {  // no RANSAC at all: direct_solve below is the whole call
        lo.scan.assign(P, ScanState());
        for (auto &sc : lo.scan) sc.reset(std::max(n_iters, 1));
    } else {
    r = run_loop(c, Model::PnP, st, &a, n_iters, conf, flags, s, lo, spec ? &dec : nullptr, false,
                 first_round ? 1 : 0);
    if (r == RSAC_OK) r = flush_setup(c, a, s);  // (a loop that launched no solve)
    c->pending_on = false;
    if (r) return r;
    if (first_round && !spec && !lo.scan[0].done) return more();
    mark(2);
    const bool refit = (flags & (RSAC_F_REFINE | RSAC_F_EPNP)) != 0;
    r = pnp_finish(c, st, a, lo, stride, K, mask_out, flags, s, refit, lo.spec_pending);
    if (r) return r;
    mark(3);
    if (lo.spec_pending) {
        bool ok = false;
        r = spec_resolve(c, st, lo, a.sample_k, conf, ok, spec_fixed, stride, s);
        if (r) return r;
        c->spec_finishes++;
        if (!ok) {
            c->spec_redos++;
            // the host's replay rules: later rounds if the scan goes on, then the finish again
            if (first_round && !lo.scan[0].done) {
                if (lo.spec_H == 0) {  // the replay started over: the first round without speculation
                    r = run_loop(c, Model::PnP, st, &a, n_iters, conf, flags, s, lo, nullptr, false, 1);
                    if (r) return r;
                }
                if (!lo.scan[0].done) return more();
            }
            if (!spec_fixed && !lo.scan[0].done) {
                // resume after the verified first round; a replay that started over (spec_H = 0)
                // runs afresh, so OpenCV's MWC states restart with the scan
                r = run_loop(c, Model::PnP, st, &a, n_iters, conf, flags, s, lo, nullptr, lo.spec_H > 0);
                if (r) return r;
            }
            r = pnp_finish(c, st, a, lo, stride, K, mask_out, flags, s, refit, false);
            if (r) return r;
        }
    }
    }  // !all_direct
    if (n_direct) {  // OpenCV's count == model_points problems: their minimal model, every point an inlier
        const bool dev_mask = (flags & RSAC_F_DEVICE_OUT) && mask_out;
        if (!dev_mask) HIPCHK(c->mask.ensure(std::max<int64_t>(st.total, 1)));
        r = direct_solve(c, Model::PnP, st, &a, dkind, dev_mask ? mask_out : c->mask.as<uint8_t>(), s);
        if (r) return r;
        HIPCHK(hipStreamSynchronize(s));
        direct_apply(c, st, dkind, lo.scan, dev_mask ? nullptr : mask_out);
    }

    mark(4);
    const double *bm = c->h_bestmodels.as<double>();
    for (int p = 0; p < P; ++p) {
        const bool ok = lo.scan[p].best >= 0;
        if (R_out) memcpy(R_out + 9 * p, bm + kModelStride * p, 9 * sizeof(double));
        if (t_out) memcpy(t_out + 3 * p, bm + kModelStride * p + 9, 3 * sizeof(double));
        if (status_out) status_out[p] = ok ? RSAC_OK : RSAC_NO_MODEL;
        if (ninl_out) ninl_out[p] = lo.scan[p].max_good;
    }
    int any = 0;
    for (int p = 0; p < P; ++p) any |= lo.scan[p].best >= 0;
    if (rows_dev) {  // the result rows on the device (rsac_pnp_ransac_batched_rows)
        HIPCHK(c->h_rowinfo.ensure(sizeof(int64_t) * 2 * P));
        int64_t *info = c->h_rowinfo.as<int64_t>();
        for (int p = 0; p < P; ++p) {
            info[2 * p] = lo.scan[p].best;
            info[2 * p + 1] = lo.scan[p].max_good;
        }
        HIPCHK(launch_pnp_rows(info, c->bestmodels.as<double>(), P, rows_dev, s));
        HIPCHK(hipStreamSynchronize(s));  // h_rowinfo is reused by the next call
    }
    if (first_round) {  // the call ran to the end: the caller has rsac_pnp_ransac's result
        const ScanState &sc = lo.scan[0];
        *first_round = rsac_scan_state{sc.niters, sc.best, sc.iter, sc.max_good, 1};
    }
    if (c->timing) fill_stats(c->last_stats);
    if (stats) fill_stats(*stats);
    mark(5);
    if (dbg_phases) {
        auto us = [&](int i, int j) { return std::chrono::duration<double, std::micro>(tp[j] - tp[i]).count(); };
        fprintf(stderr, "rsac phases (us): setup %.1f loop %.1f finish %.1f resolve %.1f out %.1f total %.1f\n",
                us(0, 1), us(1, 2), us(2, 3), us(3, 4), us(4, 5), us(0, 5));
    }
    return any ? RSAC_OK : RSAC_NO_MODEL;
}

int hom_core(rsac_ctx *c, const void *src, const void *dst, const int64_t *offsets, int32_t P, int32_t n,
             int32_t max_iters, double thr, double conf, uint64_t seed, uint32_t flags, double *H_out,
             int32_t *status_out, int32_t *ninl_out, uint8_t *mask_out, rsac_stats *stats, hipStream_t s) {
    int r = check_device(c);
    if (r) return r;
    if (P <= 0) return fail(RSAC_EINVAL, "bad problem count");
    if (thr <= 0) thr = 3.0;  // defaultRANSACReprojThreshold of findHomography
    Staged st;
    r = stage_points(c, src, dst, 2, offsets, P, n, flags, s, st);
    if (r) return r;
    r = stage_tables(c, st, nullptr, thr, s);
    if (r) return r;
    if ((flags & RSAC_F_SAMPLER_OPENCV) || (flags & RSAC_F_REFINE)) {
        r = ensure_host_points(st, 4, s);
        if (r) return r;
    }
    HomArgs a{};
    a.SX = st.d[0]; a.SY = st.d[1]; a.DX = st.d[2]; a.DY = st.d[3];
    a.offsets = c->d_off;
    a.max_n = st.max_n();
    a.thr2 = c->d_thr2;
    a.seed = seed;
    a.rng_base = 0;
    LoopOut lo;
    int n_direct = 0;  // 4-point problems: findHomography's method-0 path (direct_kinds)
    const std::vector<int8_t> dkind = direct_kinds(st, Model::Hom, 4, n_direct);
    const int64_t stride = std::max(max_iters, 1);
    if (n_direct == P) {
        r = ensure_hyp_buffers(c, P, 1, false);
        if (r) return r;
        lo.scan.assign(P, ScanState());
        for (auto &sc : lo.scan) sc.reset((int)stride);
    } else {
        r = run_loop(c, Model::Hom, st, &a, max_iters, conf, flags, s, lo);
        if (r) return r;
        r = finish_masks(c, Model::Hom, st, &a, lo, stride, mask_out, flags, s);
        if (r) return r;
    }
    if (n_direct) {  // runKernel on the 4 points, mask all ones, no LM; rows of c->mask too (the
                     // location search scores every problem from it)
        const bool dev_mask = (flags & RSAC_F_DEVICE_OUT) && mask_out;
        if (!dev_mask) HIPCHK(c->mask.ensure(std::max<int64_t>(st.total, 1)));
        r = direct_solve(c, Model::Hom, st, &a, dkind, dev_mask ? mask_out : c->mask.as<uint8_t>(), s);
        if (r) return r;
        HIPCHK(hipStreamSynchronize(s));
        direct_apply(c, st, dkind, lo.scan, dev_mask ? nullptr : mask_out);
    }
    const double *bm = c->h_bestmodels.as<double>();
    std::vector<uint8_t> tmpmask;
    const uint8_t *hm = nullptr;
    if (flags & RSAC_F_REFINE) {
        r = host_mask(c, st, mask_out, flags, s, tmpmask, &hm);
        if (r) return r;
    }
    parallel_for(P, [&](int p) {
        const ScanState &sc = lo.scan[p];
        double Hm[9];
        memcpy(Hm, bm + kModelStride * p, sizeof Hm);
        const bool ok = sc.best >= 0;
        const int64_t o = st.off[p];
        const int np = (int)(st.off[p + 1] - o);
        if (ok && (flags & RSAC_F_REFINE) && np > 4) {
            double Hr[9];
            if (hom_refine(st.h[0] + o, st.h[1] + o, st.h[2] + o, st.h[3] + o, hm + o, np, Hr)) memcpy(Hm, Hr, sizeof Hm);
        }
        if (H_out) memcpy(H_out + 9 * p, Hm, sizeof Hm);
        if (status_out) status_out[p] = ok ? RSAC_OK : RSAC_NO_MODEL;
        if (ninl_out) ninl_out[p] = sc.max_good;
    });
    int any = 0;
    for (int p = 0; p < P; ++p) any |= lo.scan[p].best >= 0;
    if (stats) {
        stats->best_hyp = lo.scan[0].best;
        stats->iters = lo.scan[0].iter;
        stats->hyps_scored = lo.scored;
        stats->n_inliers = lo.scan[0].max_good;
        stats->rounds = lo.rounds;
        stats->gpu_ms = lo.gpu_ms;
        stats->solve_ms = lo.solve_ms;
        stats->score_ms = lo.score_ms;
        stats->lo_improvements = 0;
    }
    return any ? RSAC_OK : RSAC_NO_MODEL;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" {

const char *rsac_last_error(void) { return g_err.c_str(); }
int rsac_abi_version(void) { return RSAC_ABI_VERSION; }

int rsac_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rsac_create(int device, rsac_ctx **out) {
    if (!out) return fail(RSAC_EINVAL, "null out");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RSAC_ENODEV, "no HIP device visible");
    if (device < 0 || device >= n) return fail(RSAC_EINVAL, "device %d out of range (%d devices)", device, n);
    HIPCHK(hipSetDevice(device));
    rsac_ctx *c = new rsac_ctx();
    c->device = device;
    // blocking stream: ordered with the legacy null stream, which is torch's default stream
    // (handle 0, indistinguishable from stream = NULL at the C-ABI), so device inputs written by
    // torch before a call, and device outputs read by torch after it, need no extra sync
    if (hipStreamCreateWithFlags(&c->stream, hipStreamDefault) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev2) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_pts, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_small, hipEventDisableTiming) != hipSuccess) {
        rsac_destroy(c);
        return fail(RSAC_EHIP, "stream/event creation failed");
    }
    *out = c;
    return RSAC_OK;
}

void rsac_destroy(rsac_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    DevBuf *dev[] = {&c->pts,  &c->tables,     &c->models,  &c->status,  &c->counts,    &c->subsets,
                     &c->substatus, &c->best, &c->bestmodels, &c->mask, &c->bounds_ws,
                     &c->frame, &c->fconst,   &c->fmodels, &c->queue, &c->loc, &c->lo, &c->win, &c->geo,
                     &c->epnp, &c->epnp5, &c->direct, &c->lmscr, &c->setup_scr, &c->scanrec, &c->mxpts, &c->reproj};
    for (DevBuf *b : dev) b->release();
    PinBuf *pin[] = {&c->h_lmfail, &c->h_pts, &c->h_small, &c->h_counts, &c->h_status, &c->h_subsets,
                     &c->h_substatus, &c->h_best, &c->h_bestmodels, &c->h_mask, &c->h_scanrec, &c->h_lo,
                     &c->h_epnp, &c->h_rowinfo, &c->h_direct};
    for (PinBuf *b : pin) b->release();
    c->lo_state_base = nullptr;
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->ev2) (void)hipEventDestroy(c->ev2);
    if (c->ev_pts) (void)hipEventDestroy(c->ev_pts);
    if (c->ev_small) (void)hipEventDestroy(c->ev_small);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int rsac_debug_set(rsac_ctx *c, int32_t key, int64_t value) {
    if (!c) return fail(RSAC_EINVAL, "null context");
    switch (key) {
    case RSAC_DBG_REFIT_MAX_BLOCKS:
        if (value < 0) return fail(RSAC_EINVAL, "bad block cap");
        c->dbg_refit_max_blocks = (int)std::min<int64_t>(value, kLmMaxBlocks);
        c->lm.max_blocks = pnp_refine_coresident(c->device);
        if (c->dbg_refit_max_blocks > 0) c->lm.max_blocks = std::min(c->lm.max_blocks, c->dbg_refit_max_blocks);
        return RSAC_OK;
    case RSAC_DBG_REFIT_DROP_BLOCK:
        c->lm.drop_block = value != 0;
        return RSAC_OK;
    case RSAC_DBG_MF_CELL_PTS:
        if (value < 0 || value > (1 << 30)) return fail(RSAC_EINVAL, "bad cell size");
        c->dbg_cell_pts = (int32_t)value;
        return RSAC_OK;
    case RSAC_DBG_SPEC_OVERFLOW:
        c->dbg_spec_overflow = value != 0;
        return RSAC_OK;
    case RSAC_DBG_F64_SELFTEST: {
        if (value < 0 || value > (int64_t)1 << 30) return fail(RSAC_EINVAL, "bad self-test size");
        int r = check_device(c);
        if (r) return r;
        int *d = nullptr;
        HIPCHK(hipMalloc(&d, sizeof(int)));
        hipError_t e = hipMemsetAsync(d, 0, sizeof(int), c->stream);
        if (e == hipSuccess) e = launch_f64_selftest(value, d, c->stream);
        int h = -1;
        if (e == hipSuccess) e = hipMemcpyAsync(&h, d, sizeof(int), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(d);
        HIPCHK(e);
        c->dbg_f64_selftest = h;
        return RSAC_OK;
    }
    default:
        return fail(RSAC_EINVAL, "unknown debug key %d", key);
    }
}

int rsac_debug_get(rsac_ctx *c, int32_t key, int64_t *value) {
    if (!c || !value) return fail(RSAC_EINVAL, "null argument");
    switch (key) {
    case RSAC_DBG_SPEC_FINISHES:
        *value = c->spec_finishes;
        return RSAC_OK;
    case RSAC_DBG_SPEC_REDOS:
        *value = c->spec_redos;
        return RSAC_OK;
    case RSAC_DBG_F64_SELFTEST:
        *value = c->dbg_f64_selftest;
        return RSAC_OK;
    default:
        return fail(RSAC_EINVAL, "unknown debug key %d", key);
    }
}

int rsac_refit_blocks(rsac_ctx *c, int32_t n, int32_t *ranges, int32_t *blocks) {
    if (!c || n < 0) return fail(RSAC_EINVAL, "bad arguments");
    int r = check_device(c);
    if (r) return r;
    LmScratch *lm = lm_scratch(c, c->stream);
    if (!lm) return fail(RSAC_ENOMEM, "refit scratch");
    const int nb = lm_blocks(n);
    if (ranges) *ranges = nb;
    if (blocks) *blocks = nb > 1 ? std::min(nb, lm->max_blocks) : 1;
    return RSAC_OK;
}

int rsac_set_timing(rsac_ctx *c, int32_t on) {
    if (!c) return fail(RSAC_EINVAL, "null context");
    c->timing = on != 0;
    return RSAC_OK;
}

int rsac_last_stats(rsac_ctx *c, rsac_stats *out) {
    if (!c || !out) return fail(RSAC_EINVAL, "bad arguments");
    *out = c->last_stats;
    return RSAC_OK;
}

int rsac_set_round_size(rsac_ctx *c, int64_t hyps) {
    if (!c || hyps <= 0) return fail(RSAC_EINVAL, "bad round size");
    c->round_size = hyps;
    return RSAC_OK;
}

int rsac_pnp_ransac(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9], int32_t n_iters,
                    double thr, double conf, uint64_t seed, uint32_t flags, double R_out[9], double t_out[3],
                    uint8_t *mask_out, rsac_stats *stats, void *stream) {
    if (n < 4) return fail(RSAC_ETOOFEW, "solvePnPRansac needs >= 4 correspondences (got %d)", n);
    int32_t status = 0, ninl = 0;
    return with_one_refit_block(c, [&] {
        return pnp_core(c, pts3d, pts2d, nullptr, 1, n, K, n_iters, thr, conf, seed, flags, R_out, t_out, &status,
                        &ninl, mask_out, stats, pick_stream(c, stream));
    });
}

int rsac_pnp_ransac_first_round(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                                int32_t n_iters, double thr, double conf, uint64_t seed, uint32_t flags,
                                double R_out[9], double t_out[3], uint8_t *mask_out, rsac_scan_state *st_out,
                                rsac_stats *stats, void *stream) {
    if (n < 4) return fail(RSAC_ETOOFEW, "solvePnPRansac needs >= 4 correspondences (got %d)", n);
    if (!st_out) return fail(RSAC_EINVAL, "st_out required");
    int32_t status = 0, ninl = 0;
    return with_one_refit_block(c, [&] {
        return pnp_core(c, pts3d, pts2d, nullptr, 1, n, K, n_iters, thr, conf, seed, flags, R_out, t_out, &status,
                        &ninl, mask_out, stats, pick_stream(c, stream), st_out);
    });
}

int rsac_pnp_ransac_batched_rows(rsac_ctx *c, const void *pts3d, const void *pts2d, const int64_t *offsets, int32_t P,
                                 const double *K, int32_t n_iters, double thr, double conf, uint64_t seed,
                                 uint32_t flags, double *rows_out, uint8_t *mask_out, void *stream) {
    if (!offsets || !rows_out) return fail(RSAC_EINVAL, "offsets and rows_out required");
    return with_one_refit_block(c, [&] {
        return pnp_core(c, pts3d, pts2d, offsets, P, 0, K, n_iters, thr, conf, seed, flags, nullptr, nullptr,
                        nullptr, nullptr, mask_out, nullptr, pick_stream(c, stream), nullptr, rows_out);
    });
}

int rsac_pnp_ransac_batched(rsac_ctx *c, const void *pts3d, const void *pts2d, const int64_t *offsets, int32_t P,
                            const double *K, int32_t n_iters, double thr, double conf, uint64_t seed, uint32_t flags,
                            double *R_out, double *t_out, int32_t *status_out, int32_t *ninl_out, uint8_t *mask_out,
                            void *stream) {
    if (!offsets) return fail(RSAC_EINVAL, "offsets required");
    return with_one_refit_block(c, [&] {
        return pnp_core(c, pts3d, pts2d, offsets, P, 0, K, n_iters, thr, conf, seed, flags, R_out, t_out, status_out,
                        ninl_out, mask_out, nullptr, pick_stream(c, stream));
    });
}

int rsac_homography_ransac(rsac_ctx *c, const void *src, const void *dst, int32_t n, int32_t max_iters, double thr,
                           double conf, uint64_t seed, uint32_t flags, double H_out[9], uint8_t *mask_out,
                           rsac_stats *stats, void *stream) {
    if (n < 4) return fail(RSAC_ETOOFEW, "findHomography needs >= 4 correspondences (got %d)", n);
    int32_t status = 0, ninl = 0;
    return hom_core(c, src, dst, nullptr, 1, n, max_iters, thr, conf, seed, flags, H_out, &status, &ninl, mask_out,
                    stats, pick_stream(c, stream));
}

int rsac_homography_ransac_batched(rsac_ctx *c, const void *src, const void *dst, const int64_t *offsets, int32_t P,
                                   int32_t max_iters, double thr, double conf, uint64_t seed, uint32_t flags,
                                   double *H_out, int32_t *status_out, int32_t *ninl_out, uint8_t *mask_out,
                                   void *stream) {
    if (!offsets) return fail(RSAC_EINVAL, "offsets required");
    return hom_core(c, src, dst, offsets, P, 0, max_iters, thr, conf, seed, flags, H_out, status_out, ninl_out,
                    mask_out, nullptr, pick_stream(c, stream));
}

int rsac_location_search(rsac_ctx *c, const double *pos3d, const double *pixels, int32_t n, const double *locations,
                         int32_t L, double thr, int32_t max_iters, double conf, uint32_t flags, double *H_out,
                         double *err_out, int32_t *status_out, int32_t *ninl_out, uint8_t *mask_out,
                         int32_t *n_good_out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!pos3d || !pixels || !locations || !err_out || n <= 0 || L <= 0)
        return fail(RSAC_EINVAL, "rsac_location_search: bad arguments");
    if (flags & (RSAC_F_DEVICE_IN | RSAC_F_DEVICE_SOA | RSAC_F_DEVICE_OUT))
        return fail(RSAC_EINVAL, "rsac_location_search takes host arrays");
    hipStream_t s = pick_stream(c, stream);
    // features noted on the image: pixel != (0, 0) (main_v1.py:304)
    std::vector<double> in;
    in.reserve((size_t)5 * n + 3 * L);
    int32_t ng = 0;
    for (int32_t i = 0; i < n; ++i)
        if (pixels[2 * i] != 0.0 || pixels[2 * i + 1] != 0.0) {
            in.insert(in.end(), pos3d + 3 * i, pos3d + 3 * i + 3);
            ++ng;
        }
    for (int32_t i = 0; i < n; ++i)
        if (pixels[2 * i] != 0.0 || pixels[2 * i + 1] != 0.0) in.insert(in.end(), pixels + 2 * i, pixels + 2 * i + 2);
    in.insert(in.end(), locations, locations + 3 * (size_t)L);
    if (n_good_out) *n_good_out = ng;
    if (ng < 4) return fail(RSAC_ETOOFEW, "findHomography needs >= 4 noted features (got %d)", ng);
    const size_t pairs = (size_t)L * ng;
    // device layout (f64): p3 [3 ng] px [2 ng] locs [3 L] src [2 L ng] dst [2 L ng] H [9 L] err [2 L], ok [L] i32
    const size_t nd = in.size() + 4 * pairs + 11 * (size_t)L;
    HIPCHK(c->loc.ensure(nd * sizeof(double) + sizeof(int32_t) * L));
    double *d_p3 = c->loc.as<double>(), *d_px = d_p3 + 3 * ng, *d_locs = d_px + 2 * ng, *d_src = d_locs + 3 * L;
    double *d_dst = d_src + 2 * pairs, *d_H = d_dst + 2 * pairs, *d_err = d_H + 9 * (size_t)L;
    int32_t *d_ok = (int32_t *)(d_err + 2 * (size_t)L);
    HIPCHK(hipMemcpyAsync(d_p3, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(launch_loc_pos2(d_p3, d_px, ng, d_locs, L, d_src, d_dst, s));
    std::vector<int64_t> off((size_t)L + 1);
    for (int32_t l = 0; l <= L; ++l) off[l] = (int64_t)l * ng;
    std::vector<double> H((size_t)9 * L);
    std::vector<int32_t> st(L), ninl(L);
    std::vector<uint8_t> m(pairs);
    r = hom_core(c, d_src, d_dst, off.data(), L, 0, max_iters, thr, conf, 0, flags | RSAC_F_DEVICE_IN, H.data(),
                 st.data(), ninl.data(), m.data(), nullptr, s);
    if (r < 0) return r;
    // hom_core left the RANSAC-phase masks of every location in c->mask
    std::vector<int32_t> ok(L);
    for (int32_t l = 0; l < L; ++l) ok[l] = st[l] == RSAC_OK;
    HIPCHK(hipMemcpyAsync(d_H, H.data(), H.size() * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_ok, ok.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, s));
    HIPCHK(launch_loc_score(d_src, d_dst, c->mask.as<uint8_t>(), d_H, d_ok, L, ng, thr <= 0 ? 3.0 : thr, d_err, s));
    HIPCHK(hipMemcpyAsync(err_out, d_err, sizeof(double) * 2 * L, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (H_out) memcpy(H_out, H.data(), H.size() * sizeof(double));
    if (status_out) memcpy(status_out, st.data(), sizeof(int32_t) * L);
    if (ninl_out) memcpy(ninl_out, ninl.data(), sizeof(int32_t) * L);
    if (mask_out) memcpy(mask_out, m.data(), pairs);
    return r;
}

int rsac_utm_convert(rsac_ctx *c, int inverse, const double *in, int64_t n, int32_t zone, int32_t south,
                     uint32_t flags, double *out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!in || !out || n < 0 || zone < 1 || zone > 60) return fail(RSAC_EINVAL, "bad arguments");
    if (n == 0) return RSAC_OK;
    hipStream_t s = pick_stream(c, stream);
    const bool dev = (flags & RSAC_F_DEVICE_IN) != 0;
    const double *din = in;
    double *dout = out;
    if (!dev) {
        HIPCHK(c->geo.ensure(sizeof(double) * 4 * (size_t)n));
        double *b = c->geo.as<double>();
        HIPCHK(hipMemcpyAsync(b, in, sizeof(double) * 2 * n, hipMemcpyHostToDevice, s));
        din = b;
        dout = b + 2 * n;
    }
    HIPCHK(launch_utm(inverse != 0, din, n, zone, south != 0, dout, s));
    if (!dev) {
        HIPCHK(hipMemcpyAsync(out, dout, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return RSAC_OK;
}

int rsac_dem_ray_intersect(rsac_ctx *c, const double *origins, const double *dirs, int32_t n_rays, const double *dem,
                           int32_t ny, int32_t nx, double y0, double dy, double x0, double dx, int32_t zone,
                           int32_t south, double max_search_dist, double step, int32_t min_steps, uint32_t flags,
                           double *hits_out, int8_t *status_out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!origins || !dirs || !dem || !hits_out || !status_out || n_rays < 0 || ny < 2 || nx < 2 || dy == 0.0 ||
        dx == 0.0 || !(step > 0.0) || zone < 1 || zone > 60)
        return fail(RSAC_EINVAL, "bad arguments");
    if (n_rays == 0) return RSAC_OK;
    // int(max_search_dist / step) of the reference's range()
    const double q = max_search_dist / step;
    const int32_t n_steps = q >= 2147483647.0 ? 2147483647 : (q > 0 ? (int32_t)q : 0);
    hipStream_t s = pick_stream(c, stream);
    const bool dev = (flags & RSAC_F_DEVICE_IN) != 0;
    const size_t cells = (size_t)ny * nx;
    const double *d_o = origins, *d_d = dirs, *d_dem = dem;
    double *d_hits = hits_out;
    int8_t *d_st = status_out;
    if (!dev) {
        HIPCHK(c->geo.ensure(sizeof(double) * (9 * (size_t)n_rays + cells) + (size_t)n_rays + 64));
        double *b = c->geo.as<double>();
        double *bo = b, *bd = b + 3 * (size_t)n_rays, *bh = bd + 3 * (size_t)n_rays, *bz = bh + 3 * (size_t)n_rays;
        int8_t *bs = (int8_t *)(bz + cells);
        HIPCHK(hipMemcpyAsync(bo, origins, sizeof(double) * 3 * n_rays, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(bd, dirs, sizeof(double) * 3 * n_rays, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(bz, dem, sizeof(double) * cells, hipMemcpyHostToDevice, s));
        d_o = bo; d_d = bd; d_dem = bz; d_hits = bh; d_st = bs;
    }
    HIPCHK(launch_dem_march(d_o, d_d, n_rays, d_dem, ny, nx, y0, dy, x0, dx, zone, south != 0, n_steps, step,
                            min_steps, d_hits, d_st, s));
    if (!dev) {
        HIPCHK(hipMemcpyAsync(hits_out, d_hits, sizeof(double) * 3 * n_rays, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(status_out, d_st, n_rays, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    return RSAC_OK;
}

int rsac_pnp_winner(rsac_ctx *c, const double *pts3d, const double *pts2d, int32_t n, const double K[9], double thr,
                    uint64_t seed, const int64_t *key, double *model_out, uint8_t *mask_out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!pts3d || !pts2d || !K || !key || n < 4) return fail(RSAC_EINVAL, "bad arguments");
    hipStream_t s = pick_stream(c, stream);
    HIPCHK(c->win.ensure(sizeof(double) * (kModelStride + 8)));
    double *rec = c->win.as<double>();
    double *cam = rec + kModelStride;
    const double cm[4] = {K[0], K[4], K[2], K[5]};
    HIPCHK(c->h_small.ensure(64));
    HIPCHK(hipEventSynchronize(c->ev_small));
    double *hc = c->h_small.as<double>();
    memcpy(hc, cm, sizeof cm);
    hc[4] = (double)(float)(thr * thr);
    HIPCHK(hipMemcpyAsync(cam, hc, 5 * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(c->ev_small, s));
    HIPCHK(launch_pnp_winner(pts3d, pts2d, n, cam, seed, key, rec, model_out, mask_out, s));
    return RSAC_OK;
}

int rsac_pnp_local_opt(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                       const double model_in[12], double thr, uint32_t flags, double model_out[12], int32_t *count_out,
                       int32_t *steps_out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!K || !model_in || !model_out || n < 1) return fail(RSAC_EINVAL, "bad arguments");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    r = stage_points(c, pts3d, pts2d, 3, nullptr, 1, n, flags & (RSAC_F_DEVICE_IN | RSAC_F_DEVICE_SOA), s, st);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, 1, false);
    if (r) return r;
    PnpArgs a;
    r = pnp_args(c, st, flags | RSAC_F_EXACT_ONLY, 0, 1, 0, s, a);
    if (r) return r;
    double rec[kModelStride] = {0};
    memcpy(rec, model_in, 12 * sizeof(double));
    rec[kValidSlot] = 1.0;
    HIPCHK(hipMemcpyAsync(c->models.p, rec, sizeof rec, hipMemcpyHostToDevice, s));
    // the model's own count starts the chain (local_opt recounts it on the device)
    HIPCHK(c->lo.ensure(2 * sizeof(double) * kModelStride + 64 + 2 * (size_t)n));
    int32_t *cnt = (int32_t *)(c->lo.as<double>() + 2 * kModelStride);
    HIPCHK(hipMemsetAsync(cnt, 0, sizeof(int32_t), s));
    HIPCHK(launch_pnp_model_count(a, n, c->models.as<double>(), (uint8_t *)(cnt + 16), cnt, s));
    int32_t c0 = 0;
    HIPCHK(hipMemcpyAsync(&c0, cnt, sizeof c0, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    ScanState sc;
    int32_t steps = 0;
    r = with_one_refit_block(c, [&] {
        // from the input model each time (a failed chain may have replaced the record)
        HIPCHK(hipMemcpyAsync(c->models.p, rec, sizeof rec, hipMemcpyHostToDevice, s));
        sc.reset(1 << 30);
        sc.best = 0;
        sc.max_good = c0;
        steps = 0;
        return local_opt(c, a, n, sc, 0.99, s, steps);
    });
    if (r) return r;
    HIPCHK(hipMemcpyAsync(rec, c->models.p, sizeof rec, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memcpy(model_out, rec, 12 * sizeof(double));
    if (count_out) *count_out = sc.max_good;
    if (steps_out) *steps_out = steps;
    return RSAC_OK;
}

// LM on (R, t) from the given start over the masked points (NULL = all), on the device: one
// problem's k_pnp_refine, the bits of rsac_pnp_refine (host) and orc_pnp_refine.  Host f64 AoS.
static int refine_on_device(rsac_ctx *c, const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                            const uint8_t *mask, double R[9], double t[3], hipStream_t s) {
    Staged st;
    int r = stage_points(c, pts3d, pts2d, 3, nullptr, 1, n, 0, s, st);
    if (r) return r;
    r = stage_tables(c, st, K, 1.0, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, 1, false);
    if (r) return r;
    PnpArgs a;
    r = pnp_args(c, st, RSAC_F_EXACT_ONLY, 0, 1, 0, s, a);
    if (r) return r;
    HIPCHK(c->h_bestmodels.ensure(sizeof(double) * kModelStride));
    HIPCHK(c->h_mask.ensure(std::max(n, 1)));
    double *hrec = c->h_bestmodels.as<double>();
    memset(hrec, 0, sizeof(double) * kModelStride);
    memcpy(hrec, R, 9 * sizeof(double));
    memcpy(hrec + 9, t, 3 * sizeof(double));
    hrec[kValidSlot] = 1.0;
    uint8_t *hm = c->h_mask.as<uint8_t>();
    if (mask)
        memcpy(hm, mask, n);
    else
        memset(hm, 1, n);
    HIPCHK(c->mask.ensure(std::max(n, 1)));
    HIPCHK(hipMemcpyAsync(c->bestmodels.p, hrec, sizeof(double) * kModelStride, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->mask.p, hm, n, hipMemcpyHostToDevice, s));
    HIPCHK(launch_pnp_refine(a, 1, c->mask.as<uint8_t>(), c->bestmodels.as<double>(), nullptr, s, lm_scratch(c, s),
                             st.off.data(), hrec));  // R, t also written to the pinned record
    HIPCHK(hipStreamSynchronize(s));
    if (int e = lm_check(c)) return e;
    memcpy(R, hrec, 9 * sizeof(double));
    memcpy(t, hrec + 9, 3 * sizeof(double));
    return RSAC_OK;
}

int rsac_pnp_refine_lm(rsac_ctx *c, const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                       const uint8_t *mask, double R[9], double t[3], void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n < 3 || !pts3d || !pts2d || !K || !R || !t) return fail(RSAC_EINVAL, "bad arguments");
    const double R0[9] = {R[0], R[1], R[2], R[3], R[4], R[5], R[6], R[7], R[8]}, t0[3] = {t[0], t[1], t[2]};
    return with_one_refit_block(c, [&] {
        memcpy(R, R0, sizeof R0);
        memcpy(t, t0, sizeof t0);
        return refine_on_device(c, pts3d, pts2d, n, K, mask, R, t, pick_stream(c, stream));
    });
}

int rsac_pnp_reprojection_errors(rsac_ctx *c, const double *pts3d, const double *pts2d, int32_t n, const double K[9],
                                 const double R[9], const double t[3], uint32_t flags, double *proj_out,
                                 double *err_out, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n < 0 || !pts3d || !pts2d || !K || !R || !t) return fail(RSAC_EINVAL, "bad arguments");
    if (n == 0) return RSAC_OK;
    hipStream_t s = pick_stream(c, stream);
    PoseCam pc;
    memcpy(pc.R, R, sizeof pc.R);
    memcpy(pc.t, t, sizeof pc.t);
    pc.cam[0] = K[0]; pc.cam[1] = K[4]; pc.cam[2] = K[2]; pc.cam[3] = K[5];
    if (flags & RSAC_F_DEVICE_IN)  // device inputs and outputs: enqueue only
        return launch_pnp_reproj(pts3d, pts2d, n, pc, proj_out, err_out, s) == hipSuccess
                   ? RSAC_OK
                   : fail(RSAC_EHIP, "reprojection launch failed");
    const size_t N = (size_t)n;
    HIPCHK(c->reproj.ensure(sizeof(double) * 8 * N));
    double *d3 = c->reproj.as<double>(), *d2 = d3 + 3 * N, *dp = d2 + 2 * N, *de = dp + 2 * N;
    HIPCHK(hipMemcpyAsync(d3, pts3d, sizeof(double) * 3 * N, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d2, pts2d, sizeof(double) * 2 * N, hipMemcpyHostToDevice, s));
    HIPCHK(launch_pnp_reproj(d3, d2, n, pc, proj_out ? dp : nullptr, err_out ? de : nullptr, s));
    if (proj_out) HIPCHK(hipMemcpyAsync(proj_out, dp, sizeof(double) * 2 * N, hipMemcpyDeviceToHost, s));
    if (err_out) HIPCHK(hipMemcpyAsync(err_out, de, sizeof(double) * N, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return RSAC_OK;
}

int rsac_pnp_orientation_sweep(rsac_ctx *c, const double *pts3d, const double *pts2d, int32_t n, const double *Ks,
                               int32_t n_k, int32_t n_iters, double thr, double conf, uint64_t seed, uint32_t flags,
                               int32_t min_inliers, int32_t *best_out, double *mean_err_out, double *models_out,
                               int32_t *status_out, int32_t *n_inliers_out, uint8_t *masks_out, double R_out[9],
                               double t_out[3], void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n < 4) return fail(RSAC_ETOOFEW, "solvePnPRansac needs >= 4 correspondences (got %d)", n);
    if (n_k < 1 || !pts3d || !pts2d || !Ks || !best_out) return fail(RSAC_EINVAL, "bad arguments");
    // solvePnPRefineLM on the winner needs >= 3 inliers: a lower gate would fail only after the sweep
    if (min_inliers < 3) return fail(RSAC_EINVAL, "min_inliers must be >= 3 (got %d)", min_inliers);
    if (flags & (RSAC_F_DEVICE_IN | RSAC_F_DEVICE_SOA | RSAC_F_DEVICE_OUT | RSAC_F_LO | RSAC_F_ASYNC))
        return fail(RSAC_EINVAL, "the K sweep takes host arrays (no device, LO or async flags)");
    hipStream_t s = pick_stream(c, stream);
    const size_t N = (size_t)n, P = (size_t)n_k;
    // 1. the loop over the intrinsics (testpro-K.py:58-75) as one batched call: problem k is the
    //    point set with K_k
    std::vector<double> p3(3 * N * P), p2(2 * N * P);
    std::vector<int64_t> off(P + 1);
    for (size_t k = 0; k < P; ++k) {
        memcpy(&p3[3 * N * k], pts3d, sizeof(double) * 3 * N);
        memcpy(&p2[2 * N * k], pts2d, sizeof(double) * 2 * N);
        off[k] = (int64_t)(N * k);
    }
    off[P] = (int64_t)(N * P);
    std::vector<double> R(9 * P), t(3 * P);
    std::vector<int32_t> status(P), ninl(P);
    std::vector<uint8_t> masks(N * P);
    r = rsac_pnp_ransac_batched(c, p3.data(), p2.data(), off.data(), n_k, Ks, n_iters, thr, conf, seed, flags, R.data(),
                                t.data(), status.data(), ninl.data(), masks.data(), stream);
    if (r < 0) return r;
    // 2. the gate (testpro-K.py:77) and each pose as projectPoints sees it: the shim returns
    //    rvec = Rodrigues(R), and projectPoints rotates by Rodrigues(rvec)
    std::vector<double> poses(12 * P, 0.0), cams(4 * P);
    std::vector<uint8_t> pass(P);
    for (size_t k = 0; k < P; ++k) {
        pass[k] = status[k] == RSAC_OK && ninl[k] >= min_inliers;
        double rv[3];
        rodrigues_m2v(&R[9 * k], rv);
        rodrigues_v2m(rv, &poses[12 * k]);
        memcpy(&poses[12 * k + 9], &t[3 * k], 3 * sizeof(double));
        const double *Kk = Ks + 9 * k;
        cams[4 * k] = Kk[0]; cams[4 * k + 1] = Kk[4]; cams[4 * k + 2] = Kk[2]; cams[4 * k + 3] = Kk[5];
    }
    // 3. the mean inlier reprojection error of every K on the device (testpro-K.py:80-82)
    HIPCHK(c->reproj.ensure(sizeof(double) * (5 * N + 16 * P + 2 * P) + N * P));
    double *d3 = c->reproj.as<double>(), *d2 = d3 + 3 * N, *dposes = d2 + 2 * N, *dcams = dposes + 12 * P,
           *dout = dcams + 4 * P;
    uint8_t *dmasks = (uint8_t *)(dout + 2 * P);
    HIPCHK(hipMemcpyAsync(d3, pts3d, sizeof(double) * 3 * N, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d2, pts2d, sizeof(double) * 2 * N, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dposes, poses.data(), sizeof(double) * 12 * P, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dcams, cams.data(), sizeof(double) * 4 * P, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dmasks, masks.data(), N * P, hipMemcpyHostToDevice, s));
    HIPCHK(launch_pnp_reproj_mean(d3, d2, n, n_k, dposes, dcams, dmasks, dout, s));
    std::vector<double> sums(2 * P);
    HIPCHK(hipMemcpyAsync(sums.data(), dout, sizeof(double) * 2 * P, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // 4. the first K with the strictly smallest mean (testpro-K.py:90-97)
    int best = -1;
    double best_err = __builtin_inf();
    for (size_t k = 0; k < P; ++k) {
        const double mean = sums[2 * k] / sums[2 * k + 1];
        if (mean_err_out) mean_err_out[k] = pass[k] ? mean : __builtin_nan("");
        if (pass[k] && mean < best_err) {
            best_err = mean;
            best = (int)k;
        }
    }
    *best_out = best;
    for (size_t k = 0; k < P; ++k) {
        if (models_out) {
            memcpy(models_out + 12 * k, &R[9 * k], 9 * sizeof(double));
            memcpy(models_out + 12 * k + 9, &t[3 * k], 3 * sizeof(double));
        }
        if (status_out) status_out[k] = pass[k] ? RSAC_OK : RSAC_NO_MODEL;
        if (n_inliers_out) n_inliers_out[k] = ninl[k];
    }
    if (masks_out) memcpy(masks_out, masks.data(), N * P);
    if (best < 0) return RSAC_NO_MODEL;
    // 5. solvePnPRefineLM on the winner's inliers from its pose (testpro-K.py:122-125): the
    //    reference passes the inlier subset, in index order, and the rvec of step 2
    std::vector<double> s3, s2;
    for (size_t i = 0; i < N; ++i)
        if (masks[N * best + i]) {
            s3.insert(s3.end(), pts3d + 3 * i, pts3d + 3 * i + 3);
            s2.insert(s2.end(), pts2d + 2 * i, pts2d + 2 * i + 2);
        }
    double Rr[9], tr[3];
    memcpy(Rr, &poses[12 * best], sizeof Rr);
    memcpy(tr, &poses[12 * best + 9], sizeof tr);
    r = rsac_pnp_refine_lm(c, s3.data(), s2.data(), (int32_t)(s3.size() / 3), Ks + 9 * best, nullptr, Rr, tr, stream);
    if (r < 0) return r;
    if (R_out) memcpy(R_out, Rr, sizeof Rr);
    if (t_out) memcpy(t_out, tr, sizeof tr);
    return RSAC_OK;
}

int rsac_score_poses(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                     const double *poses, int32_t n_poses, double thr, uint32_t flags, int32_t *counts_out,
                     void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n_poses <= 0 || !poses || !counts_out || !K) return fail(RSAC_EINVAL, "bad arguments");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    r = stage_points(c, pts3d, pts2d, 3, nullptr, 1, n, flags, s, st);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, n_poses, false);
    if (r) return r;
    std::vector<double> rec((size_t)n_poses * kModelStride, 0.0);
    for (int32_t h = 0; h < n_poses; ++h) {
        memcpy(&rec[(size_t)h * kModelStride], poses + 12 * h, 12 * sizeof(double));
        rec[(size_t)h * kModelStride + kValidSlot] = 1.0;
    }
    HIPCHK(hipMemcpyAsync(c->models.p, rec.data(), rec.size() * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(c->status.p, 1, (size_t)n_poses, s));  // every pose valid (the scorers read status)
    PnpArgs a;
    r = pnp_args(c, st, flags, 0, n_poses, 0, s, a);
    if (r) return r;
    a.counts_out = nullptr;  // no solve kernel zeroes the counts here
    if (a.fmodels) HIPCHK(launch_pnp_fmodels(a, 1, n_poses, s));
    HIPCHK(launch_pnp_score(a, 1, 0, n_poses, c->counts.as<int32_t>(), s));
    HIPCHK(hipStreamSynchronize(s));  // rec (host vector) must outlive the async copy
    HIPCHK(hipMemcpyAsync(counts_out, c->counts.p, sizeof(int32_t) * n_poses, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return RSAC_OK;
}

int rsac_pnp_evaluate_range(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                            int64_t hyp_begin, int64_t n_hyps, double thr, uint64_t seed, uint32_t flags,
                            int64_t *key_out, double model_out[12], uint8_t *mask_out, rsac_stats *stats,
                            void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n < 4) return fail(RSAC_ETOOFEW, "need >= 4 correspondences");
    if (n_hyps <= 0 || n_hyps > INT32_MAX || !K || !key_out) return fail(RSAC_EINVAL, "bad arguments");
    if ((flags & RSAC_F_ASYNC) && mask_out && !(flags & RSAC_F_DEVICE_OUT))
        return fail(RSAC_EINVAL, "RSAC_F_ASYNC needs a device mask (RSAC_F_DEVICE_OUT)");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    // device f64 inputs: the f32 conversion is fused into the frame launch of pnp_args
    r = stage_points(c, pts3d, pts2d, 3, nullptr, 1, n, flags & ~RSAC_F_SAMPLER_OPENCV, s, st, true);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, n_hyps, false);
    if (r) return r;
    // the best key is reduced inside the scoring kernel; only 8 bytes + the
    // winner's record (+ its mask, computed on the device) leave the GPU
    unsigned long long *dkey = (unsigned long long *)c->best.p;
    PnpArgs a;
    r = pnp_args(c, st, flags, seed, n_hyps, hyp_begin, s, a, dkey);
    if (r) return r;
    const int32_t H = (int32_t)n_hyps;
    r = ensure_epnp5(c, a, 1, H);
    if (r) return r;
    const bool async = (flags & RSAC_F_ASYNC) != 0;
    // timing events only for a synchronous call that reports stats: each event record in the
    // stream costs a gap of several microseconds between the kernels around it
    const bool timed = stats != nullptr && !async;
    if (timed) HIPCHK(hipEventRecord(c->ev0, s));
    HIPCHK(launch_pnp_solve(a, 1, 0, H, s));
    if (timed) HIPCHK(hipEventRecord(c->ev1, s));
    if (timed) {  // score_ms = the scoring kernel alone (ev1 -> ev2), then the key's reduction
        PnpArgs ak = a;
        ak.best_key = nullptr;
        HIPCHK(launch_pnp_score(ak, 1, 0, H, c->counts.as<int32_t>(), s));
        HIPCHK(hipEventRecord(c->ev2, s));
        HIPCHK(launch_pnp_best_key(a, 0, H, c->counts.as<int32_t>(), s));
    } else {
        HIPCHK(launch_pnp_score(a, 1, 0, H, c->counts.as<int32_t>(), s));
    }
    uint8_t *hmask_dev = nullptr;
    if (mask_out) {
        if (flags & RSAC_F_DEVICE_OUT) {
            hmask_dev = mask_out;
        } else {
            HIPCHK(c->mask.ensure(std::max(n, 1)));
            hmask_dev = c->mask.as<uint8_t>();
        }
    }
    HIPCHK(launch_pnp_key_finish(a, n, dkey, hmask_dev, c->bestmodels.as<double>(), async ? model_out : nullptr,
                                 async ? key_out : nullptr, s));
    if (async) {
        // results stay on the device and nothing waits: the raw packed key (0 = no model) and
        // the winner's R, t were written to the caller's device buffers in stream order
        if (stats) memset(stats, 0, sizeof(*stats));
        return RSAC_OK;
    }
    HIPCHK(c->h_bestmodels.ensure(sizeof(double) * (kModelStride + 2)));
    double *hb = c->h_bestmodels.as<double>();
    HIPCHK(hipMemcpyAsync(hb, c->bestmodels.p, sizeof(double) * kModelStride, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hb + kModelStride, dkey, sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    if (mask_out && !(flags & RSAC_F_DEVICE_OUT)) {
        HIPCHK(c->h_mask.ensure(std::max(n, 1)));
        HIPCHK(hipMemcpyAsync(c->h_mask.p, hmask_dev, n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (mask_out && !(flags & RSAC_F_DEVICE_OUT)) memcpy(mask_out, c->h_mask.p, n);
    unsigned long long key;
    memcpy(&key, hb + kModelStride, sizeof key);
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        add_times(c, stats->gpu_ms, stats->solve_ms, stats->score_ms);
        stats->hyps_scored = H;
        stats->rounds = 1;
    }
    if (key == 0) {
        *key_out = -1;
        if (stats) stats->best_hyp = -1;
        return RSAC_NO_MODEL;
    }
    *key_out = (int64_t)key;
    if (stats) {
        const uint64_t low = 0xFFFFFFFFull - (key & 0xFFFFFFFFull);
        stats->best_hyp = (int64_t)(((uint64_t)hyp_begin & ~0xFFFFFFFFull) | low);
        stats->n_inliers = (int32_t)(key >> 32);
    }
    if (model_out) memcpy(model_out, hb, 12 * sizeof(double));
    return RSAC_OK;
}

static int hypotheses_core(rsac_ctx *c, Model model, const void *a_pts, const void *b_pts, int32_t n, const double *K,
                           int64_t hyp_begin, int32_t H, double thr, uint64_t seed, uint32_t flags,
                           const int32_t *subsets, int32_t *counts_out, int8_t *status_out, double *models_out,
                           void *stream, int32_t *rows_out = nullptr) {
    int r = check_device(c);
    if (r) return r;
    if (H <= 0 || (!rows_out && (!counts_out || !status_out))) return fail(RSAC_EINVAL, "bad arguments");
    if (model == Model::PnP && !K) return fail(RSAC_EINVAL, "K required");
    if (model == Model::Fm && subsets) return fail(RSAC_EINVAL, "the fundamental-matrix sampler is Philox only");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    r = stage_points(c, a_pts, b_pts, model == Model::PnP ? 3 : 2, nullptr, 1, n, flags, s, st);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, H, subsets != nullptr);
    if (r) return r;
    if (subsets) {
        const int sk = model == Model::PnP && (flags & RSAC_F_MINIMAL_EPNP5) ? 5 : 4;  // indices per subset
        int8_t *hss = c->h_substatus.as<int8_t>();
        memcpy(c->h_subsets.p, subsets, sizeof(int32_t) * sk * (size_t)H);
        for (int32_t h = 0; h < H; ++h) {
            bool ok = true;
            for (int j = 0; j < sk; ++j) ok = ok && subsets[sk * h + j] >= 0 && subsets[sk * h + j] < n;
            hss[h] = ok ? 1 : -1;
        }
        HIPCHK(hipMemcpyAsync(c->subsets.p, c->h_subsets.p, sizeof(int32_t) * sk * (size_t)H, hipMemcpyHostToDevice,
                              s));
        HIPCHK(hipMemcpyAsync(c->substatus.p, hss, H, hipMemcpyHostToDevice, s));
    }
    if (model == Model::PnP) {
        PnpArgs a;
        r = pnp_args(c, st, flags, seed, H, hyp_begin, s, a);
        if (r) return r;
        a.subsets = subsets ? c->subsets.as<int32_t>() : nullptr;
        a.sub_status = subsets ? c->substatus.as<int8_t>() : nullptr;
        r = ensure_epnp5(c, a, 1, H);
        if (r) return r;
        HIPCHK(launch_pnp_solve(a, 1, 0, H, s));
        HIPCHK(launch_pnp_score(a, 1, 0, H, c->counts.as<int32_t>(), s));
    } else {
        HomArgs a{};
        a.SX = st.d[0]; a.SY = st.d[1]; a.DX = st.d[2]; a.DY = st.d[3];
        a.offsets = c->d_off;
        a.max_n = st.max_n();
        a.thr2 = c->d_thr2;
        a.models = c->models.as<double>();
        a.status = c->status.as<int8_t>();
        a.subsets = subsets ? c->subsets.as<int32_t>() : nullptr;
        a.sub_status = subsets ? c->substatus.as<int8_t>() : nullptr;
        a.hyp_stride = H;
        a.rng_base = hyp_begin;
        a.seed = seed;
        if (model == Model::Fm) {
            r = fm_prefilter(c, a, 1, flags, s);
            if (r) return r;
            HIPCHK(launch_fm_solve(a, 1, 0, H, s));
            HIPCHK(launch_fm_score(a, 1, 0, H, c->counts.as<int32_t>(), s));
        } else {
            HIPCHK(launch_hom_solve(a, 1, 0, H, s));
            HIPCHK(launch_hom_score(a, 1, 0, H, c->counts.as<int32_t>(), s));
        }
    }
    if (flags & RSAC_F_DEVICE_OUT) {  // device outputs: enqueued, no wait
        if (rows_out) {
            HIPCHK(launch_pack_rows(c->status.as<int8_t>(), c->counts.as<int32_t>(), H, rows_out, s));
        } else {
            HIPCHK(hipMemcpyAsync(counts_out, c->counts.p, sizeof(int32_t) * H, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(status_out, c->status.p, H, hipMemcpyDeviceToDevice, s));
        }
        if (models_out)
            HIPCHK(hipMemcpyAsync(models_out, c->models.p, sizeof(double) * kModelStride * H,
                                  hipMemcpyDeviceToDevice, s));
        return RSAC_OK;
    }
    HIPCHK(hipMemcpyAsync(counts_out, c->counts.p, sizeof(int32_t) * H, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(status_out, c->status.p, H, hipMemcpyDeviceToHost, s));
    if (models_out)
        HIPCHK(hipMemcpyAsync(models_out, c->models.p, sizeof(double) * kModelStride * H, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // PnP hypothesis records leave the validity slot to the status byte: filled in for the caller
    if (models_out && model == Model::PnP)
        for (int64_t h = 0; h < H; ++h) models_out[h * kModelStride + kValidSlot] = status_out[h] > 0 ? 1.0 : 0.0;
    return RSAC_OK;
}

int rsac_pnp_hypotheses(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                        int64_t hyp_begin, int32_t n_hyps, double thr, uint64_t seed, uint32_t flags,
                        const int32_t *subsets, int32_t *counts_out, int8_t *status_out, double *models_out,
                        void *stream) {
    return hypotheses_core(c, Model::PnP, pts3d, pts2d, n, K, hyp_begin, n_hyps, thr, seed, flags, subsets,
                           counts_out, status_out, models_out, stream);
}

int rsac_pnp_hypothesis_rows(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                             int64_t hyp_begin, int32_t n_hyps, double thr, uint64_t seed, uint32_t flags,
                             int32_t *rows_out, void *stream) {
    if (!rows_out) return fail(RSAC_EINVAL, "rows_out required");
    return hypotheses_core(c, Model::PnP, pts3d, pts2d, n, K, hyp_begin, n_hyps, thr, seed, flags | RSAC_F_DEVICE_OUT,
                           nullptr, nullptr, nullptr, nullptr, stream, rows_out);
}

int rsac_scan_device(rsac_ctx *c, rsac_scan_state *st, const int32_t *rows, int64_t count, int32_t n,
                     int32_t model_points, double confidence, int32_t stop_on_improve, int32_t *improved,
                     void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!st || count < 0 || count > INT32_MAX || n <= 0 || (count > 0 && !rows)) return fail(RSAC_EINVAL, "bad arguments");
    if (improved) *improved = 0;
    if (st->done || count == 0) return RSAC_OK;
    hipStream_t s = pick_stream(c, stream);
    const int32_t floor0 = std::max(st->max_good, model_points - 1);
    HIPCHK(c->h_scanrec.ensure(sizeof(ScanRecords)));
    ScanRecords *rec = c->h_scanrec.as<ScanRecords>();
    HIPCHK(launch_scan_rows(rows, (int32_t)count, floor0, rec, s));
    HIPCHK(hipStreamSynchronize(s));
    if (rec->nrec < 0) {  // more improvements than records: scan the copied rows exactly
        std::vector<int32_t> h(2 * (size_t)count), cn((size_t)count);
        std::vector<int8_t> sv((size_t)count);
        HIPCHK(hipMemcpyAsync(h.data(), rows, sizeof(int32_t) * 2 * count, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int64_t i = 0; i < count; ++i) {
            sv[i] = (int8_t)h[2 * i];
            cn[i] = h[2 * i + 1];
        }
        int32_t imp = 0;
        r = stop_on_improve ? rsac_scan_until_best(st, cn.data(), sv.data(), count, n, model_points, confidence, &imp)
                            : rsac_scan(st, cn.data(), sv.data(), count, n, model_points, confidence);
        if (improved) *improved = imp;
        return r;
    }
    // scan_step over the rows, replayed on the records (rsac_host.hip scan_records)
    ScanState sc;
    sc.niters = st->niters;
    sc.best = st->best;
    sc.max_good = st->max_good;
    sc.iter = st->iter;
    sc.done = st->done != 0;
    scan_records(sc, rec->idx, rec->cnt, rec->nrec, rec->first_neg, count, n, model_points, confidence,
                 stop_on_improve != 0);
    st->niters = sc.niters;
    st->best = sc.best;
    st->max_good = sc.max_good;
    st->iter = sc.iter;
    st->done = sc.done ? 1 : 0;
    if (improved) *improved = sc.improved ? 1 : 0;
    return RSAC_OK;
}

int rsac_homography_hypotheses(rsac_ctx *c, const void *src, const void *dst, int32_t n, int64_t hyp_begin,
                               int32_t n_hyps, double thr, uint64_t seed, uint32_t flags, const int32_t *subsets,
                               int32_t *counts_out, int8_t *status_out, double *models_out, void *stream) {
    return hypotheses_core(c, Model::Hom, src, dst, n, nullptr, hyp_begin, n_hyps, thr, seed, flags, subsets,
                           counts_out, status_out, models_out, stream);
}

int rsac_fundamental_hypotheses(rsac_ctx *c, const void *pts1, const void *pts2, int32_t n, int64_t hyp_begin,
                                int32_t n_hyps, double thr, uint64_t seed, uint32_t flags, int32_t *counts_out,
                                int8_t *status_out, double *models_out, void *stream) {
    return hypotheses_core(c, Model::Fm, pts1, pts2, n, nullptr, hyp_begin, n_hyps, thr, seed, flags, nullptr,
                           counts_out, status_out, models_out, stream);
}

int rsac_fundamental_ransac(rsac_ctx *c, const void *pts1, const void *pts2, int32_t n, int32_t max_iters,
                            double thr, double conf, uint64_t seed, uint32_t flags, double F_out[9],
                            uint8_t *mask_out, rsac_stats *stats, void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (n < 8) return fail(RSAC_ETOOFEW, "the 8-point fundamental matrix needs >= 8 correspondences (got %d)", n);
    if (flags & (RSAC_F_SAMPLER_OPENCV | RSAC_F_REFINE | RSAC_F_LO | RSAC_F_EPNP))
        return fail(RSAC_EINVAL, "fundamental matrix: Philox sampler only, no refit / LO");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    r = stage_points(c, pts1, pts2, 2, nullptr, 1, n, flags, s, st);
    if (r) return r;
    r = stage_tables(c, st, nullptr, thr, s);
    if (r) return r;
    HomArgs a{};
    a.SX = st.d[0]; a.SY = st.d[1]; a.DX = st.d[2]; a.DY = st.d[3];
    a.offsets = c->d_off;
    a.max_n = st.max_n();
    a.thr2 = c->d_thr2;
    a.seed = seed;
    a.rng_base = 0;
    r = ensure_hyp_buffers(c, 1, std::max(max_iters, 1), false);
    if (r) return r;
    r = fm_prefilter(c, a, 1, flags, s);
    if (r) return r;
    LoopOut lo;
    r = run_loop(c, Model::Fm, st, &a, max_iters, conf, flags, s, lo);
    if (r) return r;
    const int64_t stride = std::max(max_iters, 1);
    r = finish_masks(c, Model::Fm, st, &a, lo, stride, mask_out, flags, s);
    if (r) return r;
    const ScanState &sc = lo.scan[0];
    if (F_out) memcpy(F_out, c->h_bestmodels.as<double>(), 9 * sizeof(double));
    if (stats) {
        stats->best_hyp = sc.best;
        stats->iters = sc.iter;
        stats->hyps_scored = lo.scored;
        stats->n_inliers = sc.max_good;
        stats->rounds = lo.rounds;
        stats->gpu_ms = lo.gpu_ms;
        stats->solve_ms = lo.solve_ms;
        stats->score_ms = lo.score_ms;
        stats->lo_improvements = 0;
    }
    return sc.best >= 0 ? RSAC_OK : RSAC_NO_MODEL;
}

int rsac_pnp_mask(rsac_ctx *c, const void *pts3d, const void *pts2d, int32_t n, const double K[9],
                  const double model[12], double thr, uint32_t flags, uint8_t *mask_out, int32_t *count_out,
                  void *stream) {
    int r = check_device(c);
    if (r) return r;
    if (!model || !K) return fail(RSAC_EINVAL, "bad arguments");
    hipStream_t s = pick_stream(c, stream);
    Staged st;
    r = stage_points(c, pts3d, pts2d, 3, nullptr, 1, n, flags, s, st);
    if (r) return r;
    r = stage_tables(c, st, K, thr, s);
    if (r) return r;
    r = ensure_hyp_buffers(c, 1, 1, false);
    if (r) return r;
    double rec[kModelStride] = {0};
    memcpy(rec, model, 12 * sizeof(double));
    rec[kValidSlot] = 1.0;
    HIPCHK(hipMemcpyAsync(c->models.p, rec, sizeof rec, hipMemcpyHostToDevice, s));
    int64_t zero = 0;
    HIPCHK(hipMemcpyAsync(c->best.p, &zero, sizeof zero, hipMemcpyHostToDevice, s));
    PnpArgs a{};
    a.X = st.d[0]; a.Y = st.d[1]; a.Z = st.d[2]; a.U = st.d[3]; a.V = st.d[4];
    a.offsets = c->d_off;
    a.max_n = st.max_n();
    a.cams = c->d_cams;
    a.thr2 = c->d_thr2;
    a.models = c->models.as<double>();
    uint8_t *dmask;
    if (flags & RSAC_F_DEVICE_OUT) {
        dmask = mask_out;
    } else {
        HIPCHK(c->mask.ensure(std::max(n, 1)));
        dmask = c->mask.as<uint8_t>();
    }
    HIPCHK(launch_pnp_mask(a, 1, n, c->best.as<int64_t>(), dmask, s));
    std::vector<uint8_t> hm(std::max(n, 1));
    HIPCHK(hipMemcpyAsync(hm.data(), dmask, n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (mask_out && !(flags & RSAC_F_DEVICE_OUT)) memcpy(mask_out, hm.data(), n);
    if (count_out) {
        int32_t k = 0;
        for (int i = 0; i < n; ++i) k += hm[i];
        *count_out = k;
    }
    return RSAC_OK;
}

int rsac_pnp_refine(const double *pts3d, const double *pts2d, int32_t n, const double K[9], const uint8_t *mask,
                    double R[9], double t[3], int32_t max_iter) {
    if (n < 3 || !pts3d || !pts2d || !K || !R || !t) return fail(RSAC_EINVAL, "bad arguments");
    std::vector<float> soa((size_t)5 * n);
    for (int32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) soa[(size_t)k * n + i] = (float)pts3d[3 * i + k];
        soa[(size_t)3 * n + i] = (float)pts2d[2 * i];
        soa[(size_t)4 * n + i] = (float)pts2d[2 * i + 1];
    }
    std::vector<uint8_t> m(n, 1);
    if (mask) memcpy(m.data(), mask, n);
    const double cam[4] = {K[0], K[4], K[2], K[5]};
    const float *b = soa.data();
    return pnp_refine_lm(b, b + n, b + 2 * n, b + 3 * n, b + 4 * n, m.data(), n, cam, R, t, max_iter);
}

int rsac_pnp_epnp(const double *pts3d, const double *pts2d, int32_t n, const double K[9], const uint8_t *mask,
                  double R[9], double t[3]) {
    if (n < 4 || !pts3d || !pts2d || !K || !R || !t) return fail(RSAC_EINVAL, "bad arguments");
    std::vector<float> soa((size_t)5 * n);
    for (int32_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) soa[(size_t)k * n + i] = (float)pts3d[3 * i + k];
        soa[(size_t)3 * n + i] = (float)pts2d[2 * i];
        soa[(size_t)4 * n + i] = (float)pts2d[2 * i + 1];
    }
    std::vector<uint8_t> m(n, 1);
    if (mask) memcpy(m.data(), mask, n);
    const double cam[4] = {K[0], K[4], K[2], K[5]};
    const float *b = soa.data();
    return pnp_epnp_host(b, b + n, b + 2 * n, b + 3 * n, b + 4 * n, m.data(), n, cam, R, t) ? RSAC_OK : RSAC_NO_MODEL;
}

int rsac_pnp_epnp_minimal(const double *pts3d, const double *pts2d, const double K[9], double R[9], double t[3]) {
    if (!pts3d || !pts2d || !K || !R || !t) return fail(RSAC_EINVAL, "bad arguments");
    float X[5], Y[5], Z[5], U[5], V[5];
    for (int i = 0; i < 5; ++i) {
        X[i] = (float)pts3d[3 * i];
        Y[i] = (float)pts3d[3 * i + 1];
        Z[i] = (float)pts3d[3 * i + 2];
        U[i] = (float)pts2d[2 * i];
        V[i] = (float)pts2d[2 * i + 1];
    }
    cvq::epnp5_pose(X, Y, Z, U, V, Cam{K[0], K[4], K[2], K[5]}, R, t);
    return RSAC_OK;
}

int rsac_homography_fit(const double *src, const double *dst, int32_t n, const uint8_t *mask, double H_out[9]) {
    if (n < 4 || !src || !dst || !H_out) return fail(RSAC_ETOOFEW, "need >= 4 correspondences");
    std::vector<float> soa((size_t)4 * n);
    for (int32_t i = 0; i < n; ++i) {
        soa[i] = (float)src[2 * i];
        soa[(size_t)n + i] = (float)src[2 * i + 1];
        soa[(size_t)2 * n + i] = (float)dst[2 * i];
        soa[(size_t)3 * n + i] = (float)dst[2 * i + 1];
    }
    std::vector<uint8_t> m(n, 1);
    if (mask) memcpy(m.data(), mask, n);
    const float *b = soa.data();
    return hom_refine(b, b + n, b + 2 * n, b + 3 * n, m.data(), n, H_out) ? RSAC_OK : RSAC_NO_MODEL;
}

void rsac_rodrigues_v2m(const double r[3], double R[9]) { rodrigues_v2m(r, R); }
void rsac_rodrigues_m2v(const double R[9], double r[3]) { rodrigues_m2v(R, r); }
int rsac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    return update_num_iters(p, ep, model_points, max_iters);
}

int rsac_scan_until_best(rsac_scan_state *st, const int32_t *counts, const int8_t *status, int64_t count, int32_t n,
                         int32_t model_points, double confidence, int32_t *improved) {
    if (!st || count < 0 || n <= 0 || (count > 0 && (!counts || !status)))
        return fail(RSAC_EINVAL, "rsac_scan_until_best: bad arguments");
    ScanState s;
    s.niters = st->niters; s.best = st->best; s.iter = st->iter; s.max_good = st->max_good; s.done = st->done != 0;
    scan_step(s, counts, status, count, n, model_points, confidence, true);
    *st = rsac_scan_state{s.niters, s.best, s.iter, s.max_good, s.done ? 1 : 0};
    if (improved) *improved = s.improved ? 1 : 0;
    return RSAC_OK;
}

int rsac_scan_raise(rsac_scan_state *st, int32_t count, int32_t n, int32_t model_points, double confidence) {
    if (!st || n <= 0) return fail(RSAC_EINVAL, "rsac_scan_raise: bad arguments");
    if (count > st->max_good) {  // as local_opt applies it
        st->max_good = count;
        st->niters = update_num_iters(confidence, (double)(n - count) / n, model_points, (int)st->niters);
        if (st->iter >= st->niters) st->done = 1;
    }
    return RSAC_OK;
}

void rsac_scan_init(rsac_scan_state *st, int32_t max_iters) {
    if (!st) return;
    ScanState s;
    s.reset(max_iters);
    *st = rsac_scan_state{s.niters, s.best, s.iter, s.max_good, 0};
}

int rsac_scan(rsac_scan_state *st, const int32_t *counts, const int8_t *status, int64_t count, int32_t n,
              int32_t model_points, double confidence) {
    if (!st || count < 0 || n <= 0 || (count > 0 && (!counts || !status)))
        return fail(RSAC_EINVAL, "rsac_scan: bad arguments");
    ScanState s;
    s.niters = st->niters; s.best = st->best; s.iter = st->iter; s.max_good = st->max_good; s.done = st->done != 0;
    scan_step(s, counts, status, count, n, model_points, confidence);
    *st = rsac_scan_state{s.niters, s.best, s.iter, s.max_good, s.done ? 1 : 0};
    return RSAC_OK;
}

}  // extern "C"
