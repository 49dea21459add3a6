// rsac_host.h -- host-side pieces of the RANSAC driver: the OpenCV MWC
// sampler (for sampler="opencv"), RANSACUpdateNumIters, the resumable
// sequential best-model scan, Rodrigues and the non-minimal refits.
//
// These run on the CPU because they are sequential by definition (the MWC
// stream, the "first strictly greater" scan) or tiny (refits on the inliers
// of one model).  Reference semantics: RANSACPointSetRegistrator::run /
// getSubset (OpenCV ptsetreg.cpp) behind cv2.solvePnPRansac
// (main_v1.py:497) and cv2.findHomography (main_v1.py:312); the refits play
// the role of cv2.solvePnPRefineLM (main_v1.py:508) and findHomography's
// LS + LM polish.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace rsac {

// Run f(p) for p in [0, P) on up to 16 host threads (the per-problem MWC subset draws and refits
// of a batch are independent; each writes only its own outputs).  The workers are a persistent
// pool (rsac_host.hip: host_pool_run), created on first use, so a call costs a wake-up instead of
// 16 thread creations and joins (r06); a call made while the pool is busy (another thread's
// batch) runs on its own thread.  Sanitizer-checked by tests/sanitize (ThreadSanitizer).
void host_pool_run(int P, int nt, void (*fn)(void *, int), void *arg);
int host_pool_threads();

template <class F>
void parallel_for(int P, F f) {
    const int nt = std::min({host_pool_threads(), 16, (P + 7) / 8});
    if (nt <= 1) {
        for (int p = 0; p < P; ++p) f(p);
        return;
    }
    host_pool_run(P, nt, [](void *a, int p) { (*static_cast<F *>(a))(p); }, &f);
}

struct Mwc {
    uint64_t state = ~(uint64_t)0;
    uint32_t next() {
        state = (uint64_t)(uint32_t)state * 4164903690u + (state >> 32);
        return (uint32_t)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (uint32_t)(b - a) + (uint32_t)a); }
};

// OpenCV getSubset sequence for H consecutive iterations of k-point samples (out: H x k);
// hom != nullptr applies HomographyEstimatorCallback::checkSubset (sx, sy, dx, dy SoA; k = 4).
void mwc_subsets(Mwc &rng, int n, int64_t H, const float *const *hom, int32_t *out, int8_t *status, int k = 4);

int update_num_iters(double p, double ep, int model_points, int max_iters);
// update_num_iters(p, (n - c) / n, ...) through a per-thread table of its pow and logs (the scan replays)
int update_num_iters_count(double p, int n, int c, int model_points, int max_iters);

struct ScanState {
    int64_t niters = 1;
    int64_t best = -1;
    int32_t max_good = 0;
    int64_t iter = 0;
    bool done = false;
    bool improved = false;  // set by scan_step(stop_on_improve) when it stopped at a new best
    void reset(int max_iters) {
        niters = max_iters > 1 ? max_iters : 1;
        best = -1; max_good = 0; iter = 0; done = false; improved = false;
    }
};

// consume hypotheses [s.iter, s.iter + count) (counts/status indexed from 0)
// stop_on_improve: return right after a new best (s.improved set, s.iter = its index + 1)
void scan_step(ScanState &s, const int32_t *counts, const int8_t *status, int64_t count, int n, int model_points,
               double confidence, bool stop_on_improve = false);

// the round [s.iter, s.iter + H) from its improvement records (rsac_internal.h ScanRecords:
// the strict prefix maxima above the scan's floor, idx / first_neg relative to the round's
// start): identical to scan_step over the full rows
void scan_records(ScanState &s, const int32_t *idx, const int32_t *cnt, int nrec, int32_t first_neg, int64_t H, int n,
                  int model_points, double confidence, bool stop_on_improve = false);

void rodrigues_v2m(const double r[3], double R[9]);
void rodrigues_m2v(const double R[9], double r[3]);

// EPnP on the masked points (the final solve of solvePnPRansac with SOLVEPNP_P3P),
// bit-identical to k_pnp_epnp; false for < 4 inliers or a degenerate cloud.
bool pnp_epnp_host(const float *X, const float *Y, const float *Z, const float *U, const float *V, const uint8_t *mask,
                   int n, const double cam[4], double R[9], double t[3]);

// LM over (R, t) on masked correspondences (f32 SoA); returns iterations
int pnp_refine_lm(const float *X, const float *Y, const float *Z, const float *U, const float *V, const uint8_t *mask,
                  int n, const double cam[4], double R[9], double t[3], int max_iter);

// least-squares normalised DLT on the inliers + 10 LM iterations
bool hom_refine(const float *sx, const float *sy, const float *dx, const float *dy, const uint8_t *mask, int n,
                double H[9]);

}  // namespace rsac
