/*
 * rsac_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's RANSAC hot path.  Only tests/, the
 * cpu_baseline leg of bench.py and __graft_entry__.smoke() may load this
 * library, and only as the checker / the timed CPU baseline.  The product
 * (code-reproduction-ransac_amd/csrc) never links or calls it.
 *
 * What it restates
 * ----------------
 * The reference (Mendel0408/Code-Reproduction-RANSAC) contains no RANSAC
 * arithmetic of its own: it calls OpenCV (third party, NOT vendored under
 * /root/reference, version not pinned; semantics below follow the public
 * OpenCV 4.x calib3d sources: ptsetreg.cpp, fundam.cpp, solvepnp.cpp,
 * calibration.cpp):
 *   - cv2.solvePnPRansac   main_v1.py:497-502, testpro-K.py:72-75,
 *                          testpro.py:536-541, test_pro.py:515-520
 *   - cv2.findHomography   main_v1.py:312, process.py:200, test02.py:263,
 *                          testpro.py:350, test_pro.py:351
 *   - cv2.projectPoints    testpro-K.py:33 (compute_reprojection_error)
 *   - cv2.solvePnPRefineLM main_v1.py:508-509, testpro-K.py:122-125
 *   - cv2.Rodrigues        main_v1.py:895, testpro-K.py:84
 * and re-scores in Python (main_v1.py:332-348, 419).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - homography RANSAC (MWC sampler, OpenCV getSubset/checkSubset, f32 error,
 *     RANSAC-phase mask) is pinned against the 24 complete findHomography
 *     blocks recorded in the reference's debug.log (tests/golden/);
 *   - PnP, OpenCV's default minimal solver (EPnP on 5-point MWC samples, the mode every reference
 *     call site runs) and the Rodrigues round trip of its models are OpenCV's own operation
 *     sequence (cv_epnp.c: undistortPoints' f32 round trip, epnp.cpp, lapack.cpp's JacobiSVD,
 *     cvRodrigues2), unfused, and the default here (ORC_SEQ_CV).  The round-4/5 restatement of that
 *     solver (ORC_SEQ_RR: round-robin Jacobi, fused steps) stays for the decision-change study
 *     (scripts/epnp_variants.py, profiles/r06/epnp_variants.md), as does its unfused build
 *     (liboracle_unfused.so).  PnP parity vs OpenCV itself is *unpinned* (OpenCV is absent) except
 *     for the loose known-answer camera origin of testpro-K.py:234; GPU parity is against this
 *     restatement.
 *   - The north-star P3P kernel (Lambda Twist, Persson & Nordberg, ECCV 2018; OpenCV's P3P is a
 *     different algorithm and no reference call selects it), the LM refit, the non-minimal EPnP of
 *     the P3P mode's final solve and the fundamental-matrix solver are this project's own
 *     arithmetic: explicit fma() where the GPU fuses (the same correctly rounded result on every
 *     backend).
 *   - OpenCV's count == model_points branches ([OpenCV, unvendored] solvepnp.cpp
 *     solvePnPRansac: 4 points, or 5 under the default flags -> one solvePnP on all points, every
 *     index an inlier, no final solve; fundam.cpp findHomography: 4 points -> runKernel, mask all
 *     ones, no LM) are restated in pnp_direct and orc_hom_ransac.
 *
 * Numerics contract shared with the HIP path (bit-exact on counts/masks/models):
 *   compile with -ffp-contract=off, no -ffast-math; every quantity that decides a count is
 *   computed as OpenCV computes it where OpenCV defines it (computeError: f64 projection of
 *   f32-rounded inputs, rounded to f32, f32 squared error, `err <= (float)(thr*thr)`; the EPnP-5
 *   models above; the homography DLT and error), with only + - * / sqrt (libm's hypot, acos, sin
 *   and cos restated deterministically); fused operations appear only in the project's own
 *   solvers listed above, written explicitly as fma().
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#define ORC_API __attribute__((visibility("default")))

#ifdef ORC_UNFUSED
/* liboracle_unfused.so (test infrastructure for the decision-change study): every explicit fused
 * step of the restated solvers evaluated as a rounded product and a rounded sum */
#define fma(a, b, c) ((a) * (b) + (c))
#endif

/* The EPnP-5 minimal solver and the Rodrigues round trip of the PnP models:
 *   ORC_SEQ_CV (default) OpenCV's operation sequence (cv_epnp.c orc_cv_epnp, orc_cv_rvec_roundtrip);
 *   ORC_SEQ_RR           this project's round-4/5 EPnP (round-robin Jacobi, Householder betas,
 *                        polar-factor rotation; orc_pnp_epnp) and Rodrigues (polar Newton), kept
 *                        for the comparison of tests/test_cv_epnp.py and scripts/epnp_variants.py */
enum { ORC_SEQ_CV = 0, ORC_SEQ_RR = 1 };
static int g_seq = ORC_SEQ_CV;
ORC_API void orc_set_sequence(int v) { g_seq = v; }
ORC_API int orc_get_sequence(void) { return g_seq; }
ORC_API int orc_cv_epnp(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                        const int32_t *idx, int n, const double cam[4], double R[9], double t[3]);
ORC_API void orc_cv_rvec_roundtrip(double R[9]);
ORC_API void orc_cv_rodrigues_m2v(const double Rin[9], double r[3]);
ORC_API void orc_cv_rodrigues_v2m(const double rin[3], double R[9]);

/* ------------------------------------------------------------------------ */
/* RNG 1: OpenCV cv::RNG, multiply-with-carry, seeded (uint64)-1 in         */
/* RANSACPointSetRegistrator::run (ptsetreg.cpp) -- behind every cv2.* call  */
/* listed above.                                                             */
/* ------------------------------------------------------------------------ */
ORC_API uint32_t orc_mwc_next(uint64_t *st) {
    *st = (uint64_t)(uint32_t)(*st) * 4164903690u + (*st >> 32);
    return (uint32_t)(*st);
}

ORC_API int orc_mwc_uniform(uint64_t *st, int a, int b) {
    if (a == b) return a;
    uint32_t r = orc_mwc_next(st);
    return (int)(r % (uint32_t)(b - a) + (uint32_t)a);
}

/* ------------------------------------------------------------------------ */
/* RNG 2: Philox-4x32-10 (Salmon et al., SC'11), the counter-based sampler  */
/* the north star asks for.  key = seed, counter = (hyp_lo, hyp_hi,          */
/* problem, block).                                                          */
/* ------------------------------------------------------------------------ */
ORC_API void orc_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
    uint32_t key[2], ctr[4], buf[4];
    int pos;
} orc_stream;

static void stream_init(orc_stream *s, uint64_t seed, uint32_t problem, uint64_t hyp) {
    s->key[0] = (uint32_t)seed; s->key[1] = (uint32_t)(seed >> 32);
    s->ctr[0] = (uint32_t)hyp; s->ctr[1] = (uint32_t)(hyp >> 32);
    s->ctr[2] = problem; s->ctr[3] = 0;
    s->pos = 4;
}

static uint32_t stream_next(orc_stream *s) {
    if (s->pos == 4) {
        orc_philox4x32_10(s->ctr, s->key, s->buf);
        s->ctr[3] += 1u;
        s->pos = 0;
    }
    return s->buf[s->pos++];
}

/* multiply-shift range reduction: floor(r * n / 2^32) */
static int stream_index(orc_stream *s, int n) {
    return (int)(((uint64_t)stream_next(s) * (uint64_t)(uint32_t)n) >> 32);
}

#define ORC_MAX_DRAWS_PER_SUBSET 256
#define ORC_MAX_SUBSET_ATTEMPTS 10000 /* getSubset(..., rng, 10000) in RANSACPointSetRegistrator::run */

/* draw s distinct indices from the hypothesis' stream; -1 on exhaustion */
static int stream_subset(orc_stream *st, int n, int s, int32_t *idx) {
    int draws = 0;
    for (int i = 0; i < s; ++i) {
        for (;;) {
            if (draws++ >= ORC_MAX_DRAWS_PER_SUBSET) return -1;
            int r = stream_index(st, n);
            int dup = 0;
            for (int j = 0; j < i; ++j) dup |= (idx[j] == r);
            if (!dup) { idx[i] = r; break; }
        }
    }
    return 0;
}

ORC_API int orc_philox_subset(uint64_t seed, uint32_t problem, uint64_t hyp, int n, int s, int32_t *idx) {
    if (n < s) return -1;
    orc_stream st;
    stream_init(&st, seed, problem, hyp);
    return stream_subset(&st, n, s, idx);
}

/* ------------------------------------------------------------------------ */
/* RANSACUpdateNumIters (ptsetreg.cpp), used after every new best model.     */
/* ------------------------------------------------------------------------ */
static int cv_round(double v) { return (int)lrint(v); }

ORC_API int orc_update_num_iters(double p, double ep, int model_points, int max_iters) {
    if (model_points <= 0) return -1;
    p = p > 0. ? p : 0.; p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
    double num = 1. - p; if (num < DBL_MIN) num = DBL_MIN;
    double denom = 1. - pow(1. - ep, model_points);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : cv_round(num / denom);
}

/* Sequential best-model selection of RANSACPointSetRegistrator::run:
 * iterate hypotheses in index order while iter < niters; status<0 = subset
 * not found (break; failure if at iter 0), status==0 = kernel produced no
 * model (continue), else a model whose count replaces the best iff
 * count > max(best, model_points-1); niters shrinks on each new best. */
ORC_API int64_t orc_scan(const int32_t *counts, const int8_t *status, int64_t H, int n, int model_points,
                         double confidence, int max_iters, int32_t *best_count_out, int64_t *iters_out) {
    int64_t niters = max_iters > 1 ? max_iters : 1;
    int64_t best = -1, i;
    int32_t max_good = 0;
    for (i = 0; i < H && i < niters; ++i) {
        if (status[i] < 0) { if (i == 0) best = -1; break; }
        if (status[i] == 0) continue;
        int32_t c = counts[i];
        int32_t floor_c = max_good > model_points - 1 ? max_good : model_points - 1;
        if (c > floor_c) {
            best = i; max_good = c;
            niters = orc_update_num_iters(confidence, (double)(n - c) / n, model_points, (int)niters);
        }
    }
    if (best_count_out) *best_count_out = max_good;
    if (iters_out) *iters_out = i;
    return best;
}

/* ------------------------------------------------------------------------ */
/* Projection + error (PnPRansacCallback::computeError -> projectPoints with */
/* zero distortion, calibration.cpp), the formula of testpro-K.py:32-36.     */
/* Inputs are the f32-rounded points (solvePnPRansac converts to CV_32F).    */
/* ------------------------------------------------------------------------ */
ORC_API float orc_pnp_err(const double R[9], const double t[3], const double cam[4],
                          float Xf, float Yf, float Zf, float uf, float vf) {
    double X = Xf, Y = Yf, Z = Zf;
    double x = R[0] * X + R[1] * Y; x = x + R[2] * Z; x = x + t[0];
    double y = R[3] * X + R[4] * Y; y = y + R[5] * Z; y = y + t[1];
    double z = R[6] * X + R[7] * Y; z = z + R[8] * Z; z = z + t[2];
    double iz = (z != 0.0) ? 1.0 / z : 1.0;
    x = x * iz; y = y * iz;
    double pu = x * cam[0] + cam[2];
    double pv = y * cam[1] + cam[3];
    float dx = uf - (float)pu;
    float dy = vf - (float)pv;
    float e1 = dx * dx, e2 = dy * dy;
    return e1 + e2;
}

ORC_API float orc_thr2(double thr) { return (float)(thr * thr); }

/* compute_reprojection_error (testpro-K.py:32-36) itself: cv2.projectPoints of the f64 inputs
 * (no CV_32F conversion there) in f64, then np.linalg.norm(pixels - projected, axis=1) =
 * sqrt(dx*dx + dy*dy) per point.  proj (n x 2) and err (n) optional. */
ORC_API void orc_reproj_errors(const double R[9], const double t[3], const double cam[4], const double *p3,
                               const double *p2, int n, double *proj, double *err) {
    for (int i = 0; i < n; ++i) {
        const double X = p3[3 * i], Y = p3[3 * i + 1], Z = p3[3 * i + 2];
        double x = R[0] * X + R[1] * Y; x = x + R[2] * Z; x = x + t[0];
        double y = R[3] * X + R[4] * Y; y = y + R[5] * Z; y = y + t[1];
        double z = R[6] * X + R[7] * Y; z = z + R[8] * Z; z = z + t[2];
        double iz = (z != 0.0) ? 1.0 / z : 1.0;
        x = x * iz; y = y * iz;
        const double pu = x * cam[0] + cam[2], pv = y * cam[1] + cam[3];
        const double dx = p2[2 * i] - pu, dy = p2[2 * i + 1] - pv;
        if (proj) { proj[2 * i] = pu; proj[2 * i + 1] = pv; }
        if (err) err[i] = sqrt(dx * dx + dy * dy);
    }
}

/* np.mean of the inliers' errors (testpro-K.py:80-82), in the summation order of the GPU's
 * wave reduction: lane l (0..63) sums the masked errors of points l, l + 64, ... ascending, then
 * the xor butterfly over the 64 lane sums (o = 32 .. 1).  -> the sum; *count = inliers. */
ORC_API double orc_reproj_mean_sum(const double R[9], const double t[3], const double cam[4], const double *p3,
                                   const double *p2, const uint8_t *mask, int n, int *count) {
    double v[64];
    int c = 0;
    for (int l = 0; l < 64; ++l) {
        v[l] = 0.0;
        for (int i = l; i < n; i += 64)
            if (mask[i]) {
                double e;
                orc_reproj_errors(R, t, cam, p3 + 3 * i, p2 + 2 * i, 1, NULL, &e);
                v[l] = v[l] + e;
                ++c;
            }
    }
    for (int o = 32; o > 0; o >>= 1) {
        double w[64];
        for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ o];
        memcpy(v, w, sizeof v);
    }
    *count = c;
    return v[0];
}

ORC_API int32_t orc_pnp_count(const double R[9], const double t[3], const double cam[4],
                              const float *X, const float *Y, const float *Z, const float *U, const float *V,
                              int n, float thr2, uint8_t *mask) {
    int32_t c = 0;
    for (int i = 0; i < n; ++i) {
        float e = orc_pnp_err(R, t, cam, X[i], Y[i], Z[i], U[i], V[i]);
        int f = e <= thr2;
        if (mask) mask[i] = (uint8_t)f;
        c += f;
    }
    return c;
}

/* ------------------------------------------------------------------------ */
/* P3P: Lambda Twist (Persson & Nordberg 2018), restated.  3 bearings y_k    */
/* (unit), 3 world points x_k -> up to 4 (R, t) with y_k ~ R x_k + t.        */
/* ------------------------------------------------------------------------ */
static void root2real(double b, double c, double *r1, double *r2, int *ok) {
    double v = b * b - 4.0 * c;
    if (v < 0.0) { *r1 = 0.5 * b; *r2 = 0.5 * b; *ok = 0; return; }
    double y = sqrt(v);
    if (b < 0.0) { *r1 = 0.5 * (-b + y); *r2 = 2.0 * c / (-b + y); }
    else { *r1 = 2.0 * c / (-b - y); *r2 = 0.5 * (-b - y); }
    *ok = 1;
}

/* one real root of g^3 + b g^2 + c g + d: start near the sharpest root, then
 * Newton (at most 50 steps, stop once |f| <= 1e-13 after the 7th) */
static double cubic_root(double b, double c, double d) {
    double r0;
    if (b * b >= 3.0 * c) {
        double v = sqrt(b * b - 3.0 * c);
        double t1 = (-b - v) / 3.0;
        double k = ((t1 + b) * t1 + c) * t1 + d;
        if (k > 0.0) {
            r0 = t1 - sqrt(-k / (3.0 * t1 + b));
        } else {
            double t2 = (-b + v) / 3.0;
            k = ((t2 + b) * t2 + c) * t2 + d;
            r0 = t2 + sqrt(-k / (3.0 * t2 + b));
        }
    } else {
        r0 = -b / 3.0;
        if (fabs((3.0 * r0 + 2.0 * b) * r0 + c) < 1e-4) r0 = r0 + 1.0;
    }
    /* Newton: at least 7 steps, stop at |f| <= 1e-13, at most 12 (the published solver allows
     * 50; lanes whose |f| stalls at the rounding level above 1e-13 -- about 4 % of C2's samples --
     * then stop at 12 instead of 50, so a GPU wave no longer runs 50 divisions for one of them) */
    for (int it = 0; it < 12; ++it) {
        /* Horner by fma (rsac_math.h cubic_root, r05) */
        double fx = fma(fma(r0 + b, r0, c), r0, d);
        if (it >= 7 && !(fabs(fx) > 1e-13)) break;
        double fpx = fma(3.0 * r0 + 2.0 * b, r0, c);
        r0 = r0 - fx / fpx;
    }
    return r0;
}

/* eigenvectors of the two non-zero eigenvalues of a symmetric 3x3 A whose
 * third eigenvalue is known to be 0; columns: v1 (|e1|>=|e2|), v2 */
static void eig_known0(const double A[9], double v1[3], double v2[3], double *e1o, double *e2o) {
    double a00 = A[0], a01 = A[1], a02 = A[2], a11 = A[4], a12 = A[5], a22 = A[8];
    double a01sq = a01 * a01;
    double b = -a00 - a11 - a22;
    double c = fma(a11, a22, fma(a00, a11 + a22, fma(-a12, a12, fma(-a02, a02, -a01sq))));
    double e1, e2; int ok;
    root2real(b, c, &e1, &e2, &ok);
    if (fabs(e1) < fabs(e2)) { double tmp = e1; e1 = e2; e2 = tmp; }
    double m0011 = -a00 * a11;
    double pr0 = fma(a01, a12, -(a02 * a11));
    double pr1 = fma(a01, a02, -(a00 * a12));
    {
        double e = e1;
        double tmp = 1.0 / (fma(-e, e, fma(e, a00 + a11, m0011)) + a01sq);
        double q1 = -fma(e, a02, pr0) * tmp;
        double q2 = -fma(e, a12, pr1) * tmp;
        double rn = 1.0 / sqrt(fma(q2, q2, q1 * q1) + 1.0);
        v1[0] = q1 * rn; v1[1] = q2 * rn; v1[2] = rn;
    }
    {
        double e = e2;
        double tmp = 1.0 / (fma(-e, e, fma(e, a00 + a11, m0011)) + a01sq);
        double q1 = -fma(e, a02, pr0) * tmp;
        double q2 = -fma(e, a12, pr1) * tmp;
        double rn = 1.0 / sqrt(fma(q2, q2, q1 * q1) + 1.0);
        v2[0] = q1 * rn; v2[1] = q2 * rn; v2[2] = rn;
    }
    *e1o = e1; *e2o = e2;
}

static double lt_resid(const double L[3], double a12, double a13, double a23, double b12, double b13, double b23,
                       double r[3]) {
    double l1 = L[0], l2 = L[1], l3 = L[2];
    /* fma chains (rsac_math.h lt_resid, r05) */
    r[0] = fma(b12 * l1, l2, fma(l2, l2, l1 * l1)) - a12;
    r[1] = fma(b13 * l1, l3, fma(l3, l3, l1 * l1)) - a13;
    r[2] = fma(b23 * l2, l3, fma(l3, l3, l2 * l2)) - a23;
    return fabs(r[0]) + fabs(r[1]) + fabs(r[2]);
}

static void lt_refine(double L[3], double a12, double a13, double a23, double b12, double b13, double b23) {
    for (int it = 0; it < 5; ++it) {
        double r[3];
        double s0 = lt_resid(L, a12, a13, a23, b12, b13, b23, r);
        if (s0 < 1e-10) break;
        double l1 = L[0], l2 = L[1], l3 = L[2];
        double j0 = fma(b12, l2, 2.0 * l1);  /* dr1/dl1 */
        double j1 = fma(b12, l1, 2.0 * l2);  /* dr1/dl2 */
        double j3 = fma(b13, l3, 2.0 * l1);  /* dr2/dl1 */
        double j5 = fma(b13, l1, 2.0 * l3);  /* dr2/dl3 */
        double j7 = fma(b23, l3, 2.0 * l2);  /* dr3/dl2 */
        double j8 = fma(b23, l2, 2.0 * l3);  /* dr3/dl3 */
        double det = 1.0 / (-j0 * j5 * j7 - j1 * j3 * j8);
        double d0 = fma(j1 * j5, r[2], fma(-j1 * j8, r[1], -j5 * j7 * r[0]));
        double d1 = fma(-j0 * j5, r[2], fma(j0 * j8, r[1], -j3 * j8 * r[0]));
        double d2 = fma(-j1 * j3, r[2], fma(-j0 * j7, r[1], j3 * j7 * r[0]));
        double Ln[3];
        Ln[0] = fma(-det, d0, l1); Ln[1] = fma(-det, d1, l2); Ln[2] = fma(-det, d2, l3);
        double rn[3];
        double s1 = lt_resid(Ln, a12, a13, a23, b12, b13, b23, rn);
        if (s1 > s0) break;
        L[0] = Ln[0]; L[1] = Ln[1]; L[2] = Ln[2];
    }
}

static void cross3(const double a[3], const double b[3], double c[3]) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* inverse of the 3x3 (row-major) by the adjugate; 0 if singular */
static int inv3(const double M[9], double I[9]) {
    double c00 = M[4] * M[8] - M[5] * M[7];
    double c01 = M[5] * M[6] - M[3] * M[8];
    double c02 = M[3] * M[7] - M[4] * M[6];
    double det = M[0] * c00 + M[1] * c01 + M[2] * c02;
    if (det == 0.0 || !isfinite(det)) return 0;
    double id = 1.0 / det;
    I[0] = c00 * id; I[1] = (M[2] * M[7] - M[1] * M[8]) * id; I[2] = (M[1] * M[5] - M[2] * M[4]) * id;
    I[3] = c01 * id; I[4] = (M[0] * M[8] - M[2] * M[6]) * id; I[5] = (M[2] * M[3] - M[0] * M[5]) * id;
    I[6] = c02 * id; I[7] = (M[1] * M[6] - M[0] * M[7]) * id; I[8] = (M[0] * M[4] - M[1] * M[3]) * id;
    return 1;
}

/* y: 3 unit bearings (row k = bearing k); x: 3 world points.  Returns the
 * number of solutions written to Rs (k*9) / ts (k*3). */
ORC_API int orc_p3p(const double y[9], const double x[9], double Rs[36], double ts[12]) {
    const double *y1 = y, *y2 = y + 3, *y3 = y + 6;
    const double *x1 = x, *x2 = x + 3, *x3 = x + 6;
    double b12 = -2.0 * fma(y1[2], y2[2], fma(y1[1], y2[1], y1[0] * y2[0]));
    double b13 = -2.0 * fma(y1[2], y3[2], fma(y1[1], y3[1], y1[0] * y3[0]));
    double b23 = -2.0 * fma(y2[2], y3[2], fma(y2[1], y3[1], y2[0] * y3[0]));
    double d12[3], d13[3], d23[3], d12xd13[3];
    for (int k = 0; k < 3; ++k) { d12[k] = x1[k] - x2[k]; d13[k] = x1[k] - x3[k]; d23[k] = x2[k] - x3[k]; }
    cross3(d12, d13, d12xd13);
    double a12 = fma(d12[2], d12[2], fma(d12[1], d12[1], d12[0] * d12[0]));
    double a13 = fma(d13[2], d13[2], fma(d13[1], d13[1], d13[0] * d13[0]));
    double a23 = fma(d23[2], d23[2], fma(d23[1], d23[1], d23[0] * d23[0]));

    double c31 = -0.5 * b13, c23 = -0.5 * b23, c12 = -0.5 * b12;
    double blob = c12 * c23 * c31 - 1.0;
    double s31 = 1.0 - c31 * c31, s23 = 1.0 - c23 * c23, s12 = 1.0 - c12 * c12;

    /* fma chains (rsac_math.h lt_common, r05) */
    double p3 = a13 * fma(a23, s31, -(a13 * s23));
    double p2 = fma(a23 * (a23 - a12), s31, fma(a13 * (2.0 * a12 + a13), s23, 2.0 * blob * a23 * a13));
    double p1 = fma(-(2.0 * a12), fma(a13, s23, blob * a23), fma(-(a12 * a12), s23, a23 * (a13 - a23) * s12));
    double p0 = a12 * fma(a12, s23, -(a23 * s12));
    if (p3 == 0.0 || !isfinite(p3)) return 0;
    double ip3 = 1.0 / p3;
    p2 = p2 * ip3; p1 = p1 * ip3; p0 = p0 * ip3;
    double g = cubic_root(p2, p1, p0);

    double A[9];
    A[0] = a23 * (1.0 - g);
    A[1] = (a23 * b12) * 0.5;
    A[2] = (a23 * b13 * g) * (-0.5);
    A[4] = a23 - a12 + a13 * g;
    A[5] = b23 * (a13 * g - a12) * 0.5;
    A[8] = g * (a13 - a23) - a12;
    A[3] = A[1]; A[6] = A[2]; A[7] = A[5];

    double v1[3], v2[3], e1, e2;
    eig_known0(A, v1, v2, &e1, &e2);
    double vq = -e2 / e1;
    double v = sqrt(vq > 0.0 ? vq : 0.0);

    double Ls[4][3];
    int valid = 0;
    for (int sgn = 0; sgn < 2; ++sgn) {
        double s = sgn == 0 ? v : -v;
        double w2 = 1.0 / fma(s, v2[0], -v1[0]);
        double w0 = fma(-s, v2[1], v1[1]) * w2;
        double w1 = fma(-s, v2[2], v1[2]) * w2;
        double a = 1.0 / (fma(-(a12 * b13), w1, (a13 - a12) * w1 * w1) - a12);
        double b = fma(-(2.0 * w0 * w1), a12 - a13, fma(-(a12 * b13), w0, a13 * b12 * w1)) * a;
        double c = (fma(a13 * b12, w0, (a13 - a12) * w0 * w0) + a13) * a;
        if (b * b - 4.0 * c >= 0.0) {
            double tau[2]; int ok;
            root2real(b, c, &tau[0], &tau[1], &ok);
            for (int q = 0; q < 2; ++q) {
                if (tau[q] > 0.0) {
                    double tq = tau[q];
                    double d = a23 / (tq * (b23 + tq) + 1.0);
                    if (d > 0.0) {
                        double l2 = sqrt(d);
                        double l3 = tq * l2;
                        double l1 = w0 * l2 + w1 * l3;
                        if (l1 >= 0.0) { Ls[valid][0] = l1; Ls[valid][1] = l2; Ls[valid][2] = l3; ++valid; }
                    }
                }
            }
        }
    }
    for (int i = 0; i < valid; ++i) lt_refine(Ls[i], a12, a13, a23, b12, b13, b23);

    double Xm[9] = {d12[0], d13[0], d12xd13[0], d12[1], d13[1], d12xd13[1], d12[2], d13[2], d12xd13[2]};
    double Xi[9];
    if (!inv3(Xm, Xi)) return 0;
    int nout = 0;
    for (int i = 0; i < valid; ++i) {
        double ry1[3], ry2[3], ry3[3], yd1[3], yd2[3], yd1xd2[3];
        for (int k = 0; k < 3; ++k) { ry1[k] = y1[k] * Ls[i][0]; ry2[k] = y2[k] * Ls[i][1]; ry3[k] = y3[k] * Ls[i][2]; }
        for (int k = 0; k < 3; ++k) { yd1[k] = ry1[k] - ry2[k]; yd2[k] = ry1[k] - ry3[k]; }
        cross3(yd1, yd2, yd1xd2);
        double Ym[9] = {yd1[0], yd2[0], yd1xd2[0], yd1[1], yd2[1], yd1xd2[1], yd1[2], yd2[2], yd1xd2[2]};
        double *R = Rs + 9 * nout, *t = ts + 3 * nout;
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc)
                R[3 * r + cc] = fma(Ym[3 * r + 2], Xi[6 + cc], fma(Ym[3 * r + 1], Xi[3 + cc], Ym[3 * r] * Xi[cc]));
        int fin = 1;
        for (int r = 0; r < 3; ++r) {
            double rx = fma(R[3 * r + 2], x1[2], fma(R[3 * r + 1], x1[1], R[3 * r] * x1[0]));
            t[r] = ry1[r] - rx;
            fin &= isfinite(t[r]) != 0;
        }
        for (int k = 0; k < 9; ++k) fin &= isfinite(R[k]) != 0;
        if (fin) ++nout;
    }
    return nout;
}

/* bearing of pixel (u, v): K^-1 [u v 1]^T normalised (skew ignored, as in
 * cvProjectPoints2Internal which reads only fx, fy, cx, cy) */
static void bearing(const double cam[4], float uf, float vf, double out[3]) {
    double xn = ((double)uf - cam[2]) / cam[0];
    double yn = ((double)vf - cam[3]) / cam[1];
    double nrm = sqrt(xn * xn + yn * yn + 1.0);
    out[0] = xn / nrm; out[1] = yn / nrm; out[2] = 1.0 / nrm;
}

/* 4-point minimal PnP kernel (as OpenCV's SOLVEPNP_P3P with 4 points: solve
 * on the first three, keep the solution that reprojects the fourth best).
 * Returns 1 and (R, t) when a model exists, 0 otherwise. */
ORC_API int orc_pnp_minimal(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                            const int32_t idx[4], const double cam[4], double R[9], double t[3]) {
    double yb[9], xw[9];
    for (int k = 0; k < 3; ++k) {
        int i = idx[k];
        bearing(cam, U[i], V[i], yb + 3 * k);
        xw[3 * k] = X[i]; xw[3 * k + 1] = Y[i]; xw[3 * k + 2] = Z[i];
    }
    double Rs[36], ts[12];
    int ns = orc_p3p(yb, xw, Rs, ts);
    if (ns == 0) return 0;
    int i4 = idx[3];
    double X4 = X[i4], Y4 = Y[i4], Z4 = Z[i4];
    int best = -1;
    double best_e = 0.0;
    for (int s = 0; s < ns; ++s) {
        const double *Rk = Rs + 9 * s, *tk = ts + 3 * s;
        double x = fma(Rk[2], Z4, fma(Rk[1], Y4, Rk[0] * X4)) + tk[0];
        double y = fma(Rk[5], Z4, fma(Rk[4], Y4, Rk[3] * X4)) + tk[1];
        double z = fma(Rk[8], Z4, fma(Rk[7], Y4, Rk[6] * X4)) + tk[2];
        double iz = (z != 0.0) ? 1.0 / z : 1.0;
        double du = (x * iz) * cam[0] + cam[2] - (double)U[i4];
        double dv = (y * iz) * cam[1] + cam[3] - (double)V[i4];
        double e = du * du + dv * dv;
        if (!(e == e)) continue;
        if (best < 0 || e < best_e) { best = s; best_e = e; }
    }
    if (best < 0) return 0;
    memcpy(R, Rs + 9 * best, 9 * sizeof(double));
    memcpy(t, ts + 3 * best, 3 * sizeof(double));
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Homography (HomographyEstimatorCallback, fundam.cpp) for findHomography   */
/* at main_v1.py:312 / process.py:200.                                       */
/* ------------------------------------------------------------------------ */

/* haveCollinearPoints(m, count): only the last point against every pair */
static int have_collinear(const float *px, const float *py, const int32_t *idx, int count) {
    int i = count - 1;
    for (int j = 0; j < i; ++j) {
        double dx1 = (double)(px[idx[j]] - px[idx[i]]);
        double dy1 = (double)(py[idx[j]] - py[idx[i]]);
        for (int k = 0; k < j; ++k) {
            double dx2 = (double)(px[idx[k]] - px[idx[i]]);
            double dy2 = (double)(py[idx[k]] - py[idx[i]]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

static double det3_rows(double a0, double a1, double b0, double b1, double c0, double c1) {
    /* Matx33d determinant of [[a0 a1 1],[b0 b1 1],[c0 c1 1]] (OpenCV's expansion) */
    return a0 * (b1 * 1. - c1 * 1.) - a1 * (b0 * 1. - c0 * 1.) + 1. * (b0 * c1 - c0 * b1);
}

/* checkSubset(ms1, ms2, 4): collinearity in src and dst, then the
 * orientation-consistency test of Marquez-Neila et al. */
ORC_API int orc_hom_check_subset(const float *sx, const float *sy, const float *dx, const float *dy,
                                 const int32_t idx[4]) {
    if (have_collinear(sx, sy, idx, 4) || have_collinear(dx, dy, idx, 4)) return 0;
    static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    int negative = 0;
    for (int i = 0; i < 4; ++i) {
        const int *q = tt[i];
        int p0 = idx[q[0]], p1 = idx[q[1]], p2 = idx[q[2]];
        double dA = det3_rows(sx[p0], sy[p0], sx[p1], sy[p1], sx[p2], sy[p2]);
        double dB = det3_rows(dx[p0], dy[p0], dx[p1], dy[p1], dx[p2], dy[p2]);
        negative += dA * dB < 0;
    }
    return negative == 0 || negative == 4;
}

/* normalisation of HomographyEstimatorCallback::runKernel */
typedef struct { double cMx, cMy, cmx, cmy, sMx, sMy, smx, smy; } hnorm;

static int hom_norm(const float *sx, const float *sy, const float *dx, const float *dy, const int32_t *idx,
                    int count, hnorm *h) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < count; ++i) {
        int p = idx ? idx[i] : i;
        cmx += dx[p]; cmy += dy[p];
        cMx += sx[p]; cMy += sy[p];
    }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
    for (int i = 0; i < count; ++i) {
        int p = idx ? idx[i] : i;
        smx += fabs(dx[p] - cmx); smy += fabs(dy[p] - cmy);
        sMx += fabs(sx[p] - cMx); sMy += fabs(sy[p] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return 0;
    h->smx = count / smx; h->smy = count / smy; h->sMx = count / sMx; h->sMy = count / sMy;
    h->cmx = cmx; h->cmy = cmy; h->cMx = cMx; h->cMy = cMy;
    return 1;
}

static void mat3mul(const double A[9], const double B[9], double C[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

/* H = invHnorm * Hn * Hnorm2, then scaled by 1/H22 (convertTo) */
static void hom_denorm(const hnorm *h, const double Hn[9], double H[9]) {
    double invHnorm[9] = {1. / h->smx, 0, h->cmx, 0, 1. / h->smy, h->cmy, 0, 0, 1};
    double Hnorm2[9] = {h->sMx, 0, -h->cMx * h->sMx, 0, h->sMy, -h->cMy * h->sMy, 0, 0, 1};
    double T[9], H0[9];
    mat3mul(invHnorm, Hn, T);
    mat3mul(T, Hnorm2, H0);
    double sc = 1. / H0[8];
    for (int k = 0; k < 9; ++k) H[k] = H0[k] * sc;
}

/* Minimal 4-point kernel of this build: the normalised DLT of runKernel,
 * solved as the 8x8 system with h22 = 1 by Gaussian elimination with
 * partial pivoting (first max on ties).  Exactly determined for 4 points,
 * so it is the same model as OpenCV's LtL null vector up to rounding. */
ORC_API int orc_hom_minimal(const float *sx, const float *sy, const float *dx, const float *dy,
                            const int32_t idx[4], double H[9]) {
    hnorm nm;
    if (!hom_norm(sx, sy, dx, dy, idx, 4, &nm)) return 0;
    double A[8][9];
    for (int i = 0; i < 4; ++i) {
        int p = idx[i];
        double x = (dx[p] - nm.cmx) * nm.smx, y = (dy[p] - nm.cmy) * nm.smy;
        double X = (sx[p] - nm.cMx) * nm.sMx, Y = (sy[p] - nm.cMy) * nm.sMy;
        double *r0 = A[2 * i], *r1 = A[2 * i + 1];
        r0[0] = X; r0[1] = Y; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0; r0[6] = -x * X; r0[7] = -x * Y; r0[8] = x;
        r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = X; r1[4] = Y; r1[5] = 1; r1[6] = -y * X; r1[7] = -y * Y; r1[8] = y;
    }
    for (int k = 0; k < 8; ++k) {
        int piv = k;
        double pm = fabs(A[k][k]);
        for (int r = k + 1; r < 8; ++r) {
            double v = fabs(A[r][k]);
            if (v > pm) { pm = v; piv = r; }
        }
        if (!(pm > 1e-10)) return 0;
        if (piv != k)
            for (int j = 0; j < 9; ++j) { double tmp = A[k][j]; A[k][j] = A[piv][j]; A[piv][j] = tmp; }
        for (int r = k + 1; r < 8; ++r) {
            double f = A[r][k] / A[k][k];
            for (int j = k + 1; j < 9; ++j) A[r][j] = A[r][j] - f * A[k][j];
        }
    }
    double h[8];
    for (int k = 7; k >= 0; --k) {
        double s = A[k][8];
        for (int j = k + 1; j < 8; ++j) s = s - A[k][j] * h[j];
        h[k] = s / A[k][k];
    }
    double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    hom_denorm(&nm, Hn, H);
    for (int k = 0; k < 9; ++k) if (!isfinite(H[k])) return 0;
    return 1;
}

/* HomographyEstimatorCallback::computeError, all in f32 */
ORC_API float orc_hom_err(const double H[9], float x, float y, float u, float v) {
    float h0 = (float)H[0], h1 = (float)H[1], h2 = (float)H[2], h3 = (float)H[3];
    float h4 = (float)H[4], h5 = (float)H[5], h6 = (float)H[6], h7 = (float)H[7];
    float ww = 1.f / (h6 * x + h7 * y + 1.f);
    float ex = (h0 * x + h1 * y + h2) * ww - u;
    float ey = (h3 * x + h4 * y + h5) * ww - v;
    float e1 = ex * ex, e2 = ey * ey;
    return e1 + e2;
}

ORC_API int32_t orc_hom_count(const double H[9], const float *sx, const float *sy, const float *dx, const float *dy,
                              int n, float thr2, uint8_t *mask) {
    int32_t c = 0;
    for (int i = 0; i < n; ++i) {
        int f = orc_hom_err(H, sx[i], sy[i], dx[i], dy[i]) <= thr2;
        if (mask) mask[i] = (uint8_t)f;
        c += f;
    }
    return c;
}

/* ------------------------------------------------------------------------ */
/* Subset generation                                                          */
/* ------------------------------------------------------------------------ */

/* OpenCV getSubset(m1, m2, ms1, ms2, rng, 10000) with checkPartialSubsets ==
 * false, run sequentially for H hypotheses sharing one MWC state.  For the
 * homography model the checkSubset test is applied (pass sx..dy), for PnP
 * pass NULL (PnPRansacCallback has no checkSubset).  status[h] = 1 found,
 * -1 not found (the RANSAC loop then stops). */
ORC_API void orc_mwc_subsets(uint64_t *state, int n, int s, int64_t H, const float *sx, const float *sy,
                             const float *dx, const float *dy, int32_t *out, int8_t *status) {
    if (n < s) { /* run() returns no model when count < modelPoints: nothing is drawn */
        for (int64_t h = 0; h < H; ++h) status[h] = -1;
        return;
    }
    for (int64_t h = 0; h < H; ++h) {
        int32_t *idx = out + s * h;
        int found = 0;
        for (int att = 0; att < ORC_MAX_SUBSET_ATTEMPTS; ++att) {
            for (int i = 0; i < s; ++i) {
                int r;
                for (;;) {
                    r = orc_mwc_uniform(state, 0, n);
                    int dup = 0;
                    for (int j = 0; j < i; ++j) dup |= (idx[j] == r);
                    if (!dup) break;
                }
                idx[i] = r;
            }
            if (sx && !orc_hom_check_subset(sx, sy, dx, dy, idx)) continue;
            found = 1;
            break;
        }
        status[h] = found ? 1 : -1;
        if (!found) {
            for (int64_t g = h + 1; g < H; ++g) status[g] = -1;
            return;
        }
    }
}

/* Philox subsets for the homography model: attempts until checkSubset
 * passes, all drawn from the hypothesis' own stream. */
static int philox_hom_subset(orc_stream *st, int n, const float *sx, const float *sy, const float *dx,
                             const float *dy, int32_t idx[4]) {
    for (int att = 0; att < ORC_MAX_SUBSET_ATTEMPTS; ++att) {
        if (stream_subset(st, n, 4, idx) < 0) return -1;
        if (orc_hom_check_subset(sx, sy, dx, dy, idx)) return 0;
    }
    return -1;
}

/* ------------------------------------------------------------------------ */
/* Per-hypothesis evaluation (what the GPU computes): status, count, model.  */
/* subsets == NULL -> Philox sampler (seed, problem, hyp0 + h).              */
/* models: H x 16 doubles (R 9, t 3, pad); may be NULL.                      */
/* ------------------------------------------------------------------------ */
ORC_API int orc_pnp_epnp(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                         const uint8_t *mask, int n, const double cam[4], double R_out[9], double t_out[3]);

/* The minimal solver of solvePnPRansac's default SOLVEPNP_ITERATIVE mode (OpenCV solvepnp.cpp:
 * model_points = 5, ransac_kernel_method = SOLVEPNP_EPNP; PnPRansacCallback::runKernel): EPnP on
 * the 5 sampled points, in sample order, every point in (the frame centred on the first). */
ORC_API int orc_pnp_minimal_epnp5(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                  const int32_t idx[5], const double cam[4], double R[9], double t[3]) {
    if (g_seq == ORC_SEQ_CV) return orc_cv_epnp(X, Y, Z, U, V, idx, 5, cam, R, t);
    float x[5], y[5], z[5], u[5], v[5];
    uint8_t m[5] = {1, 1, 1, 1, 1};
    for (int j = 0; j < 5; ++j) {
        x[j] = X[idx[j]]; y[j] = Y[idx[j]]; z[j] = Z[idx[j]]; u[j] = U[idx[j]]; v[j] = V[idx[j]];
    }
    return orc_pnp_epnp(x, y, z, u, v, m, 5, cam, R, t);
}

ORC_API void orc_rvec_roundtrip(double R[9]);

/* k = 4: P3P on 4-point samples (SOLVEPNP_P3P); k = 5: EPnP on 5-point samples (the default).
 * subsets: H x k indices (the OpenCV sampler), else Philox subsets of size k.
 * rvec_rt: each model's R -> Rodrigues(Rodrigues(R)) before it is counted (OpenCV keeps the
 * model as rvec; RSAC_F_RVEC_ROUNDTRIP). */
ORC_API void orc_pnp_hypotheses_k(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                  int n, const double cam[4], float thr2, uint64_t seed, uint32_t problem,
                                  int64_t hyp0, int64_t H, int k, const int32_t *subsets, const int8_t *sub_status,
                                  int32_t *counts, int8_t *status, double *models, int rvec_rt) {
    for (int64_t h = 0; h < H; ++h) {
        int32_t idx[5];
        double R[9] = {0}, t[3] = {0};
        int8_t st;
        if (subsets) {
            st = sub_status ? sub_status[h] : 1;
            memcpy(idx, subsets + k * h, sizeof(int32_t) * k);
        } else {
            st = orc_philox_subset(seed, problem, (uint64_t)(hyp0 + h), n, k, idx) < 0 ? -1 : 1;
        }
        int32_t c = 0;
        if (st > 0) {
            st = (int8_t)(k == 5 ? orc_pnp_minimal_epnp5(X, Y, Z, U, V, idx, cam, R, t)
                                 : orc_pnp_minimal(X, Y, Z, U, V, idx, cam, R, t));
            if (st && rvec_rt) orc_rvec_roundtrip(R);
            if (st) c = orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, NULL);
        }
        counts[h] = c;
        status[h] = st;
        if (models) {
            double *m = models + 16 * h;
            memset(m, 0, 16 * sizeof(double));
            memcpy(m, R, 9 * sizeof(double));
            memcpy(m + 9, t, 3 * sizeof(double));
        }
    }
}

ORC_API void orc_pnp_hypotheses(const float *X, const float *Y, const float *Z, const float *U, const float *V, int n,
                                const double cam[4], float thr2, uint64_t seed, uint32_t problem, int64_t hyp0,
                                int64_t H, const int32_t *subsets, const int8_t *sub_status, int32_t *counts,
                                int8_t *status, double *models) {
    orc_pnp_hypotheses_k(X, Y, Z, U, V, n, cam, thr2, seed, problem, hyp0, H, 4, subsets, sub_status, counts, status,
                         models, 0);
}

ORC_API void orc_hom_hypotheses(const float *sx, const float *sy, const float *dx, const float *dy, int n,
                                float thr2, uint64_t seed, uint32_t problem, int64_t hyp0, int64_t H,
                                const int32_t *subsets, const int8_t *sub_status, int32_t *counts, int8_t *status,
                                double *models) {
    for (int64_t h = 0; h < H; ++h) {
        int32_t idx[4];
        double Hm[9] = {0};
        int8_t st;
        if (subsets) {
            st = sub_status ? sub_status[h] : 1;
            memcpy(idx, subsets + 4 * h, sizeof(idx));
        } else {
            orc_stream s;
            stream_init(&s, seed, problem, (uint64_t)(hyp0 + h));
            st = (n >= 4 && philox_hom_subset(&s, n, sx, sy, dx, dy, idx) == 0) ? 1 : -1;
        }
        int32_t c = 0;
        if (st > 0) {
            st = (int8_t)orc_hom_minimal(sx, sy, dx, dy, idx, Hm);
            if (st) c = orc_hom_count(Hm, sx, sy, dx, dy, n, thr2, NULL);
        }
        counts[h] = c;
        status[h] = st;
        if (models) {
            double *m = models + 16 * h;
            memset(m, 0, 16 * sizeof(double));
            memcpy(m, Hm, 9 * sizeof(double));
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Rodrigues (cv::Rodrigues, main_v1.py:895; [OpenCV 4.x, unvendored]        */
/* calibration.cpp cvRodrigues2).  The steps of cvRodrigues2 -- checkRange   */
/* (-100, 100), the SVD orthogonalisation R = U Vt, the angle from the       */
/* antisymmetric part, the theta ~ pi branch -- in + - * / sqrt only, so the */
/* GPU (rsac_math.h rodrigues_*_det) gives the same bits: acos via fdlibm's  */
/* reduction and the asin series (26 exactly rounded coefficients, |x|<=1/2),*/
/* sin / cos via a 2-part pi/2 reduction and Taylor polynomials to y^22,     */
/* U Vt as the polar factor by Newton's iteration X <- (X + X^-T)/2.          */
/* ------------------------------------------------------------------------ */
static const double RD_PIO2_HI = 0x1.921fb54442d18p+0, RD_PIO2_LO = 0x1.1a62633145c07p-54;
static const double RD_PIO2_A = 0x1.921fb544p+0, RD_PIO2_B = 0x1.0b4611a626331p-34;
static const double RD_2_OVER_PI = 0x1.45f306dc9c883p-1;
/* (2k)! / (4^k (k!)^2 (2k+1)), k = 1..26: asin(x) = x + x z Q(z), z = x^2 */
static const double RD_ASIN[26] = {
    0x1.5555555555555p-3, 0x1.3333333333333p-4, 0x1.6db6db6db6db7p-5, 0x1.f1c71c71c71c7p-6, 0x1.6e8ba2e8ba2e9p-6,
    0x1.1c4ec4ec4ec4fp-6, 0x1.c99999999999ap-7, 0x1.7a87878787878p-7, 0x1.3fde50d79435ep-7, 0x1.12ef3cf3cf3cfp-7,
    0x1.df3bd37a6f4dfp-8, 0x1.a6863d70a3d71p-8, 0x1.782dda12f684cp-8, 0x1.51ba308d3dcb1p-8, 0x1.31683bdef7bdfp-8,
    0x1.15ee9d45d1746p-8, 0x1.fcaf8fb6db6dbp-9, 0x1.d3d2a8e0dd67dp-9, 0x1.b026f57b13b14p-9, 0x1.90cb77f60c7cep-9,
    0x1.750de64d7d05fp-9, 0x1.5c5f56efaaaabp-9, 0x1.464c0950f7d47p-9, 0x1.3275586c5f2f0p-9, 0x1.208d3570ae5a6p-9,
    0x1.1052bc5fa960ap-9};
/* (-1)^k / (2k+1)!, k = 1..10 and (-1)^k / (2k)!, k = 2..11 */
static const double RD_SIN[10] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13,
                                  0x1.71de3a556c734p-19, -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                                  -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49, -0x1.2f49b46814157p-57,
                                  0x1.71b8ef6dcf572p-66};
static const double RD_COS[10] = {0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
                                  -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37,
                                  0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53, 0x1.e542ba4020225p-62,
                                  -0x1.0ce396db7f853p-70};

static double rd_horner(const double *c, int n, double z) {
    double p = c[n - 1];
    for (int i = n - 2; i >= 0; --i) p = p * z + c[i];
    return p;
}

ORC_API double orc_rd_acos(double x) {
    if (x >= 1.0) return 0.0;
    if (x <= -1.0) return 2.0 * RD_PIO2_HI;
    double ax = fabs(x);
    if (ax <= 0.5) {
        double z = x * x;
        double r = x * z * rd_horner(RD_ASIN, 26, z);
        return RD_PIO2_HI - (x - (RD_PIO2_LO - r));
    }
    double z = (1.0 - ax) * 0.5;
    double s = sqrt(z);
    double w = s * z * rd_horner(RD_ASIN, 26, z);
    if (x > 0.0) return 2.0 * (s + w);
    return 2.0 * (RD_PIO2_HI - (s + (w - RD_PIO2_LO)));
}

ORC_API void orc_rd_sincos(double th, double *sn, double *cs) {
    double fn = (double)(int64_t)(th * RD_2_OVER_PI + 0.5);
    int n = (int)((int64_t)fn & 3);
    double y = (th - fn * RD_PIO2_A) - fn * RD_PIO2_B;
    double z = y * y;
    double ps = RD_SIN[9], pc = RD_COS[9];
    for (int i = 8; i >= 0; --i) {
        ps = ps * z + RD_SIN[i];
        pc = pc * z + RD_COS[i];
    }
    double s = y + y * z * ps;
    double hz = 0.5 * z, w = 1.0 - hz;
    double c = w + (((1.0 - w) - hz) + z * z * pc);
    *sn = n == 0 ? s : n == 1 ? c : n == 2 ? -s : -c;
    *cs = n == 0 ? c : n == 1 ? -s : n == 2 ? -c : s;
}

/* polar factor of X (OpenCV: U Vt of SVD::compute): Newton steps until no element moves by more
 * than 1e-15, at most 30; singular X unchanged */
static void rd_polar(double X[9]) {
    for (int it = 0; it < 30; ++it) {
        double cf[9];
        cf[0] = X[4] * X[8] - X[5] * X[7];
        cf[1] = X[5] * X[6] - X[3] * X[8];
        cf[2] = X[3] * X[7] - X[4] * X[6];
        cf[3] = X[2] * X[7] - X[1] * X[8];
        cf[4] = X[0] * X[8] - X[2] * X[6];
        cf[5] = X[1] * X[6] - X[0] * X[7];
        cf[6] = X[1] * X[5] - X[2] * X[4];
        cf[7] = X[2] * X[3] - X[0] * X[5];
        cf[8] = X[0] * X[4] - X[1] * X[3];
        double det = X[0] * cf[0] + X[1] * cf[1] + X[2] * cf[2];
        if (!(fabs(det) > 1e-30) || !isfinite(det)) return;
        double id = 1.0 / det, mv = 0.0;
        for (int k = 0; k < 9; ++k) {
            double nx = 0.5 * (X[k] + cf[k] * id);
            double d = fabs(nx - X[k]);
            mv = d > mv ? d : mv;
            X[k] = nx;
        }
        if (!(mv > 1e-15)) return;
    }
}

ORC_API void orc_rodrigues_v2m(const double r[3], double R[9]) {
    if (g_seq == ORC_SEQ_CV) {
        orc_cv_rodrigues_v2m(r, R);
        return;
    }
    double th = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th < DBL_EPSILON) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double s, c;
    orc_rd_sincos(th, &s, &c);
    double c1 = 1. - c, it = 1. / th;
    double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    R[0] = c + c1 * x * x;     R[1] = c1 * x * y - s * z; R[2] = c1 * x * z + s * y;
    R[3] = c1 * x * y + s * z; R[4] = c + c1 * y * y;     R[5] = c1 * y * z - s * x;
    R[6] = c1 * x * z - s * y; R[7] = c1 * y * z + s * x; R[8] = c + c1 * z * z;
}

ORC_API void orc_rodrigues_m2v(const double Rin[9], double r[3]) {
    if (g_seq == ORC_SEQ_CV) {
        orc_cv_rodrigues_m2v(Rin, r);
        return;
    }
    double R[9];
    for (int k = 0; k < 9; ++k) {
        if (!(fabs(Rin[k]) <= 100.0)) { r[0] = r[1] = r[2] = 0; return; }  /* checkRange */
        R[k] = Rin[k];
    }
    rd_polar(R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double th = orc_rd_acos(c);
    if (s < 1e-5) {
        if (c > 0) { r[0] = r[1] = r[2] = 0; return; }
        double t;
        t = (R[0] + 1) * 0.5; rx = sqrt(t > 0 ? t : 0);
        t = (R[4] + 1) * 0.5; ry = sqrt(t > 0 ? t : 0) * (R[1] < 0 ? -1. : 1.);
        t = (R[8] + 1) * 0.5; rz = sqrt(t > 0 ? t : 0) * (R[2] < 0 ? -1. : 1.);
        if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
        th = th / sqrt(rx * rx + ry * ry + rz * rz);
        r[0] = rx * th; r[1] = ry * th; r[2] = rz * th;
        return;
    }
    double vth = 1 / (2 * s) * th;
    r[0] = rx * vth; r[1] = ry * vth; r[2] = rz * vth;
}

/* PnPRansacCallback stores a minimal model as (rvec, tvec) and computeError projects through
 * Rodrigues(rvec) (solvepnp.cpp; main_v1.py:497, testpro-K.py:72): the rotation it scores is
 * Rodrigues(Rodrigues(R)) (RSAC_F_RVEC_ROUNDTRIP) */
ORC_API void orc_rvec_roundtrip(double R[9]) {
    if (g_seq == ORC_SEQ_CV) {
        orc_cv_rvec_roundtrip(R);
        return;
    }
    double rv[3];
    orc_rodrigues_m2v(R, rv);
    orc_rodrigues_v2m(rv, R);
}

/* ------------------------------------------------------------------------ */
/* Fundamental matrix RANSAC (BASELINE.json configs[3]).  The reference has  */
/* no implementation ("parity against the restatement only"), */
/* so this block defines the semantics the HIP path reproduces bit for bit:  */
/* Philox 8-point samples, Hartley-normalised 8-point DLT with Gauss-Jordan  */
/* full pivoting, rank 2 via the smallest right-singular direction (Jacobi   */
/* on F^T F), unit Frobenius norm; Sampson test r^2 <= T (a^2+b^2+a'^2+b'^2) */
/* in f64 with explicit fma; RANSACUpdateNumIters with 8 model points.       */
/* ------------------------------------------------------------------------ */
static int fm_norm8(const float *x, const float *y, double *cx, double *cy, double *s) {
    double ax = 0.0, ay = 0.0;
    for (int i = 0; i < 8; ++i) { ax = ax + (double)x[i]; ay = ay + (double)y[i]; }
    ax = ax * 0.125; ay = ay * 0.125;
    double d = 0.0;
    for (int i = 0; i < 8; ++i) {
        double dx = (double)x[i] - ax, dy = (double)y[i] - ay;
        d = d + sqrt(dx * dx + dy * dy);
    }
    d = d * 0.125;
    if (!(d > 1e-300)) return 0;
    *cx = ax; *cy = ay; *s = 1.4142135623730951 / d;
    return 1;
}

static void sym3_min_evec(double A[9], double v[3]) {
    double V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 12; ++sweep) {
        double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        double dia = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (off <= 1e-34 * dia || off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double apq = A[p * 3 + q];
                if (fabs(apq) < 1e-300) continue;
                double theta = (A[q * 3 + q] - A[p * 3 + p]) / (2.0 * apq);
                double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(tt * tt + 1.0), sn = tt * c;
                for (int k = 0; k < 3; ++k) {
                    double akp = A[k * 3 + p], akq = A[k * 3 + q];
                    A[k * 3 + p] = c * akp - sn * akq;
                    A[k * 3 + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    double apk = A[p * 3 + k], aqk = A[q * 3 + k];
                    A[p * 3 + k] = c * apk - sn * aqk;
                    A[q * 3 + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
                    V[k * 3 + p] = c * vkp - sn * vkq;
                    V[k * 3 + q] = sn * vkp + c * vkq;
                }
            }
    }
    int mi = 0;
    if (A[4] < A[mi * 4]) mi = 1;
    if (A[8] < A[mi * 4]) mi = 2;
    v[0] = V[mi]; v[1] = V[3 + mi]; v[2] = V[6 + mi];
}

ORC_API int orc_fm_minimal8(const float *x1, const float *y1, const float *x2, const float *y2, double F[9]) {
    double c1x, c1y, s1, c2x, c2y, s2;
    if (!fm_norm8(x1, y1, &c1x, &c1y, &s1) || !fm_norm8(x2, y2, &c2x, &c2y, &s2)) return 0;
    double A[8][9], amax = 0.0;
    for (int i = 0; i < 8; ++i) {
        double u1 = ((double)x1[i] - c1x) * s1, v1 = ((double)y1[i] - c1y) * s1;
        double u2 = ((double)x2[i] - c2x) * s2, v2 = ((double)y2[i] - c2y) * s2;
        A[i][0] = u2 * u1; A[i][1] = u2 * v1; A[i][2] = u2;
        A[i][3] = v2 * u1; A[i][4] = v2 * v1; A[i][5] = v2;
        A[i][6] = u1;      A[i][7] = v1;      A[i][8] = 1.0;
        for (int j = 0; j < 9; ++j) amax = fabs(A[i][j]) > amax ? fabs(A[i][j]) : amax;
    }
    int perm[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
    for (int r = 0; r < 8; ++r) {
        int pr = r, pc = r;
        double best = -1.0;
        for (int i = r; i < 8; ++i)
            for (int j = r; j < 9; ++j)
                if (fabs(A[i][j]) > best) { best = fabs(A[i][j]); pr = i; pc = j; }
        if (!(best > 1e-12 * amax)) return 0;
        if (pr != r)
            for (int j = 0; j < 9; ++j) { double t = A[r][j]; A[r][j] = A[pr][j]; A[pr][j] = t; }
        if (pc != r) {
            for (int i = 0; i < 8; ++i) { double t = A[i][r]; A[i][r] = A[i][pc]; A[i][pc] = t; }
            int tp = perm[r]; perm[r] = perm[pc]; perm[pc] = tp;
        }
        double ip = 1.0 / A[r][r];
        for (int i = 0; i < 8; ++i) {
            if (i == r) continue;
            double f = A[i][r] * ip;
            if (f == 0.0) continue;
            for (int j = r; j < 9; ++j) A[i][j] = A[i][j] - f * A[r][j];
        }
    }
    double f[9];
    f[perm[8]] = 1.0;
    for (int r = 0; r < 8; ++r) f[perm[r]] = -A[r][8] / A[r][r];
    double M[9], v[3], Fr[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = f[i] * f[j] + f[3 + i] * f[3 + j] + f[6 + i] * f[6 + j];
    sym3_min_evec(M, v);
    for (int i = 0; i < 3; ++i) {
        double w = f[3 * i] * v[0] + f[3 * i + 1] * v[1] + f[3 * i + 2] * v[2];
        for (int j = 0; j < 3; ++j) Fr[3 * i + j] = f[3 * i + j] - w * v[j];
    }
    double T1[9] = {s1, 0.0, -s1 * c1x, 0.0, s1, -s1 * c1y, 0.0, 0.0, 1.0};
    double T2t[9] = {s2, 0.0, 0.0, 0.0, s2, 0.0, -s2 * c2x, -s2 * c2y, 1.0};
    double tmp[9];
    mat3mul(T2t, Fr, tmp);
    mat3mul(tmp, T1, F);
    double nrm = 0.0;
    for (int k = 0; k < 9; ++k) nrm = nrm + F[k] * F[k];
    if (!(nrm > 1e-300) || !isfinite(nrm)) return 0;
    double in = 1.0 / sqrt(nrm);
    for (int k = 0; k < 9; ++k) F[k] = F[k] * in;
    return 1;
}

ORC_API int orc_fm_inlier(const double F[9], double x1, double y1, double x2, double y2, double T) {
    double a = fma(F[0], x1, fma(F[1], y1, F[2]));
    double b = fma(F[3], x1, fma(F[4], y1, F[5]));
    double c = fma(F[6], x1, fma(F[7], y1, F[8]));
    double a2 = fma(F[0], x2, fma(F[3], y2, F[6]));
    double b2 = fma(F[1], x2, fma(F[4], y2, F[7]));
    double r = fma(x2, a, fma(y2, b, c));
    double den = fma(a, a, fma(b, b, fma(a2, a2, b2 * b2)));
    return r * r <= T * den;
}

ORC_API int32_t orc_fm_count(const double F[9], const float *x1, const float *y1, const float *x2, const float *y2,
                             int n, float thr2, uint8_t *mask) {
    int32_t c = 0;
    for (int i = 0; i < n; ++i) {
        int f = orc_fm_inlier(F, x1[i], y1[i], x2[i], y2[i], (double)thr2);
        if (mask) mask[i] = (uint8_t)f;
        c += f;
    }
    return c;
}

/* hypotheses [hyp0, hyp0+H): Philox 8-subsets, status 1 model / 0 degenerate / -1 no subset */
ORC_API void orc_fm_hypotheses(const float *x1, const float *y1, const float *x2, const float *y2, int n, float thr2,
                               uint64_t seed, int64_t hyp0, int64_t H, int32_t *counts, int8_t *status,
                               double *models) {
    for (int64_t h = 0; h < H; ++h) {
        int32_t idx[8];
        double F[9] = {0};
        int8_t st = -1;
        if (orc_philox_subset(seed, 0, (uint64_t)(hyp0 + h), n, 8, idx) == 0) {
            float a[8], b[8], c[8], d[8];
            for (int j = 0; j < 8; ++j) { a[j] = x1[idx[j]]; b[j] = y1[idx[j]]; c[j] = x2[idx[j]]; d[j] = y2[idx[j]]; }
            st = orc_fm_minimal8(a, b, c, d, F) ? 1 : 0;
            if (st == 0) memset(F, 0, sizeof F);
        }
        status[h] = st;
        counts[h] = st > 0 ? orc_fm_count(F, x1, y1, x2, y2, n, thr2, NULL) : 0;
        if (models) {
            memset(models + 16 * h, 0, 16 * sizeof(double));
            memcpy(models + 16 * h, F, sizeof F);
            models[16 * h + 12] = st > 0 ? 1.0 : 0.0;
        }
    }
}

/* orc_fm_hypotheses over `threads` host threads (OpenMP, hypotheses in chunks of 16): the C4 CPU
 * baseline's multi-core leg; every hypothesis' result is the single-thread one. */
ORC_API void orc_fm_hypotheses_mt(const float *x1, const float *y1, const float *x2, const float *y2, int n,
                                  float thr2, uint64_t seed, int64_t hyp0, int64_t H, int32_t *counts, int8_t *status,
                                  int threads) {
#pragma omp parallel for num_threads(threads) schedule(dynamic, 16)
    for (int64_t h = 0; h < H; ++h)
        orc_fm_hypotheses(x1, y1, x2, y2, n, thr2, seed, hyp0 + h, 1, counts + h, status + h, NULL);
}

ORC_API int64_t orc_fm_ransac(const float *x1, const float *y1, const float *x2, const float *y2, int n, double thr,
                              double confidence, int max_iters, uint64_t seed, double Fout[9], uint8_t *mask,
                              int32_t *n_inliers, int64_t *iters_used) {
    int64_t H = max_iters > 1 ? max_iters : 1;
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * H);
    int8_t *status = (int8_t *)malloc(H);
    double *models = (double *)malloc(sizeof(double) * 16 * H);
    float thr2 = orc_thr2(thr);
    orc_fm_hypotheses(x1, y1, x2, y2, n, thr2, seed, 0, H, counts, status, models);
    int32_t good = 0;
    int64_t best = orc_scan(counts, status, H, n, 8, confidence, max_iters, &good, iters_used);
    if (best >= 0) {
        memcpy(Fout, models + 16 * best, 9 * sizeof(double));
        orc_fm_count(Fout, x1, y1, x2, y2, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = good;
    free(counts); free(status); free(models);
    return best;
}

/* ------------------------------------------------------------------------ */
/* Final refits (non-minimal solve on the RANSAC inliers).                   */
/* ------------------------------------------------------------------------ */

/* Pose LM (final solvePnP / solvePnPRefineLM, main_v1.py:508-509,
 * testpro-K.py:122-125): increments d = (rotation 3, translation 3), R <- Cay(d) R
 * (Cayley map), damping lam*diag(J^T J), lam x0.1 on success / x10 on failure,
 * at most 20 iterations, stop when the relative cost decrease < 1e-12 or
 * |d| < FLT_EPSILON (|t| + 1) (CvLevMarq's step criterion of solvePnP).
 * The pose is refined in the frame centred on the first point c (t' = R c + t).
 * Sums use the GPU kernel's block-compacted order: nb = lm_blocks(n) contiguous ranges of
 * lm_chunk(n) points (one range up to 4096 points, then ranges of ~1024, at most 64); the
 * masked points of range b, ascending, dealt round-robin to slots b*512 + p%512; per-slot
 * sums in order, a 64-lane butterfly per wave of 64 slots (x += x[lane ^ o], o = 32..1),
 * each range's 8 wave sums left to right, then the nb range sums left to right -- so the
 * HIP kernel k_pnp_refine (one block per range, one exchanged sum per term) reproduces this
 * bit for bit. */
#define LM_THREADS 512
#define LM_MAX_BLOCKS 64
#define LM_ONE_BLOCK 4096
#define LM_BLOCK_POINTS 1024
#define LM_TERMS 27

static int lm_blocks(int n) {
    if (n <= LM_ONE_BLOCK) return 1;
    int nb = (n + LM_BLOCK_POINTS - 1) / LM_BLOCK_POINTS;
    return nb < LM_MAX_BLOCKS ? nb : LM_MAX_BLOCKS;
}
static int lm_chunk(int n) {
    int nb = lm_blocks(n);
    return (int)(((int64_t)n + nb - 1) / nb);
}

typedef struct { const float *X, *Y, *Z, *U, *V; const uint8_t *mask; int n; double cam[4]; double *part; double c[3]; } lmctx;

static void lm_point(const lmctx *c, const double *R, const double *t, int i, double *acc) {
    double Xd = (double)c->X[i] - c->c[0], Yd = (double)c->Y[i] - c->c[1], Zd = (double)c->Z[i] - c->c[2];
    double u = c->U[i], v = c->V[i];
    /* dot products and accumulations as fma chains (rsac_math.h pnp_lm_point, r05) */
    double px = fma(R[2], Zd, fma(R[1], Yd, R[0] * Xd));
    double py = fma(R[5], Zd, fma(R[4], Yd, R[3] * Xd));
    double pz = fma(R[8], Zd, fma(R[7], Yd, R[6] * Xd));
    double cx = px + t[0], cy = py + t[1], cz = pz + t[2];
    double iz = 1.0 / cz;
    double ru = c->cam[0] * cx * iz + c->cam[2] - u;
    double rv = c->cam[1] * cy * iz + c->cam[3] - v;
    double dux = c->cam[0] * iz, duz = -c->cam[0] * cx * iz * iz;
    double dvy = c->cam[1] * iz, dvz = -c->cam[1] * cy * iz * iz;
    double Ju[6], Jv[6];
    Ju[0] = duz * py;             Ju[1] = dux * pz - duz * px; Ju[2] = -dux * py;
    Jv[0] = -dvy * pz + dvz * py; Jv[1] = -dvz * px;           Jv[2] = dvy * px;
    Ju[3] = dux; Ju[4] = 0; Ju[5] = duz;
    Jv[3] = 0; Jv[4] = dvy; Jv[5] = dvz;
    int q = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = 0; b <= a; ++b, ++q) acc[q] = fma(Jv[a], Jv[b], fma(Ju[a], Ju[b], acc[q]));
    for (int a = 0; a < 6; ++a) acc[21 + a] = fma(Jv[a], rv, fma(Ju[a], ru, acc[21 + a]));
}

static double lm_cost_point(const lmctx *c, const double *R, const double *t, int i) {
    double Xd = (double)c->X[i] - c->c[0], Yd = (double)c->Y[i] - c->c[1], Zd = (double)c->Z[i] - c->c[2];
    double u = c->U[i], v = c->V[i];
    double x = fma(R[2], Zd, fma(R[1], Yd, R[0] * Xd)) + t[0];
    double y = fma(R[5], Zd, fma(R[4], Yd, R[3] * Xd)) + t[1];
    double z = fma(R[8], Zd, fma(R[7], Yd, R[6] * Xd)) + t[2];
    double iz = 1.0 / z;
    double ru = c->cam[0] * x * iz + c->cam[2] - u;
    double rv = c->cam[1] * y * iz + c->cam[3] - v;
    return fma(rv, rv, ru * ru);
}

/* nv = LM_TERMS: normal equations; nv = 1: cost */
static void lm_reduce(lmctx *c, const double *R, const double *t, int nv, double *out) {
    double *part = c->part;
    const int nb = lm_blocks(c->n), C = lm_chunk(c->n), S = nb * LM_THREADS;
    for (int q = 0; q < S * nv; ++q) part[q] = 0.0;
    for (int b = 0; b < nb; ++b) {
        int hi = (int64_t)(b + 1) * C < c->n ? (b + 1) * C : c->n, p = 0;
        for (int i = b * C; i < hi; ++i) {
            if (!c->mask[i]) continue;
            const int slot = b * LM_THREADS + p++ % LM_THREADS;
            if (nv == 1) part[slot] += lm_cost_point(c, R, t, i);
            else lm_point(c, R, t, i, part + slot * nv);
        }
    }
    double v[64], w[64];
    for (int b = 0; b < nb; ++b)
        for (int q = 0; q < nv; ++q) {
            double bsum = 0.0;
            for (int wv = 0; wv < LM_THREADS / 64; ++wv) {
                for (int l = 0; l < 64; ++l) v[l] = part[((b * (LM_THREADS / 64) + wv) * 64 + l) * nv + q];
                for (int o = 32; o > 0; o >>= 1) {
                    for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ o];
                    for (int l = 0; l < 64; ++l) v[l] = w[l];
                }
                bsum = wv == 0 ? v[0] : bsum + v[0]; /* a range's 8 wave sums left to right */
            }
            out[q] = b == 0 ? bsum : out[q] + bsum; /* range sums left to right */
        }
}

/* (A + lam diag(A)) x = b, A 6x6 SPD, Cholesky; divisions by a pivot are multiplications
 * by its reciprocal */
static int chol6(const double *A, double lam, const double *b, double *x) {
    double L[36], y[6], inv[6];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = A[i * 6 + j];
            if (i == j) s = fma(lam, A[i * 6 + i], s);
            for (int k = 0; k < j; ++k) s = fma(-L[i * 6 + k], L[j * 6 + k], s);  /* fused (r05) */
            if (i == j) {
                if (!(s > 0)) return 0;
                L[i * 6 + i] = sqrt(s);
                inv[i] = 1.0 / L[i * 6 + i];
            } else {
                L[i * 6 + j] = s * inv[j];
            }
        }
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s = fma(-L[i * 6 + k], y[k], s);
        y[i] = s * inv[i];
    }
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int k = i + 1; k < 6; ++k) s = fma(-L[k * 6 + i], x[k], s);
        x[i] = s * inv[i];
    }
    return 1;
}

/* Rn = Cay(d) R: the rotation of the quaternion (1, d/2) */
static void cayley(const double *d, const double *R, double *Rn) {
    double w0 = 0.5 * d[0], w1 = 0.5 * d[1], w2 = 0.5 * d[2];
    double a = w0 * w0, b = w1 * w1, c = w2 * w2;
    double is = 1.0 / (1.0 + a + b + c);
    double Q[9];
    Q[0] = (1.0 + a - b - c) * is;       Q[1] = 2.0 * (w0 * w1 - w2) * is; Q[2] = 2.0 * (w0 * w2 + w1) * is;
    Q[3] = 2.0 * (w0 * w1 + w2) * is;    Q[4] = (1.0 - a + b - c) * is;   Q[5] = 2.0 * (w1 * w2 - w0) * is;
    Q[6] = 2.0 * (w0 * w2 - w1) * is;    Q[7] = 2.0 * (w1 * w2 + w0) * is; Q[8] = (1.0 - a - b + c) * is;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rn[3 * i + j] = Q[3 * i] * R[j] + Q[3 * i + 1] * R[3 + j] + Q[3 * i + 2] * R[6 + j];
}

ORC_API int orc_pnp_refine(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                           const uint8_t *mask, int n, const double cam[4], double R[9], double t[3], int max_iter) {
    if (n <= 0) return 0;
    lmctx c = {X, Y, Z, U, V, mask, n, {cam[0], cam[1], cam[2], cam[3]}, NULL, {X[0], Y[0], Z[0]}};
    c.part = (double *)malloc(sizeof(double) * lm_blocks(n) * LM_THREADS * LM_TERMS);
    /* refit frame centred on the first point: t' = R c + t */
    for (int j = 0; j < 3; ++j) t[j] = R[3 * j] * c.c[0] + R[3 * j + 1] * c.c[1] + R[3 * j + 2] * c.c[2] + t[j];
    double lam = 1e-3, cost, acc[LM_TERMS];
    lm_reduce(&c, R, t, 1, &cost);
    int it;
    for (it = 0; it < max_iter; ++it) {
        double A[36], g[6];
        lm_reduce(&c, R, t, LM_TERMS, acc);
        int q = 0;
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b <= a; ++b, ++q) A[a * 6 + b] = A[b * 6 + a] = acc[q];
        for (int a = 0; a < 6; ++a) g[a] = -acc[21 + a];
        int accepted = 0;
        while (!accepted) {
            double d[6], Rn[9], tn[3], cn;
            if (!chol6(A, lam, g, d)) {
                lam *= 10;
                if (lam > 1e10) goto done;
                continue;
            }
            cayley(d, R, Rn);
            for (int j = 0; j < 3; ++j) tn[j] = t[j] + d[3 + j];
            lm_reduce(&c, Rn, tn, 1, &cn);
            if (cn < cost) {
                double rel = (cost - cn) / (cost > 1e-300 ? cost : 1e-300);
                memcpy(R, Rn, sizeof(Rn));
                memcpy(t, tn, sizeof(tn));
                cost = cn;
                lam = lam * 0.1 > 1e-12 ? lam * 0.1 : 1e-12;
                accepted = 1;
                double dd = 0, tt = 0;
                for (int j = 0; j < 6; ++j) dd += d[j] * d[j];
                for (int j = 0; j < 3; ++j) tt += t[j] * t[j];
                if (rel < 1e-12 || sqrt(dd) < 1.1920928955078125e-07 * (sqrt(tt) + 1.0)) { it = it + 1; goto done; }
            } else {
                lam *= 10;
                if (lam > 1e10) goto done;
            }
        }
    }
done:
    for (int j = 0; j < 3; ++j) t[j] = t[j] - (R[3 * j] * c.c[0] + R[3 * j + 1] * c.c[1] + R[3 * j + 2] * c.c[2]);
    free(c.part);
    return it;
}

/* Symmetric eigen-decomposition by cyclic Jacobi (the method of cv::eigen):
 * A (n x n, destroyed) -> eigenvalues on its diagonal, eigenvectors in the
 * columns of V.  Sweeps stop when the off-diagonal mass falls below 1e-32 of
 * the matrix's (relative precision ~1e-16). */
static void jacobi_sym(int n, double *A, double *V) {
    double frob = 0;
    for (int i = 0; i < n * n; ++i) frob += A[i] * A[i];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0;
        for (int i = 0; i < n; ++i)
            for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
        if (off <= 1e-32 * frob || off < 1e-300) break;
        for (int p = 0; p < n; ++p)
            for (int q = p + 1; q < n; ++q) {
                double apq = A[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                double app = A[p * n + p], aqq = A[q * n + q];
                double theta = (aqq - app) / (2.0 * apq);
                double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
                for (int k = 0; k < n; ++k) {
                    double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

/* eigenvector of the smallest eigenvalue (the LS homography of runKernel) */
static void jacobi_min_evec(int n, double *A, double *v_out) {
    double V[81];
    jacobi_sym(n, A, V);
    int mi = 0;
    for (int i = 1; i < n; ++i)
        if (A[i * n + i] < A[mi * n + mi]) mi = i;
    for (int k = 0; k < n; ++k) v_out[k] = V[k * n + mi];
}

/* HomographyRefineCallback::compute (fundam.cpp): residuals proj - dst over the
 * inliers (x2), Jacobian w.r.t. h0..h7 (h8 = 1). */
static void hom_lm_compute(const double *h, const float *sx, const float *sy, const float *dx, const float *dy,
                           const uint8_t *mask, int n, double *r, double *J) {
    int q = 0;
    for (int i = 0; i < n; ++i) {
        if (!mask[i]) continue;
        double Mx = sx[i], My = sy[i];
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        r[2 * q] = xi - dx[i];
        r[2 * q + 1] = yi - dy[i];
        if (J) {
            double *j0 = J + 16 * q, *j1 = j0 + 8;
            j0[0] = Mx * ww; j0[1] = My * ww; j0[2] = ww; j0[3] = j0[4] = j0[5] = 0.;
            j0[6] = -Mx * ww * xi; j0[7] = -My * ww * xi;
            j1[0] = j1[1] = j1[2] = 0.; j1[3] = Mx * ww; j1[4] = My * ww; j1[5] = ww;
            j1[6] = -Mx * ww * yi; j1[7] = -My * ww * yi;
        }
        ++q;
    }
}

/* A = J^T J, v = J^T r (m residuals, 8 parameters) */
static void lm_normal(const double *J, const double *r, int m, double *A, double *v) {
    for (int a = 0; a < 8; ++a) {
        v[a] = 0;
        for (int b = 0; b < 8; ++b) A[a * 8 + b] = 0;
    }
    for (int k = 0; k < m; ++k) {
        const double *jr = J + 8 * k;
        for (int a = 0; a < 8; ++a) {
            v[a] += jr[a] * r[k];
            for (int b = 0; b < 8; ++b) A[a * 8 + b] += jr[a] * jr[b];
        }
    }
}

/* 8x8 symmetric A -> eigenvalues W (diagonal) and vectors V; eigenvalues with
 * |w| <= 8 eps max|w| are zeroed (cv::solve / cv::invert with DECOMP_EIG drop them). */
static void eig8(const double *A, double *W, double *V) {
    memcpy(W, A, 64 * sizeof(double));
    jacobi_sym(8, W, V);
    double wmax = 0;
    for (int i = 0; i < 8; ++i) wmax = fmax(wmax, fabs(W[i * 8 + i]));
    double tol = wmax * 8 * DBL_EPSILON;
    for (int i = 0; i < 8; ++i)
        if (fabs(W[i * 8 + i]) <= tol) W[i * 8 + i] = 0;
}

/* x = A^+ b (cv::solve DECOMP_EIG) */
static void sym_solve_eig(const double *A, const double *b, double *x) {
    double W[64], V[64];
    eig8(A, W, V);
    for (int i = 0; i < 8; ++i) x[i] = 0;
    for (int e = 0; e < 8; ++e) {
        double w = W[e * 8 + e];
        if (w == 0) continue;
        double c = 0;
        for (int k = 0; k < 8; ++k) c += V[k * 8 + e] * b[k];
        c /= w;
        for (int k = 0; k < 8; ++k) x[k] += c * V[k * 8 + e];
    }
}

/* max_a |(A^+)_aa| (cv::invert DECOMP_EIG, diagonal only) */
static double max_diag_pinv(const double *A) {
    double W[64], V[64], maxval = DBL_EPSILON;
    eig8(A, W, V);
    for (int a = 0; a < 8; ++a) {
        double d = 0;
        for (int e = 0; e < 8; ++e)
            if (W[e * 8 + e] != 0) d += V[a * 8 + e] * V[a * 8 + e] / W[e * 8 + e];
        maxval = fmax(maxval, fabs(d));
    }
    return maxval;
}

/* cv::LMSolver::run (levmarq.cpp, OpenCV 4.x LMSolverImpl): damping lambda * diag(A0)
 * with A0 = J^T J at the start, gain-ratio schedule Rlo 0.25 / Rhi 0.75, lambda -> 0
 * below lc, restart from 1/max diag(A^-1); stop after maxIters or when |d|inf <
 * FLT_EPSILON or |r|inf < FLT_EPSILON.  Parameters h0..h7. */
static int hom_lm_opencv(const float *sx, const float *sy, const float *dx, const float *dy, const uint8_t *mask,
                         int n, double H[9], int max_iters) {
    int m = 0;
    for (int i = 0; i < n; ++i) m += mask[i] != 0;
    if (m == 0) return 0;
    m *= 2;
    double *r = (double *)malloc(sizeof(double) * m * 2);
    double *rd = r + m;
    double *J = (double *)malloc(sizeof(double) * m * 8);
    double x[9], xd[9], A[64], Ap[64], v[8], D[8], d[8], tmp[8];
    memcpy(x, H, sizeof x);
    memcpy(xd, H, sizeof xd);
    hom_lm_compute(x, sx, sy, dx, dy, mask, n, r, J);
    double S = 0;
    for (int k = 0; k < m; ++k) S += r[k] * r[k];
    lm_normal(J, r, m, A, v);
    for (int a = 0; a < 8; ++a) D[a] = A[a * 8 + a];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        memcpy(Ap, A, sizeof Ap);
        for (int a = 0; a < 8; ++a) Ap[a * 8 + a] += lambda * D[a];
        sym_solve_eig(Ap, v, d);
        for (int a = 0; a < 8; ++a) xd[a] = x[a] - d[a];
        hom_lm_compute(xd, sx, sy, dx, dy, mask, n, rd, NULL);
        double Sd = 0;
        for (int k = 0; k < m; ++k) Sd += rd[k] * rd[k];
        /* temp_d = 2 v - A d ; dS = d . temp_d */
        double dS = 0;
        for (int a = 0; a < 8; ++a) {
            double ad = 0;
            for (int b = 0; b < 8; ++b) ad += A[a * 8 + b] * d[b];
            tmp[a] = 2 * v[a] - ad;
            dS += d[a] * tmp[a];
        }
        double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int a = 0; a < 8; ++a) t += d[a] * v[a];
            double nu = (Sd - S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = fmin(fmax(nu, 2.), 10.);
            if (lambda == 0) {
                /* lc = 1 / max |diag(A^-1)| */
                double maxval = max_diag_pinv(A);
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            memcpy(x, xd, 8 * sizeof(double));
            hom_lm_compute(x, sx, sy, dx, dy, mask, n, r, J);
            lm_normal(J, r, m, A, v);
        }
        iter++;
        double dinf = 0, rinf = 0;
        for (int a = 0; a < 8; ++a) dinf = fmax(dinf, fabs(d[a]));
        for (int k = 0; k < m; ++k) rinf = fmax(rinf, fabs(r[k]));
        if (!(iter < max_iters && dinf >= FLT_EPSILON && rinf >= FLT_EPSILON)) break;
    }
    memcpy(H, x, 8 * sizeof(double));
    H[8] = 1.0;
    free(r);
    free(J);
    return iter;
}

/* non-minimal refit of findHomography (fundam.cpp): least-squares
 * normalised DLT on the inliers, then 10 LM iterations on the
 * reprojection error (HomographyRefineCallback). */
ORC_API int orc_hom_refine(const float *sx, const float *sy, const float *dx, const float *dy, const uint8_t *mask,
                           int n, double H[9]) {
    int32_t *idx = (int32_t *)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    int m = 0;
    for (int i = 0; i < n; ++i) if (mask[i]) idx[m++] = i;
    if (m < 4) { free(idx); return 0; }
    hnorm nm;
    if (!hom_norm(sx, sy, dx, dy, idx, m, &nm)) { free(idx); return 0; }
    double LtL[81] = {0};
    for (int i = 0; i < m; ++i) {
        int p = idx[i];
        double x = (dx[p] - nm.cmx) * nm.smx, y = (dy[p] - nm.cmy) * nm.smy;
        double X = (sx[p] - nm.cMx) * nm.sMx, Y = (sy[p] - nm.cMy) * nm.sMy;
        double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) LtL[j * 9 + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < j; ++k) LtL[j * 9 + k] = LtL[k * 9 + j];
    free(idx);
    double hv[9];
    jacobi_min_evec(9, LtL, hv);
    hom_denorm(&nm, hv, H);
    hom_lm_opencv(sx, sy, dx, dy, mask, n, H, 10);
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Whole loops (what cv2.solvePnPRansac / cv2.findHomography run).           */
/* sampler: 0 = Philox (seed, problem 0), 1 = OpenCV MWC (seed ignored).     */
/* Returns best hypothesis index (<0: no model); mask = RANSAC-phase mask.   */
/* ------------------------------------------------------------------------ */
/* OpenCV's `model_points == npoints` branch of solvePnPRansac ([OpenCV 4.x, unvendored]
 * modules/calib3d/src/solvepnp.cpp; call sites main_v1.py:497-502, testpro-K.py:72-75): no
 * RANSAC.  model_points is 4 for SOLVEPNP_P3P / AP3P and for npoints == 4 (kernel P3P), 5
 * otherwise (kernel EPnP), so 4 points always, and 5 points under the default flags (k == 5),
 * call solvePnP once with that kernel on all the points in input order; every index is an
 * inlier and there is no final solve.  A failed solve: no model, no inliers.
 * Returns 1 when the branch applies (outputs written), 0 when RANSAC runs. */
static int pnp_direct(const float *X, const float *Y, const float *Z, const float *U, const float *V, int n,
                      const double cam[4], int k, int rvec_rt, double R[9], double t[3], uint8_t *mask,
                      int32_t *n_inliers, int64_t *iters_used, int64_t *best) {
    if (!(n == 4 || (n == 5 && k == 5))) return 0;
    static const int32_t idx[5] = {0, 1, 2, 3, 4};
    const int ok = n == 4 ? orc_pnp_minimal(X, Y, Z, U, V, idx, cam, R, t)
                          : orc_pnp_minimal_epnp5(X, Y, Z, U, V, idx, cam, R, t);
    if (ok && rvec_rt) orc_rvec_roundtrip(R);  /* the pose as Rodrigues(rvec) */
    if (mask) memset(mask, ok ? 1 : 0, n);
    if (n_inliers) *n_inliers = ok ? n : 0;
    if (iters_used) *iters_used = 0;
    *best = ok ? 0 : -1;
    return 1;
}

/* k: the sample size / minimal solver (4 P3P, 5 EPnP), also RANSACUpdateNumIters' model_points */
ORC_API int64_t orc_pnp_ransac_k(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                 int n, const double cam[4], double thr, double confidence, int max_iters,
                                 uint64_t seed, int sampler, int k, double R[9], double t[3], uint8_t *mask,
                                 int32_t *n_inliers, int64_t *iters_used, int rvec_rt) {
    int64_t direct_best;
    if (pnp_direct(X, Y, Z, U, V, n, cam, k, rvec_rt, R, t, mask, n_inliers, iters_used, &direct_best))
        return direct_best;
    int64_t H = max_iters > 1 ? max_iters : 1;
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * H);
    int8_t *status = (int8_t *)malloc(H);
    double *models = (double *)malloc(sizeof(double) * 16 * H);
    int32_t *subs = NULL;
    int8_t *sst = NULL;
    if (sampler == 1) {
        subs = (int32_t *)malloc(sizeof(int32_t) * k * H);
        sst = (int8_t *)malloc(H);
        uint64_t st = ~(uint64_t)0;
        orc_mwc_subsets(&st, n, k, H, NULL, NULL, NULL, NULL, subs, sst);
    }
    float thr2 = orc_thr2(thr);
    orc_pnp_hypotheses_k(X, Y, Z, U, V, n, cam, thr2, seed, 0, 0, H, k, subs, sst, counts, status, models, rvec_rt);
    int32_t good = 0;
    int64_t best = orc_scan(counts, status, H, n, k, confidence, max_iters, &good, iters_used);
    if (best >= 0) {
        memcpy(R, models + 16 * best, 9 * sizeof(double));
        memcpy(t, models + 16 * best + 9, 3 * sizeof(double));
        orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = good;
    free(counts); free(status); free(models); free(subs); free(sst);
    return best;
}

ORC_API int64_t orc_pnp_ransac(const float *X, const float *Y, const float *Z, const float *U, const float *V, int n,
                               const double cam[4], double thr, double confidence, int max_iters, uint64_t seed,
                               int sampler, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                               int64_t *iters_used) {
    return orc_pnp_ransac_k(X, Y, Z, U, V, n, cam, thr, confidence, max_iters, seed, sampler, 4, R, t, mask, n_inliers,
                            iters_used, 0);
}

/* The same loop as OpenCV runs it, one hypothesis at a time: it stops as soon as the iteration
 * bound (RANSACUpdateNumIters after each new best) is reached, so it scores only `iters`
 * hypotheses -- the CPU ms-to-best-model baseline (bench.py cpu_baseline).  Philox sampler.
 * Same results as orc_pnp_ransac (tests/test_oracle_golden.py). */
/* k: sample size / minimal solver (4 P3P, 5 EPnP-5, also model_points); sampler 0 Philox, 1 the
 * MWC getSubset sequence drawn one subset per iteration, as OpenCV draws it (the C1 CPU leg:
 * main_v1.py:497 / testpro-K.py:72 run EPnP-5 on MWC samples) */
ORC_API int64_t orc_pnp_ransac_seq_k(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                     int n, const double cam[4], double thr, double confidence, int max_iters,
                                     uint64_t seed, int sampler, int k, double R[9], double t[3], uint8_t *mask,
                                     int32_t *n_inliers, int64_t *iters_used, int rvec_rt) {
    int64_t direct_best;
    if (pnp_direct(X, Y, Z, U, V, n, cam, k, rvec_rt, R, t, mask, n_inliers, iters_used, &direct_best))
        return direct_best;
    const float thr2 = orc_thr2(thr);
    int64_t niters = max_iters > 1 ? max_iters : 1, best = -1, h = 0;
    int32_t good = 0;
    double bm[16] = {0};
    uint64_t mwc = ~(uint64_t)0;
    for (; h < niters; ++h) {
        int32_t c, sub[5];
        int8_t st, sst = 1;
        double m[16];
        if (sampler == 1) {
            orc_mwc_subsets(&mwc, n, k, 1, NULL, NULL, NULL, NULL, sub, &sst);
            orc_pnp_hypotheses_k(X, Y, Z, U, V, n, cam, thr2, seed, 0, h, 1, k, sub, &sst, &c, &st, m, rvec_rt);
        } else {
            orc_pnp_hypotheses_k(X, Y, Z, U, V, n, cam, thr2, seed, 0, h, 1, k, NULL, NULL, &c, &st, m, rvec_rt);
        }
        if (st < 0) break;
        if (st == 0) continue;
        if (c > (good > k - 1 ? good : k - 1)) {
            best = h;
            good = c;
            memcpy(bm, m, sizeof bm);
            niters = orc_update_num_iters(confidence, (double)(n - c) / n, k, (int)niters);
        }
    }
    if (iters_used) *iters_used = h;
    if (best >= 0) {
        memcpy(R, bm, 9 * sizeof(double));
        memcpy(t, bm + 9, 3 * sizeof(double));
        orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = good;
    return best;
}

ORC_API int64_t orc_pnp_ransac_seq(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                   int n, const double cam[4], double thr, double confidence, int max_iters,
                                   uint64_t seed, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                                   int64_t *iters_used) {
    return orc_pnp_ransac_seq_k(X, Y, Z, U, V, n, cam, thr, confidence, max_iters, seed, 0, 4, R, t, mask, n_inliers,
                                iters_used, 0);
}

/* orc_pnp_hypotheses over `threads` host threads (OpenMP, hypotheses dealt in chunks of 64):
 * the CPU baseline's multi-core leg; every hypothesis' result is the single-thread one. */
ORC_API void orc_pnp_hypotheses_mt(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                   int n, const double cam[4], float thr2, uint64_t seed, int64_t hyp0, int64_t H,
                                   int32_t *counts, int8_t *status, int threads) {
#pragma omp parallel for num_threads(threads) schedule(dynamic, 64)
    for (int64_t h = 0; h < H; ++h)
        orc_pnp_hypotheses(X, Y, Z, U, V, n, cam, thr2, seed, 0, hyp0 + h, 1, NULL, NULL, counts + h, status + h, NULL);
}

/* LO-RANSAC (BASELINE.json configs[4], C5; Chum et al. 2003, simple LO):
 * the OpenCV loop above, except that whenever hypothesis i becomes the best
 * (count > max(best, 3)) a local optimisation runs before hypothesis i+1:
 *     M, c = model_i, count_i
 *     repeat at most 4 times:
 *         M' = orc_pnp_refine(M, inliers(M))   (the final-refit LM)
 *         c' = count(M');  if c' <= c: stop;  M, c = M', c'
 *     best := (M, c);  niters := RANSACUpdateNumIters(conf, (n - c)/n, 4, niters)
 * Returns the seeding hypothesis; R, t = the best (locally optimised) model,
 * mask = its RANSAC-test inliers, *n_inliers = c. */
#define LO_STEPS 4
/* the local optimisation of one new best (R, t with `count` inliers), in place;
 * returns the final count, *steps = refits that raised it */
ORC_API int32_t orc_pnp_local_opt(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                  int n, const double cam[4], float thr2, double R[9], double t[3], int32_t count,
                                  int32_t *steps) {
    uint8_t *m0 = (uint8_t *)malloc(n > 0 ? n : 1), *m1 = (uint8_t *)malloc(n > 0 ? n : 1);
    int32_t c = count, k = 0;
    orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, m0);
    for (int step = 0; step < LO_STEPS; ++step) {
        double NR[9], Nt[3];
        memcpy(NR, R, sizeof NR);
        memcpy(Nt, t, sizeof Nt);
        orc_pnp_refine(X, Y, Z, U, V, m0, n, cam, NR, Nt, 20);
        int32_t c2 = orc_pnp_count(NR, Nt, cam, X, Y, Z, U, V, n, thr2, m1);
        if (c2 <= c) break;
        memcpy(R, NR, sizeof NR);
        memcpy(t, Nt, sizeof Nt);
        c = c2;
        uint8_t *tm = m0; m0 = m1; m1 = tm;
        ++k;
    }
    if (steps) *steps = k;
    free(m0);
    free(m1);
    return c;
}

/* lazy = 1: each hypothesis is drawn, solved and counted when the scan reaches it, so the loop
 * stops at the iteration bound as OpenCV's does (the C5 CPU leg); lazy = 0: all max_iters are
 * evaluated first (the form the GPU's rounds are checked against).  Same results either way. */
static int64_t pnp_ransac_lo_impl(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                  int n, const double cam[4], double thr, double confidence, int max_iters,
                                  uint64_t seed, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                                  int64_t *iters_used, int32_t *lo_improvements, int lazy) {
    int64_t direct_best;
    if (lo_improvements) *lo_improvements = 0;
    if (pnp_direct(X, Y, Z, U, V, n, cam, 4, 0, R, t, mask, n_inliers, iters_used, &direct_best)) return direct_best;
    int64_t H = max_iters > 1 ? max_iters : 1;
    const int64_t Hm = lazy ? 1 : H;
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * Hm);
    int8_t *status = (int8_t *)malloc(Hm);
    double *models = (double *)malloc(sizeof(double) * 16 * Hm);
    float thr2 = orc_thr2(thr);
    if (!lazy) orc_pnp_hypotheses(X, Y, Z, U, V, n, cam, thr2, seed, 0, 0, H, NULL, NULL, counts, status, models);
    int64_t niters = H, best = -1, i;
    int32_t max_good = 0, nlo = 0;
    double BR[9] = {0}, Bt[3] = {0};
    for (i = 0; i < H && i < niters; ++i) {
        const int64_t j = lazy ? 0 : i;
        if (lazy) orc_pnp_hypotheses(X, Y, Z, U, V, n, cam, thr2, seed, 0, i, 1, NULL, NULL, counts, status, models);
        if (status[j] < 0) break;
        if (status[j] == 0) continue;
        int32_t c = counts[j];
        int32_t floor_c = max_good > 3 ? max_good : 3;
        if (c <= floor_c) continue;
        best = i; max_good = c;
        niters = orc_update_num_iters(confidence, (double)(n - c) / n, 4, (int)niters);
        double MR[9], Mt[3];
        memcpy(MR, models + 16 * j, sizeof MR);
        memcpy(Mt, models + 16 * j + 9, sizeof Mt);
        int32_t steps = 0;
        c = orc_pnp_local_opt(X, Y, Z, U, V, n, cam, thr2, MR, Mt, c, &steps);
        nlo += steps;
        if (c > max_good) {
            max_good = c;
            niters = orc_update_num_iters(confidence, (double)(n - c) / n, 4, (int)niters);
        }
        memcpy(BR, MR, sizeof BR);
        memcpy(Bt, Mt, sizeof Bt);
    }
    if (best >= 0) {
        memcpy(R, BR, sizeof BR);
        memcpy(t, Bt, sizeof Bt);
        orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = max_good;
    if (iters_used) *iters_used = i;
    if (lo_improvements) *lo_improvements = nlo;
    free(counts); free(status); free(models);
    return best;
}

/* The C5 CPU baseline over `threads` host threads: OpenCV's LO loop is sequential (each new best
 * changes the iteration bound the next hypothesis is judged against), so the hypotheses are
 * evaluated in rounds (256, doubling to 4096, as the GPU's adaptive rounds) with OpenMP, and each
 * round is scanned -- and every new best locally optimised -- in index order on one thread, up to
 * the bound.  Results equal orc_pnp_ransac_lo's. */
ORC_API int64_t orc_pnp_ransac_lo_mt(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                     int n, const double cam[4], double thr, double confidence, int max_iters,
                                     uint64_t seed, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                                     int64_t *iters_used, int32_t *lo_improvements, int threads) {
    int64_t direct_best;
    if (lo_improvements) *lo_improvements = 0;
    if (pnp_direct(X, Y, Z, U, V, n, cam, 4, 0, R, t, mask, n_inliers, iters_used, &direct_best)) return direct_best;
    const int64_t H = max_iters > 1 ? max_iters : 1;
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * 4096);
    int8_t *status = (int8_t *)malloc(4096);
    double *models = (double *)malloc(sizeof(double) * 16 * 4096);
    const float thr2 = orc_thr2(thr);
    int64_t niters = H, best = -1, i = 0, cur = 256;
    int32_t max_good = 0, nlo = 0;
    double BR[9] = {0}, Bt[3] = {0};
    int stop = 0;
    for (int64_t hb = 0; hb < H && hb < niters && !stop; hb += cur, cur = cur < 4096 ? 2 * cur : 4096) {
        const int64_t hr = (hb + cur < H ? cur : H - hb);
#pragma omp parallel for num_threads(threads) schedule(dynamic, 4)
        for (int64_t h = 0; h < hr; ++h)
            orc_pnp_hypotheses(X, Y, Z, U, V, n, cam, thr2, seed, 0, hb + h, 1, NULL, NULL, counts + h, status + h,
                               models + 16 * h);
        for (i = hb; i < hb + hr && i < niters; ++i) {
            const int64_t j = i - hb;
            if (status[j] < 0) { stop = 1; break; }
            if (status[j] == 0) continue;
            int32_t c = counts[j];
            int32_t floor_c = max_good > 3 ? max_good : 3;
            if (c <= floor_c) continue;
            best = i; max_good = c;
            niters = orc_update_num_iters(confidence, (double)(n - c) / n, 4, (int)niters);
            double MR[9], Mt[3];
            memcpy(MR, models + 16 * j, sizeof MR);
            memcpy(Mt, models + 16 * j + 9, sizeof Mt);
            int32_t steps = 0;
            c = orc_pnp_local_opt(X, Y, Z, U, V, n, cam, thr2, MR, Mt, c, &steps);
            nlo += steps;
            if (c > max_good) {
                max_good = c;
                niters = orc_update_num_iters(confidence, (double)(n - c) / n, 4, (int)niters);
            }
            memcpy(BR, MR, sizeof BR);
            memcpy(Bt, Mt, sizeof Bt);
        }
    }
    if (best >= 0) {
        memcpy(R, BR, sizeof BR);
        memcpy(t, Bt, sizeof Bt);
        orc_pnp_count(R, t, cam, X, Y, Z, U, V, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = max_good;
    if (iters_used) *iters_used = i;
    if (lo_improvements) *lo_improvements = nlo;
    free(counts); free(status); free(models);
    return best;
}

ORC_API int64_t orc_pnp_ransac_lo(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                  int n, const double cam[4], double thr, double confidence, int max_iters,
                                  uint64_t seed, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                                  int64_t *iters_used, int32_t *lo_improvements) {
    return pnp_ransac_lo_impl(X, Y, Z, U, V, n, cam, thr, confidence, max_iters, seed, R, t, mask, n_inliers,
                              iters_used, lo_improvements, 0);
}

ORC_API int64_t orc_pnp_ransac_lo_seq(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                                      int n, const double cam[4], double thr, double confidence, int max_iters,
                                      uint64_t seed, double R[9], double t[3], uint8_t *mask, int32_t *n_inliers,
                                      int64_t *iters_used, int32_t *lo_improvements) {
    return pnp_ransac_lo_impl(X, Y, Z, U, V, n, cam, thr, confidence, max_iters, seed, R, t, mask, n_inliers,
                              iters_used, lo_improvements, 1);
}

ORC_API int64_t orc_hom_ransac(const float *sx, const float *sy, const float *dx, const float *dy, int n, double thr,
                               double confidence, int max_iters, uint64_t seed, int sampler, double Hout[9],
                               uint8_t *mask, int32_t *n_inliers, int64_t *iters_used) {
    if (n == 4) {
        /* findHomography's `method == 0 || npoints == 4` branch ([OpenCV 4.x, unvendored]
         * modules/calib3d/src/fundam.cpp; main_v1.py:312): runKernel on the 4 points in input
         * order (no checkSubset), mask all ones, and no LM (that runs only for npoints > 4).
         * runKernel for 4 points is this build's minimal kernel (orc_hom_minimal). */
        static const int32_t idx[4] = {0, 1, 2, 3};
        const int ok = orc_hom_minimal(sx, sy, dx, dy, idx, Hout);
        if (mask) memset(mask, ok ? 1 : 0, 4);
        if (n_inliers) *n_inliers = ok ? 4 : 0;
        if (iters_used) *iters_used = 0;
        return ok ? 0 : -1;
    }
    int64_t H = max_iters > 1 ? max_iters : 1;
    int32_t *counts = (int32_t *)malloc(sizeof(int32_t) * H);
    int8_t *status = (int8_t *)malloc(H);
    double *models = (double *)malloc(sizeof(double) * 16 * H);
    int32_t *subs = NULL;
    int8_t *sst = NULL;
    if (sampler == 1) {
        subs = (int32_t *)malloc(sizeof(int32_t) * 4 * H);
        sst = (int8_t *)malloc(H);
        uint64_t st = ~(uint64_t)0;
        orc_mwc_subsets(&st, n, 4, H, sx, sy, dx, dy, subs, sst);
    }
    float thr2 = orc_thr2(thr);
    orc_hom_hypotheses(sx, sy, dx, dy, n, thr2, seed, 0, 0, H, subs, sst, counts, status, models);
    int32_t good = 0;
    int64_t best = orc_scan(counts, status, H, n, 4, confidence, max_iters, &good, iters_used);
    if (best >= 0) {
        memcpy(Hout, models + 16 * best, 9 * sizeof(double));
        orc_hom_count(Hout, sx, sy, dx, dy, n, thr2, mask);
    } else if (mask) {
        memset(mask, 0, n);
    }
    if (n_inliers) *n_inliers = good;
    free(counts); free(status); free(models); free(subs); free(sst);
    return best;
}

/* ------------------------------------------------------------------------
 * EPnP on the inliers (Lepetit, Moreno-Noguer, Fua 2009): the final solve of
 * cv2.solvePnPRansac when the minimal solver is P3P (OpenCV re-solves the
 * inliers with SOLVEPNP_EPNP; main_v1.py:497).  The steps of
 * OpenCV's epnp.cpp: control points from the centroid and the principal axes,
 * barycentric alphas, M^T M, its 4 smallest eigenvectors, L 6x10 and rho, beta
 * approximations 1-3 each + 5 Gauss-Newton steps, the pose by SVD of the
 * cross-covariance, the lowest mean reprojection error wins.  Numerics of this
 * project (no OpenCV here to pin them): Jacobi eigen-decompositions (M^T M's
 * 12 x 12 in round-robin order, ep_jacobi_rr; the 3 x 3 ones cyclic),
 * Householder least squares, M^T M assembled from per-control-point-pair sums,
 * the frame centred on the problem's first point, sums in the GPU order
 * (LM_THREADS strided partials, 64-lane butterfly, wave sums in order).
 * ------------------------------------------------------------------------ */
#define EP_MAXV 40

typedef struct { const float *X, *Y, *Z, *U, *V; const uint8_t *mask; int n; double cam[4]; double c[3]; double *part; } epctx;
typedef void (*ep_fn)(const void *prm, double X, double Y, double Z, double u, double v, double *acc);

static void ep_reduce(epctx *c, int nv, ep_fn f, const void *prm, double *out) {
    double *part = c->part;
    if (c->n <= 64) {
        /* every point in its own slot of wave 0, the other slots +0: the same tree restricted to the
         * first m = 2^k >= n lanes.  Levels o >= m add a lane whose coset holds only empty slots
         * (+0.0, which also turns a -0.0 sum into +0.0, as the full tree does), and so does the sum
         * over the 7 empty waves.  Bit-identical to the loop below, without its 512 x nv slots
         * (the EPnP-5 minimal solver reduces 5 points per hypothesis). */
        int m = 1;
        while (m < c->n) m <<= 1;
        for (int q = 0; q < m * nv; ++q) part[q] = 0.0;
        for (int i = 0; i < c->n; ++i)
            if (c->mask[i])
                f(prm, (double)c->X[i] - c->c[0], (double)c->Y[i] - c->c[1], (double)c->Z[i] - c->c[2],
                  (double)c->U[i], (double)c->V[i], part + i * nv);
        double v[64], w[64];
        for (int q = 0; q < nv; ++q) {
            for (int l = 0; l < m; ++l) v[l] = part[l * nv + q];
            for (int o = 32; o > 0; o >>= 1) {
                if (o >= m) {
                    for (int l = 0; l < m; ++l) v[l] = v[l] + 0.0;
                    continue;
                }
                for (int l = 0; l < m; ++l) w[l] = v[l] + v[l ^ o];
                for (int l = 0; l < m; ++l) v[l] = w[l];
            }
            out[q] = LM_THREADS / 64 > 1 ? v[0] + 0.0 : v[0];
        }
        return;
    }
    for (int q = 0; q < LM_THREADS * nv; ++q) part[q] = 0.0;
    for (int tid = 0; tid < LM_THREADS; ++tid)
        for (int i = tid; i < c->n; i += LM_THREADS)
            if (c->mask[i])
                f(prm, (double)c->X[i] - c->c[0], (double)c->Y[i] - c->c[1], (double)c->Z[i] - c->c[2],
                  (double)c->U[i], (double)c->V[i], part + tid * nv);
    double wsum[LM_THREADS / 64][EP_MAXV], v[64], w[64];
    for (int wv = 0; wv < LM_THREADS / 64; ++wv)
        for (int q = 0; q < nv; ++q) {
            for (int l = 0; l < 64; ++l) v[l] = part[(wv * 64 + l) * nv + q];
            for (int o = 32; o > 0; o >>= 1) {
                for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ o];
                for (int l = 0; l < 64; ++l) v[l] = w[l];
            }
            wsum[wv][q] = v[0];
        }
    for (int q = 0; q < nv; ++q) {
        double s = wsum[0][q];
        for (int wv = 1; wv < LM_THREADS / 64; ++wv) s = s + wsum[wv][q];
        out[q] = s;
    }
}

/* the rotation of pair (p, q) (rsac_math.h jrr_rotation): 0 (skipped) for apq = 0 or, from the fifth
   sweep on, apq negligible next to both diagonal entries (the rule of Numerical Recipes' jacobi).
   t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)) = sg |w| / h, theta = d / w, d = aqq - app,
   w = 2 apq, h = |d| + sqrt(d^2 + w^2); cs = 1 / sqrt(t^2 + 1) = h / sqrt(h^2 + w^2),
   sn = t cs = sg |w| / sqrt(h^2 + w^2) (one division) */
static int ep_rot(int sweep, double app, double aqq, double apq, double *cs, double *sn) {
    if (!(apq != 0.0)) return 0;
    if (sweep >= 4) {
        double g = 100.0 * fabs(apq);
        if (fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq)) return 0;
    }
    double d = aqq - app, w = 2.0 * apq;
    double sg = (d == 0.0 || ((d < 0.0) == (w < 0.0))) ? 1.0 : -1.0;
    double aw = fabs(w), h = fabs(d) + sqrt(d * d + w * w);
    double iq = 1.0 / sqrt(h * h + aw * aw);
    *cs = h * iq;
    *sn = sg * aw * iq;
    return 1;
}

/* one rotated pair (x_p, x_q) -> (c x_p - s x_q, s x_p + c x_q), c times the element's own value
   fused with the rounded product of s and the other (rsac_math.h jrr_lo / jrr_hi, r05) */
static double ep_rr_lo(double c, double s, double xp, double xq) { return fma(c, xp, -(s * xq)); }
static double ep_rr_hi(double c, double s, double xp, double xq) { return fma(c, xq, s * xp); }
/* cyclic Jacobi, symmetric N x N (destroyed): d eigenvalues, V[i*N+k] k-th eigenvector; the
   rotation and skip rule of ep_rot, the fused element updates ep_rr_lo / ep_rr_hi (r05) */
static void ep_jacobi(int N, double *A, double *V, double *d) {
    for (int i = 0; i < N * N; ++i) V[i] = 0.0;
    for (int i = 0; i < N; ++i) V[i * N + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int p = 0; p < N; ++p) {
            diag = diag + A[p * N + p] * A[p * N + p];
            for (int q = p + 1; q < N; ++q) off = off + A[p * N + q] * A[p * N + q];
        }
        if (!(off > 1e-32 * diag)) break;
        for (int p = 0; p < N - 1; ++p)
            for (int q = p + 1; q < N; ++q) {
                double cs, sn;
                if (!ep_rot(sweep, A[p * N + p], A[q * N + q], A[p * N + q], &cs, &sn)) continue;
                for (int k = 0; k < N; ++k) {
                    double akp = A[k * N + p], akq = A[k * N + q];
                    A[k * N + p] = ep_rr_lo(cs, sn, akp, akq);
                    A[k * N + q] = ep_rr_hi(cs, sn, akp, akq);
                }
                for (int k = 0; k < N; ++k) {
                    double apk = A[p * N + k], aqk = A[q * N + k];
                    A[p * N + k] = ep_rr_lo(cs, sn, apk, aqk);
                    A[q * N + k] = ep_rr_hi(cs, sn, apk, aqk);
                }
                for (int k = 0; k < N; ++k) {
                    double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = ep_rr_lo(cs, sn, vkp, vkq);
                    V[k * N + q] = ep_rr_hi(cs, sn, vkp, vkq);
                }
            }
    }
    for (int k = 0; k < N; ++k) d[k] = A[k * N + k];
}

/* round-robin ("parallel order") Jacobi, symmetric N x N, N even (EPnP's 12 x 12 M^T M): a sweep
   is N - 1 steps; step r pairs position i with position N - 1 - i, where position 0 holds index 0
   and position m > 0 holds 1 + (m - 1 + r) % (N - 1) (circle method).  All pairs' rotations are
   formed from the matrix at the step's start, then applied to the columns (every row), the rows
   and V's columns.  The pairs are disjoint, so each element's sequence of operations is fixed
   (the device runs a step's pairs on different lanes).  Sweep test as ep_jacobi; the rotation's
   t from d = aqq - app and w = 2 apq (one division fewer than through theta), and from the fifth
   sweep on a pair whose apq is negligible next to both diagonal entries is skipped (the rule of
   Numerical Recipes' jacobi).  Each rotated element is ep_rr_lo / ep_rr_hi: one rounding fewer
   than c a - s b (r05). */
static int ep_rr_pos(int N, int r, int m) { return m == 0 ? 0 : 1 + (m - 1 + r) % (N - 1); }
static void ep_jacobi_rr(int N, double *A, double *V, double *d) {
    int P[8], Q[8];
    double cs[8], sn[8];
    const int H = N / 2;
    for (int i = 0; i < N * N; ++i) V[i] = 0.0;
    for (int i = 0; i < N; ++i) V[i * N + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        /* diag in p order; off = the rows' partial sums (q > p, q order) added in row order */
        double off = 0.0, diag = 0.0;
        for (int p = 0; p < N; ++p) {
            diag = diag + A[p * N + p] * A[p * N + p];
            double rp = 0.0;
            for (int q = p + 1; q < N; ++q) rp = rp + A[p * N + q] * A[p * N + q];
            off = off + rp;
        }
        if (!(off > 1e-32 * diag)) break;
        for (int r = 0; r < N - 1; ++r) {
            for (int i = 0; i < H; ++i) {
                int a = ep_rr_pos(N, r, i), b = ep_rr_pos(N, r, N - 1 - i);
                int p = a < b ? a : b, q = a < b ? b : a;
                double apq = A[p * N + q], app = A[p * N + p], aqq = A[q * N + q];
                P[i] = p; Q[i] = q;
                cs[i] = 1.0; sn[i] = 0.0;
                (void)ep_rot(sweep, app, aqq, apq, &cs[i], &sn[i]);
            }
            /* a skipped pair applies cs = 1, sn = 0 like any other (no special case, so the device
               runs every step branch-free with the same bits) */
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < H; ++i) {
                    double akp = A[k * N + P[i]], akq = A[k * N + Q[i]];
                    A[k * N + P[i]] = ep_rr_lo(cs[i], sn[i], akp, akq);
                    A[k * N + Q[i]] = ep_rr_hi(cs[i], sn[i], akp, akq);
                }
            for (int i = 0; i < H; ++i) {
                for (int k = 0; k < N; ++k) {
                    double apk = A[P[i] * N + k], aqk = A[Q[i] * N + k];
                    A[P[i] * N + k] = ep_rr_lo(cs[i], sn[i], apk, aqk);
                    A[Q[i] * N + k] = ep_rr_hi(cs[i], sn[i], apk, aqk);
                }
            }
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < H; ++i) {
                    double vkp = V[k * N + P[i]], vkq = V[k * N + Q[i]];
                    V[k * N + P[i]] = ep_rr_lo(cs[i], sn[i], vkp, vkq);
                    V[k * N + Q[i]] = ep_rr_hi(cs[i], sn[i], vkp, vkq);
                }
        }
    }
    for (int k = 0; k < N; ++k) d[k] = A[k * N + k];
}

/* eigenvalue indices by decreasing value, ties keep the lower index first (insertion sort) */
static void ep_order(int N, const double *d, int *o) {
    for (int i = 0; i < N; ++i) o[i] = i;
    for (int i = 1; i < N; ++i) {
        int k = o[i], j = i - 1;
        while (j >= 0 && d[o[j]] < d[k]) { o[j + 1] = o[j]; --j; }
        o[j + 1] = k;
    }
}

/* min |A x - b|, A 6 x N (N <= 5), Householder QR; a vanishing pivot gives x_k = 0.  Sums of
   products and the reflector updates accumulate by fma (rsac_math.h householder_ls, r05) */
static void ep_lsq(int N, double *A, double *b, double *x) {
    const int M = 6;
    for (int k = 0; k < N; ++k) {
        double nrm = 0.0, v[6], vv = 0.0, sdot, f;
        for (int i = k; i < M; ++i) nrm = fma(A[i * N + k], A[i * N + k], nrm);
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        double alpha = A[k * N + k] > 0.0 ? -nrm : nrm;
        for (int i = k; i < M; ++i) v[i] = A[i * N + k];
        v[k] = v[k] - alpha;
        for (int i = k; i < M; ++i) vv = fma(v[i], v[i], vv);
        if (vv == 0.0) continue;
        for (int j = k; j < N; ++j) {
            sdot = 0.0;
            for (int i = k; i < M; ++i) sdot = fma(v[i], A[i * N + j], sdot);
            f = 2.0 * sdot / vv;
            for (int i = k; i < M; ++i) A[i * N + j] = fma(-f, v[i], A[i * N + j]);
        }
        sdot = 0.0;
        for (int i = k; i < M; ++i) sdot = fma(v[i], b[i], sdot);
        f = 2.0 * sdot / vv;
        for (int i = k; i < M; ++i) b[i] = fma(-f, v[i], b[i]);
    }
    for (int k = N - 1; k >= 0; --k) {
        double s = b[k];
        for (int j = k + 1; j < N; ++j) s = fma(-A[k * N + j], x[j], s);
        double rkk = A[k * N + k];
        x[k] = fabs(rkk) > 1e-300 ? s / rkk : 0.0;
    }
}

typedef struct { double c[3], ci[9]; } ep_alpha;

static void ep_alphas(const ep_alpha *f, double X, double Y, double Z, double *a) {
    double dx = X - f->c[0], dy = Y - f->c[1], dz = Z - f->c[2];
    for (int j = 0; j < 3; ++j) a[1 + j] = fma(f->ci[3 * j + 2], dz, fma(f->ci[3 * j + 1], dy, f->ci[3 * j] * dx));
    a[0] = 1.0 - a[1] - a[2] - a[3];
}

static void ep_f_mean(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    acc[0] += X; acc[1] += Y; acc[2] += Z; acc[3] += 1.0;
}
static void ep_f_cov(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    const double *c0 = (const double *)prm;
    double x = X - c0[0], y = Y - c0[1], z = Z - c0[2];
    acc[0] = fma(x, x, acc[0]); acc[1] = fma(x, y, acc[1]); acc[2] = fma(x, z, acc[2]);
    acc[3] = fma(y, y, acc[3]); acc[4] = fma(y, z, acc[4]); acc[5] = fma(z, z, acc[5]);
}
typedef struct { ep_alpha af; double cam[4]; } ep_pair_prm;
static void ep_f_pairs(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    const ep_pair_prm *p = (const ep_pair_prm *)prm;
    double a[4];
    ep_alphas(&p->af, X, Y, Z, a);
    double du = p->cam[2] - u, dv = p->cam[3] - v, w = fma(dv, dv, du * du);
    int q = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j, q += 4) {
            double aa = a[i] * a[j];
            acc[q] += aa;
            acc[q + 1] = fma(aa, du, acc[q + 1]);
            acc[q + 2] = fma(aa, dv, acc[q + 2]);
            acc[q + 3] = fma(aa, w, acc[q + 3]);
        }
}
typedef struct { ep_alpha af; double cc[4][3]; double pc0[3]; double c0[3]; } ep_pose_prm;
static void ep_f_pc0(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    const ep_pose_prm *p = (const ep_pose_prm *)prm;
    double a[4];
    ep_alphas(&p->af, X, Y, Z, a);
    for (int j = 0; j < 3; ++j) acc[j] += fma(a[3], p->cc[3][j], fma(a[2], p->cc[2][j], fma(a[1], p->cc[1][j], a[0] * p->cc[0][j])));
}
static void ep_f_cross(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    const ep_pose_prm *p = (const ep_pose_prm *)prm;
    double a[4], pc[3];
    ep_alphas(&p->af, X, Y, Z, a);
    for (int j = 0; j < 3; ++j)
        pc[j] = fma(a[3], p->cc[3][j], fma(a[2], p->cc[2][j], fma(a[1], p->cc[1][j], a[0] * p->cc[0][j]))) - p->pc0[j];
    double pw[3] = {X - p->c0[0], Y - p->c0[1], Z - p->c0[2]};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) acc[3 * i + j] = fma(pc[i], pw[j], acc[3 * i + j]);
}
typedef struct { double R[9], t[3], cam[4]; } ep_err_prm;
static void ep_f_err(const void *prm, double X, double Y, double Z, double u, double v, double *acc) {
    const ep_err_prm *p = (const ep_err_prm *)prm;
    const double *R = p->R, *t = p->t;
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double iz = 1.0 / (R[6] * X + R[7] * Y + R[8] * Z + t[2]);
    double du = u - (p->cam[2] + p->cam[0] * x * iz), dv = v - (p->cam[3] + p->cam[1] * y * iz);
    acc[0] += sqrt(du * du + dv * dv);
}

/* R = U V^T of the cross-covariance H (SVD via the eigen-decomposition of H^T H), last row
 * negated when det < 0 (OpenCV's estimate_R_and_t); 0 when H has rank < 2.  ep_rotation's route
 * for a nearly singular H (rsac_math.h epnp_rotation_svd). */
static int ep_rotation_svd(const double *H, double *R) {
    double B[9], V[9], d[3], v[3][3], u[3][3];
    int o[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) B[3 * i + j] = H[i] * H[j] + H[3 + i] * H[3 + j] + H[6 + i] * H[6 + j];
    ep_jacobi(3, B, V, d);
    ep_order(3, d, o);
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) v[k][i] = V[3 * i + o[k]];
    double s0 = sqrt(d[o[0]] > 0.0 ? d[o[0]] : 0.0);
    if (!(s0 > 0.0)) return 0;
    for (int k = 0; k < 3; ++k) {
        double sk = sqrt(d[o[k]] > 0.0 ? d[o[k]] : 0.0);
        if (k < 2 || sk > 1e-10 * s0) {
            if (!(sk > 1e-10 * s0)) return 0;
            for (int i = 0; i < 3; ++i) u[k][i] = (H[3 * i] * v[k][0] + H[3 * i + 1] * v[k][1] + H[3 * i + 2] * v[k][2]) / sk;
        } else {
            u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
            u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
            u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
        }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = u[0][i] * v[0][j] + u[1][i] * v[1][j] + u[2][i] * v[2][j];
    double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0.0)
        for (int j = 0; j < 3; ++j) R[6 + j] = -R[6 + j];
    return 1;
}

/* the orthogonal polar factor of a well-conditioned 3 x 3 X, in place (rsac_math.h polar_newton3):
   Newton's X <- (g X + X^-T / g) / 2, X^-T = cof(X) / det X, g = (|X^-T|_F / |X|_F)^(1/2) while a step
   moves an element by more than 1e-2, g = 1 after, until no element moves by more than 1e-15 (at
   most 30 steps) */
static void ep_polar(double *X) {
    int scale = 1;
    for (int it = 0; it < 30; ++it) {
        double Y[9];
        Y[0] = X[4] * X[8] - X[5] * X[7];
        Y[1] = X[5] * X[6] - X[3] * X[8];
        Y[2] = X[3] * X[7] - X[4] * X[6];
        Y[3] = X[2] * X[7] - X[1] * X[8];
        Y[4] = X[0] * X[8] - X[2] * X[6];
        Y[5] = X[1] * X[6] - X[0] * X[7];
        Y[6] = X[1] * X[5] - X[2] * X[4];
        Y[7] = X[2] * X[3] - X[0] * X[5];
        Y[8] = X[0] * X[4] - X[1] * X[3];
        double det = X[0] * Y[0] + X[1] * Y[1] + X[2] * Y[2];
        if (!(fabs(det) > 1e-300) || !isfinite(det)) return;
        double id = 1.0 / det;
        for (int k = 0; k < 9; ++k) Y[k] = Y[k] * id;
        double g = 1.0, ig = 1.0;
        if (scale) {
            double sx = 0.0, sy = 0.0;
            for (int k = 0; k < 9; ++k) {
                sx = sx + X[k] * X[k];
                sy = sy + Y[k] * Y[k];
            }
            g = sqrt(sqrt(sy / sx));
            ig = 1.0 / g;
        }
        double mv = 0.0;
        for (int k = 0; k < 9; ++k) {
            double nx = 0.5 * (g * X[k] + ig * Y[k]);
            double dd = fabs(nx - X[k]);
            mv = dd > mv ? dd : mv;
            X[k] = nx;
        }
        if (!(mv > 1e-15)) return;
        scale = mv > 1e-2;
    }
}

/* ep_rotation_svd's R: the polar factor of H (ep_polar) when |det H| > 1e-10 |H|_F^3 (full rank),
 * else ep_rotation_svd itself (rsac_math.h epnp_rotation) */
static int ep_rotation(const double *H, double *R) {
    double n2 = 0.0;
    for (int k = 0; k < 9; ++k) n2 = n2 + H[k] * H[k];
    double dh = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) + H[2] * (H[3] * H[7] - H[4] * H[6]);
    if (!(fabs(dh) > 1e-10 * n2 * sqrt(n2))) return ep_rotation_svd(H, R);
    for (int k = 0; k < 9; ++k) R[k] = H[k];
    ep_polar(R);
    double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0.0)
        for (int j = 0; j < 3; ++j) R[6 + j] = -R[6 + j];
    return 1;
}

/* 5 Gauss-Newton steps on the betas */
static void ep_gauss_newton(const double *L, const double *rho, double *be) {
    for (int it = 0; it < 5; ++it) {
        double A[24], b[6], x[4];
        for (int i = 0; i < 6; ++i) {
            const double *r = L + 10 * i;
            /* fma chains in OpenCV's term order (rsac_math.h epnp_gauss_newton, r05) */
            A[4 * i + 0] = fma(r[6], be[3], fma(r[3], be[2], fma(r[1], be[1], 2.0 * r[0] * be[0])));
            A[4 * i + 1] = fma(r[7], be[3], fma(r[4], be[2], fma(2.0 * r[2], be[1], r[1] * be[0])));
            A[4 * i + 2] = fma(r[8], be[3], fma(2.0 * r[5], be[2], fma(r[4], be[1], r[3] * be[0])));
            A[4 * i + 3] = fma(2.0 * r[9], be[3], fma(r[8], be[2], fma(r[7], be[1], r[6] * be[0])));
            double q = r[0] * be[0] * be[0];
            q = fma(r[1] * be[0], be[1], q);
            q = fma(r[2] * be[1], be[1], q);
            q = fma(r[3] * be[0], be[2], q);
            q = fma(r[4] * be[1], be[2], q);
            q = fma(r[5] * be[2], be[2], q);
            q = fma(r[6] * be[0], be[3], q);
            q = fma(r[7] * be[1], be[3], q);
            q = fma(r[8] * be[2], be[3], q);
            q = fma(r[9] * be[3], be[3], q);
            b[i] = rho[i] - q;
        }
        ep_lsq(4, A, b, x);
        for (int j = 0; j < 4; ++j) be[j] = be[j] + x[j];
    }
}

/* returns 1 and (R, t) in the input frame, or 0 (< 4 inliers / degenerate cloud; R, t untouched) */
ORC_API int orc_pnp_epnp(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                         const uint8_t *mask, int n, const double cam[4], double R_out[9], double t_out[3]) {
    if (n <= 0) return 0;
    epctx c = {X, Y, Z, U, V, mask, n, {cam[0], cam[1], cam[2], cam[3]}, {X[0], Y[0], Z[0]}, NULL};
    c.part = (double *)malloc(sizeof(double) * (n <= 64 ? 64 : LM_THREADS) * EP_MAXV);
    int ok = 0;
    double s4[4], cw[4][3], cov[6];
    ep_reduce(&c, 4, ep_f_mean, NULL, s4);
    double nn = s4[3];
    if (!(nn >= 4.0)) goto out;
    for (int j = 0; j < 3; ++j) cw[0][j] = s4[j] / nn;
    ep_reduce(&c, 6, ep_f_cov, cw[0], cov);
    {
        double A[9] = {cov[0], cov[1], cov[2], cov[1], cov[3], cov[4], cov[2], cov[4], cov[5]}, Vv[9], d[3];
        int o[3];
        ep_jacobi(3, A, Vv, d);
        ep_order(3, d, o);
        for (int i = 1; i < 4; ++i) {
            double ev = d[o[i - 1]];
            double kk = sqrt((ev > 0.0 ? ev : 0.0) / nn);
            for (int j = 0; j < 3; ++j) cw[i][j] = cw[0][j] + kk * Vv[3 * j + o[i - 1]];
        }
    }
    ep_alpha af;
    for (int j = 0; j < 3; ++j) af.c[j] = cw[0][j];
    {
        double cc[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = cw[j][i] - cw[0][i];
        double m00 = cc[4] * cc[8] - cc[5] * cc[7], m01 = cc[5] * cc[6] - cc[3] * cc[8], m02 = cc[3] * cc[7] - cc[4] * cc[6];
        double det = cc[0] * m00 + cc[1] * m01 + cc[2] * m02;
        double nrm = 0.0;
        for (int q = 0; q < 9; ++q) nrm = nrm + cc[q] * cc[q];
        if (!(fabs(det) > 1e-12 * nrm * sqrt(nrm))) goto out;
        double id = 1.0 / det;
        af.ci[0] = m00 * id;
        af.ci[1] = (cc[2] * cc[7] - cc[1] * cc[8]) * id;
        af.ci[2] = (cc[1] * cc[5] - cc[2] * cc[4]) * id;
        af.ci[3] = m01 * id;
        af.ci[4] = (cc[0] * cc[8] - cc[2] * cc[6]) * id;
        af.ci[5] = (cc[2] * cc[3] - cc[0] * cc[5]) * id;
        af.ci[6] = m02 * id;
        af.ci[7] = (cc[1] * cc[6] - cc[0] * cc[7]) * id;
        af.ci[8] = (cc[0] * cc[4] - cc[1] * cc[3]) * id;
    }
    double pairs[40];
    {
        ep_pair_prm pp;
        pp.af = af;
        memcpy(pp.cam, cam, sizeof(pp.cam));
        ep_reduce(&c, 40, ep_f_pairs, &pp, pairs);
    }
    double ut[4][12], L[60], rho[6], be3[3][4];
    int valid[3];
    {
        double A[144], Vv[144], d[12];
        int o[12], q = 0;
        const double fx = cam[0], fy = cam[1];
        for (int i = 0; i < 4; ++i)
            for (int j = i; j < 4; ++j, q += 4) {
                double s0 = pairs[q], su = pairs[q + 1], sv = pairs[q + 2], sw = pairs[q + 3];
                double blk[9] = {fx * fx * s0, 0.0, fx * su, 0.0, fy * fy * s0, fy * sv, fx * su, fy * sv, sw};
                for (int p = 0; p < 3; ++p)
                    for (int r = 0; r < 3; ++r) {
                        A[12 * (3 * i + p) + 3 * j + r] = blk[3 * p + r];
                        A[12 * (3 * j + r) + 3 * i + p] = blk[3 * p + r];
                    }
            }
        ep_jacobi_rr(12, A, Vv, d);
        ep_order(12, d, o);
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 12; ++j) ut[i][j] = Vv[12 * j + o[11 - i]];
        /* L 6x10 (compute_L_6x10) */
        int a = 0, b = 1;
        for (int i = 0; i < 6; ++i) {
            double dv[4][3];
            for (int p = 0; p < 4; ++p)
                for (int qq = 0; qq < 3; ++qq) dv[p][qq] = ut[p][3 * a + qq] - ut[p][3 * b + qq];
            ++b;
            if (b > 3) { ++a; b = a + 1; }
#define EPDOT(p, qd) fma(dv[p][2], dv[qd][2], fma(dv[p][1], dv[qd][1], dv[p][0] * dv[qd][0]))
            double *r = L + 10 * i;
            r[0] = EPDOT(0, 0);
            r[1] = 2.0 * EPDOT(0, 1);
            r[2] = EPDOT(1, 1);
            r[3] = 2.0 * EPDOT(0, 2);
            r[4] = 2.0 * EPDOT(1, 2);
            r[5] = EPDOT(2, 2);
            r[6] = 2.0 * EPDOT(0, 3);
            r[7] = 2.0 * EPDOT(1, 3);
            r[8] = 2.0 * EPDOT(2, 3);
            r[9] = EPDOT(3, 3);
#undef EPDOT
        }
        q = 0;
        for (int i = 0; i < 4; ++i)
            for (int j = i + 1; j < 4; ++j, ++q) {
                double dx = cw[i][0] - cw[j][0], dy = cw[i][1] - cw[j][1], dz = cw[i][2] - cw[j][2];
                rho[q] = fma(dz, dz, fma(dy, dy, dx * dx));
            }
        for (int ap = 1; ap <= 3; ++ap) {
            double *be = be3[ap - 1], bb[6];
            for (int j = 0; j < 4; ++j) be[j] = 0.0;
            for (int i = 0; i < 6; ++i) bb[i] = rho[i];
            int okk = 1;
            if (ap == 1) {
                static const int cols[4] = {0, 1, 3, 6};
                double AA[24], x[4];
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 4; ++j) AA[4 * i + j] = L[10 * i + cols[j]];
                ep_lsq(4, AA, bb, x);
                double sg = x[0] < 0.0 ? -1.0 : 1.0;
                be[0] = sqrt(sg * x[0]);
                okk = be[0] != 0.0;
                if (okk)
                    for (int j = 1; j < 4; ++j) be[j] = sg * x[j] / be[0];
            } else if (ap == 2) {
                double AA[18], x[3];
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 3; ++j) AA[3 * i + j] = L[10 * i + j];
                ep_lsq(3, AA, bb, x);
                if (x[0] < 0.0) { be[0] = sqrt(-x[0]); be[1] = x[2] < 0.0 ? sqrt(-x[2]) : 0.0; }
                else { be[0] = sqrt(x[0]); be[1] = x[2] > 0.0 ? sqrt(x[2]) : 0.0; }
                if (x[1] < 0.0) be[0] = -be[0];
            } else {
                double AA[30], x[5];
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 5; ++j) AA[5 * i + j] = L[10 * i + j];
                ep_lsq(5, AA, bb, x);
                if (x[0] < 0.0) { be[0] = sqrt(-x[0]); be[1] = x[2] < 0.0 ? sqrt(-x[2]) : 0.0; }
                else { be[0] = sqrt(x[0]); be[1] = x[2] > 0.0 ? sqrt(x[2]) : 0.0; }
                if (x[1] < 0.0) be[0] = -be[0];
                okk = be[0] != 0.0;
                if (okk) be[2] = x[3] / be[0];
            }
            if (okk) ep_gauss_newton(L, rho, be);
            valid[ap - 1] = okk;
        }
    }
    int first = -1;
    for (int i = 0; i < n; ++i)
        if (mask[i]) { first = i; break; }
    if (first < 0) goto out;
    double a1[4];
    ep_alphas(&af, (double)X[first] - c.c[0], (double)Y[first] - c.c[1], (double)Z[first] - c.c[2], a1);
    double best = 0.0, bR[9], bt[3];
    int have = 0;
    for (int ap = 0; ap < 3; ++ap) {
        if (!valid[ap]) continue;
        const double *be = be3[ap];
        ep_pose_prm pp;
        pp.af = af;
        for (int j = 0; j < 3; ++j) pp.c0[j] = cw[0][j];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 3; ++j)
                pp.cc[i][j] = fma(be[3], ut[3][3 * i + j], fma(be[2], ut[2][3 * i + j], fma(be[1], ut[1][3 * i + j], be[0] * ut[0][3 * i + j])));
        double z1 = fma(a1[3], pp.cc[3][2], fma(a1[2], pp.cc[2][2], fma(a1[1], pp.cc[1][2], a1[0] * pp.cc[0][2])));
        if (z1 < 0.0)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 3; ++j) pp.cc[i][j] = -pp.cc[i][j];
        ep_reduce(&c, 3, ep_f_pc0, &pp, pp.pc0);
        for (int j = 0; j < 3; ++j) pp.pc0[j] = pp.pc0[j] / nn;
        double H[9];
        ep_reduce(&c, 9, ep_f_cross, &pp, H);
        ep_err_prm ep;
        if (!ep_rotation(H, ep.R)) continue;
        for (int i = 0; i < 3; ++i) ep.t[i] = pp.pc0[i] - fma(ep.R[3 * i + 2], cw[0][2], fma(ep.R[3 * i + 1], cw[0][1], ep.R[3 * i] * cw[0][0]));
        memcpy(ep.cam, cam, sizeof(ep.cam));
        double es;
        ep_reduce(&c, 1, ep_f_err, &ep, &es);
        double err = es / nn;
        if (!have || err < best) {
            have = 1;
            best = err;
            memcpy(bR, ep.R, sizeof(bR));
            memcpy(bt, ep.t, sizeof(bt));
        }
    }
    if (!have) goto out;
    for (int j = 0; j < 3; ++j) bt[j] = bt[j] - (bR[3 * j] * c.c[0] + bR[3 * j + 1] * c.c[1] + bR[3 * j + 2] * c.c[2]);
    memcpy(R_out, bR, sizeof(bR));
    memcpy(t_out, bt, sizeof(bt));
    ok = 1;
out:
    free(c.part);
    return ok;
}
