/*
 * cv_epnp.c -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so with rsac_oracle.c).
 *
 * OpenCV's own operation sequence for the minimal solver every reference PnP call runs:
 * cv2.solvePnPRansac with the default flags (main_v1.py:497-502, testpro-K.py:72-75,
 * testpro.py:536-541, test_pro.py:515-520) draws 5-point subsets and solves each with
 * solvePnP(..., SOLVEPNP_EPNP) ([OpenCV 4.x, unvendored] solvepnp.cpp solvePnPRansac /
 * PnPRansacCallback::runKernel / solvePnPGeneric), then stores the model as (rvec, tvec), so
 * computeError projects through Rodrigues(rvec).  OpenCV is not vendored under /root/reference
 * and not installed here; the steps below restate, in order, the public OpenCV 4.x sources:
 *
 *   solvePnPGeneric (SOLVEPNP_EPNP): undistortPoints(ipoints, K, dist = 0) -> the normalised
 *     points (u - cx) * (1/fx) in double, stored in the input's type (CV_32F inside RANSAC:
 *     rounded to f32; undistort.dispatch.cpp cvUndistortPointsInternal: with zero coefficients
 *     the 5 fixed-point iterations and the identity R are exact), then epnp(K, opoints, them).
 *   epnp.cpp: init_points (us = x * fu + uc), choose_control_points (centroid of the raw
 *     coordinates; PCA by cvMulTransposed + cvSVD of PW0^T PW0), compute_barycentric_coordinates
 *     (cvInvert(CC, CV_SVD)), fill_M, cvMulTransposed(M) + cvSVD(M^T M, U_T), compute_L_6x10,
 *     compute_rho, find_betas_approx_1..3 (cvSolve(..., CV_SVD)), gauss_newton (5 steps of
 *     epnp::qr_solve), compute_R_and_t (compute_ccs, compute_pcs, solve_for_sign,
 *     estimate_R_and_t by cvSVD of the cross-covariance, reprojection_error), the first lowest
 *     of the three errors.
 *   lapack.cpp: JacobiSVDImpl_<double> (one-sided Jacobi in cyclic pair order, eps 10 DBL_EPSILON,
 *     hypot rotation, selection sort, row normalisation with the RNG(0x12345678) fill of null
 *     directions), _SVDcompute (the transposed input), SVBkSbImpl_ (threshold 2 DBL_EPSILON sum w),
 *     cv::solve DECOMP_SVD, cv::invert DECOMP_SVD.  matmul.cpp MulTransposedR (sequential sums).
 *   calibration.cpp cvRodrigues2: matrix -> vector through cvSVD + cvGEMM (R = U V^T), vector ->
 *     matrix as c I + c1 r r^T + s [r]x element by element.
 *
 * Arithmetic: -ffp-contract=off, every sum left to right as written in those sources, no fused
 * operations (OpenCV's x86 baseline build has none).  The two libm dependencies are restated
 * deterministically so the GPU gives the same bits: hypot (cvq_hypot below: glibc 2.35's own
 * algorithm, bit-identical to this host's libm outside operands below 2^-509, which JacobiSVD's
 * rotations do not reach) and cos / sin / acos of the Rodrigues conversion (rsac_oracle.c
 * orc_rd_*: polynomials with exactly rounded coefficients, ~1 ulp from libm).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

ORC_API double orc_rd_acos(double x);
ORC_API void orc_rd_sincos(double th, double *sn, double *cs);

/* hypot(x, y) as glibc 2.35 computes it on x86-64 (sysdeps/ieee754/dbl-64/e_hypot.c: the non-FMA
 * kernel of C. F. Borges, "An Improved Algorithm for hypot(a, b)", 2019, with glibc's scaling of
 * huge / tiny operands).  tests/test_cv_epnp.py checks it against this host's libm.  Every
 * operation is a rounded + - * / sqrt, so the GPU (rsac_cvepnp.h hypot_glibc) gives the same bits. */
static double cvq_hypot_kernel(double ax, double ay) {
    double t1, t2;
    double h = sqrt(ax * ax + ay * ay);
    if (h <= 2.0 * ay) {
        double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

ORC_API double cvq_hypot(double x, double y) {
    if (!isfinite(x) || !isfinite(y)) {
        if (isinf(x) || isinf(y)) return INFINITY;
        return x + y;
    }
    x = fabs(x);
    y = fabs(y);
    const double ax = x < y ? y : x, ay = x < y ? x : y;
    if (ax > 0x1p+511) {
        if (ay <= ax * 0x1p-54) return ax + ay;
        return cvq_hypot_kernel(ax * 0x1p-600, ay * 0x1p-600) / 0x1p-600;
    }
    if (ay < 0x1p-511) {
        if (ax >= ay / 0x1p-54) return ax + ay;
        return cvq_hypot_kernel(ax / 0x1p-600, ay / 0x1p-600) * 0x1p-600;
    }
    if (ay <= ax * 0x1p-54) return ax + ay;
    return cvq_hypot_kernel(ax, ay);
}

/* cv::RNG (MWC, CV_RNG_COEFF 4164903690) */
static uint32_t cvq_rng_next(uint64_t *st) {
    *st = (uint64_t)(uint32_t)(*st) * 4164903690u + (*st >> 32);
    return (uint32_t)(*st);
}

/* lapack.cpp JacobiSVDImpl_<double>(At, astep, W, Vt, vstep, m, n, n1, DBL_MIN, 10 DBL_EPSILON):
 * At is n x m (row stride astep), its rows the columns being orthogonalised; Vt n x n (stride
 * vstep) or NULL; the first n1 rows of At are normalised on exit. */
/* test hook: how many rows JacobiSVD has filled with a random direction (zero singular values),
 * per matrix size n (tests/test_cv_epnp.py checks that the degenerate fixtures reach the branch) */
static long g_fill[16];
ORC_API long orc_cvq_fill_events(int n) { return n >= 0 && n < 16 ? g_fill[n] : 0; }
/* study hook (scripts/jacobi_sweeps.py): per matrix size n, how many decompositions ran k sweeps,
 * and how many rotations (pairs not skipped) sweep k made in total */
static long g_sweeps[16][32], g_rots[16][32];
ORC_API long orc_cvq_sweep_hist(int n, int k) { return n >= 0 && n < 16 && k >= 0 && k < 32 ? g_sweeps[n][k] : 0; }
ORC_API long orc_cvq_rot_hist(int n, int k) { return n >= 0 && n < 16 && k >= 0 && k < 32 ? g_rots[n][k] : 0; }

ORC_API void cvq_jacobi_svd(double *At, int astep, double *Wout, double *Vt, int vstep, int m, int n, int n1) {
    const double minval = DBL_MIN, eps = DBL_EPSILON * 10;
    double W[16];
    int max_iter = m > 30 ? m : 30;
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sd;
        if (Vt) {
            for (int k = 0; k < n; ++k) Vt[i * vstep + k] = 0;
            Vt[i * vstep + i] = 1;
        }
    }
    int iter;
    for (iter = 0; iter < max_iter; ++iter) {
        int changed = 0;
        for (int i = 0; i < n - 1; ++i)
            for (int j = i + 1; j < n; ++j) {
                double *Ai = At + i * astep, *Aj = At + j * astep;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; ++k) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = cvq_hypot(p, beta), c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; ++k) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (n < 16 && iter < 32) __atomic_fetch_add(&g_rots[n][iter], 1, __ATOMIC_RELAXED);
                if (Vt) {
                    double *Vi = Vt + i * vstep, *Vj = Vt + j * vstep;
                    for (int k = 0; k < n; ++k) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    if (n < 16) __atomic_fetch_add(&g_sweeps[n][iter < max_iter ? iter + 1 : 31], 1, __ATOMIC_RELAXED);
    for (int i = 0; i < n; ++i) {
        double sd = 0;
        for (int k = 0; k < m; ++k) {
            double t = At[i * astep + k];
            sd += t * t;
        }
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; ++i) {
        int j = i;
        for (int k = i + 1; k < n; ++k)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            if (Vt) {
                for (int k = 0; k < m; ++k) { t = At[i * astep + k]; At[i * astep + k] = At[j * astep + k]; At[j * astep + k] = t; }
                for (int k = 0; k < n; ++k) { t = Vt[i * vstep + k]; Vt[i * vstep + k] = Vt[j * vstep + k]; Vt[j * vstep + k] = t; }
            }
        }
    }
    for (int i = 0; i < n; ++i) Wout[i] = W[i];
    if (!Vt) return;
    uint64_t rng = 0x12345678;
    for (int i = 0; i < n1; ++i) {
        double sd = i < n ? W[i] : 0;
        if (sd <= minval && n < 16) __atomic_fetch_add(&g_fill[n], 1, __ATOMIC_RELAXED);
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            /* a zero singular value: a random vector, projected off the earlier rows, normalised */
            const double val0 = 1. / m;
            for (int k = 0; k < m; ++k) At[i * astep + k] = (cvq_rng_next(&rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
                for (int j = 0; j < i; ++j) {
                    sd = 0;
                    for (int k = 0; k < m; ++k) sd += At[i * astep + k] * At[j * astep + k];
                    double asum = 0;
                    for (int k = 0; k < m; ++k) {
                        double t = At[i * astep + k] - sd * At[j * astep + k];
                        At[i * astep + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; ++k) At[i * astep + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; ++k) {
                double t = At[i * astep + k];
                sd += t * t;
            }
            sd = sqrt(sd);
        }
        double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; ++k) At[i * astep + k] *= s;
    }
}

/* _SVDcompute of a square 3 x 3 S with u and vt wanted: temp_a = S^T, JacobiSVD(temp_a, w, temp_v,
 * 3, 3, 3).  ut = temp_a on exit (row k = the k-th left singular vector), vt = temp_v (row k = the
 * k-th right singular vector), w descending. */
ORC_API void cvq_svd3(const double S[9], double w[3], double ut[9], double vt[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) ut[3 * i + j] = S[3 * j + i];
    cvq_jacobi_svd(ut, 3, w, vt, 3, 3, 3, 3);
}

/* R = U V^T of the 3 x 3 SVD: sum_k ut[k][i] vt[k][j] left to right (epnp::estimate_R_and_t's
 * dot(abt_u + 3i, abt_v + 3j); cvRodrigues2's cvGEMM(U, V, GEMM_A_T)) */
static void cvq_uvt(const double ut[9], const double vt[9], double R[9]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = ut[i] * vt[j] + ut[3 + i] * vt[3 + j] + ut[6 + i] * vt[6 + j];
}

/* cv::invert(S, X, DECOMP_SVD) of a 3 x 3: SVD::compute, then SVD::backSubst with no right-hand
 * side (SVBkSbImpl_: x += v_i (u_i / w_i) over |w_i| > 2 DBL_EPSILON sum w, MatrAXPY order) */
ORC_API void cvq_invert3(const double S[9], double X[9]) {
    double w[3], ut[9], vt[9], buf[3];
    cvq_svd3(S, w, ut, vt);
    double threshold = 0;
    for (int i = 0; i < 3; ++i) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int q = 0; q < 9; ++q) X[q] = 0;
    for (int i = 0; i < 3; ++i) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        for (int j = 0; j < 3; ++j) buf[j] = ut[3 * i + j] * wi;
        for (int r = 0; r < 3; ++r) {
            double s = vt[3 * i + r];
            for (int j = 0; j < 3; ++j) X[3 * r + j] = X[3 * r + j] + s * buf[j];
        }
    }
}

/* cv::solve(A, b, x, DECOMP_SVD), A 6 x k (k <= 5, row-major), b 6 x 1: a = A^T, JacobiSVD(a, w, v,
 * 6, k), SVBkSb(6, k, w, a^T, v^T, b): x += v_i ((u_i . b) / w_i) over |w_i| > 2 DBL_EPSILON sum w */
ORC_API void cvq_solve6(const double *A, int k, const double *b, double *x) {
    double a[5 * 6], w[5], v[5 * 5];
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < 6; ++j) a[6 * i + j] = A[k * j + i];
    cvq_jacobi_svd(a, 6, w, v, 5, 6, k, k);
    double threshold = 0;
    for (int i = 0; i < k; ++i) threshold += w[i];
    threshold *= DBL_EPSILON * 2;
    for (int j = 0; j < k; ++j) x[j] = 0;
    for (int i = 0; i < k; ++i) {
        double wi = w[i];
        if (fabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < 6; ++j) s += a[6 * i + j] * b[j];
        s *= wi;
        for (int j = 0; j < k; ++j) x[j] = x[j] + s * v[5 * i + j];
    }
}

/* cvMulTransposed(src, dst, 1): dst = src^T src, each upper element a sequential sum over the
 * rows (MulTransposedR), then completeSymm */
static void cvq_mul_transposed(const double *src, int rows, int cols, double *dst) {
    for (int i = 0; i < cols; ++i)
        for (int j = i; j < cols; ++j) {
            double s = 0;
            for (int k = 0; k < rows; ++k) s += src[k * cols + i] * src[k * cols + j];
            dst[i * cols + j] = s;
        }
    for (int i = 0; i < cols; ++i)
        for (int j = 0; j < i; ++j) dst[i * cols + j] = dst[j * cols + i];
}

/* ---- epnp.cpp ---------------------------------------------------------------------------- */
typedef struct {
    int n;
    double fu, fv, uc, vc;
    double *pws, *us, *alphas, *pcs, *M, *PW0;  /* 3n, 2n, 4n, 3n, 24n, 3n doubles */
    double cws[4][3], ccs[4][3];
} cvq_epnp;

static double cvq_dot(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double cvq_dist2(const double *p1, const double *p2) {
    return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

static void cvq_choose_control_points(cvq_epnp *e) {
    const int n = e->n;
    e->cws[0][0] = e->cws[0][1] = e->cws[0][2] = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) e->cws[0][j] += e->pws[3 * i + j];
    for (int j = 0; j < 3; ++j) e->cws[0][j] /= n;
    double *PW0 = e->PW0, ptp[9], dc[3], uct[9], vt[9];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) PW0[3 * i + j] = e->pws[3 * i + j] - e->cws[0][j];
    cvq_mul_transposed(PW0, n, 3, ptp);
    cvq_svd3(ptp, dc, uct, vt);
    for (int i = 1; i < 4; ++i) {
        double k = sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; ++j) e->cws[i][j] = e->cws[0][j] + k * uct[3 * (i - 1) + j];
    }
}

static void cvq_compute_barycentric_coordinates(cvq_epnp *e) {
    double cc[9], ci[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = e->cws[j][i] - e->cws[0][i];
    cvq_invert3(cc, ci);
    for (int i = 0; i < e->n; ++i) {
        const double *pi = e->pws + 3 * i;
        double *a = e->alphas + 4 * i;
        for (int j = 0; j < 3; ++j)
            a[1 + j] = ci[3 * j] * (pi[0] - e->cws[0][0]) + ci[3 * j + 1] * (pi[1] - e->cws[0][1]) +
                       ci[3 * j + 2] * (pi[2] - e->cws[0][2]);
        a[0] = 1.0f - a[1] - a[2] - a[3];
    }
}

static void cvq_fill_M(const cvq_epnp *e, double *M, int row, const double *as, double u, double v) {
    double *M1 = M + row * 12, *M2 = M1 + 12;
    for (int i = 0; i < 4; ++i) {
        M1[3 * i] = as[i] * e->fu;
        M1[3 * i + 1] = 0.0;
        M1[3 * i + 2] = as[i] * (e->uc - u);
        M2[3 * i] = 0.0;
        M2[3 * i + 1] = as[i] * e->fv;
        M2[3 * i + 2] = as[i] * (e->vc - v);
    }
}

static void cvq_compute_L_6x10(const double *ut, double *l_6x10) {
    const double *v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
    double dv[4][6][3];
    for (int i = 0; i < 4; ++i) {
        int a = 0, b = 1;
        for (int j = 0; j < 6; ++j) {
            dv[i][j][0] = v[i][3 * a] - v[i][3 * b];
            dv[i][j][1] = v[i][3 * a + 1] - v[i][3 * b + 1];
            dv[i][j][2] = v[i][3 * a + 2] - v[i][3 * b + 2];
            b++;
            if (b > 3) { a++; b = a + 1; }
        }
    }
    for (int i = 0; i < 6; ++i) {
        double *row = l_6x10 + 10 * i;
        row[0] = cvq_dot(dv[0][i], dv[0][i]);
        row[1] = 2.0f * cvq_dot(dv[0][i], dv[1][i]);
        row[2] = cvq_dot(dv[1][i], dv[1][i]);
        row[3] = 2.0f * cvq_dot(dv[0][i], dv[2][i]);
        row[4] = 2.0f * cvq_dot(dv[1][i], dv[2][i]);
        row[5] = cvq_dot(dv[2][i], dv[2][i]);
        row[6] = 2.0f * cvq_dot(dv[0][i], dv[3][i]);
        row[7] = 2.0f * cvq_dot(dv[1][i], dv[3][i]);
        row[8] = 2.0f * cvq_dot(dv[2][i], dv[3][i]);
        row[9] = cvq_dot(dv[3][i], dv[3][i]);
    }
}

static void cvq_compute_rho(const cvq_epnp *e, double *rho) {
    rho[0] = cvq_dist2(e->cws[0], e->cws[1]);
    rho[1] = cvq_dist2(e->cws[0], e->cws[2]);
    rho[2] = cvq_dist2(e->cws[0], e->cws[3]);
    rho[3] = cvq_dist2(e->cws[1], e->cws[2]);
    rho[4] = cvq_dist2(e->cws[1], e->cws[3]);
    rho[5] = cvq_dist2(e->cws[2], e->cws[3]);
}

/* find_betas_approx_1: [B11 B12 B13 B14] */
static void cvq_betas1(const double *L, const double *rho, double *betas) {
    double l[24], b4[4];
    for (int i = 0; i < 6; ++i) {
        l[4 * i] = L[10 * i]; l[4 * i + 1] = L[10 * i + 1]; l[4 * i + 2] = L[10 * i + 3]; l[4 * i + 3] = L[10 * i + 6];
    }
    cvq_solve6(l, 4, rho, b4);
    if (b4[0] < 0) {
        betas[0] = sqrt(-b4[0]);
        betas[1] = -b4[1] / betas[0];
        betas[2] = -b4[2] / betas[0];
        betas[3] = -b4[3] / betas[0];
    } else {
        betas[0] = sqrt(b4[0]);
        betas[1] = b4[1] / betas[0];
        betas[2] = b4[2] / betas[0];
        betas[3] = b4[3] / betas[0];
    }
}

/* find_betas_approx_2: [B11 B12 B22] */
static void cvq_betas2(const double *L, const double *rho, double *betas) {
    double l[18], b3[3];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 3; ++j) l[3 * i + j] = L[10 * i + j];
    cvq_solve6(l, 3, rho, b3);
    if (b3[0] < 0) {
        betas[0] = sqrt(-b3[0]);
        betas[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
    } else {
        betas[0] = sqrt(b3[0]);
        betas[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
    }
    if (b3[1] < 0) betas[0] = -betas[0];
    betas[2] = 0.0;
    betas[3] = 0.0;
}

/* find_betas_approx_3: [B11 B12 B22 B13 B23] */
static void cvq_betas3(const double *L, const double *rho, double *betas) {
    double l[30], b5[5];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 5; ++j) l[5 * i + j] = L[10 * i + j];
    cvq_solve6(l, 5, rho, b5);
    if (b5[0] < 0) {
        betas[0] = sqrt(-b5[0]);
        betas[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
    } else {
        betas[0] = sqrt(b5[0]);
        betas[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
    }
    if (b5[1] < 0) betas[0] = -betas[0];
    betas[2] = b5[3] / betas[0];
    betas[3] = 0.0;
}

/* epnp::qr_solve (Householder, 6 x 4): returns without touching X when a column vanishes */
static void cvq_qr_solve(double *A, double *b, double *X) {
    const int nr = 6, nc = 4;
    double A1[6], A2[6];
    double *pA = A, *ppAkk = pA;
    for (int k = 0; k < nc; k++) {
        double *ppAik1 = ppAkk, eta = fabs(*ppAik1);
        for (int i = k + 1; i < nr; i++) {
            double elt = fabs(*ppAik1);
            if (eta < elt) eta = elt;
            ppAik1 += nc;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
            return;
        } else {
            double *ppAik2 = ppAkk, sum2 = 0.0, inv_eta = 1. / eta;
            for (int i = k; i < nr; i++) {
                *ppAik2 *= inv_eta;
                sum2 += *ppAik2 * *ppAik2;
                ppAik2 += nc;
            }
            double sigma = sqrt(sum2);
            if (*ppAkk < 0) sigma = -sigma;
            *ppAkk += sigma;
            A1[k] = sigma * *ppAkk;
            A2[k] = -eta * sigma;
            for (int j = k + 1; j < nc; j++) {
                double *ppAik = ppAkk, sum = 0;
                for (int i = k; i < nr; i++) {
                    sum += *ppAik * ppAik[j - k];
                    ppAik += nc;
                }
                double tau = sum / A1[k];
                ppAik = ppAkk;
                for (int i = k; i < nr; i++) {
                    ppAik[j - k] -= tau * *ppAik;
                    ppAik += nc;
                }
            }
        }
        ppAkk += nc + 1;
    }
    double *ppAjj = pA, *pb = b;
    for (int j = 0; j < nc; j++) {
        double *ppAij = ppAjj, tau = 0;
        for (int i = j; i < nr; i++) {
            tau += *ppAij * pb[i];
            ppAij += nc;
        }
        tau /= A1[j];
        ppAij = ppAjj;
        for (int i = j; i < nr; i++) {
            pb[i] -= tau * *ppAij;
            ppAij += nc;
        }
        ppAjj += nc + 1;
    }
    double *pX = X;
    pX[nc - 1] = pb[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double *ppAij = pA + i * nc + (i + 1), sum = 0;
        for (int j = i + 1; j < nc; j++) {
            sum += *ppAij * pX[j];
            ppAij++;
        }
        pX[i] = (pb[i] - sum) / A2[i];
    }
}

static void cvq_gauss_newton(const double *L, const double *rho, double betas[4]) {
    double a[24], b[6], x[4] = {0};
    for (int k = 0; k < 5; k++) {
        for (int i = 0; i < 6; i++) {
            const double *rowL = L + i * 10;
            double *rowA = a + i * 4;
            rowA[0] = 2 * rowL[0] * betas[0] + rowL[1] * betas[1] + rowL[3] * betas[2] + rowL[6] * betas[3];
            rowA[1] = rowL[1] * betas[0] + 2 * rowL[2] * betas[1] + rowL[4] * betas[2] + rowL[7] * betas[3];
            rowA[2] = rowL[3] * betas[0] + rowL[4] * betas[1] + 2 * rowL[5] * betas[2] + rowL[8] * betas[3];
            rowA[3] = rowL[6] * betas[0] + rowL[7] * betas[1] + rowL[8] * betas[2] + 2 * rowL[9] * betas[3];
            b[i] = rho[i] - (rowL[0] * betas[0] * betas[0] + rowL[1] * betas[0] * betas[1] + rowL[2] * betas[1] * betas[1] +
                             rowL[3] * betas[0] * betas[2] + rowL[4] * betas[1] * betas[2] + rowL[5] * betas[2] * betas[2] +
                             rowL[6] * betas[0] * betas[3] + rowL[7] * betas[1] * betas[3] + rowL[8] * betas[2] * betas[3] +
                             rowL[9] * betas[3] * betas[3]);
        }
        cvq_qr_solve(a, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

static void cvq_estimate_R_and_t(cvq_epnp *e, double R[3][3], double t[3]) {
    const int n = e->n;
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < 3; ++j) {
            pc0[j] += e->pcs[3 * i + j];
            pw0[j] += e->pws[3 * i + j];
        }
    for (int j = 0; j < 3; ++j) {
        pc0[j] /= n;
        pw0[j] /= n;
    }
    double abt[9] = {0}, d[3], ut[9], vt[9];
    for (int i = 0; i < n; ++i) {
        const double *pc = e->pcs + 3 * i, *pw = e->pws + 3 * i;
        for (int j = 0; j < 3; ++j) {
            abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
            abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
            abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
        }
    }
    cvq_svd3(abt, d, ut, vt);
    double Rm[9];
    cvq_uvt(ut, vt, Rm);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = Rm[3 * i + j];
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                       R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
        R[2][0] = -R[2][0];
        R[2][1] = -R[2][1];
        R[2][2] = -R[2][2];
    }
    t[0] = pc0[0] - cvq_dot(R[0], pw0);
    t[1] = pc0[1] - cvq_dot(R[1], pw0);
    t[2] = pc0[2] - cvq_dot(R[2], pw0);
}

static double cvq_reprojection_error(const cvq_epnp *e, double R[3][3], const double t[3]) {
    double sum2 = 0.0;
    for (int i = 0; i < e->n; ++i) {
        const double *pw = e->pws + 3 * i;
        double Xc = cvq_dot(R[0], pw) + t[0];
        double Yc = cvq_dot(R[1], pw) + t[1];
        double inv_Zc = 1.0 / (cvq_dot(R[2], pw) + t[2]);
        double ue = e->uc + e->fu * Xc * inv_Zc;
        double ve = e->vc + e->fv * Yc * inv_Zc;
        double u = e->us[2 * i], v = e->us[2 * i + 1];
        sum2 += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
    }
    return sum2 / e->n;
}

static double cvq_compute_R_and_t(cvq_epnp *e, const double *ut, const double *betas, double R[3][3], double t[3]) {
    /* compute_ccs */
    for (int i = 0; i < 4; ++i) e->ccs[i][0] = e->ccs[i][1] = e->ccs[i][2] = 0.0f;
    for (int i = 0; i < 4; ++i) {
        const double *v = ut + 12 * (11 - i);
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) e->ccs[j][k] += betas[i] * v[3 * j + k];
    }
    /* compute_pcs */
    for (int i = 0; i < e->n; ++i) {
        const double *a = e->alphas + 4 * i;
        double *pc = e->pcs + 3 * i;
        for (int j = 0; j < 3; ++j)
            pc[j] = a[0] * e->ccs[0][j] + a[1] * e->ccs[1][j] + a[2] * e->ccs[2][j] + a[3] * e->ccs[3][j];
    }
    /* solve_for_sign */
    if (e->pcs[2] < 0.0) {
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 3; ++j) e->ccs[i][j] = -e->ccs[i][j];
        for (int i = 0; i < e->n; ++i) {
            e->pcs[3 * i] = -e->pcs[3 * i];
            e->pcs[3 * i + 1] = -e->pcs[3 * i + 1];
            e->pcs[3 * i + 2] = -e->pcs[3 * i + 2];
        }
    }
    cvq_estimate_R_and_t(e, R, t);
    return cvq_reprojection_error(e, R, t);
}

/* epnp::compute_pose on pws (n x 3) and us (n x 2, already x * fu + uc); cam = fx fy cx cy */
static void cvq_compute_pose(cvq_epnp *e, double Rout[9], double tout[3]) {
    cvq_choose_control_points(e);
    cvq_compute_barycentric_coordinates(e);
    double *M = e->M;
    double mtm[144], d[12], vt[144];
    for (int i = 0; i < e->n; ++i) cvq_fill_M(e, M, 2 * i, e->alphas + 4 * i, e->us[2 * i], e->us[2 * i + 1]);
    cvq_mul_transposed(M, 2 * e->n, 12, mtm);
    /* cvSVD(&MtM, &D, &Ut, 0, CV_SVD_MODIFY_A | CV_SVD_U_T): JacobiSVD of MtM^T (= MtM), ut = the
       normalised rows (V is computed by _SVDcompute and dropped) */
    double ut[144];
    for (int i = 0; i < 12; ++i)
        for (int j = 0; j < 12; ++j) ut[12 * i + j] = mtm[12 * j + i];
    cvq_jacobi_svd(ut, 12, d, vt, 12, 12, 12, 12);
    double L[60], rho[6], Betas[4][4], rep_errors[4], Rs[4][3][3], ts[4][3];
    cvq_compute_L_6x10(ut, L);
    cvq_compute_rho(e, rho);
    cvq_betas1(L, rho, Betas[1]);
    cvq_gauss_newton(L, rho, Betas[1]);
    rep_errors[1] = cvq_compute_R_and_t(e, ut, Betas[1], Rs[1], ts[1]);
    cvq_betas2(L, rho, Betas[2]);
    cvq_gauss_newton(L, rho, Betas[2]);
    rep_errors[2] = cvq_compute_R_and_t(e, ut, Betas[2], Rs[2], ts[2]);
    cvq_betas3(L, rho, Betas[3]);
    cvq_gauss_newton(L, rho, Betas[3]);
    rep_errors[3] = cvq_compute_R_and_t(e, ut, Betas[3], Rs[3], ts[3]);
    int N = 1;
    if (rep_errors[2] < rep_errors[1]) N = 2;
    if (rep_errors[3] < rep_errors[N]) N = 3;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) Rout[3 * i + j] = Rs[N][i][j];
        tout[i] = ts[N][i];
    }
}

/* cvRodrigues2, 3 x 3 -> 3 x 1 (calibration.cpp): checkRange(-100, 100), R = U V^T of cvSVD,
 * the angle from the antisymmetric part, the theta ~ pi branch */
ORC_API void orc_cv_rodrigues_m2v(const double Rin[9], double r[3]) {
    double R[9], w[3], ut[9], vt[9];
    for (int k = 0; k < 9; ++k) {
        if (!(Rin[k] >= -100.0 && Rin[k] < 100.0)) { r[0] = r[1] = r[2] = 0; return; }
    }
    cvq_svd3(Rin, w, ut, vt);
    cvq_uvt(ut, vt, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = orc_rd_acos(c);
    if (s < 1e-5) {
        double t;
        if (c > 0)
            rx = ry = rz = 0;
        else {
            t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    r[0] = rx;
    r[1] = ry;
    r[2] = rz;
}

/* cvRodrigues2, 3 x 1 -> 3 x 3: R[k] = c I[k] + c1 rrt[k] + s [r]x[k] */
ORC_API void orc_cv_rodrigues_v2m(const double rin[3], double R[9]) {
    double rx = rin[0], ry = rin[1], rz = rin[2];
    double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    static const double I[] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    double s, c;
    orc_rd_sincos(theta, &s, &c);
    double c1 = 1. - c;
    double itheta = theta ? 1. / theta : 0.;
    rx *= itheta;
    ry *= itheta;
    rz *= itheta;
    double rrt[] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    double r_x[] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * r_x[k];
}

ORC_API void orc_cv_rvec_roundtrip(double R[9]) {
    double rv[3];
    orc_cv_rodrigues_m2v(R, rv);
    orc_cv_rodrigues_v2m(rv, R);
}

/* solvePnP(opoints, ipoints, K, 0, SOLVEPNP_EPNP) on n points: f32 object points, f32 pixels
 * (solvePnPRansac's CV_32F copies), K = (fx, fy, cx, cy).  undistortPoints to f32 normalised
 * coordinates, then epnp.  Returns 1 (OpenCV's EPnP always reports a pose; NaN propagates). */
ORC_API int orc_cv_epnp(const float *X, const float *Y, const float *Z, const float *U, const float *V,
                        const int32_t *idx, int n, const double cam[4], double R[9], double t[3]) {
    cvq_epnp e;
    if (n < 4) return 0;
    double *buf = (double *)malloc(sizeof(double) * 39 * (size_t)n);
    if (!buf) return 0;
    e.pws = buf; e.us = buf + 3 * n; e.alphas = buf + 5 * n; e.pcs = buf + 9 * n; e.M = buf + 12 * n;
    e.PW0 = buf + 36 * n;
    const double fx = cam[0], fy = cam[1], cx = cam[2], cy = cam[3];
    const double ifx = 1. / fx, ify = 1. / fy;
    e.n = n;
    e.fu = fx; e.fv = fy; e.uc = cx; e.vc = cy;
    for (int i = 0; i < n; ++i) {
        const int p = idx ? idx[i] : i;
        e.pws[3 * i] = X[p];
        e.pws[3 * i + 1] = Y[p];
        e.pws[3 * i + 2] = Z[p];
        /* cvUndistortPointsInternal: x = (u - cx) * ifx, stored as CV_32F (through a volatile:
           gcc 11's -O3 SLP vectoriser dropped this rounding) */
        volatile float xn = (float)(((double)U[p] - cx) * ifx);
        volatile float yn = (float)(((double)V[p] - cy) * ify);
        /* epnp::init_points: us = x * fu + uc */
        e.us[2 * i] = (double)xn * e.fu + e.uc;
        e.us[2 * i + 1] = (double)yn * e.fv + e.vc;
    }
    cvq_compute_pose(&e, R, t);
    free(buf);
    return 1;
}
