// rsac_cvepnp.h -- OpenCV's operation sequence for solvePnPRansac's default minimal solver, host +
// device (the GPU kernels k_cvepnp5_a / _svd / _c and the host twin rsac_pnp_epnp_minimal).
//
// cv2.solvePnPRansac with the default flags (main_v1.py:497-502, testpro-K.py:72-75,
// testpro.py:536-541, test_pro.py:515-520) solves each 5-point subset with
// solvePnP(..., SOLVEPNP_EPNP) and keeps the model as (rvec, tvec) ([OpenCV 4.x, unvendored]
// solvepnp.cpp solvePnPRansac / PnPRansacCallback / solvePnPGeneric).  Restated here step by
// step, every sum left to right as those sources write it, no fused operation (the library is
// built with -ffp-contract=off; OpenCV's x86 baseline has no FMA):
//   undistortPoints to CV_32F normalised coordinates, epnp::init_points (x * fu + uc),
//   choose_control_points (raw centroid, cvMulTransposed, cvSVD), compute_barycentric_coordinates
//   (cvInvert CV_SVD), fill_M + cvMulTransposed + cvSVD(M^T M, U_T), compute_L_6x10,
//   compute_rho, find_betas_approx_1..3 (cvSolve CV_SVD), gauss_newton (epnp::qr_solve),
//   compute_R_and_t (ccs, pcs, solve_for_sign, estimate_R_and_t by cvSVD, reprojection_error),
//   the first lowest error; then cvRodrigues2 both ways (cvSVD + cvGEMM; c I + c1 r r^T + s [r]x).
// lapack.cpp JacobiSVDImpl_<double> is the decomposition behind every cvSVD / cvSolve / cvInvert.
// The oracle restates the same steps independently (oracle/cv_epnp.c); GPU == oracle bit for bit.
// libm's hypot is restated as glibc 2.35's algorithm (hypot_glibc; bit-identical to this host's
// libm, tests/test_cv_epnp.py), cos / sin / acos as rsac_math.h rodr_*.
#pragma once

#include "rsac_math.h"

namespace rsac {
namespace cvq {

constexpr double kDblEps = 0x1p-52;                 // DBL_EPSILON
constexpr double kDblMin = 0x1p-1022;               // DBL_MIN
constexpr double kSvdEps = 0x1p-52 * 10;            // JacobiSVD's eps (DBL_EPSILON * 10)

// hypot(x, y) as glibc 2.35 computes it on x86-64 (e_hypot.c: Borges' non-FMA kernel with glibc's
// scaling of huge / tiny operands): rounded + - * / sqrt only, so host, device and the oracle
// (oracle/cv_epnp.c cvq_hypot) agree; tests/test_cv_epnp.py holds it to this host's libm
RSAC_HD double hypot_kernel(double ax, double ay) {
    double t1, t2;
    double h = dsqrt(ax * ax + ay * ay);
    if (h <= 2.0 * ay) {
        const double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        const double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}
RSAC_HD double hypot_glibc(double x, double y) {
    if (!dfinite(x) || !dfinite(y)) {
        if (__builtin_isinf(x) || __builtin_isinf(y)) return __builtin_huge_val();
        return x + y;
    }
    x = dabs(x);
    y = dabs(y);
    const double ax = x < y ? y : x, ay = x < y ? x : y;
    if (ax > 0x1p+511) {
        if (ay <= ax * 0x1p-54) return ax + ay;
        return hypot_kernel(ax * 0x1p-600, ay * 0x1p-600) / 0x1p-600;
    }
    if (ay < 0x1p-511) {
        if (ax >= ay / 0x1p-54) return ax + ay;
        return hypot_kernel(ax / 0x1p-600, ay / 0x1p-600) * 0x1p-600;
    }
    if (ay <= ax * 0x1p-54) return ax + ay;
    return hypot_kernel(ax, ay);
}

// JacobiSVDImpl_'s rotation of the pair (a = W[i], b = W[j], p = Ai . Aj), p already doubled:
// (c, s) by the hypot form and its two branches
RSAC_HD void svd_rotation(double p, double a, double b, double &c, double &s) {
    const double beta = a - b, gamma = hypot_glibc(p, beta);
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        s = dsqrt(delta / gamma);
        c = p / (gamma * s * 2);
    } else {
        c = dsqrt((gamma + beta) / (gamma * 2));
        s = p / (gamma * c * 2);
    }
}

// Branch-free forms of hypot_glibc and svd_rotation (the GPU's anti-diagonal JacobiSVD runs up to
// six rotations side by side, and a branch per rotation would serialise them): every case's
// operations are computed and the one the branchy form takes is selected, so the bits are equal.
// FAST: the roots and quotients by the fast cores (dsqrt_fast / ddiv_fast), valid under
// svd_rotation_sel's range condition below.
template <bool FAST>
RSAC_HD double hypot_glibc_sel_t(double x, double y) {
    const double fx = dabs(x), fy = dabs(y);
    const double ax = fx < fy ? fy : fx, ay = fx < fy ? fx : fy;
    if constexpr (FAST) {
        // under svd_rotation_sel's range condition x, y are finite and ax lies in [2^-250, 2^202]:
        // never huge, and a tiny ay (< 2^-511) is below ax 2^-54, glibc's ax + ay case
        const double h0 = dsqrt_fast(ax * ax + ay * ay);
        const double d1 = h0 - ay, d2 = h0 - ax;
        const double t1a = ax * (2.0 * d1 - ax), t2a = (d1 - 2.0 * (ax - ay)) * d1;
        const double t1b = 2.0 * d2 * (ax - 2.0 * ay), t2b = (4.0 * d2 - ay) * ay + d2 * d2;
        const bool first = h0 <= 2.0 * ay;
        const double t1 = first ? t1a : t1b, t2 = first ? t2a : t2b;
        const double h = h0 - ddiv_fast(t1 + t2, 2.0 * h0);
        return ay <= ax * 0x1p-54 ? ax + ay : h;
    }
    const bool huge = ax > 0x1p+511, tiny = !huge && ay < 0x1p-511;
    // glibc: kernel(ax SCALE, ay SCALE) / SCALE for huge operands, kernel(ax / SCALE, ay / SCALE) SCALE
    // for tiny ones (SCALE = 2^-600): exact power-of-two scalings either way
    const double up = huge ? 0x1p-600 : tiny ? 0x1p+600 : 1.0, down = huge ? 0x1p+600 : tiny ? 0x1p-600 : 1.0;
    const double sx = ax * up, sy = ay * up;
    const double h0 = dsqrt(sx * sx + sy * sy);
    const double d1 = h0 - sy, d2 = h0 - sx;
    const double t1a = sx * (2.0 * d1 - sx), t2a = (d1 - 2.0 * (sx - sy)) * d1;
    const double t1b = 2.0 * d2 * (sx - 2.0 * sy), t2b = (4.0 * d2 - sy) * sy + d2 * d2;
    const bool first = h0 <= 2.0 * sy;
    const double t1 = first ? t1a : t1b, t2 = first ? t2a : t2b;
    const double h = (h0 - (t1 + t2) / (2.0 * h0)) * down;
    const bool small = huge ? ay <= ax * 0x1p-54 : tiny ? ax >= ay / 0x1p-54 : ay <= ax * 0x1p-54;
    double r = small ? ax + ay : h;
    if (!dfinite(x) || !dfinite(y)) r = (__builtin_isinf(x) || __builtin_isinf(y)) ? __builtin_huge_val() : x + y;
    return r;
}
RSAC_HD double hypot_glibc_sel(double x, double y) { return hypot_glibc_sel_t<false>(x, y); }
template <bool FAST>
RSAC_HD void svd_rotation_sel_t(double p, double a, double b, double &c, double &s) {
    const double beta = a - b, gamma = hypot_glibc_sel_t<FAST>(p, beta);
    const bool neg = beta < 0;
    // beta < 0: s = sqrt(((gamma - beta) 0.5) / gamma), c = p / (gamma s 2); else
    // c = sqrt((gamma + beta) / (gamma 2)), s = p / (gamma c 2)
    const double num = neg ? (gamma - beta) * 0.5 : gamma + beta, den = neg ? gamma : gamma * 2;
    double r, o;
    if constexpr (FAST) {
        r = dsqrt_fast(ddiv_fast(num, den));
        o = ddiv_fast(p, gamma * r * 2);
    } else {
        r = dsqrt(num / den);
        o = p / (gamma * r * 2);
    }
    c = neg ? o : r;
    s = neg ? r : o;
}
// JacobiSVDImpl_'s (c, s) for the pair (p doubled, a = W[i], b = W[j]); `need` = false: a skipped
// pair, whose (c, s) the caller discards.  On the device (RSAC_FAST_F64) the fast cores run when
// both norms lie in [2^-200, 2^200]: then |p| <= sqrt(ab) (Cauchy-Schwarz, up to rounding) and a
// pair that is not skipped has |p| > 10 DBL_EPSILON sqrt(ab) > 2^-250, so gamma, h0 lie in
// [2^-248, 2^203], the root arguments in [2^-496, 2^404] or [1/2, 1], every operand of a quotient
// (the kernel's t1 + t2 a multiple of 2^-708 or zero, whose quotient only h0 - q sees) inside the
// fast division's range, and each result equals the IEEE form's.  A lane outside the range that
// needs its result runs the IEEE form in a branch (rare: the norms are squared row norms of
// M^T M or of L's 6 x K columns).
RSAC_HD void svd_rotation_sel(double p, double a, double b, double &c, double &s, bool need = true) {
#if RSAC_DEV_FAST_F64
    const bool in = (a >= 0x1p-200) & (a <= 0x1p+200) & (b >= 0x1p-200) & (b <= 0x1p+200);
    if (need & !in) {
        asm volatile("" ::: "memory");  // a branch, not a select
        svd_rotation_sel_t<false>(p, a, b, c, s);
    } else {
        svd_rotation_sel_t<true>(p, a, b, c, s);
    }
#else
    svd_rotation_sel_t<false>(p, a, b, c, s);
#endif
}

RSAC_HD uint32_t rng_next(uint64_t &st) {
    st = (uint64_t)(uint32_t)st * 4164903690u + (st >> 32);
    return (uint32_t)st;
}

// lapack.cpp JacobiSVDImpl_<double>(At, W, Vt, m = M, n = N, n1 = N, DBL_MIN, 10 DBL_EPSILON) with Vt
// (every caller here passes one: _SVDcompute with u wanted, cv::solve): At's N rows (the columns
// of the decomposed matrix) are orthogonalised in cyclic pair order, W = their norms, sorted
// descending with the rows of At and Vt, the rows of At normalised (a zero one replaced by a
// random direction orthogonal to the earlier rows).
// n1 (<= N): the rows normalised on exit (OpenCV's n1 = n; a zero-padded caller passes its real
// column count).  Device code takes the branch-free rotation (svd_rotation_sel, selects for a
// skipped pair): the same bits, and the lanes of a wave do not diverge on every pair.
template <int M, int N>
RSAC_HD void jacobi_svd(double (&At)[N][M], double (&Wout)[N], double (&Vt)[N][N], int n1 = N) {
    double W[N];
    constexpr int max_iter = M > 30 ? M : 30;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) sd += At[i][k] * At[i][k];
        W[i] = sd;
#pragma unroll
        for (int k = 0; k < N; ++k) Vt[i][k] = 0;
        Vt[i][i] = 1;
    }
    for (int iter = 0; iter < max_iter; ++iter) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; ++i)
#pragma unroll
            for (int j = i + 1; j < N; ++j) {
                const double a = W[i], b = W[j];
                double p = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) p += At[i][k] * At[j][k];
#if RSAC_DEV_FAST_F64
                // the skip test and the rotation by the fast cores when both norms lie in
                // svd_rotation_sel's range (then a b in [2^-400, 2^400]); a pair with p == 0 and a
                // b not NaN skips exactly (0 <= eps sqrt(ab)), as every pair of a zero-padded column
                // does; any other lane runs the IEEE test and rotation in a branch
                bool skip;
                double c, s;
                {
                    const double ab = a * b;
                    const bool fastc = (a >= 0x1p-200) & (a <= 0x1p+200) & (b >= 0x1p-200) & (b <= 0x1p+200);
                    const bool trivial = (p == 0.0) & (ab == ab);
                    if (!fastc & !trivial) {
                        asm volatile("" ::: "memory");  // a branch, not a select
                        skip = dabs(p) <= kSvdEps * dsqrt(ab);
                        svd_rotation_sel_t<false>(p * 2, a, b, c, s);
                    } else {
                        skip = fastc ? dabs(p) <= kSvdEps * dsqrt_fast(ab) : true;
                        svd_rotation_sel_t<true>(p * 2, a, b, c, s);
                    }
                }
#else
                const bool skip = dabs(p) <= kSvdEps * dsqrt(a * b);
#ifndef __HIP_DEVICE_COMPILE__
                if (skip) continue;
#endif
                p *= 2;
                double c, s;
#ifdef __HIP_DEVICE_COMPILE__
                svd_rotation_sel(p, a, b, c, s, !skip);  // a skipped pair's (c, s) are discarded
#else
                svd_rotation(p, a, b, c, s);
#endif
#endif
                double na = 0, nb = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    const double t0 = c * At[i][k] + s * At[j][k];
                    const double t1 = -s * At[i][k] + c * At[j][k];
                    At[i][k] = skip ? At[i][k] : t0;
                    At[j][k] = skip ? At[j][k] : t1;
                    na += t0 * t0;
                    nb += t1 * t1;
                }
                W[i] = skip ? a : na;
                W[j] = skip ? b : nb;
                changed = changed || !skip;
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    const double t0 = c * Vt[i][k] + s * Vt[j][k];
                    const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                    Vt[i][k] = skip ? Vt[i][k] : t0;
                    Vt[j][k] = skip ? Vt[j][k] : t1;
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) sd += At[i][k] * At[i][k];
        W[i] = dsqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < N - 1; ++i) {
        int j = i;
#pragma unroll
        for (int k = i + 1; k < N; ++k)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            // row j (j > i) swapped with row i; static indices through a select over the candidates
#pragma unroll
            for (int q = i + 1; q < N; ++q)
                if (q == j) {
                    double t = W[i]; W[i] = W[q]; W[q] = t;
#pragma unroll
                    for (int k = 0; k < M; ++k) { t = At[i][k]; At[i][k] = At[q][k]; At[q][k] = t; }
#pragma unroll
                    for (int k = 0; k < N; ++k) { t = Vt[i][k]; Vt[i][k] = Vt[q][k]; Vt[q][k] = t; }
                }
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) Wout[i] = W[i];
    uint64_t rng = 0x12345678;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (i >= n1) break;
        double sd = W[i];
        for (int ii = 0; ii < 100 && sd <= kDblMin; ii++) {
            const double val0 = 1. / M;
#pragma unroll
            for (int k = 0; k < M; ++k) At[i][k] = (rng_next(rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) sd += At[i][k] * At[j][k];
                    double asum = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) {
                        const double t = At[i][k] - sd * At[j][k];
                        At[i][k] = t;
                        asum += dabs(t);
                    }
                    asum = asum > kSvdEps * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) At[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < M; ++k) sd += At[i][k] * At[i][k];
            sd = dsqrt(sd);
        }
        const double s = sd > kDblMin ? 1 / sd : 0.;
#pragma unroll
        for (int k = 0; k < M; ++k) At[i][k] *= s;
    }
}

// _SVDcompute of a 3 x 3 S (u and vt wanted): JacobiSVD of S^T; ut[k] = the k-th left singular
// vector, vt[k] the k-th right one, w descending
RSAC_HD void svd3(const double S[9], double (&w)[3], double (&ut)[3][3], double (&vt)[3][3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) ut[i][j] = S[3 * j + i];
    jacobi_svd<3, 3>(ut, w, vt);
}

// U V^T of svd3: sum_k ut[k][i] vt[k][j] left to right (estimate_R_and_t's dot(abt_u + 3i,
// abt_v + 3j); cvRodrigues2's cvGEMM(U, V, GEMM_A_T))
RSAC_HD void uvt3(const double (&ut)[3][3], const double (&vt)[3][3], double R[9]) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) R[3 * i + j] = ut[0][i] * vt[0][j] + ut[1][i] * vt[1][j] + ut[2][i] * vt[2][j];
}

// cv::invert(S, X, DECOMP_SVD), 3 x 3: x += v_i (u_i / w_i) over |w_i| > 2 DBL_EPSILON sum w
// (SVBkSbImpl_ with no right-hand side, MatrAXPY order)
RSAC_HD void invert3(const double S[9], double X[9]) {
    double w[3], ut[3][3], vt[3][3], buf[3];
    svd3(S, w, ut, vt);
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) threshold += w[i];
    threshold *= kDblEps * 2;
#pragma unroll
    for (int q = 0; q < 9; ++q) X[q] = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double wi = w[i];
        if (dabs(wi) <= threshold) continue;
        wi = 1 / wi;
#pragma unroll
        for (int j = 0; j < 3; ++j) buf[j] = ut[i][j] * wi;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double s = vt[i][r];
#pragma unroll
            for (int j = 0; j < 3; ++j) X[3 * r + j] = X[3 * r + j] + s * buf[j];
        }
    }
}

// cv::solve(A, b, x, DECOMP_SVD), A 6 x K: a = A^T, JacobiSVD(a, w, v, 6, K), then
// x += v_i ((u_i . b) / w_i) over |w_i| > 2 DBL_EPSILON sum w (SVBkSbImpl_, nb = 1)
template <int K>
RSAC_HD void solve6(const double (&A)[6][K], const double (&b)[6], double (&x)[K]) {
    double a[K][6], w[K], v[K][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) a[i][j] = A[j][i];
    jacobi_svd<6, K>(a, w, v);
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) threshold += w[i];
    threshold *= kDblEps * 2;
#pragma unroll
    for (int j = 0; j < K; ++j) x[j] = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double wi = w[i];
        if (dabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) s += a[i][j] * b[j];
        s *= wi;
#pragma unroll
        for (int j = 0; j < K; ++j) x[j] = x[j] + s * v[i][j];
    }
}

// solve6<K> on a 6 x 5 matrix whose columns K .. 4 are zero (x[K..4] = 0 on return): the padded
// columns' pairs are all skipped (p = +0 <= eps sqrt(a 0) = 0), they sort last with norm 0, only
// the first K rows are normalised (n1 = K), and they add +0 to the threshold and nothing to x, so
// x[0..K-1] are solve6<K>'s bits.  One instruction stream for the three beta estimates.
RSAC_HD void solve6_padded(const double (&A)[6][5], int K, const double (&b)[6], double (&x)[5]) {
    double a[5][6], w[5], v[5][5];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) a[i][j] = A[j][i];
    jacobi_svd<6, 5>(a, w, v, K);
    double threshold = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) threshold += w[i];
    threshold *= kDblEps * 2;
#pragma unroll
    for (int j = 0; j < 5; ++j) x[j] = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        double wi = w[i];
        if (dabs(wi) <= threshold) continue;
        wi = 1 / wi;
        double s = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) s += a[i][j] * b[j];
        s *= wi;
#pragma unroll
        for (int j = 0; j < 5; ++j) x[j] = x[j] + s * v[i][j];
    }
}

RSAC_HD double dot3(const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// epnp::qr_solve of the 6 x 4 Gauss-Newton system (Householder): a vanishing column returns
// with X untouched
RSAC_HD void qr_solve(double (&A)[6][4], double (&b)[6], double (&X)[4]) {
    double A1[4], A2[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        double eta = dabs(A[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++) {
            // OpenCV reads the pointer before advancing it: row k again, then rows k+1 .. 4
            const double elt = dabs(A[i - 1][k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;
        double sum2 = 0.0;
        const double inv_eta = 1. / eta;
#pragma unroll
        for (int i = k; i < 6; i++) {
            A[i][k] *= inv_eta;
            sum2 += A[i][k] * A[i][k];
        }
        double sigma = dsqrt(sum2);
        if (A[k][k] < 0) sigma = -sigma;
        A[k][k] += sigma;
        A1[k] = sigma * A[k][k];
        A2[k] = -eta * sigma;
#pragma unroll
        for (int j = k + 1; j < 4; j++) {
            double sum = 0;
#pragma unroll
            for (int i = k; i < 6; i++) sum += A[i][k] * A[i][j];
            const double tau = sum / A1[k];
#pragma unroll
            for (int i = k; i < 6; i++) A[i][j] -= tau * A[i][k];
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        double tau = 0;
#pragma unroll
        for (int i = j; i < 6; i++) tau += A[i][j] * b[i];
        tau /= A1[j];
#pragma unroll
        for (int i = j; i < 6; i++) b[i] -= tau * A[i][j];
    }
    X[3] = b[3] / A2[3];
#pragma unroll
    for (int i = 2; i >= 0; i--) {
        double sum = 0;
#pragma unroll
        for (int j = i + 1; j < 4; j++) sum += A[i][j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

// epnp::gauss_newton: 5 steps; x persists across the steps (a singular step re-adds the last one)
RSAC_HD void gauss_newton(const double (&L)[6][10], const double (&rho)[6], double (&be)[4]) {
    double x[4] = {0, 0, 0, 0};
    for (int k = 0; k < 5; k++) {
        double A[6][4], b[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            const double *r = L[i];
            A[i][0] = 2 * r[0] * be[0] + r[1] * be[1] + r[3] * be[2] + r[6] * be[3];
            A[i][1] = r[1] * be[0] + 2 * r[2] * be[1] + r[4] * be[2] + r[7] * be[3];
            A[i][2] = r[3] * be[0] + r[4] * be[1] + 2 * r[5] * be[2] + r[8] * be[3];
            A[i][3] = r[6] * be[0] + r[7] * be[1] + r[8] * be[2] + 2 * r[9] * be[3];
            b[i] = rho[i] - (r[0] * be[0] * be[0] + r[1] * be[0] * be[1] + r[2] * be[1] * be[1] + r[3] * be[0] * be[2] +
                             r[4] * be[1] * be[2] + r[5] * be[2] * be[2] + r[6] * be[0] * be[3] + r[7] * be[1] * be[3] +
                             r[8] * be[2] * be[3] + r[9] * be[3] * be[3]);
        }
        qr_solve(A, b, x);
#pragma unroll
        for (int i = 0; i < 4; i++) be[i] += x[i];
    }
}

// find_betas_approx_1..3 on one instruction stream (the GPU's three lanes per hypothesis): the
// column subset of L zero-padded to 6 x 5 (solve6_padded), then OpenCV's sign rules by selects
RSAC_HD void betas_approx_padded(int approx, const double (&L)[6][10], const double (&rho)[6], double (&be)[4]) {
    double l[6][5], x[5];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        l[i][0] = L[i][0];
        l[i][1] = L[i][1];
        l[i][2] = approx == 1 ? L[i][3] : L[i][2];
        l[i][3] = approx == 1 ? L[i][6] : approx == 3 ? L[i][3] : 0.0;
        l[i][4] = approx == 3 ? L[i][4] : 0.0;
    }
    solve6_padded(l, approx == 1 ? 4 : approx == 2 ? 3 : 5, rho, x);
    if (approx == 1) {
        const bool neg = x[0] < 0;
        be[0] = dsqrt(neg ? -x[0] : x[0]);
        be[1] = (neg ? -x[1] : x[1]) / be[0];
        be[2] = (neg ? -x[2] : x[2]) / be[0];
        be[3] = (neg ? -x[3] : x[3]) / be[0];
    } else {
        // approx 2 (b3 = x[0..2]) and 3 (b5 = x[0..4]) share the first two betas' rule
        if (x[0] < 0) {
            be[0] = dsqrt(-x[0]);
            be[1] = (x[2] < 0) ? dsqrt(-x[2]) : 0.0;
        } else {
            be[0] = dsqrt(x[0]);
            be[1] = (x[2] > 0) ? dsqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) be[0] = -be[0];
        be[2] = approx == 3 ? x[3] / be[0] : 0.0;
        be[3] = 0.0;
    }
}

// find_betas_approx_1..3 (approx = 1, 2, 3): the 6 x 4 / 6 x 3 / 6 x 5 column subsets of L,
// cvSolve(CV_SVD), OpenCV's sign rules
RSAC_HD void betas_approx(int approx, const double (&L)[6][10], const double (&rho)[6], double (&be)[4]) {
    if (approx == 1) {
        double l[6][4], b4[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            l[i][0] = L[i][0]; l[i][1] = L[i][1]; l[i][2] = L[i][3]; l[i][3] = L[i][6];
        }
        solve6<4>(l, rho, b4);
        if (b4[0] < 0) {
            be[0] = dsqrt(-b4[0]);
            be[1] = -b4[1] / be[0];
            be[2] = -b4[2] / be[0];
            be[3] = -b4[3] / be[0];
        } else {
            be[0] = dsqrt(b4[0]);
            be[1] = b4[1] / be[0];
            be[2] = b4[2] / be[0];
            be[3] = b4[3] / be[0];
        }
    } else if (approx == 2) {
        double l[6][3], b3[3];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) l[i][j] = L[i][j];
        solve6<3>(l, rho, b3);
        if (b3[0] < 0) {
            be[0] = dsqrt(-b3[0]);
            be[1] = (b3[2] < 0) ? dsqrt(-b3[2]) : 0.0;
        } else {
            be[0] = dsqrt(b3[0]);
            be[1] = (b3[2] > 0) ? dsqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) be[0] = -be[0];
        be[2] = 0.0;
        be[3] = 0.0;
    } else {
        double l[6][5], b5[5];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 5; ++j) l[i][j] = L[i][j];
        solve6<5>(l, rho, b5);
        if (b5[0] < 0) {
            be[0] = dsqrt(-b5[0]);
            be[1] = (b5[2] < 0) ? dsqrt(-b5[2]) : 0.0;
        } else {
            be[0] = dsqrt(b5[0]);
            be[1] = (b5[2] > 0) ? dsqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) be[0] = -be[0];
        be[2] = b5[3] / be[0];
        be[3] = 0.0;
    }
}

// cvRodrigues2 3 x 3 -> 3 x 1: checkRange(-100, 100) else zeros, R = U V^T (cvSVD + cvGEMM), the
// angle from the antisymmetric part, the theta ~ pi branch
RSAC_HD void rodrigues_m2v(const double Rin[9], double r[3]) {
    bool in_range = true;
#pragma unroll
    for (int k = 0; k < 9; ++k) in_range = in_range && (Rin[k] >= -100.0 && Rin[k] < 100.0);
    if (!in_range) {
        r[0] = r[1] = r[2] = 0.0;
        return;
    }
    double w[3], ut[3][3], vt[3][3], R[9];
    svd3(Rin, w, ut, vt);
    uvt3(ut, vt, R);
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = dsqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = rodr_acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t;
            t = (R[0] + 1) * 0.5;
            rx = dsqrt(t > 0. ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = dsqrt(t > 0. ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = dsqrt(t > 0. ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (dabs(rx) < dabs(ry) && dabs(rx) < dabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= dsqrt(rx * rx + ry * ry + rz * rz);
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

// cvRodrigues2 3 x 1 -> 3 x 3: R[k] = c I[k] + c1 rrt[k] + s [r]x[k]
RSAC_HD void rodrigues_v2m(const double rin[3], double R[9]) {
    double rx = rin[0], ry = rin[1], rz = rin[2];
    const double theta = dsqrt(rx * rx + ry * ry + rz * rz);
    if (theta < kDblEps) {
#pragma unroll
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double s, c;
    rodr_sincos(theta, s, c);
    const double c1 = 1. - c;
    const double itheta = theta ? 1. / theta : 0.;
    rx *= itheta;
    ry *= itheta;
    rz *= itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double r_x[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = c * I[k] + c1 * rrt[k] + s * r_x[k];
}

// the rotation computeError projects with: Rodrigues(Rodrigues(R)) (RSAC_F_RVEC_ROUNDTRIP)
RSAC_HD void rvec_roundtrip(double R[9]) {
    double rv[3];
    rodrigues_m2v(R, rv);
    rodrigues_v2m(rv, R);
}

// ---- epnp.cpp on the 5 sampled points ----------------------------------------------------------
constexpr int kMtmUpper = 78;  // upper triangle of the 12 x 12 M^T M, row by row

struct Epnp5 {
    double fu, fv, uc, vc;
    double pws[5][3], us[5][2], alphas[5][4], cws[4][3];
};

// solvePnPGeneric's undistortPoints (CV_32F out) + epnp::init_points on the sample (f32 inputs:
// solvePnPRansac's CV_32F copies)
RSAC_HD void epnp5_init(const float (&X)[5], const float (&Y)[5], const float (&Z)[5], const float (&U)[5],
                        const float (&V)[5], const Cam &k, Epnp5 &e) {
    e.fu = k.fx;
    e.fv = k.fy;
    e.uc = k.cx;
    e.vc = k.cy;
    const double ifx = 1. / k.fx, ify = 1. / k.fy;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        e.pws[i][0] = X[i];
        e.pws[i][1] = Y[i];
        e.pws[i][2] = Z[i];
        const float xn = (float)(((double)U[i] - k.cx) * ifx);
        const float yn = (float)(((double)V[i] - k.cy) * ify);
        e.us[i][0] = (double)xn * e.fu + e.uc;
        e.us[i][1] = (double)yn * e.fv + e.vc;
    }
}

// choose_control_points + compute_barycentric_coordinates
RSAC_HD void epnp5_frame(Epnp5 &e) {
    e.cws[0][0] = e.cws[0][1] = e.cws[0][2] = 0;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) e.cws[0][j] += e.pws[i][j];
#pragma unroll
    for (int j = 0; j < 3; ++j) e.cws[0][j] /= 5;
    double pw0[5][3], ptp[9];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) pw0[i][j] = e.pws[i][j] - e.cws[0][j];
    // cvMulTransposed(PW0, PW0^T PW0, 1): sequential sums over the rows, then the lower mirror
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) {
            double s = 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) s += pw0[k][i] * pw0[k][j];
            ptp[3 * i + j] = s;
            ptp[3 * j + i] = s;
        }
    double dc[3], uct[3][3], vt[3][3];
    svd3(ptp, dc, uct, vt);
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        const double kk = dsqrt(dc[i - 1] / 5);
#pragma unroll
        for (int j = 0; j < 3; ++j) e.cws[i][j] = e.cws[0][j] + kk * uct[i - 1][j];
    }
    double cc[9], ci[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = e.cws[j][i] - e.cws[0][i];
    invert3(cc, ci);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        double *a = e.alphas[i];
#pragma unroll
        for (int j = 0; j < 3; ++j)
            a[1 + j] = ci[3 * j] * (e.pws[i][0] - e.cws[0][0]) + ci[3 * j + 1] * (e.pws[i][1] - e.cws[0][1]) +
                       ci[3 * j + 2] * (e.pws[i][2] - e.cws[0][2]);
        a[0] = 1.0 - a[1] - a[2] - a[3];
    }
}

// M^T M of fill_M's 10 x 12 M (cvMulTransposed: element (c, d), c <= d, the sum over the rows in
// order).  Row 2i of M is (a_ia fu, 0, a_ia (uc - u_i)) per control point a, row 2i + 1
// (0, a_ia fv, a_ia (vc - v_i)); a product with a structural zero is +-0 and leaves a sum that
// starts at +0 unchanged, so only the non-zero terms are added, in row order.
RSAC_HD void epnp5_mtm(const Epnp5 &e, double *mtm /* kMtmUpper */) {
    double m0[5][12], m1[5][12];  // the non-structural entries of rows 2i and 2i + 1 (0 elsewhere)
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            m0[i][3 * a] = e.alphas[i][a] * e.fu;
            m0[i][3 * a + 1] = 0.0;
            m0[i][3 * a + 2] = e.alphas[i][a] * (e.uc - e.us[i][0]);
            m1[i][3 * a] = 0.0;
            m1[i][3 * a + 1] = e.alphas[i][a] * e.fv;
            m1[i][3 * a + 2] = e.alphas[i][a] * (e.vc - e.us[i][1]);
        }
    int q = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c)
#pragma unroll
        for (int d = c; d < 12; ++d, ++q) {
            const int x = c % 3, y = d % 3;
            const bool r0 = x != 1 && y != 1;  // row 2i contributes: neither column is a fv column
            const bool r1 = x != 0 && y != 0;  // row 2i + 1 contributes: neither is a fu column
            double s = 0;
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                if (r0) s += m0[i][c] * m0[i][d];
                if (r1) s += m1[i][c] * m1[i][d];
            }
            mtm[q] = s;
        }
}

// compute_L_6x10 from the eigenvector rows v[0..3] = ut rows 11, 10, 9, 8
RSAC_HD void epnp_l6x10(const double (&v)[4][12], double (&L)[6][10]) {
    double dv[4][6][3];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int a = 0, b = 1;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            dv[i][j][0] = v[i][3 * a] - v[i][3 * b];
            dv[i][j][1] = v[i][3 * a + 1] - v[i][3 * b + 1];
            dv[i][j][2] = v[i][3 * a + 2] - v[i][3 * b + 2];
            b++;
            if (b > 3) {
                a++;
                b = a + 1;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double *row = L[i];
        row[0] = dot3(dv[0][i], dv[0][i]);
        row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
        row[2] = dot3(dv[1][i], dv[1][i]);
        row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
        row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
        row[5] = dot3(dv[2][i], dv[2][i]);
        row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
        row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
        row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
        row[9] = dot3(dv[3][i], dv[3][i]);
    }
}

RSAC_HD double dist2(const double *p1, const double *p2) {
    return (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) + (p1[2] - p2[2]) * (p1[2] - p2[2]);
}

RSAC_HD void epnp_rho(const Epnp5 &e, double (&rho)[6]) {
    rho[0] = dist2(e.cws[0], e.cws[1]);
    rho[1] = dist2(e.cws[0], e.cws[2]);
    rho[2] = dist2(e.cws[0], e.cws[3]);
    rho[3] = dist2(e.cws[1], e.cws[2]);
    rho[4] = dist2(e.cws[1], e.cws[3]);
    rho[5] = dist2(e.cws[2], e.cws[3]);
}

// compute_R_and_t for one beta estimate: ccs, pcs, solve_for_sign, estimate_R_and_t,
// reprojection_error (returned)
RSAC_HD double epnp5_r_and_t(const Epnp5 &e, const double (&v)[4][12], const double (&be)[4], double R[9],
                             double t[3]) {
    double ccs[4][3], pcs[5][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) ccs[j][0] = ccs[j][1] = ccs[j][2] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int k = 0; k < 3; ++k) ccs[j][k] += be[i] * v[i][3 * j + k];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            pcs[i][j] = e.alphas[i][0] * ccs[0][j] + e.alphas[i][1] * ccs[1][j] + e.alphas[i][2] * ccs[2][j] +
                        e.alphas[i][3] * ccs[3][j];
    if (pcs[0][2] < 0.0) {
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) pcs[i][j] = -pcs[i][j];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            pc0[j] += pcs[i][j];
            pw0[j] += e.pws[i][j];
        }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        pc0[j] /= 5;
        pw0[j] /= 5;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            abt[3 * j] += (pcs[i][j] - pc0[j]) * (e.pws[i][0] - pw0[0]);
            abt[3 * j + 1] += (pcs[i][j] - pc0[j]) * (e.pws[i][1] - pw0[1]);
            abt[3 * j + 2] += (pcs[i][j] - pc0[j]) * (e.pws[i][2] - pw0[2]);
        }
    double d[3], ut[3][3], vt[3][3];
    svd3(abt, d, ut, vt);
    uvt3(ut, vt, R);
    const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                       R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
    if (det < 0) {
        R[6] = -R[6];
        R[7] = -R[7];
        R[8] = -R[8];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
    double sum2 = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const double *pw = e.pws[i];
        const double Xc = dot3(R, pw) + t[0];
        const double Yc = dot3(R + 3, pw) + t[1];
        const double inv_Zc = 1.0 / (dot3(R + 6, pw) + t[2]);
        const double ue = e.uc + e.fu * Xc * inv_Zc;
        const double ve = e.vc + e.fv * Yc * inv_Zc;
        const double u = e.us[i][0], vv = e.us[i][1];
        sum2 += dsqrt((u - ue) * (u - ue) + (vv - ve) * (vv - ve));
    }
    return sum2 / 5;
}

// epnp::compute_pose's pick among the three estimates: N = 1; 2 if err2 < err1; 3 if err3 < err[N]
RSAC_HD int epnp_pick(const double (&err)[3]) {
    int N = 0;
    if (err[1] < err[0]) N = 1;
    if (err[2] < err[N]) N = 2;
    return N;
}

// the 12 x 12 JacobiSVD of M^T M, serially (the host twin; the GPU runs it on 4 lanes, k_cvepnp5_svd,
// with the same operations), returning ut rows 11, 10, 9, 8
RSAC_HD void epnp_mtm_vectors(const double *mtm, double (&v)[4][12]) {
    double At[12][12], W[12], Vt[12][12];
    int q = 0;
#pragma unroll
    for (int c = 0; c < 12; ++c)
#pragma unroll
        for (int d = c; d < 12; ++d, ++q) At[c][d] = At[d][c] = mtm[q];
    jacobi_svd<12, 12>(At, W, Vt);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 12; ++k) v[i][k] = At[11 - i][k];
}

// solvePnP(SOLVEPNP_EPNP) on the 5 sampled points (host twin of the three kernels): always a pose
// (NaN propagates as in OpenCV)
RSAC_HD void epnp5_pose(const float (&X)[5], const float (&Y)[5], const float (&Z)[5], const float (&U)[5],
                        const float (&V)[5], const Cam &k, double R[9], double t[3]) {
    Epnp5 e;
    epnp5_init(X, Y, Z, U, V, k, e);
    epnp5_frame(e);
    double mtm[kMtmUpper], v[4][12], L[6][10], rho[6], err[3], Rs[3][9], ts[3][3];
    epnp5_mtm(e, mtm);
    epnp_mtm_vectors(mtm, v);
    epnp_l6x10(v, L);
    epnp_rho(e, rho);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        double be[4];
        betas_approx(a + 1, L, rho, be);
        gauss_newton(L, rho, be);
        err[a] = epnp5_r_and_t(e, v, be, Rs[a], ts[a]);
    }
    const int N = epnp_pick(err);
#pragma unroll
    for (int q = 0; q < 9; ++q) R[q] = Rs[N][q];
#pragma unroll
    for (int q = 0; q < 3; ++q) t[q] = ts[N][q];
}

}  // namespace cvq
}  // namespace rsac
