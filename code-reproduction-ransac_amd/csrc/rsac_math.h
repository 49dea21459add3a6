// rsac_math.h -- host+device arithmetic of the RANSAC hot path.
//
// Everything here decides inlier counts, so it is written to one numerics
// contract (DESIGN.md "Numerics"): compiled with -ffp-contract=off, only
// + - * / sqrt (IEEE, correctly rounded on gfx950 and x86-64), no FMA unless
// written explicitly.  The CPU restatement in oracle/ follows the same
// contract and the GPU results are checked against it bit-for-bit.
//
// Reference call sites served: cv2.solvePnPRansac (main_v1.py:497,
// testpro-K.py:72), cv2.findHomography (main_v1.py:312, process.py:200),
// cv2.projectPoints (testpro-K.py:33).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define RSAC_HD __host__ __device__ __forceinline__
#define RSAC_NOINLINE __host__ __device__ __attribute__((noinline)) inline
// phase timestamps of block 0 (timing builds: -DRSAC_TRACE, scripts/trace_build.sh)
#ifdef RSAC_TRACE
#define RSAC_TRACE_MARK(red, phase) (red).mark(phase)
#else
#define RSAC_TRACE_MARK(red, phase) ((void)0)
#endif

namespace rsac {

constexpr int kMaxDrawsPerSubset = 256;
constexpr int kMaxSubsetAttempts = 10000;  // getSubset(..., rng, 10000) of RANSACPointSetRegistrator::run
constexpr int kModelStride = 16;           // doubles per hypothesis record (R 9, t 3, valid, pad 3) / (H 9, valid@12)
// slot 12: validity of single-model records (the winners' bestmodels, uploaded poses, the LO
// chain's records, homography / fundamental hypotheses).  PnP hypothesis records (the minimal
// solves' output) leave it unwritten: their validity is the status byte (status > 0), and the
// solve writes 96 of each record's 128 bytes (k_pnp_solve WRITE_SIZE 19.2 -> 16.1 MB per 100k
// hypotheses, r05; scripts/ubench/jacobi_probe.py novalid)
constexpr int kValidSlot = 12;

RSAC_HD bool dfinite(double v) { return __builtin_isfinite(v); }
// a * b + c with one rounding (the oracle's fma(); correctly rounded on every backend)
RSAC_HD double dfma(double a, double b, double c) { return __builtin_fma(a, b, c); }
RSAC_HD double dabs(double v) { return __builtin_fabs(v); }

RSAC_HD double dsqrt(double v) { return __builtin_sqrt(v); }

// Correctly rounded f64 square root and division with a shorter dependent chain, for operands a
// caller has proven to lie in range.  The compiler lowers sqrt to v_rsq_f64 + Newton steps, wrapped
// in a scaling of x < 2^-767 (by 2^256, undone by ldexp) and a class select for 0 / +inf; division
// to v_rcp_f64 + two Newton steps + Markstein's correction, wrapped in v_div_scale / v_div_fmas /
// v_div_fixup.  Where the wrapping is the identity -- sqrt: x in [2^-767, DBL_MAX]; division: no
// v_div_scale case (operand exponents less than 768 apart, |n| > 2^-969, no denormal operand or
// quotient) and a finite nonzero quotient -- the cores below are those same operations, so the
// result is the IEEE one; 5 (sqrt) and 2 (division) of the compiler's dependent instructions leave
// the chain.  A zero numerator gives a zero of possibly the wrong sign.  Host code (and builds
// without RSAC_FAST_F64) uses the IEEE operators.
// (on by default; -DRSAC_FAST_F64=0 builds the IEEE operators everywhere, for A/B runs)
#ifndef RSAC_FAST_F64
#define RSAC_FAST_F64 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && RSAC_FAST_F64
#define RSAC_DEV_FAST_F64 1
__device__ __forceinline__ double dsqrt_fast(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double ddiv_fast(double n, double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = n * r;
    const double rem = __builtin_fma(-d, q, n);
    return __builtin_fma(rem, r, q);
}
#else
#define RSAC_DEV_FAST_F64 0
RSAC_HD double dsqrt_fast(double x) { return __builtin_sqrt(x); }
RSAC_HD double ddiv_fast(double n, double d) { return n / d; }
#endif

// ---------------------------------------------------------------------------
// Rodrigues (cv::Rodrigues, [OpenCV 4.x, unvendored] calibration.cpp cvRodrigues2; main_v1.py:895,
// testpro-K.py:84): acos, sin and cos as polynomials with exactly rounded series coefficients
// (about 1 ulp from the true values, not libm's bits), so host, device and the oracle
// (rsac_oracle.c orc_rd_*) give the same bits; the rest of cvRodrigues2 is rsac_cvepnp.h.
// ---------------------------------------------------------------------------
constexpr double kPio2Hi = 0x1.921fb54442d18p+0, kPio2Lo = 0x1.1a62633145c07p-54;
constexpr double kPio2A = 0x1.921fb544p+0, kPio2B = 0x1.0b4611a626331p-34;  // pi/2: 33 bits + the rest
constexpr double k2OverPi = 0x1.45f306dc9c883p-1;

// asin(x) = x + x z Q(z), z = x^2 <= 1/4: Q(z) = sum_k (2k)! / (4^k (k!)^2 (2k + 1)) z^(k-1), k = 1..26
RSAC_HD double rodr_asin_q(double z) {
    const double c[26] = {0x1.5555555555555p-3, 0x1.3333333333333p-4, 0x1.6db6db6db6db7p-5, 0x1.f1c71c71c71c7p-6,
                          0x1.6e8ba2e8ba2e9p-6, 0x1.1c4ec4ec4ec4fp-6, 0x1.c99999999999ap-7, 0x1.7a87878787878p-7,
                          0x1.3fde50d79435ep-7, 0x1.12ef3cf3cf3cfp-7, 0x1.df3bd37a6f4dfp-8, 0x1.a6863d70a3d71p-8,
                          0x1.782dda12f684cp-8, 0x1.51ba308d3dcb1p-8, 0x1.31683bdef7bdfp-8, 0x1.15ee9d45d1746p-8,
                          0x1.fcaf8fb6db6dbp-9, 0x1.d3d2a8e0dd67dp-9, 0x1.b026f57b13b14p-9, 0x1.90cb77f60c7cep-9,
                          0x1.750de64d7d05fp-9, 0x1.5c5f56efaaaabp-9, 0x1.464c0950f7d47p-9, 0x1.3275586c5f2f0p-9,
                          0x1.208d3570ae5a6p-9, 0x1.1052bc5fa960ap-9};
    double p = c[25];
#pragma unroll
    for (int i = 24; i >= 0; --i) p = p * z + c[i];
    return p;
}

// acos(x), x in [-1, 1] (callers clamp), with fdlibm's argument reduction
RSAC_HD double rodr_acos(double x) {
    if (x >= 1.0) return 0.0;
    if (x <= -1.0) return 2.0 * kPio2Hi;
    const double ax = dabs(x);
    if (ax <= 0.5) {
        const double z = x * x;
        const double r = x * z * rodr_asin_q(z);  // asin(x) - x
        return kPio2Hi - (x - (kPio2Lo - r));
    }
    const double z = (1.0 - ax) * 0.5;  // acos(|x|) = 2 asin(sqrt(z))
    const double s = dsqrt(z);
    const double w = s * z * rodr_asin_q(z);
    if (x > 0.0) return 2.0 * (s + w);
    return 2.0 * (kPio2Hi - (s + (w - kPio2Lo)));  // pi - 2 asin(s)
}

// sin and cos of th >= 0: the nearest multiple n of pi/2 taken off in two parts (exact products for
// n < 2^20), then the Taylor polynomials on [-pi/4, pi/4] (to y^21 / y^22)
RSAC_HD void rodr_sincos(double th, double &sn, double &cs) {
    const double fn = (double)(int64_t)(th * k2OverPi + 0.5);
    const int n = (int)((int64_t)fn & 3);
    const double y = (th - fn * kPio2A) - fn * kPio2B;
    const double z = y * y;
    const double sc[10] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
                           -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49,
                           -0x1.2f49b46814157p-57, 0x1.71b8ef6dcf572p-66};
    const double cc[10] = {0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16, -0x1.27e4fb7789f5cp-22,
                           0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45, -0x1.6827863b97d97p-53,
                           0x1.e542ba4020225p-62, -0x1.0ce396db7f853p-70};
    double ps = sc[9], pc = cc[9];
#pragma unroll
    for (int i = 8; i >= 0; --i) {
        ps = ps * z + sc[i];
        pc = pc * z + cc[i];
    }
    const double s = y + y * z * ps;
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double c = w + (((1.0 - w) - hz) + z * z * pc);
    sn = n == 0 ? s : n == 1 ? c : n == 2 ? -s : -c;
    cs = n == 0 ? c : n == 1 ? -s : n == 2 ? -c : s;
}

// ---------------------------------------------------------------------------
// Philox-4x32-10: counter (hyp_lo, hyp_hi, problem, block), key = seed.
// ---------------------------------------------------------------------------
struct Philox {
    uint32_t k0, k1, c0, c1, c2, c3;
    uint32_t b[4];
    int pos;

    RSAC_HD void init(uint64_t seed, uint32_t problem, uint64_t hyp) {
        k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32);
        c0 = (uint32_t)hyp; c1 = (uint32_t)(hyp >> 32); c2 = problem; c3 = 0;
        pos = 4;
    }
    RSAC_HD void block() {
        uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3, q0 = k0, q1 = k1;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            uint64_t p0 = (uint64_t)0xD2511F53u * x0;
            uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
            uint32_t n0 = (uint32_t)(p1 >> 32) ^ x1 ^ q0;
            uint32_t n1 = (uint32_t)p1;
            uint32_t n2 = (uint32_t)(p0 >> 32) ^ x3 ^ q1;
            uint32_t n3 = (uint32_t)p0;
            x0 = n0; x1 = n1; x2 = n2; x3 = n3;
            q0 += 0x9E3779B9u; q1 += 0xBB67AE85u;
        }
        b[0] = x0; b[1] = x1; b[2] = x2; b[3] = x3;
        c3 += 1u;
        pos = 0;
    }
    RSAC_HD uint32_t next() {
        if (pos == 4) block();
        uint32_t v = pos == 0 ? b[0] : pos == 1 ? b[1] : pos == 2 ? b[2] : b[3];
        ++pos;
        return v;
    }
    RSAC_HD int index(int n) { return (int)(((uint64_t)next() * (uint64_t)(uint32_t)n) >> 32); }

    // s distinct indices, -1 once the per-subset draw budget is spent
    template <int S>
    RSAC_HD int subset(int n, int32_t (&idx)[S]) {
        int draws = 0;
#pragma unroll
        for (int i = 0; i < S; ++i) {
            for (;;) {
                if (draws++ >= kMaxDrawsPerSubset) return -1;
                int r = index(n);
                bool dup = false;
#pragma unroll
                for (int j = 0; j < S; ++j) dup |= (j < i) && (idx[j] == r);
                if (!dup) { idx[i] = r; break; }
            }
        }
        return 0;
    }
};

// ---------------------------------------------------------------------------
// PnP reprojection error: projectPoints (f64 from f32-rounded inputs, zero
// distortion), rounded to f32, squared distance in f32.
// ---------------------------------------------------------------------------
struct Cam {
    double fx, fy, cx, cy;
};

}  // namespace rsac
#include "rsac_cvepnp.h"
namespace rsac {

// cv::Rodrigues both ways in OpenCV's operation sequence (rsac_cvepnp.h: cvRodrigues2 through
// JacobiSVD, c I + c1 r r^T + s [r]x element by element)
RSAC_HD void rodrigues_v2m_det(const double r[3], double R[9]) { cvq::rodrigues_v2m(r, R); }
RSAC_HD void rodrigues_m2v_det(const double Rin[9], double r[3]) { cvq::rodrigues_m2v(Rin, r); }
// PnPRansacCallback keeps each minimal model as (rvec, tvec) and computeError projects through
// Rodrigues(rvec): R' = Rodrigues(Rodrigues(R)) is the rotation OpenCV scores (RSAC_F_RVEC_ROUNDTRIP)
RSAC_HD void rodrigues_roundtrip(double R[9]) { cvq::rvec_roundtrip(R); }

RSAC_HD float pnp_err(const double *R, const double *t, const Cam &k, double X, double Y, double Z, float uf,
                      float vf) {
    double x = R[0] * X + R[1] * Y; x = x + R[2] * Z; x = x + t[0];
    double y = R[3] * X + R[4] * Y; y = y + R[5] * Z; y = y + t[1];
    double z = R[6] * X + R[7] * Y; z = z + R[8] * Z; z = z + t[2];
    double iz = (z != 0.0) ? 1.0 / z : 1.0;
    x = x * iz; y = y * iz;
    double pu = x * k.fx + k.cx;
    double pv = y * k.fy + k.cy;
    float dx = uf - (float)pu;
    float dy = vf - (float)pv;
    float e1 = dx * dx, e2 = dy * dy;
    return e1 + e2;
}

// compute_reprojection_error (testpro-K.py:32-36): cv2.projectPoints of f64 inputs in f64 (the
// operations of pnp_err, zero distortion, no rounding to f32), then np.linalg.norm of the pixel
// residual: sqrt(dx^2 + dy^2).  pu, pv: the projection (projectPoints' output).
RSAC_HD double pnp_reproj_err(const double *R, const double *t, const Cam &k, double X, double Y, double Z, double u,
                              double v, double &pu, double &pv) {
    double x = R[0] * X + R[1] * Y; x = x + R[2] * Z; x = x + t[0];
    double y = R[3] * X + R[4] * Y; y = y + R[5] * Z; y = y + t[1];
    double z = R[6] * X + R[7] * Y; z = z + R[8] * Z; z = z + t[2];
    double iz = (z != 0.0) ? 1.0 / z : 1.0;
    x = x * iz; y = y * iz;
    pu = x * k.fx + k.cx;
    pv = y * k.fy + k.cy;
    const double dx = u - pu, dy = v - pv;
    const double s2 = dx * dx + dy * dy;
    return dsqrt(s2);
}

// ---------------------------------------------------------------------------
// P3P, Lambda Twist (Persson & Nordberg, ECCV 2018).
// ---------------------------------------------------------------------------
RSAC_HD void root2real(double b, double c, double &r1, double &r2) {
    double v = b * b - 4.0 * c;
    if (v < 0.0) { r1 = 0.5 * b; r2 = 0.5 * b; return; }
    double y = dsqrt(v);
    if (b < 0.0) { r1 = 0.5 * (-b + y); r2 = 2.0 * c / (-b + y); }
    else { r1 = 2.0 * c / (-b - y); r2 = 0.5 * (-b - y); }
}

RSAC_HD double cubic_root(double b, double c, double d) {
    double r0;
    if (b * b >= 3.0 * c) {
        double v = dsqrt(b * b - 3.0 * c);
        double t1 = (-b - v) / 3.0;
        double k = ((t1 + b) * t1 + c) * t1 + d;
        if (k > 0.0) {
            r0 = t1 - dsqrt(-k / (3.0 * t1 + b));
        } else {
            double t2 = (-b + v) / 3.0;
            k = ((t2 + b) * t2 + c) * t2 + d;
            r0 = t2 + dsqrt(-k / (3.0 * t2 + b));
        }
    } else {
        r0 = -b / 3.0;
        if (dabs((3.0 * r0 + 2.0 * b) * r0 + c) < 1e-4) r0 = r0 + 1.0;
    }
    /* Newton: at least 7 steps, stop at |f| <= 1e-13, at most 12 (the published solver allows
     * 50; lanes whose |f| stalls at the rounding level above 1e-13 -- about 4 % of C2's samples --
     * then stop at 12 instead of 50, so a GPU wave no longer runs 50 divisions for one of them) */
    for (int it = 0; it < 12; ++it) {
        // Horner by fma (r05; the oracle's cubic_root alike)
        double fx = dfma(dfma(r0 + b, r0, c), r0, d);
        if (it >= 7 && !(dabs(fx) > 1e-13)) break;
        double fpx = dfma(3.0 * r0 + 2.0 * b, r0, c);
        r0 = r0 - fx / fpx;
    }
    return r0;
}

RSAC_HD double lt_resid(double l1, double l2, double l3, double a12, double a13, double a23, double b12, double b13,
                        double b23, double &r0, double &r1, double &r2) {
    // (fma chains from r05, the oracle's lt_resid alike)
    r0 = dfma(b12 * l1, l2, dfma(l2, l2, l1 * l1)) - a12;
    r1 = dfma(b13 * l1, l3, dfma(l3, l3, l1 * l1)) - a13;
    r2 = dfma(b23 * l2, l3, dfma(l3, l3, l2 * l2)) - a23;
    return dabs(r0) + dabs(r1) + dabs(r2);
}

RSAC_HD void lt_refine(double &L0, double &L1, double &L2, double a12, double a13, double a23, double b12,
                       double b13, double b23) {
    for (int it = 0; it < 5; ++it) {
        double r0, r1, r2;
        double s0 = lt_resid(L0, L1, L2, a12, a13, a23, b12, b13, b23, r0, r1, r2);
        if (s0 < 1e-10) break;
        double l1 = L0, l2 = L1, l3 = L2;
        double j0 = dfma(b12, l2, 2.0 * l1);
        double j1 = dfma(b12, l1, 2.0 * l2);
        double j3 = dfma(b13, l3, 2.0 * l1);
        double j5 = dfma(b13, l1, 2.0 * l3);
        double j7 = dfma(b23, l3, 2.0 * l2);
        double j8 = dfma(b23, l2, 2.0 * l3);
        double det = 1.0 / (-j0 * j5 * j7 - j1 * j3 * j8);
        double d0 = dfma(j1 * j5, r2, dfma(-j1 * j8, r1, -j5 * j7 * r0));
        double d1 = dfma(-j0 * j5, r2, dfma(j0 * j8, r1, -j3 * j8 * r0));
        double d2 = dfma(-j1 * j3, r2, dfma(-j0 * j7, r1, j3 * j7 * r0));
        double n0 = dfma(-det, d0, l1), n1 = dfma(-det, d1, l2), n2 = dfma(-det, d2, l3);
        double q0, q1, q2;
        double s1 = lt_resid(n0, n1, n2, a12, a13, a23, b12, b13, b23, q0, q1, q2);
        if (s1 > s0) break;
        L0 = n0; L1 = n1; L2 = n2;
    }
}

// y: 3 unit bearings (row-major 3x3), x: 3 world points.  Writes up to 4
// (R, t); returns the count.
// One candidate (lambda1..3) of the Lambda Twist solver: Gauss-Newton refine, then
// the pose from the scaled bearings; emitted if finite.  Returns 1 if emitted.
// The pose of refined lambdas (l1..l3): false when not finite
RSAC_HD bool p3p_pose_of(double l1, double l2, double l3, const double *y1, const double *y2, const double *y3,
                         const double *x1, const double *Xi, double (&R)[9], double (&t)[3]) {
    double ry1[3], ry2[3], ry3[3], yd1[3], yd2[3], yc[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { ry1[k] = y1[k] * l1; ry2[k] = y2[k] * l2; ry3[k] = y3[k] * l3; }
#pragma unroll
    for (int k = 0; k < 3; ++k) { yd1[k] = ry1[k] - ry2[k]; yd2[k] = ry1[k] - ry3[k]; }
    yc[0] = yd1[1] * yd2[2] - yd1[2] * yd2[1];
    yc[1] = yd1[2] * yd2[0] - yd1[0] * yd2[2];
    yc[2] = yd1[0] * yd2[1] - yd1[1] * yd2[0];
    const double Y[9] = {yd1[0], yd2[0], yc[0], yd1[1], yd2[1], yc[1], yd1[2], yd2[2], yc[2]};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int cc = 0; cc < 3; ++cc)
            R[3 * r + cc] = dfma(Y[3 * r + 2], Xi[6 + cc], dfma(Y[3 * r + 1], Xi[3 + cc], Y[3 * r] * Xi[cc]));  // (r05: fma)
    bool fin = true;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double rx = dfma(R[3 * r + 2], x1[2], dfma(R[3 * r + 1], x1[1], R[3 * r] * x1[0]));
        t[r] = ry1[r] - rx;
        fin = fin && dfinite(t[r]);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) fin = fin && dfinite(R[k]);
    return fin;
}
template <class Emit>
RSAC_HD int p3p_pose(double l1, double l2, double l3, double a12, double a13, double a23, double b12, double b13,
                     double b23, const double *y1, const double *y2, const double *y3, const double *x1,
                     const double *Xi, Emit &emit) {
    lt_refine(l1, l2, l3, a12, a13, a23, b12, b13, b23);
    double R[9], t[3];
    if (!p3p_pose_of(l1, l2, l3, y1, y2, y3, x1, Xi, R, t)) return 0;
    emit(R, t);
    return 1;
}

// The Lambda Twist solver in three pieces, so that the GPU can also run the (up to 4)
// candidates of one sample on 4 lanes (k_pnp_solve_l<4>) with the same operations:
//   lt_common: the cubic, the two eigenvectors, v and the inverse of [d12 d13 d12xd13]
//   lt_sign:   for s = +v / -v: w0, w1 and the quadratic's roots tau (false: no real root)
//   lt_tau:    one root: lambdas, Gauss-Newton refine, pose, emit (1 if emitted)
struct LtCommon {
    double a12, a13, a23, b12, b13, b23, v, v1[3], v2[3], Xi[9];
};

RSAC_HD bool lt_common(const double *y, const double *x, LtCommon &L) {
    const double *y1 = y, *y2 = y + 3, *y3 = y + 6;
    const double *x1 = x, *x2 = x + 3, *x3 = x + 6;
    double b12 = -2.0 * dfma(y1[2], y2[2], dfma(y1[1], y2[1], y1[0] * y2[0]));
    double b13 = -2.0 * dfma(y1[2], y3[2], dfma(y1[1], y3[1], y1[0] * y3[0]));
    double b23 = -2.0 * dfma(y2[2], y3[2], dfma(y2[1], y3[1], y2[0] * y3[0]));
    double d12[3], d13[3], d23[3], d12xd13[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { d12[k] = x1[k] - x2[k]; d13[k] = x1[k] - x3[k]; d23[k] = x2[k] - x3[k]; }
    d12xd13[0] = d12[1] * d13[2] - d12[2] * d13[1];
    d12xd13[1] = d12[2] * d13[0] - d12[0] * d13[2];
    d12xd13[2] = d12[0] * d13[1] - d12[1] * d13[0];
    double a12 = dfma(d12[2], d12[2], dfma(d12[1], d12[1], d12[0] * d12[0]));
    double a13 = dfma(d13[2], d13[2], dfma(d13[1], d13[1], d13[0] * d13[0]));
    double a23 = dfma(d23[2], d23[2], dfma(d23[1], d23[1], d23[0] * d23[0]));

    double c31 = -0.5 * b13, c23 = -0.5 * b23, c12 = -0.5 * b12;
    double blob = c12 * c23 * c31 - 1.0;
    double s31 = 1.0 - c31 * c31, s23 = 1.0 - c23 * c23, s12 = 1.0 - c12 * c12;
    // (fma chains from r05, the oracle's orc_p3p / eig_known0 alike)
    double p3 = a13 * dfma(a23, s31, -(a13 * s23));
    double p2 = dfma(a23 * (a23 - a12), s31, dfma(a13 * (2.0 * a12 + a13), s23, 2.0 * blob * a23 * a13));
    double p1 = dfma(-(2.0 * a12), dfma(a13, s23, blob * a23), dfma(-(a12 * a12), s23, a23 * (a13 - a23) * s12));
    double p0 = a12 * dfma(a12, s23, -(a23 * s12));
    if (p3 == 0.0 || !dfinite(p3)) return false;
    double ip3 = 1.0 / p3;
    p2 = p2 * ip3; p1 = p1 * ip3; p0 = p0 * ip3;
    double g = cubic_root(p2, p1, p0);

    double A00 = a23 * (1.0 - g);
    double A01 = (a23 * b12) * 0.5;
    double A02 = (a23 * b13 * g) * (-0.5);
    double A11 = a23 - a12 + a13 * g;
    double A12 = b23 * (a13 * g - a12) * 0.5;
    double A22 = g * (a13 - a23) - a12;

    // eigenvectors of the two non-zero eigenvalues (the third is 0)
    double e1, e2;
    {
        double a01sq = A01 * A01;
        double b = -A00 - A11 - A22;
        double c = dfma(A11, A22, dfma(A00, A11 + A22, dfma(-A12, A12, dfma(-A02, A02, -a01sq))));
        root2real(b, c, e1, e2);
        if (dabs(e1) < dabs(e2)) { double tmp = e1; e1 = e2; e2 = tmp; }
        double m0011 = -A00 * A11;
        double pr0 = dfma(A01, A12, -(A02 * A11));
        double pr1 = dfma(A01, A02, -(A00 * A12));
        {
            double e = e1;
            double tmp = 1.0 / (dfma(-e, e, dfma(e, A00 + A11, m0011)) + a01sq);
            double q1 = -dfma(e, A02, pr0) * tmp;
            double q2 = -dfma(e, A12, pr1) * tmp;
            double rn = 1.0 / dsqrt(dfma(q2, q2, q1 * q1) + 1.0);
            L.v1[0] = q1 * rn; L.v1[1] = q2 * rn; L.v1[2] = rn;
        }
        {
            double e = e2;
            double tmp = 1.0 / (dfma(-e, e, dfma(e, A00 + A11, m0011)) + a01sq);
            double q1 = -dfma(e, A02, pr0) * tmp;
            double q2 = -dfma(e, A12, pr1) * tmp;
            double rn = 1.0 / dsqrt(dfma(q2, q2, q1 * q1) + 1.0);
            L.v2[0] = q1 * rn; L.v2[1] = q2 * rn; L.v2[2] = rn;
        }
    }
    double vq = -e2 / e1;
    L.v = dsqrt(vq > 0.0 ? vq : 0.0);

    // X = [d12 d13 d12xd13] (columns), its inverse by the adjugate
    double M[9] = {d12[0], d13[0], d12xd13[0], d12[1], d13[1], d12xd13[1], d12[2], d13[2], d12xd13[2]};
    {
        double c00 = M[4] * M[8] - M[5] * M[7];
        double c01 = M[5] * M[6] - M[3] * M[8];
        double c02 = M[3] * M[7] - M[4] * M[6];
        double det = M[0] * c00 + M[1] * c01 + M[2] * c02;
        if (det == 0.0 || !dfinite(det)) return false;
        double id = 1.0 / det;
        L.Xi[0] = c00 * id; L.Xi[1] = (M[2] * M[7] - M[1] * M[8]) * id; L.Xi[2] = (M[1] * M[5] - M[2] * M[4]) * id;
        L.Xi[3] = c01 * id; L.Xi[4] = (M[0] * M[8] - M[2] * M[6]) * id; L.Xi[5] = (M[2] * M[3] - M[0] * M[5]) * id;
        L.Xi[6] = c02 * id; L.Xi[7] = (M[1] * M[6] - M[0] * M[7]) * id; L.Xi[8] = (M[0] * M[4] - M[1] * M[3]) * id;
    }
    L.a12 = a12; L.a13 = a13; L.a23 = a23; L.b12 = b12; L.b13 = b13; L.b23 = b23;
    return true;
}

RSAC_HD bool lt_sign(const LtCommon &L, int sgn, double &w0, double &w1, double *tau) {
    const double a12 = L.a12, a13 = L.a13, b12 = L.b12, b13 = L.b13;
    double s = sgn == 0 ? L.v : -L.v;
    double w2 = 1.0 / dfma(s, L.v2[0], -L.v1[0]);
    w0 = dfma(-s, L.v2[1], L.v1[1]) * w2;
    w1 = dfma(-s, L.v2[2], L.v1[2]) * w2;
    double a = 1.0 / (dfma(-(a12 * b13), w1, (a13 - a12) * w1 * w1) - a12);
    double b = dfma(-(2.0 * w0 * w1), a12 - a13, dfma(-(a12 * b13), w0, a13 * b12 * w1)) * a;
    double c = (dfma(a13 * b12, w0, (a13 - a12) * w0 * w0) + a13) * a;
    if (!(b * b - 4.0 * c >= 0.0)) return false;
    root2real(b, c, tau[0], tau[1]);
    return true;
}

template <class Emit>
RSAC_HD int lt_tau(const LtCommon &L, double w0, double w1, double tq, const double *y, const double *x, Emit &emit) {
    if (!(tq > 0.0)) return 0;
    double d = L.a23 / (tq * (L.b23 + tq) + 1.0);
    if (!(d > 0.0)) return 0;
    double l2 = dsqrt(d);
    double l3 = tq * l2;
    double l1 = w0 * l2 + w1 * l3;
    if (!(l1 >= 0.0)) return 0;
    return p3p_pose(l1, l2, l3, L.a12, L.a13, L.a23, L.b12, L.b13, L.b23, y, y + 3, y + 6, x, L.Xi, emit);
}

// Every solution (R, t), in the order of the restatement's solution list, is
// handed to emit(R, t) as it is built: no solution arrays, so the GPU solver
// keeps everything in registers.  Returns the number of solutions.
template <class Emit>
RSAC_HD int p3p_lambdatwist(const double *y, const double *x, Emit &&emit) {
    LtCommon L;
    if (!lt_common(y, x, L)) return 0;
    int nout = 0;
    for (int sgn = 0; sgn < 2; ++sgn) {
        double w0, w1, tau[2];
        if (lt_sign(L, sgn, w0, w1, tau))
            for (int q = 0; q < 2; ++q) nout += lt_tau(L, w0, w1, tau[q], y, x, emit);
    }
    return nout;
}

RSAC_HD void bearing(const Cam &k, float uf, float vf, double *out) {
    double xn = ((double)uf - k.cx) / k.fx;
    double yn = ((double)vf - k.cy) / k.fy;
    double nrm = dsqrt(xn * xn + yn * yn + 1.0);
    out[0] = xn / nrm; out[1] = yn / nrm; out[2] = 1.0 / nrm;
}

// squared reprojection error of the sample's 4th point under (R, t) (NaN: unusable)
RSAC_HD double pnp_fourth_error(const double *Rk, const double *tk, const float (&X)[4], const float (&Y)[4],
                                const float (&Z)[4], const float (&U)[4], const float (&V)[4], const Cam &k) {
    const double X4 = X[3], Y4 = Y[3], Z4 = Z[3];
    const double x = dfma(Rk[2], Z4, dfma(Rk[1], Y4, Rk[0] * X4)) + tk[0];
    const double y = dfma(Rk[5], Z4, dfma(Rk[4], Y4, Rk[3] * X4)) + tk[1];
    const double z = dfma(Rk[8], Z4, dfma(Rk[7], Y4, Rk[6] * X4)) + tk[2];
    const double iz = (z != 0.0) ? 1.0 / z : 1.0;
    const double du = (x * iz) * k.fx + k.cx - (double)U[3];
    const double dv = (y * iz) * k.fy + k.cy - (double)V[3];
    return du * du + dv * dv;
}

// 4-point minimal PnP: P3P on the first three, disambiguated by the fourth.
// pts: per sample point (X, Y, Z, u, v) already gathered; yb: the first three points' bearings
// (bearing(), here or from a table of them built with the same function)
RSAC_HD bool pnp_minimal_yb(const float (&X)[4], const float (&Y)[4], const float (&Z)[4], const float (&U)[4],
                            const float (&V)[4], const Cam &k, const double (&yb)[9], double *R, double *t) {
    double xw[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        xw[3 * j] = X[j]; xw[3 * j + 1] = Y[j]; xw[3 * j + 2] = Z[j];
    }
    bool have = false;
    double best_e = 0.0;
    // the 4th point picks the solution: smallest reprojection error, first one on ties
    const int ns = p3p_lambdatwist(yb, xw, [&](const double *Rk, const double *tk) {
        const double e = pnp_fourth_error(Rk, tk, X, Y, Z, U, V, k);
        if (!(e == e)) return;
        if (!have || e < best_e) {
            have = true;
            best_e = e;
#pragma unroll
            for (int q = 0; q < 9; ++q) R[q] = Rk[q];
#pragma unroll
            for (int q = 0; q < 3; ++q) t[q] = tk[q];
        }
    });
    if (ns == 0 || !have) return false;
    return true;
}
// pnp_minimal_yb for one GPU lane: the best candidate is held as its refined lambdas (3 doubles
// instead of R and t's 12, fewer registers live across the candidate loop) and its pose is
// rebuilt from them at the end with p3p_pose_of's operations: the same candidates in the same
// order (p3p_lambdatwist), the same first-smallest rule, the same bits
RSAC_HD bool pnp_minimal_lam(const float (&X)[4], const float (&Y)[4], const float (&Z)[4], const float (&U)[4],
                             const float (&V)[4], const Cam &k, const double (&yb)[9], double (&R)[9], double (&t)[3]) {
    double xw[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        xw[3 * j] = X[j]; xw[3 * j + 1] = Y[j]; xw[3 * j + 2] = Z[j];
    }
    LtCommon L;
    if (!lt_common(yb, xw, L)) return false;
    bool have = false;
    double best_e = 0.0, bl[3] = {0.0, 0.0, 0.0};
    // both signs' (w0, w1, tau) first: v, v1, v2 are then dead across the candidate loop
    double w0s[2], w1s[2], taus[2][2];
    bool oks[2];
#pragma unroll
    for (int sgn = 0; sgn < 2; ++sgn) oks[sgn] = lt_sign(L, sgn, w0s[sgn], w1s[sgn], taus[sgn]);
    for (int sgn = 0; sgn < 2; ++sgn) {
        if (!oks[sgn]) continue;
        const double w0 = w0s[sgn], w1 = w1s[sgn];
        for (int q = 0; q < 2; ++q) {
            // lt_tau, then p3p_pose
            const double tq = taus[sgn][q];
            if (!(tq > 0.0)) continue;
            const double d = L.a23 / (tq * (L.b23 + tq) + 1.0);
            if (!(d > 0.0)) continue;
            double l2 = dsqrt(d);
            double l3 = tq * l2;
            double l1 = w0 * l2 + w1 * l3;
            if (!(l1 >= 0.0)) continue;
            lt_refine(l1, l2, l3, L.a12, L.a13, L.a23, L.b12, L.b13, L.b23);
            double Rk[9], tk[3];
            if (!p3p_pose_of(l1, l2, l3, yb, yb + 3, yb + 6, xw, L.Xi, Rk, tk)) continue;
            const double e = pnp_fourth_error(Rk, tk, X, Y, Z, U, V, k);
            if (!(e == e)) continue;
            if (!have || e < best_e) {
                have = true;
                best_e = e;
                bl[0] = l1; bl[1] = l2; bl[2] = l3;
            }
        }
    }
    if (!have) return false;
    return p3p_pose_of(bl[0], bl[1], bl[2], yb, yb + 3, yb + 6, xw, L.Xi, R, t);
}
RSAC_HD bool pnp_minimal(const float (&X)[4], const float (&Y)[4], const float (&Z)[4], const float (&U)[4],
                         const float (&V)[4], const Cam &k, double *R, double *t) {
    double yb[9];
#pragma unroll
    for (int j = 0; j < 3; ++j) bearing(k, U[j], V[j], yb + 3 * j);
    return pnp_minimal_yb(X, Y, Z, U, V, k, yb, R, t);
}

// ---------------------------------------------------------------------------
// Homography (HomographyEstimatorCallback): checkSubset, minimal solver,
// f32 error.
// ---------------------------------------------------------------------------
RSAC_HD bool have_collinear4(const float (&px)[4], const float (&py)[4]) {
    // only the last point against every pair of earlier ones (count = 4)
    const int i = 3;
    for (int j = 0; j < i; ++j) {
        double dx1 = (double)(px[j] - px[i]);
        double dy1 = (double)(py[j] - py[i]);
        for (int q = 0; q < j; ++q) {
            double dx2 = (double)(px[q] - px[i]);
            double dy2 = (double)(py[q] - py[i]);
            if (dabs(dx2 * dy1 - dy2 * dx1) <= 1.1920928955078125e-07 * (dabs(dx1) + dabs(dy1) + dabs(dx2) + dabs(dy2)))
                return true;
        }
    }
    return false;
}

RSAC_HD double det3_rows(double a0, double a1, double b0, double b1, double c0, double c1) {
    return a0 * (b1 * 1. - c1 * 1.) - a1 * (b0 * 1. - c0 * 1.) + 1. * (b0 * c1 - c0 * b1);
}

RSAC_HD bool hom_check_subset(const float (&sx)[4], const float (&sy)[4], const float (&dx)[4], const float (&dy)[4]) {
    if (have_collinear4(sx, sy) || have_collinear4(dx, dy)) return false;
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    int negative = 0;
    for (int i = 0; i < 4; ++i) {
        int p0 = tt[i][0], p1 = tt[i][1], p2 = tt[i][2];
        double dA = det3_rows(sx[p0], sy[p0], sx[p1], sy[p1], sx[p2], sy[p2]);
        double dB = det3_rows(dx[p0], dy[p0], dx[p1], dy[p1], dx[p2], dy[p2]);
        negative += dA * dB < 0;
    }
    return negative == 0 || negative == 4;
}

RSAC_HD void mat3mul(const double *A, const double *B, double *C) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// normalised 4-point DLT, 8x8 Gaussian elimination with partial pivoting
RSAC_HD bool hom_minimal(const float (&sx)[4], const float (&sy)[4], const float (&dx)[4], const float (&dy)[4],
                         double *H) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) { cmx += dx[i]; cmy += dy[i]; cMx += sx[i]; cMy += sy[i]; }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        smx += dabs(dx[i] - cmx); smy += dabs(dy[i] - cmy);
        sMx += dabs(sx[i] - cMx); sMy += dabs(sy[i] - cMy);
    }
    const double eps = 2.220446049250313e-16;
    if (dabs(smx) < eps || dabs(smy) < eps || dabs(sMx) < eps || dabs(sMy) < eps) return false;
    smx = 4 / smx; smy = 4 / smy; sMx = 4 / sMx; sMy = 4 / sMy;
    double A[8][9];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double x = (dx[i] - cmx) * smx, y = (dy[i] - cmy) * smy;
        double X = (sx[i] - cMx) * sMx, Y = (sy[i] - cMy) * sMy;
        double *r0 = A[2 * i], *r1 = A[2 * i + 1];
        r0[0] = X; r0[1] = Y; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0; r0[6] = -x * X; r0[7] = -x * Y; r0[8] = x;
        r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = X; r1[4] = Y; r1[5] = 1; r1[6] = -y * X; r1[7] = -y * Y; r1[8] = y;
    }
    for (int k = 0; k < 8; ++k) {
        int piv = k;
        double pm = dabs(A[k][k]);
        for (int r = k + 1; r < 8; ++r) {
            double v = dabs(A[r][k]);
            if (v > pm) { pm = v; piv = r; }
        }
        if (!(pm > 1e-10)) return false;
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
    double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9], H0[9];
    mat3mul(invHnorm, Hn, T);
    mat3mul(T, Hnorm2, H0);
    double sc = 1. / H0[8];
    bool fin = true;
#pragma unroll
    for (int q = 0; q < 9; ++q) { H[q] = H0[q] * sc; fin = fin && dfinite(H[q]); }
    return fin;
}

RSAC_HD float hom_err(const float *h, float x, float y, float u, float v) {
    float ww = 1.f / (h[6] * x + h[7] * y + 1.f);
    float ex = (h[0] * x + h[1] * y + h[2]) * ww - u;
    float ey = (h[3] * x + h[4] * y + h[5]) * ww - v;
    float e1 = ex * ex, e2 = ey * ey;
    return e1 + e2;
}

// ---------------------------------------------------------------------------
// Fundamental matrix (BASELINE.json configs[3]; no reference implementation
// exists -- SURVEY.md §8d -- so this restatement defines the semantics):
//   minimal solver: normalised 8-point DLT (Hartley: centroid, mean distance
//   sqrt 2), null vector by Gauss-Jordan with full pivoting, rank 2 by removing
//   the smallest right-singular direction (Jacobi on F^T F), denormalised, unit
//   Frobenius norm;
//   inlier test: Sampson distance r^2 / (a^2 + b^2 + a'^2 + b'^2) <= thr^2,
//   evaluated division-free as r^2 <= T (a^2 + b^2 + a'^2 + b'^2) in f64 with
//   explicit fma (bit-identical on every backend).
// ---------------------------------------------------------------------------

RSAC_HD bool fm_norm8(const float (&x)[8], const float (&y)[8], double &cx, double &cy, double &s) {
    cx = 0.0;
    cy = 0.0;
    for (int i = 0; i < 8; ++i) {
        cx = cx + (double)x[i];
        cy = cy + (double)y[i];
    }
    cx = cx * 0.125;
    cy = cy * 0.125;
    double d = 0.0;
    for (int i = 0; i < 8; ++i) {
        const double dx = (double)x[i] - cx, dy = (double)y[i] - cy;
        d = d + dsqrt(dx * dx + dy * dy);
    }
    d = d * 0.125;
    if (!(d > 1e-300)) return false;
    s = 1.4142135623730951 / d;
    return true;
}

// eigenvector of the smallest eigenvalue of a symmetric 3x3 (cyclic Jacobi, 12 sweeps max)
RSAC_HD void sym3_min_evec(double (&A)[9], double (&v)[3]) {
    double V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int sweep = 0; sweep < 12; ++sweep) {
        const double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        const double dia = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (off <= 1e-34 * dia || off < 1e-300) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                const double apq = A[p * 3 + q];
                if (dabs(apq) < 1e-300) continue;
                const double theta = (A[q * 3 + q] - A[p * 3 + p]) / (2.0 * apq);
                const double tt = (theta >= 0 ? 1.0 : -1.0) / (dabs(theta) + dsqrt(theta * theta + 1.0));
                const double c = 1.0 / dsqrt(tt * tt + 1.0), sn = tt * c;
                for (int k = 0; k < 3; ++k) {
                    const double akp = A[k * 3 + p], akq = A[k * 3 + q];
                    A[k * 3 + p] = c * akp - sn * akq;
                    A[k * 3 + q] = sn * akp + c * akq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double apk = A[p * 3 + k], aqk = A[q * 3 + k];
                    A[p * 3 + k] = c * apk - sn * aqk;
                    A[q * 3 + k] = sn * apk + c * aqk;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k * 3 + p], vkq = V[k * 3 + q];
                    V[k * 3 + p] = c * vkp - sn * vkq;
                    V[k * 3 + q] = sn * vkp + c * vkq;
                }
            }
    }
    int mi = 0;
    if (A[4] < A[mi * 4]) mi = 1;
    if (A[8] < A[mi * 4]) mi = 2;
    v[0] = V[mi];
    v[1] = V[3 + mi];
    v[2] = V[6 + mi];
}

RSAC_HD bool fm_finish(const double (&f)[9], double c1x, double c1y, double s1, double c2x, double c2y, double s2,
                       double *F);

// x1,y1 -> x2,y2 (x2^T F x1 = 0); F row-major 3x3.  false for degenerate samples.
RSAC_HD bool fm_minimal8(const float (&x1)[8], const float (&y1)[8], const float (&x2)[8], const float (&y2)[8],
                         double *F) {
    double c1x, c1y, s1, c2x, c2y, s2;
    if (!fm_norm8(x1, y1, c1x, c1y, s1) || !fm_norm8(x2, y2, c2x, c2y, s2)) return false;
    double A[8][9];
    double amax = 0.0;
    for (int i = 0; i < 8; ++i) {
        const double u1 = ((double)x1[i] - c1x) * s1, v1 = ((double)y1[i] - c1y) * s1;
        const double u2 = ((double)x2[i] - c2x) * s2, v2 = ((double)y2[i] - c2y) * s2;
        A[i][0] = u2 * u1; A[i][1] = u2 * v1; A[i][2] = u2;
        A[i][3] = v2 * u1; A[i][4] = v2 * v1; A[i][5] = v2;
        A[i][6] = u1;      A[i][7] = v1;      A[i][8] = 1.0;
        for (int j = 0; j < 9; ++j) amax = dabs(A[i][j]) > amax ? dabs(A[i][j]) : amax;
    }
    int perm[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
    for (int r = 0; r < 8; ++r) {
        int pr = r, pc = r;
        double best = -1.0;
        for (int i = r; i < 8; ++i)
            for (int j = r; j < 9; ++j)
                if (dabs(A[i][j]) > best) { best = dabs(A[i][j]); pr = i; pc = j; }
        if (!(best > 1e-12 * amax)) return false;
        if (pr != r)
            for (int j = 0; j < 9; ++j) { const double tmp = A[r][j]; A[r][j] = A[pr][j]; A[pr][j] = tmp; }
        if (pc != r) {
            for (int i = 0; i < 8; ++i) { const double tmp = A[i][r]; A[i][r] = A[i][pc]; A[i][pc] = tmp; }
            const int tp = perm[r]; perm[r] = perm[pc]; perm[pc] = tp;
        }
        const double ip = 1.0 / A[r][r];
        for (int i = 0; i < 8; ++i) {
            if (i == r) continue;
            const double f = A[i][r] * ip;
            if (f == 0.0) continue;
            for (int j = r; j < 9; ++j) A[i][j] = A[i][j] - f * A[r][j];
        }
    }
    double f[9];
    f[perm[8]] = 1.0;
    for (int r = 0; r < 8; ++r) f[perm[r]] = -A[r][8] / A[r][r];
    return fm_finish(f, c1x, c1y, s1, c2x, c2y, s2, F);
}

// the rest of the 8-point solver from the null vector f of the normalised system: rank 2,
// denormalisation, unit Frobenius norm (shared by fm_minimal8 and the GPU's 8-lane solver)
RSAC_HD bool fm_finish(const double (&f)[9], double c1x, double c1y, double s1, double c2x, double c2y, double s2,
                       double *F) {
    // rank 2: Fn (I - v v^T), v the smallest right-singular vector of Fn
    double M[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = f[i] * f[j] + f[3 + i] * f[3 + j] + f[6 + i] * f[6 + j];
    double v[3];
    sym3_min_evec(M, v);
    double Fr[9];
    for (int i = 0; i < 3; ++i) {
        const double w = f[3 * i] * v[0] + f[3 * i + 1] * v[1] + f[3 * i + 2] * v[2];
        for (int j = 0; j < 3; ++j) Fr[3 * i + j] = f[3 * i + j] - w * v[j];
    }
    // F = T2^T Fr T1, T = [[s, 0, -s cx], [0, s, -s cy], [0, 0, 1]]
    const double T1[9] = {s1, 0.0, -s1 * c1x, 0.0, s1, -s1 * c1y, 0.0, 0.0, 1.0};
    const double T2t[9] = {s2, 0.0, 0.0, 0.0, s2, 0.0, -s2 * c2x, -s2 * c2y, 1.0};
    double tmp[9];
    mat3mul(T2t, Fr, tmp);
    mat3mul(tmp, T1, F);
    double nrm = 0.0;
    for (int k = 0; k < 9; ++k) nrm = nrm + F[k] * F[k];
    if (!(nrm > 1e-300) || !dfinite(nrm)) return false;
    const double in = 1.0 / dsqrt(nrm);
    for (int k = 0; k < 9; ++k) F[k] = F[k] * in;
    return true;
}

// Sampson test, division-free
RSAC_HD bool fm_inlier(const double *F, double x1, double y1, double x2, double y2, double T) {
    const double a = dfma(F[0], x1, dfma(F[1], y1, F[2]));
    const double b = dfma(F[3], x1, dfma(F[4], y1, F[5]));
    const double c = dfma(F[6], x1, dfma(F[7], y1, F[8]));
    const double a2 = dfma(F[0], x2, dfma(F[3], y2, F[6]));
    const double b2 = dfma(F[1], x2, dfma(F[4], y2, F[7]));
    const double r = dfma(x2, a, dfma(y2, b, c));
    const double den = dfma(a, a, dfma(b, b, dfma(a2, a2, b2 * b2)));
    return r * r <= T * den;
}

// ---------------------------------------------------------------------------
// Pose refinement: Levenberg-Marquardt on the reprojection error of the
// inliers (the final solvePnP / solvePnPRefineLM step, main_v1.py:508-509,
// testpro-K.py:122-125).  Parameters: a rotation increment d[0..2] applied as
// R <- Cay(d) R (Cayley map: + - * / only, so every backend rounds the same)
// and a translation increment d[3..5].  The pose is refined in a frame centred
// on the problem's first point c (X - c exact in f64; t' = R c + t): UTM-scale
// coordinates would otherwise couple rotation and translation badly.
//
// One summation order on every backend (GPU kernel k_pnp_refine, host
// rsac_pnp_refine, oracle orc_pnp_refine), "block-compacted": the points are cut
// into nb = lm_blocks(n) contiguous ranges of lm_chunk(n) indices; within range b
// the masked points, in ascending index order, are dealt round-robin to 512 slots
// (the p-th masked point of the range to slot b * 512 + p % 512); each slot sums
// its points in order, a 64-lane tree per wave of 64 slots (x += x[lane ^ o],
// o = 32 .. 1), each range's 8 wave sums left to right, then the nb range sums left
// to right.  The GPU runs one block per range and stages the range's masked points
// in LDS once per refit, so every thread gets ceil(inliers of the range / 512)
// points and no outlier costs a pass; the blocks exchange one sum per term.
// ---------------------------------------------------------------------------
constexpr int kLmThreads = 512;
constexpr int kLmMaxBlocks = 64;
constexpr int kLmOneBlock = 4096;     // one range up to this many points
constexpr int kLmBlockPoints = 1024;  // range length above it: ~2 inliers per thread at 50 %
RSAC_HD int lm_blocks(int n) {
    if (n <= kLmOneBlock) return 1;
    const int nb = (n + kLmBlockPoints - 1) / kLmBlockPoints;
    return nb < kLmMaxBlocks ? nb : kLmMaxBlocks;
}
RSAC_HD int lm_chunk(int n) {
    const int nb = lm_blocks(n);
    return (int)(((int64_t)n + nb - 1) / nb);
}
constexpr int kLmTerms = 27;  // J^T J lower triangle (21, row-major packed), J^T r (6)
constexpr int kLmMaxIter = 20;
constexpr int kRedMax = 40;   // widest reduction (EPnP's pair sums)

// adds point (X, Y, Z) -> (u, v)'s terms of J^T J and J^T r to acc.  The rotation's dot products
// and the accumulations are fma chains (r05; the oracle's lm_point alike)
RSAC_HD void pnp_lm_point(const double *R, const double *t, const Cam &k, double Xd, double Yd, double Zd, double u,
                          double v, double *acc) {
    const double px = dfma(R[2], Zd, dfma(R[1], Yd, R[0] * Xd));
    const double py = dfma(R[5], Zd, dfma(R[4], Yd, R[3] * Xd));
    const double pz = dfma(R[8], Zd, dfma(R[7], Yd, R[6] * Xd));
    const double cx = px + t[0], cy = py + t[1], cz = pz + t[2];
    const double iz = 1.0 / cz;
    const double ru = k.fx * cx * iz + k.cx - u;
    const double rv = k.fy * cy * iz + k.cy - v;
    const double dux = k.fx * iz, duz = -k.fx * cx * iz * iz;
    const double dvy = k.fy * iz, dvz = -k.fy * cy * iz * iz;
    double Ju[6], Jv[6];
    Ju[0] = duz * py;             Ju[1] = dux * pz - duz * px; Ju[2] = -dux * py;
    Jv[0] = -dvy * pz + dvz * py; Jv[1] = -dvz * px;           Jv[2] = dvy * px;
    Ju[3] = dux; Ju[4] = 0; Ju[5] = duz;
    Jv[3] = 0; Jv[4] = dvy; Jv[5] = dvz;
    int q = 0;
    for (int a = 0; a < 6; ++a)
        for (int b = 0; b <= a; ++b, ++q) acc[q] = dfma(Jv[a], Jv[b], dfma(Ju[a], Ju[b], acc[q]));
    for (int a = 0; a < 6; ++a) acc[21 + a] = dfma(Jv[a], rv, dfma(Ju[a], ru, acc[21 + a]));
}

RSAC_HD double pnp_lm_cost_point(const double *R, const double *t, const Cam &k, double Xd, double Yd, double Zd,
                                 double u, double v) {
    const double x = dfma(R[2], Zd, dfma(R[1], Yd, R[0] * Xd)) + t[0];
    const double y = dfma(R[5], Zd, dfma(R[4], Yd, R[3] * Xd)) + t[1];
    const double z = dfma(R[8], Zd, dfma(R[7], Yd, R[6] * Xd)) + t[2];
    const double iz = 1.0 / z;
    const double ru = k.fx * x * iz + k.cx - u;
    const double rv = k.fy * y * iz + k.cy - v;
    return dfma(rv, rv, ru * ru);
}

// (A + lam diag(A)) x = b by Cholesky, A 6 x 6 SPD, on the packed normal equations of
// pnp_lm_point (acc: J^T J lower triangle row-major, then J^T r): A[i][j] = acc[i (i + 1) / 2
// + j], b = -J^T r; false if not positive definite.  Divisions by the pivots are
// multiplications by their reciprocals (6 divisions, not 33: the GPU refit runs this on every
// thread of the block, between two reductions, reading acc from LDS).
// FAST (device): the pivots' roots and reciprocals, the Cayley map's reciprocal and the step
// test's roots by the fast cores (rsac_math.h top); `bad` is set when an operand leaves their
// range, and the caller then redoes the step with the IEEE operators (lm_solve_step), so the
// result is the same bits either way.
RSAC_HD bool lm_in300(double v) { return (dabs(v) >= 0x1p-300) & (dabs(v) <= 0x1p+300); }
RSAC_HD bool lm_root_ok(double v) { return (v >= 0x1p-767) & (v <= 0x1.fffffffffffffp+1023); }
template <bool FAST>
RSAC_HD bool chol6_solve_packed_t(const double *acc, double lam, double *x, bool &bad) {
    double L[36], y[6], inv[6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            double s = acc[i * (i + 1) / 2 + j];
            if (i == j) s = dfma(lam, acc[i * (i + 1) / 2 + i], s);
            for (int q = 0; q < j; ++q) s = dfma(-L[i * 6 + q], L[j * 6 + q], s);  // (r05: fused, the oracle's chol6 alike)
            if (i == j) {
                if (!(s > 0)) return false;
                if constexpr (FAST) {
                    L[i * 6 + i] = dsqrt_fast(s);
                    inv[i] = ddiv_fast(1.0, L[i * 6 + i]);
                    bad = bad | !lm_root_ok(s) | !lm_in300(L[i * 6 + i]);
                } else {
                    L[i * 6 + i] = dsqrt(s);
                    inv[i] = 1.0 / L[i * 6 + i];
                }
            } else {
                L[i * 6 + j] = s * inv[j];
            }
        }
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double s = -acc[21 + i];
        for (int q = 0; q < i; ++q) s = dfma(-L[i * 6 + q], y[q], s);
        y[i] = s * inv[i];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
        double s = y[i];
        for (int q = i + 1; q < 6; ++q) s = dfma(-L[q * 6 + i], x[q], s);
        x[i] = s * inv[i];
    }
    return true;
}
RSAC_HD bool chol6_solve_packed(const double *acc, double lam, double *x) {
    bool bad = false;
    return chol6_solve_packed_t<false>(acc, lam, x, bad);
}

// Rn = Cay(d) R, Cay(d) = the rotation of the quaternion (1, d/2) (first order: I + [d]x)
template <bool FAST>
RSAC_HD void cayley_apply_t(const double *d, const double *R, double *Rn, bool &bad) {
    const double w0 = 0.5 * d[0], w1 = 0.5 * d[1], w2 = 0.5 * d[2];
    const double a = w0 * w0, b = w1 * w1, c = w2 * w2;
    const double den = 1.0 + a + b + c;
    double is;
    if constexpr (FAST) {
        is = ddiv_fast(1.0, den);
        bad = bad | !lm_in300(den);
    } else {
        is = 1.0 / den;
    }
    double Q[9];
    Q[0] = (1.0 + a - b - c) * is;       Q[1] = 2.0 * (w0 * w1 - w2) * is; Q[2] = 2.0 * (w0 * w2 + w1) * is;
    Q[3] = 2.0 * (w0 * w1 + w2) * is;    Q[4] = (1.0 - a + b - c) * is;   Q[5] = 2.0 * (w1 * w2 - w0) * is;
    Q[6] = 2.0 * (w0 * w2 - w1) * is;    Q[7] = 2.0 * (w1 * w2 + w0) * is; Q[8] = (1.0 - a - b + c) * is;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) Rn[3 * i + j] = Q[3 * i] * R[j] + Q[3 * i + 1] * R[3 + j] + Q[3 * i + 2] * R[6 + j];
}
RSAC_HD void cayley_apply(const double *d, const double *R, double *Rn) {
    bool bad = false;
    cayley_apply_t<false>(d, R, Rn, bad);
}

// The LM loop.  Red provides normal(R, t, acc[27]) and cost(R, t), reduced in the
// order above; on the GPU every thread of the block runs this loop in lockstep
// (all decisions depend on reduced, block-uniform values).  Returns iterations.
// A reducer with kFused = true also provides cost_normal(R, t, acc) = cost(R, t) with
// normal(R, t, acc) in the same pass (each term reduced in the same order as alone): the
// accepted candidate's normal equations are then not recomputed, one reduction per iteration.
template <class Red, class = void>
struct LmFused {
    static constexpr bool value = false;
};
template <class Red>
struct LmFused<Red, decltype((void)Red::kFused)> {
    static constexpr bool value = Red::kFused;
};

// One LM step's solve: d from (A + lam diag(A)) d = -J^T r (false: not positive definite), the
// candidate Rn = Cay(d) R, tn = t + d[3..5], and CvLevMarq's step criterion on it, |d| <
// FLT_EPSILON (|tn| + 1) (used only if the candidate is accepted, when tn becomes t).
template <bool FAST>
RSAC_HD bool lm_solve_step_t(const double *acc, double lam, const double *R, const double *t, double *Rn, double *tn,
                             bool &small, bool &bad) {
    double d[6];
    if (!chol6_solve_packed_t<FAST>(acc, lam, d, bad)) return false;
    cayley_apply_t<FAST>(d, R, Rn, bad);
    for (int j = 0; j < 3; ++j) tn[j] = t[j] + d[3 + j];
    double dd = 0, tt = 0;
    for (int j = 0; j < 6; ++j) dd += d[j] * d[j];
    for (int j = 0; j < 3; ++j) tt += tn[j] * tn[j];
    if constexpr (FAST) {
        small = dsqrt_fast(dd) < 1.1920928955078125e-07 * (dsqrt_fast(tt) + 1.0);
        bad = bad | !lm_root_ok(dd) | !lm_root_ok(tt);
    } else {
        small = dsqrt(dd) < 1.1920928955078125e-07 * (dsqrt(tt) + 1.0);
    }
    return true;
}
RSAC_HD bool lm_solve_step(const double *acc, double lam, const double *R, const double *t, double *Rn, double *tn,
                           bool &small) {
    bool bad = false;
    return lm_solve_step_t<false>(acc, lam, R, t, Rn, tn, small, bad);
}
// A reducer with kSolveStep = true provides solve_step(...) = lm_solve_step(...) (the GPU
// reducer: one wave solves, the block reads the result)
template <class Red, class = void>
struct LmSolveStep {
    static constexpr bool value = false;
};
template <class Red>
struct LmSolveStep<Red, decltype((void)Red::kSolveStep)> {
    static constexpr bool value = Red::kSolveStep;
};

// Red::acc_buf(k), k = 0, 1: two buffers of kLmTerms doubles for the current and the next
// normal equations (the GPU reducer's are in LDS, written by its reductions)
template <class Red>
RSAC_HD int pnp_lm_refine(Red &red, double *R, double *t, int max_iter) {
    constexpr bool fused = LmFused<Red>::value;
    double lam = 1e-3;
    RSAC_TRACE_MARK(red, 10);
    double *acc = red.acc_buf(0), *acc_next = red.acc_buf(1);
    bool have_next = false;
    double cost;
    if constexpr (fused) {  // the start's cost and normal equations in one pass
        cost = red.cost_normal(R, t, acc_next);
        have_next = true;
    } else {
        cost = red.cost(R, t);
    }
    RSAC_TRACE_MARK(red, 11);
    int it;
    for (it = 0; it < max_iter; ++it) {
        if (fused && have_next) {
            double *tmp = acc;  // the accepted candidate's normal equations
            acc = acc_next;
            acc_next = tmp;
        } else {
            red.normal(R, t, acc);
        }
        RSAC_TRACE_MARK(red, 12);
        bool accepted = false;
        while (!accepted) {
            double Rn[9], tn[3];
            bool small, ok;
            if constexpr (LmSolveStep<Red>::value) ok = red.solve_step(acc, lam, R, t, Rn, tn, small);
            else ok = lm_solve_step(acc, lam, R, t, Rn, tn, small);
            if (!ok) {
                lam *= 10;
                if (lam > 1e10) return it;
                continue;
            }
            RSAC_TRACE_MARK(red, 13);
            double cn;
            // a step already below the step criterion needs only the candidate's cost: accepted, the
            // loop ends; rejected, the next try re-solves the current normal equations (r06: the
            // last pass of most refits is then the 1-term cost reduction, the same bits)
            if constexpr (fused) cn = small ? red.cost(Rn, tn) : red.cost_normal(Rn, tn, acc_next);
            else cn = red.cost(Rn, tn);
            RSAC_TRACE_MARK(red, 14);
            if (cn < cost) {
                have_next = true;
                const double rel = (cost - cn) / (cost > 1e-300 ? cost : 1e-300);
                for (int j = 0; j < 9; ++j) R[j] = Rn[j];
                for (int j = 0; j < 3; ++j) t[j] = tn[j];
                cost = cn;
                lam = lam * 0.1 > 1e-12 ? lam * 0.1 : 1e-12;
                accepted = true;
                // converged: negligible cost decrease, or a step below FLT_EPSILON relative to
                // the pose (CvLevMarq's criterion for solvePnP, on |d| / (|t| + 1))
                if (rel < 1e-12 || small) return it + 1;
            } else {
                lam *= 10;
                if (lam > 1e10) return it;
            }
        }
    }
    return it;
}

// t' = R c + t and back (the centred frame of the refit)
RSAC_HD void lm_to_centred(const double *R, const double *c, double *t) {
    for (int j = 0; j < 3; ++j) t[j] = R[3 * j] * c[0] + R[3 * j + 1] * c[1] + R[3 * j + 2] * c[2] + t[j];
}
RSAC_HD void lm_from_centred(const double *R, const double *c, double *t) {
    for (int j = 0; j < 3; ++j) t[j] = t[j] - (R[3 * j] * c[0] + R[3 * j + 1] * c[1] + R[3 * j + 2] * c[2]);
}

// the wave trees of slots part[slot * nv + q], each block's 8 wave sums left to right, then
// the block sums (kLmThreads slots each) left to right
inline void lm_tree_host(const double *part, int slots, int nv, double *out) {
    double v[64], w[64];
    for (int q = 0; q < nv; ++q) out[q] = 0.0;
    for (int b = 0; b < slots / kLmThreads; ++b)
        for (int q = 0; q < nv; ++q) {
            double bsum = 0.0;
            for (int wv = 0; wv < kLmThreads / 64; ++wv) {
                for (int l = 0; l < 64; ++l) v[l] = part[((b * kLmThreads / 64 + wv) * 64 + l) * nv + q];
                for (int o = 32; o > 0; o >>= 1) {
                    for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ o];
                    for (int l = 0; l < 64; ++l) v[l] = w[l];
                }
                bsum = wv == 0 ? v[0] : bsum + v[0];  // wave sums left to right
            }
            out[q] = b == 0 ? bsum : out[q] + bsum;  // block sums left to right
        }
}

// Host/oracle-side mirror of the GPU EPnP reduction: sum f(i, acc) over points with
// mask[i] != 0, point i to slot i % kLmThreads; part: kLmThreads * nv doubles.
template <class F>
inline void lm_reduce_host(int n, const uint8_t *mask, int nv, double *part, double *out, F f) {
    for (int q = 0; q < kLmThreads * nv; ++q) part[q] = 0.0;
    for (int tid = 0; tid < kLmThreads; ++tid)
        for (int i = tid; i < n; i += kLmThreads)
            if (mask[i]) f(i, part + tid * nv);
    lm_tree_host(part, kLmThreads, nv, out);
}

// the LM refit's block-compacted order (above); part: lm_blocks(n) * kLmThreads * nv doubles
template <class F>
inline void lm_reduce_blocks_host(int n, const uint8_t *mask, int nv, double *part, double *out, F f) {
    const int nb = lm_blocks(n), C = lm_chunk(n);
    for (int q = 0; q < nb * kLmThreads * nv; ++q) part[q] = 0.0;
    for (int b = 0; b < nb; ++b) {
        const int64_t end = (int64_t)(b + 1) * C;
        const int hi = end < n ? (int)end : n;
        int p = 0;
        for (int i = b * C; i < hi; ++i)
            if (mask[i]) f(i, part + (b * kLmThreads + p++ % kLmThreads) * nv);
    }
    lm_tree_host(part, nb * kLmThreads, nv, out);
}

// ---------------------------------------------------------------------------
// EPnP (Lepetit, Moreno-Noguer, Fua, IJCV 2009) on the inliers: the
// non-minimal final solve of cv2.solvePnPRansac when its minimal solver is
// P3P (OpenCV re-solves the inliers with SOLVEPNP_EPNP, main_v1.py:497 with
// flags=SOLVEPNP_P3P).  Steps as OpenCV's epnp.cpp:
// control points from the centroid and principal axes, barycentric alphas,
// M^T M (12 x 12), its 4 smallest eigenvectors, the L 6x10 / rho system,
// beta approximations 1, 2, 3 each polished by 5 Gauss-Newton steps, the pose
// of each by the SVD of the centred cross-covariance, the one with the lowest
// mean reprojection error wins.  Own numerics (no OpenCV to pin against):
// Jacobi eigen-decompositions, Householder least squares, and the frame
// centred on the problem's first point, as the LM refit.  The O(n) sums go
// through Red (the summation order of lm_reduce_host / GpuLmReducer).
// ---------------------------------------------------------------------------
constexpr int kEpnpPairSums = 40;  // 10 control-point pairs x 4 sums

// the rotation of pair (p, q): false (skipped) for apq = 0 or, from the fifth sweep on, apq
// negligible next to both diagonal entries (Numerical Recipes' rule).  With d = aqq - app, w = 2 apq,
// h = |d| + sqrt(d^2 + w^2): t = sgn(theta) / (|theta| + sqrt(theta^2 + 1)) = sg |w| / h (theta =
// d / w), so cs = 1 / sqrt(t^2 + 1) = h / sqrt(h^2 + w^2) and sn = t cs = sg |w| / sqrt(h^2 + w^2):
// two square roots and one division in the chain (r05; one division fewer than forming t first).
// MᵀM's entries are far from the squares' overflow.
RSAC_HD bool jrr_rotation(int sweep, double app, double aqq, double apq, double &cs, double &sn) {
    if (!(apq != 0.0)) return false;
    if (sweep >= 4) {
        const double g = 100.0 * dabs(apq);
        if (dabs(app) + g == dabs(app) && dabs(aqq) + g == dabs(aqq)) return false;
    }
    const double d = aqq - app, w = 2.0 * apq;
    const double sg = (d == 0.0 || ((d < 0.0) == (w < 0.0))) ? 1.0 : -1.0;
    const double aw = dabs(w), h = dabs(d) + dsqrt(d * d + w * w);
    const double iq = 1.0 / dsqrt(h * h + aw * aw);
    cs = h * iq;
    sn = sg * aw * iq;
    return true;
}
// Cyclic Jacobi of a symmetric N x N matrix (row-major, destroyed): d[k]
// eigenvalues, V[i * N + k] the k-th eigenvector.  Fixed rotation order; the rotation and its
// skip rule are jrr_rotation's (r05: two square roots and one division in the chain, not three
// divisions).
// (N <= 4: the rotation loops unrolled, every index static, so a GPU lane keeps A and V in
// registers; the order of operations is the same either way)
// One rotated pair of elements (x_p, x_q) -> (c x_p - s x_q, s x_p + c x_q), each as c times its
// own element fused with the rounded product of s and the other (r05: one multiply and one fma
// per element instead of two multiplies and an add; the oracle's ep_jacobi / ep_jacobi_rr, the
// host and the device forms use exactly these two expressions)
RSAC_HD double jrr_lo(double c, double s, double xp, double xq) { return dfma(c, xp, -(s * xq)); }
RSAC_HD double jrr_hi(double c, double s, double xp, double xq) { return dfma(c, xq, s * xp); }
template <int N>
RSAC_HD void jacobi_eig(double *A, double *V, double *d) {
    constexpr int U = N <= 4 ? N : 1;
    for (int i = 0; i < N * N; ++i) V[i] = 0.0;
    for (int i = 0; i < N; ++i) V[i * N + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0, diag = 0.0;
#pragma unroll U
        for (int p = 0; p < N; ++p) {
            diag = diag + A[p * N + p] * A[p * N + p];
#pragma unroll U
            for (int q = p + 1; q < N; ++q) off = off + A[p * N + q] * A[p * N + q];
        }
        if (!(off > 1e-32 * diag)) break;
#pragma unroll U
        for (int p = 0; p < N - 1; ++p)
#pragma unroll U
            for (int q = p + 1; q < N; ++q) {
                double c, sn;
                if (!jrr_rotation(sweep, A[p * N + p], A[q * N + q], A[p * N + q], c, sn)) continue;
#pragma unroll U
                for (int k = 0; k < N; ++k) {
                    const double akp = A[k * N + p], akq = A[k * N + q];
                    A[k * N + p] = jrr_lo(c, sn, akp, akq);
                    A[k * N + q] = jrr_hi(c, sn, akp, akq);
                }
#pragma unroll U
                for (int k = 0; k < N; ++k) {
                    const double apk = A[p * N + k], aqk = A[q * N + k];
                    A[p * N + k] = jrr_lo(c, sn, apk, aqk);
                    A[q * N + k] = jrr_hi(c, sn, apk, aqk);
                }
#pragma unroll U
                for (int k = 0; k < N; ++k) {
                    const double vkp = V[k * N + p], vkq = V[k * N + q];
                    V[k * N + p] = jrr_lo(c, sn, vkp, vkq);
                    V[k * N + q] = jrr_hi(c, sn, vkp, vkq);
                }
            }
    }
    for (int k = 0; k < N; ++k) d[k] = A[k * N + k];
}

// Round-robin ("parallel order") Jacobi of a symmetric N x N matrix, N even (EPnP's 12 x 12 M^T M):
// a sweep is N - 1 steps, each rotating N / 2 disjoint pairs whose parameters all come from the
// matrix at the step's start; then the columns of every pair (every row), the rows of every pair,
// and V's columns.  Pairs are disjoint, so each element sees one fixed sequence of operations
// whatever the order within a phase: the GPU runs a step's pairs on different lanes
// with the bits of this loop.  Schedule (circle method): in step r, position 0
// holds index 0 and position m > 0 holds 1 + (m - 1 + r) % (N - 1); pair i is positions i and
// N - 1 - i, p the smaller index.  Sweep test as jacobi_eig; the rotation by jrr_rotation.
RSAC_HD constexpr int jrr_pos(int N, int r, int m) { return m == 0 ? 0 : 1 + (m - 1 + r) % (N - 1); }
// jrr_rotation without branches (the GPU's block form): every lane forms the parameters, a skipped
// pair then selects cs 1, sn 0; the same bits as jrr_rotation
RSAC_HD void jrr_rotation_sel(int sweep, double app, double aqq, double apq, double &cs, double &sn) {
    const double d = aqq - app, w = 2.0 * apq;
    const double sg = (d == 0.0 || ((d < 0.0) == (w < 0.0))) ? 1.0 : -1.0;
    const double aw = dabs(w), h = dabs(d) + dsqrt(d * d + w * w);
    const double iq = 1.0 / dsqrt(h * h + aw * aw);
    const double g = 100.0 * dabs(apq);
    const bool skip = !(apq != 0.0) || (sweep >= 4 && dabs(app) + g == dabs(app) && dabs(aqq) + g == dabs(aqq));
    const double c = h * iq, sv = sg * aw * iq;
    cs = skip ? 1.0 : c;
    sn = skip ? 0.0 : sv;
}
// the sweep test's sums: diag = sum_p A_pp^2 in p order; off = sum over the rows p, in order, of
// the row's partial sum_{q > p} A_pq^2 in q order (r05: a row's partial is one lane's, so the
// 16-lane kernel forms it from its registers)
template <int N>
RSAC_HD void jacobi_eig_rr(double *A, double *V, double *d) {
    static_assert(N % 2 == 0, "round-robin Jacobi needs an even order");
    constexpr int H = N / 2;
    for (int i = 0; i < N * N; ++i) V[i] = 0.0;
    for (int i = 0; i < N; ++i) V[i * N + i] = 1.0;
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int p = 0; p < N; ++p) {
            diag = diag + A[p * N + p] * A[p * N + p];
            double rp = 0.0;
            for (int q = p + 1; q < N; ++q) rp = rp + A[p * N + q] * A[p * N + q];
            off = off + rp;
        }
        if (!(off > 1e-32 * diag)) break;
        for (int r = 0; r < N - 1; ++r) {
            int P[H], Q[H];
            double cs[H], sn[H];
            for (int i = 0; i < H; ++i) {
                const int a = jrr_pos(N, r, i), b = jrr_pos(N, r, N - 1 - i);
                const int p = a < b ? a : b, q = a < b ? b : a;
                P[i] = p;
                Q[i] = q;
                cs[i] = 1.0;
                sn[i] = 0.0;
                (void)jrr_rotation(sweep, A[p * N + p], A[q * N + q], A[p * N + q], cs[i], sn[i]);
            }
            // a skipped pair applies cs = 1, sn = 0 like any other (the device runs branch-free)
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < H; ++i) {
                    const double akp = A[k * N + P[i]], akq = A[k * N + Q[i]];
                    A[k * N + P[i]] = jrr_lo(cs[i], sn[i], akp, akq);
                    A[k * N + Q[i]] = jrr_hi(cs[i], sn[i], akp, akq);
                }
            for (int i = 0; i < H; ++i) {
                for (int k = 0; k < N; ++k) {
                    const double apk = A[P[i] * N + k], aqk = A[Q[i] * N + k];
                    A[P[i] * N + k] = jrr_lo(cs[i], sn[i], apk, aqk);
                    A[Q[i] * N + k] = jrr_hi(cs[i], sn[i], apk, aqk);
                }
            }
            for (int k = 0; k < N; ++k)
                for (int i = 0; i < H; ++i) {
                    const double vkp = V[k * N + P[i]], vkq = V[k * N + Q[i]];
                    V[k * N + P[i]] = jrr_lo(cs[i], sn[i], vkp, vkq);
                    V[k * N + Q[i]] = jrr_hi(cs[i], sn[i], vkp, vkq);
                }
        }
    }
    for (int k = 0; k < N; ++k) d[k] = A[k * N + k];
}

// order[] = eigenvalue indices by decreasing value (ties: lower index first)
template <int N>
RSAC_HD void eig_order_desc(const double *d, int *order) {
    for (int i = 0; i < N; ++i) order[i] = i;
    for (int i = 1; i < N; ++i) {
        const int k = order[i];
        int j = i - 1;
        while (j >= 0 && d[order[j]] < d[k]) {
            order[j + 1] = order[j];
            --j;
        }
        order[j + 1] = k;
    }
}

// Least squares min |A x - b|, A M x N row-major (M >= N), by Householder QR;
// A and b are destroyed.  A vanishing pivot gives x_k = 0.  Sums of products and the reflector
// updates accumulate by fma (r05; the oracle's ep_lsq alike)
template <int M, int N>
RSAC_HD void householder_ls(double *A, double *b, double *x) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        double nrm = 0.0;
#pragma unroll
        for (int i = k; i < M; ++i) nrm = dfma(A[i * N + k], A[i * N + k], nrm);
        nrm = dsqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k * N + k] > 0.0 ? -nrm : nrm;
        double v[M];
#pragma unroll
        for (int i = k; i < M; ++i) v[i] = A[i * N + k];
        v[k] = v[k] - alpha;
        double vv = 0.0;
#pragma unroll
        for (int i = k; i < M; ++i) vv = dfma(v[i], v[i], vv);
        if (vv == 0.0) continue;
#pragma unroll
        for (int j = k; j < N; ++j) {
            double sdot = 0.0;
#pragma unroll
            for (int i = k; i < M; ++i) sdot = dfma(v[i], A[i * N + j], sdot);
            const double f = 2.0 * sdot / vv;
#pragma unroll
            for (int i = k; i < M; ++i) A[i * N + j] = dfma(-f, v[i], A[i * N + j]);
        }
        double sdot = 0.0;
#pragma unroll
        for (int i = k; i < M; ++i) sdot = dfma(v[i], b[i], sdot);
        const double f = 2.0 * sdot / vv;
#pragma unroll
        for (int i = k; i < M; ++i) b[i] = dfma(-f, v[i], b[i]);
    }
#pragma unroll
    for (int k = N - 1; k >= 0; --k) {
        double sacc = b[k];
#pragma unroll
        for (int j = k + 1; j < N; ++j) sacc = dfma(-A[k * N + j], x[j], sacc);
        const double rkk = A[k * N + k];
        x[k] = dabs(rkk) > 1e-300 ? sacc / rkk : 0.0;
    }
}

struct EpnpFrame {
    double cw[4][3];   // control points (centred frame)
    double ci[9];      // inverse of [cw1 - cw0, cw2 - cw0, cw3 - cw0] (columns)
};

// what the barycentric coordinates need: cw0 and the inverse (kept small for the sums' registers)
struct EpnpAlpha {
    double c[3], ci[9];
};

RSAC_HD EpnpAlpha epnp_alpha_frame(const EpnpFrame &f) {
    EpnpAlpha a;
    for (int j = 0; j < 3; ++j) a.c[j] = f.cw[0][j];
    for (int j = 0; j < 9; ++j) a.ci[j] = f.ci[j];
    return a;
}

RSAC_HD void epnp_alphas(const EpnpAlpha &f, double X, double Y, double Z, double *a) {
    const double dx = X - f.c[0], dy = Y - f.c[1], dz = Z - f.c[2];
    // (dot products as fma chains from r05, the oracle's ep_alphas alike; also cc, pc and H below)
    for (int j = 0; j < 3; ++j) a[1 + j] = dfma(f.ci[3 * j + 2], dz, dfma(f.ci[3 * j + 1], dy, f.ci[3 * j] * dx));
    a[0] = 1.0 - a[1] - a[2] - a[3];
}

// one point's terms of the control-point pair sums, pairs 5 H .. 5 H + 4 of (0,0) (0,1) (0,2)
// (0,3) (1,1) (1,2) (1,3) (2,2) (2,3) (3,3): a_i a_j times 1, (cx - u), (cy - v), |(cx - u, cy - v)|^2
template <int H>
RSAC_HD void epnp_pair_acc(const EpnpAlpha &af, const Cam &k, double X, double Y, double Z, double u, double v,
                           double *acc) {
    constexpr int pi[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3}, pj[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
    double a[4];
    epnp_alphas(af, X, Y, Z, a);
    const double du = k.cx - u, dv = k.cy - v, w = dfma(dv, dv, du * du);
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        const double aa = a[pi[5 * H + r]] * a[pj[5 * H + r]];
        acc[4 * r] += aa;
        acc[4 * r + 1] = dfma(aa, du, acc[4 * r + 1]);
        acc[4 * r + 2] = dfma(aa, dv, acc[4 * r + 2]);
        acc[4 * r + 3] = dfma(aa, w, acc[4 * r + 3]);
    }
}

// the 6 x 10 L matrix of the betas' quadratic forms (OpenCV compute_L_6x10)
RSAC_HD void epnp_l6x10(const double *const v[4], double *L) {
    int a = 0, b = 1;
    for (int i = 0; i < 6; ++i) {
        double dv[4][3];
        for (int p = 0; p < 4; ++p)
            for (int q = 0; q < 3; ++q) dv[p][q] = v[p][3 * a + q] - v[p][3 * b + q];
        ++b;
        if (b > 3) {
            ++a;
            b = a + 1;
        }
        double *r = L + 10 * i;
        auto dot = [&](int p, int q) { return dfma(dv[p][2], dv[q][2], dfma(dv[p][1], dv[q][1], dv[p][0] * dv[q][0])); };
        r[0] = dot(0, 0);
        r[1] = 2.0 * dot(0, 1);
        r[2] = dot(1, 1);
        r[3] = 2.0 * dot(0, 2);
        r[4] = 2.0 * dot(1, 2);
        r[5] = dot(2, 2);
        r[6] = 2.0 * dot(0, 3);
        r[7] = 2.0 * dot(1, 3);
        r[8] = 2.0 * dot(2, 3);
        r[9] = dot(3, 3);
    }
}

// 5 Gauss-Newton steps on the betas (OpenCV gauss_newton)
RSAC_HD void epnp_gauss_newton(const double *L, const double *rho, double *be) {
    // (not unrolled: a latency-bound GPU lane then runs one iteration's code five times from a warm
    // instruction cache instead of five cold copies)
#pragma unroll 1
    for (int it = 0; it < 5; ++it) {
        double A[24], b[6], x[4];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double *r = L + 10 * i;
            // the Jacobian row and the residual as fma chains in OpenCV's term order (r05; the
            // oracle's ep_gauss_newton alike)
            A[4 * i + 0] = dfma(r[6], be[3], dfma(r[3], be[2], dfma(r[1], be[1], 2.0 * r[0] * be[0])));
            A[4 * i + 1] = dfma(r[7], be[3], dfma(r[4], be[2], dfma(2.0 * r[2], be[1], r[1] * be[0])));
            A[4 * i + 2] = dfma(r[8], be[3], dfma(2.0 * r[5], be[2], dfma(r[4], be[1], r[3] * be[0])));
            A[4 * i + 3] = dfma(2.0 * r[9], be[3], dfma(r[8], be[2], dfma(r[7], be[1], r[6] * be[0])));
            double q = r[0] * be[0] * be[0];
            q = dfma(r[1] * be[0], be[1], q);
            q = dfma(r[2] * be[1], be[1], q);
            q = dfma(r[3] * be[0], be[2], q);
            q = dfma(r[4] * be[1], be[2], q);
            q = dfma(r[5] * be[2], be[2], q);
            q = dfma(r[6] * be[0], be[3], q);
            q = dfma(r[7] * be[1], be[3], q);
            q = dfma(r[8] * be[2], be[3], q);
            q = dfma(r[9] * be[3], be[3], q);
            b[i] = rho[i] - q;
        }
        householder_ls<6, 4>(A, b, x);
        for (int j = 0; j < 4; ++j) be[j] = be[j] + x[j];
    }
}

// R = U V^T of the 3 x 3 cross-covariance H = sum (pc - pc0)(pw - pw0)^T, with
// OpenCV's determinant fix (negate the last row); false if H has rank < 2.  By the eigen-
// decomposition of H^T H: epnp_rotation's route for a nearly singular H.
RSAC_HD bool epnp_rotation_svd(const double *H, double *R) {
    double B[9], V[9], d[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) B[3 * i + j] = H[i] * H[j] + H[3 + i] * H[3 + j] + H[6 + i] * H[6 + j];
    jacobi_eig<3>(B, V, d);
    int o[3];
    eig_order_desc<3>(d, o);
    double v[3][3], u[3][3];
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < 3; ++i) v[k][i] = V[3 * i + o[k]];
    const double s0 = dsqrt(d[o[0]] > 0.0 ? d[o[0]] : 0.0);
    if (!(s0 > 0.0)) return false;
    for (int k = 0; k < 3; ++k) {
        const double sk = dsqrt(d[o[k]] > 0.0 ? d[o[k]] : 0.0);
        if (k < 2 || sk > 1e-10 * s0) {
            if (!(sk > 1e-10 * s0)) return false;
            for (int i = 0; i < 3; ++i) u[k][i] = (H[3 * i] * v[k][0] + H[3 * i + 1] * v[k][1] + H[3 * i + 2] * v[k][2]) / sk;
        } else {  // rank 2: complete U by the cross product
            u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
            u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
            u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
        }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = u[0][i] * v[0][j] + u[1][i] * v[1][j] + u[2][i] * v[2][j];
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0.0)
        for (int j = 0; j < 3; ++j) R[6 + j] = -R[6 + j];
    return true;
}

// The orthogonal polar factor U V^T of a well-conditioned 3 x 3 X (in place) by Newton's iteration
// X <- (g X + X^-T / g) / 2, X^-T = cof(X) / det X, with Frobenius scaling g = (|X^-T|_F / |X|_F)^(1/2)
// while a step moves an element by more than 1e-2 and g = 1 after, until no element moves by more
// than 1e-15 (at most 30 steps).  (Unscaled, it is the classical polar Newton step.)
RSAC_HD void polar_newton3(double X[9]) {
    bool scale = true;
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
        const double det = X[0] * Y[0] + X[1] * Y[1] + X[2] * Y[2];
        if (!(dabs(det) > 1e-300) || !dfinite(det)) return;
        const double id = 1.0 / det;
#pragma unroll
        for (int k = 0; k < 9; ++k) Y[k] = Y[k] * id;
        double g = 1.0, ig = 1.0;
        if (scale) {
            double sx = 0.0, sy = 0.0;
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                sx = sx + X[k] * X[k];
                sy = sy + Y[k] * Y[k];
            }
            g = dsqrt(dsqrt(sy / sx));
            ig = 1.0 / g;
        }
        double mv = 0.0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            const double nx = 0.5 * (g * X[k] + ig * Y[k]);
            const double d = dabs(nx - X[k]);
            mv = d > mv ? d : mv;
            X[k] = nx;
        }
        if (!(mv > 1e-15)) return;
        scale = mv > 1e-2;
    }
}

// epnp_rotation_svd's R: for |det H| > 1e-10 |H|_F^3 (then the smallest singular value exceeds
// 1e-10 of the largest: full rank) the polar factor of H by polar_newton3 (r05: some 8 short steps
// in place of two 3 x 3 Jacobi eigen-decompositions), else epnp_rotation_svd itself
RSAC_HD bool epnp_rotation(const double *H, double *R) {
    double n2 = 0.0;
#pragma unroll
    for (int k = 0; k < 9; ++k) n2 = n2 + H[k] * H[k];
    const double dh = H[0] * (H[4] * H[8] - H[5] * H[7]) - H[1] * (H[3] * H[8] - H[5] * H[6]) +
                      H[2] * (H[3] * H[7] - H[4] * H[6]);
    if (!(dabs(dh) > 1e-10 * n2 * dsqrt(n2))) return epnp_rotation_svd(H, R);
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = H[k];
    polar_newton3(R);
    const double det = R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) +
                       R[2] * (R[3] * R[7] - R[4] * R[6]);
    if (det < 0.0)
        for (int j = 0; j < 3; ++j) R[6 + j] = -R[6 + j];
    return true;
}

// Stage 1 -> stage 2 record (per problem; device memory between the GPU passes).
struct EpnpStage1 {
    EpnpFrame f;
    double pairs[kEpnpPairSums];
    double n;   // inlier count
    double ok;  // 1: a frame exists (>= 4 inliers, non-degenerate)
};

// Stage 2 -> stage 3 record: the serial middle's results.
struct EpnpStage2 {
    double ut[4][12];  // eigenvectors of M^T M's 4 smallest eigenvalues, smallest first
    double be[3][4];   // betas of approximations 1, 2, 3 (after Gauss-Newton)
    double valid[3];
};

// The serial middle's scratch.
struct EpnpShared {
    double A[144], V[144], d[12];
    double L[60], rho[6];
};

// Stage 2, the serial middle of EPnP (O(1), on the host): M^T M from the pair
// sums, its eigenvectors, L and rho, the three beta estimates with Gauss-Newton.
RSAC_HD void epnp_mtm(EpnpShared *sh, const double *pairs, const Cam &k) {
    int q = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = i; j < 4; ++j, q += 4) {
            const double s0 = pairs[q], su = pairs[q + 1], sv = pairs[q + 2], sw = pairs[q + 3];
            const double blk[9] = {k.fx * k.fx * s0, 0.0, k.fx * su, 0.0, k.fy * k.fy * s0, k.fy * sv,
                                   k.fx * su, k.fy * sv, sw};
            for (int p = 0; p < 3; ++p)
                for (int r = 0; r < 3; ++r) {
                    sh->A[12 * (3 * i + p) + 3 * j + r] = blk[3 * p + r];
                    sh->A[12 * (3 * j + r) + 3 * i + p] = blk[3 * p + r];
                }
        }
}

// One beta estimate of stage 2 (approximation 1, 2 or 3) from L and rho, polished by Gauss-Newton:
// false if it is not usable (OpenCV epnp.cpp find_betas_approx_1..3 + gauss_newton)
RSAC_HD bool epnp_beta(int approx, const double *L, const double *rho, double *be) {
    for (int j = 0; j < 4; ++j) be[j] = 0.0;
    double b[6];
    for (int i = 0; i < 6; ++i) b[i] = rho[i];
    bool ok = true;
    // the estimate's columns of L (1: 0 1 3 6, beta1^2, b1 b2, b1 b3, b1 b4; 2: 0 1 2, beta1^2, b1 b2,
    // b2^2; 3: 0..4, beta1^2, b1 b2, b2^2, b1 b3, b2 b3), zero-padded to 5: householder_ls skips a zero
    // column's reflection, leaves it zero and gives it x = 0, so x[0, N) carry the 6 x N solve's bits
    // and the three estimates run one instruction stream
    double A[30], x[5];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const int col = approx == 1 ? (j == 2 ? 3 : j == 3 ? 6 : j) : j;
            const bool used = approx == 1 ? j < 4 : approx == 2 ? j < 3 : true;
            A[5 * i + j] = used ? L[10 * i + col] : 0.0;
        }
    householder_ls<6, 5>(A, b, x);
    if (approx == 1) {
        const double sg = x[0] < 0.0 ? -1.0 : 1.0;
        be[0] = dsqrt(sg * x[0]);
        ok = be[0] != 0.0;
        if (ok)
            for (int j = 1; j < 4; ++j) be[j] = sg * x[j] / be[0];
    } else {  // 2 and 3
        if (x[0] < 0.0) {
            be[0] = dsqrt(-x[0]);
            be[1] = x[2] < 0.0 ? dsqrt(-x[2]) : 0.0;
        } else {
            be[0] = dsqrt(x[0]);
            be[1] = x[2] > 0.0 ? dsqrt(x[2]) : 0.0;
        }
        if (x[1] < 0.0) be[0] = -be[0];
        if (approx == 3) {
            ok = be[0] != 0.0;
            if (ok) be[2] = x[3] / be[0];
        }
    }
    if (ok) epnp_gauss_newton(L, rho, be);
    return ok;
}

// L (6 x 10) from the eigenvectors and rho (the squared control-point distances)
RSAC_HD void epnp_l_rho(const EpnpStage1 &s1, const EpnpStage2 &s2, double *L, double *rho) {
    const EpnpFrame &f = s1.f;
    const double *vv[4] = {s2.ut[0], s2.ut[1], s2.ut[2], s2.ut[3]};
    epnp_l6x10(vv, L);
    int q = 0;
    for (int a = 0; a < 4; ++a)
        for (int b = a + 1; b < 4; ++b, ++q) {
            const double dx = f.cw[a][0] - f.cw[b][0], dy = f.cw[a][1] - f.cw[b][1], dz = f.cw[a][2] - f.cw[b][2];
            rho[q] = dfma(dz, dz, dfma(dy, dy, dx * dx));
        }
}

// Stage 2 after the eigen-decomposition: s2.ut (the eigenvectors of M^T M's 4 smallest
// eigenvalues) given, the L 6x10 / rho system and the three beta estimates with Gauss-Newton.
// (epnp_stage2 below; the GPU's minimal EPnP runs the 12 x 12 Jacobi on 6 or 64 lanes in between,
// and the three estimates)
__host__ __device__ inline void epnp_stage2_post(const EpnpStage1 &s1, EpnpStage2 &s2) {
    double L[60], rho[6];
    epnp_l_rho(s1, s2, L, rho);
#pragma unroll
    for (int approx = 1; approx <= 3; ++approx) s2.valid[approx - 1] = epnp_beta(approx, L, rho, s2.be[approx - 1]);
}

__host__ __device__ inline void epnp_stage2(const EpnpStage1 &s1, const Cam &k, EpnpStage2 &s2) {
    EpnpShared shm;
    EpnpShared *sh = &shm;
    epnp_mtm(sh, s1.pairs, k);
    jacobi_eig_rr<12>(sh->A, sh->V, sh->d);
    int o[12];
    eig_order_desc<12>(sh->d, o);
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 12; ++j) s2.ut[i][j] = sh->V[12 * j + o[11 - i]];
    epnp_stage2_post(s1, s2);
}

// Red provides:
//   template <int NV, class F> void sum(F f, double *out): out[q] = sum over the inliers of
//     f(X, Y, Z, u, v, acc) (acc[NV]; coordinates in the centred frame), in the fixed order;
//   bool first(double *p): the first inlier's centred coordinates.
// Every thread runs the stages; values are block-uniform.

// Stage 1 (O(n) sums): the inlier count, centroid, principal axes -> control points and
// the barycentric frame, the control-point pair sums of M^T M.  s1.ok = 0 for < 4 inliers or
// a degenerate (e.g. planar) cloud.
template <class Red>
RSAC_HD void epnp_stage1(Red &red, const Cam &k, EpnpStage1 &s1) {
    s1.ok = 0.0;
    double s4[4];
    red.template sum<4>([](double X, double Y, double Z, double, double, double *acc) {
        acc[0] += X; acc[1] += Y; acc[2] += Z; acc[3] += 1.0;
    }, s4);
    const double n = s4[3];
    s1.n = n;
    if (!(n >= 4.0)) return;
    EpnpFrame &f = s1.f;
    for (int j = 0; j < 3; ++j) f.cw[0][j] = s4[j] / n;
    const double c0x = f.cw[0][0], c0y = f.cw[0][1], c0z = f.cw[0][2];
    double cov[6];
    red.template sum<6>([=](double X, double Y, double Z, double, double, double *acc) {
        const double x = X - c0x, y = Y - c0y, z = Z - c0z;
        acc[0] = dfma(x, x, acc[0]); acc[1] = dfma(x, y, acc[1]); acc[2] = dfma(x, z, acc[2]);
        acc[3] = dfma(y, y, acc[3]); acc[4] = dfma(y, z, acc[4]); acc[5] = dfma(z, z, acc[5]);
    }, cov);
    {
        double A[9] = {cov[0], cov[1], cov[2], cov[1], cov[3], cov[4], cov[2], cov[4], cov[5]}, V[9], d[3];
        jacobi_eig<3>(A, V, d);
        int o[3];
        eig_order_desc<3>(d, o);
        for (int i = 1; i < 4; ++i) {
            const double ev = d[o[i - 1]];
            const double kk = dsqrt((ev > 0.0 ? ev : 0.0) / n);
            for (int j = 0; j < 3; ++j) f.cw[i][j] = f.cw[0][j] + kk * V[3 * j + o[i - 1]];
        }
    }
    {
        double cc[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 1; j < 4; ++j) cc[3 * i + j - 1] = f.cw[j][i] - f.cw[0][i];
        const double m00 = cc[4] * cc[8] - cc[5] * cc[7], m01 = cc[5] * cc[6] - cc[3] * cc[8],
                     m02 = cc[3] * cc[7] - cc[4] * cc[6];
        const double det = cc[0] * m00 + cc[1] * m01 + cc[2] * m02;
        double nrm = 0.0;
        for (int q = 0; q < 9; ++q) nrm = nrm + cc[q] * cc[q];
        if (!(dabs(det) > 1e-12 * nrm * dsqrt(nrm))) return;  // planar / degenerate cloud
        const double id = 1.0 / det;
        f.ci[0] = m00 * id;
        f.ci[1] = (cc[2] * cc[7] - cc[1] * cc[8]) * id;
        f.ci[2] = (cc[1] * cc[5] - cc[2] * cc[4]) * id;
        f.ci[3] = m01 * id;
        f.ci[4] = (cc[0] * cc[8] - cc[2] * cc[6]) * id;
        f.ci[5] = (cc[2] * cc[3] - cc[0] * cc[5]) * id;
        f.ci[6] = m02 * id;
        f.ci[7] = (cc[1] * cc[6] - cc[0] * cc[7]) * id;
        f.ci[8] = (cc[0] * cc[4] - cc[1] * cc[3]) * id;
    }
    // M^T M (12 x 12) = sum over points of kron(a a^T, G), G = m1 m1^T + m2 m2^T for the two rows
    // m1 = (fx, 0, cx - u), m2 = (0, fy, cy - v) of fill_M: per control-point pair (i <= j)
    // the sums of a_i a_j times 1, (cx - u), (cy - v), (cx - u)^2 + (cy - v)^2; two passes of
    // 5 pairs each (register pressure), each sum's order unchanged
    const EpnpAlpha af = epnp_alpha_frame(f);
    red.template sum<kEpnpPairSums / 2>([=](double X, double Y, double Z, double u, double v, double *acc) {
        epnp_pair_acc<0>(af, k, X, Y, Z, u, v, acc);
    }, s1.pairs);
    red.template sum<kEpnpPairSums / 2>([=](double X, double Y, double Z, double u, double v, double *acc) {
        epnp_pair_acc<1>(af, k, X, Y, Z, u, v, acc);
    }, s1.pairs + kEpnpPairSums / 2);
    s1.ok = 1.0;
}

// Stage 3 for one beta estimate: the camera-frame control points (sign from the first inlier's
// depth a1), the pose by SVD of the centred cross-covariance, the mean reprojection error.
// false when the cross-covariance is degenerate.
template <class Red>
RSAC_HD bool epnp_pose_err(Red &red, const Cam &k, const EpnpStage1 &s1, const EpnpStage2 &s2, const double *be,
                           const double (&a1)[4], double (&Rk)[9], double (&tk)[3], double &err) {
    const double n = s1.n;
    const EpnpAlpha af = epnp_alpha_frame(s1.f);
    const double c0x = s1.f.cw[0][0], c0y = s1.f.cw[0][1], c0z = s1.f.cw[0][2];
    double cc[4][3];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 3; ++j)
            cc[i][j] = dfma(be[3], s2.ut[3][3 * i + j],
                            dfma(be[2], s2.ut[2][3 * i + j], dfma(be[1], s2.ut[1][3 * i + j], be[0] * s2.ut[0][3 * i + j])));
    const double z1 = dfma(a1[3], cc[3][2], dfma(a1[2], cc[2][2], dfma(a1[1], cc[1][2], a1[0] * cc[0][2])));
    if (z1 < 0.0)
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 3; ++j) cc[i][j] = -cc[i][j];
    double pc0[3];
    red.template sum<3>([=](double X, double Y, double Z, double, double, double *acc) {
        double a[4];
        epnp_alphas(af, X, Y, Z, a);
        for (int j = 0; j < 3; ++j) acc[j] += dfma(a[3], cc[3][j], dfma(a[2], cc[2][j], dfma(a[1], cc[1][j], a[0] * cc[0][j])));
    }, pc0);
    for (int j = 0; j < 3; ++j) pc0[j] = pc0[j] / n;
    double H[9];
    red.template sum<9>([=](double X, double Y, double Z, double, double, double *acc) {
        double a[4], pc[3];
        epnp_alphas(af, X, Y, Z, a);
        for (int j = 0; j < 3; ++j)
            pc[j] = dfma(a[3], cc[3][j], dfma(a[2], cc[2][j], dfma(a[1], cc[1][j], a[0] * cc[0][j]))) - pc0[j];
        const double pw[3] = {X - c0x, Y - c0y, Z - c0z};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) acc[3 * i + j] = dfma(pc[i], pw[j], acc[3 * i + j]);
    }, H);
    if (!epnp_rotation(H, Rk)) return false;
    for (int i = 0; i < 3; ++i) tk[i] = pc0[i] - dfma(Rk[3 * i + 2], c0z, dfma(Rk[3 * i + 1], c0y, Rk[3 * i] * c0x));
    double es;
    const double R0 = Rk[0], R1 = Rk[1], R2 = Rk[2], R3 = Rk[3], R4 = Rk[4], R5 = Rk[5], R6 = Rk[6], R7 = Rk[7],
                 R8 = Rk[8], t0 = tk[0], t1 = tk[1], t2 = tk[2];
    red.template sum<1>([=](double X, double Y, double Z, double u, double v, double *acc) {
        const double x = R0 * X + R1 * Y + R2 * Z + t0;
        const double y = R3 * X + R4 * Y + R5 * Z + t1;
        const double iz = 1.0 / (R6 * X + R7 * Y + R8 * Z + t2);
        const double du = u - (k.cx + k.fx * x * iz), dv = v - (k.cy + k.fy * y * iz);
        acc[0] += dsqrt(du * du + dv * dv);
    }, &es);
    err = es / n;
    return true;
}

// Stage 3 (O(n) sums): for each valid beta estimate its pose and mean reprojection error
// (epnp_pose_err); the lowest wins, the first on ties.  (R, t) in the centred frame; false if none.
template <class Red>
RSAC_HD bool epnp_stage3(Red &red, const Cam &k, const EpnpStage1 &s1, const EpnpStage2 &s2, double *R_out,
                         double *t_out) {
    const EpnpAlpha af = epnp_alpha_frame(s1.f);
    double p1[3], a1[4];
    if (!red.first(p1)) return false;
    epnp_alphas(af, p1[0], p1[1], p1[2], a1);
    double best_err = 0.0, bestR[9], bestt[3];
    bool have = false;
#pragma unroll
    for (int approx = 0; approx < 3; ++approx) {
        if (s2.valid[approx] == 0.0) continue;
        double Rk[9], tk[3], err;
        if (!epnp_pose_err(red, k, s1, s2, s2.be[approx], a1, Rk, tk, err)) continue;
        if (!have || err < best_err) {
            have = true;
            best_err = err;
            for (int j = 0; j < 9; ++j) bestR[j] = Rk[j];
            for (int j = 0; j < 3; ++j) bestt[j] = tk[j];
        }
    }
    if (!have) return false;
    for (int j = 0; j < 9; ++j) R_out[j] = bestR[j];
    for (int j = 0; j < 3; ++j) t_out[j] = bestt[j];
    return true;
}

// EPnP of one problem on the host: the three stages in a row (the GPU runs stages 1 and 3 as
// kernels and stage 2 on the host, with the same functions).
template <class Red>
inline bool pnp_epnp(Red &red, const Cam &k, double *R_out, double *t_out) {
    EpnpStage1 s1;
    epnp_stage1(red, k, s1);
    if (s1.ok == 0.0) return false;
    EpnpStage2 s2;
    epnp_stage2(s1, k, s2);
    return epnp_stage3(red, k, s1, s2, R_out, t_out);
}

}  // namespace rsac
