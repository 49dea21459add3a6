// rsac_kernels.hip -- gfx950 kernels of the RANSAC hot path.
//
//   pnp_prepare   f64 AoS (as numpy / cv2 hold it) -> f32 SoA, the CV_32F
//                 conversion of solvePnPRansac (main_v1.py:497)
//   pnp_solve     one LANE per hypothesis: Philox subset (or a host-made
//                 OpenCV subset), P3P in registers, 4th-point pick
//   pnp_score     work queue of 32-hypothesis units x all points: f32 records
//                 staged in LDS, points in registers per lane, division-free
//                 f32 test with exact f64 fallback, counts by ballot +
//                 popcount, block-reduced through LDS (+ fused best key)
//   pnp_mask      RANSAC-phase mask of the winners
//   hom_*         the same skeleton for cv2.findHomography (main_v1.py:312)
//
// Layout in HBM (per call, problem-concatenated): X[N] Y[N] Z[N] U[N] V[N]
// float32 (20 B per correspondence, the algorithmic bytes of SURVEY.md §8d);
// models [P][H][16] f64 (R 9, t 3, valid flag); counts [P][H] int32.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "rsac_geo.h"
#include "rsac_internal.h"
#include "rsac_math.h"

namespace rsac {

// ---------------------------------------------------------------------------
// input conversion
// ---------------------------------------------------------------------------
__global__ void k_pnp_prepare(const double *__restrict__ p3, const double *__restrict__ p2, int64_t n,
                              float *__restrict__ X, float *__restrict__ Y, float *__restrict__ Z,
                              float *__restrict__ U, float *__restrict__ V) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        X[i] = (float)p3[3 * i];
        Y[i] = (float)p3[3 * i + 1];
        Z[i] = (float)p3[3 * i + 2];
        U[i] = (float)p2[2 * i];
        V[i] = (float)p2[2 * i + 1];
    }
}

__global__ void k_hom_prepare(const double *__restrict__ s, const double *__restrict__ d, int64_t n,
                              float *__restrict__ SX, float *__restrict__ SY, float *__restrict__ DX,
                              float *__restrict__ DY) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        SX[i] = (float)s[2 * i];
        SY[i] = (float)s[2 * i + 1];
        DX[i] = (float)d[2 * i];
        DY[i] = (float)d[2 * i + 1];
    }
}

// ---------------------------------------------------------------------------
// PnP frame for the float32 pre-filter (DESIGN.md "Scoring").
// Each problem is re-centred on the midpoint c of its bounding box; points
// are kept as f32 offsets XC = fl32(Xf - c).  B bounds |XC|, rho the rounding
// of XC.  fconst holds the per-problem f32 constants of the error bound.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int f2ord(float f) {
    int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

constexpr double kU32 = 5.9604644775390625e-08;  // 2^-24, unit roundoff of float32

// the PnP scoring launch's counters (PnpArgs::queue, words 0..3): unit queue, units finished,
// flagged-iteration records appended, records taken (k_pnp_score_mf); reset before each launch
// Split work queue (k_pnp_score_mw): kQSub unit counters and kQSub flagged-record counters, one
// 128-byte line each.  Atomics on one address serialise (≈10 ns each on MI355X, measured: a
// single counter for 62 500 wave units cost ≈0.45 ms), so block b draws its units from counter
// b % kQSub (units u ≡ b mod kQSub) and appends its flagged records to segment b % kQSub.
constexpr int kQSub = 8;
constexpr int kQWords = 32 + 64 * kQSub;  // ints of the queue buffer used by the PnP kernels
__device__ __forceinline__ int *unit_queue(int *q, int k) { return q + 32 + 32 * k; }
// k_fm_score_q's counters (HomArgs::fm_queue = queue + 8): words kQWords + 32 k of the buffer
constexpr int kFmQOff = kQWords - 8;
__device__ __forceinline__ int *fm_unit_queue(int *fq, int k) { return fq + kFmQOff + 32 * k; }

__device__ __forceinline__ void reset_pnp_queue(int *q) {
    q[0] = 0;
    q[1] = 0;
    q[2] = 0;
    q[3] = 0;
#pragma unroll
    for (int k = 0; k < kQSub; ++k) {
        *unit_queue(q, k) = 0;
    }
}

// ws: [0, 5P) mins, [5P, 10P) maxes of X Y Z U V (ordered-int encoding), pre-set by memset
__global__ __launch_bounds__(256) void k_pnp_bounds(PnpArgs a, int32_t P, int *__restrict__ ws) {
    __shared__ float sl[4][5], sh[4][5];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    float lo[5], hi[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float v[5] = {a.X[p0 + i], a.Y[p0 + i], a.Z[p0 + i], a.U[p0 + i], a.V[p0 + i]};
#pragma unroll
        for (int k = 0; k < 5; ++k) { lo[k] = fminf(lo[k], v[k]); hi[k] = fmaxf(hi[k], v[k]); }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    }
    __syncthreads();
    if (threadIdx.x < 5 && n > 0) {
        const int k = threadIdx.x;
        const float l = fminf(fminf(sl[0][k], sl[1][k]), fminf(sl[2][k], sl[3][k]));
        const float h = fmaxf(fmaxf(sh[0][k], sh[1][k]), fmaxf(sh[2][k], sh[3][k]));
        atomicMin(ws + 5 * prob + k, f2ord(l));
        atomicMax(ws + 5 * P + 5 * prob + k, f2ord(h));
    }
}

// B >= |XC|inf of a problem from its ordered-int bounds wlo[0..2], whi[0..2] (the frame's f[3];
// recomputed identically wherever needed)
__device__ __forceinline__ double frame_bound2(const int *__restrict__ wlo, const int *__restrict__ whi, int n) {
    double B = 0;
    if (n > 0)
        for (int k = 0; k < 3; ++k) {
            const double lo = ord2f(wlo[k]), hi = ord2f(whi[k]);
            B = fmax(B, (hi - lo) * 0.5);
        }
    return B * (1.0 + 4.0 * kU32) + 1e-30;
}
// the same for problem prob of the bounds workspace ws ([0, 5P) mins, [5P, 10P) maxes)
__device__ __forceinline__ double frame_bound(const int *__restrict__ ws, int32_t P, int prob, int n) {
    return frame_bound2(ws + 5 * prob, ws + 5 * P + 5 * prob, n);
}

// k_pnp_bounds for one problem in one 1024-thread block: min / max written directly (the
// encoding of k_pnp_init + atomics, identical values), best key and work queue reset
__global__ __launch_bounds__(1024) void k_pnp_bounds1(PnpArgs a, int *__restrict__ ws) {
    __shared__ float sl[16][5], sh[16][5];
    const int64_t p0 = a.offsets[0];
    const int n = (int)(a.offsets[1] - p0);
    float lo[5], hi[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
    for (int i = threadIdx.x; i < n; i += 1024) {
        const float v[5] = {a.X[p0 + i], a.Y[p0 + i], a.Z[p0 + i], a.U[p0 + i], a.V[p0 + i]};
#pragma unroll
        for (int k = 0; k < 5; ++k) { lo[k] = fminf(lo[k], v[k]); hi[k] = fmaxf(hi[k], v[k]); }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    __syncthreads();
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        float l = sl[0][k], h = sh[0][k];
        for (int w = 1; w < 16; ++w) { l = fminf(l, sl[w][k]); h = fmaxf(h, sh[w][k]); }
        // as k_pnp_init (0x7F7F7F7F / 0x80808080) then atomicMin / Max of f2ord
        ws[k] = n > 0 ? min(0x7F7F7F7F, f2ord(l)) : 0x7F7F7F7F;
        ws[5 + k] = n > 0 ? max((int)0x80808080, f2ord(h)) : (int)0x80808080;
    }
    if (threadIdx.x == 0) {
        if (a.best_key) *a.best_key = 0ull;
        reset_pnp_queue(a.queue);
    }
}

// The per-problem terms of write_fmodel_mx's band (frame[8..15]), computed once per problem
// instead of once per hypothesis (with fconst's f32 T, Trel and Cmax: q6, q7): s = sqrt(T) (1 when
// T is out of range), c1 = 2 Cmax / s, Trel' / T, sqrt(1.00001 T), umax, and for the evaluation
// error of the three rows an upward reciprocal of |sc_r| = (fx, fy, s): RN(RN(1/|sc|)(1 + 2^-50))
// >= (1/|sc|)(1 + 2^-52), so RN(err x it) >= err / |sc| (the division it replaces)
__device__ __forceinline__ void pnp_frame_mx_consts(double *f, double fx, double fy, double T, double q6, double q7) {
    const bool t_ok = T > 1e-12 && T < 1e30;
    const double s = t_ok ? sqrt(T) : 1.0;
    const double Cp = 2.0 * q7, Trelp = q6 + 1e-6 * T;
    f[8] = s;
    f[9] = Cp / s;
    f[10] = Trelp / T;
    f[11] = sqrt(T * 1.00001);
    f[12] = q7 / (2.5 * kU32);
    const double up = 1.0 + 0x1p-50;
    f[13] = (1.0 / fx) * up;
    f[14] = (1.0 / fy) * up;
    f[15] = (1.0 / s) * up;
}

// Per problem: frame = {c0 c1 c2 (bbox centre), B >= |XC|inf, rho >= |XC - (Xf - c)|,
// max|Xf|, wmax (bound on |x/z| of any projection within thr of a pixel), 0};
// fconst = {fx fy cx cy T 2.002 sqrt(T) 1e-6 T thr 2/fx 2/fy cu cv cc0} (see the scoring kernel).
// cgiven: the frame's centre (else the bounding box's midpoint); B then bounds |X - c| from the
// bounds around that centre
// wlo / whi: the problem's five ordered-int minima / maxima (X Y Z U V)
__device__ void pnp_frame_core(const PnpArgs &a, int prob, const int *__restrict__ wlo, const int *__restrict__ whi,
                               double *__restrict__ frame, float *__restrict__ fconst,
                               const double *cgiven = nullptr) {
    const int n = (int)(a.offsets[prob + 1] - a.offsets[prob]);
    const double *cm = a.cams + 4 * prob;
    const double fx = fabs(cm[0]), fy = fabs(cm[1]), cx = cm[2], cy = cm[3];
    const double T = a.thr2[prob];
    const double thr = sqrt(T);
    double c[3] = {0, 0, 0}, du = 0, dv = 0;
    if (n > 0) {
        for (int k = 0; k < 3; ++k) c[k] = ((double)ord2f(wlo[k]) + (double)ord2f(whi[k])) * 0.5;
        du = fmax(fabs(ord2f(wlo[3]) - cx), fabs(ord2f(whi[3]) - cx));
        dv = fmax(fabs(ord2f(wlo[4]) - cy), fabs(ord2f(whi[4]) - cy));
    }
    double B = frame_bound2(wlo, whi, n);
    if (cgiven) {
        double Bg = 0;
        for (int k = 0; k < 3; ++k) {
            c[k] = cgiven[k];
            if (n > 0)
                Bg = fmax(Bg, fmax((double)ord2f(whi[k]) - c[k], c[k] - (double)ord2f(wlo[k])));
        }
        B = Bg * (1.0 + 4.0 * kU32) + 1e-30;
    }
    double *f = frame + (int64_t)prob * kFrameStride;
    f[0] = c[0]; f[1] = c[1]; f[2] = c[2];
    f[3] = B;
    f[4] = 2.0 * kU32 * B;
    f[5] = fmax(fmax(fabs(c[0]), fabs(c[1])), fabs(c[2])) + B;
    f[6] = fmax(2.0 * (du + thr) / fx, 2.0 * (dv + thr) / fy) + 2e-3;  // wmax (>= every per-point wa, wb)
    f[7] = 0;
    float *q = fconst + (int64_t)prob * kFconstStride;
    pnp_frame_mx_consts(f, fx, fy, T, (double)(float)(4e-6 * T + 1e-30),
                        (double)(float)(2.5 * kU32 * (du + dv + fabs(cx) + fabs(cy) + 2.0 * thr + 3.0) + 1e-6));
    q[0] = (float)cm[0]; q[1] = (float)cm[1]; q[2] = (float)cx; q[3] = (float)cy;
    q[4] = (float)T;
    q[5] = (float)(2.002 * thr);
    q[6] = (float)(4e-6 * T + 1e-30);
    // Cmax >= C_i = 2.5u (|u_i - cx| + |v_i - cy| + |cx| + |cy| + 2 thr + 2), the rounding part of D
    q[7] = (float)(2.5 * kU32 * (du + dv + fabs(cx) + fabs(cy) + 2.0 * thr + 3.0) + 1e-6);
    q[8] = 0.f;
    q[9] = (T > 1e-12 && T < 1e30) ? (float)(1.0 / thr) : 1.f;  // k_pnp_score_sc: u' = (u - cx) / sqrt(T)
    q[10] = 0.f;
    // k_pnp_score_mf: the centred coordinates are MFMA operands as they are (f16 hi + lo), so
    // |XC| <= B must stay inside the f16 range; small scenes would spend the band on the f16
    // subnormal floor (the form-1 kernel path takes both)
    q[11] = (B <= 32768.0 && B >= 0.015625) ? 1.f : 0.f;
    q[12] = 0.f;
    for (int k = 13; k < kFconstStride; ++k) q[k] = 0.f;
}
__device__ void pnp_frame_one(const PnpArgs &a, int32_t P, int prob, const int *__restrict__ ws,
                              double *__restrict__ frame, float *__restrict__ fconst,
                              const double *cgiven = nullptr) {
    pnp_frame_core(a, prob, ws + 5 * prob, ws + 5 * P + 5 * prob, frame, fconst, cgiven);
}

// MFMA point operands (PnpArgs::PF / UV, k_pnp_score_mf) of one point from its centred
// coordinates and pixel: f16 hi + lo of XC YC ZC (hi = RN(x), lo = RN(x - hi): |x - hi - lo| <=
// 2^-22 |x| + 2^-25), the constant feature 1, the same four pairs x 2^-11 (exact: powers of 2,
// the B operand facing the hypotheses' lo parts x 2^11), and the scaled pixel offsets u' v' of
// k_pnp_score_sc.  A non-finite coordinate stages the decided-outlier point of k_pnp_score_sc
// (the origin, pixel at 3e38).
struct MxPixel {
    float cx, cy, inv_s;
};
__device__ __forceinline__ MxPixel mx_pixel(const PnpArgs &a, int prob) {
    const double T = a.thr2[prob];
    const float inv_s = (T > 1e-12 && T < 1e30) ? (float)(1.0 / sqrt(T)) : 1.f;  // = fconst[9]
    return MxPixel{(float)a.cams[4 * prob + 2], (float)a.cams[4 * prob + 3], inv_s};
}
__device__ __forceinline__ uint32_t mx_pack2(_Float16 lo16, _Float16 hi16) {
    return (uint32_t)__builtin_bit_cast(uint16_t, lo16) | ((uint32_t)__builtin_bit_cast(uint16_t, hi16) << 16);
}
constexpr float kMxLoScale = 0x1p-11f;  // B x 2^-11 faces A_lo x 2^11
__device__ __forceinline__ void mx_point(const PnpArgs &a, int64_t q, float xc, float yc, float zc, float uu,
                                         float vv, const MxPixel &k) {
    const bool ok = __builtin_isfinite(xc) && __builtin_isfinite(yc) && __builtin_isfinite(zc) &&
                    __builtin_isfinite(uu) && __builtin_isfinite(vv);
    uint4 f = make_uint4(0u, 0x3C000000u, 0u, 0u);  // {0, 0, 0, 1 | 0, 0, 0, 0}
    uint4 g = make_uint4(0u, mx_pack2((_Float16)0.0f, (_Float16)kMxLoScale), 0u, 0u);
    float2 uv = make_float2(3.0e38f, 3.0e38f);
    if (ok) {
        const _Float16 hx = (_Float16)xc, hy = (_Float16)yc, hz = (_Float16)zc;
        const _Float16 lx = (_Float16)(xc - (float)hx), ly = (_Float16)(yc - (float)hy), lz = (_Float16)(zc - (float)hz);
        f = make_uint4(mx_pack2(hx, hy), mx_pack2(hz, (_Float16)1.0f), mx_pack2(lx, ly), mx_pack2(lz, (_Float16)0.0f));
        const _Float16 k11 = (_Float16)kMxLoScale;
        g = make_uint4(mx_pack2(hx * k11, hy * k11), mx_pack2(hz * k11, k11), mx_pack2(lx * k11, ly * k11),
                       mx_pack2(lz * k11, (_Float16)0.0f));
        uv = make_float2((uu - k.cx) * k.inv_s, (vv - k.cy) * k.inv_s);
    }
    a.PF[2 * q] = f;
    a.PF[2 * q + 1] = g;
    a.UV[q] = uv;
}

// centred coordinates; block 0 of each problem also writes the problem's frame and
// constants (one launch instead of two).  The centre is recomputed from the bounds
// in every block with the frame's own arithmetic.
__global__ __launch_bounds__(256) void k_pnp_center(PnpArgs a, int32_t P, const int *__restrict__ ws,
                                                    double *__restrict__ frame, float *__restrict__ fconst,
                                                    float *__restrict__ XC, float *__restrict__ YC,
                                                    float *__restrict__ ZC) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    if (blockIdx.x == 0 && threadIdx.x == 0) pnp_frame_one(a, P, prob, ws, frame, fconst);
    double cc[3] = {0, 0, 0};
    if (n > 0)
        for (int k = 0; k < 3; ++k)
            cc[k] = ((double)ord2f(ws[5 * prob + k]) + (double)ord2f(ws[5 * P + 5 * prob + k])) * 0.5;
    const double c0 = cc[0], c1 = cc[1], c2 = cc[2];
    const MxPixel mk = mx_pixel(a, prob);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int64_t q = p0 + i;
        const float xc = (float)((double)a.X[q] - c0), yc = (float)((double)a.Y[q] - c1),
                    zc = (float)((double)a.Z[q] - c2);
        if (XC) {  // (no caller keeps them from r06: sc_unit centres X, Y, Z itself)
            XC[q] = xc;
            YC[q] = yc;
            ZC[q] = zc;
        }
        if (a.PF) mx_point(a, q, xc, yc, zc, a.U[q], a.V[q], mk);
    }
}

// A batch of short problems (each <= kSetupBatchMaxN points), one 256-thread block per problem:
// k_pnp_prepare (CONVERT: the f64 AoS inputs rounded to the f32 SoA) + k_pnp_init + k_pnp_bounds
// + k_pnp_center in one launch instead of four, the same values (the f32 conversion, the
// ordered-int bounds as the sentinels + atomics leave them, the bounding-box frame, the centred
// and MFMA coordinates).  CONVERT = false: the points are already a.X .. a.V.
template <bool CONVERT>
__global__ __launch_bounds__(256) void k_pnp_setup_b(const double *__restrict__ p3, const double *__restrict__ p2,
                                                     PnpArgs a, int32_t P, float *__restrict__ X,
                                                     float *__restrict__ Y, float *__restrict__ Z,
                                                     float *__restrict__ U, float *__restrict__ V,
                                                     int *__restrict__ ws, double *__restrict__ frame,
                                                     float *__restrict__ fconst, float *__restrict__ XC,
                                                     float *__restrict__ YC, float *__restrict__ ZC) {
    __shared__ float sl[4][5], sh[4][5];
    __shared__ int wsl[10];
    const int prob = blockIdx.x;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const float *sX = CONVERT ? X : a.X, *sY = CONVERT ? Y : a.Y, *sZ = CONVERT ? Z : a.Z;
    const float *sU = CONVERT ? U : a.U, *sV = CONVERT ? V : a.V;
    float lo[5], hi[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
#pragma unroll 4
    for (int j = threadIdx.x; j < n; j += 256) {
        const int64_t i = p0 + j;
        float v[5];
        if constexpr (CONVERT) {
            v[0] = (float)p3[3 * i]; v[1] = (float)p3[3 * i + 1]; v[2] = (float)p3[3 * i + 2];
            v[3] = (float)p2[2 * i]; v[4] = (float)p2[2 * i + 1];
            X[i] = v[0]; Y[i] = v[1]; Z[i] = v[2]; U[i] = v[3]; V[i] = v[4];
        } else {
            v[0] = a.X[i]; v[1] = a.Y[i]; v[2] = a.Z[i]; v[3] = a.U[i]; v[4] = a.V[i];
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) { lo[k] = fminf(lo[k], v[k]); hi[k] = fmaxf(hi[k], v[k]); }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    __syncthreads();
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        const float l = fminf(fminf(sl[0][k], sl[1][k]), fminf(sl[2][k], sl[3][k]));
        const float h = fmaxf(fmaxf(sh[0][k], sh[1][k]), fmaxf(sh[2][k], sh[3][k]));
        // as k_pnp_init's sentinels (0x7F7F7F7F / 0x80808080) after atomicMin / Max of f2ord
        const int wl = n > 0 ? min(0x7F7F7F7F, f2ord(l)) : 0x7F7F7F7F;
        const int wh = n > 0 ? max((int)0x80808080, f2ord(h)) : (int)0x80808080;
        ws[5 * prob + k] = wl;
        ws[5 * P + 5 * prob + k] = wh;
        wsl[k] = wl;
        wsl[5 + k] = wh;
    }
    if (prob == 0 && threadIdx.x == 0) {
        if (a.best_key) *a.best_key = 0ull;
        reset_pnp_queue(a.queue);
    }
    __syncthreads();
    if (threadIdx.x == 0) pnp_frame_core(a, prob, wsl, wsl + 5, frame, fconst);
    double cc[3] = {0, 0, 0};
    if (n > 0)
        for (int k = 0; k < 3; ++k) cc[k] = ((double)ord2f(wsl[k]) + (double)ord2f(wsl[5 + k])) * 0.5;
    const MxPixel mk = mx_pixel(a, prob);
    for (int j = threadIdx.x; j < n; j += 256) {  // this thread's own stores above: visible
        const int64_t q = p0 + j;
        const float xc = (float)((double)sX[q] - cc[0]), yc = (float)((double)sY[q] - cc[1]),
                    zc = (float)((double)sZ[q] - cc[2]);
        if (XC) {  // (no caller keeps them from r06: sc_unit centres X, Y, Z itself)
            XC[q] = xc;
            YC[q] = yc;
            ZC[q] = zc;
        }
        if (a.PF) mx_point(a, q, xc, yc, zc, sU[q], sV[q], mk);
    }
}

// One problem of up to 65536 points, inputs as device f64 AoS: k_pnp_prepare + k_pnp_bounds1 +
// k_pnp_center in one 1024-thread block (one launch instead of three; the same values: the f32
// conversion, the ordered-int bounds, the frame and the centred / MFMA coordinates)
__global__ __launch_bounds__(1024) void k_pnp_setup1(const double *__restrict__ p3, const double *__restrict__ p2,
                                                     PnpArgs a, float *__restrict__ X, float *__restrict__ Y,
                                                     float *__restrict__ Z, float *__restrict__ U,
                                                     float *__restrict__ V, int *__restrict__ ws,
                                                     double *__restrict__ frame, float *__restrict__ fconst,
                                                     float *__restrict__ XC, float *__restrict__ YC,
                                                     float *__restrict__ ZC) {
    __shared__ float sl[16][5], sh[16][5];
    __shared__ int wsl[10];
    const int n = (int)(a.offsets[1] - a.offsets[0]);  // offsets[0] = 0 (one problem)
    float lo[5], hi[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
#pragma unroll 4
    for (int i = threadIdx.x; i < n; i += 1024) {
        const float v[5] = {(float)p3[3 * i], (float)p3[3 * i + 1], (float)p3[3 * i + 2], (float)p2[2 * i],
                            (float)p2[2 * i + 1]};
        X[i] = v[0]; Y[i] = v[1]; Z[i] = v[2]; U[i] = v[3]; V[i] = v[4];
#pragma unroll
        for (int k = 0; k < 5; ++k) { lo[k] = fminf(lo[k], v[k]); hi[k] = fmaxf(hi[k], v[k]); }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    __syncthreads();
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        float l = sl[0][k], h = sh[0][k];
        for (int w = 1; w < 16; ++w) { l = fminf(l, sl[w][k]); h = fmaxf(h, sh[w][k]); }
        const int wl = n > 0 ? min(0x7F7F7F7F, f2ord(l)) : 0x7F7F7F7F;
        const int wh = n > 0 ? max((int)0x80808080, f2ord(h)) : (int)0x80808080;
        ws[k] = wl;
        ws[5 + k] = wh;
        wsl[k] = wl;
        wsl[5 + k] = wh;
    }
    if (threadIdx.x == 0) {
        if (a.best_key) *a.best_key = 0ull;
        reset_pnp_queue(a.queue);
    }
    __syncthreads();
    if (threadIdx.x == 0) pnp_frame_one(a, 1, 0, wsl, frame, fconst);
    double cc[3] = {0, 0, 0};
    if (n > 0)
        for (int k = 0; k < 3; ++k) cc[k] = ((double)ord2f(wsl[k]) + (double)ord2f(wsl[5 + k])) * 0.5;
    const MxPixel mk = mx_pixel(a, 0);
    for (int i = threadIdx.x; i < n; i += 1024) {  // this thread's own stores above: visible
        const float xc = (float)((double)X[i] - cc[0]), yc = (float)((double)Y[i] - cc[1]),
                    zc = (float)((double)Z[i] - cc[2]);
        if (XC) {  // (no caller keeps them from r06: sc_unit centres X, Y, Z itself)
            XC[i] = xc;
            YC[i] = yc;
            ZC[i] = zc;
        }
        if (a.PF) mx_point(a, i, xc, yc, zc, U[i], V[i], mk);
    }
}

// One problem, inputs as device f64 AoS, no MFMA features: conversion, centring and bounds in
// one pass over a full grid (one point per thread).  The frame is centred on the first point
// (known before any reduction, so every block centres its own points at once); the last block
// to finish (ticket) reduces the blocks' bounds, writes the frame and resets the ticket.  The
// pre-filter's bounds hold for any centre, so counts do not depend on the choice.
// CONVERT = false: the points are already the f32 SoA a.X .. a.V (p3, p2, X .. V unused)
// (the body takes its block index and block count: k_pnp_setup_solve4 runs it on its first blocks)
template <bool CONVERT>
__device__ __forceinline__ void setup_fc_body(const double *__restrict__ p3, const double *__restrict__ p2,
                                              const PnpArgs &a, float *__restrict__ X, float *__restrict__ Y,
                                              float *__restrict__ Z, float *__restrict__ U, float *__restrict__ V,
                                              int *__restrict__ ws, double *__restrict__ frame,
                                              float *__restrict__ fconst, float *__restrict__ XC,
                                              float *__restrict__ YC, float *__restrict__ ZC, float *part, int *ticket,
                                              const int bid, const int nblk) {
    __shared__ float sl[4][5], sh[4][5];
    const int64_t p0 = a.offsets[0];
    const int n = (int)(a.offsets[1] - p0);
    double c[3];
    if constexpr (CONVERT) {
        c[0] = (double)(float)p3[0]; c[1] = (double)(float)p3[1]; c[2] = (double)(float)p3[2];
    } else {
        c[0] = n > 0 ? (double)a.X[p0] : 0.0; c[1] = n > 0 ? (double)a.Y[p0] : 0.0; c[2] = n > 0 ? (double)a.Z[p0] : 0.0;
    }
    float lo[5], hi[5];
    const MxPixel mk = mx_pixel(a, 0);
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
    for (int j = bid * 256 + threadIdx.x; j < n; j += nblk * 256) {
        const int64_t i = p0 + j;
        float v[5];
        if constexpr (CONVERT) {
            v[0] = (float)p3[3 * i]; v[1] = (float)p3[3 * i + 1]; v[2] = (float)p3[3 * i + 2];
            v[3] = (float)p2[2 * i]; v[4] = (float)p2[2 * i + 1];
            X[i] = v[0]; Y[i] = v[1]; Z[i] = v[2]; U[i] = v[3]; V[i] = v[4];
        } else {
            v[0] = a.X[i]; v[1] = a.Y[i]; v[2] = a.Z[i]; v[3] = a.U[i]; v[4] = a.V[i];
        }
        const float xc = (float)((double)v[0] - c[0]), yc = (float)((double)v[1] - c[1]),
                    zc = (float)((double)v[2] - c[2]);
        if (XC) {  // (no caller keeps them from r06: sc_unit centres X, Y, Z itself)
            XC[i] = xc;
            YC[i] = yc;
            ZC[i] = zc;
        }
        if (a.PF) mx_point(a, i, xc, yc, zc, v[3], v[4], mk);
#pragma unroll
        for (int k = 0; k < 5; ++k) { lo[k] = fminf(lo[k], v[k]); hi[k] = fmaxf(hi[k], v[k]); }
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        const float l = fminf(fminf(sl[0][k], sl[1][k]), fminf(sl[2][k], sl[3][k]));
        const float h = fmaxf(fmaxf(sh[0][k], sh[1][k]), fmaxf(sh[2][k], sh[3][k]));
        __hip_atomic_store(part + 10 * bid + k, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(part + 10 * bid + 5 + k, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains (sc1 stores)
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1) == nblk - 1;
    __syncthreads();
    if (!last) return;
    // the last block: every block's bounds are in (sc1 stores drained before each ticket add);
    // thread b loads block b's (all in flight at once), then min / max across the block
    __shared__ int wsl[10];
#pragma unroll
    for (int k = 0; k < 5; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
    if ((int)threadIdx.x < nblk)
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            lo[k] = __hip_atomic_load(part + 10 * threadIdx.x + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            hi[k] = __hip_atomic_load(part + 10 * threadIdx.x + 5 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
#pragma unroll
    for (int k = 0; k < 5; ++k)
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    __syncthreads();  // sl / sh are rewritten
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < 5; ++k) { sl[wave][k] = lo[k]; sh[wave][k] = hi[k]; }
    __syncthreads();
    if (threadIdx.x < 5) {
        const int k = threadIdx.x;
        const float l = fminf(fminf(sl[0][k], sl[1][k]), fminf(sl[2][k], sl[3][k]));
        const float h = fmaxf(fmaxf(sh[0][k], sh[1][k]), fmaxf(sh[2][k], sh[3][k]));
        const int wl = n > 0 ? min(0x7F7F7F7F, f2ord(l)) : 0x7F7F7F7F;
        const int wh = n > 0 ? max((int)0x80808080, f2ord(h)) : (int)0x80808080;
        ws[k] = wl;
        ws[5 + k] = wh;
        wsl[k] = wl;
        wsl[5 + k] = wh;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        pnp_frame_one(a, 1, 0, wsl, frame, fconst, c);
        if (a.best_key) *a.best_key = 0ull;
        reset_pnp_queue(a.queue);
        *ticket = 0;  // for the next call (stream order)
    }
}
template <bool CONVERT>
__global__ __launch_bounds__(256) void k_pnp_setup_fc(const double *__restrict__ p3, const double *__restrict__ p2,
                                                      PnpArgs a, float *__restrict__ X, float *__restrict__ Y,
                                                      float *__restrict__ Z, float *__restrict__ U,
                                                      float *__restrict__ V, int *__restrict__ ws,
                                                      double *__restrict__ frame, float *__restrict__ fconst,
                                                      float *__restrict__ XC, float *__restrict__ YC,
                                                      float *__restrict__ ZC, float *part, int *ticket) {
    setup_fc_body<CONVERT>(p3, p2, a, X, Y, Z, U, V, ws, frame, fconst, XC, YC, ZC, part, ticket, (int)blockIdx.x,
                           (int)gridDim.x);
}

// f32 record of one pose for the pre-filter, in the form the scoring launch reads (PnpArgs::fform):
// 2 = the MFMA record of k_pnp_score_mf (write_fmodel_mx) when the problem's centred coordinates
// fit the f16 operands (fconst[11] != 0), else 1 = the scaled record of k_pnp_score_sc
// (write_fmodel_sc; also every small round, round_args)
__device__ __forceinline__ void write_fmodel_sc(const double *R, const double *t, bool valid, const double *frame,
                                                const double *cam, const float *fconst, float *fm);

__device__ __forceinline__ void write_fmodel_mx(const double *R, const double *t, bool valid, const double *frame,
                                                const double *cam, const float *fconst, float *fm);

__device__ __forceinline__ void write_fmodel(const double *R, const double *t, bool valid, const double *frame,
                                             const double *cam, const float *fconst, float *fm, int form) {
    if (form == 2 && fconst[11] != 0.f)
        write_fmodel_mx(R, t, valid, frame, cam, fconst, fm);
    else
        write_fmodel_sc(R, t, valid, frame, cam, fconst, fm);
}

// Scaled record (k_pnp_score_sc, DESIGN.md "Scoring: scaled form").  The z row is multiplied
// by s = sqrt(T) and the kernel's pixel offsets by 1/s (u' = (u - cx) / s), so that
//   q1 = u' z' + xs,  q2 = v' z' + ys,  D = q1^2 + q2^2 - z'^2   (z' = s z)
// has the sign of e - T with no T z^2 term, and the band is linear in |z'|: a pair is decided
// when |D| - a |z'| > b.  Bound (zeta = z' / s, the computed depth in z units): the f32 kernel's
//   Mz = (2.002 s |zeta| + Dz) Dz + Trel' zeta^2,  Dz = D0 + C' |zeta|,
// with C' = 2 Cmax (u' carries three roundings instead of one) and Trel' = Trel + 1e-6 T (the
// rounding of D itself), and zeta^2 <= Zeta |zeta| for |zeta| <= Zeta = (r1 B + |t'z|) + ez, the
// largest depth of any point of the problem.  b also covers the depth guard (b >= K and
// b >= T zg^2: an inlier verdict implies |zeta| > zg; for |zeta| <= zg an outlier verdict
// implies |q| > sqrt(T) |z|), as band_consts does for beta.
//   { -fx R0 -fx R1 -fx R2 | -fy R3 -fy R4 -fy R5 | s R6 s R7 s R8 | -fx t'x -fy t'y s t'z | a b zg 0 }
// b = +inf (every pair recounted exactly) when T or the coordinate magnitudes leave the range
// where the f32 evaluation cannot overflow.
__device__ __forceinline__ void write_fmodel_sc(const double *R, const double *t, bool valid, const double *frame,
                                                const double *cam, const float *fconst, float *fm) {
    if (!valid) {  // already the kernel's decided-outlier form: z' = 0, xs = 1 (D = 1), b = -inf
#pragma unroll
        for (int q = 0; q < kFModelStride; ++q) fm[q] = 0.f;
        fm[9] = 1.f;
        fm[13] = -__builtin_inff();
        fm[14] = -1.f;
        fm[15] = -__builtin_inff();
        return;
    }
    const double B = frame[3], rho = frame[4], cmax = frame[5], wmax = frame[6];
    const double fx = fabs(cam[0]), fy = fabs(cam[1]);
    const double T = fconst[4];
    const bool t_ok = T > 1e-12 && T < 1e30;
    const double s = t_ok ? sqrt(T) : 1.0;
    const double sc[3] = {-cam[0], -cam[1], s};
    double eps[3], mag[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double tp = R[3 * r] * frame[0] + R[3 * r + 1] * frame[1] + R[3 * r + 2] * frame[2] + t[r];
        const double r1 = fabs(R[3 * r]) + fabs(R[3 * r + 1]) + fabs(R[3 * r + 2]);
        eps[r] = 8.0 * kU32 * (r1 * B + fabs(tp)) + r1 * rho + 4e-15 * (r1 * cmax + fabs(t[r]));
        mag[r] = r1 * B + fabs(tp);  // bound on |camera-frame coordinate r| over the problem
#pragma unroll
        for (int q = 0; q < 3; ++q) fm[3 * r + q] = (float)(sc[r] * R[3 * r + q]);
        fm[9 + r] = (float)(sc[r] * tp);
    }
    const double D0 = 1.01 * (fx * eps[0] + fy * eps[1] + eps[2] * (fx + fy) * wmax);
    const double zg = 100.0 * (fmax(eps[0], eps[1]) + wmax * eps[2]) + 2.02 * eps[2] + 1e-30;
    const double Cp = 2.0 * (double)fconst[7], Trelp = (double)fconst[6] + 1e-6 * T;
    const double c1 = Cp / s;                     // Dz = D0 + c1 |z'|
    const double Zp = s * (mag[2] + eps[2]) * (1.0 + 1e-6);  // >= |z'| of every point
    double a = 1.01 * (D0 * (2.002 + 2.0 * c1) + (c1 * (2.002 + c1) + Trelp / T) * Zp);
    double b = 1.01 * D0 * D0;
    const double zr = zg + eps[2];
    const double Kq = D0 + Cp * zr + sqrt(T * 1.00001) * zr;
    b = fmax(b, (1.0 + 1e-6) * Kq * Kq);
    b = fmax(b, T * zg * zg * (1.0 + 1e-5));
    // q, z' and D stay far below the f32 range: |q| <= fx|x| + fy|y| + |u - cx| |z| (+ the band)
    const double umax = (double)fconst[7] / (2.5 * kU32);  // >= |u - cx| + |v - cy| (pnp_frame_one)
    const double qmax = fx * mag[0] + fy * mag[1] + umax * (mag[2] + eps[2]) + D0;
    const bool fits = t_ok && qmax < 1e17 && Zp < 1e17 && a * Zp < 1e30 && b < 1e30;
    if (!fits) {
        // every pair undecided (b = +inf) and recounted exactly; the rows are zeroed so D = 0 and
        // t = 0 stay finite for every pair, pads included (rows past the f32 range would make D a
        // NaN whose sign bit the fast count reads: r06, an EPnP pose with |t| ~ 1e37)
#pragma unroll
        for (int q = 0; q < 12; ++q) fm[q] = 0.f;
    }
    fm[12] = fits ? (float)a : 0.f;
    fm[13] = fits ? (float)b : __builtin_inff();
    fm[14] = (float)zg;
    fm[15] = fits ? (float)((b + a * Zp) * (1.0 + 1e-6)) : __builtin_inff();  // constant band b + a Zmax
}

// The band constants of the scaled form (write_fmodel_sc's formulas) from the camera-frame
// evaluation error bounds eps (rows x y z) and the row magnitudes mag: {a, b, zg, b + a Zp}; fits =
// false when a quantity of the test could leave the f32 range (then b = +inf: every pair recounted
// exactly)
struct ScBand {
    double a, b, zg, bcb, Zp, qmax;
};
// for write_fmodel_mx, with the frame's per-problem terms (pnp_frame_mx_consts: s, 2 Cmax / s,
// Trel' / T, sqrt(1.00001 T), umax, computed once per problem)
__device__ __forceinline__ ScBand sc_band_h(const double (&eps)[3], const double (&mag)[3], double fx, double fy,
                                            double wmax, double T, const double *frame, const float *fconst) {
    ScBand r;
    const double s = frame[8], c1 = frame[9], Trel_T = frame[10], sqT = frame[11], umax = frame[12];
    const double D0 = 1.01 * (fx * eps[0] + fy * eps[1] + eps[2] * (fx + fy) * wmax);
    r.zg = 100.0 * (fmax(eps[0], eps[1]) + wmax * eps[2]) + 2.02 * eps[2] + 1e-30;
    const double Cp = 2.0 * (double)fconst[7];
    r.Zp = s * (mag[2] + eps[2]) * (1.0 + 1e-6);
    r.a = 1.01 * (D0 * (2.002 + 2.0 * c1) + (c1 * (2.002 + c1) + Trel_T) * r.Zp);
    r.b = 1.01 * D0 * D0;
    const double zr = r.zg + eps[2];
    const double Kq = D0 + Cp * zr + sqT * zr;
    r.b = fmax(r.b, (1.0 + 1e-6) * Kq * Kq);
    r.b = fmax(r.b, T * r.zg * r.zg * (1.0 + 1e-5));
    r.qmax = fx * mag[0] + fy * mag[1] + umax * (mag[2] + eps[2]) + D0;
    r.bcb = (r.b + r.a * r.Zp) * (1.0 + 1e-6);
    return r;
}

// MFMA record (k_pnp_score_mf, DESIGN.md "Scoring: MFMA form").  The three rows of the scaled
// form, (xs, ys, z') = sc_r (R_r . XC + t'_r) with sc = (-fx, -fy, sqrt(T)), are the A operands of
// v_mfma_f32_32x32x16_f16: per row the coefficients of XC, YC, ZC and of the constant feature
// (sc_r t'_r), all of one hypothesis scaled by lambda = 2^k so that the largest lies in
// (2^14, 2^15], split into f16 hi = RN(A) and lo = RN(A - hi) (stored x 2^11).  The kernel forms
// sum_k (hi_k + lo_k)(Bhi_k + Blo_k) with the point operands of mx_point; the test then runs on
// lambda-scaled quantities, exactly as on the unscaled ones (powers of 2), with a' = lambda a and
// b' = lambda^2 b.  Error of one row's output (lambda units), per feature k:
//   |dA_k| |B~_k| + |A_k| |dB_k|   (dA_k: this hypothesis' exact split error, plus the f16
//                                   subnormal operands in case the matrix core flushes them; lo
//                                   is stored x 2^11 and faces B x 2^-11 (mx_point), so it is
//                                   normal unless |A_k| < 2^-14; dB_k <= 2^-21 |B_k| + 2^-13 with
//                                   the same allowance for both copies of B)
//   + 2^-20 sum_k |A~_k| |B~_k|     (16 exact f32 products summed in round-to-nearest f32 in
//                                   any order: gamma_15 < 16u)
// in camera units eps_r = that / (lambda |sc_r|) + the centring and f64 terms of write_fmodel_sc,
// about 3x its 8u (r1 B + |t'|).  Layout: f16 hi rows 0..2 (4 each: XC YC ZC 1) | f16 lo x 2^11
// rows | f32 { a', b', zg, b'_cb }.
__device__ __forceinline__ void write_fmodel_mx(const double *R, const double *t, bool valid, const double *frame,
                                                const double *cam, const float *fconst, float *fm) {
    _Float16 *hm = reinterpret_cast<_Float16 *>(fm);
    if (!valid) {  // the kernel's decided-outlier form: xs = 1 (D = 1), b' = -inf
#pragma unroll
        for (int q = 0; q < kFModelStride; ++q) fm[q] = 0.f;
        hm[3] = (_Float16)1.0f;
        fm[13] = -__builtin_inff();
        fm[14] = -1.f;
        fm[15] = -__builtin_inff();
        return;
    }
    const double B = frame[3], rho = frame[4], cmax = frame[5], wmax = frame[6];
    const double fx = fabs(cam[0]), fy = fabs(cam[1]);
    const double T = fconst[4];
    const bool t_ok = T > 1e-12 && T < 1e30;
    const double s = frame[8];  // sqrt(T), 1 when T is out of range (pnp_frame_mx_consts)
    const double sc[3] = {-cam[0], -cam[1], s};
    double A[3][4], r1[3], mag[3], tp[3];
    double M = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        tp[r] = R[3 * r] * frame[0] + R[3 * r + 1] * frame[1] + R[3 * r + 2] * frame[2] + t[r];
        r1[r] = fabs(R[3 * r]) + fabs(R[3 * r + 1]) + fabs(R[3 * r + 2]);
        mag[r] = r1[r] * B + fabs(tp[r]);
#pragma unroll
        for (int k = 0; k < 3; ++k) A[r][k] = sc[r] * R[3 * r + k];
        A[r][3] = sc[r] * tp[r];
#pragma unroll
        for (int k = 0; k < 4; ++k) M = fmax(M, fabs(A[r][k]));
    }
    int e = 0;
    (void)frexp(M, &e);  // M = m 2^e, m in [0.5, 1)
    const int kx = min(120, max(-120, 15 - e));
    const double lam = ldexp(1.0, kx);
    const double Bs = B * (1.0 + 0x1p-20) + 0x1p-14;  // >= |B~_k| of every point (k < 3)
    double eps[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double dA = 0.0, SA = 0.0, AB = 0.0;  // sum dA_k Bmax_k, sum_{k<3} |A_k|, sum |A_k| Bmax_k
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double v = A[r][k] * lam;
            const _Float16 hi = (_Float16)(float)v;
            const _Float16 lo = (_Float16)(float)((v - (double)hi) * 0x1p11);  // lo x 2^11: normal unless v is tiny
            hm[4 * r + k] = hi;
            hm[12 + 4 * r + k] = lo;
            const double h = (double)hi, l = (double)lo * 0x1p-11;
            double d = fabs(v - h - l);
            if (fabs(h) < 0x1p-14) d += fabs(h);  // subnormal operands: allow for a flush to zero
            if (fabs((double)lo) < 0x1p-14) d += fabs(l);
            const double bm = k < 3 ? Bs : 1.0;
            dA += d * bm;
            AB += fabs(v) * bm;
            if (k < 3) SA += fabs(v);
        }
        // A side + B side (2^-21 relative on XC YC ZC, 2^-13 absolute) + the accumulation (16u: 16
        // exact products summed in round-to-nearest f32, any order)
        const double err = 1.001 * (dA + 0x1p-21 * AB + 0x1p-13 * SA + 0x1p-20 * (AB + dA + 0x1p-13 * SA + 1.0));
        // err / (lam |sc_r|), rounded up: the frame's upward reciprocal of |sc_r| and the exact 2^-kx
        eps[r] = ldexp(err * frame[13 + r], -kx) + r1[r] * rho + 4e-15 * (r1[r] * cmax + fabs(t[r]));
    }
    ScBand bd = sc_band_h(eps, mag, fx, fy, wmax, T, frame, fconst);
    const double ap = bd.a * lam, bp = bd.b * lam * lam, cbp = bd.bcb * lam * lam;
    // M lam <= 2^15: the scale was not clamped (|t| past ~1e36 would put f16 infinities in the
    // operands, and the fast count would read a NaN's sign bit: r06, a degenerate EPnP pose)
    const bool fits = t_ok && M > 0.0 && M * lam <= 0x1p15 && bd.qmax * lam < 1e17 && bd.Zp * lam < 1e17 &&
                      ap * bd.Zp * lam < 1e30 && bp < 1e30 && cbp < 1e30 && bp > 1e-30;
    if (!fits) {  // every pair undecided and recounted exactly; zero operands keep D = t = 0 finite
#pragma unroll
        for (int q = 0; q < 24; ++q) hm[q] = (_Float16)0.0f;
    }
    fm[12] = fits ? (float)ap : 0.f;
    fm[13] = fits ? (float)bp : __builtin_inff();
    fm[14] = (float)bd.zg;
    fm[15] = fits ? (float)cbp : __builtin_inff();
}

__global__ void k_pnp_fmodels(PnpArgs a, int32_t H) {
    const int prob = blockIdx.y;
    const int h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h == 0 && prob == 0 && a.queue) reset_pnp_queue(a.queue);  // the scoring launch that follows starts at 0
    if (h >= H) return;
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    const double *m = a.models + rec * kModelStride;
    write_fmodel(m, m + 9, a.status[rec] > 0, a.frame + (int64_t)prob * kFrameStride, a.cams + 4 * prob,
                 a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);
}

// ---------------------------------------------------------------------------
// PnP: sample + minimal solve, one lane per hypothesis
// ---------------------------------------------------------------------------
// 124 VGPRs, 4 waves/SIMD (r04: the best candidate held as its refined lambdas); asking for 5 waves
// spills (scripts/ubench/probes_r04.patch keeps the knob)
__global__ __launch_bounds__(256) void k_pnp_solve(PnpArgs a, int64_t hyp_begin, int32_t H) {
    const int prob = blockIdx.y;
    const int hl = blockIdx.x * blockDim.x + threadIdx.x;
    // every round's scoring launch follows a solve on the same stream: reset its work queue here
    if (hl == 0 && prob == 0) {
        if (a.queue) reset_pnp_queue(a.queue);
    }
    if (hl >= H) return;
    const int64_t h = hyp_begin + hl;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    double *m = a.models + rec * kModelStride;
    int32_t idx[4];
    int8_t st = 1;
    if (a.subsets) {
        st = a.sub_status[rec];
#pragma unroll
        for (int j = 0; j < 4; ++j) idx[j] = a.subsets[rec * 4 + j];
    } else {
        Philox rng;
        rng.init(a.seed, 0u, (uint64_t)(a.rng_base + h));
        st = (n >= 4 && rng.subset<4>(n, idx) == 0) ? 1 : -1;
    }
    double R[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t[3] = {0, 0, 0};
    if (st > 0) {
        float X[4], Y[4], Z[4], U[4], V[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t i = p0 + idx[j];
            X[j] = a.X[i]; Y[j] = a.Y[i]; Z[j] = a.Z[i]; U[j] = a.U[i]; V[j] = a.V[i];
        }
        const double *c = a.cams + 4 * prob;
        Cam k{c[0], c[1], c[2], c[3]};
        // (a per-point table of bearings written by the setup measured no faster: the solve then
        // waits on three gathers per sample instead of computing them, r04)
        double yb[9];
#pragma unroll
        for (int j = 0; j < 3; ++j) bearing(k, U[j], V[j], yb + 3 * j);
        st = pnp_minimal_lam(X, Y, Z, U, V, k, yb, R, t) ? 1 : 0;
        if (st > 0 && a.rvec_rt) rodrigues_roundtrip(R);
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = R[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];
    a.status[rec] = st;  // the record's validity (kValidSlot is left unwritten)
    if (a.counts_out) a.counts_out[rec] = 0;  // the scoring launch that follows may accumulate
    if (a.fmodels)
        write_fmodel(R, t, st > 0, a.frame + (int64_t)prob * kFrameStride, a.cams + 4 * prob,
                     a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);
}

// The default minimal solver of solvePnPRansac (SOLVEPNP_ITERATIVE: 5-point samples, each solved
// by solvePnP(SOLVEPNP_EPNP); [OpenCV 4.x, unvendored] solvepnp.cpp PnPRansacCallback::runKernel)
// in OpenCV's own operation sequence (rsac_cvepnp.h, the oracle's oracle/cv_epnp.c), three
// launches:
//   k_cvepnp5_a    one lane per hypothesis: the sample, undistortPoints' f32 normalised points,
//                  the control points (cvSVD of PW0^T PW0), the barycentric alphas (cvInvert),
//                  fill_M + cvMulTransposed: M^T M's upper triangle, alphas and control points
//                  into the launch-local scratch;
//   k_cvepnp5_svd  six lanes per hypothesis, ten per wave: cvSVD(M^T M)'s JacobiSVDImpl_ -- the
//                  cyclic pair order run by anti-diagonals (each row sees the sequential loop's
//                  operations), lane m making pair m of each diagonal on rows kept in LDS, every
//                  sum over k = 0..11 left to right in one lane; then the row norms, the selection
//                  sort and the normalisation of the four smallest rows (a zero row's random fill
//                  in memory, cvq_fill_rows);
//   k_cvepnp5_c    three lanes per hypothesis, one beta estimate each (find_betas_approx_1..3 +
//                  gauss_newton + compute_R_and_t), epnp::compute_pose's pick, the Rodrigues
//                  round trip of the (rvec, tvec) model, the records.
// Per hypothesis a.epnp holds kEpnpRec doubles at the launch-local position prob * H + hl:
// [0, 78) M^T M's upper triangle (stage 1) / [0, 144) the 12 rows and [144, 156) their norms
// (the rare fill path) / [0, 48) the sorted rows 8 .. 11, normalised (stage 2); [156, 176) the
// alphas and [176, 188) the control points (stage 1).
constexpr int kCvRows = 0, kCvW = 144, kCvAlpha = 156, kCvCws = 176;
static_assert(kCvCws + 12 <= kEpnpRec, "cv EPnP scratch");

// the sample of hypothesis rec (OpenCV subsets or Philox), status 1 drawn / -1 not
__device__ __forceinline__ int8_t epnp5_sample(const PnpArgs &a, int64_t rec, int64_t h, int n, int32_t (&idx)[5]) {
    if (a.subsets) {
#pragma unroll
        for (int j = 0; j < 5; ++j) idx[j] = a.subsets[rec * 5 + j];
        return a.sub_status[rec];
    }
    Philox rng;
    rng.init(a.seed, 0u, (uint64_t)(a.rng_base + h));
    return (n >= 5 && rng.subset<5>(n, idx) == 0) ? 1 : -1;
}
// the sample's points (solvePnPRansac's CV_32F copies)
struct Epnp5Pts {
    float X[5], Y[5], Z[5], U[5], V[5];
};
__device__ __forceinline__ void epnp5_gather(const PnpArgs &a, int64_t p0, const int32_t (&idx)[5], Epnp5Pts &q) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const int64_t i = p0 + idx[j];
        q.X[j] = a.X[i]; q.Y[j] = a.Y[i]; q.Z[j] = a.Z[i]; q.U[j] = a.U[i]; q.V[j] = a.V[i];
    }
}

// 1 of 3: sample, epnp's set-up through M^T M
__global__ __launch_bounds__(256) void k_cvepnp5_a(PnpArgs a, int64_t hyp_begin, int32_t H) {
    const int prob = blockIdx.y;
    const int hl = blockIdx.x * blockDim.x + threadIdx.x;
    if (hl == 0 && prob == 0) {
        if (a.queue) reset_pnp_queue(a.queue);
    }
    if (hl >= H) return;
    const int64_t h = hyp_begin + hl;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    int32_t idx[5];
    const int8_t st = epnp5_sample(a, rec, h, n, idx);
    if (st > 0) {
        Epnp5Pts q;
        epnp5_gather(a, p0, idx, q);
        const double *cm = a.cams + 4 * prob;
        cvq::Epnp5 e;
        cvq::epnp5_init(q.X, q.Y, q.Z, q.U, q.V, Cam{cm[0], cm[1], cm[2], cm[3]}, e);
        cvq::epnp5_frame(e);
        double *E = a.epnp + ((int64_t)prob * H + hl) * kEpnpRec;
        cvq::epnp5_mtm(e, E);
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) E[kCvAlpha + 4 * i + j] = e.alphas[i][j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) E[kCvCws + 3 * i + j] = e.cws[i][j];
    }
    a.status[rec] = st;
}

// 2 of 3: the 12 x 12 JacobiSVD, six lanes per hypothesis
// JacobiSVDImpl_'s tail in memory (one lane, the rare case of a row norm <= DBL_MIN): the selection
// sort of the 12 rows by their norms and the normalisation of every row, a zero one replaced by
// RNG(0x12345678)'s random direction projected off the earlier rows (rsac_cvepnp.h jacobi_svd);
// rows 8 .. 11 end at [0, 48)
__device__ __attribute__((noinline)) void cvq_fill_rows(double *E) {
    double *A = E + kCvRows, *W = E + kCvW;
    for (int i = 0; i < 11; ++i) {
        int j = i;
        for (int k = i + 1; k < 12; ++k)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < 12; ++k) { t = A[12 * i + k]; A[12 * i + k] = A[12 * j + k]; A[12 * j + k] = t; }
        }
    }
    uint64_t rng = 0x12345678;
    for (int i = 0; i < 12; ++i) {
        double sd = W[i];
        for (int ii = 0; ii < 100 && sd <= cvq::kDblMin; ii++) {
            const double val0 = 1. / 12;
            for (int k = 0; k < 12; ++k) A[12 * i + k] = (cvq::rng_next(rng) & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
                for (int j = 0; j < i; ++j) {
                    sd = 0;
                    for (int k = 0; k < 12; ++k) sd += A[12 * i + k] * A[12 * j + k];
                    double asum = 0;
                    for (int k = 0; k < 12; ++k) {
                        const double t = A[12 * i + k] - sd * A[12 * j + k];
                        A[12 * i + k] = t;
                        asum += dabs(t);
                    }
                    asum = asum > cvq::kSvdEps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < 12; ++k) A[12 * i + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < 12; ++k) sd += A[12 * i + k] * A[12 * i + k];
            sd = dsqrt(sd);
        }
        const double s = sd > cvq::kDblMin ? 1 / sd : 0.;
        for (int k = 0; k < 12; ++k) A[12 * i + k] *= s;
    }
    for (int k = 0; k < 48; ++k) E[k] = A[96 + k];
}

// JacobiSVDImpl_'s cyclic pair order (i < j, i outer) run by anti-diagonals: rotation (i, j) reads
// rows i and j as the last earlier rotation touching each left them, so the pairs of one
// anti-diagonal i + j = t (disjoint rows) are independent, and running t = 1 .. 21 in turn gives every
// row the sequential loop's operations in its order.  Lane m of a hypothesis's six owns pair
// i = max(0, t - 11) + m of diagonal t (at most six pairs): it reads rows i, j and their norms from
// the hypothesis's LDS copy of the matrix, makes OpenCV's whole rotation on them alone (every sum
// over k = 0..11 left to right in one lane), and writes them back.  The six lanes are one wave's:
// its LDS operations execute in order, so a diagonal reads what the last one wrote without a barrier
// (lds_wave_order keeps the compiler from moving them).  A sweep is 21 dependent steps of one
// rotation per lane, where the quad layout (r06 first cut) ran all 66 on every lane.  A hypothesis
// whose sweep changed nothing stays as it is in further sweeps (every pair skips again), so the wave
// sweeps until none of its hypotheses changed (at most OpenCV's 30).
constexpr int kSvdHpw = 10;      // hypotheses per wave (60 of 64 lanes)
constexpr int kSvdStride = 158;  // LDS doubles per hypothesis: rows [12][12], norms [12], 16-B pad
__device__ __forceinline__ void lds_wave_order() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void cvsvd_load_row(const double *S, int r, double (&x)[12]) {
    const double2 *v = (const double2 *)(S + 12 * r);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double2 w = v[k];
        x[2 * k] = w.x;
        x[2 * k + 1] = w.y;
    }
}
__device__ __forceinline__ void cvsvd_store_row(double *S, int r, const double (&x)[12]) {
    double2 *v = (double2 *)(S + 12 * r);
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = make_double2(x[2 * k], x[2 * k + 1]);
}

__global__ __launch_bounds__(256) void k_cvepnp5_svd(PnpArgs a, int64_t hyp_begin, int32_t H) {
    extern __shared__ __attribute__((aligned(16))) double svd_lds[];  // [waves][kSvdHpw][kSvdStride]
    const int prob = blockIdx.y;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / 6, m = lane - 6 * g;
    const int hl = (blockIdx.x * (int)(blockDim.x >> 6) + wave) * kSvdHpw + g;
    if (g >= kSvdHpw || hl >= H) return;  // six-lane-uniform from here on
    const int64_t rec = (int64_t)prob * a.hyp_stride + hyp_begin + hl;
    if (a.status[rec] <= 0) return;
    double *E = a.epnp + ((int64_t)prob * H + hl) * kEpnpRec;
    double *S = svd_lds + (wave * kSvdHpw + g) * kSvdStride;  // row r at S[12 r], norms at S[144]
    // At = (M^T M)^T = M^T M from the upper triangle: lane m fills rows 2m, 2m + 1 (JacobiSVDImpl_'s
    // initial W, their squared norms, is formed from the rows where it is used, below)
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int r = 2 * m + rr;
        double x[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) {
            const int lo = r < c ? r : c, hi = r < c ? c : r;
            x[c] = E[lo * 12 - lo * (lo - 1) / 2 + (hi - lo)];
        }
        cvsvd_store_row(S, r, x);
    }
    lds_wave_order();
    // JacobiSVDImpl_'s W[i] is always sum_k At[i][k]^2 of the stored row, in k order: the initial
    // norms are that sum, and a rotation sets W[i] = sum_k t0_k t0_k of exactly the t0_k it stores
    // as the row (a skip changes neither).  So a step forms both norms from the rows it loads,
    // beside their dot product -- three independent 12-term chains -- and no W is kept in LDS
    // (r06: the norm store and reload, ~150 cycles of a step's critical path, are gone).  The sums
    // start at their first product, not at 0 + it: a norm's products are >= +0, so 0 + x == x; p
    // differs from 0 + ... only in the sign of an all-zero sum, which the skip test treats alike
    // (|p| = 0), and a NaN norm makes the rotation NaN either way.  A step is branch-free up to the
    // skip test (an idle lane reads rows 0 and 1 and discards the result).
    for (int iter = 0; iter < 30; ++iter) {
        bool changed = false;
        for (int t = 1; t <= 21; ++t) {
            const int i = (t > 11 ? t - 11 : 0) + m, j = t - i;
            const bool act = i < j;
            const int li = act ? i : 0, lj = act ? j : 1;
            double Ai[12], Aj[12];
            cvsvd_load_row(S, li, Ai);
            cvsvd_load_row(S, lj, Aj);
            double wa = Ai[0] * Ai[0], wb = Aj[0] * Aj[0], p = Ai[0] * Aj[0];
#pragma unroll
            for (int k = 1; k < 12; ++k) {
                wa += Ai[k] * Ai[k];
                wb += Aj[k] * Aj[k];
                p += Ai[k] * Aj[k];
            }
            // the skip test's root by the fast core when both norms lie in the rotation's fast range
            // (their product in [2^-400, 2^400]); p and the core are formed before the branch for
            // the other lanes, so the scheduler still interleaves them
            const double ab = wa * wb;
            const bool in = (wa >= 0x1p-200) & (wa <= 0x1p+200) & (wb >= 0x1p-200) & (wb <= 0x1p+200);
            double sab = dsqrt_fast(ab);
            asm volatile("" ::"v"(p), "v"(sab));
            if (!in) {
                asm volatile("" ::: "memory");
                sab = dsqrt(ab);
            }
            if (act && !(dabs(p) <= cvq::kSvdEps * sab)) {
                double c, s, Pi[12], Pj[12];
                cvq::svd_rotation_sel(p * 2, wa, wb, c, s);
#pragma unroll
                for (int k = 0; k < 12; ++k) {
                    Pi[k] = c * Ai[k] + s * Aj[k];
                    Pj[k] = -s * Ai[k] + c * Aj[k];
                }
                cvsvd_store_row(S, i, Pi);
                cvsvd_store_row(S, j, Pj);
                changed = true;
            }
            lds_wave_order();
        }
        if (!__any(changed)) break;
    }
    // the row norms, the selection sort (descending, first maximum), the normalisation
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int r = 2 * m + rr;
        double x[12], sd = 0;
        cvsvd_load_row(S, r, x);
#pragma unroll
        for (int k = 0; k < 12; ++k) sd += x[k] * x[k];
        S[144 + r] = dsqrt(sd);
    }
    lds_wave_order();
    double W[12];
    int perm[12];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        W[r] = S[144 + r];
        perm[r] = r;
    }
#pragma unroll
    for (int i = 0; i < 11; ++i) {
        int j = i;
#pragma unroll
        for (int k = i + 1; k < 12; ++k)
            if (W[j] < W[k]) j = k;
#pragma unroll
        for (int k = i + 1; k < 12; ++k)
            if (k == j) {
                const double tw = W[i]; W[i] = W[k]; W[k] = tw;
                const int tp = perm[i]; perm[i] = perm[k]; perm[k] = tp;
            }
    }
    if (W[11] > cvq::kDblMin) {
        // rows 8 .. 11 (every row's norm > DBL_MIN: no random fill anywhere), times 1 / norm: lane
        // m < 4 writes row 8 + m
        if (m < 4) {
            int r = 0;
            double w = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (q == m) {
                    r = perm[8 + q];
                    w = W[8 + q];
                }
            const double inv = 1 / w;
            double x[12];
            cvsvd_load_row(S, r, x);
#pragma unroll
            for (int k = 0; k < 12; ++k) E[m * 12 + k] = x[k] * inv;
        }
        return;
    }
    // a row of zero norm: lane 0 puts the rows and their (unsorted) norms in memory and finishes there
    if (m == 0) {
        for (int r = 0; r < 12; ++r) {
            for (int k = 0; k < 12; ++k) E[kCvRows + 12 * r + k] = S[12 * r + k];
            E[kCvW + r] = S[144 + r];
        }
        cvq_fill_rows(E);
    }
}

// 3 of 3: lane c of a group of three takes estimate c + 1, then epnp::compute_pose's pick,
// Rodrigues(Rodrigues(R)) (the (rvec, tvec) model computeError projects), the records
__global__ __launch_bounds__(256) void k_cvepnp5_c(PnpArgs a, int64_t hyp_begin, int32_t H, int hpw) {
#ifdef RSAC_TRACE
    const unsigned long long tk0 = __builtin_amdgcn_s_memtime();
#endif
    const int prob = blockIdx.y;
    const int lane = threadIdx.x & 63, g = lane / 3, c = lane - 3 * g;
    const int hl = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * hpw + g;
    const bool live = g < hpw && hl < H;
    const int64_t h = hyp_begin + hl;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    const double *E = a.epnp + ((int64_t)prob * H + hl) * kEpnpRec;
    int8_t st = live ? a.status[rec] : -1;
    double R[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t[3] = {0, 0, 0}, err = 0.0;
    if (st > 0) {
        double L[6][10], rho[6], be[4];
        {
            double v[4][12];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int k = 0; k < 12; ++k) v[i][k] = E[(3 - i) * 12 + k];
            cvq::epnp_l6x10(v, L);
            cvq::Epnp5 cw;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) cw.cws[i][j] = E[kCvCws + 3 * i + j];
            cvq::epnp_rho(cw, rho);
        }
#ifdef RSAC_TRACE
        const unsigned long long tc0 = __builtin_amdgcn_s_memtime();
        asm volatile("; trace sink %0" ::"v"(L[5][9] + rho[5]) : "memory");
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tc1 = __builtin_amdgcn_s_memtime();
#endif
        cvq::betas_approx_padded(c + 1, L, rho, be);  // one instruction stream for the three lanes
#ifdef RSAC_TRACE
        asm volatile("; trace sink %0" ::"v"(be[0] + be[3]) : "memory");
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tc2 = __builtin_amdgcn_s_memtime();
#endif
        cvq::gauss_newton(L, rho, be);
#ifdef RSAC_TRACE
        asm volatile("; trace sink %0" ::"v"(be[0] + be[3]) : "memory");
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tc3 = __builtin_amdgcn_s_memtime();
#endif
        int32_t idx[5];
        (void)epnp5_sample(a, rec, h, n, idx);
        Epnp5Pts q;
        epnp5_gather(a, p0, idx, q);
        const double *cm = a.cams + 4 * prob;
        cvq::Epnp5 e;
        cvq::epnp5_init(q.X, q.Y, q.Z, q.U, q.V, Cam{cm[0], cm[1], cm[2], cm[3]}, e);
#pragma unroll
        for (int i = 0; i < 5; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) e.alphas[i][j] = E[kCvAlpha + 4 * i + j];
        double v[4][12];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int k = 0; k < 12; ++k) v[i][k] = E[(3 - i) * 12 + k];
        err = cvq::epnp5_r_and_t(e, v, be, R, t);
#ifdef RSAC_TRACE
        asm volatile("; trace sink %0" ::"v"(err + R[0] + t[2]) : "memory");
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tc4 = __builtin_amdgcn_s_memtime();
        if (hl == 0 && prob == 0)
            printf("epnp c lane %d: setup %llu betas %llu gauss-newton %llu r_and_t %llu cycles (from kernel start %llu)\n",
                   c, tc1 - tc0, tc2 - tc1, tc3 - tc2, tc4 - tc3, tc1 - tk0);
#endif
    }
    // epnp::compute_pose's pick over the group's three lanes (estimates 1, 2, 3)
    const int base = 3 * g;
    const double err3[3] = {__shfl(err, base), __shfl(err, base + 1), __shfl(err, base + 2)};
    const int src = base + cvq::epnp_pick(err3);
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = __shfl(R[k], src);
#pragma unroll
    for (int k = 0; k < 3; ++k) t[k] = __shfl(t[k], src);
    if (!live || c != 0) return;
    // OpenCV's EPnP always reports a pose (a degenerate sample's NaN scores no inlier); the
    // winner's (rvec, tvec) model is Rodrigues(Rodrigues(R)) (on all three lanes before the pick
    // the stage took 85 instead of 78 us, r06)
    if (st > 0) {
        st = 1;
#ifdef RSAC_TRACE
        const unsigned long long tr0 = __builtin_amdgcn_s_memtime();
#endif
        if (a.rvec_rt) rodrigues_roundtrip(R);
#ifdef RSAC_TRACE
        asm volatile("; trace sink %0" ::"v"(R[0] + R[8]) : "memory");
        __builtin_amdgcn_s_waitcnt(0);
        if (hl == 0 && prob == 0)
            printf("epnp c roundtrip %llu cycles, total %llu\n", __builtin_amdgcn_s_memtime() - tr0,
                   __builtin_amdgcn_s_memtime() - tk0);
#endif
    }
    double *m = a.models + rec * kModelStride;
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = R[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];
    a.status[rec] = st;  // the record's validity (kValidSlot is left unwritten)
    if (a.counts_out) a.counts_out[rec] = 0;
    if (a.fmodels)
        write_fmodel(R, t, st > 0, a.frame + (int64_t)prob * kFrameStride, a.cams + 4 * prob,
                     a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);
}

// Small rounds (an adaptive run's first 256 hypotheses: one block, every lane's latency is the
// launch's): four lanes per hypothesis.  All four draw the sample and run lt_common; lane c
// then takes candidate c = (sign, root) of the Lambda Twist solution list (lt_sign, lt_tau:
// the operations of p3p_lambdatwist for that candidate) and its 4th-point error; the four
// lanes pick the smallest error, the lowest candidate on ties (= pnp_minimal's first-one rule),
// and the winner writes the record.  Results equal k_pnp_solve's bit for bit.

// gather(p0, idx, X, Y, Z, U, V): the sample's f32 points
template <int L, class Gather>
__device__ __forceinline__ void solve_l_body(const PnpArgs &a, int64_t hyp_begin, int32_t H, const int prob,
                                             const int gt, Gather gather) {
    constexpr int CPL = 4 / L;  // Lambda Twist candidates per lane: lane c takes c CPL .. c CPL + CPL - 1
    const int hl = gt / L, lc = gt % L;
    if (gt == 0 && prob == 0) {
        if (a.queue) reset_pnp_queue(a.queue);
    }
    const bool live = hl < H;  // the L lanes of a hypothesis share it: shuffles stay in the group
    const int64_t h = hyp_begin + hl;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    int32_t idx[4] = {0, 0, 0, 0};
    int8_t st = -1;
    if (live) {
        if (a.subsets) {
            st = a.sub_status[rec];
#pragma unroll
            for (int j = 0; j < 4; ++j) idx[j] = a.subsets[rec * 4 + j];
        } else {
            Philox rng;
            rng.init(a.seed, 0u, (uint64_t)(a.rng_base + h));
            st = (n >= 4 && rng.subset<4>(n, idx) == 0) ? 1 : -1;
        }
    }
    double R[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t[3] = {0, 0, 0};
    double e = 0.0;
    int mine = 4;  // the lane's first smallest-error candidate (4: none emitted with a usable error)
    const Cam k{a.cams[4 * prob], a.cams[4 * prob + 1], a.cams[4 * prob + 2], a.cams[4 * prob + 3]};
    if (st > 0) {
        float X[4], Y[4], Z[4], U[4], V[4];
        gather(p0, idx, X, Y, Z, U, V);
        double yb[9], xw[9];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            bearing(k, U[j], V[j], yb + 3 * j);
            xw[3 * j] = X[j]; xw[3 * j + 1] = Y[j]; xw[3 * j + 2] = Z[j];
        }
        LtCommon Lc;
        double w0, w1, tau[2];
        if (lt_common(yb, xw, Lc) && lt_sign(Lc, (lc * CPL) >> 1, w0, w1, tau)) {
            for (int r = 0; r < CPL; ++r) {
                const int cand = lc * CPL + r;
                auto emit = [&](const double *Rk, const double *tk) {
                    const double ek = pnp_fourth_error(Rk, tk, X, Y, Z, U, V, k);
                    if (!(ek == ek)) return;
                    if (mine < 4 && !(ek < e)) return;  // the first smallest stays
                    mine = cand;
                    e = ek;
#pragma unroll
                    for (int q = 0; q < 9; ++q) R[q] = Rk[q];
#pragma unroll
                    for (int q = 0; q < 3; ++q) t[q] = tk[q];
                };
                (void)lt_tau(Lc, w0, w1, tau[cand & 1], yb, xw, emit);
            }
        }
    }
    // the group's winner: smallest e, then the lowest candidate (all L lanes agree)
    int win = mine;
    double we = mine < 4 ? e : 0.0;
#pragma unroll
    for (int o = 1; o < L; o <<= 1) {
        const int ow = __shfl_xor(win, o);
        const double oe = __shfl_xor(we, o);
        if (ow < 4 && (win == 4 || oe < we || (oe == we && ow < win))) {
            win = ow;
            we = oe;
        }
    }
    if (!live) return;
    const bool ok = win < 4;
    if (ok ? mine != win : lc != 0) return;  // one writer per hypothesis
    const int8_t sv = st > 0 ? (ok ? 1 : 0) : st;
    double *m = a.models + rec * kModelStride;
    if (sv > 0 && a.rvec_rt) rodrigues_roundtrip(R);
    if (!ok)
        for (int q = 0; q < 9; ++q) R[q] = 0.0;
    if (!ok)
        for (int q = 0; q < 3; ++q) t[q] = 0.0;
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = R[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];
    a.status[rec] = sv;  // the record's validity (kValidSlot is left unwritten)
    if (a.counts_out) a.counts_out[rec] = 0;
    if (a.fmodels)
        write_fmodel(R, t, sv > 0, a.frame + (int64_t)prob * kFrameStride, a.cams + 4 * prob,
                     a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);
}
template <int L>
__global__ __launch_bounds__(256) void k_pnp_solve_l(PnpArgs a, int64_t hyp_begin, int32_t H) {
    solve_l_body<L>(a, hyp_begin, H, (int)blockIdx.y, (int)(blockIdx.x * blockDim.x + threadIdx.x),
                    [&](int64_t p0, const int32_t(&idx)[4], float(&X)[4], float(&Y)[4], float(&Z)[4], float(&U)[4],
                        float(&V)[4]) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int64_t i = p0 + idx[j];
                            X[j] = a.X[i]; Y[j] = a.Y[i]; Z[j] = a.Z[i]; U[j] = a.U[i]; V[j] = a.V[i];
                        }
                    });
}
// One problem's first P3P round fused with its set-up (r06): blocks [0, gs) run k_pnp_setup_fc's
// conversion / bounds / frame / centring pass over the f64 inputs, the others k_pnp_solve_l<4>,
// whose samples read the same f64 inputs and round them as the conversion does.  The frame does
// not exist while the solve runs, so the solve writes no f32 records (a.fmodels = nullptr here)
// and the round's scaled-form scorer builds them from the f64 models (PnpArgs::fm_inline).  One
// launch and one dependent dispatch fewer, and the set-up overlaps the solve.
__global__ __launch_bounds__(256) void k_pnp_setup_solve4(const double *__restrict__ p3, const double *__restrict__ p2,
                                                          PnpArgs a, float *__restrict__ X, float *__restrict__ Y,
                                                          float *__restrict__ Z, float *__restrict__ U,
                                                          float *__restrict__ V, int *__restrict__ ws,
                                                          double *__restrict__ frame, float *__restrict__ fconst,
                                                          float *part, int *ticket, int gs, int64_t hyp_begin,
                                                          int32_t H) {
    if ((int)blockIdx.x < gs) {
        setup_fc_body<true>(p3, p2, a, X, Y, Z, U, V, ws, frame, fconst, nullptr, nullptr, nullptr, part, ticket,
                            (int)blockIdx.x, gs);
        return;
    }
    PnpArgs sa = a;
    sa.fmodels = nullptr;
    solve_l_body<4>(sa, hyp_begin, H, 0, ((int)blockIdx.x - gs) * 256 + (int)threadIdx.x,
                    [&](int64_t p0, const int32_t(&idx)[4], float(&Xs)[4], float(&Ys)[4], float(&Zs)[4], float(&Us)[4],
                        float(&Vs)[4]) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int64_t i = p0 + idx[j];
                            Xs[j] = (float)p3[3 * i]; Ys[j] = (float)p3[3 * i + 1]; Zs[j] = (float)p3[3 * i + 2];
                            Us[j] = (float)p2[2 * i]; Vs[j] = (float)p2[2 * i + 1];
                        }
                    });
}

// RSAC_DBG_F64_SELFTEST: the fast f64 cores against the IEEE operators, bit for bit, on random
// operands inside the ranges their callers prove (rsac_math.h, rsac_cvepnp.h svd_rotation_sel) and
// on the ranges' ends; every differing result adds one to *bad
__device__ __forceinline__ double st_rand(Philox &r, int emin, int emax) {
    const uint64_t m = ((uint64_t)r.next() << 32 | r.next()) & 0xFFFFFFFFFFFFFull;
    const int e = emin + (int)(r.next() % (uint32_t)(emax - emin + 1));
    return __builtin_bit_cast(double, (uint64_t)(e + 1023) << 52 | m);
}
__global__ __launch_bounds__(256) void k_f64_selftest(int64_t n, int *bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Philox r;
    r.init(0x5EEDF64ull, 7u, (uint64_t)i);
    int nb = 0;
    auto same = [](double x, double y) { return __builtin_bit_cast(uint64_t, x) == __builtin_bit_cast(uint64_t, y); };
    // roots: x in [2^-767, DBL_MAX]; the first lanes take the ends
    double x = st_rand(r, -767, 1023);
    if (i == 0) x = 0x1p-767;
    if (i == 1) x = 0x1.fffffffffffffp+1023;
    nb += !same(dsqrt_fast(x), __builtin_sqrt(x));
    // quotients: |n|, |d| in [2^-300, 2^300] (either sign)
    double nn = st_rand(r, -300, 299), dd = st_rand(r, -300, 299);
    if (i == 2) { nn = 0x1p-300; dd = 0x1.fffffffffffffp+299; }
    if (i == 3) { nn = 0x1.fffffffffffffp+299; dd = 0x1p-300; }
    if (r.next() & 1) nn = -nn;
    if (r.next() & 1) dd = -dd;
    nb += !same(ddiv_fast(nn, dd), nn / dd);
    nb += !same(ddiv_fast(1.0, dd), 1.0 / dd);
    // the Jacobi rotation: a, b in [2^-200, 2^200], p of a pair that is not skipped
    // (10 DBL_EPSILON sqrt(ab) < |p| <= sqrt(ab)), doubled as the callers pass it
    const double a = st_rand(r, -200, 199), b = (r.next() & 3) == 0 ? a : st_rand(r, -200, 199);
    const double sab = __builtin_sqrt(a * b);
    const double f = (double)(r.next() >> 8) * 0x1p-24;  // [0, 1)
    double p = sab * (f < 0.5 ? 1e-14 + f * 1e-3 : f);
    if (!(dabs(p) > cvq::kSvdEps * sab)) p = sab;
    if (r.next() & 1) p = -p;
    double c0, s0, c1, s1;
    cvq::svd_rotation_sel_t<true>(2 * p, a, b, c0, s0);
    cvq::svd_rotation_sel_t<false>(2 * p, a, b, c1, s1);
    nb += !same(c0, c1) || !same(s0, s1);
    if (nb) atomicAdd(bad, nb);
}
hipError_t launch_f64_selftest(int64_t n, int *bad, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_f64_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, bad);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// PnP scoring.  The product path is the MFMA kernel k_pnp_score_mf (its small-round and
// out-of-f16-range forms run the scaled-form body sc_unit); RSAC_F_EXACT_ONLY selects the
// all-f64 kernel k_pnp_score, whose counts the pre-filter kernels must reproduce bit for bit.
// ---------------------------------------------------------------------------
// counts of the block's hypotheses (sum of the 4 waves' partials) and, when
// a.best_key is set, one atomicMax of the block's best packed key
// counts of the block's hypotheses (sum of the 4 waves' partials) and, when
// a.best_key is set, one atomicMax of the block's best packed key
template <int HB>
__device__ __forceinline__ void pnp_score_epilogue(const PnpArgs &a, const int (&red)[4][HB], int prob, int64_t h0,
                                                   int nh, int lane, int32_t *__restrict__ counts) {
    int s = 0;
    if (lane < nh) {
        s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
        counts[(int64_t)prob * a.hyp_stride + h0 + lane] = s;
    }
    if (a.best_key) {
        unsigned long long k = 0;
        if (lane < nh && s > 0) {
            const uint64_t g = (uint64_t)(a.rng_base + h0 + lane);
            k = ((unsigned long long)(uint32_t)s << 32) | (0xFFFFFFFFull - (g & 0xFFFFFFFFull));
        }
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long other = __shfl_xor(k, o);
            k = other > k ? other : k;
        }
        if (lane == 0 && k) atomicMax(a.best_key, k);
    }
}


// ---------------------------------------------------------------------------
// Scaled-form scoring kernel (records of write_fmodel_sc).  Per (hypothesis, point) pair:
//   xs, ys, z' = record rows . (XC, YC, ZC) + t'        9 FMA
//   q1 = u' z' + xs, q2 = v' z' + ys                    2 FMA  (u' = (u - cx) / sqrt(T))
//   D = q1^2 + q2^2 - z'^2                              3      (sign of e - T)
//   t = |D| - a |z'|                                    1 FMA  (abs source modifiers)
//   inlier count: ballot(D < 0)                         1 compare
//   undecided: min3 of the t's over the lane's points   1/2 per pair, then one compare per
//                                                      hypothesis: !(min t > b)
// 16.5 vector instructions per pair against 18 for k_pnp_score_ab.  The fast count takes D < 0
// for every pair; for a hypothesis with an undecided pair on the tile, sc_fallback recomputes
// the tile's pairs (same operations, same bits) and replaces the fast verdict of each undecided
// pair by the exact f64 test.  Points with a non-finite coordinate are staged as decided
// outliers (the exact test says outlier for them: NaN / inf error), so D is never NaN.
// ---------------------------------------------------------------------------
struct ScPair {
    float D, t;
};

__device__ __forceinline__ ScPair sc_pair(const float *m, float x, float y, float zc, float u, float v) {
    const float xs = __builtin_fmaf(m[0], x, __builtin_fmaf(m[1], y, __builtin_fmaf(m[2], zc, m[9])));
    const float ys = __builtin_fmaf(m[3], x, __builtin_fmaf(m[4], y, __builtin_fmaf(m[5], zc, m[10])));
    const float z = __builtin_fmaf(m[6], x, __builtin_fmaf(m[7], y, __builtin_fmaf(m[8], zc, m[11])));
    const float q1 = __builtin_fmaf(u, z, xs);
    const float q2 = __builtin_fmaf(v, z, ys);
    const float D = __builtin_fmaf(-z, z, __builtin_fmaf(q1, q1, q2 * q2));
    const float tt = __builtin_fmaf(-m[12], __builtin_fabsf(z), __builtin_fabsf(D));
    return ScPair{D, tt};
}

// exact recount of the undecided pairs of the flagged hypotheses (wund) on this lane's points:
// returns this lane's share of the count corrections (lane h: hypothesis h's)
template <int P>
__device__ __forceinline__ int sc_fallback(const PnpArgs &a, int prob, int64_t p0, int n, int64_t rec0, int base,
                                           int lane, uint32_t wund, const float *mlds, const float (&px)[P],
                                           const float (&py)[P], const float (&pz)[P], const float (&pu)[P],
                                           const float (&pv)[P]) {
    const double *cm = a.cams + 4 * prob;
    const Cam k{cm[0], cm[1], cm[2], cm[3]};
    const float thr2 = a.thr2[prob];
    int cnt = 0;
#pragma unroll 1
    while (wund) {
        const int h = __builtin_ctz(wund);
        wund &= wund - 1;
        const float *m = mlds + h * kFModelStride;
        const double *md = a.models + (rec0 + h) * kModelStride;
        const bool mv = a.status[rec0 + h] > 0;
        int cc = 0;
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int i = base + j * 64 + lane;
            const ScPair r = sc_pair(m, px[j], py[j], pz[j], pu[j], pv[j]);
            const bool und = !(r.t > m[13]);
            bool ex = false;
            if (und && i < n) {
                const int64_t q = p0 + i;
                ex = mv &&
                     pnp_err(md, md + 9, k, (double)a.X[q], (double)a.Y[q], (double)a.Z[q], a.U[q], a.V[q]) <= thr2;
            }
            cc += __popcll(__ballot(und && ex)) - __popcll(__ballot(und && r.D < 0.f));
        }
        cnt += (lane == h) ? cc : 0;
    }
    return cnt;
}

// One work unit of the scaled-form kernel: hypotheses [h0, h0 + nh) of problem prob (records at
// rec0) over the points [start, n) of the problem (p0 its first point).  The unit's HB records are
// staged in mlds; the counts are added atomically into zeroed counts.  Shared with
// k_pnp_score_mf, which runs its problems outside the f16 operand range through it.
// NW: waves of the block (4; 2 in k_pnp_score_mf<2>)
template <int P, int HB, int NW = 4>
__device__ __forceinline__ void sc_unit(const PnpArgs &a, int prob, int64_t h0, int nh, int64_t p0, int start, int n,
                                        int lane, int wave, int (*red)[HB], float *mlds, int32_t *__restrict__ counts) {
    constexpr int kStride = NW * 64 * P;  // points one pass of the block covers
    const float *__restrict__ fc = a.fconst + (int64_t)prob * kFconstStride;
    const float cx = fc[2], cy = fc[3], inv_s = fc[9];
    const int64_t rec0 = (int64_t)prob * a.hyp_stride + h0;
    if (threadIdx.x < HB) {
        // one thread per record; past the round or no model: z' = 0, xs = 1 (D = 1 > 0, a
        // decided outlier) and b = -inf (never undecided)
        const int hq = threadIdx.x;
        float *dst = mlds + hq * kFModelStride;
        bool valid;
        if (a.fm_inline) {  // the record the solve would have written (k_pnp_setup_solve4)
            const int64_t rec = rec0 + hq;
            const double *md = a.models + rec * kModelStride;
            valid = hq < nh && a.status[rec] > 0;
            if (valid) write_fmodel_sc(md, md + 9, true, a.frame + (int64_t)prob * kFrameStride, a.cams + 4 * prob, fc,
                                       dst);
            valid = valid && dst[14] >= 0.f;
            if (!valid)
#pragma unroll
                for (int q = 0; q < 16; ++q) dst[q] = 0.f;
        } else {
            const float *src = a.fmodels + (rec0 + hq) * kFModelStride;
            valid = hq < nh && src[14] >= 0.f;
#pragma unroll
            for (int q = 0; q < 16; ++q) dst[q] = valid ? src[q] : 0.f;
        }
        if (!valid) {
            dst[9] = 1.f;
            dst[13] = -__builtin_inff();
            dst[15] = -__builtin_inff();
        }
    }
    __syncthreads();
    // the points centred on the problem's frame centre c as the setup kernels centre them,
    // (float)((double)X - c) (r06: computed here per tile instead of read from a stored copy;
    // the batch setup writes 12 B per point less, C3 24 MB per call)
    const double *fr = a.frame + (int64_t)prob * kFrameStride;
    const double c0 = fr[0], c1 = fr[1], c2 = fr[2];
    const float *__restrict__ X = a.X + p0, *__restrict__ Y = a.Y + p0, *__restrict__ Z = a.Z + p0;
    const float *__restrict__ U = a.U + p0, *__restrict__ V = a.V + p0;

    int cnt = 0;
    for (int base = start + wave * 64 * P; base < n; base += kStride) {
        float px[P], py[P], pz[P], pu[P], pv[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int i = base + j * 64 + lane;
            const bool in = i < n;
            const int ii = in ? i : 0;
            const float x = (float)((double)X[ii] - c0), y = (float)((double)Y[ii] - c1),
                        z = (float)((double)Z[ii] - c2), uu = U[ii], vv = V[ii];
            // out of range or a non-finite coordinate: a pixel at 3e38 at the centre's depth
            // makes the pair a decided outlier (or D = xs^2 + ys^2 >= 0 when z' = 0)
            const bool ok = in && __builtin_isfinite(x) && __builtin_isfinite(y) && __builtin_isfinite(z) &&
                            __builtin_isfinite(uu) && __builtin_isfinite(vv);
            px[j] = ok ? x : 0.f;
            py[j] = ok ? y : 0.f;
            pz[j] = ok ? z : 0.f;
            pu[j] = ok ? (uu - cx) * inv_s : 3.0e38f;
            pv[j] = ok ? (vv - cy) * inv_s : 3.0e38f;
        }
        int ccl = 0;        // lane h: hypothesis h's fast count (D < 0) of this tile
        uint32_t wund = 0;  // bit h: hypothesis h has an undecided pair (wave-uniform)
#pragma unroll 4
        for (int h = 0; h < HB; ++h) {
            const float *m = mlds + h * kFModelStride;
            int cc = 0;
            float tmin = __builtin_inff();
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const ScPair r = sc_pair(m, px[j], py[j], pz[j], pu[j], pv[j]);
                cc += __popcll(__ballot(r.D < 0.f));
                tmin = __builtin_fminf(tmin, r.t);
            }
            const uint64_t und = __ballot(!(tmin > m[13]));
            // v_writelane_b32 (no clang builtin); the lane select goes through M0 (two SGPR
            // operands would exceed the constant bus), which the compiler loads itself ("{m0}")
            asm("v_writelane_b32 %0, %1, %2" : "+v"(ccl) : "s"(cc), "{m0}"(h));
            wund |= und ? (1u << h) : 0u;
        }
        cnt += ccl;
        if (__builtin_expect(wund != 0, 0))
            cnt += sc_fallback<P>(a, prob, p0, n, rec0, base, lane, wund, mlds, px, py, pz, pu, pv);
    }
    if (lane < HB) red[wave][lane] = cnt;
    __syncthreads();
    if (wave == 0 && lane < nh) {
        int sum = red[0][lane];
#pragma unroll
        for (int w = 1; w < NW; ++w) sum += red[w][lane];
        if (sum) atomicAdd(&counts[(int64_t)prob * a.hyp_stride + h0 + lane], sum);
    }
}

// Work units (launch_sc): the tiles (problem, 32 hypotheses) are numbered problem-major; the
// first tb of them are one unit each (all their points, one pass of the block per cell of
// 64 x 4 x P points), the rest one unit per cell, so the queue ends with cell-sized units that
// even out the blocks' finishing times.  Counts are added atomically into zeroed counts.
template <int P, int HB, int W = 4>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W, 8))) void k_pnp_score_sc(
    PnpArgs a, int64_t hyp_begin, int32_t H, int32_t n_prob, int *__restrict__ queue, int32_t *__restrict__ counts,
    int tb, int cells) {
    static_assert(HB <= 32, "undecided bits per wave");
    constexpr int kStride = 4 * 64 * P;  // points one pass of the block covers: one cell
    __shared__ int red[4][HB];
    __shared__ int unit_s;
    __shared__ __attribute__((aligned(16))) float mlds[HB * kFModelStride];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_per_prob = (H + HB - 1) / HB;
    const int n_units = tb + (tiles_per_prob * n_prob - tb) * cells;
    for (;;) {
        if (threadIdx.x == 0) unit_s = atomicAdd(queue, 1);
        __syncthreads();
        const int unit = __builtin_amdgcn_readfirstlane(unit_s);
        if (unit >= n_units) break;  // uniform: every wave of every block reaches it
        int tile, c0, c1;             // the unit's tile and cells [c0, c1)
        if (unit < tb) {
            tile = unit;
            c0 = 0;
            c1 = cells;
        } else {
            tile = tb + (unit - tb) / cells;
            c0 = (unit - tb) % cells;
            c1 = c0 + 1;
        }
        const int prob = tile / tiles_per_prob;
        const int64_t h0 = hyp_begin + (int64_t)(tile % tiles_per_prob) * HB;
        const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
        const int64_t p0 = a.offsets[prob];
        const int n_all = (int)(a.offsets[prob + 1] - p0);
        const int start = c0 * kStride;
        const int n = min(n_all, c1 * kStride);  // this unit's points: [start, n)
        if (start < n_all)  // else a cell past a short problem of a batch (uniform)
            sc_unit<P, HB>(a, prob, h0, nh, p0, start, n, lane, wave, red, mlds, counts);
        __syncthreads();  // red, mlds and unit_s are rewritten by the next unit
    }
}

// ---------------------------------------------------------------------------
// MFMA scoring kernel (variant 60; records of write_fmodel_mx, points of mx_point).
//
// xs, ys, z' of 8 hypotheses x 32 points come out of one v_mfma_f32_32x32x16_f16: the A operand
// (32 rows x K 16) holds row r of hypothesis 8t + i/4 in row i (i % 4 = r; r = 3 unused) as
// [hi x4 | hi x4] (lanes 0-31, K 0-7) and [lo x4 | lo x4] (lanes 32-63, K 8-15); the B operand
// (K 16 x 32 points) is every point's PF record [hi XC YC ZC 1 | lo XC YC ZC 0] in both halves,
// so the sum over K is (hi + lo)(Bhi + Blo) for each feature (the four products of a feature are
// exact in f32).  Output map (gfx950): column = lane & 31, row = (reg & 3) + 8 (reg >> 2) +
// 4 (lane >> 5), so lane (c, half) holds xs ys z' of hypotheses 8t + 2g + half (g = 0..3) at
// point c in registers 4g .. 4g + 2.  The VALU then runs the scaled-form test of
// k_pnp_score_sc on them (q1 q2 D: 5, t: 1, count: 1, band minimum: 0.5 per pair):
//   count: the sign bit of D (D is never -0 or NaN: D = -z'^2 + X with X = q1^2 + q2^2 >= +0,
//          and the staged operands are finite), two tiles' bits as 0xFF bytes (v_perm_b32)
//          summed into 255 x the count (v_sad_u8);
//   band:  min3 of the t's of both tiles per slot, compared with b' every CHK iterations.
// A wave runs 2 x 32 points per iteration over all 32 hypotheses of the unit (4 MFMA groups);
// a flagged (slot, window) is recomputed (the same MFMA, the same VALU bits) and its undecided
// pairs take the exact f64 test (pnp_err), as sc_fallback does, so counts equal the exact
// kernel's.  Problems whose centred coordinates leave the f16 range (fconst[11] = 0) carry
// form-1 records and run the sc_unit body.
// ---------------------------------------------------------------------------
typedef _Float16 mf_h8 __attribute__((ext_vector_type(8)));
typedef float mf_f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float mf_min3(float a, float b, float c) {
    float d;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));  // no canonicalising v_max
    return d;
}
__device__ __forceinline__ uint32_t mf_sgn(float x) { return __float_as_uint(x) >> 31; }
// c + 255 ([a < 0] + [b < 0]) in two instructions: v_perm_b32 gathers the two sign bits as 0x00 /
// 0xFF bytes (selectors 9, 11: a byte of copies of bit 31 of src1, src0; 12: zero) and v_sad_u8
// adds the bytes (sum of |byte - 0|) to c
__device__ __forceinline__ uint32_t mf_cnt255(uint32_t c, float a, float b) {
    return __builtin_amdgcn_sad_u8(__builtin_amdgcn_perm(__float_as_uint(a), __float_as_uint(b), 0x0C0C0B09u), 0u, c);
}

struct MfPair {
    float D, t;
};
// the test quantities of slot g of an MFMA output (lambda units; the expressions of sc_pair)
__device__ __forceinline__ MfPair mf_pair(const mf_f16v &x, int g, float2 uv, float ag) {
    const float z = x[4 * g + 2];
    const float q1 = __builtin_fmaf(uv.x, z, x[4 * g]);
    const float q2 = __builtin_fmaf(uv.y, z, x[4 * g + 1]);
    const float D = __builtin_fmaf(-z, z, __builtin_fmaf(q1, q1, q2 * q2));
    const float tt = __builtin_fmaf(-ag, __builtin_fabsf(z), __builtin_fabsf(D));
    return MfPair{D, tt};
}


// global-memory view of a pointer: the kernel's PnpArgs also reaches an out-of-line function by
// reference, after which the compiler no longer infers the address space of its pointer fields
// and would issue flat loads (counted in lgkmcnt with the LDS reads of the hot loop)
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T *gview(const T *p) {
    return (const __attribute__((address_space(1))) T *)p;
}

// one iteration's point operands (tiles [base, base + 32) and [base + 32, base + 64) of the unit)
typedef uint32_t mf_u4 __attribute__((ext_vector_type(4)));
typedef float mf_f2 __attribute__((ext_vector_type(2)));
typedef uint32_t mf_u2 __attribute__((ext_vector_type(2)));
// (lanes 0-31 load a point's first PF record, lanes 32-63 its x 2^-11 copy: hf = lane >> 5)
__device__ __forceinline__ void mf_load_full(const uint4 *__restrict__ PFg, const float2 *__restrict__ UVg, int base,
                                             int col, int hf, mf_h8 &Ba, mf_h8 &Bb, float2 &ua, float2 &ub) {
    const auto PF = gview(reinterpret_cast<const mf_u4 *>(PFg));
    const auto UV = gview(reinterpret_cast<const mf_f2 *>(UVg));
    const int ia = base + col, ib = ia + 32;
    const mf_u4 pa = PF[2 * ia + hf], pb = PF[2 * ib + hf];
    const mf_f2 va = UV[ia], vb = UV[ib];
    Ba = __builtin_bit_cast(mf_h8, pa);
    Bb = __builtin_bit_cast(mf_h8, pb);
    ua = make_float2(va.x, va.y);
    ub = make_float2(vb.x, vb.y);
}
__device__ __forceinline__ void mf_load_part(const uint4 *__restrict__ PFg, const float2 *__restrict__ UVg, int base,
                                             int n, int col, int hf, mf_h8 &Ba, mf_h8 &Bb, float2 &ua, float2 &ub) {
    const auto PF = gview(reinterpret_cast<const mf_u4 *>(PFg));
    const auto UV = gview(reinterpret_cast<const mf_f2 *>(UVg));
    const int ia = base + col, ib = ia + 32;
    // the origin with its constant feature (1, or 2^-11 in the scaled copy)
    const mf_u4 none = {0u, hf ? 0x10000000u : 0x3C000000u, 0u, 0u};
    const mf_f2 far = {3.0e38f, 3.0e38f};
    const mf_u4 pa = ia < n ? PF[2 * ia + hf] : none, pb = ib < n ? PF[2 * ib + hf] : none;
    const mf_f2 va = ia < n ? UV[ia] : far, vb = ib < n ? UV[ib] : far;
    Ba = __builtin_bit_cast(mf_h8, pa);
    Bb = __builtin_bit_cast(mf_h8, pb);
    ua = make_float2(va.x, va.y);
    ub = make_float2(vb.x, vb.y);
}
__device__ __forceinline__ void mf_load(const uint4 *__restrict__ PF, const float2 *__restrict__ UV, int base, int n,
                                        int col, int hf, mf_h8 &Ba, mf_h8 &Bb, float2 &ua, float2 &ub) {
    if (base + 64 <= n)
        mf_load_full(PF, UV, base, col, hf, Ba, Bb, ua, ub);
    else
        mf_load_part(PF, UV, base, n, col, hf, Ba, Bb, ua, ub);
}

// the A operand of MFMA group t for this lane (row col & 31: hypothesis 8t + (col >> 2), row
// col & 3; hi in lanes 0-31, lo in 32-63); past the round: xs = 1 (D = 1, a decided outlier)
__device__ __forceinline__ mf_h8 mf_operand(const float *__restrict__ recs, int t, int col, int half, int nh) {
    const int r = col & 3, j = 8 * t + (col >> 2);
    mf_u2 w = {0u, 0u};
    if (r < 3 && j < nh)
        w = *gview(reinterpret_cast<const mf_u2 *>(reinterpret_cast<const char *>(recs + j * kFModelStride) +
                                                   half * 24 + r * 8));
    else if (r == 0 && half == 0 && j >= nh)
        w.y = 0x3C000000u;
    const mf_u4 v = {w.x, w.y, w.x, w.y};
    return __builtin_bit_cast(mf_h8, v);
}

// the A operand of MFMA group t (mf_operand's values) from an unconditional load: the index is
// clamped into the unit and the value replaced afterwards, so the unit's loads issue together
// instead of one conditional load (and wait) after another
__device__ __forceinline__ mf_h8 mw_operand(const float *__restrict__ recs, int t, int col, int half, int nh) {
    const int r = col & 3, j = 8 * t + (col >> 2);
    const int jj = min(j, nh - 1), rr = min(r, 2);
    mf_u2 w = *gview(reinterpret_cast<const mf_u2 *>(reinterpret_cast<const char *>(recs + jj * kFModelStride) +
                                                     half * 24 + rr * 8));
    if (!(r < 3 && j < nh)) {
        w.x = 0u;
        w.y = (r == 0 && half == 0 && j >= nh) ? 0x3C000000u : 0u;
    }
    const mf_u4 v = {w.x, w.y, w.x, w.y};
    return __builtin_bit_cast(mf_h8, v);
}

// exact recount of one flagged iteration of a unit (one wave; hypotheses rec0 .. rec0 + nh of the
// problem whose points start at p0 and whose unit ends at point n): the MFMA and the VALU test of
// the flagged slots fl are redone (same operands, same bits) and each undecided pair's fast
// verdict (D < 0) is replaced by the exact f64 test (pnp_err); the corrections go to the unit's
// LDS array lcorr (index: hypothesis within the unit), which the epilogue folds into the counts.
// Every load that does not depend on the test (point operands, the slopes and bands of the 32
// hypotheses, the lane's two points in f32) is issued up front; per flagged group the A
// operand, per slot with an undecided pair its model.
__device__ __forceinline__ void mf_recount(const PnpArgs &a, int64_t rec0, int64_t p0, int n, uint32_t fl, int nh,
                                           int base, int col, int half, int *lcorr) {
    const int prob = (int)(rec0 / a.hyp_stride);
    const float *__restrict__ recs = a.fmodels + rec0 * kFModelStride;
    mf_h8 Ba, Bb;
    float2 ua, ub;
    mf_load(a.PF + 2 * p0, a.UV + p0, base, n, col, half, Ba, Bb, ua, ub);
    // lane c < 32: a' and b' of hypothesis c (read by the others through a lane shuffle)
    const int jc = min(col, nh - 1);
    const float a_c = gview(recs)[jc * kFModelStride + 12], b_c = gview(recs)[jc * kFModelStride + 13];
    const int ia = base + col, ib = ia + 32;
    const int64_t qa = p0 + min(ia, n - 1), qb = p0 + min(ib, n - 1);
    const float Xa = a.X[qa], Ya = a.Y[qa], Za = a.Z[qa], Uxa = a.U[qa], Vxa = a.V[qa];
    const float Xb = a.X[qb], Yb = a.Y[qb], Zb = a.Z[qb], Uxb = a.U[qb], Vxb = a.V[qb];
    const double *cm = a.cams + 4 * prob;
    const Cam k{cm[0], cm[1], cm[2], cm[3]};
    const float thr2 = a.thr2[prob];
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
        const uint32_t ft = (fl >> (4 * t)) & 15u;
        if (!ft) continue;  // uniform
        const mf_h8 At = mw_operand(recs, t, col, half, nh);
        const mf_f16v xa = __builtin_amdgcn_mfma_f32_32x32x16_f16(At, Ba, mf_f16v{}, 0, 0, 0);
        const mf_f16v xb = __builtin_amdgcn_mfma_f32_32x32x16_f16(At, Bb, mf_f16v{}, 0, 0, 0);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (!((ft >> g) & 1u)) continue;  // uniform
            const int j = 8 * t + 2 * g + half;  // this lane's hypothesis
            const bool live = j < nh;
            const float aj = __shfl(a_c, j), bj = __shfl(b_c, j);
            const float ag = live ? aj : 0.f;
            const float bg = live ? bj : -__builtin_inff();
            const MfPair ra = mf_pair(xa, g, ua, ag), rb = mf_pair(xb, g, ub, ag);
            const bool wa = !(ra.t > bg) && ia < n, wb = !(rb.t > bg) && ib < n;
            if (wa || wb) {
                const double *md = a.models + (rec0 + j) * kModelStride;
                const bool mv = a.status[rec0 + j] > 0;
                int c = 0;
                if (wa)
                    c += (mv && pnp_err(md, md + 9, k, (double)Xa, (double)Ya, (double)Za, Uxa, Vxa) <= thr2 ? 1 : 0) -
                         (ra.D < 0.f ? 1 : 0);
                if (wb)
                    c += (mv && pnp_err(md, md + 9, k, (double)Xb, (double)Yb, (double)Zb, Uxb, Vxb) <= thr2 ? 1 : 0) -
                         (rb.D < 0.f ? 1 : 0);
                if (c) atomicAdd(&lcorr[j], c);
            }
        }
    }
}

// the form-1 body for problems outside the f16 operand range (rare: kept out of line, so its
// registers do not constrain the MFMA loop's).  The arguments are read from the kernel's argument
// segment (PnpArgs is the first kernel argument, offset 0): passing the kernel parameter by
// reference would give it an address, and the compiler then copies all of PnpArgs to scratch
// in every wave and reads every field in the hot kernel from there (≈50 MB of scratch writes per
// C2 launch)
typedef const __attribute__((address_space(4))) PnpArgs *KernargPnp;
__device__ __forceinline__ KernargPnp kernarg_pnp() {
    return (KernargPnp)__builtin_amdgcn_kernarg_segment_ptr();
}
template <int W>
__device__ __attribute__((noinline)) void mf_sc_unit(KernargPnp ka, int prob, int64_t h0, int nh, int64_t p0,
                                                     int start, int n, int lane, int wave, int (*red)[32], float *mlds,
                                                     int32_t *__restrict__ counts) {
    const PnpArgs a = *(const PnpArgs *)ka;  // generic view (the host pass has no address spaces)
    sc_unit<8, 32, W>(a, prob, h0, nh, p0, start, n, lane, wave, red, mlds, counts);
}


// One unit of k_pnp_score_mf: hypotheses [h0, h0 + nh) of problem prob (records at rec0) over
// the points [start, n) of the problem (p0 its first point, n_all_pts its length).  Per
// iteration a wave takes 2 x 32 points: 4 MFMA groups x 2 tiles, the counts (255 x, v_sad_u8)
// and each slot's band check (the smaller t of its two pairs against b'); a flagged iteration
// goes to the wave's LDS list (at most kWrec: the launcher bounds a unit's points by 256 kWrec).  After its point loop the wave recounts its listed iterations
// exactly (mf_recount) into the unit's LDS corrections, which the epilogue adds to the counts.
// waves per block of k_pnp_score_mf<W>: 4 for long problems; 2 for batches of short ones, whose
// units then run twice the iterations per wave over the same unit overhead (launch_mf; C3
// 1.081 -> 1.028 ms, while C2 at 2 waves is 66 % slower: scripts/mf_ab.py)
// wave priority (s_setprio) of the scorer: raised (2) from the end of a wave's point loop through
// its recounts, the count epilogue and the next unit's staging, back to 0 for the point loop, so
// the waves a block's barriers wait for get the SIMD first (C2 scoring -1 %, scripts/mf_ab.py r03d).
// (The static-priority and hand-scheduled asm probes of rounds 3-4 are kept as
// scripts/ubench/probes_r04.patch; DESIGN.md §3 has their numbers.)
constexpr int kMfLongW = 4;   // waves per block for one long problem
constexpr int kMfShortW = 2;  // waves per block for batches of short problems (C3)
// the batch instance (W = kMfShortW: many short problems, C3) loads iteration i + 1's point
// operands before iteration i computes: its problems' points miss L2 more often (C3 92 % hits
// against C2's 98 %, profiles/r05/pmc_scorer_c2_c3.json) and the prefetch took C3 0.956 -> 0.931 ms,
// while the long-problem instance ran 4 % slower with it (scripts/mf_ab.py, r05).  (The A/B
// builds of these choices and of mf_tid's opacity are scripts/ubench/mf_knobs_r05.patch.)
constexpr int kMfPrefetchW = kMfShortW;
constexpr int kMfW = kMfLongW;
constexpr int kWrec = 64;        // flagged iterations a wave lists per unit

// the thread index as a value the compiler cannot hoist: the unit's lane-dependent offsets are then
// formed inside each unit (a few integer instructions) instead of being held across the unit loop,
// where at the 168-VGPR budget of 3 waves/SIMD they were spilled (548 B of scratch per lane, r04)
__device__ __forceinline__ int mf_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

template <int W>
__device__ __forceinline__ void mf_unit(const PnpArgs &a, int prob, int64_t h0, int nh, int64_t p0, int start, int n,
                                        int n_all_pts, uint32_t (*cl)[16][64], float (*ab)[2][4][4],
                                        mf_h8 (*alds)[64], uint2 (*wrec)[kWrec], int *lcorr,
                                        int32_t *__restrict__ counts) {
    constexpr int HB = 32, T = 64 * W;  // T: threads = points one pass of the block covers
    const int tid = mf_tid();
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int col = lane & 31, half = lane >> 5;
    const int64_t rec0 = (int64_t)prob * a.hyp_stride + h0;
    const float *__restrict__ recs = a.fmodels + rec0 * kFModelStride;
    if (tid < HB) {
        lcorr[tid] = 0;  // the unit's corrections (before the barrier)
        // a' and b' of slot (t, g, half) = hypothesis 8t + 2g + half; past the round: b' = -inf
        // (records without a model carry a' = 0, b' = -inf themselves)
        const int j = tid;
        const bool v = j < nh;
        ab[0][j & 1][j >> 3][(j >> 1) & 3] = v ? gview(recs)[j * kFModelStride + 12] : 0.f;
        ab[1][j & 1][j >> 3][(j >> 1) & 3] = v ? gview(recs)[j * kFModelStride + 13] : -__builtin_inff();
    }
    // the unit's A operands (the same for every wave): entry (t, lane) holds group t's
    for (int e = tid; e < 256; e += T) {
        const int tl = e & 63;
        alds[e >> 6][tl] = mf_operand(recs, e >> 6, tl & 31, tl >> 5, nh);
    }
    __syncthreads();
    const uint4 *__restrict__ PF = a.PF + 2 * p0;
    const float2 *__restrict__ UV = a.UV + p0;
    uint32_t vc[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) vc[t][g] = 0u;
    int nw = 0;  // flagged iterations in the wave's list (uniform)
    const int b0 = start + wave * 64;
    const int iters = n > b0 ? (n - b0 + T - 1) / T : 0;
    // the A operands in registers for the whole unit; the slopes a' and bands b' are read from
    // LDS per group, ahead of the group's MFMAs (in registers they would cost 32 VGPRs)
    mf_h8 Ar[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) Ar[t] = alds[t][lane];
    auto body = [&](int i, const mf_h8 &Ba, const mf_h8 &Bb, const float2 &ua, const float2 &ub)
        __attribute__((always_inline)) {
        // each slot's band compared as soon as its two t's exist: min(t_a, t_b) <= b' flags the
        // slot; no minima are held across the iteration
        uint32_t fl = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float4 av = *reinterpret_cast<const float4 *>(&ab[0][half][t][0]);
            const float4 bv = *reinterpret_cast<const float4 *>(&ab[1][half][t][0]);
            const mf_f16v xa = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t], Ba, mf_f16v{}, 0, 0, 0);
            const mf_f16v xb = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t], Bb, mf_f16v{}, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float ag = g == 0 ? av.x : g == 1 ? av.y : g == 2 ? av.z : av.w;
                const float bg = g == 0 ? bv.x : g == 1 ? bv.y : g == 2 ? bv.z : bv.w;
                const MfPair ra = mf_pair(xa, g, ua, ag), rb = mf_pair(xb, g, ub, ag);
                vc[t][g] = mf_cnt255(vc[t][g], ra.D, rb.D);  // 255 x the count
                fl |= __ballot(!(__builtin_fminf(ra.t, rb.t) > bg)) ? (1u << (4 * t + g)) : 0u;
            }
        }
        if (__builtin_expect(fl != 0, 0)) {
            if (lane == 0) wrec[wave][nw] = make_uint2((uint32_t)i, fl);
            ++nw;
        }
    };
    const int full = n >= b0 + 64 ? (n - b0 - 64) / T + 1 : 0;  // iterations with 64 points in range
    __builtin_amdgcn_s_setprio(0);
    if constexpr (W == kMfPrefetchW) {
    if (full > 0) {  // the next iteration's operands in flight while this one computes
        mf_h8 Ba, Bb;
        float2 ua, ub;
        mf_load_full(PF, UV, b0, col, half, Ba, Bb, ua, ub);
        for (int i = 0; i < full; ++i) {
            mf_h8 Na = Ba, Nb = Bb;
            float2 na = ua, nb = ub;
            if (i + 1 < full) mf_load_full(PF, UV, b0 + T * (i + 1), col, half, Na, Nb, na, nb);
            body(i, Ba, Bb, ua, ub);
            Ba = Na; Bb = Nb; ua = na; ub = nb;
        }
    }
    } else {
    for (int i = 0; i < full; ++i) {
        mf_h8 Ba, Bb;
        float2 ua, ub;
        mf_load_full(PF, UV, b0 + T * i, col, half, Ba, Bb, ua, ub);
        body(i, Ba, Bb, ua, ub);
    }
    }
    if (full < iters) {
        mf_h8 Ba, Bb;
        float2 ua, ub;
        mf_load_part(PF, UV, b0 + T * full, n, col, half, Ba, Bb, ua, ub);
        body(full, Ba, Bb, ua, ub);
    }
    // the wave's flagged iterations recounted here: the wave's exact-test latency overlaps the
    // other blocks' waves on its SIMD
    __builtin_amdgcn_s_setprio(2);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll 1
    for (int k = 0; k < nw; ++k) {
        const uint2 w = wrec[wave][k];
        mf_recount(a, rec0, p0, n, w.y, nh, b0 + T * (int)w.x, col, half, lcorr);
    }
    // counts: lane (c, half) of wave w holds slot (t, g)'s count over its points; hypothesis j =
    // 8t + 2g + half sums 4 waves x 32 lanes (8 threads of 16 values each, then a shuffle tree)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) cl[wave][4 * t + g][lane] = vc[t][g];
    __syncthreads();
    constexpr int TPH = T / 32, LPT = 32 / TPH;  // threads per hypothesis, lanes per thread
    const int j = tid / TPH, p = tid % TPH;
    const int slot = 4 * (j >> 3) + ((j >> 1) & 3), l0 = (j & 1) * 32 + LPT * p;
    uint32_t sum = 0;
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
        for (int l = 0; l < LPT; ++l) sum += cl[w][slot][l0 + l];
#pragma unroll
    for (int o = 1; o < TPH; o <<= 1) sum += __shfl_xor(sum, o);
    if (p == 0 && j < nh) {
        // + the unit's corrections (in LDS, complete at the barrier above).  A unit over all of
        // its problem's points is the only writer of its counts: a store (an atomic is
        // acknowledged by the device's coherence point, and every later wait of the wave would
        // wait for it); cells add theirs
        const int cj = (int)(sum / 255u) + lcorr[j];
        if (start == 0 && n == n_all_pts)
            counts[rec0 + j] = cj;
        else if (cj)
            atomicAdd(&counts[rec0 + j], cj);
    }
}

// Units from the split queue: block b takes units b % kQSub + kQSub i from counter b % kQSub.
// Unit numbering as k_pnp_score_sc (the first tb tiles whole, then one unit per cell of cell_pts
// points).  Problems whose centred coordinates leave the f16 operand range (fconst[11] = 0) carry
// form-1 records and run the sc_unit body.  3 waves per SIMD (168 VGPRs; forcing 4 spills and
// costs 23 %, scripts/mf_ab.py).
template <int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(3, 8))) void k_pnp_score_mf(
    PnpArgs a, int64_t hyp_begin, int32_t H, int32_t n_prob, int *__restrict__ queue, int32_t *__restrict__ counts,
    int tb, int cells, int cell_pts) {
    constexpr int HB = 32;
    // the unit index, double-buffered by iteration parity: thread 0 writes the next unit's slot
    // while the other waves may still be reading this one's (a skipped cell runs no barrier
    // between the read at the loop's top and that write)
    __shared__ int unit_s[2];
    __shared__ uint32_t cl[W][16][64];
    __shared__ __attribute__((aligned(16))) float ab[2][2][4][4];
    __shared__ uint2 wrec[W][kWrec];
    __shared__ int lcorr[32];  // the unit's exact-recount corrections
    __shared__ mf_h8 alds[4][64];
    __shared__ int red[4][HB];                                                 // sc_unit
    __shared__ __attribute__((aligned(16))) float mlds[HB * kFModelStride];  // sc_unit
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_per_prob = (H + HB - 1) / HB;
    // whole-tile units by XCD: blocks are dealt round-robin over the 8 XCDs, so counter k (blocks
    // b = k mod 8) runs on XCD k; its units k + 8 i take the contiguous tiles k cpx + i, and a
    // problem's tiles (and points) stay in one XCD's L2 (C3: 1.109 -> 1.077 ms per call, C2 +-0,
    // scripts/mf_ab.py --c3).  Units past tb are empty.  Placement changes speed only.
    const int cpx = (tb + kQSub - 1) / kQSub, tbx = cpx * kQSub;
    const int n_units = tbx + (tiles_per_prob * n_prob - tb) * cells;
    const int qk = blockIdx.x % kQSub;  // this block's units: qk + kQSub i, i from counter qk
    int *const uq = unit_queue(queue, qk);
    int last_prob = -1, n_all = 0;
    int64_t p0 = 0;
    bool in_range = false;
    if (threadIdx.x == 0) unit_s[0] = qk + kQSub * atomicAdd(uq, 1);
    __syncthreads();
    for (int par = 0;; par ^= 1) {
        const int unit = __builtin_amdgcn_readfirstlane(unit_s[par]);
        if (unit >= n_units) break;  // uniform: every wave of every block reaches it
        // the next unit's index, in flight while this unit runs: the library is built with the
        // atomic optimizer off (Makefile), so the compiler waits for the result only where it is
        // used, at the unit's end
        int nx = 0;
        if (threadIdx.x == 0) nx = atomicAdd(uq, 1);
        int tile, c0, c1;
        if (unit < tbx) {
            tile = (unit % kQSub) * cpx + unit / kQSub;
            c0 = 0;
            c1 = cells;
        } else {
            tile = tb + (unit - tbx) / cells;
            c0 = (unit - tbx) % cells;
            c1 = c0 + 1;
        }
        if (unit < tbx && tile >= tb) {  // an empty unit (uniform): the slot protocol as a skipped cell
            if (threadIdx.x == 0) {
                asm volatile("" : "+v"(nx));
                unit_s[par ^ 1] = qk + kQSub * nx;
            }
            __syncthreads();
            continue;
        }
        const int prob = tile / tiles_per_prob;
        const int64_t h0 = hyp_begin + (int64_t)(tile % tiles_per_prob) * HB;
        const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
        if (prob != last_prob) {  // uniform; once per call for one problem
            p0 = a.offsets[prob];
            n_all = (int)(a.offsets[prob + 1] - p0);
            in_range = a.fconst[(int64_t)prob * kFconstStride + 11] != 0.f;
            last_prob = prob;
        }
        const int start = c0 * cell_pts;
        const int n = min(n_all, c1 * cell_pts);
        if (start < n_all) {  // else a cell past a short problem of a batch (uniform)
            if (in_range)
                mf_unit<W>(a, prob, h0, nh, p0, start, n, n_all, cl, ab, alds, wrec, lcorr, counts);
            else
                mf_sc_unit<W>(kernarg_pnp(), prob, h0, nh, p0, start, n, lane, wave, red, mlds, counts);
        }
        // the next unit (the other slot); the empty asm keeps the arithmetic on nx (and so the
        // wait for it) here
        if (threadIdx.x == 0) {
            asm volatile("" : "+v"(nx));
            unit_s[par ^ 1] = qk + kQSub * nx;
        }
        __syncthreads();  // the unit's LDS and the slot are rewritten by the next unit
    }
}


// ---------------------------------------------------------------------------
// PnP scoring.  Block = 4 waves; a block owns HB consecutive hypotheses of
// one problem, its waves split that problem's points (tiles of 64*P per
// wave).  Each lane keeps P correspondences in registers (f64 X Y Z, f32 u
// v) and runs every hypothesis of the block over them; the hypothesis'
// model is wave-uniform (SGPRs).  Lane h accumulates the count of
// hypothesis h; waves are summed through LDS at the end.
// ---------------------------------------------------------------------------
template <int P, int HB>
__global__ __launch_bounds__(256) void k_pnp_score(PnpArgs a, int64_t hyp_begin, int32_t H, int32_t *__restrict__ counts) {
    static_assert(HB <= 64, "one lane per hypothesis of the block");
    __shared__ int red[4][HB];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t h0 = hyp_begin + (int64_t)blockIdx.x * HB;
    const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const double *c = a.cams + 4 * prob;
    const Cam k{c[0], c[1], c[2], c[3]};
    const float thr2 = a.thr2[prob];
    const double *__restrict__ mb = a.models + ((int64_t)prob * a.hyp_stride + h0) * kModelStride;
    const int8_t *__restrict__ sb = a.status + (int64_t)prob * a.hyp_stride + h0;
    const float *__restrict__ X = a.X + p0, *__restrict__ Y = a.Y + p0, *__restrict__ Z = a.Z + p0;
    const float *__restrict__ U = a.U + p0, *__restrict__ V = a.V + p0;

    int cnt = 0;
    for (int base = wave * 64 * P; base < n; base += 4 * 64 * P) {
        double px[P], py[P], pz[P];
        float pu[P], pv[P];
        bool in[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int i = base + j * 64 + lane;
            in[j] = i < n;
            const int ii = in[j] ? i : 0;
            px[j] = X[ii]; py[j] = Y[ii]; pz[j] = Z[ii];
            pu[j] = U[ii]; pv[j] = V[ii];
        }
        for (int h = 0; h < nh; ++h) {
            const double *__restrict__ m = mb + h * kModelStride;
            if (sb[h] <= 0) continue;
            const double R[9] = {m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8]};
            const double t[3] = {m[9], m[10], m[11]};
            int cc = 0;
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const float e = pnp_err(R, t, k, px[j], py[j], pz[j], pu[j], pv[j]);
                cc += __popcll(__ballot(in[j] && e <= thr2));
            }
            cnt += (lane == h) ? cc : 0;
        }
    }
    if (lane < HB) red[wave][lane] = cnt;
    __syncthreads();
    if (wave == 0) pnp_score_epilogue<HB>(a, red, prob, h0, nh, lane, counts);
}

// mask of one model per problem (best[prob] indexes the models buffer; <0 = none)
// model_out (optional): block 0 of every problem also copies the winner's record there
// (k_gather_models' output, one launch fewer)
__device__ __forceinline__ void pnp_mask_body(const PnpArgs &a, int prob, int64_t b, uint8_t *__restrict__ mask,
                                              double *__restrict__ model_out, double *__restrict__ host_model_out) {
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    if (model_out && blockIdx.x == 0 && threadIdx.x < kModelStride) {
        // (a hypothesis record's validity is its status byte; the per-problem copy carries it in
        // kValidSlot)
        const int q = threadIdx.x;
        const double v = b < 0 ? 0.0 : q == kValidSlot ? (a.status[b] > 0 ? 1.0 : 0.0) : a.models[b * kModelStride + q];
        model_out[(int64_t)prob * kModelStride + threadIdx.x] = v;
        if (host_model_out) host_model_out[(int64_t)prob * kModelStride + threadIdx.x] = v;  // pinned host copy
    }
    const double *c = a.cams + 4 * prob;
    const Cam k{c[0], c[1], c[2], c[3]};
    const float thr2 = a.thr2[prob];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint8_t f = 0;
        if (b >= 0) {
            const double *m = a.models + b * kModelStride;
            const int64_t q = p0 + i;
            f = pnp_err(m, m + 9, k, (double)a.X[q], (double)a.Y[q], (double)a.Z[q], a.U[q], a.V[q]) <= thr2;
        }
        mask[p0 + i] = f;
    }
}
__global__ void k_pnp_mask(PnpArgs a, const int64_t *__restrict__ best, int64_t best0, uint8_t *__restrict__ mask,
                           double *__restrict__ model_out, double *__restrict__ host_model_out) {
    const int prob = blockIdx.y;
    // best0: the one problem's record, no upload
    pnp_mask_body(a, prob, best ? best[prob] : best0, mask, model_out, host_model_out);
}

// mask of the hypothesis named by a packed key (problem 0, records from hypothesis 0)
__global__ void k_pnp_mask_key(PnpArgs a, int32_t n, const unsigned long long *__restrict__ key,
                               uint8_t *__restrict__ mask) {
    const unsigned long long k = *key;
    const double *c = a.cams;
    const Cam cam{c[0], c[1], c[2], c[3]};
    const float thr2 = a.thr2[0];
    const double *m = nullptr;
    if (k) {
        const uint64_t low = 0xFFFFFFFFull - (k & 0xFFFFFFFFull);
        const int64_t h = (int64_t)((low - ((uint64_t)a.rng_base & 0xFFFFFFFFull)) & 0xFFFFFFFFull);
        m = a.models + h * kModelStride;
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        mask[i] = m ? (pnp_err(m, m + 9, cam, (double)a.X[i], (double)a.Y[i], (double)a.Z[i], a.U[i], a.V[i]) <= thr2)
                    : 0;
}

// The end of an evaluate_range call in one launch: the record named by the packed key
// -> rec16 (and R, t -> model12, the raw key -> key_out, when given) and its
// RANSAC-test mask (when given).
__global__ void k_pnp_key_finish(PnpArgs a, int32_t n, const unsigned long long *__restrict__ key,
                                 uint8_t *__restrict__ mask, double *__restrict__ rec16, double *__restrict__ model12,
                                 int64_t *__restrict__ key_out) {
    const unsigned long long k = *key;
    const double *m = nullptr;
    if (k) {
        const uint64_t low = 0xFFFFFFFFull - (k & 0xFFFFFFFFull);
        const int64_t h = (int64_t)((low - ((uint64_t)a.rng_base & 0xFFFFFFFFull)) & 0xFFFFFFFFull);
        m = a.models + h * kModelStride;
    }
    if (blockIdx.x == 0 && threadIdx.x < kModelStride) {
        const int q = threadIdx.x;
        const double v = m ? (q == kValidSlot ? 1.0 : m[q]) : 0.0;  // a nonzero key: status > 0 (k_best_key)
        rec16[q] = v;
        if (model12 && q < 12) model12[q] = v;
        if (key_out && q == 0) *key_out = (int64_t)k;
    }
    if (!mask) return;
    const double *c = a.cams;
    const Cam cam{c[0], c[1], c[2], c[3]};
    const float thr2 = a.thr2[0];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        mask[i] = m ? (pnp_err(m, m + 9, cam, (double)a.X[i], (double)a.Y[i], (double)a.Z[i], a.U[i], a.V[i]) <= thr2)
                    : 0;
}

// per-call state reset in one launch: bounds sentinels, best key, work-queue counter
__global__ void k_pnp_init(int32_t P, int *__restrict__ ws, unsigned long long *__restrict__ key,
                           int *__restrict__ queue) {
    for (int i = threadIdx.x; i < 10 * P; i += blockDim.x) ws[i] = i < 5 * P ? 0x7F7F7F7F : (int)0x80808080;
    if (threadIdx.x == 0) {
        if (key) *key = 0ull;
        reset_pnp_queue(queue);
    }
}

// ---------------------------------------------------------------------------
// Homography
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hom_solve(HomArgs a, int64_t hyp_begin, int32_t H) {
    const int prob = blockIdx.y;
    const int hl = blockIdx.x * blockDim.x + threadIdx.x;
    if (hl >= H) return;
    const int64_t h = hyp_begin + hl;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    double *m = a.models + rec * kModelStride;
    float sx[4], sy[4], dx[4], dy[4];
    int8_t st = 1;
    if (a.subsets) {
        st = a.sub_status[rec];
        if (st > 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t i = p0 + a.subsets[rec * 4 + j];
                sx[j] = a.SX[i]; sy[j] = a.SY[i]; dx[j] = a.DX[i]; dy[j] = a.DY[i];
            }
        }
    } else if (n < 4) {
        st = -1;
    } else {
        Philox rng;
        rng.init(a.seed, 0u, (uint64_t)(a.rng_base + h));
        st = -1;
        for (int att = 0; att < kMaxSubsetAttempts; ++att) {
            int32_t idx[4];
            if (rng.subset<4>(n, idx) < 0) break;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t i = p0 + idx[j];
                sx[j] = a.SX[i]; sy[j] = a.SY[i]; dx[j] = a.DX[i]; dy[j] = a.DY[i];
            }
            if (hom_check_subset(sx, sy, dx, dy)) { st = 1; break; }
        }
    }
    double Hm[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (st > 0) st = hom_minimal(sx, sy, dx, dy, Hm) ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = Hm[q];
    m[kValidSlot] = st > 0 ? 1.0 : 0.0;
    a.status[rec] = st;
}

template <int P, int HB>
__global__ __launch_bounds__(256) void k_hom_score(HomArgs a, int64_t hyp_begin, int32_t H, int32_t *__restrict__ counts) {
    __shared__ int red[4][HB];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t h0 = hyp_begin + (int64_t)blockIdx.x * HB;
    const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const float thr2 = a.thr2[prob];
    const double *__restrict__ mb = a.models + ((int64_t)prob * a.hyp_stride + h0) * kModelStride;
    const float *__restrict__ SX = a.SX + p0, *__restrict__ SY = a.SY + p0;
    const float *__restrict__ DX = a.DX + p0, *__restrict__ DY = a.DY + p0;
    int cnt = 0;
    for (int base = wave * 64 * P; base < n; base += 4 * 64 * P) {
        float sx[P], sy[P], dx[P], dy[P];
        bool in[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int i = base + j * 64 + lane;
            in[j] = i < n;
            const int ii = in[j] ? i : 0;
            sx[j] = SX[ii]; sy[j] = SY[ii]; dx[j] = DX[ii]; dy[j] = DY[ii];
        }
        for (int h = 0; h < nh; ++h) {
            const double *__restrict__ m = mb + h * kModelStride;
            if (m[kValidSlot] == 0.0) continue;
            float hf[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) hf[q] = (float)m[q];
            int cc = 0;
#pragma unroll
            for (int j = 0; j < P; ++j) cc += __popcll(__ballot(in[j] && hom_err(hf, sx[j], sy[j], dx[j], dy[j]) <= thr2));
            cnt += (lane == h) ? cc : 0;
        }
    }
    if (lane < HB) red[wave][lane] = cnt;
    __syncthreads();
    if (threadIdx.x < nh) {
        const int s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        counts[(int64_t)prob * a.hyp_stride + h0 + threadIdx.x] = s;
    }
}

// Small problems (<= kLanePts points: the 12-feature scenes of main_v1.py and
// testpro-K.py): one lane per hypothesis over all of the problem's points,
// staged once per block in LDS.  The tile kernels would leave most lanes idle.
__global__ __launch_bounds__(256) void k_hom_score_lane(HomArgs a, int64_t hyp_begin, int32_t H,
                                                        int32_t *__restrict__ counts) {
    __shared__ float sp[4][kLanePts];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    for (int i = threadIdx.x; i < n; i += 256) {
        sp[0][i] = a.SX[p0 + i]; sp[1][i] = a.SY[p0 + i]; sp[2][i] = a.DX[p0 + i]; sp[3][i] = a.DY[p0 + i];
    }
    __syncthreads();
    const int hl = blockIdx.x * 256 + threadIdx.x;
    if (hl >= H) return;
    const int64_t rec = (int64_t)prob * a.hyp_stride + hyp_begin + hl;
    const double *__restrict__ m = a.models + rec * kModelStride;
    int cnt = 0;
    if (m[kValidSlot] != 0.0) {
        const float thr2 = a.thr2[prob];
        float hf[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) hf[q] = (float)m[q];
        for (int i = 0; i < n; ++i) cnt += hom_err(hf, sp[0][i], sp[1][i], sp[2][i], sp[3][i]) <= thr2;
    }
    counts[rec] = cnt;
}

// PnP twin: the exact f64 error (pnp_err, the oracle's formula) per pair -- at
// these sizes the f32 pre-filter buys nothing.  Optional fused best key.
__global__ __launch_bounds__(256) void k_pnp_score_lane(PnpArgs a, int64_t hyp_begin, int32_t H,
                                                        int32_t *__restrict__ counts) {
    __shared__ float sp[5][kLanePts];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    for (int i = threadIdx.x; i < n; i += 256) {
        sp[0][i] = a.X[p0 + i]; sp[1][i] = a.Y[p0 + i]; sp[2][i] = a.Z[p0 + i];
        sp[3][i] = a.U[p0 + i]; sp[4][i] = a.V[p0 + i];
    }
    __syncthreads();
    const int hl = blockIdx.x * 256 + threadIdx.x;
    int cnt = 0;
    if (hl < H) {
        const int64_t rec = (int64_t)prob * a.hyp_stride + hyp_begin + hl;
        const double *__restrict__ m = a.models + rec * kModelStride;
        if (a.status[rec] > 0) {
            const double *cm = a.cams + 4 * prob;
            const Cam k{cm[0], cm[1], cm[2], cm[3]};
            const float thr2 = a.thr2[prob];
            for (int i = 0; i < n; ++i)
                cnt += pnp_err(m, m + 9, k, (double)sp[0][i], (double)sp[1][i], (double)sp[2][i], sp[3][i],
                               sp[4][i]) <= thr2;
        }
        counts[rec] = cnt;
    }
    if (a.best_key) {
        unsigned long long key = 0;
        if (hl < H && cnt > 0) {
            const uint64_t g = (uint64_t)(a.rng_base + hyp_begin + hl);
            key = ((unsigned long long)(uint32_t)cnt << 32) | (0xFFFFFFFFull - (g & 0xFFFFFFFFull));
        }
        for (int o = 32; o > 0; o >>= 1) {
            const unsigned long long other = __shfl_xor(key, o);
            key = other > key ? other : key;
        }
        if ((threadIdx.x & 63) == 0 && key) atomicMax(a.best_key, key);
    }
}

__global__ void k_hom_mask(HomArgs a, const int64_t *__restrict__ best, int64_t best0, uint8_t *__restrict__ mask) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t b = best ? best[prob] : best0;  // best0: the one problem's record, no upload
    const float thr2 = a.thr2[prob];
    float hf[8];
    if (b >= 0) {
        const double *m = a.models + b * kModelStride;
#pragma unroll
        for (int q = 0; q < 8; ++q) hf[q] = (float)m[q];
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint8_t f = 0;
        const int64_t q = p0 + i;
        if (b >= 0) f = hom_err(hf, a.SX[q], a.SY[q], a.DX[q], a.DY[q]) <= thr2;
        mask[q] = f;
    }
}

__global__ void k_gather_models(const double *__restrict__ models, const int64_t *__restrict__ rec, int64_t rec0,
                                int32_t P, double *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * kModelStride) return;
    const int p = i / kModelStride, q = i % kModelStride;
    const int64_t r = rec ? rec[p] : rec0;
    out[i] = r >= 0 ? models[r * kModelStride + q] : 0.0;
}

// OpenCV's count == model_points branch (solvePnPRansac / findHomography): problem p's result is the
// one minimal model of its points in input order -- record p of rec4 (4-point kind) or rec5 (5-point
// kind) -- copied to out[p] (and the pinned host_out[p]), and every one of its points is an inlier
// when that model exists, none when it does not.  One block per problem; kind[p] == 0: untouched.
__global__ void k_direct_finish(const double *__restrict__ rec4, const double *__restrict__ rec5,
                                const int8_t *__restrict__ st4, const int8_t *__restrict__ st5,
                                const int8_t *__restrict__ kind, const int64_t *__restrict__ offsets,
                                double *__restrict__ out, double *__restrict__ host_out, uint8_t *__restrict__ mask) {
    const int p = blockIdx.x;
    const int k = kind[p];
    if (k == 0) return;
    const double *m = (k == 5 ? rec5 : rec4) + (int64_t)p * kModelStride;
    const bool ok = (k == 5 ? st5 : st4)[p] > 0;  // the solve's status byte (PnP records leave kValidSlot)
    const int t = threadIdx.x;
    if (t < kModelStride) {
        const double v = t == kValidSlot ? (ok ? 1.0 : 0.0) : m[t];
        out[(int64_t)p * kModelStride + t] = v;
        if (host_out) host_out[(int64_t)p * kModelStride + t] = v;
    }
    const int64_t o = offsets[p];
    if (mask && t < (int)(offsets[p + 1] - o)) mask[o + t] = ok ? 1 : 0;
}

// packed key of the best hypothesis of a range (count desc, index asc):
// (count << 32) | (0xFFFFFFFF - (hyp_begin + h)); *key must be 0 on entry.
__global__ __launch_bounds__(256) void k_best_key(const int32_t *__restrict__ counts,
                                                  const int8_t *__restrict__ status, int32_t H, int64_t hyp_begin,
                                                  unsigned long long *__restrict__ key) {
    unsigned long long best = 0;
    for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < H; h += gridDim.x * blockDim.x) {
        if (status[h] > 0 && counts[h] > 0) {
            const uint64_t g = (uint64_t)(hyp_begin + h);
            const unsigned long long k =
                ((unsigned long long)(uint32_t)counts[h] << 32) | (0xFFFFFFFFull - (g & 0xFFFFFFFFull));
            best = k > best ? k : best;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long other = __shfl_xor(best, o);
        best = other > best ? other : best;
    }
    // one atomic per block: thousands of same-address atomics serialise in L2
    __shared__ unsigned long long wbest[4];
    if ((threadIdx.x & 63) == 0) wbest[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x == 0) {
        best = wbest[0];
        for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = wbest[w] > best ? wbest[w] : best;
        if (best) atomicMax(key, best);
    }
}

// the device replay of a problem's scan on its records (scan_records of rsac_host.hip): one wave,
// wave-uniform; ridx / rcnt in LDS, written before the call
__device__ __forceinline__ int64_t scan_decide(const int32_t *ridx, const int32_t *rcnt, int nrec, int first_neg, int H,
                                               int model_points, int prob, int64_t stride, const ScanDecide &dec,
                                               ScanRecords &o, int lane, bool write = true) {
    // scan_records (rsac_host.hip) on the records lane 0 just wrote.  update_num_iters'
    // logarithms (the latency) for every record at once, lane r for record r; the
    // sequential part on them is uniform across the wave.
    __builtin_amdgcn_wave_barrier();
    const int nr = nrec <= kScanRecs ? nrec : 0;
    double p = dec.confidence;
    p = p > 0. ? p : 0.; p = p < 1. ? p : 1.;
    double num = 1. - p;
    if (num < 2.2250738585072014e-308) num = 2.2250738585072014e-308;
    num = log(num);
    double ldenom = 0.;
    int zero = 0;  // update_num_iters returns 0 (denominator below DBL_MIN)
    const int32_t np = dec.offsets ? (int32_t)(dec.offsets[prob + 1] - dec.offsets[prob]) : dec.n;
    if (lane < nr) {
        double ep = (double)(np - rcnt[lane]) / np;
        ep = ep > 0. ? ep : 0.; ep = ep < 1. ? ep : 1.;
        const double denom = 1. - pow(1. - ep, model_points);
        if (denom < 2.2250738585072014e-308) zero = 1;
        else ldenom = log(denom);
    }
    int64_t niters = dec.max_iters > 1 ? dec.max_iters : 1, best = -1;
    for (int r = 0; r < nr; ++r) {
        const double ld = __shfl(ldenom, r);
        const int z = __shfl(zero, r);
        const int64_t stop = first_neg < niters ? first_neg : niters;
        if (ridx[r] >= stop) break;
        best = ridx[r];
        const int mi = (int)niters;
        niters = z ? 0 : ((ld >= 0 || -num >= mi * (-ld)) ? mi : (int)lrint(num / ld));
    }
    const int64_t stop = first_neg < niters ? first_neg : niters;
    // fixed budget: the round is the whole budget, so the replay always ends in it
    const bool done = nrec <= kScanRecs && (dec.fixed || stop < H || H >= niters);
    // not done: the speculative finish has no model (cheap no-op); the record index of problem
    // prob's winner (problem 0: the hypothesis itself)
    const int64_t pick = done && best >= 0 ? (int64_t)prob * stride + best : -1;
    if (lane == 0 && write) {
        dec.best_out[prob] = pick;
        o.dev_best = (int32_t)best;
        o.dev_done = done;
    }
    return pick;
}

// One wave's replay of a problem's scan over its round (c, st: the problem's count and status
// rows): the prefix-maximum records (ridx, rcnt in LDS, lane 0 writes; at most kScanRecs kept,
// nrec counts them all) and the first status < 0 (H if none); nrec and first_neg wave-uniform.
__device__ __forceinline__ void scan_wave(const int32_t *__restrict__ c, const int8_t *__restrict__ st, int H,
                                          int model_points, int lane, int32_t *ridx, int32_t *rcnt, int &nrec_out,
                                          int &first_neg_out) {
    int floor_c = model_points - 1;  // the scan's floor: max(s - 1, best count so far)
    int nrec = 0, first_neg = H;
    // 8 steps' loads in flight at a time (one step's round trip each was the kernel's time)
    constexpr int U = 8;
    bool stop = false;
    for (int b0 = 0; b0 < H && !stop; b0 += 64 * U) {
        int8_t svs[U];
        int32_t cvs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + 64 * u + lane;
            svs[u] = i < H ? st[i] : (int8_t)0;
            cvs[u] = i < H ? c[i] : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (stop) break;
            const int b = b0 + 64 * u, i = b + lane;
            const int8_t sv = svs[u];
            const uint64_t neg = __ballot(sv < 0);
            const int lim = neg ? b + __builtin_ctzll(neg) : H;  // hypotheses before the first status < 0
            int v = (i < lim && sv > 0) ? cvs[u] : -1;
            // candidates: above the floor; take them in order, each raising the floor
            uint64_t cand = __ballot(v > floor_c);
            while (cand) {
                const int l = __builtin_ctzll(cand);
                const int cv = __shfl(v, l);
                if (nrec < kScanRecs && lane == 0) {
                    ridx[nrec] = b + l;
                    rcnt[nrec] = cv;
                }
                ++nrec;
                floor_c = cv;
                cand = __ballot(v > floor_c && lane > l);
            }
            if (neg) {
                first_neg = lim;
                stop = true;
            }
        }
    }
    nrec_out = nrec;
    first_neg_out = first_neg;
}

// one wave per problem: 64 hypotheses per step, the running maximum carried across steps
__global__ __launch_bounds__(256) void k_scan_records(const int32_t *__restrict__ counts,
                                                      const int8_t *__restrict__ status, int64_t stride, int32_t P,
                                                      int32_t H, int model_points, ScanRecords *__restrict__ out,
                                                      ScanDecide dec) {
    // records kept in LDS and written out once: out may be pinned host memory (no copy back)
    __shared__ int32_t sidx[4][kScanRecs], scnt[4][kScanRecs];
    const int prob = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (prob >= P) return;  // wave-uniform
    const int lane = threadIdx.x & 63;
    int32_t *ridx = sidx[threadIdx.x >> 6], *rcnt = scnt[threadIdx.x >> 6];
    int nrec, first_neg;
    scan_wave(counts + (int64_t)prob * stride, status + (int64_t)prob * stride, H, model_points, lane, ridx, rcnt,
              nrec, first_neg);
    ScanRecords &o = out[prob];
    if (lane == 0) {
        o.nrec = nrec <= kScanRecs ? nrec : -1;
        o.first_neg = first_neg;
        for (int r = 0; r < nrec && r < kScanRecs; ++r) {
            o.idx[r] = ridx[r];
            o.cnt[r] = rcnt[r];
        }
    }
    if (dec.best_out && (dec.fixed || prob == 0)) {  // wave-uniform
        __builtin_amdgcn_wave_barrier();
        (void)scan_decide(ridx, rcnt, nrec, first_neg, H, model_points, prob, stride, dec, o, lane);
    }
}
// The speculative finish's scan and masks in one launch (one PnP problem, rounds below
// kScanBlockH; the kernel takes any number of problems, the host launches it for one): block
// (x, prob)'s first wave replays problem prob's scan (scan_wave + scan_decide, the operations of
// k_scan_records; block 0 writes the records and the pick), then the block masks its points for
// the pick as k_pnp_mask does, and block 0 gathers the winner's record.  Every block replays the
// scan itself (a few records), so no block waits for another (r05: one launch and its dispatch
// gap fewer on the ms-to-best path).
__global__ __launch_bounds__(256) void k_scan_mask(const int32_t *__restrict__ counts, const int8_t *__restrict__ status,
                                                   int64_t stride, int32_t H, int model_points, ScanRecords *out,
                                                   ScanDecide dec, PnpArgs a, uint8_t *__restrict__ mask,
                                                   double *__restrict__ model_out, double *__restrict__ host_model_out) {
    __shared__ int32_t ridx[kScanRecs], rcnt[kScanRecs];
    __shared__ int64_t sbest;
    const int prob = blockIdx.y;
    if (threadIdx.x < 64) {  // wave 0
        const int lane = threadIdx.x;
        int nrec, first_neg;
        scan_wave(counts + (int64_t)prob * stride, status + (int64_t)prob * stride, H, model_points, lane, ridx, rcnt,
                  nrec, first_neg);
        ScanRecords &o = out[prob];
        const bool lead = blockIdx.x == 0;
        if (lead && lane == 0) {
            o.nrec = nrec <= kScanRecs ? nrec : -1;
            o.first_neg = first_neg;
            for (int r = 0; r < nrec && r < kScanRecs; ++r) {
                o.idx[r] = ridx[r];
                o.cnt[r] = rcnt[r];
            }
        }
        __builtin_amdgcn_wave_barrier();
        const int64_t b = scan_decide(ridx, rcnt, nrec, first_neg, H, model_points, prob, stride, dec, o, lane, lead);
        if (lane == 0) sbest = b;
    }
    __syncthreads();
    pnp_mask_body(a, prob, sbest, mask, model_out, host_model_out);
}

// k_scan_records for long rounds (H >= kScanBlockH: a fixed budget of 100k hypotheses, C4): one
// 1024-thread block per problem instead of one wave stepping 64 hypotheses at a time (C4: 778 us
// for one 100k round).  Thread t owns the contiguous range [t L, t L + L): pass 1 finds its first
// status < 0 and the maximum count before it; a block min gives first_neg and an exclusive
// block prefix maximum (from the floor model_points - 1) the floor each range starts from; pass 2
// lists each range's strict prefix maxima above its floor, placed by an exclusive block prefix
// sum of the per-range counts.  The records, their order and nrec (-1 past kScanRecs) are those
// of the one-wave scan; then wave 0 replays them (scan_decide).
constexpr int kScanBlockH = 8192;
__global__ __launch_bounds__(1024) void k_scan_records_blk(const int32_t *__restrict__ counts,
                                                           const int8_t *__restrict__ status, int64_t stride,
                                                           int32_t H, int model_points, ScanRecords *__restrict__ out,
                                                           ScanDecide dec) {
    // wave w takes the contiguous segment [w S, (w + 1) S) and walks it 64 hypotheses a step,
    // lane l reading hypothesis step + l (coalesced): pass 1 its first status < 0 and the largest
    // valid count before it; pass 2, from the floor the earlier segments leave, the strict prefix
    // maxima (a step with no count above the floor costs one compare and one ballot)
    __shared__ int32_t ridx[kScanRecs], rcnt[kScanRecs];
    __shared__ int32_t widx[16][kScanRecs], wcnt[16][kScanRecs];
    __shared__ int32_t wmx[16], wng[16], wnr[16];
    const int prob = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int32_t *c = counts + (int64_t)prob * stride;
    const int8_t *st = status + (int64_t)prob * stride;
    const int S = ((H + 15) / 16 + 63) & ~63;
    const int s0 = min(H, wave * S), s1 = min(H, s0 + S);
    // pass 1 (8 steps' loads in flight at a time)
    constexpr int U = 8;
    int lneg = H, lmax = -1;
    for (int b0 = s0; b0 < s1 && lneg == H; b0 += 64 * U) {
        int8_t sv[U];
        int32_t cv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + 64 * u + lane;
            sv[u] = i < s1 ? st[i] : (int8_t)0;
            cv[u] = i < s1 ? c[i] : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (lneg != H) break;
            const unsigned long long neg = __ballot(sv[u] < 0);
            const int f = neg ? (int)__builtin_ctzll(neg) : 64;
            if (sv[u] > 0 && lane < f) lmax = max(lmax, cv[u]);
            if (neg) lneg = b0 + 64 * u + f;
        }
    }
    for (int o = 32; o > 0; o >>= 1) lmax = max(lmax, __shfl_xor(lmax, o));
    if (lane == 0) {
        wmx[wave] = lmax;
        wng[wave] = lneg;
    }
    __syncthreads();
    int first_neg = H, floor_c = model_points - 1;
#pragma unroll
    for (int w = 0; w < 16; ++w) first_neg = min(first_neg, wng[w]);
    for (int w = 0; w < wave; ++w)
        if (w * S < first_neg) floor_c = max(floor_c, wmx[w]);  // segments from the first status < 0 on take no part
    // pass 2
    const int lim = min(s1, first_neg);
    int nr = 0, f = floor_c;
    for (int b0 = s0; b0 < lim; b0 += 64 * U) {
        int32_t vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + 64 * u + lane;
            const int8_t sv = i < lim ? st[i] : (int8_t)0;
            const int32_t cv = i < lim ? c[i] : -1;
            vv[u] = sv > 0 ? cv : -1;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b0 + 64 * u + lane;
            const int32_t v = vv[u];
            if (__ballot(v > f) == 0) continue;
            int pm = v;  // inclusive prefix maximum over the step's lanes
            for (int o = 1; o < 64; o <<= 1) {
                const int up = __shfl_up(pm, o);
                if (lane >= o) pm = max(pm, up);
            }
            int ex = __shfl_up(pm, 1);
            if (lane == 0) ex = -1;
            unsigned long long rec = __ballot(v > f && v > ex);
            while (rec) {
                const int r = (int)__builtin_ctzll(rec);
                rec &= rec - 1;
                if (nr < kScanRecs && lane == r) {
                    widx[wave][nr] = i;
                    wcnt[wave][nr] = v;
                }
                ++nr;
            }
            f = max(f, __shfl(pm, 63));
        }
    }
    if (lane == 0) wnr[wave] = nr;
    __syncthreads();
    if (wave != 0) return;
    int total = 0;
    for (int w = 0; w < 16; ++w) {  // the segments' records in order
        const int nw = wnr[w];
        if (lane < nw && lane < kScanRecs && total + lane < kScanRecs) {
            ridx[total + lane] = widx[w][lane];
            rcnt[total + lane] = wcnt[w][lane];
        }
        total += nw;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    ScanRecords &o = out[prob];
    if (lane == 0) {
        o.nrec = total <= kScanRecs ? total : -1;
        o.first_neg = first_neg;
        for (int r = 0; r < total && r < kScanRecs; ++r) {
            o.idx[r] = ridx[r];
            o.cnt[r] = rcnt[r];
        }
    }
    if (dec.best_out && (dec.fixed || prob == 0)) scan_decide(ridx, rcnt, total, first_neg, H, model_points, prob,
                                                                stride, dec, o, lane);
}

// The record pass of rsac_scan_device (the multi-GPU adaptive loop's scan of a gathered round):
// one wave over rows [0, count) of {status, count} int32 pairs: the strict prefix maxima above
// floor0 (every improvement a sequential scan could make there, in order; the host applies the
// iteration bound), at most kScanRecs, and the first status < 0.  out: pinned host memory.
__global__ __launch_bounds__(64) void k_scan_rows(const int32_t *__restrict__ rows, int32_t count, int32_t floor0,
                                                  ScanRecords *__restrict__ out) {
    __shared__ int32_t ridx[kScanRecs], rcnt[kScanRecs];
    const int lane = threadIdx.x;
    int floor_c = floor0, nrec = 0, first_neg = count;
    for (int b = 0; b < count; b += 64) {
        const int i = b + lane;
        const int sv = i < count ? rows[2 * i] : 0;
        const uint64_t neg = __ballot(sv < 0);
        const int lim = neg ? b + __builtin_ctzll(neg) : count;
        const int v = (i < lim && sv > 0) ? rows[2 * i + 1] : -1;
        uint64_t cand = __ballot(v > floor_c);
        while (cand) {
            const int l = __builtin_ctzll(cand);
            const int cv = __shfl(v, l);
            if (nrec < kScanRecs && lane == 0) {
                ridx[nrec] = b + l;
                rcnt[nrec] = cv;
            }
            ++nrec;
            floor_c = cv;
            cand = __ballot(v > floor_c && lane > l);
        }
        if (neg) {
            first_neg = lim;
            break;
        }
    }
    if (lane == 0) {
        out->nrec = nrec <= kScanRecs ? nrec : -1;
        out->first_neg = first_neg;
        for (int r = 0; r < nrec && r < kScanRecs; ++r) {
            out->idx[r] = ridx[r];
            out->cnt[r] = rcnt[r];
        }
    }
}

hipError_t launch_scan_rows(const int32_t *rows, int32_t count, int32_t floor0, ScanRecords *out, hipStream_t s) {
    hipLaunchKernelGGL(k_scan_rows, dim3(1), dim3(64), 0, s, rows, count, floor0, out);
    return hipGetLastError();
}

// {status, count} rows of hypotheses [0, H) of problem 0 (the multi-GPU round's exchange format)
__global__ void k_pack_rows(const int8_t *__restrict__ status, const int32_t *__restrict__ counts, int32_t H,
                            int32_t *__restrict__ rows) {
    for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < H; h += gridDim.x * blockDim.x)
        reinterpret_cast<int2 *>(rows)[h] = make_int2((int)status[h], counts[h]);
}

hipError_t launch_pack_rows(const int8_t *status, const int32_t *counts, int32_t H, int32_t *rows, hipStream_t s) {
    unsigned g = (unsigned)((std::max(H, 1) + 255) / 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pack_rows, dim3(g), dim3(256), 0, s, status, counts, H, rows);
    return hipGetLastError();
}

hipError_t launch_scan_records(const int32_t *counts, const int8_t *status, int64_t stride, int32_t P, int32_t H,
                               int model_points, ScanRecords *out, hipStream_t s, ScanDecide dec) {
    if (H >= kScanBlockH)
        hipLaunchKernelGGL(k_scan_records_blk, dim3(P), dim3(1024), 0, s, counts, status, stride, H, model_points,
                           out, dec);
    else
        hipLaunchKernelGGL(k_scan_records, dim3((P + 3) / 4), dim3(256), 0, s, counts, status, stride, P, H,
                           model_points, out, dec);
    return hipGetLastError();
}

// model record of the key's hypothesis -> out[16] (zeros when key == 0)
__global__ void k_key_model(const double *__restrict__ models, const unsigned long long *__restrict__ key,
                            int64_t hyp_begin, double *__restrict__ out) {
    const int q = threadIdx.x;
    if (q >= kModelStride) return;
    const unsigned long long k = *key;
    if (k == 0) { out[q] = 0.0; return; }
    const uint64_t low = 0xFFFFFFFFull - (k & 0xFFFFFFFFull);
    const int64_t h = (int64_t)((low - ((uint64_t)hyp_begin & 0xFFFFFFFFull)) & 0xFFFFFFFFull);
    out[q] = q == kValidSlot ? 1.0 : models[h * kModelStride + q];  // a nonzero key: status > 0 (k_best_key)
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }
static_assert(true, "");

constexpr int kScoreP = 8;
constexpr int kScoreHB = 32;

hipError_t launch_pnp_prepare(const double *p3, const double *p2, int64_t n, float *X, float *Y, float *Z, float *U,
                              float *V, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    unsigned g = cdiv(n, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_pnp_prepare, dim3(g), dim3(256), 0, s, p3, p2, n, X, Y, Z, U, V);
    return hipGetLastError();
}

hipError_t launch_hom_prepare(const double *src, const double *dst, int64_t n, float *SX, float *SY, float *DX,
                              float *DY, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    unsigned g = cdiv(n, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_hom_prepare, dim3(g), dim3(256), 0, s, src, dst, n, SX, SY, DX, DY);
    return hipGetLastError();
}

// rounds of at most this many hypotheses (problems x hypotheses) are solved 4 lanes per
// hypothesis (k_pnp_solve_l<4>); larger ones one lane per hypothesis (k_pnp_solve)
constexpr int64_t kSolve4MaxHyps = 4096;

hipError_t launch_pnp_frame(const PnpArgs &a, int32_t P, int32_t max_n, int32_t *ws, float *XC, float *YC, float *ZC,
                            double *frame, float *fconst, hipStream_t s, const PnpPrepare *prep) {
    if (P > 1 && max_n <= kSetupBatchMaxN) {
        // a batch of short problems: conversion (when deferred), bounds, frame and centring in
        // one launch, one block per problem
        if (prep && prep->p3)
            hipLaunchKernelGGL(k_pnp_setup_b<true>, dim3(P), dim3(256), 0, s, prep->p3, prep->p2, a, P, prep->X,
                               prep->Y, prep->Z, prep->U, prep->V, ws, frame, fconst, XC, YC, ZC);
        else
            hipLaunchKernelGGL(k_pnp_setup_b<false>, dim3(P), dim3(256), 0, s, (const double *)nullptr,
                               (const double *)nullptr, a, P, (float *)nullptr, (float *)nullptr, (float *)nullptr,
                               (float *)nullptr, (float *)nullptr, ws, frame, fconst, XC, YC, ZC);
        return hipGetLastError();
    }
    if (prep && prep->p3) {  // the deferred f64 -> f32 conversion of one problem, fused
        if (P != 1 || max_n > 65536) return hipErrorInvalidValue;
        if (prep->part && prep->ticket) {
            unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
            if (g > kSetupMaxBlocks) g = kSetupMaxBlocks;
            hipLaunchKernelGGL(k_pnp_setup_fc<true>, dim3(g), dim3(256), 0, s, prep->p3, prep->p2, a, prep->X,
                               prep->Y, prep->Z, prep->U, prep->V, ws, frame, fconst, XC, YC, ZC, prep->part,
                               prep->ticket);
        } else {
            hipLaunchKernelGGL(k_pnp_setup1, dim3(1), dim3(1024), 0, s, prep->p3, prep->p2, a, prep->X, prep->Y,
                               prep->Z, prep->U, prep->V, ws, frame, fconst, XC, YC, ZC);
        }
        return hipGetLastError();
    }
    if (P == 1 && prep && prep->part && prep->ticket) {
        // one problem already in f32: bounds, frame and centring in one full-grid launch
        unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
        if (g > kSetupMaxBlocks) g = kSetupMaxBlocks;
        hipLaunchKernelGGL(k_pnp_setup_fc<false>, dim3(g), dim3(256), 0, s, (const double *)nullptr,
                           (const double *)nullptr, a, (float *)nullptr, (float *)nullptr, (float *)nullptr,
                           (float *)nullptr, (float *)nullptr, ws, frame, fconst, XC, YC, ZC, prep->part,
                           prep->ticket);
        return hipGetLastError();
    }
    if (P == 1 && max_n <= 65536) {
        // one block: no atomics, so no initialisation launch (it also resets the key and queue)
        hipLaunchKernelGGL(k_pnp_bounds1, dim3(1), dim3(1024), 0, s, a, ws);
    } else {
        hipLaunchKernelGGL(k_pnp_init, dim3(1), dim3(256), 0, s, P, ws, a.best_key, a.queue);
        unsigned g = cdiv(max_n > 0 ? max_n : 1, 2048);
        if (g > 32) g = 32;
        hipLaunchKernelGGL(k_pnp_bounds, dim3(g, P), dim3(256), 0, s, a, P, ws);
    }
    unsigned g2 = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g2 > 1024) g2 = 1024;
    hipLaunchKernelGGL(k_pnp_center, dim3(g2, P), dim3(256), 0, s, a, P, ws, frame, fconst, XC, YC, ZC);
    return hipGetLastError();
}

// a round of at most kSmallRoundTiles hypothesis tiles (an adaptive run's first 256
// hypotheses) is scored by the scaled-form small-round instance (2 points per lane, so the cells
// fill the GPU); its records are written in form 1 (the solve and the scoring launch apply the
// same rule)
constexpr int64_t kSmallRoundTiles = 16;
// ... on problems of at most this many points: longer ones (C5's 100k) give the MFMA kernel
// enough cells even for 256 hypotheses (r06: C5's first round 42.5 us on the scaled form)
constexpr int32_t kSmallRoundMaxN = 32768;

static bool small_round(int32_t P, int32_t H, int32_t max_n) {
    return (int64_t)P * ((H + 31) / 32) <= kSmallRoundTiles && max_n <= kSmallRoundMaxN;
}
static PnpArgs round_args(const PnpArgs &a, int32_t P, int32_t H) {
    PnpArgs ka = a;
    if (ka.fform == 2 && small_round(P, H, a.max_n)) ka.fform = 1;
    return ka;
}

hipError_t launch_pnp_fmodels(const PnpArgs &a, int32_t P, int32_t H, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_fmodels, dim3(cdiv(H, 256), P), dim3(256), 0, s, round_args(a, P, H), H);
    return hipGetLastError();
}

// rounds up to this many hypotheses (one lane each: <= 4 waves per SIMD) run the P3P solve on two
// lanes per hypothesis, two Lambda Twist candidates each (r06, scripts/gpu_r06_solve2.sh: the
// kernel 33.6 -> 36 us but the C2 step 0.2600 -> 0.2580 ms in three interleaved rounds, as the
// solve of one step overlaps the other stream's scoring better); larger rounds (C3) stay on one
constexpr int64_t kSolve2MaxHyps = 262144;

bool pnp_setup_fusable(const PnpArgs &a, int32_t H) {
    return a.sample_k == 4 && a.fmodels && !a.exact_only && H <= kSolve4MaxHyps && a.max_n > kLanePts &&
           small_round(1, H, a.max_n);
}

hipError_t launch_pnp_solve(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s,
                            const PnpSetupFuse *fuse) {
    PnpArgs ka = round_args(a, P, H);
    if (a.sample_k == 5) {  // EPnP-5 in OpenCV's sequence: k_cvepnp5_a / _svd / _c
        if (!a.epnp) return hipErrorInvalidValue;  // its scratch (ensure_epnp5) is required
        // short rounds (an adaptive run's first 256 hypotheses): their latency is one hypothesis',
        // so one wave per block in stages 1 and 3
        const bool short_round = (int64_t)P * H <= 2048;
        const int tb = short_round ? 64 : 256;
        hipLaunchKernelGGL(k_cvepnp5_a, dim3(cdiv(H, tb), P), dim3(tb), 0, s, ka, hyp_begin, H);
        hipLaunchKernelGGL(k_cvepnp5_svd, dim3(cdiv(cdiv(H, kSvdHpw), tb / 64), P), dim3(tb),
                           (tb / 64) * kSvdHpw * kSvdStride * sizeof(double), s, ka, hyp_begin, H);
        const int hpw = 21;  // hypotheses per wave of stage 3 (3 lanes each)
        hipLaunchKernelGGL(k_cvepnp5_c, dim3(cdiv(cdiv(H, hpw), tb / 64), P), dim3(tb), 0, s, ka, hyp_begin, H, hpw);
    }
    // one problem's deferred set-up beside the 4-lane solve (the round's scorer builds the records)
    else if (fuse) {
        const PnpPrepare &pr = fuse->prep;
        if (P != 1 || H > kSolve4MaxHyps || !pr.p3 || !pr.part || !pr.ticket || fuse->max_n > 65536)
            return hipErrorInvalidValue;
        unsigned gs = cdiv(fuse->max_n > 0 ? fuse->max_n : 1, 256);
        if (gs > kSetupMaxBlocks) gs = kSetupMaxBlocks;
        hipLaunchKernelGGL(k_pnp_setup_solve4, dim3(gs + cdiv(4 * (int64_t)H, 256)), dim3(256), 0, s, pr.p3, pr.p2,
                           ka, pr.X, pr.Y, pr.Z, pr.U, pr.V, fuse->ws, fuse->frame, fuse->fconst, pr.part, pr.ticket,
                           (int)gs, hyp_begin, H);
    }
    // a few waves of hypotheses in all: their latency is the launch's, so spread each over 4 lanes
    else if ((int64_t)P * H <= kSolve4MaxHyps)
        hipLaunchKernelGGL(k_pnp_solve_l<4>, dim3(cdiv(4 * (int64_t)H, 256), P), dim3(256), 0, s, ka, hyp_begin, H);
    else if ((int64_t)P * H <= kSolve2MaxHyps)
        hipLaunchKernelGGL(k_pnp_solve_l<2>, dim3(cdiv(2 * (int64_t)H, 256), P), dim3(256), 0, s, ka, hyp_begin, H);
    else
        hipLaunchKernelGGL(k_pnp_solve, dim3(cdiv(H, 256), P), dim3(256), 0, s, ka, hyp_begin, H);
    return hipGetLastError();
}

// blocks of `kern` (`threads` threads) the whole GPU keeps resident
template <class Kern>
static int resident_blocks(Kern kern, int threads = 256) {
    int dev = 0, cus = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, 0);
    return std::max(1, cus) * std::max(1, per_cu);
}

// grid of a split-queue launch (block b takes the units = b mod kQSub): enough blocks for every
// residue class that has units, else at most the resident blocks
static unsigned queue_grid(int64_t units, int resident) {
    const int64_t g = std::max<int64_t>(std::min<int64_t>(units, resident), std::min<int64_t>(units, kQSub));
    return (unsigned)std::max<int64_t>(1, g);
}

// the cell units add their counts atomically onto these zeros: a failed memset must fail the launch
static hipError_t zero_counts(int32_t *counts, int64_t hyp_begin, int32_t H, int32_t P, int64_t stride,
                              hipStream_t s) {
    if (P == 1) return hipMemsetAsync(counts + hyp_begin, 0, sizeof(int32_t) * H, s);
    return hipMemset2DAsync(counts + hyp_begin, sizeof(int32_t) * stride, 0, sizeof(int32_t) * H, P, s);
}

static void launch_best_key_of(const PnpArgs &a, int64_t hyp_begin, int32_t H, const int32_t *counts, hipStream_t s) {
    unsigned g = cdiv(H, 1024);
    if (g > 128) g = 128;
    hipLaunchKernelGGL(k_best_key, dim3(g), dim3(256), 0, s, counts + hyp_begin, a.status + hyp_begin, H,
                       a.rng_base + hyp_begin, a.best_key);
}

hipError_t launch_pnp_best_key(const PnpArgs &a, int64_t hyp_begin, int32_t H, const int32_t *counts, hipStream_t s) {
    if (a.best_key) launch_best_key_of(a, hyp_begin, H, counts, s);
    return hipGetLastError();
}

// k_pnp_score_sc (small rounds, form-1 records): whole-tile units for all but the last
// `resident` tiles, which go as one unit per cell (64 x 4 x P points): the cells even out the
// blocks' finishing times.  Counts are zeroed (by the solve kernel, else here) and added
// atomically; the best key is reduced afterwards.
template <int P, int W>
static hipError_t launch_sc(const PnpArgs &a, int32_t P_, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    auto kern = k_pnp_score_sc<P, 32, W>;
    static const int resident = resident_blocks(kern);
    const int64_t cells = std::max<int64_t>(1, ((int64_t)a.max_n + 256 * P - 1) / (256 * P));
    const int64_t tiles = (int64_t)P_ * ((H + 31) / 32);
    const int64_t cell_tiles = std::min<int64_t>(tiles, resident);
    const int64_t tb = tiles - cell_tiles;
    const int64_t units = tb + cell_tiles * cells;
    if (a.counts_out != counts) {
        const hipError_t e = zero_counts(counts, hyp_begin, H, P_, a.hyp_stride, s);
        if (e != hipSuccess) return e;
    }
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(units, resident));
    PnpArgs ka = a;
    ka.best_key = nullptr;  // reduced below from the complete counts
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, ka, hyp_begin, H, P_, a.queue, counts, (int)tb,
                       (int)cells);
    if (a.best_key) launch_best_key_of(a, hyp_begin, H, counts, s);
    return hipGetLastError();
}

// k_pnp_score_mf: whole-tile units, then one unit per cell for the last `resident` tiles (as
// launch_sc); cells of 2048 points, halved (down to 256, one iteration per wave) while the units
// would not fill the resident grid (an adaptive run's first rounds).  A wave lists at most kWrec
// flagged iterations per unit, so problems longer than 256 kWrec points run every tile by cells
// (of up to that length; shorter while the units would not give each resident block four).
// Returns hipErrorInvalidValue only for launches past the int32 unit space.
// Batches of short problems (more than one problem, every one of at most kMfShortN points) run the
// 2-wave instance.
constexpr int64_t kMfShortN = 4096;
template <int W>
static hipError_t launch_mf_w(const PnpArgs &a, int32_t P_, int64_t hyp_begin, int32_t H, int32_t *counts,
                              hipStream_t s) {
    constexpr int kMfT = 64 * W;
    static const int resident = resident_blocks(k_pnp_score_mf<W>, kMfT);
    if (a.counts_out != counts) {
        const hipError_t e = zero_counts(counts, hyp_begin, H, P_, a.hyp_stride, s);
        if (e != hipSuccess) return e;
    }
    const int64_t max_n = std::max<int64_t>(1, a.max_n);
    const int64_t tiles = (int64_t)P_ * ((H + 31) / 32);
    int64_t cell_pts = 2048;
    while (cell_pts > 256 && tiles * ((max_n + cell_pts - 1) / cell_pts) < resident) cell_pts /= 2;
    int64_t cell_tiles = std::min<int64_t>(tiles, resident);
    constexpr int64_t win_pts = (int64_t)kMfT * kWrec;
    if (max_n > win_pts) {
        int64_t cp = win_pts;
        while (cp > cell_pts && tiles * ((max_n + cp - 1) / cp) < 4 * resident) cp /= 2;
        cell_pts = cp;
        cell_tiles = tiles;
    }
    if (a.dbg_cell_pts > 0) {  // test hook: every tile by cells of dbg_cell_pts points (a multiple of 256)
        cell_pts = std::min<int64_t>(std::max<int64_t>(256, a.dbg_cell_pts / 256 * 256), win_pts);
        cell_tiles = tiles;
    }
    const int64_t cells = (max_n + cell_pts - 1) / cell_pts;
    const int64_t tb = tiles - cell_tiles;
    const int64_t units = tb + cell_tiles * cells;
    if (units + kQSub * (int64_t)resident > INT32_MAX || tiles * 32 > INT32_MAX) return hipErrorInvalidValue;
    PnpArgs ka = a;
    ka.best_key = nullptr;  // reduced below from the complete counts
    hipLaunchKernelGGL(k_pnp_score_mf<W>, dim3(queue_grid(units, resident)), dim3(kMfT), 0, s, ka, hyp_begin, H,
                       P_, a.queue, counts, (int)tb, (int)cells, (int)cell_pts);
    if (a.best_key) launch_best_key_of(a, hyp_begin, H, counts, s);
    return hipGetLastError();
}
static hipError_t launch_mf(const PnpArgs &a, int32_t P_, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    if (P_ > 1 && a.max_n <= kMfShortN) return launch_mf_w<kMfShortW>(a, P_, hyp_begin, H, counts, s);
    return launch_mf_w<kMfW>(a, P_, hyp_begin, H, counts, s);
}

hipError_t launch_pnp_score(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    if (a.max_n > 0 && a.max_n <= kLanePts) {
        hipLaunchKernelGGL(k_pnp_score_lane, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H, counts);
    } else if (a.fmodels && !a.exact_only) {
        if (small_round(P, H, a.max_n)) {  // form-1 records (round_args): the small-round instance
            return launch_sc<2, 5>(a, P, hyp_begin, H, counts, s);
        }
        return launch_mf(a, P, hyp_begin, H, counts, s);
    } else
        hipLaunchKernelGGL((k_pnp_score<kScoreP, kScoreHB>), dim3(cdiv(H, kScoreHB), P), dim3(256), 0, s, a,
                           hyp_begin, H, counts);
    return hipGetLastError();
}

bool scan_mask_fusable(int32_t H) { return H < kScanBlockH; }
hipError_t launch_scan_mask(const ScanFuse &f, const PnpArgs &a, int32_t P, int32_t max_n, uint8_t *mask,
                            double *model_out, double *host_model_out, hipStream_t s) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_scan_mask, dim3(g, P), dim3(256), 0, s, f.counts, f.status, f.stride, f.H, f.model_points,
                       f.out, f.dec, a, mask, model_out, host_model_out);
    return hipGetLastError();
}
hipError_t launch_pnp_mask(const PnpArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s, int64_t best0, double *model_out, double *host_model_out) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pnp_mask, dim3(g, P), dim3(256), 0, s, a, best, best0, mask, model_out, host_model_out);
    return hipGetLastError();
}

hipError_t launch_hom_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s) {
    hipLaunchKernelGGL(k_hom_solve, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H);
    return hipGetLastError();
}

hipError_t launch_hom_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    if (a.max_n > 0 && a.max_n <= kLanePts)
        hipLaunchKernelGGL(k_hom_score_lane, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H, counts);
    else
        hipLaunchKernelGGL((k_hom_score<kScoreP, kScoreHB>), dim3(cdiv(H, kScoreHB), P), dim3(256), 0, s, a, hyp_begin,
                           H, counts);
    return hipGetLastError();
}

hipError_t launch_hom_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s, int64_t best0) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_hom_mask, dim3(g, P), dim3(256), 0, s, a, best, best0, mask);
    return hipGetLastError();
}

hipError_t launch_direct_finish(const double *rec4, const double *rec5, const int8_t *st4, const int8_t *st5,
                                const int8_t *kind, const int64_t *offsets, int32_t P, double *out, double *host_out,
                                uint8_t *mask, hipStream_t s) {
    hipLaunchKernelGGL(k_direct_finish, dim3(P), dim3(64), 0, s, rec4, rec5, st4, st5, kind, offsets, out, host_out,
                       mask);
    return hipGetLastError();
}

hipError_t launch_gather_models(const double *models, const int64_t *rec, int32_t P, double *out, hipStream_t s,
                                int64_t rec0) {
    hipLaunchKernelGGL(k_gather_models, dim3(cdiv((int64_t)P * kModelStride, 256)), dim3(256), 0, s, models, rec, rec0, P,
                       out);
    return hipGetLastError();
}

// (ok, n_inliers, R 9, t 3) per problem from the winners' records (device) and the host's final
// scan (pinned, read over the bus): the C3 problem-shard rows, handed to the all-gather on the
// device (rsac_pnp_ransac_batched_rows)
__global__ void k_pnp_rows(const int64_t *__restrict__ info, const double *__restrict__ models, int32_t P,
                           double *__restrict__ rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * 14) return;
    const int p = i / 14, q = i % 14;
    const bool ok = info[2 * p] >= 0;
    double v = 0.0;
    if (q == 0) v = ok ? 1.0 : 0.0;
    else if (q == 1) v = ok ? (double)info[2 * p + 1] : 0.0;
    else if (ok) v = models[(int64_t)p * kModelStride + (q - 2)];
    rows[i] = v;
}

hipError_t launch_pnp_rows(const int64_t *info, const double *models, int32_t P, double *rows, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_rows, dim3(cdiv((int64_t)P * 14, 256)), dim3(256), 0, s, info, models, P, rows);
    return hipGetLastError();
}

hipError_t launch_pnp_mask_key(const PnpArgs &a, int32_t n, const unsigned long long *key, uint8_t *mask,
                               hipStream_t s) {
    unsigned g = cdiv(n > 0 ? n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pnp_mask_key, dim3(g), dim3(256), 0, s, a, n, key, mask);
    return hipGetLastError();
}

hipError_t launch_pnp_key_finish(const PnpArgs &a, int32_t n, const unsigned long long *key, uint8_t *mask,
                                 double *rec16, double *model12, int64_t *key_out, hipStream_t s) {
    unsigned g = mask ? cdiv(n > 0 ? n : 1, 256) : 1;
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pnp_key_finish, dim3(g), dim3(256), 0, s, a, n, key, mask, rec16, model12, key_out);
    return hipGetLastError();
}

hipError_t launch_key_model(const double *models, const unsigned long long *key, int64_t rng_base, double *out,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_key_model, dim3(1), dim3(64), 0, s, models, key, rng_base, out);
    return hipGetLastError();
}

hipError_t launch_best_key(const int32_t *counts, const int8_t *status, int32_t H, int64_t hyp_begin,
                           unsigned long long *key, const double *models, double *model_out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(key, 0, sizeof(unsigned long long), s);
    if (e != hipSuccess) return e;
    unsigned g = cdiv(H, 1024);
    if (g > 128) g = 128;
    hipLaunchKernelGGL(k_best_key, dim3(g), dim3(256), 0, s, counts, status, H, hyp_begin, key);
    hipLaunchKernelGGL(k_key_model, dim3(1), dim3(64), 0, s, models, key, hyp_begin, model_out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Camera-location search (find_homographies / find_homography, main_v1.py:254-348)
// ---------------------------------------------------------------------------
// pos2 of every (location l, noted feature i): p = pos3d_i - loc_l, reordered
// (p2, p1, p0) and divided by p0 (main_v1.py:305-308), f64 as numpy; dst = the
// feature's pixel.  Output AoS, problem l = rows [l n, (l + 1) n).
__global__ void k_loc_pos2(const double *__restrict__ p3, const double *__restrict__ px, int32_t n,
                           const double *__restrict__ locs, int32_t L, double *__restrict__ src,
                           double *__restrict__ dst) {
    const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (k >= (int64_t)L * n) return;
    const int l = (int)(k / n), i = (int)(k % n);
    const double d0 = p3[3 * i] - locs[3 * l];
    const double d1 = p3[3 * i + 1] - locs[3 * l + 1];
    const double d2 = p3[3 * i + 2] - locs[3 * l + 2];
    src[2 * k] = d2 / d0;
    src[2 * k + 1] = d1 / d0;
    dst[2 * k] = px[2 * i];
    dst[2 * k + 1] = px[2 * i + 1];
}

// 3x3 inverse by the adjugate (numpy.linalg.inv's LU differs only by rounding)
__device__ __forceinline__ void inv3(const double *A, double *B) {
    const double c0 = A[4] * A[8] - A[5] * A[7];
    const double c1 = A[5] * A[6] - A[3] * A[8];
    const double c2 = A[3] * A[7] - A[4] * A[6];
    const double id = 1.0 / (A[0] * c0 + A[1] * c1 + A[2] * c2);
    B[0] = c0 * id; B[1] = (A[2] * A[7] - A[1] * A[8]) * id; B[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    B[3] = c1 * id; B[4] = (A[0] * A[8] - A[2] * A[6]) * id; B[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    B[6] = c2 * id; B[7] = (A[1] * A[6] - A[0] * A[7]) * id; B[8] = (A[0] * A[4] - A[1] * A[3]) * id;
}

__device__ __forceinline__ double proj_dist(const double *A, double x, double y, double u, double v) {
    const double w = A[6] * x + A[7] * y + A[8];
    const double px = (A[0] * x + A[1] * y + A[2]) / w, py = (A[3] * x + A[4] * y + A[5]) / w;
    return sqrt((u - px) * (u - px) + (v - py) * (v - py));
}

// One wave per location.  With H = findHomography's result and M = inv(H) (main_v1.py:314):
//   err1 = sum_{mask} |p1 - dehom(inv(M) pos2)|     (main_v1.py:333-347)
//   err2 = sum_{mask} |pos2 - dehom(M p1)| + (#not mask) * thr   (main_v1.py:347, 419)
// Locations without a model get (0, 0), which the driver maps to 1e6 (main_v1.py:864).
__global__ __launch_bounds__(64) void k_loc_score(const double *__restrict__ src, const double *__restrict__ dst,
                                                  const uint8_t *__restrict__ mask, const double *__restrict__ H,
                                                  const int32_t *__restrict__ ok, int32_t n, double thr,
                                                  double *__restrict__ err) {
    const int l = blockIdx.x, lane = threadIdx.x;
    if (!ok[l]) {
        if (lane == 0) err[2 * l] = err[2 * l + 1] = 0.0;
        return;
    }
    double M[9], Mi[9];
    inv3(H + 9 * l, M);
    inv3(M, Mi);
    double e1 = 0.0, e2 = 0.0;
    int nout = 0;
    for (int i = lane; i < n; i += 64) {
        const int64_t k = (int64_t)l * n + i;
        const double sx = src[2 * k], sy = src[2 * k + 1], u = dst[2 * k], v = dst[2 * k + 1];
        if (mask[k]) {
            e1 += proj_dist(Mi, sx, sy, u, v);
            e2 += proj_dist(M, u, v, sx, sy);
        } else {
            ++nout;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        e1 += __shfl_xor(e1, o);
        e2 += __shfl_xor(e2, o);
        nout += __shfl_xor(nout, o);
    }
    if (lane == 0) {
        err[2 * l] = e1;
        err[2 * l + 1] = e2 + (double)nout * thr;
    }
}

hipError_t launch_loc_pos2(const double *p3, const double *px, int32_t n, const double *locs, int32_t L, double *src,
                           double *dst, hipStream_t s) {
    const int64_t total = (int64_t)L * n;
    hipLaunchKernelGGL(k_loc_pos2, dim3(cdiv(total > 0 ? total : 1, 256)), dim3(256), 0, s, p3, px, n, locs, L, src,
                       dst);
    return hipGetLastError();
}

hipError_t launch_loc_score(const double *src, const double *dst, const uint8_t *mask, const double *H,
                            const int32_t *ok, int32_t L, int32_t n, double thr, double *err, hipStream_t s) {
    hipLaunchKernelGGL(k_loc_score, dim3(L), dim3(64), 0, s, src, dst, mask, H, ok, n, thr, err);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Final pose refit of every problem's winner on its RANSAC inliers (LM of
// rsac_math.h, the final solvePnP step), one block per problem.  The block's
// reductions use the summation order the host (rsac_pnp_refine) and the oracle
// mirror, so the refined pose is bit-identical on every backend.
// ---------------------------------------------------------------------------
constexpr int kLmRed = kLmTerms + 1;  // widest LM reduction: normal equations + cost

// LDS of k_pnp_refine: the staged points (SoA, [5][kLmStage]), then, multi-range only, the nb
// range sums of a reduction ([range][kLmRed]).  Ranges are one of up to 4096 points, else
// ~1024 points (lm_blocks / lm_chunk of rsac_math.h: lm_chunk(n) <= kLmStage for every
// n <= kLmMaxBlocks * kLmStage = 262144, checked in tests/test_abi.py).  A block stages the
// masked points of all the ranges it owns once per refit when their indices fit one tile
// (always, when it owns one range and n <= 262144); otherwise every pass re-stages each range
// tile by tile in the same order.
constexpr int kLmStage = 8 * kLmThreads;
constexpr int kLmLdsBytes = 5 * kLmStage * 4 + kLmMaxBlocks * kLmRed * 8;
static_assert(kLmBlockPoints <= kLmStage, "a range of ~1024 points fits one tile");
static_assert(kLmOneBlock <= kLmStage, "a one-range problem of up to 4096 points fits one tile");
static_assert(kLmMaxBlocks * kLmRed * 2 <= 8 * kLmThreads, "one sweep pass covers every granule");

typedef __attribute__((address_space(1))) unsigned long long lm_gu64;
constexpr unsigned kLmSpinLimit = 1u << 20;  // ~1 s of polls: a range whose sums never arrive ends the waits

struct GpuLmReducer {
    static constexpr bool kFused = true;  // cost_normal: one pass for a candidate (rsac_math.h)
    const float *X, *Y, *Z, *U, *V;
    const uint8_t *mask;
    int n;
    Cam k;
    double c0, c1, c2;  // centre of the refit frame
    double (*wsum)[kLmRed];  // LDS [kLmThreads / 64][kLmRed]
    // the nb ranges of the block-compacted order (rsac_math.h).  The problem's G blocks share
    // them: block x owns ranges x, x + G, x + 2G, ... (G = nb unless the device cannot hold nb
    // blocks at once; launch_pnp_refine).  Every reduction yields one sum per range and term;
    // with G > 1 they are handed over as data-tagged granules (gran, below), no barrier
    int nb = 1;
    int first = 0, G = 1, nown = 1;  // this block's first range, the range stride, ranges owned
    float *stage = nullptr;  // LDS [5][cap]: compacted X Y Z U V of the owned ranges
    int cap = kLmStage;
    int *scan = nullptr;     // LDS [kLmThreads / 64]: wave totals
    int *rbase = nullptr;    // LDS [kLmMaxBlocks]: owned range k's staged points start at stage[rbase[k]] ...
    int *rcnt = nullptr;     // LDS [kLmMaxBlocks]: ... and number rcnt[k]
    int staged = -1;         // masked points staged once for the whole refit; -1: re-staged per pass
    // multi-block hand-off (cdna_hip_programming.md Guideline 16, R2): range r's sum of term q
    // goes out as two 8-byte {tag, 32-bit half} granules, stored sc1 by thread q of the owning
    // block; every block sweeps all nb * nv * 2 granules with sc1 loads until each carries this
    // reduction's tag (launch tag | reduction index: unique per launch, the host zeroes the
    // granules on wrap), into LDS (wsums), and sums them left to right.  Two alternating granule
    // buffers: a block overwrites buffer k % 2 only after every block has stored reduction
    // k - 1, i.e. finished reading reduction k - 2.
    lm_gu64 *gran = nullptr;  // [2][kLmMaxBlocks][kLmRed][2]
    unsigned tag_base = 0;
    int phase = 0;
    double *wsums = nullptr;  // LDS [kLmMaxBlocks][kLmRed]: the ranges' sums
    // block-uniform: a reduction's sums never all arrived (a block that was never resident);
    // the remaining reductions return NaN without waiting and the kernel reports the failure
    bool broken = false;
    double (*accs)[kLmRed] = nullptr;  // LDS [2][kLmRed]: pnp_lm_refine's normal equations
    double *res = nullptr;             // LDS [1]: a cost reduction's result
    __device__ double *acc_buf(int k) { return accs[k]; }
    // the LM step's solve (Cholesky, Cayley map, step test: ~300 dependent f64 operations) runs
    // on wave 0 alone, not on the 8 waves two to a SIMD; the block reads the candidate from
    // LDS.  Two alternating buffers: wave 0 writes buffer k + 1 while the others may still read k.
    static constexpr bool kSolveStep = true;
    double (*steps)[16] = nullptr;  // LDS [2][16]: Rn[9], tn[3], ok, small
    int nstep = 0;
    __device__ bool solve_step(const double *acc, double lam, const double *R, const double *t, double *Rn,
                               double *tn, bool &small) {
        double *sb = steps[nstep++ & 1];
        if (threadIdx.x < 64) {
            double r[9], u[3];
            bool sm = false, bad = false;
            // the fast cores' form; an operand outside their range redoes the step in IEEE form
            // (the same bits; the values are wave-uniform, so is the branch)
            bool ok = lm_solve_step_t<RSAC_FAST_F64 != 0>(acc, lam, R, t, r, u, sm, bad);
            if (bad) ok = lm_solve_step(acc, lam, R, t, r, u, sm);
            if (threadIdx.x == 0) {
                for (int j = 0; j < 9; ++j) sb[j] = r[j];
                for (int j = 0; j < 3; ++j) sb[9 + j] = u[j];
                sb[12] = ok ? 1.0 : 0.0;
                sb[13] = sm ? 1.0 : 0.0;
            }
        }
        __syncthreads();
        for (int j = 0; j < 9; ++j) Rn[j] = sb[j];
        for (int j = 0; j < 3; ++j) tn[j] = sb[9 + j];
        small = sb[13] != 0.0;
        return sb[12] != 0.0;
    }

    __device__ void range_of(int r, int &lo, int &hi) const {
        const int C = lm_chunk(n);
        lo = r * C;
        hi = (int)min((int64_t)n, (int64_t)lo + C);
    }

    // the masked points of [tlo, thi) (at most cap - base indices), ascending, into
    // stage[.][base, base + cnt); returns cnt (block-uniform).  Thread t covers indices
    // tlo + (cap / 512) t, ...
    __device__ int stage_tile(int tlo, int thi, int base) {
        const int per = cap / kLmThreads;  // 8 or 4
        const int first_i = tlo + per * (int)threadIdx.x;
        unsigned bits = 0;
        for (int j = 0; j < per; ++j)
            if (first_i + j < thi && mask[first_i + j]) bits |= 1u << j;
        const int cnt = __popc(bits);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        int incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        __syncthreads();  // the previous tile's readers are done with stage and scan
        if (lane == 63) scan[wave] = incl;
        __syncthreads();
        int pos = base + incl - cnt, tot = 0;
        for (int w = 0; w < kLmThreads / 64; ++w) {
            const int v = scan[w];
            pos += w < wave ? v : 0;
            tot += v;
        }
        for (int j = 0; j < per; ++j)
            if (bits >> j & 1u) {
                const int i = first_i + j;
                stage[pos] = X[i];
                stage[cap + pos] = Y[i];
                stage[2 * cap + pos] = Z[i];
                stage[3 * cap + pos] = U[i];
                stage[4 * cap + pos] = V[i];
                ++pos;
            }
        __syncthreads();
        return tot;
    }
    // block b0 of a problem whose ranges are shared by `stride` blocks
    __device__ void set_ranges(int b0, int stride) {
        first = b0;
        G = stride;
        nown = (nb - b0 + G - 1) / G;
        int span = 0;
        for (int r = b0; r < nb; r += G) {
            int lo, hi;
            range_of(r, lo, hi);
            span += hi - lo;
        }
        if (span > cap) return;  // staged = -1: tiles per pass
        int base = 0;
        for (int kk = 0, r = b0; r < nb; r += G, ++kk) {
            int lo, hi;
            range_of(r, lo, hi);
            const int cnt = stage_tile(lo, hi, base);
            if (threadIdx.x == 0) {
                rbase[kk] = base;
                rcnt[kk] = cnt;
            }
            base += cnt;
        }
        __syncthreads();
        staged = base;
    }
    // f(Xd, Yd, Zd, u, v) over this thread's points of owned range kk: the range's masked
    // points p = thread, thread + 512, ... of the compacted order
    template <class F>
    __device__ void for_points(int kk, F f) {
        auto point = [&](int q) {
            f((double)stage[q] - c0, (double)stage[cap + q] - c1, (double)stage[2 * cap + q] - c2,
              (double)stage[3 * cap + q], (double)stage[4 * cap + q]);
        };
        if (staged >= 0) {
            const int b = rbase[kk], cnt = rcnt[kk];
            for (int q = threadIdx.x; q < cnt; q += kLmThreads) point(b + q);
            return;
        }
        int lo, hi;
        range_of(first + kk * G, lo, hi);
        int p0 = 0;  // compacted position of the tile's first point
        for (int tlo = lo; tlo < hi; tlo += cap) {
            const int cnt = stage_tile(tlo, min(hi, tlo + cap), 0);
            for (int q = ((int)threadIdx.x - p0 % kLmThreads + kLmThreads) % kLmThreads; q < cnt; q += kLmThreads)
                point(q);
            p0 += cnt;
        }
    }

    // a + (the value of lane l + o): lane l < o gets the pair (l, l ^ o) of the xor butterfly,
    // so after o = 32, 16, ..., 1 lane 0 holds the butterfly's sum bit for bit (only lane 0's
    // sum is used).  o = 32 / 16 cross rows: v_permlane32_swap / v_permlane16_swap; o <= 8 stay
    // in a row of 16: DPP row_shl.  No LDS traffic (ds_bpermute was ~5 us for 27 terms).
    template <int O>
    __device__ static double add_down(double a) {
        const int lo = __double2loint(a), hi = __double2hiint(a);
        int dlo, dhi;
        if constexpr (O == 32) {
            dlo = __builtin_amdgcn_permlane32_swap(lo, lo, false, false)[1];
            dhi = __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[1];
        } else if constexpr (O == 16) {
            dlo = __builtin_amdgcn_permlane16_swap(lo, lo, false, false)[1];
            dhi = __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[1];
        } else {
            dlo = __builtin_amdgcn_update_dpp(0, lo, 0x100 + O, 0xf, 0xf, false);  // row_shl:O
            dhi = __builtin_amdgcn_update_dpp(0, hi, 0x100 + O, 0xf, 0xf, false);
        }
        return a + __hiloint2double(dhi, dlo);
    }

    // x + y of lanes l and l ^ O in the halves a reduce-scatter keeps (O = 32, 16): lanes with bit O
    // clear keep x's pair, the others y's; v_permlane{32,16}_swap moves each half to the lane that
    // adds it, and the sum is the xor butterfly's (own + partner on the lower lane; the upper lane's
    // y[l - O] + y[l] is the lower lane's own + partner)
    template <int O>
    __device__ static double add_swap(double x, double y) {
        const int xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
        int nxl, nxh, nyl, nyh;
        if constexpr (O == 32) {
            const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
            const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
            nxl = l[0]; nyl = l[1]; nxh = h[0]; nyh = h[1];
        } else {
            const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
            const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
            nxl = l[0]; nyl = l[1]; nxh = h[0]; nyh = h[1];
        }
        return __hiloint2double(nxh, nxl) + __hiloint2double(nyh, nyl);
    }

    // the range sum of every term of a[0, NV): the wave trees, then the 8 wave sums left to
    // right; the result is valid in thread q < NV (returns 0 elsewhere)
    template <int NV>
    __device__ double range_sum(double *a) {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        if constexpr (NV == 28) {
            // the fused cost + normal equations: the same butterfly as a reduce-scatter.  Level 32
            // pairs term q with q + 14, level 16 pairs q with q + 7 (add_swap), so a lane adds 14
            // then 7 terms instead of 28 twice; levels 8 .. 1 as below on the 7 left.  Every lane
            // pair holds one value (a + b == b + a), so each term gets the butterfly's bits; term
            // 7 r + j ends in c[j] of lane 16 r.  (r05: 21 adds and 42 swaps where the plain trees
            // spent 56 adds and 112 cross-lane moves on the first two levels)
            double b[14], c[7];
#pragma unroll
            for (int q = 0; q < 14; ++q) b[q] = add_swap<32>(a[q], a[q + 14]);
#pragma unroll
            for (int q = 0; q < 7; ++q) c[q] = add_swap<16>(b[q], b[q + 7]);
#pragma unroll
            for (int q = 0; q < 7; ++q) c[q] = add_down<8>(c[q]);
#pragma unroll
            for (int q = 0; q < 7; ++q) c[q] = add_down<4>(c[q]);
#pragma unroll
            for (int q = 0; q < 7; ++q) c[q] = add_down<2>(c[q]);
#pragma unroll
            for (int q = 0; q < 7; ++q) c[q] = add_down<1>(c[q]);
#ifdef RSAC_TRACE
            mark(21);
#endif
            if ((lane & 15) == 0)
#pragma unroll
                for (int j = 0; j < 7; ++j) wsum[wave][7 * (lane >> 4) + j] = c[j];
        } else {
            // levels outside, terms inside: the NV reductions are independent and overlap
            for (int q = 0; q < NV; ++q) a[q] = add_down<32>(a[q]);
            for (int q = 0; q < NV; ++q) a[q] = add_down<16>(a[q]);
            for (int q = 0; q < NV; ++q) a[q] = add_down<8>(a[q]);
            for (int q = 0; q < NV; ++q) a[q] = add_down<4>(a[q]);
            for (int q = 0; q < NV; ++q) a[q] = add_down<2>(a[q]);
            for (int q = 0; q < NV; ++q) a[q] = add_down<1>(a[q]);
#ifdef RSAC_TRACE
            mark(21);
#endif
            if (lane == 0)
                for (int q = 0; q < NV; ++q) wsum[wave][q] = a[q];
        }
        const int nv = NV;
        __syncthreads();
        double bsum = 0.0;
        if (threadIdx.x < nv) {
            const int q = threadIdx.x;
            bsum = wsum[0][q];
            for (int w = 1; w < kLmThreads / 64; ++w) bsum = bsum + wsum[w][q];
        }
        return bsum;
    }

    // sums f's terms a[0, NV) over the masked points in the order of rsac_math.h into
    // out[0, NV) (LDS, written by threads q < NV; complete when this returns)
    template <int NV, class F>
    __device__ void sum_terms(F f, double *out) {
        if (nb > 1 && G > 1) ++phase;
        const unsigned long long tag = (unsigned long long)(tag_base | (unsigned)phase) << 32;
        lm_gu64 *g = gran + (size_t)(phase & 1) * kLmMaxBlocks * kLmRed * 2;
        for (int kk = 0; kk < nown; ++kk) {
            double a[NV];
            for (int q = 0; q < NV; ++q) a[q] = 0.0;
            for_points(kk, [&](double Xd, double Yd, double Zd, double u, double v) { f(Xd, Yd, Zd, u, v, a); });
#ifdef RSAC_TRACE
            mark(20);
#endif
            const double bsum = range_sum<NV>(a);
            const int r = first + kk * G;
            if (threadIdx.x < NV) {
                const int q = threadIdx.x;
                if (nb == 1) {
                    out[q] = bsum;
                } else if (G == 1) {
                    wsums[r * kLmRed + q] = bsum;  // every range in this block: straight to LDS
                } else {  // thread q (wave 0) publishes range r's term q
                    lm_gu64 *gw = g + ((size_t)r * kLmRed + q) * 2;
                    __hip_atomic_store(gw, tag | (unsigned)__double2loint(bsum), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(gw + 1, tag | (unsigned)__double2hiint(bsum), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (kk + 1 < nown) __syncthreads();  // this range's readers of wsum are done
        }
        if (nb == 1) {
            __syncthreads();  // out is complete; wsum is free for the next reduction
            return;
        }
#ifdef RSAC_TRACE
        mark(22);
#endif
        if (G > 1) {
            // sweep: granule j = (range b, term q, half h), j = (b NV + q) 2 + h, at most 8 per
            // thread (64 ranges x 28 terms x 2 = 3584 <= 8 x 512), all in flight; a pass re-reads
            // the ones whose tag is not yet this reduction's
            const int tot = nb * NV * 2;
            unsigned *ws32 = (unsigned *)wsums;
            unsigned pending = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j * kLmThreads + (int)threadIdx.x < tot) pending |= 1u << j;
            bool late = false;
            for (unsigned spins = 0; pending && !broken; ++spins) {
                unsigned long long x[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int i = j * kLmThreads + threadIdx.x;
                    const int bb = i / (2 * NV), rr = i - bb * 2 * NV;
                    x[j] = (pending >> j & 1u) ? __hip_atomic_load(g + (size_t)bb * kLmRed * 2 + rr, __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT)
                                               : 0ull;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (!(pending >> j & 1u) || (x[j] & 0xFFFFFFFF00000000ull) != tag) continue;
                    const int i = j * kLmThreads + threadIdx.x;
                    const int bb = i / (2 * NV), rr = i - bb * 2 * NV;
                    ws32[bb * kLmRed * 2 + rr] = (unsigned)x[j];
                    pending &= ~(1u << j);
                }
                if (pending) {
                    if (spins >= kLmSpinLimit) {  // a range's sums never arrived: stop waiting (no hang)
                        late = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            broken = __syncthreads_or(broken || late) != 0;  // block-uniform from here on
        } else {
            __syncthreads();
        }
#ifdef RSAC_TRACE
        mark(23);
#endif
        // thread q < NV sums term q over the nb range sums, left to right
        if (threadIdx.x < NV) {
            const int q = threadIdx.x;
            double s = wsums[q];
            for (int bb = 1; bb < nb; ++bb) s = s + wsums[bb * kLmRed + q];
            out[q] = broken ? __builtin_nan("") : s;
        }
        __syncthreads();
    }
    __device__ void normal(const double *R, const double *t, double *acc) {
        sum_terms<kLmTerms>([&](double Xd, double Yd, double Zd, double u, double v,
                                double *a) { pnp_lm_point(R, t, k, Xd, Yd, Zd, u, v, a); },
                            acc);
    }
#ifdef RSAC_TRACE
    unsigned long long stamp[96], cyc[96];
    int phase_of[96];
    int ns = 0;
    __device__ void mark(int phase) {
        __syncthreads();
        if (ns < 96) {
            stamp[ns] = __builtin_amdgcn_s_memrealtime();
            cyc[ns] = __builtin_amdgcn_s_memtime();
            phase_of[ns++] = phase;
        }
    }
    __device__ void dump() {
        if (threadIdx.x == 0 && blockIdx.x == 0)
            for (int i = 1; i < ns; ++i)
                printf("trace %d->%d %llu ticks %llu cycles\n", phase_of[i - 1], phase_of[i], stamp[i] - stamp[i - 1],
                       cyc[i] - cyc[i - 1]);
    }
#endif
    __device__ double cost(const double *R, const double *t) {
        sum_terms<1>([&](double Xd, double Yd, double Zd, double u, double v,
                         double *a) { a[0] += pnp_lm_cost_point(R, t, k, Xd, Yd, Zd, u, v); },
                     res);
        return res[0];
    }
    // cost(R, t) and normal(R, t) in one pass: per-slot partials and reductions are term by
    // term the same as the separate passes'
    __device__ double cost_normal(const double *R, const double *t, double *acc) {
        sum_terms<kLmRed>(
            [&](double Xd, double Yd, double Zd, double u, double v, double *a) {
                pnp_lm_point(R, t, k, Xd, Yd, Zd, u, v, a);
                a[kLmTerms] += pnp_lm_cost_point(R, t, k, Xd, Yd, Zd, u, v);
            },
            acc);  // acc: an acc_buf (kLmRed wide), the cost in its last slot
        return acc[kLmTerms];
    }
};

// one problem per blockIdx.y (prob_base + y).  A problem of nb = lm_blocks(n) > 1 ranges runs in
// a launch of its own with G <= nb blocks (stride, = gridDim.x unless a test drops a block),
// block x owning ranges x, x + G, ...; all G blocks must be co-resident (launch_pnp_refine caps
// G at the device's limit).  fail (pinned host word): set when a reduction's sums never arrived;
// block 0 then writes the start pose back instead of a refined one.
__global__ __launch_bounds__(kLmThreads) void k_pnp_refine(PnpArgs a, const uint8_t *__restrict__ mask,
                                                           double *__restrict__ models, int32_t *__restrict__ iters,
                                                           int prob_base, unsigned long long *gran, unsigned tag_base,
                                                           double *host_models, const double *src,
                                                           const int32_t *stop, int stride, int32_t *fail) {
    __shared__ double wsum[kLmThreads / 64][kLmRed];
    __shared__ double accs[2][kLmRed], res[1], steps[2][16];
    __shared__ int scan[kLmThreads / 64];
    __shared__ int rtab[2][kLmMaxBlocks];
    __shared__ __attribute__((aligned(16))) char lds[kLmLdsBytes];  // 94 KB
    const int prob = prob_base + blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int nb = lm_blocks(n);
    if ((int)blockIdx.x >= nb) return;  // block-uniform; this problem uses fewer blocks
    if ((nb > 1) != (gran != nullptr)) return;  // the other launch's problem (launch_pnp_refine)
    if (stop && *stop) return;  // an LO chain that already ended (k_pnp_lo_count)
    double *m = models + (int64_t)prob * kModelStride;
    // src: the start record (else m itself); block 0 writes the whole record to m at the end
    const double *ms = src ? src + (int64_t)prob * kModelStride : m;
    if (ms[kValidSlot] == 0.0) {  // no model: block-uniform exit
        if (threadIdx.x == 0 && blockIdx.x == 0 && iters) iters[prob] = 0;
        if (src && blockIdx.x == 0 && threadIdx.x < kModelStride) m[threadIdx.x] = ms[threadIdx.x];
        if (host_models && blockIdx.x == 0 && threadIdx.x < 12)
            host_models[(int64_t)prob * kModelStride + threadIdx.x] = ms[threadIdx.x];
        return;
    }
    const double *cm = a.cams + 4 * prob;
    const double c[3] = {(double)a.X[p0], (double)a.Y[p0], (double)a.Z[p0]};
    GpuLmReducer red{a.X + p0, a.Y + p0, a.Z + p0, a.U + p0, a.V + p0, mask + p0,
                     n, Cam{cm[0], cm[1], cm[2], cm[3]}, c[0], c[1], c[2], wsum};
    red.nb = nb;
    red.stage = (float *)lds;
    red.cap = kLmStage;
    red.scan = scan;
    red.rbase = rtab[0];
    red.rcnt = rtab[1];
    red.gran = (lm_gu64 *)gran;
    red.tag_base = tag_base;
    red.wsums = (double *)(lds + 5 * kLmStage * 4);
    red.accs = accs;
    red.res = res;
    red.steps = steps;
    red.set_ranges(blockIdx.x, nb > 1 ? stride : 1);
    double R[9], t[3];
    for (int j = 0; j < 9; ++j) R[j] = ms[j];
    for (int j = 0; j < 3; ++j) t[j] = ms[9 + j];
    lm_to_centred(R, c, t);
    int it = pnp_lm_refine(red, R, t, kLmMaxIter);
#ifdef RSAC_TRACE
    red.mark(99);
    red.dump();
#endif
    lm_from_centred(R, c, t);
    if (red.broken) {  // block-uniform: report, and keep the start pose
        if (threadIdx.x == 0 && fail) __hip_atomic_store(fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int j = 0; j < 9; ++j) R[j] = ms[j];
        for (int j = 0; j < 3; ++j) t[j] = ms[9 + j];
        it = 0;
    }
    // every block read m before its first contribution, and block 0 got past the first
    // reduction only with every block's: no barrier before block 0 overwrites m
    __syncthreads();  // every thread of this block has read m before thread 0 overwrites it
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        if (src)
            for (int j = 12; j < kModelStride; ++j) m[j] = ms[j];
        for (int j = 0; j < 9; ++j) m[j] = R[j];
        for (int j = 0; j < 3; ++j) m[9 + j] = t[j];
        if (iters) iters[prob] = it;
        if (host_models) {  // pinned host memory: the result without a copy launch
            double *h = host_models + (int64_t)prob * kModelStride;
            for (int j = 0; j < 9; ++j) h[j] = R[j];
            for (int j = 0; j < 3; ++j) h[9 + j] = t[j];
        }
    }
}

int pnp_refine_coresident(int device) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pnp_refine, kLmThreads, 0) != hipSuccess) return 1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 1;
    const int64_t lim = (int64_t)per_cu * cus;
    return (int)std::max<int64_t>(1, std::min<int64_t>(lim, kLmMaxBlocks));
}

// EPnP of every problem's winner on its RANSAC inliers (rsac_math.h pnp_epnp),
// one block per problem; the same summation order as the host (pnp_epnp_host).
constexpr int kEpThreads = 256;  // real threads; the sums keep kLmThreads (512) virtual ones

struct GpuEpnpReducer {
    const float *X, *Y, *Z, *U, *V;
    const uint8_t *mask;
    int n;
    double c0, c1, c2;
    double (*wsum)[kRedMax];  // LDS [kLmThreads / 64][kRedMax]
    int *wmin;                // LDS [kEpThreads / 64]

    // Thread t accumulates virtual threads t and t + 256 of the kLmThreads-strided order in
    // separate partials, so the sums equal the 512-thread order bit for bit while each thread
    // has twice the registers of a 512-thread block.
    template <int NV, class F>
    __device__ void sum(F f, double *out) {
        double a0[NV], a1[NV];
        for (int q = 0; q < NV; ++q) a0[q] = a1[q] = 0.0;
#pragma unroll 1
        for (int i = threadIdx.x; i < n; i += kLmThreads)
            if (mask[i])
                f((double)X[i] - c0, (double)Y[i] - c1, (double)Z[i] - c2, (double)U[i], (double)V[i], a0);
#pragma unroll 1
        for (int i = threadIdx.x + kEpThreads; i < n; i += kLmThreads)
            if (mask[i])
                f((double)X[i] - c0, (double)Y[i] - c1, (double)Z[i] - c2, (double)U[i], (double)V[i], a1);
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        for (int q = 0; q < NV; ++q) {
            double v0 = a0[q], v1 = a1[q];
            for (int o = 32; o > 0; o >>= 1) {
                v0 = v0 + __shfl_xor(v0, o);
                v1 = v1 + __shfl_xor(v1, o);
            }
            if (lane == 0) {
                wsum[wave][q] = v0;
                wsum[wave + kEpThreads / 64][q] = v1;
            }
        }
        __syncthreads();
        for (int q = 0; q < NV; ++q) {
            double v = wsum[0][q];
            for (int w = 1; w < kLmThreads / 64; ++w) v = v + wsum[w][q];
            out[q] = v;
        }
        __syncthreads();
    }
    __device__ bool first(double *p) {
        int m = 0x7fffffff;
        for (int i = threadIdx.x; i < n; i += kEpThreads)
            if (mask[i]) {
                m = i;
                break;
            }
        for (int o = 32; o > 0; o >>= 1) m = min(m, __shfl_xor(m, o));
        if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = m;
        __syncthreads();
        m = wmin[0];
        for (int w = 1; w < kEpThreads / 64; ++w) m = min(m, wmin[w]);
        __syncthreads();
        if (m == 0x7fffffff) return false;
        p[0] = (double)X[m] - c0;
        p[1] = (double)Y[m] - c1;
        p[2] = (double)Z[m] - c2;
        return true;
    }
};

// EPnP stage 1 (sums -> frame + pair sums) and stage 3 (pose candidates) of every problem's
// winner, one block per problem; stage 2 (12 x 12 eigenvectors, betas) runs on the host in
// between (rsac_api.hip).  Problems without a model write s1.ok = 0.
__device__ GpuEpnpReducer epnp_reducer(const PnpArgs &a, const uint8_t *mask, int prob, double (*wsum)[kRedMax],
                                       int *wmin) {
    const int64_t p0 = a.offsets[prob];
    return GpuEpnpReducer{a.X + p0, a.Y + p0, a.Z + p0, a.U + p0, a.V + p0, mask + p0,
                          (int)(a.offsets[prob + 1] - p0), (double)a.X[p0], (double)a.Y[p0], (double)a.Z[p0],
                          wsum, wmin};
}

__global__ __launch_bounds__(kEpThreads) void k_pnp_epnp_s1(PnpArgs a, const uint8_t *__restrict__ mask,
                                                            const double *__restrict__ models, EpnpStage1 *st1) {
    __shared__ double wsum[kLmThreads / 64][kRedMax];
    __shared__ int wmin[kEpThreads / 64];
    const int prob = blockIdx.x;
    if (models[(int64_t)prob * kModelStride + kValidSlot] == 0.0) {  // no model: block-uniform exit
        if (threadIdx.x == 0) st1[prob].ok = 0.0;
        return;
    }
    const double *cm = a.cams + 4 * prob;
    GpuEpnpReducer red = epnp_reducer(a, mask, prob, wsum, wmin);
    EpnpStage1 s1;
    epnp_stage1(red, Cam{cm[0], cm[1], cm[2], cm[3]}, s1);
    if (threadIdx.x == 0) st1[prob] = s1;
}

__global__ __launch_bounds__(kEpThreads) void k_pnp_epnp_s3(PnpArgs a, const uint8_t *__restrict__ mask,
                                                            const EpnpStage1 *__restrict__ st1,
                                                            const EpnpStage2 *__restrict__ st2,
                                                            double *__restrict__ models) {
    __shared__ double wsum[kLmThreads / 64][kRedMax];
    __shared__ int wmin[kEpThreads / 64];
    const int prob = blockIdx.x;
    if (st1[prob].ok == 0.0) return;  // block-uniform
    const double *cm = a.cams + 4 * prob;
    GpuEpnpReducer red = epnp_reducer(a, mask, prob, wsum, wmin);
    double R[9], t[3];
    const bool ok = epnp_stage3(red, Cam{cm[0], cm[1], cm[2], cm[3]}, st1[prob], st2[prob], R, t);
    if (ok && threadIdx.x == 0) {
        const double c[3] = {red.c0, red.c1, red.c2};
        lm_from_centred(R, c, t);
        double *m = models + (int64_t)prob * kModelStride;
        for (int j = 0; j < 9; ++j) m[j] = R[j];
        for (int j = 0; j < 3; ++j) m[9 + j] = t[j];
    }
}

hipError_t launch_pnp_epnp_s1(const PnpArgs &a, int32_t P, const uint8_t *mask, const double *models,
                              EpnpStage1 *st1, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_epnp_s1, dim3(P), dim3(kEpThreads), 0, s, a, mask, models, st1);
    return hipGetLastError();
}

hipError_t launch_pnp_epnp_s3(const PnpArgs &a, int32_t P, const uint8_t *mask, const EpnpStage1 *st1,
                              const EpnpStage2 *st2, double *models, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_epnp_s3, dim3(P), dim3(kEpThreads), 0, s, a, mask, st1, st2, models);
    return hipGetLastError();
}

hipError_t launch_pnp_refine(const PnpArgs &a, int32_t P, const uint8_t *mask, double *models, int32_t *iters,
                             hipStream_t s, LmScratch *scratch, const int64_t *host_off, double *host_models,
                             const double *src, const int32_t *stop) {
    // every problem of up to 4096 points (and, with host_off unknown, every problem) in one
    // launch, one block each; each larger problem in a launch of its own: G = min(lm_blocks(n),
    // the co-resident limit) blocks share its ranges and hand their range sums over as tagged
    // granules (G = 1: one block walks all the ranges, same order, no exchange)
    const int nb_max = lm_blocks(a.max_n);
    if (!(P == 1 && nb_max > 1))  // (one large problem: only the multi-block launch has work)
        hipLaunchKernelGGL(k_pnp_refine, dim3(1, P), dim3(kLmThreads), 0, s, a, mask, models, iters, 0,
                           (unsigned long long *)nullptr, 0u, host_models, src, stop, 1, (int32_t *)nullptr);
    if (nb_max > 1) {
        if (!scratch || !scratch->gran || scratch->max_blocks < 1) return hipErrorInvalidValue;
        for (int p = 0; p < P; ++p) {
            const int np = host_off ? (int)(host_off[p + 1] - host_off[p]) : a.max_n;
            const int nb = lm_blocks(np);
            if (nb <= 1) continue;
            const int G = std::min(nb, scratch->max_blocks);
            // test hook (RSAC_DBG_REFIT_DROP_BLOCK): one block of the stride is never launched
            const int launched = scratch->drop_block && G > 1 ? G - 1 : G;
            // tag = launch (22 bits, never 0) << 10 | reduction index (< 1024): unique among the
            // granules in memory, which are zeroed whenever the launch counter wraps
            if (++scratch->launch >= (1u << 22)) {
                const hipError_t e = hipMemsetAsync(scratch->gran, 0, kLmGranuleBytes, s);
                if (e != hipSuccess) return e;
                scratch->launch = 1;
            }
            if (!scratch->coop || launched < 2) {
                hipLaunchKernelGGL(k_pnp_refine, dim3(launched, 1), dim3(kLmThreads), 0, s, a, mask, models, iters,
                                   p, scratch->gran, scratch->launch << 10, host_models, src, stop, G, scratch->fail);
                continue;
            }
            // the runtime either makes the G blocks co-resident or refuses the launch; refused
            // (other work holds the CUs), one block walks every range: the same bits, no exchange
            PnpArgs ka = a;
            const uint8_t *kmask = mask;
            double *kmodels = models, *khm = host_models;
            int32_t *kiters = iters, *kfail = scratch->fail;
            int kp = p, kstride = G;
            unsigned long long *kgran = scratch->gran;
            unsigned ktag = scratch->launch << 10;
            const double *ksrc = src;
            const int32_t *kstop = stop;
            void *args[] = {&ka, &kmask, &kmodels, &kiters, &kp, &kgran, &ktag, &khm, &ksrc, &kstop, &kstride, &kfail};
            const hipError_t e = hipLaunchCooperativeKernel((const void *)k_pnp_refine, dim3(launched, 1),
                                                            dim3(kLmThreads), args, 0, s);
            if (e == hipErrorCooperativeLaunchTooLarge) {
                (void)hipGetLastError();
                hipLaunchKernelGGL(k_pnp_refine, dim3(1, 1), dim3(kLmThreads), 0, s, a, mask, models, iters, p,
                                   scratch->gran, scratch->launch << 10, host_models, src, stop, 1, scratch->fail);
            } else if (e != hipSuccess) {
                return e;
            }
        }
    }
    return hipGetLastError();
}

// RANSAC-test mask and inlier count of one model record (problem 0): the
// local-optimisation step of LO-RANSAC.  *count must be zero on entry.
__global__ __launch_bounds__(256) void k_pnp_model_count(PnpArgs a, const double *__restrict__ m,
                                                         uint8_t *__restrict__ mask, int32_t *__restrict__ count) {
    const int64_t p0 = a.offsets[0];
    const int n = (int)(a.offsets[1] - p0);
    const Cam k{a.cams[0], a.cams[1], a.cams[2], a.cams[3]};
    const float thr2 = a.thr2[0];
    const bool valid = m[kValidSlot] != 0.0;
    int local = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int64_t q = p0 + i;
        const bool f = valid && pnp_err(m, m + 9, k, (double)a.X[q], (double)a.Y[q], (double)a.Z[q], a.U[q], a.V[q]) <=
                                    thr2;
        mask[q] = f;
        local += f;
    }
    for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(count, local);
}

// One LO-RANSAC step's recount (rsac_api.hip local_opt), decided on the device so that the
// whole chain of steps is enqueued at once: the mask and count of record m; the block that
// finishes last (ticket) compares the count with st->cur.  step < 0: the chain's start (st is
// initialised with cur = init_cur).  step >= 0: a no-op once an earlier step stopped the
// chain; a higher count makes m the best (st->best_buf = step's output buffer, improvements++)
// and, when best_out is set, copies m there; otherwise the chain stops.  count / ticket go back
// to 0, and the state is mirrored into pinned host memory (host_st).
__global__ __launch_bounds__(256) void k_pnp_lo_count(PnpArgs a, double *__restrict__ m,
                                                      uint8_t *__restrict__ mask, LoState *st, int step,
                                                      int32_t init_cur, double *best_out, LoState *host_st) {
    __shared__ int wsum[4];
    if (step >= 0 && st->stopped) return;  // block-uniform; written only by an earlier launch
    const int64_t p0 = a.offsets[0];
    const int n = (int)(a.offsets[1] - p0);
    const Cam k{a.cams[0], a.cams[1], a.cams[2], a.cams[3]};
    const float thr2 = a.thr2[0];
    // the chain's start (step < 0) is the scan's best hypothesis record, valid by construction
    // (a count above the floor needs status > 0) but without kValidSlot (hypothesis records leave
    // it to the status byte): stamped here for the refits and recounts that copy and read it
    const bool valid = step < 0 || m[kValidSlot] != 0.0;
    if (step < 0 && blockIdx.x == 0 && threadIdx.x == 0) m[kValidSlot] = 1.0;
    int local = 0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int64_t q = p0 + i;
        const bool f = valid && pnp_err(m, m + 9, k, (double)a.X[q], (double)a.Y[q], (double)a.Z[q], a.U[q], a.V[q]) <=
                                    thr2;
        mask[q] = f;
        local += f;
    }
    for (int o = 32; o > 0; o >>= 1) local += __shfl_xor(local, o);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = local;
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int blk = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    // count (low word) and ticket (high word) in one 64-bit atomic: the block that takes the last
    // ticket gets every other block's count in the returned value, so no fence orders two atomics
    // (r06: a __threadfence and a second atomic per block before)
    const unsigned long long old =
        atomicAdd(reinterpret_cast<unsigned long long *>(&st->count), (1ull << 32) | (unsigned)blk);
    if ((unsigned)(old >> 32) != gridDim.x - 1) return;
    // the last block: every block's count is in
    const int total = (int)(unsigned)old + blk;
    LoState v;
    if (step < 0) {
        v.cur = init_cur;
        v.stopped = 0;
        v.best_buf = 0;
        v.improvements = 0;
    } else {
        v.cur = __hip_atomic_load(&st->cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v.stopped = 0;
        v.best_buf = __hip_atomic_load(&st->best_buf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        v.improvements = __hip_atomic_load(&st->improvements, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (total > v.cur) {
            v.cur = total;
            v.best_buf = (step + 1) & 1;
            ++v.improvements;
            if (best_out)
                for (int q = 0; q < kModelStride; ++q) best_out[q] = m[q];
        } else {
            v.stopped = 1;
        }
    }
    v.count = 0;
    v.ticket = 0;
    v.last_total = total;
    __hip_atomic_store(&st->cur, v.cur, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->stopped, v.stopped, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->best_buf, v.best_buf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->improvements, v.improvements, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&st->ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (host_st) *host_st = v;
}

hipError_t launch_pnp_lo_count(const PnpArgs &a, int32_t n, double *model, uint8_t *mask, LoState *st, int step,
                               int32_t init_cur, double *best_out, LoState *host_st, hipStream_t s) {
    // 8 points per thread: one ticket atomic per 2048 points (the atomics of one address
    // serialise, ~10 ns each; 391 blocks at 100k points before r06)
    unsigned g = cdiv(n > 0 ? n : 1, 2048);
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_pnp_lo_count, dim3(g), dim3(256), 0, s, a, model, mask, st, step, init_cur, best_out,
                       host_st);
    return hipGetLastError();
}

hipError_t launch_pnp_model_count(const PnpArgs &a, int32_t n, const double *model, uint8_t *mask, int32_t *count,
                                  hipStream_t s) {
    unsigned g = cdiv(n > 0 ? n : 1, 256);
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(k_pnp_model_count, dim3(g), dim3(256), 0, s, a, model, mask, count);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fundamental matrix RANSAC (BASELINE.json configs[3]): the homography skeleton
// with an 8-point sample, the normalised 8-point solver and the Sampson test
// (rsac_math.h).  HomArgs: SX SY = image-1 points, DX DY = image-2 points.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Float32 Sampson pre-filter (BASELINE configs[3]).  The f32 test runs in a
// normalised frame: x^ = (x - c) / s per image (c = the f32 midpoint of the
// problem's bounding box, s a common power of 2 >= every half-range), so that
// r = x2^T F x1 does not cancel between pixel-scale terms.  With
// F^ = T2^T F T1 (T = [[s, 0, cx], [0, s, cy], [0, 0, 1]]): r^ = r,
// (a^, b^) = s (a, b), (a2^, b2^) = s (a2, b2), so r^2 <= T den  <=>  r^2 <= (T / s^2) den^.
// Per pair, in f32 with the f64 kernel's operation order:
//   a b c = F^ (x1^ y1^ 1),  a2 b2 = F^T (x2^ y2^ 1) (first two),  r = x2^ a + y2^ b + c,
//   den = a^2 + b^2 + a2^2 + b2^2,   decided inlier  r^2 < A den - beta1,
//                                    decided outlier r^2 > C den + beta2,
// otherwise the pair is recounted with the exact f64 test (fm_inlier, pixel frame), so the
// counts equal the f64 kernel's bit for bit.  Error model per hypothesis (u = 2^-24; X^ Y^ bounds
// of |x^| |y^|, exact x^ vs its f32 evaluation <= u |x^|; A^ B^ C^ A2^ B2^ absolute row / column
// sums of F^ against the bounds, Rp the pixel-frame analogue for the f64 kernel's own rounding):
//   |a32 - a^| <= e_a = 4.1u A^ + 1e-15 (A^ + s Ap),  likewise b c a2 b2;  e = max of them;
//   |r32 - r|  <= e_r = 7.5u (X2^ A^ + Y2^ B^ + C^) + 1e-15 Rp;
//   |den32 - den^| <= 4 e sqrt(den^) + 4 e^2 + 4.01u den32;
// with 2|r| e_r <= eta r^2 + e_r^2 / eta and 4 e sqrt(den) <= eta den + 4 e^2 / eta (eta = 1e-3),
// T^ = T / s^2:
//   A = T^ (1 - 6u) / (1 + eta)^2,  beta1 = (1 + 1/eta)(e_r^2 + 4 T^ e^2) / (1 + eta)
//   C = T^ (1 + 6u) / (1 - eta)^2,  beta2 = (e_r^2 / eta + 4 T^ e^2 (1 + 1/eta) / (1 - eta)) / (1 - eta)
// each with 1e-6 slack for the f32 rounding of A den -+ beta and the f64 kernel's own rounding.
// Record: F^ (9 f32), A, beta1, C, beta2; an invalid model is a decided outlier everywhere.
// ---------------------------------------------------------------------------
struct FmFrame {
    float c[4];      // x1 y1 x2 y2 centres
    float is;        // 1 / s
    double s;        // power of 2
    double hb[4];    // bounds of |x^| per coordinate
    double pb[4];    // bounds of |x| (pixel frame)
};

// ws: per problem 4 ordered-int minima then 4 maxima (k_fm_bounds); identical in every kernel
__device__ __forceinline__ FmFrame fm_frame(const int *ws, int prob) {
    FmFrame f;
    double half = 0;
    for (int k = 0; k < 4; ++k) {
        const float lo = ord2f(ws[8 * prob + k]), hi = ord2f(ws[8 * prob + 4 + k]);
        f.c[k] = (lo <= hi) ? (lo + hi) * 0.5f : 0.f;  // empty problem: lo = +inf, hi = -inf
        f.pb[k] = fmax(fabs((double)lo), fabs((double)hi));
        half = fmax(half, fmax((double)hi - f.c[k], (double)f.c[k] - lo));
    }
    int e = 0;
    (void)frexp(half > 0 && half < 1e30 ? half : 1.0, &e);
    f.s = ldexp(1.0, e);  // >= half
    f.is = (float)(1.0 / f.s);
    for (int k = 0; k < 4; ++k) {
        const float lo = ord2f(ws[8 * prob + k]), hi = ord2f(ws[8 * prob + 4 + k]);
        f.hb[k] = fmax((double)hi - f.c[k], (double)f.c[k] - lo) * (1.0 + 1.2e-7) / f.s;
    }
    return f;
}

__device__ __forceinline__ void fm_write_record(const double *F, bool valid, const int *ws, int prob, double T,
                                                float *rec) {
    const FmFrame fr = fm_frame(ws, prob);
    bool finite = valid;
    for (int q = 0; q < 9; ++q) finite = finite && isfinite(F[q]);
    if (!valid || !finite || !(fr.hb[0] == fr.hb[0]) || !(fr.pb[0] < 1e30) || !(fr.pb[2] < 1e30)) {
#pragma unroll
        for (int q = 0; q < kFModelStride; ++q) rec[q] = 0.f;
        if (!valid) {
            rec[10] = 1.f;   // lo = -1: never an inlier
            rec[12] = -1.f;  // hi = -1 < r^2 = 0: an outlier
        } else {
            rec[9] = rec[11] = __builtin_nanf("");  // every pair undecided: the f64 test decides
        }
        return;
    }
    const double s = fr.s;
    // F^ = T2^T F T1
    double G[9];  // F T1
    for (int i = 0; i < 3; ++i) {
        G[3 * i] = F[3 * i] * s;
        G[3 * i + 1] = F[3 * i + 1] * s;
        G[3 * i + 2] = F[3 * i] * fr.c[0] + F[3 * i + 1] * fr.c[1] + F[3 * i + 2];
    }
    double Fh[9];
    for (int j = 0; j < 3; ++j) {
        Fh[j] = s * G[j];
        Fh[3 + j] = s * G[3 + j];
        Fh[6 + j] = fr.c[2] * G[j] + fr.c[3] * G[3 + j] + G[6 + j];
    }
    const double X1 = fr.hb[0], Y1 = fr.hb[1], X2 = fr.hb[2], Y2 = fr.hb[3];
    const double Ar = fabs(Fh[0]) * X1 + fabs(Fh[1]) * Y1 + fabs(Fh[2]);
    const double Br = fabs(Fh[3]) * X1 + fabs(Fh[4]) * Y1 + fabs(Fh[5]);
    const double Cr = fabs(Fh[6]) * X1 + fabs(Fh[7]) * Y1 + fabs(Fh[8]);
    const double A2 = fabs(Fh[0]) * X2 + fabs(Fh[3]) * Y2 + fabs(Fh[6]);
    const double B2 = fabs(Fh[1]) * X2 + fabs(Fh[4]) * Y2 + fabs(Fh[7]);
    // pixel-frame sums (the f64 kernel's rounding, ~1e-16 relative of these)
    const double P1 = fr.pb[0], Q1 = fr.pb[1], P2 = fr.pb[2], Q2 = fr.pb[3];
    const double Ap = fmax(fmax(fabs(F[0]) * P1 + fabs(F[1]) * Q1 + fabs(F[2]), fabs(F[3]) * P1 + fabs(F[4]) * Q1 + fabs(F[5])),
                           fmax(fabs(F[0]) * P2 + fabs(F[3]) * Q2 + fabs(F[6]), fabs(F[1]) * P2 + fabs(F[4]) * Q2 + fabs(F[7])));
    const double Rp = P2 * (fabs(F[0]) * P1 + fabs(F[1]) * Q1 + fabs(F[2])) +
                      Q2 * (fabs(F[3]) * P1 + fabs(F[4]) * Q1 + fabs(F[5])) + fabs(F[6]) * P1 + fabs(F[7]) * Q1 + fabs(F[8]);
    constexpr double u = 5.9604644775390625e-08, eta = 1e-3;
    const double e = 4.1 * u * fmax(fmax(Ar, Br), fmax(fmax(A2, B2), Cr)) + 1e-15 * (fmax(fmax(Ar, Br), fmax(A2, B2)) + s * Ap);
    const double er = 7.5 * u * (X2 * Ar + Y2 * Br + Cr) + 1e-15 * Rp;
    const double Th = T / (s * s);
    const double Alo = Th * (1.0 - 6.0 * u) / ((1.0 + eta) * (1.0 + eta)) * (1.0 - 1e-6);
    const double b1 = (1.0 + 1.0 / eta) * (er * er + 4.0 * Th * e * e) / (1.0 + eta) * (1.0 + 1e-6);
    const double Chi = Th * (1.0 + 6.0 * u) / ((1.0 - eta) * (1.0 - eta)) * (1.0 + 1e-6);
    const double b2 = (er * er / eta + 4.0 * Th * e * e * (1.0 + 1.0 / eta) / (1.0 - eta)) / (1.0 - eta) * (1.0 + 1e-6);
#pragma unroll
    for (int q = 0; q < 9; ++q) rec[q] = (float)Fh[q];
    // A rounded down, the others up (float conversion rounds to nearest: nudge by 2^-23)
    rec[9] = (float)(Alo * (1.0 - 1.2e-7));
    rec[10] = (float)(b1 * (1.0 + 1.2e-7));
    rec[11] = (float)(Chi * (1.0 + 1.2e-7));
    rec[12] = (float)(b2 * (1.0 + 1.2e-7));
    rec[13] = rec[14] = rec[15] = 0.f;
}

struct FmTest {
    bool lt, gt;
};
__device__ __forceinline__ FmTest fm_test_f32(const float *m, float x1, float y1, float x2, float y2) {
    const float a = __builtin_fmaf(m[0], x1, __builtin_fmaf(m[1], y1, m[2]));
    const float b = __builtin_fmaf(m[3], x1, __builtin_fmaf(m[4], y1, m[5]));
    const float c = __builtin_fmaf(m[6], x1, __builtin_fmaf(m[7], y1, m[8]));
    const float a2 = __builtin_fmaf(m[0], x2, __builtin_fmaf(m[3], y2, m[6]));
    const float b2 = __builtin_fmaf(m[1], x2, __builtin_fmaf(m[4], y2, m[7]));
    const float r = __builtin_fmaf(x2, a, __builtin_fmaf(y2, b, c));
    const float r2 = r * r;
    const float den = __builtin_fmaf(a, a, __builtin_fmaf(b, b, __builtin_fmaf(a2, a2, b2 * b2)));
    return FmTest{r2 < __builtin_fmaf(m[9], den, -m[10]), r2 > __builtin_fmaf(m[11], den, m[12])};
}

// min / max of x1 y1 x2 y2 of every problem (ordered-int encoding; ws: P x 8, preset to
// +max / -max by launch_fm_bounds); a NaN coordinate poisons the problem's frame (all pairs
// then fall back to the f64 test)
__global__ __launch_bounds__(256) void k_fm_bounds(HomArgs a, int *__restrict__ ws) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    float lo[4], hi[4];
    bool nan = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) { lo[k] = __builtin_inff(); hi[k] = -__builtin_inff(); }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float v[4] = {a.SX[p0 + i], a.SY[p0 + i], a.DX[p0 + i], a.DY[p0 + i]};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lo[k] = fminf(lo[k], v[k]);
            hi[k] = fmaxf(hi[k], v[k]);
            nan = nan || v[k] != v[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    }
    if (__ballot(nan)) { lo[0] = -__builtin_inff(); hi[0] = __builtin_inff(); }
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            atomicMin(ws + 8 * prob + k, f2ord(lo[k]));
            atomicMax(ws + 8 * prob + 4 + k, f2ord(hi[k]));
        }
    }
}

// ws preset: minima to INT_MAX, maxima to INT_MIN (ordered-int encoding)
__global__ void k_fm_bounds_init(int32_t P, int *__restrict__ ws) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 8 * P; i += gridDim.x * blockDim.x)
        ws[i] = (i % 8) < 4 ? 0x7FFFFFFF : (int)0x80000000;
}

// fm_minimal8 on 8 lanes (one row of the 8 x 9 DLT system per lane, in registers): the same
// operations in the same order, so the same bits (tests: every hypothesis against the oracle).
// The one-lane form keeps A, its row / column swaps and the permutation in scratch (704 B per
// lane; 620 MB of WRITE_SIZE per 100k hypotheses, C4); here a row swap is a lane exchange, a
// column swap selects over the row's 9 registers, and the pivot search is a group reduction.
// g: the group's first lane; q = lane - g: this lane's point and row.  Group-uniform result.
__device__ __forceinline__ bool fm_minimal8_g8(float x1, float y1, float x2, float y2, int g, int q, double *F) {
    // Hartley normalisation of both images (fm_norm8): the sums in point order on every lane
    double c[2][2], sc[2];
#pragma unroll
    for (int im = 0; im < 2; ++im) {
        const float xs = im ? x2 : x1, ys = im ? y2 : y1;
        double cx = 0.0, cy = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            cx = cx + (double)__shfl(xs, g + k);
            cy = cy + (double)__shfl(ys, g + k);
        }
        cx = cx * 0.125;
        cy = cy * 0.125;
        const double dx = (double)xs - cx, dy = (double)ys - cy;
        const double tq = dsqrt(dx * dx + dy * dy);
        double d = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) d = d + __shfl(tq, g + k);
        d = d * 0.125;
        if (!(d > 1e-300)) return false;
        c[im][0] = cx;
        c[im][1] = cy;
        sc[im] = 1.4142135623730951 / d;
    }
    const double u1 = ((double)x1 - c[0][0]) * sc[0], v1 = ((double)y1 - c[0][1]) * sc[0];
    const double u2 = ((double)x2 - c[1][0]) * sc[1], v2 = ((double)y2 - c[1][1]) * sc[1];
    double A[9] = {u2 * u1, u2 * v1, u2, v2 * u1, v2 * v1, v2, u1, v1, 1.0};
    double amax = 0.0;
#pragma unroll
    for (int j = 0; j < 9; ++j) amax = dabs(A[j]) > amax ? dabs(A[j]) : amax;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        const double w = __shfl_xor(amax, o);
        amax = w > amax ? w : amax;
    }
    int perm[9] = {0, 1, 2, 3, 4, 5, 6, 7, 8};
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        // pivot: the first maximum of |A[i][j]|, i >= r, j >= r, in row-major order
        double best = q >= r ? -1.0 : -2.0;
        int pc = r;
#pragma unroll
        for (int j = r; j < 9; ++j)
            if (q >= r && dabs(A[j]) > best) { best = dabs(A[j]); pc = j; }
        int pr = q;
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const double ob = __shfl_xor(best, o);
            const int opr = __shfl_xor(pr, o), opc = __shfl_xor(pc, o);
            if (ob > best || (ob == best && opr < pr)) { best = ob; pr = opr; pc = opc; }
        }
        if (!(best > 1e-12 * amax)) return false;
        if (pr != r) {  // group-uniform: rows r and pr trade lanes
            const int src = g + (q == r ? pr : q == pr ? r : q);
#pragma unroll
            for (int j = 0; j < 9; ++j) A[j] = __shfl(A[j], src);
        }
        if (pc != r) {
            double apc = A[r];
#pragma unroll
            for (int j = r + 1; j < 9; ++j) apc = j == pc ? A[j] : apc;
            const double ar = A[r];
#pragma unroll
            for (int j = r + 1; j < 9; ++j) A[j] = j == pc ? ar : A[j];
            A[r] = apc;
            int ppc = perm[r];
#pragma unroll
            for (int j = r + 1; j < 9; ++j) ppc = j == pc ? perm[j] : ppc;
            const int pr0 = perm[r];
#pragma unroll
            for (int j = r + 1; j < 9; ++j) perm[j] = j == pc ? pr0 : perm[j];
            perm[r] = ppc;
        }
        double prow[9];
#pragma unroll
        for (int j = r; j < 9; ++j) prow[j] = __shfl(A[j], g + r);
        const double ip = 1.0 / prow[r];
        if (q != r) {
            const double f = A[r] * ip;
            if (f != 0.0) {
#pragma unroll
                for (int j = r; j < 9; ++j) A[j] = A[j] - f * prow[j];
            }
        }
    }
    // f[perm[r]] = -A[r][8] / A[r][r]; f[perm[8]] = 1
    double arr = A[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) arr = q == j ? A[j] : arr;
    const double val = -A[8] / arr;
    double f[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) f[k] = perm[8] == k ? 1.0 : 0.0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const double fr = __shfl(val, g + r);
#pragma unroll
        for (int k = 0; k < 9; ++k) f[k] = perm[r] == k ? fr : f[k];
    }
    return fm_finish(f, c[0][0], c[0][1], sc[0], c[1][0], c[1][1], sc[1], F);
}

// 8 lanes per hypothesis (fm_minimal8_g8): 32 hypotheses per 256-thread block
__global__ __launch_bounds__(256) void k_fm_solve_g8(HomArgs a, int64_t hyp_begin, int32_t H) {
    const int prob = blockIdx.y;
    const int lane = threadIdx.x & 63, q = lane & 7, g = lane & ~7;
    const int hl = blockIdx.x * 32 + (threadIdx.x >> 3);
    const bool live = hl < H;  // group-uniform; dead groups still reach every shuffle
    const int64_t h = hyp_begin + (live ? hl : 0);
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    int8_t st = -1;
    double F[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    bool go = false;
    float x1 = 0.f, y1 = 0.f, x2 = 0.f, y2 = 0.f;
    if (n >= 8) {
        Philox rng;
        rng.init(a.seed, 0u, (uint64_t)(a.rng_base + h));
        int32_t idx[8];
        if (rng.subset<8>(n, idx) == 0) {
            int my = idx[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) my = q == j ? idx[j] : my;
            const int64_t i = p0 + my;
            x1 = a.SX[i]; y1 = a.SY[i]; x2 = a.DX[i]; y2 = a.DY[i];
            go = true;
        }
    }
    if (go) {  // group-uniform (the subset is the group's)
        st = fm_minimal8_g8(x1, y1, x2, y2, g, q, F) ? 1 : 0;
        if (st == 0)
#pragma unroll
            for (int k = 0; k < 9; ++k) F[k] = 0.0;
    }
    if (!live || q != 0) return;
    const int64_t rec = (int64_t)prob * a.hyp_stride + h;
    double *m = a.models + rec * kModelStride;
#pragma unroll
    for (int k = 0; k < 9; ++k) m[k] = F[k];
    m[kValidSlot] = st > 0 ? 1.0 : 0.0;
    a.status[rec] = st;
    if (a.fmodels) fm_write_record(F, st > 0, a.fbounds, prob, (double)a.thr2[prob], a.fmodels + rec * kFModelStride);
}

// hypotheses x points tiles (points in registers, hypothesis wave-uniform), exact f64 test
template <int P, int HB>
__global__ __launch_bounds__(256) void k_fm_score(HomArgs a, int64_t hyp_begin, int32_t H, int32_t *__restrict__ counts) {
    __shared__ int red[4][HB];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t h0 = hyp_begin + (int64_t)blockIdx.x * HB;
    const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const double T = (double)a.thr2[prob];
    const double *__restrict__ mb = a.models + ((int64_t)prob * a.hyp_stride + h0) * kModelStride;
    const float *__restrict__ SX = a.SX + p0, *__restrict__ SY = a.SY + p0;
    const float *__restrict__ DX = a.DX + p0, *__restrict__ DY = a.DY + p0;
    int cnt = 0;
    for (int base = wave * 64 * P; base < n; base += 4 * 64 * P) {
        double x1[P], y1[P], x2[P], y2[P];
        bool in[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int i = base + j * 64 + lane;
            in[j] = i < n;
            const int ii = in[j] ? i : 0;
            x1[j] = SX[ii]; y1[j] = SY[ii]; x2[j] = DX[ii]; y2[j] = DY[ii];
        }
        for (int h = 0; h < nh; ++h) {
            const double *__restrict__ m = mb + h * kModelStride;
            if (m[kValidSlot] == 0.0) continue;
            double F[9];
#pragma unroll
            for (int q = 0; q < 9; ++q) F[q] = m[q];
            int cc = 0;
#pragma unroll
            for (int j = 0; j < P; ++j) cc += __popcll(__ballot(in[j] && fm_inlier(F, x1[j], y1[j], x2[j], y2[j], T)));
            cnt += (lane == h) ? cc : 0;
        }
    }
    if (lane < HB) red[wave][lane] = cnt;
    __syncthreads();
    if (threadIdx.x < nh) {
        const int s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        counts[(int64_t)prob * a.hyp_stride + h0 + threadIdx.x] = s;
    }
}

__global__ __launch_bounds__(256) void k_fm_score_lane(HomArgs a, int64_t hyp_begin, int32_t H,
                                                       int32_t *__restrict__ counts) {
    __shared__ float sp[4][kLanePts];
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    for (int i = threadIdx.x; i < n; i += 256) {
        sp[0][i] = a.SX[p0 + i]; sp[1][i] = a.SY[p0 + i]; sp[2][i] = a.DX[p0 + i]; sp[3][i] = a.DY[p0 + i];
    }
    __syncthreads();
    const int hl = blockIdx.x * 256 + threadIdx.x;
    if (hl >= H) return;
    const int64_t rec = (int64_t)prob * a.hyp_stride + hyp_begin + hl;
    const double *__restrict__ m = a.models + rec * kModelStride;
    int cnt = 0;
    if (m[kValidSlot] != 0.0) {
        const double T = (double)a.thr2[prob];
        double F[9];
        for (int q = 0; q < 9; ++q) F[q] = m[q];
        for (int i = 0; i < n; ++i) cnt += fm_inlier(F, sp[0][i], sp[1][i], sp[2][i], sp[3][i], T);
    }
    counts[rec] = cnt;
}

// f32 Sampson pre-filter (record: fm_write_record) on a work queue (the layout of
// k_pnp_score_sc; undecided pairs recounted with the exact f64 test): tiles of 32 hypotheses,
// whole-tile units for all but the last `resident` tiles, which go one unit per cell of
// 64 x 4 x P points; the lean hypothesis loop (all 32 staged records, counts by v_writelane,
// undecided flags in an SGPR mask); counts added atomically into zeroed counts.
template <int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_fm_score_q(
    HomArgs a, int64_t hyp_begin, int32_t H, int32_t n_prob, int32_t *__restrict__ counts, int tb, int cells) {
    constexpr int HB = 32;
    constexpr int kStride = 4 * 64 * P;
    __shared__ int red[4][HB];
    __shared__ int unit_s;
    __shared__ __attribute__((aligned(16))) float mlds[HB * kFModelStride];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_per_prob = (H + HB - 1) / HB;
    const int n_units = tb + (tiles_per_prob * n_prob - tb) * cells;
    // split queue (as k_pnp_score_mf): block b takes units b % kQSub + kQSub i from counter b % kQSub
    int *const uq = fm_unit_queue(a.fm_queue, blockIdx.x % kQSub);
    for (;;) {
        if (threadIdx.x == 0) unit_s = blockIdx.x % kQSub + kQSub * atomicAdd(uq, 1);
        __syncthreads();
        const int unit = __builtin_amdgcn_readfirstlane(unit_s);
        if (unit >= n_units) break;  // uniform
        int tile, c0, c1;
        if (unit < tb) {
            tile = unit;
            c0 = 0;
            c1 = cells;
        } else {
            tile = tb + (unit - tb) / cells;
            c0 = (unit - tb) % cells;
            c1 = c0 + 1;
        }
        const int prob = tile / tiles_per_prob;
        const int64_t h0 = hyp_begin + (int64_t)(tile % tiles_per_prob) * HB;
        const int nh = (int)min((int64_t)HB, hyp_begin + H - h0);
        const int64_t p0 = a.offsets[prob];
        const int n_all = (int)(a.offsets[prob + 1] - p0);
        const int start = c0 * kStride;
        const int n = min(n_all, c1 * kStride);
        if (start >= n_all) {
            __syncthreads();
            continue;
        }
        const int64_t rec0 = (int64_t)prob * a.hyp_stride + h0;
        if (threadIdx.x < HB) {  // past the round: fm_write_record's "no model" form (decided outlier)
            const int hq = threadIdx.x;
            float *dst = mlds + hq * kFModelStride;
            const float *src = a.fmodels + (rec0 + hq) * kFModelStride;
            const bool in = hq < nh;
#pragma unroll
            for (int q = 0; q < kFModelStride; ++q) dst[q] = in ? src[q] : 0.f;
            if (!in) {
                dst[10] = 1.f;
                dst[12] = -1.f;
            }
        }
        __syncthreads();
        const float *__restrict__ SX = a.SX + p0, *__restrict__ SY = a.SY + p0;
        const float *__restrict__ DX = a.DX + p0, *__restrict__ DY = a.DY + p0;
        const FmFrame fr = fm_frame(a.fbounds, prob);
        int cnt = 0;
        for (int base = start + wave * 64 * P; base < n; base += kStride) {
            float x1[P], y1[P], x2[P], y2[P];  // normalised frame
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int i = base + j * 64 + lane;
                const bool in = i < n;
                const int ii = in ? i : 0;
                x1[j] = (SX[ii] - fr.c[0]) * fr.is;
                y1[j] = (SY[ii] - fr.c[1]) * fr.is;
                x2[j] = (DX[ii] - fr.c[2]) * fr.is;
                // out-of-range lanes: y2 = 3e38 makes the pair a decided outlier (or undecided)
                y2[j] = in ? (DY[ii] - fr.c[3]) * fr.is : 3.0e38f;
            }
            int ccl = 0;
            uint32_t wund = 0;
#pragma unroll 4
            for (int h = 0; h < HB; ++h) {
                const float *m = mlds + h * kFModelStride;
                int cc = 0;
                uint64_t und = 0;
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const FmTest r = fm_test_f32(m, x1[j], y1[j], x2[j], y2[j]);
                    const uint64_t mi = __ballot(r.lt);
                    const uint64_t mo = __ballot(r.gt);
                    cc += __popcll(mi);
                    und |= ~(mi | mo);
                }
                // v_writelane_b32 (no clang builtin); lane select through M0; SALU operands
                asm("v_writelane_b32 %0, %1, %2" : "+v"(ccl) : "s"(cc), "{m0}"(h));
                wund |= und ? (1u << h) : 0u;
            }
            cnt += ccl;
            if (__builtin_expect(wund != 0, 0)) {
                const double T = (double)a.thr2[prob];
#pragma unroll 1
                while (wund) {
                    const int h = __builtin_ctz(wund);
                    wund &= wund - 1;
                    const float *m = mlds + h * kFModelStride;
                    const double *md = a.models + (rec0 + h) * kModelStride;
                    int cc = 0;
#pragma unroll 1
                    for (int j = 0; j < P; ++j) {
                        const int i = base + j * 64 + lane;
                        const FmTest r = fm_test_f32(m, x1[j], y1[j], x2[j], y2[j]);
                        const bool ex = !(r.lt | r.gt) && i < n && md[kValidSlot] != 0.0 &&
                                        fm_inlier(md, (double)SX[i], (double)SY[i], (double)DX[i], (double)DY[i], T);
                        cc += __popcll(__ballot(ex));
                    }
                    cnt += (lane == h) ? cc : 0;
                }
            }
        }
        if (lane < HB) red[wave][lane] = cnt;
        __syncthreads();
        if (wave == 0 && lane < nh) {
            const int sum = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
            if (sum) atomicAdd(&counts[rec0 + lane], sum);
        }
        __syncthreads();  // red, mlds and unit_s are rewritten by the next unit
    }
}

__global__ void k_fm_mask(HomArgs a, const int64_t *__restrict__ best, int64_t best0, uint8_t *__restrict__ mask) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t b = best ? best[prob] : best0;  // best0: the one problem's record, no upload
    const double T = (double)a.thr2[prob];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int64_t q = p0 + i;
        mask[q] = b >= 0 && fm_inlier(a.models + b * kModelStride, a.SX[q], a.SY[q], a.DX[q], a.DY[q], T);
    }
}

hipError_t launch_fm_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s) {
    hipLaunchKernelGGL(k_fm_solve_g8, dim3(cdiv(H, 32), P), dim3(256), 0, s, a, hyp_begin, H);
    return hipGetLastError();
}

hipError_t launch_fm_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts, hipStream_t s) {
    if (a.max_n > 0 && a.max_n <= kLanePts)
        hipLaunchKernelGGL(k_fm_score_lane, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H, counts);
    else if (a.fmodels && a.fm_queue) {
        // k_fm_score_q: whole-tile units, then the last `resident` tiles by cells (launch_sc)
        constexpr int FP = 8;
        static const int resident = resident_blocks(k_fm_score_q<FP>);
        const int64_t cells = std::max<int64_t>(1, ((int64_t)a.max_n + 256 * FP - 1) / (256 * FP));
        const int64_t tiles = (int64_t)P * ((H + 31) / 32);
        const int64_t cell_tiles = std::min<int64_t>(tiles, resident);
        const int64_t tb = tiles - cell_tiles, units = tb + cell_tiles * cells;
        hipError_t e = hipMemsetAsync(a.fm_queue + kFmQOff, 0, 32 * kQSub * sizeof(int), s);
        if (e == hipSuccess) {
            if (P == 1)
                e = hipMemsetAsync(counts + hyp_begin, 0, sizeof(int32_t) * H, s);
            else
                e = hipMemset2DAsync(counts + hyp_begin, sizeof(int32_t) * a.hyp_stride, 0, sizeof(int32_t) * H, P, s);
        }
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_fm_score_q<FP>, dim3(queue_grid(units, resident)), dim3(256), 0, s, a, hyp_begin, H, P, counts, (int)tb,
                           (int)cells);
    } else
        hipLaunchKernelGGL((k_fm_score<4, 32>), dim3(cdiv(H, 32), P), dim3(256), 0, s, a, hyp_begin, H, counts);
    return hipGetLastError();
}

hipError_t launch_fm_bounds(const HomArgs &a, int32_t P, int32_t max_n, int *ws, hipStream_t s) {
    hipLaunchKernelGGL(k_fm_bounds_init, dim3(cdiv(8 * P, 256)), dim3(256), 0, s, P, ws);
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 2048);
    if (g > 64) g = 64;
    hipLaunchKernelGGL(k_fm_bounds, dim3(g, P), dim3(256), 0, s, a, ws);
    return hipGetLastError();
}

hipError_t launch_fm_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                          hipStream_t s, int64_t best0) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_fm_mask, dim3(g, P), dim3(256), 0, s, a, best, best0, mask);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Winner re-derivation (rsac_pnp_winner): the hypothesis named by a device-
// resident packed key is re-solved from its Philox counter (the same draw and
// P3P as k_pnp_solve, from the f64 AoS inputs rounded to f32 exactly as
// k_pnp_prepare rounds them), then its RANSAC-test mask.  No host round trip.
// cam: fx fy cx cy thr2 (f64).
// ---------------------------------------------------------------------------
__global__ void k_pnp_winner_solve(const double *__restrict__ p3, const double *__restrict__ p2, int32_t n,
                                   const double *__restrict__ cam, uint64_t seed, const int64_t *__restrict__ key,
                                   double *__restrict__ rec, double *__restrict__ model_out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long kk = (unsigned long long)*key;
    double R[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, t[3] = {0, 0, 0};
    bool ok = false;
    if (kk != 0 && n >= 4) {
        const uint64_t idx = 0xFFFFFFFFull - (kk & 0xFFFFFFFFull);
        Philox rng;
        rng.init(seed, 0u, idx);
        int32_t id[4];
        if (rng.subset<4>(n, id) == 0) {
            float X[4], Y[4], Z[4], U[4], V[4];
            for (int j = 0; j < 4; ++j) {
                X[j] = (float)p3[3 * id[j]]; Y[j] = (float)p3[3 * id[j] + 1]; Z[j] = (float)p3[3 * id[j] + 2];
                U[j] = (float)p2[2 * id[j]]; V[j] = (float)p2[2 * id[j] + 1];
            }
            const Cam k{cam[0], cam[1], cam[2], cam[3]};
            ok = pnp_minimal(X, Y, Z, U, V, k, R, t);
        }
    }
    for (int q = 0; q < 9; ++q) rec[q] = ok ? R[q] : 0.0;
    for (int q = 0; q < 3; ++q) rec[9 + q] = ok ? t[q] : 0.0;
    rec[kValidSlot] = ok ? 1.0 : 0.0;
    if (model_out)
        for (int q = 0; q < 12; ++q) model_out[q] = rec[q];
}

__global__ void k_pnp_winner_mask(const double *__restrict__ p3, const double *__restrict__ p2, int32_t n,
                                  const double *__restrict__ cam, const double *__restrict__ rec,
                                  uint8_t *__restrict__ mask) {
    const Cam k{cam[0], cam[1], cam[2], cam[3]};
    const float thr2 = (float)cam[4];
    const bool valid = rec[kValidSlot] != 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const double X = (float)p3[3 * i], Y = (float)p3[3 * i + 1], Z = (float)p3[3 * i + 2];
        mask[i] = valid && pnp_err(rec, rec + 9, k, X, Y, Z, (float)p2[2 * i], (float)p2[2 * i + 1]) <= thr2;
    }
}

hipError_t launch_pnp_winner(const double *p3, const double *p2, int32_t n, const double *cam, uint64_t seed,
                             const int64_t *key, double *rec, double *model_out, uint8_t *mask, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_winner_solve, dim3(1), dim3(64), 0, s, p3, p2, n, cam, seed, key, rec, model_out);
    if (mask) {
        unsigned g = cdiv(n > 0 ? n : 1, 256);
        if (g > 1024) g = 1024;
        hipLaunchKernelGGL(k_pnp_winner_mask, dim3(g), dim3(256), 0, s, p3, p2, n, cam, rec, mask);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// compute_reprojection_error (testpro-K.py:32-36) on f64 inputs: cv2.projectPoints + the
// residual's L2 norm per point (pnp_reproj_err).  p3 / p2: f64 AoS (device).
// ---------------------------------------------------------------------------
// one pose: the projections (proj, n x 2, optional) and errors (err, n, optional)
__global__ void k_pnp_reproj(const double *__restrict__ p3, const double *__restrict__ p2, int32_t n, PoseCam pc,
                             double *__restrict__ proj, double *__restrict__ err) {
    const Cam k{pc.cam[0], pc.cam[1], pc.cam[2], pc.cam[3]};
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        double pu, pv;
        const double e = pnp_reproj_err(pc.R, pc.t, k, p3[3 * i], p3[3 * i + 1], p3[3 * i + 2], p2[2 * i],
                                        p2[2 * i + 1], pu, pv);
        if (proj) {
            proj[2 * i] = pu;
            proj[2 * i + 1] = pv;
        }
        if (err) err[i] = e;
    }
}

// the mean inlier error of every problem p (testpro-K.py:80-82: np.mean over the inliers): one
// wave per problem over the shared points, poses[p] (R 9, t 3) and cams[p] (fx fy cx cy), masks
// p x n.  Order (the oracle's orc_reproj_mean): lane l sums its points l, l + 64, ... ascending,
// then the xor butterfly (o = 32 .. 1) of the 64 lane sums; out[p] = {sum, count}
__global__ __launch_bounds__(64) void k_pnp_reproj_mean(const double *__restrict__ p3, const double *__restrict__ p2,
                                                        int32_t n, const double *__restrict__ poses,
                                                        const double *__restrict__ cams,
                                                        const uint8_t *__restrict__ masks, double *__restrict__ out) {
    const int p = blockIdx.x, lane = threadIdx.x;
    const double *m = poses + 12 * p;
    const Cam k{cams[4 * p], cams[4 * p + 1], cams[4 * p + 2], cams[4 * p + 3]};
    const uint8_t *mk = masks + (int64_t)p * n;
    double s = 0.0;
    int c = 0;
    for (int i = lane; i < n; i += 64)
        if (mk[i]) {
            double pu, pv;
            s = s + pnp_reproj_err(m, m + 9, k, p3[3 * i], p3[3 * i + 1], p3[3 * i + 2], p2[2 * i], p2[2 * i + 1],
                                   pu, pv);
            ++c;
        }
    for (int o = 32; o > 0; o >>= 1) {
        s = s + __shfl_xor(s, o);
        c += __shfl_xor(c, o);
    }
    if (lane == 0) {
        out[2 * p] = s;
        out[2 * p + 1] = (double)c;
    }
}

hipError_t launch_pnp_reproj(const double *p3, const double *p2, int32_t n, const PoseCam &pc, double *proj,
                             double *err, hipStream_t s) {
    unsigned g = cdiv(n > 0 ? n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pnp_reproj, dim3(g), dim3(256), 0, s, p3, p2, n, pc, proj, err);
    return hipGetLastError();
}

hipError_t launch_pnp_reproj_mean(const double *p3, const double *p2, int32_t n, int32_t P, const double *poses,
                                  const double *cams, const uint8_t *masks, double *out, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_reproj_mean, dim3(P), dim3(64), 0, s, p3, p2, n, poses, cams, masks, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Geodesy and the DEM ray march (rsac_geo.h): one lane per point / ray
// ---------------------------------------------------------------------------
__global__ void k_utm_inverse(const double *__restrict__ en, int64_t n, TmConst k, UtmZone z,
                              double *__restrict__ lonlat) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        utm_inverse(k, z, en[2 * i], en[2 * i + 1], lonlat[2 * i], lonlat[2 * i + 1]);
}

__global__ void k_utm_forward(const double *__restrict__ lonlat, int64_t n, TmConst k, UtmZone z,
                              double *__restrict__ en) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        utm_forward(k, z, lonlat[2 * i], lonlat[2 * i + 1], en[2 * i], en[2 * i + 1]);
}

// Position of step base + t of one coordinate: closed form when the stride is
// exact (stride_closed_form), else the reference's additions one by one with
// thread t keeping the value at its step.  Returns the position at base + W.
template <int W>
__device__ __forceinline__ double stride_positions(double x, double c, int t, double &xt) {
    double delta;
    if (stride_closed_form(x, c, W, delta)) {
        xt = x + (double)t * delta;
        return x + (double)W * delta;
    }
    xt = x;
#pragma unroll 4
    for (int j = 0; j < W; ++j) {
        if (j == t) xt = x;
        x = x + c;
    }
    return x;
}

// ray_intersect_dem (main_v1.py:635-656), WPR waves per ray.  The block's
// W = 64 * WPR threads evaluate W consecutive steps of one ray at a time
// (thread t: step base + t); the ray's positions follow the reference's
// sequential additions exactly (stride_positions).  The first step, in order,
// that leaves the DEM (status 2) or hits (status 0) ends the ray.
template <int WPR>
__global__ __launch_bounds__(256) void k_dem_march(const double *__restrict__ o, const double *__restrict__ d,
                                                   int32_t n, DemGrid g, TmConst k, UtmZone z, int32_t n_steps,
                                                   double step, int32_t min_steps, double *__restrict__ hits,
                                                   int8_t *__restrict__ status) {
    static_assert(WPR == 1 || WPR == 4, "barriers assume one ray per block when WPR > 1");
    constexpr int W = 64 * WPR;
    constexpr int kRaysPerBlock = 4 / WPR;
    __shared__ int first[2][WPR];
    const int t = threadIdx.x % W;
    const int slot = threadIdx.x / W;
    const int ray = blockIdx.x * kRaysPerBlock + slot;
    const int lane = threadIdx.x & 63, wave = t >> 6;
    const bool live = ray < n;  // uniform per ray group; dead groups still join the barriers
    const int r = live ? ray : 0;
    double p0 = o[3 * r], p1 = o[3 * r + 1], p2 = o[3 * r + 2];
    const double c0 = step * d[3 * r], c1 = step * d[3 * r + 1], c2 = step * d[3 * r + 2];
    int found = -1;  // the chunk thread whose step ended the ray (uniform per ray)
    bool found_off = false;
    double q0 = 0.0, q1 = 0.0, q2 = 0.0;
    int parity = 0;
    for (int base = 0; base < n_steps; base += W) {
        p0 = stride_positions<W>(p0, c0, t, q0);
        p1 = stride_positions<W>(p1, c1, t, q1);
        p2 = stride_positions<W>(p2, c2, t, q2);
        const int s = base + t;
        bool ev = false;
        if (live && s < n_steps) {
            double lon, lat, elev;
            utm_inverse_fast(k, z, q0, q1, lon, lat);
            found_off = !dem_interp(g, lat, lon, elev);
            ev = found_off || (s >= min_steps && q2 <= elev);
        }
        const unsigned long long m = __ballot(ev);
        int f = m ? (wave * 64 + __builtin_ctzll(m)) : W;
        if constexpr (WPR > 1) {
            if (lane == 0) first[parity][wave] = f;
            __syncthreads();
            f = W;
            for (int w = 0; w < WPR; ++w) f = min(f, first[parity][w]);
            parity ^= 1;
        }
        if (f < W) {
            found = f;
            break;
        }
    }
    if (!live) return;
    const double nan = __builtin_nan("");
    if (found < 0) {
        if (t == 0) {
            hits[3 * ray] = nan;
            hits[3 * ray + 1] = nan;
            hits[3 * ray + 2] = nan;
            status[ray] = 1;
        }
    } else if (t == found) {
        hits[3 * ray] = found_off ? nan : q0;
        hits[3 * ray + 1] = found_off ? nan : q1;
        hits[3 * ray + 2] = found_off ? nan : q2;
        status[ray] = found_off ? 2 : 0;
    }
}

hipError_t launch_utm(bool inverse, const double *in, int64_t n, int zone, bool south, double *out, hipStream_t s) {
    const TmConst k = tm_const();
    const UtmZone z = utm_zone(zone, south);
    unsigned g = cdiv(n > 0 ? n : 1, 256);
    if (g > 4096) g = 4096;
    if (inverse)
        hipLaunchKernelGGL(k_utm_inverse, dim3(g), dim3(256), 0, s, in, n, k, z, out);
    else
        hipLaunchKernelGGL(k_utm_forward, dim3(g), dim3(256), 0, s, in, n, k, z, out);
    return hipGetLastError();
}

hipError_t launch_dem_march(const double *o, const double *d, int32_t n, const double *dem, int32_t ny, int32_t nx,
                            double y0, double dy, double x0, double dx, int zone, bool south, int32_t n_steps,
                            double step, int32_t min_steps, double *hits, int8_t *status, hipStream_t s) {
    const DemGrid g{dem, ny, nx, y0, dy, x0, dx};
    const TmConst k = tm_const();
    const UtmZone z = utm_zone(zone, south);
    // a block (4 waves, 256 steps per pass) per ray: measured faster than a wave per ray at every
    // batch size (64 / 1024 / 4096 rays: 0.20 / 0.38 / 0.85 ms vs 0.46 / 0.53 / 1.09 ms) -- the
    // rays' lengths differ by 10x, and per-ray blocks keep every SIMD busy to the end
    hipLaunchKernelGGL(k_dem_march<4>, dim3(n > 0 ? n : 1), dim3(256), 0, s, o, d, n, g, k, z, n_steps, step,
                       min_steps, hits, status);
    return hipGetLastError();
}

}  // namespace rsac
