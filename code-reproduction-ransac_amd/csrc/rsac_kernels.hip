// rsac_kernels.hip -- gfx950 kernels of the RANSAC hot path.
//
//   pnp_prepare   f64 AoS (as numpy / cv2 hold it) -> f32 SoA, the CV_32F
//                 conversion of solvePnPRansac (main_v1.py:497)
//   pnp_solve     one LANE per hypothesis: Philox subset (or a host-made
//                 OpenCV subset), P3P in registers, 4th-point pick
//   pnp_score     hypotheses x points tile: points held in registers per
//                 lane, models in SGPRs (uniform scalar loads), inlier
//                 counts by ballot + popcount, block-reduced through LDS
//   pnp_mask      RANSAC-phase mask of the winners
//   hom_*         the same skeleton for cv2.findHomography (main_v1.py:312)
//
// Layout in HBM (per call, problem-concatenated): X[N] Y[N] Z[N] U[N] V[N]
// float32 (20 B per correspondence, the algorithmic bytes of SURVEY.md §8d);
// models [P][H][16] f64 (R 9, t 3, valid flag); counts [P][H] int32.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
// PnP: sample + minimal solve, one lane per hypothesis
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pnp_solve(PnpArgs a, int64_t hyp_begin, int32_t H) {
    const int prob = blockIdx.y;
    const int hl = blockIdx.x * blockDim.x + threadIdx.x;
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
        st = pnp_minimal(X, Y, Z, U, V, k, R, t) ? 1 : 0;
    }
#pragma unroll
    for (int q = 0; q < 9; ++q) m[q] = R[q];
#pragma unroll
    for (int q = 0; q < 3; ++q) m[9 + q] = t[q];
    m[kValidSlot] = st > 0 ? 1.0 : 0.0;
    a.status[rec] = st;
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
            if (m[kValidSlot] == 0.0) continue;
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
    if (threadIdx.x < nh) {
        const int s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        counts[(int64_t)prob * a.hyp_stride + h0 + threadIdx.x] = s;
    }
}

// mask of one model per problem (best[prob] indexes the models buffer; <0 = none)
__global__ void k_pnp_mask(PnpArgs a, const int64_t *__restrict__ best, uint8_t *__restrict__ mask) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t b = best[prob];
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

__global__ void k_hom_mask(HomArgs a, const int64_t *__restrict__ best, uint8_t *__restrict__ mask) {
    const int prob = blockIdx.y;
    const int64_t p0 = a.offsets[prob];
    const int n = (int)(a.offsets[prob + 1] - p0);
    const int64_t b = best[prob];
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

__global__ void k_gather_models(const double *__restrict__ models, const int64_t *__restrict__ rec, int32_t P,
                                double *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P * kModelStride) return;
    const int p = i / kModelStride, q = i % kModelStride;
    const int64_t r = rec[p];
    out[i] = r >= 0 ? models[r * kModelStride + q] : 0.0;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static inline unsigned cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

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

hipError_t launch_pnp_solve(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s) {
    hipLaunchKernelGGL(k_pnp_solve, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H);
    return hipGetLastError();
}

hipError_t launch_pnp_score(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    hipLaunchKernelGGL((k_pnp_score<kScoreP, kScoreHB>), dim3(cdiv(H, kScoreHB), P), dim3(256), 0, s, a, hyp_begin, H,
                       counts);
    return hipGetLastError();
}

hipError_t launch_pnp_mask(const PnpArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pnp_mask, dim3(g, P), dim3(256), 0, s, a, best, mask);
    return hipGetLastError();
}

hipError_t launch_hom_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s) {
    hipLaunchKernelGGL(k_hom_solve, dim3(cdiv(H, 256), P), dim3(256), 0, s, a, hyp_begin, H);
    return hipGetLastError();
}

hipError_t launch_hom_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s) {
    hipLaunchKernelGGL((k_hom_score<kScoreP, kScoreHB>), dim3(cdiv(H, kScoreHB), P), dim3(256), 0, s, a, hyp_begin, H,
                       counts);
    return hipGetLastError();
}

hipError_t launch_hom_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s) {
    unsigned g = cdiv(max_n > 0 ? max_n : 1, 256);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_hom_mask, dim3(g, P), dim3(256), 0, s, a, best, mask);
    return hipGetLastError();
}

hipError_t launch_gather_models(const double *models, const int64_t *rec, int32_t P, double *out, hipStream_t s) {
    hipLaunchKernelGGL(k_gather_models, dim3(cdiv((int64_t)P * kModelStride, 256)), dim3(256), 0, s, models, rec, P,
                       out);
    return hipGetLastError();
}

}  // namespace rsac
