// Microbenchmark: cycles per (hypothesis, point) pair of two inner loops of the PnP scoring test
// on gfx950, all CUs busy, 4 waves per SIMD, data in L2:
//   VALU  : the k_pnp_score_sc loop (8 points per lane in registers, a hypothesis record from
//           LDS, 9 FMA + q1 q2 + D + t + compare/ballot + min3 per pair)
//   MFMA  : xs, ys, z' of 8 hypotheses x 32 points from one v_mfma_f32_32x32x16_f16 (f16 hi/lo
//           operands), then the same q1 q2 D t test on the VALU (7.5 instructions per pair);
//           inlier counts by ballot popcounts (MODE 1) or per-lane VALU counters (MODE 2)
// Prints ms and pairs/s; the real kernel's rate is 1e9 pairs in ~0.35 ms (C2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int NPTS = 10240;  // points per problem (L2 resident)

// ---------------------------------------------------------------- VALU form
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_valu(
    const float *__restrict__ X, const float *__restrict__ Y, const float *__restrict__ Z,
    const float *__restrict__ U, const float *__restrict__ V, const float *__restrict__ rec, int units,
    int *__restrict__ out) {
    constexpr int P = 8, HB = 32;
    __shared__ float mlds[HB * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x < HB * 16) mlds[threadIdx.x] = rec[threadIdx.x];
    if (threadIdx.x + 256 < HB * 16) mlds[threadIdx.x + 256] = rec[threadIdx.x + 256];
    __syncthreads();
    int total = 0;
    uint32_t wundall = 0;
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        int cnt = 0;
        for (int base = wave * 64 * P; base < NPTS; base += 4 * 64 * P) {
            float px[P], py[P], pz[P], pu[P], pv[P];
#pragma unroll
            for (int j = 0; j < P; ++j) {
                const int i = base + j * 64 + lane;
                px[j] = X[i]; py[j] = Y[i]; pz[j] = Z[i]; pu[j] = U[i]; pv[j] = V[i];
            }
            int ccl = 0;
            uint32_t wund = 0;
#pragma unroll 4
            for (int h = 0; h < HB; ++h) {
                const float *m = mlds + h * 16;
                int cc = 0;
                float tmin = __builtin_inff();
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const float xs = __builtin_fmaf(m[2], pz[j], __builtin_fmaf(m[1], py[j], __builtin_fmaf(m[0], px[j], m[9])));
                    const float ys = __builtin_fmaf(m[5], pz[j], __builtin_fmaf(m[4], py[j], __builtin_fmaf(m[3], px[j], m[10])));
                    const float z = __builtin_fmaf(m[8], pz[j], __builtin_fmaf(m[7], py[j], __builtin_fmaf(m[6], px[j], m[11])));
                    const float q1 = __builtin_fmaf(pu[j], z, xs), q2 = __builtin_fmaf(pv[j], z, ys);
                    const float D = __builtin_fmaf(-z, z, __builtin_fmaf(q1, q1, q2 * q2));
                    const float tt = __builtin_fmaf(-m[12], __builtin_fabsf(z), __builtin_fabsf(D));
                    cc += __popcll(__ballot(D < 0.f));
                    tmin = __builtin_fminf(tmin, tt);
                }
                const uint64_t und = __ballot(!(tmin > m[13]));
                asm("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(ccl) : "s"(cc), "s"(h) : "m0");
                wund |= und ? (1u << h) : 0u;
            }
            cnt += ccl;
            wundall |= wund;
        }
        total += cnt;
    }
    out[blockIdx.x * 256 + threadIdx.x] = total + (int)wundall;
}

// ---------------------------------------------------------------- MFMA form
// A operands: NT groups of 8 hypotheses (lane row = lane & 31: hypothesis 2 (r>>2)... see kernel
// notes), band slopes a per (group, slot); B: per point 8 f16 (Xh Yh Zh Ch Xl Yl Zl Cl)
template <int MODE, int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_mfma(
    const uint4 *__restrict__ PF, const float *__restrict__ U, const float *__restrict__ V,
    const uint4 *__restrict__ AO, const float *__restrict__ AS, int units, int *__restrict__ out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31;
    h8 A[NT];
    float av[NT][4], tmin[NT][4];
    int vc[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        A[t] = __builtin_bit_cast(h8, AO[t * 64 + lane]);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            av[t][g] = AS[(t * 4 + g) * 64 + lane];
            tmin[t][g] = __builtin_inff();
            vc[t][g] = 0;
        }
    }
    int sc[NT][4][2];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) sc[t][g][0] = sc[t][g][1] = 0;
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        for (int base = wave * 32; base < NPTS; base += 4 * 32) {
            const int i = base + col;
            const h8 B = __builtin_bit_cast(h8, PF[i]);
            const float pu = U[i], pv = V[i];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f16v acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[t], B, f16v{}, 0, 0, 0);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float xs = acc[4 * g], ys = acc[4 * g + 1], z = acc[4 * g + 2];
                    const float q1 = __builtin_fmaf(pu, z, xs), q2 = __builtin_fmaf(pv, z, ys);
                    const float D = __builtin_fmaf(-z, z, __builtin_fmaf(q1, q1, q2 * q2));
                    const float tt = __builtin_fmaf(-av[t][g], __builtin_fabsf(z), __builtin_fabsf(D));
                    tmin[t][g] = __builtin_fminf(tmin[t][g], tt);
                    if constexpr (MODE == 1) {
                        const uint64_t m = __ballot(D < 0.f);
                        sc[t][g][0] += __popc((uint32_t)m);
                        sc[t][g][1] += __popc((uint32_t)(m >> 32));
                    } else {
                        vc[t][g] += D < 0.f ? 1 : 0;
                    }
                }
            }
        }
    }
    int r = 0;
    float tm = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            r += vc[t][g] + sc[t][g][0] * 3 + sc[t][g][1] * 5;
            tm += tmin[t][g];
        }
    out[blockIdx.x * 256 + threadIdx.x] = r + (tm > 1e30f ? 1 : 0);
}


__device__ __forceinline__ float amin3(float a, float b, float c) {
    float d;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ float amin3abs(float a, float b, float c) {
    float d;
    asm("v_min3_f32 %0, %1, |%2|, |%3|" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ uint32_t sgn(float x) { return __builtin_bit_cast(uint32_t, x) >> 31; }

// two 32-point tiles per iteration: the count of a slot adds both tiles' sign bits (v_add3), the
// band minimum folds both tiles' values (v_min3); CB: constant band (min over |D|)
template <bool CB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_mfma2(
    const uint4 *__restrict__ PF, const float *__restrict__ U, const float *__restrict__ V,
    const uint4 *__restrict__ AO, const float *__restrict__ AS, int units, int *__restrict__ out) {
    constexpr int NT = 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane & 31;
    h8 A[NT];
    float av[NT][4], tmin[NT][4];
    uint32_t vc[NT][4];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        A[t] = __builtin_bit_cast(h8, AO[t * 64 + lane]);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            av[t][g] = AS[(t * 4 + g) * 64 + lane];
            tmin[t][g] = __builtin_inff();
            vc[t][g] = 0;
        }
    }
    for (int u = blockIdx.x; u < units; u += gridDim.x) {
        for (int base = wave * 64; base < NPTS; base += 4 * 64) {
            const int i = base + col, i2 = i + 32;
            const h8 Ba = __builtin_bit_cast(h8, PF[i]);
            const h8 Bb = __builtin_bit_cast(h8, PF[i2]);
            const float pua = U[i], pva = V[i], pub = U[i2], pvb = V[i2];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const f16v aa = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[t], Ba, f16v{}, 0, 0, 0);
                const f16v ab = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[t], Bb, f16v{}, 0, 0, 0);
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const float za = aa[4 * g + 2], zb = ab[4 * g + 2];
                    const float q1a = __builtin_fmaf(pua, za, aa[4 * g]), q2a = __builtin_fmaf(pva, za, aa[4 * g + 1]);
                    const float q1b = __builtin_fmaf(pub, zb, ab[4 * g]), q2b = __builtin_fmaf(pvb, zb, ab[4 * g + 1]);
                    const float Da = __builtin_fmaf(-za, za, __builtin_fmaf(q1a, q1a, q2a * q2a));
                    const float Db = __builtin_fmaf(-zb, zb, __builtin_fmaf(q1b, q1b, q2b * q2b));
                    if constexpr (CB) {
                        tmin[t][g] = amin3abs(tmin[t][g], Da, Db);
                    } else {
                        const float ta = __builtin_fmaf(-av[t][g], __builtin_fabsf(za), __builtin_fabsf(Da));
                        const float tb = __builtin_fmaf(-av[t][g], __builtin_fabsf(zb), __builtin_fabsf(Db));
                        tmin[t][g] = amin3(tmin[t][g], ta, tb);
                    }
                    vc[t][g] += sgn(Da) + sgn(Db);
                }
            }
        }
    }
    int r = 0;
    float tm = 0.f;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            r += (int)vc[t][g];
            tm += tmin[t][g];
        }
    out[blockIdx.x * 256 + threadIdx.x] = r + (tm > 1e30f ? 1 : 0);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4;  // 4 waves per SIMD
    const int units = blocks * 8;  // each block: 8 units of 32 hypotheses x NPTS points
    std::vector<float> h(NPTS * 5);
    for (int i = 0; i < NPTS * 5; ++i) h[i] = (float)((i * 7919) % 1000) * 0.37f - 150.f;
    std::vector<float> rec(32 * 16);
    for (int i = 0; i < 32 * 16; ++i) rec[i] = (float)((i * 131) % 97) * 0.01f - 0.4f;
    std::vector<uint16_t> pf(NPTS * 8), ao(4 * 64 * 8);
    for (size_t i = 0; i < pf.size(); ++i) { _Float16 v = (_Float16)((float)((i * 37) % 200) * 0.5f - 50.f); pf[i] = __builtin_bit_cast(uint16_t, v); }
    for (size_t i = 0; i < ao.size(); ++i) { _Float16 v = (_Float16)((float)((i * 53) % 100) * 0.02f - 1.f); ao[i] = __builtin_bit_cast(uint16_t, v); }
    std::vector<float> as(4 * 4 * 64, 0.01f);
    float *dX, *drec, *das;
    uint4 *dpf, *dao;
    int *dout;
    hipMalloc(&dX, sizeof(float) * NPTS * 5);
    hipMalloc(&drec, sizeof(float) * 32 * 16);
    hipMalloc(&dpf, sizeof(uint16_t) * pf.size());
    hipMalloc(&dao, sizeof(uint16_t) * ao.size());
    hipMalloc(&das, sizeof(float) * as.size());
    hipMalloc(&dout, sizeof(int) * blocks * 256);
    hipMemcpy(dX, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice);
    hipMemcpy(drec, rec.data(), sizeof(float) * rec.size(), hipMemcpyHostToDevice);
    hipMemcpy(dpf, pf.data(), sizeof(uint16_t) * pf.size(), hipMemcpyHostToDevice);
    hipMemcpy(dao, ao.data(), sizeof(uint16_t) * ao.size(), hipMemcpyHostToDevice);
    hipMemcpy(das, as.data(), sizeof(float) * as.size(), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double pairs = (double)units * 32 * NPTS;
    const char *names[] = {"VALU sc loop", "MFMA NT=4 ballot", "MFMA NT=4 vcount", "MFMA NT=2 ballot",
                           "MFMA NT=2 vcount", "MFMA2 slope add3", "MFMA2 CB add3"};
    for (int m = 0; m < 7; ++m) {
        auto launch = [&]() {
            const float *U = dX + 3 * NPTS, *V = dX + 4 * NPTS;
            switch (m) {
                case 0: hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, dX, dX + NPTS, dX + 2 * NPTS, U, V, drec, units, dout); break;
                case 1: hipLaunchKernelGGL((k_mfma<1, 4>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units, dout); break;
                case 2: hipLaunchKernelGGL((k_mfma<2, 4>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units, dout); break;
                // NT = 2: 16 hypotheses per wave-tile, twice the units for the same pairs
                case 3: hipLaunchKernelGGL((k_mfma<1, 2>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units * 2, dout); break;
                case 4: hipLaunchKernelGGL((k_mfma<2, 2>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units * 2, dout); break;
                case 5: hipLaunchKernelGGL((k_mfma2<false>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units, dout); break;
                case 6: hipLaunchKernelGGL((k_mfma2<true>), dim3(blocks), dim3(256), 0, 0, dpf, U, V, dao, das, units, dout); break;
            }
        };
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        printf("%-20s %.3f ms  %.3g pairs/s  -> 1e9 pairs in %.3f ms\n", names[m], ms, pairs / (ms * 1e-3),
               1e9 / (pairs / (ms * 1e-3)) * 1e3);
    }
    return 0;
}
