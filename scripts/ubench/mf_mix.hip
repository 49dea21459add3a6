// Microbenchmark: the point loop of k_pnp_score_mf without its memory side.  Per iteration and
// wave: 4 MFMA groups x (2 v_mfma_f32_32x32x16_f16 + the VALU test of 8 pairs: q1 q2, D, t, the
// 255 x count by v_perm + v_sad_u8, the band minimum and its ballot), the same source as the
// kernel's body, operands in registers (made opaque per iteration so nothing is hoisted).  Prints
// the time per wave-iteration and the VALU issue rate per SIMD at 2, 3 and 4 blocks (waves per
// SIMD) per CU: the ceiling of the kernel's instruction mix, against which the kernel's own rate
// (profiles/pmc_score_issue.json) is read.
//   scripts/ubench/mf_mix.sh (counts each mode's loop instructions in the ISA, then builds)
#include <hip/hip_runtime.h>
#include <cstdio>
#ifndef SGB_VALU
#define SGB_VALU 64
#endif

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t cnt255(uint32_t c, float a, float b) {
    return __builtin_amdgcn_sad_u8(__builtin_amdgcn_perm(__float_as_uint(a), __float_as_uint(b), 0x0C0C0B09u), 0u, c);
}
struct Pair {
    float D, t;
};
__device__ __forceinline__ Pair pair(const f16v &x, int g, float2 uv, float ag) {
    const float z = x[4 * g + 2];
    const float q1 = __builtin_fmaf(uv.x, z, x[4 * g]);
    const float q2 = __builtin_fmaf(uv.y, z, x[4 * g + 1]);
    const float D = __builtin_fmaf(-z, z, __builtin_fmaf(q1, q1, q2 * q2));
    const float tt = __builtin_fmaf(-ag, __builtin_fabsf(z), __builtin_fabsf(D));
    return Pair{D, tt};
}

// MODE 0: the kernel's body; 1: no MFMA (its outputs made opaque per group instead); 2: MFMA and
// the FMAs of the pairs only (D summed, no count / band); 3: neither MFMA nor count / band;
// 4: the kernel's body with group t + 1's MFMAs issued before group t's VALU
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 8))) void k(float *out, int iters, float s) {
    const int lane = threadIdx.x & 63, half = lane >> 5;
    h8 Ar[4];
    float4 av[4], bv[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int e = 0; e < 8; ++e) Ar[t][e] = (_Float16)(s * (lane + e + t));
        av[t] = make_float4(1e-6f * s, 2e-6f * s, 3e-6f * s, 4e-6f * s);
        bv[t] = make_float4(-1e30f, -1e30f, -1e30f, -1e30f * s);  // the band never hit
    }
    h8 Ba, Bb;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        Ba[e] = (_Float16)(s * (lane - e));
        Bb[e] = (_Float16)(s * (lane + 2 * e));
    }
    float2 ua = make_float2(s * lane, -s * lane), ub = make_float2(0.5f * s, s + half);
    uint32_t vc[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) vc[t][g] = 0u;
    uint32_t flacc = 0;
    f16v xa0, xb0;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        xa0[e] = s * (lane + e);
        xb0[e] = s * (lane - e);
    }
    for (int i = 0; i < iters; ++i) {
        asm volatile("" : "+v"(Ba), "+v"(Bb), "+v"(ua), "+v"(ub));  // a new iteration's operands
        uint32_t fl = 0;
        f16v xa_n, xb_n;  // MODE 4: group t + 1's MFMAs issued before group t's VALU
        if constexpr (MODE == 4) {
            xa_n = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[0], Ba, f16v{}, 0, 0, 0);
            xb_n = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[0], Bb, f16v{}, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            f16v xa, xb;
            if constexpr (MODE == 4) {
                xa = xa_n;
                xb = xb_n;
                if (t < 3) {
                    xa_n = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t + 1], Ba, f16v{}, 0, 0, 0);
                    xb_n = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t + 1], Bb, f16v{}, 0, 0, 0);
                }
            } else if constexpr (MODE == 0 || MODE == 2) {
                xa = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t], Ba, f16v{}, 0, 0, 0);
                xb = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ar[t], Bb, f16v{}, 0, 0, 0);
            } else {  // loop-carried registers, declared rewritten: no instruction
                asm volatile("" : "+v"(xa0), "+v"(xb0));
                xa = xa0;
                xb = xb0;
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float ag = g == 0 ? av[t].x : g == 1 ? av[t].y : g == 2 ? av[t].z : av[t].w;
                const float bg = g == 0 ? bv[t].x : g == 1 ? bv[t].y : g == 2 ? bv[t].z : bv[t].w;
                const Pair ra = pair(xa, g, ua, ag), rb = pair(xb, g, ub, ag);
                if constexpr (MODE <= 1 || MODE == 4) {
                    vc[t][g] = cnt255(vc[t][g], ra.D, rb.D);
                    fl |= __ballot(!(__builtin_fminf(ra.t, rb.t) > bg)) ? (1u << (4 * t + g)) : 0u;
                } else {
                    vc[t][g] += __float_as_uint(ra.t + rb.t);
                }
            }
        }
        if constexpr (MODE == 4) {  // order: MFMA g0, MFMA g1, VALU g0, MFMA g2, VALU g1, MFMA g3, VALU g2, VALU g3
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, SGB_VALU, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, SGB_VALU, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, SGB_VALU, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, SGB_VALU, 0);
        }
        flacc |= fl;
    }
    uint32_t r = flacc;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) r += vc[t][g];
    out[blockIdx.x * 256 + threadIdx.x] = (float)r;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    (void)hipMalloc(&out, sizeof(float) * 256 * cus * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4000;
    const int valu[5] = {VALU0, VALU1, VALU2, VALU3, VALU4};  // per wave-iteration, from the ISA (incl. MFMA)
    const char *names[5] = {"kernel body", "no MFMA", "MFMA + pair FMAs", "pair FMAs only", "MFMA one group ahead"};
    for (int m = 0; m < 5; ++m)
        for (int bpc : {2, 3, 4}) {
            const int blocks = cus * bpc;  // 4 waves per block, one per SIMD
            auto launch = [&]() {
                switch (m) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f); break;
                }
            };
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            ms /= 5;
            const double cyc = ms * 1e-3 * 2.4e9;           // SIMD cycles at 2.4 GHz
            const double wave_iters = (double)bpc * iters;  // per SIMD
            const double per_quad = wave_iters * valu[m] / (cyc / 4.0);
            printf("%-18s blocks/CU %d: %.3f ms, %5.0f cycles per wave-iteration per SIMD, %.3f VALU per "
                   "quad-cycle (%.3f of 2; %d VALU per wave-iteration)\n",
                   names[m], bpc, ms, cyc / wave_iters, per_quad, per_quad / 2, valu[m]);
        }
    return 0;
}
