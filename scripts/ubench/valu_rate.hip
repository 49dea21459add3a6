// Microbenchmark: wave64 VALU issue rate on gfx950 for the instruction mixes of the PnP scoring
// kernels (plain f32 FMA, packed f32 FMA, FMA + v_cmp/ballot/popcount, FMA + MFMA).
// Prints cycles per VALU instruction per SIMD for 4 and 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int ITERS = 2048;

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, float s0, int *cnt) {
    float a[8];
    f2 p[4];
    for (int j = 0; j < 8; ++j) a[j] = s0 * (threadIdx.x + j);
    for (int j = 0; j < 4; ++j) p[j] = f2{a[2 * j], a[2 * j + 1]};
    int c = 0;
    h8 A = h8{1, 2, 3, 4, 5, 6, 7, 8};
    h8 B = h8{(_Float16)s0, 2, 3, 4, 5, 6, 7, 8};
    f16v acc = f16v{};
    for (int it = 0; it < ITERS; ++it) {
        if constexpr (MODE == 0) {  // 8 independent fma chains: 8 VALU
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], s0, 0.5f);
        } else if constexpr (MODE == 1) {  // 4 packed fma: 4 VALU, 8 FMAs
#pragma unroll
            for (int j = 0; j < 4; ++j) p[j] = __builtin_elementwise_fma(p[j], f2{s0, s0}, f2{0.5f, 0.5f});
        } else if constexpr (MODE == 2) {  // 8 fma + 2 cmp/ballot/popcount: 10 VALU + SALU
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], s0, 0.5f);
            c += __popcll(__ballot(a[0] < a[1]));
            c += __popcll(__ballot(a[2] > a[3]));
        } else if constexpr (MODE == 3) {  // 8 fma + 1 MFMA 32x32x16 f16 every iteration
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(A, B, acc, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], s0, 0.5f);
        } else if constexpr (MODE == 4) {  // 8 fma + 2 cmp counted per lane (v_cndmask/v_addc)
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = __builtin_fmaf(a[j], s0, 0.5f);
            c += a[0] < a[1] ? 1 : 0;
            c += a[2] > a[3] ? 1 : 0;
        }
    }
    float r = 0;
    for (int j = 0; j < 8; ++j) r += a[j];
    for (int j = 0; j < 4; ++j) r += p[j].x + p[j].y;
    for (int j = 0; j < 16; ++j) r += acc[j];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if (c == 12345) cnt[0] = c;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    int *cnt;
    hipMalloc(&out, sizeof(float) * 256 * cus * 16);
    hipMalloc(&cnt, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"8 fma", "4 pk_fma (8 FMAs)", "8 fma + 2 ballot/popc", "8 fma + 1 mfma32x32x16", "8 fma + 2 cmp->vcnt"};
    const int valu[] = {8, 4, 10, 8, 12};
    for (int wps : {4, 8}) {
        const int blocks = cus * wps;  // 256 threads = 4 waves = one per SIMD
        for (int m = 0; m < 5; ++m) {
            auto launch = [&]() {
                switch (m) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, cnt); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, cnt); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, cnt); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, cnt); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, 0.999f, cnt); break;
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
            // per SIMD: wps waves x ITERS x valu instructions
            const double instr = (double)wps * ITERS * valu[m];
            const double cyc = ms * 1e-3 * 2.4e9;
            printf("waves/SIMD %d  %-28s %.3f ms  %.2f cycles per VALU instr (at 2.4 GHz)\n", wps, names[m], ms,
                   cyc / instr);
        }
    }
    return 0;
}
