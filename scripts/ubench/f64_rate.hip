// Microbenchmark: f64 VALU costs on gfx950 for the P3P / EPnP solve kernels (one lane per
// hypothesis, all-f64 arithmetic).  For each operation: the issue cost (cycles per wave-instruction
// per SIMD, 8 independent chains per lane, 2 and 4 waves per SIMD) and the dependent latency
// (one chain, one wave per SIMD).  Cycles from s_memtime in every wave (the shader clock), wall
// time from HIP events.  The solve's `roofline_solve` weights its PMC instruction mix
// (SQ_INSTS_VALU_{FMA,MUL,ADD,TRANS}_F64, profiles/r04_solve_mix.json) by these costs.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/f64_rate scripts/ubench/f64_rate.hip && /tmp/f64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 1024;

__device__ __forceinline__ double op(int m, double x, double s) {
    switch (m) {
        case 0: return __builtin_fma(x, s, 0.5);              // v_fma_f64
        case 1: return x * s;                                  // v_mul_f64
        case 2: return x + s;                                  // v_add_f64
        case 3: return __builtin_amdgcn_rcp(x) + s;            // v_rcp_f64 (+ add)
        case 4: return __builtin_amdgcn_rsq(x) + s;            // v_rsq_f64 (+ add)
        case 5: return s / x;                                  // IEEE division (the compiler's sequence)
        case 6: return __builtin_sqrt(x) + s;                  // IEEE sqrt (the compiler's sequence) + add
        default: return __builtin_fma(x, s, 0.5);
    }
}

template <int M, int CH>
__global__ __launch_bounds__(256) void k(double *out, double s, long long *cyc) {
    double a[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) a[j] = 1.0 + 1e-3 * (threadIdx.x + j);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int j = 0; j < CH; ++j) a[j] = op(M, a[j], s);
        if (M >= 3) {
#pragma unroll
            for (int j = 0; j < CH; ++j) a[j] = a[j] * 0.5 + 0.75;  // keep the operands in range
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double r = 0;
#pragma unroll
    for (int j = 0; j < CH; ++j) r += a[j];
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int M, int CH>
void run(const char *name, int cus, double *out, long long *cyc, long long *hc, int wps, int extra_valu) {
    const int blocks = cus * wps;  // 256 threads = one wave per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((k<M, CH>), dim3(blocks), dim3(256), 0, 0, out, 0.999, cyc);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<M, CH>), dim3(blocks), dim3(256), 0, 0, out, 0.999, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(hc, cyc, sizeof(long long) * blocks * 4, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < blocks * 4; ++i) mean += (double)hc[i];
    mean /= blocks * 4;
    // per wave: ITERS x CH operations; per SIMD wps waves share the issue
    const double per_op = mean / ((double)ITERS * CH);
    printf("%-34s chains %d waves/SIMD %d: %7.2f cycles per op per wave, %7.2f cycles per op per SIMD "
           "(%d extra VALU per op), wall %.3f ms, clock %.2f GHz\n",
           name, CH, wps, per_op, per_op / wps, extra_valu, ms, mean / (ms * 1e-3) * 1e-9);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double *out;
    long long *cyc;
    hipMalloc(&out, sizeof(double) * 256 * cus * 8);
    hipMalloc(&cyc, sizeof(long long) * cus * 8 * 4);
    long long *hc = new long long[cus * 8 * 4];
    printf("throughput (8 independent chains per lane)\n");
    for (int wps : {2, 4}) {
        run<0, 8>("v_fma_f64", cus, out, cyc, hc, wps, 0);
        run<1, 8>("v_mul_f64", cus, out, cyc, hc, wps, 0);
        run<2, 8>("v_add_f64", cus, out, cyc, hc, wps, 0);
        run<3, 8>("v_rcp_f64 + add + fma", cus, out, cyc, hc, wps, 2);
        run<4, 8>("v_rsq_f64 + add + fma", cus, out, cyc, hc, wps, 2);
        run<5, 8>("IEEE f64 division + fma", cus, out, cyc, hc, wps, 1);
        run<6, 8>("IEEE f64 sqrt + add + fma", cus, out, cyc, hc, wps, 2);
    }
    printf("latency (one chain, one wave per SIMD)\n");
    run<0, 1>("v_fma_f64", cus, out, cyc, hc, 1, 0);
    run<1, 1>("v_mul_f64", cus, out, cyc, hc, 1, 0);
    run<2, 1>("v_add_f64", cus, out, cyc, hc, 1, 0);
    run<3, 1>("v_rcp_f64 + add + fma", cus, out, cyc, hc, 1, 2);
    run<4, 1>("v_rsq_f64 + add + fma", cus, out, cyc, hc, 1, 2);
    run<5, 1>("IEEE f64 division + fma", cus, out, cyc, hc, 1, 1);
    run<6, 1>("IEEE f64 sqrt + add + fma", cus, out, cyc, hc, 1, 2);
    return 0;
}
