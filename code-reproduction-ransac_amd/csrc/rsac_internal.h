// rsac_internal.h -- kernel argument blocks and launchers shared by the
// kernels (rsac_kernels.hip) and the host driver (rsac_api.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsac {

// PnP problem set on the device.  Problem p owns points [offsets[p],
// offsets[p+1]) of the SoA arrays; its hypothesis records live at
// [p * hyp_stride, p * hyp_stride + H).
// Hypothesis h of problem p (h counted from the start of the call) is record
// p * hyp_stride + h; its Philox counter is (rng_base + h, stream), so a
// shard of one problem's hypothesis space is selected by rng_base.  Every
// problem of a batch uses the same stream (0): a batched call equals the loop
// of single calls it replaces, as each cv2 call restarts OpenCV's RNG.
struct PnpArgs {
    const float *X, *Y, *Z, *U, *V;
    const int64_t *offsets;  // P + 1
    const double *cams;      // P x (fx, fy, cx, cy)
    const float *thr2;       // P
    double *models;          // P x hyp_stride x 16
    int8_t *status;          // P x hyp_stride
    const int32_t *subsets;  // optional P x hyp_stride x 4 (OpenCV sampler)
    const int8_t *sub_status;
    int64_t hyp_stride;
    int64_t rng_base;
    uint64_t seed;
};

struct HomArgs {
    const float *SX, *SY, *DX, *DY;
    const int64_t *offsets;
    const float *thr2;
    double *models;
    int8_t *status;
    const int32_t *subsets;
    const int8_t *sub_status;
    int64_t hyp_stride;
    int64_t rng_base;
    uint64_t seed;
};

// copy model records rec[p] (<0: zero) into out[p][16]
hipError_t launch_gather_models(const double *models, const int64_t *rec, int32_t P, double *out, hipStream_t s);

hipError_t launch_pnp_prepare(const double *p3, const double *p2, int64_t n, float *X, float *Y, float *Z, float *U,
                              float *V, hipStream_t s);
hipError_t launch_hom_prepare(const double *src, const double *dst, int64_t n, float *SX, float *SY, float *DX,
                              float *DY, hipStream_t s);
// solve / score hypotheses [hyp_begin, hyp_begin + H) of every problem
hipError_t launch_pnp_solve(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s);
hipError_t launch_pnp_score(const PnpArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s);
hipError_t launch_pnp_mask(const PnpArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s);
hipError_t launch_hom_solve(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, hipStream_t s);
hipError_t launch_hom_score(const HomArgs &a, int32_t P, int64_t hyp_begin, int32_t H, int32_t *counts,
                            hipStream_t s);
hipError_t launch_hom_mask(const HomArgs &a, int32_t P, int32_t max_n, const int64_t *best, uint8_t *mask,
                           hipStream_t s);

}  // namespace rsac
