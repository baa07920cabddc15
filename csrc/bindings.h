// C launch API of the mxllm gfx950 kernels (csrc/kernels/*.hip).
// All functions return 0 on success, a hipError_t (>0) or -1 on bad arguments.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {
// rmsnorm.hip
int mx_rmsnorm_fwd(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* y,
                   uint16_t* h_out, float* rstd, int T, int H, float eps, hipStream_t stream);
int mx_rmsnorm_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* w, const float* rstd,
                   const uint16_t* dres, uint16_t* dx, float* dwp, int T, int H, int rpb,
                   hipStream_t stream);
int mx_colsum_f32(const float* p, float* out, int nblk, int H, hipStream_t stream);

// misc.hip
int mx_segmented_mean_i32(const int32_t* codes, const int64_t* offs, float* out, int nseg,
                          hipStream_t stream);
int mx_sqnorm_f32(const float* x, int64_t n, float* out, hipStream_t stream);
}
