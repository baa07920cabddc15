// RMSNorm forward / backward for gfx950.
//
// Memory-bound: one 256-thread workgroup per row, each lane owning ITERS
// 16-byte chunks (8 bf16) of the row in registers, so the row is read once
// and written once.  Optional fused residual add on the forward
// (h = x + r; y = norm(h)) and fused residual-gradient add on the backward
// (dx += dres) remove one full HBM pass each per transformer sub-block.
//
// dγ: each backward workgroup walks ROWS rows with a fixed lane->column map, so
// its γ-gradient partial stays in registers; partials [nblk, H] f32 are summed
// by a second tiny kernel (two-stage, no atomics -> bitwise reproducible).
#include "common.h"

namespace mx {

template <int ITERS, bool RESID>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
    const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
    uint16_t* __restrict__ h_out, float* __restrict__ rstd_out, int H, int ldy, float eps) {
  __shared__ float scratch[16];
  const int row = blockIdx.x;
  const size_t base = (size_t)row * H;
  float v[ITERS][8];
  float ss = 0.f;
  // gamma is loaded up front with the row, so its HBM latency overlaps the
  // row's instead of following the reduction (small-T decode calls are
  // latency-bound: one workgroup per row)
  u16x8 gw[ITERS];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < H) gw[it] = *reinterpret_cast<const u16x8*>(w + c);
  }
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < H) {
      u16x8 a = *reinterpret_cast<const u16x8*>(x + base + c);
      u16x8 hb;
      if constexpr (RESID) {
        u16x8 r = *reinterpret_cast<const u16x8*>(res + base + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float s = bf2f(a[j]) + bf2f(r[j]);
          hb[j] = f2bf(s);
          v[it][j] = bf2f(hb[j]);  // normalise the rounded residual, as stored
        }
        *reinterpret_cast<u16x8*>(h_out + base + c) = hb;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[it][j] = bf2f(a[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[it][j] * v[it][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[it][j] = 0.f;
    }
  }
  ss = block_sum(ss, scratch);
  const float rs = rsqrtf(ss / (float)H + eps);
  if (threadIdx.x == 0) rstd_out[row] = rs;
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < H) {
      const u16x8 g = gw[it];
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[it][j] * rs * bf2f(g[j]));
      *reinterpret_cast<u16x8*>(y + (size_t)row * ldy + c) = o;
    }
  }
}

// dx = rstd * (dy*w - x * rstd^2 * mean(dy*w*x))  [+ dres]
// dwp[blk, :] = sum_{rows of blk} dy * x * rstd
template <int ITERS, bool DRES, bool DW>
__global__ void __launch_bounds__(256) rmsnorm_bwd_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
    const uint16_t* __restrict__ w, const float* __restrict__ rstd,
    const uint16_t* __restrict__ dres, uint16_t* __restrict__ dx,
    float* __restrict__ dwp, int T, int H, int ldr, int ldx, int rows_per_blk) {
  __shared__ float scratch[16];
  float gw[ITERS][8];
  float acc[ITERS][8];
#pragma unroll
  for (int it = 0; it < ITERS; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[it][j] = 0.f;
    if (c < H) {
      u16x8 g = *reinterpret_cast<const u16x8*>(w + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) gw[it][j] = bf2f(g[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gw[it][j] = 0.f;
    }
  }
  const int r0 = blockIdx.x * rows_per_blk;
  const int r1 = min(T, r0 + rows_per_blk);
  for (int row = r0; row < r1; ++row) {
    const size_t base = (size_t)row * H;
    const float rs = rstd[row];
    float xv[ITERS][8], gv[ITERS][8];
    u16x8 rv[ITERS];  // the residual gradient, loaded with x / dy so its latency hides under the row sum
    float dot = 0.f;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int c = (it * 256 + threadIdx.x) * 8;
      if (c < H) {
        u16x8 a = *reinterpret_cast<const u16x8*>(x + base + c);
        u16x8 d = *reinterpret_cast<const u16x8*>(dy + base + c);
        if constexpr (DRES) rv[it] = *reinterpret_cast<const u16x8*>(dres + (size_t)row * ldr + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xv[it][j] = bf2f(a[j]);
          const float dd = bf2f(d[j]);
          gv[it][j] = dd * gw[it][j];
          dot += gv[it][j] * xv[it][j];
          if constexpr (DW) acc[it][j] += dd * xv[it][j] * rs;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { xv[it][j] = 0.f; gv[it][j] = 0.f; }
      }
    }
    dot = block_sum(dot, scratch);
    const float k = dot * rs * rs * rs / (float)H;
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int c = (it * 256 + threadIdx.x) * 8;
      if (c < H) {
        u16x8 o;
        if constexpr (DRES) {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(rs * gv[it][j] - xv[it][j] * k + bf2f(rv[it][j]));
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = f2bf(rs * gv[it][j] - xv[it][j] * k);
        }
        *reinterpret_cast<u16x8*>(dx + (size_t)row * ldx + c) = o;
      }
    }
  }
  if constexpr (DW) {
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int c = (it * 256 + threadIdx.x) * 8;
      if (c < H) {
        float* p = dwp + (size_t)blockIdx.x * H + c;
        *reinterpret_cast<f32x4*>(p) = f32x4{acc[it][0], acc[it][1], acc[it][2], acc[it][3]};
        *reinterpret_cast<f32x4*>(p + 4) = f32x4{acc[it][4], acc[it][5], acc[it][6], acc[it][7]};
      }
    }
  }
}

// Sum partials [nblk, H] over nblk -> out[H] f32.  Block = 64 column-lanes x 4
// row-slices, each lane owning 4 consecutive columns (16-B loads); the 4 slices
// are combined through LDS.  Deterministic (fixed order, no atomics).
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ p, float* __restrict__ out,
                                                     int nblk, int H) {
  __shared__ f32x4 red[4][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + cl) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < H) {
#pragma unroll 8
    for (int b = sl; b < nblk; b += 4) s += *reinterpret_cast<const f32x4*>(p + (size_t)b * H + c);
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < H) {
    f32x4 t = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    *reinterpret_cast<f32x4*>(out + c) = t;
  }
}

}  // namespace mx

using namespace mx;

#define FWD_CASE(IT)                                                                                  \
  case IT:                                                                                            \
    if (res)                                                                                          \
      rmsnorm_fwd_kernel<IT, true><<<T, 256, 0, stream>>>(x, res, w, y, h_out, rstd, H, ldy, eps);     \
    else                                                                                              \
      rmsnorm_fwd_kernel<IT, false><<<T, 256, 0, stream>>>(x, res, w, y, h_out, rstd, H, ldy, eps);    \
    break;

static int iters_for(int H) {
  const int chunks = (H / 8 + 255) / 256;
  if (chunks <= 1) return 1;
  if (chunks <= 2) return 2;
  if (chunks <= 4) return 4;
  return 8;
}

// ldy: row stride of y in elements (>= H, multiple of 8): y may be the left part of a
// wider buffer (the LoRA-augmented GEMM input [x | s t], mxllm/ops/linear.py)
extern "C" int mx_rmsnorm_fwd(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* y,
                              uint16_t* h_out, float* rstd, int T, int H, int ldy, float eps, hipStream_t stream) {
  if (H % 8 != 0 || H > 8 * 256 * 8 || T <= 0 || ldy < H || ldy % 8) return -1;
  switch (iters_for(H)) { FWD_CASE(1) FWD_CASE(2) FWD_CASE(4) FWD_CASE(8) }
  return (int)hipGetLastError();
}

#define BWD_LAUNCH(IT, DR, DW_)                                                                       \
  rmsnorm_bwd_kernel<IT, DR, DW_><<<nblk, 256, 0, stream>>>(dy, x, w, rstd, dres, dx, dwp, T, H, ldr, ldx, rpb)
#define BWD_CASE(IT)                                                                                  \
  case IT:                                                                                            \
    if (dres) {                                                                                       \
      if (dwp) BWD_LAUNCH(IT, true, true); else BWD_LAUNCH(IT, true, false);                          \
    } else {                                                                                          \
      if (dwp) BWD_LAUNCH(IT, false, true); else BWD_LAUNCH(IT, false, false);                        \
    }                                                                                                 \
    break;

// rows_per_blk chosen by the caller; dwp may be null (frozen γ).  Returns nblk.
// ldr / ldx: row strides (elements) of dres and dx (>= H, multiple of 8)
extern "C" int mx_rmsnorm_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* w, const float* rstd,
                              const uint16_t* dres, uint16_t* dx, float* dwp, int T, int H, int ldr, int ldx,
                              int rpb, hipStream_t stream) {
  if (H % 8 != 0 || H > 8 * 256 * 8 || T <= 0 || rpb <= 0 || ldx < H || ldx % 8 || (dres && (ldr < H || ldr % 8)))
    return -1;
  const int nblk = (T + rpb - 1) / rpb;
  switch (iters_for(H)) { BWD_CASE(1) BWD_CASE(2) BWD_CASE(4) BWD_CASE(8) }
  return (int)hipGetLastError();
}

extern "C" int mx_colsum_f32(const float* p, float* out, int nblk, int H, hipStream_t stream) {
  if (H % 4 != 0) return -1;
  colsum_kernel<<<(H / 4 + 63) / 64, 256, 0, stream>>>(p, out, nblk, H);
  return (int)hipGetLastError();
}
