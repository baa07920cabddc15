// Shared pieces of the fused decode GEMMs (skinny_gemm.hip bf16 weights, fp8_gemm.hip e4m3
// weights): the RMSNorm prologue and the SwiGLU / RoPE+KV-append epilogues.  Every piece
// reproduces the rounding of the standalone kernel it replaces (rmsnorm.hip forward,
// elementwise.hip SwiGLU, decode.hip rope_append), so a fused step is bit-identical.
#pragma once

#include "common.h"

namespace mx {

// the same expression as the SwiGLU kernels (elementwise.hip sigmoid_f): bit-identical outputs
__device__ __forceinline__ float dfuse_silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

struct SkNorm {
  const uint16_t* delta;  // [M, K] sub-block output added to the residual (nullptr: plain RMSNorm)
  int64_t ldd;
  const uint16_t* gamma;  // [K]
  uint16_t* h_out;        // [M, K] (row stride K): h + delta, written by workgroup 0
  float eps;
};

struct SkRope {
  const float* cosb;     // [max_pos, 64]
  const float* sinb;
  const int32_t* pos;    // [M] position of the new token
  const int32_t* slots;  // [M] cache slot (nullptr: row index)
  uint16_t* q;           // [M, Hq, 128]
  uint16_t* kc;          // [slots, Hkv, max_seq, 128], or paged [blocks, Hkv, block, 128]
  uint16_t* vc;
  int Hq, Hkv, max_seq;  // max_seq: the cache's sequence dimension (the block size when paged)
  const int32_t* bt;     // paged: block table [slots, maxb] (nullptr: contiguous)
  int maxb;
};

// Weight row of channel c (0..15) of workgroup blk in the paired layouts:
//  SWO : 8 gate rows blk*8 .. +7 and the matching up rows F + blk*8 .. +7;
//  ROPE: head blk/8, first-half rows 8 (blk%8) .. +7 and the matching second-half rows (+64).
template <bool SWO>
__device__ __forceinline__ int64_t dfuse_row(int blk, int c, int F) {
  if constexpr (SWO) return (int64_t)blk * 8 + (c & 7) + (c >= 8 ? F : 0);
  else return (int64_t)(blk >> 3) * 128 + (blk & 7) * 8 + (c & 7) + (c >= 8 ? 64 : 0);
}

// RMSNorm (with the residual add when na.delta) of M <= 4 rows of X into xs [M, K] (LDS),
// by a 512-thread workgroup: rows m = q, q + 2, ... by wave group q, each group with
// rmsnorm.hip's 256-thread mapping and summation order.  Workgroup 0 stores h + delta.
__device__ __forceinline__ void dfuse_norm_rows(const uint16_t* __restrict__ X, int64_t ldx, int M, int K,
                                                const SkNorm& na, uint16_t* xs, float (*nscr)[4], float* nrs) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int q = w >> 2, tq = tid & 255;
  for (int m0 = 0; m0 < M; m0 += 2) {
    const int m = m0 + q;
    float ss = 0.f;
    if (m < M) {
      for (int cc = tq * 8; cc < K; cc += 2048) {
        const u16x8 hv = *reinterpret_cast<const u16x8*>(X + (int64_t)m * ldx + cc);
        u16x8 hb = hv;
        if (na.delta) {
          const u16x8 dv = *reinterpret_cast<const u16x8*>(na.delta + (int64_t)m * na.ldd + cc);
#pragma unroll
          for (int j = 0; j < 8; ++j) hb[j] = f2bf(bf2f(dv[j]) + bf2f(hv[j]));
          if (blockIdx.x == 0) *reinterpret_cast<u16x8*>(na.h_out + (int64_t)m * K + cc) = hb;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(hb[j]);
          ss += v * v;
        }
        *reinterpret_cast<u16x8*>(xs + (int64_t)m * K + cc) = hb;
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) nscr[q][w & 3] = ss;
    __syncthreads();
    if (m < M && tq == 0) {
      float r = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) r += nscr[q][i];
      nrs[m] = rsqrtf(r / (float)K + na.eps);
    }
    __syncthreads();
  }
  // normalise in place (each thread rewrites the chunks it stored)
  for (int m0 = 0; m0 < M; m0 += 2) {
    const int m = m0 + q;
    if (m < M) {
      const float rs = nrs[m];
      for (int cc = tq * 8; cc < K; cc += 2048) {
        u16x8* px = reinterpret_cast<u16x8*>(xs + (int64_t)m * K + cc);
        const u16x8 hb = *px;
        const u16x8 gw = *reinterpret_cast<const u16x8*>(na.gamma + cc);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(hb[j]) * rs * bf2f(gw[j]));
        *px = o;
      }
    }
  }
  __syncthreads();
}

// Split-K decode attention partials (decode.hip decode_attn_*: per (row, q-head, split) the
// running max / sum in part_ml [M, Hq, nsplit, 2] and the unnormalised output in part_o
// [M, Hq, nsplit, 128]) merged into the attention output rows xs [M, Hq * 128] (LDS) -- the
// o-projection GEMM's X -- with decode_combine_kernel's arithmetic and order (same bits).
struct SkMerge {
  const float* ml;
  const float* po;
  int nsplit;
};

__device__ __forceinline__ void dfuse_merge_rows(int M, int K, const SkMerge& mg, uint16_t* xs) {
  const int ns = mg.nsplit;
  for (int e = threadIdx.x * 8; e < M * K; e += blockDim.x * 8) {
    const int m = e / K, col = e % K, hq = col >> 7, d0 = col & 127;
    const int64_t bh = (int64_t)m * (K >> 7) + hq;
    const float* ml = mg.ml + bh * ns * 2;
    u16x8 out;
    if (ns <= 8) {
      float mv[8], lv[8];
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const bool on = s < ns;
        mv[s] = on ? ml[2 * s] : -INFINITY;
        lv[s] = on ? ml[2 * s + 1] : 0.f;
      }
      float Mx = -INFINITY;
#pragma unroll
      for (int s = 0; s < 8; ++s) Mx = fmaxf(Mx, mv[s]);
      float wgt[8], L = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        wgt[s] = mv[s] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mv[s] - Mx);
        if (mv[s] != -INFINITY) L += wgt[s] * lv[s];
      }
#pragma unroll
      for (int j = 0; j < 8; j += 4) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
          if (s < ns && mv[s] != -INFINITY) {
            const f32x4 ov = *reinterpret_cast<const f32x4*>(mg.po + (bh * ns + s) * 128 + d0 + j);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[i] += wgt[s] * ov[i];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) out[j + i] = f2bf(L > 0.f ? acc[i] / L : 0.f);
      }
    } else {
      float Mx = -INFINITY;
      for (int s = 0; s < ns; ++s) Mx = fmaxf(Mx, ml[2 * s]);
      float L = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < ns; ++s) {
        const float mm = ml[2 * s];
        if (mm == -INFINITY) continue;
        const float wg = __builtin_amdgcn_exp2f(mm - Mx);
        L += wg * ml[2 * s + 1];
        const float* op = mg.po + (bh * ns + s) * 128 + d0;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += wg * op[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) out[i] = f2bf(L > 0.f ? acc[i] / L : 0.f);
    }
    *reinterpret_cast<u16x8*>(xs + e) = out;
  }
  __syncthreads();
}

// Epilogues.  Lane (c, g) of the reducing wave holds v = channels 4g..4g+3 (final f32 values,
// weight scale applied) of token m = c (+ 16 mb); the paired channels are in lane ^ 32.  Every
// lane of the wave must call (the pairing is a lane shuffle).
__device__ __forceinline__ void dfuse_swiglu_store(const f32x4& v, int g, int m, int M, uint16_t* Y, int64_t ldy,
                                                   int blk) {
  f32x4 up;
#pragma unroll
  for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(v[i], 32, 64);
  if (g < 2 && m < M) {
    u16x4 o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = f2bf(dfuse_silu(bf2f(f2bf(v[i]))) * bf2f(f2bf(up[i])));
    *reinterpret_cast<u16x4*>(Y + (int64_t)m * ldy + (int64_t)blk * 8 + 4 * g) = o;
  }
}

__device__ __forceinline__ void dfuse_rope_store(const f32x4& v, int g, int m, int M, int blk, const SkRope& rp) {
  f32x4 hi;
#pragma unroll
  for (int i = 0; i < 4; ++i) hi[i] = __shfl_xor(v[i], 32, 64);
  if (g < 2 && m < M) {
    const int head = blk >> 3, i0 = (blk & 7) * 8 + 4 * g;
    const int p = rp.pos[m];
    const int slot = rp.slots ? rp.slots[m] : m;
    u16x4 y1, y2;
    uint16_t* dst;
    if (head >= rp.Hq + rp.Hkv) {  // v: no rotation
#pragma unroll
      for (int i = 0; i < 4; ++i) y1[i] = f2bf(v[i]), y2[i] = f2bf(hi[i]);
      dst = rp.vc + kv_row(rp.bt, rp.maxb, rp.max_seq, slot, rp.Hkv, head - rp.Hq - rp.Hkv, p) * 128;
    } else {
      const float* cp = rp.cosb + (int64_t)p * 64 + i0;
      const float* sp = rp.sinb + (int64_t)p * 64 + i0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // rope_append's arithmetic on the bf16-rounded projection
        const float a = bf2f(f2bf(v[i])), bb = bf2f(f2bf(hi[i]));
        y1[i] = f2bf(a * cp[i] - bb * sp[i]);
        y2[i] = f2bf(bb * cp[i] + a * sp[i]);
      }
      dst = head < rp.Hq ? rp.q + ((int64_t)m * rp.Hq + head) * 128
                         : rp.kc + kv_row(rp.bt, rp.maxb, rp.max_seq, slot, rp.Hkv, head - rp.Hq, p) * 128;
    }
    *reinterpret_cast<u16x4*>(dst + i0) = y1;
    *reinterpret_cast<u16x4*>(dst + 64 + i0) = y2;
  }
}

}  // namespace mx
