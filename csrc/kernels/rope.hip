// Llama-3 RoPE fused with the QKV head split / merge.
//
// forward  rope_split : qkv [T, (Hq+2Hkv)*D] token-major (the projection GEMM's
//   output) -> q [B,Hq,S,D], k [B,Hkv,S,D] rotated, v [B,Hkv,S,D] copied —
//   the head-major layout the attention kernels stage tiles from contiguously.
// backward rope_merge : attention's f32 dq [B,Hq,S,D] and per-q-head dk/dv
//   partials [B,Hq,S,D] -> GQA group sum + inverse rotation -> d(qkv) bf16
//   token-major, ready for the projection's backward GEMM.
// cos/sin come from a host-precomputed f32 table [P, D/2] (no device trig).
// "rotate-half" pairing: (x[i], x[i + D/2]).  Each lane owns 8 pairs = two
// 16-B chunks.
#include "common.h"

namespace mx {

template <int D>
__global__ void __launch_bounds__(256) rope_split_kernel(const uint16_t* __restrict__ qkv,
                                                         const float* __restrict__ cosb,
                                                         const float* __restrict__ sinb,
                                                         const int32_t* __restrict__ positions,
                                                         uint16_t* __restrict__ q, uint16_t* __restrict__ k,
                                                         uint16_t* __restrict__ v, int B, int S, int Hq, int Hkv) {
  constexpr int HALF = D / 2, CPH = HALF / 8;  // chunks per head
  const int NH = Hq + 2 * Hkv;
  const int64_t n = (int64_t)B * S * NH * CPH;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int cc = (int)(i % CPH);
    const int64_t th = i / CPH;
    const int head = (int)(th % NH);
    const int64_t t = th / NH;
    const int b = (int)(t / S), s = (int)(t % S);
    const int c = cc * 8;
    const uint16_t* src = qkv + t * (int64_t)NH * D + (int64_t)head * D;
    u16x8 x1 = *reinterpret_cast<const u16x8*>(src + c);
    u16x8 x2 = *reinterpret_cast<const u16x8*>(src + HALF + c);
    uint16_t* dst;
    if (head < Hq) {
      dst = q + (((int64_t)b * Hq + head) * S + s) * D;
    } else if (head < Hq + Hkv) {
      dst = k + (((int64_t)b * Hkv + (head - Hq)) * S + s) * D;
    } else {
      dst = v + (((int64_t)b * Hkv + (head - Hq - Hkv)) * S + s) * D;
      *reinterpret_cast<u16x8*>(dst + c) = x1;
      *reinterpret_cast<u16x8*>(dst + HALF + c) = x2;
      continue;
    }
    const int pos = positions ? positions[t] : s;
    const float* cp = cosb + (int64_t)pos * HALF + c;
    const float* sp = sinb + (int64_t)pos * HALF + c;
    f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
    f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
    u16x8 y1, y2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cj = j < 4 ? c0[j & 3] : c1[j & 3];
      const float sj = j < 4 ? s0[j & 3] : s1[j & 3];
      const float a = bf2f(x1[j]), bb = bf2f(x2[j]);
      y1[j] = f2bf(rope_lo(a, bb, cj, sj));
      y2[j] = f2bf(rope_hi(a, bb, cj, sj));
    }
    *reinterpret_cast<u16x8*>(dst + c) = y1;
    *reinterpret_cast<u16x8*>(dst + HALF + c) = y2;
  }
}

template <int D>
__global__ void __launch_bounds__(256) rope_merge_bwd_kernel(const float* __restrict__ dq,
                                                             const float* __restrict__ dkp,
                                                             const float* __restrict__ dvp,
                                                             const float* __restrict__ cosb,
                                                             const float* __restrict__ sinb,
                                                             uint16_t* __restrict__ dqkv, int B, int S, int Hq,
                                                             int Hkv, int kv_heads_in, int64_t ldq, int head0) {
  constexpr int HALF = D / 2, CPH = HALF / 8;
  const int NH = Hq + 2 * Hkv;
  const int NHW = NH - head0;         // heads this call writes: head0 .. NH-1 (head0 = Hq: the dQ kernel did q)
  const int rep = kv_heads_in / Hkv;  // partials per kv head (Hq for per-q-head partials, Hkv if pre-summed)
  const int64_t n = (int64_t)B * S * NHW * CPH;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int cc = (int)(i % CPH);
    const int64_t th = i / CPH;
    const int head = head0 + (int)(th % NHW);
    const int64_t t = th / NHW;
    const int b = (int)(t / S), s = (int)(t % S);
    const int c = cc * 8;
    float a1[8], a2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { a1[j] = 0.f; a2[j] = 0.f; }
    const float* srcs;
    int nsum;
    int64_t stride;
    if (head < Hq) {
      srcs = dq + (((int64_t)b * Hq + head) * S + s) * D;
      nsum = 1;
      stride = 0;
    } else {
      const int g = head < Hq + Hkv ? head - Hq : head - Hq - Hkv;
      const float* base = head < Hq + Hkv ? dkp : dvp;
      srcs = base + (((int64_t)b * kv_heads_in + (int64_t)g * rep) * S + s) * D;
      nsum = rep;
      stride = (int64_t)S * D;
    }
    for (int r = 0; r < nsum; ++r) {
      const float* p = srcs + r * stride;
      f32x4 u0 = *reinterpret_cast<const f32x4*>(p + c), u1 = *reinterpret_cast<const f32x4*>(p + c + 4);
      f32x4 w0 = *reinterpret_cast<const f32x4*>(p + HALF + c), w1 = *reinterpret_cast<const f32x4*>(p + HALF + c + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a1[j] += u0[j]; a1[j + 4] += u1[j];
        a2[j] += w0[j]; a2[j + 4] += w1[j];
      }
    }
    uint16_t* dst = dqkv + t * ldq + (int64_t)head * D;
    u16x8 y1, y2;
    if (head >= Hq + Hkv) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { y1[j] = f2bf(a1[j]); y2[j] = f2bf(a2[j]); }
    } else {
      const float* cp = cosb + (int64_t)s * HALF + c;
      const float* sp = sinb + (int64_t)s * HALF + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float cj = cp[j], sj = sp[j];
        y1[j] = f2bf(__builtin_fmaf(a1[j], cj, a2[j] * sj));  // explicit contraction: the dQ kernel's
        y2[j] = f2bf(__builtin_fmaf(a2[j], cj, -(a1[j] * sj)));  // epilogue and this give the same bits
      }
    }
    *reinterpret_cast<u16x8*>(dst + c) = y1;
    *reinterpret_cast<u16x8*>(dst + HALF + c) = y2;
  }
}

}  // namespace mx

using namespace mx;

static int grid_for(int64_t items) {
  int64_t b = (items + 255) / 256;
  return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

extern "C" int mx_rope_split(const uint16_t* qkv, const float* cosb, const float* sinb, const int32_t* positions,
                             uint16_t* q, uint16_t* k, uint16_t* v, int B, int S, int Hq, int Hkv, int D,
                             hipStream_t stream) {
  const int64_t items = (int64_t)B * S * (Hq + 2 * Hkv) * (D / 16);
  if (items <= 0) return 0;
  if (D == 128)
    rope_split_kernel<128><<<grid_for(items), 256, 0, stream>>>(qkv, cosb, sinb, positions, q, k, v, B, S, Hq, Hkv);
  else if (D == 64)
    rope_split_kernel<64><<<grid_for(items), 256, 0, stream>>>(qkv, cosb, sinb, positions, q, k, v, B, S, Hq, Hkv);
  else if (D == 32)
    rope_split_kernel<32><<<grid_for(items), 256, 0, stream>>>(qkv, cosb, sinb, positions, q, k, v, B, S, Hq, Hkv);
  else
    return -1;
  return (int)hipGetLastError();
}

// ldq: row stride of dqkv in elements (>= (Hq + 2 Hkv) D, multiple of 8); the rows may
// be the left part of the LoRA-augmented backward GEMM operand (mxllm/ops/linear.py)
extern "C" int mx_rope_merge_bwd(const float* dq, const float* dkp, const float* dvp, const float* cosb,
                                 const float* sinb, uint16_t* dqkv, int B, int S, int Hq, int Hkv, int kv_heads_in,
                                 int D, int64_t ldq, hipStream_t stream, int head0) {
  if (head0 != 0 && head0 != Hq) return -1;  // all heads, or the k / v heads only (dq == nullptr allowed)
  const int64_t items = (int64_t)B * S * (Hq + 2 * Hkv - head0) * (D / 16);
  if (items <= 0) return 0;
  if (kv_heads_in % Hkv || ldq < (int64_t)(Hq + 2 * Hkv) * D || ldq % 8) return -1;
#define MERGE(DD)                                                                                       \
  rope_merge_bwd_kernel<DD><<<grid_for(items), 256, 0, stream>>>(dq, dkp, dvp, cosb, sinb, dqkv, B, S, Hq, Hkv, \
                                                                 kv_heads_in, ldq, head0)
  if (D == 128) MERGE(128);
  else if (D == 64) MERGE(64);
  else if (D == 32) MERGE(32);
  else return -1;
#undef MERGE
  return (int)hipGetLastError();
}
