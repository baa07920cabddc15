// bf16 weight-streaming GEMM for decode on gfx950: Y[M, N] = X[M, K] . W[N, K]^T with M <= 32
// tokens (serving path, SURVEY §2.4 K14 neighbourhood).  A decode step reads every weight once;
// for the small projections of an 8B model (34-117 MB) hipBLASLt's skinny solutions stream at
// 1.7-4.5 TB/s (archive/profiles/r2x_skinny_gemm.md), latency-bound: too few bytes in flight per CU.
//
// Same structure as the fp8 weight kernel (fp8_gemm.hip) without the dequantisation:
//  * workgroup = 8 waves = 16 output channels; the waves split K in eight contiguous parts
//    and meet in LDS; N/16 workgroups;
//  * v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand (16 channels x 32 k) and X^T
//    as the B operand (32 k x 16 tokens); lane (c, g) loads k = 16g .. 16g+15 of each 64-k
//    chunk of channel c as two 16-B loads = the A fragments of the chunk's two MFMA k-steps,
//    and the X fragments use the same k permutation;
//  * 8 chunks' loads are issued before the first is used: 256 B of weights per lane in
//    flight, 128 KB per workgroup.
//  * SWO (SwiGLU output, the decode MLP's gate|up projection, W = [gate; up] [2F, K]): a
//    workgroup's 16 channels are 8 gate rows n..n+7 and the matching 8 up rows F+n..F+n+7, so
//    the epilogue holds both halves of its 8 outputs and writes silu(g) * u [M, F] directly
//    (g, u rounded to bf16 first, as the separate GEMM + SwiGLU kernels round them: same bits).
//    Same weight stream as the plain kernel; one launch and the [M, 2F] round trip less.
//  * NORM (decode, M <= 4 rows): the RMSNorm (with the residual add) that produces X runs in
//    the prologue: every workgroup rebuilds the normalised rows in LDS from the residual h
//    (and the sub-block output `delta`), with the thread mapping, summation order and
//    rounding of rmsnorm.hip's forward kernel (same bits); workgroup 0 stores h + delta.
//    The X fragments then come from LDS.  Saves the two RMSNorm launches of every layer.
//  * ROPE (decode QKV projection, head_dim 128): a workgroup's 16 channels are 8 first-half
//    channels i..i+7 of one head and the matching second-half channels 64+i..64+i+7, so the
//    epilogue holds both halves of each rotation pair and does decode.hip rope_append's work:
//    rotated q rows -> q, rotated k and plain v rows -> the KV cache at (slot, pos).  Saves the
//    rope_append launch of every layer.
#include <cstdlib>

#include "common.h"
#include "decode_fuse.h"

namespace mx {

typedef __bf16 bf16x8_sk __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma16_sk(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_sk, a), __builtin_bit_cast(bf16x8_sk, b),
                                                 c, 0, 0, 0);
}

// MB: 16-token blocks (1 or 2); X rows >= M are clamped to M-1 and discarded.
// NC: 16-channel groups per workgroup: each X fragment then feeds NC MFMAs, so X traffic per
// streamed weight byte drops NC-fold (it equals the weight traffic at 16 tokens with NC = 1).
template <int MB, int NC, bool SWO = false, bool NORM = false, bool ROPE = false, bool MERGE = false>
__global__ void __launch_bounds__(512) skinny_gemm_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                          const uint16_t* __restrict__ W, int64_t ldw,
                                                          uint16_t* __restrict__ Y, int64_t ldy, int M, int K,
                                                          int F = 0, SkNorm na = {}, SkRope rp = {},
                                                          SkMerge mg = {}) {
  static_assert(!SWO || NC == 1, "SwiGLU epilogue: one channel group");
  static_assert(!ROPE || (NC == 1 && !SWO), "RoPE epilogue: one channel group");
  static_assert(!NORM || (MB == 1 && NC == 1), "fused RMSNorm: <= 16 rows, one channel group");
  static_assert(!MERGE || (MB == 1 && NC == 1 && !NORM && !SWO && !ROPE), "fused split merge: plain GEMM rows");
  constexpr bool LDSX = NORM || MERGE;  // X rows built in LDS by the prologue
  constexpr int NW = 8, UNR = NC == 1 ? 8 : 4;
  __shared__ f32x4 red[NW][NC][MB][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NC;
  const int kq = K / NW;  // this wave's K part
  const uint16_t* wrow[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    // SWO: channel c < 8 -> gate row blockIdx.x * 8 + c, c >= 8 -> the matching up row
    // ROPE: head blockIdx.x / 8, pair base 8 (blockIdx.x % 8); c >= 8 -> the second-half row
    const int64_t wr = (SWO || ROPE) ? dfuse_row<SWO>(blockIdx.x, c, F) : (int64_t)(n0 + 16 * j + c);
    wrow[j] = W + wr * ldw + (int64_t)w * kq + 16 * g;
  }
  const uint16_t* xr[MB];
  const int nit = kq / 64;
  // NORM: the first UNR chunks' weight loads go out before the prologue, so the weight stream's
  // latency overlaps the RMSNorm instead of following it
  u16x8 apre[UNR][NC][2];
  if constexpr (LDSX) {
    if (nit >= UNR) {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          apre[u][j][0] = *reinterpret_cast<const u16x8*>(wrow[j] + u * 64);
          apre[u][j][1] = *reinterpret_cast<const u16x8*>(wrow[j] + u * 64 + 8);
        }
    }
  }
  if constexpr (LDSX) {
    extern __shared__ __attribute__((aligned(16))) uint16_t xs[];  // [M, K] normalised / merged rows
    if constexpr (NORM) {
      __shared__ float nscr[2][4];
      __shared__ float nrs[4];
      dfuse_norm_rows(X, ldx, M, K, na, xs, nscr, nrs);
    } else {
      dfuse_merge_rows(M, K, mg, xs);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) xr[mb] = xs + (int64_t)min(mb * 16 + c, M - 1) * K + (int64_t)w * kq + 16 * g;
  } else {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) xr[mb] = X + (int64_t)min(mb * 16 + c, M - 1) * ldx + (int64_t)w * kq + 16 * g;
  }

  f32x4 acc[NC][MB];
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[j][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load = [&](int k, u16x8 (&a)[NC][2], u16x8 (&b)[MB][2]) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      a[j][0] = *reinterpret_cast<const u16x8*>(wrow[j] + k);
      a[j][1] = *reinterpret_cast<const u16x8*>(wrow[j] + k + 8);
    }
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      b[mb][0] = *reinterpret_cast<const u16x8*>(xr[mb] + k);
      b[mb][1] = *reinterpret_cast<const u16x8*>(xr[mb] + k + 8);
    }
  };
  auto step = [&](const u16x8 (&a)[NC][2], const u16x8 (&b)[MB][2]) {
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        acc[j][mb] = mfma16_sk(a[j][0], b[mb][0], acc[j][mb]);
        acc[j][mb] = mfma16_sk(a[j][1], b[mb][1], acc[j][mb]);
      }
  };
  int it = 0;
  if constexpr (LDSX) {
    if (nit >= UNR) {  // first block: weights prefetched above, X fragments from LDS
      u16x8 b[UNR][MB][2];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) {
          b[u][mb][0] = *reinterpret_cast<const u16x8*>(xr[mb] + u * 64);
          b[u][mb][1] = *reinterpret_cast<const u16x8*>(xr[mb] + u * 64 + 8);
        }
#pragma unroll
      for (int u = 0; u < UNR; ++u) step(apre[u], b[u]);
      it = UNR;
    }
  }
  for (; it + UNR <= nit; it += UNR) {
    u16x8 a[UNR][NC][2], b[UNR][MB][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) load((it + u) * 64, a[u], b[u]);
#pragma unroll
    for (int u = 0; u < UNR; ++u) step(a[u], b[u]);
  }
  for (; it < nit; ++it) {
    u16x8 a[NC][2], b[MB][2];
    load(it * 64, a, b);
    step(a, b);
  }
  // C[row = channel 4g + i][col = token c] per (group, m-block): sum the NW K parts
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) red[w][j][mb][lane] = acc[j][mb];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        f32x4 s = red[0][j][mb][lane];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) s += red[ww][j][mb][lane];
        const int m = mb * 16 + c;
        if constexpr (ROPE) {
          dfuse_rope_store(s, g, m, M, blockIdx.x, rp);
        } else if constexpr (SWO) {
          dfuse_swiglu_store(s, g, m, M, Y, ldy, blockIdx.x);
        } else if (m < M) {
          u16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = f2bf(s[i]);
          *reinterpret_cast<u16x4*>(Y + (int64_t)m * ldy + n0 + 16 * j + 4 * g) = o;
        }
      }
  }
}

}  // namespace mx

using namespace mx;

// y = rmsnorm(h [+ delta]) . W^T (or with the SwiGLU epilogue: W = [gate; up], y [M, N/2]) for
// M <= 4 decode rows: the RMSNorm in the GEMM prologue (see NORM above).  h [M, K] (row stride
// ldh), delta [M, K] (row stride ldd) or nullptr, gamma [K]; h_out [M, K] (row stride K) gets
// h + delta when delta is given.  Requires M * K <= 32768 (64 KiB of LDS), K % 512 == 0.
// Decode QKV projection with the RoPE / KV-cache append in the epilogue (see ROPE above), and
// optionally the RMSNorm in the prologue (h, delta, gamma as mx_skinny_norm_gemm; norm = 0: X = h
// as is, any M <= 16).  w [(Hq + 2 Hkv) * 128, K]; q out [M, Hq, 128].
extern "C" int mx_skinny_rope_gemm(const uint16_t* h, int64_t ldh, int norm, const uint16_t* delta, int64_t ldd,
                                   const uint16_t* gamma, float eps, uint16_t* h_out, const uint16_t* w, int64_t ldw,
                                   const float* cosb, const float* sinb, const int32_t* pos, const int32_t* slots,
                                   uint16_t* q, uint16_t* kc, uint16_t* vc, int Hq, int Hkv, int max_seq,
                                   const int32_t* bt, int maxb, int M, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  const int N = (Hq + 2 * Hkv) * 128;
  if (M > (norm ? 4 : 16) || (norm && (int64_t)M * K > 32768) || K % 512 || ldh % 8 || ldd % 8 || ldw % 8 ||
      ldh < K || ldw < K || (norm && delta && (ldd < K || !h_out)))
    return -1;
  const SkRope rp{cosb, sinb, pos, slots, q, kc, vc, Hq, Hkv, max_seq, bt, maxb};
  if (norm) {
    const SkNorm na{delta, ldd, gamma, h_out, eps};
    skinny_gemm_kernel<1, 1, false, true, true><<<N / 16, 512, (size_t)M * K * 2, stream>>>(
        h, ldh, w, ldw, nullptr, 0, M, K, 0, na, rp);
  } else {
    skinny_gemm_kernel<1, 1, false, false, true><<<N / 16, 512, 0, stream>>>(h, ldh, w, ldw, nullptr, 0, M, K, 0,
                                                                               SkNorm{}, rp);
  }
  return (int)hipGetLastError();
}

// y[M, N] = merge(split partials) . W^T: the decode o-projection with decode.hip's split-K
// attention merge (decode_combine_kernel) in its prologue -- every workgroup rebuilds the
// attention output rows [M, Hq * 128] in LDS from part_ml [M, Hq, nsplit, 2] / part_o
// [M, Hq, nsplit, 128] (same bits as the combine kernel).  Saves the combine launch of every
// layer.  M <= 4, M * K <= 32768, K = Hq * 128 (% 512), N % 16 == 0.
extern "C" int mx_skinny_merge_gemm(const float* ml, const float* po, int nsplit, const uint16_t* w, int64_t ldw,
                                    uint16_t* y, int64_t ldy, int M, int N, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 4 || (int64_t)M * K > 32768 || N % 16 || K % 512 || ldw % 8 || ldy % 4 || ldw < K || ldy < N ||
      nsplit < 1)
    return -1;
  const SkMerge mg{ml, po, nsplit};
  skinny_gemm_kernel<1, 1, false, false, false, true><<<N / 16, 512, (size_t)M * K * 2, stream>>>(
      nullptr, 0, w, ldw, y, ldy, M, K, 0, SkNorm{}, SkRope{}, mg);
  return (int)hipGetLastError();
}

extern "C" int mx_skinny_norm_gemm(const uint16_t* h, int64_t ldh, const uint16_t* delta, int64_t ldd,
                                   const uint16_t* gamma, float eps, uint16_t* h_out, const uint16_t* w,
                                   int64_t ldw, uint16_t* y, int64_t ldy, int M, int N, int K, int swiglu,
                                   hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 4 || (int64_t)M * K > 32768 || N % 16 || K % 512 || ldh % 8 || ldd % 8 || ldw % 8 || ldy % 4 ||
      ldh < K || ldw < K || (delta && (ldd < K || !h_out)))
    return -1;
  const SkNorm na{delta, ldd, gamma, h_out, eps};
  const size_t lds = (size_t)M * K * 2;
  if (swiglu) {
    const int Fh = N / 2;
    if (Fh % 8 || ldy < Fh) return -1;
    skinny_gemm_kernel<1, 1, true, true><<<Fh / 8, 512, lds, stream>>>(h, ldh, w, ldw, y, ldy, M, K, Fh, na);
  } else {
    if (ldy < N) return -1;
    skinny_gemm_kernel<1, 1, false, true><<<N / 16, 512, lds, stream>>>(h, ldh, w, ldw, y, ldy, M, K, 0, na);
  }
  return (int)hipGetLastError();
}

// X [M, K] bf16 (row stride ldx), W [N, K] bf16 (row stride ldw), Y [M, N] bf16 (row stride
// ldy).  Requires M in 1..32, N % 16 == 0, K % 512 == 0, ldx / ldw multiples of 8, ldy of 4.
extern "C" int mx_skinny_gemm(const uint16_t* x, int64_t ldx, const uint16_t* w, int64_t ldw, uint16_t* y,
                              int64_t ldy, int M, int N, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 32 || N % 16 || K % 512 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K || ldy < N) return -1;
  // MXLLM_SKINNY_NC: channel groups per workgroup (1, 2 or 4; default 1).  Two or four groups
  // cut the X traffic but halve / quarter the workgroups; measured at the Llama 8B / 70B decode
  // shapes they won only on the 8B qkv projection (archive/profiles/r2x_skinny_gemm.md)
  static const int nc_env = [] {
    const char* e = getenv("MXLLM_SKINNY_NC");
    return e && *e ? atoi(e) : 0;
  }();
  int nc = nc_env ? nc_env : 1;
  while (nc > 1 && (N % (16 * nc) || N / (16 * nc) < 128)) nc >>= 1;
#define SKG(MBV, NCV) skinny_gemm_kernel<MBV, NCV><<<N / (16 * NCV), 512, 0, stream>>>(x, ldx, w, ldw, y, ldy, M, K)
  if (M <= 16) {
    if (nc >= 4) SKG(1, 4); else if (nc == 2) SKG(1, 2); else SKG(1, 1);
  } else {
    if (nc >= 4) SKG(2, 4); else if (nc == 2) SKG(2, 2); else SKG(2, 1);
  }
#undef SKG
  return (int)hipGetLastError();
}

// y[M, F] = silu(g) * u with [g | u] = x[M, K] . W[2F, K]^T, W = [gate; up] rows: the decode
// MLP's gate|up projection with the SwiGLU in its epilogue.  Same contract as mx_skinny_gemm
// with N = 2F, plus F % 8 == 0.
extern "C" int mx_skinny_gemm_swiglu(const uint16_t* x, int64_t ldx, const uint16_t* w, int64_t ldw, uint16_t* y,
                                     int64_t ldy, int M, int F, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 32 || F % 8 || K % 512 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K || ldy < F) return -1;
  if (M <= 16)
    skinny_gemm_kernel<1, 1, true><<<F / 8, 512, 0, stream>>>(x, ldx, w, ldw, y, ldy, M, K, F);
  else
    skinny_gemm_kernel<2, 1, true><<<F / 8, 512, 0, stream>>>(x, ldx, w, ldw, y, ldy, M, K, F);
  return (int)hipGetLastError();
}
