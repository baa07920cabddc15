// FP8 (OCP e4m3) weight-only GEMM for decode on gfx950: Y[M, N] = X[M, K] . (s[n] * Q[N, K])^T
// with M <= 32 tokens, bf16 activations / output, f32 accumulation (serving path,
// SURVEY §2.4 K14 neighbourhood: the decode step is bound by streaming every weight
// once, so 1-byte weights halve its HBM traffic; the bf16 GEMMs already stream at
// ~5.6 TB/s).
//
// Structure (memory-bound; the MFMA is nearly free):
//  * workgroup = 8 waves = 16 output channels; the waves split K in eight contiguous
//    parts and their partial sums meet in LDS; N/16 workgroups per GEMM, and the k
//    loop issues 8 chunks' loads before using any, so every CU keeps many 16-B
//    weight loads in flight;
//  * v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand (16 channels x 32 k)
//    and X^T as the B operand (32 k x 16 tokens): one MFMA chain per 16-token block;
//  * each lane loads 16 contiguous fp8 bytes (k = 16g .. 16g+15 of a 64-k chunk), so
//    the two MFMA k-steps of the chunk take k = 16g + 8s + j (permuted inside the
//    chunk); the X fragments use the same permutation (16-B bf16 loads);
//  * dequantisation without a conversion table: the quantiser never emits a zero or
//    subnormal code (see mxllm/serve/quant.py), so for every code
//    bf16 = sign<<15 | ((e4m3 & 0x7F) << 4) + (120 << 7)   (exponent rebias 7 -> 127),
//    two bytes at a time with 32-bit ALU ops (byte permute, and, shift-add, and-or);
//  * the per-channel scale is applied once in the epilogue.
#include <cstdlib>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8_f8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16_f8(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_f8, a), __builtin_bit_cast(bf16x8_f8, b),
                                                 c, 0, 0, 0);
}

// two e4m3 bytes (bits 0-7 and 8-15 of w16) -> packed bf16x2
__device__ __forceinline__ uint32_t e4m3x2_to_bf16x2(uint32_t w) {
  const uint32_t x = __builtin_amdgcn_perm(0u, w, 0x0c010c00u);  // b0 -> bits 0-7, b1 -> bits 16-23
  const uint32_t mag = ((x & 0x007F007Fu) << 4) + 0x3C003C00u;
  return mag | ((x << 8) & 0x80008000u);
}

__device__ __forceinline__ u16x8 dequant8(uint32_t lo, uint32_t hi) {
  const uint32_t a = e4m3x2_to_bf16x2(lo), b = e4m3x2_to_bf16x2(lo >> 16);
  const uint32_t c = e4m3x2_to_bf16x2(hi), d = e4m3x2_to_bf16x2(hi >> 16);
  return __builtin_bit_cast(u16x8, u32x4{a, b, c, d});
}

// MB: 16-token blocks (1 or 2); X rows >= M are clamped to M-1 and discarded.
// NW waves per workgroup split K into NW contiguous parts (more loads in flight for
// the projections with few output channels: o / down have only N/16 = 512 workgroups).
// NC: 16-channel groups per wave (1 or 2).  Every workgroup reads its waves' K parts of
// X once; with M distinct tokens that is M*2 bytes per k against 16*NC weight bytes, so
// for 6..16 tokens NC = 2 halves the X traffic per streamed weight byte (the X
// fragments of a chunk feed both channel groups' MFMAs).
template <int MB, int NW, int NC>
__global__ void __launch_bounds__(64 * NW) w8a16_gemm_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                             const uint8_t* __restrict__ Q,
                                                             const float* __restrict__ scale, uint16_t* __restrict__ Y,
                                                             int64_t ldy, int M, int N, int K) {
  __shared__ f32x4 red[NW][NC][MB][64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NC;
  const int kq = K / NW;  // this wave's K part
  const uint8_t* qrow[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) qrow[j] = Q + (int64_t)(n0 + 16 * j + c) * K + (int64_t)w * kq + 16 * g;
  const uint16_t* xr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xr[mb] = X + (int64_t)min(mb * 16 + c, M - 1) * ldx + (int64_t)w * kq + 16 * g;

  f32x4 acc[NC][MB];
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc[j][mb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one 64-k chunk: 16 fp8 weights per channel group and 2 x 8 activations per lane,
  // two MFMA k-steps per (group, token block)
  auto step = [&](const u32x4 (&q)[NC], const u16x8 (&b)[MB][2]) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const u16x8 a0 = dequant8(q[j][0], q[j][1]);  // k = 16g + 0..7   (MFMA step 0)
      const u16x8 a1 = dequant8(q[j][2], q[j][3]);  // k = 16g + 8..15  (MFMA step 1)
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        acc[j][mb] = mfma16_f8(a0, b[mb][0], acc[j][mb]);
        acc[j][mb] = mfma16_f8(a1, b[mb][1], acc[j][mb]);
      }
    }
  };
  auto load = [&](int k, u32x4 (&q)[NC], u16x8 (&b)[MB][2]) {
#pragma unroll
    for (int j = 0; j < NC; ++j) q[j] = *reinterpret_cast<const u32x4*>(qrow[j] + k);
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      b[mb][0] = *reinterpret_cast<const u16x8*>(xr[mb] + k);
      b[mb][1] = *reinterpret_cast<const u16x8*>(xr[mb] + k + 8);
    }
  };
  // batches of UNR chunks: all of a batch's loads are issued before its first use, so
  // UNR 16-B weight loads per lane and group are in flight (a plain loop waits on each)
  constexpr int UNR = 8;
  const int nit = kq / 64;
  int it = 0;
  for (; it + UNR <= nit; it += UNR) {
    u32x4 q[UNR][NC];
    u16x8 b[UNR][MB][2];
#pragma unroll
    for (int u = 0; u < UNR; ++u) load((it + u) * 64, q[u], b[u]);
#pragma unroll
    for (int u = 0; u < UNR; ++u) step(q[u], b[u]);
  }
  for (; it < nit; ++it) {
    u32x4 q[NC];
    u16x8 b[MB][2];
    load(it * 64, q, b);
    step(q, b);
  }
  // C[row = channel 4g + i][col = token c] per (group, m-block): sum the NW K parts
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) red[w][j][mb][lane] = acc[j][mb];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        f32x4 s = red[0][j][mb][lane];
#pragma unroll
        for (int ww = 1; ww < NW; ++ww) s += red[ww][j][mb][lane];
        const int m = mb * 16 + c;
        if (m < M) {
          const int n = n0 + 16 * j + 4 * g;
          const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + n);
          u16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = f2bf(s[i] * sc[i]);
          *reinterpret_cast<u16x4*>(Y + (int64_t)m * ldy + n) = o;
        }
      }
    }
  }
}

// Per-token activation quantisation for the fp8 x fp8 GEMM path: one workgroup per
// row, amax -> scale = amax / 448, codes = e4m3(x / scale) by the hardware pack
// conversion (OCP e4m3 on gfx950, round to nearest even).  16-B loads; the second
// pass re-reads the row from L1/L2.
__global__ void __launch_bounds__(256) quant_rows_e4m3_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                              uint8_t* __restrict__ Q, float* __restrict__ S, int K) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  const uint16_t* x = X + row * ldx;
  float amax = 0.f;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + c);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(v[j])));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  amax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = fmaxf(amax, 1e-12f) * (1.f / 448.f);
  const float inv = 1.f / sc;
  if (threadIdx.x == 0) S[row] = sc;
  uint8_t* q = Q + row * (int64_t)K;
  for (int c = threadIdx.x * 8; c < K; c += 256 * 8) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + c);
    int lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[0]) * inv, bf2f(v[1]) * inv, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[2]) * inv, bf2f(v[3]) * inv, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[4]) * inv, bf2f(v[5]) * inv, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(bf2f(v[6]) * inv, bf2f(v[7]) * inv, hi, true);
    *reinterpret_cast<uint2*>(q + c) = make_uint2((uint32_t)lo, (uint32_t)hi);
  }
}

}  // namespace mx

using namespace mx;

// X [M, K] bf16 (row stride ldx), Q [N, K] e4m3 codes, scale [N] f32 (per output channel),
// Y [M, N] bf16 (row stride ldy).  Requires M in 1..32, N % 16 == 0, K % 512 == 0,
// ldx a multiple of 8, ldy of 4.
extern "C" int mx_w8a16_gemm(const uint16_t* x, int64_t ldx, const uint8_t* q, const float* scale, uint16_t* y,
                             int64_t ldy, int M, int N, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 32 || N % 16 || K % 512 || ldx % 8 || ldy % 4 || ldx < K || ldy < N) return -1;
  // two channel groups per wave for 6..16 tokens when that still leaves >= 256 workgroups
  // (70B fp8 decode step, one group -> two: 22.0 -> 21.1 ms at 8 tokens, but 18.5 -> 19.3 ms
  // at 4; archive/profiles/r1g_fp8_decode_ab.md), and for 4..5 tokens on the long-K projections
  // (70B down, 4 tokens: 50.8 -> 44.1 us; archive/profiles/r4x/).
  // Effective routing: mxllm/serve/quant.py sends calls of more than SMALL_M (8) tokens to
  // hipBLASLt's fp8 GEMM, so from Python the two-group variant runs at 6..8 tokens; 9..16
  // reach it only through a direct w8_linear call (or MXLLM_W8_SMALL_M=16).
  // MXLLM_W8_NC (read per call, A/B switch): 1 / 2 / 4 forces that many channel groups per wave
  // wherever the grid keeps >= 128 workgroups
  const char* e = getenv("MXLLM_W8_NC");
  const int force = e && *e ? atoi(e) : 0;
  if (force == 4 && M <= 16 && N % 64 == 0 && N / 64 >= 128)
    w8a16_gemm_kernel<1, 8, 4><<<N / 64, 512, 0, stream>>>(x, ldx, q, scale, y, ldy, M, N, K);
  else if (M <= 16 && N % 32 == 0 &&
           ((force == 2 && N / 32 >= 128) || (!force && N / 32 >= 256 && (M >= 6 || (M >= 4 && K >= 16384)))))
    w8a16_gemm_kernel<1, 8, 2><<<N / 32, 512, 0, stream>>>(x, ldx, q, scale, y, ldy, M, N, K);
  else if (M <= 16) w8a16_gemm_kernel<1, 8, 1><<<N / 16, 512, 0, stream>>>(x, ldx, q, scale, y, ldy, M, N, K);
  else w8a16_gemm_kernel<2, 8, 1><<<N / 16, 512, 0, stream>>>(x, ldx, q, scale, y, ldy, M, N, K);
  return (int)hipGetLastError();
}

// x [M, K] bf16 rows (stride ldx) -> q [M, K] e4m3 codes, s [M] f32.  K % 8 == 0.
extern "C" int mx_quant_rows_e4m3(const uint16_t* x, int64_t ldx, uint8_t* q, float* s, int64_t M, int K,
                                  hipStream_t stream) {
  if (M <= 0) return 0;
  if (K % 8 || ldx % 8 || ldx < K) return -1;
  quant_rows_e4m3_kernel<<<(unsigned)M, 256, 0, stream>>>(x, ldx, q, s, K);
  return (int)hipGetLastError();
}

// Dequantise Q [N, K] e4m3 codes to bf16 W [N, K] = scale[n] * code (prefill path:
// large-M GEMMs run on hipBLASLt in bf16).  Eight codes per thread.
__global__ void __launch_bounds__(256) w8_dequant_kernel(const uint8_t* __restrict__ Q,
                                                         const float* __restrict__ scale, uint16_t* __restrict__ W,
                                                         int64_t n8, int K) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const uint2 q = *reinterpret_cast<const uint2*>(Q + i * 8);
    const u16x8 v = dequant8(q.x, q.y);
    const float s = scale[(i * 8) / K];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[j]) * s);
    *reinterpret_cast<u16x8*>(W + i * 8) = o;
  }
}

extern "C" int mx_w8_dequant(const uint8_t* q, const float* scale, uint16_t* w, int64_t N, int K, hipStream_t stream) {
  if (K % 8) return -1;
  const int64_t n8 = N * (int64_t)K / 8;
  if (n8 <= 0) return 0;
  const int grid = (int)std::min<int64_t>(8192, (n8 + 255) / 256);
  w8_dequant_kernel<<<grid, 256, 0, stream>>>(q, scale, w, n8, K);
  return (int)hipGetLastError();
}
