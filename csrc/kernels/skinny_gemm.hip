// bf16 weight-streaming GEMM for decode on gfx950: Y[M, N] = X[M, K] . W[N, K]^T with M <= 32
// tokens (serving path, SURVEY §2.4 K14 neighbourhood).  A decode step reads every weight once;
// for the small projections of an 8B model (34-117 MB) hipBLASLt's skinny solutions stream at
// 1.7-4.5 TB/s (profiles/r2x_skinny_gemm.md), latency-bound: too few bytes in flight per CU.
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
#include <cstdlib>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8_sk __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma16_sk(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_sk, a), __builtin_bit_cast(bf16x8_sk, b),
                                                 c, 0, 0, 0);
}

// MB: 16-token blocks (1 or 2); X rows >= M are clamped to M-1 and discarded.
// NC: 16-channel groups per workgroup: each X fragment then feeds NC MFMAs, so X traffic per
// streamed weight byte drops NC-fold (it equals the weight traffic at 16 tokens with NC = 1).
__device__ __forceinline__ float silu_sk(float x) { return x / (1.f + __expf(-x)); }

template <int MB, int NC, bool SWO = false>
__global__ void __launch_bounds__(512) skinny_gemm_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                          const uint16_t* __restrict__ W, int64_t ldw,
                                                          uint16_t* __restrict__ Y, int64_t ldy, int M, int K,
                                                          int F = 0) {
  static_assert(!SWO || NC == 1, "SwiGLU epilogue: one channel group");
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
    const int64_t wr = SWO ? (int64_t)blockIdx.x * 8 + (c & 7) + (c >= 8 ? F : 0) : (int64_t)(n0 + 16 * j + c);
    wrow[j] = W + wr * ldw + (int64_t)w * kq + 16 * g;
  }
  const uint16_t* xr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xr[mb] = X + (int64_t)min(mb * 16 + c, M - 1) * ldx + (int64_t)w * kq + 16 * g;

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
  const int nit = kq / 64;
  int it = 0;
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
        if constexpr (SWO) {
          // lane (c, g) holds channels 4g..4g+3: gate outputs for g < 2, the up outputs of the
          // same columns in lane (c, g + 2) = lane ^ 32
          f32x4 up;
#pragma unroll
          for (int i = 0; i < 4; ++i) up[i] = __shfl_xor(s[i], 32, 64);
          if (g < 2 && m < M) {
            u16x4 o;
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = f2bf(silu_sk(bf2f(f2bf(s[i]))) * bf2f(f2bf(up[i])));
            *reinterpret_cast<u16x4*>(Y + (int64_t)m * ldy + (int64_t)blockIdx.x * 8 + 4 * g) = o;
          }
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

// X [M, K] bf16 (row stride ldx), W [N, K] bf16 (row stride ldw), Y [M, N] bf16 (row stride
// ldy).  Requires M in 1..32, N % 16 == 0, K % 512 == 0, ldx / ldw multiples of 8, ldy of 4.
extern "C" int mx_skinny_gemm(const uint16_t* x, int64_t ldx, const uint16_t* w, int64_t ldw, uint16_t* y,
                              int64_t ldy, int M, int N, int K, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 32 || N % 16 || K % 512 || ldx % 8 || ldw % 8 || ldy % 4 || ldx < K || ldw < K || ldy < N) return -1;
  // MXLLM_SKINNY_NC: channel groups per workgroup (1, 2 or 4; default 1).  Two or four groups
  // cut the X traffic but halve / quarter the workgroups; measured at the Llama 8B / 70B decode
  // shapes they won only on the 8B qkv projection (profiles/r2x_skinny_gemm.md)
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
