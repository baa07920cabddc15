// RMSNorm (+ residual add) that also writes the rank-r LoRA tail of the projection consuming its
// output ("emit the forward x A^T tails from the RMSNorm kernel").
//
// A LoRA projection runs ONE augmented GEMM on x_aug = [x | s x A^T] (mxllm/ops/linear.py
// _LoRAAugFn).  The norm writes x as the left part of that buffer; the tail s x A^T was a separate
// lora_xwt launch + split reduction that re-read x from HBM (70B: 64 MB per call, 19 + 6 us for
// its fixed cost, 2 calls per layer: q/k/v and gate-up).  Here the norm's workgroup owns 16 rows
// and computes the tail from the bf16 values it just stored, with MFMA:
//   * 16 waves; wave w owns columns [w H/16, (w + 1) H/16) of all 16 rows, lane (r = l & 15,
//     q = l >> 4) the 8 columns 32 i + 8 q of row r in step i -- the B-operand layout of
//     v_mfma_f32_16x16x32_bf16, so the normalised 16 x 32 block of step i IS the MFMA operand and
//     the adapter rows V[16 nb + r] at the same columns the A operand (L2-resident: V is <= 1 MB);
//   * the row sum of squares: two lane shuffles + 16 waves through LDS, fixed order;
//   * the 16 waves' partial [16 adapters x 16 rows] tiles are summed through LDS in wave order
//     (deterministic), scaled by s, rounded to bf16 and stored in columns [H, H + pad) (zeros past
//     the adapter rows, as lora_xwt writes them).
// Same normalisation expression as rmsnorm_fwd_kernel (csrc/kernels/rmsnorm.hip); the row sum of
// squares is added in a different order (fp32 rounding of rstd), the tail sums in MFMA order.
#include "common.h"

namespace mx {

namespace {
typedef __bf16 nbf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 nl_mfma(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(nbf16x8_t, a), __builtin_bit_cast(nbf16x8_t, b),
                                                 c, 0, 0, 0);
}
constexpr int kNLW = 16;  // waves per workgroup = rows per workgroup
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float bflo(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bfhi(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }
}  // namespace

// partial tiles of the 16 waves -> out[row0 + rr, H + cc] = bf16(alpha * sum_w), cc < pad (<= 64)
template <int NRB>
__device__ __forceinline__ void nl_tail_store(const f32x4 (&acc)[NRB], float* red, int wave, int lane,
                                              uint16_t* __restrict__ out, int64_t ldo, int64_t row0, int H, int pad,
                                              float alpha) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int nb = 0; nb < NRB; ++nb)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[(wave * NRB * 16 + nb * 16 + 4 * q + j) * 17 + r] = acc[nb][j];
  __syncthreads();
  const int rr = threadIdx.x & 15, cc = threadIdx.x >> 4;
  if (cc < pad) {
    float s = 0.f;
    if (cc < 16 * NRB) {
#pragma unroll
      for (int w = 0; w < kNLW; ++w) s += red[(w * NRB * 16 + cc) * 17 + rr];
    }
    out[(row0 + rr) * ldo + H + cc] = f2bf(alpha * s);
  }
}

// y[row, 0:H] = bf16(h * rstd * w) with h = x (+ res, rounded to bf16 and stored to h_out);
// y[row, H:H+pad] = bf16(alpha * y[row, 0:H] . V[0:16 NRB, :]^T) (zeros past 16 NRB).
// Wave w owns row 16 blockIdx + w; lane l its 16-B chunks l + 64 j (j < NCH = H / 512): every load and
// store is one row's 1 KB contiguous.  The tail: four rounds over column quarters -- each wave drops its
// row's quarter of y into LDS, then takes H / 64 columns of all 16 rows as MFMA B operands.
template <int NCH, bool RESID, int NRB>
__global__ void __launch_bounds__(1024) rmsnorm_lora_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
    uint16_t* __restrict__ y, uint16_t* __restrict__ h_out, float* __restrict__ rstd_out, int H, int64_t ldy,
    float eps, const uint16_t* __restrict__ V, int64_t ldv, float alpha, int pad) {
  constexpr int QC = NCH * 128;       // columns per round (H / 4)
  constexpr int YS = QC + 8;          // LDS row stride (elements): rows 16 B apart in the bank space
  constexpr int KS = NCH / 4;         // 32-column MFMA steps per wave per round (QC / 16 / 32)
  constexpr int RED = kNLW * NRB * 16 * 17;
  constexpr int LDSF = (16 * YS / 2) > RED ? (16 * YS / 2) : RED;
  __shared__ float lds[LDSF];
  uint16_t* ys = reinterpret_cast<uint16_t*>(lds);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = (int64_t)blockIdx.x * 16, row = row0 + wave;
  uint32_t hv[NCH][4];  // packed bf16 pairs: h, then y
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (i % 4 == 0 && i) __builtin_amdgcn_sched_barrier(0);  // bounded loads in flight: no spill
    const int c = (lane + 64 * i) * 8;
    const u32x4 a = *reinterpret_cast<const u32x4*>(x + row * H + c);
    if constexpr (RESID) {
      const u32x4 rv = *reinterpret_cast<const u32x4*>(res + row * H + c);
      u32x4 hb;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        hb[j] = (uint32_t)f2bf(bflo(a[j]) + bflo(rv[j])) | ((uint32_t)f2bf(bfhi(a[j]) + bfhi(rv[j])) << 16);
      *reinterpret_cast<u32x4*>(h_out + row * H + c) = hb;
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[i][j] = hb[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[i][j] = a[j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lo = bflo(hv[i][j]), hi = bfhi(hv[i][j]);
      ss += lo * lo;
      ss += hi * hi;
    }
  }
  // opaque to hipcc: the normalisation re-expands the packed pairs instead of keeping the fp32
  // expansions live across the reduction
#pragma unroll
  for (int i = 0; i < NCH; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(hv[i][j]));
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd_out[row] = rs;
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (i % 4 == 0 && i) __builtin_amdgcn_sched_barrier(0);
    const int c = (lane + 64 * i) * 8;
    const u32x4 g = *reinterpret_cast<const u32x4*>(w + c);
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (uint32_t)f2bf(bflo(hv[i][j]) * rs * bflo(g[j])) | ((uint32_t)f2bf(bfhi(hv[i][j]) * rs * bfhi(g[j])) << 16);
      hv[i][j] = o[j];
    }
    *reinterpret_cast<u32x4*>(y + row * ldy + c) = o;
  }
  // tail: lane (r, q) = (l & 15, l >> 4) of wave w reads rows r, columns wq0 + 32 k + 8 q of the round
  const int r = lane & 15, q = lane >> 4;
  f32x4 acc[NRB];
#pragma unroll
  for (int nb = 0; nb < NRB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wq0 = wave * (QC / 16);
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
    // adapter rows (L2) of this round's first two steps issued before the barrier, the rest after the
    // quarter's LDS writes (which retire its hv chunks): bounded registers
    constexpr int PF = KS < 2 ? KS : 2;
    u16x8 vf[KS][NRB];
#pragma unroll
    for (int k = 0; k < PF; ++k)
#pragma unroll
      for (int nb = 0; nb < NRB; ++nb)
        vf[k][nb] = *reinterpret_cast<const u16x8*>(V + (int64_t)(nb * 16 + r) * ldv + rd * QC + wq0 + 32 * k + 8 * q);
    if (rd) __syncthreads();  // every wave done reading the previous quarter
#pragma unroll
    for (int i = 0; i < NCH / 4; ++i) {  // this round's chunks of the lane: columns rd QC + 8 l + 512 i
      const int ch = rd * (NCH / 4) + i;
      const u32x4 o = {hv[ch][0], hv[ch][1], hv[ch][2], hv[ch][3]};
      *reinterpret_cast<u32x4*>(ys + wave * YS + (lane + 64 * i) * 8) = o;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = PF; k < KS; ++k)
#pragma unroll
      for (int nb = 0; nb < NRB; ++nb)
        vf[k][nb] = *reinterpret_cast<const u16x8*>(V + (int64_t)(nb * 16 + r) * ldv + rd * QC + wq0 + 32 * k + 8 * q);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const u16x8 b = *reinterpret_cast<const u16x8*>(ys + r * YS + wq0 + 32 * k + 8 * q);
#pragma unroll
      for (int nb = 0; nb < NRB; ++nb) acc[nb] = nl_mfma(vf[k][nb], b, acc[nb]);
    }
  }
  __syncthreads();  // the y image is dead: its LDS holds the reduction
  nl_tail_store<NRB>(acc, lds, wave, lane, y, ldy, row0, H, pad, alpha);
}

}  // namespace mx

using namespace mx;

// T % 16 == 0, H % 512 == 0 with H / 512 in {4, 8, 16}, 1 <= rows <= 64 (<= 48 at H 8192; adapter rows of V, each
// of H bf16 at stride ldv), 16 ceil(rows / 16) <= pad <= 64, 16-B aligned rows.  -1 otherwise.
extern "C" int mx_rmsnorm_lora_fwd(const uint16_t* x, const uint16_t* res, const uint16_t* w, uint16_t* y,
                                   uint16_t* h_out, float* rstd, int T, int H, int64_t ldy, float eps,
                                   const uint16_t* V, int64_t ldv, int rows, float alpha, int pad,
                                   hipStream_t stream) {
  const int nch = H / 512, nrb = (rows + 15) / 16;
  if (T <= 0 || T % 16 || H % 512 || (nch != 4 && nch != 8 && nch != 16) || rows < 1 || rows > 64 ||
      pad < 16 * nrb || pad > 64 || ldy < H + pad || ldy % 8 || ldv < H || ldv % 8 || (res && !h_out))
    return -1;
  if (nch == 16 && nrb == 4) return -1;  // 49-64 adapter rows at H 8192 spill (not a Llama-3.1 LoRA shape)
  if (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)V | (uintptr_t)res | (uintptr_t)h_out) & 15) return -1;
#define NL_F(NC, RS, NB)                                                                                        \
  rmsnorm_lora_fwd_kernel<NC, RS, NB><<<T / 16, 1024, 0, stream>>>(x, res, w, y, h_out, rstd, H, ldy, eps, V, ldv, \
                                                                   alpha, pad)
#define NL_NB(NC, RS)                      \
  switch (nrb) {                           \
    case 1: NL_F(NC, RS, 1); break;        \
    case 2: NL_F(NC, RS, 2); break;        \
    case 3: NL_F(NC, RS, 3); break;        \
    default: if (NC < 16) NL_F(NC < 16 ? NC : 8, RS, 4); break; \
  }
#define NL_NC(RS)                          \
  if (nch == 4) {                          \
    NL_NB(4, RS)                           \
  } else if (nch == 8) {                   \
    NL_NB(8, RS)                           \
  } else {                                 \
    NL_NB(16, RS)                          \
  }
  if (res) {
    NL_NC(true)
  } else {
    NL_NC(false)
  }
#undef NL_NC
#undef NL_NB
#undef NL_F
  return (int)hipGetLastError();
}
