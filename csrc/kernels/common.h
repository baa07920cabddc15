// mxllm — shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//  * bf16 tensors are passed as `const uint16_t*` (raw bits) so loads can be
//    vectorised as 16-byte `u16x8` (G13 of the CDNA HIP guide: hipcc never
//    auto-vectorises scalar bf16 loads).
//  * a wavefront is 64 lanes: every wave-level idiom here hard-codes 64.
//  * f32 -> bf16 goes through __float2bfloat16, which hipcc -O3 lowers to a
//    single v_cvt_pk_bf16_f32 on gfx950 (NaN-preserving, RNE).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <type_traits>

namespace mx {

constexpr int kWave = 64;

typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// Rotate-half RoPE of the pair (a, b) = (x[d], x[d + D/2]) by (c, s) = (cos, sin) of d's frequency,
// with the contraction pinned (one explicit fma each) so every kernel that applies it -- rope_split,
// the gemm8 RoPE epilogue and the tail-balanced sum pass -- produces the same bits.
__device__ __forceinline__ float rope_lo(float a, float b, float c, float s) { return __builtin_fmaf(a, c, -(b * s)); }
__device__ __forceinline__ float rope_hi(float a, float b, float c, float s) { return __builtin_fmaf(b, c, a * s); }
__device__ __forceinline__ float bf2f(uint16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<uint16_t*>(&h);
}

// SwiGLU gradient, s = sigmoid(g) by the hardware reciprocal:
//   dg = dm u s (1 + g (1 - s)),  du = dm g s.
// The one multiply-add is an explicit FMA and the rest are product chains, so
// -ffp-contract=fast has nothing left to contract.  Every kernel that produces
// dgu (elementwise.hip swiglu_bwd, lora.hip swiglu_lora, the gemm8 SwiGLU-backward
// epilogue) therefore gives the same bits.
__device__ __forceinline__ void swiglu_grad(float dm, float g, float u, float& dg, float& du) {
  const float s = __builtin_amdgcn_rcpf(1.f + __expf(-g));
  dg = dm * u * s * __builtin_fmaf(g, 1.f - s, 1.f);
  du = dm * g * s;
}

// two f32 -> packed bf16x2 in one u32 (lo in bits 0..15)
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024. `scratch` must hold >= 16 floats.
// Every thread receives the result.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += scratch[i];
  return r;
}

__device__ __forceinline__ float block_max(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
  for (int i = 0; i < nw; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// XCD-aware, bijective remap of a 1-D workgroup id (guide §5, "XCD swizzle must
// be bijective"): consecutive logical tiles land on the same XCD (shared L2).
// Speed only — correctness never depends on placement.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// Bijective remap for grids of (outer, bh) work items, bid = outer * BH + bh, whose cost
// varies with `outer` (causal attention: heaviest outer index first).  Workgroups are dealt
// round-robin over the 8 XCDs (MI355X_MICROARCH "Workgroup dispatch"): blocks b, b + 8, ...
// share one.  xcd_remap above gives each XCD a CONTIGUOUS bid range, i.e. a narrow band of
// outer indices, so one XCD ran all the heavy blocks while another idled (causal attention
// at B2 Hq64: 644 µs where the per-CU work is ~410).  Here XCD x takes the KV groups (G
// consecutive q-heads sharing one K/V head) {x, x + 8, ...} -> K / V stay in one L2 -- and
// walks them through every outer index in dispatch order, so every XCD sees the same
// heavy-to-light mix.  Falls back to identity (round-robin already balances) when BH is not
// a multiple of 8 G.
__device__ __forceinline__ int xcd_balance(int orig, int nwg, int BH, int G) {
  if ((nwg & 7) || G <= 0 || BH % (8 * G) || nwg % BH) return orig;
  const int x = orig & 7, j = orig >> 3, per = BH >> 3;
  const int outer = j / per, lb = j % per;
  const int bh = ((lb / G) * 8 + x) * G + lb % G;
  return outer * BH + bh;
}

// ---- KV cache addressing (decode kernels) ----
// Per layer the cache is [rows, Hkv, SEQ, D] bf16.  Contiguous (bt == nullptr): rows =
// slots, SEQ = max_seq.  Paged (bt = block table [slots, maxb] int32): rows = pool blocks,
// SEQ = the block size; token p of slot s lives in block bt[s][p / SEQ] at row p % SEQ.
// Returns the token-row index (multiply by D for the element offset).
__device__ __forceinline__ int64_t kv_row(const int32_t* __restrict__ bt, int maxb, int seq, int slot, int Hkv,
                                          int hk, int p) {
  if (!bt) return ((int64_t)slot * Hkv + hk) * seq + p;
  const int blk = bt[(int64_t)slot * maxb + p / seq];
  return ((int64_t)blk * Hkv + hk) * seq + (p % seq);
}

// ---- LDS-DMA-friendly transposed reads (used by the attention kernels) ----
// ds_read_b64_tr_b16 as inline asm with an immediate offset: invisible to hipcc's
// waitcnt pass, which otherwise drains every in-flight LDS-DMA (vmcnt(0)) before a
// builtin tr-read (it cannot tell that the read misses the DMA's buffer).  The caller
// waits with lds_wait() / lds_wait_le() and pins each result behind the wait with pin().
// LDS operations of a wave complete in order, so counted lgkmcnt waits are exact for
// the asm reads and conservative for anything the compiler interleaves.
template <int OFF>
__device__ __forceinline__ u16x4 trd_asm(uint32_t lds_addr) {
  u16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(lds_addr), "i"(OFF));
  return v;
}
// transposed read at base + off; `off` folds into the instruction's immediate when it
// is a compile-time constant < 64 KiB
__device__ __forceinline__ u16x4 trd_off(uint32_t base, int off) {
  u16x4 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(off));
  else
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(base + (uint32_t)off));
  return v;
}
// 16-B row read at base + off (immediate when constant), same waitcnt contract as trd_off
__device__ __forceinline__ u16x8 rd128_off(uint32_t base, int off) {
  u16x8 v;
  if (__builtin_constant_p(off) && off >= 0 && off < 65536)
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(base), "i"(off));
  else
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(base + (uint32_t)off));
  return v;
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// at most n LDS operations of this wave still outstanding (n folds to a constant after unrolling)
__device__ __forceinline__ void lds_wait_le(int n) {
  switch (n) {
#define MX_LGKM(N) case N: asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory"); break;
    MX_LGKM(15) MX_LGKM(14) MX_LGKM(13) MX_LGKM(12) MX_LGKM(11) MX_LGKM(10) MX_LGKM(9) MX_LGKM(8)
    MX_LGKM(7) MX_LGKM(6) MX_LGKM(5) MX_LGKM(4) MX_LGKM(3) MX_LGKM(2) MX_LGKM(1)
#undef MX_LGKM
    default: asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); break;
  }
}
__device__ __forceinline__ void pin(u16x4& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(u16x8& v) { asm volatile("" : "+v"(v)); }
// byte address of a __shared__ object in the LDS aperture
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(__attribute__((address_space(3))) const char*)p;
}

}  // namespace mx

#define MX_CHECK_LAUNCH() (void)hipGetLastError()
