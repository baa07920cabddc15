// mxllm — LoRA rank-r GEMMs for gfx950 (MI355X): the skinny products around a
// frozen projection that hipBLASLt tiles poorly (measured at the Llama-3.1-70B
// shapes, T = 4096 tokens: 28-141 us per call, 1.5-4x off the HBM roofline).
//
//   lora_xwt : out[M, 64c] = alpha * X[M, K] . V[64c, K]^T        (c = 1, 2, ...)
//              forward  s x A^T  (V = A, zero-padded rows)  -> x_aug tail
//              backward s dy B   (V = B^T, a transposed copy kept by FusedLinear)
//   lora_xtg : out[n, j] (+)= alpha * sum_t X[t, n] . G[t, j]     (batched problems)
//              dA   = g^T x      (X = x,    G = the dy_aug tail, all R columns)
//              dB_i = dy_i^T st_i (X = dy_i, G = 16-column block i of the x_aug tail)
//
// Both are HBM-streaming reductions (arithmetic intensity <= 64 FLOP/B): the
// design goal is one pass over the big operand at full bandwidth with enough
// workgroups to fill 256 CUs, so both split their reduction across the 4 waves
// of a workgroup AND across workgroups (grid.y), and finish with an ORDERED
// reduction: the last workgroup of a tile to arrive (agent-scope counter, no
// spinning) sums the fp32 partials in split order -> bit-reproducible results.
//
// lora_xwt: the reduction index k is contiguous in both operands, so MFMA
// fragments come straight from HBM/L2 into registers (v_mfma_f32_16x16x32_bf16,
// lane (c, g) holds row c and k = 16 g + 8 p .. +7 of each 64-k block, p = k-step);
// a wave owns a 64 x 64 output tile (16 accumulators) and double-buffers its
// 64-k blocks in registers.
// lora_xtg: the reduction index t is the ROW index of both operands, so each
// wave streams 64-row blocks of X (64 columns = 128 B per row) and G through
// LDS-DMA (global_load_lds, source-swizzled 16-B chunks, double-buffered per
// wave, no workgroup barrier in the loop) and reads both MFMA operands with
// ds_read_b64_tr_b16 (the attention-V recipe: t permuted inside each 32-row
// k-step identically for both operands).  Reference: the reference has no LoRA
// path at all (fine-tuning is a planned-but-missing module,
// reference src/distributed_inference.py:61-76); the math follows PEFT's LoRA.
#include "common.h"
#include <stdlib.h>
#include <string.h>

namespace mx {

namespace {

typedef __bf16 lbf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) const void* lgptr_t;
typedef __attribute__((address_space(3))) void* llptr_t;

__device__ __forceinline__ f32x4 lmfma(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(lbf16x8_t, a), __builtin_bit_cast(lbf16x8_t, b),
                                                 c, 0, 0, 0);
}

constexpr int kRS = 68;  // fp32 row stride of the 64 x 64 reduction images (16-B aligned, g-rows 16 banks apart)
constexpr int kMaxTiles = 16384;

// per-tile arrival counters of the ordered split reduction; zero at load, reset
// to zero by the last workgroup of every tile (all LoRA kernels of a process run
// on one stream, so calls never interleave on a counter)
__device__ unsigned int g_xwt_cnt[kMaxTiles];
__device__ unsigned int g_xtg_cnt[kMaxTiles];

// true in exactly one workgroup of the tile: the last of `S` to arrive.  Every
// thread's partial stores are made visible at agent scope before the arrival.
__device__ __forceinline__ bool arrive_last(unsigned int* cnt, int S, int* s_flag) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = atomicAdd(cnt, 1u);
    *s_flag = prev == (unsigned)(S - 1);
    if (*s_flag) *cnt = 0u;
  }
  __syncthreads();
  const bool last = *s_flag;
  if (last) __threadfence();  // acquire: the other workgroups' partials
  return last;
}

// The same hand-off without fences (guide §6 Guideline 16, sc1 form): partials are
// stored write-through (relaxed agent-scope atomic stores = sc1), every storing wave
// drains them before the barrier, one relaxed agent-scope ticket publishes them, and the
// last arriver reads them with sc1 loads (no stale L1 copy, no acquire needed).
__device__ __forceinline__ void st4_sc1(float* p, const float4& v) {
  __hip_atomic_store(p + 0, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 2, v.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p + 3, v.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld4_sc1(const float* p) {
  float* q = const_cast<float*>(p);
  return float4{__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)};
}
__device__ __forceinline__ bool arrive_last_sc1(unsigned int* cnt, int S, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(S - 1);
    if (last) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag;
}

}  // namespace

// ------------------------------------------------------------------ lora_xwt
// grid (M/64, S), 256 threads; M % 64 == 0, K % 64 == 0; writes out[:, 0:64].
__global__ void __launch_bounds__(256, 1) lora_xwt_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                          const uint16_t* __restrict__ V, int64_t ldv,
                                                          uint16_t* __restrict__ out, int64_t ldo,
                                                          float* __restrict__ ws, int M, int K, int S, float alpha,
                                                          int fused_red) {
  __shared__ __attribute__((aligned(16))) float red[4][64 * kRS];
  __shared__ int s_last;
  const int mtiles = M >> 6, mt = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: keeps the block loop scalar
  const int nb = K >> 6, nw = S * 4, gw = split * 4 + w;
  const int b0 = (int)((int64_t)gw * nb / nw), b1 = (int)((int64_t)(gw + 1) * nb / nw);
  const uint16_t* xp = X + (int64_t)(mt * 64 + c) * ldx + 16 * g;
  const uint16_t* vp = V + (int64_t)c * ldv + 16 * g;
  const int64_t xrb = 16 * ldx, vcb = 16 * ldv;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto load = [&](int b, u16x8(&xr)[4][2], u16x8(&vr)[4][2]) {
    const int k0 = b * 64;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        xr[i][p] = *reinterpret_cast<const u16x8*>(xp + i * xrb + k0 + 8 * p);
        vr[i][p] = *reinterpret_cast<const u16x8*>(vp + i * vcb + k0 + 8 * p);
      }
  };
  auto comp = [&](const u16x8(&xr)[4][2], const u16x8(&vr)[4][2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = lmfma(xr[i][p], vr[j][p], acc[i][j]);
  };
  u16x8 xA[4][2], vA[4][2], xB[4][2], vB[4][2];
  int b = b0;
  if (b < b1) load(b, xA, vA);
  // two blocks per trip, the next block's loads issued before this block's MFMAs
  // (sched_barrier: the scheduler would otherwise sink them below the MFMAs and
  // leave one block in flight)
  for (; b + 1 < b1; b += 2) {
    load(b + 1, xB, vB);
    __builtin_amdgcn_sched_barrier(0);
    comp(xA, vA);
    __builtin_amdgcn_sched_barrier(0);
    load(min(b + 2, b1 - 1), xA, vA);  // unconditional (a redundant reload at the end): no branch in the loop
    __builtin_amdgcn_sched_barrier(0);
    comp(xB, vB);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (b < b1) comp(xA, vA);
  // 4 waves -> one 64 x 64 tile (fixed wave order)
  float* rw = red[w];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) rw[(16 * i + 4 * g + e) * kRS + 16 * j + c] = acc[i][j][e];
  __syncthreads();
  float4 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e4 = tid + 256 * q, row = e4 >> 4, col = (e4 & 15) * 4;
    float4 s = *reinterpret_cast<const float4*>(&red[0][row * kRS + col]);
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const float4 t = *reinterpret_cast<const float4*>(&red[ww][row * kRS + col]);
      s.x += t.x, s.y += t.y, s.z += t.z, s.w += t.w;
    }
    v[q] = s;
  }
  if (S > 1) {
    float* wp = ws + ((int64_t)split * mtiles + mt) * 4096;
#pragma unroll
    for (int q = 0; q < 4; ++q) reinterpret_cast<float4*>(wp)[tid + 256 * q] = v[q];
    if (!fused_red) return;  // lora_xwt_reduce_kernel finishes
    if (!arrive_last(&g_xwt_cnt[mt], S, &s_last)) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 s = reinterpret_cast<const float4*>(ws + (int64_t)mt * 4096)[tid + 256 * q];
      for (int sp = 1; sp < S; ++sp) {
        const float4 t = reinterpret_cast<const float4*>(ws + ((int64_t)sp * mtiles + mt) * 4096)[tid + 256 * q];
        s.x += t.x, s.y += t.y, s.z += t.z, s.w += t.w;
      }
      v[q] = s;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e4 = tid + 256 * q, row = e4 >> 4, col = (e4 & 15) * 4;
    uint2 o;
    o.x = pack_bf16x2(alpha * v[q].x, alpha * v[q].y);
    o.y = pack_bf16x2(alpha * v[q].z, alpha * v[q].w);
    *reinterpret_cast<uint2*>(out + (int64_t)(mt * 64 + row) * ldo + col) = o;
  }
}

// lora_xwt through LDS: the same product, with BOTH operands staged by LDS-DMA in
// full 128-B lines (8 rows x 128 B per wave instruction) instead of fragment-shaped
// register loads (16 rows x 64 B per instruction, which keep the texture path busy
// ~2x for the same bytes).  Per wave: 2 stages x (X 8 KiB + V 8 KiB), its own
// region, no workgroup barrier in the loop; the issuing wave's counted vmcnt orders
// its ds_reads behind its DMA.  Image: 64 rows x 128 B, 16-B chunk ch of row r at
// chunk position ch ^ (r & 7) — conflict-free for the ds_read_b128 fragment reads
// (row c of a 16-row block, chunk 4 ks + g) under gfx950's ds_read_b128 lane groups.
// grid (M/64, S), 256 threads; M % 64 == 0, K % 64 == 0; writes out[:, 0:64].
__global__ void __launch_bounds__(256, 1) lora_xwt_lds_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                              const uint16_t* __restrict__ V, int64_t ldv,
                                                              uint16_t* __restrict__ out, int64_t ldo,
                                                              float* __restrict__ ws, int M, int K, int S,
                                                              float alpha, int fused_red) {
  constexpr int TB = 8192, STG = 16384, WREG = 2 * STG;
  // ONE shared object (a second one can make hipcc drain vmcnt in the loop); the
  // last-arriver flag lives in its tail
  __shared__ __attribute__((aligned(16))) char smem[4 * WREG + 16];
  int* s_last = reinterpret_cast<int*>(smem + 4 * WREG);
  const int mtiles = M >> 6, mt = blockIdx.x, split = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nb = K >> 6, nw = S * 4, gw = split * 4 + w;
  const int b0 = (int)((int64_t)gw * nb / nw), b1 = (int)((int64_t)(gw + 1) * nb / nw);
  char* wreg = smem + w * WREG;
  const uint32_t wbase = lds_addr(wreg);
  // DMA sources: lane -> row 8 q + (lane >> 3), LDS chunk position lane & 7 holds
  // source chunk (lane & 7) ^ (row & 7)
  const int lrow = lane >> 3, sch = (lane & 7) ^ lrow;
  const uint16_t* xsrc = X + (int64_t)(mt * 64 + lrow) * ldx + 8 * sch;
  const uint16_t* vsrc = V + (int64_t)lrow * ldv + 8 * sch;
  auto issue = [&](int b, int s) {
    const int k0 = b * 64;
    char* xs = wreg + s * STG;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_global_load_lds((lgptr_t)(xsrc + (int64_t)(8 * q) * ldx + k0), (llptr_t)(xs + q * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_global_load_lds((lgptr_t)(vsrc + (int64_t)(8 * q) * ldv + k0), (llptr_t)(xs + TB + q * 1024),
                                       16, 0, 0);
  };
  // fragment reads: row 16 i + c, chunk 4 ks + g  ->  position (g ^ (c & 7)) ^ 4 ks
  const uint32_t rb0 = wbase + c * 128 + 16 * (g ^ (c & 7));
  const uint32_t rb1 = wbase + c * 128 + 16 * ((g ^ (c & 7)) ^ 4);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto block = [&](auto SC, int b) {
    constexpr int s = decltype(SC)::value;
    if (b + 1 < b1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // this block landed, the next may fly
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u16x8 xa[2][4], va[2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[0][i] = rd128_off(rb0, s * STG + i * 2048);
      xa[1][i] = rd128_off(rb1, s * STG + i * 2048);
      va[0][i] = rd128_off(rb0, s * STG + TB + i * 2048);
      va[1][i] = rd128_off(rb1, s * STG + TB + i * 2048);
    }
    lds_wait();
    __builtin_amdgcn_sched_barrier(0);  // the MFMAs below must not be hoisted above the wait
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pin(xa[0][i]), pin(xa[1][i]), pin(va[0][i]), pin(va[1][i]);
    }
    if (b + 2 < b1) issue(b + 2, s);  // refill this stage (its reads have retired)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = lmfma(xa[ks][i], va[ks][j], acc[i][j]);
  };
  if (b0 < b1) issue(b0, 0);
  if (b0 + 1 < b1) issue(b0 + 1, 1);
  for (int b = b0; b < b1; b += 2) {
    block(std::integral_constant<int, 0>{}, b);
    if (b + 1 < b1) block(std::integral_constant<int, 1>{}, b + 1);
  }
  // 4 waves -> one 64 x 64 tile (each wave's own region: its DMA has drained)
  float* rw = reinterpret_cast<float*>(wreg);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) rw[(16 * i + 4 * g + e) * kRS + 16 * j + c] = acc[i][j][e];
  __syncthreads();
  float4 v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e4 = tid + 256 * q, row = e4 >> 4, col = (e4 & 15) * 4;
    float4 s = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(smem) + row * kRS + col);
#pragma unroll
    for (int ww = 1; ww < 4; ++ww) {
      const float4 t = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(smem + ww * WREG) +
                                                        row * kRS + col);
      s.x += t.x, s.y += t.y, s.z += t.z, s.w += t.w;
    }
    v[q] = s;
  }
  if (S > 1) {
    float* wp = ws + ((int64_t)split * mtiles + mt) * 4096;
    if (!fused_red) {  // lora_xwt_reduce_kernel finishes
#pragma unroll
      for (int q = 0; q < 4; ++q) reinterpret_cast<float4*>(wp)[tid + 256 * q] = v[q];
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) st4_sc1(wp + 4 * (tid + 256 * q), v[q]);
    if (!arrive_last_sc1(&g_xwt_cnt[mt], S, s_last)) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // fixed split order (bit-reproducible, = the reduce kernel)
      float4 s = ld4_sc1(ws + (int64_t)mt * 4096 + 4 * (tid + 256 * q));
      for (int sp = 1; sp < S; ++sp) {
        const float4 t = ld4_sc1(ws + ((int64_t)sp * mtiles + mt) * 4096 + 4 * (tid + 256 * q));
        s.x += t.x, s.y += t.y, s.z += t.z, s.w += t.w;
      }
      v[q] = s;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e4 = tid + 256 * q, row = e4 >> 4, col = (e4 & 15) * 4;
    uint2 o;
    o.x = pack_bf16x2(alpha * v[q].x, alpha * v[q].y);
    o.y = pack_bf16x2(alpha * v[q].z, alpha * v[q].w);
    *reinterpret_cast<uint2*>(out + (int64_t)(mt * 64 + row) * ldo + col) = o;
  }
}

// split partials ws[S][M/64][64][64] -> out (fixed split order); grid (64 / ROWS) M/64, ROWS rows
// per workgroup (16 by default: at M 4096 the one-tile-per-workgroup grid of 64 workgroups left
// this pass latency-bound, ~6 us per call; MXLLM_LORA_XWT_RED_ROWS=64 restores it for A/B)
__global__ void __launch_bounds__(256) lora_xwt_reduce_kernel(const float* __restrict__ ws, int S, int mtiles,
                                                              uint16_t* __restrict__ out, int64_t ldo, float alpha,
                                                              int qpw) {
  const int per = 4 / qpw;  // workgroups per 64-row tile
  const int mt = blockIdx.x / per, tid = threadIdx.x;
  for (int q = (blockIdx.x % per) * qpw; q < (blockIdx.x % per + 1) * qpw; ++q) {
    const int e4 = tid + 256 * q, row = e4 >> 4, col = (e4 & 15) * 4;
    float4 s = reinterpret_cast<const float4*>(ws + (int64_t)mt * 4096)[e4];
    for (int sp = 1; sp < S; ++sp) {
      const float4 t = reinterpret_cast<const float4*>(ws + ((int64_t)sp * mtiles + mt) * 4096)[e4];
      s.x += t.x, s.y += t.y, s.z += t.z, s.w += t.w;
    }
    uint2 o;
    o.x = pack_bf16x2(alpha * s.x, alpha * s.y);
    o.y = pack_bf16x2(alpha * s.z, alpha * s.w);
    *reinterpret_cast<uint2*>(out + (int64_t)(mt * 64 + row) * ldo + col) = o;
  }
}

// ------------------------------------------------------------------ lora_xtg
struct XtgProb {
  const uint16_t* X;  // [T, >= n0 + Nx] row stride ldx (column 0 of this problem)
  const uint16_t* G;  // [T, >= 64] row stride ldg (column 0 of the 64-wide operand tail)
  uint16_t* out;      // element (n, j) at out[n * os_n + j * os_j]
  int64_t ldx, ldg, os_n, os_j;
  int Nx, jb0, JB, tile0;  // jb0: first 16-col block of G; JB blocks (<= 4); narrow when JB == 1
};
constexpr int kMaxProb = 8;
struct XtgArgs {
  XtgProb p[kMaxProb];
  int np, T, S, ntiles;
  float alpha;
  int accumulate;
  int fused_red;  // 1: last-arriving workgroup reduces; 0: lora_xtg_reduce_kernel does
  int narrow3;    // 1: narrow-G problems stream through three stages per wave (0: two, A/B)
  int wt;         // 1: each WAVE owns a 64-col tile over all T rows (4 adjacent tiles per workgroup,
                  // S == 1, no cross-wave reduction); 0: the 4 waves split one tile's rows
                  // (xtg_wave_tiles: the large launches only)
};

// 16-B chunk swizzle of a 128-B LDS row: conflict-free ds_read_b64_tr_b16 of
// rows 4 g + qq (each 32-lane half reads 8 rows x 32 B onto 8 distinct 32-B bank groups)
__device__ __forceinline__ int xsw(int row) { return (((row >> 1) & 1) << 2) | (((row >> 2) & 1) << 1); }

// grid (ntiles, S), 256 threads; T % 64 == 0, every Nx % 64 == 0.
__global__ void __launch_bounds__(256, 1) lora_xtg_kernel(const XtgArgs a, float* __restrict__ ws) {
  constexpr int XB = 8192, STG = 16384, WREG = 2 * STG;  // per wave: 2 stages x (X 8 KiB + G <= 8 KiB)
  __shared__ __attribute__((aligned(16))) char smem[4 * WREG];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: keeps the block loop scalar
  const int tile = a.wt ? blockIdx.x * 4 + w : blockIdx.x, split = blockIdx.y;
  if (a.wt && tile >= a.ntiles) return;  // wave-uniform; the wt path has no workgroup barrier
  // this tile's problem, selected with uniform conditional copies (a dynamic index
  // into the kernel-argument array would be lowered through scratch)
  XtgProb P = a.p[0];
#pragma unroll
  for (int i = 1; i < kMaxProb; ++i)
    if (i < a.np && tile >= a.p[i].tile0) P = a.p[i];
  const int n0 = (tile - P.tile0) * 64;
  const bool wide = P.JB > 1;
  const int JB = P.JB;
  const int qq = c >> 2, pp = c & 3;
  const int nblk = a.T >> 6, nw = a.wt ? a.S : a.S * 4, gw = a.wt ? split : split * 4 + w;
  const int b0 = (int)((int64_t)gw * nblk / nw), b1 = (int)((int64_t)(gw + 1) * nblk / nw);
  char* wreg = smem + w * WREG;
  const uint32_t wbase = lds_addr(wreg);

  // LDS-DMA sources (lane-linear 1-KiB destinations): X rows 8 q + (lane >> 3)
  const int xrow = lane >> 3, xch = (lane & 7) ^ xsw(lane >> 3);
  const uint16_t* xsrc = P.X + (int64_t)xrow * P.ldx + n0 + 8 * xch;
  const uint16_t* gsrc = wide ? P.G + (int64_t)xrow * P.ldg + 16 * P.jb0 + 8 * xch
                              : P.G + (int64_t)(lane >> 1) * P.ldg + 16 * P.jb0 + 8 * (lane & 1);
  auto issue = [&](int b, int s) {
    const int64_t t0 = (int64_t)b * 64;
    char* xs = wreg + s * STG;
#pragma unroll
    for (int q = 0; q < 8; ++q)
      __builtin_amdgcn_global_load_lds((lgptr_t)(xsrc + (t0 + 8 * q) * P.ldx), (llptr_t)(xs + q * 1024), 16, 0, 0);
    if (wide) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
        __builtin_amdgcn_global_load_lds((lgptr_t)(gsrc + (t0 + 8 * q) * P.ldg), (llptr_t)(xs + XB + q * 1024), 16, 0,
                                         0);
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((lgptr_t)(gsrc + (t0 + 32 * q) * P.ldg), (llptr_t)(xs + XB + q * 1024), 16,
                                         0, 0);
    }
  };
  // transposed-read lane bases: row 4 g + qq of each 16-row group, logical cols 16 blk + 4 pp
  const int fl = xsw(4 * g + qq);
  uint32_t xb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xb[i] = wbase + (4 * g + qq) * 128 + 16 * ((2 * i + (pp >> 1)) ^ fl) + 8 * (pp & 1);
  const uint32_t gnb = wbase + XB + (4 * g + qq) * 32 + 8 * pp;  // narrow G image: 32-B rows

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto block = [&](auto SC, int b) {
    constexpr int s = decltype(SC)::value;
    // this block's DMA has landed (the next block's may still be in flight)
    if (b + 1 < b1) {
      if (wide) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    u16x4 xr[2][2][4], gr[2][2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) xr[ks][h][i] = trd_off(xb[i], s * STG + (32 * ks + 16 * h) * 128);
        if (wide) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < JB) gr[ks][h][j] = trd_off(xb[j], s * STG + XB + (32 * ks + 16 * h) * 128);
        } else {
          gr[ks][h][0] = trd_off(gnb, s * STG + (32 * ks + 16 * h) * 32);
        }
      }
    lds_wait();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) pin(xr[ks][h][i]);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < JB) pin(gr[ks][h][j]);
      }
    if (b + 2 < b1) issue(b + 2, s);  // refill this stage (its reads have retired)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j >= JB) continue;
        const u16x8 bf = u16x8{gr[ks][0][j][0], gr[ks][0][j][1], gr[ks][0][j][2], gr[ks][0][j][3],
                               gr[ks][1][j][0], gr[ks][1][j][1], gr[ks][1][j][2], gr[ks][1][j][3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u16x8 af = u16x8{xr[ks][0][i][0], xr[ks][0][i][1], xr[ks][0][i][2], xr[ks][0][i][3],
                                 xr[ks][1][i][0], xr[ks][1][i][1], xr[ks][1][i][2], xr[ks][1][i][3]};
          acc[i][j] = lmfma(af, bf, acc[i][j]);
        }
      }
    }
  };
  if (wide || !a.narrow3) {
    if (b0 < b1) issue(b0, 0);
    if (b0 + 1 < b1) issue(b0 + 1, 1);
    for (int b = b0; b < b1; b += 2) {
      block(std::integral_constant<int, 0>{}, b);
      if (b + 1 < b1) block(std::integral_constant<int, 1>{}, b + 1);
    }
  } else {
    // narrow G (one 16-column block, 2 KiB per 64-row block): a stage is X 8 KiB + G 2 KiB, so the
    // wave's 32 KiB hold THREE stages -- two blocks in flight behind the one being read instead of
    // one (~80 KiB of DMA in flight per CU, the HBM-latency cover of MI355X_MICROARCH §Indexed
    // rows; with two stages these streams ran at ~3.6 TB/s, archive/profiles/r4_final6)
    constexpr int STN = XB + 2048;
    auto issue3 = [&](int b, int st) {
      const int64_t t0 = (int64_t)b * 64;
      char* xs = wreg + st * STN;
#pragma unroll
      for (int q = 0; q < 8; ++q)
        __builtin_amdgcn_global_load_lds((lgptr_t)(xsrc + (t0 + 8 * q) * P.ldx), (llptr_t)(xs + q * 1024), 16, 0, 0);
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((lgptr_t)(gsrc + (t0 + 32 * q) * P.ldg), (llptr_t)(xs + XB + q * 1024), 16,
                                         0, 0);
    };
    auto block3 = [&](auto SC, int b) {
      constexpr int st = decltype(SC)::value;
      // this block's 10 DMA instructions landed; the (up to two) later blocks' may still fly
      if (b + 2 < b1) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
      else if (b + 1 < b1) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      u16x4 xr[2][2][4], gr[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int i = 0; i < 4; ++i) xr[ks][h][i] = trd_off(xb[i], st * STN + (32 * ks + 16 * h) * 128);
          gr[ks][h] = trd_off(gnb, st * STN + (32 * ks + 16 * h) * 32);
        }
      lds_wait();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int i = 0; i < 4; ++i) pin(xr[ks][h][i]);
          pin(gr[ks][h]);
        }
      if (b + 3 < b1) issue3(b + 3, st);  // refill this stage (its reads have retired)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const u16x8 bf = u16x8{gr[ks][0][0], gr[ks][0][1], gr[ks][0][2], gr[ks][0][3],
                               gr[ks][1][0], gr[ks][1][1], gr[ks][1][2], gr[ks][1][3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u16x8 af = u16x8{xr[ks][0][i][0], xr[ks][0][i][1], xr[ks][0][i][2], xr[ks][0][i][3],
                                 xr[ks][1][i][0], xr[ks][1][i][1], xr[ks][1][i][2], xr[ks][1][i][3]};
          acc[i][0] = lmfma(af, bf, acc[i][0]);
        }
      }
    };
    if (b0 < b1) issue3(b0, 0);
    if (b0 + 1 < b1) issue3(b0 + 1, 1);
    if (b0 + 2 < b1) issue3(b0 + 2, 2);
    for (int b = b0; b < b1; b += 3) {
      block3(std::integral_constant<int, 0>{}, b);
      if (b + 1 < b1) block3(std::integral_constant<int, 1>{}, b + 1);
      if (b + 2 < b1) block3(std::integral_constant<int, 2>{}, b + 2);
    }
  }
  // 4 waves -> one 64 x 16 JB tile in LDS (each wave's own region; its DMA has drained)
  float* rw = reinterpret_cast<float*>(wreg);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (j >= JB) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) rw[(16 * i + 4 * g + e) * kRS + 16 * j + c] = acc[i][j][e];
    }
  if (a.wt) {  // this wave's whole tile (S == 1): read its own image back, write the outputs
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const int J = 16 * JB, nel = 64 * J;
    const bool jfast = P.os_j == 1;
    for (int e = lane; e < nel; e += 64) {
      const int n = jfast ? e / J : (e & 63), j = jfast ? e % J : (e >> 6);
      uint16_t* o = P.out + (int64_t)(n0 + n) * P.os_n + (int64_t)j * P.os_j;
      const float r = a.alpha * rw[n * kRS + j] + (a.accumulate ? bf2f(*o) : 0.f);
      *o = f2bf(r);
    }
    return;
  }
  __syncthreads();
  const int J = 16 * JB, nel = 64 * J;
  const bool jfast = P.os_j == 1;
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q;
    v[q] = 0.f;
    if (e < nel) {
      const int n = jfast ? e / J : (e & 63), j = jfast ? e % J : (e >> 6);
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) s += reinterpret_cast<const float*>(smem + ww * WREG)[n * kRS + j];
      v[q] = s;
    }
  }
  if (a.S > 1) {
    float* wp = ws + ((int64_t)split * a.ntiles + tile) * 4096;
    if (!a.fused_red) {  // lora_xtg_reduce_kernel finishes
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (tid + 256 * q < nel) wp[tid + 256 * q] = v[q];
      return;
    }
    // in-launch merge, sc1 hand-off (see arrive_last_sc1)
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (tid + 256 * q < nel) __hip_atomic_store(wp + tid + 256 * q, v[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!arrive_last_sc1(&g_xtg_cnt[tile], a.S, &s_last)) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = tid + 256 * q;
      if (e < nel) {
        float s = __hip_atomic_load(ws + (int64_t)tile * 4096 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int sp = 1; sp < a.S; ++sp)
          s += __hip_atomic_load(ws + ((int64_t)sp * a.ntiles + tile) * 4096 + e, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        v[q] = s;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int e = tid + 256 * q;
    if (e < nel) {
      const int n = jfast ? e / J : (e & 63), j = jfast ? e % J : (e >> 6);
      uint16_t* o = P.out + (int64_t)(n0 + n) * P.os_n + (int64_t)j * P.os_j;
      const float r = a.alpha * v[q] + (a.accumulate ? bf2f(*o) : 0.f);
      *o = f2bf(r);
    }
  }
}

// split partials -> outputs (fixed split order); grid ntiles
__global__ void __launch_bounds__(256) lora_xtg_reduce_kernel(const XtgArgs a, const float* __restrict__ ws) {
  const int tile = blockIdx.x, tid = threadIdx.x;
  XtgProb P = a.p[0];
#pragma unroll
  for (int i = 1; i < kMaxProb; ++i)
    if (i < a.np && tile >= a.p[i].tile0) P = a.p[i];
  const int n0 = (tile - P.tile0) * 64, J = 16 * P.JB, nel = 64 * J;
  const bool jfast = P.os_j == 1;
  for (int e = tid; e < nel; e += 256) {
    float s = ws[(int64_t)tile * 4096 + e];
    for (int sp = 1; sp < a.S; ++sp) s += ws[((int64_t)sp * a.ntiles + tile) * 4096 + e];
    const int n = jfast ? e / J : (e & 63), j = jfast ? e % J : (e >> 6);
    uint16_t* o = P.out + (int64_t)(n0 + n) * P.os_n + (int64_t)j * P.os_j;
    *o = f2bf(a.alpha * s + (a.accumulate ? bf2f(*o) : 0.f));
  }
}

// ------------------------------------------------------------------ SwiGLU + LoRA tail
// The SwiGLU pass that also produces the rank-r LoRA product of its own output for the
// neighbouring augmented GEMM, so that product no longer re-streams the [T, F] / [T, 2F]
// tensor through lora_xwt (70B: 235 MB per layer forward, 470 MB backward):
//   FWD: m = silu(g) u            -> out[:, :F];   tail = s m . V^T   (V = A of the down projection, [*, F])
//   BWD: dg, du (swiglu_bwd math) -> out[:, :2F];  tail = s [dg | du] . V^T   (V = B^T of gate-up, [*, 2F])
// grid (T/16, CS), 256 threads.  A workgroup owns 16 token rows and a contiguous range of
// 128-column tiles of F.  Per tile every thread moves 16 B per operand (row tid >> 4, chunk
// tid & 15: 256-B row segments, the same coalescing as the plain SwiGLU kernels), writes the
// bf16 result to global AND to a double-buffered LDS image, and after ONE barrier the 4 waves
// read that image back as MFMA A-fragments (wave w: columns 32 w .. 32 w + 31 of the tile;
// BWD: of the dg and the du image) against V fragments straight from L2 (16 rank rows x 64 B).
// The next tile's operands are loaded before this tile's math, after this tile's V loads, so
// the MFMA's counted wait never drains the prefetch.  Per-wave 16 x 16 NRB fp32 accumulators
// -> LDS -> one partial per (split, row block) in ws; swiglu_lora_reduce_kernel sums the CS
// partials in split order (bit-reproducible), scales by s and writes the whole pad (zeros past
// 16 NRB columns).  The elementwise math is bitwise that of swiglu_fwd_kernel /
// swiglu_bwd_kernel (csrc/kernels/elementwise.hip).
constexpr int kSlRow = 136;  // LDS image row stride (elements): 272 B -> conflict-free b128 fragment reads

__device__ __forceinline__ float sl_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

template <bool BWD, int NRB, int RBW>
__global__ void __launch_bounds__(256) swiglu_lora_kernel(const uint16_t* __restrict__ gu,
                                                          const uint16_t* __restrict__ dm, uint16_t* __restrict__ out,
                                                          int64_t ldo, const uint16_t* __restrict__ V, int64_t ldv,
                                                          float* __restrict__ ws, int F, int CS) {
  // RBW 16-row blocks per workgroup share every V fragment (V is read from L2 / the MALL once per
  // 16 RBW tokens instead of once per 16)
  constexpr int NP = BWD ? 2 : 1;  // LDS images per tile (BWD: dg, du)
  constexpr int NC = 16 * NRB;
  __shared__ __attribute__((aligned(16))) uint16_t img[2][NP][RBW][16 * kSlRow];
  __shared__ __attribute__((aligned(16))) float red[4][16][NC + 4];
  const int rg = blockIdx.x, split = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, r = lane & 15, gq = lane >> 4;
  const int row = tid >> 4, ch = tid & 15;
  const int tiles = F >> 7;
  const int t0 = (int)((int64_t)split * tiles / CS), t1 = (int)((int64_t)(split + 1) * tiles / CS);
  const int64_t tok = (int64_t)rg * 16 * RBW + row;
  const uint16_t* grow = gu + tok * (2 * (int64_t)F) + 8 * ch;
  const uint16_t* drow = dm + tok * (int64_t)F + 8 * ch;  // BWD only
  uint16_t* orow = out + tok * ldo + 8 * ch;
  const int64_t gstep = 16 * (2 * (int64_t)F), dstep = 16 * (int64_t)F, ostep = 16 * ldo;  // next row block
  const uint16_t* vrow = V + (int64_t)r * ldv + 32 * w + 8 * gq;
  const int wofs = row * kSlRow + 8 * ch, rofs = r * kSlRow + 32 * w + 8 * gq;

  f32x4 acc[RBW][NRB];
#pragma unroll
  for (int i = 0; i < RBW; ++i)
#pragma unroll
    for (int b = 0; b < NRB; ++b) acc[i][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  u16x8 g[RBW], u[RBW], d[RBW], vf[NP][NRB];
  auto vload = [&](int t) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int b = 0; b < NRB; ++b)
        vf[p][b] = *reinterpret_cast<const u16x8*>(vrow + (int64_t)(16 * b) * ldv + p * F + (t << 7));
  };
  auto load = [&](int t, u16x8(&g_)[RBW], u16x8(&u_)[RBW], u16x8(&d_)[RBW]) {
    const int c = t << 7;
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      g_[i] = *reinterpret_cast<const u16x8*>(grow + i * gstep + c);
      u_[i] = *reinterpret_cast<const u16x8*>(grow + i * gstep + F + c);
      if (BWD) d_[i] = *reinterpret_cast<const u16x8*>(drow + i * dstep + c);
    }
  };
  if (t0 < t1) {
    load(t0, g, u, d);
    vload(t0);
  }
  for (int t = t0; t < t1; ++t) {
    const int c = t << 7, buf = (t - t0) & 1;
    u16x8 gn[RBW], un[RBW], dn[RBW];
    load(t + 1 < t1 ? t + 1 : t, gn, un, dn);  // the last trip reloads its own tile (no branch)
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      u16x8 o0, o1;
      if (!BWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gf = bf2f(g[i][j]);
          o0[j] = f2bf(gf * sl_sigmoid(gf) * bf2f(u[i][j]));
        }
        *reinterpret_cast<u16x8*>(orow + i * ostep + c) = o0;
        *reinterpret_cast<u16x8*>(&img[buf][0][i][wofs]) = o0;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gf = bf2f(g[i][j]), uf = bf2f(u[i][j]), df = bf2f(d[i][j]);
          float dg, du;
          swiglu_grad(df, gf, uf, dg, du);
          o0[j] = f2bf(dg);
          o1[j] = f2bf(du);
        }
        *reinterpret_cast<u16x8*>(orow + i * ostep + c) = o0;
        *reinterpret_cast<u16x8*>(orow + i * ostep + F + c) = o1;
        *reinterpret_cast<u16x8*>(&img[buf][0][i][wofs]) = o0;
        *reinterpret_cast<u16x8*>(&img[buf][NP - 1][i][wofs]) = o1;
      }
    }
    __syncthreads();  // the image is complete; the other buffer's readers (trip t-1) are past it
#pragma unroll
    for (int i = 0; i < RBW; ++i)
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(&img[buf][p][i][rofs]);
#pragma unroll
        for (int b = 0; b < NRB; ++b) acc[i][b] = lmfma(a, vf[p][b], acc[i][b]);
      }
    vload(t + 1 < t1 ? t + 1 : t);  // next tile's V fragments under this tile's tail and the next math
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      g[i] = gn[i], u[i] = un[i];
      if (BWD) d[i] = dn[i];
    }
  }
  // per row block: 4 waves -> one 16 x NC partial (fixed wave order)
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    __syncthreads();  // red reused per row block
#pragma unroll
    for (int b = 0; b < NRB; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][4 * gq + e][16 * b + r] = acc[i][b][e];
    __syncthreads();
    float* wp = ws + ((int64_t)split * (gridDim.x * RBW) + rg * RBW + i) * (16 * NC);
    for (int k = tid; k < 16 * NC; k += 256) {
      const int rr = k / NC, cc = k % NC;
      wp[k] = ((red[0][rr][cc] + red[1][rr][cc]) + red[2][rr][cc]) + red[3][rr][cc];
    }
  }
}

// ws[CS][T/16][16][NC] -> tail[:, 0:pad] = bf16(alpha * sum over splits), zeros past NC; grid T/16
__global__ void __launch_bounds__(256) swiglu_lora_reduce_kernel(const float* __restrict__ ws, int CS, int NC, int pad,
                                                                 uint16_t* __restrict__ tail, int64_t ldo, float alpha) {
  const int rb = blockIdx.x, nrb = gridDim.x;
  for (int i = threadIdx.x; i < 16 * pad; i += 256) {
    const int rr = i / pad, cc = i % pad;
    float v = 0.f;
    if (cc < NC)
      for (int sp = 0; sp < CS; ++sp) v += ws[(((int64_t)sp * nrb + rb) * 16 + rr) * NC + cc];
    tail[((int64_t)rb * 16 + rr) * ldo + cc] = f2bf(alpha * v);
  }
}

// lora_xwt, row-tiled ("tile") form: out[:, 0:pad] = alpha X V[:16 NRB]^T with the structure of
// swiglu_lora_kernel minus the elementwise math: a workgroup owns 16 RBW token rows and a range
// of 128-column tiles; per tile each thread loads RBW 16-B pieces of X (256-B row segments),
// stores them to a double-buffered LDS image, one barrier, and each wave multiplies its 32-column
// slice of all RBW row blocks against NRB V fragments from L2 (loaded one tile ahead, SHARED by the
// RBW row blocks).  Only the 16 NRB rows of V that hold the adapter are read (the LDS-DMA kernels
// above multiply all 64 padded rows and re-read V once per 64 rows).  Partials ws[CS][T/16][16][NC]
// -> swiglu_lora_reduce_kernel (fixed split order).  grid (T / (16 RBW), CS), 256 threads.
template <int NRB, int RBW>
__global__ void __launch_bounds__(256) lora_xwt_tile_kernel(const uint16_t* __restrict__ X, int64_t ldx,
                                                            const uint16_t* __restrict__ V, int64_t ldv,
                                                            float* __restrict__ ws, int K, int CS) {
  constexpr int NC = 16 * NRB;
  __shared__ __attribute__((aligned(16))) uint16_t img[2][RBW][16 * kSlRow];
  __shared__ __attribute__((aligned(16))) float red[4][16][NC + 4];
  const int rg = blockIdx.x, split = blockIdx.y, tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6, r = lane & 15, gq = lane >> 4;
  const int row = tid >> 4, ch = tid & 15;
  const int tiles = K >> 7;
  const int t0 = (int)((int64_t)split * tiles / CS), t1 = (int)((int64_t)(split + 1) * tiles / CS);
  const uint16_t* xrow = X + ((int64_t)rg * 16 * RBW + row) * ldx + 8 * ch;
  const int64_t xstep = 16 * ldx;  // next 16-row block
  const uint16_t* vrow = V + (int64_t)r * ldv + 32 * w + 8 * gq;
  const int wofs = row * kSlRow + 8 * ch, rofs = r * kSlRow + 32 * w + 8 * gq;

  f32x4 acc[RBW][NRB];
#pragma unroll
  for (int i = 0; i < RBW; ++i)
#pragma unroll
    for (int b = 0; b < NRB; ++b) acc[i][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  u16x8 x[RBW], vf[NRB];
  auto xload = [&](int t, u16x8(&dst)[RBW]) {
#pragma unroll
    for (int i = 0; i < RBW; ++i) dst[i] = *reinterpret_cast<const u16x8*>(xrow + i * xstep + (t << 7));
  };
  auto vload = [&](int t) {
#pragma unroll
    for (int b = 0; b < NRB; ++b) vf[b] = *reinterpret_cast<const u16x8*>(vrow + (int64_t)(16 * b) * ldv + (t << 7));
  };
  if (t0 < t1) {
    xload(t0, x);
    vload(t0);
  }
  for (int t = t0; t < t1; ++t) {
    const int buf = (t - t0) & 1;
    u16x8 xn[RBW];
    xload(t + 1 < t1 ? t + 1 : t, xn);  // the last trip reloads its own tile (no branch)
#pragma unroll
    for (int i = 0; i < RBW; ++i) *reinterpret_cast<u16x8*>(&img[buf][i][wofs]) = x[i];
    __syncthreads();  // image complete; the other buffer's readers (trip t-1) are past it
#pragma unroll
    for (int i = 0; i < RBW; ++i) {
      const u16x8 a = *reinterpret_cast<const u16x8*>(&img[buf][i][rofs]);
#pragma unroll
      for (int b = 0; b < NRB; ++b) acc[i][b] = lmfma(a, vf[b], acc[i][b]);
    }
    vload(t + 1 < t1 ? t + 1 : t);
#pragma unroll
    for (int i = 0; i < RBW; ++i) x[i] = xn[i];
  }
  // per row block: 4 waves -> one 16 x NC partial (fixed wave order)
#pragma unroll
  for (int i = 0; i < RBW; ++i) {
    __syncthreads();  // red reused per row block
#pragma unroll
    for (int b = 0; b < NRB; ++b)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[w][4 * gq + e][16 * b + r] = acc[i][b][e];
    __syncthreads();
    float* wp = ws + ((int64_t)split * (gridDim.x * RBW) + rg * RBW + i) * (16 * NC);
    for (int k = tid; k < 16 * NC; k += 256) {
      const int rr = k / NC, cc = k % NC;
      wp[k] = ((red[0][rr][cc] + red[1][rr][cc]) + red[2][rr][cc]) + red[3][rr][cc];
    }
  }
}

}  // namespace mx

using namespace mx;

static int lora_env(const char* name, int dflt);

// row blocks of 16 tokens per workgroup sharing the V fragments (MXLLM_SWIGLU_LORA_RBW: 1, 2 or 4;
// clamped to divide T / 16).  2 by default: 70B backward 273 -> 249 us, headline -2.6 ms (r4p)
static int swiglu_lora_rbw(int T) {
  int rbw = lora_env("MXLLM_SWIGLU_LORA_RBW", 2);
  rbw = rbw >= 4 ? 4 : (rbw >= 2 ? 2 : 1);
  while (rbw > 1 && (T / 16) % rbw) rbw >>= 1;
  return rbw;
}

static int swiglu_lora_splits(int T, int F) {
  const int tiles = F / 128, rbs = T / (16 * swiglu_lora_rbw(T));
  int cs = lora_env("MXLLM_SWIGLU_LORA_CS", 0);
  if (cs <= 0) cs = (512 + rbs - 1) / rbs;  // ~512 workgroups (T 4096: 2 splits; measured best of 1-16, r4h)
  cs = cs < 1 ? 1 : cs;
  cs = cs > tiles ? tiles : cs;
  return cs > 32 ? 32 : cs;
}

extern "C" int64_t mx_swiglu_lora_ws(int T, int F, int nrb) {
  if (T <= 0 || F < 128) return 0;
  return (int64_t)swiglu_lora_splits(T, F) * T * 16 * nrb;
}

// bwd = 0: out[T, F (+pad)] = swiglu(gu), tail out[:, F:F+pad] = alpha m V^T (V [>= 16 nrb, F]);
// bwd = 1: out[T, 2F (+pad)] = swiglu_bwd(dm, gu), tail out[:, 2F:2F+pad] = alpha dgu V^T (V [.., 2F]).
// T % 16 == 0, F % 128 == 0, 1 <= nrb <= 4, 16 nrb <= pad, 16-B aligned rows.
extern "C" int mx_swiglu_lora(int bwd, const uint16_t* gu, const uint16_t* dm, uint16_t* out, int64_t ldo,
                              const uint16_t* V, int64_t ldv, int nrb, int pad, float alpha, float* ws, int T, int F,
                              hipStream_t stream) {
  if (T <= 0) return 0;
  if (T % 16 || F % 128 || nrb < 1 || nrb > 4 || pad < 16 * nrb || pad % 8 || ldo % 8 || ldv % 8 ||
      ldo < (bwd ? 2 * (int64_t)F : F) + pad || ((uintptr_t)gu | (uintptr_t)out | (uintptr_t)V) % 16 ||
      (bwd && (!dm || (uintptr_t)dm % 16)))
    return (int)hipErrorInvalidValue;
  const int CS = swiglu_lora_splits(T, F), RBW = swiglu_lora_rbw(T);
  const dim3 grid(T / (16 * RBW), CS);
#define MX_SL_R(B, N, R) swiglu_lora_kernel<B, N, R><<<grid, 256, 0, stream>>>(gu, dm, out, ldo, V, ldv, ws, F, CS)
#define MX_SL(B, N)                                 \
  do {                                              \
    if (RBW == 4) MX_SL_R(B, N, 4);                 \
    else if (RBW == 2) MX_SL_R(B, N, 2);            \
    else MX_SL_R(B, N, 1);                          \
  } while (0)
  if (bwd) {
    switch (nrb) { case 1: MX_SL(true, 1); break; case 2: MX_SL(true, 2); break;
                   case 3: MX_SL(true, 3); break; default: MX_SL(true, 4); break; }
  } else {
    switch (nrb) { case 1: MX_SL(false, 1); break; case 2: MX_SL(false, 2); break;
                   case 3: MX_SL(false, 3); break; default: MX_SL(false, 4); break; }
  }
#undef MX_SL
#undef MX_SL_R
  swiglu_lora_reduce_kernel<<<T / 16, 256, 0, stream>>>(ws, CS, 16 * nrb, pad, out + (bwd ? 2 * (int64_t)F : F), ldo,
                                                        alpha);
  return (int)hipGetLastError();
}

// split count of the ordered split reduction: ~512 workgroups, >= 2 blocks per wave
static int lora_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
static int lora_splits(int tiles, int blocks, int smax) {
  if (tiles <= 0) return 1;
  const int target = lora_env("MXLLM_LORA_WGS", 256);  // tuning knob: workgroups to aim for
  int S = (target + tiles - 1) / tiles;
  S = S < 1 ? 1 : (S > smax ? smax : S);
  while (S > 1 && blocks / (4 * S) < 2) --S;
  return S;
}

// lora_xtg with one 64-col tile per WAVE (XtgArgs::wt) where that still fills the chip with one
// workgroup per CU and no row split (>= 4 waves x 256 CUs = 1,024 tiles: the 70B gate-up gradients): 119.1 -> 100.1 us per launch at T 4096 (profiles/r6g/: one round of 256 workgroups instead
// of four of 1,024, and no cross-wave reduction); the smaller launches do not qualify and measured
// the same when forced.  MXLLM_LORA_XTG_WT=0 restores the row-split form (read per call: A/B)
static bool xtg_wave_tiles(int ntiles) {
  return lora_env("MXLLM_LORA_XTG_WT", 1) == 1 && ntiles >= lora_env("MXLLM_LORA_XTG_WT_MIN", 1024);
}

// lora_xwt kernel choice (MXLLM_LORA_XWT, read per call: an in-process A/B can flip it):
// "lds" (default) = the 64-row LDS-DMA kernel, "reg" = the register-fragment kernel (both on all
// 64 padded rows of V), "tile" = lora_xwt_tile_kernel (adapter rows only; needs M % 16, K % 128,
// <= 64 adapter rows, 16-B aligned rows).  The tile kernel measured 3-7 us SLOWER on the 64-84 MB
// calls of the 70B step (archive/profiles/r4i: those calls are bound by their fixed cost, not by bytes).
static int xwt_mode() {
  const char* kv = getenv("MXLLM_LORA_XWT");
  if (kv && !strcmp(kv, "reg")) return 2;
  if (kv && !strcmp(kv, "tile")) return 0;
  return 1;
}
static bool xwt_tile_ok(const void* X, int64_t ldx, const void* V, int64_t ldv, int M, int K, int rows) {
  return xwt_mode() == 0 && M % 16 == 0 && K % 128 == 0 && rows > 0 && rows <= 64 && ldx % 8 == 0 &&
         ldv % 8 == 0 && (uintptr_t)X % 16 == 0 && (uintptr_t)V % 16 == 0;
}
static int xwt_rbw(int M) { return M % 64 == 0 ? 4 : (M % 32 == 0 ? 2 : 1); }
static int xwt_tile_splits(int M, int K) {
  const int groups = M / (16 * xwt_rbw(M)), tiles = K / 128;
  int cs = lora_env("MXLLM_LORA_XWT_CS", 0);
  if (cs <= 0) cs = (512 + groups - 1) / groups;  // ~512 workgroups
  cs = cs < 1 ? 1 : cs;
  return cs > tiles ? tiles : cs;
}

// fp32 workspace floats needed by mx_lora_xwt (M, K, adapter rows; 0 = all) / mx_lora_xtg (total 64-col tiles, T)
extern "C" int64_t mx_lora_xwt_ws(int M, int K, int rows) {
  const int S = M >= 64 && K >= 64 ? lora_splits(M / 64, K / 64, 16) : 1;
  const int64_t dma = S > 1 ? (int64_t)S * (M / 64) * 4096 : 0;
  if (rows > 0 && rows <= 64 && M % 16 == 0 && K % 128 == 0 && xwt_mode() == 0) {
    const int64_t tile = (int64_t)xwt_tile_splits(M, K) * M * 16 * ((rows + 15) / 16);
    return tile > dma ? tile : dma;
  }
  return dma;
}
extern "C" int64_t mx_lora_xtg_ws(int ntiles, int T) {
  if (xtg_wave_tiles(ntiles)) return 0;
  const int S = lora_splits(ntiles, T / 64, 8);
  return S > 1 ? (int64_t)S * ntiles * 4096 : 0;
}

// out[:, 0:Vrows] = alpha X V^T.  rows > 0: only V's first `rows` rows are non-zero (the adapter;
// the rest is padding) -> the row-tiled kernel computes those and writes zeros past them.
extern "C" int mx_lora_xwt(const uint16_t* X, int64_t ldx, const uint16_t* V, int64_t ldv, int Vrows, uint16_t* out,
                           int64_t ldo, float* ws, int M, int K, float alpha, int rows, hipStream_t stream) {
  if (M <= 0) return 0;
  if (xwt_tile_ok(X, ldx, V, ldv, M, K, rows) && rows <= Vrows && ldo % 4 == 0) {
    const int nrb = (rows + 15) / 16, rbw = xwt_rbw(M), CS = xwt_tile_splits(M, K);
    const dim3 grid(M / (16 * rbw), CS);
#define MX_XT(N, R) lora_xwt_tile_kernel<N, R><<<grid, 256, 0, stream>>>(X, ldx, V, ldv, ws, K, CS)
#define MX_XT_N(R)                                  \
  switch (nrb) {                                    \
    case 1: MX_XT(1, R); break;                     \
    case 2: MX_XT(2, R); break;                     \
    case 3: MX_XT(3, R); break;                     \
    default: MX_XT(4, R); break;                    \
  }
    if (rbw == 4) { MX_XT_N(4) } else if (rbw == 2) { MX_XT_N(2) } else { MX_XT_N(1) }
#undef MX_XT_N
#undef MX_XT
    swiglu_lora_reduce_kernel<<<M / 16, 256, 0, stream>>>(ws, CS, 16 * nrb, Vrows, out, ldo, alpha);
    return (int)hipGetLastError();
  }
  if (M % 64 || K % 64 || Vrows % 64 || M / 64 > kMaxTiles) return (int)hipErrorInvalidValue;
  const int mtiles = M / 64, S = lora_splits(mtiles, K / 64, 16);
  const int fused = lora_env("MXLLM_LORA_FUSED_RED", 0);
  // LDS-staged kernel (16-B aligned rows required by its 16-B DMA pieces); the
  // register-fragment kernel stays for A/B (MXLLM_LORA_XWT=reg)
  const bool lds = xwt_mode() != 2 && ((uintptr_t)X % 16 == 0) && ((uintptr_t)V % 16 == 0) && ldx % 8 == 0 &&
                   ldv % 8 == 0;
  for (int c0 = 0; c0 < Vrows; c0 += 64) {
    if (lds)
      lora_xwt_lds_kernel<<<dim3(mtiles, S), 256, 0, stream>>>(X, ldx, V + (int64_t)c0 * ldv, ldv, out + c0, ldo, ws,
                                                               M, K, S, alpha, fused);
    else
      lora_xwt_kernel<<<dim3(mtiles, S), 256, 0, stream>>>(X, ldx, V + (int64_t)c0 * ldv, ldv, out + c0, ldo, ws, M,
                                                           K, S, alpha, fused);
    if (S > 1 && !fused) {
      const int qpw = lora_env("MXLLM_LORA_XWT_RED_ROWS", 16) >= 64 ? 4 : 1;
      lora_xwt_reduce_kernel<<<(4 / qpw) * mtiles, 256, 0, stream>>>(ws, S, mtiles, out + c0, ldo, alpha, qpw);
    }
  }
  return (int)hipGetLastError();
}

// Batched sum_t X[t, n] G[t, j] problems (see XtgProb).  desc: np rows of
// {X, G, out, ldx, ldg, os_n, os_j, Nx, jb0, JB} as int64; ws: mx_lora_xtg_ws floats.
extern "C" int mx_lora_xtg(const int64_t* desc, int np, int T, float alpha, int accumulate, float* ws,
                           hipStream_t stream) {
  if (np <= 0 || np > kMaxProb || T % 64) return (int)hipErrorInvalidValue;
  if (T == 0) return 0;
  XtgArgs a{};
  int ntiles = 0;
  for (int i = 0; i < np; ++i) {
    const int64_t* d = desc + i * 10;
    XtgProb& p = a.p[i];
    p.X = reinterpret_cast<const uint16_t*>(d[0]);
    p.G = reinterpret_cast<const uint16_t*>(d[1]);
    p.out = reinterpret_cast<uint16_t*>(d[2]);
    p.ldx = d[3], p.ldg = d[4], p.os_n = d[5], p.os_j = d[6];
    p.Nx = (int)d[7], p.jb0 = (int)d[8], p.JB = (int)d[9];
    if (p.Nx <= 0 || p.Nx % 64 || p.JB < 1 || p.JB > 4) return (int)hipErrorInvalidValue;
    p.tile0 = ntiles;
    ntiles += p.Nx / 64;
  }
  if (ntiles > kMaxTiles) return (int)hipErrorInvalidValue;
  a.np = np, a.T = T, a.ntiles = ntiles, a.alpha = alpha;
  a.wt = xtg_wave_tiles(ntiles);
  a.S = a.wt ? 1 : lora_splits(ntiles, T / 64, 8);
  a.accumulate = accumulate;
  a.fused_red = a.wt ? 0 : lora_env("MXLLM_LORA_FUSED_RED", 0);
  a.narrow3 = lora_env("MXLLM_LORA_XTG_STAGES", 3) == 3;
  lora_xtg_kernel<<<dim3(a.wt ? (ntiles + 3) / 4 : ntiles, a.S), 256, 0, stream>>>(a, ws);
  if (a.S > 1 && !a.fused_red) lora_xtg_reduce_kernel<<<ntiles, 256, 0, stream>>>(a, ws);
  return (int)hipGetLastError();
}
