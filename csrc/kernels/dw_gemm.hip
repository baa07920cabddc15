// Weight-gradient GEMM on token-major operands for gfx950.
//
//   C[M, N] = beta * C + alpha * dY^T X,   dY [T, M] and X [T, N] row-major (token-major),
//   reduction over the T tokens, fp32 accumulation, C fp32 or bf16.
//
// Both operands arrive as the producers wrote them: the reduction dimension is the ROW index of
// each, so neither is "k-contiguous".  hipBLASLt runs this form ("NT") at 0.93-1.15 PF on the
// Llama projections, which is why mxllm/ops/linear.py transposed both operands first (HIP
// transpose, 4.4-6.4 TB/s) and called the 1.2-1.5 PF "TN" kernel -- 258 transpose launches /
// 6.9 ms per 8B step, 642 / 73 ms per 70B ZeRO-3 rank step.  Here the transpose happens in the
// LDS read instead:
//  * workgroup = 4 waves, 256 x 256 output tile, 2 x 2 waves of 128 x 128 (4 x 4 blocks of
//    v_mfma_f32_32x32x16_bf16, 256 fp32 accumulators per lane);
//  * 32-token stages of dY[:, m0:m0+256] and X[:, n0:n0+256] stream into LDS by LDS-DMA
//    (global_load_lds_dwordx4, 8 x 1-KiB lane-linear pieces per wave and stage) through a
//    4-stage ring (128 KiB) with two stages in flight across every barrier (counted vmcnt, raw
//    s_barrier: guide §5 T3/T4); each 512-B row is stored as a 16-B-chunk XOR-swizzled image
//    (chunk ^ swz(row) inside each 256-B half), produced by permuting each lane's SOURCE chunk;
//  * MFMA operand fragments (8 consecutive tokens of one row of dY^T / column of X) are
//    ds_read_b64_tr_b16 transposed reads of those images: conflict-free (a 16-lane group reads
//    4 rows x 32 B that the swizzle puts on 32 distinct banks);
//  * the next 16-token step's fragments are read under the current step's MFMAs (<= 8 LDS
//    reads outstanding);
//  * workgroup -> tile: XCD-contiguous ranges (xcd_remap) of a grouped order (4 m-tiles x every
//    n-tile), so the ~32 co-resident tiles of one XCD share their dY / X panels in its L2.
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8_d __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(1))) const void* dgptr_t;
typedef __attribute__((address_space(3))) void* dlptr_t;

__device__ __forceinline__ f32x16 mfma32d(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_d, a), __builtin_bit_cast(bf16x8_d, b),
                                                 c, 0, 0, 0);
}

// 16-B chunk swizzle inside a 256-B half row (row & 15 only)
__device__ __forceinline__ int dswz16(int row) { return (((row & 3) << 2) | ((row >> 2) & 3)) & 15; }
__device__ __forceinline__ int dphys(int lc, int row) { return (lc & 16) | ((lc & 15) ^ dswz16(row)); }

constexpr int kDwBM = 256, kDwBN = 256, kDwBK = 32, kDwRowB = 512;
constexpr int kDwHalf = kDwBK * kDwRowB;  // one operand of one stage: 16 KiB
constexpr int kDwStage = 2 * kDwHalf;     // A | B
constexpr int kDwNB = 4;                  // stage ring: 128 KiB of LDS


// lane holds C[m0 + 128 wm + 32 i + 8 (r / 4) + 4 hh + r % 4][n0 + 128 wn + 32 j + lane % 32]; per m-block
// the 64 old values (beta) are loaded before any store (independent loads in flight)
template <bool OUT_F32, bool BETA, int NJ = 4>
__device__ __forceinline__ void dw_epilogue(const f32x16 (&acc)[4][NJ], void* __restrict__ C, int64_t ldc, int m0,
                                            int n0, int wm, int wn, int hh, int lane, float alpha) {
  const int ncol = n0 + 32 * NJ * wn + (lane & 31);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float old[NJ][16];
    if constexpr (BETA) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + 128 * wm + 32 * i + 8 * (r >> 2) + 4 * hh + (r & 3);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int64_t idx = m * ldc + ncol + 32 * j;
          if constexpr (OUT_F32)
            old[j][r] = reinterpret_cast<const float*>(C)[idx];
          else
            old[j][r] = bf2f(reinterpret_cast<const uint16_t*>(C)[idx]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + 128 * wm + 32 * i + 8 * (r >> 2) + 4 * hh + (r & 3);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float v = acc[i][j][r] * alpha;
        if constexpr (BETA) v += old[j][r];
        const int64_t idx = m * ldc + ncol + 32 * j;
        if constexpr (OUT_F32)
          reinterpret_cast<float*>(C)[idx] = v;
        else
          reinterpret_cast<uint16_t*>(C)[idx] = f2bf(v);
      }
    }
  }
}

template <bool OUT_F32, bool BETA>
__global__ void __launch_bounds__(256, 1)
dw_gemm_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
               void* __restrict__ C, int64_t ldc, int M, int N, int T, const float* __restrict__ alpha_t,
               float alpha_f) {
  // ONE __shared__ array (a second LDS object makes hipcc drain vmcnt before ds_reads)
  __shared__ __attribute__((aligned(1024))) char smem[kDwNB * kDwStage];
  const int nM = M / kDwBM, nN = N / kDwBN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int pm, pn;
  {
    constexpr int GM = 4;
    const int per = GM * nN, grp = L / per, first = grp * GM;
    const int rows = min(GM, nM - first), in = L - grp * per;
    pm = first + in % rows;
    pn = in / rows;
  }
  const int m0 = pm * kDwBM, n0 = pn * kDwBN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  // ---- LDS-DMA sources: per stage and operand 16 x 1-KiB pieces (rows 2q, 2q + 1); wave w
  // stores pieces q = 4 w + i of both operands (8 glds per wave and stage)
  constexpr int PPW = kDwBK / 2 / 4;  // pieces per wave and operand
  int aoff[PPW], boff[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int row = 2 * (PPW * w + i) + (lane >> 5), pc = lane & 31;
    const int lc = dphys(pc, row);  // XOR is an involution: the logical chunk stored in slot pc
    aoff[i] = row * (int)lda + 8 * lc;
    boff[i] = row * (int)ldb + 8 * lc;
  }
  const uint16_t* Ab = A + m0;
  const uint16_t* Bb = B + n0;
  auto issue = [&](int kt) __attribute__((always_inline)) {
    const uint16_t* a = Ab + (int64_t)kt * kDwBK * lda;
    const uint16_t* b = Bb + (int64_t)kt * kDwBK * ldb;
    char* da = smem + (kt % kDwNB) * kDwStage;
    char* db = da + kDwHalf;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      __builtin_amdgcn_global_load_lds((dgptr_t)(a + aoff[i]), (dlptr_t)(da + (PPW * w + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((dgptr_t)(b + boff[i]), (dlptr_t)(db + (PPW * w + i) * 1024), 16, 0, 0);
    }
  };

  // ---- transposed-read lane bases: rows 4 hh + tq (rA) and 8 + 4 hh + tq (rB) of each 16-token
  // step; logical column 32 blk + 16 (g & 1) + 4 tp  ->  lane (g, li) receives 4 tokens of column
  // 32 blk + 16 (g & 1) + li (the MFMA row/column l % 32), tokens {4hh..4hh+3, 8+4hh..8+4hh+3}
  // (the same permutation of the 16-token step for both operands)
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3, hh = lane >> 5;
  const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t abase[4][2], bbase[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int la = wm * 16 + 4 * i + 2 * (g & 1) + (tp >> 1);
    const int lb = wn * 16 + 4 * i + 2 * (g & 1) + (tp >> 1);
    abase[i][0] = lds0 + rA * kDwRowB + 16 * dphys(la, rA) + 8 * (tp & 1);
    abase[i][1] = lds0 + rB * kDwRowB + 16 * dphys(la, rB) + 8 * (tp & 1);
    bbase[i][0] = lds0 + kDwHalf + rA * kDwRowB + 16 * dphys(lb, rA) + 8 * (tp & 1);
    bbase[i][1] = lds0 + kDwHalf + rB * kDwRowB + 16 * dphys(lb, rB) + 8 * (tp & 1);
  }

  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Stage kt lives in ring slot kt % 4.  Two stages are in flight across every barrier: at the top
  // of iteration kt a counted vmcnt retires this wave's stage-kt DMA (stage kt + 1 stays in flight),
  // the raw barrier makes every wave's part visible and certifies that all waves finished reading
  // stage kt - 1, and stage kt + 2 is issued into slot (kt + 2) % 4, last read in iteration kt - 2.
  // Raw s_barrier, never __syncthreads(): its fence would drain the in-flight DMA (vmcnt(0)).
  const int nk = T / kDwBK;
  issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2);
    const uint32_t so = (uint32_t)(kt % kDwNB) * kDwStage;
    uint32_t ab[4][2], bb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ab[i][0] = abase[i][0] + so;
      ab[i][1] = abase[i][1] + so;
      bb[i][0] = bbase[i][0] + so;
      bb[i][1] = bbase[i][1] + so;
    }
    u16x4 fa[2][4][2], fb[2][4][2];  // [step parity][block][rA / rB]
    auto read_a = [&](int p, int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[p][i][0] = trd_off(ab[i][0], ks * 16 * kDwRowB);
        fa[p][i][1] = trd_off(ab[i][1], ks * 16 * kDwRowB);
      }
    };
    auto read_b = [&](int p, int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fb[p][i][0] = trd_off(bb[i][0], ks * 16 * kDwRowB);
        fb[p][i][1] = trd_off(bb[i][1], ks * 16 * kDwRowB);
      }
    };
    auto mma_rows = [&](int p, int i0) __attribute__((always_inline)) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = i0; i < i0 + 2; ++i) {
        const u16x8 a = u16x8{fa[p][i][0][0], fa[p][i][0][1], fa[p][i][0][2], fa[p][i][0][3],
                              fa[p][i][1][0], fa[p][i][1][1], fa[p][i][1][2], fa[p][i][1][3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const u16x8 b = u16x8{fb[p][j][0][0], fb[p][j][0][1], fb[p][j][0][2], fb[p][j][0][3],
                                fb[p][j][1][0], fb[p][j][1][1], fb[p][j][1][2], fb[p][j][1][3]};
          acc[i][j] = mfma32d(a, b, acc[i][j]);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    };
    read_a(0, 0);
    lds_wait_le(7);  // <= 15 LDS reads outstanding (4-bit lgkmcnt)
    read_b(0, 0);
    lds_wait();
#pragma unroll
    for (int ks = 0; ks < kDwBK / 16; ++ks) {
      const int p = ks & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pin(fa[p][i][0]);
        pin(fa[p][i][1]);
        pin(fb[p][i][0]);
        pin(fb[p][i][1]);
      }
      const bool nxt = ks + 1 < kDwBK / 16;
      if (nxt) read_a(p ^ 1, ks + 1);  // 8 reads in flight under the first half of the MFMAs
      mma_rows(p, 0);
      if (nxt) {
        lds_wait_le(0);  // A(ks + 1) landed (had 8 MFMAs of time): keeps <= 8 reads in flight
        read_b(p ^ 1, ks + 1);
      }
      mma_rows(p, 2);
      if (nxt) lds_wait_le(0);
    }
  }

  dw_epilogue<OUT_F32, BETA>(acc, C, ldc, m0, n0, wm, wn, hh, lane, alpha_f * (alpha_t ? alpha_t[0] : 1.f));
}


// Round-3 first form (verified on the MI355X, profiles/r3m): two 64-token stages, vmcnt(0) +
// __syncthreads() per stage.  Kept beside the ring form for same-process A/B (MXLLM_DW_GEMM).
constexpr int kD1BK = 64, kD1Stage = kD1BK * kDwRowB;  // 32 KiB per operand and stage

template <bool OUT_F32, bool BETA>
__global__ void __launch_bounds__(256, 1)
dw_gemm_dbuf_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
                    void* __restrict__ C, int64_t ldc, int M, int N, int T, const float* __restrict__ alpha_t,
                    float alpha_f) {
  __shared__ __attribute__((aligned(1024))) char smem[4 * kD1Stage];  // A0 | B0 | A1 | B1
  const int nM = M / kDwBM, nN = N / kDwBN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int pm, pn;
  {
    constexpr int GM = 4;
    const int per = GM * nN, grp = L / per, first = grp * GM;
    const int rows = min(GM, nM - first), in = L - grp * per;
    pm = first + in % rows;
    pn = in / rows;
  }
  const int m0 = pm * kDwBM, n0 = pn * kDwBN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  int aoff[8], boff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 2 * (8 * w + i) + (lane >> 5), pc = lane & 31;
    const int lc = dphys(pc, row);
    aoff[i] = row * (int)lda + 8 * lc;
    boff[i] = row * (int)ldb + 8 * lc;
  }
  const uint16_t* Ab = A + m0;
  const uint16_t* Bb = B + n0;
  auto issue = [&](int kt, int buf) __attribute__((always_inline)) {
    const uint16_t* a = Ab + (int64_t)kt * kD1BK * lda;
    const uint16_t* b = Bb + (int64_t)kt * kD1BK * ldb;
    char* da = smem + buf * 2 * kD1Stage;
    char* db = da + kD1Stage;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_global_load_lds((dgptr_t)(a + aoff[i]), (dlptr_t)(da + (8 * w + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((dgptr_t)(b + boff[i]), (dlptr_t)(db + (8 * w + i) * 1024), 16, 0, 0);
    }
  };
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3, hh = lane >> 5;
  const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t abase[4][2], bbase[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int la = wm * 16 + 4 * i + 2 * (g & 1) + (tp >> 1);
    const int lb = wn * 16 + 4 * i + 2 * (g & 1) + (tp >> 1);
    abase[i][0] = lds0 + rA * kDwRowB + 16 * dphys(la, rA) + 8 * (tp & 1);
    abase[i][1] = lds0 + rB * kDwRowB + 16 * dphys(la, rB) + 8 * (tp & 1);
    bbase[i][0] = lds0 + kD1Stage + rA * kDwRowB + 16 * dphys(lb, rA) + 8 * (tp & 1);
    bbase[i][1] = lds0 + kD1Stage + rB * kDwRowB + 16 * dphys(lb, rB) + 8 * (tp & 1);
  }
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = T / kD1BK;
  issue(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const uint32_t so = (uint32_t)cur * 2 * kD1Stage;
    uint32_t ab[4][2], bb[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ab[i][0] = abase[i][0] + so;
      ab[i][1] = abase[i][1] + so;
      bb[i][0] = bbase[i][0] + so;
      bb[i][1] = bbase[i][1] + so;
    }
    u16x4 fa[2][4][2], fb[2][4][2];
    auto read_a = [&](int p, int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[p][i][0] = trd_off(ab[i][0], ks * 16 * kDwRowB);
        fa[p][i][1] = trd_off(ab[i][1], ks * 16 * kDwRowB);
      }
    };
    auto read_b = [&](int p, int ks) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fb[p][i][0] = trd_off(bb[i][0], ks * 16 * kDwRowB);
        fb[p][i][1] = trd_off(bb[i][1], ks * 16 * kDwRowB);
      }
    };
    auto mma_rows = [&](int p, int i0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = i0; i < i0 + 2; ++i) {
        const u16x8 a = u16x8{fa[p][i][0][0], fa[p][i][0][1], fa[p][i][0][2], fa[p][i][0][3],
                              fa[p][i][1][0], fa[p][i][1][1], fa[p][i][1][2], fa[p][i][1][3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const u16x8 b = u16x8{fb[p][j][0][0], fb[p][j][0][1], fb[p][j][0][2], fb[p][j][0][3],
                                fb[p][j][1][0], fb[p][j][1][1], fb[p][j][1][2], fb[p][j][1][3]};
          acc[i][j] = mfma32d(a, b, acc[i][j]);
        }
      }
    };
    read_a(0, 0);
    lds_wait_le(7);
    read_b(0, 0);
    lds_wait();
#pragma unroll
    for (int ks = 0; ks < kD1BK / 16; ++ks) {
      const int p = ks & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pin(fa[p][i][0]);
        pin(fa[p][i][1]);
        pin(fb[p][i][0]);
        pin(fb[p][i][1]);
      }
      const bool nxt = ks + 1 < kD1BK / 16;
      if (nxt) read_a(p ^ 1, ks + 1);
      mma_rows(p, 0);
      if (nxt) {
        lds_wait_le(0);
        read_b(p ^ 1, ks + 1);
      }
      mma_rows(p, 2);
      if (nxt) lds_wait_le(0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
  }
  dw_epilogue<OUT_F32, BETA>(acc, C, ldc, m0, n0, wm, wn, hh, lane, alpha_f * (alpha_t ? alpha_t[0] : 1.f));
}


// 8-wave form (MXLLM_DW_GEMM=w8): 2 waves per SIMD (guide §5 template geometry), each wave
// 128 (m) x 64 (n) = 4 x 2 blocks (128 accumulators), the same 4-stage BK-32 ring as the 4-wave
// ring form; while one wave of a SIMD waits on its transposed reads the other issues MFMAs.
template <bool OUT_F32, bool BETA>
__global__ void __launch_bounds__(512, 1)
dw_gemm_w8_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
                  void* __restrict__ C, int64_t ldc, int M, int N, int T, const float* __restrict__ alpha_t,
                  float alpha_f) {
  __shared__ __attribute__((aligned(1024))) char smem[kDwNB * kDwStage];
  const int nM = M / kDwBM, nN = N / kDwBN;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  int pm, pn;
  {
    constexpr int GM = 4;
    const int per = GM * nN, grp = L / per, first = grp * GM;
    const int rows = min(GM, nM - first), in = L - grp * per;
    pm = first + in % rows;
    pn = in / rows;
  }
  const int m0 = pm * kDwBM, n0 = pn * kDwBN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  // per stage and operand 16 pieces; wave w stores pieces 2 w, 2 w + 1 of both (4 glds)
  int aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 2 * (2 * w + i) + (lane >> 5), pc = lane & 31;
    const int lc = dphys(pc, row);
    aoff[i] = row * (int)lda + 8 * lc;
    boff[i] = row * (int)ldb + 8 * lc;
  }
  const uint16_t* Ab = A + m0;
  const uint16_t* Bb = B + n0;
  auto issue = [&](int kt) __attribute__((always_inline)) {
    const uint16_t* a = Ab + (int64_t)kt * kDwBK * lda;
    const uint16_t* b = Bb + (int64_t)kt * kDwBK * ldb;
    char* da = smem + (kt % kDwNB) * kDwStage;
    char* db = da + kDwHalf;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_global_load_lds((dgptr_t)(a + aoff[i]), (dlptr_t)(da + (2 * w + i) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((dgptr_t)(b + boff[i]), (dlptr_t)(db + (2 * w + i) * 1024), 16, 0, 0);
    }
  };
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3, hh = lane >> 5;
  const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t abase[4][2], bbase[2][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int la = wm * 16 + 4 * i + 2 * (g & 1) + (tp >> 1);
    abase[i][0] = lds0 + rA * kDwRowB + 16 * dphys(la, rA) + 8 * (tp & 1);
    abase[i][1] = lds0 + rB * kDwRowB + 16 * dphys(la, rB) + 8 * (tp & 1);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int lb = wn * 8 + 4 * j + 2 * (g & 1) + (tp >> 1);
    bbase[j][0] = lds0 + kDwHalf + rA * kDwRowB + 16 * dphys(lb, rA) + 8 * (tp & 1);
    bbase[j][1] = lds0 + kDwHalf + rB * kDwRowB + 16 * dphys(lb, rB) + 8 * (tp & 1);
  }
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = T / kDwBK;
  issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk)
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2);
    const uint32_t so = (uint32_t)(kt % kDwNB) * kDwStage;
    uint32_t ab[4][2], bb[2][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ab[i][0] = abase[i][0] + so;
      ab[i][1] = abase[i][1] + so;
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bb[j][0] = bbase[j][0] + so;
      bb[j][1] = bbase[j][1] + so;
    }
    u16x4 fa[2][4][2], fb[2][2][2];
    auto read = [&](int p, int ks) __attribute__((always_inline)) {  // 12 reads (<= 15 outstanding)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        fb[p][j][0] = trd_off(bb[j][0], ks * 16 * kDwRowB);
        fb[p][j][1] = trd_off(bb[j][1], ks * 16 * kDwRowB);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        fa[p][i][0] = trd_off(ab[i][0], ks * 16 * kDwRowB);
        fa[p][i][1] = trd_off(ab[i][1], ks * 16 * kDwRowB);
      }
    };
    read(0, 0);
    lds_wait();
#pragma unroll
    for (int ks = 0; ks < kDwBK / 16; ++ks) {
      const int p = ks & 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pin(fa[p][i][0]);
        pin(fa[p][i][1]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        pin(fb[p][j][0]);
        pin(fb[p][j][1]);
      }
      const bool nxt = ks + 1 < kDwBK / 16;
      if (nxt) read(p ^ 1, ks + 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const u16x8 a = u16x8{fa[p][i][0][0], fa[p][i][0][1], fa[p][i][0][2], fa[p][i][0][3],
                              fa[p][i][1][0], fa[p][i][1][1], fa[p][i][1][2], fa[p][i][1][3]};
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const u16x8 b = u16x8{fb[p][j][0][0], fb[p][j][0][1], fb[p][j][0][2], fb[p][j][0][3],
                                fb[p][j][1][0], fb[p][j][1][1], fb[p][j][1][2], fb[p][j][1][3]};
          acc[i][j] = mfma32d(a, b, acc[i][j]);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (nxt) lds_wait();
    }
  }
  dw_epilogue<OUT_F32, BETA, 2>(acc, C, ldc, m0, n0, wm, wn, hh, lane, alpha_f * (alpha_t ? alpha_t[0] : 1.f));
}

}  // namespace mx

using namespace mx;

// Shapes the kernel takes: M, N multiples of 256, T a multiple of 64, 16-B aligned rows.  Returns
// -1 (nothing launched) otherwise; the caller then uses the transpose + hipBLASLt path.
extern "C" int mx_dw_gemm(const uint16_t* dy, int64_t lda, const uint16_t* x, int64_t ldb, void* out, int64_t ldc,
                          int out_f32, int M, int N, int T, float beta, const float* alpha_t, float alpha_f,
                          hipStream_t stream) {
  if (M <= 0 || N <= 0 || T <= 0 || M % kDwBM || N % kDwBN || T % kDwBK) return -1;
  if (lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N) return -1;
  if ((int64_t)63 * lda + M > (int64_t)1 << 31 || (int64_t)63 * ldb + N > (int64_t)1 << 31) return -1;
  if (((uintptr_t)dy | (uintptr_t)x) & 15) return -1;
  if (beta != 0.f && beta != 1.f) return -1;
  const int grid = (M / kDwBM) * (N / kDwBN);
  const bool acc = beta != 0.f;
  // MXLLM_DW_GEMM (read per call: same-process A/B): w8 (default, fastest: profiles/r3m) = 8 waves on
  // the 4-stage BK-32 ring; ring = 4 waves on that ring; dbuf = 4 waves, two BK-64 buffers
  const char* fe = getenv("MXLLM_DW_GEMM");
  const bool ring = fe && fe[0] == 'r', w8 = !(fe && (fe[0] == 'r' || fe[0] == 'd'));
  if (!ring && !w8 && T % kD1BK) return -1;
#define DW_LAUNCH(F, BT)                                                                                        \
  do {                                                                                                          \
    if (w8)                                                                                                     \
      dw_gemm_w8_kernel<F, BT><<<grid, 512, 0, stream>>>(dy, lda, x, ldb, out, ldc, M, N, T, alpha_t, alpha_f);  \
    else if (ring)                                                                                              \
      dw_gemm_kernel<F, BT><<<grid, 256, 0, stream>>>(dy, lda, x, ldb, out, ldc, M, N, T, alpha_t, alpha_f);     \
    else                                                                                                        \
      dw_gemm_dbuf_kernel<F, BT><<<grid, 256, 0, stream>>>(dy, lda, x, ldb, out, ldc, M, N, T, alpha_t, alpha_f); \
  } while (0)
  if (out_f32) {
    if (acc) DW_LAUNCH(true, true); else DW_LAUNCH(true, false);
  } else {
    if (acc) DW_LAUNCH(false, true); else DW_LAUNCH(false, false);
  }
#undef DW_LAUNCH
  return (int)hipGetLastError();
}
