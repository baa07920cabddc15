// Causal GQA flash-attention backward for gfx950 (SURVEY §2.4 K7 bwd).
//
// Recompute-P formulation (guide App. B "Attention backward"): per tile
//   S = Q K^T, P = exp2(S*sl - lse2), dP = dO V^T, dS = P (dP - delta),
//   dV^T += dO^T P, dK^T += Q^T dS, dQ += dS K   (x softmax scale for dQ, dK)
//
// Decomposition (sized for small-batch fine-tuning shapes, e.g. B=2, Hq=64,
// S=2048 -> 2048 workgroups instead of the 128 a per-KV-head split would give):
//  * workgroup = 4 waves = 128 keys of ONE q-head (32 keys per wave, key on the
//    MFMA lane); it sweeps all q tiles (64 rows) that can see its keys;
//  * K and V fragments of the wave's keys stay in registers (B operands of S
//    and dP); S/dP accumulators, converted to bf16, are directly the B
//    operands of dV^T and dK^T (no LDS round trip); dO^T / Q^T fragments via
//    ds_read_b64_tr_b16 from the same swizzled tile images used for row reads;
//  * dS crosses LDS once ([key][q] image), the workgroup then computes its
//    64 x D dQ contribution over all 128 keys with MFMA and adds it to an f32
//    dQ with no-return atomics (256-B row segments per wave instruction);
//    128 keys per workgroup -> 320 FLOP per atomic byte;
//  * dK/dV are per-q-head partials [B,Hq,Sk,D] f32; the GQA group sum is
//    fused into the inverse-RoPE merge kernel (rope.hip), so no atomics and a
//    deterministic dK/dV;
//  * heaviest key blocks (most visible q tiles) scheduled first.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8_b __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4_b;

__device__ __forceinline__ f32x16 mfma32b(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_b, a), __builtin_bit_cast(bf16x8_b, b),
                                                 c, 0, 0, 0);
}
__device__ __forceinline__ u16x4 trd(const char* p) {
  return __builtin_bit_cast(u16x4, __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_b*)(p)));
}
// (trd_asm / lds_wait / pin: common.h)
// 16-B chunk swizzle of the 128-B rows of a dS^T image ([key][64 q] bf16).  A
// half-wave's transposed read touches rows 4a..4a+3, four chunks each: row parity
// already splits the 64 banks, and bit 2 of the XOR (from row bit 1) moves rows
// 4a+2/4a+3 to the other half of the chunks -> conflict-free (swzb<8> left rows
// 4a and 4a+2 on the same banks: 2-way conflicts, a third of the dQ kernel's
// LDS cycles in SQ_LDS_BANK_CONFLICT).  Depends on row bits 1..3 only, so a
// 16-row step stays an immediate offset.
__device__ __forceinline__ int swz8b(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }

template <int CH>
__device__ __forceinline__ int swzb(int row) {
  return (((row & 3) << 2) | ((row >> 2) & 3)) & (CH - 1);
}

// delta[b,h,q] = sum_d dO[b,q,h,d] * O[b,q,h,d]   (token-major inputs)
// D/8 lanes per row, 16-B loads of both operands, shuffle-reduced (G13).
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(const uint16_t* __restrict__ dO,
                                                             const uint16_t* __restrict__ O,
                                                             float* __restrict__ delta, int B, int S, int Hq,
                                                             int64_t ldo) {
  constexpr int LPR = D / 8;  // lanes per row
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPR;  // over B*S*Hq (token-major order)
  const int sub = threadIdx.x % LPR;
  const bool valid = row < (int64_t)B * S * Hq;
  float s = 0.f;
  if (valid) {
    const u16x8 a = *reinterpret_cast<const u16x8*>(dO + row * D + sub * 8);
    const u16x8 c = *reinterpret_cast<const u16x8*>(O + (row / Hq) * ldo + (row % Hq) * D + sub * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += bf2f(a[j]) * bf2f(c[j]);
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (valid && sub == 0) {
    const int h = (int)(row % Hq);
    const int64_t t = row / Hq;
    const int b = (int)(t / S), q = (int)(t % S);
    delta[((int64_t)b * Hq + h) * S + q] = s;
  }
}

// DQM: dQ hand-off mode. 1 = f32 atomics into dQ [B,Hq,S_pad,D];
// 2 = deterministic: plain stores of this key block's dQ partial into
//     dQ + kb * B*Hq*S_pad*D, summed in key-block order by attn_bwd_dq_reduce;
// 3 = split (default): no dQ work here; dS^T is stored (bf16) to a [BH, S_pad/64, Sk_pad, 64]
//     buffer passed in place of dQ and attn_bwd_dq_kernel computes dQ = dS K per q block
//     (no atomics, deterministic, and the key-block kernel loses 1/5 of its MFMAs and
//     its dS LDS round trip);
// 0 = dropped (ablation timing only).
template <int D, bool CAUSAL, int DQM = 1>
__global__ void __launch_bounds__(256, 1)
attn_bwd_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                float* __restrict__ dQ, float* __restrict__ dKp, float* __restrict__ dVp, int B, int Hq, int Hkv,
                int S, int Sk, int off, float sl, float scale, int S_pad) {
  constexpr int BN = 128, BQ = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int KIMG = BN * ROWB;      // K image [128][D]
  constexpr int QT = BQ * ROWB;        // one Q tile / dO tile [64][D]
  constexpr int DSROWB = BQ * 2;       // dS image row: 64 q bf16 = 128 B
  constexpr int DSIMG = BN * DSROWB;   // [128 keys][64 q]
  constexpr int LPT_K = BN * CH / 256;
  constexpr int SEGS = QT / 1024;      // 1-KiB LDS-DMA segments per tile
  constexpr int NT = (2 * DB + 3) / 4; // dQ output tiles per wave
  // LDS: K image | 2 x (Q tile, dO tile, lse[64], delta[64]) | dS image  -- ONE array (guide §5 trap 4a)
  constexpr int BUF = 2 * QT + 2 * BQ * 4;
  __shared__ __attribute__((aligned(16))) char smem[KIMG + 2 * BUF + DSIMG];
  char* kimg = smem;
  char* dsi = smem + KIMG + 2 * BUF;
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;

  const int nkb = (Sk + BN - 1) / BN;
  const int BH = B * Hq;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BH, Hq / Hkv);
  const int kb = bid / BH;  // ascending: key block 0 sees the most q tiles (causal) -> heaviest first
  const int bh = bid % BH;
  if (kb >= nkb) return;
  const int b = bh / Hq, h = bh % Hq, hk = h / (Hq / Hkv);
  const uint16_t* Qp = Q + (size_t)(b * Hq + h) * S * D;
  const uint16_t* Kp = K + (size_t)(b * Hkv + hk) * Sk * D;
  const uint16_t* Vp = V + (size_t)(b * Hkv + hk) * Sk * D;
  const size_t dstride = (size_t)Hq * D;  // token-major row stride of dO
  const uint16_t* dOp = dO + (size_t)b * S * dstride + (size_t)h * D;
  const float* lsep = LSE + (size_t)(b * Hq + h) * S;
  const float* delp = DELTA + (size_t)(b * Hq + h) * S;
  // rows padded to S_pad: the tail tile's atomics / stores need no guard
  float* dQp = dQ + (DQM == 2 ? (size_t)kb * BH * S_pad * D : 0) + (size_t)(b * Hq + h) * S_pad * D;
  // DQM 3: dS^T of this q head, blocked by 64-q tiles: [S_pad/64][Sk_pad keys][64 q] bf16,
  // so one (64-q tile, key range) piece is contiguous for both the writer and the reader
  uint16_t* dstp = reinterpret_cast<uint16_t*>(dQ) + (size_t)(b * Hq + h) * (nkb * BN) * S_pad;

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int k0 = kb * BN;
  const int key = k0 + 32 * w + r;  // this lane's key
  const int kld = min(key, Sk - 1);

  // K image (whole WG) + per-wave K/V fragments (clamped rows; masked later)
  if constexpr (DQM != 3) {  // the split mode computes dQ in attn_bwd_dq_kernel: no K image here
#pragma unroll
    for (int i = 0; i < LPT_K; ++i) {
      const int c = tid + 256 * i, row = c / CH, ch = c % CH, kk = min(k0 + row, Sk - 1);
      *reinterpret_cast<u16x8*>(kimg + row * ROWB + 16 * (ch ^ swzb<CH>(row))) =
          *reinterpret_cast<const u16x8*>(Kp + (size_t)kk * D + ch * 8);
    }
  }
  u16x8 kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    kf[s] = *reinterpret_cast<const u16x8*>(Kp + (size_t)kld * D + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const u16x8*>(Vp + (size_t)kld * D + 16 * s + 8 * hh);
  }
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[d][j] = 0.f; dv[d][j] = 0.f; }

  int qstart = 0;
  if (CAUSAL) qstart = max(0, (k0 - off) / BQ * BQ);
  const int nqt = qstart < S ? (S - qstart + BQ - 1) / BQ : 0;

  // LDS-DMA of q tile `it` into buffer `buf`: Q / dO rows (swizzle via source
  // chunk permutation), lse / delta by wave 0 (4 B per lane).
  // Q / dO rows by range-checked buffer_load ... lds: per-lane source offsets are loop-invariant
  // (one VALU add per piece for the tile step), rows past S read as zeros (masked: p = 0)
  const int orec = (int)(((size_t)(S - 1) * dstride + D) * 2);
  static_assert(SEGS / 4 <= 4, "at most 4 pieces per wave");
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  i32x4_t qoff = {0, 0, 0, 0}, ooff = {0, 0, 0, 0};  // (a vector: a captured int array drops the host stub)
#pragma unroll
  for (int i = 0; i < SEGS / 4; ++i) {
    const int seg = w * (SEGS / 4) + i;
    const int byte = seg * 1024 + lane * 16;
    const int row = byte / ROWB, slot = (byte % ROWB) / 16;
    const int ch = slot ^ swzb<CH>(row);
    qoff[i] = row * ROWB + ch * 16;
    ooff[i] = (int)(row * dstride * 2) + ch * 16;
  }
  auto glds = [&](int it, int buf) {
    char* qt = smem + KIMG + buf * BUF;
    char* dot = qt + QT;
    char* ld = dot + QT;
    const int q0 = qstart + it * BQ;
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc((void*)Qp, 0, S * ROWB, 0x00020000);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc((void*)dOp, 0, orec, 0x00020000);
#pragma unroll
    for (int i = 0; i < SEGS / 4; ++i) {
      const int seg = w * (SEGS / 4) + i;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lptr_t)(qt + seg * 1024), 16, qoff[i] + q0 * ROWB, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ors, (lptr_t)(dot + seg * 1024), 16,
                                               ooff[i] + (int)(q0 * dstride * 2), 0, 0, 0);
    }
    if (w == 0) {
      const int q = min(q0 + lane, S - 1);
      __builtin_amdgcn_global_load_lds((gptr_t)(lsep + q), (lptr_t)(ld), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((gptr_t)(delp + q), (lptr_t)(ld + BQ * 4), 4, 0, 0);
    }
  };

  f32x16 pend[NT];  // dQ tile of the previous iteration, added after the next barrier
  int pend_q0 = -1;
  // dQ hand-off through a buffer descriptor: the per-lane part of the address is
  // loop-invariant (voff), the tile / row-group part is wave-uniform (soffset,
  // SALU) and the row-in-group part an immediate -> no VALU address math per atomic
  const __amdgpu_buffer_rsrc_t dq_rsrc = __builtin_amdgcn_make_buffer_rsrc(dQp, 0, 0x7fffffff, 0x00020000);
  const int dq_voff = ((4 * hh) * D + r) * 4;
  auto flush_dq = [&]() {
    if (DQM == 0 || pend_q0 < 0) return;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tile = w + 4 * t;
      if (tile < 2 * DB) {
        const int m = tile / DB, db = tile % DB;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          // q = pend_q0 + 32m + (j&3) + 8(j>>2) + 4hh ; column db*32 + r
          const int soff = ((pend_q0 + 32 * m + 8 * (j >> 2)) * D + db * 32) * 4;
          const int ioff = (j & 3) * D * 4;
          if constexpr (DQM == 2)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pend[t][j]), dq_rsrc,
                                                      dq_voff + ioff, soff, 0);
          else
            __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(pend[t][j], dq_rsrc, dq_voff + ioff, soff, 0);
        }
      }
    }
  };

  // DQM 3: this wave's dS^T (32 keys x 64 q, bf16) of the previous q tile, stored after
  // the next barrier so the stores drain during a whole tile of compute
  u16x4 dsv[2][4];
  int ds_q0 = -1;
  auto flush_ds = [&]() {
    if constexpr (DQM == 3) {
      if (ds_q0 < 0) return;
      uint16_t* rowp = dstp + ((size_t)(ds_q0 / BQ) * (nkb * BN) + (k0 + 32 * w + r)) * BQ;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<u16x4*>(rowp + 32 * m + 8 * gq + 4 * hh) = dsv[m][gq];
    }
  };

  if (nqt > 0) glds(0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): prologue loads retired (visible to the waitcnt pass)
  __syncthreads();
  for (int it = 0; it < nqt; ++it) {
    const int q0 = qstart + it * BQ;
    const int buf = it & 1;
    const char* qt = smem + KIMG + buf * BUF;
    const char* dot = qt + QT;
    const float* lse_s = reinterpret_cast<const float*>(dot + QT);
    const float* del_s = lse_s + BQ;
    if (it + 1 < nqt) glds(it + 1, buf ^ 1);  // prefetch next tile (its buffer was last read before the barrier)
    flush_dq();                              // previous tile's dQ atomics overlap this tile's MFMAs
    flush_ds();
    const bool need_mask = (q0 + BQ > S) || (k0 + BN > Sk) || (CAUSAL && (k0 + 32 * w + 31 > q0 + off));
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      f32x16 sa, dp;
#pragma unroll
      for (int j = 0; j < 16; ++j) { sa[j] = 0.f; dp[j] = 0.f; }
      const int qr = 32 * m + r;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int o = qr * ROWB + 16 * ((2 * s + hh) ^ swzb<CH>(qr));
        sa = mfma32b(*reinterpret_cast<const u16x8*>(qt + o), kf[s], sa);
        dp = mfma32b(*reinterpret_cast<const u16x8*>(dot + o), vf[s], dp);
      }
      // rows of sa/dp: q = q0 + 32m + (j&3) + 8(j>>2) + 4hh ; column = key (lane)
      f32x4 lv[4], dl[4];
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        lv[gq] = *reinterpret_cast<const f32x4*>(lse_s + 32 * m + 8 * gq + 4 * hh);
        dl[gq] = *reinterpret_cast<const f32x4*>(del_s + 32 * m + 8 * gq + 4 * hh);
      }
      if (need_mask) {  // wave-uniform; branch-free selects
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int q = q0 + 32 * m + (j & 3) + 8 * (j >> 2) + 4 * hh;
          const bool dead = (key >= Sk) | (q >= S) | (CAUSAL & (key > q + off));
          const float p = dead ? 0.f : __builtin_amdgcn_exp2f(sa[j] * sl - lv[j >> 2][j & 3]);
          sa[j] = p;
          dp[j] = p * (dp[j] - dl[j >> 2][j & 3]);  // dS
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float p = __builtin_amdgcn_exp2f(sa[j] * sl - lv[j >> 2][j & 3]);
          sa[j] = p;
          dp[j] = p * (dp[j] - dl[j >> 2][j & 3]);
        }
      }
      // dV^T += dO^T P ; dK^T += Q^T dS   (k index = q rows of this m-subtile)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = f2bf(sa[8 * s2 + j]);
          sb[j] = f2bf(dp[8 * s2 + j]);
        }
        const int rb = 32 * m + 16 * s2 + 4 * hh;
        const int rowA = rb + tq, rowB = rb + 8 + tq;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          const int chunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
          const int oA = rowA * ROWB + 16 * (chunk ^ swzb<CH>(rowA)) + 8 * (tp & 1);
          const int oB = rowB * ROWB + 16 * (chunk ^ swzb<CH>(rowB)) + 8 * (tp & 1);
          const u16x4 a0 = trd(dot + oA), a1 = trd(dot + oB);
          dv[db] = mfma32b(u16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]}, pb, dv[db]);
          const u16x4 b0 = trd(qt + oA), b1 = trd(qt + oB);
          dk[db] = mfma32b(u16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]}, sb, dk[db]);
        }
      }
      // dS -> LDS image [key][q] (bf16): 4 consecutive q per 8-byte write
      const int krow = 32 * w + r;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int q = 32 * m + 8 * gq + 4 * hh;  // local q, multiple of 4
        const int chunk = q >> 3;
        u16x4 v4 = u16x4{f2bf(dp[4 * gq]), f2bf(dp[4 * gq + 1]), f2bf(dp[4 * gq + 2]), f2bf(dp[4 * gq + 3])};
        if constexpr (DQM == 3)
          dsv[m][gq] = v4;
        else
          *reinterpret_cast<u16x4*>(dsi + krow * DSROWB + 16 * (chunk ^ swz8b(krow)) + 8 * hh) = v4;
      }
    }
    if constexpr (DQM == 3) {
      ds_q0 = q0;
      __syncthreads();  // this tile's Q/dO buffer consumed; next tile's DMA landed
      continue;
    }
    __syncthreads();  // dS image complete (also retires the DMA + atomics issued above)
    // dQ[q0 .. q0+63][:] = scale * dS[64 x 128] . K[128 x D]  -> kept in `pend`, added next iteration
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tile = w + 4 * t;
      if (tile < 2 * DB) {
        const int m = tile / DB, db = tile % DB;
        f32x16 acc;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 0.f;
#pragma unroll
        for (int s = 0; s < BN / 16; ++s) {
          const int kbse = 16 * s + 4 * hh;
          const int rA = kbse + tq, rB = kbse + 8 + tq;
          const int qchunk = (32 * m + 16 * (g & 1) + 4 * tp) >> 3;
          const u16x4 a0 = trd(dsi + rA * DSROWB + 16 * (qchunk ^ swz8b(rA)) + 8 * (tp & 1));
          const u16x4 a1 = trd(dsi + rB * DSROWB + 16 * (qchunk ^ swz8b(rB)) + 8 * (tp & 1));
          const int dchunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
          const u16x4 b0 = trd(kimg + rA * ROWB + 16 * (dchunk ^ swzb<CH>(rA)) + 8 * (tp & 1));
          const u16x4 b1 = trd(kimg + rB * ROWB + 16 * (dchunk ^ swzb<CH>(rB)) + 8 * (tp & 1));
          acc = mfma32b(u16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]},
                        u16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]}, acc);
        }
        pend[t] = acc * scale;
        if constexpr (DQM == 0) asm volatile("" ::"v"(pend[t][0]));
      }
    }
    pend_q0 = q0;
    __syncthreads();  // dS image consumed; next tile's DMA landed
  }
  flush_dq();
  flush_ds();
  // write per-q-head dK/dV partials: C rows = d, col = key (lane)
  if (key < Sk) {
    float* dkq = dKp + ((size_t)(b * Hq + h) * Sk + key) * D;
    float* dvq = dVp + ((size_t)(b * Hq + h) * Sk + key) * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = db * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(dkq + d) =
            f32x4{dk[db][4 * gq] * scale, dk[db][4 * gq + 1] * scale, dk[db][4 * gq + 2] * scale,
                  dk[db][4 * gq + 3] * scale};
        *reinterpret_cast<f32x4*>(dvq + d) = f32x4{dv[db][4 * gq], dv[db][4 * gq + 1], dv[db][4 * gq + 2],
                                                  dv[db][4 * gq + 3]};
      }
  }
}

// Split-mode (3) key-block kernel at TWO waves per SIMD (D = 128; MXLLM_ATTN_BWD8=0 selects the
// kernel above).  Workgroup = 8 waves = 128 keys of one q head, as above, but wave (kg = w & 3,
// m = w >> 2) owns 32 keys x the 32-row half m of every 64-row q tile: S, dP, P, dS and the dV / dK
// products of one half per wave, so each wave carries half the q work and its K / V fragments come
// from LDS images of the key block instead of registers — the register file then holds two
// waves per SIMD (the hardware interleaves one wave's softmax VALU with the other's MFMAs, which
// the one-wave kernel cannot).  The two halves' dK / dV partials are summed through LDS at the end.
template <bool CAUSAL, bool PROF = false>
__global__ void __launch_bounds__(512, 1)
attn_bwd8_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                 const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                 uint16_t* __restrict__ dST, float* __restrict__ dKp, float* __restrict__ dVp, int B, int Hq,
                 int Hkv, int S, int Sk, int off, float sl, float scale, int S_pad, int prio, int hpw,
                 uint32_t* __restrict__ prof = nullptr) {
  constexpr int D = 128, BN = 128, BQ = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int KIMG = BN * ROWB;     // K (or V) image [128][D]
  constexpr int QT = BQ * ROWB;       // Q / dO tile [64][D]
  constexpr int BUF = 2 * QT + 2 * BQ * 4;
  constexpr int SEGS = QT / 1024;     // 16 pieces per tile, 2 per wave
  constexpr int LDSB = 2 * KIMG + 2 * BUF;
  static_assert(LDSB >= 4 * 2 * DB * 16 * 64 * 4, "dK/dV pair reduction reuses the tile LDS");
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];  // (XOR addressing: 256-B aligned bases)
  char* kimg = smem;
  char* vimg = smem + KIMG;
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;

  uint64_t t_entry = 0;
  if constexpr (PROF) t_entry = __builtin_amdgcn_s_memtime();
  const int nkb = (Sk + BN - 1) / BN;
  // a workgroup = one key block x `hpw` q-heads of one KV group, looped over in turn: the K / V
  // images load once and dK / dV accumulate over the heads in registers; it writes partial
  // b * (Hq / hpw) + hp of dKp / dVp (the merge kernel sums the Hq / hpw / Hkv partials per KV head)
  const int HP = Hq / hpw;  // partials per batch row
  const int BHP = B * HP;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BHP, (Hq / Hkv) / hpw);
  const int kb = bid / BHP;
  const int bhp = bid % BHP;
  if (kb >= nkb) return;
  const int b = bhp / HP, hp = bhp % HP, h0 = hp * hpw, hk = h0 / (Hq / Hkv);
  const uint16_t* Kp = K + (size_t)(b * Hkv + hk) * Sk * D;
  const uint16_t* Vp = V + (size_t)(b * Hkv + hk) * Sk * D;
  const size_t dstride = (size_t)Hq * D;
  auto Qp = [&](int h) { return Q + (size_t)(b * Hq + h) * S * D; };
  auto dOp = [&](int h) { return dO + (size_t)b * S * dstride + (size_t)h * D; };
  auto lsep = [&](int h) { return LSE + (size_t)(b * Hq + h) * S; };
  auto delp = [&](int h) { return DELTA + (size_t)(b * Hq + h) * S; };
  auto dstp = [&](int h) { return dST + (size_t)(b * Hq + h) * (nkb * BN) * S_pad; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = w & 3, m = w >> 2;
  const int r = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int k0 = kb * BN;
  const int key = k0 + 32 * kg + r;

  // K / V images of the key block (rows past Sk read as zeros: masked)
  {
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)Kp, 0, Sk * ROWB, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)Vp, 0, Sk * ROWB, 0x00020000);
#pragma unroll
    for (int i = 0; i < KIMG / 1024 / 8; ++i) {
      const int seg = w * (KIMG / 1024 / 8) + i;
      const int row = seg * (1024 / ROWB) + lane / (ROWB / 16), slot = lane % (ROWB / 16);
      const int vo = (k0 + row) * ROWB + 16 * (slot ^ swzb<CH>(row));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(kimg + seg * 1024), 16, vo, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(vimg + seg * 1024), 16, vo, 0, 0, 0);
    }
  }
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[d][j] = 0.f; dv[d][j] = 0.f; }

  int qstart = 0;
  if (CAUSAL) qstart = max(0, (k0 - off) / BQ * BQ);
  const int nqt = qstart < S ? (S - qstart + BQ - 1) / BQ : 0;
  const int nit = nqt * hpw;  // flattened (head, q tile) iterations

  // Q / dO tile pieces: 2 per wave (one Q, one dO), range-checked buffer loads
  const int orec = (int)(((size_t)(S - 1) * dstride + D) * 2);
  const int pseg = w * (SEGS / 8);
  static_assert(SEGS / 8 == 2, "two pieces per wave");
  typedef int i32x2_t __attribute__((ext_vector_type(2)));
  i32x2_t qoff = {0, 0}, ooff = {0, 0};  // (a vector: a captured int array drops the host stub)
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // the swizzle depends on the row: each piece has its own offsets
    const int prow = (pseg + i) * (1024 / ROWB) + lane / (ROWB / 16), pslot = lane % (ROWB / 16);
    const int pch = pslot ^ swzb<CH>(prow);
    qoff[i] = prow * ROWB + pch * 16;
    ooff[i] = (int)(prow * dstride * 2) + pch * 16;
  }
  // piece k of the DMA of q tile `it` into buffer `buf`: 0..3 = Q / dO rows, 4 = lse + delta
  // (wave 0); glds = all of them
  // (hj, it): head h0 + hj, q tile it
  auto glds_piece = [&](int hj, int it, int buf, int k) {
    char* qt = smem + 2 * KIMG + buf * BUF;
    char* dot = qt + QT;
    char* ld = dot + QT;
    const int h = h0 + hj;
    const int q0 = (prio & 2) ? qstart : qstart + it * BQ;  // (prio & 2: timing ablation, same tile)
    if (k < 4) {
      const int i = k >> 1;
      if ((k & 1) == 0) {
        const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc((void*)Qp(h), 0, S * ROWB, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lptr_t)(qt + (pseg + i) * 1024), 16, qoff[i] + q0 * ROWB, 0,
                                                 0, 0);
      } else {
        const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc((void*)dOp(h), 0, orec, 0x00020000);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ors, (lptr_t)(dot + (pseg + i) * 1024), 16,
                                                 ooff[i] + (int)(q0 * dstride * 2), 0, 0, 0);
      }
    } else if (w == 0) {
      const int q = min(q0 + lane, S - 1);
      __builtin_amdgcn_global_load_lds((gptr_t)(lsep(h) + q), (lptr_t)(ld), 4, 0, 0);
      __builtin_amdgcn_global_load_lds((gptr_t)(delp(h) + q), (lptr_t)(ld + BQ * 4), 4, 0, 0);
    }
  };
  auto glds = [&](int hj, int it, int buf) {
#pragma unroll
    for (int k = 0; k < 5; ++k) glds_piece(hj, it, buf, k);
  };

  u16x4 dsv[4];
  int ds_q0 = -1, ds_h = h0;
  auto flush_ds_piece = [&](int gq) {
    if (ds_q0 < 0) return;
    uint16_t* rowp = dstp(ds_h) + ((size_t)(ds_q0 / BQ) * (nkb * BN) + key) * BQ + 32 * m;
    *reinterpret_cast<u16x4*>(rowp + 8 * gq + 4 * hh) = dsv[gq];
  };
  auto flush_ds = [&]() {
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) flush_ds_piece(gq);
  };

  // transposed-read lane offsets into a q tile (rows 32m + 4hh + tq (+8); chunk of d-block db);
  // the 16-row step s2 and the dO tile are immediates, the buffer a per-tile add
  // Every address below is (lane base) ^ (step bits): the swizzle XOR only touches byte bits
  // 4..7 of a 256-B row, row and buffer bases are multiples of 256, so the d-block (bits 6-7)
  // and the 32-B k step (bits 5-7) apply as one v_xor instead of one offset register each.
  const uint32_t tile_base = lds_addr(smem + 2 * KIMG);
  static_assert(ROWB == 256 && (BUF % 256) == 0 && (KIMG % 256) == 0, "XOR addressing assumes 256-B rows");
  uint32_t trA, trB;  // transposed reads of a q tile: rows 32m + 4hh + tq (+8), d-block 0
  {
    const int rowA = 32 * m + 4 * hh + tq, rowB = rowA + 8;
    const int chunk = (16 * (g & 1) + 4 * tp) >> 3;
    trA = rowA * ROWB + 16 * (chunk ^ swzb<CH>(rowA)) + 8 * (tp & 1);
    trB = rowB * ROWB + 16 * (chunk ^ swzb<CH>(rowB)) + 8 * (tp & 1);
  }
  // S / dP operand rows: q row 32m + r of the tile and key row 32kg + r of the K image share
  // row & 15, hence the swizzle: k step s reads chunk (2s + hh) ^ swz at base ^ (32 s)
  const int swz = swzb<CH>(r);
  const uint32_t qrowb = (32 * m + r) * ROWB + 16 * (hh ^ swz);
  const uint32_t krowb = lds_addr(kimg) + (32 * kg + r) * ROWB + 16 * (hh ^ swz);
  if ((prio & 1) && m == 1) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half (waves 4-7)
  if (nit > 0) glds(0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  // PROF: per-wave cycle sums of the loop phases (s_memtime at phase boundaries; diagnostic
  // build only, MXLLM_ATTN_PROF=1): issue, S/dP MFMAs issued, softmax done, dV/dK issued, barrier
  uint32_t ph[5] = {0, 0, 0, 0, 0};
  uint64_t tp0 = 0;
  auto mark = [&](int k) {
    if constexpr (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph[k] += (uint32_t)(t - tp0);
      tp0 = t;
    }
  };
  uint64_t t_beg = 0, rt_beg = 0;
  if constexpr (PROF) {
    t_beg = __builtin_amdgcn_s_memtime();
    rt_beg = __builtin_amdgcn_s_memrealtime();
  }
  int hj = 0, it = 0;  // head / q tile of flattened iteration L
  for (int L = 0; L < nit; ++L) {
    if constexpr (PROF) tp0 = __builtin_amdgcn_s_memtime();
    const int q0 = qstart + it * BQ;
    const int buf = L & 1;
    const int nx_it = it + 1 < nqt ? it + 1 : 0, nx_hj = it + 1 < nqt ? hj : hj + 1;  // next iteration
    const char* qt = smem + 2 * KIMG + buf * BUF;
    const char* dot = qt + QT;
    const float* lse_s = reinterpret_cast<const float*>(dot + QT);
    const float* del_s = lse_s + BQ;
    // spread (prio & 16, default): the next tile's DMA pieces go out one per S/dP k step and the
    // previous tile's dS stores one per dV/dK step -- issued in one burst at the loop top, the 8
    // waves' vector-memory instructions queued behind each other and the low-priority half
    // stalled there ~2000 cycles per tile (phase profile, archive/profiles/r2z_bwd8_phase_cycles.txt)
    const bool spread = (prio & 16) != 0;
    const bool more = L + 1 < nit;
    if (!spread) {
      if (more) glds(nx_hj, nx_it, buf ^ 1);
      flush_ds();
    } else if (prio & 64) {
      flush_ds();
    }
    mark(0);
    const bool need_mask = (q0 + BQ > S) || (k0 + BN > Sk) || (CAUSAL && (k0 + 32 * kg + 31 > q0 + 32 * m + off));
    f32x16 sa, dp;
#pragma unroll
    for (int j = 0; j < 16; ++j) { sa[j] = 0.f; dp[j] = 0.f; }
    {  // S = Q K^T, dP = dO V^T: asm row reads one k step ahead of their MFMAs (counted waits)
      const uint32_t qb = tile_base + buf * BUF + qrowb, kb2 = krowb;
      u16x8 f[2][4];
      auto ld = [&](int st, u16x8 (&x)[4]) {
        const uint32_t qa = qb ^ (uint32_t)(32 * st), ka = kb2 ^ (uint32_t)(32 * st);
        x[0] = rd128_off(qa, 0);
        x[1] = rd128_off(ka, 0);
        x[2] = rd128_off(qa, QT);
        x[3] = rd128_off(ka, KIMG);
      };
      ld(0, f[0]);
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st + 1 < KS) ld(st + 1, f[(st + 1) & 1]);
        lds_wait_le(st + 1 < KS ? 4 : 0);
        u16x8(&x)[4] = f[st & 1];
#pragma unroll
        for (int y = 0; y < 4; ++y) pin(x[y]);
        sa = mfma32b(x[0], x[1], sa);
        dp = mfma32b(x[2], x[3], dp);
        if (spread && (st & 1) == 0 && more) glds_piece(nx_hj, nx_it, buf ^ 1, st >> 1);
        if (spread && st == KS - 1 && more) glds_piece(nx_hj, nx_it, buf ^ 1, 4);
        // pin the DMA issue order: the counted end-of-tile wait assumes every DMA piece
        // precedes the 4 dS^T stores; no instruction is scheduled across this point
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    mark(1);
    // rows of sa/dp: q = q0 + 32m + (j&3) + 8(j>>2) + 4hh ; column = key (lane)
    if (need_mask) {  // wave-uniform: two straight-line bodies, branch-free selects
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(lse_s + 32 * m + 8 * gq + 4 * hh);
        const f32x4 dl = *reinterpret_cast<const f32x4*>(del_s + 32 * m + 8 * gq + 4 * hh);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int j = 4 * gq + jj;
          const int q = q0 + 32 * m + jj + 8 * gq + 4 * hh;
          const bool dead = (key >= Sk) | (q >= S) | (CAUSAL & (key > q + off));
          const float p = dead ? 0.f : __builtin_amdgcn_exp2f(sa[j] * sl - lv[jj]);
          sa[j] = p;
          dp[j] = p * (dp[j] - dl[jj]);
        }
      }
    } else {
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(lse_s + 32 * m + 8 * gq + 4 * hh);
        const f32x4 dl = *reinterpret_cast<const f32x4*>(del_s + 32 * m + 8 * gq + 4 * hh);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int j = 4 * gq + jj;
          const float p = __builtin_amdgcn_exp2f(sa[j] * sl - lv[jj]);
          sa[j] = p;
          dp[j] = p * (dp[j] - dl[jj]);
        }
      }
    }
    // dV^T += dO^T P ; dK^T += Q^T dS   (k index = the 32 q rows of this half).  The transposed
    // reads are asm (trd_off) with counted lgkmcnt waits: as builtins, hipcc's waitcnt pass
    // drains the next tile's LDS-DMA (vmcnt(0)) before the first of them
    u16x8 pb[2], sb[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pb[s2][j] = f2bf(sa[8 * s2 + j]);
        sb[s2][j] = f2bf(dp[8 * s2 + j]);
      }
    if constexpr (PROF) asm volatile("" ::"v"(pb[1]), "v"(sb[1]));
    mark(2);
    const uint32_t tbase = tile_base + buf * BUF;
    const uint32_t ta = tbase + trA, tb = tbase + trB;
    u16x4 tr[2][4];
    auto issue = [&](int i, u16x4 (&t)[4]) {
      const int s2 = i / DB, db = i % DB;
      const uint32_t a = ta ^ (uint32_t)(64 * db), bb = tb ^ (uint32_t)(64 * db);
      t[0] = trd_off(a, s2 * 16 * ROWB + QT);  // dO^T rows (A operand of dV)
      t[1] = trd_off(bb, s2 * 16 * ROWB + QT);
      t[2] = trd_off(a, s2 * 16 * ROWB);       // Q^T rows (A operand of dK)
      t[3] = trd_off(bb, s2 * 16 * ROWB);
    };
    // the dV/dK steps below store the previous tile's dS^T (4 pieces) after this tile's DMA went
    // out: those stores are then this wave's youngest vector-memory operations
    const bool ds_young = spread && (prio & 64) == 0 && ds_q0 >= 0;
    issue(0, tr[0]);
#pragma unroll
    for (int i = 0; i < 2 * DB; ++i) {
      if (i + 1 < 2 * DB) issue(i + 1, tr[(i + 1) & 1]);
      lds_wait_le(i + 1 < 2 * DB ? 4 : 0);
      u16x4(&t)[4] = tr[i & 1];
#pragma unroll
      for (int x = 0; x < 4; ++x) pin(t[x]);
      const int s2 = i / DB, db = i % DB;
      dv[db] = mfma32b(u16x8{t[0][0], t[0][1], t[0][2], t[0][3], t[1][0], t[1][1], t[1][2], t[1][3]}, pb[s2], dv[db]);
      dk[db] = mfma32b(u16x8{t[2][0], t[2][1], t[2][2], t[2][3], t[3][0], t[3][1], t[3][2], t[3][3]}, sb[s2], dk[db]);
      // dS stores here, not among the S/dP steps: next to the in-flight LDS-DMA they stalled
      // issue (B16 5.13 -> 6.09 ms); (prio & 64: at the loop top instead, A/B)
      if (spread && (i & 1) == 0 && (prio & 64) == 0) flush_ds_piece(i >> 1);
      __builtin_amdgcn_sched_barrier(0);  // the dS^T stores stay after the DMA and in this order
    }
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
      dsv[gq] = u16x4{f2bf(dp[4 * gq]), f2bf(dp[4 * gq + 1]), f2bf(dp[4 * gq + 2]), f2bf(dp[4 * gq + 3])};
    ds_q0 = q0;
    ds_h = h0 + hj;
    mark(3);
    // this wave's DMA for the next tile landed.  prio & 256: counted wait -- vmcnt(4) leaves the 4
    // dS^T stores (issued after the DMA; loads, stores and LDS-DMA retire in issue order) in flight
    // across the barrier instead of waiting for their completion
    static_assert(2 * DB == 8, "4 dS store pieces per tile (D = 128)");
#ifdef MXLLM_ATTN_BWD_NO_COUNTED_WAIT
    constexpr bool kCounted = false;  // build fallback: mxllm/_build.py found the ISA invariant broken
#else
    constexpr bool kCounted = true;
#endif
    if (kCounted && (prio & 256) && ds_young) {
      // raw barrier: __syncthreads()'s fence would wait for the stores (vmcnt(0)) after all; the
      // LDS reads of this tile are retired (lgkmcnt(0)), the DMA by the counted wait
      __builtin_amdgcn_s_waitcnt(0x0074);  // vmcnt(4) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();        // ... every wave's; this tile's buffers consumed
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      __syncthreads();                     // ... and every wave's; this tile's buffers consumed
    }
    mark(4);
    it = nx_it;
    hj = nx_hj;
  }
  if constexpr (PROF) {
    if (lane < 5) {
      uint32_t v = ph[0];
#pragma unroll
      for (int k = 1; k < 5; ++k) v = lane == k ? ph[k] : v;
      prof[((size_t)blockIdx.x * 8 + w) * 16 + lane] = v;
    }
    if (lane == 5) prof[((size_t)blockIdx.x * 8 + w) * 16 + 5] = (uint32_t)nit;
    const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memtime() - t_beg);
    const uint32_t drt = (uint32_t)(__builtin_amdgcn_s_memrealtime() - rt_beg);
    if (lane == 6) prof[((size_t)blockIdx.x * 8 + w) * 16 + 6] = dt;
    if (lane == 7) prof[((size_t)blockIdx.x * 8 + w) * 16 + 7] = drt;
    if (lane == 8) prof[((size_t)blockIdx.x * 8 + w) * 16 + 8] = (uint32_t)(t_beg - t_entry);
  }
  flush_ds();
  // sum the two halves' partials: m = 1 waves park theirs in LDS ([kg][value][lane], conflict-free)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem) + (size_t)kg * (2 * DB * 16) * 64 + lane;
  if (m == 1) {
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        red[((db * 16) + j) * 64] = dk[db][j];
        red[((DB * 16) + db * 16 + j) * 64] = dv[db][j];
      }
  }
  __syncthreads();
  if (m == 0 && key < Sk) {
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        dk[db][j] += red[((db * 16) + j) * 64];
        dv[db][j] += red[((DB * 16) + db * 16 + j) * 64];
      }
    float* dkq = dKp + ((size_t)bhp * Sk + key) * D;
    float* dvq = dVp + ((size_t)bhp * Sk + key) * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = db * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(dkq + d) =
            f32x4{dk[db][4 * gq] * scale, dk[db][4 * gq + 1] * scale, dk[db][4 * gq + 2] * scale,
                  dk[db][4 * gq + 3] * scale};
        *reinterpret_cast<f32x4*>(dvq + d) = f32x4{dv[db][4 * gq], dv[db][4 * gq + 1], dv[db][4 * gq + 2],
                                                  dv[db][4 * gq + 3]};
      }
  }
  if constexpr (PROF) {
    const uint64_t t_end = __builtin_amdgcn_s_memtime();
    if (lane == 9) prof[((size_t)blockIdx.x * 8 + w) * 16 + 9] = (uint32_t)(t_end - t_beg);
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n in [0, 15] (immediate per case; inline asm is
// invisible to hipcc's waitcnt pass)
__device__ __forceinline__ void vm_wait_le(int n) {
  switch (n) {
#define MX_VMC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    MX_VMC(1) MX_VMC(2) MX_VMC(3) MX_VMC(4) MX_VMC(5) MX_VMC(6) MX_VMC(7) MX_VMC(8)
    MX_VMC(9) MX_VMC(10) MX_VMC(11) MX_VMC(12) MX_VMC(13) MX_VMC(14) MX_VMC(15)
#undef MX_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// ============================================================================================
// Measured-slower backward variant: compiled only with -DMXLLM_ATTN_EXPERIMENTS.
// The default build has ONE D = 128 backward family: attn_bwd8_kernel + attn_bwd_dq_kernel.
#ifdef MXLLM_ATTN_EXPERIMENTS
// Staggered split-mode key-block kernel (MXLLM_ATTN_BWD8=2).  Same work split
// as attn_bwd8_kernel (8 waves = 4 key groups x 2 q halves, 128 keys of one q head per workgroup),
// but the two q halves run HALF A TILE apart: each tile is two phases -- A: S = Q K^T, dP = dO V^T
// and the softmax, B: dV^T += dO^T P, dK^T += Q^T dS -- separated by a barrier, and waves 4-7 start
// one barrier late.  One half's softmax VALU then runs under the other half's MFMAs (in
// attn_bwd8_kernel both halves hit the softmax at the same time behind one barrier per tile, and the
// faster half waited ~1,260 cycles per tile: archive/profiles/r4ad/README.md).  The offset needs the Q / dO
// tiles of THREE iterations in LDS (a 3-slot ring, 96 KB + the 64 KB K / V images = the CU's whole
// 160 KB), so lse / delta no longer go through LDS: each wave loads its 32 rows' values one
// iteration ahead into one VGPR (lanes 0-31 lse, 32-63 delta) and broadcasts them with shuffles.
// Issue / wait schedule (barrier numbers of the leading half: tile L = barriers 2L .. 2L+2):
//   lead (waves 0-3) issues iteration L+2's DMA and L+1's lse/delta at the start of its phase B(L),
//   lag (waves 4-7) at the start of its phase A(L) -- both right after slot (L+2) % 3 was last read
//   (barrier 2L+1) -- and each waits for iteration L+1's DMA only at the barrier before which it
//   must have landed (2L+2 for the lead's B(L), 2L+2 for the lag's A(L)), with counted vmcnt waits
//   that leave the newer loads / DMA / dS^T stores in flight (retirement is in issue order; the
//   issue order is pinned with sched_barrier).  1.5 tiles of DMA lookahead instead of 1.
template <bool CAUSAL>
__global__ void __launch_bounds__(512, 1)
attn_bwd8s_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                  const uint16_t* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                  uint16_t* __restrict__ dST, float* __restrict__ dKp, float* __restrict__ dVp, int B, int Hq,
                  int Hkv, int S, int Sk, int off, float sl, float scale, int S_pad, int hpw) {
  constexpr int D = 128, BN = 128, BQ = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int KIMG = BN * ROWB;  // K (or V) image [128][D]: 32 KB
  constexpr int QT = BQ * ROWB;    // Q / dO tile [64][D]: 16 KB
  constexpr int SLOT = 2 * QT;     // ring slot: Q tile | dO tile
  constexpr int NSLOT = 3;
  constexpr int LDSB = 2 * KIMG + NSLOT * SLOT;
  static_assert(LDSB <= 160 * 1024, "the CU's LDS");
  static_assert(LDSB >= 4 * 2 * DB * 16 * 64 * 4, "dK/dV pair reduction reuses the tile LDS");
  constexpr int SEGS = QT / 1024;
  static_assert(SEGS / 8 == 2, "two pieces per wave");
  __shared__ __attribute__((aligned(1024))) char smem[LDSB];
  char* kimg = smem;
  char* vimg = smem + KIMG;
  typedef __attribute__((address_space(3))) void* lptr_t;

  const int nkb = (Sk + BN - 1) / BN;
  const int HP = Hq / hpw;
  const int BHP = B * HP;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BHP, (Hq / Hkv) / hpw);
  const int kb = bid / BHP;
  const int bhp = bid % BHP;
  if (kb >= nkb) return;
  const int b = bhp / HP, hp = bhp % HP, h0 = hp * hpw, hk = h0 / (Hq / Hkv);
  const uint16_t* Kp = K + (size_t)(b * Hkv + hk) * Sk * D;
  const uint16_t* Vp = V + (size_t)(b * Hkv + hk) * Sk * D;
  const size_t dstride = (size_t)Hq * D;
  auto Qp = [&](int h) { return Q + (size_t)(b * Hq + h) * S * D; };
  auto dOp = [&](int h) { return dO + (size_t)b * S * dstride + (size_t)h * D; };
  auto dstp = [&](int h) { return dST + (size_t)(b * Hq + h) * (nkb * BN) * S_pad; };

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kg = w & 3, m = w >> 2;  // m = 0: the leading half, 1: the lagging half
  const int r = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int k0 = kb * BN;
  const int key = k0 + 32 * kg + r;

  {  // K / V images of the key block (rows past Sk read as zeros: masked)
    const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)Kp, 0, Sk * ROWB, 0x00020000);
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)Vp, 0, Sk * ROWB, 0x00020000);
#pragma unroll
    for (int i = 0; i < KIMG / 1024 / 8; ++i) {
      const int seg = w * (KIMG / 1024 / 8) + i;
      const int row = seg * (1024 / ROWB) + lane / (ROWB / 16), slot = lane % (ROWB / 16);
      const int vo = (k0 + row) * ROWB + 16 * (slot ^ swzb<CH>(row));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(kimg + seg * 1024), 16, vo, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(vimg + seg * 1024), 16, vo, 0, 0, 0);
    }
  }
  f32x16 dk[DB], dv[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < 16; ++j) { dk[d][j] = 0.f; dv[d][j] = 0.f; }

  int qstart = 0;
  if (CAUSAL) qstart = max(0, (k0 - off) / BQ * BQ);
  const int nqt = qstart < S ? (S - qstart + BQ - 1) / BQ : 0;
  const int nit = nqt * hpw;  // flattened (head, q tile) iterations

  const int orec = (int)(((size_t)(S - 1) * dstride + D) * 2);
  const int pseg = w * (SEGS / 8);
  typedef int i32x2_t __attribute__((ext_vector_type(2)));
  i32x2_t qoff = {0, 0}, ooff = {0, 0};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int prow = (pseg + i) * (1024 / ROWB) + lane / (ROWB / 16), pslot = lane % (ROWB / 16);
    const int pch = pslot ^ swzb<CH>(prow);
    qoff[i] = prow * ROWB + pch * 16;
    ooff[i] = (int)(prow * dstride * 2) + pch * 16;
  }
  // iteration L -> (head offset hj, q tile it)
  auto iter = [&](int L, int& hj, int& it) {
    hj = L / nqt;
    it = L - hj * nqt;
  };
  // this wave's 4 DMA pieces (2 Q, 2 dO) of iteration L into ring slot L % 3
  auto dma_to = [&](int L, int slot) {
    int hj, it;
    iter(L, hj, it);
    const int h = h0 + hj, q0 = qstart + it * BQ;
    char* qt = smem + 2 * KIMG + slot * SLOT;
    char* dot = qt + QT;
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc((void*)Qp(h), 0, S * ROWB, 0x00020000);
    const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc((void*)dOp(h), 0, orec, 0x00020000);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lptr_t)(qt + (pseg + i) * 1024), 16, qoff[i] + q0 * ROWB, 0, 0,
                                               0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ors, (lptr_t)(dot + (pseg + i) * 1024), 16,
                                               ooff[i] + (int)(q0 * dstride * 2), 0, 0, 0);
    }
  };
  // lse (lanes 0-31) / delta (lanes 32-63) of this wave's 32 rows of iteration L: ONE load
  auto ldload = [&](int L) -> float {
    int hj, it;
    iter(L, hj, it);
    const int h = h0 + hj;
    const int q = min(qstart + it * BQ + 32 * m + r, S - 1);
    const float* base = (hh ? DELTA : LSE) + (size_t)(b * Hq + h) * S;
    return base[q];
  };


  const uint32_t tile_base = lds_addr(smem + 2 * KIMG);
  static_assert(ROWB == 256 && (SLOT % 256) == 0 && (KIMG % 256) == 0, "XOR addressing assumes 256-B rows");
  uint32_t trA, trB;
  {
    const int rowA = 32 * m + 4 * hh + tq, rowB = rowA + 8;
    const int chunk = (16 * (g & 1) + 4 * tp) >> 3;
    trA = rowA * ROWB + 16 * (chunk ^ swzb<CH>(rowA)) + 8 * (tp & 1);
    trB = rowB * ROWB + 16 * (chunk ^ swzb<CH>(rowB)) + 8 * (tp & 1);
  }
  const int swz = swzb<CH>(r);
  const uint32_t qrowb = (32 * m + r) * ROWB + 16 * (hh ^ swz);
  const uint32_t krowb = lds_addr(kimg) + (32 * kg + r) * ROWB + 16 * (hh ^ swz);

  // prologue: K / V images, iterations 0 and 1, lse / delta of iteration 0; all landed
  float ldc = 0.f, ldn = 0.f;
  if (nit > 0) {
    ldc = ldload(0);
    dma_to(0, 0);
  }
  if (nit > 1) dma_to(1, 1);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  if (m == 1) __builtin_amdgcn_s_barrier();  // the lagging half starts one barrier late

  // ops this wave issues per iteration: the next lse/delta (1) and the DMA two iterations ahead (4)
  // -- UNCONDITIONALLY (past the last iteration: the last iteration's data again, into the slot
  // nobody reads any more), so every iteration issues the same ops and hipcc's own waits for the
  // lse/delta register stay counted -- and the previous iteration's dS^T stores (4, from L = 1 on)
  auto issue_ahead = [&](int L) {
    ldn = ldload(min(L + 1, nit - 1));
    __builtin_amdgcn_sched_barrier(0);
    dma_to(min(L + 2, nit - 1), (L + 2) % NSLOT);
    __builtin_amdgcn_sched_barrier(0);
  };

  int hj = 0, it = 0;
  for (int L = 0; L < nit; ++L) {
    const int q0 = qstart + it * BQ;
    const uint32_t sbase = tile_base + (uint32_t)(L % NSLOT) * SLOT;
    // ================= phase A: S, dP, softmax
    if (m == 1) issue_ahead(L);
    const bool need_mask = (q0 + BQ > S) || (k0 + BN > Sk) || (CAUSAL && (k0 + 32 * kg + 31 > q0 + 32 * m + off));
    f32x16 sa, dp;
#pragma unroll
    for (int j = 0; j < 16; ++j) { sa[j] = 0.f; dp[j] = 0.f; }
    {
      const uint32_t qb = sbase + qrowb, kb2 = krowb;
      u16x8 f[2][4];
      auto ld = [&](int st, u16x8 (&x)[4]) {
        const uint32_t qa = qb ^ (uint32_t)(32 * st), ka = kb2 ^ (uint32_t)(32 * st);
        x[0] = rd128_off(qa, 0);
        x[1] = rd128_off(ka, 0);
        x[2] = rd128_off(qa, QT);
        x[3] = rd128_off(ka, KIMG);
      };
      ld(0, f[0]);
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st + 1 < KS) ld(st + 1, f[(st + 1) & 1]);
        lds_wait_le(st + 1 < KS ? 4 : 0);
        u16x8(&x)[4] = f[st & 1];
#pragma unroll
        for (int y = 0; y < 4; ++y) pin(x[y]);
        sa = mfma32b(x[0], x[1], sa);
        dp = mfma32b(x[2], x[3], dp);
      }
    }
    // rows of sa/dp: q = q0 + 32m + (j&3) + 8(j>>2) + 4hh ; lse / delta of row 32m + rr in lane rr / 32 + rr
#pragma unroll
    for (int gq = 0; gq < 4; ++gq)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = 4 * gq + jj;
        const int rr = 8 * gq + 4 * hh + jj;
        const float lv = __shfl(ldc, rr, 64);
        const float dl = __shfl(ldc, 32 + rr, 64);
        float p;
        if (need_mask) {
          const int q = q0 + 32 * m + jj + 8 * gq + 4 * hh;
          const bool dead = (key >= Sk) | (q >= S) | (CAUSAL & (key > q + off));
          p = dead ? 0.f : __builtin_amdgcn_exp2f(sa[j] * sl - lv);
        } else {
          p = __builtin_amdgcn_exp2f(sa[j] * sl - lv);
        }
        sa[j] = p;
        dp[j] = p * (dp[j] - dl);
      }
    u16x8 pb[2], sb[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pb[s2][j] = f2bf(sa[8 * s2 + j]);
        sb[s2][j] = f2bf(dp[8 * s2 + j]);
      }
    if (m == 1 && L >= 1) {
      // lag, end of A(L): iteration L+1's DMA (issued in A(L-1)) lands before the barrier that
      // opens it for the leading half; newer ops (B(L-1)'s 4 stores, this A's 5 issues) may pend
      vm_wait_le(4 + 1 + 4);
    }
    lds_wait();
    __builtin_amdgcn_s_barrier();
    // ================= phase B: dV^T += dO^T P, dK^T += Q^T dS
    if (m == 0) issue_ahead(L);
    const uint32_t ta = sbase + trA, tb = sbase + trB;
    u16x4 tr[2][4];
    auto issue_tr = [&](int i, u16x4 (&t)[4]) {
      const int s2 = i / DB, db = i % DB;
      const uint32_t a = ta ^ (uint32_t)(64 * db), bb = tb ^ (uint32_t)(64 * db);
      t[0] = trd_off(a, s2 * 16 * ROWB + QT);
      t[1] = trd_off(bb, s2 * 16 * ROWB + QT);
      t[2] = trd_off(a, s2 * 16 * ROWB);
      t[3] = trd_off(bb, s2 * 16 * ROWB);
    };
    issue_tr(0, tr[0]);
#pragma unroll
    for (int i = 0; i < 2 * DB; ++i) {
      if (i + 1 < 2 * DB) issue_tr(i + 1, tr[(i + 1) & 1]);
      lds_wait_le(i + 1 < 2 * DB ? 4 : 0);
      u16x4(&t)[4] = tr[i & 1];
#pragma unroll
      for (int x = 0; x < 4; ++x) pin(t[x]);
      const int s2 = i / DB, db = i % DB;
      dv[db] = mfma32b(u16x8{t[0][0], t[0][1], t[0][2], t[0][3], t[1][0], t[1][1], t[1][2], t[1][3]}, pb[s2], dv[db]);
      dk[db] = mfma32b(u16x8{t[2][0], t[2][1], t[2][2], t[2][3], t[3][0], t[3][1], t[3][2], t[3][3]}, sb[s2], dk[db]);
    }
    {  // this iteration's dS^T (4 stores; not kept live across the loop: the register budget)
      uint16_t* rowp = dstp(h0 + hj) + ((size_t)(q0 / BQ) * (nkb * BN) + key) * BQ + 32 * m;
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<u16x4*>(rowp + 8 * gq + 4 * hh) =
            u16x4{f2bf(dp[4 * gq]), f2bf(dp[4 * gq + 1]), f2bf(dp[4 * gq + 2]), f2bf(dp[4 * gq + 3])};
    }
    __builtin_amdgcn_sched_barrier(0);
    if (m == 0 && L >= 1) {
      // lead, end of B(L): iteration L+1's DMA (issued in B(L-1)) lands before this barrier;
      // newer ops (B(L-1)'s 4 stores, this B's 5 issues and 4 stores) may pend
      vm_wait_le(4 + 1 + 4 + 4);
    }
    lds_wait();
    __builtin_amdgcn_s_barrier();
    ldc = ldn;
    iter(L + 1, hj, it);
  }
  if (m == 0) __builtin_amdgcn_s_barrier();  // match the lagging half's extra barrier
  // the unconditional look-ahead DMA of the last iterations may still be writing ring slots the
  // reduction below reuses
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // sum the two halves' partials: m = 1 waves park theirs in LDS ([kg][value][lane], conflict-free)
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem) + (size_t)kg * (2 * DB * 16) * 64 + lane;
  if (m == 1) {
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        red[((db * 16) + j) * 64] = dk[db][j];
        red[((DB * 16) + db * 16 + j) * 64] = dv[db][j];
      }
  }
  __syncthreads();
  if (m == 0 && key < Sk) {
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        dk[db][j] += red[((db * 16) + j) * 64];
        dv[db][j] += red[((DB * 16) + db * 16 + j) * 64];
      }
    float* dkq = dKp + ((size_t)bhp * Sk + key) * D;
    float* dvq = dVp + ((size_t)bhp * Sk + key) * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = db * 32 + 8 * gq + 4 * hh;
        *reinterpret_cast<f32x4*>(dkq + d) =
            f32x4{dk[db][4 * gq] * scale, dk[db][4 * gq + 1] * scale, dk[db][4 * gq + 2] * scale,
                  dk[db][4 * gq + 3] * scale};
        *reinterpret_cast<f32x4*>(dvq + d) = f32x4{dv[db][4 * gq], dv[db][4 * gq + 1], dv[db][4 * gq + 2],
                                                  dv[db][4 * gq + 3]};
      }
  }
}

#endif  // MXLLM_ATTN_EXPERIMENTS

// Deterministic dQ: dq[b,h,q,:] = sum over the key blocks that visited q (ascending kb)
// of the partials written by attn_bwd_kernel<.., DQM=2>.  One thread per 4 floats.
template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256) attn_bwd_dq_reduce(const float* __restrict__ part, float* __restrict__ dq,
                                                          int BH, int S, int S_pad, int nkb, int off) {
  constexpr int V = D / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)BH * S * V) return;
  const int c = (int)(i % V);
  const int64_t row = i / V;
  const int q = (int)(row % S);
  const int64_t bh = row / S;
  const size_t kstride = (size_t)BH * S_pad * D;
  const float* p = part + ((size_t)bh * S_pad + q) * D + 4 * c;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int kb = 0; kb < nkb; ++kb) {
    if (CAUSAL && max(0, (kb * 128 - off) / 64 * 64) > q) break;  // key blocks past q never visited it
    acc += *reinterpret_cast<const f32x4*>(p + kb * kstride);
  }
  *reinterpret_cast<f32x4*>(dq + row * D + 4 * c) = acc;
}


// dQ for the split backward (DQM 3): one workgroup per (QB x 64 q rows, q head), 4 waves
// per 64-row sub-block, all sharing each streamed K tile (QB=2 halves K traffic):
// dQ[q][:] = scale * sum over 64-key tiles of dS[64 x 64] . K[64 x D], with dS^T tiles
// ([key][q] bf16, written by attn_bwd_kernel<.., 3>, blocked per 64-q tile) and K tiles
// streamed through LDS by LDS-DMA in an NSTAGE ring (NSTAGE-1 tiles in flight while one
// is consumed; counted vmcnt waits + bare s_barrier so no barrier drains the ring),
// inline-asm tr-reads for both MFMA operands (a builtin tr-read would make hipcc drain
// the in-flight DMA), f32 accumulators in registers, one plain store: no atomics.
template <int D, bool CAUSAL, int QB>
__global__ void __launch_bounds__(256 * QB, 1)
attn_bwd_dq_kernel(const uint16_t* __restrict__ dST, const uint16_t* __restrict__ K, float* __restrict__ dQ,
                   int B, int Hq, int Hkv, int S, int Sk, int off, int S_pad, int Sk_pad, float scale,
                   uint16_t* __restrict__ dqkv = nullptr, int64_t ldq = 0, const float* __restrict__ cosb = nullptr,
                   const float* __restrict__ sinb = nullptr) {
  constexpr int BK = 64, BQ = 64, CH = D / 8, ROWB = D * 2, DB = D / 32;
  constexpr int DSROWB = BQ * 2;     // dS^T image row: 64 q = 128 B
  constexpr int KT = BK * ROWB;      // K tile [64][D]
  constexpr int DT = BK * DSROWB;    // one dS^T tile [64 keys][64 q]
  constexpr int BUF = KT + QB * DT;
  constexpr int NSTAGE = QB == 2 ? 4 : 3;
  constexpr int NT = (2 * DB + 3) / 4;
  constexpr int KSEG = KT / 1024, DSEG = DT / 1024;     // 1-KiB LDS-DMA segments
  constexpr int NW = 4 * QB;                            // waves
  constexpr int PER_WAVE = (KSEG + QB * DSEG) / NW;     // glds instructions per wave per stage
  static_assert((KSEG + QB * DSEG) % NW == 0, "stage must split evenly over the waves");
  static_assert(PER_WAVE <= 15, "vmcnt immediate");
  __shared__ __attribute__((aligned(16))) char smem[NSTAGE * BUF];
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;

  const int nqb = (S + BQ * QB - 1) / (BQ * QB);
  const int BH = B * Hq;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BH, Hq / Hkv);
  const int qb = nqb - 1 - bid / BH;  // causal: last q blocks see the most keys -> first
  const int bh = bid % BH;
  const int b = bh / Hq, h = bh % Hq, hk = h / (Hq / Hkv);
  const int q0 = qb * BQ * QB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sub = w / 4, wl = w % 4;  // 64-row sub-block of this wave, wave index within it
  const int r = lane & 31, hh = lane >> 5;
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const uint16_t* dsp = dST + (size_t)bh * Sk_pad * S_pad;
  const uint16_t* Kp = K + (size_t)(b * Hkv + hk) * Sk * D;
  // 64-key tiles the key-block kernel wrote for this workgroup (last sub-block) and for
  // this wave's sub-block (tiles past it were never written: skipped)
  int kend = Sk, kend_w = Sk;
  if (CAUSAL) {
    kend = min(Sk, q0 + BQ * QB + off);
    kend_w = min(Sk, q0 + BQ * (sub + 1) + off);
  }
  const int nkt = (kend + BK - 1) / BK;
  const int nkt_w = (kend_w + BK - 1) / BK;
  const int qsub0 = q0 + BQ * sub;

  auto glds = [&](int it) {
    char* kt = smem + (it % NSTAGE) * BUF;
    const int kb0 = it * BK;
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int seg = w * PER_WAVE + i;
      if (seg < KSEG) {
        const int byte = seg * 1024 + lane * 16;
        const int row = byte / ROWB, slot = (byte % ROWB) / 16;
        const int ch = slot ^ swzb<CH>(row);
        const int kk = min(kb0 + row, Sk - 1);
        __builtin_amdgcn_global_load_lds((gptr_t)(Kp + (size_t)kk * D + ch * 8), (lptr_t)(kt + seg * 1024), 16, 0,
                                         0);
      } else {
        const int sg = seg - KSEG;          // over QB dS^T tiles
        const int jt = sg / DSEG, sgl = sg % DSEG;
        const int byte = sgl * 1024 + lane * 16;
        const int row = byte / DSROWB, slot = (byte % DSROWB) / 16;
        const int ch = slot ^ swz8b(row);
        const int qt64 = q0 / BQ + jt;  // 64-q tile index; clamp a tail tile past S_pad
        const int qtc = min(qt64, S_pad / BQ - 1);
        __builtin_amdgcn_global_load_lds((gptr_t)(dsp + ((size_t)qtc * Sk_pad + kb0 + row) * BQ + ch * 8),
                                         (lptr_t)(kt + KT + jt * DT + sgl * 1024), 16, 0, 0);
      }
    }
  };

  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[t][j] = 0.f;
  // per-lane byte offsets of this wave's MFMA fragments inside one stage buffer
  // (the k-step s only adds a compile-time 16-row offset: the swizzle of rows
  // 16s + r0 does not depend on s)
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)smem;
  uint32_t aA[NT], aB[NT], bA[NT], bB[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tile = min(wl + 4 * t, 2 * DB - 1);
    const int m = tile / DB, db = tile % DB;
    const int rA0 = 4 * hh + tq, rB0 = rA0 + 8;
    const int qchunk = (32 * m + 16 * (g & 1) + 4 * tp) >> 3;
    const int dchunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
    aA[t] = KT + sub * DT + rA0 * DSROWB + 16 * (qchunk ^ swz8b(rA0)) + 8 * (tp & 1);
    aB[t] = KT + sub * DT + rB0 * DSROWB + 16 * (qchunk ^ swz8b(rB0)) + 8 * (tp & 1);
    bA[t] = rA0 * ROWB + 16 * (dchunk ^ swzb<CH>(rA0)) + 8 * (tp & 1);
    bB[t] = rB0 * ROWB + 16 * (dchunk ^ swzb<CH>(rB0)) + 8 * (tp & 1);
  }

#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p)
    if (p < nkt) glds(p);
  for (int it = 0; it < nkt; ++it) {
    // this wave's DMA for stage `it` retired (up to NSTAGE-2 later stages may stay in
    // flight), then every wave's
    const int ahead = min(NSTAGE - 2, nkt - 1 - it);
    if (ahead >= 2) __builtin_amdgcn_s_waitcnt(0x0F70 | ((2 * PER_WAVE) & 0xF) | (((2 * PER_WAVE) >> 4) << 14));
    else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | (PER_WAVE & 0xF) | ((PER_WAVE >> 4) << 14));
    else __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();  // also: every wave finished stage it-1, whose buffer is refilled below
    if (it + NSTAGE - 1 < nkt) glds(it + NSTAGE - 1);
    if (it < nkt_w) {
      const uint32_t sb = lds0 + (uint32_t)((it % NSTAGE) * BUF);
      if constexpr (NT == 2 && DB == 4) {
        // D = 128: this wave's two tiles are (m = 0, db = wl) and (m = 1, db = wl): one set
        // of K fragments feeds both (3 tr-reads per MFMA instead of 4; the loop is LDS-bound)
        u16x4 fa[2][4][2], fb[4][2];
#define MX_DQ_READ2(S)                                                 \
  fb[S][0] = trd_asm<S * 16 * ROWB>(sb + bA[0]);                       \
  fb[S][1] = trd_asm<S * 16 * ROWB>(sb + bB[0]);                       \
  fa[0][S][0] = trd_asm<S * 16 * DSROWB>(sb + aA[0]);                  \
  fa[0][S][1] = trd_asm<S * 16 * DSROWB>(sb + aB[0]);                  \
  fa[1][S][0] = trd_asm<S * 16 * DSROWB>(sb + aA[1]);                  \
  fa[1][S][1] = trd_asm<S * 16 * DSROWB>(sb + aB[1]);
        MX_DQ_READ2(0) MX_DQ_READ2(1) MX_DQ_READ2(2) MX_DQ_READ2(3)
#undef MX_DQ_READ2
        lds_wait_le(12);  // k steps 0 and 1 landed (steps 2 and 3 still in flight)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          pin(fb[s2][0]); pin(fb[s2][1]);
          pin(fa[0][s2][0]); pin(fa[0][s2][1]); pin(fa[1][s2][0]); pin(fa[1][s2][1]);
        }
#pragma unroll
        for (int s2 = 0; s2 < BK / 16; ++s2) {
          if (s2 == 2) {
            lds_wait();
#pragma unroll
            for (int x = 2; x < 4; ++x) {
              pin(fb[x][0]); pin(fb[x][1]);
              pin(fa[0][x][0]); pin(fa[0][x][1]); pin(fa[1][x][0]); pin(fa[1][x][1]);
            }
          }
          const u16x4 b0 = fb[s2][0], b1 = fb[s2][1];
          const u16x8 bf = u16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const u16x4 a0 = fa[t][s2][0], a1 = fa[t][s2][1];
            acc[t] = mfma32b(u16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]}, bf, acc[t]);
          }
        }
        continue;
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (wl + 4 * t < 2 * DB) {
          u16x4 fa[4][2], fb[4][2];
#define MX_DQ_READ(S)                                                  \
  fa[S][0] = trd_asm<S * 16 * DSROWB>(sb + aA[t]);                     \
  fa[S][1] = trd_asm<S * 16 * DSROWB>(sb + aB[t]);                     \
  fb[S][0] = trd_asm<S * 16 * ROWB>(sb + bA[t]);                       \
  fb[S][1] = trd_asm<S * 16 * ROWB>(sb + bB[t]);
          MX_DQ_READ(0) MX_DQ_READ(1) MX_DQ_READ(2) MX_DQ_READ(3)
#undef MX_DQ_READ
          lds_wait();
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) {
            pin(fa[s2][0]); pin(fa[s2][1]); pin(fb[s2][0]); pin(fb[s2][1]);
          }
#pragma unroll
          for (int s2 = 0; s2 < BK / 16; ++s2) {
            const u16x4 a0 = fa[s2][0], a1 = fa[s2][1], b0 = fb[s2][0], b1 = fb[s2][1];
            acc[t] = mfma32b(u16x8{a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]},
                             u16x8{b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]}, acc[t]);
          }
        }
      }
    }
  }
  // dqkv (D = 128): the q columns of the token-major d(qkv) directly -- scaled, the inverse RoPE
  // applied in fp32 and rounded to bf16 once, the arithmetic of rope_merge_bwd_kernel -- instead of
  // an fp32 dQ that kernel re-reads (70B training shape: 134 MB written + 134 MB read per layer
  // become 67 MB written).  The rotate-half partner of column d is d +- 64, held by wave wl ^ 2 of
  // the sub-block: the tile goes through LDS ([sub][64 rows][128] fp32, the freed stage buffers).
  if constexpr (D == 128) {
    if (dqkv != nullptr) {
      static_assert(QB * BQ * D * 4 <= NSTAGE * BUF, "dQ exchange tile fits the stage buffers");
      lds_wait();
      __syncthreads();  // every wave past its last stage reads (the last stage waited vmcnt(0))
      float* xs = reinterpret_cast<float*>(smem) + (size_t)sub * BQ * D;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int tile = wl + 4 * t;
        if (tile < 2 * DB) {
          const int m = tile / DB, db = tile % DB;
#pragma unroll
          for (int j = 0; j < 16; ++j)
            xs[(32 * m + (j & 3) + 8 * (j >> 2) + 4 * hh) * D + db * 32 + r] = acc[t][j] * scale;
        }
      }
      __syncthreads();
      constexpr int HALF = D / 2;
      for (int u = wl * 64 + lane; u < BQ * (HALF / 8); u += 256) {
        const int row = u / (HALF / 8), c = (u % (HALF / 8)) * 8;
        const int q = qsub0 + row;
        if (q >= S) continue;
        const float* x = xs + row * D;
        const f32x4 u0 = *reinterpret_cast<const f32x4*>(x + c), u1 = *reinterpret_cast<const f32x4*>(x + c + 4);
        const f32x4 w0 = *reinterpret_cast<const f32x4*>(x + HALF + c);
        const f32x4 w1 = *reinterpret_cast<const f32x4*>(x + HALF + c + 4);
        const float a1[8] = {u0[0], u0[1], u0[2], u0[3], u1[0], u1[1], u1[2], u1[3]};
        const float a2[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
        const float* cp = cosb + (int64_t)q * HALF + c;
        const float* sp = sinb + (int64_t)q * HALF + c;
        u16x8 y1, y2;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float cj = cp[j], sj = sp[j];
          y1[j] = f2bf(__builtin_fmaf(a1[j], cj, a2[j] * sj));  // same contraction as rope_merge_bwd_kernel
          y2[j] = f2bf(__builtin_fmaf(a2[j], cj, -(a1[j] * sj)));
        }
        uint16_t* dst = dqkv + ((int64_t)b * S + q) * ldq + (int64_t)h * D;
        *reinterpret_cast<u16x8*>(dst + c) = y1;
        *reinterpret_cast<u16x8*>(dst + HALF + c) = y2;
      }
      return;
    }
  }
  // C layout: row = qsub0 + 32m + (j&3) + 8(j>>2) + 4hh, col = db*32 + r
  float* dqp = dQ + (size_t)bh * S * D;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tile = wl + 4 * t;
    if (tile < 2 * DB) {
      const int m = tile / DB, db = tile % DB;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int q = qsub0 + 32 * m + (j & 3) + 8 * (j >> 2) + 4 * hh;
        if (q < S) dqp[(size_t)q * D + db * 32 + r] = acc[t][j] * scale;
      }
    }
  }
}

}  // namespace mx

using namespace mx;

// o: token-major rows with row stride ldo (elements); dout contiguous [B, S, Hq*D].
// dq_mode 1 (atomic): dq [B,Hq,ceil(S/64)*64,D] f32 must be ZEROED by the caller (padded
//   rows absorb the unguarded tail atomics).
// dq_mode 2 (deterministic): work = ceil(Sk/128) * B*Hq*ceil(S/64)*64*D floats (no
//   zeroing); dq receives the result unpadded [B,Hq,S,D], reduced in a fixed order.
// dq_mode 3 (split, default): work = B*Hq * ceil(Sk/128)*128 * ceil(S/64)*64 bf16 (dS^T,
//   no zeroing); dq receives [B,Hq,S,D] from attn_bwd_dq_kernel.  Deterministic.
// delta: workspace [B,Hq,S].
// q-heads per workgroup of the 8-wave backward (split mode, D = 128): the largest of 4 / 2 / 1
// that divides the GQA group and still leaves >= 2 workgroups per CU (512) for the causal
// heavy-to-light balance; MXLLM_ATTN_BWD8_HPW forces a value.  1 on every other path.
static bool attn_bwd8_on() {
  static const bool on = [] {  // MXLLM_ATTN_BWD8=0: the one-wave-per-SIMD split kernel (A/B)
    const char* e = getenv("MXLLM_ATTN_BWD8");
    return !(e && e[0] == '0');
  }();
  return on;
}
#ifdef MXLLM_ATTN_EXPERIMENTS
static bool attn_bwd8_stagger() {  // MXLLM_ATTN_BWD8=2: the staggered half-tile schedule (read per call: A/B)
  const char* e = getenv("MXLLM_ATTN_BWD8");
  return e && e[0] == '2';
}
#endif
static int attn_bwd8_hpw(int B, int Hq, int Hkv, int S, int Sk, int D, int dq_mode) {
  (void)S;
  if (dq_mode != 3 || D != 128 || !attn_bwd8_on() || Hkv <= 0 || Hq % Hkv) return 1;
  const char* fe = getenv("MXLLM_ATTN_BWD8_HPW");  // read per call (tests sweep it)
  const int forced = fe && *fe ? atoi(fe) : 0;
  const int G = Hq / Hkv, nkb = (Sk + 127) / 128;
  if (forced > 0) return G % forced == 0 ? forced : 1;
  for (int hpw = 4; hpw > 1; hpw >>= 1)
    if (G % hpw == 0 && (int64_t)nkb * B * (Hq / hpw) >= 512) return hpw;
  return 1;
}

// dK / dV partial heads mx_attn_bwd writes per batch row (dKp / dVp are [B, this, Sk, D] f32;
// each KV head's partials are consecutive: sum them to get dK / dV)
extern "C" int mx_attn_bwd_partial_heads(int B, int Hq, int Hkv, int S, int Sk, int D, int dq_mode) {
  return Hq / attn_bwd8_hpw(B, Hq, Hkv, S, Sk, D, dq_mode);
}

extern "C" int mx_attn_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                           const uint16_t* dout, const float* lse, float* delta, float* dq, float* dkp, float* dvp,
                           int B, int Hq, int Hkv, int S, int Sk, int D, int causal, float scale, int dq_mode,
                           void* work, int64_t ldo, hipStream_t stream, uint16_t* dqkv, int64_t ldq,
                           const float* cosb, const float* sinb) {
  if (B <= 0 || S <= 0 || Sk <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv) return -1;
  if (dq_mode < 1 || dq_mode > 3 || (dq_mode > 1 && !work)) return -1;
  // dqkv: the split dQ kernel writes d(q) with the inverse RoPE into it (D = 128, split mode only)
  if (dqkv && (dq_mode != 3 || D != 128 || !cosb || !sinb || ldq % 8 || causal < 0)) return -1;
  const int64_t rows = (int64_t)B * S * Hq;
  const int64_t dthreads = rows * (D / 8);
  const unsigned dgrid = (unsigned)((dthreads + 255) / 256);
  if (D == 128) attn_bwd_delta_kernel<128><<<dgrid, 256, 0, stream>>>(dout, o, delta, B, S, Hq, ldo);
  else if (D == 64) attn_bwd_delta_kernel<64><<<dgrid, 256, 0, stream>>>(dout, o, delta, B, S, Hq, ldo);
  else if (D == 32) attn_bwd_delta_kernel<32><<<dgrid, 256, 0, stream>>>(dout, o, delta, B, S, Hq, ldo);
  else return -1;
  const int nkb = (Sk + 127) / 128;
  const int grid = nkb * B * Hq;
  const float sl = scale * 1.4426950408889634f;
  const int off = Sk - S;
  const int S_pad = (S + 63) / 64 * 64;  // dq / dS^T rows are padded (see contract above)
#ifdef MXLLM_ATTN_EXPERIMENTS
  if (causal < 0) {  // ablation: no dQ work at all (timing experiments only; dq left untouched)
    attn_bwd_kernel<128, true, 0><<<grid, 256, 0, stream>>>(q, k, v, dout, lse, delta, dq, dkp, dvp, B, Hq, Hkv,
                                                            S, Sk, off, sl, scale, S_pad);
    return (int)hipGetLastError();
  }
#else
  if (causal < 0) return -1;
#endif
  float* dqk = dq_mode == 1 ? dq : reinterpret_cast<float*>(work);
  const bool bwd8 = attn_bwd8_on();
  // MXLLM_ATTN_BWD8_PRIO (bit flags, default 273): 1 = s_setprio 1 for waves 4-7, 16 = spread the
  // DMA / dS-store issue over the MFMA steps; 256 (with 16) = counted end-of-tile wait that leaves
  // the dS^T stores in flight (B2 S2048: 0.627 -> 0.599 ms, headline -2.9 ms; archive/profiles/r4ad/);
  // 2 = timing ablation (same q tile every step, wrong results)
  static const int bwd8_prio = [] {
    const char* e = getenv("MXLLM_ATTN_BWD8_PRIO");
    return e && *e ? atoi(e) : 273;
  }();
  const int hpw = attn_bwd8_hpw(B, Hq, Hkv, S, Sk, D, dq_mode);
  const int grid8 = nkb * B * (Hq / hpw);
#ifdef MXLLM_ATTN_EXPERIMENTS
  static const bool bwd8_prof = [] {  // MXLLM_ATTN_PROF=1: phase-cycle report of the 8-wave kernel (stderr)
    const char* e = getenv("MXLLM_ATTN_PROF");
    return e && e[0] == '1';
  }();
  if (dq_mode == 3 && D == 128 && bwd8 && bwd8_prof) {
    uint16_t* dst = reinterpret_cast<uint16_t*>(work);
    uint32_t* pbuf = nullptr;
    const size_t n = (size_t)grid8 * 128;
    if (hipMalloc(&pbuf, n * 4) != hipSuccess) return -1;
    (void)hipMemsetAsync(pbuf, 0, n * 4, stream);
    if (causal)
      attn_bwd8_kernel<true, true><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S,
                                                              Sk, off, sl, scale, S_pad, bwd8_prio, hpw, pbuf);
    else
      attn_bwd8_kernel<false, true><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S,
                                                               Sk, off, sl, scale, S_pad, bwd8_prio, hpw, pbuf);
    std::vector<uint32_t> h(n);
    (void)hipMemcpyAsync(h.data(), pbuf, n * 4, hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    (void)hipFree(pbuf);
    double sum[2][5] = {}, tiles[2] = {}, tt = 0, rt = 0, pro = 0, epi = 0;
    for (size_t wv = 0; wv < (size_t)grid8 * 8; ++wv) {
      const int half = (int)(wv % 8) >> 2;
      for (int kk = 0; kk < 5; ++kk) sum[half][kk] += h[wv * 16 + kk];
      tiles[half] += h[wv * 16 + 5];
      tt += h[wv * 16 + 6];
      rt += h[wv * 16 + 7];
      pro += h[wv * 16 + 8];
      epi += (double)h[wv * 16 + 9] - h[wv * 16 + 6];
    }
    const double nwv = (double)grid8 * 8;
    fprintf(stderr, "[attn_bwd8 prof] s_memtime rate %.0f MHz; per wave: prologue %.0f, loop %.0f, epilogue %.0f cycles\n",
            rt > 0 ? 100.0 * tt / rt : 0.0, pro / nwv, tt / nwv, epi / nwv);
    for (int half = 0; half < 2; ++half)
      fprintf(stderr, "[attn_bwd8 prof] waves %d-%d cycles/tile: issue %.0f  S,dP %.0f  softmax %.0f  dV,dK %.0f  barrier %.0f\n",
              4 * half, 4 * half + 3, sum[half][0] / tiles[half], sum[half][1] / tiles[half], sum[half][2] / tiles[half],
              sum[half][3] / tiles[half], sum[half][4] / tiles[half]);
  } else if (dq_mode == 3 && D == 128 && bwd8 && attn_bwd8_stagger()) {
    uint16_t* dst = reinterpret_cast<uint16_t*>(work);
    if (causal)
      attn_bwd8s_kernel<true><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S, Sk,
                                                         off, sl, scale, S_pad, hpw);
    else
      attn_bwd8s_kernel<false><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S, Sk,
                                                          off, sl, scale, S_pad, hpw);
  } else
#endif
  if (dq_mode == 3 && D == 128 && bwd8) {
    uint16_t* dst = reinterpret_cast<uint16_t*>(work);
    if (causal)
      attn_bwd8_kernel<true><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S, Sk,
                                                        off, sl, scale, S_pad, bwd8_prio, hpw);
    else
      attn_bwd8_kernel<false><<<grid8, 512, 0, stream>>>(q, k, v, dout, lse, delta, dst, dkp, dvp, B, Hq, Hkv, S, Sk,
                                                         off, sl, scale, S_pad, bwd8_prio, hpw);
  } else {
#define BWD(DD, C)                                                                                                  \
  do {                                                                                                              \
    if (dq_mode == 3)                                                                                               \
      attn_bwd_kernel<DD, C, 3><<<grid, 256, 0, stream>>>(q, k, v, dout, lse, delta, dqk, dkp, dvp, B, Hq, Hkv, S,  \
                                                          Sk, off, sl, scale, S_pad);                               \
    else if (dq_mode == 2)                                                                                          \
      attn_bwd_kernel<DD, C, 2><<<grid, 256, 0, stream>>>(q, k, v, dout, lse, delta, dqk, dkp, dvp, B, Hq, Hkv, S,  \
                                                          Sk, off, sl, scale, S_pad);                               \
    else                                                                                                            \
      attn_bwd_kernel<DD, C, 1><<<grid, 256, 0, stream>>>(q, k, v, dout, lse, delta, dqk, dkp, dvp, B, Hq, Hkv, S,  \
                                                          Sk, off, sl, scale, S_pad);                               \
  } while (0)
  if (D == 128) { if (causal) BWD(128, true); else BWD(128, false); }
  else if (D == 64) { if (causal) BWD(64, true); else BWD(64, false); }
  else if (D == 32) { if (causal) BWD(32, true); else BWD(32, false); }
  else return -1;
#undef BWD
  }
  if (dq_mode == 2) {
    const int64_t n = (int64_t)B * Hq * S * (D / 4);
    const unsigned rg = (unsigned)((n + 255) / 256);
    float* part = reinterpret_cast<float*>(work);
#define RED(DD)                                                                                                 \
  do {                                                                                                          \
    if (causal) attn_bwd_dq_reduce<DD, true><<<rg, 256, 0, stream>>>(part, dq, B * Hq, S, S_pad, nkb, off);     \
    else attn_bwd_dq_reduce<DD, false><<<rg, 256, 0, stream>>>(part, dq, B * Hq, S, S_pad, nkb, off);           \
  } while (0)
    if (D == 128) RED(128);
    else if (D == 64) RED(64);
    else RED(32);
#undef RED
  } else if (dq_mode == 3) {
    // 128 q rows per workgroup (every K tile feeds two 64-row sub-blocks); D=32 keeps 64
    // MXLLM_ATTN_DQ_QB=2 (experiment): D = 128 with 128 q rows per workgroup and a 4-deep ring
#ifdef MXLLM_ATTN_EXPERIMENTS
    static const int qb128 = [] {
      const char* e = getenv("MXLLM_ATTN_DQ_QB");
      return e && e[0] == '2' ? 2 : 4;
    }();
#else
    constexpr int qb128 = 4;
#endif
    const int qbs = D == 128 ? qb128 : (D == 64 ? 2 : 1);
    const int qgrid = ((S + 64 * qbs - 1) / (64 * qbs)) * B * Hq;
    const uint16_t* dst = reinterpret_cast<const uint16_t*>(work);
#define DQK(DD)                                                                                                   \
  do {                                                                                                            \
    constexpr int QB = DD == 128 ? 4 : (DD == 64 ? 2 : 1);                                                        \
    if (causal)                                                                                                   \
      attn_bwd_dq_kernel<DD, true, QB><<<qgrid, 256 * QB, 0, stream>>>(dst, k, dq, B, Hq, Hkv, S, Sk, off, S_pad,  \
                                                                       nkb * 128, scale, dqkv, ldq, cosb, sinb);  \
    else                                                                                                          \
      attn_bwd_dq_kernel<DD, false, QB><<<qgrid, 256 * QB, 0, stream>>>(dst, k, dq, B, Hq, Hkv, S, Sk, off, S_pad, \
                                                                        nkb * 128, scale, dqkv, ldq, cosb, sinb); \
  } while (0)
#ifdef MXLLM_ATTN_EXPERIMENTS
    if (D == 128 && qbs == 2) {
      if (causal)
        attn_bwd_dq_kernel<128, true, 2><<<qgrid, 512, 0, stream>>>(dst, k, dq, B, Hq, Hkv, S, Sk, off, S_pad, nkb * 128,
                                                                   scale, dqkv, ldq, cosb, sinb);
      else
        attn_bwd_dq_kernel<128, false, 2><<<qgrid, 512, 0, stream>>>(dst, k, dq, B, Hq, Hkv, S, Sk, off, S_pad,
                                                                    nkb * 128, scale, dqkv, ldq, cosb, sinb);
    } else
#endif
    if (D == 128) DQK(128);
    else if (D == 64) DQK(64);
    else DQK(32);
#undef DQK
  }
  return (int)hipGetLastError();
}
