// Causal GQA flash-attention forward for gfx950 (SURVEY §2.4 K7 fwd, K13).
//
// Layouts: q [B,Hq,S,D], k/v [B,Hkv,Sk,D] bf16 head-major (written by
// rope_split), o token-major [B,S,Hq,D] (feeds the Wo GEMM directly),
// lse [B,Hq,S] f32 in the log2 domain of the scaled scores.
//
// Structure (CDNA HIP guide App. B "Fused attention prefill"):
//  * workgroup = NW waves = 32 NW query rows (4 by default), KV tile = 64 keys;
//  * "swapped" QK^T: S^T = K . Q^T with v_mfma_f32_32x32x16_bf16, so each lane
//    owns one query column and the tile's keys sit in its 16+16 accumulator
//    registers -> row max / row sum are in-register (+1 cross-half shuffle);
//  * the f32 S^T accumulator, converted pairwise to bf16, IS the B operand of
//    O^T += V^T . P^T (guide §3 "accumulator tile as the next MFMA's operand");
//  * V^T fragments come from the row-major V tile via ds_read_b64_tr_b16 (T10);
//  * K/V tiles live in LDS as 16-B-chunk XOR-swizzled images
//    (chunk ^ ((row&3)<<2 | (row>>2)&3)): conflict-free for both the
//    ds_read_b128 row reads of K and the transposed reads of V;
//  * K/V tiles double-buffered in LDS by LDS-DMA (tile t+1 issued before tile t's
//    MFMAs); V^T read with inline-asm tr-reads so hipcc does not drain the
//    in-flight DMA before them; tile loop unrolled by two so every LDS address
//    is a per-lane base + immediate;
//  * softmax: raw-score row max, scale folded into the exp2 argument (one FMA per
//    element), cross-half max/sum by v_permlane32_swap, deferred O rescale
//    (only when a row max grows by > 2^8: guide T13);
//  * causal blocks scheduled heaviest-first, XCD-aware block remap so the
//    q-heads sharing one KV head run on the same XCD (shared L2).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include <stdlib.h>

namespace mx {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

// s_waitcnt vmcnt(N) for a compile-time N (inline asm: invisible to hipcc's waitcnt pass)
template <int N>
__device__ __forceinline__ void g8_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int CH>
__device__ __forceinline__ int swz(int row) {
  return (((row & 3) << 2) | ((row >> 2) & 3)) & (CH - 1);
}

__device__ __forceinline__ f32x16 mfma32(const u16x8& a, const u16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ds_read_b64_tr_b16: generic -> LDS address-space cast of a __shared__ pointer
__device__ __forceinline__ u16x4 tr_read(const char* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(u16x4, v);
}

// NW waves per workgroup = 32 NW query rows sharing every streamed K/V tile (2 waves per SIMD
// either way).  4 by default; 8 halves the K/V tile traffic per FLOP but measured the same
// (0.259 vs 0.257 ms at B2 S2048 Hq64 Hkv8 D128 causal: the stream is not the limiter)
// R: depth of the K/V tile ring in LDS (R - 1 tiles in flight ahead of the one being consumed).
// One tile of lookahead (R = 2) left about a quarter of every tile waiting for the next tile's DMA
// (archive/profiles/r4ah/README.md): the DMA round trip is longer than one tile of MFMAs.  With 8 waves per
// workgroup (one workgroup per CU, 256 query rows sharing every tile) a 3- or 4-deep ring fits the
// CU's 160 KB of LDS (96 / 128 KB).
// SR (split ring, 4 waves, D = 128): K in a 3-slot ring and V in a 2-slot ring = 80 KB, so two
// workgroups still share a CU, and TWO barriers per tile: M (after the softmax, before PV: this
// tile's V landed) and E (after PV: every wave is done with the V slot the next tile restages).
// Tile kt issues K(kt + 2) and V(kt + 1) during its QK^T steps, so a K tile has two tiles of MFMAs
// to land and a V tile one and a half, where the symmetric 2-slot ring gives both one.
template <int D, bool CAUSAL, int NW, bool PROF = false, int R = 2, bool SR = false>
__global__ void __launch_bounds__(64 * NW, 8 / NW)
attn_fwd_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                uint16_t* __restrict__ O, float* __restrict__ LSE, int B, int Hq, int Hkv, int S, int Sk,
                int causal_off, float sl, int ldo, int flags, uint32_t* __restrict__ prof = nullptr) {
  // PROF (diagnostic build, MXLLM_ATTN_PROF=1): per-wave s_memtime cycle sums of the tile phases
  uint32_t ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t tp0 = 0, t_entry = 0, t_loop = 0;
  auto mark = [&](int k) {
    if constexpr (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      ph[k] += (uint32_t)(t - tp0);
      tp0 = t;
    }
  };
  if constexpr (PROF) t_entry = __builtin_amdgcn_s_memtime();
  constexpr int BM = 32 * NW, BN = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int TILE = BN * ROWB;
  constexpr int LPT = BN * CH / (64 * NW);
  static_assert(LPT >= 1 && BN * CH % (64 * NW) == 0, "K/V tile must split evenly over the waves");
  static_assert(R >= 2 && R <= 4, "ring depth 2..4");
  static_assert(!SR || (NW == 4 && R == 2 && D == 128), "split ring: the 4-wave D = 128 kernel");
  // (XOR addressing: 256-B aligned)
  __shared__ __attribute__((aligned(1024))) char smem[SR ? 5 * TILE : 2 * R * TILE];
  // byte offsets of K ring slot c (from smem) and of V ring slot c (from smem + VBASE): the LDS read
  // bases carry the region start, so every slot offset stays a ds_read immediate (< 64 KiB)
  constexpr int VBASE = SR ? 3 * TILE : TILE;
  constexpr auto KOF = [](int c) constexpr { return SR ? c * TILE : c * 2 * TILE; };
  constexpr auto VOF = [](int c) constexpr { return SR ? c * TILE : c * 2 * TILE; };

  const int nqb = (S + BM - 1) / BM;
  const int BH = B * Hq;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BH, Hq / Hkv);
  const int qb = nqb - 1 - bid / BH;
  const int bh = bid % BH;
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const uint16_t* Qp = Q + ((size_t)(b * Hq + h) * S) * D;
  const uint16_t* Kp = K + ((size_t)(b * Hkv + hk) * Sk) * D;
  const uint16_t* Vp = V + ((size_t)(b * Hkv + hk) * Sk) * D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform (no divergent branches)
  // 8 waves = two per SIMD from the same workgroup: give the upper four priority 1 so the pair
  // desynchronises and one wave's softmax runs under the other's MFMAs (guide T5, static form)
  if constexpr (NW == 8) {
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
  }
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = qb * BM;
  const int qrow = q0 + 32 * w + r;
  const int qld = min(qrow, S - 1);  // clamped, unconditional loads: no phi -> no early vmcnt(0)

  u16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const u16x8*>(Qp + (size_t)qld * D + 16 * s + 8 * hh);

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM + causal_off);
  const int ntiles = kend > 0 ? (kend + BN - 1) / BN : 0;

  // K/V tiles stream straight into LDS with LDS-DMA (global_load_lds_dwordx4):
  // one wave instruction writes 1 KiB lane-linearly, so the XOR-swizzled image
  // is produced by permuting each lane's SOURCE chunk (guide rule 21) and no
  // VGPRs are spent on staging (the kernel sits at the 256-VGPR cap).
  typedef __attribute__((address_space(1))) const void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  // buffer_load ... lds through range-checked descriptors: the per-lane source offset of each
  // piece is loop-invariant (one VALU add for the tile step), rows past Sk read as zeros (masked)
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)Kp, 0, Sk * ROWB, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)Vp, 0, Sk * ROWB, 0x00020000);
  int voff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int seg = w * LPT + i;            // 1 KiB segment of the tile image
    const int byte = seg * 1024 + lane * 16;
    const int row = byte / ROWB, slot = (byte % ROWB) / 16;
    voff[i] = row * ROWB + 16 * (slot ^ swz<CH>(row));  // logical chunk stored in this slot
  }
  auto glds_piece = [&](int kt, int buf, int i) {
    char* kb = smem + buf * 2 * TILE;
    char* vb = kb + TILE;
    const int seg = w * LPT + i;
    const int off = voff[i] + kt * TILE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(kb + seg * 1024), 16, off, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(vb + seg * 1024), 16, off, 0, 0, 0);
  };
  // split ring: piece i of K tile kt into K slot ks / of V tile kt into V slot vs (SR only: slots TILE apart).
  // The source offset goes through a local: `voff[i] + ...` written straight into the builtin's argument
  // list makes hipcc's host pass drop the kernel's launch stub (undefined __device_stub__ at load)
  auto glds_k = [&](int kt, int ks, int i) {
    char* kb = smem + ks * TILE;
    const int seg = w * LPT + i;
    const int off = voff[i] + kt * TILE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(kb + seg * 1024), 16, off, 0, 0, 0);
  };
  auto glds_v = [&](int kt, int vs, int i) {
    char* vb = smem + VBASE + vs * TILE;
    const int seg = w * LPT + i;
    const int off = voff[i] + kt * TILE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(vb + seg * 1024), 16, off, 0, 0, 0);
  };
  auto glds = [&](int kt, int buf) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) glds_piece(kt, buf, i);
  };
  // flags & 1: spread the next tile's DMA over the QK^T k steps (one K + V piece per step pair)
  // instead of one burst at the tile top
  const bool spread = (flags & 1) != 0;

  f32x16 o[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < 16; ++j) o[d][j] = 0.f;
  // m_i: the (deferred) running max of this row in the log2 domain of the scaled
  // scores; l_i: running sum of exp2(s*sl - m_i)
  float m_i = -1e30f, l_i = 0.f;

  // Loop-invariant LDS byte addresses.  The XOR swizzle of a row depends only on
  // row & 15, so for every (n, s2) k-step and both ring buffers a fragment address
  // is one per-lane base + a compile-time immediate (the tile loop is unrolled by
  // two so the buffer index is static): no VALU address math in the loop.
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t va_base[DB][2];
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int chunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
    const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
    va_base[db][0] = lds0 + VBASE + rA * ROWB + 16 * (chunk ^ swz<CH>(rA)) + 8 * (tp & 1);
    va_base[db][1] = lds0 + VBASE + rB * ROWB + 16 * (chunk ^ swz<CH>(rB)) + 8 * (tp & 1);
  }

  const uint32_t kq_base = lds0 + r * ROWB + 16 * (hh ^ swz<CH>(r));  // K row r, k step 0 (D = 128 path)
  if constexpr (SR) {  // K(0), V(0), K(1)
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      if (ntiles > 0) {
        glds_k(0, 0, i);
        glds_v(0, 0, i);
      }
      if (ntiles > 1) glds_k(1, 1, i);
    }
  } else {
#pragma unroll
    for (int t = 0; t < R - 1; ++t)
      if (t < ntiles) glds(t, t);  // the ring's first R - 1 tiles
  }
  // Retire the prologue's Q loads and tile-0 DMA with a wait the compiler's
  // waitcnt pass can see (otherwise it treats them as possibly pending at the
  // loop header and drains the in-loop prefetch under the QK MFMAs).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  const int wq_hi = q0 + 32 * w + 31;

  // One 64-key tile out of ring buffer CUR (compile-time; SR: K slot CUR % 3, V slot CUR % 2).
  if constexpr (PROF) t_loop = __builtin_amdgcn_s_memtime();
  auto tile = [&](auto cur_c, int kt) {
    constexpr int CUR = decltype(cur_c)::value;
    if constexpr (PROF) tp0 = __builtin_amdgcn_s_memtime();
    constexpr int CK = SR ? CUR % 3 : CUR, CV = SR ? CUR % 2 : CUR;  // K / V slots read by this tile
    constexpr int NXT = (CUR + R - 1) % R;  // ring slot of tile kt + R - 1 (the slot tile kt - 1 used)
    constexpr int NK = (CUR + 2) % 3, NV = (CUR + 1) % 2;  // SR: slots of K(kt + 2) / V(kt + 1)
    const int kpf = kt + R - 1;             // the tile this one prefetches (SR: V(kt + 1))
    const bool more = kpf < ntiles;
    const bool morek = SR && kt + 2 < ntiles;  // SR: K(kt + 2)
    const char* kb = smem + KOF(CK);
    const bool active = !CAUSAL || (kt * BN <= wq_hi + causal_off);
    // DMA piece i of this tile's prefetch: SR K(kt + 2) then V(kt + 1), else K and V of tile kpf
    auto pf_piece = [&](int i) {
      if constexpr (SR) {
        if (morek) glds_k(kt + 2, NK, i);
        glds_v(kt + 1, NV, i);
      } else {
        glds_piece(kpf, NXT, i);
      }
    };
    if (more && (!spread || !active)) {  // prefetch R - 1 tiles ahead (SR: 2 for K, 1 for V)
#pragma unroll
      for (int i = 0; i < LPT; ++i) pf_piece(i);
    }
    f32x16 sacc[2];
    if (active) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc[n][j] = 0.f;
      if constexpr (D == 128) {
        // both 32-key chains interleaved; K rows by asm reads one k step ahead (counted waits).
        // Key rows 32n + r share row & 15 with r, hence the swizzle: k step s is base ^ (32 s),
        // the buffer and the 32-row block n are immediates
        u16x8 kf2[2][2];
        auto ld = [&](int st, u16x8 (&x)[2]) {
          const uint32_t a = kq_base ^ (uint32_t)(32 * st);
          x[0] = rd128_off(a, KOF(CK));
          x[1] = rd128_off(a, KOF(CK) + 32 * ROWB);
        };
        ld(0, kf2[0]);
#pragma unroll
        for (int st = 0; st < KS; ++st) {
          if (st + 1 < KS) ld(st + 1, kf2[(st + 1) & 1]);
          lds_wait_le(st + 1 < KS ? 2 : 0);
          u16x8(&x)[2] = kf2[st & 1];
          pin(x[0]);
          pin(x[1]);
          sacc[0] = mfma32(x[0], qf[st], sacc[0]);
          sacc[1] = mfma32(x[1], qf[st], sacc[1]);
          if (spread && more && (st % (KS / LPT)) == 0) pf_piece(st / (KS / LPT));
        }
      } else {
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          const int krow = n * 32 + r;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const u16x8 a = *reinterpret_cast<const u16x8*>(kb + krow * ROWB + 16 * ((2 * s + hh) ^ swz<CH>(krow)));
            sacc[n] = mfma32(a, qf[s], sacc[n]);
            if (spread && more && n == 0 && (s % (KS / LPT)) == 0) pf_piece(s / (KS / LPT));
          }
        }
      }
      mark(0);
      // row max of the RAW scores (the scale is folded into the exp2 argument below)
      float mx = -INFINITY;
      const bool need_mask = (kt * BN + BN > Sk) || (CAUSAL && (kt * BN + BN - 1 > q0 + 32 * w + causal_off));
      // 4 independent partial maxima (a 32-long dependent fmax chain otherwise)
      float mp[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (need_mask) {  // wave-uniform: diagonal / tail tiles only; branch-free select per element
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int key = kt * BN + n * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh;
            const bool dead = (key >= Sk) | (CAUSAL & (key > qrow + causal_off));
            const float x = dead ? -INFINITY : sacc[n][j];
            sacc[n][j] = x;
            mp[j & 3] = fmaxf(mp[j & 3], x);
          }
      } else {
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int j = 0; j < 16; ++j) mp[j & 3] = fmaxf(mp[j & 3], sacc[n][j]);
      }
      mx = fmaxf(fmaxf(mp[0], mp[1]), fmaxf(mp[2], mp[3]));
      {  // max with the other half-wave (same query column): one permlane32 swap
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      }
      // Deferred rescale (guide T13): O and l are rescaled only when some row's
      // tile max exceeds its running max by more than kThr (log2 units), so
      // probabilities stay <= 2^kThr; the decision is wave-uniform and taken before
      // this tile's P is formed, so everything at the old scale is rescaled once.
      constexpr float kThr = 8.f;
      const float mt = mx * sl;
      if (__any(mt > m_i + kThr)) {
        const float mnew = fmaxf(m_i, mt);
        const float alpha = __builtin_amdgcn_exp2f(m_i - mnew);
        l_i *= alpha;
        m_i = mnew;
#pragma unroll
        for (int d = 0; d < DB; ++d) o[d] *= alpha;
      }
      const float nm = -m_i;
      float lp[4] = {0.f, 0.f, 0.f, 0.f};  // 4 independent partial sums
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[n][j], sl, nm));
          sacc[n][j] = p;
          lp[j & 3] += p;
        }
      l_i += (lp[0] + lp[1]) + (lp[2] + lp[3]);
      if constexpr (PROF) asm volatile("" ::"v"(l_i));
      mark(1);
    } else {
      mark(5);
    }
    if constexpr (SR) {
      // M: V(kt) -- issued by the previous tile, before this tile's prefetch -- landed for this wave
      // (vector-memory ops retire in issue order: this tile's pieces may stay in flight), then for
      // every wave.  K(kt + 1), issued with it, is covered too.  Raw barrier: no fence drain.
      const int younger = (more ? LPT : 0) + (morek ? LPT : 0);
      if (younger == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (younger == LPT) g8_vmcnt<LPT>();
      else g8_vmcnt<2 * LPT>();
      __builtin_amdgcn_s_barrier();
      mark(3);
    }
    if (active) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u16x8 pb;
#pragma unroll
          for (int j = 0; j < 8; ++j) pb[j] = f2bf(sacc[n][8 * s2 + j]);
          // V^T fragments by inline-asm transposed reads (a builtin tr-read makes hipcc
          // drain the next tile's in-flight LDS-DMA here), consumed behind counted waits
          u16x4 fv[DB][2];
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            fv[db][0] = trd_off(va_base[db][0], VOF(CV) + (32 * n + 16 * s2) * ROWB);
            fv[db][1] = trd_off(va_base[db][1], VOF(CV) + (32 * n + 16 * s2) * ROWB);
          }
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            lds_wait_le(2 * (DB - 1 - db));
            pin(fv[db][0]);
            pin(fv[db][1]);
            const u16x4 va = fv[db][0], vc = fv[db][1];
            const u16x8 a = u16x8{va[0], va[1], va[2], va[3], vc[0], vc[1], vc[2], vc[3]};
            o[db] = mfma32(a, pb, o[db]);
          }
        }
      mark(2);
    }
    if constexpr (SR) {
      // E: every wave is done reading V slot CV (restaged by the next tile) and K slot CK
      lds_wait();
      __builtin_amdgcn_s_barrier();
    } else if constexpr (R == 2) {
      __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's DMA for tile kt+1 landed
      __syncthreads();                     // ... and every other wave's; buffer CUR free again
    } else {
      // tile kt + 1 landed for this wave: the DMA of the tiles issued after it (at most R - 2, 2 LPT
      // instructions each, retiring in issue order) may stay in flight.  Raw s_barrier: the fence of
      // __syncthreads would drain them.  LDS reads of slot CUR retired first (it is restaged next).
      const int after = min(R - 2, ntiles - 2 - kt);
      lds_wait();
      if (after <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if (after == 1) g8_vmcnt<2 * LPT>();
      else g8_vmcnt<4 * LPT>();
      __builtin_amdgcn_s_barrier();
    }
    mark(3);
    if constexpr (PROF) ph[4] += 1;
  };
  for (int kt = 0; kt < ntiles; kt += (SR ? 6 : R)) {
    tile(std::integral_constant<int, 0>{}, kt);
    if (kt + 1 < ntiles) tile(std::integral_constant<int, 1>{}, kt + 1);
    if constexpr (SR) {  // 6 = lcm of the K and V ring depths: static slots
      if (kt + 2 < ntiles) tile(std::integral_constant<int, 2>{}, kt + 2);
      if (kt + 3 < ntiles) tile(std::integral_constant<int, 3>{}, kt + 3);
      if (kt + 4 < ntiles) tile(std::integral_constant<int, 4>{}, kt + 4);
      if (kt + 5 < ntiles) tile(std::integral_constant<int, 5>{}, kt + 5);
    }
    if constexpr (R > 2) {
      if (kt + 2 < ntiles) tile(std::integral_constant<int, 2 % R>{}, kt + 2);
    }
    if constexpr (R > 3) {
      if (kt + 3 < ntiles) tile(std::integral_constant<int, 3 % R>{}, kt + 3);
    }
  }
  float l_tot;
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_i), __float_as_uint(l_i), false, false);
    l_tot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < S) {
    uint16_t* op = O + ((size_t)b * S + qrow) * (size_t)ldo + (size_t)h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = db * 32 + 8 * gq + 4 * hh;
        u16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = f2bf(o[db][4 * gq + j] * inv);
        *reinterpret_cast<u16x4*>(op + d) = v4;
      }
    if (hh == 0) LSE[(size_t)(b * Hq + h) * S + qrow] = m_i + __log2f(l_tot);
  }
  if constexpr (PROF) {
    const uint64_t t_end = __builtin_amdgcn_s_memtime();
    uint32_t* pw = prof + ((size_t)blockIdx.x * NW + w) * 16;
    if (lane < 6) {
      uint32_t v = ph[0];
#pragma unroll
      for (int k = 1; k < 6; ++k) v = lane == k ? ph[k] : v;
      pw[lane] = v;
    }
    if (lane == 6) pw[6] = (uint32_t)(t_loop - t_entry);
    if (lane == 7) pw[7] = (uint32_t)(t_end - t_loop);
  }
}

// ============================================================================================
// Measured-slower forward variants: compiled only with
// -DMXLLM_ATTN_EXPERIMENTS (python -m mxllm._build with MXLLM_FILE_FLAGS="attn_fwd.hip=-DMXLLM_ATTN_EXPERIMENTS").
// The default build has ONE forward family, attn_fwd_kernel<D, CAUSAL, 4>.
#ifdef MXLLM_ATTN_EXPERIMENTS
// ---------------------------------------------------------------------------------------------
// D = 128 forward with a barrier-enforced ping-pong of two wave groups (opt-in MXLLM_ATTN_FWD=pp).
// Per 64-key tile a wave's work is a serial chain -- QK^T MFMAs, the softmax VALU (32 exp2 per
// lane: ~830 cycles, as much as the tile's 1,024 MFMA cycles), the PV MFMAs -- and the two waves
// that share a SIMD in the 4-wave kernel come from different workgroups, so nothing keeps one's
// softmax under the other's MFMAs (phase profile: ~3,700 cycles per tile against a 2,048-cycle
// MFMA floor for the pair, profiles/r5f).  Here one 8-wave workgroup (256 query rows, 32 per wave)
// owns the CU; waves w and w + 4 share a SIMD, and group B (waves 4-7) runs one phase behind
// group A.  Phases alternate, separated by workgroup barriers:
//   MFMA phase of tile t:  O += V(t-1) P(t-1)  then  S(t) = K(t) Q^T   (32 MFMAs, setprio 1)
//   VALU phase of tile t:  mask, row max, deferred rescale, P(t) = exp2(...), l, bf16 pack of P(t)
// so in every phase one wave of each SIMD issues MFMAs while the other runs its softmax.  K/V
// tiles sit in a 4-slot ring (128 KB); every wave issues its pieces of tile t + 2 during its MFMA
// phase of tile t, into the slot tile t - 2 used (last read by group B two phases earlier), and
// before the barrier that opens group A's QK^T of tile t' every wave has its pieces of t' landed
// (counted vmcnt: only tile t' + 1's may still fly).  Same arithmetic as attn_fwd_kernel.
template <bool CAUSAL>
__global__ void __launch_bounds__(512, 1)
attn_fwd_pp_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                   uint16_t* __restrict__ O, float* __restrict__ LSE, int B, int Hq, int Hkv, int S, int Sk,
                   int causal_off, float sl, int ldo) {
  constexpr int D = 128, NW = 8, BM = 32 * NW, BN = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int TILE = BN * ROWB;           // 16 KiB
  constexpr int LPT = BN * CH / (64 * NW);  // DMA pieces per wave per K (and per V) tile
  constexpr int R = 4;                      // ring slots
  static_assert(LPT == 2, "8 waves x 2 pieces = one 16 KiB tile");
  __shared__ __attribute__((aligned(1024))) char smem[R * 2 * TILE];

  const int nqb = (S + BM - 1) / BM;
  const int BH = B * Hq;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BH, Hq / Hkv);
  const int qb = nqb - 1 - bid / BH;
  const int bh = bid % BH;
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const uint16_t* Qp = Q + ((size_t)(b * Hq + h) * S) * D;
  const uint16_t* Kp = K + ((size_t)(b * Hkv + hk) * Sk) * D;
  const uint16_t* Vp = V + ((size_t)(b * Hkv + hk) * Sk) * D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = w >> 2;  // 0: group A, 1: group B (one phase behind)
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = qb * BM;
  const int qrow = q0 + 32 * w + r;
  const int qld = min(qrow, S - 1);

  u16x8 qf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) qf[s] = *reinterpret_cast<const u16x8*>(Qp + (size_t)qld * D + 16 * s + 8 * hh);

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM + causal_off);
  const int ntiles = kend > 0 ? (kend + BN - 1) / BN : 0;

  typedef __attribute__((address_space(3))) void* lptr_t;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)Kp, 0, Sk * ROWB, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)Vp, 0, Sk * ROWB, 0x00020000);
  int voff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    const int seg = w * LPT + i;
    const int byte = seg * 1024 + lane * 16;
    const int row = byte / ROWB, slot = (byte % ROWB) / 16;
    voff[i] = row * ROWB + 16 * (slot ^ swz<CH>(row));
  }
  // piece i (K and V) of tile kt into ring slot kt % R (source offsets through locals: see glds_k)
  auto dma_piece = [&](int kt, int i) {
    char* kb = smem + (kt & (R - 1)) * 2 * TILE;
    char* vb = kb + TILE;
    const int seg = w * LPT + i;
    const int off = voff[i] + kt * TILE;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(kb + seg * 1024), 16, off, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(vb + seg * 1024), 16, off, 0, 0, 0);
  };

  f32x16 o[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int j = 0; j < 16; ++j) o[d][j] = 0.f;
  float m_i = -1e30f, l_i = 0.f;

  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t va_base[DB][2];
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int chunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
    const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
    va_base[db][0] = lds0 + TILE + rA * ROWB + 16 * (chunk ^ swz<CH>(rA)) + 8 * (tp & 1);
    va_base[db][1] = lds0 + TILE + rB * ROWB + 16 * (chunk ^ swz<CH>(rB)) + 8 * (tp & 1);
  }
  const uint32_t kq_base = lds0 + r * ROWB + 16 * (hh ^ swz<CH>(r));
  const int wq_hi = q0 + 32 * w + 31;
  auto active = [&](int kt) { return !CAUSAL || (kt * BN <= wq_hi + causal_off); };

  if (ntiles > 0) {
    dma_piece(0, 0);
    dma_piece(0, 1);
  }
  if (ntiles > 1) {
    dma_piece(1, 0);
    dma_piece(1, 1);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): Q, tiles 0 and 1 (visible to hipcc's waitcnt pass)
  __syncthreads();

  f32x16 sacc[2];
  u16x8 pb[2][2];  // P(t) in bf16: the B operand of the PV MFMAs, [32-key block n][16-key step s2]
#pragma unroll
  for (int n = 0; n < 2; ++n)
#pragma unroll
    for (int j = 0; j < 16; ++j) sacc[n][j] = 0.f;

  // MFMA phase of tile t: PV(t - 1), prefetch of tile t + 2, QK^T(t)
  auto mfma_phase = [&](int t) {
    const bool pv = t >= 1 && active(t - 1);
    const bool qk = t < ntiles && active(t);
    const bool pf = t + 2 < ntiles;
    __builtin_amdgcn_s_setprio(1);
    if (pv) {
      const uint32_t vo = (uint32_t)(((t - 1) & (R - 1)) * 2 * TILE);
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          u16x4 fv[DB][2];
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            fv[db][0] = trd_off(va_base[db][0] + vo, (32 * n + 16 * s2) * ROWB);
            fv[db][1] = trd_off(va_base[db][1] + vo, (32 * n + 16 * s2) * ROWB);
          }
#pragma unroll
          for (int db = 0; db < DB; ++db) {
            lds_wait_le(2 * (DB - 1 - db));
            pin(fv[db][0]);
            pin(fv[db][1]);
            const u16x4 va = fv[db][0], vc = fv[db][1];
            const u16x8 a = u16x8{va[0], va[1], va[2], va[3], vc[0], vc[1], vc[2], vc[3]};
            o[db] = mfma32(a, pb[n][s2], o[db]);
          }
        }
    }
    if (pf && !qk) {
      dma_piece(t + 2, 0);
      dma_piece(t + 2, 1);
    }
    if (qk) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) sacc[n][j] = 0.f;
      const uint32_t kb = kq_base + (uint32_t)((t & (R - 1)) * 2 * TILE);
      u16x8 kf2[2][2];
      auto ld = [&](int st, u16x8 (&x)[2]) {
        const uint32_t a = kb ^ (uint32_t)(32 * st);  // slot offsets are multiples of 32 KiB: bits 5-7 free
        x[0] = rd128_off(a, 0);
        x[1] = rd128_off(a, 32 * ROWB);
      };
      ld(0, kf2[0]);
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st + 1 < KS) ld(st + 1, kf2[(st + 1) & 1]);
        lds_wait_le(st + 1 < KS ? 2 : 0);
        u16x8(&x)[2] = kf2[st & 1];
        pin(x[0]);
        pin(x[1]);
        sacc[0] = mfma32(x[0], qf[st], sacc[0]);
        sacc[1] = mfma32(x[1], qf[st], sacc[1]);
        if (pf && st < LPT) dma_piece(t + 2, st);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // VALU phase of tile t (active): the softmax of S(t) -> P(t) in bf16, l, deferred O rescale
  auto valu_phase = [&](int t) {
    const int kt = t;
    const bool need_mask = (kt * BN + BN > Sk) || (CAUSAL && (kt * BN + BN - 1 > q0 + 32 * w + causal_off));
    float mp[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    if (need_mask) {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = kt * BN + n * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh;
          const bool dead = (key >= Sk) | (CAUSAL & (key > qrow + causal_off));
          const float x = dead ? -INFINITY : sacc[n][j];
          sacc[n][j] = x;
          mp[j & 3] = fmaxf(mp[j & 3], x);
        }
    } else {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j) mp[j & 3] = fmaxf(mp[j & 3], sacc[n][j]);
    }
    float mx = fmaxf(fmaxf(mp[0], mp[1]), fmaxf(mp[2], mp[3]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    constexpr float kThr = 8.f;
    const float mt = mx * sl;
    if (__any(mt > m_i + kThr)) {
      const float mnew = fmaxf(m_i, mt);
      const float alpha = __builtin_amdgcn_exp2f(m_i - mnew);
      l_i *= alpha;
      m_i = mnew;
#pragma unroll
      for (int d = 0; d < DB; ++d) o[d] *= alpha;
    }
    const float nm = -m_i;
    float lp[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[n][j], sl, nm));
        sacc[n][j] = p;
        lp[j & 3] += p;
      }
    l_i += (lp[0] + lp[1]) + (lp[2] + lp[3]);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[n][s2][j] = f2bf(sacc[n][8 * s2 + j]);
  };

  // phases 2t and 2t + 1: group A runs MFMA(t) then VALU(t), group B VALU(t - 1) then MFMA(t);
  // every phase ends at a workgroup barrier (the same count for every wave: 2 ntiles + 2)
  auto phase_end = [&](bool opens_qk, int tn) {
    // before group A's QK^T of tile tn: every wave's pieces of tn have landed (this wave issued at
    // most tile tn + 1's 2 LPT pieces after them; tiles 0 / 1: the prologue's wait)
    if (opens_qk && tn >= 2 && tn < ntiles) {
      if (tn + 1 < ntiles) g8_vmcnt<2 * LPT>();
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lds_wait();                    // this phase's LDS reads retired: their slot may be restaged next
    __builtin_amdgcn_s_barrier();  // raw: __syncthreads()'s fence would drain the in-flight DMA
  };
  // One loop per group (s_barrier matches arrivals, not code addresses): in a shared loop body the
  // join after every phase keeps S of one group and P of the other live at once (256 VGPRs + spills
  // of the Q fragments; 186 and none this way)
  if (ntiles > 0) {
    if (grp == 0) {
      for (int t = 0; t <= ntiles; ++t) {
        mfma_phase(t);
        phase_end(false, 0);
        if (t < ntiles && active(t)) valu_phase(t);
        phase_end(true, t + 1);
      }
    } else {
      for (int t = 0; t <= ntiles; ++t) {
        if (t >= 1 && active(t - 1)) valu_phase(t - 1);
        phase_end(false, 0);
        mfma_phase(t);
        phase_end(true, t + 1);
      }
    }
  }

  float l_tot;
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_i), __float_as_uint(l_i), false, false);
    l_tot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qrow < S) {
    uint16_t* op = O + ((size_t)b * S + qrow) * (size_t)ldo + (size_t)h * D;
#pragma unroll
    for (int db = 0; db < DB; ++db)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int d = db * 32 + 8 * gq + 4 * hh;
        u16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = f2bf(o[db][4 * gq + j] * inv);
        *reinterpret_cast<u16x4*>(op + d) = v4;
      }
    if (hh == 0) LSE[(size_t)(b * Hq + h) * S + qrow] = m_i + __log2f(l_tot);
  }
}

// ---------------------------------------------------------------------------------------------
// D = 128 forward, software-pipelined (opt-in: MXLLM_ATTN_FWD=p; measured SLOWER than the kernel
// above -- 0.300 vs 0.265 ms at B2 S2048 Hq64 Hkv8, see archive/profiles/r1d_experiments.md -- and kept for
// the record and further work).  One wave per SIMD owning the whole register file and 64 query rows (two 32-row blocks
// that share every K / V^T fragment read, so LDS reads, LDS-DMA and address work per MFMA halve),
// 4 waves = 256 rows per workgroup.  Per 64-key tile t a wave runs two phases:
//   A(t): S(t) = K(t) Q^T for both row blocks (32 MFMAs; K fragments three k-steps ahead)
//   B(t): O += V(t-1) P(t-1) (32 MFMAs)  ||  the whole softmax of S(t) -> P(t) (bf16) and l
// so the softmax VALU of one tile runs under the PV MFMAs of the previous one instead of between
// a wave's own dependent MFMA chains.  The deferred rescale (guide T13) decided in B(t) is
// applied to O at the start of B(t+1), between PV(t-1) and PV(t).  K / V tiles arrive by
// buffer_load ... lds (per-lane source offsets loop-invariant, the tile step one VALU add; rows
// past Sk come back as zeros from the descriptor's range check) into 2-slot rings, issued one
// tile ahead right after the tile's single barrier.
// register-class pins: O stays in AGPRs (touched by VALU only in the rare rescale, which must not
// turn the loop-carried O into a VGPR phi), S / P values in VGPRs (VALU softmax)
__device__ __forceinline__ void pin_a(f32x16& v) { asm volatile("" : "+a"(v)); }
__device__ __forceinline__ void pin_v(f32x16& v) { asm volatile("" : "+v"(v)); }

template <bool CAUSAL>
__global__ void __launch_bounds__(256, 1)
attn_fwd_p_kernel(const uint16_t* __restrict__ Q, const uint16_t* __restrict__ K, const uint16_t* __restrict__ V,
                  uint16_t* __restrict__ O, float* __restrict__ LSE, int B, int Hq, int Hkv, int S, int Sk,
                  int causal_off, float sl, int ldo) {
  constexpr int D = 128, BM = 256, BN = 64, CH = D / 8, ROWB = D * 2, KS = D / 16, DB = D / 32;
  constexpr int TILE = BN * ROWB;  // 16 KiB
  constexpr int KPF = 2;           // K / Q k-steps in flight
  // LDS: K slot 0 | K slot 1 | V slot 0 | V slot 1 | Q image (256 rows; Q fragments are read
  // per k-step like K's, which keeps the register file for S, P and O)
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE + BM * ROWB];
  typedef __attribute__((address_space(3))) void* lptr_t;

  const int nqb = (S + BM - 1) / BM;
  const int BH = B * Hq;
  const int bid = xcd_balance(blockIdx.x, gridDim.x, BH, Hq / Hkv);
  const int qb = nqb - 1 - bid / BH;
  const int bh = bid % BH;
  const int b = bh / Hq, h = bh % Hq;
  const int hk = h / (Hq / Hkv);
  const uint16_t* Qp = Q + ((size_t)(b * Hq + h) * S) * D;
  const uint16_t* Kp = K + ((size_t)(b * Hkv + hk) * Sk) * D;
  const uint16_t* Vp = V + ((size_t)(b * Hkv + hk) * Sk) * D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int q0 = qb * BM;
  const int qw = q0 + 64 * w;  // first row of this wave


  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM + causal_off);
  const int T = kend > 0 ? (kend + BN - 1) / BN : 0;

  // K / V tile pieces: 16 x 1 KiB per tile, 4 per wave; lane-linear LDS writes, so the XOR swizzle
  // is applied by permuting each lane's source chunk
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc((void*)Kp, 0, Sk * ROWB, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc((void*)Vp, 0, Sk * ROWB, 0x00020000);
  int voff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int seg = w * 4 + i;
    const int row = seg * 4 + (lane >> 4), slot = lane & 15;
    voff[i] = row * ROWB + 16 * (slot ^ swz<CH>(row));
  }
  {  // Q image: 64 x 1 KiB pieces, 16 per wave (rows past S read as zeros; never stored)
    const __amdgpu_buffer_rsrc_t qrs = __builtin_amdgcn_make_buffer_rsrc((void*)(Qp + (size_t)q0 * D), 0,
                                                                         (S - q0) * ROWB, 0x00020000);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int seg = w * 16 + i;
      const int row = seg * 4 + (lane >> 4), slot = lane & 15;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(qrs, (lptr_t)(smem + 4 * TILE + seg * 1024), 16,
                                               row * ROWB + 16 * (slot ^ swz<CH>(row)), 0, 0, 0);
    }
  }
  auto dma_k = [&](int kt, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(krs, (lptr_t)(smem + slot * TILE + (w * 4 + i) * 1024), 16,
                                               voff[i] + kt * TILE, 0, 0, 0);
  };
  auto dma_v = [&](int kt, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lptr_t)(smem + (2 + slot) * TILE + (w * 4 + i) * 1024), 16,
                                               voff[i] + kt * TILE, 0, 0, 0);
  };

  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const uint32_t lds0 = lds_addr(smem);
  uint32_t ka_base[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) ka_base[s] = lds0 + r * ROWB + 16 * ((2 * s + hh) ^ swz<CH>(r));
  uint32_t qa_base[KS];  // Q image rows 64w + r (+32 for the second block: an immediate)
#pragma unroll
  for (int s = 0; s < KS; ++s) qa_base[s] = ka_base[s] + 4 * TILE + 64 * w * ROWB;
  uint32_t va_base[DB][2];
#pragma unroll
  for (int db = 0; db < DB; ++db) {
    const int chunk = (db * 32 + 16 * (g & 1) + 4 * tp) >> 3;
    const int rA = 4 * hh + tq, rB = 8 + 4 * hh + tq;
    va_base[db][0] = lds0 + 2 * TILE + rA * ROWB + 16 * (chunk ^ swz<CH>(rA)) + 8 * (tp & 1);
    va_base[db][1] = lds0 + 2 * TILE + rB * ROWB + 16 * (chunk ^ swz<CH>(rB)) + 8 * (tp & 1);
  }

  f32x16 o[2][DB];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int d = 0; d < DB; ++d)
#pragma unroll
      for (int j = 0; j < 16; ++j) o[qi][d][j] = 0.f;
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int d = 0; d < DB; ++d) pin_a(o[qi][d]);
  f32x16 sa[2][2];   // S(t) of the current tile: [row block][32-key half]
  u16x8 pb[2][4];    // P of the previous tile, bf16: [row block][16-key step]
  float m_i[2] = {-1e30f, -1e30f}, l_i[2] = {0.f, 0.f};
  float alpha_p[2] = {1.f, 1.f};
  bool resc_p = false;  // O rescale pending (decided in B(t), applied before PV(t))

  // ---- phase A: S(t) = K(t) Q^T (K slot KSLOT)
  auto phase_a = [&](int kso) __attribute__((always_inline)) {
    uint32_t kad[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s) kad[s] = ka_base[s] + kso;
    // per k-step: K rows n*32 + r (shared by both row blocks) and Q rows 64w + 32qi + r (shared
    // by both key halves); the Q image row 64w + 32qi + r has the same swizzle as K row r
    u16x8 kf[KS][2], qf[KS][2];
#pragma unroll
    for (int s = 0; s < KPF; ++s) {
      kf[s][0] = rd128_off(kad[s], 0);
      kf[s][1] = rd128_off(kad[s], 32 * ROWB);
      qf[s][0] = rd128_off(qa_base[s], 0);
      qf[s][1] = rd128_off(qa_base[s], 32 * ROWB);
    }
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + KPF < KS) {
        kf[s + KPF][0] = rd128_off(kad[s + KPF], 0);
        kf[s + KPF][1] = rd128_off(kad[s + KPF], 32 * ROWB);
        qf[s + KPF][0] = rd128_off(qa_base[s + KPF], 0);
        qf[s + KPF][1] = rd128_off(qa_base[s + KPF], 32 * ROWB);
      }
      lds_wait_le(4 * ((s + KPF < KS ? s + KPF : KS - 1) - s));
      pin(kf[s][0]);
      pin(kf[s][1]);
      pin(qf[s][0]);
      pin(qf[s][1]);
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) {
          if (s == 0) {
            f32x16 z;
#pragma unroll
            for (int j = 0; j < 16; ++j) z[j] = 0.f;
            sa[qi][n] = mfma32(kf[s][n], qf[s][qi], z);
          } else {
            sa[qi][n] = mfma32(kf[s][n], qf[s][qi], sa[qi][n]);
          }
        }
    }
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int n = 0; n < 2; ++n) pin_v(sa[qi][n]);
  };

  // ---- PV(t-1) from V slot VSLOT with pb
  auto pv = [&](int vso, auto&& hook) __attribute__((always_inline)) {
    uint32_t vad[DB][2];
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      vad[db][0] = va_base[db][0] + vso;
      vad[db][1] = va_base[db][1] + vso;
    }
    u16x4 fv[4][DB][2];
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      fv[0][db][0] = trd_off(vad[db][0], 0);
      fv[0][db][1] = trd_off(vad[db][1], 0);
    }
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      if (st + 1 < 4) {
        const int off = (32 * ((st + 1) >> 1) + 16 * ((st + 1) & 1)) * ROWB;
#pragma unroll
        for (int db = 0; db < DB; ++db) {
          fv[st + 1][db][0] = trd_off(vad[db][0], off);
          fv[st + 1][db][1] = trd_off(vad[db][1], off);
        }
      }
#pragma unroll
      for (int db = 0; db < DB; ++db) {
        lds_wait_le((st + 1 < 4 ? 2 * DB : 0) + 2 * (DB - 1 - db));
        pin(fv[st][db][0]);
        pin(fv[st][db][1]);
        const u16x4 va = fv[st][db][0], vc = fv[st][db][1];
        const u16x8 a = u16x8{va[0], va[1], va[2], va[3], vc[0], vc[1], vc[2], vc[3]};
#pragma unroll
        for (int qi = 0; qi < 2; ++qi) o[qi][db] = mfma32(a, pb[qi][st], o[qi][db]);
      }
      hook(st);
    }
  };

  // ---- softmax of S(t) -> pb, l (and the rescale decision for O), in pieces that the PV(t-1)
  // steps interleave: mask (diagonal / inactive / tail tiles, its own wave-uniform branch before
  // PV), row max per block, the rescale decision, exps + row sums + bf16 P per block
  auto mask = [&](int kt) __attribute__((always_inline)) {
    const bool need_mask = (kt * BN + BN > Sk) || (CAUSAL && (kt * BN + BN - 1 > qw + causal_off));
    if (need_mask) {
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        const int qrow = qw + 32 * qi + r;
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int key = kt * BN + n * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh;
            const bool dead = (key >= Sk) | (CAUSAL & (key > qrow + causal_off));
            sa[qi][n][j] = dead ? -INFINITY : sa[qi][n][j];
          }
      }
    }
  };
  float mt[2];
  auto sm_max = [&](int qi) __attribute__((always_inline)) {
    float m0 = -INFINITY, m1 = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      m0 = fmaxf(m0, sa[qi][0][j]);
      m1 = fmaxf(m1, sa[qi][1][j]);
    }
    float mx = fmaxf(m0, m1);
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
    mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    mt[qi] = mx * sl;
  };
  auto sm_decide = [&]() __attribute__((always_inline)) {
    constexpr float kThr = 8.f;
    const bool flag = __any((mt[0] > m_i[0] + kThr) | (mt[1] > m_i[1] + kThr));
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      const float mnew = flag ? fmaxf(m_i[qi], mt[qi]) : m_i[qi];
      alpha_p[qi] = __builtin_amdgcn_exp2f(m_i[qi] - mnew);
      m_i[qi] = mnew;
    }
    resc_p = flag;
  };
  auto sm_exp = [&](int qi) __attribute__((always_inline)) {
    const float nm = -m_i[qi];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(sa[qi][n][j], sl, nm));
        sa[qi][n][j] = p;
        if (j & 1) s1 += p; else s0 += p;
      }
    l_i[qi] = l_i[qi] * alpha_p[qi] + (s0 + s1);
  };
  auto sm_pack = [&](int qi) __attribute__((always_inline)) {
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[qi][st][j] = f2bf(sa[qi][st >> 1][8 * (st & 1) + j]);
  };
  // the softmax pieces placed after PV step st
  auto sm_hook = [&](int st) __attribute__((always_inline)) {
    if (st == 0) { sm_max(0); sm_max(1); }
    if (st == 1) { sm_decide(); sm_exp(0); }
    if (st == 2) sm_exp(1);
    if (st == 3) { sm_pack(0); sm_pack(1); }
  };
  auto softmax = [&](int kt) __attribute__((always_inline)) {
    mask(kt);
#pragma unroll
    for (int st = 0; st < 4; ++st) sm_hook(st);
  };
  auto rescale = [&]() __attribute__((always_inline)) {
    if (__builtin_expect(resc_p, 0)) {
      asm volatile("s_nop 0" ::: "memory");  // keeps the rare rescale a real branch (no if-conversion)
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int d = 0; d < DB; ++d) o[qi][d] *= alpha_p[qi];
    }
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int d = 0; d < DB; ++d) pin_a(o[qi][d]);
  };

  if (T > 0) {
    dma_k(0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's Q and K(0) pieces
    __builtin_amdgcn_s_barrier();
    dma_v(0, 0);
    if (T > 1) dma_k(1, 1);
    phase_a(0);
    softmax(0);
  }
  // tile t: [wait own DMA, barrier, DMA V(t) + K(t+1)] A(t) from K slot t&1, B(t) = PV(t-1) from
  // V slot (t-1)&1 + softmax(t).  One body with run-time slots (a VALU add per fragment base per
  // tile) so the loop-carried accumulators keep one register assignment.
  for (int t = 1; t < T; ++t) {
    const int par = t & 1;
#pragma unroll
    for (int qi = 0; qi < 2; ++qi)
#pragma unroll
      for (int d = 0; d < DB; ++d) pin_a(o[qi][d]);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();
    dma_v(t, par);
    if (t + 1 < T) dma_k(t + 1, par ^ 1);
    phase_a(par * TILE);
    mask(t);
    rescale();
    pv((par ^ 1) * TILE, sm_hook);
  }
  if (T > 0) {  // PV of the last tile
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_s_barrier();
    rescale();
    pv(((T - 1) & 1) * TILE, [](int) {});
  }

#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(l_i[qi]), __float_as_uint(l_i[qi]), false, false);
    const float l_tot = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    const int qrow = qw + 32 * qi + r;
    if (qrow < S) {
      uint16_t* op = O + ((size_t)b * S + qrow) * (size_t)ldo + (size_t)h * D;
#pragma unroll
      for (int db = 0; db < DB; ++db)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int d = db * 32 + 8 * gq + 4 * hh;
          u16x4 v4;
#pragma unroll
          for (int j = 0; j < 4; ++j) v4[j] = f2bf(o[qi][db][4 * gq + j] * inv);
          *reinterpret_cast<u16x4*>(op + d) = v4;
        }
      if (hh == 0) LSE[(size_t)(b * Hq + h) * S + qrow] = m_i[qi] + __log2f(l_tot);
    }
  }
}



// env-selected D = 128 variants (A/B only): MXLLM_ATTN_FWD=p | pp, MXLLM_ATTN_FWD_WAVES=8,
// MXLLM_ATTN_FWD_RING=3 | 4 | k3, MXLLM_ATTN_PROF=1 (phase-cycle report, host-synchronising).
// Returns 1 when none is selected (the caller launches the production kernel).
static int attn_fwd_experiment(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse,
                               int B, int Hq, int Hkv, int S, int Sk, int causal, int off, float sl, int ldo,
                               int fflags, hipStream_t stream) {
  const char* fe = getenv("MXLLM_ATTN_FWD");
  const bool pipe = fe && fe[0] == 'p' && fe[1] != 'p', pingpong = fe && fe[0] == 'p' && fe[1] == 'p';
  if (pingpong) {
    const unsigned grid = ((S + 255) / 256) * B * Hq;
    if (causal) attn_fwd_pp_kernel<true><<<grid, 512, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo);
    else attn_fwd_pp_kernel<false><<<grid, 512, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo);
    return (int)hipGetLastError();
  }
  if (pipe) {
    const unsigned grid = ((S + 255) / 256) * B * Hq;
    if (causal) attn_fwd_p_kernel<true><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo);
    else attn_fwd_p_kernel<false><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo);
    return (int)hipGetLastError();
  }
  const char* we = getenv("MXLLM_ATTN_FWD_WAVES");
  const int nw128 = (we && we[0] == '8') ? 8 : 4;
  const char* re = getenv("MXLLM_ATTN_FWD_RING");
  const int ring = (re && re[0] == 'k' && re[1] == '3') ? -3 : ((re && (atoi(re) == 3 || atoi(re) == 4)) ? atoi(re) : 0);
  const char* pe = getenv("MXLLM_ATTN_PROF");
  if (nw128 == 4 && causal && pe && pe[0] == '1') {
    const unsigned grid = ((S + 127) / 128) * B * Hq;
    const size_t n = (size_t)grid * 4 * 16;
    uint32_t* pbuf = nullptr;
    if (hipMalloc(&pbuf, n * 4) != hipSuccess) return -1;
    (void)hipMemsetAsync(pbuf, 0, n * 4, stream);
    if (ring == -3)
      attn_fwd_kernel<128, true, 4, true, 2, true><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off,
                                                                            sl, ldo, fflags, pbuf);
    else
      attn_fwd_kernel<128, true, 4, true><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo,
                                                                    fflags, pbuf);
    std::vector<uint32_t> h(n);
    (void)hipMemcpyAsync(h.data(), pbuf, n * 4, hipMemcpyDeviceToHost, stream);
    (void)hipStreamSynchronize(stream);
    (void)hipFree(pbuf);
    double sm[8] = {};
    for (size_t wv = 0; wv < (size_t)grid * 4; ++wv)
      for (int kk = 0; kk < 8; ++kk) sm[kk] += h[wv * 16 + kk];
    const double nt = sm[4] > 0 ? sm[4] : 1, nwv = (double)grid * 4;
    fprintf(stderr,
            "[attn_fwd prof] cycles/tile: QK^T %.0f  softmax %.0f  PV %.0f  barrier %.0f  (skipped-tile %.0f); per wave: "
            "prologue %.0f, loop+epilogue %.0f, tiles %.1f\n",
            sm[0] / nt, sm[1] / nt, sm[2] / nt, sm[3] / nt, sm[5] / nt, sm[6] / nwv, sm[7] / nwv, nt / nwv);
    return (int)hipGetLastError();
  }
  if (ring == -3) {
    const unsigned grid = ((S + 127) / 128) * B * Hq;
    if (causal)
      attn_fwd_kernel<128, true, 4, false, 2, true><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk, off,
                                                                             sl, ldo, fflags);
    else
      attn_fwd_kernel<128, false, 4, false, 2, true><<<grid, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk,
                                                                              off, sl, ldo, fflags);
    return (int)hipGetLastError();
  }
#define FWDR(C, RR)                                                                                    \
  attn_fwd_kernel<128, C, 8, false, RR><<<((S + 255) / 256) * B * Hq, 512, 0, stream>>>(                 \
      q, k, v, o, lse, B, Hq, Hkv, S, Sk, off, sl, ldo, fflags)
  if (ring > 0) {
    if (ring == 3) { if (causal) FWDR(true, 3); else FWDR(false, 3); }
    else { if (causal) FWDR(true, 4); else FWDR(false, 4); }
    return (int)hipGetLastError();
  }
#undef FWDR
  if (nw128 == 8) {
    if (causal)
      attn_fwd_kernel<128, true, 8><<<((S + 255) / 256) * B * Hq, 512, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk,
                                                                                    off, sl, ldo, fflags);
    else
      attn_fwd_kernel<128, false, 8><<<((S + 255) / 256) * B * Hq, 512, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, Sk,
                                                                                     off, sl, ldo, fflags);
    return (int)hipGetLastError();
  }
  return 1;
}
#endif  // MXLLM_ATTN_EXPERIMENTS
}  // namespace mx

using namespace mx;

// o: token-major [B, S, Hq*D] rows with row stride ldo (elements, >= Hq*D): the rows may
// be the left part of the LoRA-augmented o-projection input (mxllm/ops/linear.py)
extern "C" int mx_attn_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse, int B,
                           int Hq, int Hkv, int S, int Sk, int D, int causal, float scale, int ldo,
                           hipStream_t stream) {
  if (B <= 0 || S <= 0) return 0;
  if (Hkv <= 0 || Hq % Hkv || ldo < Hq * D || ldo % 8) return -1;
  const float sl = scale * 1.4426950408889634f;
  const int off = Sk - S;
  static const int fflags = [] {  // MXLLM_ATTN_FWD_FLAGS (default 1): bit 0 = spread the K/V DMA issue
    const char* e = getenv("MXLLM_ATTN_FWD_FLAGS");   // (B2 0.192 -> 0.186 ms, B16 1.372 -> 1.357 ms)
    return e && *e ? atoi(e) : 1;
  }();
#ifdef MXLLM_ATTN_EXPERIMENTS
  if (D == 128) {
    const int rc = attn_fwd_experiment(q, k, v, o, lse, B, Hq, Hkv, S, Sk, causal, off, sl, ldo, fflags, stream);
    if (rc != 1) return rc;  // 1: no experiment selected
  }
#endif
#define FWD(DD, C)                                                                                       \
  attn_fwd_kernel<DD, C, 4><<<((S + 127) / 128) * B * Hq, 256, 0, stream>>>(q, k, v, o, lse, B, Hq, Hkv, S, \
                                                                             Sk, off, sl, ldo, fflags)
  if (D == 128) { if (causal) FWD(128, true); else FWD(128, false); }
  else if (D == 64) { if (causal) FWD(64, true); else FWD(64, false); }
  else if (D == 32) { if (causal) FWD(32, true); else FWD(32, false); }
  else return -1;
#undef FWD
  return (int)hipGetLastError();
}
