// Inference-side kernels for gfx950:
//   * rope_append : decode-step q/k RoPE at per-sequence positions + KV-cache append
//   * decode_attn : single-token GQA attention over a per-slot KV cache,
//                   split over the sequence (flash-decoding), memory-bound:
//                   each workgroup streams 256 keys of one (seq, kv-head) once
//                   and serves all q-heads of that group (GQA reuse);
//   * decode_combine : merges the per-split (m, l, o) partials;
//   * sample : greedy argmax or exact temperature sampling via Gumbel-max with
//              a counter-based hash RNG (one pass, no softmax materialised).
// KV cache layout per layer: [slots, Hkv, max_seq, D] bf16 (contiguous per slot
// and head: one 256-B row per token for D = 128), or PAGED: a pool of blocks
// [blocks, Hkv, block, D] addressed through a per-slot block table (common.h
// kv_row; the block size is a multiple of the 256-key decode split, so every
// split reads one contiguous block).
#include "common.h"

namespace mx {

// qkv [B, (Hq+2Hkv)*D] -> q [B, Hq, D] (rotated), K/V cache rows at pos[b]
template <int D>
__global__ void __launch_bounds__(256) rope_append_kernel(const uint16_t* __restrict__ qkv,
                                                          const float* __restrict__ cosb,
                                                          const float* __restrict__ sinb,
                                                          const int32_t* __restrict__ pos,
                                                          const int32_t* __restrict__ slots,
                                                          uint16_t* __restrict__ q, uint16_t* __restrict__ kc,
                                                          uint16_t* __restrict__ vc, int B, int Hq, int Hkv,
                                                          int max_seq, const int32_t* __restrict__ bt, int maxb) {
  constexpr int HALF = D / 2, CPH = HALF / 8;
  const int NH = Hq + 2 * Hkv;
  const int64_t n = (int64_t)B * NH * CPH;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int cc = (int)(i % CPH);
    const int head = (int)((i / CPH) % NH);
    const int b = (int)(i / ((int64_t)CPH * NH));
    const int c = cc * 8;
    const int p = pos[b];
    const int slot = slots ? slots[b] : b;
    const uint16_t* src = qkv + (int64_t)b * NH * D + (int64_t)head * D;
    u16x8 x1 = *reinterpret_cast<const u16x8*>(src + c);
    u16x8 x2 = *reinterpret_cast<const u16x8*>(src + HALF + c);
    uint16_t* dst;
    if (head >= Hq + Hkv) {
      dst = vc + kv_row(bt, maxb, max_seq, slot, Hkv, head - Hq - Hkv, p) * D;
      *reinterpret_cast<u16x8*>(dst + c) = x1;
      *reinterpret_cast<u16x8*>(dst + HALF + c) = x2;
      continue;
    }
    dst = head < Hq ? q + ((int64_t)b * Hq + head) * D
                    : kc + kv_row(bt, maxb, max_seq, slot, Hkv, head - Hq, p) * D;
    const float* cp = cosb + (int64_t)p * HALF + c;
    const float* sp = sinb + (int64_t)p * HALF + c;
    u16x8 y1, y2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float a = bf2f(x1[j]), bb = bf2f(x2[j]);
      y1[j] = f2bf(a * cp[j] - bb * sp[j]);
      y2[j] = f2bf(bb * cp[j] + a * sp[j]);
    }
    *reinterpret_cast<u16x8*>(dst + c) = y1;
    *reinterpret_cast<u16x8*>(dst + HALF + c) = y2;
  }
}

constexpr int kSplit = 256;  // keys per workgroup
constexpr int kMaxRep = 16;  // q-heads per kv-head supported

// grid (nsplit, Hkv, B); block 256 = one key per thread for the score phase.
template <int D>
__global__ void __launch_bounds__(256) decode_attn_kernel(const uint16_t* __restrict__ q,
                                                          const uint16_t* __restrict__ kc,
                                                          const uint16_t* __restrict__ vc,
                                                          const int32_t* __restrict__ lens, int len_off,
                                                          const int32_t* __restrict__ slots,
                                                          float* __restrict__ part_ml, float* __restrict__ part_o,
                                                          int Hq, int Hkv, int max_seq, int nsplit, float sl,
                                                          const int32_t* __restrict__ bt, int maxb) {
  __shared__ float qs[kMaxRep][D];
  __shared__ float ps[kMaxRep][kSplit];
  __shared__ float red[kMaxRep][4];
  __shared__ __attribute__((aligned(16))) uint16_t vs[kSplit * D];
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int rep = Hq / Hkv;
  const int len = lens[b] + len_off;
  const int slot = slots ? slots[b] : b;
  const int k_lo = split * kSplit;
  const int k_hi = min(len, k_lo + kSplit);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  float* pml = part_ml + (((int64_t)b * Hq + hk * rep) * nsplit + split) * 2;
  if (k_lo >= k_hi) {  // empty split: neutral partial
    if (tid < rep) {
      pml[(int64_t)tid * nsplit * 2] = -INFINITY;
      pml[(int64_t)tid * nsplit * 2 + 1] = 0.f;
    }
    return;
  }
  for (int i = tid; i < rep * D; i += 256) {
    const int h = i / D, d = i % D;
    qs[h][d] = bf2f(q[((int64_t)b * Hq + hk * rep + h) * D + d]);
  }
  // base such that base + key * D addresses every key of this split (a paged split lies in
  // one block: the block size is a multiple of kSplit)
  const int64_t kvb = (kv_row(bt, maxb, max_seq, slot, Hkv, hk, k_lo) - k_lo) * D;
  const uint16_t* kbase = kc + kvb;
  const uint16_t* vbase = vc + kvb;
  // stage V rows of this split into LDS (coalesced 16-B chunks)
  constexpr int CH = D / 8;
  for (int c = tid; c < kSplit * CH; c += 256) {
    const int row = c / CH, ch = c % CH, key = k_lo + row;
    u16x8 v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (key < k_hi) v = *reinterpret_cast<const u16x8*>(vbase + (int64_t)key * D + ch * 8);
    *reinterpret_cast<u16x8*>(vs + row * D + ch * 8) = v;
  }
  __syncthreads();
  const int key = k_lo + tid;
  float s[kMaxRep];
#pragma unroll
  for (int h = 0; h < kMaxRep; ++h) s[h] = -INFINITY;
  if (key < k_hi) {
#pragma unroll
    for (int h = 0; h < kMaxRep; ++h) s[h] = 0.f;
    const uint16_t* kr = kbase + (int64_t)key * D;
#pragma unroll 4
    for (int c = 0; c < D; c += 8) {
      const u16x8 kv = *reinterpret_cast<const u16x8*>(kr + c);
      float kf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) kf[j] = bf2f(kv[j]);
#pragma unroll
      for (int h = 0; h < kMaxRep; ++h) {
        if (h < rep) {
#pragma unroll
          for (int j = 0; j < 8; ++j) s[h] += qs[h][c + j] * kf[j];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < kMaxRep; ++h) s[h] *= sl;
  }
  // per-head max over the split
#pragma unroll
  for (int h = 0; h < kMaxRep; ++h) {
    if (h < rep) {
      const float m = wave_max(s[h]);
      if (lane == 0) red[h][wid] = m;
    }
  }
  __syncthreads();
  float mh[kMaxRep];
#pragma unroll
  for (int h = 0; h < kMaxRep; ++h)
    mh[h] = h < rep ? fmaxf(fmaxf(red[h][0], red[h][1]), fmaxf(red[h][2], red[h][3])) : 0.f;
  __syncthreads();
#pragma unroll
  for (int h = 0; h < kMaxRep; ++h) {
    if (h < rep) {
      const float p = key < k_hi ? __builtin_amdgcn_exp2f(s[h] - mh[h]) : 0.f;
      ps[h][tid] = p;
      const float l = wave_sum(p);
      if (lane == 0) red[h][wid] = l;
    }
  }
  __syncthreads();
  if (tid < rep) {
    pml[(int64_t)tid * nsplit * 2] = mh[tid];
    pml[(int64_t)tid * nsplit * 2 + 1] = red[tid][0] + red[tid][1] + red[tid][2] + red[tid][3];
  }
  // o[h][d] = sum_key p[h][key] v[key][d]: thread -> (h, d pair)
  const int nkeys = k_hi - k_lo;
  for (int o = tid; o < rep * (D / 2); o += 256) {
    const int h = o / (D / 2), d = (o % (D / 2)) * 2;
    float a0 = 0.f, a1 = 0.f;
    for (int kk = 0; kk < nkeys; ++kk) {
      const float p = ps[h][kk];
      const uint32_t pr = *reinterpret_cast<const uint32_t*>(vs + kk * D + d);
      a0 += p * bf2f((uint16_t)(pr & 0xffff));
      a1 += p * bf2f((uint16_t)(pr >> 16));
    }
    float* po = part_o + ((((int64_t)b * Hq + hk * rep + h) * nsplit + split) * D) + d;
    po[0] = a0;
    po[1] = a1;
  }
}

// ---------------------------------------------------------------------------
// MFMA decode attention, D = 128 (every Llama-3.x model).  Memory-bound: the
// whole point is to stream each (seq, kv-head)'s cached K/V rows once at HBM
// rate, so
//   * a workgroup = 4 waves = 256 keys of one (seq, kv-head); each wave owns 64
//     keys and keeps its own online-softmax state (no barrier in the key loop);
//   * scores for ALL q-heads of the GQA group at once with
//     v_mfma_f32_16x16x32_bf16: S^T[key][head] = K . Q^T, K rows loaded straight
//     from HBM into the A fragments (16 B per lane), Q^T (heads padded to 16)
//     as the B fragment;
//   * the S^T accumulator (head on the lane, keys in registers) converted to
//     bf16 IS the B operand of O^T[d][head] += V^T . P (keys permuted inside
//     each 32-key k-step to match the accumulator's row order);
//   * V^T fragments come from a row-major V image in LDS through
//     ds_read_b64_tr_b16; the image is filled by LDS-DMA (global_load_lds,
//     source-swizzled so the transposed reads are conflict-free);
//   * the four waves' partials are merged through LDS (each wave reuses its own
//     V region) into one (m, l, o) partial per split, the format of
//     decode_combine_kernel.
// 64 KiB LDS and < 128 VGPRs: two workgroups (8 waves) per CU, 256 KiB of K/V
// in flight per CU.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

__device__ __forceinline__ f32x4 mfma16(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b),
                                                 c, 0, 0, 0);
}

__device__ __forceinline__ u16x4 tr_read16(const char* p) {
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(u16x4, v);
}

// 16-B chunk swizzle of a 256-B row (conflict-free row and transposed reads)
__device__ __forceinline__ int dswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// stores / loads of the split partials that another workgroup of the SAME launch merges:
// write-through (sc1, relaxed agent-scope atomic store), so no release fence (an L2
// write-back per workgroup) is needed, and loads that bypass this CU's L1 (guide
// §6 Guideline 16, the sc1 hand-off form)
// st: 0 = plain store, 1 = agent-scope relaxed atomic store (sc1 write-through),
// 2 = system-scope relaxed atomic store; ld: 0 = plain load, 1 = agent, 2 = system
__device__ __forceinline__ void st_part(float* p, float v, int st) {
  if (st == 1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if (st == 2) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  else *p = v;
}
__device__ __forceinline__ float ld_part(const float* p, int ld) {
  float* q = const_cast<float*>(p);
  if (ld == 1) return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (ld == 2) return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return *p;
}

// one split of decode_attn_mfma_kernel: (m, l, o) partial of 256 keys for every
// q-head of the GQA group (see the kernel's header comment)
__device__ __forceinline__ void decode_split_body(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                  const uint16_t* __restrict__ vc, float* __restrict__ part_o,
                                                  float* __restrict__ pml, char* smem, float (*mls)[2][16], int b,
                                                  int hk, int rep, int Hq, int split, int nsplit, int k_lo, int k_hi,
                                                  int slot, int max_seq, float sl, const int32_t* __restrict__ bt,
                                                  int maxb, int Hkv, int st) {
  constexpr int D = 128, ROWB = 256, WKEYS = 64, WTILE = WKEYS * ROWB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int64_t kvb = (kv_row(bt, maxb, max_seq, slot, Hkv, hk, k_lo) - k_lo) * D;  // one block per split
  const uint16_t* kbase = kc + kvb;
  const uint16_t* vbase = vc + kvb;
  const int wk0 = k_lo + WKEYS * w;
  char* vs = smem + w * WTILE;

  // V rows of this wave -> LDS (16 x 1-KiB lane-linear DMA pieces; swizzle by
  // permuting each lane's SOURCE chunk).  Rows past k_hi duplicate a valid row
  // (finite; their probabilities are exactly 0).
#pragma unroll
  for (int seg = 0; seg < 16; ++seg) {
    const int row = seg * 4 + (lane >> 4), slt = lane & 15;
    const int ch = slt ^ dswz(row);
    const int key = min(wk0 + row, k_hi - 1);
    __builtin_amdgcn_global_load_lds((gptr_t)(vbase + (int64_t)key * D + ch * 8), (lptr_t)(vs + seg * 1024), 16, 0,
                                     0);
  }
  // Q^T fragments (B operand): lane (c, g) holds Q[head c][32 s + 8 g .. +7]
  u16x8 qf[4];
  const uint16_t* qrow = q + ((int64_t)b * Hq + hk * rep + min(c, rep - 1)) * D;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *reinterpret_cast<const u16x8*>(qrow + 32 * s + 8 * g);
    if (c >= rep) qf[s] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  // K fragments (A operand), straight from HBM: block j, k-step s ->
  // K[wk0 + 16 j + c][32 s + 8 g .. +7]
  u16x8 kf[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int key = min(wk0 + 16 * j + c, k_hi - 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) kf[j][s] = *reinterpret_cast<const u16x8*>(kbase + (int64_t)key * D + 32 * s + 8 * g);
  }
  f32x4 sacc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) sacc[j] = mfma16(kf[j][s], qf[s], sacc[j]);
  }
  // softmax over this wave's 64 keys, per head (= lane column c); lane (c, g)
  // holds keys wk0 + 16 j + 4 g + i
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int key = wk0 + 16 * j + 4 * g + i;
      const float x = key < k_hi ? sacc[j][i] * sl : -INFINITY;
      sacc[j][i] = x;
      mx = fmaxf(mx, x);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  const float mref = mx == -INFINITY ? 0.f : mx;  // wave with no valid key: all p = 0
  float ls = 0.f;
  u16x8 pb[2];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float p = __builtin_amdgcn_exp2f(sacc[j][i] - mref);
      ls += p;
      pb[j >> 1][4 * (j & 1) + i] = f2bf(p);
    }
  ls += __shfl_xor(ls, 16, 64);
  ls += __shfl_xor(ls, 32, 64);

  // O^T[d][head] += V^T . P; k-step t covers keys 32 t + {16 h + 4 g + i}
  f32x4 oacc[8];
#pragma unroll
  for (int db = 0; db < 8; ++db) oacc[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's V DMA has landed (only it reads vs)
  const int qq = c >> 2, pp = c & 3;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int r0 = 32 * t + 4 * g + qq, r1 = r0 + 16;
#pragma unroll
    for (int db = 0; db < 8; ++db) {
      const int ch = 2 * db + (pp >> 1);
      const u16x4 va = tr_read16(vs + r0 * ROWB + 16 * (ch ^ dswz(r0)) + 8 * (pp & 1));
      const u16x4 vb = tr_read16(vs + r1 * ROWB + 16 * (ch ^ dswz(r1)) + 8 * (pp & 1));
      const u16x8 a = u16x8{va[0], va[1], va[2], va[3], vb[0], vb[1], vb[2], vb[3]};
      oacc[db] = mfma16(a, pb[t], oacc[db]);
    }
  }
  // merge the four waves: each wave parks (m, l, O^T) in its own V region
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's transposed reads retired
  float* so = reinterpret_cast<float*>(vs);  // [d][16 heads]
#pragma unroll
  for (int db = 0; db < 8; ++db)
#pragma unroll
    for (int i = 0; i < 4; ++i) so[(16 * db + 4 * g + i) * 16 + c] = oacc[db][i];
  if (g == 0) {
    mls[w][0][c] = mx;
    mls[w][1][c] = ls;
  }
  __syncthreads();
  for (int idx = tid; idx < rep * D; idx += 256) {
    const int h = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) M = fmaxf(M, mls[ww][0][h]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float mw = mls[ww][0][h];
      const float f = mw == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mw - M);
      L += f * mls[ww][1][h];
      acc += f * reinterpret_cast<const float*>(smem + ww * WTILE)[d * 16 + h];
    }
    st_part(&part_o[(((int64_t)b * Hq + hk * rep + h) * nsplit + split) * D + d], acc, st);
    if (d == 0) {
      st_part(&pml[(int64_t)h * nsplit * 2], M, st);
      st_part(&pml[(int64_t)h * nsplit * 2 + 1], L, st);
    }
  }
}

// proto (fused split merge, cnt != nullptr; 0 = partials only / combine kernel):
//   1 = partials stored with agent-scope (sc1, write-through) atomic stores, read back with
//       agent-scope atomic loads, no fences;
//   2 = the same at system scope;
//   3 = agent-scope stores, an agent-scope acquire fence in the merger, plain loads;
//   4 = plain stores, one agent-scope release fence per workgroup (lane 0, after every wave's
//       vmcnt drain), acquire fence in the merger, plain loads (guide §5 in-launch split-K recipe).
__global__ void __launch_bounds__(256, 2) decode_attn_mfma_kernel(const uint16_t* __restrict__ q,
                                                                  const uint16_t* __restrict__ kc,
                                                                  const uint16_t* __restrict__ vc,
                                                                  const int32_t* __restrict__ lens, int len_off,
                                                                  const int32_t* __restrict__ slots,
                                                                  float* __restrict__ part_ml,
                                                                  float* __restrict__ part_o, int Hq, int Hkv,
                                                                  int max_seq, int nsplit, float sl,
                                                                  const int32_t* __restrict__ bt, int maxb,
                                                                  uint16_t* __restrict__ out,
                                                                  unsigned int* __restrict__ cnt, int proto) {
  constexpr int D = 128, WTILE = 64 * 256;  // 16 KiB per wave
  __shared__ __attribute__((aligned(16))) char smem[4 * WTILE];
  __shared__ float mls[4][2][16];
  __shared__ int s_last;
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int rep = Hq / Hkv;
  const int len = lens[b] + len_off;
  const int slot = slots ? slots[b] : b;
  const int k_lo = split * kSplit;
  const int k_hi = min(len, k_lo + kSplit);
  const int tid = threadIdx.x;
  const bool fused = cnt != nullptr;
  const int st = !fused ? 0 : proto == 2 ? 2 : proto == 4 ? 0 : 1;  // store mode of the partials
  float* pml = part_ml + (((int64_t)b * Hq + hk * rep) * nsplit + split) * 2;
  if (k_lo >= k_hi) {  // empty split (workgroup-uniform): neutral partial
    if (tid < rep) {
      st_part(&pml[(int64_t)tid * nsplit * 2], -INFINITY, st);
      st_part(&pml[(int64_t)tid * nsplit * 2 + 1], 0.f, st);
    }
  } else {
    decode_split_body(q, kc, vc, part_o, pml, smem, mls, b, hk, rep, Hq, split, nsplit, k_lo, k_hi, slot, max_seq,
                      sl, bt, maxb, Hkv, st);
  }
  if (!fused) return;
  // In-launch combine: the last of the nsplit workgroups of this (seq, kv-head) to arrive
  // merges the partials and resets the counter (zero again for the next call).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its partial stores done
  __syncthreads();
  if (tid == 0) {
    unsigned int* c = cnt + (int64_t)b * Hkv + hk;
    if (proto == 4) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned prev = proto == 2 ? __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                     : __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)(nsplit - 1);
    if (last) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (proto >= 3) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int ld = proto == 1 ? 1 : proto == 2 ? 2 : 0;
  // the same arithmetic, in the same order, as decode_combine_kernel
  for (int idx = tid; idx < rep * D; idx += 256) {
    const int h = idx / D, d = idx % D;
    const int64_t bh = (int64_t)b * Hq + hk * rep + h;
    const float* ml = part_ml + bh * nsplit * 2;
    float M = -INFINITY;
    for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, ld_part(ml + 2 * sp, ld));
    float L = 0.f, acc = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) {
      const float m = ld_part(ml + 2 * sp, ld);
      if (m == -INFINITY) continue;
      const float wgt = __builtin_amdgcn_exp2f(m - M);
      L += wgt * ld_part(ml + 2 * sp + 1, ld);
      acc += wgt * ld_part(part_o + (bh * nsplit + sp) * D + d, ld);
    }
    out[bh * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
  }
}

// merge splits: out[b, h, :] = sum_s exp2(m_s - M) o_s / sum_s exp2(m_s - M) l_s
template <int D>
__global__ void __launch_bounds__(D) decode_combine_kernel(const float* __restrict__ part_ml,
                                                           const float* __restrict__ part_o,
                                                           uint16_t* __restrict__ out, int nsplit) {
  const int64_t bh = blockIdx.x;
  const float* ml = part_ml + bh * nsplit * 2;
  const int d = threadIdx.x;
  if (nsplit <= 8) {
    // every partial load issued at once (one memory round trip instead of two: the outputs'
    // loads do not wait for the maxima); same arithmetic order as the loop below
    float mv[8], lv[8], ov[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const bool on = s < nsplit;
      mv[s] = on ? ml[2 * s] : -INFINITY;
      lv[s] = on ? ml[2 * s + 1] : 0.f;
      ov[s] = on ? part_o[(bh * nsplit + s) * D + d] : 0.f;
    }
    float M = -INFINITY;
#pragma unroll
    for (int s = 0; s < 8; ++s) M = fmaxf(M, mv[s]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      if (mv[s] == -INFINITY) continue;
      const float wgt = __builtin_amdgcn_exp2f(mv[s] - M);
      L += wgt * lv[s];
      acc += wgt * ov[s];
    }
    out[bh * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
    return;
  }
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f, acc = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const float m = ml[2 * s];
    if (m == -INFINITY) continue;
    const float wgt = __builtin_amdgcn_exp2f(m - M);
    L += wgt * ml[2 * s + 1];
    acc += wgt * part_o[(bh * nsplit + s) * D + d];
  }
  out[bh * D + d] = f2bf(L > 0.f ? acc / L : 0.f);
}

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

// logits [B, V] (bf16 or f32); temperature <= 0 -> greedy.  out ids [B] int64.
//
// Split over the vocabulary: grid (nchunks, B), each workgroup reduces `chunk`
// logits of one row to (max, smallest index); a second one-wave-per-row kernel
// combines the partials in chunk order.  One workgroup per row left a batch-1
// decode step with ONE CU streaming 256 KB of logits: 176 us of a 4.1 ms 8B
// step; split over ~63 workgroups it is a few microseconds.  (A last-arriver
// merge in the same kernel needed an agent-scope release fence per workgroup:
// 94 us at batch 64.)  The result (and the Gumbel noise of each (seed, row,
// step, index)) is the same as a single-pass argmax.  The partials live in a
// per-call workspace (allocated by the caller on its stream), so concurrent
// samplers on different streams of one device never share them.
constexpr int kSampMaxRows = 1024;   // rows per launch (more rows: several launches)
constexpr int kSampMaxChunks = 64;   // partials per row (= one wave in the final pass)

__device__ __forceinline__ void samp_pick(float& best, int& bi, float ov, int oi) {
  if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
}

template <typename T>
__global__ void __launch_bounds__(256) sample_kernel(const T* __restrict__ logits, int64_t* __restrict__ out, int V,
                                                     int chunk, float inv_temp, uint32_t seed, uint32_t step,
                                                     int row0, const float* __restrict__ temps,
                                                     const int64_t* __restrict__ seeds,
                                                     const int32_t* __restrict__ steps,
                                                     float* __restrict__ g_samp_val, int* __restrict__ g_samp_idx) {
  __shared__ float sv[4];
  __shared__ int si[4];
  const int lrow = blockIdx.y;
  const int64_t row = (int64_t)row0 + lrow;
  const T* x = logits + row * V;
  const int c0 = blockIdx.x * chunk, c1 = min(V, c0 + chunk);
  uint32_t nseed = seed + (uint32_t)row * 7919u;
  if (temps) {  // per-row parameters (sample_rows without top-k / top-p): noise of sampling.hip
    const float t = temps[row];
    inv_temp = t > 0.f ? 1.f / t : 0.f;
    nseed = (uint32_t)seeds[row];
    step = (uint32_t)steps[row];
  }
  float best = -INFINITY;
  int bi = c0 < V ? c0 : 0;
  for (int cb = c0 + (int)threadIdx.x; cb < c1; cb += 256 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {  // 8 independent loads in flight per thread
      const int c = cb + 256 * u;
      if constexpr (sizeof(T) == 2) v[u] = c < c1 ? bf2f(reinterpret_cast<const uint16_t*>(x)[c]) : -INFINITY;
      else v[u] = c < c1 ? reinterpret_cast<const float*>(x)[c] : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = cb + 256 * u;
      if (c >= c1) break;
      float w = v[u];
      if (inv_temp > 0.f) {
        const uint32_t h = hash3(nseed, step, (uint32_t)c);
        const float uu = ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
        w = w * inv_temp - __logf(-__logf(uu));  // Gumbel-max
      }
      if (w > best) { best = w; bi = c; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) samp_pick(best, bi, __shfl_xor(best, o, 64), __shfl_xor(bi, o, 64));
  if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = best; si[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w) samp_pick(best, bi, sv[w], si[w]);
    g_samp_val[lrow * kSampMaxChunks + blockIdx.x] = best;
    g_samp_idx[lrow * kSampMaxChunks + blockIdx.x] = bi;
  }
}

// partials of one row (chunk order) -> out[row]; grid rows, one wave
__global__ void __launch_bounds__(64) sample_final_kernel(int64_t* __restrict__ out, int nch, int row0,
                                                          const float* __restrict__ g_samp_val,
                                                          const int* __restrict__ g_samp_idx) {
  const int lrow = blockIdx.x, l = threadIdx.x;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  if (l < nch) {
    best = g_samp_val[lrow * kSampMaxChunks + l];
    bi = g_samp_idx[lrow * kSampMaxChunks + l];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) samp_pick(best, bi, __shfl_xor(best, o, 64), __shfl_xor(bi, o, 64));
  if (l == 0) out[(int64_t)row0 + lrow] = bi == 0x7fffffff ? 0 : bi;
}

}  // namespace mx

using namespace mx;

// bt / maxb: paged cache (block table [slots, maxb]; max_seq = the block size), nullptr: contiguous
extern "C" int mx_rope_append(const uint16_t* qkv, const float* cosb, const float* sinb, const int32_t* pos,
                              const int32_t* slots, uint16_t* q, uint16_t* kc, uint16_t* vc, int B, int Hq, int Hkv,
                              int D, int max_seq, const int32_t* bt, int maxb, hipStream_t stream) {
  const int64_t items = (int64_t)B * (Hq + 2 * Hkv) * (D / 16);
  if (items <= 0) return 0;
  const int grid = (int)std::min<int64_t>(1024, (items + 255) / 256);
#define RA(DD) \
  rope_append_kernel<DD><<<grid, 256, 0, stream>>>(qkv, cosb, sinb, pos, slots, q, kc, vc, B, Hq, Hkv, max_seq, bt, maxb)
  if (D == 128) RA(128); else if (D == 64) RA(64); else if (D == 32) RA(32); else return -1;
#undef RA
  return (int)hipGetLastError();
}

extern "C" int mx_decode_attn(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const int32_t* lens,
                              int len_off, const int32_t* slots, float* part_ml, float* part_o, uint16_t* out, int B,
                              int Hq, int Hkv, int D, int max_seq, int nsplit, float scale, const int32_t* bt,
                              int maxb, unsigned int* cnt, hipStream_t stream) {
  if (B <= 0) return 0;
  if (Hq % Hkv || Hq / Hkv > kMaxRep) return -1;
  if (bt && max_seq % kSplit) return -1;  // a split must lie inside one block
  dim3 grid(nsplit, Hkv, B);
  const float sl = scale * 1.4426950408889634f;
  if (D == 128) {  // out == nullptr: partials only (the o-projection merges them: skinny_gemm.hip MERGE)
    // cnt (zeroed [B * Hkv] counters, owned by the caller): the splits merge in-launch
    // MXLLM_DECODE_HANDOFF: hand-off protocol of the in-launch merge (see the kernel; read per call)
    const char* pe = getenv("MXLLM_DECODE_HANDOFF");
    const int proto = pe && *pe ? atoi(pe) : 4;
    const bool fused = out && cnt && proto >= 1 && proto <= 4;
    decode_attn_mfma_kernel<<<grid, 256, 0, stream>>>(q, kc, vc, lens, len_off, slots, part_ml, part_o, Hq, Hkv,
                                                      max_seq, nsplit, sl, bt, maxb, out, fused ? cnt : nullptr,
                                                      proto);
    if (out && !fused) decode_combine_kernel<128><<<B * Hq, 128, 0, stream>>>(part_ml, part_o, out, nsplit);
    return (int)hipGetLastError();
  }
  if (!out) return -1;
#define DA(DD)                                                                                                  \
  decode_attn_kernel<DD><<<grid, 256, 0, stream>>>(q, kc, vc, lens, len_off, slots, part_ml, part_o, Hq, Hkv, \
                                                   max_seq, nsplit, sl, bt, maxb);                              \
  decode_combine_kernel<DD><<<B * Hq, DD, 0, stream>>>(part_ml, part_o, out, nsplit)
  if (D == 64) { DA(64); } else if (D == 32) { DA(32); } else return -1;
#undef DA
  return (int)hipGetLastError();
}

// ws: float workspace of mx_sample_ws_floats(B) elements
extern "C" int64_t mx_sample_ws_floats(int B) {
  return 2 * (int64_t)std::min(B, kSampMaxRows) * kSampMaxChunks;
}

static int sample_launch(const void* logits, int is_bf16, int64_t* out, int B, int V, float temperature,
                         uint32_t seed, uint32_t step, const float* temps, const int64_t* seeds,
                         const int32_t* steps, float* ws, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V <= 0 || !ws) return -1;
  float* pv = ws;
  int* pi = reinterpret_cast<int*>(ws + (int64_t)std::min(B, kSampMaxRows) * kSampMaxChunks);
  const float it = temperature > 0.f ? 1.f / temperature : 0.f;
  int chunk = 2048, nch = (V + chunk - 1) / chunk;
  if (nch > kSampMaxChunks) {
    chunk = ((V + kSampMaxChunks - 1) / kSampMaxChunks + 255) / 256 * 256;
    nch = (V + chunk - 1) / chunk;
  }
  for (int r0 = 0; r0 < B; r0 += kSampMaxRows) {
    const dim3 grid(nch, std::min(kSampMaxRows, B - r0));
    if (is_bf16)
      sample_kernel<uint16_t><<<grid, 256, 0, stream>>>((const uint16_t*)logits, out, V, chunk, it, seed, step, r0,
                                                         temps, seeds, steps, pv, pi);
    else
      sample_kernel<float><<<grid, 256, 0, stream>>>((const float*)logits, out, V, chunk, it, seed, step, r0, temps,
                                                      seeds, steps, pv, pi);
    sample_final_kernel<<<grid.y, 64, 0, stream>>>(out, nch, r0, pv, pi);
  }
  return (int)hipGetLastError();
}

extern "C" int mx_sample(const void* logits, int is_bf16, int64_t* out, int B, int V, float temperature,
                         uint32_t seed, uint32_t step, float* ws, hipStream_t stream) {
  return sample_launch(logits, is_bf16, out, B, V, temperature, seed, step, nullptr, nullptr, nullptr, ws, stream);
}

// per-row temperature (<= 0: greedy), seed and step, no top-k / top-p: the draws of
// sampling.hip's sample_topkp_kernel for such rows (same noise), split over the vocabulary
extern "C" int mx_sample_temp_rows(const void* logits, int is_bf16, int64_t* out, int B, int V, const float* temps,
                                   const int64_t* seeds, const int32_t* steps, float* ws, hipStream_t stream) {
  return sample_launch(logits, is_bf16, out, B, V, 0.f, 0u, 0u, temps, seeds, steps, ws, stream);
}
