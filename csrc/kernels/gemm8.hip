// 8-phase bf16 GEMM for gfx950 (VERDICT r3 "next round" item 1).
//
//   C[M, N] = alpha * op(A) op(B) (+ C when BETA),  fp32 accumulation, C fp32 or bf16,
//
// with each operand in either storage order, so the three GEMM forms of a Llama training step
// run without a transpose pass:
//   forward  y  = x W^T  : A = x  [T][in]  (k-contiguous), B = W [out][in] (k-contiguous)
//   input gr dX = dY W   : A = dY [T][out] (k-contiguous), B = W [out][in] = [k][n] (n-contiguous)
//   weight gr dW = dY^T X: A = dY [T][out] = [k][m] (m-contiguous), B = X [T][in] = [k][n]
// ("NN"-form dX ran at ~1.32 PF in hipBLASLt; token-major dW needed 6.8 / 73 ms of transposes
// per 8B / 70B-ZeRO-3 step, archive/profiles/r3o, r3p, r3d).
//
// Structure (CDNA guide §5 "The 256² 8-phase template", T1-T5, T10), designed here for the two
// operand orders:
//  * workgroup 512 threads = 8 waves as 2 (M) x 4 (N), output tile 256 x 256, each wave 128 x 64 =
//    8 x 4 blocks of v_mfma_f32_16x16x32_bf16 (16x16x32 rather than 32x32x16: the chip holds a
//    ~12-15 % higher clock on it on random data, MI355X_MICROARCH "DVFS give-back" item 7);
//  * the MFMA is issued with the operands swapped (B fragment as the A operand), so each lane's
//    4 accumulator registers are 4 CONSECUTIVE output columns of one row: 8-B (bf16) / 16-B (fp32)
//    epilogue stores instead of 2-B / 4-B ones;
//  * a K-tile (BK 64) is four 16-KiB half-tile images, A0 | A1 | B0 | B1, where A0 holds the rows
//    of output quadrant a = 0 of BOTH wave rows (and B0 the columns of quadrant b = 0 of all four
//    wave columns), so each image is read in exactly one phase;
//  * every image is filled by LDS-DMA (buffer_load ... lds, 16 B per lane, 2 per wave) into a
//    lane-linear layout; the XOR swizzle that makes the MFMA-operand reads bank-conflict free is
//    applied by permuting each lane's SOURCE address (guide rule 21):
//      - k-contiguous operand: [128 rows][64 k] (128-B rows), 16-B chunk c stored at c ^ ((r>>1)&7),
//        read with ds_read_b128 (lane: row l&15, k chunk l>>4);
//      - mn-contiguous operand: [64 k][128 cols] (256-B rows), chunk c stored at c ^ 2 t(k),
//        t(k) = (k&3) | ((k>>3)&1)<<2, read with two ds_read_b64_tr_b16 per 32-k step (T10);
//  * 8 phases per two K-tiles; phase p: {this phase's LDS reads, one half-tile prefetch,
//    s_barrier, lgkmcnt(0), 16 MFMAs (one 64x32 quadrant x K 64), s_barrier}; the two wave rows run
//    one barrier apart (ping-pong: one issues MFMAs while the other reads LDS); counted
//    vmcnt(6) (three half-tiles in flight across barriers) only in phases 4 and 8, raw s_barrier
//    (never __syncthreads: its fence would drain the DMA), all LDS in one __shared__ array, LDS
//    reads as inline asm (hipcc's waitcnt pass cannot see that they miss the in-flight DMA);
//  * read/restage order (why the schedule is race free): phase 1 reads B0 then A0 of the even
//    buffer and retires the B0 reads (counted lgkmcnt) before its first barrier, phase 2 B1,
//    phase 3 A1, phase 4 nothing; the next tile's images are restaged B0 @2, A0 @3, B1 @4, A1 @5,
//    i.e. >= 2 phases after an image's last read (1 for the early-retired B0), and read >= one
//    phase after the vmcnt that retires them (guide §5 "Read a staged buffer one phase AFTER the
//    wait", with the extra barrier of the staggered wave rows);
//  * workgroup -> tile: XCD-contiguous ranges (T1, bijective) of a grouped order (8 m-tiles x all
//    n-tiles) so one XCD's co-resident tiles share their A / B panels in its L2.
// Range-checked buffer descriptors read rows past K (mn-contiguous operands) as zeros, so the
// weight-gradient form takes any token count; M and N must be multiples of 256.
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace mx {

typedef __bf16 bf16x8_g __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* g8lptr_t;

__device__ __forceinline__ f32x4 g8_mfma(const u16x8& a, const u16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_g, a), __builtin_bit_cast(bf16x8_g, b), c,
                                                 0, 0, 0);
}

constexpr int G8_HT = 16384;        // one half-tile image: 128 rows (cols) x 64 k x bf16
constexpr int G8_TILE = 4 * G8_HT;  // A0 | A1 | B0 | B1
constexpr int G8_BK = 64;

// image row r' (k-contiguous) / image column (mn-contiguous) -> row / column of the 256 tile
__device__ __forceinline__ int g8_map_b(int r, int h) { return (r >> 5) * 64 + h * 32 + (r & 31); }
__device__ __forceinline__ int g8_map_a(int r, int h) { return (r >> 6) * 128 + h * 64 + (r & 63); }

// ---- fused epilogues (forward projections, B = the weight [N][K], bf16 output) -----------------
// In the epilogue, lane l of wave (wr, wc) holds, per accumulator block j = 2 jh + jl, the 4
// consecutive VIRTUAL tile columns v = 64 wc + 32 jh + 16 jl + 4 (l >> 4) + [0, 4).  A fused epilogue
// picks which WEIGHT ROW feeds each virtual column (the B images are DMA-loaded from those rows), so
// the two operands of its elementwise op land in the SAME lane and register -- no LDS exchange:
//  G8_EPI_ROPE  (qkv projection, head dim 128: a tile = 2 heads): virtual (wc, jh, jl, q) -> head
//               column d = 32 (wc & 1) + 64 jh + 16 jl + q, so blocks jh = 0 / 1 hold the rotate-half
//               pair (d, d + 64); outputs written HEAD-MAJOR q [B,Hq,S,D], k / v [B,Hkv,S,D] (the
//               layout the attention kernels read; csrc/kernels/rope.hip rope_split, fused away)
//  G8_EPI_SWIGLU (gate-up projection, W = [gate; up], F rows each): tile pn covers gate columns
//               [128 pn, 128 pn + 128) and the same up columns: jh = 0 -> gate row 128 pn + 32 wc +
//               16 jl + q, jh = 1 -> the up row F further; outputs gu [T, 2F] (standard layout, saved
//               for the backward) AND m = silu(g) u [T, F] (elementwise.hip swiglu_fwd, fused away)
//  G8_EPI_SWIGLU_BWD (NN form: the down projection's dX GEMM dm = dy W_down, F = N columns): the
//               lane's 8 dm columns (after the bf16 swap) meet the saved gu [T, 2F] at the same
//               columns -> writes dgu [T, 2F] (and, with ep.m set, the recomputed m = silu(g) u) in
//               place of dm (elementwise.hip swiglu_bwd / swiglu_bwd_m, fused away)
// All round the GEMM result to bf16 first and then apply the exact expression of the kernel they
// replace: bitwise equal to GEMM -> rope_split / swiglu_fwd / swiglu_bwd on the same kernel's output.
constexpr int G8_EPI_NONE = 0, G8_EPI_ROPE = 1, G8_EPI_SWIGLU = 2, G8_EPI_SWIGLU_BWD = 3;

struct G8Epi {
  uint16_t* q;        // ROPE: [B, Hq, S, 128]
  uint16_t* k;        //       [B, Hkv, S, 128]
  uint16_t* v;        //       [B, Hkv, S, 128]
  const float* cosb;  //       [>= S, 64] f32 (host table, mxllm/ops/reference.py rope_tables)
  const float* sinb;
  int S, Hq, Hkv;
  uint16_t* m;        // SWIGLU: [T, F] with row stride ldm (SWIGLU_BWD: optional recomputed m)
  int64_t ldm;
  int F;
  const uint16_t* gu; // SWIGLU_BWD: the forward's [T, 2F] with row stride ldg
  int64_t ldg;
  float* sq;          // plain bf16 beta-0 output: per-tile sum of squares of the stored values
};

// weight row feeding virtual tile column v (0..255) of output tile pn (G8_EPI_SWIGLU: absolute row)
template <int EPI>
__device__ __forceinline__ int g8_epi_row(int v, int pn, int F) {
  if constexpr (EPI == G8_EPI_ROPE) {
    return (v & ~127) + ((v >> 6) & 1) * 32 + ((v >> 5) & 1) * 64 + (v & 31);
  } else if constexpr (EPI == G8_EPI_SWIGLU) {
    return (((v >> 5) & 1) ? F : 0) + 128 * pn + (v >> 6) * 32 + (v & 31);
  } else {
    return v;
  }
}
__device__ __forceinline__ int g8_t(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// per-lane byte offsets of this wave's two LDS-DMA pieces of half-tile image h of one operand
template <bool KC, bool IS_A, int EPI = G8_EPI_NONE>
__device__ __forceinline__ void g8_src_offsets(int w, int lane, int64_t ld, int h, uint32_t (&off)[2], int pn = 0,
                                               int F = 0) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int pc = 2 * w + j;
    if constexpr (KC) {
      const int r = 8 * pc + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int row = IS_A ? g8_map_a(r, h) : g8_epi_row<EPI>(g8_map_b(r, h), pn, F);
      off[j] = (uint32_t)(((int64_t)row * ld + 8 * c) * 2);
    } else {
      const int k = 4 * pc + (lane >> 4);
      const int c = (lane & 15) ^ (2 * g8_t(k));
      const int col = IS_A ? g8_map_a(8 * c, h) : g8_map_b(8 * c, h);
      off[j] = (uint32_t)(((int64_t)k * ld + col) * 2);
    }
  }
}

// lane part of the LDS address of an MFMA-operand read
//  KC: block rows rb.. (rb % 16 == 0, folded into the immediate), k-step s
__device__ __forceinline__ uint32_t g8_kc_lane(int lane, int s) {
  const int i = lane & 15, g = lane >> 4;
  return (uint32_t)(i * 128 + 16 * ((4 * s + g) ^ ((i >> 1) & 7)));
}
//  MN: block columns cb..cb+15 (one base per cb; k-step s and read r are +8192 s + 1024 r)
__device__ __forceinline__ uint32_t g8_mn_lane(int lane, int cb) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int t = q | ((g & 1) << 2);
  return (uint32_t)((8 * g + q) * 256 + 16 * (((cb >> 3) ^ (2 * t)) + (p >> 1)) + 8 * (p & 1));
}

// In-kernel cycle stamps (diagnostic build V & 4; guide §7 "In-kernel stamps"): lane 0 of wave 0
// (wave row 0) and of wave 4 (wave row 1) record s_memtime at kernel start, after the prologue,
// at the top of every K-loop iteration (2 K-tiles) and after the loop / the epilogue, plus
// s_memrealtime at start and end (clock = d memtime / d realtime x 100 MHz).  Written with
// ordinary VECTOR global stores into a buffer nothing else reads; the normal build has none.
// The stamp buffer (1.3 MB of device memory) and the stamped / ablation variants exist only in a
// diagnostic build: MXLLM_FILE_FLAGS="gemm8.hip=-DMXLLM_GEMM8_DIAG" python -m mxllm._build.
constexpr int G8_NST = 80;
#ifdef MXLLM_GEMM8_DIAG
__device__ unsigned long long g8_stamps[1024 * 2 * G8_NST];
__device__ __forceinline__ void g8_stamp(int wg, int row, int k, unsigned long long v) {
  if (wg < 1024 && k < G8_NST) g8_stamps[((size_t)wg * 2 + row) * G8_NST + k] = v;
}
#else
__device__ __forceinline__ void g8_stamp(int, int, int, unsigned long long) {}
#endif

// sum of squares of the 8 bf16 values packed in `o` (what the plain epilogue stored), added to s
__device__ __forceinline__ float g8_sq8(const uint4& o, float s) {
  const uint32_t v[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(v[i] << 16), hi = __uint_as_float(v[i] & 0xffff0000u);
    s = __builtin_fmaf(lo, lo, s);
    s = __builtin_fmaf(hi, hi, s);
  }
  return s;
}
__device__ __forceinline__ float g8_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float g8_rbf(float x) { return bf2f(f2bf(x)); }  // round through bf16

// 16-B store of blocks (jl = 0, 1) of one jh: lanes l, l + 16 swap packed pairs (permlane16_swap) so
// every lane owns 8 consecutive columns (see the plain bf16 epilogue); `dst` = this lane's 8 columns
__device__ __forceinline__ void g8_store8(uint16_t* dst, const f32x4& va, const f32x4& vb) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[0], va[1]), pack_bf16x2(vb[0], vb[1]), false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[2], va[3]), pack_bf16x2(vb[2], vb[3]), false, false);
  uint4 o;
  o.x = s0[0];
  o.y = s1[0];
  o.z = s0[1];
  o.w = s1[1];
  *reinterpret_cast<uint4*>(dst) = o;
}

template <int EPI>
__device__ __forceinline__ void g8_epilogue_fused(f32x4 (&acc)[8][4], float alpha, int ml, int pn, int wc, int lane,
                                                  int N, const G8Epi& ep, void* C, int64_t ldc) {
  // this lane's 8 stored columns start at offset u8 inside a 32-column group (after the swap)
  const int u8 = 16 * ((lane >> 4) & 1) + 8 * (lane >> 5);
  if constexpr (EPI == G8_EPI_ROPE) {
    const int head = pn * 2 + (wc >> 1);  // 128-column heads: two per tile
    uint16_t* dst;
    int Hd, hh;
    if (head < ep.Hq) {
      dst = ep.q, Hd = ep.Hq, hh = head;
    } else if (head < ep.Hq + ep.Hkv) {
      dst = ep.k, Hd = ep.Hkv, hh = head - ep.Hq;
    } else {
      dst = ep.v, Hd = ep.Hkv, hh = head - ep.Hq - ep.Hkv;
    }
    const bool rot = head < ep.Hq + ep.Hkv;
    const int d0 = 32 * (wc & 1);  // head column of block (jh 0, jl 0, lane group 0)
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = ml + qa * 64 + 16 * i;
        const int b = m / ep.S, sq = m - b * ep.S;
        f32x4 x0[2], x1[2];  // [jl]: head columns d (jh 0) and d + 64 (jh 1)
#pragma unroll
        for (int jl = 0; jl < 2; ++jl) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            x0[jl][c] = g8_rbf(acc[4 * qa + i][jl][c] * alpha);
            x1[jl][c] = g8_rbf(acc[4 * qa + i][2 + jl][c] * alpha);
          }
        }
        if (rot) {
#pragma unroll
          for (int jl = 0; jl < 2; ++jl) {
            const int f = d0 + 16 * jl + 4 * (lane >> 4);  // frequency index of x0[jl][0]
            const f32x4 cs = *reinterpret_cast<const f32x4*>(ep.cosb + (int64_t)sq * 64 + f);
            const f32x4 sn = *reinterpret_cast<const f32x4*>(ep.sinb + (int64_t)sq * 64 + f);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float a = x0[jl][c], bb = x1[jl][c];
              x0[jl][c] = rope_lo(a, bb, cs[c], sn[c]);
              x1[jl][c] = rope_hi(a, bb, cs[c], sn[c]);
            }
          }
        }
        uint16_t* row = dst + (((int64_t)b * Hd + hh) * ep.S + sq) * 128;
        g8_store8(row + d0 + u8, x0[0], x0[1]);
        g8_store8(row + d0 + 64 + u8, x1[0], x1[1]);
      }
  } else if constexpr (EPI == G8_EPI_SWIGLU_BWD) {
    const int F = N;
    const int cb = 256 * pn + 64 * wc + 16 * ((lane >> 4) & 1) + 8 * (lane >> 5);  // + 32 jp
#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      // all 16 gu loads of this half first (64 VGPRs): one memory round trip per half, not per row
      u16x8 g8[4][2], u8v[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint16_t* gr = ep.gu + (int64_t)(ml + qa * 64 + 16 * i) * ep.ldg;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          g8[i][jp] = *reinterpret_cast<const u16x8*>(gr + cb + 32 * jp);
          u8v[i][jp] = *reinterpret_cast<const u16x8*>(gr + F + cb + 32 * jp);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = ml + qa * 64 + 16 * i;
        u16x8 d8[2];
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {  // dm rounded to bf16 and swapped exactly as the plain store
          const f32x4 va = acc[4 * qa + i][2 * jp] * alpha, vb = acc[4 * qa + i][2 * jp + 1] * alpha;
          const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[0], va[1]), pack_bf16x2(vb[0], vb[1]),
                                                          false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[2], va[3]), pack_bf16x2(vb[2], vb[3]),
                                                          false, false);
          uint4 o;
          o.x = s0[0];
          o.y = s1[0];
          o.z = s0[1];
          o.w = s1[1];
          d8[jp] = __builtin_bit_cast(u16x8, o);
        }
        uint16_t* dr = reinterpret_cast<uint16_t*>(C) + m * ldc;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          u16x8 og, ou;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float dg, du;
            swiglu_grad(bf2f(d8[jp][j]), bf2f(g8[i][jp][j]), bf2f(u8v[i][jp][j]), dg, du);
            og[j] = f2bf(dg);
            ou[j] = f2bf(du);
          }
          *reinterpret_cast<u16x8*>(dr + cb + 32 * jp) = og;
          *reinterpret_cast<u16x8*>(dr + F + cb + 32 * jp) = ou;
          if (ep.m) {
            u16x8 om;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float gf = bf2f(g8[i][jp][j]);
              om[j] = f2bf(gf * __builtin_amdgcn_rcpf(1.f + __expf(-gf)) * bf2f(u8v[i][jp][j]));
            }
            *reinterpret_cast<u16x8*>(ep.m + m * ep.ldm + cb + 32 * jp) = om;
          }
        }
      }
    }
  } else {  // G8_EPI_SWIGLU
    const int F = N / 2;
    const int col = 128 * pn + 32 * wc + u8;  // gate column (up: + F; m: the same column)
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = ml + qa * 64 + 16 * i;
        f32x4 g[2], u[2], mm[2];
#pragma unroll
        for (int jl = 0; jl < 2; ++jl)
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            g[jl][c] = g8_rbf(acc[4 * qa + i][jl][c] * alpha);
            u[jl][c] = g8_rbf(acc[4 * qa + i][2 + jl][c] * alpha);
            mm[jl][c] = g[jl][c] * g8_sigmoid(g[jl][c]) * u[jl][c];
          }
        uint16_t* gu = reinterpret_cast<uint16_t*>(C) + m * ldc;
        g8_store8(gu + col, g[0], g[1]);
        g8_store8(gu + F + col, u[0], u[1]);
        g8_store8(ep.m + m * ep.ldm + col, mm[0], mm[1]);
      }
  }
}

// V != 0: timing-only ablation builds (bench/gemm8_probe.py --ablate; results are WRONG):
//   V & 1: every phase issues its 16 MFMAs twice (MFMA time per barrier doubled)
//   V & 2: no barriers in the K loop and no wave-row stagger (no LDS ordering at all)
//   V & 4: stamps only (results correct)
// PH = 4: the same images and registers on a 4-phase schedule (two quadrants = 32 MFMAs per phase,
// half the barriers; every phase retires its LDS reads before its first barrier so each image is
// restaged one phase after its last read; two half-tiles in flight across barriers, vmcnt(4))
template <bool A_KC, bool B_KC, bool OUT_F32, bool BETA, int V = 0, int PH = 8, int EPI = G8_EPI_NONE>
__global__ void __launch_bounds__(512, 1)
gemm8_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
             void* __restrict__ C, int64_t ldc, int M, int N, int K, const float* __restrict__ alpha_t,
             float alpha_f, int k0 = 0, int64_t cpart = 0, G8Epi ep = G8Epi{}) {
  static_assert(EPI == G8_EPI_NONE || (!OUT_F32 && !BETA && (EPI == G8_EPI_SWIGLU_BWD ? A_KC && !B_KC : B_KC)),
                "fused epilogues: bf16, beta 0; TN-form forwards, NN-form SwiGLU backward");
  // K split in two (gridDim.y == 2, k0 = K of part 0): part 1 covers K rows / columns k0 .. K-1 of
  // both operands and writes its own output image C + cpart (mx_gemm8_tail: the last, partial wave
  // of tiles of a GEMM runs as twice as many half-K workgroups; the images are summed after)
  if (gridDim.y > 1) {
    const int kp = blockIdx.y;
    const int64_t koff = kp ? k0 : 0;
    A += A_KC ? koff : koff * lda;
    B += B_KC ? koff : koff * ldb;
    if (kp) C = reinterpret_cast<char*>(C) + cpart * (OUT_F32 ? 4 : 2);
    K = kp ? K - k0 : k0;
  }
  // ONE __shared__ array (a second LDS object makes hipcc drain vmcnt before LDS reads: guide §5 item 4a)
  __shared__ __attribute__((aligned(1024))) char smem[2 * G8_TILE];
  const int nM = M >> 8, nN = N >> 8;
  int pm, pn;
  {
    const int L = xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = 8;
    const int per = GM * nN, grp = L / per, first = grp * GM;
    const int rows = min(GM, nM - first), in = L - grp * per;
    pm = first + in % rows;
    pn = in / rows;
  }
  const int m0 = pm << 8, n0 = pn << 8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int nk = (K + G8_BK - 1) / G8_BK;
  constexpr bool ST = (V & 4) != 0;
  const bool stw = ST && (tid == 0 || tid == 256);  // lane 0 of waves 0 and 4
  const int strow = tid >= 256;
  int sti = 0;
  if constexpr (ST) {
    if (stw) {
      g8_stamp(blockIdx.x, strow, sti++, __builtin_amdgcn_s_memtime());
      g8_stamp(blockIdx.x, strow, sti++, __builtin_amdgcn_s_memrealtime());
    }
  }

  // ---- operand descriptors (range-checked: mn-contiguous rows past K read as zeros)
  const uint16_t* abase = A_KC ? A + (int64_t)m0 * lda : A + m0;
  // SWIGLU: gate and up rows are F apart -> absolute weight rows off the start of B
  const uint16_t* bbase = B_KC ? B + (int64_t)(EPI == G8_EPI_SWIGLU ? 0 : n0) * ldb : B + n0;
  const uint32_t arec = A_KC ? (uint32_t)((255 * lda + (int64_t)nk * G8_BK) * 2) : (uint32_t)(((int64_t)K * lda - m0) * 2);
  const uint32_t brec = EPI == G8_EPI_SWIGLU ? (uint32_t)(((int64_t)(N - 1) * ldb + (int64_t)nk * G8_BK) * 2)
                        : B_KC ? (uint32_t)((255 * ldb + (int64_t)nk * G8_BK) * 2)
                               : (uint32_t)(((int64_t)K * ldb - n0) * 2);
  const __amdgpu_buffer_rsrc_t ars = __builtin_amdgcn_make_buffer_rsrc((void*)abase, 0, arec, 0x00020000);
  const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc((void*)bbase, 0, brec, 0x00020000);
  const uint32_t astep = A_KC ? G8_BK * 2 : (uint32_t)(G8_BK * lda * 2);  // bytes per K-tile
  const uint32_t bstep = B_KC ? G8_BK * 2 : (uint32_t)(G8_BK * ldb * 2);
  uint32_t aoff[2][2], boff[2][2];
  g8_src_offsets<A_KC, true>(w, lane, lda, 0, aoff[0]);
  g8_src_offsets<A_KC, true>(w, lane, lda, 1, aoff[1]);
  g8_src_offsets<B_KC, false, EPI>(w, lane, ldb, 0, boff[0], pn, N / 2);
  g8_src_offsets<B_KC, false, EPI>(w, lane, ldb, 1, boff[1], pn, N / 2);

  // issue half-tile image `img` (0 A0, 1 A1, 2 B0, 3 B1) of K-tile kt into buffer kt & 1
  auto issue = [&](int kt, int img) __attribute__((always_inline)) {
    char* dst = smem + (kt & 1) * G8_TILE + img * G8_HT + (2 * w) * 1024;
    // the K-tile offset rides in voffset: the range check covers voffset + immediate only
    if (img < 2) {
      const uint32_t so = (uint32_t)kt * astep;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (g8lptr_t)dst, 16, aoff[img][0] + so, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (g8lptr_t)(dst + 1024), 16, aoff[img][1] + so, 0, 0, 0);
    } else {
      const uint32_t so = (uint32_t)kt * bstep;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (g8lptr_t)dst, 16, boff[img - 2][0] + so, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (g8lptr_t)(dst + 1024), 16, boff[img - 2][1] + so, 0, 0, 0);
    }
  };

  // ---- LDS read bases (lane parts; + buffer / image offsets at the read)
  const uint32_t lds0 = lds_addr(smem);
  uint32_t akc[2], amn[4], bmn[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) akc[s] = g8_kc_lane(lane, s);
#pragma unroll
  for (int i = 0; i < 4; ++i) amn[i] = g8_mn_lane(lane, wr * 64 + 16 * i);
#pragma unroll
  for (int j = 0; j < 2; ++j) bmn[j] = g8_mn_lane(lane, wc * 32 + 16 * j);

  u16x8 fa[4][2], fb0[2][2], fb1[2][2];  // [block][k-step]
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // A image `img` (0/1) of buffer `buf` -> fa;  KC: ds_read_b128, MN: 2 x ds_read_b64_tr_b16 per block and k-step
  auto read_a = [&](int buf, int img) __attribute__((always_inline)) {
    const uint32_t ib = lds0 + buf * G8_TILE + img * G8_HT;
    if constexpr (A_KC) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t b = ib + akc[s];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i][s] = rd128_off(b, (wr * 64 + 16 * i) * 128);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t b = ib + amn[i];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const u16x4 lo = trd_off(b, 8192 * s), hi = trd_off(b, 8192 * s + 1024);
          fa[i][s] = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
    }
  };
  auto read_b = [&](int buf, int img, u16x8(&fb)[2][2]) __attribute__((always_inline)) {
    const uint32_t ib = lds0 + buf * G8_TILE + (2 + img) * G8_HT;
    if constexpr (B_KC) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t b = ib + akc[s];
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j][s] = rd128_off(b, (wc * 32 + 16 * j) * 128);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t b = ib + bmn[j];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const u16x4 lo = trd_off(b, 8192 * s), hi = trd_off(b, 8192 * s + 1024);
          fb[j][s] = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
    }
  };
  auto pin_a = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pin(fa[i][0]);
      pin(fa[i][1]);
    }
  };
  auto pin_b = [&](u16x8(&fb)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pin(fb[j][0]);
      pin(fb[j][1]);
    }
  };
  // quadrant (a, b): 16 MFMAs; swapped operands -> acc holds C^T blocks (4 consecutive columns per lane)
  auto mma = [&](int qa, int qb, u16x8(&fb)[2][2]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 * qa + i][2 * qb + j] = g8_mfma(fb[j][s], fa[i][s], acc[4 * qa + i][2 * qb + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  constexpr int NA = A_KC ? 8 : 16;  // LDS reads of one A image
  auto vm6 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); };
  auto vm0 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  auto vm4 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); };
  // ---- prologue: K-tile 0 (all four images) + K-tile 1's B0, A0, B1 (PH 4: B0, B1); retire tile 0
  issue(0, 2);
  issue(0, 0);
  issue(0, 3);
  issue(0, 1);
  if (nk > 1) {
    issue(1, 2);
    if constexpr (PH == 8) issue(1, 0);
    issue(1, 3);
    if constexpr (PH == 8) vm6(); else vm4();
  } else {
    vm0();
  }
  __builtin_amdgcn_s_barrier();
  if (!(V & 2) && wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
  if constexpr (ST) {
    if (stw) g8_stamp(blockIdx.x, strow, sti++, __builtin_amdgcn_s_memtime());
  }

  // one phase: reads -> prefetch -> [wait] -> barrier -> lgkmcnt(0) -> MFMA -> barrier
#define G8_SYNC_MMA(QA, QB, FB)                   \
  if constexpr (!(V & 2)) __builtin_amdgcn_s_barrier(); \
  lds_wait();                                     \
  pin_a();                                        \
  pin_b(FB);                                      \
  mma(QA, QB, FB);                                \
  if constexpr (V & 1) mma(QA, QB, FB);           \
  if constexpr (!(V & 2)) __builtin_amdgcn_s_barrier();

  if constexpr (PH == 4) {
#define G8_SYNC_MMA2(QA, QB0, FB0, QB1, FB1)              \
  __builtin_amdgcn_s_barrier();                           \
  pin_a();                                                \
  pin_b(FB0);                                             \
  pin_b(FB1);                                             \
  mma(QA, QB0, FB0);                                      \
  mma(QA, QB1, FB1);                                      \
  __builtin_amdgcn_s_barrier();
    for (int kt = 0;; kt += 2) {
      if constexpr (ST) {
        if (stw) g8_stamp(blockIdx.x, strow, sti++, __builtin_amdgcn_s_memtime());
      }
      // phase 1: buffer 0 (tile kt) B0, B1, A0; tile kt + 1's A0, A1 -> buffer 1
      read_b(0, 0, fb0);
      read_b(0, 1, fb1);
      read_a(0, 0);
      if (kt + 1 < nk) {
        issue(kt + 1, 0);
        issue(kt + 1, 1);
      }
      lds_wait();  // retired before the barrier: these images are restageable next phase
      G8_SYNC_MMA2(0, 0, fb0, 1, fb1)
      // phase 2: buffer 0 A1; tile kt + 2's B0, B1 -> buffer 0; retire tile kt + 1
      read_a(0, 1);
      if (kt + 2 < nk) {
        issue(kt + 2, 2);
        issue(kt + 2, 3);
        vm4();
      } else {
        vm0();
      }
      lds_wait();
      G8_SYNC_MMA2(1, 1, fb1, 0, fb0)
      if (kt + 1 >= nk) break;
      // phase 3: buffer 1 (tile kt + 1) B0, B1, A0; tile kt + 2's A0, A1 -> buffer 0
      read_b(1, 0, fb0);
      read_b(1, 1, fb1);
      read_a(1, 0);
      if (kt + 2 < nk) {
        issue(kt + 2, 0);
        issue(kt + 2, 1);
      }
      lds_wait();
      G8_SYNC_MMA2(0, 0, fb0, 1, fb1)
      // phase 4: buffer 1 A1; tile kt + 3's B0, B1 -> buffer 1; retire tile kt + 2
      read_a(1, 1);
      if (kt + 3 < nk) {
        issue(kt + 3, 2);
        issue(kt + 3, 3);
        vm4();
      } else {
        vm0();
      }
      lds_wait();
      G8_SYNC_MMA2(1, 1, fb1, 0, fb0)
      if (kt + 2 >= nk) break;
    }
#undef G8_SYNC_MMA2
  } else
  for (int kt = 0;; kt += 2) {
    if constexpr (ST) {
      if (stw) g8_stamp(blockIdx.x, strow, sti++, __builtin_amdgcn_s_memtime());
    }
    // phases 1-4: tile kt in buffer 0
    read_b(0, 0, fb0);
    read_a(0, 0);
    if (kt + 1 < nk) issue(kt + 1, 1);
    lds_wait_le(NA < 15 ? NA : 15);  // B0 reads retired before the barrier: B0 restageable in phase 2
    G8_SYNC_MMA(0, 0, fb0)
    read_b(0, 1, fb1);
    if (kt + 2 < nk) issue(kt + 2, 2);
    G8_SYNC_MMA(0, 1, fb1)
    read_a(0, 1);
    if (kt + 2 < nk) issue(kt + 2, 0);
    G8_SYNC_MMA(1, 1, fb1)
    if (kt + 2 < nk) {
      issue(kt + 2, 3);
      vm6();
    } else {
      vm0();
    }
    G8_SYNC_MMA(1, 0, fb0)
    if (kt + 1 >= nk) break;
    // phases 5-8: tile kt + 1 in buffer 1
    read_b(1, 0, fb0);
    read_a(1, 0);
    if (kt + 2 < nk) issue(kt + 2, 1);
    lds_wait_le(NA < 15 ? NA : 15);
    G8_SYNC_MMA(0, 0, fb0)
    read_b(1, 1, fb1);
    if (kt + 3 < nk) issue(kt + 3, 2);
    G8_SYNC_MMA(0, 1, fb1)
    read_a(1, 1);
    if (kt + 3 < nk) issue(kt + 3, 0);
    G8_SYNC_MMA(1, 1, fb1)
    if (kt + 3 < nk) {
      issue(kt + 3, 3);
      vm6();
    } else {
      vm0();
    }
    G8_SYNC_MMA(1, 0, fb0)
    if (kt + 2 >= nk) break;
  }
#undef G8_SYNC_MMA
  if (!(V & 2) && wr == 0) __builtin_amdgcn_s_barrier();  // match the stagger barrier
  if constexpr (ST) {
    if (stw) g8_stamp(blockIdx.x, strow, G8_NST - 3, __builtin_amdgcn_s_memtime());
  }

  // ---- epilogue: lane holds C[m][n .. n+3] per block
  const float alpha = alpha_f * (alpha_t ? alpha_t[0] : 1.f);
  float sqs = 0.f;  // ep.sq: this lane's sum of squares of the bf16 values it stores
  const int ml = m0 + wr * 128 + (lane & 15);
  const int nl = n0 + wc * 64 + 4 * (lane >> 4);
  if constexpr (EPI != G8_EPI_NONE) {
    g8_epilogue_fused<EPI>(acc, alpha, ml, pn, wc, lane, N, ep, C, ldc);
    return;
  }
#pragma unroll
  for (int qa = 0; qa < 2; ++qa) {
    f32x4 old[4][4];
    if constexpr (BETA) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t m = ml + qa * 64 + 16 * i;
          const int n = nl + 32 * (j >> 1) + 16 * (j & 1);
          if constexpr (OUT_F32) {
            old[i][j] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(C) + m * ldc + n);
          } else {
            const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(C) + m * ldc + n);
            old[i][j] = f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                              __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
          }
        }
    }
    if constexpr (OUT_F32) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t m = ml + qa * 64 + 16 * i;
          const int n = nl + 32 * (j >> 1) + 16 * (j & 1);
          f32x4 v = acc[4 * qa + i][j] * alpha;
          if constexpr (BETA) v += old[i][j];
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + m * ldc + n) = v;
        }
    } else {
      // bf16: blocks j, j + 1 are 16 columns apart and lanes l, l + 16 hold adjacent 4-column groups
      // of one row, so one v_permlane16_swap per packed dword pair gives every lane 8 consecutive
      // columns -> ONE 16-B store per block pair (guide T21, with the 16-lane swap) instead of two 8-B
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          f32x4 va = acc[4 * qa + i][2 * jp] * alpha, vb = acc[4 * qa + i][2 * jp + 1] * alpha;
          if constexpr (BETA) {
            va += old[i][2 * jp];
            vb += old[i][2 * jp + 1];
          }
          const auto s0 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[0], va[1]), pack_bf16x2(vb[0], vb[1]),
                                                          false, false);
          const auto s1 = __builtin_amdgcn_permlane16_swap(pack_bf16x2(va[2], va[3]), pack_bf16x2(vb[2], vb[3]),
                                                          false, false);
          const int64_t m = ml + qa * 64 + 16 * i;
          const int n = n0 + wc * 64 + 32 * jp + 16 * ((lane >> 4) & 1) + 8 * (lane >> 5);
          uint4 o;
          o.x = s0[0];
          o.y = s1[0];
          o.z = s0[1];
          o.w = s1[1];
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(C) + m * ldc + n) = o;
          if (!BETA && ep.sq) sqs = g8_sq8(o, sqs);
        }
    }
  }
  if constexpr (!OUT_F32 && !BETA) {
    if (ep.sq) {  // workgroup-uniform: one fixed-order partial per output tile (deterministic)
      sqs = wave_sum(sqs);
      __syncthreads();  // every wave is past the K loop's LDS reads (its DMA drained at the last tile)
      float* red = reinterpret_cast<float*>(smem);
      if (lane == 0) red[w] = sqs;
      __syncthreads();
      if (tid == 0) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) t += red[i];
        ep.sq[pm * nN + pn] = t;
      }
    }
  }
  if constexpr (ST) {
    if (stw) {
      g8_stamp(blockIdx.x, strow, G8_NST - 2, __builtin_amdgcn_s_memtime());
      g8_stamp(blockIdx.x, strow, G8_NST - 1, __builtin_amdgcn_s_memrealtime());
    }
  }
}

// lane id regenerated on demand (volatile asm: never hoisted, so it is not a register that must
// survive the persistent kernel's tile loop)
__device__ __forceinline__ int g8_lane() {
  int ln;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
  return ln;
}

// ---------------------------------------------------------------------------------------------
// Persistent 4-phase variant: min(tiles, CUs) workgroups, each walking output
// tiles t = L, L + G, ... (L = the XCD-contiguous remap of its id, so the G tiles in flight at a
// time form 8 contiguous ranges, one per XCD / L2).  Between two tiles the NEXT tile's prologue
// DMA (K-tile 0 and K-tile 1's B images) is issued BEFORE the current tile's epilogue stores, so
// its latency runs under the stores, and the wait for it counts the stores as still in flight
// (loads, stores and LDS-DMA retire in issue order): the stores never block the next tile's K loop.
// No workgroup launch / drain between tiles.  K loop, images, swizzles and schedule: the PH = 4
// path of gemm8_kernel above.
template <bool A_KC, bool B_KC, bool OUT_F32, bool BETA>
__global__ void __launch_bounds__(512, 1)
gemm8p_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb,
              void* __restrict__ C, int64_t ldc, int M, int N, int K, const float* __restrict__ alpha_t,
              float alpha_f) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * G8_TILE];
  const int nM = M >> 8, nN = N >> 8, tiles = nM * nN, G = gridDim.x;
  int L = xcd_remap(blockIdx.x, G);
  if (L >= tiles) return;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int nk = (K + G8_BK - 1) / G8_BK;
  const float alpha = alpha_f * (alpha_t ? alpha_t[0] : 1.f);

  auto tile_of = [&](int l, int& pm, int& pn) __attribute__((always_inline)) {
    constexpr int GM = 8;
    const int per = GM * nN, grp = l / per, first = grp * GM;
    const int rows = min(GM, nM - first), in = l - grp * per;
    pm = first + in % rows;
    pn = in / rows;
  };
  int pm, pn;
  tile_of(L, pm, pn);
  int m0 = pm << 8, n0 = pn << 8;
  const uint32_t arec = A_KC ? (uint32_t)((255 * lda + (int64_t)nk * G8_BK) * 2) : (uint32_t)(((int64_t)K * lda - m0) * 2);
  const uint32_t brec = B_KC ? (uint32_t)((255 * ldb + (int64_t)nk * G8_BK) * 2) : (uint32_t)(((int64_t)K * ldb - n0) * 2);
  // mn-contiguous operands: the record limit depends on the tile's column offset (rows past K -> 0)
  auto rsrc_a = [&](int mm0) __attribute__((always_inline)) {
    const uint16_t* base = A_KC ? A + (int64_t)mm0 * lda : A + mm0;
    const uint32_t rec = A_KC ? arec : (uint32_t)(((int64_t)K * lda - mm0) * 2);
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, rec, 0x00020000);
  };
  auto rsrc_b = [&](int nn0) __attribute__((always_inline)) {
    const uint16_t* base = B_KC ? B + (int64_t)nn0 * ldb : B + nn0;
    const uint32_t rec = B_KC ? brec : (uint32_t)(((int64_t)K * ldb - nn0) * 2);
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, rec, 0x00020000);
  };
  __amdgpu_buffer_rsrc_t ars = rsrc_a(m0), brs = rsrc_b(n0);
  const uint32_t astep = A_KC ? G8_BK * 2 : (uint32_t)(G8_BK * lda * 2);
  const uint32_t bstep = B_KC ? G8_BK * 2 : (uint32_t)(G8_BK * ldb * 2);
  // lane-derived addresses are recomputed per tile from an opaque copy of the lane id (hipcc cannot
  // hoist them out of the tile loop): they are not live across the epilogue, whose fp32 / beta
  // forms otherwise spill at the 256-VGPR budget of two waves per SIMD
  uint32_t aoff[2][2], boff[2][2];
  auto offsets = [&]() __attribute__((always_inline)) {
    const int ln = g8_lane();
    g8_src_offsets<A_KC, true>(w, ln, lda, 0, aoff[0]);
    g8_src_offsets<A_KC, true>(w, ln, lda, 1, aoff[1]);
    g8_src_offsets<B_KC, false>(w, ln, ldb, 0, boff[0]);
    g8_src_offsets<B_KC, false>(w, ln, ldb, 1, boff[1]);
  };
  offsets();
  auto issue = [&](int kt, int img) __attribute__((always_inline)) {
    char* dst = smem + (kt & 1) * G8_TILE + img * G8_HT + (2 * w) * 1024;
    if (img < 2) {
      const uint32_t so = (uint32_t)kt * astep;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (g8lptr_t)dst, 16, aoff[img][0] + so, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ars, (g8lptr_t)(dst + 1024), 16, aoff[img][1] + so, 0, 0, 0);
    } else {
      const uint32_t so = (uint32_t)kt * bstep;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (g8lptr_t)dst, 16, boff[img - 2][0] + so, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(brs, (g8lptr_t)(dst + 1024), 16, boff[img - 2][1] + so, 0, 0, 0);
    }
  };
  // the prologue DMA of a tile: K-tile 0 (4 images) + K-tile 1's B images
  auto prologue = [&]() __attribute__((always_inline)) {
    issue(0, 2);
    issue(0, 0);
    issue(0, 3);
    issue(0, 1);
    if (nk > 1) {
      issue(1, 2);
      issue(1, 3);
    }
  };

  const uint32_t lds0 = lds_addr(smem);
  uint32_t akc[2], amn[4], bmn[2];
  auto lds_lanes = [&]() __attribute__((always_inline)) {
    const int ln = g8_lane();
#pragma unroll
    for (int s = 0; s < 2; ++s) akc[s] = g8_kc_lane(ln, s);
#pragma unroll
    for (int i = 0; i < 4; ++i) amn[i] = g8_mn_lane(ln, wr * 64 + 16 * i);
#pragma unroll
    for (int j = 0; j < 2; ++j) bmn[j] = g8_mn_lane(ln, wc * 32 + 16 * j);
  };
  u16x8 fa[4][2], fb0[2][2], fb1[2][2];
  f32x4 acc[8][4];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto read_a = [&](int buf, int img) __attribute__((always_inline)) {
    const uint32_t ib = lds0 + buf * G8_TILE + img * G8_HT;
    if constexpr (A_KC) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t b = ib + akc[s];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i][s] = rd128_off(b, (wr * 64 + 16 * i) * 128);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t b = ib + amn[i];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const u16x4 lo = trd_off(b, 8192 * s), hi = trd_off(b, 8192 * s + 1024);
          fa[i][s] = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
    }
  };
  auto read_b = [&](int buf, int img, u16x8(&fb)[2][2]) __attribute__((always_inline)) {
    const uint32_t ib = lds0 + buf * G8_TILE + (2 + img) * G8_HT;
    if constexpr (B_KC) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint32_t b = ib + akc[s];
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j][s] = rd128_off(b, (wc * 32 + 16 * j) * 128);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t b = ib + bmn[j];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const u16x4 lo = trd_off(b, 8192 * s), hi = trd_off(b, 8192 * s + 1024);
          fb[j][s] = u16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
    }
  };
  auto pin_a = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pin(fa[i][0]);
      pin(fa[i][1]);
    }
  };
  auto pin_b = [&](u16x8(&fb)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pin(fb[j][0]);
      pin(fb[j][1]);
    }
  };
  auto mma = [&](int qa, int qb, u16x8(&fb)[2][2]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[4 * qa + i][2 * qb + j] = g8_mfma(fb[j][s], fa[i][s], acc[4 * qa + i][2 * qb + j]);
    __builtin_amdgcn_s_setprio(0);
  };
  auto vm4 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); };
  auto vm0 = []() __attribute__((always_inline)) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
#define G8P_SYNC_MMA2(QA, QB0, FB0, QB1, FB1) \
  __builtin_amdgcn_s_barrier();               \
  pin_a();                                    \
  pin_b(FB0);                                 \
  pin_b(FB1);                                 \
  mma(QA, QB0, FB0);                          \
  mma(QA, QB1, FB1);                          \
  __builtin_amdgcn_s_barrier();

  zero_acc();
  prologue();
  // stores of the previous tile issued after this tile's prologue DMA (0 for the first tile): the
  // in-order wait for K-tile 0 leaves them (and K-tile 1's B images) in flight
  bool stores_pending = false;
  for (;;) {
    if (stores_pending) {
      if (nk > 1) {
        if constexpr (OUT_F32) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");  // 4 DMA + 32 stores
        else asm volatile("s_waitcnt vmcnt(20)" ::: "memory");                    // 4 DMA + 16 stores
      } else {
        if constexpr (OUT_F32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      }
    } else {
      if (nk > 1) vm4(); else vm0();
    }
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier
    lds_lanes();
    offsets();
    for (int kt = 0;; kt += 2) {
      read_b(0, 0, fb0);
      read_b(0, 1, fb1);
      read_a(0, 0);
      if (kt + 1 < nk) {
        issue(kt + 1, 0);
        issue(kt + 1, 1);
      }
      lds_wait();
      G8P_SYNC_MMA2(0, 0, fb0, 1, fb1)
      read_a(0, 1);
      if (kt + 2 < nk) {
        issue(kt + 2, 2);
        issue(kt + 2, 3);
        vm4();
      } else {
        vm0();
      }
      lds_wait();
      G8P_SYNC_MMA2(1, 1, fb1, 0, fb0)
      if (kt + 1 >= nk) break;
      read_b(1, 0, fb0);
      read_b(1, 1, fb1);
      read_a(1, 0);
      if (kt + 2 < nk) {
        issue(kt + 2, 0);
        issue(kt + 2, 1);
      }
      lds_wait();
      G8P_SYNC_MMA2(0, 0, fb0, 1, fb1)
      read_a(1, 1);
      if (kt + 3 < nk) {
        issue(kt + 3, 2);
        issue(kt + 3, 3);
        vm4();
      } else {
        vm0();
      }
      lds_wait();
      G8P_SYNC_MMA2(1, 1, fb1, 0, fb0)
      if (kt + 2 >= nk) break;
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // match the stagger: every wave's LDS reads are done
    // ---- next tile's prologue DMA first (LDS is free), then this tile's epilogue
    const int cm0 = m0, cn0 = n0;
    const int Ln = L + G;
    const bool more = Ln < tiles;
    if (more) {
      tile_of(Ln, pm, pn);
      m0 = pm << 8;
      n0 = pn << 8;
      ars = rsrc_a(m0);
      brs = rsrc_b(n0);
      offsets();
      prologue();
    }
    const int ln = g8_lane();
    const int ml = cm0 + wr * 128 + (ln & 15);
    const int nl = cn0 + wc * 64 + 4 * (ln >> 4);
#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      f32x4 old[4][4];
      if constexpr (BETA) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t m = ml + qa * 64 + 16 * i;
            const int n = nl + 32 * (j >> 1) + 16 * (j & 1);
            if constexpr (OUT_F32) {
              old[i][j] = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(C) + m * ldc + n);
            } else {
              const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(C) + m * ldc + n);
              old[i][j] = f32x4{__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                                __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
            }
          }
      }
      if constexpr (OUT_F32) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int64_t m = ml + qa * 64 + 16 * i;
            const int n = nl + 32 * (j >> 1) + 16 * (j & 1);
            f32x4 v = acc[4 * qa + i][j] * alpha;
            if constexpr (BETA) v += old[i][j];
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + m * ldc + n) = v;
          }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            f32x4 va = acc[4 * qa + i][2 * jp] * alpha, vb = acc[4 * qa + i][2 * jp + 1] * alpha;
            if constexpr (BETA) {
              va += old[i][2 * jp];
              vb += old[i][2 * jp + 1];
            }
            const int64_t m = ml + qa * 64 + 16 * i;
            const int n = cn0 + wc * 64 + 32 * jp + 16 * ((ln >> 4) & 1) + 8 * (ln >> 5);
            g8_store8(reinterpret_cast<uint16_t*>(C) + m * ldc + n, va, vb);
          }
      }
    }
    if (!more) break;
    zero_acc();
    L = Ln;
    stores_pending = !BETA;  // with BETA the epilogue's loads already drained the DMA (in-order waits)
  }
#undef G8P_SYNC_MMA2
}

}  // namespace mx

using namespace mx;

// compute units of the current device (the persistent grid: one workgroup per CU)
static int g8_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t p;
    n = hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0 ? p.multiProcessorCount : 256;
  }
  return n;
}

// C[M, N] = alpha * op(A) op(B) + beta * C.  a_kc: A stored [M][K] (else [K][M]); b_kc: B stored [N][K]
// (else [K][N]); row strides in elements.  Takes M, N multiples of 256; K a multiple of 64 when an
// operand is k-contiguous (any K otherwise: rows past K read as zeros); 16-B aligned rows; beta 0 or 1;
// every operand's addressed span < 2 GiB.  Returns -1 (nothing launched) for shapes it does not take.
extern "C" int mx_gemm8(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc, void* C,
                        int64_t ldc, int out_f32, int M, int N, int K, float beta, const float* alpha_t, float alpha_f,
                        int ph, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (M & 255) || (N & 255)) return -1;
  if ((a_kc || b_kc) && (K % G8_BK)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 4 || ((uintptr_t)A | (uintptr_t)B) & 15 || ((uintptr_t)C & 15)) return -1;
  if (a_kc ? lda < K : lda < M) return -1;
  if (b_kc ? ldb < K : ldb < N) return -1;
  if (ldc < N || (!out_f32 && ldc % 8)) return -1;  // bf16 epilogue: 16-B stores
  if (beta != 0.f && beta != 1.f) return -1;
  const int64_t kpad = (int64_t)((K + G8_BK - 1) / G8_BK) * G8_BK;
  const int64_t aspan = a_kc ? 256 * lda : kpad * lda;
  const int64_t bspan = b_kc ? 256 * ldb : kpad * ldb;
  if (aspan * 2 >= ((int64_t)1 << 31) || bspan * 2 >= ((int64_t)1 << 31)) return -1;
  const int grid = (M >> 8) * (N >> 8);
  const bool acc = beta != 0.f;
  const char* phs = getenv("MXLLM_GEMM8_PH");  // read per call: overrides `ph` (same-process A/B)
  const bool ph4 = phs && *phs ? atoi(phs) == 4 : (ph == 4 || ph == 5);  // 5 = 4-phase, persistent
#define G8_L(AK, BK_, F, BT)                                                                                        \
  do {                                                                                                              \
    if (ph4)                                                                                                        \
      gemm8_kernel<AK, BK_, F, BT, 0, 4><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f); \
    else                                                                                                            \
      gemm8_kernel<AK, BK_, F, BT><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);      \
  } while (0)
#define G8_OUT(AK, BK_)                                        \
  do {                                                         \
    if (out_f32) {                                             \
      if (acc) G8_L(AK, BK_, true, true); else G8_L(AK, BK_, true, false);   \
    } else {                                                   \
      if (acc) G8_L(AK, BK_, false, true); else G8_L(AK, BK_, false, false); \
    }                                                          \
  } while (0)
#ifdef MXLLM_GEMM8_DIAG
  if (const char* st = getenv("MXLLM_GEMM8_STAMPS")) {  // diagnostic stamped build, NN bf16 beta 0
    if (a_kc && !b_kc && !out_f32 && !acc && grid <= 1024 && *st) {
      if (atoi(st) == 4)
        gemm8_kernel<true, false, false, false, 4, 4><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);
      else
        gemm8_kernel<true, false, false, false, 4, 8><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);
      return (int)hipGetLastError();
    }
  }
  if (const char* ab = getenv("MXLLM_GEMM8_ABLATE")) {  // timing-only variants, NN bf16 beta 0 (results wrong)
    const int v = atoi(ab);
    if (a_kc && !b_kc && !out_f32 && !acc && v >= 1 && v <= 3) {
      if (v == 1)
        gemm8_kernel<true, false, false, false, 1><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);
      else if (v == 2)
        gemm8_kernel<true, false, false, false, 2><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);
      else
        gemm8_kernel<true, false, false, false, 3><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f);
      return (int)hipGetLastError();
    }
  }
#endif
  const char* pe = getenv("MXLLM_GEMM8_PERSIST");  // 1 = persistent 4-phase kernel (read per call: A/B)
  const int persist = pe && *pe ? atoi(pe) : (ph == 5);
  if (persist && ph4 && grid > g8_cus()) {
    const int pg = g8_cus();
#define G8_P(AK, BK_, F, BT) \
  gemm8p_kernel<AK, BK_, F, BT><<<pg, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, alpha_f)
#define G8_PO(AK, BK_)                                                       \
  do {                                                                       \
    if (out_f32) { if (acc) G8_P(AK, BK_, true, true); else G8_P(AK, BK_, true, false); }     \
    else { if (acc) G8_P(AK, BK_, false, true); else G8_P(AK, BK_, false, false); }           \
  } while (0)
    if (a_kc && b_kc) G8_PO(true, true);
    else if (a_kc) G8_PO(true, false);
    else if (b_kc) G8_PO(false, true);
    else G8_PO(false, false);
#undef G8_PO
#undef G8_P
    return (int)hipGetLastError();
  }
  if (a_kc && b_kc)
    G8_OUT(true, true);
  else if (a_kc)
    G8_OUT(true, false);
  else if (b_kc)
    G8_OUT(false, true);
  else
    G8_OUT(false, false);
#undef G8_OUT
#undef G8_L
  return (int)hipGetLastError();
}

// Forward projection with a fused epilogue (G8Epi above), A = x [M][K] and B = W [N][K] both
// k-contiguous, 4-phase schedule.  mode 1 (ROPE): N = (Hq + 2 Hkv) * 128, M = B * S, S % 256 == 0,
// writes q / k / v head-major (C unused).  mode 2 (SWIGLU): N = 2F, F % 128 == 0, writes gu into C
// [M][ldc >= 2F] and m into ep.m [M][ldm >= F].  mode 3 (SWIGLU_BWD, NN form: A = dy [M][K], B =
// W_down [K][N]): dm -> dgu into C [M][ldc >= 2N] from ep.gu, and m into ep.m when set.  Returns -1
// (nothing launched) for other shapes.
extern "C" int mx_gemm8_epi(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, uint16_t* C, int64_t ldc,
                            int M, int N, int K, int mode, G8Epi ep, hipStream_t stream) {
  if (mode == G8_EPI_SWIGLU_BWD) {
    // NN: A = dy [M][K] k-contiguous, B = W_down [K][N] n-contiguous; C = dgu [M][ldc >= 2N]
    if (M <= 0 || N <= 0 || K <= 0 || (M & 255) || (N & 255) || K % G8_BK) return -1;
    if (lda % 8 || ldb % 8 || lda < K || ldb < N || ldc < 2 * (int64_t)N || ldc % 8 || !C || !ep.gu ||
        ep.ldg < 2 * (int64_t)N || ep.ldg % 8 || (ep.m && (ep.ldm < N || ep.ldm % 8)) ||
        (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)ep.gu | (uintptr_t)ep.m) & 15))
      return -1;
    if (256 * lda * 2 >= ((int64_t)1 << 31) || (int64_t)K * ldb * 2 >= ((int64_t)1 << 31)) return -1;
    ep.F = N;
    gemm8_kernel<true, false, false, false, 0, 4, G8_EPI_SWIGLU_BWD><<<(M >> 8) * (N >> 8), 512, 0, stream>>>(
        A, lda, B, ldb, C, ldc, M, N, K, nullptr, 1.f, 0, 0, ep);
    return (int)hipGetLastError();
  }
  if (M <= 0 || N <= 0 || K <= 0 || (M & 255) || (N & 255) || K % G8_BK) return -1;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K || ((uintptr_t)A | (uintptr_t)B) & 15) return -1;
  const int64_t aspan = 256 * lda, bspan = (int64_t)N * ldb;
  if (aspan * 2 >= ((int64_t)1 << 31) || bspan * 2 >= ((int64_t)1 << 31)) return -1;
  const int grid = (M >> 8) * (N >> 8);
  if (mode == G8_EPI_ROPE) {
    if (N != (ep.Hq + 2 * ep.Hkv) * 128 || ep.S <= 0 || ep.S % 256 || M % ep.S || !ep.q || !ep.k || !ep.v ||
        !ep.cosb || !ep.sinb || (((uintptr_t)ep.q | (uintptr_t)ep.k | (uintptr_t)ep.v) & 15))
      return -1;
    gemm8_kernel<true, true, false, false, 0, 4, G8_EPI_ROPE><<<grid, 512, 0, stream>>>(
        A, lda, B, ldb, nullptr, 0, M, N, K, nullptr, 1.f, 0, 0, ep);
  } else if (mode == G8_EPI_SWIGLU) {
    if ((N / 2) % 128 || !C || !ep.m || ldc < N || ldc % 8 || ep.ldm < N / 2 || ep.ldm % 8 ||
        (((uintptr_t)C | (uintptr_t)ep.m) & 15))
      return -1;
    ep.F = N / 2;
    gemm8_kernel<true, true, false, false, 0, 4, G8_EPI_SWIGLU><<<grid, 512, 0, stream>>>(
        A, lda, B, ldb, C, ldc, M, N, K, nullptr, 1.f, 0, 0, ep);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// Plain bf16, beta-0 gemm8 (any operand order, 4-phase schedule) that also writes one sum of squares
// of the stored bf16 values per 256 x 256 output tile into sq[(m / 256) * (N / 256) + n / 256]: the
// weight-gradient GEMMs hand the gradient-clip norm its partials (mxllm/train/trainer.py), so no
// pass re-reads the gradient for it.  Returns -1 (nothing launched) where mx_gemm8 would.
extern "C" int mx_gemm8_sq(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc,
                           uint16_t* C, int64_t ldc, int M, int N, int K, const float* alpha_t, float alpha_f,
                           float* sq, hipStream_t stream) {
  if (!sq || M <= 0 || N <= 0 || K <= 0 || (M & 255) || (N & 255)) return -1;
  if ((a_kc || b_kc) && (K % G8_BK)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8 || ((uintptr_t)A | (uintptr_t)B) & 15 || ((uintptr_t)C & 15)) return -1;
  if (a_kc ? lda < K : lda < M) return -1;
  if (b_kc ? ldb < K : ldb < N) return -1;
  if (ldc < N) return -1;
  const int64_t kpad = (int64_t)((K + G8_BK - 1) / G8_BK) * G8_BK;
  const int64_t aspan = a_kc ? 256 * lda : kpad * lda;
  const int64_t bspan = b_kc ? 256 * ldb : kpad * ldb;
  if (aspan * 2 >= ((int64_t)1 << 31) || bspan * 2 >= ((int64_t)1 << 31)) return -1;
  const int grid = (M >> 8) * (N >> 8);
  G8Epi ep{};
  ep.sq = sq;
#define G8_SQ(AK, BK_)                                                                                           \
  gemm8_kernel<AK, BK_, false, false, 0, 4><<<grid, 512, 0, stream>>>(A, lda, B, ldb, C, ldc, M, N, K, alpha_t, \
                                                                     alpha_f, 0, 0, ep)
  if (a_kc && b_kc) G8_SQ(true, true);
  else if (a_kc) G8_SQ(true, false);
  else if (b_kc) G8_SQ(false, true);
  else G8_SQ(false, false);
#undef G8_SQ
  return (int)hipGetLastError();
}

// C[m, c0 + n] = bf16(P0[m, n] + P1[m, n]) for the two K-part images of mx_gemm8_tail
__global__ void __launch_bounds__(256) g8_sum2_kernel(const float* __restrict__ P, int64_t part, int N2,
                                                      uint16_t* __restrict__ C, int64_t ldc, int64_t n_elems) {
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8; i < n_elems; i += (int64_t)gridDim.x * 256 * 8) {
    const int64_t m = i / N2;
    const int n = (int)(i - m * N2);
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(P + i), a1 = *reinterpret_cast<const f32x4*>(P + i + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(P + part + i), b1 = *reinterpret_cast<const f32x4*>(P + part + i + 4);
    uint4 o;
    o.x = pack_bf16x2(a0[0] + b0[0], a0[1] + b0[1]);
    o.y = pack_bf16x2(a0[2] + b0[2], a0[3] + b0[3]);
    o.z = pack_bf16x2(a1[0] + b1[0], a1[1] + b1[1]);
    o.w = pack_bf16x2(a1[2] + b1[2], a1[3] + b1[3]);
    *reinterpret_cast<uint4*>(C + m * ldc + n) = o;
  }
}

// g8_sum2 over whole 256 x 256 tiles of the K-part images (one workgroup per tile, the same
// arithmetic), also writing one sum of squares of the stored bf16 values per tile into sq[tile]
// (row-major tile order over the [M2, N2] region): the tail-balanced launch's share of the clip-norm
// partials (mx_gemm8_sq for the rest)
__global__ void __launch_bounds__(256) g8_sum2_sq_kernel(const float* __restrict__ P, int64_t part, int N2,
                                                         uint16_t* __restrict__ C, int64_t ldc,
                                                         float* __restrict__ sq) {
  __shared__ float red[4];
  const int tn = N2 >> 8, tm0 = blockIdx.x / tn, tn0 = blockIdx.x % tn;
  const int cu = threadIdx.x & 31, r0 = threadIdx.x >> 5;  // 8-column unit, first row
  float s = 0.f;
  for (int r = r0; r < 256; r += 8) {
    const int64_t m = (int64_t)tm0 * 256 + r;
    const int n = tn0 * 256 + cu * 8;
    const int64_t i = m * N2 + n;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(P + i), a1 = *reinterpret_cast<const f32x4*>(P + i + 4);
    const f32x4 b0 = *reinterpret_cast<const f32x4*>(P + part + i), b1 = *reinterpret_cast<const f32x4*>(P + part + i + 4);
    uint4 o;
    o.x = pack_bf16x2(a0[0] + b0[0], a0[1] + b0[1]);
    o.y = pack_bf16x2(a0[2] + b0[2], a0[3] + b0[3]);
    o.z = pack_bf16x2(a1[0] + b1[0], a1[1] + b1[1]);
    o.w = pack_bf16x2(a1[2] + b1[2], a1[3] + b1[3]);
    *reinterpret_cast<uint4*>(C + m * ldc + n) = o;
    s = g8_sq8(o, s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) sq[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Tail-balanced bf16 GEMM, beta 0, alpha 1: C[M, N] = op(A) op(B) where the tile count leaves a last
// wave of <= 128 tiles on the 256 CUs (e.g. the 70B qkv forward: 16 x 40 = 640 tiles).  The output is
// split at `at` (columns, or rows when `rows`): [0, at) runs as one plain launch of whole waves; the
// rest as ONE launch of twice as many workgroups, each over half of K (gridDim.y = 2), into two fp32
// images in `ws` (2 * its element count); g8_sum2_kernel adds them in a fixed order into C
// (deterministic).  The last wave then takes half a wave's time.  `at` and the rest multiples of 256.
extern "C" int mx_gemm8_tail(const uint16_t* A, int64_t lda, int a_kc, const uint16_t* B, int64_t ldb, int b_kc,
                             uint16_t* C, int64_t ldc, int M, int N, int K, int rows, int at, float* ws, int ph,
                             hipStream_t stream, float* sq) {
  const int lim = rows ? M : N, rest = lim - at;
  if (at <= 0 || rest <= 0 || (at & 255) || (rest & 255) || K < 2 * G8_BK) return -1;
  if ((a_kc ? lda < K : lda < M) || (b_kc ? ldb < K : ldb < N) || ldb % 8 || lda % 8 || ldc % 8) return -1;
  if (sq && (ph != 4 || (M & 255) || (N & 255))) return -1;  // partials: the 4-phase schedule, whole tiles
  // every check of the split part BEFORE the plain part launches: a -1 after a launch would
  // leave sq partials of a GEMM the caller then recomputes another way (a double-counted clip norm)
  const uint16_t* A2 = rows ? (a_kc ? A + (int64_t)at * lda : A + at) : A;
  const uint16_t* B2 = rows ? B : (b_kc ? B + (int64_t)at * ldb : B + at);
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C | (uintptr_t)A2 | (uintptr_t)B2 | (uintptr_t)ws) & 15) return -1;
  if ((a_kc || b_kc) && (K % G8_BK)) return -1;
  {
    const int64_t kpad = (int64_t)((K + G8_BK - 1) / G8_BK) * G8_BK;
    const int64_t aspan = a_kc ? 256 * lda : kpad * lda, bspan = b_kc ? 256 * ldb : kpad * ldb;
    if (aspan * 2 >= ((int64_t)1 << 31) || bspan * 2 >= ((int64_t)1 << 31) || ldc < N) return -1;
  }
  // plain part (sq: its tiles' partials first, then the split part's)
  int rc;
  if (sq)
    rc = rows ? mx_gemm8_sq(A, lda, a_kc, B, ldb, b_kc, C, ldc, at, N, K, nullptr, 1.f, sq, stream)
              : mx_gemm8_sq(A, lda, a_kc, B, ldb, b_kc, C, ldc, M, at, K, nullptr, 1.f, sq, stream);
  else
    rc = rows ? mx_gemm8(A, lda, a_kc, B, ldb, b_kc, C, ldc, 0, at, N, K, 0.f, nullptr, 1.f, ph, stream)
              : mx_gemm8(A, lda, a_kc, B, ldb, b_kc, C, ldc, 0, M, at, K, 0.f, nullptr, 1.f, ph, stream);
  if (rc) return rc;
  uint16_t* C2 = rows ? C + (int64_t)at * ldc : C + at;
  const int M2 = rows ? rest : M, N2 = rows ? N : rest;
  const int k0 = (K / G8_BK / 2) * G8_BK;  // part 0: floor(K-tiles / 2) tiles
  const int64_t part = (int64_t)M2 * N2;
  const dim3 grid((M2 >> 8) * (N2 >> 8), 2);
  const char* phs = getenv("MXLLM_GEMM8_PH");
  const bool ph4 = phs && *phs ? atoi(phs) == 4 : ph == 4;
#define G8_T(AK, BK_)                                                                                               \
  do {                                                                                                              \
    if (ph4)                                                                                                        \
      gemm8_kernel<AK, BK_, true, false, 0, 4><<<grid, 512, 0, stream>>>(A2, lda, B2, ldb, ws, N2, M2, N2, K, nullptr, \
                                                                         1.f, k0, part);                            \
    else                                                                                                            \
      gemm8_kernel<AK, BK_, true, false><<<grid, 512, 0, stream>>>(A2, lda, B2, ldb, ws, N2, M2, N2, K, nullptr, 1.f, \
                                                                   k0, part);                                       \
  } while (0)
  if (a_kc && b_kc) G8_T(true, true);
  else if (a_kc) G8_T(true, false);
  else if (b_kc) G8_T(false, true);
  else G8_T(false, false);
#undef G8_T
  if (sq) {
    const int64_t nplain = rows ? (int64_t)(at >> 8) * (N >> 8) : (int64_t)(M >> 8) * (at >> 8);
    g8_sum2_sq_kernel<<<(M2 >> 8) * (N2 >> 8), 256, 0, stream>>>(ws, part, N2, C2, ldc, sq + nplain);
    return (int)hipGetLastError();
  }
  int64_t blocks = (part / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  g8_sum2_kernel<<<(int)blocks, 256, 0, stream>>>(ws, part, N2, C2, ldc, part);
  return (int)hipGetLastError();
}

// Split part of mx_gemm8_rope_tail: the two fp32 K-part images P0, P1 [M, N2] of columns [col0, col0 + N2)
// -> bf16(P0 + P1) in a fixed order (= g8_sum2_kernel), then, per 128-column head, the rotate-half RoPE
// of rope_split_kernel (csrc/kernels/rope.hip: the same expression on the same bf16 values, so bitwise
// the tail-balanced GEMM followed by rope_split) and the head-major scatter; v heads are copied.
// One thread per (row, head, 8-column group of the head's first half).
__global__ void __launch_bounds__(256) g8_sum2_rope_kernel(const float* __restrict__ P, int64_t part, int N2, int col0,
                                                          int M, G8Epi ep) {
  const int nh = N2 >> 7;
  const int64_t n = (int64_t)M * nh * 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int g = (int)(i & 7);
    const int64_t th = i >> 3;
    const int hl = (int)(th % nh);
    const int64_t m = th / nh;
    const int head = (col0 >> 7) + hl;
    const int b = (int)(m / ep.S), sq = (int)(m - (int64_t)b * ep.S);
    const int c = hl * 128 + 8 * g;  // column inside the split part (first half of the head)
    const float* p0 = P + m * N2 + c;
    const float* p1 = P + part + m * N2 + c;
    float x1[8], x2[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(p0 + 4 * h), b0 = *reinterpret_cast<const f32x4*>(p1 + 4 * h);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(p0 + 64 + 4 * h);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(p1 + 64 + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x1[4 * h + j] = bf2f(f2bf(a0[j] + b0[j]));
        x2[4 * h + j] = bf2f(f2bf(a1[j] + b1[j]));
      }
    }
    uint16_t* dst;
    if (head < ep.Hq) {
      dst = ep.q + (((int64_t)b * ep.Hq + head) * ep.S + sq) * 128;
    } else if (head < ep.Hq + ep.Hkv) {
      dst = ep.k + (((int64_t)b * ep.Hkv + (head - ep.Hq)) * ep.S + sq) * 128;
    } else {
      dst = ep.v + (((int64_t)b * ep.Hkv + (head - ep.Hq - ep.Hkv)) * ep.S + sq) * 128;
      u16x8 y1, y2;
#pragma unroll
      for (int j = 0; j < 8; ++j) y1[j] = f2bf(x1[j]), y2[j] = f2bf(x2[j]);
      *reinterpret_cast<u16x8*>(dst + 8 * g) = y1;
      *reinterpret_cast<u16x8*>(dst + 64 + 8 * g) = y2;
      continue;
    }
    const float* cp = ep.cosb + (int64_t)sq * 64 + 8 * g;
    const float* sp = ep.sinb + (int64_t)sq * 64 + 8 * g;
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cp), c1 = *reinterpret_cast<const f32x4*>(cp + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(sp), s1 = *reinterpret_cast<const f32x4*>(sp + 4);
    u16x8 y1, y2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cj = j < 4 ? c0[j & 3] : c1[j & 3];
      const float sj = j < 4 ? s0[j & 3] : s1[j & 3];
      const float a = x1[j], bb = x2[j];
      y1[j] = f2bf(rope_lo(a, bb, cj, sj));
      y2[j] = f2bf(rope_hi(a, bb, cj, sj));
    }
    *reinterpret_cast<u16x8*>(dst + 8 * g) = y1;
    *reinterpret_cast<u16x8*>(dst + 64 + 8 * g) = y2;
  }
}

// qkv projection (A = x [M][K], B = W [N][K], both k-contiguous; N = (Hq + 2 Hkv) * 128, M = B * S) with
// the RoPE + head split fused, on the tail-balanced schedule of mx_gemm8_tail: columns [0, at) (whole
// waves of tiles) through the G8_EPI_ROPE epilogue, columns [at, N) as twice as many half-K workgroups
// into the two fp32 images in `ws` (2 * M * (N - at) floats), finished by g8_sum2_rope_kernel.  Removes
// the qkv round trip through HBM and the rope_split pass of the LoRA-augmented qkv forward, whose GEMM
// runs this tail-balanced launch anyway (70B: 16 x 40 tiles, `at` 8192 = the q heads).  Returns -1
// (nothing launched) for shapes it does not take.
extern "C" int mx_gemm8_rope_tail(const uint16_t* A, int64_t lda, const uint16_t* B, int64_t ldb, int M, int N, int K,
                                  int at, float* ws, G8Epi ep, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K < 2 * G8_BK || (M & 255) || (N & 255) || K % G8_BK) return -1;
  if (at <= 0 || at >= N || (at & 255)) return -1;
  if (lda % 8 || ldb % 8 || lda < K || ldb < K || (((uintptr_t)A | (uintptr_t)B | (uintptr_t)ws) & 15)) return -1;
  const int64_t aspan = 256 * lda, bspan = (int64_t)N * ldb;
  if (aspan * 2 >= ((int64_t)1 << 31) || bspan * 2 >= ((int64_t)1 << 31)) return -1;
  if (N != (ep.Hq + 2 * ep.Hkv) * 128 || ep.S <= 0 || ep.S % 256 || M % ep.S || !ep.q || !ep.k || !ep.v ||
      !ep.cosb || !ep.sinb || (((uintptr_t)ep.q | (uintptr_t)ep.k | (uintptr_t)ep.v) & 15) ||
      (((uintptr_t)ep.cosb | (uintptr_t)ep.sinb) & 15))
    return -1;
  // plain part: the epilogue writes q / k / v of the heads in [0, at) (tile pn covers heads 2 pn, 2 pn + 1)
  gemm8_kernel<true, true, false, false, 0, 4, G8_EPI_ROPE><<<(M >> 8) * (at >> 8), 512, 0, stream>>>(
      A, lda, B, ldb, nullptr, 0, M, at, K, nullptr, 1.f, 0, 0, ep);
  // split part: columns [at, N), two half-K images
  const int N2 = N - at;
  const int k0 = (K / G8_BK / 2) * G8_BK;
  const int64_t part = (int64_t)M * N2;
  const dim3 grid((M >> 8) * (N2 >> 8), 2);
  gemm8_kernel<true, true, true, false, 0, 4><<<grid, 512, 0, stream>>>(A, lda, B + (int64_t)at * ldb, ldb, ws, N2, M,
                                                                        N2, K, nullptr, 1.f, k0, part);
  int64_t blocks = ((int64_t)M * (N2 >> 7) * 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  g8_sum2_rope_kernel<<<(int)blocks, 256, 0, stream>>>(ws, part, N2, at, M, ep);
  return (int)hipGetLastError();
}

// copy the diagnostic stamps out (host buffer of 1024 * 2 * 80 uint64)
extern "C" int mx_gemm8_stamps(unsigned long long* host) {
#ifdef MXLLM_GEMM8_DIAG
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g8_stamps), sizeof(unsigned long long) * 1024 * 2 * G8_NST, 0,
                                  hipMemcpyDeviceToHost);
#else
  (void)host;
  return -1;  // not a diagnostic build
#endif
}
