// Memory-bound fused elementwise kernels for gfx950:
//   * swiglu fwd/bwd over a fused [gate | up] projection
//   * fused AdamW over flat buffers (fp32 master, fp32/bf16 grad, optional bf16 copy)
//   * token-embedding gather / f32-atomic scatter-add
// Every kernel moves 16 B per lane per access (G13), grid-strides with
// <= 2048 workgroups x 256 threads (G11).
#include <cstdlib>

#include "common.h"

namespace mx {

// sigmoid by the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division sequence;
// csrc/kernels/lora.hip swiglu_lora_kernel uses the identical expressions (bitwise-equal outputs)
__device__ __forceinline__ float sigmoid_f(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// m[t, c] = silu(gu[t, c]) * gu[t, F + c]
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ m,
                                                         int64_t T, int F, int64_t ldm) {
  const int64_t per_row = F / 8;
  const int64_t n = T * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i / per_row;
    const int c = (int)(i - t * per_row) * 8;
    const uint16_t* row = gu + t * (2 * (int64_t)F);
    u16x8 g = *reinterpret_cast<const u16x8*>(row + c);
    u16x8 u = *reinterpret_cast<const u16x8*>(row + F + c);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]);
      o[j] = f2bf(gf * sigmoid_f(gf) * bf2f(u[j]));
    }
    *reinterpret_cast<u16x8*>(m + t * ldm + c) = o;
  }
}

// dg = dm * u * s * (1 + g (1 - s)),  du = dm * g * s,  s = sigmoid(g)
// WM: also re-emit m = g s u (the forward's expression: bitwise its output) for a backward that
// recomputes the activation instead of saving it (mxllm/ops/linear.py _SwiGLULinearFn): gu is
// read once for both
template <bool WM>
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const uint16_t* __restrict__ dm,
                                                         const uint16_t* __restrict__ gu,
                                                         uint16_t* __restrict__ dgu, int64_t T, int F,
                                                         int64_t ldg, uint16_t* __restrict__ m) {
  const int64_t per_row = F / 8;
  const int64_t n = T * per_row;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t t = i / per_row;
    const int c = (int)(i - t * per_row) * 8;
    const uint16_t* row = gu + t * (2 * (int64_t)F);
    u16x8 g = *reinterpret_cast<const u16x8*>(row + c);
    u16x8 u = *reinterpret_cast<const u16x8*>(row + F + c);
    u16x8 d = *reinterpret_cast<const u16x8*>(dm + t * (int64_t)F + c);
    u16x8 og, ou, om;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gf = bf2f(g[j]), uf = bf2f(u[j]), df = bf2f(d[j]);
      float dg, du;
      swiglu_grad(df, gf, uf, dg, du);
      og[j] = f2bf(dg);
      ou[j] = f2bf(du);
      if constexpr (WM) om[j] = f2bf(gf * sigmoid_f(gf) * uf);
    }
    uint16_t* orow = dgu + t * ldg;
    *reinterpret_cast<u16x8*>(orow + c) = og;
    *reinterpret_cast<u16x8*>(orow + F + c) = ou;
    if constexpr (WM) *reinterpret_cast<u16x8*>(m + t * (int64_t)F + c) = om;
  }
}

// Fused AdamW, 4 elements per lane per iteration (n % 4 == 0).  ZERO: the gradient
// is cleared in the same pass (the next backward accumulates into it with beta=1),
// so no separate memset re-streams the gradient buffer.
// SPLIT: the fp32 master is stored as two 16-bit halves — ``lowp`` (the bf16 compute
// weight, the master rounded half-up on its bit pattern) and ``lo`` = master bits -
// (lowp << 16) in [-32768, 32767] — reconstructed exactly in registers.  Same
// optimizer arithmetic as the fp32 master, 2 B/param less state and HBM traffic
// (the separate bf16 copy IS the master's high half).
__device__ __forceinline__ float split_join(uint16_t h, int16_t l) {
  return __uint_as_float(((uint32_t)h << 16) + (uint32_t)(int32_t)l);
}
__device__ __forceinline__ void split_make(float x, uint16_t& h, int16_t& l) {
  const uint32_t b = __float_as_uint(x);
  h = (uint16_t)((b + 0x8000u) >> 16);
  l = (int16_t)(int32_t)(b - ((uint32_t)h << 16));
}

template <bool GRAD_BF16, bool LOWP, bool ZERO, bool SPLIT>
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, void* __restrict__ gv,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    uint16_t* __restrict__ lowp, int16_t* __restrict__ lo,
                                                    int64_t n, float lr, float b1,
                                                    float b2, float eps, float wd, float inv_bc1, float inv_bc2,
                                                    const float* __restrict__ scale_t, float scale_f) {
  const float gs = scale_f * (scale_t ? scale_t[0] : 1.f);
  const float decay = 1.f - lr * wd;
  const float step = lr * inv_bc1;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += (int64_t)gridDim.x * 256 * 4) {
    f32x4 g;
    if constexpr (GRAD_BF16) {
      u16x4 gb = *reinterpret_cast<const u16x4*>(reinterpret_cast<const uint16_t*>(gv) + i);
      g = f32x4{bf2f(gb[0]), bf2f(gb[1]), bf2f(gb[2]), bf2f(gb[3])};
      if constexpr (ZERO) *reinterpret_cast<u16x4*>(reinterpret_cast<uint16_t*>(gv) + i) = u16x4{0, 0, 0, 0};
    } else {
      g = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(gv) + i);
      if constexpr (ZERO) *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(gv) + i) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 pp;
    u16x4 hh;
    s16x4 ll;
    if constexpr (SPLIT) {
      hh = *reinterpret_cast<const u16x4*>(lowp + i);
      ll = *reinterpret_cast<const s16x4*>(lo + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) pp[j] = split_join(hh[j], ll[j]);
    } else {
      pp = *reinterpret_cast<f32x4*>(p + i);
    }
    f32x4 mm = *reinterpret_cast<f32x4*>(m + i);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + i);
    u16x4 lw;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = g[j] * gs;
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      const float den = sqrtf(vv[j] * inv_bc2) + eps;
      pp[j] = pp[j] * decay - step * mm[j] / den;
      if constexpr (SPLIT) {
        uint16_t h;
        int16_t l;
        split_make(pp[j], h, l);
        hh[j] = h;
        ll[j] = l;
      } else if constexpr (LOWP) {
        lw[j] = f2bf(pp[j]);
      }
    }
    if constexpr (SPLIT) {
      *reinterpret_cast<u16x4*>(lowp + i) = hh;
      *reinterpret_cast<s16x4*>(lo + i) = ll;
    } else {
      *reinterpret_cast<f32x4*>(p + i) = pp;
      if constexpr (LOWP) *reinterpret_cast<u16x4*>(lowp + i) = lw;
    }
    *reinterpret_cast<f32x4*>(m + i) = mm;
    *reinterpret_cast<f32x4*>(v + i) = vv;
  }
}

// fp32 master <-> (hi, lo) halves, element-wise (checkpoint load/save, init)
__global__ void __launch_bounds__(256) split_master_kernel(const float* __restrict__ x, uint16_t* __restrict__ hi,
                                                           int16_t* __restrict__ lo, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint16_t h;
    int16_t l;
    split_make(x[i], h, l);
    hi[i] = h;
    lo[i] = l;
  }
}

__global__ void __launch_bounds__(256) join_master_kernel(const uint16_t* __restrict__ hi,
                                                          const int16_t* __restrict__ lo, float* __restrict__ x,
                                                          int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    x[i] = split_join(hi[i], lo[i]);
}

// out[t, :] = W[ids[t], :]  — one 256-thread block per token row
__global__ void __launch_bounds__(256) embedding_fwd_kernel(const int64_t* __restrict__ ids,
                                                            const uint16_t* __restrict__ w,
                                                            uint16_t* __restrict__ out, int H, int64_t V) {
  const int64_t t = blockIdx.x;
  int64_t id = ids[t];
  id = id < 0 ? 0 : (id >= V ? V - 1 : id);
  const uint16_t* src = w + id * H;
  uint16_t* dst = out + t * H;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8)
    *reinterpret_cast<u16x8*>(dst + c) = *reinterpret_cast<const u16x8*>(src + c);
}

// dW[ids[t], :] += dy[t, :]  (f32 accumulator, no-return atomics; each wave
// instruction covers 64 consecutive floats = one 256-B segment)
__global__ void __launch_bounds__(256) embedding_bwd_kernel(const int64_t* __restrict__ ids,
                                                            const uint16_t* __restrict__ dy,
                                                            float* __restrict__ dw, int H, int64_t V) {
  const int64_t t = blockIdx.x;
  const int64_t id = ids[t];
  if (id < 0 || id >= V) return;
  const uint16_t* src = dy + t * H;
  float* dst = dw + id * H;
  for (int c = threadIdx.x; c < H; c += 256) atomicAdd(dst + c, bf2f(src[c]));
}

// Sparse, deterministic embedding backward into the parameter's own gradient buffer:
// sid = the batch's token ids sorted (stable), perm = their positions.  Only the rows the
// batch touched are read or written (no zero-filled full [V, H] accumulator).
//
// The sorted positions are cut into fixed chunks of EB_CH rows, one workgroup each (grid-stride),
// so a dominant id (pad / EOS in packed batches: thousands of rows of one segment) is spread over
// many workgroups instead of one walking it serially.  Inside a chunk each run of one
// id is summed in sorted order in fp32; a run wholly inside its chunk is added to `out` directly
// (fp32, or bf16 with one rounding); a run that continues into a neighbouring chunk writes an fp32
// partial (slot 0: it continues from the previous chunk; slot 1: it starts here and continues),
// and embedding_bwd_combine_kernel adds each such segment's partials in chunk order -- a fixed
// order, so the result is still bit-reproducible.
constexpr int EB_CH = 64;

template <bool F32>
__device__ __forceinline__ void eb_add_row(void* __restrict__ out, int64_t row, int H, int c, const float (&acc)[8]) {
  if constexpr (F32) {
    float* o = reinterpret_cast<float*>(out) + row * H + c;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += acc[e];
  } else {
    uint16_t* o = reinterpret_cast<uint16_t*>(out) + row * H + c;
    u16x8 cur = *reinterpret_cast<const u16x8*>(o);
#pragma unroll
    for (int e = 0; e < 8; ++e) cur[e] = f2bf(bf2f(cur[e]) + acc[e]);
    *reinterpret_cast<u16x8*>(o) = cur;
  }
}

template <bool F32>
__global__ void __launch_bounds__(256) embedding_bwd_sorted_kernel(const uint16_t* __restrict__ dy,
                                                                   const int64_t* __restrict__ sid,
                                                                   const int64_t* __restrict__ perm, int64_t T,
                                                                   int H, int64_t V, void* __restrict__ out,
                                                                   float* __restrict__ ws) {
  const int64_t nch = (T + EB_CH - 1) / EB_CH;
  for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t p0 = ch * EB_CH, p1 = min(T, p0 + EB_CH);
    for (int64_t r0 = p0; r0 < p1;) {  // runs of one id (workgroup-uniform control flow)
      const int64_t row = sid[r0];
      int64_t r1 = r0 + 1;
      while (r1 < p1 && sid[r1] == row) ++r1;
      const bool from_prev = r0 == p0 && p0 > 0 && sid[p0 - 1] == row;
      const bool to_next = r1 == p1 && p1 < T && sid[p1] == row;
      if (row >= 0 && row < V) {
        for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
          float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          for (int64_t j = r0; j < r1; ++j) {
            const u16x8 v = *reinterpret_cast<const u16x8*>(dy + perm[j] * H + c);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
          }
          if (!from_prev && !to_next) {
            eb_add_row<F32>(out, row, H, c, acc);
          } else {
            float* w = ws + (ch * 2 + (from_prev ? 0 : 1)) * (int64_t)H + c;
            *reinterpret_cast<float4*>(w) = float4{acc[0], acc[1], acc[2], acc[3]};
            *reinterpret_cast<float4*>(w + 4) = float4{acc[4], acc[5], acc[6], acc[7]};
          }
        }
      }
      r0 = r1;
    }
  }
}

// one workgroup per chunk: the chunk where a chunk-crossing segment STARTS sums its slot-1 partial
// and the following chunks' slot-0 partials in chunk order, then adds the sum into `out` once
template <bool F32>
__global__ void __launch_bounds__(256) embedding_bwd_combine_kernel(const int64_t* __restrict__ sid, int64_t T,
                                                                    int H, int64_t V, void* __restrict__ out,
                                                                    const float* __restrict__ ws) {
  const int64_t nch = (T + EB_CH - 1) / EB_CH;
  for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t p0 = ch * EB_CH, p1 = min(T, p0 + EB_CH);
    if (p1 >= T) continue;
    const int64_t row = sid[p1 - 1];
    if (sid[p1] != row || row < 0 || row >= V) continue;  // last run does not continue
    int64_t r0 = p1 - 1;
    while (r0 > p0 && sid[r0 - 1] == row) --r0;
    if (r0 == p0 && p0 > 0 && sid[p0 - 1] == row) continue;  // the segment started in an earlier chunk
    for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
      float acc[8];
      const float* w = ws + (ch * 2 + 1) * (int64_t)H + c;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = w[e];
      for (int64_t k = ch + 1; k < nch; ++k) {
        const float* w0 = ws + (k * 2) * (int64_t)H + c;
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += w0[e];
        const int64_t q1 = min(T, (k + 1) * EB_CH);
        if (!(q1 < T && sid[q1] == row)) break;  // the segment ends inside chunk k
      }
      eb_add_row<F32>(out, row, H, c, acc);
    }
  }
}

}  // namespace mx

using namespace mx;

// ws: 2 * ceil(T / 64) * H floats (partials of chunk-crossing segments; never read before written)
extern "C" int mx_embedding_bwd_sorted(const uint16_t* dy, const int64_t* sid, const int64_t* perm, int64_t T, int H,
                                       int64_t V, void* out, int out_f32, float* ws, hipStream_t stream) {
  if (T <= 0) return 0;
  if (H % 8) return -1;
  const int64_t nch = (T + EB_CH - 1) / EB_CH;
  const unsigned grid = (unsigned)(nch < 8192 ? nch : 8192);
  if (out_f32) {
    embedding_bwd_sorted_kernel<true><<<grid, 256, 0, stream>>>(dy, sid, perm, T, H, V, out, ws);
    embedding_bwd_combine_kernel<true><<<grid, 256, 0, stream>>>(sid, T, H, V, out, ws);
  } else {
    embedding_bwd_sorted_kernel<false><<<grid, 256, 0, stream>>>(dy, sid, perm, T, H, V, out, ws);
    embedding_bwd_combine_kernel<false><<<grid, 256, 0, stream>>>(sid, T, H, V, out, ws);
  }
  return (int)hipGetLastError();
}

static int grid_for(int64_t items) {
  int64_t b = (items + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

// ldm / ldg: output row strides (elements, multiples of 8): the outputs may be the left
// part of the LoRA-augmented GEMM operand buffers (mxllm/ops/linear.py)
extern "C" int mx_swiglu_fwd(const uint16_t* gu, uint16_t* m, int64_t T, int F, int64_t ldm, hipStream_t stream) {
  if (F % 8 || ldm < F || ldm % 8) return -1;
  swiglu_fwd_kernel<<<grid_for(T * (F / 8)), 256, 0, stream>>>(gu, m, T, F, ldm);
  return (int)hipGetLastError();
}

// m (optional, [T, F] dense): also write the recomputed activation
extern "C" int mx_swiglu_bwd(const uint16_t* dm, const uint16_t* gu, uint16_t* dgu, int64_t T, int F, int64_t ldg,
                             hipStream_t stream, uint16_t* m) {
  if (F % 8 || ldg < 2 * (int64_t)F || ldg % 8) return -1;
  if (m)
    swiglu_bwd_kernel<true><<<grid_for(T * (F / 8)), 256, 0, stream>>>(dm, gu, dgu, T, F, ldg, m);
  else
    swiglu_bwd_kernel<false><<<grid_for(T * (F / 8)), 256, 0, stream>>>(dm, gu, dgu, T, F, ldg, nullptr);
  return (int)hipGetLastError();
}

static int adamw_grid_cap() {
  static int cap = -1;
  if (cap < 0) {
    // workgroups of one AdamW launch (grid-stride beyond).  The overlapped update shares the GPU with the
    // next forward's GEMMs: 1,024 beats 2,048 on config 2 by 1.2-1.8 ms per step and is neutral on the
    // headline and the config-4 proxy; 768 and 512 lose (profiles/r5y/, r5z/).  MXLLM_ADAMW_GRID overrides.
    const char* e = getenv("MXLLM_ADAMW_GRID");
    cap = e ? atoi(e) : 1024;
    if (cap < 1) cap = 1024;
  }
  return cap;
}

// lo != nullptr: SPLIT master (p unused, lowp = the high half, required)
extern "C" int mx_adamw(float* p, void* g, int grad_bf16, float* m, float* v, uint16_t* lowp, int16_t* lo, int64_t n,
                        float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, const float* scale_t,
                        float scale_f, int zero_grad, hipStream_t stream) {
  if (n % 4) return -1;
  if (lo && !lowp) return -1;
  int grid = grid_for(n / 4);
  if (grid > adamw_grid_cap()) grid = adamw_grid_cap();
  const float ib1 = 1.f / bc1, ib2 = 1.f / bc2;
#define ADAM_LAUNCH(GB, LP, Z, SP)                                                                            \
  adamw_kernel<GB, LP, Z, SP><<<grid, 256, 0, stream>>>(p, g, m, v, lowp, lo, n, lr, b1, b2, eps, wd, ib1, ib2, \
                                                        scale_t, scale_f)
#define ADAM_Z(GB, LP, SP) \
  do { if (zero_grad) ADAM_LAUNCH(GB, LP, true, SP); else ADAM_LAUNCH(GB, LP, false, SP); } while (0)
  if (lo) {
    if (grad_bf16) ADAM_Z(true, true, true); else ADAM_Z(false, true, true);
  } else if (grad_bf16) {
    if (lowp) ADAM_Z(true, true, false); else ADAM_Z(true, false, false);
  } else {
    if (lowp) ADAM_Z(false, true, false); else ADAM_Z(false, false, false);
  }
#undef ADAM_Z
#undef ADAM_LAUNCH
  return (int)hipGetLastError();
}

extern "C" int mx_split_master(const float* x, uint16_t* hi, int16_t* lo, int64_t n, hipStream_t stream) {
  if (n <= 0) return 0;
  split_master_kernel<<<grid_for(n), 256, 0, stream>>>(x, hi, lo, n);
  return (int)hipGetLastError();
}

extern "C" int mx_join_master(const uint16_t* hi, const int16_t* lo, float* x, int64_t n, hipStream_t stream) {
  if (n <= 0) return 0;
  join_master_kernel<<<grid_for(n), 256, 0, stream>>>(hi, lo, x, n);
  return (int)hipGetLastError();
}

extern "C" int mx_embedding_fwd(const int64_t* ids, const uint16_t* w, uint16_t* out, int64_t T, int H,
                                int64_t V, hipStream_t stream) {
  if (H % 8 || T <= 0) return T <= 0 ? 0 : -1;
  embedding_fwd_kernel<<<(unsigned)T, 256, 0, stream>>>(ids, w, out, H, V);
  return (int)hipGetLastError();
}

extern "C" int mx_embedding_bwd(const int64_t* ids, const uint16_t* dy, float* dw, int64_t T, int H, int64_t V,
                                hipStream_t stream) {
  if (T <= 0) return 0;
  embedding_bwd_kernel<<<(unsigned)T, 256, 0, stream>>>(ids, dy, dw, H, V);
  return (int)hipGetLastError();
}
