// Batched token sampler with per-row temperature / top-k / top-p.
//
// OpenAI / LiteLLM semantics (the reference's completion() endpoint,
// src/distributed_inference.py:37): probabilities are softmax(logits / T); the
// candidate set is the top_k most likely tokens (k <= 0: all), then the
// smallest most-likely prefix of those whose mass reaches top_p of the set
// (the token that crosses top_p is kept); one token is drawn from the
// renormalised candidates.  T <= 0 is greedy argmax.
//
// (Rows without top-k / top-p take decode.hip's vocabulary-split kernel instead, same draws;
// mxllm/ops/decode.py sample_rows routes them.)  Here: one 1024-thread workgroup per row, no sort:
//  * logits map to order-preserving 32-bit keys (bf16 -> its exact f32);
//  * the k-th largest key and then the top-p boundary key are found by a
//    radix select, 11 + 11 + 10 bits, over LDS histograms: counts for top-k,
//    softmax masses exp2((x - max) * log2e / T) for top-p (restricted to the
//    top-k set).  Ties at a boundary are kept;
//  * the draw is Gumbel-max restricted to keys >= the boundary: argmax of
//    x / T + G(seed, step, index) is an EXACT sample of the renormalised
//    distribution over that set, with the same (seed, step, index) noise as the
//    greedy/temperature kernel in decode.hip, so a request's stream does not
//    depend on batching;
//  * every pass streams the row (256 KB bf16 at a 128k vocabulary) from L2 with
//    16-B loads.
// The LDS mass histogram uses float atomics: a boundary whose cumulative mass
// is within rounding of top_p * Z can move by one key between runs.
#include "common.h"

namespace mx {

__device__ __forceinline__ uint32_t okey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ uint32_t hash3s(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 15; h *= 0x2C1B3C6Du; h ^= h >> 12; h *= 0x297A2D39u; h ^= h >> 15;
  return h;
}

constexpr int kSampThreads = 1024;
constexpr int kBins = 2048;  // 11-bit digits

template <typename T>
struct RowReader {
  const T* x;
  int V;
  // calls f(index, value) for every element; 8 elements per lane per step (16 B bf16 / 2x16 B f32)
  template <typename F>
  __device__ __forceinline__ void each(F&& f) const {
    const int vec_end = (V / 8) * 8;
    const bool aligned = (((uintptr_t)x) & 15) == 0;
    if (aligned) {
      for (int base = threadIdx.x * 8; base < vec_end; base += kSampThreads * 8) {
        if constexpr (sizeof(T) == 2) {
          const u16x8 v = *reinterpret_cast<const u16x8*>(reinterpret_cast<const uint16_t*>(x) + base);
#pragma unroll
          for (int j = 0; j < 8; ++j) f(base + j, bf2f(v[j]));
        } else {
          const f32x4 a = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + base);
          const f32x4 b = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(x) + base + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) f(base + j, a[j]);
#pragma unroll
          for (int j = 0; j < 4; ++j) f(base + 4 + j, b[j]);
        }
      }
    }
    for (int c = (aligned ? vec_end : 0) + threadIdx.x; c < V; c += kSampThreads) {
      float v;
      if constexpr (sizeof(T) == 2) v = bf2f(reinterpret_cast<const uint16_t*>(x)[c]);
      else v = reinterpret_cast<const float*>(x)[c];
      f(c, v);
    }
  }
};

// Radix-select step: over elements whose key matches `prefix` on the bits above
// `shift + nbits` (and passes `keep`), histogram the next `nbits` digit with weight
// wfn(value); pick the digit where the descending cumulative weight, starting at
// `*above`, first reaches `target`; fold the weight of higher digits into `*above`.
template <typename T, typename K, typename W>
__device__ __forceinline__ uint32_t radix_digit(const RowReader<T>& rd, float* hist, float* scan, int* sel,
                                                uint32_t prefix, int shift, int nbits, K keep, W wfn, float* above,
                                                float target) {
  const int nb = 1 << nbits;
  for (int i = threadIdx.x; i < kBins; i += kSampThreads) hist[i] = 0.f;
  __syncthreads();
  const uint32_t hi_mask = (shift + nbits >= 32) ? 0u : (0xffffffffu << (shift + nbits));
  rd.each([&](int idx, float v) {
    const uint32_t k = okey(v);
    if (((k ^ prefix) & hi_mask) == 0 && keep(k)) atomicAdd(&hist[(k >> shift) & (nb - 1)], wfn(v));
  });
  __syncthreads();
  // descending inclusive suffix sums: thread t owns bins 2t, 2t+1 (kBins = 2 * threads)
  const int t = threadIdx.x;
  const float h0 = t * 2 < nb ? hist[t * 2] : 0.f, h1 = t * 2 + 1 < nb ? hist[t * 2 + 1] : 0.f;
  float mine = h0 + h1;
  // block suffix scan over threads (descending order = reverse thread order)
  const int lane = t & 63, wv = t >> 6;
  float inc = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {  // inclusive suffix within the wave (lanes >= this lane)
    const float y = __shfl_down(inc, o, 64);
    if (lane + o < 64) inc += y;
  }
  if (lane == 0) scan[wv] = inc;  // wave total
  __syncthreads();
  float after = 0.f;  // total of the waves above this one
  for (int w2 = wv + 1; w2 < kSampThreads / 64; ++w2) after += scan[w2];
  const float suf1 = after + inc - h0;  // suffix including bin 2t+1
  const float suf0 = after + inc;       // suffix including bin 2t
  const float ab = *above;
  if (t == 0) *sel = 0;
  __syncthreads();
  // the digit d with ab + suffix_excl(d) < target <= ab + suffix_incl(d); digit 0 if none
  if (t * 2 + 1 < nb && ab + (suf1 - h1) < target && ab + suf1 >= target) *sel = t * 2 + 1;
  if (t * 2 < nb && ab + (suf0 - h0) < target && ab + suf0 >= target) *sel = t * 2;
  __syncthreads();
  const int d = *sel;
  // weight of the digits above d (suffix excluding d), published by its owner
  if ((d >> 1) == t) scan[32] = (d & 1) ? (suf1 - h1) : (suf0 - h0);
  __syncthreads();
  const float ex = scan[32];
  __syncthreads();
  *above = ab + ex;
  return prefix | ((uint32_t)d << shift);
}

template <typename T>
__global__ void __launch_bounds__(kSampThreads) sample_topkp_kernel(
    const T* __restrict__ logits, int64_t* __restrict__ out, int V, const float* __restrict__ temps,
    const float* __restrict__ top_ps, const int32_t* __restrict__ top_ks, const int64_t* __restrict__ seeds,
    const int32_t* __restrict__ steps) {
  __shared__ float hist[kBins];
  __shared__ float scan[40];
  __shared__ int sel;
  __shared__ float red[16];
  __shared__ int redi[16];
  const int row = blockIdx.x;
  const RowReader<T> rd{logits + (size_t)row * V, V};
  const float temp = temps[row];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t seed = (uint32_t)seeds[row], step = (uint32_t)steps[row];

  // pass 1: max (greedy: argmax directly)
  float best = -INFINITY;
  int bi = 0x7fffffff;
  rd.each([&](int idx, float v) {
    if (v > best || (v == best && idx < bi)) { best = v; bi = idx; }
  });
  auto argmax_reduce = [&](float& b, int& i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(b, o, 64);
      const int oi = __shfl_xor(i, o, 64);
      if (ov > b || (ov == b && oi < i)) { b = ov; i = oi; }
    }
    __syncthreads();
    if (lane == 0) { red[wv] = b; redi[wv] = i; }
    __syncthreads();
    b = red[0];
    i = redi[0];
    for (int w2 = 1; w2 < kSampThreads / 64; ++w2)
      if (red[w2] > b || (red[w2] == b && redi[w2] < i)) { b = red[w2]; i = redi[w2]; }
  };
  argmax_reduce(best, bi);
  if (!(temp > 0.f)) {
    if (threadIdx.x == 0) out[row] = bi;
    return;
  }
  const float mx = best;
  const float c = 1.4426950408889634f / temp;  // exp2 domain
  const float inv_t = 1.f / temp;
  uint32_t thr = 0;  // keep keys >= thr
  const int k = top_ks[row];
  if (k > 0 && k < V) {  // k-th largest key (counts)
    float above = 0.f;
    uint32_t pre = 0;
    pre = radix_digit(rd, hist, scan, &sel, pre, 21, 11, [](uint32_t) { return true; },
                      [](float) { return 1.f; }, &above, (float)k);
    pre = radix_digit(rd, hist, scan, &sel, pre, 10, 11, [](uint32_t) { return true; },
                      [](float) { return 1.f; }, &above, (float)k);
    pre = radix_digit(rd, hist, scan, &sel, pre, 0, 10, [](uint32_t) { return true; },
                      [](float) { return 1.f; }, &above, (float)k);
    thr = pre;
  }
  const float p = top_ps[row];
  if (p < 1.f) {
    // Z over the kept set, then the top-p boundary by mass
    float z = 0.f;
    const uint32_t t0 = thr;
    rd.each([&](int, float v) {
      if (okey(v) >= t0) z += __builtin_amdgcn_exp2f((v - mx) * c);
    });
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) z += __shfl_xor(z, o, 64);
    __syncthreads();
    if (lane == 0) red[wv] = z;
    __syncthreads();
    z = 0.f;
    for (int w2 = 0; w2 < kSampThreads / 64; ++w2) z += red[w2];
    const float target = fmaxf(p, 0.f) * z;
    float above = 0.f;
    uint32_t pre = 0;
    auto keep = [t0](uint32_t kk) { return kk >= t0; };
    auto wf = [mx, c](float v) { return __builtin_amdgcn_exp2f((v - mx) * c); };
    pre = radix_digit(rd, hist, scan, &sel, pre, 21, 11, keep, wf, &above, target);
    pre = radix_digit(rd, hist, scan, &sel, pre, 10, 11, keep, wf, &above, target);
    pre = radix_digit(rd, hist, scan, &sel, pre, 0, 10, keep, wf, &above, target);
    thr = max(thr, pre);
  }
  // Gumbel-max over the kept keys
  const uint32_t tf = thr;
  float gb = -INFINITY;
  int gi = 0x7fffffff;
  rd.each([&](int idx, float v) {
    if (okey(v) < tf) return;
    const uint32_t h = hash3s(seed, step, (uint32_t)idx);  // = decode.hip sample_kernel noise of a 1-row call
    const float u = ((h >> 8) + 0.5f) * (1.0f / 16777216.0f);
    const float s = v * inv_t - __logf(-__logf(u));
    if (s > gb || (s == gb && idx < gi)) { gb = s; gi = idx; }
  });
  argmax_reduce(gb, gi);
  if (threadIdx.x == 0) out[row] = gi < V ? gi : bi;
}

}  // namespace mx

using namespace mx;

// logits [B, V] bf16 (is_bf16) or f32; per-row parameters (device arrays of B):
// temperature f32 (<= 0: greedy), top_p f32 (>= 1: off), top_k i32 (<= 0: off),
// seed i64, step i32.  out ids [B] int64.
extern "C" int mx_sample_rows(const void* logits, int is_bf16, int64_t* out, int B, int V, const float* temps,
                              const float* top_ps, const int32_t* top_ks, const int64_t* seeds, const int32_t* steps,
                              hipStream_t stream) {
  if (B <= 0) return 0;
  if (V <= 0) return -1;
  if (is_bf16)
    sample_topkp_kernel<uint16_t><<<B, kSampThreads, 0, stream>>>((const uint16_t*)logits, out, V, temps, top_ps,
                                                                  top_ks, seeds, steps);
  else
    sample_topkp_kernel<float><<<B, kSampThreads, 0, stream>>>((const float*)logits, out, V, temps, top_ps, top_ks,
                                                               seeds, steps);
  return (int)hipGetLastError();
}
