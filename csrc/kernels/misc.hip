// Small utility kernels:
//  * segmented_mean_i32: SURVEY §2.4 K16 — the batched replacement for the
//    reference's per-prompt `torch.tensor([ord(c)...]).mean().item()`
//    (reference src/utils.py:25-28).  One wave per segment, shuffle reduce.
//  * scale/accumulate helpers used by the trainer (grad scaling, sq-norm).
#include "common.h"

namespace mx {

__global__ void __launch_bounds__(256) segmented_mean_kernel(const int32_t* __restrict__ codes,
                                                             const int64_t* __restrict__ offs,
                                                             float* __restrict__ out, int nseg) {
  const int seg = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (seg >= nseg) return;
  const int64_t b = offs[seg], e = offs[seg + 1];
  // accumulate in f64 per lane: exact for code points (< 2^21) over any length
  double s = 0.0;
  for (int64_t i = b + lane; i < e; i += 64) s += (double)codes[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[seg] = (e > b) ? (float)(s / (double)(e - b)) : NAN;
}

// sum of squares of an f32 or bf16 vector: per-block partials, then ONE block sums
// them in a fixed order -> bitwise identical on every DDP rank (the grad-clip
// coefficient must not differ between replicas), no atomics.
constexpr int kSqBlocks = 2048;

template <typename T>
__global__ void __launch_bounds__(256) sqnorm_partial_kernel(const T* __restrict__ x, int64_t n,
                                                             float* __restrict__ part) {
  __shared__ float scratch[16];
  float s = 0.f;
  constexpr int V = 16 / sizeof(T);  // elements per 16-B load
  const int64_t stride = (int64_t)gridDim.x * 256 * V;
  for (int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * V; i < n; i += stride) {
    if (i + V - 1 < n) {
      if constexpr (sizeof(T) == 4) {
        f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
        s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
      } else {
        u16x8 v = *reinterpret_cast<const u16x8*>(x + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(v[j]);
          s += f * f;
        }
      }
    } else {
      for (int64_t j = i; j < n; ++j) {
        float f;
        if constexpr (sizeof(T) == 4) f = x[j];
        else f = bf2f(x[j]);
        s += f * f;
      }
    }
  }
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(256) sum_partials_kernel(const float* __restrict__ part, int n,
                                                           float* __restrict__ out) {
  __shared__ float scratch[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) out[0] = s;
}

// Batched strided 2-D copy of 16-bit elements: one launch refreshes every LoRA
// adapter's copy inside the augmented GEMM weight buffers after an optimizer
// step (mxllm/models/llama.py, FusedLinear).  desc[i] = {src, dst, rows, cols,
// src_ld, dst_ld, first_block, src_col_stride, dst_col_stride} (column strides != 1
// give transposed copies, e.g. B -> the B^T image of the LoRA backward kernel); block b belongs to the descriptor with the
// largest first_block <= b (binary search), each block copies 4096 elements -- or, for a TRANSPOSING
// descriptor (source rows contiguous, destination a column-major view: dst_ld == 1, dst_col_stride
// != 1), one 64 x 64 tile of the source (row-major tile order) through LDS, so both the reads and
// the writes are row-contiguous (mxllm/ops/linear.py copy2d_plan sizes the blocks the same way).
constexpr int kCopyBlockElems = 4096;

__global__ void __launch_bounds__(256) copy2d_batched_kernel(const int64_t* __restrict__ desc, int n) {
  int lo = 0, hi = n - 1;
  const int64_t b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) / 2;
    if (desc[mid * 9 + 6] <= b) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* d = desc + lo * 9;
  const uint16_t* src = reinterpret_cast<const uint16_t*>(d[0]);
  uint16_t* dst = reinterpret_cast<uint16_t*>(d[1]);
  const int64_t rows = d[2], cols = d[3], sld = d[4], dld = d[5], scs = d[7], dcs = d[8];
  if (scs == 1 && dld == 1 && dcs != 1) {
    // element (r, c) -> dst[c * dcs + r]: source rows in, destination rows (= source columns) out
    __shared__ uint16_t tile[64][66];
    const int64_t tcols = (cols + 63) / 64, t = b - d[6];
    const int64_t r0 = (t / tcols) * 64, c0 = (t % tcols) * 64;
    const int tr = threadIdx.x >> 6, tl = threadIdx.x & 63;
#pragma unroll 4
    for (int rr = tr; rr < 64; rr += 4)
      if (r0 + rr < rows && c0 + tl < cols) tile[rr][tl] = src[(r0 + rr) * sld + c0 + tl];
    __syncthreads();
#pragma unroll 4
    for (int cc = tr; cc < 64; cc += 4)
      if (c0 + cc < cols && r0 + tl < rows) dst[(c0 + cc) * dcs + r0 + tl] = tile[tl][cc];
    return;
  }
  const int64_t e0 = (b - d[6]) * kCopyBlockElems;
  const int64_t total = rows * cols;
  const int64_t e1 = min(total, e0 + kCopyBlockElems);
  // contiguous rows of a multiple of 8 elements on 16-B aligned bases (every LoRA adapter: A rows of
  // `in` elements, B rows of 16): 16-B units that never cross a row, the (row, unit) position
  // advanced by a fixed step instead of a 64-bit division per element (the per-element form took
  // 1.97 ms of the 70B LoRA step, profiles/r5_final/step_breakdown_70b_lora.txt)
  const bool vec = scs == 1 && dcs == 1 && cols % 8 == 0 && sld % 8 == 0 && dld % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  if (vec) {
    const int64_t c8n = cols / 8, u1 = e1 / 8;
    int64_t u = e0 / 8 + threadIdx.x;
    if (u >= u1) return;
    int64_t r = u / c8n, c = u - r * c8n;
    const int64_t dr = 256 / c8n, dc = 256 % c8n;  // dc < c8n: one wrap per step at most
    for (; u < u1; u += 256) {
      *reinterpret_cast<uint4*>(dst + r * dld + 8 * c) = *reinterpret_cast<const uint4*>(src + r * sld + 8 * c);
      c += dc;
      r += dr;
      if (c >= c8n) {
        c -= c8n;
        ++r;
      }
    }
    return;
  }
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const int64_t r = e / cols, c = e - r * cols;
    dst[r * dld + c * dcs] = src[r * sld + c * scs];
  }
}

}  // namespace mx

using namespace mx;

extern "C" int mx_copy2d_batched(const int64_t* desc, int n, int64_t total_blocks, hipStream_t stream) {
  if (n <= 0 || total_blocks <= 0) return 0;
  copy2d_batched_kernel<<<(unsigned)total_blocks, 256, 0, stream>>>(desc, n);
  return (int)hipGetLastError();
}

extern "C" int mx_segmented_mean_i32(const int32_t* codes, const int64_t* offs, float* out, int nseg,
                                     hipStream_t stream) {
  if (nseg <= 0) return 0;
  segmented_mean_kernel<<<(nseg + 3) / 4, 256, 0, stream>>>(codes, offs, out, nseg);
  return (int)hipGetLastError();
}

// out: 1 float; work: kSqBlocks floats.  bf16 != 0: x is bf16.
extern "C" int mx_sqnorm(const void* x, int bf16, int64_t n, float* out, float* work, hipStream_t stream) {
  if (n <= 0) {
    hipMemsetAsync(out, 0, sizeof(float), stream);
    return (int)hipGetLastError();
  }
  const int V = bf16 ? 8 : 4;
  int64_t blocks = (n / V + 255) / 256;
  if (blocks > kSqBlocks) blocks = kSqBlocks;
  if (blocks < 1) blocks = 1;
  if (bf16)
    sqnorm_partial_kernel<uint16_t><<<(int)blocks, 256, 0, stream>>>(reinterpret_cast<const uint16_t*>(x), n, work);
  else
    sqnorm_partial_kernel<float><<<(int)blocks, 256, 0, stream>>>(reinterpret_cast<const float*>(x), n, work);
  sum_partials_kernel<<<1, 256, 0, stream>>>(work, (int)blocks, out);
  return (int)hipGetLastError();
}

// 16-bit 2-D transpose out[c, r] = in[r, c] through a 64x64 LDS tile (full
// fine-tuning dW GEMMs: token-major activations -> token-contiguous images so
// hipBLASLt runs its reduction-contiguous kernel family, mxllm/ops/linear.py).
// 256 threads: 16-B row loads (8 threads per 64-element row, 32 rows per pass),
// 16-B row stores of the transposed tile; row stride 66 halves keeps the
// column reads at <= 2-way bank sharing.  Edge tiles fall back to scalar
// accesses.  Row strides are in elements.
namespace mx {
constexpr int kTrTile = 64;

// scale != nullptr (bf16 data): out = bf16(in * *scale), the scalar read on the device (the
// cross-entropy backward's upstream gradient folded into the dW operand's transpose)
__global__ void __launch_bounds__(256) transpose16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                          int64_t R, int64_t C, int64_t ld_in, int64_t ld_out,
                                                          const float* __restrict__ scale) {
  __shared__ uint16_t tile[kTrTile][kTrTile + 2];
  const float sc = scale ? *scale : 1.f;
  auto cv = [&](uint16_t x) -> uint16_t { return scale ? f2bf(bf2f(x) * sc) : x; };
  const int64_t r0 = (int64_t)blockIdx.y * kTrTile, c0 = (int64_t)blockIdx.x * kTrTile;
  const int t = threadIdx.x, sub = t & 7, row = t >> 3;  // 8 threads x 8 elements per row
  const bool full = (r0 + kTrTile <= R) && (c0 + kTrTile <= C) && (ld_in % 8 == 0) && (ld_out % 8 == 0);
  if (full) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int r = row + 32 * p;
      const u16x8 v = *reinterpret_cast<const u16x8*>(in + (r0 + r) * ld_in + c0 + sub * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[r][sub * 8 + j] = v[j];
    }
  } else {
    for (int e = t; e < kTrTile * kTrTile; e += 256) {
      const int r = e / kTrTile, c = e % kTrTile;
      if (r0 + r < R && c0 + c < C) tile[r][c] = in[(r0 + r) * ld_in + c0 + c];
    }
  }
  __syncthreads();
  if (full) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int c = row + 32 * p;  // output row (input column)
      u16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = cv(tile[sub * 8 + j][c]);
      *reinterpret_cast<u16x8*>(out + (c0 + c) * ld_out + r0 + sub * 8) = v;
    }
  } else {
    for (int e = t; e < kTrTile * kTrTile; e += 256) {
      const int c = e / kTrTile, r = e % kTrTile;
      if (r0 + r < R && c0 + c < C) out[(c0 + c) * ld_out + r0 + r] = cv(tile[r][c]);
    }
  }
}
}  // namespace mx

extern "C" int mx_transpose16(const void* in, void* out, int64_t R, int64_t C, int64_t ld_in, int64_t ld_out,
                              const float* scale, hipStream_t stream) {
  if (R <= 0 || C <= 0) return 0;
  if (ld_in < C || ld_out < R) return -1;
  const int64_t gx = (C + kTrTile - 1) / kTrTile, gy = (R + kTrTile - 1) / kTrTile;
  if (gy > 65535 || gx > 0x7fffffff) return -1;
  transpose16_kernel<<<dim3((unsigned)gx, (unsigned)gy), 256, 0, stream>>>(
      reinterpret_cast<const uint16_t*>(in), reinterpret_cast<uint16_t*>(out), R, C, ld_in, ld_out, scale);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ cache prefetch
// Read a weight tensor once so its lines sit in the memory-side Infinity Cache (and the
// readers' L2s) when the consumer kernel streams it: issued on a side stream beside a
// latency-bound kernel that leaves HBM idle (batch-1 decode attention), so the next
// weight-streaming GEMM reads from the cache instead of HBM.  The loaded values feed an
// XOR that is stored only when `never` (a runtime 0) is set, which keeps every load.
namespace mx {
__global__ void __launch_bounds__(256) prefetch_kernel(const uint4* __restrict__ p, int64_t n16, int never,
                                                       uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {  // four 16-B loads in flight per lane
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (never) sink[blockIdx.x * 256 + threadIdx.x] = acc;
}
}  // namespace mx

extern "C" int mx_prefetch(const void* p, int64_t bytes, int wgs, hipStream_t stream) {
  if (bytes < 16 || wgs <= 0) return 0;
  if ((uintptr_t)p % 16) return -1;
  prefetch_kernel<<<wgs, 256, 0, stream>>>(reinterpret_cast<const uint4*>(p), bytes / 16, 0, nullptr);
  return (int)hipGetLastError();
}
