// One-shot all-reduce / barrier over xGMI peer memory for latency-bound
// messages: loss / token-count / grad-norm scalars,
// parameter checksums, and a device-side barrier.
//
// The reference issues exactly one collective, a 1-element NCCL barrier
// (reference src/distributed_inference.py:18).  On an 8x MI355X node every GPU
// has a direct xGMI link to every peer, so for a few hundred bytes a ring is
// the wrong shape: each rank PUSHES its values into a slot of every peer's
// buffer (7 concurrent link writes), raises a flag in each peer, waits for the
// world's flags in its own buffer and reduces locally.  One kernel launch, one
// hop of link latency, no RCCL channel setup.
//
// Buffer of each rank (hipExtMallocWithFlags(hipDeviceMallocUncached): loads
// and stores bypass the caches, so peers' writes are visible after the acquire):
//   flags  [kMaxRanks] x 64 B   (flag of rank r at word r*16, monotonic epoch)
//   data   [2][world][max_elems] f32  (double-buffered by epoch parity)
// Parity is enough: a rank reaches epoch e+2 only after every peer raised its
// e+1 flag, i.e. after every peer finished reading epoch e's half.
//
// Every spin is bounded (s_memrealtime, 100 MHz): on timeout the kernel sets
// the host-mapped error word, writes NaN results and exits, so a dead peer
// cannot leave waves running on the GPU.
#include "common.h"

namespace {

constexpr int kMaxRanks = 16;
constexpr int kFlagStride = 16;  // uint32 words = 64 B per flag

struct Peers {
  uint32_t* flags[kMaxRanks];
  float* data[kMaxRanks];
};

template <int OP>
__device__ __forceinline__ float combine(float a, float b) {
  if constexpr (OP == 0) return a + b;
  if constexpr (OP == 1) return fmaxf(a, b);
  return fminf(a, b);
}

template <int OP>
__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(Peers peers, const float* __restrict__ in,
                                                             float* __restrict__ out, int n, int rank, int world,
                                                             uint32_t epoch, int max_elems, int* err,
                                                             long long timeout_ticks) {
  __shared__ int timed_out;
  const int tid = threadIdx.x;
  if (tid == 0) timed_out = 0;
  const size_t half = epoch & 1u;

  // 1. push my values into slot [half][rank] of every rank (self included)
  for (int p = 0; p < world; ++p) {
    float* dst = peers.data[p] + (half * world + rank) * (size_t)max_elems;
    for (int i = tid; i < n; i += blockDim.x) dst[i] = in[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 2. lane p publishes to rank p: system-scope release, then the flag
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(peers.flags[tid] + rank * kFlagStride, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }

  // 3. lane r waits for rank r's flag in my buffer (bounded)
  if (tid < world) {
    const uint32_t* f = peers.flags[rank] + tid * kFlagStride;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        timed_out = 1;
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();

  // 4. reduce in rank order: every rank computes the identical (bitwise) result
  const float* src = peers.data[rank] + half * world * (size_t)max_elems;
  const bool bad = timed_out != 0;
  for (int i = tid; i < n; i += blockDim.x) {
    float a = src[i];
    for (int r = 1; r < world; ++r) a = combine<OP>(a, src[(size_t)r * max_elems + i]);
    out[i] = bad ? __builtin_nanf("") : a;
  }
}

}  // namespace

extern "C" int mx_xgmi_allreduce(uint32_t* const* flags, float* const* data, const float* in, float* out, int n,
                                 int rank, int world, uint32_t epoch, int max_elems, int op, int* err,
                                 long long timeout_ticks, hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || n < 0 || n > max_elems) return -1;
  Peers p{};
  for (int r = 0; r < world; ++r) {
    if (!flags[r] || !data[r]) return -1;
    p.flags[r] = flags[r];
    p.data[r] = data[r];
  }
  dim3 grid(1), block(256);
  if (op == 0)
    xgmi_allreduce_kernel<0><<<grid, block, 0, stream>>>(p, in, out, n, rank, world, epoch, max_elems, err,
                                                         timeout_ticks);
  else if (op == 1)
    xgmi_allreduce_kernel<1><<<grid, block, 0, stream>>>(p, in, out, n, rank, world, epoch, max_elems, err,
                                                         timeout_ticks);
  else if (op == 2)
    xgmi_allreduce_kernel<2><<<grid, block, 0, stream>>>(p, in, out, n, rank, world, epoch, max_elems, err,
                                                         timeout_ticks);
  else
    return -1;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------
// Graph-safe bf16 one-shot all-reduce for tensor-parallel decode
// (mxllm/parallel/tensor.py: two [tokens, hidden] partial-sum reductions per
// layer, 16 KB per sequence for 70B — latency-bound).
//
// Differences from the scalar kernel above:
//  * the epoch lives in DEVICE memory (one counter per workgroup, private to
//    this rank): the kernel reads it, uses epoch+1 and writes it back, so the
//    launch arguments never change and the kernel can be captured once into
//    the decode hipGraph and replayed (a host-side epoch would be frozen into
//    the graph);
//  * G workgroups each own a contiguous chunk and a private flag row
//    flags[g][rank] in every peer buffer, so chunks proceed independently and
//    the push to the 7 peers uses many CUs' store queues;
//  * data is bf16 (16-B vector pushes), reduced in f32 in rank order then
//    rounded once: every rank gets the bitwise-identical result.
// Parity double-buffering per workgroup as above.  Bounded spins (timeout ->
// error word + NaN output).
namespace {
using mx::bf2f;
using mx::f2bf;
using mx::u16x8;

constexpr int kMaxWG = 64;

struct PeersBf {
  uint32_t* flags[kMaxRanks];   // [kMaxWG][kMaxRanks] x 64 B
  uint16_t* data[kMaxRanks];    // [2][world][max_elems] bf16
};

__global__ __launch_bounds__(256) void xgmi_allreduce_bf16_kernel(PeersBf peers, const uint16_t* __restrict__ in,
                                                                 uint16_t* __restrict__ out, int n, int chunk,
                                                                 int rank, int world, int max_elems,
                                                                 uint32_t* __restrict__ epochs, int* err,
                                                                 long long timeout_ticks) {
  __shared__ int timed_out;
  const int tid = threadIdx.x, g = blockIdx.x;
  const uint32_t epoch = epochs[g] + 1u;
  if (tid == 0) timed_out = 0;
  const size_t half = epoch & 1u;
  const int lo = g * chunk, hi = min(n, lo + chunk);

  // 1. push my chunk into slot [half][rank] of every rank (16-B vectors; n, chunk % 8 == 0)
  for (int i = lo + tid * 8; i < hi; i += 256 * 8) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(in + i);
    for (int p = 0; p < world; ++p)
      *reinterpret_cast<u16x8*>(peers.data[p] + (half * world + rank) * (size_t)max_elems + i) = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // 2. lane p publishes this chunk's flag to rank p (system-scope release)
  if (tid < world) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(peers.flags[tid] + ((size_t)g * kMaxRanks + rank) * kFlagStride, epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. lane r waits for rank r's flag of this chunk in my buffer (bounded)
  if (tid < world) {
    const uint32_t* f = peers.flags[rank] + ((size_t)g * kMaxRanks + tid) * kFlagStride;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        timed_out = 1;
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();

  // 4. reduce in rank order (f32), round once
  const uint16_t* src = peers.data[rank] + half * world * (size_t)max_elems;
  const bool bad = timed_out != 0;
  for (int i = lo + tid * 8; i < hi; i += 256 * 8) {
    float acc[8];
    const u16x8 v0 = *reinterpret_cast<const u16x8*>(src + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bf2f(v0[j]);
    for (int r = 1; r < world; ++r) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(src + (size_t)r * max_elems + i);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bad ? (uint16_t)0x7FC0 : f2bf(acc[j]);
    *reinterpret_cast<u16x8*>(out + i) = o;
  }
  if (tid == 0) epochs[g] = epoch;
}

}  // namespace

// flags/data: per-rank base pointers of the peer buffers; epochs: kMaxWG device
// counters of THIS rank.  Requires n % 8 == 0, n <= max_elems.
extern "C" int mx_xgmi_allreduce_bf16(uint32_t* const* flags, uint16_t* const* data, const uint16_t* in,
                                      uint16_t* out, int n, int rank, int world, int max_elems, uint32_t* epochs,
                                      int* err, long long timeout_ticks, hipStream_t stream) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || n <= 0 || n > max_elems || n % 8) return -1;
  PeersBf p{};
  for (int r = 0; r < world; ++r) {
    if (!flags[r] || !data[r]) return -1;
    p.flags[r] = flags[r];
    p.data[r] = data[r];
  }
  int G = (n + 2047) / 2048;
  if (G > kMaxWG) G = kMaxWG;
  int chunk = (n + G - 1) / G;
  chunk = (chunk + 7) / 8 * 8;
  G = (n + chunk - 1) / chunk;
  xgmi_allreduce_bf16_kernel<<<G, 256, 0, stream>>>(p, in, out, n, chunk, rank, world, max_elems, epochs, err,
                                                    timeout_ticks);
  return (int)hipGetLastError();
}
