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
