// Bulk peer-memory collectives inside one MI355X node: direct
// one-hop reduce-scatter / all-gather (and all-reduce = the two back to back)
// where every rank talks to all of its peers at once.
//
// Why not a ring: each MI355X has 7 point-to-point xGMI links, one per peer, so
// a ring moves every byte over ONE link per hop.  Here rank r PUSHES, for every
// peer d, the slice of its input that d owns into a staging slot in d's memory
// (7 concurrent link writes), raises one flag per (workgroup, peer) and then
// reduces (RS) or copies out (AG) the slots its peers pushed into its own
// staging.  Bytes per rank: (W-1)/W of the tensor out and in for RS, the same
// for AG: the bandwidth-optimal amount, spread over all W-1 links.
//
// The same kernels run W ranks as W PROCESSES on ONE GPU (the IPC "peer" is
// the same HBM mapped twice): that is how the multi-rank trainers are tested
// with stream-ordered collective semantics on a 1-GPU box.
//
// Staging (each rank; hipDeviceMallocUncached, exchanged once by IPC handle):
//   flags [kMaxWG][kMaxRanks] x 64 B   flag of source s for workgroup g: epoch
//   slots [G][2][W][slot_bytes]        (g, half, src): what rank src pushed to me
// Workgroup g walks pieces k = g, g + G, ... of the per-rank chunk (slot_bytes
// each); every piece is a complete exchange among the W ranks, so parity
// double-buffering is enough: a source can write half h again (epoch e + 2)
// only after it saw my flag e + 1, which I raise after consuming epoch e.
// Epochs live in device memory per workgroup (identical on every rank as long
// as every rank issues the same sequence of calls, as for any collective).
//
// Memory protocol (MI355X_MICROARCH "inter-workgroup visibility"), at SYSTEM
// scope because the consumer is another process / GPU: producer = stores ->
// every wave s_waitcnt vmcnt(0) -> barrier -> fence(release) -> asm vmcnt(0)
// -> relaxed flag store; consumer = relaxed poll -> fence(acquire) -> vmcnt(0)
// -> barrier -> loads.  Every spin is bounded (s_memrealtime, 100 MHz): on
// timeout the error word is set and the workgroup stops.
//
// Reduction: fp32, in rank order 0..W-1 -> every rank computes the identical
// bits for its chunk, and an all-reduce (RS + AG) is bitwise identical on all
// ranks.
//
// Failure: once the error word is set, no collective result is
// silently partial -- a launch that finds it set at entry, and a workgroup
// whose spin timed out, fill the output they own with NaN (so nothing that
// consumes it can look valid) and stop; the host side checks the word after
// synchronising on the communicator's last collective before the optimizer
// reads a result (mxllm/parallel/comm.py ``verify``).
#include "common.h"

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxWG = 64;
constexpr int kFlagStride = 16;  // uint32 words = 64 B per flag
constexpr size_t kFlagBytes = (size_t)kMaxWG * kMaxRanks * kFlagStride * sizeof(uint32_t);

struct Bases {
  char* b[kMaxRanks];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
__device__ __forceinline__ float ld_f(const T* p);
template <>
__device__ __forceinline__ float ld_f<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld_f<uint16_t>(const uint16_t* p) { return mx::bf2f(*p); }

// 16 B of T <-> 4 / 8 floats
template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void add(float* acc, u32x4 v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += __uint_as_float(v[j]);
  }
  __device__ static u32x4 pack(const float* acc) {
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = __float_as_uint(acc[j]);
    return o;
  }
};
template <>
struct Vec<uint16_t> {
  static constexpr int N = 8;
  __device__ static void add(float* acc, u32x4 v) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[2 * j] += __uint_as_float(v[j] << 16);
      acc[2 * j + 1] += __uint_as_float(v[j] & 0xFFFF0000u);
    }
  }
  __device__ static u32x4 pack(const float* acc) {
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = mx::pack_bf16x2(acc[2 * j], acc[2 * j + 1]);
    return o;
  }
};

// NaN over out [lo, hi) (16-B vectors), grid-strided with stride `step` vectors starting at `first`.
template <typename T>
__device__ __forceinline__ void poison(T* out, int64_t lo, int64_t hi, int64_t first, int64_t step) {
  constexpr int V = Vec<T>::N;
  const uint32_t w = sizeof(T) == 4 ? 0x7FC00000u : 0x7FC07FC0u;
  const u32x4 nan = {w, w, w, w};
  for (int64_t i = lo + first * V; i < hi; i += step * V) *reinterpret_cast<u32x4*>(out + i) = nan;
}

__device__ __forceinline__ uint32_t* flag_ptr(char* base, int g, int src) {
  return reinterpret_cast<uint32_t*>(base) + ((size_t)g * kMaxRanks + src) * kFlagStride;
}

// MODE 0: reduce-scatter  in [n] (chunk d = in[d*m, (d+1)*m), zero past n)  -> out [m]
// MODE 1: all-gather      in [m]                                              -> out [n] (out[p*m + i], < n)
// n, m are multiples of the 16-B vector (V elements); slot_bytes a multiple of 4 KB.
template <typename T, int MODE>
__global__ __launch_bounds__(256) void peer_coll_kernel(Bases P, const T* __restrict__ in, T* __restrict__ out,
                                                        int64_t n, int64_t m, int rank, int world, int slot_bytes,
                                                        uint32_t* __restrict__ epochs, int* err,
                                                        long long timeout_ticks) {
  constexpr int V = Vec<T>::N;
  __shared__ int bad;
  const int g = blockIdx.x, G = gridDim.x, tid = threadIdx.x;
  const int slot_elems = slot_bytes / (int)sizeof(T);
  const int64_t npieces = (m + slot_elems - 1) / slot_elems;
  // a communicator already broken (a peer timed out earlier): poison, move nothing, keep the epochs
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
    poison(out, 0, MODE == 0 ? m : n, (int64_t)g * 256 + tid, (int64_t)G * 256);
    return;
  }
  uint32_t epoch = epochs[g];
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int64_t k = g; k < npieces; k += G) {
    ++epoch;
    const int half = epoch & 1u;
    const int64_t o = k * (int64_t)slot_elems;
    const int len = (int)min((int64_t)slot_elems, m - o);
    // 1. push my data for every peer d into slot (g, half, rank) of d's staging
    for (int j = 1; j < world; ++j) {
      const int d = (rank + j) % world;
      T* slot = reinterpret_cast<T*>(P.b[d] + kFlagBytes + (((size_t)g * 2 + half) * world + rank) * slot_bytes);
      const int64_t src0 = MODE == 0 ? (int64_t)d * m + o : o;
      const int64_t lim = MODE == 0 ? n - src0 : m - o;  // valid elements from src0 on (RS: zero past n)
      for (int i = tid * V; i < len; i += 256 * V) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (i < lim) v = *reinterpret_cast<const u32x4*>(in + src0 + i);
        *reinterpret_cast<u32x4*>(slot + i) = v;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // 2. lane d raises my flag in rank d's staging (system-scope release)
    if (tid < world && tid != rank) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flag_ptr(P.b[tid], g, rank), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // 3. lane p waits for rank p's flag in my staging (bounded), then acquires
    if (tid < world && tid != rank) {
      const uint32_t* f = flag_ptr(P.b[rank], g, tid);
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
          bad = 1;
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (bad) {  // this workgroup's pieces from k on are never exchanged: poison them
      for (int64_t q = k; q < npieces; q += G) {
        const int64_t qo = q * (int64_t)slot_elems, qe = min(qo + (int64_t)slot_elems, m);
        if (MODE == 0) {
          poison(out, qo, qe, tid, 256);
        } else {
          for (int p = 0; p < world; ++p) {
            const int64_t b0 = (int64_t)p * m;
            poison(out, b0 + qo, min(b0 + qe, n), tid, 256);
          }
        }
      }
      break;
    }
    // 4. consume the W slots of this piece (my own contribution straight from `in`)
    const T* mine = reinterpret_cast<const T*>(P.b[rank] + kFlagBytes + ((size_t)g * 2 + half) * world * slot_bytes);
    if (MODE == 0) {
      for (int i = tid * V; i < len; i += 256 * V) {
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        for (int p = 0; p < world; ++p) {
          u32x4 v = {0u, 0u, 0u, 0u};
          if (p == rank) {
            const int64_t s = (int64_t)rank * m + o + i;
            if (s < n) v = *reinterpret_cast<const u32x4*>(in + s);
          } else {
            v = *reinterpret_cast<const u32x4*>(mine + (size_t)p * slot_elems + i);
          }
          Vec<T>::add(acc, v);
        }
        *reinterpret_cast<u32x4*>(out + o + i) = Vec<T>::pack(acc);
      }
    } else {
      for (int p = 0; p < world; ++p) {
        const T* src = p == rank ? in + o : mine + (size_t)p * slot_elems;
        T* dst = out + (int64_t)p * m + o;
        const int64_t lim = n - ((int64_t)p * m + o);
        for (int i = tid * V; i < len && i < lim; i += 256 * V)
          *reinterpret_cast<u32x4*>(dst + i) = *reinterpret_cast<const u32x4*>(src + i);
      }
    }
  }
  __syncthreads();
  if (tid == 0) epochs[g] = epoch;
}

template <typename T>
int launch(int mode, char* const* bases, const void* in, void* out, int64_t n, int64_t m, int rank, int world,
           int wgs, int slot_bytes, uint32_t* epochs, int* err, long long timeout_ticks, hipStream_t s) {
  Bases P{};
  for (int r = 0; r < world; ++r) {
    if (!bases[r]) return -1;
    P.b[r] = bases[r];
  }
  const int64_t slot_elems = slot_bytes / (int64_t)sizeof(T);
  const int64_t npieces = (m + slot_elems - 1) / slot_elems;
  const int G = (int)std::min<int64_t>(wgs, std::max<int64_t>(1, npieces));
  if (mode == 0)
    peer_coll_kernel<T, 0><<<G, 256, 0, s>>>(P, (const T*)in, (T*)out, n, m, rank, world, slot_bytes, epochs, err,
                                              timeout_ticks);
  else
    peer_coll_kernel<T, 1><<<G, 256, 0, s>>>(P, (const T*)in, (T*)out, n, m, rank, world, slot_bytes, epochs, err,
                                              timeout_ticks);
  return (int)hipGetLastError();
}

// ============================================================================================
// CU-light schedule (VERDICT r5 Missing 4): no workgroup waits on a peer except ONE wave.
// The resident kernel above keeps `wgs` workgroups spinning on peer flags for the whole call
// (24.5 % off a concurrent GEMM at 32 WGs, profiles/r5j).  Here a call is cut into segments of
// at most `cap` bytes per peer, and each segment with host epoch e (identical on every rank:
// every rank issues the same calls) is four stream-ordered launches:
//   1. pc_wait    (1 wave)  every peer has acknowledged epoch e-2 in my ack words (it has consumed
//                           what I pushed into its half e & 1 two segments ago; usually true at once)
//   2. pc_push    (G WGs)   my slices -> every peer's slot [e & 1][rank] (converted to the wire type:
//                           fp32 gradients travel as bf16 with `wire` = bf16); the last workgroup
//                           to retire raises ready[rank] = e in every peer's flag words
//   3. pc_wait    (1 wave)  ready[p] >= e in my flag words for every peer p
//   4. pc_consume (G WGs)   RS: out = fp32 sum over ranks 0..W-1 of the wire values (my own slice
//                           rounded to the wire type too, so every rank's bits are identical);
//                           AG: copies out; the last workgroup raises ack[rank] = e at every peer
// Push and consume are plain streaming kernels that exit, so between them the CUs belong to the
// compute stream.  Visibility: every thread's stores -> system-scope release fence -> barrier ->
// one acq_rel ticket; the last ticket holder raises the flags with system-scope release stores;
// the staging is uncached device memory, read by a kernel launched after the wave that saw the
// flag.  A timed-out wait sets the host error word and a device `dead` word; push and consume
// check `dead` at entry and then move nothing and fill their output with NaN.
// Light area of every staging buffer (after the resident flags and slots, so the resident
// kernel's addressing is unchanged): words ready[kMaxRanks], ack[kMaxRanks], cnt_push,
// cnt_consume, dead (64 B apart, kLightFlagBytes), then the slots [2][W][cap] (half, source).
// The light kernels get the LIGHT-area base of every rank in their Bases.
constexpr size_t kLightFlagBytes = 4096;
enum { kLReady = 0, kLAck = kMaxRanks, kLCntPush = 2 * kMaxRanks, kLCntCons, kLDead };

__device__ __forceinline__ uint32_t* lword(char* lbase, int idx) {
  return reinterpret_cast<uint32_t*>(lbase) + (size_t)idx * kFlagStride;
}

// 8 elements <-> 8 floats (exact for bf16 <-> fp32 widening, round-to-nearest-even narrowing).  Default
// cache policy: non-temporal loads / stores (and 8 items in flight) measured slower here, with no
// smaller GEMM slowdown beside them (profiles/r6b/README.md).
__device__ __forceinline__ u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
__device__ __forceinline__ void st16(void* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const u32x4 a = ld16(p), b = ld16(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = __uint_as_float(a[j]), v[4 + j] = __uint_as_float(b[j]);
}
__device__ __forceinline__ void ld8(const uint16_t* p, float (&v)[8]) {
  const u32x4 a = ld16(p);
#pragma unroll
  for (int j = 0; j < 4; ++j) v[2 * j] = __uint_as_float(a[j] << 16), v[2 * j + 1] = __uint_as_float(a[j] & 0xFFFF0000u);
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  u32x4 a, b;
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = __float_as_uint(v[j]), b[j] = __float_as_uint(v[4 + j]);
  st16(p, a);
  st16(p + 4, b);
}
__device__ __forceinline__ void st8(uint16_t* p, const float (&v)[8]) {
  u32x4 a;
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = mx::pack_bf16x2(v[2 * j], v[2 * j + 1]);
  st16(p, a);
}
template <typename W>
__device__ __forceinline__ void round_to(float (&v)[8]) {
  if constexpr (sizeof(W) == 2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = mx::bf2f(mx::f2bf(v[j]));
  }
}
__device__ __forceinline__ void nan8(float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(0x7FC00000u);
}

struct LightSeg {
  int64_t n, m, o;  // full input / chunk elements, this segment's offset in the chunk
  int len;          // elements of this segment (multiple of 8)
  int rank, world, half;
  uint32_t epoch;
  int64_t cap;  // bytes per slot
};

__device__ __forceinline__ bool light_dead(char* mine) {
  return __hip_atomic_load(lword(mine, kLDead), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// the last of gridDim.x workgroups to arrive on ticket `cnt` raises word `flag_idx` (+ rank) = epoch
// in every peer's flag area
__device__ __forceinline__ void light_raise(const Bases& P, const LightSeg& g, int cnt, int flag_idx) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this thread's stores are visible
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* c = lword(P.b[g.rank], cnt);
    const uint32_t prev = __hip_atomic_fetch_add(c, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next call starts from 0
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      for (int j = 1; j < g.world; ++j) {
        const int d = (g.rank + j) % g.world;
        __hip_atomic_store(lword(P.b[d], flag_idx + g.rank), g.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// one wave: lane p (!= rank, < world) waits until word base_idx + p of MY flag area reaches `target`
__global__ __launch_bounds__(64) void pc_wait_kernel(Bases P, int base_idx, uint32_t target, int rank, int world,
                                                      int* err, long long timeout_ticks) {
  const int p = threadIdx.x;
  char* mine = P.b[rank];
  if (p >= world || p == rank) return;
  const uint32_t* f = lword(mine, base_idx + p);
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target) < 0) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(lword(mine, kLDead), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// Both streaming kernels keep kLU (4) 8-element items per thread in flight (all loads of a group issued
// before its stores): one 8-element item per thread is only ~8 KB per workgroup in flight, a few GB/s
// per CU at HBM latency, so a given rate would need many more workgroups -- CUs taken from the
// compute stream.  Items are numbered q = item * 8 elements; thread t of workgroup b takes
// q = (b * kLU + u) * 256 + t, u < kLU, then strides by gridDim.x * kLU * 256.
constexpr int kLU = 4;

// MODE 0: reduce-scatter (slice for d = in[d*m + o, +len), zero past n); MODE 1: all-gather (in[o, +len))
template <typename T, typename W, int MODE>
__global__ __launch_bounds__(256) void pc_push_kernel(Bases P, const T* __restrict__ in, LightSeg g) {
  char* mine = P.b[g.rank];
  if (light_dead(mine)) return;  // never raise flags on a dead communicator: peers must not take garbage
  const int64_t len8 = g.len / 8, total = (int64_t)(g.world - 1) * len8;
  const int64_t step = (int64_t)gridDim.x * kLU * 256;
  for (int64_t q0 = (int64_t)blockIdx.x * kLU * 256 + threadIdx.x; q0 < total; q0 += step) {
    float v[kLU][8];
    W* dst[kLU];
#pragma unroll
    for (int u = 0; u < kLU; ++u) {
      const int64_t q = q0 + u * 256;
      dst[u] = nullptr;
      if (q >= total) continue;
      const int j = (int)(q / len8) + 1;
      const int64_t i = (q - (int64_t)(j - 1) * len8) * 8;
      const int d = (g.rank + j) % g.world;
      const int64_t src = (MODE == 0 ? (int64_t)d * g.m : 0) + g.o + i;
      if (MODE == 1 || src < g.n) {
        ld8(in + src, v[u]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
      }
      dst[u] = reinterpret_cast<W*>(P.b[d] + kLightFlagBytes + ((int64_t)g.half * g.world + g.rank) * g.cap) + i;
    }
#pragma unroll
    for (int u = 0; u < kLU; ++u)
      if (dst[u]) st8(dst[u], v[u]);
  }
  light_raise(P, g, kLCntPush, kLReady);
}

template <typename T, typename W, typename TO, int MODE>
__global__ __launch_bounds__(256) void pc_consume_kernel(Bases P, const T* __restrict__ in, TO* __restrict__ out,
                                                         LightSeg g) {
  char* mine = P.b[g.rank];
  const bool dead = light_dead(mine);
  const int64_t len8 = g.len / 8;
  const W* slots = reinterpret_cast<const W*>(mine + kLightFlagBytes + (int64_t)g.half * g.world * g.cap);
  const int64_t slot_elems = g.cap / (int64_t)sizeof(W);
  const int64_t step = (int64_t)gridDim.x * kLU * 256;
  if (MODE == 0) {
    for (int64_t q0 = (int64_t)blockIdx.x * kLU * 256 + threadIdx.x; q0 < len8; q0 += step) {
      float acc[kLU][8];
#pragma unroll
      for (int u = 0; u < kLU; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[u][e] = dead ? __uint_as_float(0x7FC00000u) : 0.f;
      if (!dead) {
        for (int p = 0; p < g.world; ++p) {  // rank order: every rank's bits identical
          float v[kLU][8];
#pragma unroll
          for (int u = 0; u < kLU; ++u) {
            const int64_t q = q0 + u * 256;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
            if (q >= len8) continue;
            const int64_t i = q * 8;
            if (p == g.rank) {
              const int64_t s = (int64_t)g.rank * g.m + g.o + i;
              if (s < g.n) ld8(in + s, v[u]);
            } else {
              ld8(slots + (int64_t)p * slot_elems + i, v[u]);
            }
          }
#pragma unroll
          for (int u = 0; u < kLU; ++u) {
            if (p == g.rank) round_to<W>(v[u]);  // my own slice as the wire carries the others'
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[u][e] += v[u][e];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kLU; ++u)
        if (q0 + u * 256 < len8) st8(out + g.o + (q0 + u * 256) * 8, acc[u]);
    }
  } else {
    const int64_t total = (int64_t)g.world * len8;
    for (int64_t q0 = (int64_t)blockIdx.x * kLU * 256 + threadIdx.x; q0 < total; q0 += step) {
      float v[kLU][8];
      int64_t dst[kLU];
#pragma unroll
      for (int u = 0; u < kLU; ++u) {
        const int64_t q = q0 + u * 256;
        dst[u] = -1;
        if (q >= total) continue;
        const int p = (int)(q / len8);
        const int64_t i = (q - (int64_t)p * len8) * 8, d = (int64_t)p * g.m + g.o + i;
        if (d >= g.n) continue;
        dst[u] = d;
        if (dead) nan8(v[u]);
        else if (p == g.rank) ld8(in + g.o + i, v[u]);
        else ld8(slots + (int64_t)p * slot_elems + i, v[u]);
      }
#pragma unroll
      for (int u = 0; u < kLU; ++u)
        if (dst[u] >= 0) st8(out + dst[u], v[u]);
    }
  }
  if (!dead) light_raise(P, g, kLCntCons, kLAck);
}

template <typename T, typename W, typename TO>
int light_launch(int mode, const Bases& P, const void* in, void* out, int64_t n, int64_t m, int rank, int world,
                 int wgs, int64_t cap, uint32_t* epoch, int* err, long long timeout_ticks, hipStream_t s) {
  const int64_t seg = cap / (int64_t)sizeof(W);  // elements per peer per segment (multiple of 8)
  for (int64_t o = 0; o < m; o += seg) {
    LightSeg g;
    g.n = n, g.m = m, g.o = o, g.len = (int)std::min<int64_t>(seg, m - o);
    g.rank = rank, g.world = world;
    g.epoch = ++*epoch;
    g.half = (int)(g.epoch & 1u);
    g.cap = cap;
    const int64_t work = (mode == 0 ? (int64_t)1 : (int64_t)world) * (g.len / 8);  // consume items
    const int G = (int)std::max<int64_t>(1, std::min<int64_t>(wgs, (work + kLU * 256 - 1) / (kLU * 256)));
    if (g.epoch > 2) pc_wait_kernel<<<1, 64, 0, s>>>(P, kLAck, g.epoch - 2, rank, world, err, timeout_ticks);
    const int Gp = (int)std::max<int64_t>(
        1, std::min<int64_t>(wgs, ((int64_t)(world - 1) * (g.len / 8) + kLU * 256 - 1) / (kLU * 256)));
    if (mode == 0) pc_push_kernel<T, W, 0><<<Gp, 256, 0, s>>>(P, (const T*)in, g);
    else pc_push_kernel<T, W, 1><<<Gp, 256, 0, s>>>(P, (const T*)in, g);
    pc_wait_kernel<<<1, 64, 0, s>>>(P, kLReady, g.epoch, rank, world, err, timeout_ticks);
    if (mode == 0) pc_consume_kernel<T, W, TO, 0><<<G, 256, 0, s>>>(P, (const T*)in, (TO*)out, g);
    else pc_consume_kernel<T, W, TO, 1><<<G, 256, 0, s>>>(P, (const T*)in, (TO*)out, g);
  }
  return (int)hipGetLastError();
}

}  // namespace

// Staging bytes one rank allocates for the resident schedule (world, wgs, slot_bytes).
extern "C" size_t mx_peer_staging_bytes(int world, int wgs, int slot_bytes) {
  return kFlagBytes + (size_t)wgs * 2 * world * slot_bytes;
}
// ... plus the light area (light_cap bytes per slot; 0 = none).  The light area starts at
// mx_peer_staging_bytes(world, wgs, slot_bytes), 4 KB aligned.
extern "C" size_t mx_peer_staging_bytes2(int world, int wgs, int slot_bytes, int64_t light_cap) {
  const size_t res = (mx_peer_staging_bytes(world, wgs, slot_bytes) + 4095) / 4096 * 4096;
  return light_cap > 0 ? res + kLightFlagBytes + (size_t)2 * world * light_cap : res;
}

// CU-light collective (see above) over the light areas `lbases` (one per rank).  mode 0 = reduce-scatter
// (sum), 1 = all-gather.  dtype / wire: 0 = fp32, 1 = bf16; the output has the input's dtype.  Supported:
// wire == dtype, or a reduce-scatter with fp32 in, bf16 on the wire, fp32 out.  n, m multiples of 8
// elements, m * world >= n, 16-B aligned pointers, light_cap a multiple of 4 KB.  `epoch`: this
// communicator's host segment counter (advanced here); `wgs`: workgroups of the push / consume kernels.
extern "C" int mx_peer_collective_light(int mode, int dtype, int wire, char* const* lbases, const void* in, void* out,
                                        int64_t n, int64_t m, int rank, int world, int wgs, int64_t light_cap,
                                        uint32_t* epoch, int* err, long long timeout_ticks, hipStream_t stream) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || wgs < 1 || wgs > 4096 || light_cap < 4096 ||
      light_cap % 4096 || n < 0 || m < 0 || n % 8 || m % 8 || (mode != 0 && mode != 1) || m * world < n ||
      dtype < 0 || dtype > 1 || wire < 0 || wire > 1 || (wire != dtype && !(mode == 0 && dtype == 0 && wire == 1)))
    return -1;
  if (((uintptr_t)in | (uintptr_t)out) & 15) return -1;
  if (m == 0) return 0;
  Bases P{};
  for (int r = 0; r < world; ++r) {
    if (!lbases[r]) return -1;
    P.b[r] = lbases[r];
  }
  if (dtype == 0 && wire == 0)
    return light_launch<float, float, float>(mode, P, in, out, n, m, rank, world, wgs, light_cap, epoch, err,
                                             timeout_ticks, stream);
  if (dtype == 1)
    return light_launch<uint16_t, uint16_t, uint16_t>(mode, P, in, out, n, m, rank, world, wgs, light_cap, epoch, err,
                                                      timeout_ticks, stream);
  return light_launch<float, uint16_t, float>(mode, P, in, out, n, m, rank, world, wgs, light_cap, epoch, err,
                                              timeout_ticks, stream);
}

// mode 0 = reduce-scatter (sum), 1 = all-gather; dtype 0 = fp32, 1 = bf16.
// Requirements (checked by the caller): 1 < world <= 16, wgs <= 64, slot_bytes % 4096 == 0,
// n and m multiples of 16 B of the dtype, m * world >= n, 16-B aligned pointers.
extern "C" int mx_peer_collective(int mode, int dtype, char* const* bases, const void* in, void* out, int64_t n,
                                  int64_t m, int rank, int world, int wgs, int slot_bytes, uint32_t* epochs, int* err,
                                  long long timeout_ticks, hipStream_t stream) {
  if (world < 2 || world > kMaxRanks || rank < 0 || rank >= world || wgs < 1 || wgs > kMaxWG || slot_bytes % 4096 ||
      n < 0 || m < 0 || (mode != 0 && mode != 1))
    return -1;
  if (m == 0) return 0;
  if (dtype == 0) return launch<float>(mode, bases, in, out, n, m, rank, world, wgs, slot_bytes, epochs, err,
                                       timeout_ticks, stream);
  if (dtype == 1) return launch<uint16_t>(mode, bases, in, out, n, m, rank, world, wgs, slot_bytes, epochs, err,
                                          timeout_ticks, stream);
  return -1;
}
