// CU-mask probe (one MI355X): which CUs / XCDs a stream created with
// hipExtStreamCreateWithCUMask runs on, and the HBM bandwidth an AdamW-shaped
// streaming kernel reaches when confined to that subset.
//
// Build: hipcc -O3 --offload-arch=gfx950 bench/cu_mask_probe.hip -o build/cu_mask_probe
// Prints one JSON line per mask.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// one record per workgroup: XCC id (0-7) and HW_ID (CU / SH / SE fields)
__global__ void where_kernel(uint32_t* out) {
  if (threadIdx.x == 0) {
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
  // keep the workgroup alive long enough that the dispatcher spreads the grid
  for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(1);
}

// AdamW-shaped traffic: read a (bf16 grad), b, c (fp32 m, v), write b, c, d.
__global__ void __launch_bounds__(256) stream_kernel(const uint2* __restrict__ g, float4* __restrict__ m,
                                                     float4* __restrict__ v, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    uint2 gg = g[i];
    float4 mm = m[i], vv = v[i];
    float gf = __uint_as_float(gg.x << 16);
    mm.x = 0.9f * mm.x + 0.1f * gf;
    mm.y = 0.9f * mm.y + 0.1f * gf;
    vv.x = 0.95f * vv.x + 0.05f * gf * gf;
    vv.w = 0.95f * vv.w + 0.05f * __uint_as_float(gg.y << 16);
    m[i] = mm;
    v[i] = vv;
  }
}

static std::vector<uint32_t> make_mask(int ncu, const std::string& kind, int k) {
  std::vector<uint32_t> w((ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i) {
    bool on = false;
    if (kind == "all") on = true;
    else if (kind == "first") on = i < k;         // bits 0..k-1
    else if (kind == "mod8") on = (i % 8) < k;    // k of every 8 consecutive bits
    else if (kind == "stride") on = (i % k) == 0; // every k-th bit
    if (on) w[i / 32] |= 1u << (i % 32);
  }
  return w;
}

int main(int argc, char** argv) {
  int dev = 0;
  CK(hipSetDevice(dev));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int ncu = prop.multiProcessorCount;
  printf("{\"device\": \"%s\", \"cus\": %d}\n", prop.gcnArchName, ncu);
  const int nwg = 4096;
  uint32_t* rec;
  CK(hipMalloc(&rec, 2 * nwg * sizeof(uint32_t)));
  const int64_t n4 = (int64_t)1 << 27;  // 512 M elements: 1 GB grad, 2 GB m, 2 GB v
  uint2* g;
  float4 *m, *v;
  CK(hipMalloc(&g, n4 * sizeof(uint2)));
  CK(hipMalloc(&m, n4 * sizeof(float4)));
  CK(hipMalloc(&v, n4 * sizeof(float4)));
  CK(hipMemset(g, 0, n4 * sizeof(uint2)));
  CK(hipMemset(m, 0, n4 * sizeof(float4)));
  CK(hipMemset(v, 0, n4 * sizeof(float4)));
  const double bytes = (double)n4 * (8 + 2 * 16 + 2 * 16);

  struct Case { std::string kind; int k; };
  std::vector<Case> cases = {{"all", 0},   {"first", 32}, {"first", 64}, {"first", 128}, {"mod8", 1}, {"mod8", 2},
                             {"mod8", 3},  {"mod8", 4},   {"stride", 8}, {"stride", 4},  {"first", 8}};
  std::vector<uint32_t> host(2 * nwg);
  for (const auto& c : cases) {
    auto mask = make_mask(ncu, c.kind, c.k);
    int bits = 0;
    for (auto w : mask) bits += __builtin_popcount(w);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size() * 32, mask.data()));
    where_kernel<<<nwg, 64, 0, s>>>(rec);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(host.data(), rec, host.size() * 4, hipMemcpyDeviceToHost));
    std::set<uint32_t> xccs, cus;
    int per_xcc[8] = {0};
    for (int b = 0; b < nwg; ++b) {
      const uint32_t x = host[2 * b] & 0xf, hw = host[2 * b + 1];
      const uint32_t cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
      xccs.insert(x);
      cus.insert((x << 16) | (se << 8) | (sh << 4) | cu);
      if (x < 8) per_xcc[x]++;
    }
    // bandwidth: several grid sizes
    double best = 0;
    int best_grid = 0;
    for (int grid : {bits * 4, bits * 8, bits * 16, 2048, 8192}) {
      if (grid < 1) continue;
      stream_kernel<<<grid, 256, 0, s>>>(g, m, v, n4);
      CK(hipStreamSynchronize(s));
      auto t0 = std::chrono::high_resolution_clock::now();
      const int reps = 3;
      for (int r = 0; r < reps; ++r) stream_kernel<<<grid, 256, 0, s>>>(g, m, v, n4);
      CK(hipStreamSynchronize(s));
      double dt = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count() / reps;
      double tbs = bytes / dt / 1e12;
      if (tbs > best) { best = tbs; best_grid = grid; }
    }
    printf("{\"mask\": \"%s%d\", \"bits\": %d, \"xccs\": %zu, \"distinct_cus\": %zu, \"wg_per_xcc\": [%d,%d,%d,%d,%d,%d,%d,%d], "
           "\"stream_TBps\": %.3f, \"grid\": %d}\n",
           c.kind.c_str(), c.k, bits, xccs.size(), cus.size(), per_xcc[0], per_xcc[1], per_xcc[2], per_xcc[3],
           per_xcc[4], per_xcc[5], per_xcc[6], per_xcc[7], best, best_grid);
    fflush(stdout);
    CK(hipStreamDestroy(s));
  }
  CK(hipFree(rec));
  CK(hipFree(g));
  CK(hipFree(m));
  CK(hipFree(v));
  return 0;
}
