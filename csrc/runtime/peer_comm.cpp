// torch.classes.mxllm.PeerComm — bulk reduce-scatter / all-gather over peer
// memory inside one node (csrc/kernels/peer_coll.hip).
//
// Lifecycle (driven by mxllm/parallel/comm.py PeerCollectives):
//   c = PeerComm(rank, world, device, wgs, slot_bytes, timeout_s)
//   h = c.handle()                      # uint8[64] hipIpcMemHandle of my staging buffer
//   ranks exchange handles through the process group (once)
//   c.open(handles[world, 64])          # hipIpcOpenMemHandle every peer's staging
//   c.reduce_scatter_(out, in)          # enqueued on the CURRENT stream (the caller's comm stream)
//   c.all_gather_(out, in)
//   c.reduce_scatter_light_(out, in, wire_bf16) / c.all_gather_light_(out, in)
//                                       # the CU-light schedule (push / one-wave wait / consume
//                                       # kernels that exit; staging light_cap bytes per slot)
//   c.error()                           # 1 once any spin timed out (host-mapped word; no sync)
//
// The Python side gives these RCCL's semantics: one private stream per
// communicator ordered after the caller's stream, an event per call that
// work.wait() makes the caller's stream wait on, and record_stream() on every
// tensor so the caching allocator keeps it alive until the collective is done.
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

extern "C" size_t mx_peer_staging_bytes(int world, int wgs, int slot_bytes);
extern "C" size_t mx_peer_staging_bytes2(int world, int wgs, int slot_bytes, int64_t light_cap);
extern "C" int mx_peer_collective_light(int mode, int dtype, int wire, char* const* lbases, const void* in, void* out,
                                        int64_t n, int64_t m, int rank, int world, int wgs, int64_t light_cap,
                                        uint32_t* epoch, int* err, long long timeout_ticks, hipStream_t stream);
extern "C" int mx_peer_collective(int mode, int dtype, char* const* bases, const void* in, void* out, int64_t n,
                                  int64_t m, int rank, int world, int wgs, int slot_bytes, uint32_t* epochs, int* err,
                                  long long timeout_ticks, hipStream_t stream);

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxWG = 64;

#define PC_CHECK(expr)                                                                       \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    TORCH_CHECK(e_ == hipSuccess, "PeerComm: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

class PeerComm : public torch::CustomClassHolder {
 public:
  PeerComm(int64_t rank, int64_t world, int64_t device, int64_t wgs, int64_t slot_bytes, double timeout_s,
           int64_t light_cap, int64_t light_wgs)
      : rank_(rank), world_(world), device_(device), wgs_(wgs), slot_bytes_(slot_bytes),
        timeout_ticks_((long long)(timeout_s * 1.0e8)), light_cap_(light_cap), light_wgs_(light_wgs) {
    TORCH_CHECK(light_cap >= 0 && light_cap % 4096 == 0 && light_cap <= ((int64_t)1 << 31),
                "PeerComm: light_cap must be a multiple of 4096 in [0, 2 GB]");
    TORCH_CHECK(light_wgs >= 1 && light_wgs <= 4096, "PeerComm: light_wgs must be in [1, 4096]");
    TORCH_CHECK(world >= 2 && world <= kMaxRanks && rank >= 0 && rank < world, "PeerComm: bad rank/world");
    TORCH_CHECK(wgs >= 1 && wgs <= kMaxWG, "PeerComm: wgs must be in [1, 64]");
    TORCH_CHECK(slot_bytes >= 4096 && slot_bytes % 4096 == 0 && slot_bytes <= (1 << 22),
                "PeerComm: slot_bytes must be a multiple of 4096 in [4 KB, 4 MB]");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device));
    light_off_ = (mx_peer_staging_bytes((int)world, (int)wgs, (int)slot_bytes) + 4095) / 4096 * 4096;
    bytes_ = mx_peer_staging_bytes2((int)world, (int)wgs, (int)slot_bytes, light_cap);
    PC_CHECK(hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached));
    PC_CHECK(hipMemset(base_, 0, bytes_));
    PC_CHECK(hipMalloc((void**)&epochs_, kMaxWG * sizeof(uint32_t)));
    PC_CHECK(hipMemset(epochs_, 0, kMaxWG * sizeof(uint32_t)));
    PC_CHECK(hipHostMalloc((void**)&err_host_, sizeof(int), hipHostMallocMapped));
    *err_host_ = 0;
    PC_CHECK(hipHostGetDevicePointer((void**)&err_dev_, err_host_, 0));
    PC_CHECK(hipDeviceSynchronize());
    bases_.assign(world, nullptr);
    peers_.assign(world, nullptr);
    bases_[rank_] = reinterpret_cast<char*>(base_);
  }

  ~PeerComm() override { close(); }

  at::Tensor handle() {
    hipIpcMemHandle_t h;
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    PC_CHECK(hipIpcGetMemHandle(&h, base_));
    auto t = at::empty({(int64_t)sizeof(h)}, at::kByte);
    std::memcpy(t.data_ptr(), &h, sizeof(h));
    return t;
  }

  void open(at::Tensor handles) {
    TORCH_CHECK(handles.dim() == 2 && handles.size(0) == world_ && handles.scalar_type() == at::kByte &&
                    handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
                "PeerComm.open: handles must be uint8 [world, 64]");
    auto hc = handles.contiguous().cpu();
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    for (int64_t r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      hipIpcMemHandle_t h;
      std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
      void* p = nullptr;
      PC_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_[r] = p;
      bases_[r] = reinterpret_cast<char*>(p);
    }
    lbases_.assign(world_, nullptr);
    if (light_cap_ > 0)
      for (int64_t r = 0; r < world_; ++r) lbases_[r] = bases_[r] + light_off_;
    opened_ = true;
  }

  // out [m] = sum over ranks of chunk `rank` of in [n] (chunk p = in[p*m, (p+1)*m), zero past n)
  void reduce_scatter_(at::Tensor out, at::Tensor in) { run(0, out, in, in.numel(), out.numel()); }

  // out [n]: out[p*m, (p+1)*m) = rank p's in [m] (truncated at n)
  void all_gather_(at::Tensor out, at::Tensor in) { run(1, out, in, out.numel(), in.numel()); }

  // CU-light schedule: out [m] = sum over ranks of chunk `rank` of in [n] (wire_bf16: fp32 in / out,
  // bf16 on the wire, fp32 sum of the bf16-rounded values)
  void reduce_scatter_light_(at::Tensor out, at::Tensor in, bool wire_bf16) {
    run_light(0, out, in, in.numel(), out.numel(), wire_bf16);
  }
  void all_gather_light_(at::Tensor out, at::Tensor in) { run_light(1, out, in, out.numel(), in.numel(), false); }
  int64_t light_cap() const { return light_cap_; }
  void set_light_wgs(int64_t w) {
    TORCH_CHECK(w >= 1 && w <= 4096, "PeerComm: light_wgs must be in [1, 4096]");
    light_wgs_ = w;
  }

  void set_timeout(double timeout_s) { timeout_ticks_ = (long long)(timeout_s * 1.0e8); }
  void clear_error() { __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE); }
  int64_t error() const { return err_host_ ? __atomic_load_n(err_host_, __ATOMIC_ACQUIRE) : 0; }
  int64_t staging_bytes() const { return (int64_t)bytes_; }

  void close() {
    if (!base_) return;
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    (void)hipDeviceSynchronize();
    for (void*& p : peers_) {
      if (p) (void)hipIpcCloseMemHandle(p);
      p = nullptr;
    }
    (void)hipFree(base_);
    (void)hipFree(epochs_);
    (void)hipHostFree(err_host_);
    base_ = nullptr;
    epochs_ = nullptr;
    err_host_ = nullptr;
    opened_ = false;
  }

 private:
  void run_light(int mode, const at::Tensor& out, const at::Tensor& in, int64_t n, int64_t m, bool wire_bf16) {
    TORCH_CHECK(base_, "PeerComm: closed");
    TORCH_CHECK(opened_, "PeerComm: open() not called");
    TORCH_CHECK(light_cap_ > 0, "PeerComm: built without a light area (light_cap 0)");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.device().index() == device_ && out.device().index() == device_,
                "PeerComm: tensors must live on cuda:", device_);
    TORCH_CHECK(in.scalar_type() == out.scalar_type() &&
                    (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "PeerComm: float32 or bfloat16 tensors of one dtype");
    TORCH_CHECK(!wire_bf16 || (mode == 0 && in.scalar_type() == at::kFloat),
                "PeerComm: a bf16 wire is for fp32 reduce-scatters");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "PeerComm: contiguous tensors");
    TORCH_CHECK(n % 8 == 0 && m % 8 == 0, "PeerComm (light): sizes must be multiples of 8 elements (n=", n, ", m=", m,
                ")");
    TORCH_CHECK(m * world_ >= n, "PeerComm: chunk ", m, " x world ", world_, " < ", n);
    TORCH_CHECK(((uintptr_t)in.data_ptr() % 16) == 0 && ((uintptr_t)out.data_ptr() % 16) == 0,
                "PeerComm: 16-byte aligned tensors");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    const int dt = in.scalar_type() == at::kFloat ? 0 : 1;
    int rc = mx_peer_collective_light(mode, dt, wire_bf16 ? 1 : dt, lbases_.data(), in.data_ptr(), out.data_ptr(), n,
                                      m, (int)rank_, (int)world_, (int)light_wgs_, light_cap_, &light_epoch_,
                                      err_dev_, timeout_ticks_, s);
    TORCH_CHECK(rc == 0, "mx_peer_collective_light failed: ", rc);
  }

  void run(int mode, const at::Tensor& out, const at::Tensor& in, int64_t n, int64_t m) {
    TORCH_CHECK(base_, "PeerComm: closed");
    TORCH_CHECK(opened_, "PeerComm: open() not called");
    TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.device().index() == device_ && out.device().index() == device_,
                "PeerComm: tensors must live on cuda:", device_);
    TORCH_CHECK(in.scalar_type() == out.scalar_type() &&
                    (in.scalar_type() == at::kFloat || in.scalar_type() == at::kBFloat16),
                "PeerComm: float32 or bfloat16 tensors of one dtype");
    TORCH_CHECK(in.is_contiguous() && out.is_contiguous(), "PeerComm: contiguous tensors");
    const int64_t vec = in.scalar_type() == at::kFloat ? 4 : 8;
    TORCH_CHECK(n % vec == 0 && m % vec == 0, "PeerComm: sizes must be multiples of 16 bytes (n=", n, ", m=", m, ")");
    TORCH_CHECK(m * world_ >= n, "PeerComm: chunk ", m, " x world ", world_, " < ", n);
    TORCH_CHECK(((uintptr_t)in.data_ptr() % 16) == 0 && ((uintptr_t)out.data_ptr() % 16) == 0,
                "PeerComm: 16-byte aligned tensors");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    int rc = mx_peer_collective(mode, in.scalar_type() == at::kFloat ? 0 : 1, bases_.data(), in.data_ptr(),
                                out.data_ptr(), n, m, (int)rank_, (int)world_, (int)wgs_, (int)slot_bytes_, epochs_,
                                err_dev_, timeout_ticks_, s);
    TORCH_CHECK(rc == 0, "mx_peer_collective failed: ", rc);
  }

  int64_t rank_, world_, device_, wgs_, slot_bytes_;
  long long timeout_ticks_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  uint32_t* epochs_ = nullptr;
  int* err_host_ = nullptr;
  int* err_dev_ = nullptr;
  bool opened_ = false;
  int64_t light_cap_ = 0, light_wgs_ = 64;
  size_t light_off_ = 0;
  uint32_t light_epoch_ = 0;  // light segments issued (identical on every rank)
  std::vector<char*> bases_, lbases_;
  std::vector<void*> peers_;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(mxllm, m) {
  m.class_<PeerComm>("PeerComm")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t, int64_t, double, int64_t, int64_t>())
      .def("reduce_scatter_light_", &PeerComm::reduce_scatter_light_)
      .def("all_gather_light_", &PeerComm::all_gather_light_)
      .def("light_cap", &PeerComm::light_cap)
      .def("set_light_wgs", &PeerComm::set_light_wgs)
      .def("handle", &PeerComm::handle)
      .def("open", &PeerComm::open)
      .def("reduce_scatter_", &PeerComm::reduce_scatter_)
      .def("all_gather_", &PeerComm::all_gather_)
      .def("error", &PeerComm::error)
      .def("set_timeout", &PeerComm::set_timeout)
      .def("clear_error", &PeerComm::clear_error)
      .def("staging_bytes", &PeerComm::staging_bytes)
      .def("close", &PeerComm::close);
}
