// torch.classes.mxllm.XgmiComm — peer-memory communicator for latency-bound
// collectives inside one MI355X node.
//
// Lifecycle (driven by mxllm/parallel/xgmi.py):
//   c = XgmiComm(rank, world, device, max_elems, timeout_s)
//   h = c.handle()                      # uint8[64] hipIpcMemHandle of my buffer
//   all ranks exchange handles (TCPStore / process group, once)
//   c.open(handles[world, 64])          # hipIpcOpenMemHandle every peer buffer
//   c.all_reduce_(t, op)                # f32 on my device, n <= max_elems; in place
//   c.barrier()                         # 0-element all-reduce (device-side)
//   c.error()                           # 1 if any spin timed out (host-mapped word)
//
// The buffer is fine-grained and uncached (hipDeviceMallocUncached) so the
// kernel's system-scope release/acquire needs no cache maintenance of the data.
// Every call advances a per-communicator epoch; all ranks must issue the same
// sequence of calls (as with any collective).
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

extern "C" int mx_xgmi_allreduce(uint32_t* const* flags, float* const* data, const float* in, float* out, int n,
                                 int rank, int world, uint32_t epoch, int max_elems, int op, int* err,
                                 long long timeout_ticks, hipStream_t stream);

extern "C" int mx_xgmi_allreduce_bf16(uint32_t* const* flags, uint16_t* const* data, const uint16_t* in,
                                      uint16_t* out, int n, int rank, int world, int max_elems, uint32_t* epochs,
                                      int* err, long long timeout_ticks, hipStream_t stream);

namespace {

constexpr int kMaxRanks = 16;
constexpr int kMaxWG = 64;  // workgroups (flag rows) of the bf16 kernel
constexpr size_t kFlagBytes = kMaxRanks * 64;

#define XG_CHECK(expr)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    TORCH_CHECK(e_ == hipSuccess, "XgmiComm: ", #expr, " failed: ", hipGetErrorString(e_)); \
  } while (0)

class XgmiComm : public torch::CustomClassHolder {
 public:
  XgmiComm(int64_t rank, int64_t world, int64_t device, int64_t max_elems, double timeout_s)
      : rank_(rank), world_(world), device_(device), max_elems_(max_elems),
        timeout_ticks_((long long)(timeout_s * 1.0e8)) {
    TORCH_CHECK(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world, "XgmiComm: bad rank/world");
    TORCH_CHECK(max_elems >= 1, "XgmiComm: max_elems must be positive");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device));
    bytes_ = kFlagBytes + 2 * (size_t)world * (size_t)max_elems * sizeof(float);
    XG_CHECK(hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached));
    XG_CHECK(hipMemset(base_, 0, bytes_));
    XG_CHECK(hipHostMalloc((void**)&err_host_, sizeof(int), hipHostMallocMapped));
    *err_host_ = 0;
    XG_CHECK(hipHostGetDevicePointer((void**)&err_dev_, err_host_, 0));
    XG_CHECK(hipDeviceSynchronize());
    flags_.assign(world, nullptr);
    data_.assign(world, nullptr);
    peers_.assign(world, nullptr);
    set_ptrs(rank_, base_);
  }

  ~XgmiComm() override { close(); }

  at::Tensor handle() {
    hipIpcMemHandle_t h;
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    XG_CHECK(hipIpcGetMemHandle(&h, base_));
    auto t = at::empty({(int64_t)sizeof(h)}, at::kByte);
    std::memcpy(t.data_ptr(), &h, sizeof(h));
    return t;
  }

  void open(at::Tensor handles) {
    TORCH_CHECK(handles.dim() == 2 && handles.size(0) == world_ && handles.scalar_type() == at::kByte &&
                    handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
                "XgmiComm.open: handles must be uint8 [world, 64]");
    auto hc = handles.contiguous().cpu();
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    for (int64_t r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      hipIpcMemHandle_t h;
      std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
      void* p = nullptr;
      XG_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_[r] = p;
      set_ptrs(r, p);
    }
    opened_ = true;
  }

  // op: 0 sum, 1 max, 2 min.  t: contiguous f32 on this communicator's device.
  at::Tensor all_reduce_(at::Tensor t, int64_t op) {
    TORCH_CHECK(opened_ || world_ == 1, "XgmiComm: open() not called");
    TORCH_CHECK(t.is_cuda() && t.device().index() == device_ && t.scalar_type() == at::kFloat && t.is_contiguous(),
                "XgmiComm.all_reduce_: expected contiguous float32 on cuda:", device_);
    TORCH_CHECK(t.numel() <= max_elems_, "XgmiComm.all_reduce_: ", t.numel(), " elements > max_elems ", max_elems_);
    launch(t.data_ptr<float>(), t.data_ptr<float>(), (int)t.numel(), (int)op);
    return t;
  }

  void barrier() {
    TORCH_CHECK(opened_ || world_ == 1, "XgmiComm: open() not called");
    launch(nullptr, nullptr, 0, 0);
  }

  void set_timeout(double timeout_s) { timeout_ticks_ = (long long)(timeout_s * 1.0e8); }
  void clear_error() { __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE); }
  int64_t error() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE); }
  int64_t epoch() const { return epoch_; }
  int64_t max_elems() const { return max_elems_; }

  void close() {
    if (!base_) return;
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    (void)hipDeviceSynchronize();
    for (void*& p : peers_) {
      if (p) (void)hipIpcCloseMemHandle(p);
      p = nullptr;
    }
    (void)hipFree(base_);
    (void)hipHostFree(err_host_);
    base_ = nullptr;
    err_host_ = nullptr;
    opened_ = false;
  }

 private:
  void set_ptrs(int64_t r, void* b) {
    flags_[r] = reinterpret_cast<uint32_t*>(b);
    data_[r] = reinterpret_cast<float*>(reinterpret_cast<char*>(b) + kFlagBytes);
  }

  void launch(const float* in, float* out, int n, int op) {
    TORCH_CHECK(base_, "XgmiComm: closed");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    const uint32_t e = (uint32_t)(++epoch_);
    int rc = mx_xgmi_allreduce(flags_.data(), data_.data(), in, out, n, (int)rank_, (int)world_, e,
                               (int)max_elems_, op, err_dev_, timeout_ticks_, s);
    TORCH_CHECK(rc == 0, "mx_xgmi_allreduce failed: ", rc);
  }

  int64_t rank_, world_, device_, max_elems_;
  long long timeout_ticks_;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  int* err_host_ = nullptr;
  int* err_dev_ = nullptr;
  int64_t epoch_ = 0;
  bool opened_ = false;
  std::vector<uint32_t*> flags_;
  std::vector<float*> data_;
  std::vector<void*> peers_;
};

// torch.classes.mxllm.XgmiGraphComm — the graph-safe bf16 sum all-reduce of
// tensor-parallel decode (csrc/kernels/xgmi.hip, mx_xgmi_allreduce_bf16).  Same
// handle exchange as XgmiComm; the epochs live in device memory, so one
// captured launch replays correctly any number of times.
class XgmiGraphComm : public torch::CustomClassHolder {
 public:
  XgmiGraphComm(int64_t rank, int64_t world, int64_t device, int64_t max_elems, double timeout_s)
      : rank_(rank), world_(world), device_(device), max_elems_(max_elems),
        timeout_ticks_((long long)(timeout_s * 1.0e8)) {
    TORCH_CHECK(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world, "XgmiGraphComm: bad rank/world");
    TORCH_CHECK(max_elems >= 8 && max_elems % 8 == 0, "XgmiGraphComm: max_elems must be a positive multiple of 8");
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device));
    flag_bytes_ = (size_t)kMaxWG * kMaxRanks * 64;
    bytes_ = flag_bytes_ + 2 * (size_t)world * (size_t)max_elems * sizeof(uint16_t);
    XG_CHECK(hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached));
    XG_CHECK(hipMemset(base_, 0, bytes_));
    XG_CHECK(hipMalloc((void**)&epochs_, kMaxWG * sizeof(uint32_t)));
    XG_CHECK(hipMemset(epochs_, 0, kMaxWG * sizeof(uint32_t)));
    XG_CHECK(hipHostMalloc((void**)&err_host_, sizeof(int), hipHostMallocMapped));
    *err_host_ = 0;
    XG_CHECK(hipHostGetDevicePointer((void**)&err_dev_, err_host_, 0));
    XG_CHECK(hipDeviceSynchronize());
    flags_.assign(world, nullptr);
    data_.assign(world, nullptr);
    peers_.assign(world, nullptr);
    set_ptrs(rank_, base_);
  }

  ~XgmiGraphComm() override { close(); }

  at::Tensor handle() {
    hipIpcMemHandle_t h;
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    XG_CHECK(hipIpcGetMemHandle(&h, base_));
    auto t = at::empty({(int64_t)sizeof(h)}, at::kByte);
    std::memcpy(t.data_ptr(), &h, sizeof(h));
    return t;
  }

  void open(at::Tensor handles) {
    TORCH_CHECK(handles.dim() == 2 && handles.size(0) == world_ && handles.scalar_type() == at::kByte &&
                    handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
                "XgmiGraphComm.open: handles must be uint8 [world, 64]");
    auto hc = handles.contiguous().cpu();
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    for (int64_t r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      hipIpcMemHandle_t h;
      std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
      void* p = nullptr;
      XG_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      peers_[r] = p;
      set_ptrs(r, p);
    }
    opened_ = true;
  }

  // in-place sum of a contiguous bf16 tensor (numel % 8 == 0, <= max_elems)
  at::Tensor all_reduce_(at::Tensor t) {
    TORCH_CHECK(opened_ || world_ == 1, "XgmiGraphComm: open() not called");
    TORCH_CHECK(base_, "XgmiGraphComm: closed");
    TORCH_CHECK(t.is_cuda() && t.device().index() == device_ && t.scalar_type() == at::kBFloat16 &&
                    t.is_contiguous(), "XgmiGraphComm.all_reduce_: expected contiguous bfloat16 on cuda:", device_);
    TORCH_CHECK(t.numel() > 0 && t.numel() <= max_elems_ && t.numel() % 8 == 0,
                "XgmiGraphComm.all_reduce_: numel ", t.numel(), " must be a multiple of 8 and <= ", max_elems_);
    c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device_));
    hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
    auto* p = reinterpret_cast<uint16_t*>(t.data_ptr());
    int rc = mx_xgmi_allreduce_bf16(flags_.data(), data_.data(), p, p, (int)t.numel(), (int)rank_, (int)world_,
                                    (int)max_elems_, epochs_, err_dev_, timeout_ticks_, s);
    TORCH_CHECK(rc == 0, "mx_xgmi_allreduce_bf16 failed: ", rc);
    return t;
  }

  void set_timeout(double timeout_s) { timeout_ticks_ = (long long)(timeout_s * 1.0e8); }
  void clear_error() { __atomic_store_n(err_host_, 0, __ATOMIC_RELEASE); }
  int64_t error() const { return __atomic_load_n(err_host_, __ATOMIC_ACQUIRE); }
  int64_t max_elems() const { return max_elems_; }

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
  void set_ptrs(int64_t r, void* b) {
    flags_[r] = reinterpret_cast<uint32_t*>(b);
    data_[r] = reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(b) + flag_bytes_);
  }

  int64_t rank_, world_, device_, max_elems_;
  long long timeout_ticks_;
  size_t flag_bytes_ = 0, bytes_ = 0;
  void* base_ = nullptr;
  uint32_t* epochs_ = nullptr;
  int* err_host_ = nullptr;
  int* err_dev_ = nullptr;
  bool opened_ = false;
  std::vector<uint32_t*> flags_;
  std::vector<uint16_t*> data_;
  std::vector<void*> peers_;
};

}  // namespace

TORCH_LIBRARY_FRAGMENT(mxllm, m) {
  m.class_<XgmiComm>("XgmiComm")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t, double>())
      .def("handle", &XgmiComm::handle)
      .def("open", &XgmiComm::open)
      .def("all_reduce_", &XgmiComm::all_reduce_)
      .def("barrier", &XgmiComm::barrier)
      .def("error", &XgmiComm::error)
      .def("set_timeout", &XgmiComm::set_timeout)
      .def("clear_error", &XgmiComm::clear_error)
      .def("epoch", &XgmiComm::epoch)
      .def("max_elems", &XgmiComm::max_elems)
      .def("close", &XgmiComm::close);
  m.class_<XgmiGraphComm>("XgmiGraphComm")
      .def(torch::init<int64_t, int64_t, int64_t, int64_t, double>())
      .def("handle", &XgmiGraphComm::handle)
      .def("open", &XgmiGraphComm::open)
      .def("all_reduce_", &XgmiGraphComm::all_reduce_)
      .def("error", &XgmiGraphComm::error)
      .def("set_timeout", &XgmiGraphComm::set_timeout)
      .def("clear_error", &XgmiGraphComm::clear_error)
      .def("max_elems", &XgmiGraphComm::max_elems)
      .def("close", &XgmiGraphComm::close);
}
