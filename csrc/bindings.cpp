// Torch op registrations for the mxllm HIP kernels (namespace torch.ops.mxllm).
//
// Kernels live in csrc/kernels/*.hip and expose plain C launchers
// (`mx_*`, taking raw pointers + hipStream_t); this file is the only one that
// includes torch headers, so kernel files compile in seconds and stay free of
// ATen.  Every op runs on the current HIP stream of the input's device.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include "bindings.h"

namespace {

// On ROCm builds torch devices are DeviceType::CUDA backed by HIP: use the
// "masquerading" guard/stream so device indices and the current stream match torch's.
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
using DevGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

#define MX_CHECK(cond, ...) TORCH_CHECK(cond, "mxllm: ", __VA_ARGS__)
#define MX_OK(call)                                                                              \
  do {                                                                                           \
    int _rc = (call);                                                                            \
    TORCH_CHECK(_rc == 0, "mxllm kernel launch failed (" #call ") rc=", _rc, " ",                 \
                hipGetErrorString((hipError_t)(_rc > 0 ? _rc : 1)));                             \
  } while (0)

inline const uint16_t* bf(const at::Tensor& t) {
  return reinterpret_cast<const uint16_t*>(t.data_ptr());
}
inline uint16_t* bfm(at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

void check_bf16(const at::Tensor& t, const char* name) {
  MX_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MX_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
  MX_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_f32(const at::Tensor& t, const char* name) {
  MX_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MX_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  MX_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// ---------------------------------------------------------------- RMSNorm
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x,
                                                           const c10::optional<at::Tensor>& res,
                                                           const at::Tensor& w, double eps) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  DevGuard g(x.device());
  const int64_t H = x.size(-1);
  const int64_t T = x.numel() / H;
  MX_CHECK(w.numel() == H, "weight size mismatch");
  auto y = at::empty_like(x);
  auto rstd = at::empty({T}, x.options().dtype(at::kFloat));
  at::Tensor h;
  const uint16_t* rp = nullptr;
  uint16_t* hp = nullptr;
  if (res.has_value()) {
    check_bf16(*res, "res");
    MX_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
    h = at::empty_like(x);
    rp = bf(*res);
    hp = bfm(h);
  }
  if (T > 0)
    MX_OK(mx_rmsnorm_fwd(bf(x), rp, bf(w), bfm(y), hp, rstd.data_ptr<float>(), (int)T, (int)H,
                         (float)eps, cur_stream()));
  if (!res.has_value()) h = x;
  return {y, rstd, h};
}

// returns (dx, dw_f32 or empty)
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x,
                                               const at::Tensor& w, const at::Tensor& rstd,
                                               const c10::optional<at::Tensor>& dres, bool need_dw) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_f32(rstd, "rstd");
  DevGuard g(x.device());
  const int64_t H = x.size(-1);
  const int64_t T = x.numel() / H;
  auto dx = at::empty_like(x);
  const uint16_t* drp = nullptr;
  if (dres.has_value()) {
    check_bf16(*dres, "dres");
    drp = bf(*dres);
  }
  // rows per block: keep >= ~2 blocks per CU on 256 CUs, amortise the dγ partial
  int rpb = 1;
  if (need_dw) {
    rpb = (int)std::max<int64_t>(1, T / 512);
    rpb = std::min(rpb, 32);
  }
  const int64_t nblk = (T + rpb - 1) / rpb;
  at::Tensor dwp, dw;
  float* dwpp = nullptr;
  if (need_dw) {
    dwp = at::empty({nblk, H}, x.options().dtype(at::kFloat));
    dw = at::empty({H}, x.options().dtype(at::kFloat));
    dwpp = dwp.data_ptr<float>();
  }
  if (T > 0) {
    MX_OK(mx_rmsnorm_bwd(bf(dy), bf(x), bf(w), rstd.data_ptr<float>(), drp, bfm(dx), dwpp, (int)T,
                         (int)H, rpb, cur_stream()));
    if (need_dw) MX_OK(mx_colsum_f32(dwpp, dw.data_ptr<float>(), (int)nblk, (int)H, cur_stream()));
  } else if (need_dw) {
    dw.zero_();
  }
  return {dx, need_dw ? dw : at::Tensor()};
}

// ---------------------------------------------------------------- misc
at::Tensor segmented_mean(const at::Tensor& codes, const at::Tensor& offsets) {
  MX_CHECK(codes.is_cuda() && codes.scalar_type() == at::kInt, "codes must be int32 GPU");
  MX_CHECK(offsets.is_cuda() && offsets.scalar_type() == at::kLong, "offsets must be int64 GPU");
  DevGuard g(codes.device());
  const int64_t n = offsets.numel() - 1;
  auto out = at::empty({std::max<int64_t>(n, 0)}, codes.options().dtype(at::kFloat));
  if (n > 0)
    MX_OK(mx_segmented_mean_i32(codes.data_ptr<int32_t>(), offsets.data_ptr<int64_t>(),
                                out.data_ptr<float>(), (int)n, cur_stream()));
  return out;
}

at::Tensor sqnorm_f32(const at::Tensor& x) {
  check_f32(x, "x");
  DevGuard g(x.device());
  auto out = at::zeros({1}, x.options());
  MX_OK(mx_sqnorm_f32(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), cur_stream()));
  return out;
}

}  // namespace

TORCH_LIBRARY(mxllm, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor? res, Tensor w, float eps) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres, bool need_dw) -> (Tensor, Tensor)");
  m.def("segmented_mean(Tensor codes, Tensor offsets) -> Tensor");
  m.def("sqnorm_f32(Tensor x) -> Tensor");
}

TORCH_LIBRARY_IMPL(mxllm, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("segmented_mean", &segmented_mean);
  m.impl("sqnorm_f32", &sqnorm_f32);
}
