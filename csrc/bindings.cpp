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
#include <algorithm>
#include <vector>

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
// a 2-D row-strided bf16 view (rows may be the left part of a wider buffer)
int64_t check_rows_bf16(const at::Tensor& t, const char* name) {
  MX_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MX_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
  MX_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.stride(0) >= t.size(1) && t.stride(0) % 8 == 0, name,
           " must be a row-major [T, H] view with a row stride that is a multiple of 8");
  return t.stride(0);
}
// [T, H] output whose rows live in a [T, H + pad] buffer (pad extra columns left to the caller)
at::Tensor empty_rows(int64_t T, int64_t H, int64_t pad, const at::TensorOptions& o) {
  if (pad <= 0) return at::empty({T, H}, o);
  return at::empty({T, H + pad}, o).narrow(1, 0, H);
}
void check_f32(const at::Tensor& t, const char* name) {
  MX_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  MX_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  MX_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// ---------------------------------------------------------------- RMSNorm
// out_pad > 0: y is returned as the [T, H] left part of a [T, H + out_pad] buffer
std::tuple<at::Tensor, at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x,
                                                           const c10::optional<at::Tensor>& res,
                                                           const at::Tensor& w, double eps, int64_t out_pad) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  DevGuard g(x.device());
  const int64_t H = x.size(-1);
  const int64_t T = x.numel() / H;
  MX_CHECK(w.numel() == H, "weight size mismatch");
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  at::Tensor y = out_pad > 0 ? empty_rows(T, H, out_pad, x.options()) : at::empty_like(x);
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
    MX_OK(mx_rmsnorm_fwd(bf(x), rp, bf(w), bfm(y), hp, rstd.data_ptr<float>(), (int)T, (int)H, (int)(H + out_pad),
                         (float)eps, cur_stream()));
  if (!res.has_value()) h = x;
  return {y, rstd, h};
}

// returns (dx, dw_f32 or empty).  dres may be a row-strided [T, H] view;
// out_pad > 0: dx is the left part of a [T, H + out_pad] buffer.
std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x,
                                               const at::Tensor& w, const at::Tensor& rstd,
                                               const c10::optional<at::Tensor>& dres, bool need_dw,
                                               int64_t out_pad) {
  check_bf16(dy, "dy");
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_f32(rstd, "rstd");
  DevGuard g(x.device());
  const int64_t H = x.size(-1);
  const int64_t T = x.numel() / H;
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  at::Tensor dx = out_pad > 0 ? empty_rows(T, H, out_pad, x.options()) : at::empty_like(x);
  const uint16_t* drp = nullptr;
  int64_t ldr = H;
  if (dres.has_value()) {
    if (dres->is_contiguous()) {
      check_bf16(*dres, "dres");
    } else {
      ldr = check_rows_bf16(*dres, "dres");
      MX_CHECK(dres->size(0) == T && dres->size(1) == H, "dres shape mismatch");
    }
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
    MX_OK(mx_rmsnorm_bwd(bf(dy), bf(x), bf(w), rstd.data_ptr<float>(), drp, bfm(dx), dwpp, (int)T, (int)H,
                         (int)ldr, (int)(H + out_pad), rpb, cur_stream()));
    if (need_dw) MX_OK(mx_colsum_f32(dwpp, dw.data_ptr<float>(), (int)nblk, (int)H, cur_stream()));
  } else if (need_dw) {
    dw.zero_();
  }
  return {dx, need_dw ? dw : at::Tensor()};
}

// ---------------------------------------------------------------- misc
// desc: int64 [n, 9] on the device (see misc.hip); total_blocks = sum of per-descriptor blocks
void copy2d_batched(const at::Tensor& desc, int64_t total_blocks) {
  MX_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 9 &&
               desc.is_contiguous(), "desc must be int64 [n, 9] on the GPU");
  DevGuard g(desc.device());
  MX_OK(mx_copy2d_batched(desc.data_ptr<int64_t>(), (int)desc.size(0), total_blocks, cur_stream()));
}

// out[C, R] = in[R, C]^T for a row-major (row-strided) 16-bit 2-D GPU tensor
// scale: optional f32 device scalar (bf16 input): out = bf16(in^T * scale)
at::Tensor transpose2d(const at::Tensor& in, const c10::optional<at::Tensor>& scale) {
  MX_CHECK(in.is_cuda() && in.dim() == 2 && in.element_size() == 2, "in must be a 2-D 16-bit GPU tensor");
  MX_CHECK(in.stride(1) == 1 && in.stride(0) >= in.size(1), "in must be a row-major (row-strided) view");
  const float* sc = nullptr;
  if (scale.has_value()) {
    MX_CHECK(in.scalar_type() == at::kBFloat16 && scale->scalar_type() == at::kFloat && scale->numel() == 1 &&
                 scale->device() == in.device(), "transpose2d scale: f32 scalar on the device, bf16 input");
    sc = scale->data_ptr<float>();
  }
  DevGuard g(in.device());
  const int64_t R = in.size(0), C = in.size(1);
  auto out = at::empty({C, R}, in.options());
  MX_OK(mx_transpose16(in.data_ptr(), out.data_ptr(), R, C, in.stride(0), R, sc, cur_stream()));
  return out;
}

// out[M, N] = beta * out + alpha * op(a) op(b) on the 8-phase MFMA GEMM (csrc/kernels/gemm8.hip).
// a: [M, K] when a_kc (k-contiguous) else [K, M]; b: [N, K] when b_kc else [K, N]; all row-strided
// bf16 views, out fp32 or bf16; alpha = alpha_f * (the optional f32 device scalar alpha_t).
// Returns false (nothing launched) for shapes the kernel does not take.
bool gemm8(const at::Tensor& a, bool a_kc, const at::Tensor& b, bool b_kc, at::Tensor& out, double beta,
           const c10::optional<at::Tensor>& alpha_t, double alpha_f, int64_t ph) {
  MX_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm8: GPU tensors");
  MX_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "gemm8: bf16 operands");
  MX_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "gemm8: fp32 / bf16 output");
  MX_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm8: 2-D operands");
  const int64_t M = a_kc ? a.size(0) : a.size(1), K = a_kc ? a.size(1) : a.size(0);
  const int64_t N = b_kc ? b.size(0) : b.size(1), Kb = b_kc ? b.size(1) : b.size(0);
  MX_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "gemm8: shape mismatch");
  if (a.stride(1) != 1 || b.stride(1) != 1 || out.stride(1) != 1) return false;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return false;
  const float* sc = nullptr;
  if (alpha_t.has_value()) {
    MX_CHECK(alpha_t->scalar_type() == at::kFloat && alpha_t->numel() == 1 && alpha_t->device() == a.device(),
             "gemm8 alpha_t: f32 scalar on the device");
    sc = alpha_t->data_ptr<float>();
  }
  DevGuard g(a.device());
  const int rc = mx_gemm8(bf(a), a.stride(0), a_kc ? 1 : 0, bf(b), b.stride(0), b_kc ? 1 : 0, out.data_ptr(),
                          out.stride(0), out.scalar_type() == at::kFloat ? 1 : 0, (int)M, (int)N, (int)K, (float)beta,
                          sc, (float)alpha_f, (int)ph, cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// out[M, N] (bf16, beta 0) = alpha op(a) op(b) that also writes one fp32 sum of squares of the stored
// values per 256 x 256 output tile into sq (>= (M / 256) * (N / 256) elements, row-major tile order):
// the gradient-clip norm's partials straight from the weight-gradient GEMMs.  False: nothing launched.
bool gemm8_sq(const at::Tensor& a, bool a_kc, const at::Tensor& b, bool b_kc, at::Tensor& out, at::Tensor& sq,
              const c10::optional<at::Tensor>& alpha_t, double alpha_f) {
  MX_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda() && sq.is_cuda(), "gemm8_sq: GPU tensors");
  MX_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
               out.scalar_type() == at::kBFloat16 && sq.scalar_type() == at::kFloat,
           "gemm8_sq: bf16 operands and output, f32 partials");
  MX_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm8_sq: 2-D operands");
  const int64_t M = a_kc ? a.size(0) : a.size(1), K = a_kc ? a.size(1) : a.size(0);
  const int64_t N = b_kc ? b.size(0) : b.size(1), Kb = b_kc ? b.size(1) : b.size(0);
  MX_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "gemm8_sq: shape mismatch");
  if (a.stride(1) != 1 || b.stride(1) != 1 || out.stride(1) != 1 || !sq.is_contiguous()) return false;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX || M % 256 || N % 256) return false;
  MX_CHECK(sq.numel() >= (M / 256) * (N / 256), "gemm8_sq: partials buffer too small");
  const float* sc = nullptr;
  if (alpha_t.has_value()) {
    MX_CHECK(alpha_t->scalar_type() == at::kFloat && alpha_t->numel() == 1 && alpha_t->device() == a.device(),
             "gemm8_sq alpha_t: f32 scalar on the device");
    sc = alpha_t->data_ptr<float>();
  }
  DevGuard g(a.device());
  const int rc = mx_gemm8_sq(bf(a), a.stride(0), a_kc ? 1 : 0, bf(b), b.stride(0), b_kc ? 1 : 0, bfm(out),
                             out.stride(0), (int)M, (int)N, (int)K, sc, (float)alpha_f, sq.data_ptr<float>(),
                             cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// out[M, N] (bf16) = op(a) op(b) with the tail-balanced launch (mx_gemm8_tail): the output split at
// `at` columns (rows when `rows`) -- whole waves of tiles before it, half-K workgroups summed through
// an fp32 workspace after it.  Returns false (nothing launched) for shapes it does not take.
bool gemm8_tail(const at::Tensor& a, bool a_kc, const at::Tensor& b, bool b_kc, at::Tensor& out, int64_t at,
                bool rows, int64_t ph, const c10::optional<at::Tensor>& sq) {
  MX_CHECK(a.is_cuda() && b.is_cuda() && out.is_cuda(), "gemm8_tail: GPU tensors");
  MX_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16,
           "gemm8_tail: bf16 operands and output");
  MX_CHECK(a.dim() == 2 && b.dim() == 2 && out.dim() == 2, "gemm8_tail: 2-D operands");
  const int64_t M = a_kc ? a.size(0) : a.size(1), K = a_kc ? a.size(1) : a.size(0);
  const int64_t N = b_kc ? b.size(0) : b.size(1), Kb = b_kc ? b.size(1) : b.size(0);
  MX_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "gemm8_tail: shape mismatch");
  const int64_t lim = rows ? M : N;
  if (a.stride(1) != 1 || b.stride(1) != 1 || out.stride(1) != 1 || at <= 0 || at >= lim) return false;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return false;
  float* sqp = nullptr;
  if (sq.has_value()) {  // one sum of squares per 256 x 256 tile (plain part's tiles, then the split part's)
    MX_CHECK(sq->scalar_type() == at::kFloat && sq->is_contiguous() && sq->device() == a.device(),
             "gemm8_tail sq: contiguous f32 on the device");
    if (M % 256 || N % 256) return false;
    MX_CHECK(sq->numel() >= (M / 256) * (N / 256), "gemm8_tail sq: partials buffer too small");
    sqp = sq->data_ptr<float>();
  }
  DevGuard g(a.device());
  auto ws = at::empty({2 * (lim - at) * (rows ? N : M)}, a.options().dtype(at::kFloat));
  const int rc = mx_gemm8_tail(bf(a), a.stride(0), a_kc ? 1 : 0, bf(b), b.stride(0), b_kc ? 1 : 0, bfm(out),
                               out.stride(0), (int)M, (int)N, (int)K, rows ? 1 : 0, (int)at, ws.data_ptr<float>(),
                               (int)ph, cur_stream(), sqp);
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// Forward qkv projection with RoPE and the head split in the GEMM epilogue (gemm8 G8_EPI_ROPE):
// x [B*S, K] (row-strided), w [(Hq + 2 Hkv) * 128, K] -> q [B, Hq, S, 128], k / v [B, Hkv, S, 128]
// (preallocated, contiguous), rotated with the f32 tables cos / sin [>= S, 64] at positions 0..S-1.
// Returns false (nothing launched) for shapes the kernel does not take.
bool gemm8_rope(const at::Tensor& x, const at::Tensor& w, const at::Tensor& cos, const at::Tensor& sin, int64_t B,
                int64_t S, int64_t Hq, int64_t Hkv, at::Tensor& q, at::Tensor& k, at::Tensor& v) {
  MX_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
           "gemm8_rope: bf16 GPU operands");
  MX_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1) && x.size(0) == B * S, "gemm8_rope: shapes");
  MX_CHECK(w.size(0) == (Hq + 2 * Hkv) * 128, "gemm8_rope: head dim 128");
  MX_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
               sin.is_contiguous() && cos.size(-1) == 64 && cos.size(0) >= S && sin.sizes() == cos.sizes(),
           "gemm8_rope: f32 [>= S, 64] tables");
  for (const at::Tensor* t : {&q, &k, &v})
    MX_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous(), "gemm8_rope: bf16 outputs");
  MX_CHECK(q.numel() == B * Hq * S * 128 && k.numel() == B * Hkv * S * 128 && v.numel() == k.numel(),
           "gemm8_rope: output sizes");
  if (x.stride(1) != 1 || w.stride(1) != 1) return false;
  DevGuard g(x.device());
  MxG8Epi ep{};
  ep.q = bfm(q);
  ep.k = bfm(k);
  ep.v = bfm(v);
  ep.cosb = cos.data_ptr<float>();
  ep.sinb = sin.data_ptr<float>();
  ep.S = (int)S;
  ep.Hq = (int)Hq;
  ep.Hkv = (int)Hkv;
  const int rc = mx_gemm8_epi(bf(x), x.stride(0), bf(w), w.stride(0), nullptr, 0, (int)x.size(0), (int)w.size(0),
                              (int)x.size(1), 1, ep, cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// gemm8_rope on the tail-balanced schedule (mx_gemm8_rope_tail): columns [0, at) through the RoPE
// epilogue, the rest as half-K images summed, rotated and scattered by one pass -- bitwise
// gemm8_tail(at) followed by rope_split.  Returns false (nothing launched) for shapes it does not take.
bool gemm8_rope_tail(const at::Tensor& x, const at::Tensor& w, const at::Tensor& cos, const at::Tensor& sin, int64_t B,
                     int64_t S, int64_t Hq, int64_t Hkv, at::Tensor& q, at::Tensor& k, at::Tensor& v, int64_t at) {
  MX_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16,
           "gemm8_rope_tail: bf16 GPU operands");
  MX_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1) && x.size(0) == B * S, "gemm8_rope_tail: shapes");
  MX_CHECK(w.size(0) == (Hq + 2 * Hkv) * 128, "gemm8_rope_tail: head dim 128");
  MX_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat && cos.is_contiguous() &&
               sin.is_contiguous() && cos.size(-1) == 64 && cos.size(0) >= S && sin.sizes() == cos.sizes(),
           "gemm8_rope_tail: f32 [>= S, 64] tables");
  for (const at::Tensor* t : {&q, &k, &v})
    MX_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous(), "gemm8_rope_tail: bf16 outputs");
  MX_CHECK(q.numel() == B * Hq * S * 128 && k.numel() == B * Hkv * S * 128 && v.numel() == k.numel(),
           "gemm8_rope_tail: output sizes");
  if (x.stride(1) != 1 || w.stride(1) != 1 || at <= 0 || at >= w.size(0)) return false;
  if (x.size(0) > INT32_MAX || x.size(1) > INT32_MAX) return false;
  DevGuard g(x.device());
  auto ws = at::empty({2 * x.size(0) * (w.size(0) - at)}, x.options().dtype(at::kFloat));
  MxG8Epi ep{};
  ep.q = bfm(q);
  ep.k = bfm(k);
  ep.v = bfm(v);
  ep.cosb = cos.data_ptr<float>();
  ep.sinb = sin.data_ptr<float>();
  ep.S = (int)S;
  ep.Hq = (int)Hq;
  ep.Hkv = (int)Hkv;
  const int rc = mx_gemm8_rope_tail(bf(x), x.stride(0), bf(w), w.stride(0), (int)x.size(0), (int)w.size(0),
                                    (int)x.size(1), (int)at, ws.data_ptr<float>(), ep, cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// Forward gate-up projection with SwiGLU in the GEMM epilogue (gemm8 G8_EPI_SWIGLU): x [T, K],
// w = [gate; up] [2F, K] -> gu [T, 2F] (the projection output, kept for the backward) and
// m = silu(gate) * up [T, F].  Returns false (nothing launched) for shapes the kernel does not take.
bool gemm8_swiglu(const at::Tensor& x, const at::Tensor& w, at::Tensor& gu, at::Tensor& m) {
  MX_CHECK(x.is_cuda() && w.is_cuda() && x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16 &&
               gu.scalar_type() == at::kBFloat16 && m.scalar_type() == at::kBFloat16,
           "gemm8_swiglu: bf16 GPU tensors");
  MX_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1) && gu.size(0) == x.size(0) &&
               gu.size(1) == w.size(0) && m.size(0) == x.size(0) && 2 * m.size(1) == w.size(0),
           "gemm8_swiglu: shapes");
  if (x.stride(1) != 1 || w.stride(1) != 1 || gu.stride(1) != 1 || m.stride(1) != 1) return false;
  DevGuard g(x.device());
  MxG8Epi ep{};
  ep.m = bfm(m);
  ep.ldm = m.stride(0);
  const int rc = mx_gemm8_epi(bf(x), x.stride(0), bf(w), w.stride(0), bfm(gu), gu.stride(0), (int)x.size(0),
                              (int)w.size(0), (int)x.size(1), 2, ep, cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// The down projection's dX GEMM with the SwiGLU backward in its epilogue (gemm8 G8_EPI_SWIGLU_BWD):
// dy [T, H] and w = W_down [H, F] -> dgu [T, 2F] from the forward's gu [T, 2F] (dm never reaches
// HBM), and with m given also m = silu(g) u [T, F] (the recompute path's dW input).  Returns false
// (nothing launched) for shapes the kernel does not take.
bool gemm8_swiglu_bwd(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& gu, at::Tensor& dgu,
                      const c10::optional<at::Tensor>& m) {
  MX_CHECK(dy.is_cuda() && w.is_cuda() && gu.is_cuda() && dy.scalar_type() == at::kBFloat16 &&
               w.scalar_type() == at::kBFloat16 && gu.scalar_type() == at::kBFloat16 &&
               dgu.scalar_type() == at::kBFloat16,
           "gemm8_swiglu_bwd: bf16 GPU tensors");
  MX_CHECK(dy.dim() == 2 && w.dim() == 2 && gu.dim() == 2 && dgu.dim() == 2 && dy.size(1) == w.size(0) &&
               gu.size(0) == dy.size(0) && gu.size(1) == 2 * w.size(1) && dgu.sizes() == gu.sizes(),
           "gemm8_swiglu_bwd: shapes");
  if (m) {
    MX_CHECK(m->scalar_type() == at::kBFloat16 && m->dim() == 2 && m->size(0) == dy.size(0) &&
                 m->size(1) == w.size(1),
             "gemm8_swiglu_bwd: m [T, F] bf16");
    if (m->stride(1) != 1) return false;
  }
  if (dy.stride(1) != 1 || w.stride(1) != 1 || gu.stride(1) != 1 || dgu.stride(1) != 1) return false;
  DevGuard g(dy.device());
  MxG8Epi ep{};
  ep.gu = bf(gu);
  ep.ldg = gu.stride(0);
  if (m) {
    ep.m = reinterpret_cast<uint16_t*>(m->data_ptr());
    ep.ldm = m->stride(0);
  }
  const int rc = mx_gemm8_epi(bf(dy), dy.stride(0), bf(w), w.stride(0), bfm(dgu), dgu.stride(0), (int)dy.size(0),
                              (int)w.size(1), (int)dy.size(1), 3, ep, cur_stream());
  if (rc == -1) return false;
  MX_OK(rc);
  return true;
}

// the gemm8 diagnostic build's cycle stamps (MXLLM_GEMM8_STAMPS): int64 [1024, 2, 80] on the host
at::Tensor gemm8_stamps() {
  auto out = at::empty({1024, 2, 80}, at::TensorOptions().dtype(at::kLong));
  MX_OK(mx_gemm8_stamps(reinterpret_cast<unsigned long long*>(out.data_ptr<int64_t>())));
  return out;
}

// A HIP stream confined to a subset of the device's CUs (hipExtStreamCreateWithCUMask):
// ``mask`` = one int per 32 CUs (bit i of word w = CU 32 w + i).  Returns the stream handle
// for torch.cuda.ExternalStream; the stream lives for the process (never destroyed).
int64_t cu_masked_stream(int64_t device, std::vector<int64_t> mask) {
  MX_CHECK(!mask.empty(), "cu_masked_stream: empty mask");
  DevGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  std::vector<uint32_t> w(mask.size());
  for (size_t i = 0; i < mask.size(); ++i) w[i] = (uint32_t)(mask[i] & 0xffffffffLL);
  hipStream_t s = nullptr;
  hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)(w.size() * 32), w.data());
  MX_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
  return (int64_t)reinterpret_cast<intptr_t>(s);
}

// read `t` once on the current stream (cache warm-up of a weight ahead of its consumer; misc.hip)
void prefetch(const at::Tensor& t, int64_t wgs) {
  MX_CHECK(t.is_cuda() && t.is_contiguous(), "prefetch: contiguous GPU tensor");
  DevGuard g(t.device());
  MX_OK(mx_prefetch(t.data_ptr(), t.numel() * t.element_size(), (int)wgs, cur_stream()));
}

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

// sum(x^2) of a contiguous f32 or bf16 GPU tensor -> f32 [1]; fixed-order reduction
at::Tensor sqnorm(const at::Tensor& x) {
  MX_CHECK(x.is_cuda() && x.is_contiguous(), "x must be a contiguous GPU tensor");
  MX_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x must be float32 or bfloat16");
  DevGuard g(x.device());
  auto opts = x.options().dtype(at::kFloat);
  auto out = at::empty({1}, opts);
  auto work = at::empty({2048}, opts);
  MX_OK(mx_sqnorm(x.data_ptr(), x.scalar_type() == at::kBFloat16 ? 1 : 0, x.numel(), out.data_ptr<float>(),
                  work.data_ptr<float>(), cur_stream()));
  return out;
}

// ---------------------------------------------------------------- SwiGLU
// out_pad > 0: outputs are [T, n] views into [T, n + out_pad] buffers
at::Tensor swiglu_fwd(const at::Tensor& gu, int64_t out_pad) {
  check_bf16(gu, "gu");
  DevGuard g(gu.device());
  const int64_t F2 = gu.size(-1);
  MX_CHECK(F2 % 16 == 0, "2F must be a multiple of 16");
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  const int64_t T = gu.numel() / F2;
  at::Tensor m;
  if (out_pad > 0) {
    m = empty_rows(T, F2 / 2, out_pad, gu.options());
  } else {
    auto sizes = gu.sizes().vec();
    sizes.back() = F2 / 2;
    m = at::empty(sizes, gu.options());
  }
  if (T > 0) MX_OK(mx_swiglu_fwd(bf(gu), bfm(m), T, (int)(F2 / 2), F2 / 2 + out_pad, cur_stream()));
  return m;
}

at::Tensor swiglu_bwd(const at::Tensor& dm, const at::Tensor& gu, int64_t out_pad) {
  check_bf16(dm, "dm");
  check_bf16(gu, "gu");
  DevGuard g(gu.device());
  const int64_t F2 = gu.size(-1);
  const int64_t T = gu.numel() / F2;
  MX_CHECK(dm.numel() == T * (F2 / 2), "dm shape mismatch");
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  at::Tensor dgu = out_pad > 0 ? empty_rows(T, F2, out_pad, gu.options()) : at::empty_like(gu);
  if (T > 0) MX_OK(mx_swiglu_bwd(bf(dm), bf(gu), bfm(dgu), T, (int)(F2 / 2), F2 + out_pad, cur_stream()));
  return dgu;
}

// swiglu_bwd that also re-emits m = swiglu(gu) (bitwise the forward's) from the same read of gu:
// the backward of a linear whose input activation was recomputed instead of saved
std::vector<at::Tensor> swiglu_bwd_m(const at::Tensor& dm, const at::Tensor& gu) {
  check_bf16(dm, "dm");
  check_bf16(gu, "gu");
  DevGuard g(gu.device());
  const int64_t F2 = gu.size(-1);
  const int64_t T = gu.numel() / F2;
  MX_CHECK(dm.numel() == T * (F2 / 2), "dm shape mismatch");
  MX_CHECK(dm.is_contiguous() && gu.is_contiguous(), "swiglu_bwd_m: dense dm / gu");
  at::Tensor dgu = at::empty_like(gu);
  at::Tensor m = at::empty({T, F2 / 2}, gu.options());
  if (T > 0) MX_OK(mx_swiglu_bwd(bf(dm), bf(gu), bfm(dgu), T, (int)(F2 / 2), F2, cur_stream(), bfm(m)));
  return {dgu, m};
}

// SwiGLU fused with the LoRA tail of its augmented-GEMM neighbour (csrc/kernels/lora.hip):
// fwd: m [T, F] in a [T, F + pad] buffer, tail = alpha m v^T (v [>= 16 nrb, F] row view);
// bwd: dgu [T, 2F] in a [T, 2F + pad] buffer, tail = alpha dgu v^T (v [>= 16 nrb, 2F]).
at::Tensor swiglu_lora(const c10::optional<at::Tensor>& dm, const at::Tensor& gu, int64_t pad, const at::Tensor& v,
                       int64_t nrb, double alpha) {
  check_bf16(gu, "gu");
  const int64_t ldv = check_rows_bf16(v, "v");
  DevGuard g(gu.device());
  const bool bwd = dm.has_value();
  const int64_t F2 = gu.size(-1), F = F2 / 2, T = gu.numel() / F2;
  MX_CHECK(gu.dim() == 2 && F % 128 == 0 && T % 16 == 0, "swiglu_lora: [T, 2F] with T % 16 == 0, F % 128 == 0");
  MX_CHECK(nrb >= 1 && nrb <= 4 && pad >= 16 * nrb && pad % 8 == 0, "swiglu_lora: 16 nrb <= pad");
  MX_CHECK(v.size(0) >= 16 * nrb && v.size(1) == (bwd ? F2 : F), "swiglu_lora: v shape");
  if (bwd) {
    check_bf16(*dm, "dm");
    MX_CHECK(dm->numel() == T * F, "swiglu_lora: dm shape");
  }
  const int64_t W = bwd ? F2 : F;
  at::Tensor out = at::empty({T, W + pad}, gu.options());
  const int64_t nws = mx_swiglu_lora_ws((int)T, (int)F, (int)nrb);
  auto ws = at::empty({nws > 0 ? nws : 1}, gu.options().dtype(at::kFloat));
  if (T > 0)
    MX_OK(mx_swiglu_lora(bwd ? 1 : 0, bf(gu), bwd ? bf(*dm) : nullptr, bfm(out), W + pad, bf(v), ldv, (int)nrb,
                         (int)pad, (float)alpha, ws.data_ptr<float>(), (int)T, (int)F, cur_stream()));
  return out.narrow(1, 0, W);
}

// ---------------------------------------------------------------- AdamW
void adamw_step(const c10::optional<at::Tensor>& master, at::Tensor grad, at::Tensor m, at::Tensor v,
                const c10::optional<at::Tensor>& lowp, const c10::optional<at::Tensor>& lo, double lr, double b1,
                double b2, double eps, double wd, double bc1, double bc2, const c10::optional<at::Tensor>& scale_t,
                double scale_f, bool zero_grad) {
  // master: fp32, or absent with ``lo`` given (split master: lowp = high half, lo = int16 low half)
  MX_CHECK(master.has_value() != lo.has_value(), "give either the fp32 master or the split low half");
  check_f32(m, "m");
  check_f32(v, "v");
  MX_CHECK(grad.is_cuda() && grad.is_contiguous(), "grad must be contiguous GPU");
  MX_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16, "grad f32/bf16");
  const int64_t n = m.numel();
  MX_CHECK(grad.numel() == n && v.numel() == n, "adamw size mismatch");
  float* mp = nullptr;
  if (master.has_value()) {
    check_f32(*master, "master");
    MX_CHECK(master->numel() == n, "master size");
    mp = master->data_ptr<float>();
  }
  DevGuard g(m.device());
  uint16_t* lp = nullptr;
  if (lowp.has_value()) {
    check_bf16(*lowp, "lowp");
    MX_CHECK(lowp->numel() == n, "lowp size");
    lp = reinterpret_cast<uint16_t*>(lowp->data_ptr());
  }
  int16_t* lop = nullptr;
  if (lo.has_value()) {
    MX_CHECK(lo->is_cuda() && lo->is_contiguous() && lo->scalar_type() == at::kShort && lo->numel() == n,
             "lo must be a contiguous int16 GPU tensor of the master's size");
    MX_CHECK(lp != nullptr, "split master needs lowp (the high half)");
    lop = lo->data_ptr<int16_t>();
  }
  const float* st = nullptr;
  if (scale_t.has_value()) {
    check_f32(*scale_t, "scale_t");
    st = scale_t->data_ptr<float>();
  }
  MX_OK(mx_adamw(mp, grad.data_ptr(), grad.scalar_type() == at::kBFloat16 ? 1 : 0, m.data_ptr<float>(),
                 v.data_ptr<float>(), lp, lop, n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1,
                 (float)bc2, st, (float)scale_f, zero_grad ? 1 : 0, cur_stream()));
}

// fp32 <-> split master halves (hi bf16 = bits rounded half-up, lo int16 = remainder)
void split_master(const at::Tensor& x, at::Tensor hi, at::Tensor lo) {
  check_f32(x, "x");
  check_bf16(hi, "hi");
  MX_CHECK(lo.is_cuda() && lo.is_contiguous() && lo.scalar_type() == at::kShort, "lo int16 contiguous GPU");
  MX_CHECK(hi.numel() == x.numel() && lo.numel() == x.numel(), "split_master size mismatch");
  DevGuard g(x.device());
  MX_OK(mx_split_master(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(hi.data_ptr()), lo.data_ptr<int16_t>(),
                        x.numel(), cur_stream()));
}

void join_master(const at::Tensor& hi, const at::Tensor& lo, at::Tensor out) {
  check_bf16(hi, "hi");
  check_f32(out, "out");
  MX_CHECK(lo.is_cuda() && lo.is_contiguous() && lo.scalar_type() == at::kShort, "lo int16 contiguous GPU");
  MX_CHECK(hi.numel() == out.numel() && lo.numel() == out.numel(), "join_master size mismatch");
  DevGuard g(out.device());
  MX_OK(mx_join_master(reinterpret_cast<const uint16_t*>(hi.data_ptr()), lo.data_ptr<int16_t>(),
                       out.data_ptr<float>(), out.numel(), cur_stream()));
}

// ---------------------------------------------------------------- embedding
at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& w) {
  check_bf16(w, "weight");
  MX_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong, "ids must be int64 GPU");
  DevGuard g(w.device());
  auto idc = ids.contiguous();
  const int64_t T = idc.numel(), H = w.size(1), V = w.size(0);
  auto out = at::empty({T, H}, w.options());
  MX_OK(mx_embedding_fwd(idc.data_ptr<int64_t>(), bf(w), bfm(out), T, (int)H, V, cur_stream()));
  return out;
}

at::Tensor embedding_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t V) {
  check_bf16(dy, "dy");
  DevGuard g(dy.device());
  auto idc = ids.contiguous();
  const int64_t H = dy.size(-1), T = idc.numel();
  auto dw = at::zeros({V, H}, dy.options().dtype(at::kFloat));
  MX_OK(mx_embedding_bwd(idc.data_ptr<int64_t>(), bf(dy), dw.data_ptr<float>(), T, (int)H, V, cur_stream()));
  return dw;
}

// out[V, H] (bf16 or f32, contiguous) += the batch's rows of dW, computed from the stably
// sorted ids (sid) and their positions (perm): only touched rows read / written.
void embedding_bwd_sorted(const at::Tensor& dy, const at::Tensor& sid, const at::Tensor& perm, at::Tensor out) {
  check_bf16(dy, "dy");
  MX_CHECK(sid.scalar_type() == at::kLong && perm.scalar_type() == at::kLong && sid.is_contiguous() &&
               perm.is_contiguous() && sid.numel() == perm.numel(), "sid / perm: int64, same length");
  MX_CHECK(out.is_contiguous() && (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16) &&
               out.dim() == 2 && out.size(1) == dy.size(-1) && dy.is_contiguous() &&
               dy.numel() == sid.numel() * dy.size(-1) && out.device() == dy.device(),
           "embedding_bwd_sorted: out [V, H] f32/bf16 contiguous, dy [T, H] contiguous");
  DevGuard g(dy.device());
  const int64_t T = sid.numel(), nch = (T + 63) / 64;
  auto ws = at::empty({std::max<int64_t>(1, 2 * nch * out.size(1))}, dy.options().dtype(at::kFloat));
  MX_OK(mx_embedding_bwd_sorted(bf(dy), sid.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), T, (int)out.size(1),
                                out.size(0), out.data_ptr(), out.scalar_type() == at::kFloat ? 1 : 0,
                                ws.data_ptr<float>(), cur_stream()));
}

// ---------------------------------------------------------------- cross-entropy
// logits [T, V] bf16 is overwritten in place with d(mean loss)/d(logits).
std::tuple<at::Tensor, at::Tensor> ce_fwd_bwd(at::Tensor logits, const at::Tensor& labels, int64_t ignore) {
  check_bf16(logits, "logits");
  MX_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong, "labels must be int64 GPU");
  DevGuard g(logits.device());
  const int64_t V = logits.size(-1), T = logits.numel() / V;
  MX_CHECK(labels.numel() == T, "labels size mismatch");
  auto lab = labels.contiguous();
  auto losses = at::empty({T}, logits.options().dtype(at::kFloat));
  auto ws = at::empty({2}, logits.options().dtype(at::kFloat));
  auto loss = at::empty({}, logits.options().dtype(at::kFloat));
  MX_OK(mx_ce_fwd_bwd(bfm(logits), lab.data_ptr<int64_t>(), losses.data_ptr<float>(), ws.data_ptr<float>(),
                      loss.data_ptr<float>(), T, (int)V, ignore, cur_stream()));
  return {loss, losses};
}

// 1 / (number of labels != ignore) as a 1-element f32 device tensor (0 when none)
at::Tensor ce_inv_count(const at::Tensor& labels, int64_t ignore) {
  MX_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong, "labels must be int64 GPU");
  DevGuard g(labels.device());
  auto lab = labels.contiguous();
  auto inv = at::empty({1}, labels.options().dtype(at::kFloat));
  MX_OK(mx_ce_inv_count(lab.data_ptr<int64_t>(), lab.numel(), ignore, inv.data_ptr<float>(), cur_stream()));
  return inv;
}

// one chunk of the chunked LM-head CE: per-row losses, logits <- (softmax - onehot) * inv_n in place
at::Tensor ce_chunk(at::Tensor logits, const at::Tensor& labels, int64_t ignore, const at::Tensor& inv_n) {
  check_bf16(logits, "logits");
  MX_CHECK(logits.is_contiguous(), "ce_chunk: contiguous logits");
  MX_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong, "labels must be int64 GPU");
  MX_CHECK(inv_n.scalar_type() == at::kFloat && inv_n.numel() == 1 && inv_n.device() == logits.device(),
           "ce_chunk: inv_n f32 device scalar");
  DevGuard g(logits.device());
  const int64_t V = logits.size(-1), T = logits.numel() / V;
  MX_CHECK(labels.numel() == T, "labels size mismatch");
  auto lab = labels.contiguous();
  auto losses = at::empty({T}, logits.options().dtype(at::kFloat));
  MX_OK(mx_ce_chunk(bfm(logits), lab.data_ptr<int64_t>(), losses.data_ptr<float>(), inv_n.data_ptr<float>(), T,
                    (int)V, ignore, cur_stream()));
  return losses;
}

// fp32-logits chunk: losses [T] returned, dl (bf16 [T, V]) <- (softmax - onehot) * inv_n
at::Tensor ce_chunk_f32(const at::Tensor& logits, at::Tensor dl, const at::Tensor& labels, int64_t ignore,
                        const at::Tensor& inv_n) {
  check_f32(logits, "logits");
  check_bf16(dl, "dl");
  MX_CHECK(logits.is_contiguous() && dl.is_contiguous() && dl.sizes() == logits.sizes(), "ce_chunk_f32: shapes");
  MX_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong, "labels must be int64 GPU");
  MX_CHECK(inv_n.scalar_type() == at::kFloat && inv_n.numel() == 1 && inv_n.device() == logits.device(),
           "ce_chunk_f32: inv_n f32 device scalar");
  DevGuard g(logits.device());
  const int64_t V = logits.size(-1), T = logits.numel() / V;
  MX_CHECK(labels.numel() == T, "labels size mismatch");
  auto lab = labels.contiguous();
  auto losses = at::empty({T}, logits.options());
  MX_OK(mx_ce_chunk_f32(logits.data_ptr<float>(), bfm(dl), lab.data_ptr<int64_t>(), losses.data_ptr<float>(),
                        inv_n.data_ptr<float>(), T, (int)V, ignore, cur_stream()));
  return losses;
}

// ---------------------------------------------------------------- RoPE split / merge
std::tuple<at::Tensor, at::Tensor, at::Tensor> rope_split(const at::Tensor& qkv, const at::Tensor& cos,
                                                          const at::Tensor& sin, int64_t B, int64_t S, int64_t Hq,
                                                          int64_t Hkv, int64_t D,
                                                          const c10::optional<at::Tensor>& positions) {
  check_bf16(qkv, "qkv");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  MX_CHECK(qkv.numel() == B * S * (Hq + 2 * Hkv) * D, "qkv shape mismatch");
  MX_CHECK(cos.size(-1) == D / 2, "rope table width");
  DevGuard g(qkv.device());
  const int32_t* pos = nullptr;
  if (positions.has_value()) {
    MX_CHECK(positions->scalar_type() == at::kInt && positions->numel() == B * S, "positions int32 [B*S]");
    pos = positions->data_ptr<int32_t>();
  } else {
    MX_CHECK(cos.size(0) >= S, "rope table too short");
  }
  auto q = at::empty({B, Hq, S, D}, qkv.options());
  auto k = at::empty({B, Hkv, S, D}, qkv.options());
  auto v = at::empty({B, Hkv, S, D}, qkv.options());
  MX_OK(mx_rope_split(bf(qkv), cos.data_ptr<float>(), sin.data_ptr<float>(), pos, bfm(q), bfm(k), bfm(v), (int)B,
                      (int)S, (int)Hq, (int)Hkv, (int)D, cur_stream()));
  return {q, k, v};
}

at::Tensor rope_merge_bwd(const at::Tensor& dq, const at::Tensor& dkp, const at::Tensor& dvp, const at::Tensor& cos,
                          const at::Tensor& sin, int64_t B, int64_t S, int64_t Hq, int64_t Hkv, int64_t D,
                          int64_t out_pad) {
  check_f32(dq, "dq");
  check_f32(dkp, "dkp");
  check_f32(dvp, "dvp");
  DevGuard g(dq.device());
  const int64_t kvin = dkp.size(1);
  MX_CHECK(dkp.dim() == 4 && dkp.size(0) == B && dkp.size(2) == S && dkp.size(3) == D, "dk partial shape");
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  const int64_t NHD = (Hq + 2 * Hkv) * D;
  auto dqkv = empty_rows(B * S, NHD, out_pad, dq.options().dtype(at::kBFloat16));
  MX_OK(mx_rope_merge_bwd(dq.data_ptr<float>(), dkp.data_ptr<float>(), dvp.data_ptr<float>(), cos.data_ptr<float>(),
                          sin.data_ptr<float>(), bfm(dqkv), (int)B, (int)S, (int)Hq, (int)Hkv, (int)kvin, (int)D,
                          NHD + out_pad, cur_stream(), 0));
  return dqkv;
}

// ---------------------------------------------------------------- attention
// out_pad > 0: o [B, S, Hq*D] is a view into [B, S, Hq*D + out_pad] (row stride Hq*D + out_pad)
std::tuple<at::Tensor, at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                                            bool causal, double scale, int64_t out_pad) {
  check_bf16(q, "q");
  check_bf16(k, "k");
  check_bf16(v, "v");
  MX_CHECK(q.dim() == 4 && k.dim() == 4 && v.sizes() == k.sizes(), "q [B,Hq,S,D], k/v [B,Hkv,Sk,D]");
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(1), Sk = k.size(2);
  MX_CHECK(k.size(0) == B && k.size(3) == D && Hq % Hkv == 0, "attention shape mismatch");
  DevGuard g(q.device());
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  auto o = out_pad > 0 ? at::empty({B, S, Hq * D + out_pad}, q.options()).narrow(2, 0, Hq * D)
                       : at::empty({B, S, Hq * D}, q.options());
  auto lse = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  MX_OK(mx_attn_fwd(bf(q), bf(k), bf(v), bfm(o), lse.data_ptr<float>(), (int)B, (int)Hq, (int)Hkv, (int)S, (int)Sk,
                    (int)D, causal ? 1 : 0, (float)scale, (int)(Hq * D + out_pad), cur_stream()));
  return {o, lse};
}

// dq_mode: 1 = f32 atomics, 2 = deterministic per-key-block partials + ordered reduce,
// 3 = split (dS^T to HBM + separate dQ kernel; default, deterministic)
// outs (optional, split mode only): preallocated f32 dq [B, Hq, S, D] and dK / dV partials
// [B, P, Sk, D] to write into (e.g. head-range views of larger tensors: the chunked long-context
// backward, mxllm/ops/attention.py) instead of fresh tensors.
std::tuple<at::Tensor, at::Tensor, at::Tensor> attn_bwd_impl(const at::Tensor& dout, const at::Tensor& q,
                                                             const at::Tensor& k, const at::Tensor& v,
                                                             const at::Tensor& o, const at::Tensor& lse, int causal,
                                                             double scale, int64_t dq_mode,
                                                             const c10::optional<at::Tensor>& dq_out = c10::nullopt,
                                                             const c10::optional<at::Tensor>& dk_out = c10::nullopt,
                                                             const c10::optional<at::Tensor>& dv_out = c10::nullopt,
                                                             uint16_t* dqkv = nullptr, int64_t ldq = 0,
                                                             const float* cosb = nullptr, const float* sinb = nullptr) {
  check_bf16(dout, "dout");
  check_f32(lse, "lse");
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(1), Sk = k.size(2);
  MX_CHECK(dout.numel() == B * S * Hq * D && o.numel() == dout.numel(), "dout/o shape");
  MX_CHECK(dq_mode >= 1 && dq_mode <= 3, "dq_mode must be 1, 2 or 3");
  // o: contiguous, or token rows with a row stride (the padded attention output)
  int64_t ldo = Hq * D;
  if (!o.is_contiguous()) {
    MX_CHECK(o.is_cuda() && o.scalar_type() == at::kBFloat16 && o.dim() == 3 && o.stride(2) == 1 &&
                 o.size(2) == Hq * D && o.stride(0) == S * o.stride(1) && o.stride(1) % 8 == 0,
             "o must be [B, S, Hq*D] with unit inner stride");
    ldo = o.stride(1);
  } else {
    check_bf16(o, "o");
  }
  DevGuard g(q.device());
  const int64_t S_pad = (S + 63) / 64 * 64;
  const int64_t nkb = (Sk + 127) / 128;
  // dK / dV partials: [B, P, Sk, D] f32, P partial heads (Hq, or fewer when a workgroup of the
  // 8-wave kernel sums several q-heads of a KV group); a KV head's partials are consecutive
  const int64_t P = (causal >= 0 && dq_mode == 3)
                        ? mx_attn_bwd_partial_heads((int)B, (int)Hq, (int)Hkv, (int)S, (int)Sk, (int)D, (int)dq_mode)
                        : Hq;
  const bool outs = dq_out.has_value() || dk_out.has_value() || dv_out.has_value();
  if (outs) {
    MX_CHECK(dq_out.has_value() && dk_out.has_value() && dv_out.has_value() && dq_mode == 3 && causal >= 0,
             "attn_bwd: preallocated outputs need all three and the split mode");
    check_f32(*dq_out, "dq_out");
    check_f32(*dk_out, "dk_out");
    check_f32(*dv_out, "dv_out");
    MX_CHECK(dq_out->numel() == B * Hq * S * D && dk_out->numel() == B * P * Sk * D &&
                 dv_out->numel() == B * P * Sk * D, "attn_bwd: output sizes");
  }
  auto dkp = outs ? *dk_out : at::empty({B, P, Sk, D}, q.options().dtype(at::kFloat));
  auto dvp = outs ? *dv_out : at::empty({B, P, Sk, D}, q.options().dtype(at::kFloat));
  auto delta = at::empty({B, Hq, S}, q.options().dtype(at::kFloat));
  if (causal >= 0 && dq_mode != 1) {
    at::Tensor work = dq_mode == 2 ? at::empty({nkb, B, Hq, S_pad, D}, q.options().dtype(at::kFloat))
                                   : at::empty({B * Hq, nkb * 128, S_pad}, q.options());
    // dqkv: the dQ kernel writes d(q) into it; no fp32 dQ at all
    auto dq = outs ? *dq_out
                   : at::empty({dqkv ? 0 : B, Hq, S, D}, q.options().dtype(at::kFloat));
    MX_OK(mx_attn_bwd(bf(q), bf(k), bf(v), bf(o), bf(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
                      dq.data_ptr<float>(), dkp.data_ptr<float>(), dvp.data_ptr<float>(), (int)B, (int)Hq, (int)Hkv,
                      (int)S, (int)Sk, (int)D, causal, (float)scale, (int)dq_mode, work.data_ptr(), ldo,
                      cur_stream(), dqkv, ldq, cosb, sinb));
    return {dq, dkp, dvp};
  }
  auto dq_pad = at::zeros({B, Hq, S_pad, D}, q.options().dtype(at::kFloat));
  MX_OK(mx_attn_bwd(bf(q), bf(k), bf(v), bf(o), bf(dout), lse.data_ptr<float>(), delta.data_ptr<float>(),
                    dq_pad.data_ptr<float>(), dkp.data_ptr<float>(), dvp.data_ptr<float>(), (int)B, (int)Hq, (int)Hkv,
                    (int)S, (int)Sk, (int)D, causal, (float)scale, 1, nullptr, ldo, cur_stream(), nullptr, 0, nullptr,
                    nullptr));
  auto dq = S_pad == S ? dq_pad : dq_pad.narrow(2, 0, S).contiguous();
  return {dq, dkp, dvp};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> attn_bwd(const at::Tensor& dout, const at::Tensor& q,
                                                        const at::Tensor& k, const at::Tensor& v, const at::Tensor& o,
                                                        const at::Tensor& lse, bool causal, double scale,
                                                        int64_t dq_mode, const c10::optional<at::Tensor>& dq_out,
                                                        const c10::optional<at::Tensor>& dk_out,
                                                        const c10::optional<at::Tensor>& dv_out) {
  return attn_bwd_impl(dout, q, k, v, o, lse, causal ? 1 : 0, scale, dq_mode, dq_out, dk_out, dv_out);
}

// The attention backward straight into d(qkv) [B*S, (Hq+2Hkv)*D (+out_pad)] bf16 (D = 128, split mode):
// the dQ kernel writes the q columns with the inverse RoPE applied, rope_merge_bwd only the k / v
// columns from the dK / dV partials -- the fp32 dQ never reaches HBM (mxllm/ops/attention.py).
at::Tensor attn_bwd_rope(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                         const at::Tensor& o, const at::Tensor& lse, bool causal, double scale, const at::Tensor& cos,
                         const at::Tensor& sin, int64_t out_pad) {
  const int64_t B = q.size(0), Hq = q.size(1), S = q.size(2), D = q.size(3);
  const int64_t Hkv = k.size(1), Sk = k.size(2);
  MX_CHECK(D == 128 && Sk == S, "attn_bwd_rope: D = 128 self-attention");
  check_f32(cos, "cos");
  check_f32(sin, "sin");
  MX_CHECK(cos.is_contiguous() && sin.is_contiguous() && cos.numel() >= S * (D / 2) && sin.numel() >= S * (D / 2),
           "cos / sin: [>= S, D/2] contiguous f32");
  MX_CHECK(out_pad >= 0 && out_pad % 8 == 0, "out_pad must be a non-negative multiple of 8");
  DevGuard g(q.device());
  const int64_t NHD = (Hq + 2 * Hkv) * D;
  auto dqkv = empty_rows(B * S, NHD, out_pad, q.options());
  auto res = attn_bwd_impl(dout, q, k, v, o, lse, causal ? 1 : 0, scale, 3, c10::nullopt, c10::nullopt, c10::nullopt,
                           bfm(dqkv), NHD + out_pad, cos.data_ptr<float>(), sin.data_ptr<float>());
  const at::Tensor& dkp = std::get<1>(res);
  const at::Tensor& dvp = std::get<2>(res);
  MX_OK(mx_rope_merge_bwd(nullptr, dkp.data_ptr<float>(), dvp.data_ptr<float>(), cos.data_ptr<float>(),
                          sin.data_ptr<float>(), bfm(dqkv), (int)B, (int)S, (int)Hq, (int)Hkv, (int)dkp.size(1), (int)D,
                          NHD + out_pad, cur_stream(), (int)Hq));
  return dqkv;
}

// timing-only ablation variants (mode: -1 = causal without dQ atomics)
std::tuple<at::Tensor, at::Tensor, at::Tensor> attn_bwd_ablate(const at::Tensor& dout, const at::Tensor& q,
                                                               const at::Tensor& k, const at::Tensor& v,
                                                               const at::Tensor& o, const at::Tensor& lse,
                                                               int64_t mode, double scale) {
  return attn_bwd_impl(dout, q, k, v, o, lse, (int)mode, scale, 1);
}

// ---------------------------------------------------------------- decode
// Paged KV caches: k_cache/v_cache [blocks, Hkv, block, D] + block_table int32 [slots, maxb]
// (token p of slot s in block block_table[s][p / block]); without a block table the caches
// are [slots, Hkv, max_seq, D].
struct KvPages {
  const int32_t* bt = nullptr;
  int maxb = 0;
};
static KvPages kv_pages(const c10::optional<at::Tensor>& block_table, const at::Tensor& k_cache) {
  KvPages pg;
  if (block_table.has_value() && block_table->defined()) {
    const at::Tensor& t = *block_table;
    MX_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.dim() == 2 && t.is_contiguous(),
             "block_table int32 [slots, max_blocks] contiguous GPU");
    MX_CHECK(k_cache.size(2) % 256 == 0, "paged KV: the block size must be a multiple of 256 tokens");
    pg.bt = t.data_ptr<int32_t>();
    pg.maxb = (int)t.size(1);
  }
  return pg;
}

// qkv [B, NH*D]; k_cache/v_cache [slots, Hkv, max_seq, D] (or paged); pos/slots int32 [B]
at::Tensor rope_append(const at::Tensor& qkv, const at::Tensor& cos, const at::Tensor& sin, const at::Tensor& pos,
                       const c10::optional<at::Tensor>& slots, at::Tensor k_cache, at::Tensor v_cache, int64_t Hq,
                       int64_t Hkv, int64_t D, const c10::optional<at::Tensor>& block_table) {
  check_bf16(qkv, "qkv");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  MX_CHECK(pos.scalar_type() == at::kInt, "pos int32");
  const int64_t B = qkv.size(0);
  MX_CHECK(qkv.size(1) == (Hq + 2 * Hkv) * D, "qkv width");
  MX_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D, "cache shape");
  DevGuard g(qkv.device());
  const int32_t* sl = nullptr;
  if (slots.has_value()) sl = slots->data_ptr<int32_t>();
  auto q = at::empty({B, Hq, D}, qkv.options());
  const KvPages pg = kv_pages(block_table, k_cache);
  MX_OK(mx_rope_append(bf(qkv), cos.data_ptr<float>(), sin.data_ptr<float>(), pos.data_ptr<int32_t>(), sl, bfm(q),
                       bfm(k_cache), bfm(v_cache), (int)B, (int)Hq, (int)Hkv, (int)D, (int)k_cache.size(2), pg.bt,
                       pg.maxb, cur_stream()));
  return q;
}

at::Tensor decode_attn(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                       const at::Tensor& lens, const c10::optional<at::Tensor>& slots, int64_t max_len, double scale,
                       int64_t len_off, const c10::optional<at::Tensor>& block_table,
                       const c10::optional<at::Tensor>& counters) {
  check_bf16(q, "q");
  MX_CHECK(lens.scalar_type() == at::kInt, "lens int32");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  const int64_t Hkv = k_cache.size(1), max_seq = k_cache.size(2);
  DevGuard g(q.device());
  // counters: int32 [>= B * Hkv], zero, owned by the caller (a decode engine): the split
  // partials are merged in-launch by the last workgroup of each (seq, kv-head), which
  // resets its counter -> no combine launch (head_dim 128)
  unsigned int* cnt = nullptr;
  if (counters.has_value() && D == 128) {
    MX_CHECK(counters->scalar_type() == at::kInt && counters->is_contiguous() && counters->numel() >= B * Hkv &&
                 counters->device() == q.device(),
             "decode_attn: counters must be a contiguous int32 tensor of >= B * Hkv zeros on q's device");
    cnt = reinterpret_cast<unsigned int*>(counters->data_ptr<int32_t>());
  }
  const KvPages pg = kv_pages(block_table, k_cache);
  const int64_t cap = pg.bt ? (int64_t)pg.maxb * max_seq : max_seq;  // positions a sequence can hold
  const int64_t nsplit = std::max<int64_t>(1, (std::min(max_len, cap) + 255) / 256);
  auto ml = at::empty({B, Hq, nsplit, 2}, q.options().dtype(at::kFloat));
  auto po = at::empty({B, Hq, nsplit, D}, q.options().dtype(at::kFloat));
  auto out = at::empty({B, Hq * D}, q.options());
  const int32_t* sl = nullptr;
  if (slots.has_value()) sl = slots->data_ptr<int32_t>();
  MX_OK(mx_decode_attn(bf(q), bf(k_cache), bf(v_cache), lens.data_ptr<int32_t>(), (int)len_off, sl, ml.data_ptr<float>(),
                       po.data_ptr<float>(), bfm(out), (int)B, (int)Hq, (int)Hkv, (int)D, (int)max_seq, (int)nsplit,
                       (float)scale, pg.bt, pg.maxb, cnt, cur_stream()));
  return out;
}

// The split-K partials without the combine: (part_ml [B, Hq, nsplit, 2], part_o [B, Hq, nsplit, D]),
// merged by the o-projection's prologue (skinny_merge_linear).  D = 128.
std::tuple<at::Tensor, at::Tensor> decode_attn_partials(const at::Tensor& q, const at::Tensor& k_cache,
                                                        const at::Tensor& v_cache, const at::Tensor& lens,
                                                        const c10::optional<at::Tensor>& slots, int64_t max_len,
                                                        double scale, int64_t len_off,
                                                        const c10::optional<at::Tensor>& block_table) {
  check_bf16(q, "q");
  MX_CHECK(lens.scalar_type() == at::kInt, "lens int32");
  const int64_t B = q.size(0), Hq = q.size(1), D = q.size(2);
  MX_CHECK(D == 128, "decode_attn_partials: head_dim 128");
  const int64_t Hkv = k_cache.size(1), max_seq = k_cache.size(2);
  DevGuard g(q.device());
  const KvPages pg = kv_pages(block_table, k_cache);
  const int64_t cap = pg.bt ? (int64_t)pg.maxb * max_seq : max_seq;
  const int64_t nsplit = std::max<int64_t>(1, (std::min(max_len, cap) + 255) / 256);
  auto ml = at::empty({B, Hq, nsplit, 2}, q.options().dtype(at::kFloat));
  auto po = at::empty({B, Hq, nsplit, D}, q.options().dtype(at::kFloat));
  const int32_t* sl = nullptr;
  if (slots.has_value()) sl = slots->data_ptr<int32_t>();
  MX_OK(mx_decode_attn(bf(q), bf(k_cache), bf(v_cache), lens.data_ptr<int32_t>(), (int)len_off, sl, ml.data_ptr<float>(),
                       po.data_ptr<float>(), nullptr, (int)B, (int)Hq, (int)Hkv, (int)D, (int)max_seq, (int)nsplit,
                       (float)scale, pg.bt, pg.maxb, nullptr, cur_stream()));
  return {ml, po};
}

// y [M, N] = merge(part_ml, part_o) . W^T (decode o-projection with the split merge in the prologue)
at::Tensor skinny_merge_linear(const at::Tensor& ml, const at::Tensor& po, const at::Tensor& w) {
  MX_CHECK(ml.is_cuda() && ml.scalar_type() == at::kFloat && ml.is_contiguous() && ml.dim() == 4 && ml.size(3) == 2,
           "part_ml f32 [M, Hq, nsplit, 2]");
  MX_CHECK(po.is_cuda() && po.scalar_type() == at::kFloat && po.is_contiguous() && po.dim() == 4 &&
               po.size(0) == ml.size(0) && po.size(1) == ml.size(1) && po.size(2) == ml.size(2) && po.size(3) == 128,
           "part_o f32 [M, Hq, nsplit, 128]");
  MX_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1, "w bf16 [N, K] rows");
  const int64_t M = ml.size(0), K = ml.size(1) * 128, N = w.size(0);
  MX_CHECK(w.size(1) == K, "w [N, Hq * 128]");
  DevGuard g(w.device());
  auto y = at::empty({M, N}, w.options());
  MX_OK(mx_skinny_merge_gemm(ml.data_ptr<float>(), po.data_ptr<float>(), (int)ml.size(2), bf(w), w.stride(0), bfm(y),
                             N, (int)M, (int)N, (int)K, cur_stream()));
  return y;
}

at::Tensor sample(const at::Tensor& logits, double temperature, int64_t seed, int64_t step) {
  MX_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "logits [B, V] contiguous GPU");
  MX_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16/f32");
  DevGuard g(logits.device());
  auto out = at::empty({logits.size(0)}, logits.options().dtype(at::kLong));
  auto ws = at::empty({std::max<int64_t>(1, mx_sample_ws_floats((int)logits.size(0)))},
                      logits.options().dtype(at::kFloat));  // per-call partials (stream-ordered allocator)
  MX_OK(mx_sample(logits.data_ptr(), logits.scalar_type() == at::kBFloat16 ? 1 : 0, out.data_ptr<int64_t>(),
                  (int)logits.size(0), (int)logits.size(1), (float)temperature, (uint32_t)seed, (uint32_t)step,
                  ws.data_ptr<float>(), cur_stream()));
  return out;
}

// per-row temperature / seed / step without top-k / top-p (the split-vocabulary kernel of
// decode.hip; same draws as sample_rows for such rows)
at::Tensor sample_temp_rows(const at::Tensor& logits, const at::Tensor& temps, const at::Tensor& seeds,
                            const at::Tensor& steps) {
  MX_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "logits [B, V] contiguous GPU");
  MX_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16/f32");
  const int64_t B = logits.size(0);
  auto chk = [&](const at::Tensor& t, at::ScalarType st, const char* name) {
    MX_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == st && t.numel() == B, name);
  };
  chk(temps, at::kFloat, "temps f32 [B]");
  chk(seeds, at::kLong, "seeds i64 [B]");
  chk(steps, at::kInt, "steps i32 [B]");
  DevGuard g(logits.device());
  auto out = at::empty({B}, logits.options().dtype(at::kLong));
  auto ws = at::empty({std::max<int64_t>(1, mx_sample_ws_floats((int)B))}, logits.options().dtype(at::kFloat));
  MX_OK(mx_sample_temp_rows(logits.data_ptr(), logits.scalar_type() == at::kBFloat16 ? 1 : 0,
                            out.data_ptr<int64_t>(), (int)B, (int)logits.size(1), temps.data_ptr<float>(),
                            seeds.data_ptr<int64_t>(), steps.data_ptr<int32_t>(), ws.data_ptr<float>(),
                            cur_stream()));
  return out;
}

at::Tensor sample_rows(const at::Tensor& logits, const at::Tensor& temps, const at::Tensor& top_p,
                       const at::Tensor& top_k, const at::Tensor& seeds, const at::Tensor& steps) {
  MX_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "logits [B, V] contiguous GPU");
  MX_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16/f32");
  const int64_t B = logits.size(0);
  auto chk = [&](const at::Tensor& t, at::ScalarType st, const char* name) {
    MX_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == st && t.numel() == B, name);
  };
  chk(temps, at::kFloat, "temps f32 [B]");
  chk(top_p, at::kFloat, "top_p f32 [B]");
  chk(top_k, at::kInt, "top_k i32 [B]");
  chk(seeds, at::kLong, "seeds i64 [B]");
  chk(steps, at::kInt, "steps i32 [B]");
  DevGuard g(logits.device());
  auto out = at::empty({B}, logits.options().dtype(at::kLong));
  MX_OK(mx_sample_rows(logits.data_ptr(), logits.scalar_type() == at::kBFloat16 ? 1 : 0, out.data_ptr<int64_t>(),
                       (int)B, (int)logits.size(1), temps.data_ptr<float>(), top_p.data_ptr<float>(),
                       top_k.data_ptr<int32_t>(), seeds.data_ptr<int64_t>(), steps.data_ptr<int32_t>(),
                       cur_stream()));
  return out;
}

}  // namespace


// ---------------------------------------------------------------- bf16 decode GEMM (serving)
// y[M, N] = x[M, K] . w[N, K]^T for M <= 32 tokens: the weight-streaming HIP kernel
// (csrc/kernels/skinny_gemm.hip).  Callers check the shape contract (mxllm/ops/linear.py).
at::Tensor skinny_linear(const at::Tensor& x, const at::Tensor& w) {
  MX_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x: bf16 [M, K] rows");
  MX_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1, "w: bf16 [N, K] rows");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  MX_CHECK(w.size(1) == K && M >= 1 && M <= 32 && N % 16 == 0 && K % 512 == 0 && x.stride(0) % 8 == 0 &&
               w.stride(0) % 8 == 0, "skinny_linear shape contract");
  DevGuard g(x.device());
  auto y = at::empty({M, N}, x.options());
  MX_OK(mx_skinny_gemm(bf(x), x.stride(0), bf(w), w.stride(0), bfm(y), N, (int)M, (int)N, (int)K, cur_stream()));
  return y;
}

// y[M, F] = swiglu(x[M, K] . w[2F, K]^T) for M <= 32 tokens, w = [gate; up] rows: the decode
// MLP's first projection with SwiGLU in the GEMM epilogue (csrc/kernels/skinny_gemm.hip).
at::Tensor skinny_linear_swiglu(const at::Tensor& x, const at::Tensor& w) {
  MX_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x: bf16 [M, K] rows");
  MX_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1, "w: bf16 [2F, K] rows");
  const int64_t M = x.size(0), K = x.size(1), F = w.size(0) / 2;
  MX_CHECK(w.size(1) == K && w.size(0) == 2 * F && M >= 1 && M <= 32 && F % 8 == 0 && K % 512 == 0 &&
               x.stride(0) % 8 == 0 && w.stride(0) % 8 == 0, "skinny_linear_swiglu shape contract");
  DevGuard g(x.device());
  auto y = at::empty({M, F}, x.options());
  MX_OK(mx_skinny_gemm_swiglu(bf(x), x.stride(0), bf(w), w.stride(0), bfm(y), F, (int)M, (int)F, (int)K,
                              cur_stream()));
  return y;
}

// Decode rows (M <= 4): y = rmsnorm(h + delta) . w^T with the RMSNorm (and residual add) in the
// GEMM prologue (csrc/kernels/skinny_gemm.hip NORM); swiglu: w = [gate; up], y = silu(g) * u.
// Returns (y, h + delta) — the new residual is h itself when delta is absent.
std::tuple<at::Tensor, at::Tensor> skinny_norm_linear(const at::Tensor& h, const c10::optional<at::Tensor>& delta,
                                                      const at::Tensor& gamma, double eps, const at::Tensor& w,
                                                      bool swiglu) {
  MX_CHECK(h.is_cuda() && h.scalar_type() == at::kBFloat16 && h.dim() == 2 && h.stride(1) == 1, "h: bf16 [M, K] rows");
  MX_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1, "w: bf16 [N, K] rows");
  const int64_t M = h.size(0), K = h.size(1), N = w.size(0);
  MX_CHECK(gamma.is_cuda() && gamma.scalar_type() == at::kBFloat16 && gamma.is_contiguous() && gamma.numel() == K,
           "gamma: bf16 [K]");
  MX_CHECK(w.size(1) == K && M >= 1 && M <= 4 && M * K <= 32768 && N % 16 == 0 && K % 512 == 0 &&
               h.stride(0) % 8 == 0 && w.stride(0) % 8 == 0 && (!swiglu || N % 16 == 0),
           "skinny_norm_linear shape contract");
  const uint16_t* dp = nullptr;
  int64_t ldd = 0;
  at::Tensor h_out = h;
  if (delta.has_value() && delta->defined()) {
    const at::Tensor& d = *delta;
    MX_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16 && d.dim() == 2 && d.size(0) == M && d.size(1) == K &&
                 d.stride(1) == 1 && d.stride(0) % 8 == 0, "delta: bf16 [M, K] rows");
    dp = bf(d);
    ldd = d.stride(0);
    h_out = at::empty({M, K}, h.options());
  }
  DevGuard g(h.device());
  const int64_t Ny = swiglu ? N / 2 : N;
  auto y = at::empty({M, Ny}, h.options());
  MX_OK(mx_skinny_norm_gemm(bf(h), h.stride(0), dp, ldd, bf(gamma), (float)eps, dp ? bfm(h_out) : nullptr, bf(w),
                            w.stride(0), bfm(y), Ny, (int)M, (int)N, (int)K, swiglu ? 1 : 0, cur_stream()));
  return {y, h_out};
}

// Decode QKV projection with the RoPE / KV-cache append in the GEMM epilogue and, when gamma is
// given, the (residual-add +) RMSNorm in its prologue (csrc/kernels/skinny_gemm.hip ROPE / NORM).
// Returns (q [M, Hq, 128] rotated, new residual); K/V rows land in the caches at (slot, pos).
std::tuple<at::Tensor, at::Tensor> skinny_qkv_rope(const at::Tensor& h, const c10::optional<at::Tensor>& delta,
                                                   const c10::optional<at::Tensor>& gamma, double eps,
                                                   const at::Tensor& w, const at::Tensor& cosb, const at::Tensor& sinb,
                                                   const at::Tensor& pos, const c10::optional<at::Tensor>& slots,
                                                   at::Tensor& k_cache, at::Tensor& v_cache, int64_t Hq, int64_t Hkv,
                                                   const c10::optional<at::Tensor>& block_table) {
  MX_CHECK(h.is_cuda() && h.scalar_type() == at::kBFloat16 && h.dim() == 2 && h.stride(1) == 1, "h: bf16 [M, K] rows");
  MX_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.stride(1) == 1, "w: bf16 [N, K] rows");
  const int64_t M = h.size(0), K = h.size(1);
  const bool norm = gamma.has_value() && gamma->defined();
  MX_CHECK(w.size(0) == (Hq + 2 * Hkv) * 128 && w.size(1) == K && M >= 1 && M <= (norm ? 4 : 16) && K % 512 == 0 &&
               (!norm || M * K <= 32768) && h.stride(0) % 8 == 0 && w.stride(0) % 8 == 0,
           "skinny_qkv_rope shape contract");
  MX_CHECK(cosb.scalar_type() == at::kFloat && sinb.scalar_type() == at::kFloat && cosb.is_contiguous() &&
               sinb.is_contiguous() && cosb.size(-1) == 64, "cos/sin f32 [max_pos, 64]");
  MX_CHECK(pos.scalar_type() == at::kInt && pos.numel() == M, "pos int32 [M]");
  check_bf16(k_cache, "k_cache");
  check_bf16(v_cache, "v_cache");
  MX_CHECK(k_cache.size(1) == Hkv && k_cache.size(3) == 128 && k_cache.is_contiguous() && v_cache.is_contiguous(),
           "caches [slots, Hkv, max_seq, 128]");
  const int32_t* sl = nullptr;
  if (slots.has_value() && slots->defined()) {
    MX_CHECK(slots->scalar_type() == at::kInt && slots->numel() == M, "slots int32 [M]");
    sl = slots->data_ptr<int32_t>();
  }
  const uint16_t* dp = nullptr;
  int64_t ldd = 0;
  at::Tensor h_out = h;
  if (norm && delta.has_value() && delta->defined()) {
    const at::Tensor& d = *delta;
    MX_CHECK(d.is_cuda() && d.scalar_type() == at::kBFloat16 && d.dim() == 2 && d.size(0) == M && d.size(1) == K &&
                 d.stride(1) == 1 && d.stride(0) % 8 == 0, "delta: bf16 [M, K] rows");
    dp = bf(d);
    ldd = d.stride(0);
    h_out = at::empty({M, K}, h.options());
  }
  if (norm)
    MX_CHECK(gamma->scalar_type() == at::kBFloat16 && gamma->is_contiguous() && gamma->numel() == K, "gamma bf16 [K]");
  DevGuard g(h.device());
  auto q = at::empty({M, Hq, 128}, h.options());
  const KvPages pg = kv_pages(block_table, k_cache);
  MX_OK(mx_skinny_rope_gemm(bf(h), h.stride(0), norm ? 1 : 0, dp, ldd, norm ? bf(*gamma) : nullptr, (float)eps,
                            dp ? bfm(h_out) : nullptr, bf(w), w.stride(0), cosb.data_ptr<float>(),
                            sinb.data_ptr<float>(), pos.data_ptr<int32_t>(), sl, bfm(q), bfm(k_cache),
                            bfm(v_cache), (int)Hq, (int)Hkv, (int)k_cache.size(2), pg.bt, pg.maxb, (int)M, (int)K, cur_stream()));
  return {q, h_out};
}

// ---------------------------------------------------------------- fp8 weights (serving)
// y[M, N] = x[M, K] . (scale[:, None] * q[N, K])^T ; q: e4m3 codes (uint8), scale f32 [N].
// M <= 32: the fused weight-streaming kernel; otherwise dequantise to bf16 and run the
// hipBLASLt GEMM.  mxllm/serve/quant.py calls this only up to SMALL_M (8) tokens and
// routes larger calls to the fp8 x fp8 hipBLASLt GEMM.
at::Tensor w8_linear(const at::Tensor& x, const at::Tensor& q, const at::Tensor& scale) {
  MX_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x: bf16 [M, K] rows");
  MX_CHECK(q.is_cuda() && q.scalar_type() == at::kByte && q.dim() == 2 && q.is_contiguous(), "q: uint8 [N, K]");
  check_f32(scale, "scale");
  const int64_t M = x.size(0), K = x.size(1), N = q.size(0);
  MX_CHECK(q.size(1) == K && scale.numel() == N, "w8_linear shapes");
  DevGuard g(x.device());
  if (M <= 32 && N % 16 == 0 && K % 512 == 0 && x.stride(0) % 8 == 0) {
    auto y = at::empty({M, N}, x.options());
    MX_OK(mx_w8a16_gemm(bf(x), x.stride(0), q.data_ptr<uint8_t>(), scale.data_ptr<float>(), bfm(y), N, (int)M,
                        (int)N, (int)K, cur_stream()));
    return y;
  }
  auto w = at::empty({N, K}, x.options());
  MX_OK(mx_w8_dequant(q.data_ptr<uint8_t>(), scale.data_ptr<float>(), bfm(w), N, (int)K, cur_stream()));
  return at::mm(x, w.t());
}

// per-token e4m3 quantisation of bf16 rows: (codes uint8 [M, K], scale f32 [M, 1])
std::tuple<at::Tensor, at::Tensor> quant_rows_e4m3(const at::Tensor& x) {
  MX_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x: bf16 [M, K] rows");
  DevGuard g(x.device());
  const int64_t M = x.size(0), K = x.size(1);
  auto q = at::empty({M, K}, x.options().dtype(at::kByte));
  auto s = at::empty({M, 1}, x.options().dtype(at::kFloat));
  MX_OK(mx_quant_rows_e4m3(bf(x), x.stride(0), q.data_ptr<uint8_t>(), s.data_ptr<float>(), M, (int)K,
                           cur_stream()));
  return {q, s};
}

at::Tensor w8_dequant(const at::Tensor& q, const at::Tensor& scale) {
  MX_CHECK(q.is_cuda() && q.scalar_type() == at::kByte && q.dim() == 2 && q.is_contiguous(), "q: uint8 [N, K]");
  check_f32(scale, "scale");
  DevGuard g(q.device());
  auto w = at::empty({q.size(0), q.size(1)}, q.options().dtype(at::kBFloat16));
  MX_OK(mx_w8_dequant(q.data_ptr<uint8_t>(), scale.data_ptr<float>(), bfm(w), q.size(0), (int)q.size(1),
                      cur_stream()));
  return w;
}

// ---------------------------------------------------------------- LoRA rank-r GEMMs
// out[:, 0:Vrows] = alpha * x . v^T (x [M, K], v [Vrows, K] row views, Vrows % 64 == 0):
// the forward s x A^T / backward s dy B products written into the augmented-GEMM tails.
// rows > 0: only v's first `rows` rows are non-zero (the adapter; the rest is padding).
void lora_xwt(const at::Tensor& x, const at::Tensor& v, at::Tensor& out, double alpha, int64_t rows) {
  const int64_t ldx = check_rows_bf16(x, "x"), ldv = check_rows_bf16(v, "v"), ldo = check_rows_bf16(out, "out");
  const int64_t M = x.size(0), K = x.size(1), Vr = v.size(0);
  MX_CHECK(v.size(1) == K && out.size(0) == M && out.size(1) >= Vr, "lora_xwt shapes");
  MX_CHECK(rows >= 0 && rows <= Vr, "lora_xwt: rows <= rows(v)");
  MX_CHECK(M % 16 == 0 && K % 64 == 0 && Vr % 64 == 0 && ldo % 4 == 0,
           "lora_xwt: M % 16, K % 64, rows(v) % 64");
  DevGuard g(x.device());
  const int64_t nws = mx_lora_xwt_ws((int)M, (int)K, (int)rows);
  auto ws = at::empty({nws > 0 ? nws : 1}, x.options().dtype(at::kFloat));
  MX_OK(mx_lora_xwt(bf(x), ldx, bf(v), ldv, (int)Vr, bfm(out), ldo, ws.data_ptr<float>(), (int)M, (int)K, (float)alpha,
                    (int)rows, cur_stream()));
}

// LoRA adapter gradients in ONE launch: ga [R, K] (+)= g^T x and the diagonal blocks
// gb[off_i : off_i + n_i, i r : (i + 1) r] (+)= dy_i^T st_i.  x [T, K], dy [T, N], and the
// tails g [T, >= 64], st [T, >= 64] (row views); r % 16 == 0.
void lora_grads(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& g, const at::Tensor& st, at::Tensor& ga,
                at::Tensor& gb, at::IntArrayRef splits, int64_t r, bool accumulate) {
  const int64_t ldx = check_rows_bf16(x, "x"), ldd = check_rows_bf16(dy, "dy");
  const int64_t ldg = check_rows_bf16(g, "g"), lds = check_rows_bf16(st, "st");
  check_bf16(ga, "ga");
  check_bf16(gb, "gb");
  const int64_t T = x.size(0), K = x.size(1), N = dy.size(1), n = (int64_t)splits.size(), R = n * r;
  MX_CHECK(dy.size(0) == T && g.size(0) == T && st.size(0) == T, "lora_grads: token counts differ");
  MX_CHECK(ga.size(0) == R && ga.size(1) == K && gb.size(0) == N && gb.size(1) == R, "lora_grads: grad shapes");
  MX_CHECK(T % 64 == 0 && K % 64 == 0 && r % 16 == 0 && r <= 64, "lora_grads: T, K multiples of 64, r of 16");
  std::vector<int64_t> desc;
  auto add = [&](const uint16_t* X, int64_t lx, const uint16_t* G, int64_t lg, int64_t gw, uint16_t* out, int64_t os_n,
                 int64_t os_j, int64_t Nx, int64_t jb0, int64_t JB) {
    // JB > 1 reads a 64-column G window starting at column 16 jb0
    MX_CHECK(JB == 1 || 16 * jb0 + 64 <= gw, "lora_grads: operand tail too narrow");
    MX_CHECK(Nx % 64 == 0, "lora_grads: split sizes must be multiples of 64");
    desc.insert(desc.end(), {(int64_t)X, (int64_t)G, (int64_t)out, lx, lg, os_n, os_j, Nx, jb0, JB});
  };
  // dA: R columns of g in chunks of <= 4 blocks
  for (int64_t j0 = 0; j0 < R; j0 += 64) {
    const int64_t jb = std::min<int64_t>(4, (R - j0) / 16);
    add(bf(x), ldx, bf(g), ldg, g.size(1), bfm(ga) + j0 * K, 1, K, K, j0 / 16, jb);
  }
  int64_t off = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t ni = splits[i];
    add(bf(dy) + off, ldd, bf(st), lds, st.size(1), bfm(gb) + off * R + i * r, R, 1, ni, i * r / 16, r / 16);
    off += ni;
  }
  MX_CHECK(off == N, "lora_grads: splits do not sum to dy's width");
  const int np = (int)(desc.size() / 10);
  MX_CHECK(np <= 8, "lora_grads: too many problems");
  int64_t ntiles = 0;
  for (int i = 0; i < np; ++i) ntiles += desc[i * 10 + 7] / 64;
  DevGuard gd(x.device());
  const int64_t nws = mx_lora_xtg_ws((int)ntiles, (int)T);
  auto ws = at::empty({nws > 0 ? nws : 1}, x.options().dtype(at::kFloat));
  MX_OK(mx_lora_xtg(desc.data(), np, (int)T, 1.0f, accumulate ? 1 : 0, ws.data_ptr<float>(), cur_stream()));
}

TORCH_LIBRARY(mxllm, m) {
  m.def("rmsnorm_fwd(Tensor x, Tensor? res, Tensor w, float eps, int out_pad=0) -> (Tensor, Tensor, Tensor)");
  m.def("rmsnorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor rstd, Tensor? dres, bool need_dw, int out_pad=0) -> (Tensor, Tensor)");
  m.def("segmented_mean(Tensor codes, Tensor offsets) -> Tensor");
  m.def("copy2d_batched(Tensor desc, int total_blocks) -> ()");
  m.def("transpose2d(Tensor x, Tensor? scale=None) -> Tensor");
  m.def("gemm8(Tensor a, bool a_kc, Tensor b, bool b_kc, Tensor(a!) out, float beta, Tensor? alpha_t=None, float alpha=1.0, int ph=8) -> bool");
  m.def("prefetch(Tensor t, int wgs) -> ()");
  m.def("cu_masked_stream(int device, int[] mask) -> int", &cu_masked_stream);  // no tensor args: catch-all
  m.def("gemm8_stamps() -> Tensor", &gemm8_stamps);
  m.def("gemm8_tail(Tensor a, bool a_kc, Tensor b, bool b_kc, Tensor(a!) out, int at, bool rows=False, int ph=4, Tensor(b!)? sq=None) -> bool");
  m.def("gemm8_rope(Tensor x, Tensor w, Tensor cos, Tensor sin, int B, int S, int Hq, int Hkv, Tensor(a!) q, Tensor(b!) k, Tensor(c!) v) -> bool");
  m.def("gemm8_rope_tail(Tensor x, Tensor w, Tensor cos, Tensor sin, int B, int S, int Hq, int Hkv, Tensor(a!) q, Tensor(b!) k, Tensor(c!) v, int at) -> bool");
  m.def("gemm8_swiglu(Tensor x, Tensor w, Tensor(a!) gu, Tensor(b!) m) -> bool");
  m.def("gemm8_sq(Tensor a, bool a_kc, Tensor b, bool b_kc, Tensor(a!) out, Tensor(b!) sq, Tensor? alpha_t=None, float alpha=1.0) -> bool");
  m.def("gemm8_swiglu_bwd(Tensor dy, Tensor w, Tensor gu, Tensor(a!) dgu, Tensor(b!)? m=None) -> bool");
  m.def("sqnorm(Tensor x) -> Tensor");
  m.def("swiglu_fwd(Tensor gu, int out_pad=0) -> Tensor");
  m.def("swiglu_bwd(Tensor dm, Tensor gu, int out_pad=0) -> Tensor");
  m.def("swiglu_bwd_m(Tensor dm, Tensor gu) -> Tensor[]");
  m.def("adamw_step(Tensor(a!)? master, Tensor(e!) grad, Tensor(b!) m, Tensor(c!) v, Tensor(d!)? lowp, Tensor(f!)? lo, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, Tensor? scale_t, float scale_f, bool zero_grad=False) -> ()");
  m.def("split_master(Tensor x, Tensor(a!) hi, Tensor(b!) lo) -> ()");
  m.def("join_master(Tensor hi, Tensor lo, Tensor(a!) out) -> ()");
  m.def("embedding_fwd(Tensor ids, Tensor w) -> Tensor");
  m.def("embedding_bwd(Tensor dy, Tensor ids, int V) -> Tensor");
  m.def("embedding_bwd_sorted(Tensor dy, Tensor sid, Tensor perm, Tensor(a!) out) -> ()");
  m.def("ce_fwd_bwd(Tensor(a!) logits, Tensor labels, int ignore_index) -> (Tensor, Tensor)");
  m.def("ce_inv_count(Tensor labels, int ignore_index) -> Tensor");
  m.def("ce_chunk(Tensor(a!) logits, Tensor labels, int ignore_index, Tensor inv_n) -> Tensor");
  m.def("ce_chunk_f32(Tensor logits, Tensor(a!) dl, Tensor labels, int ignore_index, Tensor inv_n) -> Tensor");
  m.def("rope_split(Tensor qkv, Tensor cos, Tensor sin, int B, int S, int Hq, int Hkv, int D, Tensor? positions=None) -> (Tensor, Tensor, Tensor)");
  m.def("rope_merge_bwd(Tensor dq, Tensor dkp, Tensor dvp, Tensor cos, Tensor sin, int B, int S, int Hq, int Hkv, int D, int out_pad=0) -> Tensor");
  m.def("attn_fwd(Tensor q, Tensor k, Tensor v, bool causal, float scale, int out_pad=0) -> (Tensor, Tensor)");
  m.def("rope_append(Tensor qkv, Tensor cos, Tensor sin, Tensor pos, Tensor? slots, Tensor(a!) k_cache, Tensor(b!) v_cache, int Hq, int Hkv, int D, Tensor? block_table=None) -> Tensor");
  m.def("decode_attn(Tensor q, Tensor k_cache, Tensor v_cache, Tensor lens, Tensor? slots, int max_len, float scale, int len_off=0, Tensor? block_table=None, Tensor? counters=None) -> Tensor");
  m.def("decode_attn_partials(Tensor q, Tensor k_cache, Tensor v_cache, Tensor lens, Tensor? slots, int max_len, float scale, int len_off=0, Tensor? block_table=None) -> (Tensor, Tensor)");
  m.def("skinny_merge_linear(Tensor ml, Tensor po, Tensor w) -> Tensor");
  m.def("sample(Tensor logits, float temperature, int seed, int step) -> Tensor");
  m.def("sample_rows(Tensor logits, Tensor temps, Tensor top_p, Tensor top_k, Tensor seeds, Tensor steps) -> Tensor");
  m.def("sample_temp_rows(Tensor logits, Tensor temps, Tensor seeds, Tensor steps) -> Tensor");
  m.def("w8_linear(Tensor x, Tensor q, Tensor scale) -> Tensor");
  m.def("skinny_linear(Tensor x, Tensor w) -> Tensor");
  m.def("skinny_linear_swiglu(Tensor x, Tensor w) -> Tensor");
  m.def("skinny_qkv_rope(Tensor h, Tensor? delta, Tensor? gamma, float eps, Tensor w, Tensor cos, Tensor sin, Tensor pos, Tensor? slots, Tensor(a!) k_cache, Tensor(b!) v_cache, int Hq, int Hkv, Tensor? block_table=None) -> (Tensor, Tensor)");
  m.def("skinny_norm_linear(Tensor h, Tensor? delta, Tensor gamma, float eps, Tensor w, bool swiglu) -> (Tensor, Tensor)");
  m.def("w8_dequant(Tensor q, Tensor scale) -> Tensor");
  m.def("quant_rows_e4m3(Tensor x) -> (Tensor, Tensor)");
  m.def("lora_xwt(Tensor x, Tensor v, Tensor(a!) out, float alpha, int rows=0) -> ()");
  m.def("swiglu_lora(Tensor? dm, Tensor gu, int pad, Tensor v, int nrb, float alpha) -> Tensor");
  m.def("lora_grads(Tensor x, Tensor dy, Tensor g, Tensor st, Tensor(a!) ga, Tensor(b!) gb, int[] splits, int r, bool accumulate) -> ()");
  m.def("attn_bwd_ablate(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, int mode, float scale) -> (Tensor, Tensor, Tensor)");
  m.def("attn_bwd(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal, float scale, int dq_mode=3, Tensor? dq_out=None, Tensor? dk_out=None, Tensor? dv_out=None) -> (Tensor, Tensor, Tensor)");
  m.def("attn_bwd_rope(Tensor dout, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal, float scale, Tensor cos, Tensor sin, int out_pad=0) -> Tensor");
}

TORCH_LIBRARY_IMPL(mxllm, CUDA, m) {
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("segmented_mean", &segmented_mean);
  m.impl("copy2d_batched", &copy2d_batched);
  m.impl("transpose2d", &transpose2d);
  m.impl("gemm8", &gemm8);
  m.impl("gemm8_tail", &gemm8_tail);
  m.impl("gemm8_rope", &gemm8_rope);
  m.impl("gemm8_rope_tail", &gemm8_rope_tail);
  m.impl("gemm8_swiglu", &gemm8_swiglu);
  m.impl("gemm8_sq", &gemm8_sq);
  m.impl("gemm8_swiglu_bwd", &gemm8_swiglu_bwd);
  m.impl("ce_inv_count", &ce_inv_count);
  m.impl("ce_chunk", &ce_chunk);
  m.impl("ce_chunk_f32", &ce_chunk_f32);
  m.impl("prefetch", &prefetch);
  m.impl("sqnorm", &sqnorm);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("swiglu_bwd_m", &swiglu_bwd_m);
  m.impl("adamw_step", &adamw_step);
  m.impl("split_master", &split_master);
  m.impl("join_master", &join_master);
  m.impl("embedding_fwd", &embedding_fwd);
  m.impl("embedding_bwd", &embedding_bwd);
  m.impl("embedding_bwd_sorted", &embedding_bwd_sorted);
  m.impl("ce_fwd_bwd", &ce_fwd_bwd);
  m.impl("rope_split", &rope_split);
  m.impl("rope_merge_bwd", &rope_merge_bwd);
  m.impl("attn_fwd", &attn_fwd);
  m.impl("attn_bwd", &attn_bwd);
  m.impl("attn_bwd_rope", &attn_bwd_rope);
  m.impl("attn_bwd_ablate", &attn_bwd_ablate);
  m.impl("rope_append", &rope_append);
  m.impl("decode_attn_partials", &decode_attn_partials);
  m.impl("skinny_merge_linear", &skinny_merge_linear);
  m.impl("decode_attn", &decode_attn);
  m.impl("sample", &sample);
  m.impl("sample_rows", &sample_rows);
  m.impl("sample_temp_rows", &sample_temp_rows);
  m.impl("w8_linear", &w8_linear);
  m.impl("skinny_linear", &skinny_linear);
  m.impl("skinny_linear_swiglu", &skinny_linear_swiglu);
  m.impl("skinny_qkv_rope", &skinny_qkv_rope);
  m.impl("skinny_norm_linear", &skinny_norm_linear);
  m.impl("w8_dequant", &w8_dequant);
  m.impl("quant_rows_e4m3", &quant_rows_e4m3);
  m.impl("lora_xwt", &lora_xwt);
  m.impl("swiglu_lora", &swiglu_lora);
  m.impl("lora_grads", &lora_grads);
}
