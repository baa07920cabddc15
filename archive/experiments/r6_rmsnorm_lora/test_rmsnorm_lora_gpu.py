"""RMSNorm + LoRA tail in one kernel (csrc/kernels/rmsnorm_lora.hip) against a plain PyTorch fp32
reference and against the unfused rmsnorm_fwd + lora_xwt pair it replaces."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _full(y, pad):
    """The [T, H + pad] buffer whose left part is the row view ``y``."""
    return y.as_strided((y.shape[0], y.shape[1] + pad), (y.stride(0), 1))


@pytest.mark.parametrize("T,H,rows,resid", [(4096, 8192, 48, True), (4096, 8192, 32, True), (256, 4096, 64, True),
                                            (512, 2048, 16, False), (64, 8192, 40, True)])
def test_rmsnorm_lora_fwd(gpu, T, H, rows, resid):
    from mxllm.ops._ext import native

    ops = native()
    pad, eps, alpha = 64, 1e-5, 2.0
    g = torch.Generator(device=gpu).manual_seed(T + H + rows)
    x = torch.randn(T, H, device=gpu, generator=g).bfloat16()
    res = torch.randn(T, H, device=gpu, generator=g).bfloat16() if resid else None
    w = (1 + 0.1 * torch.randn(H, device=gpu, generator=g)).bfloat16()
    vbuf = torch.zeros(64, H + pad, device=gpu, dtype=torch.bfloat16)  # as in the augmented weight buffer
    vbuf[:rows, :H] = (0.02 * torch.randn(rows, H, device=gpu, generator=g)).bfloat16()
    v = vbuf[:, :H]

    y, rstd, h = ops.rmsnorm_lora_fwd(x, res, w, eps, pad, v, alpha, rows)
    yf = _full(y, pad)
    # fp32 reference of the same op
    hr = (x.float() + res.float()).bfloat16() if resid else x
    if resid:
        assert torch.equal(h, hr)  # the residual is rounded and stored as before
    hf = hr.float()
    rs_ref = torch.rsqrt(hf.pow(2).mean(1) + eps)
    assert torch.allclose(rstd, rs_ref, rtol=1e-5, atol=0)
    y_ref = (hf * rs_ref[:, None] * w.float()).bfloat16()
    # rstd is summed in another order than the row kernel: at most a bf16 rounding flip per element
    d = (y.float() - y_ref.float()).abs()
    assert (d <= y_ref.float().abs() * 2 ** -7 + 1e-6).all()
    assert (d > 0).float().mean() < 1e-3
    tail_ref = alpha * (y.float() @ v[:rows].float().t())  # from the stored bf16 values, fp32
    tail = yf[:, H:H + rows].float()
    assert torch.allclose(tail, tail_ref, rtol=1e-2, atol=1e-2 * tail_ref.abs().max().item() / 64)
    assert torch.equal(yf[:, H + rows:], torch.zeros_like(yf[:, H + rows:]))

    # the unfused pair it replaces: the same y (up to the rstd flips) and a matching tail
    y0, rstd0, _ = ops.rmsnorm_fwd(x, res, w, eps, pad)
    ops.lora_xwt(y0, v, _full(y0, pad)[:, H:], alpha, rows)
    t0 = _full(y0, pad)[:, H:].float()
    assert torch.allclose(rstd, rstd0, rtol=1e-5, atol=0)
    assert torch.allclose(tail, t0[:, :rows], rtol=1e-2, atol=1e-2 * t0.abs().max().item() / 64)


def test_rmsnorm_lora_fwd_declines(gpu):
    """Shapes the kernel does not take raise (callers check the predicate first)."""
    from mxllm.ops._ext import native

    ops = native()
    x = torch.randn(48, 8192, device=gpu).bfloat16()  # T % 16 == 0 but H 8192 with 64 rows: declined
    w = torch.ones(8192, device=gpu, dtype=torch.bfloat16)
    v = torch.zeros(64, 8192, device=gpu, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.rmsnorm_lora_fwd(x, None, w, 1e-5, 64, v, 1.0, 64)
    with pytest.raises(RuntimeError):
        ops.rmsnorm_lora_fwd(x[:40], None, w, 1e-5, 64, v, 1.0, 16)  # T % 16
