"""gemm8 fused epilogues (csrc/kernels/gemm8.hip G8_EPI_ROPE / G8_EPI_SWIGLU forward,
G8_EPI_SWIGLU_BWD backward; mxllm/ops/fused.py) vs fp32 PyTorch references, vs the unfused
kernels they replace, and through autograd inside the Llama layer."""
import math

import pytest
import torch

from mxllm.ops import reference as ref

pytestmark = pytest.mark.gpu


def _ops():
    from mxllm.ops import native

    return native()


def _mat(rows, cols, dev, seed, scale=1.0, pad=0):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    buf = ((torch.rand(rows, cols + pad, device=dev, generator=g) * 2 - 1) * scale).to(torch.bfloat16)
    return buf[:, :cols]


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm()).item()


@pytest.mark.parametrize("B,S,Hq,Hkv,K", [(1, 256, 4, 2, 512), (2, 512, 8, 2, 1024), (1, 2048, 32, 8, 4096)])
def test_gemm8_rope_epilogue(gpu, B, S, Hq, Hkv, K):
    D = 128
    N = (Hq + 2 * Hkv) * D
    x = _mat(B * S, K, gpu, 1, pad=64)  # row-strided (LoRA-style padded rows)
    w = _mat(N, K, gpu, 2, scale=0.05)
    cos, sin = ref.rope_tables(S + 17, D, 500000.0, {"factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                     "original_max_position_embeddings": 8192}, gpu)
    q = torch.empty(B, Hq, S, D, device=gpu, dtype=torch.bfloat16)
    k = torch.empty(B, Hkv, S, D, device=gpu, dtype=torch.bfloat16)
    v = torch.empty_like(k)
    assert _ops().gemm8_rope(x, w, cos, sin, B, S, Hq, Hkv, q, k, v)
    # fp32 reference: projection -> split -> rotate-half RoPE
    y = (x.float() @ w.float().t()).view(B, S, Hq + 2 * Hkv, D)
    qr = ref.apply_rope(y[:, :, :Hq], cos, sin).transpose(1, 2)
    kr = ref.apply_rope(y[:, :, Hq:Hq + Hkv], cos, sin).transpose(1, 2)
    vr = y[:, :, Hq + Hkv:].transpose(1, 2)
    for got, want in ((q, qr), (k, kr), (v, vr)):
        assert _rel(got, want) < 5e-3
        assert (got.float() - want).abs().max().item() < 0.05 * want.abs().max().item()
    # the unfused path on the same GEMM: gemm8 (4-phase) -> rope_split, bitwise (the rotation's fma
    # contraction is pinned in both kernels: common.h rope_lo / rope_hi)
    qkv = torch.empty(B * S, N, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(x, True, w, True, qkv, 0.0, None, 1.0, 4)
    q2, k2, v2 = _ops().rope_split(qkv, cos, sin, B, S, Hq, Hkv, D)
    assert torch.equal(v, v2) and torch.equal(q, q2) and torch.equal(k, k2)


@pytest.mark.parametrize("T,F,K", [(256, 128, 512), (512, 1024, 1024), (4096, 14336, 4096)])
def test_gemm8_swiglu_epilogue(gpu, T, F, K):
    x = _mat(T, K, gpu, 3)
    w = _mat(2 * F, K, gpu, 4, scale=0.05)
    gu = torch.empty(T, 2 * F, device=gpu, dtype=torch.bfloat16)
    mbuf = torch.empty(T, F + 64, device=gpu, dtype=torch.bfloat16)
    m = mbuf[:, :F]
    assert _ops().gemm8_swiglu(x, w, gu, m)
    y = x.float() @ w.float().t()
    assert _rel(gu, y) < 5e-3
    mr = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
    assert _rel(m, mr) < 1e-2
    # bitwise equal to the unfused kernels on the same GEMM result
    gu2 = torch.empty_like(gu)
    assert _ops().gemm8(x, True, w, True, gu2, 0.0, None, 1.0, 4)
    assert torch.equal(gu, gu2)
    assert torch.equal(m, _ops().swiglu_fwd(gu2, 0))


@pytest.mark.parametrize("T,F,H,pad", [(256, 256, 512, 0), (512, 1024, 1024, 64), (4096, 14336, 4096, 0)])
def test_gemm8_swiglu_bwd_epilogue(gpu, T, F, H, pad):
    """dgu (and the recomputed m) from the down projection's dX GEMM epilogue: against fp32
    autograd, and bitwise against the unfused gemm8 NN GEMM -> swiglu_bwd / swiglu_bwd_m."""
    dy = _mat(T, H, gpu, 5)
    wd = _mat(H, F, gpu, 6, scale=0.05, pad=pad)  # W_down [H, F] (row-strided when pad)
    gu = _mat(T, 2 * F, gpu, 7, scale=2.0, pad=pad)
    dgu = torch.empty(T, 2 * F, device=gpu, dtype=torch.bfloat16)
    m = torch.empty(T, F, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8_swiglu_bwd(dy, wd, gu, dgu, m)
    guf = gu.float().requires_grad_(True)
    mr = torch.nn.functional.silu(guf[:, :F]) * guf[:, F:]
    mr.backward(dy.float() @ wd.float())
    assert _rel(dgu, guf.grad) < 1e-2
    assert _rel(m, mr.detach()) < 1e-2
    # the unfused path on the same GEMM kernel: bitwise
    dm = torch.empty(T, F, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(dy, True, wd, False, dm, 0.0, None, 1.0, 4)
    assert torch.equal(dgu, _ops().swiglu_bwd(dm, gu.contiguous(), 0))
    dgu2, m2 = _ops().swiglu_bwd_m(dm, gu.contiguous())
    assert torch.equal(dgu, dgu2) and torch.equal(m, m2)
    # without m: the same dgu
    dgu3 = torch.zeros_like(dgu)
    assert _ops().gemm8_swiglu_bwd(dy, wd, gu, dgu3)
    assert torch.equal(dgu3, dgu)


def test_gemm8_swiglu_bwd_declines_odd_shapes(gpu):
    dy = _mat(200, 512, gpu, 1)  # T % 256 != 0
    wd = _mat(512, 256, gpu, 2)
    gu = _mat(200, 512, gpu, 3)
    assert not _ops().gemm8_swiglu_bwd(dy, wd, gu, torch.empty_like(gu))


def test_fused_layer_matches_unfused_autograd(gpu, monkeypatch):
    """A 2-layer full fine-tune model (head dim 128): loss and every parameter gradient equal
    between the fused-epilogue forward and the unfused ops (the same GEMM kernel underneath)."""
    from mxllm.models import Llama, get_config
    from mxllm.ops import fused

    monkeypatch.setenv("MXLLM_GEMM8", "all")  # unfused path on gemm8 too: comparable GEMM results
    cfg = get_config("tiny-d128").replace(n_layers=2, vocab_size=512)
    torch.manual_seed(0)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=gpu)
    res = {}
    for on in (True, False):
        monkeypatch.setattr(fused, "_ON", on)
        calls = []
        for name in ("qkv_attention", "gate_up_swiglu_down"):
            real = getattr(fused, name)
            monkeypatch.setattr(fused, name, lambda *a, _r=real, _n=name, **k: (calls.append(_n), _r(*a, **k))[1])
        model = Llama(cfg, device=gpu, dtype=torch.bfloat16, seed=3)
        loss = model(ids, ids)
        loss.backward()
        res[on] = (float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters()})
        assert (len(calls) == 4) == on, calls
        monkeypatch.undo()
        monkeypatch.setenv("MXLLM_GEMM8", "all")
    (l1, g1), (l0, g0) = res[True], res[False]
    assert abs(l1 - l0) < 1e-3 * abs(l0)
    for n in g0:
        assert _rel(g1[n], g0[n]) < 2e-2, n


def test_fused_mlp_backward_matches_two_step(gpu, monkeypatch):
    """The gate-up + SwiGLU + down MLP with the SwiGLU backward in the dm GEMM's epilogue gives
    bitwise the loss and gradients of the two-step backward (dm GEMM -> swiglu_bwd) on gemm8."""
    from mxllm.models import Llama, get_config
    from mxllm.ops import fused

    monkeypatch.setenv("MXLLM_GEMM8", "all")
    cfg = get_config("tiny-d128").replace(n_layers=2, vocab_size=512)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=gpu, generator=torch.Generator(device=gpu).manual_seed(1))
    res = {}
    for on in (True, False):
        monkeypatch.setattr(fused, "_BWD_ON", on)
        calls = []
        real = fused.swiglu_bwd_gemm
        monkeypatch.setattr(fused, "swiglu_bwd_gemm", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
        model = Llama(cfg, device=gpu, dtype=torch.bfloat16, seed=3)
        loss = model(ids, ids)
        loss.backward()
        res[on] = (float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters()})
        assert (len(calls) == 2) == on, calls
    (l1, g1), (l0, g0) = res[True], res[False]
    assert l1 == l0
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n


def test_fused_mlp_recompute_m_bitwise(gpu, monkeypatch):
    """the recompute path (un-checkpointed layers of a selectively checkpointed
    run keep only gu and rebuild m) through the fused gate-up + SwiGLU epilogue, with m rebuilt by the
    dm GEMM's epilogue, gives bitwise the loss and gradients of the fused path that SAVES m -- and
    no standalone SwiGLU pass runs (``swiglu_linear`` is not called)."""
    from mxllm.models import Llama, get_config, llama

    monkeypatch.setenv("MXLLM_GEMM8", "all")
    cfg = get_config("tiny-d128").replace(n_layers=2, vocab_size=512)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=gpu, generator=torch.Generator(device=gpu).manual_seed(4))
    res = {}
    for rec in ("1", "0"):
        monkeypatch.setattr(llama, "RECOMPUTE_SWIGLU", rec)
        monkeypatch.setattr(llama, "RECOMPUTE_NORM", "0")
        calls = []
        real = llama.ops.swiglu_linear
        monkeypatch.setattr(llama.ops, "swiglu_linear", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
        model = Llama(cfg, device=gpu, dtype=torch.bfloat16, seed=3)
        loss = model(ids, ids)
        loss.backward()
        res[rec] = (float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters()})
        assert not calls, "the recompute path must not run the standalone SwiGLU"
    (l1, g1), (l0, g0) = res["1"], res["0"]
    assert l1 == l0
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n


@pytest.mark.parametrize("B,S,Hq,Hkv,K,at", [(2, 256, 4, 2, 576, 512), (1, 512, 8, 4, 1088, 1024),
                                              (2, 2048, 64, 8, 8256, 8192)])
def test_gemm8_rope_tail_bitwise(gpu, B, S, Hq, Hkv, K, at):
    """The tail-balanced qkv GEMM with RoPE fused (plain part through the epilogue, split part's sum
    pass rotating and scattering) writes bitwise the q / k / v of gemm8_tail(at) + rope_split --
    the LoRA augmented qkv forward it replaces (K = in + pad, 70B shape included)."""
    from mxllm.ops.reference import rope_tables

    N = (Hq + 2 * Hkv) * 128
    x = _mat(B * S, K, gpu, 1)
    w = _mat(N, K, gpu, 2)
    cos, sin = (t.to(gpu).float().contiguous() for t in rope_tables(S, 128, 500000.0, None))
    qkv = torch.empty(B * S, N, dtype=torch.bfloat16, device=gpu)
    assert _ops().gemm8_tail(x, True, w, True, qkv, at, False, 4)
    q0, k0, v0 = _ops().rope_split(qkv, cos, sin, B, S, Hq, Hkv, 128)
    q = torch.full((B, Hq, S, 128), float("nan"), dtype=torch.bfloat16, device=gpu)
    k = torch.full((B, Hkv, S, 128), float("nan"), dtype=torch.bfloat16, device=gpu)
    v = torch.full_like(k, float("nan"))
    assert _ops().gemm8_rope_tail(x, w, cos, sin, B, S, Hq, Hkv, q, k, v, at)
    assert torch.equal(q, q0) and torch.equal(k, k0) and torch.equal(v, v0)


def test_lora_qkv_attention_matches_unfused(gpu, monkeypatch):
    """A 2-layer LoRA model (head dim 128) whose q/k/v projection takes the tail-balanced launch:
    loss and every adapter gradient bitwise equal with the RoPE-fused LoRA qkv path
    (ops.lora_qkv_attention) and without it (augmented GEMM -> rope_split -> attention)."""
    from mxllm.models import Llama, get_config
    import importlib

    from mxllm.ops import gemm

    lin_mod = importlib.import_module("mxllm.ops.linear")  # the module (mxllm.ops.linear is also a function name)

    monkeypatch.setenv("MXLLM_GEMM8", "all")
    cfg = get_config("tiny-d128").replace(n_layers=2, vocab_size=512)
    B, S = 2, 256
    gemm._table()
    key = ("tn", B * S, (cfg.n_heads + 2 * cfg.n_kv_heads) * 128, cfg.hidden + 64, "bf16")
    monkeypatch.setitem(gemm._TAIL, key, 512)  # the unfused forward takes the same tail-balanced launch
    ids = torch.randint(0, cfg.vocab_size, (B, S), device=gpu, generator=torch.Generator(device=gpu).manual_seed(6))
    res = {}
    for on in (True, False):
        monkeypatch.setattr(lin_mod, "_LORA_QKV_ROPE", on)
        calls = []
        real = lin_mod._LoRAQKVAttnFn.apply
        monkeypatch.setattr(lin_mod._LoRAQKVAttnFn, "apply", lambda *a, _r=real: (calls.append(1), _r(*a))[1])
        model = Llama(cfg, device=gpu, dtype=torch.bfloat16, seed=3, lora_r=16)
        with torch.no_grad():
            for i, mod in enumerate(model.modules()):
                if getattr(mod, "lora_r", 0):
                    for blk in mod.lora_b_blocks():
                        blk.copy_(torch.randn(blk.shape, generator=torch.Generator().manual_seed(i)) * 0.02)
        model.sync_adapters_()
        loss = model(ids, ids)
        loss.backward()
        res[on] = (float(loss), {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None})
        assert (len(calls) == cfg.n_layers) == on, calls
        monkeypatch.setattr(lin_mod._LoRAQKVAttnFn, "apply", real)
    (l1, g1), (l0, g0) = res[True], res[False]
    assert l1 == l0
    assert set(g1) == set(g0) and g0
    for n in g0:
        assert torch.equal(g1[n], g0[n]), n
