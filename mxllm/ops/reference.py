"""Pure-PyTorch reference implementations of every mxllm op.

They define the semantics the HIP kernels must match, run the CPU path (gloo
plumbing runs / CPU tests), and serve as fp32 numerics oracles in the kernel
parity tests.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def llama3_inv_freq(head_dim: int, theta: float, scaling: dict | None) -> torch.Tensor:
    """Llama-3.1 RoPE frequencies (theta 500000, factor 8, low/high 1/4,
    original context 8192), computed in float64 on the host."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if not scaling:
        return inv
    factor = scaling.get("factor", 8.0)
    lf = scaling.get("low_freq_factor", 1.0)
    hf = scaling.get("high_freq_factor", 4.0)
    old = scaling.get("original_max_position_embeddings", 8192)
    low_wl, high_wl = old / lf, old / hf
    wl = 2 * math.pi / inv
    out = torch.where(wl > low_wl, inv / factor, inv)
    smooth = (old / wl - lf) / (hf - lf)
    mid = (1 - smooth) * out / factor + smooth * out
    is_mid = (wl >= high_wl) & (wl <= low_wl)
    return torch.where(is_mid, mid, out)


def rope_tables(seq_len: int, head_dim: int, theta: float, scaling: dict | None, device=None):
    """cos/sin tables [S, D/2] float32 (host-precomputed, guide App. B)."""
    inv = llama3_inv_freq(head_dim, theta, scaling)
    t = torch.arange(seq_len, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x [B, S, H, D] with the "rotate-half" (HF Llama) pairing (i, i + D/2)."""
    S, D = x.shape[1], x.shape[-1]
    c = cos[:S].view(1, S, 1, D // 2).float()
    s = sin[:S].view(1, S, 1, D // 2).float()
    xf = x.float()
    x1, x2 = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = True,
              scale: float | None = None) -> torch.Tensor:
    """q [B, S, Hq, D], k/v [B, Sk, Hkv, D] -> o [B, S, Hq, D]  (GQA, fp32 math).
    Causal alignment is bottom-right (query i sees keys <= i + Sk - S)."""
    B, S, Hq, D = q.shape
    Sk, Hkv = k.shape[1], k.shape[2]
    rep = Hq // Hkv
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(rep, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        i = torch.arange(S, device=q.device).view(S, 1)
        j = torch.arange(Sk, device=q.device).view(1, Sk)
        s = s.masked_fill(j > i + (Sk - S), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, vf)
    return o.transpose(1, 2).to(q.dtype)


def swiglu(gate_up: torch.Tensor) -> torch.Tensor:
    """gate_up [..., 2F] laid out [gate | up] -> silu(gate) * up  [..., F]."""
    F_ = gate_up.shape[-1] // 2
    g, u = gate_up[..., :F_].float(), gate_up[..., F_:].float()
    return (F.silu(g) * u).to(gate_up.dtype)


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    return F.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction="mean")


def adamw_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, *, lr: float, beta1: float,
           beta2: float, eps: float, weight_decay: float, step: int, grad_scale: float = 1.0,
           p_lowp: torch.Tensor | None = None) -> None:
    """Decoupled-weight-decay Adam on fp32 master ``p`` (in place)."""
    gf = g.float() * grad_scale
    m.mul_(beta1).add_(gf, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(gf, gf, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    p.mul_(1 - lr * weight_decay)
    denom = (v / bc2).sqrt_().add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if p_lowp is not None:
        p_lowp.copy_(p)
