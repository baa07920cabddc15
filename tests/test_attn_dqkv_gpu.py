"""The attention backward straight into d(qkv) (``attn_bwd_rope``: the split dQ kernel applies the
inverse RoPE and writes the q columns, rope_merge_bwd only the k / v columns) against the two-step
path (fp32 dQ + dK / dV partials -> rope_merge_bwd), which the kernel tests check against fp32."""
import math

import pytest
import torch

from mxllm.ops import reference as ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,Hq,Hkv,S,causal,pad", [(2, 8, 2, 512, True, 0), (1, 8, 8, 300, True, 64),
                                                    (2, 4, 1, 192, False, 0), (1, 64, 8, 2048, True, 64)])
def test_attn_bwd_rope_matches_two_step(gpu, B, Hq, Hkv, S, causal, pad):
    from mxllm.ops import native

    ops = native()
    torch.manual_seed(S + Hq)
    D = 128
    q = torch.randn(B, Hq, S, D, device=gpu).to(torch.bfloat16)
    k = torch.randn(B, Hkv, S, D, device=gpu).to(torch.bfloat16)
    v = torch.randn(B, Hkv, S, D, device=gpu).to(torch.bfloat16)
    do = torch.randn(B, S, Hq * D, device=gpu).to(torch.bfloat16)
    cos, sin = ref.rope_tables(S, D, 500000.0, None, gpu)
    scale = 1.0 / math.sqrt(D)
    o, lse = ops.attn_fwd(q, k, v, causal, scale)
    dq, dkp, dvp = ops.attn_bwd(do, q, k, v, o, lse, causal, scale, 3)
    want = ops.rope_merge_bwd(dq, dkp, dvp, cos, sin, B, S, Hq, Hkv, D, pad)
    got = ops.attn_bwd_rope(do, q, k, v, o, lse, causal, scale, cos, sin, pad)
    NHD = (Hq + 2 * Hkv) * D
    assert got.shape == want.shape and got.stride() == want.stride()
    g, w = got[:, :NHD].float(), want[:, :NHD].float()
    bad = (g != w).nonzero()
    assert bad.numel() == 0, (f"{bad.shape[0]} of {g.numel()} differ; max abs {float((g - w).abs().max()):.3g}; "
                              f"rows {bad[:6, 0].tolist()} cols {bad[:6, 1].tolist()} (q cols < {Hq * D}); "
                              f"got {g[bad[:6, 0], bad[:6, 1]].tolist()} want {w[bad[:6, 0], bad[:6, 1]].tolist()}")
