import torch, sys
sys.path.insert(0, '.')
from mxllm.ops import native
from mxllm.ops.reference import rope_tables
ops = native()
dev = torch.device('cuda', 0)
def mat(r, c, seed):
    g = torch.Generator(device=dev); g.manual_seed(seed)
    return ((torch.rand(r, c, device=dev, generator=g) * 2 - 1)).to(torch.bfloat16)
for (B, S, Hq, Hkv, K, at) in [(2, 256, 4, 2, 576, 512), (1, 512, 8, 4, 1088, 1024), (1, 512, 8, 4, 1088, 512), (2, 256, 8, 4, 1024, 1024), (1, 512, 8, 4, 1024, 1024)]:
    N = (Hq + 2 * Hkv) * 128
    x = mat(B * S, K, 1); w = mat(N, K, 2)
    cos, sin = (t.to(dev).float().contiguous() for t in rope_tables(S, 128, 500000.0, None))
    qkv = torch.empty(B * S, N, dtype=torch.bfloat16, device=dev)
    assert ops.gemm8_tail(x, True, w, True, qkv, at, False, 4)
    q0, k0, v0 = ops.rope_split(qkv, cos, sin, B, S, Hq, Hkv, 128)
    q = torch.full((B, Hq, S, 128), float('nan'), dtype=torch.bfloat16, device=dev)
    k = torch.full((B, Hkv, S, 128), float('nan'), dtype=torch.bfloat16, device=dev)
    v = torch.full_like(k, float('nan'))
    assert ops.gemm8_rope_tail(x, w, cos, sin, B, S, Hq, Hkv, q, k, v, at)
    torch.cuda.synchronize()
    out = []
    for name, a, b in (('q', q, q0), ('k', k, k0), ('v', v, v0)):
        ne = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
        n = int(ne.sum())
        nan = int(torch.isnan(a).sum())
        idx = ne.nonzero()[:3].tolist() if n else []
        out.append(f"{name}: diff {n} nan {nan} first {idx}")
    print((B, S, Hq, Hkv, K, at), ' | '.join(out), flush=True)
