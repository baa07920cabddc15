"""Batched strided 2-D copy (csrc/kernels/misc.hip ``copy2d_batched``: every LoRA adapter into its
augmented GEMM buffer in one launch) against torch's copy, on both of its paths: 16-B units for
contiguous, 8-element-multiple rows on aligned bases, 64 x 64 LDS tiles for transposing copies
(column-major destination views), and the element-wise fallback."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _desc(pairs):
    from mxllm.ops.linear import copy2d_plan

    rows, total = copy2d_plan(pairs)
    return torch.tensor(rows, dtype=torch.int64, device=pairs[0][0].device), total


def test_copy2d_batched_matches_torch(gpu):
    from mxllm.ops import native

    torch.manual_seed(0)
    dev = gpu
    big = torch.zeros(10240 + 64, 8192 + 64, dtype=torch.bfloat16, device=dev)  # an augmented [[W, B], [A, 0]]
    a = torch.randn(48, 8192, device=dev).to(torch.bfloat16)   # A rows -> rows 10240.. (vector path)
    bmat = torch.randn(10240, 16, device=dev).to(torch.bfloat16)  # B -> columns 8192.. (16-element rows)
    odd_src = torch.randn(37, 13, device=dev).to(torch.bfloat16)  # 13 columns: element path
    odd_dst = torch.zeros(64, 40, dtype=torch.bfloat16, device=dev)
    t_src = torch.randn(24, 40, device=dev).to(torch.bfloat16).t()  # strided source (column-major view)
    t_dst = torch.zeros(40, 24, dtype=torch.bfloat16, device=dev)
    off_dst = torch.zeros(8 * 1000 + 1, dtype=torch.bfloat16, device=dev)[1:].view(1000, 8)  # 2-B offset base
    off_src = torch.randn(1000, 8, device=dev).to(torch.bfloat16)
    # transposing copies (the B^T / A images): a column-major destination view, 64 x 64 LDS tiles,
    # ragged edges on both axes
    bt = torch.zeros(48, 10240 + 64, dtype=torch.bfloat16, device=dev)
    tr_src = torch.randn(10240, 48, device=dev).to(torch.bfloat16)
    wxt = torch.zeros(8192, 8192 + 40, dtype=torch.bfloat16, device=dev)
    tr_src2 = torch.randn(16, 8192, device=dev).to(torch.bfloat16)
    rag_dst = torch.zeros(50, 100, dtype=torch.bfloat16, device=dev)
    rag_src = torch.randn(70, 37, device=dev).to(torch.bfloat16)
    pairs = [(a, big[10240:10288, :8192]), (bmat, big[:10240, 8192:8208]), (odd_src, odd_dst[5:42, 3:16]),
             (t_src, t_dst), (off_src, off_dst), (tr_src, bt[:, :10240].t()), (tr_src2, wxt[:, 8192:8208].t()),
             (rag_src, rag_dst[3:40, 10:80].t())]
    want = [d.clone() for _, d in pairs]
    for (s, _), w in zip(pairs, want):
        w.copy_(s)
    desc, blocks = _desc(pairs)
    native().copy2d_batched(desc, blocks)
    torch.cuda.synchronize()
    for (s, d), w in zip(pairs, want):
        assert torch.equal(d, w)
    # nothing outside the destination windows was written
    assert torch.count_nonzero(big[:10240, :8192]) == 0 and torch.count_nonzero(big[:, 8208:]) == 0
    assert torch.count_nonzero(odd_dst[:5]) == 0 and torch.count_nonzero(odd_dst[:, 16:]) == 0
    assert torch.count_nonzero(bt[:, 10240:]) == 0 and torch.count_nonzero(wxt[:, :8192]) == 0
    assert torch.count_nonzero(wxt[:, 8208:]) == 0
    assert int(torch.count_nonzero(rag_dst)) == int(torch.count_nonzero(rag_src))
