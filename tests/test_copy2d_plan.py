"""Host-side plan of the batched adapter copy (mxllm/ops/linear.py ``copy2d_plan``, consumed by
csrc/kernels/misc.hip ``copy2d_batched_kernel``): descriptor rows and block counts on CPU tensors --
4,096 elements per block, or one 64 x 64 source tile per block for a transposing copy."""
import torch

from mxllm.ops.linear import copy2d_plan


def test_plan_blocks_and_descriptors():
    a = torch.zeros(48, 8192, dtype=torch.bfloat16)            # A rows -> rows of the augmented buffer
    big = torch.zeros(10304, 8256, dtype=torch.bfloat16)
    b = torch.zeros(10240, 16, dtype=torch.bfloat16)            # B -> columns of the augmented buffer
    bt = torch.zeros(48, 10240 + 64, dtype=torch.bfloat16)      # B^T image: a transposing copy
    rag_src = torch.zeros(70, 37, dtype=torch.bfloat16)
    rag_dst = torch.zeros(50, 100, dtype=torch.bfloat16)
    pairs = [(a, big[10240:10288, :8192]), (b, big[:10240, 8192:8208]),
             (torch.zeros(10240, 48, dtype=torch.bfloat16), bt[:, :10240].t()),
             (rag_src, rag_dst[3:40, 10:80].t())]
    rows, total = copy2d_plan(pairs)
    blocks = [(48 * 8192 + 4095) // 4096, (10240 * 16 + 4095) // 4096, (10240 // 64) * 1, 2 * 1]
    assert total == sum(blocks)
    firsts = [r[6] for r in rows]
    assert firsts == [sum(blocks[:i]) for i in range(len(blocks))]
    # {src, dst, rows, cols, src_ld, dst_ld, first_block, src_col_stride, dst_col_stride}
    assert rows[2][2:6] == [10240, 48, 48, 1] and rows[2][7:] == [1, 10240 + 64]
    assert rows[3][2:4] == [70, 37] and rows[3][8] == 100
    assert rows[0][7:] == [1, 1] and rows[1][5] == 8256


def test_plan_strided_source_is_not_tiled():
    src = torch.zeros(24, 40, dtype=torch.bfloat16).t()  # column-major source: the element path
    dst = torch.zeros(40, 24, dtype=torch.bfloat16)
    rows, total = copy2d_plan([(src, dst)])
    assert total == (40 * 24 + 4095) // 4096 and rows[0][7] == 40 and rows[0][8] == 1
