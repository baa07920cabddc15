"""Sampling semantics (the reference's OpenAI-compatible
completion() at /root/reference/src/distributed_inference.py:37).

CPU: the fp32 oracle applies temperature BEFORE the top-k / nucleus cut.
GPU: the batched HIP sampler (csrc/kernels/sampling.hip) draws from exactly
that distribution (empirical frequencies vs the oracle), keeps greedy rows
greedy in a mixed batch, and reproduces the temperature-only kernel's draws.
"""
import pytest
import torch

from mxllm.ops import decode as dops


def test_filter_probs_tempers_before_nucleus():
    x = torch.tensor([2.0, 1.0, 0.0, -1.0])
    cold = dops.filter_probs(x, 0.25, 0, 0.9)  # sharp: the top token alone reaches 0.9
    hot = dops.filter_probs(x, 4.0, 0, 0.9)    # flat: needs all four
    assert (cold > 0).sum() == 1 and (hot > 0).sum() == 4
    k2 = dops.filter_probs(x, 1.0, 2, 1.0)
    assert (k2 > 0).tolist() == [True, True, False, False]
    assert abs(float(k2.sum()) - 1.0) < 1e-6


def test_cpu_sample_rows_respects_support():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3, 64, generator=g)
    ids = dops.sample_rows(x, [0.0, 0.8, 1.5], [1.0, 0.5, 0.9], [0, 0, 5], [1, 2, 3], [0, 0, 0])
    assert ids[0] == x[0].argmax()
    assert dops.filter_probs(x[1], 0.8, 0, 0.5)[ids[1]] > 0
    assert dops.filter_probs(x[2], 1.5, 5, 0.9)[ids[2]] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("V,temp,top_k,top_p", [(1000, 0.7, 50, 0.9), (1000, 1.3, 0, 0.8), (777, 1.0, 20, 1.0)])
def test_gpu_sampler_frequencies(gpu, V, temp, top_k, top_p):
    g = torch.Generator().manual_seed(V)
    row = (torch.randn(V, generator=g) * 2.0).to(torch.bfloat16)
    n = 20000
    logits = row.to(gpu).unsqueeze(0).expand(n, V).contiguous()
    ids = dops.sample_rows(logits, [temp] * n, [top_p] * n, [top_k] * n, [7] * n, list(range(n))).cpu()
    ref = dops.filter_probs(row.float(), temp, top_k, top_p)
    emp = torch.bincount(ids, minlength=V).float() / n
    assert (emp[ref == 0] == 0).all(), "drew a token outside the top-k / top-p set"
    tv = 0.5 * (emp - ref).abs().sum().item()
    assert tv < 0.04, tv


@pytest.mark.gpu
def test_gpu_sampler_mixed_batch_and_vocab_128k(gpu):
    V = 128256
    x = torch.randn(4, V, device=gpu).to(torch.bfloat16)
    ids = dops.sample_rows(x, [0.0, 0.9, 0.9, 1.0], [1.0, 1.0, 0.9, 0.5], [0, 0, 0, 40], [3, 3, 3, 3],
                           [5, 5, 5, 5]).cpu()
    assert ids[0] == x[0].float().argmax().item()
    # temperature-only rows draw exactly what the single-row Gumbel kernel draws
    from mxllm.ops import native

    one = native().sample(x[1:2].contiguous(), 0.9, 3, 5).cpu()
    assert ids[1] == one[0]
    assert dops.filter_probs(x[2].float().cpu(), 0.9, 0, 0.9)[ids[2]] > 0
    assert dops.filter_probs(x[3].float().cpu(), 1.0, 40, 0.5)[ids[3]] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,V", [(torch.bfloat16, 128256), (torch.float32, 50001)])
def test_gpu_temperature_rows_split_kernel_matches_topkp_kernel(gpu, dtype, V):
    """Rows without top-k / top-p go to the vocabulary-split kernel (decode.hip); its draws
    equal the radix-select kernel's (sampling.hip) for the same (seed, step) noise."""
    from mxllm.ops import native

    B = 6
    x = torch.randn(B, V, device=gpu).to(dtype)
    temps = torch.tensor([0.0, 0.7, 1.0, 1.3, 0.0, 0.2], device=gpu)
    seeds = torch.tensor([1, 2, 3, 4, 5, 123456789], device=gpu, dtype=torch.int64)
    steps = torch.tensor([0, 9, 17, 3, 1, 1000], device=gpu, dtype=torch.int32)
    ones = torch.ones(B, device=gpu)
    zeros = torch.zeros(B, device=gpu, dtype=torch.int32)
    for _ in range(3):
        a = native().sample_temp_rows(x, temps, seeds, steps)
        b = native().sample_rows(x, temps, ones, zeros, seeds, steps)
        assert torch.equal(a, b)
        steps += 1
    # routed entry point
    ids = dops.sample_rows(x, temps.tolist(), [1.0] * B, [0] * B, seeds.tolist(), steps.tolist())
    assert torch.equal(ids, native().sample_rows(x, temps, ones, zeros, seeds, steps))


def test_top_p_zero_is_greedy_cpu():
    """top_p <= 0 (an empty nucleus) samples greedily; NaN is rejected; SamplingParams
    validates its range (the kernel and the oracle used to disagree)."""
    from mxllm.serve.engine import SamplingParams

    x = torch.randn(3, 50, generator=torch.Generator().manual_seed(1))
    ids = dops.sample_rows(x, [1.0, 2.0, 0.5], [0.0, -1.0, 1e-9], [0, 0, 0], [1, 2, 3], [0, 0, 0])
    assert ids[0] == x[0].argmax() and ids[1] == x[1].argmax()
    with pytest.raises(ValueError):
        dops.sample_rows(x, [1.0] * 3, [float("nan")] * 3, [0] * 3, [0] * 3, [0] * 3)
    with pytest.raises(ValueError):
        SamplingParams(top_p=-0.5)
    SamplingParams(top_p=0.0)


@pytest.mark.gpu
def test_top_p_zero_is_greedy_gpu(gpu):
    x = torch.randn(4, 128256, device=gpu).bfloat16()
    ids = dops.sample_rows(x, [1.0, 0.7, 1.0, 0.0], [0.0, -2.0, 0.9, 0.5], [0, 0, 0, 0], [1, 2, 3, 4], [0, 0, 0, 0])
    want = x.float().argmax(-1)
    assert ids[0] == want[0] and ids[1] == want[1] and ids[3] == want[3]


@pytest.mark.gpu
def test_concurrent_samplers_on_two_streams(gpu):
    """The vocabulary-split sampler keeps its partials in a per-call workspace: two
    samplers running concurrently on different streams do not corrupt each other."""
    from mxllm.ops import native

    xs = [torch.randn(64, 128256, device=gpu).bfloat16() for _ in range(2)]
    want = [x.float().argmax(-1) for x in xs]
    streams = [torch.cuda.Stream(gpu) for _ in range(2)]
    torch.cuda.synchronize(gpu)
    outs = [[], []]
    for _ in range(20):
        for k in range(2):
            with torch.cuda.stream(streams[k]):
                outs[k].append(native().sample(xs[k], 0.0, 0, 0))
    torch.cuda.synchronize(gpu)
    for k in range(2):
        for o in outs[k]:
            assert torch.equal(o, want[k])
