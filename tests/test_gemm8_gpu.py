"""8-phase MFMA GEMM (csrc/kernels/gemm8.hip) vs a plain-PyTorch fp32 reference.

All four operand orders (k- / mn-contiguous A and B), bf16 and fp32 output, beta 0 / 1, a
device-scalar alpha, padded row strides, odd K-tile counts and (for the weight-gradient form,
both operands token-major) token counts that are not a multiple of the 64-token K-tile: the
rows past K read as zeros through the range-checked descriptors.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from mxllm.ops import native

    return native()


def _mat(rows, cols, dev, pad=0, seed=0):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    buf = (torch.rand(rows, cols + pad, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    return buf[:, :cols]


def _check(got, ref, tol):
    err = ((got.float() - ref).norm() / ref.norm()).item()
    assert err < tol, err


@pytest.mark.parametrize("ph", ["8", "4"])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 640), (768, 512, 192)])
def test_gemm8_orders(gpu, a_kc, b_kc, M, N, K, ph, monkeypatch):
    monkeypatch.setenv("MXLLM_GEMM8_PH", ph)  # 8-phase (default) and 4-phase schedules
    a = _mat(M, K, gpu, pad=8, seed=1) if a_kc else _mat(K, M, gpu, pad=16, seed=1)
    b = _mat(N, K, gpu, pad=24, seed=2) if b_kc else _mat(K, N, gpu, pad=8, seed=2)
    A = a.float() if a_kc else a.float().t()
    B = b.float().t() if b_kc else b.float()
    ref = A @ B
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(a, a_kc, b, b_kc, out, 0.0, None, 1.0)
    _check(out, ref, 5e-3)
    out32 = torch.empty(M, N, device=gpu, dtype=torch.float32)
    assert _ops().gemm8(a, a_kc, b, b_kc, out32, 0.0, None, 1.0)
    _check(out32, ref, 1e-5)


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 1000), (1024, 4096, 4096)])
def test_gemm8_sq_partials(gpu, a_kc, b_kc, M, N, K):
    """gemm8_sq: the output is bitwise the 4-phase gemm8's, and sq holds one fp32 sum of squares of
    the stored bf16 values per 256 x 256 tile (row-major tile order), device alpha included."""
    if (a_kc or b_kc) and K % 64:
        K = 1024
    a = _mat(M, K, gpu, pad=8, seed=6) if a_kc else _mat(K, M, gpu, pad=16, seed=6)
    b = _mat(N, K, gpu, pad=24, seed=7) if b_kc else _mat(K, N, gpu, pad=8, seed=7)
    alpha = torch.tensor([0.61], device=gpu)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    sq = torch.full(((M // 256) * (N // 256) + 3,), -1.0, device=gpu)
    assert _ops().gemm8_sq(a, a_kc, b, b_kc, out, sq, alpha, 1.0)
    ref = torch.empty_like(out)
    assert _ops().gemm8(a, a_kc, b, b_kc, ref, 0.0, alpha, 1.0, 4)
    assert torch.equal(out, ref)
    want = out.float().pow(2).view(M // 256, 256, N // 256, 256).sum(dim=(1, 3)).flatten()
    got = sq[:want.numel()]
    assert torch.allclose(got, want, rtol=1e-5, atol=0), (got - want).abs().max().item()
    assert (sq[want.numel():] == -1.0).all()  # nothing past the tiles
    b2 = _mat(128, K, gpu, seed=8) if b_kc else _mat(K, 128, gpu, seed=8)
    out2 = torch.empty(M, 128, device=gpu, dtype=torch.bfloat16)
    assert not _ops().gemm8_sq(a, a_kc, b2, b_kc, out2, sq, None, 1.0)  # N % 256: declined


@pytest.mark.parametrize("f32", [True, False])
def test_gemm8_beta_alpha(gpu, f32):
    M, N, K = 512, 1024, 384
    a, b = _mat(K, M, gpu, seed=3), _mat(K, N, gpu, seed=4)  # token-major dW form
    c0 = _mat(M, N, gpu, pad=8, seed=5).to(torch.float32 if f32 else torch.bfloat16)
    out = c0.clone()
    alpha = torch.tensor([0.37], device=gpu)
    assert _ops().gemm8(a, False, b, False, out, 1.0, alpha, 2.0)
    ref = c0.float() + 0.74 * (a.float().t() @ b.float())
    _check(out, ref, 1e-5 if f32 else 5e-3)


@pytest.mark.parametrize("ph", ["8", "4"])
@pytest.mark.parametrize("T", [1, 63, 100, 1000, 4097])
def test_gemm8_weight_grad_odd_tokens(gpu, T, ph, monkeypatch):
    monkeypatch.setenv("MXLLM_GEMM8_PH", ph)
    M, N = 256, 512
    dy, x = _mat(T, M, gpu, pad=8, seed=6), _mat(T, N, gpu, pad=8, seed=7)
    out = torch.full((M, N), float("nan"), device=gpu, dtype=torch.float32)  # beta 0 must ignore it
    assert _ops().gemm8(dy, False, x, False, out, 0.0, None, 1.0)
    _check(out, dy.float().t() @ x.float(), 1e-5)


@pytest.mark.parametrize("ph", ["8", "4"])
def test_gemm8_odd_ktiles_nn(gpu, ph, monkeypatch):
    """the LoRA-augmented dX shape: K = N_out + 64 (an odd number of 64-deep K-tiles)."""
    monkeypatch.setenv("MXLLM_GEMM8_PH", ph)
    T, N, K = 512, 1024, 1024 + 64
    dya = _mat(T, K, gpu, seed=8)
    w = _mat(K, N, gpu, pad=64, seed=9)
    out = torch.empty(T, N, device=gpu, dtype=torch.bfloat16)
    assert _ops().gemm8(dya, True, w, False, out, 0.0, None, 1.0)
    _check(out, dya.float() @ w.float(), 5e-3)


def test_gemm8_declines_unsupported(gpu):
    a, b = _mat(100, 64, gpu), _mat(256, 64, gpu)
    out = torch.empty(100, 256, device=gpu, dtype=torch.bfloat16)
    assert not _ops().gemm8(a, True, b, True, out, 0.0, None, 1.0)  # M not a multiple of 256
    a2 = _mat(256, 100, gpu)
    out2 = torch.empty(256, 256, device=gpu, dtype=torch.bfloat16)
    assert not _ops().gemm8(a2, True, _mat(256, 100, gpu), True, out2, 0.0, None, 1.0)  # k-contig K % 64


def test_gemm8_identity_asymmetric(gpu):
    """A = I with an asymmetric B catches a transposed store (guide §3)."""
    n = 256
    a = torch.eye(n, device=gpu, dtype=torch.bfloat16)
    b = (torch.arange(n, device=gpu).view(n, 1) * 3 + torch.arange(n, device=gpu).view(1, n) * 0.5 - 300) / 64
    b = b.to(torch.bfloat16)
    out = torch.empty(n, n, device=gpu, dtype=torch.float32)
    assert _ops().gemm8(a, True, b, False, out, 0.0, None, 1.0)
    assert torch.equal(out, b.float())


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,n1,K", [(256, 512, 256, 640), (512, 1280, 768, 8256), (4096, 10240, 8192, 8256)])
def test_gemm8_tail_split(gpu, a_kc, b_kc, M, N, n1, K):
    """Tail-balanced launch (mx_gemm8_tail): columns [0, n1) plain, the rest as two half-K launches
    summed through fp32 images (odd K-tile counts split 64 / 65 ...): equals the fp32 reference and
    is bit-reproducible."""
    a = _mat(M, K, gpu, pad=8, seed=11) if a_kc else _mat(K, M, gpu, pad=8, seed=11)
    b = _mat(N, K, gpu, pad=8, seed=12) if b_kc else _mat(K, N, gpu, pad=8, seed=12)
    A = a.float() if a_kc else a.float().t()
    B = b.float().t() if b_kc else b.float()
    ref = A @ B
    out = torch.empty(M, N + 16, device=gpu, dtype=torch.bfloat16)[:, :N]
    assert _ops().gemm8_tail(a, a_kc, b, b_kc, out, n1, False, 4)
    _check(out, ref, 5e-3)
    _check(out[:, n1:], ref[:, n1:], 5e-3)
    again = torch.empty_like(out)
    assert _ops().gemm8_tail(a, a_kc, b, b_kc, again, n1, False, 4)
    assert torch.equal(again, out)
    # the same split along rows (M1 = n1 rows when M allows it)
    if M > 256:
        m1 = 256
        rows_out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        assert _ops().gemm8_tail(a, a_kc, b, b_kc, rows_out, m1, True, 4)
        _check(rows_out, ref, 5e-3)
        _check(rows_out[m1:], ref[m1:], 5e-3)


def _tile_sq(x):
    M, N = x.shape
    return x.float().pow(2).view(M // 256, 256, N // 256, 256).sum(dim=(1, 3)).flatten()


@pytest.mark.parametrize("rows", [False, True])
def test_gemm8_tail_sq_partials(gpu, rows):
    """The tail-balanced launch with clip-norm partials: output bitwise the plain tail launch's, one
    sum of squares per tile -- the plain part's tiles (row-major), then the split part's."""
    M, N, K, at = (768, 512, 1024, 512) if rows else (512, 1280, 8256, 768)
    a = _mat(K, M, gpu, seed=11)  # token-major dW form (both operands mn-contiguous)
    b = _mat(K, N, gpu, seed=12)
    out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    sq = torch.full(((M // 256) * (N // 256),), -1.0, device=gpu)
    assert _ops().gemm8_tail(a, False, b, False, out, at, rows, 4, sq)
    ref = torch.empty_like(out)
    assert _ops().gemm8_tail(a, False, b, False, ref, at, rows, 4)
    assert torch.equal(out, ref)
    parts = (out[:at], out[at:]) if rows else (out[:, :at], out[:, at:])
    want = torch.cat([_tile_sq(p.contiguous()) for p in parts])
    assert torch.allclose(sq, want, rtol=1e-5, atol=0), (sq - want).abs().max().item()


def test_gemm_dispatch_uses_tail_entry(gpu, monkeypatch):
    """A win-table entry with ``tail`` routes the forward GEMM through the tail-balanced launch."""
    from mxllm.ops import gemm

    M, N, K = 4096, 10240, 1024
    key = ("tn", M, N, K, "bf16")
    monkeypatch.setitem(gemm._table(), key, 4)
    assert gemm.tail_split(M, N, K) == 8192
    monkeypatch.setitem(gemm._TAIL, key, gemm.tail_split(M, N, K))
    calls = []
    real = _ops()

    class Spy:
        def __getattr__(self, k):
            if k == "gemm8_tail":
                calls.append(k)
            return getattr(real, k)

    monkeypatch.setattr(gemm, "native", lambda: Spy())
    x, w = _mat(M, K, gpu, seed=13), _mat(N, K, gpu, seed=14)
    y = gemm.mm("tn", x, w)
    assert calls == ["gemm8_tail"]
    _check(y, x.float() @ w.float().t(), 5e-3)


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("f32,beta", [(False, 0.0), (True, 0.0), (True, 1.0), (False, 1.0)])
def test_gemm8_persistent_bitwise(gpu, a_kc, b_kc, f32, beta, monkeypatch):
    """Persistent tile-looping kernel (MXLLM_GEMM8_PERSIST=1): more tiles than
    CUs (each workgroup walks several, next tile's DMA issued under the previous epilogue), odd
    K-tile counts -- bitwise equal to the one-tile-per-workgroup kernel (same K order per tile)
    and to the fp32 reference."""
    M, N, K = 4096, 4352, 704 if (a_kc or b_kc) else 700  # 16 x 17 = 272 tiles; 11 K-tiles
    a = _mat(M, K, gpu, pad=8, seed=21) if a_kc else _mat(K, M, gpu, pad=8, seed=21)
    b = _mat(N, K, gpu, pad=8, seed=22) if b_kc else _mat(K, N, gpu, pad=8, seed=22)
    A = a.float() if a_kc else a.float().t()
    B = b.float().t() if b_kc else b.float()
    dt = torch.float32 if f32 else torch.bfloat16
    c0 = _mat(M, N, gpu, seed=23).to(dt)
    outs = {}
    for p in ("0", "1"):
        monkeypatch.setenv("MXLLM_GEMM8_PERSIST", p)
        out = c0.clone()
        assert _ops().gemm8(a, a_kc, b, b_kc, out, beta, None, 1.0, 4)
        outs[p] = out
    assert torch.equal(outs["0"], outs["1"])
    ref = A @ B + (c0.float() if beta else 0.0)
    _check(outs["1"], ref, 1e-5 if f32 else 5e-3)
