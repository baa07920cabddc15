"""Llama-3.1 decoder built from mxllm ops (MI355X-first layout).

Design choices:
  * Fused projections: Wqkv = [Wq; Wk; Wv] and Wgu = [Wgate; Wup], so every
    transformer sub-block issues one large hipBLASLt GEMM per projection.
  * Residual adds are fused into the following RMSNorm (``add_rms_norm``),
    including across the layer boundary, so the residual stream is touched
    once per sub-block.
  * The attention segment (split + RoPE + flash attention) is one autograd
    node, the LM head + CE is another (``linear_cross_entropy``).
  * Weights are created directly on the target device in bf16 with a seeded
    RNG — a 70B model initialises on one MI355X in seconds, never on the host.
  * LoRA (``lora_r > 0``): base weights frozen (no weight-gradient GEMMs), one
    adapter per projection split on q, k, v, o, gate, up, down.

Reference parity: the reference repo advertises "fine-tuning of Meta Llama 3.1
70B" (reference README.md:1-3) but contains no model; this module is that model.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.utils.checkpoint as ckpt

from .. import ops
from ..ops import fused
from ..ops import reference as ref
from .config import LlamaConfig


class FusedLinear(nn.Module):
    """y = x @ W^T with W = concat(splits) [sum(splits), in]; optional per-split LoRA.

    With LoRA the frozen W lives inside an augmented buffer
    ``wbuf [N + pad, in + pad] = [[W, B], [A, 0]]`` (``pad`` = n*r rounded up to
    64) so each direction of the projection is ONE hipBLASLt GEMM
    (mxllm/ops/linear.py ``_LoRAAugFn``); ``weight`` is a view of it.  The
    adapter parameters stay ordinary (flat-buffer) parameters for DDP and the
    fused optimizer; ``Llama.sync_adapters_`` copies them into ``wbuf`` after
    every update (one batched HIP copy for the whole model).
    """

    def __init__(self, in_features: int, splits: list[int], *, dtype, device, lora_r: int = 0,
                 lora_alpha: float = 16.0, train_base: bool = True, dx_image: bool = False,
                 transposed: bool = False):
        super().__init__()
        self.in_features = in_features
        self.splits = list(splits)
        N = sum(splits)
        self.lora_r = lora_r
        self.pad = 0
        self.transposed = False
        if lora_r > 0:
            n = len(splits)
            self.scaling = lora_alpha / lora_r
            self.pad = (n * lora_r + 63) // 64 * 64
            # ``transposed``: the augmented buffer is stored as its transpose
            # [[W^T, A^T], [B^T, 0]] [in + pad, N + pad] -> the forward GEMM runs in
            # hipBLASLt's NN form and the input-gradient GEMM in the TN form (the reverse
            # of the row-major layout), with no second copy of W; A is kept as a small
            # k-contiguous copy ``wa`` for the rank-r kernel
            self.transposed = transposed and not train_base
            shape = (in_features + self.pad, N + self.pad) if self.transposed else (N + self.pad, in_features + self.pad)
            self.register_buffer("wbuf", torch.zeros(*shape, dtype=dtype, device=device), persistent=False)
            # B^T [pad, N] (zero rows past n*r): the k-contiguous operand of the
            # backward s dy B kernel (csrc/kernels/lora.hip), refreshed with wbuf
            self.register_buffer("wbt", torch.zeros(self.pad, N, dtype=dtype, device=device), persistent=False)
            if self.transposed:
                self.register_buffer("wa", torch.zeros(self.pad, in_features, dtype=dtype, device=device),
                                     persistent=False)
            # optional [W; A]^T image [in, N + pad]: the input-gradient GEMM then runs in
            # hipBLASLt's reduction-contiguous form (dx = dy_aug @ wxt^T) instead of the
            # ~15-30 % slower NN form; frozen W part refreshed by refresh_images_(), the A^T
            # columns by every adapter sync.  Costs one more copy of W (qkv/o only by default)
            if dx_image and not train_base and not self.transposed:
                self.register_buffer("wxt", torch.zeros(in_features, N + self.pad, dtype=dtype, device=device),
                                     persistent=False)
            w = self.wbuf[:in_features, :N].t() if self.transposed else self.wbuf[:N, :in_features]
            self.weight = nn.Parameter(w, requires_grad=train_base)
            # A: all splits' down-projections stacked; B: block-diagonal up-projection
            self.lora_a = nn.Parameter(torch.empty(n * lora_r, in_features, dtype=dtype, device=device))
            self.lora_b = nn.Parameter(torch.zeros(N, n * lora_r, dtype=dtype, device=device))
        else:
            self.weight = nn.Parameter(torch.empty(N, in_features, dtype=dtype, device=device),
                                       requires_grad=train_base)

    def lora_b_blocks(self):
        """Views of the diagonal blocks B_i [n_i, r] of the block-diagonal B."""
        out, off = [], 0
        for i, n_i in enumerate(self.splits):
            out.append(self.lora_b[off:off + n_i, i * self.lora_r:(i + 1) * self.lora_r])
            off += n_i
        return out

    def augmented(self) -> bool:
        """True while ``weight`` still aliases ``wbuf`` (module not moved / merged)."""
        return (self.lora_r > 0 and hasattr(self, "wbuf")
                and self.weight.data_ptr() == self.wbuf.data_ptr() and self.weight.dtype == self.wbuf.dtype)

    def adapter_copies(self):
        """(src, dst) pairs: adapter parameters -> their slots in ``wbuf``."""
        N, K, R = sum(self.splits), self.in_features, self.lora_a.shape[0]
        if self.transposed:
            return [(self.lora_a.data, self.wbuf[:K, N:N + R].t()), (self.lora_b.data, self.wbuf[K:K + R, :N].t()),
                    (self.lora_b.data, self.wbt[:R, :N].t()), (self.lora_a.data, self.wa[:R, :K])]
        out = [(self.lora_a.data, self.wbuf[N:N + R, :K]), (self.lora_b.data, self.wbuf[:N, K:K + R]),
               (self.lora_b.data, self.wbt[:R, :N].t())]
        if getattr(self, "wxt", None) is not None:
            out.append((self.lora_a.data, self.wxt[:, N:N + R].t()))
        return out

    @torch.no_grad()
    def refresh_images_(self):
        """Rebuild the transposed [W; A] image after the frozen weight changed
        (init, checkpoint load)."""
        if getattr(self, "wxt", None) is not None and self.augmented():
            K = self.in_features
            self.wxt.copy_(ops.transpose2d(self.wbuf[:, :K]))

    @torch.no_grad()
    def sync_adapter_(self):
        for src, dst in self.adapter_copies():
            dst.copy_(src)

    @torch.no_grad()
    def reset_parameters(self, std: float, gen: torch.Generator | None):
        self.weight.normal_(0.0, std, generator=gen)
        if self.lora_r > 0:
            bound = 1.0 / math.sqrt(self.in_features)
            self.lora_a.uniform_(-bound, bound, generator=gen)
            self.lora_b.zero_()
            if self.augmented():
                self.sync_adapter_()
                self.refresh_images_()

    def tail_operands(self):
        """((A rows [pad, in], R, s), (B^T rows [pad, N], R, s)): the k-contiguous operands of the
        forward / backward rank-r tails, for producers that write them (fused SwiGLU)."""
        R = self.lora_a.shape[0]
        amat = self.wa if self.transposed else self.wbuf[sum(self.splits):, :self.in_features]
        return (amat, R, self.scaling), (self.wbt, R, self.scaling)

    def forward(self, x: torch.Tensor, x_tail: bool = False, dy_tail: bool = False) -> torch.Tensor:
        if self.lora_r > 0:
            if self.augmented():
                return ops.lora_linear_aug(x, self.lora_a, self.lora_b, self.wbuf, self.splits, self.scaling,
                                           self.pad, self.wbt, getattr(self, "wxt", None),
                                           getattr(self, "wa", None) if self.transposed else None,
                                           x_tail=x_tail, dy_tail=dy_tail)
            return ops.lora_linear(x, self.weight, self.lora_a, self.lora_b, self.splits, self.scaling)
        return ops.linear(x, self.weight)


# LoRA projections that keep a transposed [W; A] image for the input-gradient GEMM
# (FusedLinear.wxt): hipBLASLt's TN form instead of the ~15 % slower NN form, for one more
# copy of W.  Measured 70B LoRA step, same box (archive/profiles/r2n_dx_image_ab.md): qkv,o 1001.3 ms
# (267.4 GB reserved) / qkv,d 990.8 ms (294.3 GB) / qkv,o,d 985.5 ms (305.3 GB of 309: too
# little headroom for multi-GPU runs).  Default qkv + d.
DX_IMAGE = tuple(x for x in os.environ.get("MXLLM_DX_IMAGE", "qkv,d").split(",") if x)
# LoRA projections whose augmented buffer is stored transposed (FusedLinear ``transposed``):
# forward GEMM in the NN form, input gradient in the TN form, same memory
LORA_T = tuple(x for x in os.environ.get("MXLLM_LORA_T", "").split(",") if x)
# full fine-tuning, selective checkpointing: recompute m = swiglu(gu) in the backward of the
# un-checkpointed layers instead of saving it (Llama._recompute_m)
RECOMPUTE_SWIGLU = os.environ.get("MXLLM_RECOMPUTE_SWIGLU", "auto")
# same layers: the normed inputs of the qkv and gate-up projections are recomputed from the
# residual stream in their backward instead of saved (ops.normed_linear); 0 = save them
RECOMPUTE_NORM = os.environ.get("MXLLM_RECOMPUTE_NORM", "auto")
# those layers' MLP through the fused gate-up + SwiGLU epilogue (m rebuilt by the dm GEMM's epilogue
# in the backward) instead of GEMM + a standalone SwiGLU pass; 0 = the unfused recompute (A/B)
REC_FUSED = os.environ.get("MXLLM_REC_FUSED", "1") != "0"


class LlamaLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, *, dtype, device, lora_r: int, lora_alpha: float, train_base: bool):
        super().__init__()
        kw = dict(dtype=dtype, device=device, lora_r=lora_r, lora_alpha=lora_alpha, train_base=train_base)
        h = cfg.hidden
        self.attn_norm = nn.Parameter(torch.ones(h, dtype=dtype, device=device), requires_grad=train_base)
        self.mlp_norm = nn.Parameter(torch.ones(h, dtype=dtype, device=device), requires_grad=train_base)
        self.wqkv = FusedLinear(h, [cfg.q_dim, cfg.kv_dim, cfg.kv_dim], dx_image="qkv" in DX_IMAGE,
                                transposed="qkv" in LORA_T, **kw)
        self.wo = FusedLinear(cfg.q_dim, [h], dx_image="o" in DX_IMAGE, transposed="o" in LORA_T, **kw)
        self.wgu = FusedLinear(h, [cfg.ffn, cfg.ffn], dx_image="gu" in DX_IMAGE, transposed="gu" in LORA_T, **kw)
        self.wd = FusedLinear(cfg.ffn, [h], dx_image="d" in DX_IMAGE, transposed="d" in LORA_T, **kw)


def ckpt_layer(setting: bool | int | None, i: int) -> bool:
    """Whether layer ``i`` is activation-checkpointed: ``True`` = every layer, an int
    ``n`` = the first ``n`` layers (selective checkpointing: the rest keep their
    activations, trading HBM for the recompute), ``False``/``0``/``None`` = none."""
    if isinstance(setting, bool) or setting is None:
        return bool(setting)
    return i < int(setting)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig, *, device=None, dtype=torch.bfloat16, lora_r: int = 0,
                 lora_alpha: float = 16.0, seed: int = 0, init: bool = True,
                 activation_checkpointing: bool | int = False):
        super().__init__()
        device = torch.device(device) if device is not None else torch.device("cpu")
        self.cfg = cfg
        self.lora = lora_r > 0
        train_base = not self.lora
        self.activation_checkpointing = activation_checkpointing
        self.mlp_recompute_ckpt = None  # checkpoint spec of a trainer that runs _layer itself (ZeRO-3)
        self.seq_parallel = None  # UlyssesAttention when the sequence is sharded (set_sequence_parallel)
        # optional ``fn(params)`` called before the parameters are first used in a forward (ZeRO-1: wait for
        # their all-gather; mxllm/parallel/zero1.py) — None = parameters are always resident
        self.param_wait = None
        self.tok_emb = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden, dtype=dtype, device=device),
                                    requires_grad=train_base)
        self.layers = nn.ModuleList([
            LlamaLayer(cfg, dtype=dtype, device=device, lora_r=lora_r, lora_alpha=lora_alpha, train_base=train_base)
            for _ in range(cfg.n_layers)])
        self.final_norm = nn.Parameter(torch.ones(cfg.hidden, dtype=dtype, device=device), requires_grad=train_base)
        if cfg.tie_embeddings:
            self.lm_head = None
            self.tok_emb._mx_no_direct = True  # two uses (embedding + head): gradient via autograd
        else:
            self.lm_head = nn.Parameter(torch.empty(cfg.vocab_size, cfg.hidden, dtype=dtype, device=device),
                                        requires_grad=train_base)
        cos, sin = ref.rope_tables(min(cfg.max_seq_len, 131072), cfg.head_dim, cfg.rope_theta, cfg.rope_scaling)
        self.register_buffer("rope_cos", cos.to(device), persistent=False)
        self.register_buffer("rope_sin", sin.to(device), persistent=False)
        if init:
            self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed: int = 0):
        dev = self.tok_emb.device
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        std = 0.02
        self.tok_emb.normal_(0.0, std, generator=gen)
        for layer in self.layers:
            for lin in (layer.wqkv, layer.wo, layer.wgu, layer.wd):
                lin.reset_parameters(std, gen)
        if self.lm_head is not None:
            self.lm_head.normal_(0.0, std, generator=gen)

    @property
    def head_weight(self) -> torch.Tensor:
        return self.tok_emb if self.lm_head is None else self.lm_head

    # ------------------------------------------------------------------ training forward
    @staticmethod
    def _pad(lin) -> int:
        """Row padding a producer leaves for a LoRA projection's rank columns."""
        return lin.pad if lin.augmented() else 0

    def _layer(self, i: int, x: torch.Tensor, h: torch.Tensor, B: int, S: int):
        cfg = self.cfg
        layer = self.layers[i]
        rec = self._recompute_m(layer, i)
        rec_x = rec and RECOMPUTE_NORM != "0"
        lora_at = (ops.lora_qkv_attention_at(x, layer.wqkv, B, S, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim)
                   if self.seq_parallel is None and layer.wqkv.lora_r and not rec_x else 0)
        if (self.seq_parallel is None and not layer.wqkv.lora_r
                and fused.qkv_attention_ok(x, layer.wqkv.weight, B, S, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim)):
            # projection + RoPE + head split in ONE GEMM epilogue (mxllm/ops/fused.py)
            o = fused.qkv_attention(x, layer.wqkv.weight, self.rope_cos, self.rope_sin, B, S, cfg.n_heads,
                                    cfg.n_kv_heads, cfg.head_dim, causal=True, out_pad=self._pad(layer.wo),
                                    norm=(h, layer.attn_norm, cfg.norm_eps) if rec_x else None)
            qkv = None
        elif lora_at:
            # LoRA: the augmented projection with RoPE + head split in its tail-balanced GEMM
            # (mxllm/ops/linear.py lora_qkv_attention): no qkv activation, no rope_split pass
            o = ops.lora_qkv_attention(x, layer.wqkv, self.rope_cos, self.rope_sin, B, S, cfg.n_heads,
                                       cfg.n_kv_heads, cfg.head_dim, lora_at, causal=True, out_pad=self._pad(layer.wo))
            qkv = None
        else:
            qkv = (ops.normed_linear(x, h, layer.attn_norm, cfg.norm_eps, layer.wqkv.weight) if rec_x
                   else layer.wqkv(x))
        if qkv is None:
            pass
        elif self.seq_parallel is not None:
            o = self.seq_parallel(qkv, self.rope_cos, self.rope_sin, B, S, cfg.n_heads, cfg.n_kv_heads,
                                  cfg.head_dim, causal=True)
        else:
            o = ops.attention_block(qkv, self.rope_cos, self.rope_sin, B, S, cfg.n_heads, cfg.n_kv_heads,
                                    cfg.head_dim, causal=True, out_pad=self._pad(layer.wo),
                                    grad_pad=self._pad(layer.wqkv))
        a = layer.wo(o)
        x, h = ops.add_rms_norm(a, h, layer.mlp_norm, cfg.norm_eps, out_pad=self._pad(layer.wgu),
                                grad_pad=self._pad(layer.wo))
        if rec and REC_FUSED and fused.gate_up_swiglu_down_ok(x, layer.wgu.weight, layer.wd.weight):
            # the same recompute (only gu, and h for x, kept) with the SwiGLU in the gate-up GEMM's
            # epilogue and m rebuilt by the backward's dm GEMM epilogue: no standalone SwiGLU pass
            d = fused.gate_up_swiglu_down(x, layer.wgu.weight, layer.wd.weight,
                                          norm=(h, layer.mlp_norm, cfg.norm_eps) if rec_x else None, recompute_m=True)
        elif rec:  # m = swiglu(gu) (and the gate-up input x) recomputed in the backward
            gu = ops.normed_linear(x, h, layer.mlp_norm, cfg.norm_eps, layer.wgu.weight) if rec_x else layer.wgu(x)
            d = ops.swiglu_linear(gu, layer.wd.weight)
        elif (not layer.wgu.lora_r and not layer.wd.lora_r
              and fused.gate_up_swiglu_down_ok(x, layer.wgu.weight, layer.wd.weight)):
            # gate-up + SwiGLU + down: the backward's dm GEMM writes dgu (mxllm/ops/fused.py)
            d = fused.gate_up_swiglu_down(x, layer.wgu.weight, layer.wd.weight)
        elif not layer.wgu.lora_r and fused.gate_up_swiglu_ok(x, layer.wgu.weight):
            # gate-up projection with SwiGLU in its epilogue (mxllm/ops/fused.py)
            m = fused.gate_up_swiglu(x, layer.wgu.weight, out_pad=self._pad(layer.wd))
            d = layer.wd(m)
        else:
            tf, tb = self._swiglu_tails(layer, x)
            m = ops.swiglu(layer.wgu(x, dy_tail=tb is not None), out_pad=self._pad(layer.wd),
                           grad_pad=self._pad(layer.wgu), tail_fwd=tf, tail_bwd=tb)
            d = layer.wd(m, x_tail=tf is not None)
        last = i + 1 == len(self.layers)
        nxt = self.final_norm if last else self.layers[i + 1].attn_norm
        x, h = ops.add_rms_norm(d, h, nxt, cfg.norm_eps, out_pad=0 if last else self._pad(self.layers[i + 1].wqkv),
                                grad_pad=self._pad(layer.wd))
        return x, h

    def _recompute_m(self, layer, i: int) -> bool:
        """Recompute the MLP activation m = swiglu(gu) (and, unless ``MXLLM_RECOMPUTE_NORM`` = 0,
        the normed qkv / gate-up inputs) in the backward instead of saving them, in the
        un-checkpointed layers of a selectively checkpointed run -- including one that checkpoints
        0 layers (memory-bound by design: the saved HBM buys more un-checkpointed layers;
        ``MXLLM_RECOMPUTE_SWIGLU`` 0 / 1 / auto)."""
        if (RECOMPUTE_SWIGLU == "0" or any(lin.lora_r > 0 for lin in (layer.wqkv, layer.wgu, layer.wd))
                or not self.training or not torch.is_grad_enabled()):
            return False
        if RECOMPUTE_SWIGLU == "1":
            return True
        ck = self.mlp_recompute_ckpt if self.mlp_recompute_ckpt is not None else self.activation_checkpointing
        return not isinstance(ck, bool) and ck is not None and not ckpt_layer(ck, i)

    def _swiglu_tails(self, layer, x: torch.Tensor):
        """LoRA tails the SwiGLU pass writes itself: the down projection's s m A^T (forward)
        and the gate-up projection's s dgu B (backward) -- None where the fused kernel does
        not take the shape (mxllm/ops/activation.py)."""
        if x.dim() != 2:
            return None, None
        T, F2 = x.shape[0], 2 * self.cfg.ffn
        tf = tb = None
        if layer.wd.augmented() and ops.lora_tail_ok(x, T, F2, layer.wd.pad, layer.wd.lora_a.shape[0]):
            tf = layer.wd.tail_operands()[0]
        if layer.wgu.augmented() and ops.lora_tail_ok(x, T, F2, layer.wgu.pad, layer.wgu.lora_a.shape[0]):
            tb = layer.wgu.tail_operands()[1]
        return tf, tb

    def _wait_groups(self):
        """Parameter groups in first-use order: embedding (+ first norm), layer i
        (+ the next layer's attn_norm it applies), head (+ final norm)."""
        if getattr(self, "_wgroups", None) is None:
            L = len(self.layers)
            g = [[self.tok_emb] + ([self.layers[0].attn_norm] if L else [])]
            for i, layer in enumerate(self.layers):
                nxt = self.final_norm if i + 1 == L else self.layers[i + 1].attn_norm
                g.append(list(layer.parameters()) + [nxt])
            g.append([self.final_norm] + ([self.lm_head] if self.lm_head is not None else []))
            self._wgroups = g
        return self._wgroups

    def hidden_states(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, S] -> final normed hidden [B*S, H]."""
        B, S = ids.shape
        wait = self.param_wait
        groups = self._wait_groups() if wait is not None else None
        if wait is not None:
            wait(groups[0])
        h = ops.embedding(ids.reshape(-1), self.tok_emb)
        x = (ops.rms_norm(h, self.layers[0].attn_norm, self.cfg.norm_eps, out_pad=self._pad(self.layers[0].wqkv))
             if len(self.layers) else h)
        for i in range(len(self.layers)):
            if wait is not None:
                wait(groups[i + 1])
            if ckpt_layer(self.activation_checkpointing, i) and self.training and torch.is_grad_enabled():
                x, h = ckpt.checkpoint(self._layer, i, x, h, B, S, use_reentrant=False)
            else:
                x, h = self._layer(i, x, h, B, S)
        if not len(self.layers):
            x = ops.rms_norm(h, self.final_norm, self.cfg.norm_eps)
        if wait is not None:
            wait(groups[-1])
        return x

    def forward(self, ids: torch.Tensor, labels: torch.Tensor | None = None, ignore_index: int = -100):
        """Training/eval forward.  With labels: mean token CE (fused head+CE).
        Without: logits [B, S, V] (bf16)."""
        B, S = ids.shape
        x = self.hidden_states(ids)
        if labels is not None:
            return ops.linear_cross_entropy(x, self.head_weight, labels.reshape(-1), ignore_index)
        return torch.matmul(x, self.head_weight.t()).view(B, S, -1)

    @torch.no_grad()
    def sync_adapters_(self) -> None:
        """Copy every LoRA adapter into its augmented GEMM buffer (after an
        optimizer step / checkpoint load / broadcast).  GPU: ONE batched HIP
        copy (csrc/kernels/misc.hip ``copy2d_batched``) for all projections."""
        lins = [m for m in self.modules() if isinstance(m, FusedLinear) and m.augmented()]
        if not lins:
            return
        pairs = [p for m in lins for p in m.adapter_copies()]
        if not pairs[0][0].is_cuda or not ops.native_available():
            for src, dst in pairs:
                dst.copy_(src)
            return
        key = tuple((s.data_ptr(), d.data_ptr()) for s, d in pairs)
        if getattr(self, "_adapter_desc_key", None) != key:
            from ..ops.linear import copy2d_plan

            rows, total = copy2d_plan(pairs)
            self._adapter_desc = torch.tensor(rows, dtype=torch.int64, device=pairs[0][0].device)
            self._adapter_blocks = total
            self._adapter_desc_key = key
        ops.native().copy2d_batched(self._adapter_desc, self._adapter_blocks)

    @torch.no_grad()
    def refresh_images_(self) -> None:
        """Rebuild derived weight images (transposed [W; A] of the LoRA
        projections) after the frozen base weights were written."""
        for m in self.modules():
            if isinstance(m, FusedLinear):
                m.refresh_images_()

    def set_sequence_parallel(self, group) -> None:
        """Shard sequences over ``group`` (Ulysses all-to-all around attention,
        mxllm/parallel/sequence.py); ``None`` turns it off.  Inputs passed to
        forward are then this rank's [B, S/P] token slice."""
        if group is None:
            self.seq_parallel = None
            return
        from ..parallel.sequence import UlyssesAttention

        self.seq_parallel = UlyssesAttention(group)

    def set_context_parallel(self, group) -> None:
        """Shard sequences over ``group`` in the zigzag layout (ring attention,
        mxllm/parallel/context.py); ``None`` turns it off.  Inputs passed to
        forward are then this rank's [B, S/P] zigzag tokens (``zigzag_shard``)."""
        if group is None:
            self.seq_parallel = None
            return
        from ..parallel.context import RingAttention

        self.seq_parallel = RingAttention(group)

    # ------------------------------------------------------------------ utilities
    def trainable_parameters(self):
        return [p for p in self.parameters() if p.requires_grad]

    def named_trainable_parameters(self):
        return [(n, p) for n, p in self.named_parameters() if p.requires_grad]

    def num_params(self, trainable_only: bool = False) -> int:
        return sum(p.numel() for p in (self.trainable_parameters() if trainable_only else self.parameters()))
