"""Hugging Face Llama checkpoints <-> mxllm (``config.json`` + safetensors shards).

A user of the reference calls a remote model through LiteLLM; moving to a local
model means bringing a Hugging Face Llama-3.x directory (reference
src/distributed_inference.py:37 names the model, config.py:37 the MODEL_NAME).
``load_hf_llama`` builds the mxllm model from such a directory and
``save_hf_llama`` writes a (fine-tuned) model back in the same layout, LoRA
merged into the projections (W + s B A), for any HF-compatible tool.

mxllm's RoPE kernels use the rotate-half pairing (i, i + D/2) that HF Llama
checkpoints are stored for, so q / k need no permutation.  Name mapping:

  model.embed_tokens.weight                      -> tok_emb
  model.layers.i.input_layernorm.weight          -> layers.i.attn_norm
  model.layers.i.post_attention_layernorm.weight -> layers.i.mlp_norm
  model.layers.i.self_attn.{q,k,v}_proj.weight   -> layers.i.wqkv.weight rows [q | k | v]
  model.layers.i.self_attn.o_proj.weight         -> layers.i.wo.weight
  model.layers.i.mlp.{gate,up}_proj.weight       -> layers.i.wgu.weight rows [gate | up]
  model.layers.i.mlp.down_proj.weight            -> layers.i.wd.weight
  model.norm.weight                              -> final_norm
  lm_head.weight                                 -> lm_head (absent when the embedding is tied)

Shards are read one tensor at a time through safetensors' memory map and copied
straight into the (device-resident) parameter, so host memory stays at one
tensor even for the 70B model.
"""
from __future__ import annotations

import json
import math
import os

import torch

from .config import LlamaConfig


def is_hf_dir(path: str | None) -> bool:
    return bool(path) and os.path.isdir(path) and os.path.exists(os.path.join(path, "config.json"))


def config_from_hf(hf: dict, name: str = "hf") -> LlamaConfig:
    """LlamaConfig from a Hugging Face ``LlamaForCausalLM`` config.json dict."""
    if hf.get("model_type", "llama") != "llama":
        raise ValueError(f"only Llama checkpoints are supported (model_type={hf.get('model_type')!r})")
    heads = hf["num_attention_heads"]
    # RoPE: transformers < 5 writes rope_theta / rope_scaling, >= 5 one rope_parameters dict
    rp = hf.get("rope_parameters") or {}
    theta = hf.get("rope_theta", rp.get("rope_theta", 10000.0))
    rs = hf.get("rope_scaling")
    if rs is None and rp.get("rope_type", "default") not in ("default", None):
        rs = rp
    if rs:
        kind = rs.get("rope_type", rs.get("type"))
        if kind != "llama3":
            raise ValueError(f"rope_scaling type {kind!r} is not supported (llama3 only)")
        rs = {k: rs[k] for k in ("factor", "low_freq_factor", "high_freq_factor", "original_max_position_embeddings")}
    bos = hf.get("bos_token_id", 128000)
    eos = hf.get("eos_token_id", 128001)
    if isinstance(eos, (list, tuple)):
        eos = eos[0]
    return LlamaConfig(
        name=name, vocab_size=hf["vocab_size"], hidden=hf["hidden_size"], n_layers=hf["num_hidden_layers"],
        n_heads=heads, n_kv_heads=hf.get("num_key_value_heads", heads), ffn=hf["intermediate_size"],
        head_dim=hf.get("head_dim") or hf["hidden_size"] // heads, rope_theta=float(theta),
        rope_scaling=rs, norm_eps=float(hf.get("rms_norm_eps", 1e-5)),
        max_seq_len=int(hf.get("max_position_embeddings", 8192)),
        tie_embeddings=bool(hf.get("tie_word_embeddings", False)), bos_id=bos if bos is not None else 128000,
        eos_id=eos if eos is not None else 128001)


def config_to_hf(cfg: LlamaConfig, dtype: torch.dtype = torch.bfloat16) -> dict:
    out = {
        "architectures": ["LlamaForCausalLM"], "model_type": "llama", "vocab_size": cfg.vocab_size,
        "hidden_size": cfg.hidden, "intermediate_size": cfg.ffn, "num_hidden_layers": cfg.n_layers,
        "num_attention_heads": cfg.n_heads, "num_key_value_heads": cfg.n_kv_heads, "head_dim": cfg.head_dim,
        "hidden_act": "silu", "max_position_embeddings": cfg.max_seq_len, "rms_norm_eps": cfg.norm_eps,
        "rope_theta": cfg.rope_theta, "tie_word_embeddings": cfg.tie_embeddings, "bos_token_id": cfg.bos_id,
        "eos_token_id": cfg.eos_id, "attention_bias": False, "mlp_bias": False,
        "torch_dtype": str(dtype).replace("torch.", ""),
    }
    # both spellings (transformers < 5 reads rope_theta / rope_scaling, >= 5 rope_parameters)
    out["rope_parameters"] = {"rope_type": "default", "rope_theta": cfg.rope_theta}
    if cfg.rope_scaling:
        out["rope_scaling"] = dict(cfg.rope_scaling, rope_type="llama3")
        out["rope_parameters"] = dict(cfg.rope_scaling, rope_type="llama3", rope_theta=cfg.rope_theta)
    return out


def load_hf_config(path: str) -> LlamaConfig:
    with open(os.path.join(path, "config.json")) as f:
        return config_from_hf(json.load(f), name=os.path.basename(os.path.normpath(path)))


def _shard_files(path: str) -> list[str]:
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        return [os.path.join(path, x) for x in files]
    files = sorted(x for x in os.listdir(path) if x.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    return [os.path.join(path, x) for x in files]


def mx_to_hf(cfg: LlamaConfig) -> dict[str, list[str]]:
    """mxllm parameter name -> the HF tensors whose rows it concatenates."""
    m = {"tok_emb": ["model.embed_tokens.weight"], "final_norm": ["model.norm.weight"]}
    if not cfg.tie_embeddings:
        m["lm_head"] = ["lm_head.weight"]
    for i in range(cfg.n_layers):
        p, q = f"layers.{i}.", f"model.layers.{i}."
        m.update({
            p + "attn_norm": [q + "input_layernorm.weight"],
            p + "mlp_norm": [q + "post_attention_layernorm.weight"],
            p + "wqkv.weight": [q + f"self_attn.{x}_proj.weight" for x in ("q", "k", "v")],
            p + "wo.weight": [q + "self_attn.o_proj.weight"],
            p + "wgu.weight": [q + "mlp.gate_proj.weight", q + "mlp.up_proj.weight"],
            p + "wd.weight": [q + "mlp.down_proj.weight"],
        })
    return m


class HFReader:
    """Tensor-at-a-time access to a Hugging Face safetensors checkpoint (memory-mapped
    shards, opened once), with a record of what was read (strict loading)."""

    def __init__(self, path: str):
        from safetensors import safe_open

        self.path = path
        self.where: dict[str, object] = {}
        self._handles = []
        for fn in _shard_files(path):
            h = safe_open(fn, framework="pt", device="cpu")
            self._handles.append(h)
            for k in h.keys():
                self.where[k] = h
        self.used: set[str] = set()

    def rows(self, names: list[str]) -> list[torch.Tensor]:
        out = []
        for n in names:
            if n not in self.where:
                raise KeyError(f"{self.path}: missing tensor {n!r}")
            out.append(self.where[n].get_tensor(n))
            self.used.add(n)
        return out

    def fill_(self, dst: torch.Tensor, names: list[str]) -> None:
        """dst [rows, ...] <- the named tensors stacked along rows (dtype / device cast)."""
        off = 0
        for t in self.rows(names):
            if tuple(t.shape[1:]) != tuple(dst.shape[1:]) or off + t.shape[0] > dst.shape[0]:
                raise ValueError(f"{names}: checkpoint shape {tuple(t.shape)} does not fit {tuple(dst.shape)}")
            dst[off:off + t.shape[0]].copy_(t.to(dst.dtype))
            off += t.shape[0]
        if off != dst.shape[0]:
            raise ValueError(f"{names}: {off} checkpoint rows for a {dst.shape[0]}-row parameter")

    def check_all_used(self, tied: bool) -> None:
        extra = sorted(k for k in self.where if k not in self.used and not k.endswith("rotary_emb.inv_freq")
                       and not (tied and k == "lm_head.weight"))
        if extra:
            raise KeyError(f"{self.path}: unexpected tensors {extra[:6]}{' ...' if len(extra) > 6 else ''}")


@torch.no_grad()
def load_hf_llama(path: str, *, device=None, dtype: torch.dtype = torch.bfloat16, lora_r: int = 0,
                  lora_alpha: float = 16.0, seed: int = 0, **model_kw):
    """Build an mxllm ``Llama`` from a Hugging Face Llama directory (strict: every
    projection / norm / embedding tensor must be present and every checkpoint tensor
    used; rotary ``inv_freq`` buffers are ignored — mxllm recomputes the tables from
    the config).  LoRA adapters (``lora_r`` > 0) start as A ~ U(±1/sqrt(in)), B = 0."""
    from .llama import Llama

    cfg = load_hf_config(path)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    model = Llama(cfg, device=dev, dtype=dtype, lora_r=lora_r, lora_alpha=lora_alpha, seed=seed, init=False,
                  **model_kw)
    rd = HFReader(path)
    params = dict(model.named_parameters())
    for name, srcs in mx_to_hf(cfg).items():
        rd.fill_(params[name].data, srcs)
    rd.check_all_used(cfg.tie_embeddings)
    if lora_r > 0:
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        for layer in model.layers:
            for lin in (layer.wqkv, layer.wo, layer.wgu, layer.wd):
                bound = 1.0 / math.sqrt(lin.in_features)
                lin.lora_a.uniform_(-bound, bound, generator=gen)
                lin.lora_b.zero_()
        model.sync_adapters_()
    model.refresh_images_()
    return model


def hf_unit_filler(path: str, cfg: LlamaConfig):
    """``fill(names, numels, flat)``: write the named mxllm parameters, flattened and
    packed in order, from the checkpoint into ``flat`` (ZeRO-3 materialises one unit
    at a time from it, mxllm/parallel/zero3.py)."""
    rd = HFReader(path)
    srcmap = mx_to_hf(cfg)

    def fill(names, shapes, flat: torch.Tensor) -> None:
        off = 0
        for n, shp in zip(names, shapes):
            k = math.prod(shp)
            rd.fill_(flat[off:off + k].view(*shp), srcmap[n])
            off += k

    return fill


def _merged_weight(lin) -> torch.Tensor:
    w = lin.weight.detach()
    if lin.lora_r > 0:
        w = (w.float() + lin.scaling * (lin.lora_b.detach().float() @ lin.lora_a.detach().float())).to(w.dtype)
    return w


def hf_state_from_mx(state: dict[str, torch.Tensor], cfg: LlamaConfig,
                     dtype: torch.dtype | None = None) -> dict[str, torch.Tensor]:
    """mxllm-named full tensors (``layers.i.wqkv.weight`` ...) -> Hugging Face names,
    the fused projections split back into their row blocks (host, contiguous)."""
    sizes = {"wqkv.weight": [cfg.q_dim, cfg.kv_dim, cfg.kv_dim], "wgu.weight": [cfg.ffn, cfg.ffn]}
    out = {}
    for name, srcs in mx_to_hf(cfg).items():
        t = state[name].detach()
        t = (t.to(dtype) if dtype is not None else t).to("cpu")
        rows = next((v for k, v in sizes.items() if name.endswith(k)), [t.shape[0]])
        off = 0
        for src, n in zip(srcs, rows):
            out[src] = t[off:off + n].contiguous()
            off += n
    return out


@torch.no_grad()
def hf_state_dict(model, merge_lora: bool = True, dtype: torch.dtype | None = None) -> dict[str, torch.Tensor]:
    """The model's tensors under Hugging Face names (host, contiguous); LoRA merged
    into the base projections when ``merge_lora`` (else the base weights alone)."""
    state = {}
    for name, p in model.named_parameters():
        if "lora_" in name:
            continue
        state[name] = p
    if merge_lora:
        for i, layer in enumerate(model.layers):
            for key in ("wqkv", "wo", "wgu", "wd"):
                state[f"layers.{i}.{key}.weight"] = _merged_weight(getattr(layer, key))
    return hf_state_from_mx(state, model.cfg, dtype)


@torch.no_grad()
def save_hf_llama(model, path: str, *, merge_lora: bool = True, max_shard_bytes: int = 5 << 30,
                  dtype: torch.dtype | None = None, cfg: LlamaConfig | None = None) -> list[str]:
    """Write ``config.json`` + ``model-0000k-of-0000n.safetensors`` (+ the index when
    sharded) loadable by ``transformers.LlamaForCausalLM.from_pretrained`` and by
    ``load_hf_llama``.  ``model``: an mxllm ``Llama`` (LoRA merged when
    ``merge_lora``) or a dict of mxllm-named full tensors with ``cfg`` (e.g. a ZeRO-3
    trainer's ``full_state_dict()``).  Returns the shard paths."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    if isinstance(model, dict):
        if cfg is None:
            raise ValueError("save_hf_llama(state_dict, ...) needs cfg")
        sd = hf_state_from_mx(model, cfg, dtype)
    else:
        cfg = model.cfg
        sd = hf_state_dict(model, merge_lora=merge_lora, dtype=dtype)
    out_dtype = next(iter(sd.values())).dtype
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(config_to_hf(cfg, out_dtype), f, indent=2)
    shards, cur, size = [], {}, 0
    for name, t in sd.items():
        nb = t.numel() * t.element_size()
        if cur and size + nb > max_shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[name] = t
        size += nb
    if cur:
        shards.append(cur)
    files = []
    if len(shards) == 1:
        files.append(os.path.join(path, "model.safetensors"))
        save_file(shards[0], files[0], metadata={"format": "pt"})
        return files
    wmap = {}
    for k, sh in enumerate(shards):
        fn = f"model-{k + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(path, fn), metadata={"format": "pt"})
        files.append(os.path.join(path, fn))
        wmap.update({n: fn for n in sh})
    total = sum(t.numel() * t.element_size() for t in sd.values())
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f, indent=2)
    return files
