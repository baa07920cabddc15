"""Llama-3.x architecture configs (SURVEY §7.6 sizing).

Presets match the published Llama-3.1 / 3.2 shapes; ``tiny`` is a small
random-init stand-in for CPU plumbing tests (BASELINE config 1).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass
class LlamaConfig:
    name: str = "tiny"
    vocab_size: int = 512
    hidden: int = 256
    n_layers: int = 2
    n_heads: int = 8
    n_kv_heads: int = 2
    ffn: int = 512
    head_dim: int = 32
    rope_theta: float = 500000.0
    rope_scaling: dict | None = field(default_factory=lambda: {
        "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 8192})
    norm_eps: float = 1e-5
    max_seq_len: int = 8192
    tie_embeddings: bool = False
    bos_id: int = 256
    eos_id: int = 257

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    def n_params(self) -> int:
        h, f = self.hidden, self.ffn
        per_layer = h * (self.q_dim + 2 * self.kv_dim) + self.q_dim * h + 3 * h * f + 2 * h
        emb = self.vocab_size * h
        return self.n_layers * per_layer + emb * (1 if self.tie_embeddings else 2) + h

    def train_flops_per_token(self, seq_len: int, lora: bool = False) -> float:
        """Model FLOPs per trained token: 6N (full) or 4N (frozen base: no weight
        grads) on the matmul params + causal attention (fwd 2*2*S/2*D*Hq per layer,
        bwd 2.5x)."""
        n_mat = self.n_params() - self.vocab_size * self.hidden * (0 if self.tie_embeddings else 1) \
            - (2 * self.n_layers + 1) * self.hidden
        k = 4.0 if lora else 6.0
        attn_fwd = 2.0 * 2.0 * (seq_len / 2.0) * self.head_dim * self.n_heads * self.n_layers
        return k * n_mat + 3.5 * attn_fwd

    def replace(self, **kw) -> "LlamaConfig":
        return dataclasses.replace(self, **kw)


PRESETS: dict[str, LlamaConfig] = {
    "tiny": LlamaConfig(),
    "llama3.2-1b": LlamaConfig(name="llama3.2-1b", vocab_size=128256, hidden=2048, n_layers=16, n_heads=32,
                               n_kv_heads=8, ffn=8192, head_dim=64, tie_embeddings=True,
                               rope_scaling={"factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                             "original_max_position_embeddings": 8192},
                               max_seq_len=131072, bos_id=128000, eos_id=128001),
    "llama3.1-8b": LlamaConfig(name="llama3.1-8b", vocab_size=128256, hidden=4096, n_layers=32, n_heads=32,
                               n_kv_heads=8, ffn=14336, head_dim=128, max_seq_len=131072,
                               bos_id=128000, eos_id=128001),
    "llama3.1-70b": LlamaConfig(name="llama3.1-70b", vocab_size=128256, hidden=8192, n_layers=80, n_heads=64,
                                n_kv_heads=8, ffn=28672, head_dim=128, max_seq_len=131072,
                                bos_id=128000, eos_id=128001),
}
PRESETS["tiny-d128"] = PRESETS["tiny"].replace(name="tiny-d128", hidden=512, n_heads=4, n_kv_heads=2,
                                               head_dim=128, ffn=1024)


def get_config(name: str, **overrides) -> LlamaConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; have {sorted(PRESETS)}")
    return PRESETS[name].replace(**overrides) if overrides else PRESETS[name]
