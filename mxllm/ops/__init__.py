"""mxllm ops: HIP/CDNA4 kernels (GPU) with pure-PyTorch reference paths (CPU).

See ``mxllm/ops/_ext.py`` for the dispatch policy (no silent GPU fallback).
"""
from ._ext import available as native_available, native, use_native  # noqa: F401
from .norm import rms_norm, add_rms_norm  # noqa: F401
from .attention import attention_block  # noqa: F401
from .activation import lora_tail_ok, swiglu  # noqa: F401
from .loss import linear_cross_entropy, cross_entropy  # noqa: F401
from .optim import SplitMaster, adamw_step_, sq_norm  # noqa: F401
from .embedding import embedding  # noqa: F401
from .linear import linear, lora_linear, lora_linear_aug, lora_qkv_attention, lora_qkv_attention_at, linear_swiglu, norm_linear, normed_linear, qkv_rope_linear, qkv_rope_ok, swiglu_linear, transpose2d  # noqa: F401
from . import reference  # noqa: F401
