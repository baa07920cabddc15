from .config import LlamaConfig, PRESETS, get_config  # noqa: F401
from .llama import Llama, FusedLinear  # noqa: F401
from .hf import is_hf_dir, load_hf_config, load_hf_llama, save_hf_llama  # noqa: F401


def model_config(name: str) -> LlamaConfig:
    """A preset name (``llama3.1-8b`` ...) or a Hugging Face Llama directory."""
    return load_hf_config(name) if is_hf_dir(name) else get_config(name)


def build_model(name: str, *, device=None, dtype=None, lora_r: int = 0, lora_alpha: float = 16.0, seed: int = 0,
                **kw) -> Llama:
    """Random-init preset, or the weights of a Hugging Face Llama directory."""
    import torch

    dtype = dtype or torch.bfloat16
    if is_hf_dir(name):
        return load_hf_llama(name, device=device, dtype=dtype, lora_r=lora_r, lora_alpha=lora_alpha, seed=seed, **kw)
    return Llama(get_config(name), device=device, dtype=dtype, lora_r=lora_r, lora_alpha=lora_alpha, seed=seed, **kw)


def tokenizer_path_for(name: str, explicit: str | None = None) -> str | None:
    """An explicit tokenizer.json, else the one shipped in a Hugging Face model directory."""
    import os

    if explicit:
        return explicit
    if is_hf_dir(name) and os.path.exists(os.path.join(name, "tokenizer.json")):
        return os.path.join(name, "tokenizer.json")
    return None
