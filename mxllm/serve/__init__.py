from .engine import Engine, SamplingParams, merge_lora_  # noqa: F401
from . import client  # noqa: F401
