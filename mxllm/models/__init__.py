from .config import LlamaConfig, PRESETS, get_config  # noqa: F401
from .llama import Llama, FusedLinear  # noqa: F401
