"""Default CONFIG (the reference imports a gitignored ``config.CONFIG``).

Keys match the reference (src/distributed_inference.py:15-16,37,53-54).  Values
here are defaults only: torchrun's MASTER_ADDR/MASTER_PORT and MXLLM_* env vars
take precedence (see mxllm/config.py).  API_BASE "local" serves completions from
mxllm's in-process engine on this rank's GPU; set it to an http URL to call an
OpenAI-compatible server (e.g. ``python -m mxllm.serve.server``).
"""
import os

CONFIG = {
    "MASTER_ADDR": os.environ.get("MASTER_ADDR", "127.0.0.1"),
    "MASTER_PORT": os.environ.get("MASTER_PORT", "29500"),
    "MODEL_NAME": os.environ.get("MXLLM_MODEL_NAME", "mxllm/llama3.1-70b"),
    "API_KEY": os.environ.get("OPENAI_API_KEY", ""),
    "API_BASE": os.environ.get("MXLLM_API_BASE", "local"),
}
