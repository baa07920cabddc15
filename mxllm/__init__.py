"""mxllm — MI355X-native (gfx950/CDNA4) distributed fine-tuning and inference.

Capabilities of naman1618/Distributed-Inference-with-PyTorch-and-LiteLLM,
re-designed MI355X-first: torchrun launch + RCCL over xGMI, own bucketed DDP
and sharded data parallel, Llama-3.1 8B/70B fine-tuning with hand-written
HIP kernels for the hot ops, and a local OpenAI/LiteLLM-compatible completion
endpoint served by mxllm's own inference engine.
"""
__version__ = "0.1.0"
