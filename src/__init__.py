"""Reference-compatible entry points (naman1618/Distributed-Inference-with-PyTorch-and-LiteLLM API surface)."""
