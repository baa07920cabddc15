"""Reference ``src/utils.py`` surface, MI355X-native.

* ``setup_logging`` — identical format/datefmt (reference src/utils.py:5-10).
* ``process_batch(model, prompts, labels, get_model_response)`` — same
  signature and 0-d tensor result (reference :12-23).  With a real mxllm
  ``Llama`` it computes a REAL next-token loss over prompt + response through
  the model; with any other module it keeps the reference's
  simulated binary-classification loss.
* ``gpu_tensor_operation(text, device)`` — float32 mean of the code points
  (reference :25-28); on a GPU it runs the batched ``segmented_mean`` HIP
  kernel.  ``gpu_tensor_operations`` does a whole batch in one launch, one
  pinned H2D copy and one D2H copy.
"""
from __future__ import annotations

import logging
import os
import sys

import torch
from torch.nn.functional import cross_entropy

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)


def setup_logging():
    logging.basicConfig(
        level=logging.INFO,
        format='%(asctime)s - %(levelname)s - %(message)s',
        datefmt='%Y-%m-%d %H:%M:%S'
    )


def process_batch(model, prompts, labels, get_model_response):
    from mxllm.models import Llama

    if isinstance(model, Llama):
        return _lm_loss(model, prompts, [get_model_response(p) for p in prompts])
    batch_loss = 0
    for prompt, label in zip(prompts, labels):
        get_model_response(prompt)
        logits = torch.randn(2)
        loss = cross_entropy(logits.unsqueeze(0), torch.tensor([int(label)]))
        batch_loss += loss
    return batch_loss / len(prompts)


def _lm_loss(model, prompts, responses, max_len: int = 512):
    from mxllm.data.tokenizer import get_tokenizer

    cfg = model.cfg
    tok = get_tokenizer(cfg.vocab_size, None, cfg.bos_id, cfg.eos_id)
    dev = model.tok_emb.device
    seqs = [tok.encode(p + "\n" + r)[:max_len + 1] for p, r in zip(prompts, responses)]
    L = max(len(s) for s in seqs)
    ids = torch.zeros(len(seqs), L - 1, dtype=torch.long)
    lab = torch.full((len(seqs), L - 1), -100, dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, :len(s) - 1] = torch.tensor(s[:-1])
        lab[i, :len(s) - 1] = torch.tensor(s[1:])
    return model(ids.to(dev), lab.to(dev))


def gpu_tensor_operations(texts, device) -> list[float]:
    """Batched K16: means of code points for every text, one kernel launch."""
    device = torch.device(device)
    codes = [ord(c) for t in texts for c in t]
    lens = [len(t) for t in texts]
    if device.type == "cuda":
        from mxllm.ops import native

        cpu = torch.tensor(codes, dtype=torch.int32).pin_memory()
        offs = torch.tensor([0] + lens, dtype=torch.int64).cumsum(0).pin_memory()
        out = native().segmented_mean(cpu.to(device, non_blocking=True), offs.to(device, non_blocking=True))
        return out.cpu().tolist()
    res = []
    off = 0
    t = torch.tensor(codes, dtype=torch.float32)
    for n in lens:
        res.append(t[off:off + n].mean().item())
        off += n
    return res


def gpu_tensor_operation(text, device):
    return float(gpu_tensor_operations([text], device)[0])
