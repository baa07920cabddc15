"""Distributed inference driver — reference ``src/distributed_inference.py``
API and behaviour, MI355X-native.

Same surface: ``setup(rank, world_size)``, ``cleanup()``, ``CustomDataset``,
``get_model_response(prompt)`` (same fallback string), ``main()`` (same flow
and log lines: "Using device:", "Starting epoch N", and per prompt on rank 0
"Prompt:", "Response:", "Label:", "GPU Result:").  Differences, all fixes of
SURVEY §0.4:
  * D3: torchrun's MASTER_ADDR/PORT are never overwritten by CONFIG;
  * D4: each process binds cuda:LOCAL_RANK; backend RCCL with GPUs, gloo on CPU;
  * D5: an exported OPENAI_API_KEY is respected;
  * D6: cleanup() on every exit path;
  * D10: offline synthetic IMDB-like data when the HF dataset is not cached;
  * completions are served by mxllm's own engine on this rank's GPU
    (API_BASE "local") as one batched generation per DataLoader batch, or by an
    OpenAI-compatible server (API_BASE http://...) with retries/backoff (D11).
Launch: ``torchrun --nproc_per_node=N src/distributed_inference.py`` or
scripts/run_node{0,1}.sh.
"""
import logging
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
# the repo root (for mxllm); src/ itself is on the path only when run as a script
# (adding it on import would shadow the top-level ``tests`` package with src/tests)
if os.path.dirname(_HERE) not in sys.path:
    sys.path.insert(0, os.path.dirname(_HERE))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from mxllm.config import load_config  # noqa: E402
from mxllm.data.datasets import CustomDataset, load_text_dataset  # noqa: E402,F401
from mxllm.parallel import runtime  # noqa: E402
from mxllm.serve import client as litellm  # noqa: E402  (LiteLLM-compatible; litellm is not installed)
from mxllm.utils.faults import maybe_inject  # noqa: E402

try:  # the reference's module layout: run as a script from src/
    from utils import setup_logging, gpu_tensor_operation, gpu_tensor_operations  # noqa: F401
    from config import CONFIG
except ImportError:  # imported as src.distributed_inference
    from src.utils import setup_logging, gpu_tensor_operation, gpu_tensor_operations  # noqa: F401
    from src.config import CONFIG

FALLBACK = "Error: Unable to get model response"
RUN = load_config(CONFIG)


def setup(rank, world_size):
    """Create the process group (env:// rendezvous) and run one barrier."""
    return runtime.init(backend=RUN.backend or None, rank=rank, world_size=world_size,
                        master_addr=CONFIG.get('MASTER_ADDR'), master_port=CONFIG.get('MASTER_PORT'))


def cleanup():
    runtime.cleanup()


def get_model_response(prompt):
    messages = [{"content": prompt, "role": "user"}]
    try:
        response = litellm.completion(CONFIG['MODEL_NAME'], messages, max_tokens=RUN.max_new_tokens,
                                      temperature=RUN.temperature, timeout=RUN.request_timeout,
                                      num_retries=RUN.num_retries)
        return response.choices[0].message.content
    except Exception as e:
        logging.error(f"Error getting model response: {e}")
        return FALLBACK


def get_model_responses(prompts):
    """Batched version: one engine pass for a local model, per-prompt HTTP otherwise."""
    if litellm.api_base in (None, "", "local", "inproc") and litellm._LOCAL:
        try:
            return litellm.batch_local(CONFIG['MODEL_NAME'], list(prompts), max_tokens=RUN.max_new_tokens,
                                       temperature=RUN.temperature)
        except Exception as e:
            logging.error(f"Error getting model response: {e}")
            return [FALLBACK] * len(prompts)
    return [get_model_response(p) for p in prompts]


def _local_engine():
    return litellm.api_base in (None, "", "local", "inproc") and bool(litellm._LOCAL)


def _submit(prompts):
    try:
        return litellm.submit_local(CONFIG['MODEL_NAME'], list(prompts), max_tokens=RUN.max_new_tokens,
                                    temperature=RUN.temperature)
    except Exception as e:
        logging.error(f"Error getting model response: {e}")
        return None


def _collect(reqs, n):
    if reqs is None:
        return [FALLBACK] * n
    try:
        return litellm.collect_local(CONFIG['MODEL_NAME'], reqs, timeout=RUN.request_timeout * max(1, n))
    except Exception as e:
        logging.error(f"Error getting model response: {e}")
        return [FALLBACK] * n


def _configure_client(device):
    if os.environ.get("OPENAI_API_KEY"):
        litellm.api_key = os.environ["OPENAI_API_KEY"]
    elif CONFIG.get('API_KEY'):
        litellm.api_key = CONFIG['API_KEY']
        os.environ.setdefault("OPENAI_API_KEY", CONFIG['API_KEY'])
    litellm.api_base = RUN.api_base or CONFIG.get('API_BASE')
    litellm.request_timeout = RUN.request_timeout
    litellm.num_retries = RUN.num_retries
    if litellm.api_base in (None, "", "local", "inproc"):
        from mxllm.serve.local import ensure_local_engine

        ensure_local_engine(CONFIG['MODEL_NAME'], device, RUN.engine_model, RUN.max_batch,
                            RUN.max_seq if device.type == "cuda" else min(RUN.max_seq, 1024), RUN.tokenizer,
                            RUN.checkpoint, RUN.seed, RUN.engine_weights, RUN.kv_pool_tokens)


def _gather_results(records, rank, world_size):
    """Opt-in (``--gather-results``): collect every rank's records on rank 0.
    The reference logs only rank 0's own shard (reference
    src/distributed_inference.py:71); that stays the default."""
    if dist.is_initialized() and world_size > 1:
        allr = [None] * world_size if rank == 0 else None
        dist.gather_object(records, allr, dst=0)
    else:
        allr = [records]
    if rank == 0:
        flat = [r for part in allr for r in part]
        logging.info(f"Gathered {len(flat)} results from {world_size} ranks")
        if RUN.results_file:
            import json

            with open(RUN.results_file, "w") as f:
                for r in flat:
                    f.write(json.dumps(r) + "\n")


def main():
    setup_logging()
    code = 0
    try:
        rank = int(os.environ.get("RANK", 0))
        world_size = int(os.environ.get("WORLD_SIZE", 1))
        env = setup(rank, world_size)

        device = env.device
        logging.info(f"Using device: {device}")

        _configure_client(device)

        texts, labels = load_text_dataset(RUN.dataset, RUN.split, RUN.n_rows, RUN.seed)
        custom_dataset = CustomDataset(texts, labels)
        train_sampler = torch.utils.data.distributed.DistributedSampler(
            custom_dataset, num_replicas=world_size, rank=rank, seed=RUN.seed)
        train_dataloader = DataLoader(custom_dataset, batch_size=RUN.batch_size, sampler=train_sampler)

        records = []
        step = 0

        def emit(epoch, prompts, labels, gpu_results, responses):
            if rank == 0:
                n = RUN.truncate
                for prompt, response, label, gpu_result in zip(prompts, responses, labels, gpu_results):
                    logging.info(f"Prompt: {prompt[:n]}...")
                    logging.info(f"Response: {response[:n]}...")
                    logging.info(f"Label: {label}")
                    logging.info(f"GPU Result: {gpu_result}\n")
            if RUN.gather_results:
                n = RUN.truncate
                records.extend({"rank": rank, "epoch": epoch, "prompt": p[:n], "response": r[:n],
                                "label": int(lb), "gpu_result": float(g)}
                               for p, r, lb, g in zip(prompts, responses, labels, gpu_results))

        # lookahead_batches > 0: keep that many DataLoader batches in flight on the
        # local engine (generated together by continuous batching), results still
        # logged batch by batch in order; 0 = one batch at a time, as the reference
        lookahead = RUN.lookahead_batches if _local_engine() else 0
        for epoch in range(RUN.epochs):
            logging.info(f"Starting epoch {epoch}")
            train_sampler.set_epoch(epoch)
            pending = []  # (prompts, labels, gpu_results, engine requests), oldest first
            for batch in train_dataloader:
                maybe_inject(RUN, rank, step)
                prompts = batch["text"]
                labels = batch["label"]

                gpu_results = gpu_tensor_operations(prompts, device)
                if lookahead > 0:
                    pending.append((prompts, labels, gpu_results, _submit(prompts)))
                    while len(pending) > lookahead:
                        p_, l_, g_, reqs = pending.pop(0)
                        emit(epoch, p_, l_, g_, _collect(reqs, len(p_)))
                else:
                    emit(epoch, prompts, labels, gpu_results, get_model_responses(prompts))
                step += 1
            for p_, l_, g_, reqs in pending:  # drained before the next "Starting epoch" line
                emit(epoch, p_, l_, g_, _collect(reqs, len(p_)))
        if RUN.gather_results:
            _gather_results(records, rank, world_size)
        if dist.is_initialized():
            runtime.barrier()
    except Exception as e:
        logging.error(f"An error occurred in the main function: {e}")
        code = 1
    finally:
        cleanup()
    if code:
        sys.exit(code)


if __name__ == "__main__":
    main()
