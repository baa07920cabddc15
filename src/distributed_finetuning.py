"""Distributed fine-tuning driver — the program the reference's launch scripts
and tests name (reference scripts/run_node0.sh:16, tests/...:4) but never
shipped.

Exposes the same ``setup``/``cleanup``/``CustomDataset`` API as
``src/distributed_inference.py`` and a real ``main()``: Llama-3.1 (tiny / 8B /
70B presets) with LoRA or full fine-tuning, mxllm's bucketed DDP over RCCL
(or ZeRO-3 sharding), fused HIP kernels, the native threaded token loader,
checkpoint/resume and fault-injection hooks.

  torchrun --nproc_per_node=8 src/distributed_finetuning.py --model llama3.1-8b \
      --finetune full --seq-len 2048 --micro-batch 2 --steps 100 --ckpt-dir /tmp/ck
"""
import logging
import math
import os
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))
# the repo root (for mxllm); src/ itself is on the path only when run as a script
# (adding it on import would shadow the top-level ``tests`` package with src/tests)
if os.path.dirname(_HERE) not in sys.path:
    sys.path.insert(0, os.path.dirname(_HERE))

import torch  # noqa: E402

from mxllm.config import load_config  # noqa: E402
from mxllm.data.datasets import CustomDataset, load_text_dataset  # noqa: E402,F401
from mxllm.parallel import runtime  # noqa: E402
from mxllm.utils.faults import maybe_inject  # noqa: E402
from mxllm.utils.metrics import MetricsWriter  # noqa: E402

try:
    from utils import setup_logging
    from config import CONFIG
except ImportError:
    from src.utils import setup_logging
    from src.config import CONFIG


def setup(rank, world_size):
    """Create the process group (env:// rendezvous, RCCL with GPUs / gloo on CPU)."""
    return runtime.init(rank=rank, world_size=world_size, master_addr=CONFIG.get('MASTER_ADDR'),
                        master_port=CONFIG.get('MASTER_PORT'))


def cleanup():
    runtime.cleanup()


def _ckpt_setting(run):
    """bool (every layer / none) or the number of leading layers checkpointed."""
    if run.activation_checkpointing and run.ckpt_layers >= 0:
        return int(run.ckpt_layers)
    return bool(run.activation_checkpointing)


def build_trainer(run, env):
    """``run.model``: a preset (random init) or a Hugging Face Llama directory (its
    weights; ZeRO-3 reads them unit by unit, so no rank holds the whole model)."""
    from mxllm.models import build_model, is_hf_dir, model_config
    from mxllm.train.trainer import OptimConfig, Trainer

    cfg = model_config(run.model)
    lora_r = run.lora_r if run.finetune == "lora" else 0
    opt = OptimConfig(lr=run.lr, weight_decay=run.weight_decay, grad_clip=run.grad_clip,
                      warmup_steps=run.warmup_steps, total_steps=run.steps)
    if run.parallel == "zero3":
        from mxllm.parallel.zero3 import Zero3Trainer

        return Zero3Trainer(cfg, env, opt, seed=run.seed, activation_checkpointing=_ckpt_setting(run),
                            init_from=run.model if is_hf_dir(run.model) else None)
    model = build_model(run.model, device=env.device, lora_r=lora_r, lora_alpha=run.lora_alpha, seed=run.seed,
                        activation_checkpointing=_ckpt_setting(run))
    return Trainer(model, env, opt, bucket_mb=run.bucket_mb, shard_optimizer=run.parallel == "zero1")


def export_hf(run, trainer, rank):
    """--save-hf DIR: the trained model as a Hugging Face Llama checkpoint (LoRA merged;
    ZeRO-3 gathers unit by unit to rank 0).  Collective for ZeRO-3 / ZeRO-1."""
    from mxllm.models import save_hf_llama

    trainer.params_ready()  # overlapped optimizer chunks / ZeRO-1 all-gathers have landed
    if run.parallel == "zero3":
        state = trainer.full_state_dict()
        if rank == 0:
            save_hf_llama(state, run.save_hf, cfg=trainer.model.cfg)
    elif rank == 0:
        save_hf_llama(trainer.model, run.save_hf)
    runtime.barrier()
    if rank == 0:
        logging.info(f"Hugging Face checkpoint written to {run.save_hf}")


def main(argv=None):
    setup_logging()
    code = 0
    try:
        run = load_config(CONFIG, sys.argv[1:] if argv is None else argv)
        rank = int(os.environ.get("RANK", 0))
        world_size = int(os.environ.get("WORLD_SIZE", 1))
        env = setup(rank, world_size)
        logging.info(f"Using device: {env.device}")

        from mxllm.data.loader import TokenLoader, pack_texts
        from mxllm.data.tokenizer import get_tokenizer
        from mxllm.models import model_config, tokenizer_path_for
        from mxllm.train import checkpoint

        trainer = build_trainer(run, env)
        sp_group, data_rank, data_world, shard = None, rank, world_size, None
        if run.sequence_parallel > 1 and run.context_parallel > 1:
            raise ValueError("--sequence-parallel and --context-parallel are alternatives")
        if run.sequence_parallel > 1 or run.context_parallel > 1:
            if run.parallel not in ("ddp", "zero1"):
                raise ValueError("--sequence-parallel / --context-parallel are supported with --parallel ddp / zero1")
            from mxllm.parallel.sequence import new_groups, shard_sequence

            sp_group, data_rank, data_world = new_groups(max(run.sequence_parallel, run.context_parallel))
            if run.context_parallel > 1:  # ring attention over zigzag-sharded sequences
                from mxllm.parallel.context import zigzag_shard

                trainer.model.set_context_parallel(sp_group)
                shard = zigzag_shard
            else:  # Ulysses all-to-all around attention
                trainer.model.set_sequence_parallel(sp_group)
                shard = shard_sequence
        mcfg = model_config(run.model)
        tok = get_tokenizer(mcfg.vocab_size, tokenizer_path_for(run.model, run.tokenizer or None), mcfg.bos_id,
                            mcfg.eos_id)
        texts, _ = load_text_dataset(run.dataset, run.split, run.n_rows, run.seed)
        tokens = pack_texts(texts, tok, getattr(tok, "eos_id", mcfg.eos_id))
        loader = TokenLoader(tokens, run.seq_len, run.micro_batch, data_rank, data_world, run.seed, env.device)
        steps_per_epoch = max(1, loader.batches_per_epoch // run.grad_accum)
        total = run.steps or run.epochs * steps_per_epoch
        start = 0
        if run.ckpt_dir and run.resume:
            extra = checkpoint.load(run.ckpt_dir, trainer)
            if extra is not None:
                loader.restore(extra["loader"])
                start = trainer.step_num
                logging.info(f"Resumed at step {start}")
        sync_check = run.check_sync_every >= 0 and run.parallel in ("ddp", "zero1")
        if sync_check:
            from mxllm.parallel.consistency import check_in_sync

            check_in_sync(trainer.flat.params, what="initial trainable parameters")
        metrics = MetricsWriter(run.metrics_file or None, rank)
        monitor = None
        if run.gpu_monitor_s > 0 and run.metrics_file and env.device.type == "cuda":
            from mxllm.utils.gpumon import GpuMonitor

            gpu_log = MetricsWriter(run.metrics_file, rank, all_ranks=True)
            monitor = GpuMonitor(env.device, run.gpu_monitor_s, lambda smp: gpu_log.write(kind="gpu", **smp)).start()
        tok_per_step = run.micro_batch * run.seq_len * run.grad_accum * data_world
        t_last, n_since = time.perf_counter(), 0
        for step in range(start, total):
            maybe_inject(run, rank, step)
            mbs = []
            for _ in range(run.grad_accum):
                ids, lab, epoch, _i = loader.next_device()
                if sp_group is not None:
                    ids, lab = shard(ids, sp_group), shard(lab, sp_group)
                mbs.append((ids, lab))
            loss = trainer.train_step(mbs)
            n_since += 1
            last = step == total - 1
            if step % run.log_every == 0 or last:
                lv = runtime.all_reduce_scalars([float(loss)], "sum")[0] / world_size
                if not math.isfinite(lv):
                    raise FloatingPointError(f"non-finite loss {lv} at step {step}")
                if env.device.type == "cuda":
                    torch.cuda.synchronize()
                dt = time.perf_counter() - t_last
                tps = tok_per_step * n_since / max(dt, 1e-9)
                gn = float(trainer.last_grad_norm) if getattr(trainer, "last_grad_norm", None) is not None else 0.0
                if rank == 0:
                    logging.info(f"step {step} epoch {epoch} loss {lv:.4f} grad_norm {gn:.3f} tokens/s {tps:.0f}")
                extra = {}
                ddp = getattr(trainer, "ddp", None)
                if ddp is not None and ddp.enabled:
                    extra = {"allreduce_bytes": ddp.bytes_per_step, "exposed_comm_ms": ddp.exposed_comm_ms()}
                if env.device.type == "cuda":
                    extra["peak_hbm_gb"] = torch.cuda.max_memory_allocated(env.device) / 1e9
                metrics.write(step=step, epoch=epoch, loss=lv, grad_norm=gn, tokens_per_s=tps, **extra)
                t_last, n_since = time.perf_counter(), 0
            if sync_check and run.check_sync_every > 0 and (step + 1) % run.check_sync_every == 0:
                trainer.params_ready()  # else the checksum may read half-updated parameters
                check_in_sync(trainer.flat.params, what=f"trainable parameters after step {step}")
            if run.ckpt_dir and run.save_every and (step + 1) % run.save_every == 0:
                checkpoint.save(run.ckpt_dir, trainer, step + 1, extra={"loader": loader.state()})
        loader.close()
        if monitor is not None:
            monitor.stop()
        if run.metrics_file and hasattr(trainer, "master_fp32"):
            # bit-level digest of the final fp32 master weights (exact integer sums of the bit
            # patterns): equal digests <=> (almost surely) bitwise-equal weights -- deterministic
            # mode / resume comparisons (scripts/compare_resume.py)
            m = trainer.master_fp32().reshape(-1).view(torch.int32)
            s1 = s2 = 0
            for lo in range(0, m.numel(), 1 << 26):
                c = m[lo:lo + (1 << 26)].to(torch.int64)
                s1 += int(c.sum())
                s2 += int((c * torch.arange(lo, lo + c.numel(), device=c.device, dtype=torch.int64).remainder_(
                    1000003)).sum())
            metrics.write(kind="final", step=total, master_bits_sum=s1, master_bits_wsum=s2, numel=m.numel())
        if run.save_hf:
            export_hf(run, trainer, rank)
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
