"""Runtime subsystems on CPU: config precedence, native token loader sharding
and resume, checkpoint round trip, torchrun end-to-end plumbing (BASELINE
config 1), 2-node emulation, fault injection (fail fast, restart + resume)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**kw):
    e = dict(os.environ)
    e.update(MXLLM_FORCE_CPU="1", OMP_NUM_THREADS="1", HF_DATASETS_OFFLINE="1", PYTHONPATH=ROOT)
    e.update({k: str(v) for k, v in kw.items()})
    return e


def test_config_precedence(monkeypatch):
    from mxllm.config import load_config

    monkeypatch.setenv("MXLLM_BATCH_SIZE", "7")
    monkeypatch.setenv("MXLLM_EPOCHS", "5")
    cfg = load_config({"MASTER_PORT": "29511", "EPOCHS": 2, "API_BASE": "http://x"}, ["--epochs", "9"])
    assert cfg.master_port == 29511 and cfg.api_base == "http://x"
    assert cfg.batch_size == 7  # env over default
    assert cfg.epochs == 9  # CLI over env over CONFIG
    d = load_config(use_env=False)
    assert (d.batch_size, d.epochs, d.truncate, d.n_rows) == (4, 3, 100, 250)  # reference constants


def test_torchrun_env_wins_over_config(monkeypatch):
    """CONFIG's MASTER_* must never clobber the launcher's."""
    from mxllm.parallel import runtime

    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_port()))
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    before = os.environ["MASTER_PORT"]
    runtime.cleanup()
    runtime.init(rank=0, world_size=1, master_addr="10.9.9.9", master_port=1)
    assert os.environ["MASTER_PORT"] == before and os.environ["MASTER_ADDR"] == "127.0.0.1"
    runtime.cleanup()


def test_token_loader_sharding_and_resume():
    from mxllm.data.loader import TokenLoader

    toks = torch.arange(0, 40 * 33, dtype=torch.int32)
    world = 4
    seen = []
    for r in range(world):
        ld = TokenLoader(toks, 32, 2, r, world, seed=5)
        ids = [ld.next()[0] for _ in range(ld.batches_per_epoch)]
        seen.append({int(x[i, 0]) for x in ids for i in range(x.shape[0])})
        ld.close()
    for a in range(world):
        for b in range(a + 1, world):
            assert not (seen[a] & seen[b]), "ranks must see disjoint sequences"
    ld = TokenLoader(toks, 32, 2, 0, 1, seed=5)
    ids, lab, _, _ = ld.next()
    assert torch.equal(ids[:, 1:], lab[:, :-1])  # labels are the next tokens
    ld.next()
    st = ld.state()
    want = ld.next()[0]
    ld.restore(st)
    assert torch.equal(ld.next()[0], want)
    ld.close()


def test_checkpoint_roundtrip(tmp_path, monkeypatch):
    monkeypatch.setenv("MXLLM_FORCE_CPU", "1")
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.train import checkpoint
    from mxllm.train.trainer import OptimConfig, Trainer

    runtime.cleanup()
    env = runtime.init(rank=0, world_size=1)
    cfg = get_config("tiny").replace(n_layers=1, vocab_size=300)
    ids = torch.randint(0, 300, (2, 16), generator=torch.Generator().manual_seed(0))
    t1 = Trainer(Llama(cfg, lora_r=4, seed=1), env, OptimConfig(lr=1e-2))
    for _ in range(3):
        t1.train_step([(ids, ids)])
    checkpoint.save(str(tmp_path), t1, 3, extra={"loader": {"epoch": 0, "cursor": 3}})
    l_next = float(t1.train_step([(ids, ids)]))
    t2 = Trainer(Llama(cfg, lora_r=4, seed=1), env, OptimConfig(lr=1e-2))
    extra = checkpoint.load(str(tmp_path), t2)
    assert extra["loader"]["cursor"] == 3 and t2.step_num == 3
    assert abs(float(t2.train_step([(ids, ids)])) - l_next) < 1e-5
    runtime.cleanup()


@pytest.mark.slow
def test_inference_plumbing_two_ranks(tmp_path):
    """BASELINE config 1: distributed_inference on the tiny stub, gloo, world 2:
    every rank sees 125 prompts x 3 epochs; rank 0 logs 375 records; the
    opt-in gather (C9) brings all 750 records, disjoint per epoch, to rank 0."""
    out = tmp_path / "results.jsonl"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_port()), "src/distributed_inference.py"], cwd=ROOT,
                       env=_env(MXLLM_MAX_NEW_TOKENS=2, MXLLM_MAX_SEQ=256, MXLLM_GATHER_RESULTS=1,
                                MXLLM_RESULTS_FILE=str(out)), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    log = r.stdout + r.stderr
    assert log.count("Prompt: ") == 375
    assert log.count("Starting epoch") == 6
    assert "An error occurred" not in log
    assert "Gathered 750 results from 2 ranks" in log
    import json

    recs = [json.loads(x) for x in out.read_text().splitlines()]
    assert len(recs) == 750
    assert sum(1 for x in recs if x["rank"] == 1) == 375


def test_inference_lookahead_same_records(tmp_path):
    """DataLoader batches kept in flight on the local engine (lookahead 8, the
    default) produce exactly the records, in exactly the order, of the
    reference's one-batch-at-a-time loop (lookahead 0)."""
    import json

    recs = {}
    for la in (0, 8):
        out = tmp_path / f"r{la}.jsonl"
        r = subprocess.run([sys.executable, "src/distributed_inference.py"], cwd=ROOT,
                           env=_env(MXLLM_MAX_NEW_TOKENS=3, MXLLM_MAX_SEQ=256, MXLLM_GATHER_RESULTS=1,
                                    MXLLM_N_ROWS=40, MXLLM_EPOCHS=2, MXLLM_LOOKAHEAD_BATCHES=la,
                                    MXLLM_RESULTS_FILE=str(out)), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        log = r.stdout + r.stderr
        assert log.count("Prompt: ") == 80 and "An error occurred" not in log
        recs[la] = [json.loads(x) for x in out.read_text().splitlines()]
    assert recs[0] == recs[8]


def test_two_node_emulation_finetune():
    """BASELINE config 5 (CPU rehearsal): two torchrun agents = two 'nodes'."""
    port = _port()
    env = _env(NPROC_PER_NODE=1, NNODES=2, MASTER_PORT=port, MASTER_ADDR="127.0.0.1")
    args = ["--steps", "3", "--seq-len", "32", "--micro-batch", "1", "--log-every", "1"]
    p1 = subprocess.Popen(["bash", "scripts/run_node1.sh"] + args, cwd=ROOT, env=env, stdout=subprocess.PIPE,
                          stderr=subprocess.STDOUT, text=True)
    p0 = subprocess.run(["bash", "scripts/run_node0.sh"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                        timeout=300)
    out1, _ = p1.communicate(timeout=120)
    assert p0.returncode == 0 and p1.returncode == 0, p0.stderr[-2000:] + out1[-2000:]
    assert "step 2" in p0.stdout + p0.stderr


@pytest.mark.parametrize("parallel", ["zero3", "zero1"])
def test_two_node_emulation_sharded(parallel):
    """BASELINE config 5 with sharding (CPU rehearsal): two torchrun agents x 2
    ranks each = world 4 across two 'nodes', full fine-tune with ZeRO-3 (sharded
    params/grads/optimizer, activation checkpointing) or ZeRO-1."""
    port = _port()
    env = _env(NPROC_PER_NODE=2, NNODES=2, MASTER_PORT=port, MASTER_ADDR="127.0.0.1")
    args = ["--steps", "3", "--seq-len", "32", "--micro-batch", "1", "--log-every", "1", "--finetune", "full",
            "--parallel", parallel] + (["--activation-checkpointing", "1"] if parallel == "zero3" else [])
    p1 = subprocess.Popen(["bash", "scripts/run_node1.sh"] + args, cwd=ROOT, env=env, stdout=subprocess.PIPE,
                          stderr=subprocess.STDOUT, text=True)
    p0 = subprocess.run(["bash", "scripts/run_node0.sh"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                        timeout=300)
    out1, _ = p1.communicate(timeout=120)
    log = p0.stdout + p0.stderr
    assert p0.returncode == 0 and p1.returncode == 0, log[-2000:] + out1[-2000:]
    assert "step 2" in log


def test_fault_injection_fails_fast():
    """A rank that dies mid-run must take the job down (non-zero exit), not hang."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(_port()), "src/distributed_finetuning.py", "--steps", "6",
                        "--seq-len", "32", "--micro-batch", "1"], cwd=ROOT,
                       env=_env(MXLLM_FAULT_RANK=1, MXLLM_FAULT_STEP=2, MXLLM_FAULT_KIND="exit",
                                MXLLM_PG_TIMEOUT_S=60), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0


@pytest.mark.parametrize("parallel", ["ddp", "zero1"])
def test_fault_restart_resumes_from_checkpoint(tmp_path, parallel):
    """--max-restarts 1 + checkpoints: the restarted job resumes and finishes
    (ZeRO-1: every rank restores its own optimizer shard)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--max-restarts", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "src/distributed_finetuning.py",
                        "--steps", "6", "--seq-len", "32", "--micro-batch", "1", "--save-every", "2", "--ckpt-dir",
                        str(tmp_path), "--parallel", parallel], cwd=ROOT,
                       env=_env(MXLLM_FAULT_RANK=0, MXLLM_FAULT_STEP=3, MXLLM_FAULT_KIND="raise",
                                MXLLM_PG_TIMEOUT_S=60), capture_output=True, text=True, timeout=400)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-3000:]
    assert "Resumed at step 2" in log
    assert open(os.path.join(tmp_path, "latest")).read().strip() == "6"
