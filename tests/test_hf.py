"""Hugging Face Llama checkpoints (mxllm/models/hf.py) against the transformers
implementation of Llama: a model loaded from an HF directory must produce the
same logits as ``transformers.LlamaForCausalLM`` on the same weights, and an
exported mxllm model (LoRA merged) must load back into transformers unchanged.
Reference contract: the reference's model is named by CONFIG MODEL_NAME
(/root/reference/src/config.py) and called through LiteLLM
(/root/reference/src/distributed_inference.py:37); a local replacement has to
take real checkpoints."""
import json
import os
import subprocess
import sys

import pytest
import torch

transformers = pytest.importorskip("transformers")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLAMA3_ROPE = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
               "original_max_position_embeddings": 8192}


def _hf_model(path, *, rope_scaling=LLAMA3_ROPE, tie=False, layers=2, seed=0):
    from transformers import LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=layers,
                      num_attention_heads=8, num_key_value_heads=2, max_position_embeddings=131072,
                      rope_theta=500000.0, rope_scaling=rope_scaling, rms_norm_eps=1e-5, tie_word_embeddings=tie,
                      bos_token_id=256, eos_token_id=257)
    torch.manual_seed(seed)
    m = LlamaForCausalLM(cfg).float().eval()
    m.save_pretrained(path, safe_serialization=True)
    return m


@pytest.mark.parametrize("rope_scaling,tie", [(LLAMA3_ROPE, False), (None, False), (LLAMA3_ROPE, True)])
def test_load_matches_transformers(tmp_path, rope_scaling, tie):
    from mxllm.models import load_hf_llama

    ref = _hf_model(tmp_path, rope_scaling=rope_scaling, tie=tie)
    m = load_hf_llama(str(tmp_path), dtype=torch.float32)
    assert m.cfg.tie_embeddings == tie and (m.cfg.rope_scaling is None) == (rope_scaling is None)
    ids = torch.randint(0, 512, (2, 200), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        a = ref(ids).logits
        b = m(ids).float()
    torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-4)


def test_export_lora_merged_loads_in_transformers(tmp_path):
    """mxllm LoRA model (non-zero B) -> save_hf_llama (merged, forced into several
    shards + index) -> transformers and load_hf_llama both reproduce its logits."""
    from transformers import LlamaForCausalLM

    from mxllm.models import load_hf_llama, save_hf_llama

    src = tmp_path / "src"
    _hf_model(src)
    m = load_hf_llama(str(src), dtype=torch.float32, lora_r=8, lora_alpha=16.0)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for layer in m.layers:
            for lin in (layer.wqkv, layer.wo, layer.wgu, layer.wd):
                lin.lora_b.copy_(torch.randn(lin.lora_b.shape, generator=g) * 0.05)
        m.sync_adapters_()
    out = tmp_path / "out"
    files = save_hf_llama(m, str(out), max_shard_bytes=1 << 20)
    assert len(files) > 1 and (out / "model.safetensors.index.json").exists()
    ids = torch.randint(0, 512, (1, 64), generator=g)
    with torch.no_grad():
        want = m(ids).float()
        got_hf = LlamaForCausalLM.from_pretrained(str(out)).float().eval()(ids).logits
        got_mx = load_hf_llama(str(out), dtype=torch.float32)(ids).float()
    torch.testing.assert_close(got_hf, want, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(got_mx, want, rtol=1e-4, atol=1e-4)


def test_strict_loading(tmp_path):
    from safetensors.torch import load_file, save_file

    from mxllm.models import load_hf_llama

    _hf_model(tmp_path)
    sd = load_file(str(tmp_path / "model.safetensors"))
    sd.pop("model.layers.1.mlp.up_proj.weight")
    save_file(sd, str(tmp_path / "model.safetensors"), metadata={"format": "pt"})
    with pytest.raises(KeyError, match="up_proj"):
        load_hf_llama(str(tmp_path), dtype=torch.float32)
    cfg = json.loads((tmp_path / "config.json").read_text())
    cfg["model_type"] = "mistral"
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    with pytest.raises(ValueError):
        load_hf_llama(str(tmp_path), dtype=torch.float32)


def test_zero3_initialises_from_hf(tmp_path):
    """ZeRO-3 materialises each unit from the checkpoint (no rank holds the whole
    model): the gathered state equals the HF tensors."""
    from safetensors.torch import load_file

    from mxllm.models import load_hf_config
    from mxllm.models.hf import hf_state_from_mx
    from mxllm.parallel.runtime import DistEnv
    from mxllm.parallel.zero3 import Zero3Trainer

    _hf_model(tmp_path)
    cfg = load_hf_config(str(tmp_path))
    env = DistEnv(0, 1, 0, 1, 0, "gloo", torch.device("cpu"))
    tr = Zero3Trainer(cfg, env, init_from=str(tmp_path))
    got = hf_state_from_mx(tr.full_state_dict(), cfg)
    want = load_file(str(tmp_path / "model.safetensors"))
    assert set(got) == set(want)
    for k, v in want.items():
        torch.testing.assert_close(got[k].float(), v.to(torch.bfloat16).float(), rtol=0, atol=0, msg=k)


@pytest.mark.parametrize("parallel", ["ddp", "zero3"])
def test_finetune_driver_from_hf_and_export(tmp_path, parallel):
    """src/distributed_finetuning.py --model <HF dir> --save-hf on 2 gloo ranks.
    DDP + LoRA (lr 1e-2): the merged export loads in transformers and moved away from
    the start.  ZeRO-3 full fine-tune at lr 0: each rank materialises its shards from
    the checkpoint and the unit-by-unit export reproduces the checkpoint exactly."""
    from safetensors.torch import load_file
    from transformers import LlamaForCausalLM

    from mxllm.models.hf import _shard_files

    src, out = tmp_path / "src", tmp_path / "out"
    ref = _hf_model(src)
    env = dict(os.environ, PYTHONPATH=ROOT, MXLLM_PG_TIMEOUT_S="120")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    args = (["--finetune", "lora", "--lora-r", "8", "--lr", "1e-2"] if parallel == "ddp" else
            ["--finetune", "full", "--parallel", "zero3", "--lr", "0"])
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                        "127.0.0.1", "--master-port", str(port), "src/distributed_finetuning.py", "--model", str(src),
                        "--steps", "3", "--seq-len", "32", "--micro-batch", "1", "--log-every", "1",
                        "--save-hf", str(out)] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    m = LlamaForCausalLM.from_pretrained(str(out)).float().eval()
    ids = torch.randint(0, 512, (1, 16))
    with torch.no_grad():
        a, b = ref(ids).logits, m(ids).logits
    assert torch.isfinite(b).all()
    if parallel == "ddp":
        assert (a - b).abs().max() > 1e-4
    else:
        want = load_file(str(src / "model.safetensors"))
        got = {}
        for fn in _shard_files(str(out)):
            got.update(load_file(fn))
        assert set(got) == set(want)
        for k, v in want.items():
            assert torch.equal(got[k], v.to(torch.bfloat16)), k


def test_server_builds_from_hf_dir(tmp_path):
    from mxllm.serve.server import build_default

    _hf_model(tmp_path, layers=1)
    eng, tok = build_default(str(tmp_path), device="cpu", max_batch=2, max_seq=128)
    out = eng.generate([tok.encode("hello")], max_new_tokens=4)
    assert len(out[0]) == 4


def test_export_cli_from_checkpoint_equals_driver_export(tmp_path):
    """``python -m mxllm export-hf`` rebuilds the merged model from the base checkpoint and the
    adapters a LoRA run saved, identical to the run's own --save-hf export."""
    from safetensors.torch import load_file

    src, a_out, b_out, ck = tmp_path / "src", tmp_path / "a", tmp_path / "b", tmp_path / "ck"
    _hf_model(src)
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "src/distributed_finetuning.py", "--model", str(src), "--finetune", "lora",
                        "--lora-r", "8", "--lora-alpha", "16", "--lr", "1e-2", "--steps", "2", "--seq-len", "32",
                        "--micro-batch", "1", "--save-every", "2", "--ckpt-dir", str(ck), "--save-hf", str(a_out)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([sys.executable, "-m", "mxllm", "export-hf", "--base", str(src), "--weights",
                        str(ck / "step_2"), "--lora-r", "8", "--lora-alpha", "16", "--out", str(b_out)],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    a, b = load_file(str(a_out / "model.safetensors")), load_file(str(b_out / "model.safetensors"))
    assert set(a) == set(b)
    for k in a:
        assert torch.equal(a[k], b[k]), k
