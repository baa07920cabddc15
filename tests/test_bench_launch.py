"""bench.py launch contract on CPU (gloo):

* ``--gpus N`` without a torchrun environment spawns N ranks itself and
  reports ``n_gpus: N`` (one JSON line on stdout);
* under torchrun, WORLD_SIZE != --gpus exits 1 before touching any device;
* the config-4 phase (ZeRO-3 full fine-tune in a fresh child job) is reported
  inside the SAME JSON line;
* the ZeRO-3 world-N emulation proxy is labelled as such.
Reference launch contract: /root/reference/scripts/run_node0.sh:10-16.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None, timeout=400):
    e = dict(os.environ if env is None else env)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        if env is None:
            e.pop(k, None)
    return subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--model", "tiny", "--steps", "2",
                           "--warmup", "1", "--seq-len", "64", *args], cwd=ROOT, env=e, capture_output=True,
                          text=True, timeout=timeout)


def _json_lines(stdout):
    return [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]


def test_self_launch_two_ranks():
    r = _bench("--gpus", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2" and j["value"] > 0
    assert j["config"]["global_batch"] == 4


def test_world_size_mismatch_exits_1():
    env = dict(os.environ, WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    r = _bench("--gpus", "2", env=env, timeout=120)
    assert r.returncode == 1
    assert "WORLD_SIZE=4" in r.stderr
    assert not _json_lines(r.stdout)


def test_config4_phase_in_same_line():
    r = _bench("--gpus", "2", "--config4", "on", "--config4-model", "tiny", "--config4-steps", "1",
               "--config4-warmup", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    c4 = j["config4_full_zero3"]
    assert "error" not in c4, c4
    assert c4["config"]["parallelism"] == "zero3-dp2" and c4["config"]["activation_checkpointing"]
    assert c4["n_gpus"] == 2 and c4["value"] > 0 and "config 4" in c4["label"]
    assert j["config"]["parallelism"] == "dp2"  # the headline itself is unchanged


def test_config3_zero1_variant_in_same_line():
    """Config 3 runs as plain DDP and, after it, as the same step with the optimizer sharded
    (ZeRO-1); both child results land in the one line."""
    r = _bench("--gpus", "2", "--config3", "on", "--config3-zero1", "on", "--full-model", "tiny", "--full-steps", "1",
               "--full-warmup", "1", "--config4", "off")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    c3, c3z = j["config3_8b_full_dp2"], j["config3_8b_full_dp2_zero1"]
    for c in (c3, c3z):
        assert "error" not in c and "skipped" not in c, c
        assert c["n_gpus"] == 2 and c["value"] > 0 and "config 3" in c["label"]
    assert "zero1" not in c3["config"]["parallelism"] and "zero1" in c3z["config"]["parallelism"]
    assert "ZeRO-1" in c3z["label"]


def test_zero3_emulation_is_labelled():
    r = _bench("--finetune", "full", "--parallel", "zero3", "--act-ckpt", "--emulate-world", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_lines(r.stdout)[0]
    assert j["emulated_world"] == 4 and "EMULATED" in j["config"]["parallelism"] and "PROXY" in j["note"]


def test_world8_rehearsal_with_config3_and_config4():
    """CPU rehearsal of the driver's 8-GPU run: ``bench.py --gpus 8`` self-launches 8
    gloo ranks; after the headline the in-process config-3 (full fine-tune, DDP over
    all 8 ranks) and the config-4 child job (ZeRO-3 over 8 ranks) report inside the
    ONE JSON line, labelled with the model that actually ran."""
    import time

    t0 = time.time()
    r = _bench("--gpus", "8", "--config3", "on", "--full-model", "tiny", "--full-steps", "1", "--full-warmup", "1",
               "--config4", "on", "--config4-model", "tiny", "--config4-steps", "1", "--config4-warmup", "1",
               timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert time.time() - t0 < 180
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    assert j["n_gpus"] == 8 and j["config"]["parallelism"] == "dp8"
    c3 = j["config3_8b_full_dp8"]
    assert "error" not in c3, c3
    assert c3["n_gpus"] == 8 and c3["config"]["finetune"].startswith("full") and "config 3" in c3["label"]
    c4 = j["config4_full_zero3"]
    assert "error" not in c4, c4
    assert c4["config"]["parallelism"] == "zero3-dp8" and c4["config"]["grad_reduce_dtype"] == "fp32"
    assert "tiny" in c4["label"] and "70B" not in c4["label"]


def test_memory_guard_checkpoints_only_when_short(monkeypatch):
    """At world > 1 the 70B headline checkpoints just enough layers when the smallest free HBM
    over the ranks is below the world-1 reserved peak + the RCCL allowance; never otherwise."""
    sys.path.insert(0, ROOT)
    import types

    import torch

    import bench
    from mxllm.parallel import runtime

    env = types.SimpleNamespace(device=torch.device("cuda", 0), world_size=8)
    need = bench.RESERVED_GB[("llama3.1-70b", "lora", 2, 2048)][0] + bench.RCCL_ALLOWANCE_GB
    for free, expect in ((need + 5.0, None), (need - 10.0, 10)):
        monkeypatch.setattr(torch.cuda, "mem_get_info", lambda d, f=free: (int(f * 1e9), int(309.2e9)))
        monkeypatch.setattr(runtime, "all_reduce_scalars", lambda xs, op="sum": list(xs))
        a = bench.parse([])
        g = bench.memory_guard(a, env)
        if expect is None:
            assert g is None and not a.act_ckpt
        else:
            assert g["checkpointed_layers"] >= 10 * 1 / 1.7 and a.act_ckpt and a.act_ckpt_layers == g["checkpointed_layers"]
    a = bench.parse([])
    assert bench.memory_guard(a, types.SimpleNamespace(device=torch.device("cuda", 0), world_size=1)) is None


def test_config4_plan_fits_free_hbm(monkeypatch):
    """The config-4 child checkpoints the fewest layers whose modelled per-rank peak + margin fits
    the smallest free HBM over the ranks; an explicit depth is honoured or skipped."""
    import argparse

    import bench

    a = argparse.Namespace(config4_act_ckpt_layers=None)
    assert bench.config4_plan(a, 308.0)[0] == 0
    assert bench.config4_plan(a, 268.0)[0] == 24
    assert bench.config4_plan(a, 200.0)[0] == 80
    assert bench.config4_plan(a, 150.0)[0] is None
    assert bench.config4_plan(a, None)[0] == 0  # CPU rehearsal: no HBM to check
    a.config4_act_ckpt_layers = 24
    assert bench.config4_plan(a, 308.0)[0] == 24 and bench.config4_plan(a, 250.0)[0] is None
    a.config4_act_ckpt_layers = None  # only m recomputed: 237.8 GB at 40, +1.56 per layer fewer
    monkeypatch.setenv("MXLLM_RECOMPUTE_NORM", "0")
    assert bench.config4_plan(a, 308.0)[0] == 8 and bench.config4_plan(a, 268.0)[0] == 32
    monkeypatch.setenv("MXLLM_RECOMPUTE_SWIGLU", "0")  # nothing recomputed: the round-3 HBM model
    assert bench.config4_plan(a, 308.0)[0] == 24 and bench.config4_plan(a, 262.0)[0] == 48


def test_config4_failed_child_is_retried_deeper(monkeypatch):
    """A failed config-4 child (the one real 8-rank measurement) is rerun with 40 layers
    checkpointed, then with every layer, and the failed attempts are recorded; an explicit depth
    is not second-guessed."""
    import argparse

    import bench

    calls = []
    fails = [1]

    def fake(a, world, ck):
        calls.append(ck)
        return {"error": "child job exit code 1"} if len(calls) <= fails[0] else {"ms_per_step": 1.0}

    monkeypatch.setattr(bench, "run_config4", fake)
    a = argparse.Namespace(config4_act_ckpt_layers=None, config4_timeout=360.0, time_budget_s=1e9, child_min_s=90.0)
    r = bench.run_config4_planned(a, 8, 308.0)
    assert calls == [0, 40] and r["ms_per_step"] == 1.0
    assert r["hbm_plan"]["checkpointed_layers"] == 40 and r["hbm_plan"]["first_attempt"]["checkpointed_layers"] == 0
    calls.clear()
    fails[0] = 2
    r = bench.run_config4_planned(a, 8, 308.0)
    assert calls == [0, 40, 80] and r["hbm_plan"]["checkpointed_layers"] == 80
    assert [f["checkpointed_layers"] for f in r["hbm_plan"]["failed_attempts"]] == [0, 40]
    calls.clear()
    fails[0] = 1
    a.config4_act_ckpt_layers = 56
    r = bench.run_config4_planned(a, 8, 308.0)
    assert calls == [56] and "error" in r
    # no budget left for a retry: the failed first attempt is reported, the retry skipped
    calls.clear()
    a.config4_act_ckpt_layers, a.time_budget_s = None, 0.0
    r = bench.run_config4_planned(a, 8, 308.0)
    assert calls == [0] and "error" in r and "time budget" in r["retry_skipped"]


def test_world8_hung_config4_child_keeps_headline_inside_budget():
    """the first 8-GPU driver run must not be lost to a slow child.  A
    config-4 child forced to hang (MXLLM_BENCH_CHILD_FAULT=config4:hang) is killed at the
    remaining budget, its retry is skipped for lack of budget, and rank 0 still prints exactly
    ONE JSON line with the headline, inside --time-budget-s."""
    import time

    budget = 150.0
    env = dict(os.environ, MXLLM_BENCH_CHILD_FAULT="config4:hang")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    r = _bench("--gpus", "8", "--config3", "off", "--config4", "on", "--config4-model", "tiny",
               "--config4-steps", "1", "--config4-warmup", "1", "--time-budget-s", str(budget),
               "--child-min-s", "20", env=env, timeout=300)
    wall = time.time() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    assert wall < budget + 10, wall
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout[-2000:]
    j = lines[0]
    assert j["n_gpus"] == 8 and j["value"] > 0 and j["config"]["parallelism"] == "dp8"
    c4 = j["config4_full_zero3"]
    assert "error" in c4 and "124" in c4["error"], c4
    assert "retry_skipped" in c4 and "time budget" in c4["retry_skipped"], c4


def test_child_phases_skipped_when_budget_is_spent():
    """With no budget left after the headline, the child phases are not started at all."""
    r = _bench("--gpus", "2", "--config4", "on", "--config4-model", "tiny", "--time-budget-s", "1",
               "--child-min-s", "5")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    assert "time budget" in lines[0]["config4_full_zero3"]["skipped"]


def test_sigterm_during_child_phase_prints_headline():
    """The driver's lease expiring (SIGTERM to bench.py) while a child job runs: the headline
    line is printed once, the child tree is killed, exit code 0."""
    import signal
    import time

    import psutil

    env = dict(os.environ, MXLLM_BENCH_CHILD_FAULT="config4:hang")
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    # world 1 (no torchrun parent): the bench process itself runs the headline, then the child
    p = subprocess.Popen([sys.executable, "bench.py", "--device", "cpu", "--model", "tiny", "--steps", "2",
                          "--warmup", "1", "--seq-len", "64", "--gpus", "1", "--config4", "on",
                          "--config4-model", "tiny", "--child-min-s", "5"],
                         cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        t_end = time.time() + 240
        seen = False
        while time.time() < t_end and p.poll() is None and not seen:
            try:
                kids = psutil.Process(p.pid).children(recursive=True)
                seen = any("zero3" in " ".join(k.cmdline()) for k in kids)
            except psutil.Error:
                pass
            time.sleep(0.5)
        assert seen, "the config-4 child job never started"
        time.sleep(3)
        kids = psutil.Process(p.pid).children(recursive=True)
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=60)
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, err[-3000:]
    lines = _json_lines(out)
    assert len(lines) == 1
    j = lines[0]
    assert j["value"] > 0 and "interrupted" in j and j["config4_full_zero3"] == {"skipped": "not reached"}
    _, alive = psutil.wait_procs(kids, timeout=30)
    assert not alive, [k.pid for k in alive]
