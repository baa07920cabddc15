#!/usr/bin/env python3
"""mxllm headline benchmark: fine-tune tokens/sec (whole node), Llama-3.1-70B DDP.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
it is launched by torchrun, one rank per GPU over RCCL.  W untimed warm-up
steps, then EXACTLY K timed optimizer steps bracketed by barrier +
device synchronize, wall time MAX over ranks; rank 0 prints ONE JSON line.

Workload (BASELINE.json metric/config): Llama-3.1-70B architecture (80 layers,
h 8192, 64/8 heads, ffn 28672, vocab 128256), random-init bf16 weights
created on device, synthetic token batches of seq_len 2048.  Each GPU holds a
FULL 141 GB bf16 replica of the model (288 GB HBM3E per MI355X) and the
fine-tune is LoRA (r=16 on q,k,v,o,gate,up,down; frozen base), so plain
data-parallel DDP runs at every N from 1 to 8 — weak scaling, per-GPU micro
batch fixed.  Every timed step is a complete step: forward through all 80
layers, fused LM-head + CE over the 128k vocab, full backward (activation
gradients through every layer + adapter gradients), bucketed RCCL all-reduce
of the adapter gradients, grad-norm clip and fused AdamW.

``--finetune full`` (e.g. with ``--model llama3.1-8b``) trains every weight
(bf16 params/grads, fp32 master + Adam moments) — BASELINE config 2/3.

BASELINE config 4 (Llama-3.1-70B FULL-parameter fine-tune, sharded over 8
GPUs): ``--finetune full --parallel zero3 --act-ckpt``.  When the headline run
is on 8 GPUs (``--config4 auto``) it is ALSO measured after the headline steps,
in a fresh 8-rank child job, and reported under ``config4_full_zero3`` in the
same JSON line.  ``--emulate-world N`` runs ZeRO-3 in one process with world-N
shard sizes (per-rank memory/compute proxy without link traffic).

``--gpus N`` without a torchrun environment spawns the N ranks itself (child
``torch.distributed.run``, rendezvous on 127.0.0.1); under torchrun a
WORLD_SIZE different from N is an error (exit 1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "fine-tune tokens/sec (whole node) Llama-3.1-70B DDP at 1/2/4/8 MI355X"
PRETTY = {"llama3.1-70b": "Llama-3.1-70B", "llama3.1-8b": "Llama-3.1-8B", "llama3.2-1b": "Llama-3.2-1B",
          "tiny": "tiny", "tiny-d128": "tiny-d128"}


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama3.1-70b")
    ap.add_argument("--finetune", choices=["lora", "full"], default="lora")
    ap.add_argument("--parallel", choices=["ddp", "zero1", "zero3"], default="ddp",
                    help="zero1 = DDP with a sharded optimizer (reduce-scatter / all-gather); "
                         "zero3 = sharded params/grads/optimizer (full fine-tuning of 70B on 8 GPUs)")
    ap.add_argument("--lora-r", type=int, default=16)
    ap.add_argument("--lora-alpha", type=float, default=32.0)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--act-ckpt", action="store_true", help="activation checkpointing per layer")
    ap.add_argument("--act-ckpt-layers", type=int, default=None,
                    help="with --act-ckpt: checkpoint only the first N layers (the rest keep activations)")
    ap.add_argument("--sp", type=int, default=1,
                    help="sequence-parallel degree (Ulysses all-to-all around attention; long-context runs)")
    ap.add_argument("--cp", type=int, default=1,
                    help="context-parallel degree (ring attention, zigzag sequence layout; long-context runs)")
    ap.add_argument("--bucket-mb", type=float, default=128.0)
    ap.add_argument("--device", default=None, help="force 'cpu' for a plumbing run")
    ap.add_argument("--layers", type=int, default=None, help="override n_layers (NOT valid for the headline)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--no-gemm-table", action="store_true", help="ignore the tuned hipBLASLt solution table")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="zero3 only: one process holding world-N shard sizes (gathers tile the local shard)")
    ap.add_argument("--config4", choices=["auto", "on", "off"], default="auto",
                    help="also measure BASELINE config 4 (70B full fine-tune, ZeRO-3) after the headline; "
                         "auto = when the headline runs on 8 GPUs")
    ap.add_argument("--config4-micro-batch", type=int, default=4)
    # selective checkpointing of the first N of 80 layers (the rest keep their activations).  Emulated
    # world-8 per-rank step, one box (archive/profiles/r4g/c4_ck*.json): N = 56 3,298 ms / 223.5 GB reserved;
    # 40: 3,141 ms / 255.2 GB; 24: 2,990 ms / 286.9 GB (~2 GB per checkpointed layer).  Default: the
    # fewest checkpointed layers (>= 40) whose reserved peak + CONFIG4_MARGIN_GB fits the smallest free
    # HBM over the ranks (config4_plan).
    ap.add_argument("--config4-act-ckpt-layers", type=int, default=None)
    ap.add_argument("--config4-model", default="llama3.1-70b", help=argparse.SUPPRESS)  # tests: tiny models
    ap.add_argument("--config4-steps", type=int, default=3)
    ap.add_argument("--config4-warmup", type=int, default=2)
    ap.add_argument("--config4-timeout", type=float, default=360.0,
                    help="hard limit for the config-4 child job; the headline line is printed either way")
    ap.add_argument("--config2", choices=["auto", "on", "off"], default="auto",
                    help="also measure BASELINE config 2 (Llama-3.1-8B FULL fine-tune, DDP) in-process after "
                         "the headline; auto = when the headline runs on 1 GPU")
    ap.add_argument("--config3", choices=["auto", "on", "off"], default="auto",
                    help="also measure BASELINE config 3 (Llama-3.1-8B FULL fine-tune, DDP over all N GPUs) "
                         "in-process after the headline; auto = when the headline runs on 8 GPUs")
    ap.add_argument("--config3-zero1", choices=["auto", "on", "off"], default="auto",
                    help="with config 3: ALSO measure it with the optimizer sharded (ZeRO-1: reduce-scatter, "
                         "AdamW on 1/N of the state, all-gather), after config 4 and only if the time budget "
                         "is left; auto = on GPUs")
    ap.add_argument("--config3-peer", choices=["auto", "on", "off"], default="auto",
                    help="with config 3: ALSO measure it with the gradient buckets all-reduced by mxllm's own peer-memory "
                         "collectives (MXLLM_COMM=peer, light schedule) instead of RCCL -- last, only if the time "
                         "budget is left; auto = on GPUs")
    ap.add_argument("--config3-timeout", type=float, default=300.0,
                    help="hard limit for the config-3 child job; the headline line is printed either way")
    ap.add_argument("--config2-mb4", choices=["auto", "on", "off"], default="auto",
                    help="with config 2: also measure it at micro-batch 4 (the reference's batch of 4)")
    ap.add_argument("--no-calibrate", dest="calibrate", action="store_false",
                    help="skip the box calibration (8192^3 bf16 GEMM TF/s, 4 GiB copy TB/s) after the timed steps")
    ap.add_argument("--full-model", default="llama3.1-8b", help=argparse.SUPPRESS)  # tests: tiny models
    ap.add_argument("--full-steps", type=int, default=10)
    ap.add_argument("--full-warmup", type=int, default=3)
    ap.add_argument("--grad-dtype", choices=["auto", "bf16", "fp32"], default="auto",
                    help="gradient accumulation / reduction dtype; auto = fp32 for zero3, bf16 otherwise")
    ap.add_argument("--time-budget-s", type=float, default=float(os.environ.get("MXLLM_BENCH_BUDGET_S", "540")),
                    help="wall-clock budget of the WHOLE command from process start (the driver's lease is "
                         "600 s): every phase after the headline gets min(its limit, what is left - "
                         f"{EMIT_MARGIN_S:.0f} s) and is skipped when that is below --child-min-s; the one JSON "
                         "line is always printed")
    ap.add_argument("--child-min-s", type=float, default=90.0,
                    help="a phase after the headline (config 2/3/4, a config-4 retry) starts only with at least "
                         "this much budget left")
    return ap.parse_args(argv)


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


_T0 = time.time()  # process start: the --time-budget-s clock
EMIT_MARGIN_S = 30.0  # kept back from every child job: killing a hung one (<= 20 s), the emit, the exit
_STATE = {"out": None, "emitted": False, "json_out": None, "child": None}


def remaining_s(a) -> float:
    """Seconds left of this process's ``--time-budget-s``."""
    return a.time_budget_s - (time.time() - _T0)


def _kill_tree(p, grace_s: float = 20.0) -> None:
    """SIGTERM the child's process group AND every descendant (torchrun starts each
    worker in a session of its own, so the group alone misses them), SIGKILL what is
    left after ``grace_s``."""
    import signal
    import subprocess

    import psutil

    try:
        kids = psutil.Process(p.pid).children(recursive=True)
    except psutil.Error:
        kids = []
    for fn in (lambda: os.killpg(p.pid, signal.SIGTERM), *[(lambda k=k: k.terminate()) for k in kids]):
        try:
            fn()
        except (OSError, psutil.Error):
            pass
    try:
        p.wait(timeout=grace_s)
    except subprocess.TimeoutExpired:
        pass
    _, alive = psutil.wait_procs(kids, timeout=max(1.0, grace_s / 4))
    for k in alive:
        try:
            k.kill()
        except psutil.Error:
            pass
    try:
        os.killpg(p.pid, signal.SIGKILL)
    except OSError:
        pass
    p.wait()


def launch_ranks(nproc: int, argv: list[str], script: str | None = None, timeout_s: float | None = None,
                 env: dict | None = None) -> int:
    """Run ``script argv`` as ``nproc`` torchrun ranks in a CHILD process group
    (one rank per GPU, rendezvous on 127.0.0.1) and relay its stdout.

    The parent never touches the GPU (``import torch`` does not initialise HIP)
    and never re-execs itself: it waits for the child and returns its exit code
    (124 when ``timeout_s`` expired: the whole tree is killed).  The stdout relay
    runs on a thread, so a child that hangs WITHOUT printing still times out.
    Reference contract: /root/reference/scripts/run_node0.sh:10-16 (torchrun,
    one process per device)."""
    import subprocess
    import threading

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script or os.path.abspath(__file__)]
    p = subprocess.Popen(cmd + list(argv), stdout=subprocess.PIPE, text=True, start_new_session=True,
                         env=env if env is not None else os.environ.copy())
    _STATE["child"] = p
    out = sys.stdout  # bound now: the caller may redirect stdout around this call

    def pump():
        for line in p.stdout:
            out.write(line)
            out.flush()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    try:
        rc = p.wait(timeout=timeout_s)
        t.join(timeout=5)
        return rc
    except (KeyboardInterrupt, subprocess.TimeoutExpired):
        _kill_tree(p, grace_s=15.0)
        return 124
    finally:
        _STATE["child"] = None


def check_world(gpus: int) -> str:
    """'launch' (no torchrun env and N > 1: spawn N ranks), 'run' (env matches
    or single process) or 'mismatch' (torchrun WORLD_SIZE != --gpus)."""
    ws = os.environ.get("WORLD_SIZE")
    if ws in (None, ""):
        return "launch" if gpus > 1 else "run"
    return "run" if int(ws) == gpus else "mismatch"


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    mode = check_world(a.gpus)
    if mode == "mismatch":
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks",
              file=sys.stderr, flush=True)
        return 1
    if mode == "launch":
        return launch_ranks(a.gpus, argv)
    if a.device == "cpu":
        os.environ["MXLLM_FORCE_CPU"] = "1"
    from mxllm.parallel import runtime

    # the timed step issues no small collectives, so the bench keeps RCCL for its
    # two bookkeeping reductions (MXLLM_XGMI=1 opts into the peer-memory path)
    os.environ.setdefault("MXLLM_XGMI", "0")
    env = runtime.init()
    out = run(a, env)
    if env.is_main:
        # from here on the headline is never lost: a SIGTERM (the driver's lease expiring) prints
        # whatever has been measured, and every later phase runs inside try/finally + the budget
        _arm_emit_on_signal(out, a.json_out)
    cuda = env.device.type == "cuda"
    headline = a.model == "llama3.1-70b" and a.finetune == "lora" and a.parallel == "ddp" and not a.layers
    c2 = a.config2 == "on" or (a.config2 == "auto" and env.world_size == 1 and headline and cuda)
    c3 = a.config3 == "on" or (a.config3 == "auto" and env.world_size == 8 and headline and cuda)
    c4 = a.config4 == "on" or (a.config4 == "auto" and env.world_size == 8 and headline and cuda)
    children = []
    if c3 and env.world_size > 1:
        children.append(("config3", f"config3_8b_full_dp{env.world_size}"))
    if c4:
        children.append(("config4", "config4_full_zero3"))
    if c3 and env.world_size > 1 and (a.config3_zero1 == "on" or (a.config3_zero1 == "auto" and cuda)):
        # the same DDP fine-tune with the optimizer sharded: after config 4, so it never costs it its budget
        children.append(("config3z", f"config3_8b_full_dp{env.world_size}_zero1"))
    if c3 and env.world_size > 1 and (a.config3_peer == "on" or (a.config3_peer == "auto" and cuda)):
        # the same DDP fine-tune over mxllm's own peer-memory collectives: last of all
        children.append(("config3p", f"config3_8b_full_dp{env.world_size}_peer"))
    try:
        if cuda and a.calibrate:
            # box speed next to the number: fixed GEMM + copy after the timed steps
            from mxllm.utils.calibrate import calibrate

            _free_gpu_memory(env)
            try:
                out["calibration"] = calibrate(env.device)
            except Exception as e:  # noqa: BLE001
                out["calibration"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        if c2 and env.world_size == 1:
            # single process: an exception (e.g. out of memory) is caught and recorded, nothing can strand
            for key, mb in (("config2_8b_full", None), ("config2_8b_full_mb4", 4)):
                if mb is not None and not (a.config2_mb4 == "on" or (a.config2_mb4 == "auto" and cuda)):
                    continue  # mb 4: the reference's batch of 4 (/root/reference/src/distributed_inference.py:59)
                if remaining_s(a) < a.child_min_s + EMIT_MARGIN_S:
                    out[key] = {"skipped": f"time budget: {remaining_s(a):.0f} s of --time-budget-s "
                                           f"{a.time_budget_s:.0f} left"}
                    continue
                out[key] = run_full(a, env, micro_batch=mb)
        if not children:
            return 0
        # Multi-rank phases run as FRESH child jobs (an exception on one rank of an in-process
        # DDP phase would strand the others in a collective): this job's ranks free their HBM, report the
        # smallest free HBM and their PIDs, non-zero ranks exit, and local rank 0 confirms every other
        # rank's process has exited (its HBM released) before it starts a child.
        _free_gpu_memory(env)
        free_gb = _min_free_gb(env)
        import socket

        pids = runtime.all_gather_objects((socket.gethostname(), os.getpid()))
        runtime.cleanup()
        if not env.is_main:
            return 0
        host = socket.gethostname()
        released = _wait_exited([p for h, p in pids if h == host and p != os.getpid()],
                                timeout_s=min(120.0, max(1.0, remaining_s(a) - EMIT_MARGIN_S)))
        out["child_phases"] = {"headline_ranks_exited_s": released, "min_free_hbm_gb_before": (
            round(free_gb, 1) if free_gb is not None else None), "time_budget_s": a.time_budget_s}
        for kind, key in children:
            out[key] = {"skipped": "not reached"}  # replaced below; what a SIGTERM emit reports
        for kind, key in children:
            try:
                if kind == "config4":
                    out[key] = run_config4_planned(a, env.world_size, free_gb)
                else:
                    out[key] = run_config3(a, env.world_size, "zero1" if kind == "config3z" else "ddp",
                                           comm="peer" if kind == "config3p" else None)
            except Exception as e:  # noqa: BLE001  the headline (and later phases) survive any phase error
                out[key] = {"error": f"{type(e).__name__}: {e}"[:500]}
        out["child_phases"]["elapsed_s"] = round(time.time() - _T0, 1)
        return 0
    finally:
        if env.is_main:
            _emit_once()
        runtime.cleanup()


def _arm_emit_on_signal(out: dict, json_out: str | None) -> None:
    """Register ``out`` as THE result line; SIGTERM/SIGINT/SIGHUP print it (once), stop a
    running child job and exit 0 — a lease that expires during the child phases still gets
    the headline."""
    import signal

    _STATE.update(out=out, json_out=json_out, emitted=False)

    def on_signal(signum, frame):  # noqa: ARG001
        out.setdefault("interrupted", f"signal {signum} after {time.time() - _T0:.0f} s; later phases not run")
        _emit_once()
        p = _STATE.get("child")
        if p is not None and p.poll() is None:
            _kill_tree(p, grace_s=5.0)
        os._exit(0)

    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        try:
            signal.signal(s, on_signal)
        except (ValueError, OSError):  # not the main thread (tests calling main() from a thread)
            pass


def _emit_once() -> None:
    if _STATE["out"] is not None and not _STATE["emitted"]:
        _STATE["emitted"] = True
        emit(_STATE["out"], _STATE["json_out"])


def _wait_exited(pids: list[int], timeout_s: float) -> float | None:
    """Seconds until every PID in ``pids`` has exited (same node), None on timeout.  A PID
    that exits between the checks (NoSuchProcess) counts as exited."""
    import psutil

    def alive(p: int) -> bool:
        try:
            return psutil.Process(p).status() != psutil.STATUS_ZOMBIE
        except (psutil.NoSuchProcess, psutil.ZombieProcess):
            return False
        except psutil.Error:
            return psutil.pid_exists(p)

    t0 = time.time()
    while time.time() - t0 < timeout_s:
        if not any(alive(p) for p in pids):
            return round(time.time() - t0, 2)
        time.sleep(0.1)
    return None


def _free_gpu_memory(env):
    import gc

    gc.collect()
    if env.device.type == "cuda":
        torch.cuda.synchronize(env.device)
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats(env.device)  # the next run's peak_hbm_gb is its own


def _min_free_gb(env) -> float | None:
    """Smallest free HBM over the ranks (GB) after this job released its caches."""
    from mxllm.parallel import runtime

    if env.device.type != "cuda":
        return None
    free = torch.cuda.mem_get_info(env.device)[0] / 1e9
    return runtime.all_reduce_scalars([free], op="min")[0]


def run_full(a, env, micro_batch: int | None = None) -> dict:
    """BASELINE config 2 (1 GPU) / config 3 (N GPUs): Llama-3.1-8B FULL-parameter
    fine-tune with plain DDP, in this process after the headline (whose model and
    caches are released first).  Same timing contract as the headline.  A failure
    is recorded in the returned dict; the headline line is printed either way."""
    import copy

    _free_gpu_memory(env)
    b = copy.copy(a)
    b.model, b.finetune, b.parallel = a.full_model, "full", "ddp"
    b.steps, b.warmup, b.layers = a.full_steps, a.full_warmup, None
    b.act_ckpt, b.act_ckpt_layers, b.sp, b.cp, b.emulate_world = False, None, 1, 1, 0
    b.grad_accum = 1
    if micro_batch is not None:
        b.micro_batch = micro_batch
    try:
        res = run(b, env)
    except Exception as e:  # noqa: BLE001  (e.g. out of memory): report, keep the headline
        res = {"error": f"{type(e).__name__}: {e}"[:500]}
    _free_gpu_memory(env)
    res.pop("vs_baseline", None)
    cfg = b.model
    res["metric"] = f"fine-tune tokens/sec (whole node) {PRETTY.get(cfg, cfg)} FULL-parameter DDP"
    res["label"] = (f"BASELINE config {2 if env.world_size == 1 else 3}: {PRETTY.get(cfg, cfg)} full-parameter "
                    f"fine-tune, DDP over {env.world_size} GPU(s), micro-batch {b.micro_batch}, measured "
                    f"in-process after the headline")
    return res


_STDOUT = sys.stdout  # the real stdout: a child phase redirects sys.stdout while it runs


def emit(out: dict, json_out: str | None):
    line = json.dumps(out)
    print(line, file=_STDOUT, flush=True)
    if json_out:
        with open(json_out, "w") as f:
            f.write(line + "\n")


def child_timeout(a, limit_s: float) -> float | None:
    """The time a child phase may take: ``min(limit_s, budget left - EMIT_MARGIN_S)``, or
    None when that is below ``--child-min-s`` (the phase is skipped)."""
    t = min(limit_s, remaining_s(a) - EMIT_MARGIN_S)
    return t if t >= a.child_min_s else None


def _budget_skip(a) -> dict:
    return {"skipped": f"time budget: {max(0.0, remaining_s(a)):.0f} s of --time-budget-s {a.time_budget_s:.0f} "
                       f"left (a phase needs --child-min-s {a.child_min_s:.0f} + {EMIT_MARGIN_S:.0f})"}


def _run_child(a, world: int, argv: list[str], timeout_s: float, tag: str = "", extra_env: dict | None = None) -> dict:
    """Run bench.py ``argv`` as a fresh ``world``-rank torchrun child job (rendezvous on
    127.0.0.1) and return its parsed JSON line (or the error).  ``timeout_s`` is capped by
    the remaining ``--time-budget-s``; below ``--child-min-s`` the job is not started.
    ``MXLLM_BENCH_CHILD_FAULT=<tag>:<kind>`` injects ``kind`` (hang | exit | raise) into rank 0
    of the child tagged ``tag`` at its first timed step (budget drills)."""
    import contextlib
    import io
    import tempfile

    if (a.device != "cpu" and torch.cuda.device_count() < world
            and os.environ.get("MXLLM_BENCH_SHARED_GPU", "0") != "1"):
        # MXLLM_BENCH_SHARED_GPU=1 (rehearsals on a 1-GPU box, with MXLLM_BACKEND=gloo MXLLM_COMM=peer):
        # the child's ranks share the visible GPU(s) (runtime.pick_device: local_rank % device_count)
        return {"skipped": f"this process sees {torch.cuda.device_count()} GPU(s), the child job needs {world}"}
    limit = child_timeout(a, timeout_s)
    if limit is None:
        return _budget_skip(a)
    fd, path = tempfile.mkstemp(suffix=".json", prefix="mxllm_child_")
    os.close(fd)
    argv = ["--gpus", str(world)] + argv + ["--config2", "off", "--config3", "off", "--config4", "off",
                                            "--no-calibrate", "--json-out", path] + (
        ["--device", a.device] if a.device else [])
    keep = {k: v for k, v in os.environ.items()
            if not (k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                          "ROLE_WORLD_SIZE", "ROLE_NAME", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
                    or k.startswith("TORCHELASTIC_") or k.startswith("TORCH_ELASTIC"))}
    fault = os.environ.get("MXLLM_BENCH_CHILD_FAULT", "")
    if fault and tag and fault.split(":")[0] == tag:
        keep.update(MXLLM_FAULT_KIND=fault.split(":", 1)[1], MXLLM_FAULT_RANK="0", MXLLM_FAULT_STEP="0")
    keep.pop("MXLLM_BENCH_CHILD_FAULT", None)
    keep.update(extra_env or {})
    t0 = time.time()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):  # the child's own JSON line must not become a second output line
        rc = launch_ranks(world, argv, timeout_s=limit, env=keep)
    res = {"error": f"child job exit code {rc}" + (f" (killed at its {limit:.0f} s limit)" if rc == 124 else ""),
           "wall_s": round(time.time() - t0, 1)}
    try:
        with open(path) as f:
            txt = f.read().strip()
        if txt:
            res = json.loads(txt)
            res["wall_s"] = round(time.time() - t0, 1)
    except (OSError, ValueError) as e:
        res["error"] = f"{res.get('error')}; no result ({e})"
    finally:
        with contextlib.suppress(OSError):
            os.remove(path)
    res.pop("vs_baseline", None)
    return res


def run_config3(a, world: int, parallel: str = "ddp", comm: str | None = None) -> dict:
    """BASELINE config 3: Llama-3.1-8B FULL fine-tune, DDP over ``world`` GPUs, as a fresh child
    job after the headline.  ``parallel`` = "zero1": the same data-parallel step with the
    optimizer sharded (mxllm/parallel/zero1.py: the buckets are reduce-scattered, each rank runs
    AdamW over its 1/N of the fp32 state, the bf16 parameters are all-gathered back under the
    next forward) -- the same link bytes as the all-reduce, 1/N of the ~38 ms AdamW per rank."""
    argv = ["--model", a.full_model, "--finetune", "full", "--parallel", parallel, "--micro-batch",
            str(a.micro_batch), "--seq-len", str(a.seq_len), "--steps", str(a.full_steps), "--warmup",
            str(a.full_warmup)]
    tag = "config3p" if comm == "peer" else ("config3" if parallel == "ddp" else "config3z")
    res = _run_child(a, world, argv, a.config3_timeout, tag=tag,
                     extra_env={"MXLLM_COMM": "peer"} if comm == "peer" else None)
    name = PRETTY.get(a.full_model, a.full_model)
    how = "DDP" if parallel == "ddp" else "DDP with a ZeRO-1 sharded optimizer"
    if comm == "peer":
        how += " over mxllm's peer-memory collectives (MXLLM_COMM=peer)"
    res["metric"] = f"fine-tune tokens/sec (whole node) {name} FULL-parameter {how}"
    res["label"] = (f"BASELINE config 3: {name} full-parameter fine-tune, {how} over {world} GPUs, "
                    f"measured after the headline in a separate job")
    return res


# config 4 per-rank HBM model (70B, micro-batch 4 x 2048, world-8 shards): reserved peak = r0 GB with
# the first n0 layers checkpointed, +per GB for each layer fewer.  The un-checkpointed layers
# recompute m = swiglu(gu) (MXLLM_RECOMPUTE_SWIGLU) and the normed qkv / gate-up inputs
# (MXLLM_RECOMPUTE_NORM) in the backward by default: 258.2 / 268.4 / 278.6 GB at 16 / 8 / 0
# (archive/profiles/r4_recompute/pass_u_*.json); m only: 237.8 GB at 40, +1.52 per layer (pass R);
# nothing recomputed: archive/profiles/r4g/c4_ck*.json.  Margin: RCCL buffers of the two ZeRO-3
# communicators + allocator slack of the real 8-rank job
CONFIG4_RESERVED = (16, 258.2, 1.30)
CONFIG4_RESERVED_M_ONLY = (40, 237.8, 1.56)
CONFIG4_RESERVED_SAVED_M = (56, 223.5, 1.98)
CONFIG4_MARGIN_GB = 14.0
CONFIG4_DEPTHS = (0, 8, 16, 24, 32, 40, 48, 56, 64, 80)


def config4_plan(a, free_gb: float | None) -> tuple[int | None, float]:
    """(checkpointed layers, HBM needed) for the config-4 child: ``--config4-act-ckpt-layers``
    when given, else the fewest of CONFIG4_DEPTHS that fit ``free_gb``; (None, need of 80) when
    even full checkpointing does not fit."""
    if os.environ.get("MXLLM_RECOMPUTE_SWIGLU", "auto") == "0":
        n0, r0, per = CONFIG4_RESERVED_SAVED_M
    elif os.environ.get("MXLLM_RECOMPUTE_NORM", "auto") == "0":
        n0, r0, per = CONFIG4_RESERVED_M_ONLY
    else:
        n0, r0, per = CONFIG4_RESERVED
    need = lambda ck: r0 + (n0 - ck) * per + CONFIG4_MARGIN_GB  # noqa: E731
    if a.config4_act_ckpt_layers is not None:
        ck = a.config4_act_ckpt_layers
        return (ck if free_gb is None or free_gb >= need(ck) else None), need(ck)
    for ck in CONFIG4_DEPTHS:
        if free_gb is None or free_gb >= need(ck):
            return ck, need(ck)
    return None, need(80)


def run_config4_planned(a, world: int, free_gb: float | None) -> dict:
    """Config-4 child with the checkpoint depth from ``config4_plan``; a failed child (e.g. RCCL
    buffers beyond the HBM model) is rerun with 40 layers checkpointed (~50 GB more headroom than
    0), then with every layer -- insurance for the one real 8-rank measurement.  The plan (and the
    failed attempts) is recorded as ``hbm_plan``."""
    ck, need = config4_plan(a, free_gb)
    if ck is None:
        return {"skipped": f"min free HBM over the ranks {free_gb:.1f} GB < {need:.0f} GB the "
                           f"config-4 child needs with every layer checkpointed"}
    res = run_config4(a, world, ck)
    failed = []
    if a.config4_act_ckpt_layers is None:
        for retry in (40, 80):
            if "error" not in res or retry <= ck:
                continue
            if child_timeout(a, a.config4_timeout) is None:  # a retry only when the budget covers it
                res["retry_skipped"] = _budget_skip(a)["skipped"]
                break
            failed.append({"checkpointed_layers": ck, "error": res["error"]})
            ck = retry
            res = run_config4(a, world, ck)
    res["hbm_plan"] = {"min_free_hbm_gb": None if free_gb is None else round(free_gb, 1),
                       "need_gb": round(need, 1), "checkpointed_layers": ck}
    if failed:
        res["hbm_plan"]["first_attempt"] = failed[0]
        res["hbm_plan"]["failed_attempts"] = failed
    return res


def run_config4(a, world: int, ckpt_layers: int = 40) -> dict:
    """70B full-parameter ZeRO-3 fine-tune (activation checkpointing of the first
    ``ckpt_layers`` layers) on ``world`` GPUs as a child torchrun job; returns its parsed
    JSON (or the error)."""
    argv = ["--model", a.config4_model, "--finetune", "full", "--parallel", "zero3",
            "--act-ckpt", "--micro-batch", str(a.config4_micro_batch), "--seq-len", str(a.seq_len),
            "--act-ckpt-layers", str(ckpt_layers),
            "--steps", str(a.config4_steps), "--warmup", str(a.config4_warmup)]
    res = _run_child(a, world, argv, a.config4_timeout, tag="config4")
    name = PRETTY.get(a.config4_model, a.config4_model)
    res["label"] = (f"BASELINE config 4: {name} FULL-parameter fine-tune, ZeRO-3 sharded over "
                    f"{world} GPUs, activation checkpointing, measured after the headline in a separate job")
    return res


# peak HBM RESERVED by the caching allocator for a world-1 run of a configuration (driver record
# BENCH_r02.json / archive/profiles/r3h/bench_default.json), and the activation memory one checkpointed
# layer gives back (70B, 2 x 2048 tokens: ~150 GB of activations over 80 layers)
RESERVED_GB = {("llama3.1-70b", "lora", 2, 2048): (294.3, 1.7)}
RCCL_ALLOWANCE_GB = 3.0  # communicator buffers + DDP bucket slack at world > 1


def memory_guard(a, env) -> dict | None:
    """At world > 1 the headline runs beside RCCL's buffers with ~15 GB of HBM to spare at
    world 1.  If the smallest free HBM over the ranks is below the world-1 reserved peak plus
    an RCCL allowance, checkpoint just enough layers to fit (every rank takes the same decision
    from the all-reduced minimum) instead of risking an out-of-memory error mid-step, which
    would strand the other ranks in a collective.  Returns the record of that decision, or
    None when the configuration fits as is."""
    from mxllm.parallel import runtime

    key = (a.model, a.finetune, a.micro_batch, a.seq_len)
    if env.device.type != "cuda" or env.world_size == 1 or a.act_ckpt or a.layers or key not in RESERVED_GB:
        return None
    need, per_layer = RESERVED_GB[key]
    need += RCCL_ALLOWANCE_GB
    free = runtime.all_reduce_scalars([torch.cuda.mem_get_info(env.device)[0] / 1e9], op="min")[0]
    if free >= need:
        return None
    import math

    n = math.ceil((need - free) / per_layer) + 2
    a.act_ckpt, a.act_ckpt_layers = True, n
    return {"min_free_hbm_gb": round(free, 1), "need_gb": round(need, 1), "checkpointed_layers": n}


def _gemm_desc(tuned: bool) -> str:
    """Which GEMM implementations the step may use (mxllm/ops/gemm.py dispatch)."""
    from mxllm.ops import gemm

    lib = "hipBLASLt/rocBLAS" + (" (tuned solution table)" if tuned else "")
    if gemm.deterministic():
        return "gemm8 (hand-written MFMA HIP kernel) for every shape it takes, DETERMINISTIC mode; " + lib + " otherwise"
    pol = gemm._policy()
    if pol == "0":
        return lib
    if pol == "all":
        return "gemm8 (hand-written MFMA HIP kernel) wherever it takes the shape; " + lib + " otherwise"
    return f"{lib} + gemm8 (hand-written MFMA HIP kernel) on the {len(gemm._table())} measured-win shapes"


def run(a, env) -> dict:
    """Build the trainer, run W warm-up + K timed steps, return the JSON dict."""
    from mxllm.models import Llama, get_config
    from mxllm.parallel import runtime
    from mxllm.train.trainer import OptimConfig, Trainer
    from mxllm.data import SyntheticTokens

    dev = env.device
    from mxllm.utils import gemm_tuning

    tuned = gemm_tuning.enable() if not a.no_gemm_table else False
    guard = memory_guard(a, env)
    cfg = get_config(a.model)
    if a.layers:
        cfg = cfg.replace(n_layers=a.layers)
    torch.manual_seed(0)
    lora_r = a.lora_r if a.finetune == "lora" else 0
    t0 = time.perf_counter()
    opt = OptimConfig(lr=1e-4, weight_decay=0.0, grad_clip=1.0)
    emulated = 0
    ckpt = a.act_ckpt if (not a.act_ckpt or a.act_ckpt_layers is None) else a.act_ckpt_layers
    gd = a.grad_dtype if a.grad_dtype != "auto" else ("fp32" if a.parallel == "zero3" else "bf16")
    gdt = torch.float32 if gd == "fp32" else None
    if a.parallel == "zero3":
        if a.finetune != "full":
            raise SystemExit("--parallel zero3 requires --finetune full")
        from mxllm.parallel.zero3 import Zero3Trainer

        if a.emulate_world > 1:
            if env.world_size > 1:
                raise SystemExit("--emulate-world is a single-process proxy")
            emulated = a.emulate_world
        trainer = Zero3Trainer(cfg, env, opt, seed=1234, activation_checkpointing=ckpt,
                               emulate_world=emulated, grad_dtype=gdt)
        model = trainer.model
    else:
        model = Llama(cfg, device=dev, dtype=torch.bfloat16, lora_r=lora_r, lora_alpha=a.lora_alpha, seed=1234,
                      activation_checkpointing=ckpt)
        trainer = Trainer(model, env, opt, bucket_mb=a.bucket_mb, shard_optimizer=a.parallel == "zero1",
                          grad_dtype=gdt)
    sp_group, data_rank, shard_fn = None, env.rank, None
    if a.sp > 1 and a.cp > 1:
        raise SystemExit("--sp and --cp are alternatives")
    if a.sp > 1 or a.cp > 1:
        if a.parallel == "zero3":
            raise SystemExit("--sp / --cp are supported with --parallel ddp / zero1")
        from mxllm.parallel.sequence import new_groups, shard_sequence

        sp_group, data_rank, _ = new_groups(max(a.sp, a.cp))
        if a.cp > 1:
            from mxllm.parallel.context import zigzag_shard

            model.set_context_parallel(sp_group)
            shard_fn = zigzag_shard
        else:
            model.set_sequence_parallel(sp_group)
            shard_fn = shard_sequence
    data = SyntheticTokens(cfg.vocab_size, a.micro_batch, a.seq_len, dev, seed=1, rank=data_rank)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    init_s = time.perf_counter() - t0

    def step():
        mbs = [data.next() for _ in range(a.grad_accum)]
        if sp_group is not None:  # every rank of an SP/CP group gets the same sequences, keeps its slice
            mbs = [(shard_fn(i, sp_group), shard_fn(l, sp_group)) for i, l in mbs]
        return trainer.train_step(mbs)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    fault = None
    if os.environ.get("MXLLM_FAULT_KIND"):  # drills (MXLLM_BENCH_CHILD_FAULT): misbehave at a timed step
        import types

        from mxllm.utils.faults import maybe_inject

        fault = types.SimpleNamespace(fault_kind=os.environ["MXLLM_FAULT_KIND"],
                                      fault_rank=int(os.environ.get("MXLLM_FAULT_RANK", "0")),
                                      fault_step=int(os.environ.get("MXLLM_FAULT_STEP", "0")))
    loss = None
    for _ in range(a.warmup):
        loss = step()
    sync()
    runtime.barrier()
    sync()
    t_start = time.perf_counter()
    for i in range(a.steps):
        if fault is not None:
            maybe_inject(fault, env.rank, i)
        loss = step()
    sync()
    runtime.barrier()
    sync()
    elapsed = time.perf_counter() - t_start
    gpu_sample = {}
    if dev.type == "cuda" and os.environ.get("MXLLM_BENCH_SMI", "1") != "0":
        from mxllm.utils.gpumon import sample_device

        gpu_sample = sample_device(dev.index)  # clocks / power right after the timed steps
    elapsed = runtime.all_reduce_scalars([elapsed], op="max")[0]
    loss_v = float(loss.float().item()) if loss is not None else float("nan")
    world = emulated or env.world_size  # emulation: tokens of ONE rank of that world
    sq = max(a.sp, a.cp)
    tokens_per_step = a.micro_batch * a.seq_len * a.grad_accum * env.world_size // sq
    tps = tokens_per_step * a.steps / elapsed if a.steps else 0.0
    ms = 1e3 * elapsed / max(1, a.steps)
    peak_gb = torch.cuda.max_memory_allocated(dev) / 1e9 if dev.type == "cuda" else 0.0
    reserved_gb = torch.cuda.max_memory_reserved(dev) / 1e9 if dev.type == "cuda" else 0.0
    total_gb = torch.cuda.mem_get_info(dev)[1] / 1e9 if dev.type == "cuda" else 0.0
    flops_tok = cfg.train_flops_per_token(a.seq_len, lora=(a.finetune == "lora"))
    mfu = tps * flops_tok / (env.world_size * 2.5e15) if dev.type == "cuda" else 0.0
    if a.parallel == "zero3":
        par = f"zero3-dp{world}" + (" (EMULATED on 1 GPU: world-%d shard sizes, no link traffic)" % world
                                    if emulated else "")
    else:
        par = (f"dp{env.world_size // a.sp}-sp{a.sp}" if a.sp > 1 else
               f"dp{env.world_size // a.cp}-cp{a.cp}" if a.cp > 1 else f"dp{env.world_size}")
        if a.parallel == "zero1":
            par += "-zero1" if getattr(trainer, "zero1", None) is not None else " (zero1 requested: world 1 = ddp)"
    out = {
        "metric": METRIC,
        "value": round(tps, 2),
        "unit": "tokens/s",
        "n_gpus": env.world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (random token ids, random-init weights)",
        "config": {
            "model": PRETTY.get(cfg.name, cfg.name) + (f" ({cfg.n_layers} layers)" if a.layers else ""),
            "global_batch": a.micro_batch * a.grad_accum * env.world_size // sq,
            "seq_len": a.seq_len,
            "parallelism": par,
            "finetune": (f"lora r={lora_r} alpha={a.lora_alpha} on q,k,v,o,gate,up,down; frozen bf16 base"
                         if a.finetune == "lora" else "full (bf16 params+grads, fp32 master/Adam)"),
            "micro_batch": a.micro_batch,
            "grad_accum": a.grad_accum,
            "activation_checkpointing": (a.act_ckpt if a.act_ckpt_layers is None or not a.act_ckpt
                                         else f"first {a.act_ckpt_layers} of {cfg.n_layers} layers"),
            "optimizer": "fused AdamW (HIP), grad clip 1.0" + (
                ", per-layer updates overlapped with the next forward" if getattr(trainer, "overlap_optimizer", False)
                else ""),
            "grad_reduce_dtype": gd,
            "gemm": _gemm_desc(tuned),
        },
        "tokens_per_sec_per_gpu": round(tps / env.world_size, 2),
        "model_tflops_per_gpu": round(tps * flops_tok / env.world_size / 1e12, 1),
        "mfu_vs_2.5PF_dense": round(mfu, 4),
        "peak_hbm_gb": round(peak_gb, 1),
        "peak_hbm_reserved_gb": round(reserved_gb, 1),
        "hbm_total_gb": round(total_gb, 1),
        "init_s": round(init_s, 1),
        "final_loss": round(loss_v, 4),
        "grad_comm": (getattr(trainer.ddp.comm, "kind", None) if a.parallel != "zero3" and trainer.ddp.enabled
                      else None),
        "allreduce_mb_per_step": (round(trainer.ddp.bytes_per_step / 2 ** 20, 1)
                                  if a.parallel != "zero3" and trainer.ddp.enabled else 0.0),
        "exposed_comm_ms_last_step": (round(trainer.ddp.exposed_comm_ms(), 3)
                                      if a.parallel != "zero3" and trainer.ddp.enabled and a.steps
                                      and trainer.ddp.exposed_comm_ms() is not None else None),
        "gpu_after_timed_steps": {k: gpu_sample[k] for k in ("gfx_clock_mhz", "socket_power_w", "temp_hotspot_c")
                                  if k in gpu_sample},
        "trainable_params": (cfg.n_params() if a.parallel == "zero3" else model.num_params(trainable_only=True)),
    }
    if a.parallel == "zero3":
        # which communicator layout / optimizer schedule actually ran
        c = trainer.comm
        out["zero3"] = {
            "comms": ("split: all-gathers and reduce-scatters on two communicators" if c.real and c.rs_pg is not None
                      and c.rs_pg is not c.ag_pg else "single communicator" if c.real else "none (world 1 / emulated)"),
            "comm_backend": c.kind,
            "adamw": "per unit on a side stream, overlapped with the next forward" if trainer.overlap_optimizer
                     else "one launch after the backward",
            "rmsnorm_unit": "replicated (all-reduced gradient, no re-gather)",
            "max_inflight_reduce_scatters": trainer.max_inflight,
            "rs_wire": c.rs_wire,
        }
        steps_run = a.warmup + a.steps
        if steps_run and world > 1:
            # link bytes this rank sends per step (all-gathers bf16; reduce-scatters at the wire dtype)
            out["zero3"]["sent_gb_per_step"] = {k: round(v / steps_run / 1e9, 2) for k, v in c.sent_bytes.items()}
    if guard is not None:
        out["memory_guard"] = guard
    if emulated:
        out["emulated_world"] = emulated
        out["note"] = ("PROXY: one GPU holding one rank's world-%d shards; value/ms exclude all collective "
                       "time and are per emulated rank" % emulated)
    return out


if __name__ == "__main__":
    sys.exit(main() or 0)
