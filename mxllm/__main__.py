"""``python -m mxllm <command>`` (also the ``mxllm`` console script).

  serve      OpenAI-compatible server (mxllm.serve.server; same flags)
  build      compile the gfx950 native library (mxllm._build; same flags)
  export-hf  a trained model as a Hugging Face Llama directory: base weights (a preset with
             its seed, or an HF directory) + the weights an mxllm run saved (a checkpoint
             step directory's model.safetensors: LoRA adapters, or full weights), LoRA merged
  info       native library provenance, devices, tuned-table status
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def _export_hf(argv) -> int:
    ap = argparse.ArgumentParser(prog="mxllm export-hf")
    ap.add_argument("--base", required=True, help="preset name (random init with --seed) or Hugging Face directory")
    ap.add_argument("--weights", default="", help="mxllm checkpoint step directory or a .safetensors of named weights")
    ap.add_argument("--lora-r", type=int, default=0, help="LoRA rank the run trained with (0 = full weights)")
    ap.add_argument("--lora-alpha", type=float, default=32.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-shard-gb", type=float, default=5.0)
    a = ap.parse_args(argv)
    import torch

    from .models import build_model, save_hf_llama
    from .train.checkpoint import load_model_weights

    model = build_model(a.base, device="cpu", dtype=torch.bfloat16, lora_r=a.lora_r, lora_alpha=a.lora_alpha,
                        seed=a.seed)
    if a.weights:
        load_model_weights(model, a.weights)  # step dir (DDP / ZeRO-1 / ZeRO-3) or .safetensors
    files = save_hf_llama(model, a.out, max_shard_bytes=int(a.max_shard_gb * (1 << 30)))
    print(json.dumps({"out": a.out, "files": [os.path.basename(f) for f in files]}))
    return 0


def _info(argv) -> int:
    import torch

    out = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
           "devices": [torch.cuda.get_device_name(i) for i in range(torch.cuda.device_count())]
           if torch.cuda.is_available() else []}
    here = os.path.dirname(os.path.abspath(__file__))
    bi = os.path.join(here, "_C.buildinfo.json")
    if os.path.exists(bi):
        with open(bi) as f:
            out["native_build"] = json.load(f)
    out["native_library"] = os.path.exists(os.path.join(here, "_C.so"))
    out["gemm_table"] = os.path.exists(os.path.join(here, "tuning", "tunableop_gfx950.csv"))
    print(json.dumps(out, indent=1))
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "serve":
        from .serve.server import main as serve_main

        serve_main(rest)
        return 0
    if cmd == "build":
        from ._build import main as build_main

        return build_main(rest) or 0
    if cmd == "export-hf":
        return _export_hf(rest)
    if cmd == "info":
        return _info(rest)
    print(f"unknown command {cmd!r}\n{__doc__}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
