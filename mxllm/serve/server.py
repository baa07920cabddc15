"""OpenAI-compatible HTTP server backed by the mxllm engine.

Endpoints: POST /v1/chat/completions, POST /v1/completions (both with
optional SSE streaming), GET /v1/models, GET /health, GET /metrics
(Prometheus text).  This is the local stand-in for the "LiteLLM-compatible
API endpoint" hosting Llama-3.1-70B that the reference calls remotely
(reference README.md:18, docs/setup_guide.md:10).

Run:  python -m mxllm.serve.server --model llama3.1-8b --port 8000
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import time
import uuid

import torch
from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

from .engine import Engine, SamplingParams

log = logging.getLogger("mxllm.server")


def _stop_ids(tok, stop):
    if not stop:
        return ()
    if isinstance(stop, str):
        stop = [stop]
    ids = []
    for s in stop:
        enc = tok.encode(s, bos=False)
        if len(enc) == 1:
            ids.append(enc[0])
    return tuple(ids)


def build_app(engine: Engine, tokenizer, model_name: str, api_key: str | None = None):
    app = FastAPI(title="mxllm OpenAI-compatible server")
    engine.start()
    stats = {"requests": 0, "errors": 0, "prompt_tokens": 0, "completion_tokens": 0}

    def auth(req: Request):
        if api_key:
            h = req.headers.get("authorization", "")
            if h != f"Bearer {api_key}":
                raise HTTPException(status_code=401, detail="invalid api key")

    async def run(prompt_ids, body):
        params = SamplingParams(
            max_new_tokens=int(body.get("max_tokens") or body.get("max_completion_tokens") or 128),
            temperature=float(body.get("temperature", 0.0) or 0.0),
            top_p=float(body.get("top_p", 1.0) or 1.0),
            top_k=int(body.get("top_k", 0) or 0),
            stop_ids=_stop_ids(tokenizer, body.get("stop")),
            seed=int(body.get("seed", 0) or 0),
        )
        r = engine.submit(prompt_ids, params)
        while not r.done.is_set():
            await asyncio.sleep(0.002)
        if r.error:
            stats["errors"] += 1
            raise HTTPException(status_code=500, detail=r.error)
        stats["prompt_tokens"] += len(prompt_ids)
        stats["completion_tokens"] += len(r.output)
        return r

    def usage(r):
        return {"prompt_tokens": len(r.prompt), "completion_tokens": len(r.output),
                "total_tokens": len(r.prompt) + len(r.output)}

    @app.get("/health")
    async def health():
        return {"status": "ok", "model": model_name, "active": len(engine.active), "waiting": len(engine.waiting)}

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "owned_by": "mxllm"}]}

    @app.get("/metrics")
    async def metrics():
        lines = [f"mxllm_requests_total {stats['requests']}", f"mxllm_errors_total {stats['errors']}",
                 f"mxllm_prompt_tokens_total {stats['prompt_tokens']}",
                 f"mxllm_completion_tokens_total {stats['completion_tokens']}",
                 f"mxllm_engine_steps_total {engine.steps}", f"mxllm_active_sequences {len(engine.active)}",
                 f"mxllm_waiting_requests {len(engine.waiting)}",
                 f"mxllm_ttft_seconds_sum {engine.ttft_sum:.6f}", f"mxllm_ttft_seconds_count {engine.finished}",
                 f"mxllm_request_latency_seconds_sum {engine.latency_sum:.6f}",
                 f"mxllm_request_latency_seconds_count {engine.finished}",
                 f"mxllm_prefill_tokens_total {engine.prefill_tokens}",
                 f"mxllm_prefill_seconds_total {engine.prefill_s:.6f}",
                 f"mxllm_decode_tokens_total {engine.decode_tokens}",
                 f"mxllm_decode_seconds_total {engine.decode_s:.6f}"]
        return PlainTextResponse("\n".join(lines) + "\n")

    @app.post("/v1/chat/completions")
    @app.post("/chat/completions")
    async def chat(req: Request):
        auth(req)
        body = await req.json()
        stats["requests"] += 1
        msgs = body.get("messages") or []
        ids = tokenizer.apply_chat_template(msgs)
        if body.get("stream"):
            return StreamingResponse(_stream(ids, body, chat=True), media_type="text/event-stream")
        r = await run(ids, body)
        text = tokenizer.decode([t for t in r.output if t not in engine.eos_ids])
        return JSONResponse({
            "id": f"chatcmpl-{uuid.uuid4().hex[:24]}", "object": "chat.completion", "created": int(time.time()),
            "model": body.get("model", model_name),
            "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                         "finish_reason": r.finish_reason}],
            "usage": usage(r)})

    @app.post("/v1/completions")
    @app.post("/completions")
    async def completions(req: Request):
        auth(req)
        body = await req.json()
        stats["requests"] += 1
        prompt = body.get("prompt", "")
        ids = tokenizer.encode(prompt if isinstance(prompt, str) else prompt[0])
        if body.get("stream"):
            return StreamingResponse(_stream(ids, body, chat=False), media_type="text/event-stream")
        r = await run(ids, body)
        text = tokenizer.decode([t for t in r.output if t not in engine.eos_ids])
        return JSONResponse({
            "id": f"cmpl-{uuid.uuid4().hex[:24]}", "object": "text_completion", "created": int(time.time()),
            "model": body.get("model", model_name),
            "choices": [{"index": 0, "text": text, "finish_reason": r.finish_reason}], "usage": usage(r)})

    @app.post("/v1/embeddings")
    @app.post("/embeddings")
    async def embeddings(req: Request):
        """OpenAI embeddings: ``input`` a string, a list of strings, a token list or a
        list of token lists; mean-pooled final hidden states, unit norm."""
        auth(req)
        body = await req.json()
        stats["requests"] += 1
        inp = body.get("input", "")
        if inp == "" or inp == [] or (isinstance(inp, list) and any(x == "" or x == [] for x in inp)):
            return JSONResponse({"error": {"message": "empty input", "type": "invalid_request_error"}},
                                status_code=400)
        if isinstance(inp, str):
            seqs = [tokenizer.encode(inp)]
        elif inp and all(isinstance(x, int) for x in inp):
            seqs = [list(inp)]
        else:
            seqs = [tokenizer.encode(x) if isinstance(x, str) else list(x) for x in inp]
        if not seqs or any(not q for q in seqs):
            return JSONResponse({"error": {"message": "empty input", "type": "invalid_request_error"}},
                                status_code=400)
        try:
            vec = await asyncio.get_running_loop().run_in_executor(None, engine.embed, seqs)
        except (ValueError, NotImplementedError) as e:
            return JSONResponse({"error": {"message": str(e), "type": "invalid_request_error"}}, status_code=400)
        n = sum(len(q) for q in seqs)
        return JSONResponse({
            "object": "list", "model": body.get("model", model_name),
            "data": [{"object": "embedding", "index": i, "embedding": v.tolist()} for i, v in enumerate(vec)],
            "usage": {"prompt_tokens": n, "total_tokens": n}})

    async def _stream(ids, body, chat: bool):
        r = engine.submit(ids, SamplingParams(
            max_new_tokens=int(body.get("max_tokens") or body.get("max_completion_tokens") or 128),
            temperature=float(body.get("temperature", 0.0) or 0.0), top_p=float(body.get("top_p", 1.0) or 1.0),
            top_k=int(body.get("top_k", 0) or 0), stop_ids=_stop_ids(tokenizer, body.get("stop")),
            seed=int(body.get("seed", 0) or 0)))
        sent = 0
        cid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        while True:
            done = r.done.is_set()
            toks = r.output[sent:]
            if toks:
                sent += len(toks)
                text = tokenizer.decode([t for t in toks if t not in engine.eos_ids])
                if chat:
                    chunk = {"id": cid, "object": "chat.completion.chunk", "model": model_name,
                             "choices": [{"index": 0, "delta": {"content": text}, "finish_reason": None}]}
                else:
                    chunk = {"id": cid, "object": "text_completion", "model": model_name,
                             "choices": [{"index": 0, "text": text, "finish_reason": None}]}
                yield f"data: {json.dumps(chunk)}\n\n"
            if done and sent >= len(r.output):
                break
            await asyncio.sleep(0.005)
        fin = {"id": cid, "object": "chat.completion.chunk" if chat else "text_completion", "model": model_name,
               "choices": [{"index": 0, ("delta" if chat else "text"): ({} if chat else ""),
                            "finish_reason": r.finish_reason}]}
        yield f"data: {json.dumps(fin)}\n\n"
        yield "data: [DONE]\n\n"

    @app.on_event("shutdown")
    async def _shutdown():
        engine.stop()

    return app


def build_default(model: str = "tiny", device: str | None = None, max_batch: int = 8, max_seq: int = 2048,
                  checkpoint: str | None = None, tokenizer_path: str | None = None, seed: int = 0,
                  weights: str = "bf16", tp_group=None):
    """Engine + tokenizer.  ``tp_group``: this rank serves its tensor-parallel
    shard (mxllm/parallel/tensor.py) of the model; the full model is built (or
    loaded) on the rank's GPU, sliced and freed."""
    from ..data.tokenizer import get_tokenizer
    from ..models import build_model, tokenizer_path_for

    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    # ``model``: a preset name or a Hugging Face Llama directory (its weights and tokenizer.json)
    m = build_model(model, device=device, seed=seed)
    cfg = m.cfg
    tokenizer_path = tokenizer_path_for(model, tokenizer_path)
    if checkpoint:
        from ..train.checkpoint import load_model_weights

        load_model_weights(m, checkpoint)
    m.eval()
    if tp_group is not None:
        import torch.distributed as dist

        from ..parallel.tensor import shard_llama

        m = shard_llama(m, dist.get_rank(tp_group), dist.get_world_size(tp_group))
        if str(device).startswith("cuda"):
            torch.cuda.empty_cache()
    if weights == "fp8":
        from .quant import quantize_model_fp8_

        quantize_model_fp8_(m)
    tok = get_tokenizer(cfg.vocab_size, tokenizer_path, cfg.bos_id, cfg.eos_id)
    eng = Engine(m, max_batch=max_batch, max_seq=max_seq, eos_ids=(cfg.eos_id, getattr(tok, "eos_id", cfg.eos_id)),
                 tp_group=tp_group)
    return eng, tok


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default=os.environ.get("MXLLM_MODEL", "tiny"),
                    help="preset name, or a Hugging Face Llama directory (config.json + safetensors + tokenizer.json)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--max-batch", type=int, default=8)
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--tokenizer", default=None)
    ap.add_argument("--api-key", default=os.environ.get("MXLLM_API_KEY"))
    ap.add_argument("--served-name", default=None)
    ap.add_argument("--weights", choices=["bf16", "fp8"], default=os.environ.get("MXLLM_ENGINE_WEIGHTS", "bf16"),
                    help="fp8: e4m3 projection weights (serving quantisation, mxllm/serve/quant.py)")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree: launch with torchrun --nproc-per-node=TP; rank 0 serves HTTP, "
                         "the other ranks follow its schedule")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    group, env = None, None
    if a.tp > 1:
        import torch.distributed as dist

        from ..parallel import runtime

        env = runtime.init()
        if env.world_size != a.tp:
            raise SystemExit(f"--tp {a.tp} needs exactly {a.tp} ranks (torchrun --nproc-per-node={a.tp})")
        group = dist.group.WORLD
    eng, tok = build_default(a.model, None, a.max_batch, a.max_seq, a.checkpoint, a.tokenizer, weights=a.weights,
                             tp_group=group)
    if group is not None:
        eng.enable_tp_sync()
        if env.rank != 0:
            try:
                eng.follow()
            finally:
                runtime.cleanup()
            return
    app = build_app(eng, tok, a.served_name or os.path.basename(os.path.normpath(a.model)), a.api_key)
    import uvicorn

    try:
        uvicorn.run(app, host=a.host, port=a.port, log_level="warning")
    finally:
        if group is not None:
            eng.stop()
            runtime.cleanup()


if __name__ == "__main__":
    main()
