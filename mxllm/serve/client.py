"""LiteLLM-compatible ``completion(model, messages)`` client.

Mirrors the slice of the LiteLLM API the reference uses
(reference src/distributed_inference.py:7-8, 34-41, 53-54):
``completion(model, messages)`` returning an object with
``.choices[0].message.content``, and a module-level ``api_base``.
LiteLLM itself is not installed in this image, so this module
can stand in for it: ``from mxllm.serve import client as litellm``.

Routing:
  * ``api_base`` in (None, "", "local", "inproc") -> an in-process mxllm Engine
    registered with ``register_local(model, engine, tokenizer)``;
  * otherwise an OpenAI-compatible HTTP endpoint ``{api_base}/chat/completions``
    (an mxllm server or any OpenAI-compatible server), Bearer auth from
    ``api_key`` / ``OPENAI_API_KEY``.
Failures are retried with exponential backoff + full jitter and a per-request
timeout (the reference has neither — SURVEY D11 / A5).

Also the other LiteLLM entry points a caller of the reference is likely to
reach for: ``completion(..., stream=True)`` (an iterator of chunks with
``.choices[0].delta.content``; SSE from the server, token deltas from the local
engine), ``acompletion`` (awaitable; ``stream=True`` gives an async iterator)
and ``batch_completion`` (one in-process engine pass for many conversations).
"""
from __future__ import annotations

import logging
import os
import random
import time
from dataclasses import dataclass, field

log = logging.getLogger("mxllm.client")

api_base: str | None = None
api_key: str | None = None
request_timeout: float = 120.0
num_retries: int = 3

_LOCAL: dict[str, tuple] = {}


@dataclass
class Message:
    content: str
    role: str = "assistant"

    def __getitem__(self, k):
        return getattr(self, k)


@dataclass
class Choice:
    message: Message
    index: int = 0
    finish_reason: str | None = "stop"

    def __getitem__(self, k):
        return getattr(self, k)


@dataclass
class Delta:
    content: str | None = None
    role: str | None = None

    def __getitem__(self, k):
        return getattr(self, k)


@dataclass
class StreamChoice:
    delta: Delta
    index: int = 0
    finish_reason: str | None = None

    def __getitem__(self, k):
        return getattr(self, k)


@dataclass
class ModelResponse:
    choices: list
    model: str = ""
    usage: dict = field(default_factory=dict)
    id: str = ""

    def __getitem__(self, k):
        return getattr(self, k)


class CompletionError(RuntimeError):
    pass


def register_local(model: str, engine, tokenizer) -> None:
    """Serve ``model`` from an in-process Engine (no HTTP)."""
    _LOCAL[model] = (engine, tokenizer)


def unregister_local(model: str | None = None) -> None:
    if model is None:
        _LOCAL.clear()
    else:
        _LOCAL.pop(model, None)


def _local_engine(model: str):
    """The in-process (engine, tokenizer) for ``model``: its own registration, or the only
    one registered; anything else is an error (never a silent pick among several)."""
    if model in _LOCAL:
        return _LOCAL[model]
    if len(_LOCAL) == 1:
        return next(iter(_LOCAL.values()))
    raise CompletionError(f"no local engine registered for model {model!r}")


def _local(model, messages, max_tokens, temperature, **kw) -> ModelResponse:
    eng, tok = _local_engine(model)
    ids = tok.apply_chat_template(messages)
    out = eng.generate([ids], max_new_tokens=max_tokens, temperature=temperature,
                       top_p=kw.get("top_p", 1.0), seed=kw.get("seed", 0))[0]
    text = tok.decode([t for t in out if t not in eng.eos_ids])
    return ModelResponse([Choice(Message(text))], model=model,
                         usage={"prompt_tokens": len(ids), "completion_tokens": len(out)})


def batch_local(model: str, prompts: list[str], max_tokens: int = 32, temperature: float = 0.0) -> list[str]:
    """Batched in-process generation for a list of user prompts (one engine pass)."""
    eng, tok = _local_engine(model)
    ids = [tok.apply_chat_template([{"role": "user", "content": p}]) for p in prompts]
    outs = eng.generate(ids, max_new_tokens=max_tokens, temperature=temperature)
    return [tok.decode([t for t in o if t not in eng.eos_ids]) for o in outs]


def submit_local(model: str, prompts: list[str], max_tokens: int = 32, temperature: float = 0.0) -> list:
    """Queue user prompts on the in-process engine WITHOUT waiting (the engine's
    background loop batches them with everything else in flight); returns
    request handles for ``collect_local``."""
    from .engine import SamplingParams

    eng, tok = _local_engine(model)
    eng.start()
    ids = [tok.apply_chat_template([{"role": "user", "content": p}]) for p in prompts]
    return [eng.submit(i, SamplingParams(max_new_tokens=max_tokens, temperature=temperature)) for i in ids]


def collect_local(model: str, requests: list, timeout: float | None = None) -> list[str]:
    """Wait for requests from ``submit_local`` and detokenize (raises on an engine error)."""
    eng, tok = _local_engine(model)
    out = []
    for r in requests:
        if not r.done.wait(timeout):
            raise CompletionError("local engine request timed out")
        if r.error:
            raise CompletionError(f"local engine: {r.error}")
        out.append(tok.decode([t for t in r.output if t not in eng.eos_ids]))
    return out


def _http(model, messages, base, key, timeout, max_tokens, temperature, **kw) -> ModelResponse:
    import httpx

    url = base.rstrip("/")
    if not url.endswith("/chat/completions"):
        url += "/chat/completions"
    headers = {"Content-Type": "application/json"}
    if key:
        headers["Authorization"] = f"Bearer {key}"
    body = {"model": model, "messages": messages, "max_tokens": max_tokens, "temperature": temperature}
    body.update({k: v for k, v in kw.items() if k in ("top_p", "stop", "seed", "top_k")})
    r = httpx.post(url, json=body, headers=headers, timeout=timeout)
    if r.status_code == 429 or r.status_code >= 500:
        raise _Retryable(f"HTTP {r.status_code}: {r.text[:200]}")
    if r.status_code != 200:
        raise CompletionError(f"HTTP {r.status_code}: {r.text[:200]}")
    j = r.json()
    ch = [Choice(Message(c["message"]["content"], c["message"].get("role", "assistant")), c.get("index", i),
                 c.get("finish_reason")) for i, c in enumerate(j["choices"])]
    return ModelResponse(ch, model=j.get("model", model), usage=j.get("usage", {}), id=j.get("id", ""))


class _Retryable(Exception):
    pass


def _is_local(base) -> bool:
    return base in (None, "", "local", "inproc") or str(base).startswith("local://")


def _local_stream(model, messages, max_tokens, temperature, **kw):
    """Token deltas from the in-process engine's background loop as they are produced."""
    from .engine import SamplingParams

    eng, tok = _local_engine(model)
    eng.start()
    ids = tok.apply_chat_template(messages)
    r = eng.submit(ids, SamplingParams(max_new_tokens=max_tokens, temperature=temperature,
                                       top_p=kw.get("top_p", 1.0), top_k=kw.get("top_k", 0), seed=kw.get("seed", 0)))
    sent, first = 0, True
    while True:
        done = r.done.wait(0.002)
        toks = r.output[sent:]
        if toks:
            sent += len(toks)
            text = tok.decode([t for t in toks if t not in eng.eos_ids])
            yield ModelResponse([StreamChoice(Delta(text, "assistant" if first else None))], model=model)
            first = False
        if done and sent >= len(r.output):
            break
    if r.error:
        raise CompletionError(f"local engine: {r.error}")
    yield ModelResponse([StreamChoice(Delta(None), finish_reason=r.finish_reason or "stop")], model=model)


def _http_stream(model, messages, base, key, timeout, max_tokens, temperature, **kw):
    """Server-sent-event chunks of an OpenAI-compatible endpoint."""
    import json

    import httpx

    url = base.rstrip("/")
    if not url.endswith("/chat/completions"):
        url += "/chat/completions"
    headers = {"Content-Type": "application/json"}
    if key:
        headers["Authorization"] = f"Bearer {key}"
    body = {"model": model, "messages": messages, "max_tokens": max_tokens, "temperature": temperature,
            "stream": True}
    body.update({k: v for k, v in kw.items() if k in ("top_p", "stop", "seed", "top_k")})
    with httpx.stream("POST", url, json=body, headers=headers, timeout=timeout) as r:
        if r.status_code != 200:
            r.read()
            raise CompletionError(f"HTTP {r.status_code}: {r.text[:200]}")
        for line in r.iter_lines():
            if not line.startswith("data: "):
                continue
            data = line[6:]
            if data.strip() == "[DONE]":
                break
            j = json.loads(data)
            ch = j["choices"][0]
            d = ch.get("delta") or {}
            yield ModelResponse([StreamChoice(Delta(d.get("content"), d.get("role")), ch.get("index", 0),
                                              ch.get("finish_reason"))], model=j.get("model", model),
                                id=j.get("id", ""))


def completion(model: str, messages: list[dict], *, api_base: str | None = None, api_key: str | None = None,
               timeout: float | None = None, num_retries: int | None = None, max_tokens: int = 128,
               temperature: float = 0.0, backoff_base: float = 0.5, backoff_max: float = 8.0, stream: bool = False,
               **kw):
    """LiteLLM ``completion``: a ModelResponse, or with ``stream=True`` an iterator of
    chunks (``chunk.choices[0].delta.content``).  A stream is not retried once it
    has started."""
    base = api_base if api_base is not None else globals()["api_base"]
    key = api_key or globals()["api_key"] or os.environ.get("OPENAI_API_KEY")
    timeout = timeout if timeout is not None else request_timeout
    retries = num_retries if num_retries is not None else globals()["num_retries"]
    if stream:
        if _is_local(base):
            return _local_stream(model, messages, max_tokens, temperature, **kw)
        return _http_stream(model, messages, base, key, timeout, max_tokens, temperature, **kw)
    if _is_local(base):
        return _local(model, messages, max_tokens, temperature, **kw)
    attempt = 0
    while True:
        try:
            return _http(model, messages, base, key, timeout, max_tokens, temperature, **kw)
        except CompletionError:
            raise
        except Exception as e:  # noqa: BLE001 — connection errors, timeouts, 429/5xx
            attempt += 1
            if attempt > retries:
                raise CompletionError(f"completion failed after {retries} retries: {e}") from e
            delay = random.uniform(0, min(backoff_max, backoff_base * 2 ** (attempt - 1)))
            log.warning("completion attempt %d failed (%s); retrying in %.2fs", attempt, e, delay)
            time.sleep(delay)


async def acompletion(model: str, messages: list[dict], **kw):
    """LiteLLM ``acompletion``: awaitable ``completion`` (the blocking work runs in a
    worker thread); with ``stream=True`` an async iterator of chunks."""
    import asyncio

    if kw.get("stream"):
        it = completion(model, messages, **kw)

        async def agen():
            loop = asyncio.get_running_loop()
            sentinel = object()
            while True:
                chunk = await loop.run_in_executor(None, next, it, sentinel)
                if chunk is sentinel:
                    return
                yield chunk
        return agen()
    return await asyncio.to_thread(completion, model, messages, **kw)


def batch_completion(model: str, messages: list[list[dict]], *, api_base: str | None = None, max_tokens: int = 128,
                     temperature: float = 0.0, **kw) -> list[ModelResponse]:
    """LiteLLM ``batch_completion``: one response per conversation.  In-process
    engine: ONE batched generation (continuous batching over all of them);
    HTTP: the requests run concurrently."""
    base = api_base if api_base is not None else globals()["api_base"]
    if _is_local(base):
        eng, tok = _local_engine(model)
        ids = [tok.apply_chat_template(m) for m in messages]
        outs = eng.generate(ids, max_new_tokens=max_tokens, temperature=temperature, top_p=kw.get("top_p", 1.0),
                            top_k=kw.get("top_k", 0), seed=kw.get("seed", 0))
        return [ModelResponse([Choice(Message(tok.decode([t for t in o if t not in eng.eos_ids])))], model=model,
                              usage={"prompt_tokens": len(i), "completion_tokens": len(o)})
                for i, o in zip(ids, outs)]
    from concurrent.futures import ThreadPoolExecutor

    with ThreadPoolExecutor(max_workers=min(16, max(1, len(messages)))) as ex:
        futs = [ex.submit(completion, model, m, api_base=base, max_tokens=max_tokens, temperature=temperature, **kw)
                for m in messages]
        return [f.result() for f in futs]


@dataclass
class EmbeddingResponse:
    data: list
    model: str = ""
    usage: dict = field(default_factory=dict)
    object: str = "list"

    def __getitem__(self, k):
        return getattr(self, k)


def embedding(model: str, input, *, api_base: str | None = None, api_key: str | None = None,
              timeout: float | None = None, **kw) -> EmbeddingResponse:
    """LiteLLM ``embedding``: ``input`` a string or a list of strings; ``.data[i]["embedding"]``
    (mean-pooled final hidden states of the served model, unit norm)."""
    base = api_base if api_base is not None else globals()["api_base"]
    texts = [input] if isinstance(input, str) else list(input)
    if _is_local(base):
        eng, tok = _local_engine(model)
        seqs = [tok.encode(t) for t in texts]
        vec = eng.embed(seqs)
        n = sum(len(q) for q in seqs)
        return EmbeddingResponse([{"object": "embedding", "index": i, "embedding": v.tolist()}
                                  for i, v in enumerate(vec)], model=model,
                                 usage={"prompt_tokens": n, "total_tokens": n})
    import httpx

    key = api_key or globals()["api_key"] or os.environ.get("OPENAI_API_KEY")
    url = base.rstrip("/")
    if not url.endswith("/embeddings"):
        url += "/embeddings"
    headers = {"Authorization": f"Bearer {key}"} if key else {}
    r = httpx.post(url, json={"model": model, "input": texts}, headers=headers,
                   timeout=timeout if timeout is not None else request_timeout)
    if r.status_code != 200:
        raise CompletionError(f"HTTP {r.status_code}: {r.text[:200]}")
    j = r.json()
    return EmbeddingResponse(j["data"], model=j.get("model", model), usage=j.get("usage", {}))


@dataclass
class TextChoice:
    text: str
    index: int = 0
    finish_reason: str | None = "stop"

    def __getitem__(self, k):
        return getattr(self, k)


def text_completion(model: str, prompt: str, *, api_base: str | None = None, api_key: str | None = None,
                    timeout: float | None = None, max_tokens: int = 128, temperature: float = 0.0, **kw):
    """LiteLLM ``text_completion``: a raw prompt (no chat template); ``.choices[0].text``."""
    base = api_base if api_base is not None else globals()["api_base"]
    if _is_local(base):
        eng, tok = _local_engine(model)
        ids = tok.encode(prompt)
        out = eng.generate([ids], max_new_tokens=max_tokens, temperature=temperature, top_p=kw.get("top_p", 1.0),
                           top_k=kw.get("top_k", 0), seed=kw.get("seed", 0))[0]
        text = tok.decode([t for t in out if t not in eng.eos_ids])
        return ModelResponse([TextChoice(text, finish_reason="length" if len(out) >= max_tokens else "stop")],
                             model=model, usage={"prompt_tokens": len(ids), "completion_tokens": len(out)})
    import httpx

    key = api_key or globals()["api_key"] or os.environ.get("OPENAI_API_KEY")
    url = base.rstrip("/")
    if not url.endswith("/completions"):
        url += "/completions"
    headers = {"Authorization": f"Bearer {key}"} if key else {}
    body = {"model": model, "prompt": prompt, "max_tokens": max_tokens, "temperature": temperature}
    body.update({k: v for k, v in kw.items() if k in ("top_p", "stop", "seed", "top_k")})
    r = httpx.post(url, json=body, headers=headers, timeout=timeout if timeout is not None else request_timeout)
    if r.status_code != 200:
        raise CompletionError(f"HTTP {r.status_code}: {r.text[:200]}")
    j = r.json()
    c = j["choices"][0]
    return ModelResponse([TextChoice(c.get("text", ""), c.get("index", 0), c.get("finish_reason"))],
                         model=j.get("model", model), usage=j.get("usage", {}))
