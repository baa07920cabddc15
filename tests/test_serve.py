"""Inference engine + OpenAI-compatible server + LiteLLM-compatible client (CPU).

SURVEY §4.2 item 3: the framework's own server on localhost with the tiny
model; ``completion()`` over HTTP, the reference's error fallback string,
retry/backoff (A5).
"""
import socket
import threading
import time

import pytest
import torch

from mxllm.data.tokenizer import ByteTokenizer
from mxllm.models import Llama, get_config
from mxllm.serve import client
from mxllm.serve.engine import Engine


@pytest.fixture(scope="module")
def tiny_engine():
    torch.manual_seed(0)
    cfg = get_config("tiny")
    m = Llama(cfg, seed=0).eval()
    return Engine(m, max_batch=4, max_seq=256)


def test_greedy_decode_matches_full_forward(tiny_engine):
    m = tiny_engine.model
    prompt = [5, 9, 77, 1, 300]
    out = tiny_engine.generate([prompt], max_new_tokens=6)[0]
    seq = list(prompt)
    with torch.no_grad():
        for _ in range(6):
            seq.append(int(m(torch.tensor([seq]))[0, -1].float().argmax()))
    assert out == seq[len(prompt):]


def test_continuous_batching_is_order_independent(tiny_engine):
    prompts = [[i, i + 1, i + 2] for i in range(1, 10)]  # 9 prompts through 4 slots
    batched = tiny_engine.generate(prompts, max_new_tokens=5)
    single = [tiny_engine.generate([p], max_new_tokens=5)[0] for p in prompts]
    assert batched == single


def test_batched_prefill_matches_single(tiny_engine):
    """Prompts of different lengths prefilled together in one pass (and split
    into several passes by the prefill token budget) generate exactly what
    each prompt generates alone."""
    prompts = [[7] * 3, list(range(20, 61)), [1, 2], list(range(100, 117))]
    single = [tiny_engine.generate([p], max_new_tokens=4)[0] for p in prompts]
    assert tiny_engine.generate(prompts, max_new_tokens=4) == single
    eng = Engine(tiny_engine.model, max_batch=4, max_seq=256, prefill_tokens=20)
    assert eng.generate(prompts, max_new_tokens=4) == single


def test_engine_serving_stats(tiny_engine):
    before = tiny_engine.stats()["requests_finished"]
    tiny_engine.generate([[1, 2, 3], [4, 5]], max_new_tokens=4)
    st = tiny_engine.stats()
    assert st["requests_finished"] == before + 2
    assert st["mean_ttft_s"] > 0 and st["mean_latency_s"] >= st["mean_ttft_s"]
    assert st["decode_tokens_per_s"] > 0 and st["prefill_tokens_per_s"] > 0


def test_sampling_temperature_reproducible(tiny_engine):
    a = tiny_engine.generate([[3, 4, 5]], max_new_tokens=8, temperature=1.0, seed=7)
    b = tiny_engine.generate([[3, 4, 5]], max_new_tokens=8, temperature=1.0, seed=7)
    assert a == b


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def server(tiny_engine):
    import uvicorn

    from mxllm.serve.server import build_app

    port = _free_port()
    app = build_app(tiny_engine, ByteTokenizer(512), "tiny-test", api_key="sekret")
    cfg = uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error")
    srv = uvicorn.Server(cfg)
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.05)
    yield f"http://127.0.0.1:{port}/v1"
    srv.should_exit = True
    th.join(10)
    tiny_engine.stop()


def test_http_completion_roundtrip(server):
    r = client.completion("tiny-test", [{"role": "user", "content": "hello"}], api_base=server, api_key="sekret",
                          max_tokens=5, timeout=30)
    assert isinstance(r.choices[0].message.content, str)
    assert r.usage["completion_tokens"] >= 1


def test_http_auth_rejected(server):
    with pytest.raises(client.CompletionError):
        client.completion("tiny-test", [{"role": "user", "content": "x"}], api_base=server, api_key="wrong",
                          max_tokens=2, timeout=30)


def test_http_models_and_stream(server):
    import httpx

    j = httpx.get(server + "/models", timeout=10).json()
    assert j["data"][0]["id"] == "tiny-test"
    with httpx.stream("POST", server + "/chat/completions", timeout=30, headers={"Authorization": "Bearer sekret"},
                      json={"messages": [{"role": "user", "content": "hi"}], "max_tokens": 4, "stream": True}) as s:
        lines = [ln for ln in s.iter_lines() if ln]
    assert lines[-1] == "data: [DONE]"


def test_fallback_string_on_dead_endpoint(monkeypatch):
    import src.distributed_inference as di

    monkeypatch.setattr(client, "api_base", f"http://127.0.0.1:{_free_port()}/v1")
    monkeypatch.setattr(di.RUN, "num_retries", 1)
    monkeypatch.setattr(di.RUN, "request_timeout", 2.0)
    assert di.get_model_response("hi") == "Error: Unable to get model response"


def test_retry_with_backoff(monkeypatch):
    calls = {"n": 0}

    def flaky(*a, **k):
        calls["n"] += 1
        if calls["n"] < 3:
            raise client._Retryable("HTTP 429")
        return client.ModelResponse([client.Choice(client.Message("ok"))])

    monkeypatch.setattr(client, "_http", flaky)
    r = client.completion("m", [{"role": "user", "content": "x"}], api_base="http://x", num_retries=3,
                          backoff_base=0.001)
    assert r.choices[0].message.content == "ok" and calls["n"] == 3
    calls["n"] = -10
    with pytest.raises(client.CompletionError):
        client.completion("m", [], api_base="http://x", num_retries=2, backoff_base=0.001)


def test_local_inproc_route(tiny_engine):
    client.register_local("tiny-local", tiny_engine, ByteTokenizer(512))
    try:
        r = client.completion("tiny-local", [{"role": "user", "content": "abc"}], api_base="local", max_tokens=3)
        assert isinstance(r.choices[0].message.content, str)
    finally:
        client.unregister_local("tiny-local")


def test_http_stream_and_async_and_batch(server):
    """LiteLLM streaming (SSE deltas), acompletion and batch_completion over HTTP."""
    import asyncio

    msgs = [{"role": "user", "content": "hello"}]
    full = client.completion("tiny-test", msgs, api_base=server, api_key="sekret", max_tokens=6, timeout=30)
    chunks = list(client.completion("tiny-test", msgs, api_base=server, api_key="sekret", max_tokens=6,
                                    timeout=30, stream=True))
    assert chunks[-1].choices[0].finish_reason is not None
    streamed = "".join(c.choices[0].delta.content or "" for c in chunks)
    assert streamed == full.choices[0].message.content  # greedy: same text either way
    r = asyncio.run(client.acompletion("tiny-test", msgs, api_base=server, api_key="sekret", max_tokens=6,
                                       timeout=30))
    assert r.choices[0].message.content == full.choices[0].message.content
    many = client.batch_completion("tiny-test", [msgs, [{"role": "user", "content": "other"}]], api_base=server,
                                   api_key="sekret", max_tokens=4, timeout=30)
    assert len(many) == 2 and all(isinstance(m.choices[0].message.content, str) for m in many)


def test_local_stream_and_batch(tiny_engine):
    client.register_local("tiny-local2", tiny_engine, ByteTokenizer(512))
    try:
        msgs = [{"role": "user", "content": "abc"}]
        full = client.completion("tiny-local2", msgs, api_base="local", max_tokens=5)
        chunks = list(client.completion("tiny-local2", msgs, api_base="local", max_tokens=5, stream=True))
        assert "".join(c.choices[0].delta.content or "" for c in chunks) == full.choices[0].message.content
        outs = client.batch_completion("tiny-local2", [msgs, msgs], api_base="local", max_tokens=5)
        assert [o.choices[0].message.content for o in outs] == [full.choices[0].message.content] * 2
    finally:
        client.unregister_local("tiny-local2")  # the module's server keeps using the running engine


def test_embeddings_http_and_local(server, tiny_engine):
    """/v1/embeddings + client.embedding(): unit-norm mean-pooled hidden states,
    deterministic, distinct for distinct inputs, identical over HTTP and in process,
    and equal to the model's own hidden states."""
    r = client.embedding("tiny-test", ["hello world", "something else"], api_base=server, api_key="sekret",
                         timeout=30)
    v = torch.tensor([d["embedding"] for d in r.data])
    assert v.shape[0] == 2 and torch.allclose(v.norm(dim=1), torch.ones(2), atol=1e-4)
    assert (v[0] - v[1]).abs().max() > 1e-3
    again = client.embedding("tiny-test", "hello world", api_base=server, api_key="sekret", timeout=30)
    assert torch.allclose(torch.tensor(again.data[0]["embedding"]), v[0], atol=1e-6)
    tok = ByteTokenizer(512)
    client.register_local("tiny-emb", tiny_engine, tok)
    try:
        loc = client.embedding("tiny-emb", ["hello world"], api_base="local")
        want = torch.nn.functional.normalize(
            tiny_engine.model.hidden_states(torch.tensor([tok.encode("hello world")])).float().mean(0), dim=0)
        torch.testing.assert_close(torch.tensor(loc.data[0]["embedding"]), want, rtol=1e-5, atol=1e-5)
    finally:
        client.unregister_local("tiny-emb")
    import httpx

    bad = httpx.post(server + "/embeddings", json={"model": "tiny-test", "input": ""},
                     headers={"Authorization": "Bearer sekret"}, timeout=30)
    assert bad.status_code == 400


def test_text_completion_http_and_local(server, tiny_engine):
    r = client.text_completion("tiny-test", "Once upon", api_base=server, api_key="sekret", max_tokens=5, timeout=30)
    assert isinstance(r.choices[0].text, str) and r.usage["completion_tokens"] <= 5
    client.register_local("tiny-tc", tiny_engine, ByteTokenizer(512))
    try:
        loc = client.text_completion("tiny-tc", "Once upon", api_base="local", max_tokens=5)
        assert loc.choices[0].text == r.choices[0].text  # greedy, same weights and tokenizer
    finally:
        client.unregister_local("tiny-tc")


def test_fp8_weight_engine_cpu():
    """Serving with e4m3 projection weights (CPU reference path): the model keeps
    generating and its prefill logits stay close to the bf16 model's."""
    from mxllm.serve.quant import W8Linear, quantize_model_fp8_

    cfg = get_config("tiny")
    prompt = [5, 9, 77, 1, 300, 12, 44]
    ref = Engine(Llama(cfg, seed=4).eval(), max_batch=2, max_seq=128)
    m8 = Llama(cfg, seed=4).eval()
    quantize_model_fp8_(m8)
    assert isinstance(m8.layers[0].wqkv, W8Linear)
    eng = Engine(m8, max_batch=2, max_seq=128)
    cos = torch.nn.functional.cosine_similarity(eng.prefill(0, prompt), ref.prefill(0, prompt), dim=0).item()
    assert cos > 0.99, cos
    assert len(eng.generate([prompt], max_new_tokens=5)[0]) == 5
