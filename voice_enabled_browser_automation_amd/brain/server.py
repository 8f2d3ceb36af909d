"""Brain service: ``GET /health``, ``POST /parse``, ``GET /metrics`` (parity with apps/brain/src/server.ts).

Request flow (apps/brain/src/server.ts:89-139):
  ParseRequest validation -> 400 {error:"invalid_request", detail}
  prompt (system + few-shots + user JSON) -> intent engine
     engine raises            -> 500 {error:"llm_error", detail}
     reply fails ParseResponse -> ONE repair call with the repair system note
  final validation fails      -> 422 {error:"schema_validation_failed", detail}
  200 -> ParseResponse with zod-style defaults filled.

With the LLM engine the grammar makes the first answer schema-valid, so the repair path only
runs for engines without constrained decoding (or injected faults in tests).

Engines (VWA_BRAIN_ENGINE): ``llm`` (on-GPU Llama + constrained decoding; VWA_LLM_MODEL, VWA_TP),
``keyword`` (rule-based, CPU), or any object passed to ``build_app(engine=...)``.
"""
from __future__ import annotations

import asyncio
import json
import os
import time
from typing import Any, Optional

from aiohttp import web

from ..contracts import ParseRequest, ParseResponse, safe_parse
from ..utils.context import cap_context
from ..utils.metrics import Metrics
from .prompt import messages_for
from .tp_engine import TPIntentEngine  # noqa: F401  (re-exported: the TP control plane)
from ..utils.env import knob

SERVICE_NAME = "brain-ts"  # byte-compatible /health payload (apps/brain/src/server.ts:87)


def build_app(engine: Any = None) -> web.Application:
    if engine is None:
        engine = make_engine_from_env()
    app = web.Application()
    app["engine"] = engine
    app["lock"] = asyncio.Lock()
    app["metrics"] = Metrics("brain")

    async def health(_req: web.Request) -> web.Response:
        failed = getattr(app["engine"], "failed", None)
        if failed is not None:  # a TP group that lost lockstep: the process is about to exit
            return web.json_response({"status": "error", "service": SERVICE_NAME, "detail": str(failed)}, status=503)
        return web.json_response({"status": "ok", "service": SERVICE_NAME})

    async def metrics(_req: web.Request) -> web.Response:
        snap = app["metrics"].snapshot()
        eng = app["engine"]
        st = getattr(eng, "last_stats", None)
        if st:
            snap["last_request"] = st
        if hasattr(eng, "engine_stats"):
            snap["engine"] = eng.engine_stats()
        return web.json_response(snap)

    async def call(eng, messages):
        if hasattr(eng, "submit_async"):
            # continuous batching: concurrent requests decode together on the scheduler thread
            eng.start()
            return json.loads(await asyncio.wrap_future(eng.submit_async(messages)))
        async with app["lock"]:  # engines without a scheduler: serial requests
            return await asyncio.get_running_loop().run_in_executor(None, eng, messages)

    async def on_cleanup(_app):
        if hasattr(app["engine"], "stop"):
            app["engine"].stop()

    async def parse(req: web.Request) -> web.Response:
        m: Metrics = app["metrics"]
        t0 = time.perf_counter()
        try:
            body = await req.json()
        except Exception:  # noqa: BLE001
            body = None
        pr = safe_parse(ParseRequest, body)
        if not pr.success:
            m.inc("invalid_request")
            return web.json_response({"error": "invalid_request", "detail": pr.format_error()}, status=400)
        request = pr.data
        # bounded context: whatever a client accumulated, the prompt stays
        # inside the model's window (oldest keys evicted first)
        if isinstance(request.get("context"), dict):
            request = {**request, "context": cap_context(request["context"])}
        eng = app["engine"]
        try:
            out = await call(eng, messages_for(request))
            first = safe_parse(ParseResponse, out)
            if not first.success:
                m.inc("repairs")
                out = await call(eng, messages_for(request, repair=True))
        except Exception as e:  # noqa: BLE001
            m.inc("llm_error")
            return web.json_response({"error": "llm_error", "detail": str(e) or e.__class__.__name__}, status=500)
        final = safe_parse(ParseResponse, out)
        if not final.success:
            m.inc("schema_validation_failed")
            return web.json_response({"error": "schema_validation_failed", "detail": final.format_error()}, status=422)
        m.observe("parse_ms", (time.perf_counter() - t0) * 1e3)
        m.inc("ok")
        st = getattr(eng, "last_stats", None) or {}
        if "prefill_ms" in st:  # engine-side request spans (TTFT ~ queue + prefill; decode rate)
            m.observe("ttft_ms", st.get("queue_ms", 0.0) + st["prefill_ms"])
            m.observe("decode_ms", st["decode_ms"])
            if st.get("decode_ms", 0) > 0:
                toks = st.get("decode_steps", 0) + st.get("forced_tokens", 0)
                m.observe("decode_tok_per_s", toks / (st["decode_ms"] / 1e3))
        return web.json_response(final.data)

    app.on_cleanup.append(on_cleanup)
    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics)
    app.router.add_post("/parse", parse)
    return app


def make_engine_from_env():
    kind = knob("VWA_BRAIN_ENGINE")
    if kind == "keyword":
        from .intent_engine import FakeIntentEngine, keyword_intents

        return FakeIntentEngine(fn=keyword_intents)
    if kind == "llm":
        return build_llm_engine()
    raise ValueError(f"unknown VWA_BRAIN_ENGINE={kind!r}")


def build_llm_engine(model_name: Optional[str] = None, device: Optional[str] = None):
    """Intent LLM from env: VWA_LLM_MODEL (llama3-8b | llama3-70b | llama3.2-1b | llama-tiny |
    gpt2-small | gpt2-tiny), VWA_LLM_WEIGHTS (safetensors dir; random init if unset), VWA_DTYPE
    (bf16 | fp8 weights for Llama), VWA_TP,
    VWA_MAX_SESSIONS, VWA_BUDGET_CHARS, VWA_SEED.  GPT-2 is the
    CPU config (BASELINE.json config 1): plain-text prompt layout, GPT-2 vocabulary."""
    import torch

    from ..models.config import GPT2Config, get_config
    from ..parallel.tp import init_distributed
    from ..runtime.engine import LLMEngine
    from ..runtime.weights import load_llm
    from ..tokenizer import load_tokenizer
    from .intent_engine import LLMIntentEngine
    from .prompt import llama3_chat, plain_chat

    name = model_name or knob("VWA_LLM_MODEL")
    cfg = get_config(name)
    seed = knob("VWA_SEED")
    dev = device or ("cuda" if torch.cuda.is_available() else "cpu")
    sessions = knob("VWA_MAX_SESSIONS")
    budget = knob("VWA_BUDGET_CHARS")
    wpath = knob("VWA_LLM_WEIGHTS") or None  # safetensors checkpoint (HF names)
    if isinstance(cfg, GPT2Config):
        model = load_llm(name, device=dev, seed=seed, weights_path=wpath)
        eng = LLMEngine(model, max_seqs=sessions, max_model_len=cfg.max_pos)
        eng.capture_all()
        return LLMIntentEngine(eng, load_tokenizer("gpt2"), budget_chars=budget, chat_format=plain_chat)
    tp = init_distributed(tp_size=knob("VWA_TP"))
    model = load_llm(name, device=dev, tp=tp, seed=seed, weights_path=wpath,
                     wdtype=knob("VWA_DTYPE"))
    eng = LLMEngine(model, max_seqs=sessions, max_model_len=4096)
    from ..utils.busy_flag import from_env

    flag = from_env(create=True)  # shared-GPU deployment: no chained launch while the ASR runs
    if flag is not None and tp.size == 1:
        hold = knob("VWA_ASR_BUSY_HOLD_MS")
        eng.chain_gate = lambda: flag.busy(hold)
    eng.capture_all()
    ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=budget, chat_format=llama3_chat)
    return TPIntentEngine(ie, tp) if tp.size > 1 else ie


def main():
    from ..utils.env import load_dotenv

    load_dotenv()
    port = knob("BRAIN_PORT")
    engine = make_engine_from_env()
    if isinstance(engine, TPIntentEngine) and engine.tp.rank != 0:
        engine.worker_loop()  # TP worker: no HTTP, follows rank 0's requests
        return
    print(f"[brain] listening on http://127.0.0.1:{port}", flush=True)
    web.run_app(build_app(engine), host="127.0.0.1", port=port, print=None)


if __name__ == "__main__":
    main()
