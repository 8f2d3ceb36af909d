"""Brain /parse service (port of apps/brain/test/parse.test.ts + error paths of server.ts:89-139).

The engine is mocked at the module boundary like the reference's vi.spyOn(llm, "callLLMJSON")."""
import asyncio

from aiohttp.test_utils import TestClient, TestServer

from voice_enabled_browser_automation_amd.brain.intent_engine import FakeIntentEngine, keyword_intents
from voice_enabled_browser_automation_amd.brain.server import build_app


def call(engine, method, path, json=None):
    async def go():
        async with TestClient(TestServer(build_app(engine))) as c:
            r = await c.request(method, path, json=json)
            return r.status, await r.json()

    return asyncio.run(go())


def test_health():
    assert call(FakeIntentEngine({}), "GET", "/health") == (200, {"status": "ok", "service": "brain-ts"})


def test_validates_simple_search_intent():
    eng = FakeIntentEngine({"version": "1.0", "intents": [{"type": "search", "args": {"query": "wireless earbuds"},
                                                            "priority": 0, "requires_confirmation": False}],
                            "context_updates": {"query": "wireless earbuds"}, "confidence": 0.9,
                            "tts_summary": "Searching for wireless earbuds."})
    st, j = call(eng, "POST", "/parse", {"text": "search wireless earbuds"})
    assert st == 200
    assert j["version"] == "1.0" and j["intents"][0]["type"] == "search" and j["confidence"] > 0.5
    # prompt = system + 10 few-shot messages + user JSON (apps/brain/src/server.ts:98-105)
    msgs = eng.calls[0]
    assert msgs[0]["role"] == "system" and len(msgs) == 12 and msgs[-1]["role"] == "user"


def test_upload_with_confirmation_and_tts():
    eng = FakeIntentEngine({"version": "1.0", "intents": [
        {"type": "upload", "target": {"strategy": "auto", "selector": "input[type='file']"},
         "args": {"fileRef": "resume://latest"}, "priority": 0, "requires_confirmation": True, "retries": 1},
        {"type": "click", "target": {"strategy": "text", "text": "Submit"}, "args": {}, "priority": 1,
         "requires_confirmation": True}], "context_updates": {}, "confidence": 0.75,
        "tts_summary": "I will upload your resume and then click submit. Please confirm.", "follow_up_question": None})
    st, j = call(eng, "POST", "/parse", {"text": "upload my resume and submit the application"})
    assert st == 200
    assert any(i["type"] == "upload" for i in j["intents"])
    assert j["tts_summary"]
    assert all(isinstance(i["requires_confirmation"], bool) for i in j["intents"])


def test_follow_up_low_confidence():
    eng = FakeIntentEngine({"version": "1.0", "intents": [{"type": "unknown", "args": {}, "priority": 0,
                                                            "requires_confirmation": False}],
                            "context_updates": {}, "confidence": 0.5,
                            "follow_up_question": "Which job title and location should I search for?"})
    st, j = call(eng, "POST", "/parse", {"text": "apply for that job"})
    assert st == 200 and j["confidence"] <= 0.6 and "which job" in j["follow_up_question"].lower()


def test_invalid_request_400():
    st, j = call(FakeIntentEngine({}), "POST", "/parse", {"text": ""})
    assert st == 400 and j["error"] == "invalid_request"
    st, j = call(FakeIntentEngine({}), "POST", "/parse", {"text": "x", "bogus": 1})
    assert st == 400


def test_llm_error_500():
    st, j = call(FakeIntentEngine(fail=RuntimeError("model crashed")), "POST", "/parse", {"text": "hi"})
    assert st == 500 and j == {"error": "llm_error", "detail": "model crashed"}


def test_single_repair_then_ok():
    good = {"version": "1.0", "intents": [{"type": "back"}], "confidence": 0.7}
    eng = FakeIntentEngine([{"oops": True}, good])
    st, j = call(eng, "POST", "/parse", {"text": "go back"})
    assert st == 200 and j["intents"][0]["type"] == "back"
    assert len(eng.calls) == 2 and eng.calls[1][-1]["role"] == "system"  # repair note appended


def test_repair_fails_422():
    eng = FakeIntentEngine([{"oops": True}, {"still": "bad"}])
    st, j = call(eng, "POST", "/parse", {"text": "go back"})
    assert st == 422 and j["error"] == "schema_validation_failed"
    assert len(eng.calls) == 2


def test_keyword_engine_and_metrics():
    eng = FakeIntentEngine(fn=keyword_intents)
    st, j = call(eng, "POST", "/parse", {"text": "search noise cancelling headphones"})
    assert st == 200 and j["intents"][0] == {"type": "search", "args": {"query": "noise cancelling headphones"},
                                             "priority": 0, "requires_confirmation": False, "retries": 1}
    st, m = call(eng, "GET", "/metrics")
    assert st == 200 and m["service"] == "brain"


def test_concurrent_parse_requests_batch_on_llm_engine():
    """Real (tiny, CPU) LLM engine behind /parse: concurrent HTTP requests are decoded together by
    the continuous-batching scheduler and all come back schema-valid."""
    from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
    from voice_enabled_browser_automation_amd.models.config import LLAMA_PRESETS
    from voice_enabled_browser_automation_amd.models.llama import LlamaModel
    from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
    from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cpu", seed=1)
    ie = LLMIntentEngine(LLMEngine(m, max_seqs=4, max_model_len=2048, kv_blocks=800), load_tokenizer("llama3"),
                         budget_chars=200)

    async def go():
        async with TestClient(TestServer(build_app(ie))) as c:
            rs = await asyncio.gather(*[c.post("/parse", json={"text": t}) for t in
                                        ("scroll down", "go back", "search for laptops")])
            return [(r.status, await r.json()) for r in rs]

    res = asyncio.run(go())
    assert all(st == 200 and j["version"] == "1.0" and j["intents"] for st, j in res)
    es = ie.engine_stats()
    assert es["kv_blocks_total"] == 800 and 0 < es["kv_blocks_used"] < 800  # static prefix stays cached
    assert es["samples_per_iteration"] > 1 and es["grammar_rejects"] == 0
    assert ie.batch_stats["max_active"] >= 2
    assert ie._thread is None  # scheduler stopped on app cleanup
