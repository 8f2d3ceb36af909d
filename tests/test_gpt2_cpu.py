"""GPT-2 intent parser on CPU (BASELINE.json config 1: canned transcript -> GPT-2 -> /parse, no GPU).

Same engine contract as Llama: ragged decode through the paged cache == full prefill, grammar-
constrained answers are schema-valid, the brain service runs it from env configuration."""
import asyncio

import torch
from aiohttp.test_utils import TestClient, TestServer

from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
from voice_enabled_browser_automation_amd.brain.prompt import plain_chat
from voice_enabled_browser_automation_amd.brain.server import build_app, build_llm_engine
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.models.config import get_config
from voice_enabled_browser_automation_amd.models.gpt2 import GPT2Model
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer


def test_gpt2_tokenizer_layout():
    t = load_tokenizer("gpt2")
    assert t.vocab_size == 50257 and t.token_to_id("<|endoftext|>") == 50256
    s = 'search "wireless earbuds" under $50'
    assert t.decode(t.encode(s)) == s
    assert t.token_bytes()[50256] == b""


def test_gpt2_ragged_decode_matches_prefill():
    m = GPT2Model(get_config("gpt2-tiny"), device="cpu", seed=2)
    torch.manual_seed(0)
    toks = torch.randint(0, 50257, (100,)).tolist()
    eA = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=40)
    a = eA.new_sequence(toks, use_prefix_cache=False)
    la = eA.prefill(a).clone()  # 100 rows: flash (prefill) path
    eB = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=40)
    b = eB.new_sequence(toks[:70], use_prefix_cache=False)
    eB.prefill(b)
    lb = None
    for t in toks[70:]:
        lb = eB.run_rows([(b, t)])
    assert torch.allclose(la, lb, atol=2e-3, rtol=2e-3), (la - lb).abs().max()


def test_gpt2_intent_parse_valid_and_cached():
    m = GPT2Model(get_config("gpt2-tiny"), device="cpu", seed=0)
    ie = LLMIntentEngine(LLMEngine(m, max_seqs=2, max_model_len=2048), load_tokenizer("gpt2"), budget_chars=260,
                         chat_format=plain_chat)
    for text in ("search wireless earbuds", "scroll down"):
        out = ie.parse({"text": text, "context": {}})
        assert safe_parse(ParseResponse, out).success
    assert ie.last_stats["cached_prefix_tokens"] > 1000


def test_brain_service_with_gpt2_from_env(monkeypatch):
    monkeypatch.setenv("VWA_LLM_MODEL", "gpt2-tiny")
    monkeypatch.setenv("VWA_BUDGET_CHARS", "260")
    eng = build_llm_engine(device="cpu")

    async def go():
        async with TestClient(TestServer(build_app(eng))) as c:
            r = await c.post("/parse", json={"text": "go back"})
            return r.status, await r.json()

    st, j = asyncio.run(go())
    assert st == 200 and j["version"] == "1.0" and j["intents"]
