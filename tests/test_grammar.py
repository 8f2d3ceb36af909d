"""Grammar-constrained decoding engine (csrc/runtime/grammar.cpp): every masked random walk ends
in a schema-valid ParseResponse, the few-shot answers are accepted, budgets close the JSON,
jump-forward emits only forced bytes."""
import json
import random

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from voice_enabled_browser_automation_amd.brain.prompt import FEWSHOTS, compact
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.grammar import CompiledGrammar, intent_grammar, ir_from_json_schema
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer


@pytest.fixture(scope="module")
def tok():
    return load_tokenizer("llama3")


@pytest.fixture(scope="module")
def g(tok):
    return intent_grammar(tok)


def walk(g, tok, seed, budget, prefer_long=False):
    rng = random.Random(seed)
    tb = tok.token_bytes()
    mask = np.zeros(g.words, dtype=np.int32)
    m = g.matcher(budget)
    out = b""
    steps = 0
    while not m.is_accept():
        f = m.forced_prefix()
        if f:
            assert m.accept_bytes(f)
            out += f
            continue
        m.fill_mask(mask)
        bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[: g.vocab_size]
        ids = np.nonzero(bits)[0]
        assert len(ids) > 0, out
        if prefer_long:
            ids = sorted(ids, key=lambda i: -len(tb[i]))[:50]
        i = int(rng.choice(list(ids)))
        assert m.can_accept_token(i)
        assert m.accept_token(i), (out, i)
        out += tb[i]
        steps += 1
        assert steps < 2000
    return out, m


def test_fewshot_answers_accepted(g):
    for _, ans in FEWSHOTS:
        text = compact(ans)
        m = g.matcher(2000)
        if "tts_summary" in ans and len(ans["tts_summary"]) > 96:
            continue
        assert m.accept_bytes(text.encode()), text
        assert m.is_accept()


@settings(max_examples=25, deadline=None)
@given(seed=st.integers(0, 10 ** 6), budget=st.integers(150, 700), prefer_long=st.booleans())
def test_random_constrained_walks_are_schema_valid(tok, g, seed, budget, prefer_long):
    out, m = walk(g, tok, seed, budget, prefer_long)
    assert len(out) <= budget
    obj = json.loads(out)
    assert safe_parse(ParseResponse, obj).success, out


def test_rejects_invalid_prefixes(g):
    m = g.matcher(1000)
    assert not m.accept_bytes(b'{"version":"2.0"')
    m = g.matcher(1000)
    assert m.accept_bytes(b'{"version":"1.0","intents":[{"type":"')
    assert not m.clone().accept_bytes(b'fly"')
    assert m.clone().accept_bytes(b'search"')


def test_jump_forward_structure(g):
    m = g.matcher(1000)
    assert m.forced_prefix() == b'{"version":"1.0","intents":[{"type":"'
    m.accept_bytes(m.forced_prefix())
    m.accept_bytes(b"search")
    assert m.forced_prefix() == b'","args":{'


def test_eos_only_when_complete(g, tok):
    eot = tok.token_to_id("<|eot_id|>")
    m = g.matcher(1000)
    assert not m.can_accept_token(eot)
    _, m2 = walk(g, tok, 1, 300)
    assert m2.is_accept() and m2.can_accept_token(eot)
    mask = np.zeros(g.words, dtype=np.int32)
    m2.fill_mask(mask)
    bits = np.unpackbits(mask.view(np.uint8), bitorder="little")[: g.vocab_size]
    assert set(np.nonzero(bits)[0].tolist()) <= {eot, tok.token_to_id("<|end_of_text|>")}


def test_generic_json_schema_compiler(tok):
    schema = {"type": "object", "properties": {"n": {"type": "integer", "minimum": 0, "maximum": 3},
                                               "tags": {"type": "array", "items": {"type": "string", "maxLength": 5},
                                                        "maxItems": 2},
                                               "ok": {"type": "boolean"}},
              "required": ["n", "ok"]}
    cg = CompiledGrammar(ir_from_json_schema(schema), tok.token_bytes(), [tok.token_to_id("<|eot_id|>")])
    for text, ok in [('{"n":3,"ok":true}', True), ('{"n":4,"ok":true}', False), ('{"n":1,"tags":["ab"],"ok":false}', True),
                     ('{"n":1,"tags":["abcdef"],"ok":false}', False), ('{"ok":true}', False),
                     ('{"n":01,"ok":true}', False)]:
        m = cg.matcher(1000)
        assert (m.accept_bytes(text.encode()) and m.is_accept()) == ok, text


def test_integer_ranges_never_dead_end(g):
    """timeout_ms is an integer >= 1 (schema.ts: int().positive()): a leading "0" can never be
    completed (no digit may follow it, 0 is out of range), so the grammar must not admit it --
    that dead state surfaced as an all-empty mask under concurrent sampling.  Every admitted
    digit string must still be completable; the bounds are enforced exactly."""
    pre = b'{"version":"1.0","intents":[{"type":"back","args":{},"priority":0,"requires_confirmation":false,"timeout_ms":'
    for digits, ok in ((b"0", False), (b"1", True), (b"600000", True), (b"600001", False), (b"60000", True),
                       (b"9", True), (b"01", False)):
        m = g.matcher(512)
        assert m.accept_bytes(pre)
        assert m.accept_bytes(digits) == ok, digits
    # retries: 0..3 -> "0" fine, "4" not
    pre_r = b'{"version":"1.0","intents":[{"type":"back","args":{},"priority":0,"requires_confirmation":false,"retries":'
    for digits, ok in ((b"0", True), (b"3", True), (b"4", False), (b"10", False)):
        m = g.matcher(512)
        assert m.accept_bytes(pre_r)
        assert m.accept_bytes(digits) == ok, digits
