"""Contract tests: v1 intent schema (apps/brain/src/schema.ts) and the legacy v0 shape
(packages/schemas/test/intent.test.ts:5-53, ported 1:1)."""
import pytest

from voice_enabled_browser_automation_amd.contracts import (INTENT_TYPES, ExecuteRequest, Intent, ParseRequest,
                                                           ParseResponse, parse_intent, safe_parse)


# ---- packages/schemas/test/intent.test.ts (v0)
def test_v0_minimal_navigate():
    it = parse_intent({"intent": "navigate", "utterance": "go to bestbuy", "confidence": 0.9,
                       "target": {"url": "https://www.bestbuy.com"}})
    assert it.intent == "navigate"
    assert it.target.url.startswith("https://www.bestbuy.com")


def test_v0_filter_sort_params():
    it = parse_intent({"intent": "filter", "utterance": "under 50 sorted by price asc", "confidence": 0.85,
                       "params": {"filters": [{"field": "price", "op": "<=", "value": 50}],
                                  "sorting": {"field": "price", "order": "asc"}}})
    assert it.params.filters[0].op == "<="
    assert it.params.sorting.order == "asc"


def test_v0_rejects_invalid_confidence():
    with pytest.raises(Exception):
        parse_intent({"intent": "navigate", "utterance": "go", "confidence": 2})


def test_v0_extract_fields_export():
    it = parse_intent({"intent": "extract", "utterance": "export results as csv", "confidence": 0.8,
                       "params": {"fields": ["title", "price", "rating", "url"], "format": "csv",
                                  "filename": "earbuds.csv"}})
    assert len(it.params.fields) > 0 and it.params.format == "csv"


# ---- v1
def test_intent_types_are_the_19_of_the_reference():
    assert len(INTENT_TYPES) == 19 and INTENT_TYPES[0] == "search" and INTENT_TYPES[-1] == "unknown"


def test_parse_response_defaults_and_omission():
    r = safe_parse(ParseResponse, {"version": "1.0", "intents": [{"type": "search", "args": {"query": "x"}}],
                                   "confidence": 0.9})
    assert r.success
    d = r.data
    assert d["context_updates"] == {}
    assert d["intents"][0] == {"type": "search", "args": {"query": "x"}, "priority": 0,
                               "requires_confirmation": False, "retries": 1}
    assert "tts_summary" not in d and "follow_up_question" not in d


def test_parse_response_keeps_explicit_null_follow_up():
    d = safe_parse(ParseResponse, {"version": "1.0", "intents": [{"type": "back"}], "confidence": 0.5,
                                   "follow_up_question": None}).data
    assert d["follow_up_question"] is None


@pytest.mark.parametrize("bad", [
    {"version": "1.1", "intents": [{"type": "back"}], "confidence": 0.5},
    {"version": "1.0", "intents": [], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "fly"}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back"}], "confidence": 1.5},
    {"version": "1.0", "intents": [{"type": "back", "retries": 4}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back", "timeout_ms": 0}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back", "extra": 1}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back", "target": {"strategy": "auto", "foo": 1}}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back", "requires_confirmation": "true"}], "confidence": 0.5},
    {"version": "1.0", "intents": [{"type": "back"}], "confidence": 0.5, "unexpected": True},
])
def test_parse_response_rejects(bad):
    r = safe_parse(ParseResponse, bad)
    assert not r.success
    assert "_errors" in r.format_error()


def test_integer_valued_floats_are_ints_like_js():
    d = safe_parse(Intent, {"type": "click", "priority": 2.0, "retries": 3}).data
    assert d["priority"] == 2 and isinstance(d["priority"], int)
    assert not safe_parse(Intent, {"type": "click", "priority": 1.5}).success


def test_target_partial_strategy_default_not_applied():
    d = safe_parse(Intent, {"type": "click", "target": {"selector": "a"}}).data
    assert d["target"] == {"selector": "a"}


def test_parse_request():
    assert not safe_parse(ParseRequest, {"text": ""}).success
    assert "text is empty" in str(safe_parse(ParseRequest, {"text": ""}).format_error())
    d = safe_parse(ParseRequest, {"text": "hi"}).data
    assert d == {"text": "hi", "context": {}}
    assert not safe_parse(ParseRequest, {"text": "hi", "foo": 1}).success
    assert not safe_parse(ParseRequest, [1, 2]).success


def test_execute_request():
    assert not safe_parse(ExecuteRequest, {"intents": []}).success
    d = safe_parse(ExecuteRequest, {"intents": [{"type": "back"}], "options": {"headless": True}}).data
    assert d["options"] == {"headless": True} and "session_id" not in d
