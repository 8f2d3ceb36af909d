"""JSON-schema -> grammar IR compiler + Python handle on the native constrained-decoding engine.

`ir_from_json_schema` compiles the subset of JSON Schema that pydantic emits for the contracts
(object/properties/required, additionalProperties, enum/const, string/number/integer/boolean/
null, array items/minItems/maxItems, anyOf) plus *generation bounds* (maxLength, maxItems,
maxProperties, fraction digits, nesting depth for free-form values) into the compact IR parsed by
csrc/runtime/grammar.cpp.  `parse_response_schema()` is the generation schema for the brain's
ParseResponse (apps/brain/src/schema.ts:60-69) with the key order of the zod definition.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from ..contracts.schema import INTENT_TYPES, TARGET_STRATEGIES


class _IRBuilder:
    def __init__(self):
        self.nodes: List[dict] = []
        self.memo: Dict[str, int] = {}

    def add(self, node: dict) -> int:
        key = json.dumps(node, sort_keys=True)
        if key in self.memo:
            return self.memo[key]
        self.nodes.append(node)
        self.memo[key] = len(self.nodes) - 1
        return self.memo[key]

    def any_value(self, depth: int, str_max: int = 48, max_items: int = 4, max_props: int = 3) -> int:
        opts = [self.add({"t": "str", "max": str_max}), self.add({"t": "num", "min": -1e6, "max": 1e6, "frac": 3}),
                self.add({"t": "bool"}), self.add({"t": "null"})]
        if depth > 0:
            inner = self.any_value(depth - 1, str_max, max_items, max_props)
            opts.append(self.add({"t": "arr", "item": inner, "min": 0, "max": max_items}))
            opts.append(self.add({"t": "rec", "v": inner, "max": max_props, "klen": 24}))
        return self.add({"t": "alt", "opts": opts})


def ir_from_json_schema(schema: Dict[str, Any], *, str_max: int = 64, any_depth: int = 1, max_items: int = 4,
                        max_props: int = 3, frac: int = 3) -> str:
    """Compile a JSON-schema dict (pydantic style, ``$defs`` refs allowed) into IR JSON text."""
    b = _IRBuilder()
    defs = schema.get("$defs", {})

    def comp(s: Dict[str, Any]) -> int:
        if "$ref" in s:
            return comp(defs[s["$ref"].split("/")[-1]])
        if "anyOf" in s:
            return b.add({"t": "alt", "opts": [comp(o) for o in s["anyOf"]]})
        if "const" in s:
            return b.add({"t": "const", "s": json.dumps(s["const"], separators=(",", ":"))})
        if "enum" in s:
            vals = s["enum"]
            if all(isinstance(v, str) for v in vals):
                return b.add({"t": "enum", "vals": list(vals)})
            return b.add({"t": "alt", "opts": [b.add({"t": "const", "s": json.dumps(v)}) for v in vals]})
        t = s.get("type")
        if isinstance(t, list):
            return b.add({"t": "alt", "opts": [comp({**s, "type": x}) for x in t]})
        if t == "object":
            props = s.get("properties")
            if props:
                req = set(s.get("required", []))
                return b.add({"t": "obj", "props": [[k, comp(v), k in req] for k, v in props.items()]})
            ap = s.get("additionalProperties", True)
            vnode = comp(ap) if isinstance(ap, dict) else b.any_value(any_depth, str_max, max_items, max_props)
            return b.add({"t": "rec", "v": vnode, "max": s.get("maxProperties", max_props), "klen": 24})
        if t == "array":
            item = comp(s["items"]) if "items" in s else b.any_value(any_depth - 1, str_max, max_items, max_props)
            return b.add({"t": "arr", "item": item, "min": s.get("minItems", 0), "max": s.get("maxItems", max_items)})
        if t == "string":
            return b.add({"t": "str", "max": s.get("maxLength", str_max)})
        if t == "integer":
            return b.add({"t": "int", "min": s.get("minimum", -10 ** 9), "max": s.get("maximum", 10 ** 9)})
        if t == "number":
            return b.add({"t": "num", "min": s.get("minimum", -1e6), "max": s.get("maximum", 1e6),
                          "frac": s.get("x-frac", frac)})
        if t == "boolean":
            return b.add({"t": "bool"})
        if t == "null":
            return b.add({"t": "null"})
        return b.any_value(any_depth, str_max, max_items, max_props)

    root = comp(schema)
    return json.dumps({"root": root, "nodes": b.nodes}, separators=(",", ":"))


def parse_response_schema(*, max_intents: int = 3, str_max: int = 48, summary_max: int = 96) -> Dict[str, Any]:
    """Generation schema for ParseResponse (apps/brain/src/schema.ts:39-69), zod key order.

    Generation bounds keep a random-init model's output near the reference few-shot size
    (230-598 chars, apps/brain/src/server.ts:36-81); the validation schema is still the strict
    pydantic one (contracts/schema.py).
    """
    s = {"type": "string", "maxLength": str_max}
    target = {"type": "object", "properties": {
        "strategy": {"enum": list(TARGET_STRATEGIES)}, "selector": s, "text": s, "role": s, "name": s},
        "required": []}
    free = {"type": "object", "maxProperties": 3}
    intent = {"type": "object", "properties": {
        "type": {"enum": list(INTENT_TYPES)},
        "args": free,
        "target": target,
        "priority": {"type": "integer", "minimum": 0, "maximum": 9},
        "requires_confirmation": {"type": "boolean"},
        "timeout_ms": {"type": "integer", "minimum": 1, "maximum": 600000},
        "retries": {"type": "integer", "minimum": 0, "maximum": 3},
        "clarification": s,
    }, "required": ["type", "args", "priority", "requires_confirmation"]}
    return {"type": "object", "properties": {
        "version": {"const": "1.0"},
        "intents": {"type": "array", "items": intent, "minItems": 1, "maxItems": max_intents},
        "context_updates": {"type": "object", "maxProperties": 3},
        "confidence": {"type": "number", "minimum": 0, "maximum": 1, "x-frac": 2},
        "tts_summary": {"type": "string", "maxLength": summary_max},
        "follow_up_question": {"anyOf": [{"type": "string", "maxLength": summary_max}, {"type": "null"}]},
    }, "required": ["version", "intents", "context_updates", "confidence"]}


def native():
    from ..ops import _vwa_native  # type: ignore

    return _vwa_native


class CompiledGrammar:
    """A grammar bound to a tokenizer vocabulary (shared mask cache across requests)."""

    def __init__(self, ir_json: str, token_bytes: List[bytes], eos_ids: List[int], cache_cap: int = 8192):
        N = native()
        self.ir_json = ir_json
        self.grammar = N.Grammar(ir_json)
        self.vocab = N.Vocab(token_bytes, list(eos_ids))
        self.compiled = N.Compiled(self.grammar, self.vocab, cache_cap)
        self.words = self.vocab.words()
        self.vocab_size = self.vocab.size()

    def matcher(self, budget: int = 1 << 30):
        return native().Matcher(self.compiled, budget)

    def stats(self) -> dict:
        c = self.compiled
        return {"mask_cache_hits": c.hits, "mask_cache_misses": c.misses, "mask_miss_ms": round(c.miss_ms, 3)}


def intent_grammar(tokenizer, eos_ids: Optional[List[int]] = None, **kw) -> CompiledGrammar:
    ir = ir_from_json_schema(parse_response_schema(**kw))
    if eos_ids is None:
        eos_ids = [i for i in (tokenizer.token_to_id("<|eot_id|>"), tokenizer.token_to_id("<|end_of_text|>"),
                               tokenizer.token_to_id("<|endoftext|>")) if i is not None]
    return CompiledGrammar(ir, tokenizer.token_bytes(), eos_ids)
