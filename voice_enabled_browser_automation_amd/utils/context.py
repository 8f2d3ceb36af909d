"""Bounded conversation context (SURVEY.md §5.7 "cap context").

The reference merges every brain reply's ``context_updates`` into the connection's context with
no bound (apps/voice/src/server.ts:162-170), and the whole context is serialised into every
prompt (apps/brain/src/server.ts:104).  A long voice session therefore grows the prompt until it
no longer fits the model (here: ``max_model_len``), and every later command fails.

``merge_context`` keeps the merged object under a byte budget (compact JSON) by evicting the
OLDEST keys first; "age" is the order of the last update, so a key that keeps being refreshed
(url, query) stays.  ``cap_context`` applies the same budget to a context received over HTTP
(the brain caps whatever a client sends before it builds the prompt).
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional
from .env import knob

DEFAULT_MAX_BYTES = 2048  # ~600 Llama-3 tokens: the ~1.1k-token prompt stays well inside 4096


def max_context_bytes() -> int:
    try:
        return max(0, knob("VWA_CONTEXT_MAX_BYTES"))
    except ValueError:
        return DEFAULT_MAX_BYTES


def _size(obj: Any) -> int:
    return len(json.dumps(obj, separators=(",", ":"), ensure_ascii=False, default=str).encode("utf-8"))


def cap_context(ctx: Dict[str, Any], max_bytes: Optional[int] = None) -> Dict[str, Any]:
    """A copy of ``ctx`` (insertion order = age, oldest first) whose compact JSON fits
    ``max_bytes``: oldest keys are dropped first; a single value larger than the whole budget is
    dropped as well."""
    cap = max_context_bytes() if max_bytes is None else max_bytes
    out = dict(ctx)
    if _size(out) <= cap:
        return out
    # sizes per entry ("key":value,) -- evict from the front until the remainder fits
    sizes = {k: _size({k: v}) - 1 for k, v in out.items()}  # minus one brace pair, plus a comma
    total = 2 + sum(sizes.values())
    for k in list(out):
        if total <= cap:
            break
        total -= sizes.pop(k)
        del out[k]
    return out


def merge_context(ctx: Dict[str, Any], updates: Dict[str, Any], max_bytes: Optional[int] = None) -> Dict[str, Any]:
    """{...ctx, ...updates} with updated keys moved to the young end, then capped."""
    merged = {k: v for k, v in ctx.items() if k not in updates}
    merged.update(updates)
    return cap_context(merged, max_bytes)
