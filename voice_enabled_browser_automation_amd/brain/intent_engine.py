"""Intent engines: the on-node replacement of `callLLMJSON` (apps/brain/src/llm.ts:19-30).

`LLMIntentEngine` runs the Llama-class model through runtime.engine.LLMEngine with
grammar-constrained decoding:

* the static prompt prefix is served from the paged-KV prefix cache; only the request suffix is
  prefilled;
* **jump-forward**: whenever the grammar admits exactly one continuation (keys, punctuation,
  closing brackets, budget-forced closes) those bytes are tokenised and appended in the SAME
  forward as the previously sampled token (one ragged step of 1 + k rows), so forced JSON
  structure costs no extra decode steps;
* the token mask for step t is computed on the CPU (native grammar engine, GIL released) while
  the GPU runs step t's forward; the mask upload + sampling kernel follow on the same stream;
* a character budget (``budget_chars``) guarantees the JSON can always be closed, so every
  request terminates with a schema-valid ParseResponse.

`FakeIntentEngine` is the test double (the reference mocks callLLMJSON with vi.spyOn,
apps/brain/test/parse.test.ts:7-21).
"""
from __future__ import annotations

import json
import time
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..grammar import CompiledGrammar, intent_grammar
from .prompt import llama3_chat, messages_for


class IntentEngineError(RuntimeError):
    pass


class LLMIntentEngine:
    name = "llm"

    def __init__(self, engine, tokenizer, grammar: Optional[CompiledGrammar] = None, *, budget_chars: int = 512,
                 temperature: float = 0.1, max_steps: int = 400, seed: int = 0):
        self.engine = engine
        self.tok = tokenizer
        self.grammar = grammar or intent_grammar(tokenizer)
        self.budget_chars = budget_chars
        self.temperature = temperature
        self.max_steps = max_steps
        dev = engine.device
        self.dev = dev
        pin = dev.type == "cuda"
        W = self.grammar.words
        self.h_mask = torch.zeros(1, W, dtype=torch.int32, pin_memory=pin)
        self.h_mask_np = self.h_mask.numpy().reshape(-1)
        self.d_mask = torch.zeros(1, W, dtype=torch.int32, device=dev)
        self.d_temp = torch.full((1,), float(temperature), dtype=torch.float32, device=dev)
        self.d_seed = torch.tensor([seed], dtype=torch.int64, device=dev)
        self.d_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.d_tok = torch.zeros(1, dtype=torch.int32, device=dev)
        self.h_tok = torch.zeros(1, dtype=torch.int32, pin_memory=pin)
        self.part_val = torch.zeros(64, dtype=torch.float32, device=dev)
        self.part_idx = torch.zeros(64, dtype=torch.int32, device=dev)
        self.last_stats: Dict[str, Any] = {}
        self._prefix_ids: Dict[str, List[int]] = {}
        self._head_len = 0

    # ------------------------------------------------------------------ helpers
    def _encode_prompt(self, messages) -> List[int]:
        head, tail = llama3_chat(messages)
        ids = self._prefix_ids.get(head)
        if ids is None:
            ids = self.tok.encode(head)
            self._prefix_ids = {head: ids}
        self._head_len = len(ids)
        return ids + self.tok.encode(tail)

    def _sample(self, logits: torch.Tensor) -> int:
        ops.sample(logits, mask=self.d_mask, temperature=self.d_temp if self.temperature > 0 else None,
                   seed=self.d_seed, step=self.d_step, out_tokens=self.d_tok, part_val=self.part_val,
                   part_idx=self.part_idx)
        if self.dev.type == "cuda":
            self.h_tok.copy_(self.d_tok, non_blocking=True)
            torch.cuda.current_stream().synchronize()
            return int(self.h_tok[0])
        return int(self.d_tok[0])

    def _run(self, seq, toks: List[int]) -> torch.Tensor:
        logits = None
        for i in range(0, len(toks), 64):
            chunk = toks[i : i + 64]
            logits = self.engine.run_rows([(seq, t) for t in chunk])[-1:]
        return logits

    # ------------------------------------------------------------------ generation
    def generate(self, messages: List[Dict[str, str]]) -> str:
        t0 = time.perf_counter()
        eng = self.engine
        ids = self._encode_prompt(messages)
        seq = eng.new_sequence(ids)
        cached = seq.n_computed
        try:
            logits = eng.prefill(seq)
            t_prefill = time.perf_counter()
            m = self.grammar.matcher(self.budget_chars)
            out = bytearray()
            steps = forced_toks = 0
            forced = m.forced_prefix()
            if forced:
                m.accept_bytes(forced)
                out += forced
                ftoks = self.tok.encode(forced.decode("ascii"))
                forced_toks += len(ftoks)
                logits = self._run(seq, ftoks)
            while not m.is_accept():
                if steps >= self.max_steps:
                    raise IntentEngineError("decode step limit reached")
                m.fill_mask(self.h_mask_np)  # CPU, overlaps the in-flight forward
                self.d_mask.copy_(self.h_mask, non_blocking=True)
                tok = self._sample(logits)
                steps += 1
                if tok < 0 or not m.accept_token(tok):
                    raise IntentEngineError(f"sampler returned a token the grammar rejects ({tok})")
                out += self.grammar_bytes(tok)
                if m.is_accept():
                    seq.tokens.append(tok)
                    break
                forced = m.forced_prefix()
                ftoks: List[int] = []
                if forced:
                    m.accept_bytes(forced)
                    out += forced
                    ftoks = self.tok.encode(forced.decode("ascii"))
                    forced_toks += len(ftoks)
                logits = self._run(seq, [tok] + ftoks)
            t_end = time.perf_counter()
            self.last_stats = dict(prompt_tokens=len(ids), cached_prefix_tokens=cached,
                                   prefill_tokens=len(ids) - cached, decode_steps=steps, forced_tokens=forced_toks,
                                   output_chars=len(out), prefill_ms=(t_prefill - t0) * 1e3,
                                   decode_ms=(t_end - t_prefill) * 1e3, total_ms=(t_end - t0) * 1e3)
            return out.decode("utf-8")
        finally:
            # only the static system + few-shot prefix is shared across requests; the request's
            # own suffix and answer are never served from cache (no replay of repeated commands)
            eng.free_sequence(seq, publish_upto=self._head_len)

    def grammar_bytes(self, tok: int) -> bytes:
        return self.tok.token_bytes()[tok]

    def __call__(self, messages: List[Dict[str, str]]) -> Any:
        """callLLMJSON parity: returns the parsed JSON object."""
        return json.loads(self.generate(messages))

    def parse(self, request: Dict[str, Any], repair: bool = False) -> Any:
        return self(messages_for(request, repair=repair))


class FakeIntentEngine:
    """Deterministic stand-in (tests / CPU-only service runs): returns a canned or computed reply."""

    name = "fake"

    def __init__(self, reply: Optional[Any] = None, fn: Optional[Callable[[List[Dict[str, str]]], Any]] = None,
                 fail: Optional[BaseException] = None):
        self.reply = reply
        self.fn = fn
        self.fail = fail
        self.calls: List[List[Dict[str, str]]] = []

    def __call__(self, messages):
        self.calls.append(messages)
        if self.fail is not None:
            raise self.fail
        if self.fn is not None:
            return self.fn(messages)
        if isinstance(self.reply, list):  # sequence of replies (first call, repair call, ...)
            return self.reply[min(len(self.calls) - 1, len(self.reply) - 1)]
        return self.reply

    def parse(self, request, repair=False):
        return self(messages_for(request, repair=repair))


def keyword_intents(messages) -> Dict[str, Any]:
    """Rule-based fallback engine used when no model is configured (keeps /parse usable on CPU)."""
    req = json.loads(messages[-1]["content"]) if messages[-1]["role"] == "user" else json.loads(messages[-2]["content"])
    text = req.get("text", "").lower()
    it: Dict[str, Any]
    if text.startswith("search") or "search for" in text:
        q = text.split("search", 1)[1].replace("for ", "", 1).strip()
        it = {"type": "search", "args": {"query": q}, "priority": 0, "requires_confirmation": False}
    elif text.startswith(("go to", "open ", "navigate")) and "." in text:
        url = text.split()[-1]
        it = {"type": "navigate", "args": {"url": url if url.startswith("http") else "https://" + url}, "priority": 0,
              "requires_confirmation": False}
    elif "scroll" in text:
        it = {"type": "scroll", "args": {"direction": "up" if "up" in text else "down"}, "priority": 0,
              "requires_confirmation": False}
    elif "back" in text:
        it = {"type": "back", "args": {}, "priority": 0, "requires_confirmation": False}
    elif "screenshot" in text:
        it = {"type": "screenshot", "args": {"label": "voice"}, "priority": 0, "requires_confirmation": False}
    else:
        return {"version": "1.0", "intents": [{"type": "unknown", "args": {}, "priority": 0,
                                               "requires_confirmation": False}],
                "context_updates": {}, "confidence": 0.4, "follow_up_question": "What should I do on the page?"}
    return {"version": "1.0", "intents": [it], "context_updates": {}, "confidence": 0.7,
            "tts_summary": f"Running {it['type']}."}
