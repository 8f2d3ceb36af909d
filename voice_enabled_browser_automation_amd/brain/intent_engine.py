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
  request terminates with a schema-valid ParseResponse;
* **continuous batching**: concurrent requests (voice sessions) decode together, one ragged
  forward + one masked-sampling launch per iteration for all of them.

`FakeIntentEngine` is the test double (the reference mocks callLLMJSON with vi.spyOn,
apps/brain/test/parse.test.ts:7-21).
"""
from __future__ import annotations

import json
import threading
import time
from collections import deque
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..grammar import CompiledGrammar, intent_grammar
from .prompt import llama3_chat, messages_for


class IntentEngineError(RuntimeError):
    pass


@dataclass
class IntentRequest:
    """One in-flight parse: prompt -> sequence -> grammar matcher -> JSON bytes."""

    messages: List[Dict[str, str]]
    ids: List[int] = field(default_factory=list)
    seq: Any = None
    matcher: Any = None
    out: bytearray = field(default_factory=bytearray)
    feed: List[int] = field(default_factory=list)   # tokens to append before the next sample
    steps: int = 0
    forced: int = 0
    cached: int = 0
    t_submit: float = 0.0
    t_start: float = 0.0
    t_first: float = 0.0
    t_end: float = 0.0
    done: bool = False
    text: Optional[str] = None
    error: Optional[BaseException] = None
    future: Any = None
    diag: Optional[str] = None

    def stats(self, t_end: float) -> Dict[str, Any]:
        return dict(prompt_tokens=len(self.ids), cached_prefix_tokens=self.cached,
                    prefill_tokens=len(self.ids) - self.cached, decode_steps=self.steps, forced_tokens=self.forced,
                    output_chars=len(self.out), queue_ms=(self.t_start - self.t_submit) * 1e3,
                    prefill_ms=(self.t_first - self.t_start) * 1e3, decode_ms=(t_end - self.t_first) * 1e3,
                    total_ms=(t_end - self.t_start) * 1e3)


_TOK_PENDING = -0x7A7A7A7A  # never a token id nor the sampler's -1 failure code


class LLMIntentEngine:
    """Grammar-constrained intent decoding with continuous batching.

    Every scheduler iteration (``step``) runs ONE ragged forward over all active requests --
    each contributes its pending rows (last sampled token + jump-forward tokens) and gets its
    logits row back (the LM head runs on one row per request) -- then one masked sampling
    launch for all of them.  New requests are admitted between iterations (prefix-cached
    prompt, prefill of all but the last prompt token, which joins the batched forward), and
    finished ones leave immediately, so a burst of voice sessions shares every weight read.
    """

    name = "llm"

    def __init__(self, engine, tokenizer, grammar: Optional[CompiledGrammar] = None, *, budget_chars: int = 512,
                 temperature: float = 0.1, max_steps: int = 400, seed: int = 0, max_active: Optional[int] = None,
                 chat_format: Callable[[List[Dict[str, str]]], Tuple[str, str]] = llama3_chat):
        self.engine = engine
        self.chat_format = chat_format
        self.tok = tokenizer
        self.grammar = grammar or intent_grammar(tokenizer)
        self.budget_chars = budget_chars
        self.temperature = temperature
        self.max_steps = max_steps
        self.max_active = max_active or engine.max_seqs
        self.max_rows = engine.bufs.max_rows
        dev = engine.device
        self.dev = dev
        pin = dev.type == "cuda"
        self._cuda_index = (dev.index if dev.index is not None else torch.cuda.current_device()) if pin else None
        R, W = self.max_active, self.grammar.words
        self.h_mask = torch.zeros(R, W, dtype=torch.int32, pin_memory=pin)
        self.h_mask_np = self.h_mask.numpy()
        self.d_mask = torch.zeros(R, W, dtype=torch.int32, device=dev)
        self.d_temp = torch.full((R,), float(temperature), dtype=torch.float32, device=dev)
        self.d_seed = torch.tensor([seed], dtype=torch.int64, device=dev)
        self.d_step = torch.zeros(1, dtype=torch.int32, device=dev)
        self.d_tok = torch.zeros(R, dtype=torch.int32, device=dev)
        self.h_tok = torch.zeros(R, dtype=torch.int32, pin_memory=pin)
        self.h_tok_np = self.h_tok.numpy()
        # wait for the sampled tokens by polling the pinned readback buffer (sentinel -> token)
        # instead of a stream synchronize: the GPU idles from the sampler's end until the host
        # has posted the next step, so the wake-up latency is on the critical path
        self.spin_wait = pin and ops.env_flag("VWA_SPIN_WAIT")
        # LM head under the grammar mask (LLMEngine.head_logits): the vocab tiles no row may sample
        # are skipped -- 42 % of the tiles live per step on average on the intent grammar
        self.masked_head = ops.env_flag("VWA_MASKED_HEAD")
        # zero-copy host buffers (GPU): the LM head and the sampler read the grammar masks straight
        # from the pinned host rows and the sampler stores the tokens into pinned host memory -- no
        # H2D mask copy and no D2H token copy per step (each a DMA start on the critical path)
        self.zero_copy = pin and ops.env_flag("VWA_ZERO_COPY")
        self.part_val = torch.zeros(R * 64, dtype=torch.float32, device=dev)
        self.part_idx = torch.zeros(R * 64, dtype=torch.int32, device=dev)
        self.last_stats: Dict[str, Any] = {}
        self.last_batch: List[Dict[str, Any]] = []
        self.batch_stats = dict(iterations=0, rows=0, sampled=0, max_active=0)
        # host-side time per scheduler phase (where a decode step's wall time goes)
        self.timing = dict(build_launch_ms=0.0, mask_ms=0.0, sample_launch_ms=0.0, gpu_wait_ms=0.0, post_ms=0.0,
                           admit_prefill_ms=0.0)
        self._prefix_ids: Dict[str, List[int]] = {}
        self._head_len = 0
        self.waiting: Deque[IntentRequest] = deque()
        self.active: List[IntentRequest] = []
        self._lock = threading.Lock()
        self._wake = threading.Condition(self._lock)
        self._thread: Optional[threading.Thread] = None
        self._stop = False

    # ------------------------------------------------------------------ helpers
    def _encode_prompt(self, messages) -> List[int]:
        head, tail = self.chat_format(messages)
        ids = self._prefix_ids.get(head)
        if ids is None:
            ids = self.tok.encode(head)
            self._prefix_ids = {head: ids}
        self._head_len = len(ids)
        return ids + self.tok.encode(tail)

    def grammar_bytes(self, tok: int) -> bytes:
        return self.tok.token_bytes()[tok]

    def _jump_forward(self, r: IntentRequest) -> None:
        forced = r.matcher.forced_prefix()
        if forced:
            r.matcher.accept_bytes(forced)
            r.out += forced
            # the grammar forces a small set of strings (JSON syntax, keys, enum values): their
            # standalone encodings are cached (a tokenizer call is ~9 us, 1-2 per sampled token)
            cache = self.__dict__.setdefault("_forced_ids", {})
            ftoks = cache.get(forced)
            if ftoks is None:
                ftoks = self.tok.encode(forced.decode("ascii"))
                if len(cache) < 8192:
                    cache[forced] = ftoks
            r.forced += len(ftoks)
            r.feed += ftoks

    def _admit(self, r: IntentRequest) -> None:
        """Admit one request on its own (prefill included)."""
        self._admit_begin(r)
        self.engine.prefill(r.seq, upto=len(r.ids) - 1)
        self._admit_end(r)

    def _admit_begin(self, r: IntentRequest) -> None:
        """Prompt -> sequence (prefix-cache match) + grammar matcher; the prefill is left to the
        caller (batched over every request admitted in the same iteration)."""
        eng = self.engine
        r.t_start = time.perf_counter()
        r.ids = self._encode_prompt(r.messages)
        r.matcher = self.grammar.matcher(self.budget_chars)
        if r.matcher.min_completion() > self.budget_chars:
            raise IntentEngineError(f"budget_chars={self.budget_chars} is below the shortest schema-valid "
                                    f"answer ({r.matcher.min_completion()} chars)")
        r.seq = eng.new_sequence(r.ids)
        r.cached = r.seq.n_computed
        if r.cached >= len(r.ids):  # whole prompt cached: recompute its last token for logits
            r.seq.n_computed = r.cached = len(r.ids) - 1

    def _admit_end(self, r: IntentRequest) -> None:
        r.t_first = time.perf_counter()
        r.feed = [r.ids[-1]]  # the last prompt token joins the batched step
        self._jump_forward(r)

    def _finish(self, r: IntentRequest, error: Optional[BaseException] = None) -> None:
        r.done = True
        r.error = error
        if error is None:
            r.text = r.out.decode("utf-8")
        if r.seq is not None:
            # only the static system + few-shot prefix is shared across requests; the request's
            # own suffix and answer are never served from cache (no replay of repeated commands)
            self.engine.free_sequence(r.seq, publish_upto=self._head_len)
            r.seq = None
        r.t_end = time.perf_counter()
        self.last_stats = r.stats(r.t_end)
        if r.future is not None:
            if error is None:
                r.future.set_result(r.text)
            else:
                r.future.set_exception(error)

    # ------------------------------------------------------------------ scheduler
    def submit(self, messages: List[Dict[str, str]], future=None) -> IntentRequest:
        r = IntentRequest(messages=messages, t_submit=time.perf_counter(), future=future)
        with self._lock:
            self.waiting.append(r)
            self._wake.notify()
        return r

    def has_work(self) -> bool:
        return bool(self.active or self.waiting)

    def step(self) -> List[IntentRequest]:
        """One scheduler iteration; returns the requests that finished in it."""
        finished: List[IntentRequest] = []
        admitted: List[IntentRequest] = []
        while len(self.active) + len(admitted) < self.max_active:
            with self._lock:
                if not self.waiting:
                    break
                r = self.waiting.popleft()
            try:
                self._admit_begin(r)
                admitted.append(r)
            except Exception as e:  # noqa: BLE001
                self._finish(r, e)
                finished.append(r)
        if admitted:
            # ONE batched prefill of every admitted request's prompt suffix (all but its last
            # token, which joins the decode step below)
            ta = time.perf_counter()
            try:
                self.engine.prefill_batch([(r.seq, len(r.ids) - 1) for r in admitted])
                self.timing["admit_prefill_ms"] += (time.perf_counter() - ta) * 1e3
            except Exception as e:  # noqa: BLE001
                if getattr(getattr(self.engine.model, "tp", None), "size", 1) > 1:
                    raise  # TP: lockstep is lost -- brain/tp_engine.py ends the group
                for r in admitted:
                    self._finish(r, e)
                    finished.append(r)
                admitted = []
            for r in admitted:
                self._admit_end(r)
                self.active.append(r)
        if not self.active:
            return finished
        # rows: each request's pending tokens; requests that do not fit wait one iteration, a
        # feed longer than the row cap is consumed in pieces (sampled once it is exhausted)
        rows, last, batch, budget = [], [], [], self.max_rows
        for r in self.active:
            if not r.feed or budget <= 0:
                continue
            take = r.feed[:budget]
            if len(take) < len(r.feed) and rows:
                continue
            rows += [(r.seq, t) for t in take]
            budget -= len(take)
            r.feed = r.feed[len(take):]
            if not r.feed:
                last.append(len(rows) - 1)
                batch.append(r)
        if not rows:
            return finished
        tm = self.timing
        t0 = time.perf_counter()
        if last:
            self.engine.run_rows(rows, logits_for=last, check=False, defer_head=True)
        else:
            # only part of one long feed fits this iteration: its rows still have to reach the KV
            # cache (nothing is sampled -- no LM head -- so the step is verified synchronously)
            self.engine.run_rows(rows, logits_for=[len(rows) - 1], check=True, defer_head=True)
        t1 = time.perf_counter()
        tm["build_launch_ms"] += (t1 - t0) * 1e3
        self.batch_stats["iterations"] += 1
        self.batch_stats["rows"] += len(rows)
        self.batch_stats["max_active"] = max(self.batch_stats["max_active"], len(self.active))
        if not batch:
            return finished
        n = len(batch)
        for i, r in enumerate(batch):  # CPU grammar masks overlap the in-flight forward
            r.matcher.fill_mask(self.h_mask_np[i])
        t2 = time.perf_counter()
        if not self.zero_copy:
            self.d_mask[:n].copy_(self.h_mask[:n], non_blocking=True)
        mask = self.h_mask if self.zero_copy else self.d_mask
        # the LM head under the same masks: only vocab tiles some row may sample are computed
        logits = self.engine.head_logits(col_mask=mask if self.masked_head else None, mask_rows=n, gather=False)
        toks = self._sample(logits, n, self.engine.step_fail_word())
        self.engine.host_synced()  # the sampled tokens are back: the step's staging copy has run
        if any(t == -2 for t in toks):
            # the forward's chained launch timed out at a grid barrier (tokens -2 from the
            # sampler's fail word): re-run the step on the per-kernel path and sample again
            logits = self.engine.recover_step()
            toks = self._sample(logits, n, None)
        t4 = time.perf_counter()
        tm["mask_ms"] += (t2 - t1) * 1e3
        tm["sample_launch_ms"] += (self._t3 - t2) * 1e3
        tm["gpu_wait_ms"] += (t4 - self._t3) * 1e3
        self.batch_stats["sampled"] += n
        if any(t == -1 for t in toks):
            self._diagnose(batch, toks, logits, n)
        self._accept(batch, toks, finished)
        if finished:
            self.active = [r for r in self.active if not r.done]
        tm["post_ms"] += (time.perf_counter() - t4) * 1e3
        return finished

    def _sample(self, logits: torch.Tensor, n: int, fail_word: Optional[torch.Tensor]) -> List[int]:
        """Masked sampling of the n logits rows (masks already in d_mask) and the token readback."""
        zc = self.zero_copy
        if zc and self.spin_wait:
            self.h_tok_np[:n] = _TOK_PENDING  # before the launch: the sampler stores into it directly
        self.engine.sample(logits, mask=self.h_mask if zc else self.d_mask,
                           temperature=self.d_temp if self.temperature > 0 else None, seed=self.d_seed,
                           step=self.d_step, out_tokens=self.h_tok if zc else self.d_tok,
                           part_val=self.part_val[: n * 64], part_idx=self.part_idx[: n * 64], fail_word=fail_word)
        if self.dev.type == "cuda" and zc and self.spin_wait:
            t3 = time.perf_counter()
            hv = self.h_tok_np[:n]
            deadline = t3 + 0.05
            while (hv == _TOK_PENDING).any():
                if time.perf_counter() > deadline:  # long step: block on the stream instead
                    torch.cuda.current_stream().synchronize()
                    break
            # (the sampler's system-scope int32 stores land whole; the masks it and the LM head
            # read are done by then -- the host may overwrite them for the next step)
            toks = hv.tolist()
        elif self.dev.type == "cuda":
            if self.spin_wait:
                self.h_tok_np[:n] = _TOK_PENDING
            if zc:
                t3 = time.perf_counter()
                torch.cuda.current_stream().synchronize()
                self._t3 = t3
                return self.h_tok[:n].tolist()
            self.h_tok[:n].copy_(self.d_tok[:n], non_blocking=True)
            t3 = time.perf_counter()
            if self.spin_wait:
                hv = self.h_tok_np[:n]
                deadline = t3 + 0.05
                while (hv == _TOK_PENDING).any():
                    if time.perf_counter() > deadline:  # long step (or none in flight): block instead
                        break
            # always end on the stream: the spin only sees the copy START landing -- its bytes are
            # not written atomically per int32 (seen with two processes on one GPU: the low byte
            # of a token over the sentinel's upper bytes, 0x85858561), so the values are read
            # only after the copy completed.  Polled with stream queries (a blocking synchronize
            # measured +38 us per iteration: its wake-up, not the copy)
            st = torch.cuda.current_stream()
            if self.spin_wait:
                while not st.query():
                    if time.perf_counter() > deadline:
                        break
            st.synchronize()
            toks = self.h_tok[:n].tolist()
        else:
            t3 = time.perf_counter()
            toks = self.d_tok[:n].tolist()
        self._t3 = t3
        return toks

    def _diagnose(self, batch, toks, logits, n) -> None:
        """A -1 token means no admissible token had a finite logit: record what the row looked like
        (mask population, finite admissible logits) in the request's error for the logs."""
        for i, (r, t) in enumerate(zip(batch, toks)):
            if t != -1:
                continue
            words = torch.from_numpy(self.h_mask_np[i].copy()).to(torch.int64) & 0xFFFFFFFF
            bits = ((words[:, None] >> torch.arange(32)[None, :]) & 1).reshape(-1).bool()
            row = logits[i].float().cpu()
            lo = self.engine.model.v_start if getattr(self.engine.model, "tp", None) and self.engine.model.tp.size > 1 else 0
            adm = bits[lo : lo + row.shape[0]]
            vals = row[adm[: row.shape[0]]]
            r.diag = (f"row {i}/{n}: {int(bits.sum())} admissible tokens, {int(torch.isfinite(vals).sum())} finite "
                      f"admissible logits, row finite {int(torch.isfinite(row).sum())}/{row.numel()}, step {r.steps}, "
                      f"out {bytes(r.out[-40:])!r}")

    def _accept(self, batch: List[IntentRequest], toks: List[int], finished: List[IntentRequest]) -> None:
        for r, tok in zip(batch, toks):
            r.steps += 1
            m = r.matcher
            if tok < 0 or not m.accept_token(tok):
                self.batch_stats["rejects"] = self.batch_stats.get("rejects", 0) + 1
                self._finish(r, IntentEngineError(f"sampler returned a token the grammar rejects ({tok})"
                                                  + (f": {r.diag}" if getattr(r, "diag", None) else "")))
            else:
                r.out += self.grammar_bytes(tok)
                if m.is_accept():
                    r.seq.tokens.append(tok)
                    self._finish(r)
                elif r.steps >= self.max_steps:
                    self._finish(r, IntentEngineError("decode step limit reached"))
                else:
                    r.feed = [tok]
                    self._jump_forward(r)
            if r.done:
                finished.append(r)

    def engine_stats(self) -> Dict[str, Any]:
        """Scheduler + KV-cache state for /metrics (batch size, KV utilisation, grammar cache)."""
        eng = self.engine
        bm = eng.blocks
        used = bm.num_blocks - bm.n_free()
        it = max(1, self.batch_stats["iterations"])
        out = {"active": len(self.active), "waiting": len(self.waiting),
               "kv_blocks_used": used, "kv_blocks_total": bm.num_blocks,
               "kv_utilisation": round(used / max(1, bm.num_blocks), 4),
               "rows_per_iteration": round(self.batch_stats["rows"] / it, 3),
               "samples_per_iteration": round(self.batch_stats["sampled"] / it, 3),
               "grammar_rejects": self.batch_stats.get("rejects", 0),
               "host_ms": {k: round(v, 1) for k, v in self.timing.items()}}
        out.update(self.grammar.stats())
        out.update({k: v for k, v in eng.stats.items()})
        return out

    def run_until_idle(self) -> None:
        while self.has_work():
            self.step()

    def generate_many(self, messages_list: List[List[Dict[str, str]]]) -> List[str]:
        """Decode a batch of requests together (continuous batching); raises the first error."""
        reqs = [self.submit(m) for m in messages_list]
        while not all(r.done for r in reqs):
            self.step()
        self.last_batch = [dict(r.stats(r.t_end), latency_ms=(r.t_end - r.t_submit) * 1e3) for r in reqs]
        for r in reqs:
            if r.error is not None:
                raise r.error
        return [r.text for r in reqs]

    def generate(self, messages: List[Dict[str, str]]) -> str:
        return self.generate_many([messages])[0]

    def __call__(self, messages: List[Dict[str, str]]) -> Any:
        """callLLMJSON parity: returns the parsed JSON object."""
        return json.loads(self.generate(messages))

    def parse(self, request: Dict[str, Any], repair: bool = False) -> Any:
        return self(messages_for(request, repair=repair))

    def parse_many(self, requests: List[Dict[str, Any]]) -> List[Any]:
        return [json.loads(t) for t in self.generate_many([messages_for(r) for r in requests])]

    # ------------------------------------------------------------------ background serving
    def start(self) -> None:
        """Run the scheduler on a background thread (the brain service submits into it)."""
        if self._thread is not None:
            return
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="intent-scheduler", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        with self._lock:
            self._stop = True
            self._wake.notify()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None

    def _loop(self) -> None:
        if self.dev.type == "cuda":
            # the scheduler thread inherits no current device: use the model's ("cuda" with no
            # index means the device that was current when the engine was built)
            torch.cuda.set_device(self._cuda_index)
        while True:
            with self._lock:
                while not self._stop and not self.waiting and not self.active:
                    self._wake.wait()
                if self._stop:
                    return
            try:
                self.step()
            except Exception as e:  # noqa: BLE001  (fail every in-flight request, keep serving)
                for r in self.active:
                    self._finish(r, e)
                self.active = []

    def submit_async(self, messages: List[Dict[str, str]]):
        """concurrent.futures.Future resolved with the JSON text (requires start())."""
        fut: Future = Future()
        self.submit(messages, future=fut)
        return fut


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
