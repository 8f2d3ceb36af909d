"""Streaming recognition with Deepgram-compatible events (replaces the Deepgram live connection,
apps/voice/src/deepgram.ts:33-51).

The voice server feeds raw PCM16 LE 16 kHz mono frames (the UI sends ~60 ms packets,
apps/web/src/App.tsx:279-288).  A session keeps the current utterance buffer and:

* energy VAD on 20 ms frames tracks speech start and trailing silence;
* every ``partial_every_s`` of new speech it runs a recognition pass and emits an interim result
  (``is_final: false``), like Deepgram's interim_results;
* **local agreement**: the token prefix on which the last two interim hypotheses agree is
  *committed* -- later passes force it as the decoder prefix (prefilled in one ragged step with
  the SOT tokens) and decode only the continuation, so a long utterance does not re-decode its
  whole transcript at every partial, and the committed words never flicker;
* on an endpoint (``endpoint_silence_s`` of silence after speech, ``VWA_ENDPOINT_MS``), on
  ``flush()`` (client end-of-utterance) or when the 30 s Whisper window is full, it emits a final
  result (``is_final: true, speech_final: true``) and starts a new utterance;
* **speculative final**: once the trailing silence reaches ``spec_silence_s``
  (``VWA_SPEC_FINAL_MS``, shorter than the endpoint) the final recognition pass is started in the
  background on the utterance so far; if the silence lasts to the endpoint its result IS the final
  (no pass after the endpoint), if speech resumes it is discarded -- so the final costs the
  endpoint wait alone, not endpoint + a recognition pass (Deepgram's live endpointing finalises
  without a client-side wait, deepgram.ts:36-45);
* the VAD threshold adapts to the noise floor (``max(energy_threshold, noise_mult x floor)``; the
  floor is bootstrapped from a stationary mic-open period and kept by the non-speech frames), so a
  noisy microphone still endpoints.

Recognition passes go through a *recognizer* (``recognize(pcm, prefix) -> Hypothesis``).
``AsrBatcher`` is the serving recognizer: one scheduler thread per GPU engine that gathers the
pending passes of ALL live sessions and runs them as one batch (``AsrEngine.decode_many``: one
batched encoder pass, then one ragged decode step per token for every session) -- the
session-DP unit of a GPU.

Events use the Deepgram ``Results`` shape that the unchanged UI and voice logic read
(``payload.is_final``, ``payload.channel.alternatives[0].transcript``; apps/voice/src/server.ts:112,123).
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np


def results_event(text: str, *, is_final: bool, start: float, duration: float, model: str,
                  confidence: float = 0.0) -> Dict:
    return {
        "type": "Results",
        "channel_index": [0, 1],
        "duration": round(duration, 3),
        "start": round(start, 3),
        "is_final": is_final,
        "speech_final": is_final,
        "channel": {"alternatives": [{"transcript": text, "confidence": confidence, "words": []}]},
        "metadata": {"model_info": {"name": model}},
    }


@dataclass
class Hypothesis:
    """One recognition pass: the full transcript's token ids (forced prefix included) and text."""

    tokens: List[int] = field(default_factory=list)
    text: str = ""


class TextRecognizer:
    """Adapter for a plain ``transcribe(pcm) -> str`` callable (tests, CPU stand-ins): no token
    ids, so no committed prefix (local agreement is a no-op)."""

    def __init__(self, fn: Callable[[np.ndarray], str]):
        self.fn = fn

    def recognize(self, pcm: np.ndarray, prefix: Sequence[int] = ()) -> Hypothesis:
        return Hypothesis([], self.fn(pcm).strip())


def _as_recognizer(r: Any):
    return r if hasattr(r, "recognize") else TextRecognizer(r)


def recognize_async(rec: Any, pcm: np.ndarray, prefix: Sequence[int] = ()) -> Future:
    """A recognition pass that runs in the background when the recognizer can (AsrBatcher: queued
    for the next GPU batch), else synchronously into an already completed Future."""
    if hasattr(rec, "recognize_async"):
        return rec.recognize_async(pcm, prefix)
    fut: Future = Future()
    try:
        fut.set_result(rec.recognize(pcm, prefix))
    except BaseException as e:  # noqa: BLE001
        fut.set_exception(e)
    return fut


def common_prefix(a: Sequence[int], b: Sequence[int]) -> int:
    n = min(len(a), len(b))
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


class StreamingAsrSession:
    def __init__(self, recognizer: Any, *, rate: int = 16000, model_name: str = "whisper",
                 partial_every_s: float = 1.0, endpoint_silence_s: Optional[float] = None,
                 energy_threshold: Optional[float] = None, max_window_s: float = 30.0, min_speech_s: float = 0.2,
                 local_agreement: bool = True, spec_silence_s: Optional[float] = None,
                 noise_mult: Optional[float] = None):
        from ..utils.env import knob

        self.rec = _as_recognizer(recognizer)
        self.rate = rate
        self.model_name = model_name
        self.partial_every = int(partial_every_s * rate)
        if endpoint_silence_s is None:
            endpoint_silence_s = knob("VWA_ENDPOINT_MS") / 1000.0
        if spec_silence_s is None:
            spec_silence_s = knob("VWA_SPEC_FINAL_MS") / 1000.0
        self.endpoint = int(endpoint_silence_s * rate)
        # speculative final pass after this much trailing silence (0: off; never later than the endpoint)
        self.spec_at = min(int(spec_silence_s * rate), self.endpoint) if spec_silence_s > 0 else 0
        self.thresh = knob("VWA_VAD_THRESHOLD") if energy_threshold is None else energy_threshold
        self.noise_mult = knob("VWA_VAD_NOISE_MULT") if noise_mult is None else noise_mult
        self.noise_floor = 0.0  # tracked non-speech frame RMS (0: not known)
        self._boot: Optional[List[float]] = []  # frame RMS of the stream's first 300 ms
        self._spec: Optional[Future] = None  # the speculative final pass in flight
        self.max_window = int(max_window_s * rate)
        self.min_speech = int(min_speech_s * rate)
        self.local_agreement = local_agreement
        self.frame = rate // 50  # 20 ms
        # the utterance buffer: preallocated to the window (+ one packet), appended in place --
        # no per-frame re-concatenation of the whole utterance
        self._pcm = np.zeros(self.max_window + 4 * rate, dtype=np.int16)
        self._n = 0
        self._carry = b""
        self.t_offset = 0.0          # stream time of buf[0]
        self.speech = 0              # speech samples in the utterance
        self.trailing_silence = 0
        self.since_partial = 0
        self.last_partial = ""
        self.committed: List[int] = []   # agreed token prefix of the current utterance
        self.prev_tokens: List[int] = []  # previous interim hypothesis
        self.stats: Dict[str, float] = {"partials": 0, "finals": 0, "asr_ms": 0.0, "passes": 0,
                                        "committed_tokens": 0, "spec_started": 0, "spec_used": 0,
                                        "spec_discarded": 0}
        # on_speculative(text): called (from the recognizer's thread) when a speculative final pass
        # finishes while it still covers the utterance -- the voice server starts the brain on it
        # (voice/server.py: the brain's latency then overlaps the rest of the endpoint wait)
        self.on_speculative: Optional[Callable[[str], None]] = None
        # vad_events (Deepgram's live option of that name, off by default there too): push() also
        # returns {"type": "SpeechStarted"} when speech begins or resumes after a speculative final
        self.vad_events = False

    # ------------------------------------------------------------------ internals
    @property
    def buf(self) -> np.ndarray:
        """The current utterance's samples (a view of the preallocated buffer)."""
        return self._pcm[: self._n]

    def _append(self, fr: np.ndarray) -> None:
        if self._n + len(fr) > len(self._pcm):  # (never with the window cut; a safety net)
            self._pcm = np.concatenate([self._pcm, np.zeros(max(len(fr), len(self._pcm) // 2), dtype=np.int16)])
        self._pcm[self._n : self._n + len(fr)] = fr
        self._n += len(fr)

    def _run(self) -> Hypothesis:
        t0 = time.perf_counter()
        hyp = self.rec.recognize(self.buf, self.committed if self.local_agreement else ())
        self.stats["asr_ms"] += (time.perf_counter() - t0) * 1e3
        self.stats["passes"] += 1
        return hyp

    def _track_floor(self, rms: float) -> None:
        """Bootstrap the noise floor from the stream's first 300 ms (the mic-open moment) when that
        audio is stationary (frame RMS within 2x: hiss, hum -- not a speech onset) and quiet enough
        (mult x level <= 10 x the fixed threshold); afterwards the non-speech frames maintain it."""
        if self._boot is None or self.noise_mult <= 0.0:
            return
        self._boot.append(rms)
        if len(self._boot) < 15:
            return
        lo, hi = min(self._boot), max(self._boot)
        med = float(np.median(self._boot))
        if hi <= 2.0 * max(lo, 1e-6) and self.noise_mult * med <= 10.0 * self.thresh:
            self.noise_floor = max(self.noise_floor, med)
        self._boot = None

    def _floor_cap(self) -> float:
        """The highest noise floor the VAD tracks: the bootstrap's own ceiling (mult x floor <= 10 x
        the fixed threshold)."""
        return 10.0 * self.thresh / self.noise_mult if self.noise_mult > 0.0 else 0.0

    def _reset_utterance(self) -> None:
        self.t_offset += self._n / self.rate
        self._n = 0
        self.speech = self.trailing_silence = self.since_partial = 0
        self.last_partial = ""
        self.committed = []
        self.prev_tokens = []
        self._drop_spec()

    def _drop_spec(self) -> None:
        if self._spec is not None:
            self.stats["spec_discarded"] += 1
            self._spec = None

    def _start_spec(self) -> None:
        """The final pass, started during the trailing silence (see module docstring)."""
        self.stats["spec_started"] += 1
        self._spec_t0 = time.perf_counter()
        fut = recognize_async(self.rec, self.buf.copy(), self.committed if self.local_agreement else ())
        self._spec = fut
        if self.on_speculative is not None:
            fut.add_done_callback(self._spec_ready)

    def _spec_ready(self, fut: Future) -> None:
        if self._spec is not fut or fut.cancelled() or fut.exception() is not None:
            return  # (speech resumed meanwhile, or a failed pass: the endpoint runs the final itself)
        try:
            self.on_speculative(fut.result().text)
        except Exception:  # noqa: BLE001  (a listener failure must not break recognition)
            pass

    def _final(self, use_spec: bool = True) -> List[Dict]:
        out: List[Dict] = []
        if self.speech >= self.min_speech and len(self.buf):
            hyp = None
            if use_spec and self._spec is not None:
                try:
                    hyp = self._spec.result()
                    self.stats["spec_used"] += 1
                    self.stats["asr_ms"] += (time.perf_counter() - self._spec_t0) * 1e3
                    self.stats["passes"] += 1
                    self._spec = None
                except Exception:  # noqa: BLE001  (a failed background pass: run the final now)
                    self._drop_spec()
            if hyp is None:
                hyp = self._run()
            out.append(results_event(hyp.text, is_final=True, start=self.t_offset, duration=len(self.buf) / self.rate,
                                     model=self.model_name))
            self.stats["finals"] += 1
        self._reset_utterance()
        return out

    def _partial(self) -> List[Dict]:
        hyp = self._run()
        if self.local_agreement and hyp.tokens:
            # LocalAgreement-2: what two consecutive hypotheses agree on is stable
            n = common_prefix(self.prev_tokens, hyp.tokens)
            if n > len(self.committed):
                self.stats["committed_tokens"] += n - len(self.committed)
                self.committed = list(hyp.tokens[:n])
            self.prev_tokens = list(hyp.tokens)
        if hyp.text == self.last_partial:
            return []
        self.last_partial = hyp.text
        self.stats["partials"] += 1
        return [results_event(hyp.text, is_final=False, start=self.t_offset, duration=len(self.buf) / self.rate,
                              model=self.model_name)]

    # ------------------------------------------------------------------ API
    def push(self, data: bytes) -> List[Dict]:
        data = self._carry + bytes(data)
        if len(data) % 2:
            self._carry, data = data[-1:], data[:-1]
        else:
            self._carry = b""
        pcm = np.frombuffer(data, dtype="<i2")
        events: List[Dict] = []
        for i in range(0, len(pcm), self.frame):
            fr = pcm[i : i + self.frame]
            if len(fr) == 0:
                continue
            self._append(fr)
            rms = float(np.sqrt(np.mean(fr.astype(np.float32) ** 2)))
            self._track_floor(rms)
            if rms >= max(self.thresh, self.noise_mult * self.noise_floor):
                if self.vad_events and (self.speech == 0 or self._spec is not None):
                    # Deepgram's VAD event (vad_events): speech begins -- a new utterance, or the
                    # speaker resumed after a speculative final (the voice server holds / drops
                    # what it started on the previous words: voice/server.py commit policy)
                    events.append({"type": "SpeechStarted", "channel": [0, 1],
                                   "timestamp": round(self.t_offset + self._n / self.rate, 3)})
                self.speech += len(fr)
                self.trailing_silence = 0
                self._drop_spec()  # speech resumed: the speculative final no longer covers the utterance
            else:
                self.trailing_silence += len(fr)
                # non-speech frames: the floor falls fast to quieter frames, rises slowly (0.3 % /
                # frame) and only between utterances (never from an utterance's own pauses), capped
                # at the bootstrap's ceiling -- steady soft speech or a TV in the background cannot
                # walk the threshold up until quiet speakers stop being detected
                if self.noise_floor > 0.0:
                    if rms < self.noise_floor:
                        self.noise_floor = 0.8 * self.noise_floor + 0.2 * rms
                    elif self.speech == 0:
                        self.noise_floor = min(rms, self.noise_floor * 1.003, self._floor_cap())
            if self.speech > 0:
                self.since_partial += len(fr)
            if self.speech >= self.min_speech and self.trailing_silence >= self.endpoint:
                events += self._final()
            elif len(self.buf) >= self.max_window:
                events += self._final(use_spec=False)
            elif (self.spec_at and self._spec is None and self.speech >= self.min_speech
                  and self.trailing_silence >= self.spec_at):
                self._start_spec()
            elif self.speech == 0 and self.trailing_silence >= self.endpoint:
                # leading silence: drop it, keep the stream clock
                self.t_offset += self._n / self.rate
                self._n = 0
                self.trailing_silence = 0
        if self.speech >= self.min_speech and self.since_partial >= self.partial_every:
            self.since_partial = 0
            events += self._partial()
        return events

    def flush(self) -> List[Dict]:
        return self._final()  # (a speculative pass in flight covers the utterance: speech since would have dropped it)

    def close(self) -> None:
        pass


# ---------------------------------------------------------------------------------- recognizers
class EngineRecognizer:
    """Serial recognizer on an AsrEngine (one pass at a time, caller's thread)."""

    def __init__(self, asr_engine, *, max_tokens: int = 96):
        self.eng = asr_engine
        self.max_tokens = max_tokens

    def recognize(self, pcm: np.ndarray, prefix: Sequence[int] = ()) -> Hypothesis:
        prefix = list(prefix)[: self.eng.max_prefix()]  # the prefix the decoder actually forces
        toks = self.eng.decode_many([self.eng.pcm_to_audio(pcm)], [prefix], max_tokens=self.max_tokens)[0]
        full = prefix + toks
        return Hypothesis(full, self.eng.tok.decode(full).strip())


class AsrBatcher:
    """Cross-session batching of recognition passes on one ASR engine (one GPU).

    ``recognize`` is called from the voice server's worker threads (one blocking call per session
    pass); the scheduler thread takes EVERY pass queued since its last batch -- up to the
    engine's free session slots -- and runs them as one ``decode_many`` batch.  While a batch is
    on the GPU the next one accumulates, so under load each GPU pass serves many sessions."""

    def __init__(self, asr_engine, *, max_tokens: int = 96, max_batch: Optional[int] = None,
                 tokens_per_s: Optional[float] = None):
        """tokens_per_s: fixed-work mode for benchmarks on random-init weights (which emit EOT at
        random): every pass decodes exactly round(audio seconds x tokens_per_s) transcript tokens
        in all (committed prefix included), as bench.py's ``exact_tokens``."""
        self.eng = asr_engine
        self.max_tokens = max_tokens
        self.tokens_per_s = tokens_per_s
        self.max_batch = max_batch or len(asr_engine.free_slots)
        self._q: List[tuple] = []
        self._cv = threading.Condition()
        self._stop = False
        self.stats = {"batches": 0, "passes": 0, "max_batch": 0, "gpu_ms": 0.0}
        # shared-GPU deployment: the brain reads this to keep its persistent chained decode launch
        # off the GPU while recognition runs (utils/busy_flag.py; launch.py sets the path)
        from ..utils.busy_flag import from_env

        self.busy = from_env(create=True)
        dev = getattr(asr_engine.model, "device", None)
        self._cuda_index = None
        if dev is not None and getattr(dev, "type", "cpu") == "cuda":
            import torch

            self._cuda_index = dev.index if dev.index is not None else torch.cuda.current_device()
        self._thread = threading.Thread(target=self._loop, name="asr-batcher", daemon=True)
        self._thread.start()

    def recognize(self, pcm: np.ndarray, prefix: Sequence[int] = ()) -> Hypothesis:
        return self.recognize_async(pcm, prefix).result()

    def recognize_async(self, pcm: np.ndarray, prefix: Sequence[int] = ()) -> Future:
        """Queue a pass for the next GPU batch; the Future resolves to its Hypothesis."""
        fut: Future = Future()
        with self._cv:
            if self._stop:
                raise RuntimeError("ASR batcher stopped")
            # (cut to what the decoder forces: the hypothesis is built on the prefix it really used)
            self._q.append((np.array(pcm, dtype=np.int16, copy=True), list(prefix)[: self.eng.max_prefix()], fut))
            self._cv.notify()
        return fut

    def rows_per_batch(self) -> float:
        return self.stats["passes"] / max(1, self.stats["batches"])

    def queue_depth(self) -> int:
        """Recognition passes waiting for the next GPU batch (the router's load signal)."""
        with self._cv:
            return len(self._q)

    def _loop(self) -> None:
        if self._cuda_index is not None:
            import torch

            torch.cuda.set_device(self._cuda_index)
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if self._stop and not self._q:
                    return
                batch, self._q = self._q[: self.max_batch], self._q[self.max_batch :]
            t0 = time.perf_counter()
            if self.busy is not None:
                self.busy.enter()
            try:
                audios = [self.eng.pcm_to_audio(p) for p, _, _ in batch]
                kw = dict(max_tokens=self.max_tokens)
                if self.tokens_per_s:
                    kw = dict(exact_tokens=max(1, min(self.max_tokens, max(
                        int(round(len(p) / 16000 * self.tokens_per_s)) - len(pre) for p, pre, _ in batch))))
                toks = self.eng.decode_many(audios, [pre for _, pre, _ in batch], **kw)
                for (_, pre, fut), t in zip(batch, toks):
                    full = pre + t
                    fut.set_result(Hypothesis(full, self.eng.tok.decode(full).strip()))
            except BaseException as e:  # noqa: BLE001  (fail this batch's passes, keep serving)
                for _, _, fut in batch:
                    if not fut.done():
                        fut.set_exception(e)
            finally:
                if self.busy is not None:
                    self.busy.leave()
            n = len(batch)
            self.stats["batches"] += 1
            self.stats["passes"] += n
            self.stats["max_batch"] = max(self.stats["max_batch"], n)
            self.stats["gpu_ms"] += (time.perf_counter() - t0) * 1e3

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=30)


def make_asr_transcriber(asr_engine, *, tokens_per_s: Optional[float] = None) -> Callable[[np.ndarray], str]:
    """Adapter: AsrEngine -> transcribe(pcm int16) callable (fixed-work mode with tokens_per_s)."""

    def fn(pcm: np.ndarray) -> str:
        audio = asr_engine.pcm_to_audio(pcm)
        if tokens_per_s:
            n = max(1, int(round(len(pcm) / 16000 * tokens_per_s)))
            return asr_engine.transcribe(audio, exact_tokens=n)
        return asr_engine.transcribe(audio)

    return fn
