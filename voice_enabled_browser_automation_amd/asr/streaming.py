"""Streaming recognition with Deepgram-compatible events (replaces the Deepgram live connection,
apps/voice/src/deepgram.ts:33-51).

The voice server feeds raw PCM16 LE 16 kHz mono frames (the UI sends ~60 ms packets,
apps/web/src/App.tsx:279-288).  A session keeps the current utterance buffer and:

* energy VAD on 20 ms frames tracks speech start and trailing silence;
* every ``partial_every_s`` of new speech it re-transcribes the buffer and emits an interim
  result (``is_final: false``), like Deepgram's interim_results;
* on an endpoint (``endpoint_silence_s`` of silence after speech), on ``flush()`` (client
  end-of-utterance) or when the 30 s Whisper window is full, it emits a final result
  (``is_final: true, speech_final: true``) and starts a new utterance.

Events use the Deepgram ``Results`` shape that the unchanged UI and voice logic read
(``payload.is_final``, ``payload.channel.alternatives[0].transcript``; apps/voice/src/server.ts:112,123).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, List, Optional

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


class StreamingAsrSession:
    def __init__(self, transcribe: Callable[[np.ndarray], str], *, rate: int = 16000, model_name: str = "whisper",
                 partial_every_s: float = 1.0, endpoint_silence_s: float = 0.6, energy_threshold: float = 300.0,
                 max_window_s: float = 30.0, min_speech_s: float = 0.2):
        self.transcribe = transcribe
        self.rate = rate
        self.model_name = model_name
        self.partial_every = int(partial_every_s * rate)
        self.endpoint = int(endpoint_silence_s * rate)
        self.thresh = energy_threshold
        self.max_window = int(max_window_s * rate)
        self.min_speech = int(min_speech_s * rate)
        self.frame = rate // 50  # 20 ms
        self.buf = np.zeros(0, dtype=np.int16)
        self._carry = b""
        self.t_offset = 0.0          # stream time of buf[0]
        self.speech = 0              # speech samples in the utterance
        self.trailing_silence = 0
        self.since_partial = 0
        self.last_partial = ""
        self.stats: Dict[str, float] = {"partials": 0, "finals": 0, "asr_ms": 0.0}

    # ------------------------------------------------------------------ internals
    def _run(self) -> str:
        t0 = time.perf_counter()
        text = self.transcribe(self.buf)
        self.stats["asr_ms"] += (time.perf_counter() - t0) * 1e3
        return text.strip()

    def _final(self) -> List[Dict]:
        out: List[Dict] = []
        if self.speech >= self.min_speech and len(self.buf):
            text = self._run()
            out.append(results_event(text, is_final=True, start=self.t_offset, duration=len(self.buf) / self.rate,
                                     model=self.model_name))
            self.stats["finals"] += 1
        self.t_offset += len(self.buf) / self.rate
        self.buf = np.zeros(0, dtype=np.int16)
        self.speech = self.trailing_silence = self.since_partial = 0
        self.last_partial = ""
        return out

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
            self.buf = np.concatenate([self.buf, fr])
            rms = float(np.sqrt(np.mean(fr.astype(np.float32) ** 2)))
            if rms >= self.thresh:
                self.speech += len(fr)
                self.trailing_silence = 0
            else:
                self.trailing_silence += len(fr)
            if self.speech > 0:
                self.since_partial += len(fr)
            if self.speech >= self.min_speech and self.trailing_silence >= self.endpoint:
                events += self._final()
            elif len(self.buf) >= self.max_window:
                events += self._final()
            elif self.speech == 0 and self.trailing_silence >= self.endpoint:
                # leading silence: drop it, keep the stream clock
                self.t_offset += len(self.buf) / self.rate
                self.buf = np.zeros(0, dtype=np.int16)
                self.trailing_silence = 0
        if self.speech >= self.min_speech and self.since_partial >= self.partial_every:
            self.since_partial = 0
            text = self._run()
            if text != self.last_partial:
                self.last_partial = text
                events.append(results_event(text, is_final=False, start=self.t_offset,
                                            duration=len(self.buf) / self.rate, model=self.model_name))
                self.stats["partials"] += 1
        return events

    def flush(self) -> List[Dict]:
        return self._final()


def make_asr_transcriber(asr_engine, *, tokens_per_s: Optional[float] = None) -> Callable[[np.ndarray], str]:
    """Adapter: AsrEngine -> transcribe(pcm int16) callable."""

    def fn(pcm: np.ndarray) -> str:
        audio = asr_engine.pcm_to_audio(pcm)
        if tokens_per_s:
            n = max(1, int(round(len(pcm) / 16000 * tokens_per_s)))
            return asr_engine.transcribe(audio, exact_tokens=n)
        return asr_engine.transcribe(audio)

    return fn
