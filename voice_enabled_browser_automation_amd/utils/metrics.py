"""Tiny in-process metrics registry behind every service's ``GET /metrics`` (JSON).

The reference has console logging only; here each service keeps counters and
latency histograms (p50/p95 over a bounded window).
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict, deque
from typing import Deque, Dict


class Metrics:
    def __init__(self, service: str, window: int = 2048):
        self.service = service
        self.started = time.time()
        self._lock = threading.Lock()
        self.counters: Dict[str, int] = defaultdict(int)
        self.samples: Dict[str, Deque[float]] = defaultdict(lambda: deque(maxlen=window))

    def inc(self, name: str, n: int = 1) -> None:
        with self._lock:
            self.counters[name] += n

    def observe(self, name: str, value: float) -> None:
        with self._lock:
            self.samples[name].append(float(value))

    @staticmethod
    def _pct(xs, q: float) -> float:
        if not xs:
            return 0.0
        s = sorted(xs)
        i = min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))
        return s[i]

    def snapshot(self) -> dict:
        with self._lock:
            out = {"service": self.service, "uptime_s": round(time.time() - self.started, 3),
                   "counters": dict(self.counters), "latency": {}}
            for k, v in self.samples.items():
                xs = list(v)
                out["latency"][k] = {"n": len(xs), "p50": round(self._pct(xs, 0.5), 3),
                                     "p95": round(self._pct(xs, 0.95), 3),
                                     "mean": round(sum(xs) / len(xs), 3) if xs else 0.0}
            return out
