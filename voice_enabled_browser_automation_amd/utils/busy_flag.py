"""A cross-process "GPU busy" word in /dev/shm: the voice worker's ASR batcher marks the intervals
in which recognition passes run on the GPU it shares with the brain, and the brain's decode loop
reads it before every step to choose its launch form (runtime/engine.py ``chain_gate``): the
persistent chained launch needs every CU (its workgroups wait for co-resident peers at grid
barriers, so a concurrent ASR kernel stalls it -- measured 3.72-3.76 vs 3.61-3.62 ms per step under
live ASR load, profiles/r4_service_chain_ab.jsonl), while with the recognizer idle -- one session,
whose user has stopped speaking when the brain decodes -- it is the fast form (~10 % per step).

Layout: u64 busy count (passes in flight), u64 CLOCK_MONOTONIC ns of the last change.  Plain
aligned 8-byte stores / loads (atomic on x86-64); the reader only needs a recent value."""
from __future__ import annotations

import mmap
import os
import struct
import time
from typing import Optional

_SIZE = 64


class BusyFlag:
    def __init__(self, path: str, create: bool = False):
        self.path = path
        flags = os.O_RDWR | (os.O_CREAT if create else 0)
        fd = os.open(path, flags, 0o600)
        try:
            if create and os.fstat(fd).st_size < _SIZE:
                os.ftruncate(fd, _SIZE)
            self._m = mmap.mmap(fd, _SIZE)
        finally:
            os.close(fd)

    def enter(self) -> None:
        n = struct.unpack_from("<Q", self._m, 0)[0]
        struct.pack_into("<QQ", self._m, 0, n + 1, time.monotonic_ns())

    def leave(self) -> None:
        n = struct.unpack_from("<Q", self._m, 0)[0]
        struct.pack_into("<QQ", self._m, 0, max(0, n - 1), time.monotonic_ns())

    def busy(self, hold_ms: float = 0.0) -> bool:
        """True while a pass runs, or (hold_ms) within hold_ms after the last one ended."""
        n, t = struct.unpack_from("<QQ", self._m, 0)
        if n:
            return True
        return hold_ms > 0 and (time.monotonic_ns() - t) < hold_ms * 1e6

    def close(self) -> None:
        self._m.close()


def from_env(create: bool = False) -> Optional[BusyFlag]:
    from .env import knob

    path = knob("VWA_ASR_BUSY_FILE")
    if not path:
        return None
    try:
        return BusyFlag(path, create=create)
    except OSError:
        return None
