"""Per-iteration control channel of the TP brain (brain/tp_engine.py).

The lockstep scheduler sends one message per decode iteration from rank 0 to the other ranks of
its TP group: the requests admitted in that iteration (usually none) and a stop flag.  Round 5
sent it as a gloo broadcast -- a TCP round trip on the critical path of every iteration, while
the leader's first chained launch already waits at its first in-launch all-reduce round for the
workers (SURVEY.md §5.8 "small pinned-host broadcast").  One TP group is one
node, so the message now goes through a /dev/shm ring (csrc/runtime/shm_channel.cpp: sequence-
numbered slots, per-reader acks, spin-then-sleep waits without the GIL, a leader heartbeat word).
gloo stays for the setup (the channel's name) and for failures.

    chan = make_channel(tp_rank, tp_size, ctl_group)   # collective over the TP group's gloo group
    chan.send(obj)          # rank 0
    obj = chan.recv()       # ranks 1..

``VWA_TP_CONTROL``: ``shm`` (default) or ``gloo`` (the round-5 broadcast, kept for A/B and for
ranks that do not share a node).
"""
from __future__ import annotations

import os
import pickle
import uuid
from typing import Any, Optional

from ..utils.env import knob


class GlooChannel:
    """The round-5 control message: a 1-int length header + the pickled payload over gloo."""

    kind = "gloo"

    def __init__(self, rank: int, group):
        self.rank, self.group = rank, group

    def send(self, obj: Any) -> None:
        self._bcast(obj)

    def recv(self) -> Any:
        return self._bcast(None)

    def _bcast(self, obj):
        import torch
        import torch.distributed as dist

        data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL) if self.rank == 0 else b""
        hdr = torch.tensor([len(data)], dtype=torch.int64)
        dist.broadcast(hdr, src=0, group=self.group)
        n = int(hdr[0])
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8) if self.rank == 0 else torch.empty(n, dtype=torch.uint8)
        if n:
            dist.broadcast(buf, src=0, group=self.group)
        return obj if self.rank == 0 else pickle.loads(buf.numpy().tobytes())

    def beat(self) -> None:
        pass

    def close(self) -> None:
        pass


class ShmChannel:
    """/dev/shm broadcast ring (native); rank 0 writes, ranks 1..n-1 read (reader index rank-1).
    A payload larger than a slot goes out over gloo behind a marker message."""

    kind = "shm"
    _BIG = b"\x00VWA_BIG"

    def __init__(self, rank: int, world: int, group, *, slot_bytes: int = 1 << 20, n_slots: int = 8,
                 dead_s: Optional[float] = None):
        import torch.distributed as dist

        from ..grammar import native

        N = native()
        self.rank, self.world, self.group = rank, world, group
        self.dead_s = knob("VWA_TP_DEAD_S") if dead_s is None else dead_s
        self._gloo = GlooChannel(rank, group)
        box = [f"vwa_tp_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
        if rank == 0:
            self.ch = N.ShmChannel(box[0], n_readers=max(1, world - 1), slot_bytes=slot_bytes, n_slots=n_slots,
                                   create=True)
        dist.broadcast_object_list(box, src=0, group=group)
        if rank != 0:
            self.ch = N.ShmChannel(box[0], create=False)
        dist.barrier(group=group)
        if rank == 0:
            self.ch.unlink()  # every rank has it mapped: nothing is left in /dev/shm, even after a crash
        self.name = box[0]

    def send(self, obj: Any) -> None:
        data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        if len(data) > self.ch.slot_bytes:
            self.ch.publish(self._BIG, 60.0)
            self._gloo.send(obj)
            return
        self.ch.publish(data, 60.0)

    def recv(self) -> Any:
        data = self.ch.receive(self.rank - 1, -1.0, self.dead_s)
        if data == self._BIG:
            return self._gloo.recv()
        return pickle.loads(data)

    def beat(self) -> None:
        self.ch.beat()

    def close(self) -> None:
        self.ch = None


def make_channel(rank: int, world: int, group, kind: Optional[str] = None):
    """Collective over ``group`` (every rank of the TP group calls it)."""
    kind = kind or knob("VWA_TP_CONTROL")
    if kind == "gloo" or world <= 1:
        return GlooChannel(rank, group)
    if kind != "shm":
        raise ValueError(f"VWA_TP_CONTROL must be shm or gloo, not {kind!r}")
    return ShmChannel(rank, world, group)
