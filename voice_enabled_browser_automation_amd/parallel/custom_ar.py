"""One-shot xGMI all-reduce for decode-sized TP messages (csrc/kernels/allreduce.hip).

Setup (once per TP group): every rank allocates its staging + flag buffers as uncached device
memory (hipExtMallocWithFlags(hipDeviceMallocUncached), checked with hipPointerGetAttributes),
exports IPC handles, the handles are all-gathered over the (CPU) control group, and every rank
maps its peers' buffers.  A preflight at group start then checks P2P access for every pair of
the group's devices (hipDeviceCanAccessPeer, by PCI id) and runs one all-reduce self-test with a
host-side deadline, so a group whose links do not work fails at start with a named error
(``TPPreflightError``) instead of hanging in its first decode step.  After that each call is ONE
kernel launch -- capturable inside the decode hipGraph -- that reads all peers' inputs directly
over the point-to-point xGMI links (one hop) instead of RCCL's 2(N-1)-step ring.  Messages larger
than the buffer go to RCCL.

Enabled on GPU TP groups by default (``VWA_CUSTOM_AR=0`` disables); the multi-process test runs
two ranks on one GPU (IPC within a device works the same way as across devices).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..utils.env import knob


class TPPreflightError(RuntimeError):
    """A TP group cannot run its decode collectives (no P2P path between two of its GPUs, or the
    one-shot all-reduce self-test failed / did not finish)."""


def peer_access_report(ctl_group, rank: int, world: int) -> dict:
    """Collective: every rank's device PCI id, and for each pair of DIFFERENT devices whether this
    rank's device can map the peer's (hipDeviceCanAccessPeer; -1: the peer's device is not visible
    to this process).  Ranks sharing one device (tests, gloo rehearsals) need no P2P."""
    E = ops.ext()
    dev = torch.cuda.current_device()
    mine = E.pci_id(dev)
    ids = [None] * world
    dist.all_gather_object(ids, mine, group=ctl_group)
    local = {E.pci_id(d): d for d in range(torch.cuda.device_count())}
    access = {}
    for p, pid in enumerate(ids):
        if p == rank or pid == mine:
            continue
        access[p] = int(E.can_access_peer(dev, local[pid])) if pid in local else -1
    return {"pci": ids, "access": access}


class OneShotAllReduce:
    def __init__(self, rank: int, world: int, ctl_group, *, max_elems: int = 64 * 8192, preflight: bool = True,
                 selftest_s: float = 20.0):
        max_elems = -(-max_elems // 512) * 512
        E = ops.ext()
        self.rank, self.world, self.max_elems = rank, world, max_elems
        if preflight:
            rep = peer_access_report(ctl_group, rank, world)
            self.peer_report = rep
            bad = [p for p, ok in rep["access"].items() if ok == 0]
            flags = [None] * world
            dist.all_gather_object(flags, bad, group=ctl_group)  # every rank fails together
            if any(flags):
                raise TPPreflightError(f"no P2P access between TP ranks' GPUs: {[(r, b) for r, b in enumerate(flags) if b]} "
                                       f"(PCI ids {rep['pci']}); the one-shot all-reduce needs xGMI peer mapping")
        self.state = E.ar_create(rank, world, max_elems)
        mine = E.ar_handles(self.state)
        allh = [None] * world
        dist.all_gather_object(allh, mine.numpy().tobytes(), group=ctl_group)
        for p, hb in enumerate(allh):
            if p != rank:
                E.ar_open_peer(self.state, p, torch.frombuffer(bytearray(hb), dtype=torch.uint8))
        dist.barrier(group=ctl_group)
        if preflight:
            self.self_test(ctl_group, selftest_s)

    def self_test(self, ctl_group, timeout_s: float = 20.0) -> None:
        """One all-reduce of (rank + 1) on every rank; the kernel's waits are bounded (error word),
        the host waits at most ``timeout_s`` for it -> TPPreflightError on a wrong sum, an error
        word or a deadline miss (on every rank: the verdicts are exchanged)."""
        import time

        x = torch.full((4096,), float(self.rank + 1), dtype=torch.bfloat16, device="cuda")
        want = float(self.world * (self.world + 1) // 2)
        ev = torch.cuda.Event()
        self(x)
        ev.record()
        t0 = time.monotonic()
        while not ev.query():
            if time.monotonic() - t0 > timeout_s:
                break
            time.sleep(0.001)
        done = ev.query()
        why = ""
        if not done:
            why = f"did not finish in {timeout_s} s"
        elif self.error():
            why = "a peer never signalled (bounded wait hit)"
        elif not bool((x.float() == want).all()):
            why = f"wrong sum {x.float().unique().tolist()[:4]} (want {want})"
        verdicts = [None] * self.world
        dist.all_gather_object(verdicts, why, group=ctl_group)
        if any(verdicts):
            raise TPPreflightError("one-shot all-reduce self-test failed: " +
                                   "; ".join(f"rank {r}: {v}" for r, v in enumerate(verdicts) if v))

    def sample_buffers(self, words: int, device):
        """(xin [>= words], xout [>= world * words]) int32 exchange buffers of the vocab-parallel
        sampler (ops.sample_tp), grown on demand and reused (the calls are stream-ordered)."""
        have = getattr(self, "_sbuf", None)
        if have is None or have[0].numel() < words:
            n = max(words, 4096)
            self._sbuf = (torch.zeros(n, dtype=torch.int32, device=device),
                          torch.zeros(self.world * n, dtype=torch.int32, device=device))
        return self._sbuf

    def gather(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One-shot all-gather of an int32 [n] tensor -> [world, n] (every rank, rank order)."""
        if out is None:
            out = torch.empty((self.world, t.numel()), dtype=torch.int32, device=t.device)
        ops.ext().ar_gather(self.state, t.contiguous(), out)
        return out

    def fits(self, t: torch.Tensor) -> bool:
        return t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() <= self.max_elems and t.numel() % 8 == 0

    def __call__(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        out = t if out is None else out
        ops.ext().ar_allreduce(self.state, t, out)
        return out

    def error(self) -> bool:
        return bool(ops.ext().ar_error(self.state))

    def close(self) -> None:
        if self.state:
            ops.ext().ar_destroy(self.state)
            self.state = 0


def maybe_custom_ar(tp, ctl_group) -> Optional[OneShotAllReduce]:
    """Attach a one-shot all-reduce to a GPU TP context (None on CPU / disabled / TP=1)."""
    if tp.size <= 1 or not torch.cuda.is_available() or not knob("VWA_CUSTOM_AR"):
        return None
    return OneShotAllReduce(tp.rank, tp.size, ctl_group)
