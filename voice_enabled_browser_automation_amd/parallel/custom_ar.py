"""One-shot xGMI all-reduce for decode-sized TP messages (csrc/kernels/allreduce.hip).

Setup (once per TP group): every rank allocates its staging + flag buffers with hipMalloc,
exports IPC handles, the handles are all-gathered over the (CPU) control group, and every rank
maps its peers' buffers.  After that each call is ONE kernel launch -- capturable inside the
decode hipGraph -- that reads all peers' inputs directly over the point-to-point xGMI links
(one hop) instead of RCCL's 2(N-1)-step ring.  Messages larger than the buffer go to RCCL.

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


class OneShotAllReduce:
    def __init__(self, rank: int, world: int, ctl_group, *, max_elems: int = 64 * 8192):
        max_elems = -(-max_elems // 512) * 512
        E = ops.ext()
        self.rank, self.world, self.max_elems = rank, world, max_elems
        self.state = E.ar_create(rank, world, max_elems)
        mine = E.ar_handles(self.state)
        allh = [None] * world
        dist.all_gather_object(allh, mine.numpy().tobytes(), group=ctl_group)
        for p, hb in enumerate(allh):
            if p != rank:
                E.ar_open_peer(self.state, p, torch.frombuffer(bytearray(hb), dtype=torch.uint8))
        dist.barrier(group=ctl_group)

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
