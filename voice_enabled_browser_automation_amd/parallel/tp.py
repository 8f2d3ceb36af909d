"""Tensor-parallel / data-parallel process-group plumbing (one process per GPU).

`torch.distributed` with backend "nccl" is RCCL on ROCm; on CPU (tests) the same code runs
over gloo.  The LLM needs exactly these collectives:

* C1/C2  all-reduce of the row-parallel o_proj / down_proj outputs (decode: d*2 bytes per row,
         i.e. 8 KiB for Llama-3-8B -- latency bound; the residual is folded into rank 0's
         GEMM epilogue so the all-reduce result IS the new residual stream);
* C3     all-reduce of the vocab-parallel embedding rows (one per step);
* C4     vocab-parallel sampling: each rank's partial (value, id) maxima are exchanged ([B, 2]
         per chunk, ops.sample / csrc sample_tp over the one-shot IPC all-gather), never logits;
* C5     broadcast (weights are generated deterministically on every rank, so only the
         random seed needs to agree -- no weight traffic at init);
* C6     all-gather of per-rank metrics (DP router).

Layout of ranks on one 8-GPU node: TP groups are contiguous ranks (xGMI is a full mesh, so
any contiguous group has direct links), DP replicas are the TP groups.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist
from ..utils.env import knob


@dataclass
class TPContext:
    rank: int = 0
    size: int = 1
    group: Optional[object] = None
    dp_rank: int = 0
    dp_size: int = 1
    custom_ar: Optional[object] = None  # parallel.custom_ar.OneShotAllReduce (GPU TP groups)
    ctl: Optional[object] = None  # CPU (gloo) group of this TP group: the serving control plane

    @staticmethod
    def single() -> "TPContext":
        return TPContext()

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the TP group: one-shot xGMI kernel for decode-sized bf16 messages,
        RCCL otherwise."""
        if self.size > 1:
            if self.custom_ar is not None and t.is_cuda and self.custom_ar.fits(t):
                self.custom_ar(t)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def all_gather_vocab(self, local: torch.Tensor, vocab: int) -> torch.Tensor:
        """[n, V_shard] logits shards -> [n, V] (diagnostics / prefill checks only: the decode loop
        samples vocab-parallel and never gathers logits).  Shards are padded to the common
        32-aligned shard width for the collective."""
        n, vp = local.shape
        per = ((vocab + self.size - 1) // self.size + 31) // 32 * 32
        pad = torch.full((n, per), float("-inf"), dtype=local.dtype, device=local.device)
        pad[:, :vp] = local
        parts = [torch.empty_like(pad) for _ in range(self.size)]
        dist.all_gather(parts, pad, group=self.group)
        return torch.cat(parts, dim=1)[:, :vocab].contiguous()

    def barrier(self):
        if self.size > 1:
            dist.barrier(group=self.group)


def init_distributed(tp_size: Optional[int] = None, backend: Optional[str] = None) -> TPContext:
    """Initialise torch.distributed from torchrun env vars and split ranks into TP groups.

    Returns TPContext for this rank. Single-process runs return TPContext.single().
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return TPContext.single()
    rank = int(os.environ.get("RANK", "0"))
    if not dist.is_initialized():
        if backend is None:
            backend = knob("VWA_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            local = int(os.environ.get("LOCAL_RANK", rank))
            # gloo rehearsal of a multi-rank run on fewer GPUs: ranks share devices round-robin
            torch.cuda.set_device(local if backend == "nccl" else local % torch.cuda.device_count())
        dist.init_process_group(backend=backend)
    tp = tp_size or world
    assert world % tp == 0, f"world {world} not divisible by tp {tp}"
    groups = [dist.new_group(list(range(s, s + tp))) for s in range(0, world, tp)]
    gi = rank // tp
    ctx = TPContext(rank=rank % tp, size=tp, group=groups[gi], dp_rank=gi, dp_size=world // tp)
    if tp > 1:
        # one gloo group per TP group (every rank takes part in creating every group): the brain's
        # lockstep control messages (brain/tp_engine.py) and the IPC handle exchange of the custom
        # all-reduce stay off the GPU and within the group
        ctl = [dist.new_group(list(range(s, s + tp)), backend="gloo") for s in range(0, world, tp)]
        ctx.ctl = ctl[gi]
        if torch.cuda.is_available():
            from .custom_ar import maybe_custom_ar

            ctx.custom_ar = maybe_custom_ar(ctx, ctl[gi])
    return ctx
