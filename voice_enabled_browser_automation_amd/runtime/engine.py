"""LLM execution engine: sequences, paged KV, ragged decode steps, hipGraph capture (N3).

A *step* runs M token rows through the model.  Rows may belong to different sequences
(continuous batching of concurrent voice sessions) or be consecutive tokens of one sequence
(jump-forward of grammar-forced tokens, short prompt suffixes).  Every row carries its own
position, KV slot, block-table row and context length, so one code path -- the MFMA skinny
GEMMs + paged decode attention -- serves all of them, and its launch shape depends only on
the row bucket M.  Each bucket (1, 2, 4, ..., 64) is captured once into a hipGraph
(torch.cuda.CUDAGraph on ROCm) and replayed: the ~165 kernels of a Llama-3-8B step are
then one graph launch instead of ~165 Python-driven launches.

Longer prompt chunks (> 64 rows) go through the prefill path eagerly: the hand-written tiled
MFMA GEMM (csrc/kernels/gemm.hip) and flash attention over the paged cache with a causal query
offset for a cold prompt; several requests' suffixes behind a cached prefix are batched into one
ragged forward (``prefill_batch``).

Sampling runs after the forward on the same stream so the CPU can compute the grammar mask
for this step while the GPU is busy with the forward (see brain.intent_engine).
"""
from __future__ import annotations

import itertools
import os
from dataclasses import dataclass, field
from types import SimpleNamespace
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from .. import ops
from .kv_cache import BlockManager, PagedKVCache
from ..utils.env import knob

# Row buckets of the captured step graphs (VWA_ROW_BUCKETS overrides).  48 between the powers of
# two: a 44-row step of 32 concurrent sessions (+ jump-forward rows) pays for 48 rows, not 64 --
# fp8 4.71 vs 5.05 ms, 32 sessions p50 447 vs 459 ms.  12: the 8-session steps (~13 rows) -- the
# streaming GEMMs' X staging makes 8..16-row steps cost ~72 us per row (8: 4.04, 12: 4.36, 16:
# 4.61 ms bf16, profiles/r4_rows_buckets_8_16.jsonl).  (24 measured the same as 32: the one
# 128-row GEMM tile and the attention floor dominate there.)
BUCKETS = tuple(int(b) for b in knob("VWA_ROW_BUCKETS").split(","))


class TPGroupFailure(RuntimeError):
    """A tensor-parallel decode step lost lockstep (a chained launch timed out waiting for a peer
    rank's in-launch all-reduce round): this process's KV cache and round counters can no longer
    be trusted, so the whole TP group must be restarted (brain/tp_engine.py)."""


def bucket_for(n: int) -> int:
    for b in BUCKETS:
        if n <= b:
            return b
    raise ValueError(f"{n} rows exceed the largest decode bucket")


_SEQ_UIDS = itertools.count()

# Decode attention reads the prompt prefix the step's sessions share (the same prefix-cached
# blocks) once per group of rows across sessions (attention.hip / mq_attention.h cascade);
# VWA_SHARED_ATTN=0: once per session
SHARED_ATTN = knob("VWA_SHARED_ATTN")
# Batched admission prefill: causal flash attention over [requests x longest suffix] instead of the
# decode-attention kernel in 64-row slices (VWA_PREFILL_FLASH=0: slices)
PREFILL_FLASH = knob("VWA_PREFILL_FLASH")


@dataclass
class Sequence_:
    sid: int                     # block-table row
    tokens: List[int] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)
    n_computed: int = 0          # tokens whose K/V are in the cache
    n_cached_prefix: int = 0     # tokens served from the prefix cache
    uid: int = field(default_factory=lambda: next(_SEQ_UIDS))  # unique for the process lifetime


class StepBuffers:
    """Device buffers with fixed addresses (graph inputs/outputs) + pinned host staging."""

    def __init__(self, model, max_rows: int, max_seqs: int, max_blocks_per_seq: int, max_ctx: int, device):
        i32 = dict(dtype=torch.int32, device=device)
        dt = model.dtype
        self.max_rows = max_rows
        self.max_ctx = max_ctx
        # all per-row metadata lives in ONE device buffer (and one pinned host mirror) so a step
        # needs a single H2D copy: [tokens | positions | seq_ids | ctx_lens | slots (int64) | sel |
        # shared] (sel = the rows whose logits the step returns: one per sequence, not one per token
        # row; shared = [P, n_real]: the first P keys of the step's real rows are the same cached
        # prompt blocks -- the decode attention reads them once per group of sessions)
        R = max_rows
        # per-ROW copy of each row's sequence block table (chained attention: read in the same round
        # trip as seq_ids / ctx_lens instead of a dependent table load); <= 128 blocks per sequence.
        # It sits right behind the step metadata in ONE buffer (device and pinned host alike), so a
        # step's upload is one copy node (measured in the bench trace: two copies were 2 + 3 us of
        # GPU time plus a 4 us scheduling gap per decode step)
        self.rt_cols = max_blocks_per_seq if max_blocks_per_seq <= 128 and max_blocks_per_seq % 2 == 0 else 0
        C = max(2, self.rt_cols)
        T = (7 * R + 2 + 15) // 16 * 16  # row table at a 64-byte aligned offset
        self.meta_all = torch.zeros(T + R * C, **i32)
        self.meta = self.meta_all[: 7 * R + 2]
        self.tokens = self.meta[0:R]
        self.positions = self.meta[R : 2 * R]
        self.seq_ids = self.meta[2 * R : 3 * R]
        self.ctx_lens = self.meta[3 * R : 4 * R]
        self.slots = self.meta[4 * R : 6 * R].view(torch.int64)
        self.sel = self.meta[6 * R : 7 * R]
        self.shared = self.meta[7 * R : 7 * R + 2]
        self.ctx_lens.fill_(1)
        self.slots.fill_(-1)
        self.block_table = torch.zeros(max_seqs, max_blocks_per_seq, **i32)
        d = model.cfg.hidden
        self.hidden = torch.zeros(max_rows, d, dtype=dt, device=device)
        self.hidden_sel = torch.zeros(max_rows, d, dtype=dt, device=device)
        self.q = torch.zeros(max_rows, model.nq * model.hd, dtype=dt, device=device)
        self.attn = torch.zeros_like(self.q)
        self.act = torch.zeros(max_rows, model.F, dtype=dt, device=device)
        self.logits_local = torch.zeros(max_rows, model.v_end - model.v_start, dtype=torch.float32, device=device)
        self.logits = self.logits_local  # (vocab-parallel: the decode loop never gathers full logits)
        ns = ops.decode_n_splits(max_ctx)
        self.part_o = torch.zeros(max_rows * ns * model.nq * model.hd, dtype=torch.float32, device=device)
        self.part_ml = torch.zeros(max_rows * ns * model.nq * 2, dtype=torch.float32, device=device)
        self.attn_cnt = torch.zeros(max_rows * model.nkv, dtype=torch.int32, device=device)  # chunk tickets
        pin = torch.device(device).type == "cuda"
        self.h_meta_all = torch.zeros(T + R * C, dtype=torch.int32, pin_memory=pin)
        self.h_meta = self.h_meta_all[: 7 * R + 2]
        self.h_i32 = self.h_meta[: 4 * R].view(4, R)
        self.h_slots = self.h_meta[4 * R : 6 * R].view(torch.int64)
        self.h_sel = self.h_meta[6 * R : 7 * R]
        self.np_shared = self.h_meta[7 * R : 7 * R + 2].numpy()
        # rows whose hidden state feeds the LM head when the step computed every row (L == M):
        # gathered on the device through a pinned staging copy (a torch.tensor(list, device=...)
        # here was a pageable, host-blocking copy that waited for the whole step -- measured: 9 of
        # 172 iterations at 32 sessions stalled ~4.6 ms each)
        self.h_head_idx = torch.zeros(R, dtype=torch.int64, pin_memory=pin)
        self.head_idx = torch.zeros(R, dtype=torch.int64, device=device)
        self.row_table = self.meta_all[T:].view(R, C)
        self.h_row_table = self.h_meta_all[T:].view(R, C)
        self.np_row_table = self.h_row_table.numpy()
        self.h_i32[3].fill_(1)  # the same inert rows as the device copy (captured graphs upload it)
        self.h_slots.fill_(-1)
        self.h_table = torch.zeros(max_seqs, max_blocks_per_seq, dtype=torch.int32, pin_memory=pin)
        self.table_dirty = True
        # numpy views of the pinned staging buffers: the per-step row metadata is written with a
        # handful of slice assignments instead of ~5 torch element writes per row
        self.np_i32 = self.h_i32.numpy()
        self.np_slots = self.h_slots.numpy()
        self.np_sel = self.h_sel.numpy()
        self.np_table = self.h_table.numpy()

    def upload(self, n_rows: int, meta: bool = True) -> None:
        """H2D copy of the step metadata (skipped when the replayed graph contains it) and of the
        block table when it changed."""
        if meta:
            self.meta.copy_(self.h_meta, non_blocking=True)
        if self.table_dirty:
            self.block_table.copy_(self.h_table, non_blocking=True)
            self.table_dirty = False


class LLMEngine:
    def __init__(self, model, *, max_seqs: int = 8, max_model_len: int = 4096, block_size: int = 16,
                 kv_blocks: Optional[int] = None, kv_gb: Optional[float] = None, use_graphs: Optional[bool] = None,
                 max_rows: int = 64):
        self.model = model
        self.device = model.device
        self.block_size = block_size
        self.max_model_len = max_model_len
        self.max_seqs = max_seqs
        cfg = model.cfg
        if kv_blocks is None and kv_gb is None and knob("VWA_KV_GB").strip().lower() == "auto":
            # size the paged KV from the per-GPU HBM plan (runtime/memory_plan.py): what the weights,
            # step buffers and workspaces leave of the 288 GB
            from .memory_plan import plan_memory

            free, _total = torch.cuda.mem_get_info(self.device) if self.device.type == "cuda" else (0, 0)
            # VWA_SHARED_GB: HBM a co-located service keeps (launch.py sets it when the voice
            # worker's ASR shares this GPU)
            shared = knob("VWA_SHARED_GB")
            plan = plan_memory(cfg, model.tp.size, wdtype=getattr(model, "wdtype", "bf16"), block_size=block_size,
                               max_rows=max_rows, max_ctx=max_model_len, shared_gb=shared)
            kv_blocks = plan.kv_blocks
            if free:
                # never more than the device has free now (other processes, fragmentation), minus
                # headroom for what is allocated after the KV: step buffers, graph pools, GEMM and
                # prefill scratch, and the co-located service
                per = PagedKVCache.bytes_per_block(cfg.n_layers, model.nkv, model.hd, block_size)
                head = plan.step_buffers + plan.workspace + int(4e9) + int(shared * 1e9)
                kv_blocks = min(kv_blocks, max(0, int(free * 0.95) - head) // per)
            self.memory_plan = plan
        if kv_blocks is None:
            if kv_gb is None:
                kv_gb = float(knob("VWA_KV_GB") or 0)
            if kv_gb > 0:
                kv_blocks = PagedKVCache.blocks_for_budget(kv_gb * 1e9, cfg.n_layers, model.nkv, model.hd, block_size)
            else:
                kv_blocks = max_seqs * (max_model_len // block_size) * 2 + 1
        self.kv = PagedKVCache(cfg.n_layers, model.nkv, model.hd, block_size, kv_blocks, device=self.device,
                               dtype=model.dtype)
        self.blocks = BlockManager(kv_blocks, block_size)
        self.max_blocks_per_seq = (max_model_len + block_size - 1) // block_size
        self.bufs = StepBuffers(model, max_rows, max_seqs, self.max_blocks_per_seq, max_model_len, self.device)
        self.free_sids = list(range(max_seqs - 1, -1, -1))
        self.seqs: Dict[int, Sequence_] = {}
        if use_graphs is None:
            use_graphs = ops.env_flag("VWA_HIPGRAPH")
        self.use_graphs = bool(use_graphs) and self.device.type == "cuda"
        self.graphs: Dict[Tuple[int, int, bool], Tuple[torch.cuda.CUDAGraph, torch.Tensor]] = {}
        # chain_gate() -> True: this step must not use the persistent chained launch (the GPU is
        # shared with a busy ASR worker, utils/busy_flag.py); graphs are kept per launch form
        self.chain_gate = None
        self._gated = False
        self.graph_pool = None
        self.stats = dict(steps=0, rows=0, prefill_tokens=0, cached_tokens=0, graph_replays=0)
        self._last_step = None  # (rows, logits_for, n_computed before) of a chained step, for recover_step
        # True from a step's launch until the host knows the stream has passed it: the pinned
        # staging rows (h_meta, h_row_table) are read by that step's H2D copy -- inside the
        # replayed graph -- so the next step may only rewrite them once it has executed
        self._staging_inflight = False
        self._head_rows: Optional[torch.Tensor] = None  # the last step's hidden rows for head_logits()
        self._shared_cache: Dict[tuple, int] = {}  # sequences of a step -> shared prefix blocks

    # ------------------------------------------------------------------ sequences
    def new_sequence(self, tokens: Sequence[int], use_prefix_cache: bool = True) -> Sequence_:
        if not self.free_sids:
            raise RuntimeError("too many concurrent sequences")
        sid = self.free_sids.pop()
        seq = Sequence_(sid=sid, tokens=list(tokens))
        if use_prefix_cache:
            blocks, n = self.blocks.match_prefix(seq.tokens)
            seq.blocks = blocks
            seq.n_computed = n
            seq.n_cached_prefix = n
            self.stats["cached_tokens"] += n
        self.seqs[sid] = seq
        self._sync_table(seq)
        return seq

    def free_sequence(self, seq: Sequence_, publish: bool = True, publish_upto: Optional[int] = None) -> None:
        """Release a sequence; publish its first ``publish_upto`` computed tokens (default all) to the
        prefix cache."""
        if publish:
            n = seq.n_computed if publish_upto is None else min(seq.n_computed, publish_upto)
            self.blocks.register_prefix(seq.tokens, seq.blocks, n)
        self.blocks.release(seq.blocks)
        seq.blocks = []
        self.seqs.pop(seq.sid, None)
        self.free_sids.append(seq.sid)

    def _ensure_blocks(self, seq: Sequence_, n_tokens: int) -> None:
        need = (n_tokens + self.block_size - 1) // self.block_size
        if need > self.max_blocks_per_seq:
            raise RuntimeError(f"sequence exceeds max_model_len={self.max_model_len}")
        if need > len(seq.blocks):
            seq.blocks += self.blocks.allocate(need - len(seq.blocks))
            self._sync_table(seq)

    def _sync_table(self, seq: Sequence_) -> None:
        row = self.bufs.np_table[seq.sid]
        row[:] = 0
        row[: len(seq.blocks)] = seq.blocks
        self.bufs.table_dirty = True

    def _shared_prefix(self, rows: List[Tuple[Sequence_, int]], min_ctx: int) -> int:
        """Keys (a multiple of 32) that every row of the step reads from the SAME physical blocks:
        the prefix-cached prompt the sessions share (decode attention reads them once per group of
        rows across sessions).  0 below 128 keys or for a single sequence.  Cached per set of
        sequences (it changes only when a session joins or leaves)."""
        if not SHARED_ATTN:
            return 0
        seqs = {}
        for seq, _ in rows:
            seqs.setdefault(seq.sid, seq)
        if len(seqs) < 2:
            return 0
        key = tuple(s.uid for s in seqs.values())
        nb = self._shared_cache.get(key)
        if nb is None:
            lim = min(len(s.blocks) for s in seqs.values())
            t = self.bufs.np_table[list(seqs)][:, :lim]
            eq = (t == t[0]).all(0)
            nb = int(lim if eq.all() else eq.argmin())
            if len(self._shared_cache) > 256:
                self._shared_cache.clear()
            self._shared_cache[key] = nb
        P = min(nb * self.block_size, min_ctx) // 32 * 32
        return P if P >= 128 else 0

    def slot_of(self, seq: Sequence_, pos: int) -> int:
        return seq.blocks[pos // self.block_size] * self.block_size + pos % self.block_size

    # ------------------------------------------------------------------ forward
    def _forward_rows(self, M: int, L: int, upload_meta: bool = False) -> torch.Tensor:
        if upload_meta:
            # inside a captured graph: the pinned -> device metadata copy is the graph's first node,
            # so a replay is one host call instead of a copy + a replay
            b = self.bufs
            n = (b.meta_all.numel() - b.row_table.numel() + M * b.row_table.shape[1]) if b.rt_cols and M <= 4 \
                else b.meta.numel()
            b.meta_all[:n].copy_(b.h_meta_all[:n], non_blocking=True)
        return self.model.forward(self.bufs, M, self.kv, n_sel=None if L == M else L, head=False)

    def _capture(self, M: int, L: int):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._forward_rows(M, L, upload_meta=True)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        if self.graph_pool is None:
            self.graph_pool = torch.cuda.graph_pool_handle()
        with torch.cuda.graph(g, pool=self.graph_pool):
            out = self._forward_rows(M, L, upload_meta=True)
        self.graphs[(M, L, self._gated)] = (g, out)
        return self.graphs[(M, L, self._gated)]

    def capture_all(self, buckets: Sequence[int] = BUCKETS, logit_buckets: Sequence[int] = (1,)) -> None:
        """Capture the (row bucket, logit-row bucket) graphs up front; others are captured on
        first use.  Default: every row bucket with one logit row (single-session decode with
        jump-forward) plus the all-rows variant."""
        if not self.use_graphs:
            return
        for M in buckets:
            if M > self.bufs.max_rows:
                continue
            for L in tuple(logit_buckets) + (M,):
                if L <= M and (M, L, self._gated) not in self.graphs:
                    self._capture(M, L)
        torch.cuda.synchronize()

    def run_rows(self, rows: List[Tuple[Sequence_, int]], logits_for: Optional[List[int]] = None,
                 check: bool = True, defer_head: bool = False) -> Optional[torch.Tensor]:
        """Append one token per row (row = (seq, token)); return f32 logits of the rows listed in
        ``logits_for`` ([len(logits_for), V], default: every row).

        The step graph ends at the final hidden rows; the LM head is its own launch.
        ``defer_head=True`` returns None and leaves it to ``head_logits(col_mask=...)``, so the
        caller can compute the grammar mask on the CPU while the layers run and have the LM head
        skip the vocab tiles no row may sample.

        Rows of the same sequence must be consecutive and in order.  Selecting rows (typically
        the last row of each sequence) keeps the LM head -- the largest GEMM of a step -- at one
        row per sequence when jump-forward appends forced tokens.

        A step that ran the chained launch (models/llama.py) is only valid if none of its grid
        barriers timed out (workgroups not co-resident: another process's persistent kernel on
        the GPU).  ``check=True`` synchronises and verifies that here, re-running the step on the
        per-kernel path if needed.  ``check=False`` leaves it to the caller, who passes
        ``step_fail_word()`` to the sampler (tokens come back as -2 on a failed step) and calls
        ``recover_step()`` -- so the hot decode loop pays no extra synchronisation.
        """
        n = len(rows)
        M = bucket_for(n)
        b = self.bufs
        if self._staging_inflight:
            # back-to-back steps with no host sync in between (several admissions in one scheduler
            # iteration, partial feeds, non-chained check=False steps): the previous step's copy of
            # the staging rows may still be queued behind its forward
            torch.cuda.current_stream().synchronize()
            self._staging_inflight = False
        if getattr(self, "_chain_retry_at", None) is not None:
            self._maybe_rearm_chain()
        if logits_for is None or len(logits_for) == n:
            nl, L = n, M
        else:
            nl = len(logits_for)
            L = min(bucket_for(nl), M)
            if L < M:  # (L == M: no saving -- compute every row and index on the host side)
                b.np_sel[:nl] = logits_for
                b.np_sel[nl:L] = logits_for[-1]
        pending: Dict[int, int] = {}
        bs = self.block_size
        toks, poss, sids, slots = [], [], [], []
        rtab = b.np_row_table if b.rt_cols and M <= 4 else None
        for seq, tok in rows:
            sid = seq.sid
            pos = pending.get(sid, seq.n_computed)
            if pos // bs >= len(seq.blocks):
                self._ensure_blocks(seq, pos + 1)
            if pos >= len(seq.tokens):
                seq.tokens.append(tok)
            toks.append(tok)
            poss.append(pos)
            sids.append(sid)
            slots.append(seq.blocks[pos // bs] * bs + pos % bs)
            pending[sid] = pos + 1
        if rtab is not None:  # after the loop: a later row of a sequence may have added its last block
            for i, (seq, _) in enumerate(rows):
                rtab[i, : len(seq.blocks)] = seq.blocks
        hi = b.np_i32
        hi[0, :n] = toks
        hi[1, :n] = poss
        hi[2, :n] = sids
        hi[3, :n] = hi[1, :n] + 1
        b.np_slots[:n] = slots
        b.np_shared[0] = self._shared_prefix(rows, min(poss) + 1)
        b.np_shared[1] = n
        if M > n:  # padded rows: no KV write, 1-token context on scratch block 0
            hi[0:3, n:M] = 0
            hi[3, n:M] = 1
            b.np_slots[n:M] = -1
        b.upload(M, meta=not self.use_graphs)  # the step graphs copy the metadata themselves
        if rtab is not None and not self.use_graphs:
            b.row_table[:M].copy_(b.h_row_table[:M], non_blocking=True)
        if self.chain_gate is not None:
            self._gated = bool(self.chain_gate())
            self.model._chain_gated = self._gated
            self.stats["gated_steps"] = self.stats.get("gated_steps", 0) + int(self._gated)
        chained = self._uses_chain(M)
        if chained:
            self.stats["chained_steps"] = self.stats.get("chained_steps", 0) + 1
        self._last_step = (list(rows), logits_for, {sid: self.seqs[sid].n_computed for sid in pending}) \
            if chained else None
        if self.use_graphs:
            g, hs = self.graphs.get((M, L, self._gated)) or self._capture(M, L)
            g.replay()
            self.stats["graph_replays"] += 1
        else:
            hs = self._forward_rows(M, L)
        self._staging_inflight = self.device.type == "cuda"
        for sid, ln in pending.items():
            self.seqs[sid].n_computed = ln
        self.stats["steps"] += 1
        self.stats["rows"] += n
        if self.stats["steps"] % 64 == 0:
            self._check_chain()
        if check and chained and self.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
            self._staging_inflight = False
            if self.model.chain_error():
                self._head_rows = None
                return self.recover_step()
        if L == M and nl != n:
            b.h_head_idx[:nl] = torch.as_tensor(logits_for, dtype=torch.int64)
            idx = b.head_idx[:nl]
            idx.copy_(b.h_head_idx[:nl], non_blocking=hs.device.type == "cuda")
            self._head_rows = hs.index_select(0, idx)
        else:
            self._head_rows = hs[:nl]
        if defer_head:
            return None
        return self.head_logits()

    def host_synced(self) -> None:
        """The caller has observed the stream past the last step (e.g. read its sampled tokens):
        the next run_rows may rewrite the pinned staging rows without a synchronize."""
        self._staging_inflight = False

    def head_logits(self, col_mask: Optional[torch.Tensor] = None, mask_rows: int = 1,
                    gather: bool = True) -> torch.Tensor:
        """LM head of the last ``run_rows`` step's selected rows -> f32 logits [rows, V].
        col_mask: the sampler's int32 token bitmask rows (row i <-> logits row i); vocab tiles with
        no admissible token in the first ``mask_rows`` rows are skipped and their logits are stale
        (read them only through the same mask).  gather=False under TP: this rank's vocab shard
        (feed it to ``sample``)."""
        hs = self._head_rows
        assert hs is not None, "head_logits() needs a run_rows() step first"
        if gather:
            return self.model.lm_logits(self.bufs, hs, col_mask=col_mask, mask_rows=mask_rows)
        return self.model.lm_logits(self.bufs, hs, col_mask=col_mask, mask_rows=mask_rows, gather=False)

    def sample(self, logits: torch.Tensor, **kw) -> torch.Tensor:
        """ops.sample over ``head_logits(gather=False)`` output: vocab-parallel under TP (the
        shard's global offset and the TP group come from the model)."""
        m = self.model
        tp = getattr(m, "tp", None)
        if tp is not None and tp.size > 1:
            kw.update(v_offset=m.v_start, tp=tp)
        return ops.sample(logits, **kw)

    def _uses_chain(self, M: int) -> bool:
        ok = getattr(self.model, "_chain_any", None) or getattr(self.model, "_chain_ok", None)
        return bool(ok is not None and ok(M))

    def step_fail_word(self) -> Optional[torch.Tensor]:
        """The device word that is nonzero if the last step's chained launch timed out (None when
        the last step did not run the chain): pass it to ops.sample as ``fail_word``."""
        if self._last_step is None:
            return None
        return self.model.chain_error_word()

    def recover_step(self) -> torch.Tensor:
        """After a chained step failed (its grid barrier timed out, so its logits -- and the K/V it
        wrote -- are invalid): switch the model to per-kernel launches, drop the captured graphs,
        clear the error word and re-run the same rows (their K/V slots are rewritten).  Returns
        the re-run step's logits.  Call only after the host has synchronised with the step."""
        import warnings

        rows, logits_for, pre = self._last_step
        self._last_step = None
        self._tp_chain_fatal()
        warnings.warn("chained decode launch timed out at a grid barrier; re-running the step with "
                      "per-kernel launches")
        word = self.model.chain_error_word()
        self.model.disable_chain()
        if word is not None:
            word.zero_()
        if getattr(self, "_chain_err_h", None) is not None:
            self._chain_err_h.zero_()  # the pinned copy may hold this failure: _check_chain must not re-see it
        self.graphs.clear()
        self.stats["chain_fallbacks"] = self.stats.get("chain_fallbacks", 0) + 1
        self._schedule_chain_retry()
        self.stats["steps"] -= 1
        self.stats["rows"] -= len(rows)
        for sid, n_done in pre.items():
            self.seqs[sid].n_computed = n_done
        return self.run_rows(rows, logits_for)

    def _check_chain(self, blocking: bool = False) -> None:
        """Health check of the chained decode launch (models/llama.py): a grid-barrier spin that
        timed out (workgroups not co-resident, e.g. another persistent kernel on the GPU) leaves an
        error word; the model then falls back to per-kernel launches and the graphs are recaptured.
        Non-blocking by default: reads the word copied to pinned memory at the previous check (the
        step has been synchronised since) and queues the next copy."""
        m = self.model
        if getattr(m, "chain_error", None) is None or getattr(m, "_chain_disabled", False):
            return  # (already on the per-kernel path: a recovery handled this failure)
        if blocking or self.device.type != "cuda":
            err = m.chain_error()
        else:
            word = m.chain_error_word()
            if word is None:
                return
            if getattr(self, "_chain_err_h", None) is None:
                self._chain_err_h = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            err = bool(self._chain_err_h.item() != 0)
            self._chain_err_h.copy_(word, non_blocking=True)
        if err:
            import warnings

            self._tp_chain_fatal()
            warnings.warn("chained decode launch timed out at a grid barrier; using per-kernel launches")
            m.disable_chain()
            self.graphs.clear()
            self.stats["chain_fallbacks"] = self.stats.get("chain_fallbacks", 0) + 1
            self._schedule_chain_retry()

    def _tp_chain_fatal(self) -> None:
        """Under tensor parallelism a chained launch that timed out (a peer's rounds never came)
        leaves the ranks' in-launch round counters and K/V in disagreement: no per-rank fallback
        can restore lockstep, so the step fails loudly: brain/tp_engine.py fails the in-flight
        requests and exits the process, and the launcher restarts the TP group."""
        tp = getattr(self.model, "tp", None)
        if tp is not None and tp.size > 1:
            raise TPGroupFailure("chained TP decode launch timed out waiting for a peer rank")

    def _schedule_chain_retry(self) -> None:
        """A chain timeout usually means another kernel held CUs for a while (e.g. the ASR engine
        on another stream of the same GPU): the chained launch is re-armed after 256 steps, then
        after 512, 1024, ... (capped at 65536) if it keeps failing (``VWA_CHAIN_RETRY=0``: never)."""
        if not ops.env_flag("VWA_CHAIN_RETRY") or not hasattr(self.model, "enable_chain"):
            return
        self._chain_backoff = min(2 * getattr(self, "_chain_backoff", 128), 1 << 16)
        self._chain_retry_at = self.stats["steps"] + self._chain_backoff

    def _maybe_rearm_chain(self) -> None:
        at = getattr(self, "_chain_retry_at", None)
        if at is None or self.stats["steps"] < at:
            return
        self._chain_retry_at = None
        if self.device.type == "cuda":
            torch.cuda.current_stream().synchronize()  # no launch in flight uses the counters
        if getattr(self.bufs, "attn_cnt", None) is not None:
            self.bufs.attn_cnt.zero_()
        self.model.enable_chain()
        self.graphs.clear()
        self.stats["chain_rearms"] = self.stats.get("chain_rearms", 0) + 1

    def prefill_batch(self, items: List[Tuple[Sequence_, int]], chunk: int = 2048) -> None:
        """Admission prefill of several requests in as few forwards as possible: the K/V of every
        ``seq.tokens[n_computed:upto]`` for each (seq, upto).  Sequences whose uncached part is
        longer than what sits before it (a cold prompt: its own self-attention dominates) take the
        single-sequence path (flash attention); the others -- prompt suffixes behind the cached
        static prefix, ~85 tokens each for the intent prompt -- are concatenated into ONE ragged
        row set (each row: its sequence, position, KV slot, causal context), run through the
        step graphs when they fit a decode bucket and otherwise as eager forwards of up to
        ``chunk`` rows: the projections then run as prompt-sized MFMA GEMMs (gemm.hip) shared by
        every request instead of one weight pass per request (reference: each /parse sends its
        prompt independently, apps/brain/src/server.ts:98-105).  No logits are computed."""
        rows: List[Tuple[Sequence_, int]] = []
        for seq, upto in items:
            end = min(upto, len(seq.tokens))
            todo = end - seq.n_computed
            if todo <= 0:
                continue
            if todo > seq.n_computed and todo > self.bufs.max_rows:
                self.prefill(seq, upto=end)
                continue
            rows += [(seq, t) for t in seq.tokens[seq.n_computed:end]]
        if not rows:
            return
        self.stats["prefill_tokens"] += len(rows)
        self.stats["batched_prefills"] = self.stats.get("batched_prefills", 0) + 1
        if len(rows) <= self.bufs.max_rows:
            self.run_rows(rows, logits_for=[len(rows) - 1], check=True, defer_head=True)
            self._head_rows = None
            return
        if self._staging_inflight and self.device.type == "cuda":
            torch.cuda.current_stream().synchronize()
            self._staging_inflight = False
        for i in range(0, len(rows), chunk):
            self._ragged_forward(rows[i : i + chunk])

    def _ragged_forward(self, rows: List[Tuple[Sequence_, int]]) -> None:
        """One eager forward of ragged rows (more than the step buckets hold): the decode-mode
        model forward over scratch buffers sized for them; attention in 64-row slices."""
        n = len(rows)
        bs = self.block_size
        pending: Dict[int, int] = {}
        toks, poss, sids, slots = [], [], [], []
        for seq, tok in rows:
            pos = pending.get(seq.sid, seq.n_computed)
            if pos // bs >= len(seq.blocks):
                self._ensure_blocks(seq, pos + 1)
            toks.append(tok)
            poss.append(pos)
            sids.append(seq.sid)
            slots.append(seq.blocks[pos // bs] * bs + pos % bs)
            pending[seq.sid] = pos + 1
        if self.bufs.table_dirty:
            self.bufs.block_table.copy_(self.bufs.h_table, non_blocking=self.device.type == "cuda")
            self.bufs.table_dirty = False
        dev, m = self.device, self.model
        i32 = dict(dtype=torch.int32)
        meta = torch.tensor([toks, poss, sids, [p + 1 for p in poss]], **i32)
        if dev.type == "cuda":
            meta = meta.pin_memory().to(dev, non_blocking=True)
        d = m.cfg.hidden
        scratch = SimpleNamespace(
            tokens=meta[0], positions=meta[1], seq_ids=meta[2], ctx_lens=meta[3],
            slots=torch.tensor(slots, dtype=torch.int64).to(dev, non_blocking=dev.type == "cuda"),
            block_table=self.bufs.block_table, max_ctx=self.bufs.max_ctx,
            hidden=torch.empty(n, d, dtype=m.dtype, device=dev),
            q=torch.empty(n, m.nq * m.hd, dtype=m.dtype, device=dev),
            attn=torch.empty(n, m.nq * m.hd, dtype=m.dtype, device=dev),
            act=torch.empty(n, getattr(m, "F", getattr(m.cfg, "ffn", d)), dtype=m.dtype, device=dev),
            part_o=self.bufs.part_o, part_ml=self.bufs.part_ml, attn_cnt=self.bufs.attn_cnt,
            logits_local=self.bufs.logits_local, logits=self.bufs.logits,
            flash=self._ragged_flash(sids, poss) if dev.type == "cuda" else None)
        m.forward(scratch, n, self.kv, head=False)
        for sid, ln in pending.items():
            self.seqs[sid].n_computed = ln

    def _ragged_flash(self, sids: List[int], poss: List[int]) -> Optional[SimpleNamespace]:
        """Ragged rows made of whole per-sequence runs (consecutive positions, one run per
        sequence -- the batched admission prefill): the batched causal flash attention layout for
        them ([B runs, S = longest run] queries at absolute offsets, each run's own block-table row)
        -- one launch per layer instead of the decode kernel over 64-row slices."""
        if not PREFILL_FLASH:
            return None
        runs: List[List[int]] = []  # [sid, first row, rows, first position]
        for i, (sid, pos) in enumerate(zip(sids, poss)):
            if runs and runs[-1][0] == sid and pos == poss[i - 1] + 1:
                runs[-1][2] += 1
            else:
                runs.append([sid, i, 1, pos])
        # (one run -- a single request's suffix -- keeps the decode kernel's key-split slices:
        # the batched flash launch then has 32 workgroups for the whole GPU, 41 vs 35 us per
        # layer on the headline's 85-row suffix, profiles/r6_prefill_flash_b1_rejected.md)
        if len(runs) < 2 or len({r[0] for r in runs}) != len(runs):
            return None
        B, S = len(runs), max(r[2] for r in runs)
        if B * S > 2 * len(sids):  # one long run among short ones: mostly padding queries -- slices
            return None
        dst = torch.empty(len(sids), dtype=torch.int64)
        for b, (_, i0, cnt, _) in enumerate(runs):
            dst[i0 : i0 + cnt] = torch.arange(b * S, b * S + cnt)
        dev = self.device
        meta = torch.tensor([[r[3] for r in runs], [r[3] + r[2] for r in runs], [r[0] for r in runs]],
                            dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        return SimpleNamespace(B=B, S=S, dst=dst.pin_memory().to(dev, non_blocking=True), q_offsets=meta[0],
                               k_lens=meta[1], table=self.bufs.block_table.index_select(0, meta[2]),
                               max_k=max(r[3] + r[2] for r in runs))

    def prefill(self, seq: Sequence_, chunk: int = 2048, upto: Optional[int] = None) -> Optional[torch.Tensor]:
        """Compute K/V for seq.tokens[n_computed:upto] (default: all tokens); returns f32 logits
        of the last computed token [1, V] (None if there was nothing to compute)."""
        end = len(seq.tokens) if upto is None else min(upto, len(seq.tokens))
        todo = end - seq.n_computed
        if todo <= 0:
            return None
        self.stats["prefill_tokens"] += todo
        logits = None
        while seq.n_computed < end:
            start = seq.n_computed
            n = min(chunk, end - start)
            if n <= self.bufs.max_rows:
                toks = seq.tokens[start : start + n]
                logits = self.run_rows([(seq, t) for t in toks], logits_for=[n - 1])
                continue
            self._ensure_blocks(seq, start + n)
            if self.bufs.table_dirty:
                self.bufs.block_table.copy_(self.bufs.h_table)
                self.bufs.table_dirty = False
            dev = self.device
            pos = torch.arange(start, start + n, dtype=torch.int32)
            slots = torch.tensor([self.slot_of(seq, int(p)) for p in pos], dtype=torch.int64)
            m = self.model
            scratch = SimpleNamespace(
                tokens=torch.tensor(seq.tokens[start : start + n], dtype=torch.int32, device=dev),
                positions=pos.to(dev), slots=slots.to(dev), block_table=self.bufs.block_table,
                hidden=torch.empty(n, m.cfg.hidden, dtype=m.dtype, device=dev),
                q=torch.empty(n, m.nq * m.hd, dtype=m.dtype, device=dev),
                act=torch.empty(n, m.F, dtype=m.dtype, device=dev),
                logits_local=self.bufs.logits_local, logits=self.bufs.logits, max_ctx=self.bufs.max_ctx,
                part_o=self.bufs.part_o, part_ml=self.bufs.part_ml, attn_cnt=self.bufs.attn_cnt,
            )
            logits = m.forward(scratch, n, self.kv, prefill_seq=seq.sid, q_offset=start,
                               logits_rows=slice(n - 1, n))
            seq.n_computed = start + n
        return logits
