"""Per-GPU HBM plan of an intent-LLM rank ("KV sizing from 288 GB/GPU").

One process per GPU; under tensor parallelism every rank holds 1/T of each projection (column-
parallel QKV / gate-up, row-parallel o / down), 1/T of the vocabulary (embedding rows and LM-head
rows, 32-aligned shards) and the KV heads of its query heads.  Every projection is stored ONCE,
in the pre-tiled MFMA layout (ops.TiledWeight) or as OCP fp8 + per-row scales.  What is left of
the GPU after weights, step buffers and workspaces goes to paged KV (or ``kv_gb`` caps it).

    plan_memory(get_config("llama3-70b"), tp=8)  ->  per-rank bytes by category + KV capacity

The plan is pure arithmetic (no allocation), so it is checked on CPU for configurations that
cannot be instantiated here (tests/test_memory_plan_cpu.py: 70B at TP=8), and the engine uses
``kv_blocks`` from it when VWA_KV_GB is "auto".
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Dict, Optional

HBM_BYTES_MI355X = 288 * 1000 ** 3  # 288 GB HBM3E per GPU


@dataclass
class MemoryPlan:
    tp: int
    wdtype: str
    weights: int           # projections + LM head shard (+ fp8 scales)
    embedding: int         # this rank's vocab shard of the token embedding
    step_buffers: int      # fixed-address decode buffers (hidden / q / act / logits / partials)
    workspace: int         # GEMM split-K workspace + one-shot all-reduce staging
    kv_bytes_per_token: int
    kv_blocks: int
    kv_bytes: int
    reserve: int           # runtime / allocator slack
    hbm: int

    @property
    def total(self) -> int:
        return self.weights + self.embedding + self.step_buffers + self.workspace + self.kv_bytes + self.reserve

    @property
    def kv_tokens(self) -> int:
        return self.kv_bytes // max(1, self.kv_bytes_per_token)

    def as_dict(self) -> Dict[str, float]:
        d = asdict(self)
        d.update(total=self.total, kv_tokens=self.kv_tokens, fits=self.total <= self.hbm)
        return d


def _shard(n: int, t: int, align: int = 1) -> int:
    return ((n + t - 1) // t + align - 1) // align * align


def plan_memory(cfg, tp: int = 1, *, wdtype: str = "bf16", kv_gb: Optional[float] = None, block_size: int = 16,
                max_rows: int = 64, max_ctx: int = 4096, hbm: int = HBM_BYTES_MI355X,
                reserve_frac: float = 0.06, gemm_ws_floats: Optional[int] = None, ar_max_elems: int = 64 * 8192,
                shared_gb: float = 0.0, prefill_rows: int = 2048) -> MemoryPlan:
    """Bytes per rank.  ``kv_gb`` None: all remaining HBM after the rest (minus the reserve)
    becomes KV; otherwise that many GB (capped at what remains).  ``shared_gb``: HBM left to a
    co-located service (the voice worker's ASR on a shared single GPU).  The workspace counts the
    GEMM split-K workspace (ops.GEMM_WS_FLOATS), the batched-prefill scratch rows and, under TP,
    the one-shot all-reduce staging + all-gather + chained-layer regions (allreduce.hip)."""
    if gemm_ws_floats is None:
        from .. import ops

        gemm_ws_floats = ops.GEMM_WS_FLOATS
    assert cfg.n_heads % tp == 0 and cfg.n_kv_heads % tp == 0, "TP must divide the head counts"
    d, hd, L = cfg.hidden, cfg.head_dim, cfg.n_layers
    nq, nkv, F = cfg.n_heads // tp, cfg.n_kv_heads // tp, cfg.ffn // tp
    v_per = _shard(cfg.vocab_size, tp, 32)
    elem = 1 if wdtype == "fp8" else 2
    per_layer_rows = (nq + 2 * nkv) * hd + d + 2 * F + d          # qkv, o, gate/up, down output rows
    per_layer = ((nq + 2 * nkv) * hd * d + d * nq * hd + 2 * F * d + d * F) * elem
    scales = per_layer_rows * 4 if wdtype == "fp8" else 0
    lm = v_per * d * elem + (v_per * 4 if wdtype == "fp8" else 0)
    weights = L * (per_layer + scales) + lm
    embedding = v_per * d * 2
    n_splits = -(-max_ctx // 128)
    step = max_rows * (2 * d + 2 * nq * hd + F) * 2 + max_rows * v_per * 4 \
        + max_rows * n_splits * nq * (hd + 2) * 4
    prefill = prefill_rows * (2 * d + 2 * nq * hd + F) * 2  # runtime/engine.py _ragged_forward scratch
    ar = 2 * ar_max_elems * 2 + 2 * 64 * 1024 * 4 + 2 * 16 * 8192 * 4  # staging, gather, chain regions
    workspace = gemm_ws_floats * 4 + prefill + (ar if tp > 1 else 0)
    kv_tok = 2 * L * nkv * hd * 2
    reserve = int(hbm * reserve_frac) + int(shared_gb * 1e9)
    free = hbm - weights - embedding - step - workspace - reserve
    want = free if kv_gb is None else min(free, int(kv_gb * 1e9))
    per_block = kv_tok * block_size
    blocks = max(0, want // per_block)
    return MemoryPlan(tp=tp, wdtype=wdtype, weights=weights, embedding=embedding, step_buffers=step,
                      workspace=workspace, kv_bytes_per_token=kv_tok, kv_blocks=int(blocks),
                      kv_bytes=int(blocks * per_block), reserve=reserve, hbm=hbm)
