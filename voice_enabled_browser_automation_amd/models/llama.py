"""Llama-3 family decoder (the intent-parsing LLM: replaces the hosted chat model called at
apps/brain/src/llm.ts:22-27).

MI355X-first layout (see ops/__init__.py): fused + row-permuted QKV with the input RMSNorm
gamma folded in, interleaved gate/up with the post-attention gamma folded in, final-norm
gamma folded into the LM head.  A decode layer is therefore 5 kernels:

    skinny_gemm_qkv (rms + QKV + RoPE + paged-KV write) -> decode_attention ->
    skinny_gemm(o_proj, residual epilogue) -> skinny_gemm_swiglu (rms + gate/up + SiLU*up) ->
    skinny_gemm(down, residual epilogue)

Tensor parallelism (one process per GPU, torch.distributed over RCCL/xGMI):
column-parallel QKV (heads split) and gate/up, row-parallel o/down with ONE all-reduce each
(rank 0 adds the residual in its epilogue, the others contribute their partial product, the
all-reduce then produces h_new = h + sum_r partial_r in place; decode steps of <= 4 rows do
both all-reduces as in-launch rounds of the chained layer), vocab-parallel embedding (one
all-reduce) and LM head whose logits stay sharded: the sampler exchanges per-rank partial maxima,
never logits (ops.sample tp=...).  Weights are generated (or loaded) full-size per layer with a
deterministic generator and sliced, so a TP model is numerically the same model as TP=1.
"""
from __future__ import annotations

import weakref
from dataclasses import dataclass
from typing import List, Optional

import torch

from .. import ops
from ..parallel.tp import TPContext
from .config import LlamaConfig


@dataclass
class LlamaLayerWeights:
    qkv: torch.Tensor   # [(nq_l + 2 nkv_l) * hd, d]   permuted rows, input-norm folded
    o: torch.Tensor     # [d, nq_l * hd]
    gu: torch.Tensor    # [2 * F_l, d]  interleaved gate/up, post-attn norm folded
    down: torch.Tensor  # [d, F_l]


def _randn(gen: torch.Generator, shape, std: float, device, dtype) -> torch.Tensor:
    t = torch.empty(shape, device=device, dtype=torch.float32)
    t.normal_(0.0, std, generator=gen)
    return t.to(dtype)


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, *, device="cpu", dtype=torch.bfloat16, tp: Optional[TPContext] = None,
                 seed: int = 0, weights: Optional[dict] = None, wdtype: str = "bf16"):
        """wdtype: "bf16", or "fp8" (OCP e4m3 projection + LM-head weights with per-row scales,
        W8A8 decode GEMMs on the fp8 MFMA; embeddings, norms and the KV cache stay bf16)."""
        self.cfg = cfg
        self.wdtype = wdtype
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPContext.single()
        T = self.tp.size
        assert cfg.n_heads % T == 0 and cfg.n_kv_heads % T == 0, "TP size must divide the head counts"
        assert cfg.ffn % (16 * T) == 0 and cfg.vocab_size % 1 == 0
        self.nq = cfg.n_heads // T
        self.nkv = cfg.n_kv_heads // T
        self.F = cfg.ffn // T
        self.hd = cfg.head_dim
        V = cfg.vocab_size
        # vocab shards start on 32-token boundaries: the grammar mask words (32 tokens each) and
        # the masked LM head's tile skipping then line up with every shard
        self.v_per = ((V + T - 1) // T + 31) // 32 * 32
        self.v_start = self.tp.rank * self.v_per
        self.v_end = min(V, self.v_start + self.v_per)
        # (32-aligned shards can leave the last ranks past the end of a small vocabulary: refuse)
        if (T - 1) * self.v_per >= V:
            raise ValueError(f"vocab {V} cannot be split into {T} 32-aligned shards (last shard empty)")
        self.rope = ops.rope_table(cfg.max_pos, cfg.head_dim, cfg.rope_theta, device=self.device)
        self.scale = cfg.head_dim ** -0.5
        if self.device.type == "meta":
            self._init_meta()  # shapes only (memory planning / sharding checks of configs too big to build)
        elif weights is not None:
            self._load(weights)
        else:
            self._init_random(seed)
        if wdtype == "fp8":
            self._quantize_fp8()
        elif wdtype != "bf16":
            raise ValueError(f"unsupported weight dtype {wdtype!r} (bf16 | fp8)")
        elif self.device.type == "cuda" and dtype == torch.bfloat16 and ops.env_flag("VWA_TILED_WEIGHTS"):
            self._tile_weights()

    def _tile_weights(self) -> None:
        """Every projection + the LM head re-laid out ONCE into the pre-tiled MFMA-fragment order
        (ops.TiledWeight; the row-major copy is freed): the decode streaming / chained kernels read
        it with 1 KB contiguous load instructions (Llama-3-8B layer tail 89.6 vs 101.4 us,
        tools/chain_probe.py) and the prefill / many-row GEMM (gemm.hip) stages it to LDS as is."""
        T = ops.TiledWeight
        for L in self.layers:
            L.qkv, L.o, L.gu, L.down = T(L.qkv), T(L.o), T(L.gu), T(L.down)
        self.lm_head = T(self.lm_head)
        torch.cuda.empty_cache()

    def _quantize_fp8(self) -> None:
        """OCP e4m3 + per-row scales; on the GPU stored once, in the fp8 tiled layout
        (ops.tile_weight_fp8) the W8A8 streaming kernel and the fp8 GEMM read."""
        tiled = self.device.type == "cuda" and ops.env_flag("VWA_TILED_WEIGHTS")
        q = lambda w: ops.FP8Weight.quantize(w, tiled=tiled)  # noqa: E731
        for L in self.layers:
            L.qkv, L.o, L.gu, L.down = q(L.qkv), q(L.o), q(L.gu), q(L.down)
        self.lm_head = q(self.lm_head)
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def param_bytes(self) -> int:
        """Resident bytes of every weight this rank holds (projections, LM head, embedding shard,
        fp8 scales): one copy each."""
        ts = [self.lm_head] + [t for L in self.layers for t in (L.qkv, L.o, L.gu, L.down)]
        n = sum(t.numel() * t.element_size() for t in ts) + self.embed.numel() * self.embed.element_size()
        n += sum(t.scale.numel() * 4 for t in ts if isinstance(t, ops.FP8Weight))
        return n

    # ------------------------------------------------------------------ weights
    def _shard_layer(self, q, k, v, o, g, u, dn, in_norm, post_norm):
        cfg, T, r, hd = self.cfg, self.tp.size, self.tp.rank, self.hd
        qs = q.view(cfg.n_heads, hd, -1)[r * self.nq : (r + 1) * self.nq].reshape(-1, cfg.hidden)
        ks = k.view(cfg.n_kv_heads, hd, -1)[r * self.nkv : (r + 1) * self.nkv].reshape(-1, cfg.hidden)
        vs = v.view(cfg.n_kv_heads, hd, -1)[r * self.nkv : (r + 1) * self.nkv].reshape(-1, cfg.hidden)
        qkv = torch.cat([qs, ks, vs], 0)
        qkv = ops.fold_norm(qkv, in_norm)
        qkv = ops.permute_qkv_rows(qkv, self.nq + 2 * self.nkv, hd)
        os_ = o[:, r * self.nq * hd : (r + 1) * self.nq * hd].contiguous()
        F = self.F
        gs, us = g[r * F : (r + 1) * F], u[r * F : (r + 1) * F]
        gu = ops.interleave_gate_up(ops.fold_norm(gs, post_norm), ops.fold_norm(us, post_norm))
        ds = dn[:, r * F : (r + 1) * F].contiguous()
        return LlamaLayerWeights(qkv=qkv.contiguous(), o=os_, gu=gu, down=ds)

    def _init_random(self, seed: int):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        gen = torch.Generator(device=dev)
        std = cfg.init_std
        gen.manual_seed(seed * 1000003 + 1)
        embed = _randn(gen, (cfg.vocab_size, cfg.hidden), std, dev, dt)
        self.embed = self._vocab_shard(embed)
        ones = torch.ones(cfg.hidden, device=dev, dtype=dt)
        self.layers: List[LlamaLayerWeights] = []
        for li in range(cfg.n_layers):
            gen.manual_seed(seed * 1000003 + 7919 * (li + 2))
            q = _randn(gen, (cfg.n_heads * cfg.head_dim, cfg.hidden), std, dev, dt)
            k = _randn(gen, (cfg.n_kv_heads * cfg.head_dim, cfg.hidden), std, dev, dt)
            v = _randn(gen, (cfg.n_kv_heads * cfg.head_dim, cfg.hidden), std, dev, dt)
            o = _randn(gen, (cfg.hidden, cfg.n_heads * cfg.head_dim), std, dev, dt)
            g = _randn(gen, (cfg.ffn, cfg.hidden), std, dev, dt)
            u = _randn(gen, (cfg.ffn, cfg.hidden), std, dev, dt)
            dn = _randn(gen, (cfg.hidden, cfg.ffn), std, dev, dt)
            self.layers.append(self._shard_layer(q, k, v, o, g, u, dn, ones, ones))
            del q, k, v, o, g, u, dn
        gen.manual_seed(seed * 1000003 + 3)
        if cfg.tie_embeddings:
            lm = embed
        else:
            lm = _randn(gen, (cfg.vocab_size, cfg.hidden), std, dev, dt)
        self.lm_head = ops.fold_norm(lm[self.v_start : self.v_end], ones).contiguous()
        del embed, lm
        if self.device.type == "cuda":
            torch.cuda.empty_cache()

    def _init_meta(self):
        cfg, hd, F = self.cfg, self.hd, self.F
        e = lambda *shape: torch.empty(*shape, device="meta", dtype=self.dtype)  # noqa: E731
        self.embed = e(self.v_end - self.v_start, cfg.hidden)
        self.layers = [LlamaLayerWeights(qkv=e((self.nq + 2 * self.nkv) * hd, cfg.hidden), o=e(cfg.hidden, self.nq * hd),
                                         gu=e(2 * F, cfg.hidden), down=e(cfg.hidden, F))
                       for _ in range(cfg.n_layers)]
        self.lm_head = e(self.v_end - self.v_start, cfg.hidden)

    def _vocab_shard(self, embed: torch.Tensor) -> torch.Tensor:
        """This rank's rows [v_start, v_end) of the token embedding (SURVEY.md §2.7 K14 / §2.8 C3:
        rows outside the shard embed to zero, the all-reduce after the gather completes them)."""
        if self.tp.size == 1:
            return embed
        return embed[self.v_start : self.v_end].contiguous()

    def _load(self, w: dict):
        """HF-layout state dict (safetensors names); sharded + fused on load."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        get = lambda n: w[n].to(device=dev, dtype=dt)  # noqa: E731
        embed = get("model.embed_tokens.weight")
        self.embed = self._vocab_shard(embed)
        self.layers = []
        for li in range(cfg.n_layers):
            p = f"model.layers.{li}."
            self.layers.append(self._shard_layer(
                get(p + "self_attn.q_proj.weight"), get(p + "self_attn.k_proj.weight"),
                get(p + "self_attn.v_proj.weight"), get(p + "self_attn.o_proj.weight"),
                get(p + "mlp.gate_proj.weight"), get(p + "mlp.up_proj.weight"), get(p + "mlp.down_proj.weight"),
                get(p + "input_layernorm.weight"), get(p + "post_attention_layernorm.weight")))
        lm = get("lm_head.weight") if "lm_head.weight" in w else embed
        self.lm_head = ops.fold_norm(lm[self.v_start : self.v_end], get("model.norm.weight")).contiguous()

    def weight_bytes(self) -> int:
        """Bytes streamed per decode step (projections + LM head, one layout of each; one
        embedding row is noise)."""
        ts = [self.lm_head] + [t for L in self.layers for t in (L.qkv, L.o, L.gu, L.down)]
        return sum(t.numel() * t.element_size() for t in ts)

    # ------------------------------------------------------------------ forward
    def _rms_stats(self, M: int):
        """The two RMS-statistics buffers of the per-kernel many-row path (None when the projections
        run elsewhere: <= 16 rows -- the streaming kernels fuse the RMSNorm themselves -- CPU, or TP,
        whose row-parallel outputs are partial sums until the all-reduce)."""
        if M <= ops.SKINNY_MAX_M or self.device.type != "cuda" or self.tp.size > 1 or \
                not ops.env_flag("VWA_RMS_HANDOFF"):
            return None
        if getattr(self, "_ss", None) is None:
            # (int64: u64 fixed-point sums, ops.SS_SCALE -- integer atomics keep them reproducible)
            self._ss = torch.zeros(2, 4096, dtype=torch.int64, device=self.device)
        if M > self._ss.shape[1]:
            return None
        # (the residual GEMMs keep ss[0] zero between forwards; cleared here too, so an interrupted
        # forward cannot leave partial sums behind)
        self._ss[0].zero_()
        return self._ss[0], self._ss[1]

    def _row_parallel(self, x: torch.Tensor, w: torch.Tensor, h: torch.Tensor, ss=None):
        """h <- h + x @ w^T summed over TP ranks (one all-reduce, residual folded into rank 0).
        ss = (out, zero): the rows' sums of squares go to ``out``, ``zero`` is cleared (one rank)."""
        if self.tp.size == 1:
            ops.linear(x, w, out=h, residual=h, ss_out=ss[0] if ss else None, ss_zero=ss[1] if ss else None)
        else:
            if self.tp.rank == 0:
                ops.linear(x, w, out=h, residual=h)
            else:
                ops.linear(x, w, out=h)
            self.tp.all_reduce(h)

    # ---- chained layer tail (o_proj -> gate/up -> down -> next QKV in one launch; M <= 4 rows)
    def _chain_ok(self, M: int) -> bool:
        # 5..16 rows (jump-forward feeds, concurrent sessions): the chain without its attention
        # phase, the down projection streaming X with the weights (skinny_stream.hip XG2)
        # fp8: the W8A16 chain over the fp8 tiled weights (<= 4 rows: no X streaming)
        fp8_ok = self.wdtype == "fp8" and M <= 4 and isinstance(self.layers[0].o, ops.FP8Weight) and self.layers[0].o.tiled
        # TP > 1: the one-shot all-reduce buffers carry the in-launch rounds (chain_tp_reduce)
        tp_ok = self.tp.size == 1 or (getattr(self.tp, "custom_ar", None) is not None and ops.env_flag("VWA_CHAIN_TP"))
        return (M <= ops.env_int("VWA_CHAIN_MAX_ROWS") and tp_ok and (self.wdtype == "bf16" or fp8_ok)
                and self.device.type == "cuda" and not getattr(self, "_chain_disabled", False)
                and not getattr(self, "_chain_gated", False)
                and ops.env_flag("VWA_CHAIN") and ops.native_available())

    def _chain_any(self, M: int) -> bool:
        """Whether a step of M rows runs a chained launch: the engine then checks the launch's
        barrier error word and re-runs a timed-out step on the per-kernel path.  (Round 4's 2-phase
        o_proj -> gate/up chain for 5..16 rows measured no faster -- its barrier cost what the saved
        launch gap did, profiles/r4_chain2_o_gu_rows.jsonl -- and was removed in round 5.)"""
        return self._chain_ok(M)

    def disable_chain(self) -> None:
        self._chain_disabled = True
        self.reset_chains()

    def enable_chain(self) -> None:
        """Re-arm the chained launch after a fallback (runtime/engine.py retries with backoff): a
        timed-out launch leaves partial arrivals in the barrier tickets, split-tile tickets and
        the error word, so they restart from zero (call with no chained launch in flight).
        Under TP the ranks' in-launch round counters would no longer agree: never re-armed."""
        if self.tp.size > 1:
            return
        for t in (getattr(self, "_chain_bar", None), getattr(self, "_chain_work", None)):
            if t is not None:
                t.zero_()
        self._chain_disabled = False
        self.reset_chains()

    def reset_chains(self) -> None:
        """Drop every cached chain descriptor (they embed raw device pointers of the buffers)."""
        self._chains = weakref.WeakKeyDictionary()

    def chain_descs(self):
        """Every cached descriptor entry over all live engines' buffers (tests / diagnostics)."""
        return [v for d in getattr(self, "_chains", {}).values() for k, v in d.items() if k[0] != "multi"]

    def _chain_desc(self, bufs, kv, M: int, li: int):
        """(descriptor, n_phases, lds) of layer li's chained tail for this engine's buffers,
        built on first use (an eager warm-up call precedes every graph capture).

        The descriptors hold raw device pointers into ``bufs`` and ``kv``, so the cache lives in
        a WeakKeyDictionary keyed on the StepBuffers object itself (an entry dies with its
        engine's buffers; a new engine can never see a stale one through a reused ``id()``) and
        the inner key carries the KV pointers and the context bound it was built for."""
        if not isinstance(getattr(self, "_chains", None), weakref.WeakKeyDictionary):
            self.reset_chains()
        cache = self._chains.setdefault(bufs, {})
        key = (M, li, kv.k[li].data_ptr(), kv.v[li].data_ptr(), bufs.max_ctx)
        if key in cache:
            return cache[key]
        if getattr(self, "_chain_bar", None) is None:
            self._chain_bar, self._chain_bar_mode, self._chain_work = ops.chain_buffers(self.device)
        L = self.layers[li]
        nxt = li + 1 < len(self.layers)
        N = self.layers[li + 1] if nxt else None
        # the layer's decode attention as the launch's first phase (VWA_CHAIN_ATTN, default on;
        # same-box bench A/B/A: GPU time per decode step 3868 vs 3897 / 3907 us, p50 276 vs 284 /
        # 285 ms, profiles/r1_bench_results.jsonl; skinny_stream.hip chain_kernel)
        # (the chained attention addresses K/V through per-row copies of the block table, which
        # the step buffers keep for contexts of <= 128 blocks, in 16-token blocks: otherwise the
        # separate launch)
        attn = (M <= 4 and self.hd == 128 and self.nq // self.nkv in (4, 8) and ops.env_flag("VWA_CHAIN_ATTN")
                and ops.decode_n_splits(bufs.max_ctx) > 1 and getattr(bufs, "rt_cols", 0) > 0
                and kv.k[li].shape[2] == 16)
        a = {}
        if attn:
            lay = ops.KVLayout.paged(kv.k[li], kv.v[li], bufs.block_table)
            a = dict(a_q=bufs.q[:M], a_k=lay.k, a_v=lay.v, a_table=lay.table, a_block_size=lay.block_size,
                     a_sb=lay.sb, a_sh=lay.sh, a_st=lay.st, a_ctx=bufs.ctx_lens, a_seq=bufs.seq_ids,
                     a_scale=self.scale, a_n_splits=ops.decode_n_splits(bufs.max_ctx), a_part_o=bufs.part_o,
                     a_part_ml=bufs.part_ml, a_counters=bufs.attn_cnt, a_row_table=bufs.row_table)
            if ops.env_flag("VWA_CHAIN_PLAN"):
                # the attention partition is the same for every layer of a step: layer 0's launch
                # writes each workgroup's item, layers 1.. read it (mq_attention.h step plan)
                if getattr(bufs, "attn_plan", None) is None:
                    bufs.attn_plan = torch.zeros(1024 * 16, dtype=torch.int32, device=self.device)
                a.update(a_plan=bufs.attn_plan, a_plan_mode=1 if li == 0 else 2)
        f8 = isinstance(L.o, ops.FP8Weight)
        tiled = f8 or isinstance(L.o, ops.TiledWeight)
        wsel = (lambda w: w.w8) if f8 else (lambda w: w.t) if tiled else (lambda w: w)  # noqa: E731
        sc = {}
        if f8:  # W8A16 chain: fp8 tiled weights converted to bf16 in registers, per-row scales in the epilogues
            sc = dict(s_o=L.o.scale, s_gu=L.gu.scale, s_down=L.down.scale, s_qkv=N.qkv.scale if nxt else None)
        def make(a):
            return ops.ext().chain_make(
                bufs.hidden[:M], bufs.attn[:M], bufs.act[:M], wsel(L.o), wsel(L.gu), wsel(L.down), self.cfg.rms_eps,
                wsel(N.qkv) if nxt else None, self.nq, self.nkv, self.hd,
                bufs.positions if nxt else None, bufs.slots if nxt else None, self.rope if nxt else None,
                bufs.q[:M] if nxt else None, kv.k[li + 1] if nxt else None, kv.v[li + 1] if nxt else None,
                self._chain_bar, self._chain_work, None, self._chain_bar_mode, **a, w_tiled=tiled, **sc,
                tp_ar=self.tp.custom_ar.state if self.tp.size > 1 else 0)

        desc, lds = make(a)
        if not desc.numel() and attn:
            # shapes the attention phase cannot share a launch with (Llama-3-70B at 3-4 rows: the
            # 28672-wide down-projection X rows exceed LDS, and X streaming has no attention
            # instantiation): chain the tail, the decode attention as its own launch
            attn = False
            desc, lds = make({})
        cache[key] = (desc, 4 if nxt else 3, lds, self.nq // self.nkv if attn else 0) if desc.numel() else None
        return cache[key]

    def _chain_multi(self, bufs, kv, M: int):
        """(descriptors, lds, attn_g, n) of ONE launch over all n = L layers (4-phase tails with the
        attention phase, the last one a 3-phase tail; skinny_stream.hip chain_kernel MULTI), or None
        when some layer cannot take it (per-layer chained / per-kernel launches then).  The
        descriptors are the per-layer ones (_chain_desc) concatenated into one device array; layer
        0's writes the attention step plan that layers 1.. of the same launch read, so a plan can
        never be stale (a per-layer launch whose layer 0 dropped its attention phase would
        have left layers 1.. reading an older step's entry)."""
        n = len(self.layers)
        if n < 3 or not ops.env_flag("VWA_CHAIN_MULTI") or self.tp.size > 1 and not ops.env_flag("VWA_CHAIN_TP"):
            return None
        cache = self._chains.setdefault(bufs, {}) if isinstance(getattr(self, "_chains", None), weakref.WeakKeyDictionary) else None
        key = ("multi", M, tuple(kv.k[li].data_ptr() for li in range(n)),
               tuple(kv.v[li].data_ptr() for li in range(n)), bufs.max_ctx)
        if cache is not None and key in cache:
            return cache[key]
        ds = [self._chain_desc(bufs, kv, M, li) for li in range(n)]
        ok = (all(d is not None and d[3] > 0 for d in ds) and all(d[1] == 4 for d in ds[:-1]) and ds[-1][1] == 3
              and len({(d[2], d[3]) for d in ds}) == 1)
        lds = ds[0][2] if ok else 0
        # the instantiations: o_proj in 32-column tiles (bf16) or fp8 weights, no X streaming
        ok = ok and not (lds >> 24) & 1 and ((lds >> 25) & 1) != ((lds >> 26) & 1)
        out = (torch.cat([d[0] for d in ds]), lds, ds[0][3], n) if ok else None
        self._chains.setdefault(bufs, {})[key] = out
        return out

    def chain_error_word(self):
        """The device word a timed-out chain barrier sets (None before the first chained launch)."""
        return ops.chain_error_word(getattr(self, "_chain_bar", None))

    def chain_error(self) -> bool:
        """True when a chained launch's grid barrier timed out (results of that step are invalid)."""
        bar = getattr(self, "_chain_bar", None)
        return bool(bar is not None and int(bar.view(torch.int64)[160].item()) != 0)

    def forward(self, bufs, M: int, kv, *, prefill_seq: Optional[int] = None, q_offset: int = 0,
                logits_rows: Optional[slice] = None, n_sel: Optional[int] = None, head: bool = True) -> torch.Tensor:
        """Run M token rows described by ``bufs`` (runtime.buffers.StepBuffers).

        Decode/ragged mode (M <= 64): each row is one token of some sequence (seq_ids /
        ctx_lens / positions / slots per row).  Prefill mode (prefill_seq given): the M rows are
        consecutive tokens of table row ``prefill_seq`` starting at position q_offset.
        Returns f32 logits [rows, vocab] (all ranks, gathered under TP) for every row, for
        ``logits_rows``, or (``n_sel``) for the rows listed in ``bufs.sel[:n_sel]``.  head=False:
        the final hidden rows instead (``lm_logits`` turns them into logits -- the engine runs the
        LM head outside the step graph, under the sampler's grammar mask).
        """
        cfg = self.cfg
        h = bufs.hidden[:M]
        ops.embedding(bufs.tokens, self.embed, out=h, rows=M, vocab_start=self.v_start)
        if self.tp.size > 1:
            self.tp.all_reduce(h)  # vocab-parallel embedding: every row is non-zero on one rank only
        qbuf = bufs.q[:M] if M <= bufs.q.shape[0] else torch.empty((M, self.nq * self.hd), dtype=self.dtype,
                                                                      device=self.device)
        chain = prefill_seq is None and self._chain_ok(M)
        # prompt suffix behind a cached prefix (few queries, long keys): the decode attention
        # kernel in <= 64-row slices (per-row causal context, K/V split over many workgroups)
        # instead of flash attention's one workgroup per 64 queries x head (measured 82 us/layer
        # for 84 queries over 1.1k keys: 64 workgroups each walking every key tile)
        pf_slices = None
        if (prefill_seq is not None and q_offset >= M and M <= 256 and self.device.type == "cuda"
                and ops.env_flag("VWA_PREFILL_DECODE_ATTN")):
            i32 = dict(dtype=torch.int32, device=self.device)
            pf_ctx = torch.arange(q_offset + 1, q_offset + M + 1, **i32)
            pf_sid = torch.full((M,), prefill_seq, **i32)
            pf_slices = [(i, min(M, i + 64)) for i in range(0, M, 64)]
            pf_out = torch.empty((M, self.nq * self.hd), dtype=self.dtype, device=self.device)
        # > 16 rows on one rank (the tiled GEMMs): each residual GEMM hands the sums of squares of the
        # rows it writes to the next RMSNorm (ss[0]: after o_proj -> gate/up, ss[1]: after down ->
        # next QKV) and zeroes the other buffer, so no row_rstd launch (GemmParams::ss_*)
        ss = self._rms_stats(M) if not chain else None
        # every layer as ONE chained launch when each of them can take it
        multi = self._chain_multi(bufs, kv, M) if chain else None
        for li, L in enumerate(self.layers):
            kc, vc = kv.k[li], kv.v[li]
            if multi is not None and li < multi[3]:
                if li == 0:
                    ops.qkv_rope_write(h, L.qkv, None, fuse_rms=True, eps=cfg.rms_eps, n_q_heads=self.nq,
                                       n_kv_heads=self.nkv, head_dim=self.hd, rope=self.rope, positions=bufs.positions,
                                       slots=bufs.slots, q_out=qbuf, k_cache=kc, v_cache=vc)
                    ops.ext().chain_run(multi[0], 4, multi[1], h, multi[2], 0, multi[3])
                continue
            if chain and li > 0:
                q = qbuf  # written by the previous layer's chained launch
            else:
                q = ops.qkv_rope_write(h, L.qkv, None, fuse_rms=True, eps=cfg.rms_eps, n_q_heads=self.nq,
                                       n_kv_heads=self.nkv, head_dim=self.hd, rope=self.rope,
                                       positions=bufs.positions, slots=bufs.slots, q_out=qbuf, k_cache=kc, v_cache=vc,
                                       ss_in=ss[1] if ss is not None and li > 0 else None)
            d = self._chain_desc(bufs, kv, M, li) if chain else None
            if d is not None:
                # chained layer: [decode attention ->] o_proj -> gate/up -> down [-> next QKV]
                if not d[3]:
                    ops.decode_attention(q, ops.KVLayout.paged(kc, vc, bufs.block_table), bufs.ctx_lens,
                                         bufs.seq_ids, n_q_heads=self.nq, n_kv_heads=self.nkv, head_dim=self.hd,
                                         scale=self.scale, max_ctx=bufs.max_ctx, out=bufs.attn[:M],
                                         part_o=bufs.part_o, part_ml=bufs.part_ml, counters=bufs.attn_cnt,
                                         shared=getattr(bufs, "shared", None))
                ops.ext().chain_run(d[0], d[1], d[2], h, d[3])
                continue
            chain = False  # shapes the chain cannot take: per-kernel path from here on
            if prefill_seq is None:
                # (ragged rows: a decode step, or the batched admission prefill of several requests'
                # prompt suffixes -- runtime/engine.py prefill_batch -- in 64-row attention slices)
                attn = bufs.attn[:M]
                fl = getattr(bufs, "flash", None)
                if fl is not None:  # whole per-request runs (batched admission prefill)
                    ops.flash_attention_runs(q, kc, vc, fl, n_q_heads=self.nq, n_kv_heads=self.nkv,
                                             head_dim=self.hd, scale=self.scale, out=attn)
                else:
                    ops.decode_attention_rows(q, ops.KVLayout.paged(kc, vc, bufs.block_table), bufs.ctx_lens,
                                              bufs.seq_ids, n_q_heads=self.nq, n_kv_heads=self.nkv, head_dim=self.hd,
                                              scale=self.scale, max_ctx=bufs.max_ctx, out=attn, part_o=bufs.part_o,
                                              part_ml=bufs.part_ml, counters=bufs.attn_cnt,
                                              shared=getattr(bufs, "shared", None))
            elif pf_slices is not None:
                attn = pf_out
                lay = ops.KVLayout.paged(kc, vc, bufs.block_table)
                for i, j in pf_slices:
                    ops.decode_attention(q[i:j], lay, pf_ctx[i:j], pf_sid[i:j], n_q_heads=self.nq,
                                         n_kv_heads=self.nkv, head_dim=self.hd, scale=self.scale,
                                         max_ctx=bufs.max_ctx, out=attn[i:j], part_o=bufs.part_o,
                                         part_ml=bufs.part_ml, counters=bufs.attn_cnt)
            else:
                table = bufs.block_table[prefill_seq : prefill_seq + 1]
                q4 = q.view(1, M, self.nq, self.hd)
                attn4 = torch.empty_like(q4)
                ops.flash_attention(q4, ops.KVLayout.paged(kc, vc, table), Sk=q_offset + M, n_kv_heads=self.nkv,
                                    causal=True, scale=self.scale, q_offset=q_offset, out=attn4)
                attn = attn4.view(M, self.nq * self.hd)
            self._row_parallel(attn, L.o, h, ss and (ss[0], ss[1]))
            act = bufs.act[:M] if M <= bufs.act.shape[0] else None
            act = ops.linear_swiglu(h, L.gu, fuse_rms=True, eps=cfg.rms_eps, out=act, ss_in=ss and ss[0])
            self._row_parallel(act, L.down, h, ss and (ss[1], ss[0]))
        if n_sel is not None:
            hs = torch.index_select(h, 0, bufs.sel[:n_sel], out=bufs.hidden_sel[:n_sel])
        else:
            hs = h[logits_rows if logits_rows is not None else slice(0, M)]
        return self.lm_logits(bufs, hs) if head else hs

    def lm_logits(self, bufs, hs: torch.Tensor, col_mask: Optional[torch.Tensor] = None,
                  mask_rows: int = 1, gather: bool = True) -> torch.Tensor:
        """Final RMSNorm (folded into the weights) + LM head of the hidden rows ``hs`` -> f32 logits
        [rows, vocab] (``gather=False`` under TP: this rank's shard [rows, v_end - v_start], tokens
        v_start.. -- what the vocab-parallel sampler takes; the decode loop never gathers logits).
        col_mask (the sampler's int32 token bitmask rows): only the vocab tiles with an admissible
        token in one of the first ``mask_rows`` rows are computed (ops.linear); the other logits
        are stale and must only be read through the mask."""
        n = hs.shape[0]
        local = bufs.logits_local[:n] if n <= bufs.logits_local.shape[0] else None
        mk = {}
        if col_mask is not None and self.v_start % 32 == 0 and col_mask.shape[1] * 32 >= self.v_end:
            mk = dict(col_mask=col_mask, col_mask_off=self.v_start // 32, mask_rows=mask_rows)
        local = ops.linear(hs, self.lm_head, out=local, fuse_rms=True, eps=self.cfg.rms_eps, out_dtype=torch.float32,
                           **mk)
        if self.tp.size == 1 or not gather:
            return local
        return self.tp.all_gather_vocab(local, self.cfg.vocab_size)


def move_model(model, device) -> None:
    """Move every tensor attribute (incl. dataclass layer records) of a model to `device` in place."""
    import dataclasses

    device = torch.device(device)

    def mv(obj):
        if isinstance(obj, (torch.Tensor, ops.FP8Weight, ops.TiledWeight)):
            return obj.to(device)
        if dataclasses.is_dataclass(obj) and not isinstance(obj, type):
            for f in dataclasses.fields(obj):
                setattr(obj, f.name, mv(getattr(obj, f.name)))
            return obj
        if isinstance(obj, list):
            return [mv(x) for x in obj]
        if isinstance(obj, tuple):
            return tuple(mv(x) for x in obj)
        return obj

    for k, v in list(vars(model).items()):
        if k == "cfg":
            continue
        setattr(model, k, mv(v))
    model.device = device
