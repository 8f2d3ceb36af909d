"""GPT-2 family decoder: the CPU-config intent parser (BASELINE.json config 1: canned transcript
-> GPT-2-small intent parser, no GPU), drop-in for LlamaModel behind runtime.engine.LLMEngine.

Same engine contract as models/llama.py (per-row metadata in ``bufs``, paged KV, ragged decode
rows, optional logit-row selection), so the grammar-constrained scheduler, prefix cache and
continuous batching are shared.  On the GPU every op is the same native kernel family:
embedding with learned positions (K14), LayerNorm (K4), fused QKV GEMM + paged KV write with
RoPE disabled (K9/K12), paged decode attention or causal flash attention (K10/K6), bias + GELU
and bias + residual GEMM epilogues (K12).

Deviations from the public checkpoint layout, by design:
* learned positions are sized by ``max_pos`` (2048 by default; the public model has 1024, too
  short for the ~1.1k-token intent prompt);
* the MLP activation is the erf GELU of the native epilogue (GPT-2 used the tanh
  approximation; |difference| < 1e-3 per activation);
* QKV rows are stored in the per-head permuted order shared with the Llama kernels.
The reference has no local model (its intent parser is a hosted chat model, apps/brain/src/llm.ts:
17-27), so numerical parity with the public GPT-2 is "parity unpinned".
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch

from .. import ops
from ..parallel.tp import TPContext
from .config import GPT2Config


@dataclass
class GPT2LayerWeights:
    ln1_w: torch.Tensor
    ln1_b: torch.Tensor
    qkv: torch.Tensor     # [3 * d, d] permuted per-head rows
    qkv_b: torch.Tensor   # [3 * d]   (same permutation)
    proj: torch.Tensor    # [d, d]
    proj_b: torch.Tensor
    ln2_w: torch.Tensor
    ln2_b: torch.Tensor
    fc: torch.Tensor      # [4d, d]
    fc_b: torch.Tensor
    fc2: torch.Tensor     # [d, 4d]
    fc2_b: torch.Tensor


class GPT2Model:
    def __init__(self, cfg: GPT2Config, *, device="cpu", dtype: Optional[torch.dtype] = None,
                 tp: Optional[TPContext] = None, seed: int = 0, weights: Optional[dict] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        # CPU config runs f32 (no bf16 GEMM units to feed); GPU runs bf16 through the native kernels
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.tp = tp or TPContext.single()
        assert self.tp.size == 1, "GPT-2 (CPU intent-parser config) is single-device"
        self.nq = self.nkv = cfg.n_heads
        self.hd = cfg.hidden // cfg.n_heads
        self.F = cfg.ffn
        self.v_start, self.v_end = 0, cfg.vocab_size
        self.scale = self.hd ** -0.5
        if weights is not None:
            self._load(weights)
        else:
            self._init_random(seed)

    # ------------------------------------------------------------------ weights
    def _perm_qkv(self, w: torch.Tensor) -> torch.Tensor:
        return ops.permute_qkv_rows(w, 3 * self.cfg.n_heads, self.hd)

    def _layer(self, ln1_w, ln1_b, qkv, qkv_b, proj, proj_b, ln2_w, ln2_b, fc, fc_b, fc2, fc2_b):
        d = self.cfg.hidden
        return GPT2LayerWeights(
            ln1_w=ln1_w, ln1_b=ln1_b, qkv=self._perm_qkv(qkv).contiguous(),
            qkv_b=self._perm_qkv(qkv_b.view(3 * d, 1)).view(-1).contiguous(), proj=proj.contiguous(),
            proj_b=proj_b, ln2_w=ln2_w, ln2_b=ln2_b, fc=fc.contiguous(), fc_b=fc_b, fc2=fc2.contiguous(),
            fc2_b=fc2_b)

    def _init_random(self, seed: int):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        d, std = cfg.hidden, cfg.init_std
        gen = torch.Generator(device=dev)

        def rnd(*shape, s=std):
            t = torch.empty(shape, device=dev, dtype=torch.float32)
            t.normal_(0.0, s, generator=gen)
            return t.to(dt)

        def const(v, n):
            return torch.full((n,), v, device=dev, dtype=dt)

        gen.manual_seed(seed * 1000003 + 11)
        self.wte = rnd(cfg.vocab_size, d)
        self.wpe = rnd(cfg.max_pos, d, s=0.01)
        self.layers: List[GPT2LayerWeights] = []
        resid_std = std / (2 * cfg.n_layers) ** 0.5  # GPT-2's scaled init of residual projections
        for li in range(cfg.n_layers):
            gen.manual_seed(seed * 1000003 + 7919 * (li + 2))
            self.layers.append(self._layer(
                const(1.0, d), const(0.0, d), rnd(3 * d, d), const(0.0, 3 * d), rnd(d, d, s=resid_std),
                const(0.0, d), const(1.0, d), const(0.0, d), rnd(cfg.ffn, d), const(0.0, cfg.ffn),
                rnd(d, cfg.ffn, s=resid_std), const(0.0, d)))
        self.lnf_w, self.lnf_b = const(1.0, d), const(0.0, d)
        self.lm_head = self.wte  # tied

    def _load(self, w: dict):
        """HF GPT-2 state dict (Conv1D weights are [in, out]: transposed here)."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = lambda n: w[n].to(device=dev, dtype=dt)  # noqa: E731
        pre = "transformer." if "transformer.wte.weight" in w else ""
        self.wte = g(pre + "wte.weight")
        wpe = g(pre + "wpe.weight")
        if wpe.shape[0] < cfg.max_pos:  # extend learned positions for the long intent prompt
            ext = wpe[-1:].expand(cfg.max_pos - wpe.shape[0], -1)
            wpe = torch.cat([wpe, ext], 0)
        self.wpe = wpe.contiguous()
        self.layers = []
        for li in range(cfg.n_layers):
            p = f"{pre}h.{li}."
            self.layers.append(self._layer(
                g(p + "ln_1.weight"), g(p + "ln_1.bias"), g(p + "attn.c_attn.weight").t(), g(p + "attn.c_attn.bias"),
                g(p + "attn.c_proj.weight").t(), g(p + "attn.c_proj.bias"), g(p + "ln_2.weight"),
                g(p + "ln_2.bias"), g(p + "mlp.c_fc.weight").t(), g(p + "mlp.c_fc.bias"),
                g(p + "mlp.c_proj.weight").t(), g(p + "mlp.c_proj.bias")))
        self.lnf_w, self.lnf_b = g(pre + "ln_f.weight"), g(pre + "ln_f.bias")
        self.lm_head = self.wte

    def weight_bytes(self) -> int:
        n = self.wte.numel() + self.wpe.numel()
        for L in self.layers:
            n += L.qkv.numel() + L.proj.numel() + L.fc.numel() + L.fc2.numel()
        return n * self.wte.element_size()

    # ------------------------------------------------------------------ forward
    def forward(self, bufs, M: int, kv, *, prefill_seq: Optional[int] = None, q_offset: int = 0,
                logits_rows: Optional[slice] = None, n_sel: Optional[int] = None, head: bool = True) -> torch.Tensor:
        """Same contract as LlamaModel.forward (runtime.engine.StepBuffers rows)."""
        cfg = self.cfg
        eps = cfg.ln_eps
        h = bufs.hidden[:M]
        ops.embedding(bufs.tokens, self.wte, pos_table=self.wpe, positions=bufs.positions, out=h, rows=M)
        qbuf = bufs.q[:M] if M <= bufs.q.shape[0] else torch.empty((M, cfg.hidden), dtype=self.dtype,
                                                                      device=self.device)
        for li, L in enumerate(self.layers):
            kc, vc = kv.k[li], kv.v[li]
            x = ops.layernorm(h, L.ln1_w, L.ln1_b, eps=eps)
            q = ops.qkv_rope_write(x, L.qkv, L.qkv_b, fuse_rms=False, eps=eps, n_q_heads=self.nq,
                                   n_kv_heads=self.nkv, head_dim=self.hd, rope=None, positions=bufs.positions,
                                   slots=bufs.slots, q_out=qbuf, k_cache=kc, v_cache=vc)
            if prefill_seq is None:
                attn = bufs.attn[:M]
                ops.decode_attention_rows(q, ops.KVLayout.paged(kc, vc, bufs.block_table), bufs.ctx_lens, bufs.seq_ids,
                                     n_q_heads=self.nq, n_kv_heads=self.nkv, head_dim=self.hd, scale=self.scale,
                                     max_ctx=bufs.max_ctx, out=attn, part_o=bufs.part_o, part_ml=bufs.part_ml,
                                     counters=bufs.attn_cnt)
            else:
                table = bufs.block_table[prefill_seq : prefill_seq + 1]
                q4 = q.view(1, M, self.nq, self.hd)
                attn4 = torch.empty_like(q4)
                ops.flash_attention(q4, ops.KVLayout.paged(kc, vc, table), Sk=q_offset + M, n_kv_heads=self.nkv,
                                    causal=True, scale=self.scale, q_offset=q_offset, out=attn4)
                attn = attn4.view(M, cfg.hidden)
            ops.linear(attn, L.proj, L.proj_b, out=h, residual=h)
            x = ops.layernorm(h, L.ln2_w, L.ln2_b, eps=eps)
            act = bufs.act[:M] if M <= bufs.act.shape[0] else None
            act = ops.linear(x, L.fc, L.fc_b, out=act, act="gelu")
            ops.linear(act, L.fc2, L.fc2_b, out=h, residual=h)
        if n_sel is not None:
            hs = torch.index_select(h, 0, bufs.sel[:n_sel], out=bufs.hidden_sel[:n_sel])
        else:
            hs = h[logits_rows if logits_rows is not None else slice(0, M)]
        return self.lm_logits(bufs, hs) if head else hs

    def lm_logits(self, bufs, hs: torch.Tensor, col_mask: Optional[torch.Tensor] = None,
                  mask_rows: int = 1, gather: bool = True) -> torch.Tensor:
        """Final LayerNorm + tied LM head -> f32 logits (same contract as LlamaModel.lm_logits)."""
        hs = ops.layernorm(hs, self.lnf_w, self.lnf_b, eps=self.cfg.ln_eps)
        n = hs.shape[0]
        out = bufs.logits_local[:n] if n <= bufs.logits_local.shape[0] else None
        V = self.lm_head.shape[0]
        if hs.is_cuda and V % 16:
            # GPT-2's 50257-token vocabulary is not a multiple of the kernels' 16-column tiles: the
            # tied head runs zero-padded to the next multiple (built once) into a scratch, and the
            # real columns are copied out -- no vendor GEMM for the odd shape
            pad = getattr(self, "_lm_pad", None)
            if pad is None or pad.device != hs.device:
                pad = torch.zeros(((V + 15) // 16 * 16, self.lm_head.shape[1]), dtype=self.lm_head.dtype, device=hs.device)
                pad[:V] = self.lm_head
                self._lm_pad = pad
            full = ops.scratch(hs.device, "gpt2_logits", n * pad.shape[0]).view(n, pad.shape[0])
            ops.linear(hs, pad, out=full, out_dtype=torch.float32, col_mask=col_mask, mask_rows=mask_rows)
            if out is None:
                return full[:, :V].contiguous()
            out.copy_(full[:, :V])
            return out
        return ops.linear(hs, self.lm_head, out=out, out_dtype=torch.float32, col_mask=col_mask, mask_rows=mask_rows)
