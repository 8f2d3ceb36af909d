"""Whisper encoder-decoder ASR (replaces Deepgram Nova-3 live STT: apps/voice/src/deepgram.ts:33-45).

Encoder (one pass per 30 s window, batch of sessions = DP):
    log_mel (HIP, K2) -> conv1d+GELU (HIP MFMA implicit GEMM, K3) -> conv1d/s2+GELU+pos (K3)
    -> L x [layernorm (K4) -> QKV GEMM (gemm.hip tiled MFMA) + bias -> flash attention (HIP MFMA, K5)
            -> out-proj + bias + residual (K-epilogue) -> layernorm -> fc1 + bias + GELU -> fc2 + residual]
    -> layernorm -> cross-attention K/V for every decoder layer (computed once per window).
Decoder (per token, hipGraph-captured per batch bucket):
    embedding + learned positions (K14) -> L x [fused QKV skinny GEMM + bias + paged self-KV write
    (K12 QKV epilogue, no RoPE) -> decode attention (K10) -> out-proj residual epilogue -> q skinny
    GEMM -> cross attention over the window's K/V (K7) -> out-proj residual -> fc1 GELU epilogue ->
    fc2 residual epilogue] -> tied LM head (f32) -> masked greedy sampling (K13).  Every decoder
    LayerNorm is folded into the GEMM that consumes it (fold_decoder_norms): 8 launches per layer.
"""
from __future__ import annotations

import math
import weakref
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from .. import ops
from ..ops import reference as ref
from .config import WhisperConfig
from .llama import move_model  # noqa: F401  (re-export)


WDEC_LEVELS = ("qkv", "xq_x", "self_attn", "o_xq", "cross_attn", "xo", "fc1", "fc2")
# gemm ids of the persistent decoder (whisper_dec.hip G_*; WdecLayer::g order) and their levels
WDEC_GEMMS = ("qkv", "o", "xq", "xo", "fc1", "fc2", "xq_o")
WDEC_GEMM_LEVEL = (0, 3, 1, 5, 6, 7, 3)


# role-plan variants for A/B probes (tools/wdec_probe.py --role-opts): att_pen = penalty for a
# refill right before this workgroup's next attention level; sat = "fc2" (self-attention heads on
# the fc2-only workgroups first) or "tail" (on the last workgroups)
WDEC_ROLE_OPTS: dict = {}


def wdec_roles(nwg: int, d: int, H: int, ffn: int, nch: int):
    """Role table of the persistent Whisper decoder (csrc/kernels/whisper_dec.hip): per workgroup
    32 ints -- slot kinds (gemm id, WDEC_GEMMS, or -1), tiles, parts, refill levels, self-attention
    head, cross-attention item, the level after which the next layer's cross K/V chunk is
    prefetched, and the mask of levels it completes -- plus the producer count of each level.

    Every layer's weights are spread so each workgroup holds at most 5 slots of 5 loads per wave
    (one 16-column tile of a K = d projection per slot; an fc2 tile, K = 4 d, takes slots 1..P,
    P = ceil(d / 320): 4 for whisper-large, 2 for tiny):
    fc2 tiles on workgroups [0, d/16), QKV tiles on the last 3 d / 16, the out / cross projections
    and fc1 in the free slots of the rest (at most 2 tiles of a level per workgroup: the epilogue
    finishes 2 in one round), the x part of the cross query last -- on QKV workgroups, which have
    its row staged.  A slot is refilled right after the level that used it (its next use is a
    layer later); workgroups that run the self-attention refill after it, so the attention's loads
    do not queue behind 40-200 KB of weights.  Cross-attention items (head, key chunk) go to the
    fc2 workgroups, idle from the QKV level to fc2; self-attention heads to workgroups with idle
    levels after it."""
    import numpy as np

    assert ffn == 4 * d and d % 128 == 0 and d <= 1536
    n_qkv, n_d, n_ff = 3 * d // 16, d // 16, ffn // 16
    n_p2 = -(-(ffn // 32) // 40)  # slots per fc2 tile (40 slices of 32 k each)
    n_x = H * nch
    if nwg < max(n_qkv, n_d + 16, n_x, H) or n_d > nwg:
        raise ValueError(f"wdec_roles: {nwg} workgroups cannot hold the decoder's tiles")
    R = np.full((nwg, 32), -1, dtype=np.int32)
    R[:, 10:15] = 0
    kind, tile, part, rel = R[:, 0:5], R[:, 5:10], R[:, 10:15], R[:, 15:20]
    GQ, GO, GXQ, GXO, G1, G2, GXQO = range(7)
    LQ, LXQX, LS, LOXQ, LX = 0, 1, 2, 3, 4
    lvl_of = WDEC_GEMM_LEVEL
    for t in range(n_d):  # fc2: slots 1..n_p2 of workgroup t
        kind[t, 1:1 + n_p2], tile[t, 1:1 + n_p2], part[t, 1:1 + n_p2] = G2, t, np.arange(n_p2)
    q0 = nwg - n_qkv
    for t in range(n_qkv):
        kind[q0 + t, 0], tile[q0 + t, 0] = GQ, t
    # self-attention heads: on the fc2-only workgroups [0, q0) first, then on the last ones
    # (QKV + cross out-proj + fc1: two idle levels after the attention for their refills) -- not
    # on fc2 + QKV workgroups, whose 5 slots and cross item leave no idle level for theirs
    opts = WDEC_ROLE_OPTS
    if opts.get("sat", "fc2") == "tail":
        sat = list(range(nwg - 1, nwg - 1 - H, -1))
    else:
        sat = list(range(min(H, q0))) + list(range(nwg - 1, nwg - 1 - max(0, H - q0), -1))
    R[sat, 20] = np.arange(H)
    R[:n_x, 21] = np.arange(n_x)
    R[:n_x, 22] = LX
    free = [(s, w) for s in range(1, 5) for w in range(nwg) if kind[w, s] < 0 and w >= n_d]
    free.sort()
    fi = 0
    for gm, n in ((GO, n_d), (GXQO, n_d), (GXO, n_d), (G1, n_ff), (GXQ, n_d)):
        for t in range(n):
            while fi < len(free) and (
                    sum(1 for s in range(5) if kind[free[fi][1], s] >= 0
                        and lvl_of[kind[free[fi][1], s]] == lvl_of[gm]) >= 2
                    or (gm == GXQ and (kind[free[fi][1], 0] != GQ or R[free[fi][1], 20] >= 0))):
                fi += 1
            if fi >= len(free):
                raise ValueError("wdec_roles: not enough free slots")
            s, w = free[fi]
            fi += 1
            kind[w, s], tile[w, s] = gm, t
    work = np.zeros(nwg, dtype=np.int64)
    for w in range(nwg):
        m = 0
        for s in range(5):
            if kind[w, s] >= 0:
                m |= 1 << lvl_of[kind[w, s]]
        if R[w, 20] >= 0:
            m |= 1 << LS
        if R[w, 21] >= 0:
            m |= 1 << LX
        work[w] = m
    # refill points: a slot may be refilled after ANY level its workgroup runs (after its use: the
    # next layer's tile; before it: this layer's).  The refill's bytes share the CU's in-order
    # memory queue with the next level's activation loads, so each slot goes to the level with the
    # longest run of idle levels behind it (measured: a 40 KB refill right before the next level's
    # X staging held that staging ~1.6 us), spreading slots over equally good points.  (The x part
    # of the cross query is off the critical path: it counts as no gap.)
    crit = [lv for lv in range(8) if lv != LXQX]
    for w in range(nwg):
        W = [lv for lv in crit if (work[w] >> lv) & 1]
        pos = {lv: crit.index(lv) for lv in W}
        gap = {lv: ((pos[W[(i + 1) % len(W)]] - pos[lv] - 1) % 7) + (7 if len(W) == 1 else 0) for i, lv in enumerate(W)}
        nxt = {lv: W[(i + 1) % len(W)] for i, lv in enumerate(W)}
        att_pen = {lv: (opts.get("att_pen", 0.0) if nxt[lv] in (LS, LX) else 0.0) for lv in W}
        if (work[w] >> LXQX) & 1:
            gap[LXQX] = -1
        load = {lv: 0 for lv in gap}
        if R[w, 21] >= 0:
            load[LX] += 96  # the cross K / V chunk (KB) issued after the cross-attention
        for s in range(5):
            k = kind[w, s]
            if k < 0:
                continue
            kb = 40
            # (a level right before this workgroup's next one is the last resort: its refill
            # holds that level's row loads -- measured 1.2 us late QKV on WGs 16..19)
            # (the x part of the cross query runs right after the QKV level: its slot is never
            # refilled there -- that would load THIS layer's tile behind every QKV refill)
            cand = [lv for lv in gap if not (lvl_of[k] == LXQX and lv < LXQX)]
            best = max(cand, key=lambda lv: (gap[lv] - load[lv] / 80.0 - (0.5 if gap[lv] == 0 else 0.0)
                                             - att_pen.get(lv, 0.0), lv == lvl_of[k]))
            rel[w, s] = best
            load[best] += kb
    R[:, 23] = work
    n_prod = [int(((work >> lvl) & 1).sum()) for lvl in range(8)]
    return R, n_prod


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2, dtype=torch.float32))
    t = torch.arange(length, dtype=torch.float32)[:, None] * inv[None, :]
    return torch.cat([torch.sin(t), torch.cos(t)], dim=1)


@dataclass
class EncLayer:
    ln1_w: torch.Tensor; ln1_b: torch.Tensor
    qkv: torch.Tensor; qkv_b: torch.Tensor      # [3d, d] natural order (q,k,v)
    o: torch.Tensor; o_b: torch.Tensor
    ln2_w: torch.Tensor; ln2_b: torch.Tensor
    fc1: torch.Tensor; fc1_b: torch.Tensor
    fc2: torch.Tensor; fc2_b: torch.Tensor


@dataclass
class DecLayer:
    ln1_w: torch.Tensor; ln1_b: torch.Tensor
    qkv: torch.Tensor; qkv_b: torch.Tensor      # permuted rows (skinny QKV epilogue layout)
    o: torch.Tensor; o_b: torch.Tensor
    lnx_w: torch.Tensor; lnx_b: torch.Tensor
    xq: torch.Tensor; xq_b: torch.Tensor
    xk: torch.Tensor; xv: torch.Tensor; xv_b: torch.Tensor
    xo: torch.Tensor; xo_b: torch.Tensor
    ln2_w: torch.Tensor; ln2_b: torch.Tensor
    fc1: torch.Tensor; fc1_b: torch.Tensor
    fc2: torch.Tensor; fc2_b: torch.Tensor
    # decode-path copies with the preceding LayerNorm folded in (ops.fold_layernorm):
    # (weight * gamma, bias + weight @ beta, row sums of the folded weight)
    f_qkv: Optional[tuple] = None
    f_xq: Optional[tuple] = None
    f_fc1: Optional[tuple] = None


class WhisperModel:
    def __init__(self, cfg: WhisperConfig, *, device="cpu", dtype=torch.bfloat16, seed: int = 0,
                 weights=None, tile_decoder: Optional[bool] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        d, H = cfg.d_model, cfg.n_heads
        self.H, self.hd = H, cfg.head_dim
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed * 7 + 11)
        std = cfg.init_std

        def rn(*shape, s=std):
            t = torch.empty(shape, device=self.device, dtype=torch.float32)
            t.normal_(0.0, s, generator=gen)
            return t.to(dtype)

        def ones(n):
            return torch.ones(n, device=self.device, dtype=dtype)

        def zeros(n):
            return torch.zeros(n, device=self.device, dtype=dtype)

        F = cfg.ffn
        # conv weights stored [Cout, 3*Cin] in (kk, ci) order for the implicit-GEMM kernel
        self.conv1_w, self.conv1_b = rn(d, 3 * cfg.n_mels), rn(d, s=0.01)
        self.conv2_w, self.conv2_b = rn(d, 3 * d), rn(d, s=0.01)
        self.pos_enc = sinusoids(cfg.n_audio_ctx, d).to(self.device, dtype)
        self.enc: List[EncLayer] = []
        for _ in range(cfg.n_enc_layers):
            self.enc.append(EncLayer(ones(d), zeros(d), rn(3 * d, d), rn(3 * d, s=0.01), rn(d, d), rn(d, s=0.01),
                                     ones(d), zeros(d), rn(F, d), rn(F, s=0.01), rn(d, F), rn(d, s=0.01)))
        self.enc_ln_w, self.enc_ln_b = ones(d), zeros(d)
        self.tok_emb = rn(cfg.vocab_size, d)
        self.pos_emb = rn(cfg.n_text_ctx, d, s=0.01)
        self.dec: List[DecLayer] = []
        for _ in range(cfg.n_dec_layers):
            qkv = rn(3 * d, d)
            qkv_b = rn(3 * d, s=0.01)
            qkv_b[d : 2 * d] = 0  # Whisper's key projection has no bias
            qkv_p = ops.permute_qkv_rows(qkv, 3 * H, self.hd)
            qkv_bp = ops.permute_qkv_rows(qkv_b[:, None], 3 * H, self.hd)[:, 0].contiguous()
            self.dec.append(DecLayer(ones(d), zeros(d), qkv_p, qkv_bp, rn(d, d), rn(d, s=0.01), ones(d), zeros(d),
                                     rn(d, d), rn(d, s=0.01), rn(d, d), rn(d, d), rn(d, s=0.01), rn(d, d),
                                     rn(d, s=0.01), ones(d), zeros(d), rn(F, d), rn(F, s=0.01), rn(d, F),
                                     rn(d, s=0.01)))
        self.dec_ln_w, self.dec_ln_b = ones(d), zeros(d)
        if weights is not None:
            self._load(weights)
        # tied LM head padded to a multiple of 16 rows (MFMA column tile); padded ids are masked
        vp = (cfg.vocab_size + 15) // 16 * 16
        self.vocab_padded = vp
        self.lm_head = torch.zeros(vp, d, device=self.device, dtype=dtype)
        self.lm_head[: cfg.vocab_size] = self.tok_emb
        self.fold_decoder_norms()
        # front-end constants
        self.window = torch.hann_window(400, periodic=True, device=self.device)
        self.mel_fb = ref.mel_filterbank(n_mels=cfg.n_mels).to(self.device)
        # conv stem on the GEMM path: mel channels zero-padded to a 128 multiple (3*C % 128 == 0),
        # zero-padded row buffers per batch size (conv padding = the buffers' pad rows)
        self.mel_ch = ops.conv_channels(cfg.n_mels)
        self.conv1_wp = ops.pad_conv_weight(self.conv1_w, self.mel_ch)
        self._stem: dict = {}
        # GPU: the encoder-side GEMM weights (conv stem, encoder projections: M = 1500 x sessions
        # rows on the tiled MFMA GEMM) are kept ONLY in the pre-tiled layout
        if self.device.type == "cuda":
            self.conv1_wp = ops.TiledWeight(self.conv1_wp)
            self.conv2_wt = ops.TiledWeight(self.conv2_w)
            for L in self.enc:
                L.qkv, L.o, L.fc1, L.fc2 = (ops.TiledWeight(t) for t in (L.qkv, L.o, L.fc1, L.fc2))
        else:
            self.conv2_wt = self.conv2_w
        # decode-step weights in the pre-tiled layout when they stream from HBM (more than the
        # 256 MB Infinity Cache per token: large-v3's 1.5 GB); cache-resident small models keep the
        # row-major layout for the one-tile kernel.  Measured per layer at M = 1 (tools/
        # bench_whisper_decode.py, K = 1280): QKV 8.1 -> 6.5 us, fc1 11.2 -> 8.3, fc2 12.3 -> 9.6,
        # LM head 43 -> 28 (tiled + the 4-wave K split).
        if tile_decoder is None:
            tile_decoder = self.decoder_bytes() > (256 << 20)
        self.dec_tiled = bool(tile_decoder) and self.device.type == "cuda"
        if self.dec_tiled:
            self._tile_decoder()

    def _load(self, w) -> None:
        """HF WhisperForConditionalGeneration names (safetensors, runtime.weights.LazySafetensors)."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        d, H = cfg.d_model, self.H
        g = lambda n: w[n].to(device=dev, dtype=dt)  # noqa: E731

        def conv(n):  # [Cout, Cin, 3] -> [Cout, 3*Cin] in (kk, ci) order
            t = g(n)
            return t.permute(0, 2, 1).reshape(t.shape[0], -1).contiguous()

        def qkv(pre):
            wq, wk, wv = g(pre + "q_proj.weight"), g(pre + "k_proj.weight"), g(pre + "v_proj.weight")
            bq, bv = g(pre + "q_proj.bias"), g(pre + "v_proj.bias")
            return torch.cat([wq, wk, wv]), torch.cat([bq, torch.zeros_like(bq), bv])

        e, dd = "model.encoder.", "model.decoder."
        self.conv1_w, self.conv1_b = conv(e + "conv1.weight"), g(e + "conv1.bias")
        self.conv2_w, self.conv2_b = conv(e + "conv2.weight"), g(e + "conv2.bias")
        if e + "embed_positions.weight" in w:
            self.pos_enc = g(e + "embed_positions.weight")
        self.enc = []
        for i in range(cfg.n_enc_layers):
            p = f"{e}layers.{i}."
            wqkv, bqkv = qkv(p + "self_attn.")
            self.enc.append(EncLayer(
                g(p + "self_attn_layer_norm.weight"), g(p + "self_attn_layer_norm.bias"), wqkv, bqkv,
                g(p + "self_attn.out_proj.weight"), g(p + "self_attn.out_proj.bias"), g(p + "final_layer_norm.weight"),
                g(p + "final_layer_norm.bias"), g(p + "fc1.weight"), g(p + "fc1.bias"), g(p + "fc2.weight"),
                g(p + "fc2.bias")))
        self.enc_ln_w, self.enc_ln_b = g(e + "layer_norm.weight"), g(e + "layer_norm.bias")
        self.tok_emb = g(dd + "embed_tokens.weight")
        self.pos_emb = g(dd + "embed_positions.weight")
        self.dec = []
        for i in range(cfg.n_dec_layers):
            p = f"{dd}layers.{i}."
            wqkv, bqkv = qkv(p + "self_attn.")
            x = p + "encoder_attn."
            self.dec.append(DecLayer(
                g(p + "self_attn_layer_norm.weight"), g(p + "self_attn_layer_norm.bias"),
                ops.permute_qkv_rows(wqkv, 3 * H, self.hd),
                ops.permute_qkv_rows(bqkv[:, None], 3 * H, self.hd)[:, 0].contiguous(),
                g(p + "self_attn.out_proj.weight"), g(p + "self_attn.out_proj.bias"),
                g(p + "encoder_attn_layer_norm.weight"), g(p + "encoder_attn_layer_norm.bias"),
                g(x + "q_proj.weight"), g(x + "q_proj.bias"), g(x + "k_proj.weight"), g(x + "v_proj.weight"),
                g(x + "v_proj.bias"), g(x + "out_proj.weight"), g(x + "out_proj.bias"),
                g(p + "final_layer_norm.weight"), g(p + "final_layer_norm.bias"), g(p + "fc1.weight"),
                g(p + "fc1.bias"), g(p + "fc2.weight"), g(p + "fc2.bias")))
        self.dec_ln_w, self.dec_ln_b = g(dd + "layer_norm.weight"), g(dd + "layer_norm.bias")

    def fold_decoder_norms(self) -> None:
        """Fold every decoder LayerNorm into the projection that consumes it (self-attention QKV,
        cross-attention query, fc1, LM head): a decode step then has no LayerNorm launches; the
        streaming GEMM computes each row's mean / rstd from the activation rows it stages anyway
        (8 instead of 11 kernels per layer).  The unfolded weights stay for the encoder-side
        cross K/V projections and checkpoint round trips."""
        fold = ops.fold_layernorm
        for L in self.dec:
            L.f_qkv = fold(L.qkv, L.qkv_b, L.ln1_w, L.ln1_b)
            L.f_xq = fold(L.xq, L.xq_b, L.lnx_w, L.lnx_b)
            L.f_fc1 = fold(L.fc1, L.fc1_b, L.ln2_w, L.ln2_b)
        self.f_lm = fold(self.lm_head, None, self.dec_ln_w, self.dec_ln_b)

    def decoder_bytes(self) -> int:
        """Weight bytes one decode step streams (decoder projections + LM head)."""
        n = sum(t.numel() for L in self.dec for t in (L.qkv, L.o, L.xq, L.xo, L.fc1, L.fc2))
        return (n + self.lm_head.numel()) * self.lm_head.element_size()

    def _tile_decoder(self) -> None:
        """Decode-path projections -> TiledWeight (the folded QKV / cross-query / fc1 / LM head
        copies and the out-proj / fc2 weights); the unfolded copies stay row-major for the
        prompt-sized paths and checkpoint round trips."""
        T = ops.TiledWeight
        for L in self.dec:
            L.o, L.xo, L.fc2 = T(L.o), T(L.xo), T(L.fc2)
            L.f_qkv, L.f_xq, L.f_fc1 = ((T(w), b, c) for (w, b, c) in (L.f_qkv, L.f_xq, L.f_fc1))
        w, b, c = self.f_lm
        self.f_lm = (T(w), b, c)

    # ------------------------------------------------------------------ encoder
    def log_mel(self, audio: torch.Tensor, n_frames: int = 3000, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """audio: f32 samples (<= 30 s). Returns [n_frames, n_mels] bf16 (channels-last); ``out``: a
        [n_frames, n_mels] view to write (e.g. a row of mel_batch(), whose rows are mel_ch apart)."""
        pad = torch.zeros(n_frames * 160, dtype=torch.float32, device=self.device)
        n = min(audio.numel(), pad.numel())
        pad[:n] = audio[:n]
        if out is None:
            out = torch.empty(n_frames, self.cfg.n_mels, dtype=self.dtype, device=self.device)
        return ops.log_mel(pad, n_frames=n_frames, window=self.window, mel_fb=self.mel_fb,
                           out=out)

    def _stem_buffers(self, B: int, T: int):
        """(mel view [B, T, mel_ch], conv1-output view [B, T, d]) of zero-padded row buffers, cached
        per (B, T); their pad rows / channels are never written, so they stay zero."""
        key = (B, T)
        if key not in self._stem:
            _, mv = ops.padded_rows(B, T, self.mel_ch, dtype=self.dtype, device=self.device)
            _, cv = ops.padded_rows(B, T, self.cfg.d_model, dtype=self.dtype, device=self.device)
            self._stem[key] = (mv, cv)
        return self._stem[key]

    def mel_batch(self, audios: Sequence[torch.Tensor], n_frames: int = 3000) -> torch.Tensor:
        """Log-mel of every utterance straight into the conv stem's padded input buffer; returns
        the [B, n_frames, mel_ch] view encode() takes without a copy."""
        mv, _ = self._stem_buffers(len(audios), n_frames)
        for i, a in enumerate(audios):
            self.log_mel(a, n_frames, out=mv[i, :, : self.cfg.n_mels])
        return mv

    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        """mel [B, 3000, n_mels] (or mel_batch()'s [B, 3000, mel_ch] view) -> encoder states [B, 1500, d]."""
        cfg = self.cfg
        B, T = mel.shape[0], mel.shape[1]
        mv, cv = self._stem_buffers(B, T)
        if mel.data_ptr() != mv.data_ptr() or mel.shape != mv.shape:
            mv[:, :, : cfg.n_mels] = mel[:, :, : cfg.n_mels]
        x = ops.conv1d_gelu(mv, self.conv1_wp, self.conv1_b, stride=1, out=cv, padded=True)
        x = ops.conv1d_gelu(x, self.conv2_wt, self.conv2_b, stride=2, pos=self.pos_enc, padded=True)
        T, d = x.shape[1], x.shape[2]
        x = x.reshape(B * T, d)
        table = torch.arange(B, dtype=torch.int32, device=self.device)[:, None]
        for L in self.enc:
            h = ops.layernorm(x, L.ln1_w, L.ln1_b, eps=cfg.ln_eps)
            qkv = ops.linear(h, L.qkv, L.qkv_b).view(B, T, 3, self.H, self.hd)
            # strided q / k / v views: the flash kernel addresses rows by stride (no copies)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
            att = ops.flash_attention(q, ops.KVLayout.contiguous(k, v, table), Sk=T, n_kv_heads=self.H, causal=False,
                                      scale=self.hd ** -0.5)
            x = ops.linear(att.view(B * T, d), L.o, L.o_b, residual=x)
            h = ops.layernorm(x, L.ln2_w, L.ln2_b, eps=cfg.ln_eps)
            h = ops.linear(h, L.fc1, L.fc1_b, act="gelu")
            x = ops.linear(h, L.fc2, L.fc2_b, residual=x)
        x = ops.layernorm(x, self.enc_ln_w, self.enc_ln_b, eps=cfg.ln_eps)
        return x.view(B, T, d)

    def cross_kv(self, enc: torch.Tensor, out=None):
        """Per decoder layer cross-attention K/V [B, T, H, hd] (computed once per window).
        out: per layer (k, v) contiguous [B, T, H, hd] destinations (e.g. a run of the decode
        buffers' session slots) the projections write straight into -- no copies."""
        B, T, d = enc.shape
        x = enc.reshape(B * T, d)
        res = []
        for li, L in enumerate(self.dec):
            ko, vo = (None, None) if out is None else (out[li][0].view(B * T, d), out[li][1].view(B * T, d))
            k = ops.linear(x, L.xk, out=ko).view(B, T, self.H, self.hd)
            v = ops.linear(x, L.xv, L.xv_b, out=vo).view(B, T, self.H, self.hd)
            res.append((k, v))
        return res

    # ------------------------------------------------------------------ decoder step
    # ---- chained decode launches (skinny_stream.hip chain_kernel SEQ 2 / SEQ 1; M <= 4 rows).
    # Opt-in (VWA_CHAIN_ASR=1): measured (tools/asr_timing.py, 1 row, 40 tokens) 2.32 vs 2.26 ms
    # per token for whisper-large-v3 and 260 vs 244 us for whisper-tiny -- the decoder's
    # phases are 0.3-13 MB each, so every phase is latency-bound and a grid barrier (~4-5 us,
    # arrival spread + two-level atomics in uncached memory) costs what a kernel boundary does.
    def _chain_ok(self, M: int) -> bool:
        return (M <= 4 and self.device.type == "cuda" and self.dtype == torch.bfloat16
                and not getattr(self, "_chain_disabled", False) and ops.env_flag("VWA_CHAIN_ASR")
                and ops.native_available() and all(hasattr(L, "f_qkv") for L in self.dec))

    def disable_chain(self) -> None:
        self._chain_disabled = True
        self._wdec_disabled = True  # (a timed-out persistent launch: its counters are out of step)
        self.reset_chains()

    def reset_chains(self) -> None:
        """Drop every cached chain descriptor (they embed raw device pointers of the buffers)."""
        self._chains = weakref.WeakKeyDictionary()

    def chain_descs(self):
        return [v for d in getattr(self, "_chains", {}).values() for v in d.values()]

    def chain_error_word(self):
        return ops.chain_error_word(getattr(self, "_chain_bar", None))

    def chain_error(self) -> bool:
        w = self.chain_error_word()
        if w is not None and int(w.item()) != 0:
            return True
        # every persistent-decoder state (one per runner's buffers) has its own error word
        for st in list(getattr(self, "_wdec", {}).values()) if getattr(self, "_wdec", None) else []:
            if st is not None and int(st["cnt"].view(torch.int64)[1024].item()) != 0:
                return True
        return False

    def _chain_descs(self, bufs, M: int, li: int):
        """Layer li's two chained launches for these buffers, built on first use:
        middle = self-attn out-proj + residual -> LN cross-attn query (store to bufs.q);
        tail = cross-attn out-proj + residual -> LN fc1 + GELU -> fc2 + residual [-> next layer's
        LN self-attn QKV + self-KV write].  Each entry (descriptor, n_phases, lds) or None."""
        # keyed on the buffers object itself (weakly): the descriptors embed its raw pointers
        if not isinstance(getattr(self, "_chains", None), weakref.WeakKeyDictionary):
            self.reset_chains()
        cache = self._chains.setdefault(bufs, {})
        key = (M, li)
        if key in cache:
            return cache[key]
        if getattr(self, "_chain_bar", None) is None:
            self._chain_bar, self._chain_bar_mode, self._chain_work = ops.chain_buffers(self.device)
        L, eps = self.dec[li], self.cfg.ln_eps
        x, att, q, f = bufs.hidden[:M], bufs.att[:M], bufs.q[:M], bufs.f[:M]
        common = dict(eps=eps, n_heads=self.H, head_dim=self.hd, bar=self._chain_bar, work=self._chain_work,
                      bar_mode=self._chain_bar_mode)
        (wq, bq, cq), (w1, b1, c1) = L.f_xq, L.f_fc1
        common["w_tiled"] = self.dec_tiled
        wt = lambda t: t.t if isinstance(t, ops.TiledWeight) else t  # noqa: E731
        mid = ops.ext().chain_make_seq(2, [att, x], [wt(L.o), wt(wq)], [L.o_b, bq], [None, cq], [x, q], [1, 0],
                                       positions=None, slots=None, k_cache=None, v_cache=None, **common)
        X, W, B, C, Y, E = ([att, x, f], [wt(L.xo), wt(w1), wt(L.fc2)], [L.xo_b, b1, L.fc2_b], [None, c1, None],
                            [x, f, x], [1, 3, 1])
        nxt = li + 1 < len(self.dec)
        if nxt:
            wn, bn, cn = self.dec[li + 1].f_qkv
            X, W, B, C, Y, E = X + [x], W + [wt(wn)], B + [bn], C + [cn], Y + [q], E + [4]
        tail = ops.ext().chain_make_seq(1, X, W, B, C, Y, E, positions=bufs.positions if nxt else None,
                                        slots=bufs.slots if nxt else None,
                                        k_cache=bufs.k_cache[li + 1] if nxt else None,
                                        v_cache=bufs.v_cache[li + 1] if nxt else None, **common)
        cache[key] = ((mid[0], 2, mid[1]) if mid[0].numel() else None,
                      (tail[0], len(E), tail[1]) if tail[0].numel() else None)
        return cache[key]

    # ---- persistent decoder (csrc/kernels/whisper_dec.hip wdec_kernel): a one-row step of the
    # Whisper model (tiny .. large: d a multiple of 128 up to 1536, ffn 4 d, head_dim 64) as ONE launch
    # over every decoder layer; each workgroup's weight tiles stay in its registers a layer ahead.
    def _wdec_ok(self, M: int) -> bool:
        cfg = self.cfg
        return (M == 1 and self.device.type == "cuda" and cfg.d_model % 128 == 0 and cfg.d_model <= 1536
                and cfg.ffn == 4 * cfg.d_model and self.hd == 64 and cfg.n_dec_layers >= 2
                and not getattr(self, "_wdec_disabled", False) and ops.env_flag("VWA_ASR_PERSIST")
                and ops.native_available())

    def _wdec_state(self, bufs):
        """(layer descriptors, roles, n_prod, counters, partials, grid) for these buffers, built once
        (the descriptors embed raw pointers of the buffers and the weights)."""
        if not isinstance(getattr(self, "_wdec", None), weakref.WeakKeyDictionary):
            self._wdec = weakref.WeakKeyDictionary()
        st = self._wdec.get(bufs)
        if st is not None:
            return st
        cfg = self.cfg
        E = ops.ext()
        grid = int(E.device_cus(bufs.hidden))  # one workgroup per CU, all resident
        # cross-attention key chunks per head: 4 (8 measured: the cross level 0.3 us shorter, the
        # merge in the cross out-projection's staging 3.2 us longer, profiles/r6_wdec_nch_ab.jsonl)
        nch = 4
        try:
            roles, n_prod = wdec_roles(grid, cfg.d_model, self.H, cfg.ffn, nch)
        except ValueError:  # (a partitioned device with too few CUs for the tiles: per-kernel launches)
            self._wdec_disabled = True
            return None
        # the kernel reads pre-tiled weights: a model whose decoder stays row-major (small models:
        # _tile_decoder only above 256 MB) gets tiled copies for it here, kept alive in the state
        keep = []

        def wt(t):
            if isinstance(t, ops.TiledWeight):
                return t.t
            keep.append(ops.tile_weight(t))
            return keep[-1]

        flat = []
        for li, L in enumerate(self.dec):
            (wq, bq, cq), (wx, bx, cx), (w1, b1, c1) = L.f_qkv, L.f_xq, L.f_fc1
            wxo, bxo = self._wdec_xq_o(L)
            flat += [wt(wq), bq, cq, wt(L.o), L.o_b, None, wt(wx), bx, cx, wt(L.xo), L.xo_b, None,
                     wt(w1), b1, c1, wt(L.fc2), L.fc2_b, None, wt(wxo), bxo, None,
                     bufs.k_cache[li], bufs.v_cache[li], bufs.cross[li][0], bufs.cross[li][1]]
        layers = E.wdec_layers(flat, len(self.dec), bufs.hidden)
        cnt = E.alloc_uncached_i32(4096, bufs.hidden)  # level counters [8][8] x 128 B + error word
        xpart = torch.zeros(self.H * nch * 68 + 3 * cfg.d_model, dtype=torch.float32, device=self.device)
        T = bufs.cross[0][0].shape[1]
        w_lm = wt(self.f_lm[0])
        st = dict(layers=layers, roles=torch.from_numpy(roles).to(self.device), n_prod=n_prod, cnt=cnt, xpart=xpart,
                  keep=keep, lm_w=w_lm,
                  ints=[len(self.dec), cfg.d_model, self.H, cfg.ffn, T, bufs.k_cache.shape[3],
                        bufs.block_table.shape[1], nch, -(-T // nch), bufs.cross[0][0].shape[0], grid])
        self._wdec[bufs] = st
        return st

    def _wdec_xq_o(self, L):
        """The cross query's att part (whisper_dec.hip level OXQ): Wg Wo (pre-tiled bf16) and
        Wg bo, Wg = the LayerNorm-folded cross-query weight -- x1 Wg^T = x Wg^T + att (Wg Wo)^T +
        Wg bo.  Built once per layer (3.3 MB each), in f32 then rounded."""
        if getattr(L, "_xq_o", None) is None:
            dense = lambda t: (t.dense() if isinstance(t, ops.TiledWeight) else t).float()  # noqa: E731
            wg, wo = dense(L.f_xq[0]), dense(L.o)
            w = (wg @ wo).to(torch.bfloat16)
            b = (wg @ L.o_b.float()).to(torch.bfloat16) if L.o_b is not None else None
            L._xq_o = (ops.TiledWeight(w), b)
        return L._xq_o

    def wdec_error_word(self, bufs=None):
        """The error word of the persistent decoder's state for ``bufs`` (default: the first one)."""
        d = getattr(self, "_wdec", None)
        if not d:
            return None
        st = d.get(bufs) if bufs is not None else next(iter(d.values()), None)
        return None if st is None else st["cnt"].view(torch.int64)[1024:1025]

    def _wdec_emb_ok(self, bufs) -> bool:
        """The launch builds the step's embedding row itself (layer 0): the position table covers
        every KV position of a session."""
        return self.pos_emb.shape[0] >= bufs.block_table.shape[1] * bufs.k_cache.shape[3]

    def _wdec_step(self, bufs, smp: Optional[list] = None, base_block: int = 0) -> torch.Tensor:
        """Every decoder layer of a one-row step and the LM head (folded final LayerNorm) in ONE
        launch -- with the embedding of bufs.tokens[0] / bufs.positions[0] built by layer 0
        (_wdec_emb_ok; else it must be in bufs.hidden[0]) and, with ``smp`` (the device loop,
        asr/engine.py), the greedy masked argmax + the loop advance as its last step.  Returns the
        f32 logits row [1, V]."""
        st = self._wdec_state(bufs)
        _, b, c = self.f_lm
        lm = [st["lm_w"], b if b is not None else st.setdefault("no_bias", torch.empty(0, dtype=torch.bfloat16,
                                                                                  device=self.device)),
              c, bufs.logits[0]]
        emb = [self.tok_emb, self.pos_emb, bufs.tokens, bufs.positions] if self._wdec_emb_ok(bufs) else None
        ops.ext().wdec_run(st["layers"], st["roles"],
                           [bufs.hidden, bufs.h, bufs.q, bufs.att, bufs.f, st["xpart"], bufs.seq_ids, bufs.ctx_lens,
                            bufs.slots, bufs.block_table, bufs.cross_table, st["cnt"]],
                           st["ints"], self.cfg.ln_eps, self.hd ** -0.5, st["n_prod"], st.get("ts"),
                           int(st.get("opt", ops.env_int("VWA_WDEC_OPT"))), lm, emb, smp, base_block)
        return bufs.logits[:1]

    def wdec_loop_step(self, bufs, mask: torch.Tensor, tok: torch.Tensor, step: torch.Tensor, out: torch.Tensor,
                       cnt: torch.Tensor, base_block: int) -> bool:
        """One device-loop decode step (asr/engine.py _loop_step) as ONE launch: layers, LM head,
        greedy masked argmax, advance.  False when the persistent decoder does not take this step
        (the caller runs the separate launches)."""
        if not (self._wdec_ok(1) and self._wdec_emb_ok(bufs) and self._wdec_state(bufs) is not None):
            return False
        st = self._wdec_state(bufs)
        part = st.get("smp_part")
        if part is None:
            part = st["smp_part"] = torch.zeros(2 * st["ints"][10], dtype=torch.float32, device=self.device)
        self._wdec_step(bufs, [mask.view(torch.int32).reshape(-1), tok, step, part, out, cnt, bufs.tokens,
                               bufs.positions, bufs.ctx_lens, bufs.slots], base_block)
        return True

    def decode_step(self, bufs, M: int) -> torch.Tensor:
        """M token rows (bufs: tokens/positions/slots/seq_ids/ctx_lens + self cache + cross K/V).
        Returns f32 logits [M, vocab].  Eight launches per layer; with VWA_CHAIN_ASR=1 and M <= 4
        four (self-attention, chained out-proj -> cross query, cross-attention, chained out-proj
        -> MLP -> next QKV); one row of whisper-large with VWA_ASR_PERSIST: ONE launch for every
        layer (whisper_dec.hip)."""
        cfg = self.cfg
        d = cfg.d_model
        x = bufs.hidden[:M]
        eps = cfg.ln_eps
        if self._wdec_ok(M) and self._wdec_state(bufs) is not None:  # (embedding, layers, LM head: one launch)
            if not self._wdec_emb_ok(bufs):
                ops.embedding(bufs.tokens, self.tok_emb, pos_table=self.pos_emb, positions=bufs.positions, out=x,
                              rows=M)
            return self._wdec_step(bufs)
        ops.embedding(bufs.tokens, self.tok_emb, pos_table=self.pos_emb, positions=bufs.positions, out=x, rows=M)
        chain = self._chain_ok(M)
        qkv_done = False
        for li, L in enumerate(self.dec):
            mid = tail = None
            if chain:
                mid, tail = self._chain_descs(bufs, M, li)
                if mid is None or tail is None:
                    chain = False  # shapes the chain cannot take: per-kernel path
            if qkv_done:
                q = bufs.q[:M]  # written by the previous layer's chained launch
            else:
                w, b, c = L.f_qkv  # self_attn_layer_norm folded in
                q = ops.qkv_rope_write(x, w, b, fuse_rms=False, eps=eps, n_q_heads=self.H, n_kv_heads=self.H,
                                       head_dim=self.hd, rope=None, positions=bufs.positions, slots=bufs.slots,
                                       q_out=bufs.q, k_cache=bufs.k_cache[li], v_cache=bufs.v_cache[li], ln_c=c)
            att = ops.decode_attention(q, ops.KVLayout.paged(bufs.k_cache[li], bufs.v_cache[li], bufs.block_table),
                                       bufs.ctx_lens, bufs.seq_ids, n_q_heads=self.H, n_kv_heads=self.H,
                                       head_dim=self.hd, scale=self.hd ** -0.5, max_ctx=bufs.max_ctx,
                                       out=bufs.att[:M], part_o=bufs.part_o, part_ml=bufs.part_ml,
                                       counters=bufs.attn_cnt)
            if chain:
                ops.ext().chain_run(mid[0], mid[1], mid[2], x, 0, 2)
                xq = bufs.q[:M]
            else:
                ops.linear(att, L.o, L.o_b, out=x, residual=x)
                w, b, c = L.f_xq  # encoder_attn_layer_norm folded in
                xq = ops.linear(x, w, b, out=bufs.q[:M], eps=eps, ln_c=c)
            ck, cv = bufs.cross[li]
            att = ops.decode_attention(xq, ops.KVLayout.contiguous(ck, cv, bufs.cross_table), bufs.cross_lens,
                                       bufs.seq_ids, n_q_heads=self.H, n_kv_heads=self.H, head_dim=self.hd,
                                       scale=self.hd ** -0.5, max_ctx=ck.shape[1], out=bufs.att[:M],
                                       part_o=bufs.part_o, part_ml=bufs.part_ml,
                                       counters=bufs.attn_cnt)
            if chain:
                ops.ext().chain_run(tail[0], tail[1], tail[2], x, 0, 1)
                qkv_done = tail[1] == 4
                continue
            qkv_done = False
            ops.linear(att, L.xo, L.xo_b, out=x, residual=x)
            w, b, c = L.f_fc1  # final_layer_norm folded in
            f = ops.linear(x, w, b, act="gelu", out=bufs.f[:M], eps=eps, ln_c=c)
            ops.linear(f, L.fc2, L.fc2_b, out=x, residual=x)
        w, b, c = self.f_lm  # decoder layer_norm folded into the tied LM head
        return ops.linear(x, w, b, out=bufs.logits[:M], eps=eps, ln_c=c)
