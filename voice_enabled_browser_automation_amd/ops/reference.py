"""Plain-PyTorch (f32 math) reference implementations of every kernel in csrc/kernels.

Used on CPU tensors (tests, the CPU config) and as the numerics oracle for the HIP kernels.
Semantics (layouts, permutations, epilogues) match the kernels exactly.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F


def _rms_scale(xf: torch.Tensor, eps: float) -> torch.Tensor:
    return torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)


def linear(x, w, bias=None, *, out, residual=None, act="none", fuse_rms=False, eps=1e-5):
    xf = x.float()
    if fuse_rms:
        xf = xf * _rms_scale(xf, eps)
    y = xf @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    if act == "gelu":
        y = F.gelu(y)
    if residual is not None:
        y = y + residual.float()
    out.copy_(y.to(out.dtype))
    return out


def linear_swiglu(x, w_gu, *, fuse_rms=False, eps=1e-5, out):
    xf = x.float()
    if fuse_rms:
        xf = xf * _rms_scale(xf, eps)
    gu = xf @ w_gu.float().t()
    M, F2 = gu.shape
    t = gu.view(M, F2 // 32, 2, 16)
    h = F.silu(t[:, :, 0, :]) * t[:, :, 1, :]
    out.copy_(h.reshape(M, F2 // 2).to(out.dtype))
    return out


def _apply_rope(x: torch.Tensor, positions: torch.Tensor, rope: torch.Tensor) -> torch.Tensor:
    # x [M, H, D] natural layout; rotate-half convention
    D = x.shape[-1]
    half = D // 2
    cs = rope[positions.long()]  # [M, half, 2]
    c = cs[..., 0][:, None, :]
    s = cs[..., 1][:, None, :]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def write_kv(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor):
    bs = k_cache.shape[2]
    for m in range(k.shape[0]):
        s = int(slots[m])
        if s < 0:
            continue
        b, o = divmod(s, bs)
        k_cache[b, :, o, :] = k[m].to(k_cache.dtype)
        v_cache[b, :, o, :] = v[m].to(v_cache.dtype)


def qkv_rope_write(x, w_qkv, bias, *, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, rope, positions, slots, q_out,
                   k_cache, v_cache):
    from . import unpermute_qkv_cols

    M = x.shape[0]
    xf = x.float()
    if fuse_rms:
        xf = xf * _rms_scale(xf, eps)
    y = xf @ w_qkv.float().t()
    if bias is not None:
        y = y + bias.float()
    H = n_q_heads + 2 * n_kv_heads
    y = unpermute_qkv_cols(y, H, head_dim).view(M, H, head_dim)
    q, k, v = y[:, :n_q_heads], y[:, n_q_heads : n_q_heads + n_kv_heads], y[:, n_q_heads + n_kv_heads :]
    if rope is not None:
        q = _apply_rope(q, positions[:M], rope)
        k = _apply_rope(k, positions[:M], rope)
    # kernels round to bf16 before storing; mimic
    q_out[:M] = q.reshape(M, -1).to(q_out.dtype)
    write_kv(k, v, slots[:M], k_cache, v_cache)


def rmsnorm(x, w, *, eps=1e-5, residual=None, residual_out=None, out):
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
        residual_out.copy_(xf.to(residual_out.dtype))
    y = xf * _rms_scale(xf, eps)
    if w is not None:
        y = y * w.float()
    out.copy_(y.to(out.dtype))
    return out


def layernorm(x, w, b, *, eps=1e-5, residual=None, residual_out=None, out):
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
        residual_out.copy_(xf.to(residual_out.dtype))
    y = F.layer_norm(xf, (xf.shape[-1],), w.float(), b.float(), eps)
    out.copy_(y.to(out.dtype))
    return out


def embedding(ids, table, *, pos_table=None, positions=None, vocab_start=0, out):
    n = out.shape[0]
    idl = ids[:n].long() - vocab_start
    valid = (idl >= 0) & (idl < table.shape[0])
    e = table[idl.clamp(0, table.shape[0] - 1)].float() * valid[:, None].float()
    if pos_table is not None:
        e = e + pos_table[positions[:n].long()].float()
    out.copy_(e.to(out.dtype))
    return out


def _flat(x):
    """The whole storage of x as a 1-D view (strided views: offsets are relative to x's first element)."""
    n_el = x.untyped_storage().nbytes() // x.element_size()
    return x.as_strided((n_el,), (1,), 0)[x.storage_offset():]


def _gather_kv_heads(kv, seq: int, n: int, heads: int):
    """K, V [heads, n, D] (f32) for tokens 0..n-1 of table row `seq`, every kv head at once: the
    cache storage viewed as [blocks, heads, block_size, D] (the layout's strides), the sequence's
    blocks picked with one index_select."""
    bs = kv.block_size
    D = kv.k.shape[-1]
    nb = (n + bs - 1) // bs
    blk = kv.table[seq][:nb].long()

    def g(x):
        n_el = x.untyped_storage().nbytes() // x.element_size() - x.storage_offset()
        nblocks = (n_el - (heads - 1) * kv.sh - (bs - 1) * kv.st - D) // kv.sb + 1
        v = x.as_strided((nblocks, heads, bs, D), (kv.sb, kv.sh, kv.st, 1), x.storage_offset())
        return v.index_select(0, blk).permute(1, 0, 2, 3).reshape(heads, nb * bs, D)[:, :n].float()

    return g(kv.k), g(kv.v)


def decode_attention(q, kv, ctx_lens, seq_ids, *, n_q_heads, n_kv_heads, head_dim, scale, out):
    """Per row: softmax(q K^T * scale) V over the row's first ctx_len cached tokens, every head of
    the row in one batched product (GQA: G query heads per kv head).  Rows of one sequence share
    one gather of its K/V (the longest context among them)."""
    rows = q.shape[0]
    G = n_q_heads // n_kv_heads
    ctx = [int(c) for c in ctx_lens[:rows]]
    sids = [int(s) for s in seq_ids[:rows]]
    cache = {}
    for r in range(rows):
        n, seq = ctx[r], sids[r]
        if n == 0:
            out[r, : n_q_heads * head_dim] = 0
            continue
        if seq not in cache:
            nmax = max(c for c, s in zip(ctx, sids) if s == seq)
            cache[seq] = _gather_kv_heads(kv, seq, nmax, n_kv_heads)
        K, V = cache[seq]
        K, V = K[:, :n], V[:, :n]
        qv = q[r, : n_q_heads * head_dim].float().view(n_kv_heads, G, head_dim)
        p = torch.softmax(torch.einsum("hgd,hnd->hgn", qv, K) * scale, dim=-1)
        o = torch.einsum("hgn,hnd->hgd", p, V)
        out[r, : n_q_heads * head_dim] = o.reshape(-1).to(out.dtype)
    return out


def flash_attention(q, kv, *, Sk, n_kv_heads, causal, scale, q_offset=0, out, k_lens=None, q_offsets=None):
    B, Sq, Hq, D = q.shape
    G = Hq // n_kv_heads
    for b in range(B):
        sk = int(k_lens[b]) if k_lens is not None else Sk
        qo = int(q_offsets[b]) if q_offsets is not None else q_offset
        K, V = _gather_kv_heads(kv, b, sk, n_kv_heads)  # [Hkv, sk, D]
        qq = q[b].float().view(Sq, n_kv_heads, G, D)
        s = torch.einsum("qhgd,hkd->hgqk", qq, K) * scale
        if causal:
            qi = torch.arange(Sq)[:, None] + qo
            kj = torch.arange(sk)[None, :]
            s = s.masked_fill(kj > qi, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgqk,hkd->qhgd", p, V)
        out[b] = o.reshape(Sq, Hq, D).to(out.dtype)
    return out


def _splitmix64(x: int) -> int:
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


def gumbel_keys(logits_row: torch.Tensor, T: float, seed: int, step: int, row: int, v_offset: int = 0) -> torch.Tensor:
    """Exact replica of the kernel's counter-based Gumbel noise (vectorised); column j is global
    token id v_offset + j (a vocab shard under tensor parallelism)."""
    m = (1 << 64) - 1
    base = _splitmix64((seed & m) ^ _splitmix64((step * 0x100000001B3 + row) & m))
    V = logits_row.shape[0]
    v = torch.arange(v_offset, v_offset + V, dtype=torch.int64)
    # vectorised splitmix64 on uint64 emulated with python ints is slow; use numpy uint64
    import numpy as np

    x = (np.uint64(base) ^ v.numpy().astype(np.uint64))
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    u = ((x >> np.uint64(41)).astype(np.float32) + np.float32(0.5)) * np.float32(1.0 / 8388608.0)
    g = -np.log(-np.log(u))
    return logits_row.float() / T + torch.from_numpy(g.astype(np.float32))


def sample_partial(logits, *, mask, temperature, seed, step, v_offset=0):
    """Per-row best (key, global token id) over a logits shard whose column j is token
    v_offset + j: the kernel's partial stage (no step advance).  (-inf, -1) for an empty row."""
    rows, V = logits.shape
    sd = int(seed.reshape(-1)[0]) & ((1 << 64) - 1)
    st = int(step.reshape(-1)[0])
    vals = torch.full((rows,), float("-inf"), dtype=torch.float32)
    idx = torch.full((rows,), -1, dtype=torch.int64)
    lg = logits.detach().float().cpu()
    for r in range(rows):
        T = float(temperature[r]) if temperature is not None else 0.0
        key = gumbel_keys(lg[r], T, sd, st, r, v_offset) if T > 0 else lg[r].clone()
        if mask is not None:
            words = mask[r].detach().cpu().to(torch.int64) & 0xFFFFFFFF
            bits = ((words[:, None] >> torch.arange(32)[None, :]) & 1).reshape(-1)[v_offset : v_offset + V].bool()
            key = key.masked_fill(~bits, float("-inf"))
        if not (torch.isinf(key).all() and key.max() < 0):
            j = int(torch.argmax(key))  # first maximum: the lowest id wins ties, as in the kernel
            vals[r], idx[r] = key[j], v_offset + j
    return vals, idx


def merge_partials(vals: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """[n_src, rows] partial maxima -> token per row (largest key, lowest id on ties; -1 if none)."""
    n_src, rows = vals.shape
    out = torch.full((rows,), -1, dtype=torch.int64)
    for r in range(rows):
        best_v, best_i = float("-inf"), -1
        for p in range(n_src):
            v, i = float(vals[p, r]), int(idx[p, r])
            if i < 0:
                continue
            if best_i < 0 or v > best_v or (v == best_v and i < best_i):
                best_v, best_i = v, i
        out[r] = best_i
    return out


def sample(logits, *, mask, temperature, seed, step, out_tokens, v_offset=0):
    vals, idx = sample_partial(logits, mask=mask, temperature=temperature, seed=seed, step=step, v_offset=v_offset)
    out_tokens[: logits.shape[0]] = idx.to(out_tokens.dtype).to(out_tokens.device)
    step.add_(1)
    return out_tokens


def pcm16_to_f32(pcm, ratio, out):
    n_out = out.numel()
    if ratio == 1.0:
        out.copy_(pcm[:n_out].float() / 32768.0)
        return out
    src = torch.arange(n_out, dtype=torch.float64) * ratio
    j = src.floor().long()
    f = (src - j).float()
    j1 = (j + 1).clamp(max=pcm.numel() - 1)
    j = j.clamp(max=pcm.numel() - 1)
    out.copy_(((1 - f) * pcm[j].float() + f * pcm[j1].float()) / 32768.0)
    return out


def log_mel(audio, *, n_frames, window, mel_fb, out):
    """Whisper log-mel of a padded window -> out bf16 [n_frames, n_mels] (channels-last)."""
    stft = torch.stft(audio.float(), 400, 160, window=window.float(), center=True, pad_mode="reflect",
                      return_complex=True)
    mag = stft[..., :n_frames].abs() ** 2  # [201, frames]
    mel = mel_fb.float() @ mag
    lg = torch.clamp(mel, min=1e-10).log10()
    lg = torch.maximum(lg, lg.max() - 8.0)
    lg = (lg + 4.0) / 4.0
    out.copy_(lg.t().to(out.dtype))
    return out


def conv1d_gelu(x, w, b, *, stride, pos=None, out):
    B, Tin, Cin = x.shape
    Cout = w.shape[0]
    wt = w.float().view(Cout, 3, Cin).permute(0, 2, 1)  # [co, ci, kk]
    y = F.conv1d(x.float().transpose(1, 2), wt, None if b is None else b.float(), stride=stride, padding=1)
    y = F.gelu(y).transpose(1, 2)
    if pos is not None:
        y = y + pos[: y.shape[1]].float()[None]
    out.copy_(y.to(out.dtype))
    return out


def mel_filterbank(sr: int = 16000, n_fft: int = 400, n_mels: int = 80) -> torch.Tensor:
    """Slaney-style mel filterbank (librosa default, as used by Whisper) [n_mels, n_fft//2+1]."""

    def hz_to_mel(f):
        f = torch.as_tensor(f, dtype=torch.float64)
        f_sp = 200.0 / 3
        mels = f / f_sp
        min_log_hz = 1000.0
        min_log_mel = min_log_hz / f_sp
        logstep = math.log(6.4) / 27.0
        return torch.where(f >= min_log_hz, min_log_mel + torch.log(f / min_log_hz) / logstep, mels)

    def mel_to_hz(m):
        f_sp = 200.0 / 3
        freqs = f_sp * m
        min_log_hz = 1000.0
        min_log_mel = min_log_hz / f_sp
        logstep = math.log(6.4) / 27.0
        return torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), freqs)

    n_bins = n_fft // 2 + 1
    fftfreqs = torch.linspace(0, sr / 2, n_bins, dtype=torch.float64)
    mel_pts = torch.linspace(float(hz_to_mel(0.0)), float(hz_to_mel(sr / 2)), n_mels + 2, dtype=torch.float64)
    hz = mel_to_hz(mel_pts)
    fdiff = hz[1:] - hz[:-1]
    ramps = hz[:, None] - fftfreqs[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    weights = torch.clamp(torch.minimum(lower, upper), min=0.0)
    enorm = 2.0 / (hz[2 : n_mels + 2] - hz[:n_mels])
    weights = weights * enorm[:, None]
    return weights.float()
