"""Per-op bitwise reproducibility: each op runs several times on the same inputs and the outputs
are compared bit for bit (tools/repro_check.py finds THAT a model is not reproducible; this finds
which op).  One JSON line per op.

    python tools/repro_ops.py"""
import json
import os
import sys
import zlib

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402

DEV, BF = "cuda", torch.bfloat16


def crc(t):
    return zlib.crc32(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())


def check(name, fn, reps=5):
    outs = set()
    for _ in range(reps):
        outs.add(crc(fn()))
    print(json.dumps(dict(op=name, same=len(outs) == 1, variants=len(outs))), flush=True)


def rnd(*s, scale=1.0):
    return (torch.randn(*s, device=DEV) * scale).to(BF)


def main():
    ops.ext()
    torch.manual_seed(0)
    # Whisper-tiny encoder shapes
    T, d, H, hd, F = 1500, 384, 6, 64, 1536
    x = rnd(T, d)
    lw, lb = rnd(d) + 1, rnd(d, scale=0.1)
    check("layernorm_1500x384", lambda: ops.layernorm(x, lw, lb, eps=1e-5))
    for name, (N, K) in {"qkv": (3 * d, d), "o": (d, d), "fc1": (F, d), "fc2": (d, F)}.items():
        w = ops.TiledWeight(rnd(N, K, scale=0.05))
        b = rnd(N, scale=0.1)
        xi = rnd(T, K)
        check(f"linear_tiled_{name}_1500", lambda: ops.linear(xi, w, b))
        check(f"linear_tiled_{name}_1500_gelu", lambda: ops.linear(xi, w, b, act="gelu"))
        r = rnd(T, N)
        check(f"linear_tiled_{name}_1500_resid", lambda: ops.linear(xi, w, b, residual=r))
    qkv = rnd(1, T, 3, H, hd)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    table = torch.arange(1, dtype=torch.int32, device=DEV)[:, None]
    check("flash_attn_encoder", lambda: ops.flash_attention(q, ops.KVLayout.contiguous(k, v, table), Sk=T,
                                                            n_kv_heads=H, causal=False, scale=hd ** -0.5))
    # conv stem
    from voice_enabled_browser_automation_amd.models.config import get_config
    from voice_enabled_browser_automation_amd.models.whisper import WhisperModel
    m = WhisperModel(get_config("whisper-tiny"), device=DEV, seed=1)
    audio = torch.randn(160000, device=DEV) * 0.1
    mel = m.mel_batch([audio])
    mv, cv = m._stem_buffers(1, 3000)
    check("conv1", lambda: ops.conv1d_gelu(mv, m.conv1_wp, m.conv1_b, stride=1, out=cv, padded=True).clone())
    c1 = ops.conv1d_gelu(mv, m.conv1_wp, m.conv1_b, stride=1, out=cv, padded=True)
    check("conv2", lambda: ops.conv1d_gelu(c1, m.conv2_wt, m.conv2_b, stride=2, pos=m.pos_enc, padded=True))
    check("encode", lambda: m.encode(mel))
    # decode attention (multi-query kernel): Llama GQA hd 128 at ctx ~1100, Whisper hd 64
    for nq, nkv, hd, ctx, rows in ((32, 8, 128, 1100, 1), (32, 8, 128, 1100, 4), (6, 6, 64, 40, 1),
                                   (6, 6, 64, 1500, 1)):
        bs = 16
        nblk = (ctx + bs - 1) // bs + 1
        kc = rnd(nblk * rows, nkv, bs, hd)
        vc = rnd(nblk * rows, nkv, bs, hd)
        table = torch.arange(nblk * rows, dtype=torch.int32, device=DEV).view(rows, nblk)
        qd = rnd(rows, nq * hd)
        lens = torch.full((rows,), ctx, dtype=torch.int32, device=DEV)
        sid = torch.arange(rows, dtype=torch.int32, device=DEV)
        od = torch.empty(rows, nq * hd, dtype=BF, device=DEV)
        check(f"decode_attn_hd{hd}_ctx{ctx}_rows{rows}",
              lambda: ops.decode_attention(qd, ops.KVLayout.paged(kc, vc, table), lens, sid, n_q_heads=nq,
                                           n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5, max_ctx=ctx + 16,
                                           out=od).clone())
    # Llama-3-8B shapes: prefill GEMM (85 rows), decode GEMV (1 row)
    for M in (85, 1):
        for name, (N, K) in {"qkv": (6144, 4096), "down": (4096, 14336)}.items():
            w = ops.TiledWeight(rnd(N, K, scale=0.02))
            xi = rnd(M, K)
            check(f"llama_linear_{name}_{M}", lambda: ops.linear(xi, w))
            check(f"llama_linear_{name}_{M}_rms", lambda: ops.linear(xi, w, fuse_rms=True))


if __name__ == "__main__":
    main()
