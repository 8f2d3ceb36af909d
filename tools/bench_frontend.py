"""ASR front-end / encoder kernels vs the PyTorch-ROCm library ops on the model shapes.

    python tools/bench_frontend.py [--json gpurun_out/frontend.jsonl]

Each case: median of 30 event-timed launches.  Ours: log-mel (f32 MFMA DFT + mel projection,
audio.hip), conv stem (batched implicit GEMM, gemm.hip), flash attention (32x32x16 MFMA,
attention.hip).  Reference: torch.stft + matmul, F.conv1d (MIOpen) + gelu, and
scaled_dot_product_attention -- library kernels only timed here, never used by the framework.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.ops import reference as ref  # noqa: E402

BF = torch.bfloat16


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = "cuda"
    ops.ext()
    rows = []

    def emit(name, ours, lib, flops=None):
        r = {"case": name, "ours_us": round(ours, 1), "torch_us": round(lib, 1) if lib else None,
             "speedup": round(lib / ours, 2) if lib else None}
        if flops:
            r["tflops"] = round(flops / ours / 1e6, 1)
        rows.append(r)
        print(json.dumps(r), flush=True)

    # log-mel of a 30 s window (80 and 128 mels)
    audio = torch.randn(480000, device=dev) * 0.1
    window = torch.hann_window(400, periodic=True, device=dev)
    for nm in (80, 128):
        fb = ref.mel_filterbank(n_mels=nm).to(dev)
        out = torch.empty(3000, nm, dtype=BF, device=dev)
        ours = timeit(lambda: ops.log_mel(audio, n_frames=3000, window=window, mel_fb=fb, out=out))

        def lib():
            st = torch.stft(audio, 400, 160, window=window, return_complex=True)
            p = st[:, :-1].abs() ** 2
            m = torch.clamp(fb @ p, min=1e-10).log10()
            return (torch.maximum(m, m.max() - 8.0) + 4.0) / 4.0

        emit(f"log_mel.{nm}", ours, timeit(lib), flops=2 * 3000 * 416 * 400 + 2 * 3000 * 208 * nm)

    # conv stem (whisper-tiny / large-v3): stride-1 mel conv and stride-2 conv + pos
    for name, cin, d in (("tiny", 80, 384), ("large", 128, 1280)):
        for B in (1, 8):
            cp = ops.conv_channels(cin)
            _, mv = ops.padded_rows(B, 3000, cp, dtype=BF, device=dev)
            mv.copy_(torch.randn(B, 3000, cp, device=dev).to(BF))
            _, cv = ops.padded_rows(B, 3000, d, dtype=BF, device=dev)
            w1 = ops.TiledWeight((torch.randn(d, 3 * cp, device=dev) * 0.02).to(BF))
            w2 = ops.TiledWeight((torch.randn(d, 3 * d, device=dev) * 0.02).to(BF))
            b = torch.zeros(d, device=dev, dtype=BF)
            pos = torch.randn(1500, d, device=dev).to(BF)
            y2 = torch.empty(B, 1500, d, device=dev, dtype=BF)

            def stem():
                ops.conv1d_gelu(mv, w1, b, stride=1, out=cv, padded=True)
                ops.conv1d_gelu(cv, w2, b, stride=2, pos=pos, out=y2, padded=True)

            wt1 = w1.dense().view(d, 3, cp).permute(0, 2, 1).contiguous()
            wt2 = w2.dense().view(d, 3, d).permute(0, 2, 1).contiguous()
            xt = mv.transpose(1, 2).contiguous()

            def lib():
                h = F.gelu(F.conv1d(xt, wt1, b, padding=1))
                return F.gelu(F.conv1d(h, wt2, b, stride=2, padding=1)).transpose(1, 2) + pos

            fl = 2 * B * (3000 * d * 3 * cp + 1500 * d * 3 * d)
            emit(f"conv_stem.{name}.B{B}", timeit(stem), timeit(lib), flops=fl)

    # flash attention: whisper encoder (non-causal, D 64) and Llama-3-8B 1011-token prefill (causal GQA)
    for name, B, S, H, Hkv, D, causal in (("enc.tiny", 1, 1500, 6, 6, 64, False),
                                          ("enc.tiny", 8, 1500, 6, 6, 64, False),
                                          ("enc.large", 1, 1500, 20, 20, 64, False),
                                          ("enc.large", 4, 1500, 20, 20, 64, False),
                                          ("prefill.llama8b", 1, 1011, 32, 8, 128, True)):
        q = torch.randn(B, S, H, D, device=dev).to(BF)
        k = torch.randn(B, S, Hkv, D, device=dev).to(BF)
        v = torch.randn_like(k)
        tab = torch.arange(B, dtype=torch.int32, device=dev)[:, None]
        o = torch.empty_like(q)
        kv = ops.KVLayout.contiguous(k, v, tab)
        ours = timeit(lambda: ops.flash_attention(q, kv, Sk=S, n_kv_heads=Hkv, causal=causal, scale=D ** -0.5,
                                                  out=o))
        qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if Hkv != H:
            kt, vt = kt.repeat_interleave(H // Hkv, 1), vt.repeat_interleave(H // Hkv, 1)
        lib = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=causal))
        fl = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
        emit(f"flash.{name}.B{B}", ours, lib, flops=fl)
    if args.json:
        with open(args.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
