"""ASR front-end kernels, each launched ITERS times eagerly: the target program of rocprofv3
hardware-counter passes (tools/gpu_recipes.sh frontend; summary: tools/pmc_summary.py).

Shapes: log-mel (80 / 128 mels, one 30 s window), the conv stem of whisper-tiny and large-v3
(padded-buffer path: the batched implicit GEMM), flash attention for the whisper-tiny / large-v3
encoder (B = 1 and 8 / 4) and the Llama-3-8B 1011-token causal prefill.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from voice_enabled_browser_automation_amd.ops import reference as ref  # noqa: E402

ITERS = 6
BF = torch.bfloat16


def main():
    dev = "cuda"
    ops.ext()
    torch.manual_seed(0)
    audio = torch.randn(480000, device=dev) * 0.1
    window = torch.hann_window(400, periodic=True, device=dev)
    for nm in (80, 128):
        fb = ref.mel_filterbank(n_mels=nm).to(dev)
        mel = torch.empty(3000, nm, dtype=BF, device=dev)
        for _ in range(ITERS):
            ops.log_mel(audio, n_frames=3000, window=window, mel_fb=fb, out=mel)
    torch.cuda.synchronize()
    for cin, d in ((80, 384), (128, 1280)):
        cp = ops.conv_channels(cin)
        _, mv = ops.padded_rows(1, 3000, cp, dtype=BF, device=dev)
        mv.copy_(torch.randn(1, 3000, cp, device=dev).to(BF))
        _, cv = ops.padded_rows(1, 3000, d, dtype=BF, device=dev)
        w1 = ops.TiledWeight((torch.randn(d, 3 * cp, device=dev) * 0.02).to(BF))
        w2 = ops.TiledWeight((torch.randn(d, 3 * d, device=dev) * 0.02).to(BF))
        b = torch.zeros(d, device=dev, dtype=BF)
        pos = torch.randn(1500, d, device=dev).to(BF)
        y = torch.empty(1, 1500, d, device=dev, dtype=BF)
        for _ in range(ITERS):
            ops.conv1d_gelu(mv, w1, b, stride=1, out=cv, padded=True)
        for _ in range(ITERS):
            ops.conv1d_gelu(cv, w2, b, stride=2, pos=pos, out=y, padded=True)
    torch.cuda.synchronize()
    for B, S, H, Hkv, D, causal in ((1, 1500, 6, 6, 64, False), (8, 1500, 6, 6, 64, False),
                                    (1, 1500, 20, 20, 64, False), (4, 1500, 20, 20, 64, False),
                                    (1, 1011, 32, 8, 128, True)):
        q = torch.randn(B, S, H, D, device=dev).to(BF)
        k = torch.randn(B, S, Hkv, D, device=dev).to(BF)
        v = torch.randn_like(k)
        tab = torch.arange(B, dtype=torch.int32, device=dev)[:, None]
        o = torch.empty_like(q)
        for _ in range(ITERS):
            ops.flash_attention(q, ops.KVLayout.contiguous(k, v, tab), Sk=S, n_kv_heads=Hkv, causal=causal,
                                scale=D ** -0.5, out=o)
    torch.cuda.synchronize()
    print("pmc_frontend done", flush=True)


if __name__ == "__main__":
    main()
