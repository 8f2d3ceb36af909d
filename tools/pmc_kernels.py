"""Hot kernels of the voice->intent path, each launched a few times eagerly: the target program
for rocprofv3 hardware-counter passes (one counter group per run; see tools/pmc_summary.py).

Shapes are the headline config's: Llama-3-8B decode GEMMs at M = 1 (weights rotated over
copies larger than the 256 MB Infinity Cache, as decode streams 15 GB per token), decode
attention (1 row and a 64-row prompt chunk, ctx 1100), flash attention (Whisper-large encoder,
Llama 1k prefill), the Whisper-large conv stem and the log-mel front end.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402

ITERS = 6


def main():
    dev = "cuda"
    ops.ext()
    torch.manual_seed(0)
    for name, N, K in (("qkv", 6144, 4096), ("o_proj", 4096, 4096), ("down", 4096, 14336), ("lm_head", 128256, 4096)):
        x = torch.randn(1, K, device=dev).to(torch.bfloat16)
        ncopy = max(1, int(0.6e9 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        y = torch.empty(1, N, device=dev, dtype=torch.float32 if name == "lm_head" else torch.bfloat16)
        for i in range(ITERS):
            ops.linear(x, ws[i % ncopy], out=y)
        torch.cuda.synchronize()
        del ws
    # gate/up + SwiGLU epilogue
    x = torch.randn(1, 4096, device=dev).to(torch.bfloat16)
    ws = [(torch.randn(28672, 4096, device=dev) * 0.02).to(torch.bfloat16) for _ in range(3)]
    h = torch.empty(1, 14336, device=dev, dtype=torch.bfloat16)
    for i in range(ITERS):
        ops.linear_swiglu(x, ws[i % 3], fuse_rms=True, out=h)
    torch.cuda.synchronize()
    del ws
    # the same gate/up on the fp8 path (OCP e4m3 weights, per-row scales, fp8 MFMA)
    ws = [ops.FP8Weight.quantize((torch.randn(28672, 4096, device=dev) * 0.02).to(torch.bfloat16))
          for _ in range(5)]
    for i in range(ITERS):
        ops.linear_swiglu(x, ws[i % 5], fuse_rms=True, out=h)
    torch.cuda.synchronize()
    del ws
    # decode attention (multi-query MFMA kernel): 1 row, then a 64-row prompt chunk of one sequence
    nq, nkv, hd, bs, ctx = 32, 8, 128, 16, 1100
    per = 2048 // bs
    kc = torch.randn(per + 8, nkv, bs, hd, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    table = (torch.randperm(per + 7, device=dev)[:per].to(torch.int32) + 1).view(1, per)
    kv = ops.KVLayout.paged(kc, vc, table)
    for rows in (1, 64):
        q = torch.randn(rows, nq * hd, device=dev).to(torch.bfloat16)
        out = torch.empty_like(q)
        cl = torch.arange(ctx - rows + 1, ctx + 1, dtype=torch.int32, device=dev)
        sid = torch.zeros(rows, dtype=torch.int32, device=dev)
        for _ in range(ITERS):
            ops.decode_attention(q, kv, cl, sid, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                                 max_ctx=2048, out=out)
    torch.cuda.synchronize()
    # flash attention: Whisper-large encoder (non-causal, 20 heads x 64) and Llama prefill (causal GQA)
    for B, S, H, Hkv, D, causal in ((1, 1500, 20, 20, 64, False), (1, 1024, 32, 8, 128, True)):
        q = torch.randn(B, S, H, D, device=dev).to(torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device=dev).to(torch.bfloat16)
        v = torch.randn_like(k)
        tab = torch.arange(B, dtype=torch.int32, device=dev)[:, None]
        o = torch.empty_like(q)
        for _ in range(ITERS):
            ops.flash_attention(q, ops.KVLayout.contiguous(k, v, tab), Sk=S, n_kv_heads=Hkv, causal=causal,
                                scale=D ** -0.5, out=o)
    torch.cuda.synchronize()
    # Whisper-large conv stem (stride-2 conv, 1280 -> 1280 channels) and the log-mel front end
    x = torch.randn(1, 3000, 1280, device=dev).to(torch.bfloat16)
    w = (torch.randn(1280, 3 * 1280, device=dev) * 0.02).to(torch.bfloat16)
    b = torch.zeros(1280, device=dev, dtype=torch.bfloat16)
    for _ in range(ITERS):
        ops.conv1d_gelu(x, w, b, stride=2)
    from voice_enabled_browser_automation_amd.ops import reference as ref

    audio = torch.randn(480000, device=dev) * 0.1
    window = torch.hann_window(400, periodic=True, device=dev)
    fb = ref.mel_filterbank(n_mels=128).to(dev)
    mel = torch.empty(3000, 128, dtype=torch.bfloat16, device=dev)
    for _ in range(ITERS):
        ops.log_mel(audio, n_frames=3000, window=window, mel_fb=fb, out=mel)
    torch.cuda.synchronize()
    # round 3: the tiled MFMA GEMM (gemm.hip) on the prompt-suffix / cold-prompt gate-up shape,
    # bf16 and W8A8, and the chained decode layer (chain_kernel) of a Llama-3-8B-shaped model
    for M in (85, 1011):
        xg = torch.randn(M, 4096, device=dev).to(torch.bfloat16)
        wg = ops.TiledWeight((torch.randn(28672, 4096, device=dev) * 0.02).to(torch.bfloat16))
        hg = torch.empty(M, 14336, device=dev, dtype=torch.bfloat16)
        for _ in range(ITERS):
            ops.linear_swiglu(xg, wg, fuse_rms=True, out=hg)
        del wg
    wq = ops.FP8Weight.quantize((torch.randn(28672, 4096, device=dev) * 0.02).to(torch.bfloat16), tiled=True)
    xg = torch.randn(85, 4096, device=dev).to(torch.bfloat16)
    hg = torch.empty(85, 14336, device=dev, dtype=torch.bfloat16)
    for _ in range(ITERS):
        ops.linear_swiglu(xg, wq, fuse_rms=True, out=hg)
    del wq
    torch.cuda.synchronize()
    from voice_enabled_browser_automation_amd.models.config import LlamaConfig
    from voice_enabled_browser_automation_amd.models.llama import LlamaModel
    from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine

    cfg = LlamaConfig(name="pmc8b", n_layers=3)  # Llama-3-8B layer shapes (3 layers: 1.3 GB > MALL)
    m = LlamaModel(cfg, device=dev, seed=1)
    e = LLMEngine(m, max_seqs=1, max_model_len=2048, use_graphs=False)
    s = e.new_sequence(list(range(1000, 2100)), use_prefix_cache=False)
    e.prefill(s)
    for i in range(ITERS):
        e.run_rows([(s, 7 + i)])
    torch.cuda.synchronize()
    print("pmc_kernels done", flush=True)


if __name__ == "__main__":
    main()
