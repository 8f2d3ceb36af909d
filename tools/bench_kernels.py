"""Kernel microbenchmarks on the Llama-3-8B decode shapes (M = 1..32) and attention.

Reports time and effective HBM bandwidth of the MFMA skinny GEMM against torch.matmul
(hipBLASLt) on identical random data, interleaved in one process (guide §5.4 rule 24).
Usage: python tools/bench_kernels.py [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402


def timeit(fn, iters=40, reps=5):
    """GPU time per call: `iters` calls captured in one hipGraph, replayed `reps` times
    (no Python/launch gaps in the measurement)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(reps):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / (iters * reps) * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default="gemm,attn,flash", help="comma list of floor,gemm,gemm8,wfirst,attn,flash,mall")
    args = ap.parse_args()
    only = set(args.only.split(","))
    dev = "cuda"
    torch.manual_seed(0)
    res = []
    shapes = [("qkv", 6144, 4096), ("o_proj", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
              ("lm_head", 128256, 4096)]
    for M in ((1, 4, 16, 32) if "gemm" in only else ()):
        for name, N, K in shapes:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            # rotate over enough weight copies (>= 1 GiB) that the 256 MiB Infinity Cache cannot
            # serve them: decode streams 16 GB of distinct weights per token.
            ncopy = max(1, int(1.0e9 // (N * K * 2)) + 1)
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            it = [0]

            def ours():
                it[0] = (it[0] + 1) % ncopy
                ops.ext().skinny_gemm(x, ws[it[0]], None, y, 0, False, 1e-5, None)

            variants = {}
            for mode, cap, ks in ((0, 256, 8), (1, 256, 8), (1, 512, 4), (1, 768, 4)):
                ops.ext().set_skinny_mode(mode, cap, ks)
                variants[f"m{mode}_g{cap}_k{ks}"] = round(timeit(ours), 2)
            ops.ext().set_skinny_mode(1, 256, 0)

            def blas():
                it[0] = (it[0] + 1) % ncopy
                torch.matmul(x, ws[it[0]].t())

            t_ours = timeit(ours)
            t_blas = timeit(blas)
            del ws
            gb = N * K * 2 / 1e9
            r = dict(kernel="skinny_gemm", shape=name, M=M, N=N, K=K, us=round(t_ours, 2), variants=variants,
                     tbps=round(gb / (t_ours * 1e-6) / 1e3, 3), hipblaslt_us=round(t_blas, 2),
                     hipblaslt_tbps=round(gb / (t_blas * 1e-6) / 1e3, 3))
            print(json.dumps(r), flush=True)
            res.append(r)
    # small decoder GEMMs (Whisper): latency-bound, weights cache-resident across decode tokens;
    # one-tile kernel (m0) vs the persistent streaming kernel at several grid caps / wave splits
    small = [("tiny_qkv", 1152, 384), ("tiny_o", 384, 384), ("tiny_fc1", 1536, 384), ("tiny_fc2", 384, 1536),
             ("tiny_lm", 51872, 384), ("lv3_qkv", 3840, 1280), ("lv3_o", 1280, 1280), ("lv3_fc1", 5120, 1280), ("lv3_fc2", 1280, 5120)]
    for name, N, K in (small if "small" in only else ()):
        x = torch.randn(1, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        y = torch.empty(1, N, device=dev, dtype=torch.bfloat16)
        variants = {}
        ops.ext().set_small_gemm_bytes(0)  # measure each kernel as selected, not the size routing
        for mode, cap, ks in ((0, 256, 8), (1, 256, 8), (1, 128, 8), (1, 64, 8), (1, 32, 8), (1, 64, 4), (1, 32, 4)):
            ops.ext().set_skinny_mode(mode, cap, ks)
            variants[f"m{mode}_g{cap}_k{ks}"] = round(timeit(lambda: ops.ext().skinny_gemm(x, w, None, y, 0, False,
                                                                                             1e-5, None)), 2)
        ops.ext().set_skinny_mode(1, 256, 0)
        ops.ext().set_small_gemm_bytes(4 << 20)
        r = dict(kernel="skinny_small", shape=name, M=1, N=N, K=K, variants=variants)
        print(json.dumps(r), flush=True)
        res.append(r)
    # launch floor: the smallest kernels in the decode graph (graph-replayed like everything here)
    if "floor" in only:
        ids = torch.zeros(1, dtype=torch.int32, device=dev)
        tab = torch.randn(1024, 4096, device=dev).to(torch.bfloat16)
        o1 = torch.empty(1, 4096, device=dev, dtype=torch.bfloat16)
        r = dict(kernel="launch_floor", embedding_1row_us=round(timeit(lambda: ops.embedding(ids, tab, out=o1)), 2),
                 torch_fill_us=round(timeit(lambda: o1.fill_(1.0)), 2))
        print(json.dumps(r), flush=True)
        res.append(r)
    # prologue order A/B: first weight item before / after the X staging (+ fused RMSNorm)
    for M in ((1, 4) if "wfirst" in only else ()):
        for name, N, K in shapes[:4]:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            ncopy = max(1, int(1.0e9 // (N * K * 2)) + 1)
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            it = [0]
            out = {}
            for rms in (False, True):
                for wf in (0, 2):
                    def f():
                        it[0] = (it[0] + 1) % ncopy
                        ops.ext().skinny_gemm(x, ws[it[0]], None, y, 0, rms, 1e-5, None)
                    ops.ext().set_skinny_mode(1, 256, 8, wf)
                    out[f"rms{int(rms)}_wf{wf}"] = round(timeit(f), 2)
            ops.ext().set_skinny_mode(1, 256, 0, 2)
            del ws
            r = dict(kernel="prologue_order", shape=name, M=M, **out)
            print(json.dumps(r), flush=True)
            res.append(r)
    # fp8 (W8A8) streaming GEMM on the same shapes, vs torch._scaled_mm (hipBLASLt fp8) where available
    for M in ((1, 4, 16) if "gemm8" in only else ()):
        for name, N, K in shapes:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            ncopy = max(1, int(1.0e9 // (N * K)) + 1)
            ws = [ops.FP8Weight.quantize(torch.randn(N, K, device=dev) * 0.02) for _ in range(ncopy)]
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            it = [0]
            fits = ops._fp8_stream_fits(M, K)

            def ours8():
                it[0] = (it[0] + 1) % ncopy
                w8 = ws[it[0]]
                ops.ext().skinny_gemm(x, w8.w8, None, y, 0, False, 1e-5, None, w8.scale)

            def smm():
                it[0] = (it[0] + 1) % ncopy
                ops._fp8_matmul(x, ws[it[0]])

            t8 = timeit(ours8) if fits else float("nan")
            try:
                ts = timeit(smm)
            except Exception:  # noqa: BLE001
                ts = float("nan")
            del ws
            gb = N * K / 1e9
            r = dict(kernel="skinny_gemm_fp8", shape=name, M=M, N=N, K=K, us=round(t8, 2),
                     tbps=round(gb / (t8 * 1e-6) / 1e3, 3), scaled_mm_us=round(ts, 2))
            print(json.dumps(r), flush=True)
            res.append(r)
    # Infinity-Cache (MALL) experiment: GEMM time when its weights were read by the previous
    # kernel (prefetched into the 256 MB memory-side cache) vs cold
    for name, N, K in (shapes[1:3] if "mall" in only else ()):
        M = 1
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ncopy = max(1, int(1.0e9 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(ncopy)]
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        acc = torch.empty((), device=dev, dtype=torch.int64)
        it = [0]

        def pf():
            it[0] = (it[0] + 1) % ncopy
            torch.sum(ws[it[0]].view(torch.int32), dim=(0, 1), out=acc)

        def pf_gemm():
            pf()
            ops.ext().skinny_gemm(x, ws[it[0]], None, y, 0, False, 1e-5, None)

        def cold():
            it[0] = (it[0] + 1) % ncopy
            ops.ext().skinny_gemm(x, ws[it[0]], None, y, 0, False, 1e-5, None)

        t_pf, t_both, t_cold = timeit(pf), timeit(pf_gemm), timeit(cold)
        r = dict(kernel="mall_prefetch", shape=name, N=N, K=K, cold_us=round(t_cold, 2),
                 after_prefetch_us=round(t_both - t_pf, 2), prefetch_us=round(t_pf, 2))
        print(json.dumps(r), flush=True)
        res.append(r)
        del ws
    # decode attention, Llama-3-8B geometry, ctx 1200
    nq, nkv, hd, bs = 32, 8, 128, 16
    for rows, ctx in (((1, 64), (1, 256), (1, 512), (1, 1200), (1, 2000), (8, 1200), (32, 1200))
                      if "attn" in only else ()):
        blocks = rows * ((ctx + bs - 1) // bs) + 8
        kc = torch.randn(blocks, nkv, bs, hd, device=dev).to(torch.bfloat16)
        vc = torch.randn_like(kc)
        per = (ctx + bs - 1) // bs
        table = torch.arange(rows * per, device=dev, dtype=torch.int32).view(rows, per)
        q = torch.randn(rows, nq * hd, device=dev).to(torch.bfloat16)
        out = torch.empty_like(q)
        cl = torch.full((rows,), ctx, dtype=torch.int32, device=dev)
        sid = torch.arange(rows, dtype=torch.int32, device=dev)
        kv = ops.KVLayout.paged(kc, vc, table)
        n_splits = ops.decode_n_splits(2048)
        po = torch.empty(rows * n_splits * nq * hd, device=dev)
        pm = torch.empty(rows * n_splits * nq * 2, device=dev)
        t = timeit(lambda: ops.decode_attention(q, kv, cl, sid, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                                                scale=hd ** -0.5, max_ctx=2048, out=out, part_o=po, part_ml=pm))
        gb = rows * ctx * nkv * hd * 2 * 2 / 1e9
        r = dict(kernel="decode_attention", rows=rows, ctx=ctx, us=round(t, 2), tbps=round(gb / (t * 1e-6) / 1e3, 3))
        print(json.dumps(r), flush=True)
        res.append(r)
    # flash attention: whisper-tiny encoder and llama prefill
    for name, B, S, H, Hkv, D, causal in (("whisper_tiny_enc", 1, 1500, 6, 6, 64, False),
                                          ("whisper_large_enc", 1, 1500, 20, 20, 64, False),
                                          ("llama_prefill_1k", 1, 1024, 32, 8, 128, True)) if "flash" in only else ():
        q = torch.randn(B, S, H, D, device=dev).to(torch.bfloat16)
        k = torch.randn(B, S, Hkv, D, device=dev).to(torch.bfloat16)
        v = torch.randn_like(k)
        table = torch.arange(B, dtype=torch.int32, device=dev)[:, None]
        kv = ops.KVLayout.contiguous(k, v, table)
        out = torch.empty_like(q)
        t = timeit(lambda: ops.flash_attention(q, kv, Sk=S, n_kv_heads=Hkv, causal=causal, scale=D ** -0.5, out=out))
        fl = 4 * B * H * S * S * D / (2 if causal else 1)
        r = dict(kernel="flash_attention", shape=name, us=round(t, 2), tflops=round(fl / (t * 1e-6) / 1e12, 2))
        print(json.dumps(r), flush=True)
        res.append(r)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
