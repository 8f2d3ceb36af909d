"""Whisper-large-v3 decoder GEMM shapes at M = 1 with HBM-resident weights (rotated over copies
larger than the 256 MB Infinity Cache, as one decode token streams 1.5 GB): row-major one-tile
kernel, row-major streaming kernel, and the streaming kernel on the pre-tiled layout.

    python tools/bench_whisper_decode.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    dev, bf = "cuda", torch.bfloat16
    E = ops.ext()
    for name, N, K in (("qkv", 3840, 1280), ("o", 1280, 1280), ("fc1", 5120, 1280), ("fc2", 1280, 5120),
                       ("lm_head", 51872, 1280)):
        ncopy = max(2, int(0.5e9 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(bf) for _ in range(ncopy)]
        wt = [ops.tile_weight(w) for w in ws]
        x = torch.randn(1, K, device=dev).to(bf)
        y = torch.empty(1, N, device=dev, dtype=bf)
        i = [0]

        def run(tiled, w_list):
            def f():
                w = w_list[i[0] % ncopy]
                i[0] += 1
                E.skinny_gemm(x, w, None, y, 0, False, 1e-5, None, None, None, tiled)
            return f

        r = {"shape": name, "N": N, "K": K, "MB": round(N * K * 2 / 1e6, 2)}
        E.set_small_gemm_bytes(64 << 20)
        E.set_skinny_mode(0, 256, 8, 2)
        r["rowmajor_onetile_us"] = round(timeit(run(False, ws)), 2)
        E.set_small_gemm_bytes(0)
        for cap, ks in ((256, 8), (128, 8), (256, 4)):
            E.set_skinny_mode(1, cap, ks, 2)
            r[f"rowmajor_stream_g{cap}_k{ks}_us"] = round(timeit(run(False, ws)), 2)
            r[f"tiled_stream_g{cap}_k{ks}_us"] = round(timeit(run(True, wt)), 2)
        E.set_skinny_mode(1, 256, 0, 2)
        E.set_small_gemm_bytes(4 << 20)
        best = min(v for k, v in r.items() if k.endswith("_us"))
        r["best_tbps"] = round(N * K * 2 / (best * 1e-6) / 1e12, 3)
        print(json.dumps(r), flush=True)
        del ws, wt


if __name__ == "__main__":
    main()
