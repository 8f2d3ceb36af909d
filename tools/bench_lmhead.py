"""Llama-3-8B LM head (128256 x 4096, 1 row, pre-tiled bf16, HBM-resident: rotated over copies
past the Infinity Cache) on the streaming kernel: K-split waves x grid cap sweep.

    python tools/bench_lmhead.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    E = ops.ext()
    dev, bf = "cuda", torch.bfloat16
    for name, N, K in (("llama8b.lm_head", 128256, 4096), ("llama8b.qkv", 6144, 4096), ("llama8b.o", 4096, 4096)):
        ncopy = max(2, int(0.6e9 // (N * K * 2)) + 1)
        ws = [ops.tile_weight((torch.randn(N, K, device=dev) * 0.02).to(bf)) for _ in range(ncopy)]
        x = torch.randn(1, K, device=dev).to(bf)
        y = torch.empty(1, N, device=dev, dtype=torch.float32 if "lm" in name else bf)
        i = [0]

        def f():
            i[0] += 1
            E.skinny_gemm(x, ws[i[0] % ncopy], None, y, 0, False, 1e-5, None, None, None, True)

        r = {"shape": name, "MB": round(N * K * 2 / 1e6, 1)}
        for cap in (256, 512, 1024):
            for ks in (4, 8):
                E.set_skinny_mode(1, cap, ks, 2)
                r[f"g{cap}_k{ks}_us"] = round(timeit(f), 2)
        E.set_skinny_mode(1, 256, 0, 2)
        best = min(v for k, v in r.items() if k.endswith("_us"))
        r["best_tbps"] = round(N * K * 2 / best / 1e6, 2)
        print(json.dumps(r), flush=True)
        del ws


if __name__ == "__main__":
    main()
