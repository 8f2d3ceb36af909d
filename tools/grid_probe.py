"""Streaming-GEMM grid A/B (diagnostic): decode shapes at grid cap 256 (one 8-wave workgroup per
CU) vs 512 (two per CU: 16 waves streaming).  tools/latency_probe.hip measured the tiled weight
stream at 6.2 TB/s with 8 waves per CU and 6.8 TB/s with 16."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402


def main():
    dev = "cuda"
    E = ops.ext()
    bf = torch.bfloat16
    shapes = {"lm_head": (128256, 4096, 1, 1), "gate_up": (28672, 4096, 3, 5), "down": (4096, 14336, 3, 5),
              "qkv": (6144, 4096, 6, 5), "o_proj": (4096, 4096, 8, 5)}
    res = {}
    for name, (N, K, copies, M) in shapes.items():
        ws = [ops.TiledWeight((torch.randn(N, K, device=dev) * 0.02).to(bf)) for _ in range(copies)]
        x = torch.randn(M, K, device=dev).to(bf)
        out = torch.empty(M, N, dtype=torch.float32 if name == "lm_head" else bf, device=dev)
        for cap in (256, 512, 256, 512):
            E.set_skinny_mode(1, cap, 8, 2)
            for i in range(3):
                ops.linear(x, ws[i % copies], out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 30
            e0.record()
            for i in range(n):
                ops.linear(x, ws[i % copies], out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            res.setdefault(name, {}).setdefault(str(cap), []).append(round(us, 2))
        del ws
        torch.cuda.empty_cache()
    E.set_skinny_mode(1, 256, 0, 2)
    print(json.dumps({"kernel": "grid_probe", "us": res}))


if __name__ == "__main__":
    main()
