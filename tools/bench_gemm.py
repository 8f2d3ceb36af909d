"""Tiled MFMA GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.matmul) on the model shapes.

    python tools/bench_gemm.py [--json gpurun_out/gemm.jsonl]
Each shape: median of 50 timed launches (events), bf16 in / bf16 out, TFLOP/s and effective
weight-streaming TB/s (weight bytes / time: the bound for few-row shapes).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("llama8b.qkv", 85, 6144, 4096), ("llama8b.o", 85, 4096, 4096), ("llama8b.gu", 85, 28672, 4096),
    ("llama8b.down", 85, 4096, 14336),
    ("llama8b.qkv", 32, 6144, 4096), ("llama8b.gu", 32, 28672, 4096), ("llama8b.down", 64, 4096, 14336),
    ("llama8b.qkv", 1011, 6144, 4096), ("llama8b.o", 1011, 4096, 4096), ("llama8b.gu", 1011, 28672, 4096),
    ("llama8b.down", 1011, 4096, 14336),
    ("whisper-tiny.qkv", 1500, 1152, 384), ("whisper-tiny.fc1", 1500, 1536, 384), ("whisper-tiny.fc2", 1500, 384, 1536),
    ("whisper-large.qkv", 1500, 3840, 1280), ("whisper-large.fc1", 1500, 5120, 1280),
    ("whisper-large.fc2", 1500, 1280, 5120),
]


def timeit(fn, n=50):
    for _ in range(5):
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
    ap.add_argument("--cold", action="store_true",
                    help="prompt shapes only, weights rotated over copies > the 256 MB Infinity Cache (as a real "
                         "prefill reads each layer's weights from HBM)")
    a = ap.parse_args()
    ops.ext()
    dev = torch.device("cuda")
    rows = []
    for name, M, N, K in SHAPES:
        if a.cold and M < 1000:
            continue
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        ncopy = max(1, int(0.8e9 // (N * K * 2)) + 1) if a.cold else 1
        ws = [(torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16) for _ in range(ncopy)]
        tws = [ops.TiledWeight(w) for w in ws]
        w, tw = ws[0], tws[0]
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        i = [0]

        def nxt(lst):
            i[0] += 1
            return lst[i[0] % ncopy]

        t_ref = timeit(lambda: torch.matmul(x, nxt(ws).t()))
        ops.ext().gemm_set_p8(0)
        t_128 = timeit(lambda: ops.gemm(x, nxt(tws), out))
        ops.ext().gemm_set_p8(1)
        t_p8 = timeit(lambda: ops.gemm(x, nxt(tws), out)) if M >= 256 and N % 256 == 0 else None
        ops.ext().gemm_set_p8(2)
        t_own = timeit(lambda: ops.gemm(x, nxt(tws), out))
        ops.gemm(x, tw, out)
        ref = torch.matmul(x.float(), w.float().t())
        err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        fl = 2.0 * M * N * K
        r = dict(shape=name, M=M, N=N, K=K, hipblaslt_us=round(t_ref, 1), gemm_us=round(t_own, 1),
                 tile128_us=round(t_128, 1), tile256_8phase_us=None if t_p8 is None else round(t_p8, 1),
                 speedup=round(t_ref / t_own, 3), gemm_tflops=round(fl / t_own / 1e6, 1),
                 gemm_weight_tbps=round(N * K * 2 / t_own / 1e6, 2), rel_err=round(err, 5))
        r["cold"] = bool(a.cold)
        rows.append(r)
        print(json.dumps(r), flush=True)
        del ws, tws
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
