"""Decode-step GPU time vs rows per step (continuous batching: M concurrent sessions, one token
each), and batched admission prefill vs one prefill per request -- Llama-3-8B (or any preset)
at the intent prompt's shape: a shared ~1k-token cached prefix + an ~85-token suffix per request.

    python tools/rows_sweep.py [--model llama3-8b] [--dtype bf16] [--rows 1,8,16,32,64] [--json out.jsonl]

Per M: the step graph's replay (layers + all-rows LM head over the full vocab, like a decode
iteration without the grammar mask) timed with HIP events over ITERS replays, each appending one
token per row.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import BUCKETS, LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    ap.add_argument("--rows", default="1,2,4,8,16,32,64")
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--prefix", type=int, default=1024)
    ap.add_argument("--suffix", type=int, default=85)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-prefill-bench", action="store_true", help="skip the admission prefill comparison")
    a = ap.parse_args()
    ops.ext()
    dev = torch.device("cuda")
    rows_list = [int(x) for x in a.rows.split(",")]
    R = max(rows_list)
    m = LlamaModel(get_config(a.model), device=dev, seed=1, wdtype=a.dtype)
    e = LLMEngine(m, max_seqs=R, max_model_len=2048, use_graphs=True)
    g = torch.Generator().manual_seed(0)
    head = torch.randint(1000, 100000, (a.prefix,), generator=g).tolist()
    s0 = e.new_sequence(head)
    e.prefill(s0)
    e.free_sequence(s0)
    out = []

    def emit(rec):
        print(json.dumps(rec), flush=True)
        out.append(rec)

    # ---- admission prefill: R requests' suffixes, batched vs one by one
    suf = [torch.randint(1000, 100000, (a.suffix,), generator=g).tolist() for _ in range(R)]
    for mode in (() if a.no_prefill_bench else ("serial", "batched", "serial", "batched")):
        seqs = [e.new_sequence(head + s) for s in suf]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode == "serial":
            for s in seqs:
                e.prefill(s)
        else:
            e.prefill_batch([(s, len(s.tokens)) for s in seqs])
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        emit({"what": "admission_prefill", "mode": mode, "requests": R, "suffix_tokens": a.suffix,
              "cached_prefix": a.prefix, "ms": round(ms, 3), "ms_per_request": round(ms / R, 3)})
        for s in seqs:
            e.free_sequence(s, publish=False)
    # ---- decode step vs rows
    seqs = [e.new_sequence(head + s) for s in suf]
    e.prefill_batch([(s, len(s.tokens)) for s in seqs])
    e.capture_all(buckets=tuple(b for b in BUCKETS if b <= R), logit_buckets=())
    for M in rows_list:
        rows = lambda: [(seqs[i], 7) for i in range(M)]  # noqa: E731
        for _ in range(3):
            e.run_rows(rows(), check=False)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ts, hs = [], []
        for _ in range(a.iters):
            rr = rows()
            ev[0].record()
            h0 = time.perf_counter()
            e.run_rows(rr, check=False, defer_head=True)
            hs.append((time.perf_counter() - h0) * 1e6)
            ev[1].record()
            torch.cuda.synchronize()
            e.host_synced()
            ts.append(ev[0].elapsed_time(ev[1]))
        fwd = sorted(ts)[len(ts) // 2]
        host_us = sorted(hs)[len(hs) // 2]  # CPU time of building + launching the step
        ts = []
        for _ in range(a.iters):
            ev[0].record()
            e.run_rows(rows(), check=False)
            ev[1].record()
            torch.cuda.synchronize()
            e.host_synced()
            ts.append(ev[0].elapsed_time(ev[1]))
        full = sorted(ts)[len(ts) // 2]
        emit({"what": "decode_step", "model": a.model, "dtype": a.dtype, "rows": M, "chained": m._chain_ok(M),
              "layers_ms": round(fwd, 3), "with_lm_head_ms": round(full, 3), "host_launch_us": round(host_us, 1),
              "weight_GB": round(m.weight_bytes() / 1e9, 2), "ctx": len(seqs[0].tokens)})
    if a.json:
        with open(a.json, "a") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
