"""BASELINE.json config 1 on the CPU: canned transcripts -> /parse with the GPT-2-small intent
parser (random-init weights, grammar-constrained decoding, prefix-cached prompt head), no GPU, no
audio.  The reference's equivalent is one `gpt-4o-mini` JSON-mode round trip per command
(/root/reference/apps/brain/src/server.ts:89-139, llm.ts:17-27).

    python tools/bench_cpu_parse.py [--n 10] [--threads 8] [--llm gpt2-small]

Prints one JSON line: p50 / p90 /parse latency, decode steps, schema validity.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--llm", default="gpt2-small")
    a = ap.parse_args()
    import torch

    torch.set_num_threads(a.threads)
    from voice_enabled_browser_automation_amd.brain.prompt import COMMANDS
    from voice_enabled_browser_automation_amd.brain.server import build_llm_engine
    from voice_enabled_browser_automation_amd.contracts.schema import ParseResponse, safe_parse

    t0 = time.perf_counter()
    brain = build_llm_engine(a.llm, device="cpu")
    load_s = time.perf_counter() - t0
    lat, steps, ok = [], [], 0
    for i in range(a.warmup + a.n):
        req = {"text": COMMANDS[i % len(COMMANDS)], "context": {"url": "https://www.bestbuy.com"}}
        t = time.perf_counter()
        out = brain.parse(req)
        dt = (time.perf_counter() - t) * 1e3
        if i >= a.warmup:
            lat.append(dt)
            steps.append(brain.last_stats.get("decode_steps", 0))
            ok += int(safe_parse(ParseResponse, out).success)
    lat.sort()
    print(json.dumps({
        "tool": "bench_cpu_parse", "config": f"{a.llm} on CPU ({a.threads} threads), text-only /parse",
        "n": a.n, "p50_ms": round(statistics.median(lat), 1), "p90_ms": round(lat[int(0.9 * (len(lat) - 1))], 1),
        "decode_steps_mean": round(sum(steps) / len(steps), 1), "valid": f"{ok}/{a.n}", "load_s": round(load_s, 1),
        "data": "COMMANDS transcripts, random-init weights"}))


if __name__ == "__main__":
    main()
