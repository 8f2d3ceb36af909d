"""Target program for rocprofv3 counter passes over the chained decode layer (chain_kernel) of a
Llama model with the named config's layer shapes: a few layers (more than the 256 MB Infinity
Cache, so the weights stream from HBM as in a real decode step), a 1100-token prompt, then
ITERS eager 1-row decode steps.  Summarise the passes with tools/pmc_summary.py.

    rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv \
        -d gpurun_out/pmc70/p1 -- python tools/pmc_chain.py --model llama3-70b --layers 3
"""
import argparse
import dataclasses
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp8"))
    a = ap.parse_args()
    ops.ext()
    cfg = dataclasses.replace(get_config(a.model), n_layers=a.layers)
    m = LlamaModel(cfg, device="cuda", seed=1, wdtype=a.dtype)
    e = LLMEngine(m, max_seqs=1, max_model_len=2048, use_graphs=False)
    s = e.new_sequence(list(range(1000, 2100)), use_prefix_cache=False)
    e.prefill(s)
    torch.cuda.synchronize()
    for i in range(a.iters):
        e.run_rows([(s, 7 + i + r) for r in range(a.rows)])
    torch.cuda.synchronize()
    print(f"pmc_chain done: {cfg.name} x{a.layers} layers, {a.rows} row(s), chained="
          f"{sum(v is not None for v in m.chain_descs())}, weight GB/layer="
          f"{(m.weight_bytes() - m.lm_head.numel() * 2) / a.layers / 1e9:.3f}", flush=True)


if __name__ == "__main__":
    main()
