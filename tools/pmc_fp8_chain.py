"""fp8 decode step (W8A16 chained layer over the fp8 tiled weights, fp8 LM head) of a
Llama-3-8B-shaped model, launched ITERS times eagerly: the rocprofv3 --pmc target for the fp8
decode's HBM bytes and MFMA use (tools/gpu_recipes.sh pmc, summary by tools/pmc_summary.py).

3 layers (0.65 GB of fp8 weights > the 256 MB Infinity Cache, as the full model's 7.5 GB per
token), 1 row at ~1.1k context, the bench's shape.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import LlamaConfig  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402

ITERS = 6


def main():
    ops.ext()
    cfg = LlamaConfig(name="pmc8b-fp8", n_layers=3)
    m = LlamaModel(cfg, device="cuda", seed=1, wdtype="fp8")
    e = LLMEngine(m, max_seqs=1, max_model_len=2048, use_graphs=False)
    s = e.new_sequence(list(range(1000, 2100)), use_prefix_cache=False)
    e.prefill(s)
    torch.cuda.synchronize()
    for i in range(ITERS):
        e.run_rows([(s, 7 + i)])
    torch.cuda.synchronize()
    print("pmc_fp8_chain done", flush=True)


if __name__ == "__main__":
    main()
