"""cProfile of the intent engine's host side during decode (which Python / native calls sit
between two GPU steps).  python tools/host_profile.py [--llm llama3-8b] > gpurun_out/host_prof.txt"""
import argparse
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine  # noqa: E402
from voice_enabled_browser_automation_amd.brain.prompt import COMMANDS  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--n", type=int, default=6)
    ap.add_argument("--concurrent", type=int, default=0, help="profile rounds of C requests decoded together")
    a = ap.parse_args()
    ops.ext()
    m = LlamaModel(get_config(a.llm), device="cuda", seed=2)
    eng = LLMEngine(m, max_seqs=max(4, a.concurrent), max_model_len=2048)
    brain = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=512, temperature=0.1, seed=1234)
    eng.capture_all()
    for i in range(2):
        brain.parse({"text": COMMANDS[i], "context": {"url": "https://www.bestbuy.com"}})
    torch.cuda.synchronize()
    reqs = [{"text": COMMANDS[i % len(COMMANDS)], "context": {"url": "https://www.bestbuy.com"}}
            for i in range(max(1, a.concurrent))]
    if a.concurrent:
        brain.parse_many(reqs)
    pr = cProfile.Profile()
    pr.enable()
    for i in range(a.n):
        if a.concurrent:
            brain.parse_many(reqs)
        else:
            brain.parse(reqs[i % len(reqs)])
    pr.disable()
    it = brain.batch_stats["iterations"]
    print("iterations", it, "timing_ms", {k: round(v, 1) for k, v in brain.timing.items()})
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(40)
    st.print_callees("run_rows")
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
