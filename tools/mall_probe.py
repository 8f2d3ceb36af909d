"""Does reading a decode step's first weights during the host gap help the step?  The Infinity
Cache (256 MB MALL) holds whatever was read last: after a decode step that is the LAST layers, so
layer 0 streams from HBM.  Here each 1-row Llama-3-8B decode step (the chained multi-layer launch,
engine graph replay) is timed with CUDA events, with and without a read of layer 0's weights
(QKV, o_proj, the first part of gate/up: --mb) right before it -- the work the host gap (~40 us of
idle GPU per step) could hide.

    python tools/mall_probe.py [--mb 200] [--steps 30]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=float, default=200.0)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    ops.ext()
    m = LlamaModel(get_config("llama3-8b"), device="cuda", seed=2)
    eng = LLMEngine(m, max_seqs=2, max_model_len=2048)
    eng.capture_all()
    torch.manual_seed(0)
    seq = eng.new_sequence(torch.randint(0, 120000, (1000,)).tolist())
    eng.prefill(seq)
    L0 = m.layers[0]
    raw = lambda w: (w.t if isinstance(w, ops.TiledWeight) else getattr(w, "w8", w))  # noqa: E731
    parts = [raw(L0.qkv), raw(L0.o), raw(L0.gu)]
    flat = [p.reshape(-1).view(torch.uint8) for p in parts]
    budget = int(a.mb * 2 ** 20)
    views = []
    for f in flat:
        n = min(f.numel(), budget)
        if n <= 0:
            break
        views.append(f[:n].view(torch.int32))
        budget -= n
    sink = torch.zeros(1, dtype=torch.int64, device="cuda")
    out = {}
    for mode in ("cold", "prefetch", "cold", "prefetch"):
        ts = []
        for i in range(a.steps):
            if mode == "prefetch":
                for v in views:  # (a reduction reads every byte once)
                    sink += v.sum(dtype=torch.int64)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.run_rows([(seq, 1234 + i)], check=False)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        out.setdefault(mode, []).append(round(statistics.median(ts[3:]), 1))
    print(json.dumps(dict(tool="mall_probe", prefetch_mb=a.mb, step_us=out)), flush=True)


if __name__ == "__main__":
    main()
