"""Op-by-op CPU vs GPU comparison of the Llama prefill path (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import LlamaConfig  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel, move_model  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402

CFG = LlamaConfig(name="t", vocab_size=4096, hidden=512, n_layers=3, n_heads=8, n_kv_heads=2, head_dim=64,
                  ffn=1024, max_pos=2048)
rec = []
for name in ("embedding", "qkv_rope_write", "flash_attention", "decode_attention", "linear", "linear_swiglu"):
    f = getattr(ops, name)

    def wrap(*a, _f=f, _n=name, **k):
        out = _f(*a, **k)
        if os.environ.get("NOREC"):
            rec.append((_n, out))
            return out
        rec.append((_n, out.detach().float().cpu().clone()))
        return out
    setattr(ops, name, wrap)


def run(model, toks, n, graphs=False):
    rec.clear()
    e = LLMEngine(model, max_seqs=2, max_model_len=512, kv_blocks=80, block_size=16, use_graphs=graphs)
    s = e.new_sequence(toks, use_prefix_cache=False)
    e.prefill(s, chunk=n)
    return list(rec)


torch.manual_seed(0)
toks = torch.randint(0, CFG.vocab_size, (140,)).tolist()[:120]
cpu = LlamaModel(CFG, device="cpu", seed=5)
a = run(cpu, toks, 2048)
gpu = LlamaModel(CFG, device="cpu", seed=5)
move_model(gpu, "cuda")
for graphs in (False, True, False):
    b = run(gpu, toks, 2048, graphs)
    print("graphs", graphs, [(n, round((x.float().cpu() - y.float().cpu()).abs().max().item(), 4))
                             for (n, x), (_, y) in zip(a, b)][-3:])
if os.environ.get("NOREC"):
    sys.exit(0)
for n in (120, 64):
    cpu = LlamaModel(CFG, device="cpu", seed=5)
    a = run(cpu, toks, n)
    gpu = LlamaModel(CFG, device="cpu", seed=5)
    move_model(gpu, "cuda")
    b = run(gpu, toks, n)
    print("chunk", n, "ops", len(a), len(b))
    for i, ((na, x), (nb, y)) in enumerate(zip(a, b)):
        err = (x - y).abs().max().item() if x.shape == y.shape else float("nan")
        print(f"{i:3d} {na:16s} {tuple(x.shape)} {tuple(y.shape)} err={err:.4f} ref_max={x.abs().max().item():.3f}")
