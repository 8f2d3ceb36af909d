"""Debug: chained vs per-kernel single steps of n rows (fresh engine per n), two FFN widths."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import LlamaConfig  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402

ops.ext()
os.environ["VWA_CHAIN_MAX_ROWS"] = "16"
for ffn in (4096, 14336):
    cfg = LlamaConfig(name="dbg", vocab_size=4096, hidden=4096, n_layers=2, n_heads=32, n_kv_heads=8, head_dim=128,
                      ffn=ffn, max_pos=2048)
    model = LlamaModel(cfg, device="cuda", seed=5)
    torch.manual_seed(1)
    toks = torch.randint(0, cfg.vocab_size, (80,)).tolist()
    for n in (1, 4, 5, 8, 9, 16):
        outs = {}
        for chain in ("0", "1"):
            os.environ["VWA_CHAIN"] = chain
            e = LLMEngine(model, max_seqs=2, max_model_len=256, kv_blocks=20, block_size=16, use_graphs=False)
            s = e.new_sequence(toks[:30], use_prefix_cache=False)
            e.prefill(s)
            outs[chain] = e.run_rows([(s, t) for t in toks[30:30 + n]]).float().cpu()
            d = [v for v in model.chain_descs() if v is not None]
            xg = [int((v[2] >> 24) & 1) for v in d]
            e.free_sequence(s, publish=False)
            del e
            model.reset_chains()
        a, b = outs["1"], outs["0"]
        err = (a - b).abs().max().item()
        rows_err = [(a[i] - b[i]).abs().max().item() for i in range(a.shape[0])]
        print(f"ffn={ffn} n={n} err={err:.4f} ref_max={b.abs().max().item():.3f} xg={xg} rows={[round(x, 3) for x in rows_err]}",
              flush=True)
