"""Debug/validation of the fp8 (W8A8) path at Llama-3-8B shapes on the GPU:
1. eager gemm_fp8 vs the dequantised emulation for M = 17 / 32 / 64 on the qkv / gu / down shapes;
2. engine steps of 17..64 rows with hipGraphs vs without (finite, equal logits)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402


def main():
    ops.ext()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    ok = True
    for (N, K) in ((6144, 4096), (28672, 4096), (4096, 14336)):
        w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        wq = ops.FP8Weight.quantize(w, tiled=True)
        for M in (9, 17, 32, 64):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            out = ops.linear(x, wq, fuse_rms=True)
            xr, wr, _ = ops._ref_w8(x.float(), ops.FP8Weight(wq.rows(), wq.scale), True, 1e-5)
            exp = xr @ wr.t()
            err = (out.float() - exp).abs().max().item() / (exp.abs().max().item() + 1e-6)
            fin = bool(torch.isfinite(out).all())
            ok &= fin and err < 0.03
            print(f"linear N={N} K={K} M={M} rel_err={err:.4f} finite={fin}", flush=True)
    cfg = get_config(os.environ.get("FP8_CHECK_MODEL", "llama3-8b"))
    m = LlamaModel(cfg, device=dev, seed=2, wdtype="fp8")
    toks = torch.randint(0, 1000, (200,)).tolist()
    res = {}
    for graphs in (False, True):
        e = LLMEngine(m, max_seqs=64, max_model_len=512, use_graphs=graphs)
        if graphs:
            e.capture_all()
        seqs = [e.new_sequence(toks[i:i + 20], use_prefix_cache=False) for i in range(40)]
        for s in seqs:
            e.prefill(s)
        outs = []
        for n in (17, 32, 40):
            lg = e.run_rows([(s, toks[30 + i]) for i, s in enumerate(seqs[:n])]).float().cpu().clone()
            outs.append(lg)
            print(f"graphs={graphs} rows={n} finite={bool(torch.isfinite(lg).all())} absmax={lg.abs().max().item():.3f}",
                  flush=True)
        res[graphs] = outs
        for s in seqs:
            e.free_sequence(s, publish=False)
        del e
    for a, b in zip(res[False], res[True]):
        err = (a - b).abs().max().item()
        ok &= bool(torch.isfinite(b).all()) and err < 0.05 * (1 + a.abs().max().item())
        print(f"graphs vs eager max_err={err:.4f}", flush=True)
    print("FP8_CHECK", "PASS" if ok else "FAIL", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
