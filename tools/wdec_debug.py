"""Localise a mismatch of the persistent Whisper decoder (csrc/kernels/whisper_dec.hip) against the
per-kernel path: run the same one-row step both ways on the same weights / caches and compare
what each level leaves behind (per-layer self K / V rows at the step's slot, the last layer's cross
query, fc1 output and the final hidden row, the logits)."""
import dataclasses
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel  # noqa: E402


def main():
    ops.ext()
    n_layers = int(os.environ.get("WDEC_DBG_LAYERS", "2"))
    steps = int(os.environ.get("WDEC_DBG_STEPS", "3"))
    sess = int(os.environ.get("WDEC_DBG_SESS", "0"))
    cfg = dataclasses.replace(get_config("whisper-large-v3"), n_enc_layers=1, n_dec_layers=n_layers)
    m = WhisperModel(cfg, device="cuda", seed=3, tile_decoder=True)
    torch.manual_seed(4)
    enc = torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16)

    def snap(r, slot_row):
        b = r.b
        blk, off = slot_row // r.bs, slot_row % r.bs
        out = {}
        for li in range(n_layers):
            out[f"k{li}"] = b.k_cache[li][blk, :, off].float().cpu().clone()
            out[f"v{li}"] = b.v_cache[li][blk, :, off].float().cpu().clone()
        out["q"] = b.q[0].float().cpu().clone()
        out["f"] = b.f[0].float().cpu().clone()
        out["att"] = b.att[0].float().cpu().clone()
        out["x_final"] = (b.hidden if n_layers % 2 == 0 else b.h)[0].float().cpu().clone()
        return out

    res = {}
    for persist in (False, True):
        os.environ["VWA_ASR_PERSIST"] = "1" if persist else "0"
        r = WhisperRunner(m, max_sessions=sess + 1, use_graphs=False)
        r.set_cross(sess, enc)
        for p in range(steps):
            lg = r.step([(sess, (13 * p) % 1000, p)]).float().cpu().clone()
        torch.cuda.synchronize()
        slot = (1 + sess * r.bps + p // r.bs) * r.bs + p % r.bs
        s = snap(r, slot)
        s["logits"] = lg[0]
        res[persist] = s
        if persist:
            st = next(iter(m._wdec.values()))
            res["err"] = int(st["cnt"].view(torch.int64)[1024].item())
            res["cnt"] = st["cnt"].view(torch.int64)[: 8 * 8 * 16 : 16].view(8, 8).sum(1).tolist()
    for k in res[False]:
        a, b = res[True][k], res[False][k]
        d = (a - b).abs()
        print(json.dumps(dict(buf=k, max_err=round(d.max().item(), 5), ref_max=round(b.abs().max().item(), 4),
                              argmax_err=int(d.argmax().item()), got=round(a.flatten()[d.argmax()].item(), 4),
                              want=round(b.flatten()[d.argmax()].item(), 4))), flush=True)
    print(json.dumps(dict(err_word=res["err"], counter_sums=res["cnt"])), flush=True)


if __name__ == "__main__":
    main()
