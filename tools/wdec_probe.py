"""Per-level timing of the persistent Whisper decoder (csrc/kernels/whisper_dec.hip) from its
s_memrealtime stamps (WdecParams::ts, 100 MHz): for every level of every layer, across the
workgroups that run it --

  hand-off   the level's first release (stamp 1) minus the previous level's LAST completion (stamp 3)
  stage      release -> activation row staged (stamp 2, GEMM levels)
  body       staged (or release) -> completion (stamp 3): MFMAs, reduce, epilogue, store drain
  span       previous level's last completion -> this level's last completion

(the x part of the cross query, level xq_x, runs beside the chain: body only) reported as the
median over layers 1..L-1 (layer 0 carries the launch ramp), plus the whole
launch time from the host and the decode us/token of the same model.

    python tools/wdec_probe.py [--layers 32] [--steps 20] [--opt 0] [--json out.jsonl]
"""
import argparse
import dataclasses
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.whisper import WDEC_LEVELS, WhisperModel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asr", default="whisper-large-v3")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--opt", type=int, default=0)
    ap.add_argument("--json", default=None)
    ap.add_argument("--role-opts", default="", help="role-plan variant, e.g. att_pen=1,sat=tail")
    a = ap.parse_args()
    ops.ext()
    os.environ["VWA_ASR_PERSIST"] = "1"
    from voice_enabled_browser_automation_amd.models import whisper as W
    for kv in filter(None, a.role_opts.split(",")):
        k, v = kv.split("=")
        W.WDEC_ROLE_OPTS[k] = v if k == "sat" else float(v)
    base = get_config(a.asr)
    a.layers = a.layers or base.n_dec_layers
    cfg = dataclasses.replace(base, n_enc_layers=1, n_dec_layers=a.layers)
    m = WhisperModel(cfg, device="cuda", seed=0, tile_decoder=True)
    torch.manual_seed(0)
    enc = torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16)
    r = WhisperRunner(m, max_sessions=1, use_graphs=True)
    r.set_cross(0, enc)
    r.step([(0, 5, 0)])
    st = next(iter(m._wdec.values()))
    grid, L = st["ints"][10], a.layers
    st["opt"] = a.opt
    # timing without stamps first (graph replays of one position: the launch's work is the same)
    for _ in range(3):
        r.step([(0, 7, 1)])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r.step([(0, 7, 1)])
    torch.cuda.synchronize()
    step_us = (time.perf_counter() - t0) / a.steps * 1e6
    # stamped launches (ts is a kernel argument: recapture)
    ts = torch.zeros(grid * L * 8 * 4, dtype=torch.int64, device="cuda")
    st["ts"] = ts
    r.graphs.clear()
    rows = []
    for _ in range(5):
        ts.zero_()
        r.step([(0, 7, 1)])
        torch.cuda.synchronize()
        rows.append(ts.view(grid, L, 8, 4).cpu())
    err = m.chain_error()
    res = {lv: dict(handoff=[], stage=[], body=[], span=[]) for lv in WDEC_LEVELS}
    late = {lv: {} for lv in WDEC_LEVELS}  # workgroup -> completion minus the level's median, per layer
    for t in rows:
        t = t.double() / 100.0  # 100 MHz -> us
        done_prev = None
        for li in range(L):
            for lvl, name in enumerate(WDEC_LEVELS):
                s = t[:, li, lvl]
                act = s[:, 3] > 0
                if not act.any():
                    continue
                ids = act.nonzero().flatten().tolist()
                s = s[act]
                rel, stg, dn = s[:, 1], s[:, 2], s[:, 3]
                if li > 0:
                    med = float(dn.median())
                    for wg, v in zip(ids, dn.tolist()):
                        late[name].setdefault(wg, []).append(v - med)
                off = name == "xq_x"  # (off the critical path: not part of the level chain)
                if done_prev is not None and li > 0 and not off:
                    res[name]["handoff"].append(float(rel.min() - done_prev))
                    res[name]["span"].append(float(dn.max() - done_prev))
                if (stg > 0).all():  # (attention levels: stamp 2 = softmax done)
                    res[name]["stage"].append(float((stg - rel).median()))
                    res[name]["body"].append(float((dn - stg).median()))
                else:
                    res[name]["body"].append(float((dn - rel).median()))
                if not off:
                    done_prev = float(dn.max())
    out = dict(tool="wdec_probe", asr=a.asr, layers=L, opt=a.opt, role_opts=a.role_opts, grid=grid, step_us=round(step_us, 1),
               per_layer_us=round(step_us / L, 2), error=bool(err))
    for name, d in res.items():
        out[name] = {k: round(statistics.median(v), 2) for k, v in d.items() if v}
    out["layer_span_us"] = round(sum(out[n].get("span", 0) for n in WDEC_LEVELS if n != "xq_x"), 2)
    for name in WDEC_LEVELS:  # the workgroups that finish a level latest (median lateness, us)
        lw = sorted(((statistics.median(v), wg) for wg, v in late[name].items()), reverse=True)[:4]
        out[name]["late"] = [[wg, round(v, 2)] for v, wg in lw]
    print(json.dumps(out), flush=True)
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(out) + "\n")


if __name__ == "__main__":
    main()
