"""Transcripts of the bench's synthetic utterances through the per-kernel and the persistent
Whisper decoder (fixed 40-token work, greedy): how many differ and where the first differing
token is -- numerics near-ties of random-init weights vs a real divergence.

    python tools/asr_mode_diff.py [--asr whisper-tiny] [--n 8]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import synth_speech  # noqa: E402
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.asr.engine import AsrEngine  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel  # noqa: E402
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asr", default="whisper-tiny")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--tokens", type=int, default=40)
    a = ap.parse_args()
    ops.ext()
    m = WhisperModel(get_config(a.asr), device="cuda", seed=1)  # (bench.py's seed)
    toks = {}
    for mode in ("0", "1"):
        os.environ["VWA_ASR_PERSIST"] = mode
        eng = AsrEngine(m, load_tokenizer("whisper"), max_sessions=2)
        toks[mode] = [eng.decode_many([eng.pcm_to_audio(synth_speech(10.0, seed=i))], exact_tokens=a.tokens)[0]
                      for i in range(a.n)]
    diff = []
    for i, (x, y) in enumerate(zip(toks["0"], toks["1"])):
        if x != y:
            k = next(j for j in range(min(len(x), len(y))) if x[j] != y[j]) if any(
                p != q for p, q in zip(x, y)) else min(len(x), len(y))
            diff.append([i, k])
    print(json.dumps(dict(tool="asr_mode_diff", asr=a.asr, n=a.n, tokens=a.tokens, differing=len(diff),
                          first_diff_token=diff, distinct_transcripts=len({tuple(t) for t in toks["0"]}),
                          example_per_kernel=toks["0"][0], example_persistent=toks["1"][0])), flush=True)


if __name__ == "__main__":
    main()
