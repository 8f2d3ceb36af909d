"""Host-driven vs device-resident Whisper decode on the bench's synthetic utterances (same
transcripts expected).  python tools/asr_loop_check.py [--asr whisper-tiny]"""
import argparse
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
    a = ap.parse_args()
    ops.ext()
    m = WhisperModel(get_config(a.asr), device="cuda", seed=0)
    eng = AsrEngine(m, load_tokenizer("whisper"), max_sessions=2)
    bad = 0
    for i in range(4):
        audio = eng.pcm_to_audio(synth_speech(10.0, seed=100 + i))
        eng.device_loop = False
        h = eng.transcribe(audio, exact_tokens=40)
        eng.device_loop = True
        d = eng.transcribe(audio, exact_tokens=40)
        print(i, "same" if h == d else "DIFF", repr(h[:60]), repr(d[:60]), flush=True)
        bad += h != d
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
