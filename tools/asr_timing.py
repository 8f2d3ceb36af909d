"""Whisper transcription time split (encoder / decoder) with and without the chained decoder
launches (models/whisper.py, skinny_stream.hip chain_kernel SEQ 1/2), fixed 40-token work on the
bench's synthetic 10 s utterance.  One JSON line per mode.
python tools/asr_timing.py [--asr whisper-large-v3] [--reps 10]

decode_us_per_token = host time from the encoder's launch to the last token / tokens (includes the
encoder and cross K/V projections still running after their launch); decode_gpu_us_per_token = the
decoder's stream time (4-token prompt step + the token loop, CUDA events) / tokens."""
import argparse
import json
import os
import statistics
import sys
import time

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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tokens", type=int, default=40)
    ap.add_argument("--batch", default="", help="also time transcribe_many over B utterances (comma list)")
    ap.add_argument("--modes", default="0,p",
                    help="decoder forms to time: 0 per-kernel, 1 chained launches (VWA_CHAIN_ASR), p the persistent "
                         "one-launch decoder (VWA_ASR_PERSIST, whisper-large)")
    ap.add_argument("--small-max-m", type=int, default=None,
                    help="A/B: rows up to which small weights take the one-tile kernel (16: the tiled GEMM above 16)")
    a = ap.parse_args()
    ops.ext()
    if a.small_max_m is not None:
        ops.SMALL_MAX_M = a.small_max_m
    m = WhisperModel(get_config(a.asr), device="cuda", seed=0)
    if a.batch:  # concurrent sessions' batched pass (bench.py --concurrent: one per round)
        sizes = [int(x) for x in a.batch.split(",")]
        eng = AsrEngine(m, load_tokenizer("whisper"), max_sessions=max(sizes))
        for B in sizes:
            audios = [eng.pcm_to_audio(synth_speech(10.0, seed=100 + j)) for j in range(B)]
            for _ in range(2):
                eng.transcribe_many(audios, exact_tokens=a.tokens)
            ts, enc, dec = [], [], []
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                eng.transcribe_many(audios, exact_tokens=a.tokens)
                ts.append((time.perf_counter() - t0) * 1e3)
                s = getattr(eng, "last_stats", {}) or {}
                enc.append(s.get("encode_ms", 0.0))
                dec.append(s.get("decode_ms", 0.0))
            print(json.dumps(dict(tool="asr_timing", asr=a.asr, batch=B, tokens=a.tokens,
                                  total_ms=round(statistics.median(ts), 2), encode_ms=round(statistics.median(enc), 2),
                                  decode_ms=round(statistics.median(dec), 2))), flush=True)
        return
    audio = None
    texts = {}
    for chain in a.modes.split(","):
        os.environ["VWA_CHAIN_ASR"] = "1" if chain == "1" else "0"
        os.environ["VWA_ASR_PERSIST"] = "1" if chain == "p" else "0"
        m.reset_chains()
        eng = AsrEngine(m, load_tokenizer("whisper"), max_sessions=2)
        audio = eng.pcm_to_audio(synth_speech(10.0, seed=100))
        for _ in range(2):
            eng.transcribe(audio, exact_tokens=a.tokens)
        enc, dec, tot, dgpu = [], [], [], []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            texts[chain] = eng.transcribe(audio, exact_tokens=a.tokens)
            s = eng.last_stats
            enc.append(s["encode_ms"])
            dec.append(s["decode_ms"])
            tot.append(s["total_ms"])
            if s.get("decode_gpu_ms") is not None:
                dgpu.append(s["decode_gpu_ms"])
        print(json.dumps(dict(tool="asr_timing", asr=a.asr, chain=chain == "1", persistent=chain == "p",
                              persistent_used=bool(getattr(m, "_wdec", None)), tokens=a.tokens,
                              encode_ms=round(statistics.median(enc), 2), decode_ms=round(statistics.median(dec), 2),
                              total_ms=round(statistics.median(tot), 2),
                              decode_us_per_token=round(1e3 * statistics.median(dec) / a.tokens, 1),
                              # the decoder's own stream time (prompt step + token loop), from events:
                              # decode_ms starts when the encoder is LAUNCHED, so it also holds the
                              # encoder / cross K/V tail still running then
                              decode_gpu_us_per_token=round(1e3 * statistics.median(dgpu) / a.tokens, 1) if dgpu else None,
                              chained=bool(m.chain_descs()))), flush=True)
    if len(texts) >= 2:
        print(json.dumps(dict(tool="asr_timing", same_text=len(set(texts.values())) == 1,
                              modes=list(texts), error=bool(m.chain_error()))), flush=True)


if __name__ == "__main__":
    main()
