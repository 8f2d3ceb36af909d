"""Run-to-run reproducibility of the two models (same inputs -> the same bits): Whisper encoder
states and greedy transcripts over repeated calls, and the Llama intent parse at temperature 0.
One JSON line per check.

    python tools/repro_check.py [--reps 4]"""
import argparse
import json
import os
import sys
import zlib

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import COMMANDS, synth_speech  # noqa: E402
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.asr.engine import AsrEngine  # noqa: E402
from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer  # noqa: E402


def crc(t: torch.Tensor) -> int:
    return zlib.crc32(t.detach().contiguous().view(torch.uint8).cpu().numpy().tobytes())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--llm", default="llama3-8b")
    a = ap.parse_args()
    ops.ext()
    dev = torch.device("cuda", 0)
    whisper = WhisperModel(get_config("whisper-tiny"), device=dev, seed=1)
    asr = AsrEngine(whisper, load_tokenizer("whisper"), max_sessions=2)
    for u in range(3):
        audio = asr.pcm_to_audio(synth_speech(10.0, seed=u))
        mel = whisper.mel_batch([audio])
        mels = [crc(mel)]
        enc = [crc(whisper.encode(mel))]
        for _ in range(a.reps - 1):
            mel = whisper.mel_batch([audio])
            mels.append(crc(mel))
            enc.append(crc(whisper.encode(mel)))
        toks = [tuple(asr.decode_many([audio], exact_tokens=40)[0]) for _ in range(a.reps)]
        print(json.dumps(dict(check="whisper", utt=u, mel_same=len(set(mels)) == 1, enc_same=len(set(enc)) == 1,
                              tokens_same=len(set(toks)) == 1, n_variants=len(set(toks)))), flush=True)
    llama = LlamaModel(get_config(a.llm), device=dev, seed=2)
    engine = LLMEngine(llama, max_seqs=4, max_model_len=2048, use_graphs=True)
    engine.capture_all()
    g = torch.Generator().manual_seed(5)
    prompt = torch.randint(0, 120000, (1000,), generator=g).tolist()

    def greedy(n=24):
        seq = engine.new_sequence(prompt, use_prefix_cache=False)
        lg = engine.prefill(seq)
        pre = crc(lg)
        toks = []
        t = int(lg.argmax(-1)[0])
        for _ in range(n):
            toks.append(t)
            lg = engine.run_rows([(seq, t)])
            t = int(lg.argmax(-1)[0])
        engine.free_sequence(seq, publish=False)
        return pre, tuple(toks), crc(lg)

    for mode in ("chain", "per_kernel"):
        if mode == "per_kernel":
            llama.disable_chain()
        res = [greedy() for _ in range(a.reps)]
        print(json.dumps(dict(check="llama_engine_greedy", mode=mode,
                              prefill_logits_same=len({r[0] for r in res}) == 1,
                              tokens_same=len({r[1] for r in res}) == 1,
                              last_logits_same=len({r[2] for r in res}) == 1)), flush=True)
    del engine, llama
    torch.cuda.empty_cache()
    llama = LlamaModel(get_config(a.llm), device=dev, seed=2)
    engine = LLMEngine(llama, max_seqs=4, max_model_len=2048, use_graphs=True)
    brain = LLMIntentEngine(engine, load_tokenizer("llama3"), budget_chars=512, temperature=0.0, seed=1234)
    engine.capture_all()
    for i in range(3):
        req = {"text": COMMANDS[i], "context": {"url": "https://www.bestbuy.com"}}
        outs = [brain.parse(req) for _ in range(a.reps)]
        print(json.dumps(dict(check="llama_greedy", req=i, same=len(set(map(str, outs))) == 1,
                              n_variants=len(set(map(str, outs))))), flush=True)


if __name__ == "__main__":
    main()
