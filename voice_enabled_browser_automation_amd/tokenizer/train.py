"""Offline BPE tokenizer builder.

There is no network on the build/GPU hosts, so the real Llama-3 / Whisper
tokenizer files cannot be fetched. This module trains byte-level BPE
tokenizers with the SAME vocabulary sizes and special-token layout as the
public models on a local text corpus (Python sources and docs on the image),
so that prompt/response token counts -- which set prefill and decode work --
are realistic (~3.5-4 chars/token on English/JSON), unlike a byte tokenizer.

* ``llama3``: 128000 BPE tokens + 256 special tokens (ids 128000..128255,
  ``<|begin_of_text|>``=128000, ``<|end_of_text|>``=128001,
  ``<|start_header_id|>``=128006, ``<|end_header_id|>``=128007,
  ``<|eot_id|>``=128009) -> 128256 total.
* ``whisper``: 50257 BPE tokens (GPT-2 sized; also used for the GPT-2-small
  CPU config) + Whisper's multilingual special tokens -> 51865 total
  (51866 for large-v3, which adds one language token).

The reference calls vendor models instead (apps/brain/src/llm.ts:22-27,
apps/voice/src/deepgram.ts:33-45); it has no tokenizer of its own.

Run: ``python -m voice_enabled_browser_automation_amd.tokenizer.train``
"""
from __future__ import annotations

import gzip
import os
import sys

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")

# cl100k/Llama-3 style pre-tokenisation split pattern.
SPLIT_PATTERN = (
    r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+"
)

CORPUS_ROOTS = ["/usr/local/lib/python3.10/dist-packages", "/usr/share/doc", "/usr/lib/python3"]

def _iter_corpus(max_bytes: int):
    # Generic text only: no benchmark/prompt strings are injected, so the
    # merges are not tuned to the command set being measured.
    total = 0
    for root in CORPUS_ROOTS:
        for dp, _dn, fn in sorted(os.walk(root)):
            for f in sorted(fn):
                if not f.endswith((".py", ".md", ".rst", ".txt")):
                    continue
                p = os.path.join(dp, f)
                try:
                    with open(p, "r", encoding="utf-8", errors="ignore") as fh:
                        s = fh.read()
                except OSError:
                    continue
                if not s:
                    continue
                total += len(s)
                # chunk to keep memory small in the trainer
                for i in range(0, len(s), 1 << 16):
                    yield s[i : i + (1 << 16)]
                if total >= max_bytes:
                    return


def whisper_special_tokens(n_vocab: int = 51865) -> list[str]:
    langs = [
        "en", "zh", "de", "es", "ru", "ko", "fr", "ja", "pt", "tr", "pl", "ca", "nl", "ar", "sv", "it", "id",
        "hi", "fi", "vi", "he", "uk", "el", "ms", "cs", "ro", "da", "hu", "ta", "no", "th", "ur", "hr", "bg",
        "lt", "la", "mi", "ml", "cy", "sk", "te", "fa", "lv", "bn", "sr", "az", "sl", "kn", "et", "mk", "br",
        "eu", "is", "hy", "ne", "mn", "bs", "kk", "sq", "sw", "gl", "mr", "pa", "si", "km", "sn", "yo", "so",
        "af", "oc", "ka", "be", "tg", "sd", "gu", "am", "yi", "lo", "uz", "fo", "ht", "ps", "tk", "nn", "mt",
        "sa", "lb", "my", "bo", "tl", "mg", "as", "tt", "haw", "ln", "ha", "ba", "jw", "su",
    ]
    if n_vocab == 51866:
        langs = langs + ["yue"]
    toks = ["<|endoftext|>", "<|startoftranscript|>"] + [f"<|{l}|>" for l in langs]
    toks += ["<|translate|>", "<|transcribe|>", "<|startoflm|>", "<|startofprev|>", "<|nospeech|>", "<|notimestamps|>"]
    toks += [f"<|{i * 0.02:.2f}|>" for i in range(1501)]
    assert 50257 + len(toks) == n_vocab, (len(toks), n_vocab)
    return toks


def llama3_special_tokens() -> list[str]:
    named = {
        0: "<|begin_of_text|>", 1: "<|end_of_text|>", 6: "<|start_header_id|>", 7: "<|end_header_id|>",
        8: "<|eom_id|>", 9: "<|eot_id|>", 10: "<|python_tag|>",
    }
    return [named.get(i, f"<|reserved_special_token_{i}|>") for i in range(256)]


def train(kind: str, max_bytes: int = 160_000_000) -> str:
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    if kind == "llama3":
        n_bpe, specials = 128000, llama3_special_tokens()
    elif kind == "whisper":
        # 50257 regular BPE ids (GPT-2 sized); <|endoftext|>=50257, <|startoftranscript|>=50258, ...
        n_bpe, specials = 50257, whisper_special_tokens()
    else:
        raise ValueError(kind)
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence(
        [
            pre_tokenizers.Split(Regex(SPLIT_PATTERN), behavior="isolated"),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False),
        ]
    )
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(
        vocab_size=n_bpe,
        min_frequency=2,
        show_progress=False,
        initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
        special_tokens=[],
    )
    tok.train_from_iterator(_iter_corpus(max_bytes), trainer=trainer)
    got = tok.get_vocab_size()
    if got < n_bpe:
        # pad with unreachable filler tokens so ids line up with the real model
        tok.add_tokens([f"<|pad_{i}|>" for i in range(n_bpe - got)])
    tok.add_special_tokens(specials)
    os.makedirs(ASSET_DIR, exist_ok=True)
    out = os.path.join(ASSET_DIR, f"{kind}_tokenizer.json.gz")
    with gzip.open(out, "wt", encoding="utf-8") as fh:
        fh.write(tok.to_str())
    return out


if __name__ == "__main__":
    kinds = sys.argv[1:] or ["llama3", "whisper"]
    for k in kinds:
        print(k, "->", train(k), flush=True)
