"""Tokenizers (byte-level BPE, HF `tokenizers` runtime) with the Llama-3 / Whisper id layouts.

The vocab files are built offline by ``tokenizer.train`` (no network: the public files cannot be
fetched) and shipped gzipped in ``assets/``.  A real ``tokenizer.json`` can be used instead by
pointing ``VWA_LLAMA_TOKENIZER`` / ``VWA_WHISPER_TOKENIZER`` at it.
"""
from __future__ import annotations

import functools
import gzip
import json
import os
from typing import List, Optional
from ..utils.env import knob

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


@functools.lru_cache(maxsize=1)
def _byte_decoder() -> dict:
    """Inverse of GPT-2's bytes_to_unicode (byte-level BPE symbol -> byte)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


class Tokenizer:
    def __init__(self, tok, kind: str):
        self._tok = tok
        self.kind = kind
        self.vocab_size = tok.get_vocab_size()
        self._bytes: Optional[List[bytes]] = None
        self.special_ids = set()
        for t, i in tok.get_vocab(with_added_tokens=True).items():
            if t.startswith("<|") and t.endswith("|>"):
                self.special_ids.add(i)

    def encode(self, text: str) -> List[int]:
        return self._tok.encode(text, add_special_tokens=False).ids

    def decode(self, ids: List[int], skip_special: bool = True) -> str:
        return self._tok.decode(ids, skip_special_tokens=skip_special)

    def token_to_id(self, t: str) -> Optional[int]:
        return self._tok.token_to_id(t)

    def token_bytes(self) -> List[bytes]:
        """Raw bytes of every id (b'' for special/added tokens)."""
        if self._bytes is None:
            dec = _byte_decoder()
            out: List[bytes] = []
            for i in range(self.vocab_size):
                if i in self.special_ids:
                    out.append(b"")
                    continue
                s = self._tok.id_to_token(i)
                if s is None:
                    out.append(b"")
                    continue
                try:
                    out.append(bytes(dec[ch] for ch in s))
                except KeyError:
                    out.append(b"")
            self._bytes = out
        return self._bytes

    def decode_bytes(self, ids: List[int]) -> bytes:
        tb = self.token_bytes()
        return b"".join(tb[i] for i in ids if 0 <= i < len(tb))


@functools.lru_cache(maxsize=4)
def load_tokenizer(kind: str = "llama3") -> Tokenizer:
    from tokenizers import Tokenizer as HFTok

    env = {"llama3": "VWA_LLAMA_TOKENIZER", "whisper": "VWA_WHISPER_TOKENIZER", "gpt2": "VWA_GPT2_TOKENIZER"}.get(kind)
    path = knob(env) if env else None
    if path:
        tok = HFTok.from_file(path)
    elif kind == "gpt2":
        tok = HFTok.from_str(json.dumps(_gpt2_layout(_asset_json("whisper"))))
    else:
        tok = HFTok.from_str(json.dumps(_asset_json(kind)))
    return Tokenizer(tok, kind)


def _asset_json(kind: str) -> dict:
    with gzip.open(os.path.join(ASSET_DIR, f"{kind}_tokenizer.json.gz"), "rt", encoding="utf-8") as fh:
        return json.load(fh)


GPT2_PATTERN = r"""'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"""


def _gpt2_layout(d: dict) -> dict:
    """GPT-2 id layout (50257 ids, <|endoftext|> = 50256) derived from the byte-level BPE shared
    with the Whisper vocabulary: the last merge is dropped so the BPE part ends at 50255, the
    Whisper special tokens are removed, and the GPT-2 pre-tokenizer regex is used."""
    m = d["model"]
    last = max(m["vocab"].values())
    m["vocab"] = {t: i for t, i in m["vocab"].items() if i < last}
    m["merges"] = m["merges"][:-1]
    d["added_tokens"] = [{"id": last, "content": "<|endoftext|>", "single_word": False, "lstrip": False,
                          "rstrip": False, "normalized": False, "special": True}]
    d["pre_tokenizer"] = {"type": "Sequence", "pretokenizers": [
        {"type": "Split", "pattern": {"Regex": GPT2_PATTERN}, "behavior": "Isolated", "invert": False},
        {"type": "ByteLevel", "add_prefix_space": False, "trim_offsets": True, "use_regex": False}]}
    d["post_processor"] = None
    return d
