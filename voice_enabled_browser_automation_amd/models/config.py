"""Model configurations (public architecture hyper-parameters; weights are random-init or
loaded from safetensors).  The reference calls hosted models instead
(gpt-4o-mini: apps/brain/src/llm.ts:9; Deepgram nova-3: apps/voice/src/server.ts:106); the
north star (BASELINE.json) names these on-node replacements.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Optional


@dataclass(frozen=True)
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_pos: int = 8192
    tie_embeddings: bool = False
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128009)
    init_std: float = 0.02


@dataclass(frozen=True)
class GPT2Config:
    name: str = "gpt2-small"
    vocab_size: int = 50257
    hidden: int = 768
    n_layers: int = 12
    n_heads: int = 12
    ffn: int = 3072
    # n_positions is 1024 in the public config; the intent prompt is ~1.1k tokens, so the
    # CPU config runs with 2048 learned positions.
    max_pos: int = 2048
    ln_eps: float = 1e-5
    bos_id: int = 50256
    eos_ids: tuple = (50256,)
    init_std: float = 0.02

    @property
    def head_dim(self) -> int:
        return self.hidden // self.n_heads

    @property
    def n_kv_heads(self) -> int:
        return self.n_heads


@dataclass(frozen=True)
class WhisperConfig:
    name: str = "whisper-tiny"
    n_mels: int = 80
    n_audio_ctx: int = 1500
    d_model: int = 384
    n_heads: int = 6
    n_enc_layers: int = 4
    n_dec_layers: int = 4
    n_text_ctx: int = 448
    vocab_size: int = 51865
    ln_eps: float = 1e-5
    init_std: float = 0.02
    # special tokens (multilingual layout)
    eot: int = 50257
    sot: int = 50258
    lang_en: int = 50259
    transcribe: int = 50359
    no_timestamps: int = 50363

    @property
    def head_dim(self) -> int:
        return self.d_model // self.n_heads

    @property
    def ffn(self) -> int:
        return 4 * self.d_model


LLAMA_PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(name="llama3-70b", hidden=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn=28672),
    "llama3.2-1b": LlamaConfig(name="llama3.2-1b", hidden=2048, n_layers=16, n_heads=32, n_kv_heads=8, head_dim=64,
                               ffn=8192, tie_embeddings=True),
    # small shapes for CPU tests (vocab kept at the real tokenizer size so the grammar works)
    "llama-tiny": LlamaConfig(name="llama-tiny", hidden=256, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=64,
                              ffn=512, max_pos=4096),
}

GPT2_PRESETS = {
    "gpt2-small": GPT2Config(),
    "gpt2-tiny": GPT2Config(name="gpt2-tiny", hidden=128, n_layers=2, n_heads=2, ffn=512),
}

WHISPER_PRESETS = {
    "whisper-tiny": WhisperConfig(),
    "whisper-base": WhisperConfig(name="whisper-base", d_model=512, n_heads=8, n_enc_layers=6, n_dec_layers=6),
    "whisper-small": WhisperConfig(name="whisper-small", d_model=768, n_heads=12, n_enc_layers=12, n_dec_layers=12),
    "whisper-large-v3": WhisperConfig(name="whisper-large-v3", n_mels=128, d_model=1280, n_heads=20, n_enc_layers=32,
                                      n_dec_layers=32, vocab_size=51866, lang_en=50259, transcribe=50360,
                                      no_timestamps=50364),
    "whisper-test": WhisperConfig(name="whisper-test", d_model=128, n_heads=2, n_enc_layers=2, n_dec_layers=2),
}


def get_config(name: str):
    for table in (LLAMA_PRESETS, GPT2_PRESETS, WHISPER_PRESETS):
        if name in table:
            return table[name]
    raise KeyError(f"unknown model preset {name!r}")
