"""Config / flag system.

* ``load_dotenv()`` mirrors the reference's two dotenv loads (app ``.env`` then repo-root
  ``.env``; the first value wins and real environment variables are never overridden:
  apps/brain/src/server.ts:10-11).
* ``Settings`` is the one typed view of every knob: the reference's variable names are kept
  verbatim for drop-in parity, plus the engine flags (VWA_*).
"""
from __future__ import annotations

import os
from typing import Optional

from pydantic import BaseModel


def _parse_env_file(path: str) -> dict:
    out = {}
    try:
        with open(path, "r", encoding="utf-8") as fh:
            for line in fh:
                line = line.strip()
                if not line or line.startswith("#") or "=" not in line:
                    continue
                k, v = line.split("=", 1)
                k = k.strip()
                if k.startswith("export "):
                    k = k[7:].strip()
                v = v.strip()
                if len(v) >= 2 and v[0] == v[-1] and v[0] in "\"'":
                    v = v[1:-1]
                out[k] = v
    except OSError:
        pass
    return out


def load_dotenv(app_dir: Optional[str] = None) -> None:
    cwd = app_dir or os.getcwd()
    for path in (os.path.join(cwd, ".env"), os.path.join(cwd, "..", "..", ".env")):
        for k, v in _parse_env_file(path).items():
            os.environ.setdefault(k, v)


class Settings(BaseModel):
    # reference variables (names kept)
    LLM_BASE_URL: str = "https://api.openai.com"
    LLM_API_KEY: str = ""
    LLM_MODEL: str = "gpt-4o-mini"
    BRAIN_PORT: int = 8090
    VOICE_PORT: int = 7072
    DEEPGRAM_API_KEY: Optional[str] = None
    DEEPGRAM_MODEL: str = "nova-3"
    BRAIN_URL: str = "http://127.0.0.1:8090/parse"
    EXECUTOR_URL: str = "http://127.0.0.1:7081"
    EXECUTOR_PORT: int = 7081
    ARTIFACTS_DIR: str = ".artifacts"
    EXECUTOR_HEADLESS: bool = False
    BROWSERBASE_API_KEY: Optional[str] = None
    BROWSERBASE_PROJECT_ID: Optional[str] = None
    BROWSERBASE_API_BASE: str = "https://api.browserbase.com/v1"
    # engine flags
    VWA_ASR_MODEL: str = "whisper-tiny"
    VWA_LLM_MODEL: str = "llama3-8b"
    VWA_BRAIN_ENGINE: str = "keyword"
    VWA_ASR_ENGINE: str = "none"
    VWA_TP: int = 1
    VWA_DP: int = 1
    VWA_DTYPE: str = "bf16"
    VWA_MAX_SESSIONS: int = 8
    VWA_HIPGRAPH: bool = True
    VWA_CHAIN: bool = True  # chained Llama decode layer tail (skinny_stream.hip chain_kernel SEQ 0)
    VWA_CHAIN_ASR: bool = False  # chained Whisper decoder launches (SEQ 1 / 2; measured no gain)
    VWA_MASKED_HEAD: bool = True  # LM head skips the vocab tiles the grammar mask excludes (intent decode)
    VWA_KV_GB: float = 0.0
    VWA_DEBOUNCE_MS: float = 1000.0
    VWA_BUDGET_CHARS: int = 512
    VWA_PARTIAL_EVERY_S: float = 1.0

    @classmethod
    def from_env(cls) -> "Settings":
        vals = {}
        for name, field in cls.model_fields.items():
            if name in os.environ:
                raw = os.environ[name]
                if field.annotation in (bool,):
                    vals[name] = raw.strip().lower() == "true" or raw.strip() == "1"
                else:
                    vals[name] = raw
        return cls(**vals)
