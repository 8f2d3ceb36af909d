"""Config / flag system: ONE typed settings object for every knob.

* ``load_dotenv()`` mirrors the reference's two dotenv loads (app ``.env`` then repo-root
  ``.env``; the first value wins and real environment variables are never overridden:
  apps/brain/src/server.ts:10-11).
* ``Settings`` declares every knob -- the reference's variable names verbatim (drop-in parity:
  apps/brain/src/llm.ts:7-9, apps/voice/src/server.ts:64-72, apps/executor/src/*.ts) plus the
  engine's ``VWA_*`` flags -- with its type, default and meaning.
* ``knob(name)`` is how code reads a knob: the environment value parsed with the declared type, or
  the declared default.  An undeclared name raises (a typo or an undocumented knob fails loudly;
  ``tests/test_settings_cpu.py`` also checks that every ``VWA_*`` name in the sources is declared).
  It reads the environment at call time, so a process (or a test) that changes a variable sees the
  change; ``settings()`` is the parsed snapshot a service takes at startup.
"""
from __future__ import annotations

import os
from typing import Any, Optional

from pydantic import BaseModel, Field


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
    # ---- reference variables (names kept)
    LLM_BASE_URL: str = Field("https://api.openai.com", description="reference brain LLM endpoint (unused on-node)")
    LLM_API_KEY: str = Field("", description="reference brain LLM key (unused on-node)")
    LLM_MODEL: str = Field("gpt-4o-mini", description="reference brain model name (reported in /health)")
    BRAIN_PORT: int = Field(8090, description="brain HTTP port")
    VOICE_PORT: int = Field(7072, description="voice HTTP/WS port (the DP router's port with several workers)")
    WEB_PORT: int = Field(5173, description="web UI port")
    EXECUTOR_PORT: int = Field(7081, description="executor HTTP port")
    DEEPGRAM_API_KEY: Optional[str] = Field(None, description="reference STT key (unused: on-node ASR)")
    DEEPGRAM_MODEL: str = Field("nova-3", description="reference STT model name (unused)")
    BRAIN_URL: str = Field("http://127.0.0.1:8090/parse", description="voice -> brain /parse URL")
    EXECUTOR_URL: str = Field("http://127.0.0.1:7081", description="voice -> executor base URL")
    ARTIFACTS_DIR: str = Field(".artifacts", description="executor screenshots / extracts")
    UPLOAD_DIR: str = Field(".uploads", description="executor file uploads")
    EXECUTOR_HEADLESS: bool = Field(False, description="launch the local browser headless")
    CDP_URL: Optional[str] = Field(None, description="attach the executor to a running browser's DevTools endpoint")
    CHROME_PATH: Optional[str] = Field(None, description="browser binary for the local session")
    BROWSERBASE_API_KEY: Optional[str] = Field(None, description="Browserbase cloud sessions")
    BROWSERBASE_PROJECT_ID: Optional[str] = Field(None, description="Browserbase project")
    BROWSERBASE_API_BASE: str = Field("https://api.browserbase.com/v1", description="Browserbase REST base")
    # ---- services / deployment
    VWA_BRAIN_ENGINE: str = Field("keyword", description="brain engine: keyword | llm | gpt2")
    VWA_ASR_ENGINE: str = Field("none", description="voice recognizer: none (passthrough) | whisper")
    VWA_ASR_MODEL: str = Field("whisper-tiny", description="Whisper config name (models/config.py)")
    VWA_ASR_WEIGHTS: Optional[str] = Field(None, description="safetensors checkpoint for the ASR (random init otherwise)")
    VWA_LLM_MODEL: str = Field("llama3-8b", description="Llama config name (models/config.py)")
    VWA_LLM_WEIGHTS: Optional[str] = Field(None, description="safetensors checkpoint for the LLM (random init otherwise)")
    VWA_DTYPE: str = Field("bf16", description="LLM weight dtype: bf16 | fp8")
    VWA_SEED: int = Field(0, description="random-init seed / sampling seed")
    VWA_TP: int = Field(1, description="tensor-parallel degree of the brain")
    VWA_DP: int = Field(1, description="voice workers behind the session router")
    VWA_MAX_SESSIONS: int = Field(8, description="concurrent sessions per engine (ASR slots, LLM sequences)")
    VWA_BUDGET_CHARS: int = Field(512, description="intent JSON character budget (grammar closes within it)")
    VWA_BRAIN_GPUS: str = Field("", description="launch.py: brain GPU list override")
    VWA_VOICE_GPUS: str = Field("", description="launch.py: voice GPU list override")
    VWA_VOICE_BASE_PORT: int = Field(7100, description="first port of the per-GPU voice workers")
    VWA_BRAIN_MAX_RESTARTS: int = Field(5, description="brain (TP group) restarts per 10 min before giving up")
    VWA_MASTER_PORT: Optional[str] = Field(None, description="TP rendezvous port of the first brain start")
    VWA_SHARED_CHAIN: str = Field("0", description="brain sharing its GPU with a voice worker keeps the chained decode")
    VWA_SHARED_CHAIN_GRID_DIV: Optional[str] = Field(None, description="that chained launch on CUs / k workgroups")
    VWA_SHARED_GB: float = Field(0.0, description="HBM a co-located service keeps (KV auto-sizing leaves it free)")
    VWA_WATCHDOG_S: float = Field(2.0, description="DP router: health poll period")
    VWA_WATCHDOG_FAILS: int = Field(2, description="DP router: failed polls before a worker is declared dead")
    VWA_TP_HEARTBEAT_S: float = Field(5.0, description="idle TP leader control heartbeat")
    VWA_TP_CONTROL: str = Field("shm", description="TP brain per-iteration control channel: shm (/dev/shm ring, parallel/control.py) or gloo (broadcast)")
    VWA_TP_DEAD_S: float = Field(60.0, description="TP worker: the leader counts as dead after this long without a control message or heartbeat (shm channel)")
    VWA_DIST_BACKEND: Optional[str] = Field(None, description="torch.distributed backend override (nccl = RCCL)")
    VWA_CUSTOM_AR: bool = Field(True, description="one-shot IPC all-reduce for small TP messages (else RCCL)")
    VWA_BROWSER_DRIVER: str = Field("auto", description="executor browser driver: auto | cdp | playwright")
    VWA_LLAMA_TOKENIZER: Optional[str] = Field(None, description="tokenizer.json for the Llama brain (bundled otherwise)")
    VWA_WHISPER_TOKENIZER: Optional[str] = Field(None, description="tokenizer.json for Whisper (bundled otherwise)")
    VWA_GPT2_TOKENIZER: Optional[str] = Field(None, description="tokenizer.json for the GPT-2 brain (bundled otherwise)")
    # ---- voice path (streaming ASR / debounce)
    VWA_DEBOUNCE_MS: float = Field(1000.0, description="final transcript -> brain call debounce (reference: 1000)")
    VWA_COMMIT_MS: float = Field(0.0, description="voice: silence after the speech end before pending finals are a command (0: the ASR endpoint; speech resuming earlier holds them -- voice/server.py commit policy)")
    VWA_SPEC_BRAIN: bool = Field(True, description="voice: start the brain on the ASR's speculative final pass (its answer is used only for exactly that text)")
    VWA_ASR_BUSY_FILE: Optional[str] = Field(None, description="/dev/shm word the voice worker's ASR batcher marks busy while recognition runs (shared-GPU deployment: the brain's decode uses the chained launch only while it is idle; launch.py sets it)")
    VWA_ASR_BUSY_HOLD_MS: float = Field(20.0, description="brain: keep the per-kernel decode form this long after the last ASR pass ended")
    VWA_ENDPOINT_MS: float = Field(300.0, description="trailing silence that ends an utterance (VAD endpoint)")
    VWA_SPEC_FINAL_MS: float = Field(120.0, description="trailing silence that starts the speculative final pass (0: off)")
    VWA_VAD_THRESHOLD: float = Field(300.0, description="speech frame RMS floor (PCM16 units)")
    VWA_VAD_NOISE_MULT: float = Field(3.0, description="speech frame RMS >= this x the tracked noise floor")
    VWA_PARTIAL_EVERY_S: float = Field(1.0, description="interim result period during speech")
    VWA_ASR_TOKENS_PER_S: float = Field(0.0, description="fixed-work transcripts (benchmarks on random weights; 0: off)")
    VWA_CONTEXT_MAX_BYTES: int = Field(2048, description="per-session context cap sent to the brain")
    # ---- engine
    VWA_HIPGRAPH: bool = Field(True, description="replay decode steps from captured hipGraphs")
    VWA_KV_GB: str = Field("0", description="paged-KV budget in GB, 0: per max_seqs x max_len, auto: HBM plan")
    VWA_ROW_BUCKETS: str = Field("1,2,4,8,12,16,32,48,64", description="decode row buckets of the captured graphs")
    VWA_SHARED_ATTN: bool = Field(True, description="decode attention reads a shared prompt prefix once per row group")
    VWA_PREFILL_FLASH: bool = Field(True, description="batched admission prefill through one causal flash launch")
    VWA_RMS_HANDOFF: bool = Field(True, description="> 16-row steps: residual GEMMs hand the next RMSNorm its row statistics (no row_rstd launches)")
    VWA_FP8_A16_ROWS: int = Field(64, description="fp8 weights: rows up to which the > 16-row GEMM runs W8A16 (no activation quantisation)")
    VWA_PREFILL_DECODE_ATTN: bool = Field(True, description="cached-prefix prompt suffix through the decode attention")
    VWA_TILED_WEIGHTS: bool = Field(True, description="keep projection weights only in the MFMA-tiled layout")
    VWA_MASKED_HEAD: bool = Field(True, description="LM head computes only the vocab tiles the grammar admits")
    VWA_SPIN_WAIT: bool = Field(True, description="wait for a step's tokens by polling the pinned readback")
    VWA_ZERO_COPY: bool = Field(True, description="grammar masks written straight into pinned step memory")
    VWA_ASR_DEVICE_LOOP: bool = Field(True, description="single-session Whisper greedy loop resident on the GPU")
    VWA_CHAIN: bool = Field(True, description="chained Llama decode layer (skinny_stream.hip chain_kernel)")
    VWA_CHAIN_ATTN: bool = Field(True, description="decode attention as the chained launch's phase 0")
    VWA_CHAIN_MAX_ROWS: int = Field(4, description="rows per step the chained launch takes")
    VWA_CHAIN_TP: bool = Field(True, description="chained launch with in-launch TP all-reduce rounds")
    VWA_CHAIN_RETRY: bool = Field(True, description="re-arm the chain after a barrier-timeout fallback")
    VWA_CHAIN_ASR: bool = Field(False, description="chained Whisper decoder launches (measured slower; off)")
    VWA_WDEC_OPT: int = Field(0, description="diagnostic: schedule option bits of the persistent Whisper decoder (whisper_dec.hip kOpt*; 0 = the measured defaults)")
    VWA_ASR_PERSIST: bool = Field(True, description="one-row Whisper decode steps (every width, tiny .. large) as ONE persistent launch: embedding, every decoder layer, LM head and, in the device loop, argmax + advance (csrc/kernels/whisper_dec.hip); needs every CU free: off when the GPU is shared with a persistent brain launch")
    VWA_CHAIN_GRID_DIV: Optional[str] = Field(None, description="chained launch on CUs / k workgroups (shared GPU)")
    VWA_CHAIN_PLAN: bool = Field(True, description="chained attention: layer 0 writes the step's work plan, layers 1.. read it")
    VWA_CHAIN_MULTI: bool = Field(True, description="chained decode: all layers in ONE launch (skinny_stream.hip chain_kernel MULTI)")
    VWA_CHAIN_BAR_MODE: int = Field(2, description="chained launches' grid barrier: 2 two-level tickets + scalar polls (default), 4 no-return arrivals + polled sum of the 8 group counters")
    VWA_CHAIN_SCHED: Optional[str] = Field(None, description="DIAGNOSTIC: chained schedule override name=value,...")
    VWA_GEMM_QKV: bool = Field(True, description="> 16-row QKV: rotary + KV write in the tiled GEMM epilogue")
    VWA_GEMM_P8: Optional[str] = Field(None, description="DIAGNOSTIC: 256x256 8-phase GEMM eligibility override")
    VWA_GEMM_SPLIT_FILL: Optional[str] = Field(None, description="DIAGNOSTIC: split-K fill target (% of CUs)")
    VWA_SKINNY_X_SKEW: Optional[str] = Field(None, description="DIAGNOSTIC: LDS X-row skew of the streaming GEMM")
    VWA_ATTN_IMPL: Optional[str] = Field(None, description="DIAGNOSTIC: decode attention implementation")
    VWA_KERNEL_SO: Optional[str] = Field(None, description="DIAGNOSTIC: another build of the kernel library (A/B)")
    VWA_STRICT_NATIVE: bool = Field(False, description="vendor-library fallbacks in the op layer raise (tests, bench)")
    VWA_BENCH_CONCURRENT: int = Field(0, description="bench.py: concurrent sessions (0: the single-session headline)")
    # ---- build
    VWA_FORCE_BUILD: bool = Field(False, description="__graft_entry__.build(): recompile every source")
    VWA_HIPCC_EXTRA: str = Field("", description="extra hipcc flags (experiments)")

    @classmethod
    def from_env(cls) -> "Settings":
        return cls(**{name: knob(name) for name in cls.model_fields})


_TRUE = ("1", "true", "yes", "on")


def _parse(name: str, raw: str) -> Any:
    ann = Settings.model_fields[name].annotation
    raw = raw.strip()
    if ann is bool:
        return raw.lower() in _TRUE
    if ann is int:
        return int(raw) if raw else Settings.model_fields[name].default
    if ann is float:
        return float(raw) if raw else Settings.model_fields[name].default
    return raw


def knob(name: str) -> Any:
    """The typed value of a declared knob: the environment's (parsed with the declared type) or the
    declared default.  Raises KeyError for an undeclared name and ValueError for an unparsable
    value (a bad setting is an error, not a silent default)."""
    field = Settings.model_fields.get(name)
    if field is None:
        raise KeyError(f"undeclared knob {name!r}: add it to utils/env.py Settings")
    raw = os.environ.get(name)
    if raw is None:
        return field.default
    try:
        return _parse(name, raw)
    except ValueError as e:
        raise ValueError(f"{name}={raw!r}: {e}") from e


def settings() -> Settings:
    """A parsed snapshot of every knob (services take one at startup)."""
    return Settings.from_env()
