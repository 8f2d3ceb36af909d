"""Headline benchmark: voice-to-intent p50 latency (ms) + ASR RTF, 10 s utterance, Llama-3-8B brain.

One step = one voice command end to end on the on-node engines:
    10 s PCM16 16 kHz utterance -> pcm16->f32 (HIP) -> Whisper log-mel (HIP) -> encoder -> greedy
    decode of the transcript (fixed work: 4 text tokens per second of audio) -> ParseRequest
    {text: transcript, context} -> Llama-3-8B intent parse (prefix-cached prompt, grammar-
    constrained + jump-forward decoding, <= 512 output chars) -> ParseResponse validation.

This replaces the reference path Deepgram STT -> 1 s debounce -> OpenAI JSON mode
(apps/voice/src/server.ts:111-231, apps/brain/src/server.ts:89-139).  `value` is the p50
ENGINE latency (audio fully received -> validated intent); `parity_p50_ms` adds the
reference's fixed 1000 ms debounce (apps/voice/src/server.ts:229).

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling -- every rank serves its own
voice sessions (ASR data-parallel, one LLM replica per rank), or with --tp every TP group serves
them through the served control plane (brain/tp_engine.TPIntentEngine: the group leader runs the
sessions, its peers follow the leader's scheduler iterations in lockstep); the reported p50 is
over ALL sessions of all ranks / groups.

Data: synthetic speech-like audio, random-init weights of the named architectures.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time
import zlib

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.asr.engine import AsrEngine  # noqa: E402
from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine  # noqa: E402
from voice_enabled_browser_automation_amd.brain.prompt import COMMANDS  # noqa: E402
from voice_enabled_browser_automation_amd.brain.tp_engine import TPIntentEngine  # noqa: E402
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import get_config  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel  # noqa: E402
from voice_enabled_browser_automation_amd.parallel.tp import init_distributed  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer  # noqa: E402
from voice_enabled_browser_automation_amd.utils.env import knob  # noqa: E402

METRIC = "voice-to-intent p50 latency (ms) + ASR RTF; 10s utterance; Llama-3-8B brain"


def synth_speech(seconds: float, seed: int, rate: int = 16000) -> np.ndarray:
    """Speech-like PCM16: voiced segments (f0 + 3 formants, syllable-rate AM) and pauses."""
    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    t = np.arange(n) / rate
    f0 = 110 + 30 * np.sin(2 * np.pi * 0.3 * t + rng.uniform(0, 6))
    phase = 2 * np.pi * np.cumsum(f0) / rate
    sig = np.zeros(n)
    for k, (f, a) in enumerate(((700, 1.0), (1200, 0.5), (2600, 0.25))):
        sig += a * np.sin(phase * (k + 1) + rng.uniform(0, 6)) * (1 + 0.3 * np.sin(2 * np.pi * f / 400 * t))
    env = np.clip(np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 6)), 0, None) ** 0.5
    words = (np.sin(2 * np.pi * 0.7 * t + rng.uniform(0, 6)) > -0.6).astype(float)
    sig = sig * env * words + 0.02 * rng.standard_normal(n)
    sig = sig / (np.abs(sig).max() + 1e-9) * 0.6
    return (sig * 32767).astype(np.int16)


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def drive_sessions(brain, tp, world: int, n: int, one, start: int = 0):
    """Run n voice commands through ``one(i)`` between world barriers, as the served deployment
    does: without TP every rank runs its own; with TP (``brain`` a TPIntentEngine) the group
    leader runs them and its peers follow the leader's scheduler iterations in lockstep
    (``worker_loop``) until the leader stops the group.  -> (results of the leader / every DP
    rank, wall-clock ms between the barriers)."""
    follower = tp.size > 1 and tp.rank != 0
    _sync()
    if world > 1:
        torch.distributed.barrier()
    _sync()
    t0 = time.perf_counter()
    out = []
    if follower:
        brain.worker_loop()
    else:
        for i in range(n):
            out.append(one(start + i))
        if tp.size > 1:
            brain.stop()
    _sync()
    if world > 1:
        torch.distributed.barrier()
    _sync()
    return out, (time.perf_counter() - t0) * 1e3


def gather(obj, world: int):
    """Every rank's object (rank order); followers contribute empty results."""
    if world == 1:
        return [obj]
    out = [None] * world
    torch.distributed.all_gather_object(out, obj)
    return out


def run_concurrent(args, C, asr, brain, utterances, asr_tokens, world, tp):
    """C voice sessions arriving together on every rank: one batched ASR pass, then all C intent
    parses decoded with continuous batching.  Per-session latency = ASR batch + that session's
    parse completion.  Not part of the headline value."""
    asr_ms = []

    def round_(k):
        pcms = [utterances[(k * C + j) % len(utterances)] for j in range(C)]
        t0 = time.perf_counter()
        texts = asr.transcribe_many([asr.pcm_to_audio(p) for p in pcms], exact_tokens=asr_tokens)
        t_asr = (time.perf_counter() - t0) * 1e3
        asr_ms.append(t_asr)
        reqs = [{"text": t if t.strip() else COMMANDS[j % len(COMMANDS)], "context": {"url": "https://www.bestbuy.com"}}
                for j, t in enumerate(texts)]
        outs = brain.parse_many(reqs)
        ok = sum(safe_parse(ParseResponse, o).success for o in outs)
        return [t_asr + b["latency_ms"] for b in brain.last_batch], ok

    drive_sessions(brain, tp, world, 1, round_)  # warm-up round
    it0 = dict(brain.batch_stats)
    tm0 = dict(getattr(brain, "timing", {}))
    asr_ms.clear()
    rounds, el = drive_sessions(brain, tp, world, args.steps, round_, start=1)
    lat = [x for l, _o in rounds for x in l]
    ok = sum(o for _l, o in rounds)
    bs = {k: brain.batch_stats[k] - it0.get(k, 0) for k in ("iterations", "rows", "sampled")}
    allr = gather({"el": el, "ok": ok, "lat": lat}, world)
    all_lat = [x for a in allr for x in a["lat"]]
    el_max = max(a["el"] for a in allr)
    return {"sessions_per_rank": C, "p50_ms": round(statistics.median(all_lat), 3),
            "p90_ms": round(float(np.percentile(all_lat, 90)), 3),
            "throughput_utt_per_s": round(len(all_lat) / (el_max / 1e3), 3),
            "valid_intents": f"{sum(a['ok'] for a in allr)}/{len(all_lat)}",
            "rows_per_iteration": round(bs["rows"] / max(1, bs["iterations"]), 2),
            "samples_per_iteration": round(bs["sampled"] / max(1, bs["iterations"]), 2),
            "iterations_per_round": round(bs["iterations"] / max(1, args.steps), 1),
            "asr_batch_ms_mean": round(statistics.mean(asr_ms), 2) if asr_ms else None,
            # per scheduler iteration, host-side clock (ms): launch of the step, grammar masks
            # (overlapping the GPU), head + sampler launch, waiting for the tokens, accept / jump-forward
            "iteration_ms": {k: round((v - tm0.get(k, 0.0)) / max(1, bs["iterations"]), 3)
                             for k, v in getattr(brain, "timing", {}).items()}}


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without torchrun: run N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code.  Runs before this process
    touches the GPU (torch.cuda.device_count() does not initialise it)."""
    import subprocess

    have = torch.cuda.device_count()
    if have < n:
        raise SystemExit(f"bench.py --gpus {n}: only {have} GPU(s) visible -- refusing to time fewer GPUs "
                         f"than requested (one rank per GPU over RCCL)")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    # strict native mode: an op that would fall back to a vendor library raises (ops.vendor_fallback)
    os.environ.setdefault("VWA_STRICT_NATIVE", "1")
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--asr", default=knob("VWA_ASR_MODEL"))
    ap.add_argument("--llm", default=knob("VWA_LLM_MODEL"))
    ap.add_argument("--tp", type=int, default=knob("VWA_TP"))
    ap.add_argument("--audio-s", type=float, default=10.0)
    ap.add_argument("--asr-tokens-per-s", type=float, default=4.0)
    ap.add_argument("--budget-chars", type=int, default=512)
    ap.add_argument("--debounce-ms", type=float, default=1000.0, help="reference debounce added for parity_p50_ms")
    ap.add_argument("--concurrent", type=int, default=knob("VWA_BENCH_CONCURRENT"),
                    help="also measure C concurrent voice sessions per rank (batched ASR + continuous-batched "
                         "intent decoding); reported under 'concurrent', outside the headline value")
    ap.add_argument("--dtype", default=knob("VWA_DTYPE"), choices=("bf16", "fp8"),
                    help="LLM weight dtype: bf16 (headline config) or fp8 (W8A8 on the fp8 MFMA, config 5)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={env_world}: one rank per GPU expected")

    tp = init_distributed(tp_size=args.tp if int(os.environ.get("WORLD_SIZE", "1")) > 1 else None)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU (MI355X)")
    if (knob("VWA_DIST_BACKEND") or "nccl") != "nccl":
        local = local % torch.cuda.device_count()  # gloo rehearsal on fewer GPUs than ranks
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ops.ext()  # native kernels are mandatory
    use_graphs = not args.no_graphs

    t_load = time.time()
    wcfg, lcfg = get_config(args.asr), get_config(args.llm)
    whisper = WhisperModel(wcfg, device=dev, seed=1)
    C = max(0, args.concurrent)
    asr = AsrEngine(whisper, load_tokenizer("whisper"), max_sessions=max(2, C), use_graphs=use_graphs)
    llama = LlamaModel(lcfg, device=dev, tp=tp, seed=2, wdtype=args.dtype)
    engine = LLMEngine(llama, max_seqs=max(4, C), max_model_len=2048, use_graphs=use_graphs)
    brain = LLMIntentEngine(engine, load_tokenizer("llama3"), budget_chars=args.budget_chars, temperature=0.1,
                            seed=1234)  # every replica does the same work (weak scaling; TP lockstep)
    engine.capture_all()
    if tp.size > 1:  # the served TP control plane (brain/server.py uses the same engine)
        brain = TPIntentEngine(brain, tp)
    torch.cuda.synchronize()
    load_s = time.time() - t_load

    asr_tokens = int(math.ceil(args.audio_s * args.asr_tokens_per_s))
    # the same utterances on every rank: a DP replica's work per step is then exactly the 1-GPU
    # work (weak scaling measures interference, not a different mix of transcripts / intent
    # lengths), and the ranks of a TP group decode in lockstep
    utterances = [synth_speech(args.audio_s, seed=i) for i in range(8)]

    last = {}

    def one(i: int):
        pcm = utterances[i % len(utterances)]
        t0 = time.perf_counter()
        audio = asr.pcm_to_audio(pcm)
        text = asr.transcribe(audio, exact_tokens=asr_tokens)
        t_asr = time.perf_counter()
        cmd = COMMANDS[i % len(COMMANDS)]
        req = {"text": text if text.strip() else cmd, "context": {"url": "https://www.bestbuy.com"}}
        out = brain.parse(req)
        ok = safe_parse(ParseResponse, out).success
        t1 = time.perf_counter()
        last["text"], last["out"] = text, out
        return (t1 - t0) * 1e3, (t_asr - t0) * 1e3, ok

    drive_sessions(brain, tp, world, args.warmup, one)
    tm0, it0 = dict(brain.timing), brain.batch_stats["iterations"]

    def timed_one(i):
        r = one(i)
        stats = dict(brain.last_stats)
        if args.verbose and rank == 0:
            # (crc32 of the transcript and of the intent JSON: run-to-run reproducibility checks)
            print(json.dumps({"step": i - args.warmup, "latency_ms": round(r[0], 2), "asr_ms": round(r[1], 2),
                              "text_crc": zlib.crc32(str(last.get("text")).encode()),
                              "out_crc": zlib.crc32(str(last.get("out")).encode()), **stats}), flush=True)
        return r + (stats,)

    res_steps, elapsed = drive_sessions(brain, tp, world, args.steps, timed_one, start=args.warmup)
    lat = [r[0] for r in res_steps]
    asr_ms = [r[1] for r in res_steps]
    oks = [r[2] for r in res_steps]
    llm_stats = [r[3] for r in res_steps]
    n_it = max(1, brain.batch_stats["iterations"] - it0)
    host_us = {k.replace("_ms", "_us"): round((brain.timing[k] - tm0[k]) * 1e3 / n_it, 1) for k in tm0}

    conc = run_concurrent(args, C, asr, brain, utterances, asr_tokens, world, tp) if C > 1 else None

    # gather every session's latency across ranks (weak scaling: p50 over all sessions; TP
    # followers ran no sessions of their own)
    allr = gather({"el": elapsed, "lat": lat, "asr": asr_ms, "ok": int(sum(oks))}, world)
    # evidence that the collective backend really saw every rank on its own GPU
    rccl_world, n_devices, backend = 1, 1, None
    if world > 1:
        backend = str(torch.distributed.get_backend())
        rccl_world = torch.distributed.get_world_size()
        pr = torch.cuda.get_device_properties(dev)
        ident = torch.tensor([float(pr.pci_domain_id), float(pr.pci_bus_id), float(pr.pci_device_id)],
                             dtype=torch.float64, device=dev)
        ids = [torch.zeros_like(ident) for _ in range(world)]
        torch.distributed.all_gather(ids, ident)
        n_devices = len({tuple(a.tolist()) for a in ids})
    K = args.steps
    elapsed_max = max(a["el"] for a in allr)
    all_lat = [x for a in allr for x in a["lat"]]
    all_asr = [x for a in allr for x in a["asr"]]
    n_ok = sum(a["ok"] for a in allr)
    if rank == 0:
        p50 = statistics.median(all_lat)
        rtf = statistics.median(all_asr) / (args.audio_s * 1e3)
        dec = [s.get("decode_steps", 0) for s in llm_stats]
        res = {
            "metric": METRIC,
            "value": round(p50, 3),
            "unit": "ms",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / K, 3),
            "higher_is_better": False,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic 16 kHz speech-like audio, random-init weights",
            "config": {"model": f"{args.asr} + {args.llm}", "global_batch": world // tp.size, "seq_len": None,
                       "parallelism": f"dp{world // tp.size}" + (f"-tp{tp.size}" if tp.size > 1 else ""),
                       "audio_s": args.audio_s, "asr_tokens": asr_tokens, "budget_chars": args.budget_chars,
                       "hipgraph": use_graphs},
            "asr_rtf": round(rtf, 5),
            "p90_ms": round(float(np.percentile(all_lat, 90)), 3),
            "parity_p50_ms": round(p50 + args.debounce_ms, 3),
            "asr_p50_ms": round(statistics.median(all_asr), 3),
            "llm_p50_ms": round(statistics.median([a - b for a, b in zip(all_lat, all_asr)]), 3),
            "llm_decode_steps_mean": round(sum(dec) / max(1, len(dec)), 2),
            "llm_forced_tokens_mean": round(sum(s.get("forced_tokens", 0) for s in llm_stats) / max(1, K), 2),
            "llm_prefill_tokens_mean": round(sum(s.get("prefill_tokens", 0) for s in llm_stats) / max(1, K), 2),
            "valid_intents": f"{n_ok}/{len(all_lat)}",
            "decode_iteration_host_us": host_us,
            "throughput_utt_per_s": round(len(all_lat) / (elapsed_max / 1e3), 3),
            "load_s": round(load_s, 1),
            "rccl_world": rccl_world,
            "distinct_devices": n_devices,
            "dist_backend": backend,
            "tp": tp.size,
        }
        if conc is not None:
            res["concurrent"] = conc
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
