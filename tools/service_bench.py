"""Product-path latency through the services (VERDICT r3 missing #4): speech end ->
``intent`` frame over WS ``/stream``, with the brain and voice services as separate processes on
the GPU(s) they would get from launch.py and a stub executor.

    python tools/service_bench.py --sessions 1,8 --debounce 0,1000 --commit 0,700 --chain 1,0 --json out.jsonl

Per (chain, debounce, sessions): every session opens ``/stream``, sets the page context, then
streams utterances of ``--audio-s`` seconds of synthetic speech as 60 ms PCM16 packets paced in
real time (a microphone, apps/web/src/App.tsx:279-288), followed by silence packets until the
``intent`` frame arrives.  Reported per utterance:

* speech_end_to_final_ms -- last speech packet sent -> ``transcript_final`` (the VAD endpoint,
  ``--endpoint-ms`` = VWA_ENDPOINT_MS; the final recognition pass runs speculatively from
  ``--spec-ms`` of trailing silence on, so it is normally done by the endpoint);
* final_to_intent_ms -- ``transcript_final`` -> ``intent`` (the debounce, the HTTP hop to the
  brain, the grammar-constrained parse, the reply);
* speech_end_to_intent_ms -- the sum: what a user waits after they stop speaking.

The brain and the voice worker share GPU 0 (launch.py's single-GPU placement) unless
``--brain-gpu`` / ``--voice-gpu`` say otherwise; ``--chain`` toggles the brain's chained decode
launch (VWA_CHAIN), which then runs beside the live ASR kernels.  Random-init weights: the ASR runs
in fixed-work mode (VWA_ASR_TOKENS_PER_S, 4 tokens per second of audio, as bench.py).
"""
import argparse
import asyncio
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "voice_enabled_browser_automation_amd"
from voice_enabled_browser_automation_amd.utils.env import knob  # noqa: E402


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def paused_speech(seconds: float, seed: int, max_pause_ms: float = 650.0, rate: int = 16000) -> np.ndarray:
    """A spoken command with pauses: voiced words of 0.25-0.7 s separated by gaps of 0.1 s to
    ``max_pause_ms`` (the first two >= 300 ms, i.e. longer than the ASR endpoint -- the pauses a
    speaker makes inside one command), ending on a word; silence is a low noise floor."""
    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    out = (rng.standard_normal(n) * 30).astype(np.float64)
    t, words = 0.0, []
    while True:
        w = rng.uniform(0.25, 0.7)
        if t + w > seconds:
            break
        words.append((t, t + w))
        t += w
        lo = 0.3 if len(words) <= 2 else 0.1  # the first two gaps are longer than the endpoint
        g = rng.uniform(lo, max(lo, max_pause_ms / 1000.0))
        if t + g + 0.25 > seconds:
            break
        t += g
    for a, b in words:
        i, j = int(a * rate), int(b * rate)
        seg = synth_speech(b - a, seed=int(rng.integers(1 << 30)), rate=rate)[: j - i].astype(np.float64)
        out[i : i + len(seg)] += seg
    end = int(words[-1][1] * rate)
    return np.clip(out[:end], -32767, 32767).astype(np.int16)


def synth_speech(seconds: float, seed: int, rate: int = 16000) -> np.ndarray:
    """Continuously voiced syllables (amplitude envelope >= 0.35 everywhere: NO pauses -- one
    word's signal for paused_speech, or a pause-free utterance)."""
    rng = np.random.default_rng(seed)
    t = np.arange(int(seconds * rate)) / rate
    f0 = 110 + 30 * np.sin(2 * np.pi * 0.3 * t + rng.uniform(0, 6))
    phase = 2 * np.pi * np.cumsum(f0) / rate
    sig = np.zeros(len(t))
    for k, a in enumerate((1.0, 0.5, 0.25)):
        sig += a * np.sin(phase * (k + 1) + rng.uniform(0, 6))
    env = 0.35 + 0.65 * np.clip(np.sin(2 * np.pi * 4.0 * t + rng.uniform(0, 6)), 0, None) ** 0.5
    sig = sig * env
    sig = sig / (np.abs(sig).max() + 1e-9) * 0.6
    return (sig * 32767).astype(np.int16)


def spawn(module: str, env_extra: dict, log: str) -> subprocess.Popen:
    env = dict(os.environ, **env_extra)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.Popen([sys.executable, "-u", "-m", module], env=env, cwd=ROOT,
                            stdout=open(log, "w"), stderr=subprocess.STDOUT)


async def wait_health(url: str, proc: subprocess.Popen, timeout: float) -> None:
    import aiohttp

    t0 = time.time()
    async with aiohttp.ClientSession() as s:
        while time.time() - t0 < timeout:
            if proc.poll() is not None:
                raise RuntimeError(f"{url}: service exited with {proc.returncode}")
            try:
                async with s.get(url) as r:
                    if r.status == 200:
                        return
            except aiohttp.ClientError:
                pass
            await asyncio.sleep(0.5)
    raise TimeoutError(url)


async def start_stub_executor():
    """/execute stub (the executor service's contract without a browser): {session_id, results}."""
    from aiohttp import web

    async def execute(req):
        body = await req.json()
        return web.json_response({"session_id": body.get("session_id") or "bench",
                                  "results": [{"intent": i, "ok": True} for i in body.get("intents", [])],
                                  "artifacts": {"dir": ""}})

    async def health(_r):
        return web.json_response({"status": "ok", "service": "executor"})

    app = web.Application()
    app.router.add_post("/execute", execute)
    app.router.add_get("/health", health)
    runner = web.AppRunner(app)
    await runner.setup()
    port = free_port()
    await web.TCPSite(runner, "127.0.0.1", port).start()
    return runner, port


async def session(url: str, idx: int, n_utt: int, audio_s: float, out: list, max_pause_ms: float = 0.0,
                  gap_s: float = 1.5) -> None:
    """One microphone: utterances of ``audio_s`` s (``max_pause_ms`` > 0: paused_speech), packets
    sent at the END of their 60 ms (a packet exists only once it is captured: App.tsx:279-288
    sends when >= 60 ms have accumulated), ``gap_s`` of silence between utterances.  Per
    utterance: the first intent frame after the speech end, and every intent frame the utterance
    produced -- more than one, or one before the speech ended, is a split command."""
    import aiohttp

    pkt = 960  # 60 ms at 16 kHz
    silence = np.zeros(pkt, np.int16).tobytes()
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(url, max_msg_size=0) as ws:
            await ws.send_str(json.dumps({"type": "context_update", "payload": {"url": "https://www.bestbuy.com"}}))
            marks: dict = {"intents": [], "finals": []}
            got = asyncio.Event()

            async def reader():
                async for msg in ws:
                    if msg.type != aiohttp.WSMsgType.TEXT:
                        continue
                    f = json.loads(msg.data)
                    now = time.perf_counter()
                    if f["type"] == "transcript_final":
                        marks["finals"].append(now)
                    elif f["type"] == "intent":
                        marks["intents"].append(now)
                        marks["valid"] = isinstance(f.get("payload"), dict) and "intents" in f["payload"]
                        if marks.get("t_end") is not None:
                            got.set()

            rd = asyncio.ensure_future(reader())
            t_next = time.perf_counter()

            async def send_paced(chunk: bytes):
                nonlocal t_next
                t_next += pkt / 16000
                await asyncio.sleep(max(0.0, t_next - time.perf_counter()))  # captured, then sent
                await ws.send_bytes(chunk)

            for u in range(n_utt):
                seed = 1000 * idx + u
                pcm = paused_speech(audio_s, seed, max_pause_ms) if max_pause_ms > 0 else synth_speech(audio_s, seed)
                marks.update(intents=[], finals=[], t_end=None, valid=False)
                got.clear()
                for i in range(0, len(pcm), pkt):
                    await send_paced(pcm[i : i + pkt].tobytes())
                t_end = time.perf_counter()  # the packet holding the last speech samples is sent
                marks["t_end"] = t_end
                if any(t >= t_end for t in marks["intents"]):
                    got.set()
                deadline = t_end + 30.0
                while not got.is_set() and time.perf_counter() < deadline:  # the mic keeps sending silence
                    await send_paced(silence)
                for _ in range(int(gap_s / 0.06)):  # silence between utterances (late split intents land here)
                    await send_paced(silence)
                after = [t for t in marks["intents"] if t >= t_end]
                if after:
                    t_int = after[0]
                    fins = [t for t in marks["finals"] if t <= t_int]
                    fin = fins[-1] if fins else t_int
                    out.append({"session": idx, "utt": u, "valid": marks.get("valid", False),
                                "intent_frames": len(marks["intents"]),
                                "split": len(marks["intents"]) > 1 or len(after) < len(marks["intents"]),
                                "finals": len(marks["finals"]),
                                "speech_end_to_final_ms": (fin - t_end) * 1e3,
                                "final_to_intent_ms": (t_int - fin) * 1e3,
                                "speech_end_to_intent_ms": (t_int - t_end) * 1e3})
                else:
                    out.append({"session": idx, "utt": u, "timeout": True,
                                "intent_frames": len(marks["intents"]), "split": bool(marks["intents"])})
            await ws.send_str(json.dumps({"type": "close"}))
            rd.cancel()


def pct(v, q):
    return round(float(np.percentile(v, q)), 1) if v else None


async def run_matrix(a) -> list:
    import aiohttp

    logs = os.path.join(ROOT, "gpurun_out", "service_bench")
    os.makedirs(logs, exist_ok=True)
    ex_runner, ex_port = await start_stub_executor()
    results = []
    try:
        for chain in a.chain:
            bport = free_port()
            # chain "gate": the shared-GPU deployment of launch.py (round 6) -- the chained launch
            # only while the ASR batcher's busy word is clear (utils/busy_flag.py)
            busy = f"/dev/shm/vwa_bench_busy_{os.getpid()}" if chain == "gate" else ""
            benv = {"VWA_BRAIN_ENGINE": a.brain_engine, "VWA_LLM_MODEL": a.llm, "BRAIN_PORT": str(bport),
                    "VWA_CHAIN": "1" if chain == "gate" else chain, "HIP_VISIBLE_DEVICES": a.brain_gpu,
                    "VWA_MAX_SESSIONS": str(max(a.sessions)), "VWA_DTYPE": a.dtype, "VWA_SHARED_GB": "24"}
            if busy:
                benv["VWA_ASR_BUSY_FILE"] = busy
            brain = spawn(f"{PKG}.brain.server", benv, os.path.join(logs, f"brain_chain{chain}.log"))
            try:
                t0 = time.time()
                await wait_health(f"http://127.0.0.1:{bport}/health", brain, a.load_timeout)
                brain_load_s = time.time() - t0
                for deb, commit in [(d, c) for d in a.debounce for c in a.commit]:
                    vport = free_port()
                    venv = {"VWA_ASR_ENGINE": a.asr_engine, "VWA_ASR_MODEL": a.asr, "VOICE_PORT": str(vport),
                            "BRAIN_URL": f"http://127.0.0.1:{bport}/parse",
                            "EXECUTOR_URL": f"http://127.0.0.1:{ex_port}", "VWA_DEBOUNCE_MS": deb,
                            "HIP_VISIBLE_DEVICES": a.voice_gpu, "VWA_MAX_SESSIONS": str(max(a.sessions)),
                            "VWA_ASR_TOKENS_PER_S": str(a.asr_tokens_per_s),
                            "VWA_ENDPOINT_MS": str(a.endpoint_ms), "VWA_SPEC_FINAL_MS": str(a.spec_ms),
                            "VWA_COMMIT_MS": str(commit), "VWA_SPEC_BRAIN": a.spec_brain}
                    if busy:
                        venv["VWA_ASR_BUSY_FILE"] = busy
                    if a.brain_gpu == a.voice_gpu:  # (launch.py's shared-GPU rule for the ASR)
                        from voice_enabled_browser_automation_amd.launch import shared_voice_env

                        venv.update(shared_voice_env(os.environ, benv))
                    voice = spawn(f"{PKG}.voice.server", venv,
                                  os.path.join(logs, f"voice_chain{chain}_deb{deb}_commit{commit}.log"))
                    try:
                        await wait_health(f"http://127.0.0.1:{vport}/health", voice, a.load_timeout)
                        url = f"http://127.0.0.1:{vport}/stream"
                        # warm-up: one utterance (graph captures, prefix cache of the prompt head)
                        await session(url, 99, 1, a.audio_s, [], a.max_pause_ms)
                        for n in a.sessions:
                            out: list = []
                            t0 = time.perf_counter()
                            await asyncio.gather(*(session(url, i, a.utterances, a.audio_s, out, a.max_pause_ms)
                                                   for i in range(n)))
                            wall = time.perf_counter() - t0
                            ok = [r for r in out if not r.get("timeout")]
                            e2i = [r["speech_end_to_intent_ms"] for r in ok]
                            rec = {"what": "service_latency", "chain": chain, "debounce_ms": float(deb),
                                   "commit_ms": float(commit), "spec_brain": a.spec_brain, "sessions": n,
                                   "speech": f"paused (<= {a.max_pause_ms:g} ms gaps)" if a.max_pause_ms > 0
                                   else "continuous", "packet_timing": "end of packet",
                                   "utterances": len(out), "timeouts": len(out) - len(ok),
                                   "split_commands": sum(bool(r.get("split")) for r in out),
                                   "intent_frames": sum(r.get("intent_frames", 0) for r in out),
                                   "asr_finals_per_utterance": pct([r["finals"] for r in ok], 50),
                                   "valid_intents": f"{sum(r['valid'] for r in ok)}/{len(out)}",
                                   "audio_s": a.audio_s, "asr": a.asr, "llm": a.llm, "dtype": a.dtype,
                                   "endpoint_ms": a.endpoint_ms, "spec_final_ms": a.spec_ms,
                                   "speech_end_to_intent_p50_ms": pct(e2i, 50),
                                   "speech_end_to_intent_p95_ms": pct(e2i, 95),
                                   "speech_end_to_final_p50_ms": pct([r["speech_end_to_final_ms"] for r in ok], 50),
                                   "final_to_intent_p50_ms": pct([r["final_to_intent_ms"] for r in ok], 50),
                                   "final_to_intent_p95_ms": pct([r["final_to_intent_ms"] for r in ok], 95),
                                   "wall_s": round(wall, 2), "brain_load_s": round(brain_load_s, 1)}
                            async with aiohttp.ClientSession() as s:
                                async with s.get(f"http://127.0.0.1:{bport}/metrics") as r:
                                    bm = await r.json()
                            eng = bm.get("engine", {})
                            rec["brain_chain_fallbacks"] = eng.get("chain_fallbacks", 0)
                            rec["brain_rows_per_iteration"] = eng.get("rows_per_iteration")
                            rec["brain_chained_steps"] = eng.get("chained_steps", 0)
                            rec["brain_gated_steps"] = eng.get("gated_steps", 0)
                            rec["brain_steps"] = eng.get("steps", 0)
                            rec["brain_host_ms"] = eng.get("host_ms")
                            print(json.dumps(rec), flush=True)
                            results.append(rec)
                    finally:
                        voice.terminate()
                        voice.wait(timeout=30)
            finally:
                brain.terminate()
                brain.wait(timeout=60)
    finally:
        await ex_runner.cleanup()
    return results


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", default="1,8")
    ap.add_argument("--debounce", default="0,1000")
    ap.add_argument("--commit", default="0", help="voice VWA_COMMIT_MS values (silence that ends a command)")
    ap.add_argument("--spec-brain", default="1", help="voice VWA_SPEC_BRAIN")
    ap.add_argument("--max-pause-ms", type=float, default=650.0,
                    help="paused speech: longest pause inside a command (0: continuous speech, round 5's)")
    ap.add_argument("--chain", default="gate",
                    help="brain VWA_CHAIN: 1, 0, or gate (the single-GPU deployment: chained while the ASR is idle)")
    ap.add_argument("--utterances", type=int, default=20, help="utterances per session per point")
    ap.add_argument("--endpoint-ms", type=float, default=knob("VWA_ENDPOINT_MS"))
    ap.add_argument("--spec-ms", type=float, default=knob("VWA_SPEC_FINAL_MS"))
    ap.add_argument("--audio-s", type=float, default=5.0)
    ap.add_argument("--asr", default="whisper-tiny")
    ap.add_argument("--asr-engine", default="whisper")
    ap.add_argument("--asr-tokens-per-s", type=float, default=4.0)
    ap.add_argument("--llm", default="llama3-8b")
    ap.add_argument("--brain-engine", default="llm")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--brain-gpu", default="0")
    ap.add_argument("--voice-gpu", default="0")
    ap.add_argument("--load-timeout", type=float, default=600)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    a.sessions = [int(x) for x in a.sessions.split(",")]
    a.debounce = a.debounce.split(",")
    a.commit = a.commit.split(",")
    a.chain = a.chain.split(",")
    res = asyncio.run(run_matrix(a))
    if a.json:
        with open(a.json, "a") as f:
            for r in res:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
