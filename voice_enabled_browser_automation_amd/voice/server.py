"""Voice service: ``GET /health``, ``GET /metrics``, WebSocket ``/stream`` (parity with
apps/voice/src/server.ts:60-304).

Per connection:
  * binary frames = raw PCM16 LE 16 kHz mono -> on-node streaming ASR (asr/streaming.py) ->
    ``transcript_partial`` / ``transcript_final`` frames carrying Deepgram-shaped payloads;
  * final transcripts are aggregated and debounced (``VWA_DEBOUNCE_MS``, reference fixed 1000 ms:
    :229) before ``POST BRAIN_URL`` {text, context};
  * commit policy for pauses (the reference only merges finals that land inside its debounce):
    the recognizer's VAD events (``SpeechStarted``) hold the pending text while the user speaks
    again -- a pause longer than the ASR endpoint is not a command boundary until ``VWA_COMMIT_MS``
    of silence have passed since the speech end; the brain is started SPECULATIVELY on the
    speculative final pass (``VWA_SPEC_BRAIN``), so its latency hides in the endpoint / commit
    wait, and its answer is used only if the committed text is exactly the text it parsed (and
    the context did not change meanwhile) -- otherwise it is dropped and the merged text parsed;
  * brain reply -> ``intent`` frame, ``tts`` frame (tts_summary), context merge of
    ``context_updates``, safe/risky split: safe intents go to ``POST EXECUTOR_URL/execute`` with
    the connection's executor session id (``execution_result`` / ``execution_error``), risky
    ones produce ``confirmation_required``;
  * JSON control frames: ``{"type":"close"}``, ``{"type":"context_update","payload":{...}}``,
    and ``{"type":"flush"}`` (end of utterance: finalise without waiting for silence).

Races of the reference fixed here: brain calls of one connection are serialised
by a per-connection lock (context updates apply in utterance order), and its executor calls run
one at a time from a per-connection queue, so the executor session id is assigned in order; sends
after a client disconnect are dropped.  As in the reference (server.ts:186-224) the execution is
NOT awaited on the brain path: ``intent``, ``tts`` and ``confirmation_required`` go out as soon as
the brain answers, and the next utterance's brain call does not wait for a browser run.
"""
from __future__ import annotations

import asyncio
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, Optional

import aiohttp
from aiohttp import WSMsgType, web

from ..utils.context import merge_context
from ..utils.metrics import Metrics
from ..utils.env import knob

VERSION = "0.1.0"


async def post_json_and_return(session: aiohttp.ClientSession, url: str, body: Any) -> Any:
    """postJsonAndReturn parity (apps/voice/src/server.ts:15-52): non-JSON reply -> {ok: False}."""
    async with session.post(url, json=body) as resp:
        text = await resp.text()
    try:
        return json.loads(text)
    except ValueError:
        return {"ok": False}


def build_app(asr_factory: Optional[Callable[[], Any]] = None, *, brain_url: Optional[str] = None,
              executor_url: Optional[str] = None, debounce_ms: Optional[float] = None,
              commit_ms: Optional[float] = None, spec_brain: Optional[bool] = None) -> web.Application:
    """asr_factory() -> a StreamingAsrSession-like object (push(bytes)->events, flush()->events);
    None = passthrough mode (no recognizer, as the reference without DEEPGRAM_API_KEY)."""
    app = web.Application()
    app["metrics"] = Metrics("voice")
    app["live"] = 0  # open /stream sessions (reported to the DP router's metrics gather)
    # one worker per live session pass: a session's recognition pass blocks its worker inside the
    # recognizer (asr/streaming.py AsrBatcher), whose single scheduler thread batches the passes
    # of all sessions onto the GPU -- so the pool only needs to be as wide as the session count
    app["asr_pool"] = ThreadPoolExecutor(max_workers=knob("VWA_MAX_SESSIONS") + 4,
                                         thread_name_prefix="asr")
    app["asr_factory"] = asr_factory
    app["exec_tasks"] = set()  # executor queues still draining after their connection closed
    brain_url = brain_url or knob("BRAIN_URL")
    executor_url = executor_url or knob("EXECUTOR_URL")
    if debounce_ms is None:
        debounce_ms = knob("VWA_DEBOUNCE_MS")
    commit_ms = knob("VWA_COMMIT_MS") if commit_ms is None else commit_ms
    spec_brain = knob("VWA_SPEC_BRAIN") if spec_brain is None else spec_brain
    # the ASR final fires endpoint_ms after the speech end: the commit window's rest comes after it
    hold_s = max(debounce_ms, commit_ms - knob("VWA_ENDPOINT_MS")) / 1000.0

    async def on_startup(app_):
        app_["http"] = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=120))

    async def on_cleanup(app_):
        for t in list(app_["exec_tasks"]):
            t.cancel()
        await app_["http"].close()
        app_["asr_pool"].shutdown(wait=False)

    app.on_startup.append(on_startup)
    app.on_cleanup.append(on_cleanup)

    async def health(_req):
        return web.json_response({"status": "ok", "service": "voice", "version": VERSION})

    async def metrics(_req):
        snap = app["metrics"].snapshot()
        batcher = getattr(asr_factory, "batcher", None)
        if batcher is not None:  # cross-session ASR batching: passes per GPU batch
            snap["asr_batcher"] = dict(batcher.stats, rows_per_batch=round(batcher.rows_per_batch(), 3),
                                       queue_depth=batcher.queue_depth())
        snap["live_sessions"] = app["live"]
        return web.json_response(snap)

    async def stream(req: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse()
        await ws.prepare(req)
        m: Metrics = app["metrics"]
        m.inc("connections")
        loop = asyncio.get_running_loop()
        # per-utterance span (monotonic): first audio -> final transcript -> brain reply
        # pending: final text not yet sent to the brain; spec: a speculative brain call {text, ctx,
        # task}; ctx: context version (a speculative answer is only used for the context it saw)
        st: Dict[str, Any] = {"context": {}, "pending": "", "debounce": None, "session_id": None, "closed": False,
                              "t_final": None, "t_utt": None, "spec": None, "ctx": 0, "procs": set()}
        lock = asyncio.Lock()

        async def send(obj):
            if st["closed"] or ws.closed:
                return
            try:
                await ws.send_str(json.dumps(obj))
            except (ConnectionResetError, RuntimeError):
                st["closed"] = True

        # connection-state frames as the reference sends them for its Deepgram socket
        # (apps/voice/src/server.ts:233-250): "deepgram_connected" once the recognizer exists, then
        # the recognizer's own state events {state: open|close|error, info}; a recognizer that
        # cannot be created -> error "deepgram_connect_failed" and the connection stays up
        # without transcription (as the reference, whose audio then goes nowhere)
        asr = None
        if asr_factory is not None:
            try:
                asr = asr_factory()
            except Exception as e:  # noqa: BLE001
                print(f"[voice] recognizer start failed: {e}", flush=True)
                m.inc("asr_connect_failed")
                await send({"type": "error", "payload": "deepgram_connect_failed"})
            else:
                await send({"type": "info", "payload": "deepgram_connected"})
                await send({"type": "info", "payload": {"state": "open"}})
                if hasattr(asr, "vad_events"):
                    asr.vad_events = True
                    asr.on_speculative = lambda text: loop.call_soon_threadsafe(on_speculative_final, text)
        else:
            await send({"type": "warn", "payload": "no_api_key; running in passthrough"})

        async def asr_call(fn, *a):
            """One recognizer call on the worker pool; an engine failure is reported as the
            reference reports a Deepgram socket error ({state: "error", info}) and the session
            continues (the next audio retries)."""
            try:
                return await loop.run_in_executor(app["asr_pool"], fn, *a)
            except Exception as e:  # noqa: BLE001
                m.inc("asr_errors")
                await send({"type": "info", "payload": {"state": "error", "info": str(e) or e.__class__.__name__}})
                return []

        async def run_executor(safe):
            try:
                resp = await post_json_and_return(app["http"], f"{executor_url}/execute",
                                                  {**({"session_id": st["session_id"]} if st["session_id"] else {}),
                                                   "intents": safe})
                st["session_id"] = resp.get("session_id", st["session_id"]) if isinstance(resp, dict) else st["session_id"]
                await send({"type": "execution_result",
                            "payload": f"Executed {len(safe)} actions successfully. Session: {st['session_id']}"})
                m.inc("executions")
            except Exception as e:  # noqa: BLE001
                await send({"type": "execution_error", "payload": f"Execution failed: {e}"})
                m.inc("execution_errors")

        # executor calls of this connection, in order, off the brain path (the reference fires
        # /execute without awaiting it, server.ts:186-219; one at a time here so session ids chain)
        exec_q: asyncio.Queue = asyncio.Queue()

        async def exec_worker():
            while True:
                safe = await exec_q.get()
                if safe is None:
                    return
                await run_executor(safe)

        exec_task = asyncio.ensure_future(exec_worker())

        async def call_brain(text: str):
            """One /parse call (serialised per connection: context updates apply in order)."""
            async with lock:
                t0 = time.perf_counter()
                try:
                    resp = await post_json_and_return(app["http"], brain_url, {"text": text, "context": st["context"]})
                except Exception as e:  # noqa: BLE001
                    m.inc("brain_errors")
                    print(f"[voice] brain post failed: {e}", flush=True)
                    return None
                m.observe("brain_ms", (time.perf_counter() - t0) * 1e3)
                return resp

        async def process(combined: str):
            """Commit one command: the speculative answer if it parsed exactly this text under the
            current context, else a fresh brain call; then deliver it."""
            sp, st["spec"] = st["spec"], None
            if sp is not None and sp["text"] == combined and sp["ctx"] == st["ctx"]:
                resp = await sp["task"]
                m.inc("spec_brain_used")
                if resp is None:
                    resp = await call_brain(combined)
            else:
                if sp is not None:
                    m.inc("spec_brain_dropped")
                resp = await call_brain(combined)
            if resp is not None:
                await deliver(resp)

        async def deliver(resp):
            async with lock:
                await send({"type": "intent", "payload": resp})
                now = time.perf_counter()
                m.inc("commands")
                if st["t_final"] is not None:
                    m.observe("final_to_intent_ms", (now - st["t_final"]) * 1e3)
                if st["t_utt"] is not None:
                    m.observe("utterance_to_intent_ms", (now - st["t_utt"]) * 1e3)
                    st["t_utt"] = None
                if isinstance(resp, dict) and resp.get("tts_summary"):
                    await send({"type": "tts", "payload": resp["tts_summary"]})
                if isinstance(resp, dict) and isinstance(resp.get("context_updates"), dict):
                    st["context"] = merge_context(st["context"], resp["context_updates"])
                    st["ctx"] += 1
                intents = resp.get("intents") if isinstance(resp, dict) else None
                if isinstance(intents, list):
                    safe = [i for i in intents if not (isinstance(i, dict) and i.get("requires_confirmation"))]
                    risky = [i for i in intents if isinstance(i, dict) and i.get("requires_confirmation")]
                    if safe:
                        exec_q.put_nowait(safe)
                    if risky:
                        await send({"type": "confirmation_required",
                                    "payload": f"{len(risky)} risky actions require manual confirmation"})

        async def debounced():
            try:
                await asyncio.sleep(hold_s)
            except asyncio.CancelledError:
                return
            combined = st["pending"].strip()
            st["pending"] = ""
            st["debounce"] = None
            if combined:
                await process(combined)

        def start_debounce():
            t = asyncio.ensure_future(debounced())
            st["debounce"] = t
            st["procs"].add(t)  # (tracked until done: a disconnect lets a committing call finish)
            t.add_done_callback(st["procs"].discard)

        def on_speculative_final(text: str):
            """The ASR's speculative final pass finished (the user has been silent for
            VWA_SPEC_FINAL_MS): parse pending + it now, commit later (process)."""
            text = (text or "").strip()
            if not spec_brain or not text or st["closed"]:
                return
            cand = f"{st['pending']} {text}" if st["pending"] else text
            sp = st["spec"]
            if sp is not None and sp["text"] == cand and sp["ctx"] == st["ctx"]:
                return
            m.inc("spec_brain_started")
            st["spec"] = {"text": cand, "ctx": st["ctx"], "task": asyncio.ensure_future(call_brain(cand))}

        async def handle_events(events):
            for ev in events:
                if ev.get("type") == "SpeechStarted":
                    # the user speaks (again): nothing pending is a finished command yet
                    if st["debounce"] is not None:
                        st["debounce"].cancel()
                        st["debounce"] = None
                        m.inc("commits_held")
                    continue
                is_final = bool(ev.get("is_final") or (ev.get("channel") or {}).get("is_final"))
                await send({"type": "transcript_final" if is_final else "transcript_partial", "payload": ev})
                if not is_final:
                    continue
                alt = ((ev.get("channel") or {}).get("alternatives") or [{}])[0]
                text = (alt.get("transcript") or "").strip()
                if not text:
                    continue
                m.inc("finals")
                st["t_final"] = time.perf_counter()
                if st["t_utt"] is not None:
                    m.observe("speech_to_final_ms", (st["t_final"] - st["t_utt"]) * 1e3)
                st["pending"] = f"{st['pending']} {text}" if st["pending"] else text
                if st["debounce"] is not None:
                    st["debounce"].cancel()
                start_debounce()

        app["live"] += 1
        try:
            async for msg in ws:
                if msg.type == WSMsgType.BINARY:
                    m.inc("audio_frames")
                    if st["t_utt"] is None:
                        st["t_utt"] = time.perf_counter()
                    if asr is not None:
                        t_push = time.perf_counter()
                        events = await asr_call(asr.push, msg.data)
                        dt = time.perf_counter() - t_push
                        m.observe("asr_push_ms", dt * 1e3)
                        # a recognition pass ran: real-time factor = pass time over the seconds of
                        # audio that pass recognised (the utterance buffer it covered)
                        covered = max((float(ev.get("duration") or 0.0) for ev in events), default=0.0)
                        if covered > 0:
                            m.observe("asr_rtf", dt / covered)
                        await handle_events(events)
                elif msg.type == WSMsgType.TEXT:
                    try:
                        ctl = json.loads(msg.data)
                    except ValueError:
                        continue
                    if not isinstance(ctl, dict):
                        continue
                    if ctl.get("type") == "close":
                        await ws.close()
                        break
                    if ctl.get("type") == "context_update" and isinstance(ctl.get("payload"), dict):
                        st["context"] = merge_context(st["context"], ctl["payload"])
                        st["ctx"] += 1
                    elif ctl.get("type") == "flush" and asr is not None:
                        events = await asr_call(asr.flush)
                        await handle_events(events)
                elif msg.type in (WSMsgType.ERROR, WSMsgType.CLOSE):
                    break
        finally:
            app["live"] -= 1
            st["closed"] = True
            if st["debounce"] is not None:
                st["debounce"].cancel()  # (still sleeping: a command nobody finished saying)
            if asr is not None and hasattr(asr, "close"):
                asr.close()
            # queued executions still run (the reference's fire-and-forget promises do); their
            # frames are dropped once the socket is closed.  A command already committing (its
            # brain call in flight) still enqueues its safe intents: the sentinel goes in after it
            # (ADVICE r5 -- enqueued behind the sentinel they were silently dropped)
            inflight = [t for t in st["procs"] if not t.done()]

            async def close_exec():
                if inflight:
                    await asyncio.gather(*inflight, return_exceptions=True)
                exec_q.put_nowait(None)

            closer = asyncio.ensure_future(close_exec())
            for t in (closer, exec_task):
                app["exec_tasks"].add(t)
                t.add_done_callback(app["exec_tasks"].discard)
        return ws

    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics)
    app.router.add_get("/stream", stream)
    return app


def asr_factory_from_env() -> Optional[Callable[[], Any]]:
    kind = knob("VWA_ASR_ENGINE")
    if kind == "none":
        return None
    import torch

    from ..asr.engine import AsrEngine
    from ..asr.streaming import AsrBatcher, StreamingAsrSession
    from ..models.config import get_config
    from ..models.whisper import WhisperModel
    from ..tokenizer import load_tokenizer

    name = knob("VWA_ASR_MODEL")
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    wpath = knob("VWA_ASR_WEIGHTS")
    if wpath:
        from ..runtime.weights import LazySafetensors

    model = WhisperModel(get_config(name), device=dev, weights=LazySafetensors(wpath) if wpath else None)
    eng = AsrEngine(model, load_tokenizer("whisper"),
                    max_sessions=knob("VWA_MAX_SESSIONS"))
    # VWA_ASR_TOKENS_PER_S: fixed-work transcripts for benchmarks on random-init weights
    tps = knob("VWA_ASR_TOKENS_PER_S") or None
    batcher = AsrBatcher(eng, tokens_per_s=tps)
    every = knob("VWA_PARTIAL_EVERY_S")

    def factory():
        return StreamingAsrSession(batcher, model_name=name, partial_every_s=every)

    factory.batcher = batcher
    return factory


def main():
    from ..utils.env import load_dotenv

    load_dotenv()
    port = knob("VOICE_PORT")
    print(f"[voice] http/ws listening on http://127.0.0.1:{port}", flush=True)
    # binds all interfaces, as the reference (apps/voice/src/server.ts:80)
    web.run_app(build_app(asr_factory_from_env()), host="0.0.0.0", port=port, print=None)


if __name__ == "__main__":
    main()
