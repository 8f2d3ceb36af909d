"""Voice session router: ASR data parallelism across the GPUs of a node (SURVEY.md §2.2 "ASR
session-DP", §5.3 "engine watchdog").

The reference runs one voice process whose every WebSocket owns one Deepgram stream
(apps/voice/src/server.ts:97-108).  Here each GPU runs its own voice worker (voice/server.py,
one process per GPU, pinned with HIP_VISIBLE_DEVICES, on VWA_VOICE_BASE_PORT + i); this router
listens on VOICE_PORT with the same ``/health`` and ``/stream`` surface and

* assigns every new WebSocket to the healthy worker with the fewest live sessions;
* proxies frames both ways unchanged (binary PCM in, JSON events out: byte-compatible);
* gathers every worker's ``/metrics`` on each watchdog round (per-rank ASR RTF,
  batcher queue depth, live sessions, speech->final latency) into its own ``/metrics``
  (``workers[i].stats`` + a node-level ``aggregate``);
* runs a watchdog that probes every worker's ``/health`` each ``VWA_WATCHDOG_S`` seconds; a
  worker that fails ``VWA_WATCHDOG_FAILS`` probes in a row is taken out of rotation, and the
  sessions it was serving are moved to a healthy worker: the client gets an
  ``{"type":"info","payload":"asr_failover"}`` frame and its stream continues there (audio
  in flight on the dead worker is lost; the conversation context travels with the client's
  next ``context_update``).
"""
from __future__ import annotations

import asyncio
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional

import aiohttp
from aiohttp import WSMsgType, web

from ..utils.metrics import Metrics
from .server import VERSION
from ..utils.env import knob


@dataclass
class Worker:
    url: str                      # http://127.0.0.1:PORT
    healthy: bool = True
    fails: int = 0
    sessions: int = 0
    clients: set = field(default_factory=set)
    stats: dict = field(default_factory=dict)  # last gathered /metrics summary


def worker_summary(snap: dict) -> dict:
    """The per-rank fields of a voice worker's /metrics snapshot the router aggregates."""
    lat = snap.get("latency") or {}
    bat = snap.get("asr_batcher") or {}

    def p50(k):
        return (lat.get(k) or {}).get("p50")

    return {"live_sessions": snap.get("live_sessions"), "asr_rtf_p50": p50("asr_rtf"),
            "asr_push_ms_p50": p50("asr_push_ms"), "speech_to_final_ms_p50": p50("speech_to_final_ms"),
            "utterance_to_intent_ms_p50": p50("utterance_to_intent_ms"), "queue_depth": bat.get("queue_depth"),
            "rows_per_batch": bat.get("rows_per_batch"), "finals": (snap.get("counters") or {}).get("finals", 0)}


def aggregate(stats: List[dict]) -> dict:
    """Node-level view over the ranks' summaries (sums of counts, max queue, mean / max RTF)."""
    def vals(k):
        return [s[k] for s in stats if s.get(k) is not None]

    rtf = vals("asr_rtf_p50")
    return {"ranks_reporting": len(stats), "live_sessions": sum(vals("live_sessions")),
            "finals": sum(vals("finals")), "max_queue_depth": max(vals("queue_depth"), default=0),
            "asr_rtf_p50_mean": round(sum(rtf) / len(rtf), 6) if rtf else None,
            "asr_rtf_p50_max": max(rtf, default=None)}


def build_router(worker_urls: List[str], *, probe_s: Optional[float] = None,
                 max_fails: Optional[int] = None) -> web.Application:
    app = web.Application()
    app["workers"] = [Worker(u.rstrip("/")) for u in worker_urls]
    app["metrics"] = Metrics("voice-router")
    probe_s = float(knob("VWA_WATCHDOG_S")) if probe_s is None else probe_s
    max_fails = int(knob("VWA_WATCHDOG_FAILS")) if max_fails is None else max_fails

    def pick(exclude: Optional[Worker] = None) -> Optional[Worker]:
        live = [w for w in app["workers"] if w.healthy and w is not exclude]
        return min(live, key=lambda w: w.sessions) if live else None

    async def probe(w: Worker) -> bool:
        try:
            async with app["http"].get(w.url + "/health", timeout=aiohttp.ClientTimeout(total=probe_s)) as r:
                return r.status == 200
        except (aiohttp.ClientError, asyncio.TimeoutError):
            return False

    async def gather(w: Worker) -> None:
        try:
            async with app["http"].get(w.url + "/metrics", timeout=aiohttp.ClientTimeout(total=probe_s)) as r:
                if r.status == 200:
                    w.stats = worker_summary(await r.json())
        except (aiohttp.ClientError, asyncio.TimeoutError, ValueError):
            pass

    async def watchdog():
        while True:
            await asyncio.sleep(probe_s)
            for w in app["workers"]:
                ok = await probe(w)
                if ok:
                    await gather(w)
                    w.fails = 0
                    if not w.healthy:
                        w.healthy = True
                        app["metrics"].inc("worker_recovered")
                    continue
                w.fails += 1
                if w.healthy and w.fails >= max_fails:
                    w.healthy = False
                    app["metrics"].inc("worker_down")
                    for client in list(w.clients):  # drain: move live sessions off the dead worker
                        client.move.set()

    async def on_startup(app_):
        app_["http"] = aiohttp.ClientSession()
        app_["watchdog"] = asyncio.create_task(watchdog())

    async def on_cleanup(app_):
        app_["watchdog"].cancel()
        await app_["http"].close()

    app.on_startup.append(on_startup)
    app.on_cleanup.append(on_cleanup)

    async def health(_req):
        live = sum(w.healthy for w in app["workers"])
        return web.json_response({"status": "ok" if live else "degraded", "service": "voice", "version": VERSION,
                                  "workers": len(app["workers"]), "healthy_workers": live})

    async def metrics(_req):
        snap = app["metrics"].snapshot()
        snap["workers"] = [{"url": w.url, "healthy": w.healthy, "sessions": w.sessions, "stats": w.stats}
                           for w in app["workers"]]
        snap["aggregate"] = aggregate([w.stats for w in app["workers"] if w.healthy and w.stats])
        return web.json_response(snap)

    class _Client:
        def __init__(self):
            self.move = asyncio.Event()

    async def stream(req: web.Request) -> web.WebSocketResponse:
        ws = web.WebSocketResponse()
        await ws.prepare(req)
        m: Metrics = app["metrics"]
        m.inc("connections")
        client = _Client()
        worker = pick()
        if worker is None:
            await ws.send_json({"type": "error", "payload": "no healthy ASR worker"})
            await ws.close()
            return ws
        first = True
        while worker is not None and not ws.closed:
            worker.sessions += 1
            worker.clients.add(client)
            client.move.clear()
            moved = False
            try:
                async with app["http"].ws_connect(worker.url + "/stream") as up:
                    if not first:
                        await ws.send_json({"type": "info", "payload": "asr_failover"})
                        m.inc("failovers")
                    first = False

                    async def down_pump():
                        async for msg in up:
                            if msg.type == WSMsgType.TEXT:
                                if not ws.closed:
                                    await ws.send_str(msg.data)
                            elif msg.type == WSMsgType.BINARY:
                                if not ws.closed:
                                    await ws.send_bytes(msg.data)
                            else:
                                break

                    async def up_pump():
                        async for msg in ws:
                            if msg.type == WSMsgType.BINARY:
                                await up.send_bytes(msg.data)
                            elif msg.type == WSMsgType.TEXT:
                                await up.send_str(msg.data)
                            else:
                                break

                    tasks = {asyncio.ensure_future(down_pump()), asyncio.ensure_future(up_pump()),
                             asyncio.ensure_future(client.move.wait())}
                    done, pending = await asyncio.wait(tasks, return_when=asyncio.FIRST_COMPLETED)
                    for t in pending:
                        t.cancel()
                    # the watchdog moved us, or the upstream ended under an open client: a worker
                    # that still answers /health closed the session on purpose (client "close")
                    if ws.closed:
                        moved = False
                    elif client.move.is_set() or not worker.healthy:
                        moved = True
                    else:
                        moved = not await probe(worker)
            except (aiohttp.ClientError, asyncio.TimeoutError, ConnectionResetError):
                moved = not ws.closed
            finally:
                worker.sessions -= 1
                worker.clients.discard(client)
            if not moved:
                break
            worker.fails = max(worker.fails, max_fails)  # do not hand this session back to it
            worker.healthy = False
            worker = pick(exclude=worker)
            if worker is None:
                await ws.send_json({"type": "error", "payload": "no healthy ASR worker"})
        if not ws.closed:
            await ws.close()
        return ws

    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics)
    app.router.add_get("/stream", stream)
    return app


def main():
    from ..utils.env import load_dotenv

    load_dotenv()
    port = int(knob("VOICE_PORT"))
    base = int(knob("VWA_VOICE_BASE_PORT"))
    n = int(knob("VWA_DP"))
    urls = [f"http://127.0.0.1:{base + i}" for i in range(n)]
    print(f"[voice-router] ws://127.0.0.1:{port}/stream -> {json.dumps(urls)}", flush=True)
    web.run_app(build_router(urls), host="127.0.0.1", port=port, print=None)


if __name__ == "__main__":
    main()
