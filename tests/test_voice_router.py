"""Voice DP router: least-sessions assignment across per-GPU voice workers, transparent frame
proxying, and the watchdog failover when a worker dies (SURVEY.md §2.2 session-DP, §5.3)."""
import asyncio
import json

import aiohttp
from aiohttp import web
from aiohttp.test_utils import TestServer

from voice_enabled_browser_automation_amd.voice.router import build_router
from voice_enabled_browser_automation_amd.voice.server import build_app


class _Echo:
    """ASR session double: every pushed packet becomes a final transcript naming the worker."""

    def __init__(self, tag):
        self.tag = tag

    def push(self, data):
        return [{"type": "Results", "is_final": True, "speech_final": True,
                 "channel": {"alternatives": [{"transcript": f"{self.tag}:{len(data)}"}]}}]

    def flush(self):
        return []


def test_router_balances_proxies_and_fails_over():
    async def go():
        workers = []
        for tag in ("w0", "w1"):
            srv = TestServer(build_app(lambda t=tag: _Echo(t), brain_url="http://127.0.0.1:9/parse",
                                       executor_url="http://127.0.0.1:9", debounce_ms=60000))
            await srv.start_server()
            workers.append(srv)
        router = TestServer(build_router([str(w.make_url("")) for w in workers], probe_s=0.2, max_fails=1))
        await router.start_server()
        async with aiohttp.ClientSession() as http:
            h = await (await http.get(router.make_url("/health"))).json()
            assert h["status"] == "ok" and h["healthy_workers"] == 2
            a = await http.ws_connect(router.make_url("/stream"))
            b = await http.ws_connect(router.make_url("/stream"))

            async def transcript(ws):
                while True:
                    msg = json.loads((await ws.receive(timeout=10)).data)
                    if msg["type"] == "transcript_final":
                        return msg["payload"]["channel"]["alternatives"][0]["transcript"]

            await a.send_bytes(b"\0" * 320)
            await b.send_bytes(b"\0" * 640)
            ta, tb = await transcript(a), await transcript(b)
            assert {ta.split(":")[0], tb.split(":")[0]} == {"w0", "w1"}  # one session per worker
            assert ta.endswith(":320") and tb.endswith(":640")  # frames proxied unchanged
            # C6 metrics gather: after a watchdog round every rank reports its live session + final
            agg = None
            for _ in range(40):
                await asyncio.sleep(0.1)
                agg = (await (await http.get(router.make_url("/metrics"))).json())["aggregate"]
                if agg.get("ranks_reporting") == 2 and agg.get("finals") == 2:
                    break
            assert agg["ranks_reporting"] == 2 and agg["live_sessions"] == 2 and agg["finals"] == 2, agg
            # kill the worker serving `a`: its session moves to the survivor
            dead = 0 if ta.startswith("w0") else 1
            await workers[dead].close()
            got = None
            for _ in range(50):
                msg = await a.receive(timeout=10)
                if msg.type == aiohttp.WSMsgType.TEXT and json.loads(msg.data).get("payload") == "asr_failover":
                    got = True
                    break
            assert got
            await a.send_bytes(b"\0" * 100)
            assert (await transcript(a)) == f"w{1 - dead}:100"
            m = await (await http.get(router.make_url("/metrics"))).json()
            assert m["counters"]["failovers"] >= 1 and sum(w["healthy"] for w in m["workers"]) == 1
            await a.close()
            await b.close()
        await router.close()
        for w in workers:
            await w.close()

    asyncio.run(go())


def test_launch_gpu_plan():
    from voice_enabled_browser_automation_amd.launch import plan_gpus

    assert plan_gpus(8, tp=2) == {"brain": ["0", "1"], "voice": ["2", "3", "4", "5", "6", "7"], "shared": False}
    assert plan_gpus(2) == {"brain": ["0"], "voice": ["1"], "shared": False}
    assert plan_gpus(1) == {"brain": ["0"], "voice": ["0"], "shared": True}
    assert plan_gpus(8, tp=8)["shared"]  # every GPU is a TP rank: the voice worker shares GPU 0
    assert plan_gpus(8, brain="3", voice="4,5") == {"brain": ["3"], "voice": ["4", "5"], "shared": False}
