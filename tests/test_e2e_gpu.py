"""End to end on the GPU through the three services: WS PCM16 frames -> voice service with the
real streaming Whisper ASR (native kernels, device-resident decode loop) -> debounce -> brain
/parse with the real Llama intent engine (chained decode launches, grammar-constrained) ->
executor /execute against a fake page.  Every frame type the reference's voice server emits on
this path is checked (apps/voice/src/server.ts:111-231)."""
import asyncio
import json
import os

import numpy as np
import pytest
import torch
from aiohttp.test_utils import TestClient, TestServer

from fakes import FakePage
from voice_enabled_browser_automation_amd import ops
from voice_enabled_browser_automation_amd.asr.engine import AsrEngine
from voice_enabled_browser_automation_amd.asr.streaming import StreamingAsrSession, make_asr_transcriber
from voice_enabled_browser_automation_amd.brain.server import build_app as build_brain, build_llm_engine
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.executor.server import build_app as build_executor
from voice_enabled_browser_automation_amd.executor.session import Session, SessionManager
from voice_enabled_browser_automation_amd.models.config import get_config
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer
from voice_enabled_browser_automation_amd.voice.server import build_app as build_voice

pytestmark = pytest.mark.gpu


def _speech(seconds: float) -> np.ndarray:
    t = np.arange(int(seconds * 16000)) / 16000
    sig = np.sin(2 * np.pi * 180 * t) * (1 + 0.5 * np.sin(2 * np.pi * 3 * t)) * 9000
    return sig.astype(np.int16)


def test_voice_to_intent_to_execution_on_gpu(tmp_path):
    ops.ext()
    asr = AsrEngine(WhisperModel(get_config("whisper-tiny"), device="cuda", seed=0), load_tokenizer("whisper"),
                    max_sessions=2)
    transcribe = make_asr_transcriber(asr, tokens_per_s=4.0)
    brain_engine = build_llm_engine("llama-tiny", device="cuda")

    async def factory(sid):
        d = str(tmp_path / "art" / sid)
        os.makedirs(d, exist_ok=True)
        return Session(id=sid, page=FakePage(), dir=d)

    async def recv_until(ws, want, timeout=60.0):
        got = []
        while not any(g["type"] in want for g in got):
            msg = await asyncio.wait_for(ws.receive(), timeout)
            got.append(json.loads(msg.data))
        return got

    async def go():
        async with TestServer(build_brain(brain_engine)) as bs, \
                TestServer(build_executor(SessionManager(factory), upload_dir=str(tmp_path / "up"))) as es:
            vapp = build_voice(lambda: StreamingAsrSession(transcribe, model_name="whisper-tiny"),
                               brain_url=str(bs.make_url("/parse")), executor_url=str(es.make_url("")).rstrip("/"),
                               debounce_ms=20)
            async with TestClient(TestServer(vapp)) as c:
                ws = await c.ws_connect("/stream")
                assert json.loads((await ws.receive()).data) == {"type": "info", "payload": "deepgram_connected"}
                assert json.loads((await ws.receive()).data) == {"type": "info", "payload": {"state": "open"}}
                await ws.send_str(json.dumps({"type": "context_update", "payload": {"url": "https://www.bestbuy.com"}}))
                pcm = _speech(2.0).tobytes()
                for i in range(0, len(pcm), 1920):  # 60 ms packets, as the UI sends them
                    await ws.send_bytes(pcm[i:i + 1920])
                await ws.send_str(json.dumps({"type": "flush"}))
                got = await recv_until(ws, {"intent"})
                types = [g["type"] for g in got]
                assert "transcript_final" in types and types.index("transcript_final") < types.index("intent")
                fin = next(g for g in got if g["type"] == "transcript_final")["payload"]
                assert fin["is_final"] is True and isinstance(fin["channel"]["alternatives"][0]["transcript"], str)
                intent = next(g for g in got if g["type"] == "intent")["payload"]
                assert safe_parse(ParseResponse, intent).success, intent
                # safe intents auto-execute, risky ones are reported: one of the outcome frames follows
                outcome = await recv_until(ws, {"execution_result", "execution_error", "confirmation_required"})
                assert outcome[-1]["type"] in ("execution_result", "execution_error", "confirmation_required")
                await ws.close()
                m = await (await c.get("/metrics")).json()
                assert m["counters"]["finals"] >= 1

    asyncio.run(go())
    torch.cuda.synchronize()


def test_eight_concurrent_streaming_sessions_on_gpu():
    """8 live WebSocket sessions streaming 60 ms PCM packets into the voice service: the ASR
    batcher (asr/streaming.py) runs every session's recognition pass in shared GPU batches
    (Whisper-tiny, hipGraph decode); reports speech_to_final_ms p50/p95 per session."""
    import statistics
    import time

    from voice_enabled_browser_automation_amd.asr.streaming import AsrBatcher

    ops.ext()
    eng = AsrEngine(WhisperModel(get_config("whisper-tiny"), device="cuda", seed=0), load_tokenizer("whisper"),
                    max_sessions=8)
    batcher = AsrBatcher(eng, max_tokens=24)

    def factory():
        return StreamingAsrSession(batcher, model_name="whisper-tiny", partial_every_s=0.5, endpoint_silence_s=0.3)

    factory.batcher = batcher
    lat = {}

    async def client(c, i):
        ws = await c.ws_connect("/stream")
        await ws.receive()
        await ws.receive()
        pcm = np.concatenate([_speech(1.5 + 0.1 * i), np.zeros(8000, np.int16)]).tobytes()
        t0 = time.perf_counter()
        done = asyncio.Event()

        async def reader():
            while True:
                msg = await ws.receive()
                if msg.type != 1:
                    return
                if json.loads(msg.data)["type"] == "transcript_final":
                    lat[i] = (time.perf_counter() - t0) * 1e3
                    done.set()
                    return

        rd = asyncio.ensure_future(reader())
        for j in range(0, len(pcm), 1920):
            await ws.send_bytes(pcm[j:j + 1920])
            await asyncio.sleep(0.06)  # real-time pacing, as a microphone
        await asyncio.wait_for(rd, 60)
        await ws.close()

    async def go():
        async with TestClient(TestServer(build_voice(factory, debounce_ms=10))) as c:
            await asyncio.gather(*(client(c, i) for i in range(8)))
            return await (await c.get("/metrics")).json()

    try:
        m = asyncio.run(go())
    finally:
        batcher.close()
    vals = sorted(lat.values())
    assert len(vals) == 8
    audio_ms = [(1.5 + 0.1 * i) * 1e3 + 500 for i in range(8)]
    print(json.dumps({"sessions": 8, "speech_to_final_ms_p50": round(statistics.median(vals), 1),
                      "speech_to_final_ms_p95": round(vals[-1], 1), "audio_ms_mean": round(sum(audio_ms) / 8, 1),
                      "asr_rows_per_batch": round(batcher.rows_per_batch(), 2), "batches": batcher.stats["batches"],
                      "max_batch": batcher.stats["max_batch"]}), flush=True)
    assert m["asr_batcher"]["max_batch"] > 1 and batcher.rows_per_batch() > 1.0
