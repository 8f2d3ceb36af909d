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
