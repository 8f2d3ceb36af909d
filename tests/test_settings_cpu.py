"""The one typed settings object (utils/env.py): every knob the code reads is
declared there with its type and default, and reads go through ``knob()``."""
import os
import re

import pytest

from voice_enabled_browser_automation_amd.utils.env import Settings, knob, settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = [os.path.join(ROOT, "voice_enabled_browser_automation_amd"), os.path.join(ROOT, "csrc"),
           os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]


def _source_files():
    for s in SOURCES:
        if os.path.isfile(s):
            yield s
            continue
        for d, _dirs, files in os.walk(s):
            for f in files:
                if f.endswith((".py", ".cpp", ".hip", ".h")):
                    yield os.path.join(d, f)


def test_every_vwa_knob_in_the_sources_is_declared():
    names = set()
    for path in _source_files():
        with open(path, encoding="utf-8") as fh:
            names |= set(re.findall(r"\bVWA_[A-Z0-9_]+\b", fh.read()))
    # (names that are not environment variables: C++ macros of the kernel sources)
    names = {n for n in names if not n.startswith(("VWA_CHAIN_LAUNCH", "VWA_DEVICE", "VWA_TIE", "VWA_ONLY_MULTI"))
             and n != "VWA_TX"}
    missing = sorted(n for n in names if n not in Settings.model_fields)
    assert not missing, f"undeclared knobs (add them to utils/env.py Settings): {missing}"


def test_no_direct_environment_reads_of_declared_knobs():
    """Service and engine code reads knobs through knob(), not os.environ (the build script and
    the torch.distributed rendezvous variables aside)."""
    pat = re.compile(r"os\.environ(?:\.get)?\s*[\(\[]\s*\"([A-Z0-9_]+)\"")
    offenders = []
    for path in _source_files():
        if not path.endswith(".py") or path.endswith(os.path.join("ops", "build.py")) or path.endswith("env.py"):
            continue
        with open(path, encoding="utf-8") as fh:
            for name in pat.findall(fh.read()):
                if name in Settings.model_fields:
                    offenders.append(f"{os.path.relpath(path, ROOT)}: {name}")
    assert not offenders, offenders


def test_knob_types_defaults_and_errors(monkeypatch):
    monkeypatch.delenv("VWA_ENDPOINT_MS", raising=False)
    assert knob("VWA_ENDPOINT_MS") == Settings.model_fields["VWA_ENDPOINT_MS"].default
    monkeypatch.setenv("VWA_ENDPOINT_MS", "250")
    assert knob("VWA_ENDPOINT_MS") == 250.0
    monkeypatch.setenv("VWA_CHAIN", "0")
    assert knob("VWA_CHAIN") is False
    monkeypatch.setenv("VWA_CHAIN", "on")
    assert knob("VWA_CHAIN") is True
    monkeypatch.setenv("VWA_MAX_SESSIONS", "12")
    assert knob("VWA_MAX_SESSIONS") == 12
    monkeypatch.setenv("VWA_MAX_SESSIONS", "twelve")
    with pytest.raises(ValueError):
        knob("VWA_MAX_SESSIONS")
    with pytest.raises(KeyError):
        knob("VWA_NOT_A_KNOB")
    monkeypatch.setenv("VWA_MAX_SESSIONS", "16")
    s = settings()
    assert s.VWA_MAX_SESSIONS == 16 and s.VWA_CHAIN is True and s.BRAIN_PORT == 8090


def test_services_take_their_config_from_settings(monkeypatch):
    from voice_enabled_browser_automation_amd.asr.streaming import StreamingAsrSession

    monkeypatch.setenv("VWA_ENDPOINT_MS", "420")
    monkeypatch.setenv("VWA_SPEC_FINAL_MS", "100")
    monkeypatch.setenv("VWA_VAD_THRESHOLD", "500")
    s = StreamingAsrSession(lambda pcm: "x")
    assert s.endpoint == int(0.42 * 16000) and s.spec_at == 1600 and s.thresh == 500.0
