"""Executor: intent interpreter (union of actions.ts + actions.js) against a fake Page, and the
HTTP service (/health, /uploads, /execute, /close) with an injected session factory."""
import asyncio
import json
import os

import aiohttp
from aiohttp.test_utils import TestClient, TestServer

from voice_enabled_browser_automation_amd.executor.actions import resolve_file_ref, run_intents
from voice_enabled_browser_automation_amd.executor.server import build_app
from voice_enabled_browser_automation_amd.executor.session import Session, SessionManager

from fakes import FakePage


def run(page, tmp_path, intents):
    return asyncio.run(run_intents(page, str(tmp_path), intents, upload_dir=str(tmp_path / "up")))


def test_navigate_wait_for_extract_table(tmp_path):
    # port of apps/executor/test/actions.test.ts:27-42
    page = FakePage()
    res = run(page, tmp_path, [
        {"type": "navigate", "args": {"url": "https://example.com"}},
        {"type": "wait_for", "args": {"selector": "[data-test=\"results\"]", "timeoutMs": 1000}},
        {"type": "extract_table", "args": {"limit": 5}},
    ])
    assert res[0]["ok"] and res[1]["ok"] and res[2]["ok"]
    assert isinstance(res[2]["data"], list) and res[2]["data"][0]["price"] == "$9.99"
    assert os.path.exists(res[2]["data_paths"]["json"]) and os.path.exists(res[2]["data_paths"]["csv"])
    assert all(r.get("screenshot") for r in res)


def test_search_uses_scored_analysis_then_enter(tmp_path):
    page = FakePage()
    res = run(page, tmp_path, [{"type": "search", "args": {"query": "wireless earbuds"}}])
    assert res[0]["ok"]
    assert ("fill", 'input[name="q"]', "wireless earbuds") in page.calls
    assert ("press", 'input[name="q"]', "Enter") in page.calls


def test_search_legacy_fallback_keyboard(tmp_path):
    sels = {'input[name="q"]', 'input[type="search"]', 'input[aria-label*="Search" i]',
            'input[placeholder*="Search" i]', "#search", 'input[name*="search" i]'}
    page = FakePage(missing_selectors=sels)
    res = run(page, tmp_path, [{"type": "search", "args": {"query": "tv"}, "retries": 0}])
    assert res[0]["ok"] and ("kb_type", "tv") in page.calls and ("kb_press", "Enter") in page.calls


def test_click_by_text_selector_role(tmp_path):
    page = FakePage()
    res = run(page, tmp_path, [
        {"type": "click", "target": {"text": "add to cart"}},
        {"type": "click", "target": {"selector": "#search-list li:nth-of-type(2) a"}},
        {"type": "click", "target": {"role": "button", "name": "Submit"}},
    ])
    assert all(r["ok"] for r in res)
    assert ("click", "#buy") in page.calls
    assert ("click", "#search-list li:nth-of-type(2) a") in page.calls
    assert ("locator_click", "role", ("button", "Submit")) in page.calls


def test_filter_sort_type_select_scroll_back_forward(tmp_path):
    page = FakePage()
    res = run(page, tmp_path, [
        {"type": "filter", "args": {"price": {"lte": 50}}},
        {"type": "sort", "args": {"by": "price", "order": "asc"}},
        {"type": "type", "target": {"selector": "#email"}, "args": {"value": "a@b.c"}},
        {"type": "select", "target": {"selector": "#size"}, "args": {"value": "M"}},
        {"type": "scroll", "args": {"direction": "down"}},
        {"type": "back"}, {"type": "forward"}, {"type": "screenshot", "args": {"label": "x"}},
    ])
    assert all(r["ok"] for r in res), [r.get("error") for r in res]
    assert ("fill", "#max", "50") in page.calls
    assert ("select_option", "#sort", "price low to high", None) in page.calls
    assert ("fill", "#email", "a@b.c") in page.calls
    assert "go_back" in page.names() and "go_forward" in page.names()


def test_unsupported_and_summarize(tmp_path):
    page = FakePage()
    res = run(page, tmp_path, [{"type": "confirm"}, {"type": "unknown"}, {"type": "extract"}, {"type": "summarize"}])
    assert [r["ok"] for r in res] == [False, False, False, True]
    assert res[0]["error"] == "Unsupported intent type: confirm"
    assert "brain" in res[3]["data"]["note"]


def test_retries_are_honoured(tmp_path):
    page = FakePage(missing_selectors={"#nope"})
    res = run(page, tmp_path, [{"type": "click", "target": {"selector": "#nope"}, "retries": 2}])
    assert not res[0]["ok"] and res[0]["attempts"] == 3
    assert res[0]["error"]


def test_upload_resolves_extension(tmp_path):
    up = tmp_path / "up"
    up.mkdir()
    (up / "abc123.pdf").write_bytes(b"%PDF")
    assert resolve_file_ref("resume://abc123", str(up)).endswith("abc123.pdf")
    assert resolve_file_ref("resume://latest", str(up)).endswith("abc123.pdf")
    page = FakePage()
    res = run(page, tmp_path, [{"type": "upload", "args": {"fileRef": "resume://abc123"},
                                "target": {"selector": "input[type=\"file\"]"}}])
    assert res[0]["ok"]
    assert any(c[0] == "set_input_files" and c[2].endswith(".pdf") for c in page.calls)


def _app(tmp_path):
    pages = {}

    async def factory(sid):
        d = str(tmp_path / "art" / sid)
        os.makedirs(d, exist_ok=True)
        pages[sid] = FakePage()
        return Session(id=sid, page=pages[sid], dir=d)

    return build_app(SessionManager(factory), upload_dir=str(tmp_path / "uploads")), pages


def test_executor_http_service(tmp_path):
    app, pages = _app(tmp_path)

    async def go():
        async with TestClient(TestServer(app)) as c:
            r = await c.get("/health")
            assert await r.json() == {"status": "ok", "service": "executor"}
            r = await c.post("/execute", json={"intents": []})
            assert r.status == 400 and (await r.json())["error"] == "invalid_request"
            r = await c.post("/execute", json={"intents": [{"type": "navigate", "args": {"url": "https://a.com"}}]})
            j = await r.json()
            assert r.status == 200 and j["results"][0]["ok"] and j["artifacts"]["dir"]
            sid = j["session_id"]
            r = await c.post("/execute", json={"session_id": sid, "intents": [{"type": "back"}]})
            assert (await r.json())["session_id"] == sid and len(pages) == 1  # session reused
            pages[sid].closed = True  # browser closed by the user -> liveness probe recreates it
            r = await c.post("/execute", json={"session_id": sid, "intents": [{"type": "back"}]})
            assert (await r.json())["results"][0]["ok"] and pages[sid].calls == [("go_back",)] + pages[sid].calls[1:]
            fd = aiohttp.FormData()
            fd.add_field("file", b"%PDF-1.4", filename="resume.pdf", content_type="application/pdf")
            r = await c.post("/uploads", data=fd)
            j = await r.json()
            assert j["fileRef"].startswith("resume://") and j["path"].endswith(".pdf")
            r = await c.post("/close", json={})
            assert r.status == 400 and (await r.json()) == {"error": "session_id required"}
            r = await c.post("/close", json={"session_id": sid})
            assert (await r.json()) == {"ok": True}
            r = await c.options("/execute", headers={"Origin": "http://localhost:5173"})
            assert r.headers.get("Access-Control-Allow-Origin") == "http://localhost:5173"

    asyncio.run(go())


def test_synthesised_selectors_are_escaped():
    """ids with ':' / '.' (framework markup) and quotes in attribute values
    give broken selectors when synthesised raw (reference dom-analyzer.ts:78-86); the page script
    escapes them (CSS.escape, or the same backslash rule without it) -- mirrored in Python."""
    from voice_enabled_browser_automation_amd.executor.dom_analyzer import ANALYZE_JS, synth_selector

    assert synth_selector("INPUT", {"id": "search:q.1"}) == "#search\\:q\\.1"
    assert synth_selector("input", {"name": 'a"b'}) == 'input[name="a\\"b"]'
    assert synth_selector("button", {"data-testid": "go"}) == '[data-testid="go"]'
    assert synth_selector("A", {}) == "a"
    assert "CSS.escape" in ANALYZE_JS and "d.selector === 'a'" not in ANALYZE_JS
