"""The Playwright-free CDP driver (executor/cdp.py) against a fake DevTools endpoint.

No browser exists in this image, so the fake speaks the protocol side only: it answers the
commands the driver sends (targets, flattened sessions, Runtime.evaluate of the driver's page
scripts, input events, DOM file inputs, screenshots, history) from a small Python model of a page
and records every command, so the tests check the wire traffic the executor's intents produce.
"""
import asyncio
import base64
import json
import re

import pytest
from aiohttp import web

from voice_enabled_browser_automation_amd.executor import cdp
from voice_enabled_browser_automation_amd.executor.actions import run_intents
from voice_enabled_browser_automation_amd.executor.session import SessionManager, _cdp_factory

PNG = b"\x89PNG\r\n\x1a\nfake"


class FakeBrowser:
    def __init__(self):
        self.log = []           # (method, params, sessionId)
        self.url = "about:blank"
        self.history = ["about:blank"]
        self.hist_i = 0
        self.values = {}        # selector -> filled value
        self.visible = {'input[name="q"]', "#go", 'select[name="sort"]', "input[type=file]"}
        self.options = {'select[name="sort"]': ["Price Low to High", "Price High to Low"]}

    def evaluate(self, expr):
        m = re.search(r"\)\(\.\.\.(\[.*\])\)$", expr, re.S)
        args = json.loads(m.group(1)) if m else []
        if expr == "document.readyState":
            return "complete"
        if "const attrs = (el)" in expr:  # DOM analysis (dom_analyzer.ANALYZE_JS)
            return {"url": self.url, "title": "fake",
                    "searchElements": [{"selector": 'input[name="q"]', "type": "search", "text": "",
                                        "placeholder": "Search", "attributes": {"name": "q", "type": "search"},
                                        "bbox": {"x": 0, "y": 0, "width": 400, "height": 30},
                                        "isVisible": True, "isEnabled": True}],
                    "buttons": [], "links": [], "forms": [], "filters": [], "navigationElements": []}
        if "'visible' : el ? 'attached'" in expr:
            return "visible" if args[0] in self.visible or args[0].startswith("[data-vwa-mark") else "none"
        if "desc.set.call" in expr:  # fill
            self.values[args[0]] = args[1]
            return "ok"
        if "getBoundingClientRect" in expr:
            return [120.0, 40.0] if args[0] in self.visible or args[0].startswith("[data-vwa-mark") else None
        if "o.label || o.text" in expr:  # select_option
            opts = self.options.get(args[0])
            if opts is None:
                return "missing"
            return "ok" if args[2] in opts else "nooption"
        if "new RegExp(src, flags)" in expr:  # get_by_text
            return f'[data-vwa-mark="{args[2]}"]' if re.search(args[0], "Sort by", re.I if "i" in args[1] else 0) else None
        if "implicit" in expr:  # get_by_role
            return f'[data-vwa-mark="{args[2]}"]' if args[0] == "button" else None
        if ".focus()" in expr:
            return None
        if "scrollBy" in expr:
            return None
        return None

    async def handler(self, request):
        ws = web.WebSocketResponse(max_msg_size=0)
        await ws.prepare(request)
        async for msg in ws:
            d = json.loads(msg.data)
            meth, p, sid = d["method"], d.get("params", {}), d.get("sessionId")
            self.log.append((meth, p, sid))
            res, events = {}, []
            if meth == "Target.createTarget":
                res = {"targetId": "T1"}
            elif meth == "Target.attachToTarget":
                res = {"sessionId": "S1"}
            elif meth == "Page.navigate":
                self.url = p["url"]
                self.history = self.history[: self.hist_i + 1] + [p["url"]]
                self.hist_i += 1
                res = {"frameId": "F1"}
                events.append("Page.domContentEventFired")
            elif meth == "Page.getNavigationHistory":
                res = {"currentIndex": self.hist_i,
                       "entries": [{"id": 100 + i, "url": u} for i, u in enumerate(self.history)]}
            elif meth == "Page.navigateToHistoryEntry":
                self.hist_i = p["entryId"] - 100
                self.url = self.history[self.hist_i]
                events.append("Page.domContentEventFired")
            elif meth == "Runtime.evaluate":
                res = {"result": {"type": "object", "value": self.evaluate(p["expression"])}}
            elif meth == "Page.getLayoutMetrics":
                res = {"cssContentSize": {"x": 0, "y": 0, "width": 1366, "height": 2400}}
            elif meth == "Page.captureScreenshot":
                res = {"data": base64.b64encode(PNG).decode()}
            elif meth == "DOM.getDocument":
                res = {"root": {"nodeId": 1}}
            elif meth == "DOM.querySelector":
                res = {"nodeId": 7 if p["selector"] in self.visible else 0}
            elif meth == "Bogus.method":
                await ws.send_str(json.dumps({"id": d["id"], "error": {"code": -32601, "message": "not found"}}))
                continue
            await ws.send_str(json.dumps({"id": d["id"], "result": res, **({"sessionId": sid} if sid else {})}))
            for ev in events:
                await ws.send_str(json.dumps({"method": ev, "params": {"timestamp": 1.0}, "sessionId": sid}))
            if meth == "Browser.close":
                await ws.close()
        return ws

    def sent(self, method):
        return [(p, s) for m, p, s in self.log if m == method]


async def _serve(fake):
    app = web.Application()
    app.router.add_get("/devtools/browser/x", fake.handler)

    async def version(_):
        return web.json_response({"webSocketDebuggerUrl": f"ws://127.0.0.1:{port}/devtools/browser/x"})

    app.router.add_get("/json/version", version)
    runner = web.AppRunner(app)
    await runner.setup()
    site = web.TCPSite(runner, "127.0.0.1", 0)
    await site.start()
    port = site._server.sockets[0].getsockname()[1]
    return runner, port


def test_cdp_page_commands_and_sessions(tmp_path):
    async def main():
        fake = FakeBrowser()
        runner, port = await _serve(fake)
        try:
            conn = await cdp.connect(f"http://127.0.0.1:{port}")  # resolved through /json/version
            page = await conn.new_page()
            assert fake.sent("Target.attachToTarget")[0][0] == {"targetId": "T1", "flatten": True}
            await page.goto("https://example.com", timeout=2000)
            assert fake.url == "https://example.com"
            # every page command carries the flattened session id
            assert all(s == "S1" for m, _, s in fake.log if m.split(".")[0] in ("Page", "Runtime", "Input", "DOM"))
            await page.fill('input[name="q"]', "earbuds")
            assert fake.values['input[name="q"]'] == "earbuds"
            await page.press('input[name="q"]', "Enter")
            keys = fake.sent("Input.dispatchKeyEvent")
            assert keys[0][0]["type"] == "keyDown" and keys[0][0]["windowsVirtualKeyCode"] == 13
            await page.click("#go")
            mouse = [p["type"] for p, _ in fake.sent("Input.dispatchMouseEvent")]
            assert mouse == ["mouseMoved", "mousePressed", "mouseReleased"]
            assert fake.sent("Input.dispatchMouseEvent")[1][0]["x"] == 120.0
            assert await page.select_option('select[name="sort"]', label="Price Low to High") == ["Price Low to High"]
            with pytest.raises(cdp.CdpError):
                await page.select_option('select[name="sort"]', label="Newest")
            await page.get_by_text(re.compile("sort", re.I)).first.click(timeout=1000)
            await page.get_by_role("button", name="Add").first.click(timeout=1000)
            with pytest.raises(TimeoutError):
                await page.get_by_role("link", name="nothing").first.click(timeout=300)
            with pytest.raises(TimeoutError):
                await page.wait_for_selector("#absent", timeout=250)
            f = tmp_path / "cv.pdf"
            f.write_bytes(b"%PDF")
            await page.set_input_files("input[type=file]", str(f))
            assert fake.sent("DOM.setFileInputFiles")[0][0] == {"files": [str(f)], "nodeId": 7}
            shot = tmp_path / "a" / "s.png"
            assert await page.screenshot(path=str(shot), full_page=True) == PNG
            assert shot.read_bytes() == PNG
            clip = fake.sent("Page.captureScreenshot")[0][0]["clip"]
            assert clip["height"] == 2400 and fake.sent("Page.captureScreenshot")[0][0]["captureBeyondViewport"]
            await page.goto("https://example.com/p2", timeout=2000)
            await page.go_back(timeout=2000)
            assert fake.url == "https://example.com"
            await page.go_forward(timeout=2000)
            assert fake.url == "https://example.com/p2"
            assert await page.evaluate("(a, b) => a + b", 1, 2) is None  # fake: unknown script
            assert "...[1, 2]" in fake.sent("Runtime.evaluate")[-1][0]["expression"]
            with pytest.raises(cdp.CdpError, match="not found"):
                await conn.send("Bogus.method")
            assert not page.is_closed()
            await conn.close()
            assert page.is_closed() and not conn.is_connected()
        finally:
            await runner.cleanup()

    asyncio.run(main())


def test_executor_intents_over_cdp(tmp_path, monkeypatch):
    """The executor's session manager falls back to the CDP driver without Playwright and runs a
    navigate -> search -> sort -> screenshot plan over it."""
    async def main():
        fake = FakeBrowser()
        runner, port = await _serve(fake)
        try:
            monkeypatch.setenv("CDP_URL", f"http://127.0.0.1:{port}")
            monkeypatch.setenv("ARTIFACTS_DIR", str(tmp_path / "art"))
            mgr = SessionManager(factory=_cdp_factory)
            s = await mgr.open_session()
            assert isinstance(s.page, cdp.CdpPage)
            res = await run_intents(s.page, s.dir, [
                {"type": "navigate", "args": {"url": "https://www.bestbuy.com"}},
                {"type": "search", "args": {"query": "wireless earbuds"}},
                {"type": "scroll", "args": {"direction": "down"}},
                {"type": "screenshot", "args": {"label": "done"}},
            ], upload_dir=str(tmp_path / "up"))
            assert [r["ok"] for r in res] == [True, True, True, True], res
            assert fake.url == "https://www.bestbuy.com"
            assert fake.values.get('input[name="q"]') == "wireless earbuds"
            assert fake.sent("Page.captureScreenshot")
            await mgr.close_session(s.id)
            assert fake.sent("Browser.close")
        finally:
            await runner.cleanup()

    asyncio.run(main())


def test_driver_selection(monkeypatch):
    from voice_enabled_browser_automation_amd.executor import session

    monkeypatch.setenv("VWA_BROWSER_DRIVER", "cdp")
    assert session._driver() == "cdp"
    monkeypatch.delenv("VWA_BROWSER_DRIVER")
    try:
        import playwright  # noqa: F401
        want = "playwright"
    except ImportError:
        want = "cdp"
    assert session._driver() == want
    monkeypatch.setenv("CHROME_PATH", "/nonexistent/chrome")
    monkeypatch.setenv("PATH", "/nonexistent")
    assert cdp.find_chrome() is None
