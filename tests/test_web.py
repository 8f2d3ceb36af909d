"""UI shell (apps/web parity): the page renders the Start control (the reference's App.test
expects it, apps/web/src/App.test.tsx:9), speaks the same WS/HTTP endpoints, and the static
server serves it."""
import asyncio

from aiohttp.test_utils import TestClient, TestServer

from voice_enabled_browser_automation_amd.web.server import build_app


def test_ui_shell_served_with_start_button_and_endpoints():
    async def go():
        async with TestClient(TestServer(build_app())) as c:
            r = await c.get("/")
            return r.status, r.headers.get("content-type", ""), await r.text()

    st, ct, html = asyncio.run(go())
    assert st == 200 and "text/html" in ct
    assert ">Start<" in html and ">Stop<" in html
    assert ":7072/stream" in html and ":7081" in html  # voice WS and executor defaults
    assert "pcm16-tap" in html and "/uploads" in html and "/execute" in html
