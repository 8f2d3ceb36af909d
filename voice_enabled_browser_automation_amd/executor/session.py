"""Browser session manager (apps/executor/src/session.ts).

* in-memory map session_id -> Session(browser, context, page, artifact dir);
* local Chrome via Playwright (``EXECUTOR_HEADLESS``), or a Browserbase remote browser over CDP
  when ``BROWSERBASE_API_KEY`` + ``BROWSERBASE_PROJECT_ID`` are set (session.ts:35-44);
* fixes of the reference: a per-session asyncio.Lock serialises concurrent
  /execute calls on one page, and a liveness probe recreates a session whose page/browser was
  closed (the README promises this, session.ts:26 never checked);
* flags are read at call time (the reference reads them at import time, before dotenv runs:
  SURVEY.md §3.5).

Playwright is an optional runtime dependency (not installable in this image): without it the
sessions run on the built-in CDP driver (``executor/cdp.py``: local Chrome with remote debugging,
``CDP_URL``, or Browserbase's CDP ``connectUrl``); ``VWA_BROWSER_DRIVER=playwright|cdp`` forces
one.  Tests inject a page factory or a fake CDP endpoint.
"""
from __future__ import annotations

import asyncio
import os
import uuid
from dataclasses import dataclass, field
from typing import Any, Awaitable, Callable, Dict, Optional
from ..utils.env import knob


@dataclass
class Session:
    id: str
    page: Any
    dir: str
    browser: Any = None
    context: Any = None
    pw: Any = None
    lock: asyncio.Lock = field(default_factory=asyncio.Lock)


PageFactory = Callable[[str], Awaitable[Session]]


def artifacts_dir() -> str:
    return knob("ARTIFACTS_DIR")


async def _cdp_factory(sid: str) -> Session:
    """Playwright-free session (executor/cdp.py): a CDP endpoint from ``CDP_URL``, a Browserbase
    session's ``connectUrl``, or a local Chrome launched with remote debugging."""
    from . import cdp

    d = os.path.join(artifacts_dir(), sid)
    os.makedirs(d, exist_ok=True)
    bb_key, bb_proj = knob("BROWSERBASE_API_KEY"), knob("BROWSERBASE_PROJECT_ID")
    if knob("CDP_URL"):
        conn = await cdp.connect(knob("CDP_URL"))
    elif bb_key and bb_proj:
        from .browserbase import create_browserbase_session

        conn = await cdp.connect((await create_browserbase_session(bb_key, bb_proj))["connectUrl"])
    else:
        conn = await cdp.launch_chrome(headless=knob("EXECUTOR_HEADLESS"))
    page = await conn.new_page()
    return Session(id=sid, page=page, dir=d, browser=conn)


def _driver() -> str:
    """``VWA_BROWSER_DRIVER``: playwright | cdp | auto (default: Playwright when importable)."""
    want = knob("VWA_BROWSER_DRIVER")
    if want != "auto":
        return want
    try:
        import playwright.async_api  # type: ignore  # noqa: F401
        return "playwright"
    except ImportError:
        return "cdp"


async def _playwright_factory(sid: str) -> Session:
    if _driver() == "cdp":
        return await _cdp_factory(sid)
    from playwright.async_api import async_playwright  # type: ignore
    d = os.path.join(artifacts_dir(), sid)
    os.makedirs(d, exist_ok=True)
    pw = await async_playwright().start()
    bb_key, bb_proj = knob("BROWSERBASE_API_KEY"), knob("BROWSERBASE_PROJECT_ID")
    if bb_key and bb_proj:
        from .browserbase import create_browserbase_session

        bb = await create_browserbase_session(bb_key, bb_proj)
        browser = await pw.chromium.connect_over_cdp(bb["connectUrl"])
        context = browser.contexts[0] if browser.contexts else await browser.new_context()
    else:
        headless = knob("EXECUTOR_HEADLESS")
        try:
            browser = await pw.chromium.launch(channel="chrome", headless=headless)
        except Exception:  # noqa: BLE001  (no branded Chrome: bundled chromium, as the legacy session.js)
            browser = await pw.chromium.launch(headless=headless)
        context = await browser.new_context(viewport={"width": 1366, "height": 768})
    page = await context.new_page()
    return Session(id=sid, page=page, dir=d, browser=browser, context=context, pw=pw)


class SessionManager:
    def __init__(self, factory: Optional[PageFactory] = None):
        self.factory = factory or _playwright_factory
        self.sessions: Dict[str, Session] = {}
        self._create_lock = asyncio.Lock()

    @staticmethod
    def _alive(s: Session) -> bool:
        try:
            closed = s.page.is_closed() if hasattr(s.page, "is_closed") else False
            if closed:
                return False
            if s.browser is not None and hasattr(s.browser, "is_connected"):
                return bool(s.browser.is_connected())
        except Exception:  # noqa: BLE001
            return False
        return True

    async def open_session(self, existing_id: Optional[str] = None) -> Session:
        async with self._create_lock:
            if existing_id and existing_id in self.sessions:
                s = self.sessions[existing_id]
                if self._alive(s):
                    return s
                await self.close_session(existing_id, _locked=True)
            sid = existing_id or str(uuid.uuid4())
            s = await self.factory(sid)
            self.sessions[sid] = s
            return s

    async def close_session(self, sid: str, _locked: bool = False) -> None:
        s = self.sessions.pop(sid, None)
        if s is None:
            return
        for obj, meth in ((s.context, "close"), (s.browser, "close"), (s.pw, "stop")):
            if obj is not None and hasattr(obj, meth):
                try:
                    await getattr(obj, meth)()
                except Exception:  # noqa: BLE001
                    pass

    def get_session(self, sid: str) -> Optional[Session]:
        return self.sessions.get(sid)
