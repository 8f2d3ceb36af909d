"""Playwright-free browser driver over the Chrome DevTools Protocol (CDP).

The reference drives Chrome through Playwright (apps/executor/src/session.ts:46-53, local Chrome)
or connects Playwright to a Browserbase CDP endpoint (session.ts:35-44).  Playwright is not part
of this image, so the executor would otherwise have no browser at all; this module speaks CDP
directly over one WebSocket (aiohttp) and exposes the subset of Playwright's async ``Page`` API
that ``executor/actions.py`` and ``executor/dom_analyzer.py`` call:

    goto, evaluate, wait_for_selector, wait_for_load_state, fill, press, click, select_option,
    set_input_files, go_back, go_forward, screenshot, keyboard.type / keyboard.press,
    get_by_text(...).first.click(), get_by_role(...).first.click(), is_closed

Endpoints:

* ``launch_chrome()`` starts a local Chrome / Chromium (``CHROME_PATH`` or the first of
  google-chrome / chromium / chromium-browser / chrome on PATH) with
  ``--remote-debugging-port=0`` and reads the browser WebSocket URL it prints;
* ``connect(endpoint)`` takes a ``ws://`` browser URL (e.g. Browserbase's ``connectUrl``) or an
  ``http://host:port`` DevTools address (resolved through ``/json/version``).

One browser connection multiplexes its pages with flattened target sessions
(``Target.attachToTarget {flatten: true}``): every command carries the page's ``sessionId``.
"""
from __future__ import annotations

import asyncio
import base64
import itertools
import json
import os
import re
import shutil
import subprocess
import tempfile
import threading
from typing import Any, Dict, List, Optional

import aiohttp
from ..utils.env import knob

# Keys Input.dispatchKeyEvent needs spelled out (Playwright key names)
_KEYS = {
    "Enter": dict(key="Enter", code="Enter", windowsVirtualKeyCode=13, text="\r"),
    "Tab": dict(key="Tab", code="Tab", windowsVirtualKeyCode=9),
    "Escape": dict(key="Escape", code="Escape", windowsVirtualKeyCode=27),
    "Backspace": dict(key="Backspace", code="Backspace", windowsVirtualKeyCode=8),
    "ArrowDown": dict(key="ArrowDown", code="ArrowDown", windowsVirtualKeyCode=40),
    "ArrowUp": dict(key="ArrowUp", code="ArrowUp", windowsVirtualKeyCode=38),
}

# element lookup shared by the page-side helpers: a CSS selector, or a marker attribute set by
# get_by_text / get_by_role on the element they resolved
_VISIBLE_JS = "(el) => !!el && (el.offsetWidth > 0 || el.offsetHeight > 0 || el.getClientRects().length > 0)"

_FILL_JS = r"""
(sel, value) => {
  const el = document.querySelector(sel);
  if (!el) return 'missing';
  el.scrollIntoView({block: 'center'});
  el.focus();
  const proto = el instanceof HTMLTextAreaElement ? HTMLTextAreaElement.prototype
              : el instanceof HTMLSelectElement ? HTMLSelectElement.prototype : HTMLInputElement.prototype;
  const desc = Object.getOwnPropertyDescriptor(proto, 'value');
  if (el.isContentEditable) el.textContent = value;
  else if (desc && desc.set) desc.set.call(el, value);
  else el.value = value;
  el.dispatchEvent(new Event('input', {bubbles: true}));
  el.dispatchEvent(new Event('change', {bubbles: true}));
  return 'ok';
}
"""

_CENTER_JS = r"""
(sel) => {
  const el = document.querySelector(sel);
  if (!el) return null;
  el.scrollIntoView({block: 'center', inline: 'center'});
  const r = el.getBoundingClientRect();
  if (r.width === 0 && r.height === 0) return null;
  return [r.left + r.width / 2, r.top + r.height / 2];
}
"""

_SELECT_JS = r"""
(sel, by, want) => {
  const el = document.querySelector(sel);
  if (!el || el.tagName !== 'SELECT') return 'missing';
  const opts = Array.from(el.options);
  const o = opts.find(o => by === 'label' ? (o.label || o.text).trim() === want : o.value === want);
  if (!o) return 'nooption';
  el.value = o.value;
  o.selected = true;
  el.dispatchEvent(new Event('input', {bubbles: true}));
  el.dispatchEvent(new Event('change', {bubbles: true}));
  return 'ok';
}
"""

# Marks the first visible element whose text (or aria-label / value) matches the pattern and
# returns a selector for it.  Innermost match wins (Playwright's getByText semantics).
_MARK_TEXT_JS = r"""
(src, flags, mark) => {
  const re = new RegExp(src, flags);
  const vis = (el) => el.offsetWidth > 0 || el.offsetHeight > 0 || el.getClientRects().length > 0;
  let best = null;
  for (const el of document.querySelectorAll('body *')) {
    if (!vis(el) || ['SCRIPT', 'STYLE', 'NOSCRIPT'].includes(el.tagName)) continue;
    const own = Array.from(el.childNodes).filter(n => n.nodeType === 3).map(n => n.textContent).join(' ');
    const txt = (own.trim() || el.getAttribute('aria-label') || (el.tagName === 'INPUT' ? el.value : '') || '').trim();
    if (txt && re.test(txt)) { best = el; break; }
  }
  if (!best) return null;
  best.setAttribute('data-vwa-mark', mark);
  return `[data-vwa-mark="${mark}"]`;
}
"""

_MARK_ROLE_JS = r"""
(role, name, mark) => {
  const implicit = {button: 'button,input[type=button],input[type=submit],input[type=reset]',
                    link: 'a[href]', textbox: 'input:not([type]),input[type=text],input[type=email],textarea',
                    searchbox: 'input[type=search]', checkbox: 'input[type=checkbox]', radio: 'input[type=radio]',
                    combobox: 'select', option: 'option', heading: 'h1,h2,h3,h4,h5,h6', img: 'img'};
  const cands = Array.from(document.querySelectorAll(`[role="${role}"]` + (implicit[role] ? ',' + implicit[role] : '')));
  const vis = (el) => el.offsetWidth > 0 || el.offsetHeight > 0 || el.getClientRects().length > 0;
  const low = (name || '').toLowerCase();
  for (const el of cands) {
    if (!vis(el)) continue;
    const acc = (el.getAttribute('aria-label') || el.innerText || el.value || el.getAttribute('title') || el.getAttribute('alt') || '').trim().toLowerCase();
    if (!low || acc.includes(low)) {
      el.setAttribute('data-vwa-mark', mark);
      return `[data-vwa-mark="${mark}"]`;
    }
  }
  return null;
}
"""


class CdpError(RuntimeError):
    pass


class CdpConnection:
    """One browser-level WebSocket: request/response by id, events dispatched to waiters."""

    def __init__(self, ws, http: aiohttp.ClientSession, proc: Optional[subprocess.Popen] = None,
                 profile_dir: Optional[str] = None):
        self.ws = ws
        self.http = http
        self.proc = proc
        self.profile_dir = profile_dir
        self._ids = itertools.count(1)
        self._pending: Dict[int, asyncio.Future] = {}
        self._waiters: List[tuple] = []  # (method, session_id, predicate, future)
        self._closed = False
        self._reader = asyncio.ensure_future(self._read())

    async def _read(self) -> None:
        try:
            async for msg in self.ws:
                if msg.type != aiohttp.WSMsgType.TEXT:
                    continue
                data = json.loads(msg.data)
                if "id" in data:
                    fut = self._pending.pop(data["id"], None)
                    if fut is not None and not fut.done():
                        if "error" in data:
                            fut.set_exception(CdpError(f"{data['error'].get('message')} ({data['error'].get('code')})"))
                        else:
                            fut.set_result(data.get("result", {}))
                    continue
                meth, sid, params = data.get("method"), data.get("sessionId"), data.get("params", {})
                for w in list(self._waiters):
                    m, s, pred, fut = w
                    if m == meth and (s is None or s == sid) and not fut.done() and (pred is None or pred(params)):
                        fut.set_result(params)
                        self._waiters.remove(w)
        finally:
            self._closed = True
            for fut in self._pending.values():
                if not fut.done():
                    fut.set_exception(CdpError("CDP connection closed"))
            self._pending.clear()

    @property
    def closed(self) -> bool:
        return self._closed

    async def send(self, method: str, params: Optional[Dict[str, Any]] = None, session_id: Optional[str] = None,
                   timeout: float = 30.0) -> Dict[str, Any]:
        if self._closed:
            raise CdpError("CDP connection closed")
        mid = next(self._ids)
        msg: Dict[str, Any] = {"id": mid, "method": method, "params": params or {}}
        if session_id:
            msg["sessionId"] = session_id
        fut = asyncio.get_running_loop().create_future()
        self._pending[mid] = fut
        await self.ws.send_str(json.dumps(msg))
        try:
            return await asyncio.wait_for(fut, timeout)
        finally:
            self._pending.pop(mid, None)

    def expect(self, method: str, session_id: Optional[str] = None, predicate=None) -> asyncio.Future:
        """A future for the next ``method`` event (register BEFORE the command that causes it)."""
        fut = asyncio.get_running_loop().create_future()
        self._waiters.append((method, session_id, predicate, fut))
        return fut

    async def new_page(self, viewport=(1366, 768)) -> "CdpPage":
        tid = (await self.send("Target.createTarget", {"url": "about:blank"}))["targetId"]
        sid = (await self.send("Target.attachToTarget", {"targetId": tid, "flatten": True}))["sessionId"]
        page = CdpPage(self, tid, sid)
        await page._init(viewport)
        return page

    async def close(self) -> None:
        if not self._closed:
            try:
                await self.send("Browser.close", timeout=5.0)
            except Exception:  # noqa: BLE001
                pass
        try:
            await self.ws.close()
        except Exception:  # noqa: BLE001
            pass
        self._reader.cancel()
        await self.http.close()
        if self.proc is not None:
            try:
                self.proc.terminate()
                self.proc.wait(timeout=5)
            except Exception:  # noqa: BLE001
                self.proc.kill()
        if self.profile_dir:
            shutil.rmtree(self.profile_dir, ignore_errors=True)

    def is_connected(self) -> bool:
        return not self._closed


class _Keyboard:
    def __init__(self, page: "CdpPage"):
        self.page = page

    async def type(self, text: str, delay: float = 0) -> None:
        for ch in text:
            await self.page._send("Input.dispatchKeyEvent", {"type": "keyDown", "text": ch, "key": ch})
            await self.page._send("Input.dispatchKeyEvent", {"type": "keyUp", "key": ch})
            if delay:
                await asyncio.sleep(delay / 1000.0)

    async def press(self, key: str) -> None:
        spec = _KEYS.get(key, dict(key=key, text=key if len(key) == 1 else None))
        down = {"type": "keyDown", **{k: v for k, v in spec.items() if v is not None}}
        await self.page._send("Input.dispatchKeyEvent", down)
        await self.page._send("Input.dispatchKeyEvent", {"type": "keyUp", "key": spec["key"],
                                                         **({"code": spec["code"]} if "code" in spec else {})})


class _Locator:
    """``page.get_by_text(...)`` / ``page.get_by_role(...)``: resolved lazily; ``.first`` is itself."""

    def __init__(self, page: "CdpPage", js: str, args: List[Any]):
        self.page, self.js, self.args = page, js, args

    @property
    def first(self) -> "_Locator":
        return self

    async def click(self, timeout: float = 15000) -> None:
        deadline = asyncio.get_running_loop().time() + timeout / 1000.0
        mark = f"m{next(self.page._marks)}"
        while True:
            sel = await self.page.evaluate(self.js, *self.args, mark)
            if sel:
                return await self.page.click(sel, timeout=max(1.0, (deadline - asyncio.get_running_loop().time()) * 1e3))
            if asyncio.get_running_loop().time() > deadline:
                raise TimeoutError(f"locator {self.args[:2]!r} resolved to no visible element")
            await asyncio.sleep(0.1)


class CdpPage:
    """The Playwright-Page subset the executor uses, over one flattened CDP target session."""

    def __init__(self, conn: CdpConnection, target_id: str, session_id: str):
        self.conn = conn
        self.target_id = target_id
        self.session_id = session_id
        self.keyboard = _Keyboard(self)
        self._marks = itertools.count(1)
        self._closed = False

    async def _send(self, method: str, params: Optional[Dict[str, Any]] = None, timeout: float = 30.0):
        return await self.conn.send(method, params, session_id=self.session_id, timeout=timeout)

    async def _init(self, viewport) -> None:
        await self._send("Page.enable")
        await self._send("Runtime.enable")
        if viewport:
            await self._send("Emulation.setDeviceMetricsOverride",
                             {"width": viewport[0], "height": viewport[1], "deviceScaleFactor": 1, "mobile": False})

    def is_closed(self) -> bool:
        return self._closed or self.conn.closed

    async def close(self) -> None:
        if not self._closed:
            self._closed = True
            try:
                await self.conn.send("Target.closeTarget", {"targetId": self.target_id})
            except Exception:  # noqa: BLE001
                pass

    # ------------------------------------------------------------------ script evaluation
    async def evaluate(self, expression: str, *args: Any) -> Any:
        """Playwright semantics: a function source is called with ``args``; anything else is an
        expression.  Promises are awaited, the result comes back by value (JSON)."""
        src = expression.strip()
        is_fn = bool(re.match(r"^(async\s+)?(function\b|\(|[A-Za-z_$][\w$]*\s*=>)", src))
        if is_fn:
            expr = f"({src})(...{json.dumps(list(args))})"
        else:
            expr = src
        r = await self._send("Runtime.evaluate", {"expression": expr, "returnByValue": True, "awaitPromise": True,
                                                  "userGesture": True})
        if "exceptionDetails" in r:
            ex = r["exceptionDetails"]
            raise CdpError("page script failed: " + str((ex.get("exception") or {}).get("description") or ex.get("text")))
        return (r.get("result") or {}).get("value")

    # ------------------------------------------------------------------ navigation
    async def _wait_ready(self, timeout: float, state: str = "domcontentloaded") -> None:
        want = ("interactive", "complete") if state == "domcontentloaded" else ("complete",)
        deadline = asyncio.get_running_loop().time() + timeout / 1000.0
        while True:
            try:
                rs = await self.evaluate("document.readyState")
                if rs in want:
                    return
            except CdpError:
                pass  # execution context being replaced by the navigation
            if asyncio.get_running_loop().time() > deadline:
                raise TimeoutError(f"page did not reach {state} within {timeout} ms")
            await asyncio.sleep(0.05)

    async def goto(self, url: str, wait_until: str = "domcontentloaded", timeout: float = 15000) -> None:
        ev = "Page.domContentEventFired" if wait_until == "domcontentloaded" else "Page.loadEventFired"
        fut = self.conn.expect(ev, self.session_id)
        r = await self._send("Page.navigate", {"url": url}, timeout=timeout / 1000.0)
        if r.get("errorText"):
            fut.cancel()
            raise CdpError(f"navigation to {url} failed: {r['errorText']}")
        try:
            await asyncio.wait_for(fut, timeout / 1000.0)
        except asyncio.TimeoutError:
            await self._wait_ready(1000, wait_until)

    async def wait_for_load_state(self, state: str = "load", timeout: float = 15000) -> None:
        await self._wait_ready(timeout, "domcontentloaded" if state == "domcontentloaded" else "load")

    async def _history(self, delta: int, timeout: float) -> None:
        h = await self._send("Page.getNavigationHistory")
        i = h["currentIndex"] + delta
        if not 0 <= i < len(h["entries"]):
            return  # Playwright returns null when there is no entry: not an error
        fut = self.conn.expect("Page.domContentEventFired", self.session_id)
        await self._send("Page.navigateToHistoryEntry", {"entryId": h["entries"][i]["id"]})
        try:
            await asyncio.wait_for(fut, timeout / 1000.0)
        except asyncio.TimeoutError:
            await self._wait_ready(1000)

    async def go_back(self, timeout: float = 15000) -> None:
        await self._history(-1, timeout)

    async def go_forward(self, timeout: float = 15000) -> None:
        await self._history(+1, timeout)

    # ------------------------------------------------------------------ element actions
    async def wait_for_selector(self, selector: str, timeout: float = 15000, state: str = "visible") -> None:
        deadline = asyncio.get_running_loop().time() + timeout / 1000.0
        js = f"(sel) => {{ const el = document.querySelector(sel); return ({_VISIBLE_JS})(el) ? 'visible' : el ? 'attached' : 'none'; }}"
        ok = ("visible",) if state == "visible" else ("visible", "attached")
        while True:
            if await self.evaluate(js, selector) in ok:
                return
            if asyncio.get_running_loop().time() > deadline:
                raise TimeoutError(f"waiting for selector {selector!r} ({state}) timed out after {timeout} ms")
            await asyncio.sleep(0.1)

    async def fill(self, selector: str, value: str, timeout: float = 15000) -> None:
        await self.wait_for_selector(selector, timeout=timeout)
        if await self.evaluate(_FILL_JS, selector, str(value)) != "ok":
            raise CdpError(f"fill: no element for {selector!r}")

    async def press(self, selector: str, key: str, timeout: float = 15000) -> None:
        await self.wait_for_selector(selector, timeout=timeout)
        await self.evaluate("(sel) => document.querySelector(sel).focus()", selector)
        await self.keyboard.press(key)

    async def click(self, selector: str, timeout: float = 15000) -> None:
        await self.wait_for_selector(selector, timeout=timeout)
        pt = await self.evaluate(_CENTER_JS, selector)
        if not pt:
            raise CdpError(f"click: {selector!r} has no box")
        x, y = float(pt[0]), float(pt[1])
        await self._send("Input.dispatchMouseEvent", {"type": "mouseMoved", "x": x, "y": y})
        for t in ("mousePressed", "mouseReleased"):
            await self._send("Input.dispatchMouseEvent", {"type": t, "x": x, "y": y, "button": "left", "clickCount": 1})

    async def select_option(self, selector: str, value: Optional[str] = None, label: Optional[str] = None,
                            timeout: float = 15000) -> List[str]:
        await self.wait_for_selector(selector, timeout=timeout, state="attached")
        by, want = ("label", label) if label is not None else ("value", value)
        r = await self.evaluate(_SELECT_JS, selector, by, str(want))
        if r != "ok":
            raise CdpError(f"select_option: {r} for {selector!r} ({by}={want!r})")
        return [str(want)]

    async def set_input_files(self, selector: str, files, timeout: float = 15000) -> None:
        await self.wait_for_selector(selector, timeout=timeout, state="attached")
        paths = [os.path.abspath(f) for f in ([files] if isinstance(files, str) else files)]
        root = (await self._send("DOM.getDocument", {"depth": 0}))["root"]["nodeId"]
        node = (await self._send("DOM.querySelector", {"nodeId": root, "selector": selector}))["nodeId"]
        if not node:
            raise CdpError(f"set_input_files: no element for {selector!r}")
        await self._send("DOM.setFileInputFiles", {"files": paths, "nodeId": node})

    def get_by_text(self, pattern) -> _Locator:
        if isinstance(pattern, re.Pattern):
            src, flags = pattern.pattern, "i" if pattern.flags & re.I else ""
        else:
            src, flags = re.escape(str(pattern)), "i"
        return _Locator(self, _MARK_TEXT_JS, [src, flags])

    def get_by_role(self, role: str, name: Optional[str] = None) -> _Locator:
        return _Locator(self, _MARK_ROLE_JS, [role, name or ""])

    # ------------------------------------------------------------------ screenshots
    async def screenshot(self, path: Optional[str] = None, full_page: bool = False) -> bytes:
        params: Dict[str, Any] = {"format": "png"}
        if full_page:
            m = await self._send("Page.getLayoutMetrics")
            cs = m.get("cssContentSize") or m.get("contentSize") or {}
            w, h = max(1, int(cs.get("width", 1366))), max(1, int(cs.get("height", 768)))
            params.update(clip={"x": 0, "y": 0, "width": w, "height": h, "scale": 1}, captureBeyondViewport=True)
        data = base64.b64decode((await self._send("Page.captureScreenshot", params, timeout=60.0))["data"])
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            with open(path, "wb") as f:
                f.write(data)
        return data


# ---------------------------------------------------------------------- endpoints
def find_chrome() -> Optional[str]:
    p = knob("CHROME_PATH")
    if p and os.path.isfile(p):
        return p
    for name in ("google-chrome", "google-chrome-stable", "chromium", "chromium-browser", "chrome"):
        w = shutil.which(name)
        if w:
            return w
    return None


async def connect(endpoint: str, proc: Optional[subprocess.Popen] = None,
                  profile_dir: Optional[str] = None) -> CdpConnection:
    http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None))
    try:
        ws_url = endpoint
        if endpoint.startswith("http://") or endpoint.startswith("https://"):
            async with http.get(endpoint.rstrip("/") + "/json/version") as r:
                ws_url = (await r.json(content_type=None))["webSocketDebuggerUrl"]
        ws = await http.ws_connect(ws_url, max_msg_size=0, heartbeat=None)
    except BaseException:
        await http.close()
        raise
    return CdpConnection(ws, http, proc, profile_dir)


def _drain(stream) -> None:
    try:
        for _ in stream:
            pass
    except (OSError, ValueError):
        pass


async def launch_chrome(headless: bool = True, executable: Optional[str] = None,
                        timeout: float = 30.0) -> CdpConnection:
    exe = executable or find_chrome()
    if not exe:
        raise RuntimeError("no Chrome / Chromium found (set CHROME_PATH) and playwright is not installed")
    prof = tempfile.mkdtemp(prefix="vwa-chrome-")
    args = [exe, "--remote-debugging-port=0", f"--user-data-dir={prof}", "--no-first-run",
            "--no-default-browser-check", "--window-size=1366,768", "--disable-dev-shm-usage"]
    if hasattr(os, "geteuid") and os.geteuid() == 0:
        args.append("--no-sandbox")  # Chrome refuses to run as root with its sandbox (Playwright's default too)
    args.append("about:blank")
    if headless:
        args.insert(1, "--headless=new")
    proc = subprocess.Popen(args, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    loop = asyncio.get_running_loop()

    def _read_url() -> Optional[str]:
        url = None
        for line in proc.stderr:  # "DevTools listening on ws://127.0.0.1:PORT/devtools/browser/<id>"
            m = re.search(r"DevTools listening on (ws://\S+)", line)
            if m:
                url = m.group(1)
                break
        if url is not None:
            # keep draining: Chrome logs to stderr for its whole life, and a full 64 KB pipe would
            # block its next log write (the browser hangs mid-session)
            threading.Thread(target=_drain, args=(proc.stderr,), name="chrome-stderr", daemon=True).start()
        return url

    try:
        url = await asyncio.wait_for(loop.run_in_executor(None, _read_url), timeout)
    except asyncio.TimeoutError:
        url = None
    if not url:
        proc.kill()
        shutil.rmtree(prof, ignore_errors=True)
        raise RuntimeError(f"{exe} did not report a DevTools endpoint")
    return await connect(url, proc, prof)
