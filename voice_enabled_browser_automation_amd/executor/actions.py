"""Intent interpreter: runs validated intents against a browser page.

Union of the reference's live TypeScript interpreter (apps/executor/src/actions.ts:28-304: DOM-
analysis targeting, scored search box, price-range filter, sort <select>, extract, scroll, back,
screenshot) and its older JavaScript one (apps/executor/src/actions.js: forward, wait_for,
upload, select, summarize, role/name clicks, selector-list fallbacks), as SURVEY.md §2.4
prescribes.  Differences from the reference, on purpose:

* ``retries`` (0..3) is honoured: a failing step is re-attempted ``retries`` more times;
* ``timeout_ms`` bounds every wait of the step (default 15000 ms, actions.ts:24-26);
* ``extract_table`` honours ``target.selector``, ``args.columns`` and ``args.limit``;
* ``upload`` resolves ``resume://<id>`` to the stored file WITH its extension (the reference
  drops it: server.ts:54 vs actions.js:194).

The page object is Playwright's async Page (or any object with the same methods: tests use a
fake).  Every step ends with a full-page screenshot, errors are caught per step and execution
continues (actions.ts:295-300).
"""
from __future__ import annotations

import asyncio
import glob
import os
import re
import time
from typing import Any, Dict, List, Optional

from .artifacts import screenshot_path, write_csv, write_json
from .dom_analyzer import DOMAnalyzer, best_search_element, find_by_selector, find_by_text
from ..utils.env import knob

DEFAULT_TIMEOUT_MS = 15000
SEARCH_WAIT_MS = 5000
LEGACY_SEARCH_SELECTORS = ['input[name="q"]', 'input[type="search"]', 'input[aria-label*="Search" i]',
                           'input[placeholder*="Search" i]', "#search", 'input[name*="search" i]']
UPLOAD_DIR = knob("UPLOAD_DIR")

EXTRACT_JS = r"""
([sel, limit, columns]) => {
  let cards = [];
  if (sel) {
    const root = document.querySelector(sel);
    if (root) cards = Array.from(root.querySelectorAll('[data-sku], li, article, .sku-item, .product, [data-testid*="product"], .item'));
    if (!cards.length) cards = Array.from(document.querySelectorAll(sel));
  }
  if (!cards.length) cards = Array.from(document.querySelectorAll('[data-testid*="product"], .product, .item, [data-sku], .sku-item, article'));
  const out = [];
  const priceRe = /\$\s?\d+[.,]?\d*/;
  for (const c of cards) {
    const text = (c.innerText || '').trim();
    if (!text) continue;
    const row = {};
    const head = c.querySelector('h1,h2,h3,h4,a');
    row.title = ((head && head.innerText) || text).trim().split(/\s+/).slice(0, 8).join(' ');
    const m = text.match(priceRe);
    row.price = m ? m[0] : '';
    for (const col of (columns || [])) {
      if (col in row) continue;
      const el = c.querySelector(`[class*="${col}" i], [data-test*="${col}" i], [aria-label*="${col}" i]`);
      if (el) row[col] = (el.innerText || el.getAttribute('href') || '').trim();
      else if (col === 'url') { const a = c.querySelector('a[href]'); row[col] = a ? a.href : ''; }
      else row[col] = '';
    }
    out.push(row);
    if (out.length >= limit) break;
  }
  return out;
}
"""


def _tmo(intent: Dict[str, Any]) -> int:
    t = intent.get("timeout_ms")
    return int(t) if isinstance(t, (int, float)) and t > 0 else DEFAULT_TIMEOUT_MS


def resolve_file_ref(ref: str, upload_dir: str = UPLOAD_DIR) -> Optional[str]:
    if not isinstance(ref, str):
        return None
    if ref.startswith("resume://"):
        fid = ref[len("resume://"):]
        if fid == "latest":
            files = sorted(glob.glob(os.path.join(upload_dir, "*")), key=os.path.getmtime)
            return files[-1] if files else None
        for cand in [os.path.join(upload_dir, fid)] + sorted(glob.glob(os.path.join(upload_dir, glob.escape(fid) + ".*"))):
            if os.path.isfile(cand):
                return cand
        return None
    return ref if os.path.isfile(ref) else None


class IntentRunner:
    def __init__(self, page, artifact_dir: str, upload_dir: str = UPLOAD_DIR):
        self.page = page
        self.dir = artifact_dir
        self.upload_dir = upload_dir
        self._analysis: Optional[Dict[str, Any]] = None

    async def cap(self, label: str) -> Optional[str]:
        path = screenshot_path(self.dir, label)
        try:
            await self.page.screenshot(path=path, full_page=True)
            return path
        except Exception:  # noqa: BLE001
            return None

    async def analysis(self) -> Dict[str, Any]:
        if self._analysis is None:
            self._analysis = await DOMAnalyzer(self.page).analyze_page()
        return self._analysis

    def invalidate(self) -> None:
        self._analysis = None

    # ------------------------------------------------------------------ handlers
    async def do_navigate(self, it, step):
        url = (it.get("args") or {}).get("url")
        if not url:
            raise ValueError("navigate requires args.url")
        if not re.match(r"^[a-zA-Z][a-zA-Z0-9+.-]*:", url):
            url = "https://" + url
        await self.page.goto(url, wait_until="domcontentloaded", timeout=_tmo(it))
        self.invalidate()
        step["screenshot"] = await self.cap("navigate")

    async def do_search(self, it, step):
        q = (it.get("args") or {}).get("query") or (it.get("args") or {}).get("q")
        if not q:
            raise ValueError("search requires args.query")
        sel = None
        try:
            a = await self.analysis()
            best = best_search_element(a)
            if best:
                sel = best["selector"]
                step["pageAnalysis"] = {"searchElements": len(a.get("searchElements", [])), "chosen": sel}
        except Exception:  # noqa: BLE001
            sel = None
        tried = []
        for cand in ([sel] if sel else []) + LEGACY_SEARCH_SELECTORS:
            tried.append(cand)
            try:
                await self.page.wait_for_selector(cand, timeout=min(SEARCH_WAIT_MS, _tmo(it)), state="visible")
                await self.page.fill(cand, str(q))
                await self.page.press(cand, "Enter")
                step["data"] = {"selector": cand}
                break
            except Exception:  # noqa: BLE001
                continue
        else:
            # legacy last resort: type into the focused page and submit (actions.js:54-58)
            await self.page.keyboard.type(str(q), delay=20)
            await self.page.keyboard.press("Enter")
            step["data"] = {"selector": None, "tried": tried}
        self.invalidate()
        step["screenshot"] = await self.cap("search")

    async def do_click(self, it, step):
        tgt = it.get("target") or {}
        text, sel, role, name = tgt.get("text"), tgt.get("selector"), tgt.get("role"), tgt.get("name")
        if text:
            try:
                a = await self.analysis()
                el = find_by_text(a, text)
            except Exception:  # noqa: BLE001
                el = None
            if el:
                await self.page.click(el["selector"], timeout=_tmo(it))
            else:
                await self.page.get_by_text(re.compile(re.escape(text), re.I)).first.click(timeout=_tmo(it))
        elif sel:
            await self.page.click(sel, timeout=_tmo(it))
        elif role:
            await self.page.get_by_role(role, name=name).first.click(timeout=_tmo(it))
        elif name:
            await self.page.get_by_text(re.compile(re.escape(name), re.I)).first.click(timeout=_tmo(it))
        else:
            raise ValueError("click requires target.text, target.selector or target.role")
        self.invalidate()
        step["screenshot"] = await self.cap("click")

    async def do_filter(self, it, step):
        args = it.get("args") or {}
        price = args.get("price") if isinstance(args.get("price"), dict) else {}
        lte = price.get("lte", args.get("max", args.get("price_max")))
        gte = price.get("gte", args.get("min", args.get("price_min")))
        if lte is None and gte is None:
            raise ValueError("filter requires args.price.{lte,gte}")
        done = False
        try:
            a = await self.analysis()
            for f in a.get("filters", []):
                els = f.get("elements", [])
                if f.get("type") == "range" and len(els) >= 2:
                    if gte is not None:
                        await self.page.fill(els[0]["selector"], str(gte))
                    if lte is not None:
                        await self.page.fill(els[1]["selector"], str(lte))
                        await self.page.press(els[1]["selector"], "Enter")
                    done = True
                    break
        except Exception:  # noqa: BLE001
            done = False
        if not done:  # legacy (actions.js:62-76)
            if lte is not None:
                s = 'input[aria-label*="Max" i]'
                await self.page.fill(s, str(lte))
                await self.page.press(s, "Enter")
            if gte is not None:
                s = 'input[aria-label*="Min" i]'
                await self.page.fill(s, str(gte))
                await self.page.press(s, "Enter")
        self.invalidate()
        step["screenshot"] = await self.cap("filter")

    async def do_sort(self, it, step):
        args = it.get("args") or {}
        by = str(args.get("by", "price")).lower()
        order = str(args.get("order", "asc")).lower()
        asc = order in ("asc", "ascending", "low", "low to high")
        label = f"{by} low to high" if asc else f"{by} high to low"
        done = False
        try:
            a = await self.analysis()
            for f in a.get("filters", []):
                if f.get("type") != "dropdown":
                    continue
                el = f["elements"][0]
                attrs = el.get("attributes") or {}
                if "sort" in (attrs.get("name", "") + attrs.get("id", "") + f.get("label", "")).lower():
                    for lab in (label, label.title(), label.capitalize()):
                        try:
                            await self.page.select_option(el["selector"], label=lab, timeout=_tmo(it))
                            done = True
                            break
                        except Exception:  # noqa: BLE001
                            continue
                if done:
                    break
        except Exception:  # noqa: BLE001
            done = False
        if not done:  # legacy: open a Sort control, pick the option by text (actions.js:77-101)
            await self.page.get_by_text(re.compile(r"sort", re.I)).first.click(timeout=_tmo(it))
            pat = r"low to high" if asc else r"high to low"
            await self.page.get_by_text(re.compile(pat, re.I)).first.click(timeout=_tmo(it))
        step["data"] = {"by": by, "order": "asc" if asc else "desc"}
        self.invalidate()
        step["screenshot"] = await self.cap("sort")

    async def do_type(self, it, step):
        sel = (it.get("target") or {}).get("selector")
        val = (it.get("args") or {}).get("value", (it.get("args") or {}).get("text"))
        if not sel or val is None:
            raise ValueError("type requires target.selector and args.value")
        await self.page.fill(sel, str(val), timeout=_tmo(it))
        step["screenshot"] = await self.cap("type")

    async def do_select(self, it, step):
        sel = (it.get("target") or {}).get("selector")
        val = (it.get("args") or {}).get("value")
        if not sel or val is None:
            raise ValueError("select requires target.selector and args.value")
        try:
            await self.page.select_option(sel, label=str(val), timeout=_tmo(it))
        except Exception:  # noqa: BLE001
            await self.page.select_option(sel, value=str(val), timeout=_tmo(it))
        step["screenshot"] = await self.cap("select")

    async def do_extract_table(self, it, step):
        args = it.get("args") or {}
        sel = (it.get("target") or {}).get("selector")
        limit = int(args.get("limit", 10) or 10)
        cols = args.get("columns") if isinstance(args.get("columns"), list) else []
        if sel:
            try:
                await self.page.wait_for_selector(sel, timeout=_tmo(it))
            except Exception:  # noqa: BLE001
                pass
        rows = await self.page.evaluate(EXTRACT_JS, [sel, limit, [str(c) for c in cols]])
        rows = rows if isinstance(rows, list) else []
        rows = rows[:limit]
        if cols:
            rows = [{c: r.get(c, "") for c in cols} for r in rows]
        base = f"extract-{int(time.time() * 1000)}"
        step["data"] = rows
        step["data_paths"] = {"json": write_json(self.dir, base + ".json", rows),
                              "csv": write_csv(self.dir, base + ".csv", rows)}
        step["screenshot"] = await self.cap("extract")

    async def do_scroll(self, it, step):
        args = it.get("args") or {}
        px = int(args.get("pixels", 800) or 800)
        dy = -px if str(args.get("direction", "down")).lower() == "up" else px
        await self.page.evaluate("(dy) => window.scrollBy({top: dy, behavior: 'smooth'})", dy)
        step["screenshot"] = await self.cap("scroll")

    async def do_back(self, it, step):
        await self.page.go_back(timeout=_tmo(it))
        self.invalidate()
        step["screenshot"] = await self.cap("back")

    async def do_forward(self, it, step):
        await self.page.go_forward(timeout=_tmo(it))
        self.invalidate()
        step["screenshot"] = await self.cap("forward")

    async def do_wait_for(self, it, step):
        args = it.get("args") or {}
        sel = args.get("selector") or (it.get("target") or {}).get("selector")
        tmo = int(args.get("timeoutMs", it.get("timeout_ms") or DEFAULT_TIMEOUT_MS))
        if not sel:
            raise ValueError("wait_for requires args.selector")
        await self.page.wait_for_selector(sel, timeout=tmo, state="visible")
        step["screenshot"] = await self.cap("wait_for")

    async def do_upload(self, it, step):
        ref = (it.get("args") or {}).get("fileRef")
        path = resolve_file_ref(ref, self.upload_dir)
        if not path:
            raise FileNotFoundError(f"file not found for fileRef {ref!r}")
        sel = (it.get("target") or {}).get("selector") or 'input[type="file"]'
        await self.page.set_input_files(sel, path, timeout=_tmo(it))
        step["data"] = {"file": os.path.basename(path)}
        step["screenshot"] = await self.cap("upload")

    async def do_screenshot(self, it, step):
        step["screenshot"] = await self.cap((it.get("args") or {}).get("label") or "screenshot")

    async def do_summarize(self, it, step):
        step["data"] = {"note": "summarize should be handled by the brain"}

    HANDLERS = {
        "navigate": do_navigate, "search": do_search, "click": do_click, "filter": do_filter, "sort": do_sort,
        "type": do_type, "select": do_select, "extract_table": do_extract_table, "scroll": do_scroll,
        "back": do_back, "forward": do_forward, "wait_for": do_wait_for, "upload": do_upload,
        "screenshot": do_screenshot, "summarize": do_summarize,
    }

    async def run(self, intents: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
        results = []
        for it in intents:  # array order = execution order (priority is informational, as in the reference)
            step: Dict[str, Any] = {"intent": it, "ok": True}
            h = self.HANDLERS.get(it.get("type"))
            if h is None:
                step["ok"] = False
                step["error"] = f"Unsupported intent type: {it.get('type')}"
                results.append(step)
                continue
            attempts = 1 + max(0, min(3, int(it.get("retries", 0) or 0)))
            t0 = time.perf_counter()
            for a in range(attempts):
                try:
                    await h(self, it, step)
                    step["ok"] = True
                    step.pop("error", None)
                    break
                except Exception as e:  # noqa: BLE001
                    step["ok"] = False
                    step["error"] = str(e) or e.__class__.__name__
                    if a + 1 < attempts:
                        await asyncio.sleep(0.2)
                        self.invalidate()
            step["attempts"] = a + 1
            step["latencyMs"] = round((time.perf_counter() - t0) * 1e3, 2)
            results.append(step)
        return results


async def run_intents(page, artifact_dir: str, intents: List[Dict[str, Any]], upload_dir: str = UPLOAD_DIR):
    """apps/executor/src/actions.ts:28 `runIntents(page, dir, intents)`."""
    return await IntentRunner(page, artifact_dir, upload_dir).run(intents)
