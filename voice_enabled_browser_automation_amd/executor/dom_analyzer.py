"""DOM analyzer: page introspection for element targeting (apps/executor/src/dom-analyzer.ts).

The reference issues six `$$eval` round trips per analysis (:41-74), one of them over every DOM
node (`$$eval("*")`, :310).  Here ONE `page.evaluate` runs a single script in the page that
returns the whole `PageAnalysis` (url, title, searchElements, buttons, links, forms, filters,
navigationElements), walking the document once.  Selector synthesis keeps the reference's order
(`#id` -> `[data-testid=...]` -> `tag[name=...]` -> bare tag; :78-86) and visibility test
(offsetHeight > 0).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

ANALYZE_JS = r"""
() => {
  // ids / attribute values are escaped: an id like "a:b" or "x.y" (frequent in framework-generated
  // markup) is otherwise a broken selector -- the reference synthesises them raw
  // (dom-analyzer.ts:78-86)
  const ident = (s) => (window.CSS && CSS.escape) ? CSS.escape(s) : s.replace(/([^A-Za-z0-9_-])/g, '\\$1');
  const qv = (s) => s.replace(/\\/g, '\\\\').replace(/"/g, '\\"');
  const sel = (el) => {
    if (el.id) return '#' + ident(el.id);
    const dt = el.getAttribute('data-testid');
    if (dt) return `[data-testid="${qv(dt)}"]`;
    const nm = el.getAttribute('name');
    const tag = el.tagName.toLowerCase();
    if (nm) return `${tag}[name="${qv(nm)}"]`;
    return tag;
  };
  const attrs = (el) => { const a = {}; for (const x of Array.from(el.attributes)) a[x.name] = x.value; return a; };
  const box = (el) => { const r = el.getBoundingClientRect(); return {x: r.x, y: r.y, width: r.width, height: r.height}; };
  const desc = (el, type) => ({
    selector: sel(el), type,
    text: ((el.innerText || el.value || '') + '').trim().slice(0, 200),
    placeholder: el.getAttribute('placeholder') || '',
    attributes: attrs(el), bbox: box(el),
    isVisible: el.offsetHeight > 0, isEnabled: !el.disabled,
  });
  const low = (s) => (s || '').toLowerCase();
  const out = {url: location.href, title: document.title, searchElements: [], buttons: [], links: [],
               forms: [], filters: [], navigationElements: []};
  for (const inp of Array.from(document.querySelectorAll('input'))) {
    const t = low(inp.type), ph = low(inp.placeholder), al = low(inp.getAttribute('aria-label')),
          nm = low(inp.name), id = low(inp.id);
    if (t === 'search' || ph.includes('search') || al.includes('search') || nm.includes('search') || nm === 'q' || id.includes('search'))
      out.searchElements.push(desc(inp, 'input'));
  }
  for (const b of Array.from(document.querySelectorAll('button, input[type="button"], input[type="submit"], [role="button"]')))
    if (b.offsetHeight > 0) out.buttons.push(desc(b, 'button'));
  for (const a of Array.from(document.querySelectorAll('a[href]')).slice(0, 500)) {
    if (a.offsetHeight > 0) out.links.push(desc(a, 'link'));
  }
  for (const f of Array.from(document.querySelectorAll('form'))) {
    const inputs = Array.from(f.querySelectorAll('input, textarea, select')).map((e) => desc(e, e.tagName.toLowerCase() === 'select' ? 'select' : (e.tagName.toLowerCase() === 'textarea' ? 'textarea' : 'input')));
    const sb = f.querySelector('button[type="submit"], input[type="submit"], button');
    out.forms.push({selector: sel(f), inputs, submitButton: sb ? desc(sb, 'button') : undefined});
  }
  // filters: selects, checkbox groups, numeric range inputs (price min/max), text filters
  for (const s of Array.from(document.querySelectorAll('select'))) {
    const lab = s.getAttribute('aria-label') || s.name || s.id || '';
    out.filters.push({type: 'dropdown', label: lab, elements: [desc(s, 'select')]});
  }
  const ranges = {};
  for (const inp of Array.from(document.querySelectorAll('input[type="number"], input[inputmode="numeric"], input[type="text"]'))) {
    const key = low(inp.getAttribute('aria-label') + ' ' + inp.name + ' ' + inp.placeholder + ' ' + inp.id);
    if (key.includes('price') || key.includes('min') || key.includes('max')) {
      const grp = key.includes('price') ? 'price' : 'range';
      (ranges[grp] = ranges[grp] || []).push(desc(inp, 'input'));
    }
  }
  for (const [lab, els] of Object.entries(ranges)) out.filters.push({type: 'range', label: lab, elements: els});
  const boxes = Array.from(document.querySelectorAll('input[type="checkbox"]')).slice(0, 50);
  if (boxes.length) out.filters.push({type: 'checkbox', label: 'checkboxes', elements: boxes.map((b) => desc(b, 'input'))});
  for (const n of Array.from(document.querySelectorAll('nav a, [role="navigation"] a, header a')).slice(0, 100))
    out.navigationElements.push(desc(n, 'link'));
  return out;
}
"""


def css_ident(s: str) -> str:
    """The selector synthesis' identifier escaping (ANALYZE_JS ``ident`` without CSS.escape):
    every character outside [A-Za-z0-9_-] backslash-escaped."""
    return "".join(c if (c.isascii() and (c.isalnum() or c in "_-")) else "\\" + c for c in s)


def synth_selector(tag: str, attrs: Dict[str, str]) -> str:
    """Python mirror of ANALYZE_JS ``sel`` (tests; same order as dom-analyzer.ts:78-86)."""
    def qv(v: str) -> str:
        return v.replace("\\", "\\\\").replace('"', '\\"')

    if attrs.get("id"):
        return "#" + css_ident(attrs["id"])
    if attrs.get("data-testid"):
        return f'[data-testid="{qv(attrs["data-testid"])}"]'
    if attrs.get("name"):
        return f'{tag.lower()}[name="{qv(attrs["name"])}"]'
    return tag.lower()


class DOMAnalyzer:
    def __init__(self, page):
        self.page = page

    async def analyze_page(self) -> Dict[str, Any]:
        try:
            await self.page.wait_for_load_state("domcontentloaded")
        except Exception:  # noqa: BLE001
            pass
        res = await self.page.evaluate(ANALYZE_JS)
        if not isinstance(res, dict):
            res = {}
        for k in ("searchElements", "buttons", "links", "forms", "filters", "navigationElements"):
            res.setdefault(k, [])
        res.setdefault("url", getattr(self.page, "url", ""))
        res.setdefault("title", "")
        return res


def search_element_score(el: Dict[str, Any]) -> int:
    """apps/executor/src/actions.ts:318-329 scoring."""
    a = el.get("attributes", {}) or {}
    s = 0
    if (a.get("name") or "") == "q":
        s += 10
    if (a.get("type") or "").lower() == "search":
        s += 8
    if "search" in (el.get("placeholder") or "").lower():
        s += 6
    if "search" in (a.get("aria-label") or "").lower():
        s += 5
    bbox = el.get("bbox") or {}
    if (bbox.get("width") or 0) > 200:
        s += 2
    return s


def best_search_element(analysis: Dict[str, Any]) -> Optional[Dict[str, Any]]:
    cands = [e for e in analysis.get("searchElements", []) if e.get("isVisible", True) and e.get("isEnabled", True)]
    if not cands:
        return None
    return max(cands, key=search_element_score)


def find_by_text(analysis: Dict[str, Any], text: str) -> Optional[Dict[str, Any]]:
    t = text.lower()
    for e in list(analysis.get("buttons", [])) + list(analysis.get("links", [])):
        if t in (e.get("text") or "").lower() or t in ((e.get("attributes") or {}).get("aria-label") or "").lower():
            return e
    return None


def find_by_selector(analysis: Dict[str, Any], selector: str) -> Optional[Dict[str, Any]]:
    for e in list(analysis.get("buttons", [])) + list(analysis.get("links", [])) + list(analysis.get("searchElements", [])):
        if e.get("selector") == selector:
            return e
    return None
