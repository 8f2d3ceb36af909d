"""Test doubles: a duck-typed async Playwright Page (like apps/executor/test/actions.test.ts:5-24)."""
import re


class FakeLocator:
    def __init__(self, page, kind, arg):
        self.page, self.kind, self.arg = page, kind, arg

    @property
    def first(self):
        return self

    async def click(self, timeout=None):
        self.page.calls.append(("locator_click", self.kind, getattr(self.arg, "pattern", self.arg)))
        if self.page.fail_locators:
            raise TimeoutError("locator not found")


class FakeKeyboard:
    def __init__(self, page):
        self.page = page

    async def type(self, text, delay=0):
        self.page.calls.append(("kb_type", text))

    async def press(self, key):
        self.page.calls.append(("kb_press", key))


class FakePage:
    def __init__(self, analysis=None, extract_rows=None, missing_selectors=(), fail_locators=False):
        self.calls = []
        self.url = "about:blank"
        self.history = []
        self.fwd = []
        self.analysis = analysis if analysis is not None else {
            "url": "about:blank", "title": "Fake", "searchElements": [
                {"selector": "input[name=\"q\"]", "type": "input", "placeholder": "Search", "attributes": {"name": "q"},
                 "bbox": {"width": 300}, "isVisible": True, "isEnabled": True}],
            "buttons": [{"selector": "#buy", "type": "button", "text": "Add to cart", "attributes": {}}],
            "links": [], "forms": [],
            "filters": [{"type": "dropdown", "label": "sort", "elements": [{"selector": "#sort", "attributes": {"id": "sort"}}]},
                        {"type": "range", "label": "price", "elements": [{"selector": "#min"}, {"selector": "#max"}]}],
            "navigationElements": []}
        self.extract_rows = extract_rows if extract_rows is not None else [{"title": "X", "price": "$9.99"}]
        self.missing = set(missing_selectors)
        self.fail_locators = fail_locators
        self.keyboard = FakeKeyboard(self)
        self.closed = False

    def is_closed(self):
        return self.closed

    async def goto(self, url, wait_until=None, timeout=None):
        self.calls.append(("goto", url))
        self.history.append(self.url)
        self.url = url

    async def wait_for_load_state(self, state=None):
        self.calls.append(("load_state", state))

    async def title(self):
        return "Fake"

    async def evaluate(self, script, arg=None):
        self.calls.append(("evaluate", script[:40], arg))
        if "searchElements" in script:
            return self.analysis
        if "priceRe" in script:
            return self.extract_rows
        return None

    async def screenshot(self, path=None, full_page=False):
        self.calls.append(("screenshot", path))
        if path:
            with open(path, "wb") as fh:
                fh.write(b"\x89PNG")

    async def wait_for_selector(self, sel, timeout=None, state=None):
        self.calls.append(("wait_for_selector", sel, timeout))
        if sel in self.missing:
            raise TimeoutError(f"timeout waiting for {sel}")

    async def fill(self, sel, value, timeout=None):
        if sel in self.missing:
            raise TimeoutError(sel)
        self.calls.append(("fill", sel, value))

    async def press(self, sel, key, timeout=None):
        self.calls.append(("press", sel, key))

    async def click(self, sel, timeout=None):
        if sel in self.missing:
            raise TimeoutError(sel)
        self.calls.append(("click", sel))

    async def select_option(self, sel, label=None, value=None, timeout=None):
        if label is not None and "high to low" not in label.lower() and "low to high" not in label.lower() and sel == "#strict":
            raise ValueError("no such label")
        self.calls.append(("select_option", sel, label, value))

    async def go_back(self, timeout=None):
        self.calls.append(("go_back",))

    async def go_forward(self, timeout=None):
        self.calls.append(("go_forward",))

    async def set_input_files(self, sel, path, timeout=None):
        self.calls.append(("set_input_files", sel, path))

    def get_by_text(self, pattern):
        return FakeLocator(self, "text", pattern)

    def get_by_role(self, role, name=None):
        return FakeLocator(self, "role", (role, name))

    def names(self):
        return [c[0] for c in self.calls]
