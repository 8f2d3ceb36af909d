"""Browserbase remote-browser session creation over REST (apps/executor/src/browserbase.ts:10-39).

``POST {BROWSERBASE_API_BASE}/sessions`` with header ``X-BB-API-Key`` and ``{"projectId": ...}``;
the reply's ``connectUrl`` is a CDP endpoint Playwright connects to.
"""
from __future__ import annotations

import os
from typing import Any, Dict

import aiohttp
from ..utils.env import knob


async def create_browserbase_session(api_key: str, project_id: str, api_base: str = "") -> Dict[str, Any]:
    base = api_base or knob("BROWSERBASE_API_BASE")
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=60)) as s:
        async with s.post(f"{base}/sessions", json={"projectId": project_id},
                          headers={"X-BB-API-Key": api_key, "Content-Type": "application/json"}) as r:
            if r.status >= 300:
                raise RuntimeError(f"Browserbase session create failed: {r.status} {await r.text()}")
            data = await r.json()
    if "connectUrl" not in data:
        raise RuntimeError("Browserbase reply has no connectUrl")
    return data
