"""Static server for the UI shell on :5173 (replaces the Vite dev server, apps/web/vite.config.ts:7-9)."""
from __future__ import annotations

import os

from aiohttp import web
from ..utils.env import knob

STATIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static")


def build_app() -> web.Application:
    app = web.Application()

    async def index(_req):
        return web.FileResponse(os.path.join(STATIC, "index.html"))

    app.router.add_get("/", index)
    app.router.add_static("/static/", STATIC)
    return app


def main():
    port = int(knob("WEB_PORT"))
    print(f"[web] http://127.0.0.1:{port}", flush=True)
    web.run_app(build_app(), host="127.0.0.1", port=port, print=None)


if __name__ == "__main__":
    main()
