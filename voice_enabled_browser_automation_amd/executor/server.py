"""Executor service: ``GET /health``, ``POST /uploads``, ``POST /execute``, ``POST /close``,
``GET /metrics`` (parity with apps/executor/src/server.ts:23-100; CORS ``origin: true``).

/execute validates an ExecuteRequest (400 ``invalid_request``), opens or reuses the browser
session, runs the intents under the session's lock and replies
``{session_id, results: StepResult[], artifacts: {dir}}``.
/uploads takes a multipart body, stores the first file as ``.uploads/<uuid><ext>`` and replies
``{fileRef: "resume://<uuid>", path}`` (the interpreter resolves the extension).
"""
from __future__ import annotations

import os
import time
import uuid
from typing import Optional

from aiohttp import web

from ..contracts import ExecuteRequest, safe_parse
from ..utils.metrics import Metrics
from .actions import run_intents
from .session import SessionManager
from ..utils.env import knob


@web.middleware
async def cors(request: web.Request, handler):
    origin = request.headers.get("Origin", "*")
    if request.method == "OPTIONS":
        resp = web.Response(status=204)
    else:
        resp = await handler(request)
    resp.headers["Access-Control-Allow-Origin"] = origin
    resp.headers["Vary"] = "Origin"
    resp.headers["Access-Control-Allow-Methods"] = "GET,POST,OPTIONS"
    resp.headers["Access-Control-Allow-Headers"] = request.headers.get("Access-Control-Request-Headers", "content-type")
    return resp


def build_app(sessions: Optional[SessionManager] = None, upload_dir: Optional[str] = None) -> web.Application:
    app = web.Application(middlewares=[cors], client_max_size=64 * 1024 * 1024)
    app["sessions"] = sessions or SessionManager()
    app["upload_dir"] = upload_dir or knob("UPLOAD_DIR")
    app["metrics"] = Metrics("executor")

    async def health(_req):
        return web.json_response({"status": "ok", "service": "executor"})

    async def metrics(_req):
        return web.json_response(app["metrics"].snapshot())

    async def uploads(req: web.Request):
        reader = await req.multipart()
        os.makedirs(app["upload_dir"], exist_ok=True)
        async for part in reader:
            if part.filename is None:
                continue
            fid = str(uuid.uuid4())
            ext = os.path.splitext(part.filename)[1][:16]
            path = os.path.join(app["upload_dir"], fid + ext)
            with open(path, "wb") as fh:
                while True:
                    chunk = await part.read_chunk(1 << 16)
                    if not chunk:
                        break
                    fh.write(chunk)
            app["metrics"].inc("uploads")
            return web.json_response({"fileRef": f"resume://{fid}", "path": os.path.abspath(path)})
        return web.json_response({"error": "no file"}, status=500)

    async def execute(req: web.Request):
        m: Metrics = app["metrics"]
        try:
            body = await req.json()
        except Exception:  # noqa: BLE001
            body = None
        pr = safe_parse(ExecuteRequest, body)
        if not pr.success:
            m.inc("invalid_request")
            return web.json_response({"error": "invalid_request", "detail": pr.format_error()}, status=400)
        data = pr.data
        t0 = time.perf_counter()
        s = await app["sessions"].open_session(data.get("session_id"))
        async with s.lock:
            results = await run_intents(s.page, s.dir, data["intents"], upload_dir=app["upload_dir"])
        for r in results:
            m.inc("steps_ok" if r.get("ok") else "steps_failed")
            if "latencyMs" in r:
                m.observe("step_ms", r["latencyMs"])
        m.observe("execute_ms", (time.perf_counter() - t0) * 1e3)
        return web.json_response({"session_id": s.id, "results": results, "artifacts": {"dir": s.dir}})

    async def close(req: web.Request):
        try:
            body = await req.json()
        except Exception:  # noqa: BLE001
            body = {}
        sid = body.get("session_id") if isinstance(body, dict) else None
        if not sid:
            return web.json_response({"error": "session_id required"}, status=400)
        await app["sessions"].close_session(sid)
        return web.json_response({"ok": True})

    app.router.add_get("/health", health)
    app.router.add_get("/metrics", metrics)
    app.router.add_post("/uploads", uploads)
    app.router.add_post("/execute", execute)
    app.router.add_post("/close", close)
    app.router.add_route("OPTIONS", "/{tail:.*}", lambda r: web.Response(status=204))
    return app


def main():
    from ..utils.env import load_dotenv

    load_dotenv()
    port = knob("EXECUTOR_PORT")
    print(f"[executor] listening on http://127.0.0.1:{port}", flush=True)
    web.run_app(build_app(), host="127.0.0.1", port=port, print=None)


if __name__ == "__main__":
    main()
