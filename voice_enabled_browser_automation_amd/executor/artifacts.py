"""Artifact writers (apps/executor/src/artifacts.ts:4-26): JSON / CSV outputs and screenshot paths."""
from __future__ import annotations

import csv
import json
import os
import time
from typing import Any, Dict, List


def write_json(dir_: str, name: str, data: Any) -> str:
    os.makedirs(dir_, exist_ok=True)
    path = os.path.join(dir_, name)
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(data, fh, indent=2, ensure_ascii=False)
    return path


def write_csv(dir_: str, name: str, rows: List[Dict[str, Any]]) -> str:
    os.makedirs(dir_, exist_ok=True)
    path = os.path.join(dir_, name)
    headers: List[str] = []
    for r in rows:
        for k in r.keys():
            if k not in headers:
                headers.append(k)
    with open(path, "w", encoding="utf-8", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=headers)
        w.writeheader()
        for r in rows:
            w.writerow({k: r.get(k, "") for k in headers})
    return path


def screenshot_path(dir_: str, label: str) -> str:
    """`<dir>/<ms>-<label>.png` (apps/executor/src/actions.ts:37-41)."""
    os.makedirs(dir_, exist_ok=True)
    safe = "".join(ch if ch.isalnum() or ch in "-_" else "_" for ch in label)[:64] or "step"
    return os.path.join(dir_, f"{int(time.time() * 1000)}-{safe}.png")
