"""Start the four services (brain :8090, voice :7072, executor :7081, web :5173) as separate
processes, like ``pnpm dev`` in each app of the reference (README.md:83-97).

    python -m voice_enabled_browser_automation_amd.launch            # keyword brain, no ASR (CPU)
    VWA_BRAIN_ENGINE=llm VWA_ASR_ENGINE=whisper python -m voice_enabled_browser_automation_amd.launch

GPU placement on one node (plan_gpus): the brain (LLM) takes GPUs 0..TP-1 and the voice service
(ASR) every remaining GPU, one voice worker per GPU behind the session router (session DP);
VWA_BRAIN_GPUS / VWA_VOICE_GPUS (comma lists) override.  With VWA_TP>1 the brain is launched
through torch.distributed.run with one process per GPU.  When only one GPU is visible the two
share it: the brain then runs without the chained decode launch (VWA_CHAIN=0) -- that kernel keeps
one workgroup resident on every CU behind grid barriers, which a co-located ASR would starve
(it would time out and fall back per step).
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time

PKG = "voice_enabled_browser_automation_amd"


def _spawn(module: str, env_extra: dict, torchrun_nproc: int = 0) -> subprocess.Popen:
    env = dict(os.environ)
    env.update(env_extra)
    if torchrun_nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun_nproc}",
               "--master-addr", "127.0.0.1", "--master-port", env.get("VWA_MASTER_PORT", "29611"), "-m", module]
    else:
        cmd = [sys.executable, "-m", module]
    return subprocess.Popen(cmd, env=env)


def _ids(v: str) -> list:
    return [g.strip() for g in v.split(",") if g.strip()]


def plan_gpus(n_gpus: int, tp: int = 1, brain: str = "", voice: str = "") -> dict:
    """-> {"brain": [ids], "voice": [ids], "shared": bool}: the brain on GPUs 0..tp-1, the voice
    workers on the rest (or explicit lists); shared = a brain GPU also hosts a voice worker."""
    n = max(1, n_gpus)
    b = _ids(brain) or [str(i) for i in range(min(tp, n))]
    v = _ids(voice) or ([str(i) for i in range(n) if str(i) not in b] or [b[0]])
    return {"brain": b, "voice": v, "shared": bool(set(b) & set(v))}


def _visible_gpus() -> int:
    try:
        import torch  # device_count() reads the device list without initialising the HIP runtime

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 1


def main():
    tp = int(os.environ.get("VWA_TP", "1") or 1)
    plan = plan_gpus(_visible_gpus(), tp, os.environ.get("VWA_BRAIN_GPUS", ""), os.environ.get("VWA_VOICE_GPUS", ""))
    voice_gpus = plan["voice"]
    benv = {"HIP_VISIBLE_DEVICES": ",".join(plan["brain"])}
    if plan["shared"]:
        benv["VWA_CHAIN"] = os.environ.get("VWA_CHAIN", "0")
    procs = [_spawn(f"{PKG}.brain.server", benv, tp)]
    if len(voice_gpus) > 1:
        # ASR session-DP: one voice worker per GPU behind the router on VOICE_PORT (voice/router.py)
        base = int(os.environ.get("VWA_VOICE_BASE_PORT", "7100"))
        for i, g in enumerate(voice_gpus):
            procs.append(_spawn(f"{PKG}.voice.server", {"HIP_VISIBLE_DEVICES": g, "VOICE_PORT": str(base + i)}))
        procs.append(_spawn(f"{PKG}.voice.router", {"VWA_DP": str(len(voice_gpus))}))
    else:
        procs.append(_spawn(f"{PKG}.voice.server", {"HIP_VISIBLE_DEVICES": voice_gpus[0] if voice_gpus else "0"}))
    procs += [_spawn(f"{PKG}.executor.server", {}), _spawn(f"{PKG}.web.server", {})]

    def stop(*_a):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        sys.exit(0)

    signal.signal(signal.SIGINT, stop)
    signal.signal(signal.SIGTERM, stop)
    while True:
        for p in procs:
            if p.poll() is not None:
                print(f"[launch] a service exited with {p.returncode}; stopping", flush=True)
                stop()
        time.sleep(1.0)


if __name__ == "__main__":
    main()
