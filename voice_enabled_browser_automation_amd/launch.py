"""Start the four services (brain :8090, voice :7072, executor :7081, web :5173) as separate
processes, like ``pnpm dev`` in each app of the reference (README.md:83-97).

    python -m voice_enabled_browser_automation_amd.launch            # keyword brain, no ASR (CPU)
    VWA_BRAIN_ENGINE=llm VWA_ASR_ENGINE=whisper python -m voice_enabled_browser_automation_amd.launch

GPU placement on one node: the brain (LLM) and the voice service (ASR) each pin their own
GPU via HIP_VISIBLE_DEVICES (VWA_BRAIN_GPUS / VWA_VOICE_GPUS, default "0"); with VWA_TP>1 the
brain is launched through torch.distributed.run with one process per GPU.  A comma list in
VWA_VOICE_GPUS (e.g. "4,5,6,7") starts one voice worker per GPU behind the session router.
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


def main():
    tp = int(os.environ.get("VWA_TP", "1") or 1)
    voice_gpus = [g for g in os.environ.get("VWA_VOICE_GPUS", "0").split(",") if g.strip()]
    procs = [_spawn(f"{PKG}.brain.server", {"HIP_VISIBLE_DEVICES": os.environ.get("VWA_BRAIN_GPUS", "0")}, tp)]
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
