"""Start the four services (brain :8090, voice :7072, executor :7081, web :5173) as separate
processes, like ``pnpm dev`` in each app of the reference (README.md:83-97).

    python -m voice_enabled_browser_automation_amd.launch            # keyword brain, no ASR (CPU)
    VWA_BRAIN_ENGINE=llm VWA_ASR_ENGINE=whisper python -m voice_enabled_browser_automation_amd.launch

GPU placement on one node (plan_gpus): the brain (LLM) takes GPUs 0..TP-1 and the voice service
(ASR) every remaining GPU, one voice worker per GPU behind the session router (session DP);
VWA_BRAIN_GPUS / VWA_VOICE_GPUS (comma lists) override.  With VWA_TP>1 the brain is launched
through torch.distributed.run with one process per GPU.  When only one GPU is visible the two
share it (shared_gpu_env: the brain uses the chained decode launch only while the ASR is idle --
a busy word in /dev/shm).  The brain is restartable: a TP group that loses lockstep exits and is started again in fresh
processes while the other services keep serving (Supervisor).
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from .utils.env import knob

PKG = "voice_enabled_browser_automation_amd"


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(module: str, env_extra: dict, torchrun_nproc: int = 0, restart: int = 0) -> subprocess.Popen:
    env = dict(os.environ)
    env.update(env_extra)
    if torchrun_nproc > 1:
        # VWA_MASTER_PORT only for the first start: a restarted group gets a fresh rendezvous port
        # (the previous group's port may still be in TIME_WAIT)
        port = (env.get("VWA_MASTER_PORT") if restart == 0 else None) or str(_free_port())
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun_nproc}",
               "--master-addr", "127.0.0.1", "--master-port", port, "-m", module]
    else:
        cmd = [sys.executable, "-m", module]
    return subprocess.Popen(cmd, env=env)


class Supervisor:
    """Keeps the services running.  A service marked restartable (the brain: its TP group exits
    with brain/tp_engine.FATAL_EXIT_CODE when it loses lockstep, and any brain crash is an LLM
    failure the reference survives with 500s, apps/brain/src/server.ts:122-126) is started again
    in FRESH processes -- never re-exec'd from a process that touched the GPU -- with exponential
    backoff, at most ``max_restarts`` times per ``window_s``; the other services keep running
    meanwhile (voice answers brain errors as the reference does).  Any other exit, or a restart
    budget spent, stops everything.  The backoff is a scheduled restart time, not a sleep: the
    other services (and SIGTERM) are still watched while a restart is pending."""

    def __init__(self, spawn=None, max_restarts: int = 5, window_s: float = 600.0, backoff_s: float = 1.0,
                 clock=time.monotonic, log=print):
        self.spawn = spawn or _spawn
        self.max_restarts = max_restarts
        self.window_s = window_s
        self.backoff_s = backoff_s
        self.clock = clock
        self.log = log
        # [name, args, restartable, proc, restart times, restart due at (None: running), restarts]
        self.services = []

    def add(self, name: str, module: str, env_extra: dict, torchrun_nproc: int = 0, restartable: bool = False):
        proc = self.spawn(module, env_extra, torchrun_nproc)
        self.services.append([name, (module, env_extra, torchrun_nproc), restartable, proc, [], None, 0])
        return proc

    def procs(self):
        return [s[3] for s in self.services]

    def pending_restarts(self) -> int:
        return sum(1 for s in self.services if s[5] is not None)

    def poll_once(self) -> bool:
        """Check every service once; schedule / perform the restarts that are allowed.  Never blocks.
        False = stop everything."""
        now = self.clock()
        for svc in self.services:
            name, args, restartable, proc, times, due, n = svc
            if due is not None:
                if now >= due:
                    svc[5] = None
                    svc[6] = n + 1
                    times.append(now)
                    svc[3] = self.spawn(*args, restart=n + 1)
                continue
            rc = proc.poll()
            if rc is None:
                continue
            times[:] = [t for t in times if now - t < self.window_s]
            if not restartable or len(times) >= self.max_restarts:
                self.log(f"[launch] {name} exited with {rc}; stopping" +
                         (f" ({len(times)} restarts in {self.window_s:.0f} s)" if restartable else ""))
                return False
            delay = self.backoff_s * (2 ** len(times))
            self.log(f"[launch] {name} exited with {rc}; restarting it in fresh processes in {delay:.1f} s "
                     f"(restart {len(times) + 1}/{self.max_restarts})")
            svc[5] = now + delay
        return True

    def stop(self) -> None:
        for svc in self.services:
            svc[5] = None  # (a pending restart is cancelled)
        for p in self.procs():
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in self.procs():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()


def _ids(v: str) -> list:
    return [g.strip() for g in v.split(",") if g.strip()]


def plan_gpus(n_gpus: int, tp: int = 1, brain: str = "", voice: str = "", parent_visible: str = "") -> dict:
    """-> {"brain": [ids], "voice": [ids], "shared": bool}: the brain on GPUs 0..tp-1, the voice
    workers on the rest (or explicit lists); shared = a brain GPU also hosts a voice worker.
    ``parent_visible`` (the launcher's own HIP_VISIBLE_DEVICES list): the planned ordinals index
    into it, so a launcher given GPUs 4,5 places its children on 4 and 5 -- a child's
    HIP_VISIBLE_DEVICES replaces the inherited mask rather than narrowing it."""
    n = max(1, n_gpus)
    b = _ids(brain) or [str(i) for i in range(min(tp, n))]
    v = _ids(voice) or ([str(i) for i in range(n) if str(i) not in b] or [b[0]])
    shared = bool(set(b) & set(v))
    par = _ids(parent_visible)
    if par:
        m = lambda ids: [par[int(i)] if i.isdigit() and int(i) < len(par) else i for i in ids]  # noqa: E731
        b, v = m(b), m(v)
    return {"brain": b, "voice": v, "shared": shared}


def _parent_visible() -> str:
    return os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES") or ""


def shared_gpu_env(env, busy_file: str = "") -> dict:
    """Brain settings when it shares its GPU with a voice worker.  Under live streaming-ASR load the
    chained launch's persistent workgroups wait for the ASR kernels to drain from their CUs (the
    step measured 3.72-3.76 ms of GPU wait vs 3.61-3.62 ms per-kernel, tools/service_bench.py,
    profiles/r4_service_chain_ab.jsonl), but with the recognizer idle -- one session whose user
    stopped speaking -- the chain is ~10 % faster.  So (round 6) the two share a busy word
    (``busy_file``, utils/busy_flag.py: the ASR batcher marks its passes) and the brain picks the
    launch form per step (runtime/engine.py chain_gate).  VWA_SHARED_CHAIN=0 forces per-kernel
    launches (round 5's default), =1 the chain always; VWA_SHARED_CHAIN_GRID_DIV=k gives it CUs/k
    workgroups."""
    mode = env.get("VWA_SHARED_CHAIN", "gate" if busy_file else "0")
    out = {"VWA_CHAIN": env.get("VWA_CHAIN", "0" if mode == "0" else "1"),
           # HBM the voice worker's ASR keeps (the brain's auto KV sizing leaves it free)
           "VWA_SHARED_GB": env.get("VWA_SHARED_GB", "24")}
    if mode == "gate" and busy_file:
        out["VWA_ASR_BUSY_FILE"] = busy_file
    div = env.get("VWA_SHARED_CHAIN_GRID_DIV")
    if div:
        out["VWA_CHAIN_GRID_DIV"] = div
    return out


def shared_voice_env(env, brain_env: dict) -> dict:
    """Voice-worker settings on a GPU shared with the brain.  The persistent Whisper-large decoder
    (VWA_ASR_PERSIST, whisper_dec.hip) and the brain's chained launch are both one-workgroup-per-CU
    persistent kernels from different processes: if their workgroup dispatch interleaved, each
    would wait for workgroups the other holds until its bounded spins gave up.  So the ASR keeps
    per-kernel launches whenever the brain may chain (an explicit VWA_ASR_PERSIST wins)."""
    brain_chains = brain_env.get("VWA_CHAIN", "1") != "0"
    return {"VWA_ASR_PERSIST": env.get("VWA_ASR_PERSIST", "0" if brain_chains else "1")}


def _visible_gpus() -> int:
    try:
        import torch  # device_count() reads the device list without initialising the HIP runtime

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 1


def main():
    tp = knob("VWA_TP")
    plan = plan_gpus(_visible_gpus(), tp, knob("VWA_BRAIN_GPUS"), knob("VWA_VOICE_GPUS"),
                     parent_visible=_parent_visible())
    voice_gpus = plan["voice"]
    benv = {"HIP_VISIBLE_DEVICES": ",".join(plan["brain"])}
    venv = {}
    if plan["shared"]:
        busy = f"/dev/shm/vwa_asr_busy_{os.getpid()}"
        benv.update(shared_gpu_env(os.environ, busy))
        if benv.get("VWA_ASR_BUSY_FILE"):
            venv["VWA_ASR_BUSY_FILE"] = busy
        venv.update(shared_voice_env(os.environ, benv))
    sup = Supervisor(max_restarts=knob("VWA_BRAIN_MAX_RESTARTS"))
    sup.add("brain", f"{PKG}.brain.server", benv, tp, restartable=True)
    if len(voice_gpus) > 1:
        # ASR session-DP: one voice worker per GPU behind the router on VOICE_PORT (voice/router.py)
        base = knob("VWA_VOICE_BASE_PORT")
        for i, g in enumerate(voice_gpus):
            sup.add(f"voice{i}", f"{PKG}.voice.server", {"HIP_VISIBLE_DEVICES": g, "VOICE_PORT": str(base + i)})
        sup.add("router", f"{PKG}.voice.router", {"VWA_DP": str(len(voice_gpus))})
    else:
        sup.add("voice", f"{PKG}.voice.server", {"HIP_VISIBLE_DEVICES": voice_gpus[0] if voice_gpus else "0", **venv})
    sup.add("executor", f"{PKG}.executor.server", {})
    sup.add("web", f"{PKG}.web.server", {})

    def stop(*_a):
        sup.stop()
        sys.exit(0)

    signal.signal(signal.SIGINT, stop)
    signal.signal(signal.SIGTERM, stop)
    while sup.poll_once():
        time.sleep(1.0)
    stop()


if __name__ == "__main__":
    main()
