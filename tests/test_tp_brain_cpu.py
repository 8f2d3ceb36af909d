"""TP brain serving on CPU over gloo (brain/tp_engine.py, launch.py Supervisor): continuous batching
in lockstep across a 2-rank TP group, the fatal-exit policy when a rank loses lockstep, and the
launcher restarting only the brain.  Reference behaviour: concurrent /parse calls are served
independently and an LLM failure is a 500, not an outage (apps/brain/src/server.ts:89-139)."""
import os
import socket
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
from voice_enabled_browser_automation_amd.brain.tp_engine import FATAL_EXIT_CODE, TPIntentEngine
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.models.config import LlamaConfig
from voice_enabled_browser_automation_amd.models.llama import LlamaModel
from voice_enabled_browser_automation_amd.parallel.tp import TPContext
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

TINY = LlamaConfig(name="tiny2", hidden=256, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=64, ffn=512, max_pos=4096)
TEXTS = ["search wireless earbuds", "scroll down", "sort by price", "go back"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(tp):
    m = LlamaModel(TINY, device="cpu", seed=5, tp=tp)
    eng = LLMEngine(m, max_seqs=4, max_model_len=2048, kv_blocks=600)
    return LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=160, temperature=0.1, seed=11)


def _reqs():
    return [{"text": t, "context": {"url": "https://www.bestbuy.com"}} for t in TEXTS]


def _worker(rank, world, port, q, fault_rank):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext(rank=rank, size=world, group=dist.group.WORLD)
    ie = _engine(tp)

    def fatal(e):  # the default policy (os._exit(FATAL_EXIT_CODE)), reporting first
        q.put(("fatal", rank, type(e).__name__))
        time.sleep(1.0)
        os._exit(FATAL_EXIT_CODE)

    tpe = TPIntentEngine(ie, tp, on_fatal=fatal)
    if rank == fault_rank:
        # what a chained TP launch whose peer never arrived does (runtime/engine.py)
        orig = ie.step

        def faulty():
            if tpe.iterations == 3:
                ie.engine._tp_chain_fatal()
            return orig()

        ie.step = faulty
    if rank == 0:
        try:
            outs = tpe.parse_many(_reqs())
        except Exception as e:  # noqa: BLE001
            q.put(("client_error", rank, type(e).__name__))
            time.sleep(5.0)  # the scheduler thread's fatal handler ends the process
            os._exit(1)
        q.put(("batch", rank, dict(tpe.batch_stats)))
        tpe.stop()
    else:
        outs = tpe.worker_loop()
    q.put(("outs", rank, outs))
    dist.destroy_process_group()


def _spawn(world, fault_rank=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fault_rank)) for r in range(world)]
    for p in procs:
        p.start()
    return procs, q


def test_tp2_continuous_batching_in_lockstep():
    """4 concurrent requests on a TP=2 group: they decode together (several samples per
    iteration), both ranks produce the same answers, equal to the TP=1 engine's batch."""
    torch.set_num_threads(4)
    want = _engine(TPContext.single()).parse_many(_reqs())
    procs, q = _spawn(2)
    msgs = [q.get(timeout=600) for _ in range(3)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    outs = {r: o for kind, r, o in msgs if kind == "outs"}
    stats = next(o for kind, _r, o in msgs if kind == "batch")
    assert outs[0] == outs[1], "rank 1 diverged from rank 0"
    assert all(safe_parse(ParseResponse, o).success for o in outs[0])
    assert outs[0] == want
    assert stats["sampled"] / stats["iterations"] > 1.5, stats  # continuous batching, not serial requests
    assert stats["max_active"] == 4


def test_tp_rank_losing_lockstep_ends_the_whole_group():
    """A chained-launch timeout on one rank (TPGroupFailure) is terminal for the group: the
    failing rank and its peer both exit with FATAL_EXIT_CODE (no process stays up reporting
    healthy with stale round counters), and rank 0's pending requests fail (-> 500 llm_error)."""
    procs, q = _spawn(2, fault_rank=1)
    for p in procs:
        p.join(timeout=300)
    assert [p.exitcode for p in procs] == [FATAL_EXIT_CODE, FATAL_EXIT_CODE]
    msgs = []
    while not q.empty():
        msgs.append(q.get(timeout=5))
    assert ("fatal", 1, "TPGroupFailure") in msgs
    assert any(k == "fatal" and r == 0 for k, r, _ in msgs)
    assert not any(k == "outs" and r == 0 for k, r, _ in msgs)


class _FakeProc:
    def __init__(self, name, rc=None):
        self.name, self.rc, self.signals = name, rc, []

    def poll(self):
        return self.rc

    def send_signal(self, s):
        self.signals.append(s)
        self.rc = -s

    def wait(self, timeout=None):
        return self.rc

    def kill(self):
        self.rc = -9


def test_supervisor_restarts_only_the_brain():
    from voice_enabled_browser_automation_amd.launch import Supervisor

    spawned = []

    def spawn(module, env, nproc, restart=0):
        p = _FakeProc(module)
        spawned.append((module, nproc, p, restart))
        return p

    t = [0.0]
    sup = Supervisor(spawn=spawn, max_restarts=2, window_s=100.0, backoff_s=0.5, clock=lambda: t[0],
                     log=lambda *_: None)
    brain = sup.add("brain", "pkg.brain.server", {}, 2, restartable=True)
    voice = sup.add("voice", "pkg.voice.server", {})
    assert sup.poll_once()
    brain.rc = FATAL_EXIT_CODE  # the TP group exited after losing lockstep
    assert sup.poll_once() and sup.pending_restarts() == 1 and len(spawned) == 2  # scheduled, not slept
    voice.rc = None
    t[0] += 0.25
    assert sup.poll_once() and len(spawned) == 2  # backoff (0.5 s) not over: others still watched
    t[0] += 0.3
    assert sup.poll_once()
    assert len(spawned) == 3 and spawned[-1][:2] == ("pkg.brain.server", 2)  # a fresh torchrun group
    assert spawned[-1][3] == 1  # a restart: the launcher picks a fresh rendezvous port
    assert sup.procs()[1] is voice and voice.rc is None and not voice.signals
    sup.procs()[0].rc = FATAL_EXIT_CODE
    assert sup.poll_once()
    t[0] += 1.0  # second restart (backoff doubled)
    assert sup.poll_once() and len(spawned) == 4 and spawned[-1][3] == 2
    sup.procs()[0].rc = FATAL_EXIT_CODE
    assert not sup.poll_once()  # restart budget spent: stop everything
    sup.stop()
    assert voice.signals  # now the rest is stopped too


def test_supervisor_stops_on_a_non_restartable_exit():
    from voice_enabled_browser_automation_amd.launch import Supervisor

    sup = Supervisor(spawn=lambda m, e, n, restart=0: _FakeProc(m), log=lambda *_: None)
    sup.add("brain", "b", {}, restartable=True)
    ex = sup.add("executor", "e", {})
    ex.rc = 1
    assert not sup.poll_once()


def test_plan_gpus_maps_through_the_parent_mask():
    from voice_enabled_browser_automation_amd.launch import plan_gpus, shared_gpu_env

    assert plan_gpus(2, 1, parent_visible="4,5") == {"brain": ["4"], "voice": ["5"], "shared": False}
    assert plan_gpus(4, 2, parent_visible="") == {"brain": ["0", "1"], "voice": ["2", "3"], "shared": False}
    p = plan_gpus(1, 1, parent_visible="6")
    assert p == {"brain": ["6"], "voice": ["6"], "shared": True}
    assert shared_gpu_env({})["VWA_CHAIN"] == "0"
    assert shared_gpu_env({"VWA_SHARED_CHAIN": "1"})["VWA_CHAIN"] == "1"
    # round 6: with a busy word the brain keeps the chain and gates it on the ASR's activity
    g = shared_gpu_env({}, "/dev/shm/vwa_asr_busy_test")
    assert g["VWA_CHAIN"] == "1" and g["VWA_ASR_BUSY_FILE"] == "/dev/shm/vwa_asr_busy_test"
    assert "VWA_ASR_BUSY_FILE" not in shared_gpu_env({"VWA_SHARED_CHAIN": "0"}, "/dev/shm/x")
    # the ASR's persistent decoder only beside a brain that never runs its persistent launch
    from voice_enabled_browser_automation_amd.launch import shared_voice_env

    assert shared_voice_env({}, g)["VWA_ASR_PERSIST"] == "0"
    assert shared_voice_env({}, shared_gpu_env({"VWA_SHARED_CHAIN": "0"}))["VWA_ASR_PERSIST"] == "1"
    assert shared_voice_env({"VWA_ASR_PERSIST": "1"}, g)["VWA_ASR_PERSIST"] == "1"


def test_asr_busy_flag_gates_the_chained_launch(tmp_path):
    """utils/busy_flag.py: the ASR batcher's passes mark the shared word busy (with a hold after
    the last one); the brain engine's chain_gate reads it before every step."""
    import numpy as np

    from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
    from voice_enabled_browser_automation_amd.utils.busy_flag import BusyFlag

    path = str(tmp_path / "busy")
    w, r = BusyFlag(path, create=True), BusyFlag(path)
    assert not r.busy(0.0)
    w.enter()
    assert r.busy(0.0)
    w.leave()
    assert not r.busy(0.0) and r.busy(10_000.0)  # within the hold
    m = LlamaModel(TINY, device="cpu", seed=1)
    e = LLMEngine(m, max_seqs=1, max_model_len=256, kv_blocks=40)
    e.chain_gate = lambda: r.busy(0.0)
    s = e.new_sequence([1, 2, 3, 4], use_prefix_cache=False)
    e.prefill(s)
    w.enter()
    a = e.run_rows([(s, 5)])
    assert e.stats["gated_steps"] == 1 and m._chain_gated
    w.leave()
    b = e.run_rows([(s, 6)])
    assert e.stats["gated_steps"] == 1 and not m._chain_gated
    assert np.isfinite(a.numpy()).all() and np.isfinite(b.numpy()).all()


def test_brain_health_reports_a_failed_tp_group():
    import asyncio

    from aiohttp.test_utils import TestClient, TestServer

    from voice_enabled_browser_automation_amd.brain.server import build_app

    class Failed:
        failed = RuntimeError("chained TP decode launch timed out waiting for a peer rank")

    async def go():
        async with TestClient(TestServer(build_app(engine=Failed()))) as c:
            r = await c.get("/health")
            return r.status, await r.json()

    status, body = asyncio.run(go())
    assert status == 503 and body["status"] == "error"


def _idle_worker(rank, world, port, q):
    import datetime

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tp = TPContext(rank=rank, size=world, group=dist.group.WORLD)
    # a control group whose collectives time out after 2 s: without the leader's heartbeat the
    # worker's broadcast raises during the idle period below and the group would be restarted
    ctl = dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=2))

    def fatal(e):
        q.put(("fatal", rank, repr(e)))
        os._exit(FATAL_EXIT_CODE)

    tpe = TPIntentEngine(_engine(tp), tp, ctl_group=ctl, on_fatal=fatal, heartbeat_s=0.3)
    if rank == 0:
        tpe.start()
        time.sleep(4.0)  # idle for twice the control group's timeout
        outs = tpe.parse_many(_reqs()[:1])
        q.put(("beats", rank, tpe.heartbeats))
        tpe.stop()
    else:
        outs = tpe.worker_loop()
    q.put(("outs", rank, outs))
    dist.destroy_process_group()


def test_idle_tp_group_survives_past_the_control_timeout():
    """an idle leader must keep the workers' control broadcast alive (heartbeat), so
    a quiet period longer than the gloo timeout is not turned into a fatal group restart."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_idle_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    msgs = []
    while not q.empty():
        msgs.append(q.get())
    assert [p.exitcode for p in procs] == [0, 0], msgs
    assert not [m for m in msgs if m[0] == "fatal"], msgs
    beats = next(m[2] for m in msgs if m[0] == "beats")
    assert beats >= 5, msgs
    outs = {r: o for kind, r, o in msgs if kind == "outs"}
    assert outs[0] == outs[1] and safe_parse(ParseResponse, outs[0][0]).success


def _bench_worker(rank, world, port, q):
    """bench.py's session driver over the served TP control plane: rank 0 runs
    the sessions through TPIntentEngine, rank 1 follows in lockstep, world barriers around."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), VWA_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    import bench
    from voice_enabled_browser_automation_amd.parallel.tp import init_distributed

    tp = init_distributed(tp_size=2)
    assert tp.size == 2 and tp.ctl is not None
    brain = TPIntentEngine(_engine(tp), tp)
    reqs = _reqs()

    def one(i):
        out = brain.parse(reqs[i % len(reqs)])
        return safe_parse(ParseResponse, out).success, out

    bench.drive_sessions(brain, tp, world, 1, one)  # warm-up
    res, el = bench.drive_sessions(brain, tp, world, 3, one, start=1)
    allr = bench.gather({"rank": rank, "n": len(res), "ok": sum(r[0] for r in res),
                         "outs": [r[1] for r in res], "it": brain.iterations}, world)
    q.put(("done", rank, allr, el))
    dist.destroy_process_group()


def test_bench_tp_control_path_over_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    assert [p.exitcode for p in procs] == [0, 0]
    msgs = {}
    while not q.empty():
        kind, r, allr, el = q.get()
        msgs[r] = (allr, el)
    allr = msgs[0][0]
    assert allr[0]["n"] == 3 and allr[0]["ok"] == 3  # the leader ran the sessions, all valid
    assert allr[1]["n"] == 0  # the follower ran none of its own...
    assert allr[1]["it"] == allr[0]["it"] > 0  # ...but every scheduler iteration in lockstep
    assert all(safe_parse(ParseResponse, o).success for o in allr[0]["outs"])
