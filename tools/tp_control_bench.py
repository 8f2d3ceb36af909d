"""Per-iteration control latency of the TP brain's lockstep channel (parallel/control.py): /dev/shm
ring vs the round-5 gloo broadcast, at world 2 / 4 / 8 ranks on the CPU.

Rank 0 sends ``iters`` control messages (the empty admission header the scheduler sends on most
decode iterations, plus a send timestamp), ``gap_us`` apart -- the decode step that separates two
control messages; every other rank receives them and records receive time - send time (both
CLOCK_MONOTONIC, comparable across processes).  Reported: median / p90 / max over ranks' medians.

    python tools/tp_control_bench.py [--worlds 2,4,8] [--iters 400] [--gap-us 300] [--json out]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, kind, iters, gap_us, q):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from voice_enabled_browser_automation_amd.parallel.control import make_channel

    ch = make_channel(rank, world, dist.group.WORLD, kind=kind)
    lat = []
    dist.barrier()
    for i in range(iters + 20):
        if rank == 0:
            t_end = time.perf_counter_ns() + gap_us * 1000
            while time.perf_counter_ns() < t_end:  # the decode step between two messages
                pass
            ch.send(([], False, time.perf_counter_ns()))
        else:
            msg = ch.recv()
            if i >= 20:
                lat.append((time.perf_counter_ns() - msg[2]) / 1e3)
    dist.barrier()
    q.put((rank, lat))
    ch.close()
    dist.destroy_process_group()


def measure(world: int, kind: str, iters: int = 400, gap_us: int = 300) -> dict:
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, kind, iters, gap_us, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    meds = [statistics.median(v) for r, v in res.items() if r != 0]
    allv = sorted(x for r, v in res.items() if r != 0 for x in v)
    return dict(world=world, kind=kind, iters=iters, gap_us=gap_us, median_us=round(statistics.median(allv), 2),
                p90_us=round(allv[int(0.9 * (len(allv) - 1))], 2), max_rank_median_us=round(max(meds), 2),
                exitcodes=[p.exitcode for p in procs])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--gap-us", type=int, default=300)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    for w in [int(x) for x in a.worlds.split(",")]:
        for kind in ("shm", "gloo"):
            r = measure(w, kind, a.iters, a.gap_us)
            print(json.dumps(r), flush=True)
            if a.json:
                with open(a.json, "a") as f:
                    f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
