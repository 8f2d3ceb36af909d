"""Multi-rank check of the one-shot all-reduce (run under torchrun; ranks may share one GPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 \
        tools/ar_check.py
Compares against the fp32 sum of the same inputs for several message sizes, eager and inside a
captured hipGraph, then times it against RCCL/gloo all_reduce.
"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd.parallel.custom_ar import OneShotAllReduce  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    ar = OneShotAllReduce(rank, world, dist.group.WORLD, max_elems=64 * 4096)  # (preflight + self-test inside)
    if os.environ.get("VWA_AR_CHECK_REPORT") and rank == 0:
        print("PREFLIGHT", ar.peer_report, flush=True)
    ok = True
    for n in (4096, 8 * 4096, 64 * 4096, 1000 * 8):
        torch.manual_seed(100 + n)
        xs = [torch.randn(n) for _ in range(world)]  # every rank builds all inputs (same seed)
        exp = sum(x.to(torch.bfloat16).float() for x in xs)
        t = xs[rank].to(torch.bfloat16).cuda()
        ar(t)
        torch.cuda.synchronize()
        err = (t.float().cpu() - exp).abs().max().item()
        ok &= err < 0.05
        if rank == 0:
            print(f"n={n} max_err={err:.4f}", flush=True)
    # graph capture + replays (epochs advance inside the kernel)
    x = torch.full((8 * 4096,), float(rank + 1), dtype=torch.bfloat16, device="cuda")
    buf = torch.empty_like(x)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        buf.copy_(x)
        ar(buf)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        buf.copy_(x)
        ar(buf)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    gerr = (buf.float() - want).abs().max().item()
    ok &= gerr == 0
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 200 * 1e6
    if rank == 0:
        print(f"graph_err={gerr} oneshot_graph_us={us:.1f} error_flag={ar.error()}", flush=True)
    # one-shot all-gather (vocab-parallel sampler exchange), eager and replayed
    for n in (1, 100, 4096):
        mine = torch.arange(n, dtype=torch.int32, device="cuda") + 1000 * rank
        got = ar.gather(mine)
        torch.cuda.synchronize()
        want_g = torch.stack([torch.arange(n, dtype=torch.int32) + 1000 * p for p in range(world)])
        ok &= bool(torch.equal(got.cpu(), want_g))
    src = torch.full((64,), rank + 7, dtype=torch.int32, device="cuda")
    gout = torch.zeros((world, 64), dtype=torch.int32, device="cuda")
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        ar.gather(src, gout)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g2):
        ar.gather(src, gout)
    for k in range(10):
        src.fill_(rank + 7 + k)
        g2.replay()
        torch.cuda.synchronize()
        ok &= bool(all(int(gout[p, 0]) == p + 7 + k for p in range(world)))
    if rank == 0:
        print(f"gather_ok={ok}", flush=True)
    ok &= not ar.error()
    dist.barrier()
    ar.close()
    res = torch.tensor([int(ok)])
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if rank == 0:
        print("AR_CHECK", "PASS" if res.item() else "FAIL", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if res.item() else 1)


if __name__ == "__main__":
    main()
