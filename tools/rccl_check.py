"""RCCL (torch.distributed backend "nccl" on ROCm) through the framework's own process-group setup
(parallel/tp.py init_distributed): the collectives the TP / DP paths hand to RCCL -- all-reduce of
prefill-sized messages, the vocab all-gather, broadcast, all-gather of per-rank metrics -- on GPU
tensors, checked against the exact sums.  Run under torchrun, one rank per GPU:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        tools/rccl_check.py
(RCCL refuses two ranks on ONE device; the 1-GPU test box runs it with N = 1.)
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ.setdefault("VWA_DIST_BACKEND", "nccl")
    from voice_enabled_browser_automation_amd.parallel.tp import TPContext, init_distributed

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:  # init_distributed short-circuits a single process: initialise RCCL itself
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, init_method="tcp://127.0.0.1:" + os.environ.get(
            "MASTER_PORT", "29511"))
        tp = TPContext(rank=0, size=1, group=dist.group.WORLD)
    else:
        tp = init_distributed(tp_size=world)
    assert dist.get_backend() == "nccl", dist.get_backend()
    rank = dist.get_rank()
    dev = torch.device("cuda", torch.cuda.current_device())
    ok = True
    for n in (4096, 1 << 20, 9 << 20):  # decode-sized, 2 MB, 18 MB (Llama-3-70B prefill rows, bf16)
        x = torch.full((n,), float(rank + 1), dtype=torch.bfloat16, device=dev)
        dist.all_reduce(x, group=tp.group)
        ok &= bool((x.float() == world * (world + 1) / 2).all())
    v = torch.arange(1000, dtype=torch.float32, device=dev).view(2, 500) + 1000 * rank
    full = tp.all_gather_vocab(v, 1000 * world) if world > 1 else v
    ok &= full.shape == (2, 500 * world) or world == 1
    b = torch.full((64,), 7.0 if rank == 0 else 0.0, device=dev)
    dist.broadcast(b, src=0)
    ok &= bool((b == 7.0).all())
    m = [None] * world
    dist.all_gather_object(m, {"rank": rank, "rtf": 0.001 * (rank + 1)})
    ok &= [d["rank"] for d in m] == list(range(world))
    torch.cuda.synchronize()
    print(f"rank {rank}: backend {dist.get_backend()} world {world} ok {ok}", flush=True)
    dist.barrier()
    if rank == 0 and ok:
        print("RCCL_CHECK PASS", flush=True)
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
