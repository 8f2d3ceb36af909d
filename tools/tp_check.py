"""Tensor-parallel Llama on the GPU kernels vs TP=1 (run under torchrun; ranks may share a GPU).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29556 \
        tools/tp_check.py
    VWA_TP_CHECK_CFG=70b VWA_TP_CHECK_LAYERS=2 python -m torch.distributed.run --nproc-per-node 8 ... tools/tp_check.py
Every rank builds the TP shard of the same random model (deterministic per-layer generator),
runs prefill + ragged decode through the engine -- eagerly AND with every decode step replayed
from a hipGraph -- with the one-shot IPC all-reduce for the vocab-parallel embedding and the
row-parallel outputs, and compares the (diagnostically gathered) logits with a TP=1 model run
on the same device.  Decode steps of <= 4 rows run the chained layer (one launch per layer) with
the row-parallel all-reduces as in-launch rounds over the same IPC buffers
(skinny_stream.hip chain_tp_reduce).  Then the vocab-parallel sampler (partial maxima -> one-shot IPC all-gather
-> merge, ops.sample tp=...) is checked token for token against the TP=1 full-vocab sampler,
under grammar-like random masks and temperature.  VWA_DIST_BACKEND selects the control /
large-message backend (gloo when two ranks share one GPU, RCCL needs one GPU per rank); the
decode step itself contains no torch.distributed call, so it is graph-captured either way.
"""
import math
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from voice_enabled_browser_automation_amd import ops  # noqa: E402
from voice_enabled_browser_automation_amd.models.config import LlamaConfig  # noqa: E402
from voice_enabled_browser_automation_amd.models.llama import LlamaModel  # noqa: E402
from voice_enabled_browser_automation_amd.parallel.tp import TPContext, init_distributed  # noqa: E402
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine  # noqa: E402

CFGS = {
    "small": LlamaConfig(name="tp", vocab_size=4096, hidden=512, n_layers=3, n_heads=8, n_kv_heads=4, head_dim=64,
                         ffn=1024, max_pos=1024),
    # Llama-3-70B layer shapes (hidden 8192, 64 q / 8 kv heads, FFN 28672, vocab 128256): at TP=8
    # every rank holds 8 q heads, 1 kv head, an FFN slice of 3584 and a 16032-token vocab shard
    "70b": LlamaConfig(name="tp70b", vocab_size=128256, hidden=8192, n_layers=3, n_heads=64, n_kv_heads=8,
                       head_dim=128, ffn=28672, max_pos=1024),
}
CFG = CFGS[os.environ.get("VWA_TP_CHECK_CFG", "small")]
if os.environ.get("VWA_TP_CHECK_LAYERS"):
    import dataclasses

    CFG = dataclasses.replace(CFG, n_layers=int(os.environ["VWA_TP_CHECK_LAYERS"]))


def run(model, toks, graphs):
    e = LLMEngine(model, max_seqs=2, max_model_len=512, kv_blocks=80, use_graphs=graphs)
    if graphs:
        e.capture_all()
    torch.cuda.synchronize()
    if model.tp.size > 1:  # (as the serving control plane does per iteration: ranks start aligned)
        dist.barrier()
    s = e.new_sequence(toks[:100], use_prefix_cache=False)
    out = [e.prefill(s).float().cpu().clone()]
    for t in toks[100:104]:
        out.append(e.run_rows([(s, t)]).float().cpu().clone())
    out.append(e.run_rows([(s, t) for t in toks[104:110]], logits_for=[5]).float().cpu().clone())
    return out, e


def sample_check(tp, dev, ref_model, tp_model):
    """Tokens of the vocab-parallel sampler == tokens of the full-vocab sampler on the same logits."""
    torch.manual_seed(1)
    rows, V = 5, CFG.vocab_size
    full = torch.randn(rows, V, device=dev) * 2
    words = (V + 31) // 32
    mask = torch.randint(-2**31, 2**31 - 1, (rows, words), dtype=torch.int64).to(torch.int32).to(dev)
    temp = torch.full((rows,), 0.3, device=dev)
    seed = torch.tensor([99], dtype=torch.int64, device=dev)
    ok = True
    for step0 in range(4):
        want = torch.zeros(rows, dtype=torch.int32, device=dev)
        ops.sample(full, mask=mask, temperature=temp if step0 % 2 else None, seed=seed,
                   step=torch.tensor([step0], dtype=torch.int32, device=dev), out_tokens=want)
        got = torch.zeros(rows, dtype=torch.int32, device=dev)
        shard = full[:, tp_model.v_start : tp_model.v_end].contiguous()
        ops.sample(shard, mask=mask, temperature=temp if step0 % 2 else None, seed=seed,
                   step=torch.tensor([step0], dtype=torch.int32, device=dev), out_tokens=got,
                   v_offset=tp_model.v_start, tp=tp)
        torch.cuda.synchronize()
        ok &= torch.equal(got.cpu(), want.cpu())
    return ok


def install_nan_trace(tp):
    """VWA_TP_CHECK_TRACE=1: every kernel wrapper the Llama forward calls synchronises and checks
    its output; the first non-finite result is printed (rank, op, shapes) once."""
    state = {"done": False, "n": 0}

    def wrap(name, fn, pick):
        def run(*a, **k):
            r = fn(*a, **k)
            state["n"] += 1
            if not state["done"]:
                t = pick(a, k, r)
                torch.cuda.synchronize()
                if t is not None and not torch.isfinite(t.float()).all():
                    state["done"] = True
                    ins = [tuple(x.shape) for x in a if isinstance(x, torch.Tensor)]
                    fin = [bool(torch.isfinite(x.float()).all()) for x in a if isinstance(x, torch.Tensor)]
                    print(f"[rank {tp.rank}] first non-finite output: op #{state['n']} {name} in={ins} "
                          f"inputs_finite={fin} out={tuple(t.shape)}", flush=True)
            return r
        return run

    out_of = lambda a, k, r: r if isinstance(r, torch.Tensor) else k.get("out")  # noqa: E731
    for name in ("qkv_rope_write", "decode_attention_rows", "linear", "linear_swiglu", "embedding"):
        setattr(ops, name, wrap(name, getattr(ops, name), out_of))
    ar = tp.all_reduce
    tp.all_reduce = wrap("tp.all_reduce", ar, lambda a, k, r: r)


def ar_self_check(tp, dev):
    """The one-shot all-reduce alone (bf16, decode row counts 1..64 of this config's hidden size):
    rank r contributes (r + 1) * x, the sum is (world (world + 1) / 2) * x on every rank."""
    if tp.custom_ar is None:
        return True
    ok = True
    g = torch.Generator(device="cpu").manual_seed(3)
    for rows in (1, 2, 8, 64):
        x = (torch.randn(rows, CFG.hidden, generator=g) * 0.1).to(torch.bfloat16)
        t = (x.float() * (tp.rank + 1)).to(torch.bfloat16).to(dev)
        want = sum((x.float() * (r + 1)).to(torch.bfloat16).float() for r in range(tp.size))
        for _ in range(3):
            t2 = t.clone()
            tp.all_reduce(t2)
            torch.cuda.synchronize()
            err = (t2.float().cpu() - want).abs().max().item()
            ok &= math.isfinite(err) and err < 0.02 * (1 + want.abs().max().item())
        if tp.rank == 0:
            print(f"oneshot_allreduce rows={rows} err={err:.4g} error_word={tp.custom_ar.error()}", flush=True)
    return ok


def main():
    os.environ.setdefault("VWA_DIST_BACKEND", "gloo")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > torch.cuda.device_count():
        # ranks share a GPU: each chained (persistent) launch takes 1/world of the CUs so every
        # rank's launch is resident at once (their in-launch all-reduce rounds wait on each other)
        os.environ.setdefault("VWA_CHAIN_GRID_DIV", str(world))
    tp = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    ar_ok = ar_self_check(tp, dev)
    if os.environ.get("VWA_TP_CHECK_TRACE") == "1":
        install_nan_trace(tp)
    torch.manual_seed(0)
    toks = torch.randint(0, CFG.vocab_size, (110,)).tolist()
    ref_model = LlamaModel(CFG, device=dev, seed=7, tp=TPContext.single())
    ref, _ = run(ref_model, toks, graphs=False)
    ok = True
    for graphs in (False, True):
        m = LlamaModel(CFG, device=dev, seed=7, tp=tp)
        got, e = run(m, toks, graphs=graphs)
        errs = [(a - b).abs().max().item() for a, b in zip(got, ref)]
        ok &= all(math.isfinite(x) for x in errs)  # (max() would skip a NaN after the first entry)
        ok &= max(errs) < 0.05 * (1 + max(r.abs().max().item() for r in ref))
        if graphs:
            ok &= e.stats["graph_replays"] >= 5
        # the 1-row decode steps ran the chained layer with its in-launch all-reduce rounds
        n_chain = sum(v is not None for v in m.chain_descs())
        want_chain = tp.custom_ar is not None and os.environ.get("VWA_CHAIN_TP", "1") != "0"
        ok &= (n_chain > 0) == want_chain and not m.chain_error()
        if tp.rank == 0:
            print(f"graphs={graphs} custom_ar={tp.custom_ar is not None} embed_rows={m.embed.shape[0]} "
                  f"replays={e.stats['graph_replays']} chained_layers={n_chain} chain_error={m.chain_error()} "
                  f"max_errs={[round(x, 4) for x in errs]}", flush=True)
    s_ok = sample_check(tp, dev, ref_model, m)
    ok &= s_ok and ar_ok
    if tp.custom_ar is not None:
        ok &= not tp.custom_ar.error()
    if tp.rank == 0:
        print(f"vocab_parallel_sampling_equal={s_ok}", flush=True)
    res = torch.tensor([int(ok)])
    dist.all_reduce(res, op=dist.ReduceOp.MIN)
    if tp.rank == 0:
        print("TP_CHECK", "PASS" if res.item() else "FAIL", flush=True)
    dist.barrier()
    if tp.custom_ar is not None:
        tp.custom_ar.close()
    dist.destroy_process_group()
    sys.exit(0 if res.item() else 1)


if __name__ == "__main__":
    main()
