"""Decode-attention latency + numerics probe (graph-replayed GPU time per call).

Shapes the engines actually run: Llama-3-8B geometry (32 q / 8 kv heads x 128, paged KV) with
one sequence of 1..64 rows (last sampled token + jump-forward rows, or a prompt-suffix chunk),
R independent sessions of one row each, and the Whisper decoder's cross/self attention
(MHA, head_dim 64).  Each shape runs on both kernels (ops.set_attention_impl) and is checked
against the fp32 torch reference.
Usage: python tools/attn_probe.py [--json out.json] [--impls mq,split]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from bench_kernels import timeit  # noqa: E402


def case(rows, ctx, same_seq, nq=32, nkv=8, hd=128, bs=16, max_ctx=2048, shared=0, use_shared=True,
         n_splits=None):
    dev = "cuda"
    n_seq = 1 if same_seq else rows
    per = (max_ctx + bs - 1) // bs
    blocks = n_seq * per + 8
    kc = torch.randn(blocks, nkv, bs, hd, device=dev).to(torch.bfloat16)
    vc = torch.randn_like(kc)
    # shuffled physical blocks: the layout the block manager produces after churn
    perm = torch.randperm(blocks - 1, device=dev)[: n_seq * per].to(torch.int32) + 1
    table = perm.view(n_seq, per).contiguous()
    if shared:  # sessions over one cached prompt prefix: the same physical blocks (prefix cache)
        table[:, : shared // bs] = table[0, : shared // bs]
    q = torch.randn(rows, nq * hd, device=dev).to(torch.bfloat16)
    out = torch.empty_like(q)
    if same_seq:
        cl = torch.arange(ctx - rows + 1, ctx + 1, dtype=torch.int32, device=dev)
        sid = torch.zeros(rows, dtype=torch.int32, device=dev)
    else:
        cl = torch.full((rows,), ctx, dtype=torch.int32, device=dev)
        sid = torch.arange(rows, dtype=torch.int32, device=dev)
    kv = ops.KVLayout.paged(kc, vc, table)
    ns = ops.decode_n_splits(max_ctx)
    po = torch.empty(rows * ns * nq * hd, device=dev)
    pm = torch.empty(rows * ns * nq * 2, device=dev)
    cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=dev)

    sh = torch.tensor([shared, rows], dtype=torch.int32, device=dev) if shared and use_shared else None

    def f():
        ops.decode_attention(q, kv, cl, sid, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                             max_ctx=max_ctx, out=out, part_o=po, part_ml=pm, counters=cnt, shared=sh,
                             n_splits=n_splits)

    t = timeit(f)
    f()
    torch.cuda.synchronize()
    ref = ops.reference.decode_attention(q.cpu(), ops.KVLayout.paged(kc.cpu(), vc.cpu(), table.cpu()), cl.cpu(),
                                         sid.cpu(), n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                                         out=torch.empty(q.shape, dtype=q.dtype))
    err = (out.cpu().float() - ref.float()).abs().max().item()
    kv_mb = (n_seq * ctx - (n_seq - 1) * shared) * nkv * hd * 2 * 2 / 1e6
    return dict(kernel="decode_attention", rows=rows, ctx=ctx, same_seq=same_seq, shared=shared,
                grouped=bool(sh is not None), n_splits=n_splits,
                heads=f"{nq}/{nkv}x{hd}",
                us=round(t, 2), kv_mb=round(kv_mb, 2), max_err=round(err, 4))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--impls", default="mq,split")
    ap.add_argument("--only-llama", action="store_true", help="skip the Whisper / 70B shapes")
    ap.add_argument("--split-sweep", action="store_true",
                    help="sessions over a shared prefix: chunk cap x shared-prefix grouping on / off")
    args = ap.parse_args()
    torch.manual_seed(0)
    res = []
    shapes = [dict(rows=1, ctx=1100, same_seq=True), dict(rows=2, ctx=1100, same_seq=True),
              dict(rows=4, ctx=1100, same_seq=True), dict(rows=8, ctx=1100, same_seq=True),
              dict(rows=21, ctx=1100, same_seq=True), dict(rows=64, ctx=1100, same_seq=True),
              dict(rows=8, ctx=1100, same_seq=False), dict(rows=32, ctx=1100, same_seq=False),
              # sessions sharing the cached 1k-token intent prompt prefix (the serving case)
              dict(rows=8, ctx=1200, same_seq=False, shared=1024), dict(rows=16, ctx=1200, same_seq=False, shared=1024),
              dict(rows=32, ctx=1200, same_seq=False, shared=1024), dict(rows=64, ctx=1200, same_seq=False, shared=1024),
              dict(rows=1, ctx=300, same_seq=True), dict(rows=1, ctx=2000, same_seq=True),
              # Whisper decoder: cross-attention over the 1500-frame window, self-attention
              dict(rows=1, ctx=1500, same_seq=True, nq=6, nkv=6, hd=64),
              dict(rows=1, ctx=1500, same_seq=True, nq=20, nkv=20, hd=64),
              dict(rows=1, ctx=44, same_seq=True, nq=20, nkv=20, hd=64, max_ctx=448),
              # Llama-3-70B at TP=8: one kv head, 8 q heads per rank
              dict(rows=1, ctx=1100, same_seq=True, nq=8, nkv=1, hd=128)]
    if args.split_sweep:
        shapes = [dict(rows=r, ctx=1200, same_seq=False, shared=1024, use_shared=u, n_splits=ns)
                  for r in (8, 16, 32, 64) for u in (True, False) for ns in (None, 8, 4, 2, 1)]
    if args.only_llama:
        shapes = [s for s in shapes if s.get("nq", 32) == 32]
    for impl in args.impls.split(","):
        ops.set_attention_impl(impl)
        for sh in shapes:
            r = dict(impl=impl, **case(**sh))
            print(json.dumps(r), flush=True)
            res.append(r)
    ops.set_attention_impl("mq")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
