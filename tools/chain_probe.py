"""Chained layer-tail launch vs separate launches on Llama-3-8B decode shapes (M rows), with
per-phase s_memrealtime stamps (100 MHz) from every workgroup of the chained kernel.

    python tools/chain_probe.py [--rows 1] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import voice_enabled_browser_automation_amd.ops as ops  # noqa: E402
from tools.bench_kernels import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--json", default=None)
    ap.add_argument("--bar-mode", type=int, default=2)
    ap.add_argument("--attn", action="store_true", help="decode attention (ctx 1100) as the first phase")
    ap.add_argument("--no-wait", action="store_true",
                    help="DIAGNOSTIC: barriers arrive but never wait (wrong results): phase cost without dependencies")
    ap.add_argument("--row-table", action="store_true", help="(always on: the chained attention requires them)")
    ap.add_argument("--ctx", type=int, default=1100, help="attention context length (tokens)")
    ap.add_argument("--n-splits", type=int, default=0, help="attention chunks per kv head cap (0: decode_n_splits(2048))")
    ap.add_argument("--kv-tok-major", action="store_true",
                    help="K/V blocks stored [block][token][head][dim] (a head's 16 tokens at 2 KB stride) "
                         "instead of [block][head][token][dim] (4 KB contiguous per head)")
    ap.add_argument("--warm-kv", action="store_true",
                    help="diagnostic: a standalone decode attention over the same K/V right before each chained "
                         "launch (its stamps then show the attention with warm caches / TLB)")
    ap.add_argument("--row-major", dest="tiled", action="store_false",
                    help="row-major [N, K] weights instead of the pre-tiled layout (ops.tile_weight)")
    ap.add_argument("--fp8", action="store_true", help="fp8 tiled weights (the W8A16 chain, ops.FP8Weight)")
    ap.add_argument("--no-plan", action="store_true",
                    help="(--attn) every launch derives the attention partition itself (no step plan)")
    ap.add_argument("--no-stamps", action="store_true",
                    help="launch without the per-phase stamps (their stores and waits slow the phases slightly)")
    ap.add_argument("--multi", type=int, default=0,
                    help="(--attn) also time N layers as ONE launch (chain_kernel MULTI; each layer its own K/V "
                         "cache, weights rotating over the copies): reports multi_layer_us = launch / N")
    a = ap.parse_args()
    if a.no_wait:
        a.bar_mode = 5 if a.bar_mode >= 4 else 3
    dev, bf = "cuda", torch.bfloat16
    E = ops.ext()
    torch.manual_seed(0)
    M, d, F, nq, nkv, hd = a.rows, 4096, 14336, 32, 8, 128
    ncopy = 3  # rotate weights over > 256 MB Infinity Cache
    mk = lambda *s: (torch.randn(*s, device=dev) * 0.02).to(bf)  # noqa: E731
    Ws = [dict(o=mk(d, nq * hd), gu=mk(2 * F, d), down=mk(d, F), qkv=mk((nq + 2 * nkv) * hd, d)) for _ in range(ncopy)]
    h, att, act = mk(M, d), mk(M, nq * hd), mk(M, F)
    q = torch.zeros(M, nq * hd, dtype=bf, device=dev)
    kc = torch.zeros(64, nkv, 16, hd, dtype=bf, device=dev)
    vc = torch.zeros_like(kc)
    pos = torch.arange(M, dtype=torch.int32, device=dev)
    slots = torch.arange(M, dtype=torch.int64, device=dev)
    rope = ops.rope_table(4096, hd, 5e5, device=dev)
    bar = E.alloc_uncached_i32(1024, torch.empty(1, device=dev)) if a.bar_mode >= 2 else \
        torch.zeros(1024, dtype=torch.int32, device=dev)
    ts = torch.zeros(1024 * 64, dtype=torch.int64, device=dev)  # 64 stamp slots per workgroup
    work = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    akw, ag = {}, 0
    if a.attn:  # the layer's attention over a 1100-token paged context as phase 0
        ctx, bs = a.ctx, 16
        nblk = (ctx + M + bs - 1) // bs + 1
        if a.kv_tok_major:
            akc = (torch.randn(nblk + 4, bs, nkv, hd, device=dev) * 0.5).to(bf).permute(0, 2, 1, 3)
            akv = torch.randn(nblk + 4, bs, nkv, hd, device=dev).to(bf).permute(0, 2, 1, 3)
        else:
            akc = (torch.randn(nblk + 4, nkv, bs, hd, device=dev) * 0.5).to(bf)
            akv = torch.randn_like(akc)
        table = (torch.randperm(nblk + 3, device=dev)[:nblk].to(torch.int32) + 1).view(1, nblk)
        lay = ops.KVLayout.paged(akc, akv, table)
        ns0 = ops.decode_n_splits(2048)
        ns = a.n_splits or ns0
        akw = dict(a_q=mk(M, nq * hd), a_k=akc, a_v=akv, a_table=table, a_block_size=bs, a_sb=lay.sb, a_sh=lay.sh,
                   a_st=lay.st, a_ctx=torch.arange(ctx, ctx + M, dtype=torch.int32, device=dev) + 1,
                   a_seq=torch.zeros(M, dtype=torch.int32, device=dev), a_scale=hd ** -0.5, a_n_splits=ns,
                   a_part_o=torch.zeros(M * ns0 * nq * hd, device=dev), a_part_ml=torch.zeros(M * ns0 * nq * 2, device=dev),
                   a_counters=torch.zeros(M * nkv, dtype=torch.int32, device=dev))
        ag = nq // nkv
        if True:  # per-row copies of the sequence's block table (required by the chained attention)
            rt = torch.zeros(M, 128, dtype=torch.int32, device=dev)
            rt[:, :nblk] = table[0]
            akw["a_row_table"] = rt
    if a.attn:  # the QKV phase writes the step's new keys into the attention's own paged cache
        kc, vc = akw["a_k"], akw["a_v"]  # (as the engine's next layer: same blocks, same table)
        tb = akw["a_table"][0].long()
        p_new = torch.arange(a.ctx, a.ctx + M, device=dev)
        slots = tb[p_new // 16] * 16 + p_new % 16
    sck = [{} for _ in Ws]
    if a.fp8:
        a.tiled = True
        for w, sc in zip(Ws, sck):
            for k in ("o", "gu", "down", "qkv"):
                f = ops.FP8Weight.quantize(w[k], tiled=True)
                w[k + "_t"], sc["s_" + k] = f.w8, f.scale
                w[k] = f  # the separate launches run the same fp8 weights
    elif a.tiled:  # the descriptors hold raw pointers: keep the tiled copies alive in Ws
        for w in Ws:
            w.update({k + "_t": ops.tile_weight(w[k]) for k in ("o", "gu", "down", "qkv")})
    wt = (lambda w, k: w[k + "_t"]) if a.tiled else (lambda w, k: w[k])  # noqa: E731
    plan = {}
    if a.attn and not a.no_plan:  # layers 1.. of a step: the plan layer 0 wrote (written once below)
        plan = dict(a_plan=torch.zeros(1024 * 16, dtype=torch.int32, device=dev), a_plan_mode=2)

    def make(w, sc, pl):
        return E.chain_make(h, att, act, wt(w, "o"), wt(w, "gu"), wt(w, "down"), 1e-5, wt(w, "qkv"), nq, nkv, hd, pos,
                            slots, rope, q, kc, vc, bar, work, None if a.no_stamps else ts, a.bar_mode, **akw,
                            w_tiled=a.tiled, **sc, **pl)

    descs = [make(w, sc, plan) for w, sc in zip(Ws, sck)]
    if plan:
        wdesc, wlds = make(Ws[0], sck[0], dict(plan, a_plan_mode=1))
        E.chain_run(wdesc, 4, wlds, h, ag)
    it = [0]

    def chained():
        it[0] = (it[0] + 1) % ncopy
        dsc, lds = descs[it[0]]
        if a.warm_kv and a.attn:
            ops.decode_attention(akw["a_q"], ops.KVLayout.paged(akw["a_k"], akw["a_v"], akw["a_table"]), akw["a_ctx"],
                                 akw["a_seq"], n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                                 max_ctx=2048, out=akw["a_q"].new_empty(akw["a_q"].shape), part_o=akw["a_part_o"],
                                 part_ml=akw["a_part_ml"], counters=akw["a_counters"])
        E.chain_run(dsc, 4, lds, h, ag)

    def separate():
        it[0] = (it[0] + 1) % ncopy
        w = Ws[it[0]]
        if a.attn:
            ops.decode_attention(akw["a_q"], ops.KVLayout.paged(akw["a_k"], akw["a_v"], akw["a_table"]), akw["a_ctx"],
                                 akw["a_seq"], n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                                 max_ctx=2048, out=att, part_o=akw["a_part_o"], part_ml=akw["a_part_ml"],
                                 counters=akw["a_counters"])
        ops.linear(att, w["o"], out=h, residual=h)
        ops.linear_swiglu(h, w["gu"], fuse_rms=True, eps=1e-5, out=act)
        ops.linear(act, w["down"], out=h, residual=h)
        ops.qkv_rope_write(h, w["qkv"], None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                           rope=rope, positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)

    multi_us = None
    if a.multi > 1 and a.attn:
        # N layers, layer i on weight copy i % ncopy and its own paged K/V (same table); layer 0
        # writes the step plan, layers 1.. read it (as the engine's multi-layer launch)
        mplan = torch.zeros(1024 * 16, dtype=torch.int32, device=dev)
        kvs = [(torch.randn_like(akw["a_k"]) * 0.5, torch.randn_like(akw["a_v"])) for _ in range(a.multi + 1)]
        mds = []
        for li in range(a.multi):
            w = Ws[li % ncopy]
            kw = dict(akw, a_k=kvs[li][0], a_v=kvs[li][1])
            mds.append(E.chain_make(h, att, act, wt(w, "o"), wt(w, "gu"), wt(w, "down"), 1e-5, wt(w, "qkv"), nq, nkv,
                                    hd, pos, slots, rope, q, kvs[li + 1][0], kvs[li + 1][1], bar, work, None, a.bar_mode,
                                    **kw, w_tiled=a.tiled, **sck[li % ncopy], a_plan=mplan,
                                    a_plan_mode=1 if li == 0 else 2))
        mcat = torch.cat([d[0] for d in mds])
        mlds = mds[0][1]

        def multi():
            E.chain_run(mcat, 4, mlds, h, ag, 0, a.multi)

        def per_layer():
            for d in mds:
                E.chain_run(d[0], 4, d[1], h, ag)

        multi()
        torch.cuda.synchronize()
        assert int(bar.view(torch.int64)[160].item()) == 0, "barrier timeout (multi)"
        multi_us = timeit(multi) / a.multi
        per_layer_us = timeit(per_layer) / a.multi
        assert int(bar.view(torch.int64)[160].item()) == 0, "barrier timeout (multi)"
    chained()  # one launch first: a broken barrier shows up as the error word, not a long run
    torch.cuda.synchronize()
    assert int(bar.view(torch.int64)[160].item()) == 0, "barrier timeout"
    t_sep = 0.0 if a.no_wait else timeit(separate)
    t_ch = timeit(chained)
    assert int(bar.view(torch.int64)[160].item()) == 0, "barrier timeout"
    # stamps of the last launch: [start, end0, wait0, end1, wait1, end2, wait2, end3]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    ns_ = 9 if a.attn else 8
    st = ts.view(-1, 64)[:cus, :ns_].double().cpu()
    st = (st - st[:, :1].min()) * 10e-3  # us
    med = st.median(dim=0).values.tolist()
    mx = st.max(dim=0).values.tolist()
    mn = st.min(dim=0).values.tolist()
    if a.attn:  # in-attention stamps 9..14 of the attention workgroups (slots stay 0 elsewhere)
        full = ts.view(-1, 64)[:cus].double().cpu()
        t0 = full[:, 0].min()
        att = full[full[:, 9] > 0]
        names = ["ctx_known", "q_ready", "pre_sync", "meta_landed", "kv_issue", "merged", "kv_landed", "meta_regs", "n_items", "loop_top", "ctxmax", "chunk_known", "pre_loop"]
        extra = {}
        for j, nm in enumerate(names):
            col = att[:, 9 + j]
            col = col[col > 0]
            if col.numel():
                extra[nm] = [round(float((col.median() - t0) * 10e-3), 2), round(float((col.max() - t0) * 10e-3), 2)]
    r = dict(kernel="chain_probe", rows=M, plan=bool(plan), fp8=a.fp8, ctx=a.ctx if a.attn else None, warm_kv=a.warm_kv, n_splits=a.n_splits, kv_tok_major=a.kv_tok_major, bar_mode=a.bar_mode, tiled=a.tiled, row_table=a.row_table, separate_us=round(t_sep, 2), chained_us=round(t_ch, 2),
             stamps_med_us=[round(x, 2) for x in med], stamps_min_us=[round(x, 2) for x in mn],
             stamps_max_us=[round(x, 2) for x in mx],
             legend=("start,end_attn," if a.attn else "start,") + "end_o,wait_o,end_gu,wait_gu,end_down,wait_down,end_qkv")
    if a.attn:
        r["attn_stamps_med_max_us"] = extra
        # phase stamps split by role: workgroups that ran an attention item vs the others
        isatt = full[:, 9] > 0
        for nm, sel in (("attn_wg", isatt), ("other_wg", ~isatt)):
            if int(sel.sum()):
                for slot, key in ((12, "meta_landed"), (56, "idle_issued")):
                    col = full[sel, slot]
                    col = col[col > t0]
                    if col.numel():
                        r[f"{nm}_{key}"] = [round(float((col.median() - t0) * 10e-3), 2),
                                            round(float((col.max() - t0) * 10e-3), 2)]
                s = st[sel]
                r[nm] = dict(n=int(sel.sum()), med=[round(x, 2) for x in s.median(dim=0).values.tolist()],
                             max=[round(x, 2) for x in s.max(dim=0).values.tolist()],
                             argmax=[int(i) for i in torch.nonzero(sel).flatten()[s.argmax(dim=0)].tolist()])
                # in-phase stamps (chain_phase pst): o_proj entry, X staged, scales, item0, fin0,
                # item1, fin1 | gate/up entry, X staged, scales
                ph = {}
                # chain_phase pst: phase i at slots 22 + 8 i + k
                kn = ["entry", "xstaged", "scales", "item0", "fin0", "item1", "fin1"]
                for j, pn in [(8 * i + k, f"{pre}_{n}") for i, pre in enumerate(["o", "gu", "down", "qkv"])
                              for k, n in enumerate(kn)]:
                    col = full[sel, 22 + j]
                    col = col[col > 0]
                    if col.numel():
                        ph[pn] = [round(float((col.median() - t0) * 10e-3), 2), round(float((col.max() - t0) * 10e-3), 2),
                                  int(col.numel())]
                r[nm + "_phase"] = ph
    if multi_us is not None:
        r.update(multi_layers=a.multi, multi_layer_us=round(multi_us, 2), per_layer_launch_us=round(per_layer_us, 2))
    r["env"] = {k: v for k, v in os.environ.items() if k.startswith("VWA_CHAIN")}
    r["layer_us"] = round(float(mx[-1]), 2)
    print(json.dumps(r), flush=True)
    if a.json:
        with open(a.json, "a") as f:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
