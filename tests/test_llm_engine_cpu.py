"""LLM engine on CPU (reference ops): paged KV + ragged decode == full prefill, prefix cache,
grammar-constrained intent generation, and tensor parallelism over gloo (world size 2)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.models.config import LLAMA_PRESETS, LlamaConfig
from voice_enabled_browser_automation_amd.models.llama import LlamaModel
from voice_enabled_browser_automation_amd.parallel.tp import TPContext
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.runtime.kv_cache import BlockManager
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

SMALL = LlamaConfig(name="t", vocab_size=512, hidden=128, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=32,
                    ffn=256, max_pos=1024)


def test_block_manager_prefix_cache():
    bm = BlockManager(num_blocks=16, block_size=4)
    toks = list(range(13))
    blocks = bm.allocate(4)
    bm.register_prefix(toks, blocks, 13)
    bm.release(blocks)
    hit, n = bm.match_prefix(toks + [99])
    assert n == 12 and hit == blocks[:3]
    hit2, n2 = bm.match_prefix([7] + toks)
    assert n2 == 0 and hit2 == []
    bm.release(hit)
    # exhaustion evicts unreferenced cached blocks instead of failing
    got = bm.allocate(15)
    assert len(set(got)) == 15 and 0 not in got


def test_ragged_decode_matches_full_prefill():
    torch.manual_seed(0)
    m = LlamaModel(SMALL, device="cpu", seed=3)
    toks = torch.randint(0, 512, (90,)).tolist()
    # A: full prefill (flash path, 90 rows)
    eA = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
    sA = eA.new_sequence(toks, use_prefix_cache=False)
    la = eA.prefill(sA)
    # B: prefill 60 rows (ragged path) then decode the remaining 30 tokens one by one
    eB = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
    sB = eB.new_sequence(toks[:60], use_prefix_cache=False)
    eB.prefill(sB)
    lb = None
    for t in toks[60:]:
        lb = eB.run_rows([(sB, t)])
    assert torch.allclose(la.float(), lb.float(), atol=3e-2, rtol=3e-2), (la - lb).abs().max()
    # C: jump-forward style multi-row step of one sequence
    eC = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
    sC = eC.new_sequence(toks[:70], use_prefix_cache=False)
    eC.prefill(sC)
    lc = eC.run_rows([(sC, t) for t in toks[70:]])[-1:]
    assert torch.allclose(la.float(), lc.float(), atol=3e-2, rtol=3e-2)


def test_intent_engine_constrained_valid_and_prefix_cached():
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cpu", seed=1)
    eng = LLMEngine(m, max_seqs=2, max_model_len=2048, kv_blocks=400)
    ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=200)
    for text in ["search wireless earbuds", "open the second result"]:
        out = ie.parse({"text": text, "context": {}})
        assert safe_parse(ParseResponse, out).success
        assert ie.last_stats["output_chars"] <= 200
    assert ie.last_stats["cached_prefix_tokens"] > 900  # static system + few-shot prefix served from cache
    assert ie.last_stats["forced_tokens"] > 0  # jump-forward engaged


def test_logit_row_selection_matches_all_rows():
    torch.manual_seed(0)
    m = LlamaModel(SMALL, device="cpu", seed=3)
    toks = torch.randint(0, 512, (40,)).tolist()
    outs = []
    for sel in (None, [2, 5]):
        e = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
        a = e.new_sequence(toks[:20], use_prefix_cache=False)
        b = e.new_sequence(toks[20:37], use_prefix_cache=False)
        e.prefill(a)
        e.prefill(b)
        rows = [(a, toks[37]), (a, toks[38]), (a, toks[39]), (b, 1), (b, 2), (b, 3)]
        lg = e.run_rows(rows, logits_for=sel)
        outs.append(lg if sel is not None else lg[[2, 5]])
    assert outs[0].shape == outs[1].shape == (2, 512)
    assert torch.allclose(outs[0].float(), outs[1].float(), atol=1e-3)


def test_intent_engine_continuous_batching_matches_sequential_greedy():
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cpu", seed=1)
    texts = ["search wireless earbuds", "open the second result", "scroll down", "go back"]
    reqs = [{"text": t, "context": {}} for t in texts]
    seq_out = []
    eng = LLMEngine(m, max_seqs=4, max_model_len=2048, kv_blocks=800)
    ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=160, temperature=0.0)
    for r in reqs:
        seq_out.append(ie.parse(r))
    eng2 = LLMEngine(m, max_seqs=4, max_model_len=2048, kv_blocks=800)
    ie2 = LLMIntentEngine(eng2, load_tokenizer("llama3"), budget_chars=160, temperature=0.0, max_active=3)
    batch_out = ie2.parse_many(reqs)
    for a in batch_out:
        assert safe_parse(ParseResponse, a).success
    assert ie2.batch_stats["max_active"] == 3  # 4 requests through 3 slots: admission mid-flight
    assert ie2.batch_stats["sampled"] > ie2.batch_stats["iterations"]  # iterations shared by requests
    assert batch_out == seq_out  # greedy: batching does not change any request's answer


def test_intent_engine_background_scheduler():
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cpu", seed=1)
    eng = LLMEngine(m, max_seqs=4, max_model_len=2048, kv_blocks=800)
    with pytest.raises(Exception, match="budget_chars=100"):
        LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=100).parse({"text": "x", "context": {}})
    ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=200)
    ie.start()
    try:
        from voice_enabled_browser_automation_amd.brain.prompt import messages_for

        futs = [ie.submit_async(messages_for({"text": t, "context": {}})) for t in ("scroll up", "take a screenshot")]
        import json

        for f in futs:
            assert safe_parse(ParseResponse, json.loads(f.result(timeout=300))).success
    finally:
        ie.stop()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tp_worker(rank, world, port, toks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tp = TPContext(rank=rank, size=world, group=dist.group.WORLD)
        m = LlamaModel(SMALL, device="cpu", seed=3, tp=tp)
        e = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
        s = e.new_sequence(toks[:40], use_prefix_cache=False)
        e.prefill(s)
        logits = e.run_rows([(s, toks[40]), (s, toks[41])])
        if rank == 0:
            q.put(logits.float().numpy().copy())  # by value: a torch tensor travels as a shared fd the exiting worker may close first
    finally:
        dist.destroy_process_group()


def test_tensor_parallel_gloo_matches_single():
    torch.manual_seed(0)
    toks = torch.randint(0, 512, (42,)).tolist()
    m = LlamaModel(SMALL, device="cpu", seed=3)
    e = LLMEngine(m, max_seqs=2, max_model_len=256, kv_blocks=64, block_size=16)
    s = e.new_sequence(toks[:40], use_prefix_cache=False)
    e.prefill(s)
    ref = e.run_rows([(s, toks[40]), (s, toks[41])]).float()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, toks, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = torch.from_numpy(q.get(timeout=300))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got.shape == ref.shape
    assert torch.allclose(got, ref, atol=3e-2, rtol=3e-2), (got - ref).abs().max()


def test_long_forced_feed_is_consumed_in_pieces():
    """A jump-forward feed longer than the engine's row cap is run in pieces: every piece reaches
    the KV cache (greedy answers equal the ones of an engine whose row cap takes the feed whole)."""
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cpu", seed=1)
    outs, stats, rows = [], [], []
    for max_rows in (64, 4):
        eng = LLMEngine(m, max_seqs=2, max_model_len=2048, kv_blocks=400, max_rows=max_rows)
        ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=160, temperature=0.0)
        outs.append(ie.parse({"text": "search wireless earbuds", "context": {}}))
        stats.append(dict(ie.batch_stats))
        rows.append(eng.stats["rows"])
    assert safe_parse(ParseResponse, outs[1]).success
    assert stats[1]["iterations"] > stats[0]["iterations"]  # the capped engine split some feeds
    assert rows[0] == rows[1]  # ... and still ran every fed token through the model
    assert outs[0] == outs[1]


def test_sampler_fail_word_marks_every_row():
    from voice_enabled_browser_automation_amd import ops

    logits = torch.randn(3, 64)
    out = torch.zeros(3, dtype=torch.int32)
    kw = dict(mask=None, temperature=None, seed=torch.tensor([0]), step=torch.zeros(1, dtype=torch.int32),
              out_tokens=out)
    ops.sample(logits, fail_word=torch.zeros(1, dtype=torch.int64), **kw)
    assert out.tolist() == logits.argmax(-1).tolist()
    ops.sample(logits, fail_word=torch.ones(1, dtype=torch.int64), **kw)
    assert out.tolist() == [-2, -2, -2]


def test_reference_attention_matches_per_head_loops():
    """The CPU attention (ops/reference.py: every head of a row in one batched product, one K/V
    gather per sequence) equals plain per-(row, head) softmax(q K^T) V over the paged cache --
    GQA, ragged contexts, rows of one sequence at different positions, a contiguous-layout
    causal prefill."""
    import math

    import torch

    from voice_enabled_browser_automation_amd import ops
    from voice_enabled_browser_automation_amd.ops import reference as ref

    g = torch.Generator().manual_seed(0)
    nq, nkv, D, bs, nblk = 8, 2, 32, 4, 40
    kc = torch.randn(nblk, nkv, bs, D, generator=g)
    vc = torch.randn(nblk, nkv, bs, D, generator=g)
    table = torch.randperm(nblk, generator=g)[:24].view(2, 12).to(torch.int32)
    kv = ops.KVLayout.paged(kc, vc, table)
    ctx = torch.tensor([5, 6, 7, 30, 1], dtype=torch.int32)
    sid = torch.tensor([0, 0, 0, 1, 1], dtype=torch.int32)
    q = torch.randn(5, nq * D, generator=g)
    out = torch.empty_like(q)
    ref.decode_attention(q, kv, ctx, sid, n_q_heads=nq, n_kv_heads=nkv, head_dim=D, scale=D ** -0.5, out=out)
    G = nq // nkv
    for r in range(5):
        n, s = int(ctx[r]), int(sid[r])
        toks = [(int(table[s, t // bs]), t % bs) for t in range(n)]
        for h in range(nq):
            K = torch.stack([kc[b, h // G, o] for b, o in toks])
            V = torch.stack([vc[b, h // G, o] for b, o in toks])
            p = torch.softmax(K @ q[r, h * D:(h + 1) * D] / math.sqrt(D), 0)
            assert torch.allclose(out[r, h * D:(h + 1) * D], p @ V, atol=1e-5)
    # contiguous [B, S, H, D] layout, causal with a query offset
    B, S, Sq = 2, 9, 4
    k = torch.randn(B, S, nkv, D, generator=g)
    v = torch.randn(B, S, nkv, D, generator=g)
    qq = torch.randn(B, Sq, nq, D, generator=g)
    o = torch.empty_like(qq)
    ref.flash_attention(qq, ops.KVLayout.contiguous(k, v, torch.arange(B, dtype=torch.int32)[:, None]), Sk=S,
                        n_kv_heads=nkv, causal=True, scale=D ** -0.5, q_offset=S - Sq, out=o)
    for b in range(B):
        for i in range(Sq):
            for h in range(nq):
                n = S - Sq + i + 1
                p = torch.softmax(k[b, :n, h // G] @ qq[b, i, h] / math.sqrt(D), 0)
                assert torch.allclose(o[b, i, h], p @ v[b, :n, h // G], atol=1e-5)


def test_batched_admission_prefill_matches_serial_prefill():
    """runtime/engine.py prefill_batch: several requests' prompt suffixes behind a cached prefix in
    ONE ragged forward (> 64 rows: eager scratch forward, attention in 64-row slices; <= 64 rows:
    a step bucket) leave the same K/V -- and hence the same next-token logits -- as one prefill per
    request; a cold prompt among them takes the single-sequence path."""
    torch.manual_seed(0)
    m = LlamaModel(SMALL, device="cpu", seed=3)
    head = torch.randint(0, 512, (64,)).tolist()
    tails = [torch.randint(0, 512, (n,)).tolist() for n in (40, 33, 27)]
    cold = torch.randint(0, 512, (80,)).tolist()

    def make():
        e = LLMEngine(m, max_seqs=5, max_model_len=256, kv_blocks=120, block_size=16)
        s0 = e.new_sequence(head)
        e.prefill(s0)
        e.free_sequence(s0)  # publishes the shared head to the prefix cache
        seqs = [e.new_sequence(head + t) for t in tails] + [e.new_sequence(cold)]
        assert all(s.n_computed == 64 for s in seqs[:3]) and seqs[3].n_computed == 0
        return e, seqs

    def next_logits(e, seqs):
        return [e.run_rows([(s, 7)]).float().clone() for s in seqs]

    eA, sA = make()
    for s in sA:
        eA.prefill(s)
    want = next_logits(eA, sA)
    eB, sB = make()
    eB.prefill_batch([(s, len(s.tokens)) for s in sB])  # 100 suffix rows + one cold prompt
    assert [s.n_computed for s in sB] == [len(s.tokens) for s in sB]
    assert eB.stats["batched_prefills"] == 1
    got = next_logits(eB, sB)
    for a, b in zip(got, want):
        assert torch.allclose(a, b, atol=2e-2, rtol=2e-2), (a - b).abs().max()
    eC, sC = make()
    eC.prefill_batch([(s, len(s.tokens)) for s in sC[1:3]])  # 60 rows: one step-bucket forward
    for a, b in zip(next_logits(eC, sC[1:3]), want[1:3]):
        assert torch.allclose(a, b, atol=2e-2, rtol=2e-2), (a - b).abs().max()


def test_rms_statistics_handoff_paths_without_the_tiled_gemm():
    """ops.linear's RMS-statistics arguments (GemmParams::ss_*, used by the > 16-row GPU path)
    keep their meaning on paths without the hand-off: ss_out gets the squares of the stored rows
    added, ss_zero is cleared, ss_in is ignored (the consumer computes its own 1/rms)."""
    import voice_enabled_browser_automation_amd.ops as ops

    torch.manual_seed(0)
    M, K, N = 20, 256, 128
    x, h = torch.randn(M, K).to(torch.bfloat16), torch.randn(M, N).to(torch.bfloat16)
    w = (torch.randn(N, K) * 0.05).to(torch.bfloat16)
    ss = torch.full((2, 64), 3, dtype=torch.int64)  # (u64 fixed point, ops.SS_SCALE units)
    ss[0].zero_()
    out = h.clone()
    ops.linear(x, w, out=out, residual=out, ss_out=ss[0], ss_zero=ss[1])
    assert torch.all(ss[1] == 0)
    torch.testing.assert_close(ops.ss_float(ss[0, :M]).float(), out.float().pow(2).sum(-1), rtol=1e-5, atol=1e-3)
    assert torch.all(ss[0, M:] == 0)
    ref = h.clone()
    ops.linear(x, w, out=ref, residual=ref)
    assert torch.equal(out, ref)
    gu = ops.interleave_gate_up((torch.randn(64, N) * 0.05).to(torch.bfloat16), (torch.randn(64, N) * 0.05).to(torch.bfloat16))
    a = ops.linear_swiglu(out, gu, fuse_rms=True, eps=1e-5, ss_in=ss[0])
    b = ops.linear_swiglu(out, gu, fuse_rms=True, eps=1e-5)
    assert torch.equal(a, b)
