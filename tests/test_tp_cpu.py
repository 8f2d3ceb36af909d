"""Tensor-parallel intent decoding on CPU over gloo (4 ranks): the brain's TP control plane
(brain/server.py TPIntentEngine: rank 0 broadcasts each request, every rank decodes in lockstep)
with the vocab-parallel embedding (one all-reduce) and vocab-parallel sampling (partial maxima
exchanged, never logits).  All ranks must produce the same schema-valid answers, equal to the
TP=1 engine's (the Gumbel noise and tie-break use global token ids)."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from voice_enabled_browser_automation_amd import ops
from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
from voice_enabled_browser_automation_amd.brain.server import TPIntentEngine
from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
from voice_enabled_browser_automation_amd.models.config import LlamaConfig
from voice_enabled_browser_automation_amd.models.llama import LlamaModel
from voice_enabled_browser_automation_amd.ops import reference as ref
from voice_enabled_browser_automation_amd.parallel.tp import TPContext
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

TINY4 = LlamaConfig(name="tiny4", hidden=256, n_layers=2, n_heads=8, n_kv_heads=4, head_dim=32, ffn=512,
                    max_pos=4096)
TEXTS = ["search wireless earbuds", "scroll down"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(tp):
    m = LlamaModel(TINY4, device="cpu", seed=5, tp=tp)
    eng = LLMEngine(m, max_seqs=2, max_model_len=2048, kv_blocks=300)
    return LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=160, temperature=0.1, seed=11)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tp = TPContext(rank=rank, size=world, group=dist.group.WORLD)
        ie = _engine(tp)
        assert ie.engine.model.embed.shape[0] == ie.engine.model.v_end - ie.engine.model.v_start  # sharded
        tpe = TPIntentEngine(ie, tp)
        if rank == 0:
            outs = [tpe.parse({"text": t, "context": {"url": "https://www.bestbuy.com"}}) for t in TEXTS]
            tpe.stop()
        else:
            outs = tpe.worker_loop()
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def test_tp4_intent_engine_lockstep_matches_single():
    torch.set_num_threads(4)
    single = _engine(TPContext.single())
    want = [single.parse({"text": t, "context": {"url": "https://www.bestbuy.com"}}) for t in TEXTS]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(got) == [0, 1, 2, 3]
    for r in range(4):
        assert got[r] == got[0], f"rank {r} diverged from rank 0"
    for o in got[0]:
        assert safe_parse(ParseResponse, o).success
    assert got[0] == want


def test_vocab_parallel_sampling_equals_full_vocab_sampling():
    """The shard-wise partial maxima merged across ranks pick exactly the full-vocab token."""
    torch.manual_seed(0)
    rows, V, T = 3, 1000, 4
    logits = torch.randn(rows, V) * 3
    words = (V + 31) // 32
    mask = torch.randint(-2**31, 2**31 - 1, (rows, words), dtype=torch.int64).to(torch.int32)
    temp = torch.full((rows,), 0.7)
    seed, step = torch.tensor([123]), torch.tensor([5], dtype=torch.int32)
    full = torch.zeros(rows, dtype=torch.int32)
    ops.sample(logits, mask=mask, temperature=temp, seed=seed, step=step.clone(), out_tokens=full)
    per = ((V + T - 1) // T + 31) // 32 * 32
    vals, idx = [], []
    for r in range(T):
        lo, hi = r * per, min(V, (r + 1) * per)
        v, i = ref.sample_partial(logits[:, lo:hi], mask=mask, temperature=temp, seed=seed, step=step, v_offset=lo)
        vals.append(v)
        idx.append(i)
    merged = ref.merge_partials(torch.stack(vals), torch.stack(idx))
    assert merged.tolist() == full.tolist()
