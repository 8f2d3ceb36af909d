"""HBM plan per rank (runtime/memory_plan.py) vs the weights a sharded model really holds, on the
meta device: Llama-3-70B at TP=8 (BASELINE config 4: 288 GB/GPU KV sizing), Llama-3-8B at TP=2
(config 3) and fp8 (config 5).  One weight copy per projection; vocab-parallel embedding."""
import pytest

from voice_enabled_browser_automation_amd.models.config import get_config
from voice_enabled_browser_automation_amd.models.llama import LlamaModel
from voice_enabled_browser_automation_amd.parallel.tp import TPContext
from voice_enabled_browser_automation_amd.runtime.memory_plan import HBM_BYTES_MI355X, plan_memory


@pytest.mark.parametrize("name,tp,wdtype", [("llama3-70b", 8, "bf16"), ("llama3-8b", 2, "bf16"),
                                            ("llama3-8b", 1, "fp8"), ("llama3-70b", 8, "fp8")])
def test_plan_matches_sharded_model(name, tp, wdtype):
    cfg = get_config(name)
    plan = plan_memory(cfg, tp, wdtype=wdtype)
    held = []
    for r in range(tp):
        m = LlamaModel(cfg, device="meta", tp=TPContext(rank=r, size=tp), wdtype=wdtype)
        held.append(m.param_bytes())
        assert m.embed.shape[0] == m.v_end - m.v_start and m.lm_head.shape[0] == m.v_end - m.v_start
    assert max(held) == plan.weights + plan.embedding  # rank 0 holds a full-width shard
    assert plan.as_dict()["fits"] and plan.total <= HBM_BYTES_MI355X
    total_params = sum(held)
    if name == "llama3-70b" and wdtype == "bf16":
        # ~70.6 B parameters x 2 B over 8 ranks: ~17.6 GB per rank, ~230 GB of KV left per GPU
        assert 16.5e9 < held[0] < 18.5e9
        assert 135e9 < total_params < 145e9
        assert plan.kv_bytes > 200e9
        # 40 KiB of K/V per token per rank (2 x 80 layers x 1 kv head x 128 x 2 B)
        assert plan.kv_bytes_per_token == 2 * 80 * 1 * 128 * 2
        assert plan.kv_tokens > 5_000_000  # 32 sessions x 4k context is < 3 % of it
    if wdtype == "fp8":
        bf = plan_memory(cfg, tp, wdtype="bf16")
        assert plan.weights < 0.52 * bf.weights


def test_kv_budget_cap():
    cfg = get_config("llama3-8b")
    p = plan_memory(cfg, 1, kv_gb=10)
    assert 9.9e9 < p.kv_bytes <= 10e9 and p.kv_blocks * 16 * p.kv_bytes_per_token == p.kv_bytes
