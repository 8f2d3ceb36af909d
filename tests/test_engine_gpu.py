"""Whole-model numerics on the GPU: the native-kernel engine (hipGraph-replayed ragged decode,
prefill path, streaming GEMMs, fused attention) against the CPU reference engine with the SAME
weights, for Llama (GQA + RoPE) and Whisper (encoder + decoder with cross-attention)."""
import math

import numpy as np
import pytest
import torch

from voice_enabled_browser_automation_amd import ops
from voice_enabled_browser_automation_amd.asr.engine import AsrEngine
from voice_enabled_browser_automation_amd.models.config import LlamaConfig, get_config
from voice_enabled_browser_automation_amd.models.llama import LlamaModel, move_model
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

pytestmark = pytest.mark.gpu

CFG = LlamaConfig(name="t", vocab_size=4096, hidden=512, n_layers=3, n_heads=8, n_kv_heads=2, head_dim=64,
                  ffn=1024, max_pos=2048)


def _run(model, toks, split):
    e = LLMEngine(model, max_seqs=2, max_model_len=512, kv_blocks=80, block_size=16)
    s = e.new_sequence(toks[:split], use_prefix_cache=False)
    # clone: on the CPU engine .float().cpu() is a view of the step's logits buffer
    out = [e.prefill(s).float().cpu().clone()]
    out.append(e.run_rows([(s, toks[split])]).float().cpu().clone())
    out.append(e.run_rows([(s, t) for t in toks[split + 1 :]])[-1:].float().cpu().clone())
    return out


def test_llama_gpu_engine_matches_cpu_reference():
    ops.ext()
    torch.manual_seed(0)
    toks = torch.randint(0, CFG.vocab_size, (140,)).tolist()
    cpu = LlamaModel(CFG, device="cpu", seed=5)
    ref = _run(cpu, toks, 120)
    gpu = LlamaModel(CFG, device="cpu", seed=5)
    move_model(gpu, "cuda")
    got = _run(gpu, toks, 120)
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert err < 0.05 * (1 + b.abs().max().item()), (i, err)
        assert int(a.argmax()) == int(b.argmax()) or err < 0.02


def test_whisper_gpu_matches_cpu_reference():
    ops.ext()
    tok = load_tokenizer("whisper")
    cpu = WhisperModel(get_config("whisper-test"), device="cpu", seed=3)
    gpu = WhisperModel(get_config("whisper-test"), device="cpu", seed=3)
    move_model(gpu, "cuda")
    pcm = (np.sin(np.arange(16000 * 3) * 2 * np.pi * 330 / 16000) * 7000).astype(np.int16)
    a_cpu = AsrEngine(cpu, tok, max_sessions=1)
    a_gpu = AsrEngine(gpu, tok, max_sessions=1)
    mel_c = cpu.log_mel(a_cpu.pcm_to_audio(pcm))
    mel_g = gpu.log_mel(a_gpu.pcm_to_audio(pcm))
    assert (mel_c.float() - mel_g.float().cpu()).abs().max() < 0.05
    enc_c = cpu.encode(mel_c[None])
    enc_g = gpu.encode(mel_g[None])
    assert (enc_c.float() - enc_g.float().cpu()).abs().max() < 0.1 * (1 + enc_c.float().abs().max())
    tc = a_cpu.transcribe(a_cpu.pcm_to_audio(pcm), exact_tokens=6)
    tg = a_gpu.transcribe(a_gpu.pcm_to_audio(pcm), exact_tokens=6)
    assert isinstance(tg, str) and a_gpu.last_stats["tokens"] == 6
    # greedy decode of identical weights: first tokens agree (bf16 noise may flip late near-ties)
    assert tc[:4] == tg[:4] or len(tc) == 0


def test_intent_engine_continuous_batching_gpu():
    """Concurrent sessions through the hipGraph engine: every answer schema-valid, iterations
    shared across requests, logit-row selection graphs in use."""
    from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
    from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse
    from voice_enabled_browser_automation_amd.models.config import LLAMA_PRESETS

    ops.ext()
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cuda", seed=1)
    eng = LLMEngine(m, max_seqs=8, max_model_len=2048)
    eng.capture_all()
    ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=256, temperature=0.1, max_active=6)
    texts = ["search wireless earbuds", "open the second result", "scroll down", "go back", "sort by price",
             "take a screenshot", "filter by brand sony", "type hello into the search box"]
    outs = ie.parse_many([{"text": t, "context": {}} for t in texts])
    assert all(safe_parse(ParseResponse, o).success for o in outs)
    assert ie.batch_stats["max_active"] == 6
    assert ie.batch_stats["sampled"] > 2 * ie.batch_stats["iterations"]
    assert any(L < M for (M, L, _gated) in eng.graphs)


def test_masked_lm_head_gives_the_dense_heads_answers():
    """The grammar-masked LM head (LLMEngine.head_logits(col_mask=...)) skips the vocab tiles no
    row may sample; the admissible logits are the dense head's, so the sampled answers are the
    same token for token (one session and a continuous batch)."""
    from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
    from voice_enabled_browser_automation_amd.models.config import LLAMA_PRESETS

    ops.ext()
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cuda", seed=4)
    assert isinstance(m.lm_head, ops.TiledWeight)  # the streaming kernel (the masked path) runs the head
    texts = ["search wireless earbuds", "scroll down", "sort by price", "go back"]
    outs = {}
    for masked in (True, False):
        eng = LLMEngine(m, max_seqs=4, max_model_len=2048)
        ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=200, temperature=0.1, seed=7)
        ie.masked_head = masked
        outs[masked] = [ie.generate(ie_msgs) for ie_msgs in
                        ([{"role": "user", "content": t}] for t in texts[:1])]
        outs[masked] += ie.generate_many([[{"role": "user", "content": t}] for t in texts])
        m.reset_chains()
    assert outs[True] == outs[False]


def test_gpt2_gpu_engine_matches_cpu_reference():
    """GPT-2 (LayerNorm, learned positions, biased QKV without RoPE, GELU MLP, MHA head_dim 64)
    through the native kernels vs the CPU reference with the same bf16 weights."""
    from voice_enabled_browser_automation_amd.models.gpt2 import GPT2Model

    ops.ext()
    torch.manual_seed(0)
    cfg = get_config("gpt2-tiny")
    toks = torch.randint(0, cfg.vocab_size, (140,)).tolist()
    cpu = GPT2Model(cfg, device="cpu", dtype=torch.bfloat16, seed=4)
    ref = _run(cpu, toks, 120)
    gpu = GPT2Model(cfg, device="cpu", dtype=torch.bfloat16, seed=4)
    move_model(gpu, "cuda")
    got = _run(gpu, toks, 120)
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert err < 0.05 * (1 + b.abs().max().item()), (i, err)


def test_llama_fp8_gpu_engine_matches_cpu_emulation():
    """fp8 (W8A8) Llama through the fp8-MFMA decode GEMMs vs the CPU emulation of the same
    quantisation (same quantised weights)."""
    ops.ext()
    torch.manual_seed(0)
    toks = torch.randint(0, CFG.vocab_size, (140,)).tolist()
    cpu = LlamaModel(CFG, device="cpu", seed=5, wdtype="fp8")
    ref = _run(cpu, toks, 120)
    gpu = LlamaModel(CFG, device="cpu", seed=5, wdtype="fp8")
    move_model(gpu, "cuda")
    got = _run(gpu, toks, 120)
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert err < 0.08 * (1 + b.abs().max().item()), (i, err)


@pytest.mark.parametrize("cfg,grid_div", [
    (CFG, 1),
    (LlamaConfig(name="t8", vocab_size=4096, hidden=4096, n_layers=2, n_heads=32, n_kv_heads=8, head_dim=128,
                 ffn=14336, max_pos=2048), 1),
    # one rank of Llama-3-70B at TP=8 (8 q heads, ONE kv head, FFN slice 3584) on 1/8 of the CUs, as
    # when eight ranks share a GPU (tools/tp_check.py)
    (LlamaConfig(name="t70r", vocab_size=4096, hidden=8192, n_layers=2, n_heads=8, n_kv_heads=1, head_dim=128,
                 ffn=3584, max_pos=2048), 8)],
    ids=["small", "llama8b-layers", "llama70b-tp8-rank-griddiv8"])
def test_chained_layer_tail_matches_per_kernel_path(cfg, grid_div, monkeypatch):
    """The chained decode launch (o_proj -> gate/up -> down -> next layer's QKV behind grid
    barriers, skinny_stream.hip chain_kernel) against the per-kernel path on the same weights,
    for 1, 2 and 4 rows (the small config leaves most workgroups without a tile; the 8B-shaped
    one gives them several items per phase)."""
    ops.ext()
    monkeypatch.setenv("VWA_CHAIN_GRID_DIV", str(grid_div))
    torch.manual_seed(0)
    toks = torch.randint(0, cfg.vocab_size, (40,)).tolist()
    model = LlamaModel(cfg, device="cuda", seed=2)

    engines = []  # kept alive: the chain descriptor cache is weakly keyed on each engine's buffers

    def run(chain: bool):
        monkeypatch.setenv("VWA_CHAIN", "1" if chain else "0")
        e = LLMEngine(model, max_seqs=2, max_model_len=256, kv_blocks=20, block_size=16)
        engines.append(e)
        s = e.new_sequence(toks[:30], use_prefix_cache=False)
        e.prefill(s)
        out, i = [], 30
        for n in (1, 2, 4, 1):
            out.append(e.run_rows([(s, t) for t in toks[i:i + n]]).float().cpu().clone())
            i += n
        e.free_sequence(s, publish=False)
        return out

    ref = run(False)
    got = run(True)
    assert not model.chain_error()
    if cfg.head_dim == 128:  # decode attention as the chained launch's first phase
        monkeypatch.setenv("VWA_CHAIN_ATTN", "1")
        model.reset_chains()
        got_a = run(True)
        # 1-row steps there preload gate/up's item 2 into LDS during the attention window
        # (ChainParams::lds_item: the whole 160 KB of LDS)
        assert any(v[2] & 0xFFFFFF == 160 * 1024 for v in model.chain_descs())
        # o_proj in 32-column tiles (ChainParams::o_nt2, one epilogue per workgroup) and in 16
        for sched, bit in (("o_nt2=1", 1), ("o_nt2=0", 0)):
            monkeypatch.setenv("VWA_CHAIN_SCHED", sched)
            model.reset_chains()
            got_o = run(True)
            assert any((v[2] >> 26) & 1 == bit for v in model.chain_descs())
            for a, b in zip(got_o, ref):
                err = (a - b).abs().max().item()
                assert math.isfinite(err) and err < 0.02 * (1 + b.abs().max().item()), (sched, err)
        monkeypatch.delenv("VWA_CHAIN_SCHED")
        monkeypatch.setenv("VWA_CHAIN_ATTN", "0")  # and the separate attention launch
        model.reset_chains()
        got = run(True)
        for a, b in zip(got_a, ref):
            err = (a - b).abs().max().item()
            assert math.isfinite(err) and err < 0.02 * (1 + b.abs().max().item()), err
    assert model.chain_descs() and all(v is not None for v in model.chain_descs())
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("cfg,wdtype", [
    (LlamaConfig(name="t8x4", vocab_size=4096, hidden=4096, n_layers=4, n_heads=32, n_kv_heads=8, head_dim=128,
                 ffn=14336, max_pos=2048), "bf16"),
    (LlamaConfig(name="t8x4", vocab_size=4096, hidden=4096, n_layers=4, n_heads=32, n_kv_heads=8, head_dim=128,
                 ffn=14336, max_pos=2048), "fp8"),
    (LlamaConfig(name="t70x3", vocab_size=4096, hidden=8192, n_layers=3, n_heads=64, n_kv_heads=8, head_dim=128,
                 ffn=28672, max_pos=2048), "bf16")],
    ids=["llama8b-4layers", "llama8b-4layers-fp8", "llama70b-3layers-gqa8"])
def test_multi_layer_chained_launch_matches_per_layer_launches(cfg, wdtype, monkeypatch):
    """All layers in ONE chained launch (skinny_stream.hip chain_kernel MULTI: the QKV phase
    feeds the next layer's attention through an in-launch barrier that only attention workgroups
    wait on) give the SAME bits as one chained launch per layer, and match the per-kernel path,
    over steps of 1, 2, 4 and 1 rows and a second session (contexts that differ per row)."""
    ops.ext()
    torch.manual_seed(0)
    toks = torch.randint(0, cfg.vocab_size, (80,)).tolist()
    model = LlamaModel(cfg, device="cuda", seed=5, wdtype=wdtype)
    engines = []

    def run(chain: bool, multi: bool):
        monkeypatch.setenv("VWA_CHAIN", "1" if chain else "0")
        monkeypatch.setenv("VWA_CHAIN_MULTI", "1" if multi else "0")
        model.reset_chains()
        e = LLMEngine(model, max_seqs=2, max_model_len=512, kv_blocks=40, block_size=16)
        engines.append(e)
        s = e.new_sequence(toks[:40], use_prefix_cache=False)
        s2 = e.new_sequence(toks[5:23], use_prefix_cache=False)
        e.prefill(s)
        e.prefill(s2)
        out, i = [], 40
        for rows in ([(s, toks[40])], [(s, toks[41]), (s2, toks[42])], [(s, t) for t in toks[43:47]],
                     [(s2, toks[47])], [(s, toks[48])]):
            out.append(e.run_rows(rows).float().cpu().clone())
        return out

    ref = run(False, False)
    per_layer = run(True, False)
    got = run(True, True)
    assert not model.chain_error()
    # the multi-layer launch's schedule options (grid barrier by default; per-kv-group QKV counters,
    # the K/V prefetch, the attention-window item of the fp8 chain): the same bits every way
    for sched in ("qkv_flags=1", "qkv_flags=1,kv_pf=1", "kv_pf=1", "attn_pre=0"):
        monkeypatch.setenv("VWA_CHAIN_SCHED", sched)
        other = run(True, True)
        assert not model.chain_error()
        for a, b in zip(other, got):
            assert torch.equal(a, b), (sched, (a - b).abs().max().item())
    monkeypatch.delenv("VWA_CHAIN_SCHED")
    multis = [v for d in model._chains.values() for k, v in d.items() if k[0] == "multi"]
    # (70B shapes at 3-4 rows chain the tail without the attention phase: those steps stay per layer)
    assert any(v is not None and v[3] == cfg.n_layers for v in multis), "no multi-layer launch"
    for a, b in zip(got, per_layer):
        assert torch.equal(a, b), (a - b).abs().max().item()
    # (fp8: the chain is W8A16, the per-kernel path W8A8 -- that equivalence is
    # test_fp8_chained_layer_is_w8a16's; here only the bitwise match above and finiteness)
    tol = 0.03 if wdtype == "bf16" else float("inf")
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert math.isfinite(err) and err < tol * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("grid_div,max_len", [(1, 256), (8, 512)], ids=["full-grid", "griddiv8"])
def test_llama70b_shape_chained_layers_match_f32_reference(grid_div, max_len, monkeypatch):
    """Llama-3-70B layer shapes (hidden 8192, 64 q / 8 kv heads -> GQA 8:1, FFN 28672; BASELINE
    config 4 at TP=1) through the chained decode launch -- decode attention as phase 0 at 1-2
    rows, the tail alone with a separate attention launch at 3-4 rows, where the 28672-wide down
    rows no longer fit LDS next to the attention -- against the CPU f32 reference engine on the
    same bf16 weights (2 layers, small vocab), with rows of one and of two sessions.  griddiv8:
    32 workgroups (eight ranks sharing a GPU), where every workgroup runs an attention item AND
    several o_proj items (the path whose staging wave once computed an unloaded item: NaN)."""
    import copy

    ops.ext()
    monkeypatch.setenv("VWA_CHAIN_GRID_DIV", str(grid_div))
    torch.manual_seed(0)
    cfg = LlamaConfig(name="t70", vocab_size=4096, hidden=8192, n_layers=2, n_heads=64, n_kv_heads=8, head_dim=128,
                      ffn=28672, max_pos=2048)
    toks = torch.randint(0, cfg.vocab_size, (60,)).tolist()
    cpu = LlamaModel(cfg, device="cpu", seed=3)
    gpu = copy.deepcopy(cpu)
    move_model(gpu, "cuda")
    gpu._tile_weights()

    def run(model):
        e = LLMEngine(model, max_seqs=3, max_model_len=max_len, kv_blocks=60, block_size=16)
        s = e.new_sequence(toks[:30], use_prefix_cache=False)
        s2 = e.new_sequence(toks[10:37], use_prefix_cache=False)
        out = [e.prefill(s).float().cpu().clone(), e.prefill(s2).float().cpu().clone()]
        for rows in ([(s, toks[40])], [(s, toks[41]), (s2, toks[42])], [(s, toks[43]), (s, toks[44])],
                     [(s, toks[45]), (s, toks[46]), (s2, toks[47])],
                     [(s, toks[48]), (s, toks[49]), (s2, toks[50]), (s2, toks[51])]):
            out.append(e.run_rows(rows).float().cpu().clone())
        return out, e

    ref, _ = run(cpu)
    got, e = run(gpu)
    assert not gpu.chain_error()
    descs = gpu.chain_descs()
    assert descs and all(v is not None for v in descs), "a 70B-shape step left the chained launch"
    assert any(v[3] == 8 for v in descs), "no step chained the GQA-8 decode attention"
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert math.isfinite(err) and err < 0.03 * (1 + b.abs().max().item()), (i, err)


def test_chain_timeout_falls_back_to_per_kernel_launches():
    """A grid-barrier timeout (error word set by the chained kernel) switches the model to the
    per-kernel path and drops the captured graphs (runtime/engine.py _check_chain)."""
    ops.ext()
    model = LlamaModel(CFG, device="cuda", seed=4)
    e = LLMEngine(model, max_seqs=1, max_model_len=128, kv_blocks=10, block_size=16)
    s = e.new_sequence(list(range(10)), use_prefix_cache=False)
    e.prefill(s)
    a = e.run_rows([(s, 11)]).float().cpu()
    assert model.chain_descs() and not model.chain_error()
    model._chain_bar.view(torch.int64)[160] = 1  # what a timed-out spin writes
    e._check_chain()  # non-blocking: queues the copy of the error word ...
    torch.cuda.synchronize()
    e._check_chain()  # ... and acts on it at the next check
    assert e.stats.get("chain_fallbacks") == 1 and not e.graphs and not model._chain_ok(1)
    b = e.run_rows([(s, 12)]).float().cpu()
    assert torch.isfinite(a).all() and torch.isfinite(b).all()


def test_failed_chained_step_is_rerun_on_per_kernel_path(monkeypatch):
    """A chained step whose barrier timed out is never served: the sampler's fail word turns its
    tokens into -2 and recover_step() re-runs the same rows on the per-kernel path (same logits
    as an engine that never chained, sequence state rolled back and re-advanced)."""
    ops.ext()
    model = LlamaModel(CFG, device="cuda", seed=4)
    toks = list(range(10, 24))

    def engine():
        e = LLMEngine(model, max_seqs=1, max_model_len=128, kv_blocks=10, block_size=16)
        s = e.new_sequence(toks[:10], use_prefix_cache=False)
        e.prefill(s)
        return e, s

    monkeypatch.setenv("VWA_CHAIN", "0")
    e0, s0 = engine()
    ref = [e0.run_rows([(s0, t)]).float().cpu() for t in toks[10:13]]
    monkeypatch.setenv("VWA_CHAIN", "1")
    e, s = engine()
    a = e.run_rows([(s, toks[10])]).float().cpu()  # chained + verified (check=True)
    logits = e.run_rows([(s, toks[11])], check=False)
    word = e.step_fail_word()
    assert word is not None and model.chain_descs()
    word.fill_(1)  # what a timed-out barrier spin writes, after the forward in stream order
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    ops.sample(logits, mask=None, temperature=None, seed=torch.zeros(1, dtype=torch.int64, device="cuda"),
               step=torch.zeros(1, dtype=torch.int32, device="cuda"), out_tokens=out, fail_word=word)
    assert out[:1].tolist() == [-2]
    b = e.recover_step().float().cpu()
    assert e.stats["chain_fallbacks"] == 1 and not model._chain_ok(1) and not model.chain_error()
    assert s.n_computed == 12
    c = e.run_rows([(s, toks[12])]).float().cpu()
    for got, want in zip((a, b, c), ref):
        err = (got - want).abs().max().item()
        assert err < 0.02 * (1 + want.abs().max().item()), err


def test_asr_device_decode_loop_matches_host_loop():
    """The device-resident greedy loop (sampled token fed back on the GPU, decode_advance kernel,
    step graphs replayed back to back) produces the same tokens as the host-driven loop, in the
    fixed-work and the stop-at-EOT modes."""
    ops.ext()
    tok = load_tokenizer("whisper")
    m = WhisperModel(get_config("whisper-test"), device="cuda", seed=3)
    a = AsrEngine(m, tok, max_sessions=2)
    pcm = (np.sin(np.arange(16000 * 2) * 2 * np.pi * 250 / 16000) * 6000).astype(np.int16)
    audio = a.pcm_to_audio(pcm)
    for kw in (dict(exact_tokens=12), dict(max_tokens=20)):
        a.device_loop = False
        host = a.transcribe(audio, **kw)
        n_host = a.last_stats["tokens"]
        a.device_loop = True
        dev = a.transcribe(audio, **kw)
        assert dev == host and a.last_stats["tokens"] == n_host, (kw, host, dev)
    assert a.loop_graphs


def test_prefix_cached_prefill_decode_attention_slices(monkeypatch):
    """A prompt suffix behind a cached prefix runs its attention through the decode kernel in
    <= 64-row slices; logits match the flash-attention path."""
    ops.ext()
    torch.manual_seed(0)
    toks = torch.randint(0, CFG.vocab_size, (300,)).tolist()
    model = LlamaModel(CFG, device="cuda", seed=6)

    def run(flag: str):
        monkeypatch.setenv("VWA_PREFILL_DECODE_ATTN", flag)
        e = LLMEngine(model, max_seqs=2, max_model_len=512, kv_blocks=60, block_size=16)
        head = e.new_sequence(toks[:208])
        e.prefill(head)
        e.free_sequence(head)  # publishes the 208-token prefix
        s = e.new_sequence(toks)  # 13 cached blocks, 92-token suffix with q_offset 208
        assert s.n_computed == 208
        return e.prefill(s).float().cpu()

    a, b = run("1"), run("0")
    err = (a - b).abs().max().item()
    assert err < 0.02 * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("name", ["whisper-test", "whisper-tiny", "whisper-large-v3"])
def test_whisper_chained_decoder_matches_per_kernel_path(name, monkeypatch):
    """The chained Whisper decoder launches (out-proj -> LN cross query; out-proj -> LN fc1 GELU
    -> fc2 -> next layer's LN QKV + self-KV write, skinny_stream.hip chain_kernel SEQ 2 / 1)
    against the per-kernel path on the same weights and caches, for 1, 2 and 4 rows over a few
    positions (large-v3: its layer shapes, 3 decoder layers)."""
    from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner

    ops.ext()
    cfg = get_config(name)
    if name == "whisper-large-v3":
        import dataclasses

        cfg = dataclasses.replace(cfg, n_enc_layers=1, n_dec_layers=3)
    m = WhisperModel(cfg, device="cuda", seed=7)
    torch.manual_seed(1)
    enc = torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16)

    runners = []  # kept alive: the chain descriptor cache is weakly keyed on each runner's buffers

    def run(chain: bool):
        monkeypatch.setenv("VWA_CHAIN_ASR", "1" if chain else "0")
        r = WhisperRunner(m, max_sessions=2, use_graphs=False)
        runners.append(r)
        r.set_cross(0, enc)
        r.set_cross(1, enc)
        out, pos = [], 0
        for n in (1, 2, 4, 1, 4):
            rows = [(i % 2, (7 * pos + 3 * i) % 1000, pos + i // 2) for i in range(n)]
            out.append(r.step(rows).float().cpu().clone())
            pos += 2
        return out

    ref = run(False)
    got = run(True)
    assert not m.chain_error()
    assert m.chain_descs() and all(a is not None and b is not None for a, b in m.chain_descs())
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("graphs,model", [(False, "whisper-large-v3"), (True, "whisper-large-v3"),
                                          (True, "whisper-tiny")])
def test_whisper_persistent_decoder_matches_per_kernel_path(graphs, model, monkeypatch):
    """The persistent whisper-large decoder step (whisper_dec.hip: every layer in ONE launch,
    weights a layer ahead in registers, counter hand-offs) against the per-kernel path on the same
    weights, caches and cross K/V: one row per step, two sessions, contexts up to 70 keys (several
    KV blocks), 4 decoder layers; replayed from a hipGraph too."""
    import dataclasses

    from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner

    ops.ext()
    cfg = dataclasses.replace(get_config(model), n_enc_layers=1, n_dec_layers=4)
    m = WhisperModel(cfg, device="cuda", seed=3)
    assert m.dec_tiled == (model == "whisper-large-v3")  # (tiny: the kernel gets tiled copies)
    torch.manual_seed(4)
    enc = [torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16) for _ in range(2)]
    runners = []

    def run(persist: bool):
        monkeypatch.setenv("VWA_ASR_PERSIST", "1" if persist else "0")
        r = WhisperRunner(m, max_sessions=2, use_graphs=graphs)
        runners.append(r)
        r.set_cross(0, enc[0])
        r.set_cross(1, enc[1])
        out = []
        for p in range(70):
            for s in (0, 1):
                lg = r.step([(s, (13 * p + 5 * s) % 1000, p)])
                if p % 9 == 0 or p == 69:
                    out.append(lg.float().cpu().clone())
        return out

    ref = run(False)
    got = run(True)
    assert m._wdec and not m.chain_error()
    for i, (a, b) in enumerate(zip(got, ref)):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), (i, err)


@pytest.mark.parametrize("model", ["whisper-large-v3", "whisper-tiny"])
def test_whisper_persistent_device_loop_is_one_launch_and_matches(model, monkeypatch):
    """The device-resident greedy loop (asr/engine.py) with the persistent decoder: each step is ONE
    launch (embedding from the tables, every layer, LM head, masked argmax, advance) and gives the
    per-kernel loop's tokens; 4 decoder layers, two utterances decoded back to back."""
    import dataclasses

    from voice_enabled_browser_automation_amd.asr.engine import AsrEngine
    from voice_enabled_browser_automation_amd.tokenizer import load_tokenizer

    ops.ext()
    cfg = dataclasses.replace(get_config(model), n_enc_layers=1, n_dec_layers=4)
    m = WhisperModel(cfg, device="cuda", seed=11)
    torch.manual_seed(12)
    audios = [torch.randn(16000 * 3, device="cuda") * 0.1 for _ in range(2)]
    outs = {}
    for persist in ("0", "1"):
        monkeypatch.setenv("VWA_ASR_PERSIST", persist)
        eng = AsrEngine(m, load_tokenizer("whisper"), max_sessions=2)
        outs[persist] = [eng.decode_many([a], exact_tokens=24)[0] for a in audios]
        if persist == "1":
            assert m._wdec and not m.chain_error()
            # the loop graph of one step holds a single kernel launch
            st = next(iter(m._wdec.values()))
            assert "smp_part" in st
    assert outs["1"] == outs["0"], (outs["0"], outs["1"])


def test_wdec_counters_survive_launch_sequences(monkeypatch):
    """Counter bases across many launches of the persistent decoder (monotonic counters, no reset):
    200 steps in a row keep matching the per-kernel path at the end."""
    import dataclasses

    from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner

    ops.ext()
    cfg = dataclasses.replace(get_config("whisper-large-v3"), n_enc_layers=1, n_dec_layers=2)
    m = WhisperModel(cfg, device="cuda", seed=8)
    torch.manual_seed(5)
    enc = torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16)
    runners = []

    def run(persist: bool):
        monkeypatch.setenv("VWA_ASR_PERSIST", "1" if persist else "0")
        r = WhisperRunner(m, max_sessions=1, use_graphs=True)
        runners.append(r)
        r.set_cross(0, enc)
        for _ in range(50):  # the same position again and again: 200 launches
            for p in range(4):
                lg = r.step([(0, (7 * p) % 1000, p)])
        return lg.float().cpu().clone()

    ref = run(False)
    got = run(True)
    assert not m.chain_error()
    err = (got - ref).abs().max().item()
    assert err < 0.02 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("chain", [False, True])
def test_whisper_tiled_decoder_matches_row_major(chain, monkeypatch):
    """Decode-step weights in the pre-tiled layout (large models: WhisperModel._tile_decoder; the
    streaming kernel with the 4-wave K split at K = 1280) give the logits of the row-major
    decoder on the same weights -- per-kernel path and chained launches."""
    import dataclasses

    from voice_enabled_browser_automation_amd.asr.engine import WhisperRunner

    ops.ext()
    cfg = dataclasses.replace(get_config("whisper-large-v3"), n_enc_layers=1, n_dec_layers=2)
    m_rm = WhisperModel(cfg, device="cuda", seed=5, tile_decoder=False)
    m_t = WhisperModel(cfg, device="cuda", seed=5, tile_decoder=True)
    assert m_t.dec_tiled and not m_rm.dec_tiled and isinstance(m_t.dec[0].fc2, ops.TiledWeight)
    torch.manual_seed(2)
    enc = torch.randn(1, cfg.n_audio_ctx, cfg.d_model, device="cuda").to(torch.bfloat16)
    runners = []

    def run(m, ch):
        monkeypatch.setenv("VWA_CHAIN_ASR", "1" if ch else "0")
        r = WhisperRunner(m, max_sessions=1, use_graphs=False)
        runners.append(r)
        r.set_cross(0, enc)
        return [r.step([(0, (11 * p) % 1000, p)]).float().cpu().clone() for p in range(4)]

    ref = run(m_rm, False)
    got = run(m_t, chain)
    assert not m_t.chain_error()
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


def test_chain_is_rearmed_after_backoff(monkeypatch):
    """After a fallback the engine re-arms the chained launch (fresh barrier counters) once the
    backoff has passed; the re-armed chained steps match an engine that never chained."""
    ops.ext()
    model = LlamaModel(CFG, device="cuda", seed=4)
    toks = list(range(30, 46))

    def engine():
        e = LLMEngine(model, max_seqs=1, max_model_len=128, kv_blocks=10, block_size=16)
        s = e.new_sequence(toks[:10], use_prefix_cache=False)
        e.prefill(s)
        return e, s

    monkeypatch.setenv("VWA_CHAIN", "0")
    e0, s0 = engine()
    ref = [e0.run_rows([(s0, t)]).float().cpu() for t in toks[10:14]]
    monkeypatch.setenv("VWA_CHAIN", "1")
    e, s = engine()
    got = [e.run_rows([(s, toks[10])]).float().cpu()]
    model._chain_bar.view(torch.int64)[160] = 1  # a timed-out spin (left partial arrivals too)
    model._chain_bar.view(torch.int64)[16] += 3
    e._check_chain(blocking=True)
    assert e.stats["chain_fallbacks"] == 1 and not model._chain_ok(1)
    assert e._chain_retry_at == e.stats["steps"] + 256
    got.append(e.run_rows([(s, toks[11])]).float().cpu())  # per-kernel path
    e._chain_retry_at = e.stats["steps"]  # backoff elapsed
    got += [e.run_rows([(s, t)]).float().cpu() for t in toks[12:14]]
    assert e.stats["chain_rearms"] == 1 and model._chain_ok(1) and model.chain_descs()
    assert not model.chain_error()
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("sched", ["", "d_nt2=1", "d_nt2=0"])
def test_chained_layer_tail_5_to_16_rows(sched, monkeypatch):
    """Steps of 5..16 rows on the chained launch (VWA_CHAIN_MAX_ROWS): no attention phase, the
    down projection streaming its X fragments with the weights (its 14336-wide rows do not fit LDS
    above 5 rows: ChainPhase::xg), in 16- and 32-column tiles (ChainParams::d_nt2) -- against the
    per-kernel path on 8B-shaped layers."""
    ops.ext()
    if sched:
        monkeypatch.setenv("VWA_CHAIN_SCHED", sched)
    cfg = LlamaConfig(name="t8x", vocab_size=4096, hidden=4096, n_layers=2, n_heads=32, n_kv_heads=8, head_dim=128,
                      ffn=14336, max_pos=2048)
    torch.manual_seed(1)
    toks = torch.randint(0, cfg.vocab_size, (80,)).tolist()
    model = LlamaModel(cfg, device="cuda", seed=5)
    engines = []

    def run(chain: bool):
        monkeypatch.setenv("VWA_CHAIN", "1" if chain else "0")
        e = LLMEngine(model, max_seqs=2, max_model_len=256, kv_blocks=20, block_size=16)
        engines.append(e)
        s = e.new_sequence(toks[:30], use_prefix_cache=False)
        e.prefill(s)
        out, i = [], 30
        for n in (5, 8, 16, 3, 1):
            out.append(e.run_rows([(s, t) for t in toks[i:i + n]]).float().cpu().clone())
            i += n
        e.free_sequence(s, publish=False)
        return out

    monkeypatch.setenv("VWA_CHAIN_MAX_ROWS", "16")
    ref = run(False)
    got = run(True)
    assert not model.chain_error()
    descs = [v for v in model.chain_descs() if v is not None]
    assert any((v[2] >> 24) & 1 for v in descs), "no descriptor streams X with the weights"
    if sched:
        assert any((v[2] >> 27) & 1 for v in descs) == (sched == "d_nt2=1")
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


def test_intent_engine_recovers_from_a_failed_chained_step(monkeypatch):
    """LLMIntentEngine.step's own recovery path: the forward's chained launch "times
    out" (its error word set in stream order after the forward) -> the zero-copy sampler stores
    -2 tokens -> recover_step re-runs the rows on the per-kernel path and the same iteration
    samples again: the answers are schema-valid and reproducible, one fallback is counted."""
    from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine

    ops.ext()
    cfg = LlamaConfig(name="t8r", vocab_size=128256, hidden=1024, n_layers=2, n_heads=8, n_kv_heads=2,
                      head_dim=128, ffn=2048, max_pos=4096)
    model = LlamaModel(cfg, device="cuda", seed=6)
    texts = ["search wireless earbuds", "scroll down"]

    def answers(chain: bool, fail_at: int = -1):
        monkeypatch.setenv("VWA_CHAIN", "1" if chain else "0")
        model.enable_chain()
        eng = LLMEngine(model, max_seqs=2, max_model_len=2048)
        ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=160, temperature=0.1, seed=3)
        assert ie.zero_copy and ie.spin_wait
        calls = [0, False]
        orig = eng.run_rows

        def run_rows(*a, **k):
            out = orig(*a, **k)
            calls[0] += 1
            # the first chained (<= 4-row) sampled step from the fail_at-th call on
            if fail_at > 0 and calls[0] >= fail_at and not calls[1] and k.get("check") is False:
                w = eng.step_fail_word()
                if w is not None:
                    w.fill_(1)  # what a timed-out barrier spin writes (stream-ordered after the forward)
                    calls[1] = True
            return out

        eng.run_rows = run_rows
        outs = [ie.generate([{"role": "user", "content": t}]) for t in texts]
        assert fail_at < 0 or calls[1], "no chained step was failed"
        return outs, eng

    from voice_enabled_browser_automation_amd.contracts import ParseResponse, safe_parse

    # (the chained and per-kernel paths round differently, so a recovered run is compared with an
    # identically injected one -- recovery must be deterministic -- and checked for validity)
    got, eng = answers(True, fail_at=6)
    assert eng.stats.get("chain_fallbacks") == 1
    again, eng2 = answers(True, fail_at=6)
    assert eng2.stats.get("chain_fallbacks") == 1
    assert got == again
    import json as _json

    assert all(safe_parse(ParseResponse, _json.loads(o)).success for o in got)
    model.enable_chain()


@pytest.mark.parametrize("cfg", [CFG, LlamaConfig(name="t8f", vocab_size=4096, hidden=4096, n_layers=2, n_heads=32,
                                                  n_kv_heads=8, head_dim=128, ffn=14336, max_pos=2048)],
                         ids=["small", "llama8b-layers"])
def test_fp8_chained_layer_is_w8a16(cfg, monkeypatch):
    """fp8 tiled weights through the chained decode launch (skinny_stream.hip chain_kernel F8:
    e4m3 items converted to bf16 in registers, per-row scales in the epilogues) == a bf16 model
    holding the dequantised weights on the per-kernel path (W8A16 semantics), 1 / 2 / 4 rows."""
    ops.ext()
    torch.manual_seed(0)
    toks = torch.randint(0, cfg.vocab_size, (40,)).tolist()
    m8 = LlamaModel(cfg, device="cuda", seed=3, wdtype="fp8")
    assert isinstance(m8.layers[0].o, ops.FP8Weight) and m8.layers[0].o.tiled
    mb = LlamaModel(cfg, device="cuda", seed=3)
    deq = lambda w: ops.TiledWeight(w.dequant(torch.bfloat16))  # noqa: E731
    for Lb, L8 in zip(mb.layers, m8.layers):
        Lb.qkv, Lb.o, Lb.gu, Lb.down = deq(L8.qkv), deq(L8.o), deq(L8.gu), deq(L8.down)
    # layer 0's QKV runs before the chained launch (the W8A8 skinny kernel on both sides)
    mb.layers[0].qkv = m8.layers[0].qkv
    engines = []

    def run(model, chain):
        monkeypatch.setenv("VWA_CHAIN", "1" if chain else "0")
        e = LLMEngine(model, max_seqs=2, max_model_len=256, kv_blocks=20, block_size=16)
        engines.append(e)
        s = e.new_sequence(toks[:1], use_prefix_cache=False)
        e.prefill(s)
        for t in toks[1:30]:  # one-row steps: the whole cache under the same (W8A16) semantics
            e.run_rows([(s, t)], defer_head=True)
        out, i = [], 30
        for n in (1, 2, 4, 1):
            # the final hidden rows (the fp8 LM head's activation quantisation would turn tiny
            # rounding differences into whole e4m3 steps)
            e.run_rows([(s, t) for t in toks[i:i + n]], defer_head=True)
            out.append(e._head_rows.float().cpu().clone())
            i += n
        return out

    ref = run(mb, False)
    got = run(m8, True)
    assert m8.chain_descs() and all(v is not None for v in m8.chain_descs()), "fp8 chain not built"
    assert not m8.chain_error()
    for a, b in zip(got, ref):
        err = (a - b).abs().max().item()
        assert err < 0.02 * (1 + b.abs().max().item()), err


@pytest.mark.parametrize("flash", ["1", "0"])
def test_batched_admission_prefill_gpu(flash, monkeypatch):
    """GPU batched admission prefill (runtime/engine.py prefill_batch, > 64 ragged rows): the
    per-request runs' causal attention as ONE batched flash launch per layer (VWA_PREFILL_FLASH=1,
    the default) or the decode kernel over 64-row slices -- the same K/V, hence the same next-token
    logits, as one prefill per request."""
    import voice_enabled_browser_automation_amd.runtime.engine as eng_mod

    monkeypatch.setattr(eng_mod, "PREFILL_FLASH", flash == "1")
    torch.manual_seed(0)
    m = LlamaModel(CFG, device="cuda", seed=3)
    head = torch.randint(0, 4096, (200,)).tolist()
    tails = [torch.randint(0, 4096, (n,)).tolist() for n in (40, 33, 27, 85, 60)]

    def make():
        e = LLMEngine(m, max_seqs=6, max_model_len=512, kv_blocks=200, block_size=16)
        s0 = e.new_sequence(head)
        e.prefill(s0)
        e.free_sequence(s0)
        return e, [e.new_sequence(head + t) for t in tails]

    def next_logits(e, seqs):
        return [e.run_rows([(s, 7)]).float().clone() for s in seqs]

    eA, sA = make()
    for s in sA:
        eA.prefill(s)
    want = next_logits(eA, sA)
    eB, sB = make()
    calls = []
    orig = ops.flash_attention_runs
    monkeypatch.setattr(ops, "flash_attention_runs", lambda *a, **k: calls.append(1) or orig(*a, **k))
    eB.prefill_batch([(s, len(s.tokens)) for s in sB])  # 245 suffix rows behind the cached head
    assert bool(calls) == (flash == "1")
    got = next_logits(eB, sB)
    for a, b in zip(got, want):
        assert torch.isfinite(a).all()
        assert torch.allclose(a, b, atol=3e-2, rtol=3e-2), (a - b).abs().max()


def test_intent_parses_and_transcripts_are_reproducible():
    """Same weights, inputs and sampler seed -> the same bits from two fresh engines: the
    many-row RMS statistics add as integers (GemmParams::ss_*), every split reduction sums in a
    fixed order, and the flash-attention form whose results moved by an ulp from run to run is
    gone (tools/repro_check.py / repro_ops.py found both)."""
    from voice_enabled_browser_automation_amd.brain.intent_engine import LLMIntentEngine
    from voice_enabled_browser_automation_amd.models.config import LLAMA_PRESETS

    ops.ext()
    m = LlamaModel(LLAMA_PRESETS["llama-tiny"], device="cuda", seed=4)
    texts = ["search wireless earbuds on the first page of results", "scroll down", "sort by price", "go back"]
    outs = []
    for _ in range(2):
        eng = LLMEngine(m, max_seqs=4, max_model_len=2048)
        eng.capture_all()
        ie = LLMIntentEngine(eng, load_tokenizer("llama3"), budget_chars=200, temperature=0.1, seed=7)
        outs.append(ie.parse_many([{"text": t, "context": {}} for t in texts]))
        m.reset_chains()
    assert outs[0] == outs[1]
    w = WhisperModel(get_config("whisper-tiny"), device="cuda", seed=1)
    asr = AsrEngine(w, load_tokenizer("whisper"), max_sessions=2)
    g = torch.Generator().manual_seed(3)
    audio = (torch.randn(16000 * 5, generator=g) * 0.1).to("cuda")
    mel = w.mel_batch([audio])
    enc = [w.encode(mel).clone() for _ in range(3)]
    assert all(torch.equal(enc[0], e) for e in enc[1:])
    toks = [asr.decode_many([audio], exact_tokens=24)[0] for _ in range(2)]
    assert toks[0] == toks[1]
