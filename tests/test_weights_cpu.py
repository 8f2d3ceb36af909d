"""Checkpoint loading (safetensors, HF names) against independent plain-PyTorch implementations of
the public architectures: proves the on-load fusions (QKV row permutation for the RoPE epilogue,
norm-gamma folding, gate/up interleave, GPT-2 Conv1D transposes) preserve the math."""
import math

import torch
from safetensors.torch import save_file

from voice_enabled_browser_automation_amd.models.config import GPT2Config, LlamaConfig, get_config
from voice_enabled_browser_automation_amd.models.whisper import WhisperModel
from voice_enabled_browser_automation_amd.runtime.engine import LLMEngine
from voice_enabled_browser_automation_amd.runtime.weights import LazySafetensors, load_llm

LCFG = LlamaConfig(name="t", vocab_size=300, hidden=128, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=32,
                   ffn=256, max_pos=256, rope_theta=10000.0)


def _engine_logits(model, toks):
    e = LLMEngine(model, max_seqs=1, max_model_len=128, kv_blocks=16, block_size=16)
    s = e.new_sequence(toks, use_prefix_cache=False)
    return e.run_rows([(s, t) for t in toks]).float().clone()


def _llama_hf(cfg, gen):
    r = lambda *s: torch.randn(*s, generator=gen) * 0.05  # noqa: E731
    d, hd = cfg.hidden, cfg.head_dim
    w = {"model.embed_tokens.weight": r(cfg.vocab_size, d), "model.norm.weight": 1 + r(d),
         "lm_head.weight": r(cfg.vocab_size, d)}
    for i in range(cfg.n_layers):
        p = f"model.layers.{i}."
        w.update({p + "self_attn.q_proj.weight": r(cfg.n_heads * hd, d),
                  p + "self_attn.k_proj.weight": r(cfg.n_kv_heads * hd, d),
                  p + "self_attn.v_proj.weight": r(cfg.n_kv_heads * hd, d),
                  p + "self_attn.o_proj.weight": r(d, cfg.n_heads * hd),
                  p + "mlp.gate_proj.weight": r(cfg.ffn, d), p + "mlp.up_proj.weight": r(cfg.ffn, d),
                  p + "mlp.down_proj.weight": r(d, cfg.ffn), p + "input_layernorm.weight": 1 + r(d),
                  p + "post_attention_layernorm.weight": 1 + r(d)})
    return w


def _llama_reference(cfg, w, toks):
    """HF LlamaForCausalLM semantics (rotate-half RoPE, RMSNorm, SwiGLU, GQA), f32."""
    f = {k: v.float() for k, v in w.items()}
    T, hd = len(toks), cfg.head_dim
    x = f["model.embed_tokens.weight"][toks]
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd, 2).float() / hd))
    ang = torch.arange(T).float()[:, None] * inv[None]
    cos, sin = torch.cat([ang.cos()] * 2, -1), torch.cat([ang.sin()] * 2, -1)

    def rms(v, g):
        return v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + cfg.rms_eps) * g

    def rope(t):
        rot = torch.cat([-t[..., hd // 2:], t[..., : hd // 2]], -1)
        return t * cos[:, None] + rot * sin[:, None]

    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(cfg.n_layers):
        p = f"model.layers.{i}."
        h = rms(x, f[p + "input_layernorm.weight"])
        q = rope((h @ f[p + "self_attn.q_proj.weight"].t()).view(T, cfg.n_heads, hd))
        k = rope((h @ f[p + "self_attn.k_proj.weight"].t()).view(T, cfg.n_kv_heads, hd))
        v = (h @ f[p + "self_attn.v_proj.weight"].t()).view(T, cfg.n_kv_heads, hd)
        rep = cfg.n_heads // cfg.n_kv_heads
        k, v = k.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
        att = torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(hd) + mask
        o = torch.einsum("hqk,khd->qhd", att.softmax(-1), v).reshape(T, -1)
        x = x + o @ f[p + "self_attn.o_proj.weight"].t()
        h = rms(x, f[p + "post_attention_layernorm.weight"])
        g = torch.nn.functional.silu(h @ f[p + "mlp.gate_proj.weight"].t()) * (h @ f[p + "mlp.up_proj.weight"].t())
        x = x + g @ f[p + "mlp.down_proj.weight"].t()
    return rms(x, f["model.norm.weight"]) @ f["lm_head.weight"].t()


def test_llama_safetensors_load_matches_hf_semantics(tmp_path, monkeypatch):
    from voice_enabled_browser_automation_amd.models import config

    monkeypatch.setitem(config.LLAMA_PRESETS, "llama-ckpt-test", LCFG)
    w = _llama_hf(LCFG, torch.Generator().manual_seed(0))
    save_file({k: v.to(torch.bfloat16).contiguous() for k, v in w.items()}, str(tmp_path / "model.safetensors"))
    lazy = LazySafetensors(str(tmp_path))
    assert "lm_head.weight" in lazy and len(lazy) == len(w)
    m = load_llm("llama-ckpt-test", device="cpu", weights_path=str(tmp_path))
    toks = [5, 17, 250, 3, 99, 42, 7, 128]
    got = _engine_logits(m, toks)
    exp = _llama_reference(LCFG, {k: v.to(torch.bfloat16) for k, v in w.items()}, toks)
    assert (got - exp).abs().max() < 0.03 * (1 + exp.abs().max()), (got - exp).abs().max()


def test_gpt2_safetensors_load_matches_hf_semantics(tmp_path, monkeypatch):
    from voice_enabled_browser_automation_amd.models import config

    cfg = GPT2Config(name="gpt2-ckpt-test", vocab_size=300, hidden=64, n_layers=2, n_heads=2, ffn=256, max_pos=64)
    monkeypatch.setitem(config.GPT2_PRESETS, "gpt2-ckpt-test", cfg)
    gen = torch.Generator().manual_seed(1)
    r = lambda *s: torch.randn(*s, generator=gen) * 0.05  # noqa: E731
    d = cfg.hidden
    w = {"wte.weight": r(cfg.vocab_size, d), "wpe.weight": r(32, d), "ln_f.weight": 1 + r(d), "ln_f.bias": r(d)}
    for i in range(cfg.n_layers):
        p = f"h.{i}."
        w.update({p + "ln_1.weight": 1 + r(d), p + "ln_1.bias": r(d), p + "attn.c_attn.weight": r(d, 3 * d),
                  p + "attn.c_attn.bias": r(3 * d), p + "attn.c_proj.weight": r(d, d), p + "attn.c_proj.bias": r(d),
                  p + "ln_2.weight": 1 + r(d), p + "ln_2.bias": r(d), p + "mlp.c_fc.weight": r(d, cfg.ffn),
                  p + "mlp.c_fc.bias": r(cfg.ffn), p + "mlp.c_proj.weight": r(cfg.ffn, d), p + "mlp.c_proj.bias": r(d)})
    save_file({k: v.contiguous() for k, v in w.items()}, str(tmp_path / "model.safetensors"))
    m = load_llm("gpt2-ckpt-test", device="cpu", weights_path=str(tmp_path))
    toks = [1, 50, 299, 7, 8, 100]
    got = _engine_logits(m, toks)
    # HF GPT2LMHeadModel semantics (Conv1D: y = x @ W + b), erf GELU as in this implementation
    T, H, hd = len(toks), cfg.n_heads, d // cfg.n_heads
    ln = torch.nn.functional.layer_norm
    x = w["wte.weight"][toks] + w["wpe.weight"][:T]
    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(cfg.n_layers):
        p = f"h.{i}."
        h = ln(x, (d,), w[p + "ln_1.weight"], w[p + "ln_1.bias"], cfg.ln_eps)
        q, k, v = (h @ w[p + "attn.c_attn.weight"] + w[p + "attn.c_attn.bias"]).view(T, 3, H, hd).unbind(1)
        att = (torch.einsum("qhd,khd->hqk", q, k) / math.sqrt(hd) + mask).softmax(-1)
        x = x + torch.einsum("hqk,khd->qhd", att, v).reshape(T, d) @ w[p + "attn.c_proj.weight"] + w[p + "attn.c_proj.bias"]
        h = ln(x, (d,), w[p + "ln_2.weight"], w[p + "ln_2.bias"], cfg.ln_eps)
        h = torch.nn.functional.gelu(h @ w[p + "mlp.c_fc.weight"] + w[p + "mlp.c_fc.bias"])
        x = x + h @ w[p + "mlp.c_proj.weight"] + w[p + "mlp.c_proj.bias"]
    exp = ln(x, (d,), w["ln_f.weight"], w["ln_f.bias"], cfg.ln_eps) @ w["wte.weight"].t()
    assert (got - exp).abs().max() < 1e-3 * (1 + exp.abs().max()), (got - exp).abs().max()


def test_whisper_safetensors_load(tmp_path):
    cfg = get_config("whisper-test")
    ref = WhisperModel(cfg, device="cpu", seed=0)
    d, nm = cfg.d_model, cfg.n_mels
    gen = torch.Generator().manual_seed(2)
    r = lambda *s: (torch.randn(*s, generator=gen) * 0.05).to(torch.bfloat16)  # noqa: E731
    e, dd = "model.encoder.", "model.decoder."
    w = {e + "conv1.weight": r(d, nm, 3), e + "conv1.bias": r(d), e + "conv2.weight": r(d, d, 3), e + "conv2.bias": r(d),
         e + "layer_norm.weight": r(d), e + "layer_norm.bias": r(d), dd + "embed_tokens.weight": r(cfg.vocab_size, d),
         dd + "embed_positions.weight": r(cfg.n_text_ctx, d), dd + "layer_norm.weight": r(d),
         dd + "layer_norm.bias": r(d)}

    def attn(p):
        return {p + "q_proj.weight": r(d, d), p + "q_proj.bias": r(d), p + "k_proj.weight": r(d, d),
                p + "v_proj.weight": r(d, d), p + "v_proj.bias": r(d), p + "out_proj.weight": r(d, d),
                p + "out_proj.bias": r(d)}

    def mlp_norms(p, names):
        out = {p + "fc1.weight": r(cfg.ffn, d), p + "fc1.bias": r(cfg.ffn), p + "fc2.weight": r(d, cfg.ffn),
               p + "fc2.bias": r(d)}
        for n in names:
            out[p + n + ".weight"], out[p + n + ".bias"] = r(d), r(d)
        return out

    for i in range(cfg.n_enc_layers):
        p = f"{e}layers.{i}."
        w.update(attn(p + "self_attn."))
        w.update(mlp_norms(p, ["self_attn_layer_norm", "final_layer_norm"]))
    for i in range(cfg.n_dec_layers):
        p = f"{dd}layers.{i}."
        w.update(attn(p + "self_attn."))
        w.update(attn(p + "encoder_attn."))
        w.update(mlp_norms(p, ["self_attn_layer_norm", "encoder_attn_layer_norm", "final_layer_norm"]))
    save_file(w, str(tmp_path / "model.safetensors"))
    m = WhisperModel(cfg, device="cpu", weights=LazySafetensors(str(tmp_path / "model.safetensors")))
    assert torch.equal(m.conv1_w, w[e + "conv1.weight"].permute(0, 2, 1).reshape(d, -1))
    assert torch.equal(m.dec[1].xv_b, w[f"{dd}layers.1.encoder_attn.v_proj.bias"])
    assert torch.equal(m.lm_head[: cfg.vocab_size], w[dd + "embed_tokens.weight"])
    mel = ref.log_mel(torch.zeros(16000))
    enc = m.encode(mel[None])
    assert enc.shape == (1, cfg.n_audio_ctx, d) and torch.isfinite(enc.float()).all()


def test_tiled_weight_layout_and_cpu_routing():
    """ops.tile_weight: the 4 KB block of (16-row tile T, 128-wide k-group kg) holds, at [s][lane][e],
    W[16 T + lane % 16][128 kg + 32 (lane // 16) + 8 s + e] (the MFMA B fragments in wave-load
    order, vwa_kernels.h SkinnyParams::w_tiled); untile_weight inverts it; CPU ops on a TiledWeight
    use its row-major copy."""
    from voice_enabled_browser_automation_amd import ops
    from voice_enabled_browser_automation_amd.ops import reference as ref

    torch.manual_seed(0)
    w = torch.randn(48, 384).to(torch.bfloat16)
    t = ops.tile_weight(w)
    assert t.shape == w.shape and torch.equal(ops.untile_weight(t), w)
    blk = t.reshape(-1).view(48 // 16, 384 // 128, 4, 64, 8)
    for T, kg, s, lane, e in [(0, 0, 0, 0, 0), (2, 1, 3, 63, 7), (1, 2, 2, 17, 4)]:
        assert blk[T, kg, s, lane, e] == w[16 * T + lane % 16, 128 * kg + 32 * (lane // 16) + 8 * s + e]
    tw = ops.TiledWeight(w)
    x = torch.randn(3, 384).to(torch.bfloat16)
    out = ops.linear(x, tw, fuse_rms=True)
    exp = torch.empty(3, 48, dtype=torch.bfloat16)
    ref.linear(x, w, None, out=exp, fuse_rms=True)
    assert torch.equal(out, exp)
    assert tw.numel() == w.numel() and tw.shape == w.shape
