"""Numerics of every gfx950 HIP kernel vs the plain-PyTorch f32 reference (ops/reference.py).

All tests run the native kernel path (ops.ext() must load: no fallback) on cuda:0.
"""
import math

import pytest
import torch

import voice_enabled_browser_automation_amd.ops as ops
from voice_enabled_browser_automation_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


@pytest.fixture(scope="module", autouse=True)
def _native():
    ops.ext()  # fail loudly if the extension is missing
    torch.manual_seed(0)


def rnd(*shape, scale=1.0, dtype=BF):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


def close(a, b, atol, rtol=2e-2):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > tol {tol}"


@pytest.fixture(params=[(0, 256, 8), (1, 256, 8, 0), (1, 768, 4), (1, 256, 8, 2)],
                ids=["tile", "stream8_xfirst", "stream4", "stream8"])
def skinny_mode(request):
    ops.ext().set_skinny_mode(*request.param)
    ops.ext().set_small_gemm_bytes(0)  # every shape on the selected kernel (no small-weight routing)
    yield request.param
    ops.ext().set_skinny_mode(1, 256, 0, 2)
    ops.ext().set_small_gemm_bytes(4 << 20)


@pytest.mark.parametrize("M", [1, 5, 17, 40])
@pytest.mark.parametrize("fuse_rms", [False, True])
def test_skinny_store_resid_gelu(M, fuse_rms, skinny_mode):
    K, N = 1024, 384
    x = rnd(M, K)
    w = rnd(N, K, scale=0.05)
    b = rnd(N, scale=0.1)
    for act, res in (("none", None), ("none", rnd(M, N)), ("gelu", None)):
        out = torch.empty(M, N, dtype=BF, device=DEV)
        ops.linear(x, w, b, out=out, residual=res, act=act, fuse_rms=fuse_rms, eps=1e-5)
        exp = torch.empty(M, N, dtype=BF)
        ref.linear(x.cpu(), w.cpu(), b.cpu(), out=exp, residual=None if res is None else res.cpu(), act=act,
                   fuse_rms=fuse_rms, eps=1e-5)
        close(out, exp, 2e-2)


@pytest.mark.parametrize("M", [3, 6, 16])
def test_skinny_large_k_residual(M, skinny_mode):
    """Down-projection shape (K = 14336): past 5 rows X no longer fits in LDS and the streaming
    kernel reads X fragments from global memory (XG variant)."""
    K, N = 14336, 512
    x = rnd(M, K)
    w = rnd(N, K, scale=0.02)
    res = rnd(M, N)
    out = torch.empty(M, N, dtype=BF, device=DEV)
    ops.linear(x, w, out=out, residual=res)
    exp = torch.empty(M, N, dtype=BF)
    ref.linear(x.cpu(), w.cpu(), None, out=exp, residual=res.cpu())
    close(out, exp, 3e-2)


def test_skinny_f32_out_large_n_and_inplace_residual(skinny_mode):
    M, K, N = 3, 4096, 4096
    x = rnd(M, K)
    w = rnd(N, K, scale=0.02)
    logits = torch.empty(M, N, dtype=torch.float32, device=DEV)
    ops.linear(x, w, out=logits, fuse_rms=True)
    exp = torch.empty(M, N, dtype=torch.float32)
    ref.linear(x.cpu(), w.cpu(), out=exp, fuse_rms=True)
    close(logits, exp, 1e-2)
    h = rnd(M, N)
    h0 = h.clone()
    ops.linear(x, w, out=h, residual=h)
    exp = torch.empty(M, N, dtype=BF)
    ref.linear(x.cpu(), w.cpu(), out=exp, residual=h0.cpu())
    close(h, exp, 3e-2)


@pytest.mark.parametrize("M", [1, 33])
def test_skinny_swiglu(M, skinny_mode):
    K, F = 512, 256
    x = rnd(M, K)
    wg, wu = rnd(F, K, scale=0.05), rnd(F, K, scale=0.05)
    wgu = ops.interleave_gate_up(wg, wu)
    out = ops.linear_swiglu(x, wgu, fuse_rms=True)
    xf = x.float().cpu()
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    exp = torch.nn.functional.silu(xf @ wg.float().cpu().t()) * (xf @ wu.float().cpu().t())
    close(out, exp, 2e-2)
    # prefill-sized rows: the tiled MFMA GEMM (gemm.hip) with the SwiGLU epilogue
    x2 = rnd(80, K)
    out2 = ops.linear_swiglu(x2, wgu)
    exp2 = torch.nn.functional.silu(x2.float().cpu() @ wg.float().cpu().t()) * (x2.float().cpu() @ wu.float().cpu().t())
    close(out2, exp2, 3e-2)


def _kv_setup(nq, nkv, hd, blocks=16, bs=16):
    kc = torch.zeros(blocks, nkv, bs, hd, dtype=BF, device=DEV)
    vc = torch.zeros_like(kc)
    return kc, vc


@pytest.mark.parametrize("M", [1, 7, 40, 70])
def test_qkv_rope_write(M, skinny_mode):
    nq, nkv, hd, K = 8, 2, 128, 512
    H = nq + 2 * nkv
    w = rnd(H * hd, K, scale=0.05)
    wp = ops.permute_qkv_rows(w, H, hd)
    x = rnd(M, K)
    rope = ops.rope_table(256, hd, 500000.0, device=DEV)
    pos = torch.randint(0, 200, (M,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(16 * 16, device=DEV)[:M].to(torch.int64)
    kc, vc = _kv_setup(nq, nkv, hd)
    q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
    ops.qkv_rope_write(x, wp, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, rope=rope,
                       positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.zeros(M, nq * hd, dtype=BF)
    ref.qkv_rope_write(x.cpu(), wp.cpu(), None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                       rope=rope.cpu(), positions=pos.cpu(), slots=slots.cpu(), q_out=q2, k_cache=kc2, v_cache=vc2)
    close(q, q2, 3e-2)
    close(kc, kc2, 3e-2)
    close(vc, vc2, 3e-2)


@pytest.mark.parametrize("small_bytes", [0, 4 << 20], ids=["stream", "one_tile"])
@pytest.mark.parametrize("M", [1, 6, 16, 24, 40, 64])
def test_folded_layernorm_linear_and_qkv(M, small_bytes):
    """LayerNorm folded into the GEMM (mean/rstd from the streamed / staged rows) vs LayerNorm ->
    linear in f32, on the persistent streaming kernel and on the one-tile kernel small weights
    are routed to (skinny_gemm.hip; 17..64 rows with small weights: its MT row tiles, one launch,
    no LayerNorm kernel -- ops._small_rows).  Inputs carry a
    large mean (the residual stream's offset) to exercise the mean * rowsum correction."""
    ops.ext().set_small_gemm_bytes(small_bytes)
    try:
        _folded_layernorm_case(M)
    finally:
        ops.ext().set_small_gemm_bytes(4 << 20)


def _folded_layernorm_case(M):
    K, N = 384, 512
    x = (torch.randn(M, K, device=DEV) * 2 + 3).to(BF)
    gamma, beta = rnd(K, scale=0.5) + 1, rnd(K, scale=0.2)
    w, b = rnd(N, K, scale=0.05), rnd(N, scale=0.1)
    wf, bf, c = ops.fold_layernorm(w, b, gamma, beta)
    xf = torch.nn.functional.layer_norm(x.float().cpu(), (K,), gamma.float().cpu(), beta.float().cpu(), 1e-5)
    res = rnd(M, N)
    for act, r in (("none", None), ("gelu", None), ("none", res)):
        out = torch.empty(M, N, dtype=BF, device=DEV)
        ops.linear(x, wf, bf, out=out, act=act, residual=r, eps=1e-5, ln_c=c)
        exp = xf @ w.float().cpu().t() + b.float().cpu()
        if act == "gelu":
            exp = torch.nn.functional.gelu(exp)
        if r is not None:
            exp = exp + r.float().cpu()
        close(out, exp, 3e-2)
    # QKV epilogue with the folded norm (Whisper decoder self-attention: no RoPE)
    H, hd = 4, 64
    wq, bq = rnd(3 * H * hd, K, scale=0.05), rnd(3 * H * hd, scale=0.1)
    wqp = ops.permute_qkv_rows(wq, 3 * H, hd)
    bqp = ops.permute_qkv_rows(bq[:, None], 3 * H, hd)[:, 0].contiguous()
    wfq, bfq, cq = ops.fold_layernorm(wqp, bqp, gamma, beta)
    pos = torch.arange(M, dtype=torch.int32, device=DEV)
    slots = torch.randperm(8 * 16, device=DEV)[:M].to(torch.int64)
    kc, vc = _kv_setup(H, H, hd, blocks=8)
    q = torch.zeros(M, H * hd, dtype=BF, device=DEV)
    ops.qkv_rope_write(x, wfq, bfq, fuse_rms=False, eps=1e-5, n_q_heads=H, n_kv_heads=H, head_dim=hd, rope=None,
                       positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc, ln_c=cq)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.zeros(M, H * hd, dtype=BF)
    ref.qkv_rope_write(xf.to(BF), wqp.cpu(), bqp.cpu(), fuse_rms=False, eps=1e-5, n_q_heads=H, n_kv_heads=H,
                       head_dim=hd, rope=None, positions=pos.cpu(), slots=slots.cpu(), q_out=q2, k_cache=kc2,
                       v_cache=vc2)
    close(q, q2, 3e-2)
    close(kc, kc2, 3e-2)
    close(vc, vc2, 3e-2)


def test_norms():
    for D in (384, 4096):
        x, r = rnd(9, D), rnd(9, D)
        w, b = rnd(D), rnd(D)
        ro = torch.empty_like(x)
        y = ops.rmsnorm(x, w, eps=1e-5, residual=r, residual_out=ro)
        ro2 = torch.empty(9, D, dtype=BF)
        y2 = ref.rmsnorm(x.cpu(), w.cpu(), eps=1e-5, residual=r.cpu(), residual_out=ro2, out=torch.empty(9, D, dtype=BF))
        close(y, y2, 3e-2)
        close(ro, ro2, 2e-2)
        y = ops.layernorm(x, w, b, eps=1e-5)
        y2 = ref.layernorm(x.cpu(), w.cpu(), b.cpu(), eps=1e-5, out=torch.empty(9, D, dtype=BF))
        close(y, y2, 3e-2)


def test_bias_act_embedding():
    x, b, r = rnd(5, 64), rnd(64), rnd(5, 64)
    y = torch.empty_like(x)
    ops.ext().bias_act(x, b, r, y, 1)
    exp = torch.nn.functional.gelu(x.float() + b.float()) + r.float()
    close(y, exp, 2e-2)
    table = rnd(100, 64)
    pos_table = rnd(50, 64)
    ids = torch.tensor([3, 99, 0, 150], dtype=torch.int32, device=DEV)
    positions = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device=DEV)
    out = ops.embedding(ids, table, pos_table=pos_table, positions=positions, vocab_start=0)
    exp = ref.embedding(ids.cpu(), table.cpu(), pos_table=pos_table.cpu(), positions=positions.cpu(),
                        out=torch.empty(4, 64, dtype=BF))
    close(out, exp, 1e-2)


@pytest.mark.parametrize("hd,nq,nkv", [(128, 32, 8), (64, 6, 6)])
@pytest.mark.parametrize("ctx", [1, 100, 700])
def test_decode_attention_paged(hd, nq, nkv, ctx):
    bs, blocks = 16, 64
    kc = rnd(blocks, nkv, bs, hd)
    vc = rnd(blocks, nkv, bs, hd)
    rows = 3
    table = torch.stack([torch.randperm(blocks, device=DEV)[:48] for _ in range(2)]).to(torch.int32)
    seq_ids = torch.tensor([0, 1, 0], dtype=torch.int32, device=DEV)
    ctx_lens = torch.tensor([ctx, max(1, ctx // 2), min(ctx + 3, 48 * bs)], dtype=torch.int32, device=DEV)
    q = rnd(rows, nq * hd)
    kv = ops.KVLayout.paged(kc, vc, table)
    out = torch.empty_like(q)
    ops.decode_attention(q, kv, ctx_lens, seq_ids, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                         max_ctx=48 * bs, out=out)
    kvc = ops.KVLayout.paged(kc.cpu(), vc.cpu(), table.cpu())
    exp = ref.decode_attention(q.cpu(), kvc, ctx_lens.cpu(), seq_ids.cpu(), n_q_heads=nq, n_kv_heads=nkv,
                               head_dim=hd, scale=hd ** -0.5, out=torch.empty(rows, nq * hd, dtype=BF))
    close(out, exp, 2e-2)
    out1 = torch.empty_like(q)
    ops.decode_attention(q, kv, torch.clamp(ctx_lens, max=64), seq_ids, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                         scale=hd ** -0.5, max_ctx=64, out=out1)
    exp1 = ref.decode_attention(q.cpu(), kvc, torch.clamp(ctx_lens.cpu(), max=64), seq_ids.cpu(), n_q_heads=nq,
                                n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                                out=torch.empty(rows, nq * hd, dtype=BF))
    close(out1, exp1, 2e-2)


@pytest.fixture(params=["mq", "split"])
def attn_impl(request):
    ops.set_attention_impl(request.param)
    yield request.param
    ops.set_attention_impl("mq")


@pytest.mark.parametrize("hd,nq,nkv", [(128, 32, 8), (128, 8, 1), (64, 6, 6), (64, 8, 4)])
def test_decode_attention_row_groups(hd, nq, nkv, attn_impl):
    """Ragged step as the engines build it: jump-forward runs of one sequence (consecutive
    positions, shared K/V), single rows of other sessions, and a run longer than one row group
    (16 / G rows); contexts straddle chunk boundaries and one row sees a single key."""
    bs, blocks = 16, 160
    kc = rnd(blocks, nkv, bs, hd)
    vc = rnd(blocks, nkv, bs, hd)
    table = torch.stack([torch.randperm(blocks, device=DEV)[:40] for _ in range(4)]).to(torch.int32)
    seqs = [0] * 5 + [1] + [2] * 19 + [3]
    ctx = list(range(300, 305)) + [1] + list(range(620, 639)) + [129]
    rows = len(seqs)
    seq_ids = torch.tensor(seqs, dtype=torch.int32, device=DEV)
    ctx_lens = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    q = rnd(rows, nq * hd)
    kv = ops.KVLayout.paged(kc, vc, table)
    out = torch.empty_like(q)
    cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
    for _ in range(2):  # second launch: tickets must have been left zero
        ops.decode_attention(q, kv, ctx_lens, seq_ids, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                             scale=hd ** -0.5, max_ctx=40 * bs, out=out, counters=cnt)
    assert int(cnt.abs().sum()) == 0
    exp = ref.decode_attention(q.cpu(), ops.KVLayout.paged(kc.cpu(), vc.cpu(), table.cpu()), ctx_lens.cpu(),
                               seq_ids.cpu(), n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                               out=torch.empty(rows, nq * hd, dtype=BF))
    close(out, exp, 2e-2)


def test_decode_attention_cross_contiguous(attn_impl):
    """Whisper cross-attention: contiguous [B, 1500, H, 64] encoder K/V, one block per session."""
    B, T, H, hd = 3, 1500, 6, 64
    k, v = rnd(B, T, H, hd), rnd(B, T, H, hd)
    table = torch.arange(B, dtype=torch.int32, device=DEV)[:, None].contiguous()
    seq_ids = torch.tensor([2, 0, 1, 1], dtype=torch.int32, device=DEV)
    lens = torch.full((4,), T, dtype=torch.int32, device=DEV)
    q = rnd(4, H * hd)
    out = torch.empty_like(q)
    ops.decode_attention(q, ops.KVLayout.contiguous(k, v, table), lens, seq_ids, n_q_heads=H, n_kv_heads=H,
                         head_dim=hd, scale=hd ** -0.5, max_ctx=T, out=out)
    exp = ref.decode_attention(q.cpu(), ops.KVLayout.contiguous(k.cpu(), v.cpu(), table.cpu()), lens.cpu(),
                               seq_ids.cpu(), n_q_heads=H, n_kv_heads=H, head_dim=hd, scale=hd ** -0.5,
                               out=torch.empty(4, H * hd, dtype=BF))
    close(out, exp, 2e-2)


def test_flash_attention_causal_paged_prefix():
    hd, nq, nkv, bs = 128, 8, 2, 16
    blocks = 40
    kc, vc = rnd(blocks, nkv, bs, hd), rnd(blocks, nkv, bs, hd)
    table = torch.randperm(blocks, device=DEV)[:32].to(torch.int32)[None]
    Sk, Sq = 300, 77
    q = rnd(1, Sq, nq, hd)
    kv = ops.KVLayout.paged(kc, vc, table)
    out = ops.flash_attention(q, kv, Sk=Sk, n_kv_heads=nkv, causal=True, scale=hd ** -0.5, q_offset=Sk - Sq)
    exp = ref.flash_attention(q.cpu(), ops.KVLayout.paged(kc.cpu(), vc.cpu(), table.cpu()), Sk=Sk, n_kv_heads=nkv,
                              causal=True, scale=hd ** -0.5, q_offset=Sk - Sq, out=torch.empty(1, Sq, nq, hd, dtype=BF))
    close(out, exp, 2e-2)


@pytest.mark.parametrize("B,S,H,D", [(2, 1500, 6, 64), (1, 1500, 20, 64), (1, 333, 4, 128)])
def test_flash_attention_encoder_shapes(B, S, H, D):
    # Whisper encoder shapes (tiny / large-v3) and a ragged 128-dim one, strided q / k / v views of
    # one fused QKV buffer (the encoder's layout)
    qkv = rnd(B, S, 3, H, D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    table = torch.arange(B, dtype=torch.int32, device=DEV)[:, None]
    out = ops.flash_attention(q, ops.KVLayout.contiguous(k, v, table), Sk=S, n_kv_heads=H, causal=False,
                              scale=D ** -0.5)
    exp = torch.nn.functional.scaled_dot_product_attention(q.float().transpose(1, 2), k.float().transpose(1, 2),
                                                           v.float().transpose(1, 2)).transpose(1, 2)
    close(out, exp.cpu(), 2e-2)


def test_flash_attention_deferred_rescale():
    # scores whose running max climbs by more than the deferred-rescale threshold across tiles (keys
    # scaled up along the sequence) and very negative / very positive rows: the rare rescale branch.
    # The kernel folds scale * log2(e) into Q before rounding it to bf16 (its MFMA operand); with
    # these extreme scores (|s| ~ 60 in log2 units) that rounding alone moves near-tie softmax rows
    # by ~0.1, so the reference rounds Q the same way and the test checks the rescale logic.
    # (Own generator: the data must not depend on which tests ran before.)
    g = torch.Generator(device=DEV).manual_seed(11)
    B, S, H, D = 1, 700, 2, 64

    def r(*s):
        return torch.randn(*s, device=DEV, generator=g).to(BF)

    q = r(B, S, H, D) * 4
    k = r(B, S, H, D) * torch.linspace(0.2, 3.0, S, device=DEV).to(BF)[None, :, None, None]
    v = r(B, S, H, D)
    q[:, :50] *= 2
    q[:, 50:100] *= -2
    table = torch.arange(B, dtype=torch.int32, device=DEV)[:, None]
    sl2 = D ** -0.5 * 1.4426950408889634
    qs = (q.float() * sl2).to(BF).float()  # the kernel's Q operand
    for causal in (False, True):
        out = ops.flash_attention(q, ops.KVLayout.contiguous(k, v, table), Sk=S, n_kv_heads=H, causal=causal,
                                  scale=D ** -0.5)
        s = torch.einsum("bqhd,bkhd->bhqk", qs, k.float())
        if causal:
            s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=DEV).triu(1), float("-inf"))
        p = torch.exp2(s - s.amax(-1, keepdim=True))
        exp = torch.einsum("bhqk,bkhd->bqhd", p / p.sum(-1, keepdim=True), v.float())
        close(out, exp.cpu(), 3e-2)


def test_flash_attention_encoder_contiguous():
    B, S, H, D = 2, 150, 6, 64
    q, k, v = rnd(B, S, H, D), rnd(B, S, H, D), rnd(B, S, H, D)
    table = torch.arange(B, dtype=torch.int32, device=DEV)[:, None]
    kv = ops.KVLayout.contiguous(k, v, table)
    out = ops.flash_attention(q, kv, Sk=S, n_kv_heads=H, causal=False, scale=D ** -0.5)
    exp = torch.nn.functional.scaled_dot_product_attention(q.float().transpose(1, 2), k.float().transpose(1, 2),
                                                           v.float().transpose(1, 2)).transpose(1, 2)
    close(out, exp.cpu(), 2e-2)


def test_skinny_stream_many_tiles_and_k_tail(skinny_mode):
    # K = 384 (3 k-groups: waves with empty ranges), N spanning several persistent tiles per WG
    for M, K, N in ((1, 384, 51872), (4, 14336, 4096), (16, 1280, 5120)):
        x = rnd(M, K)
        w = rnd(N, K, scale=0.03)
        out = torch.empty(M, N, dtype=torch.float32, device=DEV)
        ops.linear(x, w, out=out, fuse_rms=True)
        exp = torch.empty(M, N, dtype=torch.float32)
        ref.linear(x.cpu(), w.cpu(), out=exp, fuse_rms=True)
        close(out, exp, 1e-2)


def test_sample_greedy_masked_and_gumbel():
    rows, V = 3, 128256
    logits = torch.randn(rows, V, device=DEV)
    words = (V + 31) // 32
    mask = torch.zeros(rows, words, dtype=torch.int32, device=DEV)
    allowed = [torch.randint(0, V, (50,)) for _ in range(rows)]
    mcpu = torch.zeros(rows, words, dtype=torch.int64)
    for r in range(rows):
        for a in allowed[r].tolist():
            mcpu[r, a // 32] |= 1 << (a % 32)
    mask.copy_(((mcpu + 2 ** 31) % 2 ** 32 - 2 ** 31).to(torch.int32))
    seed = torch.tensor([1234], dtype=torch.int64, device=DEV)
    step = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = torch.empty(rows, dtype=torch.int32, device=DEV)
    ops.sample(logits, mask=mask, temperature=None, seed=seed, step=step, out_tokens=out)
    for r in range(rows):
        al = allowed[r].to(DEV)
        assert int(out[r]) == int(al[torch.argmax(logits[r, al])])
    temp = torch.full((rows,), 0.7, device=DEV)
    step0 = int(step.item())
    ops.sample(logits, mask=mask, temperature=temp, seed=seed, step=step, out_tokens=out)
    exp = torch.empty(rows, dtype=torch.int32)
    ref.sample(logits.cpu(), mask=mask.cpu(), temperature=temp.cpu(), seed=seed.cpu(),
               step=torch.tensor([step0], dtype=torch.int32), out_tokens=exp)
    assert out.cpu().tolist() == exp.tolist()


def test_audio_frontend_and_conv():
    sr = 16000
    pcm = (torch.sin(torch.arange(sr * 2) * 2 * math.pi * 440 / sr) * 8000).to(torch.int16).to(DEV)
    f = ops.pcm16_to_f32(pcm)
    close(f, pcm.float().cpu() / 32768, 1e-6)
    n_frames = 3000
    audio = torch.zeros(n_frames * 160, device=DEV)
    audio[: f.numel()] = f
    window = torch.hann_window(400, periodic=True, device=DEV)
    fb = ref.mel_filterbank(n_mels=80).to(DEV)
    out = torch.empty(n_frames, 80, dtype=BF, device=DEV)
    ops.log_mel(audio, n_frames=n_frames, window=window, mel_fb=fb, out=out)
    exp = ref.log_mel(audio.cpu(), n_frames=n_frames, window=window.cpu(), mel_fb=fb.cpu(),
                      out=torch.empty(n_frames, 80, dtype=BF))
    close(out, exp, 3e-2)
    x = rnd(1, 3000, 80)
    w = rnd(384, 3 * 80, scale=0.05)
    b = rnd(384, scale=0.1)
    y = ops.conv1d_gelu(x, w, b, stride=1)
    y2 = ref.conv1d_gelu(x.cpu(), w.cpu(), b.cpu(), stride=1, out=torch.empty(1, 3000, 384, dtype=BF))
    close(y, y2, 3e-2)
    pos = rnd(1500, 384)
    z = ops.conv1d_gelu(y, rnd(384, 3 * 384, scale=0.02), b, stride=2, pos=pos)
    assert z.shape == (1, 1500, 384)


def test_log_mel_mfma_128_noise():
    # large-v3 front end (128 mels) on broadband noise + a tone: every bin and mel tile carries energy
    n_frames = 3000
    g = torch.Generator().manual_seed(3)
    a = torch.randn(n_frames * 160, generator=g) * 0.05
    a[:32000] += torch.sin(torch.arange(32000) * 2 * math.pi * 1000 / 16000) * 0.3
    audio = a.to(DEV)
    window = torch.hann_window(400, periodic=True, device=DEV)
    fb = ref.mel_filterbank(n_mels=128).to(DEV)
    out = torch.empty(n_frames, 128, dtype=BF, device=DEV)
    ops.log_mel(audio, n_frames=n_frames, window=window, mel_fb=fb, out=out)
    exp = ref.log_mel(audio.cpu(), n_frames=n_frames, window=window.cpu(), mel_fb=fb.cpu(),
                      out=torch.empty(n_frames, 128, dtype=torch.float32))
    assert (out.float().cpu() - exp).abs().max().item() < 1.2e-2  # bf16 rounding of values in [-1.5, 1.5]


@pytest.mark.parametrize("Cin,Cout,stride,B", [(128, 384, 1, 2), (384, 384, 2, 3), (1280, 1280, 2, 1)])
def test_conv_stem_implicit_gemm(Cin, Cout, stride, B):
    # the stem's padded-buffer path (no copy) against F.conv1d: batches are separate zero-padded slabs
    Tin = 3000
    _, xv = ops.padded_rows(B, Tin, Cin, dtype=BF, device=DEV)
    xv.copy_(rnd(B, Tin, Cin))
    w = rnd(Cout, 3 * Cin, scale=0.03)
    b = rnd(Cout, scale=0.1)
    Tout = (Tin - 1) // stride + 1
    pos = rnd(Tout, Cout) if stride == 2 else None
    y = ops.conv1d_gelu(xv, w, b, stride=stride, pos=pos, padded=True)
    yt = ops.conv1d_gelu(xv, ops.TiledWeight(w), b, stride=stride, pos=pos, padded=True)
    assert torch.equal(y, yt)  # pre-tiled weights: same products, same order
    exp = ref.conv1d_gelu(xv.cpu(), w.cpu(), b.cpu(), stride=stride, pos=None if pos is None else pos.cpu(),
                          out=torch.empty(B, Tout, Cout, dtype=torch.float32))
    close(y, exp, 3e-2)


# ----------------------------------------------------------------------------- fp8 (W8A8)
def _fp8_cpu(w8: "ops.FP8Weight") -> "ops.FP8Weight":
    return w8.to("cpu")


@pytest.mark.parametrize("M", [1, 5, 16, 40])
def test_fp8_linear_epilogues(M):
    """OCP e4m3 weights x per-row-quantised activations on the fp8 MFMA (decode rows <= 16) or the
    large-M fp8 path, against the CPU emulation of the same W8A8 rounding."""
    K, N = 1024, 384
    x = rnd(M, K)
    w8 = ops.FP8Weight.quantize(rnd(N, K, scale=0.05))
    b = rnd(N, scale=0.1)
    for act, res, rms, odt in (("none", None, False, BF), ("none", rnd(M, N), True, BF), ("gelu", None, False, BF),
                               ("none", None, True, torch.float32)):
        out = torch.empty(M, N, dtype=odt, device=DEV)
        ops.linear(x, w8, b if act == "gelu" else None, out=out, residual=res, act=act, fuse_rms=rms, eps=1e-5)
        exp = torch.empty(M, N, dtype=odt)
        ops.linear(x.cpu(), _fp8_cpu(w8), b.cpu() if act == "gelu" else None, out=exp,
                   residual=None if res is None else res.cpu(), act=act, fuse_rms=rms, eps=1e-5)
        close(out, exp, 3e-2)


def test_fp8_large_k_and_swiglu():
    M, K, F = 8, 4096, 512
    x = rnd(M, K)
    wgu = ops.FP8Weight.quantize(ops.interleave_gate_up(rnd(F, K, scale=0.02), rnd(F, K, scale=0.02)))
    out = ops.linear_swiglu(x, wgu, fuse_rms=True, eps=1e-5)
    exp = torch.empty(M, F, dtype=BF)
    ops.linear_swiglu(x.cpu(), _fp8_cpu(wgu), fuse_rms=True, eps=1e-5, out=exp)
    close(out, exp, 3e-2)
    # down-projection shape: K = 14336 fits the fp8 LDS staging up to 10 rows
    xd = rnd(6, 14336)
    wd = ops.FP8Weight.quantize(rnd(256, 14336, scale=0.02))
    res = rnd(6, 256)
    o = torch.empty(6, 256, dtype=BF, device=DEV)
    ops.linear(xd, wd, out=o, residual=res)
    e = torch.empty(6, 256, dtype=BF)
    ops.linear(xd.cpu(), _fp8_cpu(wd), out=e, residual=res.cpu())
    close(o, e, 3e-2)


@pytest.mark.parametrize("M", [1, 9])
def test_fp8_qkv_rope_write(M):
    nq, nkv, hd, K = 8, 2, 128, 512
    H = nq + 2 * nkv
    w8 = ops.FP8Weight.quantize(ops.permute_qkv_rows(rnd(H * hd, K, scale=0.05), H, hd))
    x = rnd(M, K)
    rope = ops.rope_table(256, hd, 500000.0, device=DEV)
    pos = torch.randint(0, 200, (M,), dtype=torch.int32, device=DEV)
    slots = torch.randperm(16 * 16, device=DEV)[:M].to(torch.int64)
    kc, vc = _kv_setup(nq, nkv, hd)
    q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
    ops.qkv_rope_write(x, w8, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, rope=rope,
                       positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.zeros(M, nq * hd, dtype=BF)
    ops.qkv_rope_write(x.cpu(), _fp8_cpu(w8), None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv,
                       head_dim=hd, rope=rope.cpu(), positions=pos.cpu(), slots=slots.cpu(), q_out=q2, k_cache=kc2,
                       v_cache=vc2)
    close(q, q2, 3e-2)
    close(kc, kc2, 3e-2)
    close(vc, vc2, 3e-2)


@pytest.mark.parametrize("M", [1, 4, 9, 16])
def test_tiled_weights_match_row_major(M):
    """Pre-tiled bf16 weights (ops.tile_weight / TiledWeight, SkinnyParams::w_tiled) on the
    streaming kernel give the row-major results for every decode epilogue: store (f32 out, the LM
    head), residual, the down shape (K = 14336, XG variant past 5 rows), SwiGLU and QKV + RoPE +
    paged-KV write."""
    K, N = 4096, 1024
    x = rnd(M, K)
    w = rnd(N, K, scale=0.02)
    tw = ops.TiledWeight(w)
    assert torch.equal(ops.untile_weight(tw.t), w)
    a = torch.empty(M, N, dtype=torch.float32, device=DEV)
    b = torch.empty_like(a)
    ops.linear(x, w, out=a, fuse_rms=True)
    ops.linear(x, tw, out=b, fuse_rms=True)
    close(b, a, 1e-3, 1e-3)
    xd, wd, res = rnd(M, 14336), rnd(512, 14336, scale=0.01), rnd(M, 512)
    a, b = res.clone(), res.clone()
    ops.linear(xd, wd, out=a, residual=a)
    ops.linear(xd, ops.TiledWeight(wd), out=b, residual=b)
    close(b, a, 1e-2, 1e-2)
    gu = ops.interleave_gate_up(rnd(512, K, scale=0.02), rnd(512, K, scale=0.02))
    a = ops.linear_swiglu(x, gu, fuse_rms=True)
    b = ops.linear_swiglu(x, ops.TiledWeight(gu), fuse_rms=True)
    close(b, a, 1e-2, 1e-2)
    nq, nkv, hd = 8, 2, 128
    wq = ops.permute_qkv_rows(rnd((nq + 2 * nkv) * hd, K, scale=0.02), nq + 2 * nkv, hd)
    rope = ops.rope_table(512, hd, 5e5, device=DEV)
    pos = torch.arange(7, 7 + M, dtype=torch.int32, device=DEV)
    slots = torch.arange(M, dtype=torch.int64, device=DEV) + 3
    outs = []
    for ww in (wq, ops.TiledWeight(wq)):
        kc = torch.zeros(4, nkv, 16, hd, dtype=BF, device=DEV)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
        ops.qkv_rope_write(x, ww, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                           rope=rope, positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        close(b, a, 1e-2, 1e-2)


@pytest.mark.parametrize("M", [1, 3])
@pytest.mark.parametrize("tiled", [False, True])
def test_masked_lm_head_computes_only_admissible_tiles(M, tiled):
    """Grammar-masked LM head (SkinnyParams::col_mask, ops.linear(col_mask=...)): every 16-column
    tile with an admissible bit in one of the mask rows equals the dense f32 result, every other
    column of ``out`` is left untouched; a word offset (vocab shard under TP) shifts the bits."""
    K, N, W = 4096, 8192, 300
    x = rnd(M, K)
    w = rnd(N, K, scale=0.02)
    wt = ops.TiledWeight(w) if tiled else w
    dense = torch.empty(M, N, dtype=torch.float32, device=DEV)
    ops.linear(x, w, out=dense, fuse_rms=True)
    g = torch.Generator().manual_seed(3)
    for off in (0, 7):
        bits = torch.rand(M, W * 32, generator=g) < 0.004  # sparse, scattered
        bits[0, (off * 32 + 5000):(off * 32 + 5040)] = True  # and one dense run
        words = torch.zeros(M, W, dtype=torch.int64)
        for b in range(32):
            words |= bits[:, b::32].long() << b
        mask = words.to(torch.int32).to(DEV)  # (bit 31 wraps to the sign: same bits)
        out = torch.full((M, N), float("nan"), dtype=torch.float32, device=DEV)
        ops.linear(x, wt, out=out, fuse_rms=True, col_mask=mask, col_mask_off=off, mask_rows=M)
        cols = bits[:, off * 32 : off * 32 + N].any(0)
        live = cols.view(-1, 16).any(1).repeat_interleave(16)
        assert 0 < int(live.sum()) < N
        o = out.cpu()
        assert torch.isnan(o[:, ~live]).all(), "a tile without admissible tokens was computed"
        close(o[:, live], dense.cpu()[:, live], 1e-3, 1e-3)


@pytest.mark.parametrize("M", [17, 64, 85, 1011, 1500])
@pytest.mark.parametrize("tiled", [False, True])
def test_tiled_mfma_gemm_epilogues(M, tiled):
    """The LDS-tiled MFMA GEMM (csrc/kernels/gemm.hip) for M > 16 rows -- prefill, many-row decode
    steps, the Whisper encoder -- on pre-tiled and row-major weights, every epilogue, with and
    without split-K (small M x N), against the f32 reference."""
    for (N, K) in ((384, 384), (1024, 4096), (2048, 512)):  # (the last: the 256 x 256 tile from 512 rows)
        x = rnd(M, K)
        w = rnd(N, K, scale=K ** -0.5)
        wt = ops.TiledWeight(w) if tiled else w
        b = rnd(N, scale=0.1)
        xc, wc, bc = x.cpu(), w.cpu(), b.cpu()
        for act, fuse in (("none", False), ("none", True), ("gelu", False)):
            out = torch.empty(M, N, dtype=BF, device=DEV)
            ops.linear(x, wt, b, out=out, act=act, fuse_rms=fuse)
            exp = torch.empty(M, N, dtype=BF)
            ref.linear(xc, wc, bc, out=exp, act=act, fuse_rms=fuse)
            close(out, exp, 2e-2)
        res = rnd(M, N)
        exp = torch.empty(M, N, dtype=BF)
        ref.linear(xc, wc, None, out=exp, residual=res.cpu(), fuse_rms=True)
        ops.linear(x, wt, out=res, residual=res, fuse_rms=True)  # in place: h = h + rms(x) W^T
        close(res, exp, 3e-2)
        o32 = torch.empty(M, N, dtype=torch.float32, device=DEV)
        ops.linear(x, wt, out=o32)
        e32 = torch.empty(M, N, dtype=torch.float32)
        ref.linear(xc, wc, None, out=e32)
        close(o32, e32, 2e-3, 2e-3)
    gu = ops.interleave_gate_up(rnd(512, 1024, scale=0.03), rnd(512, 1024, scale=0.03))
    x = rnd(M, 1024)
    got = ops.linear_swiglu(x, ops.TiledWeight(gu) if tiled else gu, fuse_rms=True)
    exp = torch.empty(M, 512, dtype=BF)
    ref.linear_swiglu(x.cpu(), gu.cpu(), fuse_rms=True, out=exp)
    close(got, exp, 2e-2)


@pytest.mark.parametrize("M", [256, 300, 1011])
def test_gemm_8phase_256_tile(M):
    """The 256 x 256 8-phase pipelined GEMM (gemm.hip P8; forced on every eligible shape) on
    pre-tiled weights: every epilogue, split-K (few tiles) and a partial last row block, against
    the f32 reference -- then back to the measured routing."""
    E = ops.ext()
    E.gemm_set_p8(1)
    try:
        for (N, K) in ((512, 4096), (4096, 1024), (2048, 512)):
            x = rnd(M, K)
            w = rnd(N, K, scale=K ** -0.5)
            wt = ops.TiledWeight(w)
            b = rnd(N, scale=0.1)
            xc, wc, bc = x.cpu(), w.cpu(), b.cpu()
            for act, fuse in (("none", False), ("gelu", True)):
                out = torch.empty(M, N, dtype=BF, device=DEV)
                ops.linear(x, wt, b, out=out, act=act, fuse_rms=fuse)
                exp = torch.empty(M, N, dtype=BF)
                ref.linear(xc, wc, bc, out=exp, act=act, fuse_rms=fuse)
                close(out, exp, 2e-2)
            res = rnd(M, N)
            exp = torch.empty(M, N, dtype=BF)
            ref.linear(xc, wc, None, out=exp, residual=res.cpu())
            ops.linear(x, wt, out=res, residual=res)
            close(res, exp, 3e-2)
        gu = ops.interleave_gate_up(rnd(1024, 1024, scale=0.03), rnd(1024, 1024, scale=0.03))
        x = rnd(M, 1024)
        got = ops.linear_swiglu(x, ops.TiledWeight(gu), fuse_rms=True)
        exp = torch.empty(M, 1024, dtype=BF)
        ref.linear_swiglu(x.cpu(), gu.cpu(), fuse_rms=True, out=exp)
        close(got, exp, 2e-2)
    finally:
        E.gemm_set_p8(2)


def test_gemm_8phase_split_k_down_projection():
    """Measured routing (mode 2): the 1011-row Llama-3-8B down projection (K = 14336) runs the
    8-phase kernel in 4 split-K slices with the residual applied by the reduce kernel -- against
    an f32 reference (GPU fp32 matmul of the same bf16 operands)."""
    M, N, K = 1011, 4096, 14336
    x = rnd(M, K)
    w = rnd(N, K, scale=K ** -0.5)
    res = rnd(M, N)
    exp = (x.float() @ w.float().t() + res.float())
    ops.linear(x, ops.TiledWeight(w), out=res, residual=res)
    close(res, exp, 3e-2)


def test_gemm_replaces_hipblaslt(monkeypatch):
    """No projection of > 16 rows reaches torch.matmul (hipBLASLt) any more."""
    def boom(*a, **k):
        raise AssertionError("torch.matmul used for a bf16 projection")

    monkeypatch.setattr(torch, "matmul", boom)
    x = rnd(300, 2048)
    for w in (rnd(768, 2048, scale=0.02), ops.TiledWeight(rnd(768, 2048, scale=0.02))):
        ops.linear(x, w, fuse_rms=True)
        ops.linear_swiglu(x, w, fuse_rms=True)


@pytest.mark.parametrize("M", [17, 100])
def test_gemm_qkv_rope_kv_write(M):
    """> 16-row QKV projection: tiled GEMM into a scratch row block + the RoPE / paged-KV kernel ==
    the reference projection + rotary + cache write."""
    K, nq, nkv, hd = 1024, 4, 2, 128
    w = ops.permute_qkv_rows(rnd((nq + 2 * nkv) * hd, K, scale=0.03), nq + 2 * nkv, hd)
    x = rnd(M, K)
    rope = ops.rope_table(512, hd, 5e5, device=DEV)
    pos = torch.arange(3, 3 + M, dtype=torch.int32, device=DEV)
    slots = torch.arange(M, dtype=torch.int64, device=DEV) + 5
    res = []
    for dev, ww in ((DEV, ops.TiledWeight(w)), ("cpu", w.cpu())):
        kc = torch.zeros(16, nkv, 16, hd, dtype=BF, device=dev)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF, device=dev)
        ops.qkv_rope_write(x.to(dev), ww, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                           rope=rope.to(dev), positions=pos.to(dev), slots=slots.to(dev), q_out=q, k_cache=kc,
                           v_cache=vc)
        res.append((q, kc, vc))
    for a, b in zip(*res):
        close(a, b, 3e-2)


@pytest.mark.parametrize("M", [1, 4, 16, 17, 40, 64, 85, 1011])
def test_fp8_tiled_weights_w8a8(M):
    """fp8 weights in the fp8 tiled layout (ops.tile_weight_fp8): the W8A8 streaming kernel (<= 16
    rows), the W8A16 tiled GEMM (gemm.hip W8: 17..FP8_A16_ROWS rows, e4m3 tiles converted on the LDS
    read) and the W8A8 tiled GEMM (gemm.hip F8, more rows) against the CPU emulation of the same
    rounding, for the store / residual / SwiGLU / QKV epilogues."""
    assert ops.FP8_A16_ROWS == 64  # (the row classes above)
    K, N = 4096, 1024
    x = rnd(M, K)
    w = rnd(N, K, scale=K ** -0.5)
    wq = ops.FP8Weight.quantize(w, tiled=True)
    assert wq.tiled and torch.equal(ops.untile_weight_fp8(wq.w8).view(torch.uint8),
                                    ops.FP8Weight.quantize(w, tiled=False).w8.view(torch.uint8))
    wc = ops.FP8Weight(wq.rows().cpu(), wq.scale.cpu())
    out = torch.empty(M, N, dtype=BF, device=DEV)
    ops.linear(x, wq, out=out, fuse_rms=True)
    exp = ops.linear(x.cpu(), wc, fuse_rms=True)
    close(out, exp, 3e-2, 3e-2)
    res = rnd(M, N)
    exp = ops.linear(x.cpu(), wc, residual=res.cpu())
    ops.linear(x, wq, out=res, residual=res)
    close(res, exp, 3e-2, 3e-2)
    gu = ops.interleave_gate_up(rnd(512, K, scale=K ** -0.5), rnd(512, K, scale=K ** -0.5))
    gq = ops.FP8Weight.quantize(gu, tiled=True)
    got = ops.linear_swiglu(x, gq, fuse_rms=True)
    exp = ops.linear_swiglu(x.cpu(), ops.FP8Weight(gq.rows().cpu(), gq.scale.cpu()), fuse_rms=True)
    close(got, exp, 3e-2, 3e-2)
    nq, nkv, hd = 4, 2, 128
    wqkv = ops.permute_qkv_rows(rnd((nq + 2 * nkv) * hd, K, scale=K ** -0.5), nq + 2 * nkv, hd)
    qq = ops.FP8Weight.quantize(wqkv, tiled=True)
    rope = ops.rope_table(2048, hd, 5e5, device=DEV)
    pos = torch.arange(M, dtype=torch.int32, device=DEV)
    slots = torch.arange(M, dtype=torch.int64, device=DEV)
    outs = []
    for dev, ww in ((DEV, qq), ("cpu", ops.FP8Weight(qq.rows().cpu(), qq.scale.cpu()))):
        nb = (M + 15) // 16 + 1
        kc = torch.zeros(nb, nkv, 16, hd, dtype=BF, device=dev)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF, device=dev)
        ops.qkv_rope_write(x.to(dev), ww, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                           rope=rope.to(dev), positions=pos.to(dev), slots=slots.to(dev), q_out=q, k_cache=kc,
                           v_cache=vc)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        close(a, b, 4e-2, 4e-2)


@pytest.mark.parametrize("M", [600, 1011])
def test_fp8_gemm_large_tile(M):
    """W8A8 tiled GEMM on the 256 x 256 workgroup tile (>= 512 rows, N % 256 == 0) vs emulation."""
    K, N = 1024, 2048
    x = rnd(M, K)
    w = rnd(N, K, scale=K ** -0.5)
    wq = ops.FP8Weight.quantize(w, tiled=True)
    out = torch.empty(M, N, dtype=BF, device=DEV)
    ops.linear(x, wq, out=out, fuse_rms=True)
    exp = ops.linear(x.cpu(), ops.FP8Weight(wq.rows().cpu(), wq.scale.cpu()), fuse_rms=True)
    close(out, exp, 3e-2, 3e-2)


@pytest.mark.parametrize("M", [1, 2, 4, 8])
def test_llama70b_tp8_per_rank_decode_shapes(M):
    """One rank's decode projections of Llama-3-70B at TP=8 (BASELINE config 4): o_proj
    [8192, 1024] and down [8192, 3584] (row-parallel, residual epilogue), gate/up [2 x 3584, 8192]
    (SwiGLU) and QKV [(8 + 2) x 128, 8192] (1 kv head: RoPE + paged-KV write) on pre-tiled weights
    through the streaming kernel, against the f32 reference."""
    d, F, nq, nkv, hd = 8192, 3584, 8, 1, 128
    x = rnd(M, d)
    res = rnd(M, d)
    for N, K in ((d, nq * hd), (d, F)):
        xi, w = rnd(M, K), rnd(N, K, scale=0.02)
        out = res.clone()
        ops.linear(xi, ops.TiledWeight(w), out=out, residual=out)
        want = ref.linear(xi.cpu(), w.cpu(), None, out=res.clone().cpu(), residual=res.cpu())
        close(out, want, 2e-2)
    gu = ops.interleave_gate_up(rnd(F, d, scale=0.02), rnd(F, d, scale=0.02))
    a = ops.linear_swiglu(x, ops.TiledWeight(gu), fuse_rms=True)
    b = ref.linear_swiglu(x.cpu(), gu.cpu(), fuse_rms=True, eps=1e-5, out=torch.empty(M, F, dtype=BF))
    close(a, b, 2e-2)
    H = nq + 2 * nkv
    wq = ops.permute_qkv_rows(rnd(H * hd, d, scale=0.02), H, hd)
    rope = ops.rope_table(512, hd, 5e5, device=DEV)
    pos = torch.arange(7, 7 + M, dtype=torch.int32, device=DEV)
    slots = torch.arange(M, dtype=torch.int64, device=DEV) + 3
    kc = torch.zeros(4, nkv, 16, hd, dtype=BF, device=DEV)
    vc = torch.zeros_like(kc)
    q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
    ops.qkv_rope_write(x, ops.TiledWeight(wq), None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv,
                       head_dim=hd, rope=rope, positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)
    kc2, vc2 = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q2 = torch.zeros(M, nq * hd, dtype=BF)
    ref.qkv_rope_write(x.cpu(), wq.cpu(), None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                       rope=rope.cpu(), positions=pos.cpu(), slots=slots.cpu(), q_out=q2, k_cache=kc2, v_cache=vc2)
    for a, b in ((q, q2), (kc, kc2), (vc, vc2)):
        assert torch.isfinite(a.float()).all()
        close(a, b, 3e-2)


def test_quant_fp8_rows_with_rstd():
    """The fp8 row quantiser's optional RMSNorm output (one row pass for the W8A8 GEMM's two row
    statistics) equals row_rstd, and the codes / scales are unchanged by it."""
    E = ops.ext()
    for M, K in ((33, 4096), (64, 14336)):
        x = rnd(M, K)
        q1 = torch.empty(M, K, dtype=torch.float8_e4m3fn, device=DEV)
        q2 = torch.empty_like(q1)
        s1 = torch.empty(M, device=DEV)
        s2 = torch.empty(M, device=DEV)
        r1 = torch.empty(M, device=DEV)
        r2 = torch.empty(M, device=DEV)
        E.quant_fp8_rows(x, q1, s1)
        E.quant_fp8_rows(x, q2, s2, r2, 1e-5)
        E.row_rstd(x, r1, 1e-5)
        assert torch.equal(q1.view(torch.uint8), q2.view(torch.uint8)) and torch.equal(s1, s2)
        exp = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
        torch.testing.assert_close(r2, exp, rtol=1e-4, atol=0)
        torch.testing.assert_close(r2, r1, rtol=1e-5, atol=0)


@pytest.mark.parametrize("M", [17, 48, 300])
@pytest.mark.parametrize("kind", ["bf16", "fp8", "rowmajor"])
def test_gemm_qkv_epilogue_fused(M, kind, monkeypatch):
    """The QKV projection with the rotary + paged-KV write in the tiled GEMM's epilogue (EPI_QKV:
    one-launch split-K at few rows, the plain / 256^2 epilogue at 300) == GEMM + rope_kv_write and
    the f32 reference, Llama-3-8B head geometry; a negative slot writes no cache row."""
    K, nq, nkv, hd = 4096, 32, 8, 128
    w = ops.permute_qkv_rows(rnd((nq + 2 * nkv) * hd, K, scale=K ** -0.5), nq + 2 * nkv, hd)
    ww = {"bf16": lambda: ops.TiledWeight(w), "fp8": lambda: ops.FP8Weight.quantize(w, tiled=True),
          "rowmajor": lambda: w}[kind]()
    x = rnd(M, K)
    rope = ops.rope_table(2048, hd, 5e5, device=DEV)
    pos = torch.arange(100, 100 + M, dtype=torch.int32, device=DEV)
    slots = torch.randperm(40 * 16, device=DEV)[:M].to(torch.int64)
    slots[M // 2] = -1

    def run(fused):
        monkeypatch.setattr(ops, "GEMM_QKV_FUSED", fused)
        kc = torch.zeros(40, nkv, 16, hd, dtype=BF, device=DEV)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
        ops.qkv_rope_write(x, ww, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, rope=rope,
                           positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc)
        torch.cuda.synchronize()
        return q, kc, vc

    fused, plain = run(True), run(False)
    for a, b in zip(fused, plain):
        close(a, b, 3e-2, 3e-2)
    if kind != "fp8":
        kc = torch.zeros(40, nkv, 16, hd, dtype=BF)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF)
        ops.qkv_rope_write(x.cpu(), w.cpu(), None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd,
                           rope=rope.cpu(), positions=pos.cpu(), slots=slots.cpu(), q_out=q, k_cache=kc, v_cache=vc)
        for a, b in zip(fused, (q, kc, vc)):
            close(a, b, 3e-2, 3e-2)


@pytest.mark.parametrize("hd,nq,nkv", [(128, 32, 8), (128, 8, 1), (64, 8, 4)])
@pytest.mark.parametrize("n_sess,P", [(3, 128), (8, 1024), (32, 1024), (61, 512)])
def test_decode_attention_shared_prefix(hd, nq, nkv, n_sess, P):
    """Sessions over one prefix-cached prompt (the same physical blocks for the first P keys): the
    multi-query kernel's shared-prefix grouping ([P, n_real] words) == the reference and == the
    per-session grouping; runs of jump-forward rows, a session whose own keys end exactly at P,
    padded rows behind the real ones (seq 0, one key), counters left zero."""
    bs, per = 16, 100
    blocks = 8 + n_sess * per
    kc = rnd(blocks, nkv, bs, hd)
    vc = rnd(blocks, nkv, bs, hd)
    table = (torch.randperm(blocks - 8, device=DEV)[: n_sess * per] + 8).to(torch.int32).view(n_sess, per).contiguous()
    table[:, : P // bs] = table[0, : P // bs]
    seqs, ctx = [], []
    g = torch.Generator().manual_seed(n_sess)
    for s in range(n_sess):
        if s == 1:
            own = [0]  # own keys end exactly at P
        else:
            own = [int(torch.randint(1, 300, (1,), generator=g))]
        if s % 5 == 2:  # a jump-forward run of consecutive positions
            own = [own[0] + i for i in range(int(torch.randint(2, 6, (1,), generator=g)))]
        for o in own:
            if len(seqs) < 64:
                seqs.append(s)
                ctx.append(P + o if o else P)
    n_real = len(seqs)
    pad = min(64, n_real + 3) - n_real
    seqs += [0] * pad
    ctx += [1] * pad
    rows = len(seqs)
    seq_ids = torch.tensor(seqs, dtype=torch.int32, device=DEV)
    ctx_lens = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    q = rnd(rows, nq * hd)
    kv = ops.KVLayout.paged(kc, vc, table)
    cnt = torch.zeros(rows * nkv, dtype=torch.int32, device=DEV)
    shared = torch.tensor([P, n_real], dtype=torch.int32, device=DEV)
    outs = []
    for sh in (shared, None, shared):
        out = torch.empty_like(q)
        ops.decode_attention(q, kv, ctx_lens, seq_ids, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                             max_ctx=per * bs, out=out, counters=cnt, shared=sh)
        outs.append(out)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0
    exp = ref.decode_attention(q.cpu(), ops.KVLayout.paged(kc.cpu(), vc.cpu(), table.cpu()), ctx_lens.cpu(),
                               seq_ids.cpu(), n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, scale=hd ** -0.5,
                               out=torch.empty(rows, nq * hd, dtype=BF))
    close(outs[0][:n_real], exp[:n_real], 2e-2)
    close(outs[1][:n_real], exp[:n_real], 2e-2)
    assert torch.equal(outs[0], outs[2])



@pytest.mark.parametrize("M", [17, 40, 85, 600])
@pytest.mark.parametrize("wdt", ["bf16", "fp8"])
def test_rms_statistics_handoff(M, wdt):
    """Many-row residual GEMMs hand the next RMSNorm its row statistics (GemmParams::ss_*): the
    residual epilogue (direct, or in the split-K reduce) adds the squares of the stored bf16 rows
    to ss_out and zeroes ss_zero; the consumers (SwiGLU / QKV GEMMs, bf16 and W8A16 -- W8A8 keeps
    its quantiser's own 1/rms) read rsqrt(ss / K + eps) instead of a row_rstd launch -- equal to
    the row_rstd path."""
    d, F = 4096, 1024
    wrap = (lambda w: ops.FP8Weight.quantize(w)) if wdt == "fp8" else ops.TiledWeight  # noqa: E731
    wo, wgu = wrap(rnd(d, d, scale=d ** -0.5)), wrap(ops.interleave_gate_up(rnd(F, d, scale=0.02), rnd(F, d, scale=0.02)))
    x, h0 = rnd(M, d), rnd(M, d)
    ss = torch.full((2, 4096), 7, dtype=torch.int64, device=DEV)  # (u64 fixed point, ops.SS_SCALE)
    ss[0].zero_()
    h = h0.clone()
    ops.linear(x, wo, out=h, residual=h, ss_out=ss[0], ss_zero=ss[1])
    assert torch.all(ss[1] == 0)
    want = h.float().pow(2).sum(-1)
    close(ops.ss_float(ss[0, :M]).float(), want, 1e-3 * float(want.max()), 1e-4)
    assert torch.all(ss[0, M:] == 0)
    # integer atomics: the same statistics bits on every run
    ss2 = torch.zeros(4096, dtype=torch.int64, device=DEV)
    h2 = h0.clone()
    ops.linear(x, wo, out=h2, residual=h2, ss_out=ss2)
    assert torch.equal(ss2, ss[0])
    h_ref = h0.clone()
    ops.linear(x, wo, out=h_ref, residual=h_ref)
    assert torch.equal(h, h_ref)
    a = ops.linear_swiglu(h, wgu, fuse_rms=True, eps=1e-5, ss_in=ss[0])
    b = ops.linear_swiglu(h, wgu, fuse_rms=True, eps=1e-5)
    close(a, b, 1e-2, 1e-2)
    nq, nkv, hd = 4, 2, 128
    wq = wrap(ops.permute_qkv_rows(rnd((nq + 2 * nkv) * hd, d, scale=d ** -0.5), nq + 2 * nkv, hd))
    rope = ops.rope_table(2048, hd, 5e5, device=DEV)
    pos = torch.arange(M, dtype=torch.int32, device=DEV)
    slots = torch.arange(M, dtype=torch.int64, device=DEV)
    outs = []
    for s_in in (ss[0], None):
        nb = (M + 15) // 16 + 1
        kc = torch.zeros(nb, nkv, 16, hd, dtype=BF, device=DEV)
        vc = torch.zeros_like(kc)
        q = torch.zeros(M, nq * hd, dtype=BF, device=DEV)
        ops.qkv_rope_write(h, wq, None, fuse_rms=True, eps=1e-5, n_q_heads=nq, n_kv_heads=nkv, head_dim=hd, rope=rope,
                           positions=pos, slots=slots, q_out=q, k_cache=kc, v_cache=vc, ss_in=s_in)
        outs.append((q, kc, vc))
    for u, v in zip(*outs):
        close(u, v, 1e-2, 1e-2)



@pytest.mark.parametrize("hd", [64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("qmul", [1.0, 8.0])
def test_flash_attention_is_bitwise_reproducible(hd, causal, qmul):
    """The same inputs give the same output bits on every launch.  qmul = 8: scores scaled x8 (the
    'extreme' inputs on which round 5's D = 64 kernel still varied by 1-2 ulps -- its inline-asm
    v_max3 read the last MFMA's accumulators inside the hazard window, common.h vmax3)."""
    T, H = 700, 4
    qkv = rnd(1, T, 3, H, hd)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    q = (q.float() * qmul).to(BF)
    table = torch.zeros(1, 1, dtype=torch.int32, device=DEV)
    outs = [ops.flash_attention(q, ops.KVLayout.contiguous(k, v, table), Sk=T, n_kv_heads=H, causal=causal,
                                scale=hd ** -0.5).clone() for _ in range(10)]
    assert all(torch.equal(outs[0], o) for o in outs[1:])
    ref_o = torch.nn.functional.scaled_dot_product_attention(
        q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2), is_causal=causal).transpose(1, 2)
    close(outs[0], ref_o, 2e-2 * qmul)
