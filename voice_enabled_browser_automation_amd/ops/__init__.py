"""Op layer: every hot op of the ASR + intent-LLM stack.

On a GPU tensor the op runs the hand-written gfx950 HIP kernel from ``_vwa_kernels.so``
(csrc/kernels/*.hip); if that library is missing on a GPU host the op raises -- there is no
silent eager fallback.  On CPU tensors the op runs the torch reference in ``ops.reference``,
which is also the numerics oracle for the kernel tests (tests/test_kernels_gpu.py).

Layout conventions shared by kernels, reference and models:

* weights are bf16 ``[N, K]`` (out x in) row-major;
* fused QKV weights are row-permuted per head (``permute_qkv_rows``) so rotary pairs
  (d, d+hd/2) sit in columns c and c^8 of one 16-column MFMA tile;
* fused gate/up weights are interleaved per 16 rows (``interleave_gate_up``) so the SwiGLU
  epilogue sees matching gate/up columns in one workgroup;
* RMSNorm gammas are folded into the following projection's columns (``fold_norm``); the
  kernels apply the per-row 1/rms themselves;
* paged KV cache per layer: ``[num_blocks, n_kv_heads, block_size, head_dim]`` bf16.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

from ..utils.env import knob
from . import reference as ref

_EXT = None
_EXT_ERR: Optional[BaseException] = None


def ext():
    """Load the native kernel library (once). Raises if unavailable."""
    global _EXT, _EXT_ERR
    if _EXT is not None:
        return _EXT
    if _EXT_ERR is not None:
        raise RuntimeError(f"native gfx950 kernel library unavailable: {_EXT_ERR}") from _EXT_ERR
    try:
        alt = knob("VWA_KERNEL_SO")  # (A/B experiments: another build of the same library)
        if alt:
            import importlib.machinery
            import importlib.util

            name = __name__ + "._vwa_kernels"
            spec = importlib.util.spec_from_file_location(
                name, alt, loader=importlib.machinery.ExtensionFileLoader(name, alt))
            m = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(m)
        else:
            from . import _vwa_kernels as m  # type: ignore

        # diagnostic overrides (utils/env.py Settings; defaults are the measured-best settings)
        impl = knob("VWA_ATTN_IMPL")
        if impl:
            m.set_attention_impl(ATTENTION_IMPLS[impl])
        p8 = knob("VWA_GEMM_P8")  # 0: 128x128 GEMM only, 1: 256x256 8-phase wherever eligible
        if p8 not in (None, ""):
            m.gemm_set_p8(int(p8))
        xsk = knob("VWA_SKINNY_X_SKEW")  # LDS-staged X rows: 64-B skew every 4 rows (1) / none (0)
        if xsk not in (None, ""):
            m.skinny_set_x_skew(int(xsk))
        fill = knob("VWA_GEMM_SPLIT_FILL")  # split-K until tiles x splits >= this % of CUs
        if fill not in (None, ""):
            m.gemm_set_split_fill(int(fill))
        _EXT = m
        return m
    except BaseException as e:  # noqa: BLE001
        _EXT_ERR = e
        raise RuntimeError(
            "native gfx950 kernel library _vwa_kernels.so failed to load; build it with "
            "`python -m voice_enabled_browser_automation_amd.ops.build`"
        ) from e


def native_available() -> bool:
    try:
        ext()
        return True
    except RuntimeError:
        return False


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------- fp8 weights
FP8_MAX = 448.0  # OCP e4m3fn


def tile_weight_fp8(w8: torch.Tensor) -> torch.Tensor:
    """fp8 counterpart of tile_weight: per 16-row tile T and 128-wide k-group kg one contiguous
    2 KB block [s 0..1][lane 0..63][16 B], lane = 16 g + n holding W8[16 T + n][128 kg + 32 g + 16 s
    .. + 16) -- the W8A8 streaming kernel's per-lane bytes (skinny_fp8_kernel) and the fp8 GEMM's
    B fragments (gemm.hip F8), so every load instruction reads 1 KB contiguous."""
    N, K = w8.shape
    assert N % 16 == 0 and K % 128 == 0, "tile_weight_fp8 needs N % 16 == 0 and K % 128 == 0"
    t = w8.view(torch.uint8).reshape(N // 16, 16, K // 128, 4, 2, 16)   # [T, n, kg, g, s, e]
    return t.permute(0, 2, 4, 3, 1, 5).contiguous().view(N, K).view(torch.float8_e4m3fn)


def untile_weight_fp8(t: torch.Tensor) -> torch.Tensor:
    N, K = t.shape
    u = t.view(torch.uint8).reshape(N // 16, K // 128, 2, 4, 16, 16)     # [T, kg, s, g, n, e]
    return u.permute(0, 4, 1, 3, 2, 5).contiguous().view(N, K).view(torch.float8_e4m3fn)


class FP8Weight:
    """OCP e4m3 weight [N, K] with a per-output-row f32 scale (VWA_DTYPE=fp8).

    ``tiled``: w8 is in the fp8 tiled layout (tile_weight_fp8), the one copy the GPU kernels read:
    decode GEMMs (<= 16 rows) run the W8A8 streaming kernel (activations quantised per row on the
    fly, dynamic amax/448 scale, fp8 MFMA) and larger row counts the W8A8 tiled GEMM (gemm.hip F8,
    X quantised by one row-quantisation kernel).  The CPU reference emulates the same rounding.
    """

    __slots__ = ("w8", "scale", "tiled")

    def __init__(self, w8: torch.Tensor, scale: torch.Tensor, tiled: bool = False):
        self.w8, self.scale, self.tiled = w8, scale, tiled

    @staticmethod
    def quantize(w: torch.Tensor, tiled: Optional[bool] = None) -> "FP8Weight":
        """tiled None: the tiled layout on a GPU (the only one its kernels read), row-major on the CPU."""
        if tiled is None:
            tiled = w.is_cuda and w.shape[0] % 16 == 0 and w.shape[1] % 128 == 0
        wf = w.float()
        scale = (wf.abs().amax(dim=1) / FP8_MAX).clamp_min(1e-12)
        w8 = (wf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).contiguous()
        if tiled:
            w8 = tile_weight_fp8(w8)
        return FP8Weight(w8, scale.contiguous(), tiled)

    def rows(self) -> torch.Tensor:
        """The row-major e4m3 matrix."""
        return untile_weight_fp8(self.w8) if self.tiled else self.w8

    def dequant(self, dtype=torch.float32) -> torch.Tensor:
        return (self.rows().float() * self.scale[:, None]).to(dtype)

    @property
    def shape(self):
        return self.w8.shape

    @property
    def device(self):
        return self.w8.device

    def numel(self) -> int:
        return self.w8.numel()

    def element_size(self) -> int:
        return 1

    def to(self, device) -> "FP8Weight":
        """Moved to a GPU, a row-major weight takes the tiled layout its kernels read (one copy);
        moved to the CPU, the reference's row-major layout."""
        dev = torch.device(device)
        w8 = self.w8
        N, K = w8.shape
        if dev.type == "cuda" and not self.tiled and N % 16 == 0 and K % 128 == 0:
            return FP8Weight(tile_weight_fp8(w8).to(dev), self.scale.to(dev), True)
        if dev.type == "cpu" and self.tiled:
            return FP8Weight(untile_weight_fp8(w8.to(dev)), self.scale.to(dev), False)
        return FP8Weight(w8.to(dev), self.scale.to(dev), self.tiled)


def quant_rows_fp8(x: torch.Tensor) -> torch.Tensor:
    """Per-row dynamic e4m3 quantise -> dequantise (f32), the activation rounding of the W8A8 path."""
    xf = x.float()
    s = (xf.abs().amax(dim=1, keepdim=True) / FP8_MAX)
    s = torch.where(s > 0, s, torch.ones_like(s))
    return (xf / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float() * s


def _ref_w8(x: torch.Tensor, w, fuse_rms: bool, eps: float):
    """(x, w) for the torch reference: the GPU path's rounding when w is fp8 -- W8A16 (x unquantised)
    for 17..FP8_A16_ROWS rows, W8A8 emulation otherwise (rms from the unquantised x)."""
    if not isinstance(w, FP8Weight):
        return x, w, fuse_rms
    if SKINNY_MAX_M < x.shape[0] <= FP8_A16_ROWS:
        return x, w.dequant(), fuse_rms
    xf = x.float()
    if fuse_rms:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
        # the kernel applies 1/rms after the product; quantising x or x/rms gives the same codes
    return quant_rows_fp8(xf), w.dequant(), False


def _fp8_stream_fits(M: int, K: int, nt: int = 1) -> bool:
    ks = 8
    return M <= 16 and M * (K + 16) + (ks * nt * 4 * 64 + 32) * 4 <= 160 * 1024


_SCALED_MM_OK: Optional[bool] = None


def vendor_fallback(what: str) -> None:
    """Called on every op path that leaves the hand-written kernels for a vendor library (hipBLASLt
    through torch.matmul / torch._scaled_mm) on a GPU tensor.  VWA_STRICT_NATIVE=1 (the GPU tests,
    bench.py) turns it into an error, so a new shape landing on a silent fallback is caught; the
    count is kept either way (``vendor_fallbacks``)."""
    vendor_fallbacks[what] = vendor_fallbacks.get(what, 0) + 1
    if knob("VWA_STRICT_NATIVE"):
        raise RuntimeError(f"strict native mode: {what} would fall back to a vendor library")


vendor_fallbacks: Dict[str, int] = {}


def _fp8_matmul(x: torch.Tensor, w: "FP8Weight") -> torch.Tensor:
    """x [M, K] bf16 @ W8^T for large M with an UNTILED fp8 weight (tiled ones take gemm_fp8):
    hipBLASLt fp8 GEMM with row-wise scales, or dequantise."""
    global _SCALED_MM_OK
    vendor_fallback(f"fp8 matmul {tuple(x.shape)} x {tuple(w.shape)}")
    if _SCALED_MM_OK is not False and hasattr(torch, "_scaled_mm"):
        try:
            x8 = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
            sx = torch.empty((x.shape[0], 1), dtype=torch.float32, device=x.device)
            ext().quant_fp8_rows(x, x8, sx)  # one HIP kernel: row amax -> scale -> e4m3
            y = torch._scaled_mm(x8, w.w8.t(), scale_a=sx, scale_b=w.scale[None, :].contiguous(),
                                 out_dtype=torch.bfloat16)
            _SCALED_MM_OK = True
            return y
        except (RuntimeError, TypeError):
            _SCALED_MM_OK = False
    return torch.matmul(x, w.dequant(x.dtype).t())


# ----------------------------------------------------------------------------- tiled bf16 weights
def tile_weight(w: torch.Tensor) -> torch.Tensor:
    """Pre-tiled copy of a bf16 weight [N, K] for the decode kernels (vwa_kernels.h
    SkinnyParams::w_tiled): per 16-row tile T and 128-wide k-group kg, one contiguous 4 KB block
    [s][lane][8] with lane = 16 * g + n holding W[16 T + n][128 kg + 32 g + 8 s + e], i.e. the
    MFMA B-operand fragments in the order the wave loads them -- each load instruction then
    reads 1 KB contiguous instead of 16 B pieces of 32 cache lines.  Same shape [N, K], so the
    host-side shape checks are unchanged; only the element order differs."""
    N, K = w.shape
    assert N % 16 == 0 and K % 128 == 0, "tile_weight needs N % 16 == 0 and K % 128 == 0"
    t = w.reshape(N // 16, 16, K // 128, 4, 4, 8)          # [T, n, kg, g, s, e]
    return t.permute(0, 2, 4, 3, 1, 5).contiguous().view(N, K)  # [T, kg, s, g, n, e]


def untile_weight(t: torch.Tensor) -> torch.Tensor:
    """Inverse of tile_weight (tests)."""
    N, K = t.shape
    return t.reshape(N // 16, K // 128, 4, 4, 16, 8).permute(0, 4, 1, 3, 2, 5).contiguous().view(N, K)


class TiledWeight:
    """A bf16 projection weight stored ONLY in the pre-tiled layout ``t`` = tile_weight(w) (same
    [N, K] shape, MFMA B-fragment element order).  Every GPU consumer reads it directly: the decode
    streaming / chained kernels (1 KB contiguous load instructions) and the LDS-tiled GEMM for
    prefill and > 16-row steps (gemm.hip copies the 4 KB fragment blocks to LDS verbatim) -- so
    the model keeps one copy of each weight.  ``dense()`` rebuilds the row-major matrix for the
    CPU reference and diagnostics."""

    __slots__ = ("t",)

    def __init__(self, w: Optional[torch.Tensor] = None, t: Optional[torch.Tensor] = None):
        self.t = tile_weight(w) if t is None else t

    def dense(self) -> torch.Tensor:
        return untile_weight(self.t)

    @property
    def w(self) -> torch.Tensor:  # row-major view for legacy callers (materialised on demand)
        return self.dense()

    @property
    def shape(self):
        return self.t.shape

    @property
    def device(self):
        return self.t.device

    @property
    def dtype(self):
        return self.t.dtype

    def numel(self) -> int:
        return self.t.numel()

    def element_size(self) -> int:
        return self.t.element_size()

    def to(self, device) -> "TiledWeight":
        return TiledWeight(t=self.t.to(device))


def _stream_ok(x: torch.Tensor, w) -> bool:
    """Decode rows (<= SKINNY_MAX_M) the streaming kernel takes with a pre-tiled weight."""
    return x.shape[0] <= SKINNY_MAX_M and x.shape[1] % 128 == 0 and w.shape[0] % 16 == 0


def plain(w):
    """The row-major tensor of a weight (TiledWeight -> dense(); anything else unchanged)."""
    return w.dense() if isinstance(w, TiledWeight) else w


# ----------------------------------------------------------------------------- layout helpers
def qkv_row_perm(head_dim: int) -> torch.Tensor:
    half = head_dim // 2
    idx = []
    for t in range(head_dim // 16):
        idx += [8 * t + p for p in range(8)] + [half + 8 * t + p for p in range(8)]
    return torch.tensor(idx, dtype=torch.long)


def permute_qkv_rows(w: torch.Tensor, n_heads_total: int, head_dim: int) -> torch.Tensor:
    perm = qkv_row_perm(head_dim)
    full = torch.cat([perm + h * head_dim for h in range(n_heads_total)])
    return w[full].contiguous()


_UNPERM: dict = {}


def unpermute_qkv_cols(y: torch.Tensor, n_heads_total: int, head_dim: int) -> torch.Tensor:
    key = (n_heads_total, head_dim, str(y.device))
    full = _UNPERM.get(key)
    if full is None:  # (a pure function of the sizes: built once, the CPU decode calls it per layer)
        perm = qkv_row_perm(head_dim)
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(head_dim)
        full = _UNPERM[key] = torch.cat([inv + h * head_dim for h in range(n_heads_total)]).to(y.device)
    return y[..., full]


def interleave_gate_up(w_gate: torch.Tensor, w_up: torch.Tensor) -> torch.Tensor:
    F, K = w_gate.shape
    assert F % 16 == 0
    g = w_gate.view(F // 16, 16, K)
    u = w_up.view(F // 16, 16, K)
    return torch.stack([g, u], dim=1).reshape(2 * F, K).contiguous()


def fold_norm(w: torch.Tensor, gamma: torch.Tensor) -> torch.Tensor:
    return (w.float() * gamma.float()[None, :]).to(w.dtype)


def fold_layernorm(w: torch.Tensor, bias: Optional[torch.Tensor], gamma: torch.Tensor, beta: torch.Tensor):
    """LayerNorm(gamma, beta) folded into the following linear (w, bias).

    LN(x) @ w^T + b = rstd * (x @ (w*gamma)^T - mean * c) + (b + w @ beta),  c[n] = sum_k (w*gamma)[n, k]
    Returns (w*gamma, b + w@beta, c) -- c is computed from the ROUNDED folded weights so the
    kernel's mean term cancels exactly what its GEMM accumulates.
    """
    wf = w.float()
    wg = (wf * gamma.float()[None, :]).to(w.dtype).contiguous()
    b = wf @ beta.float()
    if bias is not None:
        b = b + bias.float()
    return wg, b.to(w.dtype).contiguous(), wg.float().sum(1).contiguous()


_LN_UNIT: dict = {}


def _layernorm_plain(x: torch.Tensor, eps: float) -> torch.Tensor:
    """(x - mean) * rstd (no affine): the input of a linear whose LayerNorm affine is folded in."""
    key = (x.shape[1], str(x.device), x.dtype)
    if key not in _LN_UNIT:
        _LN_UNIT[key] = (torch.ones(x.shape[1], dtype=x.dtype, device=x.device),
                         torch.zeros(x.shape[1], dtype=x.dtype, device=x.device))
    one, zero = _LN_UNIT[key]
    return layernorm(x, one, zero, eps=eps)


def _ln_fold_fits(x: torch.Tensor, w) -> bool:
    return (_gpu(x) and not isinstance(w, FP8Weight) and x.shape[1] % 128 == 0 and w.shape[0] % 16 == 0
            and (x.shape[0] <= SKINNY_MAX_M or _small_rows(x, w)))


SMALL_MAX_M = 64         # rows the one-tile kernel (skinny_gemm.hip) takes with small weights
SMALL_BYTES = 4 << 20    # ... and what "small" is (the library's set_small_gemm_bytes default)


def _small_rows(x: torch.Tensor, w) -> bool:
    """17..64 rows with a small row-major bf16 weight (Whisper-tiny's decoder projections at a
    batched decode step): ONE launch of the one-tile kernel, with the folded LayerNorm, instead of
    a LayerNorm launch + the tiled GEMM's split-K pair (profiles/r4_asr_tiny_batch32_kernel_stats.md)."""
    return (SKINNY_MAX_M < x.shape[0] <= SMALL_MAX_M and isinstance(w, torch.Tensor) and not isinstance(w, TiledWeight)
            and w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and w.dim() == 2
            and w.shape[0] * w.shape[1] * 2 <= SMALL_BYTES and x.shape[1] % 128 == 0 and w.shape[0] % 16 == 0)


def rope_table(max_pos: int, head_dim: int, theta: float, device=None, scaling: Optional[dict] = None) -> torch.Tensor:
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / head_dim))
    if scaling:  # Llama-3.1 style frequency scaling
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        wl = 2 * math.pi / inv
        smooth = ((old / wl) - lo) / (hi - lo)
        scaled = torch.where(wl > old / lo, inv / factor, inv)
        mid = (wl <= old / lo) & (wl >= old / hi)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    pos = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    tab = torch.stack([torch.cos(pos), torch.sin(pos)], dim=-1).float()
    return tab.to(device) if device is not None else tab


# ----------------------------------------------------------------------------- scratch
_SCRATCH: dict = {}
_SCRATCH_RETIRED: list = []


def scratch(device, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
    """A per-device reusable buffer of at least ``numel`` elements (stream-ordered users only).
    A buffer outgrown by a larger request is RETIRED, never freed: a captured hipGraph may still
    address it (its replays keep using the old address while eager calls move to the new one)."""
    key = (str(device), name, dtype)
    t = _SCRATCH.get(key)
    if t is None or t.numel() < numel:
        if t is not None:
            _SCRATCH_RETIRED.append(t)
        t = torch.empty(max(numel, 1024), dtype=dtype, device=device)
        _SCRATCH[key] = t
    return t[:numel]


GEMM_WS_FLOATS = 32 << 20  # split-K workspace (128 MB per device: 4 f32 slices of a 1k x 4096 output)
# (a one-launch split-K -- the last slice of each tile reducing -- measured no faster at 32 decode
# rows: the write-through drain + ticket + L2-missing partial loads cost what the reduce launch
# does, fp8 o / down 26.3 vs 20.2 + 5.2 us, profiles/r4_gemm_one_launch_ab.md; removed in round 5.
# Round 6: the reduce loading all 8 slabs of an 8-way split in ONE batch instead of two batches of
# 4 -- same bits -- measured 0.3-1.6 % slower whole steps at 32-64 rows, fp8 and bf16,
# profiles/r6_reduce_one_batch_rejected_*.jsonl; not kept)


_GEMM_EPI = {"none": 0, "resid": 1, "swiglu": 2, "gelu": 3}


def _rstd(x: torch.Tensor, eps: float) -> torch.Tensor:
    """Per-row 1/rms of x (the RMSNorm of a projection whose gamma is folded into its weight)."""
    rstd = scratch(x.device, "gemm_rstd", x.shape[0])
    ext().row_rstd(x, rstd, eps)
    return rstd


def gemm(x: torch.Tensor, w, out: torch.Tensor, *, epi: str = "none", bias: Optional[torch.Tensor] = None,
         residual: Optional[torch.Tensor] = None, fuse_rms: bool = False, eps: float = 1e-5,
         ss_out: Optional[torch.Tensor] = None, ss_zero: Optional[torch.Tensor] = None,
         ss_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The hand-written LDS-tiled MFMA GEMM (csrc/kernels/gemm.hip) for M > 16 rows:
    out = epi(rms(x) @ w^T + bias); w a TiledWeight (its single pre-tiled copy) or a row-major bf16
    [N, K] tensor.  fuse_rms: the per-row 1/rms of x scales the product (gamma folded into w) --
    from ``ss_in`` (the rows' sums of squares, handed off by the GEMM that wrote x) when given, else
    one row_rstd launch.  ss_out / ss_zero (residual epilogue): see GemmParams::ss_*."""
    E = ext()
    rstd = _rstd(x, eps) if fuse_rms and ss_in is None else None
    tiled = isinstance(w, TiledWeight)
    wt = w.t if tiled else w
    ws = scratch(x.device, "gemm_ws", GEMM_WS_FLOATS)
    E.gemm(x, wt, bias, out, _GEMM_EPI[epi], rstd, residual, tiled, ws, ss_out, ss_zero,
           ss_in if fuse_rms else None, eps)
    return out


def _rows16(t: Optional[torch.Tensor]) -> bool:
    return t is None or (t.stride(-1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0)


def _fp8_staging(x: torch.Tensor, K: int):
    M = x.shape[0]
    x8 = scratch(x.device, "gemm_x8", M * K, torch.uint8).view(torch.float8_e4m3fn)
    return x8, scratch(x.device, "gemm_sx", M), scratch(x.device, "gemm_rstd", M)


def _fp8_input(x: torch.Tensor, fuse_rms: bool, eps: float):
    """(x8 [M, K], sx, rstd or None): x quantised per row by one kernel that also yields the
    RMSNorm 1/rms.  (Round 4's opt-in hand-off -- the previous GEMM's split-K reduce quantising its
    output rows -- measured slower in whole fp8 steps, profiles/r4_gemm_ab.md; removed in round 5.)"""
    M, K = x.shape
    x8, sx, rs = _fp8_staging(x, K)
    ext().quant_fp8_rows(x, x8[: M * K].view(M, K), sx, rs if fuse_rms else None, eps)
    return x8[: M * K].view(M, K), sx, (rs if fuse_rms else None)


# fp8 weights, > 16 rows: up to this many rows the tiled GEMM runs W8A16 (bf16 x, the e4m3 tiles
# converted to bf16 on the LDS read: no per-row quantisation launch -- the decode steps of many
# sessions are weight-streaming bound), above it W8A8 (the fp8 MFMA: prompt-sized, compute bound)
FP8_A16_ROWS = knob("VWA_FP8_A16_ROWS")


def gemm_fp8(x: torch.Tensor, w: "FP8Weight", out: torch.Tensor, *, epi: str = "none",
             bias: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None, fuse_rms: bool = False,
             eps: float = 1e-5, ss_out: Optional[torch.Tensor] = None, ss_zero: Optional[torch.Tensor] = None,
             ss_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp8-weight tiled MFMA GEMM (gemm.hip) for M > 16 rows.  <= FP8_A16_ROWS rows: W8A16 (bf16 x,
    weights converted in-kernel).  More: W8A8 -- x is quantised per row (amax / 448, one kernel that
    also yields the RMSNorm 1/rms), the fp8 MFMA runs on the tiled fp8 weight.  The scales (and the
    RMSNorm 1/rms of the unquantised x) apply in the epilogue."""
    E = ext()
    ws = scratch(x.device, "gemm_ws", GEMM_WS_FLOATS)
    if x.shape[0] <= FP8_A16_ROWS:
        E.gemm_fp8(x, None, w.w8, w.scale, bias, out, _GEMM_EPI[epi],
                   _rstd(x, eps) if fuse_rms and ss_in is None else None, residual, ws, ss_out, ss_zero,
                   ss_in if fuse_rms else None, eps)
        return out
    x8, sx, rstd = _fp8_input(x, fuse_rms, eps)  # (the quantiser yields the 1/rms: ss_in unused)
    E.gemm_fp8(x8, sx, w.w8, w.scale, bias, out, _GEMM_EPI[epi], rstd, residual, ws, ss_out, ss_zero)
    return out


def gemm_fp8_ok(x: torch.Tensor, w, out: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None) -> bool:
    return (isinstance(w, FP8Weight) and w.tiled and _gpu(x) and x.dtype == torch.bfloat16 and w.shape[0] % 16 == 0
            and w.shape[1] % 128 == 0 and _rows16(x) and _rows16(out) and _rows16(residual))


def gemm_ok(x: torch.Tensor, w, out: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None) -> bool:
    """Shapes the tiled GEMM takes (bf16 weights, N % 16, K % 128, 16-byte aligned rows)."""
    if isinstance(w, FP8Weight) or not _gpu(x) or x.dtype != torch.bfloat16:
        return False
    wt = w.t if isinstance(w, TiledWeight) else w
    return (wt.dtype == torch.bfloat16 and wt.shape[0] % 16 == 0 and wt.shape[1] % 128 == 0 and _rows16(x)
            and _rows16(out) and _rows16(residual))


# ----------------------------------------------------------------------------- GEMM family
# Rows handled by the MFMA streaming (skinny) kernels; above this the hand-written LDS-tiled MFMA
# GEMM (gemm.hip) takes the step (continuous batching of many sessions, prefill).
SKINNY_MAX_M = 16
# (round 4 built a 17..64-row form of the streaming kernel -- X streamed with the weights, MT = 2 /
# 4 row fragments -- and measured it slower than the tiled GEMM for whole decode steps, 32 rows
# 6.89 vs 5.65 ms, 64 rows 11.0 vs 6.9 ms, profiles/r4_rows_sweep_*; removed in round 5.)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *, out: Optional[torch.Tensor] = None,
           residual: Optional[torch.Tensor] = None, act: str = "none", fuse_rms: bool = False, eps: float = 1e-5,
           out_dtype: Optional[torch.dtype] = None, ln_c: Optional[torch.Tensor] = None,
           col_mask: Optional[torch.Tensor] = None, col_mask_off: int = 0, mask_rows: int = 1,
           ss_out: Optional[torch.Tensor] = None, ss_zero: Optional[torch.Tensor] = None,
           ss_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = act(rms(x) @ w^T + bias) [+ residual].

    GPU: decode rows (<= SKINNY_MAX_M) -> the MFMA streaming GEMM with fused epilogue; more rows
    -> the LDS-tiled MFMA GEMM (gemm.hip) with the same epilogues.  torch.matmul + the HIP
    epilogue kernels only for shapes neither kernel takes.
    ln_c (from fold_layernorm): x goes through a LayerNorm whose affine is folded into (w, bias);
    decode rows compute its mean/rstd inside the streaming GEMM, other shapes normalise first.
    col_mask (int32 token bitmask rows, the sampler's grammar mask; plain store epilogue): the
    streaming kernel computes only the 16-column tiles with an admissible bit (word col_mask_off
    onward) in one of the first mask_rows rows and leaves the other columns of ``out`` untouched
    -- they must only be read through the same mask.  Other paths compute every column.
    ss_out / ss_zero / ss_in: the RMS statistics hand-off of the tiled GEMMs (ops.gemm); a path
    without it honours ss_out / ss_zero with torch ops and computes its own 1/rms.
    """
    ss = dict(ss_out=ss_out, ss_zero=ss_zero, ss_in=ss_in, used=False)
    out = _linear_impl(x, w, bias, out, residual, act, fuse_rms, eps, out_dtype, ln_c, col_mask, col_mask_off,
                       mask_rows, ss)
    if not ss["used"] and (ss_out is not None or ss_zero is not None):  # (paths without the hand-off)
        if ss_zero is not None:
            ss_zero.zero_()
        if ss_out is not None:
            ss_out[: x.shape[0]] += ss_fixed(out.float().pow(2).sum(-1))
    return out


SS_SCALE = 16777216.0  # RMS statistics hand-off: u64 fixed point in 2^-24 units (GemmParams::ss_*)


def ss_fixed(sq: torch.Tensor) -> torch.Tensor:
    """f32 sums of squares -> the hand-off's int64 fixed point (2^-24 units, rounded to nearest as
    gemm.hip ss_fix does; clamped below the int64 maximum)."""
    return torch.floor(sq.float() * SS_SCALE + 0.5).clamp(max=9.2e18).to(torch.int64)


def ss_float(ss: torch.Tensor) -> torch.Tensor:
    """The hand-off's fixed-point sums of squares -> f64 values."""
    return ss.double() / SS_SCALE


def _linear_impl(x, w, bias, out, residual, act, fuse_rms, eps, out_dtype, ln_c, col_mask, col_mask_off, mask_rows,
                 ss):
    M = x.shape[0]

    def ssk():  # the hand-off arguments for the tiled GEMMs (which take them)
        ss["used"] = True
        return dict(ss_out=ss["ss_out"], ss_zero=ss["ss_zero"], ss_in=ss["ss_in"])

    mk = {}
    if col_mask is not None and residual is None and act == "none" and bias is None and ln_c is None:
        mk = dict(col_mask=col_mask, col_mask_off=col_mask_off, mask_rows=mask_rows)
    dt = out_dtype or (x.dtype if out is None else out.dtype)
    if out is None:
        out = torch.empty((M, w.shape[0]), dtype=dt, device=x.device)
    if isinstance(w, TiledWeight):
        if _gpu(x) and _stream_ok(x, w) and (ln_c is None or _ln_fold_fits(x, w)):
            epi = {"none": 0, "gelu": 3}[act]
            if residual is not None:
                assert act == "none"
                epi = 1
            ext().skinny_gemm(x, w.t, bias, out, epi, fuse_rms and ln_c is None, eps, residual, None, ln_c, True,
                              **mk)
            return out
        if ln_c is not None:
            return linear(_layernorm_plain(x, eps), w, bias, out=out, residual=residual, act=act, out_dtype=out_dtype)
        if _gpu(x) and gemm_ok(x, w, out, residual) and (act == "none" or residual is None) and \
                (out.dtype == torch.bfloat16 or (residual is None and act == "none")):
            e = "resid" if residual is not None else ("gelu" if act == "gelu" else "none")
            return gemm(x, w, out, epi=e, bias=bias, residual=residual, fuse_rms=fuse_rms, eps=eps, **ssk())
        w = w.dense()
    if ln_c is not None:
        if _ln_fold_fits(x, w):
            epi = {"none": 0, "gelu": 3}[act] if residual is None else 1
            ext().skinny_gemm(x, w, bias, out, epi, False, eps, residual, None, ln_c)
            return out
        return linear(_layernorm_plain(x, eps), w, bias, out=out, residual=residual, act=act, out_dtype=out_dtype)
    if not _gpu(x):
        xr, wr, fr = _ref_w8(x, w, fuse_rms, eps)
        return ref.linear(xr, wr, bias, out=out, residual=residual, act=act, fuse_rms=fr, eps=eps)
    E = ext()
    fp8 = isinstance(w, FP8Weight)
    if ((M <= SKINNY_MAX_M and x.shape[1] % 128 == 0 and w.shape[0] % 16 == 0
            and (not fp8 or _fp8_stream_fits(M, x.shape[1]))) or (not fp8 and not mk and _small_rows(x, w))):
        epi = {"none": 0, "gelu": 3}[act]
        if residual is not None:
            assert act == "none"
            epi = 1
        if fp8:
            E.skinny_gemm(x, w.w8, bias, out, epi, fuse_rms, eps, residual, w.scale, None, w.tiled)
        else:
            E.skinny_gemm(x, w, bias, out, epi, fuse_rms, eps, residual, **mk)
        return out
    e = "resid" if residual is not None else ("gelu" if act == "gelu" else "none")
    plain_epi = (act == "none" or residual is None) and (out.dtype == torch.bfloat16 or (residual is None and act == "none"))
    if fp8 and plain_epi and gemm_fp8_ok(x, w, out, residual):
        return gemm_fp8(x, w, out, epi=e, bias=bias, residual=residual, fuse_rms=fuse_rms, eps=eps, **ssk())
    if not fp8 and plain_epi and gemm_ok(x, w, out, residual):
        return gemm(x, w, out, epi=e, bias=bias, residual=residual, fuse_rms=fuse_rms, eps=eps, **ssk())
    if fp8 and w.tiled:
        w = FP8Weight(w.rows(), w.scale)  # (shapes the tiled kernels reject: dequantising path)
    xin = rmsnorm(x, None, eps=eps) if fuse_rms else x
    if not fp8:
        vendor_fallback(f"linear {tuple(x.shape)} x {tuple(w.shape)}")
    y = _fp8_matmul(xin, w) if fp8 else torch.matmul(xin, w.t())
    if bias is not None or act != "none" or residual is not None:
        if y.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and y.shape[1] % 8 == 0:
            E.bias_act(y, bias, residual, out, 1 if act == "gelu" else 0)
            return out
        y = y.float()
        if bias is not None:
            y = y + bias.float()
        if act == "gelu":
            y = torch.nn.functional.gelu(y)
        if residual is not None:
            y = y + residual.float()
    out.copy_(y)
    return out


def linear_swiglu(x: torch.Tensor, w_gu: torch.Tensor, *, fuse_rms: bool = False, eps: float = 1e-5,
                  out: Optional[torch.Tensor] = None, ss_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up of the interleaved gate/up projection (ops.interleave_gate_up); ss_in: the
    rows' handed-off sums of squares for the fused RMSNorm (tiled GEMM paths, see ops.gemm)."""
    M = x.shape[0]
    F = w_gu.shape[0] // 2
    if out is None:
        out = torch.empty((M, F), dtype=x.dtype, device=x.device)
    if isinstance(w_gu, TiledWeight):
        if _gpu(x) and _stream_ok(x, w_gu):
            ext().skinny_gemm_swiglu(x, w_gu.t, None, out, fuse_rms, eps, None, True)
            return out
        if _gpu(x) and gemm_ok(x, w_gu, out):
            return gemm(x, w_gu, out, epi="swiglu", fuse_rms=fuse_rms, eps=eps, ss_in=ss_in)
        w_gu = w_gu.dense()
    if not _gpu(x):
        xr, wr, fr = _ref_w8(x, w_gu, fuse_rms, eps)
        return ref.linear_swiglu(xr, wr, fuse_rms=fr, eps=eps, out=out)
    E = ext()
    fp8 = isinstance(w_gu, FP8Weight)
    if M <= SKINNY_MAX_M and (not fp8 or _fp8_stream_fits(M, x.shape[1], nt=2)):
        if fp8:
            E.skinny_gemm_swiglu(x, w_gu.w8, None, out, fuse_rms, eps, w_gu.scale, w_gu.tiled)
        else:
            E.skinny_gemm_swiglu(x, w_gu, None, out, fuse_rms, eps)
        return out
    if fp8 and gemm_fp8_ok(x, w_gu, out):
        return gemm_fp8(x, w_gu, out, epi="swiglu", fuse_rms=fuse_rms, eps=eps, ss_in=ss_in)
    if not fp8 and gemm_ok(x, w_gu, out):
        return gemm(x, w_gu, out, epi="swiglu", fuse_rms=fuse_rms, eps=eps, ss_in=ss_in)
    if fp8 and w_gu.tiled:
        w_gu = FP8Weight(w_gu.rows(), w_gu.scale)
    xin = rmsnorm(x, None, eps=eps) if fuse_rms else x
    if not fp8:
        vendor_fallback(f"linear_swiglu {tuple(x.shape)} x {tuple(w_gu.shape)}")
    gu = _fp8_matmul(xin, w_gu) if fp8 else torch.matmul(xin, w_gu.t())
    E.swiglu(gu, out)
    return out


# > 16-row QKV projections with the rotary + paged-KV write in the tiled GEMM's epilogue (gemm.hip
# EPI_QKV; with split-K: in the slab reduction) -- no qkv scratch round trip, no rope_kv_write
# launch.  VWA_GEMM_QKV=0: GEMM -> qkv scratch -> rope_kv_write
GEMM_QKV_FUSED = knob("VWA_GEMM_QKV")


def _gemm_qkv(x, w, bias, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, rope, positions, slots, q_out, k_cache,
              v_cache, ss_in=None) -> None:
    E = ext()
    M, K = x.shape
    ws = scratch(x.device, "gemm_ws", GEMM_WS_FLOATS)
    common = (n_q_heads, n_kv_heads, head_dim, rope is not None, positions, slots, rope, q_out, k_cache, v_cache)
    if isinstance(w, FP8Weight):
        if M <= FP8_A16_ROWS:  # W8A16 (see gemm_fp8)
            hand = fuse_rms and ss_in is not None
            E.gemm_qkv(x, None, w.w8, w.scale, bias, _rstd(x, eps) if fuse_rms and not hand else None, True, ws,
                       *common, ss_in if hand else None, eps)
            return
        x8, sx, rstd = _fp8_input(x, fuse_rms, eps)
        E.gemm_qkv(x8, sx, w.w8, w.scale, bias, rstd, True, ws, *common)
        return
    hand = fuse_rms and ss_in is not None
    rstd = _rstd(x, eps) if fuse_rms and not hand else None
    tiled = isinstance(w, TiledWeight)
    E.gemm_qkv(x, None, w.t if tiled else w, None, bias, rstd, tiled, ws, *common, ss_in if hand else None, eps)


def qkv_rope_write(x: torch.Tensor, w_qkv: torch.Tensor, bias: Optional[torch.Tensor], *, fuse_rms: bool, eps: float,
                   n_q_heads: int, n_kv_heads: int, head_dim: int, rope: Optional[torch.Tensor],
                   positions: torch.Tensor, slots: torch.Tensor, q_out: torch.Tensor, k_cache: torch.Tensor,
                   v_cache: torch.Tensor, ln_c: Optional[torch.Tensor] = None,
                   ss_in: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused QKV projection + rotary + paged KV write. Returns q_out[:M] (natural layout).
    ln_c: folded LayerNorm on x (see linear).  ss_in: handed-off sums of squares (see ops.gemm)."""
    M = x.shape[0]
    if isinstance(w_qkv, TiledWeight):
        if _gpu(x) and _stream_ok(x, w_qkv) and (ln_c is None or _ln_fold_fits(x, w_qkv)):
            ext().skinny_gemm_qkv(x, w_qkv.t, bias, fuse_rms and ln_c is None, eps, n_q_heads, n_kv_heads, head_dim,
                                  rope is not None, positions, slots, rope, q_out, k_cache, v_cache, None, ln_c, True)
            return q_out[:M]
        if ln_c is not None:
            x, ln_c = _layernorm_plain(x, eps), None
        if _gpu(x) and gemm_ok(x, w_qkv) and GEMM_QKV_FUSED:
            _gemm_qkv(x, w_qkv, bias, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, rope, positions, slots, q_out,
                      k_cache, v_cache, ss_in)
            return q_out[:M]
        if _gpu(x) and gemm_ok(x, w_qkv):
            qkv = scratch(x.device, "qkv", M * w_qkv.shape[0], torch.bfloat16).view(M, w_qkv.shape[0])
            gemm(x, w_qkv, qkv, bias=bias, fuse_rms=fuse_rms, eps=eps)
            ext().rope_kv_write(qkv, n_q_heads, n_kv_heads, head_dim, rope is not None, positions, slots, rope, q_out,
                                k_cache, v_cache)
            return q_out[:M]
        w_qkv = w_qkv.dense()
    if ln_c is not None:
        if _ln_fold_fits(x, w_qkv):
            ext().skinny_gemm_qkv(x, w_qkv, bias, False, eps, n_q_heads, n_kv_heads, head_dim, rope is not None,
                                  positions, slots, rope, q_out, k_cache, v_cache, None, ln_c)
            return q_out[:M]
        x = _layernorm_plain(x, eps)
    if not _gpu(x):
        x, w_qkv, fuse_rms = _ref_w8(x, w_qkv, fuse_rms, eps)
        ref.qkv_rope_write(x, w_qkv, bias, fuse_rms=fuse_rms, eps=eps, n_q_heads=n_q_heads, n_kv_heads=n_kv_heads,
                           head_dim=head_dim, rope=rope, positions=positions, slots=slots, q_out=q_out,
                           k_cache=k_cache, v_cache=v_cache)
        return q_out[:M]
    E = ext()
    use_rope = rope is not None
    fp8 = isinstance(w_qkv, FP8Weight)
    if M > SKINNY_MAX_M and (gemm_fp8_ok(x, w_qkv) if fp8 else gemm_ok(x, w_qkv)) and GEMM_QKV_FUSED:
        _gemm_qkv(x, w_qkv, bias, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, rope, positions, slots, q_out,
                  k_cache, v_cache, ss_in)
        return q_out[:M]
    if M > SKINNY_MAX_M and (gemm_fp8_ok(x, w_qkv) if fp8 else gemm_ok(x, w_qkv)):
        qkv = scratch(x.device, "qkv", M * w_qkv.shape[0], torch.bfloat16).view(M, w_qkv.shape[0])
        (gemm_fp8 if fp8 else gemm)(x, w_qkv, qkv, bias=bias, fuse_rms=fuse_rms, eps=eps)
        E.rope_kv_write(qkv, n_q_heads, n_kv_heads, head_dim, use_rope, positions, slots, rope, q_out, k_cache,
                        v_cache)
        return q_out[:M]
    if M <= SKINNY_MAX_M and (not fp8 or _fp8_stream_fits(M, x.shape[1])):
        if fp8:
            E.skinny_gemm_qkv(x, w_qkv.w8, bias, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, use_rope, positions,
                              slots, rope, q_out, k_cache, v_cache, w_qkv.scale, None, w_qkv.tiled)
        else:
            E.skinny_gemm_qkv(x, w_qkv, bias, fuse_rms, eps, n_q_heads, n_kv_heads, head_dim, use_rope, positions,
                              slots, rope, q_out, k_cache, v_cache)
        return q_out[:M]
    if fp8 and w_qkv.tiled:
        w_qkv = FP8Weight(w_qkv.rows(), w_qkv.scale)
    xin = rmsnorm(x, None, eps=eps) if fuse_rms else x
    if not fp8:
        vendor_fallback(f"qkv {tuple(x.shape)} x {tuple(w_qkv.shape)}")
    qkv = _fp8_matmul(xin, w_qkv) if fp8 else torch.matmul(xin, w_qkv.t())
    if bias is not None:
        qkv = qkv + bias
    E.rope_kv_write(qkv, n_q_heads, n_kv_heads, head_dim, use_rope, positions, slots, rope, q_out, k_cache, v_cache)
    return q_out[:M]


# ----------------------------------------------------------------------------- norms / elementwise
def rmsnorm(x: torch.Tensor, w: Optional[torch.Tensor], *, eps: float = 1e-5, residual: Optional[torch.Tensor] = None,
            residual_out: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if out is None:
        out = torch.empty_like(x)
    if not _gpu(x):
        return ref.rmsnorm(x, w, eps=eps, residual=residual, residual_out=residual_out, out=out)
    ext().rmsnorm(x, residual, residual_out, w, out, eps)
    return out


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, *, eps: float = 1e-5,
              residual: Optional[torch.Tensor] = None, residual_out: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if out is None:
        out = torch.empty_like(x)
    if not _gpu(x):
        return ref.layernorm(x, w, b, eps=eps, residual=residual, residual_out=residual_out, out=out)
    ext().layernorm(x, residual, residual_out, w, b, out, eps)
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, *, pos_table: Optional[torch.Tensor] = None,
              positions: Optional[torch.Tensor] = None, vocab_start: int = 0,
              out: Optional[torch.Tensor] = None, rows: Optional[int] = None) -> torch.Tensor:
    n = rows if rows is not None else ids.shape[0]
    if out is None:
        out = torch.empty((n, table.shape[1]), dtype=table.dtype, device=table.device)
    if not _gpu(table):
        return ref.embedding(ids[:n], table, pos_table=pos_table, positions=None if positions is None else positions[:n],
                             vocab_start=vocab_start, out=out)
    ext().embedding(ids, table, pos_table, positions, out, vocab_start)
    return out


# ----------------------------------------------------------------------------- attention
class KVLayout:
    """Addressing for the attention kernels (see csrc/kernels/vwa_kernels.h KVView)."""

    __slots__ = ("k", "v", "table", "block_size", "sb", "sh", "st")

    def __init__(self, k, v, table, block_size, sb, sh, st):
        self.k, self.v, self.table = k, v, table
        self.block_size, self.sb, self.sh, self.st = int(block_size), int(sb), int(sh), int(st)

    @staticmethod
    def paged(k_cache: torch.Tensor, v_cache: torch.Tensor, block_table: torch.Tensor) -> "KVLayout":
        # [num_blocks, n_kv, bs, hd]
        return KVLayout(k_cache, v_cache, block_table, k_cache.shape[2], k_cache.stride(0), k_cache.stride(1),
                        k_cache.stride(2))

    @staticmethod
    def contiguous(k: torch.Tensor, v: torch.Tensor, table: torch.Tensor) -> "KVLayout":
        # [B, S, H, D]: one block per sequence
        return KVLayout(k, v, table, k.shape[1], k.stride(0), k.stride(2), k.stride(1))


def decode_split_tokens() -> int:
    return 128  # chunk granularity of the decode-attention grid (attention.hip kMqChunk)


ATTENTION_IMPLS = {"split": 0, "mq": 1}


def set_attention_impl(name: str) -> None:
    """Decode-attention kernel: "mq" (multi-query MFMA, default) or "split" (VALU split-K)."""
    ext().set_attention_impl(ATTENTION_IMPLS[name])


_COUNTERS: dict = {}


def split_counters(device, n: int) -> torch.Tensor:
    """Zeroed int32 chunk tickets for decode attention (the kernel leaves them zero).  Engines
    that capture hipGraphs allocate their own (StepBuffers.attn_cnt) before capture."""
    t = _COUNTERS.get(str(device))
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
        _COUNTERS[str(device)] = t
    return t


def chain_buffers(device):
    """(barrier words, bar_mode, work) for one model's chained decode launches
    (skinny_stream.hip chain_kernel): barrier words in L2-uncached memory polled with scalar
    loads (bar_mode 2: the poll does not queue behind the next phase's weight loads), plain
    memory + vector polls (bar_mode 1) if the uncached allocation is unavailable; work = split-tile
    tickets + partial slots.  One set per model: launches sharing a set must be stream-ordered."""
    try:
        bar, mode = ext().alloc_uncached_i32(1024, torch.empty(1, device=device)), 2
        # VWA_CHAIN_BAR_MODE=4: no-return arrivals on the 8 group counters, waiters poll their sum
        # (one scalar round trip) -- the last arrival is not two dependent atomics away from release
        if knob("VWA_CHAIN_BAR_MODE") == 4:
            mode = 4
    except RuntimeError:
        bar, mode = torch.zeros(1024, dtype=torch.int32, device=device), 1
    return bar, mode, torch.zeros(1 << 20, dtype=torch.int32, device=device)


def chain_error_word(bar: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """The device word a timed-out chain barrier sets (skinny_stream.hip chain_wait)."""
    return None if bar is None else bar.view(torch.int64)[160:161]


def decode_n_splits(max_ctx: int) -> int:
    return max(1, -(-int(max_ctx) // decode_split_tokens()))


def decode_attention(q: torch.Tensor, kv: KVLayout, ctx_lens: torch.Tensor, seq_ids: torch.Tensor, *,
                     n_q_heads: int, n_kv_heads: int, head_dim: int, scale: float, max_ctx: int,
                     out: torch.Tensor, part_o: Optional[torch.Tensor] = None,
                     part_ml: Optional[torch.Tensor] = None, counters: Optional[torch.Tensor] = None,
                     shared: Optional[torch.Tensor] = None, n_splits: Optional[int] = None) -> torch.Tensor:
    """One query row per token; ``max_ctx`` bounds every row's context (fixes the grid, so the
    launch is graph-capturable while contexts grow).  ``shared``: int32 [P, n_real] on the device
    (the step buffers' shared-prefix words, runtime/engine.py): the first P keys of rows
    0 .. n_real-1 are the same physical K/V blocks (the cached prompt every session shares), so the
    multi-query kernel reads them once per group of rows across sessions.  ``n_splits`` (tuning
    probes): cap on the key chunks (partial slots) per row group, default max_ctx / 128."""
    n_splits = min(n_splits or 1 << 30, decode_n_splits(max_ctx))
    if not _gpu(q):
        return ref.decode_attention(q, kv, ctx_lens, seq_ids, n_q_heads=n_q_heads, n_kv_heads=n_kv_heads,
                                    head_dim=head_dim, scale=scale, out=out)
    assert ext().attention_split_tokens() == decode_split_tokens()
    if part_o is None:
        rows = q.shape[0]
        part_o = torch.empty((rows * n_splits * n_q_heads * head_dim,), dtype=torch.float32, device=q.device)
        part_ml = torch.empty((rows * n_splits * n_q_heads * 2,), dtype=torch.float32, device=q.device)
    if counters is None:
        counters = split_counters(q.device, q.shape[0] * n_kv_heads)
    ext().decode_attention(q, kv.k, kv.v, kv.table, kv.block_size, kv.sb, kv.sh, kv.st, ctx_lens, seq_ids, n_q_heads,
                           n_kv_heads, head_dim, scale, n_splits, part_o, part_ml, counters, out, shared)
    return out


def decode_attention_rows(q: torch.Tensor, kv: KVLayout, ctx_lens: torch.Tensor, seq_ids: torch.Tensor, *,
                          out: torch.Tensor, slice_rows: int = 64, **kw) -> torch.Tensor:
    """decode_attention over any number of ragged rows (each row: its own sequence and causal
    context): the multi-query MFMA kernel takes <= 64 rows per launch (its row-group scan), so
    longer row sets -- batched admission prefill of several requests' prompt suffixes -- run in
    64-row slices that reuse the same partial buffers (stream-ordered)."""
    M = q.shape[0]
    if M <= slice_rows or not _gpu(q):
        return decode_attention(q, kv, ctx_lens, seq_ids, out=out, **kw)
    kw.pop("shared", None)  # (the shared-prefix words describe the whole row set)
    for i in range(0, M, slice_rows):
        j = min(M, i + slice_rows)
        decode_attention(q[i:j], kv, ctx_lens[i:j], seq_ids[i:j], out=out[i:j], **kw)
    return out


def flash_attention_runs(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, runs, *, n_q_heads: int,
                         n_kv_heads: int, head_dim: int, scale: float, out: torch.Tensor) -> torch.Tensor:
    """Causal attention of ragged rows that are whole per-sequence runs (runtime/engine.py
    _ragged_flash: B runs of <= S consecutive positions, run b at absolute offset q_offsets[b] over
    its own block-table row): scattered into a [B, S] query block, one batched flash-attention
    launch, gathered back.  The padding queries of short runs compute rows nobody reads."""
    B, S, hq = runs.B, runs.S, n_q_heads * head_dim
    qp = scratch(q.device, "runs_q", B * S * hq, q.dtype).view(B * S, hq)
    op = scratch(q.device, "runs_o", B * S * hq, q.dtype).view(B * S, hq)
    qp.index_copy_(0, runs.dst, q)
    flash_attention(qp.view(B, S, n_q_heads, head_dim), KVLayout.paged(k_cache, v_cache, runs.table), Sk=runs.max_k,
                    n_kv_heads=n_kv_heads, causal=True, scale=scale, out=op.view(B, S, n_q_heads, head_dim),
                    k_lens=runs.k_lens, q_offsets=runs.q_offsets)
    return torch.index_select(op, 0, runs.dst, out=out)


def flash_attention(q: torch.Tensor, kv: KVLayout, *, Sk: int, n_kv_heads: int, causal: bool, scale: float,
                    q_offset: int = 0, out: Optional[torch.Tensor] = None,
                    k_lens: Optional[torch.Tensor] = None, q_offsets: Optional[torch.Tensor] = None) -> torch.Tensor:
    """q: [B, Sq, Hq, D]; keys of batch b through kv (table row b)."""
    if out is None:
        out = torch.empty_like(q)
    if not _gpu(q):
        return ref.flash_attention(q, kv, Sk=Sk, n_kv_heads=n_kv_heads, causal=causal, scale=scale,
                                   q_offset=q_offset, out=out, k_lens=k_lens, q_offsets=q_offsets)
    ext().flash_attention(q, kv.k, kv.v, kv.table, kv.block_size, kv.sb, kv.sh, kv.st, out, Sk, n_kv_heads, causal,
                          q_offset, q_offsets, k_lens, scale)
    return out


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, *, mask: Optional[torch.Tensor], temperature: Optional[torch.Tensor],
           seed: torch.Tensor, step: torch.Tensor, out_tokens: torch.Tensor,
           part_val: Optional[torch.Tensor] = None, part_idx: Optional[torch.Tensor] = None,
           n_chunks: int = 64, fail_word: Optional[torch.Tensor] = None, v_offset: int = 0, tp=None) -> torch.Tensor:
    """Masked Gumbel-max sampling (greedy without temperature).  ``fail_word``: a device int64
    that, when nonzero at sampling time, turns every output token into -2 (the chained
    forward's grid-barrier timeout word: the logits of that step are invalid).

    Vocab parallel (``tp`` a TPContext of size > 1): ``logits`` is this rank's shard, column j =
    token ``v_offset + j``; every rank gets the same tokens, equal to what a TP=1 sampler draws
    from the full logits (noise and tie-break use global ids).  On GPU TP groups: partial maxima
    -> one-shot IPC all-gather of [rows, chunks] (value, id) pairs -> merge (sample_tp, no host
    sync, no RCCL); elsewhere the partial maxima are all-gathered with torch.distributed."""
    rows = logits.shape[0]
    if tp is not None and getattr(tp, "size", 1) > 1:
        return _sample_tp(logits, mask=mask, temperature=temperature, seed=seed, step=step, out_tokens=out_tokens,
                          fail_word=fail_word, v_offset=v_offset, tp=tp)
    if not _gpu(logits):
        out = ref.sample(logits, mask=mask, temperature=temperature, seed=seed, step=step, out_tokens=out_tokens,
                         v_offset=v_offset)
        if fail_word is not None and int(fail_word.reshape(-1)[0]) != 0:
            out[:rows] = -2
        return out
    if part_val is None:
        part_val = torch.empty((rows * n_chunks,), dtype=torch.float32, device=logits.device)
        part_idx = torch.empty((rows * n_chunks,), dtype=torch.int32, device=logits.device)
    ext().sample(logits, mask, temperature, seed, step, out_tokens, part_val, part_idx, fail_word, v_offset)
    return out_tokens


def tp_sample_chunks(tp_size: int) -> int:
    """Partial-maximum chunks per row and rank under vocab parallelism (64 over the whole vocab)."""
    return max(8, 64 // max(1, tp_size))


def _sample_tp(logits, *, mask, temperature, seed, step, out_tokens, fail_word, v_offset, tp):
    import torch.distributed as dist

    rows = logits.shape[0]
    car = getattr(tp, "custom_ar", None)
    if _gpu(logits) and car is not None:
        C = tp_sample_chunks(tp.size)
        xin, xout = car.sample_buffers(rows * C * 2, logits.device)
        ext().sample_tp(logits, mask, temperature, seed, step, out_tokens, xin, xout, C, fail_word, v_offset,
                        car.state, tp.size)
        return out_tokens
    vals, idx = ref.sample_partial(logits, mask=mask, temperature=temperature, seed=seed, step=step,
                                   v_offset=v_offset)
    dev = logits.device if (_gpu(logits) and dist.get_backend(tp.group) == "nccl") else torch.device("cpu")
    mine = torch.stack([vals.double(), idx.double()]).to(dev)
    parts = [torch.empty_like(mine) for _ in range(tp.size)]
    dist.all_gather(parts, mine, group=tp.group)
    allv = torch.stack([p[0].cpu() for p in parts])
    alli = torch.stack([p[1].cpu().long() for p in parts])
    toks = ref.merge_partials(allv, alli)
    if fail_word is not None and int(fail_word.reshape(-1)[0]) != 0:
        toks[:] = -2
    out_tokens[:rows] = toks.to(out_tokens.dtype).to(out_tokens.device)
    step.add_(1)
    return out_tokens


# ----------------------------------------------------------------------------- audio
def pcm16_to_f32(pcm: torch.Tensor, in_rate: int = 16000, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    ratio = in_rate / 16000.0
    n_out = int(pcm.numel() / ratio)
    if out is None:
        out = torch.empty((n_out,), dtype=torch.float32, device=pcm.device)
    if not _gpu(pcm):
        return ref.pcm16_to_f32(pcm, ratio, out)
    ext().pcm16_to_f32(pcm, out, ratio)
    return out


_LOGMEL_TABLES: dict = {}


def logmel_tables(mel_fb: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """MFMA fragment-ordered constants of the log-mel kernel (audio.hip logmel_mfma_kernel):
    the DFT basis [26 tiles = 13 bin tiles x (cos, sin)][25][64 lanes][4] with
    basis[T][s4][l][j] = cos|sin(2 pi n b / 400), n = 4 (4 s4 + j) + (l >> 4), b = 16 (T >> 1) + (l & 15)
    (0 for b > 200; exact f64 phase), and the filterbank [n_mels / 16][13][64][4] with
    fbf[t][s4][l][j] = fb[16 t + (l & 15)][4 (4 s4 + j) + (l >> 4)].  Cached per filterbank tensor."""
    key = (mel_fb.data_ptr(), tuple(mel_fb.shape), str(mel_fb.device))
    hit = _LOGMEL_TABLES.get(key)
    if hit is not None:
        return hit[1], hit[2]
    lane = torch.arange(64, dtype=torch.float64)
    ks = (4 * torch.arange(25, dtype=torch.float64)[:, None] + torch.arange(4, dtype=torch.float64)[None, :])  # [25, 4]
    n = 4 * ks[:, None, :] + torch.floor(lane / 16)[None, :, None]  # [25, 64, 4]
    tiles = []
    for bt in range(13):
        b = 16 * bt + (lane % 16)[None, :, None]
        ph = 2 * math.pi * torch.remainder(n * b, 400) / 400
        ok = (b <= 200).to(torch.float64)
        tiles += [torch.cos(ph) * ok, torch.sin(ph) * ok]
    basis = torch.stack(tiles).float().contiguous().to(mel_fb.device)
    n_mels = mel_fb.shape[0]
    mt = (n_mels + 15) // 16
    fb = torch.zeros(mt * 16, 208, dtype=torch.float32)
    fb[:n_mels, :201] = mel_fb.detach().float().cpu()
    l = torch.arange(64)
    kidx = (4 * (4 * torch.arange(13)[:, None, None] + torch.arange(4)[None, None, :]) + (l // 16)[None, :, None])
    fbf = torch.stack([fb[16 * t + (l % 16)[None, :, None], kidx] for t in range(mt)]).contiguous().to(mel_fb.device)
    _LOGMEL_TABLES[key] = (mel_fb, basis, fbf)  # (keeps mel_fb alive: its data_ptr cannot be reused)
    return basis, fbf


def log_mel(audio: torch.Tensor, *, n_frames: int, window: torch.Tensor, mel_fb: torch.Tensor, out: torch.Tensor,
            scratch: Optional[torch.Tensor] = None, max_buf: Optional[torch.Tensor] = None) -> torch.Tensor:
    """audio: padded f32 samples (n_frames*160 for Whisper) -> out bf16 [n_frames, n_mels]."""
    if not _gpu(audio):
        return ref.log_mel(audio, n_frames=n_frames, window=window, mel_fb=mel_fb, out=out)
    n_mels = mel_fb.shape[0]
    if scratch is None:
        scratch = torch.empty((n_frames * n_mels,), dtype=torch.float32, device=audio.device)
    if max_buf is None:
        max_buf = torch.empty((1,), dtype=torch.float32, device=audio.device)
    basis, fbf = logmel_tables(mel_fb)
    ext().log_mel(audio, n_frames, window, basis, fbf, n_mels, scratch, max_buf, out)
    return out


def padded_rows(B: int, T: int, C: int, *, dtype, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """A zero [B, T + 2, C] buffer and its [B, T, C] data view (rows 1..T): the input layout of
    conv1d_gelu (one zero row in front of and behind every batch's rows = the conv's padding)."""
    buf = torch.zeros(B, T + 2, C, dtype=dtype, device=device)
    return buf, buf[:, 1 : T + 1]


def conv_channels(cin: int) -> int:
    """Input channels of the GEMM conv path: 3*C must be a multiple of the GEMM's 128-deep k-group."""
    return (cin + 127) // 128 * 128


def pad_conv_weight(w: torch.Tensor, cp: int) -> torch.Tensor:
    """[Cout, 3*Cin] ((kk, ci) order) -> [Cout, 3*cp] with zero columns for the padded channels."""
    cout, k3 = w.shape
    cin = k3 // 3
    if cin == cp:
        return w.contiguous()
    wp = torch.zeros(cout, 3, cp, dtype=w.dtype, device=w.device)
    wp[:, :, :cin] = w.view(cout, 3, cin)
    return wp.view(cout, 3 * cp)


def conv1d_gelu(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], *, stride: int,
                pos: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                padded: bool = False) -> torch.Tensor:
    """x [B, Tin, Cin] channels-last, w [Cout, 3*Cin] ([co][kk][ci]) -> [B, Tout, Cout] =
    gelu(conv1d(x, k=3, pad=1, stride) + b) (+ pos[:Tout]).

    GPU: a batched implicit GEMM on the tiled MFMA GEMM (gemm.hip).  ``padded=True``: x is the
    data view of a padded_rows buffer with 3*Cin % 128 == 0 (the model's stem buffers: no copy);
    otherwise x is copied into one (channels zero-padded to conv_channels(Cin))."""
    B, Tin, Cin = x.shape
    Tout = (Tin + 2 - 3) // stride + 1
    if out is None:
        out = torch.empty((B, Tout, w.shape[0]), dtype=x.dtype, device=x.device)
    if not _gpu(x):
        return ref.conv1d_gelu(x, plain(w), b, stride=stride, pos=pos, out=out)
    if not padded:
        cp = conv_channels(Cin)
        _, xv = padded_rows(B, Tin, cp, dtype=x.dtype, device=x.device)
        xv[:, :, :Cin] = x
        x, w = xv, pad_conv_weight(plain(w), cp)
    tiled = isinstance(w, TiledWeight)
    ext().conv1d_gelu(x, w.t if tiled else w, b, pos, out, stride, tiled)
    return out


def env_flag(name: str) -> bool:
    """A boolean knob (utils/env.py Settings: declared type and default)."""
    return bool(knob(name))


def env_int(name: str) -> int:
    return int(knob(name))
