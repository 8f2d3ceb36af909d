#include <mutex>
// PyTorch bindings for the gfx950 kernel library.
//
// Every entry point validates shapes/dtypes/devices on the host BEFORE launching (a bad
// shape must never reach a kernel: an out-of-bounds access can reset the whole node), then
// launches on the current HIP stream of the tensor's device -- so each op is capturable in a
// torch.cuda.CUDAGraph (= hipGraph on ROCm).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include "kernels/vwa_kernels.h"

namespace {

using at::Tensor;

// torch-ROCm exposes GPUs as device type "cuda"; the masquerading accessor returns the stream
// torch itself launches on (including the capture stream inside torch.cuda.graph).
hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

const uint16_t* bfp(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
uint16_t* bfp_mut(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const uint16_t* bfp_opt(const c10::optional<Tensor>& t) { return t.has_value() ? bfp(*t) : nullptr; }

void check_bf16(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bf16");
}
void check_contig_rows(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must be row-contiguous");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}
void check_rc(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " launch failed with code ", rc); }

// skinny GEMM dispatch: 1 = persistent streaming kernel when the shape fits (default), 0 = one-tile kernel
int g_skinny_mode = 1;
int g_grid_cap = 256;
int g_ks = 0;  // K-split waves of the streaming kernel; 0 = by shape (skinny_ks)
int g_w_first = 2;  // 0: never, 1: only with the fused RMSNorm prologue, 2: always (measured best)
void set_skinny_mode(int64_t mode, int64_t grid_cap, int64_t ks, int64_t w_first) {
  g_skinny_mode = (int)mode;
  g_grid_cap = (int)grid_cap;
  g_ks = (int)ks;
  g_w_first = (int)w_first;
}
// Small weights (<= g_small_bytes, e.g. every Whisper-tiny projection): the one-tile kernel.
// Measured (tools/bench_kernels.py --only small, M = 1, weights cache-resident as in the ASR
// decode loop): 2.2 vs 4.3 us for 384-1536 wide projections, 3.3 vs 5.0 us for 1280 x 1280.
size_t g_small_bytes = 4u << 20;
void set_small_gemm_bytes(int64_t n) { g_small_bytes = (size_t)(n > 0 ? n : 0); }
// Also every K < 1024: the streaming kernel splits K over its 8 waves in 128-wide groups, so
// with fewer than 8 groups most of its waves idle (Whisper-tiny's 40 MB LM head, K = 384).
// Streaming-kernel K split: 4 waves when K < 2048, else 8.  Its waves take 128-wide k-groups, so
// at K = 1280 (Whisper-large-v3's decoder) 8 waves leave 6 idle in the second round; measured
// (tools/bench_whisper_decode.py, tiled weights, HBM-resident) 6.45 vs 6.83 us for QKV, 8.33 vs
// 8.97 for fc1, 27.9 vs 34.2 for the 133 MB LM head; K >= 4096 (Llama) stays at 8.
// (> 16 rows: the many-row form exists for 8 waves only)
int skinny_ks(const SkinnyParams& p) { return g_ks ? g_ks : (p.K < 2048 && p.M <= 16 ? 4 : 8); }

bool small_gemm(const SkinnyParams& p) {
  return !p.w_scale && g_small_bytes && p.M <= 64 && ((size_t)p.N * p.K * 2 <= g_small_bytes || p.K < 1024);
}

int run_skinny(int epi, const SkinnyParams& p, hipStream_t st) {
  if (g_skinny_mode == 1 && !small_gemm(p)) {
    const int r = vwa_skinny_stream(epi, &p, g_grid_cap, skinny_ks(p), st);
    if (r != -10) return r;
  }
  return vwa_skinny_gemm(epi, &p, st);
}

SkinnyParams base_params(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, bool fuse_rms, double eps,
                         const c10::optional<Tensor>& w_scale = c10::nullopt, bool w_tiled = false) {
  check_bf16(x, "x");
  if (w_scale.has_value()) {
    TORCH_CHECK(w.scalar_type() == at::kFloat8_e4m3fn && w.is_cuda(), "fp8 weights must be float8_e4m3fn on the GPU");
    TORCH_CHECK(w_scale->scalar_type() == at::kFloat && w_scale->is_contiguous() && w_scale->numel() == w.size(0),
                "w_scale must be f32 [N]");
  } else {
    check_bf16(w, "w");
  }
  check_contig_rows(x, "x");
  TORCH_CHECK(w.is_contiguous() && w.dim() == 2, "w must be contiguous [N, K]");
  TORCH_CHECK(x.size(1) == w.size(1), "K mismatch: x ", x.sizes(), " w ", w.sizes());
  // (17..64 rows: the one-tile kernel only, small bf16 weights -- ops._small_rows)
  TORCH_CHECK(x.size(0) >= 1 && x.size(0) <= 64, "skinny_gemm supports 1..64 rows (more: the tiled GEMM), got ", x.size(0));
  TORCH_CHECK(x.size(0) <= 16 || (!w_scale.has_value() && !w_tiled),
              "17..64 rows: bf16 row-major weights (the one-tile kernel) only");
  TORCH_CHECK(w.size(1) % 128 == 0, "K must be a multiple of 128");
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == w.size(0) && bias->is_contiguous(), "bias must be [N]");
  }
  SkinnyParams p{};
  p.X = bfp(x);
  p.ldx = (int)x.stride(0);
  p.W = bfp(w);
  p.M = (int)x.size(0);
  p.N = (int)w.size(0);
  p.K = (int)w.size(1);
  p.bias = bfp_opt(bias);
  p.fuse_rms = fuse_rms ? 1 : 0;
  p.eps = (float)eps;
  p.w_scale = w_scale.has_value() ? w_scale->data_ptr<float>() : nullptr;
  p.w_first = g_w_first == 2 || (g_w_first == 1 && fuse_rms);
  p.w_tiled = w_tiled ? 1 : 0;
  if (w_tiled) TORCH_CHECK(w.size(0) % 16 == 0 && w.size(1) % 128 == 0, "pre-tiled weights need N % 16 == 0, K % 128 == 0");
  // (fp8 + tiled: the fp8 tiled layout, which only the streaming kernel's W8A8 path reads)
  return p;
}

// fp8 weights run only on the streaming kernel; a shape it cannot take is an error, never a
// silent bf16 fallback (the Python layer routes those shapes to the dequantising path).
int run_skinny_checked(int epi, const SkinnyParams& p, hipStream_t st) {
  if (p.M > 16) return vwa_skinny_gemm(epi, &p, st);  // (17..64 rows: the one-tile kernel's MT row tiles)
  // pre-tiled weights (bf16 or fp8) exist only for the streaming kernel (a shape it rejects is an error)
  if (p.w_tiled) return vwa_skinny_stream(epi, &p, g_grid_cap, skinny_ks(p), st);
  if (p.w_scale || (p.fuse_rms == 2 && !small_gemm(p))) return vwa_skinny_stream(epi, &p, g_grid_cap, skinny_ks(p), st);
  return run_skinny(epi, p, st);
}

// Folded LayerNorm (fuse_rms = 2): bf16 weights, <= 16 rows (17..64: the one-tile kernel); runs on the streaming kernel, or on
// the one-tile kernel for the small GEMMs it takes (run_skinny_checked: small_gemm).
void set_ln_fold(SkinnyParams& p, const c10::optional<Tensor>& ln_c, int epi) {
  if (!ln_c.has_value()) return;
  TORCH_CHECK(p.w_scale == nullptr, "folded LayerNorm needs bf16 weights");
  TORCH_CHECK(epi != 2, "folded LayerNorm is not supported with the SwiGLU epilogue");
  TORCH_CHECK(p.M <= 64, "folded LayerNorm takes <= 64 rows (17..64: the one-tile kernel)");
  TORCH_CHECK(ln_c->is_cuda() && ln_c->scalar_type() == at::kFloat && ln_c->is_contiguous() && ln_c->numel() == p.N,
              "ln_c must be f32 [N]");
  p.fuse_rms = 2;
  p.ln_c = ln_c->data_ptr<float>();
}

// epi: 0 store, 1 residual add, 3 gelu
// col_mask (epi 0): int32 token bitmask rows [>= rows_used, words]; column n of y is the mask's bit
// col_mask_off * 32 + n (vocab shard offset under TP) -- tiles without an admissible bit in any of
// the first mask_rows rows are not computed (their y columns are left as they were)
void skinny_gemm(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor y, int64_t epi, bool fuse_rms, double eps,
                 c10::optional<Tensor> residual, c10::optional<Tensor> w_scale, c10::optional<Tensor> ln_c,
                 bool w_tiled, c10::optional<Tensor> col_mask, int64_t col_mask_off, int64_t mask_rows) {
  c10::DeviceGuard g(x.device());
  SkinnyParams p = base_params(x, w, bias, fuse_rms, eps, w_scale, w_tiled);
  TORCH_CHECK(epi == 0 || epi == 1 || epi == 3, "bad epilogue");
  set_ln_fold(p, ln_c, (int)epi);
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1, "y must be a 2-D row-contiguous GPU tensor");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == w.size(0), "y shape mismatch");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 || y.scalar_type() == at::kFloat, "y must be bf16 or f32");
  p.Y = y.data_ptr();
  p.ldy = (int)y.stride(0);
  p.y_f32 = y.scalar_type() == at::kFloat;
  if (epi == 1) {
    TORCH_CHECK(residual.has_value(), "residual epilogue needs residual");
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->dim() == 2 && residual->size(0) == x.size(0) && residual->size(1) == w.size(0) &&
                    residual->stride(1) == 1,
                "residual shape mismatch");
    p.R = bfp(*residual);
    p.ldr = (int)residual->stride(0);
  }
  if (col_mask.has_value()) {
    const Tensor& cm = *col_mask;
    TORCH_CHECK(epi == 0, "col_mask needs the store epilogue");
    TORCH_CHECK((cm.is_cuda() || cm.is_pinned()) && cm.scalar_type() == at::kInt && cm.dim() == 2 &&
                    cm.stride(1) == 1,
                "col_mask must be an int32 [rows, words] GPU or pinned host tensor with contiguous rows");
    TORCH_CHECK(mask_rows >= 1 && mask_rows <= cm.size(0) && col_mask_off >= 0 &&
                    (col_mask_off + (w.size(0) + 31) / 32) <= cm.size(1),
                "col_mask does not cover the output columns");
    p.col_mask = reinterpret_cast<const uint32_t*>(cm.data_ptr<int>()) + col_mask_off;
    p.col_mask_ld = (int)cm.stride(0);
    p.col_mask_rows = (int)mask_rows;
  }
  check_rc(run_skinny_checked((int)epi, p, cur_stream(x)), "skinny_gemm");
}

void skinny_gemm_swiglu(Tensor x, Tensor w_gu, c10::optional<Tensor> bias, Tensor h, bool fuse_rms, double eps,
                        c10::optional<Tensor> w_scale, bool w_tiled) {
  c10::DeviceGuard g(x.device());
  SkinnyParams p = base_params(x, w_gu, bias, fuse_rms, eps, w_scale, w_tiled);
  check_bf16(h, "h");
  TORCH_CHECK(h.dim() == 2 && h.stride(1) == 1 && h.size(0) == x.size(0) && h.size(1) * 2 == w_gu.size(0),
              "h must be [M, N/2]");
  TORCH_CHECK(w_gu.size(0) % 32 == 0, "gate/up rows must be a multiple of 32");
  p.Y = h.data_ptr();
  p.ldy = (int)h.stride(0);
  check_rc(run_skinny_checked(2, p, cur_stream(x)), "skinny_gemm_swiglu");
}

int device_cus(const Tensor& t) {
  static int cached[64] = {0};
  const int d = t.device().index();
  if (d >= 0 && d < 64 && cached[d]) return cached[d];
  int cus = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess, "CU count");
  if (d >= 0 && d < 64) cached[d] = cus;
  return cus;
}

// RMS statistics hand-off of the tiled GEMM (GemmParams::ss_*): ss_out (residual epilogue) gets
// the squares of the output rows added, ss_zero is zeroed (whole tensor), ss_in replaces rstd
void set_ss(GemmParams& p, int64_t epi, const c10::optional<Tensor>& ss_out, const c10::optional<Tensor>& ss_zero,
            const c10::optional<Tensor>& ss_in, double eps) {
  auto chk = [&](const Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kLong && t.is_contiguous() && t.numel() >= p.M, n,
                ": int64 [>= M] contiguous GPU tensor (u64 fixed point, 2^-24 units)");
  };
  if (ss_out.has_value()) {
    chk(*ss_out, "ss_out");
    TORCH_CHECK(epi == 1 && !p.y_f32, "ss_out: residual epilogue (bf16 rows) only");
    p.ss_out = reinterpret_cast<unsigned long long*>(ss_out->data_ptr<int64_t>());
  }
  if (ss_zero.has_value()) {
    chk(*ss_zero, "ss_zero");
    p.ss_zero = reinterpret_cast<unsigned long long*>(ss_zero->data_ptr<int64_t>());
    p.ss_zero_n = (int)ss_zero->numel();
  }
  if (ss_in.has_value()) {
    chk(*ss_in, "ss_in");
    TORCH_CHECK(p.rstd == nullptr, "ss_in replaces rstd");
    p.ss_in = reinterpret_cast<const unsigned long long*>(ss_in->data_ptr<int64_t>());
    p.ss_eps = (float)eps;
  }
}

// LDS-tiled MFMA GEMM (gemm.hip), M > 16 rows.  epi: 0 store (+bias, bf16 / f32 out), 1 residual
// add (+bias), 2 SwiGLU over interleaved gate/up tiles (y [M, N/2]), 3 GELU (+bias).  rstd: f32
// [M] per-row RMSNorm scale applied to the product (gammas folded into w).  ws: f32 split-K
// workspace (the launcher splits K only when the output tiles alone cannot fill the CUs).
void gemm(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor y, int64_t epi, c10::optional<Tensor> rstd,
          c10::optional<Tensor> residual, bool w_tiled, c10::optional<Tensor> ws, c10::optional<Tensor> ss_out,
          c10::optional<Tensor> ss_zero, c10::optional<Tensor> ss_in, double ss_eps) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_contig_rows(x, "x");
  TORCH_CHECK(w.is_contiguous() && w.dim() == 2 && w.size(1) == x.size(1), "w must be contiguous [N, K] with x's K");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm: bad epilogue");
  GemmParams p{};
  p.X = bfp(x);
  p.ldx = (int)x.stride(0);
  p.W = bfp(w);
  p.w_tiled = w_tiled ? 1 : 0;
  p.M = (int)x.size(0);
  p.N = (int)w.size(0);
  p.K = (int)w.size(1);
  TORCH_CHECK(p.N % 16 == 0 && p.K % 128 == 0, "gemm: N % 16 == 0 and K % 128 == 0 required");
  if (epi == 2) TORCH_CHECK(p.N % 32 == 0, "gemm SwiGLU: gate/up rows must be a multiple of 32");
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1 && y.size(0) == p.M &&
                  y.size(1) == (epi == 2 ? p.N / 2 : p.N),
              "y shape");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 || (y.scalar_type() == at::kFloat && epi != 2), "y bf16 (or f32)");
  p.Y = y.data_ptr();
  p.ldy = (int)y.stride(0);
  p.y_f32 = y.scalar_type() == at::kFloat;
  // (bf16 rows leave the kernel as 16-byte chunks)
  TORCH_CHECK(y.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15) == 0,
              "gemm: y rows must be 16-byte aligned");
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == p.N && bias->is_contiguous(), "bias [N]");
    p.bias = bfp(*bias);
  }
  if (epi == 1) {
    TORCH_CHECK(residual.has_value() && residual->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(residual->data_ptr()) & 15) == 0,
                "gemm: residual rows must be 16-byte aligned");
    TORCH_CHECK(residual.has_value(), "residual epilogue needs residual");
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->dim() == 2 && residual->size(0) == p.M && residual->size(1) == p.N &&
                    residual->stride(1) == 1,
                "residual shape");
    TORCH_CHECK(!p.y_f32, "residual epilogue writes bf16");
    p.R = bfp(*residual);
    p.ldr = (int)residual->stride(0);
  }
  if (rstd.has_value()) {
    TORCH_CHECK(rstd->is_cuda() && rstd->scalar_type() == at::kFloat && rstd->numel() >= p.M, "rstd f32 [M]");
    p.rstd = rstd->data_ptr<float>();
  }
  p.splits = 1;
  if (ws.has_value()) {
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == at::kFloat && ws->is_contiguous(), "ws f32");
    p.ws = ws->data_ptr<float>();
    p.splits = vwa_gemm_splits(p.M, p.N, p.K, device_cus(x), ws->numel(), 0);
    p.ws_cap = ws->numel();
  }
  p.cus = device_cus(x);
  set_ss(p, epi, ss_out, ss_zero, ss_in, ss_eps);
  check_rc(vwa_gemm((int)epi, &p, cur_stream(x)), "gemm");
}

// fp8 tiled GEMM (gemm.hip): w8 the fp8 tiled layout [N, K] with per-row scales sw, and either
// x8 OCP e4m3 [M, K] with per-row scales sx (W8A8, quant_fp8_rows) or bf16 rows with sx = None
// (W8A16: the weights convert to bf16 on the LDS read, no quantised copy of x).
void gemm_fp8(Tensor x8, c10::optional<Tensor> sx, Tensor w8, Tensor sw, c10::optional<Tensor> bias, Tensor y,
              int64_t epi, c10::optional<Tensor> rstd, c10::optional<Tensor> residual, c10::optional<Tensor> ws,
              c10::optional<Tensor> ss_out, c10::optional<Tensor> ss_zero, c10::optional<Tensor> ss_in, double ss_eps) {
  c10::DeviceGuard g(x8.device());
  if (sx.has_value()) {
    TORCH_CHECK(x8.is_cuda() && x8.scalar_type() == at::kFloat8_e4m3fn && x8.dim() == 2 && x8.stride(1) == 1 &&
                    x8.stride(0) % 16 == 0 && (reinterpret_cast<uintptr_t>(x8.data_ptr()) & 15) == 0,
                "x8: fp8 e4m3 [M, K] rows 16-byte aligned");
    TORCH_CHECK(sx->is_cuda() && sx->scalar_type() == at::kFloat && sx->numel() >= x8.size(0), "sx f32 [M]");
  } else {
    check_bf16(x8, "x");
    check_contig_rows(x8, "x");
  }
  TORCH_CHECK(w8.is_cuda() && w8.scalar_type() == at::kFloat8_e4m3fn && w8.is_contiguous() && w8.dim() == 2 &&
                  w8.size(1) == x8.size(1),
              "w8: fp8 e4m3 [N, K] (tiled)");
  TORCH_CHECK(sw.is_cuda() && sw.scalar_type() == at::kFloat && sw.numel() == w8.size(0), "sw f32 [N]");
  TORCH_CHECK(epi >= 0 && epi <= 3, "gemm_fp8: bad epilogue");
  GemmParams p{};
  p.X = reinterpret_cast<const uint16_t*>(x8.data_ptr());
  p.ldx = (int)x8.stride(0);
  p.W = reinterpret_cast<const uint16_t*>(w8.data_ptr());
  p.w_tiled = 1;
  p.M = (int)x8.size(0);
  p.N = (int)w8.size(0);
  p.K = (int)w8.size(1);
  TORCH_CHECK(p.N % 16 == 0 && p.K % 128 == 0, "gemm_fp8: N % 16 == 0 and K % 128 == 0 required");
  if (epi == 2) TORCH_CHECK(p.N % 32 == 0, "gemm_fp8 SwiGLU: gate/up rows must be a multiple of 32");
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.stride(1) == 1 && y.size(0) == p.M &&
                  y.size(1) == (epi == 2 ? p.N / 2 : p.N) && y.stride(0) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15) == 0,
              "y shape / alignment");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 || (y.scalar_type() == at::kFloat && epi != 2), "y bf16 (or f32)");
  p.Y = y.data_ptr();
  p.ldy = (int)y.stride(0);
  p.y_f32 = y.scalar_type() == at::kFloat;
  p.sx = sx.has_value() ? sx->data_ptr<float>() : nullptr;
  p.sw = sw.data_ptr<float>();
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == p.N && bias->is_contiguous(), "bias [N]");
    p.bias = bfp(*bias);
  }
  if (epi == 1) {
    TORCH_CHECK(residual.has_value(), "residual epilogue needs residual");
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->dim() == 2 && residual->size(0) == p.M && residual->size(1) == p.N &&
                    residual->stride(1) == 1 && residual->stride(0) % 8 == 0 &&
                    (reinterpret_cast<uintptr_t>(residual->data_ptr()) & 15) == 0 && !p.y_f32,
                "residual shape / alignment");
    p.R = bfp(*residual);
    p.ldr = (int)residual->stride(0);
  }
  if (rstd.has_value()) {
    TORCH_CHECK(rstd->is_cuda() && rstd->scalar_type() == at::kFloat && rstd->numel() >= p.M, "rstd f32 [M]");
    p.rstd = rstd->data_ptr<float>();
  }
  p.splits = 1;
  if (ws.has_value()) {
    TORCH_CHECK(ws->is_cuda() && ws->scalar_type() == at::kFloat && ws->is_contiguous(), "ws f32");
    p.ws = ws->data_ptr<float>();
    p.splits = vwa_gemm_splits(p.M, p.N, p.K, device_cus(x8), ws->numel(), 1);
    p.ws_cap = ws->numel();
  }
  p.cus = device_cus(x8);
  TORCH_CHECK(!ss_in.has_value() || !sx.has_value(), "ss_in: W8A16 (bf16 x) only");
  set_ss(p, epi, ss_out, ss_zero, ss_in, ss_eps);
  check_rc(vwa_gemm((int)epi, &p, cur_stream(x8)), "gemm_fp8");
}

void check_cache(const Tensor& c, const char* name);

// QKV projection on the tiled GEMM with the rotary + paged-KV write in its epilogue (gemm.hip
// EPI_QKV; > 16 rows): x bf16 (sx null) or fp8 codes x8 with per-row scales sx (W8A8); w bf16 or
// fp8 tiled with row scales sw (bf16 x + sw: W8A16).  Replaces gemm -> qkv scratch -> rope_kv_write.
void gemm_qkv(Tensor x, c10::optional<Tensor> sx, Tensor w, c10::optional<Tensor> sw, c10::optional<Tensor> bias,
              c10::optional<Tensor> rstd, bool w_tiled, Tensor ws, int64_t n_q_heads,
              int64_t n_kv_heads, int64_t head_dim, bool use_rope, Tensor positions, Tensor slots,
              c10::optional<Tensor> rope, Tensor q_out, Tensor k_cache, Tensor v_cache, c10::optional<Tensor> ss_in,
              double ss_eps) {
  c10::DeviceGuard g(x.device());
  const bool f8 = sx.has_value();
  GemmParams p{};
  if (!f8 && sw.has_value()) {  // W8A16
    check_bf16(x, "x");
    check_contig_rows(x, "x");
    TORCH_CHECK(w.scalar_type() == at::kFloat8_e4m3fn && w_tiled, "W8A16: fp8 tiled w");
    TORCH_CHECK(sw->scalar_type() == at::kFloat && sw->numel() == w.size(0), "sw f32 [N]");
    p.sw = sw->data_ptr<float>();
  } else if (f8) {
    TORCH_CHECK(x.scalar_type() == at::kFloat8_e4m3fn && x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 16 == 0 &&
                    (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0,
                "x8: fp8 e4m3 [M, K] rows 16-byte aligned");
    TORCH_CHECK(sw.has_value() && w.scalar_type() == at::kFloat8_e4m3fn && w_tiled, "W8A8: fp8 tiled w + scales");
    TORCH_CHECK(sx->scalar_type() == at::kFloat && sx->numel() >= x.size(0), "sx f32 [M]");
    TORCH_CHECK(sw->scalar_type() == at::kFloat && sw->numel() == w.size(0), "sw f32 [N]");
    p.sx = sx->data_ptr<float>();
    p.sw = sw->data_ptr<float>();
  } else {
    check_bf16(x, "x");
    check_contig_rows(x, "x");
    check_bf16(w, "w");
  }
  TORCH_CHECK(w.is_contiguous() && w.dim() == 2 && w.size(1) == x.size(1), "w [N, K] with x's K");
  p.X = reinterpret_cast<const uint16_t*>(x.data_ptr());
  p.ldx = (int)x.stride(0);
  p.W = reinterpret_cast<const uint16_t*>(w.data_ptr());
  p.w_tiled = w_tiled ? 1 : 0;
  p.M = (int)x.size(0);
  p.N = (int)w.size(0);
  p.K = (int)w.size(1);
  TORCH_CHECK(p.N == (n_q_heads + 2 * n_kv_heads) * head_dim && head_dim % 16 == 0 && p.K % 128 == 0, "qkv shape");
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(bias->numel() == p.N && bias->is_contiguous(), "bias [N]");
    p.bias = bfp(*bias);
  }
  if (rstd.has_value()) {
    TORCH_CHECK(rstd->is_cuda() && rstd->scalar_type() == at::kFloat && rstd->numel() >= p.M, "rstd f32 [M]");
    p.rstd = rstd->data_ptr<float>();
  }
  TORCH_CHECK(positions.scalar_type() == at::kInt && positions.numel() >= p.M, "positions");
  TORCH_CHECK(slots.scalar_type() == at::kLong && slots.numel() >= p.M, "slots");
  TORCH_CHECK(q_out.dim() == 2 && q_out.size(0) >= p.M && q_out.size(1) == n_q_heads * head_dim && q_out.stride(1) == 1 &&
                  q_out.stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(q_out.data_ptr()) & 15) == 0,
              "q_out rows 16-byte aligned");
  check_cache(k_cache, "k_cache");
  check_cache(v_cache, "v_cache");
  TORCH_CHECK(k_cache.stride(0) % 8 == 0 && k_cache.stride(1) % 8 == 0 && k_cache.stride(2) % 8 == 0 &&
                  k_cache.strides() == v_cache.strides() && (reinterpret_cast<uintptr_t>(k_cache.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(v_cache.data_ptr()) & 15) == 0,
              "caches: 16-byte aligned token rows");
  if (use_rope) TORCH_CHECK(rope.has_value() && rope->scalar_type() == at::kFloat && rope->is_contiguous(), "rope table");
  p.n_q_heads = (int)n_q_heads;
  p.n_kv_heads = (int)n_kv_heads;
  p.head_dim = (int)head_dim;
  p.use_rope = use_rope ? 1 : 0;
  p.positions = positions.data_ptr<int>();
  p.slots = slots.data_ptr<int64_t>();
  p.rope = use_rope ? rope->data_ptr<float>() : nullptr;
  p.q_out = bfp_mut(q_out);
  p.ldq = (int)q_out.stride(0);
  p.k_cache = bfp_mut(k_cache);
  p.v_cache = bfp_mut(v_cache);
  p.block_size = (int)k_cache.size(2);
  p.cache_sb = k_cache.stride(0);
  p.cache_sh = k_cache.stride(1);
  p.cache_st = k_cache.stride(2);
  TORCH_CHECK(ws.is_cuda() && ws.scalar_type() == at::kFloat && ws.is_contiguous(), "ws f32");
  p.ws = ws.data_ptr<float>();
  p.splits = vwa_gemm_splits(p.M, p.N, p.K, device_cus(x), ws.numel(), p.sw ? 1 : 0);
  p.ws_cap = ws.numel();
  p.cus = device_cus(x);
  TORCH_CHECK(!ss_in.has_value() || !f8, "ss_in: bf16 x only");
  set_ss(p, 5, c10::nullopt, c10::nullopt, ss_in, ss_eps);
  check_rc(vwa_gemm(5, &p, cur_stream(x)), "gemm_qkv");
}

void row_rstd(Tensor x, Tensor rstd, double eps) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_contig_rows(x, "x");
  TORCH_CHECK(rstd.is_cuda() && rstd.scalar_type() == at::kFloat && rstd.numel() >= x.size(0), "rstd f32 [M]");
  check_rc(vwa_row_rstd(bfp(x), (int)x.stride(0), (int)x.size(0), (int)x.size(1), (float)eps, rstd.data_ptr<float>(),
                        cur_stream(x)),
           "row_rstd");
}

void check_cache(const Tensor& c, const char* name) {
  check_bf16(c, name);
  // any block / head / token strides (the kernels address by stride), contiguous head_dim rows
  TORCH_CHECK(c.dim() == 4 && c.stride(3) == 1 && c.stride(0) > 0 && c.stride(1) > 0 && c.stride(2) > 0, name,
              " must be [blocks, kv_heads, block_size, head_dim] with contiguous head_dim rows");
}

// QKV epilogue operands (RoPE table, positions, paged-KV slots and cache strides) into p
void set_qkv_epilogue(SkinnyParams& p, const Tensor& w_qkv, int64_t n_q_heads, int64_t n_kv_heads, int64_t head_dim,
                      bool use_rope, const Tensor& positions, const Tensor& slots, const c10::optional<Tensor>& rope,
                      const Tensor& q_out, const Tensor& k_cache, const Tensor& v_cache) {
  TORCH_CHECK(w_qkv.size(0) == (n_q_heads + 2 * n_kv_heads) * head_dim, "w_qkv rows mismatch");
  TORCH_CHECK(head_dim % 16 == 0, "head_dim must be a multiple of 16");
  TORCH_CHECK(positions.is_cuda() && positions.scalar_type() == at::kInt && positions.numel() >= p.M,
              "positions int32 [M]");
  TORCH_CHECK(slots.is_cuda() && slots.scalar_type() == at::kLong && slots.numel() >= p.M, "slots int64 [M]");
  check_bf16(q_out, "q_out");
  TORCH_CHECK(q_out.dim() == 2 && q_out.size(0) >= p.M && q_out.size(1) == n_q_heads * head_dim, "q_out shape");
  check_cache(k_cache, "k_cache");
  check_cache(v_cache, "v_cache");
  TORCH_CHECK(k_cache.size(1) == n_kv_heads && k_cache.size(3) == head_dim, "cache shape mismatch");
  if (use_rope) {
    TORCH_CHECK(rope.has_value() && rope->scalar_type() == at::kFloat && rope->is_contiguous(), "rope table f32");
    TORCH_CHECK(rope->size(-2) == head_dim / 2, "rope table must be [max_pos, head_dim/2, 2]");
  }
  p.n_q_heads = (int)n_q_heads;
  p.n_kv_heads = (int)n_kv_heads;
  p.head_dim = (int)head_dim;
  p.use_rope = use_rope ? 1 : 0;
  p.positions = positions.data_ptr<int>();
  p.slots = slots.data_ptr<int64_t>();
  p.rope = use_rope ? rope->data_ptr<float>() : nullptr;
  p.q_out = bfp_mut(q_out);
  p.ldq = (int)q_out.stride(0);
  p.k_cache = bfp_mut(k_cache);
  p.v_cache = bfp_mut(v_cache);
  p.block_size = (int)k_cache.size(2);
  p.cache_stride_block = k_cache.stride(0);
  p.cache_stride_head = k_cache.stride(1);
  p.cache_stride_tok = k_cache.stride(2);
}

void skinny_gemm_qkv(Tensor x, Tensor w_qkv, c10::optional<Tensor> bias, bool fuse_rms, double eps, int64_t n_q_heads,
                     int64_t n_kv_heads, int64_t head_dim, bool use_rope, Tensor positions, Tensor slots,
                     c10::optional<Tensor> rope, Tensor q_out, Tensor k_cache, Tensor v_cache,
                     c10::optional<Tensor> w_scale, c10::optional<Tensor> ln_c, bool w_tiled) {
  c10::DeviceGuard g(x.device());
  SkinnyParams p = base_params(x, w_qkv, bias, fuse_rms, eps, w_scale, w_tiled);
  set_ln_fold(p, ln_c, 4);
  set_qkv_epilogue(p, w_qkv, n_q_heads, n_kv_heads, head_dim, use_rope, positions, slots, rope, q_out, k_cache,
                   v_cache);
  check_rc(run_skinny_checked(4, p, cur_stream(x)), "skinny_gemm_qkv");
}

// Workgroups of a chained launch: one per CU, or CUs / VWA_CHAIN_GRID_DIV when several processes
// share one GPU (the two-rank tensor-parallel test on a single device: both ranks' persistent
// launches must be resident at once, or their in-launch rounds wait for each other until the
// bounded spin gives up)
int chain_grid(int dev) {
  int cus = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess, "CU count");
  const char* e = std::getenv("VWA_CHAIN_GRID_DIV");
  const int div = e ? std::atoi(e) : 1;
  return div > 1 ? cus / div : cus;
}

// Chained-launch schedule (ChainParams): the measured-best settings of the round-2 A/B runs
// (profiles/r2_*): two weight items issued ahead of each barrier, phase 1's item 0 in the free
// register set of a one-item phase 0, X staged by one wave with LDS-DMA, o_proj units only on
// workgroups without an attention item, LDS items for phases 1 and 2, attention -> o_proj
// hand-off by completion count.
void chain_schedule(ChainParams& cp) {
  cp.pre2 = 1;
  cp.next0 = 1;
  cp.xdma = 1;
  cp.osub = 1;
  cp.lds_item_req = 1;
  cp.lds_item2_req = 1;
  cp.attn_flag = 1;
  // round 5 (profiles/r5_chain_xwait.md): nothing but the X pieces in a CU's memory queue until X is
  // in LDS -- chained layer 103.2-103.6 vs 105.6 us, bench GPU wait 3462-3471 vs 3558 us per step
  cp.xfirst = 1;
  cp.xwait = 1;
  // o_proj in 32-column tiles: one epilogue per workgroup (1 row 102.3 / 102.1 vs 103.5 / 103.0 us,
  // 4 rows 107.0 vs 107.5 us per layer, profiles/r5_chain_o_nt2.jsonl)
  cp.o_nt2 = 1;
  // 5..16 rows: the X-streaming down projection in 32-column tiles, half the X bytes per weight
  // byte -- 8 / 13 / 16 rows 107.8 / 113.8 / 117.1 vs 110.4 / 119.0 / 125.4 us per layer
  // (profiles/r5_chain_d_nt2.jsonl)
  cp.d_nt2 = 1;
  // the QKV phase's two items go out at the down -> QKV barrier (half the workgroups take two of its
  // 384 tiles): 100.96 / 100.84 vs 101.38 / 101.57 us (profiles/r5_chain_pre_mask.jsonl)
  cp.pre_mask = 8;
  // round 6 schedule options, all measured no better than the defaults: the
  // multi-layer launch's QKV -> next-attention hand-off by per-kv-group counters instead of the
  // grid barrier, a K/V prefetch while the attention workgroups wait, and (fp8) gate/up's item 0
  // issued by the attention workgroups during their attention
  cp.qkv_flags = 0;  // (per-kv-group counters measured 99.5 -> 100.9 us per layer: the barrier stays)
  cp.kv_prefetch = 0;  // (neutral: 99.47 vs 99.53 us per layer, profiles/r6_chain_multi_variants.jsonl)
  cp.attn_pre = 0;  // (fp8 chain: 2503.7 vs 2471.6 us GPU wait per step with it, bench.py --dtype fp8)
  // diagnostic override of the schedule (tools/chain_probe.py A/B runs): "name=value,..."
  if (const char* e = std::getenv("VWA_CHAIN_SCHED")) {
    std::string s(e);
    size_t at = 0;
    while (at < s.size()) {
      const size_t comma = s.find(',', at), eq = s.find('=', at);
      const size_t end = comma == std::string::npos ? s.size() : comma;
      if (eq != std::string::npos && eq < end) {
        const std::string k = s.substr(at, eq - at);
        const int v = std::atoi(s.substr(eq + 1, end - eq - 1).c_str());
        if (k == "pre2") cp.pre2 = v;
        else if (k == "next0") cp.next0 = v;
        else if (k == "xdma") cp.xdma = v;
        else if (k == "osub") cp.osub = v;
        else if (k == "lds1") cp.lds_item_req = v;
        else if (k == "lds2") cp.lds_item2_req = v;
        else if (k == "aflag") cp.attn_flag = v;
        else if (k == "pre_mask") cp.pre_mask = v;
        else if (k == "pre_waves") cp.pre_waves = v;
        else if (k == "xfirst") cp.xfirst = v;
        else if (k == "xwait") cp.xwait = v;
        else if (k == "xw_late") cp.xw_late = v;
        else if (k == "poll_free") cp.poll_free = v;
        else if (k == "o_nt2") cp.o_nt2 = v;
        else if (k == "d_nt2") cp.d_nt2 = v;
        else if (k == "qkv_flags") cp.qkv_flags = v;
        else if (k == "kv_pf") cp.kv_prefetch = v;
        else if (k == "attn_pre") cp.attn_pre = v;
      }
      at = end + 1;
    }
  }
}

// ---- chained decode layer tail (skinny_stream.hip, vwa_chain_*): descriptor built once on the
// host and copied to a device tensor (graph replays then only launch); M <= 4, bf16, one GPU.
void set_resid(SkinnyParams& p, const Tensor& h) {
  p.Y = h.data_ptr();
  p.ldy = (int)h.stride(0);
  p.R = bfp(h);
  p.ldr = (int)h.stride(0);
}

DecodeAttnParams decode_params(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& table,
                               int64_t block_size, int64_t sb, int64_t sh, int64_t stok, const Tensor& ctx_lens,
                               const Tensor& seq_ids, int64_t n_q_heads, int64_t n_kv_heads, int64_t head_dim,
                               double scale, int64_t n_splits, const Tensor& part_o, const Tensor& part_ml,
                               const Tensor& counters, const Tensor& out);

// Returns (descriptor uint8 tensor, dynamic LDS bytes); descriptor is empty when the shapes do
// not fit the chain (the caller keeps the per-kernel path).
std::tuple<Tensor, int64_t> chain_make(Tensor h, Tensor att, Tensor act, Tensor w_o, Tensor w_gu, Tensor w_down,
                                       double eps, c10::optional<Tensor> w_qkv, int64_t n_q_heads, int64_t n_kv_heads,
                                       int64_t head_dim, c10::optional<Tensor> positions, c10::optional<Tensor> slots,
                                       c10::optional<Tensor> rope, c10::optional<Tensor> q_out,
                                       c10::optional<Tensor> k_cache, c10::optional<Tensor> v_cache, Tensor bar,
                                       Tensor work, c10::optional<Tensor> ts, int64_t bar_mode,
                                       c10::optional<Tensor> a_q, c10::optional<Tensor> a_k, c10::optional<Tensor> a_v,
                                       c10::optional<Tensor> a_table, int64_t a_block_size, int64_t a_sb, int64_t a_sh,
                                       int64_t a_st, c10::optional<Tensor> a_ctx, c10::optional<Tensor> a_seq,
                                       double a_scale, int64_t a_n_splits, c10::optional<Tensor> a_part_o,
                                       c10::optional<Tensor> a_part_ml, c10::optional<Tensor> a_counters,
                                       bool w_tiled, c10::optional<Tensor> a_row_table,
                                       c10::optional<Tensor> s_o, c10::optional<Tensor> s_gu,
                                       c10::optional<Tensor> s_down, c10::optional<Tensor> s_qkv, int64_t tp_ar,
                                       c10::optional<Tensor> a_plan, int64_t a_plan_mode) {
  c10::DeviceGuard g(h.device());
  const int64_t M = h.size(0);
  TORCH_CHECK(att.size(0) == M && act.size(0) == M, "row counts differ");
  TORCH_CHECK(act.size(1) * 2 == w_gu.size(0) && w_gu.size(0) % 32 == 0, "act must be [M, gate_up rows / 2]");
  TORCH_CHECK(w_down.size(1) == act.size(1) && w_down.size(0) == h.size(1) && w_o.size(0) == h.size(1),
              "down / o_proj shapes");
  TORCH_CHECK(bar.is_cuda() && bar.scalar_type() == at::kInt && bar.numel() >= 384 && bar.is_contiguous() &&
                  (reinterpret_cast<uintptr_t>(bar.data_ptr()) & 127) == 0,
              "bar must be a 128-byte aligned int32[>=384] on the GPU");
  ChainParams cp{};
  // s_*: per-row scales of fp8 tiled weights (ops.tile_weight_fp8) -> the W8A16 chain
  TORCH_CHECK(s_o.has_value() == s_gu.has_value() && s_o.has_value() == s_down.has_value() &&
                  (!w_qkv.has_value() || s_qkv.has_value() == s_o.has_value()),
              "fp8 chain: every phase's weight needs its scales");
  TORCH_CHECK(!s_o.has_value() || w_tiled, "fp8 chain: tiled fp8 weights only");
  cp.ph[0].p = base_params(att, w_o, c10::nullopt, false, eps, s_o, w_tiled);
  cp.ph[0].epi = 1;
  set_resid(cp.ph[0].p, h);
  cp.ph[1].p = base_params(h, w_gu, c10::nullopt, true, eps, s_gu, w_tiled);
  cp.ph[1].epi = 2;
  check_bf16(act, "act");
  TORCH_CHECK(act.stride(1) == 1, "act rows must be contiguous");
  cp.ph[1].p.Y = act.data_ptr();
  cp.ph[1].p.ldy = (int)act.stride(0);
  cp.ph[2].p = base_params(act, w_down, c10::nullopt, false, eps, s_down, w_tiled);
  cp.ph[2].epi = 1;
  set_resid(cp.ph[2].p, h);
  cp.n = 3;
  cp.seq = 0;
  chain_schedule(cp);
  if (bar.numel() < 640) cp.qkv_flags = 0;  // (the per-group QKV counters live up to u64 word 304)
  if (w_qkv.has_value()) {
    TORCH_CHECK(positions.has_value() && slots.has_value() && q_out.has_value() && k_cache.has_value() &&
                    v_cache.has_value(),
                "the QKV phase needs positions, slots, q_out and the KV caches");
    cp.ph[3].p = base_params(h, *w_qkv, c10::nullopt, true, eps, s_qkv, w_tiled);
    cp.ph[3].epi = 4;
    set_qkv_epilogue(cp.ph[3].p, *w_qkv, n_q_heads, n_kv_heads, head_dim, rope.has_value(), *positions, *slots, rope,
                     *q_out, *k_cache, *v_cache);
    cp.n = 4;
  }
  if (tp_ar) {
    // tensor parallel (o_proj / down row-parallel): the two phases write this rank's f32 partial
    // rows into its chain regions, the in-launch rounds all-reduce them into h (chain_tp_reduce)
    TORCH_CHECK(vwa_ar_chain_tp(reinterpret_cast<void*>(tp_ar), &cp.tp) == 0, "chain TP: peers not mapped");
    TORCH_CHECK(h.stride(1) == 1 && M * h.size(1) <= cp.tp.region, "chain TP: rows exceed the chain region");
    for (int i : {0, 2}) {
      SkinnyParams& q = cp.ph[i].p;
      q.Y = cp.tp.stage[cp.tp.rank] + (i == 2 ? cp.tp.region : 0);
      q.y_f32 = 1;
      q.ldy = (int)h.size(1);
      q.R = nullptr;
    }
  }
  cp.bar = reinterpret_cast<unsigned*>(bar.data_ptr<int>());
  cp.bar_mode = (int)bar_mode;
  // work: [0, 8192) u32 split-tile tickets (zeroed, self-resetting) | f32 partial slots
  TORCH_CHECK(work.is_cuda() && work.scalar_type() == at::kInt && work.is_contiguous() && work.numel() > 8192 + 4096,
              "work must be a zeroed int32 GPU tensor of > 12288 elements");
  cp.tickets = reinterpret_cast<unsigned*>(work.data_ptr<int>());
  cp.max_tiles = 8192;
  cp.part = reinterpret_cast<float*>(work.data_ptr<int>() + 8192);
  cp.part_floats = (int)(work.numel() - 8192);
  if (ts.has_value()) {
    TORCH_CHECK(ts->is_cuda() && ts->scalar_type() == at::kLong && ts->numel() >= 1024 * 64, "ts must be int64[>=65536] (64 stamp slots per workgroup)");
    cp.ts = reinterpret_cast<unsigned long long*>(ts->data_ptr<int64_t>());
  }
  if (a_q.has_value()) {  // decode attention as the launch's first phase (its output is `att`)
    TORCH_CHECK(a_k && a_v && a_table && a_ctx && a_seq && a_part_o && a_part_ml && a_counters,
                "attention phase: every a_* tensor is required");
    TORCH_CHECK(head_dim == 128 && (n_q_heads / n_kv_heads == 4 || n_q_heads / n_kv_heads == 8) &&
                    n_q_heads % n_kv_heads == 0 && a_q->size(0) == M && M <= 64,
                "attention phase: head_dim 128, GQA group 4 or 8, one query row per chained row");
    cp.attn = decode_params(*a_q, *a_k, *a_v, *a_table, a_block_size, a_sb, a_sh, a_st, *a_ctx, *a_seq, n_q_heads,
                            n_kv_heads, head_dim, a_scale, a_n_splits, *a_part_o, *a_part_ml, *a_counters, att);
    TORCH_CHECK(a_n_splits > 1, "attention phase: the in-launch chunk merge needs n_splits > 1");
    cp.attn_g = (int)(n_q_heads / n_kv_heads);
    TORCH_CHECK(a_row_table.has_value(), "attention phase: a_row_table (per-row block tables) is required");
    TORCH_CHECK(a_block_size == 16, "attention phase: 16-token KV blocks (mq_attention.h FINE addressing)");
    {
      const Tensor& rtab = *a_row_table;
      TORCH_CHECK(rtab.is_cuda() && rtab.scalar_type() == at::kInt && rtab.dim() == 2 && rtab.is_contiguous() &&
                      rtab.size(0) >= M && rtab.size(1) <= 128 && rtab.size(1) % 2 == 0,
                  "a_row_table must be int32 [>= rows, <= 128 (even)] contiguous");
      cp.attn.row_table = rtab.data_ptr<int>();
      cp.attn.rt_stride = (int)rtab.size(1);
    }
    // step plan of the attention partition (mq_attention.h): layer 0 writes it, layers 1.. read it
    if (a_plan_mode) {
      TORCH_CHECK(a_plan_mode == 1 || a_plan_mode == 2, "a_plan_mode: 1 write, 2 read");
      TORCH_CHECK(a_plan.has_value() && a_plan->is_cuda() && a_plan->scalar_type() == at::kInt && a_plan->is_contiguous() &&
                      a_plan->numel() >= (int64_t)chain_grid(h.device().index()) * 16,
                  "a_plan must be int32 [>= grid * 16] on the GPU");
      cp.attn.plan = a_plan->data_ptr<int>();
      cp.attn.plan_mode = (int)a_plan_mode;
    }
  }
  const int lds = vwa_chain_prepare(&cp, chain_grid(h.device().index()));
  if (lds < 0) return {torch::empty({0}, torch::dtype(torch::kUInt8).device(h.device())), 0};
  Tensor host = torch::empty({(int64_t)sizeof(ChainParams)}, torch::dtype(torch::kUInt8));
  std::memcpy(host.data_ptr(), &cp, sizeof(ChainParams));
  // (bit 24 of the returned LDS size: the down phase streams X with the weights, bit 25: fp8
  // weights, bit 26: o_proj in 32-column tiles -- chain_run launches that instantiation)
  return {host.to(h.device()), (int64_t)lds | (cp.n >= 3 && cp.ph[2].xg ? (int64_t)1 << 24 : 0) |
                                    (cp.d_nt2 ? (int64_t)1 << 27 : 0) |
                                    (s_o.has_value() ? (int64_t)1 << 25 : 0) | (cp.o_nt2 ? (int64_t)1 << 26 : 0)};
}

// Whisper decoder chains (skinny_stream.hip chain_kernel SEQ 1 / 2): phase i computes
// Y[i] (=|+=) X[i] . W[i]^T + bias[i] with the epilogue epi[i] (0 store, 1 residual into Y, 3 GELU,
// 4 QKV + self-KV write, no RoPE); ln_c[i] set = LayerNorm folded into W[i] (fuse_rms 2).
std::tuple<Tensor, int64_t> chain_make_seq(int64_t seq, std::vector<Tensor> X, std::vector<Tensor> W,
                                           std::vector<c10::optional<Tensor>> bias,
                                           std::vector<c10::optional<Tensor>> ln_c, std::vector<Tensor> Y,
                                           std::vector<int64_t> epi, double eps, int64_t n_heads, int64_t head_dim,
                                           c10::optional<Tensor> positions, c10::optional<Tensor> slots,
                                           c10::optional<Tensor> k_cache, c10::optional<Tensor> v_cache, Tensor bar,
                                           Tensor work, int64_t bar_mode, bool w_tiled) {
  const size_t n = X.size();
  TORCH_CHECK(n >= 2 && n <= (size_t)kChainMaxPhases && W.size() == n && bias.size() == n && ln_c.size() == n &&
                  Y.size() == n && epi.size() == n,
              "chain_make_seq: one X/W/bias/ln_c/Y/epi per phase");
  TORCH_CHECK(seq == 1 || seq == 2, "chain_make_seq: seq 1 (Whisper tail) or 2 (Whisper middle)");
  c10::DeviceGuard g(X[0].device());
  TORCH_CHECK(bar.is_cuda() && bar.scalar_type() == at::kInt && bar.numel() >= 384 && bar.is_contiguous() &&
                  (reinterpret_cast<uintptr_t>(bar.data_ptr()) & 127) == 0,
              "bar must be a 128-byte aligned int32[>=384] on the GPU");
  TORCH_CHECK(work.is_cuda() && work.scalar_type() == at::kInt && work.is_contiguous() && work.numel() > 8192 + 4096,
              "work must be a zeroed int32 GPU tensor of > 12288 elements");
  ChainParams cp{};
  const int64_t M = X[0].size(0);
  for (size_t i = 0; i < n; ++i) {
    TORCH_CHECK(X[i].size(0) == M && Y[i].size(0) == M, "row counts differ");
    SkinnyParams& p = cp.ph[i].p;
    p = base_params(X[i], W[i], bias[i], false, eps, c10::nullopt, w_tiled);
    cp.ph[i].epi = (int)epi[i];
    set_ln_fold(p, ln_c[i], (int)epi[i]);
    if (epi[i] == 4) {
      TORCH_CHECK(positions && slots && k_cache && v_cache, "the QKV phase needs positions, slots and the KV caches");
      set_qkv_epilogue(p, W[i], n_heads, n_heads, head_dim, false, *positions, *slots, c10::nullopt, Y[i], *k_cache,
                       *v_cache);
      continue;
    }
    check_bf16(Y[i], "Y");
    TORCH_CHECK(Y[i].dim() == 2 && Y[i].stride(1) == 1 && Y[i].size(1) == W[i].size(0), "Y must be [M, N] rows");
    if (epi[i] == 1) {
      set_resid(p, Y[i]);
    } else {
      p.Y = Y[i].data_ptr();
      p.ldy = (int)Y[i].stride(0);
    }
  }
  cp.n = (int)n;
  cp.seq = (int)seq;
  cp.pre2 = 1;  // (the Llama schedule without its attention-phase and LDS-item parts)
  cp.next0 = 1;
  cp.xdma = 1;
  cp.osub = 1;
  cp.bar = reinterpret_cast<unsigned*>(bar.data_ptr<int>());
  cp.bar_mode = (int)bar_mode;
  cp.tickets = reinterpret_cast<unsigned*>(work.data_ptr<int>());
  cp.max_tiles = 8192;
  cp.part = reinterpret_cast<float*>(work.data_ptr<int>() + 8192);
  cp.part_floats = (int)(work.numel() - 8192);
  const int lds = vwa_chain_prepare(&cp, chain_grid(X[0].device().index()));
  if (lds < 0) return {torch::empty({0}, torch::dtype(torch::kUInt8).device(X[0].device())), 0};
  Tensor host = torch::empty({(int64_t)sizeof(ChainParams)}, torch::dtype(torch::kUInt8));
  std::memcpy(host.data_ptr(), &cp, sizeof(ChainParams));
  return {host.to(X[0].device()), (int64_t)lds};
}

// One-row device-resident decode loop step (see elementwise.hip decode_advance_kernel)
void decode_advance(Tensor tokens, Tensor positions, Tensor ctx_lens, Tensor slots, Tensor sampled, Tensor out,
                    Tensor counter, int64_t base_block, int64_t block_size) {
  c10::DeviceGuard g(tokens.device());
  for (const Tensor* t : {&tokens, &positions, &ctx_lens, &sampled, &out, &counter})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1, "int32 GPU tensors expected");
  TORCH_CHECK(slots.is_cuda() && slots.scalar_type() == at::kLong && slots.numel() >= 1, "slots int64");
  TORCH_CHECK(block_size > 0 && base_block >= 0, "bad block geometry");
  check_rc(vwa_decode_advance(tokens.data_ptr<int>(), positions.data_ptr<int>(), ctx_lens.data_ptr<int>(),
                              slots.data_ptr<int64_t>(), sampled.data_ptr<int>(), out.data_ptr<int>(),
                              counter.data_ptr<int>(), (int)out.numel(), (int)base_block, (int)block_size,
                              cur_stream(tokens)),
           "decode_advance");
}

// Device memory the L2 does not cache (hipDeviceMallocUncached): chain barrier words polled with
// scalar loads.  Returned as an int32 tensor whose deleter DEFERS the hipFree to the next
// allocation: the tensor may die in a garbage collection that runs inside another model's graph
// capture, where a hipFree is not permitted (seen: the whole process aborted in the GC of an
// earlier test's model during the next test's capture).
static std::mutex g_uncached_mu;
static std::vector<void*> g_uncached_pending;

Tensor alloc_uncached_i32(int64_t n, Tensor like) {
  c10::DeviceGuard g(like.device());
  {
    std::lock_guard<std::mutex> lk(g_uncached_mu);
    for (void* p : g_uncached_pending) (void)hipFree(p);
    g_uncached_pending.clear();
  }
  void* ptr = nullptr;
  TORCH_CHECK(hipExtMallocWithFlags(&ptr, (size_t)n * 4, hipDeviceMallocUncached) == hipSuccess, "uncached malloc");
  TORCH_CHECK(hipMemset(ptr, 0, (size_t)n * 4) == hipSuccess, "memset");
  return torch::from_blob(ptr, {n}, [](void* p) {
        std::lock_guard<std::mutex> lk(g_uncached_mu);
        g_uncached_pending.push_back(p);
      }, torch::dtype(torch::kInt).device(like.device()));
}

// n_layers > 1: desc holds n_layers consecutive descriptors (torch.cat of chain_make outputs of
// consecutive layers, same flags) run by ONE launch (skinny_stream.hip chain_kernel MULTI)
void chain_run(Tensor desc, int64_t n_phases, int64_t lds, Tensor like, int64_t attn_g, int64_t seq, int64_t n_layers) {
  c10::DeviceGuard g(like.device());
  TORCH_CHECK(n_layers >= 1 && desc.is_cuda() && desc.is_contiguous() &&
                  desc.numel() == n_layers * (int64_t)sizeof(ChainParams) &&
                  (reinterpret_cast<uintptr_t>(desc.data_ptr()) & 63) == 0,
              "bad chain descriptor (n_layers x sizeof(ChainParams) bytes, 64-byte aligned)");
  // one workgroup per CU: the barrier needs every workgroup resident
  check_rc(vwa_chain_launch(reinterpret_cast<const ChainParams*>(desc.data_ptr()), (int)seq, (int)n_phases, (int)attn_g,
                            (int)(lds & 0xFFFFFF), chain_grid(like.device().index()), cur_stream(like),
                            (int)((lds >> 24) & 1) * (((lds >> 27) & 1) ? 2 : 1), (int)((lds >> 25) & 1),
                            (int)((lds >> 26) & 1), (int)n_layers),
           "chain");
}

// Persistent Whisper decoder (whisper_dec.hip): per-layer descriptors from a flat list of
// 3 kWdGemms + 4 tensors per layer -- (W, bias, ln_c) of each WdecLayer::g (pre-tiled bf16 weights;
// bias / ln_c may be None), then k_cache, v_cache, cross K, cross V.
Tensor wdec_layers(std::vector<c10::optional<Tensor>> flat, int64_t n_layers, Tensor like) {
  constexpr int kPer = 3 * kWdGemms + 4;
  TORCH_CHECK(n_layers >= 1 && (int64_t)flat.size() == n_layers * kPer, "wdec_layers: 3 kWdGemms + 4 entries per layer");
  auto ptr = [&](int64_t i, bool need) -> void* {
    const auto& t = flat[(size_t)i];
    if (!t.has_value()) {
      TORCH_CHECK(!need, "wdec_layers: entry ", i, " is required");
      return nullptr;
    }
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->device() == like.device(), "wdec_layers: entry ", i,
                " must be a contiguous tensor on the model's GPU");
    return t->data_ptr();
  };
  Tensor host = torch::zeros({n_layers * (int64_t)sizeof(WdecLayer)}, torch::dtype(torch::kUInt8));
  auto* L = reinterpret_cast<WdecLayer*>(host.data_ptr());
  for (int64_t li = 0; li < n_layers; ++li) {
    const int64_t b = li * kPer;
    for (int g = 0; g < kWdGemms; ++g) {
      const auto& w = flat[(size_t)(b + 3 * g)];
      TORCH_CHECK(w.has_value() && w->scalar_type() == at::kBFloat16, "wdec_layers: bf16 weights");
      L[li].g[g].W = static_cast<const uint16_t*>(ptr(b + 3 * g, true));
      L[li].g[g].bias = static_cast<const uint16_t*>(ptr(b + 3 * g + 1, false));
      const auto& c = flat[(size_t)(b + 3 * g + 2)];
      TORCH_CHECK(!c.has_value() || c->scalar_type() == at::kFloat, "wdec_layers: ln_c f32");
      L[li].g[g].ln_c = static_cast<const float*>(ptr(b + 3 * g + 2, false));
    }
    constexpr int c0 = 3 * kWdGemms;
    L[li].k_cache = static_cast<uint16_t*>(ptr(b + c0, true));
    L[li].v_cache = static_cast<uint16_t*>(ptr(b + c0 + 1, true));
    L[li].xk = static_cast<const uint16_t*>(ptr(b + c0 + 2, true));
    L[li].xv = static_cast<const uint16_t*>(ptr(b + c0 + 3, true));
  }
  return host.to(like.device());
}

// bufs: x0, x1, q, att, f, xpart, seq_ids, ctx_lens, slots, block_table, cross_table, cnt
// ints: n_layers, d, H, ffn, T, block_size, bt_stride, nch, ch_len, sessions, grid
// lm (optional): [W pre-tiled bf16 [V, d], bias bf16 [V] or None-as-empty, column sums f32 [V], logits f32 [>= V]]
void wdec_run(Tensor layers, Tensor roles, std::vector<Tensor> bufs, std::vector<int64_t> ints, double eps,
              double scale, std::vector<int64_t> n_prod, c10::optional<Tensor> ts, int64_t opt,
              c10::optional<std::vector<Tensor>> lm, c10::optional<std::vector<Tensor>> emb,
              c10::optional<std::vector<Tensor>> smp, int64_t loop_base_block) {
  TORCH_CHECK(bufs.size() == 12 && ints.size() == 11 && n_prod.size() == kWdLevels, "wdec_run: argument counts");
  const Tensor& like = bufs[0];
  c10::DeviceGuard g(like.device());
  const int64_t grid = ints[10];
  TORCH_CHECK(layers.is_cuda() && layers.numel() == ints[0] * (int64_t)sizeof(WdecLayer), "wdec_run: layers");
  TORCH_CHECK(roles.is_cuda() && roles.scalar_type() == at::kInt && roles.is_contiguous() &&
                  roles.numel() == grid * kWdRole, "wdec_run: roles [grid, 32] int32");
  for (int i = 0; i < 5; ++i) check_bf16(bufs[(size_t)i], "wdec_run activation");
  WdecParams p{};
  p.layers = reinterpret_cast<const WdecLayer*>(layers.data_ptr());
  p.n_layers = (int)ints[0];
  p.roles = roles.data_ptr<int>();
  p.d = (int)ints[1];
  p.H = (int)ints[2];
  p.ffn = (int)ints[3];
  p.T = (int)ints[4];
  p.block_size = (int)ints[5];
  p.bt_stride = (int)ints[6];
  p.nch = (int)ints[7];
  p.ch_len = (int)ints[8];
  p.sessions = (int)ints[9];
  p.eps = (float)eps;
  p.scale = (float)scale;
  auto bf = [&](int i) { return reinterpret_cast<uint16_t*>(bufs[(size_t)i].data_ptr()); };
  p.x0 = bf(0);
  p.x1 = bf(1);
  p.q = bf(2);
  p.att = bf(3);
  p.f = bf(4);
  TORCH_CHECK(bufs[5].scalar_type() == at::kFloat && bufs[5].numel() >= (int64_t)p.H * p.nch * 68 + 3 * p.d,
              "wdec_run: xpart (cross partials + the cross query's two f32 halves + x1 tile sums)");
  p.xpart = bufs[5].data_ptr<float>();
  p.seq_ids = bufs[6].data_ptr<int>();
  p.ctx_lens = bufs[7].data_ptr<int>();
  TORCH_CHECK(bufs[8].scalar_type() == at::kLong, "wdec_run: slots int64");
  p.slots = bufs[8].data_ptr<int64_t>();
  p.block_table = bufs[9].data_ptr<int>();
  p.cross_table = bufs[10].data_ptr<int>();
  TORCH_CHECK(bufs[11].numel() >= 2 * (1280 + 16 * ints[2]),
              "wdec_run: counter words (uncached: levels, error word, sampler, per-head QKV counters)");
  p.cnt = reinterpret_cast<unsigned long long*>(bufs[11].data_ptr());
  for (int l = 0; l < kWdLevels; ++l) {
    TORCH_CHECK(n_prod[(size_t)l] > 0, "wdec_run: every level needs a producer");
    p.n_prod[l] = (int)n_prod[(size_t)l];
  }
  if (ts.has_value()) {
    TORCH_CHECK(ts->is_cuda() && ts->scalar_type() == at::kLong && ts->numel() >= grid * ints[0] * kWdLevels * 4,
                "wdec_run: ts int64 [grid * n_layers * 8 * 4]");
    p.ts = reinterpret_cast<unsigned long long*>(ts->data_ptr());
  }
  p.opt[0] = (int)opt;
  if (lm.has_value()) {
    const std::vector<Tensor>& L = *lm;
    TORCH_CHECK(L.size() == 4, "wdec_run: lm = [W, bias, ln_c, logits]");
    check_bf16(L[0], "wdec_run lm W");
    TORCH_CHECK(L[0].dim() == 2 && L[0].size(1) == p.d && L[0].size(0) % 16 == 0 && L[0].is_contiguous(),
                "wdec_run: lm W [V % 16 == 0, d] (pre-tiled)");
    const int64_t V = L[0].size(0);
    TORCH_CHECK(L[2].scalar_type() == at::kFloat && L[2].numel() == V && L[2].is_cuda(), "wdec_run: lm ln_c f32 [V]");
    TORCH_CHECK(L[3].scalar_type() == at::kFloat && L[3].is_contiguous() && L[3].numel() >= V && L[3].is_cuda(),
                "wdec_run: logits f32 [>= V]");
    p.lm_W = reinterpret_cast<const uint16_t*>(L[0].data_ptr());
    if (L[1].numel()) {
      check_bf16(L[1], "wdec_run lm bias");
      TORCH_CHECK(L[1].numel() == V, "wdec_run: lm bias [V]");
      p.lm_b = reinterpret_cast<const uint16_t*>(L[1].data_ptr());
    }
    p.lm_c = L[2].data_ptr<float>();
    p.logits = L[3].data_ptr<float>();
    p.n_vocab = (int)V;
  }
  // emb (optional): [tok_emb bf16 [rows, d], pos_emb bf16 [>= max position + 1, d], tokens int32, positions int32]
  if (emb.has_value()) {
    const std::vector<Tensor>& Em = *emb;
    TORCH_CHECK(Em.size() == 4, "wdec_run: emb = [tok_emb, pos_emb, tokens, positions]");
    check_bf16(Em[0], "wdec_run tok_emb");
    check_bf16(Em[1], "wdec_run pos_emb");
    TORCH_CHECK(Em[0].dim() == 2 && Em[0].size(1) == p.d && Em[0].is_contiguous() && Em[1].dim() == 2 &&
                    Em[1].size(1) == p.d && Em[1].is_contiguous(),
                "wdec_run: embedding tables [rows, d] contiguous");
    TORCH_CHECK(Em[2].scalar_type() == at::kInt && Em[3].scalar_type() == at::kInt && Em[2].is_cuda() && Em[3].is_cuda(),
                "wdec_run: tokens / positions int32");
    TORCH_CHECK(p.block_size > 0 && Em[1].size(0) >= (int64_t)p.bt_stride * p.block_size,
                "wdec_run: the position table covers every KV position");
    p.tok_emb = reinterpret_cast<const uint16_t*>(Em[0].data_ptr());
    p.pos_emb = reinterpret_cast<const uint16_t*>(Em[1].data_ptr());
    p.tokens = Em[2].data_ptr<int>();
    p.positions = Em[3].data_ptr<int>();
    p.emb_rows = (int)Em[0].size(0);
  }
  // smp (optional, needs lm): [mask u32-as-int32 [>= V / 32], out_tok int32, step int32, part f32 [2 grid],
  //   loop_out int32, loop_cnt int32, adv_tokens, adv_positions, adv_ctx int32, adv_slots int64]
  if (smp.has_value()) {
    const std::vector<Tensor>& S = *smp;
    TORCH_CHECK(S.size() == 10 && p.lm_W, "wdec_run: smp = 10 tensors, with the LM head");
    TORCH_CHECK(S[0].scalar_type() == at::kInt && S[0].numel() * 32 >= p.n_vocab, "wdec_run: sampler mask words");
    TORCH_CHECK(S[3].scalar_type() == at::kFloat && S[3].numel() >= 2 * grid, "wdec_run: sampler partials f32 [2 grid]");
    for (int i : {1, 2, 4, 5, 6, 7, 8}) TORCH_CHECK(S[(size_t)i].scalar_type() == at::kInt && S[(size_t)i].is_cuda(), "wdec_run: int32 loop state");
    TORCH_CHECK(S[9].scalar_type() == at::kLong && S[9].is_cuda(), "wdec_run: slots int64");
    p.smp_mask = reinterpret_cast<const uint32_t*>(S[0].data_ptr());
    p.smp_tok = S[1].data_ptr<int>();
    p.smp_step = S[2].data_ptr<int>();
    p.smp_part = S[3].data_ptr<float>();
    p.loop_out = S[4].data_ptr<int>();
    p.loop_max = (int)S[4].numel();
    p.loop_cnt = S[5].data_ptr<int>();
    p.adv_tokens = S[6].data_ptr<int>();
    p.adv_positions = S[7].data_ptr<int>();
    p.adv_ctx = S[8].data_ptr<int>();
    p.adv_slots = S[9].data_ptr<int64_t>();
    p.loop_base_block = (int)loop_base_block;
    TORCH_CHECK(bufs[11].numel() >= 2 * 1280, "wdec_run: counter words hold the sampler counters (u64 1152..1279)");
  }
  check_rc(vwa_wdec_launch(&p, (int)grid, cur_stream(like)), "wdec");
}

void rmsnorm(Tensor x, c10::optional<Tensor> residual, c10::optional<Tensor> residual_out, c10::optional<Tensor> w,
             Tensor y, double eps) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_contig_rows(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(y.is_contiguous() && y.sizes() == x.sizes(), "y shape");
  const int rows = (int)x.size(0), D = (int)x.size(1);
  if (residual.has_value()) {
    TORCH_CHECK(residual_out.has_value() && residual->is_contiguous() && residual_out->is_contiguous() &&
                    residual->sizes() == x.sizes() && residual_out->sizes() == x.sizes(),
                "residual shapes");
  }
  if (w.has_value()) TORCH_CHECK(w->numel() == D, "w must be [D]");
  check_rc(vwa_rmsnorm(bfp(x), bfp_opt(residual), residual_out.has_value() ? bfp_mut(*residual_out) : nullptr,
                       bfp_opt(w), bfp_mut(y), rows, D, (int)x.stride(0), (float)eps, cur_stream(x)),
           "rmsnorm");
}

void layernorm(Tensor x, c10::optional<Tensor> residual, c10::optional<Tensor> residual_out, Tensor w, Tensor b,
               Tensor y, double eps) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_contig_rows(x, "x");
  TORCH_CHECK(y.is_contiguous() && y.sizes() == x.sizes(), "y shape");
  const int rows = (int)x.size(0), D = (int)x.size(1);
  TORCH_CHECK(w.numel() == D && b.numel() == D, "w/b must be [D]");
  if (residual.has_value())
    TORCH_CHECK(residual_out.has_value() && residual->sizes() == x.sizes() && residual_out->sizes() == x.sizes() &&
                    residual->is_contiguous() && residual_out->is_contiguous(),
                "residual shapes");
  check_rc(vwa_layernorm(bfp(x), bfp_opt(residual), residual_out.has_value() ? bfp_mut(*residual_out) : nullptr,
                         bfp(w), bfp(b), bfp_mut(y), rows, D, (int)x.stride(0), (float)eps, cur_stream(x)),
           "layernorm");
}

void rope_kv_write(Tensor qkv, int64_t n_q_heads, int64_t n_kv_heads, int64_t head_dim, bool use_rope,
                   Tensor positions, Tensor slots, c10::optional<Tensor> rope, Tensor q_out, Tensor k_cache,
                   Tensor v_cache) {
  c10::DeviceGuard g(qkv.device());
  check_bf16(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) == (n_q_heads + 2 * n_kv_heads) * head_dim,
              "qkv shape");
  const int rows = (int)qkv.size(0);
  TORCH_CHECK(positions.scalar_type() == at::kInt && positions.numel() >= rows, "positions");
  TORCH_CHECK(slots.scalar_type() == at::kLong && slots.numel() >= rows, "slots");
  TORCH_CHECK(q_out.dim() == 2 && q_out.size(0) >= rows && q_out.size(1) == n_q_heads * head_dim, "q_out");
  check_cache(k_cache, "k_cache");
  check_cache(v_cache, "v_cache");
  if (use_rope) TORCH_CHECK(rope.has_value() && rope->scalar_type() == at::kFloat, "rope table");
  check_rc(vwa_rope_kv_write(bfp(qkv), (int)qkv.stride(0), rows, (int)n_q_heads, (int)n_kv_heads, (int)head_dim,
                             use_rope ? 1 : 0, positions.data_ptr<int>(), slots.data_ptr<int64_t>(),
                             use_rope ? rope->data_ptr<float>() : nullptr, bfp_mut(q_out), (int)q_out.stride(0),
                             bfp_mut(k_cache), bfp_mut(v_cache), (int)k_cache.size(2), k_cache.stride(0),
                             k_cache.stride(1), k_cache.stride(2), cur_stream(qkv)),
           "rope_kv_write");
}

void swiglu(Tensor gu, Tensor h) {
  c10::DeviceGuard g(gu.device());
  check_bf16(gu, "gu");
  TORCH_CHECK(gu.is_contiguous() && h.is_contiguous() && gu.dim() == 2 && h.dim() == 2 && gu.size(0) == h.size(0) &&
                  gu.size(1) == 2 * h.size(1),
              "swiglu shapes");
  check_rc(vwa_swiglu(bfp(gu), bfp_mut(h), (int)h.size(0), (int)h.size(1), cur_stream(gu)), "swiglu");
}

void bias_act(Tensor x, c10::optional<Tensor> bias, c10::optional<Tensor> residual, Tensor y, int64_t act) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.dim() == 2 && y.sizes() == x.sizes(), "bias_act shapes");
  if (bias.has_value()) TORCH_CHECK(bias->numel() == x.size(1), "bias");
  if (residual.has_value()) TORCH_CHECK(residual->sizes() == x.sizes() && residual->is_contiguous(), "residual");
  check_rc(vwa_bias_act(bfp(x), bfp_opt(bias), bfp_opt(residual), bfp_mut(y), (int)x.size(0), (int)x.size(1),
                        (int)act, cur_stream(x)),
           "bias_act");
}

KVView make_view(const Tensor& k, const Tensor& v, const Tensor& table, int64_t block_size, int64_t sb, int64_t sh,
                 int64_t stok) {
  check_bf16(k, "k");
  check_bf16(v, "v");
  TORCH_CHECK(table.scalar_type() == at::kInt && table.dim() == 2 && table.is_contiguous(), "block table int32 2-D");
  KVView kv{};
  kv.k = bfp(k);
  kv.v = bfp(v);
  kv.block_table = table.data_ptr<int>();
  kv.table_stride = (int)table.stride(0);
  kv.block_size = (int)block_size;
  kv.stride_block = sb;
  kv.stride_head = sh;
  kv.stride_tok = stok;
  return kv;
}

DecodeAttnParams decode_params(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& table, int64_t block_size, int64_t sb, int64_t sh,
                      int64_t stok, const Tensor& ctx_lens, const Tensor& seq_ids, int64_t n_q_heads, int64_t n_kv_heads,
                      int64_t head_dim, double scale, int64_t n_splits, const Tensor& part_o, const Tensor& part_ml,
                      const Tensor& counters, const Tensor& out) {
  check_bf16(q, "q");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1 && q.size(1) == n_q_heads * head_dim, "q shape");
  TORCH_CHECK(q.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(q.data_ptr()) % 16 == 0,
              "q rows must be 16-byte aligned (vector loads)");
  const int rows = (int)q.size(0);
  TORCH_CHECK(ctx_lens.scalar_type() == at::kInt && ctx_lens.numel() >= rows, "ctx_lens");
  TORCH_CHECK(seq_ids.scalar_type() == at::kInt && seq_ids.numel() >= rows, "seq_ids");
  TORCH_CHECK(out.dim() == 2 && out.size(0) >= rows && out.size(1) == n_q_heads * head_dim && out.stride(1) == 1,
              "out shape");
  TORCH_CHECK(n_splits >= 1, "n_splits");
  if (n_splits > 1) {
    TORCH_CHECK(part_o.scalar_type() == at::kFloat && part_o.numel() >= (int64_t)rows * n_splits * n_q_heads * head_dim,
                "part_o too small");
    TORCH_CHECK(part_ml.scalar_type() == at::kFloat && part_ml.numel() >= (int64_t)rows * n_splits * n_q_heads * 2,
                "part_ml too small");
    TORCH_CHECK(n_splits <= 64, "decode attention merges <= 64 chunks (context <= 16384 tokens)");
    TORCH_CHECK(counters.scalar_type() == at::kInt && counters.is_cuda() && counters.numel() >= rows * n_kv_heads,
                "counters: int32 [rows * n_kv_heads], zero-initialised, left zero by the kernel");
  }
  DecodeAttnParams p{};
  p.q = bfp(q);
  p.ldq = (int)q.stride(0);
  p.kv = make_view(k, v, table, block_size, sb, sh, stok);
  p.ctx_lens = ctx_lens.data_ptr<int>();
  p.seq_ids = seq_ids.data_ptr<int>();
  p.rows = rows;
  p.n_q_heads = (int)n_q_heads;
  p.n_kv_heads = (int)n_kv_heads;
  p.head_dim = (int)head_dim;
  p.scale = (float)scale;
  p.split_tokens = vwa_attention_split_tokens();
  p.n_splits = (int)n_splits;
  p.part_o = part_o.data_ptr<float>();
  p.part_ml = part_ml.data_ptr<float>();
  p.counters = counters.data_ptr<int>();
  p.out = bfp_mut(out);
  p.ldo = (int)out.stride(0);
  return p;
}

void decode_attention(Tensor q, Tensor k, Tensor v, Tensor table, int64_t block_size, int64_t sb, int64_t sh,
                      int64_t stok, Tensor ctx_lens, Tensor seq_ids, int64_t n_q_heads, int64_t n_kv_heads,
                      int64_t head_dim, double scale, int64_t n_splits, Tensor part_o, Tensor part_ml,
                      Tensor counters, Tensor out, c10::optional<Tensor> shared) {
  c10::DeviceGuard g(q.device());
  DecodeAttnParams p = decode_params(q, k, v, table, block_size, sb, sh, stok, ctx_lens, seq_ids, n_q_heads,
                                     n_kv_heads, head_dim, scale, n_splits, part_o, part_ml, counters, out);
  if (shared.has_value()) {
    TORCH_CHECK(shared->is_cuda() && shared->scalar_type() == at::kInt && shared->numel() >= 2 &&
                    shared->is_contiguous(),
                "shared: int32 [P, n_real] on the device");
    p.shared = shared->data_ptr<int>();
  }
  check_rc(vwa_decode_attention(&p, cur_stream(q)), "decode_attention");
}

void flash_attention(Tensor q, Tensor k, Tensor v, Tensor table, int64_t block_size, int64_t sb, int64_t sh,
                     int64_t stok, Tensor out, int64_t Sk, int64_t n_kv_heads, bool causal, int64_t q_offset,
                     c10::optional<Tensor> q_offsets, c10::optional<Tensor> k_lens, double scale) {
  c10::DeviceGuard g(q.device());
  check_bf16(q, "q");
  TORCH_CHECK(q.dim() == 4, "q must be [B, S, H, D]");
  TORCH_CHECK(q.stride(3) == 1 && out.stride(3) == 1 && out.sizes() == q.sizes(), "q/out layout");
  const int64_t D = q.size(3);
  TORCH_CHECK((q.stride(2) % 8) == 0 && (q.stride(1) % 8) == 0, "q strides must be 16-byte multiples");
  FlashAttnParams p{};
  p.q = bfp(q);
  p.q_stride_b = q.stride(0);
  p.q_stride_s = q.stride(1);
  p.q_stride_h = q.stride(2);
  p.kv = make_view(k, v, table, block_size, sb, sh, stok);
  p.o = bfp_mut(out);
  p.o_stride_b = out.stride(0);
  p.o_stride_s = out.stride(1);
  p.o_stride_h = out.stride(2);
  p.B = (int)q.size(0);
  p.Sq = (int)q.size(1);
  p.Sk = (int)Sk;
  p.n_q_heads = (int)q.size(2);
  p.n_kv_heads = (int)n_kv_heads;
  p.head_dim = (int)D;
  p.causal = causal ? 1 : 0;
  p.q_offset = (int)q_offset;
  p.q_offsets = q_offsets.has_value() ? q_offsets->data_ptr<int>() : nullptr;
  p.k_lens = k_lens.has_value() ? k_lens->data_ptr<int>() : nullptr;
  p.scale = (float)scale;
  check_rc(vwa_flash_attention(&p, cur_stream(q)), "flash_attention");
}

void embedding(Tensor ids, Tensor table, c10::optional<Tensor> pos_table, c10::optional<Tensor> positions, Tensor out,
               int64_t vocab_start) {
  c10::DeviceGuard g(ids.device());
  TORCH_CHECK(ids.scalar_type() == at::kInt, "ids int32");
  check_bf16(table, "table");
  TORCH_CHECK(table.is_contiguous() && out.is_contiguous() && out.size(1) == table.size(1), "embedding shapes");
  const int rows = (int)out.size(0);
  TORCH_CHECK(ids.numel() >= rows, "ids too short");
  if (pos_table.has_value()) TORCH_CHECK(positions.has_value() && positions->scalar_type() == at::kInt, "positions");
  check_rc(vwa_embedding(ids.data_ptr<int>(), bfp(table), bfp_opt(pos_table),
                         positions.has_value() ? positions->data_ptr<int>() : nullptr, bfp_mut(out), rows,
                         (int)table.size(1), (int)vocab_start, (int)(vocab_start + table.size(0)), cur_stream(ids)),
           "embedding");
}

struct SampleArgs {
  int rows = 0, V = 0, mask_words = 0;
  const uint32_t* mask = nullptr;
  const float* temperature = nullptr;
  const int64_t* fail = nullptr;
};

SampleArgs check_sample(const Tensor& logits, const c10::optional<Tensor>& mask,
                        const c10::optional<Tensor>& temperature, const Tensor& seed, const Tensor& step,
                        const Tensor& out_tokens, const c10::optional<Tensor>& fail_word, int64_t v_offset) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kFloat && logits.dim() == 2 && logits.stride(1) == 1,
              "logits f32 2-D on the GPU");
  SampleArgs a;
  a.rows = (int)logits.size(0);
  a.V = (int)logits.size(1);
  TORCH_CHECK(v_offset >= 0 && v_offset % 32 == 0, "v_offset must be a non-negative multiple of 32");
  if (mask.has_value()) {
    // (pinned host rows allowed: zero-copy grammar masks)
    TORCH_CHECK((mask->is_cuda() || mask->is_pinned()) && mask->scalar_type() == at::kInt && mask->dim() == 2 &&
                    mask->is_contiguous() && mask->size(0) >= a.rows,
                "mask int32 [rows, words]");
    a.mask_words = (int)mask->size(1);
    TORCH_CHECK((int64_t)a.mask_words * 32 >= v_offset + a.V, "mask too short");
    a.mask = reinterpret_cast<const uint32_t*>(mask->data_ptr<int>());
  }
  if (temperature.has_value()) {
    TORCH_CHECK(temperature->scalar_type() == at::kFloat && temperature->numel() >= a.rows, "temperature");
    a.temperature = temperature->data_ptr<float>();
  }
  TORCH_CHECK(seed.is_cuda() && step.is_cuda() && seed.scalar_type() == at::kLong && step.scalar_type() == at::kInt,
              "seed int64, step int32 (device)");
  TORCH_CHECK((out_tokens.is_cuda() || out_tokens.is_pinned()) && out_tokens.scalar_type() == at::kInt &&
                  out_tokens.numel() >= a.rows,
              "out_tokens");
  if (fail_word.has_value()) {
    TORCH_CHECK(fail_word->scalar_type() == at::kLong && fail_word->numel() >= 1 && fail_word->is_cuda(),
                "fail_word: one device int64");
    a.fail = fail_word->data_ptr<int64_t>();
  }
  return a;
}

void sample(Tensor logits, c10::optional<Tensor> mask, c10::optional<Tensor> temperature, Tensor seed, Tensor step,
            Tensor out_tokens, Tensor part_val, Tensor part_idx, c10::optional<Tensor> fail_word, int64_t v_offset) {
  c10::DeviceGuard g(logits.device());
  const SampleArgs a = check_sample(logits, mask, temperature, seed, step, out_tokens, fail_word, v_offset);
  const int n_chunks = (int)(part_val.numel() / a.rows);
  TORCH_CHECK(n_chunks >= 1 && part_idx.numel() >= (int64_t)a.rows * n_chunks, "partials");
  hipStream_t st = cur_stream(logits);
  check_rc(vwa_sample_partial(logits.data_ptr<float>(), (int)logits.stride(0), a.rows, a.V, (int)v_offset, a.mask,
                              a.mask_words, a.temperature, reinterpret_cast<const uint64_t*>(seed.data_ptr<int64_t>()),
                              step.data_ptr<int>(), part_val.data_ptr<float>(), part_idx.data_ptr<int>(), n_chunks, st),
           "sample (partial)");
  check_rc(vwa_sample_final(part_val.data_ptr<float>(), part_idx.data_ptr<int>(), n_chunks, 1, 0,
                            out_tokens.data_ptr<int>(), step.data_ptr<int>(), a.rows, a.fail, st),
           "sample (final)");
}

// Vocab-parallel sampling (SURVEY.md §2.8 C4 as [B, 2] per rank): partial maxima over this rank's
// logits shard (global ids from v_offset) into xin = [val f32 | idx i32] x [rows][n_chunks], the
// one-shot IPC all-gather of xin over the TP group, then every rank merges all ranks' partials in
// rank order -- bit-identical tokens on every rank, and the same token a TP=1 sampler draws
// (the Gumbel noise and the tie-break use global token ids).  Three launches, no host sync.
void sample_tp(Tensor logits, c10::optional<Tensor> mask, c10::optional<Tensor> temperature, Tensor seed, Tensor step,
               Tensor out_tokens, Tensor xin, Tensor xout, int64_t n_chunks, c10::optional<Tensor> fail_word,
               int64_t v_offset, int64_t ar_state, int64_t world) {
  c10::DeviceGuard g(logits.device());
  const SampleArgs a = check_sample(logits, mask, temperature, seed, step, out_tokens, fail_word, v_offset);
  const int64_t words = 2 * (int64_t)a.rows * n_chunks;
  TORCH_CHECK(n_chunks >= 1 && n_chunks <= 1024, "n_chunks");
  TORCH_CHECK(world >= 1 && world <= 8 && ar_state != 0, "TP group state");
  TORCH_CHECK(words <= vwa_ar_gather_max_words(), "sampler partials exceed the all-gather region");
  TORCH_CHECK(xin.is_cuda() && xin.scalar_type() == at::kInt && xin.is_contiguous() && xin.numel() >= words,
              "xin int32 [>= 2 * rows * n_chunks]");
  TORCH_CHECK(xout.is_cuda() && xout.scalar_type() == at::kInt && xout.is_contiguous() && xout.numel() >= world * words,
              "xout int32 [>= world * 2 * rows * n_chunks]");
  hipStream_t st = cur_stream(logits);
  int* in = xin.data_ptr<int>();
  check_rc(vwa_sample_partial(logits.data_ptr<float>(), (int)logits.stride(0), a.rows, a.V, (int)v_offset, a.mask,
                              a.mask_words, a.temperature, reinterpret_cast<const uint64_t*>(seed.data_ptr<int64_t>()),
                              step.data_ptr<int>(), reinterpret_cast<float*>(in), in + a.rows * n_chunks,
                              (int)n_chunks, st),
           "sample_tp (partial)");
  int* out = xout.data_ptr<int>();
  check_rc(vwa_ar_gather(reinterpret_cast<void*>(ar_state), in, out, words, st), "sample_tp (all-gather)");
  check_rc(vwa_sample_final(reinterpret_cast<const float*>(out), out + a.rows * n_chunks, (int)n_chunks, (int)world,
                            words, out_tokens.data_ptr<int>(), step.data_ptr<int>(), a.rows, a.fail, st),
           "sample_tp (merge)");
}

void pcm16_to_f32(Tensor pcm, Tensor out, double ratio) {
  c10::DeviceGuard g(pcm.device());
  TORCH_CHECK(pcm.scalar_type() == at::kShort && out.scalar_type() == at::kFloat, "pcm int16 -> f32");
  TORCH_CHECK(pcm.is_contiguous() && out.is_contiguous(), "contiguous");
  const int n_in = (int)pcm.numel(), n_out = (int)out.numel();
  TORCH_CHECK((int64_t)((n_out - 1) * ratio) < (int64_t)n_in + 1, "resample ratio overruns input");
  check_rc(vwa_pcm16_to_f32(pcm.data_ptr<int16_t>(), out.data_ptr<float>(), n_in, n_out, (float)ratio, cur_stream(pcm)),
           "pcm16_to_f32");
}

void log_mel(Tensor audio, int64_t n_frames, Tensor window, Tensor basis, Tensor fb_frag, int64_t n_mels,
             Tensor mel_scratch, Tensor max_buf, Tensor out) {
  c10::DeviceGuard g(audio.device());
  TORCH_CHECK(audio.scalar_type() == at::kFloat && audio.is_contiguous(), "audio f32");
  TORCH_CHECK(window.numel() == 400 && window.scalar_type() == at::kFloat && window.is_contiguous(), "n_fft=400 window");
  TORCH_CHECK(n_mels >= 1 && n_mels <= 128, "n_mels <= 128");
  const int64_t mt = (n_mels + 15) / 16;
  TORCH_CHECK(basis.scalar_type() == at::kFloat && basis.is_contiguous() && basis.numel() == 26 * 25 * 64 * 4,
              "basis: DFT fragments [26][25][64][4] f32 (ops.logmel_tables)");
  TORCH_CHECK(fb_frag.scalar_type() == at::kFloat && fb_frag.is_contiguous() && fb_frag.numel() == mt * 13 * 64 * 4,
              "fb_frag: mel filterbank fragments [n_mels/16][13][64][4] f32 (ops.logmel_tables)");
  TORCH_CHECK(mel_scratch.numel() >= n_frames * n_mels && max_buf.numel() >= 1, "scratch");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 && out.dim() == 2 && out.size(0) >= n_frames && out.size(1) == n_mels &&
                  out.stride(1) == 1,
              "out bf16 [frames, n_mels]");
  TORCH_CHECK(audio.numel() > 200, "audio too short");
  check_rc(vwa_log_mel(audio.data_ptr<float>(), (int)audio.numel(), (int)n_frames, window.data_ptr<float>(),
                       basis.data_ptr<float>(), fb_frag.data_ptr<float>(), (int)n_mels, mel_scratch.data_ptr<float>(),
                       max_buf.data_ptr<float>(), bfp_mut(out), (int)out.stride(0), cur_stream(audio)),
           "log_mel");
}

// Whisper conv stem (K3): conv1d(k=3, pad=1, stride) + bias + GELU (+ pos) as a batched implicit
// GEMM on the tiled MFMA GEMM (gemm.hip, row-major weights).  x [B, Tin, Cin] must be a view
// of a zero-padded channels-last buffer (ops.padded_rows): one zero row in front of and behind
// every batch's Tin rows, so GEMM row t is the 3*Cin contiguous elements starting at padded
// row t*stride (ldx = stride*Cin).  w [Cout, 3*Cin] in (kk, ci) order, row-major or pre-tiled.
void conv1d_gelu(Tensor x, Tensor w, c10::optional<Tensor> b, c10::optional<Tensor> pos, Tensor y, int64_t stride,
                 bool w_tiled) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 3 && x.stride(2) == 1 && x.stride(1) == x.size(2), "x must be [B, T, Cin] with contiguous rows");
  const int64_t B = x.size(0), Tin = x.size(1), Cin = x.size(2);
  TORCH_CHECK(B == 1 || x.stride(0) >= (Tin + 2) * Cin, "x batches must be (Tin + 2)-row padded slabs");
  TORCH_CHECK(x.storage_offset() >= Cin &&
                  (int64_t)(x.storage().nbytes() / 2) >= x.storage_offset() + (B - 1) * x.stride(0) + (Tin + 1) * Cin,
              "x must be a view of a zero-padded buffer (a pad row before and after each batch)");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous() && w.size(1) == 3 * Cin, "w must be [Cout, 3*Cin] ([co][kk][ci])");
  TORCH_CHECK(stride == 1 || stride == 2, "stride 1 or 2");
  const int64_t Tout = (Tin + 2 - 3) / stride + 1, Cout = w.size(0);
  TORCH_CHECK(y.dim() == 3 && y.size(0) == B && y.size(1) == Tout && y.size(2) == Cout && y.stride(2) == 1 &&
                  y.stride(1) % 8 == 0 && (B == 1 || y.stride(0) % 8 == 0) &&
                  (reinterpret_cast<uintptr_t>(y.data_ptr()) & 15) == 0,
              "y [B, Tout, Cout] with 16-byte aligned rows");
  TORCH_CHECK((3 * Cin) % 128 == 0 && Cout % 16 == 0 && Cin % 8 == 0, "conv: 3*Cin % 128 == 0, Cout % 16 == 0");
  GemmParams p{};
  p.X = bfp(x) - Cin;  // the zero row in front
  p.ldx = (int)(stride * Cin);
  p.W = bfp(w);
  p.w_tiled = w_tiled ? 1 : 0;  // ops.tile_weight layout: 1 KB contiguous B-fragment DMA per instruction
  p.M = (int)Tout;
  p.N = (int)Cout;
  p.K = (int)(3 * Cin);
  p.Y = y.data_ptr();
  p.ldy = (int)y.stride(1);
  p.splits = 1;
  p.nbatch = (int)B;
  p.bsx = x.stride(0);
  p.bsy = y.stride(0);
  if (b.has_value()) {
    check_bf16(*b, "bias");
    TORCH_CHECK(b->numel() == Cout && b->is_contiguous(), "bias [Cout]");
    p.bias = bfp(*b);
  }
  // one utterance: split-K when the output tiles alone cannot fill the CUs (large-v3 conv2: 120
  // tiles x 30 k-groups); the f32 slabs are summed by gemm_reduce_kernel with the same epilogue
  Tensor ws;
  if (B == 1 && p.K >= 1024) {  // (K = 384: the split's f32 reduce costs more than it saves)
    const int s = vwa_gemm_splits(p.M, p.N, p.K, device_cus(x), (int64_t)1 << 25, 0);
    if (s > 1) {
      ws = at::empty({(int64_t)s * p.M * p.N}, x.options().dtype(at::kFloat));
      p.ws = ws.data_ptr<float>();
      p.splits = s;
    }
  }
  int epi = 3;
  if (pos.has_value()) {
    check_bf16(*pos, "pos");
    TORCH_CHECK(pos->dim() == 2 && pos->size(0) >= Tout && pos->size(1) == Cout && pos->stride(1) == 1 &&
                    pos->stride(0) % 8 == 0 && (reinterpret_cast<uintptr_t>(pos->data_ptr()) & 15) == 0,
                "pos [>= Tout, Cout] with 16-byte aligned rows");
    p.R = bfp(*pos);
    p.ldr = (int)pos->stride(0);
    p.bsr = 0;
    epi = 4;
  }
  check_rc(vwa_gemm(epi, &p, cur_stream(x)), "conv1d_gelu");
}

}  // namespace

void quant_fp8_rows(Tensor x, Tensor q, Tensor scale, c10::optional<Tensor> rstd, double eps) {
  c10::DeviceGuard g(x.device());
  check_bf16(x, "x");
  check_contig_rows(x, "x");
  TORCH_CHECK(q.scalar_type() == at::kFloat8_e4m3fn && q.is_contiguous() && q.sizes() == x.sizes(), "q fp8 [rows, D]");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() >= x.size(0), "scale f32 [rows]");
  if (rstd.has_value())
    TORCH_CHECK(rstd->scalar_type() == at::kFloat && rstd->numel() >= x.size(0), "rstd f32 [rows]");
  check_rc(vwa_quant_fp8_rows(bfp(x), (int)x.stride(0), (int)x.size(0), (int)x.size(1),
                              reinterpret_cast<uint8_t*>(q.data_ptr()), scale.data_ptr<float>(),
                              rstd.has_value() ? rstd->data_ptr<float>() : nullptr, (float)eps, cur_stream(x)),
           "quant_fp8_rows");
}

// ---- one-shot all-reduce (opaque state handle as int64)
// TP preflight (parallel/custom_ar.py): may device `dev` map device `peer`'s memory (xGMI P2P)?
// -1 when either index is not visible to this process
int64_t can_access_peer(int64_t dev, int64_t peer) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || dev < 0 || peer < 0 || dev >= n || peer >= n) return -1;
  if (dev == peer) return 1;
  int ok = 0;
  if (hipDeviceCanAccessPeer(&ok, (int)dev, (int)peer) != hipSuccess) return -1;
  return ok;
}

// PCI location "domain:bus:device" of a visible device (a stable id across processes' masks)
std::string pci_id(int64_t dev) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, (int)sizeof(buf), (int)dev) != hipSuccess) return "";
  return std::string(buf);
}

int64_t ar_create(int64_t rank, int64_t world, int64_t max_elems) {
  void* st = vwa_ar_create((int)rank, (int)world, max_elems);
  TORCH_CHECK(st, "all-reduce buffer allocation failed (world <= 8, max_elems % 512 == 0)");
  return reinterpret_cast<int64_t>(st);
}
Tensor ar_handles(int64_t st) {
  Tensor t = torch::empty({vwa_ar_handle_bytes()}, torch::dtype(torch::kUInt8));
  check_rc(vwa_ar_handles(reinterpret_cast<void*>(st), t.data_ptr()), "hipIpcGetMemHandle");
  return t;
}
void ar_open_peer(int64_t st, int64_t p, Tensor h) {
  TORCH_CHECK(h.scalar_type() == at::kByte && h.numel() == vwa_ar_handle_bytes() && !h.is_cuda(), "ipc handle bytes");
  check_rc(vwa_ar_open_peer(reinterpret_cast<void*>(st), (int)p, h.contiguous().data_ptr()), "hipIpcOpenMemHandle");
}
void ar_allreduce(int64_t st, Tensor in, Tensor out) {
  c10::DeviceGuard g(in.device());
  check_bf16(in, "in");
  check_bf16(out, "out");
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel(), "contiguous, same size");
  check_rc(vwa_ar_allreduce(reinterpret_cast<void*>(st), bfp(in), bfp_mut(out), in.numel(), cur_stream(in)),
           "one-shot all-reduce");
}
void ar_gather(int64_t st, Tensor in, Tensor out) {
  c10::DeviceGuard g(in.device());
  TORCH_CHECK(in.is_cuda() && in.scalar_type() == at::kInt && in.is_contiguous() && out.is_cuda() &&
                  out.scalar_type() == at::kInt && out.is_contiguous() && out.numel() % in.numel() == 0 &&
                  in.numel() <= vwa_ar_gather_max_words(),
              "ar_gather: int32 in [n], out [world * n] on the GPU");
  check_rc(vwa_ar_gather(reinterpret_cast<void*>(st), in.data_ptr<int>(), out.data_ptr<int>(), in.numel(),
                         cur_stream(in)),
           "one-shot all-gather");
}
int64_t ar_error(int64_t st) { return vwa_ar_error(reinterpret_cast<void*>(st)); }
void ar_destroy(int64_t st) { vwa_ar_destroy(reinterpret_cast<void*>(st)); }

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("quant_fp8_rows", &quant_fp8_rows, py::arg("x"), py::arg("q"), py::arg("scale"),
        py::arg("rstd") = py::none(), py::arg("eps") = 1e-5);
  m.def("can_access_peer", &can_access_peer);
  m.def("pci_id", &pci_id);
  m.def("ar_create", &ar_create);
  m.def("ar_handles", &ar_handles);
  m.def("ar_open_peer", &ar_open_peer);
  m.def("ar_allreduce", &ar_allreduce);
  m.def("ar_gather", &ar_gather);
  m.def("ar_error", &ar_error);
  m.def("ar_destroy", &ar_destroy);
  m.doc() = "MI355X (gfx950) HIP kernels for the voice-web-agent inference engine";
  m.def("skinny_gemm", &skinny_gemm, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("epi"),
        py::arg("fuse_rms"), py::arg("eps"), py::arg("residual"), py::arg("w_scale") = py::none(),
        py::arg("ln_c") = py::none(), py::arg("w_tiled") = false, py::arg("col_mask") = py::none(),
        py::arg("col_mask_off") = 0, py::arg("mask_rows") = 1);
  m.def("skinny_gemm_swiglu", &skinny_gemm_swiglu, py::arg("x"), py::arg("w_gu"), py::arg("bias"), py::arg("h"),
        py::arg("fuse_rms"), py::arg("eps"), py::arg("w_scale") = py::none(), py::arg("w_tiled") = false);
  m.def("skinny_gemm_qkv", &skinny_gemm_qkv, py::arg("x"), py::arg("w_qkv"), py::arg("bias"), py::arg("fuse_rms"),
        py::arg("eps"), py::arg("n_q_heads"), py::arg("n_kv_heads"), py::arg("head_dim"), py::arg("use_rope"),
        py::arg("positions"), py::arg("slots"), py::arg("rope"), py::arg("q_out"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("w_scale") = py::none(), py::arg("ln_c") = py::none(),
        py::arg("w_tiled") = false);
  m.def("chain_make", &chain_make, py::arg("h"), py::arg("att"), py::arg("act"), py::arg("w_o"), py::arg("w_gu"),
        py::arg("w_down"), py::arg("eps"), py::arg("w_qkv"), py::arg("n_q_heads"), py::arg("n_kv_heads"),
        py::arg("head_dim"), py::arg("positions"), py::arg("slots"), py::arg("rope"), py::arg("q_out"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("bar"), py::arg("work"), py::arg("ts") = py::none(), py::arg("bar_mode") = 1,
        py::arg("a_q") = py::none(), py::arg("a_k") = py::none(), py::arg("a_v") = py::none(),
        py::arg("a_table") = py::none(), py::arg("a_block_size") = 0, py::arg("a_sb") = 0, py::arg("a_sh") = 0,
        py::arg("a_st") = 0, py::arg("a_ctx") = py::none(), py::arg("a_seq") = py::none(), py::arg("a_scale") = 0.0,
        py::arg("a_n_splits") = 0, py::arg("a_part_o") = py::none(), py::arg("a_part_ml") = py::none(),
        py::arg("a_counters") = py::none(), py::arg("w_tiled") = false, py::arg("a_row_table") = py::none(),
        py::arg("s_o") = py::none(), py::arg("s_gu") = py::none(), py::arg("s_down") = py::none(),
        py::arg("s_qkv") = py::none(), py::arg("tp_ar") = 0, py::arg("a_plan") = py::none(), py::arg("a_plan_mode") = 0);
  m.def("set_small_gemm_bytes", &set_small_gemm_bytes);
  m.def("gemm_set_p8", [](int64_t mode) { vwa_gemm_set_p8((int)mode); });
  m.def("skinny_set_x_skew", [](int64_t skew) { vwa_skinny_set_x_skew((int)skew); });
  m.def("gemm_set_split_fill", [](int64_t pct) { vwa_gemm_set_split_fill((int)pct); });
  m.def("chain_make_seq", &chain_make_seq, py::arg("seq"), py::arg("X"), py::arg("W"), py::arg("bias"),
        py::arg("ln_c"), py::arg("Y"), py::arg("epi"), py::arg("eps"), py::arg("n_heads"), py::arg("head_dim"),
        py::arg("positions"), py::arg("slots"), py::arg("k_cache"), py::arg("v_cache"), py::arg("bar"),
        py::arg("work"), py::arg("bar_mode") = 1, py::arg("w_tiled") = false);
  m.def("chain_run", &chain_run, py::arg("desc"), py::arg("n_phases"), py::arg("lds"), py::arg("like"),
        py::arg("attn_g") = 0, py::arg("seq") = 0, py::arg("n_layers") = 1);
  m.def("alloc_uncached_i32", &alloc_uncached_i32);
  m.def("device_cus", [](Tensor like) { return (int64_t)device_cus(like); });
  m.def("wdec_layers", &wdec_layers, py::arg("flat"), py::arg("n_layers"), py::arg("like"));
  m.def("wdec_run", &wdec_run, py::arg("layers"), py::arg("roles"), py::arg("bufs"), py::arg("ints"), py::arg("eps"),
        py::arg("scale"), py::arg("n_prod"), py::arg("ts") = py::none(), py::arg("opt") = 0, py::arg("lm") = py::none(),
        py::arg("emb") = py::none(), py::arg("smp") = py::none(), py::arg("loop_base_block") = 0);
  m.def("decode_advance", &decode_advance);
  m.def("gemm", &gemm, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("y"), py::arg("epi"),
        py::arg("rstd") = py::none(), py::arg("residual") = py::none(), py::arg("w_tiled") = false,
        py::arg("ws") = py::none(), py::arg("ss_out") = py::none(), py::arg("ss_zero") = py::none(),
        py::arg("ss_in") = py::none(), py::arg("ss_eps") = 1e-5);
  m.def("row_rstd", &row_rstd);
  m.def("gemm_qkv", &gemm_qkv, py::arg("x"), py::arg("sx"), py::arg("w"), py::arg("sw"), py::arg("bias"),
        py::arg("rstd"), py::arg("w_tiled"), py::arg("ws"), py::arg("n_q_heads"), py::arg("n_kv_heads"),
        py::arg("head_dim"), py::arg("use_rope"), py::arg("positions"), py::arg("slots"), py::arg("rope"),
        py::arg("q_out"), py::arg("k_cache"), py::arg("v_cache"), py::arg("ss_in") = py::none(),
        py::arg("ss_eps") = 1e-5);
  m.def("gemm_fp8", &gemm_fp8, py::arg("x8"), py::arg("sx"), py::arg("w8"), py::arg("sw"), py::arg("bias"),
        py::arg("y"), py::arg("epi"), py::arg("rstd") = py::none(), py::arg("residual") = py::none(),
        py::arg("ws") = py::none(), py::arg("ss_out") = py::none(), py::arg("ss_zero") = py::none(),
        py::arg("ss_in") = py::none(), py::arg("ss_eps") = 1e-5);
  m.def("rmsnorm", &rmsnorm);
  m.def("layernorm", &layernorm);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("swiglu", &swiglu);
  m.def("bias_act", &bias_act);
  m.def("decode_attention", &decode_attention);
  m.def("flash_attention", &flash_attention);
  m.def("embedding", &embedding);
  m.def("sample", &sample, py::arg("logits"), py::arg("mask"), py::arg("temperature"), py::arg("seed"), py::arg("step"),
        py::arg("out_tokens"), py::arg("part_val"), py::arg("part_idx"), py::arg("fail_word") = py::none(),
        py::arg("v_offset") = 0);
  m.def("sample_tp", &sample_tp);
  m.def("pcm16_to_f32", &pcm16_to_f32);
  m.def("log_mel", &log_mel);
  m.def("conv1d_gelu", &conv1d_gelu);
  m.def("set_skinny_mode", &set_skinny_mode, py::arg("mode"), py::arg("grid_cap") = 256, py::arg("ks") = 0,
        py::arg("w_first") = 2);
  m.def("attention_split_tokens", []() { return vwa_attention_split_tokens(); });
  m.def("set_attention_impl", [](int64_t impl) { vwa_set_attention_impl((int)impl); });
}
