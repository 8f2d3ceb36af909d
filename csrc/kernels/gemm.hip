// LDS-tiled MFMA GEMM for the row counts the skinny decode kernels do not take (K12, M > 16):
// the prompt suffix prefill of the intent LLM (apps/brain/src/server.ts:98-105: ~1.1k-token
// prompt, the un-cached suffix), continuous-batching steps of 17..64 rows, and the Whisper
// encoder (1500 rows per utterance).  Replaces hipBLASLt for every projection of both models.
//
//   Y[M, N] = epi( rstd[m] * (X[M, K] . W[N, K]^T) )       X bf16 row-major, f32 accumulate
//
// W layouts:
//   * tiled (ops.tile_weight, the decode kernels' layout -- the model keeps ONE copy of each
//     weight): per 16-row tile T and 128-wide k-group kg a contiguous 4 KB block
//     [s 0..3][lane 0..63][8] with lane = 16 g + n holding W[16 T + n][128 kg + 32 g + 8 s + e],
//     i.e. exactly the MFMA B fragments: the block is copied to LDS verbatim;
//   * row-major [N, K] (Whisper weights, tests): each 16-byte piece is scattered into the same
//     fragment-ordered LDS image while staging.
// Because the B fragments use the k order 32 g + 8 s + e, the A fragment of lane (row r, g) in
// sub-step s is X[r][128 kg + 32 g + 8 s .. + 8): 16-byte chunk 4 g + s of the row's k-group.
//
// Tiling (gfx950, wave64): workgroup = 4 waves (2 x 2) computing a 128 x 128 output tile, one
// k-group (128 deep) per stage: A [128 rows][128 k] (32 KB, chunk-XOR swizzled: 16 lanes reading
// one chunk column of 16 rows hit 16 distinct 16-B slots -> conflict-free ds_read_b128) and B
// [8 tiles][4 s][64 lanes][8] (32 KB, fragment order -> every ds_read_b128 is 1 KB contiguous).
// Each wave owns 64 x 64 = 4 x 4 MFMA tiles (mfma_f32_16x16x32_bf16, 64 MFMAs per stage).
// Software pipeline: the next stage's global loads are issued into registers before this
// stage's MFMAs, written to LDS after them (one LDS buffer, 64 KB -> 2 workgroups per CU).
// Grid: (row blocks x column blocks) remapped XCD-aware so the row blocks of one column block
// (same weight tile) share an XCD's L2, x split-K slices when the tile count alone cannot
// fill the 256 CUs (weight-streaming shapes: few rows) -- slices write f32 partials, a second
// kernel sums them and applies the epilogue.
//
// Epilogues (fused, after the optional per-row RMSNorm scale rstd -- gammas are folded into W):
//   0 store (+bias; bf16 or f32 out)   1 residual add (+bias)   2 SwiGLU over gate/up tiles
//   interleaved per 16 rows (ops.interleave_gate_up)   3 GELU (+bias)   4 GELU (+bias) then a
//   residual add (the Whisper conv stem's positional embedding: y = gelu(conv + b) + pos)
//
// Implicit-GEMM convolution (K3, ops.conv1d_gelu): X rows are ldx apart and K long, so a k=3
// conv over a zero-padded channels-last buffer is X row t = padded rows t*stride .. t*stride+2
// (ldx = stride*Cin, K = 3*Cin) -- the A tiles are staged through the same LDS-DMA pipeline.
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GELU = 3, EPI_GELU_RESID = 4, EPI_QKV = 5 };
template <int EPI> constexpr bool kResid = EPI == EPI_RESID || EPI == EPI_GELU_RESID;
template <int EPI> constexpr bool kGelu = EPI == EPI_GELU || EPI == EPI_GELU_RESID;

constexpr int BKG = 128;

// Workgroup shapes: BM x BN output tile, WM x WN waves, each wave (BM/WM) x (BN/WN).
//   Cfg<128, 128, 2, 2>: 4 waves of 64 x 64, 64 KB LDS -> 2 workgroups per CU -- the one in use.
//   (Measured and dropped: Cfg<256, 256, 2, 4>, 8 waves of 128 x 64, which reads 25 % fewer
//   fragment bytes from LDS per MFMA: 929 vs 915 TF/s on the 1011-row gate/up projection and
//   2-3x SLOWER on 1011-row o / down -- 64 workgroups cannot fill 256 CUs;
//   profiles/r3_gemm_bench.md.)
template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, NW = WM_ * WN_, THREADS = 64 * NW;
  static constexpr int FM = BM / WM / 16, FN = BN / WN / 16;  // MFMA fragments per wave
  static constexpr int A_BYTES = BM * 128, STAGE = BM * 128 + BN * 128;
  // W8A16 stage: a full k-group -- two bf16 A half images + the fp8 B block of every tile
  static constexpr int W8STAGE = 2 * BM * 128 + BN * 128;
  static constexpr int NCOL_MAX = BN / WN;
  static constexpr int EPI_LDS = NW * (FM * 16) * (NCOL_MAX * 2 + 16);
  static constexpr int LDS = 2 * STAGE > EPI_LDS ? 2 * STAGE : EPI_LDS;
  static constexpr int W8LDS = 2 * W8STAGE > EPI_LDS ? 2 * W8STAGE : EPI_LDS;
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "whole LDS-DMA instructions per wave");
};
using CfgS = Cfg<128, 128, 2, 2>;
// W8A16 decode tile (<= 64 rows: one row block): 64 x 128, 4 waves of 64 x 32, 32 KB stages (16 KB
// of fp8 weights each -- the W8A8 kernel's weight bytes per stage: a half-k-group bf16-style stage
// carried 8 KB and measured 1.25x slower whole decode steps), 2 workgroups per CU
using CfgW8 = Cfg<64, 128, 1, 4>;

// A-image slot swizzle: chunk c of row r sits at slot c ^ F((r >> 1) & 7).  F makes every
// ds_read_b128 lane group ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ... : two k-chunk columns g,
// 16 rows) hit 16 distinct (row parity, slot) bank groups: F maps the half-row indices
// {0,1,6,7} to the even slots and {2,3,4,5} to the odd ones, so XOR-ing the chunk index with 2
// (the other column of the group) cannot collide.  (Plain c ^ h measured 33 % bank conflicts.)
VWA_DEVICE int swz(int h) { return (0x64753120 >> (4 * h)) & 7; }

// buffer resource over [base, base + bytes): loads past the end return zero (rows >= M, weight
// tiles >= N), so the stage issue needs no bounds branches
VWA_DEVICE __amdgpu_buffer_rsrc_t rsrc(const void* base, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes < 0x7FFFFFF0ull ? bytes : 0x7FFFFFF0ull), 0x00020000);
}

VWA_DEVICE void dma16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0, 0,
                                           0);
}

// Stage hs of the block's tile (bf16: half k-group hs = 2 kg + h, k = 128 kg + 32 g + 16 h + 8 s'
// + e, s' = 0, 1), LDS-DMA'd straight into buffer `buf` (no registers): 8 wave-instructions of
// 1 KB per thread.  Each wave-instruction's LDS destination is lane-linear (base + 16 lane), so
// the A swizzle is applied on the per-lane SOURCE address (and undone on the read):
//   A image [BM rows][8 chunks of 16 B], chunk c = 2 g + s' at slot c ^ swz((row >> 1) & 7)
//   B image [BN/16 tiles][2 s'][64 lanes][16 B]: the tiled weight's fragment blocks verbatim (a
//     row-major weight gathers each lane's fragment from its row instead)
// F8 (W8A8): one FULL k-group per stage (16 fp8 = 16 B per chunk): A chunk c = 2 g + s2 holds
// X8[row][128 kg + 32 g + 16 s2 .. + 16), B the fp8 tiled block [s2][lane][16 B] of the tile
// (ops.tile_weight_fp8) -- the same stage images as a bf16 half k-group.
// W8 (W8A16, CfgW8): one FULL k-group per stage -- X as the two bf16 half-k-group A images (each as
// above) and B the fp8 tiled k-group of every tile verbatim ([tile][s2][lane][16 B]: block s2 = h
// holds the lane's k 32 g + 16 h .. + 16, both sub-steps of half h), converted to bf16 fragments on
// the LDS read -- no quantised copy of X, half the weight bytes of bf16.
template <class C, bool WT, bool F8, bool W8 = false>
VWA_DEVICE void issue_stage(const GemmParams& p, __amdgpu_buffer_rsrc_t rx, __amdgpu_buffer_rsrc_t rw, int bm,
                            int bn, int hs, char* buf) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kg = F8 || W8 ? hs : hs >> 1;
#pragma unroll
  for (int hh = 0; hh < (W8 ? 2 : 1); ++hh) {  // (W8: both bf16 half images of the k-group)
  const int ha = W8 ? hh : F8 ? 0 : hs & 1;
#pragma unroll
  for (int it = 0; it < C::BM / 8 / C::NW; ++it) {
    const int q = it * C::NW + w;  // wave-instruction index: rows 8q .. 8q + 7
    const int r = 8 * q + (lane >> 3), c = (lane & 7) ^ swz((r >> 1) & 7);
    const int m = bm + r;
    unsigned off;
    if constexpr (F8)
      off = (unsigned)((size_t)m * p.ldx + (size_t)kg * BKG + 32 * (c >> 1) + 16 * (c & 1));
    else
      off = (unsigned)(((size_t)m * p.ldx + (size_t)kg * BKG + 32 * (c >> 1) + 16 * ha + 8 * (c & 1)) * 2);
    dma16(rx, buf + hh * C::A_BYTES + q * 1024, m < p.M ? off : 0xFFFFFFF0u);
  }
  }
  const int kgn = p.K / BKG;
  const int h = F8 || W8 ? 0 : hs & 1;
  if constexpr (W8) {  // the fp8 blocks of the whole k-group, [tile][s2][lane][16 B]
#pragma unroll
    for (int it = 0; it < C::BN / 8 / C::NW; ++it) {
      const int q = it * C::NW + w, T = (bn >> 4) + (q >> 1);
      const unsigned off = T * 16 < p.N ? (unsigned)(((size_t)T * kgn + kg) * 2048 + (q & 1) * 1024 + lane * 16) : 0xFFFFFFF0u;
      dma16(rw, buf + 2 * C::A_BYTES + q * 1024, off);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < C::BN / 8 / C::NW; ++it) {
    const int q = it * C::NW + w;  // tile q >> 1, sub-step s' = q & 1
    const int tile = q >> 1, sp = q & 1;
    unsigned off;
    if constexpr (F8) {
      const int T = (bn >> 4) + tile;
      off = T * 16 < p.N ? (unsigned)(((size_t)T * kgn + kg) * 2048 + sp * 1024 + lane * 16) : 0xFFFFFFF0u;
    } else if constexpr (WT) {
      const int T = (bn >> 4) + tile;
      off = T * 16 < p.N ? (unsigned)((((size_t)T * kgn + kg) * 2048 + (2 * h + sp) * 512 + lane * 8) * 2) : 0xFFFFFFF0u;
    } else {
      const int n = bn + tile * 16 + (lane & 15), g = lane >> 4;
      off = n < p.N ? (unsigned)(((size_t)n * p.K + (size_t)kg * BKG + 32 * g + 16 * h + 8 * sp) * 2) : 0xFFFFFFF0u;
    }
    dma16(rw, buf + C::A_BYTES + q * 1024, off);
  }
}

template <class C, bool F8, bool W8 = false>
VWA_DEVICE void compute_stage(const char* buf, f32x4 (&acc)[C::FM][C::FN], int wm, int wn) {
  const int l = lane_id();
  const int rl = l & 15, g = l >> 4;
  const char* la = buf + (wm * C::FM * 16 + rl) * 128;
  const char* lb = buf + C::A_BYTES + (wn * C::FN) * 2048 + l * 16;
  if constexpr (W8) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
    // 16 e4m3 per lane and tile (both sub-steps of half h), read once; the per-row weight scale is
    // applied to the finished column in the epilogue
    uint4 w8[C::FN];
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
      w8[j] = *reinterpret_cast<const uint4*>(buf + 2 * C::A_BYTES + (wn * C::FN + j) * 2048 + h * 1024 + l * 16);
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      bf16x8 a[C::FM], b[C::FN];
      const int ch = ((2 * g + sp) ^ swz(rl >> 1)) << 4;
#pragma unroll
      for (int i = 0; i < C::FM; ++i) a[i] = *reinterpret_cast<const bf16x8*>(la + h * C::A_BYTES + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) {
        const unsigned d0 = sp ? w8[j].z : w8[j].x, d1 = sp ? w8[j].w : w8[j].y;
        uint4 bw;
        bw.x = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false));
        bw.y = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true));
        bw.z = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false));
        bw.w = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true));
        b[j] = as_bf16x8(bw);
      }
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    }
    }
  } else if constexpr (F8) {
    // one 128-deep MX MFMA per fragment pair: lane (row / column, g) supplies the 32 fp8 of
    // k 32 g .. 32 g + 32 -- A chunks 2 g and 2 g + 1 of the swizzled image, B blocks s2 = 0, 1 of
    // the fp8 tiled layout -- each read with one ds_read_b128 (conflict-free, as the bf16 path).
    // (The earlier 16x16x32 form read 8-byte halves, which the compiler merged into
    // ds_read2st64_b64 -- 16-lane groups on 32 banks: 49.8 % LDS bank conflicts,
    // profiles/r3_pmc_fp8_chain.md -- and ran at the bf16 MFMA rate.)
    i32x8 a[C::FM], b[C::FN];
    const int c0 = ((2 * g) ^ swz(rl >> 1)) << 4, c1 = ((2 * g + 1) ^ swz(rl >> 1)) << 4;
#pragma unroll
    for (int i = 0; i < C::FM; ++i) {
      const uint4 lo = *reinterpret_cast<const uint4*>(la + i * 16 * 128 + c0);
      const uint4 hi = *reinterpret_cast<const uint4*>(la + i * 16 * 128 + c1);
      a[i] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
      const uint4 lo = *reinterpret_cast<const uint4*>(lb + j * 2048);
      const uint4 hi = *reinterpret_cast<const uint4*>(lb + j * 2048 + 1024);
      b[j] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
      for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16x128_fp8(a[i], b[j], acc[i][j]);
  } else {
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      bf16x8 a[C::FM], b[C::FN];
      const int ch = ((2 * g + sp) ^ swz(rl >> 1)) << 4;  // ((row >> 1) & 7) == rl >> 1 for every fragment row
#pragma unroll
      for (int i = 0; i < C::FM; ++i) a[i] = *reinterpret_cast<const bf16x8*>(la + i * 16 * 128 + ch);
#pragma unroll
      for (int j = 0; j < C::FN; ++j) b[j] = *reinterpret_cast<const bf16x8*>(lb + j * 2048 + sp * 1024);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
    }
  }
}

// ---- 256 x 256 tile, 8 waves (2 x 4, each 128 x 64), 8-phase software pipeline (the guide's
// "256^2 8-phase template": the 128^2 two-barrier loop above is capped near 900 TF/s because each
// stage's DMA is drained by the barrier that publishes it).  A stage (one bf16 half k-group, 64
// deep) is four half-tile images of 16 KB -- A-lo (rows 0-127), A-hi (rows 128-255), B-lo
// (n-tiles 0-7), B-hi (8-15) -- in the same layouts as the 128^2 kernel.  Each stage runs 4
// phases of 16 MFMAs per wave (one C quadrant: 4 row x 2 column fragments x 2 k-substeps):
//   P0 reads A 0-3 + B 0-1, P1 B 2-3, P2 A 4-7, P3 B 0-1 (A stays in registers across P0/P1 and
//   P2/P3), with the next stages' half-tiles DMA'd behind them: P0 A-hi + B-lo and P1 B-hi of
//   stage s+1 (into the other buffer, free since the end of stage s-1), P3 A-lo of stage s+2
//   (into this buffer: its A halves were last read in P2).  The only wait on the DMA is a counted
//   vmcnt in P3 (A-lo of s+2 stays in flight).  The two wave groups (M halves) run one barrier
//   apart, so one group's LDS reads overlap the other group's MFMAs; every phase retires its reads
//   (lgkmcnt) before its first barrier, so a restage issued after that barrier by the other group
//   cannot overwrite bytes still being read, and every staged byte is read after a barrier that
//   follows every issuing wave's counted wait.
constexpr int kP8Half = 16384;
using CfgP8 = Cfg<256, 256, 2, 4>;

// half-tile `which` (0 A-lo, 1 A-hi, 2 B-lo, 3 B-hi) of stage hs into the stage image `st`:
// 16 wave-instructions of 1 KB = 2 per wave (tiled bf16 weights only)
VWA_DEVICE void p8_issue(const GemmParams& p, __amdgpu_buffer_rsrc_t rx, __amdgpu_buffer_rsrc_t rw, int bm, int bn,
                         int hs, int which, char* st) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kg = hs >> 1, h = hs & 1;
  const int kgn = p.K / BKG;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int q = it * 8 + w;
    if (which < 2) {
      const int qa = 16 * which + q;  // rows 8 qa .. 8 qa + 7
      const int r = 8 * qa + (lane >> 3), c = (lane & 7) ^ swz((r >> 1) & 7);
      const int m = bm + r;
      const unsigned off =
          (unsigned)(((size_t)m * p.ldx + (size_t)kg * BKG + 32 * (c >> 1) + 16 * h + 8 * (c & 1)) * 2);
      dma16(rx, st + qa * 1024, m < p.M ? off : 0xFFFFFFF0u);
    } else {
      const int tile = 8 * (which - 2) + (q >> 1), sp = q & 1;
      const int T = (bn >> 4) + tile;
      const unsigned off =
          T * 16 < p.N ? (unsigned)((((size_t)T * kgn + kg) * 2048 + (2 * h + sp) * 512 + lane * 8) * 2) : 0xFFFFFFF0u;
      dma16(rw, st + CfgP8::A_BYTES + (2 * tile + sp) * 1024, off);
    }
  }
}

// one phase: 16 MFMAs acc[i0 .. i0+3][j0 .. j0+1] over both k-substeps of the stage
template <int I0, int J0>
VWA_DEVICE void p8_mfma(f32x4 (&acc)[8][4], const bf16x8 (&a)[4][2], const bf16x8 (&b)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int sp = 0; sp < 2; ++sp)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[I0 + i][J0 + j] = mfma16(a[i][sp], b[j][sp], acc[I0 + i][J0 + j]);
  __builtin_amdgcn_s_setprio(0);
}

VWA_DEVICE float bias_at(const GemmParams& p, int n) { return p.bias ? bf2f(p.bias[n]) : 0.f; }

// RMS statistics hand-off (GemmParams::ss_*): sums of squares in u64 fixed point, 2^-24 units,
// each partial rounded to nearest (truncation biased every atomic add down by up to one unit --
// visible on small-norm rows).  Headroom: 2^64 / 2^24 ~ 1.1e12 per row sum; one partial is
// clamped to 9.2e18 so a handful of them cannot wrap the counter.
constexpr double kSsScale = 16777216.0;
VWA_DEVICE unsigned long long ss_fix(float sq) {
  return (unsigned long long)fminf(sq * (float)kSsScale + 0.5f, 9.2e18f);  // (>= 0)
}

// per-row RMSNorm scale: rstd[m], or from the handed-off sum of squares (ss_in), or 1
VWA_DEVICE float row_scale(const GemmParams& p, int m) {
  if (p.rstd) return p.rstd[m];
  if (p.ss_in) return rsqrtf((float)((double)p.ss_in[m] * (1.0 / kSsScale)) / (float)p.K + p.ss_eps);
  return 1.f;
}

template <int EPI>
VWA_DEVICE void store_out(const GemmParams& p, int m, int n, float v) {
  if constexpr (kResid<EPI>) v += bf2f(p.R[(size_t)m * p.ldr + n]);
  if (p.y_f32)
    reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
  else
    reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + n] = f2bf(v);
}

// EPI_QKV: output chunk n .. n+7 (o) of row m and its rotation partner n^8 (q) -> rotary (q / k
// heads) -> q_out or the paged K / V caches, 16-byte stores.  Within a head (permuted rows) the
// chunk at column 16 t + 8 hi holds dims hi * hd/2 + 8 t .. + 8, its partner the other half.
VWA_DEVICE void qkv_store(const GemmParams& p, int m, int n, const float (&o)[8], const float (&q)[8]) {
  const int hd = p.head_dim, half = hd >> 1;
  const int head = n / hd, wc = n % hd;
  const int t = wc >> 4;
  const bool hi = (wc & 8) != 0;
  const bool is_v = head >= p.n_q_heads + p.n_kv_heads;
  float y[8];
  if (p.use_rope && !is_v) {
    const float4* cs = reinterpret_cast<const float4*>(p.rope + ((size_t)p.positions[m] * half + 8 * t) * 2);
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      const float4 v = cs[e2];  // (cos, sin) of dims 2 e2, 2 e2 + 1
      const int e = 2 * e2;
      y[e] = hi ? o[e] * v.x + q[e] * v.y : o[e] * v.x - q[e] * v.y;
      y[e + 1] = hi ? o[e + 1] * v.z + q[e + 1] * v.w : o[e + 1] * v.z - q[e + 1] * v.w;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) y[e] = o[e];
  }
  const int d = (hi ? half : 0) + 8 * t;
  if (head < p.n_q_heads) {
    *reinterpret_cast<uint4*>(p.q_out + (size_t)m * p.ldq + head * hd + d) = pack8(y);
    return;
  }
  const int64_t slot = p.slots[m];
  if (slot < 0) return;
  const int kvh = is_v ? head - p.n_q_heads - p.n_kv_heads : head - p.n_q_heads;
  const int64_t idx = (slot / p.block_size) * p.cache_sb + kvh * p.cache_sh + (slot % p.block_size) * p.cache_st;
  *reinterpret_cast<uint4*>((is_v ? p.v_cache : p.k_cache) + idx + d) = pack8(y);
}

// f32 partial slab loads of the split-K reduce (AUX: buffer cache bits; the reduce runs after the
// GEMM launch's end made the slabs visible, so plain loads)
template <int AUX>
VWA_DEVICE float4 ld_f4(__amdgpu_buffer_rsrc_t r, size_t idx) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, AUX));
}

VWA_DEVICE void add8(float (&v)[8], const float4& a, const float4& b) {
  v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w; v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
}

// Split-K output items: row m, output columns c .. c+7 -- the sum of every slice's f32 partial
// (slice order: the result does not depend on which slice finished last) and the epilogue
// (SwiGLU: features c .. c+7 from the interleaved gate / up columns; QKV: also the rotation
// partner chunk c^8, then rotary + q / KV stores), 16-byte stores.
//   src0 / src1: the item's two 8-column source chunks (SwiGLU gate / up; QKV own / partner)
template <int EPI>
VWA_DEVICE int item_src0(int c) { return EPI == EPI_SWIGLU ? (c >> 4) * 32 + (c & 15) : c; }
template <int EPI>
VWA_DEVICE int item_src1(int c) { return EPI == EPI_SWIGLU ? item_src0<EPI>(c) + 16 : (c ^ 8); }
template <int EPI>
constexpr bool kTwoSrc = EPI == EPI_SWIGLU || EPI == EPI_QKV;

// sums a (src0) / b (src1) of NI items (row m, first columns c[i]); the slices in batches of ZB,
// all of a batch's loads (every item) in flight before any is used; slices past the last read
// past the slab range (the buffer returns zeros)
template <int EPI, int AUX, int NI, int ZB>
VWA_DEVICE void sum_items(const GemmParams& p, __amdgpu_buffer_rsrc_t rws, int m, const int (&c)[NI],
                          const bool (&ok)[NI], float (&a)[NI][8], float (&b)[NI][8]) {
  const size_t slab = (size_t)p.M * p.N;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) a[i][e] = b[i][e] = 0.f;
  for (int z0 = 0; z0 < p.splits; z0 += ZB) {
    float4 x[NI][ZB][2], y[NI][ZB][2];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int u = 0; u < ZB; ++u) {
        const size_t base = (size_t)(z0 + u) * slab + (size_t)m * p.N;
        const int n0 = item_src0<EPI>(c[i]), n1 = item_src1<EPI>(c[i]);
        // (an item past the row end reads offset 0 of slice z: in range, discarded)
        x[i][u][0] = ld_f4<AUX>(rws, ok[i] ? base + n0 : 0);
        x[i][u][1] = ld_f4<AUX>(rws, ok[i] ? base + n0 + 4 : 0);
        if constexpr (kTwoSrc<EPI>) {
          y[i][u][0] = ld_f4<AUX>(rws, ok[i] ? base + n1 : 0);
          y[i][u][1] = ld_f4<AUX>(rws, ok[i] ? base + n1 + 4 : 0);
        }
      }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int u = 0; u < ZB; ++u) {
        add8(a[i], x[i][u][0], x[i][u][1]);
        if constexpr (kTwoSrc<EPI>) add8(b[i], y[i][u][0], y[i][u][1]);
      }
  }
}

// epilogue of one summed item + its stores
// returns the sum of squares of the stored bf16 values (residual epilogue with ss_out; else 0)
template <int EPI>
VWA_DEVICE float finish_item(const GemmParams& p, int m, int c, const float (&a)[8], float (&b)[8]) {
  const float rs = row_scale(p, m) * (p.sx ? p.sx[m] : 1.f);
  const int n0 = item_src0<EPI>(c), n1 = item_src1<EPI>(c);
  float v[8];
  if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gs = p.sw ? p.sw[n0 + e] : 1.f, us = p.sw ? p.sw[n1 + e] : 1.f;
      v[e] = silu(a[e] * gs * rs) * (b[e] * us * rs);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = a[e] * rs * (p.sw ? p.sw[c + e] : 1.f) + bias_at(p, c + e);
      if constexpr (kGelu<EPI>) v[e] = gelu_erf(v[e]);
    }
    if constexpr (EPI == EPI_QKV) {
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = b[e] * rs * (p.sw ? p.sw[n1 + e] : 1.f) + bias_at(p, n1 + e);
      qkv_store(p, m, c, v, b);
      return 0.f;
    }
  }
  if (p.y_f32) {
#pragma unroll
    for (int e = 0; e < 8; ++e) store_out<EPI>(p, m, c + e, v[e]);
    return 0.f;
  }
  if constexpr (kResid<EPI>) {
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>(p.R + (size_t)m * p.ldr + c), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  const uint4 o = pack8(v);
  *reinterpret_cast<uint4*>(reinterpret_cast<u16*>(p.Y) + (size_t)m * p.ldy + c) = o;
  float sq = 0.f;
  if (kResid<EPI> && p.ss_out) {
    unpack8(o, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) sq += v[e] * v[e];
  }
  return sq;
}

// ss_out[m] += sq summed over the wave's lanes of each row (lanes with m < 0 add nothing): one
// atomic per row per wave when the wave lies in one row, else one per lane
VWA_DEVICE void ss_add(unsigned long long* ss_out, int m, float sq) {
  const int m0 = __builtin_amdgcn_readfirstlane(m);
  if (__ballot(m != m0) == 0ull) {
    sq = wave_sum(sq);
    if (lane_id() == 0 && m0 >= 0)
      __hip_atomic_fetch_add(gp(ss_out + m0), ss_fix(sq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (m >= 0) {
    __hip_atomic_fetch_add(gp(ss_out + m), ss_fix(sq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int EPI, int AUX>
VWA_DEVICE float reduce_item(const GemmParams& p, __amdgpu_buffer_rsrc_t rws, int m, int c) {
  const int cc[1] = {c};
  const bool ok[1] = {true};
  float a[1][8], b[1][8];
  sum_items<EPI, AUX, 1, 4>(p, rws, m, cc, ok, a, b);
  return finish_item<EPI>(p, m, c, a[0], b[0]);
}

// (round 4's 4-stage variant for one-row-block GEMMs measured slower in whole decode steps -- 128 KB
// of LDS leaves one workgroup per CU, so split-K grids above 256 workgroups ran in two rounds:
// fp8 32 rows 4.97 vs 4.36 ms, profiles/r4_gemm_ab.md -- and was removed in round 5)
template <class C, int EPI, bool WT, bool F8 = false, bool P8 = false, bool W8 = false>
__global__ __launch_bounds__(C::THREADS, C::NW == 4 ? 2 : 1) void gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int FM = C::FM, FN = C::FN;
  const int mb = (p.M + C::BM - 1) / C::BM, nb = (p.N + C::BN - 1) / C::BN;
  const int tiles = mb * nb;
  const int split = blockIdx.x / tiles % p.splits;  // split-K slice (blocks of one slice are contiguous)
  if (p.nbatch > 1) {  // batch z = blockIdx.x / (tiles * splits), splits == 1 (vwa_gemm)
    const int z = blockIdx.x / tiles;
    p.X += (size_t)z * p.bsx;
    p.Y = reinterpret_cast<char*>(p.Y) + (size_t)z * p.bsy * (p.y_f32 ? 4 : 2);
    if (p.R) p.R += (size_t)z * p.bsr;
  }
  // XCD-aware: logical tile order is column-block major, so consecutive logical tiles (same XCD)
  // share the column block's weight tile in L2
  if (p.ss_zero && blockIdx.x == 0)
    for (int i = threadIdx.x; i < p.ss_zero_n; i += C::THREADS) p.ss_zero[i] = 0ull;
  const int lt = xcd_remap((int)(blockIdx.x % tiles), tiles);
  const int bn = (lt / mb) * C::BN, bm = (lt % mb) * C::BM;
  const int KG = p.K / BKG;
  const int kg0 = split * p.kg_per_split, kg1 = min(KG, kg0 + p.kg_per_split);
  const int w = threadIdx.x >> 6, wm = w / C::WN, wn = w % C::WN;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // pipeline: two LDS buffers, the next stage's DMA in flight during this one's MFMAs; raw
  // barriers with counted vmcnt (a __syncthreads would drain the in-flight DMA)
  constexpr int SPG = F8 || W8 ? 1 : 2;  // stages per k-group
  constexpr int STG = W8 ? C::W8STAGE : C::STAGE;
  static_assert(W8 ? 2 * (C::BM / 8 / C::NW) + C::BN / 8 / C::NW == 8 : C::BM / 8 / C::NW + C::BN / 8 / C::NW == 8,
                "8 LDS-DMA instructions per thread per stage (the counted vmcnt)");
  const int h0 = SPG * kg0, nh = SPG * (kg1 - kg0);
  // X extent: the last row starts at (M-1)*ldx and is K long (rows may overlap: conv views)
  const __amdgpu_buffer_rsrc_t rx = rsrc(p.X, ((size_t)(p.M - 1) * p.ldx + p.K) * (F8 ? 1 : 2));
  const __amdgpu_buffer_rsrc_t rw = rsrc(p.W, (size_t)p.N * p.K * (F8 || W8 ? 1 : 2));
  if constexpr (P8) {
    static_assert(C::BM == 256 && C::BN == 256 && C::NW == 8 && WT && !F8, "8-phase pipeline: CfgP8, tiled bf16");
    const int l = lane_id(), rl = l & 15, g = l >> 4;
    auto stage = [&](int s) { return lds + (s & 1) * C::STAGE; };
    if (nh > 0) {
#pragma unroll
      for (int hq = 0; hq < 4; ++hq) p8_issue(p, rx, rw, bm, bn, h0, hq, stage(0));
    }
    if (nh > 1) p8_issue(p, rx, rw, bm, bn, h0 + 1, 0, stage(1));
    if (nh > 1) asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    bf16x8 a[4][2], b[2][2];
    if (wm == 1) asm volatile("s_barrier" ::: "memory");  // group 1 runs one barrier behind group 0
    for (int s = 0; s < nh; ++s) {
      const char* st = stage(s);
      const char* la = st + (wm * 128 + rl) * 128;
      const char* lb = st + C::A_BYTES + (wn * 4) * 2048 + l * 16;
      auto read_a = [&](int i0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            a[i][sp] = *reinterpret_cast<const bf16x8*>(la + (i0 + i) * 16 * 128 + (((2 * g + sp) ^ swz(rl >> 1)) << 4));
      };
      auto read_b = [&](int j0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) b[j][sp] = *reinterpret_cast<const bf16x8*>(lb + (j0 + j) * 2048 + sp * 1024);
      };
      const bool n1 = s + 1 < nh, n2 = s + 2 < nh;
      // phase = operand reads (+ DMA issue) ; lgkmcnt(0) ; barrier ; 16 MFMAs ; barrier.  The two
      // wave groups (wm) run one barrier apart, so one group's reads overlap the other's MFMAs, and
      // a buffer's reads are retired (lgkmcnt) before the barrier that lets the other group restage it
      // P0
      read_a(0);
      read_b(0);
      if (n1) {
        p8_issue(p, rx, rw, bm, bn, h0 + s + 1, 1, stage(s + 1));
        p8_issue(p, rx, rw, bm, bn, h0 + s + 1, 2, stage(s + 1));
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      p8_mfma<0, 0>(acc, a, b);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      // P1
      read_b(2);
      if (n1) p8_issue(p, rx, rw, bm, bn, h0 + s + 1, 3, stage(s + 1));
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      p8_mfma<0, 2>(acc, a, b);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      // P2
      read_a(4);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      p8_mfma<4, 2>(acc, a, b);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
      // P3 (A-lo of this buffer was last read in P2: restage it with stage s + 2).  Stage s + 1 has
      // landed for this wave (only A-lo of s + 2 may stay in flight) before this phase's first
      // barrier; with the groups a barrier apart every wave has waited by the barrier that ends the
      // phase, and the next stage is read only after it
      read_b(0);
      if (n2) p8_issue(p, rx, rw, bm, bn, h0 + s + 2, 0, stage(s + 2));
      __builtin_amdgcn_sched_barrier(0);
      if (n2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      p8_mfma<4, 0>(acc, a, b);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_barrier" ::: "memory");
    }
    if (wm == 0) asm volatile("s_barrier" ::: "memory");  // (group 1 started one barrier later)
  } else {
  if (nh > 0) issue_stage<C, WT, F8, W8>(p, rx, rw, bm, bn, h0, lds);
  if (nh > 1) issue_stage<C, WT, F8, W8>(p, rx, rw, bm, bn, h0 + 1, lds + STG);
  for (int i = 0; i < nh; ++i) {
    if (i + 1 < nh)
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");  // this stage landed everywhere
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    compute_stage<C, F8, W8>(lds + (i & 1) * STG, acc, wm, wn);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave done reading it
    if (i + 2 < nh) issue_stage<C, WT, F8, W8>(p, rx, rw, bm, bn, h0 + i + 2, lds + (i & 1) * STG);
  }
  }
  const int l = lane_id();
  const int col0 = bn + wn * FN * 16 + (l & 15);
  const int row0 = bm + wm * FM * 16 + 4 * (l >> 4);
  if (p.splits > 1) {  // f32 partial slab of this slice; gemm_reduce_kernel applies the epilogue
    float* ws = p.ws + (size_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row0 + i * 16 + r;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = col0 + j * 16;
          if (n < p.N) ws[(size_t)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }
  // per-lane epilogue operands loaded once (no load-or-constant select per element)
  float bz[FN], cz[FN], rsv[FM][4];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    bz[j] = 0.f;
    cz[j] = 1.f;
  }
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < FN; ++j) bz[j] = col0 + j * 16 < p.N ? bf2f(p.bias[col0 + j * 16]) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) rsv[i][r] = 1.f;
  if (p.rstd || p.ss_in) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) rsv[i][r] = row0 + i * 16 + r < p.M ? row_scale(p, row0 + i * 16 + r) : 1.f;
  }
  // W8A8: acc * sx[m] * sw[n] (SwiGLU: gate / up columns scale before the activation); W8A16: sw only
  if constexpr (F8 || W8) {
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) rsv[i][r] *= row0 + i * 16 + r < p.M ? p.sx[row0 + i * 16 + r] : 1.f;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) cz[j] = col0 + j * 16 < p.N ? p.sw[col0 + j * 16] : 0.f;
  }
  if (p.y_f32) {  // f32 logits (rare: prefill LM head rows) -- direct stores
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row0 + i * 16 + r;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = col0 + j * 16;
          if (n >= p.N) continue;
          float v = acc[i][j][r] * rsv[i][r] * cz[j] + bz[j];
          if constexpr (kGelu<EPI>) v = gelu_erf(v);
          if constexpr (kResid<EPI>) v += bf2f(p.R[(size_t)m * p.ldr + n]);
          reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
        }
      }
    return;
  }
  // bf16 out: the wave's tile goes through LDS (padded rows: the four row groups of a store hit
  // different banks) and leaves as 16-byte row chunks -- coalesced stores, 16-byte residual reads
  constexpr int NCOL = EPI == EPI_SWIGLU ? FN * 8 : FN * 16;  // output columns of this wave
  constexpr int RS = NCOL * 2 + (NCOL == 32 ? 32 : 16);       // LDS row stride (bytes, 16-aligned)
  constexpr int ROWS = FM * 16;
  char* wl = lds + w * (ROWS * RS);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = i * 16 + 4 * (l >> 4) + r;
      if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
        for (int j = 0; j < FN; j += 2) {
          const float gt = acc[i][j][r] * rsv[i][r] * cz[j], up = acc[i][j + 1][r] * rsv[i][r] * cz[j + 1];
          *reinterpret_cast<u16*>(wl + rl * RS + ((j >> 1) * 16 + (l & 15)) * 2) = f2bf(silu(gt) * up);
        }
      } else {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          float v = acc[i][j][r] * rsv[i][r] * cz[j] + bz[j];
          if constexpr (kGelu<EPI>) v = gelu_erf(v);
          *reinterpret_cast<u16*>(wl + rl * RS + (j * 16 + (l & 15)) * 2) = f2bf(v);
        }
      }
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  constexpr int CPR = NCOL / 8;  // 16-byte chunks per row
  const int ncols = EPI == EPI_SWIGLU ? p.N / 2 : p.N;
  const int cbase = EPI == EPI_SWIGLU ? (bn + wn * FN * 16) / 2 : bn + wn * FN * 16;
  float sqv[ROWS * CPR / 64];  // (ss_out: squares of each stored chunk)
#pragma unroll
  for (int it = 0; it < ROWS * CPR / 64; ++it) {
    sqv[it] = 0.f;
    const int idx = it * 64 + l, row = idx / CPR, ch = idx % CPR;
    const int m = bm + wm * ROWS + row, n = cbase + ch * 8;
    if (m >= p.M || n >= ncols) continue;
    uint4 v = *reinterpret_cast<const uint4*>(wl + row * RS + ch * 16);
    if constexpr (EPI == EPI_QKV) {  // (bf16-rounded like the stored projection it replaces)
      float o[8], q[8];
      unpack8(v, o);
      unpack8(*reinterpret_cast<const uint4*>(wl + row * RS + (ch ^ 1) * 16), q);
      qkv_store(p, m, n, o, q);
      continue;
    }
    if constexpr (kResid<EPI>) {
      float a[8], b[8];
      unpack8(v, a);
      unpack8(*reinterpret_cast<const uint4*>(p.R + (size_t)m * p.ldr + n), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
      v = pack8(a);
      if (p.ss_out) {
        unpack8(v, a);  // (the stored bf16 values)
#pragma unroll
        for (int e = 0; e < 8; ++e) sqv[it] += a[e] * a[e];
      }
    }
    *reinterpret_cast<uint4*>(reinterpret_cast<u16*>(p.Y) + (size_t)m * p.ldy + n) = v;
  }
  if (kResid<EPI> && p.ss_out) {  // one atomic per (row, wave): the CPR lanes of a row reduce first
#pragma unroll
    for (int it = 0; it < ROWS * CPR / 64; ++it) {
      const int idx = it * 64 + l, row = idx / CPR, ch = idx % CPR;
      const int m = bm + wm * ROWS + row;
      float sq = sqv[it];
#pragma unroll
      for (int o = 1; o < CPR; o <<= 1) sq += __shfl_xor(sq, o, 64);  // the CPR lanes of one row
      if (ch == 0 && m < p.M && cbase < ncols)
        __hip_atomic_fetch_add(gp(p.ss_out + m), ss_fix(sq), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// sum of the split-K slabs + epilogue (two-launch split-K): one thread per (row, 8 output columns)
template <int EPI>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(GemmParams p) {
  const int cpr = (EPI == EPI_SWIGLU ? p.N / 2 : p.N) / 8;
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool ok = id < (int64_t)p.M * cpr;
  const __amdgpu_buffer_rsrc_t rws = rsrc(p.ws, (size_t)p.splits * p.M * p.N * 4);
  float sq = 0.f;
  if (ok) sq = reduce_item<EPI, 0>(p, rws, (int)(id / cpr), (int)(id % cpr) * 8);
  if (kResid<EPI> && p.ss_out) ss_add(p.ss_out, ok ? (int)(id / cpr) : -1, sq);
}

// per-row 1/rms of X (the RMSNorm of a projection whose gamma is folded into W)
__global__ __launch_bounds__(256) void row_rstd_kernel(const u16* __restrict__ x, int ldx, int M, int K, float eps,
                                                       float* __restrict__ rstd) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const u16* xr = x + (size_t)row * ldx;
  float ss = 0.f;
  for (int c = lane_id() * 8; c < K; c += 64 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
  }
  ss = wave_sum(ss);
  if (lane_id() == 0) rstd[row] = rsqrtf(ss / (float)K + eps);
}

template <class C, int EPI>
int launch_cfg(const GemmParams& p, hipStream_t st) {
  const int tiles = ((p.M + C::BM - 1) / C::BM) * ((p.N + C::BN - 1) / C::BN);
  const dim3 grid(tiles * p.splits * (p.nbatch > 1 ? p.nbatch : 1));
  const int lds = 2 * C::STAGE > C::LDS ? 2 * C::STAGE : C::LDS;  // two stage buffers
  if (p.sw && p.sx)
    hipLaunchKernelGGL((gemm_kernel<C, EPI, true, true>), grid, dim3(C::THREADS), lds, st, p);
  else if (p.sw)  // W8A16: bf16 X, fp8 tiled weights, on its own tile (launch_epi)
    return -17;
  else if (p.w_tiled)
    hipLaunchKernelGGL((gemm_kernel<C, EPI, true, false>), grid, dim3(C::THREADS), lds, st, p);
  else
    hipLaunchKernelGGL((gemm_kernel<C, EPI, false, false>), grid, dim3(C::THREADS), lds, st, p);
  return 0;
}

int g_p8_mode = 2;  // 0: never, 1: every eligible shape, 2: the measured rule (p8_auto)

// Shapes the 8-phase 256^2 kernel takes: tiled bf16 weights, N % 256, one batch
bool p8_eligible(const GemmParams& p) {
  return p.w_tiled && !p.sw && p.N % 256 == 0 && p.nbatch <= 1 && p.M >= 256;
}

template <int EPI>
int launch_epi(const GemmParams& p, hipStream_t st, bool p8) {
  if (p8) {
    const int tiles = ((p.M + 255) / 256) * (p.N / 256);
    hipLaunchKernelGGL((gemm_kernel<CfgP8, EPI, true, false, true>), dim3(tiles * p.splits), dim3(CfgP8::THREADS),
                       CfgP8::LDS, st, p);
  } else if (p.sw && !p.sx) {  // W8A16
    using C = CfgW8;
    const int tiles = ((p.M + C::BM - 1) / C::BM) * ((p.N + C::BN - 1) / C::BN);
    hipLaunchKernelGGL((gemm_kernel<C, EPI, true, false, false, true>), dim3(tiles * p.splits), dim3(C::THREADS),
                       C::W8LDS, st, p);
  } else {
    launch_cfg<CfgS, EPI>(p, st);
  }
  if (p.splits > 1) {
    const int64_t n = (int64_t)p.M * (EPI == EPI_SWIGLU ? p.N / 2 : p.N) / 8;
    hipLaunchKernelGGL((gemm_reduce_kernel<EPI>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p);
  }
  return (int)hipGetLastError();
}

}  // namespace

// Split-K slices for a shape: enough workgroups to cover the CUs ~2x when the output tiles
// alone cannot (few rows: weight streaming), bounded by the k-groups and the workspace.
// Split while the workgroups cover less than this % of the CUs (0: per-dtype default).  Measured
// on the Llama-3-8B decode steps of 32 / 64 rows (tools/rows_sweep.py, profiles/r4_gemm_ab.md):
// bf16 75 % (5.08 / 5.69 ms vs 5.21 / 6.08 at 100 %), fp8 100 % (4.42 / 5.03 vs 4.62 / 5.06 at 75 %).
int g_split_fill_pct = 0;

extern "C" int vwa_gemm_splits(int M, int N, int K, int cus, int64_t ws_floats, int f8) {
  const int tiles = ((M + CfgS::BM - 1) / CfgS::BM) * ((N + CfgS::BN - 1) / CfgS::BN);
  const int KG = K / BKG;
  const int pct = g_split_fill_pct > 0 ? g_split_fill_pct : f8 ? 100 : 75;
  const int fill = (int)((int64_t)cus * pct / 100);
  int s = 1;
  while (tiles * s < fill && s * 2 <= KG && (int64_t)(s * 2) * M * N <= ws_floats) s *= 2;
  return s;
}

extern "C" void vwa_gemm_set_split_fill(int pct) { g_split_fill_pct = pct < 0 ? 0 : pct; }

extern "C" void vwa_gemm_set_p8(int mode) { g_p8_mode = mode; }

extern "C" int vwa_gemm(int epi, const GemmParams* pp, hipStream_t st) {
  GemmParams p = *pp;
  if (p.M < 1 || p.N < 16 || p.N % 16 || p.K < BKG || p.K % BKG) return -10;
  if (p.ldx % (p.sx ? 16 : 8) || (reinterpret_cast<uintptr_t>(p.X) & 15) || (reinterpret_cast<uintptr_t>(p.W) & 15))
    return -11;
  if ((p.sw && !p.w_tiled) || (p.sx && !p.sw)) return -14;  // fp8: the tiled layout; X codes need fp8 weights
  if (epi == EPI_SWIGLU && (p.N % 32 || p.y_f32)) return -12;
  if (epi == EPI_QKV && (p.y_f32 || p.head_dim % 16 || p.N != (p.n_q_heads + 2 * p.n_kv_heads) * p.head_dim ||
                         !p.q_out || !p.k_cache || !p.v_cache || !p.slots || (p.use_rope && (!p.rope || !p.positions))))
    return -16;
  if (p.splits < 1) p.splits = 1;
  // 8-phase 256^2 kernel (mode 2, measured rule, tools/bench_gemm.py): the prompt-sized shapes
  // whose 256^2 tiles alone fill the CUs (>= 256 tiles, e.g. the 1011-row gate/up), or fill them
  // with split-K slices of >= 2048 K each (the 1011-row down projection, K = 14336: 4 slices,
  // 118.5 vs 140.4 us on the 128^2 kernel and 122.5 for hipBLASLt; shorter slices lose to the
  // f32 partial traffic: o / QKV at K = 4096 58 / 92 vs 45 / 60 us).  Mode 1: every eligible shape.
  bool p8 = false;
  if (g_p8_mode && p8_eligible(p)) {
    const int tiles8 = ((p.M + 255) / 256) * (p.N / 256);
    int s = 1;
    const int KGs = p.K / BKG;
    while (p.ws && tiles8 * s < p.cus && s * 2 <= KGs && (int64_t)(s * 2) * p.M * p.N <= p.ws_cap) s *= 2;
    if (g_p8_mode == 1 || tiles8 >= 256 || (p.cus > 0 && tiles8 * s >= p.cus && p.K / s >= 2048)) {
      p8 = true;
      p.splits = s;
    }
  }
  const int KG = p.K / BKG;
  p.kg_per_split = (KG + p.splits - 1) / p.splits;
  p.splits = (KG + p.kg_per_split - 1) / p.kg_per_split;  // no empty slice
  if (p.splits > 1 && !p.ws) return -13;
  if (p.nbatch > 1 && p.splits > 1) return -15;  // batched launches take no split-K
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(p, st, p8);
    case EPI_RESID: return launch_epi<EPI_RESID>(p, st, p8);
    case EPI_SWIGLU: return launch_epi<EPI_SWIGLU>(p, st, p8);
    case EPI_GELU: return launch_epi<EPI_GELU>(p, st, p8);
    case EPI_GELU_RESID: return launch_epi<EPI_GELU_RESID>(p, st, p8);
    case EPI_QKV: return launch_epi<EPI_QKV>(p, st, p8);
    default: return -3;
  }
}

extern "C" int vwa_row_rstd(const uint16_t* x, int ldx, int M, int K, float eps, float* rstd, hipStream_t st) {
  if (M < 1 || K % 8 || ldx % 8) return -1;
  hipLaunchKernelGGL(row_rstd_kernel, dim3((M + 3) / 4), dim3(256), 0, st, x, ldx, M, K, eps, rstd);
  return (int)hipGetLastError();
}
