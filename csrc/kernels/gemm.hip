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
//   interleaved per 16 rows (ops.interleave_gate_up)   3 GELU (+bias)
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GELU = 3 };

constexpr int BM = 128, BN = 128, BKG = 128;
constexpr int kThreads = 256;
constexpr int kABytes = BM * BKG * 2;  // 32 KB
constexpr int kBBytes = BN * BKG * 2;  // 32 KB

struct Stage {
  uint4 a[8];
  uint4 b[8];
};

// global -> registers for k-group kg
template <bool WT>
VWA_DEVICE void load_stage(const GemmParams& p, int bm, int bn, int kg, Stage& st) {
  const int t = threadIdx.x;
  const int c = t & 15;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int r = it * 16 + (t >> 4);
    const int m = bm + r;
    st.a[it] = make_uint4(0u, 0u, 0u, 0u);
    if (m < p.M) st.a[it] = *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + (size_t)kg * BKG + c * 8);
  }
  const int kgn = p.K / BKG;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    if constexpr (WT) {
      const int T = (bn >> 4) + it;
      st.b[it] = make_uint4(0u, 0u, 0u, 0u);
      if (T * 16 < p.N) st.b[it] = *reinterpret_cast<const uint4*>(p.W + ((size_t)T * kgn + kg) * 2048 + t * 8);
    } else {
      const int n = bn + it * 16 + (t >> 4);
      st.b[it] = make_uint4(0u, 0u, 0u, 0u);
      if (n < p.N) st.b[it] = *reinterpret_cast<const uint4*>(p.W + (size_t)n * p.K + (size_t)kg * BKG + c * 8);
    }
  }
}

// registers -> LDS (A swizzled, B in fragment order)
template <bool WT>
VWA_DEVICE void store_stage(char* lds, const Stage& st) {
  const int t = threadIdx.x;
  const int c = t & 15;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int r = it * 16 + (t >> 4);
    *reinterpret_cast<uint4*>(lds + r * 256 + ((c ^ (r & 15)) << 4)) = st.a[it];
  }
  char* lb = lds + kABytes;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    if constexpr (WT) {
      *reinterpret_cast<uint4*>(lb + it * 4096 + t * 16) = st.b[it];
    } else {
      // row n_local = it*16 + (t>>4) of the 128-row tile, k chunk c = 4 g + s
      const int nn = t >> 4, g = c >> 2, s = c & 3;
      *reinterpret_cast<uint4*>(lb + (it * 4 + s) * 1024 + (16 * g + nn) * 16) = st.b[it];
    }
  }
}

VWA_DEVICE void compute_stage(const char* lds, f32x4 (&acc)[4][4], int wm, int wn) {
  const int l = lane_id();
  const int rl = l & 15, g = l >> 4;
  const char* la = lds + (wm * 64 + rl) * 256;
  const char* lb = lds + kABytes + (wn * 4) * 4096 + l * 16;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    bf16x8 a[4], b[4];
    const int ch = ((4 * g + s) ^ rl) << 4;  // row & 15 == rl for every fragment row
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const bf16x8*>(la + i * 16 * 256 + ch);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = *reinterpret_cast<const bf16x8*>(lb + j * 4096 + s * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(a[i], b[j], acc[i][j]);
  }
}

VWA_DEVICE float bias_at(const GemmParams& p, int n) { return p.bias ? bf2f(p.bias[n]) : 0.f; }

template <int EPI>
VWA_DEVICE void store_out(const GemmParams& p, int m, int n, float v) {
  if constexpr (EPI == EPI_RESID) v += bf2f(p.R[(size_t)m * p.ldr + n]);
  if (p.y_f32)
    reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
  else
    reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + n] = f2bf(v);
}

template <int EPI, bool WT>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int mb = (p.M + BM - 1) / BM, nb = (p.N + BN - 1) / BN;
  const int tiles = mb * nb;
  const int split = blockIdx.x / tiles;  // split-K slice (blocks of one slice are contiguous)
  // XCD-aware: logical tile order is column-block major, so consecutive logical tiles (same XCD)
  // share the column block's weight tile in L2
  const int lt = xcd_remap((int)(blockIdx.x % tiles), tiles);
  const int bn = (lt / mb) * BN, bm = (lt % mb) * BM;
  const int KG = p.K / BKG;
  const int kg0 = split * p.kg_per_split, kg1 = min(KG, kg0 + p.kg_per_split);
  const int w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  Stage st;
  if (kg0 < kg1) {
    load_stage<WT>(p, bm, bn, kg0, st);
    store_stage<WT>(lds, st);
    __syncthreads();
    for (int kg = kg0; kg < kg1; ++kg) {
      const bool more = kg + 1 < kg1;
      if (more) load_stage<WT>(p, bm, bn, kg + 1, st);  // in flight during the MFMAs
      compute_stage(lds, acc, wm, wn);
      __syncthreads();
      if (more) {
        store_stage<WT>(lds, st);
        __syncthreads();
      }
    }
  }
  const int l = lane_id();
  const int col0 = bn + wn * 64 + (l & 15);
  const int row0 = bm + wm * 64 + 4 * (l >> 4);
  if (p.splits > 1) {  // f32 partial slab of this slice; gemm_reduce_kernel applies the epilogue
    float* ws = p.ws + (size_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = row0 + i * 16 + r;
        if (m >= p.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = col0 + j * 16;
          if (n < p.N) ws[(size_t)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = row0 + i * 16 + r;
      if (m >= p.M) continue;
      const float rs = p.rstd ? p.rstd[m] : 1.f;
      if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
          const int n = col0 + j * 16;  // gate column; its up partner is n + 16
          if (n >= p.N) continue;
          const int f = ((n - (l & 15)) >> 5) * 16 + (l & 15);
          const float gt = acc[i][j][r] * rs, up = acc[i][j + 1][r] * rs;
          reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + f] = f2bf(silu(gt) * up);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = col0 + j * 16;
          if (n >= p.N) continue;
          float v = acc[i][j][r] * rs + bias_at(p, n);
          if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
          store_out<EPI>(p, m, n, v);
        }
      }
    }
}

// sum of the split-K slabs + epilogue; one thread per output element (SwiGLU: per feature)
template <int EPI>
__global__ __launch_bounds__(256) void gemm_reduce_kernel(GemmParams p) {
  const int64_t id = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int ncols = EPI == EPI_SWIGLU ? p.N / 2 : p.N;
  if (id >= (int64_t)p.M * ncols) return;
  const int m = (int)(id / ncols), c = (int)(id % ncols);
  const size_t slab = (size_t)p.M * p.N;
  const float rs = p.rstd ? p.rstd[m] : 1.f;
  if constexpr (EPI == EPI_SWIGLU) {
    const int n = (c >> 4) * 32 + (c & 15);
    float gt = 0.f, up = 0.f;
    for (int z = 0; z < p.splits; ++z) {
      gt += p.ws[z * slab + (size_t)m * p.N + n];
      up += p.ws[z * slab + (size_t)m * p.N + n + 16];
    }
    reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + c] = f2bf(silu(gt * rs) * (up * rs));
  } else {
    float v = 0.f;
    for (int z = 0; z < p.splits; ++z) v += p.ws[z * slab + (size_t)m * p.N + c];
    v = v * rs + bias_at(p, c);
    if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
    store_out<EPI>(p, m, c, v);
  }
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

template <int EPI>
int launch_epi(const GemmParams& p, hipStream_t st) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const dim3 grid(tiles * p.splits);
  const int lds = kABytes + kBBytes;
  if (p.w_tiled)
    hipLaunchKernelGGL((gemm_kernel<EPI, true>), grid, dim3(kThreads), lds, st, p);
  else
    hipLaunchKernelGGL((gemm_kernel<EPI, false>), grid, dim3(kThreads), lds, st, p);
  if (p.splits > 1) {
    const int64_t n = (int64_t)p.M * (EPI == EPI_SWIGLU ? p.N / 2 : p.N);
    hipLaunchKernelGGL((gemm_reduce_kernel<EPI>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p);
  }
  return (int)hipGetLastError();
}

}  // namespace

// Split-K slices for a shape: enough workgroups to cover the CUs ~2x when the output tiles
// alone cannot (few rows: weight streaming), bounded by the k-groups and the workspace.
extern "C" int vwa_gemm_splits(int M, int N, int K, int cus, int64_t ws_floats) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int KG = K / BKG;
  int s = 1;
  while (tiles * s < cus && s * 2 <= KG && (int64_t)(s * 2) * M * N <= ws_floats) s *= 2;
  return s;
}

extern "C" int vwa_gemm(int epi, const GemmParams* pp, hipStream_t st) {
  GemmParams p = *pp;
  if (p.M < 1 || p.N < 16 || p.N % 16 || p.K < BKG || p.K % BKG) return -10;
  if (p.ldx % 8 || (reinterpret_cast<uintptr_t>(p.X) & 15) || (reinterpret_cast<uintptr_t>(p.W) & 15)) return -11;
  if (epi == EPI_SWIGLU && (p.N % 32 || p.y_f32)) return -12;
  if (p.splits < 1) p.splits = 1;
  const int KG = p.K / BKG;
  p.kg_per_split = (KG + p.splits - 1) / p.splits;
  p.splits = (KG + p.kg_per_split - 1) / p.kg_per_split;  // no empty slice
  if (p.splits > 1 && !p.ws) return -13;
  switch (epi) {
    case EPI_STORE: return launch_epi<EPI_STORE>(p, st);
    case EPI_RESID: return launch_epi<EPI_RESID>(p, st);
    case EPI_SWIGLU: return launch_epi<EPI_SWIGLU>(p, st);
    case EPI_GELU: return launch_epi<EPI_GELU>(p, st);
    default: return -3;
  }
}

extern "C" int vwa_row_rstd(const uint16_t* x, int ldx, int M, int K, float eps, float* rstd, hipStream_t st) {
  if (M < 1 || K % 8 || ldx % 8) return -1;
  hipLaunchKernelGGL(row_rstd_kernel, dim3((M + 3) / 4), dim3(256), 0, st, x, ldx, M, K, eps, rstd);
  return (int)hipGetLastError();
}
