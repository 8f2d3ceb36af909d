// Streaming skinny GEMM (decode path, M <= 16 typically) -- persistent, software-pipelined.
//
// Same math and epilogues as skinny_gemm.hip, restructured after rocprof showed the one-tile-
// per-workgroup kernel streaming weights at only ~3.1-3.4 TB/s: every workgroup paid launch +
// prologue + LDS reduction + epilogue around a single round trip of weight loads, leaving the
// CU's memory pipe idle between workgroups.  Here:
//
//  * X (the activation rows, <= ~140 KB) is staged in LDS once per workgroup and read back with
//    ds_read_b128 -- no activation loads in the weight stream, no X registers;
//  * the fused-RMSNorm row scales are computed once from that LDS copy;
//  * each workgroup is persistent over column tiles (tile = blockIdx.x + i*gridDim.x); its KS
//    waves split K, and every wave walks a flat list of (tile, k-batch) items;
//  * weight loads are raw buffer loads (SRD with num_records = N*K*2): the next item's 16 x
//    dwordx4 per lane are issued BEFORE the current item's MFMAs (two named register sets,
//    static indices -> counted vmcnt), and past-the-end items/groups use an out-of-range offset
//    that the hardware answers with zeros and no memory traffic, so the pipeline has no
//    data-dependent load predicates;
//  * the cross-wave reduction + fused epilogue of tile t runs while tile t+1's loads are in flight.
//
// XG variant (X does not fit in LDS: e.g. the down projection, K = 14336, with more than 5 rows):
// the activation fragments are streamed from global memory alongside the weights (X is a few
// hundred KB and stays L2-resident, so the extra loads hit L2, not HBM), with the same
// two-register-set pipeline; only the reduction scratch lives in LDS.
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GELU = 3, EPI_QKV = 4 };

constexpr unsigned kOOB = 0xFFFFFFF0u;

VWA_DEVICE uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Epilogue operands that do not depend on the GEMM (residual tile, fp8 column scales, QKV row
// positions / KV slots / rotary factors) are loaded for the workgroup's FIRST tile at kernel
// start, so they are not one more dependent memory round trip after the reduction.  Thread o
// owns output o of the tile (M*16*NT <= threads for every shape the launcher accepts).
struct EpiPre {
  float r = 0.f, cs0 = 1.f, cs1 = 1.f, rc = 1.f, rsn = 0.f;
  int64_t slot = -1;
};

template <int EPI, int NT>
VWA_DEVICE void epi_values(const SkinnyParams& p, int tile, int o, EpiPre& e) {
  const int n0 = tile * 16 * NT;
  if constexpr (EPI == EPI_SWIGLU || EPI == EPI_QKV) {
    if (o >= p.M * 16) return;
    const int m = o >> 4, q = o & 15;
    if (p.w_scale) {
      e.cs0 = p.w_scale[n0 + q];
      e.cs1 = p.w_scale[n0 + (EPI == EPI_SWIGLU ? 16 + q : (q ^ 8))];
    }
    if constexpr (EPI == EPI_QKV) {
      const int hd = p.head_dim, half = hd >> 1, t = (n0 % hd) >> 4;
      e.slot = p.slots[m];
      if (p.use_rope) {
        const int di = (q < 8) ? (8 * t + q) : (8 * t + q - 8);
        const int pos = p.positions[m];
        e.rc = p.rope[((size_t)pos * half + di) * 2 + 0];
        e.rsn = p.rope[((size_t)pos * half + di) * 2 + 1];
      }
    }
  } else {
    if (o >= p.M * 16 * NT) return;
    const int m = o / (16 * NT), nn = o % (16 * NT);
    if (p.w_scale) e.cs0 = p.w_scale[n0 + nn];
    if constexpr (EPI == EPI_RESID) e.r = bf2f(p.R[(size_t)m * p.ldr + n0 + nn]);
  }
}

// Cross-wave reduction of one column tile + fused epilogue.  rs[m]: per-row scale (fused RMSNorm
// / LayerNorm rstd and, on the fp8 path, the activation quantisation scale); mus[m] (folded
// LayerNorm only, else null): row mean, removed as mean * ln_c[n]; column scales (fp8) come
// with the epilogue operands (`pre` when this is the workgroup's first tile).
template <int EPI, int NT, int KS>
VWA_DEVICE void tile_epilogue(const SkinnyParams& p, float* red, const float* rs, const float* mus, int tile,
                              f32x4 (&acc)[NT], int w, int lane, const EpiPre& pre, bool first) {
  const int M = p.M;
  const int n0 = tile * 16 * NT;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((w * NT + nt) * 4 + i) * 64 + lane] = acc[nt][i];
  __syncthreads();
  auto red_at = [&](int m, int nn) -> float {
    const int nt = nn >> 4, q = nn & 15;
    const int ln = q + 16 * (m >> 2), i = m & 3;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) s += red[((ww * NT + nt) * 4 + i) * 64 + ln];
    return s;
  };
  auto operands = [&](int o) {
    if (first && o == (int)threadIdx.x) return pre;
    EpiPre e;
    epi_values<EPI, NT>(p, tile, o, e);
    return e;
  };
  if constexpr (EPI == EPI_SWIGLU) {
    for (int o = threadIdx.x; o < M * 16; o += KS * 64) {
      const int m = o >> 4, q = o & 15;
      const EpiPre e = operands(o);
      const float sc = rs[m];
      float gv = red_at(m, q) * sc * e.cs0, uv = red_at(m, 16 + q) * sc * e.cs1;
      if (p.bias) {
        gv += bf2f(p.bias[n0 + q]);
        uv += bf2f(p.bias[n0 + 16 + q]);
      }
      reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + tile * 16 + q] = f2bf(silu(gv) * uv);
    }
  } else if constexpr (EPI == EPI_QKV) {
    const int hd = p.head_dim, half = hd >> 1;
    const int head = n0 / hd;
    const int t = (n0 % hd) >> 4;
    const bool is_v = head >= p.n_q_heads + p.n_kv_heads;
    for (int o = threadIdx.x; o < M * 16; o += KS * 64) {
      const int m = o >> 4, q = o & 15;
      const EpiPre e = operands(o);
      const float sc = rs[m];
      float v = red_at(m, q), pv = red_at(m, q ^ 8);
      if (mus) {
        v -= mus[m] * p.ln_c[n0 + q];
        pv -= mus[m] * p.ln_c[n0 + (q ^ 8)];
      }
      v *= sc * e.cs0;
      pv *= sc * e.cs1;
      if (p.bias) {
        v += bf2f(p.bias[n0 + q]);
        pv += bf2f(p.bias[n0 + (q ^ 8)]);
      }
      const int d = (q < 8) ? (8 * t + q) : (half + 8 * t + q - 8);
      if (p.use_rope && !is_v) v = (q < 8) ? (v * e.rc - pv * e.rsn) : (v * e.rc + pv * e.rsn);
      const u16 out = f2bf(v);
      if (head < p.n_q_heads) {
        p.q_out[(size_t)m * p.ldq + head * hd + d] = out;
      } else {
        const int64_t slot = e.slot;
        if (slot >= 0) {
          const int64_t blk = slot / p.block_size, off = slot % p.block_size;
          const int kvh = is_v ? head - p.n_q_heads - p.n_kv_heads : head - p.n_q_heads;
          const int64_t idx = blk * p.cache_stride_block + kvh * p.cache_stride_head + off * p.cache_stride_tok + d;
          (is_v ? p.v_cache : p.k_cache)[idx] = out;
        }
      }
    }
  } else {
    for (int o = threadIdx.x; o < M * 16 * NT; o += KS * 64) {
      const int m = o / (16 * NT), nn = o % (16 * NT);
      const int n = n0 + nn;
      const EpiPre e = operands(o);
      float v = red_at(m, nn);
      if (mus) v -= mus[m] * p.ln_c[n];
      v *= rs[m] * e.cs0;
      if (p.bias) v += bf2f(p.bias[n]);
      if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
      if constexpr (EPI == EPI_RESID) v += e.r;
      if (p.y_f32) reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
      else reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + n] = f2bf(v);
    }
  }
  __syncthreads();
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int EPI, int NT, int KS, bool XG>
__global__ __launch_bounds__(KS * 64) void skinny_stream_kernel(SkinnyParams p, int nb, int xstride) {
  constexpr int U = XG ? 2 : 4 / NT;  // k-groups (128 wide) per item
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = p.M, K = p.K, N = p.N;
  u16* xs = reinterpret_cast<u16*>(smem);
  const int xbytes = XG ? 0 : ((M * xstride * 2) + 15) & ~15;
  float* red = reinterpret_cast<float*>(smem + xbytes);  // [KS][NT][4][64]
  float* rs = red + KS * NT * 4 * 64;                     // [16] row scales (1/rms, LayerNorm rstd)
  float* mu = rs + 16;                                    // [16] row means (folded LayerNorm)
  const float* mus = (p.fuse_rms == 2) ? mu : nullptr;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nl = lane & 15, g = lane >> 4;

  EpiPre pre;
  epi_values<EPI, NT>(p, blockIdx.x, threadIdx.x, pre);  // first tile's epilogue operands, early
  const int G = K / 128;
  const int gb = (G * w) / KS, ge = (G * (w + 1)) / KS;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)N * K * 2), 0x00020000);
  // X fragments (XG): lane (row nl, k-quarter g); rows >= M read the zero OOB answer
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.X), (short)0, (int)((size_t)M * p.ldx * 2), 0x00020000);
  const int ntiles = N / (16 * NT);
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int n_items = my_tiles * nb;

  auto load_x = [&](uint4 (&xr)[U][4], int it) {
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      const bool ok = (it < n_items) && (kg < ge) && (nl < M);
      const unsigned base = ((unsigned)nl * (unsigned)p.ldx + (unsigned)(kg * 128 + 32 * g)) * 2u;
#pragma unroll
      for (int s = 0; s < 4; ++s) xr[u][s] = bload(rx, ok ? base + 16u * s : kOOB);
    }
  };

  auto load_item = [&](uint4 (&wr)[NT][U][4], int it) {
    const int tile = blockIdx.x + (it / nb) * gridDim.x;
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      const bool ok = (it < n_items) && (kg < ge);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const unsigned row = (unsigned)(tile * 16 * NT + nt * 16 + nl);
        const unsigned base = (row * (unsigned)K + (unsigned)(kg * 128 + 32 * g)) * 2u;
#pragma unroll
        for (int s = 0; s < 4; ++s) wr[nt][u][s] = bload(rw, ok ? base + 16u * s : kOOB);
      }
    }
  };

  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute_item = [&](const uint4 (&wr)[NT][U][4], const uint4 (&xr)[U][4], int it) {
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      if (kg >= ge) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 a = make_uint4(0, 0, 0, 0);
        if constexpr (XG) a = xr[u][s];
        else if (nl < M) a = *reinterpret_cast<const uint4*>(xs + nl * xstride + kg * 128 + 32 * g + 8 * s);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16(as_bf16x8(a), as_bf16x8(wr[nt][u][s]), acc[nt]);
      }
    }
  };

  auto finish_tile = [&](int it) {
    const int tile = blockIdx.x + (it / nb) * gridDim.x;
    tile_epilogue<EPI, NT, KS>(p, red, rs, mus, tile, acc, w, lane, pre, it < nb);
  };

  uint4 A[NT][U][4], B[NT][U][4];
  uint4 XA[U][4], XB[U][4];  // XG only (dead otherwise)
  // w_first: issue the first weight item before staging X (its round trip then overlaps the X
  // staging + fused-RMSNorm statistics); otherwise stage X first (the X round trip is short).
  if (p.w_first) {
    load_item(A, 0);
    if constexpr (XG) load_x(XA, 0);
  }
  // ---- stage X rows into LDS
  const int k8 = K / 8;
  if constexpr (!XG) {
    for (int c = threadIdx.x; c < M * k8; c += KS * 64) {
      const int m = c / k8, kk = c % k8;
      *reinterpret_cast<uint4*>(xs + m * xstride + kk * 8) =
          *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8);
    }
  }
  __syncthreads();
  for (int m = w; m < 16; m += KS) {
    float sc = 1.f, mean = 0.f;
    if (p.fuse_rms && m < M) {
      float s = 0.f, s1 = 0.f;
      for (int kk = lane; kk < k8; kk += 64) {
        float f[8];
        unpack8(XG ? *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8)
                   : *reinterpret_cast<const uint4*>(xs + m * xstride + kk * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s += f[j] * f[j];
          s1 += f[j];
        }
      }
      s = wave_sum(s);
      if (p.fuse_rms == 2) {  // LayerNorm: rstd from E[x^2] - mean^2
        mean = wave_sum(s1) / (float)K;
        sc = rsqrtf(fmaxf(s / (float)K - mean * mean, 0.f) + p.eps);
      } else {
        sc = rsqrtf(s / (float)K + p.eps);
      }
    }
    if (lane == 0) {
      rs[m] = sc;
      mu[m] = mean;
    }
  }
  __syncthreads();

  if (!p.w_first) {
    load_item(A, 0);
    if constexpr (XG) load_x(XA, 0);
  }
  for (int it = 0; it < n_items; it += 2) {
    load_item(B, it + 1);
    if constexpr (XG) load_x(XB, it + 1);
    compute_item(A, XA, it);
    if (it % nb == nb - 1) finish_tile(it);
    if (it + 1 >= n_items) break;
    load_item(A, it + 2);
    if constexpr (XG) load_x(XA, it + 2);
    compute_item(B, XB, it + 1);
    if ((it + 1) % nb == nb - 1) finish_tile(it + 1);
  }
}

template <int EPI, int NT, int KS, bool XG>
int launch_v(const SkinnyParams& p, hipStream_t st, int grid_cap, size_t lds, int xstride) {
  constexpr int U = XG ? 2 : 4 / NT;
  const int G = p.K / 128;
  const int per_wave = (G + KS - 1) / KS;
  const int nb = (per_wave + U - 1) / U;
  const int ntiles = p.N / (16 * NT);
  const int grid = ntiles < grid_cap ? ntiles : grid_cap;
  hipLaunchKernelGGL((skinny_stream_kernel<EPI, NT, KS, XG>), dim3(grid), dim3(KS * 64), lds, st, p, nb, xstride);
  return 0;
}

template <int EPI, int NT, int KS>
int launch(const SkinnyParams& p, hipStream_t st, int grid_cap) {
  const int xstride = p.K + 8;
  const size_t xbytes = ((size_t)p.M * xstride * 2 + 15) & ~(size_t)15;
  const size_t red = (size_t)(KS * NT * 4 * 64 + 32) * sizeof(float);  // + row scales + row means
  if (xbytes + red <= 160 * 1024) return launch_v<EPI, NT, KS, false>(p, st, grid_cap, xbytes + red, xstride);
  if ((size_t)p.M * p.ldx * 2 >= 0x7FFFFFF0ull) return -10;
  return launch_v<EPI, NT, KS, true>(p, st, grid_cap, red, xstride);
}


// ------------------------------------------------------------------------------------------
// W8A8 variant (VWA_DTYPE=fp8): W is OCP e4m3 [N, K] bytes with per-row scales, X rows are
// quantised to e4m3 once per workgroup while staging into LDS (per-row dynamic scale
// amax/448), the inner product runs on the fp8 MFMA (16x16x32, 8 bytes per lane per operand),
// and both scales are applied in the epilogue.  Weight bytes per decode step are halved.
// ------------------------------------------------------------------------------------------
template <int EPI, int NT, int KS>
__global__ __launch_bounds__(KS * 64) void skinny_fp8_kernel(SkinnyParams p, int nb, int xstride) {
  constexpr int U = 8 / NT;  // k-groups (128 wide) per item: 2 x b128 weight loads per k-group
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = p.M, K = p.K, N = p.N;
  uint8_t* xs = reinterpret_cast<uint8_t*>(smem);
  const int xbytes = ((M * xstride) + 15) & ~15;
  float* red = reinterpret_cast<float*>(smem + xbytes);  // [KS][NT][4][64]
  float* rs = red + KS * NT * 4 * 64;                     // [16] row scale (rms * x-quant scale)
  float* inv = rs + 16;                                    // [16] 1 / x-quant scale
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nl = lane & 15, g = lane >> 4;
  const int k8 = K / 8;

  EpiPre pre;
  epi_values<EPI, NT>(p, blockIdx.x, threadIdx.x, pre);  // first tile's epilogue operands, early
  // ---- per-row statistics (sum of squares for the fused RMSNorm, amax for the fp8 scale)
  for (int m = w; m < 16; m += KS) {
    float sc = 1.f, iv = 1.f;
    if (m < M) {
      float ss = 0.f, am = 0.f;
      for (int kk = lane; kk < k8; kk += 64) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          ss += f[j] * f[j];
          am = fmaxf(am, fabsf(f[j]));
        }
      }
      ss = wave_sum(ss);
      am = wave_max(am);
      const float sx = am > 0.f ? am * (1.f / 448.f) : 1.f;
      iv = 1.f / sx;
      sc = (p.fuse_rms ? rsqrtf(ss / (float)K + p.eps) : 1.f) * sx;
    }
    if (lane == 0) {
      rs[m] = sc;
      inv[m] = iv;
    }
  }
  __syncthreads();
  // ---- quantise X rows into LDS (e4m3, 8 values -> 8 bytes)
  for (int c = threadIdx.x; c < M * k8; c += KS * 64) {
    const int m = c / k8, kk = c % k8;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8), f);
    const float iv = inv[m];
    uint2 q;
    q.x = cvt_pk_fp8(f[0] * iv, f[1] * iv) | (cvt_pk_fp8(f[2] * iv, f[3] * iv) << 16);
    q.y = cvt_pk_fp8(f[4] * iv, f[5] * iv) | (cvt_pk_fp8(f[6] * iv, f[7] * iv) << 16);
    *reinterpret_cast<uint2*>(xs + m * xstride + kk * 8) = q;
  }
  __syncthreads();

  const int G = K / 128;
  const int gb = (G * w) / KS, ge = (G * (w + 1)) / KS;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)N * K), 0x00020000);
  const int ntiles = N / (16 * NT);
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int n_items = my_tiles * nb;

  auto load_item = [&](uint4 (&wr)[NT][U][2], int it) {
    const int tile = blockIdx.x + (it / nb) * gridDim.x;
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      const bool ok = (it < n_items) && (kg < ge);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const unsigned row = (unsigned)(tile * 16 * NT + nt * 16 + nl);
        const unsigned base = row * (unsigned)K + (unsigned)(kg * 128 + 32 * g);
#pragma unroll
        for (int s = 0; s < 2; ++s) wr[nt][u][s] = bload(rw, ok ? base + 16u * s : kOOB);
      }
    }
  };

  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute_item = [&](const uint4 (&wr)[NT][U][2], int it) {
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      if (kg >= ge) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        uint4 a = make_uint4(0, 0, 0, 0);
        if (nl < M) a = *reinterpret_cast<const uint4*>(xs + nl * xstride + kg * 128 + 32 * g + 16 * s);
        const long a0 = (long)(((unsigned long)a.y << 32) | a.x), a1 = (long)(((unsigned long)a.w << 32) | a.z);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const uint4 v = wr[nt][u][s];
          const long b0 = (long)(((unsigned long)v.y << 32) | v.x), b1 = (long)(((unsigned long)v.w << 32) | v.z);
          acc[nt] = mfma16_fp8(a0, b0, acc[nt]);
          acc[nt] = mfma16_fp8(a1, b1, acc[nt]);
        }
      }
    }
  };

  uint4 A[NT][U][2], B[NT][U][2];
  load_item(A, 0);
  for (int it = 0; it < n_items; it += 2) {
    load_item(B, it + 1);
    compute_item(A, it);
    if (it % nb == nb - 1)
      tile_epilogue<EPI, NT, KS>(p, red, rs, nullptr, blockIdx.x + (it / nb) * gridDim.x, acc, w, lane, pre, it < nb);
    if (it + 1 >= n_items) break;
    load_item(A, it + 2);
    compute_item(B, it + 1);
    if ((it + 1) % nb == nb - 1)
      tile_epilogue<EPI, NT, KS>(p, red, rs, nullptr, blockIdx.x + ((it + 1) / nb) * gridDim.x, acc, w, lane, pre,
                                 it + 1 < nb);
  }
}

template <int EPI, int NT, int KS>
int launch_fp8(const SkinnyParams& p, hipStream_t st, int grid_cap) {
  constexpr int U = 8 / NT;
  const int G = p.K / 128;
  const int per_wave = (G + KS - 1) / KS;
  const int nb = (per_wave + U - 1) / U;
  const int xstride = p.K + 16;
  const size_t xbytes = ((size_t)p.M * xstride + 15) & ~(size_t)15;
  const size_t lds = xbytes + (size_t)(KS * NT * 4 * 64 + 32) * sizeof(float);
  if (lds > 160 * 1024) return -10;
  const int ntiles = p.N / (16 * NT);
  const int grid = ntiles < grid_cap ? ntiles : grid_cap;
  hipLaunchKernelGGL((skinny_fp8_kernel<EPI, NT, KS>), dim3(grid), dim3(KS * 64), lds, st, p, nb, xstride);
  return 0;
}

}  // namespace

// Returns -10 when this shape does not fit the streaming kernel (caller falls back).
template <int KS>
int dispatch_ks(int epi, const SkinnyParams& p, int grid_cap, hipStream_t st) {
  if (p.w_scale) {
    switch (epi) {
      case EPI_STORE: return launch_fp8<EPI_STORE, 1, KS>(p, st, grid_cap);
      case EPI_RESID: return launch_fp8<EPI_RESID, 1, KS>(p, st, grid_cap);
      case EPI_GELU: return launch_fp8<EPI_GELU, 1, KS>(p, st, grid_cap);
      case EPI_SWIGLU: return launch_fp8<EPI_SWIGLU, 2, KS>(p, st, grid_cap);
      case EPI_QKV: return launch_fp8<EPI_QKV, 1, KS>(p, st, grid_cap);
      default: return -3;
    }
  }
  switch (epi) {
    case EPI_STORE: return launch<EPI_STORE, 1, KS>(p, st, grid_cap);
    case EPI_RESID: return launch<EPI_RESID, 1, KS>(p, st, grid_cap);
    case EPI_GELU: return launch<EPI_GELU, 1, KS>(p, st, grid_cap);
    case EPI_SWIGLU: return launch<EPI_SWIGLU, 2, KS>(p, st, grid_cap);
    case EPI_QKV: return launch<EPI_QKV, 1, KS>(p, st, grid_cap);
    default: return -3;
  }
}

// Returns -10 when this shape does not fit the streaming kernel (caller falls back).
// ks = waves per workgroup splitting K (4 or 8); grid_cap = max persistent workgroups.
extern "C" int vwa_skinny_stream(int epi, const SkinnyParams* p, int grid_cap, int ks, hipStream_t st) {
  if (p->M < 1 || p->M > 16 || p->K % 128 != 0) return -10;
  if ((size_t)p->N * p->K * (p->w_scale ? 1 : 2) >= 0x7FFFFFF0ull) return -10;
  const int r = (ks == 4) ? dispatch_ks<4>(epi, *p, grid_cap, st) : dispatch_ks<8>(epi, *p, grid_cap, st);
  if (r) return r;
  return (int)hipGetLastError();
}
