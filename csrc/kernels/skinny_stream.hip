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
#include "mq_attention.h"

using namespace vwa;

namespace {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GELU = 3, EPI_QKV = 4 };

constexpr unsigned kOOB = 0xFFFFFFF0u;

VWA_DEVICE uint4 bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// weight-stream load with cache policy AUX (gfx950 buffer aux bits: 1 sc0, 2 nt, 16 sc1): decode
// weights are read once per step by one CU, so nt (2) keeps them from displacing L2 lines
template <int AUX>
VWA_DEVICE uint4 bload_w(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, AUX);
  return make_uint4(v.x, v.y, v.z, v.w);
}
// the same with the constant part of the offset in soffset (a scalar): one VGPR offset per 4
// loads instead of one per load.  Past-the-end items use voff = kOOB2 (>= 2 GB, above every
// weight's num_records even with soffset added)
constexpr unsigned kOOB2 = 0x80000000u;
template <int AUX>
VWA_DEVICE uint4 bload_w_so(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, soff, AUX);
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

// In-launch hand-off accessors (chain kernel): agent-scope relaxed atomics compile to sc1 loads /
// stores, which bypass the non-coherent per-XCD L2 state another workgroup could have left.
template <bool SC1>
VWA_DEVICE u16 ld_u16(const u16* p) {
  if constexpr (SC1) return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return gld(p);
}
template <bool SC1>
VWA_DEVICE void st_u16(u16* p, u16 v) {
  if constexpr (SC1) __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *gp(p) = v;
}
template <bool SC1>
VWA_DEVICE void st_f32(float* p, float v) {
  if constexpr (SC1) __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *gp(p) = v;
}

template <int EPI, int NT, bool SC1 = false>
VWA_DEVICE void epi_values(const SkinnyParams& p, int tile, int o, EpiPre& e) {
  const int n0 = tile * 16 * NT;
  if constexpr (EPI == EPI_SWIGLU || EPI == EPI_QKV) {
    if (o >= p.M * 16) return;
    const int m = o >> 4, q = o & 15;
    if (p.w_scale) {
      e.cs0 = gld(p.w_scale + n0 + q);
      e.cs1 = gld(p.w_scale + n0 + (EPI == EPI_SWIGLU ? 16 + q : (q ^ 8)));
    }
    if constexpr (EPI == EPI_QKV) {
      const int hd = p.head_dim, half = hd >> 1, t = (n0 % hd) >> 4;
      e.slot = gld(p.slots + m);
      if (p.use_rope) {
        const int di = (q < 8) ? (8 * t + q) : (8 * t + q - 8);
        const int pos = gld(p.positions + m);
        e.rc = gld(p.rope + ((size_t)pos * half + di) * 2 + 0);
        e.rsn = gld(p.rope + ((size_t)pos * half + di) * 2 + 1);
      }
    }
  } else {
    if (o >= p.M * 16 * NT) return;
    const int m = o / (16 * NT), nn = o % (16 * NT);
    if (p.w_scale) e.cs0 = gld(p.w_scale + n0 + nn);
    if constexpr (EPI == EPI_RESID) e.r = p.R ? bf2f(ld_u16<SC1>(p.R + (size_t)m * p.ldr + n0 + nn)) : 0.f;
  }
}

// Cross-wave reduction of one column tile + fused epilogue.  rs[m]: per-row scale (fused RMSNorm
// / LayerNorm rstd and, on the fp8 path, the activation quantisation scale); mus[m] (folded
// LayerNorm only, else null): row mean, removed as mean * ln_c[n]; column scales (fp8) come
// with the epilogue operands (`pre` when this is the workgroup's first tile).
// MT: 16-row MFMA row fragments per tile (M <= 16 MT; MT > 1 only in the streaming kernel's
// many-row form, skinny_stream_kernel); red = [KS][NT][MT][4][64] partial sums.
template <int EPI, int NT, int KS, bool SC1 = false, int MT = 1>
VWA_DEVICE void tile_epilogue(const SkinnyParams& p, float* red, const float* rs, const float* mus, int tile,
                              f32x4 (&acc)[NT * MT], int w, int lane, const EpiPre& pre, bool first,
                              const float* partner = nullptr) {
  const int M = p.M;
  const int n0 = tile * 16 * NT;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(((w * NT + nt) * MT + mt) * 4 + i) * 64 + lane] = acc[nt * MT + mt][i];
  lds_sync();
  auto red_at = [&](int m, int nn) -> float {
    const int nt = nn >> 4, q = nn & 15, mt = MT > 1 ? m >> 4 : 0, mm = m & 15;
    const int ln = q + 16 * (mm >> 2), i = mm & 3;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) s += red[(((ww * NT + nt) * MT + mt) * 4 + i) * 64 + ln];
    // split tile (chain kernel): the other workgroup's partial sums, published with sc1 stores
    if (partner) s += __hip_atomic_load(gp(partner + m * 16 * NT + nn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return s;
  };
  auto operands = [&](int o) {
    if (first && o == VWA_TX) return pre;
    EpiPre e;
    epi_values<EPI, NT, SC1>(p, tile, o, e);
    return e;
  };
  if constexpr (EPI == EPI_SWIGLU) {
    for (int o = VWA_TX; o < M * 16; o += KS * 64) {
      const int m = o >> 4, q = o & 15;
      const EpiPre e = operands(o);
      const float sc = rs[m];
      float gv = red_at(m, q) * sc * e.cs0, uv = red_at(m, 16 + q) * sc * e.cs1;
      if (p.bias) {
        gv += bf2f(gld(p.bias + n0 + q));
        uv += bf2f(gld(p.bias + n0 + 16 + q));
      }
      st_u16<SC1>(reinterpret_cast<u16*>(p.Y) + (size_t)m * p.ldy + tile * 16 + q, f2bf(silu(gv) * uv));
    }
  } else if constexpr (EPI == EPI_QKV) {
    const int hd = p.head_dim, half = hd >> 1;
    const int head = n0 / hd;
    const int t = (n0 % hd) >> 4;
    const bool is_v = head >= p.n_q_heads + p.n_kv_heads;
    for (int o = VWA_TX; o < M * 16; o += KS * 64) {
      const int m = o >> 4, q = o & 15;
      const EpiPre e = operands(o);
      const float sc = rs[m];
      float v = red_at(m, q), pv = red_at(m, q ^ 8);
      if (mus) {
        v -= mus[m] * gld(p.ln_c + n0 + q);
        pv -= mus[m] * gld(p.ln_c + n0 + (q ^ 8));
      }
      v *= sc * e.cs0;
      pv *= sc * e.cs1;
      if (p.bias) {
        v += bf2f(gld(p.bias + n0 + q));
        pv += bf2f(gld(p.bias + n0 + (q ^ 8)));
      }
      const int d = (q < 8) ? (8 * t + q) : (half + 8 * t + q - 8);
      if (p.use_rope && !is_v) v = (q < 8) ? (v * e.rc - pv * e.rsn) : (v * e.rc + pv * e.rsn);
      const u16 out = f2bf(v);
      if (head < p.n_q_heads) {
        st_u16<SC1>(p.q_out + (size_t)m * p.ldq + head * hd + d, out);
      } else {
        const int64_t slot = e.slot;
        if (slot >= 0) {
          const int64_t blk = slot / p.block_size, off = slot % p.block_size;
          const int kvh = is_v ? head - p.n_q_heads - p.n_kv_heads : head - p.n_q_heads;
          const int64_t idx = blk * p.cache_stride_block + kvh * p.cache_stride_head + off * p.cache_stride_tok + d;
          st_u16<SC1>((is_v ? p.v_cache : p.k_cache) + idx, out);
        }
      }
    }
  } else {
    for (int o = VWA_TX; o < M * 16 * NT; o += KS * 64) {
      const int m = o / (16 * NT), nn = o % (16 * NT);
      const int n = n0 + nn;
      const EpiPre e = operands(o);
      float v = red_at(m, nn);
      if (mus) v -= mus[m] * gld(p.ln_c + n);
      v *= rs[m] * e.cs0;
      if (p.bias) v += bf2f(gld(p.bias + n));
      if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
      if constexpr (EPI == EPI_RESID) v += e.r;
      if (p.y_f32) st_f32<SC1>(reinterpret_cast<float*>(p.Y) + (size_t)m * p.ldy + n, v);
      else st_u16<SC1>(reinterpret_cast<u16*>(p.Y) + (size_t)m * p.ldy + n, f2bf(v));
    }
  }
  lds_sync();
#pragma unroll
  for (int k = 0; k < NT * MT; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// MT: 16-row MFMA row fragments per weight fragment (only MT = 1 is instantiated since round 5: the
// 17..64-row form measured slower than the tiled GEMM and was removed).
template <int EPI, int NT, int KS, bool XG, int MT = 1>
__global__ __launch_bounds__(KS * 64) void skinny_stream_kernel(SkinnyParams p, int nb, int xstride, int xskew) {
  // k-groups (128 wide) per item; MT > 1: one (the X fragments of MT row tiles share the
  // register budget of the item's weights)
  constexpr int U = MT > 1 ? 1 : XG ? 2 : 4 / NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = p.M, K = p.K, N = p.N;
  u16* xs = reinterpret_cast<u16*>(smem);
  // LDS-staged X: row m at m * xstride + (m / 4) * xskew elements.  xstride = K + 8 puts row m+1
  // one 16-B bank slot after row m; the extra 64-B skew every 4 rows (xskew 32) makes each
  // ds_read_b128 lane group ({0-3,12-15,20-27}, ...: rows nl, k-quarters g) hit 16 distinct slots
  // -- without it lanes (nl, g) and (nl + 4, g - 1)... share slots, a 2-way conflict on every read.
  const int xbytes = XG ? 0 : ((M * xstride * 2) + 4 * xskew * 2 + 15) & ~15;
  float* red = reinterpret_cast<float*>(smem + xbytes);  // [KS][NT][MT][4][64]
  auto xrow = [&](int m) { return m * xstride + (m >> 2) * xskew; };
  float* rs = red + KS * NT * MT * 4 * 64;                // [16 MT] row scales (1/rms, LayerNorm rstd)
  float* mu = rs + 16 * MT;                               // [16 MT] row means (folded LayerNorm)
  const float* mus = (p.fuse_rms == 2) ? mu : nullptr;
  const int lane = VWA_TX & 63, w = VWA_TX >> 6;
  const int nl = lane & 15, g = lane >> 4;

  EpiPre pre;
  epi_values<EPI, NT>(p, blockIdx.x, VWA_TX, pre);  // first tile's epilogue operands, early
  const int G = K / 128;
  const int gb = (G * w) / KS, ge = (G * (w + 1)) / KS;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)N * K * 2), 0x00020000);
  // X fragments (XG): lane (row nl, k-quarter g); rows >= M read the zero OOB answer
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.X), (short)0, (int)((size_t)M * p.ldx * 2), 0x00020000);
  const int ntiles = N / (16 * NT);
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  // grammar-masked LM head (p.col_mask; the launcher keeps it only for NT 1, EPI store, LDS-staged
  // X and <= 64 tiles per workgroup): this workgroup's tiles that hold an admissible token of some
  // row, compacted into lanes (lane k: the k-th live tile).  Measured on the intent grammar: 42 %
  // of the LM head's tiles live per decode step on average, 10 % at the median.
  const bool masked = NT == 1 && !XG && p.col_mask != nullptr;
  int n_live = my_tiles, live_tile = 0;
  if (masked) {
    const int tl = (int)blockIdx.x + lane * (int)gridDim.x;
    unsigned bits = 0;
    if (lane < my_tiles)
      for (int r = 0; r < p.col_mask_rows; ++r) bits |= p.col_mask[(size_t)r * p.col_mask_ld + (tl >> 1)];
    bits = (tl & 1) ? (bits >> 16) : (bits & 0xFFFFu);
    const unsigned long long live = __ballot(lane < my_tiles && bits != 0u);
    n_live = __popcll(live);
    const int rank = __popcll(live & ((1ull << lane) - 1ull));
    const int dst = ((live >> lane) & 1ull) ? rank : n_live + (lane - rank);  // a permutation of the lanes
    live_tile = __builtin_amdgcn_ds_permute(dst * 4, tl);
  }
  const int n_items = n_live * nb;
  auto tile_of = [&](int it) { return masked ? __shfl(live_tile, it / nb, 64) : (int)blockIdx.x + (it / nb) * (int)gridDim.x; };

  auto load_x = [&](uint4 (&xr)[MT][U][4], int it) {
    const int b = it % nb;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kg = gb + b * U + u, row = 16 * mt + nl;
        const bool ok = (it < n_items) && (kg < ge) && (row < M);
        const unsigned base = ((unsigned)row * (unsigned)p.ldx + (unsigned)(kg * 128 + 32 * g)) * 2u;
#pragma unroll
        for (int s = 0; s < 4; ++s) xr[mt][u][s] = bload(rx, ok ? base + 16u * s : kOOB);
      }
  };

  auto load_item = [&](uint4 (&wr)[NT][U][4], int it) {
    const int tile = tile_of(it);
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      const bool ok = (it < n_items) && (kg < ge);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if (p.w_tiled) {  // pre-tiled: 1 KB contiguous per load instruction
          const unsigned T = (unsigned)(tile * NT + nt);
          const unsigned base = ((T * (unsigned)G + (unsigned)kg) * 4u) * 1024u + (unsigned)lane * 16u;
#pragma unroll
          for (int s = 0; s < 4; ++s) wr[nt][u][s] = bload(rw, ok ? base + 1024u * s : kOOB);
        } else {
          const unsigned row = (unsigned)(tile * 16 * NT + nt * 16 + nl);
          const unsigned base = (row * (unsigned)K + (unsigned)(kg * 128 + 32 * g)) * 2u;
#pragma unroll
          for (int s = 0; s < 4; ++s) wr[nt][u][s] = bload(rw, ok ? base + 16u * s : kOOB);
        }
      }
    }
  };

  f32x4 acc[NT * MT];
#pragma unroll
  for (int k = 0; k < NT * MT; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute_item = [&](const uint4 (&wr)[NT][U][4], const uint4 (&xr)[MT][U][4], int it) {
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      if (kg >= ge) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          uint4 a = make_uint4(0, 0, 0, 0);
          if constexpr (XG) a = xr[mt][u][s];
          else if (16 * mt + nl < M)
            a = *reinterpret_cast<const uint4*>(xs + xrow(16 * mt + nl) + kg * 128 + 32 * g + 8 * s);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[nt * MT + mt] = mfma16(as_bf16x8(a), as_bf16x8(wr[nt][u][s]), acc[nt * MT + mt]);
        }
      }
    }
  };

  auto finish_tile = [&](int it) {
    tile_epilogue<EPI, NT, KS, false, MT>(p, red, rs, mus, tile_of(it), acc, w, lane, pre, !masked && it < nb);
  };

  uint4 A[NT][U][4], B[NT][U][4];
  uint4 XA[MT][U][4], XB[MT][U][4];  // XG only (dead otherwise)
  // w_first: issue the first weight item before staging X (its round trip then overlaps the X
  // staging + fused-RMSNorm statistics); otherwise stage X first (the X round trip is short).
  if (p.w_first) {
    load_item(A, 0);
    if constexpr (XG) load_x(XA, 0);
  }
  // ---- stage X rows into LDS
  const int k8 = K / 8;
  if constexpr (!XG) {
    for (int c = VWA_TX; c < M * k8; c += KS * 64) {
      const int m = c / k8, kk = c % k8;
      *reinterpret_cast<uint4*>(xs + xrow(m) + kk * 8) =
          *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8);
    }
  }
  lds_sync();
  for (int m = w; m < 16 * MT; m += KS) {
    float sc = 1.f, mean = 0.f;
    if (p.fuse_rms && m < M) {
      float s = 0.f, s1 = 0.f;
      for (int kk = lane; kk < k8; kk += 64) {
        float f[8];
        unpack8(XG ? *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8)
                   : *reinterpret_cast<const uint4*>(xs + xrow(m) + kk * 8), f);
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
  lds_sync();

  if (!p.w_first) {
    load_item(A, 0);
    if constexpr (XG) load_x(XA, 0);
  }
  // the next item into a register set is issued right after that set's compute, BEFORE the tile
  // epilogue, so two items stay in flight through every epilogue
  load_item(B, 1);
  if constexpr (XG) load_x(XB, 1);
  for (int it = 0; it < n_items; it += 2) {
    compute_item(A, XA, it);
    load_item(A, it + 2);
    if constexpr (XG) load_x(XA, it + 2);
    if (it % nb == nb - 1) finish_tile(it);
    if (it + 1 >= n_items) break;
    compute_item(B, XB, it + 1);
    load_item(B, it + 3);
    if constexpr (XG) load_x(XB, it + 3);
    if ((it + 1) % nb == nb - 1) finish_tile(it + 1);
  }
}

int g_x_skew = 32;  // LDS X row skew (elements per 4 rows; 0: none -- A/B knob, vwa_skinny_set_x_skew)

template <int EPI, int NT, int KS, bool XG, int MT = 1>
int launch_v(const SkinnyParams& p, hipStream_t st, int grid_cap, size_t lds, int xstride) {
  constexpr int U = MT > 1 ? 1 : XG ? 2 : 4 / NT;
  const int G = p.K / 128;
  const int per_wave = (G + KS - 1) / KS;
  const int nb = (per_wave + U - 1) / U;
  const int ntiles = p.N / (16 * NT);
  const int grid = ntiles < grid_cap ? ntiles : grid_cap;
  hipLaunchKernelGGL((skinny_stream_kernel<EPI, NT, KS, XG, MT>), dim3(grid), dim3(KS * 64), lds, st, p, nb, xstride,
                     XG ? 0 : g_x_skew);
  return 0;
}

template <int EPI, int NT, int KS>
int launch(const SkinnyParams& p0, hipStream_t st, int grid_cap) {
  SkinnyParams p = p0;
  const int xstride = p.K + 8;
  // (round 4's 17..64-row form -- X streamed next to the weights, 2 / 4 row fragments per weight
  // fragment -- measured slower than the tiled GEMM for whole decode steps and was removed in round
  // 5: more than 16 rows are the tiled GEMM's, gemm.hip)
  if (p.M > 16) return -10;
  const size_t xbytes = ((size_t)p.M * xstride * 2 + 4 * g_x_skew * 2 + 15) & ~(size_t)15;
  const size_t red = (size_t)(KS * NT * 4 * 64 + 32) * sizeof(float);  // + row scales + row means
  // X rows staged in LDS when they fit next to the reduction scratch; otherwise (the down
  // projection's 14336-wide rows at more than ~5 rows) streamed from L2 with the weights (XG)
  const bool lds_x = xbytes + red <= 160 * 1024;
  if (p.col_mask) {  // the masked tile list: NT 1, EPI store, LDS-staged X, <= 64 tiles per workgroup
    const int ntiles = p.N / (16 * NT), grid = ntiles < grid_cap ? ntiles : grid_cap;
    if (EPI != EPI_STORE || NT != 1 || !lds_x || (ntiles + grid - 1) / grid > 64 || p.col_mask_rows < 1)
      p.col_mask = nullptr;
  }
  if (lds_x) return launch_v<EPI, NT, KS, false>(p, st, grid_cap, xbytes + red, xstride);
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
  const int lane = VWA_TX & 63, w = VWA_TX >> 6;
  const int nl = lane & 15, g = lane >> 4;
  const int k8 = K / 8;

  EpiPre pre;
  epi_values<EPI, NT>(p, blockIdx.x, VWA_TX, pre);  // first tile's epilogue operands, early
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
  lds_sync();
  // ---- quantise X rows into LDS (e4m3, 8 values -> 8 bytes)
  for (int c = VWA_TX; c < M * k8; c += KS * 64) {
    const int m = c / k8, kk = c % k8;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8), f);
    const float iv = inv[m];
    uint2 q;
    q.x = cvt_pk_fp8(f[0] * iv, f[1] * iv) | (cvt_pk_fp8(f[2] * iv, f[3] * iv) << 16);
    q.y = cvt_pk_fp8(f[4] * iv, f[5] * iv) | (cvt_pk_fp8(f[6] * iv, f[7] * iv) << 16);
    *reinterpret_cast<uint2*>(xs + m * xstride + kk * 8) = q;
  }
  lds_sync();

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
        if (p.w_tiled) {
          // fp8 tiled layout (ops.tile_weight_fp8): the (16-row tile, k-group) block is 2 KB
          // [s][lane][16 B] -- each load instruction reads 1 KB contiguous, lane (nl, g) gets
          // W[row][128 kg + 32 g + 16 s .. + 16), the same bytes as the row-major addressing below
          const unsigned T = (unsigned)(tile * NT + nt);
          const unsigned base = (T * (unsigned)G + (unsigned)kg) * 2048u + (unsigned)lane * 16u;
#pragma unroll
          for (int s = 0; s < 2; ++s) wr[nt][u][s] = bload(rw, ok ? base + 1024u * s : kOOB);
        } else {
          const unsigned row = (unsigned)(tile * 16 * NT + nt * 16 + nl);
          const unsigned base = row * (unsigned)K + (unsigned)(kg * 128 + 32 * g);
#pragma unroll
          for (int s = 0; s < 2; ++s) wr[nt][u][s] = bload(rw, ok ? base + 16u * s : kOOB);
        }
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
  // skinny_fp8_kernel holds 16 rows (rs[16], one MFMA row fragment): more rows must go to the
  // tiled GEMM, never to silently wrong rows 16+
  if (p.M > 16) return -10;
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


// ------------------------------------------------------------------------------------------
// Chained phases (decode, M <= 4 rows): the GEMM tail of a Llama layer -- o_proj + residual ->
// RMSNorm + gate/up + SwiGLU -> down + residual [-> RMSNorm + QKV + RoPE + KV write of the next
// layer] -- as ONE persistent launch, the phases separated by grid barriers.  What this buys
// over separate launches is the weight stream: before a workgroup waits at a barrier it has
// already issued the first weight item of the next phase (weights never depend on the
// activations), so the HBM pipe keeps streaming through the barrier, and the next phase has no
// launch boundary.  Activations crossing a barrier are written and read with sc1 (agent-scope)
// accesses; the barrier itself is an arrival counter + generation word with bounded spins (a
// timed-out spin sets an error word instead of hanging the GPU).  All workgroups must be
// co-resident: the grid is one workgroup per CU.
// ------------------------------------------------------------------------------------------
constexpr int kChainSpinLimit = 1 << 18;  // ~0.3 s: a lost workgroup ends the launch, not the GPU
// the in-launch TP rounds wait for PEER PROCESSES, whose host-side skew (graph capture, Python,
// eight ranks sharing one GPU) can exceed the intra-launch bound: ~4 s before a peer is declared lost
constexpr int kChainTpSpinLimit = 1 << 22;

// Grid barrier on monotonic 64-bit tickets (no reset, no generation word, never wraps): a
// workgroup's ticket t on its counter tells it which barrier instance it is in, so it can wait for
// that instance's completion count directly.  bar (u64 words, each in its own 128-byte line):
// flat mode uses [0]; two-level mode puts group g (block id mod 8, one per XCD under round-robin
// dispatch) at [16 g] and the top counter at [128]; [160] is the timeout flag.
// Measured (tools/chain_probe.py): a reset + generation barrier cost 5-7 us from the last
// arrival to release (four dependent agent-scope round trips).  A flat counter polled with scalar loads
// on uncached memory (256 same-address atomics) measured 121 us per chained layer vs 99.6 two-level.
constexpr int kBarTop = 128, kBarErr = 160, kBarAttnDone = 176;
// multi-layer launch (chain_kernel MULTI): per-kv-group QKV completion counters, u64 words
// kBarQkv + 16 g (each on its own 128-byte line: eight counters in one line measured 2.4 us per
// layer slower than the grid barrier -- every atomic and poll of all groups on one line) --
// monotonic, + (tiles of the group) per QKV phase.  (bar: >= 320 u64 words, ops.chain_buffers)
constexpr int kBarQkv = 192, kBarQkvStride = 16;
// diagnostic stamp slots per workgroup (ChainParams::ts): 0..8 phase edges, 9..21 attention,
// 22..53 in-phase (chain_phase pst)
constexpr int kTsStride = 64;

// Sum of the 8 group counters (mode 4/5), read with scalar loads past the scalar cache: one
// round trip for all eight (they complete on lgkmcnt, not behind the wave's weight loads).
VWA_DEVICE unsigned long long bar_sum8(const unsigned long long* bar) {
  unsigned long long v0, v1, v2, v3, v4, v5, v6, v7;
  asm volatile(
      "s_load_dwordx2 %0, %8, 0x0 glc\n\t"
      "s_load_dwordx2 %1, %8, 0x80 glc\n\t"
      "s_load_dwordx2 %2, %8, 0x100 glc\n\t"
      "s_load_dwordx2 %3, %8, 0x180 glc\n\t"
      "s_load_dwordx2 %4, %8, 0x200 glc\n\t"
      "s_load_dwordx2 %5, %8, 0x280 glc\n\t"
      "s_load_dwordx2 %6, %8, 0x300 glc\n\t"
      "s_load_dwordx2 %7, %8, 0x380 glc\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(v0), "=&s"(v1), "=&s"(v2), "=&s"(v3), "=&s"(v4), "=&s"(v5), "=&s"(v6), "=&s"(v7)
      : "s"(bar)
      : "memory");
  return v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}

// Mode 4 (5 = diagnostic without the wait): arrival is a NO-RETURN add on the workgroup's group
// counter (the wave never waits for a round trip to arrive), and the waiting wave polls the sum
// of the eight group counters.  Targets: base + i * nwg, with base read once at kernel start
// (every completed launch added a multiple of nwg; this workgroup has not arrived yet, so fewer
// than nwg arrivals of this launch can be counted in it).
VWA_DEVICE unsigned long long chain_base(const unsigned long long* bar, int nwg, int mode) {
  if (mode < 4 || VWA_TX >= 64) return 0;
  const unsigned long long s = bar_sum8(bar);
  return (s / (unsigned long long)nwg) * (unsigned long long)nwg;
}

VWA_DEVICE unsigned long long chain_arrive(unsigned long long* bar, int nwg, int mode, unsigned long long& next) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores are performed
  lds_sync();
  if (mode >= 4) {
    if (VWA_TX == 0) __hip_atomic_fetch_add(gp(&bar[16 * (blockIdx.x & 7)]), 1ull, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    next += (unsigned long long)nwg;
    return next;
  }
  unsigned long long target = 0;
  if (VWA_TX == 0) {
    if (mode == 0) {
      const unsigned long long t = __hip_atomic_fetch_add(gp(&bar[0]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      target = (t / (unsigned long long)nwg + 1ull) * (unsigned long long)nwg;
    } else {
      const int grp = blockIdx.x & 7;
      const unsigned long long members = (unsigned long long)((nwg - grp + 7) >> 3);
      const unsigned long long ngroups = (unsigned long long)(nwg < 8 ? nwg : 8);
      const unsigned long long t =
          __hip_atomic_fetch_add(gp(&bar[16 * grp]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t % members == members - 1ull)
        __hip_atomic_fetch_add(gp(&bar[kBarTop]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      target = (t / members + 1ull) * ngroups;
    }
  }
  return target;
}

VWA_DEVICE void chain_wait(unsigned long long* bar, unsigned long long target, int mode) {
  if (mode == 3 || mode == 5) {  // DIAGNOSTIC ONLY (tools/chain_probe.py --no-wait): arrive, never
    lds_sync();             // wait -> wrong results; what the phases cost without dependencies
    return;
  }
  if (mode == 4) {
    if (VWA_TX < 64) {
      const unsigned long long tgt = __builtin_amdgcn_readfirstlane((unsigned)target) |
                                     ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(target >> 32)) << 32);
      int spins = 0;
      while ((long long)(bar_sum8(bar) - tgt) < 0) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kChainSpinLimit) {
          if (VWA_TX == 0) __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    lds_sync();
    return;
  }
  if (mode == 2) {
    // wave 0 polls with scalar loads (glc: past the scalar cache; bar lives in uncached memory so
    // no L2 copy can be stale): SMEM completes on lgkmcnt, so the poll is not queued behind the
    // next phase's weight loads this wave just issued (vmcnt retires in order)
    if (VWA_TX < 64) {
      const unsigned long long tgt = __builtin_amdgcn_readfirstlane((unsigned)target) |
                                     ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(target >> 32)) << 32);
      const unsigned long long* top = &bar[kBarTop];
      int spins = 0;
      while (true) {
        unsigned long long v;
        asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(top) : "memory");
        if ((long long)(v - tgt) >= 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kChainSpinLimit) {
          if (VWA_TX == 0) __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    lds_sync();
    return;
  }
  if (VWA_TX == 0) {
    unsigned long long* w = mode == 0 ? &bar[0] : &bar[kBarTop];
    int spins = 0;
    while ((long long)(__hip_atomic_load(gp(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kChainSpinLimit) {
        __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  lds_sync();
}

// Tensor-parallel round (ChainParams::tp, world > 1) after a row-parallel phase whose epilogue
// wrote this rank's f32 partial rows into stage[rank] + region * tp.region: publish (system-scope
// release, grid barrier), workgroup 0 signals every peer, every workgroup waits for every peer's
// signal (bounded: a missing peer raises the error word), then reduces its slice of the M x d rows
// into h (h += partials summed in rank order: the same bits on every rank).  The caller's next
// grid barrier orders the slices before any workgroup reads h.
VWA_DEVICE void chain_tp_reduce(const ChainParams& cp, int region, int target, unsigned long long* bar, int nwg,
                                unsigned long long& bar_next) {
  const ChainTP& tp = cp.tp;
  __threadfence_system();
  const unsigned long long gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
  chain_wait(bar, gen, cp.bar_mode);
  if (blockIdx.x == 0 && VWA_TX < tp.world)
    __hip_atomic_store(gp(tp.flag_out[VWA_TX]), target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (VWA_TX < tp.world) {
    const int* f = tp.flag_in + VWA_TX;
    int spins = 0;
    while (__hip_atomic_load(gp(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - target < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kChainTpSpinLimit) {
        __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  const SkinnyParams& hp = cp.ph[1].p;  // gate/up's X: the hidden rows h
  u16* h = const_cast<u16*>(hp.X);
  const int d = hp.K, n4 = hp.M * d / 4;  // (d % 128 == 0: a 4-float group never crosses a row)
  const int per = (n4 + nwg - 1) / nwg, lo = (int)blockIdx.x * per, hi = min(n4, lo + per);
  // every peer's partials of this 16-byte group: one system-coherent 16-byte load each (sc0 sc1,
  // the system-scope atomic load's cache bits) -- a quarter of the transactions of per-float
  // atomic loads over xGMI -- all issued before any is summed, rank order kept (identical bits)
  constexpr int kMaxW = 8;
  __amdgpu_buffer_rsrc_t rs[kMaxW];
#pragma unroll
  for (int q = 0; q < kMaxW; ++q)
    rs[q] = __builtin_amdgcn_make_buffer_rsrc(q < tp.world ? tp.stage[q] + (size_t)region * tp.region : tp.stage[0],
                                              (short)0, (int)(tp.region * sizeof(float)), 0x00020000);
  for (int i = lo + VWA_TX; i < hi; i += (int)blockDim.x) {
    const int m = (4 * i) / d, c = 4 * i - m * d;
    u32x4 part[kMaxW];
#pragma unroll
    for (int q = 0; q < kMaxW; ++q)
      if (q < tp.world) part[q] = __builtin_amdgcn_raw_buffer_load_b128(rs[q], 16 * i, 0, 17);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < kMaxW; ++q)
      if (q < tp.world) {
        const float4 f = __builtin_bit_cast(float4, part[q]);
        acc[0] += f.x;
        acc[1] += f.y;
        acc[2] += f.z;
        acc[3] += f.w;
      }
    u16* hp_ = h + (size_t)m * hp.ldx + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) st_u16<true>(hp_ + j, f2bf(bf2f(ld_u16<true>(hp_ + j)) + acc[j]));
  }
}

// Work distribution (measured: with whole tiles per workgroup, gate/up's 896 tiles over 256
// workgroups left half of them a fourth tile -- 65 us max vs 54 us median): a phase is a list of
// ntiles x nb units (unit = one k-batch of every wave's K slice of a tile) and workgroup b takes
// the contiguous range [units*b/grid, units*(b+1)/grid).  A tile whose units straddle two ranges
// is finished by whichever of its two workgroups arrives second: both publish their reduced
// partial tile (sc1 stores) into a per-tile slot and draw a ticket; the second adds the other
// slot to its own sums and runs the epilogue.  The host guarantees <= 2 workgroups per tile.
struct PhaseRange {
  int u0, n_items, gb, ge;
};

// wb0 / wn: the phase's units go to the wn workgroups [wb0, wb0 + wn) (others get none); wn = 0:
// every workgroup
template <int KS>
VWA_DEVICE PhaseRange chain_range(const ChainPhase& ph, int wb0 = 0, int wn = 0) {
  PhaseRange r;
  const int w = VWA_TX >> 6;
  const int G = ph.p.K / 128;
  r.gb = (G * w) / KS;
  r.ge = (G * (w + 1)) / KS;
  const long long units = (long long)(ph.p.N / (16 * ph.nt)) * ph.nb;
  const long long n = wn > 0 ? wn : (long long)gridDim.x, b = (long long)blockIdx.x - wb0;
  if (b < 0 || b >= n) {
    r.u0 = 0;
    r.n_items = 0;
    return r;
  }
  r.u0 = (int)(units * b / n);
  r.n_items = (int)(units * (b + 1) / n) - r.u0;
  return r;
}

// weight item `it` (unit u0 + it) of phase p into the registers wr (NT * U <= 4 groups of 4)
// XG (ChainPhase::xg, the down projection with more rows than its X fits LDS): the item is half
// the weight k-groups (U = 2: registers 0..7) plus the matching X fragments of rows nl < M
// (registers 8..15, sc1 loads -- X was written earlier in this launch; L2-resident), so the phase
// needs no X staging and no more registers
// wx = false (XG): the weights only -- an item issued before the barrier wait must not read X,
// which other workgroups are still writing; its X fragments follow after the wait (chain_load_x)
// F8 (fp8 tiled weights, ops.tile_weight_fp8): a k-group of a 16-row tile is 2 KB, two 16-byte
// loads per lane (registers (nt * U + u) * 2 + s2, 16 e4m3 each = k 32 g + 16 s2 .. + 16), so an
// item of the same 16 registers covers twice the k-groups; chain_phase converts them to bf16
// fragments in registers (v_cvt_scalef32_pk_bf16_fp8) -- W8A16, half the weight bytes
template <int NT, int U, int WA, int R, bool XG = false, bool F8 = false>
VWA_DEVICE void chain_load(const SkinnyParams& p, int nb, uint4 (&wr)[R], int it, const PhaseRange& r, bool wx = true) {
  // (XG: the weights in registers 0 .. 4 NT U - 1, the X fragments from register 8)
  static_assert(XG ? (NT * U * 4 <= 8 && 8 + U * 4 <= R && !F8) : NT * U * (F8 ? 2 : 4) == R,
                "an item fills its register set");
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)p.N * p.K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rxg =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.X), (short)0, XG ? (int)((size_t)p.M * p.ldx * 2) : 0, 0x00020000);
  const int lane = VWA_TX & 63, nl = lane & 15, g = lane >> 4;
  const int unit = r.u0 + it;
  const int tile = unit / nb, b = unit % nb;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int kg = r.gb + b * U + u;
    const bool ok = (it < r.n_items) && (kg < r.ge);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if constexpr (F8) {
        const unsigned T = (unsigned)(tile * NT + nt);
        const unsigned base = (T * (unsigned)(p.K / 128) + (unsigned)kg) * 2048u + (unsigned)lane * 16u;
        const unsigned vb = ok ? base : kOOB2;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) wr[(nt * U + u) * 2 + s2] = bload_w_so<WA>(rw, vb, 1024 * s2);
      } else if (p.w_tiled) {
        // pre-tiled weights (ops.tile_weight): each load instruction reads 1 KB contiguous.
        // Measured (tools/chain_probe.py, Llama-3-8B layer tail): 89.6 vs 101.4 us at 1 row,
        // 96.3 vs 106.8 us at 4 rows against the row-major [N, K] access
        const unsigned T = (unsigned)(tile * NT + nt);
        const unsigned base = ((T * (unsigned)(p.K / 128) + (unsigned)kg) * 4u) * 1024u + (unsigned)lane * 16u;
        const unsigned vb = ok ? base : kOOB2;
#pragma unroll
        for (int s = 0; s < 4; ++s) wr[(nt * U + u) * 4 + s] = bload_w_so<WA>(rw, vb, 1024 * s);
      } else {
        const unsigned row = (unsigned)(tile * 16 * NT + nt * 16 + nl);
        const unsigned base = (row * (unsigned)p.K + (unsigned)(kg * 128 + 32 * g)) * 2u;
        const unsigned vb = ok ? base : kOOB2;
#pragma unroll
        for (int s = 0; s < 4; ++s) wr[(nt * U + u) * 4 + s] = bload_w_so<WA>(rw, vb, 16 * s);
      }
    }
    if constexpr (XG) {
      if (!wx) continue;
      const unsigned xb =
          ok && nl < p.M ? ((unsigned)nl * (unsigned)p.ldx + (unsigned)(kg * 128 + 32 * g)) * 2u : kOOB2;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rxg, (int)xb, 16 * s, 16);
        wr[8 + u * 4 + s] = make_uint4(v.x, v.y, v.z, v.w);
      }
    }
  }
}

// the X fragments (registers 8..15) of an XG item whose weights went out before the barrier wait
template <int U, int R>
VWA_DEVICE void chain_load_x(const SkinnyParams& p, int nb, uint4 (&wr)[R], int it, const PhaseRange& r) {
  static_assert(8 + U * 4 <= R, "XG items: weight registers 0..7, X fragments from register 8");
  const __amdgpu_buffer_rsrc_t rxg =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.X), (short)0, (int)((size_t)p.M * p.ldx * 2), 0x00020000);
  const int lane = VWA_TX & 63, nl = lane & 15, g = lane >> 4;
  const int b = (r.u0 + it) % nb;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int kg = r.gb + b * U + u;
    const bool ok = (it < r.n_items) && (kg < r.ge) && nl < p.M;
    const unsigned xb = ok ? ((unsigned)nl * (unsigned)p.ldx + (unsigned)(kg * 128 + 32 * g)) * 2u : kOOB2;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rxg, (int)xb, 16 * s, 16);
      wr[8 + u * 4 + s] = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
}

// LDS item (cp.lds_item): weight item `it` of this workgroup's range of a phase, LDS-DMA'd into
// dst + wave * 16 KB in the register-set order (load k of the item -> dst + k KB, lane l's 16 bytes
// at + 16 l).  Issued during the attention window, when HBM idles behind the latency-bound
// attention and o_proj; the bandwidth-bound gate/up phase then streams one item less per
// workgroup (measured: 5.5 us per item, tools/chain_probe.py --diag-skip).  Pre-tiled weights.
// F8: the fp8 tiled item (chain_load F8: two 1 KB loads per k-group, register (nt * U + u) * 2 + s2)
template <int NT, int U, int WA, bool F8 = false>
VWA_DEVICE void chain_preload(const SkinnyParams& p, int nb, const PhaseRange& r, int it, char* dst) {
  static_assert(NT * U * (F8 ? 2 : 4) <= 16, "an item = at most 16 loads of 1 KB per wave (16 KB of LDS)");
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)p.N * p.K * 2), 0x00020000);
  const unsigned lane = VWA_TX & 63;
  char* wd = dst + (VWA_TX >> 6) * 16384;
  const int unit = r.u0 + it;
  const int tile = unit / nb, b = unit % nb;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int kg = r.gb + b * U + u;
    const bool ok = it < r.n_items && kg < r.ge;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const unsigned T = (unsigned)(tile * NT + nt);
      constexpr int LPK = F8 ? 2 : 4;  // 1 KB loads per k-group
      const unsigned base = ((T * (unsigned)(p.K / 128) + (unsigned)kg) * (unsigned)LPK) * 1024u + lane * 16u;
      const unsigned vb = ok ? base : kOOB2;
#pragma unroll
      for (int s = 0; s < LPK; ++s)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rw, (__attribute__((address_space(3))) void*)(wd + ((nt * U + u) * LPK + s) * 1024), 16, vb, 1024 * s, 0, WA);
    }
  }
}

// loads per weight item (register set): 16 with 8 waves per workgroup, 8 with 16 waves (a wave's
// VGPR budget halves with twice the waves).  fp8 (W8A16) items: 8 loads -- with 16 the fp8
// instantiations ran out of VGPRs at the barrier pre-issue (each new weight register spilled to
// scratch behind an s_waitcnt vmcnt(0): the item's loads serialised)
template <int KS, bool F8 = false>
struct ChainShape {
  static constexpr int R = (KS == 16 || F8) ? 8 : 16;
};

// W2: a plain phase in 32-column tiles (the chained o_proj, ChainParams::o_nt2; the X-streaming
// down projection, ChainParams::d_nt2: one k-group of two tiles per item, every X fragment feeds
// both -- half the X bytes per weight byte)
template <int EPI, int KS = 8, bool XG = false, bool F8 = false, bool W2 = false>
struct PhaseShape {
  static constexpr int NT = (EPI == EPI_SWIGLU || W2) ? 2 : 1;
  // (measured: QKV in half-tile units -- 384 tiles -> 3 units per workgroup, one split tile each --
  // 12.5-13.4 us vs 6.7 median / 11.5 max with whole tiles, also with the split tile processed
  // first and published before the next item's loads under a counted vmcnt)
  static constexpr int U = XG ? (W2 ? 1 : 2) : ChainShape<KS, F8>::R / 4 / NT * (F8 ? 2 : 1);
};

// the phase's first weight item (and with pre2 its second) before the barrier wait: a
// workgroup that arrives early keeps HBM busy while the grid catches up
template <int EPI, int KS, int WA, bool XG = false, bool F8 = false, bool W2 = false, int R>
VWA_DEVICE void chain_issue_first(const ChainPhase& ph, uint4 (&wr)[R], uint4 (&wr2)[R], int pre2, int wb0 = 0,
                                  int wn = 0) {
  using S = PhaseShape<EPI, KS, XG, F8, W2>;
  const PhaseRange r = chain_range<KS>(ph, wb0, wn);
  // (issued before the barrier wait: XG items without their X fragments, chain_phase adds them)
  chain_load<S::NT, S::U, WA, R, XG, F8>(ph.p, ph.nb, wr, 0, r, !XG);
  if (pre2) chain_load<S::NT, S::U, WA, R, XG, F8>(ph.p, ph.nb, wr2, 1, r, !XG);
}

// one weight item `it` of a phase into wr (the next phase's item 0 / item 1, see chain_kernel)
template <int EPI, int KS, int WA, bool XG = false, bool F8 = false, bool W2 = false, int R>
VWA_DEVICE void chain_issue_item(const ChainPhase& ph, uint4 (&wr)[R], int it, int wb0 = 0, int wn = 0) {
  using S = PhaseShape<EPI, KS, XG, F8, W2>;
  const PhaseRange r = chain_range<KS>(ph, wb0, wn);
  chain_load<S::NT, S::U, WA, R, XG, F8>(ph.p, ph.nb, wr, it, r);
}

// partial tile of a split tile: cross-wave sums of this workgroup's units -> slot (sc1)
template <int NT, int KS>
VWA_DEVICE void tile_publish(int M, float* red, f32x4 (&acc)[NT], float* slot) {
  const int lane = VWA_TX & 63, w = VWA_TX >> 6;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[((w * NT + nt) * 4 + i) * 64 + lane] = acc[nt][i];
  lds_sync();
  for (int o = VWA_TX; o < M * 16 * NT; o += KS * 64) {
    const int m = o / (16 * NT), nn = o % (16 * NT);
    const int nt = nn >> 4, q = nn & 15;
    const int ln = q + 16 * (m >> 2), i = m & 3;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) v += red[((ww * NT + nt) * 4 + i) * 64 + ln];
    st_f32<true>(slot + o, v);
  }
  lds_sync();
}

// One phase.  X0 holds this phase's item 0 (issued before the barrier wait), X1 item 1 when pre2.
// cp.xdma: the LAST wave stages X alone, by LDS-DMA (no registers, all pieces in flight at once),
// and issues no weights at the barrier -- its vmcnt queue is empty, so the X round trip is not
// queued behind weight loads; the other waves issue their item 1 at once (pre2 == 0: one item at
// the barrier), which streams while the X rows arrive.  hs = items the staging wave has already
// issued into (X0, X1).
template <int EPI, int KS, int WA, bool XG = false, bool F8 = false, bool W2 = false, int R>
VWA_DEVICE void chain_phase(const ChainParams& cp, int i, uint4 (&X0)[R], uint4 (&X1)[R], char* smem, int pre2,
                            int hs = 0, int wb0 = 0, int wn = 0, bool has0 = true) {
  constexpr int NT = PhaseShape<EPI, KS, XG, F8, W2>::NT, U = PhaseShape<EPI, KS, XG, F8, W2>::U;
  const ChainPhase& ph = cp.ph[i];
  const SkinnyParams& p = ph.p;
  const int nb = ph.nb, M = p.M, K = p.K;
  const int xstride = K + 8;
  u16* xs = reinterpret_cast<u16*>(smem);
  const int xbytes = XG ? 0 : ((M * xstride * 2) + 15) & ~15;  // (XG: X fragments stream in the items)
  float* red = reinterpret_cast<float*>(smem + xbytes);
  float* rs = red + KS * NT * 4 * 64;  // [16] row scales (1/rms or LayerNorm rstd)
  float* mu = rs + 16;                  // [16] row means (folded LayerNorm)
  int* s_flag = reinterpret_cast<int*>(rs + 32);
  const float* mus = p.fuse_rms == 2 ? mu : nullptr;
  const int lane = VWA_TX & 63, w = VWA_TX >> 6;
  const int nl = lane & 15, g = lane >> 4;
  const PhaseRange r = chain_range<KS>(ph, wb0, wn);
  const int first_tile = r.u0 / nb;
  const bool xdma = cp.xdma != 0, stager = xdma && w == KS - 1 && !XG;
  // diagnostic in-phase stamps (tools/chain_probe.py, wave 0): phase i -> slots 22 + 8 i + k
  // (entry, X staged, row scales, item 0 computed, tile 0 finished, item 1, tile 1 finished)
  auto pst = [&](int k) {
    const int slot = k < 8 ? 22 + 8 * i + k : -1;
    if (cp.ts && VWA_TX == 0 && slot >= 0) *gp(cp.ts + blockIdx.x * kTsStride + slot) = __builtin_amdgcn_s_memrealtime();
  };
  pst(0);
  if constexpr (XG) {  // X fragments of the items issued before the barrier wait (weights only)
    chain_load_x<U>(p, nb, X0, 0, r);
    if (pre2) chain_load_x<U>(p, nb, X1, 1, r);
  }
  // ---- stage X (written by the previous phase: sc1 loads) + RMSNorm row scales
  const int k8 = K / 8;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.X), (short)0, (int)((size_t)M * p.ldx * 2), 0x00020000);
  if (stager) {
    // 1 KB pieces (512 bf16 of one row) straight into the padded LDS rows, sc1 (coherent) reads
    const int pieces = K / 512;
    for (int m = 0; m < M; ++m)
      for (int j = 0; j < pieces; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(xs + m * xstride + j * 512), 16,
            (unsigned)(((size_t)m * p.ldx + j * 512) * 2 + lane * 16), 0, 0, 16);
    asm volatile("" ::: "memory");  // keep the weight loads below younger than the pieces
  }
  // cp.xfirst: a CU's vector memory requests are served in order (measured, tools/
  // crit_latency_probe.hip: a load behind 112-224 KB of the same CU's weight loads takes 2-4 us,
  // 0.12 us on a CU whose own queue is empty while the others stream) -- so the other waves issue
  // their next weight item only after the staging wave's X pieces are in the queue
  // cp.xwait: the CU's memory pipe is SHARED by its waves (measured: one wave's 28 KB of X pieces
  // land in 1.1 us on a quiet CU, 5.6 us while 7 other waves stream weights) -- so no wave issues
  // weights until the X rows are in LDS; the items pre-issued at the barrier arrival have had the
  // barrier window to land
  const bool xw = xdma && cp.xwait;
  if (xdma && cp.xfirst && !xw) lds_sync();
  auto issue_rest = [&]() {
    if (xdma && !stager && !has0) chain_load<NT, U, WA, R, XG, F8>(p, nb, X0, 0, r);  // (not issued at the barrier)
    if (xdma && !stager && (!pre2 || !has0)) chain_load<NT, U, WA, R, XG, F8>(p, nb, X1, 1, r);  // streams during the staging
  };
  if (!xw) issue_rest();

  EpiPre pre;
  if (r.n_items > 0 && !xw) epi_values<EPI, NT, true>(p, first_tile, VWA_TX, pre);
  if (stager && xw) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pieces (the staging wave issued nothing else)
  } else if (stager) {
    int nw = 0;
    if (hs < 1) {
      chain_load<NT, U, WA, R, XG, F8>(p, nb, X0, 0, r);
      ++nw;
    }
    if (hs < 2) {
      chain_load<NT, U, WA, R, XG, F8>(p, nb, X1, 1, r);
      ++nw;
    }
    // the pieces are older than the nw weight items (16 loads each): wait for them only
    if constexpr (R == 16) {
      if (nw == 2) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else if (nw == 1) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      static_assert(R == 8, "item sizes: 16 or 8 loads");
      if (nw == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if (nw == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else if (!xdma && !XG) {
    for (int c = VWA_TX; c < M * k8; c += KS * 64) {
      const int m = c / k8, kk = c % k8;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rx, (int)(((size_t)m * p.ldx + kk * 8) * 2), 0, 16);
      *reinterpret_cast<uint4*>(xs + m * xstride + kk * 8) = make_uint4(v.x, v.y, v.z, v.w);
    }
  }
  lds_sync();
  pst(1);
  // X is in LDS: the weights (and the first tile's epilogue operands) go out after the row scales
  // -- a wave whose issue blocks on a full memory queue would hold the scales barrier
  auto issue_xw = [&]() {
    issue_rest();
    if (stager) {
      if (hs < 1) chain_load<NT, U, WA, R, XG, F8>(p, nb, X0, 0, r);
      if (hs < 2) chain_load<NT, U, WA, R, XG, F8>(p, nb, X1, 1, r);
    }
    if (r.n_items > 0) epi_values<EPI, NT, true>(p, first_tile, VWA_TX, pre);
  };
  if (xw && !cp.xw_late) issue_xw();
  for (int m = w; m < 16; m += KS) {
    float sc = 1.f, mean = 0.f;
    if (p.fuse_rms && m < M && !XG) {  // (the host never folds a norm into an XG phase)
      float s = 0.f, s1 = 0.f;
      for (int kk = lane; kk < k8; kk += 64) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xs + m * xstride + kk * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s += f[j] * f[j];
          s1 += f[j];
        }
      }
      s = wave_sum(s);
      if (p.fuse_rms == 2) {  // folded LayerNorm (Whisper): rstd from E[x^2] - mean^2
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
  lds_sync();
  if (xw && cp.xw_late) issue_xw();
  pst(2);

  f32x4 acc[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](const uint4 (&wr)[R], int it) {
    const int b = (r.u0 + it) % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = r.gb + b * U + u;
      if (kg >= r.ge) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 a = make_uint4(0, 0, 0, 0);
        if constexpr (XG) a = wr[8 + u * 4 + s];
        else if (nl < M) a = *reinterpret_cast<const uint4*>(xs + nl * xstride + kg * 128 + 32 * g + 8 * s);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if constexpr (F8) {
            // 8 e4m3 of register (nt, u, s >> 1), half s & 1 -> one bf16 B fragment (k 32 g + 8 s ..);
            // the per-row scale is applied to the finished column in the epilogue (cs0 / cs1)
            const uint4 w8 = wr[(nt * U + u) * 2 + (s >> 1)];
            const unsigned d0 = (s & 1) ? w8.z : w8.x, d1 = (s & 1) ? w8.w : w8.y;
            uint4 bw;
            bw.x = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, false));
            bw.y = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d0, 1.0f, true));
            bw.z = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, false));
            bw.w = __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(d1, 1.0f, true));
            acc[nt] = mfma16(as_bf16x8(a), as_bf16x8(bw), acc[nt]);
          } else {
            acc[nt] = mfma16(as_bf16x8(a), as_bf16x8(wr[(nt * U + u) * 4 + s]), acc[nt]);
          }
        }
      }
    }
  };
  const int u1 = r.u0 + r.n_items;
  auto finish = [&](int it) {
    const int unit = r.u0 + it;
    const int tile = unit / nb;
    if (unit % nb != nb - 1 && it != r.n_items - 1) return;  // tile continues in this range
    const bool whole = tile * nb >= r.u0 && (tile + 1) * nb <= u1;
    if (whole) {
      tile_epilogue<EPI, NT, KS, true>(p, red, rs, mus, tile, acc, w, lane, pre, tile == first_tile);
      return;
    }
    // split tile: publish, ticket, the second arriver finishes it
    const int mine = tile * nb >= r.u0 ? 0 : 1;  // slot 0: owner of the tile's first unit
    const int per = M * 16 * NT;
    float* slots = cp.part + (size_t)tile * 2 * per;
    tile_publish<NT, KS>(M, red, acc, slots + mine * per);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();
    if (VWA_TX == 0) {
      const unsigned t = __hip_atomic_fetch_add(gp(&cp.tickets[tile]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == 1u;
      if (last) __hip_atomic_store(gp(&cp.tickets[tile]), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = last;
    }
    lds_sync();
    if (*s_flag) {
      tile_epilogue<EPI, NT, KS, true>(p, red, rs, mus, tile, acc, w, lane, pre, false,
                                       slots + (1 - mine) * per);
    } else {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  // items in pairs (X0, X1); an odd count is padded with one all-OOB item (zero weights, no
  // traffic, no epilogue)
  // The next item into a set is issued right after that set's compute, before the epilogue, so
  // two items stay in flight through every tile epilogue -- except after a split tile, whose
  // publish drains vmcnt (it would wait for the new loads too).
  const int n_pad = (r.n_items + 1) & ~1;
  auto split_end = [&](int it) -> bool {
    if (it >= r.n_items) return false;
    const int unit = r.u0 + it, tile = unit / nb;
    if (unit % nb != nb - 1 && it != r.n_items - 1) return false;
    return !(tile * nb >= r.u0 && (tile + 1) * nb <= u1);
  };
  if (!pre2 && !xdma) chain_load<NT, U, WA, R, XG, F8>(p, nb, X1, 1, r);
  auto ldi = [&](uint4 (&wr)[R], int idx) {
    if (idx == 2 && ((i == 1 && cp.lds_item && w < cp.lds_item_waves) ||
                     (i == 2 && cp.lds_item2 && w < cp.lds_item2_waves && !(cp.poll_free && w == 0)))) {  // preloaded (chain_preload)
      static_assert(R <= 16, "LDS item: up to 16 loads of 1 KB per wave");
      // this wave's LDS-DMA of the item must have landed (no barrier drains vmcnt any more, and
      // the compiler does not order LDS-DMA writes before these reads)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const char* src = smem + (i == 1 ? cp.lds_item : cp.lds_item2) + w * 16384 + lane * 16;
#pragma unroll
      for (int k = 0; k < R; ++k) wr[k] = *reinterpret_cast<const uint4*>(src + k * 1024);
      return;
    }
    chain_load<NT, U, WA, R, XG, F8>(p, nb, wr, idx, r);
  };
  for (int it = 0; it < n_pad; it += 2) {
    compute(X0, it);
    if (it == 0) pst(3);
    const bool e0 = !split_end(it);
    if (e0 && it + 2 < n_pad) ldi(X0, it + 2);
    finish(it);
    if (it == 0) pst(4);
    if (!e0 && it + 2 < n_pad) ldi(X0, it + 2);
    if (it + 1 >= r.n_items) break;  // padding item: no wait on it (X1 may hold the next phase's item 0)
    compute(X1, it + 1);
    if (it == 0) pst(5);
    const bool e1 = !split_end(it + 1);
    if (e1 && it + 3 < n_pad) ldi(X1, it + 3);
    finish(it + 1);
    if (it == 0) pst(6);
    if (!e1 && it + 3 < n_pad) ldi(X1, it + 3);
  }
}

// The phase sequence is static (a runtime epilogue switch measured 50+ VGPR spills):
//   SEQ 0  Llama tail       o_proj+res -> RMSNorm gate/up+SwiGLU -> down+res [-> RMSNorm QKV+RoPE+KV]
//   SEQ 1  Whisper tail     out-proj+res -> LN fc1+GELU -> fc2+res [-> LN self-attn QKV+KV]
//   SEQ 2  Whisper middle   self-attn out-proj+res -> LN cross-attn query (store)
// (Whisper LayerNorms folded into the weights, mean/rstd from the staged rows; biases in the
// epilogues.)  AG > 0 (Llama only): the layer's decode attention (GQA group AG, head_dim 128)
// runs first, as phase 0 of the same launch (mq_attention.h with 8 waves, one register set,
// outputs written through to memory); workgroups without an attention item issue their o_proj
// weights at once.  The attention phase itself is slower in the 8-wave form (13-14 us vs 10.5 us
// standalone, tools/chain_probe.py --attn), but the whole decode step gains one launch boundary
// per layer: a same-box bench A/B/A measured 3868 vs 3897 / 3907 us of GPU time per decode step,
// so this form is the model's default (VWA_CHAIN_ATTN=0 selects the separate attention launch).
template <int SEQ, int I>
struct SeqEpi {
  static constexpr int value = SEQ == 0 ? (I == 0 ? EPI_RESID : I == 1 ? EPI_SWIGLU : I == 2 ? EPI_RESID : EPI_QKV)
                               : SEQ == 1 ? (I == 0 ? EPI_RESID : I == 1 ? EPI_GELU : I == 2 ? EPI_RESID : EPI_QKV)
                                          : (I == 0 ? EPI_RESID : EPI_STORE);
};

// XG2: phase 2 (the down projection) streams its X fragments with the weights (ChainParams
// ph[2].xg: more rows than its X fits LDS, 5..16 rows, no attention phase)
// O2: phase 0 (o_proj) in 32-column tiles (ChainParams::o_nt2)
// D2: the X-streaming down projection (XG2) in 32-column tiles (ChainParams::d_nt2)
// ---- multi-layer launch: QKV -> next layer's attention, per kv group instead of a grid barrier
// The QKV phase's 16-column tiles of kv group g are the q heads g G .. g G + G - 1, k head g and v
// head g ((G + 2) hd / 16 tiles).  A workgroup that finished its QKV tiles (whole tiles: nb == 1)
// drains its stores and adds 1 per tile to its groups' counters; an attention workgroup waits only
// for the counter of ITS kv head -- the groups whose tiles finish in the phase's first round start
// their attention while the second-round tiles still run, and nobody waits for a grid barrier.
VWA_DEVICE int qkv_group(const SkinnyParams& q, int tile) {
  const int head = tile * 16 / q.head_dim, G = q.n_q_heads / q.n_kv_heads;
  return head < q.n_q_heads ? head / G : head < q.n_q_heads + q.n_kv_heads ? head - q.n_q_heads
                                                                            : head - q.n_q_heads - q.n_kv_heads;
}
VWA_DEVICE long long qkv_tiles_per_group(const SkinnyParams& q) {
  return (long long)(q.n_q_heads / q.n_kv_heads + 2) * q.head_dim / 16;
}

template <int KS>
VWA_DEVICE void qkv_signal(const ChainPhase& ph, unsigned long long* bar) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's Q / K / V stores are performed
  lds_sync();
  const PhaseRange r = chain_range<KS>(ph);
  if (VWA_TX == 0)
    for (int it = 0; it < r.n_items; ++it)
      __hip_atomic_fetch_add(gp(&bar[kBarQkv + kBarQkvStride * qkv_group(ph.p, r.u0 + it)]), 1ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 polls (scalar loads past the scalar cache, uncached words) until every group in
// [g0, g1) has reached its target; bounded like chain_wait
VWA_DEVICE void qkv_wait(unsigned long long* bar, const unsigned long long* base, unsigned long long add, int g0, int g1) {
  if (VWA_TX < 64) {
    for (int g = g0; g < g1; ++g) {
      const unsigned long long tgt = base[g] + add;
      const unsigned long long* w = &bar[kBarQkv + kBarQkvStride * g];
      int spins = 0;
      while (true) {
        unsigned long long v;
        asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(w) : "memory");
        if ((long long)(v - tgt) >= 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kChainSpinLimit) {
          if (VWA_TX == 0) __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  lds_sync();
}

// K/V prefetch of an attention workgroup's next item while it waits for the QKV counters: the
// chunk's keys older than the step's rows (never a key this launch writes) pulled into this XCD's
// L2 by LDS-DMA into a junk line of each wave's own V-image slot (mq_attention.h vimg; the wave's
// K/V waits order the DMAs before its own V-image writes, and the chain waits vmcnt(0) before any
// other LDS use of those bytes).  The attention's own K/V loads then hit L2: the cold K/V round
// trip (~4 us) leaves the critical path.  ev: the workgroup's step-plan entry (lanes:
// 3 kv head, 4 first row, 6 / 7 key range, 12 context of the group's first row).
VWA_DEVICE void kv_prefetch(const DecodeAttnParams& a, int ev, unsigned char* lds) {
  const int kvh = __builtin_amdgcn_readlane(ev, 3), r0 = __builtin_amdgcn_readlane(ev, 4);
  const int kbeg = __builtin_amdgcn_readlane(ev, 6), kend = __builtin_amdgcn_readlane(ev, 7);
  const int c0 = __builtin_amdgcn_readlane(ev, 12);
  const int nk = min(min(kend, c0 - 1) - kbeg, 128);
  if (nk <= 0 || a.kv.block_size != 16) return;
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(a.kv.k), (short)0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(a.kv.v), (short)0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(a.row_table), (short)0,
                                                                     (r0 + 1) * a.rt_stride * 4, 0x00020000);
  auto* dst = (__attribute__((address_space(3))) void*)(lds + w * kMqStep * 256);
  // 16-byte pieces: 16 per 256-byte key row; piece q of the chunk -> key kbeg + q / 16; a wave
  // takes pieces w * 64 + lane + 512 i (i < 4: nk <= 128 keys), all table loads first
  int blk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = w * 64 + lane + 512 * i, key = kbeg + q / 16;
    blk[i] = (int)__builtin_amdgcn_raw_buffer_load_b32(rt, q < nk * 16 ? (r0 * a.rt_stride + key / 16) * 4 : 0x7FFFFFF0,
                                                       0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = w * 64 + lane + 512 * i, key = kbeg + q / 16;
    if (512 * i + w * 64 >= nk * 16) break;  // wave-uniform
    const long long e = (long long)blk[i] * a.kv.stride_block + (long long)kvh * a.kv.stride_head +
                        (long long)(key & 15) * a.kv.stride_tok;
    const unsigned off = q < nk * 16 ? (unsigned)(e * 2 + (q & 15) * 16) : 0x7FFFFFF0u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, dst, 16, off, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, dst, 16, off, 0, 0, 0);
  }
}

// MULTI: ONE launch runs n_layers consecutive layers (descriptors cpp[0 .. n_layers), each a
// 4-phase Llama tail whose QKV phase feeds the next layer's attention; the last may be the
// model's last layer, a 3-phase tail).  Between layers every
// workgroup arrives at a grid barrier after its QKV tiles; only the workgroups that run an
// attention item of the next layer wait for it (they read the next layer's Q and newest K/V).  A
// workgroup the step plan (mq_attention.h, written by layer 0 of this very launch) gives no
// attention item goes straight on: it issues the next layer's o_proj weights and gate/up LDS item
// while the slow QKV tiles and the attention are still running -- no kernel boundary, no launch
// ramp, and the HBM pipe of half the CUs is busy through the QKV tail and the attention front.
// (Skipping the wait is safe for the ticket barriers: such a workgroup's next arrival happens only
// after the attention hand-off, which itself needed this barrier complete.)
template <int KS, int SEQ, int NPH, int AG, int WA, bool XG2 = false, bool F8 = false, bool O2 = false, bool D2 = false,
          bool MULTI = false>
__global__ __launch_bounds__(KS * 64) void chain_kernel(const ChainParams* __restrict__ cpp, int n_layers) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(!MULTI || (SEQ == 0 && NPH == 4 && AG > 0 && !XG2), "multi-layer launch: Llama tails with attention");
  const int nwg = (int)gridDim.x;
  unsigned long long* bar = reinterpret_cast<unsigned long long*>(cpp->bar);
  unsigned long long bar_next = chain_base(bar, nwg, cpp->bar_mode);  // mode >= 4: running target
  // TP rounds of this launch: e0 + 2 li + 1 (after layer li's o_proj), e0 + 2 li + 2 (after its
  // down); every workgroup reads e0 before its first arrival, workgroup 0 advances it after each
  // layer's last round
  const bool tpr = cpp->tp.world > 1;
  const int e0 = tpr ? __hip_atomic_load(gp(cpp->tp.epoch), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  // MULTI: the per-kv-group QKV counters' values before this launch (whole phases only: read
  // before this workgroup's first arrival, and no QKV phase of this launch starts before every
  // workgroup arrived three times); hand-off by group only with whole QKV tiles per workgroup
  unsigned long long qkv_base[8] = {};
  const bool qsig = MULTI && cpp->qkv_flags && cpp->bar_mode == 2 && cpp->ph[3].nb == 1 &&
                    cpp->ph[3].p.n_kv_heads <= 8 && cpp->attn_flag;  // (uncached words, scalar polls)
  if constexpr (MULTI) {
    if (qsig && VWA_TX < 64) {
      const unsigned long long tpg = (unsigned long long)qkv_tiles_per_group(cpp->ph[3].p);
      for (int g = 0; g < cpp->ph[3].p.n_kv_heads; ++g) {
        const unsigned long long v = __hip_atomic_load(gp(&bar[kBarQkv + kBarQkvStride * g]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        qkv_base[g] = v / tpg * tpg;
      }
    }
  }
  bool pf_prev = false, pf_next = false;  // (MULTI) the previous layer's end issued K/V prefetch DMAs
  for (int li = 0; li < (MULTI ? n_layers : 1); ++li) {
  pf_prev = pf_next;
  pf_next = false;
  const ChainParams& cp = cpp[li];  // device-resident descriptor
  // Warm the scalar cache with the whole descriptor (25 x 64-byte lines) in ONE round trip: the
  // fields are otherwise fetched behind branches and earlier fields' values, a chain of dependent
  // scalar misses (the attention prologue measured ~6 of them before its first vector load)
  static_assert(sizeof(ChainParams) <= 25 * 64, "descriptor warm-up covers 25 lines");
  {
    // (non-volatile, no memory clobber: a volatile block counts as a memory write and turns every
    // later descriptor read into a vector load; the never-true test keeps it alive)
    unsigned junk;
    asm("s_load_dword %0, %1, 0x0\n\t""s_load_dword %0, %1, 0x40\n\t""s_load_dword %0, %1, 0x80\n\t""s_load_dword %0, %1, 0xc0\n\t"
        "s_load_dword %0, %1, 0x100\n\t""s_load_dword %0, %1, 0x140\n\t""s_load_dword %0, %1, 0x180\n\t""s_load_dword %0, %1, 0x1c0\n\t"
        "s_load_dword %0, %1, 0x200\n\t""s_load_dword %0, %1, 0x240\n\t""s_load_dword %0, %1, 0x280\n\t""s_load_dword %0, %1, 0x2c0\n\t"
        "s_load_dword %0, %1, 0x300\n\t""s_load_dword %0, %1, 0x340\n\t""s_load_dword %0, %1, 0x380\n\t""s_load_dword %0, %1, 0x3c0\n\t"
        "s_load_dword %0, %1, 0x400\n\t""s_load_dword %0, %1, 0x440\n\t""s_load_dword %0, %1, 0x480\n\t""s_load_dword %0, %1, 0x4c0\n\t""s_load_dword %0, %1, 0x500\n\t"
        "s_load_dword %0, %1, 0x540\n\t""s_load_dword %0, %1, 0x580\n\t""s_load_dword %0, %1, 0x5c0\n\t""s_load_dword %0, %1, 0x600\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&s"(junk)
        : "s"(cpp + li));
    if (junk == 0x9e3779b9u) __builtin_amdgcn_s_sleep(1);
  }
  // (zeroed per layer: otherwise a path that reads a set before writing it -- only possible for
  // an all-OOB padding item -- keeps the previous layer's 128 registers live across the layer
  // loop's back edge and through the attention: spills.  Zeros cost nothing to rematerialise.)
  uint4 A[ChainShape<KS, F8>::R] = {}, B[ChainShape<KS, F8>::R] = {};
  // barrier = arrive (stores drained), issue the next phase's first weight item, then wait: the
  // weight stream is in flight while the slowest workgroup finishes
  unsigned long long gen;
  const int er = e0 + 2 * li;  // this layer's TP round base
  int nts = 0;
  auto stamp = [&]() {
    if (cp.ts && VWA_TX == 0) *gp(cp.ts + blockIdx.x * kTsStride + nts) = __builtin_amdgcn_s_memrealtime();
    ++nts;
  };
  stamp();
  constexpr int E0 = SeqEpi<SEQ, 0>::value, E1 = SeqEpi<SEQ, 1>::value, E2 = SeqEpi<SEQ, 2>::value,
                E3 = SeqEpi<SEQ, 3>::value;
  int pre0 = cp.pre2;  // phase 0's pre-issued items: two, or one for a workgroup that ran attention
  // Phase-0 window (cp.osub, attention launches): the o_proj units go only to the workgroups that
  // get no attention item -- they stream their o_proj weights during the attention, while an
  // attention workgroup loads its share only after it (measured on the critical path).
  int ob0 = 0, on = 0;
  // Phase 0 with at most one item for this workgroup (o_proj at M <= 4 rows: one tile, one
  // k-batch) never uses register set B, so B carries phase 1's first item from the start: it
  // streams during the attention phase / the launch ramp, when HBM would otherwise idle.
  bool nx = false;
  bool apre = false;  // (cp.attn_pre) phase 1's item 0 was issued into A during this workgroup's attention
  auto setup0 = [&](int n_attn) {
    const bool sub = cp.osub && n_attn > 0 && n_attn <= nwg / 2;
    ob0 = sub ? n_attn : 0;
    on = sub ? nwg - n_attn : 0;
    nx = cp.next0 && chain_range<KS>(cp.ph[0], ob0, on).n_items <= 1;
  };
  // (phase 0 always runs on (B, A) and phase 1 on (A, B): one inlined copy of each phase body --
  // swapping the sets per path measured 120 B of VGPR spills)
  auto issue0 = [&](int pre) {
    if (nx) {
      chain_issue_item<E0, KS, WA, false, F8, O2>(cp.ph[0], B, 0, ob0, on);
      chain_issue_item<E1, KS, WA, false, F8>(cp.ph[1], A, 0);
    } else {
      chain_issue_first<E0, KS, WA, false, F8, O2>(cp.ph[0], B, A, pre, ob0, on);
    }
  };
  auto preload1 = [&]() {
    chain_preload<PhaseShape<E1, KS, false, F8>::NT, PhaseShape<E1, KS, false, F8>::U, WA, F8>(
        cp.ph[1].p, cp.ph[1].nb, chain_range<KS>(cp.ph[1]), 2, smem + cp.lds_item);
  };
  if constexpr (AG > 0) {
   if (cp.attn_flag) {
    // Hand-off by completion count (cp.attn_flag): the attention workgroups publish each final
    // output (mq_body `done`) and go straight on -- no grid barrier after the attention; a
    // workgroup with o_proj units waits until all (row group, kv head) outputs are in.
    int n_attn = 0, n_final = 0;
    unsigned long long* done = &bar[kBarAttnDone];
    const bool idle = mq_body<128, AG, KS, true, false, true>(cp.attn, reinterpret_cast<unsigned char*>(smem), nwg,
                                                        (int)blockIdx.x, [&]() {
                                                          setup0(n_attn);
                                                          issue0(pre0);
                                                        }, &n_attn, [&](int k) {
                                                          if ((k == 15 || k == 10) && cp.ts) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                                          if (cp.ts && VWA_TX == 0)
                                                            *gp(cp.ts + blockIdx.x * kTsStride + k) = __builtin_amdgcn_s_memrealtime();
                                                        }, done, &n_final, [&]() {
                                                          // cp.attn_pre: an attention workgroup without o_proj
                                                          // units (osub) streams gate/up's item 0 into A through
                                                          // its attention's merge (fp8 items only: the bf16 item's
                                                          // 64 VGPRs next to the merge's spilled 124 B per lane)
                                                          if constexpr (F8) {
                                                            if (cp.attn_pre && cp.osub && n_attn > 0 && n_attn <= nwg / 2 &&
                                                                (int)blockIdx.x < n_attn) {
                                                              chain_issue_item<E1, KS, WA, false, F8>(cp.ph[1], A, 0);
                                                              apre = true;
                                                            }
                                                          }
                                                        });
    if (!idle) setup0(n_attn);
    stamp();
    // (MULTI: this wave's K/V prefetch DMAs, kv_prefetch, have landed before any LDS reuse)
    if (MULTI && !idle && pf_prev) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_sync();  // the attention's LDS readers are done (idle workgroups: the metadata's)
    if (!idle) {
      pre0 = 0;
      issue0(0);
    }
    if (cp.lds_item && (int)(VWA_TX >> 6) < cp.lds_item_waves) preload1();
    if (chain_range<KS>(cp.ph[0], ob0, on).n_items > 0) {
      if (VWA_TX < 64) {
        const unsigned long long tgt = (unsigned long long)n_final;
        int spins = 0;
        while (true) {
          unsigned long long v;
          asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(done) : "memory");
          if (v >= tgt) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kChainSpinLimit) {
            if (VWA_TX == 0) __hip_atomic_store(gp(&bar[kBarErr]), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      lds_sync();
    }
   } else {
    // idle workgroups (no attention item) issue their o_proj weights at once; the others after
    // their item, at the barrier (one item: their attention registers were live until then)
    int n_attn = 0;
    const bool idle = mq_body<128, AG, KS, true, false, true>(cp.attn, reinterpret_cast<unsigned char*>(smem), nwg,
                                                        (int)blockIdx.x, [&]() {
                                                          setup0(n_attn);
                                                          issue0(pre0);
                                                        }, &n_attn, [&](int k) {
                                                          if ((k == 15 || k == 10) && cp.ts) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                                          if (cp.ts && VWA_TX == 0)
                                                            *gp(cp.ts + blockIdx.x * kTsStride + k) = __builtin_amdgcn_s_memrealtime();
                                                        });
    if (!idle) setup0(n_attn);
    stamp();
    gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
    if (!idle) {
      pre0 = 0;
      issue0(0);
    }
    // LDS item: every workgroup right after its arrival (whose __syncthreads ends the
    // attention's use of LDS).  Measured (tools/chain_probe.py, 1 row): 101.7-102.0 vs
    // 104.2-104.9 us per layer; issued earlier (idle workgroups at once) its bytes delayed the
    // attention's K/V (+1.7 us), issued inside the o_proj phase they delayed its end (+4.5 us)
    if (cp.lds_item && (int)(VWA_TX >> 6) < cp.lds_item_waves) preload1();

    chain_wait(bar, gen, cp.bar_mode);
   }
  } else {
    setup0(0);
    issue0(pre0);
  }
  // cp.xdma: the staging wave issues nothing at the barriers (chain_phase), the others one item
  // (their second follows right at the release)
  const bool stg = cp.xdma && (VWA_TX >> 6) == KS - 1;
  const int preb = cp.xdma ? 0 : cp.pre2;
  // per-barrier override (cp.pre_mask bit i): two items issued ahead of phase i even with xdma
  auto preb_of = [&](int i) { return ((cp.pre_mask >> i) & 1) ? 1 : preb; };
  // (hand-off by count: a workgroup without o_proj units skips the phase -- its X rows may not be
  // complete yet, and nothing of it is used)
  if (!(AG > 0 && cp.attn_flag) || chain_range<KS>(cp.ph[0], ob0, on).n_items > 0)
    // hs: items the staging wave already holds -- 2 (items 0 and 1, or with nx item 0 and phase
    // 1's item 0), but only item 0 when this workgroup ran an attention item (pre0 = 0: its
    // register set A was live in the attention until then).  (A fixed 2 here left the staging
    // wave's item 1 unloaded whenever an attention workgroup also had >= 2 o_proj items -- more
    // attention items than half the grid: several sessions' rows, or a grid cut by
    // VWA_CHAIN_GRID_DIV -- and its MFMAs read stale registers: NaN / wrong o_proj tiles.)
    chain_phase<E0, KS, WA, false, F8, O2>(cp, 0, B, A, smem, nx ? 1 : pre0, nx ? 2 : 1 + (pre0 ? 1 : 0), ob0, on);
  stamp();
  if (SEQ == 0 && tpr) chain_tp_reduce(cp, 0, er + 1, bar, nwg, bar_next);
  gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
  // cp.pre_waves (> 0): only waves below it issue the next phase's items at the barrier; the others
  // issue theirs after the release, behind the X pieces (chain_phase has0 = false)
  const int wv = (int)(VWA_TX >> 6);
  const bool prew = (cp.pre_waves == 0 || wv < cp.pre_waves) && !(cp.poll_free && wv == 0);
  const bool nx1 = nx || apre;  // phase 1's item 0 already in A (o_proj's free set, or the attention window)
  if (!stg) {
    if (nx1) chain_issue_item<E1, KS, WA, false, F8>(cp.ph[1], B, 1);  // phase 1's item 0 is already in A
    else if (prew) chain_issue_first<E1, KS, WA, false, F8>(cp.ph[1], A, B, preb_of(1));
  }
  chain_wait(bar, gen, cp.bar_mode);
  // every attention output was counted and every waiter released before this barrier: reset the
  // count for the next launch (ordered before it by the kernel boundary)
  if (AG > 0 && cp.attn_flag && blockIdx.x == 0 && VWA_TX == 0)
    __hip_atomic_store(gp(&bar[kBarAttnDone]), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  stamp();
  chain_phase<E1, KS, WA, false, F8>(cp, 1, A, B, smem, nx1 ? 1 : preb_of(1), nx1 ? 1 : 0, 0, 0, nx1 || prew);
  stamp();
  if constexpr (NPH >= 3) {
    gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
    if ((!stg && prew) || XG2) chain_issue_first<E2, KS, WA, XG2, F8, D2>(cp.ph[2], A, B, preb_of(2));  // (XG2: no staging wave)
    // phase 2's LDS item (down projection): its item 2 streams through the barrier window too
    // (phase 1's LDS use ended at the arrival's __syncthreads; the region lies above phase 2's
    // X rows and scratch, which the staging wave fills after the release)
    if (cp.lds_item2 && wv < cp.lds_item2_waves && !(cp.poll_free && wv == 0))
      chain_preload<PhaseShape<E2, KS, false, F8>::NT, PhaseShape<E2, KS, false, F8>::U, WA, F8>(
          cp.ph[2].p, cp.ph[2].nb, chain_range<KS>(cp.ph[2]), 2, smem + cp.lds_item2);
    chain_wait(bar, gen, cp.bar_mode);
    stamp();
    chain_phase<E2, KS, WA, XG2, F8, D2>(cp, 2, A, B, smem, preb_of(2), 0, 0, 0, prew || XG2);
    stamp();
    if (SEQ == 0 && tpr) {
      chain_tp_reduce(cp, 1, er + 2, bar, nwg, bar_next);
      if (blockIdx.x == 0 && VWA_TX == 0)
        __hip_atomic_store(gp(cp.tp.epoch), er + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (NPH >= 4) {
   if (!MULTI || cp.n >= 4) {  // (MULTI: the model's last layer has no next QKV phase)
    gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
    if (!stg && prew) chain_issue_first<E3, KS, WA, false, F8>(cp.ph[3], A, B, preb_of(3));
    chain_wait(bar, gen, cp.bar_mode);
    stamp();
    chain_phase<E3, KS, WA, false, F8>(cp, 3, A, B, smem, preb_of(3), 0, 0, 0, prew);
    stamp();
   }
  }
  if constexpr (MULTI) {
    if (li + 1 < n_layers) {
      // layer li -> li + 1: an attention workgroup of layer li + 1 reads Q / the newest K/V only
      // once the QKV tiles of its kv group are stored (qsig: per-group counters; else a barrier)
      if (qsig) qkv_signal<KS>(cp.ph[3], bar);
      else gen = chain_arrive(bar, nwg, cp.bar_mode, bar_next);
      const DecodeAttnParams& na = cpp[li + 1].attn;
      int st = 3, ev = 0;
      if (cpp[li + 1].attn_flag && na.plan_mode == 2) {
        // this workgroup's step-plan entry (state 0 idle / 2 empty chunk: no Q, K or V read)
        const __amdgpu_buffer_rsrc_t r_pl =
            __builtin_amdgcn_make_buffer_rsrc(na.plan, (short)0, ((int)blockIdx.x + 1) * 64, 0x00020000);
        ev = (int)__builtin_amdgcn_raw_buffer_load_b32(r_pl, ((int)blockIdx.x * 16 + (VWA_TX & 15)) * 4, 0, 16);
        st = __builtin_amdgcn_readlane(ev, 10) == na.rows ? __builtin_amdgcn_readlane(ev, 2) : 3;
      }
      if (st != 0 && st != 2) {  // (idle / empty-chunk workgroups go straight on: no wait at all)
        if (st == 1 && cp.kv_prefetch) {
          kv_prefetch(na, ev, reinterpret_cast<unsigned char*>(smem));
          pf_next = true;
        }
        if (!qsig) {
          chain_wait(bar, gen, cp.bar_mode);
        } else {
          const int kvh = __builtin_amdgcn_readlane(ev, 3);
          const unsigned long long add = (unsigned long long)qkv_tiles_per_group(cp.ph[3].p) * (unsigned long long)(li + 1);
          if (st == 1) qkv_wait(bar, qkv_base, add, kvh, kvh + 1);
          else qkv_wait(bar, qkv_base, add, 0, cp.ph[3].p.n_kv_heads);  // (no plan: every group)
        }
      }
    }
  }
  }  // layers
}

}  // namespace

// Host side: fill nt / nb of every phase and return the dynamic LDS bytes the chain needs, or
// -10 when a phase does not fit (X rows must fit in LDS next to the reduction scratch, M <= 4,
// K % 128 == 0, bf16 weights).  The filled descriptor is then copied to device memory once and
// launched with vwa_chain_launch (graph-capturable: no allocation, no copy at launch).
extern "C" int vwa_chain_prepare(ChainParams* cp, int grid) {
  // (8 waves: a 16-wave form -- 1024-thread workgroups, 8-load items -- has a 128-VGPR budget;
  // compiled it spilled 200 B/lane and measured 160 vs 97 us per layer tail)
  constexpr int KS = 8;
  constexpr int R = ChainShape<KS>::R;
  if (cp->n < 2 || cp->n > kChainMaxPhases || grid < 1) return -10;
  static const int kSeq[3][kChainMaxPhases] = {{EPI_RESID, EPI_SWIGLU, EPI_RESID, EPI_QKV},
                                               {EPI_RESID, EPI_GELU, EPI_RESID, EPI_QKV},
                                               {EPI_RESID, EPI_STORE, -1, -1}};
  if (cp->seq < 0 || cp->seq > 2 || (cp->seq == 2 ? cp->n != 2 : cp->n < (cp->seq == 0 ? 2 : 3))) return -10;
  if (cp->seq == 0 && cp->n == 2) return -10;  // (round 4's o_proj -> gate/up chain: removed in round 5)
  size_t lds = 0;
  for (int i = 0; i < cp->n; ++i) {
    ChainPhase& ph = cp->ph[i];
    const SkinnyParams& p = ph.p;
    if (ph.epi != kSeq[cp->seq][i]) return -10;
    ph.nt = (ph.epi == EPI_SWIGLU) ? 2 : 1;
    // o_nt2: the chained o_proj in 32-column tiles -- one epilogue (cross-wave reduction, residual,
    // store) per workgroup instead of two at one row (Llama tail with the attention phase, bf16)
    if (i == 0 && cp->o_nt2) {
      if (cp->seq == 0 && cp->attn_g > 0 && p.w_scale == nullptr && p.N % 32 == 0) ph.nt = 2;
      else cp->o_nt2 = 0;
    }
    // 5..16 rows: only without the attention phase (its row tables hold <= 4 rows), Llama tail; a
    // phase whose X rows do not fit LDS next to the scratch streams X with the weights (xg: the
    // down projection, residual epilogue, pre-tiled weights)
    // fp8 (W8A16 chain): only the fp8 tiled layout, every phase fp8 (one kernel instantiation),
    // <= 4 rows (no X streaming with the weights)
    const bool f8 = p.w_scale != nullptr;
    if (f8 && (!p.w_tiled || cp->seq != 0)) return -10;
    if (i > 0 && f8 != (cp->ph[0].p.w_scale != nullptr)) return -10;
    const int max_rows = (cp->seq == 0 && cp->attn_g == 0 && !f8) ? 16 : 4;
    if (p.M < 1 || p.M > max_rows || p.K % 128 != 0 || p.N % (16 * ph.nt) != 0) return -10;
    const size_t xrows = ((size_t)p.M * (p.K + 8) * 2 + 15) & ~(size_t)15;
    ph.xg = 0;
    if (xrows + (size_t)(KS * ph.nt * 4 * 64 + 48) * sizeof(float) > 160 * 1024) {
      if (!(cp->seq == 0 && i == 2 && ph.epi == EPI_RESID && p.w_tiled && p.fuse_rms == 0)) return -10;
      ph.xg = 1;
    }
    // (X streaming has only the attention-less instantiation: a 70B down projection at 3-4 rows
    // -- 28672-wide X rows -- is chained with the decode attention as its own launch instead)
    if (ph.xg && (f8 || cp->attn_g > 0)) return -10;
    if (ph.xg && cp->d_nt2 && p.N % 32 == 0) ph.nt = 2;
    if (i == 2 && !(ph.xg && ph.nt == 2)) cp->d_nt2 = 0;  // (d_nt2 does not apply: the plain instantiation)
    const size_t scratch = (size_t)(KS * ph.nt * 4 * 64 + 48) * sizeof(float);
    const int U = ph.xg ? (ph.nt == 2 ? 1 : 2) : (f8 ? ChainShape<KS, true>::R : R) / 4 / ph.nt * (f8 ? 2 : 1);
    if ((size_t)p.N * p.K * 2 >= 0x7FFFFFF0ull || (size_t)p.M * p.ldx * 2 >= 0x7FFFFFF0ull) return -10;
    const int G = p.K / 128;
    const int per_wave = (G + KS - 1) / KS;
    ph.nb = (per_wave + U - 1) / U;
    const long long ntiles = p.N / (16 * ph.nt);
    const long long units = ntiles * ph.nb;
    // a tile may straddle at most two workgroup ranges (two partial slots per tile): every
    // non-empty range (floor or ceil of units / grid units, >= 1) must hold >= nb - 1 units
    const long long min_range = units / grid > 0 ? units / grid : 1;
    // (equal ranges that divide a tile's units also split each tile over exactly two workgroups)
    const bool aligned = units % grid == 0 && ph.nb % min_range == 0 && ph.nb / min_range <= 2;
    if (ph.nb > 1 && min_range < ph.nb - 1 && !aligned) return -10;
    if (ntiles > cp->max_tiles || (size_t)ntiles * 2 * p.M * 16 * ph.nt > (size_t)cp->part_floats) return -10;
    const size_t need = (ph.xg ? 0 : xrows) + scratch;  // X rows + scales, means, flag
    if (need > lds) lds = need;
  }
  if (lds > 160 * 1024) return -10;
  // LDS item (Llama tail with the attention phase, pre-tiled weights): the region above phases
  // 0 and 1's LDS (1 KB aligned) up to 160 KB holds item 2 of as many waves as fit (8 at one
  // row, 7 at 2-3, 6 at 4 rows) -- phase 2 may overlap it (the item is consumed at the start of
  // phase 1); the attention's own LDS is free again before the preload
  cp->lds_item = 0;
  cp->lds_item_waves = 0;
  if (cp->lds_item_req == 1 && cp->seq == 0 && cp->attn_g > 0 && cp->n >= 2 && cp->ph[1].p.w_tiled) {
    size_t start = 0;
    for (int i = 0; i < 2; ++i) {
      const ChainPhase& ph = cp->ph[i];
      const size_t x = ((size_t)ph.p.M * (ph.p.K + 8) * 2 + 15) & ~(size_t)15;
      const size_t need = x + (size_t)(KS * ph.nt * 4 * 64 + 48) * sizeof(float);
      if (need > start) start = need;
    }
    start = (start + 1023) & ~(size_t)1023;
    const int nw = start < 160 * 1024 ? (int)((160 * 1024 - start) / 16384) : 0;
    if (nw >= 4) {
      cp->lds_item = (int)start;
      cp->lds_item_waves = nw < KS ? nw : KS;
      lds = 160 * 1024;
    }
  }
  // LDS-DMA staging moves whole 1 KB pieces of a row (512 bf16): only for K % 512 == 0 phases
  for (int i = 0; i < cp->n; ++i)
    if (cp->ph[i].p.K % 512 != 0) cp->xdma = 0;
  // phase 2's LDS item (Llama tail): the region above phase 2's own X rows + scratch holds item 2
  // of as many waves as fit (7 at one row; the staging wave never takes one: its vmcnt queue
  // must hold nothing but the X pieces at the release)
  cp->lds_item2 = 0;
  cp->lds_item2_waves = 0;
  if (cp->lds_item2_req == 1 && cp->seq == 0 && cp->n >= 3 && cp->ph[2].p.w_tiled && !cp->ph[2].xg) {
    const ChainPhase& ph = cp->ph[2];
    const size_t x = ((size_t)ph.p.M * (ph.p.K + 8) * 2 + 15) & ~(size_t)15;
    const size_t start = (x + (size_t)(KS * ph.nt * 4 * 64 + 48) * sizeof(float) + 1023) & ~(size_t)1023;
    const int nw = start < 160 * 1024 ? (int)((160 * 1024 - start) / 16384) : 0;
    const int cap = cp->xdma ? KS - 1 : KS;
    if (nw >= 2) {
      cp->lds_item2 = (int)start;
      cp->lds_item2_waves = nw < cap ? nw : cap;
      lds = 160 * 1024;
    }
  }
  return (int)lds;
}

extern "C" int vwa_chain_launch(const ChainParams* d_cp, int seq, int n_phases, int attn_g, int lds, int grid,
                                hipStream_t st, int xg2, int f8, int o2, int n_layers) {
  if (attn_g) lds = lds > (int)MqLds<128, 8>::bytes ? lds : (int)MqLds<128, 8>::bytes;
  if (n_layers > 1) {  // one launch over n_layers consecutive Llama tails (chain_kernel MULTI)
    if (seq != 0 || n_phases != 4 || xg2 || (attn_g != 4 && attn_g != 8) || (!f8 && !o2) || (f8 && o2)) return -10;
#define VWA_CHAIN_LAUNCH_MULTI(G, F8_, O2_) \
  hipLaunchKernelGGL((chain_kernel<8, 0, 4, G, 0, false, F8_, O2_, false, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, n_layers)
    if (attn_g == 4) {
      if (f8) VWA_CHAIN_LAUNCH_MULTI(4, true, false); else VWA_CHAIN_LAUNCH_MULTI(4, false, true);
    } else {
      if (f8) VWA_CHAIN_LAUNCH_MULTI(8, true, false); else VWA_CHAIN_LAUNCH_MULTI(8, false, true);
    }
#undef VWA_CHAIN_LAUNCH_MULTI
    return (int)hipGetLastError();
  }
#ifndef VWA_ONLY_MULTI  // (register-budget experiments: compile the multi-layer instantiations alone)
  if (o2) {  // o_proj in 32-column tiles (ChainParams::o_nt2): Llama tail with the attention phase, bf16
    if (seq != 0 || f8 || xg2 || (n_phases != 3 && n_phases != 4)) return -10;
    const bool q = n_phases == 4;
#define VWA_CHAIN_LAUNCH_O2(N, G) \
  hipLaunchKernelGGL((chain_kernel<8, 0, N, G, 0, false, false, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1)
    switch (attn_g) {
      case 4: if (q) VWA_CHAIN_LAUNCH_O2(4, 4); else VWA_CHAIN_LAUNCH_O2(3, 4); break;
      case 8: if (q) VWA_CHAIN_LAUNCH_O2(4, 8); else VWA_CHAIN_LAUNCH_O2(3, 8); break;
      default: return -10;
    }
#undef VWA_CHAIN_LAUNCH_O2
    return (int)hipGetLastError();
  }
  if (xg2) {  // Llama tail of 5..16 rows: down projection with X from L2, no attention phase
    if (seq != 0 || attn_g != 0 || f8 || (n_phases != 3 && n_phases != 4)) return -10;
    if (xg2 == 2) {  // (d_nt2: 32-column down tiles)
      if (n_phases == 4) hipLaunchKernelGGL((chain_kernel<8, 0, 4, 0, 0, true, false, false, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1);
      else hipLaunchKernelGGL((chain_kernel<8, 0, 3, 0, 0, true, false, false, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1);
    } else if (n_phases == 4) {
      hipLaunchKernelGGL((chain_kernel<8, 0, 4, 0, 0, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1);
    } else {
      hipLaunchKernelGGL((chain_kernel<8, 0, 3, 0, 0, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1);
    }
    return (int)hipGetLastError();
  }
#define VWA_CHAIN_LAUNCH(S, N, G) \
  hipLaunchKernelGGL((chain_kernel<8, S, N, G, 0>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1)
#define VWA_CHAIN_LAUNCH_F8(N, G) \
  hipLaunchKernelGGL((chain_kernel<8, 0, N, G, 0, false, true>), dim3(grid), dim3(8 * 64), lds, st, d_cp, 1)
  if (f8) {  // fp8 tiled weights, W8A16 (Llama tail only)
    if (seq != 0 || (n_phases != 3 && n_phases != 4)) return -10;
    const bool q = n_phases == 4;
    switch (attn_g) {
      case 0: if (q) VWA_CHAIN_LAUNCH_F8(4, 0); else VWA_CHAIN_LAUNCH_F8(3, 0); break;
      case 4: if (q) VWA_CHAIN_LAUNCH_F8(4, 4); else VWA_CHAIN_LAUNCH_F8(3, 4); break;
      case 8: if (q) VWA_CHAIN_LAUNCH_F8(4, 8); else VWA_CHAIN_LAUNCH_F8(3, 8); break;
      default: return -10;
    }
    return (int)hipGetLastError();
  }
#undef VWA_CHAIN_LAUNCH_F8
  if (seq == 0) {
    if (n_phases != 3 && n_phases != 4) return -10;
    const bool q = n_phases == 4;
    switch (attn_g) {
      case 0: if (q) VWA_CHAIN_LAUNCH(0, 4, 0); else VWA_CHAIN_LAUNCH(0, 3, 0); break;
      case 4: if (q) VWA_CHAIN_LAUNCH(0, 4, 4); else VWA_CHAIN_LAUNCH(0, 3, 4); break;
      case 8: if (q) VWA_CHAIN_LAUNCH(0, 4, 8); else VWA_CHAIN_LAUNCH(0, 3, 8); break;
      default: return -10;
    }
  } else if (seq == 1 && attn_g == 0) {
    if (n_phases == 4) VWA_CHAIN_LAUNCH(1, 4, 0);
    else if (n_phases == 3) VWA_CHAIN_LAUNCH(1, 3, 0);
    else return -10;
  } else if (seq == 2 && attn_g == 0 && n_phases == 2) {
    VWA_CHAIN_LAUNCH(2, 2, 0);
  } else {
    return -10;
  }
#undef VWA_CHAIN_LAUNCH
  return (int)hipGetLastError();
#else
  return -10;
#endif
}

// (round 4's 32-column tiles for the plain epilogues measured slower at
// 8 / 16 rows, profiles/r4_skinny_nt2_rows.jsonl, and were removed in round 5)

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
extern "C" void vwa_skinny_set_x_skew(int skew) { g_x_skew = skew == 0 ? 0 : 32; }

extern "C" int vwa_skinny_stream(int epi, const SkinnyParams* p, int grid_cap, int ks, hipStream_t st) {
  if (p->M < 1 || p->M > 16 || p->K % 128 != 0) return -10;
  if ((size_t)p->N * p->K * (p->w_scale ? 1 : 2) >= 0x7FFFFFF0ull) return -10;
#ifdef VWA_ONLY_MULTI
  const int r = -10;
#else
  const int r = (ks == 4) ? dispatch_ks<4>(epi, *p, grid_cap, st) : dispatch_ks<8>(epi, *p, grid_cap, st);
#endif
  if (r) return r;
  return (int)hipGetLastError();
}
