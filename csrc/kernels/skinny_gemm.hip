// Skinny (decode-shaped) GEMM on MFMA with fused epilogues.
//
//   Y[M, N] = epilogue( rms_scale[m] * (X[M, K] @ W[N, K]^T) + bias )
//
// M <= 64 (decode batch rows, or forced tokens from jump-forward decoding), N, K large.
// This is the op that decides decode latency: every weight byte of the LLM is streamed
// through it once per token, so it is written as an HBM stream that feeds MFMA:
//
//  * one workgroup owns a 16*NT-column tile of W and ALL of K; its KS waves split K
//    (so a 4096x4096 projection still launches 256 WGs x 8 waves = 2048 waves);
//  * lane (n = l&15, g = l>>4) streams 64 contiguous bytes of weight row n per 128-wide
//    k-group (4 x dwordx4) and the matching X bytes; the k order inside the group is
//    permuted identically for A and B, which MFMA's k-sum does not care about;
//  * loads are issued in static batches of 4 k-groups before their MFMAs (16 KB/wave in flight);
//  * partial accumulators are reduced across waves through LDS, then a fused epilogue:
//      STORE   : y = acc*s + b                        (bf16 or f32 out, e.g. LM head logits)
//      RESID   : y = r + acc*s + b                    (o_proj / down_proj / fc2 residual add)
//      SWIGLU  : h = silu(g) * u, gate/up rows interleaved per 16-row tile (NT = 2)
//      GELU    : y = gelu(acc*s + b)                  (Whisper / GPT-2 fc1)
//      QKV     : rotary embedding (rotate-half pairs live in cols c and c^8 of one tile,
//                 thanks to a load-time row permutation) + scatter of K/V into the paged
//                 KV cache + Q write.  Replaces reference remote-LLM compute
//                 (apps/brain/src/llm.ts:22-27).
//  * fused RMSNorm: the norm's gamma is folded into W's columns at load time and the
//    per-row 1/rms is computed from the X bytes the waves stream anyway (sum of squares
//    reduced with the accumulators) -- no separate norm kernel, no extra HBM traffic.
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

enum Epi { EPI_STORE = 0, EPI_RESID = 1, EPI_SWIGLU = 2, EPI_GELU = 3, EPI_QKV = 4 };

template <int NT, int MT>
struct Frags {
  uint4 w[NT][4];
  uint4 x[MT][4];
};

template <int NT, int MT>
VWA_DEVICE void load_group(Frags<NT, MT>& f, const SkinnyParams& p, int n0, int kg, int lane) {
  const int nl = lane & 15, g = lane >> 4;
  const int k0 = kg * 128 + 32 * g;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const uint4* src = reinterpret_cast<const uint4*>(p.W + (size_t)(n0 + nt * 16 + nl) * p.K + k0);
#pragma unroll
    for (int s = 0; s < 4; ++s) f.w[nt][s] = load_nt(src + s);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int m = mt * 16 + nl;
    if (m < p.M) {
      const uint4* src = reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + k0);
#pragma unroll
      for (int s = 0; s < 4; ++s) f.x[mt][s] = src[s];
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) f.x[mt][s] = make_uint4(0, 0, 0, 0);
    }
  }
}

VWA_DEVICE float sumsq8(const uint4& v) {
  float f[8];
  unpack8(v, f);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += f[j] * f[j];
  return s;
}

VWA_DEVICE float sum8(const uint4& v) {
  float f[8];
  unpack8(v, f);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += f[j];
  return s;
}

template <int EPI, int NT, int MT, int KS>
__global__ __launch_bounds__(KS * 64) void skinny_gemm_kernel(SkinnyParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int tile = blockIdx.x;
  const int n0 = tile * 16 * NT;

  const int G = p.K / 128;
  const int gb = (G * w) / KS, ge = (G * (w + 1)) / KS;

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // row statistics of the streamed X: sum of squares (fused RMSNorm, fuse_rms 1) and, for a
  // LayerNorm folded into W (fuse_rms 2, y = rstd * (acc - mean * ln_c[n]) + bias), the sum
  const bool ln = p.fuse_rms == 2;
  float ssq[MT], ssum[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ssq[mt] = ssum[mt] = 0.f;

  // Main loop: batches of U k-groups whose loads are ALL issued before the first MFMA that
  // consumes them (static indices, no data-dependent load predicates -> hipcc emits counted
  // vmcnt waits; 16 KB+ per wave in flight).  Different waves/WGs are at different phases, so
  // the CU always has loads in flight while some waves run their MFMAs.
  constexpr int U = (MT >= 4) ? 1 : (MT == 2 ? 2 : 4);
  int kg = gb;
  for (; kg + U <= ge; kg += U) {
    Frags<NT, MT> f[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_group<NT, MT>(f[u], p, n0, kg + u, lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 a = as_bf16x8(f[u].x[mt][s]);
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16(a, as_bf16x8(f[u].w[nt][s]), acc[mt][nt]);
        }
      }
      if (p.fuse_rms) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            ssq[mt] += sumsq8(f[u].x[mt][s]);
            if (ln) ssum[mt] += sum8(f[u].x[mt][s]);
          }
      }
    }
  }
  for (; kg < ge; ++kg) {
    Frags<NT, MT> f;
    load_group<NT, MT>(f, p, n0, kg, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bf16x8 a = as_bf16x8(f.x[mt][s]);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma16(a, as_bf16x8(f.w[nt][s]), acc[mt][nt]);
      }
    }
    if (p.fuse_rms) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          ssq[mt] += sumsq8(f.x[mt][s]);
          if (ln) ssum[mt] += sum8(f.x[mt][s]);
        }
    }
  }

  // ---- cross-wave reduction through LDS: red[w][mt][nt][i][lane]
  float* red = smem;
  float* red_ssq = smem + KS * MT * NT * 4 * 64;  // [w][mt*16 + m]
  float* red_sum = red_ssq + KS * MT * 16;          // [w][mt*16 + m] (folded LayerNorm)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(((w * MT + mt) * NT + nt) * 4 + i) * 64 + lane] = acc[mt][nt][i];
  if (p.fuse_rms) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float v = ssq[mt];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) red_ssq[w * MT * 16 + mt * 16 + lane] = v;
      if (ln) {
        float t = ssum[mt];
        t += __shfl_xor(t, 16, 64);
        t += __shfl_xor(t, 32, 64);
        if (lane < 16) red_sum[w * MT * 16 + mt * 16 + lane] = t;
      }
    }
  }
  __syncthreads();

  auto red_at = [&](int m, int nn) -> float {
    const int mt = m >> 4, mi = m & 15, nt = nn >> 4, nl = nn & 15;
    const int ln = nl + 16 * (mi >> 2), i = mi & 3;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) s += red[(((ww * MT + mt) * NT + nt) * 4 + i) * 64 + ln];
    return s;
  };
  auto row_mean = [&](int m) -> float {
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) s += red_sum[ww * MT * 16 + m];
    return s / (float)p.K;
  };
  auto row_scale = [&](int m) -> float {
    if (!p.fuse_rms) return 1.f;
    float s = 0.f;
#pragma unroll
    for (int ww = 0; ww < KS; ++ww) s += red_ssq[ww * MT * 16 + m];
    if (ln) {
      const float mu = row_mean(m);
      return rsqrtf(fmaxf(s / (float)p.K - mu * mu, 0.f) + p.eps);
    }
    return rsqrtf(s / (float)p.K + p.eps);
  };
  // accumulator of (row m, column n) with the folded LayerNorm's mean term removed
  auto lin = [&](int m, int nn, int n) -> float {
    const float v = red_at(m, nn);
    return ln ? v - row_mean(m) * p.ln_c[n] : v;
  };

  const int Mrows = p.M < MT * 16 ? p.M : MT * 16;
  if constexpr (EPI == EPI_SWIGLU) {
    // tile = [16 gate rows | 16 up rows] for output columns tile*16 .. tile*16+15
    for (int o = threadIdx.x; o < Mrows * 16; o += KS * 64) {
      const int m = o >> 4, nl = o & 15;
      const float sc = row_scale(m);
      float gv = red_at(m, nl) * sc, uv = red_at(m, 16 + nl) * sc;
      if (p.bias) {
        gv += bf2f(p.bias[n0 + nl]);
        uv += bf2f(p.bias[n0 + 16 + nl]);
      }
      u16* y = reinterpret_cast<u16*>(p.Y);
      y[(size_t)m * p.ldy + tile * 16 + nl] = f2bf(silu(gv) * uv);
    }
  } else if constexpr (EPI == EPI_QKV) {
    const int hd = p.head_dim, half = hd >> 1;
    const int head = n0 / hd;
    const int t = (n0 % hd) >> 4;
    for (int o = threadIdx.x; o < Mrows * 16; o += KS * 64) {
      const int m = o >> 4, nl = o & 15;
      const float sc = row_scale(m);
      float v = lin(m, nl, n0 + nl) * sc;
      float pv = lin(m, nl ^ 8, n0 + (nl ^ 8)) * sc;
      if (p.bias) {
        v += bf2f(p.bias[n0 + nl]);
        pv += bf2f(p.bias[n0 + (nl ^ 8)]);
      }
      const int d = (nl < 8) ? (8 * t + nl) : (half + 8 * t + nl - 8);
      const bool is_v = head >= p.n_q_heads + p.n_kv_heads;
      if (p.use_rope && !is_v) {
        const int pos = p.positions[m];
        const int di = (nl < 8) ? (8 * t + nl) : (8 * t + nl - 8);
        const float c = p.rope[((size_t)pos * half + di) * 2 + 0];
        const float sn = p.rope[((size_t)pos * half + di) * 2 + 1];
        v = (nl < 8) ? (v * c - pv * sn) : (v * c + pv * sn);
      }
      const u16 out = f2bf(v);
      if (head < p.n_q_heads) {
        p.q_out[(size_t)m * p.ldq + head * hd + d] = out;
      } else {
        const int64_t slot = p.slots[m];
        if (slot >= 0) {
          const int64_t blk = slot / p.block_size, off = slot % p.block_size;
          const int kvh = is_v ? head - p.n_q_heads - p.n_kv_heads : head - p.n_q_heads;
          const int64_t idx = blk * p.cache_stride_block + kvh * p.cache_stride_head + off * p.cache_stride_tok + d;
          (is_v ? p.v_cache : p.k_cache)[idx] = out;
        }
      }
    }
  } else {
    for (int o = threadIdx.x; o < Mrows * 16 * NT; o += KS * 64) {
      const int m = o / (16 * NT), nn = o % (16 * NT);
      const int n = n0 + nn;
      float v = lin(m, nn, n) * row_scale(m);
      if (p.bias) v += bf2f(p.bias[n]);
      if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
      if constexpr (EPI == EPI_RESID) v += bf2f(p.R[(size_t)m * p.ldr + n]);
      if (p.y_f32) reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
      else reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + n] = f2bf(v);
    }
  }
}

template <int EPI, int NT, int MT, int KS>
void launch_t(const SkinnyParams& p, hipStream_t st) {
  const int ntiles = p.N / (16 * NT);
  const size_t lds = (size_t)(KS * MT * NT * 4 * 64 + 2 * KS * MT * 16) * sizeof(float);
  hipLaunchKernelGGL((skinny_gemm_kernel<EPI, NT, MT, KS>), dim3(ntiles), dim3(KS * 64), lds, st, p);
}

template <int EPI, int NT, int MT>
void launch_ks(const SkinnyParams& p, hipStream_t st) {
  if (p.K / 128 >= 8) launch_t<EPI, NT, MT, 8>(p, st);
  else launch_t<EPI, NT, MT, 4>(p, st);
}

template <int EPI, int NT>
void launch_mt(const SkinnyParams& p, hipStream_t st) {
  if (p.M <= 16) launch_ks<EPI, NT, 1>(p, st);
  else if (p.M <= 32) launch_ks<EPI, NT, 2>(p, st);
  else launch_ks<EPI, NT, 4>(p, st);
}

}  // namespace

extern "C" int vwa_skinny_gemm(int epi, const SkinnyParams* p, hipStream_t st) {
  if (p->M < 1 || p->M > 64 || p->K % 128 != 0) return -1;
  if (p->fuse_rms == 2 && (epi == EPI_SWIGLU || p->ln_c == nullptr)) return -3;
  switch (epi) {
    case EPI_STORE: if (p->N % 16) return -2; launch_mt<EPI_STORE, 1>(*p, st); break;
    case EPI_RESID: if (p->N % 16) return -2; launch_mt<EPI_RESID, 1>(*p, st); break;
    case EPI_GELU: if (p->N % 16) return -2; launch_mt<EPI_GELU, 1>(*p, st); break;
    case EPI_SWIGLU: if (p->N % 32) return -2; launch_mt<EPI_SWIGLU, 2>(*p, st); break;
    case EPI_QKV: if (p->N % 16 || p->head_dim % 16) return -2; launch_mt<EPI_QKV, 1>(*p, st); break;
    default: return -3;
  }
  return (int)hipGetLastError();
}
