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

template <int EPI, int NT, int KS>
__global__ __launch_bounds__(KS * 64) void skinny_stream_kernel(SkinnyParams p, int nb, int xstride) {
  constexpr int U = 4 / NT;  // k-groups (128 wide) per item
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int M = p.M, K = p.K, N = p.N;
  u16* xs = reinterpret_cast<u16*>(smem);
  const int xbytes = ((M * xstride * 2) + 15) & ~15;
  float* red = reinterpret_cast<float*>(smem + xbytes);  // [KS][NT][4][64]
  float* rs = red + KS * NT * 4 * 64;                     // [16]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nl = lane & 15, g = lane >> 4;

  // ---- stage X rows into LDS
  const int k8 = K / 8;
  for (int c = threadIdx.x; c < M * k8; c += KS * 64) {
    const int m = c / k8, kk = c % k8;
    *reinterpret_cast<uint4*>(xs + m * xstride + kk * 8) = *reinterpret_cast<const uint4*>(p.X + (size_t)m * p.ldx + kk * 8);
  }
  __syncthreads();
  for (int m = w; m < 16; m += KS) {
    float sc = 1.f;
    if (p.fuse_rms && m < M) {
      float s = 0.f;
      for (int kk = lane; kk < k8; kk += 64) {
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(xs + m * xstride + kk * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += f[j] * f[j];
      }
      s = wave_sum(s);
      sc = rsqrtf(s / (float)K + p.eps);
    }
    if (lane == 0) rs[m] = sc;
  }
  __syncthreads();

  const int G = K / 128;
  const int gb = (G * w) / KS, ge = (G * (w + 1)) / KS;
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<u16*>(p.W), (short)0, (int)((size_t)N * K * 2), 0x00020000);
  const int ntiles = N / (16 * NT);
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int n_items = my_tiles * nb;

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

  auto compute_item = [&](const uint4 (&wr)[NT][U][4], int it) {
    const int b = it % nb;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kg = gb + b * U + u;
      if (kg >= ge) break;  // wave-uniform
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        uint4 a = make_uint4(0, 0, 0, 0);
        if (nl < M) a = *reinterpret_cast<const uint4*>(xs + nl * xstride + kg * 128 + 32 * g + 8 * s);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[nt] = mfma16(as_bf16x8(a), as_bf16x8(wr[nt][u][s]), acc[nt]);
      }
    }
  };

  auto finish_tile = [&](int it) {
    const int tile = blockIdx.x + (it / nb) * gridDim.x;
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
    if constexpr (EPI == EPI_SWIGLU) {
      for (int o = threadIdx.x; o < M * 16; o += KS * 64) {
        const int m = o >> 4, q = o & 15;
        const float sc = rs[m];
        float gv = red_at(m, q) * sc, uv = red_at(m, 16 + q) * sc;
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
        const float sc = rs[m];
        float v = red_at(m, q) * sc, pv = red_at(m, q ^ 8) * sc;
        if (p.bias) {
          v += bf2f(p.bias[n0 + q]);
          pv += bf2f(p.bias[n0 + (q ^ 8)]);
        }
        const int d = (q < 8) ? (8 * t + q) : (half + 8 * t + q - 8);
        if (p.use_rope && !is_v) {
          const int pos = p.positions[m];
          const int di = (q < 8) ? (8 * t + q) : (8 * t + q - 8);
          const float c = p.rope[((size_t)pos * half + di) * 2 + 0];
          const float sn = p.rope[((size_t)pos * half + di) * 2 + 1];
          v = (q < 8) ? (v * c - pv * sn) : (v * c + pv * sn);
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
      for (int o = threadIdx.x; o < M * 16 * NT; o += KS * 64) {
        const int m = o / (16 * NT), nn = o % (16 * NT);
        const int n = n0 + nn;
        float v = red_at(m, nn) * rs[m];
        if (p.bias) v += bf2f(p.bias[n]);
        if constexpr (EPI == EPI_GELU) v = gelu_erf(v);
        if constexpr (EPI == EPI_RESID) v += bf2f(p.R[(size_t)m * p.ldr + n]);
        if (p.y_f32) reinterpret_cast<float*>(p.Y)[(size_t)m * p.ldy + n] = v;
        else reinterpret_cast<u16*>(p.Y)[(size_t)m * p.ldy + n] = f2bf(v);
      }
    }
    __syncthreads();
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  uint4 A[NT][U][4], B[NT][U][4];
  load_item(A, 0);
  for (int it = 0; it < n_items; it += 2) {
    load_item(B, it + 1);
    compute_item(A, it);
    if (it % nb == nb - 1) finish_tile(it);
    if (it + 1 >= n_items) break;
    load_item(A, it + 2);
    compute_item(B, it + 1);
    if ((it + 1) % nb == nb - 1) finish_tile(it + 1);
  }
}

template <int EPI, int NT, int KS>
int launch(const SkinnyParams& p, hipStream_t st, int grid_cap) {
  constexpr int U = 4 / NT;
  const int G = p.K / 128;
  const int per_wave = (G + KS - 1) / KS;
  const int nb = (per_wave + U - 1) / U;
  const int xstride = p.K + 8;
  const size_t xbytes = ((size_t)p.M * xstride * 2 + 15) & ~(size_t)15;
  const size_t lds = xbytes + (size_t)(KS * NT * 4 * 64 + 16) * sizeof(float);
  if (lds > 160 * 1024) return -10;
  const int ntiles = p.N / (16 * NT);
  const int grid = ntiles < grid_cap ? ntiles : grid_cap;
  hipLaunchKernelGGL((skinny_stream_kernel<EPI, NT, KS>), dim3(grid), dim3(KS * 64), lds, st, p, nb, xstride);
  return 0;
}

}  // namespace

// Returns -10 when this shape does not fit the streaming kernel (caller falls back).
template <int KS>
int dispatch_ks(int epi, const SkinnyParams& p, int grid_cap, hipStream_t st) {
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
  if ((size_t)p->N * p->K * 2 >= 0x7FFFFFF0ull) return -10;
  const int r = (ks == 4) ? dispatch_ks<4>(epi, *p, grid_cap, st) : dispatch_ks<8>(epi, *p, grid_cap, st);
  if (r) return r;
  return (int)hipGetLastError();
}
