// Attention kernels for gfx950.
//
// 1) decode_attention (K10, K7): one query row per (sequence | forced token), paged KV,
//    GQA group of G q-heads per kv-head handled by one workgroup so each K/V byte is read
//    once per group.  Split-K over the context in 256-key chunks (4 waves x 64 keys), the
//    waves merged in LDS and the chunks merged in-launch by the last-arriving chunk through an
//    sc1 (write-through) hand-off.  Measured history (1 row, ctx 1200, incl. launch gaps):
//    64-key single-wave splits + separate combine launch 14.4 us; same with an agent-scope
//    release/acquire fenced last-arriver merge 28 us (fences write back / invalidate the per-XCD
//    L2 per workgroup); with per-float relaxed atomics and a head-serial merge 24 us.  The grid is sized for the maximum context so the launch
//    shape is static under hipGraph capture; splits past a row's context exit early.
//    Also serves Whisper cross-attention (contiguous encoder K/V expressed as one block).
//
// 2) flash_attention (K5, K6): MFMA (16x16x32 bf16) flash-attention forward for prefill and
//    for the Whisper encoder.  "Swapped" formulation: each wave computes S^T = K.Q^T for its
//    16 queries so a query's scores sit in one lane column; P^T is then already the B
//    operand of O^T += V^T.P^T (no LDS round trip for P), and the online-softmax row
//    reductions are 2 cross-lane steps.  K is staged XOR-swizzled (conflict-free
//    ds_read_b128), V is staged transposed with a padded row.  Causal masking with an
//    absolute query offset supports prefix-cached prefill (queries at positions
//    q_offset.., keys 0..).
#include "common.h"
#include "vwa_kernels.h"
#include "mq_attention.h"

using namespace vwa;

namespace {


constexpr int kWaves = 4;              // waves per decode workgroup
constexpr int kKeysPerWave = 64;
constexpr int kSplit = kWaves * kKeysPerWave;  // keys per decode workgroup (chunk)


// One 4-wave workgroup per (row, kv head, 256-key chunk); each wave owns 64 keys.
//  Q.K: lane = key, the key row streamed with D/8 independent 16-byte loads (V loads issued
//  right behind them: their addresses do not depend on the scores).  P.V: lane = (16-byte dim
//  chunk, token group), token groups reduced with xor-shuffles.  The 4 waves' (m, l, o) are
//  merged through LDS (wave w merges q-heads g = w, w+4, ...).  A row with one active chunk
//  writes its output directly; otherwise each chunk publishes (m, l, o) with sc1 stores, draws a
//  ticket, and the last-arriving chunk merges them with sc1 loads (no release/acquire fences,
//  no second launch).  Tickets are reset by the last arriver (counters allocated zeroed).
template <int D, int G>
__global__ __launch_bounds__(kWaves * 64) void decode_attn_kernel(DecodeAttnParams p) {
  constexpr int NCH = D / 8;        // 16-byte chunks per row
  constexpr int TG = 64 / NCH;      // token groups
  constexpr int NI = kKeysPerWave / TG;  // tokens per lane in P.V
  constexpr int DPL = D / 64;       // output dims per lane in the merges
  __shared__ __attribute__((aligned(16))) float qs[G][D];
  __shared__ float sc[kWaves][G][kKeysPerWave];
  __shared__ float mlw[kWaves][G][2];
  __shared__ __attribute__((aligned(16))) float ow[kWaves][G][D];
  __shared__ float wts[kWaves][64];
  __shared__ int s_last;

  const int nkv = p.n_kv_heads, nq = p.n_q_heads;
  const int row = blockIdx.x / nkv, kvh = blockIdx.x % nkv;
  const int chunk = blockIdx.y;
  const int ctx = p.ctx_lens[row];
  const int seq = p.seq_ids[row];
  if (chunk * kSplit >= ctx) return;  // chunk past this row's context (grid sized for max_ctx)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t0 = chunk * kSplit + w * kKeysPerWave;
  const int tend = min(ctx, t0 + kKeysPerWave);  // t0 >= tend: this wave has no keys
  const int nact = (ctx + kSplit - 1) / kSplit;  // active chunks of this row

  // ---- issue K (lane = key) and V (lane = chunk c, token group tg) loads first
  const int c = lane % NCH, tg = lane / NCH;
  const int t = t0 + lane;
  uint4 kv4[NCH];
  if (t < tend) {
    const uint4* kr = reinterpret_cast<const uint4*>(p.kv.k + kv_offset(p.kv, seq, kvh, t));
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) kv4[cc] = kr[cc];
  }
  uint4 vv[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int tt = t0 + tg + TG * i;
    vv[i] = (tt < tend) ? *reinterpret_cast<const uint4*>(p.kv.v + kv_offset(p.kv, seq, kvh, tt) + c * 8)
                        : make_uint4(0, 0, 0, 0);
  }
  // q (scaled) into LDS while the K/V loads are in flight
  for (int i = threadIdx.x * 8; i < G * D; i += kWaves * 64 * 8) {
    const int g = i / D, d = i % D;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(p.q + (int64_t)row * p.ldq + (kvh * G + g) * D + d), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) qs[g][d + j] = f[j] * p.scale;
  }
  __syncthreads();

  // ---- Q.K and the wave's softmax statistics
  float s[G];
#pragma unroll
  for (int g = 0; g < G; ++g) s[g] = 0.f;
  if (t < tend) {
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      float kf[8];
      unpack8(kv4[cc], kf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float4 qa = *reinterpret_cast<const float4*>(&qs[g][cc * 8]);
        const float4 qb = *reinterpret_cast<const float4*>(&qs[g][cc * 8 + 4]);
        s[g] += qa.x * kf[0] + qa.y * kf[1] + qa.z * kf[2] + qa.w * kf[3] + qb.x * kf[4] + qb.y * kf[5] +
                qb.z * kf[6] + qb.w * kf[7];
      }
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float v = (t < tend) ? s[g] : -INFINITY;
    const float m = wave_max(v);
    const float e = (t < tend) ? __expf(v - m) : 0.f;
    const float l = wave_sum(e);
    sc[w][g][lane] = e;
    if (lane == 0) {
      mlw[w][g][0] = m;  // -inf for a wave without keys
      mlw[w][g][1] = l;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();

  // ---- P.V (V already in registers)
  float o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    float vf[8];
    unpack8(vv[i], vf);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float pg = sc[w][g][tg + TG * i];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] += pg * vf[j];
    }
  }
#pragma unroll
  for (int off = NCH; off < 64; off <<= 1)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] += __shfl_xor(o[g][j], off, 64);
  if (tg == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      *reinterpret_cast<float4*>(&ow[w][g][c * 8]) = make_float4(o[g][0], o[g][1], o[g][2], o[g][3]);
      *reinterpret_cast<float4*>(&ow[w][g][c * 8 + 4]) = make_float4(o[g][4], o[g][5], o[g][6], o[g][7]);
    }
  }
  __syncthreads();

  // ---- merge the 4 waves: wave w takes q-heads g = w, w + 4, ... (lane = DPL dims)
  const __amdgpu_buffer_rsrc_t r_o = rsrc_f32(p.part_o, (int64_t)p.rows * p.n_splits * nq * D);
  const __amdgpu_buffer_rsrc_t r_ml = rsrc_f32(p.part_ml, (int64_t)p.rows * p.n_splits * nq * 2);
  for (int g = w; g < G; g += kWaves) {
    const int h = kvh * G + g;
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) M = fmaxf(M, mlw[ww][g][0]);
    float L = 0.f, acc[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
      const float mw = mlw[ww][g][0];
      const float f = (mw == -INFINITY) ? 0.f : __expf(mw - M);
      L += mlw[ww][g][1] * f;
#pragma unroll
      for (int j = 0; j < DPL; ++j) acc[j] += ow[ww][g][lane * DPL + j] * f;
    }
    if (nact == 1) {
      const float inv = 1.f / L;
#pragma unroll
      for (int j = 0; j < DPL; ++j) p.out[(int64_t)row * p.ldo + h * D + lane * DPL + j] = f2bf(acc[j] * inv);
    } else {
      const int64_t base = ((int64_t)row * p.n_splits + chunk) * nq + h;
      if constexpr (DPL == 2) st_sc1_f2(r_o, base * D + lane * 2, acc[0], acc[1]);
      else st_sc1_f1(r_o, base * D + lane, acc[0]);
      if (lane == 0) st_sc1_f2(r_ml, base * 2, M, L);
    }
  }
  if (nact == 1) return;

  // ---- ticket: every storing wave drains its sc1 stores, then one lane counts this chunk in
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cnt = p.counters + row * nkv + kvh;
    const int ticket = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (ticket == nact - 1);
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // only orders the sc1 loads after the ticket

  // ---- last arriver: merge the nact chunks (lane = chunk for the statistics, lane = dims for o)
  for (int g = w; g < G; g += kWaves) {
    const int h = kvh * G + g;
    const int64_t hb = (int64_t)row * p.n_splits * nq + h;
    float mloc = -INFINITY, lloc = 0.f;
    if (lane < nact) {
      const float2 ml = ld_sc1_f2(r_ml, (hb + (int64_t)lane * nq) * 2);
      mloc = ml.x;
      lloc = ml.y;
    }
    const float M = wave_max(mloc);
    const float f = (lane < nact) ? __expf(mloc - M) : 0.f;
    const float L = wave_sum(lloc * f);
    wts[w][lane] = f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float acc[DPL];
#pragma unroll
    for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
    for (int sp = 0; sp < nact; ++sp) {
      const float wt = wts[w][sp];
      const int64_t idx = (hb + (int64_t)sp * nq) * D + lane * DPL;
      if constexpr (DPL == 2) {
        const float2 v = ld_sc1_f2(r_o, idx);
        acc[0] += wt * v.x;
        acc[1] += wt * v.y;
      } else {
        acc[0] += wt * ld_sc1_f1(r_o, idx);
      }
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int j = 0; j < DPL; ++j) p.out[(int64_t)row * p.ldo + h * D + lane * DPL + j] = f2bf(acc[j] * inv);
    __builtin_amdgcn_wave_barrier();
  }
}

template <int D, int G>
void launch_decode(const DecodeAttnParams& p, hipStream_t st) {
  hipLaunchKernelGGL((decode_attn_kernel<D, G>), dim3(p.rows * p.n_kv_heads, p.n_splits), dim3(kWaves * 64), 0, st,
                     p);
}

template <int D>
int dispatch_g(const DecodeAttnParams& p, hipStream_t st) {
  switch (p.n_q_heads / p.n_kv_heads) {
    case 1: launch_decode<D, 1>(p, st); break;
    case 2: launch_decode<D, 2>(p, st); break;
    case 4: launch_decode<D, 4>(p, st); break;
    case 8: launch_decode<D, 8>(p, st); break;
    default: return -2;
  }
  return 0;
}

constexpr int kMqChunk = kWaves * kMqStep;  // chunk granularity of the standalone kernel (keys)

template <int D, int G>
__global__ __launch_bounds__(kWaves * 64) void decode_mq_kernel(DecodeAttnParams p) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[MqLds<D, kWaves>::bytes];
  mq_body<D, G, kWaves, false>(p, lds, (int)gridDim.x, (int)blockIdx.x);
}

constexpr int kMqMaxGrid = 512;  // two 67 KB-LDS workgroups per CU: the whole grid is resident

template <int D>
int dispatch_mq(const DecodeAttnParams& p, hipStream_t st) {
  const int items = p.rows * p.n_kv_heads * p.n_splits;  // upper bound (every row its own group)
  const dim3 grid(items < kMqMaxGrid ? items : kMqMaxGrid), block(kWaves * 64);
  switch (p.n_q_heads / p.n_kv_heads) {
    case 1: hipLaunchKernelGGL((decode_mq_kernel<D, 1>), grid, block, 0, st, p); break;
    case 2: hipLaunchKernelGGL((decode_mq_kernel<D, 2>), grid, block, 0, st, p); break;
    case 4: hipLaunchKernelGGL((decode_mq_kernel<D, 4>), grid, block, 0, st, p); break;
    case 8: hipLaunchKernelGGL((decode_mq_kernel<D, 8>), grid, block, 0, st, p); break;
    case 16: hipLaunchKernelGGL((decode_mq_kernel<D, 16>), grid, block, 0, st, p); break;
    default: return -2;
  }
  return 0;
}

int g_attn_impl = 1;  // 1: multi-query MFMA kernel (default), 0: split VALU kernel

// ------------------------------------------------------------------------------------------
// flash attention forward (MFMA)
// ------------------------------------------------------------------------------------------
constexpr int kBQ = 64;   // queries per workgroup (4 waves x 16)
constexpr int kBK = 64;   // keys per tile

// v2 (rocprof: v1 spent 39-60% of LDS cycles in bank conflicts and exposed every key tile's global
// load latency -- 82 us/layer for 84 queries x 1.1k keys):
//  * K / V of the NEXT 64-key tile are loaded into registers while the current tile computes;
//  * V is stored row-major in the dual-use image (b) of the guide (256-byte rows, chunk XOR) and
//    read as the O^T A operand with ds_read_b64_tr_b16 (no 2-byte transposing stores);
//  * the S^T tiles read K rows in an interleaved key order (A row n of tile t in a 32-key block =
//    key 8(n>>2) + 4t + (n&3)) so each lane's probabilities are 8 consecutive keys: the two
//    transposed V reads of a 32-lane half are then 8 rows apart (conflict-free).
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void flash_attn_kernel(FlashAttnParams p) {
  constexpr int NCH = D / 8;               // 16-byte chunks per K / V row
  constexpr int NDS = D / 32;              // MFMA k-steps over head dim
  constexpr int NDT = D / 16;              // 16-row d tiles of O^T
  constexpr int LPT = kBK * NCH / 256;     // 16-byte chunks per thread per tile (K and V each)
  __shared__ __attribute__((aligned(16))) u16 ks[kBK * D];
  __shared__ __attribute__((aligned(16))) unsigned char vimg[kBK * 256];

  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int kvh = h / (p.n_q_heads / p.n_kv_heads);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int ql = lane & 15, g = lane >> 4;
  const int qoff = p.q_offsets ? p.q_offsets[b] : p.q_offset;
  const int Sk = p.k_lens ? p.k_lens[b] : p.Sk;
  const int qi = qb * kBQ + w * 16 + ql;  // query index within the batch row
  const int qpos = qoff + qi;
  const float sl2 = p.scale * 1.4426950408889634f;

  // Q^T fragments (B operand): Q[q][ds*32 + 8g + j], pre-scaled by scale*log2(e)
  bf16x8 qf[NDS];
  {
    const u16* qr = p.q + (int64_t)b * p.q_stride_b + (int64_t)qi * p.q_stride_s + (int64_t)h * p.q_stride_h;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      float f[8];
      if (qi < p.Sq) unpack8(*reinterpret_cast<const uint4*>(qr + ds * 32 + 8 * g), f);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[ds] = as_bf16x8(pack8(f));
    }
  }

  f32x4 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) oacc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  int k_end = Sk;
  if (CAUSAL) k_end = min(Sk, qoff + qb * kBQ + kBQ);

  uint4 kr[LPT], vr[LPT];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / NCH, ch = c % NCH;
      const int t = k0 + r;
      if (t < Sk) {
        const int64_t off = kv_offset(p.kv, b, kvh, t) + ch * 8;
        kr[i] = ld128(p.kv.k + off);
        vr[i] = ld128(p.kv.v + off);
      } else {
        kr[i] = make_uint4(0, 0, 0, 0);
        vr[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  if (k_end > 0) load_tile(0);
  for (int k0 = 0; k0 < k_end; k0 += kBK) {
    // ---- registers -> LDS (K swizzled rows, V image (b)); then the next tile's loads go out
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = threadIdx.x + i * 256;
      const int r = c / NCH, ch = c % NCH;
      *reinterpret_cast<uint4*>(&ks[r * D + ((ch ^ (r % NCH)) * 8)]) = kr[i];
      *reinterpret_cast<uint4*>(vimg + vimg_off(r, ch)) = vr[i];
    }
    __syncthreads();
    if (k0 + kBK < k_end) load_tile(k0 + kBK);

    // ---- S^T = K . Q^T: 2 blocks of 32 keys x 2 interleaved 16-row tiles
    f32x4 s[2][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[kk][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int r = 32 * kk + 8 * (ql >> 2) + 4 * t + (ql & 3);
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds) {
          const int ch = ds * 4 + g;
          const uint4 a = *reinterpret_cast<const uint4*>(&ks[r * D + ((ch ^ (r % NCH)) * 8)]);
          s[kk][t] = mfma16(as_bf16x8(a), qf[ds], s[kk][t]);
        }
      }
    // ---- mask + online softmax (column = this lane's query); lane holds keys 32kk + 8g + 4t + i
    float tmax = -INFINITY;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int kidx = k0 + 32 * kk + 8 * g + 4 * t + i;
          const bool ok = (kidx < Sk) && (!CAUSAL || kidx <= qpos);
          if (!ok) s[kk][t][i] = -INFINITY;
          tmax = fmaxf(tmax, s[kk][t][i]);
        }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = (m_run == -INFINITY) ? 0.f : exp2f(m_run - m_new);
    const bool any = (m_new != -INFINITY);
    float psum = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float e = (any && s[kk][t][i] != -INFINITY) ? exp2f(s[kk][t][i] - m_new) : 0.f;
          s[kk][t][i] = e;
          psum += e;
        }
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) oacc[dt] *= alpha;

    // ---- O^T += V^T . P^T per 32-key block: P^T[keys 8g..8g+7][query column]
    const int q4 = ql >> 2, p4 = ql & 3;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      float pf[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[i] = s[kk][0][i];
        pf[4 + i] = s[kk][1][i];
      }
      const bf16x8 pb = as_bf16x8(pack8(pf));
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int ch = 2 * dt + (p4 >> 1), sub = 8 * (p4 & 1);
        const uint2 lo = lds_tr16(vimg + vimg_off(32 * kk + 8 * g + q4, ch) + sub);
        const uint2 hi = lds_tr16(vimg + vimg_off(32 * kk + 8 * g + 4 + q4, ch) + sub);
        oacc[dt] = mfma16(as_bf16x8(make_uint4(lo.x, lo.y, hi.x, hi.y)), pb, oacc[dt]);
      }
    }
    __syncthreads();
  }

  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (qi < p.Sq) {
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    u16* orow = p.o + (int64_t)b * p.o_stride_b + (int64_t)qi * p.o_stride_s + (int64_t)h * p.o_stride_h;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      uint2 v;
      v.x = pack2(oacc[dt][0] * inv, oacc[dt][1] * inv);
      v.y = pack2(oacc[dt][2] * inv, oacc[dt][3] * inv);
      *reinterpret_cast<uint2*>(orow + dt * 16 + 4 * g) = v;
    }
  }
}

}  // namespace

extern "C" void vwa_set_attention_impl(int impl) { g_attn_impl = impl; }

extern "C" int vwa_decode_attention(const DecodeAttnParams* p, hipStream_t st) {
  if (p->n_kv_heads <= 0 || p->n_q_heads % p->n_kv_heads) return -1;
  int r;
  // the multi-query kernel's group scan looks at most 64 rows back (decode steps are <= 64 rows)
  if (g_attn_impl == 1 && p->rows <= 64 && (p->head_dim == 128 || p->head_dim == 64)) {
    r = p->head_dim == 128 ? dispatch_mq<128>(*p, st) : dispatch_mq<64>(*p, st);
  } else if (p->head_dim == 128) r = dispatch_g<128>(*p, st);
  else if (p->head_dim == 64) r = dispatch_g<64>(*p, st);
  else return -3;
  if (r) return r;
  return (int)hipGetLastError();
}

extern "C" int vwa_flash_attention(const FlashAttnParams* p, hipStream_t st) {
  if (p->n_kv_heads <= 0 || p->n_q_heads % p->n_kv_heads) return -1;
  dim3 grid((p->Sq + kBQ - 1) / kBQ, p->n_q_heads, p->B);
  if (p->head_dim == 128) {
    if (p->causal) hipLaunchKernelGGL((flash_attn_kernel<128, true>), grid, dim3(256), 0, st, *p);
    else hipLaunchKernelGGL((flash_attn_kernel<128, false>), grid, dim3(256), 0, st, *p);
  } else if (p->head_dim == 64) {
    if (p->causal) hipLaunchKernelGGL((flash_attn_kernel<64, true>), grid, dim3(256), 0, st, *p);
    else hipLaunchKernelGGL((flash_attn_kernel<64, false>), grid, dim3(256), 0, st, *p);
  } else {
    return -3;
  }
  return (int)hipGetLastError();
}

// chunk granularity of the decode grid (grid.y = ceil(max_ctx / this)); the split kernel's
// 256-key chunks use every other grid row
extern "C" int vwa_attention_split_tokens() { return kMqChunk; }
