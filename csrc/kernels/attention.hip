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

using namespace vwa;

namespace {

VWA_DEVICE int64_t kv_offset(const KVView& kv, int seq, int kvh, int t) {
  const int blk = kv.block_table[(int64_t)seq * kv.table_stride + t / kv.block_size];
  return (int64_t)blk * kv.stride_block + (int64_t)kvh * kv.stride_head + (int64_t)(t % kv.block_size) * kv.stride_tok;
}

constexpr int kWaves = 4;              // waves per decode workgroup
constexpr int kKeysPerWave = 64;
constexpr int kSplit = kWaves * kKeysPerWave;  // keys per decode workgroup (chunk)

// sc1 (write-through / L2-bypassing) global accesses for the in-launch hand-off (guide G16 R1)
VWA_DEVICE __amdgpu_buffer_rsrc_t rsrc_f32(float* p, int64_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(n * 4), 0x00020000);
}
VWA_DEVICE void st_sc1_f2(__amdgpu_buffer_rsrc_t r, int64_t idx, float a, float b) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, make_float2(a, b)), r, (int)(idx * 4), 0, 16);
}
VWA_DEVICE void st_sc1_f1(__amdgpu_buffer_rsrc_t r, int64_t idx, float a) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(a), r, (int)(idx * 4), 0, 16);
}
VWA_DEVICE float2 ld_sc1_f2(__amdgpu_buffer_rsrc_t r, int64_t idx) {
  return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(idx * 4), 0, 16));
}
VWA_DEVICE float ld_sc1_f1(__amdgpu_buffer_rsrc_t r, int64_t idx) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)(idx * 4), 0, 16));
}

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

// ------------------------------------------------------------------------------------------
// 3) multi-query MFMA decode attention (default; ops.set_attention_impl("split") selects 1)
// ------------------------------------------------------------------------------------------
// Work item = (row group, kv head, key chunk), one 4-wave workgroup each; the grid is capped at
// 512 resident workgroups that walk the items.  A row group is a run of up to 16/G
// consecutive rows of ONE sequence (the last sampled token plus its jump-forward rows, a
// prompt-suffix chunk, Whisper's prompt rows), so its K/V bytes are read once for all of its
// rows x GQA heads: the 16 MFMA query columns are (row, q-head) pairs.  The number of chunks
// per (group, kv head) is chosen in-kernel from the step's actual group count so the items
// fill the grid: a lone decode row spreads its context over up to 16 chunks, 32 concurrent
// sessions get one chunk each (measured first version with a static rows x heads x 16 grid:
// 64 rows of one sequence spent most of 89 us dispatching workgroups that exit at once).
// Per 32-key step a wave computes
//   S^T = K.Q^T    on the MFMA (16x16x32 bf16); K fragments come straight from the paged
//                  cache, the keys of the two 16-key tiles interleaved so that every lane
//                  ends up holding 8 consecutive keys of its query column,
//   an online softmax per query column (lane-local max/sum + 2 xor steps),
//   O^T += V^T.P^T on the MFMA: P^T is already the B operand (no LDS round trip); V rows are
//                  stored row-major into a swizzled per-wave LDS image and read back
//                  transposed with ds_read_b64_tr_b16 (the V^T A operand).
// The old kernel spent ~2 us per wave on 1024 VALU FMAs per lane for G = 4; here the same
// work is 16 MFMAs, and extra rows of a group ride along in the idle query columns.
// Chunks are sized per group from its own context (multiples of 128 keys, at most gridDim.y
// of them), and they merge in-launch through the sc1 hand-off + last-arriver ticket above.
constexpr int kMqCols = 16;                 // query columns per workgroup (group rows x G)
constexpr int kMqStep = 32;                 // keys per wave step
constexpr int kMqChunk = kWaves * kMqStep;  // chunk granularity (keys)

typedef short short4_t __attribute__((ext_vector_type(4)));

// byte offset of 16-byte chunk ch of key row r in a [32 keys][256 B] V image: the guide's T10
// (b) swizzle, conflict-free for the ds_write_b128 row stores and the transposed reads
VWA_DEVICE int vimg_off(int r, int ch) { return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3))); }

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group names row q, columns 4p..4p+3 of a 4 x 16
// bf16 block; lane i receives column i of the 4 rows (row q in element q)
VWA_DEVICE uint2 lds_tr16(const unsigned char* ptr) {
  typedef __attribute__((address_space(3))) short4_t* lds_p;
  const short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_p)(ptr));
  return __builtin_bit_cast(uint2, v);
}

// 16-byte global load through a native vector type: a struct (uint4) copy is emitted as a memcpy
// that SROA cannot promote, and the V staging registers ended up in scratch (measured: 272 B of
// scratch per lane and a vmcnt(0) after every scratch reload inside the key loop)
VWA_DEVICE uint4 ld128(const u16* ptr) {
  const u32x4 v = *reinterpret_cast<const u32x4*>(ptr);
  return make_uint4(v.x, v.y, v.z, v.w);
}

VWA_DEVICE void st_sc1_f4(__amdgpu_buffer_rsrc_t r, int64_t idx, const float* v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, make_float4(v[0], v[1], v[2], v[3])), r,
                                         (int)(idx * 4), 0, 16);
}
VWA_DEVICE float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int64_t idx) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(idx * 4), 0, 16));
}

template <bool SC1>
VWA_DEVICE void store_out(u16* dst, uint4 v) {
  if constexpr (SC1) {
    // agent-scope write-through: read by other workgroups later in the same (chained) launch
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst) + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<uint4*>(dst) = v;
  }
}

// LDS of one multi-query attention workgroup with NW waves: V images, per-wave O^T, (m, l), ticket
template <int D, int NW>
struct MqLds {
  static constexpr int OWP = D + 4;
  static constexpr int vimg = 0;
  static constexpr int ow = NW * kMqStep * 256;
  static constexpr int mlw = ow + NW * kMqCols * OWP * 4;
  static constexpr int last = mlw + NW * kMqCols * 2 * 4;
  static constexpr int bytes = last + 16;
};

// Body of the multi-query decode attention for workgroup `bid` of `grid` workgroups with NW
// waves (the standalone kernel: NW = 4; the chained layer launch: NW = 8).  SC1OUT: outputs are
// written with sc1 stores (read by another workgroup later in the same launch).
template <int D, int G, int NW, bool SC1OUT>
VWA_DEVICE void mq_body(const DecodeAttnParams& p, unsigned char* lds, int grid, int bid) {
  constexpr int kWv = NW;
  constexpr int kChunk = NW * kMqStep;     // chunk granularity (keys)
  constexpr int RG = kMqCols / G;          // rows per group
  constexpr int NKS = D / 32;              // S^T k-steps over the head dim
  constexpr int NDT = D / 16;              // O^T dim tiles
  constexpr int NCH = D / 8;               // 16-byte chunks per key row
  constexpr int NVL = kMqStep * NCH / 64;  // V row chunks per lane per step
  constexpr int OWP = D + 4;               // padded o row (floats): conflict-free float4 stores
  using L = MqLds<D, NW>;
  float* ow = reinterpret_cast<float*>(lds + L::ow);    // [NW][kMqCols][OWP]
  float* mlw = reinterpret_cast<float*>(lds + L::mlw);  // [NW][kMqCols][2]
  int& s_last = *reinterpret_cast<int*>(lds + L::last);

  const int nkv = p.n_kv_heads, nq = p.n_q_heads;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = lane & 15, g = lane >> 4;

  // ---- row groups of the whole step (<= 64 rows; every wave derives the same answer): runs of
  //      consecutive rows of one sequence, cut every RG rows from the run's start
  const int sl = lane < p.rows ? p.seq_ids[lane] : -1;
  const int cl = lane < p.rows ? p.ctx_lens[lane] : 0;  // same round trip as the sequence ids
  const int sp = __shfl(sl, lane > 0 ? lane - 1 : 0, 64);
  const unsigned long long run_starts = __ballot(lane < p.rows && (lane == 0 || sl != sp));
  const int run0 = 63 - __builtin_clzll(run_starts & ((2ull << lane) - 1ull));  // lane 0 always starts a run
  const unsigned long long leaders = __ballot(lane < p.rows && (lane - run0) % RG == 0);
  const int n_groups = __builtin_popcountll(leaders);
  const int my_rank = __builtin_popcountll(leaders & ((1ull << lane) - 1ull));
  // chunks per (group, kv head): spread the work over the grid (one item per workgroup when it
  // fits), never more than the partial buffers hold
  const int n_eff = max(1, min(p.n_splits, grid / max(1, n_groups * nkv)));
  const int n_items = n_groups * nkv * n_eff;

  for (int item = bid; item < n_items; item += grid) {
  // item -> (kv head, group, chunk); kv head fastest so a head's workgroups share one XCD (b % 8)
  const int kvh = item % nkv;
  const int gi = (item / nkv) % n_groups, chunk = item / (nkv * n_groups);
  const unsigned long long pick = __ballot(((leaders >> lane) & 1ull) && my_rank == gi);
  const int r0 = __builtin_ctzll(pick);
  const unsigned long long later = run_starts & ~((2ull << r0) - 1ull);
  const int run_end = later ? __builtin_ctzll(later) : p.rows;
  const int nr = min(RG, run_end - r0);  // rows in this group
  const int seq = __shfl(sl, r0, 64);
  __syncthreads();  // the previous item's LDS readers are done
  const int c_src = __shfl(cl, min(r0 + lane, 63), 64);
  const int c_own = lane < nr ? c_src : 0;
  int ctxmax = c_own;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) ctxmax = max(ctxmax, __shfl_xor(ctxmax, o, 64));
  const int rho = n / G;                     // group row of this lane's query column
  const int ctx_n = __shfl(c_own, rho, 64);  // its context (0 for padded columns)

  // ---- this item's chunk of the group's keys (NW waves x CL/NW keys)
  const int CL = ((ctxmax + n_eff - 1) / n_eff + kChunk - 1) / kChunk * kChunk;
  const int kbeg = chunk * CL;
  if (kbeg >= ctxmax) continue;
  const int nact = (ctxmax + CL - 1) / CL;
  const int wb = kbeg + w * (CL / kWv);
  const int we = min(ctxmax, wb + CL / kWv);
  const int nsteps = we > wb ? (we - wb + kMqStep - 1) / kMqStep : 0;
  const int kmax = ctxmax - 1;  // keys past the context are clamped (finite data, masked scores)

  // ---- Q^T fragments (B operand): Q[column n][dims 32ks + 8g ..], pre-scaled by scale*log2(e)
  bf16x8 qf[NKS];
  {
    const float qs = p.scale * 1.4426950408889634f;
    const u16* qr = p.q + (int64_t)(r0 + min(rho, nr - 1)) * p.ldq + (kvh * G + n % G) * D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(qr + 32 * ks), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = rho < nr ? f[j] * qs : 0.f;
      qf[ks] = as_bf16x8(pack8(f));
    }
  }

  // (measured: staging the wave's block-table entries in lanes and fetching them with __shfl,
  // instead of the per-key table loads below, was 1.5-3 us SLOWER on every shape)
  auto kv_off = [&](int key) -> int64_t { return kv_offset(p.kv, seq, kvh, key); };

  // K: A-operand row n of tile t is key kb + 8(n>>2) + 4t + (n&3) (so the S^T accumulator of lane
  // (n, g) holds keys kb + 8g + 4t + i); V: 32 rows x NCH chunks, chunk idx = i*64 + lane
  auto load_step = [&](int kb, uint4 (&kr)[2][NKS], uint4 (&vr)[NVL]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = min(kb + 8 * (n >> 2) + 4 * t + (n & 3), kmax);
      const u16* kp = p.kv.k + kv_off(key) + 8 * g;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) kr[t][ks] = ld128(kp + 32 * ks);
    }
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int idx = i * 64 + lane;
      const int key = min(kb + idx / NCH, kmax);
      vr[i] = ld128(p.kv.v + kv_off(key) + 8 * (idx % NCH));
    }
  };

  float m_run = -INFINITY, l_run = 0.f;  // per query column (log2 units); l is this lane's share
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned char* vi = lds + L::vimg + w * kMqStep * 256;

  auto compute_step = [&](int kb, const uint4 (&kr)[2][NKS], const uint4 (&vr)[NVL]) {
#pragma unroll
    for (int i = 0; i < NVL; ++i) {
      const int idx = i * 64 + lane;
      *reinterpret_cast<uint4*>(vi + vimg_off(idx / NCH, idx % NCH)) = vr[i];
    }
    f32x4 s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) s[t] = mfma16(as_bf16x8(kr[t][ks]), qf[ks], s[t]);
    }
    float pv[8];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = (kb + 8 * g + 4 * t + i < ctx_n) ? s[t][i] : -INFINITY;
        pv[4 * t + i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = (m_run == -INFINITY) ? 0.f : exp2f(m_run - m_new);
    float ps = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pv[j] = (pv[j] == -INFINITY) ? 0.f : exp2f(pv[j] - m_new);
      ps += pv[j];
    }
    l_run = l_run * alpha + ps;
    m_run = m_new;
    const bf16x8 pb = as_bf16x8(pack8(pv));  // P^T[keys 8g..8g+7][column n]
    const int q4 = n >> 2, p4 = n & 3;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      // V^T[dim 16dt + n][keys 8g..8g+7]: two 4-key transposed reads of the image
      const int ch = 2 * dt + (p4 >> 1), sub = 8 * (p4 & 1);
      const uint2 lo = lds_tr16(vi + vimg_off(8 * g + q4, ch) + sub);
      const uint2 hi = lds_tr16(vi + vimg_off(8 * g + 4 + q4, ch) + sub);
      o[dt] = mfma16(as_bf16x8(make_uint4(lo.x, lo.y, hi.x, hi.y)), pb, o[dt] * alpha);
    }
  };

  if (nsteps > 0) {
    uint4 kA[2][NKS], vA[NVL], kB[2][NKS], vB[NVL];
    load_step(wb, kA, vA);
    for (int s = 0; s < nsteps; s += 2) {
      if (s + 1 < nsteps) load_step(wb + (s + 1) * kMqStep, kB, vB);
      compute_step(wb + s * kMqStep, kA, vA);
      if (s + 1 >= nsteps) break;
      if (s + 2 < nsteps) load_step(wb + (s + 2) * kMqStep, kA, vA);
      compute_step(wb + (s + 1) * kMqStep, kB, vB);
    }
  }

  // ---- per-wave (m, l, O) -> LDS; O^T accumulator of lane (n, g): dims 16dt + 4g + i
  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (g == 0) {
    mlw[(w * kMqCols + n) * 2 + 0] = m_run;
    mlw[(w * kMqCols + n) * 2 + 1] = l_tot;
  }
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
    *reinterpret_cast<float4*>(&ow[(w * kMqCols + n) * OWP + 16 * dt + 4 * g]) = make_float4(o[dt][0], o[dt][1], o[dt][2], o[dt][3]);
  __syncthreads();

  // ---- merge the waves: thread -> (query column cn, 8-dim chunk dc)
  const int cn = threadIdx.x >> 4, dc = threadIdx.x & 15;
  const int crow = r0 + cn / G, ch = kvh * G + cn % G;
  const bool act = cn / G < nr && dc < NCH;
  const __amdgpu_buffer_rsrc_t r_o = rsrc_f32(p.part_o, (int64_t)p.rows * p.n_splits * nq * D);
  const __amdgpu_buffer_rsrc_t r_ml = rsrc_f32(p.part_ml, (int64_t)p.rows * p.n_splits * nq * 2);
  float acc[8];
  if (act) {
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < kWv; ++ww) M = fmaxf(M, mlw[(ww * kMqCols + cn) * 2]);
    float L = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
    for (int ww = 0; ww < kWv; ++ww) {
      const float mw = mlw[(ww * kMqCols + cn) * 2];
      const float f = (mw == -INFINITY) ? 0.f : exp2f(mw - M);
      L += mlw[(ww * kMqCols + cn) * 2 + 1] * f;
      const float4 a = *reinterpret_cast<const float4*>(&ow[(ww * kMqCols + cn) * OWP + 8 * dc]);
      const float4 b = *reinterpret_cast<const float4*>(&ow[(ww * kMqCols + cn) * OWP + 8 * dc + 4]);
      acc[0] += f * a.x; acc[1] += f * a.y; acc[2] += f * a.z; acc[3] += f * a.w;
      acc[4] += f * b.x; acc[5] += f * b.y; acc[6] += f * b.z; acc[7] += f * b.w;
    }
    if (nact == 1) {
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= inv;
      store_out<SC1OUT>(p.out + (int64_t)crow * p.ldo + ch * D + 8 * dc, pack8(acc));
    } else {
      const int64_t base = ((int64_t)crow * p.n_splits + chunk) * nq + ch;
      st_sc1_f4(r_o, base * D + 8 * dc, acc);
      st_sc1_f4(r_o, base * D + 8 * dc + 4, acc + 4);
      if (dc == 0) st_sc1_f2(r_ml, base * 2, M, L);
    }
  }
  if (nact == 1) continue;

  // ---- ticket (same protocol as the split kernel): drained sc1 stores, then one counter add
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int* cnt = p.counters + r0 * nkv + kvh;
    const int ticket = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (ticket == nact - 1);
    if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) continue;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // only orders the sc1 loads after the ticket

  // ---- last arriver: online merge of the nact chunks (sc1 loads only; measured: issuing the loads
  //      in unrolled batches of 8 chunks before combining was 2 us SLOWER in-bench, 13.6 vs 11.4 us)
  if (act) {
    const int64_t hb = (int64_t)crow * p.n_splits * nq + ch;
    float M = -INFINITY, L = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll 4
    for (int c = 0; c < nact; ++c) {
      const int64_t b = hb + (int64_t)c * nq;
      const float2 ml = ld_sc1_f2(r_ml, b * 2);
      const float4 x0 = ld_sc1_f4(r_o, b * D + 8 * dc), x1 = ld_sc1_f4(r_o, b * D + 8 * dc + 4);
      const float Mn = fmaxf(M, ml.x);
      const float fo = (M == -INFINITY) ? 0.f : exp2f(M - Mn);
      const float fc = (ml.x == -INFINITY) ? 0.f : exp2f(ml.x - Mn);
      L = L * fo + ml.y * fc;
      acc[0] = acc[0] * fo + x0.x * fc; acc[1] = acc[1] * fo + x0.y * fc;
      acc[2] = acc[2] * fo + x0.z * fc; acc[3] = acc[3] * fo + x0.w * fc;
      acc[4] = acc[4] * fo + x1.x * fc; acc[5] = acc[5] * fo + x1.y * fc;
      acc[6] = acc[6] * fo + x1.z * fc; acc[7] = acc[7] * fo + x1.w * fc;
      M = Mn;
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= inv;
    store_out<SC1OUT>(p.out + (int64_t)crow * p.ldo + ch * D + 8 * dc, pack8(acc));
  }
  }  // items
}

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
