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
// flash attention forward (MFMA 32x32x16)
// ------------------------------------------------------------------------------------------
// v3 (rocprof r3: the 16x16x32 v2 kernel ran at 5-7 % MFMA busy with 23-24 % LDS bank conflicts;
// 16 queries per wave made every K / V byte read from LDS feed only 16 columns):
//  * a wave owns 32 queries and computes S^T = K.Q^T with v_mfma_f32_32x32x16_bf16, so each K
//    fragment read from LDS serves 32 queries and a lane holds 16 keys of ONE query per 32-key block;
//  * the K rows of a block are read in a permuted order (A row R <- key kb(R)) so that lane half
//    h's 16 scores are keys {8h..8h+7, 16+8h..16+8h+7}: exactly the B operand (P^T) of
//    O^T += V^T.P^T for the two 16-key slices -- no lane exchange, no LDS round trip for P;
//  * K and V tiles both live in one swizzled image (FlashCfg::off): the 32x32x16 row reads of K
//    and the ds_read_b64_tr_b16 reads of V^T are conflict-free on it;
//  * online softmax with a deferred rescale: the running max moves (and O, l are rescaled) only
//    when a tile's max exceeds it by more than kRescale (log2 units; P <= 2^kRescale, f32 sums);
//  * 4 query waves x NS key splits (FlashCfg: 2 for D = 128, 3 for D = 64): split s takes the
//    64-key tiles s, s + NS, ... into its own double-buffered LDS images (the next tile's global
//    loads issued behind the LDS stores, one barrier per tile round); the splits' (m, l, O) merge
//    through LDS at the end.  NS waves per SIMD hide each other's MFMA -> softmax -> MFMA
//    dependency chains, and each wave's serial tile chain is 1/NS as long (the 4-wave form
//    measured ~3.6k cycles per tile, latency-bound at one wave per SIMD);
//  * the sequence's block-table row is copied to LDS once (no dependent global load per tile).
// Grid: 1-D, XCD-remapped so a (batch, head)'s query blocks share an XCD's L2 (K / V reuse);
// within a head the query blocks run last-first (causal: the longest rows start first).
constexpr int kFQ = 128;         // queries per workgroup (4 query waves x 32)
constexpr int kFK = 64;          // keys per tile
constexpr int kFTab = 1024;      // block-table entries cached in LDS
constexpr float kRescale = 8.f;  // deferred-max threshold (log2 units)

// Per head dim: key splits (wave groups of 4) per workgroup and the K / V tile image.
//  D = 128: 256-byte rows, image (b) (vimg_off), 16 KB per tile -> 2 splits (8 waves, 128 KB).
//  D = 64: the guide's image (a) with 128-byte rows -- 8-row x 32-column subtiles of 512 B,
//  off = 1024 (row >> 3) + 512 (ch >> 2) + 64 (row & 7) + 16 ((ch & 3) ^ ((row >> 2) & 3)): the same
//  bank pattern as the 256-byte-row form (512 and 1024 are multiples of the 256-byte bank cycle),
//  so its row and transposed reads stay conflict-free at half the bytes (8 KB per tile).
// DEPTH: tiles in flight in registers per split (global -> register -> LDS staging).  The tile
// fetch is latency-bound (one 16-32 KB tile per split per iteration, ~9 B/cycle/CU measured with
// DEPTH 1), so D = 64 keeps two register sets (2 tiles ahead; +16 VGPRs) -- 3 splits at depth 1
// measured no faster than 2 -- while D = 128 (32 VGPRs per set) has no room for a second.
template <int D> struct FlashCfg;
template <> struct FlashCfg<128> {
  static constexpr int NS = 2, DEPTH = 1, IMG = kFK * 256;
  static VWA_DEVICE int off(int r, int ch) { return vimg_off(r, ch); }
};
template <> struct FlashCfg<64> {
  static constexpr int NS = 2, DEPTH = 2, IMG = kFK * 128;
  static VWA_DEVICE int off(int r, int ch) {
    return 1024 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
  }
};
template <int D>
constexpr int flash_lds() {  // [split][stage][K, V] images + block table
  return FlashCfg<D>::NS * 2 * 2 * FlashCfg<D>::IMG + kFTab * 4;
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
VWA_DEVICE f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int D, bool CAUSAL>
__global__ __launch_bounds__(256 * FlashCfg<D>::NS) void flash_attn_kernel(FlashAttnParams p) {
  using FC = FlashCfg<D>;
  constexpr int NS = FC::NS, IMG = FC::IMG;
  constexpr int NCH = D / 8;            // 16-byte chunks per K / V row
  constexpr int NDS = D / 16;           // QK k-steps over the head dim
  constexpr int NDT = D / 32;           // 32-row d tiles of O^T
  constexpr int LPT = kFK * NCH / 256;  // 16-byte chunks per thread per tile (K and V each)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int* btab = reinterpret_cast<int*>(smem + NS * 2 * 2 * IMG);

  const int nqb = (p.Sq + kFQ - 1) / kFQ;
  const int nwg = nqb * p.n_q_heads * p.B;
  const int L = xcd_remap((int)blockIdx.x, nwg);
  const int hb = L / nqb, qb = nqb - 1 - L % nqb;
  const int h = hb % p.n_q_heads, b = hb / p.n_q_heads;
  const int kvh = h / (p.n_q_heads / p.n_kv_heads);
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  const int w = wid & 3, split = wid >> 2;  // query wave, key split
  const int stid = threadIdx.x & 255;       // thread index within the split
  const int col = lane & 31, hf = lane >> 5;  // query column, lane half
  const int qoff = p.q_offsets ? p.q_offsets[b] : p.q_offset;
  const int Sk = p.k_lens ? p.k_lens[b] : p.Sk;
  const int qw0 = qb * kFQ + w * 32;  // first query of this wave
  const int qi = qw0 + col;
  const int qpos = qoff + qi;
  const float sl2 = p.scale * 1.4426950408889634f;
  unsigned char* simg = smem + split * (2 * 2 * IMG);  // this split's [stage][K, V] images

  int k_end = Sk;
  if (CAUSAL) k_end = min(Sk, qoff + qb * kFQ + kFQ);
  const int nt = (k_end + kFK - 1) / kFK;
  const int k_load = min(Sk, nt * kFK);  // keys the tiles load (the last tile may pass k_end)
  const int nblk = (k_load + p.kv.block_size - 1) / p.kv.block_size;
  const bool tab_lds = nblk <= kFTab;
  if (tab_lds)
    for (int i = threadIdx.x; i < nblk; i += 256 * NS) btab[i] = p.kv.block_table[(int64_t)b * p.kv.table_stride + i];

  // Q^T fragments (B operand): lane (col, hf) holds Q[qi][16 ds + 8 hf + j], pre-scaled by scale*log2(e)
  bf16x8 qf[NDS];
  {
    const u16* qr = p.q + (int64_t)b * p.q_stride_b + (int64_t)qi * p.q_stride_s + (int64_t)h * p.q_stride_h;
#pragma unroll
    for (int ds = 0; ds < NDS; ++ds) {
      float f[8];
      if (qi < p.Sq) unpack8(ld128(qr + ds * 16 + 8 * hf), f);
      else {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[ds] = as_bf16x8(pack8(f));
    }
  }

  f32x16 oacc[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) oacc[dt][i] = 0.f;
  float m_run = 0.f, l_run = 0.f;
  __syncthreads();  // block table in LDS

  uint4 kra[LPT], vra[LPT], krb[LPT], vrb[LPT];  // register sets A, B (B: DEPTH 2 only)
  // loader: thread row r_i = (stid + 256 i) / NCH, chunk ch_i.  One block for the whole sequence
  // (contiguous K / V, e.g. the encoder): a fixed per-thread offset + t * stride_tok; paged with a
  // power-of-two block size: shifts; otherwise the general division.
  const int bs = p.kv.block_size;
  const bool one_block = bs >= k_load;
  const int lbs = (bs & (bs - 1)) == 0 ? __builtin_ctz(bs) : -1;
  const int64_t head_off = (int64_t)kvh * p.kv.stride_head;
  const int64_t blk0_off = one_block ? (int64_t)(tab_lds ? btab[0] : p.kv.block_table[(int64_t)b * p.kv.table_stride]) *
                                           p.kv.stride_block + head_off
                                     : 0;
  auto load_tile = [&](int k0, uint4 (&kr)[LPT], uint4 (&vr)[LPT]) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = stid + i * 256;
      const int r = c / NCH, ch = c % NCH;
      const int t = k0 + r;
      if (t < Sk) {
        int64_t off;
        if (one_block) {
          off = blk0_off + (int64_t)t * p.kv.stride_tok + ch * 8;
        } else {
          const int bi = lbs >= 0 ? (t >> lbs) : t / bs, bo = lbs >= 0 ? (t & (bs - 1)) : t % bs;
          const int blk = tab_lds ? btab[bi] : p.kv.block_table[(int64_t)b * p.kv.table_stride + bi];
          off = (int64_t)blk * p.kv.stride_block + head_off + (int64_t)bo * p.kv.stride_tok + ch * 8;
        }
        kr[i] = ld128(p.kv.k + off);
        vr[i] = ld128(p.kv.v + off);
      } else {
        kr[i] = make_uint4(0, 0, 0, 0);  // V rows past the end must be finite (0 * NaN = NaN)
        vr[i] = make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store_tile = [&](int stg, const uint4 (&kr)[LPT], const uint4 (&vr)[LPT]) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int c = stid + i * 256;
      const int r = c / NCH, ch = c % NCH;
      *reinterpret_cast<uint4*>(simg + (2 * stg) * IMG + FC::off(r, ch)) = kr[i];
      *reinterpret_cast<uint4*>(simg + (2 * stg + 1) * IMG + FC::off(r, ch)) = vr[i];
    }
  };

  // A-row permutation of a 32-key block: MFMA row R = (i&3) + 8(i>>2) + 4hf of register i in lane
  // half hf holds key (i&7) + 16(i>>3) + 8hf; the lane supplying A row `col` reads that key
  const int a_hi = (col >> 2) & 1, a_r = (col & 3) + 4 * (col >> 3);
  const int a_key = (a_r & 7) + 16 * (a_r >> 3) + 8 * a_hi;
  // V^T transposed reads (ds_read_b64_tr_b16): 16-lane group grp covers d 16(grp&1).. of a 32-d
  // tile and key half grp>>1; lane 4q+p names key row q, d columns 4p..4p+3
  const int grp = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int v_key = 8 * (grp >> 1) + q4;
  const int v_ch = 2 * (grp & 1) + (p4 >> 1), v_sub = 8 * (p4 & 1);

  // split s: tiles s, s + 2, ...; every split runs the same iteration count (block-wide barriers)
  constexpr int DEPTH = FC::DEPTH;
  const int iters = (nt + NS - 1) / NS;
  if (split < nt) {
    load_tile(split * kFK, kra, vra);
    store_tile(0, kra, vra);
    if (split + NS < nt) load_tile((split + NS) * kFK, DEPTH == 2 ? krb : kra, DEPTH == 2 ? vrb : vra);
    if (DEPTH == 2 && split + 2 * NS < nt) load_tile((split + 2 * NS) * kFK, kra, vra);
  }
  __syncthreads();
  bool first = true;
  // iteration `it` computes this split's local tile it from LDS stage it & 1, then stages local
  // tile it + 1 (held in register set S) and refills S with local tile it + 1 + DEPTH
  auto body = [&](int it, uint4 (&SK)[LPT], uint4 (&SV)[LPT]) {
    const int t = it * NS + split;
    if (t < nt) {
      const int k0 = t * kFK;
      const unsigned char* kimg = simg + (2 * (it & 1)) * IMG;
      const unsigned char* vimg = kimg + IMG;
      // (LDS fragments are read next to their MFMAs.  A D = 64 form that requested all of a tile's
      // K and V^T fragments up front -- 64 VGPRs -- gave results that varied by 1-2 bf16 ulps from
      // run to run (tools/repro_ops.py: 5 variants in 5 runs of the same inputs) and was no faster
      // end to end: Whisper-large-v3 encoder 3.14-3.35 vs 3.37-3.52 ms; removed)
      // ---- S^T = K.Q^T
      f32x16 s[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kk][i] = 0.f;
        const int row = 32 * kk + a_key;
#pragma unroll
        for (int ds = 0; ds < NDS; ++ds) {
          const uint4 a = *reinterpret_cast<const uint4*>(kimg + FC::off(row, 2 * ds + hf));
          s[kk] = mfma32(as_bf16x8(a), qf[ds], s[kk]);
        }
      }
      // ---- mask (only tiles that reach past Sk or the wave's first causal row)
      const bool edge = (k0 + kFK > Sk) || (CAUSAL && k0 + kFK - 1 > qoff + qw0);
      if (edge) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = k0 + 32 * kk + (i & 7) + 16 * (i >> 3) + 8 * hf;
            if (key >= Sk || (CAUSAL && key > qpos)) s[kk][i] = -INFINITY;
          }
      }
      float tm0 = vmax3(s[0][0], s[0][1], s[0][2]), tm1 = vmax3(s[1][0], s[1][1], s[1][2]);  // two chains
#pragma unroll
      for (int i = 3; i < 15; i += 2) {
        tm0 = vmax3(tm0, s[0][i], s[0][i + 1]);
        tm1 = vmax3(tm1, s[1][i], s[1][i + 1]);
      }
      const float tmax = max_halves(vmax3(tm0, tm1, vmax3(s[0][15], s[1][15], s[1][15])));
      // ---- deferred rescale: the split's first tile with a visible key sets the max (a causal tile
      // may leave a row without one: -inf contributes nothing); later tiles move it only when their
      // max exceeds it by more than kRescale
      const bool move = (first && tmax != -INFINITY) || (tmax - m_run > kRescale);
      if (__any(move)) {
        const float m_new = move ? tmax : m_run;
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        m_run = m_new;
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) oacc[dt] *= alpha;
      }
      first = first && tmax == -INFINITY;  // per lane: until a visible key
      // ---- P^T = exp2(S - m), packed bf16 per 16-key slice; row sums in f32 (4 partial sums)
      float ls[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 pb[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          float pf[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            pf[j] = __builtin_amdgcn_exp2f(s[kk][8 * ks + j] - m_run);
            ls[j & 3] += pf[j];
          }
          pb[ks] = as_bf16x8(pack8(pf));
        }
        // ---- O^T += V^T.P^T
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int kr0 = 32 * kk + 16 * ks + v_key;
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) {
            const int ch = 4 * dt + v_ch;
            const uint2 lo = lds_tr16(vimg + FC::off(kr0, ch) + v_sub);
            const uint2 hi = lds_tr16(vimg + FC::off(kr0 + 4, ch) + v_sub);
            oacc[dt] = mfma32(as_bf16x8(make_uint4(lo.x, lo.y, hi.x, hi.y)), pb[ks], oacc[dt]);
          }
        }
      }
      l_run += (ls[0] + ls[1]) + (ls[2] + ls[3]);
      if (t + NS < nt) {
        store_tile((it + 1) & 1, SK, SV);
        if (t + (DEPTH + 1) * NS < nt) load_tile((t + (DEPTH + 1) * NS) * kFK, SK, SV);
      }
    }
    __syncthreads();
  };
  if constexpr (DEPTH == 2) {
    for (int it = 0; it < iters; it += 2) {  // local tile it + 1 sits in B when it is even
      body(it, krb, vrb);
      if (it + 1 < iters) body(it + 1, kra, vra);
    }
  } else {
    for (int it = 0; it < iters; ++it) body(it, kra, vra);
  }

  // ---- merge the key splits through LDS (the tile images are free after the last barrier):
  // splits 1.. publish (m, l, O^T) per lane, split 0 combines and stores
  constexpr int MO = 64 * (NDT * 16 + 2);  // floats per (split, query wave)
  static_assert((NS - 1) * 4 * MO * 4 <= NS * 2 * 2 * IMG, "merge area fits the tile images");
  float* mo_base = reinterpret_cast<float*>(smem) + w * MO;
  if (split > 0) {
    float* mo = mo_base + (split - 1) * 4 * MO;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mo[(dt * 16 + i) * 64 + lane] = oacc[dt][i];
    mo[(NDT * 16) * 64 + lane] = first ? -INFINITY : m_run;  // a split that saw no key adds nothing
    mo[(NDT * 16 + 1) * 64 + lane] = l_run;
  }
  __syncthreads();
  if (split > 0) return;
  {
    float M = first ? -INFINITY : m_run;
#pragma unroll
    for (int sp = 1; sp < NS; ++sp) M = fmaxf(M, mo_base[(sp - 1) * 4 * MO + (NDT * 16) * 64 + lane]);
    const float a0 = __builtin_amdgcn_exp2f((first ? -INFINITY : m_run) - M);
    l_run *= a0;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) oacc[dt] *= a0;
#pragma unroll
    for (int sp = 1; sp < NS; ++sp) {
      const float* mo = mo_base + (sp - 1) * 4 * MO;
      const float a1 = __builtin_amdgcn_exp2f(mo[(NDT * 16) * 64 + lane] - M);
      l_run += mo[(NDT * 16 + 1) * 64 + lane] * a1;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) oacc[dt][i] += mo[(dt * 16 + i) * 64 + lane] * a1;
    }
  }

  // ---- epilogue: lane (col, hf) holds O^T[d][qi] for d = 32dt + (i&3) + 8(i>>2) + 4hf
  const float l_tot = sum_halves(l_run);
  if (qi < p.Sq) {
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    u16* orow = p.o + (int64_t)b * p.o_stride_b + (int64_t)qi * p.o_stride_s + (int64_t)h * p.o_stride_h;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        uint2 v;
        v.x = pack2(oacc[dt][4 * g] * inv, oacc[dt][4 * g + 1] * inv);
        v.y = pack2(oacc[dt][4 * g + 2] * inv, oacc[dt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * g + 4 * hf) = v;
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
  if (p->B <= 0 || p->Sq <= 0) return 0;
  dim3 grid(((p->Sq + kFQ - 1) / kFQ) * p->n_q_heads * p->B);
  if (p->head_dim == 128) {
    const dim3 block(256 * FlashCfg<128>::NS);
    if (p->causal) hipLaunchKernelGGL((flash_attn_kernel<128, true>), grid, block, flash_lds<128>(), st, *p);
    else hipLaunchKernelGGL((flash_attn_kernel<128, false>), grid, block, flash_lds<128>(), st, *p);
  } else if (p->head_dim == 64) {
    const dim3 block(256 * FlashCfg<64>::NS);
    if (p->causal) hipLaunchKernelGGL((flash_attn_kernel<64, true>), grid, block, flash_lds<64>(), st, *p);
    else hipLaunchKernelGGL((flash_attn_kernel<64, false>), grid, block, flash_lds<64>(), st, *p);
  } else {
    return -3;
  }
  return (int)hipGetLastError();
}

// chunk granularity of the decode grid (grid.y = ceil(max_ctx / this)); the split kernel's
// 256-key chunks use every other grid row
extern "C" int vwa_attention_split_tokens() { return kMqChunk; }
