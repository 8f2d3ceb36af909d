// Multi-query MFMA decode attention body + the paged-KV / sc1 helpers it uses, shared by the
// standalone decode kernel (attention.hip) and the chained decode-layer launch (skinny_stream.hip).
#pragma once
#include "common.h"
#include "vwa_kernels.h"

namespace {
using namespace vwa;

typedef __attribute__((address_space(1))) const int gint;  // global-space loads: vmcnt only (ld128)
VWA_DEVICE int64_t kv_offset(const KVView& kv, int seq, int kvh, int t) {
  const int blk = *(gint*)(kv.block_table + (int64_t)seq * kv.table_stride + t / kv.block_size);
  return (int64_t)blk * kv.stride_block + (int64_t)kvh * kv.stride_head + (int64_t)(t % kv.block_size) * kv.stride_tok;
}

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
// Through the GLOBAL address space: a flat (generic) load also counts on lgkmcnt, so every wait
// for an LDS op or a lane shuffle after it (the block-id shuffles of the next key's address) also
// waited for all K/V loads in flight -- the chained attention's 16 K/V loads per wave measured as
// ~5 serialized round trips (6.6 us; the same gather alone: 1.2 us, tools/latency_probe.hip)
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
VWA_DEVICE uint4 ld128(const u16* ptr) {
  const u32x4 v = *(gu32x4*)(ptr);
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
    __hip_atomic_store(gp(reinterpret_cast<unsigned long long*>(dst)), (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gp(reinterpret_cast<unsigned long long*>(dst) + 1), (unsigned long long)v.z | ((unsigned long long)v.w << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *gp(reinterpret_cast<u32x4*>(dst)) = u32x4{v.x, v.y, v.z, v.w};
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
// written with sc1 stores (read by another workgroup later in the same launch).  DB: K/V of the
// next 32-key step loaded while the current one computes (two register sets).
struct NoIdle {
  VWA_DEVICE void operator()() const {}
};
struct NoStamp {
  VWA_DEVICE void operator()(int) const {}
};

// Returns true when this workgroup had no item (after calling on_idle(), before any barrier).
// FINE (the chained launch's attention phase): chunks are multiples of ONE 32-key step, the
// steps of a chunk go to the waves round-robin, and the last arriver merges the chunks with two
// threads per (query column, 8-dim slice), every partial load issued before any is used.  A lone
// decode row then spreads its context over up to n_splits chunks (1100 keys: 12 workgroups of 96
// keys per kv head instead of 5 of 256) -- the phase is latency-bound, each workgroup's K/V bytes
// are its critical path.
// n_items_out (optional): the step's attention item count (the same in every workgroup), set
// before on_idle runs.
// stamp(k) (diagnostic, tools/chain_probe.py --attn): in-body timestamps 9..14 of the first item
// done (optional, the chained launch's attention -> o_proj hand-off): after a (row group, kv
// head)'s final output is stored and drained, one no-return add of 1 to *done -- the consumers
// wait for *n_final_out of them instead of a grid barrier.
// on_kv (optional, single-register-set form): called once per wave of a workgroup WITH an item,
// after the wave's key steps (at once for a wave without one) and before the merge -- the chained
// launch issues a weight item of a later phase there, so the attention workgroups' memory pipe is
// not idle through the attention's merge (and, for the waves without a key step, all of it).
template <int D, int G, int NW, bool SC1OUT, bool DB = true, bool FINE = false, class OnIdle = NoIdle,
          class Stamp = NoStamp, class OnKv = NoIdle>
VWA_DEVICE bool mq_body(const DecodeAttnParams& p, unsigned char* lds, int grid, int bid, OnIdle on_idle = {},
                        int* n_items_out = nullptr, Stamp stamp = {}, unsigned long long* done = nullptr,
                        int* n_final_out = nullptr, OnKv on_kv = {}) {
  constexpr int kWv = NW;
  constexpr int kChunk = FINE ? kMqStep : NW * kMqStep;  // chunk granularity (keys)
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
  const int lane = VWA_TX & 63, w = VWA_TX >> 6;
  const int n = lane & 15, g = lane >> 4;

  // ---- row groups of the whole step (<= 64 rows; every wave derives the same answer): runs of
  //      consecutive rows of one sequence, cut every RG rows from the run's start
  // per-row block tables (FINE, <= 4 rows): fetched with the sequence ids, two entries per lane
  // All of it in ONE round trip: branch-free buffer loads (past the end -> 0).  (The conditional
  // plain loads this replaces compiled to a wait after each load: five dependent round trips.)
  // FINE (the chained launch, <= 4 rows) always has them (chain_make requires a_row_table):
  // K/V addresses come from lane shuffles only, no table loads whose waits the K/V loads share
  constexpr bool rowtab = FINE;
  const __amdgpu_buffer_rsrc_t r_rt = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int*>(p.row_table), (short)0, rowtab ? p.rows * p.rt_stride * 4 : 0, 0x00020000);
  // Loaded by wave 0 only and shared through LDS (the start of the V-image area, free until the
  // first item's __syncthreads): every wave of every workgroup asking for the same few lines at
  // the launch's start is 8x the requests on the same L2 lines.  (In the first 2.5 KB: the chained
  // launch's idle workgroups LDS-DMA weights above 32 KB while other waves may still read it.)
  int* s_meta = reinterpret_cast<int*>(lds + L::vimg);  // [4][128] row tables | [64] seq ids | [64] contexts
  // ---- step plan (FINE, p.plan_mode 2): the partition depends only on the step's rows and
  //      contexts, the same for every layer, so the chained launch of layer 0 writes each
  //      workgroup's item (plan_mode 1) and layers 1.. load it -- with the row tables, in one round
  //      trip, every wave for itself: no metadata through LDS, no barrier, no ballots before the
  //      K/V loads.  Entry (16 ints): n_items, n_final, state (0 idle, 1 item, 2 empty chunk, 3 no
  //      plan: several items per workgroup), kv head, r0, nr, kbeg, kend, nact, slot, rows, -,
  //      contexts of group rows 0..3.  An entry of another row count is ignored.
  int2 rt[4];
  int ev = 0;
  bool plan = false;
  if constexpr (FINE) {
    if (p.plan_mode == 2) {
      const __amdgpu_buffer_rsrc_t r_pl = __builtin_amdgcn_make_buffer_rsrc(p.plan, (short)0, (bid + 1) * 64, 0x00020000);
      ev = (int)__builtin_amdgcn_raw_buffer_load_b32(r_pl, (bid * 16 + (lane & 15)) * 4, 0, 16);  // (sc1: written this launch)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        rt[r] = __builtin_bit_cast(int2, __builtin_amdgcn_raw_buffer_load_b64(
                                             r_rt, 2 * lane < p.rt_stride ? (r * p.rt_stride + 2 * lane) * 4 : 0x7FFFFFF0, 0, 0));
      plan = __builtin_amdgcn_readlane(ev, 2) != 3 && __builtin_amdgcn_readlane(ev, 10) == p.rows;
    }
  }
  if (w == 0 && !plan) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<int2*>(s_meta + r * 128 + 2 * lane) = __builtin_bit_cast(
          int2, __builtin_amdgcn_raw_buffer_load_b64(
                    r_rt, 2 * lane < p.rt_stride ? (r * p.rt_stride + 2 * lane) * 4 : 0x7FFFFFF0, 0, 0));
    const __amdgpu_buffer_rsrc_t r_sid =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.seq_ids), (short)0, p.rows * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t r_ctx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.ctx_lens), (short)0, p.rows * 4, 0x00020000);
    s_meta[512 + lane] = (int)__builtin_amdgcn_raw_buffer_load_b32(r_sid, lane * 4, 0, 0);
    s_meta[576 + lane] = (int)__builtin_amdgcn_raw_buffer_load_b32(r_ctx, lane * 4, 0, 0);
    if constexpr (!FINE) {
      const __amdgpu_buffer_rsrc_t r_sh =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(p.shared), (short)0, p.shared ? 8 : 0, 0x00020000);
      if (lane < 2) s_meta[640 + lane] = (int)__builtin_amdgcn_raw_buffer_load_b32(r_sh, lane * 4, 0, 0);
    }
  }
  if (!plan) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) rt[r] = *reinterpret_cast<const int2*>(s_meta + r * 128 + 2 * lane);
  }
  stamp(12);  // (diagnostic: step metadata in LDS / the plan entry in registers)
  const int sl = plan ? -1 : lane < p.rows ? s_meta[512 + lane] : -1;
  const int cl = plan ? 0 : lane < p.rows ? s_meta[576 + lane] : 0;
  stamp(16);
  const int sp = __shfl(sl, lane > 0 ? lane - 1 : 0, 64);
  const unsigned long long seq_starts = __ballot(lane < p.rows && (lane == 0 || sl != sp));
  // shared cached prefix (p.shared): rows 0 .. n_real-1 are grouped RG at a time regardless of
  // sequence (their first P keys are the same blocks), the padded rows behind them by sequence
  int P = 0, n_real = p.rows;
  if constexpr (!FINE) {
    P = s_meta[640];
    n_real = min(p.rows, s_meta[641]);
  }
  const bool cascade = !FINE && P > 0 && n_real > 0 && p.n_splits > RG;
  unsigned long long run_starts = seq_starts;
  if (cascade) {
    const unsigned long long real = n_real >= 64 ? ~0ull : ((1ull << n_real) - 1ull);
    run_starts = 1ull | (n_real < p.rows ? (1ull << n_real) : 0ull) | (seq_starts & ~real);
  }
  const int run0 = 63 - __builtin_clzll(run_starts & ((2ull << lane) - 1ull));  // lane 0 always starts a run
  const unsigned long long leaders = __ballot(lane < p.rows && (lane - run0) % RG == 0);
  const int n_groups = __builtin_popcountll(leaders);
  const int my_rank = __builtin_popcountll(leaders & ((1ull << lane) - 1ull));
  // chunks per (group, kv head): spread the work over the grid (one item per workgroup when it
  // fits), never more than the partial buffers hold
  static_assert(!FINE || NW == 8, "the FINE merge pairs two threads per (column, slice): 512 threads");
  // cascade: n_pc prefix chunks + up to RG own-key chunks (one per sequence run of the group) per
  // group -- the partial slots 0 .. n_pc + RG - 1
  // (standalone kernel: about one item per CU -- grid / 2 -- measured best over the chunk cap,
  // tools/attn_probe.py --split-sweep, profiles/r4_attn_split_sweep.jsonl: e.g. 8 sessions 14.5 vs
  // 21.2 us with a full-grid split, 16 grouped sessions 14.7 vs 23.2 us)
  const int tgt = FINE ? grid : max(1, grid / 2);
  const int n_pc = cascade ? max(1, min(p.n_splits - RG, tgt / max(1, n_groups * nkv) - RG)) : 0;
  const int n_eff = cascade ? n_pc + RG : max(1, min(FINE ? min(p.n_splits, 16) : p.n_splits, tgt / max(1, n_groups * nkv)));
  const int n_items = plan ? __builtin_amdgcn_readlane(ev, 0) : n_groups * nkv * n_eff;
  if (n_items_out) *n_items_out = n_items;
  if (n_final_out) *n_final_out = plan ? __builtin_amdgcn_readlane(ev, 1) : n_groups * nkv;
  stamp(17);
  // plan_mode 1: lanes 0..15 of wave 0 write this workgroup's entry (c: the group rows' contexts
  // in lanes 0..3)
  const bool multi = n_items > grid;
  auto write_plan = [&](int st, int kvh, int r0, int nr, int kbeg, int kend, int nact, int slot, int c) {
    if (!FINE || p.plan_mode != 1 || w != 0) return;
    const int cr = __shfl(c, lane & 3, 64);
    const int i = lane & 15;
    const int v = i == 0 ? n_items : i == 1 ? n_groups * nkv : i == 2 ? (multi ? 3 : st) : i == 3 ? kvh : i == 4 ? r0
                : i == 5 ? nr : i == 6 ? kbeg : i == 7 ? kend : i == 8 ? nact : i == 9 ? slot : i == 10 ? p.rows
                : i == 11 ? 0 : cr;
    if (lane < 16) p.plan[bid * 16 + i] = v;
  };
  if (bid >= n_items) {
    write_plan(0, 0, 0, 0, 0, 0, 0, 0, 0);
    on_idle();
    return true;
  }

  // a (group, kv head)'s final output is complete once every thread's stores drained
  auto publish = [&]() {
    if (done == nullptr) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (VWA_TX == 0) __hip_atomic_fetch_add(gp(done), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  for (int item = bid; item < n_items; item += grid) {
  if (item == bid) stamp(18);
  int kvh, r0, nr, CL, kbeg, kend, nact, slot, kv_seq, ctx_n;
  const int rho = n / G;  // group row of this lane's query column
  if (plan) {  // (one item per workgroup)
    if (__builtin_amdgcn_readlane(ev, 2) != 1) continue;  // empty chunk
    kvh = __builtin_amdgcn_readlane(ev, 3);
    r0 = __builtin_amdgcn_readlane(ev, 4);
    nr = __builtin_amdgcn_readlane(ev, 5);
    kbeg = __builtin_amdgcn_readlane(ev, 6);
    kend = __builtin_amdgcn_readlane(ev, 7);
    nact = __builtin_amdgcn_readlane(ev, 8);
    slot = __builtin_amdgcn_readlane(ev, 9);
    CL = kend - kbeg;
    kv_seq = 0;
    const int c_rho = __shfl(ev, 12 + min(rho, 3), 64);  // (rho differs per lane: a shuffle)
    ctx_n = rho < nr ? c_rho : 0;
  } else {
  // item -> (kv head, group, chunk); kv head fastest so a head's workgroups share one XCD (b % 8)
  kvh = item % nkv;
  const int gi = (item / nkv) % n_groups, chunk = item / (nkv * n_groups);
  const unsigned long long pick = __ballot(((leaders >> lane) & 1ull) && my_rank == gi);
  r0 = __builtin_ctzll(pick);
  const unsigned long long later = run_starts & ~((2ull << r0) - 1ull);
  const int run_end = later ? __builtin_ctzll(later) : p.rows;
  nr = min(RG, run_end - r0);  // rows in this group
  const int seq = __shfl(sl, r0, 64);
  if (item == bid) stamp(11);  // (diagnostic: before the item's barrier)
  __syncthreads();  // the previous item's LDS readers are done
  if (item == bid) stamp(9);  // step rows / contexts known
  const int c_src = __shfl(cl, min(r0 + lane, 63), 64);
  const int c_own = lane < nr ? c_src : 0;
  int ctxmax = c_own;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) ctxmax = max(ctxmax, __shfl_xor(ctxmax, o, 64));
  if (item == bid) stamp(19);
  ctx_n = __shfl(c_own, rho, 64);  // its context (0 for padded columns)

  // ---- this item's chunk of the group's keys (NW waves x CL/NW keys): [kbeg, kend), partial slot
  slot = chunk;
  kv_seq = seq;
  if (cascade && r0 < n_real) {
    // prefix chunks (slots 0 .. npa-1) over [0, P) for every row of the group; then one chunk per
    // sequence run j of the group with keys past P: [P, max ctx of the run), the other runs'
    // columns masked (slot npa + its rank among such runs)
    const unsigned long long gm = (nr >= 64 ? ~0ull : ((1ull << nr) - 1ull)) << r0;
    const unsigned long long subs = (seq_starts & gm) | (1ull << r0);
    const int run_of = __builtin_popcountll(subs & ((2ull << min(r0 + lane, 63)) - 1ull)) - 1;  // lane < nr
    const int nruns = __builtin_popcountll(subs);
    int own_mask = 0, my_max = 0;  // runs with own keys; this item's run's max context
    const int j = chunk - n_pc;
    for (int rr = 0; rr < nruns; ++rr) {
      int cm = (lane < nr && run_of == rr) ? c_src : 0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) cm = max(cm, __shfl_xor(cm, o, 64));
      if (cm > P) own_mask |= 1 << rr;
      if (rr == j) my_max = cm;
    }
    CL = ((P + n_pc - 1) / n_pc + kChunk - 1) / kChunk * kChunk;
    const int npa = (P + CL - 1) / CL;
    nact = npa + __builtin_popcount(own_mask);
    if (chunk < n_pc) {
      kbeg = chunk * CL;
      if (kbeg >= P) continue;
      kend = min(P, kbeg + CL);
    } else {
      if (j >= nruns || !((own_mask >> j) & 1)) continue;
      unsigned long long sb = subs;
      for (int t = 0; t < j; ++t) sb &= sb - 1ull;  // drop the first j run starts
      const int a = __builtin_ctzll(sb);
      sb &= sb - 1ull;
      const int b = sb ? __builtin_ctzll(sb) : r0 + nr;
      kbeg = P;
      kend = my_max;
      CL = (kend - kbeg + kChunk - 1) / kChunk * kChunk;
      slot = npa + __builtin_popcount(own_mask & ((1 << j) - 1));
      kv_seq = __shfl(sl, a, 64);
      if (rho < a - r0 || rho >= b - r0) ctx_n = 0;  // other runs' columns: no keys in this chunk
    }
  } else {
    CL = ((ctxmax + n_eff - 1) / n_eff + kChunk - 1) / kChunk * kChunk;
    if (cascade) CL = (ctxmax + kChunk - 1) / kChunk * kChunk;  // padded rows: one chunk
    kbeg = chunk * CL;
    if (kbeg >= ctxmax) {
      if (item == bid) write_plan(2, 0, 0, 0, 0, 0, 0, 0, 0);
      continue;
    }
    kend = min(ctxmax, kbeg + CL);
    nact = (ctxmax + CL - 1) / CL;
  }
  if (item == bid) write_plan(cascade ? 3 : 1, kvh, r0, nr, kbeg, kend, nact, slot, c_own);
  }  // (metadata path)
  // non-FINE: wave w takes the contiguous CL / NW keys from wb; FINE: the chunk's 32-key steps
  // round-robin over the waves (step s of the chunk -> wave s % NW)
  const int wb = FINE ? kbeg : kbeg + w * (CL / kWv);
  const int we = FINE ? kend : min(kend, wb + CL / kWv);
  const int nsteps = we > wb ? (we - wb + kMqStep - 1) / kMqStep : 0;
  const int kmax = kend - 1;  // keys past the chunk are clamped (finite data, masked scores)
  if (item == bid) stamp(20);

  // ---- Q^T fragments (B operand): Q[column n][dims 32ks + 8g ..], pre-scaled by scale*log2(e)
  bf16x8 qf[NKS];
  auto make_qf = [&]() {
    const float qs = p.scale * 1.4426950408889634f;
    const int64_t qo = (int64_t)(r0 + min(rho, nr - 1)) * p.ldq + (kvh * G + n % G) * D + 8 * g;
    // FINE (the chained launch): Q is written by the QKV phase of the same launch when several
    // layers run in one launch (chain_kernel MULTI), possibly on another XCD whose L2 line this
    // XCD may hold from the previous layer's attention: device-scope (sc1) loads
    const __amdgpu_buffer_rsrc_t r_q = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<u16*>(p.q), (short)0, FINE ? (int)((int64_t)p.rows * p.ldq * 2) : 0, 0x00020000);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      float f[8];
      if constexpr (FINE) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r_q, (int)((qo + 32 * ks) * 2), 0, 16);
        unpack8(make_uint4(v.x, v.y, v.z, v.w), f);
      } else {
        unpack8(ld128(p.q + qo + 32 * ks), f);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = rho < nr ? f[j] * qs : 0.f;
      qf[ks] = as_bf16x8(pack8(f));
    }
  };
  if constexpr (DB) {
    make_qf();
    if (item == bid) stamp(10);  // q fragments in registers
  }
  // (measured: staging the wave's block-table entries in lanes and fetching them with __shfl,
  // instead of the per-key table loads below, was 1.5-3 us SLOWER on every shape)
  const int2 rtr = r0 == 0 ? rt[0] : r0 == 1 ? rt[1] : r0 == 2 ? rt[2] : rt[3];  // the group's row table

  // K: A-operand row n of tile t is key kb + 8(n>>2) + 4t + (n&3) (so the S^T accumulator of lane
  // (n, g) holds keys kb + 8g + 4t + i); V: 32 rows x NCH chunks, chunk idx = i*64 + lane
  // every address first (block ids: row-table shuffles or one round of table loads), then all 16
  // loads back to back -- no wait between them
  // (the two block-id sources in separate uniform branches, each finishing its offsets: a shared
  // helper left a vmcnt(0) at every join, which also waited for the Q loads in flight)
  auto load_step = [&](int kb, uint4 (&kr)[2][NKS], uint4 (&vr)[NVL]) {
    int64_t ko[2], vo[NVL];
    auto offsets = [&](auto off) {
#pragma unroll
      for (int t = 0; t < 2; ++t) ko[t] = off(min(kb + 8 * (n >> 2) + 4 * t + (n & 3), kmax));
#pragma unroll
      for (int i = 0; i < NVL; ++i) vo[i] = off(min(kb + (i * 64 + lane) / NCH, kmax));
    };
    if constexpr (rowtab) {
      // 16-key blocks (chain_make checks) and a step start kb that is a multiple of 32: the step
      // spans exactly blocks kb/16 (even: entry .x) and kb/16 + 1 (.y) of one row-table lane, two
      // wave-uniform block ids read straight into scalars -- per key only a select and a multiply
      // (the per-key shuffles and 64-bit products before measured ~1 us of issue per step)
      const int tl = kb >> 5;
      const int64_t bA = (int64_t)__builtin_amdgcn_readlane(rtr.x, tl) * p.kv.stride_block,
                    bB = (int64_t)__builtin_amdgcn_readlane(rtr.y, tl) * p.kv.stride_block;
      const int64_t hoff = (int64_t)kvh * p.kv.stride_head;
      const int st = (int)p.kv.stride_tok;
      offsets([&](int key) -> int64_t { return ((key & 16) ? bB : bA) + hoff + (key & 15) * st; });
    } else {
      offsets([&](int key) -> int64_t { return kv_offset(p.kv, kv_seq, kvh, key); });
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) kr[t][ks] = ld128(p.kv.k + ko[t] + 8 * g + 32 * ks);
#pragma unroll
    for (int i = 0; i < NVL; ++i) vr[i] = ld128(p.kv.v + vo[i] + 8 * ((i * 64 + lane) % NCH));
  };

  float m_run = -INFINITY, l_run = 0.f;  // per query column (log2 units); l is this lane's share
  f32x4 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned char* vi = lds + L::vimg + w * kMqStep * 256;
  if (item == bid) stamp(21);

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

  if constexpr (DB) {
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
  } else {  // single register set (the chained launch holds the next GEMM's weights meanwhile)
    // the first step's K/V loads go out before the Q fragments are built (Q's round trip and
    // scaling overlap the K/V round trip)
    bool have_q = false;
    for (int s = FINE ? w : 0; s < nsteps; s += FINE ? kWv : 1) {
      uint4 kA[2][NKS], vA[NVL];
      if (item == bid && s == w) stamp(13);  // (diagnostic: about to issue the first K/V step)
      load_step(wb + s * kMqStep, kA, vA);
      if (!have_q) {
        make_qf();
        have_q = true;
      }
      if (item == bid && s == w) stamp(15);  // (diagnostic stamp 15: the wave's first K/V step landed)
      compute_step(wb + s * kMqStep, kA, vA);
    }
    // (after the wave's key steps: their K/V registers are free -- issued inside the loop the item
    // kept 64 more VGPRs live through the attention and spilled; a wave without a key step, most
    // of them at one row, issues at once and streams through the whole attention)
    if (item == bid) on_kv();
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
  const int cn = VWA_TX >> 4, dc = VWA_TX & 15;
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
      const int64_t base = ((int64_t)crow * p.n_splits + slot) * nq + ch;
      st_sc1_f4(r_o, base * D + 8 * dc, acc);
      st_sc1_f4(r_o, base * D + 8 * dc + 4, acc + 4);
      if (dc == 0) st_sc1_f2(r_ml, base * 2, M, L);
    }
  }
  if (nact == 1) {
    publish();
    continue;
  }

  // ---- ticket (same protocol as the split kernel): drained sc1 stores, then one counter add
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (VWA_TX == 0) {
    int* cnt = p.counters + r0 * nkv + kvh;
    const int ticket = __hip_atomic_fetch_add(gp(cnt), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = (ticket == nact - 1);
    if (last) __hip_atomic_store(gp(cnt), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) continue;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // only orders the sc1 loads after the ticket

  if constexpr (FINE) {
    // ---- last arriver, FINE: two threads per (column, 8-dim slice) pair, each merging every
    //      other chunk with all of its (<= n_splits / 2) partial loads in flight at once (clamped
    //      indices, zero weight past nact), then the two halves combine through LDS
    constexpr int MAXC = 8;  // chunks per thread: nact <= 2 * MAXC (host: n_splits <= 16)
    const int pr = VWA_TX & 255, hf = VWA_TX >> 8;
    const int pcn = pr >> 4, pdc = pr & 15;
    const int prow = r0 + pcn / G, pch = kvh * G + pcn % G;
    const bool pact = pcn / G < nr && pdc < NCH;
    float pm = -INFINITY, pl = 0.f, pacc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) pacc[j] = 0.f;
    if (pact) {
      const int64_t hb = (int64_t)prow * p.n_splits * nq + pch;
      float2 ml[MAXC];
      float4 x0[MAXC], x1[MAXC];
#pragma unroll
      for (int i = 0; i < MAXC; ++i) {
        const int c = min(hf + 2 * i, nact - 1);
        const int64_t b = hb + (int64_t)c * nq;
        ml[i] = ld_sc1_f2(r_ml, b * 2);
        x0[i] = ld_sc1_f4(r_o, b * D + 8 * pdc);
        x1[i] = ld_sc1_f4(r_o, b * D + 8 * pdc + 4);
      }
#pragma unroll
      for (int i = 0; i < MAXC; ++i)
        if (hf + 2 * i < nact) pm = fmaxf(pm, ml[i].x);
#pragma unroll
      for (int i = 0; i < MAXC; ++i) {
        const float f = (hf + 2 * i < nact && ml[i].x != -INFINITY) ? exp2f(ml[i].x - pm) : 0.f;
        pl += ml[i].y * f;
        pacc[0] += x0[i].x * f; pacc[1] += x0[i].y * f; pacc[2] += x0[i].z * f; pacc[3] += x0[i].w * f;
        pacc[4] += x1[i].x * f; pacc[5] += x1[i].y * f; pacc[6] += x1[i].z * f; pacc[7] += x1[i].w * f;
      }
    }
    float* xm = ow;  // reuse the per-wave O^T area: [256 pairs][10] floats of the second half
    if (hf == 1) {
      xm[pr * 10 + 0] = pm;
      xm[pr * 10 + 1] = pl;
#pragma unroll
      for (int j = 0; j < 8; ++j) xm[pr * 10 + 2 + j] = pacc[j];
    }
    __syncthreads();
    if (hf == 0 && pact) {
      const float om = xm[pr * 10 + 0];
      const float M = fmaxf(pm, om);
      const float fa = pm == -INFINITY ? 0.f : exp2f(pm - M), fb = om == -INFINITY ? 0.f : exp2f(om - M);
      const float L = pl * fa + xm[pr * 10 + 1] * fb;
      const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) pacc[j] = (pacc[j] * fa + xm[pr * 10 + 2 + j] * fb) * inv;
      store_out<SC1OUT>(p.out + (int64_t)prow * p.ldo + pch * D + 8 * pdc, pack8(pacc));
    }
    if (item == bid) stamp(14);  // merged output stored (issued)
    publish();
    continue;
  }
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
  publish();
  }  // items
  return false;
}

}  // namespace
