// Persistent Whisper decoder step (any Whisper width: d a multiple of 128 up to 1536, ffn = 4 d,
// head_dim 64 -- tiny 384 .. large 1280), one row: ONE launch for the whole token step -- the
// embedding (layer 0 builds it from the tables), every decoder layer, the LM head (a last level
// streaming the vocabulary tiles through the slots) and, in the device loop, the greedy masked
// argmax + the loop advance (workgroup 0 merges the workgroups' partials).
//
// Why: the per-kernel decoder runs eight dependent launches per
// layer, each ~5-9 us of fixed latency (dispatch, X staging, the first weight bytes, reduce,
// epilogue) for 0.3-13 MB of weights -- 2.3 ms per token for ~1.6 GB, 7x off the HBM roofline.
// Here a workgroup's share of the NEXT use of each of its weight tiles is already in its registers
// (refilled right after the level that consumed it), so a level's critical path is the hand-off of
// the activation row (a few KB through the MALL) and a few MFMAs.
//
// Levels of layer li (reference call site this replaces: /root/reference/apps/voice/src/
// deepgram.ts:36-45, the hosted recogniser):
//   0 QKV      LN1(x) . Wqkv^T + b -> q, self K / V cache row   (240 column tiles of 16)
//   1 XQX      x . Wxq^T -> xqa (f32)                             (80 tiles; off the critical path)
//   2 SATT     self-attention of the row, one workgroup per head -> att
//   3 OXQ      x1 = x + att . Wo^T + bo                           (80 tiles)
//              att . (Wxq Wo)^T + Wxq bo -> xqb (f32)             (80 tiles, same staged row)
//   4 XATT     q = LNx(x1) . Wxq^T + b from xqa + xqb and x1's mean / rstd (the out-proj tiles'
//              sums), then the cross-attention partials, (head, key chunk) per workgroup, K / V
//              chunk prefetched into LDS by LDS-DMA a layer ahead
//   5 XO       x2 = x1 + merge(partials) . Wxo^T + b              (80 tiles; the merge is the X staging)
//   6 FC1      f = GELU(LN2(x2) . W1^T + b1)                      (320 tiles)
//   7 FC2      x3 = x2 + f . W2^T + b2                            (80 tiles, K = 5120)
// (tile counts for whisper-large; QKV -> SATT optionally through per-head counters, kOptQkvByHead)
// LayerNorms are folded into the weights (ops.fold_layernorm: y = rstd (x.Wg - mean c) + b'), the
// mean / rstd come from the staged row.  The cross query needs x1 = x + att Wo^T + bo, so by
// linearity x1 Wg^T = x Wg^T + att (Wg Wo)^T + Wg bo: its x part runs while the self-attention
// does (level 1, the row QKV staged) and its att part beside the out-projection -- one dependent
// level per layer fewer than out-proj -> cross query -> cross-attention (the x1 rounding to bf16
// is the only difference; the extra 3.3 MB per layer fits the register slots).
//
// Hand-off: a producer workgroup drains its stores and adds 1 (no return) to its level's counter of
// its XCD group; consumers poll the sum of the eight group counters with scalar loads (uncached
// words: the poll does not queue behind vector loads).  Counters are monotonic: a launch adds
// n_prod[level] x n_layers to each, so every workgroup derives the launch's base from the value it
// reads at its start.  (Measured and not kept: values tagged with their (launch, layer, level) and
// the counter add issued without the store drain -- consumers then re-polled for the same store
// latency and the cross merge polled word by word: 38.2 vs 36.5 us per layer, tools/wdec_probe.py.)

// Weight slots: 5 slots x 5 loads of 1 KB per wave (100 VGPRs).  A 16-column tile of a K = 1280
// projection is 40 load-slices (k-group, 32-k slice) of the pre-tiled layout; wave w takes slices
// w, w + 8, ... -- 5 per wave = one slot (narrower models: K / 32 < 40 slices, the rest of the slot
// reads nothing).  An fc2 tile (K = 4 d) is ceil(d / 320) slots: 4 for large, 2 for tiny.
// The role table (models/whisper.py wdec_roles) gives each workgroup its slots (level, tile, part,
// refill level), its self-attention head and its cross-attention item.
#include "common.h"
#include "vwa_kernels.h"

namespace {
using namespace vwa;

constexpr int kT = 512;           // threads (8 waves, K split over the waves)
constexpr int kSlots = 5, kLps = 5;
enum { LV_QKV = 0, LV_XQX, LV_SATT, LV_OXQ, LV_XATT, LV_XO, LV_FC1, LV_FC2 };
// gemm ids (WdecLayer::g; a slot's kind): the level of each
enum { G_QKV = 0, G_O, G_XQ, G_XO, G_FC1, G_FC2, G_XQO };
// role row layout (kWdRole ints per workgroup)
enum { R_KIND = 0, R_TILE = 5, R_PART = 10, R_RELOAD = 15, R_SATT = 20, R_XATT = 21, R_XPRE = 22, R_WORK = 23 };
// LDS layout (bytes)
constexpr int L_XS = 0;          // bf16 activation row (<= 5120)
constexpr int L_RED = 10368;     // f32 [8][32] cross-wave partial sums of a level's <= 2 tiles
constexpr int L_STAT = 11392;    // f32 [16]: mean, rstd
constexpr int L_W8 = 11456;      // f32 [2][8] per-wave reduction values
constexpr int L_QF = 11520;      // f32 [64] query head
constexpr int L_P = 11776;       // f32 [512] attention weights
constexpr int L_OW = 13824;      // f32 [8][64] per-wave attention outputs
constexpr int L_VA = 15872;      // int [512] self-attention K / V row offsets (elements)
constexpr int L_KV = 65536;      // cross-attention K chunk [<= 384][64] bf16, V chunk at + 48 KB
constexpr int L_KVV = 49152;
constexpr int kLds = 163840;
constexpr int kMaxChunk = 384;
constexpr int kSpinLimit = 1 << 17;  // bounded polls: a non-resident producer ends the launch, not the GPU
constexpr int kErrWord = 1024;       // (WdecParams::cnt u64 index of the error flag)
constexpr int kHeadCnt = 1280;      // (u64 index: per-head QKV completion counters, 128 B apart, <= 48 heads)
constexpr int kSmpCnt = 1152;       // (u64 index: the fused sampler's arrival counters, 8 groups x 128 B, monotonic)

VWA_DEVICE int level_of(int gm) {
  return gm == G_QKV ? LV_QKV : gm == G_XQ ? LV_XQX : gm == G_O || gm == G_XQO ? LV_OXQ : gm == G_XO ? LV_XO
       : gm == G_FC1 ? LV_FC1 : LV_FC2;
}

// Wave-uniform values through readfirstlane.  The per-layer descriptors are read with VECTOR loads
// (the kernel stores to global memory, so the compiler cannot prove them unclobbered for scalar
// loads): a buffer resource built from such a pointer lives in VGPRs, and every buffer load through
// it became a waterfall loop -- readfirstlane / compare / exec loop with a vmcnt(0) per iteration,
// i.e. each 1 KB weight load of a refill and each self-attention V load waited for every load
// before it (60 such loads in the ISA).  Every pointer and size here is uniform by construction.
VWA_DEVICE int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
VWA_DEVICE T* uni(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v), hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}

VWA_DEVICE __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(uni(const_cast<void*>(p)), (short)0,
                                           uni((int)(bytes < 0x7FFFFFF0ll ? bytes : 0x7FFFFFF0ll)), 0x00020000);
}

// sc1 (device-coherent) loads / stores of data crossing workgroups inside the launch
VWA_DEVICE uint4 ld_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}
VWA_DEVICE void st_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off, const uint4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, r, (int)off, 0, 16);
}
VWA_DEVICE float ldf_sc1(const float* p) { return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE void stf_sc1(float* p, float v) { __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE u16 ldh_sc1(const u16* p) { return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE void sth_sc1(u16* p, u16 v) { __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

VWA_DEVICE void set_err(const WdecParams& p) {
  __hip_atomic_store(gp(p.cnt + kErrWord), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sum of a level's eight group counters in one scalar round trip (glc: past the scalar cache)
VWA_DEVICE unsigned long long cnt_sum8(const unsigned long long* c) {
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
      : "s"(c)
      : "memory");
  return v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
}

VWA_DEVICE unsigned long long* lvl_cnt(const WdecParams& p, int lvl) { return p.cnt + (size_t)lvl * 8 * 16; }

// wave 0 polls until the level's counters reach target; bounded (a timed-out spin sets the error
// word: that step's results are invalid, the host falls back to per-kernel launches)
VWA_DEVICE void wd_wait(const WdecParams& p, int lvl, unsigned long long target) {
  if (VWA_TX < 64) {
    const unsigned long long* c = lvl_cnt(p, lvl);
    int spins = 0;
    while ((long long)(cnt_sum8(c) - target) < 0) {
      __builtin_amdgcn_s_sleep(1);
      // another workgroup already gave up: this launch is invalid anyway -- do not spin out again
      if ((spins & 255) == 255 && __hip_atomic_load(gp(p.cnt + kErrWord), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        break;
      if (++spins > kSpinLimit) {
        if (VWA_TX == 0) set_err(p);
        break;
      }
    }
  }
  lds_sync();
}

// this workgroup completed level lvl: every wave's stores are performed, then one no-return add on
// the group counter
VWA_DEVICE void wd_arrive(const WdecParams& p, int lvl) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_sync();
  if (VWA_TX == 0)
    __hip_atomic_fetch_add(gp(lvl_cnt(p, lvl) + 16 * (blockIdx.x & 7)), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// QKV -> self-attention by head: the workgroup of QKV tile t adds 1 to the counter of head
// (t / 4) mod H (its 16 columns are 16 of that head's 64 q, k or v dims); the attention of head h
// waits for its 12 tiles only, not for all 3 d / 16
VWA_DEVICE unsigned long long* head_cnt(const WdecParams& p, int h) { return p.cnt + kHeadCnt + 16 * h; }
VWA_DEVICE void wd_arrive_head(const WdecParams& p, int tile) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_sync();
  if (VWA_TX == 0)
    __hip_atomic_fetch_add(gp(head_cnt(p, (tile >> 2) % p.H)), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
VWA_DEVICE void wd_wait_head(const WdecParams& p, int h, unsigned long long target) {
  if (VWA_TX < 64) {
    const unsigned long long* c = head_cnt(p, h);
    int spins = 0;
    while (true) {
      unsigned long long v;
      asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(c) : "memory");
      if ((long long)(v - target) >= 0) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        if (VWA_TX == 0) set_err(p);
        break;
      }
    }
  }
  lds_sync();
}

// diagnostic stamp k of (layer, level) (tools/wdec_probe.py): 0 entry, 1 released, 2 row staged
// (attention levels: softmax done), 3 completed
VWA_DEVICE void wd_stamp(const WdecParams& p, int li, int lvl, int k) {
  if (p.ts && VWA_TX == 0)
    *gp(p.ts + ((size_t)blockIdx.x * p.n_layers * kWdLevels + (size_t)li * kWdLevels + lvl) * 4 + k) =
        __builtin_amdgcn_s_memrealtime();
}

VWA_DEVICE int n_cols(const WdecParams& p, int gm) {
  return gm == G_QKV ? 3 * p.d : gm == G_FC1 ? p.ffn : p.d;
}
VWA_DEVICE int k_of(const WdecParams& p, int gm) { return gm == G_FC2 ? p.ffn : p.d; }

// the cross query's f32 pre-activation halves (x part, att part) behind the cross partials
// cross-attention partial of (head, chunk): [max, sum, -, -, out[64]] -- 16-byte aligned rows
constexpr int kPart = 68;
VWA_DEVICE float* xq_buf(const WdecParams& p) { return p.xpart + (size_t)p.H * p.nch * kPart; }

// slot load: part `part` (5 load-slices per wave) of tile `tile` of gemm gm's weight, layer li
VWA_DEVICE void wd_load(const WdecParams& p, int li, int gm, int tile, int part, uint4 (&wr)[kLps]) {
  const WdecGemm& g = p.layers[li].g[gm];
  const int K = k_of(p, gm), G = K >> 7;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(g.W, (long long)n_cols(p, gm) * K * 2);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
#pragma unroll
  for (int j = 0; j < kLps; ++j) {
    const int sl = w + 8 * (part * kLps + j), kg = sl >> 2, s4 = sl & 3;
    // (slices past the tile's 4 K / 128: out of the buffer -> zeros, no traffic; d < 1280)
    const unsigned off = sl < 4 * G ? ((unsigned)(tile * G + kg) * 4u + (unsigned)s4) * 1024u + (unsigned)lane * 16u
                                    : 0x7FFFFFF0u;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    wr[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// slot load of a tile of an explicit K = d weight (the LM head): all 4 d / 128 <= 40 slices, 5 per wave
VWA_DEVICE void wd_load_w(const u16* W, int n_cols, int K, int tile, uint4 (&wr)[kLps]) {
  const int G = K >> 7;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(W, (long long)n_cols * K * 2);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
#pragma unroll
  for (int j = 0; j < kLps; ++j) {
    const int sl = w + 8 * j, kg = sl >> 2, s4 = sl & 3;
    const unsigned off = sl < 4 * G ? ((unsigned)(tile * G + kg) * 4u + (unsigned)s4) * 1024u + (unsigned)lane * 16u
                                    : 0x7FFFFFF0u;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    wr[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// the MFMAs of one slot: acc (row 0 = lanes 0..15, element 0) += X . W over the slot's slices
// (nsl: the tile's slices, 4 K / 128 -- the row past K is not read)
VWA_DEVICE void wd_mma(const char* lds, int part, const uint4 (&wr)[kLps], f32x4& acc, int nsl) {
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6, nl = lane & 15, g = lane >> 4;
  const u16* xs = reinterpret_cast<const u16*>(lds + L_XS);
#pragma unroll
  for (int j = 0; j < kLps; ++j) {
    const int sl = w + 8 * (part * kLps + j), kg = sl >> 2, s4 = sl & 3;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (nl == 0 && sl < nsl) a = *reinterpret_cast<const uint4*>(xs + kg * 128 + 32 * g + 8 * s4);
    acc = mfma16(as_bf16x8(a), as_bf16x8(wr[j]), acc);
  }
}

// cross-attention K / V chunk of layer li (this workgroup's item) -> LDS by LDS-DMA (no registers;
// completes on vmcnt: the level waits for it)
VWA_DEVICE void wd_kv_prefetch(const WdecParams& p, int li, int item, char* lds) {
  const int h = item / p.nch, ch = item % p.nch;
  const int k0 = ch * p.ch_len, nk = min(p.ch_len, p.T - k0);
  const int sess = p.cross_table[p.seq_ids[0]];
  const WdecLayer& L = p.layers[li];
  const long long bytes = (long long)p.sessions * p.T * p.H * 64 * 2;
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(L.xk, bytes), rv = rsrc_of(L.xv, bytes);
  const int tx = VWA_TX, lane = tx & 63, w = uni(tx >> 6);  // (uniform: the K / V select stays scalar)
  const int n8 = (nk + 7) >> 3;  // 1 KB instructions (8 keys of 128 B) per tensor
  for (int r = w; r < 2 * n8; r += 8) {
    const bool isv = r >= n8;
    const int rr = isv ? r - n8 : r;
    const int kk = rr * 8 + (lane >> 3);
    // K rows XOR-swizzled by 16-byte chunk (LDS slot j of key kk holds chunk j ^ (kk & 7)): the
    // key-per-thread dot products read 8 different bank groups per 8 lanes instead of one
    const int chunk = isv ? (lane & 7) : ((lane & 7) ^ (kk & 7));
    const unsigned off = kk < nk ? (unsigned)(((((long long)sess * p.T + k0 + kk) * p.H + h) * 64 + chunk * 8) * 2)
                                 : 0x7FFFFFF0u;
    auto* dst = (__attribute__((address_space(3))) void*)(lds + L_KV + (isv ? L_KVV : 0) + rr * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isv ? rv : rk, dst, 16, off, 0, 0, 0);
  }
}

// block-wide max / sum of one value per thread (all threads get the result)
VWA_DEVICE float blk_max(char* lds, float v) {
  float* w8 = reinterpret_cast<float*>(lds + L_W8);
  v = wave_max(v);
  if ((VWA_TX & 63) == 0) w8[VWA_TX >> 6] = v;
  lds_sync();
  float m = w8[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) m = fmaxf(m, w8[i]);
  return m;
}
VWA_DEVICE float blk_sum(char* lds, float v) {
  float* w8 = reinterpret_cast<float*>(lds + L_W8) + 8;
  v = wave_sum(v);
  if ((VWA_TX & 63) == 0) w8[VWA_TX >> 6] = v;
  lds_sync();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += w8[i];
  return s;
}

// cross query head h -> LDS f32 [64]: q = rstd1 (xqa + xqb - mean1 c) + b' (rounded to bf16 like
// the per-kernel path's q), mean1 / rstd1 of x1 from the out-projection tiles' (sum, sum of
// squares) -- wave 0 alone (lane: column h 64 + lane, tiles lane and lane + 64), no cross-wave
// round; qc / qb: c and b' of the lane's column, loaded ahead of the release.  The loads go out
// after the K / V chunk DMAs, so every wave's vmcnt wait also covers those (the barrier then
// publishes every wave's chunk).
VWA_DEVICE void wd_xq_to_lds(const WdecParams& p, int h, char* lds, float qc, float qb) {
  float* qf = reinterpret_cast<float*>(lds + L_QF);
  const int tx = VWA_TX, nt = p.d >> 4;
  const float* xq = xq_buf(p);
  if (tx < 64) {
    const float a = ldf_sc1(xq + h * 64 + tx), b = ldf_sc1(xq + p.d + h * 64 + tx);
    const float* st2 = xq + 2 * p.d;
    float s = 0.f, s2 = 0.f;
    if (tx < nt) {
      s = ldf_sc1(st2 + 2 * tx);
      s2 = ldf_sc1(st2 + 2 * tx + 1);
    }
    if (tx + 64 < nt) {
      s += ldf_sc1(st2 + 2 * (tx + 64));
      s2 += ldf_sc1(st2 + 2 * (tx + 64) + 1);
    }
    s = wave_sum(s);
    s2 = wave_sum(s2);
    const float mean = s / (float)p.d, rstd = rsqrtf(fmaxf(s2 / (float)p.d - mean * mean, 0.f) + p.eps);
    qf[tx] = bf2f(f2bf((a + b - mean * qc) * rstd + qb));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_sync();
}

// softmax over the thread-per-key scores s (keys t < nk, others -inf): returns (max, sum); P[t] in LDS
// (w8 max slots [0, 8) and sum slots [8, 16) are distinct: no barrier between the two reductions)
VWA_DEVICE float2 wd_softmax(char* lds, float s, bool valid) {
  float* P = reinterpret_cast<float*>(lds + L_P);
  const float m = blk_max(lds, valid ? s : -INFINITY);
  const float e = valid ? __expf(s - m) : 0.f;
  P[VWA_TX] = e;
  const float l = blk_sum(lds, e);  // (its barrier publishes P)
  return make_float2(m, l);
}

// per-wave partial outputs (lane = dim) -> LDS, summed by threads < 64 after the barrier
VWA_DEVICE float wd_ow_sum(char* lds, float o) {
  float* ow = reinterpret_cast<float*>(lds + L_OW);
  const int tx = VWA_TX;
  ow[(tx >> 6) * 64 + (tx & 63)] = o;
  lds_sync();
  float s = 0.f;
  if (tx < 64) {
#pragma unroll
    for (int w = 0; w < 8; ++w) s += ow[w * 64 + tx];
  }
  return s;
}

// level 1: self-attention of head h over the row's context (<= 512 keys: one thread per key).
// The key rows' addresses are resolved ahead of the release (wd_self_attn_pre); after it q, the K
// rows and the first 8 V elements per lane are issued together -- one round trip (the newest key
// was written by this layer's QKV level).
VWA_DEVICE void wd_self_attn_pre(const WdecParams& p, int h, char* lds) {
  const int tx = VWA_TX;
  const int seq = p.seq_ids[0], ctx = min(p.ctx_lens[0], kT);
  const int bs = p.block_size;
  int* va = reinterpret_cast<int*>(lds + L_VA);
  if (tx < ctx) {
    const int blk = p.block_table[seq * p.bt_stride + tx / bs];
    va[tx] = ((blk * p.H + h) * bs + tx % bs) * 64;  // element offset of key tx's row
  }
  lds_sync();
}

VWA_DEVICE void wd_self_attn(const WdecParams& p, int li, int h, char* lds) {
  const WdecLayer& L = p.layers[li];
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  const int ctx = min(p.ctx_lens[0], kT);
  const int* va = reinterpret_cast<const int*>(lds + L_VA);
  float* qf = reinterpret_cast<float*>(lds + L_QF);
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(L.k_cache, 0x7FFFFFF0ll), rv = rsrc_of(L.v_cache, 0x7FFFFFF0ll);
  uint4 qv = make_uint4(0, 0, 0, 0);
  if (tx < 8) qv = ld_sc1_b128(rsrc_of(p.q, (long long)p.d * 2), (unsigned)((h * 64 + tx * 8) * 2));
  uint4 kr[8];
  const bool valid = tx < ctx;
  const int e0 = valid ? va[tx] : 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) kr[c] = valid ? ld_sc1_b128(rk, (unsigned)(e0 * 2 + c * 16)) : make_uint4(0, 0, 0, 0);
  float vv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int t = w + 8 * i;
    vv[i] = t < ctx ? bf2f((u16)__builtin_amdgcn_raw_buffer_load_b16(rv, (int)((va[t] + lane) * 2), 0, 16)) : 0.f;
  }
  if (tx < 8) {
    float f[8];
    unpack8(qv, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[tx * 8 + e] = f[e];
  }
  lds_sync();
  float s = -INFINITY;
  if (valid) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float f[8];
      unpack8(kr[c], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qf[c * 8 + e] * f[e];
    }
    s = acc * p.scale;
  }
  const float2 ml = wd_softmax(lds, s, valid);
  wd_stamp(p, li, LV_SATT, 2);
  const float* P = reinterpret_cast<const float*>(lds + L_P);
  float o = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int t = w + 8 * i;
    if (t < ctx) o += P[t] * vv[i];
  }
  for (int t0 = w + 64; t0 < ctx; t0 += 64) {  // (contexts beyond 64 keys: 8 keys per wave per batch)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = t0 + 8 * i;
      vv[i] = t < ctx ? bf2f((u16)__builtin_amdgcn_raw_buffer_load_b16(rv, (int)((va[t] + lane) * 2), 0, 16)) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = t0 + 8 * i;
      if (t < ctx) o += P[t] * vv[i];
    }
  }
  const float tot = wd_ow_sum(lds, o);
  if (tx < 64) sth_sc1(p.att + h * 64 + tx, f2bf(tot / ml.y));
}

// level 4: cross query of head h, then the cross-attention partial of (head, chunk) from the
// prefetched K / V chunk in LDS
VWA_DEVICE void wd_cross_attn(const WdecParams& p, int li, int item, char* lds, float qc, float qb) {
  const int h = item / p.nch, ch = item % p.nch;
  const int k0 = ch * p.ch_len, nk = min(p.ch_len, p.T - k0);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  wd_xq_to_lds(p, h, lds, qc, qb);
  const float* qf = reinterpret_cast<const float*>(lds + L_QF);
  const u16* kl = reinterpret_cast<const u16*>(lds + L_KV);
  const u16* vl = reinterpret_cast<const u16*>(lds + L_KV + L_KVV);
  float s = -INFINITY;
  const bool valid = tx < nk;
  if (valid) {
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(kl + tx * 64 + ((c ^ (tx & 7)) * 8)), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qf[c * 8 + e] * f[e];
    }
    s = acc * p.scale;
  }
  const float2 ml = wd_softmax(lds, s, valid);
  wd_stamp(p, li, LV_XATT, 2);
  const float* P = reinterpret_cast<const float*>(lds + L_P);
  // 8 keys per wave per batch, every LDS read of a batch issued before its FMAs
  float oa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int t0 = w; t0 < nk; t0 += 64) {
    float pv[8], vv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int t = min(t0 + 8 * i, nk - 1);
      pv[i] = t0 + 8 * i < nk ? P[t] : 0.f;
      vv[i] = bf2f(vl[t * 64 + lane]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) oa[i] += pv[i] * vv[i];
  }
  const float o = ((oa[0] + oa[1]) + (oa[2] + oa[3])) + ((oa[4] + oa[5]) + (oa[6] + oa[7]));
  const float tot = wd_ow_sum(lds, o);
  float* part = p.xpart + (size_t)(h * p.nch + ch) * kPart;
  if (tx < 64) stf_sc1(part + 4 + tx, tot);
  if (tx == 0) {
    stf_sc1(part, ml.x);
    stf_sc1(part + 1, ml.y);
  }
}

// X staging of a GEMM level: the activation row (bf16, written earlier in this launch or, for layer
// 0, the embedding) -> LDS; LayerNorm levels also get the row's mean / rstd (from the staged values)
// emb (layer 0 with WdecParams::tok_emb): the row is the step's embedding, built here from the
// tables (embedding_kernel's arithmetic: f32 sum of the two bf16 rows, one rounding); emb_store:
// this workgroup also writes it to x (the layer's residual / input row for every later level)
VWA_DEVICE void wd_stage(const WdecParams& p, int K, const u16* x, char* lds, bool ln, bool emb = false,
                         bool emb_store = false) {
  const int n8 = K >> 3;
  const int tx = VWA_TX;
  u16* xs = reinterpret_cast<u16*>(lds + L_XS);
  const __amdgpu_buffer_rsrc_t r = rsrc_of(x, (long long)K * 2);
  uint4 v[2];
  if (emb) {
    const int id = uni(p.tokens[0]), pos = uni(p.positions[0]);
    const bool in = id >= 0 && id < p.emb_rows;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tx + i * kT;
      v[i] = make_uint4(0, 0, 0, 0);
      if (c < n8) {
        float a[8], b[8];
        if (in) {
          unpack8(*reinterpret_cast<const uint4*>(p.tok_emb + (size_t)id * K + c * 8), a);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = 0.f;
        }
        unpack8(*reinterpret_cast<const uint4*>(p.pos_emb + (size_t)pos * K + c * 8), b);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += b[e];
        v[i] = pack8(a);
        if (emb_store) st_sc1_b128(r, (unsigned)c * 16u, v[i]);
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tx + i * kT;
      v[i] = c < n8 ? ld_sc1_b128(r, (unsigned)c * 16u) : make_uint4(0, 0, 0, 0);
    }
  }
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tx + i * kT;
    if (c < n8) {
      *reinterpret_cast<uint4*>(xs + c * 8) = v[i];
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s += f[e];
        s2 += f[e] * f[e];
      }
    }
  }
  if (ln) {  // one block reduction of (sum, sum of squares)
    float* w8 = reinterpret_cast<float*>(lds + L_W8);
    s = wave_sum(s);
    s2 = wave_sum(s2);
    if ((tx & 63) == 0) {
      w8[tx >> 6] = s;
      w8[8 + (tx >> 6)] = s2;
    }
    lds_sync();
    float ts = 0.f, ts2 = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      ts += w8[i];
      ts2 += w8[8 + i];
    }
    float* st = reinterpret_cast<float*>(lds + L_STAT);
    if (tx == 0) {
      const float mean = ts / (float)K;
      st[0] = mean;
      st[1] = rsqrtf(fmaxf(ts2 / (float)K - mean * mean, 0.f) + p.eps);
    }
  }
  lds_sync();
}

// X staging of the cross out-projection: the attention row merged from the (head, chunk)
// partials (chunk order fixed: the same bits whoever finished last).  A thread merges 4
// consecutive columns of one head: per chunk one 8-byte (max, sum) and one 16-byte output load,
// all issued before any is used (was 12 scalar loads per column, 3 columns per thread)
VWA_DEVICE void wd_stage_merge(const WdecParams& p, char* lds) {
  u16* xs = reinterpret_cast<u16*>(lds + L_XS);
  const int tx = VWA_TX, nch = p.nch;
  const int c0 = 4 * min(tx, (p.d >> 2) - 1), h = c0 >> 6, dd = c0 & 63;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(p.xpart, (long long)p.H * nch * kPart * 4);
  u32x2 ml[4];
  u32x4 ov[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int kk = min(k, nch - 1);
    const unsigned base = (unsigned)((h * nch + kk) * kPart) * 4u;
    ml[k] = __builtin_amdgcn_raw_buffer_load_b64(r, (int)base, 0, 16);
    ov[k] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(base + 16u + (unsigned)dd * 4u), 0, 16);
  }
  if (tx < (p.d >> 2)) {
    float mx = __uint_as_float(ml[0].x);
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (k < nch) mx = fmaxf(mx, __uint_as_float(ml[k].x));
    float num[4] = {0.f, 0.f, 0.f, 0.f}, den = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nch) {
        const float e = __expf(__uint_as_float(ml[k].x) - mx);
        den += e * __uint_as_float(ml[k].y);
        num[0] += e * __uint_as_float(ov[k].x);
        num[1] += e * __uint_as_float(ov[k].y);
        num[2] += e * __uint_as_float(ov[k].z);
        num[3] += e * __uint_as_float(ov[k].w);
      }
    const float inv = 1.f / den;
    uint2 pk;
    pk.x = (unsigned)f2bf(num[0] * inv) | ((unsigned)f2bf(num[1] * inv) << 16);
    pk.y = (unsigned)f2bf(num[2] * inv) | ((unsigned)f2bf(num[3] * inv) << 16);
    *reinterpret_cast<uint2*>(xs + c0) = pk;
  }
  lds_sync();
}

// cross-wave sums of the level's (<= 2) tiles in ONE LDS round + the epilogue: thread t < 16 nt
// finishes column t & 15 of tile t >> 4 (gemm gm, a second tile costs no second barrier pair);
// eb / ec / er: that column's bias, folded-LayerNorm column sum and residual, loaded ahead
VWA_DEVICE void wd_epilogue(const WdecParams& p, int li, int g0, int g1, int tl0, int tl1, int nt, const f32x4& acc0,
                            const f32x4& acc1, char* lds, u16* xout, float eb, float ec, float er) {
  float* red = reinterpret_cast<float*>(lds + L_RED);
  const float* st = reinterpret_cast<const float*>(lds + L_STAT);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  if (lane < 16) {
    red[w * 32 + lane] = acc0[0];
    red[w * 32 + 16 + lane] = acc1[0];
  }
  lds_sync();
  if (tx < 16 * nt) {
    const int tile = tx < 16 ? tl0 : tl1, gm = tx < 16 ? g0 : g1, q = tx & 15;
    const int n = tile * 16 + q;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) v += red[ww * 32 + tx];
    if (gm == G_QKV || gm == G_FC1) v = (v - st[0] * ec) * st[1];
    v += eb;
    if (gm == G_FC1) v = gelu_erf(v);
    if (gm == G_O || gm == G_XO || gm == G_FC2) {
      const u16 o = f2bf(v + er);
      sth_sc1(xout + n, o);
      if (gm == G_O) {  // the tile's (sum, sum of squares) of x1: the cross query's LayerNorm stats
        float a = bf2f(o), b = a * a;
#pragma unroll
        for (int m = 8; m > 0; m >>= 1) {
          a += __shfl_xor(a, m, 64);
          b += __shfl_xor(b, m, 64);
        }
        if (q == 0) {
          float* st2 = xq_buf(p) + 2 * p.d + 2 * tile;
          stf_sc1(st2, a);
          stf_sc1(st2 + 1, b);
        }
      }
    } else if (gm == G_FC1) {
      sth_sc1(p.f + n, f2bf(v));
    } else if (gm == G_XQ || gm == G_XQO) {
      stf_sc1(xq_buf(p) + (gm == G_XQ ? 0 : p.d) + n, v);
    } else {  // QKV: rows permuted per head (ops.permute_qkv_rows: rotary pairs c, c ^ 8)
      const int n0 = tile * 16, head = n0 >> 6, t4 = (n0 & 63) >> 4;
      const int dd = q < 8 ? 8 * t4 + q : 32 + 8 * t4 + q - 8;
      const u16 out = f2bf(v);
      if (head < p.H) {
        sth_sc1(p.q + head * 64 + dd, out);
      } else {
        const long long slot = p.slots[0];
        if (slot >= 0) {
          const WdecLayer& L = p.layers[li];
          const bool isv = head >= 2 * p.H;
          const int kvh = isv ? head - 2 * p.H : head - p.H;
          const long long blk = slot / p.block_size, off = slot % p.block_size;
          const long long idx = ((blk * p.H + kvh) * p.block_size + off) * 64 + dd;
          sth_sc1((isv ? L.v_cache : L.k_cache) + idx, out);
        }
      }
    }
  }
}

// LM head epilogue of (<= 2) tiles in one LDS round: thread t < 16 nt finishes column t & 15 of
// tile t >> 4 (lc / lb: that column's folded-LayerNorm column sum and bias, loaded with the tile)
VWA_DEVICE void argmax_merge(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {  // (sample.hip's order: the lowest id on ties)
    bv = v;
    bi = i;
  }
}

VWA_DEVICE void wd_lm_epilogue(const WdecParams& p, int tl0, int tl1, int nt, const f32x4& acc0, const f32x4& acc1,
                               char* lds, float lc, float lb, int mk, float& bv, int& bi) {
  float* red = reinterpret_cast<float*>(lds + L_RED);
  const float* st = reinterpret_cast<const float*>(lds + L_STAT);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  if (lane < 16) {
    red[w * 32 + lane] = acc0[0];
    red[w * 32 + 16 + lane] = acc1[0];
  }
  lds_sync();
  if (tx < 16 * nt) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) v += red[ww * 32 + tx];
    const int n = (tx < 16 ? tl0 : tl1) * 16 + (tx & 15);
    const float lg = (v - st[0] * lc) * st[1] + lb;
    p.logits[n] = lg;
    if (mk) argmax_merge(bv, bi, lg, n);
  }
  lds_sync();  // (red is rewritten by the next round)
}

// schedule options (WdecParams::opt[0] bits; 0 = the defaults below)
constexpr int kOptNoEpiPre = 1;    // load the epilogue operands after the row (not ahead of it)
constexpr int kOptNoSattnPre = 2;  // self-attention resolves its key addresses after its inputs landed
constexpr int kOptXqxIdle = 4;     // (diagnostic, wrong results) the x part of the cross query does no work
constexpr int kOptQkvByHead = 8;   // (opt-in) QKV -> self-attention through per-head counters: ~8 us per
                                   // launch faster, but one GPU-test mismatch on a box was not explained

__global__ __launch_bounds__(kT) void wdec_kernel(WdecParams p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int* rr = p.roles + (size_t)blockIdx.x * kWdRole;
  int kind[kSlots], klv[kSlots], tile[kSlots], part[kSlots], rl[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {  // (uniform: scalar branches and offsets)
    kind[s] = uni(rr[R_KIND + s]);  // gemm id or -1
    klv[s] = kind[s] >= 0 ? level_of(kind[s]) : -1;
    tile[s] = uni(rr[R_TILE + s]);
    part[s] = uni(rr[R_PART + s]);
    rl[s] = uni(rr[R_RELOAD + s]);
  }
  const int sattn = uni(rr[R_SATT]), xattn = uni(rr[R_XATT]), xpre = uni(rr[R_XPRE]), work = uni(rr[R_WORK]);
  const int NL = p.n_layers;
  const int opt = p.opt[0];
  if (work == 0 && !p.lm_W) return;
  // launch bases of the level counters (see the header comment)
  unsigned long long* bases = reinterpret_cast<unsigned long long*>(lds + L_RED);  // (before any tile)
  if (VWA_TX < 64) {
    for (int l = 0; l < kWdLevels; ++l) {
      const unsigned long long inc = (unsigned long long)p.n_prod[l] * (unsigned long long)NL;
      const unsigned long long s = cnt_sum8(lvl_cnt(p, l));
      if (VWA_TX == 0) bases[l] = s / inc * inc;
    }
  }
  lds_sync();
  unsigned long long base[kWdLevels];
#pragma unroll
  for (int l = 0; l < kWdLevels; ++l) {
    const unsigned long long b = bases[l];
    base[l] = __builtin_amdgcn_readfirstlane((unsigned)b) |
              ((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(b >> 32)) << 32);
  }
  lds_sync();
  // (the fused sampler's arrival counters: base of this launch, read by workgroup 0's wave 0 --
  // before any workgroup can arrive there, which needs every level, workgroup 0's included)
  // (the self-attention head's counter: 12 tiles per layer, n_layers per launch)
  unsigned long long hbase = 0;
  const bool by_head = (opt & kOptQkvByHead) != 0;
  if (by_head && sattn >= 0 && VWA_TX < 64) {
    const unsigned long long inc = 12ull * (unsigned long long)NL;
    unsigned long long v;
    const unsigned long long* c = head_cnt(p, sattn);
    asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(c) : "memory");
    hbase = v / inc * inc;
  }
  unsigned long long smp_base = 0;
  if (p.smp_mask && blockIdx.x == 0 && VWA_TX < 64) {
    const unsigned long long inc = (unsigned long long)gridDim.x;
    smp_base = cnt_sum8(p.cnt + kSmpCnt) / inc * inc;
  }
  // the level's counter target after layer pli
  auto target = [&](int l, int pli) { return base[l] + (unsigned long long)p.n_prod[l] * (unsigned long long)(pli + 1); };
  uint4 wr[kSlots][kLps];
  // initial slot loads: slots refilled after their use (refill level >= level) hold layer 0 now
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
#pragma unroll
    for (int j = 0; j < kLps; ++j) wr[s][j] = make_uint4(0, 0, 0, 0);
    if (kind[s] >= 0 && rl[s] >= klv[s]) wd_load(p, 0, kind[s], tile[s], part[s], wr[s]);
  }
  if (xattn >= 0 && xpre >= LV_XATT) wd_kv_prefetch(p, 0, xattn, lds);

  for (int li = 0; li < NL; ++li) {
    u16* xc = (li & 1) ? p.x1 : p.x0;  // this layer's input row
    u16* xo = (li & 1) ? p.x0 : p.x1;
    for (int lvl = 0; lvl < kWdLevels; ++lvl) {
      if (!((work >> lvl) & 1)) continue;
      wd_stamp(p, li, lvl, 0);
      const bool gemm = lvl != LV_SATT && lvl != LV_XATT;
      // ahead of the inputs: the epilogue's bias / LayerNorm column sums (<= 2 tiles per level),
      // the self-attention's key addresses, the cross query's column sums and bias
      float eb = 0.f, ec = 0.f, er = 0.f;  // (thread t < 16 nt: column t & 15 of tile t >> 4)
      int tl[2] = {0, 0}, tg[2] = {0, 0};
      int nt = 0;
      auto epi_ops = [&]() {
        if (VWA_TX < 16 * nt) {
          const int gm = VWA_TX < 16 ? tg[0] : tg[1];
          const WdecGemm& g = p.layers[li].g[gm];
          const int n = (VWA_TX < 16 ? tl[0] : tl[1]) * 16 + (VWA_TX & 15);
          if (g.bias && gm != G_XQ) eb = bf2f(gld(g.bias + n));
          if (g.ln_c && (gm == G_QKV || gm == G_FC1)) ec = gld(g.ln_c + n);
        }
      };
      if (gemm) {
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
          const bool last = klv[s] == lvl && (s == kSlots - 1 || kind[s + 1] != kind[s] || tile[s + 1] != tile[s]);
          if (last) {  // (selects, not a dynamic index: a private array would live in scratch)
            tl[1] = nt == 1 ? tile[s] : tl[1];
            tg[1] = nt == 1 ? kind[s] : tg[1];
            tl[0] = nt == 0 ? tile[s] : tl[0];
            tg[0] = nt == 0 ? kind[s] : tg[0];
            nt = nt < 2 ? nt + 1 : nt;
          }
        }
        if (!(opt & kOptNoEpiPre)) epi_ops();
      } else if (lvl == LV_SATT && !(opt & kOptNoSattnPre)) {
        wd_self_attn_pre(p, sattn, lds);
      } else if (lvl == LV_XATT && VWA_TX < 64) {
        const WdecGemm& g = p.layers[li].g[G_XQ];
        const int n = (xattn / p.nch) * 64 + VWA_TX;
        ec = gld(g.ln_c + n);
        eb = bf2f(gld(g.bias + n));
      }
      // release: the level's producer level (the x part of the cross query needs only the layer
      // input: nothing when this workgroup just ran the QKV level; the cross-attention also needs it)
      if (lvl == LV_XATT) wd_wait(p, LV_XQX, target(LV_XQX, li));
      if (lvl == LV_QKV || (lvl == LV_XQX && !(work & 1))) {
        if (li > 0) wd_wait(p, LV_FC2, target(LV_FC2, li - 1));
      } else if (lvl == LV_SATT && by_head) {
        wd_wait_head(p, sattn, hbase + 12ull * (unsigned long long)(li + 1));
      } else if (lvl != LV_XQX) {
        const int pl = lvl == LV_SATT ? LV_QKV : lvl - 1;
        wd_wait(p, pl, target(pl, li));
      }
      wd_stamp(p, li, lvl, 1);
      if (lvl == LV_XQX && (opt & kOptXqxIdle)) {
      } else if (lvl == LV_SATT) {
        if (opt & kOptNoSattnPre) wd_self_attn_pre(p, sattn, lds);
        wd_self_attn(p, li, sattn, lds);
      } else if (lvl == LV_XATT) {
        wd_cross_attn(p, li, xattn, lds, ec, eb);
      } else {
        // activation row + residual of this level
        const u16* xin = lvl == LV_OXQ ? p.att : lvl == LV_FC2 ? p.f : xc;
        const u16* xres = lvl == LV_XO ? xo : xc;
        u16* xout = lvl == LV_XO ? xc : xo;
        const bool resid = lvl == LV_OXQ || lvl == LV_XO || lvl == LV_FC2;
        if (resid && VWA_TX < 16 * nt)  // (in the same round trip as the row)
          er = bf2f(ldh_sc1(xres + (VWA_TX < 16 ? tl[0] : tl[1]) * 16 + (VWA_TX & 15)));
        if (lvl == LV_XO) {
          wd_stage_merge(p, lds);
        } else if (!(lvl == LV_XQX && (work & 1))) {  // (after the QKV level the row is staged already)
          // layer 0 with the tables: the QKV / cross-query-x levels build the embedding row
          // themselves; the workgroup of QKV tile 0 stores it for the residual reads
          const bool emb = p.tok_emb && li == 0 && (lvl == LV_QKV || lvl == LV_XQX);
          wd_stage(p, k_of(p, lvl == LV_FC2 ? G_FC2 : G_O), xin, lds, lvl == LV_QKV || lvl == LV_FC1, emb,
                   emb && lvl == LV_QKV && kind[0] == G_QKV && tile[0] == 0);
        }
        wd_stamp(p, li, lvl, 2);
        if (opt & kOptNoEpiPre) epi_ops();
        f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
        int j = 0;  // tiles finished before this slot
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
          if (klv[s] != lvl) continue;
          const int nsl = k_of(p, kind[s]) >> 5;
          if (j == 0) wd_mma(lds, part[s], wr[s], acc0, nsl);
          else wd_mma(lds, part[s], wr[s], acc1, nsl);
          const bool last = s == kSlots - 1 || kind[s + 1] != kind[s] || tile[s + 1] != tile[s];
          if (last) ++j;
        }
        wd_epilogue(p, li, tg[0], tg[1], tl[0], tl[1], nt, acc0, acc1, lds, xout, eb, ec, er);
      }
      if (lvl == LV_QKV && by_head) wd_arrive_head(p, tile[0]);  // (the QKV tile sits in slot 0)
      else wd_arrive(p, lvl);
      wd_stamp(p, li, lvl, 3);
      // refills a layer ahead
#pragma unroll
      for (int s = 0; s < kSlots; ++s) {
        if (kind[s] >= 0 && rl[s] == lvl) {
          const int lt = rl[s] < klv[s] ? li : li + 1;
          if (lt < NL) wd_load(p, lt, kind[s], tile[s], part[s], wr[s]);
        }
      }
      if (xattn >= 0 && xpre == lvl) {
        const int lt = xpre < LV_XATT ? li : li + 1;
        if (lt < NL) wd_kv_prefetch(p, lt, xattn, lds);
      }
    }
  }
  if (p.lm_W) {
    // LM head: tiles blockIdx.x + j grid of the padded vocabulary, a 5-slot ring; the first five
    // tiles' weights go out BEFORE the wait for the last layer's fc2 (weights never depend on the
    // activations), the rest stream behind them -- no separate launch, no launch gap
    const int G = (int)gridDim.x, NTv = p.n_vocab >> 4, b0 = (int)blockIdx.x;
    const int ntw = b0 < NTv ? (NTv - 1 - b0) / G + 1 : 0;
    const int tx = VWA_TX, q = tx & 15;
    float lc[kSlots], lb[kSlots];  // (threads < 32: column q of the slot's tile)
    int mk[kSlots];                 // (its sampler mask bit)
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    auto issue = [&](int s, int j) {
      if (j < ntw) {
        const int t = b0 + j * G;
        wd_load_w(p.lm_W, p.n_vocab, p.d, t, wr[s]);
        if (tx < 32) {
          const int n = t * 16 + q;
          lc[s] = gld(p.lm_c + n);
          lb[s] = p.lm_b ? bf2f(gld(p.lm_b + n)) : 0.f;
          mk[s] = p.smp_mask ? (int)((gld(p.smp_mask + (n >> 5)) >> (n & 31)) & 1u) : 0;
        }
      }
    };
#pragma unroll
    for (int s = 0; s < kSlots; ++s) issue(s, s);
    wd_wait(p, LV_FC2, base[LV_FC2] + (unsigned long long)p.n_prod[LV_FC2] * (unsigned long long)NL);
    wd_stage(p, p.d, ((NL - 1) & 1) ? p.x0 : p.x1, lds, true);
    for (int j0 = 0; j0 < ntw; j0 += kSlots) {
#pragma unroll
      for (int s = 0; s < kSlots; s += 2) {
        const int ja = j0 + s, jb = j0 + s + 1;
        if (ja >= ntw) break;  // (uniform)
        const bool two = s + 1 < kSlots && jb < ntw;
        f32x4 acc0 = f32x4{0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
        wd_mma(lds, 0, wr[s], acc0, p.d >> 5);
        const float c0 = lc[s], bb0 = lb[s];
        const int m0 = mk[s];
        float c1 = 0.f, bb1 = 0.f;
        int m1 = 0;
        if (s + 1 < kSlots) {
          if (two) wd_mma(lds, 0, wr[s + 1], acc1, p.d >> 5);
          c1 = lc[s + 1];
          bb1 = lb[s + 1];
          m1 = mk[s + 1];
        }
        issue(s, ja + kSlots);  // (the slot's registers are free once its MFMAs were issued)
        if (s + 1 < kSlots && two) issue(s + 1, jb + kSlots);
        wd_lm_epilogue(p, b0 + ja * G, b0 + jb * G, two ? 2 : 1, acc0, acc1, lds, tx < 16 ? c0 : c1,
                       tx < 16 ? bb0 : bb1, tx < 16 ? m0 : m1, bv, bi);
      }
    }
    if (p.smp_mask) {
      // greedy sample: the workgroup's best (wave 0, lanes < 32 hold columns) -> a partial; the
      // last workgroup to arrive merges the grid's partials and advances the device loop
      if (tx < 64) {
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
          const float ov = __shfl_xor(bv, m, 64);
          const int oi = __shfl_xor(bi, m, 64);
          argmax_merge(bv, bi, ov, oi);
        }
      }
      // (arrival as the levels do it: no-return adds spread over 8 group counters, workgroup 0
      // polls their sum -- one returning ticket on one word from 256 workgroups measured ~15 us)
      if (tx == 0) {
        stf_sc1(p.smp_part + 2 * b0, bv);
        stf_sc1(p.smp_part + 2 * b0 + 1, __int_as_float(bi));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(gp(p.cnt + kSmpCnt + 16 * (b0 & 7)), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (b0 == 0 && tx < 64) {
        int spins = 0;
        while ((long long)(cnt_sum8(p.cnt + kSmpCnt) - (smp_base + (unsigned long long)G)) < 0) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kSpinLimit) {
            if (tx == 0) set_err(p);
            break;
          }
        }
        float v = -INFINITY;
        int ix = 0x7fffffff;
        for (int k = tx; k < G; k += 64) argmax_merge(v, ix, ldf_sc1(p.smp_part + 2 * k), __float_as_int(ldf_sc1(p.smp_part + 2 * k + 1)));
#pragma unroll
        for (int m = 32; m > 0; m >>= 1) {
          const float ov = __shfl_xor(v, m, 64);
          const int oi = __shfl_xor(ix, m, 64);
          argmax_merge(v, ix, ov, oi);
        }
        if (tx == 0) {  // (decode_advance_kernel's arithmetic)
          const int tok = v == -INFINITY ? -1 : ix;
          p.smp_tok[0] = tok;
          p.smp_step[0] += 1;
          const int c = p.loop_cnt[0];
          if (c < p.loop_max) p.loop_out[c] = tok;
          p.loop_cnt[0] = c + 1;
          p.adv_tokens[0] = tok;
          const int pos = p.adv_positions[0] + 1;
          p.adv_positions[0] = pos;
          p.adv_ctx[0] = pos + 1;
          p.adv_slots[0] = (int64_t)(p.loop_base_block + pos / p.block_size) * p.block_size + pos % p.block_size;
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no LDS-DMA outstanding at the end)
}

}  // namespace

extern "C" int vwa_wdec_launch(const WdecParams* p, int grid, hipStream_t st) {
  // (whisper tiny .. large: d a multiple of 128 up to 1536 -- the merge stages <= 3 columns per
  // thread, a tile <= 40 slices of the K = d slots; ffn = 4 d staged by <= 2 x 16 B per thread)
  if (p->d % 128 != 0 || p->d > 3 * kT || p->ffn != 4 * p->d || p->ffn > 2 * kT * 8 || p->H * 64 != p->d ||
      p->n_layers < 2 || p->ch_len > kMaxChunk || p->ch_len * p->nch < p->T || p->nch > 4 || grid < 1)
    return -10;
  hipLaunchKernelGGL(wdec_kernel, dim3(grid), dim3(kT), kLds, st, *p);
  return (int)hipGetLastError();
}
