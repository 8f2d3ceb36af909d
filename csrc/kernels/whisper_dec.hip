// Persistent Whisper decoder step (whisper-large family: d = 1280, ffn = 4 d, head_dim 64), one
// row: ONE launch for every decoder layer.
//
// Why: the per-kernel decoder runs eight dependent launches per
// layer, each ~5-9 us of fixed latency (dispatch, X staging, the first weight bytes, reduce,
// epilogue) for 0.3-13 MB of weights -- 2.3 ms per token for ~1.6 GB, 7x off the HBM roofline.
// Here the eight levels of a layer are separated only by completion counters, and a workgroup's
// share of the NEXT use of each of its weight tiles is already in its registers: a level's
// critical path is the counter hand-off, the activation row (a few KB from L2 / MALL) and a few
// MFMAs -- the weight bytes stream in the background (each slot is refilled right after the level
// that consumed it, a full layer ahead of its next use).
//
// Levels of layer li (reference call site this replaces: /root/reference/apps/voice/src/
// deepgram.ts:36-45, the hosted recogniser):
//   0 QKV      LN1(x) . Wqkv^T + b -> q, self K / V cache row   (240 column tiles of 16)
//   1 SATT     self-attention of the row, one workgroup per head -> att
//   2 O        x1 = x + att . Wo^T + b                            (80 tiles)
//   3 XQ       LNx(x1) . Wxq^T + b -> q                           (80 tiles)
//   4 XATT     cross-attention partials, (head, key chunk) per workgroup, K / V chunk prefetched
//              into LDS by LDS-DMA a layer ahead
//   5 XO       x2 = x1 + merge(partials) . Wxo^T + b              (80 tiles; the merge is the X staging)
//   6 FC1      f = GELU(LN2(x2) . W1^T + b1)                      (320 tiles)
//   7 FC2      x3 = x2 + f . W2^T + b2                            (80 tiles, K = 5120)
// LayerNorms are folded into the weights (ops.fold_layernorm: y = rstd (x.Wg - mean c) + b'), the
// mean / rstd come from the staged row.  Hand-off: a producer workgroup drains its stores and adds
// 1 (no return) to its level's counter of its XCD group; consumers poll the sum of the eight group
// counters with scalar loads (uncached words: the poll does not queue behind vector loads).
// Counters are monotonic: a launch adds n_prod[level] x n_layers to each, so every workgroup
// derives the launch's base from the value it reads at its start.
//
// Weight slots: 5 slots x 5 loads of 1 KB per wave (100 VGPRs).  A 16-column tile of a K = 1280
// projection is 40 load-slices (k-group, 32-k slice) of the pre-tiled layout; wave w takes slices
// w, w + 8, ... -- 5 per wave = one slot.  An fc2 tile (K = 5120) is 20 per wave = slots 1..4.
// The role table (models/whisper.py wdec_roles) gives each workgroup its slots (level, tile, part,
// reload level), its self-attention head and its cross-attention item.
#include "common.h"
#include "vwa_kernels.h"

namespace {
using namespace vwa;

constexpr int kT = 512;           // threads (8 waves, K split over the waves)
constexpr int kSlots = 5, kLps = 5;
enum { LV_QKV = 0, LV_SATT, LV_O, LV_XQ, LV_XATT, LV_XO, LV_FC1, LV_FC2 };
// role row layout (kWdRole ints per workgroup)
enum { R_KIND = 0, R_TILE = 5, R_PART = 10, R_RELOAD = 15, R_SATT = 20, R_XATT = 21, R_XPRE = 22, R_WORK = 23 };
// LDS layout (bytes)
constexpr int L_XS = 0;          // bf16 activation row (<= 5120)
constexpr int L_RED = 10368;     // f32 [8][16] cross-wave partial sums of a tile / reductions
constexpr int L_STAT = 10880;    // f32 [16]: mean, rstd, row max / sum
constexpr int L_W8 = 10944;      // f32 [2][8] per-wave reduction values
constexpr int L_QF = 11008;      // f32 [64] query head
constexpr int L_P = 11264;       // f32 [512] attention weights
constexpr int L_OW = 13312;      // f32 [8][64] per-wave attention outputs
constexpr int L_VA = 15360;      // int [512] self-attention V row offsets (elements)
constexpr int L_KV = 65536;      // cross-attention K chunk [<= 384][64] bf16, V chunk at + 48 KB
constexpr int L_KVV = 49152;
constexpr int kLds = 163840;
constexpr int kMaxChunk = 384;
constexpr int kSpinLimit = 1 << 18;  // ~0.3 s: a non-resident workgroup ends the launch, not the GPU
constexpr int kErrWord = 1024;

VWA_DEVICE int gemm_of(int lvl) {
  return lvl == LV_QKV ? 0 : lvl == LV_O ? 1 : lvl == LV_XQ ? 2 : lvl == LV_XO ? 3 : lvl == LV_FC1 ? 4 : 5;
}

VWA_DEVICE __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(bytes < 0x7FFFFFF0ll ? bytes : 0x7FFFFFF0ll),
                                           0x00020000);
}

// sc1 (device-coherent) 16-byte load of data another workgroup wrote in this launch
VWA_DEVICE uint4 ld_sc1_b128(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}
VWA_DEVICE float ldf_sc1(const float* p) { return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE void stf_sc1(float* p, float v) { __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE u16 ldh_sc1(const u16* p) { return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
VWA_DEVICE void sth_sc1(u16* p, u16 v) { __hip_atomic_store(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

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
// word and goes on: that step's results are invalid, the host falls back to per-kernel launches)
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
        if (VWA_TX == 0) __hip_atomic_store(gp(p.cnt + kErrWord), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  lds_sync();
}

// this workgroup completed level lvl: every wave's stores are performed (the caller's vmcnt(0)),
// then one no-return add on the group counter
VWA_DEVICE void wd_arrive(const WdecParams& p, int lvl) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_sync();
  if (VWA_TX == 0)
    __hip_atomic_fetch_add(gp(lvl_cnt(p, lvl) + 16 * (blockIdx.x & 7)), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

VWA_DEVICE int n_cols(const WdecParams& p, int lvl) {
  return lvl == LV_QKV ? 3 * p.d : lvl == LV_FC1 ? p.ffn : p.d;
}
VWA_DEVICE int k_of(const WdecParams& p, int lvl) { return lvl == LV_FC2 ? p.ffn : p.d; }

// slot load: part `part` (5 load-slices per wave) of tile `tile` of level lvl's weight, layer li
VWA_DEVICE void wd_load(const WdecParams& p, int li, int lvl, int tile, int part, uint4 (&wr)[kLps]) {
  const WdecGemm& g = p.layers[li].g[gemm_of(lvl)];
  const int K = k_of(p, lvl), G = K >> 7;
  const __amdgpu_buffer_rsrc_t r = rsrc_of(g.W, (long long)n_cols(p, lvl) * K * 2);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
#pragma unroll
  for (int j = 0; j < kLps; ++j) {
    const int sl = w + 8 * (part * kLps + j), kg = sl >> 2, s4 = sl & 3;
    const unsigned off = ((unsigned)(tile * G + kg) * 4u + (unsigned)s4) * 1024u + (unsigned)lane * 16u;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    wr[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// the MFMAs of one slot: acc (row 0 = lanes 0..15, element 0) += X . W over the slot's slices
VWA_DEVICE void wd_mma(const char* lds, int part, const uint4 (&wr)[kLps], f32x4& acc) {
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6, nl = lane & 15, g = lane >> 4;
  const u16* xs = reinterpret_cast<const u16*>(lds + L_XS);
#pragma unroll
  for (int j = 0; j < kLps; ++j) {
    const int sl = w + 8 * (part * kLps + j), kg = sl >> 2, s4 = sl & 3;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (nl == 0) a = *reinterpret_cast<const uint4*>(xs + kg * 128 + 32 * g + 8 * s4);
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
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  const int n8 = (nk + 7) >> 3;  // 1 KB instructions (8 keys of 128 B) per tensor
  for (int r = w; r < 2 * n8; r += 8) {
    const bool isv = r >= n8;
    const int rr = isv ? r - n8 : r;
    const int kk = rr * 8 + (lane >> 3);
    const unsigned off = kk < nk ? (unsigned)(((((long long)sess * p.T + k0 + kk) * p.H + h) * 64 + (lane & 7) * 8) * 2)
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
  lds_sync();
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
  lds_sync();
  return s;
}

// q head h (bf16, written this launch) -> LDS f32 [64]
VWA_DEVICE void wd_q_to_lds(const WdecParams& p, int h, char* lds) {
  float* qf = reinterpret_cast<float*>(lds + L_QF);
  const int tx = VWA_TX;
  if (tx < 8) {
    const uint4 v = ld_sc1_b128(rsrc_of(p.q, (long long)p.d * 2), (unsigned)((h * 64 + tx * 8) * 2));
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int e = 0; e < 8; ++e) qf[tx * 8 + e] = f[e];
  }
  lds_sync();
}

// softmax over the thread-per-key scores s (keys t < nk, others -inf): returns (max, sum); P[t] in LDS
VWA_DEVICE float2 wd_softmax(char* lds, float s, bool valid) {
  float* P = reinterpret_cast<float*>(lds + L_P);
  const float m = blk_max(lds, valid ? s : -INFINITY);
  const float e = valid ? __expf(s - m) : 0.f;
  P[VWA_TX] = e;
  const float l = blk_sum(lds, e);  // (its barriers publish P)
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

// level 1: self-attention of head h over the row's context (<= 512 keys: one thread per key)
VWA_DEVICE void wd_self_attn(const WdecParams& p, int li, int h, char* lds) {
  const WdecLayer& L = p.layers[li];
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  const int seq = p.seq_ids[0], ctx = min(p.ctx_lens[0], kT);
  const int bs = p.block_size;
  int* va = reinterpret_cast<int*>(lds + L_VA);
  const float* qf = reinterpret_cast<const float*>(lds + L_QF);
  wd_q_to_lds(p, h, lds);
  const long long cache_bytes = 0x7FFFFFF0ll;
  const __amdgpu_buffer_rsrc_t rk = rsrc_of(L.k_cache, cache_bytes), rv = rsrc_of(L.v_cache, cache_bytes);
  float s = -INFINITY;
  const bool valid = tx < ctx;
  if (valid) {
    const int blk = p.block_table[seq * p.bt_stride + tx / bs];
    const int e0 = ((blk * p.H + h) * bs + tx % bs) * 64;  // element offset of key tx's row
    va[tx] = e0;
    uint4 kr[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) kr[c] = ld_sc1_b128(rk, (unsigned)(e0 * 2 + c * 16));
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
  const float2 ml = wd_softmax(lds, s, valid);  // (publishes va too)
  const float* P = reinterpret_cast<const float*>(lds + L_P);
  float o = 0.f;
  for (int t0 = w; t0 < ctx; t0 += 64) {  // 8 keys per wave per batch, loads first
    float vv[8];
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

// level 4: cross-attention partial of (head, chunk) from the prefetched K / V chunk in LDS
VWA_DEVICE void wd_cross_attn(const WdecParams& p, int item, char* lds) {
  const int h = item / p.nch, ch = item % p.nch;
  const int k0 = ch * p.ch_len, nk = min(p.ch_len, p.T - k0);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's K / V DMAs have landed
  wd_q_to_lds(p, h, lds);                            // (its barrier: every wave's DMAs)
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
      unpack8(*reinterpret_cast<const uint4*>(kl + tx * 64 + c * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += qf[c * 8 + e] * f[e];
    }
    s = acc * p.scale;
  }
  const float2 ml = wd_softmax(lds, s, valid);
  const float* P = reinterpret_cast<const float*>(lds + L_P);
  float o = 0.f;
  for (int t = w; t < nk; t += 8) o += P[t] * bf2f(vl[t * 64 + lane]);
  const float tot = wd_ow_sum(lds, o);
  float* part = p.xpart + (size_t)(h * p.nch + ch) * 66;
  if (tx < 64) stf_sc1(part + 2 + tx, tot);
  if (tx == 0) {
    stf_sc1(part, ml.x);
    stf_sc1(part + 1, ml.y);
  }
}

// X staging of a GEMM level: the activation row (bf16, written earlier in this launch) -> LDS;
// LayerNorm levels also get the row's mean / rstd (from the staged values)
VWA_DEVICE void wd_stage(const WdecParams& p, int lvl, const u16* x, char* lds, bool ln) {
  const int K = k_of(p, lvl), n8 = K >> 3;
  const int tx = VWA_TX;
  u16* xs = reinterpret_cast<u16*>(lds + L_XS);
  const __amdgpu_buffer_rsrc_t r = rsrc_of(x, (long long)K * 2);
  uint4 v[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tx + i * kT;
    v[i] = c < n8 ? ld_sc1_b128(r, (unsigned)c * 16u) : make_uint4(0, 0, 0, 0);
  }
  float s = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tx + i * kT;
    if (c < n8) {
      *reinterpret_cast<uint4*>(xs + c * 8) = v[i];
      if (ln) {
        float f[8];
        unpack8(v[i], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s += f[e];
          s2 += f[e] * f[e];
        }
      }
    }
  }
  if (ln) {
    float* st = reinterpret_cast<float*>(lds + L_STAT);
    const float ts = blk_sum(lds, s), ts2 = blk_sum(lds, s2);
    if (tx == 0) {
      const float mean = ts / (float)K;
      st[0] = mean;
      st[1] = rsqrtf(fmaxf(ts2 / (float)K - mean * mean, 0.f) + p.eps);
    }
  }
  lds_sync();
}

// X staging of the cross out-projection: the attention row merged from the (head, chunk)
// partials (chunk order fixed: the same bits whoever finished last)
VWA_DEVICE void wd_stage_merge(const WdecParams& p, char* lds) {
  u16* xs = reinterpret_cast<u16*>(lds + L_XS);
  const int tx = VWA_TX, nch = p.nch;
  for (int c = tx; c < p.d; c += kT) {
    const int h = c >> 6, dd = c & 63;
    const float* base = p.xpart + (size_t)h * nch * 66;
    float m[8], l[8], o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < nch) {
        m[k] = ldf_sc1(base + k * 66);
        l[k] = ldf_sc1(base + k * 66 + 1);
        o[k] = ldf_sc1(base + k * 66 + 2 + dd);
      }
    }
    float mx = m[0];
#pragma unroll
    for (int k = 1; k < 8; ++k)
      if (k < nch) mx = fmaxf(mx, m[k]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < nch) {
        const float e = __expf(m[k] - mx);
        num += e * o[k];
        den += e * l[k];
      }
    xs[c] = f2bf(num / den);
  }
  lds_sync();
}

// cross-wave sum of a tile's 16 columns + the level's epilogue (threads 0..15 store)
VWA_DEVICE void wd_epilogue(const WdecParams& p, int li, int lvl, int tile, f32x4& acc, char* lds,
                            const u16* xres, u16* xout) {
  float* red = reinterpret_cast<float*>(lds + L_RED);
  const float* st = reinterpret_cast<const float*>(lds + L_STAT);
  const int tx = VWA_TX, lane = tx & 63, w = tx >> 6;
  if (lane < 16) red[w * 16 + lane] = acc[0];
  acc = f32x4{0.f, 0.f, 0.f, 0.f};
  lds_sync();
  if (tx < 16) {
    const WdecGemm& g = p.layers[li].g[gemm_of(lvl)];
    const int n = tile * 16 + tx;
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) v += red[ww * 16 + tx];
    if (g.ln_c) v = (v - st[0] * g.ln_c[n]) * st[1];
    if (g.bias) v += bf2f(g.bias[n]);
    if (lvl == LV_FC1) v = gelu_erf(v);
    if (lvl == LV_O || lvl == LV_XO || lvl == LV_FC2) {
      v += bf2f(ldh_sc1(xres + n));
      sth_sc1(xout + n, f2bf(v));
    } else if (lvl == LV_FC1) {
      sth_sc1(p.f + n, f2bf(v));
    } else if (lvl == LV_XQ) {
      sth_sc1(p.q + n, f2bf(v));
    } else {  // QKV: rows permuted per head (ops.permute_qkv_rows: rotary pairs c, c ^ 8)
      const int n0 = tile * 16, head = n0 >> 6, t4 = (n0 & 63) >> 4, q = tx;
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
  lds_sync();  // (red is reused by the next tile)
}

__global__ __launch_bounds__(kT) void wdec_kernel(WdecParams p) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int* rr = p.roles + (size_t)blockIdx.x * kWdRole;
  int kind[kSlots], tile[kSlots], part[kSlots], rl[kSlots];
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    kind[s] = rr[R_KIND + s];
    tile[s] = rr[R_TILE + s];
    part[s] = rr[R_PART + s];
    rl[s] = rr[R_RELOAD + s];
  }
  const int sattn = rr[R_SATT], xattn = rr[R_XATT], xpre = rr[R_XPRE], work = rr[R_WORK];
  if (work == 0) return;
  const int NL = p.n_layers;
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
  uint4 wr[kSlots][kLps];
  // initial slot loads: slots refilled after their use (reload level >= level) hold layer 0 now
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
#pragma unroll
    for (int j = 0; j < kLps; ++j) wr[s][j] = make_uint4(0, 0, 0, 0);
    if (kind[s] >= 0 && rl[s] >= kind[s]) wd_load(p, 0, kind[s], tile[s], part[s], wr[s]);
  }
  if (xattn >= 0 && xpre >= LV_XATT) wd_kv_prefetch(p, 0, xattn, lds);

  for (int li = 0; li < NL; ++li) {
    uint16_t* xc = (li & 1) ? p.x1 : p.x0;  // this layer's input row
    uint16_t* xo = (li & 1) ? p.x0 : p.x1;
    for (int lvl = 0; lvl < kWdLevels; ++lvl) {
      if (!((work >> lvl) & 1)) continue;
      // inputs: the previous level of this layer (or the last level of the previous layer)
      if (li > 0 || lvl > 0) {
        const int pl = lvl > 0 ? lvl - 1 : kWdLevels - 1, pli = lvl > 0 ? li : li - 1;
        wd_wait(p, pl, base[pl] + (unsigned long long)p.n_prod[pl] * (unsigned long long)(pli + 1));
      }
      if (lvl == LV_SATT) {
        wd_self_attn(p, li, sattn, lds);
      } else if (lvl == LV_XATT) {
        wd_cross_attn(p, xattn, lds);
      } else {
        // activation row + residual of this level
        const u16* xin = lvl == LV_QKV ? xc : lvl == LV_O ? p.att : lvl == LV_XQ ? xo : lvl == LV_FC1 ? xc
                       : lvl == LV_FC2 ? p.f : nullptr;
        const u16* xres = lvl == LV_O ? xc : lvl == LV_XO ? xo : xc;
        u16* xout = lvl == LV_O ? xo : lvl == LV_XO ? xc : xo;
        if (lvl == LV_XO) wd_stage_merge(p, lds);
        else wd_stage(p, lvl, xin, lds, lvl == LV_QKV || lvl == LV_XQ || lvl == LV_FC1);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
          if (kind[s] != lvl) continue;
          wd_mma(lds, part[s], wr[s], acc);
          const bool last = s == kSlots - 1 || kind[s + 1] != lvl || tile[s + 1] != tile[s];
          if (last) wd_epilogue(p, li, lvl, tile[s], acc, lds, xres, xout);
        }
      }
      wd_arrive(p, lvl);
      // refills a layer ahead (after the arrival: its vmcnt(0) must not wait for them)
#pragma unroll
      for (int s = 0; s < kSlots; ++s) {
        if (kind[s] >= 0 && rl[s] == lvl) {
          const int lt = rl[s] < kind[s] ? li : li + 1;
          if (lt < NL) wd_load(p, lt, kind[s], tile[s], part[s], wr[s]);
        }
      }
      if (xattn >= 0 && xpre == lvl) {
        const int lt = xpre < LV_XATT ? li : li + 1;
        if (lt < NL) {
          if (lvl == LV_XATT) lds_sync();  // (every wave done reading the chunk)
          wd_kv_prefetch(p, lt, xattn, lds);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (no LDS-DMA outstanding at the end)
}

}  // namespace

extern "C" int vwa_wdec_launch(const WdecParams* p, int grid, hipStream_t st) {
  if (p->d != 1280 || p->ffn != 4 * p->d || p->H * 64 != p->d || p->n_layers < 2 || p->ch_len > kMaxChunk ||
      p->ch_len * p->nch < p->T || p->nch > 8 || grid < 1)
    return -10;
  hipLaunchKernelGGL(wdec_kernel, dim3(grid), dim3(kT), kLds, st, *p);
  return (int)hipGetLastError();
}
