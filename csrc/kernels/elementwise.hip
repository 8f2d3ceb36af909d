// Row-wise / element-wise memory-bound kernels (prefill + encoder paths).
// All use 16-byte (8 x bf16) vector accesses (guide G13) and one wave per row for the norms.
//
//  rmsnorm      : [resid_out = x + residual]; y = x * rsqrt(mean(x^2)+eps) * w     (Llama, K8)
//  layernorm    : [resid_out = x + residual]; y = (x-mu)*rstd*w + b                (Whisper/GPT-2, K4)
//  rope_kv_write: rotary + paged K/V scatter for a prefill QKV matrix in the permuted
//                 per-head layout produced by the fused weights                     (K9)
//  swiglu       : h = silu(g)*u on the interleaved gate/up layout                   (K11)
//  bias_act     : y = act(x + b) [+ residual]  (act: 0 none, 1 gelu)
//  embedding    : vocab-parallel row gather (+ learned positions)                   (K14)
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

__global__ __launch_bounds__(256) void rmsnorm_kernel(const u16* __restrict__ x, const u16* __restrict__ residual,
                                                      u16* __restrict__ residual_out, const u16* __restrict__ w,
                                                      u16* __restrict__ y, int rows, int D, int ldx, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = lane_id();
  if (row >= rows) return;
  const u16* xr = x + (size_t)row * ldx;
  float ss = 0.f;
  // D <= 8192 -> at most 16 chunks of 8 per lane; fully unrolled so v[][] stays in VGPRs
  float v[16][8];
#pragma unroll
  for (int nch = 0; nch < 16; ++nch) {
    const int c = lane * 8 + nch * 512;
    if (c >= D) break;
    uint4 a = *reinterpret_cast<const uint4*>(xr + c);
    unpack8(a, v[nch]);
    if (residual) {
      float r[8];
      unpack8(*reinterpret_cast<const uint4*>(residual + (size_t)row * D + c), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[nch][j] += r[j];
      *reinterpret_cast<uint4*>(residual_out + (size_t)row * D + c) = pack8(v[nch]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[nch][j] * v[nch][j];
  }
  ss = wave_sum(ss);
  const float rs = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane * 8 + i * 512;
    if (c >= D) break;
    float g[8], o[8];
    if (w) unpack8(*reinterpret_cast<const uint4*>(w + c), g);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = 1.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rs * g[j];
    *reinterpret_cast<uint4*>(y + (size_t)row * D + c) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void layernorm_kernel(const u16* __restrict__ x, const u16* __restrict__ residual,
                                                        u16* __restrict__ residual_out, const u16* __restrict__ w,
                                                        const u16* __restrict__ b, u16* __restrict__ y, int rows,
                                                        int D, int ldx, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = lane_id();
  if (row >= rows) return;
  const u16* xr = x + (size_t)row * ldx;
  float v[16][8];
  float s = 0.f;
#pragma unroll
  for (int nch = 0; nch < 16; ++nch) {
    const int c = lane * 8 + nch * 512;
    if (c >= D) break;
    unpack8(*reinterpret_cast<const uint4*>(xr + c), v[nch]);
    if (residual) {
      float r[8];
      unpack8(*reinterpret_cast<const uint4*>(residual + (size_t)row * D + c), r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[nch][j] += r[j];
      *reinterpret_cast<uint4*>(residual_out + (size_t)row * D + c) = pack8(v[nch]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[nch][j];
  }
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (lane * 8 + i * 512 >= D) break;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[i][j] - mu;
      q += d * d;
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = lane * 8 + i * 512;
    if (c >= D) break;
    float g[8], bb[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(w + c), g);
    unpack8(*reinterpret_cast<const uint4*>(b + c), bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mu) * rstd * g[j] + bb[j];
    *reinterpret_cast<uint4*>(y + (size_t)row * D + c) = pack8(o);
  }
}

// one thread per (row, head, 16-col tile, pair index 0..7): handles cols c and c^8 of the tile
__global__ __launch_bounds__(256) void rope_kv_kernel(const u16* __restrict__ qkv, int ldqkv, int rows, int nq,
                                                      int nkv, int hd, int use_rope, const int* __restrict__ positions,
                                                      const int64_t* __restrict__ slots, const float* __restrict__ rope,
                                                      u16* __restrict__ q_out, int ldq, u16* __restrict__ k_cache,
                                                      u16* __restrict__ v_cache, int block_size, int64_t sb,
                                                      int64_t sh, int64_t stok) {
  const int heads = nq + 2 * nkv;
  const int per_row = heads * hd / 2;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)rows * per_row) return;
  const int row = gid / per_row;
  const int r = gid % per_row;
  const int head = r / (hd / 2);
  const int within = r % (hd / 2);  // pair index 0 .. hd/2-1
  const int t = within >> 3, pi = within & 7;
  const int half = hd >> 1;
  const u16* base = qkv + (size_t)row * ldqkv + head * hd + t * 16;
  float x0 = bf2f(base[pi]);      // dim 8t+pi
  float x1 = bf2f(base[pi + 8]);  // dim half+8t+pi
  const bool is_v = head >= nq + nkv;
  if (use_rope && !is_v) {
    const int pos = positions[row];
    const int di = 8 * t + pi;
    const float c = rope[((size_t)pos * half + di) * 2], s = rope[((size_t)pos * half + di) * 2 + 1];
    const float y0 = x0 * c - x1 * s, y1 = x1 * c + x0 * s;
    x0 = y0;
    x1 = y1;
  }
  const int d0 = 8 * t + pi, d1 = half + 8 * t + pi;
  if (head < nq) {
    q_out[(size_t)row * ldq + head * hd + d0] = f2bf(x0);
    q_out[(size_t)row * ldq + head * hd + d1] = f2bf(x1);
  } else {
    const int64_t slot = slots[row];
    if (slot < 0) return;
    const int kvh = is_v ? head - nq - nkv : head - nq;
    const int64_t idx = (slot / block_size) * sb + kvh * sh + (slot % block_size) * stok;
    u16* dst = is_v ? v_cache : k_cache;
    dst[idx + d0] = f2bf(x0);
    dst[idx + d1] = f2bf(x1);
  }
}

// gu rows: per 32-col tile [16 gate | 16 up] -> h[row][tile*16 + i]
__global__ __launch_bounds__(256) void swiglu_kernel(const u16* __restrict__ gu, u16* __restrict__ h, int rows,
                                                     int F) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one per 8 outputs
  const int per_row = F / 8;
  if (gid >= (int64_t)rows * per_row) return;
  const int row = gid / per_row, c8 = gid % per_row;
  const int tile = c8 >> 1, sub = (c8 & 1) * 8;
  const u16* g = gu + (size_t)row * 2 * F + tile * 32 + sub;
  float gv[8], uv[8], o[8];
  unpack8(*reinterpret_cast<const uint4*>(g), gv);
  unpack8(*reinterpret_cast<const uint4*>(g + 16), uv);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = silu(gv[j]) * uv[j];
  *reinterpret_cast<uint4*>(h + (size_t)row * F + tile * 16 + sub) = pack8(o);
}

__global__ __launch_bounds__(256) void bias_act_kernel(const u16* __restrict__ x, const u16* __restrict__ bias,
                                                       const u16* __restrict__ residual, u16* __restrict__ y,
                                                       int rows, int N, int act) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = N / 8;
  if (gid >= (int64_t)rows * per_row) return;
  const int row = gid / per_row, c = (gid % per_row) * 8;
  float v[8], b[8];
  unpack8(*reinterpret_cast<const uint4*>(x + (size_t)row * N + c), v);
  if (bias) {
    unpack8(*reinterpret_cast<const uint4*>(bias + c), b);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += b[j];
  }
  if (act == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu_erf(v[j]);
  }
  if (residual) {
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>(residual + (size_t)row * N + c), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += r[j];
  }
  *reinterpret_cast<uint4*>(y + (size_t)row * N + c) = pack8(v);
}

__global__ __launch_bounds__(256) void embedding_kernel(const int* __restrict__ ids, const u16* __restrict__ table,
                                                        const u16* __restrict__ pos_table,
                                                        const int* __restrict__ positions, u16* __restrict__ out,
                                                        int rows, int D, int vs, int ve) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per_row = D / 8;
  if (gid >= (int64_t)rows * per_row) return;
  const int row = gid / per_row, c = (gid % per_row) * 8;
  const int id = ids[row];
  float v[8];
  if (id >= vs && id < ve) {
    unpack8(*reinterpret_cast<const uint4*>(table + (size_t)(id - vs) * D + c), v);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
  }
  if (pos_table) {
    float p[8];
    unpack8(*reinterpret_cast<const uint4*>(pos_table + (size_t)positions[row] * D + c), p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += p[j];
  }
  *reinterpret_cast<uint4*>(out + (size_t)row * D + c) = pack8(v);
}

// Per-row dynamic fp8 quantisation of activations for the large-M fp8 GEMM path (prefill):
// amax over the row -> scale = amax/448 -> e4m3 bytes.  One workgroup per row.  With rstd: the
// same pass also sums the squares (the RMSNorm 1/rms of a projection whose gamma is folded into
// W) -- one launch instead of quant + row_rstd (profiles/r4_prof_fp8_c32_kernel_stats.md: the two
// row kernels were 10.7 % of the 32-session fp8 GPU time, ~5 us each).
__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const u16* __restrict__ x, int ldx, int D,
                                                             uint8_t* __restrict__ q, float* __restrict__ scale,
                                                             float* __restrict__ rstd, float eps) {
  __shared__ float red[4], red2[4];
  const int row = blockIdx.x;
  const u16* xr = x + (size_t)row * ldx;
  float am = 0.f, ss = 0.f;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      am = fmaxf(am, fabsf(f[j]));
      ss += f[j] * f[j];
    }
  }
  am = wave_max(am);
  if (rstd) ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = am;
    red2[threadIdx.x >> 6] = ss;
  }
  __syncthreads();
  am = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sx = am > 0.f ? am * (1.f / 448.f) : 1.f;
  const float iv = 1.f / sx;
  if (threadIdx.x == 0) {
    scale[row] = sx;
    if (rstd) rstd[row] = rsqrtf((red2[0] + red2[1] + red2[2] + red2[3]) / (float)D + eps);
  }
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c), f);
    uint2 o;
    o.x = cvt_pk_fp8(f[0] * iv, f[1] * iv) | (cvt_pk_fp8(f[2] * iv, f[3] * iv) << 16);
    o.y = cvt_pk_fp8(f[4] * iv, f[5] * iv) | (cvt_pk_fp8(f[6] * iv, f[7] * iv) << 16);
    *reinterpret_cast<uint2*>(q + (size_t)row * D + c) = o;
  }
}

inline int nblk(int64_t n, int b) { return (int)((n + b - 1) / b); }

}  // namespace

extern "C" int vwa_quant_fp8_rows(const uint16_t* x, int ldx, int rows, int D, uint8_t* q, float* scale,
                                  float* rstd, float eps, hipStream_t st) {
  if (D % 8) return -1;
  hipLaunchKernelGGL(quant_fp8_rows_kernel, dim3(rows), dim3(256), 0, st, x, ldx, D, q, scale, rstd, eps);
  return (int)hipGetLastError();
}

extern "C" int vwa_rmsnorm(const uint16_t* x, const uint16_t* residual, uint16_t* residual_out, const uint16_t* w,
                           uint16_t* y, int rows, int D, int ldx, float eps, hipStream_t st) {
  if (D % 8 || D > 8192) return -1;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(nblk(rows, 4)), dim3(256), 0, st, x, residual, residual_out, w, y, rows, D,
                     ldx, eps);
  return (int)hipGetLastError();
}

extern "C" int vwa_layernorm(const uint16_t* x, const uint16_t* residual, uint16_t* residual_out, const uint16_t* w,
                             const uint16_t* b, uint16_t* y, int rows, int D, int ldx, float eps, hipStream_t st) {
  if (D % 8 || D > 8192) return -1;
  hipLaunchKernelGGL(layernorm_kernel, dim3(nblk(rows, 4)), dim3(256), 0, st, x, residual, residual_out, w, b, y,
                     rows, D, ldx, eps);
  return (int)hipGetLastError();
}

extern "C" int vwa_rope_kv_write(const uint16_t* qkv, int ldqkv, int rows, int n_q_heads, int n_kv_heads,
                                 int head_dim, int use_rope, const int* positions, const int64_t* slots,
                                 const float* rope, uint16_t* q_out, int ldq, uint16_t* k_cache, uint16_t* v_cache,
                                 int block_size, int64_t sb, int64_t sh, int64_t st_, hipStream_t st) {
  if (head_dim % 16) return -1;
  const int64_t n = (int64_t)rows * (n_q_heads + 2 * n_kv_heads) * head_dim / 2;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(nblk(n, 256)), dim3(256), 0, st, qkv, ldqkv, rows, n_q_heads, n_kv_heads,
                     head_dim, use_rope, positions, slots, rope, q_out, ldq, k_cache, v_cache, block_size, sb, sh,
                     st_);
  return (int)hipGetLastError();
}

extern "C" int vwa_swiglu(const uint16_t* gu, uint16_t* h, int rows, int F, hipStream_t st) {
  if (F % 16) return -1;
  hipLaunchKernelGGL(swiglu_kernel, dim3(nblk((int64_t)rows * F / 8, 256)), dim3(256), 0, st, gu, h, rows, F);
  return (int)hipGetLastError();
}

extern "C" int vwa_bias_act(const uint16_t* x, const uint16_t* bias, const uint16_t* residual, uint16_t* y, int rows,
                            int N, int act, hipStream_t st) {
  if (N % 8) return -1;
  hipLaunchKernelGGL(bias_act_kernel, dim3(nblk((int64_t)rows * N / 8, 256)), dim3(256), 0, st, x, bias, residual, y,
                     rows, N, act);
  return (int)hipGetLastError();
}

extern "C" int vwa_embedding(const int* ids, const uint16_t* table, const uint16_t* pos_table, const int* positions,
                             uint16_t* out, int rows, int D, int vocab_start, int vocab_end, hipStream_t st) {
  if (D % 8) return -1;
  hipLaunchKernelGGL(embedding_kernel, dim3(nblk((int64_t)rows * D / 8, 256)), dim3(256), 0, st, ids, table,
                     pos_table, positions, out, rows, D, vocab_start, vocab_end);
  return (int)hipGetLastError();
}

// ---- device-resident greedy decode (Whisper): after a step's sampler, feed the sampled token
// back as the next step's input and advance the row's position / context / KV slot, so a run of
// decode steps replays back to back with no host round trip.  out[*counter] records the token.
namespace {
__global__ void decode_advance_kernel(int* tokens, int* positions, int* ctx_lens, int64_t* slots, const int* sampled,
                                      int* out, int* counter, int max_out, int base_block, int block_size) {
  if (threadIdx.x != 0) return;
  const int tok = sampled[0];
  const int c = counter[0];
  if (c < max_out) out[c] = tok;
  counter[0] = c + 1;
  tokens[0] = tok;
  const int pos = positions[0] + 1;
  positions[0] = pos;
  ctx_lens[0] = pos + 1;
  slots[0] = (int64_t)(base_block + pos / block_size) * block_size + pos % block_size;
}
}  // namespace

extern "C" int vwa_decode_advance(int* tokens, int* positions, int* ctx_lens, int64_t* slots, const int* sampled,
                                  int* out, int* counter, int max_out, int base_block, int block_size,
                                  hipStream_t st) {
  hipLaunchKernelGGL(decode_advance_kernel, dim3(1), dim3(64), 0, st, tokens, positions, ctx_lens, slots, sampled, out,
                     counter, max_out, base_block, block_size);
  return (int)hipGetLastError();
}

