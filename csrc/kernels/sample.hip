// Grammar-masked sampling (K13).
//
// Replaces the remote JSON-mode sampling of the reference (response_format json_object,
// temperature 0.1: apps/brain/src/llm.ts:24-25).  The grammar engine (csrc/grammar) produces
// a token bitmask per row (vocab 128256 -> 4008 u32 words); this kernel applies it and
// draws a token with the Gumbel-max trick:
//     token = argmax_v  [mask(v)] * (logit_v / T + G_v),   G_v = -log(-log(u_v))
// (T <= 0 -> greedy argmax).  u_v comes from a counter-based hash of (seed, step, row, v),
// so the draw is reproducible and the kernel is hipGraph-replayable: `step` lives in device
// memory and is advanced by the last stage of the kernel itself.
// Two stages: (rows x n_chunks) partial argmax workgroups, then one workgroup per row.
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

VWA_DEVICE uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

VWA_DEVICE void argmax_merge(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

constexpr int kMaskWordsMax = 4096;  // mask words per chunk staged in LDS (16 KB)

__global__ __launch_bounds__(256) void sample_partial_kernel(const float* __restrict__ logits, int ld, int V,
                                                             int v_off, const uint32_t* __restrict__ mask,
                                                             int mask_words,
                                                             const float* __restrict__ temperature,
                                                             const uint64_t* __restrict__ seed,
                                                             const int* __restrict__ step, float* part_val,
                                                             int* part_idx, int n_chunks) {
  __shared__ float sv[256];
  __shared__ int si[256];
  __shared__ uint32_t smask[kMaskWordsMax];
  const int row = blockIdx.x, chunk = blockIdx.y;
  const int per = (V + n_chunks - 1) / n_chunks;
  const int v0 = chunk * per, v1 = min(V, v0 + per);
  // the chunk's mask words, all loaded at once into LDS: the mask may live in pinned HOST memory
  // (zero-copy: no H2D copy per step), where a per-token load would be a PCIe round trip each
  // (v_off: global id of local column 0 under vocab parallelism, a multiple of 32)
  const int w0 = v0 >> 5, nw = v1 > v0 ? ((v1 - 1) >> 5) - w0 + 1 : 0;
  if (mask)
    for (int i = threadIdx.x; i < nw; i += 256) smask[i] = mask[(int64_t)row * mask_words + (v_off >> 5) + w0 + i];
  __syncthreads();
  const float T = temperature ? temperature[row] : 0.f;
  const float invT = T > 0.f ? 1.f / T : 1.f;
  const uint64_t base = splitmix64(seed[0] ^ splitmix64((uint64_t)step[0] * 0x100000001B3ull + row));
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int v = v0 + threadIdx.x; v < v1; v += 256) {
    if (mask) {
      const uint32_t wd = smask[(v >> 5) - w0];
      if (!((wd >> (v & 31)) & 1u)) continue;
    }
    float key = logits[(int64_t)row * ld + v];
    const int gv = v_off + v;  // global token id: the noise and the index are vocab-shard invariant
    if (T > 0.f) {
      const uint64_t h = splitmix64(base ^ (uint64_t)gv);
      const float u = ((float)(h >> 41) + 0.5f) * (1.0f / 8388608.0f);  // in (0,1), exact in f32
      key = key * invT - __logf(-__logf(u));
    }
    argmax_merge(bv, bi, key, gv);
  }
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      float ov = sv[threadIdx.x + s];
      int oi = si[threadIdx.x + s];
      float cv = sv[threadIdx.x];
      int ci = si[threadIdx.x];
      argmax_merge(cv, ci, ov, oi);
      sv[threadIdx.x] = cv;
      si[threadIdx.x] = ci;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part_val[row * n_chunks + chunk] = sv[0];
    part_idx[row * n_chunks + chunk] = si[0];
  }
}

__global__ __launch_bounds__(256) void sample_final_kernel(const float* __restrict__ part_val,
                                                           const int* __restrict__ part_idx, int n_chunks,
                                                           int n_src, int64_t src_stride,
                                                           int* out_tokens, int* step, int rows,
                                                           const int64_t* __restrict__ fail_word) {
  __shared__ float sv[256];
  __shared__ int si[256];
  const int row = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int p = 0; p < n_src; ++p)
    for (int c = threadIdx.x; c < n_chunks; c += 256)
      argmax_merge(bv, bi, part_val[p * src_stride + row * n_chunks + c], part_idx[p * src_stride + row * n_chunks + c]);
  sv[threadIdx.x] = bv;
  si[threadIdx.x] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      float cv = sv[threadIdx.x];
      int ci = si[threadIdx.x];
      argmax_merge(cv, ci, sv[threadIdx.x + s], si[threadIdx.x + s]);
      sv[threadIdx.x] = cv;
      si[threadIdx.x] = ci;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    // no admissible token (empty mask) -> -1, the host treats it as a grammar error; a set
    // fail word (the forward's chained launch timed out at a grid barrier, so these logits are
    // invalid) -> -2 in every row: the host re-runs the step on the per-kernel path
    const bool failed = fail_word != nullptr && fail_word[0] != 0;
    // system scope: out_tokens may be pinned host memory the host polls (no D2H copy per step)
    __hip_atomic_store(out_tokens + row, failed ? -2 : (sv[0] == -INFINITY) ? -1 : si[0], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    if (row == rows - 1) step[0] += 1;
  }
}

}  // namespace

extern "C" int vwa_sample_partial(const float* logits, int ld, int rows, int V, int v_off, const uint32_t* mask,
                                  int mask_words, const float* temperature, const uint64_t* seed, const int* step,
                                  float* part_val, int* part_idx, int n_chunks, hipStream_t st) {
  if (n_chunks < 1 || n_chunks > 1024 || rows < 1 || (v_off & 31)) return -1;
  if (mask && ((V + n_chunks - 1) / n_chunks + 31) / 32 + 1 > kMaskWordsMax) return -10;
  if (mask && (int64_t)mask_words * 32 < (int64_t)v_off + V) return -11;
  hipLaunchKernelGGL(sample_partial_kernel, dim3(rows, n_chunks), dim3(256), 0, st, logits, ld, V, v_off, mask,
                     mask_words, temperature, seed, step, part_val, part_idx, n_chunks);
  return (int)hipGetLastError();
}

extern "C" int vwa_sample_final(const float* part_val, const int* part_idx, int n_chunks, int n_src,
                                int64_t src_stride, int* out_tokens, int* step, int rows, const int64_t* fail_word,
                                hipStream_t st) {
  if (n_chunks < 1 || n_src < 1 || rows < 1) return -1;
  hipLaunchKernelGGL(sample_final_kernel, dim3(rows), dim3(256), 0, st, part_val, part_idx, n_chunks, n_src,
                     src_stride, out_tokens, step, rows, fail_word);
  return (int)hipGetLastError();
}

extern "C" int vwa_sample(const float* logits, int ld, int rows, int V, const uint32_t* mask, int mask_words,
                          const float* temperature, const uint64_t* seed, const int* step, int* out_tokens,
                          float* part_val, int* part_idx, int n_chunks, const int64_t* fail_word, hipStream_t st) {
  const int r = vwa_sample_partial(logits, ld, rows, V, 0, mask, mask_words, temperature, seed, step, part_val,
                                   part_idx, n_chunks, st);
  if (r) return r;
  return vwa_sample_final(part_val, part_idx, n_chunks, 1, 0, out_tokens, const_cast<int*>(step), rows, fail_word, st);
}
