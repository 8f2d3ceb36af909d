// Audio front-end kernels (K1, K2) -- replace the Deepgram ingest/front-end
// (apps/voice/src/deepgram.ts:36-45, sendAudio :55-58).
//
//  pcm16_to_f32 : int16 -> f32 (/32768) with optional linear resampling (ratio = in_rate/16000)
//  log_mel      : Whisper log-mel spectrogram of a (30 s padded) window, computed on device:
//                 reflect-padded frames (n_fft 400, hop 160) x periodic Hann -> DFT power for
//                 201 bins and the mel projection, both as f32 MFMA GEMMs (logmel_mfma_kernel)
//                 -> log10(max(.,1e-10)); the global max is reduced with an order-preserving
//                 integer atomicMax; a second pass applies max(x, max-8), (x+4)/4 and writes
//                 bf16 channels-last [frames][n_mels] (the layout the conv1d stem consumes).
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

constexpr int kNFFT = 400, kHop = 160, kBins = 201;

__global__ __launch_bounds__(256) void pcm_kernel(const int16_t* __restrict__ pcm, float* __restrict__ out, int n_in,
                                                  int n_out, float ratio) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_out) return;
  if (ratio == 1.f) {
    out[i] = (float)pcm[i] * (1.f / 32768.f);
    return;
  }
  const float src = i * ratio;
  int j = (int)src;
  const float f = src - j;
  const int j1 = min(j + 1, n_in - 1);
  j = min(j, n_in - 1);
  out[i] = ((1.f - f) * pcm[j] + f * pcm[j1]) * (1.f / 32768.f);
}

VWA_DEVICE int reflect(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

VWA_DEVICE int f2ord(float f) {
  int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7fffffff;
}
VWA_DEVICE float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// ---- log-mel power + mel projection on the f32 MFMA (v_mfma_f32_16x16x4_f32: exact f32 in,
// f32 accumulate -- the spectrum keeps full precision).  One 512-thread workgroup per 16 frames:
//   frames [16][400] (reflect-padded, Hann-windowed) -> LDS
//   DFT:  C_cos / C_sin [16 frames][208 bins] = frames . basis   (13 bin tiles of 16, cos and sin
//         tiles of a bin tile in the same wave: power = c^2 + s^2 in registers) -> LDS
//   mel:  [16 frames][n_mels] = power . fb^T                     (one 16-mel tile per wave)
//   log10(max(., 1e-10)) -> f32 scratch + the global max (order-preserving integer atomicMax).
// The DFT basis (exact-phase cos / sin of 2 pi k n / 400, f64 on the host) and the filterbank are
// pre-arranged in MFMA fragment order: [tile][k-step / 4][lane][4] -- one 16-byte load per lane
// per 4 k-steps (ops.logmel_tables).  Replaces a per-bin O(N^2) VALU DFT (138 us per 30 s window,
// 58 % LDS bank conflicts: profiles/r3_pmc_counters.md row 11).
constexpr int kLmFrames = 16;        // frames per workgroup (MFMA rows)
constexpr int kLmBinTiles = 13;      // 208 >= 201 bins
constexpr int kLmXLd = 450;          // LDS row strides (floats) of the frame / power images:
constexpr int kLmPLd = 258;          //   = 2 (mod 64): the A reads (16 rows x 4 k) hit distinct banks
                                     //   per 32-lane half (20 mod 64 measured 45 % conflicts)
constexpr int kLmWaves = 8;

typedef float f32x4_t __attribute__((ext_vector_type(4)));
VWA_DEVICE f32x4 mfma_f32(float a, float b, const f32x4& c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

__global__ __launch_bounds__(kLmWaves * 64) void logmel_mfma_kernel(const float* __restrict__ audio, int n_samples,
                                                                   int n_frames, const float* __restrict__ window,
                                                                   const float4* __restrict__ basis,
                                                                   const float4* __restrict__ fbf, int n_mels,
                                                                   float* __restrict__ mel_out, int* __restrict__ max_buf) {
  __shared__ float xs[kLmFrames * kLmXLd];
  __shared__ float ps[kLmFrames * kLmPLd];
  __shared__ float red[kLmWaves];
  const int f0 = blockIdx.x * kLmFrames;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
  {  // all 13 gathers of a thread in flight together (a rolled loop waits one round trip each)
    constexpr int NG = (kLmFrames * kNFFT + kLmWaves * 64 - 1) / (kLmWaves * 64);
    float v[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int i = threadIdx.x + g * kLmWaves * 64;
      const int fr = i / kNFFT, n = i % kNFFT, f = f0 + fr;
      v[g] = (i < kLmFrames * kNFFT && f < n_frames) ? audio[reflect(f * kHop + n - kNFFT / 2, n_samples)] * window[n]
                                                      : 0.f;
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int i = threadIdx.x + g * kLmWaves * 64;
      if (i < kLmFrames * kNFFT) xs[(i / kNFFT) * kLmXLd + i % kNFFT] = v[g];
    }
  }
  __syncthreads();

  // ---- DFT: wave w takes bin tiles w and w + 8 (< 13)
  {
    const int nbt = (w + kLmWaves < kLmBinTiles) ? 2 : 1;
    f32x4 ac[2], as[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      ac[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      as[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const float* xr = xs + r * kLmXLd + kq;
    // basis fragments one 4-step group ahead (an L2 round trip per group otherwise stalls the
    // MFMA chain: 25 groups x ~600 cycles)
    const float4* bp[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int bt = min(w + t * kLmWaves, kLmBinTiles - 1);
      bp[t][0] = basis + (2 * bt) * (kNFFT / 16) * 64 + lane;
      bp[t][1] = basis + (2 * bt + 1) * (kNFFT / 16) * 64 + lane;
    }
    float4 nc[2], ns[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      nc[t] = bp[t][0][0];
      ns[t] = bp[t][1][0];
    }
    for (int s4 = 0; s4 < kNFFT / 16; ++s4) {
      float4 bc[2], bs[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        bc[t] = nc[t];
        bs[t] = ns[t];
      }
      if (s4 + 1 < kNFFT / 16) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          nc[t] = bp[t][0][(s4 + 1) * 64];
          ns[t] = bp[t][1][(s4 + 1) * 64];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = xr[(4 * s4 + j) * 4];
        const float* c0 = reinterpret_cast<const float*>(&bc[0]);
        const float* s0 = reinterpret_cast<const float*>(&bs[0]);
        ac[0] = mfma_f32(a, c0[j], ac[0]);
        as[0] = mfma_f32(a, s0[j], as[0]);
        if (nbt > 1) {
          const float* c1 = reinterpret_cast<const float*>(&bc[1]);
          const float* s1 = reinterpret_cast<const float*>(&bs[1]);
          ac[1] = mfma_f32(a, c1[j], ac[1]);
          as[1] = mfma_f32(a, s1[j], as[1]);
        }
      }
    }
    // power -> LDS: lane holds C[frame 4 kq + i][bin 16 bt + r]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t >= nbt) break;
      const int bt = w + t * kLmWaves;
#pragma unroll
      for (int i = 0; i < 4; ++i) ps[(4 * kq + i) * kLmPLd + 16 * bt + r] = ac[t][i] * ac[t][i] + as[t][i] * as[t][i];
    }
  }
  __syncthreads();

  // ---- mel projection: wave w takes mel tile w (n_mels <= 128)
  float lmax = -INFINITY;
  if (16 * w < n_mels) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* pr = ps + r * kLmPLd + kq;
    float4 fb[kLmBinTiles];  // all 13 filterbank fragments in flight at once
#pragma unroll
    for (int s4 = 0; s4 < kLmBinTiles; ++s4) fb[s4] = fbf[(w * kLmBinTiles + s4) * 64 + lane];
#pragma unroll
    for (int s4 = 0; s4 < kLmBinTiles; ++s4) {  // 52 k-steps of 4 bins
      const float* bb = reinterpret_cast<const float*>(&fb[s4]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = mfma_f32(pr[(4 * s4 + j) * 4], bb[j], acc);
    }
    const int m = 16 * w + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = f0 + 4 * kq + i;
      if (f < n_frames && m < n_mels) {
        const float lv = log10f(fmaxf(acc[i], 1e-10f));
        mel_out[(int64_t)f * n_mels + m] = lv;
        lmax = fmaxf(lmax, lv);
      }
    }
  }
  lmax = wave_max(lmax);
  if (lane == 0) red[w] = lmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mx = red[0];
#pragma unroll
    for (int i = 1; i < kLmWaves; ++i) mx = fmaxf(mx, red[i]);
    atomicMax(max_buf, f2ord(mx));
  }
}

__global__ __launch_bounds__(256) void logmel_norm_kernel(const float* __restrict__ mel, const int* __restrict__ max_buf,
                                                          u16* __restrict__ out, int n, int ld_out, int n_mels) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float mx = ord2f(max_buf[0]);
  const float v = (fmaxf(mel[i], mx - 8.f) + 4.f) * 0.25f;
  const int f = i / n_mels, m = i % n_mels;
  out[(int64_t)f * ld_out + m] = f2bf(v);
}

}  // namespace

extern "C" int vwa_pcm16_to_f32(const int16_t* pcm, float* out, int n_in, int n_out, float ratio, hipStream_t st) {
  hipLaunchKernelGGL(pcm_kernel, dim3((n_out + 255) / 256), dim3(256), 0, st, pcm, out, n_in, n_out, ratio);
  return (int)hipGetLastError();
}

extern "C" int vwa_log_mel(const float* audio, int n_samples, int n_frames, const float* window, const float* basis,
                           const float* fb_frag, int n_mels, float* mel_out, float* max_buf, uint16_t* out_bf16,
                           int ld_out, hipStream_t st) {
  if (n_mels < 1 || n_mels > 16 * kLmWaves || n_frames < 1 || n_samples <= kNFFT / 2) return -1;
  int* mb = reinterpret_cast<int*>(max_buf);
  // order-preserving encoding of -inf is a large negative int; reset every call (graph-safe memset node)
  hipMemsetAsync(mb, 0x80, sizeof(int), st);
  hipLaunchKernelGGL(logmel_mfma_kernel, dim3((n_frames + kLmFrames - 1) / kLmFrames), dim3(kLmWaves * 64), 0, st,
                     audio, n_samples, n_frames, window, reinterpret_cast<const float4*>(basis),
                     reinterpret_cast<const float4*>(fb_frag), n_mels, mel_out, mb);
  const int n = n_frames * n_mels;
  hipLaunchKernelGGL(logmel_norm_kernel, dim3((n + 255) / 256), dim3(256), 0, st, mel_out, mb, out_bf16, n, ld_out,
                     n_mels);
  return (int)hipGetLastError();
}
