// Audio front-end kernels (K1, K2) -- replace the Deepgram ingest/front-end
// (apps/voice/src/deepgram.ts:36-45, sendAudio :55-58).
//
//  pcm16_to_f32 : int16 -> f32 (/32768) with optional linear resampling (ratio = in_rate/16000)
//  log_mel      : Whisper log-mel spectrogram of a (30 s padded) window, computed on device:
//                 reflect-padded frames (n_fft 400, hop 160) x periodic Hann -> DFT power for
//                 201 bins (twiddles from a 400-entry cos table in LDS, exact integer phase
//                 (k*n mod 400)) -> mel filterbank -> log10(max(.,1e-10)); the global max is
//                 reduced with an order-preserving integer atomicMax; a second pass applies
//                 max(x, max-8), (x+4)/4 and writes bf16 channels-last [frames][n_mels]
//                 (the layout the conv1d stem consumes).
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

// one workgroup per frame
__global__ __launch_bounds__(256) void logmel_frame_kernel(const float* __restrict__ audio, int n_samples,
                                                           int n_frames, const float* __restrict__ window,
                                                           const float* __restrict__ cos_table,
                                                           const float* __restrict__ mel_fb, int n_mels,
                                                           float* __restrict__ mel_out, int* __restrict__ max_buf) {
  __shared__ float xs[kNFFT];
  __shared__ float ct[kNFFT];
  __shared__ float pw[kBins + 3];
  __shared__ float red[4];
  const int f = blockIdx.x;
  for (int n = threadIdx.x; n < kNFFT; n += 256) {
    const int idx = reflect(f * kHop + n - kNFFT / 2, n_samples);
    xs[n] = audio[idx] * window[n];
    ct[n] = cos_table[n];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kBins; k += 256) {
    float re = 0.f, im = 0.f;
    int ph = 0;  // (k*n) mod 400
    for (int n = 0; n < kNFFT; ++n) {
      const float x = xs[n];
      re += x * ct[ph];
      // sin(2*pi*ph/400) = cos(2*pi*(ph - 100)/400)
      int ps = ph - 100;
      if (ps < 0) ps += kNFFT;
      im -= x * ct[ps];
      ph += k;
      if (ph >= kNFFT) ph -= kNFFT;
    }
    pw[k] = re * re + im * im;
  }
  __syncthreads();
  float lmax = -INFINITY;
  for (int m = threadIdx.x; m < n_mels; m += 256) {
    const float* fb = mel_fb + (int64_t)m * kBins;
    float acc = 0.f;
    for (int k = 0; k < kBins; ++k) acc += fb[k] * pw[k];
    const float lv = log10f(fmaxf(acc, 1e-10f));
    mel_out[(int64_t)f * n_mels + m] = lv;
    lmax = fmaxf(lmax, lv);
  }
  lmax = wave_max(lmax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = lmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
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

extern "C" int vwa_log_mel(const float* audio, int n_samples, int n_frames, const float* window, const float* dft_cos,
                           const float* dft_sin, const float* mel_fb, int n_mels, float* mel_out, float* max_buf,
                           uint16_t* out_bf16, int ld_out, hipStream_t st) {
  (void)dft_sin;
  int* mb = reinterpret_cast<int*>(max_buf);
  // order-preserving encoding of -inf is a large negative int; reset every call (graph-safe memset node)
  hipMemsetAsync(mb, 0x80, sizeof(int), st);
  hipLaunchKernelGGL(logmel_frame_kernel, dim3(n_frames), dim3(256), 0, st, audio, n_samples, n_frames, window, dft_cos,
                     mel_fb, n_mels, mel_out, mb);
  const int n = n_frames * n_mels;
  hipLaunchKernelGGL(logmel_norm_kernel, dim3((n + 255) / 256), dim3(256), 0, st, mel_out, mb, out_bf16, n, ld_out,
                     n_mels);
  return (int)hipGetLastError();
}
