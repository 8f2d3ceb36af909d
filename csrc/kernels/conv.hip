// Whisper encoder stem (K3): conv1d(k=3, pad=1, stride s) + bias + GELU [+ positional
// embedding], as an implicit GEMM on MFMA (16x16x32 bf16).
//
//   y[b][t][co] = gelu( bias[co] + sum_{kk,ci} W[co][kk][ci] * x[b][t*s + kk - 1][ci] ) (+ pos[t][co])
//
// Channels-last everywhere (x [B][Tin][Cin], y [B][Tout][Cout]) so the GEMM's k index
// (kk, ci) walks contiguous memory: A fragments are 16-byte row loads of x, B fragments are
// 16-byte loads of the [co][kk][ci]-permuted weights.  A workgroup (4 waves) computes a
// 64(t) x 64(co) output tile; each wave 16 t x 64 co (4 accumulators).
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

__global__ __launch_bounds__(256) void conv1d_gelu_kernel(const u16* __restrict__ x, const u16* __restrict__ w,
                                                          const u16* __restrict__ bias, const u16* __restrict__ pos,
                                                          u16* __restrict__ y, int Cin, int Tin, int Cout, int Tout,
                                                          int stride) {
  const int b = blockIdx.z;
  const int t_tile = blockIdx.x * 64, co_tile = blockIdx.y * 64;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int K = 3 * Cin;
  const int t = t_tile + wv * 16 + rl;  // A row for this lane
  const u16* xb = x + (int64_t)b * Tin * Cin;

  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += 32) {
    const int k = k0 + 8 * g;
    uint4 a = make_uint4(0, 0, 0, 0);
    if (k < K && t < Tout) {
      const int kk = k / Cin, ci = k % Cin;
      const int ti = t * stride + kk - 1;
      if (ti >= 0 && ti < Tin) a = *reinterpret_cast<const uint4*>(xb + (int64_t)ti * Cin + ci);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int co = co_tile + n * 16 + rl;
      uint4 bv = make_uint4(0, 0, 0, 0);
      if (k < K && co < Cout) bv = *reinterpret_cast<const uint4*>(w + (int64_t)co * K + k);
      acc[n] = mfma16(as_bf16x8(a), as_bf16x8(bv), acc[n]);
    }
  }
  // C layout: row (t) = 4*g + i, col (co) = rl
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int co = co_tile + n * 16 + rl;
    if (co >= Cout) continue;
    const float bb = bias ? bf2f(bias[co]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int to = t_tile + wv * 16 + 4 * g + i;
      if (to >= Tout) continue;
      float v = gelu_erf(acc[n][i] + bb);
      if (pos) v += bf2f(pos[(int64_t)to * Cout + co]);
      y[((int64_t)b * Tout + to) * Cout + co] = f2bf(v);
    }
  }
}

}  // namespace

extern "C" int vwa_conv1d_gelu_pos(const uint16_t* x, const uint16_t* w, const uint16_t* b, const uint16_t* pos,
                                   uint16_t* y, int B, int Cin, int Tin, int Cout, int Tout, int stride,
                                   hipStream_t st) {
  if (Cin % 8) return -1;
  dim3 grid((Tout + 63) / 64, (Cout + 63) / 64, B);
  hipLaunchKernelGGL(conv1d_gelu_kernel, grid, dim3(256), 0, st, x, w, b, pos, y, Cin, Tin, Cout, Tout, stride);
  return (int)hipGetLastError();
}
