// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//  * activations / weights are bf16 stored as uint16_t bit patterns; math is f32;
//  * 16-byte vector loads (8 x bf16) everywhere on memory-bound paths;
//  * wave = 64 lanes; block sizes are multiples of 64;
//  * MFMA: __builtin_amdgcn_mfma_f32_16x16x32_bf16, lane maps:
//      A: lane l holds A[row l&15][k 8*(l>>4)+j], j=0..7
//      B: lane l holds B[k 8*(l>>4)+j][col l&15]
//      C: lane l holds C[row 4*(l>>4)+i][col l&15], i=0..3
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define VWA_DEVICE __device__ __forceinline__

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

namespace vwa {

constexpr int kWave = 64;

// Global-address-space view of a pointer.  Pointers read from a descriptor are generic, and a
// generic (FLAT) access also counts on lgkmcnt: every later wait for an LDS op or a lane shuffle
// then waits for it as well.  Accesses through gp() are global_* instructions (vmcnt only).
template <class T>
VWA_DEVICE __attribute__((address_space(1))) T* gp(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
template <class T>
VWA_DEVICE T gld(const T* p) {
  return *gp(p);
}

VWA_DEVICE float bf2f(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }

VWA_DEVICE u16 f2bf(float f) {
  // round-to-nearest-even via the hardware convert (v_cvt_pk_bf16_f32 on gfx950); keeps NaN a NaN
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
VWA_DEVICE uint32_t pack2(float a, float b) {
  // one v_cvt_pk_bf16_f32 (RNE) for the pair (two scalar converts + shift/or otherwise)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// max of three as ONE v_maximum3_f32 (gfx950), visible to the compiler: fmaxf would put a
// canonicalising v_max in front of every MFMA result, and the inline-asm v_max3_f32 used until
// round 5 hid its operands from the hazard recognizer -- in the flash kernel's non-masked path it
// read the last 32x32 MFMA's accumulators 3 SALU instructions after the MFMA (gfx950 needs 12 wait
// states: the compiler now emits s_nop 11 there), so tmax could see a stale score and the deferred
// rescale moved from launch to launch.  fmaximum propagates NaN, which no
// score can be (masked keys are -inf).
VWA_DEVICE float vmax3(float a, float b, float c) {
  return __builtin_elementwise_maximum(a, __builtin_elementwise_maximum(b, c));
}

// the value of lane l ^ 32 combined with lane l's: v_permlane32_swap (VALU; no LDS round trip)
VWA_DEVICE float max_halves(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax3(__uint_as_float(s[0]), __uint_as_float(s[1]), __uint_as_float(s[1]));
}
VWA_DEVICE float sum_halves(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// unpack a 16-byte vector of 8 bf16 into f32
VWA_DEVICE void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

VWA_DEVICE uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]); r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]); r.w = pack2(f[6], f[7]);
  return r;
}

// streaming (non-temporal) 16-byte load: weights are read once per decode step
VWA_DEVICE uint4 load_nt(const void* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

VWA_DEVICE bf16x8 as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

// Workgroup barrier for LDS (and control-flow) hand-offs only: this wave's LDS / scalar operations
// complete first (lgkmcnt), its VECTOR memory operations stay in flight.  __syncthreads()' workgroup
// release fence makes the compiler put s_waitcnt vmcnt(0) in front of the barrier whenever a store
// may be outstanding -- and gfx9 counts loads and stores on one in-order counter, so that drains
// every weight load a streaming kernel keeps in flight (measured: the chained layer's X staging
// "took" 6-9 us because its barrier waited for 256 KB of prefetched weights per CU).  Callers that
// need their global stores performed before the barrier wait for them explicitly.
VWA_DEVICE void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

VWA_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

VWA_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

VWA_DEVICE int lane_id() { return threadIdx.x & 63; }

// The workitem id through an empty volatile asm: every use is a fresh value, so address math
// derived from it cannot be hoisted out of an enclosing loop.  The chained decode kernels read
// their thread ids through this (VWA_TX): in the multi-layer launch (chain_kernel MULTI) LICM
// otherwise hoisted every lane-derived LDS / weight address of all four phases and the attention
// out of the layer loop -- 256 VGPRs + 650 B of scratch per lane (round 2's failed 32-layer loop
// had the same cause).
VWA_DEVICE int opaque_tid() {
  int t = (int)__builtin_amdgcn_workitem_id_x();
  asm volatile("" : "+v"(t));
  return t;
}
#define VWA_TX (::vwa::opaque_tid())

VWA_DEVICE f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// OCP fp8 e4m3 (gfx950 MFMA/cvt format): 16x16x32 MFMA with 8 fp8 per lane per operand
VWA_DEVICE f32x4 mfma16_fp8(long a, long b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
}

// OCP fp8 e4m3 on the block-scaled MX MFMA, 16x16x128 (v_mfma_scale_f32_16x16x128_f8f6f4): 32 fp8
// per lane per operand; unit E8M0 block scales (127 = 2^0) -- the per-row scales are applied in
// the epilogue.  Twice the bf16 MFMA rate per clock (MI355X_MICROARCH.md: the non-scaled 16x16x32
// fp8 form only runs at the bf16 rate) and a quarter of the instructions.  A and B take the same
// (lane, byte) -> k assignment, so any k order the operands share gives the full dot product.
using i32x8 = __attribute__((ext_vector_type(8))) int;
VWA_DEVICE f32x4 mfma16x128_fp8(const i32x8& a, const i32x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// two f32 -> two OCP e4m3 bytes (round to nearest even, saturating at +-448 via the caller's scale)
VWA_DEVICE uint32_t cvt_pk_fp8(float a, float b) {
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xFFFFu;
}

VWA_DEVICE float silu(float x) { return x / (1.f + __expf(-x)); }

VWA_DEVICE float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// Bijective XCD-aware remap of a 1-D block index (8 XCDs, each with a private L2):
// consecutive logical tiles land on the same XCD so neighbouring tiles share L2 lines.
VWA_DEVICE int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  int q = nwg / nx, r = nwg % nx;
  int x = bid % nx, i = bid / nx;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

}  // namespace vwa
