// Critical-load latency under a weight stream (diagnostic, not part of the framework).
//
// The chained decode layer (skinny_stream.hip chain_kernel) keeps HBM busy by issuing weight items
// ahead of every grid barrier; its in-phase stamps (tools/chain_probe.py, profiles/r5_*) show the
// phase's small activation read taking 3-6.5 us after each barrier release.  This probe asks how
// the round trip of one such "critical" load depends on how many weight bytes every CU keeps in
// flight: 256 workgroups x 8 waves; waves [0, nstream) stream their share of a 1 GB region as items
// of 16 x 1 KB buffer loads with SETS register sets in flight (SETS * 16 KB per wave); wave 7
// waits ~3 us for the stream to ramp, then times 12 dependent probe loads (s_memrealtime, 100 MHz):
//   mode 0  agent-scope (sc1) load of a line another workgroup (another XCD) wrote this launch
//   mode 1  plain load of a cold line (HBM miss)
//   mode 2  scalar load (glc) of an L2-uncached word (the chain barrier's poll)
//   mode 3  returning agent-scope atomic add on an L2-uncached word (the barrier ticket)
//   mode 4  scalar load (glc) of an L2-uncached line another workgroup wrote this launch (fresh data)
//   mode 5  scalar load (glc) of a normal (L2-cached) line another workgroup wrote (sc1) this launch
//
//   hipcc --offload-arch=gfx950 -O3 tools/crit_latency_probe.hip -o tools/crit_latency_probe_bin
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

constexpr int kProbes = 12;

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <int SETS>
__global__ __launch_bounds__(512) void crit(const char* W, size_t wbytes, int nstream, int mode, unsigned* X,
                                            unsigned long long* unc, const char* cold,
                                            unsigned long long* out, int* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w < nstream) {
    const unsigned nwaves = gridDim.x * nstream, wid = blockIdx.x * nstream + w;
    const unsigned per = (unsigned)(wbytes / 16384) / nwaves;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W), (short)0, (int)wbytes, 0x00020000);
    const unsigned b0 = wid * per * 16384u + lane * 16u;
    u32x4 v[SETS][16];
    unsigned acc = 0;
    auto load = [&](int s, unsigned it) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        v[s][i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(it < per ? b0 + it * 16384u + i * 1024u : 0xFFFFFFF0u), 0, 0);
    };
#pragma unroll
    for (int s = 0; s < SETS; ++s) load(s, s);
    for (unsigned it = 0; it < per; it += SETS) {
#pragma unroll
      for (int s = 0; s < SETS; ++s) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc ^= v[s][i].x ^ v[s][i].w;
        load(s, it + s + SETS);
      }
    }
    if (acc == 0x12345678u) sink[0] = (int)acc;
    return;
  }
  if (w != 7) return;
  // the line this workgroup's probes read in mode 0: written (write-through) by the NEXT workgroup
  const unsigned nb = gridDim.x, me = blockIdx.x, src = (me + 1) % nb;
  if (mode == 0)
    __hip_atomic_store(X + me * 64 + lane, 0x1000u + me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // modes 4 / 5: one fresh 64-byte line per probe, written by this workgroup for its predecessor
  unsigned* fresh = mode == 4 ? reinterpret_cast<unsigned*>(unc) + 4096 / 4 : X + 256 * 64;
  if (mode >= 4)
    for (int k = lane; k < kProbes * 16; k += 64)
      __hip_atomic_store(fresh + me * kProbes * 16 + k, 0x2000u + me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t_start = now();
  while (now() - t_start < 300) __builtin_amdgcn_s_sleep(8);  // ~3 us: the stream is at full rate
  unsigned long long lat[kProbes];
  unsigned acc = 0;
  for (int i = 0; i < kProbes; ++i) {
    const unsigned long long t0 = now();
    if (mode == 0) {
      acc += __hip_atomic_load(X + src * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (mode == 1) {
      acc += *(volatile const unsigned*)(cold + ((size_t)(me * kProbes + i) * 65536 + lane * 4));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (mode == 2) {
      unsigned long long v;
      const unsigned long long* p = unc + 16 * (me & 7);
      asm volatile("s_load_dwordx2 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
      acc += (unsigned)v;
    } else if (mode >= 4) {
      unsigned v;
      const unsigned* p = fresh + (src * kProbes + i) * 16;
      asm volatile("s_load_dword %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
      acc += v;
    } else {
      if (lane == 0)
        acc += (unsigned)__hip_atomic_fetch_add(unc + 16 * (me & 7), 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    lat[i] = now() - t0;
    __builtin_amdgcn_s_sleep(20);
  }
  if (lane == 0)
    for (int i = 0; i < kProbes; ++i) out[me * kProbes + i] = lat[i];
  if (acc == 0x12345678u) sink[1] = (int)acc;
}

// One LOADER wave per CU streams its share by LDS-DMA (1 KB per instruction) into a 128 KB ring,
// never more than INFL loads in flight (s_waitcnt vmcnt(INFL - 16) before each 16-load item);
// wave 7 probes as above (modes 0 / 1).  quiet_odd: odd workgroups do not stream (per-CU vs global
// queueing: their probes see only other CUs' traffic).
template <int INFL>
__global__ __launch_bounds__(512) void crit_loader(const char* W, size_t wbytes, int mode, int quiet_odd, unsigned* X,
                                                   const char* cold, unsigned long long* out, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char ring[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool quiet = quiet_odd && (blockIdx.x & 1);
  if (w == 0 && !quiet) {
    const unsigned nwaves = quiet_odd ? gridDim.x / 2 : gridDim.x;
    const unsigned wid = quiet_odd ? blockIdx.x / 2 : blockIdx.x;
    const unsigned per = (unsigned)(wbytes / 16384) / nwaves;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W), (short)0, (int)wbytes, 0x00020000);
    const unsigned b0 = wid * per * 16384u + lane * 16u;
    for (unsigned it = 0; it < per; ++it) {
      if constexpr (INFL == 32) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else if constexpr (INFL == 48) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(47)" ::: "memory");
      char* slot = ring + (it & 7) * 16384;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                                 b0 + it * 16384u + i * 1024u, 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
  if (w != 7) return;
  const unsigned nb = gridDim.x, me = blockIdx.x, src = (me + 1) % nb;
  if (mode == 0)
    __hip_atomic_store(X + me * 64 + lane, 0x1000u + me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t_start = now();
  while (now() - t_start < 300) __builtin_amdgcn_s_sleep(8);
  unsigned long long lat[kProbes];
  unsigned acc = 0;
  for (int i = 0; i < kProbes; ++i) {
    const unsigned long long t0 = now();
    if (mode == 0) {
      acc += __hip_atomic_load(X + src * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      acc += *(volatile const unsigned*)(cold + ((size_t)(me * kProbes + i) * 65536 + lane * 4));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lat[i] = now() - t0;
    __builtin_amdgcn_s_sleep(20);
  }
  if (lane == 0)
    for (int i = 0; i < kProbes; ++i) out[me * kProbes + i] = lat[i];
  if (acc == 0x12345678u) sink[1] = (int)acc;
}

// X staging as the chained layer does it: wave 0 of every workgroup LDS-DMAs `pieces` 1 KB pieces
// (one row of K = 512 * pieces bf16) with cache bits AUX, all in flight, and times their landing.
// copies: how many distinct copies of X the 256 workgroups spread over (1: all read the SAME bytes,
// 8: one copy per XCD by block id mod 8, 256: private).  Waves 1..nstream stream weights meanwhile.
__global__ __launch_bounds__(512) void xstage(const char* W, size_t wbytes, int nstream, const char* X, int pieces,
                                              int copies, int aux, unsigned long long* out, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w >= 1 && w <= nstream) {
    const unsigned nwaves = gridDim.x * nstream, wid = blockIdx.x * nstream + (w - 1);
    const unsigned per = (unsigned)(wbytes / 16384) / nwaves;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(W), (short)0, (int)wbytes, 0x00020000);
    const unsigned b0 = wid * per * 16384u + lane * 16u;
    u32x4 v[16];
    unsigned acc = 0;
    for (unsigned it = 0; it < per; ++it) {
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(b0 + it * 16384u + i * 1024u), 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= v[i].x ^ v[i].w;
    }
    if (acc == 0x12345678u) sink[0] = (int)acc;
    return;
  }
  if (w != 0) return;
  const unsigned long long t_start = now();
  if (nstream) while (now() - t_start < 300) __builtin_amdgcn_s_sleep(8);
  const int copy = copies == 1 ? 0 : copies == 8 ? (blockIdx.x & 7) : blockIdx.x;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(X), (short)0, 256 * 64 * 1024, 0x00020000);
  const unsigned base = (unsigned)copy * 64u * 1024u;
  const unsigned long long t0 = now();
  for (int j = 0; j < pieces; ++j) {
    if (aux == 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(lds + j * 1024), 16,
                                               base + j * 1024 + lane * 16, 0, 0, 16);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (__attribute__((address_space(3))) void*)(lds + j * 1024), 16,
                                               base + j * 1024 + lane * 16, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = now();
  if (lane == 0) out[blockIdx.x] = t1 - t0;
  if (lds[lane] == 123 && lds[1000 + lane] == 77) sink[2] = 1;
}

int main() {
  const size_t wbytes = (size_t)1 << 30, cold_bytes = (size_t)256 << 20;
  char *W, *cold;
  unsigned* X;
  unsigned long long *unc, *out;
  int* sink;
  CK(hipMalloc(&W, wbytes));
  CK(hipMalloc(&cold, cold_bytes));
  CK(hipMalloc(&X, 256 * 64 * 4 + 256 * kProbes * 64));
  CK(hipExtMallocWithFlags((void**)&unc, 4096 + 256 * kProbes * 64, hipDeviceMallocUncached));
  CK(hipMalloc(&out, 256 * kProbes * 8));
  CK(hipMalloc(&sink, 16));
  CK(hipMemset(W, 1, wbytes));
  CK(hipMemset(cold, 2, cold_bytes));
  CK(hipMemset(X, 0, 256 * 64 * 4 + 256 * kProbes * 64));
  CK(hipMemset(unc, 0, 4096 + 256 * kProbes * 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* mnames[] = {"sc1_peer_line", "cold_hbm_line", "scalar_uncached_poll", "atomic_uncached_ticket",
                          "scalar_uncached_fresh_line", "scalar_cached_fresh_line"};
  std::vector<unsigned long long> h(256 * kProbes);
  for (int sets = 1; sets <= 0; ++sets)
    for (int ns : {0, 2, 4, 7})
      for (int mode = 0; mode < 6; ++mode) {
        if ((ns == 0 && sets == 2) || mode == 2 || mode == 3 || mode == 5 || ns == 2) continue;
        auto launch = [&]() {
          if (sets == 1)
            hipLaunchKernelGGL(crit<1>, dim3(256), dim3(512), 0, 0, W, wbytes, ns, mode, X, unc, cold, out, sink);
          else
            hipLaunchKernelGGL(crit<2>, dim3(256), dim3(512), 0, 0, W, wbytes, ns, mode, X, unc, cold, out, sink);
        };
        launch();  // warm-up
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> v(h.size());
        for (size_t i = 0; i < h.size(); ++i) v[i] = h[i] * 0.01;
        std::sort(v.begin(), v.end());
        std::printf("{\"sets\": %d, \"stream_waves\": %d, \"inflight_kb_per_cu\": %d, \"probe\": \"%s\", "
                    "\"lat_us_p10_p50_p90_max\": [%.2f, %.2f, %.2f, %.2f], \"kernel_us\": %.1f, \"stream_TBps\": %.2f}\n",
                    sets, ns, sets * ns * 16, mnames[mode], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10],
                    v.back(), ms * 1e3, ns ? wbytes / (ms * 1e-3) / 1e12 : 0.0);
        std::fflush(stdout);
      }
  {  // X staging: hot spot of 256 CUs reading the same bytes?
    char* Xs;
    CK(hipMalloc(&Xs, 256 * 64 * 1024));
    CK(hipMemset(Xs, 3, 256 * 64 * 1024));
    for (int ns : {0, 7})
      for (int pieces : {8, 28})
        for (int copies : {1, 8, 256})
          for (int aux : {16, 0}) {
            hipLaunchKernelGGL(xstage, dim3(256), dim3(512), 64 * 1024, 0, W, wbytes, ns, Xs, pieces, copies, aux, out, sink);
            hipLaunchKernelGGL(xstage, dim3(256), dim3(512), 64 * 1024, 0, W, wbytes, ns, Xs, pieces, copies, aux, out, sink);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), out, 256 * 8, hipMemcpyDeviceToHost));
            std::vector<double> v(256);
            for (int b = 0; b < 256; ++b) v[b] = h[b] * 0.01;
            std::sort(v.begin(), v.end());
            std::printf("{\"xstage\": true, \"stream_waves\": %d, \"pieces_kb\": %d, \"copies\": %d, \"sc1\": %d, "
                        "\"us_p10_p50_p90_max\": [%.2f, %.2f, %.2f, %.2f]}\n", ns, pieces, copies, aux == 16,
                        v[25], v[128], v[230], v[255]);
            std::fflush(stdout);
          }
    CK(hipFree(Xs));
  }
  return 0;
  // loader-wave streaming (LDS-DMA ring), in-flight cap per CU, probes from a busy / a quiet CU
  for (int infl : {32, 48, 63})
    for (int quiet : {0, 1})
      for (int mode = 0; mode < 2; ++mode) {
        auto launch = [&]() {
          if (infl == 32)
            hipLaunchKernelGGL(crit_loader<32>, dim3(256), dim3(512), 128 * 1024, 0, W, wbytes, mode, quiet, X, cold, out, sink);
          else if (infl == 48)
            hipLaunchKernelGGL(crit_loader<48>, dim3(256), dim3(512), 128 * 1024, 0, W, wbytes, mode, quiet, X, cold, out, sink);
          else
            hipLaunchKernelGGL(crit_loader<63>, dim3(256), dim3(512), 128 * 1024, 0, W, wbytes, mode, quiet, X, cold, out, sink);
        };
        launch();
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> v;
        for (int b = 0; b < 256; ++b)
          if (!quiet || (b & 1))
            for (int i = 0; i < kProbes; ++i) v.push_back(h[b * kProbes + i] * 0.01);
        std::sort(v.begin(), v.end());
        std::printf("{\"loader_wave_lds_dma\": true, \"inflight_kb_per_cu\": %d, \"quiet_probe_cus\": %d, \"probe\": \"%s\", "
                    "\"lat_us_p10_p50_p90_max\": [%.2f, %.2f, %.2f, %.2f], \"kernel_us\": %.1f, \"stream_TBps\": %.2f}\n",
                    infl, quiet, mnames[mode], v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10], v.back(), ms * 1e3,
                    wbytes / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
      }
  return 0;
}
