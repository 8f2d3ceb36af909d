// Load-latency probe (diagnostic, not part of the framework): what a cold vector load costs on
// MI355X after the decode step's weight stream has gone through the caches -- the chained
// attention's K/V round trip measured ~6 us cold vs ~3.5 us right after another read of the same
// K/V (tools/chain_probe.py --attn / --warm-kv).  One lane times single dependent loads
// (s_memrealtime, 100 MHz) at offsets chosen to separate a new 2 MB region, a new 4 KB page, a
// new line of a touched page, and a re-read.
//
//   hipcc --offload-arch=gfx950 -O2 tools/latency_probe.hip -o tools/latency_probe && tools/latency_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

__global__ void probe(const char* base, const long long* offs, int n, unsigned long long* ticks, int* sink) {
  if (threadIdx.x != 0) return;
  int acc = 0;
  for (int i = 0; i < n; ++i) {
    const char* p = base + offs[i];
    unsigned long long t0, t1;
    int v;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    acc += v;
    ticks[i] = t1 - t0;
  }
  sink[0] = acc;
}

// the chained attention's K/V step shape: every wave of `grid` workgroups x `waves` issues 16 load
// instructions (8 "K": 16 keys x 64 B at a 256 B key stride, 8 "V": 4 keys x 256 B), all before
// the first wait, at its own 32-key range of a paged region; lane 0 stamps issue and landing
__global__ void kv_gather(const char* base, long long region, unsigned long long* ticks, int* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, n = lane & 15, g = lane >> 4;
  const long long wid = (long long)blockIdx.x * (blockDim.x >> 6) + w;
  const char* kb = base + (wid * 32 * 256) % region;  // 32 keys x 256 B per wave
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  uint4 r[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int key = 8 * (n >> 2) + 4 * (i & 1) + (n & 3);
    r[i] = *reinterpret_cast<const uint4*>(kb + key * 256 + 16 * g + 64 * (i >> 1));
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int idx = i * 64 + lane;
    r[8 + i] = *reinterpret_cast<const uint4*>(kb + (idx / 16) * 256 + 16 * (idx % 16));
  }
  unsigned acc = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc ^= r[i].x ^ r[i].w;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0) ticks[wid] = t1 - t0;
  if (acc == 0x12345678u) sink[2] = (int)acc;
}

// the chained attention's prologue: every workgroup reads the SAME step metadata (wave 0: 4 x 8 B +
// 2 x 4 B per lane over ~2.5 KB) and every wave the same 8 KB of Q (4 x 16 B per lane); lane 0 of
// wave 0 stamps the landing of both
__global__ void meta_broadcast(const char* meta, const char* q, int per_wave_q, unsigned long long* ticks, int* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long t0, t1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  unsigned acc = 0;
  if (per_wave_q || w == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 v = *reinterpret_cast<const uint4*>(q + ((w * 4 + k) * 64 + lane) % 512 * 16);
      acc ^= v.x;
    }
  }
  if (w == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) acc ^= *reinterpret_cast<const unsigned*>(meta + r * 512 + lane * 8);
    acc ^= *reinterpret_cast<const unsigned*>(meta + 2048 + lane * 4);
    acc ^= *reinterpret_cast<const unsigned*>(meta + 2304 + lane * 4);
  }
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (threadIdx.x == 0) ticks[blockIdx.x] = t1 - t0;
  if (acc == 0x12345678u) sink[3] = (int)acc;
}

// The decode GEMMs' weight stream, isolated: every wave of 256 x 8 streams its contiguous share of
// `bytes` as "items" of 16 x 1 KB-contiguous load instructions (the tiled-weight pattern) with SETS
// register sets in flight (the chained kernel: 2), consuming each set with a cheap reduction.
template <int SETS, int NL = 16>
__global__ __launch_bounds__(1024) void item_stream(const char* base, size_t bytes, int* sink) {
  const int lane = threadIdx.x & 63, wpg = blockDim.x >> 6;
  const size_t wid = (size_t)blockIdx.x * wpg + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * wpg;
  const size_t items = bytes / (NL * 1024), per = items / nwaves;
  const char* p = base + wid * per * (NL * 1024) + lane * 16;
  u32x4 r[SETS][NL];
  unsigned acc = 0;
  auto load = [&](int s, size_t it) {
#pragma unroll
    for (int i = 0; i < NL; ++i) r[s][i] = *(__attribute__((address_space(1))) const u32x4*)(p + it * (NL * 1024) + i * 1024);
  };
#pragma unroll
  for (int s = 0; s < SETS; ++s) load(s, s);
  for (size_t it = 0; it < per; it += SETS) {
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
#pragma unroll
      for (int i = 0; i < NL; ++i) acc ^= r[s][i].x ^ r[s][i].w;
      if (it + s + SETS < per) load(s, it + s + SETS);
    }
  }
  if (acc == 0x12345678u) sink[4] = (int)acc;
}

// the chained kernel's form exactly: 8 waves x SETS register sets of 16 buffer loads (32-bit
// offsets: no 64-bit address registers), loads of set s re-issued right after its use
template <int SETS>
__global__ __launch_bounds__(512) void item_stream_buf(const char* base, size_t bytes, int* sink) {
  const int lane = threadIdx.x & 63;
  const unsigned wid = blockIdx.x * 8 + (threadIdx.x >> 6), nwaves = gridDim.x * 8;
  const unsigned items = (unsigned)(bytes / 16384), per = items / nwaves;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)bytes, 0x00020000);
  u32x4 v[SETS][16];
  unsigned acc = 0;
  const unsigned b0 = wid * per * 16384u + lane * 16u;
  auto load = [&](int s, unsigned it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[s][i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(b0 + it * 16384u + i * 1024u), 0, 0);
  };
#pragma unroll
  for (int s = 0; s < SETS; ++s) load(s, s);
  for (unsigned it = 0; it < per; it += SETS) {
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= v[s][i].x ^ v[s][i].w;
      if (it + s + SETS < per) load(s, it + s + SETS);
    }
  }
  if (acc == 0x12345678u) sink[4] = (int)acc;
}

// two named register sets exactly like the chained kernel's loop (compute A, reload A, compute B,
// reload B), with a real MFMA consumer so the loads cannot be reordered past their use
__global__ __launch_bounds__(512) void item_stream_ab(const char* base, size_t bytes, int* sink) {
  const int lane = threadIdx.x & 63;
  const unsigned wid = blockIdx.x * 8 + (threadIdx.x >> 6), nwaves = gridDim.x * 8;
  const unsigned items = (unsigned)(bytes / 16384), per = items / nwaves;
  // num_records = the stream's bytes: the past-the-end sentinel below is beyond it (reads 0)
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)bytes, 0x00020000);
  const unsigned b0 = wid * per * 16384u + lane * 16u;
  u32x4 A[16], B[16];
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const bf16x8_t xv = __builtin_bit_cast(bf16x8_t, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
  auto load = [&](u32x4 (&v)[16], unsigned it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(it < per ? b0 + it * 16384u + i * 1024u : 0xFFFFFFF0u), 0, 0);
  };
  auto compute = [&](const u32x4 (&v)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xv, __builtin_bit_cast(bf16x8_t, v[i]), acc, 0, 0, 0);
  };
  load(A, 0);
  load(B, 1);
#pragma unroll 1
  for (unsigned it = 0; it < per; it += 2) {
    compute(A);
    load(A, it + 2);
    compute(B);
    load(B, it + 3);
  }
  if (acc[0] == 1234.5f) sink[4] = (int)acc[1];
}


// the two-set loop with the weight loads as inline asm and EXPLICIT waits: the compiler does not
// track these loads, so it cannot merge the sets' waits (item_stream_ab: one vmcnt(0) per
// iteration, both sets drained together); here set S is awaited with vmcnt(16 * (SETS - 1)) --
// the younger sets' loads stay in flight -- and re-issued right after its use
typedef int vwa_v4i __attribute__((ext_vector_type(4)));
#define VWA_TIE16(v) "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), \
  "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])
template <int SETS>
__global__ __launch_bounds__(512) void item_stream_asm(const char* base, size_t bytes, int* sink) {
  const int lane = threadIdx.x & 63;
  const unsigned wid = blockIdx.x * 8 + (threadIdx.x >> 6), nwaves = gridDim.x * 8;
  const unsigned items = (unsigned)(bytes / 16384), per = items / nwaves;
  // buffer descriptor words: base lo, base hi | stride 0, num_records, the flags of make_buffer_rsrc
  const unsigned long long ba = (unsigned long long)base;
  const vwa_v4i rs = {(int)(unsigned)ba, (int)((unsigned)(ba >> 32) & 0xFFFFu), (int)bytes, 0x00020000};
  const unsigned b0 = wid * per * 16384u + lane * 16u;
  u32x4 V[SETS][16];
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  const bf16x8_t xv = __builtin_bit_cast(bf16x8_t, u32x4{0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u});
  auto load = [&](u32x4 (&v)[16], unsigned it) {
    const unsigned o = it < per ? b0 + it * 16384u : 0x80000000u;  // past num_records: zeros
#pragma unroll
    for (int i = 0; i < 16; ++i)
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v[i]) : "v"(o), "s"(rs), "s"(i * 1024));
  };
  auto wait_set = [&](u32x4 (&v)[16]) {
    if constexpr (SETS == 2) asm volatile("s_waitcnt vmcnt(16)" : VWA_TIE16(v));
    else if constexpr (SETS == 3) asm volatile("s_waitcnt vmcnt(32)" : VWA_TIE16(v));
    else asm volatile("s_waitcnt vmcnt(0)" : VWA_TIE16(v));
  };
  auto compute = [&](const u32x4 (&v)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xv, __builtin_bit_cast(bf16x8_t, v[i]), acc, 0, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < SETS; ++s) load(V[s], s);
#pragma unroll 1
  for (unsigned it = 0; it < per; it += SETS) {
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
      wait_set(V[s]);
      compute(V[s]);
      load(V[s], it + s + SETS);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc[0] == 1234.5f) sink[4] = (int)acc[1];
}

// the same items, interleaved: item j of wave w sits at (j * nwaves + w) * 16 KB, so the waves in
// flight together read one contiguous region
template <int SETS>
__global__ __launch_bounds__(512) void item_stream_il(const char* base, size_t bytes, int* sink) {
  const int lane = threadIdx.x & 63;
  const size_t wid = (size_t)blockIdx.x * 8 + (threadIdx.x >> 6), nwaves = (size_t)gridDim.x * 8;
  const size_t items = bytes / 16384, per = items / nwaves;
  u32x4 r[SETS][16];
  unsigned acc = 0;
  auto load = [&](int s, size_t it) {
    const char* p = base + (it * nwaves + wid) * 16384 + lane * 16;
#pragma unroll
    for (int i = 0; i < 16; ++i) r[s][i] = *(__attribute__((address_space(1))) const u32x4*)(p + i * 1024);
  };
#pragma unroll
  for (int s = 0; s < SETS; ++s) load(s, s);
  for (size_t it = 0; it < per; it += SETS) {
#pragma unroll
    for (int s = 0; s < SETS; ++s) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc ^= r[s][i].x ^ r[s][i].w;
      if (it + s + SETS < per) load(s, it + s + SETS);
    }
  }
  if (acc == 0x12345678u) sink[4] = (int)acc;
}

// every lane of every workgroup streams its share of `bytes` (the weight stream's cache pressure)
__global__ void stream(const uint4* p, size_t n16, int* sink) {
  unsigned acc = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.w;
  }
  if (acc == 0x12345678u) sink[1] = (int)acc;
}

int main() {
  const size_t big = (size_t)1 << 30, probe_bytes = (size_t)64 << 20;
  char *A, *B;
  CK(hipMalloc(&A, big));
  CK(hipMalloc(&B, probe_bytes));
  CK(hipMemset(A, 1, big));
  CK(hipMemset(B, 2, probe_bytes));
  // offsets: a new 2 MB region, then within it +256 B (same 4 KB page, new line), +4 KB, +64 KB,
  // +1 MB (same 2 MB region), then the first offset again (re-read)
  std::vector<long long> offs;
  const char* what[] = {"new_2MB", "same_page_new_line", "next_4KB_page", "plus_64KB", "plus_1MB", "reread_first"};
  const int per = 6;
  for (int r = 0; r < 8; ++r) {
    const long long b = (long long)(r * 4 + 3) << 21;  // 8 separate 2 MB regions
    offs.insert(offs.end(), {b, b + 256, b + 4096, b + 65536, b + (1 << 20), b});
  }
  const int n = (int)offs.size();
  long long* d_offs;
  unsigned long long* d_t;
  int* d_sink;
  CK(hipMalloc(&d_offs, n * sizeof(long long)));
  CK(hipMalloc(&d_t, n * sizeof(unsigned long long)));
  CK(hipMalloc(&d_sink, 8));
  CK(hipMemcpy(d_offs, offs.data(), n * sizeof(long long), hipMemcpyHostToDevice));
  std::vector<unsigned long long> t(n);
  auto run = [&](const char* label, bool flush) {
    if (flush) hipLaunchKernelGGL(stream, dim3(1024), dim3(512), 0, 0, (const uint4*)A, big / 16, d_sink);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, B, d_offs, n, d_t, d_sink);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(t.data(), d_t, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::printf("{\"case\": \"%s\"", label);
    for (int k = 0; k < per; ++k) {
      std::vector<double> v;
      for (int r = 0; r < n / per; ++r) v.push_back(t[r * per + k] * 0.01);  // 10 ns ticks -> us
      double s = 0;
      for (double x : v) s += x;
      std::printf(", \"%s_us\": [%.2f, %.2f, %.2f]", what[k], v[0], s / v.size(), v.back());
    }
    std::printf("}\n");
  };
  // K/V-step gathers: 1 wave alone, then 128 workgroups x 3 waves (the chained attention's shape)
  {
    unsigned long long* d_g;
    CK(hipMalloc(&d_g, 4096 * sizeof(unsigned long long)));
    std::vector<unsigned long long> tg(4096);
    const long long region = (long long)32 << 20;
    auto gather = [&](const char* label, int grid, int waves, bool flush) {
      if (flush) hipLaunchKernelGGL(stream, dim3(1024), dim3(512), 0, 0, (const uint4*)A, big / 16, d_sink);
      hipLaunchKernelGGL(kv_gather, dim3(grid), dim3(64 * waves), 0, 0, B, region, d_g, d_sink);
      CK(hipDeviceSynchronize());
      const int nw = grid * waves;
      CK(hipMemcpy(tg.data(), d_g, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      std::vector<double> v(nw);
      for (int i = 0; i < nw; ++i) v[i] = tg[i] * 0.01;
      std::sort(v.begin(), v.end());
      std::printf("{\"case\": \"%s\", \"waves\": %d, \"kv_step_us_min_med_max\": [%.2f, %.2f, %.2f]}\n", label, nw,
                  v[0], v[nw / 2], v[nw - 1]);
    };
    gather("kv_step_1wave_cold", 1, 1, true);
    gather("kv_step_1wave_warm", 1, 1, false);
    gather("kv_step_128x3_cold", 128, 3, true);
    gather("kv_step_128x3_warm", 128, 3, false);
    gather("kv_step_256x8_cold", 256, 8, true);
    auto meta = [&](const char* label, int grid, int q_all, bool flush) {
      if (flush) hipLaunchKernelGGL(stream, dim3(1024), dim3(512), 0, 0, (const uint4*)A, big / 16, d_sink);
      hipLaunchKernelGGL(meta_broadcast, dim3(grid), dim3(512), 0, 0, B + (40 << 20), B + (41 << 20), q_all, d_g, d_sink);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(tg.data(), d_g, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
      std::vector<double> v(grid);
      for (int i = 0; i < grid; ++i) v[i] = tg[i] * 0.01;
      std::sort(v.begin(), v.end());
      std::printf("{\"case\": \"%s\", \"workgroups\": %d, \"meta_us_min_med_max\": [%.2f, %.2f, %.2f]}\n", label,
                  grid, v[0], v[grid / 2], v[grid - 1]);
    };
    meta("meta_1wg_cold", 1, 1, true);
    meta("meta_256wg_q_all_waves_cold", 256, 1, true);
    meta("meta_256wg_q_wave0_cold", 256, 0, true);
    meta("meta_256wg_q_all_waves_warm", 256, 1, false);
    CK(hipFree(d_g));
  }
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto bw = [&](const char* label, auto kern, int grid, size_t bytes, int threads = 512) {
      hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, (const char*)A, bytes, d_sink);  // warm-up
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), 0, 0, (const char*)A, bytes, d_sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("{\"case\": \"%s\", \"MB\": %zu, \"us_per_launch\": %.2f, \"TBps\": %.3f}\n", label, bytes >> 20,
                  ms * 200.0, bytes / (ms / 5 * 1e-3) / 1e12);
    };
    bw("items_2sets_436MB", item_stream<2>, 256, (size_t)436 << 20);
    bw("ab_2sets_8waves_436MB", item_stream_ab, 256, (size_t)436 << 20);
    bw("ab_2sets_8waves_436MB_again", item_stream_ab, 256, (size_t)436 << 20);
    bw("asm_1set_8waves_436MB", item_stream_asm<1>, 256, (size_t)436 << 20);
    bw("asm_2sets_8waves_436MB", item_stream_asm<2>, 256, (size_t)436 << 20);
    bw("asm_3sets_8waves_436MB", item_stream_asm<3>, 256, (size_t)436 << 20);
    bw("asm_2sets_8waves_436MB_again", item_stream_asm<2>, 256, (size_t)436 << 20);
    bw("ab_2sets_8waves_436MB_3rd", item_stream_ab, 256, (size_t)436 << 20);
    bw("buf_2sets_8waves_436MB", item_stream_buf<2>, 256, (size_t)436 << 20);
    bw("buf_1set_8waves_436MB", item_stream_buf<1>, 256, (size_t)436 << 20);
    bw("buf_3sets_8waves_436MB", item_stream_buf<3>, 256, (size_t)436 << 20);
    bw("buf_2sets_8waves_512wg_436MB", item_stream_buf<2>, 512, (size_t)436 << 20);
    bw("items_1set_436MB", item_stream<1>, 256, (size_t)436 << 20);
    bw("items_1set_16waves_436MB", item_stream<1>, 256, (size_t)436 << 20, 1024);
    bw("items_2sets_8loads_16waves_436MB", item_stream<2, 8>, 256, (size_t)436 << 20, 1024);
    bw("items_1set_32loads_436MB", item_stream<1, 32>, 256, (size_t)436 << 20);
    bw("items_1set_8loads_436MB", item_stream<1, 8>, 256, (size_t)436 << 20);
    bw("items_1set_4waves_436MB", item_stream<1>, 256, (size_t)436 << 20, 256);
    bw("items_2sets_8loads_436MB", item_stream<2, 8>, 256, (size_t)436 << 20);
    bw("items_4sets_8loads_436MB", item_stream<4, 8>, 256, (size_t)436 << 20);
    bw("items_4sets_4loads_436MB", item_stream<4, 4>, 256, (size_t)436 << 20);
    bw("items_8sets_4loads_436MB", item_stream<8, 4>, 256, (size_t)436 << 20);
    bw("items_1set_512wg_436MB", item_stream<1>, 512, (size_t)436 << 20);
    bw("items_2sets_8loads_512wg_436MB", item_stream<2, 8>, 512, (size_t)436 << 20);
    bw("items_2sets_1GB", item_stream<2>, 256, (size_t)1 << 30);
    bw("items_2sets_117MB", item_stream<2>, 256, (size_t)117 << 20);
    bw("items_2sets_50MB", item_stream<2>, 256, (size_t)50 << 20);
    bw("items_2sets_512wg_436MB", item_stream<2>, 512, (size_t)436 << 20);
    // linear sweep: consecutive lanes / waves / workgroups on consecutive 16-byte pieces
    auto sweep = [&](const char* label, int grid, size_t bytes) {
      hipLaunchKernelGGL(stream, dim3(grid), dim3(512), 0, 0, (const uint4*)A, bytes / 16, d_sink);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(stream, dim3(grid), dim3(512), 0, 0, (const uint4*)A, bytes / 16, d_sink);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::printf("{\"case\": \"%s\", \"MB\": %zu, \"us_per_launch\": %.2f, \"TBps\": %.3f}\n", label, bytes >> 20,
                  ms * 200.0, bytes / (ms / 5 * 1e-3) / 1e12);
    };
    sweep("linear_sweep_256wg_436MB", 256, (size_t)436 << 20);
    sweep("linear_sweep_1024wg_436MB", 1024, (size_t)436 << 20);
    sweep("linear_sweep_2048wg_1GB", 2048, (size_t)1 << 30);
    bw("items_interleaved_2sets_436MB", item_stream_il<2>, 256, (size_t)436 << 20);
  }
  run("first_touch_after_1GB_stream", true);
  run("immediate_repeat", false);
  run("repeat_after_1GB_stream", true);
  run("immediate_repeat_2", false);
  CK(hipFree(A));
  CK(hipFree(B));
  return 0;
}
