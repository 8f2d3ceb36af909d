// One-shot peer-to-peer all-reduce for decode-sized tensor-parallel messages (SURVEY.md §2.8
// C1/C2, §5.8).  RCCL's ring all-reduce pays 2(N-1) link hops of latency; a decode step's
// row-parallel output is only M x d x 2 bytes (8 KiB per row for Llama-3-8B), so here every rank
// reads all peers' inputs directly over its point-to-point xGMI links and reduces in registers:
// one hop, one kernel, graph-capturable.
//
// The buffer is cut into kMaxBlocks fixed regions of max_elems/kMaxBlocks; workgroup b always
// owns region b (every call launches all kMaxBlocks workgroups, idle ones just signal), so a
// region's epoch advances exactly once per call on every rank whatever the message size.
// Per call (epoch e, per workgroup b so no cross-workgroup ordering is needed):
//   1. copy this workgroup's chunk of the input into our IPC-shared staging buffer [e & 1]
//      (double-buffered by epoch parity, so call e+1 never overwrites what a slow peer may
//      still be reading for call e);
//   2. release (system-scope fence), then store flag[b][rank] = e into every peer's flag array;
//   3. wait until our own flag[b][p] == e for every peer p (bounded spin: a missing peer
//      raises an error word instead of hanging the GPU);
//   4. acquire (system-scope fence) and sum the chunk of all ranks' staging buffers in rank
//      order (bit-identical result on every rank) into the output.
// The IPC-shared buffers (staging, gather, chain regions, flags) are allocated L2-UNCACHED
// (hipExtMallocWithFlags hipDeviceMallocUncached; vwa_ar_create checks the type with
// hipPointerGetAttributes): a peer GPU reads them over xGMI while this GPU's L2 could otherwise
// still hold the newest stores -- with uncached memory every store and flag goes to HBM, and no
// correctness argument leans on the system-scope fences' L2 write-back.  Shared with
// hipIpcGetMemHandle / hipIpcOpenMemHandle (dmabuf).
//
// Behind the gather region: two f32 regions of the chained decode layer's in-launch all-reduce
// rounds (skinny_stream.hip chain_tp_reduce; vwa_ar_chain_tp hands the pointers to the chain).
//
// The same buffers also carry a one-shot ALL-GATHER of small int32 payloads (vwa_ar_gather: the
// vocab-parallel sampler's per-rank partial (value, index) maxima, SURVEY.md §2.8 C4 as [B, 2]
// instead of [B, V/T] logits): a separate double-buffered region behind the all-reduce staging
// and its own flag / epoch slot (index kMaxBlocks), same protocol, one workgroup.
#include "common.h"
#include "vwa_kernels.h"

using namespace vwa;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kThreads = 512;
constexpr int kMaxBlocks = 64;
constexpr int kGatherSlot = kMaxBlocks;   // flag / epoch slot of the all-gather
constexpr int kChainSlot = kMaxBlocks + 1;  // flag / epoch slot of the chained layer's in-launch rounds
constexpr int kSlots = kMaxBlocks + 2;
constexpr int64_t kGatherWords = 64 * 1024;  // int32 words per rank per call (256 KB)
constexpr int64_t kChainFloats = 16 * 8192;  // f32 per chain region: 16 rows x hidden 8192 (70B)

struct ArPeers {
  uint16_t* staging[kMaxRanks];  // each rank's staging base (2 x max_elems bf16, then 2 x kGatherWords int32)
  int* flags[kMaxRanks];         // each rank's flag array [kSlots][kMaxRanks]
};

// signal every peer (flag slot [slot][rank] in the peer's memory) and wait for every peer's
// signal in our own array; bounded: a peer that never arrives raises the error word
__device__ void ar_signal_wait(const ArPeers& peers, int slot, int rank, int world, int e, int* error) {
  if (threadIdx.x < world) {
    __threadfence_system();
    __hip_atomic_store(peers.flags[threadIdx.x] + slot * kMaxRanks + rank, e, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x < world) {
    int* f = peers.flags[rank] + slot * kMaxRanks + threadIdx.x;
    int64_t spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1ll << 24)) {  // ~seconds: a peer never arrived
        atomicExch(error, 1);
        break;
      }
    }
    __threadfence_system();
  }
  __syncthreads();
}

__global__ __launch_bounds__(kThreads) void oneshot_ar_kernel(const uint16_t* __restrict__ in, uint16_t* out,
                                                              int64_t n, int64_t max_elems,
                                                              int rank, int world, ArPeers peers, int* epochs,
                                                              int* error) {
  const int b = blockIdx.x;
  const int64_t chunk = max_elems / kMaxBlocks;
  const int64_t lo = (int64_t)b * chunk, hi = min(n, lo + chunk);
  __shared__ int s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const int e = s_epoch;
  uint16_t* mine = peers.staging[rank] + (int64_t)(e & 1) * max_elems;
  // 1. stage (16-byte vectors; n is a multiple of 8)
  for (int64_t i = lo + (int64_t)threadIdx.x * 8; i < hi; i += (int64_t)kThreads * 8)
    *reinterpret_cast<uint4*>(mine + i) = *reinterpret_cast<const uint4*>(in + i);
  __syncthreads();
  // 2. release + signal every peer, 3. wait for every peer's signal (bounded)
  ar_signal_wait(peers, b, rank, world, e, error);
  // 4. reduce in rank order
  for (int64_t i = lo + (int64_t)threadIdx.x * 8; i < hi; i += (int64_t)kThreads * 8) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int p = 0; p < world; ++p) {
      const uint16_t* src = peers.staging[p] + (int64_t)(e & 1) * max_elems + i;
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(src), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    *reinterpret_cast<uint4*>(out + i) = pack8(acc);
  }
  if (threadIdx.x == 0) epochs[b] = e;
}

// out[p * n + i] = rank p's in[i] on every rank (n <= kGatherWords int32 words); one workgroup
__global__ __launch_bounds__(kThreads) void oneshot_gather_kernel(const int* __restrict__ in, int* __restrict__ out,
                                                                  int n, int64_t gather_off, int rank, int world,
                                                                  ArPeers peers, int* epochs, int* error) {
  __shared__ int s_epoch;
  if (threadIdx.x == 0) s_epoch = epochs[kGatherSlot] + 1;
  __syncthreads();
  const int e = s_epoch;
  auto region = [&](int p) {
    return reinterpret_cast<int*>(reinterpret_cast<char*>(peers.staging[p]) + gather_off) + (int64_t)(e & 1) * kGatherWords;
  };
  int* mine = region(rank);
  for (int i = threadIdx.x; i < n; i += kThreads) mine[i] = in[i];
  __syncthreads();
  ar_signal_wait(peers, kGatherSlot, rank, world, e, error);
  for (int p = 0; p < world; ++p) {
    const int* src = region(p);
    for (int i = threadIdx.x; i < n; i += kThreads) out[(int64_t)p * n + i] = src[i];
  }
  if (threadIdx.x == 0) epochs[kGatherSlot] = e;
}

struct ArState {
  int rank = 0, world = 1;
  int64_t max_elems = 0;
  uint16_t* staging = nullptr;  // local
  int* flags = nullptr;         // local [kSlots][kMaxRanks]
  int* epochs = nullptr;        // local, private [kSlots]
  int* error = nullptr;
  ArPeers peers{};
  bool opened[kMaxRanks] = {};
};

}  // namespace

// L2-uncached device memory for the cross-device hand-offs, its type asserted
static int alloc_uncached(void** p, size_t bytes) {
  *p = nullptr;
  if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) != hipSuccess) return -1;
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, *p) != hipSuccess || a.type != hipMemoryTypeDevice ||
      (a.allocationFlags & hipDeviceMallocUncached) != hipDeviceMallocUncached) {
    (void)hipFree(*p);
    *p = nullptr;
    return -2;
  }
  return 0;
}

extern "C" {

// Allocate the local IPC-shareable buffers; returns an opaque state pointer (nullptr on error).
void* vwa_ar_create(int rank, int world, int64_t max_elems) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || max_elems % (8 * kMaxBlocks)) return nullptr;
  auto* s = new ArState();
  s->rank = rank;
  s->world = world;
  s->max_elems = max_elems;
  void* stg = nullptr;
  void* flg = nullptr;
  if (alloc_uncached(&stg, 2 * max_elems * sizeof(uint16_t) + 2 * kGatherWords * sizeof(int) +
                               2 * kChainFloats * sizeof(float)) != 0 ||
      alloc_uncached(&flg, kSlots * kMaxRanks * sizeof(int)) != 0 ||
      hipMalloc(&s->epochs, kSlots * sizeof(int)) != hipSuccess || hipMalloc(&s->error, sizeof(int)) != hipSuccess) {
    if (stg) (void)hipFree(stg);
    if (flg) (void)hipFree(flg);
    delete s;
    return nullptr;
  }
  s->staging = static_cast<uint16_t*>(stg);
  s->flags = static_cast<int*>(flg);
  (void)hipMemset(s->flags, 0, kSlots * kMaxRanks * sizeof(int));
  (void)hipMemset(s->epochs, 0, kSlots * sizeof(int));
  (void)hipMemset(s->error, 0, sizeof(int));
  (void)hipDeviceSynchronize();
  s->peers.staging[rank] = s->staging;
  s->peers.flags[rank] = s->flags;
  return s;
}

// IPC handles of the local staging and flag buffers (2 x hipIpcMemHandle_t).
int vwa_ar_handles(void* st, void* out128) {
  auto* s = static_cast<ArState*>(st);
  auto* h = static_cast<hipIpcMemHandle_t*>(out128);
  if (hipIpcGetMemHandle(&h[0], s->staging) != hipSuccess) return -1;
  if (hipIpcGetMemHandle(&h[1], s->flags) != hipSuccess) return -2;
  return 0;
}

int vwa_ar_handle_bytes() { return (int)(2 * sizeof(hipIpcMemHandle_t)); }

// Map peer p's buffers from its two IPC handles.
int vwa_ar_open_peer(void* st, int p, const void* in128) {
  auto* s = static_cast<ArState*>(st);
  if (p == s->rank) return 0;
  const auto* h = static_cast<const hipIpcMemHandle_t*>(in128);
  void* a = nullptr;
  void* f = nullptr;
  if (hipIpcOpenMemHandle(&a, h[0], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1;
  if (hipIpcOpenMemHandle(&f, h[1], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -2;
  s->peers.staging[p] = static_cast<uint16_t*>(a);
  s->peers.flags[p] = static_cast<int*>(f);
  s->opened[p] = true;
  return 0;
}

// In-place (in == out allowed) bf16 sum over the group.  n % 8 == 0, n <= max_elems.
int vwa_ar_allreduce(void* st, const uint16_t* in, uint16_t* out, int64_t n, hipStream_t stream) {
  auto* s = static_cast<ArState*>(st);
  if (n % 8 || n > s->max_elems) return -1;
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.staging[p] || !s->peers.flags[p]) return -2;
  hipLaunchKernelGGL(oneshot_ar_kernel, dim3(kMaxBlocks), dim3(kThreads), 0, stream, in, out, n, s->max_elems,
                     s->rank, s->world, s->peers, s->epochs, s->error);
  return (int)hipGetLastError();
}

// All-gather of n int32 words per rank: out[world][n].  n <= kGatherWords.
int vwa_ar_gather(void* st, const int* in, int* out, int64_t n, hipStream_t stream) {
  auto* s = static_cast<ArState*>(st);
  if (n < 0 || n > kGatherWords) return -1;
  for (int p = 0; p < s->world; ++p)
    if (!s->peers.staging[p] || !s->peers.flags[p]) return -2;
  hipLaunchKernelGGL(oneshot_gather_kernel, dim3(1), dim3(kThreads), 0, stream, in, out, (int)n,
                     (int64_t)(2 * s->max_elems * sizeof(uint16_t)), s->rank, s->world, s->peers, s->epochs,
                     s->error);
  return (int)hipGetLastError();
}

int64_t vwa_ar_gather_max_words() { return kGatherWords; }

// The chained decode layer's view of the group (ChainParams::tp): every rank's two f32 chain
// regions, the peers' flag words this rank signals, its own flag words and round counter.
// Returns -1 before every peer is mapped.
int vwa_ar_chain_tp(void* st, ChainTP* out) {
  auto* s = static_cast<ArState*>(st);
  const int64_t off = 2 * s->max_elems * (int64_t)sizeof(uint16_t) + 2 * kGatherWords * (int64_t)sizeof(int);
  *out = ChainTP{};
  out->world = s->world;
  out->rank = s->rank;
  for (int p = 0; p < s->world; ++p) {
    if (!s->peers.staging[p] || !s->peers.flags[p]) return -1;
    out->stage[p] = reinterpret_cast<float*>(reinterpret_cast<char*>(s->peers.staging[p]) + off);
    out->flag_out[p] = s->peers.flags[p] + kChainSlot * kMaxRanks + s->rank;
  }
  out->flag_in = s->flags + kChainSlot * kMaxRanks;
  out->epoch = s->epochs + kChainSlot;
  out->region = (int)kChainFloats;
  return 0;
}

// Non-zero if a call timed out waiting for a peer (sticky).
int vwa_ar_error(void* st) {
  auto* s = static_cast<ArState*>(st);
  int v = 0;
  (void)hipMemcpy(&v, s->error, sizeof(int), hipMemcpyDeviceToHost);
  return v;
}

void vwa_ar_destroy(void* st) {
  auto* s = static_cast<ArState*>(st);
  if (!s) return;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < s->world; ++p) {
    if (s->opened[p]) {
      (void)hipIpcCloseMemHandle(s->peers.staging[p]);
      (void)hipIpcCloseMemHandle(s->peers.flags[p]);
    }
  }
  (void)hipFree(s->staging);
  (void)hipFree(s->flags);
  (void)hipFree(s->epochs);
  (void)hipFree(s->error);
  delete s;
}

}  // extern "C"
