// xGMI peer-to-peer collectives for one MI355X node (gfx950).
//
// Role (SURVEY §2.3 N04, §2.5 plan item 2): RCCL carries the bandwidth-bound DDP/FSDP buckets;
// this module carries the LATENCY-bound small messages (grad-norm scalars, loss/metric
// reductions, tail buckets, barriers) where RCCL's ring/channel setup dominates. The 8 GPUs of a
// node are fully connected (one xGMI link to every peer), so a one-shot all-reduce in which
// every GPU reads its 7 peers' buffers directly uses all 7 links at once with one hop of latency.
//
// Memory model (MI355X_MICROARCH.md "inter-workgroup visibility"): per-XCD L2s are not coherent
// and a peer reads our HBM through the fabric, so a producer publishes with a SYSTEM-scope release
// (L2 write-back) before its flag store, and a consumer acquires at system scope after the poll.
// Flags live in fine-grained uncached memory (hipDeviceMallocUncached) exported over IPC.
//
// Protocol per call with sequence number e (identical on every rank, collective order):
//   one-shot:  block b copies its element range R_b of the input into its staging buffer
//              staging[e & 1], publishes, sets flag start[b][me] = e on EVERY rank, waits for
//              start[b][p] >= e from every peer, then sums R_b over all ranks' staging[e & 1].
//   two-shot:  as one-shot up to the start barrier; then rank r reduces only the sub-range r of
//              R_b into its result[e & 1], publishes, mid barrier, then gathers all W reduced
//              sub-ranges from the peers' result buffers.
// Double-buffering by e & 1 removes the closing barrier: a peer writes parity e & 1 again only
// in call e+2, after it passed call e+1's start barrier, which needs our e+1 flag, which we set
// after finishing every read of call e.
//
// Every wait is bounded by a wall-clock timeout (s_memrealtime, 100 MHz). Failure is fail-stop, never
// a silent wrong sum:
//   * a timed-out wait records the peer in the local error word, sets the abort word of EVERY rank
//     (so their pending and later calls stop waiting too) and the block writes NaN over its output;
//   * every call first reads the local error word and its own abort word: if either is set it
//     writes NaN over its whole output and returns without touching flags or peer memory;
//   * the host raises on the error word at its next synchronisation point (IpcCommunicator.check,
//     parallel/ipc.check_all from train.report / the SFT trainer / bench), and a NaN gradient or
//     grad norm is what any step that consumed a poisoned result sees in the meantime.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <cstring>
#include <stdexcept>
#include <string>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kThreads = 512;

struct IpcArgs {
  void* staging[kIpcMaxRanks];        // per rank: 2 parities x cap bytes
  void* result[kIpcMaxRanks];         // per rank: 2 parities x cap bytes (two-shot)
  uint32_t* signal[kIpcMaxRanks];     // per rank: [2 phases][kIpcMaxBlocks][kIpcMaxRanks]
  uint32_t* err;                      // local error word (0 = ok)
  int64_t cap;                        // bytes per parity
  int rank, world;
  uint32_t epoch;
  uint64_t timeout_ticks;
};

__device__ __forceinline__ uint32_t* flag_ptr(uint32_t* base, int phase, int block, int src) {
  return base + ((phase * kIpcMaxBlocks + block) * kIpcMaxRanks + src);
}

__device__ __forceinline__ uint32_t* abort_ptr(uint32_t* base) { return base + kIpcAbortWord; }

// Block-wide barrier across ranks for (phase, block). Producer side (MI355X_MICROARCH.md,
// "Valid forms"): every storing wave drains its stores, workgroup barrier, then lane i < world
// releases at SYSTEM scope (L2 write-back: the peer reads our HBM through the fabric), drains
// again (compiler hazard: the release's wait can be dropped) and stores the flag into rank i's
// signal array. Consumer side: one relaxed poll, one system-scope acquire, drain, barrier.
// Returns false (block-uniform) when a wait timed out or a peer announced an abort: the caller
// then poisons its output instead of reading peer buffers.
__device__ bool cross_rank_barrier(const IpcArgs& a, int phase, int* s_fail) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) *s_fail = 0;
  __syncthreads();
  const int b = blockIdx.x;
  if (threadIdx.x < (unsigned)a.world) {
    const int peer = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag_ptr(a.signal[peer], phase, b, a.rank), a.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flag_ptr(a.signal[a.rank], phase, b, peer);
    uint32_t* my_abort = abort_ptr(a.signal[a.rank]);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
      const uint32_t v = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - a.epoch) >= 0) break;
      if (__hip_atomic_load(my_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) {
        // a peer gave up on this (or an earlier) call: stop waiting, fail this call here too
        __hip_atomic_fetch_or(a.err, kIpcErrAborted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_fail = 1;  // benign race: every writer stores 1
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
        // the peer never arrived: record it, tell every rank (their waits on us or on it end now)
        __hip_atomic_fetch_or(a.err, 1u << (peer & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int r = 0; r < a.world; ++r) {  // (release per store: the timeout path, never hot)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(abort_ptr(a.signal[r]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        *s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  return *s_fail == 0;
}

// Entry check of every call: a set local error word or abort word means an earlier call (here or
// on a peer) failed; the call must not wait or read peers (their parities may be stale).
__device__ bool comm_poisoned(const IpcArgs& a, int* s_fail) {
  if (threadIdx.x == 0) {
    const uint32_t e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ab = __hip_atomic_load(abort_ptr(a.signal[a.rank]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const bool bad = e != 0u || ab != 0u;
    if (bad)
      __hip_atomic_fetch_or(a.err, kIpcErrSkipped | (ab != 0u ? kIpcErrAborted : 0u), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    *s_fail = bad ? 1 : 0;
  }
  __syncthreads();
  return *s_fail != 0;
}

// NaN over chunks [c0, c1) of the output (fp32 quiet NaN / a pair of bf16 quiet NaNs per word)
template <bool BF16>
__device__ void poison_range(uint4* out, int64_t c0, int64_t c1) {
  const uint32_t w = BF16 ? 0x7fc07fc0u : 0x7fc00000u;
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) out[c] = make_uint4(w, w, w, w);
}

__device__ __forceinline__ float bf16_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t rn_bf16(float f) {  // round-to-nearest-even, NaN-preserving
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t pack_bf16(float lo, float hi) { return rn_bf16(lo) | (rn_bf16(hi) << 16); }

// 16-byte chunk = 4 fp32 or 8 bf16 elements; accumulate in fp32.
template <bool BF16>
__device__ __forceinline__ void acc_chunk(float (&acc)[8], const uint4& v) {
  if constexpr (BF16) {
    acc[0] += bf16_lo(v.x); acc[1] += bf16_hi(v.x); acc[2] += bf16_lo(v.y); acc[3] += bf16_hi(v.y);
    acc[4] += bf16_lo(v.z); acc[5] += bf16_hi(v.z); acc[6] += bf16_lo(v.w); acc[7] += bf16_hi(v.w);
  } else {
    acc[0] += __uint_as_float(v.x); acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z); acc[3] += __uint_as_float(v.w);
  }
}
template <bool BF16>
__device__ __forceinline__ uint4 pack_chunk(const float (&acc)[8], float scale) {
  uint4 o;
  if constexpr (BF16) {
    o.x = pack_bf16(acc[0] * scale, acc[1] * scale); o.y = pack_bf16(acc[2] * scale, acc[3] * scale);
    o.z = pack_bf16(acc[4] * scale, acc[5] * scale); o.w = pack_bf16(acc[6] * scale, acc[7] * scale);
  } else {
    o.x = __float_as_uint(acc[0] * scale); o.y = __float_as_uint(acc[1] * scale);
    o.z = __float_as_uint(acc[2] * scale); o.w = __float_as_uint(acc[3] * scale);
  }
  return o;
}

// Reduce chunks [c0, c1) of every rank's `src` parity buffer into dst (local pointer).
template <bool BF16>
__device__ void reduce_range(const IpcArgs& a, void* const* bufs, int64_t par_off, int64_t c0, int64_t c1,
                             uint4* dst, float scale) {
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // fixed rank order 0..W-1 on every rank: bit-identical results everywhere
    for (int r = 0; r < a.world; ++r) {
      const uint4* s = reinterpret_cast<const uint4*>(static_cast<const char*>(bufs[r]) + par_off);
      acc_chunk<BF16>(acc, s[c]);
    }
    dst[c] = pack_chunk<BF16>(acc, scale);
  }
}

template <bool BF16, bool TWO_SHOT>
__global__ __launch_bounds__(kThreads) void ipc_allreduce_kernel(const IpcArgs a, const uint4* in, uint4* out,
                                                                 int64_t nchunks, float scale) {
  const int64_t per = (nchunks + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = (int64_t)blockIdx.x * per;
  const int64_t c1 = c0 + per < nchunks ? c0 + per : nchunks;
  const int64_t par = (int64_t)(a.epoch & 1u) * a.cap;
  __shared__ int s_fail;
  if (comm_poisoned(a, &s_fail)) {
    poison_range<BF16>(out, c0, c1);
    return;
  }
  uint4* mine = reinterpret_cast<uint4*>(static_cast<char*>(a.staging[a.rank]) + par);
  for (int64_t c = c0 + threadIdx.x; c < c1; c += blockDim.x) mine[c] = in[c];
  if (!cross_rank_barrier(a, 0, &s_fail)) {
    poison_range<BF16>(out, c0, c1);
    return;
  }
  if (!TWO_SHOT) {
    reduce_range<BF16>(a, a.staging, par, c0, c1, out, scale);
    return;
  }
  // two-shot: this rank reduces sub-range `rank` of R_b, then everyone gathers the sub-ranges
  const int64_t n = c1 > c0 ? c1 - c0 : 0;
  const int64_t sub = (n + a.world - 1) / a.world;
  const int64_t s0 = c0 + (int64_t)a.rank * sub < c1 ? c0 + (int64_t)a.rank * sub : c1;
  const int64_t s1 = s0 + sub < c1 ? s0 + sub : c1;
  uint4* res = reinterpret_cast<uint4*>(static_cast<char*>(a.result[a.rank]) + par);
  reduce_range<BF16>(a, a.staging, par, s0, s1, res, scale);
  if (!cross_rank_barrier(a, 1, &s_fail)) {
    poison_range<BF16>(out, c0, c1);
    return;
  }
  for (int r = 0; r < a.world; ++r) {
    const int64_t g0 = c0 + (int64_t)r * sub < c1 ? c0 + (int64_t)r * sub : c1;
    const int64_t g1 = g0 + sub < c1 ? g0 + sub : c1;
    const uint4* src = reinterpret_cast<const uint4*>(static_cast<const char*>(a.result[r]) + par);
    for (int64_t c = g0 + threadIdx.x; c < g1; c += blockDim.x) out[c] = src[c];
  }
}

// Barrier only (no payload): phase-0 flags of block 0.
__global__ __launch_bounds__(64) void ipc_barrier_kernel(const IpcArgs a) {
  __shared__ int s_fail;
  if (comm_poisoned(a, &s_fail)) return;
  cross_rank_barrier(a, 0, &s_fail);
}

IpcArgs make_args(const IpcPeers& p, uint32_t epoch) {
  IpcArgs a{};
  for (int i = 0; i < kIpcMaxRanks; ++i) {
    a.staging[i] = p.staging[i];
    a.result[i] = p.result[i];
    a.signal[i] = p.signal[i];
  }
  a.err = p.err;
  a.cap = p.cap;
  a.rank = p.rank;
  a.world = p.world;
  a.epoch = epoch;
  a.timeout_ticks = p.timeout_ticks;
  return a;
}

}  // namespace

int ipc_blocks_for(int64_t nbytes, bool two_shot) {
  // ~64 KiB per block (one-shot reads W x that), at least 1, at most kIpcMaxBlocks
  const int64_t per = two_shot ? (int64_t)256 << 10 : (int64_t)64 << 10;
  int64_t b = (nbytes + per - 1) / per;
  if (b < 1) b = 1;
  if (b > kIpcMaxBlocks) b = kIpcMaxBlocks;
  return (int)b;
}

void ipc_allreduce(const IpcPeers& peers, uint32_t epoch, DType dt, const void* in, void* out, int64_t nbytes,
                   bool two_shot, float scale, hipStream_t s) {
  const IpcArgs a = make_args(peers, epoch);
  const int64_t nchunks = nbytes / 16;
  const int blocks = ipc_blocks_for(nbytes, two_shot);
  const uint4* i4 = static_cast<const uint4*>(in);
  uint4* o4 = static_cast<uint4*>(out);
  if (dt == DType::BF16) {
    if (two_shot) hipLaunchKernelGGL((ipc_allreduce_kernel<true, true>), dim3(blocks), dim3(kThreads), 0, s, a, i4, o4, nchunks, scale);
    else hipLaunchKernelGGL((ipc_allreduce_kernel<true, false>), dim3(blocks), dim3(kThreads), 0, s, a, i4, o4, nchunks, scale);
  } else {
    if (two_shot) hipLaunchKernelGGL((ipc_allreduce_kernel<false, true>), dim3(blocks), dim3(kThreads), 0, s, a, i4, o4, nchunks, scale);
    else hipLaunchKernelGGL((ipc_allreduce_kernel<false, false>), dim3(blocks), dim3(kThreads), 0, s, a, i4, o4, nchunks, scale);
  }
}

void ipc_barrier(const IpcPeers& peers, uint32_t epoch, hipStream_t s) {
  hipLaunchKernelGGL(ipc_barrier_kernel, dim3(1), dim3(64), 0, s, make_args(peers, epoch));
}

// ---------------- host-side buffer management (IPC export / import) ----------------
static void ipc_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ipc_comm: ") + what + ": " + hipGetErrorString(e));
}

void* ipc_malloc(int64_t nbytes, bool fine_grained) {
  void* p = nullptr;
  if (fine_grained) ipc_check(hipExtMallocWithFlags(&p, (size_t)nbytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  else ipc_check(hipMalloc(&p, (size_t)nbytes), "hipMalloc");
  ipc_check(hipMemset(p, 0, (size_t)nbytes), "hipMemset");
  ipc_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return p;
}

void ipc_free(void* p) { ipc_check(hipFree(p), "hipFree"); }

void ipc_get_handle(void* p, char out[kIpcHandleBytes]) {
  hipIpcMemHandle_t h;
  ipc_check(hipIpcGetMemHandle(&h, p), "hipIpcGetMemHandle");
  static_assert(sizeof(h) <= kIpcHandleBytes, "IPC handle size");
  std::memset(out, 0, kIpcHandleBytes);
  std::memcpy(out, &h, sizeof(h));
}

void* ipc_open_handle(const char in[kIpcHandleBytes]) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, in, sizeof(h));
  void* p = nullptr;
  ipc_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return p;
}

void ipc_close_handle(void* p) { ipc_check(hipIpcCloseMemHandle(p), "hipIpcCloseMemHandle"); }

}  // namespace grt
