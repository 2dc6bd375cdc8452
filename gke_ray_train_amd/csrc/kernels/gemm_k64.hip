// Projection GEMM for gfx950, 256 x 256 x 64 tiles:  C[M][N] (+)= sum_k A[M][K] * B[N][K]
// (bf16 in, fp32 accumulate, bf16 out). Reference: the cuBLAS GEMMs under nn.Linear
// (ray-jobs/pytorch_llm_ray.py:82-87) and the HF Llama projections under SFTTrainer.train()
// (ray-jobs/fine_tune_llama_ray.py:333); SURVEY §2.3 N02, §2.6 K-B04.
//
// Structure (one workgroup per CU: 4 waves, one per SIMD, 128 x 128 outputs per wave):
//   * accumulators: 8 x 8 blocks of v_mfma_f32_16x16x32_bf16 = 256 AGPRs, pinned by inline-asm
//     MFMAs ("+a"); 128 MFMAs per 64-deep K-tile;
//   * fragments: 128 VGPRs = the tile's two 32-deep halves (kk0, kk1) for A and B. The kk1 half of
//     tile t is read from LDS under the kk0 MFMAs of tile t, the kk0 half of tile t+1 under the kk1
//     MFMAs of tile t, so every ds_read has >= 20 MFMAs of cover;
//   * LDS: two K-tile buffers (A + B each), 130 KiB. An operand tile is 32 chunks of 1040 B; chunk
//     c holds rows {128 (c >> 4) + 16 b + (c & 15)}, b = 0..7, as 128-B lines (the row's 64 k) at
//     b * 128 — one LDS-DMA instruction of one wave fills one chunk with eight whole cache lines,
//     and the 16-B pad makes the 16 rows a 16x16x32 fragment read sit in 16 different bank
//     quads (conflict-free up to one 2-way pair per lane group);
//   * global -> LDS: buffer_load ... lds (LDS-DMA, no VGPR round trip), 16 per wave per K-tile, one
//     SALU (M0) each; the tile origin lives in the buffer descriptor base (scalar), per-instruction
//     row offsets in SGPR soffsets, the lane part in one VGPR per operand;
//   * one K-tile period = 128 MFMAs with three barriers (cdna_hip_programming.md §5, "glds >1 tile in
//     flight": raw s_barrier, counted vmcnt, never vmcnt(0) in the loop):
//       MFMA  0-21  read A kk1 (tile t, buffer u)                      -> lgkmcnt(0), barrier 1
//       MFMA 22-51  read B kk1 (tile t); DMA A of tile t+2 into u (5)  -> lgkmcnt(0), barrier 2
//       MFMA 52-92  DMA A (3) + B (5) of tile t+2 into u               -> vmcnt(13), barrier 3
//       MFMA 93-127 read kk0 of tile t+1 (buffer u^1); DMA B (3)
//     Barrier 1 proves every wave has read A of buffer u for the last time (its kk0 half was read in
//     the previous period, its kk1 half before barrier 1), barrier 2 the same for B, so the DMAs of
//     tile t+2 may overwrite them. vmcnt(13) at barrier 3 leaves exactly this period's 13 DMAs in
//     flight: the 16 of the previous period (tile t+1) have landed before anyone reads tile t+1.
//     DMAs get >= one full period to land; past the last tile they re-fetch tile T-1 into a buffer
//     nobody reads again (branch-free loop, constant vmcnt);
//   * blockIdx -> tile: bijective XCD remap, then 8-row groups (T1).
// Requirements (host-checked): M % 256 == 0, N % 256 == 0, K % 128 == 0, K >= 128, row strides
// multiples of 8 elements, 16-byte aligned bases, every operand byte offset below 2^31.
#include "grt_common.h"
#include "grt_kernels.h"

#include <type_traits>
#include <utility>

namespace grt {
namespace {

constexpr int KT = 64;           // reduction depth of one tile
constexpr int CH = 1040;         // one LDS chunk: 8 rows x 128 B + 16 B pad
constexpr int TEN = 32 * CH;     // one operand tile (256 rows)
constexpr int BUFB = 2 * TEN;    // A + B of one K-tile
constexpr int LDSB = 2 * BUFB;   // two K-tile buffers = 133,120 B
constexpr int kGroupRows = 8;

// MFMA with the accumulator pinned to AGPRs; the compiler does not model the asm, every
// accumulator is next touched >= 56 MFMAs later, and the epilogue pads the final hazard.
__device__ __forceinline__ void mfma16(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// LDS-DMA of 16 B per lane to M0 + 16 * lane; M0 = wave base + OFF. Inline asm so the compiler
// neither counts it (its waitcnt pass would drain vmcnt) nor keeps M0 (declared clobbered: nothing
// else in this kernel uses it). M0 is set by s_mov from an SGPR the compiler computed: an s_add in
// the asm would clobber SCC behind the compiler's back (it schedules these statements between its
// own s_cmp / s_cselect and s_add / s_addc pairs).
template <int OFF>
__device__ __forceinline__ void dma(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc, uint32_t soff, uint32_t mbase) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :: "v"(voff), "s"(rsrc), "s"(mbase + OFF), "s"(soff) : "memory", "m0");
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- per-period schedule: what rides behind MFMA number I (0..127) --------------------------
// seg 1: A kk1 reads; seg 2: B kk1 reads + A DMAs 0-4; seg 3: A DMAs 5-7, B DMAs 0-4;
// seg 4: kk0 reads of the next tile (B0[0], A0[0], B0[1..7], A0[1..7]) + B DMAs 5-7
constexpr int kReadA1[8] = {0, 2, 5, 8, 11, 13, 16, 18};
constexpr int kReadB1[8] = {22, 25, 28, 31, 34, 37, 40, 43};
constexpr int kDmaA[8] = {23, 29, 35, 41, 47, 53, 58, 63};
constexpr int kDmaB[8] = {68, 73, 78, 83, 88, 98, 108, 118};
constexpr int kRead0First = 93;  // 16 reads at 93, 95, ..., 123
constexpr int kBar1 = 21, kBar2 = 51, kBar3 = 92;

constexpr int find8(const int (&t)[8], int i) {
  for (int q = 0; q < 8; ++q)
    if (t[q] == i) return q;
  return -1;
}

template <int EPI, int DBG>
__global__ __launch_bounds__(256, 1) void gemm_k64_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;

  // ---- tile coordinates: bijective XCD remap, then grouped order
  const int nM = p.M / 256, nN = p.N / 256, nwg = nM * nN;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupRows * nN;
  const int grp = wg / per_group, first = grp * kGroupRows;
  const int gsize = min(nM - first, kGroupRows);
  const int tm = first + (wg % per_group) % gsize, tn = (wg % per_group) / gsize;
  GRT_DEVICE_CHECK(tm < nM && tn < nN);
  const int m0 = tm * 256, n0 = tn * 256;
  const int T = p.K / KT;

  // ---- DMA addressing: wave w, instruction q fills chunk 4q + w: lane l carries row
  // 128 (q >> 2) + 16 (l >> 3) + 4 (q & 3) + w, k-chunk l & 7
  const char* abase = static_cast<const char*>(p.a) + ((int64_t)m0 * p.lda) * 2;
  const char* bbase = static_cast<const char*>(p.b) + ((int64_t)n0 * p.ldb) * 2;
  const uint32_t avoff = (uint32_t)(((16 * (lane >> 3) + w) * p.lda + 8 * (lane & 7)) * 2);
  const uint32_t bvoff = (uint32_t)(((16 * (lane >> 3) + w) * p.ldb + 8 * (lane & 7)) * 2);
  const uint32_t lda2 = (uint32_t)p.lda * 2, ldb2 = (uint32_t)p.ldb * 2;
  uint32_t soa[8], sob[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    soa[q] = (uint32_t)(128 * (q >> 2) + 4 * (q & 3)) * lda2;
    sob[q] = (uint32_t)(128 * (q >> 2) + 4 * (q & 3)) * ldb2;
  }
  const uint32_t mbase = __builtin_amdgcn_readfirstlane(lds_u32(smem) + w * CH);
  auto rsrc = [](const char* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, 0x7fffffff, 0x00020000);
  };

  // ---- fragment addressing: lane l reads row (l & 15) of a 16-row block, k-chunk (l >> 4) (+4 kk)
  const int lf = (lane & 15) * CH + (lane >> 4) * 16;
  const char* fa[2] = {smem + 0 * BUFB + 16 * wr * CH + lf, smem + 1 * BUFB + 16 * wr * CH + lf};
  const char* fb[2] = {smem + 0 * BUFB + TEN + 16 * wc * CH + lf, smem + 1 * BUFB + TEN + 16 * wc * CH + lf};
  auto frag = [](const char* base, int blk, int kk) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(base + blk * 128 + kk * 64);
  };

  // accumulators zeroed by the matrix pipe itself (MFMA with an inline-constant 0 accumulator and
  // zero operands): no VALU-write -> MFMA-read hazard, and the compiler sees each one defined by an
  // asm statement, so it neither re-materialises nor copies them
  f32x4 acc[8][8];
  {
    const bf16x8 zf = {};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(zf));
  }
  bf16x8 a0[8], a1[8], b0[8], b1[8];

  // ---- prologue: tiles 0 and 1 in flight (32 DMAs), kk0 of tile 0 into registers
  {
    const auto ra0 = rsrc(abase), rb0 = rsrc(bbase);
    const auto ra1 = rsrc(abase + (T > 1 ? KT * 2 : 0)), rb1 = rsrc(bbase + (T > 1 ? KT * 2 : 0));
    static_for<8>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      dma<0 * BUFB + 0 + q * 4 * CH>(avoff, ra0, soa[q], mbase);
    });
    static_for<8>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      dma<0 * BUFB + TEN + q * 4 * CH>(bvoff, rb0, sob[q], mbase);
    });
    static_for<8>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      dma<1 * BUFB + 0 + q * 4 * CH>(avoff, ra1, soa[q], mbase);
    });
    static_for<8>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      dma<1 * BUFB + TEN + q * 4 * CH>(bvoff, rb1, sob[q], mbase);
    });
    if constexpr (DBG & 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { b0[j] = frag(fb[0], j, 0); a0[j] = frag(fa[0], j, 0); }
    if constexpr (DBG & 1) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    if constexpr (DBG & 64) {  // debug: wave 0's first A / B fragments and the tile-0 MFMA of block (0,0)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      if (w == 0) {
        reinterpret_cast<bf16x8*>(p.c)[lane] = a0[0];
        reinterpret_cast<bf16x8*>(p.c)[64 + lane] = b0[0];
        f32x4 z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[0], a0[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        reinterpret_cast<f32x4*>(p.c)[128 + lane] = z;
      }
      return;
    }
    if constexpr (DBG & 4) {  // debug: dump buffer 0 (A and B images of tile 0) to C and stop
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      for (int x = tid; x < BUFB / 16; x += 256)
        reinterpret_cast<uint4*>(p.c)[x] = reinterpret_cast<const uint4*>(smem)[x];
      return;
    }
  }

  // ---- one K-tile period on buffer U (compile-time) for tile t
  auto period = [&](int t, auto U_) {
    constexpr int U = decltype(U_)::value;
    const int td = min(t + 2, T - 1);  // tile whose DMAs ride in this period
    const auto ra = rsrc(abase + (int64_t)td * (KT * 2));
    const auto rb = rsrc(bbase + (int64_t)td * (KT * 2));
    static_for<128>([&](auto I_) {
      constexpr int I = decltype(I_)::value;
      constexpr int kk = I / 64, i = (I % 64) / 8, j = I % 8;
      if constexpr (DBG & 2) {
        if constexpr (kk == 0) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b0[j], a0[i], acc[i][j], 0, 0, 0);
        else acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b1[j], a1[i], acc[i][j], 0, 0, 0);
      } else {
        if constexpr (kk == 0) mfma16(acc[i][j], b0[j], a0[i]);
        else mfma16(acc[i][j], b1[j], a1[i]);
      }
      constexpr int ra1q = find8(kReadA1, I), rb1q = find8(kReadB1, I);
      constexpr int dAq = find8(kDmaA, I), dBq = find8(kDmaB, I);
      if constexpr (ra1q >= 0) a1[ra1q] = frag(fa[U], ra1q, 1);
      if constexpr (rb1q >= 0) b1[rb1q] = frag(fb[U], rb1q, 1);
      if constexpr (dAq >= 0) dma<U * BUFB + 0 + dAq * 4 * CH>(avoff, ra, soa[dAq], mbase);
      if constexpr (dBq >= 0) dma<U * BUFB + TEN + dBq * 4 * CH>(bvoff, rb, sob[dBq], mbase);
      if constexpr (I >= kRead0First && I < kRead0First + 32 && (I - kRead0First) % 2 == 0) {
        constexpr int x = (I - kRead0First) / 2;  // 0: B0[0], 1: A0[0], 2..8: B0[1..7], 9..15: A0[1..7]
        if constexpr (x == 0) b0[0] = frag(fb[U ^ 1], 0, 0);
        else if constexpr (x == 1) a0[0] = frag(fa[U ^ 1], 0, 0);
        else if constexpr (x <= 8) b0[x - 1] = frag(fb[U ^ 1], x - 1, 0);
        else a0[x - 8] = frag(fa[U ^ 1], x - 8, 0);
      }
      if constexpr (I == kBar1 || I == kBar2) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      if constexpr (I == kBar3) {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(13)\n\ts_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  if constexpr (DBG & 16) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15" ::: "memory");
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) mfma16(acc[i][j], b0[j], a0[i]);
  } else {
    if constexpr (DBG & 32) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    int t = 0;
    do {  // T >= 2 (host check): no zero-trip path, so no phi copies of the accumulators at the exit
      period(t, Z{});
      period(t + 1, O{});
      t += 2;
    } while (t < T);
  }
  // the last MFMAs' results are read by VALU below: 3 x 8 wait states (8-pass XDL write -> VALU
  // read), then an empty asm "redefines" every accumulator so no read is hoisted above the pad
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (DBG & 128) {  // debug: raw fp32 accumulators of block (0,0) and (7,7) of wave 0
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (w == 0) {
      reinterpret_cast<f32x4*>(p.c)[lane] = acc[0][0];
      reinterpret_cast<f32x4*>(p.c)[64 + lane] = acc[7][7];
    }
    return;
  }

  // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + 128 wr + 16 i + (lane & 15),
  // n = n0 + 128 wc + 16 j + 4 (lane >> 4)
  bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(m0 + 128 * wr + (lane & 15)) * p.ldc + n0 + 128 * wc + 4 * (lane >> 4);
  auto store_row = [&](int i, bool accumulate) {
    bf16* crow = cbase + (int64_t)16 * i * p.ldc;
    bf16x4 old[8];
    if (accumulate) {
#pragma unroll
      for (int j = 0; j < 8; ++j) old[j] = *reinterpret_cast<const bf16x4*>(crow + 16 * j);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        r[e] = static_cast<bf16>(accumulate ? acc[i][j][e] + static_cast<float>(old[j][e]) : acc[i][j][e]);
      *reinterpret_cast<bf16x4*>(crow + 16 * j) = r;
    }
  };
  if (p.beta) {
#pragma unroll
    for (int i = 0; i < 8; ++i) store_row(i, true);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) store_row(i, false);
  }
}

}  // namespace

bool gemm_nt_k64_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  if (M <= 0 || N <= 0 || K < 128 || M % 256 || N % 256 || K % 128) return false;
  if ((M / 256) * (N / 256) > INT32_MAX) return false;
  // descriptor offsets: lane part + soffset of the 255th row + 64 k, 32-bit signed range
  if ((255 * lda + 64) * 2 >= (int64_t(1) << 31) || (255 * ldb + 64) * 2 >= (int64_t(1) << 31)) return false;
  return true;
}

void gemm_nt_k64(const GemmParams& p, hipStream_t stream) {
  const int nwg = (p.M / 256) * (p.N / 256);
  if (p.variant == 10) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 1>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 11) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 2>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 12) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 3>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 13) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 4>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 14) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 16>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 16) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 64>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 17) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 128>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 18) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 130>), dim3(nwg), dim3(256), 0, stream, p);
  else if (p.variant == 15) hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 32>), dim3(nwg), dim3(256), 0, stream, p);
  else hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, 0>), dim3(nwg), dim3(256), 0, stream, p);
}

}  // namespace grt
