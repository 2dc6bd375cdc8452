// Projection GEMM for gfx950:  C[M][N] (+)= sum_k A[M][K] * B[N][K]    (bf16 in, fp32 acc, bf16 out)
//
// Role: hand-written forms of the Llama projection GEMMs (reference: the cuBLAS GEMMs under
// nn.Linear in ray-jobs/pytorch_llm_ray.py:82-87 and the HF Llama projections under
// SFTTrainer.train(), ray-jobs/fine_tune_llama_ray.py:333). The
// training step runs the tuned hipBLASLt kernels for these (faster, profiles/r4_gemm_family.md,
// profiles/r5_gemm_k64.md); this file holds the round-4 family (variants 1-8: ping-pong 8-wave,
// 4-wave AGPR, TT / NN operand forms) and dispatches variants 9-16 to gemm_k64.hip. Only the plain
// store / accumulate epilogues exist (no fused elementwise epilogue).
//
// Design (cdna_hip_programming.md §5 "256² 8-phase template", T1-T5; MI355X_MICROARCH.md §LDS):
//   * 256 x 256 output tile per workgroup, 8 waves = 2 wave groups (rows) x 4 (cols), 128 x 64 per
//     wave = 8 x 4 accumulators of v_mfma_f32_16x16x32_bf16 (128 AGPR/VGPR);
//   * the reduction runs in 32-deep SLOTS: one slot = A[256][32] + B[256][32] = 32 KiB in LDS, a ring
//     of 4 slots (128 KiB), each filled by 4 global_load_lds_dwordx4 per thread (LDS-DMA, no VGPR
//     round trip). An image row is 64 B; the 16-B chunk c of row r sits at chunk c ^ 2*((r >> 3) & 1),
//     which makes every ds_read_b128 16-lane group of the 16x16x32 operand read conflict-free; the
//     swizzle is applied to the per-lane SOURCE address so the lane-linear DMA lands in the swizzled
//     image (rule 21);
//   * PING-PONG: the two waves of a SIMD (wave w and w+4, one per group) alternate a LOAD segment
//     (ds_read the next fragments, issue 2 DMAs) and a COMPUTE segment (16 MFMAs) between workgroup
//     barriers; group 1 runs one barrier behind group 0, so each SIMD's matrix pipe always has one
//     wave in its compute segment while the other reads LDS;
//   * a slot is consumed in two phases (the wave's upper and lower 64 rows); B fragments are read
//     once per slot, A fragments once per phase: 24 ds_read_b128 per wave per 64-deep step, the
//     minimum for this wave tile;
//   * DMA stream: slot j is issued in phases 2j-5 / 2j-4 and waited for with a COUNTED vmcnt(6) at the
//     end of every odd phase (never 0 in the main loop), i.e. 2.5 slots stay in flight across the
//     barriers; refills start only after the barrier that proves every wave finished the slot's last
//     read (the barrier-count argument is written out at the loop);
//   * C is computed transposed per MFMA (B fragment as the A operand) so each lane holds 4 consecutive
//     output columns: 8-byte stores; blockIdx -> tile: bijective XCD remap + 8-row groups (T1).
// Requirements (checked on the host): M % 256 == 0, N % 256 == 0, K % 128 == 0, K > 0, row strides
// multiples of 8 elements, 16-byte aligned bases.
#include "grt_common.h"
#include "grt_kernels.h"

#include <type_traits>

namespace grt {
namespace {

constexpr int GT = 256;            // output tile edge
constexpr int GS = 32;             // reduction depth of one ring slot
constexpr int GNT = 512;           // 8 waves
constexpr int OPB = GT * GS * 2;   // 16 KiB: one operand in one slot
constexpr int SLOTB = 2 * OPB;     // 32 KiB
constexpr int kGroupRows = 8;

// LDS-DMA of 16 bytes per lane to (wave-uniform LDS byte address) + lane * 16. Inline asm so hipcc
// does not count it: its waitcnt pass would otherwise drain vmcnt before every LDS read of the loop.
// M0 is saved and restored around the DMA (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gptr), "s"(lds_addr) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
__device__ __forceinline__ void wait_vm(int pending) {
  // pending = DMA instructions of this wave allowed to stay in flight (multiple of 2, <= 8)
  if (pending >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (pending >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (pending >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (pending >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// chunk swizzle of a 64-byte image row (see header); depends on r & 15 only
__device__ __forceinline__ int kc_swz(int r) { return ((r >> 3) & 1) << 1; }

// 16x16x32 operand fragment of rows rb .. rb+15 (rb % 16 == 0): lane l gets row rb + (l & 15),
// reduction elements 8 (l >> 4) .. +7 of the slot
__device__ __forceinline__ bf16x8 kc_frag(const char* img, int rb, int lane) {
  const int r = lane & 15;
  return *reinterpret_cast<const bf16x8*>(img + (rb + r) * 64 + 16 * ((lane >> 4) ^ kc_swz(r)));
}

template <int EPI, int PH, int RING>
__global__ __launch_bounds__(GNT, 1) void gemm_nt_kernel(const GemmParams p) {
  static_assert(PH == 1 || PH == 2, "phases per slot");
  static_assert(RING * SLOTB <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[RING * SLOTB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- tile coordinates: bijective XCD remap, then grouped order (kGroupRows row tiles per group)
  const int nM = p.M / GT, nN = p.N / GT, nwg = nM * nN;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupRows * nN;
  const int grp = wg / per_group, first = grp * kGroupRows;
  const int gsize = min(nM - first, kGroupRows);
  const int tm = first + (wg % per_group) % gsize, tn = (wg % per_group) / gsize;
  GRT_DEVICE_CHECK(tm < nM && tn < nN);
  const int m0 = tm * GT, n0 = tn * GT;

  // ---- DMA sources: thread (w, lane) fills image rows 16 (8 i + w) + (lane >> 2), chunk lane & 3
  // (linear), i = 0, 1, from source chunk (lane & 3) ^ kc_swz(row)
  const int drow = w * 16 + (lane >> 2);
  const int dch = (lane & 3) ^ kc_swz(lane >> 2);
  const bf16* asrc = static_cast<const bf16*>(p.a) + (int64_t)(m0 + drow) * p.lda + 8 * dch;
  const bf16* bsrc = static_cast<const bf16*>(p.b) + (int64_t)(n0 + drow) * p.ldb + 8 * dch;
  const int64_t astep = (int64_t)128 * p.lda, bstep = (int64_t)128 * p.ldb;
  const uint32_t lds0 = lds_addr(smem) + w * 1024;
  const int S = p.K / GS;
  auto dma_a = [&](int j) {
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + (j % RING) * SLOTB);
    glds16(asrc + j * GS, d);
    glds16(asrc + astep + j * GS, d + 8192);
  };
  auto dma_b = [&](int j) {
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + (j % RING) * SLOTB + OPB);
    glds16(bsrc + j * GS, d);
    glds16(bsrc + bstep + j * GS, d + 8192);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  // ---- DMA schedule. PH == 2: slot j is issued in phases 2j-5 (A) and 2j-4 (B), so the prologue
  // issues slots 0..2 and the odd-phase wait leaves slot j+1 and half of j+2 in flight (vmcnt(6)).
  // PH == 1: slot j is issued in phase j-(RING-2), so the prologue issues slots 0..RING-3 and the
  // per-phase wait leaves RING-3 slots in flight.
  constexpr int PRO = PH == 2 ? 3 : RING - 2;
  static_assert(PH == 1 || RING == 4, "PH == 2 schedule is written for a 4-slot ring");
  for (int j = 0; j < PRO; ++j)
    if (j < S) { dma_a(j); dma_b(j); }
  {
    int pend = 0;
    for (int j = 1; j < PRO; ++j) pend += j < S ? 4 : 0;
    wait_vm(pend);
  }
  barrier();
  if (wr == 1) barrier();  // group 1 runs one barrier behind group 0

  // ---- main loop (PH == 2 shown; PH == 1 is the same with one phase per slot). Phase P = 2 s + qm
  // reads slot s for the wave's rows qm*64..+64. Group 0 runs L_P before barrier #2P and C_P between
  // #2P and #2P+1; group 1 runs L_P between #2P and #2P+1 and C_P between #2P+1 and #2P+2. The reads
  // of slot s complete (lgkmcnt) at the start of the C segments of its last phase, so after the
  // barrier that follows group 1's last C of slot s no wave reads it any more: its buffer is refilled
  // only in phases that start after that barrier. Slot j is read first in group 0's L_{PH*j}: every
  // wave retires its own DMAs of slot j with the counted wait at the end of the phase before it.
  bf16x8 bf[4], af[PH == 2 ? 4 : 8];
  auto phase = [&](int s, auto qm_c) {
    constexpr int qm = decltype(qm_c)::value;
    const char* aimg = smem + (s % RING) * SLOTB;
    const char* bimg = aimg + OPB;
    // ---- LOAD segment
    if constexpr (qm == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = kc_frag(bimg, wc * 64 + 16 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < (PH == 2 ? 4 : 8); ++i) af[i] = kc_frag(aimg, wr * 128 + qm * 64 + 16 * i, lane);
    if constexpr (PH == 2) {
      if constexpr (qm == 1) {
        if (s + 3 < S) dma_a(s + 3);
        wait_vm((s + 2 < S ? 4 : 0) + (s + 3 < S ? 2 : 0));
      } else {
        if (s >= 1 && s + 2 < S) dma_b(s + 2);
      }
    } else {
      const int jn = s + RING - 2;
      if (jn < S) { dma_a(jn); dma_b(jn); }
      int pend = 0;
#pragma unroll
      for (int j = 2; j <= RING - 2; ++j) pend += s + j < S ? 4 : 0;
      wait_vm(pend);
    }
    barrier();
    // ---- COMPUTE segment
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < (PH == 2 ? 4 : 8); ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[qm * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[qm * 4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  for (int s = 0; s < S; ++s) {
    phase(s, Z{});
    if constexpr (PH == 2) phase(s, O{});
  }
  if (wr == 0) barrier();  // balance group 1's extra barrier

  // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + wr*128 + 16 i + (lane & 15),
  // n = n0 + wc*64 + 16 j + 4 (lane >> 4)
  const int g = lane >> 4, l16 = lane & 15;
  if constexpr (EPI == GEMM_EPI_STORE) {
    bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(m0 + wr * 128 + l16) * p.ldc + n0 + wc * 64 + 4 * g;
    auto store_row = [&](int i, bool accumulate) {
      bf16* crow = cbase + (int64_t)16 * i * p.ldc;
      bf16x4 old[4];
      if (accumulate) {
#pragma unroll
        for (int j = 0; j < 4; ++j) old[j] = *reinterpret_cast<const bf16x4*>(crow + 16 * j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
}

// ---------------------------------------------------------------------------------------------
// Variant 3: 64-deep K-tiles staged as four 128-row HALF-TILES of full 128-B rows (whole cache
// lines per DMA piece), two K-tile buffers (128 KiB). Half-tiles are quadrant-shaped: A_qm holds
// the A rows every wave reads in quadrant row qm (64 rows of each wave group), B_qn the B rows of
// quadrant column qn (32 rows of each wave column), so a half-tile is read in exactly one phase:
//   phase 0: A_0 + B_0 (12 ds_read_b128), phase 1: B_1 (4), phase 2: A_1 (8), phase 3: none
// (quadrant order (0,0) (0,1) (1,1) (1,0); B_0 stays in registers for phase 3).
// Half-tile H of K-tile t is refilled (K-tile t+2) two phases after its read, in the phase order
// B_1, A_1, A_0, B_0 (one half-tile = 2 DMAs per thread per phase) and waited for four phases
// later with a counted vmcnt(8): four half-tiles always in flight.
__device__ __forceinline__ int hswz(int r) { return (r >> 1) & 7; }  // chunk XOR of a 128-B row

// TT = true: the weight-gradient form C[P][Q] = sum_r X[r][p] Y[r][q] on token-major operands
// (a = X [R][P], b = Y [R][Q]): the half-tiles are [64 r][128 p|q] images of 256-B rows (T10 (b)
// XOR layout, whole cache lines per DMA piece) and the MFMA operands come from
// ds_read_b64_tr_b16 transposed reads — no transpose pass over dY or X.
__device__ __forceinline__ int tswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ bf16x4 tt_read(const char* base, int r0, int c0, int l16) {
  const int q = l16 >> 2, col = c0 + 4 * (l16 & 3);
  const char* a = base + (r0 + q) * 256 + 16 * ((col >> 3) ^ tswz(r0 + q)) + 8 * ((col >> 2) & 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)a);
}

template <int EPI, bool AT, bool BT>
__global__ __launch_bounds__(GNT, 1) void gemm_h_kernel(const GemmParams p) {
  constexpr int HT = 16384;  // one half-tile: 128 rows x 128 B
  constexpr int BUF = 4 * HT;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;
  const int nM = p.M / GT, nN = p.N / GT, nwg = nM * nN;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupRows * nN;
  const int grp = wg / per_group, first = grp * kGroupRows;
  const int gsize = min(nM - first, kGroupRows);
  const int tm = first + (wg % per_group) % gsize, tn = (wg % per_group) / gsize;
  GRT_DEVICE_CHECK(tm < nM && tn < nN);
  const int m0 = tm * GT, n0 = tn * GT;
  const int T = p.K / 64;

  // ---- DMA sources (per thread; + quadrant offset, + instruction i, + K-tile t). K-contiguous
  // operand: wave w, instruction i (0, 1) fills image rows 64 i + 8 w + (lane >> 3), chunk lane & 7.
  // Token-major operand: image rows (the reduction index) 32 i + 4 w + (lane >> 4), chunk lane & 15;
  // image column chunk c holds p (resp. q) columns of its quadrant-half group.
  const bf16* abase;
  const bf16* bbase;
  int64_t a_q, b_q, a_i, b_i, a_t, b_t;  // element offsets per quadrant half / instruction / K-tile
  const int kc_ch = (lane & 7) ^ ((4 * (w & 1) + (lane >> 4)) & 7);
  const int t_row0 = 4 * w + (lane >> 4);
  const int t_c = (lane & 15) ^ tswz(t_row0);
  if constexpr (!AT) {
    abase = static_cast<const bf16*>(p.a) + (int64_t)(m0 + 8 * w + (lane >> 3)) * p.lda + 8 * kc_ch;
    a_q = 64 * p.lda; a_i = 128 * p.lda; a_t = 64;
  } else {
    abase = static_cast<const bf16*>(p.a) + (int64_t)t_row0 * p.lda + m0 + (t_c >> 3) * 128 + 8 * (t_c & 7);
    a_q = 64; a_i = 32 * p.lda; a_t = 64 * p.lda;
  }
  if constexpr (!BT) {
    bbase = static_cast<const bf16*>(p.b) + (int64_t)(n0 + (w >> 2) * 64 + 8 * (w & 3) + (lane >> 3)) * p.ldb + 8 * kc_ch;
    b_q = 32 * p.ldb; b_i = 128 * p.ldb; b_t = 64;
  } else {
    bbase = static_cast<const bf16*>(p.b) + (int64_t)t_row0 * p.ldb + n0 + (t_c >> 2) * 64 + 8 * (t_c & 3);
    b_q = 32; b_i = 32 * p.ldb; b_t = 64 * p.ldb;
  }
  const uint32_t lds0 = lds_addr(smem) + w * 1024;
  // kind r: 0 = B_1, 1 = A_1, 2 = A_0, 3 = B_0 (the issue order within a K-tile period)
  auto issue = [&](int Q) {
    const int tq = Q >= 0 ? Q >> 2 : -((3 - Q) >> 2);  // floor(Q / 4)
    const int r = Q - 4 * tq;
    const int t = tq + (r < 2 ? 1 : 2);
    if (t >= T) return;
    const bool isA = r == 1 || r == 2;
    const int q = (r == 0 || r == 1) ? 1 : 0;  // quadrant half
    const int slot = isA ? q : 2 + q;          // A_0, A_1, B_0, B_1
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + (t & 1) * BUF + slot * HT);
    if (isA) {
      const bf16* s = abase + q * a_q + t * a_t;
      glds16(s, d);
      glds16(s + a_i, d + 8192);
    } else {
      const bf16* s = bbase + q * b_q + t * b_t;
      glds16(s, d);
      glds16(s + b_i, d + 8192);
    }
  };
  auto issued = [&](int Q) -> int {  // DMAs issued in phase Q
    if (Q < -6) return 0;
    const int tq = Q >= 0 ? Q >> 2 : -((3 - Q) >> 2);
    const int r = Q - 4 * tq;
    return tq + (r < 2 ? 1 : 2) < T ? 2 : 0;
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  for (int Q = -6; Q < 0; ++Q) issue(Q);
  wait_vm(issued(-4) + issued(-3) + issued(-2) + issued(-1));
  barrier();
  if (wr == 1) barrier();

  // fragment bases: row (16 blk + (lane & 15)) of an image, chunk (4 ks + (lane >> 4)) ^ hswz(row)
  const int frow = lane & 15;
  const int fb0 = frow * 128 + 16 * ((lane >> 4) ^ hswz(frow));
  const int fb1 = frow * 128 + 16 * ((4 + (lane >> 4)) ^ hswz(frow));
  const int fg = lane >> 4, fl = lane & 15;
  // rb: the block's first image row (K-contiguous operand) / image column (token-major operand)
  auto frag_kc = [&](const char* img, int rb, int ks) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(img + rb * 128 + (ks ? fb1 : fb0));
  };
  auto frag_tm = [&](const char* img, int rb, int ks) -> bf16x8 {
    const int r0 = 32 * ks + 8 * fg;
    const bf16x4 lo = tt_read(img, r0, rb, fl), hi = tt_read(img, r0 + 4, rb, fl);
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto afragh = [&](const char* img, int rb, int ks) -> bf16x8 {
    if constexpr (AT) return frag_tm(img, rb, ks); else return frag_kc(img, rb, ks);
  };
  auto bfragh = [&](const char* img, int rb, int ks) -> bf16x8 {
    if constexpr (BT) return frag_tm(img, rb, ks); else return frag_kc(img, rb, ks);
  };
  bf16x8 af[2][4], b0[2][2], b1[2][2];
  auto compute = [&](int qm, int qn, bf16x8 (&bq)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[qm * 4 + i][qn * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks][j], af[ks][i], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  for (int t = 0; t < T; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const int P = 4 * t;
    // phase 0: quadrant (0, 0), reads A_0 and B_0
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 2; ++j) b0[ks][j] = bfragh(buf + 2 * HT, wc * 32 + 16 * j, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = afragh(buf, wr * 64 + 16 * i, ks);
    }
    issue(P);
    wait_vm(issued(P - 3) + issued(P - 2) + issued(P - 1) + issued(P));
    barrier();
    compute(0, 0, b0);
    barrier();
    // phase 1: quadrant (0, 1), reads B_1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 2; ++j) b1[ks][j] = bfragh(buf + 3 * HT, wc * 32 + 16 * j, ks);
    issue(P + 1);
    wait_vm(issued(P - 2) + issued(P - 1) + issued(P) + issued(P + 1));
    barrier();
    compute(0, 1, b1);
    barrier();
    // phase 2: quadrant (1, 1), reads A_1
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = afragh(buf + HT, wr * 64 + 16 * i, ks);
    issue(P + 2);
    wait_vm(issued(P - 1) + issued(P) + issued(P + 1) + issued(P + 2));
    barrier();
    compute(1, 1, b1);
    barrier();
    // phase 3: quadrant (1, 0), registers only
    issue(P + 3);
    wait_vm(issued(P) + issued(P + 1) + issued(P + 2) + issued(P + 3));
    barrier();
    compute(1, 0, b0);
    barrier();
  }
  if (wr == 0) barrier();

  const int g = lane >> 4, l16 = lane & 15;
  bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(m0 + wr * 128 + l16) * p.ldc + n0 + wc * 64 + 4 * g;
  auto store_row = [&](int i, bool accumulate) {
    bf16* crow = cbase + (int64_t)16 * i * p.ldc;
    bf16x4 old[4];
    if (accumulate) {
#pragma unroll
      for (int j = 0; j < 4; ++j) old[j] = *reinterpret_cast<const bf16x4*>(crow + 16 * j);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
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

// ---------------------------------------------------------------------------------------------
// Variant 4: FOUR waves (one per SIMD), 128 x 128 outputs per wave (8 x 8 accumulators = 256
// AGPRs), software-pipelined inside the wave instead of ping-ponged across barriers: while the 64
// MFMAs of slot s run, the wave reads the fragments of slot s+1 (B into a second register set, each
// A block in place right after its last MFMA) and issues the LDS-DMA of slot s+R-1 through a
// buffer resource (32-bit per-lane offsets, everything else scalar); one workgroup barrier per
// 32-deep slot. Per MFMA this reads half the LDS bytes of the 128 x 64 wave tile.
__device__ __forceinline__ void bdma16(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc, uint32_t soff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds), "s"(soff) : "memory");
}

// MFMA with the accumulator pinned to AGPRs ("+a"): hipcc's allocator otherwise shuffles the 256
// loop-carried accumulators between AGPRs and VGPRs every slot (ROCm 7.2). hipcc does not model
// the asm: every accumulator is next touched >= 64 MFMAs later in the loop, and the epilogue pads
// the MFMA -> v_accvgpr_read hazard itself (s_nop after the loop).
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// lean LDS-DMA: M0 set in the same statement and declared clobbered (nothing else in these kernels
// uses M0), no save / restore: 2 scalar instructions per DMA instead of 4
__device__ __forceinline__ void bdma16_lean(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc, uint32_t soff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :: "v"(voff), "s"(rsrc), "s"(lds), "s"(soff) : "memory", "m0");
}

template <int R, bool PRIO, bool LEAN = false>
__global__ __launch_bounds__(256, 1) void gemm_nt_w4_kernel(const GemmParams p) {
  static_assert(R >= 4 && R * SLOTB <= 163840, "ring");
  __shared__ __attribute__((aligned(16))) char smem[R * SLOTB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nM = p.M / GT, nN = p.N / GT, nwg = nM * nN;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int per_group = kGroupRows * nN;
  const int grp = wg / per_group, first = grp * kGroupRows;
  const int gsize = min(nM - first, kGroupRows);
  const int tm = first + (wg % per_group) % gsize, tn = (wg % per_group) / gsize;
  GRT_DEVICE_CHECK(tm < nM && tn < nN);
  const int m0 = tm * GT, n0 = tn * GT;
  const int S = p.K / GS;

  // DMA: wave w, instruction i (0..3) of an operand fills image rows 64 i + 16 w + (lane >> 2),
  // chunk lane & 3, from source chunk (lane & 3) ^ kc_swz(row); byte offsets fit 32 bits (host check)
  const int drow = 16 * w + (lane >> 2);
  const int dch = (lane & 3) ^ kc_swz(lane >> 2);
  // descriptors from kernel arguments and constants only, so they stay in SGPRs (the asm's "s"
  // operand); every offset is in range by construction (host check: operands below 4 GiB)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), 0, 0xffffffffu, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.b), 0, 0xffffffffu, 0x00020000);
  const uint32_t avoff = (uint32_t)(((int64_t)(m0 + drow) * p.lda + 8 * dch) * 2);
  const uint32_t bvoff = (uint32_t)(((int64_t)(n0 + drow) * p.ldb + 8 * dch) * 2);
  const uint32_t astep = (uint32_t)(64 * p.lda * 2), bstep = (uint32_t)(64 * p.ldb * 2);
  const uint32_t lds0 = lds_addr(smem) + w * 1024;
  auto dma = [&](int j, int k) {  // k-th (0..7) DMA instruction of slot j (buffer j % R): 0-3 A, 4-7 B
    const int js = min(j, S - 1);
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + (j % R) * SLOTB + (k >> 2) * OPB + (k & 3) * 4096);
    if (k < 4) bdma16(avoff, ra, (k & 3) * astep + js * (GS * 2), d);
    else bdma16(bvoff, rb, (k & 3) * bstep + js * (GS * 2), d);
  };

  const int frow = lane & 15;
  const int fo = frow * 64 + 16 * ((lane >> 4) ^ kc_swz(frow));
  auto afrag = [&](int j, int mi) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + (j % R) * SLOTB + (wr * 128 + 16 * mi) * 64 + fo);
  };
  auto bfrag = [&](int j, int nj) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(smem + (j % R) * SLOTB + OPB + (wc * 128 + 16 * nj) * 64 + fo);
  };
  auto wait_pending = [&](int n) {
    if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};

  // ---- prologue: slots 0 .. R-2 in flight; fragments of slot 0 in registers; slot 1 visible
  for (int j = 0; j < R - 1; ++j)
    for (int k = 0; k < 8; ++k) dma(j, k);  // past S: a re-fetch of slot S-1
  wait_pending(8 * (R - 2));
  barrier();
  bf16x8 a[8], b0[8], b1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { b0[i] = bfrag(0, i); a[i] = afrag(0, i); }
  wait_pending(8 * (R - 3));
  barrier();

  // ---- one slot: MFMAs on (a, bc); slot s+1's B fragments into bn and each A block reloaded in
  // place after its row of MFMAs; DMA of slot s+R-1 (one instruction per row). Top-of-slot
  // invariant (barrier B_s): slot s+1 landed and visible, buffer (s-1) % R free (its fragments were
  // read during slot s-2 and consumed by slot s-1's MFMAs, all before B_s). Loads past the last
  // slot read in-bounds stale LDS and are never used.
  // Past the last slot the DMA re-fetches slot S-1 into buffer (s+R-1) % R, which is free (slot s-1
  // is consumed) and never read again: no branch in the loop, and every slot issues exactly 8 DMAs,
  // so the counted wait is a constant vmcnt(8 (R-3)).
  auto slot = [&](int s, bf16x8 (&bc)[8], bf16x8 (&bn)[8]) {
    const int jd = s + R - 1;
    const int jsrc = min(jd, S - 1);
    const uint32_t dbuf = (uint32_t)((jd % R) * SLOTB);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      // next slot's B blocks early (rows 0-3), so its first row never waits on them
      if (i < 4) { bn[2 * i] = bfrag(s + 1, 2 * i); bn[2 * i + 1] = bfrag(s + 1, 2 * i + 1); }
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        mfma_acc(acc[i][j], bc[j], a[i]);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      a[i] = afrag(s + 1, i);
      {
        const uint32_t d = __builtin_amdgcn_readfirstlane(lds0 + dbuf + (i >> 2) * OPB + (i & 3) * 4096);
        if constexpr (LEAN) {
          if (i < 4) bdma16_lean(avoff, ra, (i & 3) * astep + jsrc * (GS * 2), d);
          else bdma16_lean(bvoff, rb, (i & 3) * bstep + jsrc * (GS * 2), d);
        } else {
          if (i < 4) bdma16(avoff, ra, (i & 3) * astep + jsrc * (GS * 2), d);
          else bdma16(bvoff, rb, (i & 3) * bstep + jsrc * (GS * 2), d);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // slot s+2 must be landed before B_{s+1}; the R-3 younger slots may stay in flight
    if constexpr (R == 5) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (R == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
  };
  int s = 0;
  for (; s + 1 < S; s += 2) {
    slot(s, b0, b1);
    slot(s + 1, b1, b0);
  }
  if (s < S) slot(s, b0, b1);

  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA writes -> accvgpr reads
  // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + wr*128 + 16 i + (lane & 15),
  // n = n0 + wc*128 + 16 j + 4 (lane >> 4)
  const int g = lane >> 4, l16 = lane & 15;
  bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(m0 + wr * 128 + l16) * p.ldc + n0 + wc * 128 + 4 * g;
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

void gemm_tt2(const GemmParams& p, hipStream_t stream) {
  const int nwg = (p.M / GT) * (p.N / GT);
  hipLaunchKernelGGL((gemm_h_kernel<GEMM_EPI_STORE, true, true>), dim3(nwg), dim3(GNT), 0, stream, p);
}

void gemm_nn(const GemmParams& p, hipStream_t stream) {
  const int nwg = (p.M / GT) * (p.N / GT);
  hipLaunchKernelGGL((gemm_h_kernel<GEMM_EPI_STORE, false, true>), dim3(nwg), dim3(GNT), 0, stream, p);
}

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && K > 0 && M % GT == 0 && N % GT == 0 && K % GS == 0 && M <= INT32_MAX &&
         N <= INT32_MAX && K <= INT32_MAX && (M / GT) * (N / GT) <= INT32_MAX;
}

void gemm_nt(const GemmParams& p, hipStream_t stream) {
  const int nwg = (p.M / GT) * (p.N / GT);
  const dim3 grid(nwg), block(GNT);
  const int variant = p.variant;
  if (variant >= 9 && variant <= 16 && gemm_nt_k64_supported(p.M, p.N, p.K, p.lda, p.ldb)) {
    gemm_nt_k64(p, stream);
  } else if (variant == 4 || variant == 5) {
    if (variant == 4) hipLaunchKernelGGL((gemm_nt_w4_kernel<4, true>), grid, dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((gemm_nt_w4_kernel<5, true>), grid, dim3(256), 0, stream, p);
  } else if (variant == 6) {
    hipLaunchKernelGGL((gemm_nt_w4_kernel<5, false>), grid, dim3(256), 0, stream, p);
  } else if (variant == 7) {
    hipLaunchKernelGGL((gemm_nt_w4_kernel<4, false, true>), grid, dim3(256), 0, stream, p);
  } else if (variant == 8) {
    hipLaunchKernelGGL((gemm_nt_w4_kernel<5, false, true>), grid, dim3(256), 0, stream, p);
  } else if (variant == 3) {
    if (p.K % 64 == 0) hipLaunchKernelGGL((gemm_h_kernel<GEMM_EPI_STORE, false, false>), grid, block, 0, stream, p);
  } else if (variant == 1) hipLaunchKernelGGL((gemm_nt_kernel<GEMM_EPI_STORE, 1, 5>), grid, block, 0, stream, p);
  else if (variant == 2) hipLaunchKernelGGL((gemm_nt_kernel<GEMM_EPI_STORE, 1, 4>), grid, block, 0, stream, p);
  else hipLaunchKernelGGL((gemm_nt_kernel<GEMM_EPI_STORE, 2, 4>), grid, block, 0, stream, p);
}

}  // namespace grt
