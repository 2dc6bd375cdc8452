// Weight-gradient GEMM for gfx950:  C[P][Q] (+)= sum_r X[r][p] * Y[r][q]   (bf16 in, fp32 acc)
//
// Role: dW = dY^T · X of every Linear layer (reference: the cuBLAS wgrad GEMMs of
// nn.Linear backward inside loss.backward(), ray-jobs/pytorch_llm_ray.py:276 and the HF Llama
// projections under SFTTrainer.train(), ray-jobs/fine_tune_llama_ray.py:333).
// Both operands are stored token-major ([R][P] and [R][Q], row-major), i.e. the reduction index is
// the STRIDED one for both — the layout hipBLASLt handles worst (profiles/: ~1.05 PF on the
// Llama-2-7B wgrad shapes vs ~1.35 PF for the forward layout).
//
// Design (cdna_hip_programming.md §5 / T10):
//   * 256 x 256 output tile per workgroup, 8 waves as 2 (P) x 4 (Q), 128 x 64 outputs per wave as
//     8 x 4 v_mfma_f32_16x16x32_bf16 accumulators;
//   * reduction step 64 tokens; each stage is four 16 KiB LDS half-images [64 r][128 cols]
//     (X cols 0-127, 128-255, Y cols 0-127, 128-255), filled by global_load_lds_dwordx4 (LDS-DMA,
//     no VGPR round trip) with the XOR chunk swizzle applied to the per-lane SOURCE address so the
//     lane-linear DMA lands in the swizzled image (rule 21);
//   * MFMA operands come from ds_read_b64_tr_b16 transposed reads of those images (the reduction
//     index is the image row), conflict-free under the same XOR image (T10 (b));
//   * two stages in LDS (128 KiB): stage t+2 is issued right after stage t is consumed, and the
//     wait for stage t+1 is a counted vmcnt(8) — one stage's DMA is always in flight across the
//     raw s_barrier (never __syncthreads(), whose fence would drain it);
//   * output lanes hold 4 consecutive Q columns (the MFMA's A side is Y), so C is written (and, for
//     gradient accumulation, read) as 8-byte vectors; beta = 1 adds into C in fp32;
//   * blockIdx -> tile: bijective XCD remap, then grouped order (8 tile rows per group) so the
//     ~32 workgroups resident on one XCD share X/Y panels in that XCD's L2.
// Measured alternatives (tools/gemm_ab.py, interleaved medians; profiles/r1_gemm_wgrad_ab.md): one barrier
// per half-step with fragment prefetch across it beat (a) a 2-barrier 64-token stage (-10..15 %),
// (b) the DMA issued as a burst after the barrier instead of one instruction per 8 MFMAs, (c) a
// ping-pong schedule of the two wave rows with a barrier per phase (-15 %), and (d) 4 waves with a
// 128 x 128 block each (-17 %).
// Requirements (checked on the host): P % 256 == 0, Q % 256 == 0, R % 64 == 0, 16-byte aligned
// rows (ld % 8 == 0).
#include "grt_common.h"
#include "grt_kernels.h"

#include <type_traits>

namespace grt {
namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int TP = 256, TQ = 256, TR = 32, GNT = 512;
constexpr int kImg = TR * 256;           // one image: 32 rows x 256 bytes = 8 KiB
constexpr int kSlot = 4 * kImg;          // one half-step: 32 KiB
constexpr int kSlots = 4;
constexpr int kGroupRows = 8;

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_off(int row, int ch) { return row * 256 + 16 * (ch ^ swz(row)); }

// 16-lane group reads rows r0..r0+3, columns c0..c0+15; lane i gets column c0 + i.
__device__ __forceinline__ bf16x4 tr_read(const char* base, int r0, int c0, int l16) {
  const int q = l16 >> 2, col = c0 + 4 * (l16 & 3);
  const char* a = base + img_off(r0 + q, col >> 3) + 8 * ((col >> 2) & 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
// LDS-DMA of 16 bytes per lane to (wave-uniform LDS byte address) + lane * 16. Issued as inline asm
// so hipcc does not track it: its waitcnt pass would otherwise put vmcnt(0) in front of every LDS
// read of the loop (it cannot prove the reads miss the in-flight DMA) and serialise the pipeline.
// The kernel counts vmcnt itself.
__device__ __forceinline__ void glds16(const void* gptr, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gptr), "s"(lds_addr) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// MFMA operand: lane (g, l16) gets column c0 + l16, reduction rows rb + 8g .. rb + 8g + 7
__device__ __forceinline__ bf16x8 frag(const char* img, int rb, int c0, int g, int l16) {
  return cat(tr_read(img, rb + 8 * g, c0, l16), tr_read(img, rb + 8 * g + 4, c0, l16));
}

// NSLOT: 32 KiB LDS slots in the ring (4 or 5).
// DIAG (timing experiments only, results are wrong): 1 = L2-hot DMA source, 2 = no DMA / no barrier.
template <int NSLOT, int DIAG>
__global__ __launch_bounds__(GNT, 1) void gemm_tt_kernel(const GemmTTParams p) {
  __shared__ __attribute__((aligned(16))) char smem[NSLOT * kSlot];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int wr = w >> 2, wc = w & 3;

  // ---- tile coordinates: bijective XCD remap, then grouped order
  const int nP = p.P / TP, nQ = p.Q / TQ, nwg = nP * nQ;
  const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int per_group = kGroupRows * nQ;
  const int grp = wg / per_group, first = grp * kGroupRows;
  const int gsize = min(nP - first, kGroupRows);
  const int tp = first + (wg % per_group) % gsize, tq = (wg % per_group) / gsize;
  GRT_DEVICE_CHECK(tp < nP && tq < nQ && wg < nwg);
  const int p0 = tp * TP, q0 = tq * TQ;

  // ---- LDS ring: NSLOT slots x 32 KiB; slot k holds one 32-token half-step of four 128-column
  // images (X cols 0-127, X 128-255, Y 0-127, Y 128-255), each [32 rows][256 B], XOR-swizzled.
  // Half-step h (tokens 32h .. 32h+31) lives in slot h % NSLOT. A thread DMAs image row 4w + g; the
  // swizzle depends only on that row, so one source pointer per operand serves both halves (+256 B).
  const int row0 = 4 * w + g;
  const int ch = l16 ^ swz(row0);
  const char* xsrc = reinterpret_cast<const char*>(static_cast<const bf16*>(p.x) + (int64_t)row0 * p.ldx + p0 + 8 * ch);
  const char* ysrc = reinterpret_cast<const char*>(static_cast<const bf16*>(p.y) + (int64_t)row0 * p.ldy + q0 + 8 * ch);
  const int64_t xstep = (int64_t)32 * p.ldx * 2, ystep = (int64_t)32 * p.ldy * 2;
  const uint32_t ldsw = lds_addr(smem) + w * 1024;
  // DMA addresses of half-step h; instruction k (compile-time) of 4: 0/1 = X halves, 2/3 = Y halves
  struct Dma { const char* xs; const char* ys; uint32_t d; };
  auto dma_at = [&](int h) -> Dma {
    return Dma{DIAG == 1 ? xsrc : xsrc + h * xstep, DIAG == 1 ? ysrc : ysrc + h * ystep,
               (uint32_t)__builtin_amdgcn_readfirstlane(ldsw + (h % NSLOT) * kSlot)};
  };
  auto dma = [&](const Dma& a, int k) { glds16(((k & 2) ? a.ys : a.xs) + (k & 1) * 256, a.d + k * kImg); };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

  // ---- main loop, one barrier per half-step. Barrier B_s (top of iteration s) follows the counted
  // wait that retires the DMA of half-step s+1, so after it half-step s+1 is readable: its MFMA
  // fragments are prefetched into registers WHILE half-step s is computed (each X fragment is
  // reloaded right after its last MFMA), and the first MFMAs after the barrier never wait on LDS.
  // B_s also proves every wave has left iteration s-1, so slot (s-1) % NSLOT (last read during
  // iteration s-2) is refilled with half-step s+NSLOT-1, one DMA instruction per 8 MFMAs.
  constexpr int AHEAD = NSLOT - 1;
  const int S = p.R / 32;
  for (int h = 0; h < AHEAD && h < S; ++h) {
    const Dma a = dma_at(h);
#pragma unroll
    for (int k = 0; k < 4; ++k) dma(a, k);
  }
  const int qc = (wc & 1) * 64;
  auto yfrag = [&](int h, int j) {
    return frag(smem + (h % NSLOT) * kSlot + (2 + (wc >> 1)) * kImg, 0, qc + 16 * j, g, l16);
  };
  auto xfrag = [&](int h, int i) { return frag(smem + (h % NSLOT) * kSlot + wr * kImg, 0, 16 * i, g, l16); };
  // prologue: half-step 0 published, fragments of 0 in registers
  {
    const int pending = DIAG == 2 ? 0 : min(S, AHEAD) - 1;  // half-step 0 landed
    if (pending >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (pending == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (pending == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  bf16x8 yf[4], xf[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) yf[j] = yfrag(0, j);
#pragma unroll
  for (int i = 0; i < 8; ++i) xf[i] = xfrag(0, i);

  // one half-step; MORE / REFILL are compile-time so the MFMA stream carries no branches
  auto body = [&](int s, auto more_c, auto refill_c) {
    constexpr bool MORE = decltype(more_c)::value;
    constexpr bool REFILL = decltype(refill_c)::value && DIAG != 2;
    if (DIAG != 2) {
      // in flight after the wait: half-steps s+2 .. min(S, s+AHEAD)-1
      const int pending = REFILL ? AHEAD - 2 : min(S, s + AHEAD) - (s + 2);
      if (pending >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else if (pending == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if (pending == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const Dma an = dma_at(s + AHEAD);
    bf16x8 yn[4];
    if constexpr (MORE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) yn[j] = yfrag(s + 1, j);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[j], xf[i], acc[i][j], 0, 0, 0);
      if constexpr (MORE) xf[i] = xfrag(s + 1, i);
      if constexpr (REFILL) {
        if (i & 1) {
          __builtin_amdgcn_sched_barrier(0);
          dma(an, i >> 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    if constexpr (MORE) {
#pragma unroll
      for (int j = 0; j < 4; ++j) yf[j] = yn[j];
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int s = 0;
  for (; s + AHEAD < S; ++s) body(s, T_{}, T_{});
  for (; s + 1 < S; ++s) body(s, T_{}, F_{});
  body(s, F_{}, F_{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // ---- epilogue: lane holds C[p][q .. q+3]; the beta branch is hoisted out of the element loop
  bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(p0 + wr * 128 + l16) * p.ldc + q0 + wc * 64 + 4 * g;
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

}  // namespace

bool gemm_tt_supported(int P, int Q, int R) { return P % TP == 0 && Q % TQ == 0 && R % 64 == 0 && R > 0; }


void gemm_tt(const GemmTTParams& p, hipStream_t stream, int mode) {
  const int nwg = (p.P / TP) * (p.Q / TQ);
  const dim3 grid(nwg), block(GNT);
  if (mode == 1) hipLaunchKernelGGL((gemm_tt_kernel<5, 1>), grid, block, 0, stream, p);       // diag: L2-hot
  else if (mode == 2) hipLaunchKernelGGL((gemm_tt_kernel<5, 2>), grid, block, 0, stream, p);  // diag: no DMA
  else hipLaunchKernelGGL((gemm_tt_kernel<5, 0>), grid, block, 0, stream, p);
}

}  // namespace grt
