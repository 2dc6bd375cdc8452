// LoRA adapter kernels for gfx950: the input-dropout + down-projection and the adapter's
// input-gradient accumulation, each ONE pass over the [tokens, in] activation.
//
// Reference role: PEFT's LoRA layer on every targeted projection of the QLoRA SFT job
// (LoraConfig r=64, alpha=16, dropout=0.1 on q,k,v,o,gate,up,down; reference
// ray-jobs/fine_tune_llama_ray.py:243-254, fine_tune_config.json:6-8,30-33):
//     y = base(x) + s * B (A dropout(x)).
// Without these kernels the adapter costs, per adapted input and step, a dropout pass
// (read x, write x_d), a rank-R GEMM over x_d, and in the backward a [tokens, in] GEMM
// g·A written to a temporary plus a dropout-backward pass reading it and read-modify-writing dX —
// ~5 full passes over a [tokens, in] tensor around two skinny GEMMs the library tiles poorly.
//
//   lora_down:  h[M][R] = (x ⊙ keep / (1-p)) · A^T, A = [R][K] (the concatenated A of all
//               targets); the dropout keep-mask is the element-dropout hash of x's element index
//               (grt_common.h drop_keep, the same mask dropout_fwd/bwd_seeded use), applied in
//               registers; x_d is optionally written as a side output (the dA GEMM reads it).
//   lora_dx:    dX[M][K] (+)= keep / (1-p) ⊙ (g[M][R] · A[R][K]) from A^T = [K][R] — one
//               read-modify-write of dX, no [M][K] temporary.
// v_mfma_f32_32x32x16_bf16 throughout. Every global access is a full-row coalesced 16 B/lane load
// or store; MFMA fragments are read from padded LDS images (a first version loaded the fragments
// straight from global memory — 32 rows x 32 B per instruction, address-unit bound, 2-4x slower:
// profiles/r2_perf_experiments.md).
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// (accumulator element r of lane half h holds row 8 (r / 4) + 4 h + r % 4 of the 32-row tile)

// keep flags of 8 consecutive elements starting at a 4-aligned element index
__device__ __forceinline__ void keep8(uint64_t key, uint64_t idx0, uint32_t thr, bool (&kp)[8]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint64_t hv = hash_u64(key ^ ((idx0 >> 2) + q));
#pragma unroll
    for (int j = 0; j < 4; ++j) kp[4 * q + j] = ((uint32_t)(hv >> (16 * j)) & 0xffffu) >= thr;
  }
}

// ---- lora_down: 32 tokens per workgroup, K streamed in 128-column chunks. x: each thread loads 32 B
// of one row per chunk (8 threads cover a row's 256 B: coalesced), LD_PF chunks in flight in a
// register ring; the mask is applied in registers, x_d is stored from them (coalesced 16 B stores).
// A's [R][128] chunk is loaded coalesced one chunk ahead in registers. Both go to double-buffered
// LDS images (one barrier per chunk) from which each wave feeds two 16-wide k-steps of MFMAs
// D[R row][token] = A · x_d^T. (MFMA fragments straight from global memory touch 32 rows x 32 B
// per instruction — address-unit bound; the LDS images make every global access a full row.)
constexpr int LD_PF = 4;            // x chunks in flight per thread

__device__ __forceinline__ void drop8(bf16x8& v, uint64_t key, uint64_t idx0, uint32_t thr, float sc) {
  bool kp[8];
  keep8(key, idx0, thr, kp);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = static_cast<bf16>(kp[e] ? static_cast<float>(v[e]) * sc : 0.f);
}

template <int RB, int KC, int TB>
constexpr int lora_down_lds_bytes() {  // x images + A images; the final reduction reuses the space
  return (2 * 32 * TB * (KC + 8) * 2 + 2 * 32 * RB * (KC + 8) * 2) > (4 - TB) * RB * 16 * 64 * 4
             ? (2 * 32 * TB * (KC + 8) * 2 + 2 * 32 * RB * (KC + 8) * 2) : (4 - TB) * RB * 16 * 64 * 4;
}

// KC: K chunk (128, or 64 for half the LDS: two workgroups per CU at R = 192).
// TB: 32-token tiles per workgroup. The kernel is bound by the A chunk loads from L2 (one [R][KC]
// chunk per workgroup per chunk: R / 32 times the x bytes at TB = 1; profiles/r2_perf_experiments.md),
// so TB = 2 halves them per x byte: wave w takes token tile w % TB and k-slice w / TB of each chunk.
template <int RB, int KC, int TB, int AD = 1>  // R = 32 * RB
__global__ __launch_bounds__(256) void lora_down_kernel(const LoraDownParams P) {
  constexpr int R = 32 * RB;
  constexpr int XS = KC + 8;         // LDS row (bf16): +16 B so b128 fragment reads of 32 rows spread over banks
  constexpr int AIMG = R * XS;       // elements per A image
  constexpr int XIMG = 32 * TB * XS;  // elements per x image
  constexpr int NV = KC / 64;        // 16 B x vectors per thread per chunk and token tile (32 rows x KC / 256 threads / 8)
  constexpr int TPA = KC / 8;        // A loader threads per row
  constexpr int NA = R * TPA / 256;  // A vectors per thread per chunk
  constexpr int NSL = 4 / TB;        // k-slices per chunk (waves per token tile)
  constexpr int KSW = KC / 16 / NSL;  // 16-wide k-steps per wave per chunk
  __shared__ __attribute__((aligned(16))) char smem[lora_down_lds_bytes<RB, KC, TB>()];
  bf16* xs = reinterpret_cast<bf16*>(smem);                  // [2][32 TB][XS]
  bf16* as = reinterpret_cast<bf16*>(smem + 2 * XIMG * 2);   // [2][R][XS]
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tt = w % TB, ksl = w / TB;  // this wave's token tile and k-slice
  // split-K: blockIdx = split * (token blocks) + token block; this workgroup reduces K chunks
  // [c_lo, c_lo + nch) and writes an fp32 partial when the K range is split (lora_hsum adds them)
  const int ntb = (int)((P.M + 32 * TB - 1) / (32 * TB));
  const int tb = blockIdx.x % ntb, ksi = blockIdx.x / ntb;
  const int nch_all = P.K / KC;
  const int c_lo = ksi * nch_all / P.ksplit;
  const int nch = (ksi + 1) * nch_all / P.ksplit - c_lo;
  const int64_t t0 = (int64_t)tb * 32 * TB;
  const int lr = tid >> 3, lc = (tid & 7) * 8 * NV;  // x loader: rows lr + 32 u (u < TB), first of 8 NV columns
  const bf16* src[TB];
  bf16* xdst[TB];
  uint64_t eidx[TB];  // of this thread's first x element in each of its rows
#pragma unroll
  for (int u = 0; u < TB; ++u) {
    const int64_t ltok = t0 + lr + 32 * u;
    const bool lok = ltok < P.M;
    src[u] = static_cast<const bf16*>(P.x) + (lok ? ltok : P.M - 1) * (int64_t)P.ldx + c_lo * KC + lc;
    xdst[u] = (P.xd != nullptr && lok) ? static_cast<bf16*>(P.xd) + ltok * (int64_t)P.K + c_lo * KC + lc : nullptr;
    eidx[u] = P.offset + (uint64_t)ltok * (uint64_t)P.K + c_lo * KC + lc;
  }
  const int ar = tid / TPA, ac = (tid % TPA) * 8;  // A loader: rows ar + (256 / TPA) j, 8 columns from ac
  const bf16* asrc = static_cast<const bf16*>(P.a) + (int64_t)ar * P.K + c_lo * KC + ac;
  const bool drop = P.p > 0.f;
  const uint32_t thr = drop_thr(P.p);
  const float sc = drop ? 1.f / (1.f - P.p) : 1.f;
  const uint64_t key = hash_u64(P.seed);

  bf16x8 ring[LD_PF][TB][NV];
#pragma unroll
  for (int i = 0; i < LD_PF; ++i)
    if (i < nch) {
#pragma unroll
      for (int u = 0; u < TB; ++u)
#pragma unroll
        for (int v = 0; v < NV; ++v) ring[i][u][v] = *reinterpret_cast<const bf16x8*>(src[u] + i * KC + 8 * v);
    }
  // A chunks AD ahead in registers (GRT_LORA_DOWN_AD selects 1 or 2 at launch: template AD)
  bf16x8 areg[AD][NA];
#pragma unroll
  for (int d = 0; d < AD; ++d)
    if (d < nch) {
#pragma unroll
      for (int j = 0; j < NA; ++j)
        areg[d][j] = *reinterpret_cast<const bf16x8*>(asrc + (int64_t)j * (256 / TPA) * P.K + d * KC);
    }
  f32x16 acc[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) acc[i] = f32x16{};
  for (int c0 = 0; c0 < nch; c0 += LD_PF) {
#pragma unroll
    for (int i = 0; i < LD_PF; ++i) {
      const int c = c0 + i;
      if (c < nch) {  // block-uniform
        bf16x8 xv[TB][NV];
#pragma unroll
        for (int u = 0; u < TB; ++u)
#pragma unroll
          for (int v = 0; v < NV; ++v) xv[u][v] = ring[i][u][v];
        if (c + LD_PF < nch) {
#pragma unroll
          for (int u = 0; u < TB; ++u)
#pragma unroll
            for (int v = 0; v < NV; ++v) ring[i][u][v] = *reinterpret_cast<const bf16x8*>(src[u] + (c + LD_PF) * KC + 8 * v);
        }
        // buffer c & 1 (c0 is a multiple of LD_PF); the previous reader of this buffer was chunk
        // c - 2, which every wave finished before the barrier of chunk c - 1
        bf16* xt = xs + (i & 1) * XIMG;
        bf16* at = as + (i & 1) * AIMG;
        constexpr int ad = AD;  // register set of chunk c: (c mod AD), c0 a multiple of LD_PF (a multiple of AD)
        bf16x8(&ar_c)[NA] = areg[i % ad];
#pragma unroll
        for (int j = 0; j < NA; ++j) *reinterpret_cast<bf16x8*>(at + (ar + (256 / TPA) * j) * XS + ac) = ar_c[j];
        if (c + ad < nch) {
#pragma unroll
          for (int j = 0; j < NA; ++j)
            ar_c[j] = *reinterpret_cast<const bf16x8*>(asrc + (int64_t)j * (256 / TPA) * P.K + (c + ad) * KC);
        }
#pragma unroll
        for (int u = 0; u < TB; ++u)
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            if (drop) drop8(xv[u][v], key, eidx[u] + (uint64_t)c * KC + 8 * v, thr, sc);
            if (xdst[u] != nullptr) *reinterpret_cast<bf16x8*>(xdst[u] + c * KC + 8 * v) = xv[u][v];
            *reinterpret_cast<bf16x8*>(xt + (lr + 32 * u) * XS + lc + 8 * v) = xv[u][v];
          }
        __syncthreads();
#pragma unroll
        for (int s2 = 0; s2 < KSW; ++s2) {
          const int kk = (KSW * ksl + s2) * 16 + 8 * h;
          const bf16x8 xf = *reinterpret_cast<const bf16x8*>(xt + (32 * tt + l32) * XS + kk);
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
            acc[rb] = mfma32x32x16(*reinterpret_cast<const bf16x8*>(at + (rb * 32 + l32) * XS + kk), xf, acc[rb]);
        }
      }
    }
  }
  // reduce the k-slices of each token tile: waves of slice > 0 -> LDS (over the images), the
  // slice-0 wave of the tile sums
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [TB][NSL - 1][RB * 16 * 64]
  if (ksl > 0) {
    float* dst = red + (tt * (NSL - 1) + ksl - 1) * RB * 1024;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[(rb * 16 + r) * 64 + lane] = acc[rb][r];
  }
  __syncthreads();
  if (ksl > 0) return;
  const float* src_red = red + tt * (NSL - 1) * RB * 1024;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ix = (rb * 16 + r) * 64 + lane;
#pragma unroll
      for (int q = 0; q < NSL - 1; ++q) acc[rb][r] += src_red[q * RB * 1024 + ix];
    }
  const int64_t tok = t0 + 32 * tt + l32;
  if (tok < P.M && P.ksplit > 1) {
    float* prow = P.hpart + ((int64_t)ksi * P.M + tok) * R;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(prow + rb * 32 + 8 * q + 4 * h) =
            f32x4{acc[rb][4 * q], acc[rb][4 * q + 1], acc[rb][4 * q + 2], acc[rb][4 * q + 3]};
  } else if (tok < P.M) {
    bf16* hrow = static_cast<bf16*>(P.h) + tok * (P.ldh > 0 ? P.ldh : (int64_t)R);
    const float hs = P.hscale;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(acc[rb][4 * q + j] * hs);
        *reinterpret_cast<bf16x4*>(hrow + rb * 32 + 8 * q + 4 * h) = v;
      }
  }
}

// ---- lora_down, LDS-DMA form (default for R = 64 / 128 / 192). The register-staged kernel above
// moves every x and A chunk through VGPRs into LDS (ds_write_b128: ~79 B/clk per CU, the A chunk is
// R / 32 times the x chunk per 32 tokens); here both arrive by LDS-DMA (global_load_lds_dwordx4,
// 1 KiB per wave-instruction, XOR-swizzled 128-byte rows: conflict-free b128 fragment reads) into a
// 4-slot ring with a counted vmcnt across raw s_barriers (lora_grad.hip's pipeline). 64 tokens x
// 64 columns per chunk; wave w takes token tile w & 1 and k-steps 2 (w >> 1), +1 of each chunk.
// The dropout mask is applied to the x fragment in registers and x_d (XD) is stored from it.
constexpr int LDD_NS = 4;                      // ring slots
constexpr int LDD_KC = 64;                     // columns per chunk (128-byte rows)
__device__ __forceinline__ int swz128(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ void dma16_lds(const void* gptr, uint32_t lds_byte_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gptr), "s"(lds_byte_addr) : "memory", "m0");
}

template <int RB, bool XD>  // R = 32 RB
__global__ __launch_bounds__(256) void lora_down_dma_kernel(const LoraDownParams P) {
  constexpr int R = 32 * RB;
  constexpr int XIMG = 64 * 128, AIMG = R * 128, SLOT = XIMG + AIMG;
  constexpr int D = 2 + RB;        // DMA instructions per wave and chunk (2 x pieces + RB A pieces)
  constexpr int S = XD ? 2 : 0;    // x_d stores per wave and chunk
  __shared__ __attribute__((aligned(16))) char smem[LDD_NS * SLOT > 2 * RB * 16 * 64 * 4 ? LDD_NS * SLOT
                                                                                     : 2 * RB * 16 * 64 * 4];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tt = w & 1, ksl = w >> 1;
  const int ntb = (int)((P.M + 63) / 64);
  const int tb = blockIdx.x % ntb, ksi = blockIdx.x / ntb;
  const int nch_all = P.K / LDD_KC;
  const int c_lo = ksi * nch_all / P.ksplit;
  const int nch = (ksi + 1) * nch_all / P.ksplit - c_lo;
  const int64_t t0 = (int64_t)tb * 64;
  const bf16* X = static_cast<const bf16*>(P.x);
  const bf16* A = static_cast<const bf16*>(P.a);
  // DMA sources: lane l of a piece covers row (piece row 0) + (l >> 3), LDS position l & 7, source
  // chunk (l & 7) ^ swz(row). x: wave w fills rows 16 w .. 16 w + 15 (2 pieces); A: rows 8 RB w ..
  const int pr = lane >> 3, pp = lane & 7;
  const bf16* xsrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 16 * w + 8 * q + pr;
    const int64_t tok = min(t0 + r, P.M - 1);
    xsrc[q] = X + tok * (int64_t)P.ldx + (int64_t)c_lo * LDD_KC + 8 * (pp ^ swz128(r));
  }
  const bf16* asrc[RB];
#pragma unroll
  for (int q = 0; q < RB; ++q) {
    const int r = 8 * RB * w + 8 * q + pr;
    asrc[q] = A + (int64_t)r * P.K + (int64_t)c_lo * LDD_KC + 8 * (pp ^ swz128(r));
  }
  const uint32_t smem0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(smem);
  auto dma_chunk = [&](int c, int slot) __attribute__((always_inline)) {
    const uint32_t base = smem0 + (uint32_t)(slot * SLOT);
    const uint32_t dx = __builtin_amdgcn_readfirstlane(base + (uint32_t)(16 * w * 128));
    const uint32_t da = __builtin_amdgcn_readfirstlane(base + (uint32_t)(XIMG + 8 * RB * w * 128));
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16_lds(xsrc[q] + c * LDD_KC, dx + q * 1024);
#pragma unroll
    for (int q = 0; q < RB; ++q) dma16_lds(asrc[q] + c * LDD_KC, da + q * 1024);
  };
  // vmcnt: ops younger than chunk t's DMA are nd later chunks' DMAs and ns x_d store groups
  auto wait_chunk = [&](int nd, int ns) __attribute__((always_inline)) {
    switch (nd * 3 + ns) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(S) : "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * S) : "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D) : "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D + S) : "memory"); break;
      case 5: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D + 2 * S) : "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * D) : "memory"); break;
      case 7: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * D + S) : "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * D + 2 * S) : "memory"); break;
    }
  };
  const bool drop = P.p > 0.f;
  const uint32_t thr = drop_thr(P.p);
  const float sc = drop ? 1.f / (1.f - P.p) : 1.f;
  const uint64_t key = hash_u64(P.seed);
  const int64_t mytok = t0 + 32 * tt + l32;
  const bool tok_ok = mytok < P.M;
  // a lane past the last token reads row M-1 (clamped DMA source) and stores exactly what that row's
  // own lane stores (same mask index): every wave issues the same number of x_d stores, which the
  // counted vmcnt relies on
  const int64_t tokc = tok_ok ? mytok : P.M - 1;
  bf16* xdrow = XD ? static_cast<bf16*>(P.xd) + tokc * (int64_t)P.K + (int64_t)c_lo * LDD_KC : nullptr;
  const uint64_t eidx0 = P.offset + (uint64_t)tokc * (uint64_t)P.K + (uint64_t)c_lo * LDD_KC;

  f32x16 acc[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) acc[i] = f32x16{};
  const int pre = min(nch, LDD_NS - 1);
  for (int c = 0; c < pre; ++c) dma_chunk(c, c);
  for (int t = 0; t < nch; ++t) {
    const int slot = t % LDD_NS;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // this wave's reads of slot t-1 are done
    wait_chunk(min(2, nch - 1 - t), min(t, 2));             // chunk t landed (this wave's pieces)
    __builtin_amdgcn_s_barrier();                            // ... every wave's; slot t-1 free
    const char* xi = smem + slot * SLOT;
    const char* ai = xi + XIMG;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int ch = 2 * (2 * ksl + s2) + h;  // 16-byte chunk of this lane's 8 k (k = 16 kstep + 8 h)
      const int xr = 32 * tt + l32;
      bf16x8 xf = *reinterpret_cast<const bf16x8*>(xi + xr * 128 + 16 * (ch ^ swz128(xr)));
      if (drop) drop8(xf, key, eidx0 + (uint64_t)t * LDD_KC + 8 * ch, thr, sc);
      if (XD) *reinterpret_cast<bf16x8*>(xdrow + t * LDD_KC + 8 * ch) = xf;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const int ar = rb * 32 + l32;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ai + ar * 128 + 16 * (ch ^ swz128(ar)));
        acc[rb] = mfma32x32x16(af, xf, acc[rb]);
      }
    }
    if (t + LDD_NS - 1 < nch) dma_chunk(t + LDD_NS - 1, (t + LDD_NS - 1) % LDD_NS);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // ring consumed: the space takes the k-slice reduction
  float* red = reinterpret_cast<float*>(smem);  // [2 token tiles][RB * 16 * 64]
  if (ksl > 0) {
    float* dst = red + tt * RB * 1024;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[(rb * 16 + r) * 64 + lane] = acc[rb][r];
  }
  __syncthreads();
  if (ksl > 0) return;
  const float* src_red = red + tt * RB * 1024;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[rb][r] += src_red[(rb * 16 + r) * 64 + lane];
  if (tok_ok && P.ksplit > 1) {
    float* prow = P.hpart + ((int64_t)ksi * P.M + mytok) * R;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(prow + rb * 32 + 8 * q + 4 * h) =
            f32x4{acc[rb][4 * q], acc[rb][4 * q + 1], acc[rb][4 * q + 2], acc[rb][4 * q + 3]};
  } else if (tok_ok) {
    bf16* hrow = static_cast<bf16*>(P.h) + mytok * (P.ldh > 0 ? P.ldh : (int64_t)R);
    const float hs = P.hscale;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(acc[rb][4 * q + j] * hs);
        *reinterpret_cast<bf16x4*>(hrow + rb * 32 + 8 * q + 4 * h) = v;
      }
  }
}

// h[M][R] (row stride ldh) = bf16(hscale * sum over the ksplit fp32 partials)
__global__ __launch_bounds__(256) void lora_hsum_kernel(const float* __restrict__ part, bf16* __restrict__ h,
                                                        int64_t n4, int ksplit, int64_t stride, int R, int64_t ldh,
                                                        float hscale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    f32x4 a = *reinterpret_cast<const f32x4*>(part + 4 * i);
    for (int k = 1; k < ksplit; ++k) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(part + k * stride + 4 * i);
      a += b;
    }
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = static_cast<bf16>(a[j] * hscale);
    const int64_t e = 4 * i, row = e / R;
    *reinterpret_cast<bf16x4*>(h + row * ldh + (e - row * R)) = o;
  }
}

// ---- lora_dx: one workgroup = 64 tokens x 128 columns of dX. The dX tile's 16 B chunks are loaded
// first (coalesced, in flight during the rest); g [64][R] and A^T [128][R] are loaded with full-row
// coalesced loads into padded LDS images; each wave computes a 32-token x 64-column block
// D[k][token] = A^T · g^T over R from them, parks it in a padded fp32 LDS tile (over the images),
// and every thread then finishes four 8-column chunks: mask, scale, add, 16 B store.
constexpr int DX_TS = 132;  // fp32 tile row: 128 + 4 so the f32x4 writes of 32 rows spread over banks

// R > 128: the images hold a 64-wide slice of R at a time (a loop over the slices), so the
// workgroup's LDS stays at the fp32 tile's 33 KiB and 4 workgroups fit per CU (R = 192 at full
// width: 77 KiB, 2 per CU, ~2.8x the dX read-modify-write floor; profiles/r3_pmc_kernel_zoo.md).
template <int RS>
constexpr int lora_dx_slice() { return RS > 8 ? 64 : 16 * RS; }
template <int RS>
constexpr int lora_dx_lds_bytes() {
  return (192 * (lora_dx_slice<RS>() + 8) * 2) > (64 * DX_TS * 4) ? (192 * (lora_dx_slice<RS>() + 8) * 2)
                                                                    : (64 * DX_TS * 4);
}

template <int RS>  // R = 16 * RS
__global__ __launch_bounds__(256) void lora_dx_kernel(const LoraDxParams P) {
  constexpr int R = 16 * RS, SW = lora_dx_slice<RS>(), RP = SW + 8;  // slice width, padded image row (bf16)
  __shared__ __attribute__((aligned(16))) char smem[lora_dx_lds_bytes<RS>()];
  bf16* gimg = reinterpret_cast<bf16*>(smem);  // [64][RP]
  bf16* aimg = gimg + 64 * RP;                 // [128][RP]
  float* tile = reinterpret_cast<float*>(smem);  // [64][DX_TS], after the images are consumed
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkb = P.K / 128;
  const int64_t tb = blockIdx.x / nkb;
  const int kb = blockIdx.x % nkb;
  bf16* dx = static_cast<bf16*>(P.dx);
  const int64_t ldo = P.ld_out > 0 ? P.ld_out : (int64_t)P.K;
  const bf16* din = P.dx_in != nullptr ? static_cast<const bf16*>(P.dx_in) : dx;
  const int64_t ldi = P.dx_in != nullptr ? P.ld_in : ldo;
  const int64_t ldg = P.ldg > 0 ? P.ldg : (int64_t)R;
  bf16x8 old[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 4, col = (c & 15) * 8;
    const int64_t tok = tb * 64 + row;
    old[i] = bf16x8{};
    if (P.accumulate && tok < P.M) old[i] = *reinterpret_cast<const bf16x8*>(din + tok * ldi + kb * 128 + col);
  }
  // images: SW / 8 chunks of 16 B per row
  constexpr int CPR = SW / 8;
  const bf16* g = static_cast<const bf16*>(P.g);
  const bf16* at = static_cast<const bf16*>(P.at) + (int64_t)kb * 128 * R;
  const int tl = (w & 1) * 32 + l32;  // this lane's token row within the tile (MFMA B operand)
  f32x16 acc[2];
  acc[0] = f32x16{};
  acc[1] = f32x16{};
  for (int r0 = 0; r0 < R; r0 += SW) {
    if (r0 > 0) __syncthreads();  // every wave is done with the previous slice's images
#pragma unroll
    for (int c = tid; c < 64 * CPR; c += 256) {
      const int row = c / CPR, col = (c % CPR) * 8;
      const int64_t tok = tb * 64 + row;
      *reinterpret_cast<bf16x8*>(gimg + row * RP + col) =
          *reinterpret_cast<const bf16x8*>(g + (tok < P.M ? tok : P.M - 1) * ldg + r0 + col);
    }
#pragma unroll
    for (int c = tid; c < 128 * CPR; c += 256) {
      const int row = c / CPR, col = (c % CPR) * 8;
      *reinterpret_cast<bf16x8*>(aimg + row * RP + col) = *reinterpret_cast<const bf16x8*>(at + (int64_t)row * R + r0 + col);
    }
    __syncthreads();
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      const int kl = (w >> 1) * 64 + cb * 32;  // column block within the tile
#pragma unroll
      for (int s = 0; s < SW / 16; ++s)
        acc[cb] = mfma32x32x16(*reinterpret_cast<const bf16x8*>(aimg + (kl + l32) * RP + 16 * s + 8 * h),
                               *reinterpret_cast<const bf16x8*>(gimg + tl * RP + 16 * s + 8 * h), acc[cb]);  // D[k][token]
    }
  }
  __syncthreads();  // images consumed; the fp32 tile reuses the space
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int kl = (w >> 1) * 64 + cb * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<f32x4*>(&tile[tl * DX_TS + kl + 8 * q + 4 * h]) =
          f32x4{acc[cb][4 * q], acc[cb][4 * q + 1], acc[cb][4 * q + 2], acc[cb][4 * q + 3]};
  }
  __syncthreads();
  const bool drop = P.p > 0.f;
  const uint32_t thr = drop_thr(P.p);
  const float sc = (drop ? 1.f / (1.f - P.p) : 1.f) * P.gscale;
  const uint64_t key = hash_u64(P.seed);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i, row = c >> 4, col = (c & 15) * 8;
    const int64_t t = tb * 64 + row;
    if (t >= P.M) continue;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(&tile[row * DX_TS + col]);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(&tile[row * DX_TS + col + 4]);
    const float d[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    bool kp[8];
    if (drop) keep8(key, P.offset + (uint64_t)t * (uint64_t)P.K + kb * 128 + col, thr, kp);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = (drop && !kp[e]) ? 0.f : d[e] * sc;
      o[e] = static_cast<bf16>(static_cast<float>(old[i][e]) + v);
    }
    *reinterpret_cast<bf16x8*>(dx + t * ldo + kb * 128 + col) = o;
  }
}

// ---- lora_refresh: B_i -> the adapter tail of W' (rows off_i.., columns col0 + j r ..) and of W'^T
// (rows col0 + j r .., columns off_i ..). One workgroup = a 64-row slab of one B_i, staged in LDS so
// both the row-major and the transposed writes are full 128 B rows.
__global__ __launch_bounds__(256) void lora_refresh_kernel(const LoraRefreshParams P) {
  __shared__ bf16 tile[64][64 + 8];
  int j = 0, slab = blockIdx.x;
  while (j + 1 < P.ntarget && slab >= (P.n[j] + 63) / 64) { slab -= (P.n[j] + 63) / 64; ++j; }
  const bf16* B = static_cast<const bf16*>(P.b[j]);
  const int r0 = slab * 64, n = P.n[j];
  bf16* W = static_cast<bf16*>(P.w);
  bf16* WT = static_cast<bf16*>(P.wt);
  for (int c0 = 0; c0 < P.r; c0 += 64) {
    for (int e = threadIdx.x; e < 64 * 8; e += 256) {  // 64 rows x 8 chunks of 8 bf16
      const int rr = e >> 3, cc = (e & 7) * 8;
      if (r0 + rr < n) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(B + (int64_t)(r0 + rr) * P.r + c0 + cc);
        *reinterpret_cast<bf16x8*>(W + (int64_t)(P.off[j] + r0 + rr) * P.ldw + P.col0 + j * P.r + c0 + cc) = v;
        if (WT != nullptr) {
#pragma unroll
          for (int q = 0; q < 8; ++q) tile[rr][cc + q] = v[q];
        }
      }
    }
    if (WT == nullptr) continue;  // workgroup-uniform: no transposed copy wanted
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 8; e += 256) {  // W'^T rows = the 64 columns of the slab
      const int cc = e >> 3, rr = (e & 7) * 8;
      if (r0 + rr < n) {
        bf16x8 v;
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = tile[rr + q][cc];
        *reinterpret_cast<bf16x8*>(WT + (int64_t)(P.trow0 + j * P.r + c0 + cc) * P.ldt + P.off[j] + r0 + rr) = v;
      }
    }
    __syncthreads();
  }
}

}  // namespace

void lora_refresh(const LoraRefreshParams& p, hipStream_t s) {
  int blocks = 0;
  for (int j = 0; j < p.ntarget; ++j) blocks += (p.n[j] + 63) / 64;
  hipLaunchKernelGGL(lora_refresh_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p);
}

bool lora_down_supported(int64_t M, int K, int R, int ldx, uint64_t offset) {
  return M > 0 && K % 128 == 0 && R % 32 == 0 && R >= 32 && R <= 256 && ldx % 8 == 0 && offset % 4 == 0;
}

// 32-token tiles per workgroup: 2 from R = 96 on (the A chunk loads dominate: qkv R = 192 72.8 -> 52.2 us,
// gate_up R = 128 60.4 -> 45.5 us in the LoRA step); 1 at R = 64, where two tiles cost a workgroup
// slot per CU (62.7 -> 73.5 us; profiles/r3_lora_grad_gemms.md). GRT_LORA_DOWN_TB=1/2 forces one.
int lora_down_tb(int R) {
  static const int env = [] { const char* e = getenv("GRT_LORA_DOWN_TB"); return e ? atoi(e) : 0; }();
  if (env == 1 || env == 2) return env;
  return R >= 96 ? 2 : 1;
}

// the LDS-DMA kernel takes R = 128 / 192 (the fused gate/up and q/k/v adapters of the SFT job:
// 57 -> 44 us and 67 -> 53 us at 6144 tokens, tools/lora_kernel_bench.py); at R = 64 the
// register-staged kernel is as fast or faster (o 34 vs 34 us, down 100 vs 116 us), so it keeps
// R = 64 unless GRT_LORA_DOWN_DMA=2. GRT_LORA_DOWN_DMA=0: the register-staged kernel everywhere.
static bool lora_down_dma(int R) {
  static const int env = [] { const char* e = getenv("GRT_LORA_DOWN_DMA"); return e ? atoi(e) : 1; }();
  return env != 0 && (R == 128 || R == 192 || (env == 2 && R == 64));
}

int lora_down_splits(int64_t M, int K, int R, int cus) {
  if (lora_down_dma(R)) {
    // 64-token workgroups (R = 64: two 64 KiB workgroups per CU). Splits are chosen by whole rounds
    // of workgroups: a launch of 1.1 rounds runs as long as 2 (the last workgroups stream a whole
    // split alone), so the cost is rounds x (chunks per split + the fp32 partial a split writes, ~2
    // chunks' worth of bytes), minimised over ks = 1 .. 16 with at least 4 chunks (the ring) per split.
    const int64_t ntb = (M + 63) / 64, slots = (int64_t)cus * (R == 64 ? 2 : 1);
    const int nch = K / LDD_KC;
    int best = 1;
    int64_t best_cost = -1;
    for (int ks = 1; ks <= 16 && nch / ks >= 4; ++ks) {
      const int64_t rounds = (ntb * ks + slots - 1) / slots;
      const int64_t cost = rounds * ((nch + ks - 1) / ks + (ks > 1 ? 2 : 0));
      if (best_cost < 0 || cost < best_cost) { best_cost = cost; best = ks; }
    }
    return best;
  }
  // at least ~3 workgroups per CU at one token tile per workgroup (a single 4-wave workgroup per CU
  // leaves every per-chunk latency exposed); with two tiles per workgroup the A loads are halved
  // and one split per workgroup slot (~1-2 per CU) keeps the fp32 partials small
  const int tbw = lora_down_tb(R);
  const int64_t ntb = (M + 32 * tbw - 1) / (32 * tbw);
  const int nch = K / 128;
  int64_t ks = ((tbw == 1 ? 3 : 1) * (int64_t)cus + ntb - 1) / ntb;
  if (ks > nch) ks = nch;
  if (ks > 16) ks = 16;
  return ks < 1 ? 1 : (int)ks;
}

void lora_down(const LoraDownParams& p, hipStream_t s) {
  if (lora_down_dma(p.R)) {
    const dim3 grid((unsigned)(((p.M + 63) / 64) * p.ksplit)), block(256);
    const bool xd = p.xd != nullptr;
#define GRT_LDD(RB)                                                                                  \
  if (xd) hipLaunchKernelGGL((lora_down_dma_kernel<RB, true>), grid, block, 0, s, p);                \
  else hipLaunchKernelGGL((lora_down_dma_kernel<RB, false>), grid, block, 0, s, p);
    if (p.R == 64) { GRT_LDD(2) } else if (p.R == 128) { GRT_LDD(4) } else { GRT_LDD(6) }
#undef GRT_LDD
  } else {
  const int tbw = lora_down_tb(p.R);
  const dim3 grid((unsigned)(((p.M + 32 * tbw - 1) / (32 * tbw)) * p.ksplit)), block(256);
  // GRT_LORA_DOWN_KC=64: half the LDS per workgroup (two workgroups per CU up to R = 192); measured
  // neutral on the Llama-2-7B LoRA step (profiles/r2_perf_experiments.md), so 128 by default
  static const int kc_env = [] { const char* e = getenv("GRT_LORA_DOWN_KC"); return e ? atoi(e) : 0; }();
  const bool kc64 = kc_env == 64;
  // GRT_LORA_DOWN_AD=2: A chunks two ahead in registers (R = 64 / 128 / 192 at 128-column chunks)
  static const int ad_env = [] { const char* e = getenv("GRT_LORA_DOWN_AD"); return e ? atoi(e) : 1; }();
  const bool ad2 = ad_env == 2 && !kc64;
#define GRT_LD(N)                                                                               \
  case N:                                                                                       \
    if (tbw == 1) {                                                                             \
      if (kc64) hipLaunchKernelGGL((lora_down_kernel<N, 64, 1>), grid, block, 0, s, p);         \
      else if (ad2 && (N == 2 || N == 4 || N == 6))                                             \
        hipLaunchKernelGGL((lora_down_kernel<N, 128, 1, (N == 2 || N == 4 || N == 6) ? 2 : 1>), grid, block, 0, s, p); \
      else hipLaunchKernelGGL((lora_down_kernel<N, 128, 1>), grid, block, 0, s, p);             \
    } else { /* R > 192: 64-column chunks (the 128-column images exceed the LDS) */            \
      if (kc64) hipLaunchKernelGGL((lora_down_kernel<N, 64, 2>), grid, block, 0, s, p);         \
      else if (ad2 && (N == 2 || N == 4 || N == 6))                                             \
        hipLaunchKernelGGL((lora_down_kernel<N, (N >= 7 ? 64 : 128), 2, (N == 2 || N == 4 || N == 6) ? 2 : 1>), grid, block, 0, s, p); \
      else hipLaunchKernelGGL((lora_down_kernel<N, (N >= 7 ? 64 : 128), 2>), grid, block, 0, s, p); \
    }                                                                                           \
    break;
  switch (p.R / 32) {
    GRT_LD(1) GRT_LD(2) GRT_LD(3) GRT_LD(4) GRT_LD(5) GRT_LD(6) GRT_LD(7)
    default: GRT_LD(8)
  }
#undef GRT_LD
  }
  if (p.ksplit > 1) {
    const int64_t n4 = p.M * (int64_t)p.R / 4;
    int64_t g = (n4 + 255) / 256;
    if (g > 2048) g = 2048;
    hipLaunchKernelGGL(lora_hsum_kernel, dim3((unsigned)g), dim3(256), 0, s, p.hpart, static_cast<bf16*>(p.h), n4,
                       p.ksplit, p.M * (int64_t)p.R, p.R, p.ldh > 0 ? p.ldh : (int64_t)p.R, p.hscale);
  }
}

bool lora_dx_supported(int64_t M, int K, int R, uint64_t offset) {
  return M > 0 && K % 128 == 0 && R % 16 == 0 && R >= 16 && R <= 256 && offset % 4 == 0;
}

void lora_dx(const LoraDxParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(((p.M + 63) / 64) * (p.K / 128))), block(256);
#define GRT_LDX(N) case N: hipLaunchKernelGGL(lora_dx_kernel<N>, grid, block, 0, s, p); break;
  switch (p.R / 16) {
    GRT_LDX(1) GRT_LDX(2) GRT_LDX(3) GRT_LDX(4) GRT_LDX(5) GRT_LDX(6) GRT_LDX(7) GRT_LDX(8)
    GRT_LDX(9) GRT_LDX(10) GRT_LDX(11) GRT_LDX(12) GRT_LDX(13) GRT_LDX(14) GRT_LDX(15)
    default: hipLaunchKernelGGL(lora_dx_kernel<16>, grid, block, 0, s, p); break;
  }
#undef GRT_LDX
}

}  // namespace grt
