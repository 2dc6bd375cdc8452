// LoRA adapter gradient GEMMs for gfx950 / CDNA4: the skinny products of the LoRA backward, each
// ONE pass over its big [tokens, features] operand at HBM rate.
//
// Reference role: the backward of PEFT's LoRA layer on every adapted projection of the QLoRA SFT job
// (r = 64 on q,k,v,o,gate,up,down; reference ray-jobs/fine_tune_llama_ray.py:243-254,
// fine_tune_config.json:6-8,30-33): per target i, with dY_i the projection's
// output gradient [M tokens, n_i], h'_i = s drop(x) A_i^T [M, r] and x_d = drop(x) [M, in]:
//     g_i  = s dY_i B_i          [M, r]     (dL/dh, feeds dA and the adapter's dX)
//     dB_i = dY_i^T h'_i         [n_i, r]
//     dA   = g^T x_d             [R, in]    (all targets of one input, R = r * targets)
// These are memory-bound (the r- or R-wide side is tiny): hipBLASLt tiles them as 64x16 .. 64x64
// output tiles, so every column tile re-reads the whole [M, n] operand (2-4 reads of dY per
// product; profiles/r3_lora_grad_gemms.md). Here each big operand is read once:
//
//   lora_g    C[M][64] (+)= alpha A[M][K] B[K][64], from B^T [64][K] (row stride ldbt).
//             One workgroup = 32 rows x all of K; A and B^T tiles arrive by LDS-DMA into a 4-slot
//             ring shared by the 4 waves, which split each tile's k-steps and sum through LDS.
//   lora_tred C = A^T H, A [M][N], H [M][R] (R = 64 / 128 / 192): the token-reduction products dB
//             (A = dY_i, H = h'_i) and dA (A = x_d, H = g; stored transposed). One workgroup = 128
//             columns of A x one range of tokens (split over M to fill the chip); A and H arrive in
//             32-token tiles by LDS-DMA into a 4-slot ring (attention.hip's pipeline: swizzled image,
//             counted vmcnt across raw s_barriers) and feed the MFMAs through transposed
//             (ds_read_b64_tr_b16) reads, wave w owning columns 32w..32w+31. fp32 partials per token
//             range go to a workspace in the OUTPUT layout (staged through LDS so both layouts store
//             whole rows); lora_tred_fin sums them, scales, converts and assigns / accumulates.
// v_mfma_f32_32x32x16_bf16 throughout (cdna_hip_programming.md §3 layouts).
#include <stdlib.h>

#include <type_traits>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

__device__ __forceinline__ f32x16 mfma_bf16_32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// accumulator element r of lane half hh holds row (r & 3) + 8 (r >> 2) + 4 hh of the 32-row tile
__device__ __forceinline__ int acc_row32(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// [rows][128 x bf16] LDS image, 256 B rows, 16-byte chunks XOR-swizzled so that both the b128 row
// reads (32 rows, one chunk) and the tr_b16 column reads are conflict-free (attention.hip img_off)
__device__ __forceinline__ int swz16(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int img_byte(int row, int ch) { return row * 256 + 16 * (ch ^ swz16(row)); }
__device__ __forceinline__ bf16x4 tr_read(const char* base, int r0, int c0, int l16) {
  const int q = l16 >> 2, p = l16 & 3;
  const int col = c0 + 4 * p;
  const char* a = base + img_byte(r0 + q, col >> 3) + 8 * ((col >> 2) & 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a);
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 a, bf16x4 b) { return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7); }

__device__ __forceinline__ void dma16(const void* gptr, uint32_t lds_byte_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gptr), "s"(lds_byte_addr) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

// ---------------------------------------------------------------------------------------------
// lora_g
// ---------------------------------------------------------------------------------------------
constexpr int G_SLOT = 8192 + 16384;        // A image (32 rows) + B^T image (64 rows)

template <int D>  // D DMA instructions per tile: wait until at most `pending` tiles are in flight
__device__ __forceinline__ void wait_pending(int pending) {
  if (pending >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * D) : "memory");
  else if (pending == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One workgroup = 32 rows x all of K, so the grid is M / 32 workgroups and no k-split partials (or
// finalize launch) are needed at M >= 8 K. Per 128-column k-tile the 32 A rows and the 64 B^T rows
// arrive by LDS-DMA into a 4-slot ring (swizzled images, counted vmcnt across raw s_barriers:
// attention.hip's pipeline), both shared by the 4 waves; wave w takes k-steps 2w, 2w + 1 of each
// tile, and the 4 partial 32x64 tiles are summed through LDS at the end. (Earlier forms, per-wave
// private images with register staging — B^T re-read per wave — ran at ~half the HBM rate; 128-row
// workgroups needed a 4-way k-split and a finalize launch per product: profiles/r3_lora_grad_gemms.md.)
// With fewer than 256 row blocks the k-tiles are split over ks workgroups (fp32 partials, lora_g_fin).
// product t's entry of a parameter array: selects on the wave-uniform index (a dynamically indexed
// by-value kernel argument would be copied to scratch)
template <class T>
__device__ __forceinline__ T pick(const T (&v)[kLoraGMax], int t) {
  return t == 0 ? v[0] : t == 1 ? v[1] : t == 2 ? v[2] : v[3];
}

// G_NS ring slots: 4 (96 KiB, one workgroup per CU) or 3 (72 KiB, two per CU)
template <int G_NS>
__global__ __launch_bounds__(256) void lora_g_kernel(const LoraGParams P) {
  __shared__ __attribute__((aligned(16))) char smem[G_NS * G_SLOT];
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, l16 = lane & 15;
  const int pt = blockIdx.y;  // product
  const int nrb = (int)((P.M + 31) / 32);
  const int rb = blockIdx.x % nrb, ksi = blockIdx.x / nrb;
  const int64_t m0 = (int64_t)rb * 32;
  const int K = pick(P.K, pt);
  const int64_t lda = pick(P.lda, pt), ldbt = pick(P.ldbt, pt), ldc = pick(P.ldc, pt);
  const int nkt_all = K / 128;
  const int kt0 = ksi * nkt_all / P.ks;
  const int nt = (ksi + 1) * nkt_all / P.ks - kt0;
  const bf16* A = static_cast<const bf16*>(pick(P.a, pt));
  const bf16* BT = static_cast<const bf16*>(pick(P.bt, pt));
  // DMA sources: wave w fills A rows 8w..8w+7 (2 pieces of 4 rows) and B^T rows 16w..16w+15
  // (4 pieces); piece row 4p + g4, the XOR swizzle on the per-lane source chunk
  const bf16* asrc[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int r = 8 * w + 4 * q + g4;
    const int64_t m = min(m0 + r, P.M - 1);
    asrc[q] = A + m * lda + (int64_t)kt0 * 128 + 8 * (l16 ^ swz16(r));
  }
  const bf16* bsrc[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 16 * w + 4 * q + g4;
    bsrc[q] = BT + (int64_t)r * ldbt + (int64_t)kt0 * 128 + 8 * (l16 ^ swz16(r));
  }
  const uint32_t smem0 = lds_addr(smem);
  auto dma_tile = [&](int t, int slot) {
    const uint32_t base = smem0 + (uint32_t)(slot * G_SLOT);
    const uint32_t da = __builtin_amdgcn_readfirstlane(base + (uint32_t)(8 * w * 256));
    const uint32_t db = __builtin_amdgcn_readfirstlane(base + (uint32_t)(8192 + 16 * w * 256));
#pragma unroll
    for (int q = 0; q < 2; ++q) dma16(asrc[q] + t * 128, da + q * 1024);
#pragma unroll
    for (int q = 0; q < 4; ++q) dma16(bsrc[q] + t * 128, db + q * 1024);
  };
  f32x16 acc0 = f32x16{}, acc1 = f32x16{};
  if (nt > 0) {
    const int pre = min(nt, G_NS - 1);
    for (int t = 0; t < pre; ++t) dma_tile(t, t);
    for (int t = 0; t < nt; ++t) {
      const int slot = t % G_NS;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of slot t-1 are done
      wait_pending<6>(min(nt, t + G_NS - 1) - (t + 1));   // tile t landed (this wave's pieces)
      __builtin_amdgcn_s_barrier();                        // ... every wave's; slot t-1 free
      if (t + G_NS - 1 < nt) dma_tile(t + G_NS - 1, (t + G_NS - 1) % G_NS);
      const char* ai = smem + slot * G_SLOT;
      const char* bi = ai + 8192;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int ch = 2 * (2 * w + s2) + hh;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(ai + img_byte(l32, ch));
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(bi + img_byte(l32, ch));
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(bi + img_byte(32 + l32, ch));
        acc0 = mfma_bf16_32(af, b0, acc0);
        acc1 = mfma_bf16_32(af, b1, acc1);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // ring consumed: the space takes the 4 partial tiles
  float* part = reinterpret_cast<float*>(smem);  // [4 waves][32 rows][64 cols]
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    part[w * 2048 + acc_row32(r, hh) * 64 + l32] = acc0[r];
    part[w * 2048 + acc_row32(r, hh) * 64 + 32 + l32] = acc1[r];
  }
  __syncthreads();
  const int row = tid >> 3, c8 = (tid & 7) * 8;
  const int64_t m = m0 + row;
  if (m >= P.M) return;
  float sum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sum[e] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(&part[q * 2048 + row * 64 + c8]);
    const f32x4 b = *reinterpret_cast<const f32x4*>(&part[q * 2048 + row * 64 + c8 + 4]);
    sum[0] += a[0]; sum[1] += a[1]; sum[2] += a[2]; sum[3] += a[3];
    sum[4] += b[0]; sum[5] += b[1]; sum[6] += b[2]; sum[7] += b[3];
  }
  if (P.ks > 1) {  // fp32 partial of this k range; lora_g_fin sums them
    float* ws = P.ws + (((int64_t)pt * P.ks + ksi) * P.M + m) * 64 + c8;
    *reinterpret_cast<f32x4*>(ws) = f32x4{sum[0], sum[1], sum[2], sum[3]};
    *reinterpret_cast<f32x4*>(ws + 4) = f32x4{sum[4], sum[5], sum[6], sum[7]};
    return;
  }
  bf16* C = static_cast<bf16*>(pick(P.c, pt)) + m * ldc + c8;
  bf16x8 o;
  const bf16x8 old = P.accumulate ? *reinterpret_cast<const bf16x8*>(C) : bf16x8{};
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = static_cast<bf16>(P.alpha * sum[e] + (P.accumulate ? static_cast<float>(old[e]) : 0.f));
  *reinterpret_cast<bf16x8*>(C) = o;
}

// C[m][0..63] (+)= alpha * sum_k ws[k][m][..] (grid y = product)
__global__ __launch_bounds__(256) void lora_g_fin_kernel(const LoraGParams P) {
  const int pt = blockIdx.y;
  const int64_t n4 = P.M * 16, plane = P.M * 64;
  bf16* C = static_cast<bf16*>(pick(P.c, pt));
  const int64_t ldc = pick(P.ldc, pt);
  const float* ws = P.ws + (int64_t)pt * P.ks * plane;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
    const int64_t m = e >> 4, c = (e & 15) * 4;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + 4 * e);
    for (int k = 1; k < P.ks; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * plane + 4 * e);
    bf16x4* dst = reinterpret_cast<bf16x4*>(C + m * ldc + c);
    bf16x4 o;
    const bf16x4 old = P.accumulate ? *dst : bf16x4{};
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = static_cast<bf16>(P.alpha * s[q] + (P.accumulate ? static_cast<float>(old[q]) : 0.f));
    *dst = o;
  }
}

// ---------------------------------------------------------------------------------------------
// lora_tred
// ---------------------------------------------------------------------------------------------
constexpr int TR_NS = 4;           // ring slots
constexpr int TR_IMG = 32 * 256;   // one 32-token x 128-column image: 8 KiB

template <int RT>  // R = 32 RT
constexpr int tr_nhi() { return (32 * RT + 127) / 128; }
template <int RT>
constexpr int tr_slot() { return TR_IMG * (1 + tr_nhi<RT>()); }
template <int RT>
constexpr int tr_lds() {  // ring, or the 128 x (R + 4) fp32 output tile of the epilogue
  return TR_NS * tr_slot<RT>() > 128 * (32 * RT + 4) * 4 ? TR_NS * tr_slot<RT>() : 128 * (32 * RT + 4) * 4;
}

template <int RT>
__global__ __launch_bounds__(256) void lora_tred_kernel(const LoraTredParams P) {
  constexpr int R = 32 * RT, NHI = tr_nhi<RT>(), SLOT = tr_slot<RT>(), DPT = 2 * (1 + NHI);
  __shared__ __attribute__((aligned(16))) char smem[tr_lds<RT>()];
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, l16 = lane & 15;
  const int gb = blockIdx.x % P.nbt, ks = blockIdx.x / P.nbt;  // column block of the launch, split
  const int pt = (gb >= P.bo[1]) + (gb >= P.bo[2]) + (gb >= P.bo[3]);  // product (bo past nprod: INT_MAX)
  const int nb = gb - pick(P.bo, pt);
  const int N = pick(P.N, pt);
  const int64_t lda = pick(P.lda, pt), ldh = pick(P.ldh, pt);
  const int64_t mbeg = (int64_t)ks * P.mchunk;
  const int64_t mend = min(P.M, mbeg + P.mchunk);
  const int nt = mend > mbeg ? (int)((mend - mbeg) / 32) : 0;
  const bf16* A = static_cast<const bf16*>(pick(P.a, pt)) + (int64_t)nb * 128;
  const bf16* H = static_cast<const bf16*>(pick(P.h, pt));

  // LDS-DMA of tile t: wave w fills image rows 8w .. 8w+7 (two 1-KiB pieces of 4 rows) of the A
  // image and of every H image; the XOR swizzle is applied to the per-lane SOURCE chunk. H images
  // past column R (R = 64, or the second image at R = 192) re-read a valid chunk: never consumed.
  const uint32_t smem0 = lds_addr(smem);
  const int row0 = 8 * w + g4, row1 = row0 + 4;
  const int ch0 = l16 ^ swz16(row0), ch1 = l16 ^ swz16(row1);
  auto dma_tile = [&](int t, int slot) {
    const int64_t r0 = mbeg + 32 * t + row0, r1 = mbeg + 32 * t + row1;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(smem0 + (uint32_t)(slot * SLOT + 8 * w * 256));
    dma16(A + r0 * lda + 8 * ch0, dst);
    dma16(A + r1 * lda + 8 * ch1, dst + 1024);
#pragma unroll
    for (int hi = 0; hi < NHI; ++hi) {
      const int valid = (R - 128 * hi) >= 128 ? 16 : (R - 128 * hi) / 8;  // chunks of this image inside R
      const int c0 = 128 * hi + 8 * (ch0 % valid), c1 = 128 * hi + 8 * (ch1 % valid);
      dma16(H + r0 * ldh + c0, dst + (1 + hi) * TR_IMG);
      dma16(H + r1 * ldh + c1, dst + (1 + hi) * TR_IMG + 1024);
    }
  };

  f32x16 acc[RT];
#pragma unroll
  for (int j = 0; j < RT; ++j) acc[j] = f32x16{};
  if (nt > 0) {
    const int pre = min(nt, TR_NS - 1);
    for (int t = 0; t < pre; ++t) dma_tile(t, t);
    for (int t = 0; t < nt; ++t) {
      const int slot = t % TR_NS;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot t-1 are done
      wait_pending<DPT>(min(nt, t + TR_NS - 1) - (t + 1));  // tile t landed (this wave's pieces)
      __builtin_amdgcn_s_barrier();                         // ... every wave's; slot t-1 free
      if (t + TR_NS - 1 < nt) dma_tile(t + TR_NS - 1, (t + TR_NS - 1) % TR_NS);
      const char* ai = smem + slot * SLOT;
#pragma unroll
      for (int stp = 0; stp < 2; ++stp) {
        const int kk = 16 * stp + 4 * hh;
        const int c0 = 32 * w + (g4 & 1) * 16;
        const bf16x8 a = cat8(tr_read(ai, kk, c0, l16), tr_read(ai, kk + 8, c0, l16));
#pragma unroll
        for (int j = 0; j < RT; ++j) {
          const char* hi = ai + TR_IMG * (1 + (j >> 2));
          const int cj = 32 * (j & 3) + (g4 & 1) * 16;
          const bf16x8 b = cat8(tr_read(hi, kk, cj, l16), tr_read(hi, kk + 8, cj, l16));
          acc[j] = mfma_bf16_32(a, b, acc[j]);  // D[column of A][column of H]
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // ring consumed: the space takes the fp32 output tile
  constexpr int TS = R + 4;
  float* tile = reinterpret_cast<float*>(smem);  // [128 columns of A][R]
#pragma unroll
  for (int j = 0; j < RT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) tile[(32 * w + acc_row32(r, hh)) * TS + 32 * j + l32] = acc[j][r];
  __syncthreads();
  float* ws = P.ws + ((int64_t)ks * P.nbt + pick(P.bo, pt)) * 128 * R;  // this product's plane of the split
  if (!P.transpose) {  // ws[n][j]: thread -> 4 consecutive j of one n
    for (int e = tid; e < 128 * R / 4; e += 256) {
      const int n = e / (R / 4), j4 = (e % (R / 4)) * 4;
      *reinterpret_cast<f32x4*>(ws + (int64_t)(nb * 128 + n) * R + j4) = *reinterpret_cast<const f32x4*>(&tile[n * TS + j4]);
    }
  } else {  // ws[j][n]: thread -> 4 consecutive n of one j
    for (int e = tid; e < 128 * R / 4; e += 256) {
      const int j = e / 32, n4 = (e % 32) * 4;
      f32x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = tile[(n4 + q) * TS + j];
      *reinterpret_cast<f32x4*>(ws + (int64_t)j * N + nb * 128 + n4) = v;
    }
  }
}

// out_t[row][col] (+)= alpha * sum_ks ws[ks][plane of t][row][col], rows x cols = N_t x R (or R x N_t
// transposed); grid y = product
__global__ __launch_bounds__(256) void lora_tred_fin_kernel(const LoraTredParams P) {
  const int pt = blockIdx.y;
  const int N = pick(P.N, pt);
  const int64_t rows = P.transpose ? P.R : N, cols = P.transpose ? N : P.R;
  const int64_t n4 = rows * cols / 4, plane = (int64_t)P.nbt * 128 * P.R;
  const float* ws = P.ws + (int64_t)pick(P.bo, pt) * 128 * P.R;
  bf16* out = static_cast<bf16*>(pick(P.out, pt));
  const int64_t ldo = pick(P.ldo, pt);
  const bool acc = pick(P.accumulate, pt) != 0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n4; e += (int64_t)gridDim.x * 256) {
    const int64_t row = (4 * e) / cols, col = (4 * e) % cols;
    f32x4 s = *reinterpret_cast<const f32x4*>(ws + 4 * e);
    for (int k = 1; k < P.ks; ++k) s += *reinterpret_cast<const f32x4*>(ws + k * plane + 4 * e);
    bf16x4* dst = reinterpret_cast<bf16x4*>(out + row * ldo + col);
    bf16x4 o;
    if (acc) {
      const bf16x4 old = *dst;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = static_cast<bf16>(static_cast<float>(old[q]) + P.alpha * s[q]);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = static_cast<bf16>(P.alpha * s[q]);
    }
    *dst = o;
  }
}

}  // namespace

bool lora_g_supported(int64_t M, int K, int r) { return M > 0 && K > 0 && K % 128 == 0 && r == 64; }

// ring depth (GRT_LORA_G_NS: 4 -> one 96 KiB workgroup per CU (default), 3 -> two 72 KiB workgroups
// per CU: 1-2 % slower at the SFT shapes, tools/lora_kernel_bench.py)
static int lora_g_ns() {
  static const int ns = [] {
    const char* e = getenv("GRT_LORA_G_NS");
    return e && atoi(e) == 3 ? 3 : 4;
  }();
  return ns;
}

// k splits: only when the 32-row blocks (of all products) leave a quarter of the workgroup slots idle;
// at most 8
int lora_g_splits(int64_t M, int K, int cus, int nprod) {
  cus *= lora_g_ns() == 3 ? 2 : 1;  // workgroup slots
  const int64_t nrb = (M + 31) / 32 * nprod;
  if (4 * nrb >= 3 * (int64_t)cus) return 1;  // >= 3/4 of the CUs busy: no partials, no finalize launch
  int ks = (int)((cus + nrb - 1) / nrb);
  if (ks > 8) ks = 8;
  if (ks > K / 128) ks = K / 128;
  return ks < 1 ? 1 : ks;
}

void lora_g(const LoraGParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(((p.M + 31) / 32) * p.ks), (unsigned)p.nprod), block(256);
  if (lora_g_ns() == 3) hipLaunchKernelGGL(lora_g_kernel<3>, grid, block, 0, s, p);
  else hipLaunchKernelGGL(lora_g_kernel<4>, grid, block, 0, s, p);
  if (p.ks > 1) {
    int64_t fb = (p.M * 16 + 255) / 256;
    if (fb > 1024) fb = 1024;
    hipLaunchKernelGGL(lora_g_fin_kernel, dim3((unsigned)fb, (unsigned)p.nprod), block, 0, s, p);
  }
}

bool lora_tred_supported(int64_t M, int N, int R) {
  return M > 0 && M % 32 == 0 && N > 0 && N % 128 == 0 && (R == 64 || R == 128 || R == 192);
}

// token splits: one workgroup per CU (each split adds an N x R fp32 partial write + read: two per CU
// at N = 4096, R = 64 made the partials a quarter of the operand's bytes), at most 16, each split a
// whole number of 32-token tiles
int lora_tred_splits(int64_t M, int N, int R, int cus) {
  // workgroups per CU the splits aim at (GRT_LORA_TRED_WPC, default 1; R = 64 fits two 64 KiB
  // workgroups per CU, 5-9 % slower at the SFT shapes: tools/lora_kernel_bench.py)
  static const int wpc = [] {
    const char* e = getenv("GRT_LORA_TRED_WPC");
    return e && atoi(e) > 1 ? 2 : 1;
  }();
  if (R == 64) cus *= wpc;
  const int nblk = N / 128;
  int ks = (int)(((int64_t)cus + nblk - 1) / nblk);
  const int64_t tiles = M / 32;
  if (ks > 16) ks = 16;
  if (ks > tiles) ks = (int)tiles;
  return ks < 1 ? 1 : ks;
}

void lora_tred(const LoraTredParams& p0, hipStream_t s) {
  LoraTredParams p = p0;
  const int64_t tiles = p.M / 32;
  p.mchunk = 32 * ((tiles + p.ks - 1) / p.ks);
  const dim3 grid((unsigned)(p.nbt * p.ks)), block(256);
  switch (p.R) {
    case 64: hipLaunchKernelGGL(lora_tred_kernel<2>, grid, block, 0, s, p); break;
    case 128: hipLaunchKernelGGL(lora_tred_kernel<4>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(lora_tred_kernel<6>, grid, block, 0, s, p); break;
  }
  int nmax = 0;
  for (int t = 0; t < p.nprod; ++t) nmax = p.N[t] > nmax ? p.N[t] : nmax;
  const int64_t n4 = (int64_t)nmax * p.R / 4;
  int64_t fb = (n4 + 255) / 256;
  if (fb > 1024) fb = 1024;
  hipLaunchKernelGGL(lora_tred_fin_kernel, dim3((unsigned)fb, (unsigned)p.nprod), block, 0, s, p);
}

}  // namespace grt
