// Skinny GEMM (GEMV) for the decode step: y[m][n] = sum_k x[m][k] * W[n][k], m < M <= 4, bf16.
//
// Reference role: the per-token projections of HF ``generate`` in the post-training inference
// comparison (reference ray-jobs/fine_tune_llama_ray.py:138-146). With one to
// four tokens per step the projections are pure weight streams (an 8B model reads ~16 GB per
// token), so the kernel is built for HBM bandwidth, not MFMA: each wave owns R = 4 weight rows and
// streams them with 16-byte non-temporal loads (the weights are read once per token;
// MI355X_MICROARCH.md "nt-weights"), 4 rows x 16 B in flight per lane per K-step of 512; the
// activations (M x K, a few KB) are re-read from L1/L2 by every wave. fp32 accumulation, one
// wave-wide butterfly reduction per (m, row) at the end. Grid = N / 16 workgroups of 4 waves.
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kR = 4;  // weight rows per wave
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void bf16x8_to_f32(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// KS waves of the workgroup split K for the same kR rows (KS = 4 for N <= 8192: 4x the workgroups
// and weight bytes in flight on the small projections, whose 1-workgroup-per-CU grid left HBM
// latency exposed — o_proj ran at 3.5 TB/s), partial sums merged through LDS.
// SWI: x is the fused [gate | up] projection output [M, 2K]; the kernel multiplies by
// silu(gate) * up on the fly (the decode MLP's SwiGLU folded into the down-projection GEMV).
template <int M, int KS, bool SWI>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                   const bf16* __restrict__ w, bf16* __restrict__ y,
                                                   int64_t ldy, int N, int K) {
  __shared__ float red[4][M][kR];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int slot = wave / KS, kp = wave % KS;
  const int n0 = (blockIdx.x * (4 / KS) + slot) * kR;
  float acc[M][kR];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kR; ++r) acc[m][r] = 0.f;
  const u32x4* wr[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) wr[r] = reinterpret_cast<const u32x4*>(w + (int64_t)min(n0 + r, N - 1) * K);
#pragma unroll 2
  for (int k = (kp * 64 + lane) * 8; k < K; k += 512 * KS) {
    u32x4 wv[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) wv[r] = __builtin_nontemporal_load(wr[r] + k / 8);
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      bf16x8_to_f32(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf[m]);
      if constexpr (SWI) {
        float uf[8];
        bf16x8_to_f32(*reinterpret_cast<const u32x4*>(x + m * ldx + K + k), uf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // round like the separate SwiGLU kernel's bf16 output
          xf[m][j] = static_cast<float>(static_cast<bf16>(silu_f(xf[m][j]) * uf[j]));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float wf[8];
      bf16x8_to_f32(wv[r], wf);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[m][r] = fmaf(xf[m][j], wf[j], acc[m][r]);
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float v = acc[m][r];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][r] = v;
    }
  if constexpr (KS > 1) {
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < kR; ++r) red[wave][m][r] = acc[m][r];
    }
    __syncthreads();
    if (kp != 0) return;
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < KS; ++q) v += red[slot * KS + q][m][r];
        acc[m][r] = v;
      }
  }
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < M; ++m)
#pragma unroll
      for (int r = 0; r < kR; ++r)
        if (n0 + r < N) y[m * ldy + n0 + r] = static_cast<bf16>(acc[m][r]);
  }
}

template <int KS, bool SWI>
void launch_gemv(const bf16* x, int64_t ldx, const bf16* w, bf16* y, int64_t ldy, int M, int N, int K, hipStream_t s) {
  const int rows_per_wg = (4 / KS) * kR;
  const dim3 grid((unsigned)((N + rows_per_wg - 1) / rows_per_wg));
  switch (M) {
    case 1: hipLaunchKernelGGL((gemv_kernel<1, KS, SWI>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, N, K); break;
    case 2: hipLaunchKernelGGL((gemv_kernel<2, KS, SWI>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, N, K); break;
    case 3: hipLaunchKernelGGL((gemv_kernel<3, KS, SWI>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, N, K); break;
    default: hipLaunchKernelGGL((gemv_kernel<4, KS, SWI>), grid, dim3(256), 0, s, x, ldx, w, y, ldy, N, K); break;
  }
}

}  // namespace

int gemv_k_split(int N) {
  static const int env = [] { const char* e = getenv("GRT_GEMV_KSPLIT"); return e ? atoi(e) : -1; }();
  if (env == 1 || env == 4) return env;
  return N <= 8192 ? 4 : 1;
}

// y[M, N] = x[M, K] W^T (swiglu: x = silu(gu[:, :K]) * gu[:, K:], ldx = gu's row stride)
void gemv_bf16(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int M, int N, int K, hipStream_t s,
               bool swiglu) {
  const bf16* xb = static_cast<const bf16*>(x);
  const bf16* wb = static_cast<const bf16*>(w);
  bf16* yb = static_cast<bf16*>(y);
  const bool ks4 = gemv_k_split(N) == 4;
  if (swiglu) {
    if (ks4) launch_gemv<4, true>(xb, ldx, wb, yb, ldy, M, N, K, s);
    else launch_gemv<1, true>(xb, ldx, wb, yb, ldy, M, N, K, s);
  } else {
    if (ks4) launch_gemv<4, false>(xb, ldx, wb, yb, ldy, M, N, K, s);
    else launch_gemv<1, false>(xb, ldx, wb, yb, ldy, M, N, K, s);
  }
}

}  // namespace grt
