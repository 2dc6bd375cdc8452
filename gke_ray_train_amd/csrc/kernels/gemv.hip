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

template <int M>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                   const bf16* __restrict__ w, bf16* __restrict__ y,
                                                   int64_t ldy, int N, int K) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + wave) * kR;
  float acc[M][kR];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kR; ++r) acc[m][r] = 0.f;
  const u32x4* wr[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) wr[r] = reinterpret_cast<const u32x4*>(w + (int64_t)min(n0 + r, N - 1) * K);
#pragma unroll 2
  for (int k = lane * 8; k < K; k += 512) {
    u32x4 wv[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) wv[r] = __builtin_nontemporal_load(wr[r] + k / 8);
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) bf16x8_to_f32(*reinterpret_cast<const u32x4*>(x + m * ldx + k), xf[m]);
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
      if (lane == 0 && n0 + r < N) y[m * ldy + n0 + r] = static_cast<bf16>(v);
    }
}

}  // namespace

void gemv_bf16(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int M, int N, int K, hipStream_t s) {
  const dim3 grid((unsigned)((N + 4 * kR - 1) / (4 * kR)));
  const bf16* xb = static_cast<const bf16*>(x);
  const bf16* wb = static_cast<const bf16*>(w);
  bf16* yb = static_cast<bf16*>(y);
  switch (M) {
    case 1: hipLaunchKernelGGL(gemv_kernel<1>, grid, dim3(256), 0, s, xb, ldx, wb, yb, ldy, N, K); break;
    case 2: hipLaunchKernelGGL(gemv_kernel<2>, grid, dim3(256), 0, s, xb, ldx, wb, yb, ldy, N, K); break;
    case 3: hipLaunchKernelGGL(gemv_kernel<3>, grid, dim3(256), 0, s, xb, ldx, wb, yb, ldy, N, K); break;
    default: hipLaunchKernelGGL(gemv_kernel<4>, grid, dim3(256), 0, s, xb, ldx, wb, yb, ldy, N, K); break;
  }
}

}  // namespace grt
