// bf16 matrix transpose for the input-gradient GEMM of trainable projections.
//
// dX = dY W runs ~13-15 % faster as the TN library GEMM on a contiguous W^T than as the NN GEMM on
// W (profiles/r1_dgrad_layout_ab.jsonl), so the framework's linear op writes W^T into a persistent
// buffer during the forward — on a side stream, beside the forward GEMMs — and the backward
// consumes it. One workgroup moves a 64 x 64 tile: 16-byte row-segment loads into a padded LDS
// tile (conflict-free column reads), 16-byte row-segment stores of the transposed tile. HBM-bound:
// a 7B model's projections are 13.5 GB each way per step.
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                             int rows, int cols) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  {  // load: thread t -> tile row t/4, columns 16*(t&3) .. +15
    const int tr = t >> 2, tc = (t & 3) * 16;
    float v[16];
    load16(src + (int64_t)(r0 + tr) * cols + c0 + tc, v);
    load16(src + (int64_t)(r0 + tr) * cols + c0 + tc + 8, v + 8);
#pragma unroll
    for (int k = 0; k < 16; ++k) tile[tr][tc + k] = v[k];
  }
  __syncthreads();
  {  // store: thread t -> output row c0 + t/4 (a source column), 16 source rows
    const int oc = t >> 2, orr = (t & 3) * 16;
    float o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = tile[orr + k][oc];
    bf16* d = dst + (int64_t)(c0 + oc) * rows + r0 + orr;
    store16(d, o);
    store16(d + 8, o + 8);
  }
}

}  // namespace

void transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t s) {
  const dim3 grid((unsigned)(cols / 64), (unsigned)(rows / 64));
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, (const bf16*)src, (bf16*)dst, rows, cols);
}

}  // namespace grt
