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

// v2: one workgroup = 64 rows x 128 columns (16 KiB). Load: 4 threads per 256-byte row, 16-byte
// ds_write_b128 into an XOR-swizzled image (rows of 16 chunks; chunk ^ ((row & 3) << 2 | (row >> 2) & 3),
// the dual row-write / transposed-read image of gemm.hip). Store: gfx950's ds_read_b64_tr_b16 hands
// lane i of a 16-lane group column c0 + i of four source rows, so 4 reads give a lane 16 consecutive
// elements of one output row — 4 LDS reads + 2 global 16-byte stores per 16 outputs instead of 16
// scalar LDS reads; a wave stores 16 output rows x 128 bytes (full lines).
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
__device__ __forceinline__ int tswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int toff(int row, int ch) { return row * 256 + 16 * (ch ^ tswz(row)); }

__global__ __launch_bounds__(256) void transpose2_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                              int rows, int cols) {
  __shared__ __attribute__((aligned(16))) char img[64 * 256];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 128;
  const int t = threadIdx.x, lane = t & 63, l16 = lane & 15;
  {
    const int row = t >> 2, ch0 = (t & 3) * 4;
    const bf16* sp = src + (int64_t)(r0 + row) * cols + c0 + ch0 * 8;
    bf16x8 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const bf16x8*>(sp + 8 * k);
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<bf16x8*>(img + toff(row, ch0 + k)) = v[k];
  }
  __syncthreads();
  const int grp = t >> 4;  // 16 groups; group g handles (column block, row block) pairs g and g + 16
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int pr = grp + 16 * pp;
    const int cb = 16 * (pr >> 2), rb = 16 * (pr & 3);  // 16 source columns, 16 source rows
    bf16x4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = rb + 4 * k + (l16 >> 2), col = cb + 4 * (l16 & 3);
      const char* a = img + toff(rr, col >> 3) + 8 * ((col >> 2) & 1);
      q[k] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)a);
    }
    bf16x8 o0 = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    bf16x8 o1 = __builtin_shufflevector(q[2], q[3], 0, 1, 2, 3, 4, 5, 6, 7);
    bf16* d = dst + (int64_t)(c0 + cb + l16) * rows + r0 + rb;
    *reinterpret_cast<bf16x8*>(d) = o0;
    *reinterpret_cast<bf16x8*>(d + 8) = o1;
  }
}

}  // namespace

void transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t s) {
  static const int v1 = [] { const char* e = getenv("GRT_TRANSPOSE_V1"); return e && atoi(e) == 1; }();
  if (!v1 && cols % 128 == 0) {
    const dim3 grid((unsigned)(cols / 128), (unsigned)(rows / 64));
    hipLaunchKernelGGL(transpose2_bf16_kernel, grid, dim3(256), 0, s, (const bf16*)src, (bf16*)dst, rows, cols);
    return;
  }
  const dim3 grid((unsigned)(cols / 64), (unsigned)(rows / 64));
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, (const bf16*)src, (bf16*)dst, rows, cols);
}

}  // namespace grt
