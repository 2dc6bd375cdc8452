// Test support: fill the LDS of every CU with a bit pattern (e.g. a quiet NaN) so that a kernel
// launched next and reading LDS it never wrote — an LDS-DMA slot read before its covering vmcnt /
// barrier, a reduction array read before every wave stored its element — sees that pattern
// instead of the usually finite leftovers of the previous kernel (cdna_hip_programming.md "Read a
// staged buffer one phase AFTER the wait that retires it": early reads pass reference checks
// whenever the data happens to land first). Not used on any training path.
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kLdsBytes = 160 * 1024;  // the whole LDS of a CU: one resident workgroup per CU

__global__ __launch_bounds__(256) void lds_fill_kernel(uint32_t pattern, uint32_t* sink) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const int n = kLdsBytes / 16;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    reinterpret_cast<uint4*>(lds)[i] = make_uint4(pattern, pattern, pattern, pattern);
  __syncthreads();
  // keep the stores: a value that depends on them decides a (never taken) global write
  if (lds[(threadIdx.x * 37) % (kLdsBytes / 4)] == pattern + 1u) sink[threadIdx.x] = 1u;
}

}  // namespace

void lds_fill(uint32_t pattern, hipStream_t s) {
  static bool attr = [] {
    return hipFuncSetAttribute((const void*)lds_fill_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               kLdsBytes) == hipSuccess;
  }();
  (void)attr;
  // 4 waves of 256 single-workgroup-per-CU blocks: every CU takes at least one
  hipLaunchKernelGGL(lds_fill_kernel, dim3(1024), dim3(256), kLdsBytes, s, pattern, (uint32_t*)nullptr);
}

}  // namespace grt
