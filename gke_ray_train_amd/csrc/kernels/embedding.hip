// Token embedding for gfx950: gather forward, segmented scatter-add backward.
//
// Reference role: nn.Embedding of BasicLLM and HF Llama (reference
// ray-jobs/pytorch_llm_ray.py:80,100 and the Llama embed_tokens under fine_tune_llama_ray.py:240).
// torch's CUDA/HIP backward sorts the ids, runs several segment kernels and zero-fills the whole
// [V, d] gradient separately. Here the backward is ONE pass over the V rows of dW: rows no token
// hit are zero-filled (overwrite mode) or left alone (accumulate mode, gradient accumulation), and
// each hit row sums its tokens' dY rows in fp32 in sorted order (deterministic, no atomics), then
// writes / adds the result. The sort of the N ids (8 K for a Llama-2-7B step) stays in torch.
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kNT = 256;

// one wave per output row, 16-byte chunks
template <typename T>
__global__ __launch_bounds__(kNT) void embedding_fwd_kernel(const int64_t* __restrict__ ids,
                                                            const T* __restrict__ w, T* __restrict__ out,
                                                            int64_t n, int d, int64_t V) {
  constexpr int VE = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  for (int64_t r = (int64_t)blockIdx.x * (kNT / 64) + (threadIdx.x >> 6); r < n;
       r += (int64_t)gridDim.x * (kNT / 64)) {
    const int64_t id = ids[r];
    GRT_DEVICE_CHECK(id >= 0 && id < V);
    const T* src = w + id * d;
    T* dst = out + r * d;
    for (int c = lane * VE; c < d; c += 64 * VE)
      *reinterpret_cast<typename Vec16<T>::type*>(dst + c) = *reinterpret_cast<const typename Vec16<T>::type*>(src + c);
  }
}

// [row_start[v], row_end[v]) = the positions in the sorted id list (and in `order`) of the tokens
// of vocabulary row v; empty when v is not hit.
template <typename T>
__global__ __launch_bounds__(kNT) void embedding_bwd_kernel(const T* __restrict__ dy, const int64_t* __restrict__ order,
                                                            const int32_t* __restrict__ row_start,
                                                            const int32_t* __restrict__ row_end, T* __restrict__ dw,
                                                            int64_t V, int d, int accumulate) {
  constexpr int VE = Vec16<T>::N;
  const int lane = threadIdx.x & 63;
  for (int64_t v = (int64_t)blockIdx.x * (kNT / 64) + (threadIdx.x >> 6); v < V; v += (int64_t)gridDim.x * (kNT / 64)) {
    const int s = row_start[v];
    const int e = row_end[v];
    T* out = dw + v * d;
    if (s >= e) {  // no token of this row
      if (!accumulate) {
        float z[VE];
#pragma unroll
        for (int i = 0; i < VE; ++i) z[i] = 0.f;
        for (int c = lane * VE; c < d; c += 64 * VE) store16(out + c, z);
      }
      continue;
    }
    for (int c = lane * VE; c < d; c += 64 * VE) {
      float acc[VE];
      if (accumulate) load16(out + c, acc);
      else {
#pragma unroll
        for (int i = 0; i < VE; ++i) acc[i] = 0.f;
      }
      for (int k = s; k < e; ++k) {
        float g[VE];
        load16(dy + order[k] * d + c, g);
#pragma unroll
        for (int i = 0; i < VE; ++i) acc[i] += g[i];
      }
      store16(out + c, acc);
    }
  }
}

inline unsigned rows_grid(int64_t rows) {
  int64_t g = (rows + 3) / 4;
  return (unsigned)(g > 256 * 16 ? 256 * 16 : (g < 1 ? 1 : g));
}

}  // namespace

void embedding_fwd(DType dt, const int64_t* ids, const void* w, void* out, int64_t n, int d, int64_t V,
                   hipStream_t s) {
  if (dt == DType::BF16)
    hipLaunchKernelGGL(embedding_fwd_kernel<bf16>, dim3(rows_grid(n)), dim3(kNT), 0, s, ids, (const bf16*)w,
                       (bf16*)out, n, d, V);
  else
    hipLaunchKernelGGL(embedding_fwd_kernel<float>, dim3(rows_grid(n)), dim3(kNT), 0, s, ids, (const float*)w,
                       (float*)out, n, d, V);
}

void embedding_bwd(DType dt, const void* dy, const int64_t* order, const int32_t* row_start, const int32_t* row_end,
                   void* dw, int64_t V, int d, bool accumulate, hipStream_t s) {
  if (dt == DType::BF16)
    hipLaunchKernelGGL(embedding_bwd_kernel<bf16>, dim3(rows_grid(V)), dim3(kNT), 0, s, (const bf16*)dy, order,
                       row_start, row_end, (bf16*)dw, V, d, accumulate ? 1 : 0);
  else
    hipLaunchKernelGGL(embedding_bwd_kernel<float>, dim3(rows_grid(V)), dim3(kNT), 0, s, (const float*)dy, order,
                       row_start, row_end, (float*)dw, V, d, accumulate ? 1 : 0);
}

}  // namespace grt
