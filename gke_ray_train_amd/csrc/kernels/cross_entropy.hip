// Fused softmax cross-entropy (forward: per-row loss + logsumexp; backward: in-place dlogits).
//
// Reference roles: nn.CrossEntropyLoss on BasicLLM's [B*S, V] logits
// (reference ray-jobs/pytorch_llm_ray.py:237,275) and the HF causal-LM shifted CE with
// ignore_index=-100 behind SFTTrainer (ray-jobs/fine_tune_llama_ray.py:333). SURVEY §2.6
// K-A11 / K-B10.
//
// One 256-thread workgroup per row, one HBM pass per direction: the forward keeps an online
// (max, sum) per thread over 16-byte vectors and merges them across the workgroup; the
// backward recomputes softmax from the saved LSE and writes (p - onehot) * dloss[row] in the
// logits' own dtype, optionally over the logits buffer itself so a [tokens, 128256] fp32 copy is
// never materialised.
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kNT = 256;

template <typename T>
__global__ __launch_bounds__(kNT) void ce_fwd_kernel(const T* __restrict__ logits, int64_t ld,
                                                     const int64_t* __restrict__ labels,
                                                     float* __restrict__ loss, float* __restrict__ lse_out,
                                                     int V, int64_t ignore_index, int vec_ok) {
  constexpr int VE = Vec16<T>::N;
  __shared__ float red[2 * kNT / kWave];
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  float m = -INFINITY, s = 0.f;
  const int nvec = vec_ok ? V / VE : 0;
  for (int i = threadIdx.x; i < nvec; i += kNT) {
    float a[VE];
    load16(x + (int64_t)i * VE, a);
    float mx = a[0];
#pragma unroll
    for (int k = 1; k < VE; ++k) mx = fmaxf(mx, a[k]);
    const float mn = fmaxf(m, mx);
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < VE; ++k) acc += __expf(a[k] - mn);
    s = s * __expf(m - mn) + acc;
    m = mn;
  }
  for (int j = nvec * VE + threadIdx.x; j < V; j += kNT) {
    const float a = to_f(x[j]);
    const float mn = fmaxf(m, a);
    s = s * __expf(m - mn) + __expf(a - mn);
    m = mn;
  }
  // merge (m, s) across the workgroup
  const float gm = block_max<kNT>(m, red);
  const float sc = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  const float gs = block_sum<kNT>(sc, red);
  if (threadIdx.x == 0) {
    const float lse = gm + __logf(gs);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    loss[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - to_f(x[lab]);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void ce_bwd_kernel(const T* logits, int64_t ld,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ gscale, T* dlogits,
                                                     int64_t ldd, int V, int64_t ignore_index,
                                                     int vec_ok) {
  constexpr int VE = Vec16<T>::N;
  const int64_t row = blockIdx.x;
  const T* x = logits + row * ld;
  T* dx = dlogits + row * ldd;
  const int64_t lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ign ? 0.f : gscale[row];
  const float l = lse[row];
  const int nvec = vec_ok ? V / VE : 0;
  for (int i = threadIdx.x; i < nvec; i += kNT) {
    float a[VE];
    load16(x + (int64_t)i * VE, a);
#pragma unroll
    for (int k = 0; k < VE; ++k) {
      const int j = i * VE + k;
      a[k] = (__expf(a[k] - l) - (j == lab ? 1.f : 0.f)) * g;
    }
    store16(dx + (int64_t)i * VE, a);
  }
  for (int j = nvec * VE + threadIdx.x; j < V; j += kNT) {
    const float a = to_f(x[j]);
    dx[j] = from_f<T>((__expf(a - l) - (j == lab ? 1.f : 0.f)) * g);
  }
}

}  // namespace

void cross_entropy_fwd(DType dt, const void* logits, int64_t ld, const int64_t* labels, float* loss,
                       float* lse, int64_t rows, int V, int64_t ignore_index, hipStream_t s) {
  if (rows == 0) return;
  if (dt == DType::BF16) {
    const int vec_ok = (ld % 8 == 0) && ((uintptr_t)logits % 16 == 0);
    hipLaunchKernelGGL(ce_fwd_kernel<bf16>, dim3((unsigned)rows), dim3(kNT), 0, s, (const bf16*)logits, ld,
                       labels, loss, lse, V, ignore_index, vec_ok);
  } else {
    const int vec_ok = (ld % 4 == 0) && ((uintptr_t)logits % 16 == 0);
    hipLaunchKernelGGL(ce_fwd_kernel<float>, dim3((unsigned)rows), dim3(kNT), 0, s, (const float*)logits, ld,
                       labels, loss, lse, V, ignore_index, vec_ok);
  }
}

void cross_entropy_bwd(DType dt, const void* logits, int64_t ld, const int64_t* labels,
                       const float* lse, const float* gscale, void* dlogits, int64_t ldd,
                       int64_t rows, int V, int64_t ignore_index, hipStream_t s) {
  if (rows == 0) return;
  if (dt == DType::BF16) {
    const int vec_ok = (ld % 8 == 0) && (ldd % 8 == 0) && ((uintptr_t)logits % 16 == 0) &&
                       ((uintptr_t)dlogits % 16 == 0);
    hipLaunchKernelGGL(ce_bwd_kernel<bf16>, dim3((unsigned)rows), dim3(kNT), 0, s, (const bf16*)logits, ld,
                       labels, lse, gscale, (bf16*)dlogits, ldd, V, ignore_index, vec_ok);
  } else {
    const int vec_ok = (ld % 4 == 0) && (ldd % 4 == 0) && ((uintptr_t)logits % 16 == 0) &&
                       ((uintptr_t)dlogits % 16 == 0);
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3((unsigned)rows), dim3(kNT), 0, s, (const float*)logits, ld,
                       labels, lse, gscale, (float*)dlogits, ldd, V, ignore_index, vec_ok);
  }
}

}  // namespace grt
