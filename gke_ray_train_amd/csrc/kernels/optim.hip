// Fused optimizer kernels for gfx950: global grad-norm (clip_grad_norm_) and AdamW.
//
// Reference roles: torch.nn.utils.clip_grad_norm_(…, 1.0) + torch.optim.AdamW(wd=0.01) in the
// BasicLLM hot loop (reference ray-jobs/pytorch_llm_ray.py:236,277-278), and
// max_grad_norm=0.3 + paged_adamw_32bit in SFT (ray-jobs/fine_tune_config.json:17,19).
// SURVEY §2.6 K-A12/K-A13, K-B11/K-B12.
//
// Design: the data-parallel engines keep parameters and gradients in flat buckets, so the whole
// optimizer step is TWO passes over HBM for any model size:
//   1. sum-of-squares of the flat gradient (one fp32 partial per workgroup, no atomics),
//      finalised on device into [norm, clip_coef] — no host synchronisation, graph-capturable;
//   2. one fused AdamW pass reading p, g, m, v (+fp32 master) once and writing p, m, v once,
//      with the clip coefficient read from device memory.
// Hyper-parameters come from a small device array so lr schedules do not bake into a captured
// hipGraph. Optimizer state is always fp32 ("32-bit" AdamW); params may be bf16 or fp32.
#include <cstdlib>

#include <algorithm>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kNT = 256;
constexpr int kSumBlocks = 1024;

template <typename T, int U>
__global__ __launch_bounds__(kNT) void sumsq_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ out) {
  __shared__ float red[kNT / kWave];
  constexpr int V = Vec16<T>::N;
  const int64_t nv = n / V;
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * kNT;
  int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x;
  // U independent 16-byte loads in flight per lane (one per iteration leaves each wave waiting a full
  // HBM latency per 1 KiB). Default U = 2: 6.1 TB/s isolated vs 5.7 (U = 4) and 5.6 (U = 1), and the
  // fastest headline step of the three (scripts/r6/sumsq.sh); GRT_SUMSQ_UNROLL=0 / 4 -> U = 1 / 4
  if constexpr (U > 1) {
    float accu[U];
#pragma unroll
    for (int u = 0; u < U; ++u) accu[u] = 0.f;
    for (; i + (U - 1) * stride < nv; i += U * stride) {
      float a[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) load16(x + (i + u * stride) * V, a[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int k = 0; k < V; ++k) accu[u] += a[u][k] * a[u][k];
    }
    if constexpr (U == 4) acc = (accu[0] + accu[1]) + (accu[2] + accu[3]);
    else acc = accu[0] + accu[1];
  }
  for (; i < nv; i += stride) {
    float a[V];
    load16(x + i * V, a);
#pragma unroll
    for (int k = 0; k < V; ++k) acc += a[k] * a[k];
  }
  for (int64_t j = nv * V + (int64_t)blockIdx.x * kNT + threadIdx.x; j < n; j += stride) {
    const float a = to_f(x[j]);
    acc += a * a;
  }
  acc = block_sum<kNT>(acc, red);
  if (threadIdx.x == 0) out[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kNT) void clip_finalize_kernel(const float* __restrict__ ws, int nparts,
                                                            float max_norm, float prescale,
                                                            float* __restrict__ out) {
  __shared__ float red[kNT / kWave];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kNT) acc += ws[i];
  acc = block_sum<kNT>(acc, red);
  if (threadIdx.x == 0) {
    // prescale folds the data-parallel 1/world average into the same coefficient, so the
    // reducer can all-reduce with SUM and no separate averaging pass ever touches the grads.
    const float norm = sqrtf(acc) * prescale;
    out[0] = norm;
    out[1] = ((max_norm > 0.f) ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f) * prescale;
  }
}

// fp32 -> bf16 with stochastic rounding: add 16 random bits below the bf16 mantissa, truncate.
__device__ __forceinline__ bf16 sr_bf16(float x, uint32_t r16) {
  const uint32_t u = __float_as_uint(x);
  if ((u & 0x7f800000u) == 0x7f800000u) return static_cast<bf16>(x);  // inf / nan unchanged
  const uint32_t t = (u + r16) & 0xffff0000u;
  return static_cast<bf16>(__uint_as_float(t));  // exact: the low 16 bits are zero
}

// One AdamW element update with its fused multiply-adds spelled out, so every kernel variant (8- /
// 4-wide, scalar tail, transposing) rounds identically whatever the compiler would contract.
// FAST (default; GRT_ADAMW_FASTMATH=0 -> the IEEE forms): v_sqrt_f32 and v_rcp_f32 (1 ulp each)
// instead of the correctly rounded sqrtf / division, whose expansions (denormal scaling, div_scale /
// div_fmas / div_fixup) made up over a third of the kernel's ~57 VALU instructions per element. The
// step is power-capped (1.39 kW on every sample of the headline step, profiles/r6_power.md), so the
// update's instruction energy beside the forward costs step time even though the pass is HBM-bound.
template <bool FAST>
__device__ __forceinline__ float adam_elem(float p, float gf, float& m, float& v, float b1, float b2, float rbc2,
                                           float eps, float decay, float step) {
  m = fmaf(b1, m, (1.f - b1) * gf);
  v = fmaf(b2, v, (1.f - b2) * gf * gf);
  if constexpr (FAST) {
    const float denom = fmaf(__builtin_amdgcn_sqrtf(v), rbc2, eps);
    return fmaf(-step * m, __builtin_amdgcn_rcpf(denom), p * decay);
  } else {
    const float denom = fmaf(sqrtf(v), rbc2, eps);
    return fmaf(p, decay, -(step * m / denom));
  }
}

// 16 random bits per element for stochastic rounding, 4 elements at a time (element base4 + k in
// bits 16k .. 16k + 15), keyed by (step, flat element index): FAST = one 32-bit fmix per element
// pair; otherwise one 64-bit splitmix per 4 elements.
__device__ __forceinline__ uint32_t fmix32_o(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
template <bool FAST>
__device__ __forceinline__ uint64_t sr_bits4(uint64_t srkey, uint64_t base4) {
  if constexpr (FAST) {
    const uint64_t pr = base4 >> 1;
    const uint32_t k = (uint32_t)srkey ^ ((uint32_t)(pr >> 32) * 0x9E3779B1u);
    return (uint64_t)fmix32_o(k ^ (uint32_t)pr) | ((uint64_t)fmix32_o(k ^ (uint32_t)(pr + 1)) << 32);
  } else {
    return hash_u64(srkey ^ (base4 >> 2));
  }
}

// V elements per thread and iteration: 8 (16-byte loads of bf16 p / g, two float4 of m / v; needs
// 16-byte aligned operands) or 4 (the fallback for 8-byte aligned bf16 slices).
template <typename P, typename G, int V, bool FAST>
__global__ __launch_bounds__(kNT) void adamw_kernel(P* __restrict__ p, const G* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    float* __restrict__ master, int64_t n,
                                                    const float* __restrict__ hyper,
                                                    const float* __restrict__ gsp, uint64_t ioff) {
  static_assert(V == 4 || V == 8, "V");
  constexpr int Q = V / 4;  // float4 groups per iteration
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float bc1 = hyper[5], bc2 = hyper[6];
  const float gs = hyper[7] * (gsp ? gsp[1] : 1.f);
  const float step = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  // bf16 parameters without an fp32 master copy: stochastic rounding of the updated value
  // (hyper[8] != 0; hyper[9] = step). Updates below half a bf16 ulp (lr 2e-5 on |w| ~ 1e-2) would
  // otherwise round away entirely; SR keeps every update in expectation.
  // The random bits are a hash of (step, element index + ioff), one 64-bit hash per 4 elements: a
  // launch over a slice of a flat buffer (the overlapped optimizer's per-module chunks) or with
  // another V rounds exactly like one over the whole.
  const bool sr = sizeof(P) == 2 && master == nullptr && hyper[8] != 0.f;
  const uint64_t srkey = hash_u64(0x5352ull ^ ((uint64_t)hyper[9] << 20));
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * kNT;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < nv; i += stride) {
    const int64_t o = i * V;
    f32x4 mv[Q], vv[Q];
    float pf[V], gf[V];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      mv[q] = *reinterpret_cast<const f32x4*>(m + o + 4 * q);
      vv[q] = *reinterpret_cast<const f32x4*>(v + o + 4 * q);
    }
    if (master) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(master + o + 4 * q);
#pragma unroll
        for (int k = 0; k < 4; ++k) pf[4 * q + k] = t[k];
      }
    } else if constexpr (sizeof(P) == 2) {
      if constexpr (V == 8) {
        const bf16x8 t = *reinterpret_cast<const bf16x8*>(p + o);
#pragma unroll
        for (int k = 0; k < 8; ++k) pf[k] = to_f(t[k]);
      } else {
        const bf16x4 t = *reinterpret_cast<const bf16x4*>(p + o);
#pragma unroll
        for (int k = 0; k < 4; ++k) pf[k] = to_f(t[k]);
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(p + o + 4 * q);
#pragma unroll
        for (int k = 0; k < 4; ++k) pf[4 * q + k] = t[k];
      }
    }
    if constexpr (sizeof(G) == 2) {
      if constexpr (V == 8) {
        const bf16x8 t = *reinterpret_cast<const bf16x8*>(g + o);
#pragma unroll
        for (int k = 0; k < 8; ++k) gf[k] = to_f(t[k]) * gs;
      } else {
        const bf16x4 t = *reinterpret_cast<const bf16x4*>(g + o);
#pragma unroll
        for (int k = 0; k < 4; ++k) gf[k] = to_f(t[k]) * gs;
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const f32x4 t = *reinterpret_cast<const f32x4*>(g + o + 4 * q);
#pragma unroll
        for (int k = 0; k < 4; ++k) gf[4 * q + k] = t[k] * gs;
      }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = 4 * q + k;
        float mk = mv[q][k], vk = vv[q][k];
        pf[e] = adam_elem<FAST>(pf[e], gf[e], mk, vk, b1, b2, rbc2, eps, decay, step);
        mv[q][k] = mk;
        vv[q][k] = vk;
      }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      *reinterpret_cast<f32x4*>(m + o + 4 * q) = mv[q];
      *reinterpret_cast<f32x4*>(v + o + 4 * q) = vv[q];
    }
    if (master) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        f32x4 t;
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = pf[4 * q + k];
        *reinterpret_cast<f32x4*>(master + o + 4 * q) = t;
      }
    }
    if constexpr (sizeof(P) == 2) {
      bf16 t[V];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (sr) {
          const uint64_t h = sr_bits4<FAST>(srkey, (ioff + (uint64_t)(o + 4 * q)) & ~3ull);
#pragma unroll
          for (int k = 0; k < 4; ++k) t[4 * q + k] = sr_bf16(pf[4 * q + k], (uint32_t)(h >> (16 * k)) & 0xffffu);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) t[4 * q + k] = from_f<bf16>(pf[4 * q + k]);
        }
      }
      if constexpr (V == 8) {
        bf16x8 tv;
#pragma unroll
        for (int k = 0; k < 8; ++k) tv[k] = t[k];
        *reinterpret_cast<bf16x8*>(p + o) = tv;
      } else {
        bf16x4 tv;
#pragma unroll
        for (int k = 0; k < 4; ++k) tv[k] = t[k];
        *reinterpret_cast<bf16x4*>(p + o) = tv;
      }
    } else {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        f32x4 t;
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = pf[4 * q + k];
        *reinterpret_cast<f32x4*>(p + o + 4 * q) = t;
      }
    }
  }
  // scalar tail (n % V)
  for (int64_t j = nv * V + (int64_t)blockIdx.x * kNT + threadIdx.x; j < n; j += stride) {
    float pf = master ? master[j] : to_f(p[j]);
    const float gf = to_f(g[j]) * gs;
    float mj = m[j], vj = v[j];
    pf = adam_elem<FAST>(pf, gf, mj, vj, b1, b2, rbc2, eps, decay, step);
    m[j] = mj;
    v[j] = vj;
    if (master) master[j] = pf;
    if constexpr (sizeof(P) == 2) {
      p[j] = sr ? sr_bf16(pf, (uint32_t)(sr_bits4<FAST>(srkey, (ioff + (uint64_t)j) & ~3ull) >> (16 * ((ioff + j) & 3))) & 0xffffu)
                : from_f<P>(pf);
    } else {
      p[j] = from_f<P>(pf);
    }
  }
}

// AdamW on one bf16 weight [rows][cols] (bf16 gradient, fp32 moments, no master copy) that also
// writes W^T [cols][rows] — the operand of the next backward's TN input-gradient GEMM (13-15 %
// faster than the NN form on the Llama shapes, profiles/r1_dgrad_layout_ab.jsonl) — so the
// transpose costs one extra 2-byte write per parameter inside a pass that is HBM-bound anyway.
// One workgroup = a 64 x 128 tile: 4 threads per 256-byte row segment, the updated tile staged in
// LDS and written back transposed with 32 B row segments. Same update, stochastic rounding and
// random stream (flat index ioff + row * cols + col) as adamw_kernel.
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_o;
__device__ __forceinline__ int oswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int ooff(int row, int ch) { return row * 256 + 16 * (ch ^ oswz(row)); }

// tile = 64 rows x 128 columns (cols % 128 == 0); the updated tile goes into the XOR-swizzled LDS
// image of transpose.hip and is read back transposed with ds_read_b64_tr_b16.
template <bool FAST>
__global__ __launch_bounds__(kNT) void adamw_t_kernel(bf16* __restrict__ p, const bf16* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      bf16* __restrict__ pt, int64_t rows, int64_t cols,
                                                      const float* __restrict__ hyper,
                                                      const float* __restrict__ gsp, uint64_t ioff) {
  __shared__ __attribute__((aligned(16))) char img[64 * 256];
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float bc1 = hyper[5], bc2 = hyper[6];
  const float gs = hyper[7] * (gsp ? gsp[1] : 1.f);
  const float step = lr / bc1;
  const float rbc2 = rsqrtf(bc2);
  const float decay = 1.f - lr * wd;
  const bool sr = hyper[8] != 0.f;
  const uint64_t srkey = hash_u64(0x5352ull ^ ((uint64_t)hyper[9] << 20));
  const int64_t ntc = cols / 128;
  const int64_t tr = blockIdx.x / ntc, tc = blockIdx.x % ntc;
  // 4 threads per 256-byte row; per k the 4 threads take 4 adjacent 16-byte chunks (coalesced)
  const int tid = threadIdx.x, row = tid >> 2;
  // every load of the thread's 4 chunks is issued before the first update (the compiler otherwise
  // serialises load -> update -> store per chunk: one chunk's 96 bytes in flight per thread)
  bf16x8 pva[4], gva[4];
  f32x4 mva[4][2], vva[4][2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t o = (tr * 64 + row) * cols + tc * 128 + ((tid & 3) + 4 * k) * 8;
    pva[k] = *reinterpret_cast<const bf16x8*>(p + o);
    gva[k] = *reinterpret_cast<const bf16x8*>(g + o);
    mva[k][0] = *reinterpret_cast<const f32x4*>(m + o);
    mva[k][1] = *reinterpret_cast<const f32x4*>(m + o + 4);
    vva[k][0] = *reinterpret_cast<const f32x4*>(v + o);
    vva[k][1] = *reinterpret_cast<const f32x4*>(v + o + 4);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = (tid & 3) + 4 * k;
    const int64_t o = (tr * 64 + row) * cols + tc * 128 + ch * 8;
    const bf16x8 pv = pva[k];
    const bf16x8 gv = gva[k];
    f32x4 mv[2] = {mva[k][0], mva[k][1]};
    f32x4 vv[2] = {vva[k][0], vva[k][1]};
    bf16x8 out;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const uint64_t hsh = sr_bits4<FAST>(srkey, (ioff + (uint64_t)o + 4 * hh) & ~3ull);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = 4 * hh + q;
        const float gf = to_f(gv[e]) * gs;
        float mq = mv[hh][q], vq = vv[hh][q];
        const float pf = adam_elem<FAST>(to_f(pv[e]), gf, mq, vq, b1, b2, rbc2, eps, decay, step);
        mv[hh][q] = mq;
        vv[hh][q] = vq;
        out[e] = sr ? sr_bf16(pf, (uint32_t)(hsh >> (16 * q)) & 0xffffu) : from_f<bf16>(pf);
      }
    }
    *reinterpret_cast<f32x4*>(m + o) = mv[0];
    *reinterpret_cast<f32x4*>(m + o + 4) = mv[1];
    *reinterpret_cast<f32x4*>(v + o) = vv[0];
    *reinterpret_cast<f32x4*>(v + o + 4) = vv[1];
    *reinterpret_cast<bf16x8*>(p + o) = out;
    *reinterpret_cast<bf16x8*>(img + ooff(row, ch)) = out;
  }
  __syncthreads();
  // W^T: lane i of a 16-lane group gets column cb + i of 4 rows per transposed read
  const int l16 = tid & 15, grp = tid >> 4;
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int pr = grp + 16 * pp;
    const int cb = 16 * (pr >> 2), rb = 16 * (pr & 3);
    bf16x4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = rb + 4 * k + (l16 >> 2), col = cb + 4 * (l16 & 3);
      q[k] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_o*)(img + ooff(rr, col >> 3) + 8 * ((col >> 2) & 1)));
    }
    bf16* d = pt + (tc * 128 + cb + l16) * rows + tr * 64 + rb;
    *reinterpret_cast<bf16x8*>(d) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    *reinterpret_cast<bf16x8*>(d + 8) = __builtin_shufflevector(q[2], q[3], 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void scale_kernel(T* __restrict__ x, int64_t n, float a,
                                                    const float* __restrict__ ap) {
  const float s = ap ? ap[0] : a;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT)
    x[i] = from_f<T>(to_f(x[i]) * s);
}

unsigned grid_for(int64_t work) {
  int64_t g = (work + kNT - 1) / kNT;
  if (g > 256 * 8) g = 256 * 8;
  return (unsigned)(g < 1 ? 1 : g);
}

}  // namespace

int optim_sumsq_blocks() { return kSumBlocks; }

void sumsq_accumulate(DType dt, const void* x, int64_t n, float* ws, int slot, hipStream_t s) {
  static const int unroll = [] {
    const char* e = std::getenv("GRT_SUMSQ_UNROLL");
    return e && e[0] == '0' ? 1 : e && e[0] == '4' ? 4 : 2;
  }();
  float* out = ws + (int64_t)slot * kSumBlocks;
  const dim3 g(kSumBlocks), b(kNT);
  if (dt == DType::BF16) {
    const bf16* xb = (const bf16*)x;
    if (unroll == 4) hipLaunchKernelGGL((sumsq_kernel<bf16, 4>), g, b, 0, s, xb, n, out);
    else if (unroll == 2) hipLaunchKernelGGL((sumsq_kernel<bf16, 2>), g, b, 0, s, xb, n, out);
    else hipLaunchKernelGGL((sumsq_kernel<bf16, 1>), g, b, 0, s, xb, n, out);
  } else {
    const float* xf = (const float*)x;
    if (unroll == 4) hipLaunchKernelGGL((sumsq_kernel<float, 4>), g, b, 0, s, xf, n, out);
    else if (unroll == 2) hipLaunchKernelGGL((sumsq_kernel<float, 2>), g, b, 0, s, xf, n, out);
    else hipLaunchKernelGGL((sumsq_kernel<float, 1>), g, b, 0, s, xf, n, out);
  }
}

void clip_coef_finalize(const float* ws, int nparts, float max_norm, float prescale, float* out,
                        hipStream_t s) {
  hipLaunchKernelGGL(clip_finalize_kernel, dim3(1), dim3(kNT), 0, s, ws, nparts, max_norm, prescale, out);
}

// GRT_ADAMW_FASTMATH=0: the IEEE sqrt / division and the 64-bit stochastic-rounding hash (A/B switch)
bool adamw_fastmath() {
  static const bool f = [] { const char* e = std::getenv("GRT_ADAMW_FASTMATH"); return !(e && e[0] == '0'); }();
  return f;
}

template <typename P, typename G, bool FAST>
void launch_adamw_v(dim3 grid, hipStream_t s, P* p, const G* g, float* m, float* v, float* master, int64_t n,
                    const float* hyper, const float* gsp, uint64_t ioff) {
  // GRT_ADAMW_V4=1: always the 4-wide variant (A/B switch)
  static const bool v4 = [] { const char* e = std::getenv("GRT_ADAMW_V4"); return e && e[0] == '1'; }();
  auto a16 = [](const void* q) { return q == nullptr || reinterpret_cast<uintptr_t>(q) % 16 == 0; };
  if (!v4 && a16(p) && a16(g) && a16(m) && a16(v) && a16(master))
    hipLaunchKernelGGL((adamw_kernel<P, G, 8, FAST>), grid, dim3(kNT), 0, s, p, g, m, v, master, n, hyper, gsp, ioff);
  else
    hipLaunchKernelGGL((adamw_kernel<P, G, 4, FAST>), grid, dim3(kNT), 0, s, p, g, m, v, master, n, hyper, gsp, ioff);
}

template <typename P, typename G>
void launch_adamw(dim3 grid, hipStream_t s, P* p, const G* g, float* m, float* v, float* master, int64_t n,
                  const float* hyper, const float* gsp, uint64_t ioff) {
  if (adamw_fastmath())
    launch_adamw_v<P, G, true>(grid, s, p, g, m, v, master, n, hyper, gsp, ioff);
  else
    launch_adamw_v<P, G, false>(grid, s, p, g, m, v, master, n, hyper, gsp, ioff);
}

void adamw_step(DType pdt, DType gdt, void* p, const void* g, float* m, float* v, float* master,
                int64_t n, const float* hyper, const float* gsp, hipStream_t s, int max_blocks, int64_t ioff) {
  // workgroup cap of the grid-strided update (GRT_ADAMW_GRID_CAP, default 256 CUs x 64): fewer
  // serial load -> update -> store iterations per thread. Isolated, Llama-2-7B shapes: 2048 ->
  // 16384 workgroups is qkv 222 -> 207 us, gate_up 396 -> 373, down 200 -> 183 (65536: no further
  // gain; scripts/gpu_adamw_ab.sh, profiles/r4_batch1.md)
  static const int64_t cap = [] {
    const char* e = std::getenv("GRT_ADAMW_GRID_CAP");
    const int64_t c = e ? std::atoll(e) : 256 * 64;
    return c > 0 ? c : (int64_t)256 * 64;
  }();
  int64_t nb64 = (n / 8 + 1 + kNT - 1) / kNT;
  if (nb64 > cap) nb64 = cap;
  unsigned nb = (unsigned)(nb64 < 1 ? 1 : nb64);
  if (max_blocks > 0 && nb > (unsigned)max_blocks) nb = (unsigned)max_blocks;
  const dim3 grid(nb);
  const uint64_t io = (uint64_t)ioff;
  if (pdt == DType::BF16 && gdt == DType::BF16)
    launch_adamw(grid, s, (bf16*)p, (const bf16*)g, m, v, master, n, hyper, gsp, io);
  else if (pdt == DType::BF16)
    launch_adamw(grid, s, (bf16*)p, (const float*)g, m, v, master, n, hyper, gsp, io);
  else if (gdt == DType::BF16)
    launch_adamw(grid, s, (float*)p, (const bf16*)g, m, v, master, n, hyper, gsp, io);
  else
    launch_adamw(grid, s, (float*)p, (const float*)g, m, v, master, n, hyper, gsp, io);
}

void adamw_t_step(void* p, const void* g, float* m, float* v, void* pt, int64_t rows, int64_t cols,
                  const float* hyper, const float* gsp, hipStream_t s, int64_t ioff) {
  const dim3 grid((unsigned)((rows / 64) * (cols / 128)));
  if (adamw_fastmath())
    hipLaunchKernelGGL(adamw_t_kernel<true>, grid, dim3(kNT), 0, s, (bf16*)p, (const bf16*)g, m, v, (bf16*)pt, rows,
                       cols, hyper, gsp, (uint64_t)ioff);
  else
    hipLaunchKernelGGL(adamw_t_kernel<false>, grid, dim3(kNT), 0, s, (bf16*)p, (const bf16*)g, m, v, (bf16*)pt, rows,
                       cols, hyper, gsp, (uint64_t)ioff);
}

void scale_inplace(DType dt, void* x, int64_t n, float a, const float* a_ptr, hipStream_t s) {
  if (dt == DType::BF16)
    hipLaunchKernelGGL(scale_kernel<bf16>, dim3(grid_for(n)), dim3(kNT), 0, s, (bf16*)x, n, a, a_ptr);
  else
    hipLaunchKernelGGL(scale_kernel<float>, dim3(grid_for(n)), dim3(kNT), 0, s, (float*)x, n, a, a_ptr);
}

}  // namespace grt
