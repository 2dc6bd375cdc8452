// Elementwise / layout kernels for gfx950: SwiGLU, GELU(erf), RoPE, embedding-scale+PE, dropout.
//
// Reference roles: K-B08 SwiGLU and K-B06 RoPE of the Llama SFT path
// (reference ray-jobs/fine_tune_llama_ray.py:240), K-A02/K-A08 scale+PE / GELU / dropout of
// BasicLLM (reference ray-jobs/pytorch_llm_ray.py:57-105).
//
// All are HBM-bound: 16-byte vector accesses per lane (cdna_hip_programming.md Guideline 13),
// grid capped at 256 CUs x 8 workgroups and grid-strided (Guideline 11). RoPE reads the fused
// QKV projection output in place (row stride `ld`) and writes attention-ready q/k, so there is
// no transpose or split copy anywhere in the attention block.
#include <limits.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kNT = 256;
constexpr int kMaxGrid = 256 * 8;

inline unsigned grid_for(int64_t work) {
  int64_t g = (work + kNT - 1) / kNT;
  if (g > kMaxGrid) g = kMaxGrid;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Single-pass forms of the row-indexed elementwise kernels (RoPE at D = 128, plain SwiGLU): one work
// item per thread on a full grid with 32-bit index math, instead of a capped grid-stride loop whose
// 64-bit div / mod per item dominated the kernels' VALU. GRT_EW_FAST=0 / ew_set_fast(0) selects the
// grid-stride kernels (A/B switch); both give bitwise the same results.
int g_ew_fast = -1;
inline bool ew_fast() {
  if (g_ew_fast < 0) {
    const char* e = getenv("GRT_EW_FAST");
    g_ew_fast = e && e[0] == '0' ? 0 : 1;
  }
  return g_ew_fast != 0;
}
inline unsigned grid_full(int64_t work) { return (unsigned)((work + kNT - 1) / kNT); }

// ------------------------------- SwiGLU -------------------------------------
// gu: [rows, 2F] = [gate | up]; out = silu(gate) * up
template <typename T>
__global__ __launch_bounds__(kNT) void swiglu_fwd_kernel(const T* __restrict__ gu, T* __restrict__ out,
                                                         int64_t rows, int f, int64_t ldo) {
  constexpr int V = Vec16<T>::N;
  const int vpr = f / V;
  const int64_t total = rows * vpr;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t r = i / vpr;
    const int c = (int)(i - r * vpr) * V;
    float g[V], u[V], o[V];
    load16(gu + r * 2 * f + c, g);
    load16(gu + r * 2 * f + f + c, u);
#pragma unroll
    for (int k = 0; k < V; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
    store16(out + r * ldo + c, o);  // ldo > f: the row of a wider [x | LoRA h] buffer
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void swiglu_bwd_kernel(const T* __restrict__ gu, const T* __restrict__ dout,
                                                         T* __restrict__ dgu, int64_t rows, int f) {
  constexpr int V = Vec16<T>::N;
  const int vpr = f / V;
  const int64_t total = rows * vpr;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t r = i / vpr;
    const int c = (int)(i - r * vpr) * V;
    float g[V], u[V], d[V], dg[V], du[V];
    load16(gu + r * 2 * f + c, g);
    load16(gu + r * 2 * f + f + c, u);
    load16(dout + r * f + c, d);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float sg = sigmoidf_(g[k]);
      const float silu = g[k] * sg;
      du[k] = d[k] * silu;
      dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
    }
    store16(dgu + r * 2 * f + c, dg);
    store16(dgu + r * 2 * f + f + c, du);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void swiglu_fwd1_kernel(const T* __restrict__ gu, T* __restrict__ out, uint32_t total,
                                                          int f, int64_t ldo) {
  constexpr int V = Vec16<T>::N;
  const uint32_t i = blockIdx.x * kNT + threadIdx.x;
  if (i >= total) return;
  const uint32_t vpr = (uint32_t)(f / V), r = i / vpr;
  const int c = (int)(i - r * vpr) * V;
  float g[V], u[V], o[V];
  load16(gu + (int64_t)r * 2 * f + c, g);
  load16(gu + (int64_t)r * 2 * f + f + c, u);
#pragma unroll
  for (int k = 0; k < V; ++k) o[k] = g[k] * sigmoidf_(g[k]) * u[k];
  store16(out + (int64_t)r * ldo + c, o);
}

template <typename T>
__global__ __launch_bounds__(kNT) void swiglu_bwd1_kernel(const T* __restrict__ gu, const T* __restrict__ dout,
                                                          T* __restrict__ dgu, uint32_t total, int f) {
  constexpr int V = Vec16<T>::N;
  const uint32_t i = blockIdx.x * kNT + threadIdx.x;
  if (i >= total) return;
  const uint32_t vpr = (uint32_t)(f / V), r = i / vpr;
  const int c = (int)(i - r * vpr) * V;
  float g[V], u[V], d[V], dg[V], du[V];
  load16(gu + (int64_t)r * 2 * f + c, g);
  load16(gu + (int64_t)r * 2 * f + f + c, u);
  load16(dout + (int64_t)r * f + c, d);
#pragma unroll
  for (int k = 0; k < V; ++k) {  // same arithmetic as swiglu_bwd_kernel
    const float sg = sigmoidf_(g[k]);
    const float silu = g[k] * sg;
    du[k] = d[k] * silu;
    dg[k] = d[k] * u[k] * sg * (1.f + g[k] * (1.f - sg));
  }
  store16(dgu + (int64_t)r * 2 * f + c, dg);
  store16(dgu + (int64_t)r * 2 * f + f + c, du);
}

// ---------------- SwiGLU with the transposed copy for the weight gradient ---------------------
// The TN weight gradient of the down projection needs h^T (h = silu(gate) * up, [M, F]) and that of
// the gate/up projection needs dgu^T ([2F, M]). A separate transpose kernel re-reads what these
// kernels just wrote; here the producing kernel writes both layouts: one workgroup = 64 token rows x
// 128 columns, the row-major result stored directly and staged in an XOR-swizzled bf16 LDS image
// (16 chunks of 16 bytes per row) that gfx950's ds_read_b64_tr_b16 reads back transposed, stored as
// 16-byte row segments of the transposed output (the scheme of transpose.hip).
typedef __attribute__((address_space(3))) bf16x4 ew_lds_bf16x4_t;
__device__ __forceinline__ int ew_tswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int ew_toff(int row, int ch) { return row * 256 + 16 * (ch ^ ew_tswz(row)); }

// image [64 rows][128 cols] -> dst rows c0 + (0..127) (row stride ldt), columns r0 .. r0 + 63
__device__ __forceinline__ void ew_store_transposed(const char* img, bf16* __restrict__ dst, int64_t ldt, int64_t r0) {
  const int t = threadIdx.x, l16 = t & 15, grp = t >> 4;
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int pr = grp + 16 * pp;
    const int cb = 16 * (pr >> 2), rb = 16 * (pr & 3);
    bf16x4 q[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = rb + 4 * k + (l16 >> 2), col = cb + 4 * (l16 & 3);
      q[k] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((ew_lds_bf16x4_t*)(img + ew_toff(rr, col >> 3) + 8 * ((col >> 2) & 1)));
    }
    bf16* d = dst + (int64_t)(cb + l16) * ldt + r0 + rb;
    *reinterpret_cast<bf16x8*>(d) = __builtin_shufflevector(q[0], q[1], 0, 1, 2, 3, 4, 5, 6, 7);
    *reinterpret_cast<bf16x8*>(d + 8) = __builtin_shufflevector(q[2], q[3], 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// out [rows, f] (row stride ldo) and outT [f, rows]; rows % 64 == 0, f % 128 == 0
__global__ __launch_bounds__(256) void swiglu_fwd_t_kernel(const bf16* __restrict__ gu, bf16* __restrict__ out,
                                                           bf16* __restrict__ outT, int64_t rows, int f, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) char img[64 * 256];
  const int ncb = f / 128;
  const int64_t r0 = (int64_t)(blockIdx.x / ncb) * 64;
  const int c0 = (blockIdx.x % ncb) * 128;
  const int t = threadIdx.x, row = t >> 2;
  const bf16* src = gu + (r0 + row) * 2 * f + c0;
  bf16x8 gv[4], uv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // every load in flight before the math
    const int ch = (t & 3) + 4 * k;
    gv[k] = *reinterpret_cast<const bf16x8*>(src + ch * 8);
    uv[k] = *reinterpret_cast<const bf16x8*>(src + f + ch * 8);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = (t & 3) + 4 * k;
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float g = static_cast<float>(gv[k][j]), u = static_cast<float>(uv[k][j]);
      o[j] = static_cast<bf16>(g * sigmoidf_(g) * u);
    }
    *reinterpret_cast<bf16x8*>(out + (r0 + row) * ldo + c0 + ch * 8) = o;
    *reinterpret_cast<bf16x8*>(img + ew_toff(row, ch)) = o;
  }
  __syncthreads();
  ew_store_transposed(img, outT + (int64_t)c0 * rows, rows, r0);
}

// dgu [rows, 2f] and dguT [2f, rows]; rows % 64 == 0, f % 128 == 0
__global__ __launch_bounds__(256) void swiglu_bwd_t_kernel(const bf16* __restrict__ gu, const bf16* __restrict__ dout,
                                                           bf16* __restrict__ dgu, bf16* __restrict__ dguT,
                                                           int64_t rows, int f) {
  __shared__ __attribute__((aligned(16))) char img[2][64 * 256];
  const int ncb = f / 128;
  const int64_t r0 = (int64_t)(blockIdx.x / ncb) * 64;
  const int c0 = (blockIdx.x % ncb) * 128;
  const int t = threadIdx.x, row = t >> 2;
  const bf16* src = gu + (r0 + row) * 2 * f + c0;
  const bf16* dsrc = dout + (r0 + row) * f + c0;
  bf16x8 gv[4], uv[4], dv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = (t & 3) + 4 * k;
    gv[k] = *reinterpret_cast<const bf16x8*>(src + ch * 8);
    uv[k] = *reinterpret_cast<const bf16x8*>(src + f + ch * 8);
    dv[k] = *reinterpret_cast<const bf16x8*>(dsrc + ch * 8);
  }
  bf16* drow = dgu + (r0 + row) * 2 * f + c0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int ch = (t & 3) + 4 * k;
    bf16x8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // same arithmetic as swiglu_bwd_kernel
      const float g = static_cast<float>(gv[k][j]), u = static_cast<float>(uv[k][j]), d = static_cast<float>(dv[k][j]);
      const float sg = sigmoidf_(g);
      const float silu = g * sg;
      du[j] = static_cast<bf16>(d * silu);
      dg[j] = static_cast<bf16>(d * u * sg * (1.f + g * (1.f - sg)));
    }
    *reinterpret_cast<bf16x8*>(drow + ch * 8) = dg;
    *reinterpret_cast<bf16x8*>(drow + f + ch * 8) = du;
    *reinterpret_cast<bf16x8*>(img[0] + ew_toff(row, ch)) = dg;
    *reinterpret_cast<bf16x8*>(img[1] + ew_toff(row, ch)) = du;
  }
  __syncthreads();
  ew_store_transposed(img[0], dguT + (int64_t)c0 * rows, rows, r0);
  ew_store_transposed(img[1], dguT + (int64_t)(f + c0) * rows, rows, r0);
}

// ------------------------------- GELU (erf) ---------------------------------
template <typename T>
__global__ __launch_bounds__(kNT) void gelu_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t nv) {
  constexpr int V = Vec16<T>::N;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kNT) {
    float a[V];
    load16(x + i * V, a);
#pragma unroll
    for (int k = 0; k < V; ++k) a[k] = 0.5f * a[k] * (1.f + erff(a[k] * 0.70710678118654752f));
    store16(y + i * V, a);
  }
}
template <typename T>
__global__ __launch_bounds__(kNT) void gelu_bwd_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                       T* __restrict__ dx, int64_t nv) {
  constexpr int V = Vec16<T>::N;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kNT) {
    float a[V], g[V];
    load16(x + i * V, a);
    load16(dy + i * V, g);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const float cdf = 0.5f * (1.f + erff(a[k] * 0.70710678118654752f));
      const float pdf = 0.3989422804014327f * __expf(-0.5f * a[k] * a[k]);
      g[k] *= cdf + a[k] * pdf;
    }
    store16(dx + i * V, g);
  }
}

// ------------------------------- RoPE ---------------------------------------
// One thread = 8 rotation pairs (i .. i+7 with partners i+D/2 ..) of one (token, head).
template <typename T, bool FWD>
__global__ __launch_bounds__(kNT) void rope_kernel(const T* __restrict__ src_q, const T* __restrict__ src_k,
                                                   int64_t src_ld_q, int64_t src_ld_k,
                                                   T* __restrict__ dst_q, T* __restrict__ dst_k,
                                                   int64_t dst_ld_q, int64_t dst_ld_k,
                                                   const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                   const int32_t* __restrict__ pos, int64_t T_, int S,
                                                   int hq, int hkv, int D) {
  const int half = D / 2;
  const int gpp = half / 8;                 // 8-pair groups per head
  const int heads = hq + hkv;
  const int64_t total = T_ * heads * gpp;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int g = (int)(i % gpp);
    const int64_t th = i / gpp;
    const int h = (int)(th % heads);
    const int64_t t = th / heads;
    const int p = pos ? pos[t] : (int)(t % S);
    const T* src;
    T* dst;
    if (h < hq) {
      src = src_q + t * src_ld_q + (int64_t)h * D;
      dst = dst_q + t * dst_ld_q + (int64_t)h * D;
    } else {
      src = src_k + t * src_ld_k + (int64_t)(h - hq) * D;
      dst = dst_k + t * dst_ld_k + (int64_t)(h - hq) * D;
    }
    const int c = g * 8;
    float x1[8], x2[8], cs[8], sn[8], o1[8], o2[8];
    if constexpr (Vec16<T>::N == 8) {
      load16(src + c, x1);
      load16(src + half + c, x2);
    } else {
      load16(src + c, x1); load16(src + c + 4, x1 + 4);
      load16(src + half + c, x2); load16(src + half + c + 4, x2 + 4);
    }
    load16(cosb + (int64_t)p * half + c, cs); load16(cosb + (int64_t)p * half + c + 4, cs + 4);
    load16(sinb + (int64_t)p * half + c, sn); load16(sinb + (int64_t)p * half + c + 4, sn + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float s = FWD ? sn[k] : -sn[k];
      o1[k] = x1[k] * cs[k] - x2[k] * s;
      o2[k] = x2[k] * cs[k] + x1[k] * s;
    }
    if constexpr (Vec16<T>::N == 8) {
      store16(dst + c, o1);
      store16(dst + half + c, o2);
    } else {
      store16(dst + c, o1); store16(dst + c + 4, o1 + 4);
      store16(dst + half + c, o2); store16(dst + half + c + 4, o2 + 4);
    }
  }
}

// D = 128 (every Llama head): one thread per 8-pair group with 32-bit index math and compile-time
// group count (the generic kernel's 64-bit div / mod per item were the bulk of its VALU), one group
// per thread on a full grid so every thread's six loads are in flight together.
template <typename T, bool FWD>
__global__ __launch_bounds__(kNT) void rope128_kernel(const T* __restrict__ src_q, const T* __restrict__ src_k,
                                                      int64_t src_ld_q, int64_t src_ld_k,
                                                      T* __restrict__ dst_q, T* __restrict__ dst_k,
                                                      int64_t dst_ld_q, int64_t dst_ld_k,
                                                      const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                      const int32_t* __restrict__ pos, uint32_t total, int S,
                                                      int hq, int hkv) {
  constexpr int D = 128, half = 64;
  const uint32_t i = blockIdx.x * kNT + threadIdx.x;
  if (i >= total) return;
  const uint32_t heads = (uint32_t)(hq + hkv);
  const uint32_t th = i >> 3, t = th / heads, h = th - t * heads;
  const int c = (int)(i & 7) * 8;
  const int p = pos ? pos[t] : (int)(t % (uint32_t)S);
  const T* src = h < (uint32_t)hq ? src_q + (int64_t)t * src_ld_q + (int64_t)h * D
                                  : src_k + (int64_t)t * src_ld_k + (int64_t)(h - hq) * D;
  T* dst = h < (uint32_t)hq ? dst_q + (int64_t)t * dst_ld_q + (int64_t)h * D
                            : dst_k + (int64_t)t * dst_ld_k + (int64_t)(h - hq) * D;
  float x1[8], x2[8], cs[8], sn[8], o1[8], o2[8];
  if constexpr (Vec16<T>::N == 8) {
    load16(src + c, x1);
    load16(src + half + c, x2);
  } else {
    load16(src + c, x1); load16(src + c + 4, x1 + 4);
    load16(src + half + c, x2); load16(src + half + c + 4, x2 + 4);
  }
  const float* cr = cosb + (int64_t)p * half + c;
  const float* sr = sinb + (int64_t)p * half + c;
  load16(cr, cs); load16(cr + 4, cs + 4);
  load16(sr, sn); load16(sr + 4, sn + 4);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float s2 = FWD ? sn[k] : -sn[k];
    o1[k] = x1[k] * cs[k] - x2[k] * s2;
    o2[k] = x2[k] * cs[k] + x1[k] * s2;
  }
  if constexpr (Vec16<T>::N == 8) {
    store16(dst + c, o1);
    store16(dst + half + c, o2);
  } else {
    store16(dst + c, o1); store16(dst + c + 4, o1 + 4);
    store16(dst + half + c, o2); store16(dst + half + c + 4, o2 + 4);
  }
}


// ------------------------- decode: RoPE + KV-cache append ------------------
// The cached-decode step's q / k rotation and the cache writes in one launch: token t (batch row
// t / tpr) at position pos[t] has its q heads rotated into q_out and its rotated k heads and raw v
// heads written at cache slot pos[t] of kc / vc ([B, L, Hkv, D] with strides). A token whose position
// is outside the rope table or the cache is skipped entirely (no write), so a bad position cannot
// write out of bounds.
template <typename T>
__global__ __launch_bounds__(kNT) void rope_append_kernel(const T* __restrict__ qkv, int64_t ld, T* __restrict__ q_out,
                                                          T* __restrict__ kc, T* __restrict__ vc, int64_t c_bs,
                                                          int64_t c_ss, int64_t c_hs, int64_t v_bs, int64_t v_ss,
                                                          int64_t v_hs, const float* __restrict__ cosb,
                                                          const float* __restrict__ sinb, const int32_t* __restrict__ pos,
                                                          int64_t T_, int tpr, int S, int L, int hq, int hkv, int D) {
  const int half = D / 2;
  const int gpp = half / 8;
  const int heads = hq + 2 * hkv;
  const int64_t total = T_ * heads * gpp;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int g = (int)(i % gpp);
    const int64_t th = i / gpp;
    const int h = (int)(th % heads);
    const int64_t t = th / heads;
    const int p = pos[t];
    if (p < 0 || p >= S || p >= L) continue;
    const int64_t b = t / tpr;
    const T* src = qkv + t * ld + (int64_t)h * D;
    const int c = g * 8;
    float x1[8], x2[8], o1[8], o2[8];
    load16(src + c, x1);
    load16(src + half + c, x2);
    T* dst;
    if (h < hq + hkv) {
      float cs[8], sn[8];
      load16(cosb + (int64_t)p * half + c, cs); load16(cosb + (int64_t)p * half + c + 4, cs + 4);
      load16(sinb + (int64_t)p * half + c, sn); load16(sinb + (int64_t)p * half + c + 4, sn + 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o1[k] = x1[k] * cs[k] - x2[k] * sn[k];
        o2[k] = x2[k] * cs[k] + x1[k] * sn[k];
      }
      dst = h < hq ? q_out + (t * hq + h) * (int64_t)D : kc + b * c_bs + (int64_t)p * c_ss + (int64_t)(h - hq) * c_hs;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) { o1[k] = x1[k]; o2[k] = x2[k]; }
      dst = vc + b * v_bs + (int64_t)p * v_ss + (int64_t)(h - hq - hkv) * v_hs;
    }
    store16(dst + c, o1);
    store16(dst + half + c, o2);
  }
}

// ------------------------- embedding scale + sinusoidal PE ------------------
template <typename T>
__global__ __launch_bounds__(kNT) void scale_add_pe_kernel(const T* __restrict__ emb, const float* __restrict__ pe,
                                                           T* __restrict__ out, int64_t T_, int S, int d,
                                                           float scale) {
  constexpr int V = Vec16<T>::N;
  const int vpr = d / V;
  const int64_t total = T_ * vpr;
  for (int64_t i = (int64_t)blockIdx.x * kNT + threadIdx.x; i < total; i += (int64_t)gridDim.x * kNT) {
    const int64_t t = i / vpr;
    const int c = (int)(i - t * vpr) * V;
    float a[V];
    load16(emb + t * d + c, a);
    if (pe != nullptr) {
      float p[V];
      const float* pr = pe + (int64_t)(t % S) * d + c;
#pragma unroll
      for (int k = 0; k < V; k += 4) load16(pr + k, p + k);
#pragma unroll
      for (int k = 0; k < V; ++k) a[k] = a[k] * scale + p[k];
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) a[k] *= scale;
    }
    store16(out + t * d + c, a);
  }
}

// ------------------------------- dropout -------------------------------------
// keep-mask hash (hash_u64 / drop_thr / drop_keep): grt_common.h, shared with lora.hip
// V consecutive decisions from idx0; one hash per 4 elements when idx0 is 4-aligned
template <int V>
__device__ __forceinline__ void drop_keep_vec(uint64_t key, uint64_t idx0, uint32_t thr, bool (&keep)[V]) {
  static_assert(V % 4 == 0, "vector of whole 4-element groups");
  if ((idx0 & 3) == 0) {
#pragma unroll
    for (int q = 0; q < V / 4; ++q) {
      const uint64_t h = hash_u64(key ^ ((idx0 >> 2) + q));
#pragma unroll
      for (int j = 0; j < 4; ++j) keep[4 * q + j] = ((uint32_t)(h >> (16 * j)) & 0xffffu) >= thr;
    }
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k) keep[k] = drop_keep(key, idx0 + k, thr);
  }
}

template <typename T>
__global__ __launch_bounds__(kNT) void dropout_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ mask, int64_t n, float p,
                                                          uint64_t seed, uint64_t offset) {
  constexpr int V = Vec16<T>::N;
  const uint32_t thr = drop_thr(p);
  const float sc = 1.f / (1.f - p);
  const uint64_t key = hash_u64(seed);
  const int64_t nv = n / V;
  for (int64_t v = (int64_t)blockIdx.x * kNT + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kNT) {
    const int64_t i0 = v * V;
    float a[V];
    load16(x + i0, a);
    uint8_t mk[V];
    bool kp[V];
    drop_keep_vec<V>(key, offset + (uint64_t)i0, thr, kp);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      mk[k] = kp[k];
      a[k] = kp[k] ? a[k] * sc : 0.f;
    }
    store16(y + i0, a);
    if (mask) {
#pragma unroll
      for (int k = 0; k < V; ++k) mask[i0 + k] = mk[k];
    }
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    const bool keep = drop_keep(key, offset + (uint64_t)i, thr);
    if (mask) mask[i] = keep;
    y[i] = from_f<T>(keep ? to_f(x[i]) * sc : 0.f);
  }
}

// dx (+)= keep(i) ? dy * 1/(1-p) : 0 with keep from the stored mask (mask != null) or regenerated
// from (seed, offset)
template <typename T>
__global__ __launch_bounds__(kNT) void dropout_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ mask,
                                                          T* __restrict__ dx, int64_t n, float p, uint64_t seed,
                                                          uint64_t offset, int accumulate) {
  constexpr int V = Vec16<T>::N;
  const uint32_t thr = drop_thr(p);
  const float sc = 1.f / (1.f - p);
  const uint64_t key = hash_u64(seed);
  const int64_t nv = n / V;
  for (int64_t v = (int64_t)blockIdx.x * kNT + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kNT) {
    const int64_t i0 = v * V;
    float g[V], o[V];
    load16(dy + i0, g);
    if (accumulate) load16(dx + i0, o);
    bool kp[V];
    if (mask) {
#pragma unroll
      for (int k = 0; k < V; ++k) kp[k] = mask[i0 + k] != 0;
    } else {
      drop_keep_vec<V>(key, offset + (uint64_t)i0, thr, kp);
    }
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const bool keep = kp[k];
      const float d = keep ? g[k] * sc : 0.f;
      o[k] = accumulate ? o[k] + d : d;
    }
    store16(dx + i0, o);
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * kNT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kNT) {
    const bool keep = mask ? mask[i] != 0 : drop_keep(key, offset + (uint64_t)i, thr);
    const float d = keep ? to_f(dy[i]) * sc : 0.f;
    dx[i] = from_f<T>(accumulate ? to_f(dx[i]) + d : d);
  }
}

}  // namespace

#define GRT_DISPATCH(dt, KERNEL, ...)                                  \
  do {                                                                 \
    if ((dt) == DType::BF16) { KERNEL(bf16, __VA_ARGS__); }            \
    else { KERNEL(float, __VA_ARGS__); }                               \
  } while (0)

void swiglu_fwd(DType dt, const void* gu, void* out, int64_t rows, int f, hipStream_t s, int64_t ldo) {
  if (ldo <= 0) ldo = f;
  if (ew_fast() && rows * f / 4 < INT32_MAX) {
#define K(T, ...) hipLaunchKernelGGL(swiglu_fwd1_kernel<T>, dim3(grid_full(rows * f / Vec16<T>::N)), dim3(kNT), 0, s, \
      (const T*)gu, (T*)out, (uint32_t)(rows * f / Vec16<T>::N), f, ldo)
    GRT_DISPATCH(dt, K, 0);
#undef K
    return;
  }
#define K(T, ...) hipLaunchKernelGGL(swiglu_fwd_kernel<T>, dim3(grid_for(rows * f / Vec16<T>::N)), dim3(kNT), 0, s, (const T*)gu, (T*)out, rows, f, ldo)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void swiglu_bwd(DType dt, const void* gu, const void* dout, void* dgu, int64_t rows, int f, hipStream_t s) {
  if (ew_fast() && rows * f / 4 < INT32_MAX) {
#define K(T, ...) hipLaunchKernelGGL(swiglu_bwd1_kernel<T>, dim3(grid_full(rows * f / Vec16<T>::N)), dim3(kNT), 0, s, \
      (const T*)gu, (const T*)dout, (T*)dgu, (uint32_t)(rows * f / Vec16<T>::N), f)
    GRT_DISPATCH(dt, K, 0);
#undef K
    return;
  }
#define K(T, ...) hipLaunchKernelGGL(swiglu_bwd_kernel<T>, dim3(grid_for(rows * f / Vec16<T>::N)), dim3(kNT), 0, s, (const T*)gu, (const T*)dout, (T*)dgu, rows, f)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
bool swiglu_fwd_t(const void* gu, void* out, void* outT, int64_t rows, int f, hipStream_t s, int64_t ldo) {
  if (ldo <= 0) ldo = f;
  if (rows % 64 != 0 || f % 128 != 0 || ldo % 8 != 0 || rows / 64 * (f / 128) >= INT32_MAX) return false;
  hipLaunchKernelGGL(swiglu_fwd_t_kernel, dim3((unsigned)(rows / 64 * (f / 128))), dim3(256), 0, s,
                     (const bf16*)gu, (bf16*)out, (bf16*)outT, rows, f, ldo);
  return true;
}
bool swiglu_bwd_t(const void* gu, const void* dout, void* dgu, void* dguT, int64_t rows, int f, hipStream_t s) {
  if (rows % 64 != 0 || f % 128 != 0 || rows / 64 * (f / 128) >= INT32_MAX) return false;
  hipLaunchKernelGGL(swiglu_bwd_t_kernel, dim3((unsigned)(rows / 64 * (f / 128))), dim3(256), 0, s,
                     (const bf16*)gu, (const bf16*)dout, (bf16*)dgu, (bf16*)dguT, rows, f);
  return true;
}
void gelu_fwd(DType dt, const void* x, void* y, int64_t n, hipStream_t s) {
#define K(T, ...) hipLaunchKernelGGL(gelu_fwd_kernel<T>, dim3(grid_for(n / Vec16<T>::N)), dim3(kNT), 0, s, (const T*)x, (T*)y, n / Vec16<T>::N)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void gelu_bwd(DType dt, const void* x, const void* dy, void* dx, int64_t n, hipStream_t s) {
#define K(T, ...) hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3(grid_for(n / Vec16<T>::N)), dim3(kNT), 0, s, (const T*)x, (const T*)dy, (T*)dx, n / Vec16<T>::N)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void ew_set_fast(int on) { g_ew_fast = on ? 1 : 0; }
void rope_fwd(DType dt, const void* qkv, int64_t ld, void* q_out, void* k_out, const float* cos,
              const float* sin, const int32_t* pos, int64_t T_, int S, int hq, int hkv, int D,
              hipStream_t s) {
  const int64_t work = T_ * (hq + hkv) * (D / 16);
  if (D == 128 && work < INT32_MAX && ew_fast()) {
#define K(TY, ...) hipLaunchKernelGGL((rope128_kernel<TY, true>), dim3((unsigned)((work + kNT - 1) / kNT)), dim3(kNT), 0, s, \
      (const TY*)qkv, (const TY*)qkv + (int64_t)hq * D, ld, ld, (TY*)q_out, (TY*)k_out, (int64_t)hq * D, \
      (int64_t)hkv * D, cos, sin, pos, (uint32_t)work, S, hq, hkv)
    GRT_DISPATCH(dt, K, 0);
#undef K
    return;
  }
#define K(TY, ...) hipLaunchKernelGGL((rope_kernel<TY, true>), dim3(grid_for(work)), dim3(kNT), 0, s, \
      (const TY*)qkv, (const TY*)qkv + (int64_t)hq * D, ld, ld, (TY*)q_out, (TY*)k_out, (int64_t)hq * D, \
      (int64_t)hkv * D, cos, sin, pos, T_, S, hq, hkv, D)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void rope_append(const void* qkv, int64_t ld, void* q_out, void* kc, void* vc, int64_t c_bs, int64_t c_ss,
                 int64_t c_hs, int64_t v_bs, int64_t v_ss, int64_t v_hs, const float* cos, const float* sin,
                 const int32_t* pos, int64_t T_, int tpr, int S, int L, int hq, int hkv, int D, hipStream_t s) {
  const int64_t work = T_ * (hq + 2 * hkv) * (D / 16);
  hipLaunchKernelGGL(rope_append_kernel<bf16>, dim3(grid_for(work)), dim3(kNT), 0, s, (const bf16*)qkv, ld,
                     (bf16*)q_out, (bf16*)kc, (bf16*)vc, c_bs, c_ss, c_hs, v_bs, v_ss, v_hs, cos, sin, pos, T_, tpr,
                     S, L, hq, hkv, D);
}
void rope_bwd(DType dt, const void* dq, const void* dk, void* dqkv, int64_t ld, const float* cos,
              const float* sin, const int32_t* pos, int64_t T_, int S, int hq, int hkv, int D,
              hipStream_t s) {
  const int64_t work = T_ * (hq + hkv) * (D / 16);
  if (D == 128 && work < INT32_MAX && ew_fast()) {
#define K(TY, ...) hipLaunchKernelGGL((rope128_kernel<TY, false>), dim3((unsigned)((work + kNT - 1) / kNT)), dim3(kNT), 0, s, \
      (const TY*)dq, (const TY*)dk, (int64_t)hq * D, (int64_t)hkv * D, (TY*)dqkv, (TY*)dqkv + (int64_t)hq * D, \
      ld, ld, cos, sin, pos, (uint32_t)work, S, hq, hkv)
    GRT_DISPATCH(dt, K, 0);
#undef K
    return;
  }
#define K(TY, ...) hipLaunchKernelGGL((rope_kernel<TY, false>), dim3(grid_for(work)), dim3(kNT), 0, s, \
      (const TY*)dq, (const TY*)dk, (int64_t)hq * D, (int64_t)hkv * D, (TY*)dqkv, (TY*)dqkv + (int64_t)hq * D, \
      ld, ld, cos, sin, pos, T_, S, hq, hkv, D)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void scale_add_pe(DType dt, const void* emb, const float* pe, void* out, int64_t T_, int S, int d,
                  float scale, hipStream_t s) {
#define K(T, ...) hipLaunchKernelGGL(scale_add_pe_kernel<T>, dim3(grid_for(T_ * d / Vec16<T>::N)), dim3(kNT), 0, s, (const T*)emb, pe, (T*)out, T_, S, d, scale)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void dropout_fwd(DType dt, const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed,
                 uint64_t offset, hipStream_t s) {
#define K(T, ...) hipLaunchKernelGGL(dropout_fwd_kernel<T>, dim3(grid_for(n / Vec16<T>::N + 1)), dim3(kNT), 0, s, (const T*)x, (T*)y, mask, n, p, seed, offset)
  GRT_DISPATCH(dt, K, 0);
#undef K
}
void dropout_bwd(DType dt, const void* dy, const uint8_t* mask, void* dx, int64_t n, float p,
                 hipStream_t s, uint64_t seed, uint64_t offset, bool accumulate) {
#define K(T, ...) hipLaunchKernelGGL(dropout_bwd_kernel<T>, dim3(grid_for(n / Vec16<T>::N + 1)), dim3(kNT), 0, s, (const T*)dy, mask, (T*)dx, n, p, seed, offset, accumulate ? 1 : 0)
  GRT_DISPATCH(dt, K, 0);
#undef K
}

}  // namespace grt
