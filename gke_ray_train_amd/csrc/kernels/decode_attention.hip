// Split-K attention for the decode step (one new query token per sequence), bf16, head_dim 128.
//
// Reference role: the KV-cache decode of HF ``generate`` in the inference comparison
// (reference ray-jobs/fine_tune_llama_ray.py:138-146). With Sq = 1 the
// training flash kernel runs one workgroup per (batch, query head) that walks all cached keys in
// sequence — 32 workgroups for Llama-3.1-8B at batch 1, ~24 µs per layer. Here the cached keys of
// each (batch, kv head) are split over NS workgroups (grid ~512) that each produce a partial
// (max, sum, unnormalised output) for every query head of the GQA group; a second tiny kernel
// merges the NS partials (log-sum-exp combine) and writes bf16.
//
// Lane mapping: 16 lanes per key (8 of the 128 dims each, one 16-byte load of K and of V), 4 keys
// per wave per step, 16 keys per workgroup per step; the GQA group's query rows stay in registers
// (fp32). Partial states of the 4 key-lane-groups of a wave merge with shuffles, the 4 waves
// through LDS. Empty splits (keys beyond the valid length) emit max = -inf, sum = 0.
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int D = 128;
constexpr int kMaxG = 8;  // query heads per kv head handled per workgroup

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void cvt8(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

template <int G>
__global__ __launch_bounds__(256) void attn_decode_split_kernel(const AttnDecodeParams p) {
  __shared__ float sm_m[4][G], sm_l[4][G];
  __shared__ float sm_o[4][G][D];
  const int bh = blockIdx.x, split = blockIdx.y;
  const int b = bh / p.Hkv, hkv = bh % p.Hkv;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane >> 4, c = lane & 15;  // key lane-group, 16-byte chunk of the head dim
  int len = p.Sk;
  if (p.seqlens_k) len = min(len, p.seqlens_k[b]);
  const int per = ((len + p.NS - 1) / p.NS + 15) / 16 * 16;
  const int k0 = split * per, k1 = min(len, k0 + per);

  const bf16* Kb = (const bf16*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs + c * 8;
  const bf16* Vb = (const bf16*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs + c * 8;
  // the K / V stream is pipelined one step ahead, and its first loads are issued before the query
  // loads, so the two dependent round trips at the start overlap (most splits are 1-2 steps long)
  int j = k0 + wave * 4 + grp;
  u32x4 kraw{}, vraw{};
  if (j < k1) {
    kraw = *reinterpret_cast<const u32x4*>(Kb + (int64_t)j * p.k_ss);
    vraw = *reinterpret_cast<const u32x4*>(Vb + (int64_t)j * p.v_ss);
  }
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const bf16* qp = (const bf16*)p.q + (int64_t)b * p.q_bs + (int64_t)(hkv * G + g) * p.q_hs + c * 8;
    cvt8(*reinterpret_cast<const u32x4*>(qp), q[g]);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[g][i] *= p.scale_log2;  // scores in log2 units
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = 0.f;
  }
  for (; j < k1; j += 16) {
    float kf[8], vf[8];
    cvt8(kraw, kf);
    cvt8(vraw, vf);
    if (j + 16 < k1) {
      kraw = *reinterpret_cast<const u32x4*>(Kb + (int64_t)(j + 16) * p.k_ss);
      vraw = *reinterpret_cast<const u32x4*>(Vb + (int64_t)(j + 16) * p.v_ss);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s = fmaf(q[g][i], kf[i], s);
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
      const float mn = fmaxf(m[g], s);
      const float a = fast_exp2(m[g] - mn), e = fast_exp2(s - mn);
      l[g] = l[g] * a + e;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] = fmaf(o[g][i], a, e * vf[i]);
      m[g] = mn;
    }
  }
  // merge the 4 key lane-groups of the wave (lanes c, c+16, c+32, c+48 hold the same dims)
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {
      const float m2 = __shfl_xor(m[g], off, 64), l2 = __shfl_xor(l[g], off, 64);
      const float mn = fmaxf(m[g], m2);
      const float a = mn == -INFINITY ? 0.f : fast_exp2(m[g] - mn);
      const float a2 = mn == -INFINITY ? 0.f : fast_exp2(m2 - mn);
      l[g] = l[g] * a + l2 * a2;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] = o[g][i] * a + __shfl_xor(o[g][i], off, 64) * a2;
      m[g] = mn;
    }
    if (grp == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) sm_o[wave][g][c * 8 + i] = o[g][i];
      if (c == 0) { sm_m[wave][g] = m[g]; sm_l[wave][g] = l[g]; }
    }
  }
  __syncthreads();
  // merge the 4 waves: thread t handles (g, d) pairs
  for (int idx = threadIdx.x; idx < G * D; idx += 256) {
    const int g = idx / D, d = idx % D;
    float mm = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) mm = fmaxf(mm, sm_m[w][g]);
    float ll = 0.f, oo = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float a = mm == -INFINITY ? 0.f : fast_exp2(sm_m[w][g] - mm);
      ll += sm_l[w][g] * a;
      oo += sm_o[w][g][d] * a;
    }
    const int64_t slot = ((int64_t)(b * p.Hq + hkv * G + g) * p.NS + split);
    p.part_o[slot * D + d] = oo;
    if (d == 0) { p.part_m[slot] = mm; p.part_l[slot] = ll; }
  }
}

// One workgroup per (batch, query head), one thread per head dim. The NS <= 64 partial states are
// loaded by the lanes of wave 0 in parallel (max / weight / sum by butterflies, weights to LDS),
// then every thread sums its dimension over the splits with independent loads — two dependent
// round trips instead of a serial NS-long chain.
__global__ __launch_bounds__(128) void attn_decode_combine_kernel(const AttnDecodeParams p) {
  __shared__ float wts[64];
  __shared__ float lsum;
  const int bhq = blockIdx.x, d = threadIdx.x;
  const int b = bhq / p.Hq, hq = bhq % p.Hq;
  const int64_t base = (int64_t)bhq * p.NS;
  if (threadIdx.x < 64) {
    const int s = threadIdx.x;
    const bool ok = s < p.NS;
    const float ms = ok ? p.part_m[base + s] : -INFINITY;
    const float ls = ok ? p.part_l[base + s] : 0.f;
    float mm = ms;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) mm = fmaxf(mm, __shfl_xor(mm, off, 64));
    const float a = (mm == -INFINITY || !ok) ? 0.f : fast_exp2(ms - mm);
    float ll = ls * a;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) ll += __shfl_xor(ll, off, 64);
    wts[s] = a;
    if (s == 0) lsum = ll;
  }
  __syncthreads();
  const float* po = p.part_o + base * D + d;
  float oo = 0.f;
#pragma unroll 8
  for (int s = 0; s < p.NS; ++s) oo = fmaf(po[(int64_t)s * D], wts[s], oo);
  const float ll = lsum;
  bf16* op = (bf16*)p.o + (int64_t)b * p.o_bs + (int64_t)hq * p.o_hs + d;
  *op = static_cast<bf16>(ll > 0.f ? oo / ll : 0.f);
}

}  // namespace

int attn_decode_splits(int B, int Hkv, int Sk) {
  int ns = (512 + B * Hkv - 1) / (B * Hkv);
  const int max_ns = (Sk + 15) / 16;
  if (ns > max_ns) ns = max_ns;
  if (ns > 64) ns = 64;
  return ns < 1 ? 1 : ns;
}

void attn_decode(const AttnDecodeParams& p, hipStream_t s) {
  const dim3 g1((unsigned)(p.B * p.Hkv), (unsigned)p.NS);
  const int G = p.Hq / p.Hkv;
  switch (G) {
    case 1: hipLaunchKernelGGL(attn_decode_split_kernel<1>, g1, dim3(256), 0, s, p); break;
    case 2: hipLaunchKernelGGL(attn_decode_split_kernel<2>, g1, dim3(256), 0, s, p); break;
    case 4: hipLaunchKernelGGL(attn_decode_split_kernel<4>, g1, dim3(256), 0, s, p); break;
    default: hipLaunchKernelGGL(attn_decode_split_kernel<8>, g1, dim3(256), 0, s, p); break;
  }
  hipLaunchKernelGGL(attn_decode_combine_kernel, dim3((unsigned)(p.B * p.Hq)), dim3(D), 0, s, p);
}

}  // namespace grt
