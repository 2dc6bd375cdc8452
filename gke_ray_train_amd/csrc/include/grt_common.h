// Common device helpers for the gfx950 (CDNA4, MI355X) kernels of gke_ray_train_amd.
//
// Everything here is written for a 64-lane wavefront; no warp-32 idioms, no CUDA shims.
// bf16 is clang's native __bf16: a plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
// (round-to-nearest-even, NaN preserving), a widening cast is a 16-bit shift.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace grt {

constexpr int kWave = 64;

// Device-side bounds / invariant checks, compiled in only for the GRT_KERNEL_CHECKS=1 debugging
// build (python -m gke_ray_train_amd._build with that env var): a failed check traps the wave so
// the fault is reported at the offending kernel (rocprofv3 / dmesg) instead of corrupting memory.
#if defined(GRT_KERNEL_CHECKS) && GRT_KERNEL_CHECKS
#define GRT_DEVICE_CHECK(cond) \
  do {                         \
    if (!(cond)) __builtin_trap(); \
  } while (0)
#else
#define GRT_DEVICE_CHECK(cond) ((void)0)
#endif

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return static_cast<float>(x); }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return static_cast<bf16>(x); }

// 16-byte vector of T: 8 x bf16 or 4 x f32.
template <typename T> struct Vec16;
template <> struct Vec16<bf16> { typedef bf16x8 type; static constexpr int N = 8; };
template <> struct Vec16<float> { typedef f32x4 type; static constexpr int N = 4; };

template <typename T>
__device__ __forceinline__ void load16(const T* p, float* out) {
  typedef typename Vec16<T>::type V;
  V v = *reinterpret_cast<const V*>(p);
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) out[i] = to_f(v[i]);
}
template <typename T>
__device__ __forceinline__ void store16(T* p, const float* in) {
  typedef typename Vec16<T>::type V;
  V v;
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) v[i] = from_f<T>(in[i]);
  *reinterpret_cast<V*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t += red[i];
  __syncthreads();
  return t;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / kWave; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD (same private L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (orig >> 3);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// ---- element dropout keep-mask (elementwise.hip dropout kernels, lora.hip) ----
__device__ __forceinline__ uint64_t hash_u64(uint64_t x) {
  // splitmix64 finaliser: counter-based, stateless, graph-replay safe (seed/offset are args)
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// The keep decision of element idx is a pure function of (seed, idx), so a backward regenerates
// it instead of reading a stored mask: 16 bits of hash(key ^ (idx / 4)) against p in 1/65536
// units, key = hash(seed) (all 64 seed bits matter; computed once per thread). One hash per 4
// elements: the 64-bit multiplies of the hash are emulated with 32-bit ones on CDNA, and one hash
// per element made the kernel VALU-bound; per group it streams at memory speed. Keep probability
// 1 - round(p * 65536) / 65536. ops/_ref.py::dropout_keep_mask is the host reimplementation.
__device__ __forceinline__ uint32_t drop_thr(float p) { return (uint32_t)(p * 65536.0f + 0.5f); }
__device__ __forceinline__ bool drop_keep(uint64_t key, uint64_t idx, uint32_t thr) {
  const uint64_t h = hash_u64(key ^ (idx >> 2));
  return ((uint32_t)(h >> (16 * (idx & 3))) & 0xffffu) >= thr;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

}  // namespace grt

#define GRT_CHECK_LAUNCH() (void)hipGetLastError()
