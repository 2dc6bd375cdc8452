// 4-bit NormalFloat (NF4) block quantisation for QLoRA on gfx950.
//
// Reference role: BitsAndBytesConfig(load_in_4bit, bnb_4bit_quant_type="nf4",
// compute_dtype=bf16) in the SFT job (reference ray-jobs/fine_tune_llama_ray.py:215-227,
// ray-jobs/fine_tune_config.json:9-11); SURVEY §2.6 K-B03 / K-B14.
//
// Format: blocks of `blocksize` (64) consecutive weights share one fp32 absmax; each weight is a
// 4-bit index into the 16-level NF4 code book (quantiles of N(0,1), QLoRA paper). Two codes
// per byte, element 2i in the high nibble. Dequantisation writes 16 bytes of bf16 per lane.
#include <limits.h>
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

__constant__ float kNF4[16] = {
    -1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
    -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
    0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f, 0.33791524171829224f,
    0.44070982933044434f, 0.5626170039176941f, 0.7229568362236023f, 1.0f};

__device__ __forceinline__ uint32_t nf4_code(float x) {
  // nearest code: midpoints between sorted levels
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 15; ++i) c += (x > 0.5f * (kNF4[i] + kNF4[i + 1])) ? 1u : 0u;
  return c;
}

// one lane = 2 consecutive weights; blocksize/2 lanes share an absmax (blocksize in {32,64,128})
template <typename T>
__global__ __launch_bounds__(256) void nf4_quant_kernel(const T* __restrict__ w, uint8_t* __restrict__ q,
                                                        float* __restrict__ absmax, int64_t n, int bs) {
  const int64_t pair = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = pair * 2;
  const float a = i < n ? to_f(w[i]) : 0.f;
  const float b = i + 1 < n ? to_f(w[i + 1]) : 0.f;
  float m = fmaxf(fabsf(a), fabsf(b));
  const int lanes = bs / 2;  // lanes per quant block, power of two <= 64
  for (int o = lanes / 2; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (i < n) {
    const float inv = m > 0.f ? 1.f / m : 0.f;
    q[pair] = (uint8_t)((nf4_code(a * inv) << 4) | nf4_code(b * inv));
    if ((threadIdx.x & (lanes - 1)) == 0) absmax[i / bs] = m;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void nf4_dequant_kernel(const uint8_t* __restrict__ q,
                                                          const float* __restrict__ absmax, T* __restrict__ w,
                                                          int64_t n, int bs) {
  // one lane = 8 weights (4 code bytes)
  const int64_t n8 = n / 8;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < n8; g += (int64_t)gridDim.x * 256) {
    const uint32_t codes = *reinterpret_cast<const uint32_t*>(q + g * 4);
    const float s = absmax[(g * 8) / bs];
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t byte = (codes >> (8 * k)) & 0xFF;
      o[2 * k] = kNF4[byte >> 4] * s;
      o[2 * k + 1] = kNF4[byte & 15] * s;
    }
    if constexpr (Vec16<T>::N == 8) {
      store16(w + g * 8, o);
    } else {
      store16(w + g * 8, o);
      store16(w + g * 8 + 4, o + 4);
    }
  }
}

// Transposing dequantisation for the input-gradient GEMM (dX = dY W runs as the TN GEMM on W^T):
// one workgroup = a 64 x 64 tile of W [rows][cols] (cols a multiple of 64, so each tile row is one
// 64-weight quant block: one absmax per tile row). Dequantised into an LDS tile (padded row), then
// written transposed as 16-byte row segments of W^T [cols][rows].
__global__ __launch_bounds__(256) void nf4_dequant_t_kernel(const uint8_t* __restrict__ q,
                                                            const float* __restrict__ absmax, bf16* __restrict__ wt,
                                                            int rows, int cols, int bs) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  {  // read: thread t -> tile row t/4, 16 consecutive codes (8 bytes)
    const int tr = t >> 2, tc = (t & 3) * 16;
    const int r = r0 + tr;
    if (r < rows) {
      const int64_t e = (int64_t)r * cols + c0 + tc;
      const uint2 codes = *reinterpret_cast<const uint2*>(q + e / 2);
      const float sc = absmax[e / bs];
      const uint32_t wds[2] = {codes.x, codes.y};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t byte = (wds[k >> 2] >> (8 * (k & 3))) & 0xFF;
        tile[tr][tc + 2 * k] = kNF4[byte >> 4] * sc;
        tile[tr][tc + 2 * k + 1] = kNF4[byte & 15] * sc;
      }
    }
  }
  __syncthreads();
  {  // write: thread t -> W^T row c0 + t/4, 16 consecutive entries (rows r0 + 16*(t&3) ...)
    const int oc = t >> 2, orr = (t & 3) * 16;
    float o[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = tile[orr + k][oc];
    bf16* dst = wt + (int64_t)(c0 + oc) * rows + r0 + orr;
    if (r0 + orr + 16 <= rows) {
      store16(dst, o);
      store16(dst + 8, o + 8);
    } else {
      for (int k = 0; k < 16 && r0 + orr + k < rows; ++k) dst[k] = static_cast<bf16>(o[k]);
    }
  }
}

// ---- bf16 dequantisation, v2 (the per-use path of QLoRA without the resident cache) ----------
// v1 above looks the codes up in __constant__ memory with lane-divergent indices: one vector
// memory load per weight. v2 maps a whole code BYTE to its two levels through a 256-entry float2
// table in LDS (one ds_read_b64 per two weights; one 2 KiB table, conflict-free broadcast reads).
// Blocksize 64 only (the QLoRA format): 16 or 32 consecutive weights of a lane share one absmax.
__device__ __forceinline__ void nf4_lut_init(float2* lut) {
  const int t = threadIdx.x;  // blockDim.x == 256
  lut[t] = make_float2(kNF4[t >> 4], kNF4[t & 15]);
  __syncthreads();
}
__device__ __forceinline__ void nf4_expand8(const float2* lut, uint32_t a, uint32_t b, float s, float* o) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float2 v = lut[((k < 4 ? a : b) >> (8 * (k & 3))) & 0xFF];
    o[2 * k] = v.x * s;
    o[2 * k + 1] = v.y * s;
  }
}

// W [rows][cols] into a row-strided destination (ldo >= cols: the head of the K-concatenated
// [W | B] buffer). One lane = 16 weights of one row.
__global__ __launch_bounds__(256) void nf4_dequant2_kernel(const uint8_t* __restrict__ q,
                                                           const float* __restrict__ absmax, bf16* __restrict__ w,
                                                           int rows, int cols, int64_t ldo) {
  __shared__ float2 lut[256];
  nf4_lut_init(lut);
  const uint32_t per_row = (uint32_t)cols / 16;
  const uint32_t total = (uint32_t)rows * per_row;
  for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < total; g += gridDim.x * 256u) {
    const uint32_t r = g / per_row, c = (g - r * per_row) * 16;
    const int64_t e = (int64_t)r * cols + c;
    const uint2 codes = *reinterpret_cast<const uint2*>(q + e / 2);
    const float sc = absmax[e >> 6];
    float o[16];
    nf4_expand8(lut, codes.x, codes.y, sc, o);
    bf16* d = w + (int64_t)r * ldo + c;
    store16(d, o);
    store16(d + 8, o + 8);
  }
}

// W^T: one workgroup = a 64 x 128 tile of W. Each thread dequantises 32 weights of one row (16
// code bytes, one absmax) into a bf16 LDS image (rows of 16 XOR-swizzled 16-byte chunks); the
// transposed tile leaves through gfx950's ds_read_b64_tr_b16 as 16-byte stores of W^T rows (the
// scheme of transpose.hip's transpose2_bf16_kernel).
__device__ __forceinline__ int nf4_tswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int nf4_toff(int row, int ch) { return row * 256 + 16 * (ch ^ nf4_tswz(row)); }
typedef __attribute__((address_space(3))) bf16x4 nf4_lds_bf16x4_t;

__global__ __launch_bounds__(256) void nf4_dequant_t2_kernel(const uint8_t* __restrict__ q,
                                                             const float* __restrict__ absmax, bf16* __restrict__ wt,
                                                             int rows, int cols) {
  __shared__ float2 lut[256];
  __shared__ __attribute__((aligned(16))) char img[64 * 256];
  nf4_lut_init(lut);
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 128;
  const int t = threadIdx.x, lane = t & 63, l16 = lane & 15;
  {
    const int row = t >> 2, part = t & 3;
    const int64_t e = (int64_t)(r0 + row) * cols + c0 + part * 32;
    const uint4 codes = *reinterpret_cast<const uint4*>(q + e / 2);
    const float sc = absmax[e >> 6];
    float o[32];
    nf4_expand8(lut, codes.x, codes.y, sc, o);
    nf4_expand8(lut, codes.z, codes.w, sc, o + 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = static_cast<bf16>(o[8 * k + j]);
      *reinterpret_cast<bf16x8*>(img + nf4_toff(row, part * 4 + k)) = v;
    }
  }
  __syncthreads();
  const int grp = t >> 4;  // 16 groups; group g handles (column block, row block) pairs g and g + 16
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const int pr = grp + 16 * pp;
    const int cb = 16 * (pr >> 2), rb = 16 * (pr & 3);
    bf16x4 qv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rr = rb + 4 * k + (l16 >> 2), col = cb + 4 * (l16 & 3);
      const char* a = img + nf4_toff(rr, col >> 3) + 8 * ((col >> 2) & 1);
      qv[k] = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((nf4_lds_bf16x4_t*)a);
    }
    const bf16x8 o0 = __builtin_shufflevector(qv[0], qv[1], 0, 1, 2, 3, 4, 5, 6, 7);
    const bf16x8 o1 = __builtin_shufflevector(qv[2], qv[3], 0, 1, 2, 3, 4, 5, 6, 7);
    bf16* d = wt + (int64_t)(c0 + cb + l16) * rows + r0 + rb;
    *reinterpret_cast<bf16x8*>(d) = o0;
    *reinterpret_cast<bf16x8*>(d + 8) = o1;
  }
}

int nf4_version() {
  static const int v = [] { const char* e = getenv("GRT_NF4_DEQUANT_V1"); return e && atoi(e) == 1 ? 1 : 2; }();
  return v;
}

}  // namespace

bool nf4_dequantize_2d(const uint8_t* q, const float* absmax, void* w, int rows, int cols, int64_t ldo,
                       int blocksize, hipStream_t s) {
  if (blocksize != 64 || cols % 16 != 0 || (int64_t)rows * (cols / 16) >= (int64_t)INT32_MAX || rows < 1)
    return false;
  int64_t g = ((int64_t)rows * (cols / 16) + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(nf4_dequant2_kernel, dim3((unsigned)g), dim3(256), 0, s, q, absmax, (bf16*)w, rows, cols, ldo);
  return true;
}

void nf4_dequantize_t(const uint8_t* q, const float* absmax, void* wt, int rows, int cols, int blocksize,
                      hipStream_t s) {
  if (nf4_version() == 2 && blocksize == 64 && rows % 64 == 0 && cols % 128 == 0) {
    const dim3 grid((unsigned)(cols / 128), (unsigned)(rows / 64));
    hipLaunchKernelGGL(nf4_dequant_t2_kernel, grid, dim3(256), 0, s, q, absmax, (bf16*)wt, rows, cols);
    return;
  }
  const dim3 grid((unsigned)(cols / 64), (unsigned)((rows + 63) / 64));
  hipLaunchKernelGGL(nf4_dequant_t_kernel, grid, dim3(256), 0, s, q, absmax, (bf16*)wt, rows, cols, blocksize);
}

void nf4_quantize(DType dt, const void* w, uint8_t* q, float* absmax, int64_t n, int blocksize, hipStream_t s) {
  const unsigned grid = (unsigned)((n / 2 + 255) / 256);
  if (dt == DType::BF16)
    hipLaunchKernelGGL(nf4_quant_kernel<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)w, q, absmax, n, blocksize);
  else
    hipLaunchKernelGGL(nf4_quant_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)w, q, absmax, n, blocksize);
}

void nf4_dequantize(DType dt, const uint8_t* q, const float* absmax, void* w, int64_t n, int blocksize,
                    hipStream_t s) {
  if (dt == DType::BF16 && nf4_version() == 2 && n < INT32_MAX && reinterpret_cast<uintptr_t>(w) % 16 == 0 &&
      nf4_dequantize_2d(q, absmax, w, 1, (int)n, n, blocksize, s))
    return;
  int64_t g = (n / 8 + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  if (dt == DType::BF16)
    hipLaunchKernelGGL(nf4_dequant_kernel<bf16>, dim3((unsigned)g), dim3(256), 0, s, q, absmax, (bf16*)w, n, blocksize);
  else
    hipLaunchKernelGGL(nf4_dequant_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, q, absmax, (float*)w, n, blocksize);
}

}  // namespace grt
