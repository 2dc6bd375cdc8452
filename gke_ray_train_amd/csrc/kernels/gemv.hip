// Skinny GEMM (GEMV) for the decode step: y[m][n] = sum_k x[m][k] * W[n][k], m < M <= 4, bf16.
//
// Reference role: the per-token projections of HF ``generate`` in the post-training inference
// comparison (reference ray-jobs/fine_tune_llama_ray.py:138-146). With one to
// four tokens per step the projections are pure weight streams (an 8B model reads ~16 GB per
// token), so the kernel is built for HBM bandwidth, not MFMA: each wave owns R = 4 weight rows and
// streams them with 16-byte non-temporal loads (the weights are read once per token;
// MI355X_MICROARCH.md "nt-weights"), 4 rows x 16 B in flight per lane per K-step; the
// activations (M x K, a few KB) are re-read from L1/L2 by every wave. fp32 accumulation, one
// wave-wide butterfly reduction per (m, row), the 4 waves' K partials merged through LDS.
//
// The decode step's residual adds and RMSNorms live inside the GEMVs (no norm kernel, no launch
// and no dependent HBM round trip per norm — 65 per Llama-3.1-8B token):
//   * EPI_RESNORM (o_proj, down_proj): the epilogue writes h = bf16(y) + residual (the next
//     residual stream, rounded like torch) and adds each workgroup's sum of h^2 per row to one of
//     64 64-bit fixed-point accumulators (2^-20 units: integer atomics are associative, so the
//     sum — and the decode — stays bitwise reproducible; no fences, no counter). Workgroup 0 zeroes
//     the other of two accumulator sets, the one the next producer adds into;
//   * EPI_ROPE (qkv): each wave's 4 rows are two RoPE pairs of one head, so q / k are rotated in
//     the epilogue and written straight to the attention input and the KV cache (no rope_append);
//   * PRO_NORMX (qkv, gate_up, lm_head): every wave sums the 64 accumulators (one load, a wave
//     reduction), rstd = rsqrt(sum / K + eps), and the K loop feeds bf16(h * rstd * g) to the FMAs
//     (the separate norm kernel's rounding).
// Measured dead ends: a prologue that normalised the row in every workgroup (8-20 us per
// projection: every workgroup re-read row, residual and weight from L2) and a last-workgroup
// reduction behind a device-scope counter (+22-30 us: the release / acquire fences write back and
// invalidate the whole L2 in every workgroup).
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kR = 4;  // weight rows per wave
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void bf16x8_to_f32(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(v[i] << 16);
    f[2 * i + 1] = __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ float silu_f(float g) { return g / (1.f + __expf(-g)); }

// input transform of x
enum { PRO_NONE = 0, PRO_SWI = 1, PRO_NORMX = 2 };
// output
enum { EPI_NONE = 0, EPI_RESNORM = 1, EPI_ROPE = 2 };

constexpr float kSumsqScale = 1048576.f;  // 2^20: fixed-point units of the sum-of-squares accumulator
constexpr int kSumsqSlots = 64;           // accumulator addresses per row: workgroup b adds into b % 64

struct GemvArgs {
  const bf16* x;
  int64_t ldx;
  const bf16* w;
  bf16* y;  // EPI_RESNORM: h = y + res
  int64_t ldy;
  int N, K;
  const bf16* g;  // PRO_NORMX: norm weight [K]
  float eps;      // PRO_NORMX
  const unsigned long long* sumsq_in;  // PRO_NORMX: [M][kSumsqSlots] fixed-point partial sums of h^2
  // EPI_RESNORM
  const bf16* res;  // [M, N], row stride ldr
  int64_t ldr;
  unsigned long long* sumsq_out;   // [M][kSumsqSlots], zero at launch
  unsigned long long* sumsq_zero;  // [M][kSumsqSlots], zeroed here for the next producer
  // EPI_ROPE (the qkv projection, head_dim 128): q rotated into q_out [M, hq, 128], k rotated and v
  // written at cache slot pos[m] of kc / vc (row m = batch row m)
  bf16* q_out;
  bf16* kc;
  bf16* vc;
  int64_t c_bs, c_ss, c_hs, v_bs, v_ss, v_hs;
  const float* cosb;  // [>= rope_S, 64]
  const float* sinb;
  const int* pos;     // [M]
  int rope_S, cache_L, hq, hkv;
};

// KS waves of the workgroup split K for the same kR rows (KS = 4: 4x the workgroups and weight
// bytes in flight on the small projections, whose 1-workgroup-per-CU grid left HBM latency
// exposed — o_proj ran at 3.5 TB/s).
// PRO_SWI: x is the fused [gate | up] projection output [M, 2K]; the kernel multiplies by
// silu(gate) * up on the fly (the decode MLP's SwiGLU folded into the down-projection GEMV).
template <int M, int KS, int PRO, int EPI>
__global__ __launch_bounds__(256) void gemv_kernel(const GemvArgs a) {
  constexpr bool SWI = PRO == PRO_SWI;
  __shared__ float red[4][M][kR];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int slot = wave / KS, kp = wave % KS;
  const int n0 = (blockIdx.x * (4 / KS) + slot) * kR;
  const int N = a.N, K = a.K;
  // EPI_ROPE: the wave's 4 rows are the RoPE pairs (d, d + 64), (d + 1, d + 65) of one head, so the
  // rotation happens in the epilogue: rows hh*128 + {d, d+1, d+64, d+65}, d = 2 * (group % 32)
  const int hh = n0 / 128, d0 = 2 * ((n0 / kR) % 32);
  auto row_of = [&](int r) { return EPI == EPI_ROPE ? hh * 128 + d0 + (r & 1) + 64 * (r >> 1) : n0 + r; };
  const bf16* __restrict__ x = a.x;
  float acc[M][kR];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kR; ++r) acc[m][r] = 0.f;
  // NORMX: the 64 accumulator slots are loaded here but reduced only after the first K-step's
  // weight loads are issued (the in-order vmcnt then waits for this load alone), so the weight
  // stream starts without waiting for the statistics
  unsigned long long sq[M];
  if constexpr (PRO == PRO_NORMX) {
#pragma unroll
    for (int m = 0; m < M; ++m) sq[m] = a.sumsq_in[m * kSumsqSlots + lane];
  }
  float rstd[M];
  const u32x4* wr[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) wr[r] = reinterpret_cast<const u32x4*>(a.w + (int64_t)min(row_of(r), N - 1) * K);
  auto kstep = [&](int k, auto first, bool valid) {
    u32x4 wv[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) wv[r] = __builtin_nontemporal_load(wr[r] + k / 8);
    if constexpr (PRO == PRO_NORMX && decltype(first)::value) {
#pragma unroll
      for (int m = 0; m < M; ++m) {  // every wave sums the 64 slots itself (integer: exact)
        unsigned long long v = sq[m];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
        rstd[m] = rsqrtf(static_cast<float>(v) / kSumsqScale / K + a.eps);
      }
    }
    float gf[8];
    if constexpr (PRO == PRO_NORMX) bf16x8_to_f32(*reinterpret_cast<const u32x4*>(a.g + k), gf);
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      bf16x8_to_f32(*reinterpret_cast<const u32x4*>(x + m * a.ldx + k), xf[m]);
      if constexpr (SWI) {
        float uf[8];
        bf16x8_to_f32(*reinterpret_cast<const u32x4*>(x + m * a.ldx + K + k), uf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // round like the separate SwiGLU kernel's bf16 output
          xf[m][j] = static_cast<float>(static_cast<bf16>(silu_f(xf[m][j]) * uf[j]));
        }
      }
      if constexpr (PRO == PRO_NORMX) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {  // round like the separate norm kernel's bf16 output
          xf[m][j] = static_cast<float>(static_cast<bf16>(xf[m][j] * rstd[m] * gf[j]));
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float wf[8];
      bf16x8_to_f32(wv[r], wf);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[m][r] = fmaf(valid ? xf[m][j] : 0.f, wf[j], acc[m][r]);
    }
  };
  int k = (kp * 64 + lane) * 8;
  if constexpr (PRO == PRO_NORMX) {  // peeled first step, every lane (the reduction is wave-wide)
    kstep(min(k, K - 8), std::true_type{}, k < K);
    k += 512 * KS;
  }
#pragma unroll 2
  for (; k < K; k += 512 * KS) kstep(k, std::false_type{}, true);
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float v = acc[m][r];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][r] = v;
    }
  if constexpr (KS > 1) {
    if (lane == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < kR; ++r) red[wave][m][r] = acc[m][r];
    }
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < KS; ++q) v += red[slot * KS + q][m][r];
          acc[m][r] = v;
        }
    }
  }
  if constexpr (EPI == EPI_ROPE) {
    if (lane == 0 && kp == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int p = a.pos[m];
        if (p < 0 || p >= a.rope_S || p >= a.cache_L) continue;  // like rope_append: no write
        float y[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) y[r] = static_cast<float>(static_cast<bf16>(acc[m][r]));  // the bf16 qkv
        float o[kR];
        bf16* dst;
        if (hh < a.hq + a.hkv) {
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const float cs = a.cosb[(int64_t)p * 64 + d0 + i], sn = a.sinb[(int64_t)p * 64 + d0 + i];
            o[i] = y[i] * cs - y[i + 2] * sn;
            o[i + 2] = y[i + 2] * cs + y[i] * sn;
          }
          dst = hh < a.hq ? a.q_out + ((int64_t)m * a.hq + hh) * 128
                          : a.kc + m * a.c_bs + (int64_t)p * a.c_ss + (int64_t)(hh - a.hq) * a.c_hs;
        } else {
#pragma unroll
          for (int r = 0; r < kR; ++r) o[r] = y[r];
          dst = a.vc + m * a.v_bs + (int64_t)p * a.v_ss + (int64_t)(hh - a.hq - a.hkv) * a.v_hs;
        }
#pragma unroll
        for (int r = 0; r < kR; ++r) dst[d0 + (r & 1) + 64 * (r >> 1)] = static_cast<bf16>(o[r]);
      }
    }
  } else if constexpr (EPI == EPI_NONE) {
    if (lane == 0 && kp == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < kR; ++r)
          if (n0 + r < N) a.y[m * a.ldy + n0 + r] = static_cast<bf16>(acc[m][r]);
    }
  } else {
    __shared__ float ssq[4][M];
    if (lane == 0 && kp == 0) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          if (n0 + r < N) {
            const bf16 yb = static_cast<bf16>(acc[m][r]);
            const bf16 hb = static_cast<bf16>(static_cast<float>(yb) + static_cast<float>(a.res[m * a.ldr + n0 + r]));
            a.y[m * a.ldy + n0 + r] = hb;
            const float h = static_cast<float>(hb);
            s = fmaf(h, h, s);
          }
        }
        ssq[slot][m] = s;
      }
    }
    __syncthreads();
    if (threadIdx.x < M) {  // spread over 64 addresses: one address took 1024 serialised atomics (+13 us)
      const int m = threadIdx.x;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < 4 / KS; ++q) s += ssq[q][m];
      atomicAdd(a.sumsq_out + m * kSumsqSlots + (blockIdx.x % kSumsqSlots),
                static_cast<unsigned long long>(llrintf(s * kSumsqScale)));
    }
    if (blockIdx.x == 0 && threadIdx.x < M * kSumsqSlots) a.sumsq_zero[threadIdx.x] = 0ull;
  }
}

// Skinny MFMA GEMM for 3-16 decode rows (batched serving): with more than 2 rows the FMA GEMV
// above turns VALU-bound (batch 4: 688 tokens/s against the library's 793), while the weight stream
// is unchanged. Here each workgroup owns 16 weight rows, its KS waves split K, and every 32-wide
// K step is one v_mfma_f32_16x16x32_bf16: A = the x rows (rows >= M read as zero), B = 16 weight
// rows x 8 consecutive k per lane (16-byte non-temporal loads, kU steps in flight per lane). The
// KS partial 16x16 tiles merge through LDS. K % (32 kU) == 0.
constexpr int kU = 8;  // 32-wide K steps per wave per iteration
template <int KS>
__global__ __launch_bounds__(64 * KS) void gemv_mfma_kernel(const bf16* __restrict__ x, int64_t ldx,
                                                           const bf16* __restrict__ w, bf16* __restrict__ y,
                                                           int64_t ldy, int M, int N, int K) {
  __shared__ f32x4 red[KS][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = blockIdx.x * 16;
  const int c = lane & 15, kg = lane >> 4;
  const bf16* wr = w + (int64_t)min(n0 + c, N - 1) * K + kg * 8;
  const bool arow = c < M;
  const bf16* xr = x + (int64_t)min(c, M - 1) * ldx + kg * 8;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = wave * 32 * kU; k < K; k += KS * 32 * kU) {
    bf16x8 b[kU], a[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u)
      b[u] = __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wr + k + 32 * u)));
#pragma unroll
    for (int u = 0; u < kU; ++u) a[u] = bf16x8{};
    if (arow) {  // lanes of rows >= M issue no load (their x traffic is M / 16 of the weight's)
#pragma unroll
      for (int u = 0; u < kU; ++u) a[u] = *reinterpret_cast<const bf16x8*>(xr + k + 32 * u);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[u], acc, 0, 0, 0);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int q = 1; q < KS; ++q) acc += red[q][lane];
  const int n = n0 + c;  // D: column c, rows 4 kg .. 4 kg + 3
  if (n < N) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * kg + r;
      if (m < M) y[(int64_t)m * ldy + n] = static_cast<bf16>(acc[r]);
    }
  }
}

template <int KS, int PRO, int EPI>
void launch_gemv(const GemvArgs& a, int M, hipStream_t s) {
  const dim3 grid((unsigned)gemv_workgroups(a.N));
  switch (M) {
    case 1: hipLaunchKernelGGL((gemv_kernel<1, KS, PRO, EPI>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((gemv_kernel<2, KS, PRO, EPI>), grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL((gemv_kernel<3, KS, PRO, EPI>), grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL((gemv_kernel<4, KS, PRO, EPI>), grid, dim3(256), 0, s, a); break;
  }
}

template <int PRO, int EPI>
void launch_ks(const GemvArgs& a, int M, hipStream_t s) {
  if (gemv_k_split(a.N) == 4) launch_gemv<4, PRO, EPI>(a, M, s);
  else launch_gemv<1, PRO, EPI>(a, M, s);
}

}  // namespace

int gemv_k_split(int N) {
  static const int env = [] { const char* e = getenv("GRT_GEMV_KSPLIT"); return e ? atoi(e) : -1; }();
  if (env == 1 || env == 4) return env;
  (void)N;
  // K split over the workgroup's 4 waves at every N: Llama-3.1-8B decode gate_up 41.3 -> 35.2 us,
  // lm_head 165 -> 149 us (7.1 TB/s), the small projections as before (tools/gemv_bench.py,
  // profiles/r5_decode.md)
  return 4;
}

int gemv_workgroups(int N) {
  const int rows_per_wg = (4 / gemv_k_split(N)) * kR;
  return (N + rows_per_wg - 1) / rows_per_wg;
}

bool gemv_mfma_ok(int M, int K) { return M >= 3 && M <= 16 && K % (32 * kU) == 0; }

// y[M, N] = x[M, K] W^T (swiglu: x = silu(gu[:, :K]) * gu[:, K:], ldx = gu's row stride)
void gemv_bf16(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int M, int N, int K, hipStream_t s,
               bool swiglu) {
  if (!swiglu && gemv_mfma_ok(M, K)) {  // 3-16 rows: the MFMA skinny kernel
    const bf16* xb = static_cast<const bf16*>(x);
    const bf16* wb = static_cast<const bf16*>(w);
    bf16* yb = static_cast<bf16*>(y);
    const dim3 grid((unsigned)((N + 15) / 16));
    // 8 waves per workgroup while the grid is under ~4 workgroups per CU (N <= 16K rows)
    if (N <= 16384) hipLaunchKernelGGL(gemv_mfma_kernel<8>, grid, dim3(512), 0, s, xb, ldx, wb, yb, ldy, M, N, K);
    else hipLaunchKernelGGL(gemv_mfma_kernel<4>, grid, dim3(256), 0, s, xb, ldx, wb, yb, ldy, M, N, K);
    return;
  }
  GemvArgs a{};
  a.x = static_cast<const bf16*>(x), a.ldx = ldx, a.w = static_cast<const bf16*>(w), a.y = static_cast<bf16*>(y);
  a.ldy = ldy, a.N = N, a.K = K;
  if (swiglu) launch_ks<PRO_SWI, EPI_NONE>(a, M, s);
  else launch_ks<PRO_NONE, EPI_NONE>(a, M, s);
}

void gemv_fused_bf16(const GemvFused& f, hipStream_t s) {
  GemvArgs a{};
  a.x = static_cast<const bf16*>(f.x), a.ldx = f.ldx, a.w = static_cast<const bf16*>(f.w);
  a.y = static_cast<bf16*>(f.y), a.ldy = f.ldy, a.N = f.N, a.K = f.K;
  a.g = static_cast<const bf16*>(f.g), a.eps = f.eps, a.sumsq_in = f.sumsq_in;
  a.res = static_cast<const bf16*>(f.res), a.ldr = f.ldr, a.sumsq_out = f.sumsq_out, a.sumsq_zero = f.sumsq_zero;
  a.q_out = static_cast<bf16*>(f.q_out), a.kc = static_cast<bf16*>(f.kc), a.vc = static_cast<bf16*>(f.vc);
  a.c_bs = f.c_bs, a.c_ss = f.c_ss, a.c_hs = f.c_hs, a.v_bs = f.v_bs, a.v_ss = f.v_ss, a.v_hs = f.v_hs;
  a.cosb = f.cosb, a.sinb = f.sinb, a.pos = f.pos, a.rope_S = f.rope_S, a.cache_L = f.cache_L;
  a.hq = f.hq, a.hkv = f.hkv;
  const bool normx = f.sumsq_in != nullptr, resnorm = f.res != nullptr, rope = f.q_out != nullptr;
  if (rope && normx) launch_ks<PRO_NORMX, EPI_ROPE>(a, f.M, s);
  else if (rope) launch_ks<PRO_NONE, EPI_ROPE>(a, f.M, s);
  else if (normx && resnorm) launch_ks<PRO_NORMX, EPI_RESNORM>(a, f.M, s);
  else if (normx) launch_ks<PRO_NORMX, EPI_NONE>(a, f.M, s);
  else if (resnorm && f.swiglu) launch_ks<PRO_SWI, EPI_RESNORM>(a, f.M, s);
  else if (resnorm) launch_ks<PRO_NONE, EPI_RESNORM>(a, f.M, s);
  else if (f.swiglu) launch_ks<PRO_SWI, EPI_NONE>(a, f.M, s);
  else launch_ks<PRO_NONE, EPI_NONE>(a, f.M, s);
}

}  // namespace grt
