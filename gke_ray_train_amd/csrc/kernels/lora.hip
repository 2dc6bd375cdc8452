// LoRA adapter kernels for gfx950: the input-dropout + down-projection and the adapter's
// input-gradient accumulation, each ONE pass over the [tokens, in] activation.
//
// Reference role: PEFT's LoRA layer on every targeted projection of the QLoRA SFT job
// (LoraConfig r=64, alpha=16, dropout=0.1 on q,k,v,o,gate,up,down; reference
// ray-jobs/fine_tune_llama_ray.py:243-254, fine_tune_config.json:6-8,30-33):
//     y = base(x) + s * B (A dropout(x)).
// Without these kernels the adapter costs, per adapted input and step, a dropout pass
// (read x, write x_d), a rank-R GEMM over x_d, and in the backward a [tokens, in] GEMM
// g·A written to a temporary plus a dropout-backward pass reading it and read-modify-writing dX —
// ~5 full passes over a [tokens, in] tensor around two skinny GEMMs the library tiles poorly.
//
//   lora_down:  h[M][R] = (x ⊙ keep / (1-p)) · A^T, A = [R][K] (the concatenated A of all
//               targets); the dropout keep-mask is the element-dropout hash of x's element index
//               (grt_common.h drop_keep, the same mask dropout_fwd/bwd_seeded use), applied in
//               registers; x_d is optionally written as a side output (the dA GEMM reads it).
//               MFMA D[R][token] = A · x_d^T: one wave = 32 tokens x R, the workgroup's four waves
//               split K and reduce through LDS. Grid = tokens / 32 (256 workgroups at 8192 tokens).
//   lora_dx:    dX[M][K] (+)= keep / (1-p) ⊙ (g[M][R] · A[R][K]) from A^T = [K][R]: MFMA
//               D[k][token] = A^T · g^T over R, epilogue applies the mask and accumulates into dX
//               with 8-byte row chunks — one read-modify-write of dX, no temporary.
// v_mfma_f32_32x32x16_bf16 throughout; operands are 16-byte row fragments loaded straight from
// global memory (A / A^T / g are small and L2-resident; x is streamed once).
#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

__device__ __forceinline__ f32x16 mfma32x32x16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// (accumulator element r of lane half h holds row 8 (r / 4) + 4 h + r % 4 of the 32-row tile)

// keep flags of 8 consecutive elements starting at a 4-aligned element index
__device__ __forceinline__ void keep8(uint64_t key, uint64_t idx0, uint32_t thr, bool (&kp)[8]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const uint64_t hv = hash_u64(key ^ ((idx0 >> 2) + q));
#pragma unroll
    for (int j = 0; j < 4; ++j) kp[4 * q + j] = ((uint32_t)(hv >> (16 * j)) & 0xffffu) >= thr;
  }
}

template <int RB>  // R = 32 * RB
__global__ __launch_bounds__(256) void lora_down_kernel(const LoraDownParams P) {
  constexpr int R = 32 * RB;
  __shared__ float red[3][RB * 16 * 64];  // waves 1-3 park their partial accumulators
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t t0 = (int64_t)blockIdx.x * 32;
  const int64_t tok = t0 + l32;
  const bool tok_ok = tok < P.M;
  const bf16* xrow = static_cast<const bf16*>(P.x) + (tok_ok ? tok : P.M - 1) * (int64_t)P.ldx;
  const int kq = P.K / 4, kbeg = w * kq;
  const bool drop = P.p > 0.f;
  const uint32_t thr = drop_thr(P.p);
  const float sc = drop ? 1.f / (1.f - P.p) : 1.f;
  const uint64_t key = hash_u64(P.seed);
  const uint64_t eidx = P.offset + (uint64_t)tok * (uint64_t)P.K;  // element index of x[tok][0]

  f32x16 acc[RB];
#pragma unroll
  for (int i = 0; i < RB; ++i) acc[i] = f32x16{};
  for (int k = kbeg; k < kbeg + kq; k += 16) {
    const int kk = k + 8 * h;
    bf16x8 xf = *reinterpret_cast<const bf16x8*>(xrow + kk);
    if (drop) {
      bool kp[8];
      keep8(key, eidx + (uint64_t)kk, thr, kp);
#pragma unroll
      for (int e = 0; e < 8; ++e) xf[e] = static_cast<bf16>(kp[e] ? static_cast<float>(xf[e]) * sc : 0.f);
    }
    if (P.xd != nullptr && tok_ok) *reinterpret_cast<bf16x8*>(static_cast<bf16*>(P.xd) + tok * (int64_t)P.K + kk) = xf;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const bf16x8 af = *reinterpret_cast<const bf16x8*>(static_cast<const bf16*>(P.a) + (int64_t)(rb * 32 + l32) * P.K + kk);
      acc[rb] = mfma32x32x16(af, xf, acc[rb]);  // D[R row][token]
    }
  }
  // reduce the four K quarters: waves 1-3 -> LDS, wave 0 sums and stores
  if (w > 0) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[w - 1][(rb * 16 + r) * 64 + lane] = acc[rb][r];
  }
  __syncthreads();
  if (w == 0 && tok_ok) {
    bf16* hrow = static_cast<bf16*>(P.h) + tok * (int64_t)R;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * q + j, ix = (rb * 16 + r) * 64 + lane;
          v[j] = static_cast<bf16>(acc[rb][r] + red[0][ix] + red[1][ix] + red[2][ix]);
        }
        *reinterpret_cast<bf16x4*>(hrow + rb * 32 + 8 * q + 4 * h) = v;
      }
  }
}

template <int RS>  // R = 16 * RS
__global__ __launch_bounds__(256) void lora_dx_kernel(const LoraDxParams P) {
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkb = P.K / 128;
  const int64_t tb = blockIdx.x / nkb;
  const int kb = blockIdx.x % nkb;
  const int64_t t0 = tb * 64 + (w & 1) * 32;
  const int c0 = kb * 128 + (w >> 1) * 64;
  const int64_t tok = t0 + l32;
  const bool tok_ok = tok < P.M;
  const bf16* grow = static_cast<const bf16*>(P.g) + (tok_ok ? tok : P.M - 1) * (int64_t)(16 * RS);
  bf16x8 gf[RS];
#pragma unroll
  for (int s = 0; s < RS; ++s) gf[s] = *reinterpret_cast<const bf16x8*>(grow + 16 * s + 8 * h);
  const bool drop = P.p > 0.f;
  const uint32_t thr = drop_thr(P.p);
  const float sc = drop ? 1.f / (1.f - P.p) : 1.f;
  const uint64_t key = hash_u64(P.seed);
  const uint64_t eidx = P.offset + (uint64_t)tok * (uint64_t)P.K;
  bf16* dxrow = static_cast<bf16*>(P.dx) + tok * (int64_t)P.K;
#pragma unroll
  for (int cb = 0; cb < 2; ++cb) {
    const int cc = c0 + cb * 32;
    f32x16 acc = f32x16{};
    const bf16* arow = static_cast<const bf16*>(P.at) + (int64_t)(cc + l32) * (16 * RS);
#pragma unroll
    for (int s = 0; s < RS; ++s)
      acc = mfma32x32x16(*reinterpret_cast<const bf16x8*>(arow + 16 * s + 8 * h), gf[s], acc);  // D[k][token]
    if (tok_ok) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kc = cc + 8 * q + 4 * h;  // 4 consecutive columns kc .. kc+3 (4-aligned)
        float d[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = acc[4 * q + j] * sc;
        if (drop) {
          const uint64_t hv = hash_u64(key ^ ((eidx + (uint64_t)kc) >> 2));
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (((uint32_t)(hv >> (16 * j)) & 0xffffu) < thr) d[j] = 0.f;
        }
        bf16x4* dst = reinterpret_cast<bf16x4*>(dxrow + kc);
        bf16x4 o;
        if (P.accumulate) {
          const bf16x4 old = *dst;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = static_cast<bf16>(static_cast<float>(old[j]) + d[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = static_cast<bf16>(d[j]);
        }
        *dst = o;
      }
    }
  }
}

}  // namespace

bool lora_down_supported(int64_t M, int K, int R, int ldx, uint64_t offset) {
  return M > 0 && K % 64 == 0 && R % 32 == 0 && R >= 32 && R <= 256 && ldx % 8 == 0 && offset % 4 == 0;
}

void lora_down(const LoraDownParams& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.M + 31) / 32)), block(256);
  switch (p.R / 32) {
    case 1: hipLaunchKernelGGL(lora_down_kernel<1>, grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL(lora_down_kernel<2>, grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL(lora_down_kernel<3>, grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL(lora_down_kernel<4>, grid, block, 0, s, p); break;
    case 5: hipLaunchKernelGGL(lora_down_kernel<5>, grid, block, 0, s, p); break;
    case 6: hipLaunchKernelGGL(lora_down_kernel<6>, grid, block, 0, s, p); break;
    case 7: hipLaunchKernelGGL(lora_down_kernel<7>, grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL(lora_down_kernel<8>, grid, block, 0, s, p); break;
  }
}

bool lora_dx_supported(int64_t M, int K, int R, uint64_t offset) {
  return M > 0 && K % 128 == 0 && R % 16 == 0 && R >= 16 && R <= 256 && offset % 4 == 0;
}

void lora_dx(const LoraDxParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(((p.M + 63) / 64) * (p.K / 128))), block(256);
#define GRT_LDX(N) case N: hipLaunchKernelGGL(lora_dx_kernel<N>, grid, block, 0, s, p); break;
  switch (p.R / 16) {
    GRT_LDX(1) GRT_LDX(2) GRT_LDX(3) GRT_LDX(4) GRT_LDX(5) GRT_LDX(6) GRT_LDX(7) GRT_LDX(8)
    GRT_LDX(9) GRT_LDX(10) GRT_LDX(11) GRT_LDX(12) GRT_LDX(13) GRT_LDX(14) GRT_LDX(15)
    default: hipLaunchKernelGGL(lora_dx_kernel<16>, grid, block, 0, s, p); break;
  }
#undef GRT_LDX
}

}  // namespace grt
