// Flash attention in exact fp32 (forward + backward) for gfx950 / CDNA4.
//
// Reference role: BasicLLM trains in fp32 end to end (no autocast; reference
// ray-jobs/pytorch_llm_ray.py:75-105,274-278), so its causal self-attention with probability
// dropout 0.1 (nn.TransformerEncoderLayer, :82-86) needs an fp32 kernel; SURVEY §2.6 K-A05, §7.4
// item 2. gfx950 has no xf32/TF32 MFMA: f32 operands run on v_mfma_f32_32x32x2_f32 at the fp32
// rate (157 TF, cdna_hip_programming.md §3 "FP32-input MFMA"), bit-exact k-ordered fma chains.
//
// Same algorithm, layouts and dropout hash as the bf16 kernels (attention.hip), so the fp32 and
// bf16 paths and the fp32 math reference (ops/_ref.attention) agree mask for mask:
//   forward / dQ: per wave 32 query rows on the MFMA lane, K/V tiles of 32 keys double-buffered
//     in LDS; S^T = K Q^T (A = K rows from LDS, B = Q held in VGPRs), online softmax lane-local,
//     O^T += V^T P^T with the S^T accumulator directly as the B operand (register r of a 32x32
//     accumulator is key acc_row(r, h), so MFMA step r takes k-slot h from that key and the A
//     side reads V row acc_row(r, h)).
//   dK/dV: per wave 32 keys on the lane, K and V in VGPRs, Q/dO tiles of 32 rows in LDS;
//     S = Q K^T, dP = dO V^T, dV^T += dO^T P, dK^T += Q^T dS (no atomics).
// K-dim permutation of the QK^T / dO V^T products: MFMA step s reads d = s (lane half 0) and
// d = D/2 + s (lane half 1), so one lane's A operands for 4 consecutive steps are one 16-byte
// LDS read and its B operands are D/2 consecutive floats of its own row held in registers.
// LDS rows are padded to D + 4 floats: the ds_read_b128 row reads are conflict-free (16-lane
// groups hit 16 distinct 4-bank quads) and the b32 column reads of the P^T V products are
// contiguous within each 32-lane half.
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int NT = 256;   // 4 waves
constexpr int TK = 32;    // keys (fwd/dQ) or query rows (dK/dV) per LDS tile
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
// identical to attention.hip / ops/_ref.attn_dropout_keep
__device__ __forceinline__ float drop_factor(const AttnParams& p, uint32_t bh, int q, int k) {
  uint32_t h = p.drop_seed ^ (bh * 0x9E3779B1u);
  h = fmix32(h ^ ((uint32_t)q * 0x85EBCA77u));
  h = fmix32(h ^ ((uint32_t)k * 0xC2B2AE3Du));
  return h >= p.drop_thresh ? p.drop_scale : 0.f;
}

template <int D>
struct Tile {
  static constexpr int LDW = D + 4;                    // padded row (floats)
  static constexpr int FLOATS = TK * LDW;
  static constexpr int PER_THREAD = TK * D / 4 / NT;   // float4 chunks per thread per operand
  static_assert(PER_THREAD >= 1, "tile too small for the block");
};

// cooperative load of rows [r0, r0 + TK) of a [rows][D] fp32 matrix (row stride ld) into registers
template <int D>
__device__ __forceinline__ void tile_load(f32x4 (&reg)[Tile<D>::PER_THREAD], const float* src, int64_t ld, int r0,
                                          int rows_valid) {
#pragma unroll
  for (int i = 0; i < Tile<D>::PER_THREAD; ++i) {
    const int c = threadIdx.x + NT * i, row = c / (D / 4), col = (c % (D / 4)) * 4;
    const int gr = r0 + row;
    reg[i] = gr < rows_valid ? *reinterpret_cast<const f32x4*>(src + (int64_t)gr * ld + col) : f32x4{0, 0, 0, 0};
  }
}
template <int D>
__device__ __forceinline__ void tile_store(const f32x4 (&reg)[Tile<D>::PER_THREAD], float* lds) {
#pragma unroll
  for (int i = 0; i < Tile<D>::PER_THREAD; ++i) {
    const int c = threadIdx.x + NT * i, row = c / (D / 4), col = (c % (D / 4)) * 4;
    *reinterpret_cast<f32x4*>(lds + row * Tile<D>::LDW + col) = reg[i];
  }
}

// acc[] += A(row-tile in LDS, row = lane&31) x B(regs of this lane's own row), K = D
template <int D>
__device__ __forceinline__ f32x16 rows_x_regs(const float* lds, const float (&breg)[D / 2], f32x16 acc, int l32,
                                              int h) {
  const float* row = lds + l32 * Tile<D>::LDW + h * (D / 2);
#pragma unroll
  for (int s4 = 0; s4 < D / 8; ++s4) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(row + 4 * s4);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma(a[j], breg[4 * s4 + j], acc);
  }
  return acc;
}

// out[db] += (LDS tile)^T[d][key] x P^T[key][lane]: P^T in the 32x32 accumulator `pt`
template <int D>
__device__ __forceinline__ void lds_t_x_acc(const float* lds, const f32x16& pt, f32x16 (&out)[D / 32], int l32,
                                            int h) {
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float* row = lds + acc_row(r, h) * Tile<D>::LDW + l32;
#pragma unroll
    for (int db = 0; db < D / 32; ++db) out[db] = mfma(row[db * 32], pt[r], out[db]);
  }
}

// store a [D/32] x f32x16 transposed accumulator (rows d, lane = this thread's row) as row `dst`
template <int D>
__device__ __forceinline__ void store_row(float* dst, const f32x16 (&acc)[D / 32], float mul, int h) {
#pragma unroll
  for (int db = 0; db < D / 32; ++db)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = acc[db][4 * gg + j] * mul;
      *reinterpret_cast<f32x4*>(dst + db * 32 + 8 * gg + 4 * h) = v;
    }
}

// ------------------------------------------------------------------------------------------------
// Forward: 128 query rows per workgroup (32 per wave), 32-key tiles
// ------------------------------------------------------------------------------------------------
template <int D, bool DROP>
__global__ __launch_bounds__(NT, 2) void attn_fwd_f32_kernel(const AttnParams p) {
  using T = Tile<D>;
  __shared__ __attribute__((aligned(16))) float smem[4 * T::FLOATS];  // K[2], V[2]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  constexpr int BM = 128;
  const int nqb = (p.Sq + BM - 1) / BM;
  const int BH = p.B * p.Hq;
  const int qblk = nqb - 1 - (int)(blockIdx.x / BH);  // heaviest causal blocks first
  const int bh = blockIdx.x % BH;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  GRT_DEVICE_CHECK(b < p.B && hkv < p.Hkv && qblk >= 0);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int q0 = qblk * BM, qw0 = q0 + w * 32, myq = qw0 + l32;

  const float* Q = (const float*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
  const float* K = (const float*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const float* V = (const float*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;

  float qf[D / 2];
#pragma unroll
  for (int i = 0; i < D / 8; ++i) {
    const f32x4 v = myq < p.Sq ? *reinterpret_cast<const f32x4*>(Q + (int64_t)myq * p.q_ss + h * (D / 2) + 4 * i)
                               : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) qf[4 * i + j] = v[j];
  }

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + BM + off);
  const int nt = kend > 0 ? (kend + TK - 1) / TK : 0;

  f32x4 kreg[T::PER_THREAD], vreg[T::PER_THREAD];
  f32x16 o[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const float c = p.scale * kLog2e;

  if (nt > 0) {
    tile_load<D>(kreg, K, p.k_ss, 0, sk);
    tile_load<D>(vreg, V, p.v_ss, 0, sk);
    tile_store<D>(kreg, smem);
    tile_store<D>(vreg, smem + 2 * T::FLOATS);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1, kb = t * TK;
    const float* Kl = smem + cur * T::FLOATS;
    const float* Vl = smem + (2 + cur) * T::FLOATS;
    if (t + 1 < nt) {
      tile_load<D>(kreg, K, p.k_ss, kb + TK, sk);
      tile_load<D>(vreg, V, p.v_ss, kb + TK, sk);
    }
    if (!(p.causal && kb > qw0 + 31 + off)) {
      f32x16 s = rows_x_regs<D>(Kl, qf, f32x16{}, l32, h);
      const bool need_mask = (kb + TK > sk) || (p.causal && kb + TK - 1 > qw0 + off);
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = s[r] * c;
        if (need_mask) {
          const int key = kb + acc_row(r, h);
          if (key >= sk || (p.causal && key > myq + off)) v = -INFINITY;
        }
        s[r] = v;
        mx = fmaxf(mx, v);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float msub = (mn == -INFINITY) ? 0.f : mn;
      const float alpha = fast_exp2(m - msub);
      float rs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = fast_exp2(s[r] - msub);
        rs += e;  // normaliser over the undropped probabilities
        s[r] = DROP ? e * drop_factor(p, (uint32_t)bh, myq, kb + acc_row(r, h)) : e;
      }
      l = l * alpha + rs;
      m = mn;
#pragma unroll
      for (int i = 0; i < D / 32; ++i) o[i] *= alpha;
      lds_t_x_acc<D>(Vl, s, o, l32, h);
    }
    if (t + 1 < nt) {
      tile_store<D>(kreg, smem + (cur ^ 1) * T::FLOATS);
      tile_store<D>(vreg, smem + (2 + (cur ^ 1)) * T::FLOATS);
    }
    __syncthreads();
  }

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (myq < p.Sq) {
    float* O = (float*)p.o + (int64_t)b * p.o_bs + (int64_t)hq * p.o_hs + (int64_t)myq * p.o_ss;
    store_row<D>(O, o, inv, h);
    if (h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] = lt > 0.f ? (m + __log2f(lt)) * kLn2 : INFINITY;
  }
}

// ------------------------------------------------------------------------------------------------
// Backward
// ------------------------------------------------------------------------------------------------
// delta[b,h,q] = sum_d dO*O: one 32-lane half-wave per row
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_pre_f32_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  const int l32 = threadIdx.x & 31;
  const int64_t row = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5);
  const int64_t nrows = (int64_t)p.B * p.Hq * p.Sq;
  float acc = 0.f;
  if (row < nrows) {
    const int q = (int)(row % p.Sq);
    const int64_t bh = row / p.Sq;
    const int hq = (int)(bh % p.Hq), b = (int)(bh / p.Hq);
    const float* O = (const float*)p.o + (int64_t)b * p.o_bs + (int64_t)hq * p.o_hs + (int64_t)q * p.o_ss;
    const float* dO = (const float*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs + (int64_t)q * P.do_ss;
#pragma unroll
    for (int c = l32 * 4; c < D; c += 128) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(O + c);
      const f32x4 g = *reinterpret_cast<const f32x4*>(dO + c);
      acc += a[0] * g[0] + a[1] * g[1] + a[2] * g[2] + a[3] * g[3];
    }
  }
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < nrows && l32 == 0) P.delta[row] = acc;
}

// dK / dV: 128 keys of one (batch, kv head) per workgroup, 32 per wave (key on the lane);
// sweeps the group's query heads x 32-row query tiles.
template <int D, bool DROP>
__global__ __launch_bounds__(NT, 1) void attn_bwd_dkdv_f32_kernel(const AttnBwdParams P) {
  using T = Tile<D>;
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) float smem[4 * T::FLOATS + 4 * TK];  // Q[2], dO[2], lse[2], delta[2]
  float* lsel = smem + 4 * T::FLOATS;
  float* dell = lsel + 2 * TK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  constexpr int BN = 128;
  const int nkb = (p.Sk + BN - 1) / BN;
  const int kblk = nkb - 1 - (int)(blockIdx.x / (p.B * p.Hkv));
  const int bhk = blockIdx.x % (p.B * p.Hkv);
  const int b = bhk / p.Hkv, hkv = bhk % p.Hkv;
  const int grp = p.Hq / p.Hkv;
  GRT_DEVICE_CHECK(kblk >= 0 && grp * p.Hkv == p.Hq);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int k0 = kblk * BN, kw0 = k0 + w * 32, mykey = kw0 + l32;
  const float c = p.scale * kLog2e;

  const float* K = (const float*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const float* V = (const float*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;
  float kf[D / 2], vf[D / 2];
#pragma unroll
  for (int i = 0; i < D / 8; ++i) {
    const bool ok = mykey < sk;
    const f32x4 a = ok ? *reinterpret_cast<const f32x4*>(K + (int64_t)mykey * p.k_ss + h * (D / 2) + 4 * i)
                       : f32x4{0, 0, 0, 0};
    const f32x4 v = ok ? *reinterpret_cast<const f32x4*>(V + (int64_t)mykey * p.v_ss + h * (D / 2) + 4 * i)
                       : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) { kf[4 * i + j] = a[j]; vf[4 * i + j] = v[j]; }
  }
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  int qstart = p.causal ? max(0, k0 - off) : 0;
  qstart = (qstart / TK) * TK;
  const int nqt = qstart < p.Sq ? (p.Sq - qstart + TK - 1) / TK : 0;
  const int total = (k0 < sk) ? nqt * grp : 0;

  f32x4 qreg[T::PER_THREAD], oreg[T::PER_THREAD];
  float lse_r = 0.f, del_r = 0.f;
  auto load_q = [&](int it) {
    const int hq = hkv * grp + it / nqt;
    const int qt = qstart + (it % nqt) * TK;
    const float* Q = (const float*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
    const float* dO = (const float*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs;
    tile_load<D>(qreg, Q, p.q_ss, qt, p.Sq);
    tile_load<D>(oreg, dO, P.do_ss, qt, p.Sq);
    if (tid < TK) {
      const int q = qt + tid;
      const int64_t ri = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      lse_r = q < p.Sq ? p.lse[ri] * kLog2e : INFINITY;
      del_r = q < p.Sq ? P.delta[ri] : 0.f;
    }
  };
  auto store_q = [&](int buf) {
    tile_store<D>(qreg, smem + buf * T::FLOATS);
    tile_store<D>(oreg, smem + (2 + buf) * T::FLOATS);
    if (tid < TK) { lsel[buf * TK + tid] = lse_r; dell[buf * TK + tid] = del_r; }
  };

  if (total > 0) { load_q(0); store_q(0); }
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int qt = qstart + (it % nqt) * TK;
    const uint32_t bhq = (uint32_t)(b * p.Hq + hkv * grp + it / nqt);
    if (it + 1 < total) load_q(it + 1);
    if (!(p.causal && kw0 > qt + TK - 1 + off)) {
      const float* Ql = smem + cur * T::FLOATS;
      const float* dOl = smem + (2 + cur) * T::FLOATS;
      f32x16 s = rows_x_regs<D>(Ql, kf, f32x16{}, l32, h);
      f32x16 dp = rows_x_regs<D>(dOl, vf, f32x16{}, l32, h);
      const bool need_mask = (k0 + BN > sk) || (p.causal && kw0 + 31 > qt + off) || (qt + TK > p.Sq);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qi = acc_row(r, h), q = qt + qi;
        float pv = fast_exp2(s[r] * c - lsel[cur * TK + qi]);
        if (need_mask && (mykey >= sk || q >= p.Sq || (p.causal && mykey > q + off))) pv = 0.f;
        const float de = dell[cur * TK + qi];
        if (DROP) {
          const float z = drop_factor(p, bhq, q, mykey);
          s[r] = pv * z;                  // dV sees the dropped probabilities
          dp[r] = pv * (dp[r] * z - de);
        } else {
          s[r] = pv;
          dp[r] = pv * (dp[r] - de);
        }
      }
      lds_t_x_acc<D>(dOl, s, dv, l32, h);   // dV^T += dO^T P
      lds_t_x_acc<D>(Ql, dp, dk, l32, h);   // dK^T += Q^T dS
    }
    if (it + 1 < total) store_q(cur ^ 1);
    __syncthreads();
  }

  if (mykey < p.Sk) {
    float* dK = (float*)P.dk + (int64_t)b * P.dk_bs + (int64_t)hkv * P.dk_hs + (int64_t)mykey * P.dk_ss;
    float* dV = (float*)P.dv + (int64_t)b * P.dv_bs + (int64_t)hkv * P.dv_hs + (int64_t)mykey * P.dv_ss;
    store_row<D>(dK, dk, p.scale, h);
    store_row<D>(dV, dv, 1.f, h);
  }
}

// dQ: the forward's structure; S^T and dP^T recomputed with the query on the lane,
// dQ^T += K^T dS^T with dS^T as the B operand.
template <int D, bool DROP>
__global__ __launch_bounds__(NT, 1) void attn_bwd_dq_f32_kernel(const AttnBwdParams P) {
  using T = Tile<D>;
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) float smem[4 * T::FLOATS];  // K[2], V[2]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  constexpr int BM = 128;
  const int nqb = (p.Sq + BM - 1) / BM;
  const int BH = p.B * p.Hq;
  const int qblk = nqb - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int q0 = qblk * BM, qw0 = q0 + w * 32, myq = qw0 + l32;
  const bool qok = myq < p.Sq;

  const float* Q = (const float*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
  const float* dO = (const float*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs;
  const float* K = (const float*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const float* V = (const float*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;
  float qf[D / 2], of[D / 2];
#pragma unroll
  for (int i = 0; i < D / 8; ++i) {
    const f32x4 a = qok ? *reinterpret_cast<const f32x4*>(Q + (int64_t)myq * p.q_ss + h * (D / 2) + 4 * i)
                        : f32x4{0, 0, 0, 0};
    const f32x4 g = qok ? *reinterpret_cast<const f32x4*>(dO + (int64_t)myq * P.do_ss + h * (D / 2) + 4 * i)
                        : f32x4{0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) { qf[4 * i + j] = a[j]; of[4 * i + j] = g[j]; }
  }
  const int64_t ri = ((int64_t)b * p.Hq + hq) * p.Sq + (qok ? myq : 0);
  const float lse2 = qok ? p.lse[ri] * kLog2e : INFINITY;
  const float dlt = qok ? P.delta[ri] : 0.f;
  const float c = p.scale * kLog2e;

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + BM + off);
  const int nt = kend > 0 ? (kend + TK - 1) / TK : 0;

  f32x4 kreg[T::PER_THREAD], vreg[T::PER_THREAD];
  f32x16 dq[D / 32];
#pragma unroll
  for (int i = 0; i < D / 32; ++i) dq[i] = f32x16{};
  if (nt > 0) {
    tile_load<D>(kreg, K, p.k_ss, 0, sk);
    tile_load<D>(vreg, V, p.v_ss, 0, sk);
    tile_store<D>(kreg, smem);
    tile_store<D>(vreg, smem + 2 * T::FLOATS);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1, kb = t * TK;
    const float* Kl = smem + cur * T::FLOATS;
    const float* Vl = smem + (2 + cur) * T::FLOATS;
    if (t + 1 < nt) {
      tile_load<D>(kreg, K, p.k_ss, kb + TK, sk);
      tile_load<D>(vreg, V, p.v_ss, kb + TK, sk);
    }
    if (!(p.causal && kb > qw0 + 31 + off)) {
      f32x16 s = rows_x_regs<D>(Kl, qf, f32x16{}, l32, h);
      f32x16 dp = rows_x_regs<D>(Vl, of, f32x16{}, l32, h);
      const bool need_mask = (kb + TK > sk) || (p.causal && kb + TK - 1 > qw0 + off);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb + acc_row(r, h);
        float pv = fast_exp2(s[r] * c - lse2);
        if (need_mask && (key >= sk || (p.causal && key > myq + off))) pv = 0.f;
        const float z = DROP ? drop_factor(p, (uint32_t)bh, myq, key) : 1.f;
        s[r] = pv * (dp[r] * z - dlt);
      }
      lds_t_x_acc<D>(Kl, s, dq, l32, h);  // dQ^T += K^T dS^T
    }
    if (t + 1 < nt) {
      tile_store<D>(kreg, smem + (cur ^ 1) * T::FLOATS);
      tile_store<D>(vreg, smem + (2 + (cur ^ 1)) * T::FLOATS);
    }
    __syncthreads();
  }
  if (qok) {
    float* dQ = (float*)P.dq + (int64_t)b * P.dq_bs + (int64_t)hq * P.dq_hs + (int64_t)myq * P.dq_ss;
    store_row<D>(dQ, dq, p.scale, h);
  }
}

template <int D>
void fwd_launch(const AttnParams& p, hipStream_t s) {
  const dim3 grid((unsigned)(((p.Sq + 127) / 128) * p.B * p.Hq));
  if (p.drop_thresh) hipLaunchKernelGGL((attn_fwd_f32_kernel<D, true>), grid, dim3(NT), 0, s, p);
  else hipLaunchKernelGGL((attn_fwd_f32_kernel<D, false>), grid, dim3(NT), 0, s, p);
}

template <int D>
void bwd_launch(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = (int64_t)p.f.B * p.f.Hq * p.f.Sq;
  hipLaunchKernelGGL(attn_bwd_pre_f32_kernel<D>, dim3((unsigned)((rows + 7) / 8)), dim3(256), 0, s, p);
  const dim3 g1((unsigned)(((p.f.Sk + 127) / 128) * p.f.B * p.f.Hkv));
  const dim3 g2((unsigned)(((p.f.Sq + 127) / 128) * p.f.B * p.f.Hq));
  if (p.f.drop_thresh) {
    hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<D, true>), g1, dim3(NT), 0, s, p);
    hipLaunchKernelGGL((attn_bwd_dq_f32_kernel<D, true>), g2, dim3(NT), 0, s, p);
  } else {
    hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<D, false>), g1, dim3(NT), 0, s, p);
    hipLaunchKernelGGL((attn_bwd_dq_f32_kernel<D, false>), g2, dim3(NT), 0, s, p);
  }
}

}  // namespace

bool attn_f32_supported(int head_dim) { return head_dim == 64 || head_dim == 128; }

void attn_fwd_f32(const AttnParams& p, hipStream_t s) {
  if (p.D == 128) fwd_launch<128>(p, s);
  else fwd_launch<64>(p, s);
}

void attn_bwd_f32(const AttnBwdParams& p, hipStream_t s) {
  if (p.f.D == 128) bwd_launch<128>(p, s);
  else bwd_launch<64>(p, s);
}

}  // namespace grt
