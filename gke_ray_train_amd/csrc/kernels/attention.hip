// Flash attention (forward + backward) for gfx950 / CDNA4, bf16 in, fp32 accumulate.
//
// Reference role: the causal SDPA inside BasicLLM's nn.TransformerEncoderLayer
// (reference ray-jobs/pytorch_llm_ray.py:82-86,103) and HF Llama's sdpa attention in the SFT job
// (ray-jobs/fine_tune_llama_ray.py:240); SURVEY §2.6 K-A05 / K-B07. On ROCm torch routes SDPA to
// aotriton (Triton AOT), which this framework does not use.
//
// Layout: q/k/v/o are [B, S, H, D] with arbitrary batch/seq/head strides (last dim contiguous), so
// the kernels read straight out of the fused QKV projection and write straight into the o_proj
// input — no transposes. D = 128. GQA: query head h reads kv head h / (Hq / Hkv).
//
// MFMA mapping (v_mfma_f32_32x32x16_bf16, cdna_hip_programming.md §3):
//   forward, per wave = 32 query rows, per K/V tile = 64 keys:
//     S^T[key][q] = K · Q^T   (A = K rows from LDS, B = Q rows held in VGPRs)  -> the query is
//                  the MFMA lane, so row max / row sum of the online softmax are lane-local
//                  (+ one lane^32 exchange) and the O^T rescale needs no cross-lane traffic;
//     O^T[d][q]  += V^T · P^T  (A = V^T via ds_read_b64_tr_b16 on the row-major V tile,
//                  B = the S^T accumulator converted to bf16 in place: §3 "accumulator tile as
//                  the next MFMA's operand", with the permuted key order matched on the V side).
//   backward, per workgroup = 128 keys of one kv head (32 per wave, key on the MFMA lane):
//     S = Q·K^T, dP = dO·V^T (accumulators are directly the B operands of)
//     dV^T += dO^T · P,  dK^T += Q^T · dS  (A operands by transposed LDS reads);
//     dS crosses LDS once, transposed, for dQ = dS · K, which is added with fp32 atomics
//     (256-byte row segments, the full-rate shape of MI355X_MICROARCH.md §Global float atomics).
//   All LDS tiles use the dual row-read / transposed-read XOR image of cdna_hip_programming.md
//   T10 (b), conflict-free for both the ds_read_b128 row reads and the tr_b16 reads.
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int D = 128;
constexpr int kChunks = D / 8;  // 16-byte chunks per row

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-byte chunk `ch` of row `row` in a [rows][128 x bf16] LDS image (T10 (b))
__device__ __forceinline__ int img_off(int row, int ch) {
  return row * 256 + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}
__device__ __forceinline__ bf16x8 lds_row_read(const char* base, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(base + img_off(row, ch));
}
// transposed read: the 16-lane group reads rows r0..r0+3, columns c0..c0+15 (c0 multiple of 16);
// lane i of the group receives column c0+i of the 4 rows.
__device__ __forceinline__ bf16x4 lds_tr_read(const char* base, int r0, int c0, int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  const int col = c0 + 4 * p;
  const char* a = base + img_off(r0 + q, col >> 3) + 8 * ((col >> 2) & 1);
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a);
}

__device__ __forceinline__ bf16x8 cat(bf16x4 a, bf16x4 b) {
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 pack8(const f32x16& x, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = static_cast<bf16>(x[base + j]);
  return r;
}
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Counter-based dropout hash (must match ops/_ref.attn_dropout_keep bit for bit): murmur3 fmix32
// of the (batch*head, query, key) coordinates mixed with the per-call seed. Stateless, so the
// forward and both backward kernels regenerate the same mask without storing it.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t attn_dropout_hash(uint32_t seed, uint32_t bh, uint32_t q, uint32_t k) {
  uint32_t h = seed ^ (bh * 0x9E3779B1u);
  h = fmix32(h ^ (q * 0x85EBCA77u));
  return fmix32(h ^ (k * 0xC2B2AE3Du));
}
__device__ __forceinline__ float drop_factor(const AttnParams& p, uint32_t bh, int q, int k) {
  return attn_dropout_hash(p.drop_seed, bh, (uint32_t)q, (uint32_t)k) >= p.drop_thresh ? p.drop_scale : 0.f;
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------------------------
constexpr int FBM = 128, FBN = 64, FNT = 256;
constexpr int kTileBytes = FBN * D * 2;  // 16 KiB

template <bool DROP>
__global__ __launch_bounds__(FNT, 2) void attn_fwd_kernel(const AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kTileBytes];  // K[2], V[2]
  auto Kl = [&](int buf) -> char* { return smem + buf * kTileBytes; };
  auto Vl = [&](int buf) -> char* { return smem + (2 + buf) * kTileBytes; };

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int nqb = (p.Sq + FBM - 1) / FBM;
  const int BH = p.B * p.Hq;
  const int qblk = nqb - 1 - (int)(blockIdx.x / BH);  // heaviest (causal) blocks first
  const int bh = blockIdx.x % BH;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  GRT_DEVICE_CHECK(b < p.B && hkv < p.Hkv && qblk >= 0);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;  // bottom-right aligned causal mask
  const int q0 = qblk * FBM, qw0 = q0 + w * 32;
  const int myq = qw0 + l32;

  const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;

  // Q fragments (B operand of S^T = K Q^T): lane holds Q[myq][16ks + 8h .. +7]
  bf16x8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    if (myq < p.Sq) qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)myq * p.q_ss + ks * 16 + 8 * h);
    else qf[ks] = bf16x8{};
  }

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + FBM + off);
  const int nt = kend > 0 ? (kend + FBN - 1) / FBN : 0;

  bf16x8 kreg[4], vreg[4];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tid + FNT * r, row = i / kChunks, c = i % kChunks, key = t * FBN + row;
      if (key < sk) {
        kreg[r] = *reinterpret_cast<const bf16x8*>(K + (int64_t)key * p.k_ss + c * 8);
        vreg[r] = *reinterpret_cast<const bf16x8*>(Vg + (int64_t)key * p.v_ss + c * 8);
      } else {
        kreg[r] = bf16x8{};
        vreg[r] = bf16x8{};
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tid + FNT * r, row = i / kChunks, c = i % kChunks;
      *reinterpret_cast<bf16x8*>(Kl(buf) + img_off(row, c)) = kreg[r];
      *reinterpret_cast<bf16x8*>(Vl(buf) + img_off(row, c)) = vreg[r];
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const float c = p.scale * kLog2e;

  if (nt > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const int kb = t * FBN;
    if (t + 1 < nt) load_tile(t + 1);
    const bool skip = p.causal && (kb > qw0 + 31 + off);   // whole tile masked for this wave
    if (!skip) {
      // ---- S^T = K Q^T : two 32-key subtiles
      f32x16 s[2];
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        s[n] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
          const bf16x8 a = lds_row_read(Kl(cur), n * 32 + l32, 2 * ks + h);
          s[n] = mfma32(a, qf[ks], s[n]);
        }
      }
      // ---- online softmax (query = lane, keys = registers)
      const bool need_mask = (kb + FBN > sk) || (p.causal && kb + FBN - 1 > qw0 + off);
      float mx = -INFINITY;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = s[n][r] * c;
          if (need_mask) {
            const int key = kb + n * 32 + acc_row(r, h);
            if (key >= sk || (p.causal && key > myq + off)) v = -INFINITY;
          }
          s[n][r] = v;
          mx = fmaxf(mx, v);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m, mx);
      const float msub = (mn == -INFINITY) ? 0.f : mn;
      const float alpha = fast_exp2(m - msub);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(s[n][r] - msub);
          rs += e;  // the softmax normaliser uses the undropped probabilities
          s[n][r] = DROP ? e * drop_factor(p, (uint32_t)bh, myq, kb + n * 32 + acc_row(r, h)) : e;
        }
      l = l * alpha + rs;
      m = mn;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] *= alpha;
      // ---- O^T += V^T P^T : 4 key-steps of 16, 4 d-blocks of 32
      const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack8(s[n], 8 * st);
          const int kk = n * 32 + 16 * st + 4 * h;
#pragma unroll
          for (int db = 0; db < 4; ++db) {
            const int c0 = db * 32 + (g & 1) * 16;
            const bf16x8 a = cat(lds_tr_read(Vl(cur), kk, c0, l16), lds_tr_read(Vl(cur), kk + 8, c0, l16));
            o[db] = mfma32(a, pb, o[db]);
          }
        }
    }
    if (t + 1 < nt) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (myq < p.Sq) {
    bf16* O = (bf16*)p.o + (int64_t)b * p.o_bs + (int64_t)hq * p.o_hs + (int64_t)myq * p.o_ss;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(o[db][4 * gg + j] * inv);
        *reinterpret_cast<bf16x4*>(O + db * 32 + 8 * gg + 4 * h) = v;
      }
    if (h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] = lt > 0.f ? (m + __log2f(lt)) * kLn2 : INFINITY;
  }
}

// ---------------------------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------------------------
constexpr int BBN = 128, BBM = 32, BNT = 256;

// delta[b,h,q] = sum_d dO*O (fp32): 16 lanes x 8 elements per row, 4 rows per wave, 16 per block
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const AttnBwdParams p) {
  const int l16 = threadIdx.x & 15;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t nrows = (int64_t)p.f.B * p.f.Hq * p.f.Sq;
  float acc = 0.f;
  if (row < nrows) {
    const int q = (int)(row % p.f.Sq);
    const int64_t bh = row / p.f.Sq;
    const int hq = (int)(bh % p.f.Hq), b = (int)(bh / p.f.Hq);
    const bf16* O = (const bf16*)p.f.o + (int64_t)b * p.f.o_bs + (int64_t)hq * p.f.o_hs + (int64_t)q * p.f.o_ss;
    const bf16* dO = (const bf16*)p.dout + (int64_t)b * p.do_bs + (int64_t)hq * p.do_hs + (int64_t)q * p.do_ss;
    float a[8], g[8];
    load16(O + l16 * 8, a);
    load16(dO + l16 * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k] * g[k];
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < nrows && l16 == 0) p.delta[row] = acc;
}

// dK / dV kernel: one workgroup = 128 keys of one (batch, kv head), 32 keys per wave with the key on
// the MFMA lane; K and V fragments stay in VGPRs for the whole sweep over the group's query heads
// x (32 * NQ)-row query tiles (Q / dO tiles double-buffered in LDS, one barrier per tile). No
// atomics: dK and dV are complete in registers at the end. NQ = 2 gives every wave four independent
// MFMA accumulation chains per tile (S and dP for two 32-row halves) and halves the barriers.
template <bool DROP, int NQ>
__global__ __launch_bounds__(BNT, 1) void attn_bwd_dkdv_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  constexpr int TM = BBM * NQ;           // query rows per tile
  constexpr int QB = TM * D * 2;
  constexpr int LD = TM * kChunks / BNT;  // 16-byte chunks per thread per operand
  __shared__ __attribute__((aligned(16))) char smem[4 * QB + 2 * 2 * TM * 4];
  auto Ql = [&](int buf) -> char* { return smem + buf * QB; };
  auto dOl = [&](int buf) -> char* { return smem + (2 + buf) * QB; };
  float* lsel = (float*)(smem + 4 * QB);  // [2][TM]
  float* dell = lsel + 2 * TM;            // [2][TM]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, l16 = lane & 15;
  const int nkb = (p.Sk + BBN - 1) / BBN;
  const int kblk = nkb - 1 - (int)(blockIdx.x / (p.B * p.Hkv));  // causal: lightest key blocks last
  const int bhk = blockIdx.x % (p.B * p.Hkv);
  const int b = bhk / p.Hkv, hkv = bhk % p.Hkv;
  const int grp = p.Hq / p.Hkv;
  GRT_DEVICE_CHECK(kblk >= 0 && grp * p.Hkv == p.Hq);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int k0 = kblk * BBN;
  const int kw0 = k0 + w * 32;
  const int mykey = kw0 + l32;
  const float c = p.scale * kLog2e;

  // K / V fragments (B operands of S = Q K^T and dP = dO V^T): lane holds row `mykey`
  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;
  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    if (mykey < sk) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(K + (int64_t)mykey * p.k_ss + ks * 16 + 8 * h);
      vf[ks] = *reinterpret_cast<const bf16x8*>(Vg + (int64_t)mykey * p.v_ss + ks * 16 + 8 * h);
    } else {
      kf[ks] = bf16x8{};
      vf[ks] = bf16x8{};
    }
  }

  f32x16 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  int qstart = 0;
  if (p.causal) qstart = max(0, k0 - off);
  qstart = (qstart / BBM) * BBM;
  const int nqt = qstart < p.Sq ? (p.Sq - qstart + TM - 1) / TM : 0;
  const int total = (k0 < sk) ? nqt * grp : 0;

  bf16x8 qreg[LD], oreg[LD];
  float lse_r = 0.f, del_r = 0.f;
  auto load_q = [&](int it) {
    const int hq = hkv * grp + it / nqt;
    const int qt = qstart + (it % nqt) * TM;
    const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
    const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs;
#pragma unroll
    for (int r = 0; r < LD; ++r) {
      const int i = tid + BNT * r, row = i / kChunks, ch = i % kChunks, q = qt + row;
      if (q < p.Sq) {
        qreg[r] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)q * p.q_ss + ch * 8);
        oreg[r] = *reinterpret_cast<const bf16x8*>(dO + (int64_t)q * P.do_ss + ch * 8);
      } else {
        qreg[r] = bf16x8{};
        oreg[r] = bf16x8{};
      }
    }
    if (tid < TM) {
      const int q = qt + tid;
      const int64_t ri = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      lse_r = q < p.Sq ? p.lse[ri] * kLog2e : INFINITY;
      del_r = q < p.Sq ? P.delta[ri] : 0.f;
    }
  };
  auto store_q = [&](int buf) {
#pragma unroll
    for (int r = 0; r < LD; ++r) {
      const int i = tid + BNT * r, row = i / kChunks, ch = i % kChunks;
      *reinterpret_cast<bf16x8*>(Ql(buf) + img_off(row, ch)) = qreg[r];
      *reinterpret_cast<bf16x8*>(dOl(buf) + img_off(row, ch)) = oreg[r];
    }
    if (tid < TM) { lsel[buf * TM + tid] = lse_r; dell[buf * TM + tid] = del_r; }
  };

  if (total > 0) { load_q(0); store_q(0); }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int qt = qstart + (it % nqt) * TM;
    if (it + 1 < total) load_q(it + 1);
    if (!(p.causal && (kw0 > qt + TM - 1 + off))) {  // else: all 32 keys after every row of the tile
      f32x16 s[NQ], dp[NQ];
#pragma unroll
      for (int n = 0; n < NQ; ++n) { s[n] = f32x16{}; dp[n] = f32x16{}; }
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks)
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
          s[n] = mfma32(lds_row_read(Ql(cur), n * 32 + l32, 2 * ks + h), kf[ks], s[n]);
          dp[n] = mfma32(lds_row_read(dOl(cur), n * 32 + l32, 2 * ks + h), vf[ks], dp[n]);
        }
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const int qn = qt + n * 32;
        const bool need_mask = (k0 + BBN > sk) || (p.causal && kw0 + 31 > qn + off) || (qn + 32 > p.Sq);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const f32x4 ls = *reinterpret_cast<const f32x4*>(lsel + cur * TM + n * 32 + 8 * gg + 4 * h);
          const f32x4 de = *reinterpret_cast<const f32x4*>(dell + cur * TM + n * 32 + 8 * gg + 4 * h);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * gg + j;
            const int q = qn + 8 * gg + 4 * h + j;
            float pv = fast_exp2(s[n][r] * c - ls[j]);
            if (need_mask && (mykey >= sk || q >= p.Sq || (p.causal && mykey > q + off))) pv = 0.f;
            if (DROP) {
              const uint32_t bhq = (uint32_t)(b * p.Hq + hkv * grp + it / nqt);
              const float z = drop_factor(p, bhq, q, mykey);
              s[n][r] = pv * z;                   // dV uses the dropped probabilities
              dp[n][r] = pv * (dp[n][r] * z - de[j]);
            } else {
              s[n][r] = pv;
              dp[n][r] = pv * (dp[n][r] - de[j]);
            }
          }
        }
      }
#pragma unroll
      for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pb = pack8(s[n], 8 * st);
          const bf16x8 sb = pack8(dp[n], 8 * st);
          const int kk = n * 32 + 16 * st + 4 * h;
#pragma unroll
          for (int db = 0; db < 4; ++db) {
            const int c0 = db * 32 + (g & 1) * 16;
            const bf16x8 oa = cat(lds_tr_read(dOl(cur), kk, c0, l16), lds_tr_read(dOl(cur), kk + 8, c0, l16));
            dv[db] = mfma32(oa, pb, dv[db]);
            const bf16x8 qa = cat(lds_tr_read(Ql(cur), kk, c0, l16), lds_tr_read(Ql(cur), kk + 8, c0, l16));
            dk[db] = mfma32(qa, sb, dk[db]);
          }
        }
    }
    if (it + 1 < total) store_q(cur ^ 1);
    __syncthreads();
  }

  if (mykey < p.Sk) {
    bf16* dK = (bf16*)P.dk + (int64_t)b * P.dk_bs + (int64_t)hkv * P.dk_hs + (int64_t)mykey * P.dk_ss;
    bf16* dV = (bf16*)P.dv + (int64_t)b * P.dv_bs + (int64_t)hkv * P.dv_hs + (int64_t)mykey * P.dv_ss;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 a, v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          a[j] = static_cast<bf16>(dk[db][4 * gg + j] * p.scale);
          v[j] = static_cast<bf16>(dv[db][4 * gg + j]);
        }
        *reinterpret_cast<bf16x4*>(dK + db * 32 + 8 * gg + 4 * h) = a;
        *reinterpret_cast<bf16x4*>(dV + db * 32 + 8 * gg + 4 * h) = v;
      }
  }
}

// dQ kernel: the forward's structure (32 query rows per wave, query on the MFMA lane, K/V tiles of
// 64 keys double-buffered in LDS). S^T = K Q^T and dP^T = V dO^T are recomputed, dS^T stays in
// registers and feeds dQ^T += K^T dS^T as the B operand (K^T by transposed reads of the same K
// tile). lse and delta are lane-local. No atomics, dQ written once in bf16.
template <bool DROP>
__global__ __launch_bounds__(FNT, 2) void attn_bwd_dq_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) char smem[4 * kTileBytes];  // K[2], V[2]
  auto Kl = [&](int buf) -> char* { return smem + buf * kTileBytes; };
  auto Vl = [&](int buf) -> char* { return smem + (2 + buf) * kTileBytes; };

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, l16 = lane & 15;
  const int nqb = (p.Sq + FBM - 1) / FBM;
  const int BH = p.B * p.Hq;
  const int qblk = nqb - 1 - (int)(blockIdx.x / BH);
  const int bh = blockIdx.x % BH;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int q0 = qblk * FBM, qw0 = q0 + w * 32;
  const int myq = qw0 + l32;
  const bool qok = myq < p.Sq;

  const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
  const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs;
  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;

  bf16x8 qf[D / 16], of[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    if (qok) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)myq * p.q_ss + ks * 16 + 8 * h);
      of[ks] = *reinterpret_cast<const bf16x8*>(dO + (int64_t)myq * P.do_ss + ks * 16 + 8 * h);
    } else {
      qf[ks] = bf16x8{};
      of[ks] = bf16x8{};
    }
  }
  const int64_t ri = ((int64_t)b * p.Hq + hq) * p.Sq + (qok ? myq : 0);
  const float lse2 = qok ? p.lse[ri] * kLog2e : INFINITY;
  const float dlt = qok ? P.delta[ri] : 0.f;
  const float c = p.scale * kLog2e;

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + FBM + off);
  const int nt = kend > 0 ? (kend + FBN - 1) / FBN : 0;

  bf16x8 kreg[4], vreg[4];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tid + FNT * r, row = i / kChunks, ch = i % kChunks, key = t * FBN + row;
      if (key < sk) {
        kreg[r] = *reinterpret_cast<const bf16x8*>(K + (int64_t)key * p.k_ss + ch * 8);
        vreg[r] = *reinterpret_cast<const bf16x8*>(Vg + (int64_t)key * p.v_ss + ch * 8);
      } else {
        kreg[r] = bf16x8{};
        vreg[r] = bf16x8{};
      }
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = tid + FNT * r, row = i / kChunks, ch = i % kChunks;
      *reinterpret_cast<bf16x8*>(Kl(buf) + img_off(row, ch)) = kreg[r];
      *reinterpret_cast<bf16x8*>(Vl(buf) + img_off(row, ch)) = vreg[r];
    }
  };

  f32x16 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x16{};

  if (nt > 0) { load_tile(0); store_tile(0); }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const int kb = t * FBN;
    if (t + 1 < nt) load_tile(t + 1);
    const bool skip = p.causal && (kb > qw0 + 31 + off);
    if (!skip) {
      const bool need_mask = (kb + FBN > sk) || (p.causal && kb + FBN - 1 > qw0 + off);
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) {
          s = mfma32(lds_row_read(Kl(cur), n * 32 + l32, 2 * ks + h), qf[ks], s);
          dp = mfma32(lds_row_read(Vl(cur), n * 32 + l32, 2 * ks + h), of[ks], dp);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float pv = fast_exp2(s[r] * c - lse2);
          const int key = kb + n * 32 + acc_row(r, h);
          if (need_mask) {
            if (key >= sk || (p.causal && key > myq + off)) pv = 0.f;
          }
          const float z = DROP ? drop_factor(p, (uint32_t)bh, myq, key) : 1.f;
          s[r] = pv * (dp[r] * z - dlt);
        }
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 sb = pack8(s, 8 * st);
          const int kk = n * 32 + 16 * st + 4 * h;
#pragma unroll
          for (int db = 0; db < 4; ++db) {
            const int c0 = db * 32 + (g & 1) * 16;
            const bf16x8 a = cat(lds_tr_read(Kl(cur), kk, c0, l16), lds_tr_read(Kl(cur), kk + 8, c0, l16));
            dq[db] = mfma32(a, sb, dq[db]);
          }
        }
      }
    }
    if (t + 1 < nt) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (qok) {
    bf16* dQ = (bf16*)P.dq + (int64_t)b * P.dq_bs + (int64_t)hq * P.dq_hs + (int64_t)myq * P.dq_ss;
#pragma unroll
    for (int db = 0; db < 4; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(dq[db][4 * gg + j] * p.scale);
        *reinterpret_cast<bf16x4*>(dQ + db * 32 + 8 * gg + 4 * h) = v;
      }
  }
}

}  // namespace

void attn_fwd(const AttnParams& p, hipStream_t s) {
  const int nqb = (p.Sq + FBM - 1) / FBM;
  const dim3 grid((unsigned)(nqb * p.B * p.Hq));
  if (p.drop_thresh) hipLaunchKernelGGL(attn_fwd_kernel<true>, grid, dim3(FNT), 0, s, p);
  else hipLaunchKernelGGL(attn_fwd_kernel<false>, grid, dim3(FNT), 0, s, p);
}

int64_t attn_bwd_workspace_floats(int B, int Hq, int Sq, int Dh) {
  (void)Dh;
  return (int64_t)B * Hq * Sq;  // delta
}

void attn_bwd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = (int64_t)p.f.B * p.f.Hq * p.f.Sq;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, s, p);
  const int nkb = (p.f.Sk + BBN - 1) / BBN;
  const int nqb = (p.f.Sq + FBM - 1) / FBM;
  const dim3 g1((unsigned)(nkb * p.f.B * p.f.Hkv)), g2((unsigned)(nqb * p.f.B * p.f.Hq));
  static const int nq = [] { const char* e = getenv("GRT_ATTN_BWD_NQ"); return e ? atoi(e) : 2; }();
  if (p.f.drop_thresh) {
    if (nq == 1) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<true, 1>), g1, dim3(BNT), 0, s, p);
    else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<true, 2>), g1, dim3(BNT), 0, s, p);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, g2, dim3(FNT), 0, s, p);
  } else {
    if (nq == 1) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<false, 1>), g1, dim3(BNT), 0, s, p);
    else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<false, 2>), g1, dim3(BNT), 0, s, p);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, g2, dim3(FNT), 0, s, p);
  }
}

}  // namespace grt
