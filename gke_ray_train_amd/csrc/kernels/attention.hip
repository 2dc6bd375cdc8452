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

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------------------------
constexpr int FBM = 128, FBN = 64, FNT = 256;
constexpr int kTileBytes = FBN * D * 2;  // 16 KiB

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
          s[n][r] = e;
          rs += e;
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

// delta[b,h,q] = sum_d dO*O   (fp32), one wave per (b, h, q) row
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const AttnBwdParams p) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nrows = (int64_t)p.f.B * p.f.Hq * p.f.Sq;
  if (row >= nrows) return;
  const int q = (int)(row % p.f.Sq);
  const int64_t bh = row / p.f.Sq;
  const int hq = (int)(bh % p.f.Hq), b = (int)(bh / p.f.Hq);
  const bf16* O = (const bf16*)p.f.o + (int64_t)b * p.f.o_bs + (int64_t)hq * p.f.o_hs + (int64_t)q * p.f.o_ss;
  const bf16* dO = (const bf16*)p.dout + (int64_t)b * p.do_bs + (int64_t)hq * p.do_hs + (int64_t)q * p.do_ss;
  float acc = 0.f;
  if (lane < D / 8) {
    float a[8], g[8];
    load16(O + lane * 8, a);
    load16(dO + lane * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k] * g[k];
  }
  acc = wave_sum(acc);
  if (lane == 0) p.delta[row] = acc;
}

__global__ __launch_bounds__(BNT, 1) void attn_bwd_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  // LDS: K img [128][D], V img [128][D], Q img [2][32][D], dO img [2][32][D], dS^T [128][32],
  // lse/delta [2][32]
  constexpr int KB = BBN * D * 2, QB = BBM * D * 2, SB = BBN * BBM * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * KB + 4 * QB + SB + 2 * 2 * BBM * 4];
  char* Kl = smem;
  char* Vl = smem + KB;
  auto Ql = [&](int buf) -> char* { return smem + 2 * KB + buf * QB; };
  auto dOl = [&](int buf) -> char* { return smem + 2 * KB + (2 + buf) * QB; };
  char* dSl = smem + 2 * KB + 4 * QB;
  float* lsel = (float*)(smem + 2 * KB + 4 * QB + SB);  // [2][32]
  float* dell = lsel + 2 * BBM;                          // [2][32]

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, l16 = lane & 15;
  const int nkb = (p.Sk + BBN - 1) / BBN;
  const int kblk = blockIdx.x % nkb;
  const int bhk = blockIdx.x / nkb;
  const int b = bhk / p.Hkv, hkv = bhk % p.Hkv;
  const int grp = p.Hq / p.Hkv;
  const int sk = p.seqlens_k ? min(p.Sk, p.seqlens_k[b]) : p.Sk;
  const int off = p.Sk - p.Sq;
  const int k0 = kblk * BBN;
  const int kw0 = k0 + w * 32;
  const int mykey = kw0 + l32;
  const float c = p.scale * kLog2e;

  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + (int64_t)hkv * p.v_hs;

  // K, V tiles of this workgroup -> LDS (8 chunks per thread each)
#pragma unroll
  for (int r = 0; r < (BBN * kChunks) / BNT; ++r) {
    const int i = tid + BNT * r, row = i / kChunks, ch = i % kChunks, key = k0 + row;
    bf16x8 kv = bf16x8{}, vv = bf16x8{};
    if (key < sk) {
      kv = *reinterpret_cast<const bf16x8*>(K + (int64_t)key * p.k_ss + ch * 8);
      vv = *reinterpret_cast<const bf16x8*>(Vg + (int64_t)key * p.v_ss + ch * 8);
    }
    *reinterpret_cast<bf16x8*>(Kl + img_off(row, ch)) = kv;
    *reinterpret_cast<bf16x8*>(Vl + img_off(row, ch)) = vv;
  }

  f32x16 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { dk[i] = f32x16{}; dv[i] = f32x16{}; }

  // first query row that can see this key block
  int qstart = 0;
  if (p.causal) qstart = max(0, k0 - off);
  qstart = (qstart / BBM) * BBM;
  const int nqt = qstart < p.Sq ? (p.Sq - qstart + BBM - 1) / BBM : 0;
  const int total = nqt * grp;  // (head, q-tile) iterations

  bf16x8 qreg[2], oreg[2];
  float lse_r = 0.f, del_r = 0.f;
  auto load_q = [&](int it) {
    const int hq = hkv * grp + it / nqt;
    const int qt = qstart + (it % nqt) * BBM;
    const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + (int64_t)hq * p.q_hs;
    const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + (int64_t)hq * P.do_hs;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + BNT * r, row = i / kChunks, ch = i % kChunks, q = qt + row;
      if (q < p.Sq) {
        qreg[r] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)q * p.q_ss + ch * 8);
        oreg[r] = *reinterpret_cast<const bf16x8*>(dO + (int64_t)q * P.do_ss + ch * 8);
      } else {
        qreg[r] = bf16x8{};
        oreg[r] = bf16x8{};
      }
    }
    if (tid < BBM) {
      const int q = qt + tid;
      const int64_t ri = ((int64_t)b * p.Hq + hq) * p.Sq + q;
      lse_r = q < p.Sq ? p.lse[ri] * kLog2e : INFINITY;
      del_r = q < p.Sq ? P.delta[ri] : 0.f;
    }
  };
  auto store_q = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + BNT * r, row = i / kChunks, ch = i % kChunks;
      *reinterpret_cast<bf16x8*>(Ql(buf) + img_off(row, ch)) = qreg[r];
      *reinterpret_cast<bf16x8*>(dOl(buf) + img_off(row, ch)) = oreg[r];
    }
    if (tid < BBM) { lsel[buf * BBM + tid] = lse_r; dell[buf * BBM + tid] = del_r; }
  };

  if (total > 0) { load_q(0); store_q(0); }
  __syncthreads();

  for (int it = 0; it < total; ++it) {
    const int cur = it & 1;
    const int hq = hkv * grp + it / nqt;
    const int qt = qstart + (it % nqt) * BBM;
    if (it + 1 < total) load_q(it + 1);

    // ---- S = Q K^T and dP = dO V^T (key on lane, q on registers)
    f32x16 s = f32x16{}, dp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      const bf16x8 kb = lds_row_read(Kl, w * 32 + l32, 2 * ks + h);
      const bf16x8 qa = lds_row_read(Ql(cur), l32, 2 * ks + h);
      s = mfma32(qa, kb, s);
      const bf16x8 vb = lds_row_read(Vl, w * 32 + l32, 2 * ks + h);
      const bf16x8 oa = lds_row_read(dOl(cur), l32, 2 * ks + h);
      dp = mfma32(oa, vb, dp);
    }
    // ---- P, dS
    const bool need_mask = (k0 + BBN > sk) || (p.causal && kw0 + 31 > qt + off) || (qt + BBM > p.Sq);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qi = acc_row(r, h);
      const int q = qt + qi;
      float pv = fast_exp2(s[r] * c - lsel[cur * BBM + qi]);
      if (need_mask && (mykey >= sk || q >= p.Sq || (p.causal && mykey > q + off))) pv = 0.f;
      s[r] = pv;
      dp[r] = pv * (dp[r] - dell[cur * BBM + qi]);
    }
    // ---- dV^T += dO^T P ; dK^T += Q^T dS   (A operands via transposed LDS reads)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const bf16x8 pb = pack8(s, 8 * st);
      const bf16x8 sb = pack8(dp, 8 * st);
      const int kk = 16 * st + 4 * h;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int c0 = db * 32 + (g & 1) * 16;
        const bf16x8 oa = cat(lds_tr_read(dOl(cur), kk, c0, l16), lds_tr_read(dOl(cur), kk + 8, c0, l16));
        dv[db] = mfma32(oa, pb, dv[db]);
        const bf16x8 qa = cat(lds_tr_read(Ql(cur), kk, c0, l16), lds_tr_read(Ql(cur), kk + 8, c0, l16));
        dk[db] = mfma32(qa, sb, dk[db]);
      }
    }
    // ---- dS^T -> LDS [key][q] (bf16), 4 x 8-byte writes per lane
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(dp[4 * gg + j]);
      *reinterpret_cast<bf16x4*>(dSl + (w * 32 + l32) * (BBM * 2) + (8 * gg + 4 * h) * 2) = v;
    }
    __syncthreads();
    // ---- dQ[q][d-block w] += dS[q][128 keys] K[128 keys][d]
    {
      f32x16 dq = f32x16{};
#pragma unroll
      for (int ks = 0; ks < BBN / 16; ++ks) {
        // A: lane holds dS[q = l32][key = 16ks + 8h + j]  (tr read of the [key][q] image, 64-B rows)
        const int kr = 16 * ks + 8 * h;
        const int qq = (g & 1) * 16 + 4 * (l16 & 3);
        const char* a0 = dSl + (kr + (l16 >> 2)) * (BBM * 2) + qq * 2;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 4 * BBM * 2));
        // B: lane holds K[key = 16ks + 8h + j][d = 32w + l32]
        const int c0 = w * 32 + (g & 1) * 16;
        const bf16x8 kbv = cat(lds_tr_read(Kl, kr, c0, l16), lds_tr_read(Kl, kr + 4, c0, l16));
        dq = mfma32(cat(lo, hi), kbv, dq);
      }
      float* dqa = P.dq_acc + (((int64_t)b * p.Hq + hq) * p.Sq) * D;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qt + acc_row(r, h);
        if (q < p.Sq) atomicAdd(dqa + (int64_t)q * D + w * 32 + l32, dq[r] * p.scale);
      }
    }
    if (it + 1 < total) store_q(cur ^ 1);
    __syncthreads();
  }

  // ---- write dK, dV (lane = key, registers = d)
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

// dq (bf16, strided) = dq_acc (fp32, [B, Hq, Sq, D])
__global__ __launch_bounds__(256) void attn_dq_convert_kernel(const AttnBwdParams p) {
  const int64_t n = (int64_t)p.f.B * p.f.Hq * p.f.Sq * (D / 8);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % (D / 8));
    const int64_t row = i / (D / 8);
    const int q = (int)(row % p.f.Sq);
    const int64_t bh = row / p.f.Sq;
    const int hq = (int)(bh % p.f.Hq), b = (int)(bh / p.f.Hq);
    float a[8];
    load16(p.dq_acc + row * D + c * 8, a);
    load16(p.dq_acc + row * D + c * 8 + 4, a + 4);
    bf16* dst = (bf16*)p.dq + (int64_t)b * p.dq_bs + (int64_t)hq * p.dq_hs + (int64_t)q * p.dq_ss + c * 8;
    store16(dst, a);
  }
}

}  // namespace

void attn_fwd(const AttnParams& p, hipStream_t s) {
  const int nqb = (p.Sq + FBM - 1) / FBM;
  const dim3 grid((unsigned)(nqb * p.B * p.Hq));
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(FNT), 0, s, p);
}

int64_t attn_bwd_workspace_floats(int B, int Hq, int Sq, int Dh) {
  return (int64_t)B * Hq * Sq * Dh + (int64_t)B * Hq * Sq;
}

void attn_bwd(const AttnBwdParams& p, hipStream_t s) {
  const int64_t rows = (int64_t)p.f.B * p.f.Hq * p.f.Sq;
  (void)hipMemsetAsync(p.dq_acc, 0, sizeof(float) * rows * D, s);
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, p);
  const int nkb = (p.f.Sk + BBN - 1) / BBN;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3((unsigned)(nkb * p.f.B * p.f.Hkv)), dim3(BNT), 0, s, p);
  int64_t g = (rows * (D / 8) + 255) / 256;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(attn_dq_convert_kernel, dim3((unsigned)g), dim3(256), 0, s, p);
}

}  // namespace grt
