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
//   forward and dQ, per wave = 32 query rows on the MFMA lane:
//     S^T[key][q] = K · Q^T  (A = K rows from LDS, B = Q rows held in VGPRs) -> row max / row sum
//                  of the online softmax are lane-local (+ one permlane32 swap);
//     O^T[d][q] += V^T · P^T, dQ^T += K^T · dS^T  (A = V^T / K^T by ds_read_b64_tr_b16 transposed
//                  reads of the row-major tile, B = the S^T accumulator converted to bf16 in place:
//                  §3 "accumulator tile as the next MFMA's operand");
//   dK / dV, per wave = 32 keys on the MFMA lane, K / V fragments in VGPRs for the whole sweep:
//     S = Q·K^T, dP = dO·V^T, then dV^T += dO^T · P and dK^T += Q^T · dS (transposed reads).
//   No atomics anywhere: dQ and dK / dV come from separate kernels, each complete in registers.
// Pipeline shared by the three kernels (cdna_hip_programming.md "Pipelining across barriers"):
//   * the streamed operand (K / V for forward and dQ, Q / dO + row statistics for dK / dV) arrives
//     in 32-row tiles by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) into a 4-slot ring,
//     with the XOR chunk swizzle applied to the per-lane SOURCE address (rule 21); two tiles stay
//     in flight behind a counted vmcnt across a raw s_barrier (never __syncthreads);
//   * software pipeline: the S (and dP) MFMAs of tile t+1 are issued ahead of tile t's VALU work
//     (exponentials, dS) and its accumulation MFMAs, in one basic block;
//   * the loop is unrolled over the ring, so every LDS address is a per-lane base + an immediate;
//   * masks (causal diagonal, key padding) are selects on the tiles that touch them only; padded
//     query rows carry lse = +inf and need none;
//   * forward: deferred rescale of the online softmax (T13).
//   All LDS tiles use the dual row-read / transposed-read XOR image of cdna_hip_programming.md
//   T10 (b), conflict-free for both the ds_read_b128 row reads and the tr_b16 reads.
// Measured on MI355X (B8 S1024 H32 D128 causal, tools/attn_ab.py; profiles/r2_attention.md).
#include <limits.h>
#include <stdlib.h>

#include <type_traits>
#include <utility>

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

// max over lanes l and l ^ 32 by v_permlane32_swap (a VALU op; no LDS round trip): after the
// swap of x with itself, element 0 holds the lower half's value and element 1 the upper's in
// every lane.
__device__ __forceinline__ float halves_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Deferred rescale (cdna_hip_programming.md T13): the running max m only moves when some row of
// the wave sees a tile max more than kDeferLog2 above it, so most tiles skip the O / l rescale;
// between rescales the exponentiated scores are bounded by 2^kDeferLog2 (exact in fp32 l / O,
// bf16 P keeps its relative precision).
constexpr float kDeferLog2 = 8.f;

// 16-byte LDS-DMA per lane to (wave-uniform LDS byte address) + lane * 16; M0 is written in the
// same statement (compiler-reserved). Not tracked by hipcc's waitcnt pass: the kernel counts vmcnt.
__device__ __forceinline__ void lds_dma16(const void* gptr, uint32_t lds_byte_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(gptr), "s"(lds_byte_addr) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}
__device__ __forceinline__ int img_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// f(integral_constant<int, I>) for I in the sequence, unrolled at compile time (ring slots and
// register-set parity stay compile-time constants in the pipelined loops)
template <class F, int... I>
__device__ __forceinline__ void static_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// s_waitcnt vmcnt(4 * tiles): the DMA of `tiles` 4-instruction tiles may stay in flight
__device__ __forceinline__ void wait_tiles4(int tiles) {
  if (tiles >= 4) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (tiles == 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (tiles == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (tiles == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Forward: 4 waves x 32 query rows, 32-key K / V tiles through the ring, 16 MFMAs per tile and
// wave, two workgroups per CU. (A 256-row / 8-wave workgroup, halving the K / V bytes per FLOP,
// measured slower at S = 1024 from the causal tail; an explicit MFMA / VALU interleave by
// sched_group_barrier measured neutral-to-slower: profiles/r2_attention.md.)
// ---------------------------------------------------------------------------------------------
constexpr int F3M = 128, F3N = 32, F3NT = 256, F3NSLOT = 4;
constexpr int F3IMG = F3N * D * 2;   // 8 KiB
constexpr int F3SLOT = 2 * F3IMG;    // K, V

// Workgroup -> (batch*head, q-blocks) of the q-block kernels (forward, dQ; grid: q_grid()).
// sched 0: one q-block per workgroup, heaviest (causal) first.
// sched 1: causal pairs — heavy block nqb-1-j then light block j in one workgroup (equal work per
//   workgroup: no tail of heavy blocks), and the pairs of one (batch, head), then of the heads of one
//   GQA group, dealt to consecutive workgroups of ONE XCD (bijective remap, cdna_hip_programming.md
//   §5 "XCD swizzle must be bijective"): a head's workgroups stream its K / V tiles together, so all
//   but the first read of a tile hit that XCD's L2 instead of going to HBM.
struct QJobs {
  int bh;
  int blk0, blk1;  // blk1 = -1: none (scalars, not an array: a runtime-indexed array is promoted to LDS)
};
__device__ __forceinline__ QJobs q_jobs(int sched, int nqb, int BH) {
  QJobs j;
  if (sched == 1) {
    const int npair = (nqb + 1) >> 1, nwg = BH * npair;
    const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    j.bh = L / npair;
    const int pr = L % npair;
    j.blk0 = nqb - 1 - pr;
    j.blk1 = pr != nqb - 1 - pr ? pr : -1;
  } else {
    j.bh = blockIdx.x % BH;
    j.blk0 = nqb - 1 - (int)(blockIdx.x / BH);
    j.blk1 = -1;
  }
  return j;
}
__host__ __device__ inline unsigned q_grid(int sched, int nqb, int BH) {
  return (unsigned)(sched == 1 ? BH * ((nqb + 1) / 2) : BH * nqb);
}

// NS: ring slots (4: 64 KiB; 5: 80 KiB = half the CU's LDS, the most two workgroups per CU allow)
template <bool DROP, int NS>
__global__ __launch_bounds__(F3NT, 2) void attn_fwd_kernel(const AttnParams p) {
  __shared__ __attribute__((aligned(16))) char smem[NS * F3SLOT];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, l16 = lane & 15;
  const int nqb = (p.Sq + F3M - 1) / F3M;  // grid: the longest sequence
  const int BH = p.B * p.Hq;
  const QJobs jobs = q_jobs(p.sched, nqb, BH);
  const int bh = jobs.bh;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  GRT_DEVICE_CHECK(b < p.B && hkv < p.Hkv && jobs.blk0 >= 0 && jobs.blk0 < nqb);
  // one call per block of this workgroup; inlined twice, so the second block's registers are
  // allocated independently (a loop over the two blocks spilled the dQ kernel)
  auto run_block = [&](const int qblk) {
  int Sq = p.Sq, Sk = p.Sk;
  int64_t tok0 = 0;  // padding-free packing: this sequence's first token row
  if (p.cu_seqlens) {
    tok0 = p.cu_seqlens[b];
    Sq = Sk = p.cu_seqlens[b + 1] - (int)tok0;
    if (qblk * F3M >= Sq) return;  // workgroup-uniform: the sequence is shorter than the longest
  }
  const int sk = p.seqlens_k ? min(Sk, p.seqlens_k[b]) : Sk;
  const int off = Sk - Sq;  // bottom-right aligned causal mask
  const int q0 = qblk * F3M, qw0 = q0 + w * 32;
  const int myq = qw0 + l32;

  const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + tok0 * p.q_ss + (int64_t)hq * p.q_hs;
  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + tok0 * p.k_ss + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + tok0 * p.v_ss + (int64_t)hkv * p.v_hs;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) {
    if (myq < Sq) qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (int64_t)myq * p.q_ss + ks * 16 + 8 * h);
    else qf[ks] = bf16x8{};
  }
  const int klim = p.causal ? min(sk - 1, myq + off) : sk - 1;   // keys <= klim are kept
  const int kmask = p.causal ? min(sk, qw0 + off + 1) : sk;      // tiles reaching past need the mask
  // the wave's last kept key: tiles past it are masked for all 32 rows (the causal band of a
  // 128-row block, 3 - w tiles for wave w) and skip their math (p.skip_dead)
  const int klast = p.skip_dead && p.causal ? min(sk - 1, qw0 + 31 + off) : INT_MAX;

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + F3M + off);
  const int nt = kend > 0 ? (kend + F3N - 1) / F3N : 0;

  const uint32_t smem0 = lds_u32(smem);
  // wave w fills image rows 8w .. 8w+7 of K and V: two 1-KiB pieces of 4 rows per image
  const int row0 = 8 * w + g, row1 = row0 + 4;
  const int ch0 = l16 ^ img_swz(row0), ch1 = l16 ^ img_swz(row1);
  // per-lane source offsets of the two rows, fixed for the whole sweep: a tile inside the sequence
  // then costs one 64-bit add per DMA (the tile base is uniform, SALU); only the tile that crosses
  // the end takes the clamped per-lane row arithmetic (64-bit multiplies: quarter-rate VALU)
  // (32-bit: a row of a 32-row tile times the row stride; one VGPR each)
  const uint32_t ko0 = (uint32_t)(row0 * p.k_ss + ch0 * 8), ko1 = (uint32_t)(row1 * p.k_ss + ch1 * 8);
  const uint32_t vo0 = (uint32_t)(row0 * p.v_ss + ch0 * 8), vo1 = (uint32_t)(row1 * p.v_ss + ch1 * 8);
  auto dma_tile = [&](int t, uint32_t slot_off) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(8 * w * 256));
    if (p.dma_fast && (t + 1) * F3N <= Sk) {
      const bf16* kt = K + (int64_t)(t * F3N) * p.k_ss;
      const bf16* vt = Vg + (int64_t)(t * F3N) * p.v_ss;
      lds_dma16(kt + ko0, dst);
      lds_dma16(vt + vo0, dst + F3IMG);
      lds_dma16(kt + ko1, dst + 1024);
      lds_dma16(vt + vo1, dst + F3IMG + 1024);
      return;
    }
    const int64_t k0r = min(t * F3N + row0, Sk - 1), k1r = min(t * F3N + row1, Sk - 1);  // past Sk: masked
    lds_dma16(K + k0r * p.k_ss + ch0 * 8, dst);
    lds_dma16(Vg + k0r * p.v_ss + ch0 * 8, dst + F3IMG);
    lds_dma16(K + k1r * p.k_ss + ch1 * 8, dst + 1024);
    lds_dma16(Vg + k1r * p.v_ss + ch1 * 8, dst + F3IMG + 1024);
  };
  auto wait_dma = [&](int pending_tiles) { wait_tiles4(pending_tiles); };  // 4 DMA instructions per tile
  // S^T = K Q^T of the tile in slot SL; the 8 K-row fragments are read into registers before the
  // MFMA chain so the reads are in flight together (not one LDS round trip per MFMA)
  auto qk = [&](auto slot_c) {
    constexpr int SL = decltype(slot_c)::value;
    const char* ki = smem + SL * F3SLOT;
    bf16x8 kr[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) kr[ks] = lds_row_read(ki, l32, 2 * ks + h);
    f32x16 s = f32x16{};
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) s = mfma32(kr[ks], qf[ks], s);
    // three K fragments in flight ahead of the MFMA chain (the default schedule waits on each read)
    __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
    return s;
  };
  // -inf on the masked keys of tile t, applied only on tiles that touch the diagonal / key padding
  auto apply_mask = [&](int t, f32x16& s) {
    const int kb = t * F3N;
    if (kb + F3N > kmask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = kb + acc_row(r, h) <= klim ? s[r] : -INFINITY;
    }
  };

  f32x16 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;  // m in log2 units of the scaled scores
  const float c = p.scale * kLog2e;

  // one pipeline step. Order: the branchy parts first (ring wait / barrier / DMA, tile t's mask,
  // row max and deferred rescale), then ONE basic block holding S^T of tile t+1 (independent
  // MFMAs), tile t's exponentials and its P V MFMAs.
  auto step = [&](int t, auto slot_c, f32x16& s_c, f32x16& s_n) {
    constexpr int SL = decltype(slot_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < nt) wait_dma(min(nt, t + NS - 1) - (t + 2));
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < nt) dma_tile(t + NS - 1, (uint32_t)(((SL + NS - 1) % NS) * F3SLOT));

    apply_mask(t, s_c);
    float mx = fmaxf(s_c[0], s_c[1]);
#pragma unroll
    for (int r = 2; r < 16; ++r) mx = fmaxf(mx, s_c[r]);
    mx = halves_max(mx) * c;  // tile row max, log2 units (-inf: every key masked)
    if (__any(mx > m + kDeferLog2)) {
      const float mn = fmaxf(m, mx);
      const float alpha = mn == -INFINITY ? 1.f : fast_exp2(m - mn);
      l *= alpha;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] *= alpha;
      m = mn;
    }
    const float msub = m == -INFINITY ? 0.f : m;

    s_n = qk(std::integral_constant<int, (SL + 1) % NS>{});  // past the end: dropped
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = fast_exp2(fmaf(s_c[r], c, -msub));
      rs += e;  // the softmax normaliser uses the undropped probabilities
      s_c[r] = DROP ? e * drop_factor(p, (uint32_t)bh, myq, t * F3N + acc_row(r, h)) : e;
    }
    l += rs;
    const char* vi = smem + SL * F3SLOT + F3IMG;
    bf16x8 va[2][4];
#pragma unroll
    for (int stp = 0; stp < 2; ++stp) {
      const int kk = 16 * stp + 4 * h;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int c0 = db * 32 + (g & 1) * 16;
        va[stp][db] = cat(lds_tr_read(vi, kk, c0, l16), lds_tr_read(vi, kk + 8, c0, l16));
      }
    }
#pragma unroll
    for (int stp = 0; stp < 2; ++stp) {
      const bf16x8 pb = pack8(s_c, 8 * stp);
#pragma unroll
      for (int db = 0; db < 4; ++db) o[db] = mfma32(va[stp][db], pb, o[db]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
  };

  if (nt > 0) {
    const int pre = min(nt, NS - 1);
    for (int t = 0; t < pre; ++t) dma_tile(t, (uint32_t)(t * F3SLOT));
    wait_dma(pre - 1);
    __builtin_amdgcn_s_barrier();
    // unrolled over whole ring revolutions with an even step count (slot and S register set static)
    constexpr int UNR = NS % 2 == 0 ? NS : 2 * NS;
    f32x16 sA = qk(std::integral_constant<int, 0>{}), sB;
    auto step_i = [&](int t0, auto i_c) {
      constexpr int I = decltype(i_c)::value;
      if constexpr (I & 1) step(t0 + I, std::integral_constant<int, I % NS>{}, sB, sA);
      else step(t0 + I, std::integral_constant<int, I % NS>{}, sA, sB);
    };
    // tiles past klast are masked for every row of this wave: their exponentials would be 0 and
    // their P V products add nothing, so the wave's math stops at ntl and it only keeps the later
    // tiles' barriers and its share of their DMA (the drain below). A separate loop rather than an
    // early exit inside the step: a branch out of the pipelined body spilled 239 VGPRs.
    const int ntl = klast == INT_MAX ? nt : min(nt, max(0, klast / F3N + 1));
    int t = 0;
    for (; t + UNR <= ntl; t += UNR) static_for([&](auto i_c) { step_i(t, i_c); }, std::make_integer_sequence<int, UNR>{});
    static_for([&](auto i_c) { if (t + decltype(i_c)::value < ntl) step_i(t, i_c); }, std::make_integer_sequence<int, UNR - 1>{});
    for (t = ntl; t < nt; ++t) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 1 < nt) wait_dma(min(nt, t + NS - 1) - (t + 2));
      __builtin_amdgcn_s_barrier();
      if (t + NS - 1 < nt) dma_tile(t + NS - 1, (uint32_t)(((t + NS - 1) % NS) * F3SLOT));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  // O rows as 16-byte stores (cdna_hip_programming.md T21): lane l (h = 0) holds columns
  // 8 gg .. 8 gg + 3 of its row and lane l + 32 columns 8 gg + 4 .. 8 gg + 7; one v_permlane32_swap
  // per dword of the (gg, gg + 1) pair gives lanes 0-31 columns 8 gg .. 8 gg + 7 and lanes 32-63
  // columns 8 gg + 8 .. 8 gg + 15 — half the store instructions. Every lane takes part in the swap.
  bf16* O = (bf16*)p.o + (int64_t)b * p.o_bs + (tok0 + min(myq, Sq - 1)) * p.o_ss + (int64_t)hq * p.o_hs;
#pragma unroll
  for (int db = 0; db < 4; ++db)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      union { bf16x4 v; uint32_t u[2]; } a, c2;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a.v[j] = static_cast<bf16>(o[db][8 * gp + j] * inv);
        c2.v[j] = static_cast<bf16>(o[db][8 * gp + 4 + j] * inv);
      }
      const auto r0 = __builtin_amdgcn_permlane32_swap(a.u[0], c2.u[0], false, false);
      const auto r1 = __builtin_amdgcn_permlane32_swap(a.u[1], c2.u[1], false, false);
      if (myq < Sq) {
        *reinterpret_cast<uint4*>(O + db * 32 + 16 * gp + 8 * h) = make_uint4(r0[0], r1[0], r0[1], r1[1]);
        if (p.o_t != nullptr) {  // O^T: this lane's row, head dims d of a (before the swap): one 64-B
          // segment per element across the 32 lanes of a half-wave
          bf16* ot = static_cast<bf16*>(p.o_t) + (int64_t)(hq * D) * p.ot_ld + (p.cu_seqlens ? 0 : (int64_t)b * p.Sq) +
                     tok0 + myq;
          const int d0 = db * 32 + 8 * (2 * gp) + 4 * h, d1 = db * 32 + 8 * (2 * gp + 1) + 4 * h;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            ot[(int64_t)(d0 + j) * p.ot_ld] = a.v[j];
            ot[(int64_t)(d1 + j) * p.ot_ld] = c2.v[j];
          }
        }
      }
    }
  if (myq < Sq) {
    if (h == 0 && p.lse)
      p.lse[((int64_t)b * p.Hq + hq) * p.Sq + myq] = lt > 0.f ? (m + __log2f(lt)) * kLn2 : INFINITY;
  }
  };
  run_block(jobs.blk0);
  if (jobs.blk1 >= 0) {  // every wave is done with the ring (LDS reads, its own DMAs) before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    run_block(jobs.blk1);
  }
}

// ---------------------------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------------------------
// Row statistics live in a padded workspace: per (batch, query head) a row of sq_pad(Sq) floats of
// delta = rowsum(dO * O) and of lse2 = lse * log2(e) (+inf on the padding rows, so their
// probabilities come out exactly 0 with no mask): query tiles of 32 rows never straddle a head, the
// 16-byte DMA pieces are aligned, and no row index needs a bounds check.
__host__ __device__ inline int sq_pad(int Sq) { return (Sq + 31) / 32 * 32; }

__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(const AttnBwdParams p) {
  const int l16 = threadIdx.x & 15;
  const int Sqp = sq_pad(p.f.Sq);
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t nrows = (int64_t)p.f.B * p.f.Hq * Sqp;
  if (row >= nrows) return;
  const int q = (int)(row % Sqp);
  const int64_t bh = row / Sqp;
  float acc = 0.f;
  const int hq = (int)(bh % p.f.Hq), b = (int)(bh / p.f.Hq);
  int Sq = p.f.Sq;
  int64_t tok0 = 0;
  if (p.f.cu_seqlens) {
    tok0 = p.f.cu_seqlens[b];
    Sq = p.f.cu_seqlens[b + 1] - (int)tok0;
  }
  if (q < Sq) {
    const bf16* O = (const bf16*)p.f.o + (int64_t)b * p.f.o_bs + (int64_t)hq * p.f.o_hs + (tok0 + q) * p.f.o_ss;
    const bf16* dO = (const bf16*)p.dout + (int64_t)b * p.do_bs + (int64_t)hq * p.do_hs + (tok0 + q) * p.do_ss;
    float a[8], g[8];
    load16(O + l16 * 8, a);
    load16(dO + l16 * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += a[k] * g[k];
  }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 16);
  if (l16 == 0) {
    float* lse2 = p.delta + nrows;
    p.delta[row] = acc;
    lse2[row] = q < Sq ? p.f.lse[bh * p.f.Sq + q] * kLog2e : INFINITY;
  }
}


// dK / dV: one workgroup = 128 keys of one (batch, kv head), 32 keys per wave on the MFMA lane,
// K / V fragments in registers for the whole sweep over the group's query heads x 32-row query
// tiles (Q / dO tiles and their row statistics through the ring). Per tile the wave does 32 MFMAs
// (S, dP, dV^T, dK^T, 8 each); the S accumulator starts at -inf on masked (query, key) pairs of
// the diagonal / padding tiles. One workgroup (one wave per SIMD) per CU: K / V fragments and the
// dK / dV accumulators take ~450 registers. Heaviest (earliest, causal) key blocks launch first.
// Backward epilogue with the RoPE of the forward undone in registers: the accumulator's element
// (db, 4 gg + j) is head dim d = 32 db + 8 gg + 4 h + j, so the rotation pair (d, d + 64) is
// (db, db + 2) of the same lane — x1 c + x2 s / x2 c - x1 s with the position's cos / sin rows
// (rope_kernel<.., false>), rounded to bf16 once.
// Optional transposed copy of a [tokens, heads x D] gradient for the TN weight-gradient GEMM of the
// fused QKV projection (the producer writes dqkv^T beside dqkv, so no transpose kernel re-reads it):
// element (token, d) of this lane's row at p[d * ld]; p == nullptr when not requested. The 32
// lanes of a half-wave hold 32 consecutive tokens, so each element store is one 64-byte segment.
struct TCopy {
  bf16* p;
  int64_t ld;
};
__device__ __forceinline__ void st_t(const TCopy& tc, int d, const bf16x4& v) {
  if (tc.p != nullptr) {
#pragma unroll
    for (int j = 0; j < 4; ++j) tc.p[(int64_t)(d + j) * tc.ld] = v[j];
  }
}
__device__ __forceinline__ TCopy tcopy(const AttnBwdParams& P, int row0, int head, int64_t tok) {
  if (P.dqkv_t == nullptr) return TCopy{nullptr, 0};
  return TCopy{static_cast<bf16*>(P.dqkv_t) + (int64_t)(row0 + head * D) * P.t_ld + tok, P.t_ld};
}

__device__ __forceinline__ void store_unrotated(const f32x16 (&acc)[4], float scale, const float* __restrict__ cr,
                                                const float* __restrict__ sr, bf16* dst, int h,
                                                const TCopy& tc = TCopy{nullptr, 0}) {
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int d = db * 32 + 8 * gg + 4 * h;
      const f32x4 c = *reinterpret_cast<const f32x4*>(cr + d);
      const f32x4 sn = *reinterpret_cast<const f32x4*>(sr + d);
      bf16x4 lo, hi;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x1 = acc[db][4 * gg + j] * scale, x2 = acc[db + 2][4 * gg + j] * scale;
        lo[j] = static_cast<bf16>(x1 * c[j] + x2 * sn[j]);
        hi[j] = static_cast<bf16>(x2 * c[j] - x1 * sn[j]);
      }
      *reinterpret_cast<bf16x4*>(dst + d) = lo;
      *reinterpret_cast<bf16x4*>(dst + d + D / 2) = hi;
      st_t(tc, d, lo);
      st_t(tc, d + D / 2, hi);
    }
}

constexpr int K2N = 128, K2M = 32, K2NT = 256, K2NSLOT = 4;
constexpr int K2IMG = K2M * D * 2;           // one 32-row image: 8 KiB
constexpr int K2SLOT = 2 * K2IMG + 4 * 1024;  // Q image, dO image, per-wave statistics copy

// (An explicit whole-step interleave — tile t+1's S / dP MFMAs each followed by 5 of tile t's VALU
// ops — measured slower: B8 S1024 H32 backward 428 -> 444 us, GQA 407 -> 451; r3_attn_schedule.md.)
template <bool DROP>
__global__ __launch_bounds__(K2NT, 1) void attn_bwd_dkdv_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) char smem[K2NSLOT * K2SLOT];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int g = lane >> 4, l16 = lane & 15;
  const int BHk = p.B * p.Hkv;
  const int nkb = (p.Sk + K2N - 1) / K2N;
  // sched 0: one key block per workgroup, heaviest (earliest, causal) first; sched 1: key blocks
  // paired light + heavy, the pairs of one (batch, kv head) on one XCD (see q_jobs)
  QJobs jobs;
  if (p.sched == 1) {
    jobs = q_jobs(1, nkb, BHk);
  } else {
    jobs.bh = blockIdx.x % BHk;
    jobs.blk0 = (int)(blockIdx.x / BHk);
    jobs.blk1 = -1;
  }
  const int bhk = jobs.bh;
  const int b = bhk / p.Hkv, hkv = bhk % p.Hkv;
  const int grp = p.Hq / p.Hkv;
  // one call per block of this workgroup; inlined twice, so the second block's registers are
  // allocated independently (a loop over the two blocks spilled the dQ kernel)
  auto run_block = [&](const int kblk) {
  int Sq = p.Sq, Sk = p.Sk;
  int64_t tok0 = 0;  // padding-free packing: this sequence's first token row
  if (p.cu_seqlens) {
    tok0 = p.cu_seqlens[b];
    Sq = Sk = p.cu_seqlens[b + 1] - (int)tok0;
    if (kblk * K2N >= Sk) return;  // workgroup-uniform: the sequence is shorter than the longest
  }
  GRT_DEVICE_CHECK(grp * p.Hkv == p.Hq && kblk * K2N < Sk);
  const int sk = p.seqlens_k ? min(Sk, p.seqlens_k[b]) : Sk;
  const int off = Sk - Sq;
  const int k0 = kblk * K2N, kw0 = k0 + w * 32, mykey = kw0 + l32;
  const float c = p.scale * kLog2e;
  const int Sqp = sq_pad(p.Sq);  // workspace row stride: the longest sequence
  const float* lse2 = P.delta + (int64_t)p.B * p.Hq * Sqp;

  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + tok0 * p.k_ss + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + tok0 * p.v_ss + (int64_t)hkv * p.v_hs;
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

  int qstart = p.causal ? max(0, k0 - off) : 0;
  qstart = (qstart / K2M) * K2M;
  const int nqt = qstart < Sq ? (Sq - qstart + K2M - 1) / K2M : 0;
  const int total = (k0 < sk) ? nqt * grp : 0;
  // per-lane mask: probability of (q, mykey) kept iff mykey < sk and (non-causal or q >= qlim)
  const int qlim = mykey < sk ? (p.causal ? mykey - off : INT_MIN) : INT_MAX;
  // the tile starting at query qt needs the mask iff qt < qmask (diagonal) or the block has padding
  const int qmask = (k0 + K2N > sk) ? INT_MAX : (p.causal ? kw0 + 31 - off : INT_MIN);

  // ---- LDS-DMA of tile j into a slot: wave w fills image rows 8w .. 8w+7 of Q and dO (two 1-KiB
  // pieces each; the XOR swizzle goes on the per-lane SOURCE chunk) and its own copy of the tile's
  // 32 lse2 and 32 delta values (lanes 0-7 / 8-15; lanes 16-63 repeat them).
  const uint32_t smem0 = lds_u32(smem);
  const int row0 = 8 * w + g, row1 = row0 + 4;
  const int ch0 = l16 ^ img_swz(row0), ch1 = l16 ^ img_swz(row1);
  const int sl = l16 & 7;
  const int64_t st_lane = (l16 < 8 ? (int64_t)p.B * p.Hq * Sqp : 0) + 4 * sl;  // lse2 | delta
  const uint32_t qo0 = (uint32_t)(row0 * p.q_ss + ch0 * 8), qo1 = (uint32_t)(row1 * p.q_ss + ch1 * 8);
  const uint32_t oo0 = (uint32_t)(row0 * P.do_ss + ch0 * 8), oo1 = (uint32_t)(row1 * P.do_ss + ch1 * 8);
  auto dma_tile = [&](int hq, int qt, uint32_t slot_off) {
    const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + tok0 * p.q_ss + (int64_t)hq * p.q_hs;
    const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + tok0 * P.do_ss + (int64_t)hq * P.do_hs;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(8 * w * 256));
    if (p.dma_fast && qt + K2M <= Sq) {  // tile inside the sequence: uniform base + fixed per-lane offsets
      const bf16* qb = Q + (int64_t)qt * p.q_ss;
      const bf16* ob = dO + (int64_t)qt * P.do_ss;
      lds_dma16(qb + qo0, dst);
      lds_dma16(ob + oo0, dst + K2IMG);
      lds_dma16(qb + qo1, dst + 1024);
      lds_dma16(ob + oo1, dst + K2IMG + 1024);
    } else {
      const int64_t q0r = min(qt + row0, Sq - 1), q1r = min(qt + row1, Sq - 1);  // past Sq: lse2 = +inf
      lds_dma16(Q + q0r * p.q_ss + ch0 * 8, dst);
      lds_dma16(dO + q0r * P.do_ss + ch0 * 8, dst + K2IMG);
      lds_dma16(Q + q1r * p.q_ss + ch1 * 8, dst + 1024);
      lds_dma16(dO + q1r * P.do_ss + ch1 * 8, dst + K2IMG + 1024);
    }
    const int64_t ri = ((int64_t)b * p.Hq + hq) * Sqp + qt;
    lds_dma16(P.delta + st_lane + ri,
              __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(2 * K2IMG + w * 1024)));
  };
  auto wait_dma = [&](int pending_tiles) {  // 5 DMA instructions per tile
    if (pending_tiles >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (pending_tiles == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // S and dP of the tile at query qt in slot SL (query rows in registers, key on the lane)
  auto sdp = [&](int qt, auto slot_c, f32x16& s, f32x16& dp) {
    constexpr int SL = decltype(slot_c)::value;
    const char* qi = smem + SL * K2SLOT;
    s = f32x16{};
    if (qt < qmask) {  // wave-uniform: the tile touches the diagonal / key padding
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = qt + acc_row(r, h) >= qlim ? 0.f : -INFINITY;
    }
    dp = f32x16{};
    bf16x8 fq[D / 16], fd[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      fq[ks] = lds_row_read(qi, l32, 2 * ks + h);
      fd[ks] = lds_row_read(qi + K2IMG, l32, 2 * ks + h);
    }
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      s = mfma32(fq[ks], kf[ks], s);
      dp = mfma32(fd[ks], vf[ks], dp);
    }
    // keep three fragment pairs in flight ahead of the MFMAs that consume them (the default
    // schedule issues each read right before its MFMA behind lgkmcnt(0): one wave per SIMD has no
    // partner wave to cover that latency)
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
  };

  // tile cursors (query head, query start): the tile being consumed, the next one, the DMA one
  int cur_h = 0, cur_q = qstart;
  auto advance = [&](int& hh, int& qq) {
    qq += K2M;
    if (qq >= Sq) { qq = qstart; ++hh; }
  };
  int nxt_h = cur_h, nxt_q = cur_q;
  advance(nxt_h, nxt_q);
  int dma_h = 0, dma_q = qstart;

  auto step = [&](int t, auto slot_c, f32x16& s_c, f32x16& dp_c, f32x16& s_n, f32x16& dp_n) {
    constexpr int SL = decltype(slot_c)::value;
    // tile t+1 landed for every wave, and every wave is done with tile t-1 (its slot is refilled)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < total) wait_dma(min(total, t + K2NSLOT - 1) - (t + 2));
    __builtin_amdgcn_s_barrier();
    if (t + K2NSLOT - 1 < total) {
      dma_tile(hkv * grp + dma_h, dma_q, (uint32_t)(((SL + K2NSLOT - 1) % K2NSLOT) * K2SLOT));
      advance(dma_h, dma_q);
    }

    const char* qi = smem + SL * K2SLOT;
    const float* st = reinterpret_cast<const float*>(qi + 2 * K2IMG + w * 1024);
    f32x4 lsv[4], dev[4];  // tile t's row statistics, read before tile t+1's S / dP
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      lsv[gg] = *reinterpret_cast<const f32x4*>(st + 8 * gg + 4 * h);
      dev[gg] = *reinterpret_cast<const f32x4*>(st + 32 + 8 * gg + 4 * h);
    }

    sdp(nxt_q, std::integral_constant<int, (SL + 1) % K2NSLOT>{}, s_n, dp_n);  // past the end: dropped

    bf16x8 pb[2], sb[2];
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const f32x4 ls = lsv[gg];
      const f32x4 de = dev[gg];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * gg + j;
        const float pv = fast_exp2(fmaf(s_c[r], c, -ls[j]));
        if (DROP) {
          const float z = drop_factor(p, (uint32_t)(b * p.Hq + hkv * grp + cur_h), cur_q + 8 * gg + 4 * h + j, mykey);
          s_c[r] = pv * z;                  // dV uses the dropped probabilities
          dp_c[r] = pv * (dp_c[r] * z - de[j]);
        } else {
          s_c[r] = pv;
          dp_c[r] = pv * (dp_c[r] - de[j]);
        }
      }
    }
    pb[0] = pack8(s_c, 0);
    pb[1] = pack8(s_c, 8);
    sb[0] = pack8(dp_c, 0);
    sb[1] = pack8(dp_c, 8);
    // dV^T += dO^T P, dK^T += Q^T dS (transposed reads of tile t's images)
    bf16x8 oa[2][4], qa[2][4];
#pragma unroll
    for (int stp = 0; stp < 2; ++stp) {
      const int kk = 16 * stp + 4 * h;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int c0 = db * 32 + (g & 1) * 16;
        oa[stp][db] = cat(lds_tr_read(qi + K2IMG, kk, c0, l16), lds_tr_read(qi + K2IMG, kk + 8, c0, l16));
        qa[stp][db] = cat(lds_tr_read(qi, kk, c0, l16), lds_tr_read(qi, kk + 8, c0, l16));
      }
    }
#pragma unroll
    for (int stp = 0; stp < 2; ++stp)
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        dv[db] = mfma32(oa[stp][db], pb[stp], dv[db]);
        dk[db] = mfma32(qa[stp][db], sb[stp], dk[db]);
      }
    // the transposed reads run three fragments (6 reads) ahead of their MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
    cur_h = nxt_h;
    cur_q = nxt_q;
    advance(nxt_h, nxt_q);
  };

  if (total > 0) {
    const int pre = min(total, K2NSLOT - 1);
    for (int j = 0; j < pre; ++j) {
      dma_tile(hkv * grp + dma_h, dma_q, (uint32_t)(j * K2SLOT));
      advance(dma_h, dma_q);
    }
    wait_dma(pre - 1);
    __builtin_amdgcn_s_barrier();
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    f32x16 sA, dpA, sB, dpB;
    sdp(cur_q, I0{}, sA, dpA);
    int t = 0;
    for (; t + K2NSLOT <= total; t += K2NSLOT) {  // one ring revolution: slots 0..3, register sets A/B
      step(t, I0{}, sA, dpA, sB, dpB);
      step(t + 1, I1{}, sB, dpB, sA, dpA);
      step(t + 2, I2{}, sA, dpA, sB, dpB);
      step(t + 3, I3{}, sB, dpB, sA, dpA);
    }
    if (t < total) step(t, I0{}, sA, dpA, sB, dpB);
    if (t + 1 < total) step(t + 1, I1{}, sB, dpB, sA, dpA);
    if (t + 2 < total) step(t + 2, I2{}, sA, dpA, sB, dpB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (mykey < Sk) {
    bf16* dK = (bf16*)P.dk + (int64_t)b * P.dk_bs + (int64_t)hkv * P.dk_hs + (tok0 + mykey) * P.dk_ss;
    bf16* dV = (bf16*)P.dv + (int64_t)b * P.dv_bs + (int64_t)hkv * P.dv_hs + (tok0 + mykey) * P.dv_ss;
    const int64_t tokg = (p.cu_seqlens ? 0 : (int64_t)b * p.Sk) + tok0 + mykey;
    const TCopy tk = tcopy(P, P.t_row_k, hkv, tokg), tv = tcopy(P, P.t_row_v, hkv, tokg);
    if (P.rope_cos)
      store_unrotated(dk, p.scale, P.rope_cos + (int64_t)mykey * (D / 2), P.rope_sin + (int64_t)mykey * (D / 2), dK, h,
                      tk);
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
        if (!P.rope_cos) {
          *reinterpret_cast<bf16x4*>(dK + db * 32 + 8 * gg + 4 * h) = a;
          st_t(tk, db * 32 + 8 * gg + 4 * h, a);
        }
        *reinterpret_cast<bf16x4*>(dV + db * 32 + 8 * gg + 4 * h) = v;
        st_t(tv, db * 32 + 8 * gg + 4 * h, v);
      }
  }
  };
  run_block(jobs.blk0);
  if (jobs.blk1 >= 0) {  // every wave is done with the ring (LDS reads, its own DMAs) before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    run_block(jobs.blk1);
  }
}

// dK / dV, wave-pair form (default without dropout; GRT_ATTN_DKDV=1 selects the 4-wave kernel above). The
// 4-wave kernel holds K, V, dK^T and dV^T of its 32 keys in one wave (~440 registers: one wave per
// SIMD, nothing covers its exponentials, LDS reads and barrier; 25 % MFMA busy,
// profiles/r3_pmc_kernel_zoo.md). Here the work of 32 keys is split over a wave PAIR on one SIMD
// (waves w and w + 4 share a SIMD):
//   S-wave  (w < 4): K fragments, dV^T accumulators: S = Q K^T, P = exp2(c S - lse2) -> LDS,
//                    dV^T += dO^T P;
//   dP-wave (w >= 4): V fragments, dK^T accumulators: dP = dO V^T, then for the PREVIOUS tile
//                    (whose P its partner published before this tile's barrier)
//                    dS = P (dP - delta), dK^T += Q^T dS.
// Each wave fits in < 256 registers, so two waves per SIMD hide each other's VALU / LDS latency.
// The dP-wave lags one tile, so the ring keeps the previous tile's Q image resident: 5 slots, DMA
// three tiles ahead (slot of tile t + 3 = slot of tile t - 2). P crosses LDS as fp32 (the numerics
// of the 4-wave kernel), double-buffered by tile parity. One barrier per tile, plus one after the
// sweep for the dP-wave's last tile. Same masks, dropout hash, RoPE epilogue and schedule.
constexpr int K3N = 128, K3M = 32, K3NT = 512, K3NS = 5, K3PD = K3NS - 2;
constexpr int K3IMG = K3M * D * 2;                // one 32-row image: 8 KiB
constexpr int K3SLOT = 2 * K3IMG + 8 * 1024;      // Q image, dO image, 8 per-wave statistics copies
constexpr int K3XW = 64 * 16 * 4;                 // one wave's P tile: 64 lanes x 16 fp32
constexpr int K3X = 4 * K3XW;                     // the 4 pairs
constexpr int K3LDS = K3NS * K3SLOT + 2 * K3X;    // 120 + 32 = 152 KiB

template <bool DROP>
__global__ __launch_bounds__(K3NT, 1) void attn_bwd_dkdv2_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) char smem[K3LDS];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int pr = w & 3;
  const bool swave = w < 4;
  const int g = lane >> 4, l16 = lane & 15;
  const int BHk = p.B * p.Hkv;
  const int nkb = (p.Sk + K3N - 1) / K3N;
  QJobs jobs;
  if (p.sched == 1) {
    jobs = q_jobs(1, nkb, BHk);
  } else {
    jobs.bh = blockIdx.x % BHk;
    jobs.blk0 = (int)(blockIdx.x / BHk);
    jobs.blk1 = -1;
  }
  const int bhk = jobs.bh;
  const int b = bhk / p.Hkv, hkv = bhk % p.Hkv;
  const int grp = p.Hq / p.Hkv;
  // one instantiation per role (SW: S-wave), so neither role's registers are live in the other's code
  auto run_block = [&](const int kblk, auto role_c) __attribute__((always_inline)) {
  constexpr bool SW = decltype(role_c)::value;
  int Sq = p.Sq, Sk = p.Sk;
  int64_t tok0 = 0;
  if (p.cu_seqlens) {
    tok0 = p.cu_seqlens[b];
    Sq = Sk = p.cu_seqlens[b + 1] - (int)tok0;
    if (kblk * K3N >= Sk) return;  // workgroup-uniform
  }
  GRT_DEVICE_CHECK(grp * p.Hkv == p.Hq && kblk * K3N < Sk);
  const int sk = p.seqlens_k ? min(Sk, p.seqlens_k[b]) : Sk;
  const int off = Sk - Sq;
  const int k0 = kblk * K3N, kw0 = k0 + pr * 32, mykey = kw0 + l32;
  const float c = p.scale * kLog2e;
  const int Sqp = sq_pad(p.Sq);

  // K (S-wave) or V (dP-wave) fragments of this lane's key, for the whole sweep
  const bf16* KV = SW ? (const bf16*)p.k + (int64_t)b * p.k_bs + tok0 * p.k_ss + (int64_t)hkv * p.k_hs
                         : (const bf16*)p.v + (int64_t)b * p.v_bs + tok0 * p.v_ss + (int64_t)hkv * p.v_hs;
  const int64_t kv_ss = SW ? p.k_ss : p.v_ss;
  bf16x8 kv[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks)
    kv[ks] = mykey < sk ? *reinterpret_cast<const bf16x8*>(KV + (int64_t)mykey * kv_ss + ks * 16 + 8 * h) : bf16x8{};
  f32x16 acc[4];  // dV^T (S-wave) / dK^T (dP-wave)
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x16{};

  int qstart = p.causal ? max(0, k0 - off) : 0;
  qstart = (qstart / K3M) * K3M;
  const int nqt = qstart < Sq ? (Sq - qstart + K3M - 1) / K3M : 0;
  const int total = (k0 < sk) ? nqt * grp : 0;
  const int qlim = mykey < sk ? (p.causal ? mykey - off : INT_MIN) : INT_MAX;
  const int qmask = (k0 + K3N > sk) ? INT_MAX : (p.causal ? kw0 + 31 - off : INT_MIN);
  // query tiles ending at or before dead_q hold no query at or past this pair's first key: every
  // (query, key) of theirs is masked (causal), and with keys past sk the tile is masked anyway
  const int dead_q = p.skip_dead && p.causal && !DROP ? kw0 - off : INT_MIN;

  // LDS-DMA of a tile: wave w fills image rows 4w .. 4w+3 of Q and of dO (one 1-KiB piece each)
  // and its own copy of the tile's 32 lse2 and 32 delta values (3 instructions per wave and tile)
  const uint32_t smem0 = lds_u32(smem);
  const int row = 4 * w + g, ch = l16 ^ img_swz(row);
  const int64_t st_lane = ((l16 & 15) < 8 ? (int64_t)p.B * p.Hq * Sqp : 0) + 4 * (l16 & 7);  // lse2 | delta
  const uint32_t qo = (uint32_t)(row * p.q_ss + ch * 8), oo = (uint32_t)(row * P.do_ss + ch * 8);
  auto dma_tile = [&](int hq, int qt, uint32_t slot_off) __attribute__((always_inline)) {
    const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + tok0 * p.q_ss + (int64_t)hq * p.q_hs;
    const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + tok0 * P.do_ss + (int64_t)hq * P.do_hs;
    const uint32_t dst = __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(4 * w * 256));
    if (p.dma_fast && qt + K3M <= Sq) {  // tile inside the sequence: uniform base + fixed per-lane offsets
      lds_dma16(Q + (int64_t)qt * p.q_ss + qo, dst);
      lds_dma16(dO + (int64_t)qt * P.do_ss + oo, dst + K3IMG);
    } else {
      const int64_t qr = min(qt + row, Sq - 1);  // past Sq: lse2 = +inf, p = 0
      lds_dma16(Q + qr * p.q_ss + ch * 8, dst);
      lds_dma16(dO + qr * P.do_ss + ch * 8, dst + K3IMG);
    }
    const int64_t ri = ((int64_t)b * p.Hq + hq) * Sqp + qt;
    lds_dma16(P.delta + st_lane + ri, __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(2 * K3IMG + w * 1024)));
  };
  auto wait_dma = [&](int pending_tiles) __attribute__((always_inline)) {  // 3 DMA instructions per tile
    if (pending_tiles >= 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (pending_tiles == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  float* const xbase = reinterpret_cast<float*>(smem + K3NS * K3SLOT) + pr * (K3XW / 4);

  // tile cursors: consumed (cur), previous (prv: the dP-wave's lagging tile), DMA
  int cur_h = 0, cur_q = qstart, prv_h = 0, prv_q = qstart, dma_h = 0, dma_q = qstart;
  auto advance = [&](int& hh, int& qq) __attribute__((always_inline)) {
    qq += K3M;
    if (qq >= Sq) { qq = qstart; ++hh; }
  };
  f32x16 dpc = f32x16{};  // dP-wave: dP of the tile it finishes next

  // dP-wave: finish tile `tp` (slot image `pi`, P in parity buffer of tp): dS, dK^T += Q^T dS
  auto finish = [&](int tp, const char* pi) __attribute__((always_inline)) {
    const float* st = reinterpret_cast<const float*>(pi + 2 * K3IMG + w * 1024);
    const float* xi = xbase + (tp & 1) * (K3X / 4);
    f32x16 ds;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 pv = *reinterpret_cast<const f32x4*>(xi + (q * 64 + lane) * 4);
      const f32x4 de = *reinterpret_cast<const f32x4*>(st + 32 + 8 * q + 4 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * q + j;
        if (DROP) {
          const float z = drop_factor(p, (uint32_t)(b * p.Hq + hkv * grp + prv_h), prv_q + 8 * q + 4 * h + j, mykey);
          ds[r] = pv[j] * (dpc[r] * z - de[j]);
        } else {
          ds[r] = pv[j] * (dpc[r] - de[j]);
        }
      }
    }
    const bf16x8 sb0 = pack8(ds, 0), sb1 = pack8(ds, 8);
    __builtin_amdgcn_sched_barrier(0);  // scheduling regions bound the live fragments (2 waves/SIMD)
#pragma unroll
    for (int stp = 0; stp < 2; ++stp) {
      const int kk = 16 * stp + 4 * h;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int c0 = db * 32 + (g & 1) * 16;
        const bf16x8 a = cat(lds_tr_read(pi, kk, c0, l16), lds_tr_read(pi, kk + 8, c0, l16));
        acc[db] = mfma32(a, stp ? sb1 : sb0, acc[db]);
      }
    }
  };

  auto step = [&](int t, auto slot_c) __attribute__((always_inline)) {
    constexpr int SL = decltype(slot_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS reads / P stores done
    wait_dma(min(total - 1, t + K3PD - 1) - t);           // tile t landed (this wave's pieces)
    __builtin_amdgcn_s_barrier();                         // ... every wave's; P of tile t-1 published
    if (t + K3PD < total) {
      dma_tile(hkv * grp + dma_h, dma_q, (uint32_t)(((SL + K3PD) % K3NS) * K3SLOT));
      advance(dma_h, dma_q);
    }
    const char* qi = smem + SL * K3SLOT;
    // causal tiles whose queries all precede this pair's first key (the first `pr` tiles of each
    // head's sweep): p = dS = 0 there, so both roles skip their math (p.skip_dead; energy only: the
    // workgroup's barrier cadence is set by the other pairs)
    const bool dead_c = cur_q + K3M <= dead_q, dead_p = prv_q + K3M <= dead_q;
    if constexpr (SW) {
     if (!dead_c) {
      const float* st = reinterpret_cast<const float*>(qi + 2 * K3IMG + w * 1024);
      f32x16 s = f32x16{};
      if (cur_q < qmask) {  // wave-uniform: the tile touches the diagonal / key padding
#pragma unroll
        for (int r = 0; r < 16; ++r) s[r] = cur_q + acc_row(r, h) >= qlim ? 0.f : -INFINITY;
      }
      bf16x8 fq[D / 16];
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) fq[ks] = lds_row_read(qi, l32, 2 * ks + h);
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) s = mfma32(fq[ks], kv[ks], s);
      __builtin_amdgcn_sched_barrier(0);
      float* xo = xbase + (t & 1) * (K3X / 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 ls = *reinterpret_cast<const f32x4*>(st + 8 * q + 4 * h);
        f32x4 pv;
#pragma unroll
        for (int j = 0; j < 4; ++j) pv[j] = fast_exp2(fmaf(s[4 * q + j], c, -ls[j]));
        *reinterpret_cast<f32x4*>(xo + (q * 64 + lane) * 4) = pv;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          s[4 * q + j] = DROP ? pv[j] * drop_factor(p, (uint32_t)(b * p.Hq + hkv * grp + cur_h),
                                                    cur_q + 8 * q + 4 * h + j, mykey)
                              : pv[j];  // dV uses the dropped probabilities
      }
      const bf16x8 pb0 = pack8(s, 0), pb1 = pack8(s, 8);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int stp = 0; stp < 2; ++stp) {
        const int kk = 16 * stp + 4 * h;
#pragma unroll
        for (int db = 0; db < 4; ++db) {
          const int c0 = db * 32 + (g & 1) * 16;
          const bf16x8 a = cat(lds_tr_read(qi + K3IMG, kk, c0, l16), lds_tr_read(qi + K3IMG, kk + 8, c0, l16));
          acc[db] = mfma32(a, stp ? pb1 : pb0, acc[db]);
        }
      }
     }
    } else {  // the previous tile first: its dP is the only one live (register budget of 2 waves/SIMD)
      if (t > 0 && !dead_p) finish(t - 1, smem + ((SL + K3NS - 1) % K3NS) * K3SLOT);
      __builtin_amdgcn_sched_barrier(0);
      if (!dead_c) {
        bf16x8 fd[D / 16];
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) fd[ks] = lds_row_read(qi + K3IMG, l32, 2 * ks + h);
        dpc = f32x16{};
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) dpc = mfma32(fd[ks], kv[ks], dpc);
      }
    }
    prv_h = cur_h;
    prv_q = cur_q;
    advance(cur_h, cur_q);
  };

  if (total > 0) {
    const int pre = min(total, K3PD);
    for (int j = 0; j < pre; ++j) {
      dma_tile(hkv * grp + dma_h, dma_q, (uint32_t)(j * K3SLOT));
      advance(dma_h, dma_q);
    }
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    int t = 0;
    for (; t + K3NS <= total; t += K3NS) {  // one ring revolution
      step(t, I0{});
      step(t + 1, I1{});
      step(t + 2, I2{});
      step(t + 3, I3{});
      step(t + 4, I4{});
    }
    if (t < total) step(t, I0{});
    if (t + 1 < total) step(t + 1, I1{});
    if (t + 2 < total) step(t + 2, I2{});
    if (t + 3 < total) step(t + 3, I3{});
    // the dP-wave's last tile: its P is published at this barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (!SW) {
      if (prv_q + K3M > dead_q) finish(total - 1, smem + ((total - 1) % K3NS) * K3SLOT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (mykey < Sk) {
    const int64_t tokg = (p.cu_seqlens ? 0 : (int64_t)b * p.Sk) + tok0 + mykey;
    if constexpr (SW) {
      bf16* dV = (bf16*)P.dv + (int64_t)b * P.dv_bs + (int64_t)hkv * P.dv_hs + (tok0 + mykey) * P.dv_ss;
      const TCopy tv = tcopy(P, P.t_row_v, hkv, tokg);
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(acc[db][4 * gg + j]);
          *reinterpret_cast<bf16x4*>(dV + db * 32 + 8 * gg + 4 * h) = v;
          st_t(tv, db * 32 + 8 * gg + 4 * h, v);
        }
    } else {
      bf16* dK = (bf16*)P.dk + (int64_t)b * P.dk_bs + (int64_t)hkv * P.dk_hs + (tok0 + mykey) * P.dk_ss;
      const TCopy tk = tcopy(P, P.t_row_k, hkv, tokg);
      if (P.rope_cos) {
        store_unrotated(acc, p.scale, P.rope_cos + (int64_t)mykey * (D / 2), P.rope_sin + (int64_t)mykey * (D / 2), dK, h,
                        tk);
      } else {
#pragma unroll
        for (int db = 0; db < 4; ++db)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            bf16x4 a;
#pragma unroll
            for (int j = 0; j < 4; ++j) a[j] = static_cast<bf16>(acc[db][4 * gg + j] * p.scale);
            *reinterpret_cast<bf16x4*>(dK + db * 32 + 8 * gg + 4 * h) = a;
            st_t(tk, db * 32 + 8 * gg + 4 * h, a);
          }
      }
    }
  }
  };
  auto run_role = [&](auto role_c) __attribute__((always_inline)) {
    run_block(jobs.blk0, role_c);
    if (jobs.blk1 >= 0) {  // every wave is done with the ring and the P buffers before they are refilled
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      run_block(jobs.blk1, role_c);
    }
  };
  if (swave) run_role(std::true_type{});
  else run_role(std::false_type{});
}

// dQ: the forward's mapping (32 query rows per wave on the MFMA lane, 4 waves = 128 rows) over
// 32-key K / V tiles through the ring; S^T / dP^T are recomputed and dS^T feeds dQ^T += K^T dS^T.
// 24 MFMAs per tile and wave; two workgroups per CU (64 KiB LDS each). Masking: -inf in the S^T
// accumulator's initial value on the diagonal / padding tiles.
constexpr int Q2M = 128, Q2N = 32, Q2NT = 256, Q2NSLOT = 4;
constexpr int Q2IMG = Q2N * D * 2;   // one 32-key image: 8 KiB
constexpr int Q2SLOT = 2 * Q2IMG;    // K, V

template <bool DROP>
__global__ __launch_bounds__(Q2NT, 2) void attn_bwd_dq_kernel(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  __shared__ __attribute__((aligned(16))) char smem[Q2NSLOT * Q2SLOT];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int g = lane >> 4, l16 = lane & 15;
  const int nqb = (p.Sq + Q2M - 1) / Q2M;  // grid: the longest sequence
  const int BH = p.B * p.Hq;
  const QJobs jobs = q_jobs(p.sched, nqb, BH);  // see the forward
  const int bh = jobs.bh;
  const int b = bh / p.Hq, hq = bh % p.Hq;
  const int hkv = hq / (p.Hq / p.Hkv);
  GRT_DEVICE_CHECK(b < p.B && hkv < p.Hkv && jobs.blk0 >= 0 && jobs.blk0 < nqb);
  // one call per block of this workgroup; inlined twice, so the second block's registers are
  // allocated independently (a loop over the two blocks spilled the dQ kernel)
  auto run_block = [&](const int qblk) {
  int Sq = p.Sq, Sk = p.Sk;
  int64_t tok0 = 0;  // padding-free packing: this sequence's first token row
  if (p.cu_seqlens) {
    tok0 = p.cu_seqlens[b];
    Sq = Sk = p.cu_seqlens[b + 1] - (int)tok0;
    if (qblk * Q2M >= Sq) return;  // workgroup-uniform: the sequence is shorter than the longest
  }
  const int sk = p.seqlens_k ? min(Sk, p.seqlens_k[b]) : Sk;
  const int off = Sk - Sq;
  const int q0 = qblk * Q2M, qw0 = q0 + w * 32;
  const int myq = qw0 + l32;
  const bool qok = myq < Sq;
  const int Sqp = sq_pad(p.Sq);  // workspace row stride: the longest sequence

  const bf16* Q = (const bf16*)p.q + (int64_t)b * p.q_bs + tok0 * p.q_ss + (int64_t)hq * p.q_hs;
  const bf16* dO = (const bf16*)P.dout + (int64_t)b * P.do_bs + tok0 * P.do_ss + (int64_t)hq * P.do_hs;
  const bf16* K = (const bf16*)p.k + (int64_t)b * p.k_bs + tok0 * p.k_ss + (int64_t)hkv * p.k_hs;
  const bf16* Vg = (const bf16*)p.v + (int64_t)b * p.v_bs + tok0 * p.v_ss + (int64_t)hkv * p.v_hs;

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
  const int64_t ri = (int64_t)bh * Sqp + min(myq, Sqp - 1);
  const float lse2 = P.delta[(int64_t)BH * Sqp + ri];  // +inf on padding rows: p = 0
  const float dlt = P.delta[ri];
  const float c = p.scale * kLog2e;
  // per-lane mask: key kept iff key < sk and (non-causal or key <= myq + off)
  const int klim = p.causal ? min(sk - 1, myq + off) : sk - 1;
  // first key past which a tile needs the mask for some lane of this wave
  const int kmask = p.causal ? min(sk, qw0 + off + 1) : sk;
  const int klast = p.skip_dead && p.causal && !DROP ? min(sk - 1, qw0 + 31 + off) : INT_MAX;  // see the forward

  int kend = sk;
  if (p.causal) kend = min(kend, q0 + Q2M + off);
  const int nt = kend > 0 ? (kend + Q2N - 1) / Q2N : 0;

  // LDS-DMA of tile t into slot t % Q2NSLOT: wave w fills image rows 8w .. 8w+7 of K and V.
  // Per-lane source offsets are fixed (row 8w + 4k + g, swizzled chunk); only the key base moves.
  const uint32_t smem0 = lds_u32(smem);
  const int row0 = 8 * w + g, row1 = row0 + 4;
  const int ch0 = l16 ^ img_swz(row0), ch1 = l16 ^ img_swz(row1);
  auto dma_tile = [&](int t, uint32_t slot_off) {
    const int64_t k0r = min(t * Q2N + row0, Sk - 1), k1r = min(t * Q2N + row1, Sk - 1);  // past Sk: masked
    const uint32_t dst = __builtin_amdgcn_readfirstlane(smem0 + slot_off + (uint32_t)(8 * w * 256));
    lds_dma16(K + k0r * p.k_ss + ch0 * 8, dst);
    lds_dma16(Vg + k0r * p.v_ss + ch0 * 8, dst + Q2IMG);
    lds_dma16(K + k1r * p.k_ss + ch1 * 8, dst + 1024);
    lds_dma16(Vg + k1r * p.v_ss + ch1 * 8, dst + Q2IMG + 1024);
  };
  auto wait_dma = [&](int pending_tiles) {  // 4 DMA instructions per tile
    if (pending_tiles >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (pending_tiles == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // S^T and dP^T of tile t from slot SL; masked keys enter as -inf through the initial accumulator
  auto sdp = [&](int t, auto slot_c, f32x16& s, f32x16& dp) {
    constexpr int SL = decltype(slot_c)::value;
    const char* ki = smem + SL * Q2SLOT;
    const int kb = t * Q2N;
    s = f32x16{};
    if (kb + Q2N > kmask) {  // wave-uniform: the tile touches the diagonal / key padding
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] = kb + acc_row(r, h) <= klim ? 0.f : -INFINITY;
    }
    dp = f32x16{};
    bf16x8 fk[D / 16], fv[D / 16];
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      fk[ks] = lds_row_read(ki, l32, 2 * ks + h);
      fv[ks] = lds_row_read(ki + Q2IMG, l32, 2 * ks + h);
    }
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      s = mfma32(fk[ks], qf[ks], s);
      dp = mfma32(fv[ks], of[ks], dp);
    }
    // two fragment pairs in flight ahead of the MFMAs (see the dK / dV kernel)
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
  };

  f32x16 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x16{};

  using I0 = std::integral_constant<int, 0>;
  auto step = [&](int t, auto slot_c, f32x16& s_c, f32x16& dp_c, f32x16& s_n, f32x16& dp_n) {
    constexpr int SL = decltype(slot_c)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + 1 < nt) wait_dma(min(nt, t + Q2NSLOT - 1) - (t + 2));
    __builtin_amdgcn_s_barrier();
    if (t + Q2NSLOT - 1 < nt) dma_tile(t + Q2NSLOT - 1, (uint32_t)(((SL + Q2NSLOT - 1) % Q2NSLOT) * Q2SLOT));
    if (t * Q2N > klast) return;  // tile t (and every later one) masked for the whole wave: p = dS = 0

    sdp(t + 1, std::integral_constant<int, (SL + 1) % Q2NSLOT>{}, s_n, dp_n);  // past the end: dropped

#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = fast_exp2(fmaf(s_c[r], c, -lse2));
      const float z = DROP ? drop_factor(p, (uint32_t)bh, myq, t * Q2N + acc_row(r, h)) : 1.f;
      s_c[r] = pv * (dp_c[r] * z - dlt);
    }
    const char* ki = smem + SL * Q2SLOT;
#pragma unroll
    for (int stp = 0; stp < 2; ++stp) {
      const bf16x8 sb = pack8(s_c, 8 * stp);
      const int kk = 16 * stp + 4 * h;
#pragma unroll
      for (int db = 0; db < 4; ++db) {
        const int c0 = db * 32 + (g & 1) * 16;
        const bf16x8 a = cat(lds_tr_read(ki, kk, c0, l16), lds_tr_read(ki, kk + 8, c0, l16));
        dq[db] = mfma32(a, sb, dq[db]);
      }
    }
  };

  if (nt > 0) {
    const int pre = min(nt, Q2NSLOT - 1);
    for (int t = 0; t < pre; ++t) dma_tile(t, (uint32_t)(t * Q2SLOT));
    wait_dma(pre - 1);
    __builtin_amdgcn_s_barrier();
    f32x16 sA, dpA, sB, dpB;
    sdp(0, I0{}, sA, dpA);
    int t = 0;
    for (; t + Q2NSLOT <= nt; t += Q2NSLOT) {  // one ring revolution: slots 0..3, register sets A/B
      step(t, I0{}, sA, dpA, sB, dpB);
      step(t + 1, std::integral_constant<int, 1>{}, sB, dpB, sA, dpA);
      step(t + 2, std::integral_constant<int, 2>{}, sA, dpA, sB, dpB);
      step(t + 3, std::integral_constant<int, 3>{}, sB, dpB, sA, dpA);
    }
    if (t < nt) step(t, I0{}, sA, dpA, sB, dpB);
    if (t + 1 < nt) step(t + 1, std::integral_constant<int, 1>{}, sB, dpB, sA, dpA);
    if (t + 2 < nt) step(t + 2, std::integral_constant<int, 2>{}, sA, dpA, sB, dpB);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (qok) {
    bf16* dQ = (bf16*)P.dq + (int64_t)b * P.dq_bs + (int64_t)hq * P.dq_hs + (tok0 + myq) * P.dq_ss;
    const TCopy tq = tcopy(P, P.t_row_q, hq, (p.cu_seqlens ? 0 : (int64_t)b * p.Sq) + tok0 + myq);
    if (P.rope_cos) {
      store_unrotated(dq, p.scale, P.rope_cos + (int64_t)myq * (D / 2), P.rope_sin + (int64_t)myq * (D / 2), dQ, h, tq);
    } else {
#pragma unroll
      for (int db = 0; db < 4; ++db)
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          bf16x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = static_cast<bf16>(dq[db][4 * gg + j] * p.scale);
          *reinterpret_cast<bf16x4*>(dQ + db * 32 + 8 * gg + 4 * h) = v;
          st_t(tq, db * 32 + 8 * gg + 4 * h, v);
        }
    }
  }
  };
  run_block(jobs.blk0);
  if (jobs.blk1 >= 0) {  // every wave is done with the ring (LDS reads, its own DMAs) before it is refilled
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    run_block(jobs.blk1);
  }
}

}  // namespace

namespace {
// bit mask of the kernels that use the causal-pair schedule: 1 = forward, 2 = dQ, 4 = dK / dV
// (-1: not set yet -> GRT_ATTN_SCHED, default 7: all three kernels pair when the paired grid fills
// the chip; B8 S1024 H32: forward -10 %, backward -6 %: profiles/r3_attn_schedule.md)
int g_sched = -1;
// dK / dV kernel: 2 = wave-pair (default), 1 = the 4-wave kernel (GRT_ATTN_DKDV, attn_set_dkdv_form)
int g_dkdv = -1;
int dkdv_form() {
  if (g_dkdv < 0) {
    const char* e = getenv("GRT_ATTN_DKDV");
    g_dkdv = e && atoi(e) == 1 ? 1 : 2;
  }
  return g_dkdv;
}
int g_skip_dead = -1;
int skip_dead_now() {
  if (g_skip_dead < 0) {
    const char* e = getenv("GRT_ATTN_SKIP");
    g_skip_dead = e && atoi(e) == 0 ? 0 : 1;
  }
  return g_skip_dead;
}
int g_dma_fast = -1;
int dma_fast_now() {
  if (g_dma_fast < 0) {
    const char* e = getenv("GRT_ATTN_DMA_FAST");
    g_dma_fast = e && atoi(e) == 0 ? 0 : 1;
  }
  return g_dma_fast;
}
// the fast addressing keeps per-lane row offsets in 32 bits (24-bit multiplies): every row stride
// of the streamed operands must be below 2^24 elements
int dma_fast_for(const AttnParams& p, int64_t do_ss) {
  const int64_t lim = (int64_t)1 << 24;
  return dma_fast_now() && p.q_ss < lim && p.k_ss < lim && p.v_ss < lim && do_ss < lim && p.q_ss >= 0 &&
         p.k_ss >= 0 && p.v_ss >= 0 && do_ss >= 0;
}
int sched_now() {
  if (g_sched < 0) {
    const char* e = getenv("GRT_ATTN_SCHED");
    g_sched = e ? atoi(e) : 7;
  }
  return g_sched;
}
}  // namespace

// The causal pairs halve the grid: take them only when the paired grid still fills every
// workgroup slot of the chip (B8 S1024 H32: 2048 dK/dV workgroups -> 1024 pairs on 256 CUs, -6 % backward;
// B2 S2048 Hkv8: 256 dK/dV workgroups -> 128 pairs would leave half the CUs idle, +3 %).
static int cu_count() {
  static const int n = [] {
    int d = 0, c = 256;
    hipGetDevice(&d);
    hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d);
    return c > 0 ? c : 256;
  }();
  return n;
}
static int pair_if_fills(int want, int nblk, int groups, int per_cu) {
  return want && (int64_t)groups * ((nblk + 1) / 2) >= (int64_t)cu_count() * per_cu ? 1 : 0;
}

void attn_set_schedule(int s) { g_sched = s; }
void attn_set_dkdv_form(int f) { g_dkdv = f == 1 ? 1 : 2; }
int attn_get_dkdv_form() { return dkdv_form(); }
void attn_set_dma_fast(int on) { g_dma_fast = on ? 1 : 0; }
void attn_set_skip_dead(int on) { g_skip_dead = on ? 1 : 0; }
int attn_get_schedule() { return sched_now(); }

// Padding-free packing (cu_seqlens): the grid is sized for the longest sequence, so a shorter one's
// heavy block of a causal pair exits at once and the pair's work is no longer equal — pairs off
// (LoRA step at 6656 packed tokens 33.1 -> 31.4 ms per 1K tokens; profiles/r3_varlen_attention.md).
static int sched_for(const AttnParams& p, int bit) { return p.cu_seqlens ? 0 : (sched_now() >> bit) & 1; }

void attn_fwd(const AttnParams& p0, hipStream_t s) {
  AttnParams p = p0;
  p.dma_fast = dma_fast_for(p, 0);
  p.skip_dead = skip_dead_now();
  const int nqb = (p.Sq + F3M - 1) / F3M;
  p.sched = pair_if_fills(sched_for(p, 0), nqb, p.B * p.Hq, 2);
  const dim3 grid(q_grid(p.sched, nqb, p.B * p.Hq));
  // (a 5-slot ring, 3 tiles in flight, spills 41 VGPRs with its 10-step unroll: not instantiated)
  if (p.drop_thresh) hipLaunchKernelGGL((attn_fwd_kernel<true, F3NSLOT>), grid, dim3(F3NT), 0, s, p);
  else hipLaunchKernelGGL((attn_fwd_kernel<false, F3NSLOT>), grid, dim3(F3NT), 0, s, p);
}

int64_t attn_bwd_workspace_floats(int B, int Hq, int Sq, int Dh) {
  (void)Dh;
  return 2 * (int64_t)B * Hq * sq_pad(Sq);  // delta and lse2, rows padded to 32
}

void attn_bwd(const AttnBwdParams& p0, hipStream_t s) {
  AttnBwdParams p = p0;
  p.f.dma_fast = dma_fast_for(p.f, p.do_ss);
  p.f.skip_dead = skip_dead_now();
  const int64_t rows = (int64_t)p.f.B * p.f.Hq * sq_pad(p.f.Sq);
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((unsigned)((rows + 15) / 16)), dim3(256), 0, s, p);
  const int nkb = (p.f.Sk + K2N - 1) / K2N;
  const int nqb = (p.f.Sq + Q2M - 1) / Q2M;
  AttnBwdParams pk = p, pq = p;
  pk.f.sched = pair_if_fills(sched_for(p.f, 2), nkb, p.f.B * p.f.Hkv, 1);
  pq.f.sched = pair_if_fills(sched_for(p.f, 1), nqb, p.f.B * p.f.Hq, 2);
  const dim3 g1(q_grid(pk.f.sched, nkb, p.f.B * p.f.Hkv)), g2(q_grid(pq.f.sched, nqb, p.f.B * p.f.Hq));
  static_assert(K3N == K2N, "both dK / dV forms take 128-key blocks (same grid)");
  // the wave-pair form: B8 S1024 H32 backward 425 -> 412 us, GQA 32:8 even; with probability
  // dropout it is slower (142 -> 150 us at B2 S1024 p 0.1: the dP-wave recomputes the keep hash the
  // S-wave already drew), so dropout keeps the 4-wave kernel (tools/attn_dkdv_ab.py, profiles/r4_attention.md)
  const bool pair = dkdv_form() == 2 && !p.f.drop_thresh;
  if (p.f.drop_thresh) {
    if (pair) hipLaunchKernelGGL(attn_bwd_dkdv2_kernel<true>, g1, dim3(K3NT), 0, s, pk);
    else hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, g1, dim3(K2NT), 0, s, pk);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, g2, dim3(Q2NT), 0, s, pq);
  } else {
    if (pair) hipLaunchKernelGGL(attn_bwd_dkdv2_kernel<false>, g1, dim3(K3NT), 0, s, pk);
    else hipLaunchKernelGGL(attn_bwd_dkdv_kernel<false>, g1, dim3(K2NT), 0, s, pk);
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, g2, dim3(Q2NT), 0, s, pq);
  }
}

}  // namespace grt
