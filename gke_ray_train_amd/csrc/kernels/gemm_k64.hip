// Projection GEMM for gfx950, 256 x 256 x 64 tiles:  C[M][N] (+)= sum_k A[M][K] * B[N][K]
// (bf16 in, fp32 accumulate, bf16 out). Reference: the cuBLAS GEMMs under nn.Linear
// (ray-jobs/pytorch_llm_ray.py:82-87) and the HF Llama projections under SFTTrainer.train()
// (ray-jobs/fine_tune_llama_ray.py:333); SURVEY §2.3 N02, §2.6 K-B04.
//
// Status (profiles/r5_gemm_k64.md): 91-99 % of the tuned hipBLASLt kernel on the 15 Llama-2-7B
// step shapes, every element checked against fp32 (tests/test_gemm_gpu.py). The training step keeps
// the library for plain GEMMs; this kernel is reachable through gemm_nt variants 9-16.
//
// Structure (one workgroup per CU: 4 waves, one per SIMD, 128 x 128 outputs per wave):
//   * accumulators: 8 x 8 blocks of v_mfma_f32_16x16x32_bf16 in LITERAL AGPRs a0-a255 (one
//     clobber statement at entry allocates them; the MFMA statements name them directly, so the
//     compiler never copies or spills accumulators); 128 MFMAs per 64-deep K-tile;
//   * fragments: the K-tile's two 32-deep halves (kk0, kk1) of A and B in VGPRs (SCHED 2: kk1
//     double-buffered, read one period ahead);
//   * LDS: two K-tile buffers (A + B each), 130 KiB. An operand tile is 32 chunks of 1040 B; chunk
//     c holds rows {128 (c >> 4) + 16 b + (c & 15)}, b = 0..7, as 128-B lines (the row's 64 k) at
//     b * 128 -- one LDS-DMA instruction of one wave fills one chunk with eight whole cache lines,
//     and the 16-B pad puts the 16 rows of a fragment read in different bank quads;
//   * global -> LDS: buffer_load ... lds (LDS-DMA, no VGPR round trip), 16 per wave per K-tile. The
//     tile origin lives in the buffer descriptor (SGPRs), per-instruction row offsets in SGPR
//     soffsets, the lane part in one VGPR per operand; each DMA rides in one asm statement with an
//     MFMA (M0 written first: the MFMA covers the M0 -> DMA wait state);
//   * SCHED 1 (variants 9, 10): per period three barriers -- A kk1 reads -> lgkmcnt(0), barrier 1;
//     B kk1 reads + A DMAs of K-tile t+2 -> lgkmcnt(0), barrier 2; A/B DMAs -> vmcnt(12), barrier 3;
//     kk0 reads of K-tile t+1 + the last B DMAs (schedule tables kReadA1 ... below);
//     SCHED 2 (variants 11, 12): two barriers, reads of the next K-tile bunched after barrier B
//     (slower: the LDS port, not the barriers, is the constraint -- profiles/r5_gemm_k64.md);
//   * PERSIST (variants 9, 11): grid = #CUs, the K pipeline runs across a workgroup's output tiles
//     (the last two periods of a tile DMA the next tile's first two K-tiles), so between tiles only
//     the epilogue remains; an out-of-range DMA uses a zero-record descriptor (no memory traffic);
//   * epilogue: AGPR reads after the MFMA -> VALU wait states, bf16 pack, v_permlane16_swap so each
//     lane stores 8 consecutive columns (16-B stores); beta = 1 adds the old C;
//   * blockIdx -> tile: bijective XCD remap, then 8-row groups (T1).
// Requirements (host-checked): M % 256 == 0, N % 256 == 0, K % 128 == 0, K >= 128, row strides
// multiples of 8 elements, 16-byte aligned bases, every operand byte offset below 2^31.
#include "grt_common.h"
#include "grt_kernels.h"

#include <algorithm>
#include <type_traits>
#include <utility>

namespace grt {
namespace {

constexpr int KT = 64;           // reduction depth of one tile
constexpr int CH = 1040;         // one LDS chunk: 8 rows x 128 B + 16 B pad
constexpr int TEN = 32 * CH;     // one operand tile (256 rows)
constexpr int BUFB = 2 * TEN;    // A + B of one K-tile
constexpr int LDSB = 2 * BUFB;   // two K-tile buffers = 133,120 B
constexpr int kGroupRows = 8;

// The 8 x 8 accumulator blocks live in LITERAL AGPRs: block (i, j) = a[4 (8 i + j) .. +3]. A
// statement at kernel entry declares all 256 AGPRs clobbered, which makes the kernel descriptor
// allocate them; the compiler's own values need ~140-190 arch VGPRs, so it never allocates into the
// AGPR file. Every MFMA statement repeats the clobber list: without it the compiler treats the AGPRs
// as dead between statements and adds accvgpr copies of its own; the price is an s_nop 0 between
// consecutive MFMA statements (free here: removing every wait and barrier gains only 1-3 %,
// profiles/r5_gemm_k64.md). ZERO: the first K-tile of an output tile starts from the constant 0.
#define GRT_ACC_CLOBBERS "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"
template <int N, bool ZERO>
__device__ __forceinline__ void mfma_acc(const bf16x8& a, const bf16x8& b) {
  if constexpr (ZERO)
    asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, 0" :: "v"(a), "v"(b), "i"(N), "i"(N + 3) : GRT_ACC_CLOBBERS);
  else
    asm volatile("v_mfma_f32_16x16x32_bf16 a[%c2:%c3], %0, %1, a[%c2:%c3]" :: "v"(a), "v"(b), "i"(N), "i"(N + 3) : GRT_ACC_CLOBBERS);
}
// MFMA + the LDS-DMA that rides behind it in ONE statement (the compiler pads an s_nop between an
// MFMA and any following inline asm, as it cannot see what the asm reads; the DMA reads no MFMA
// result). M0 = wave base + OFF is written first; the MFMA between the write and the DMA is the
// M0 -> LDS-DMA wait state. SCC is declared clobbered (s_add), so the compiler never schedules the
// statement between its own s_cmp / s_cselect or s_add / s_addc pairs.
template <int N, bool ZERO, int OFF>
__device__ __forceinline__ void mfma_acc_dma(const bf16x8& a, const bf16x8& b, uint32_t voff,
                                             __amdgpu_buffer_rsrc_t rsrc, uint32_t soff, uint32_t mbase) {
  if constexpr (ZERO)
    asm volatile("s_add_u32 m0, %5, %6\n\tv_mfma_f32_16x16x32_bf16 a[%c7:%c8], %0, %1, 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds"
                 :: "v"(a), "v"(b), "v"(voff), "s"(rsrc), "s"(soff), "s"(mbase), "i"(OFF), "i"(N), "i"(N + 3)
                 : "memory", "m0", "scc");
  else
    asm volatile("s_add_u32 m0, %5, %6\n\tv_mfma_f32_16x16x32_bf16 a[%c7:%c8], %0, %1, a[%c7:%c8]\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds"
                 :: "v"(a), "v"(b), "v"(voff), "s"(rsrc), "s"(soff), "s"(mbase), "i"(OFF), "i"(N), "i"(N + 3)
                 : "memory", "m0", "scc");
}
// accumulator block at a[N .. N+3] -> VGPRs (after the MFMA -> VALU-read pad)
template <int N>
__device__ __forceinline__ f32x4 acc_read() {
  float x0, x1, x2, x3;
  asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\tv_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
               : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3) : "i"(N), "i"(N + 1), "i"(N + 2), "i"(N + 3));
  return f32x4{x0, x1, x2, x3};
}

// prologue DMA (no MFMA to hide the M0 -> LDS-DMA wait state behind: explicit s_nop)
template <int OFF>
__device__ __forceinline__ void dma(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc, uint32_t soff, uint32_t mbase) {
  asm volatile("s_add_u32 m0, %2, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :: "v"(voff), "s"(rsrc), "s"(mbase), "s"(soff), "i"(OFF) : "memory", "m0", "scc");
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)(p);
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- per-period schedule: what rides behind MFMA number I (0..127) --------------------------
// seg 1 (0-21): A kk1 reads -> lgkmcnt(0), barrier 1
// seg 2 (22-47): B kk1 reads + A DMAs 0-3 -> lgkmcnt(0), barrier 2
// seg 3 (48-79): A DMAs 4-7, B DMAs 0-3 -> vmcnt(12), barrier 3
// seg 4 (80-127): kk0 reads of the next tile (B0[0], A0[0], B0[1..7], A0[1..7]) at 80..110, B DMAs 4-7
// (the last read lands >= 17 MFMAs before the next period's first MFMA)
constexpr int kReadA1[8] = {0, 2, 5, 8, 11, 13, 16, 18};
constexpr int kReadB1[8] = {22, 24, 27, 30, 33, 36, 39, 42};
constexpr int kDmaA[8] = {23, 29, 35, 41, 49, 53, 57, 61};
constexpr int kDmaB[8] = {65, 69, 73, 77, 85, 95, 105, 115};
constexpr int kRead0First = 80;  // 16 reads at 80, 82, ..., 110
constexpr int kBar1 = 21, kBar2 = 47, kBar3 = 79;
constexpr int kDmaBeforeBar3 = 12;

// SCHED 2: every fragment of a K-tile is read in the period BEFORE it is multiplied (kk1 fragments
// double-buffered in registers: a1[U] / b1[U]), so a period needs only two barriers and its DMAs can
// start right after the first:
// seg 1 (0-15): lgkmcnt(0), barrier A (every wave's reads of this buffer done)
// seg 2 (16-79): 16 DMAs of K-tile t+2 into this buffer at 16, 20, ..., 76 -> vmcnt(16), barrier B
// seg 3 (80-127): 32 reads of the next buffer (kk0 into a0 / b0, then kk1 into a1[U^1] / b1[U^1])
// The last DMA of a period has 131 MFMAs (~1.3 us) before the barrier that waits for it (SCHED 1: 92).
constexpr int kBarA2 = 15, kDma2First = 16, kBarB2 = 79, kRead2First = 80;

constexpr int find8(const int (&t)[8], int i) {
  for (int q = 0; q < 8; ++q)
    if (t[q] == i) return q;
  return -1;
}

// PERSIST: grid = min(#tiles, #CUs); workgroup b takes the tiles of rounds k = 0, 1, ... (tile
// round_base + remap(b) of round k, round_base = k * G). The K pipeline runs straight across output
// tiles: the last two periods of a tile DMA the first two K-tiles of the workgroup's next tile, and
// the last period's kk0 reads are already that tile's first fragments, so between tiles only the
// epilogue remains (no prologue, no pipeline drain). Without PERSIST the grid is one workgroup per
// tile (A/B reference).
// DIAG (timing experiments only, results wrong): 1 = no vmcnt wait at barrier 3, 2 = no lgkmcnt(0)
// at barriers 1 / 2, 4 = no s_barrier
template <int EPI, bool PERSIST, int SCHED, int DIAG = 0>
__global__ __launch_bounds__(256, 1) void gemm_k64_kernel(const GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[LDSB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 1, wc = w & 1;
  const int nM = p.M / 256, nN = p.N / 256, ntiles = nM * nN;
  const int G = gridDim.x, b = blockIdx.x;
  const int T = p.K / KT;  // even, >= 2 (host check)

  // this workgroup's tile of round k, or -1 when the round has no tile for it
  auto tile_of = [&](int k, int& tm, int& tn) __attribute__((always_inline)) -> bool {
    const int base = k * G;
    if (base >= ntiles) return false;
    const int nr = min(G, ntiles - base);
    const int r = xcd_remap(b, G);
    if (r >= nr) return false;
    const int lin = base + r;
    const int per_group = kGroupRows * nN;
    const int grp = lin / per_group, first = grp * kGroupRows;
    const int gsize = min(nM - first, kGroupRows);
    // wave-uniform by construction; readfirstlane makes it provable (the descriptors built from
    // it must sit in SGPRs)
    tm = __builtin_amdgcn_readfirstlane(first + (lin % per_group) % gsize);
    tn = __builtin_amdgcn_readfirstlane((lin % per_group) / gsize);
    return true;
  };

  // ---- DMA addressing: wave w, instruction q fills chunk 4q + w: lane l carries row
  // 128 (q >> 2) + 16 (l >> 3) + 4 (q & 3) + w, k-chunk l & 7
  const uint32_t avoff = (uint32_t)(((16 * (lane >> 3) + w) * p.lda + 8 * (lane & 7)) * 2);
  const uint32_t bvoff = (uint32_t)(((16 * (lane >> 3) + w) * p.ldb + 8 * (lane & 7)) * 2);
  const uint32_t lda2 = (uint32_t)p.lda * 2, ldb2 = (uint32_t)p.ldb * 2;
  uint32_t soa[8], sob[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    soa[q] = (uint32_t)(128 * (q >> 2) + 4 * (q & 3)) * lda2;
    sob[q] = (uint32_t)(128 * (q >> 2) + 4 * (q & 3)) * ldb2;
  }
  const uint32_t mbase = __builtin_amdgcn_readfirstlane(lds_u32(smem) + w * CH);
  auto rsrc = [](const char* base, int num) __attribute__((always_inline)) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, num, 0x00020000);
  };
  // 32-bit offsets (host check: every operand below 2 GiB) keep the address math on the SALU, so
  // the descriptors built from it are SGPR values (the asm "s" operands)
  auto a_tile = [&](int tm) __attribute__((always_inline)) { return static_cast<const char*>(p.a) + (uint32_t)(tm * 256) * lda2; };
  auto b_tile = [&](int tn) __attribute__((always_inline)) { return static_cast<const char*>(p.b) + (uint32_t)(tn * 256) * ldb2; };

  // ---- fragment addressing: lane l reads row (l & 15) of a 16-row block, k-chunk (l >> 4) (+4 kk)
  const int lf = (lane & 15) * CH + (lane >> 4) * 16;
  const char* fa[2] = {smem + 0 * BUFB + 16 * wr * CH + lf, smem + 1 * BUFB + 16 * wr * CH + lf};
  const char* fb[2] = {smem + 0 * BUFB + TEN + 16 * wc * CH + lf, smem + 1 * BUFB + TEN + 16 * wc * CH + lf};
  auto frag = [](const char* base, int blk, int kk) __attribute__((always_inline)) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(base + blk * 128 + kk * 64);
  };

  int tm, tn;
  if (!tile_of(0, tm, tn)) return;  // whole workgroup: uniform
  asm volatile("" ::: GRT_ACC_CLOBBERS);  // allocates the AGPR file (see mfma_acc)
  bf16x8 a0[8], b0[8], a1[SCHED == 2 ? 2 : 1][8], b1[SCHED == 2 ? 2 : 1][8];

  // ---- prologue (once per workgroup): K-tiles 0 and 1 of the first tile in flight, kk0 of K-tile 0
  {
    const auto ra = rsrc(a_tile(tm), 0x7fffffff), rb = rsrc(b_tile(tn), 0x7fffffff);
    const auto ra1 = rsrc(a_tile(tm) + KT * 2, 0x7fffffff), rb1 = rsrc(b_tile(tn) + KT * 2, 0x7fffffff);
    static_for<8>([&](auto Q) __attribute__((always_inline)) { dma<0 * BUFB + 0 + decltype(Q)::value * 4 * CH>(avoff, ra, soa[decltype(Q)::value], mbase); });
    static_for<8>([&](auto Q) __attribute__((always_inline)) { dma<0 * BUFB + TEN + decltype(Q)::value * 4 * CH>(bvoff, rb, sob[decltype(Q)::value], mbase); });
    static_for<8>([&](auto Q) __attribute__((always_inline)) { dma<1 * BUFB + 0 + decltype(Q)::value * 4 * CH>(avoff, ra1, soa[decltype(Q)::value], mbase); });
    static_for<8>([&](auto Q) __attribute__((always_inline)) { dma<1 * BUFB + TEN + decltype(Q)::value * 4 * CH>(bvoff, rb1, sob[decltype(Q)::value], mbase); });
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 8; ++j) { b0[j] = frag(fb[0], j, 0); a0[j] = frag(fa[0], j, 0); }
    if constexpr (SCHED == 2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { b1[0][j] = frag(fb[0], j, 1); a1[0][j] = frag(fa[0], j, 1); }
    }
  }

  // ---- one K-tile period on buffer U (compile-time); FIRST: K-tile 0 of an output tile (its kk0
  // MFMAs start the accumulators at 0). ra / rb: the DMA source of this period (K-tile t+2 of this
  // tile, or K-tile t+2-T of the next one, or nothing)
  auto period = [&](auto U_, auto FIRST_, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb) __attribute__((always_inline)) {
    constexpr int U = decltype(U_)::value;
    constexpr bool ZERO = decltype(FIRST_)::value && (true);
    if constexpr (SCHED == 2) {
      static_for<128>([&](auto I_) __attribute__((always_inline)) {
        constexpr int I = decltype(I_)::value;
        constexpr int kk = I / 64, i = (I % 64) / 8, j = I % 8;
        constexpr int dq = (I >= kDma2First && I < kDma2First + 64 && (I - kDma2First) % 4 == 0) ? (I - kDma2First) / 4 : -1;
        constexpr int dqa = dq >= 0 && dq < 8 ? dq : 0, dqb = dq >= 8 ? dq - 8 : 0;
        constexpr uint32_t m0off = dq < 8 ? U * BUFB + 0 + dqa * 4 * CH : U * BUFB + TEN + dqb * 4 * CH;
        bf16x8& af = kk == 0 ? a0[i] : a1[U][i];
        bf16x8& bfr = kk == 0 ? b0[j] : b1[U][j];
        if constexpr (dq >= 0) {
          const uint32_t vo = dq < 8 ? avoff : bvoff;
          const uint32_t so = dq < 8 ? soa[dqa] : sob[dqb];
          const auto rs = dq < 8 ? ra : rb;
          mfma_acc_dma<4 * (8 * i + j), ZERO && kk == 0, m0off>(bfr, af, vo, rs, so, mbase);
        } else {
          mfma_acc<4 * (8 * i + j), ZERO && kk == 0>(bfr, af);
        }
        if constexpr (I >= kRead2First) {
          // 32 reads at 80, 81, 83, 84, ... 126: x = 0..15 kk0, 16..31 kk1; within each,
          // B[0], A[0], B[1..7], A[1..7]
          constexpr int x0 = (2 * (I - kRead2First) + 2) / 3;  // first x with 80 + 3x/2 >= I
          constexpr bool hit = x0 < 32 && kRead2First + (3 * x0) / 2 == I;
          if constexpr (hit) {
            constexpr int x = x0 & 15, rk = x0 >> 4;
            constexpr bool isb = x == 0 || (x >= 2 && x <= 8);
            constexpr int blk = x == 0 ? 0 : x == 1 ? 0 : x <= 8 ? x - 1 : x - 8;
            if constexpr (rk == 0) {
              if constexpr (isb) b0[blk] = frag(fb[U ^ 1], blk, 0);
              else a0[blk] = frag(fa[U ^ 1], blk, 0);
            } else {
              if constexpr (isb) b1[U ^ 1][blk] = frag(fb[U ^ 1], blk, 1);
              else a1[U ^ 1][blk] = frag(fa[U ^ 1], blk, 1);
            }
          }
        }
        if constexpr (I == kBarA2) {
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if constexpr (I == kBarB2) {
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      return;
    }
    static_for<128>([&](auto I_) __attribute__((always_inline)) {
      constexpr int I = decltype(I_)::value;
      constexpr int kk = I / 64, i = (I % 64) / 8, j = I % 8;
      constexpr int ra1q = find8(kReadA1, I), rb1q = find8(kReadB1, I);
      constexpr int dAq = find8(kDmaA, I), dBq = find8(kDmaB, I);
      constexpr uint32_t m0off = dAq >= 0 ? U * BUFB + 0 + dAq * 4 * CH : U * BUFB + TEN + (dBq >= 0 ? dBq : 0) * 4 * CH;
      bf16x8& af = kk == 0 ? a0[i] : a1[0][i];
      bf16x8& bfr = kk == 0 ? b0[j] : b1[0][j];
      if constexpr (dAq >= 0 || dBq >= 0) {
        constexpr int q = dAq >= 0 ? dAq : dBq;
        const uint32_t vo = dAq >= 0 ? avoff : bvoff;
        const uint32_t so = dAq >= 0 ? soa[q] : sob[q];
        const auto rs = dAq >= 0 ? ra : rb;
        mfma_acc_dma<4 * (8 * i + j), ZERO && kk == 0, m0off>(bfr, af, vo, rs, so, mbase);
      } else {
        mfma_acc<4 * (8 * i + j), ZERO && kk == 0>(bfr, af);
      }
      if constexpr (ra1q >= 0) a1[0][ra1q] = frag(fa[U], ra1q, 1);
      if constexpr (rb1q >= 0) b1[0][rb1q] = frag(fb[U], rb1q, 1);
      if constexpr (I >= kRead0First && I < kRead0First + 32 && (I - kRead0First) % 2 == 0) {
        constexpr int x = (I - kRead0First) / 2;  // 0: B0[0], 1: A0[0], 2..8: B0[1..7], 9..15: A0[1..7]
        if constexpr (x == 0) b0[0] = frag(fb[U ^ 1], 0, 0);
        else if constexpr (x == 1) a0[0] = frag(fa[U ^ 1], 0, 0);
        else if constexpr (x <= 8) b0[x - 1] = frag(fb[U ^ 1], x - 1, 0);
        else a0[x - 8] = frag(fa[U ^ 1], x - 8, 0);
      }
      if constexpr (I == kBar1 || I == kBar2) {
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(DIAG & 2)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (!(DIAG & 4)) asm volatile("s_barrier" ::: "memory");
      }
      if constexpr (I == kBar3) {
        static_assert(kDmaBeforeBar3 == 12, "vmcnt below");
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (!(DIAG & 1)) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        if constexpr (!(DIAG & 4)) asm volatile("s_barrier" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using Z = std::integral_constant<int, 0>;
  using O = std::integral_constant<int, 1>;
  using Fy = std::integral_constant<bool, true>;
  using Fn = std::integral_constant<bool, false>;

  const int r = lane & 15, g = lane >> 4;
  const int cofs = ((g & 1) ? 16 : 0) + ((g & 2) ? 8 : 0);
  for (int k = 0;; ++k) {
    // next tile of this workgroup (DMA target of the last two periods)
    int ntm = 0, ntn = 0;
    const bool has_next = __builtin_amdgcn_readfirstlane((PERSIST && tile_of(k + 1, ntm, ntn)) ? 1 : 0) != 0;
    const char* abase = a_tile(tm);
    const char* bbase = b_tile(tn);
    const char* anext = a_tile(has_next ? ntm : tm);
    const char* bnext = b_tile(has_next ? ntn : tn);
    auto src = [&](int t, const char* cur, const char* nxt) __attribute__((always_inline)) {
      // K-tile t + 2 of this tile, else K-tile t + 2 - T of the next tile, else no records
      // (selects, not branches: one descriptor either way)
      const bool here = t + 2 < T;
      const char* base = here ? cur + (uint32_t)(t + 2) * (KT * 2) : nxt + (uint32_t)(t + 2 - T) * (KT * 2);
      return rsrc(base, (here || has_next) ? 0x7fffffff : 0);
    };
    period(Z{}, Fy{}, src(0, abase, anext), src(0, bbase, bnext));
    period(O{}, Fn{}, src(1, abase, anext), src(1, bbase, bnext));
    for (int t = 2; t < T; t += 2) {
      period(Z{}, Fn{}, src(t, abase, anext), src(t, bbase, bnext));
      period(O{}, Fn{}, src(t + 1, abase, anext), src(t + 1, bbase, bnext));
    }
    // ---- epilogue. The last MFMAs' results are read by VALU: 3 x 8 wait states (8-pass XDL
    // write -> VALU read), then an empty asm redefines every accumulator so no read is hoisted
    // above the pad. Lane (r, g) holds C[m][n .. n+3] of block (i, j), m = m0 + 128 wr + 16 i + r,
    // n = n0 + 128 wc + 16 j + 4 g; for a block pair (j, j+1) one v_permlane16_swap per dword (odd
    // 16-lane rows of the first operand <-> even rows of the second) leaves each lane 8 consecutive
    // columns: g = 0 block j cols 0-7, g = 1 block j+1 cols 0-7, g = 2 block j cols 8-15, g = 3
    // block j+1 cols 8-15 -> one 16-B store per lane and pair (T21). The stores join the vmcnt
    // stream; the next tile's barrier-3 vmcnt(12) simply also covers them.
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bf16* cbase = static_cast<bf16*>(p.c) + (int64_t)(tm * 256 + 128 * wr + r) * p.ldc + tn * 256 + 128 * wc + cofs;
    auto pack2 = [](float a_, float b_) __attribute__((always_inline)) -> uint32_t {
      const bf16x2 v = {static_cast<bf16>(a_), static_cast<bf16>(b_)};
      return __builtin_bit_cast(uint32_t, v);
    };
    auto swap = [](f32x4& x, f32x4& y, auto E_) __attribute__((always_inline)) {
      constexpr int e = decltype(E_)::value;
      const auto v = __builtin_amdgcn_permlane16_swap(__float_as_uint(x[e]), __float_as_uint(y[e]), false, false);
      x[e] = __uint_as_float(v[0]);
      y[e] = __uint_as_float(v[1]);
    };
    auto store_pair = [&](auto I_, auto JP_, bool accumulate) __attribute__((always_inline)) {
      constexpr int i = decltype(I_)::value, jp = decltype(JP_)::value;
      bf16* crow = cbase + (int64_t)16 * i * p.ldc + 32 * jp;
      f32x4 x = acc_read<4 * (8 * i + 2 * jp)>(), y = acc_read<4 * (8 * i + 2 * jp + 1)>();
      if (accumulate) {
        static_for<4>([&](auto E_) __attribute__((always_inline)) { swap(x, y, E_); });
        const bf16x8 old = *reinterpret_cast<const bf16x8*>(crow);
        uint4 o;
        o.x = pack2(x[0] + (float)old[0], x[1] + (float)old[1]);
        o.y = pack2(x[2] + (float)old[2], x[3] + (float)old[3]);
        o.z = pack2(y[0] + (float)old[4], y[1] + (float)old[5]);
        o.w = pack2(y[2] + (float)old[6], y[3] + (float)old[7]);
        *reinterpret_cast<uint4*>(crow) = o;
      } else {
        const uint32_t x0 = pack2(x[0], x[1]), x1 = pack2(x[2], x[3]);
        const uint32_t y0 = pack2(y[0], y[1]), y1 = pack2(y[2], y[3]);
        const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        *reinterpret_cast<uint4*>(crow) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    };
    auto store_rows = [&](bool accumulate) __attribute__((always_inline)) {
      static_for<8>([&](auto I_) __attribute__((always_inline)) { static_for<4>([&](auto JP_) __attribute__((always_inline)) { store_pair(I_, JP_, accumulate); }); });
    };
    if (p.beta) store_rows(true);
    else store_rows(false);
    if (!has_next) break;
    tm = ntm;
    tn = ntn;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outstanding at exit
}

}  // namespace

bool gemm_nt_k64_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb) {
  if (M <= 0 || N <= 0 || K < 128 || M % 256 || N % 256 || K % 128) return false;
  if ((M / 256) * (N / 256) > INT32_MAX) return false;
  // descriptor offsets: lane part + soffset of the 255th row + 64 k, 32-bit signed range
  if ((255 * lda + 64) * 2 >= (int64_t(1) << 31) || (255 * ldb + 64) * 2 >= (int64_t(1) << 31)) return false;
  return true;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

void gemm_nt_k64(const GemmParams& p, hipStream_t stream) {
  const int ntiles = (p.M / 256) * (p.N / 256);
  const int G = std::min(ntiles, num_cus());
  switch (p.variant) {
    case 10: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, false, 1>), dim3(ntiles), dim3(256), 0, stream, p); break;
    case 11: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 2>), dim3(G), dim3(256), 0, stream, p); break;
    case 12: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, false, 2>), dim3(ntiles), dim3(256), 0, stream, p); break;
    case 13: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 1, 1>), dim3(G), dim3(256), 0, stream, p); break;
    case 14: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 1, 2>), dim3(G), dim3(256), 0, stream, p); break;
    case 15: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 1, 4>), dim3(G), dim3(256), 0, stream, p); break;
    case 16: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 1, 7>), dim3(G), dim3(256), 0, stream, p); break;
    default: hipLaunchKernelGGL((gemm_k64_kernel<GEMM_EPI_STORE, true, 1>), dim3(G), dim3(256), 0, stream, p); break;
  }
}

}  // namespace grt
