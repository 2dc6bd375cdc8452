// Host-side launcher API of the HIP kernels. Kernel translation units (*.hip) implement these;
// the torch bindings (bindings/ops.cpp) call them with raw pointers on the current HIP stream.
// Keeping torch headers out of the device TUs keeps them fast to compile and free of any
// framework coupling.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace grt {

enum class DType : int { F32 = 0, BF16 = 1 };

// ---------------- normalisation (norm.hip) ----------------
// y = norm(x [+ residual]) * w [+ b]; writes rstd (and mean for LayerNorm) per row in fp32.
// If residual != nullptr, h = x + residual is written to h_out (the new residual stream).
void rmsnorm_fwd(DType dt, const void* x, const void* residual, const void* w, void* y, void* h_out,
                 float* rstd, int64_t rows, int d, float eps, hipStream_t s,
                 int64_t ldy = 0);
// dx = d/dh (norm) + dres ; dw accumulated through fp32 partials (workspace of
// rmsnorm_bwd_workspace(rows, d) floats).
// dw_t != null: the weight gradient is written in the parameter dtype straight into dw_t (a
// gradient-buffer slot; accumulate != 0 adds to it) instead of dw_f32.
void rmsnorm_bwd(DType dt, const void* dy, const void* h, const void* w, const float* rstd,
                 const void* dres, void* dx, float* dw_f32, float* ws, int64_t rows, int d,
                 hipStream_t s, void* dw_t = nullptr, int accumulate = 0);
int64_t norm_bwd_workspace_floats(int64_t rows, int d);
void layernorm_fwd(DType dt, const void* x, const void* residual, const void* w, const void* b,
                   void* y, void* h_out, float* mean, float* rstd, int64_t rows, int d, float eps,
                   hipStream_t s);
void layernorm_bwd(DType dt, const void* dy, const void* h, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* dw_f32, float* db_f32,
                   float* ws, int64_t rows, int d, hipStream_t s);

// ---------------- elementwise (elementwise.hip) ----------------
void swiglu_fwd(DType dt, const void* gu, void* out, int64_t rows, int f, hipStream_t s, int64_t ldo = 0);
// bf16 SwiGLU that also writes the transposed result for the TN weight gradient (out^T [f, rows],
// dgu^T [2f, rows]); false = shape not handled (rows % 64, f % 128)
bool swiglu_fwd_t(const void* gu, void* out, void* outT, int64_t rows, int f, hipStream_t s, int64_t ldo = 0);
bool swiglu_bwd_t(const void* gu, const void* dout, void* dgu, void* dguT, int64_t rows, int f, hipStream_t s);
void swiglu_bwd(DType dt, const void* gu, const void* dout, void* dgu, int64_t rows, int f,
                hipStream_t s);
// GELU (erf form) with optional fused dropout mask (uint8, 1 = keep, scale applied).
void gelu_fwd(DType dt, const void* x, void* y, int64_t n, hipStream_t s);
void gelu_bwd(DType dt, const void* x, const void* dy, void* dx, int64_t n, hipStream_t s);
// RoPE (rotate-half convention). qkv: [T, (hq + 2*hkv) * D] fused projection output with row
// stride `ld`; writes q_out [T, hq, D], k_out [T, hkv, D] contiguous. cos/sin: [S, D/2] fp32,
// position of token t is pos[t] (int32) or t % S when pos == nullptr.
void ew_set_fast(int on);  // 1 = single-pass 32-bit-index RoPE (D = 128) / SwiGLU kernels (default), 0 = grid-stride kernels
void rope_fwd(DType dt, const void* qkv, int64_t ld, void* q_out, void* k_out, const float* cos,
              const float* sin, const int32_t* pos, int64_t T, int S, int hq, int hkv, int D,
              hipStream_t s);
// Inverse rotation of dq/dk, written into the q and k column ranges of dqkv (row stride ld).
// decode: rotate q (-> q_out [T, hq, D]) and k of each token, write k and v at cache slot pos[t] of
// row t / tpr of kc / vc (bf16)
void rope_append(const void* qkv, int64_t ld, void* q_out, void* kc, void* vc, int64_t c_bs, int64_t c_ss,
                 int64_t c_hs, int64_t v_bs, int64_t v_ss, int64_t v_hs, const float* cos, const float* sin,
                 const int32_t* pos, int64_t T_, int tpr, int S, int L, int hq, int hkv, int D, hipStream_t s);
void rope_bwd(DType dt, const void* dq, const void* dk, void* dqkv, int64_t ld, const float* cos,
              const float* sin, const int32_t* pos, int64_t T, int S, int hq, int hkv, int D,
              hipStream_t s);
// out = emb * scale + pe[t % S]   (BasicLLM input path; pe may be null)
void scale_add_pe(DType dt, const void* emb, const float* pe, void* out, int64_t T, int S, int d,
                  float scale, hipStream_t s);
// Dropout with a counter-based hash RNG; mask bytes written for backward.
void dropout_fwd(DType dt, const void* x, void* y, uint8_t* mask, int64_t n, float p, uint64_t seed,
                 uint64_t offset, hipStream_t s);
// mask may be null in both: fwd then stores no mask, bwd regenerates keep(i) from (seed, offset);
// bwd with accumulate adds into dx.
void dropout_bwd(DType dt, const void* dy, const uint8_t* mask, void* dx, int64_t n, float p,
                 hipStream_t s, uint64_t seed = 0, uint64_t offset = 0, bool accumulate = false);

// ---------------- cross entropy (cross_entropy.hip) ----------------
void cross_entropy_fwd(DType dt, const void* logits, int64_t ld, const int64_t* labels, float* loss,
                       float* lse, int64_t rows, int V, int64_t ignore_index, hipStream_t s);
// dlogits = (softmax - onehot) * gscale[row]  (gscale = dloss per row); may alias logits.
void cross_entropy_bwd(DType dt, const void* logits, int64_t ld, const int64_t* labels,
                       const float* lse, const float* gscale, void* dlogits, int64_t ldd,
                       int64_t rows, int V, int64_t ignore_index, hipStream_t s);

// ---------------- optimizer (optim.hip) ----------------
// Sum of squares of flat tensors; writes partials into ws[nblocks] then total into out[0].
int optim_sumsq_blocks();
void sumsq_accumulate(DType dt, const void* x, int64_t n, float* ws, int slot, hipStream_t s);
// Finalise: norm = sqrt(sum(ws[0:nparts])) * prescale; out[0] = norm,
// out[1] = min(1, max_norm / (norm + 1e-6)) * prescale  (clip disabled when max_norm <= 0).
void clip_coef_finalize(const float* ws, int nparts, float max_norm, float prescale, float* out,
                        hipStream_t s);
// Fused AdamW on a flat range. hyper (device): [lr, beta1, beta2, eps, weight_decay, bc1, bc2,
// grad_scale]; grad_scale_ptr (device, may be null) multiplies grads (clip coefficient).
// max_blocks > 0 caps the grid (grid-stride loop): a bandwidth-throttled update that can run
// beside compute-bound kernels on another stream without starving them (parallel/overlap.py).
void adamw_step(DType pdt, DType gdt, void* p, const void* g, float* m, float* v, float* master,
                int64_t n, const float* hyper, const float* grad_scale_ptr, hipStream_t s, int max_blocks = 0,
                int64_t index_offset = 0);  // element index of p[0] in its flat buffer (stochastic rounding)
// AdamW of one bf16 weight [rows][cols] (bf16 grad, fp32 moments, no master; rows % 64, cols % 128 == 0)
// that also writes its transpose pt [cols][rows]; ioff = flat index of p[0] (stochastic rounding).
void adamw_t_step(void* p, const void* g, float* m, float* v, void* pt, int64_t rows, int64_t cols,
                  const float* hyper, const float* grad_scale_ptr, hipStream_t s, int64_t ioff);
// Scale in place: x *= a (device scalar pointer or host value when a_ptr == null).
void scale_inplace(DType dt, void* x, int64_t n, float a, const float* a_ptr, hipStream_t s);

// ---------------- LoRA adapter (lora.hip) ----------------
// h[M][R] = (x ⊙ keep/(1-p)) · A^T, A [R][K]; keep = the element-dropout hash of x's element index
// (offset + row*K + col, as dropout_fwd_seeded); xd (optional) receives x ⊙ keep/(1-p).
struct LoraDownParams {
  const void* x; const void* a; void* h; void* xd;
  int64_t M; int K; int R; int ldx;
  float p; uint64_t seed; uint64_t offset;
  int ksplit = 1; float* hpart = nullptr;  // split-K: fp32 partials [ksplit][M][R], summed into h
  int64_t ldh = 0;      // h row stride (0 = R); > R: h is the tail of a [x | h] row buffer
  float hscale = 1.f;   // h = hscale * drop(x) A^T (the LoRA scaling folded in)
};
int lora_down_splits(int64_t M, int K, int R, int cus);
bool lora_down_supported(int64_t M, int K, int R, int ldx, uint64_t offset);
void lora_down(const LoraDownParams& p, hipStream_t s);
// dX[M][K] (+)= keep/(1-p) ⊙ (g[M][R] · A[R][K]), given A^T = at [K][R] (same keep mask as lora_down)
struct LoraDxParams {
  const void* g; const void* at; void* dx;
  int64_t M; int K; int R;
  float p; uint64_t seed; uint64_t offset; int accumulate;
  int64_t ldg = 0;            // g row stride (0 = R)
  const void* dx_in = nullptr; int64_t ld_in = 0;  // accumulate from dx_in (row stride ld_in), not dx
  int64_t ld_out = 0;         // dx row stride (0 = K)
  float gscale = 1.f;         // dx (+)= gscale * keep / (1-p) * (g A)
};
// Copy LoRA B_i [n_i, r] into the adapter tail of the K-concatenated weight W' [out, ldw] (columns
// [col0 + j r, col0 + (j+1) r) of rows [off_i, off_i + n_i)) and of its transpose W'^T (rows
// col0 + j r .. , row stride ldt), for up to 4 targets in one launch.
struct LoraRefreshParams {
  const void* b[4]; int off[4]; int n[4]; int ntarget; int r;
  void* w; int64_t ldw; void* wt; int64_t ldt; int col0;
  int trow0;  // W'^T row of the first adapter block (col0 for the full transpose; 0 for a B^T buffer)
};
void lora_refresh(const LoraRefreshParams& p, hipStream_t s);
bool lora_dx_supported(int64_t M, int K, int R, uint64_t offset);
void lora_dx(const LoraDxParams& p, hipStream_t s);

// ---------------- LoRA gradient GEMMs (lora_grad.hip) ----------------
// C[M][64] (+)= alpha * A[M][K] B[K][64], from B^T [64][K] (row stride ldbt). Up to 4 products
// of the same M (the targets of one adapted module: grid y = product) in one launch; product t
// uses a[t], bt[t], c[t] with reduction length K[t].
constexpr int kLoraGMax = 4;
struct LoraGParams {
  const void* a[kLoraGMax]; int64_t lda[kLoraGMax]; const void* bt[kLoraGMax]; int64_t ldbt[kLoraGMax];
  void* c[kLoraGMax]; int64_t ldc[kLoraGMax]; int K[kLoraGMax];
  int nprod = 1;
  int64_t M; float alpha; int accumulate;
  int ks = 1; float* ws = nullptr;  // k splits (lora_g_splits) through the fp32 workspace [nprod][ks][M][64]
};
bool lora_g_supported(int64_t M, int K, int r);
int lora_g_splits(int64_t M, int K, int cus, int nprod = 1);
void lora_g(const LoraGParams& p, hipStream_t s);
// out (+)= alpha * A^T H, A [M][N], H [M][R]: out [N][R] (row stride ldo), or [R][N] when transpose;
// ks token splits through the fp32 workspace ws [ks][N * R] (lora_tred_splits)
// Up to 4 products of the same M and R in one launch (the dB_i of one adapted module's targets):
// product t owns the 128-column blocks [bo[t], bo[t] + N[t] / 128) of the launch; its partials
// sit at column offset 128 bo[t] of each split's [sum N][R] plane.
constexpr int kLoraTredMax = 4;
struct LoraTredParams {
  const void* a[kLoraTredMax]; int64_t lda[kLoraTredMax]; const void* h[kLoraTredMax]; int64_t ldh[kLoraTredMax];
  void* out[kLoraTredMax]; int64_t ldo[kLoraTredMax]; int N[kLoraTredMax]; int bo[kLoraTredMax];
  int accumulate[kLoraTredMax];
  int nprod = 1; int nbt;  // products, total column blocks
  float* ws; int64_t M; int R; int ks; int64_t mchunk; int transpose; float alpha;
};
bool lora_tred_supported(int64_t M, int N, int R);
int lora_tred_splits(int64_t M, int N, int R, int cus);
void lora_tred(const LoraTredParams& p, hipStream_t s);

// ---------------- attention (attention.hip) ----------------
struct AttnParams {
  const void* q; const void* k; const void* v; void* o; float* lse;
  int64_t q_bs, q_ss, q_hs;   // strides (elements) for batch, seq, head; last dim contiguous
  int64_t k_bs, k_ss, k_hs;
  int64_t v_bs, v_ss, v_hs;
  int64_t o_bs, o_ss, o_hs;
  int B, Sq, Sk, Hq, Hkv, D;
  float scale;
  int causal;
  const int32_t* seqlens_k;   // optional per-batch valid key length (right padding), may be null
  // optional padding-free packing (bf16 kernels): sequence b is token rows [cu[b], cu[b+1]) of the
  // packed q / k / v / o (batch strides 0); B = number of sequences, Sq = Sk = the longest
  // sequence; causal self-attention inside each sequence; positions restart at 0 per sequence
  const int32_t* cu_seqlens;
  // attention-probability dropout (0 = off): element (b*Hq + hq, q, k) is kept iff
  // attn_dropout_hash(seed, bh, q, k) >= drop_thresh (= p * 2^32); kept values scaled by drop_scale
  uint32_t drop_seed;
  uint32_t drop_thresh;
  float drop_scale;
  // workgroup schedule of one bf16 kernel, set by the launchers from the attn_set_schedule() mask
  // (1 = forward, 2 = dQ, 4 = dK / dV): 0 = one block per workgroup, heaviest first; 1 = causal pairs
  int sched;
  // set by the launchers (attn_set_dma_fast, GRT_ATTN_DMA_FAST, default 1): tiles that lie inside the
  // sequence take their LDS-DMA source addresses as a uniform tile base + per-lane offsets fixed for
  // the sweep (one 64-bit add per DMA) instead of the clamped per-lane row arithmetic
  int dma_fast;
  // optional (bf16 forward, D = 128): the output also written transposed, o_t[(hq D + d) * ot_ld + token]
  // ([Hq D, tokens]) for the o projection's TN weight gradient
  void* o_t; int64_t ot_ld;
  // set by the launchers (attn_set_skip_dead, GRT_ATTN_SKIP, default 1): in the causal band a wave
  // whose rows mask every key of a tile skips that tile's math (forward, dQ and wave-pair dK / dV kernels; it still
  // takes part in the tile's barrier and LDS-DMA)
  int skip_dead;
};
void attn_set_schedule(int s);
int attn_get_schedule();
void attn_set_dkdv_form(int f);  // 1 = 4-wave dK / dV kernel, 2 = wave-pair kernel (default)
int attn_get_dkdv_form();
void attn_set_dma_fast(int on);  // 1 = hoisted DMA addressing (default), 0 = per-tile clamped addressing
void attn_set_skip_dead(int on);  // 1 = skip fully masked causal tiles per wave (default), 0 = compute them
void attn_fwd(const AttnParams& p, hipStream_t s);
struct AttnBwdParams {
  AttnParams f;
  const void* dout; int64_t do_bs, do_ss, do_hs;
  void* dq; int64_t dq_bs, dq_ss, dq_hs;
  void* dk; int64_t dk_bs, dk_ss, dk_hs;
  void* dv; int64_t dv_bs, dv_ss, dv_hs;
  float* delta;    // fp32 workspace of attn_bwd_workspace_floats(): delta and lse2 rows
  // optional (bf16 kernels, D = 128): q / k were RoPE-rotated at position = sequence index; the
  // epilogues write dQ / dK already un-rotated (cos / sin fp32 [>= max(Sq, Sk), D / 2])
  const float* rope_cos; const float* rope_sin;
  // optional (bf16 kernels, self-attention over a fused QKV gradient): the epilogues also write the
  // transposed gradient dqkv^T [(Hq + 2 Hkv) D, tokens] (row stride t_ld = tokens) for the TN weight
  // gradient of the QKV projection; rows t_row_q / t_row_k / t_row_v start the Q / K / V sections
  void* dqkv_t; int64_t t_ld; int t_row_q, t_row_k, t_row_v;
};
void attn_bwd(const AttnBwdParams& p, hipStream_t s);
int64_t attn_bwd_workspace_floats(int B, int Hq, int Sq, int D);
// decode (Sq = 1) split-K attention (decode_attention.hip): bf16, head_dim 128, Hq / Hkv in {1,2,4,8}
struct AttnDecodeParams {
  const void* q; const void* k; const void* v; void* o;
  int64_t q_bs, q_hs, k_bs, k_ss, k_hs, v_bs, v_ss, v_hs, o_bs, o_hs;
  int B, Hq, Hkv, Sk, NS;
  const int32_t* seqlens_k;   // valid keys per batch row (may be null: all Sk)
  float scale_log2;           // softmax scale * log2(e)
  float* part_o; float* part_m; float* part_l;  // workspace [B, Hq, NS, (D | 1 | 1)]
};
int attn_decode_splits(int B, int Hkv, int Sk);
void attn_decode(const AttnDecodeParams& p, hipStream_t s);
// exact-fp32 variants (attention_f32.hip): same params with fp32 tensors, head_dim 64 or 128
bool attn_f32_supported(int head_dim);
void attn_fwd_f32(const AttnParams& p, hipStream_t s);
void attn_bwd_f32(const AttnBwdParams& p, hipStream_t s);

// ---------------- 4-bit NormalFloat (nf4.hip) ----------------
void nf4_quantize(DType dt, const void* w, uint8_t* q, float* absmax, int64_t n, int blocksize,
                  hipStream_t s);
void nf4_dequantize(DType dt, const uint8_t* q, const float* absmax, void* w, int64_t n,
                    int blocksize, hipStream_t s);
// W^T [cols][rows] (bf16) from the NF4 codes of W [rows][cols]; cols % 64 == 0, blocksize 64
// bf16 W [rows][cols] into a row-strided destination (row stride ldo elements); false = shape not
// handled (blocksize != 64, cols % 16 != 0)
bool nf4_dequantize_2d(const uint8_t* q, const float* absmax, void* w, int rows, int cols, int64_t ldo,
                       int blocksize, hipStream_t s);
void nf4_dequantize_t(const uint8_t* q, const float* absmax, void* wt, int rows, int cols, int blocksize,
                      hipStream_t s);

// ---------------- token embedding (embedding.hip) ----------------
// out[i] = w[ids[i]]; rows of d elements (d % 8 == 0 for bf16, % 4 for fp32)
void embedding_fwd(DType dt, const int64_t* ids, const void* w, void* out, int64_t n, int d, int64_t V,
                   hipStream_t s);
// dW[v] (+)= sum_{k in [row_start[v], row_end[v])} dy[order[k]]; empty rows are zeroed (overwrite)
// or untouched (accumulate).
void embedding_bwd(DType dt, const void* dy, const int64_t* order, const int32_t* row_start, const int32_t* row_end,
                   void* dw, int64_t V, int d, bool accumulate, hipStream_t s);

// ---------------- weight-gradient GEMM (gemm.hip) ----------------
// C[P][Q] (+)= sum_r X[r][p] * Y[r][q]; X [R][P], Y [R][Q], C [P][Q] row-major bf16.
struct GemmTTParams {
  const void* x;  // bf16
  const void* y;  // bf16
  void* c;        // bf16
  int P, Q, R;
  int64_t ldx, ldy, ldc;
  int beta;  // 1: C += result (gradient accumulation), 0: C = result
};
bool gemm_tt_supported(int P, int Q, int R);
void gemm_tt(const GemmTTParams& p, hipStream_t stream, int mode = 0);  // mode != 0: diagnostics

// ---------------- projection GEMM (gemm_mfma.hip) ----------------
// C[M][N] (+)= sum_k A[M][K] * B[N][K]; A, B, C row-major bf16 with row strides lda/ldb/ldc.
enum GemmEpilogue : int {
  GEMM_EPI_STORE = 0,   // C = AB^T (beta = 1: C += AB^T)
};
struct GemmParams {
  const void* a;
  const void* b;
  void* c;
  int M, N, K;
  int64_t lda, ldb, ldc;
  int beta;
  int epi;
  int variant;  // pipeline variant (A/B experiments); 0 = default
};
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K);
void gemm_nt(const GemmParams& p, hipStream_t stream);
// 256x256x64-tile kernel (gemm_k64.hip): M, N % 256, K % 128, K >= 128, byte offsets below 2^31
bool gemm_nt_k64_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb);
void gemm_nt_k64(const GemmParams& p, hipStream_t stream);
// weight-gradient form on token-major operands: C[M][N] (+)= sum_k A[k][m] * B[k][n] (a = A [K][M],
// b = B [K][N]); M % 256 == 0, N % 256 == 0, K % 64 == 0
void gemm_tt2(const GemmParams& p, hipStream_t stream);
// input-gradient form without a transposed copy: C[M][N] (+)= sum_k A[M][k] * B[k][N] (a = A [M][K]
// row-major, b = B [K][N] row-major, i.e. dX = dY W on the weight as stored)
void gemm_nn(const GemmParams& p, hipStream_t stream);

// ---------------- transpose (transpose.hip) ----------------
// dst [cols][rows] = src [rows][cols]^T, bf16, rows and cols multiples of 64, row-major contiguous
void transpose_bf16(const void* src, void* dst, int rows, int cols, hipStream_t s);

// ---------------- decode GEMV (gemv.hip) ----------------
// y[m][n] = sum_k x[m][k] * w[n][k] for m < M <= 4; bf16, K % 8 == 0, rows 16-byte aligned
// swiglu: x is the fused [gate | up] output [M, 2K] and the GEMV input is silu(gate) * up
void gemv_bf16(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, int M, int N, int K, hipStream_t s,
               bool swiglu = false);
// 3 <= M <= 16 and K % 256 == 0 (no swiglu): gemv_bf16 runs the MFMA skinny kernel (M up to 16)
bool gemv_mfma_ok(int M, int K);
// The decode step's residual adds / RMSNorms folded into the GEMVs (gemv.hip header):
//   sumsq_in != null: the GEMV input is bf16(x * rsqrt(sum_j sumsq_in[m][j] * 2^-20 / K + eps) * g)
//   (x = the residual stream h, sumsq_in [M][64] its fixed-point partial sums of squares);
//   res != null: y = bf16(x W^T) + res (the next h); its sums of squares are added into sumsq_out
//   [M][64] (zero at launch) and sumsq_zero [M][64] is zeroed for the next producer.
// gemv_workgroups(N): grid size of a GEMV with N output rows.
struct GemvFused {
  const void* x;
  int64_t ldx;
  const void* w;
  void* y;
  int64_t ldy;
  int M, N, K;
  bool swiglu;
  const void* g;
  float eps;
  const unsigned long long* sumsq_in;
  const void* res;
  int64_t ldr;
  unsigned long long* sumsq_out;
  unsigned long long* sumsq_zero;
  // q_out != null (qkv projection, head_dim 128, N = (hq + 2 hkv) * 128): RoPE at position pos[m]
  // in the epilogue; q -> q_out [M, hq, 128], k / v -> cache slot pos[m] of kc / vc [B, L, hkv, 128]
  void* q_out;
  void* kc;
  void* vc;
  int64_t c_bs, c_ss, c_hs, v_bs, v_ss, v_hs;
  const float* cosb;
  const float* sinb;
  const int* pos;
  int rope_S, cache_L, hq, hkv;
};
void gemv_fused_bf16(const GemvFused& f, hipStream_t s);
int gemv_k_split(int N);
int gemv_workgroups(int N);

// ---------------- xGMI peer-to-peer collectives (ipc_comm.hip) ----------------
constexpr int kIpcMaxRanks = 8;
constexpr int kIpcMaxBlocks = 64;
constexpr int kIpcHandleBytes = 64;
// Per-rank view of the communicator: every rank's staging / result / signal buffers (peer
// entries are IPC-opened mappings), this rank's error word, bytes per parity buffer.
struct IpcPeers {
  void* staging[kIpcMaxRanks];
  void* result[kIpcMaxRanks];
  uint32_t* signal[kIpcMaxRanks];
  uint32_t* err;
  int64_t cap;
  int rank, world;
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
};
// signal buffer: [2 phases][kIpcMaxBlocks][kIpcMaxRanks] uint32 flags, then one abort word that any
// peer sets (system scope) when a wait of its own timed out, padded to 256 bytes.
constexpr int kIpcAbortWord = 2 * kIpcMaxBlocks * kIpcMaxRanks;
constexpr int64_t kIpcSignalBytes = 2LL * kIpcMaxBlocks * kIpcMaxRanks * 4 + 256;
// error word bits: bit r (< kIpcMaxRanks) = a wait for rank r timed out here; kIpcErrAborted = a peer
// announced a timeout; kIpcErrSkipped = a later call found the word set and did not run. Any set bit
// makes every later call of the communicator write NaN to its output without waiting (fail-stop).
constexpr uint32_t kIpcErrAborted = 1u << 30;
constexpr uint32_t kIpcErrSkipped = 1u << 31;
int ipc_blocks_for(int64_t nbytes, bool two_shot);
// out = scale * sum over ranks of in (nbytes a multiple of 16, <= cap); in == out allowed.
void ipc_allreduce(const IpcPeers& peers, uint32_t epoch, DType dt, const void* in, void* out, int64_t nbytes,
                   bool two_shot, float scale, hipStream_t s);
void ipc_barrier(const IpcPeers& peers, uint32_t epoch, hipStream_t s);
void* ipc_malloc(int64_t nbytes, bool fine_grained);
void ipc_free(void* p);
void ipc_get_handle(void* p, char out[kIpcHandleBytes]);
void* ipc_open_handle(const char in[kIpcHandleBytes]);
void ipc_close_handle(void* p);

// test support (debug_lds.hip): every CU's LDS filled with `pattern` on stream s
void lds_fill(uint32_t pattern, hipStream_t s);

}  // namespace grt
