// RMSNorm / LayerNorm forward + backward for gfx950, with a fused residual add.
//
// Role in the reference: every Llama decoder layer runs two RMSNorms and BasicLLM's post-LN
// nn.TransformerEncoderLayer runs two LayerNorms after a residual add
// (reference ray-jobs/pytorch_llm_ray.py:82-86).
//
// Design (memory-bound, MI355X_MICROARCH.md §HBM):
//   * one 64-lane wave per row, 16-byte vector loads (8 x bf16 / 4 x f32 per lane),
//     the row stays in VGPRs between the reduction and the normalisation (one HBM read);
//   * the residual add is fused: h = x + residual is produced and stored in the same pass,
//     so the decoder layer never runs a separate elementwise add;
//   * backward keeps the weight-gradient partial sums in registers across the rows a
//     workgroup visits and writes one fp32 slab per workgroup; a second tiny kernel sums the
//     slabs column-wise (no float atomics, bitwise reproducible).
#include <stdlib.h>

#include "grt_common.h"
#include "grt_kernels.h"

namespace grt {
namespace {

constexpr int kNT = 256;          // 4 waves per workgroup
constexpr int kRowsPerBlock = kNT / kWave;
constexpr int kBwdMaxBlocks = 512;  // measured best for d=4096 rows=8192 (256: 89 us, 512: 74 us, 1024: 81 us)

// Forward: every load of the row (x, residual, weight) is issued before the first use, so a wave
// has the whole row in flight at once. (A per-chunk `if (ch < nchunk)` around load -> add -> store
// made hipcc close every chunk with vmcnt(0): one 16 B load pair in flight per wave, 2.6 TB/s.)
// FULL: d / V is exactly MAXC x 64 chunks (every Llama / BasicLLM width) -> no guards at all;
// otherwise loads are clamped to the last chunk and the stores are guarded.
template <typename T, int MAXC, bool RMS, bool RES, bool FULL>
__global__ __launch_bounds__(kNT) void norm_fwd_kernel(const T* __restrict__ x,
                                                       const T* __restrict__ res,
                                                       const T* __restrict__ w,
                                                       const T* __restrict__ b, T* __restrict__ y,
                                                       T* __restrict__ h_out, float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int64_t rows,
                                                       int d, float eps, int64_t ldy) {
  constexpr int V = Vec16<T>::N;
  typedef typename Vec16<T>::type VT;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nchunk = d / V;
  const T* xr = x + row * d;
  const T* rr = RES ? res + row * d : nullptr;
  VT xv[MAXC], rv[MAXC], wvv[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = FULL ? lane + c * kWave : min(lane + c * kWave, nchunk - 1);
    xv[c] = *reinterpret_cast<const VT*>(xr + ch * V);
    if (RES) rv[c] = *reinterpret_cast<const VT*>(rr + ch * V);
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = FULL ? lane + c * kWave : min(lane + c * kWave, nchunk - 1);
    wvv[c] = *reinterpret_cast<const VT*>(w + ch * V);
  }
  float hv[MAXC][V];
  float s1 = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const bool ok = FULL || lane + c * kWave < nchunk;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      float t = to_f(xv[c][i]);
      if (RES) t = to_f(from_f<T>(t + to_f(rv[c][i])));  // round like torch
      hv[c][i] = ok ? t : 0.f;
      s1 += RMS ? hv[c][i] * hv[c][i] : hv[c][i];
    }
    if (RES && ok) store16(h_out + row * d + (lane + c * kWave) * V, hv[c]);
  }
  s1 = wave_sum(s1);
  float mu = 0.f, rstd;
  if (RMS) {
    rstd = rsqrtf(s1 / d + eps);
  } else {
    mu = s1 / d;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const bool ok = FULL || lane + c * kWave < nchunk;
#pragma unroll
      for (int i = 0; i < V; ++i) { const float t = hv[c][i] - mu; s2 += ok ? t * t : 0.f; }
    }
    s2 = wave_sum(s2);
    rstd = rsqrtf(s2 / d + eps);
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + c * kWave;
    if (FULL || ch < nchunk) {
      float o[V];
      if (!RMS && b != nullptr) {
        float bv[V];
        load16(b + ch * V, bv);
#pragma unroll
        for (int i = 0; i < V; ++i) o[i] = (hv[c][i] - mu) * rstd * to_f(wvv[c][i]) + bv[i];
      } else {
#pragma unroll
        for (int i = 0; i < V; ++i) o[i] = (hv[c][i] - mu) * rstd * to_f(wvv[c][i]);
      }
      store16(y + row * ldy + ch * V, o);  // ldy > d: the row of a wider [x | LoRA h] buffer
    }
  }
  if (lane == 0) {
    rstd_out[row] = rstd;
    if (!RMS) mean_out[row] = mu;
  }
}

// Backward: one 256-thread workgroup per row (grid-strided), each thread owns MAXC 16-byte
// column chunks, so the dw/db partial sums stay in a handful of VGPRs per thread for every
// row the workgroup visits and are written once as this workgroup's fp32 slab. The next row's
// h / dy / residual-gradient chunks are loaded (clamped, unconditional) before this row's
// reduction barriers, so a row's loads are always in flight behind the previous row's math.
template <typename T, int MAXC, bool RMS, bool RES>
__global__ __launch_bounds__(kNT) void norm_bwd_kernel(const T* __restrict__ dy,
                                                       const T* __restrict__ h,
                                                       const T* __restrict__ w,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const T* __restrict__ dres, T* __restrict__ dx,
                                                       float* __restrict__ ws, int64_t rows, int d) {
  constexpr int V = Vec16<T>::N;
  typedef typename Vec16<T>::type VT;
  __shared__ float red[2 * kRowsPerBlock];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nchunk = d / V;
  float dwp[MAXC][V], dbp[MAXC][V], wv[MAXC][V];
  int chs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    chs[c] = min(tid + c * kNT, nchunk - 1);
#pragma unroll
    for (int i = 0; i < V; ++i) { dwp[c][i] = 0.f; dbp[c][i] = 0.f; }
    load16(w + chs[c] * V, wv[c]);
  }
  VT hn[MAXC], dn[MAXC], rn[MAXC];
  auto load_row = [&](int64_t rr) {
    rr = rr < rows ? rr : rows - 1;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      hn[c] = *reinterpret_cast<const VT*>(h + rr * d + chs[c] * V);
      dn[c] = *reinterpret_cast<const VT*>(dy + rr * d + chs[c] * V);
      if (RES) rn[c] = *reinterpret_cast<const VT*>(dres + rr * d + chs[c] * V);
    }
  };
  load_row(blockIdx.x);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    VT hc[MAXC], dc[MAXC], rc[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) { hc[c] = hn[c]; dc[c] = dn[c]; if (RES) rc[c] = rn[c]; }
    load_row(row + gridDim.x);
    const float r = rstd[row];
    const float mu = RMS ? 0.f : mean[row];
    float xh[MAXC][V], g[MAXC][V];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const bool ok = tid + c * kNT < nchunk;
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const float dv = ok ? to_f(dc[c][i]) : 0.f;
        xh[c][i] = (to_f(hc[c][i]) - mu) * r;
        g[c][i] = dv * wv[c][i];
        sg += g[c][i];
        sgx += g[c][i] * xh[c][i];
        dwp[c][i] += dv * xh[c][i];
        if (!RMS) dbp[c][i] += dv;
      }
    }
    // two-value block reduction, one barrier pair per row
    sgx = wave_sum(sgx);
    if (!RMS) sg = wave_sum(sg);
    if (lane == 0) { red[wid] = sgx; red[kRowsPerBlock + wid] = sg; }
    __syncthreads();
    float tsgx = 0.f, tsg = 0.f;
#pragma unroll
    for (int i = 0; i < kRowsPerBlock; ++i) { tsgx += red[i]; tsg += red[kRowsPerBlock + i]; }
    __syncthreads();
    tsgx /= d;
    tsg = RMS ? 0.f : tsg / d;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = tid + c * kNT;
      if (ch < nchunk) {
        float o[V];
#pragma unroll
        for (int i = 0; i < V; ++i) o[i] = (RES ? to_f(rc[c][i]) : 0.f) + r * (g[c][i] - tsg - xh[c][i] * tsgx);
        store16(dx + row * d + ch * V, o);
      }
    }
  }
  if (ws == nullptr) return;  // frozen weight (LoRA / QLoRA): no dw / db slab, no column sums
  float* wsb = ws + (int64_t)blockIdx.x * 2 * d;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = tid + c * kNT;
    if (ch < nchunk) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        wsb[ch * V + i] = dwp[c][i];
        wsb[d + ch * V + i] = dbp[c][i];
      }
    }
  }
}

// dw[j] = sum_b ws[b][0][j], db[j] = sum_b ws[b][1][j] over ncols (= d for RMSNorm, 2d for
// LayerNorm). One workgroup = 64 columns x 4 row phases; each thread keeps 4 independent
// accumulators so the slab loads (256 contiguous bytes per wave) stay in flight.
// GO: output type of dw / db (float, or bf16 written straight into a gradient buffer; ACC adds
// to what the buffer holds).
// One workgroup = kColsumCols columns x (256 / kColsumCols) slab-row groups: 16 columns per
// workgroup gives 256 workgroups at d = 4096 (64 columns left 3/4 of the CUs idle: 22 us per call
// in the headline step for a 16 MB slab)
constexpr int kColsumCols = 16;
constexpr int kColsumGroups = kNT / kColsumCols;
template <typename GO, bool ACC>
__global__ __launch_bounds__(kNT) void colsum_kernel(const float* __restrict__ ws, int nb, int d, int ncols,
                                                     GO* __restrict__ dw, GO* __restrict__ db) {
  __shared__ float red[kColsumGroups][kColsumCols];
  const int c = threadIdx.x % kColsumCols, rg = threadIdx.x / kColsumCols;
  const int j = blockIdx.x * kColsumCols + c;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (j < ncols) {
    const int64_t ld = 2 * (int64_t)d;
    constexpr int G = kColsumGroups;
    int b = rg;
    for (; b + 3 * G < nb; b += 4 * G) {
      a0 += ws[(int64_t)b * ld + j];
      a1 += ws[(int64_t)(b + G) * ld + j];
      a2 += ws[(int64_t)(b + 2 * G) * ld + j];
      a3 += ws[(int64_t)(b + 3 * G) * ld + j];
    }
    for (; b < nb; b += G) a0 += ws[(int64_t)b * ld + j];
  }
  red[rg][c] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (rg == 0 && j < ncols) {
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < kColsumGroups; ++g) s += red[g][c];
    GO* out = j < d ? dw : db;
    const int jj = j < d ? j : j - d;
    if (out) out[jj] = from_f<GO>(ACC ? to_f(out[jj]) + s : s);
  }
}

template <typename T, bool RMS>
void launch_fwd(const void* x, const void* res, const void* w, const void* b, void* y, void* h_out,
                float* mean, float* rstd, int64_t rows, int d, float eps, hipStream_t s, int64_t ldy = 0) {
  if (ldy <= 0) ldy = d;
  constexpr int V = Vec16<T>::N;
  const int per_lane = (d / V + kWave - 1) / kWave;
  const dim3 grid((unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock));
#define GRT_NF4(MC, RES, FULL)                                                                  \
  hipLaunchKernelGGL((norm_fwd_kernel<T, MC, RMS, RES, FULL>), grid, dim3(kNT), 0, s, (const T*)x, \
                     (const T*)res, (const T*)w, (const T*)b, (T*)y, (T*)h_out, mean, rstd, rows,     \
                     d, eps, ldy)
#define GRT_NF(MC)                                                     \
  do {                                                                 \
    const bool full = (d / V) == (MC) * kWave;                         \
    if (res != nullptr) { if (full) GRT_NF4(MC, true, true); else GRT_NF4(MC, true, false); }   \
    else { if (full) GRT_NF4(MC, false, true); else GRT_NF4(MC, false, false); }              \
  } while (0)
  if (per_lane <= 1) GRT_NF(1);
  else if (per_lane <= 2) GRT_NF(2);
  else if (per_lane <= 4) GRT_NF(4);
  else if (per_lane <= 8) GRT_NF(8);
  else if (per_lane <= 16) GRT_NF(16);
  else GRT_NF(32);
#undef GRT_NF
#undef GRT_NF4
}

int bwd_max_blocks() {
  // workgroups of the backward (each keeps a dw partial slab); GRT_NORM_BWD_BLOCKS overrides for A/B
  static const int v = [] {
    const char* e = getenv("GRT_NORM_BWD_BLOCKS");
    const int n = e ? atoi(e) : kBwdMaxBlocks;
    return n > 0 ? n : kBwdMaxBlocks;
  }();
  return v;
}

int bwd_blocks(int64_t rows) {
  const int mb = bwd_max_blocks();
  return (int)(rows < mb ? (rows > 0 ? rows : 1) : mb);
}

template <typename T, bool RMS>
void launch_bwd(const void* dy, const void* h, const void* w, const float* mean, const float* rstd,
                const void* dres, void* dx, float* dw, float* db, float* ws, int64_t rows, int d,
                hipStream_t s, void* dw_t = nullptr, int accumulate = 0) {
  constexpr int V = Vec16<T>::N;
  const int per_thr = (d / V + kNT - 1) / kNT;
  const int nb = bwd_blocks(rows);
  const size_t lds = 0;
#define GRT_NB2(MC, RES)                                                                            \
  hipLaunchKernelGGL((norm_bwd_kernel<T, MC, RMS, RES>), dim3(nb), dim3(kNT), lds, s, (const T*)dy, \
                     (const T*)h, (const T*)w, mean, rstd, (const T*)dres, (T*)dx, ws, rows, d)
#define GRT_NB(MC)                                      \
  do {                                                  \
    if (dres != nullptr) GRT_NB2(MC, true);             \
    else GRT_NB2(MC, false);                            \
  } while (0)
  if (per_thr <= 1) GRT_NB(1);
  else if (per_thr <= 2) GRT_NB(2);
  else if (per_thr <= 4) GRT_NB(4);
  else GRT_NB(8);
#undef GRT_NB
#undef GRT_NB2
  if (ws == nullptr) return;
  const int ncols = RMS ? d : 2 * d;
  const dim3 cg((ncols + kColsumCols - 1) / kColsumCols);
  if (dw_t != nullptr && RMS) {  // weight gradient in T, straight into its gradient slot
    if (accumulate)
      hipLaunchKernelGGL((colsum_kernel<T, true>), cg, dim3(kNT), 0, s, ws, nb, d, ncols, (T*)dw_t, (T*)nullptr);
    else
      hipLaunchKernelGGL((colsum_kernel<T, false>), cg, dim3(kNT), 0, s, ws, nb, d, ncols, (T*)dw_t, (T*)nullptr);
  } else {
    hipLaunchKernelGGL((colsum_kernel<float, false>), cg, dim3(kNT), 0, s, ws, nb, d, ncols, dw, db);
  }
}

}  // namespace

int64_t norm_bwd_workspace_floats(int64_t rows, int d) { return (int64_t)bwd_blocks(rows) * 2 * d; }

void rmsnorm_fwd(DType dt, const void* x, const void* residual, const void* w, void* y, void* h_out,
                 float* rstd, int64_t rows, int d, float eps, hipStream_t s, int64_t ldy) {
  if (dt == DType::BF16)
    launch_fwd<bf16, true>(x, residual, w, nullptr, y, h_out, nullptr, rstd, rows, d, eps, s, ldy);
  else
    launch_fwd<float, true>(x, residual, w, nullptr, y, h_out, nullptr, rstd, rows, d, eps, s, ldy);
}

void rmsnorm_bwd(DType dt, const void* dy, const void* h, const void* w, const float* rstd,
                 const void* dres, void* dx, float* dw_f32, float* ws, int64_t rows, int d,
                 hipStream_t s, void* dw_t, int accumulate) {
  if (dt == DType::BF16)
    launch_bwd<bf16, true>(dy, h, w, nullptr, rstd, dres, dx, dw_f32, nullptr, ws, rows, d, s, dw_t, accumulate);
  else
    launch_bwd<float, true>(dy, h, w, nullptr, rstd, dres, dx, dw_f32, nullptr, ws, rows, d, s, dw_t, accumulate);
}

void layernorm_fwd(DType dt, const void* x, const void* residual, const void* w, const void* b,
                   void* y, void* h_out, float* mean, float* rstd, int64_t rows, int d, float eps,
                   hipStream_t s) {
  if (dt == DType::BF16)
    launch_fwd<bf16, false>(x, residual, w, b, y, h_out, mean, rstd, rows, d, eps, s);
  else
    launch_fwd<float, false>(x, residual, w, b, y, h_out, mean, rstd, rows, d, eps, s);
}

void layernorm_bwd(DType dt, const void* dy, const void* h, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* dw_f32, float* db_f32,
                   float* ws, int64_t rows, int d, hipStream_t s) {
  if (dt == DType::BF16)
    launch_bwd<bf16, false>(dy, h, w, mean, rstd, dres, dx, dw_f32, db_f32, ws, rows, d, s);
  else
    launch_bwd<float, false>(dy, h, w, mean, rstd, dres, dx, dw_f32, db_f32, ws, rows, d, s);
}

}  // namespace grt
