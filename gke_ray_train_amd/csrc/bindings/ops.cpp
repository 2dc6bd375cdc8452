// torch <-> HIP kernel bindings for gke_ray_train_amd._C.
//
// Every op launches on the caller's current HIP stream (graph-capturable: no allocation
// besides the torch caching allocator, no synchronisation) and checks shapes/strides on the
// host BEFORE launch so a hand-written kernel never sees operands its grid does not expect.
#include <climits>
#include <torch/extension.h>

#include <algorithm>
#include <cmath>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "grt_kernels.h"
#include "grt_sdma.h"

namespace {

using at::Tensor;
using c10::optional;

hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

grt::DType dtype_of(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return grt::DType::BF16;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "gke_ray_train_amd kernels support bf16/fp32, got ", t.scalar_type());
  return grt::DType::F32;
}

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_contig(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_vec(const Tensor& t, int64_t d, const char* name) {
  const int64_t vec = t.scalar_type() == at::kBFloat16 ? 8 : 4;
  TORCH_CHECK(d % vec == 0, name, ": last dim ", d, " must be a multiple of ", vec);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
const void* ptr_or_null(const optional<Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------ norms
// pad > 0: y is the [rows, d] view of a [rows, d + pad] buffer (row stride d + pad) whose last pad
// columns a consumer fills (the LoRA h of a K-concatenated projection, peft/lora.py)
std::vector<Tensor> rmsnorm_fwd(const Tensor& x, const optional<Tensor>& residual, const Tensor& w,
                                double eps, int64_t pad) {
  check_contig(x, "x");
  check_contig(w, "w");
  c10::OptionalDeviceGuard g(x.device());
  const int64_t d = x.size(-1), rows = x.numel() / d;
  check_vec(x, d, "x");
  TORCH_CHECK(w.numel() == d && w.scalar_type() == x.scalar_type(), "weight shape/dtype mismatch");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0 && (pad == 0 || x.dim() == 2), "rmsnorm_fwd: pad % 8 == 0 on [rows, d]");
  auto y = pad == 0 ? at::empty_like(x) : at::empty({rows, d + pad}, x.options()).narrow(1, 0, d);
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  Tensor h;
  if (residual.has_value()) {
    check_contig(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->scalar_type() == x.scalar_type(), "residual mismatch");
    h = at::empty_like(x);
  }
  grt::rmsnorm_fwd(dtype_of(x), x.data_ptr(), ptr_or_null(residual), w.data_ptr(), y.data_ptr(),
                   residual.has_value() ? h.data_ptr() : nullptr, rstd.data_ptr<float>(), rows, (int)d,
                   (float)eps, cur_stream(x), d + pad);
  return {y, residual.has_value() ? h : x, rstd};
}

// dw_out given: the weight gradient goes straight into it (parameter dtype, e.g. a data-parallel
// gradient slot; accumulate adds) and the second result is dw_out itself.
std::vector<Tensor> rmsnorm_bwd(const Tensor& dy, const Tensor& h, const Tensor& w, const Tensor& rstd,
                                const optional<Tensor>& dres, const optional<Tensor>& dw_out, bool accumulate) {
  check_contig(dy, "dy");
  check_contig(h, "h");
  c10::OptionalDeviceGuard g(dy.device());
  const int64_t d = h.size(-1), rows = h.numel() / d;
  TORCH_CHECK(dy.sizes() == h.sizes() && dy.scalar_type() == h.scalar_type(), "dy/h mismatch");
  if (dres.has_value()) {
    check_contig(*dres, "dres");
    TORCH_CHECK(dres->sizes() == h.sizes() && dres->scalar_type() == h.scalar_type(), "dres mismatch");
  }
  if (dw_out.has_value()) {
    check_contig(*dw_out, "dw_out");
    TORCH_CHECK(dw_out->numel() == d && dw_out->scalar_type() == h.scalar_type(), "dw_out: [d] in the dtype of h");
  }
  auto dx = at::empty_like(h);
  Tensor dw = dw_out.has_value() ? *dw_out : at::empty({d}, h.options().dtype(at::kFloat));
  auto ws = at::empty({grt::norm_bwd_workspace_floats(rows, (int)d)}, h.options().dtype(at::kFloat));
  grt::rmsnorm_bwd(dtype_of(h), dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(),
                   ptr_or_null(dres), dx.data_ptr(), dw_out.has_value() ? nullptr : dw.data_ptr<float>(),
                   ws.data_ptr<float>(), rows, (int)d, cur_stream(h),
                   dw_out.has_value() ? dw.data_ptr() : nullptr, accumulate ? 1 : 0);
  return {dx, dw};
}

// dX only (frozen norm weight: LoRA / QLoRA): no weight-gradient slab, no column-sum launch
Tensor rmsnorm_bwd_dx(const Tensor& dy, const Tensor& h, const Tensor& w, const Tensor& rstd,
                      const optional<Tensor>& dres) {
  check_contig(dy, "dy");
  check_contig(h, "h");
  c10::OptionalDeviceGuard g(dy.device());
  const int64_t d = h.size(-1), rows = h.numel() / d;
  TORCH_CHECK(dy.sizes() == h.sizes() && dy.scalar_type() == h.scalar_type(), "dy/h mismatch");
  TORCH_CHECK(w.numel() == d && w.scalar_type() == h.scalar_type() && rstd.numel() == rows, "w / rstd shapes");
  if (dres.has_value()) {
    check_contig(*dres, "dres");
    TORCH_CHECK(dres->sizes() == h.sizes() && dres->scalar_type() == h.scalar_type(), "dres mismatch");
  }
  auto dx = at::empty_like(h);
  grt::rmsnorm_bwd(dtype_of(h), dy.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr<float>(),
                   ptr_or_null(dres), dx.data_ptr(), nullptr, nullptr, rows, (int)d, cur_stream(h), nullptr, 0);
  return dx;
}

std::vector<Tensor> layernorm_fwd(const Tensor& x, const optional<Tensor>& residual, const Tensor& w,
                                  const optional<Tensor>& b, double eps) {
  check_contig(x, "x");
  c10::OptionalDeviceGuard g(x.device());
  const int64_t d = x.size(-1), rows = x.numel() / d;
  check_vec(x, d, "x");
  TORCH_CHECK(w.numel() == d && w.scalar_type() == x.scalar_type(), "weight shape/dtype mismatch");
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
  Tensor h;
  if (residual.has_value()) {
    check_contig(*residual, "residual");
    TORCH_CHECK(residual->sizes() == x.sizes(), "residual mismatch");
    h = at::empty_like(x);
  }
  grt::layernorm_fwd(dtype_of(x), x.data_ptr(), ptr_or_null(residual), w.data_ptr(), ptr_or_null(b),
                     y.data_ptr(), residual.has_value() ? h.data_ptr() : nullptr, mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), rows, (int)d, (float)eps, cur_stream(x));
  return {y, residual.has_value() ? h : x, mean, rstd};
}

std::vector<Tensor> layernorm_bwd(const Tensor& dy, const Tensor& h, const Tensor& w, const Tensor& mean,
                                  const Tensor& rstd, const optional<Tensor>& dres) {
  check_contig(dy, "dy");
  check_contig(h, "h");
  c10::OptionalDeviceGuard g(dy.device());
  const int64_t d = h.size(-1), rows = h.numel() / d;
  auto dx = at::empty_like(h);
  auto dw = at::empty({d}, h.options().dtype(at::kFloat));
  auto db = at::empty({d}, h.options().dtype(at::kFloat));
  auto ws = at::empty({grt::norm_bwd_workspace_floats(rows, (int)d)}, h.options().dtype(at::kFloat));
  grt::layernorm_bwd(dtype_of(h), dy.data_ptr(), h.data_ptr(), w.data_ptr(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), ptr_or_null(dres), dx.data_ptr(), dw.data_ptr<float>(),
                     db.data_ptr<float>(), ws.data_ptr<float>(), rows, (int)d, cur_stream(h));
  return {dx, dw, db};
}

// ------------------------------------------------------------------ elementwise
Tensor swiglu_fwd(const Tensor& gu, int64_t pad) {  // pad: as rmsnorm_fwd (a LoRA-tail row buffer)
  check_contig(gu, "gu");
  c10::OptionalDeviceGuard g(gu.device());
  const int64_t two_f = gu.size(-1), rows = gu.numel() / two_f, f = two_f / 2;
  check_vec(gu, f, "gu");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0 && (pad == 0 || gu.dim() == 2), "swiglu_fwd: pad % 8 == 0 on [rows, 2f]");
  auto sizes = gu.sizes().vec();
  sizes.back() = f;
  auto out = pad == 0 ? at::empty(sizes, gu.options()) : at::empty({rows, f + pad}, gu.options()).narrow(1, 0, f);
  grt::swiglu_fwd(dtype_of(gu), gu.data_ptr(), out.data_ptr(), rows, (int)f, cur_stream(gu), f + pad);
  return out;
}
Tensor swiglu_bwd(const Tensor& gu, const Tensor& dout) {
  check_contig(gu, "gu");
  check_contig(dout, "dout");
  c10::OptionalDeviceGuard g(gu.device());
  const int64_t two_f = gu.size(-1), rows = gu.numel() / two_f, f = two_f / 2;
  TORCH_CHECK(dout.numel() == rows * f, "dout shape mismatch");
  auto dgu = at::empty_like(gu);
  grt::swiglu_bwd(dtype_of(gu), gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), rows, (int)f, cur_stream(gu));
  return dgu;
}
// (out, out^T) or None when the shape is not handled
std::vector<Tensor> swiglu_fwd_t(const Tensor& gu, int64_t pad) {
  check_contig(gu, "gu");
  c10::OptionalDeviceGuard g(gu.device());
  const int64_t two_f = gu.size(-1), rows = gu.numel() / two_f, f = two_f / 2;
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && gu.is_cuda(), "swiglu_fwd_t: bf16 on the device");
  TORCH_CHECK(pad >= 0 && pad % 8 == 0 && (pad == 0 || gu.dim() == 2), "swiglu_fwd_t: pad % 8 == 0 on [rows, 2f]");
  if (rows % 64 != 0 || f % 128 != 0 || reinterpret_cast<uintptr_t>(gu.data_ptr()) % 16 != 0) return {};
  auto sizes = gu.sizes().vec();
  sizes.back() = f;
  auto out = pad == 0 ? at::empty(sizes, gu.options()) : at::empty({rows, f + pad}, gu.options()).narrow(1, 0, f);
  auto outT = at::empty({f, rows}, gu.options());
  if (!grt::swiglu_fwd_t(gu.data_ptr(), out.data_ptr(), outT.data_ptr(), rows, (int)f, cur_stream(gu), f + pad))
    return {};
  return {out, outT};
}
// (dgu, dgu^T) or None when the shape is not handled
std::vector<Tensor> swiglu_bwd_t(const Tensor& gu, const Tensor& dout) {
  check_contig(gu, "gu");
  check_contig(dout, "dout");
  c10::OptionalDeviceGuard g(gu.device());
  const int64_t two_f = gu.size(-1), rows = gu.numel() / two_f, f = two_f / 2;
  TORCH_CHECK(dout.numel() == rows * f && dout.scalar_type() == gu.scalar_type(), "dout shape mismatch");
  TORCH_CHECK(gu.scalar_type() == at::kBFloat16 && gu.is_cuda(), "swiglu_bwd_t: bf16 on the device");
  if (rows % 64 != 0 || f % 128 != 0 || reinterpret_cast<uintptr_t>(gu.data_ptr()) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16 != 0)
    return {};
  auto dgu = at::empty_like(gu);
  auto dguT = at::empty({two_f, rows}, gu.options());
  if (!grt::swiglu_bwd_t(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), rows, (int)f, cur_stream(gu)))
    return {};
  return {dgu, dguT};
}
Tensor gelu_fwd(const Tensor& x) {
  check_contig(x, "x");
  c10::OptionalDeviceGuard g(x.device());
  check_vec(x, x.numel(), "x");
  auto y = at::empty_like(x);
  grt::gelu_fwd(dtype_of(x), x.data_ptr(), y.data_ptr(), x.numel(), cur_stream(x));
  return y;
}
Tensor gelu_bwd(const Tensor& x, const Tensor& dy) {
  check_contig(x, "x");
  check_contig(dy, "dy");
  c10::OptionalDeviceGuard g(x.device());
  check_vec(x, x.numel(), "x");
  auto dx = at::empty_like(x);
  grt::gelu_bwd(dtype_of(x), x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), cur_stream(x));
  return dx;
}

void check_rope(const Tensor& cos, const Tensor& sin, const optional<Tensor>& pos, int64_t T, int64_t S, int64_t D) {
  check_contig(cos, "cos");
  check_contig(sin, "sin");
  TORCH_CHECK(cos.scalar_type() == at::kFloat && sin.scalar_type() == at::kFloat, "cos/sin must be fp32");
  TORCH_CHECK(cos.size(-1) == D / 2 && cos.numel() >= S * (D / 2) && sin.sizes() == cos.sizes(), "cos/sin shape");
  TORCH_CHECK(D % 16 == 0, "head_dim must be a multiple of 16");
  if (pos.has_value()) {
    check_contig(*pos, "pos");
    TORCH_CHECK(pos->scalar_type() == at::kInt && pos->numel() == T, "pos must be int32 [T]");
  }
}

// qkv: [T, ld] (row-contiguous), returns q [T, hq, D], k [T, hkv, D]
std::vector<Tensor> rope_fwd(const Tensor& qkv, const Tensor& cos, const Tensor& sin,
                             const optional<Tensor>& pos, int64_t hq, int64_t hkv, int64_t D, int64_t S) {
  check_cuda(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be [T, ld] with unit column stride");
  c10::OptionalDeviceGuard g(qkv.device());
  const int64_t T = qkv.size(0), ld = qkv.stride(0);
  TORCH_CHECK(qkv.size(1) >= (hq + hkv) * D, "qkv too narrow");
  TORCH_CHECK(ld % 8 == 0 && reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0, "qkv alignment");
  check_rope(cos, sin, pos, T, S, D);
  auto q = at::empty({T, hq, D}, qkv.options());
  auto k = at::empty({T, hkv, D}, qkv.options());
  grt::rope_fwd(dtype_of(qkv), qkv.data_ptr(), ld, q.data_ptr(), k.data_ptr(), cos.data_ptr<float>(),
                sin.data_ptr<float>(), pos.has_value() ? pos->data_ptr<int32_t>() : nullptr, T, (int)S,
                (int)hq, (int)hkv, (int)D, cur_stream(qkv));
  return {q, k};
}

// decode: q = rope(q) [T, hq, D]; kc[t / tpr, pos[t]] = rope(k), vc[t / tpr, pos[t]] = v (caches
// [B, L, hkv, D], last dim contiguous); a token whose position is outside [0, min(S, L)) is skipped
// entirely by the kernel (no cache write, its q row left unwritten)
Tensor rope_append(const Tensor& qkv, const Tensor& cos, const Tensor& sin, const Tensor& pos, int64_t hq, int64_t hkv,
                   int64_t D, int64_t S, Tensor& kc, Tensor& vc, int64_t tpr) {
  check_cuda(qkv, "qkv");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.scalar_type() == at::kBFloat16, "qkv must be bf16 [T, ld]");
  c10::OptionalDeviceGuard g(qkv.device());
  const int64_t T = qkv.size(0), ld = qkv.stride(0);
  TORCH_CHECK(qkv.size(1) >= (hq + 2 * hkv) * D && D % 16 == 0, "qkv too narrow / head dim");
  TORCH_CHECK(ld % 8 == 0 && reinterpret_cast<uintptr_t>(qkv.data_ptr()) % 16 == 0, "qkv alignment");
  check_rope(cos, sin, pos, T, S, D);
  for (const Tensor* c : {&kc, &vc}) {
    check_cuda(*c, "cache");
    TORCH_CHECK(c->dim() == 4 && c->size(2) == hkv && c->size(3) == D && c->stride(3) == 1 &&
                c->scalar_type() == at::kBFloat16, "cache must be bf16 [B, L, hkv, D] with unit last stride");
    TORCH_CHECK(c->stride(0) % 8 == 0 && c->stride(1) % 8 == 0 && c->stride(2) % 8 == 0 &&
                reinterpret_cast<uintptr_t>(c->data_ptr()) % 16 == 0, "cache alignment");
  }
  TORCH_CHECK(tpr >= 1 && T % tpr == 0 && T / tpr == kc.size(0) && vc.sizes() == kc.sizes(),
              "rope_append: T = B * tokens-per-row");
  auto q = at::empty({T, hq, D}, qkv.options());
  grt::rope_append(qkv.data_ptr(), ld, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), kc.stride(0), kc.stride(1),
                   kc.stride(2), vc.stride(0), vc.stride(1), vc.stride(2), cos.data_ptr<float>(), sin.data_ptr<float>(),
                   pos.data_ptr<int32_t>(), T, (int)tpr, (int)S, (int)kc.size(1), (int)hq, (int)hkv, (int)D,
                   cur_stream(qkv));
  return q;
}

void rope_bwd(const Tensor& dq, const Tensor& dk, Tensor& dqkv, const Tensor& cos, const Tensor& sin,
              const optional<Tensor>& pos, int64_t hq, int64_t hkv, int64_t D, int64_t S) {
  check_contig(dq, "dq");
  check_contig(dk, "dk");
  TORCH_CHECK(dqkv.dim() == 2 && dqkv.stride(1) == 1, "dqkv must be [T, ld]");
  c10::OptionalDeviceGuard g(dq.device());
  const int64_t T = dqkv.size(0), ld = dqkv.stride(0);
  TORCH_CHECK(dq.numel() == T * hq * D && dk.numel() == T * hkv * D, "dq/dk shape");
  check_rope(cos, sin, pos, T, S, D);
  grt::rope_bwd(dtype_of(dq), dq.data_ptr(), dk.data_ptr(), dqkv.data_ptr(), ld, cos.data_ptr<float>(),
                sin.data_ptr<float>(), pos.has_value() ? pos->data_ptr<int32_t>() : nullptr, T, (int)S,
                (int)hq, (int)hkv, (int)D, cur_stream(dq));
}

Tensor scale_add_pe(const Tensor& emb, const optional<Tensor>& pe, int64_t S, double scale) {
  check_contig(emb, "emb");
  c10::OptionalDeviceGuard g(emb.device());
  const int64_t d = emb.size(-1), T = emb.numel() / d;
  check_vec(emb, d, "emb");
  if (pe.has_value()) {
    check_contig(*pe, "pe");
    TORCH_CHECK(pe->scalar_type() == at::kFloat && pe->numel() >= S * d, "pe must be fp32 [>=S, d]");
  }
  auto out = at::empty_like(emb);
  grt::scale_add_pe(dtype_of(emb), emb.data_ptr(), pe.has_value() ? pe->data_ptr<float>() : nullptr,
                    out.data_ptr(), T, (int)S, (int)d, (float)scale, cur_stream(emb));
  return out;
}

void check_drop_p(double p) { TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1), got ", p); }

std::vector<Tensor> dropout_fwd(const Tensor& x, double p, int64_t seed, int64_t offset) {
  check_contig(x, "x");
  check_drop_p(p);
  c10::OptionalDeviceGuard g(x.device());
  auto y = at::empty_like(x);
  auto mask = at::empty(x.sizes(), x.options().dtype(at::kByte));
  grt::dropout_fwd(dtype_of(x), x.data_ptr(), y.data_ptr(), mask.data_ptr<uint8_t>(), x.numel(), (float)p,
                   (uint64_t)seed, (uint64_t)offset, cur_stream(x));
  return {y, mask};
}
Tensor dropout_bwd(const Tensor& dy, const Tensor& mask, double p) {
  check_contig(dy, "dy");
  check_drop_p(p);
  TORCH_CHECK(mask.numel() == dy.numel(), "dropout_bwd: mask / dy sizes differ");
  check_contig(mask, "mask");
  c10::OptionalDeviceGuard g(dy.device());
  auto dx = at::empty_like(dy);
  grt::dropout_bwd(dtype_of(dy), dy.data_ptr(), mask.data_ptr<uint8_t>(), dx.data_ptr(), dy.numel(), (float)p,
                   cur_stream(dy));
  return dx;
}
// mask-free variants: forward stores no mask; backward regenerates it and can accumulate into dx
Tensor dropout_fwd_seeded(const Tensor& x, double p, int64_t seed, int64_t offset) {
  check_contig(x, "x");
  check_drop_p(p);
  c10::OptionalDeviceGuard g(x.device());
  auto y = at::empty_like(x);
  grt::dropout_fwd(dtype_of(x), x.data_ptr(), y.data_ptr(), nullptr, x.numel(), (float)p, (uint64_t)seed,
                   (uint64_t)offset, cur_stream(x));
  return y;
}
void dropout_bwd_seeded(const Tensor& dy, const Tensor& dx, double p, int64_t seed, int64_t offset, bool accumulate) {
  check_contig(dy, "dy");
  check_contig(dx, "dx");
  check_drop_p(p);
  TORCH_CHECK(dy.numel() == dx.numel() && dy.scalar_type() == dx.scalar_type(), "dropout_bwd_seeded: shapes");
  c10::OptionalDeviceGuard g(dy.device());
  grt::dropout_bwd(dtype_of(dy), dy.data_ptr(), nullptr, dx.data_ptr(), dy.numel(), (float)p, cur_stream(dy),
                   (uint64_t)seed, (uint64_t)offset, accumulate);
}

// ------------------------------------------------------------------ LoRA adapter
// compute units of a device (cached)
static int device_cus(int dev) {
  static int cache[64] = {0};
  if (dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cache[dev] = v;
  }
  return cache[dev];
}

// (h, xd) = lora_down(x [M, K], a [R, K]): h = (x * keep / (1-p)) a^T, xd = x * keep / (1-p) when
// want_xd (same keep mask as dropout_fwd_seeded(x, p, seed, offset)). Returns {} when the shape is
// not supported by the kernel (the caller falls back to the torch path).
std::vector<Tensor> lora_down(const Tensor& x, const Tensor& a, double p, int64_t seed, int64_t offset,
                              bool want_xd, const optional<Tensor>& h_out, double hscale) {
  check_cuda(x, "x");
  check_contig(a, "a");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && a.dim() == 2 && a.size(1) == x.size(1), "lora_down: shapes");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && a.scalar_type() == at::kBFloat16, "lora_down: bf16");
  check_drop_p(p);
  const int64_t M = x.size(0);
  const int K = (int)x.size(1), R = (int)a.size(0);
  if (!grt::lora_down_supported(M, K, R, (int)x.stride(0), (uint64_t)offset) ||
      reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(a.data_ptr()) % 16)
    return {};
  c10::OptionalDeviceGuard g(x.device());
  Tensor h;
  if (h_out.has_value()) {  // e.g. the LoRA tail of the [x | h] row buffer (row stride > R)
    h = *h_out;
    TORCH_CHECK(h.dim() == 2 && h.size(0) == M && h.size(1) == R && h.stride(1) == 1 && h.stride(0) % 8 == 0 &&
                    h.scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(h.data_ptr()) % 16 == 0,
                "lora_down: h_out must be bf16 [M, R], unit column stride, 16-byte aligned rows");
  } else {
    h = at::empty({M, R}, x.options());
  }
  Tensor xd;
  if (want_xd) xd = at::empty({M, K}, x.options());
  grt::LoraDownParams lp{};
  lp.x = x.data_ptr(); lp.a = a.data_ptr(); lp.h = h.data_ptr(); lp.xd = want_xd ? xd.data_ptr() : nullptr;
  lp.M = M; lp.K = K; lp.R = R; lp.ldx = (int)x.stride(0);
  lp.p = (float)p; lp.seed = (uint64_t)seed; lp.offset = (uint64_t)offset;
  lp.ldh = h.stride(0); lp.hscale = (float)hscale;
  static const int split_env = [] { const char* e = getenv("GRT_LORA_DOWN_SPLIT"); return e ? atoi(e) : 0; }();
  lp.ksplit = split_env > 0 ? std::min(split_env, K / 128) : grt::lora_down_splits(M, K, R, device_cus(x.device().index()));
  Tensor hpart;
  if (lp.ksplit > 1) {
    hpart = at::empty({(int64_t)lp.ksplit, M, R}, x.options().dtype(at::kFloat));
    lp.hpart = hpart.data_ptr<float>();
  }
  grt::lora_down(lp, cur_stream(x));
  if (want_xd) return {h, xd};
  return {h};
}

// dx [M, K] (+)= keep / (1-p) * (g [M, R] @ at^T), at = A^T [K, R]; returns false (nothing done)
// when the shape is not supported by the kernel.
// g and dx may be row-strided (unit column stride); dx_in given: dx = dx_in + ... (dx_in row-strided too)
bool lora_dx(const Tensor& g, const Tensor& at, const Tensor& dx, double p, int64_t seed, int64_t offset,
             bool accumulate, const optional<Tensor>& dx_in, double gscale) {
  check_contig(at, "at");
  for (const Tensor* t : {&g, &dx}) {
    check_cuda(*t, "lora_dx operand");
    TORCH_CHECK(t->dim() == 2 && t->stride(1) == 1 && t->stride(0) % 8 == 0, "lora_dx: row-major operands");
  }
  if (dx_in.has_value()) {
    TORCH_CHECK(dx_in->sizes() == dx.sizes() && dx_in->stride(1) == 1 && dx_in->stride(0) % 8 == 0 &&
                    dx_in->scalar_type() == at::kBFloat16 && reinterpret_cast<uintptr_t>(dx_in->data_ptr()) % 16 == 0,
                "lora_dx: dx_in like dx");
  }
  TORCH_CHECK(g.dim() == 2 && at.dim() == 2 && dx.dim() == 2 && g.size(0) == dx.size(0) &&
                  at.size(0) == dx.size(1) && at.size(1) == g.size(1), "lora_dx: shapes");
  TORCH_CHECK(g.scalar_type() == at::kBFloat16 && at.scalar_type() == at::kBFloat16 &&
                  dx.scalar_type() == at::kBFloat16, "lora_dx: bf16");
  check_drop_p(p);
  const int64_t M = dx.size(0);
  const int K = (int)dx.size(1), R = (int)g.size(1);
  if (!grt::lora_dx_supported(M, K, R, (uint64_t)offset) || reinterpret_cast<uintptr_t>(dx.data_ptr()) % 16 ||
      reinterpret_cast<uintptr_t>(g.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(at.data_ptr()) % 16)
    return false;
  c10::OptionalDeviceGuard dg(dx.device());
  grt::LoraDxParams lp{};
  lp.g = g.data_ptr(); lp.at = at.data_ptr(); lp.dx = dx.data_ptr();
  lp.M = M; lp.K = K; lp.R = R;
  lp.p = (float)p; lp.seed = (uint64_t)seed; lp.offset = (uint64_t)offset; lp.accumulate = accumulate ? 1 : 0;
  lp.ldg = g.stride(0); lp.ld_out = dx.stride(0); lp.gscale = (float)gscale;
  if (dx_in.has_value()) { lp.dx_in = dx_in->data_ptr(); lp.ld_in = dx_in->stride(0); }
  grt::lora_dx(lp, cur_stream(dx));
  return true;
}

static bool rowmajor_bf16(const Tensor& t) {
  return t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 &&
         t.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
}

// c [M, 64] (+)= alpha * a [M, K] @ bt^T, bt = B^T [64, K] (lora_grad.hip); all row-major with unit
// column stride (row-strided views allowed). Returns false (nothing done) when unsupported.
// lora_g_group: up to 4 such products of the same M (one adapted module's targets) in one launch.
static bool lora_g_impl(const std::vector<Tensor>& as, const std::vector<Tensor>& bts, const std::vector<Tensor>& cs,
                        double alpha, bool accumulate) {
  const int n = (int)as.size();
  if (n < 1 || n > grt::kLoraGMax || (int)bts.size() != n || (int)cs.size() != n) return false;
  grt::LoraGParams p{};
  const int64_t M = as[0].size(0);
  int kmax = 0;
  for (int t = 0; t < n; ++t) {
    const Tensor &a = as[t], &bt = bts[t], &c = cs[t];
    if (!rowmajor_bf16(a) || !rowmajor_bf16(bt) || !rowmajor_bf16(c)) return false;
    const int K = (int)a.size(1);
    if (a.size(0) != M || bt.size(0) != c.size(1) || bt.size(1) != K || c.size(0) != M ||
        !grt::lora_g_supported(M, K, (int)c.size(1)) || c.stride(0) % 4 != 0 || c.get_device() != cs[0].get_device())
      return false;
    p.a[t] = a.data_ptr(); p.lda[t] = a.stride(0); p.bt[t] = bt.data_ptr(); p.ldbt[t] = bt.stride(0);
    p.c[t] = c.data_ptr(); p.ldc[t] = c.stride(0); p.K[t] = K;
    kmax = std::max(kmax, K);
  }
  for (int t = n; t < grt::kLoraGMax; ++t) {  // unused slots mirror product 0 (never indexed)
    p.a[t] = p.a[0]; p.lda[t] = p.lda[0]; p.bt[t] = p.bt[0]; p.ldbt[t] = p.ldbt[0];
    p.c[t] = p.c[0]; p.ldc[t] = p.ldc[0]; p.K[t] = p.K[0];
  }
  const Tensor& c0 = cs[0];
  c10::OptionalDeviceGuard dg(c0.device());
  p.nprod = n; p.M = M; p.alpha = (float)alpha; p.accumulate = accumulate ? 1 : 0;
  int kmin = kmax;
  for (int t = 0; t < n; ++t) kmin = std::min(kmin, p.K[t]);
  p.ks = grt::lora_g_splits(M, kmin, device_cus(c0.get_device()), n);
  Tensor ws;
  if (p.ks > 1) {
    ws = at::empty({(int64_t)n * p.ks * M * 64}, c0.options().dtype(at::kFloat));
    p.ws = ws.data_ptr<float>();
  }
  grt::lora_g(p, cur_stream(c0));
  return true;
}

bool lora_g(const Tensor& a, const Tensor& bt, const Tensor& c, double alpha, bool accumulate) {
  return lora_g_impl({a}, {bt}, {c}, alpha, accumulate);
}

bool lora_g_group(const std::vector<Tensor>& as, const std::vector<Tensor>& bts, const std::vector<Tensor>& cs,
                  double alpha, bool accumulate) {
  return lora_g_impl(as, bts, cs, alpha, accumulate);
}

// out (+)= alpha * a^T @ h, a [M, N], h [M, R]: out [N, R], or [R, N] when transpose (lora_grad.hip);
// fp32 token-split partials in a workspace from the caching allocator. False when unsupported.
// lora_tred_group: up to 4 such products of the same M and R (non-transposed; one adapted module's
// dB_i) in one launch, each assigning or accumulating.
static bool lora_tred_impl(const std::vector<Tensor>& as, const std::vector<Tensor>& hs, const std::vector<Tensor>& outs,
                           double alpha, const std::vector<bool>& accumulate, bool transpose) {
  const int n = (int)as.size();
  if (n < 1 || n > grt::kLoraTredMax || (int)hs.size() != n || (int)outs.size() != n || (int)accumulate.size() != n ||
      (transpose && n != 1))
    return false;
  const int64_t M = as[0].size(0);
  const int R = (int)hs[0].size(1);
  grt::LoraTredParams p{};
  int nbt = 0;
  for (int t = 0; t < n; ++t) {
    const Tensor &a = as[t], &h = hs[t], &out = outs[t];
    if (!rowmajor_bf16(a) || !rowmajor_bf16(h) || !rowmajor_bf16(out)) return false;
    const int N = (int)a.size(1);
    if (a.size(0) != M || h.size(0) != M || h.size(1) != R || !grt::lora_tred_supported(M, N, R)) return false;
    if (transpose ? (out.size(0) != R || out.size(1) != N) : (out.size(0) != N || out.size(1) != R)) return false;
    if (out.stride(0) % 4 != 0 || out.get_device() != outs[0].get_device()) return false;
    p.a[t] = a.data_ptr(); p.lda[t] = a.stride(0); p.h[t] = h.data_ptr(); p.ldh[t] = h.stride(0);
    p.out[t] = out.data_ptr(); p.ldo[t] = out.stride(0); p.N[t] = N; p.bo[t] = nbt;
    p.accumulate[t] = accumulate[t] ? 1 : 0;
    nbt += N / 128;
  }
  for (int t = n; t < grt::kLoraTredMax; ++t) {  // unused slots: never selected (bo past every block)
    p.a[t] = p.a[0]; p.lda[t] = p.lda[0]; p.h[t] = p.h[0]; p.ldh[t] = p.ldh[0];
    p.out[t] = p.out[0]; p.ldo[t] = p.ldo[0]; p.N[t] = p.N[0]; p.bo[t] = INT_MAX; p.accumulate[t] = 0;
  }
  const Tensor& o0 = outs[0];
  c10::OptionalDeviceGuard dg(o0.device());
  p.nprod = n; p.nbt = nbt; p.M = M; p.R = R;
  p.ks = grt::lora_tred_splits(M, nbt * 128, R, device_cus(o0.get_device()));
  Tensor ws = at::empty({(int64_t)p.ks * nbt * 128 * R}, o0.options().dtype(at::kFloat));
  p.ws = ws.data_ptr<float>();
  p.transpose = transpose ? 1 : 0; p.alpha = (float)alpha;
  grt::lora_tred(p, cur_stream(o0));
  return true;
}

bool lora_tred(const Tensor& a, const Tensor& h, const Tensor& out, double alpha, bool accumulate, bool transpose) {
  return lora_tred_impl({a}, {h}, {out}, alpha, {accumulate}, transpose);
}

bool lora_tred_group(const std::vector<Tensor>& as, const std::vector<Tensor>& hs, const std::vector<Tensor>& outs,
                     double alpha, const std::vector<bool>& accumulate) {
  return lora_tred_impl(as, hs, outs, alpha, accumulate, false);
}

// B_i [n_i, r] -> the adapter tail of W' [out, ldw] (columns col0 + j r ..) and of W'^T [.., ldt]
void lora_refresh(const std::vector<Tensor>& bs, const std::vector<int64_t>& offs, Tensor& w,
                  const optional<Tensor>& wt_opt, int64_t col0, int64_t wt_row0) {
  if (wt_row0 < 0) wt_row0 = col0;  // W'^T rows of the adapter block (a separate B^T buffer: 0)
  TORCH_CHECK(!bs.empty() && bs.size() <= 4 && offs.size() == bs.size(), "lora_refresh: 1-4 targets");
  TORCH_CHECK(w.dim() == 2 && w.stride(1) == 1 && w.scalar_type() == at::kBFloat16, "lora_refresh: bf16 W'");
  Tensor wt = wt_opt.has_value() ? *wt_opt : w.t();  // no W'^T: only the shape checks use the view
  if (wt_opt.has_value())
    TORCH_CHECK(wt.dim() == 2 && wt.stride(1) == 1 && wt.scalar_type() == at::kBFloat16 && wt.stride(0) % 8 == 0,
                "lora_refresh: bf16 W'^T");
  grt::LoraRefreshParams p{};
  p.ntarget = (int)bs.size();
  p.r = (int)bs[0].size(1);
  TORCH_CHECK(p.r % 64 == 0 && col0 % 8 == 0 && w.stride(0) % 8 == 0, "lora_refresh: r % 64");
  for (size_t j = 0; j < bs.size(); ++j) {
    check_contig(bs[j], "B");
    TORCH_CHECK(bs[j].scalar_type() == at::kBFloat16 && bs[j].size(1) == p.r && bs[j].size(0) % 64 == 0 &&
                    offs[j] % 8 == 0 && offs[j] + bs[j].size(0) <= w.size(0) &&
                    col0 + (int64_t)(j + 1) * p.r <= w.size(1) && wt_row0 + (int64_t)(j + 1) * p.r <= wt.size(0) &&
                    (!wt_opt.has_value() || offs[j] + bs[j].size(0) <= wt.size(1)),
                "lora_refresh: B_i bf16 [n % 64 == 0, r] inside W'");
    p.b[j] = bs[j].data_ptr(); p.off[j] = (int)offs[j]; p.n[j] = (int)bs[j].size(0);
  }
  p.w = w.data_ptr(); p.ldw = w.stride(0); p.col0 = (int)col0; p.trow0 = (int)wt_row0;
  p.wt = wt_opt.has_value() ? wt.data_ptr() : nullptr;
  p.ldt = wt_opt.has_value() ? wt.stride(0) : 0;
  c10::OptionalDeviceGuard g(w.device());
  grt::lora_refresh(p, cur_stream(w));
}

// ------------------------------------------------------------------ cross entropy
std::vector<Tensor> ce_fwd(const Tensor& logits, const Tensor& labels, int64_t ignore_index) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, V] row-major");
  check_contig(labels, "labels");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0), "labels must be int64 [N]");
  c10::OptionalDeviceGuard g(logits.device());
  const int64_t N = logits.size(0);
  auto loss = at::empty({N}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({N}, logits.options().dtype(at::kFloat));
  grt::cross_entropy_fwd(dtype_of(logits), logits.data_ptr(), logits.stride(0), labels.data_ptr<int64_t>(),
                         loss.data_ptr<float>(), lse.data_ptr<float>(), N, (int)logits.size(1), ignore_index,
                         cur_stream(logits));
  return {loss, lse};
}
Tensor ce_bwd(const Tensor& logits, const Tensor& labels, const Tensor& lse, const Tensor& gscale,
              int64_t ignore_index, bool inplace) {
  check_cuda(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [N, V] row-major");
  check_contig(gscale, "gscale");
  TORCH_CHECK(gscale.scalar_type() == at::kFloat && gscale.numel() == logits.size(0), "gscale fp32 [N]");
  c10::OptionalDeviceGuard g(logits.device());
  Tensor d = inplace ? logits : at::empty_like(logits, at::MemoryFormat::Contiguous);
  grt::cross_entropy_bwd(dtype_of(logits), logits.data_ptr(), logits.stride(0), labels.data_ptr<int64_t>(),
                         lse.data_ptr<float>(), gscale.data_ptr<float>(), d.data_ptr(), d.stride(0),
                         logits.size(0), (int)logits.size(1), ignore_index, cur_stream(logits));
  return d;
}

// ------------------------------------------------------------------ optimizer
int64_t sumsq_blocks() { return grt::optim_sumsq_blocks(); }
void sumsq(const Tensor& x, Tensor& ws, int64_t slot) {
  check_contig(x, "x");
  check_contig(ws, "ws");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.numel() >= (slot + 1) * grt::optim_sumsq_blocks(), "ws too small");
  c10::OptionalDeviceGuard g(x.device());
  grt::sumsq_accumulate(dtype_of(x), x.data_ptr(), x.numel(), ws.data_ptr<float>(), (int)slot, cur_stream(x));
}
void clip_finalize(const Tensor& ws, int64_t nparts, double max_norm, double prescale, Tensor& out) {
  check_contig(ws, "ws");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 2, "out must be fp32 [2]");
  c10::OptionalDeviceGuard g(ws.device());
  grt::clip_coef_finalize(ws.data_ptr<float>(), (int)nparts, (float)max_norm, (float)prescale, out.data_ptr<float>(),
                          cur_stream(ws));
}
void adamw(Tensor& p, const Tensor& gr, Tensor& m, Tensor& v, const optional<Tensor>& master, const Tensor& hyper,
           const optional<Tensor>& gscale, int64_t max_blocks, int64_t index_offset) {
  TORCH_CHECK(index_offset >= 0 && index_offset % 4 == 0, "adamw: index_offset must be a multiple of 4");
  check_contig(p, "p");
  check_contig(gr, "g");
  check_contig(m, "m");
  check_contig(v, "v");
  const int64_t n = p.numel();
  TORCH_CHECK(gr.numel() == n && m.numel() == n && v.numel() == n, "adamw size mismatch");
  TORCH_CHECK(m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat, "adam state must be fp32");
  TORCH_CHECK(hyper.scalar_type() == at::kFloat && hyper.numel() >= 10 && hyper.is_cuda(),
              "hyper fp32[10] on device: lr, b1, b2, eps, wd, bc1, bc2, gscale, stochastic_rounding, step");
  for (const Tensor* t : std::initializer_list<const Tensor*>{&p, &gr, &m, &v})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0 ||
                    (t->element_size() == 2 && reinterpret_cast<uintptr_t>(t->data_ptr()) % 8 == 0),
                "adamw operands must be vector aligned");
  if (master.has_value()) {
    check_contig(*master, "master");
    TORCH_CHECK(master->numel() == n && master->scalar_type() == at::kFloat, "master fp32 [n]");
  }
  c10::OptionalDeviceGuard g(p.device());
  grt::adamw_step(dtype_of(p), dtype_of(gr), p.data_ptr(), gr.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(),
                  master.has_value() ? master->data_ptr<float>() : nullptr, n, hyper.data_ptr<float>(),
                  gscale.has_value() ? gscale->data_ptr<float>() : nullptr, cur_stream(p), (int)max_blocks,
                  index_offset);
}
// AdamW on a bf16 weight [rows, cols] that also writes pt = W^T [cols, rows] (see optim.hip)
void adamw_t(Tensor& p, const Tensor& gr, Tensor& m, Tensor& v, const Tensor& hyper, const optional<Tensor>& gscale,
             Tensor& pt, int64_t index_offset) {
  for (const Tensor* t : std::initializer_list<const Tensor*>{&p, &gr, &m, &v, &pt}) check_contig(*t, "adamw_t operand");
  TORCH_CHECK(p.dim() == 2 && p.size(0) % 64 == 0 && p.size(1) % 128 == 0, "adamw_t: rows % 64 == 0, cols % 128 == 0");
  TORCH_CHECK(p.scalar_type() == at::kBFloat16 && gr.scalar_type() == at::kBFloat16 && pt.scalar_type() == at::kBFloat16,
              "adamw_t: bf16 param / grad / transpose");
  TORCH_CHECK(m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat, "adamw_t: fp32 moments");
  TORCH_CHECK(gr.numel() == p.numel() && m.numel() == p.numel() && v.numel() == p.numel(), "adamw_t: sizes");
  TORCH_CHECK(pt.dim() == 2 && pt.size(0) == p.size(1) && pt.size(1) == p.size(0), "adamw_t: pt must be [cols, rows]");
  TORCH_CHECK(hyper.scalar_type() == at::kFloat && hyper.numel() >= 10 && hyper.is_cuda(), "hyper fp32[10] on device");
  TORCH_CHECK(index_offset >= 0 && index_offset % 4 == 0, "adamw_t: index_offset must be a multiple of 4");
  for (const Tensor* t : std::initializer_list<const Tensor*>{&p, &gr, &m, &v, &pt})
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "adamw_t operands must be 16-byte aligned");
  c10::OptionalDeviceGuard g(p.device());
  grt::adamw_t_step(p.data_ptr(), gr.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(), pt.data_ptr(), p.size(0),
                    p.size(1), hyper.data_ptr<float>(), gscale.has_value() ? gscale->data_ptr<float>() : nullptr,
                    cur_stream(p), index_offset);
}

void scale_(Tensor& x, double a, const optional<Tensor>& a_ptr) {
  check_contig(x, "x");
  c10::OptionalDeviceGuard g(x.device());
  grt::scale_inplace(dtype_of(x), x.data_ptr(), x.numel(), (float)a,
                     a_ptr.has_value() ? a_ptr->data_ptr<float>() : nullptr, cur_stream(x));
}

// ------------------------------------------------------------------ attention
void check_bshd(const Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.dim() == 4, name, " must be [B, S, H, D]");
  TORCH_CHECK(t.stride(3) == 1, name, ": head_dim must be contiguous");
  if (t.scalar_type() == at::kBFloat16) {
    TORCH_CHECK(t.size(3) == 128, name, ": bf16 kernels need head_dim 128");
  } else {
    TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be bf16 or fp32");
    TORCH_CHECK(grt::attn_f32_supported((int)t.size(3)), name, ": fp32 kernels need head_dim 64 or 128");
  }
  const int64_t vec = 16 / t.element_size();
  TORCH_CHECK(t.stride(0) % vec == 0 && t.stride(1) % vec == 0 && t.stride(2) % vec == 0 &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, ": strides must keep 16-byte alignment");
}

grt::AttnParams make_params(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o, Tensor& lse,
                            double scale, bool causal, const optional<Tensor>& seqlens_k,
                            const optional<Tensor>& cu_seqlens = {}, int64_t max_seqlen = 0) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  check_bshd(o, "o");
  TORCH_CHECK(k.sizes() == v.sizes(), "k/v shape mismatch");
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() &&
                  o.scalar_type() == q.scalar_type(), "q/k/v/o dtype mismatch");
  TORCH_CHECK(k.size(3) == q.size(3), "head_dim mismatch");
  TORCH_CHECK(q.size(0) == k.size(0) && o.sizes() == q.sizes(), "batch/out shape mismatch");
  TORCH_CHECK(q.size(2) % k.size(2) == 0, "Hq must be a multiple of Hkv");
  const bool packed = cu_seqlens.has_value();
  const int64_t nseq = packed ? cu_seqlens->numel() - 1 : q.size(0);
  const int64_t sq_rows = packed ? max_seqlen : q.size(1);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == nseq * q.size(2) * sq_rows,
              "lse must be fp32 [B, Hq, Sq] ([num_seqs, Hq, max_seqlen] when packed)");
  grt::AttnParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr(); p.o = o.data_ptr(); p.lse = lse.data_ptr<float>();
  p.q_bs = q.stride(0); p.q_ss = q.stride(1); p.q_hs = q.stride(2);
  p.k_bs = k.stride(0); p.k_ss = k.stride(1); p.k_hs = k.stride(2);
  p.v_bs = v.stride(0); p.v_ss = v.stride(1); p.v_hs = v.stride(2);
  p.o_bs = o.stride(0); p.o_ss = o.stride(1); p.o_hs = o.stride(2);
  p.B = (int)q.size(0); p.Sq = (int)q.size(1); p.Sk = (int)k.size(1);
  p.Hq = (int)q.size(2); p.Hkv = (int)k.size(2); p.D = (int)q.size(3);
  p.scale = (float)scale;
  p.causal = causal ? 1 : 0;
  if (causal) TORCH_CHECK(p.Sk >= p.Sq, "causal attention needs Sk >= Sq");
  p.seqlens_k = nullptr;
  if (seqlens_k.has_value()) {
    check_contig(*seqlens_k, "seqlens_k");
    TORCH_CHECK(seqlens_k->scalar_type() == at::kInt && seqlens_k->numel() == q.size(0), "seqlens_k int32 [B]");
    p.seqlens_k = seqlens_k->data_ptr<int32_t>();
  }
  p.cu_seqlens = nullptr;
  if (packed) {  // padding-free: [1, T, H, D] tensors, sequence b = token rows [cu[b], cu[b+1])
    check_contig(*cu_seqlens, "cu_seqlens");
    TORCH_CHECK(cu_seqlens->scalar_type() == at::kInt && cu_seqlens->is_cuda() && nseq >= 1,
                "cu_seqlens must be int32 [num_seqs + 1] on the device");
    TORCH_CHECK(q.scalar_type() == at::kBFloat16, "packed (cu_seqlens) attention: bf16 kernels");
    TORCH_CHECK(q.size(0) == 1 && k.size(1) == q.size(1), "packed attention: q / k / v are [1, T, H, D]");
    TORCH_CHECK(causal && !seqlens_k.has_value(), "packed attention is causal self-attention without seqlens_k");
    TORCH_CHECK(max_seqlen >= 1 && max_seqlen <= q.size(1), "max_seqlen must be in [1, T]");
    p.cu_seqlens = cu_seqlens->data_ptr<int32_t>();
    p.B = (int)nseq;
    p.Sq = p.Sk = (int)max_seqlen;
    p.q_bs = p.k_bs = p.v_bs = p.o_bs = 0;
  }
  p.drop_seed = 0;
  p.drop_thresh = 0;
  p.drop_scale = 1.f;
  return p;
}

void set_dropout(grt::AttnParams& p, double dropout_p, int64_t seed) {
  TORCH_CHECK(dropout_p >= 0.0 && dropout_p < 1.0, "attention dropout p must be in [0, 1)");
  if (dropout_p <= 0.0) return;
  p.drop_seed = (uint32_t)(seed & 0xffffffffLL);
  p.drop_thresh = (uint32_t)std::min(4294967295.0, std::ceil(dropout_p * 4294967296.0));
  if (p.drop_thresh == 0) p.drop_thresh = 1;
  p.drop_scale = (float)(1.0 / (1.0 - dropout_p));
}

std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& out,
                             double scale, bool causal, const optional<Tensor>& seqlens_k, double dropout_p,
                             int64_t seed, const optional<Tensor>& cu_seqlens, int64_t max_seqlen,
                             const optional<Tensor>& o_t) {
  c10::OptionalDeviceGuard g(q.device());
  Tensor o = out.has_value() ? *out : at::empty(q.sizes(), q.options());
  auto lse = cu_seqlens.has_value()
                 ? at::empty({cu_seqlens->numel() - 1, q.size(2), max_seqlen}, q.options().dtype(at::kFloat))
                 : at::empty({q.size(0), q.size(2), q.size(1)}, q.options().dtype(at::kFloat));
  auto p = make_params(q, k, v, o, lse, scale, causal, seqlens_k, cu_seqlens, max_seqlen);
  set_dropout(p, dropout_p, seed);
  if (o_t.has_value()) {  // transposed output [Hq * D, B * S] beside o (o projection's weight gradient)
    check_contig(*o_t, "o_t");
    TORCH_CHECK(q.scalar_type() == at::kBFloat16 && p.D == 128 && o_t->scalar_type() == at::kBFloat16 &&
                    o_t->dim() == 2 && o_t->size(0) == (int64_t)p.Hq * p.D && o_t->size(1) == q.size(0) * q.size(1),
                "attn_fwd o_t: bf16, head_dim 128, shape [Hq * D, B * S]");
    p.o_t = o_t->data_ptr();
    p.ot_ld = o_t->size(1);
  }
  if (q.scalar_type() == at::kFloat) grt::attn_fwd_f32(p, cur_stream(q));
  else grt::attn_fwd(p, cur_stream(q));
  return {o, lse};
}

std::vector<Tensor> attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                             Tensor& lse, const optional<Tensor>& dq_out, const optional<Tensor>& dk_out,
                             const optional<Tensor>& dv_out, double scale, bool causal,
                             const optional<Tensor>& seqlens_k, double dropout_p, int64_t seed,
                             const optional<Tensor>& rope_cos, const optional<Tensor>& rope_sin,
                             const optional<Tensor>& cu_seqlens, int64_t max_seqlen, const optional<Tensor>& dqkv_t) {
  c10::OptionalDeviceGuard g(q.device());
  check_bshd(dout, "dout");
  TORCH_CHECK(dout.sizes() == q.sizes(), "dout shape");
  auto p = make_params(q, k, v, o, lse, scale, causal, seqlens_k, cu_seqlens, max_seqlen);
  set_dropout(p, dropout_p, seed);
  Tensor dq = dq_out.has_value() ? *dq_out : at::empty(q.sizes(), q.options());
  Tensor dk = dk_out.has_value() ? *dk_out : at::empty(k.sizes(), k.options());
  Tensor dv = dv_out.has_value() ? *dv_out : at::empty(v.sizes(), v.options());
  check_bshd(dq, "dq");
  check_bshd(dk, "dk");
  check_bshd(dv, "dv");
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(), "grad shapes");
  auto ws = at::empty({grt::attn_bwd_workspace_floats(p.B, p.Hq, p.Sq, p.D)}, q.options().dtype(at::kFloat));
  grt::AttnBwdParams bp{};
  bp.f = p;
  bp.dout = dout.data_ptr(); bp.do_bs = dout.stride(0); bp.do_ss = dout.stride(1); bp.do_hs = dout.stride(2);
  bp.dq = dq.data_ptr(); bp.dq_bs = dq.stride(0); bp.dq_ss = dq.stride(1); bp.dq_hs = dq.stride(2);
  bp.dk = dk.data_ptr(); bp.dk_bs = dk.stride(0); bp.dk_ss = dk.stride(1); bp.dk_hs = dk.stride(2);
  bp.dv = dv.data_ptr(); bp.dv_bs = dv.stride(0); bp.dv_ss = dv.stride(1); bp.dv_hs = dv.stride(2);
  if (cu_seqlens.has_value()) bp.do_bs = bp.dq_bs = bp.dk_bs = bp.dv_bs = 0;  // packed: one token axis
  bp.delta = ws.data_ptr<float>();
  TORCH_CHECK(rope_cos.has_value() == rope_sin.has_value(), "attn_bwd: rope_cos and rope_sin together");
  if (rope_cos.has_value()) {  // dQ / dK written un-rotated (q / k were rotated at position = index)
    check_contig(*rope_cos, "rope_cos");
    check_contig(*rope_sin, "rope_sin");
    TORCH_CHECK(q.scalar_type() == at::kBFloat16 && p.D == 128, "attn_bwd rope epilogue: bf16, head_dim 128");
    TORCH_CHECK(rope_cos->scalar_type() == at::kFloat && rope_sin->sizes() == rope_cos->sizes() &&
                    rope_sin->scalar_type() == at::kFloat && rope_cos->dim() == 2 && rope_cos->size(1) == p.D / 2 &&
                    rope_cos->size(0) >= std::max(p.Sq, p.Sk),
                "attn_bwd: rope tables fp32 [>= max(Sq, Sk), D / 2]");
    bp.rope_cos = rope_cos->data_ptr<float>();
    bp.rope_sin = rope_sin->data_ptr<float>();
  }
  TORCH_CHECK(dout.scalar_type() == q.scalar_type() && dq.scalar_type() == q.scalar_type() &&
                  dk.scalar_type() == q.scalar_type() && dv.scalar_type() == q.scalar_type(), "grad dtype mismatch");
  if (dqkv_t.has_value()) {  // transposed fused-QKV gradient [(Hq + 2 Hkv) D, B * S] beside dq / dk / dv
    check_contig(*dqkv_t, "dqkv_t");
    TORCH_CHECK(q.scalar_type() == at::kBFloat16 && p.D == 128 && dqkv_t->scalar_type() == at::kBFloat16,
                "attn_bwd dqkv_t: bf16, head_dim 128");
    TORCH_CHECK(p.Sq == p.Sk && dqkv_t->dim() == 2 && dqkv_t->size(0) == (int64_t)(p.Hq + 2 * p.Hkv) * p.D &&
                    dqkv_t->size(1) == q.size(0) * q.size(1),
                "attn_bwd dqkv_t: self-attention, shape [(Hq + 2 Hkv) * D, B * S]");
    bp.dqkv_t = dqkv_t->data_ptr();
    bp.t_ld = dqkv_t->size(1);
    bp.t_row_q = 0;
    bp.t_row_k = p.Hq * p.D;
    bp.t_row_v = (p.Hq + p.Hkv) * p.D;
  }
  if (q.scalar_type() == at::kFloat) grt::attn_bwd_f32(bp, cur_stream(q));
  else grt::attn_bwd(bp, cur_stream(q));
  return {dq, dk, dv};
}

Tensor attn_decode(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& seqlens_k, double scale) {
  check_bshd(q, "q");
  check_bshd(k, "k");
  check_bshd(v, "v");
  TORCH_CHECK(q.scalar_type() == at::kBFloat16 && k.scalar_type() == at::kBFloat16 && v.scalar_type() == at::kBFloat16,
              "attn_decode: bf16");
  TORCH_CHECK(q.size(1) == 1, "attn_decode: one query token per sequence");
  TORCH_CHECK(k.sizes() == v.sizes() && k.size(0) == q.size(0), "attn_decode: k/v shapes");
  const int64_t Hq = q.size(2), Hkv = k.size(2);
  TORCH_CHECK(Hq % Hkv == 0, "attn_decode: Hq % Hkv");
  const int64_t G = Hq / Hkv;
  TORCH_CHECK(G == 1 || G == 2 || G == 4 || G == 8, "attn_decode: GQA group must be 1, 2, 4 or 8");
  c10::OptionalDeviceGuard g(q.device());
  grt::AttnDecodeParams p{};
  p.q = q.data_ptr(); p.k = k.data_ptr(); p.v = v.data_ptr();
  auto o = at::empty(q.sizes(), q.options());
  p.o = o.data_ptr();
  p.q_bs = q.stride(0); p.q_hs = q.stride(2);
  p.k_bs = k.stride(0); p.k_ss = k.stride(1); p.k_hs = k.stride(2);
  p.v_bs = v.stride(0); p.v_ss = v.stride(1); p.v_hs = v.stride(2);
  p.o_bs = o.stride(0); p.o_hs = o.stride(2);
  p.B = (int)q.size(0); p.Hq = (int)Hq; p.Hkv = (int)Hkv; p.Sk = (int)k.size(1);
  p.NS = grt::attn_decode_splits(p.B, p.Hkv, p.Sk);
  p.seqlens_k = nullptr;
  if (seqlens_k.has_value()) {
    check_contig(*seqlens_k, "seqlens_k");
    TORCH_CHECK(seqlens_k->scalar_type() == at::kInt && seqlens_k->numel() == q.size(0), "seqlens_k int32 [B]");
    p.seqlens_k = seqlens_k->data_ptr<int32_t>();
  }
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  auto ws = at::empty({(int64_t)p.B * Hq * p.NS * (128 + 2)}, q.options().dtype(at::kFloat));
  p.part_o = ws.data_ptr<float>();
  p.part_m = p.part_o + (int64_t)p.B * Hq * p.NS * 128;
  p.part_l = p.part_m + (int64_t)p.B * Hq * p.NS;
  grt::attn_decode(p, cur_stream(q));
  return o;
}

// ------------------------------------------------------------------ NF4
std::vector<Tensor> nf4_quantize(const Tensor& w, int64_t blocksize) {
  check_contig(w, "w");
  c10::OptionalDeviceGuard g(w.device());
  const int64_t n = w.numel();
  TORCH_CHECK(n % blocksize == 0 && (blocksize == 32 || blocksize == 64 || blocksize == 128),
              "numel must be a multiple of blocksize (32/64/128)");
  auto q = at::empty({n / 2}, w.options().dtype(at::kByte));
  auto absmax = at::empty({n / blocksize}, w.options().dtype(at::kFloat));
  grt::nf4_quantize(dtype_of(w), w.data_ptr(), q.data_ptr<uint8_t>(), absmax.data_ptr<float>(), n, (int)blocksize,
                    cur_stream(w));
  return {q, absmax};
}
Tensor nf4_dequantize(const Tensor& q, const Tensor& absmax, int64_t n, int64_t blocksize, at::ScalarType dt,
                      const optional<Tensor>& out) {
  check_contig(q, "q");
  check_contig(absmax, "absmax");
  c10::OptionalDeviceGuard g(q.device());
  TORCH_CHECK(q.numel() * 2 == n && absmax.numel() * blocksize == n, "nf4 shapes");
  Tensor w = out.has_value() ? *out : at::empty({n}, q.options().dtype(dt));
  TORCH_CHECK(w.numel() == n && w.is_contiguous(), "out shape");
  grt::nf4_dequantize(dtype_of(w), q.data_ptr<uint8_t>(), absmax.data_ptr<float>(), w.data_ptr(), n, (int)blocksize,
                      cur_stream(q));
  return w;
}

// dequantise into out ([rows, cols] bf16 view, unit column stride, any row stride: the W head of a
// K-concatenated [W | B] buffer); false when the shape is not handled
bool nf4_dequantize_into(const Tensor& q, const Tensor& absmax, Tensor out, int64_t blocksize) {
  check_contig(q, "q");
  check_contig(absmax, "absmax");
  TORCH_CHECK(out.dim() == 2 && out.scalar_type() == at::kBFloat16 && out.stride(1) == 1 && out.is_cuda(),
              "nf4_dequantize_into: out must be a 2-D bf16 view with unit column stride");
  const int64_t rows = out.size(0), cols = out.size(1);
  TORCH_CHECK(q.numel() * 2 == rows * cols && absmax.numel() * blocksize == rows * cols, "nf4 shapes");
  TORCH_CHECK(rows <= INT32_MAX && cols <= INT32_MAX, "nf4_dequantize_into: dims");
  if (out.stride(0) % 8 != 0 || reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 != 0) return false;  // 16-byte stores
  c10::OptionalDeviceGuard g(q.device());
  return grt::nf4_dequantize_2d(q.data_ptr<uint8_t>(), absmax.data_ptr<float>(), out.data_ptr(), (int)rows,
                                (int)cols, out.stride(0), (int)blocksize, cur_stream(q));
}

Tensor nf4_dequantize_t(const Tensor& q, const Tensor& absmax, int64_t rows, int64_t cols, int64_t blocksize) {
  check_contig(q, "q");
  check_contig(absmax, "absmax");
  TORCH_CHECK(blocksize == 64 && cols % 64 == 0, "nf4_dequantize_t: blocksize 64 and cols % 64 == 0");
  TORCH_CHECK(q.numel() * 2 == rows * cols && absmax.numel() * blocksize == rows * cols, "nf4 shapes");
  TORCH_CHECK(rows <= INT32_MAX && cols <= INT32_MAX, "nf4_dequantize_t: dims");
  c10::OptionalDeviceGuard g(q.device());
  Tensor wt = at::empty({cols, rows}, q.options().dtype(at::kBFloat16));
  grt::nf4_dequantize_t(q.data_ptr<uint8_t>(), absmax.data_ptr<float>(), wt.data_ptr(), (int)rows, (int)cols,
                        (int)blocksize, cur_stream(q));
  return wt;
}

void transpose_into(const Tensor& src, Tensor& dst) {
  check_contig(src, "src");
  check_contig(dst, "dst");
  TORCH_CHECK(src.dim() == 2 && dst.dim() == 2 && src.scalar_type() == at::kBFloat16 &&
                  dst.scalar_type() == at::kBFloat16, "transpose: 2-D bf16");
  const int64_t R = src.size(0), Cc = src.size(1);
  TORCH_CHECK(dst.size(0) == Cc && dst.size(1) == R, "transpose: dst must be [cols, rows]");
  TORCH_CHECK(R % 64 == 0 && Cc % 64 == 0 && R <= INT32_MAX && Cc <= INT32_MAX, "transpose: dims must be multiples of 64");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "transpose: 16-byte alignment");
  c10::OptionalDeviceGuard g(src.device());
  grt::transpose_bf16(src.data_ptr(), dst.data_ptr(), (int)R, (int)Cc, cur_stream(src));
}

// dst <- src (same byte count, contiguous) on the GPU tensor's current stream by a DMA (SDMA)
// engine, never by a blit kernel on the compute units: hipMemcpyDeviceToDeviceNoCU with the pointers
// as they are (a pinned host tensor is addressed through its device mapping). The offloaded
// optimizer's device -> host moment write-backs otherwise run as ROCclr __amd_rocclr_copyBuffer
// kernels beside the step's compute (profiles/r5_offload70.md).
void copy_sdma(Tensor& dst, const Tensor& src) {
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "copy_sdma: contiguous tensors");
  const int64_t n = dst.numel() * dst.element_size();
  TORCH_CHECK(n == src.numel() * src.element_size(), "copy_sdma: byte counts differ");
  TORCH_CHECK(dst.is_cuda() || src.is_cuda(), "copy_sdma: one side must be a GPU tensor");
  TORCH_CHECK((dst.is_cuda() || dst.is_pinned()) && (src.is_cuda() || src.is_pinned()),
              "copy_sdma: host tensors must be pinned");
  if (n == 0) return;
  const Tensor& g = dst.is_cuda() ? dst : src;
  c10::OptionalDeviceGuard guard(g.device());
  const hipError_t e = hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), (size_t)n, hipMemcpyDeviceToDeviceNoCU,
                                      cur_stream(g));
  TORCH_CHECK(e == hipSuccess, "copy_sdma: hipMemcpyAsync: ", hipGetErrorString(e));
}

// dst (pinned host) <- src (device) on an SDMA engine, ordered on src's current stream through the
// HSA runtime (csrc/bindings/sdma_copy.cpp): the HIP route above still lands on a blit kernel for a
// device -> host copy on this image (profiles/r6_offload_link.md).
void sdma_d2h(Tensor& dst, const Tensor& src, int64_t producer_stream) {
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous(), "sdma_d2h: contiguous tensors");
  TORCH_CHECK(src.is_cuda() && !dst.is_cuda() && dst.is_pinned(), "sdma_d2h: device source, pinned host destination");
  const int64_t n = dst.numel() * dst.element_size();
  TORCH_CHECK(n == src.numel() * src.element_size(), "sdma_d2h: byte counts differ");
  c10::OptionalDeviceGuard guard(src.device());
  grt::sdma_d2h(dst.data_ptr(), src.data_ptr(), (size_t)n, src.get_device(), cur_stream(src),
                reinterpret_cast<hipStream_t>(producer_stream));
}

py::dict sdma_stats(int64_t device) {
  const grt::SdmaStats st = grt::sdma_stats((int)device);
  py::dict d;
  d["copies"] = st.copies;
  d["bytes"] = st.bytes;
  d["busy_s"] = st.busy_ns * 1e-9;
  d["error"] = st.error;
  d["engine"] = st.engine;
  d["engines_available"] = st.engines_available;
  d["engines_preferred"] = st.engines_preferred;
  return d;
}

// y = x W^T for 1-4 rows (1-16 rows when K % 256 == 0: 3+ rows run on MFMA); swiglu: x = [gate | up]
// [M, 2K] -> y = (silu(gate) * up) W^T
Tensor gemv(const Tensor& x, const Tensor& w, bool swiglu) {
  check_cuda(x, "x");
  check_contig(w, "w");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == (swiglu ? 2 : 1) * w.size(1),
              swiglu ? "gemv_swiglu: gu [M, 2K], w [N, K]" : "gemv: x [M, K], w [N, K]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "gemv: bf16");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK((M >= 1 && M <= 4) || (!swiglu && grt::gemv_mfma_ok((int)M, (int)K)),
              "gemv: 1..4 rows (5..16 without swiglu and with K % 256 == 0)");
  TORCH_CHECK(K % 8 == 0 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "gemv: K and row stride multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "gemv: 16-byte alignment");
  TORCH_CHECK(N <= INT32_MAX && K <= INT32_MAX, "gemv: dims");
  c10::OptionalDeviceGuard g(x.device());
  Tensor y = at::empty({M, N}, x.options());
  grt::gemv_bf16(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), N, (int)M, (int)N, (int)K, cur_stream(x),
                 swiglu);
  return y;
}

// Decode GEMV with the residual add / RMSNorm folded in (gemv.hip). sumsq: int64 [2, M, 64] fixed-point
// accumulators (zero-initialised once; the producers keep them consistent), slot: 0 / 1.
//   g given: y = bf16(x * rstd * g) W^T with rstd from sumsq[slot] (x = the residual stream h);
//   res given: y = bf16(x W^T) + res, its sums of squares added into sumsq[slot], sumsq[1 - slot]
//   zeroed for the next producer.
//   cos given (qkv, head_dim 128): RoPE in the epilogue at position pos[m]; returns q [M, hq, 128],
//   k / v written to cache slot pos[m] of kc / vc (rope_append semantics: bad positions write nothing).
Tensor gemv_fused(const Tensor& x, const Tensor& w, const Tensor& sumsq, int64_t slot, bool swiglu,
                  const c10::optional<Tensor>& g, const c10::optional<Tensor>& res, double eps,
                  const c10::optional<Tensor>& cos, const c10::optional<Tensor>& sin, const c10::optional<Tensor>& pos,
                  const c10::optional<Tensor>& kc, const c10::optional<Tensor>& vc, int64_t hq, int64_t hkv) {
  check_cuda(x, "x");
  check_contig(w, "w");
  check_contig(sumsq, "sumsq");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == (swiglu ? 2 : 1) * w.size(1), "gemv_fused: x [M, K], w [N, K]");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16, "gemv_fused: bf16");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(M >= 1 && M <= 4 && K % 8 == 0 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "gemv_fused: 1..4 rows, K % 8");
  TORCH_CHECK(N <= INT32_MAX && K <= INT32_MAX, "gemv_fused: dims");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "gemv_fused: 16-byte alignment");
  TORCH_CHECK(sumsq.scalar_type() == at::kLong && sumsq.numel() % 2 == 0 && sumsq.numel() / 2 >= M * 64 &&
                  (slot == 0 || slot == 1),
              "gemv_fused: sumsq int64 [2, >= M, 64], slot 0 / 1");
  auto* acc = reinterpret_cast<unsigned long long*>(sumsq.data_ptr<int64_t>());
  const int64_t stride = sumsq.numel() / 2;
  grt::GemvFused f{};
  f.x = x.data_ptr(), f.ldx = x.stride(0), f.w = w.data_ptr(), f.M = (int)M, f.N = (int)N, f.K = (int)K;
  f.swiglu = swiglu, f.eps = (float)eps;
  const bool normx = g.has_value() && g->defined();
  const bool resnorm = res.has_value() && res->defined();
  const bool rope = cos.has_value() && cos->defined();
  TORCH_CHECK(!(normx && resnorm) && (normx || resnorm || rope),
              "gemv_fused: g (normalise the input) or res (residual epilogue), and / or cos (RoPE epilogue)");
  TORCH_CHECK(!(rope && (resnorm || swiglu)), "gemv_fused: the RoPE epilogue is for the qkv projection");
  Tensor q;
  if (rope) {
    TORCH_CHECK(sin.has_value() && pos.has_value() && kc.has_value() && vc.has_value(), "gemv_fused: rope needs sin / pos / kc / vc");
    check_rope(*cos, *sin, *pos, M, cos->numel() / 64, 128);
    TORCH_CHECK(hq > 0 && hkv > 0 && N == (hq + 2 * hkv) * 128, "gemv_fused: rope N == (hq + 2 hkv) * 128");
    for (const Tensor* c : {&*kc, &*vc}) {
      check_cuda(*c, "cache");
      TORCH_CHECK(c->dim() == 4 && c->size(0) == M && c->size(2) == hkv && c->size(3) == 128 && c->stride(3) == 1 &&
                      c->scalar_type() == at::kBFloat16,
                  "gemv_fused: cache bf16 [M, L, hkv, 128]");
    }
    TORCH_CHECK(vc->sizes() == kc->sizes(), "gemv_fused: kc / vc shapes");
    q = at::empty({M, hq, 128}, x.options());
    f.q_out = q.data_ptr(), f.kc = kc->data_ptr(), f.vc = vc->data_ptr();
    f.c_bs = kc->stride(0), f.c_ss = kc->stride(1), f.c_hs = kc->stride(2);
    f.v_bs = vc->stride(0), f.v_ss = vc->stride(1), f.v_hs = vc->stride(2);
    f.cosb = cos->data_ptr<float>(), f.sinb = sin->data_ptr<float>(), f.pos = pos->data_ptr<int32_t>();
    f.rope_S = (int)(cos->numel() / 64), f.cache_L = (int)kc->size(1), f.hq = (int)hq, f.hkv = (int)hkv;
  }
  if (normx) {
    TORCH_CHECK(!swiglu, "gemv_fused: normx and swiglu are exclusive");
    check_contig(*g, "g");
    TORCH_CHECK(g->scalar_type() == at::kBFloat16 && g->numel() == K && reinterpret_cast<uintptr_t>(g->data_ptr()) % 16 == 0,
                "gemv_fused: g bf16 [K], 16-byte aligned");
    f.g = g->data_ptr(), f.sumsq_in = acc + slot * stride;
  } else if (resnorm) {
    check_cuda(*res, "res");
    TORCH_CHECK(res->dim() == 2 && res->size(0) == M && res->size(1) == N && res->stride(1) == 1 &&
                    res->scalar_type() == at::kBFloat16, "gemv_fused: res bf16 [M, N]");
    f.res = res->data_ptr(), f.ldr = res->stride(0);
    f.sumsq_out = acc + slot * stride, f.sumsq_zero = acc + (1 - slot) * stride;
  }
  c10::OptionalDeviceGuard dg(x.device());
  Tensor y = rope ? q : at::empty({M, N}, x.options());
  f.y = rope ? nullptr : y.data_ptr(), f.ldy = N;
  grt::gemv_fused_bf16(f, cur_stream(x));
  return y;
}

// ------------------------------------------------------------------ embedding
Tensor embedding_fwd(const Tensor& ids, const Tensor& w) {
  check_contig(ids, "ids");
  check_contig(w, "weight");
  TORCH_CHECK(ids.scalar_type() == at::kLong && w.dim() == 2, "embedding: int64 ids, 2-D weight");
  const int64_t d = w.size(1);
  TORCH_CHECK(d % 8 == 0, "embedding: row width must be a multiple of 8");
  c10::OptionalDeviceGuard g(w.device());
  auto out = at::empty({ids.numel(), d}, w.options());
  grt::embedding_fwd(dtype_of(w), ids.data_ptr<int64_t>(), w.data_ptr(), out.data_ptr(), ids.numel(), (int)d,
                     w.size(0), cur_stream(w));
  return out;
}

void embedding_bwd(const Tensor& dy, const Tensor& ids, const Tensor& dw, bool accumulate) {
  check_contig(dy, "dy");
  check_contig(dw, "dw");
  TORCH_CHECK(ids.scalar_type() == at::kLong, "embedding_bwd: int64 ids");
  TORCH_CHECK(dy.dim() == 2 && dw.dim() == 2 && dy.size(1) == dw.size(1) && dy.size(0) == ids.numel(),
              "embedding_bwd: shapes");
  TORCH_CHECK(dy.scalar_type() == dw.scalar_type(), "embedding_bwd: dtype");
  c10::OptionalDeviceGuard g(dy.device());
  const int64_t V = dw.size(0);
  auto flat = ids.reshape({-1});
  auto sorted = flat.sort();
  auto vals = std::get<0>(sorted);
  auto order = std::get<1>(sorted).contiguous();
  // segment bounds of every vocabulary row by binary search: no unique() (its output size would
  // force a device->host sync in the middle of the backward)
  auto rows = at::arange(V, vals.options());
  auto row_start = at::searchsorted(vals, rows, /*out_int32=*/true, /*right=*/false);
  auto row_end = at::searchsorted(vals, rows, /*out_int32=*/true, /*right=*/true);
  grt::embedding_bwd(dtype_of(dy), dy.data_ptr(), order.data_ptr<int64_t>(), row_start.data_ptr<int32_t>(),
                     row_end.data_ptr<int32_t>(), dw.data_ptr(), V, (int)dy.size(1), accumulate, cur_stream(dy));
}

// ------------------------------------------------------------------ weight-gradient GEMM
// out[P][Q] (+)= x[R][P]^T @ y[R][Q]  (dW = dY^T X); returns false when the shape is unsupported
bool gemm_wgrad(const Tensor& x, const Tensor& y, const Tensor& out, bool accumulate, int64_t mode) {
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && out.dim() == 2, "gemm_wgrad: 2-D operands");
  TORCH_CHECK(x.scalar_type() == at::kBFloat16 && y.scalar_type() == at::kBFloat16 &&
                  out.scalar_type() == at::kBFloat16, "gemm_wgrad: bf16 operands");
  TORCH_CHECK(x.is_cuda() && y.is_cuda() && out.is_cuda(), "gemm_wgrad: device tensors");
  const int64_t R = x.size(0), P = x.size(1), Q = y.size(1);
  TORCH_CHECK(y.size(0) == R && out.size(0) == P && out.size(1) == Q, "gemm_wgrad: shape mismatch");
  if (x.stride(1) != 1 || y.stride(1) != 1 || out.stride(1) != 1) return false;
  if (x.stride(0) % 8 || y.stride(0) % 8 || out.stride(0) % 8) return false;
  for (const Tensor* t : std::initializer_list<const Tensor*>{&x, &y, &out})
    if (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) return false;
  if (P > INT32_MAX || Q > INT32_MAX || R > INT32_MAX || !grt::gemm_tt_supported((int)P, (int)Q, (int)R))
    return false;
  c10::OptionalDeviceGuard g(x.device());
  grt::GemmTTParams p{x.data_ptr(), y.data_ptr(), out.data_ptr(), (int)P, (int)Q, (int)R,
                      x.stride(0), y.stride(0), out.stride(0), accumulate ? 1 : 0};
  grt::gemm_tt(p, cur_stream(x), (int)mode);
  return true;
}

// ------------------------------------------------------------------ projection GEMM
// out[M][N] (+)= a[M][K] @ b[N][K]^T on the hand-written MFMA kernel; returns false (nothing
// launched) when the shape / layout is outside what the kernel tiles, so callers can fall back.
bool gemm_supported(const Tensor& a, const Tensor& b, const Tensor& out) {
  if (a.dim() != 2 || b.dim() != 2 || out.dim() != 2) return false;
  if (a.scalar_type() != at::kBFloat16 || b.scalar_type() != at::kBFloat16 || out.scalar_type() != at::kBFloat16)
    return false;
  if (!a.is_cuda() || !b.is_cuda() || !out.is_cuda()) return false;
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  if (b.size(1) != K || out.size(0) != M || out.size(1) != N) return false;
  if (a.stride(1) != 1 || b.stride(1) != 1 || out.stride(1) != 1) return false;
  if (a.stride(0) % 8 || b.stride(0) % 8 || out.stride(0) % 8) return false;
  for (const Tensor* t : std::initializer_list<const Tensor*>{&a, &b, &out})
    if (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) return false;
  // the kernel's buffer descriptors address A and B with 32-bit byte offsets
  if (M * a.stride(0) * 2 >= (int64_t(1) << 31) || N * b.stride(0) * 2 >= (int64_t(1) << 31)) return false;
  return grt::gemm_nt_supported(M, N, K);
}

bool gemm_nt(const Tensor& a, const Tensor& b, const Tensor& out, bool accumulate, int64_t variant) {
  if (!gemm_supported(a, b, out)) return false;
  c10::OptionalDeviceGuard g(a.device());
  grt::GemmParams p{a.data_ptr(), b.data_ptr(), out.data_ptr(), (int)a.size(0), (int)b.size(0), (int)a.size(1),
                    a.stride(0), b.stride(0), out.stride(0), accumulate ? 1 : 0, grt::GEMM_EPI_STORE, (int)variant};
  grt::gemm_nt(p, cur_stream(a));
  return true;
}

// out[P][Q] (+)= x[R][P]^T @ y[R][Q] (dW = dY^T X) on the half-tile MFMA kernel reading the
// token-major operands through transposed LDS reads; false when the shape does not tile
bool gemm_wgrad2(const Tensor& x, const Tensor& y, const Tensor& out, bool accumulate) {
  if (x.dim() != 2 || y.dim() != 2 || out.dim() != 2) return false;
  if (x.scalar_type() != at::kBFloat16 || y.scalar_type() != at::kBFloat16 || out.scalar_type() != at::kBFloat16)
    return false;
  if (!x.is_cuda() || !y.is_cuda() || !out.is_cuda()) return false;
  const int64_t R = x.size(0), P = x.size(1), Q = y.size(1);
  if (y.size(0) != R || out.size(0) != P || out.size(1) != Q) return false;
  if (x.stride(1) != 1 || y.stride(1) != 1 || out.stride(1) != 1) return false;
  if (x.stride(0) % 8 || y.stride(0) % 8 || out.stride(0) % 8) return false;
  for (const Tensor* t : std::initializer_list<const Tensor*>{&x, &y, &out})
    if (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) return false;
  if (P % 256 || Q % 256 || R % 64 || R == 0 || P > INT32_MAX || Q > INT32_MAX || R > INT32_MAX) return false;
  c10::OptionalDeviceGuard g(x.device());
  grt::GemmParams p{x.data_ptr(), y.data_ptr(), out.data_ptr(), (int)P, (int)Q, (int)R,
                    x.stride(0), y.stride(0), out.stride(0), accumulate ? 1 : 0, grt::GEMM_EPI_STORE, 0};
  grt::gemm_tt2(p, cur_stream(x));
  return true;
}

// out[M][N] (+)= a[M][K] @ b[K][N] (dX = dY W on W as stored [N_out][K_in]); false when unsupported
bool gemm_nn(const Tensor& a, const Tensor& b, const Tensor& out, bool accumulate) {
  if (a.dim() != 2 || b.dim() != 2 || out.dim() != 2) return false;
  if (a.scalar_type() != at::kBFloat16 || b.scalar_type() != at::kBFloat16 || out.scalar_type() != at::kBFloat16)
    return false;
  if (!a.is_cuda() || !b.is_cuda() || !out.is_cuda()) return false;
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  if (b.size(0) != K || out.size(0) != M || out.size(1) != N) return false;
  if (a.stride(1) != 1 || b.stride(1) != 1 || out.stride(1) != 1) return false;
  if (a.stride(0) % 8 || b.stride(0) % 8 || out.stride(0) % 8) return false;
  for (const Tensor* t : std::initializer_list<const Tensor*>{&a, &b, &out})
    if (reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) return false;
  if (M % 256 || N % 256 || K % 64 || K == 0 || M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return false;
  c10::OptionalDeviceGuard g(a.device());
  grt::GemmParams p{a.data_ptr(), b.data_ptr(), out.data_ptr(), (int)M, (int)N, (int)K,
                    a.stride(0), b.stride(0), out.stride(0), accumulate ? 1 : 0, grt::GEMM_EPI_STORE, 0};
  grt::gemm_nn(p, cur_stream(a));
  return true;
}

// ------------------------------------------------------------------ xGMI IPC collectives
int64_t ipc_alloc(int64_t nbytes, bool fine_grained, int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  return reinterpret_cast<int64_t>(grt::ipc_malloc(nbytes, fine_grained));
}
void ipc_free_ptr(int64_t p, int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  grt::ipc_free(reinterpret_cast<void*>(p));
}
py::bytes ipc_handle(int64_t p, int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  char h[grt::kIpcHandleBytes];
  grt::ipc_get_handle(reinterpret_cast<void*>(p), h);
  return py::bytes(h, grt::kIpcHandleBytes);
}
int64_t ipc_open(const py::bytes& handle, int64_t device) {
  std::string h = handle;
  TORCH_CHECK((int)h.size() == grt::kIpcHandleBytes, "ipc_open: handle must be ", grt::kIpcHandleBytes, " bytes");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  return reinterpret_cast<int64_t>(grt::ipc_open_handle(h.data()));
}
void ipc_close(int64_t p, int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  grt::ipc_close_handle(reinterpret_cast<void*>(p));
}

grt::IpcPeers make_peers(const std::vector<int64_t>& staging, const std::vector<int64_t>& result,
                         const std::vector<int64_t>& signal, const Tensor& err, int64_t cap, int64_t rank,
                         int64_t timeout_ticks) {
  const int64_t W = (int64_t)staging.size();
  TORCH_CHECK(W >= 1 && W <= grt::kIpcMaxRanks, "ipc: world size must be 1..", grt::kIpcMaxRanks);
  TORCH_CHECK((int64_t)result.size() == W && (int64_t)signal.size() == W, "ipc: pointer lists differ in length");
  TORCH_CHECK(rank >= 0 && rank < W, "ipc: bad rank");
  check_contig(err, "err");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1, "ipc: err must be an int32 device tensor");
  grt::IpcPeers p{};
  for (int64_t i = 0; i < W; ++i) {
    TORCH_CHECK(staging[i] && result[i] && signal[i], "ipc: null peer buffer");
    p.staging[i] = reinterpret_cast<void*>(staging[i]);
    p.result[i] = reinterpret_cast<void*>(result[i]);
    p.signal[i] = reinterpret_cast<uint32_t*>(signal[i]);
  }
  p.err = reinterpret_cast<uint32_t*>(err.data_ptr());
  p.cap = cap;
  p.rank = (int)rank;
  p.world = (int)W;
  p.timeout_ticks = (uint64_t)timeout_ticks;
  return p;
}

void ipc_allreduce(const std::vector<int64_t>& staging, const std::vector<int64_t>& result,
                   const std::vector<int64_t>& signal, const Tensor& err, int64_t cap, int64_t rank, int64_t epoch,
                   int64_t timeout_ticks, const Tensor& in, const Tensor& out, bool two_shot, double scale) {
  const grt::IpcPeers p = make_peers(staging, result, signal, err, cap, rank, timeout_ticks);
  check_contig(in, "in");
  check_contig(out, "out");
  TORCH_CHECK(in.device() == err.device() && out.device() == err.device(), "ipc: tensors on another device");
  TORCH_CHECK(in.scalar_type() == out.scalar_type() && in.numel() == out.numel(), "ipc: in/out mismatch");
  const int64_t nbytes = in.numel() * in.element_size();
  TORCH_CHECK(nbytes % 16 == 0, "ipc: message must be a multiple of 16 bytes (pad it)");
  TORCH_CHECK(nbytes <= cap, "ipc: message of ", nbytes, " bytes exceeds the buffer (", cap, ")");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "ipc: 16-byte alignment required");
  c10::OptionalDeviceGuard g(in.device());
  grt::ipc_allreduce(p, (uint32_t)epoch, dtype_of(in), in.data_ptr(), out.data_ptr(), nbytes, two_shot, (float)scale,
                     cur_stream(in));
}

void ipc_barrier(const std::vector<int64_t>& staging, const std::vector<int64_t>& result,
                 const std::vector<int64_t>& signal, const Tensor& err, int64_t cap, int64_t rank, int64_t epoch,
                 int64_t timeout_ticks) {
  const grt::IpcPeers p = make_peers(staging, result, signal, err, cap, rank, timeout_ticks);
  c10::OptionalDeviceGuard g(err.device());
  grt::ipc_barrier(p, (uint32_t)epoch, cur_stream(err));
}

// A HIP stream whose dispatches may only use the CUs set in `mask` (32 CUs per word). Used for
// side-stream work (the overlapped optimizer) that must leave the other CUs to the compute
// stream's GEMMs instead of filling every CU's wave slots. Returned as an integer handle for
// torch.cuda.ExternalStream; it lives for the process (streams are few and reused).
int64_t cu_masked_stream(const std::vector<int64_t>& mask, int64_t device) {
  TORCH_CHECK(!mask.empty(), "cu_masked_stream: empty mask");
  std::vector<uint32_t> words(mask.size());
  bool any = false;
  for (size_t i = 0; i < mask.size(); ++i) {
    TORCH_CHECK(mask[i] >= 0 && mask[i] <= 0xffffffffLL, "cu_masked_stream: mask word out of range");
    words[i] = (uint32_t)mask[i];
    any = any || words[i] != 0;
  }
  TORCH_CHECK(any, "cu_masked_stream: mask selects no CU");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words.size(), words.data());
  TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
  return reinterpret_cast<int64_t>(s);
}

std::vector<int64_t> stream_cu_mask(int64_t stream, int64_t words) {
  TORCH_CHECK(words > 0 && words <= 64, "stream_cu_mask: 1..64 words");
  std::vector<uint32_t> w((size_t)words, 0u);
  const hipError_t e = hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)words, w.data());
  TORCH_CHECK(e == hipSuccess, "hipExtStreamGetCUMask: ", hipGetErrorString(e));
  return std::vector<int64_t>(w.begin(), w.end());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gke_ray_train_amd HIP kernels for gfx950 (MI355X)";
  m.def("rmsnorm_fwd", &rmsnorm_fwd, py::arg("x"), py::arg("residual"), py::arg("w"), py::arg("eps"),
        py::arg("pad") = 0);
  m.def("rmsnorm_bwd", &rmsnorm_bwd, py::arg("dy"), py::arg("h"), py::arg("w"), py::arg("rstd"), py::arg("dres"),
        py::arg("dw_out") = py::none(), py::arg("accumulate") = false);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("swiglu_fwd", &swiglu_fwd, py::arg("gu"), py::arg("pad") = 0);
  m.def("swiglu_bwd", &swiglu_bwd);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("rope_fwd", &rope_fwd);
  m.def("rope_bwd", &rope_bwd);
  m.def("rope_append", &rope_append);
  m.def("scale_add_pe", &scale_add_pe);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("dropout_bwd", &dropout_bwd);
  m.def("dropout_fwd_seeded", &dropout_fwd_seeded);
  m.def("lora_down", &lora_down, py::arg("x"), py::arg("a"), py::arg("p"), py::arg("seed"), py::arg("offset"),
        py::arg("want_xd"), py::arg("h_out") = py::none(), py::arg("hscale") = 1.0);
  m.def("lora_dx", &lora_dx, py::arg("g"), py::arg("at"), py::arg("dx"), py::arg("p"), py::arg("seed"),
        py::arg("offset"), py::arg("accumulate"), py::arg("dx_in") = py::none(), py::arg("gscale") = 1.0);
  m.def("lora_refresh", &lora_refresh, py::arg("bs"), py::arg("offs"), py::arg("w"), py::arg("wt"), py::arg("col0"),
        py::arg("wt_row0") = -1);
  m.def("lora_g", &lora_g, py::arg("a"), py::arg("bt"), py::arg("c"), py::arg("alpha"), py::arg("accumulate"));
  m.def("lora_g_group", &lora_g_group, py::arg("a"), py::arg("bt"), py::arg("c"), py::arg("alpha"),
        py::arg("accumulate"));
  m.def("lora_tred", &lora_tred, py::arg("a"), py::arg("h"), py::arg("out"), py::arg("alpha"), py::arg("accumulate"),
        py::arg("transpose"));
  m.def("lora_tred_group", &lora_tred_group, py::arg("a"), py::arg("h"), py::arg("out"), py::arg("alpha"),
        py::arg("accumulate"));
  m.def("dropout_bwd_seeded", &dropout_bwd_seeded);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("sumsq_blocks", &sumsq_blocks);
  m.def("lds_fill", [](int64_t pattern, int64_t device) {
    c10::OptionalDeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
    grt::lds_fill((uint32_t)pattern, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device).stream());
  }, "test support: fill every CU's LDS with a 32-bit pattern (stale-LDS-read detection)");
  m.def("sumsq", &sumsq);
  m.def("clip_finalize", &clip_finalize);
  m.def("adamw", &adamw, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("master"),
        py::arg("hyper"), py::arg("gscale"), py::arg("max_blocks") = 0, py::arg("index_offset") = 0);
  m.def("adamw_t", &adamw_t);
  m.def("scale_", &scale_);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("out"), py::arg("scale"),
        py::arg("causal"), py::arg("seqlens_k"), py::arg("dropout_p") = 0.0, py::arg("seed") = 0,
        py::arg("cu_seqlens") = py::none(), py::arg("max_seqlen") = 0, py::arg("o_t") = py::none());
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("scale"), py::arg("causal"),
        py::arg("seqlens_k"), py::arg("dropout_p") = 0.0, py::arg("seed") = 0, py::arg("rope_cos") = py::none(),
        py::arg("rope_sin") = py::none(), py::arg("cu_seqlens") = py::none(), py::arg("max_seqlen") = 0,
        py::arg("dqkv_t") = py::none());
  m.def("attn_set_schedule", &grt::attn_set_schedule,
        "bf16 attention causal-pair / XCD-grouped schedule, bit mask: 1 = forward, 2 = dQ, 4 = dK/dV");
  m.def("attn_get_schedule", &grt::attn_get_schedule);
  m.def("attn_set_dkdv_form", &grt::attn_set_dkdv_form, "dK / dV kernel: 1 = 4-wave, 2 = wave-pair (default)");
  m.def("attn_get_dkdv_form", &grt::attn_get_dkdv_form);
  m.def("attn_set_dma_fast", &grt::attn_set_dma_fast, "1 = hoisted LDS-DMA addressing (default), 0 = clamped per tile");
  m.def("ew_set_fast", &grt::ew_set_fast, "1 = single-pass RoPE (D = 128) / SwiGLU kernels (default), 0 = grid-stride kernels");
  m.def("attn_set_skip_dead", &grt::attn_set_skip_dead,
        "1 = forward / dK-dV waves skip the causal tiles they mask entirely (default), 0 = compute them");
  m.def("nf4_quantize", &nf4_quantize);
  m.def("nf4_dequantize", &nf4_dequantize);
  m.def("nf4_dequantize_t", &nf4_dequantize_t);
  m.def("nf4_dequantize_into", &nf4_dequantize_into);
  m.def("rmsnorm_bwd_dx", &rmsnorm_bwd_dx);
  m.def("swiglu_fwd_t", &swiglu_fwd_t);
  m.def("swiglu_bwd_t", &swiglu_bwd_t);
  m.def("transpose_into", &transpose_into);
  m.def("copy_sdma", &copy_sdma);
  m.def("sdma_d2h", &sdma_d2h, py::arg("dst"), py::arg("src"), py::arg("producer_stream") = 0,
        "pinned host <- device on an SDMA engine, ordered on the source's current stream; producer_stream "
        "(a raw stream handle): the stream whose work so far wrote src");
  m.def("sdma_stats", &sdma_stats, "copies / bytes / worker busy seconds / first error of the SDMA copier");
  m.def("sdma_clear_error", [](int64_t device) { grt::sdma_clear_error((int)device); });
  m.def("gemv", &gemv, py::arg("x"), py::arg("w"), py::arg("swiglu") = false);
  m.def("gemv_fused", &gemv_fused, py::arg("x"), py::arg("w"), py::arg("sumsq"), py::arg("slot"),
        py::arg("swiglu") = false, py::arg("g") = py::none(), py::arg("res") = py::none(), py::arg("eps") = 1e-5,
        py::arg("cos") = py::none(), py::arg("sin") = py::none(), py::arg("pos") = py::none(),
        py::arg("kc") = py::none(), py::arg("vc") = py::none(), py::arg("hq") = 0, py::arg("hkv") = 0);
  m.def("attn_decode", &attn_decode);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("gemm_wgrad", &gemm_wgrad, py::arg("x"), py::arg("y"), py::arg("out"), py::arg("accumulate"),
        py::arg("mode") = 0);
  m.def("gemm_supported", &gemm_supported, py::arg("a"), py::arg("b"), py::arg("out"));
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("accumulate") = false,
        py::arg("variant") = 0);
  m.def("gemm_wgrad2", &gemm_wgrad2, py::arg("x"), py::arg("y"), py::arg("out"), py::arg("accumulate") = false);
  m.def("gemm_nn", &gemm_nn, py::arg("a"), py::arg("b"), py::arg("out"), py::arg("accumulate") = false);
  m.def("ipc_alloc", &ipc_alloc);
  m.def("ipc_free", &ipc_free_ptr);
  m.def("ipc_handle", &ipc_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("ipc_allreduce", &ipc_allreduce);
  m.def("ipc_barrier", &ipc_barrier);
  m.def("cu_masked_stream", &cu_masked_stream);
  m.def("stream_cu_mask", &stream_cu_mask);
  m.attr("IPC_MAX_RANKS") = grt::kIpcMaxRanks;
  m.attr("IPC_SIGNAL_BYTES") = grt::kIpcSignalBytes;
}
