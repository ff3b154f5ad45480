// pybind11 registrations of the non-GEMM kernels.  Host-side validation of every
// pointer/shape/dtype happens here before the launch.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CK(cond, ...) TORCH_CHECK(cond, __VA_ARGS__)
#define GPU(x) CK((x).is_cuda(), #x " must be a GPU tensor")
#define BF16(x) CK((x).scalar_type() == at::kBFloat16 && (x).is_contiguous(), #x " must be contiguous bf16")
#define F32(x) CK((x).scalar_type() == at::kFloat && (x).is_contiguous(), #x " must be contiguous fp32")
#define HIP_OK(expr)                                                                  \
  do {                                                                                \
    int _e = (expr);                                                                  \
    CK(_e == 0, "HIP launch failed: ", hipGetErrorString((hipError_t)_e)); \
  } while (0)

template <class T>
T* optr(const c10::optional<at::Tensor>& t) {
  return t ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// ---------------------------------------------------------------- batch norm
void bn_stats_(const at::Tensor& x, const at::Tensor& ws, int64_t C) {
  GPU(x); BF16(x); F32(ws);
  CK(C % 8 == 0 && x.numel() % C == 0, "bn_stats: C % 8 and numel % C");
  CK(ws.numel() >= (int64_t)bn_partial_rows(x.numel() / C, (int)C) * 2 * C, "bn_stats: workspace too small");
  at::DeviceGuard g(x.device());
  HIP_OK(bn_stats(x.data_ptr(), ws.data_ptr<float>(), x.numel() / C, (int)C, cur_stream()));
}

void splitk_finalize_(const at::Tensor& ws, const at::Tensor& y, int64_t C, c10::optional<at::Tensor> bias, bool relu,
                      c10::optional<at::Tensor> stats, int64_t splits, int64_t brows, int64_t zbias) {
  GPU(ws); F32(ws); BF16(y);
  CK(C % 8 == 0 && y.numel() % C == 0 && y.is_contiguous() && ws.is_contiguous(), "splitk_finalize: shapes");
  // splits == 0: ws is the [M, C] atomic accumulator (zeroed again); splits > 0: `splits` [M, C] slabs
  CK(splits >= 0 && ws.numel() >= std::max<int64_t>(splits, 1) * y.numel() && (splits > 0 || ws.numel() == y.numel()),
     "splitk_finalize: workspace size");
  // brows > 0 (replica batching): rows r use bias + (r / brows) * zbias
  if (bias) {
    F32(*bias);
    CK(brows > 0 ? (zbias % 4 == 0 && bias->numel() >= ((y.numel() / C - 1) / brows) * zbias + C) : bias->numel() == C,
       "splitk_finalize: bias [C] (or per-replica biases every zbias elements)");
  }
  if (stats) { F32(*stats); CK(stats->numel() == (int64_t)kBnShards * 2 * C, "splitk_finalize: stats [32, 2, C]"); }
  at::DeviceGuard g(ws.device());
  HIP_OK(splitk_finalize(ws.data_ptr<float>(), y.data_ptr(), optr<const float>(bias), optr<float>(stats), y.numel() / C,
                         (int)C, relu ? 1 : 0, (int)splits, (long)y.numel(), cur_stream(), (long)brows, (long)zbias));
}

int64_t bn_partial_rows_(int64_t M, int64_t C) { return bn_partial_rows(M, (int)C); }

// S (partial rows) = ws.numel() / (2C)
void bn_finalize_(const at::Tensor& ws, int64_t M, int64_t C, c10::optional<at::Tensor> gamma,
                  c10::optional<at::Tensor> beta, double eps, double momentum, c10::optional<at::Tensor> rmean,
                  c10::optional<at::Tensor> rvar, const at::Tensor& smean, const at::Tensor& sinv,
                  const at::Tensor& scale, const at::Tensor& shift) {
  GPU(ws); F32(ws); F32(smean); F32(sinv); F32(scale); F32(shift);
  CK(smean.numel() >= C && sinv.numel() >= C && scale.numel() >= C && shift.numel() >= C, "bn_finalize: sizes");
  CK(ws.numel() % (2 * C) == 0, "bn_finalize: ws must be [S][2][C]");
  at::DeviceGuard g(ws.device());
  HIP_OK(bn_finalize(ws.data_ptr<float>(), (int)(ws.numel() / (2 * C)), M, (int)C, optr<const float>(gamma),
                     optr<const float>(beta), (float)eps, (float)momentum, optr<float>(rmean), optr<float>(rvar),
                     smean.data_ptr<float>(), sinv.data_ptr<float>(), scale.data_ptr<float>(),
                     shift.data_ptr<float>(), cur_stream()));
}

void bn_apply_(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift, c10::optional<at::Tensor> resid,
               const at::Tensor& y, int64_t C, bool relu, c10::optional<at::Tensor> mask,
               c10::optional<at::Tensor> res_scale, c10::optional<at::Tensor> res_shift) {
  GPU(x); BF16(x); BF16(y); F32(scale); F32(shift);
  CK(C % 8 == 0 && x.numel() % C == 0 && y.numel() == x.numel(), "bn_apply: shapes");
  if (resid) { BF16(*resid); CK(resid->numel() == x.numel(), "bn_apply: resid shape"); }
  CK(res_scale.has_value() == res_shift.has_value() && (!res_scale || resid), "bn_apply: res_scale/res_shift pair needs resid");
  if (res_scale) {
    F32(*res_scale); F32(*res_shift);
    CK(res_scale->numel() == C && res_shift->numel() == C && res_scale->is_contiguous() && res_shift->is_contiguous(),
       "bn_apply: res_scale/res_shift [C]");
  }
  if (mask) {
    CK(mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() >= (x.numel() / 8 + 3) / 4 * 4,
       "bn_apply: mask must be uint8 [numel / 8 rounded up to 4] (one byte per 8 channels)");
  }
  at::DeviceGuard g(x.device());
  HIP_OK(bn_apply(x.data_ptr(), scale.data_ptr<float>(), shift.data_ptr<float>(), optr<const void>(resid), y.data_ptr(),
                  optr<void>(mask), x.numel() / C, (int)C, relu ? 1 : 0, cur_stream(), optr<const float>(res_scale),
                  optr<const float>(res_shift)));
}

// relu mask mode: 0 none; 1 from y (forward output); 2 recomputed from x*scale+shift
void bn_bwd_reduce_(const at::Tensor& dy, const at::Tensor& x, c10::optional<at::Tensor> y,
                    c10::optional<at::Tensor> scale, c10::optional<at::Tensor> shift, const at::Tensor& mean,
                    const at::Tensor& ws, int64_t C, int64_t mode) {
  GPU(dy); BF16(dy); BF16(x); F32(mean); F32(ws);
  CK(dy.numel() == x.numel() && x.numel() % C == 0 && C % 8 == 0, "bn_bwd_reduce: shapes");
  if (mode == 1) { CK(y.has_value(), "mode 1 needs y"); BF16(*y); CK(y->numel() == x.numel(), "bn_bwd_reduce: y shape"); }
  if (mode == 3) CK(y.has_value() && y->scalar_type() == at::kByte && y->numel() >= x.numel() / 8,
                    "mode 3 needs the uint8 bit mask of bn_apply");
  CK(mode >= 0 && mode <= 3, "bn_bwd_reduce: mode");
  if (mode == 2) { CK(scale.has_value() && shift.has_value(), "mode 2 needs scale/shift"); F32(*scale); F32(*shift); }
  CK(ws.numel() >= (int64_t)bn_partial_rows(x.numel() / C, (int)C) * 2 * C, "bn_bwd_reduce: workspace too small");
  at::DeviceGuard g(x.device());
  HIP_OK(bn_bwd_reduce(dy.data_ptr(), x.data_ptr(), optr<const void>(y), optr<const float>(scale),
                       optr<const float>(shift), mean.data_ptr<float>(), ws.data_ptr<float>(), x.numel() / C, (int)C,
                       (int)mode, cur_stream()));
}

void bn_bwd_finalize_(const at::Tensor& ws, int64_t M, int64_t C, c10::optional<at::Tensor> gamma,
                      const at::Tensor& mean, const at::Tensor& invstd, c10::optional<at::Tensor> dgamma,
                      c10::optional<at::Tensor> dbeta, const at::Tensor& coef) {
  GPU(ws); F32(ws); F32(mean); F32(invstd); F32(coef);
  CK(coef.numel() >= 3 * C, "bn_bwd_finalize: coef size");
  CK(ws.numel() % (2 * C) == 0, "bn_bwd_finalize: ws must be [S][2][C]");
  at::DeviceGuard g(ws.device());
  HIP_OK(bn_bwd_finalize(ws.data_ptr<float>(), (int)(ws.numel() / (2 * C)), M, (int)C, optr<const float>(gamma), mean.data_ptr<float>(),
                         invstd.data_ptr<float>(), optr<float>(dgamma), optr<float>(dbeta), coef.data_ptr<float>(),
                         cur_stream()));
}

void bn_bwd_dx_(const at::Tensor& dy, const at::Tensor& x, c10::optional<at::Tensor> y,
                c10::optional<at::Tensor> scale, c10::optional<at::Tensor> shift, const at::Tensor& coef,
                const at::Tensor& dx, c10::optional<at::Tensor> dres, int64_t C, int64_t mode) {
  GPU(dy); BF16(dy); BF16(x); BF16(dx); F32(coef);
  CK(dy.numel() == x.numel() && dx.numel() == x.numel() && x.numel() % C == 0 && C % 8 == 0, "bn_bwd_dx: shapes");
  CK(coef.numel() >= 3 * C, "bn_bwd_dx: coef size");
  if (mode == 1) { CK(y.has_value(), "mode 1 needs y"); BF16(*y); CK(y->numel() == x.numel(), "bn_bwd_dx: y shape"); }
  if (mode == 3) CK(y.has_value() && y->scalar_type() == at::kByte && y->numel() >= x.numel() / 8,
                    "mode 3 needs the uint8 bit mask of bn_apply");
  CK(mode >= 0 && mode <= 3, "bn_bwd_dx: mode");
  if (mode == 2) { CK(scale.has_value() && shift.has_value(), "mode 2 needs scale/shift"); F32(*scale); F32(*shift); }
  if (dres) { BF16(*dres); CK(dres->numel() == x.numel(), "bn_bwd_dx: dres shape"); }
  at::DeviceGuard g(x.device());
  HIP_OK(bn_bwd_dx(dy.data_ptr(), x.data_ptr(), optr<const void>(y), optr<const float>(scale),
                   optr<const float>(shift), coef.data_ptr<float>(), dx.data_ptr(), optr<void>(dres), x.numel() / C,
                   (int)C, (int)mode, cur_stream()));
}

// bn_bwd_dx plus the fused reduce of a second BN consuming dy' (the ResNet downsample BN): x2 [M, C] bf16,
// mean2 [C], ws2 [bn_partial_rows(M, C)][2][C] (every row written)
void bn_bwd_dx_red_(const at::Tensor& dy, const at::Tensor& x, c10::optional<at::Tensor> y,
                    c10::optional<at::Tensor> scale, c10::optional<at::Tensor> shift, const at::Tensor& coef,
                    const at::Tensor& dx, int64_t C, int64_t mode, const at::Tensor& x2, const at::Tensor& mean2,
                    const at::Tensor& ws2) {
  GPU(dy); BF16(dy); BF16(x); BF16(dx); F32(coef); BF16(x2); F32(mean2); F32(ws2);
  CK(dy.numel() == x.numel() && dx.numel() == x.numel() && x2.numel() == x.numel() && x.numel() % C == 0 && C % 8 == 0,
     "bn_bwd_dx_red: shapes");
  CK(coef.numel() >= 3 * C && mean2.numel() >= C, "bn_bwd_dx_red: coef / mean2 size");
  CK(ws2.numel() >= (int64_t)bn_partial_rows(x.numel() / C, (int)C) * 2 * C, "bn_bwd_dx_red: workspace too small");
  if (mode == 1) { CK(y.has_value(), "mode 1 needs y"); BF16(*y); CK(y->numel() == x.numel(), "bn_bwd_dx_red: y shape"); }
  if (mode == 3) CK(y.has_value() && y->scalar_type() == at::kByte && y->numel() >= x.numel() / 8,
                    "mode 3 needs the uint8 bit mask of bn_apply");
  CK(mode >= 0 && mode <= 3, "bn_bwd_dx_red: mode");
  if (mode == 2) { CK(scale.has_value() && shift.has_value(), "mode 2 needs scale/shift"); F32(*scale); F32(*shift); }
  at::DeviceGuard g(x.device());
  HIP_OK(bn_bwd_dx(dy.data_ptr(), x.data_ptr(), optr<const void>(y), optr<const float>(scale),
                   optr<const float>(shift), coef.data_ptr<float>(), dx.data_ptr(), nullptr, x.numel() / C, (int)C,
                   (int)mode, cur_stream(), x2.data_ptr(), mean2.data_ptr<float>(), ws2.data_ptr<float>()));
}

// stem BN backward through the 3x3 / 2 / pad-1 max pool: dy [N, Ho, Wo, C] pooled gradient, am its argmax
// bytes, x [N, H, W, C] the pre-BN conv output; phase 0: reduce partials into ws; phase 1: dx with coef
void pool3s2_bn_bwd_(const at::Tensor& dy, const at::Tensor& am, const at::Tensor& x, const at::Tensor& scale,
                     const at::Tensor& shift, const at::Tensor& mean, const at::Tensor& coef_or_ws,
                     c10::optional<at::Tensor> dx, int64_t k) {
  GPU(dy); BF16(dy); BF16(x); F32(scale); F32(shift); F32(mean); F32(coef_or_ws);
  CK(dy.dim() == 4 && x.dim() == 4 && dy.size(0) == x.size(0) && dy.size(3) == x.size(3) && dy.is_contiguous() &&
     x.is_contiguous(), "pool3s2_bn_bwd: NHWC dy / x");
  CK(am.scalar_type() == at::kByte && am.numel() == dy.numel() && am.is_contiguous(), "pool3s2_bn_bwd: argmax bytes");
  const int N = (int)x.size(0), H = (int)x.size(1), W = (int)x.size(2), C = (int)x.size(3);
  const int Ho = (int)dy.size(1), Wo = (int)dy.size(2);
  CK(pool3s2_bn_bwd_ok(N, H, W, C, Ho, Wo, (int)k), "pool3s2_bn_bwd: 3x3 / 2 / pad-1 (k = 3) or 2x2 / 2 (k = 2) pool, ",
     "C % 8 == 0, C <= 2048");
  CK(scale.numel() >= C && shift.numel() >= C && mean.numel() >= C, "pool3s2_bn_bwd: per-channel vectors");
  if (dx) {
    BF16(*dx);
    CK(dx->numel() == x.numel() && dx->is_contiguous() && coef_or_ws.numel() >= 3 * C, "pool3s2_bn_bwd: dx / coef");
  } else {
    CK(coef_or_ws.numel() % (2 * C) == 0 && coef_or_ws.numel() / (2 * C) <= 16384, "pool3s2_bn_bwd: ws [S][2][C]");
  }
  at::DeviceGuard g(x.device());
  HIP_OK(pool3s2_bn_bwd(dy.data_ptr(), am.data_ptr<uint8_t>(), x.data_ptr(), scale.data_ptr<float>(),
                        shift.data_ptr<float>(), mean.data_ptr<float>(), dx ? coef_or_ws.data_ptr<float>() : nullptr,
                        dx ? nullptr : coef_or_ws.data_ptr<float>(), (int)(coef_or_ws.numel() / (2 * C)),
                        dx ? dx->data_ptr() : nullptr, N, H, W, C, Ho, Wo,
                        cur_stream(), (int)k));
}

// ---------------------------------------------------------------- pooling
void maxpool_fwd_(const at::Tensor& x, const at::Tensor& y, const at::Tensor& am, int64_t kh, int64_t kw, int64_t sh,
                  int64_t sw, int64_t ph, int64_t pw, c10::optional<at::Tensor> scale, c10::optional<at::Tensor> shift) {
  GPU(x); BF16(x); BF16(y);
  CK(am.scalar_type() == at::kByte && am.is_contiguous(), "argmax must be uint8");
  CK(x.dim() == 4 && y.dim() == 4, "maxpool: NHWC tensors");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Ho = y.size(1), Wo = y.size(2);
  CK(C % 8 == 0 && y.size(0) == N && y.size(3) == C && am.numel() == y.numel(), "maxpool: shapes");
  CK(kh * kw <= 256, "maxpool: window too large for byte argmax");
  at::DeviceGuard g(x.device());
  CK(scale.has_value() == shift.has_value(), "maxpool: scale and shift together");
  if (scale) {
    F32(*scale); F32(*shift);
    CK(scale->numel() == C && shift->numel() == C && scale->is_contiguous() && shift->is_contiguous() &&
           ((uintptr_t)scale->data_ptr() % 16) == 0 && ((uintptr_t)shift->data_ptr() % 16) == 0,
       "maxpool: per-channel scale / shift [C], 16-B aligned");
  }
  HIP_OK(maxpool_fwd(x.data_ptr(), y.data_ptr(), am.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                     cur_stream(), optr<const float>(scale), optr<const float>(shift)));
}

void maxpool_bwd_(const at::Tensor& dy, const at::Tensor& am, const at::Tensor& dx, int64_t kh, int64_t kw, int64_t sh,
                  int64_t sw, int64_t ph, int64_t pw) {
  GPU(dy); BF16(dy); BF16(dx);
  const int N = dx.size(0), H = dx.size(1), W = dx.size(2), C = dx.size(3), Ho = dy.size(1), Wo = dy.size(2);
  CK(C % 8 == 0 && dy.size(3) == C && am.numel() == dy.numel(), "maxpool_bwd: shapes");
  at::DeviceGuard g(dy.device());
  HIP_OK(maxpool_bwd(dy.data_ptr(), am.data_ptr<uint8_t>(), dx.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw,
                     cur_stream()));
}

void avgpool_fwd_(const at::Tensor& x, const at::Tensor& y) {
  GPU(x); BF16(x); BF16(y);
  CK(x.dim() == 4, "avgpool: NHWC");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  CK(C % 8 == 0 && y.numel() == (int64_t)N * C, "avgpool: shapes");
  at::DeviceGuard g(x.device());
  HIP_OK(avgpool_global_fwd(x.data_ptr(), y.data_ptr(), N, HW, C, cur_stream()));
}

void avgpool_bwd_(const at::Tensor& dy, const at::Tensor& dx) {
  GPU(dy); BF16(dy); BF16(dx);
  const int N = dx.size(0), HW = dx.size(1) * dx.size(2), C = dx.size(3);
  CK(C % 8 == 0 && dy.numel() == (int64_t)N * C, "avgpool_bwd: shapes");
  at::DeviceGuard g(dy.device());
  HIP_OK(avgpool_global_bwd(dy.data_ptr(), dx.data_ptr(), N, HW, C, cur_stream()));
}

// ---------------------------------------------------------------- loss
void softmax_xent_(const at::Tensor& logits, c10::optional<at::Tensor> labels, c10::optional<at::Tensor> probs,
                   c10::optional<at::Tensor> loss_rows, c10::optional<at::Tensor> dlogits, double grad_scale, double smoothing,
                   int64_t ignore_index, c10::optional<at::Tensor> grad_scale_dev, c10::optional<at::Tensor> loss_out,
                   double out_scale, int64_t zrows) {
  GPU(logits);
  CK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) >= logits.size(1),
     "softmax_xent: logits [B,K] with unit column stride");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  CK(bf || logits.scalar_type() == at::kFloat, "softmax_xent: logits bf16/fp32");
  const int B = logits.size(0), K = logits.size(1);
  CK(loss_rows.has_value() || loss_out.has_value(), "softmax_xent: loss_rows and/or loss_out");
  if (loss_rows) { F32(*loss_rows); CK(loss_rows->numel() == B, "loss_rows size"); }
  // zrows > 0 (replica batching): loss_out[z] = the loss of rows [z * zrows, (z + 1) * zrows)
  const int64_t nz = zrows > 0 ? (B + zrows - 1) / zrows : 1;
  if (loss_out) { F32(*loss_out); CK(loss_out->numel() == nz && nz <= 64 && B <= 4096, "softmax_xent: loss_out [B / zrows <= 64], B <= 4096 (one workgroup)"); }
  CK(zrows == 0 || loss_out.has_value(), "softmax_xent: zrows needs loss_out");
  CK((labels.has_value()) != (probs.has_value()), "exactly one of labels/probs");
  if (labels) CK(labels->scalar_type() == at::kLong && labels->numel() == B, "labels int64 [B]");
  if (probs) { F32(*probs); CK(probs->numel() == (int64_t)B * K, "probs [B,K]"); }
  const long ld = logits.stride(0);
  if (dlogits)
    CK(dlogits->scalar_type() == logits.scalar_type() && dlogits->dim() == 2 && dlogits->size(0) == B &&
           dlogits->stride(0) == ld && dlogits->stride(1) == 1,
       "dlogits: same layout as logits");
  if (grad_scale_dev) { F32(*grad_scale_dev); CK(grad_scale_dev->numel() == 1 && grad_scale_dev->is_cuda(), "grad_scale_dev: one fp32 on the GPU"); }
  at::DeviceGuard g(logits.device());
  HIP_OK(softmax_xent(logits.data_ptr(), bf ? 1 : 0, optr<const int64_t>(labels), optr<const float>(probs),
                      optr<float>(loss_rows), optr<void>(dlogits), B, K, ld, (float)grad_scale, (float)smoothing,
                      (int)ignore_index, cur_stream(), optr<const float>(grad_scale_dev), optr<float>(loss_out),
                      (float)out_scale, (int)zrows));
}

void label_count_inv_(const at::Tensor& labels, int64_t ignore_index, const at::Tensor& inv) {
  GPU(labels); F32(inv);
  CK(labels.scalar_type() == at::kLong && labels.is_contiguous() && inv.numel() == 1, "label_count_inv: int64 labels, inv [1]");
  at::DeviceGuard g(labels.device());
  HIP_OK(label_count_inv(labels.data_ptr<int64_t>(), labels.numel(), (int)ignore_index, inv.data_ptr<float>(), cur_stream()));
}

void rows_sum_scaled_(const at::Tensor& rows, double scale, c10::optional<at::Tensor> dev, const at::Tensor& out) {
  GPU(rows); F32(rows); F32(out);
  CK(rows.is_contiguous() && out.numel() == 1, "rows_sum_scaled: rows contiguous, out [1]");
  if (dev) { F32(*dev); CK(dev->numel() == 1, "rows_sum_scaled: dev [1]"); }
  at::DeviceGuard g(rows.device());
  HIP_OK(rows_sum_scaled(rows.data_ptr<float>(), rows.numel(), (float)scale, optr<const float>(dev), out.data_ptr<float>(),
                         cur_stream()));
}

void scale_bf16_dev_(const at::Tensor& x, const at::Tensor& s_dev) {
  GPU(x); BF16(x); F32(s_dev);
  CK(x.is_contiguous() && x.numel() % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) == 0 && s_dev.numel() == 1,
     "scale_bf16_dev: contiguous, 16-B aligned, numel % 8 == 0; s_dev [1]");
  at::DeviceGuard g(x.device());
  HIP_OK(scale_bf16_dev(x.data_ptr(), x.numel(), s_dev.data_ptr<float>(), cur_stream()));
}

// ---------------------------------------------------------------- elementwise
void cast_f32_bf16_(const at::Tensor& x, const at::Tensor& y) {
  GPU(x); F32(x); BF16(y);
  CK(x.numel() == y.numel(), "cast: sizes");
  at::DeviceGuard g(x.device());
  HIP_OK(cast_f32_bf16(x.data_ptr<float>(), y.data_ptr(), x.numel(), cur_stream()));
}
void cast_bf16_f32_(const at::Tensor& x, const at::Tensor& y) {
  GPU(x); BF16(x); F32(y);
  CK(x.numel() == y.numel(), "cast: sizes");
  at::DeviceGuard g(x.device());
  HIP_OK(cast_bf16_f32(x.data_ptr(), y.data_ptr<float>(), x.numel(), cur_stream()));
}
void sum_rows_bf16_(const at::Tensor& x, const at::Tensor& y) {
  GPU(x); BF16(x); BF16(y);
  CK(x.dim() == 2 && x.is_contiguous() && y.is_contiguous() && y.numel() == x.size(1), "sum_rows_bf16: x [R, n], y [n]");
  CK(x.size(1) % 8 == 0 && (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16) == 0 &&
         (reinterpret_cast<uintptr_t>(y.data_ptr()) % 16) == 0, "sum_rows_bf16: n % 8 == 0, 16-B aligned rows");
  at::DeviceGuard g(x.device());
  HIP_OK(sum_rows_bf16(x.data_ptr(), y.data_ptr(), (int)x.size(0), x.size(1), cur_stream()));
}
void relu_bwd_(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& dx) {
  GPU(dy); BF16(dy); BF16(y); BF16(dx);
  CK(dy.numel() == y.numel() && dx.numel() == y.numel(), "relu_bwd: sizes");
  at::DeviceGuard g(dy.device());
  HIP_OK(relu_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel(), cur_stream()));
}
void add_bf16_(const at::Tensor& a, const at::Tensor& b, const at::Tensor& y) {
  GPU(a); BF16(a); BF16(b); BF16(y);
  CK(a.numel() == b.numel() && y.numel() == a.numel(), "add: sizes");
  at::DeviceGuard g(a.device());
  HIP_OK(add_bf16(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), cur_stream()));
}
void transpose_bf16_(const at::Tensor& x, const at::Tensor& y) {
  GPU(x); BF16(y);
  CK(x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "transpose: x must be 2-D bf16, unit column stride");
  CK(y.dim() == 2 && y.size(0) == x.size(1) && y.size(1) == x.size(0), "transpose: y must be [C][R]");
  CK(x.size(0) % 8 == 0 && x.size(1) % 8 == 0 && x.stride(0) % 8 == 0, "transpose: R, C, ld must be multiples of 8");
  at::DeviceGuard g(x.device());
  HIP_OK(transpose_bf16(x.data_ptr(), y.data_ptr(), (int)x.size(0), (int)x.size(1), x.stride(0), cur_stream()));
}
// relu_y / relu_dx: fused ReLU backward (relu_dx = dy * (relu_y > 0), and db sums relu_dx); N % 8 == 0 only
void bias_grad_(const at::Tensor& dy, const at::Tensor& db, int64_t N, bool accumulate, c10::optional<at::Tensor> relu_y,
                c10::optional<at::Tensor> relu_dx, int64_t zcount, int64_t zdb) {
  GPU(dy); BF16(dy); F32(db);
  CK(zcount >= 1 && dy.numel() % (N * zcount) == 0 && db.numel() >= (zcount - 1) * zdb + N, "bias_grad: shapes");
  // the kernels read dy as a dense [M][N] array (row stride N, 16-B vectors): no strided views
  CK(dy.is_contiguous() && db.is_contiguous(), "bias_grad: dy and db must be contiguous");
  CK(relu_y.has_value() == relu_dx.has_value(), "bias_grad: relu_y and relu_dx together");
  if (relu_y) {
    BF16(*relu_y); BF16(*relu_dx);
    CK(N % 8 == 0 && relu_y->is_contiguous() && relu_dx->is_contiguous() && relu_y->numel() == dy.numel() &&
           relu_dx->numel() == dy.numel(), "bias_grad: fused ReLU needs N % 8 == 0 and dense y / dx like dy");
  }
  at::DeviceGuard g(dy.device());
  const long M = dy.numel() / N / zcount;
  at::Tensor ws;  // deterministic mode: partial rows from the caching allocator (stream-ordered)
  if (deterministic() && zcount == 1) ws = at::empty({(int64_t)bias_grad_rows(M) * N}, dy.options().dtype(at::kFloat));
  HIP_OK(bias_grad(dy.data_ptr(), db.data_ptr<float>(), M, (int)N, accumulate ? 1 : 0, cur_stream(),
                   ws.defined() ? ws.data_ptr<float>() : nullptr, relu_y ? relu_y->data_ptr() : nullptr,
                   relu_dx ? relu_dx->data_ptr() : nullptr, (int)zcount, (long)zdb));
}
// zero several contiguous device buffers (4-B multiples, 16-B aligned, one device) in one launch
void zero_ranges_(const std::vector<at::Tensor>& ts) {
  ZeroRanges r{};
  TORCH_CHECK(ts.size() <= (size_t)kMaxZeroRanges, "zero_ranges: at most ", kMaxZeroRanges, " buffers");
  for (const auto& t : ts) {
    GPU(t);
    TORCH_CHECK(t.is_contiguous() && t.device() == ts[0].device(), "zero_ranges: contiguous buffers on one device");
    const long bytes = (long)t.numel() * (long)t.element_size();
    if (bytes == 0) continue;
    TORCH_CHECK(bytes % 4 == 0 && (uintptr_t)t.data_ptr() % 16 == 0, "zero_ranges: 16-B aligned, 4-B multiple buffers");
    const int k = r.count++;
    r.p[k] = t.data_ptr();
    r.pre[k + 1] = r.pre[k] + bytes / 16;
    r.tail_words[k] = (int)((bytes % 16) / 4);
  }
  if (r.count == 0) return;
  at::DeviceGuard guard(ts[0].device());
  HIP_OK(zero_ranges(r, cur_stream()));
}

// out[i] = src_storage[idx[i]] (0 where idx < 0); idx holds element offsets from src.data_ptr() that the
// caller derived from src's own strides (ops/fused_blocks.py:_s2d_tables), all inside src's storage
void gather_bf16_(const at::Tensor& src, const at::Tensor& idx, const at::Tensor& out, int64_t src_extent) {
  GPU(src);
  GPU(idx);
  GPU(out);
  CK(src.scalar_type() == at::kBFloat16 && out.scalar_type() == at::kBFloat16 && out.is_contiguous(), "gather_bf16: bf16");
  CK(idx.scalar_type() == at::kInt && idx.is_contiguous() && idx.numel() == out.numel(), "gather_bf16: int32 idx per output");
  CK(src_extent >= 0 && (int64_t)src.storage().nbytes() / 2 - src.storage_offset() >= src_extent,
     "gather_bf16: src_extent past src's storage");
  at::DeviceGuard guard(out.device());
  HIP_OK(gather_bf16(src.data_ptr(), idx.data_ptr<int>(), out.data_ptr(), out.numel(), cur_stream()));
}

// dst_storage[idx[i]] += src[i] for idx[i] >= 0 (idx injective: each destination from one source)
void scatter_add_f32_(const at::Tensor& src, const at::Tensor& idx, const at::Tensor& dst, int64_t dst_extent) {
  GPU(src);
  GPU(idx);
  GPU(dst);
  F32(src);
  CK(dst.scalar_type() == at::kFloat, "scatter_add_f32: fp32 destination");
  CK(idx.scalar_type() == at::kInt && idx.is_contiguous() && idx.numel() == src.numel(), "scatter_add_f32: int32 idx per source");
  CK(dst_extent >= 0 && (int64_t)dst.storage().nbytes() / 4 - dst.storage_offset() >= dst_extent,
     "scatter_add_f32: dst_extent past dst's storage");
  at::DeviceGuard guard(dst.device());
  HIP_OK(scatter_add_f32(src.data_ptr<float>(), idx.data_ptr<int>(), dst.data_ptr<float>(), src.numel(), cur_stream()));
}

void pad_cols_bf16_(const at::Tensor& x, const at::Tensor& out) {
  GPU(x); BF16(x); BF16(out);
  CK(x.dim() >= 1 && x.stride(-1) == 1 && out.is_contiguous() && out.dim() == x.dim(), "pad_cols: unit column stride");
  const long K = x.size(-1), Kp = out.size(-1), R = K ? x.numel() / K : 0;
  CK(out.numel() == R * Kp && Kp >= K && Kp % 2 == 0, "pad_cols: out [..., Kp >= K], Kp even");
  // rows of x: every leading dimension must collapse to one row stride
  long ldx = x.dim() >= 2 ? x.stride(-2) : K;
  for (int d = x.dim() - 3; d >= 0; --d) CK(x.stride(d) == x.stride(d + 1) * x.size(d + 1), "pad_cols: x rows must have one stride");
  at::DeviceGuard g(x.device());
  HIP_OK(pad_cols_bf16(x.data_ptr(), ldx, out.data_ptr(), R, (int)K, (int)Kp, cur_stream()));
}
void im2col_(const at::Tensor& x, const at::Tensor& col, int64_t ho, int64_t wo, int64_t sh, int64_t sw,
             std::vector<int> dh, std::vector<int> dw, int64_t kpad) {
  GPU(x); BF16(x); BF16(col);
  CK(x.dim() == 4, "im2col: NHWC input");
  CK(dh.size() == dw.size() && dh.size() <= 64, "im2col: taps");
  const int N = x.size(0);
  CK(col.numel() == (int64_t)N * ho * wo * kpad, "im2col: col size");
  CK(kpad >= (int64_t)dh.size() * x.size(3), "im2col: kpad");
  at::DeviceGuard g(x.device());
  HIP_OK(im2col(x.data_ptr(), col.data_ptr(), N, x.size(1), x.size(2), x.size(3), ho, wo, sh, sw, (int)dh.size(),
                dh.data(), dw.data(), (int)kpad, cur_stream()));
}
void s2d_pad_(const at::Tensor& x, const at::Tensor& y, int64_t pad) {
  GPU(x); BF16(x); BF16(y);
  CK(x.dim() == 4 && x.size(3) <= 4 && y.dim() == 4 && y.size(3) == 16 && y.size(0) == x.size(0), "s2d_pad: shapes");
  CK(2 * y.size(1) >= x.size(1) + 2 * pad && 2 * y.size(2) >= x.size(2) + 2 * pad, "s2d_pad: output too small");
  at::DeviceGuard g(x.device());
  HIP_OK(s2d_pad(x.data_ptr(), y.data_ptr(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                 (int)y.size(1), (int)y.size(2), (int)pad, cur_stream()));
}

void normalize_u8_(const at::Tensor& x, const at::Tensor& y, const at::Tensor& mean, const at::Tensor& invstd,
                   int64_t C, int64_t CP) {
  GPU(x);
  CK(x.scalar_type() == at::kByte && x.is_contiguous(), "normalize_u8: uint8 input");
  BF16(y); F32(mean); F32(invstd);
  CK(x.numel() % C == 0 && y.numel() == x.numel() / C * CP && CP >= C, "normalize_u8: shapes");
  at::DeviceGuard g(x.device());
  HIP_OK(normalize_u8(x.data_ptr<uint8_t>(), y.data_ptr(), x.numel() / C, (int)C, (int)CP, mean.data_ptr<float>(),
                      invstd.data_ptr<float>(), cur_stream()));
}

// ---------------------------------------------------------------- optimizers
#define OPT_CHECK(w, g)                                                        \
  GPU(w); F32(w); F32(g);                                                      \
  CK((w).numel() == (g).numel() && (w).numel() % 4 == 0, "optimizer: flat sizes (multiple of 4)")

void sgd_step_(const at::Tensor& w, const at::Tensor& g, c10::optional<at::Tensor> mom, c10::optional<at::Tensor> w16,
               double lr, double momentum, double dampening, double wd, bool nesterov, double gscale) {
  OPT_CHECK(w, g);
  if (mom) { F32(*mom); CK(mom->numel() == w.numel(), "momentum size"); }
  if (w16) { BF16(*w16); CK(w16->numel() == w.numel(), "w16 size"); }
  CK(momentum == 0.0 || mom.has_value(), "sgd: momentum buffer required");
  at::DeviceGuard gd(w.device());
  HIP_OK(sgd_step(w.data_ptr<float>(), g.data_ptr<float>(), optr<float>(mom), optr<void>(w16), w.numel(), (float)lr,
                  (float)momentum, (float)dampening, (float)wd, nesterov ? 1 : 0, (float)gscale, cur_stream()));
}
void adam_step_(const at::Tensor& w, const at::Tensor& g, const at::Tensor& m, const at::Tensor& v,
                c10::optional<at::Tensor> w16, double lr, double b1, double b2, double eps, double wd, int64_t mode,
                double bc1, double bc2, double gscale, c10::optional<at::Tensor> tstep,
                c10::optional<at::Tensor> tick_ctr) {
  OPT_CHECK(w, g);
  F32(m); F32(v);
  if (tstep) { F32(*tstep); CK(tstep->numel() == 1 && tstep->device() == w.device(), "adam: step counter"); }
  if (mode & 4)
    CK(tstep && tick_ctr && tick_ctr->scalar_type() == at::kInt && tick_ctr->numel() == 1 &&
           tick_ctr->device() == w.device(), "adam: the fused tick needs the step counter and an int32 [1] tick_ctr");
  CK(m.numel() == w.numel() && v.numel() == w.numel(), "adam: state sizes");
  if (w16) { BF16(*w16); CK(w16->numel() == w.numel(), "w16 size"); }
  at::DeviceGuard gd(w.device());
  HIP_OK(adam_step(w.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), optr<void>(w16),
                   w.numel(), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (int)mode, (float)bc1,
                   (float)bc2, (float)gscale, optr<float>(tstep), cur_stream(),
                   tick_ctr ? reinterpret_cast<unsigned*>(tick_ctr->data_ptr<int>()) : nullptr));
}
void commit_delta_(const at::Tensor& W, const at::Tensor& center, const at::Tensor& X, c10::optional<at::Tensor> w16,
                   double scale, bool elastic) {
  GPU(W); F32(W); F32(center); F32(X);
  CK(W.is_contiguous() && center.is_contiguous() && X.is_contiguous() && center.numel() == W.numel() &&
         X.numel() == W.numel() && W.numel() % 4 == 0, "commit_delta: contiguous fp32 of one size (n % 4 == 0)");
  if (w16) { BF16(*w16); CK(w16->numel() == W.numel(), "commit_delta: w16 size"); }
  at::DeviceGuard g(W.device());
  HIP_OK(commit_delta(W.data_ptr<float>(), center.data_ptr<float>(), X.data_ptr<float>(), optr<void>(w16), W.numel(),
                      (float)scale, elastic ? 1 : 0, cur_stream()));
}
void commit_apply_(const std::vector<at::Tensor>& xs, const at::Tensor& center, c10::optional<at::Tensor> W,
                   c10::optional<at::Tensor> w16) {
  GPU(center); F32(center);
  CK(center.is_contiguous() && center.numel() % 4 == 0, "commit_apply: contiguous center, n % 4 == 0");
  CK(!xs.empty() && xs.size() <= (size_t)kMaxCommitPeers, "commit_apply: 1..16 exchange buffers");
  CommitPtrs ptrs{};
  for (size_t j = 0; j < xs.size(); ++j) {
    F32(xs[j]);
    CK(xs[j].is_cuda() && xs[j].is_contiguous() && xs[j].numel() == center.numel(), "commit_apply: exchange buffer size");
    ptrs.p[j] = xs[j].data_ptr<float>();
  }
  if (W) { F32(*W); CK(W->is_contiguous() && W->numel() == center.numel(), "commit_apply: W size"); }
  if (w16) { BF16(*w16); CK(W && w16->numel() == center.numel(), "commit_apply: w16 needs W, same size"); }
  at::DeviceGuard g(center.device());
  HIP_OK(commit_apply(ptrs, (int)xs.size(), center.data_ptr<float>(), W ? W->data_ptr<float>() : nullptr,
                      optr<void>(w16), center.numel(), cur_stream()));
}
// mode 0: full commit on one GPU; 1: partial sum into `sum` (multi-GPU round); 2: apply the all-reduced `sum`
void commit_replicas_(const std::vector<at::Tensor>& ws, const std::vector<c10::optional<at::Tensor>>& w16s,
                      const std::vector<double>& scales, const at::Tensor& center, c10::optional<at::Tensor> sum,
                      bool elastic, int64_t mode) {
  GPU(center); F32(center);
  CK(center.numel() % 4 == 0, "commit_replicas: n % 4 == 0");
  CK(ws.size() <= (size_t)kMaxReplicas && w16s.size() == ws.size() && scales.size() == ws.size(),
     "commit_replicas: up to 16 replicas, one w16 (or None) and one scale each");
  CK(mode >= 0 && mode <= 2 && (mode == 0 || sum), "commit_replicas: mode 0 / 1 / 2 (1 and 2 need sum)");
  ReplicaPtrs rp{};
  for (size_t r = 0; r < ws.size(); ++r) {
    F32(ws[r]);
    CK(ws[r].device() == center.device() && ws[r].numel() == center.numel(), "commit_replicas: replica arena size");
    rp.w[r] = ws[r].data_ptr<float>();
    if (w16s[r]) {
      BF16(*w16s[r]);
      CK(w16s[r]->device() == center.device() && w16s[r]->numel() == center.numel(), "commit_replicas: w16 size");
      rp.w16[r] = w16s[r]->data_ptr();
    }
    rp.scale[r] = (float)scales[r];
  }
  if (sum) { F32(*sum); CK(sum->device() == center.device() && sum->numel() == center.numel(), "commit_replicas: sum"); }
  at::DeviceGuard g(center.device());
  HIP_OK(commit_replicas(rp, (int)ws.size(), center.data_ptr<float>(), optr<float>(sum), center.numel(),
                         elastic ? 1 : 0, (int)mode, cur_stream()));
}
// copies mini-batch (ctr % nbatch[q]) of each resident shard srcs[q] ([nbatch[q] * rows, ...]) into dsts[q];
// nbatch: one count for every copy, or one per copy (ragged replica shards)
void batch_fetch_(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts, const at::Tensor& ctr,
                  py::object nbatch) {
  CK(!srcs.empty() && srcs.size() <= (size_t)kMaxBatchCopies && dsts.size() == srcs.size(), "batch_fetch: 1..",
     kMaxBatchCopies, " copies");
  CK(ctr.is_cuda() && ctr.scalar_type() == at::kInt && ctr.numel() == 1, "batch_fetch: int32 step counter");
  std::vector<int64_t> nbs;
  if (py::isinstance<py::int_>(nbatch)) nbs.assign(srcs.size(), nbatch.cast<int64_t>());
  else nbs = nbatch.cast<std::vector<int64_t>>();
  CK(nbs.size() == srcs.size(), "batch_fetch: one batch count, or one per copy");
  BatchCopy bc{};
  for (size_t q = 0; q < srcs.size(); ++q) {
    const at::Tensor &s = srcs[q], &d = dsts[q];
    CK(s.is_cuda() && d.is_cuda() && s.is_contiguous() && d.is_contiguous() && s.scalar_type() == d.scalar_type() &&
           s.device() == ctr.device() && d.device() == ctr.device(),
       "batch_fetch: contiguous GPU tensors of one dtype on the counter's device");
    CK(nbs[q] >= 1, "batch_fetch: nbatch >= 1");
    const long bytes = (long)d.numel() * (long)d.element_size();
    CK((long)s.numel() * (long)s.element_size() >= bytes * nbs[q], "batch_fetch: shard smaller than nbatch batches");
    bc.src[q] = s.data_ptr();
    bc.dst[q] = d.data_ptr();
    bc.bytes[q] = bytes;
    bc.nbatch[q] = nbs[q];
  }
  at::DeviceGuard g(ctr.device());
  HIP_OK(batch_fetch(bc, (int)srcs.size(), ctr.data_ptr<int>(), cur_stream()));
}
// loss [R] with hist [R, cap] (replica batching: one shared counter) or loss [1] with hist [cap];
// steps (int32 [R]): ragged replicas record only while live; ts (fp32 [R]): their Adam counters tick
void step_record_(const at::Tensor& loss, c10::optional<at::Tensor> hist, const at::Tensor& ctr,
                  c10::optional<at::Tensor> steps, c10::optional<at::Tensor> ts) {
  F32(loss);
  const int64_t R = loss.numel();
  CK(loss.is_cuda() && loss.is_contiguous() && R >= 1 && R <= 64, "step_record: 1..64 fp32 losses on the GPU");
  CK(ctr.is_cuda() && ctr.scalar_type() == at::kInt && ctr.numel() == 1 && ctr.device() == loss.device(),
     "step_record: int32 step counter on the loss device");
  if (hist) {
    F32(*hist);
    CK(hist->device() == loss.device() && hist->is_contiguous() && (R == 1 || (hist->dim() == 2 && hist->size(0) == R)),
       "step_record: history [cap] (or [R, cap] for R losses) on the loss device");
  }
  if (steps) CK(steps->is_cuda() && steps->scalar_type() == at::kInt && steps->numel() == R &&
                    steps->device() == loss.device(), "step_record: int32 steps [R] on the loss device");
  if (ts) { F32(*ts); CK(ts->is_cuda() && ts->numel() == R && ts->device() == loss.device(), "step_record: ts [R]"); }
  at::DeviceGuard g(loss.device());
  HIP_OK(step_record(loss.data_ptr<float>(), optr<float>(hist), hist ? (int)(hist->numel() / R) : 0, ctr.data_ptr<int>(),
                     cur_stream(), (int)R, steps ? steps->data_ptr<int>() : nullptr, optr<float>(ts)));
}
// stacked replica optimizer (replica.hip opt_stack_step): w / g / s1 / s2 fp32 [R, n], w16 bf16 [R, n] or None
void opt_stack_step_(int64_t opt, const at::Tensor& w, const at::Tensor& g, c10::optional<at::Tensor> s1,
                     c10::optional<at::Tensor> s2, c10::optional<at::Tensor> w16, const at::Tensor& ctr,
                     const at::Tensor& steps, c10::optional<at::Tensor> ts, double lr, double mu, double b1, double b2,
                     double eps, double wd, int64_t amode) {
  F32(w); F32(g);
  CK(w.is_cuda() && w.dim() == 2 && w.is_contiguous() && g.sizes() == w.sizes() && g.is_contiguous() &&
         g.device() == w.device(), "opt_stack_step: w, g [R, n] contiguous on one GPU");
  const int64_t R = w.size(0), n = w.size(1);
  for (auto* t : {&s1, &s2}) if (*t) { F32(**t); CK((*t)->sizes() == w.sizes() && (*t)->is_contiguous() &&
                                                       (*t)->device() == w.device(), "opt_stack_step: state [R, n]"); }
  if (w16) CK(w16->scalar_type() == at::kBFloat16 && w16->sizes() == w.sizes() && w16->is_contiguous() &&
                  w16->device() == w.device(), "opt_stack_step: bf16 copy [R, n]");
  CK(ctr.is_cuda() && ctr.scalar_type() == at::kInt && ctr.numel() == 1 && ctr.device() == w.device(),
     "opt_stack_step: int32 step counter");
  CK(steps.is_cuda() && steps.scalar_type() == at::kInt && steps.numel() == R && steps.device() == w.device(),
     "opt_stack_step: int32 steps [R]");
  if (ts) { F32(*ts); CK(ts->numel() == R && ts->device() == w.device(), "opt_stack_step: ts [R]"); }
  at::DeviceGuard dg(w.device());
  HIP_OK(opt_stack_step((int)opt, w.data_ptr<float>(), g.data_ptr<float>(), optr<float>(s1), optr<float>(s2),
                        w16 ? w16->data_ptr() : nullptr, n, (int)R, ctr.data_ptr<int>(), steps.data_ptr<int>(),
                        optr<float>(ts), (float)lr, (float)mu, (float)b1, (float)b2, (float)eps, (float)wd, (int)amode,
                        cur_stream()));
}
void prob_xent_(const at::Tensor& p, c10::optional<at::Tensor> labels, c10::optional<at::Tensor> target,
                const at::Tensor& loss_rows, const at::Tensor& dp, double eps, double scale, int64_t ignore_index) {
  GPU(p); F32(p); F32(loss_rows); F32(dp);
  CK(p.dim() == 2 && dp.sizes() == p.sizes() && loss_rows.numel() == p.size(0), "prob_xent: p [B, K], dp, loss_rows [B]");
  CK((labels.has_value()) != (target.has_value()), "prob_xent: labels OR target");
  if (labels) CK(labels->scalar_type() == at::kLong && labels->is_contiguous() && labels->numel() == p.size(0),
                 "prob_xent: int64 labels [B]");
  if (target) { F32(*target); CK(target->sizes() == p.sizes(), "prob_xent: target [B, K]"); }
  at::DeviceGuard g(p.device());
  HIP_OK(prob_xent(p.data_ptr<float>(), labels ? labels->data_ptr<int64_t>() : nullptr, optr<const float>(target),
                   loss_rows.data_ptr<float>(), dp.data_ptr<float>(), (int)p.size(0), (int)p.size(1), (float)eps,
                   (float)scale, (int)ignore_index, cur_stream()));
}
void slab_reduce_(const at::Tensor& ws, int64_t splits, const at::Tensor& c, int64_t M, int64_t N, int64_t ldc,
                  double beta) {
  GPU(ws); F32(ws); GPU(c);
  CK(c.scalar_type() == at::kFloat, "slab_reduce: fp32 c");
  CK(splits >= 1 && ws.numel() >= splits * M * N && ldc >= N && c.numel() >= (M - 1) * ldc + N,
     "slab_reduce: ws [splits, M, N], c [M, ldc]");
  at::DeviceGuard g(ws.device());
  HIP_OK(slab_reduce(ws.data_ptr<float>(), (int)splits, c.data_ptr<float>(), M, (int)N, ldc, (float)beta, cur_stream()));
}
void mse_fwd_bwd_(const at::Tensor& pred, const at::Tensor& target, const at::Tensor& loss, const at::Tensor& grad) {
  F32(pred); F32(target); F32(loss); F32(grad);
  CK(pred.is_cuda() && pred.numel() == target.numel() && grad.numel() == pred.numel() && loss.numel() == 1,
     "mse: pred / target / grad sizes");
  at::DeviceGuard gd(pred.device());
  HIP_OK(mse_fwd_bwd(pred.data_ptr<float>(), target.data_ptr<float>(), pred.numel(), loss.data_ptr<float>(),
                     grad.data_ptr<float>(), cur_stream()));
}
void etl_minmax_(const at::Tensor& x, const at::Tensor& y, double o_min, double scale, double n_min) {
  CK(x.is_cuda() && x.scalar_type() == at::kDouble && y.scalar_type() == at::kDouble && x.is_contiguous() &&
         y.is_contiguous() && x.numel() == y.numel(), "etl_minmax: contiguous fp64 x / y of equal size");
  at::DeviceGuard gd(x.device());
  HIP_OK(etl_minmax(x.data_ptr<double>(), y.data_ptr<double>(), x.numel(), o_min, scale, n_min, cur_stream()));
}
void etl_one_hot_(const at::Tensor& labels, const at::Tensor& y, const at::Tensor& bad) {
  CK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous(), "etl_one_hot: int64 labels");
  CK(y.scalar_type() == at::kDouble && y.dim() == 2 && y.size(0) == labels.numel() && y.is_contiguous(),
     "etl_one_hot: y [n, K] fp64");
  CK(bad.scalar_type() == at::kInt && bad.numel() == 1, "etl_one_hot: int32 flag");
  at::DeviceGuard gd(y.device());
  HIP_OK(etl_one_hot(labels.data_ptr<int64_t>(), y.data_ptr<double>(), labels.numel(), (int)y.size(1),
                     bad.data_ptr<int>(), cur_stream()));
}
void etl_argmax_(const at::Tensor& x, const at::Tensor& out) {
  CK(x.is_cuda() && x.scalar_type() == at::kDouble && x.dim() == 2 && x.stride(1) == 1, "etl_argmax: x [rows, K] fp64");
  CK(out.scalar_type() == at::kLong && out.numel() == x.size(0), "etl_argmax: out int64 [rows]");
  at::DeviceGuard gd(x.device());
  HIP_OK(etl_argmax(x.data_ptr<double>(), x.size(0), (int)x.size(1), x.stride(0), out.data_ptr<int64_t>(),
                    cur_stream()));
}
void step_tick_(const at::Tensor& t) {
  F32(t);
  CK(t.is_cuda() && t.numel() == 1, "step counter: one fp32 element on the GPU");
  at::DeviceGuard gd(t.device());
  HIP_OK(step_tick(t.data_ptr<float>(), cur_stream()));
}
void adagrad_step_(const at::Tensor& w, const at::Tensor& g, const at::Tensor& acc, c10::optional<at::Tensor> w16,
                   double lr, double eps, double wd, double gscale) {
  OPT_CHECK(w, g);
  F32(acc);
  CK(acc.numel() == w.numel(), "adagrad: state size");
  if (w16) BF16(*w16);
  at::DeviceGuard gd(w.device());
  HIP_OK(adagrad_step(w.data_ptr<float>(), g.data_ptr<float>(), acc.data_ptr<float>(), optr<void>(w16), w.numel(),
                      (float)lr, (float)eps, (float)wd, (float)gscale, cur_stream()));
}
void rmsprop_step_(const at::Tensor& w, const at::Tensor& g, const at::Tensor& acc, c10::optional<at::Tensor> w16,
                   double lr, double rho, double eps, double wd, double gscale) {
  OPT_CHECK(w, g);
  F32(acc);
  CK(acc.numel() == w.numel(), "rmsprop: state size");
  if (w16) BF16(*w16);
  at::DeviceGuard gd(w.device());
  HIP_OK(rmsprop_step(w.data_ptr<float>(), g.data_ptr<float>(), acc.data_ptr<float>(), optr<void>(w16), w.numel(),
                      (float)lr, (float)rho, (float)eps, (float)wd, (float)gscale, cur_stream()));
}
void sumsq_(const at::Tensor& x, const at::Tensor& out) {
  GPU(x); F32(x); F32(out);
  CK(x.numel() % 4 == 0, "sumsq: multiple of 4");
  at::DeviceGuard gd(x.device());
  HIP_OK(sumsq_f32(x.data_ptr<float>(), x.numel(), out.data_ptr<float>(), cur_stream()));
}

}  // namespace

void register_ops(py::module& m) {
  m.attr("BN_SHARDS") = (int)kBnShards;
  m.def("bn_stats", &bn_stats_);
  m.def("splitk_finalize", &splitk_finalize_, py::arg("ws"), py::arg("y"), py::arg("C"), py::arg("bias"), py::arg("relu"),
        py::arg("stats"), py::arg("splits") = 0, py::arg("brows") = 0, py::arg("zbias") = 0);
  m.def("bn_partial_rows", &bn_partial_rows_);
  m.def("bn_finalize", &bn_finalize_);
  m.def("bn_apply", &bn_apply_, py::arg("x"), py::arg("scale"), py::arg("shift"), py::arg("resid"), py::arg("y"),
        py::arg("C"), py::arg("relu"), py::arg("mask") = py::none(), py::arg("res_scale") = py::none(),
        py::arg("res_shift") = py::none());
  m.def("bn_bwd_reduce", &bn_bwd_reduce_);
  m.def("bn_bwd_finalize", &bn_bwd_finalize_);
  m.def("bn_bwd_dx", &bn_bwd_dx_);
  m.def("bn_bwd_dx_red", &bn_bwd_dx_red_);
  m.def("pool3s2_bn_bwd", &pool3s2_bn_bwd_, py::arg("dy"), py::arg("am"), py::arg("x"), py::arg("scale"),
        py::arg("shift"), py::arg("mean"), py::arg("coef_or_ws"), py::arg("dx"), py::arg("k") = 3);
  m.def("pool3s2_bn_bwd_ok", [](int64_t N, int64_t H, int64_t W, int64_t C, int64_t Ho, int64_t Wo, int64_t k) {
    return pool3s2_bn_bwd_ok((int)N, (int)H, (int)W, (int)C, (int)Ho, (int)Wo, (int)k);
  });
  m.def("maxpool_fwd", &maxpool_fwd_, "NHWC max pool (byte argmax); optional fused BN affine + ReLU on load",
        py::arg("x"), py::arg("y"), py::arg("am"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"),
        py::arg("ph"), py::arg("pw"), py::arg("scale") = py::none(), py::arg("shift") = py::none());
  m.def("maxpool_bwd", &maxpool_bwd_);
  m.def("avgpool_fwd", &avgpool_fwd_);
  m.def("avgpool_bwd", &avgpool_bwd_);
  m.def("softmax_xent", &softmax_xent_, "fused softmax cross-entropy", py::arg("logits"), py::arg("labels"),
        py::arg("probs"), py::arg("loss_rows"), py::arg("dlogits"), py::arg("grad_scale"), py::arg("smoothing"),
        py::arg("ignore_index"), py::arg("grad_scale_dev") = py::none(), py::arg("loss_out") = py::none(),
        py::arg("out_scale") = 1.0, py::arg("zrows") = 0);
  m.def("label_count_inv", &label_count_inv_);
  m.def("rows_sum_scaled", &rows_sum_scaled_);
  m.def("pad_cols_bf16", &pad_cols_bf16_, "zero-padded copy of a row-strided bf16 view");
  m.def("zero_ranges", &zero_ranges_, "zero up to 8 contiguous device buffers in one launch", py::arg("buffers"));
  m.def("gather_bf16", &gather_bf16_, "out[i] = src[idx[i]] (0 where idx < 0)", py::arg("src"), py::arg("idx"),
        py::arg("out"), py::arg("src_extent"));
  m.def("scatter_add_f32", &scatter_add_f32_, "dst[idx[i]] += src[i] (idx injective, < 0 skipped)", py::arg("src"),
        py::arg("idx"), py::arg("dst"), py::arg("dst_extent"));
  m.def("scale_bf16_dev", &scale_bf16_dev_);
  m.def("cast_f32_bf16", &cast_f32_bf16_);
  m.def("sum_rows_bf16", &sum_rows_bf16_);
  m.def("cast_bf16_f32", &cast_bf16_f32_);
  m.def("relu_bwd", &relu_bwd_);
  m.def("add_bf16", &add_bf16_);
  m.def("bias_grad", &bias_grad_, py::arg("dy"), py::arg("db"), py::arg("N"), py::arg("accumulate"),
        py::arg("relu_y") = py::none(), py::arg("relu_dx") = py::none(), py::arg("zcount") = 1, py::arg("zdb") = 0);
  m.def("transpose_bf16", &transpose_bf16_);
  m.def("im2col", &im2col_);
  m.def("normalize_u8", &normalize_u8_);
  m.def("s2d_pad", &s2d_pad_);
  m.def("sgd_step", &sgd_step_);
  m.def("adam_step", &adam_step_, "fused Adam/AdamW", py::arg("w"), py::arg("g"), py::arg("m"), py::arg("v"),
        py::arg("w16"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("mode"),
        py::arg("bc1"), py::arg("bc2"), py::arg("gscale"), py::arg("tstep") = py::none(),
        py::arg("tick_ctr") = py::none());
  m.def("step_tick", &step_tick_);
  m.def("mse_fwd_bwd", &mse_fwd_bwd_);
  m.def("prob_xent", &prob_xent_);
  m.def("slab_reduce", &slab_reduce_);
  m.def("commit_delta", &commit_delta_);
  m.def("commit_apply", &commit_apply_);
  m.def("commit_replicas", &commit_replicas_, "one commit round over R co-located replicas", py::arg("ws"),
        py::arg("w16s"), py::arg("scales"), py::arg("center"), py::arg("sum") = py::none(), py::arg("elastic") = false,
        py::arg("mode") = 0);
  m.def("batch_fetch", &batch_fetch_);
  m.def("step_record", &step_record_, py::arg("loss"), py::arg("hist"), py::arg("ctr"), py::arg("steps") = py::none(),
        py::arg("ts") = py::none());
  m.def("opt_stack_step", &opt_stack_step_);
  m.def("etl_minmax", &etl_minmax_);
  m.def("etl_one_hot", &etl_one_hot_);
  m.def("etl_argmax", &etl_argmax_);
  m.def("adagrad_step", &adagrad_step_);
  m.def("rmsprop_step", &rmsprop_step_);
  m.def("sumsq", &sumsq_);
}
