// pybind11 registrations of the Keras layer element-wise kernels (kernels/layer_ops.hip) and the
// fp32 MFMA GEMM (kernels/gemm_f32.hip).  Shapes, dtypes and contiguity are validated here.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CK(cond, ...) TORCH_CHECK(cond, __VA_ARGS__)
#define HIP_OK(expr)                                                       \
  do {                                                                     \
    int _e = (expr);                                                       \
    CK(_e == 0, "HIP launch failed: ", hipGetErrorString((hipError_t)_e)); \
  } while (0)

// bf16 or fp32, contiguous, on the GPU; returns 1 for bf16
int float_kind(const at::Tensor& t, const char* what) {
  CK(t.is_cuda() && t.is_contiguous(), what, " must be a contiguous GPU tensor");
  CK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, what, " must be bf16 or fp32");
  return t.scalar_type() == at::kBFloat16 ? 1 : 0;
}
void same(const at::Tensor& a, const at::Tensor& b, const char* what) {
  CK(a.scalar_type() == b.scalar_type() && a.numel() == b.numel(), what, ": dtype / size mismatch");
}

void act_fwd_(const at::Tensor& x, const at::Tensor& y, int64_t code) {
  const int bf = float_kind(x, "act_fwd x");
  float_kind(y, "act_fwd y");
  same(x, y, "act_fwd");
  CK(code >= ACT_C_LINEAR && code <= ACT_C_GELU, "act_fwd: unknown activation code");
  at::DeviceGuard g(x.device());
  HIP_OK(act_fwd(x.data_ptr(), y.data_ptr(), x.numel(), (int)code, bf, cur_stream()));
}

void act_bwd_(const at::Tensor& dy, const at::Tensor& ref, const at::Tensor& dx, int64_t code) {
  const int bf = float_kind(dy, "act_bwd dy");
  float_kind(ref, "act_bwd ref");
  float_kind(dx, "act_bwd dx");
  same(dy, ref, "act_bwd");
  same(dy, dx, "act_bwd");
  at::DeviceGuard g(dy.device());
  HIP_OK(act_bwd(dy.data_ptr(), ref.data_ptr(), dx.data_ptr(), dy.numel(), (int)code, bf, cur_stream()));
}

void softmax_fwd_(const at::Tensor& x, const at::Tensor& y) {
  const int bf = float_kind(x, "softmax x");
  float_kind(y, "softmax y");
  same(x, y, "softmax");
  const int64_t N = x.size(-1);
  at::DeviceGuard g(x.device());
  HIP_OK(softmax_rows_fwd(x.data_ptr(), y.data_ptr(), x.numel() / N, (int)N, bf, cur_stream()));
}

void softmax_bwd_(const at::Tensor& dy, const at::Tensor& y, const at::Tensor& dx) {
  const int bf = float_kind(dy, "softmax_bwd dy");
  float_kind(y, "softmax_bwd y");
  float_kind(dx, "softmax_bwd dx");
  same(dy, y, "softmax_bwd");
  same(dy, dx, "softmax_bwd");
  const int64_t N = y.size(-1);
  at::DeviceGuard g(dy.device());
  HIP_OK(softmax_rows_bwd(dy.data_ptr(), y.data_ptr(), dx.data_ptr(), dy.numel() / N, (int)N, bf, cur_stream()));
}

// dstep (optional fp32 [1] GPU tensor): device step counter mixed into the seed (graph-replayed steps)
void dropout_(const at::Tensor& x, const at::Tensor& y, double p, int64_t seed, c10::optional<at::Tensor> dstep) {
  const int bf = float_kind(x, "dropout x");
  float_kind(y, "dropout y");
  same(x, y, "dropout");
  CK(p >= 0.0 && p < 1.0, "dropout: rate must be in [0, 1)");
  if (dstep) CK(dstep->is_cuda() && dstep->scalar_type() == at::kFloat && dstep->numel() == 1 &&
                    dstep->device() == x.device(), "dropout: dstep must be an fp32 [1] tensor on x's device");
  const uint32_t thresh = drop_t8(p);  // rate quantised to 1/256 (ddl_ops.h)
  at::DeviceGuard g(x.device());
  HIP_OK(dropout_apply(x.data_ptr(), y.data_ptr(), x.numel(), (unsigned long long)seed, thresh, drop_scale8(thresh),
                       bf, cur_stream(), dstep ? dstep->data_ptr<float>() : nullptr));
}

void avgpool2d_fwd_(const at::Tensor& x, const at::Tensor& y, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                    int64_t ph, int64_t pw) {
  const int bf = float_kind(x, "avgpool2d x");
  float_kind(y, "avgpool2d y");
  CK(x.dim() == 4 && y.dim() == 4 && x.size(0) == y.size(0) && x.size(3) == y.size(3), "avgpool2d: NHWC shapes");
  CK(x.scalar_type() == y.scalar_type(), "avgpool2d: dtypes");
  at::DeviceGuard g(x.device());
  HIP_OK(avgpool2d_fwd(x.data_ptr(), y.data_ptr(), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                       (int)y.size(1), (int)y.size(2), (int)kh, (int)kw, (int)sh, (int)sw, (int)ph, (int)pw, bf,
                       cur_stream()));
}

void avgpool2d_bwd_(const at::Tensor& dy, const at::Tensor& dx, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                    int64_t ph, int64_t pw) {
  const int bf = float_kind(dy, "avgpool2d_bwd dy");
  float_kind(dx, "avgpool2d_bwd dx");
  CK(dy.dim() == 4 && dx.dim() == 4 && dx.size(0) == dy.size(0) && dx.size(3) == dy.size(3), "avgpool2d_bwd: shapes");
  CK(dx.scalar_type() == dy.scalar_type(), "avgpool2d_bwd: dtypes");
  at::DeviceGuard g(dy.device());
  HIP_OK(avgpool2d_bwd(dy.data_ptr(), dx.data_ptr(), (int)dx.size(0), (int)dx.size(1), (int)dx.size(2),
                       (int)dx.size(3), (int)dy.size(1), (int)dy.size(2), (int)kh, (int)kw, (int)sh, (int)sw, (int)ph,
                       (int)pw, bf, cur_stream()));
}

void colsum_f32_(const at::Tensor& dy, const at::Tensor& db) {
  CK(dy.is_cuda() && dy.scalar_type() == at::kFloat && dy.is_contiguous(), "colsum_f32: dy contiguous fp32");
  CK(db.is_cuda() && db.scalar_type() == at::kFloat && db.is_contiguous(), "colsum_f32: db contiguous fp32");
  const int64_t N = db.numel();
  CK(N > 0 && dy.numel() % N == 0 && dy.size(-1) == N, "colsum_f32: dy [M][N], db [N]");
  at::DeviceGuard g(dy.device());
  HIP_OK(colsum_f32(dy.data_ptr<float>(), db.data_ptr<float>(), dy.numel() / N, (int)N, cur_stream()));
}

// C[M][N] = alpha * A B + beta * C (+ bias) (relu); A(m,k) = a[m*sam + k*sak], B(k,n) = b[k*sbk + n*sbn]
void gemm_f32_(const at::Tensor& a, int64_t sam, int64_t sak, const at::Tensor& b, int64_t sbk, int64_t sbn,
               const at::Tensor& c, int64_t ldc, int64_t M, int64_t N, int64_t K, double alpha, double beta,
               c10::optional<at::Tensor> bias, bool relu) {
  for (const at::Tensor* t : {&a, &b, &c})
    CK(t->is_cuda() && t->scalar_type() == at::kFloat, "gemm_f32: fp32 GPU tensors");
  CK(c.is_contiguous() || (c.dim() == 2 && c.stride(1) == 1), "gemm_f32: C rows must be dense");
  // the furthest element each operand's index expression reaches must lie inside its storage
  auto reach = [](int64_t r, int64_t sr, int64_t k, int64_t sk) { return (r - 1) * sr + (k - 1) * sk; };
  if (M > 0 && N > 0 && K > 0) {
    CK(reach(M, sam, K, sak) < a.numel(), "gemm_f32: A strides exceed the tensor");
    CK(reach(K, sbk, N, sbn) < b.numel(), "gemm_f32: B strides exceed the tensor");
  }
  if (M > 0 && N > 0) CK((M - 1) * ldc + N <= c.numel(), "gemm_f32: C too small");
  if (bias) CK(bias->is_cuda() && bias->scalar_type() == at::kFloat && bias->numel() >= N, "gemm_f32: bias [N] fp32");
  at::DeviceGuard g(a.device());
  HIP_OK(gemm_f32(a.data_ptr<float>(), sam, sak, b.data_ptr<float>(), sbk, sbn, c.data_ptr<float>(), ldc, (int)M,
                  (int)N, (int)K, (float)alpha, (float)beta, bias ? bias->data_ptr<float>() : nullptr, relu ? 1 : 0,
                  cur_stream()));
}

void transpose_f32_(const at::Tensor& x, const at::Tensor& y) {
  CK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 2, "transpose_f32: x [R][C]");
  CK(y.is_cuda() && y.scalar_type() == at::kFloat && y.is_contiguous() && y.numel() == x.numel(), "transpose_f32: y");
  at::DeviceGuard g(x.device());
  HIP_OK(transpose_f32(x.data_ptr<float>(), y.data_ptr<float>(), (int)x.size(0), (int)x.size(1), cur_stream()));
}

void embedding_fwd_(const at::Tensor& ids, const at::Tensor& table, const at::Tensor& out, const at::Tensor& bad) {
  CK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "embedding: ids contiguous int64");
  const int bf = float_kind(table, "embedding table");
  float_kind(out, "embedding out");
  CK(table.dim() == 2 && out.scalar_type() == table.scalar_type() && out.numel() == ids.numel() * table.size(1),
     "embedding: out [n][D] of the table dtype");
  CK(bad.is_cuda() && bad.scalar_type() == at::kInt && bad.numel() >= 1, "embedding: bad flag int32");
  at::DeviceGuard g(ids.device());
  HIP_OK(embedding_gather(ids.data_ptr<int64_t>(), table.data_ptr(), out.data_ptr(), ids.numel(), (int)table.size(1),
                          table.size(0), bad.data_ptr<int>(), bf, cur_stream()));
}

void embedding_bwd_(const at::Tensor& ids, const at::Tensor& dy, const at::Tensor& gw) {
  CK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "embedding_bwd: ids contiguous int64");
  const int bf = float_kind(dy, "embedding_bwd dy");
  CK(gw.is_cuda() && gw.scalar_type() == at::kFloat && gw.is_contiguous() && gw.dim() == 2, "embedding_bwd: gw fp32");
  CK(dy.numel() == ids.numel() * gw.size(1), "embedding_bwd: dy [n][D]");
  at::DeviceGuard g(ids.device());
  HIP_OK(embedding_scatter(ids.data_ptr<int64_t>(), dy.data_ptr(), gw.data_ptr<float>(), ids.numel(),
                           (int)gw.size(1), gw.size(0), bf, cur_stream()));
}

// out [Ci][nt][Co] = w [Co][T][Ci] gathered at the given taps
// Job table of taps_batch (host uint8 tensor of TapsJob records; the caller keeps it on the device): every
// src [Co][KH][KW][Ci] (or [N][K]) contiguous bf16, dst [Ci][nt][Co] (or [K][N]).  Returns (table, total blocks).
py::tuple taps_batch_table(const std::vector<at::Tensor>& srcs, const std::vector<at::Tensor>& dsts,
                           const std::vector<std::vector<int64_t>>& taps) {
  CK(!srcs.empty() && srcs.size() == dsts.size() && taps.size() == srcs.size(), "taps_batch_table: one dst / taps per src");
  const int64_t n = (int64_t)srcs.size();
  at::Tensor table = at::zeros({n * (int64_t)sizeof(TapsJob)}, at::TensorOptions().dtype(at::kByte));
  TapsJob* jb = reinterpret_cast<TapsJob*>(table.data_ptr());
  int64_t blocks = 0;
  for (int64_t j = 0; j < n; ++j) {
    const at::Tensor &w = srcs[j], &o = dsts[j];
    CK(w.is_cuda() && o.is_cuda() && w.scalar_type() == at::kBFloat16 && o.scalar_type() == at::kBFloat16 &&
           w.is_contiguous() && o.is_contiguous() && (w.dim() == 4 || w.dim() == 2) && o.device() == w.device(),
       "taps_batch_table: contiguous bf16 GPU tensors, src [Co][KH][KW][Ci] or [N][K]");
    const int64_t Co = w.size(0), Ci = w.size(-1), T = w.dim() == 4 ? w.size(1) * w.size(2) : 1;
    const int64_t nt = (int64_t)taps[j].size();
    CK(nt >= 1 && nt <= kMaxFilterTaps && o.numel() == Ci * nt * Co, "taps_batch_table: dst [Ci][nt][Co]");
    jb[j].src = reinterpret_cast<const uint16_t*>(w.data_ptr());
    jb[j].dst = reinterpret_cast<uint16_t*>(o.data_ptr());
    jb[j].Co = (int)Co;
    jb[j].T = (int)T;
    jb[j].Ci = (int)Ci;
    jb[j].nt = (int)nt;
    jb[j].blk0 = (int)blocks;
    for (int64_t i = 0; i < nt; ++i) {
      CK(taps[j][i] >= 0 && taps[j][i] < T, "taps_batch_table: tap out of range");
      jb[j].taps[i] = (int16_t)taps[j][i];
    }
    blocks += taps_job_blocks((int)Co, (int)Ci, (int)nt, (int)T);
    CK(blocks < (int64_t(1) << 31), "taps_batch_table: grid too large");
  }
  return py::make_tuple(table, blocks);
}
void taps_batch_(const at::Tensor& table, int64_t njobs, int64_t blocks) {
  CK(table.is_cuda() && table.scalar_type() == at::kByte && table.numel() == njobs * (int64_t)sizeof(TapsJob),
     "taps_batch: the device copy of taps_batch_table's table");
  at::DeviceGuard g(table.device());
  HIP_OK(taps_batch(reinterpret_cast<const TapsJob*>(table.data_ptr()), (int)njobs, (int)blocks, cur_stream()));
}

// zcount > 1 (replica batching): zcount filters every zw elements from w's storage, outputs [zcount][Ci][nt][Co]
void filter_taps_transpose_(const at::Tensor& w, const at::Tensor& out, std::vector<int64_t> taps, int64_t zcount,
                            int64_t zw) {
  CK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 4,
     "filter_taps_transpose: w [Co][KH][KW][Ci] contiguous bf16");
  const int64_t Co = w.size(0), T = w.size(1) * w.size(2), Ci = w.size(3), nt = (int64_t)taps.size();
  CK(nt >= 1 && nt <= kMaxFilterTaps, "filter_taps_transpose: 1..64 taps");
  CK(out.is_cuda() && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.numel() == zcount * Ci * nt * Co,
     "filter_taps_transpose: out [zcount][Ci][nt][Co] contiguous bf16");
  CK(zcount == 1 || (zw >= Co * T * Ci && w.storage_offset() * 2 + (zcount - 1) * zw * 2 + Co * T * Ci * 2 <=
                                              (int64_t)w.storage().nbytes()),
     "filter_taps_transpose: zcount filters every zw elements must lie inside w's storage");
  FilterTaps ft{};
  for (int64_t i = 0; i < nt; ++i) {
    CK(taps[i] >= 0 && taps[i] < T, "filter_taps_transpose: tap out of range");
    ft.t[i] = (int16_t)taps[i];
  }
  at::DeviceGuard g(w.device());
  HIP_OK(filter_taps_transpose(w.data_ptr(), out.data_ptr(), (int)Co, (int)T, (int)Ci, ft, (int)nt, cur_stream(),
                               (int)zcount, (long)zw, (long)(Ci * nt * Co)));
}

}  // namespace

void register_layer_ops(py::module& m) {
  m.def("act_fwd", &act_fwd_, "y = act(x) (bf16/fp32)");
  m.def("act_bwd", &act_bwd_, "dx = dy * act'(ref), ref = y (x for GELU)");
  m.def("softmax_fwd", &softmax_fwd_, "softmax over the last axis");
  m.def("softmax_bwd", &softmax_bwd_, "softmax backward");
  m.def("dropout", &dropout_, "counter-hash dropout (forward and backward)", py::arg("x"), py::arg("y"), py::arg("p"),
        py::arg("seed"), py::arg("dstep") = py::none());
  m.def("avgpool2d_fwd", &avgpool2d_fwd_, "NHWC average pooling");
  m.def("avgpool2d_bwd", &avgpool2d_bwd_, "NHWC average pooling backward");
  m.def("colsum_f32", &colsum_f32_, "db += column sums of dy (fp32)");
  m.def("gemm_f32", &gemm_f32_, "fp32 MFMA GEMM with element strides", py::arg("a"), py::arg("sam"), py::arg("sak"),
        py::arg("b"), py::arg("sbk"), py::arg("sbn"), py::arg("c"), py::arg("ldc"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("alpha") = 1.0, py::arg("beta") = 0.0, py::arg("bias") = py::none(),
        py::arg("relu") = false);
  m.def("transpose_f32", &transpose_f32_, "y = x^T (fp32)");
  m.def("taps_batch_table", &taps_batch_table);
  m.def("taps_batch", &taps_batch_);
  m.def("filter_taps_transpose", &filter_taps_transpose_, "conv dgrad filter: out[ci][t][co] = w[co][taps[t]][ci]",
        py::arg("w"), py::arg("out"), py::arg("taps"), py::arg("zcount") = 1, py::arg("zw") = 0);
  m.def("embedding_fwd", &embedding_fwd_, "Keras Embedding gather (bf16/fp32 table)");
  m.def("embedding_bwd", &embedding_bwd_, "Keras Embedding gradient scatter-add into fp32");
  m.attr("ACT_CODES") = py::dict(py::arg("linear") = (int)ACT_C_LINEAR, py::arg("relu") = (int)ACT_C_RELU,
                                 py::arg("tanh") = (int)ACT_C_TANH, py::arg("sigmoid") = (int)ACT_C_SIGMOID,
                                 py::arg("hard_sigmoid") = (int)ACT_C_HARD_SIGMOID, py::arg("elu") = (int)ACT_C_ELU,
                                 py::arg("selu") = (int)ACT_C_SELU, py::arg("softplus") = (int)ACT_C_SOFTPLUS,
                                 py::arg("gelu") = (int)ACT_C_GELU);
}
