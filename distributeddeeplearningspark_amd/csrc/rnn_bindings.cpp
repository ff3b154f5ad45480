// pybind11 registrations of the persistent GRU / LSTM kernels (kernels/rnn.hip).  The input
// projection and the parameter-gradient contractions are plain fp32 library GEMMs (ATen);
// the recurrences run in the hand-written kernels.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

int cell_id(const std::string& cell) {
  TORCH_CHECK(cell == "gru" || cell == "lstm", "rnn: cell must be 'gru' or 'lstm'");
  return cell == "gru" ? 0 : 1;
}

py::tuple rnn_fwd_(const std::string& cell, const at::Tensor& x, const at::Tensor& W, const at::Tensor& U,
                   c10::optional<at::Tensor> b, bool rs) {
  const int c = cell_id(cell);
  const int G = c == 0 ? 3 : 4;
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 3, "rnn_fwd: x [B,T,I] fp32 on GPU");
  const int64_t B = x.size(0), T = x.size(1), I = x.size(2), H = U.size(0);
  TORCH_CHECK(W.size(0) == I && W.size(1) == G * H && U.size(1) == G * H, "rnn_fwd: W [I,GH], U [H,GH]");
  TORCH_CHECK(W.scalar_type() == at::kFloat && U.scalar_type() == at::kFloat, "rnn_fwd: fp32 weights");
  at::DeviceGuard g(x.device());
  at::Tensor xc = x.contiguous(), Wc = W.contiguous();
  at::Tensor bc = b ? b->contiguous() : at::Tensor();
  at::Tensor xw;
  if (!rnn_fuses_input((int)H, (int)I)) {  // wide inputs / generic kernels: one projection GEMM first
    xw = at::matmul(xc.reshape({B * T, I}), Wc);
    if (b) xw.add_(bc);
    xw = xw.contiguous();
  }
  auto opt = x.options();
  at::Tensor hs = at::empty({B, T + 1, H}, opt);
  at::Tensor cs = c == 1 ? at::empty({B, T + 1, H}, opt) : at::empty({0}, opt);
  at::Tensor gates = at::empty({B, T, G * H}, opt);
  at::Tensor y = rs ? at::empty({B, T, H}, opt) : at::empty({B, H}, opt);
  at::Tensor Uc = U.contiguous();
  int e = rnn_fwd(c, xw.defined() ? xw.data_ptr<float>() : nullptr, xc.data_ptr<float>(), Wc.data_ptr<float>(),
                  bc.defined() ? bc.data_ptr<float>() : nullptr, (int)I, Uc.data_ptr<float>(), hs.data_ptr<float>(),
                  c == 1 ? cs.data_ptr<float>() : nullptr, gates.data_ptr<float>(), y.data_ptr<float>(), (int)B,
                  (int)T, (int)H, rs ? 1 : 0, cur_stream());
  TORCH_CHECK(e == 0, "rnn_fwd launch failed: ", hipGetErrorString((hipError_t)e));
  py::list saved;
  saved.append(hs);
  saved.append(cs);
  saved.append(gates);
  return py::make_tuple(y, saved);
}

// Returns (dx | None, dW | None, dU | None, db | None).  On the fast path the parameter
// gradients are accumulated into gW / gU / gb (fp32 arena slices) in-kernel and None is
// returned for them; dx is only computed when need_dx.
py::tuple rnn_bwd_(const std::string& cell, const at::Tensor& dy, const at::Tensor& x, const at::Tensor& W,
                   const at::Tensor& U, c10::optional<at::Tensor> b, bool rs, std::vector<at::Tensor> saved,
                   c10::optional<at::Tensor> gW, c10::optional<at::Tensor> gU, c10::optional<at::Tensor> gb,
                   bool need_dx) {
  const int c = cell_id(cell);
  const int G = c == 0 ? 3 : 4;
  const int64_t B = x.size(0), T = x.size(1), I = x.size(2), H = U.size(0);
  TORCH_CHECK(saved.size() == 3, "rnn_bwd: saved = [hs, cs, gates]");
  const at::Tensor& hs = saved[0];
  const at::Tensor& cs = saved[1];
  const at::Tensor& gates = saved[2];
  at::DeviceGuard g(x.device());
  at::Tensor dyc = dy.contiguous();
  at::Tensor Uc = U.contiguous();
  at::Tensor UT = rnn_bwd_uses_ut((int)H) ? U.t().contiguous() : Uc;
  at::Tensor dgates = at::empty({B, T, G * H}, x.options());
  int e = rnn_bwd(c, dyc.data_ptr<float>(), Uc.data_ptr<float>(), UT.data_ptr<float>(), hs.data_ptr<float>(),
                  c == 1 ? cs.data_ptr<float>() : nullptr, gates.data_ptr<float>(), dgates.data_ptr<float>(), (int)B,
                  (int)T, (int)H, rs ? 1 : 0, cur_stream());
  TORCH_CHECK(e == 0, "rnn_bwd launch failed: ", hipGetErrorString((hipError_t)e));
  at::Tensor dg = dgates.view({B * T, G * H});
  at::Tensor xc = x.contiguous();
  py::object dx = py::none();
  if (need_dx) dx = py::cast(at::matmul(dg, W.t()).view({B, T, I}));
  const bool fused = rnn_fast_path((int)H) && gU && gW && (gb.has_value() == b.has_value());
  if (fused) {
    for (const auto* t : {&*gU, &*gW})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "rnn_bwd: fp32 contiguous grad buffers");
    TORCH_CHECK(gU->numel() == H * G * H && gW->numel() == I * G * H, "rnn_bwd: grad buffer sizes");
    if (gb) TORCH_CHECK(gb->scalar_type() == at::kFloat && gb->numel() == G * H, "rnn_bwd: bias grad buffer");
    e = rnn_param_grad(c, dg.data_ptr<float>(), hs.data_ptr<float>(), gates.data_ptr<float>(), xc.data_ptr<float>(),
                       gU->data_ptr<float>(), gW->data_ptr<float>(), gb ? gb->data_ptr<float>() : nullptr, (int)B,
                       (int)T, (int)H, (int)I, cur_stream());
    TORCH_CHECK(e == 0, "rnn_param_grad launch failed: ", hipGetErrorString((hipError_t)e));
    return py::make_tuple(dx, py::none(), py::none(), py::none());
  }
  at::Tensor x2 = xc.reshape({B * T, I});
  at::Tensor dW = at::matmul(x2.t(), dg);
  at::Tensor db = b ? dg.sum(0) : at::Tensor();
  at::Tensor hp = hs.narrow(1, 0, T).reshape({B * T, H});
  at::Tensor dU;
  if (c == 0) {
    dU = at::empty_like(U);
    dU.narrow(1, 0, 2 * H).copy_(at::matmul(hp.t(), dg.narrow(1, 0, 2 * H)));
    at::Tensor rh = gates.view({B * T, G * H}).narrow(1, H, H) * hp;
    dU.narrow(1, 2 * H, H).copy_(at::matmul(rh.t(), dg.narrow(1, 2 * H, H)));
  } else {
    dU = at::matmul(hp.t(), dg);
  }
  return py::make_tuple(dx, dW, dU, db.defined() ? py::cast(db) : py::none());
}

}  // namespace

void register_rnn(py::module& m) {
  m.def("rnn_fwd", &rnn_fwd_, "persistent GRU/LSTM forward (fp32)");
  m.def("rnn_bwd", &rnn_bwd_, "persistent GRU/LSTM backward (fp32)", py::arg("cell"), py::arg("dy"), py::arg("x"),
        py::arg("W"), py::arg("U"), py::arg("b"), py::arg("rs"), py::arg("saved"), py::arg("gW") = py::none(),
        py::arg("gU") = py::none(), py::arg("gb") = py::none(), py::arg("need_dx") = true);
}
