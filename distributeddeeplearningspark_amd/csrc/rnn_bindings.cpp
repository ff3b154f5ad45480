// pybind11 registrations of the persistent GRU / LSTM / SimpleRNN kernels (kernels/rnn.hip).
// The input projection, the input gradient and (off the fused path) the parameter-gradient
// contractions run on the fp32 MFMA GEMM (kernels/gemm_f32.hip); no library GEMM is called.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

int cell_id(const std::string& cell) {
  TORCH_CHECK(cell == "gru" || cell == "lstm" || cell == "rnn", "rnn: cell must be 'gru', 'lstm' or 'rnn'");
  return cell == "gru" ? 0 : (cell == "lstm" ? 1 : 2);
}
int gates_of(int c) { return c == 0 ? 3 : (c == 1 ? 4 : 1); }

// C[M][N] (fp32, row-major ldc) = alpha * A B + beta * C with element strides (gemm_f32)
void f32mm(const at::Tensor& a, long sam, long sak, const at::Tensor& b, long sbk, long sbn, at::Tensor& c, long ldc,
           int64_t M, int64_t N, int64_t K, float beta = 0.f, const float* bias = nullptr) {
  const int e = gemm_f32(a.data_ptr<float>(), sam, sak, b.data_ptr<float>(), sbk, sbn, c.data_ptr<float>(), ldc, (int)M,
                         (int)N, (int)K, 1.f, beta, bias, 0, cur_stream());
  TORCH_CHECK(e == 0, "gemm_f32 launch failed: ", hipGetErrorString((hipError_t)e));
}

py::tuple rnn_fwd_(const std::string& cell, const at::Tensor& x, const at::Tensor& W, const at::Tensor& U,
                   c10::optional<at::Tensor> b, bool rs, int64_t act, int64_t ract) {
  const int c = cell_id(cell);
  const int G = gates_of(c);
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.dim() == 3, "rnn_fwd: x [B,T,I] fp32 on GPU");
  const int64_t B = x.size(0), T = x.size(1), I = x.size(2), H = U.size(0);
  TORCH_CHECK(W.size(0) == I && W.size(1) == G * H && U.size(1) == G * H, "rnn_fwd: W [I,GH], U [H,GH]");
  TORCH_CHECK(W.scalar_type() == at::kFloat && U.scalar_type() == at::kFloat, "rnn_fwd: fp32 weights");
  at::DeviceGuard g(x.device());
  at::Tensor xc = x.contiguous(), Wc = W.contiguous();
  at::Tensor bc = b ? b->contiguous() : at::Tensor();
  at::Tensor xw;
  const bool reg = rnn_reg_path(c, (int)H, (int)act, (int)ract);
  if (!(reg && rnn_fuses_input((int)H, (int)I))) {  // wide inputs / generic kernels: one projection GEMM first
    xw = at::empty({B * T, G * H}, x.options());
    f32mm(xc, I, 1, Wc, G * H, 1, xw, G * H, B * T, G * H, I, 0.f, bc.defined() ? bc.data_ptr<float>() : nullptr);
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
                  (int)T, (int)H, rs ? 1 : 0, (int)act, (int)ract, cur_stream());
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
                   bool need_dx, int64_t act, int64_t ract) {
  const int c = cell_id(cell);
  const int G = gates_of(c);
  const bool reg = rnn_reg_path(c, (int)U.size(0), (int)act, (int)ract);
  const int64_t B = x.size(0), T = x.size(1), I = x.size(2), H = U.size(0);
  TORCH_CHECK(saved.size() == 3, "rnn_bwd: saved = [hs, cs, gates]");
  const at::Tensor& hs = saved[0];
  const at::Tensor& cs = saved[1];
  const at::Tensor& gates = saved[2];
  at::DeviceGuard g(x.device());
  at::Tensor dyc = dy.contiguous();
  at::Tensor Uc = U.contiguous();
  at::Tensor UT = Uc;
  if (!reg) {  // the generic kernels read U^T [GH][H]
    UT = at::empty({G * H, H}, U.options());
    const int et = transpose_f32(Uc.data_ptr<float>(), UT.data_ptr<float>(), (int)H, (int)(G * H), cur_stream());
    TORCH_CHECK(et == 0, "transpose_f32 launch failed");
  }
  at::Tensor dgates = at::empty({B, T, G * H}, x.options());
  int e = rnn_bwd(c, dyc.data_ptr<float>(), Uc.data_ptr<float>(), UT.data_ptr<float>(), hs.data_ptr<float>(),
                  c == 1 ? cs.data_ptr<float>() : nullptr, gates.data_ptr<float>(), dgates.data_ptr<float>(), (int)B,
                  (int)T, (int)H, rs ? 1 : 0, (int)act, (int)ract, cur_stream());
  TORCH_CHECK(e == 0, "rnn_bwd launch failed: ", hipGetErrorString((hipError_t)e));
  at::Tensor dg = dgates.view({B * T, G * H});
  at::Tensor xc = x.contiguous();
  py::object dx = py::none();
  at::Tensor Wc = W.contiguous();
  if (need_dx) {  // dx[bt][i] = sum_j dg[bt][j] W[i][j]
    at::Tensor dxt = at::empty({B * T, I}, x.options());
    f32mm(dg, G * H, 1, Wc, 1, G * H, dxt, I, B * T, I, G * H);
    dx = py::cast(dxt.view({B, T, I}));
  }
  const bool fused = (c != 0 || (2 * H) % 64 == 0) && gU && gW && (gb.has_value() == b.has_value());
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
  // unfused parameter gradients (no arena buffers given, or a GRU whose H does not tile): the
  // same one-launch kernel into fresh zeroed buffers
  at::Tensor dW = at::zeros({I, G * H}, x.options());
  at::Tensor dU = at::zeros({H, G * H}, x.options());
  at::Tensor db = b ? at::zeros({G * H}, x.options()) : at::Tensor();
  if (c != 0 || (2 * H) % 64 == 0) {
    e = rnn_param_grad(c, dg.data_ptr<float>(), hs.data_ptr<float>(), gates.data_ptr<float>(), xc.data_ptr<float>(),
                       dU.data_ptr<float>(), dW.data_ptr<float>(), b ? db.data_ptr<float>() : nullptr, (int)B, (int)T,
                       (int)H, (int)I, cur_stream());
    TORCH_CHECK(e == 0, "rnn_param_grad launch failed: ", hipGetErrorString((hipError_t)e));
  } else {
    // GRU with 2H not a multiple of 64: dU = [h_{t-1}]^T dg for z,r and [r*h_{t-1}]^T dg for h
    at::Tensor hp = hs.narrow(1, 0, T).contiguous().view({B * T, H});
    at::Tensor rh = gates.view({B * T, G * H}).narrow(1, H, H).mul(hp).contiguous();
    f32mm(xc, 1, I, dg, G * H, 1, dW, G * H, I, G * H, B * T);
    f32mm(hp, 1, H, dg, G * H, 1, dU, G * H, H, 2 * H, B * T);
    at::Tensor dUh = dU.narrow(1, 2 * H, H);
    at::Tensor dgh = dg.narrow(1, 2 * H, H);
    const int e2 = gemm_f32(rh.data_ptr<float>(), 1, H, dgh.data_ptr<float>(), G * H, 1, dUh.data_ptr<float>(), G * H,
                            (int)H, (int)H, (int)(B * T), 1.f, 0.f, nullptr, 0, cur_stream());
    TORCH_CHECK(e2 == 0, "gemm_f32 launch failed");
    if (b) {
      const int e3 = colsum_f32(dg.data_ptr<float>(), db.data_ptr<float>(), B * T, (int)(G * H), cur_stream());
      TORCH_CHECK(e3 == 0, "colsum_f32 launch failed");
    }
  }
  return py::make_tuple(dx, dW, dU, db.defined() ? py::cast(db) : py::none());
}

// Replica-batched training step of R co-located RNN(H) -> Dense(K) / MSE replicas (kernels/rnn.hip,
// rnn_replica_step): every list holds one entry per replica; None entries of the optional lists are
// absent biases / optimizer states.  All tensors fp32, contiguous, on one device.
float* fptr(const py::handle& o, const char* what, int64_t numel = -1) {
  if (o.is_none()) return nullptr;
  at::Tensor t = o.cast<at::Tensor>();
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), "rnn_replica_step: ", what,
              " must be a contiguous fp32 GPU tensor");
  TORCH_CHECK(numel < 0 || t.numel() >= numel, "rnn_replica_step: ", what, " too small");
  return t.data_ptr<float>();
}

void rnn_replica_step_(const std::string& cell, py::list xs, py::list ys, py::list Ws, py::list Us, py::list bs,
                       py::list Wds, py::list bds, py::list gWs, py::list gUs, py::list gbs, py::list gWds,
                       py::list gbds, py::list hists, at::Tensor ctr, std::vector<int64_t> nbs,
                       std::vector<int64_t> steps, at::Tensor live, int64_t B, at::Tensor hs,
                       at::Tensor cs, at::Tensor gates, at::Tensor hlast, at::Tensor dh, at::Tensor dgates,
                       py::list ws, py::list gs, py::list s1s, py::list s2s, py::list ts, int64_t opt, double lr,
                       double p1, double p2, double eps, double wd, int64_t amode) {
  const int c = cell_id(cell);
  TORCH_CHECK(c == 0 || c == 1, "rnn_replica_step: GRU or LSTM");
  const int G = gates_of(c);
  const int R = (int)xs.size();
  TORCH_CHECK(R >= 1 && R <= kMaxRnnRep, "rnn_replica_step: 1..", kMaxRnnRep, " replicas");
  for (py::list* l : {&ys, &Ws, &Us, &bs, &Wds, &bds, &gWs, &gUs, &gbs, &gWds, &gbds, &hists, &ws, &gs, &s1s, &s2s, &ts})
    TORCH_CHECK((int)l->size() == R, "rnn_replica_step: one entry per replica in every list");
  at::Tensor x0 = xs[0].cast<at::Tensor>(), U0 = Us[0].cast<at::Tensor>(), Wd0 = Wds[0].cast<at::Tensor>();
  TORCH_CHECK(x0.dim() == 3, "rnn_replica_step: x shards [rows, T, I]");
  const int64_t T = x0.size(1), I = x0.size(2), H = U0.size(0), K = Wd0.size(0);
  TORCH_CHECK(U0.size(1) == G * H && Wd0.size(1) == H, "rnn_replica_step: U [H, GH], Dense kernel [K, H]");
  TORCH_CHECK(rnn_replica_ok(c, (int)H, (int)I, (int)K, (int)B), "rnn_replica_step: unsupported H / I / K / B");
  TORCH_CHECK(ctr.is_cuda() && ctr.scalar_type() == at::kInt && ctr.numel() >= 1, "rnn_replica_step: int32 ctr");
  TORCH_CHECK(live.is_cuda() && live.scalar_type() == at::kInt && live.numel() >= R && live.device() == ctr.device(),
              "rnn_replica_step: int32 live flags [R] on the counter's device");
  TORCH_CHECK((int)nbs.size() == R && (int)steps.size() == R, "rnn_replica_step: batches and steps per replica");
  const int64_t RB = R * B;
  const int64_t n = ws[0].cast<at::Tensor>().numel();
  RnnRep rp{};
  OptRep op{};
  for (int r = 0; r < R; ++r) {
    const int64_t nb = nbs[r];
    TORCH_CHECK(nb >= 1 && steps[r] >= 0 && steps[r] < (1LL << 31), "rnn_replica_step: batches >= 1, steps >= 0");
    rp.nbr[r] = (int)nb;
    rp.steps[r] = (int)steps[r];
    rp.x[r] = fptr(xs[r], "x shard", nb * B * T * I);
    rp.y[r] = fptr(ys[r], "y shard", nb * B * K);
    rp.W[r] = fptr(Ws[r], "W", I * G * H);
    rp.U[r] = fptr(Us[r], "U", H * G * H);
    rp.b[r] = fptr(bs[r], "b", G * H);
    rp.Wd[r] = fptr(Wds[r], "Dense kernel", K * H);
    rp.bd[r] = fptr(bds[r], "Dense bias", K);
    rp.gW[r] = fptr(gWs[r], "gW", I * G * H);
    rp.gU[r] = fptr(gUs[r], "gU", H * G * H);
    rp.gb[r] = fptr(gbs[r], "gb", G * H);
    rp.gWd[r] = fptr(gWds[r], "gWd", K * H);
    rp.gbd[r] = fptr(gbds[r], "gbd", K);
    TORCH_CHECK(!bs[r].is_none() && !gbs[r].is_none(), "rnn_replica_step: recurrent bias required");
    TORCH_CHECK(bds[r].is_none() == gbds[r].is_none(), "rnn_replica_step: Dense bias and its gradient together");
    rp.hist[r] = fptr(hists[r], "history", steps[r]);  // one slot per step the replica takes
    TORCH_CHECK(rp.hist[r], "rnn_replica_step: history required");
    op.w[r] = fptr(ws[r], "weights", n);
    op.g[r] = fptr(gs[r], "grads", n);
    op.s1[r] = fptr(s1s[r], "optimizer state", n);
    op.s2[r] = fptr(s2s[r], "optimizer state 2", n);
    op.t[r] = fptr(ts[r], "step counter", 1);
    TORCH_CHECK(ws[r].cast<at::Tensor>().numel() == n, "rnn_replica_step: equal arena sizes");
    if (opt == 2) TORCH_CHECK(op.s1[r] && op.s2[r] && op.t[r], "rnn_replica_step: Adam needs m, v and t");
    if (opt == 1) TORCH_CHECK(op.s1[r], "rnn_replica_step: Adagrad needs its accumulator");
  }
  rp.ctr = ctr.data_ptr<int>();
  rp.live = live.data_ptr<int>();
  rp.B = (int)B;
  rp.K = (int)K;
  float* hsp = fptr(py::cast(hs), "hs", RB * (T + 1) * H);
  float* csp = c == 1 ? fptr(py::cast(cs), "cs", RB * (T + 1) * H) : nullptr;
  float* gp = fptr(py::cast(gates), "gates", RB * T * G * H);
  float* hl = fptr(py::cast(hlast), "h_last", RB * H);
  float* dhp = fptr(py::cast(dh), "dh", RB * H);
  float* dgp = fptr(py::cast(dgates), "dgates", RB * T * G * H);
  at::DeviceGuard g(x0.device());
  const int e = rnn_replica_step(c, rp, R, (int)T, (int)H, (int)I, hsp, csp, gp, hl, dhp, dgp, op, n, (int)opt,
                                 (float)lr, (float)p1, (float)p2, (float)eps, (float)wd, (int)amode, cur_stream());
  TORCH_CHECK(e == 0, "rnn_replica_step launch failed: ", hipGetErrorString((hipError_t)e));
}

}  // namespace

void register_rnn(py::module& m) {
  m.def("rnn_fwd", &rnn_fwd_, "persistent GRU/LSTM/SimpleRNN forward (fp32)", py::arg("cell"), py::arg("x"),
        py::arg("W"), py::arg("U"), py::arg("b"), py::arg("rs"), py::arg("act") = (int64_t)ACT_C_TANH,
        py::arg("ract") = (int64_t)ACT_C_HARD_SIGMOID);
  m.def("rnn_bwd", &rnn_bwd_, "persistent GRU/LSTM backward (fp32)", py::arg("cell"), py::arg("dy"), py::arg("x"),
        py::arg("W"), py::arg("U"), py::arg("b"), py::arg("rs"), py::arg("saved"), py::arg("gW") = py::none(),
        py::arg("gU") = py::none(), py::arg("gb") = py::none(), py::arg("need_dx") = true,
        py::arg("act") = (int64_t)ACT_C_TANH, py::arg("ract") = (int64_t)ACT_C_HARD_SIGMOID);
  m.def("rnn_replica_step", &rnn_replica_step_, "one training step of R co-located RNN -> Dense / MSE replicas");
  m.def("rnn_replica_ok", [](const std::string& cell, int64_t H, int64_t I, int64_t K, int64_t B) {
    return rnn_replica_ok(cell_id(cell), (int)H, (int)I, (int)K, (int)B);
  });
}
