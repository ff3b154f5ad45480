// pybind11 registrations of the transformer kernels (attention, LayerNorm, embeddings).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include <algorithm>
#include <cmath>

#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CK(cond, ...) TORCH_CHECK(cond, __VA_ARGS__)
#define GPU(x) CK((x).is_cuda(), #x " must be a GPU tensor")
#define BF16(x) CK((x).scalar_type() == at::kBFloat16 && (x).is_contiguous(), #x " must be contiguous bf16")
#define F32(x) CK((x).scalar_type() == at::kFloat && (x).is_contiguous(), #x " must be contiguous fp32")
#define I64(x) CK((x).scalar_type() == at::kLong && (x).is_contiguous(), #x " must be contiguous int64")
#define HIP_OK(expr)                                                          \
  do {                                                                        \
    int _e = (expr);                                                          \
    CK(_e == 0, "HIP launch failed: ", hipGetErrorString((hipError_t)_e)); \
  } while (0)

template <class T>
T* optr(const c10::optional<at::Tensor>& t) {
  return t ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}


// qkv: [B*S, ld] bf16 (row stride ld, 2-D view allowed), heads of 64
AttnParams make_params(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t q_off, int64_t k_off,
                       int64_t v_off, const at::Tensor& o, const at::Tensor& lse, c10::optional<at::Tensor> lens,
                       double scale, double drop_p, int64_t seed) {
  GPU(qkv);
  CK(qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 2 && qkv.stride(1) == 1, "attn: qkv [tokens, ld] bf16");
  CK(qkv.size(0) == B * S, "attn: qkv rows must be B*S");
  CK(S % 128 == 0, "attn: sequence length must be a multiple of 128, got ", S);
  const int64_t ld = qkv.stride(0);
  CK(ld % 8 == 0 && q_off % 8 == 0 && k_off % 8 == 0 && v_off % 8 == 0, "attn: 16-B aligned rows/offsets");
  CK(std::max({q_off, k_off, v_off}) + H * 64 <= qkv.size(1), "attn: head columns exceed qkv width");
  CK(((uintptr_t)qkv.data_ptr() % 16) == 0, "attn: qkv 16-B aligned");
  CK(o.scalar_type() == at::kBFloat16 && o.dim() == 2 && o.stride(1) == 1 && o.size(0) == B * S &&
         o.size(1) >= H * 64 && o.stride(0) % 8 == 0,
     "attn: o [tokens, >=H*64] bf16");
  F32(lse);
  CK(lse.numel() == B * H * S, "attn: lse [B,H,S]");
  if (lens) {
    CK(lens->scalar_type() == at::kInt && lens->is_contiguous() && lens->numel() == B, "attn: lens int32 [B]");
  }
  CK(drop_p >= 0 && drop_p < 1, "attn: dropout p in [0,1)");
  AttnParams p{};
  p.qkv = reinterpret_cast<const uint16_t*>(qkv.data_ptr());
  p.ld = ld;
  p.q_off = (int)q_off;
  p.k_off = (int)k_off;
  p.v_off = (int)v_off;
  p.o = reinterpret_cast<uint16_t*>(o.data_ptr());
  p.ldo = o.stride(0);
  p.lse = lse.data_ptr<float>();
  p.lens = optr<const int>(lens);
  p.B = (int)B;
  p.H = (int)H;
  p.S = (int)S;
  p.scale = (float)scale;
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  // attention dropout rate quantised to 1/256 (ops/transformer.py attn_drop_t8); the kept
  // probabilities are scaled by the inverse of the quantised keep rate
  p.drop_t8 = drop_t8(drop_p);
  p.drop_scale = drop_scale8(p.drop_t8);
  p.drop_seed = (unsigned long long)seed;
  return p;
}

void attn_fwd_(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t q_off, int64_t k_off, int64_t v_off,
               const at::Tensor& o, const at::Tensor& lse, c10::optional<at::Tensor> lens, double scale, double drop_p,
               int64_t seed) {
  AttnParams p = make_params(qkv, B, S, H, q_off, k_off, v_off, o, lse, lens, scale, drop_p, seed);
  at::DeviceGuard g(qkv.device());
  HIP_OK(attn_fwd(p, cur_stream()));
}

void attn_bwd_(const at::Tensor& qkv, int64_t B, int64_t S, int64_t H, int64_t q_off, int64_t k_off, int64_t v_off,
               const at::Tensor& o, const at::Tensor& lse, c10::optional<at::Tensor> lens, double scale, double drop_p,
               int64_t seed, const at::Tensor& dout, const at::Tensor& dvec, const at::Tensor& dqkv) {
  AttnParams p = make_params(qkv, B, S, H, q_off, k_off, v_off, o, lse, lens, scale, drop_p, seed);
  CK(dout.scalar_type() == at::kBFloat16 && dout.dim() == 2 && dout.stride(1) == 1 && dout.size(0) == B * S &&
         dout.stride(0) % 8 == 0,
     "attn_bwd: dout [tokens, ld] bf16");
  F32(dvec);
  CK(dvec.numel() == B * H * S, "attn_bwd: dvec [B,H,S]");
  CK(dqkv.scalar_type() == at::kBFloat16 && dqkv.dim() == 2 && dqkv.stride(1) == 1 && dqkv.size(0) == B * S &&
         dqkv.size(1) >= std::max({q_off, k_off, v_off}) + H * 64,
     "attn_bwd: dqkv [tokens, >= qkv width] bf16");
  p.dout = reinterpret_cast<const uint16_t*>(dout.data_ptr());
  p.lddo = dout.stride(0);
  p.dvec = dvec.data_ptr<float>();
  p.dqkv = reinterpret_cast<uint16_t*>(dqkv.data_ptr());
  p.lddqkv = dqkv.stride(0);
  at::DeviceGuard g(qkv.device());
  HIP_OK(attn_bwd(p, cur_stream()));
}

void layernorm_fwd_(const at::Tensor& x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                    const at::Tensor& y, const at::Tensor& mean, const at::Tensor& rstd, double eps, double drop_p,
                    int64_t seed) {
  GPU(x); BF16(x); BF16(y); F32(mean); F32(rstd);
  const int64_t H = x.size(-1), M = x.numel() / H;
  CK(H % 8 == 0 && H <= 4096, "layernorm: H % 8 == 0 and H <= 4096");
  CK(y.numel() == x.numel() && mean.numel() == M && rstd.numel() == M, "layernorm: shapes");
  if (gamma) { F32(*gamma); CK(gamma->numel() == H && (uintptr_t)gamma->data_ptr() % 16 == 0, "gamma [H], 16-B aligned"); }
  if (beta) { F32(*beta); CK(beta->numel() == H && (uintptr_t)beta->data_ptr() % 16 == 0, "beta [H], 16-B aligned"); }
  at::DeviceGuard g(x.device());
  HIP_OK(layernorm_fwd(x.data_ptr(), optr<const float>(gamma), optr<const float>(beta), y.data_ptr(),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(), M, (int)H, (float)eps, (float)drop_p,
                       (unsigned long long)seed, cur_stream()));
}

int64_t ln_partial_rows_(int64_t M) { return ln_partial_rows(M); }
int64_t ln_bwd_rows_(int64_t M, int64_t H) { return ln_bwd_rows(M, (int)H); }

void layernorm_bwd_(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& mean, const at::Tensor& rstd,
                    c10::optional<at::Tensor> gamma, const at::Tensor& dx, c10::optional<at::Tensor> dx_drop,
                    double drop_p, int64_t seed, c10::optional<at::Tensor> ws, double in_drop_p, int64_t in_seed,
                    int64_t parts) {
  GPU(dy); BF16(dy); BF16(x); BF16(dx); F32(mean); F32(rstd);
  const int64_t H = x.size(-1), M = x.numel() / H;
  CK(H % 8 == 0 && H <= 4096, "layernorm_bwd: H % 8 == 0 and H <= 4096");
  CK(dy.numel() == x.numel() && dx.numel() == x.numel() && mean.numel() == M && rstd.numel() == M, "shapes");
  if (gamma) { F32(*gamma); CK(gamma->numel() == H && (uintptr_t)gamma->data_ptr() % 16 == 0, "gamma [H], 16-B aligned"); }
  if (dx_drop) { BF16(*dx_drop); CK(dx_drop->numel() == x.numel(), "dx_drop shape"); }
  const int P = ln_bwd_rows(M, (int)H);
  CK(parts == 2 || parts == 3, "layernorm_bwd: parts must be 2 or 3");
  if (ws) { F32(*ws); CK(ws->numel() >= (int64_t)P * parts * H, "layernorm_bwd: ws must hold [P][parts][H]"); }
  at::DeviceGuard g(x.device());
  HIP_OK(layernorm_bwd(dy.data_ptr(), x.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       optr<const float>(gamma), dx.data_ptr(), optr<void>(dx_drop), dx_drop ? (float)drop_p : 0.f,
                       (unsigned long long)seed, optr<float>(ws), P, M, (int)H, (float)in_drop_p,
                       (unsigned long long)in_seed, (int)parts, cur_stream()));
}

void embed_word_grad_(const at::Tensor& sorted_ids, const at::Tensor& perm, const at::Tensor& ds,
                      const at::Tensor& gword) {
  GPU(ds); I64(sorted_ids); I64(perm); BF16(ds); F32(gword);
  const int64_t T = sorted_ids.numel(), H = ds.size(-1);
  CK(perm.numel() == T && ds.numel() == T * H && gword.size(-1) == H && H % 8 == 0, "embed_word_grad: shapes");
  at::DeviceGuard g(ds.device());
  HIP_OK(embed_word_grad(sorted_ids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), ds.data_ptr(),
                         gword.data_ptr<float>(), T, (int)H, cur_stream()));
}

// deterministic word-embedding gradient from a STABLE sort of the ids (DDL_DETERMINISTIC=1)
void embed_word_grad_det_(const at::Tensor& sorted_ids, const at::Tensor& perm, const at::Tensor& ds,
                          const at::Tensor& gword) {
  GPU(ds); I64(sorted_ids); I64(perm); BF16(ds); F32(gword);
  const int64_t T = sorted_ids.numel(), H = ds.size(-1);
  CK(perm.numel() == T && ds.numel() == T * H && gword.dim() == 2 && gword.size(1) == H && H % 8 == 0,
     "embed_word_grad_det: sorted_ids / perm [T], ds [T, H], gword [V, H]");
  at::DeviceGuard g(ds.device());
  at::Tensor part = at::empty({embed_word_grad_det_ws(T, (int)H)}, ds.options().dtype(at::kFloat));
  HIP_OK(embed_word_grad_det(sorted_ids.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), ds.data_ptr(),
                             gword.data_ptr<float>(), T, (int)H, gword.size(0), part.data_ptr<float>(), cur_stream()));
}

void embed_word_grad_atomic_(const at::Tensor& ids, const at::Tensor& ds, const at::Tensor& gword) {
  GPU(ds); I64(ids); BF16(ds); F32(gword);
  const int64_t T = ids.numel(), H = ds.size(-1);
  CK(ids.is_contiguous() && ds.is_contiguous() && gword.is_contiguous() && ds.numel() == T * H &&
         gword.dim() == 2 && gword.size(1) == H && H % 2 == 0, "embed_word_grad_atomic: ids [T], ds [T, H], gword [V, H]");
  at::DeviceGuard g(ds.device());
  HIP_OK(embed_word_grad_atomic(ids.data_ptr<int64_t>(), ds.data_ptr(), gword.data_ptr<float>(), T, (int)H,
                                gword.size(0), cur_stream()));
}

void embed_pos_grad_(const at::Tensor& ds, const at::Tensor& gpos, int64_t B, int64_t S) {
  GPU(ds); BF16(ds); F32(gpos);
  const int64_t H = ds.size(-1);
  CK(ds.numel() == B * S * H && gpos.size(0) >= S && gpos.size(1) == H && H % 2 == 0, "embed_pos_grad: shapes");
  at::DeviceGuard g(ds.device());
  HIP_OK(embed_pos_grad(ds.data_ptr(), gpos.data_ptr<float>(), (int)B, (int)S, (int)H, cur_stream()));
}

void colsum_partials_(const at::Tensor& ws, int64_t P, int64_t N, const at::Tensor& out, bool accumulate,
                      int64_t ld) {
  GPU(ws); F32(ws); F32(out);
  if (ld <= 0) ld = N;
  CK(ld >= N && ws.numel() >= (P - 1) * ld + N && out.numel() >= N, "colsum_partials: sizes");
  at::DeviceGuard g(ws.device());
  HIP_OK(colsum_partials(ws.data_ptr<float>(), (int)P, (int)N, out.data_ptr<float>(), accumulate ? 1 : 0,
                         cur_stream(), (long)ld));
}

void embed_fwd_(const at::Tensor& ids, c10::optional<at::Tensor> types, const at::Tensor& word, const at::Tensor& pos,
                const at::Tensor& type, const at::Tensor& out, int64_t S) {
  GPU(ids); I64(ids); BF16(word); BF16(pos); BF16(type); BF16(out);
  const int64_t H = word.size(1), T = ids.numel();
  CK(H % 8 == 0 && pos.size(1) == H && type.size(1) == H && out.numel() == T * H, "embed_fwd: shapes");
  CK(T % S == 0 && pos.size(0) >= S, "embed_fwd: tokens = B*S and S <= max positions");
  if (types) { I64(*types); CK(types->numel() == T, "types [T]"); }
  at::DeviceGuard g(ids.device());
  HIP_OK(embed_fwd(ids.data_ptr<int64_t>(), optr<const int64_t>(types), word.data_ptr(), pos.data_ptr(),
                   type.data_ptr(), out.data_ptr(), T, (int)S, (int)H, cur_stream()));
}

int64_t embed_partial_rows_(int64_t T) { return ln_partial_rows(T); }

// MLM head rows: out [B*P, H] = rows b*S + pos[b][i] of h [B*S, H]; mlm_scatter_: its backward into dh [B*S, H]
void mlm_gather_(const at::Tensor& h, const at::Tensor& pos, const at::Tensor& out, int64_t S) {
  GPU(h); BF16(h); I64(pos); BF16(out);
  CK(pos.is_cuda() && out.is_cuda() && pos.device() == h.device() && out.device() == h.device(), "mlm_gather: one GPU");
  CK(h.dim() == 2 && pos.dim() == 2 && h.size(0) == pos.size(0) * S && out.size(0) == pos.numel() &&
         out.size(1) == h.size(1) && h.size(1) % 8 == 0 && h.size(1) <= 2048,
     "mlm_gather: h [B*S, H], pos [B, P], out [B*P, H], H % 8 == 0, H <= 2048");
  at::DeviceGuard g(h.device());
  HIP_OK(mlm_gather(h.data_ptr(), pos.data_ptr<int64_t>(), out.data_ptr(), (int)pos.size(0), (int)S, (int)pos.size(1),
                    (int)h.size(1), cur_stream()));
}
void mlm_scatter_(const at::Tensor& dout, const at::Tensor& pos, const at::Tensor& dh, int64_t S) {
  GPU(dout); BF16(dout); I64(pos); BF16(dh);
  CK(pos.is_cuda() && dh.is_cuda() && pos.device() == dout.device() && dh.device() == dout.device(), "mlm_scatter: one GPU");
  CK(dh.dim() == 2 && pos.dim() == 2 && dh.size(0) == pos.size(0) * S && dout.size(0) == pos.numel() &&
         dout.size(1) == dh.size(1) && dh.size(1) % 8 == 0 && dh.size(1) <= 2048,
     "mlm_scatter: dout [B*P, H], pos [B, P], dh [B*S, H], H % 8 == 0, H <= 2048");
  at::DeviceGuard g(dh.device());
  HIP_OK(mlm_scatter(dout.data_ptr(), pos.data_ptr<int64_t>(), dh.data_ptr(), (int)pos.size(0), (int)S,
                     (int)pos.size(1), (int)dh.size(1), cur_stream()));
}

void embed_bwd_(const at::Tensor& ids, c10::optional<at::Tensor> types, const at::Tensor& ds,
                c10::optional<at::Tensor> gword, c10::optional<at::Tensor> gpos, c10::optional<at::Tensor> wsT,
                int64_t ntypes, int64_t S) {
  GPU(ids); I64(ids); BF16(ds);
  const int64_t T = ids.numel(), H = ds.size(-1);
  CK(H % 8 == 0 && H <= 2048 && ds.numel() == T * H, "embed_bwd: H % 8 == 0, H <= 2048");
  CK(ntypes >= 1 && ntypes <= 2, "embed_bwd: 1 or 2 token types");
  if (types) { I64(*types); CK(types->numel() == T, "types [T]"); }
  if (gword) { F32(*gword); CK(gword->size(-1) == H, "gword [V][H]"); }
  if (gpos) { F32(*gpos); CK(gpos->size(-1) == H && gpos->size(0) >= S, "gpos [P][H]"); }
  const int P = ln_partial_rows(T);
  if (wsT) { F32(*wsT); CK(wsT->numel() >= (int64_t)P * ntypes * H, "embed_bwd: wsT [P][ntypes][H]"); }
  at::DeviceGuard g(ids.device());
  HIP_OK(embed_bwd(ids.data_ptr<int64_t>(), optr<const int64_t>(types), ds.data_ptr(), optr<float>(gword),
                   optr<float>(gpos), optr<float>(wsT), P, (int)ntypes, T, (int)S, (int)H, cur_stream()));
}

}  // namespace

void register_transformer(py::module& m) {
  m.def("attn_fwd", &attn_fwd_, py::arg("qkv"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("q_off"),
        py::arg("k_off"), py::arg("v_off"), py::arg("o"), py::arg("lse"), py::arg("lens") = py::none(),
        py::arg("scale") = 0.125, py::arg("drop_p") = 0.0, py::arg("seed") = 0);
  m.def("attn_bwd", &attn_bwd_, py::arg("qkv"), py::arg("B"), py::arg("S"), py::arg("H"), py::arg("q_off"),
        py::arg("k_off"), py::arg("v_off"), py::arg("o"), py::arg("lse"), py::arg("lens"), py::arg("scale"),
        py::arg("drop_p"), py::arg("seed"), py::arg("dout"), py::arg("dvec"), py::arg("dqkv"));
  m.def("layernorm_fwd", &layernorm_fwd_, py::arg("x"), py::arg("gamma"), py::arg("beta"), py::arg("y"),
        py::arg("mean"), py::arg("rstd"), py::arg("eps"), py::arg("drop_p") = 0.0, py::arg("seed") = 0);
  m.def("ln_partial_rows", &ln_partial_rows_);
  m.def("ln_bwd_rows", &ln_bwd_rows_, "partial rows written by layernorm_bwd for M rows of width H");
  m.def("layernorm_bwd", &layernorm_bwd_, py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("rstd"),
        py::arg("gamma"), py::arg("dx"), py::arg("dx_drop"), py::arg("drop_p"), py::arg("seed"), py::arg("ws"),
        py::arg("in_drop_p") = 0.0, py::arg("in_seed") = 0, py::arg("parts") = 2);
  m.def("embed_word_grad", &embed_word_grad_);
  m.def("embed_word_grad_atomic", &embed_word_grad_atomic_);
  m.def("embed_word_grad_det", &embed_word_grad_det_);
  m.def("set_deterministic", [](bool on) { set_deterministic(on ? 1 : 0); });
  m.def("deterministic", []() { return deterministic() != 0; });
  m.def("embed_pos_grad", &embed_pos_grad_);
  m.def("colsum_partials", &colsum_partials_, py::arg("ws"), py::arg("P"), py::arg("N"), py::arg("out"),
        py::arg("accumulate"), py::arg("ld") = 0);
  m.def("embed_fwd", &embed_fwd_);
  m.def("mlm_gather", &mlm_gather_);
  m.def("mlm_scatter", &mlm_scatter_);
  m.def("embed_partial_rows", &embed_partial_rows_);
  m.def("embed_bwd", &embed_bwd_);
}
