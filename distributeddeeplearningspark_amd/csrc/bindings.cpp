// Python bindings of the native layer: HIP kernel launchers + host runtime.
// Every launcher validates shapes/dtypes/devices here (host side) before a kernel
// is launched, so a wrong call fails loudly instead of faulting the GPU.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <ATen/DeviceGuard.h>

#include "ddl_gemm.h"
#include "ddl_ops.h"

namespace py = pybind11;
using namespace ddl;

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be fp32")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    int _e = (expr);                                                                   \
    TORCH_CHECK(_e == 0, "HIP launch failed: ", hipGetErrorString((hipError_t)_e)); \
  } while (0)

void fill_geom(ConvGeom& g, const py::dict& d) {
  g.n = d["n"].cast<int>();
  g.hi = d["hi"].cast<int>();
  g.wi = d["wi"].cast<int>();
  g.c = d["c"].cast<int>();
  g.ho = d["ho"].cast<int>();
  g.wo = d["wo"].cast<int>();
  g.sh = d["sh"].cast<int>();
  g.sw = d["sw"].cast<int>();
  g.tap_c = d["tap_c"].cast<int>();
  g.tap_shift = (g.tap_c > 0 && (g.tap_c & (g.tap_c - 1)) == 0) ? __builtin_ctz((unsigned)g.tap_c) : -1;
  auto dh = d["dh"].cast<std::vector<int>>();
  auto dw = d["dw"].cast<std::vector<int>>();
  std::vector<int> wt = d.contains("wt") ? d["wt"].cast<std::vector<int>>() : std::vector<int>(dh.size(), 0);
  TORCH_CHECK(dh.size() == dw.size() && dh.size() <= (size_t)kMaxTaps && wt.size() == dh.size(), "bad tap table");
  g.ntaps = (int)dh.size();
  for (size_t i = 0; i < dh.size(); ++i) {
    TORCH_CHECK(dh[i] >= -128 && dh[i] < 128 && dw[i] >= -128 && dw[i] < 128, "tap offset out of int8 range");
    g.dh[i] = (int8_t)dh[i];
    g.dw[i] = (int8_t)dw[i];
    g.wt[i] = (int16_t)wt[i];
  }
}

// C[m][n] = alpha * sum_k A(m,k) B(n,k) (+ epilogue).  Modes: see ddl_gemm.h.
void gemm(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, int64_t M, int64_t N, int64_t K,
          int64_t a_mode, int64_t b_mode, int64_t lda, int64_t ldb, int64_t ldc, int64_t epi, int64_t tile,
          int64_t k_split, double alpha, double beta, c10::optional<at::Tensor> bias,
          c10::optional<at::Tensor> resid, int64_t ldr, int64_t relu, c10::optional<py::dict> geom,
          c10::optional<py::dict> outmap, int64_t b_kdiv, int64_t b_tap_stride,
          c10::optional<at::Tensor> stats, c10::optional<at::Tensor> aux, double drop_p, int64_t drop_seed,
          c10::optional<at::Tensor> resid_mask, c10::optional<at::Tensor> bnr_x, c10::optional<at::Tensor> bnr_mask,
          c10::optional<at::Tensor> bnr_mean, int64_t rsub_h, int64_t rsub_w, c10::optional<at::Tensor> bnr_scale, c10::optional<at::Tensor> bnr_shift, int64_t split_stride,
          int64_t zcount, int64_t za, int64_t zb, int64_t zc, int64_t zbias, std::vector<int64_t> cls_tap0,
          std::vector<int64_t> cls_nt, std::vector<int64_t> cls_coff) {
  CHECK_CUDA(a);
  CHECK_CUDA(b);
  CHECK_CUDA(c);
  CHECK_BF16(a);
  CHECK_BF16(b);
  if (epi == EPI_BF16) { CHECK_BF16(c); } else { CHECK_F32(c); }
  const bool k_vec = a_mode == OP_KC || a_mode == OP_KC_GATHER || a_mode == OP_KC_GATHER8 || b_mode == OP_KC;
  TORCH_CHECK(!k_vec || K % 8 == 0, "gemm: K-contiguous operands need K % 8 == 0 (16-B vectors), got ", K);
  if (a_mode == OP_KC) TORCH_CHECK(lda % 8 == 0, "gemm: lda must be a multiple of 8");
  if (b_mode == OP_KC) TORCH_CHECK(ldb % 8 == 0, "gemm: ldb must be a multiple of 8");
  if (a_mode == OP_RC) TORCH_CHECK(lda % 8 == 0, "gemm: lda must be a multiple of 8");
  if (b_mode == OP_RC || b_mode == OP_RC_TAPS) TORCH_CHECK(ldb % 8 == 0, "gemm: ldb must be a multiple of 8");
  TORCH_CHECK(((uintptr_t)a.data_ptr() % 16) == 0 && ((uintptr_t)b.data_ptr() % 16) == 0, "gemm: operands must be 16-B aligned");
  TORCH_CHECK(k_split > 0 && k_split % 64 == 0, "gemm: k_split must be a positive multiple of 64");
  TORCH_CHECK(tile >= 0 && tile <= kTileConv3, "gemm: bad tile id");
  if (tile == kTileStream) {
    TORCH_CHECK(a_mode == OP_KC && (b_mode == OP_KC || b_mode == OP_RC) && epi == EPI_BF16 && !outmap.has_value() &&
                    relu <= ACT_RELU && drop_p == 0.0 && beta == 0.0 && k_split >= K,
                "gemm stream: KC x (KC|RC) operands, bf16 epilogue without GELU/dropout/outmap/beta/split-K");
    TORCH_CHECK(gemm_stream_panel((int)N, (int)K) > 0, "gemm stream: unsupported (N, K) = (", N, ", ", K, ")");
    TORCH_CHECK(ldc % 8 == 0 && ((uintptr_t)c.data_ptr() % 16) == 0, "gemm stream: 16-B aligned output rows");
    TORCH_CHECK(!resid || (ldr % 4 == 0 && ((uintptr_t)resid->data_ptr() % 8) == 0), "gemm stream: resid alignment");
  }
  if (tile == kTile256) {
    TORCH_CHECK(a_mode <= OP_RC && b_mode <= OP_RC && !outmap.has_value(), "gemm256: plain KC/RC operands only");
    TORCH_CHECK(K % 64 == 0 && k_split % 64 == 0, "gemm256: K and k_split must be multiples of 64");
    TORCH_CHECK(M >= 8 && N >= 8, "gemm256: M, N >= 8");
  }
  const int bm = (tile == 0 || tile == 1) ? 128 : 64;
  const int bn = (tile == 0 || tile == 2) ? 128 : 64;
  if (a_mode == OP_RC || a_mode == OP_RC_GATHER) TORCH_CHECK(M % 8 == 0, "gemm: row-contiguous A needs M % 8 == 0");
  if (b_mode == OP_RC || b_mode == OP_RC_GATHER || b_mode == OP_RC_GATHER8 || b_mode == OP_RC_TAPS)
    TORCH_CHECK(N % 8 == 0, "gemm: row-contiguous B needs N % 8 == 0");
  GemmParams p{};
  p.a = a.data_ptr();
  p.b = b.data_ptr();
  p.c = c.data_ptr();
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.M = (int)M;
  p.N = (int)N;
  p.K = (int)K;
  p.k_split = (int)k_split;
  p.a_mode = (int)a_mode;
  p.b_mode = (int)b_mode;
  p.b_kdiv = (int)b_kdiv;
  p.b_tap_stride = b_tap_stride;
  p.alpha = (float)alpha;
  p.beta = (float)beta;
  TORCH_CHECK(relu >= ACT_NONE && relu <= ACT_GELU_BWD, "gemm: bad activation code");
  TORCH_CHECK(epi == EPI_BF16 || (relu == 0 && drop_p == 0.0), "gemm: activation/dropout need the bf16 epilogue");
  p.relu = (int)relu;
  if (relu >= ACT_GELU) {
    TORCH_CHECK(aux.has_value(), "gemm: GELU epilogues need the aux (pre-activation) tensor");
    CHECK_CUDA(*aux);
    CHECK_BF16(*aux);
    TORCH_CHECK(aux->numel() >= (M - 1) * ldc + N && ((uintptr_t)aux->data_ptr() % 16) == 0, "gemm: aux size/alignment");
    p.aux = aux->data_ptr();
  }
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "gemm: dropout p in [0, 1)");
  if (drop_p > 0.0) {
    p.drop_thresh = drop_t8(drop_p);  // threshold byte: the rate quantised to 1/256 (ddl_ops.h)
    p.drop_scale = drop_scale8(p.drop_thresh);
    p.drop_seed = (unsigned long long)drop_seed;
  }
  p.ldr = ldr;
  if (bias) {
    CHECK_CUDA(*bias);
    CHECK_F32(*bias);
    TORCH_CHECK(bias->numel() >= N, "bias too short");
    TORCH_CHECK((uintptr_t)bias->data_ptr() % 16 == 0, "gemm: bias must be 16-B aligned (vector loads)");
    p.bias = bias->data_ptr<float>();
  }
  if (resid) {
    CHECK_CUDA(*resid);
    CHECK_BF16(*resid);
    p.resid = resid->data_ptr();
  }
  if (rsub_h > 0) {
    TORCH_CHECK(resid.has_value() && epi == EPI_BF16 && !outmap.has_value() && !resid_mask.has_value() && rsub_w > 0 &&
                    M % (rsub_h * rsub_w) == 0,
                "gemm: a stride-2 residual needs resid (bf16, no outmap / mask) and M = N * rsub_h * rsub_w");
    const int64_t hs = (rsub_h + 1) / 2, ws_ = (rsub_w + 1) / 2;
    TORCH_CHECK(resid->numel() >= ((M / (rsub_h * rsub_w)) * hs * ws_ - 1) * ldr + N, "gemm: stride-2 residual too small");
    p.rsub_h = (int)rsub_h;
    p.rsub_w = (int)rsub_w;
  }
  if (resid_mask) {
    TORCH_CHECK(resid.has_value() && epi == EPI_BF16 && !outmap.has_value(), "gemm: resid_mask needs a residual (bf16, no outmap)");
    TORCH_CHECK(resid_mask->scalar_type() == at::kByte && resid_mask->is_contiguous() && ldr % 8 == 0 &&
                    resid_mask->numel() >= ((M - 1) * ldr + N + 7) / 8,
                "gemm: resid_mask must be uint8 [M * ldr / 8] with ldr % 8 == 0");
    p.resid_mask = resid_mask->data_ptr<uint8_t>();
  }
  if (geom) {
    fill_geom(p.g, *geom);
    // the gathering operand modes compute element offsets in 32 bits (ddl_gemm_kernel.h)
    TORCH_CHECK((int64_t)p.g.n * p.g.hi * p.g.wi * p.g.c < (int64_t(1) << 31),
                "gemm: a gathered tensor must have fewer than 2^31 elements");
    if (a_mode == OP_KC_GATHER)  // (parity classes: each class's K = its taps * C, checked below)
      TORCH_CHECK(p.g.tap_c % 64 == 0 && (cls_nt.empty() ? K == (int64_t)p.g.ntaps * p.g.tap_c : K <= (int64_t)p.g.ntaps * p.g.tap_c),
                  "conv A gather: tap_c % 64 and K = taps*C");
    if (b_mode == OP_RC_GATHER) TORCH_CHECK(p.g.tap_c % bn == 0 && N == (int64_t)p.g.ntaps * p.g.tap_c, "conv B gather: tap_c % BN and N = taps*C");
    if (b_mode == OP_RC_TAPS) TORCH_CHECK(b_kdiv % 64 == 0 && K == (int64_t)p.g.ntaps * b_kdiv, "conv B taps: kdiv % 64 and K = taps*kdiv");
    if (a_mode == OP_KC_GATHER8) TORCH_CHECK(p.g.tap_c % 8 == 0 && K == (int64_t)p.g.ntaps * p.g.tap_c, "conv A gather8: tap_c % 8 and K = taps*C");
    if (b_mode == OP_RC_GATHER8) TORCH_CHECK(p.g.tap_c % 8 == 0 && N == (int64_t)p.g.ntaps * p.g.tap_c, "conv B gather8: tap_c % 8 and N = taps*C");
    if (a_mode == OP_KC_GATHER || a_mode == OP_KC_GATHER8) TORCH_CHECK(p.g.c == p.g.tap_c, "gather: c == tap_c");
  } else {
    TORCH_CHECK(a_mode <= OP_RC && b_mode <= OP_RC, "gather modes need a geometry");
  }
  if (outmap) {
    const auto& d = *outmap;
    p.om.enabled = 1;
    p.om.gh = d["gh"].cast<int>();
    p.om.gw = d["gw"].cast<int>();
    p.om.hy = d["hy"].cast<int>();
    p.om.wy = d["wy"].cast<int>();
    p.om.so = d["so"].cast<int>();
    p.om.oh = d["oh"].cast<int>();
    p.om.ow = d["ow"].cast<int>();
    p.om.zero_siblings = d.contains("zero") ? d["zero"].cast<int>() : 0;
  }
  if (stats) {
    CHECK_CUDA(*stats);
    CHECK_F32(*stats);
    TORCH_CHECK(epi == EPI_BF16, "fused stats need the bf16 epilogue");
    TORCH_CHECK(stats->numel() >= (int64_t)kStatShards * 2 * N, "stats workspace too small");
    p.stats = stats->data_ptr<float>();
  }
  if (bnr_x) {
    TORCH_CHECK(stats.has_value() && bnr_mean.has_value() && epi == EPI_BF16 && tile != kTile256,
                "gemm: the fused BN-backward reduction needs a stats workspace, the mean and a bf16 epilogue");
    TORCH_CHECK(tile == kTileStream || (N % 4 == 0 && ldc % 8 == 0 && !bias && relu == 0 && !aux &&
                                        drop_p == 0.0 && (a_mode == OP_KC || (a_mode == OP_KC_GATHER && b_mode == OP_KC))),
                "gemm: BN-backward reduce outside the streaming kernel: plain or gathered-A data-gradient, N % 4 == 0, "
                "ldc % 8 == 0, no bias / activation (a residual and a parity-class output map are allowed)");
    CHECK_CUDA(*bnr_x);
    CHECK_BF16(*bnr_x);
    TORCH_CHECK(bnr_x->is_contiguous() && bnr_x->numel() >= (M - 1) * ldc + N && ((uintptr_t)bnr_x->data_ptr() % 16) == 0,
                "gemm: bnr_x must be a 16-B aligned bf16 [M][ldc]");
    CHECK_F32(*bnr_mean);
    TORCH_CHECK(bnr_mean->numel() >= N && ((uintptr_t)bnr_mean->data_ptr() % 16) == 0, "gemm: bnr_mean [N], 16-B aligned");
    p.bnr_x = bnr_x->data_ptr();
    p.bnr_mean = bnr_mean->data_ptr<float>();
    if (bnr_mask) {
      TORCH_CHECK(bnr_mask->scalar_type() == at::kByte && bnr_mask->is_contiguous() && ldc % 8 == 0 &&
                      bnr_mask->numel() >= ((M - 1) * ldc + N + 7) / 8,
                  "gemm: bnr_mask must be uint8 [M * ldc / 8]");
      p.bnr_mask = bnr_mask->data_ptr<uint8_t>();
    }
    if (bnr_scale || bnr_shift) {  // mode-2 mask (ReLU of the BN output recomputed from x)
      TORCH_CHECK(bnr_scale && bnr_shift && !bnr_mask && (tile != kTileStream || !resid),
                  "gemm: bnr scale/shift (no mask bits; no residual on the streaming kernel)");
      CHECK_F32(*bnr_scale);
      CHECK_F32(*bnr_shift);
      TORCH_CHECK(bnr_scale->numel() >= N && bnr_shift->numel() >= N && ((uintptr_t)bnr_scale->data_ptr() % 16) == 0 &&
                      ((uintptr_t)bnr_shift->data_ptr() % 16) == 0,
                  "gemm: bnr scale / shift [N], 16-B aligned");
      p.bnr_scale = bnr_scale->data_ptr<float>();
      p.bnr_shift = bnr_shift->data_ptr<float>();
    }
  }
  (void)bm;
  if (tile == kTileConv3)
    TORCH_CHECK(conv3x3_halo_ok(p) && epi == EPI_BF16, "gemm conv3x3: needs a 3x3 / stride-1 / pad-1 KC_GATHER x KC "
                "conv with C % 64 == 0, N % 64 == 0, no split-K and at most bias/ReLU/statistics in the epilogue");
  if (split_stride > 0) {
    const int64_t splits = (K + k_split - 1) / k_split;
    TORCH_CHECK(epi == EPI_F32 && beta == 0.0 && split_stride >= M * ldc && c.numel() >= splits * split_stride,
                "gemm: split-K slabs need EPI_F32, beta = 0 and a workspace of splits x split_stride floats");
    p.split_stride = split_stride;
  }
  if (zcount > 1 && cls_nt.empty()) {  // replica batching: z-th operands / output / bias at element offsets z * (za, zb, zc, zbias)
    TORCH_CHECK(tile >= 0 && tile <= 3 && !stats && !bnr_x && !outmap && !resid && !aux && drop_p == 0.0 &&
                    split_stride == 0 && relu <= ACT_RELU && za >= 0 && zb >= 0 && zc >= 0 && zbias >= 0,
                "gemm: replica batching (zcount > 1) runs the 64/128 tiles with at most bias / ReLU / split-K atomics");
    TORCH_CHECK(za % 8 == 0 && zb % 8 == 0 && (epi == EPI_BF16 ? zc % 8 : zc % 4) == 0 && zbias % 4 == 0,
                "gemm: replica strides must keep 16-B alignment");
    TORCH_CHECK(c.numel() >= (zcount - 1) * zc + (M - 1) * ldc + N, "gemm: output too small for zcount replicas");
    TORCH_CHECK(!bias || bias->numel() >= (zcount - 1) * zbias + N, "gemm: bias too short for zcount replicas");
    p.zcount = (int)zcount;
    p.za = za;
    p.zb = zb;
    p.zc = zc;
    p.zbias = zbias;
  }
  if (!cls_nt.empty()) {  // parity classes of a strided data-gradient in one launch (GemmParams::zcls)
    const int64_t nc = (int64_t)cls_nt.size();
    TORCH_CHECK(nc <= kMaxZCls && (int64_t)cls_tap0.size() == nc && (int64_t)cls_coff.size() == nc && zcount == nc,
                "gemm: parity classes need cls_tap0 / cls_nt / cls_coff of zcount <= ", kMaxZCls, " entries");
    TORCH_CHECK(tile >= 0 && tile <= 3 && a_mode == OP_KC_GATHER && b_mode == OP_KC && epi == EPI_BF16 && outmap &&
                    p.om.oh == 0 && p.om.ow == 0 && !p.om.zero_siblings && !stats && !bnr_x && !resid && !aux && !bias &&
                    drop_p == 0.0 && relu == 0 && split_stride == 0 && za == 0 && zb == 0 && zc == 0 && zbias == 0,
                "gemm: parity classes run KC_GATHER x KC on the 64/128 tiles with a plain bf16 output map");
    TORCH_CHECK(p.om.gh > 0 && p.om.gw > 0 && M % ((int64_t)p.om.gh * p.om.gw) == 0, "gemm: classes need M = n * gh * gw");
    const int64_t nimg = M / ((int64_t)p.om.gh * p.om.gw);
    const int64_t last_row = ((nimg - 1) * p.om.hy + (int64_t)(p.om.gh - 1) * p.om.so) * p.om.wy + (int64_t)(p.om.gw - 1) * p.om.so;
    int64_t kmax = 0;
    for (int64_t z = 0; z < nc; ++z) {
      TORCH_CHECK(cls_nt[z] > 0 && cls_tap0[z] >= 0 && cls_tap0[z] + cls_nt[z] <= p.g.ntaps, "gemm: class taps out of range");
      TORCH_CHECK(cls_coff[z] >= 0 && cls_coff[z] % 8 == 0 && cls_coff[z] + last_row * ldc + N <= c.numel(),
                  "gemm: class output offset out of range");
      TORCH_CHECK((cls_tap0[z] + cls_nt[z]) * (int64_t)p.g.tap_c <= ldb, "gemm: class filter columns past ldb");
      kmax = std::max(kmax, cls_nt[z] * (int64_t)p.g.tap_c);
      p.cls_tap0[z] = (int)cls_tap0[z];
      p.cls_nt[z] = (int)cls_nt[z];
      p.cls_coff[z] = cls_coff[z];
    }
    TORCH_CHECK(K == kmax && k_split >= K, "gemm: classes need K = the largest class's K and no split-K");
    p.zcls = 1;
    p.zcount = (int)nc;
  }
  at::DeviceGuard guard(a.device());
  HIP_OK(launch_gemm_bf16(p, (int)epi, (int)tile, cur_stream()));
}

// 3x3 / stride-1 / pad-1 weight gradient, halo kernel (conv3x3.hip): gw[Co][3][3][Ci] (fp32) += dW.
// ws: fp32 slab workspace of splits * Co * 9 * Ci floats (plain stores + reduce kernel), or None (atomics).
void conv3x3_wgrad(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& gw, const c10::optional<at::Tensor>& ws,
                   int64_t splits, int64_t tpb, bool pp) {
  CHECK_CUDA(dy);
  CHECK_CUDA(x);
  CHECK_CUDA(gw);
  CHECK_BF16(dy);
  CHECK_BF16(x);
  CHECK_F32(gw);
  CHECK_CONTIG(dy);
  CHECK_CONTIG(x);
  CHECK_CONTIG(gw);
  TORCH_CHECK(x.dim() == 4 && gw.dim() == 4 && gw.size(1) == 3 && gw.size(2) == 3 && gw.size(3) == x.size(3),
              "conv3x3_wgrad: x [N, H, W, Ci], gw [Co, 3, 3, Ci]");
  const int n = (int)x.size(0), h = (int)x.size(1), w = (int)x.size(2), ci = (int)x.size(3), co = (int)gw.size(0);
  TORCH_CHECK(dy.numel() == (int64_t)n * h * w * co, "conv3x3_wgrad: dy must be [N, H, W, Co] (stride 1, pad 1)");
  TORCH_CHECK(conv3x3_wgrad_ok(n, h, w, ci, co), "conv3x3_wgrad: needs Ci, Co % 64 == 0 and a <= 256-pixel row tiling");
  int s_plan = 0, t_plan = 0, ntiles = 0;
  conv3x3_wgrad_plan(n, h, w, ci, co, 1, 1, s_plan, t_plan, ntiles);
  TORCH_CHECK(splits >= 1 && tpb >= 1 && (splits - 1) * tpb < ntiles && splits * tpb >= ntiles,
              "conv3x3_wgrad: splits x tiles-per-split must cover the pixel tiles exactly once");
  float* wsp = nullptr;
  if (ws) {
    CHECK_CUDA(*ws);
    CHECK_F32(*ws);
    TORCH_CHECK(ws->is_contiguous() && ws->numel() >= splits * co * 9 * (int64_t)ci, "conv3x3_wgrad: workspace too small");
    wsp = ws->data_ptr<float>();
  }
  at::DeviceGuard guard(x.device());
  HIP_OK(launch_conv3x3_wgrad(reinterpret_cast<const uint16_t*>(dy.data_ptr()), reinterpret_cast<const uint16_t*>(x.data_ptr()),
                              gw.data_ptr<float>(), wsp, n, h, w, ci, co, (int)splits, (int)tpb, pp, cur_stream()));
}

py::object conv3x3_wgrad_plan_py(int64_t n, int64_t h, int64_t w, int64_t ci, int64_t co, int64_t blocks_per_cu,
                                 int64_t cus) {
  if (!conv3x3_wgrad_ok((int)n, (int)h, (int)w, (int)ci, (int)co)) return py::none();
  int splits = 0, tpb = 0, ntiles = 0;
  conv3x3_wgrad_plan((int)n, (int)h, (int)w, (int)ci, (int)co, (int)blocks_per_cu, (int)cus, splits, tpb, ntiles);
  return py::make_tuple(splits, tpb);
}

}  // namespace

void register_ops(py::module& m);      // ops_bindings.cpp style registrations (elementwise, norms, ...)
void register_runtime(py::module& m);  // host runtime (parameter server, ingest)
void register_transformer(py::module& m);  // attention, LayerNorm, embeddings
void register_rnn(py::module& m);          // persistent GRU / LSTM / SimpleRNN
void register_layer_ops(py::module& m);    // Keras layer element-wise ops, fp32 GEMM

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X-native kernels and runtime of distributeddeeplearningspark_amd";
  m.def("gemm", &gemm, "MFMA implicit-GEMM (bf16 in, fp32 accumulate)", py::arg("a"), py::arg("b"), py::arg("c"),
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("a_mode"), py::arg("b_mode"), py::arg("lda"),
        py::arg("ldb"), py::arg("ldc"), py::arg("epi"), py::arg("tile"), py::arg("k_split"), py::arg("alpha") = 1.0,
        py::arg("beta") = 0.0, py::arg("bias") = py::none(), py::arg("resid") = py::none(), py::arg("ldr") = 0,
        py::arg("relu") = false, py::arg("geom") = py::none(), py::arg("outmap") = py::none(),
        py::arg("b_kdiv") = 0, py::arg("b_tap_stride") = 0, py::arg("stats") = py::none(),
        py::arg("aux") = py::none(), py::arg("drop_p") = 0.0, py::arg("drop_seed") = 0,
        py::arg("resid_mask") = py::none(), py::arg("bnr_x") = py::none(), py::arg("bnr_mask") = py::none(),
        py::arg("bnr_mean") = py::none(), py::arg("rsub_h") = 0, py::arg("rsub_w") = 0,
        py::arg("bnr_scale") = py::none(), py::arg("bnr_shift") = py::none(),
        py::arg("split_stride") = 0, py::arg("zcount") = 1, py::arg("za") = 0, py::arg("zb") = 0, py::arg("zc") = 0,
        py::arg("zbias") = 0, py::arg("cls_tap0") = std::vector<int64_t>{}, py::arg("cls_nt") = std::vector<int64_t>{},
        py::arg("cls_coff") = std::vector<int64_t>{});
  m.def("conv3x3_wgrad", &conv3x3_wgrad, "3x3 stride-1 weight gradient (halo kernel): gw += dW", py::arg("dy"),
        py::arg("x"), py::arg("gw"), py::arg("ws"), py::arg("splits"), py::arg("tpb"), py::arg("pp") = false);
  m.def("conv3x3_wgrad_plan", &conv3x3_wgrad_plan_py,
        "(splits, tiles per split) of the 3x3 weight-gradient halo kernel, or None when it does not apply",
        py::arg("n"), py::arg("h"), py::arg("w"), py::arg("ci"), py::arg("co"), py::arg("blocks_per_cu"),
        py::arg("cus"));
  m.attr("ACT_NONE") = (int)ACT_NONE;
  m.attr("ACT_RELU") = (int)ACT_RELU;
  m.attr("ACT_GELU") = (int)ACT_GELU;
  m.attr("ACT_GELU_BWD") = (int)ACT_GELU_BWD;
  m.attr("OP_KC") = (int)OP_KC;
  m.attr("OP_RC") = (int)OP_RC;
  m.attr("OP_KC_GATHER") = (int)OP_KC_GATHER;
  m.attr("OP_RC_GATHER") = (int)OP_RC_GATHER;
  m.attr("OP_RC_TAPS") = (int)OP_RC_TAPS;
  m.attr("OP_KC_GATHER8") = (int)OP_KC_GATHER8;
  m.attr("OP_RC_GATHER8") = (int)OP_RC_GATHER8;
  m.attr("EPI_BF16") = (int)EPI_BF16;
  m.attr("EPI_F32") = (int)EPI_F32;
  m.attr("EPI_F32_ATOMIC") = (int)EPI_F32_ATOMIC;
  register_ops(m);
  register_transformer(m);
  register_rnn(m);
  register_layer_ops(m);
  register_runtime(m);
}
