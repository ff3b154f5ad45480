// Host-visible parameter block for the MFMA implicit-GEMM kernel family.
//
// One kernel template covers every GEMM-shaped op of the framework:
//   * plain GEMMs with either operand K-contiguous ("KC") or row-contiguous ("RC"),
//     i.e. NT / NN / TN / TT in BLAS terms (Linear fwd / dgrad / wgrad, 1x1 conv);
//   * NHWC implicit-GEMM convolution: forward and data-gradient gather the A
//     operand through a tap table (KC_GATHER), weight-gradient gathers the B
//     operand (RC_GATHER); the data-gradient reads the weights through a tap
//     table (RC_TAPS) and can scatter its output to a strided grid (stride-2
//     parity classes).
// C[m][n] = sum_k A(m,k) * B(n,k)
#pragma once
#include <stdint.h>

namespace ddl {

enum OperandMode : int {
  OP_KC = 0,         // addr = ptr + r*ld + k
  OP_RC = 1,         // addr = ptr + k*ld + r
  OP_KC_GATHER = 2,  // conv input gather: r = output pixel, k = tap*C + c
  OP_RC_GATHER = 3,  // conv input gather: k = output pixel, r = tap*C + c
  OP_RC_TAPS = 4,    // weight [co][tap][c]: r = c, k = tap*Co + co
  OP_KC_GATHER8 = 5, // as KC_GATHER for small channel counts (C % 8 == 0): tap looked up per 16-B vector
  OP_RC_GATHER8 = 6, // as RC_GATHER for C % 8 == 0
};

enum EpilogueMode : int {
  EPI_BF16 = 0,        // bf16 store of alpha*acc (+bias)(+resid)(relu)
  EPI_F32 = 1,         // fp32 store of alpha*acc + beta*C
  EPI_F32_ATOMIC = 2,  // fp32 atomicAdd of alpha*acc (split-K)
  // EPI_BF16 restricted to alpha / bias / ReLU / BN statistics (no residual, output map, GELU
  // or dropout).  A separate instantiation because the full epilogue's live state raises the
  // kernel's VGPR allocation (134 -> occupancy 3 blocks/CU for the 128x128 conv kernel); the
  // launcher picks it whenever the call does not use the extra features.
  EPI_BF16_LITE = 3,
  // bf16 store of alpha*acc plus the fused BatchNorm-backward partial sums of the stored values
  // (GemmParams::bnr_*) — the LDS-DMA GEMM and halo-conv kernels' form of the streaming kernel's BNR
  // read-out (selected by the launchers when bnr_x is set on a non-streaming tile)
  EPI_BF16_BNR = 4,
};

constexpr int kMaxTaps = 64;
constexpr int kMaxZCls = 4;  // parity classes per batched data-gradient launch (stride 2)

struct ConvGeom {
  int n, hi, wi, c;   // gathered NHWC tensor
  int ho, wo;         // iteration grid over pixels
  int sh, sw;         // stride on that grid
  int ntaps;
  int tap_c;          // channels per tap inside the gathered dimension
  int tap_shift;      // log2(tap_c) when tap_c is a power of two, else -1 (per-vector tap lookups)
  int8_t dh[kMaxTaps];
  int8_t dw[kMaxTaps];
  int16_t wt[kMaxTaps];  // weight tap index (OP_RC_TAPS)
};

struct OutMap {       // scatter of output rows to a strided NHWC grid (dgrad parity classes)
  int enabled;
  int gh, gw;         // row grid (rows m -> (n, i, j))
  int hy, wy;         // destination spatial dims
  int so;             // destination stride
  int oh, ow;         // destination offsets
  int zero_siblings;  // also write zeros to the other so*so-1 positions of each cell
};

struct GemmParams {
  const void* a; long lda;
  const void* b; long ldb;
  void* c; long ldc;
  int M, N, K;
  int k_split;        // K elements per split (multiple of 64)
  int a_mode, b_mode;
  // RC_TAPS: k -> (tap = k / kdiv, co = k % kdiv); addr = ptr + co*ldb + wt[tap]*tap_stride + r
  int b_kdiv; long b_tap_stride;
  ConvGeom g;
  OutMap om;
  const float* bias;
  const void* resid; long ldr;
  // optional ReLU bit mask of the residual (bn.hip mode-3 layout: byte (m*ldr + n) / 8, bit n % 8):
  // resid is added only where the bit is set — the masked gradient of a residual BN is formed in
  // the consumer's epilogue instead of being written out by the BN backward sweep
  const uint8_t* resid_mask;
  float alpha, beta;
  // bf16 epilogue activation (field name kept from the first version):
  //   ACT_NONE, ACT_RELU (after the residual add), ACT_GELU (aux <- pre-activation),
  //   ACT_GELU_BWD (v *= gelu'(aux[m][n]), the data-gradient of a GELU-fused Linear)
  int relu;
  // optional fused per-column batch statistics of the stored bf16 output:
  // stats[shard][0][n] += sum, stats[shard][1][n] += sum of squares (shard = tile % kStatShards)
  float* stats;
  void* aux;          // bf16 [M][ldc]: pre-activation (ACT_GELU out / ACT_GELU_BWD in)
  // dropout applied after bias/activation and before the residual add:
  // keep element (m, n) iff drop_keep(drop_seed, m*N + n, drop_thresh) (ddl_common.h: drop_thresh is the
  // threshold byte t8), kept values * drop_scale
  uint32_t drop_thresh;
  float drop_scale;
  unsigned long long drop_seed;
  // fused BatchNorm-backward reduction of the STORED output d (the gradient arriving at a BN whose
  // input is bnr_x): instead of the forward statistics, ``stats`` receives
  //   stats[shard][0][n] += sum_m d(m,n) * relu(m,n),  stats[shard][1][n] += sum_m d * relu * (x(m,n) - mean[n])
  // with relu(m,n) the bn.hip mode-3 bit of bnr_mask, or (mode 2) x(m,n) * bnr_scale[n] + bnr_shift[n] > 0,
  // or all ones when neither is given — the partial sums of bn_bwd_reduce, so that sweep (a full read of
  // d and x) is skipped for that BN.  Streaming kernel: mask bits only; LDS-DMA GEMM / halo conv:
  // EPI_BF16_BNR, either mask form.
  const void* bnr_x;        // bf16 [M][ldc]
  const uint8_t* bnr_mask;  // bit (m*ldc + n) of the ReLU mask, or null
  const float* bnr_mean;    // [N] batch mean of bnr_x
  const float* bnr_scale;   // [N] BN scale / shift of the forward (mode-2 mask), or null
  const float* bnr_shift;
  // stride-2 residual: when rsub_h > 0 the output rows m = (n, i, j) form an [N][rsub_h][rsub_w] grid
  // and ``resid`` lives on its stride-2 subgrid ([N][(rsub_h+1)/2][(rsub_w+1)/2], row stride ldr):
  // rows with even (i, j) add resid row ((n * Hs + i/2) * Ws + j/2), the others add nothing — the
  // data-gradient of a ResNet stride-2 1x1 downsample shortcut, added at half resolution instead of
  // being scattered (with zeros) to full resolution first
  int rsub_h, rsub_w;
  // tile raster of the LDS-DMA GEMM kernel: > 1 walks groups of group_m M-tiles across all N-tiles
  // (M fastest inside a group) so the tiles resident on one XCD share fewer A rows and B columns
  // (set by launch_gemm_bf16 from DDL_GEMM_GROUP_M; 0 = row-major over the tiles)
  int group_m;
  // split-K through partial SLABS (plain stores, EPI_F32 only): split s writes its partial C at
  // c + s * split_stride (elements, ldc unchanged); a reduce pass sums the slabs in split order
  // (slab_reduce: deterministic, and ~4x the store rate of the fp32 atomics it replaces).  0 = off.
  long split_stride;
  // replica batching (gemm_dma_kernel only): blockIdx.z = z selects operands a + z*za, b + z*zb (bf16
  // elements), output c + z*zc and bias + z*zbias (elements) — the co-located replicas of one model, each
  // with its own weights, as ONE launch (parallel/replica_seq.py).  0 / unused when gridDim.z == 1.
  int zcount;
  long za, zb, zc, zbias;
  // parity classes of a strided data-gradient as ONE launch (gemm_dma_kernel, KC_GATHER x KC; zcls = 1,
  // zcount = classes): class z = blockIdx.z reduces K = cls_nt[z] * g.tap_c over taps [cls_tap0[z],
  // cls_tap0[z] + cls_nt[z]) of the tap table, reads B from column cls_tap0[z] * g.tap_c of the shared
  // [N][taps * tap_c] class-ordered filter and writes C at element offset cls_coff[z] (the class's
  // (oh, ow) cell offset in the OutMap grid, whose own oh / ow stay 0).  ops/conv.py:conv_dgrad_native.
  int zcls;
  int cls_tap0[kMaxZCls], cls_nt[kMaxZCls];
  long cls_coff[kMaxZCls];
};

enum Activation : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_GELU_BWD = 3 };

constexpr int kStatShards = 32;
constexpr int kTile256 = 4;     // tile id of the 256x256 ping-pong kernel (ddl_gemm256.h)
constexpr int kTileStream = 5;  // tile id of the weight-stationary streaming kernel (gemm_stream.hip)
constexpr int kTileConv3 = 6;   // tile id of the 3x3 stride-1 halo convolution kernel (conv3x3.hip)

// the halo kernel applies to this (KC_GATHER x KC, 3x3 / stride 1 / pad 1) GEMM
bool conv3x3_halo_ok(const GemmParams& p);

// 3x3 / stride-1 / pad-1 weight gradient with the input halo in LDS (conv3x3.hip): applicability, split plan
// (pixel-tile splits and tiles per workgroup) and launch; ws = [splits][Co][9 Ci] fp32 slabs reduced into gw by
// a second kernel, or nullptr for atomic accumulation into gw [Co][9 Ci]; pp: the 512-thread ping-pong form
// (plan it with blocks_per_cu = 1)
bool conv3x3_wgrad_ok(int n, int h, int w, int ci, int co);
void conv3x3_wgrad_plan(int n, int h, int w, int ci, int co, int blocks_per_cu, int cus, int& splits, int& tpb,
                        int& ntiles);
int launch_conv3x3_wgrad(const uint16_t* dy, const uint16_t* x, float* gw, float* ws, int n, int h, int w, int ci,
                         int co, int splits, int tpb, bool pp, void* stream);

// panel width of the streaming kernel for (N, K), 0 when it does not apply
int gemm_stream_panel(int N, int K);

// host launcher (defined in gemm_bf16.hip); returns hipError_t as int
int launch_gemm_bf16(const GemmParams& p, int epi, int tile, void* stream);

}  // namespace ddl
