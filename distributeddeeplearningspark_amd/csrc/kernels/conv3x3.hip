// 3x3 stride-1 pad-1 NHWC convolution on MFMA with an input HALO staged in LDS (gfx950).
//
// Why: the implicit-GEMM kernel gathers the A operand once per TAP — every input pixel crosses
// the L2 -> LDS path 9 times per output-channel tile, and at ~30 B/clk/CU of gathered L2 -> LDS
// bandwidth a 128x128 tile is capped near half the MFMA rate (PMC: 20-27 % MFMA, 45-55 % of wave
// time parked on s_waitcnt / barriers; profiles/r2/pmc_conv3x3_*.txt).  Here a workgroup owns a
// block of whole output rows (P <= 256 pixels: R rows of one image, or IMG whole images when an
// image has <= 256 pixels), stages the (R+2) x (W+2) input halo ONCE per 64-channel chunk, and
// reads all nine taps' A fragments from it at tap-shifted LDS rows; only the weights stream per
// tap (double-buffered LDS-DMA, the next tap's tile in flight under the current tap's MFMAs).
// Padding is exact: out-of-image halo pixels are DMA'd from the zero page.
//
// Used for the forward conv and, through the flipped filter, for the stride-1 data-gradient
// (ops/conv.py).  C % 64 == 0, Co % 64 == 0 (BN = 64 or 128 output channels per workgroup).
//
// Layout per workgroup (256 threads = 4 waves as 2 (pixels) x 2 (channels)):
//   halo   [HRpad rows][64 ch] bf16, 128-B rows, 16-B chunks XOR-swizzled by (row & 6).  A
//          fragment reads 16 CONSECUTIVE halo rows starting at an arbitrary row (pixel base +
//          tap offset); ds_read_b128 serves lanes {0-3,12-15,20-27} (rows R..R+3, R+12..R+15 at
//          chunk q and R+4..R+11 at chunk q^1) etc. in one LDS cycle only if their 16-B slots
//          differ.  The GEMM kernels' (row>>1)&7 swizzle does that for 16-aligned R only; XOR with
//          (row & 6) does it for every R (exhaustive search over the pair-index windows) — the
//          PMC count of SQ_LDS_BANK_CONFLICT drops to the image-row wraps;
//   B ring 2 x [BN rows][64 ch] (ddl_gemm_kernel.h Operand<BN, OP_KC> images).
// Each wave: 8 pixel fragments (128 pixels) x BN/32 channel fragments of 16; per tap and
// 64-channel chunk 8 x (BN/32) x 2 v_mfma_f32_16x16x32_bf16.
#include "ddl_gemm_kernel.h"

namespace ddl {
namespace {

constexpr int C3_MAX_HALO_ROWS = 384;  // 48 KB of halo

struct Conv3Tiling {
  int img, rows, w;   // tile = img images x rows output rows x w columns (img > 1 only when rows == H)
  int P;              // output pixels per tile
  int hh, ww;         // halo image: (rows + 2) x (w + 2) per image
  int hr, hr_pad;     // halo rows, rounded up to 32 (4 waves x 8 rows per DMA instruction)
  int tiles_img, tiles_row;  // tiles along the image index and along the rows of one image
};

// NB: weight-tile ring depth.  NB = 3: the tile for step s+1 goes into the slot read in step
// s-2, which every wave left before the barrier opening step s-1 — one barrier per tap (plus one
// per 64-channel chunk for the halo reload).  NB = 2 (BN = 128: a third 16-KB slot would cost the
// second workgroup per CU): the slot was read in step s-1, so each step also closes on a barrier.
// FR: 16-pixel fragments per wave along the tile's pixels (the two pixel waves split the tile at
// FR * 16): 8 covers a full 256-pixel tile; 7 serves the 196-pixel tiles every ResNet-50 stage
// plans (7 rows of 28, one 14x14 image, four 7x7 images) — with 8 the second pixel wave spent 3 of
// its 8 fragments on rows past the tile, so every tap paid 16 MFMA blocks for 12.25 of work.
template <int BN, int EPI, int NB, int FR = 8, bool PRIO = false>
__global__ __launch_bounds__(NTHREADS, 2) void conv3x3_halo_kernel(const GemmParams p, const Conv3Tiling t) {
  constexpr int RN = BN / 32;  // channel fragments per wave (2 waves along N)
  constexpr int B_BYTES = BN * BK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  char* bring = smem + t.hr_pad * 128;

  const ConvGeom& g = p.g;
  const int H = g.hi, W = g.wi, C = g.c, N = g.n;
  const int tiles_n = (p.N + BN - 1) / BN;
  int bid, split;
  grid_tile(bid, split);
  const int tp = bid / tiles_n, tn = bid - tp * tiles_n;
  const int n0 = tn * BN;
  const int timg = tp / t.tiles_row, trow = tp - timg * t.tiles_row;
  const int img0 = timg * t.img, oy0 = trow * t.rows;
  const long m0 = ((long)img0 * H + oy0) * W;
  const int mend = (int)min((long)p.M, m0 + t.P);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int wn0 = wn * (BN / 2);

  // halo row of each of this lane's FR pixel fragments (tap (0,0) = top-left of the 3x3 window)
  int abase[FR];
#pragma unroll
  for (int i = 0; i < FR; ++i) {
    const int px = wm * (16 * FR) + 16 * i + (lane & 15);
    if (px < t.P) {
      const int im = px / (t.rows * t.w);
      const int rem = px - im * t.rows * t.w;
      const int oy = rem / t.w, ox = rem - oy * t.w;
      abase[i] = im * t.hh * t.ww + oy * t.ww + ox;
    } else {
      abase[i] = 0;  // beyond the tile: computed on row 0, never stored (mend)
    }
  }

  Operand<BN, OP_KC> B;
  B.init(p.b, p.ldb, p.N, n0, p.K, g);

  const bf16_t* x = reinterpret_cast<const bf16_t*>(p.a);
  const int halo_instr = t.hr_pad / 32;  // 1-KB DMA pieces per wave
  // Source of each of this lane's halo pieces for channel chunk 0 (element offset, -1 = padding):
  // resolved once — the (image, row, column) of a halo row costs two integer divisions, which the
  // per-chunk staging paid again for every 64-channel chunk.  The halo image is < 2^31 elements.
  constexpr int kMaxHaloInstr = C3_MAX_HALO_ROWS / 32;
  int hofs[kMaxHaloInstr];
#pragma unroll
  for (int j = 0; j < kMaxHaloInstr; ++j) {
    hofs[j] = -1;
    const int piece = wid + 4 * j;
    const int h = piece * 8 + (lane >> 3);
    if (j < halo_instr && h < t.hr) {
      const int chunk = (lane & 7) ^ (h & 6);  // source-side swizzle (LDS-DMA writes lane-linearly)
      const int im = h / (t.hh * t.ww);
      const int rem = h - im * t.hh * t.ww;
      const int hy = rem / t.ww, hx = rem - hy * t.ww;
      const int n = img0 + im, iy = oy0 + hy - 1, ix = hx - 1;
      if (n < N && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
        hofs[j] = ((n * H + iy) * W + ix) * C + chunk * 8;
    }
  }
  const uint32_t halo_lds = lds_addr(halo) + (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
  auto stage_halo = [&](int kc) {
#pragma unroll
    for (int j = 0; j < kMaxHaloInstr; ++j) {
      if (j < halo_instr) {
        const void* src = hofs[j] >= 0 ? (const void*)(x + hofs[j] + kc * 64) : (const void*)ddl_zero_page;
        dma16(src, halo_lds + (uint32_t)(j * 4096));
      }
    }
  };
  auto stage_b = [&](int s, char* buf) {
    const int kc = s / 9, tap = s - kc * 9;
    B.dma(buf, tap * C + kc * 64, g, 0, 0, wid);
  };

  f32x4 acc[FR][RN];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int steps = (C / 64) * 9;
  stage_halo(0);
  stage_b(0, bring);
  for (int s = 0; s < steps; ++s) {
    const int kc = s / 9, tap = s - kc * 9;
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // halo chunk kc and weight tile s landed for every wave
    if (s + 1 < steps) stage_b(s + 1, bring + ((s + 1) % NB) * B_BYTES);
    const char* lb = bring + (s % NB) * B_BYTES;
    const int r = tap / 3, c3 = tap - r * 3;
    const int toff = r * t.ww + c3;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[FR], bfr[RN];
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = B.frag(lb, kk, j, wn0, lane);
#pragma unroll
      for (int i = 0; i < FR; ++i) {
        const int row = abase[i] + toff;
        const int ch = kk * 4 + (lane >> 4);
        af[i] = *reinterpret_cast<const bf16x8*>(halo + row * 128 + ((ch ^ (row & 6)) << 4));
      }
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);  // D^T (bf16 epilogue)
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    }
    if (NB == 2 || tap == 8) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done with weight tile s (and, at tap 8, the halo)
    }
    if (tap == 8 && s + 1 < steps) stage_halo(kc + 1);
  }

  gemm_epilogue<FR, RN, EPI>(p, acc, m0 + wm * (16 * FR), n0 + wn0, lane, bid, mend);
}

Conv3Tiling plan(const GemmParams& p) {
  const ConvGeom& g = p.g;
  Conv3Tiling t{};
  const int H = g.hi, W = g.wi;
  t.w = W;
  if (H * W <= 256) {
    t.rows = H;
    t.img = std::max(1, std::min(256 / (H * W), C3_MAX_HALO_ROWS / ((H + 2) * (W + 2))));
  } else {
    t.img = 1;
    t.rows = 0;
    for (int r = std::min(H, 256 / std::max(W, 1)); r >= 1; --r)
      if (H % r == 0 && (r + 2) * (W + 2) <= C3_MAX_HALO_ROWS) { t.rows = r; break; }
  }
  t.P = t.img * t.rows * t.w;
  t.hh = t.rows + 2;
  t.ww = W + 2;
  t.hr = t.img * t.hh * t.ww;
  t.hr_pad = (t.hr + 31) / 32 * 32;
  t.tiles_row = t.rows > 0 ? H / t.rows : 0;
  t.tiles_img = (g.n + t.img - 1) / t.img;
  return t;
}

template <int BN, int EPI, int NB, int FR, bool PRIO>
int launch_fr_p(const GemmParams& p, const Conv3Tiling& t, hipStream_t s) {
  const int blocks = t.tiles_img * t.tiles_row * ((p.N + BN - 1) / BN);
  const size_t lds = (size_t)t.hr_pad * 128 + NB * BN * BK * 2;
  static bool attr = [] {  // dynamic LDS above 64 KB must be allowed explicitly (at most 96 KB here)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_halo_kernel<BN, EPI, NB, FR, PRIO>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               C3_MAX_HALO_ROWS * 128 + NB * BN * BK * 2) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((conv3x3_halo_kernel<BN, EPI, NB, FR, PRIO>), dim3(blocks), dim3(NTHREADS), lds, s, p, t);
  return (int)hipGetLastError();
}

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && e[0] ? atoi(e) : dflt;
}

// DDL_CONV3X3_PRIO=1: raise the wave priority over the MFMA block (experiment knob)
template <int BN, int EPI, int NB, int FR>
int launch_fr(const GemmParams& p, const Conv3Tiling& t, hipStream_t s) {
  static const bool prio = env_int("DDL_CONV3X3_PRIO", 0) == 1;
  return prio ? launch_fr_p<BN, EPI, NB, FR, true>(p, t, s) : launch_fr_p<BN, EPI, NB, FR, false>(p, t, s);
}

// fragments per pixel wave: the fewest that cover half the tile (7 for the 196-pixel ResNet tiles)
template <int BN, int EPI, int NB>
int launch(const GemmParams& p, const Conv3Tiling& t, hipStream_t s) {
  static const bool fr_off = [] {  // DDL_CONV3X3_FR8=1: always 8 fragments (A/B knob)
    const char* e = getenv("DDL_CONV3X3_FR8");
    return e && e[0] == '1';
  }();
  if (!fr_off && t.P <= 2 * 16 * 7) return launch_fr<BN, EPI, NB, 7>(p, t, s);
  return launch_fr<BN, EPI, NB, 8>(p, t, s);
}

}  // namespace

// The halo kernel applies to this GEMM (host check; the Python side mirrors it in ops/conv.py).
bool conv3x3_halo_ok(const GemmParams& p) {
  const ConvGeom& g = p.g;
  if (p.a_mode != OP_KC_GATHER || p.b_mode != OP_KC || p.om.enabled || p.resid || p.aux || p.drop_thresh ||
      p.relu > ACT_RELU || p.k_split < p.K)
    return false;
  if (g.ntaps != 9 || g.sh != 1 || g.sw != 1 || g.hi != g.ho || g.wi != g.wo || g.c % 64 || g.c != g.tap_c ||
      p.N % 64 || p.K != 9 * g.c || p.ldc != p.N || p.ldb != p.K)
    return false;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      if (g.dh[r * 3 + c] != r - 1 || g.dw[r * 3 + c] != c - 1) return false;
  const Conv3Tiling t = plan(p);
  return t.rows > 0 && t.P >= 64 && t.hr <= C3_MAX_HALO_ROWS && p.M == g.n * g.hi * g.wi;
}

int launch_conv3x3(const GemmParams& p, int epi, hipStream_t s) {
  if (!conv3x3_halo_ok(p) || epi != EPI_BF16) return (int)hipErrorInvalidValue;
  const Conv3Tiling t = plan(p);
  // 64-channel tiles when 128 would leave the chip under-filled or the output has 64 channels
  const int tiles_px = t.tiles_img * t.tiles_row;
  static const int force_bn = [] {  // DDL_CONV3X3_BN=64|128: experiments
    const char* e = getenv("DDL_CONV3X3_BN");
    return e ? atoi(e) : 0;
  }();
  const bool bn128 = p.N % 128 == 0 && (force_bn ? force_bn == 128 : (long)tiles_px * (p.N / 128) >= 2L * 256);
  static const int nb128 = env_int("DDL_CONV3X3_NB", 2);  // 3: third weight slot (1 workgroup per CU)
  if (p.bnr_x) return bn128 ? launch<128, EPI_BF16_BNR, 2>(p, t, s) : launch<64, EPI_BF16_BNR, 3>(p, t, s);
  if (bn128) return nb128 == 3 ? launch<128, EPI_BF16_LITE, 3>(p, t, s) : launch<128, EPI_BF16_LITE, 2>(p, t, s);
  return launch<64, EPI_BF16_LITE, 3>(p, t, s);
}

}  // namespace ddl
