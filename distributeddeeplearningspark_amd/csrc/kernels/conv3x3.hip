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
#include "ddl_ops.h"

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
template <int BN, int EPI, int NB, int FR = 8>
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
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);  // D^T (bf16 epilogue)
    }
    if (NB == 2 || tap == 8) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done with weight tile s (and, at tap 8, the halo)
    }
    if (tap == 8 && s + 1 < steps) stage_halo(kc + 1);
  }

  gemm_epilogue<FR, RN, EPI>(p, acc, m0 + wm * (16 * FR), n0 + wn0, lane, bid, mend);
}

// max_px: pixels per tile (256 for the forward / data-gradient kernels; 224 for the weight gradient, whose
// ping-pong pair of 256-pixel tiles would not fit the LDS — the same tilings for every ResNet-50 stage)
Conv3Tiling plan(const GemmParams& p, int max_px = 256) {
  const ConvGeom& g = p.g;
  Conv3Tiling t{};
  const int H = g.hi, W = g.wi;
  t.w = W;
  if (H * W <= max_px) {
    t.rows = H;
    t.img = std::max(1, std::min(max_px / (H * W), C3_MAX_HALO_ROWS / ((H + 2) * (W + 2))));
  } else {
    t.img = 1;
    t.rows = 0;
    for (int r = std::min(H, max_px / std::max(W, 1)); r >= 1; --r)
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

template <int BN, int EPI, int NB, int FR>
int launch_fr(const GemmParams& p, const Conv3Tiling& t, hipStream_t s) {
  const int blocks = t.tiles_img * t.tiles_row * ((p.N + BN - 1) / BN);
  const size_t lds = (size_t)t.hr_pad * 128 + NB * BN * BK * 2;
  static bool attr = [] {  // dynamic LDS above 64 KB must be allowed explicitly (at most 96 KB here)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_halo_kernel<BN, EPI, NB, FR>),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               C3_MAX_HALO_ROWS * 128 + NB * BN * BK * 2) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((conv3x3_halo_kernel<BN, EPI, NB, FR>), dim3(blocks), dim3(NTHREADS), lds, s, p, t);
  return (int)hipGetLastError();
}

// fragments per pixel wave: the fewest that cover half the tile (7 for the 196-pixel ResNet tiles)
template <int BN, int EPI, int NB>
int launch(const GemmParams& p, const Conv3Tiling& t, hipStream_t s) {
  if (t.P <= 2 * 16 * 7) return launch_fr<BN, EPI, NB, 7>(p, t, s);
  return launch_fr<BN, EPI, NB, 8>(p, t, s);
}

// ------------------------------------------------------------------------------------------------
// 3x3 stride-1 pad-1 WEIGHT gradient with the input halo in LDS:
//   dW[co][tap][ci] += sum_p dy[p][co] * x[p + tap][ci]      (M = Co, N = 9 Ci, K = pixels)
// The gathered implicit GEMM (RC x RC_GATHER) re-fetches every input pixel once per tap and per
// 128-column tile and runs at 12-17 % MFMA (profiles/r2/pmc_conv3x3_halo_v2.txt: 56 % of wave time
// parked).  Here a workgroup owns a 64 co x 64 ci x 9 tap output block and walks pixel tiles (the
// forward kernel's row tiling, <= 256 pixels): per tile it stages dy [Ppad][64 co] (the RC image the
// GEMM kernels read with ds_read_b64_tr_b16) and the x halo once, and all nine taps read their B
// fragments from the halo at tap-shifted rows — 36 MFMAs per 40 transposed LDS reads per wave and
// 32-pixel step, no per-tap global traffic.  Waves: 2 (co) x 2 (ci), 32 x 32 x 9 taps each.
//
// Halo image CHUNK-major: [8 chunks of 8 channels][SC rows][16 B], SC = 64 G + 4 rows.  A transposed
// fragment read touches rows b + {0..3, 8..11} of two chunks; same-parity rows of one chunk fall on
// distinct banks and SC = 4 (mod 8) puts the second chunk on the other 32 banks, so the read is
// conflict-free with NO swizzle — which makes a tap shift a constant byte offset (toff * 16, an
// immediate of ds_read: WW is a template parameter) instead of per-read swizzle arithmetic.  The LDS-DMA
// fills 64 consecutive rows of one chunk per wave-instruction (G groups x 8 chunks); the 4 rows between
// chunk images are never written or read.
struct WgradArgs {
  const bf16_t* dy;  // [M][Co]
  const bf16_t* x;   // [N][H][W][Ci]
  float* out;        // SLAB: [splits][Co][9 Ci] partial slabs (plain stores); else [Co][9 Ci] (+= by atomics)
  int n, h, w, ci, co;
  int ntiles, tpb;   // pixel tiles and tiles per workgroup (blockIdx split s walks [s tpb, (s+1) tpb))
};

// One pixel tile of the weight-gradient product (both kernels below): KT 32-pixel steps x 9 taps x
// 2 x 2 MFMAs per wave, software-pipelined — the next tap's B fragments (and at tap 8 the next step's A
// fragments and tap-0 B fragments, whose halo rows were read one step ahead) are issued before the
// current tap's MFMAs, so a wave alone on its SIMD (the ping-pong kernel's computing half) does not
// stall on LDS latency at every tap or step boundary.
template <int WW, int SC, int KT>
__device__ __forceinline__ void wgrad_tile_mma(f32x4 (&acc)[9][2][2], const char* halo, const char* dyl,
                                               const int* hbt, const int (&ao)[2][2], const int boff, const int k1) {
  auto tr2 = [](const char* p1, const char* p2) {
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)p1);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)p2);
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
  };
  constexpr int JS = 2 * SC * 16;  // next 16-channel fragment: two chunks on
  auto bload = [&](int r1, int r2, int tap, bf16x8 (&bf)[2]) {
    const int toff = ((tap / 3) * WW + (tap % 3)) * 16;
    const char* b1 = halo + boff + r1 * 16 + toff;
    const char* b2 = halo + boff + r2 * 16 + toff;
    bf[0] = tr2(b1, b2);
    bf[1] = tr2(b1 + JS, b2 + JS);
  };
  // B fragments run TWO taps ahead of the MFMAs (a tap is only 4 MFMAs = 64 cycles, less than the
  // transposed reads' latency): slot t % 3 holds tap t, and 9 % 3 == 0 keeps the slots aligned across
  // steps; the next step's A fragments are read at tap 7
  int hb1 = hbt[k1], hb2 = hbt[k1 + 4];
  const int k1n = (KT > 1 ? 32 : 0) + k1;
  int nhb1 = hbt[k1n], nhb2 = hbt[k1n + 4];
  bf16x8 af[2], bs[3][2];
  af[0] = tr2(dyl + ao[0][0], dyl + ao[0][1]);
  af[1] = tr2(dyl + ao[1][0], dyl + ao[1][1]);
  bload(hb1, hb2, 0, bs[0]);
  bload(hb1, hb2, 1, bs[1]);
#pragma unroll 1
  for (int kk = 0; kk < KT; ++kk) {
    const int kn = kk + 1 < KT ? kk + 1 : kk;  // clamped: the last step re-reads its own rows
    const int kn2 = kk + 2 < KT ? kk + 2 : KT - 1;
    const int nnhb1 = hbt[kn2 * 32 + k1], nnhb2 = hbt[kn2 * 32 + k1 + 4];
    bf16x8 an[2];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 2 <= 8) bload(hb1, hb2, tap + 2, bs[(tap + 2) % 3]);
      else bload(nhb1, nhb2, tap - 7, bs[(tap + 2) % 3]);
      if (tap == 7) {
        const char* ab = dyl + kn * 4096;
        an[0] = tr2(ab + ao[0][0], ab + ao[0][1]);
        an[1] = tr2(ab + ao[1][0], ab + ao[1][1]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[tap][i][j] = mfma16x16x32(af[i], bs[tap % 3][j], acc[tap][i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    af[0] = an[0];
    af[1] = an[1];
    hb1 = nhb1;
    hb2 = nhb2;
    nhb1 = nnhb1;
    nhb2 = nnhb2;
  }
}

template <int G, int KT>
constexpr int wgrad_lds_bytes() { return 8 * (64 * G + 4) * 16 + KT * 32 * 128 + KT * 32 * 4; }

template <int WW, int G, int KT, bool SLAB>
__global__ __launch_bounds__(NTHREADS, 2) void conv3x3_wgrad_kernel(const WgradArgs a, const Conv3Tiling t) {
  constexpr int SC = 64 * G + 4;  // rows per chunk image
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* halo = smem;
  char* dyl = smem + 8 * SC * 16;
  int* hbt = reinterpret_cast<int*>(dyl + KT * 32 * 128);  // halo row of each tile pixel (tap (0, 0))
  const int ci_tiles = a.ci / 64;
  int bid, split;
  grid_tile(bid, split);
  const int tco = bid / ci_tiles, tci = bid - tco * ci_tiles;
  const int co0 = tco * 64, ci0 = tci * 64;
  const int tp_beg = split * a.tpb, tp_end = min(a.ntiles, tp_beg + a.tpb);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * 32, wn0 = (wid & 1) * 32;
  const int M = a.n * a.h * a.w;

  // tile-independent tables: the halo row of every tile pixel (pixels past the tile read row 0, finite
  // data, against zero dy rows), and this lane's halo rows (g * 64 + lane) decoded to (image, y, x)
  for (int px = threadIdx.x; px < KT * 32; px += NTHREADS) {
    int r = 0;
    if (px < t.P) {
      const int im = px / (t.rows * t.w);
      const int rem = px - im * t.rows * t.w;
      const int oy = rem / t.w, ox = rem - oy * t.w;
      r = im * t.hh * WW + oy * WW + ox;
    }
    hbt[px] = r;
  }
  int hcode[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int hrow = g * 64 + lane;
    hcode[g] = -1;
    if (hrow < t.hr) {
      const int im = hrow / (t.hh * WW);
      const int rem = hrow - im * t.hh * WW;
      const int hy = rem / WW, hx = rem - hy * WW;
      hcode[g] = (im << 20) | (hy << 10) | hx;
    }
  }
  __syncthreads();  // the pixel table is read by every wave
  const uint32_t halo_lds = lds_addr(halo);
  const uint32_t dy_lds = lds_addr(dyl) + (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;

  auto stage = [&](int tp) {
    const int timg = tp / t.tiles_row, trow = tp - timg * t.tiles_row;
    const int img0 = timg * t.img, oy0 = trow * t.rows;
    const int m0 = (img0 * a.h + oy0) * a.w;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int code = hcode[g];
      const int n = img0 + (code >> 20), iy = oy0 + ((code >> 10) & 1023) - 1, ix = (code & 1023) - 1;
      const bool ok = code >= 0 && n < a.n && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      const bf16_t* src = a.x + ((n * a.h + iy) * a.w + ix) * a.ci + ci0;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {  // this wave's chunks: wid and wid + 4
        const int c = wid + 4 * h2;
        dma16(ok ? (const void*)(src + c * 8) : (const void*)ddl_zero_page,
              halo_lds + (uint32_t)__builtin_amdgcn_readfirstlane(c * SC * 16 + g * 1024));
      }
    }
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int r = (wid + 4 * j) * 8 + (lane >> 3);
      const int m = m0 + r;
      const bool ok = r < t.P && m < M;
      const int chunk = (lane & 7) ^ (rc_swz<64>(r) << 1);
      const void* src = ok ? (const void*)(a.dy + (long)m * a.co + co0 + chunk * 8) : (const void*)ddl_zero_page;
      dma16(src, dy_lds + (uint32_t)(j * 4096));
    }
  };

  f32x4 acc[9][2][2];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment geometry (the RC fragment of ddl_gemm_kernel.h): k rows 8 (lane>>4) + q and + 4,
  // columns 4 (lane & 3) .. + 3 of each 16-wide fragment
  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int k1 = 8 * g4 + q;  // + 32 kk; rc_swz<64> of it does not depend on kk
  int ao[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int k = k1 + 4 * h2, col = wm0 + 16 * i + 4 * pq;
      ao[i][h2] = k * 128 + ((((col >> 3) ^ (rc_swz<64>(k) << 1))) << 4) + (col & 7) * 2;
    }
  // B: chunk (wn0 / 8 + 2 j + pq / 2), byte (pq & 1) * 8 of the row
  const int boff = ((wn0 >> 3) + (pq >> 1)) * (SC * 16) + (pq & 1) * 8;

  for (int tp = tp_beg; tp < tp_end; ++tp) {
    stage(tp);
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // this tile's dy and halo (and, first time, the pixel table) landed
    wgrad_tile_mma<WW, SC, KT>(acc, halo, dyl, hbt, ao, boff, k1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading this tile before the next one lands
  }

  // D orientation: acc[tap][i][j][e] = dW[co0 + wm0 + 16i + 4(lane>>4) + e][tap][ci0 + wn0 + 16j + (lane&15)]
  // -> each wave-instruction covers 4 rows x 64 contiguous bytes
  const long ldo = 9L * a.ci;
  float* out = a.out + (SLAB ? (long)split * a.co * ldo : 0L);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + wm0 + 16 * i + 4 * g4 + e;
          const int ci = ci0 + wn0 + 16 * j + (lane & 15);
          float* c = out + (long)co * ldo + tap * a.ci + ci;
          if constexpr (SLAB) *c = acc[tap][i][j][e];
          else atomicAdd(c, acc[tap][i][j][e]);
        }
}

// Ping-pong form: ONE 512-thread workgroup per CU, two halves of 4 waves with an LDS tile buffer each.
// Phases alternate: half A computes a pixel tile while half B's LDS-DMA of its next tile lands, then the
// roles swap (one workgroup barrier per phase) — the load latency hides under the other half's MFMAs
// within the workgroup, as the two co-resident workgroups of the kernel above do, but both halves
// accumulate the SAME 64 x 64 x 9 output block: they are merged through LDS at the end and the CU writes
// one partial slab (or one set of atomics) instead of two — half the split-K output traffic.
template <int G, int KT>
constexpr int wgrad_pp_lds_bytes() { return 2 * (8 * (64 * G + 4) * 16 + KT * 32 * 128) + KT * 32 * 4; }

template <int WW, int G, int KT, bool SLAB>
__global__ __launch_bounds__(512, 1) void conv3x3_wgrad_pp_kernel(const WgradArgs a, const Conv3Tiling t) {
  constexpr int SC = 64 * G + 4;
  constexpr int BUF = 8 * SC * 16 + KT * 32 * 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* hbt = reinterpret_cast<int*>(smem + 2 * BUF);
  const int ci_tiles = a.ci / 64;
  int bid, split;
  grid_tile(bid, split);
  const int tco = bid / ci_tiles, tci = bid - tco * ci_tiles;
  const int co0 = tco * 64, ci0 = tci * 64;
  const int tp_beg = split * a.tpb, tp_end = min(a.ntiles, tp_beg + a.tpb);
  const int nt = max(0, tp_end - tp_beg);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int grp = __builtin_amdgcn_readfirstlane(wid >> 2), w4 = wid & 3;
  const int wm0 = (w4 >> 1) * 32, wn0 = (w4 & 1) * 32;
  const int M = a.n * a.h * a.w;
  char* halo = smem + grp * BUF;
  char* dyl = halo + 8 * SC * 16;

  for (int px = threadIdx.x; px < KT * 32; px += 512) {
    int r = 0;
    if (px < t.P) {
      const int im = px / (t.rows * t.w);
      const int rem = px - im * t.rows * t.w;
      const int oy = rem / t.w, ox = rem - oy * t.w;
      r = im * t.hh * WW + oy * WW + ox;
    }
    hbt[px] = r;
  }
  int hcode[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int hrow = g * 64 + lane;
    hcode[g] = -1;
    if (hrow < t.hr) {
      const int im = hrow / (t.hh * WW);
      const int rem = hrow - im * t.hh * WW;
      const int hy = rem / WW, hx = rem - hy * WW;
      hcode[g] = (im << 20) | (hy << 10) | hx;
    }
  }
  const uint32_t halo_lds = lds_addr(halo);
  const uint32_t dy_lds = lds_addr(dyl) + (uint32_t)__builtin_amdgcn_readfirstlane(w4) * 1024u;
  auto stage = [&](int tp) {  // this half's 4 waves stage tile tp into its buffer
    const int timg = tp / t.tiles_row, trow = tp - timg * t.tiles_row;
    const int img0 = timg * t.img, oy0 = trow * t.rows;
    const int m0 = (img0 * a.h + oy0) * a.w;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int code = hcode[g];
      const int n = img0 + (code >> 20), iy = oy0 + ((code >> 10) & 1023) - 1, ix = (code & 1023) - 1;
      const bool ok = code >= 0 && n < a.n && (unsigned)iy < (unsigned)a.h && (unsigned)ix < (unsigned)a.w;
      const bf16_t* src = a.x + ((n * a.h + iy) * a.w + ix) * a.ci + ci0;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int c = w4 + 4 * h2;
        dma16(ok ? (const void*)(src + c * 8) : (const void*)ddl_zero_page,
              halo_lds + (uint32_t)__builtin_amdgcn_readfirstlane(c * SC * 16 + g * 1024));
      }
    }
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int r = (w4 + 4 * j) * 8 + (lane >> 3);
      const int m = m0 + r;
      const bool ok = r < t.P && m < M;
      const int chunk = (lane & 7) ^ (rc_swz<64>(r) << 1);
      const void* src = ok ? (const void*)(a.dy + (long)m * a.co + co0 + chunk * 8) : (const void*)ddl_zero_page;
      dma16(src, dy_lds + (uint32_t)(j * 4096));
    }
  };

  f32x4 acc[9][2][2];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[tp][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int k1 = 8 * g4 + q;
  int ao[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int k = k1 + 4 * h2, col = wm0 + 16 * i + 4 * pq;
      ao[i][h2] = k * 128 + ((((col >> 3) ^ (rc_swz<64>(k) << 1))) << 4) + (col & 7) * 2;
    }
  const int boff = ((wn0 >> 3) + (pq >> 1)) * (SC * 16) + (pq & 1) * 8;

  // phase ph: half (ph & 1) computes tile tp_beg + ph from its buffer while the other half's next tile
  // (staged right after the previous phase) lands; ONE call site of the tile body, uniform branches only
  if (grp < nt) stage(tp_beg + grp);
  if (grp == 0) wait_vmcnt<0>();
  __syncthreads();  // the pixel table, and half A's first tile
  for (int ph = 0; ph < nt; ++ph) {
    const bool mine = (ph & 1) == grp;
    if (mine) wgrad_tile_mma<WW, SC, KT>(acc, halo, dyl, hbt, ao, boff, k1);
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (mine && ph + 2 < nt) stage(tp_beg + ph + 2);  // this half's buffer is free again
  }
  wait_vmcnt<0>();

  // merge the halves through LDS (both tile buffers are free): entry e = tap*4 + 2i + j in four rounds of 9;
  // half B sends rounds 0-1 to half A, half A sends rounds 2-3 to half B; each then writes what it kept
  DDL_LDS f32x4* xm = (DDL_LDS f32x4*)(smem);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int sender = r < 2 ? 1 : 0;
    if (grp == sender) {
#pragma unroll
      for (int el = 0; el < 9; ++el) {
        const int e = 9 * r + el;
        xm[(el * 4 + w4) * 64 + lane] = acc[e >> 2][(e >> 1) & 1][e & 1];
      }
    }
    __syncthreads();
    if (grp != sender) {
#pragma unroll
      for (int el = 0; el < 9; ++el) {
        const int e = 9 * r + el;
        acc[e >> 2][(e >> 1) & 1][e & 1] += xm[(el * 4 + w4) * 64 + lane];
      }
    }
    __syncthreads();
  }

  const long ldo = 9L * a.ci;
  float* out = a.out + (SLAB ? (long)split * a.co * ldo : 0L);
#pragma unroll
  for (int e = 0; e < 36; ++e) {
    const int tap = e >> 2, i = (e >> 1) & 1, j = e & 1;
    if ((grp == 0) != (e < 18)) continue;  // half A wrote rounds 0-1 (entries 0..17)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int co = co0 + wm0 + 16 * i + 4 * g4 + v;
      const int ci = ci0 + wn0 + 16 * j + (lane & 15);
      float* c = out + (long)co * ldo + tap * a.ci + ci;
      if constexpr (SLAB) *c = acc[tap][i][j][v];
      else atomicAdd(c, acc[tap][i][j][v]);
    }
  }
}

// gw[i] += sum over the slabs of ws[s][i]: float4 per lane, the slabs split into groups of G whose
// partial sums are added atomically (one group when there are few slabs)
__global__ __launch_bounds__(256) void wgrad_slab_reduce_kernel(const float4* __restrict__ ws, float* __restrict__ gw,
                                                                long n4, int slabs, int per_group) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int s0 = blockIdx.y * per_group, s1 = min(slabs, s0 + per_group);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int s = s0;
  for (; s + 3 < s1; s += 4) {  // four slab loads in flight; adds in slab order (same bits)
    float4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = ws[(long)(s + q) * n4 + i];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      acc.x += v[q].x;
      acc.y += v[q].y;
      acc.z += v[q].z;
      acc.w += v[q].w;
    }
  }
  for (; s < s1; ++s) {
    const float4 v = ws[(long)s * n4 + i];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  float* o = gw + 4 * i;
  if (gridDim.y == 1) {
    float4 g = *reinterpret_cast<float4*>(o);
    g.x += acc.x;
    g.y += acc.y;
    g.z += acc.z;
    g.w += acc.w;
    *reinterpret_cast<float4*>(o) = g;
  } else {
    atomicAdd(o, acc.x);
    atomicAdd(o + 1, acc.y);
    atomicAdd(o + 2, acc.z);
    atomicAdd(o + 3, acc.w);
  }
}

template <int WW, int G, int KT, bool SLAB>
int launch_wgrad_v(const WgradArgs& a, const Conv3Tiling& t, dim3 grid, bool pp, hipStream_t s) {
  if (pp) {
    constexpr int lds = wgrad_pp_lds_bytes<G, KT>();
    static_assert(lds <= 160 * 1024, "one workgroup per CU");
    static bool attr = [] {
      return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_wgrad_pp_kernel<WW, G, KT, SLAB>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
    }();
    (void)attr;
    hipLaunchKernelGGL((conv3x3_wgrad_pp_kernel<WW, G, KT, SLAB>), grid, dim3(512), lds, s, a, t);
    return (int)hipGetLastError();
  }
  constexpr int lds = wgrad_lds_bytes<G, KT>();
  static_assert(lds <= 80 * 1024, "two workgroups per CU");
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&conv3x3_wgrad_kernel<WW, G, KT, SLAB>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL((conv3x3_wgrad_kernel<WW, G, KT, SLAB>), grid, dim3(NTHREADS), lds, s, a, t);
  return (int)hipGetLastError();
}

// Instantiated tilings (halo width WW, 64-row halo groups G, 32-pixel steps KT): the ResNet-50 stages at
// 224^2 (56, 28, 14 and 7 pixels wide; every one plans 196- or 224-pixel tiles) and VGG-16's 8 / 4 / 2
// pixel blocks.  Others take the GEMM path.
constexpr int kWgradPx = 224;

int wgrad_variant(const Conv3Tiling& t) {
  const int G = (t.hr + 63) / 64, KT = (t.P + 31) / 32;
  if (KT == 7) {
    if (t.ww == 58 && G == 6) return 0;
    if (t.ww == 30 && G == 5) return 1;
    if (t.ww == 16 && G == 4) return 2;
    if (t.ww == 9 && G == 6) return 3;
  }
  // VGG-16 (CIFAR, batch 256) blocks 3-5: 8x8 (3 images per tile), 4x4 (10), 2x2 (24) — whole images
  // per tile, the last tile partial (its missing images read zero halo rows against zero dy rows).  The
  // 32x32 / 16x16 blocks take 128-pixel row tiles (kWgradPx: 256-pixel tiles would need 166 KB of LDS for
  // the ping-pong pair).
  if (KT == 4 && t.ww == 34 && G == 4) return 7;  // 32x32: 4 rows per tile
  if (KT == 4 && t.ww == 18 && G == 3) return 8;  // 16x16: 8 rows per tile
  if (KT == 6 && t.ww == 10 && G == 5) return 4;
  if (KT == 5 && t.ww == 6 && G == 6) return 5;
  if (KT == 3 && t.ww == 4 && G == 6) return 6;
  return -1;
}

template <bool SLAB>
int launch_wgrad(const WgradArgs& a, const Conv3Tiling& t, dim3 grid, bool pp, hipStream_t s) {
  switch (wgrad_variant(t)) {
    case 0: return launch_wgrad_v<58, 6, 7, SLAB>(a, t, grid, pp, s);
    case 1: return launch_wgrad_v<30, 5, 7, SLAB>(a, t, grid, pp, s);
    case 2: return launch_wgrad_v<16, 4, 7, SLAB>(a, t, grid, pp, s);
    case 3: return launch_wgrad_v<9, 6, 7, SLAB>(a, t, grid, pp, s);
    case 4: return launch_wgrad_v<10, 5, 6, SLAB>(a, t, grid, pp, s);
    case 5: return launch_wgrad_v<6, 6, 5, SLAB>(a, t, grid, pp, s);
    case 6: return launch_wgrad_v<4, 6, 3, SLAB>(a, t, grid, pp, s);
    case 7: return launch_wgrad_v<34, 4, 4, SLAB>(a, t, grid, pp, s);
    case 8: return launch_wgrad_v<18, 3, 4, SLAB>(a, t, grid, pp, s);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace

// Plan of the 3x3 weight-gradient halo kernel: tiles, splits and the slab workspace size (floats;
// 0 = atomics).  blocks_per_cu: workgroups the split aims for per CU (the kernel fits 2).
bool conv3x3_wgrad_ok(int n, int h, int w, int ci, int co) {
  if (ci % 64 || co % 64 || n <= 0 || (long)n * h * w * std::max(ci, co) >= (1L << 31)) return false;
  GemmParams p{};
  p.g.n = n;
  p.g.hi = h;
  p.g.wi = w;
  const Conv3Tiling t = plan(p, kWgradPx);
  return t.rows > 0 && t.P >= 64 && t.P <= 256 && t.hr <= C3_MAX_HALO_ROWS && wgrad_variant(t) >= 0;
}

void conv3x3_wgrad_plan(int n, int h, int w, int ci, int co, int blocks_per_cu, int cus, int& splits, int& tpb,
                        int& ntiles) {
  GemmParams p{};
  p.g.n = n;
  p.g.hi = h;
  p.g.wi = w;
  const Conv3Tiling t = plan(p, kWgradPx);
  ntiles = t.tiles_img * t.tiles_row;
  const int pairs = (co / 64) * (ci / 64);
  const int want = std::max(1, (blocks_per_cu * cus + pairs - 1) / pairs);
  tpb = std::max(1, (ntiles + std::min(want, ntiles) - 1) / std::min(want, ntiles));
  splits = (ntiles + tpb - 1) / tpb;
}

int launch_conv3x3_wgrad(const bf16_t* dy, const bf16_t* x, float* gw, float* ws, int n, int h, int w, int ci, int co,
                         int splits, int tpb, bool pp, void* stream) {
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GemmParams p{};
  p.g.n = n;
  p.g.hi = h;
  p.g.wi = w;
  const Conv3Tiling t = plan(p, kWgradPx);
  WgradArgs a{dy, x, ws ? ws : gw, n, h, w, ci, co, t.tiles_img * t.tiles_row, tpb};
  const dim3 grid((co / 64) * (ci / 64), splits);
  int rc = ws ? launch_wgrad<true>(a, t, grid, pp, s) : launch_wgrad<false>(a, t, grid, pp, s);
  if (rc || !ws) return rc;
  const long n4 = (long)co * 9 * ci / 4;
  // deterministic mode: every slab of an element summed by one lane in split order (no atomics)
  const int per_group = (n4 >= 65536 || deterministic()) ? splits : 16;  // enough workgroups either way
  const dim3 rgrid((unsigned)((n4 + 255) / 256), (unsigned)((splits + per_group - 1) / per_group));
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, rgrid, dim3(256), 0, s, reinterpret_cast<const float4*>(ws), gw, n4,
                     splits, per_group);
  return (int)hipGetLastError();
}

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
  const bool bn128 = p.N % 128 == 0 && (long)tiles_px * (p.N / 128) >= 2L * 256;
  if (p.bnr_x) return bn128 ? launch<128, EPI_BF16_BNR, 2>(p, t, s) : launch<64, EPI_BF16_BNR, 3>(p, t, s);
  if (bn128) return launch<128, EPI_BF16_LITE, 2>(p, t, s);
  return launch<64, EPI_BF16_LITE, 3>(p, t, s);
}

}  // namespace ddl
