// Four-wave MFMA GEMM with 128-row wave tiles for gfx950 (plain KC / RC operands, K % 64 == 0).
//
// Why: the 128x128 kernels give each wave a 64x64 tile, so every 16 MFMAs of a 32-deep k-step read
// 8 KB of fragments from LDS and the block re-stages 32 KB per 64-deep K-tile; four such blocks per
// CU keep the LDS array ~75 % busy for the MFMA time and hide the HBM latency only through
// co-resident blocks (rocprof: 36 % MFMA busy, 50 % wait on BERT FFN1).  Here one 256-thread
// workgroup per CU owns a 256 x BN output tile and each wave a 128 x BN/2 tile (8 x BN/32 MFMA
// blocks: 256 accumulators, held in AGPRs, at BN = 256):
//   * per 32-deep k-step a wave reads 16 fragments (16 KB) for 64 MFMAs, half the LDS bytes per
//     MFMA of the 64x64 wave tile, and the DMA bytes per MFMA halve with the 256-wide block;
//   * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip) into a
//     ring of K-tile stages (BN 256: 2 x 64 KB, BN 128: 3 x 48 KB) with one barrier per K-tile;
//     a K-tile of MFMAs (2048 / 1024 cycles per wave) covers each fetch (two at BN 128);
//   * the 128-row half-tile images, swizzles and fragment readers are the 256x256 kernel's
//     (ddl_gemm256.h): ds_read_b128 for K-contiguous operands, ds_read_b64_tr_b16 for
//     row-contiguous ones, conflict-free.
// Epilogue: the shared gemm_epilogue on the 8 x BN/32 fragment array of each wave — the slim one (bias /
// ReLU / BN statistics), the LDS-staged row epilogue for everything else (GELU / dropout / residual),
// fp32 stores, split-K partial slabs or atomics.
#pragma once
#include "ddl_gemm256.h"

namespace ddl {
namespace w4 {

constexpr int THREADS = 256;
constexpr int HALF = 128 * 64 * 2;  // bytes of one half-tile slot (128 rows x 64 k)

// Stage rows [r0, r0 + 128) x k [k0, k0 + 64) of an operand into one 16-KB slot: 16 1-KB blocks,
// 4 LDS-DMA wave-instructions per wave (the 256x256 kernel's image, written by 4 waves instead of 8).
template <int MODE>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ ptr, long ld, int rows, int r0, int k0, char* slot,
                                      int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int blk = i * 4 + wid;
    const bf16_t* src;
    if constexpr (MODE == OP_KC) {  // block = 8 rows x 128 B
      const int row = blk * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      const int gr = min(r0 + row, rows - 1);  // rows past the end: any valid row (outputs discarded)
      src = ptr + (long)gr * ld + k0 + ch * 8;
    } else {  // RC: block = 4 k-rows x 256 B (128 columns)
      const int k = blk * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ g256::rc_sw(k);
      const int gc = min(r0 + ch * 8, rows - 8);
      src = (ptr + (long)k0 * ld) + ((long)k * ld + gc);  // the second term is K-tile invariant (hoisted)
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (g256::lds_t*)(slot + blk * 1024), 16, 0, 0);
  }
}

template <int BN>
constexpr int stages() { return BN == 256 ? 2 : 3; }
template <int BN>
constexpr int lds_bytes() { return stages<BN>() * (2 + BN / 128) * HALF; }

}  // namespace w4

template <int BN, int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(w4::THREADS, 1) void gemm_w4_kernel(const GemmParams p) {
  using namespace w4;
  static_assert(BN == 256 || BN == 128, "w4: 256x256 or 256x128 tiles");
  constexpr int NB = BN / 128;      // B half-tiles per stage
  constexpr int SLOTS = 2 + NB;     // half-tiles per stage
  constexpr int ST = stages<BN>();  // ring depth
  constexpr int RN = BN / 32;       // 16-column fragments per wave
  constexpr int PER = SLOTS * 4;    // LDS-DMA wave-instructions per wave per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tiles_n = (p.N + BN - 1) / BN;
  int bid, split;
  grid_tile(bid, split);
  int tm, tn;
  tile_raster<256>(p, bid, tiles_n, tm, tn);
  const int m0 = tm * 256, n0 = tn * BN;
  const int kbeg = split * p.k_split;
  const int nk = (min(p.K, kbeg + p.k_split) - kbeg) >> 6;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b);

  auto slot = [&](int st, int h) -> char* { return smem + (st * SLOTS + h) * HALF; };
  auto stage_tile = [&](int t, int st) {
    const int k0 = kbeg + t * 64;
    stage<AMODE>(A, p.lda, p.M, m0, k0, slot(st, 0), wid, lane);
    stage<AMODE>(A, p.lda, p.M, m0 + 128, k0, slot(st, 1), wid, lane);
    stage<BMODE>(B, p.ldb, p.N, n0, k0, slot(st, 2), wid, lane);
    if constexpr (NB == 2) stage<BMODE>(B, p.ldb, p.N, n0 + 128, k0, slot(st, 3), wid, lane);
  };
  const int bh = NB == 2 ? 2 + wc : 2;   // this wave's B half-tile
  const int bc = NB == 2 ? 0 : 64 * wc;  // its first column inside that half

  f32x4 acc[8][RN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one 32-deep k-step: A rows 16i of the wave's A half, B columns bc + 16j
  auto frags = [&](int st, int kk, bf16x8 (&af)[8], bf16x8 (&bfr)[RN]) {
    const char* sa = slot(st, wr);
    const char* sb = slot(st, bh);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = g256::frag<AMODE>(sa, 16 * i, kk, lane);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = g256::frag<BMODE>(sb, bc + 16 * j, kk, lane);
  };
  auto mma = [&](const bf16x8 (&af)[8], const bf16x8 (&bfr)[RN]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if constexpr (epi_dt(EPI))
          acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);
        else
          acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
  };
  // Ring of ST stages, one barrier per K-tile at its start: tile t has landed for this wave (tile
  // t + 1 may stay in flight at ST = 3), the barrier publishes it to every wave and proves every wave
  // is done with tile t - 1, whose slot is refilled with tile t + ST - 1 right away.  (Double-buffering
  // the fragments across K-tiles makes the compiler rotate the accumulators through VGPRs every
  // iteration — 190 extra moves per 64 MFMAs at BN 128 — so the k-steps read their fragments in place.)
#pragma unroll
  for (int s = 0; s < ST - 1; ++s)
    if (s < nk) stage_tile(s, s);
  int cur = 0;
  for (int t = 0; t < nk; ++t) {
    if (ST >= 3 && t + 1 < nk) wait_vmcnt<PER>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + ST - 1 < nk) stage_tile(t + ST - 1, cur == 0 ? ST - 1 : cur - 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[8], bfr[RN];
      frags(cur, kk, af, bfr);
      mma(af, bfr);
    }
    cur = cur + 1 == ST ? 0 : cur + 1;
  }
  if constexpr (EPI == EPI_BF16_ROW) __syncthreads();  // the ring becomes the row epilogue's staging area
  static_assert(EPI != EPI_BF16, "w4: the full bf16 epilogue runs as EPI_BF16_ROW (on the 8 x RN array the "
                                 "unrolled one spills ~260 dwords per lane)");
  gemm_epilogue<8, RN, EPI>(p, acc, m0 + 128 * wr, n0 + (BN / 2) * wc, lane, bid, -1,
                            reinterpret_cast<float*>(smem + wid * row_epi_bytes<RN>()), (long)split * p.split_stride);
}

template <int BN, int AMODE, int BMODE, int EPI>
inline int launch_w4(const GemmParams& p, hipStream_t s) {
  constexpr int lds = w4::lds_bytes<BN>();
  static const bool attr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_w4_kernel<BN, AMODE, BMODE, EPI>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
  if (!attr) return (int)hipErrorInvalidValue;
  const int tiles = ((p.M + 255) / 256) * ((p.N + BN - 1) / BN);
  const int splits = (p.K + p.k_split - 1) / p.k_split;
  hipLaunchKernelGGL((gemm_w4_kernel<BN, AMODE, BMODE, EPI>), dim3(tiles, splits), dim3(w4::THREADS), lds, s, p);
  return (int)hipGetLastError();
}

}  // namespace ddl
