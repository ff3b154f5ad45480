// Persistent ping-pong MFMA GEMM for gfx950: one 512-thread workgroup per CU walks a list of
// 256 x BN output tiles (plain K-contiguous operands, K % 64 == 0).
//
//   * 8 waves = 2 ping-pong groups of 4 (waves 0-3 / 4-7: every SIMD holds one wave of each).  Group 1
//     runs one barrier behind group 0, so while one group issues its MFMA burst the other issues its
//     fragment reads and LDS-DMA staging (s_setprio(1) around the bursts).
//   * The K loop is cut into k-halves (32 deep).  A phase = one k-half: read the wave's A / B fragments of
//     the k-half (ds_read_b128), stage a later k-half, barrier, one MFMA burst, barrier.
//   * LDS holds a ring of 4 k-half slots ([256 A rows | BN B rows] x 64 B, the 16-B chunks of a row XOR-
//     swizzled by a 2-bit function of (row >> 2) so every ds_read_b128 lane group hits 16 distinct bank
//     slots).  The staging stream runs across tile boundaries: the k-halves of a CU's next tile are in
//     flight while it finishes and writes back the current one, so a tile costs no prologue.  Slot
//     (p + 3) % 4 is refilled in phase p, one phase after its last read (every wave retires its fragment
//     reads with lgkmcnt(0) before the phase's first barrier), and waited for with a counted vmcnt in
//     phase p + 2 (two k-halves stay in flight across every barrier).
//   * Tiles: min(tiles, CUs) persistent workgroups; workgroup b takes tiles r * G + xcd_remap(b), so the
//     tiles in flight on one XCD are a contiguous block of the grouped raster (tile_raster, group_m) and
//     share A rows / B rows in that XCD's L2.
// Epilogue: the shared gemm_epilogue (bias / GELU / dropout / residual / ReLU / BN statistics) on the
// wave's (256 / WM) x (BN / (8 / WM)) D^T accumulators, right after the tile's last burst.
#pragma once
#include "ddl_gemm_kernel.h"

namespace ddl {
namespace gpp {

constexpr int THREADS = 512;
constexpr int RING = 4;

// 2-bit chunk swizzle of a 64-B LDS row: g[(row >> 2) & 3] with g = {0, 2, 3, 1}
__device__ __forceinline__ int kh_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

template <int BN>
struct Geo {
  static constexpr int A_BYTES = 256 * 64;  // 256 rows x 32 k x 2 B
  static constexpr int B_BYTES = BN * 64;
  static constexpr int SLOT = A_BYTES + B_BYTES;
  static constexpr int GA = 256 / 16 / 8;  // 1-KB LDS-DMA wave-instructions per wave per k-half
  static constexpr int GB = BN / 16 / 8;
  static constexpr int G = GA + GB;
  static_assert(BN % 128 == 0, "BN: multiple of 128 (whole DMA blocks per wave)");
};

// Stage rows [r0, r0 + R) x k [k0, k0 + 32) of a KC operand into the slot at LDS byte address `lds`:
// R / 16 1-KB blocks, block blk = 16 rows x 64 B written lane-linearly; the swizzle is applied to the
// global source (lane -> row blk * 16 + lane / 4, LDS chunk lane % 4 holds k-chunk (lane % 4) ^ swz).
// Rows past the end read the last row (their outputs are never stored).
template <int R, int NW = 8>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ ptr, long ld, int rows, int r0, int k0, uint32_t lds,
                                      int wid, int lane) {
#pragma unroll
  for (int i = 0; i < R / 16 / NW; ++i) {
    const int blk = i * NW + wid;
    const int row = blk * 16 + (lane >> 2);
    const int c = (lane & 3) ^ kh_swz(row);
    const int gr = min(r0 + row, rows - 1);
    dma16(ptr + (long)gr * ld + k0 + c * 8, lds + (uint32_t)blk * 1024u);
  }
}

// The epilogue over the wave's RM x RN accumulator fragments in EM x EN chunks (the full epilogue's
// GELU / residual / dropout state per fragment spills when applied to all 8 x 4 fragments at once).
// Compile-time recursion, so every accumulator index stays static (a runtime-indexed chunk loop that
// the unroller gives up on puts the whole accumulator array in scratch).
template <int RM, int RN, int EPI, int I0, int J0>
__device__ __forceinline__ void epilogue_chunks(const GemmParams& p, f32x4 (&acc)[RM][RN], int mb, int nb, int lane,
                                                int bid) {
  constexpr bool FULL = EPI == EPI_BF16 || EPI == EPI_BF16_BNR;
  constexpr int EM = FULL && RM > 2 ? 2 : RM, EN = FULL && RN > 2 ? 2 : RN;
  f32x4 sub[EM][EN];
#pragma unroll
  for (int i = 0; i < EM; ++i)
#pragma unroll
    for (int j = 0; j < EN; ++j) sub[i][j] = acc[I0 + i][J0 + j];
  gemm_epilogue<EM, EN, EPI>(p, sub, mb + 16 * I0, nb + 16 * J0, lane, bid);
  if constexpr (J0 + EN < RN) epilogue_chunks<RM, RN, EPI, I0, J0 + EN>(p, acc, mb, nb, lane, bid);
  else if constexpr (I0 + EM < RM) epilogue_chunks<RM, RN, EPI, I0 + EM, 0>(p, acc, mb, nb, lane, bid);
}

}  // namespace gpp

// WM: waves along M (2: 128-row wave tiles, 4: 64-row wave tiles); the other 8 / WM waves split BN.
template <int BN, int WM, int EPI, int RING = 4>
__global__ __launch_bounds__(gpp::THREADS, 1) void gemm_pp_kernel(const GemmParams p, const int tiles) {
  constexpr int AHEAD = RING - 1;  // k-halves staged ahead of the one being read
  using Gm = gpp::Geo<BN>;
  constexpr int WN = 8 / WM;
  constexpr int TM = 256 / WM, TN = BN / WN;  // per-wave output tile
  constexpr int RM = TM / 16, RN = TN / 16;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(1024))) char smem[RING * Gm::SLOT];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wid >> 2;  // ping-pong group
  const int wm = wid / WN, wn = wid % WN;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b);
  const uint32_t lds0 = lds_addr(smem);
  const int tiles_n = (p.N + BN - 1) / BN;
  const int G = gridDim.x;
  const int order = xcd_remap(blockIdx.x, G);
  const int my_tiles = tiles > order ? (tiles - order + G - 1) / G : 0;
  const int nkh = p.K >> 5;
  const int P = my_tiles * nkh;  // phases (k-halves) of this workgroup

  // staging cursor (wave-uniform): k-half sh of my tile sr at (sm0, sn0)
  int sr = 0, sh = 0, sm0 = 0, sn0 = 0;
  auto tile_origin = [&](int r, int& m0, int& n0) __attribute__((always_inline)) {
    int tm, tn;
    tile_raster<256>(p, r * G + order, tiles_n, tm, tn);
    m0 = tm * 256;
    n0 = tn * BN;
  };
  if (P > 0) tile_origin(0, sm0, sn0);
  auto stage_next = [&](int q) __attribute__((always_inline)) {  // stage k-half q (== the cursor) into slot q % 4, advance the cursor
    const uint32_t slot = lds0 + (uint32_t)((q % RING) * Gm::SLOT);
    gpp::stage<256>(A, p.lda, p.M, sm0, sh * 32, slot, wid, lane);
    gpp::stage<BN>(B, p.ldb, p.N, sn0, sh * 32, slot + Gm::A_BYTES, wid, lane);
    if (++sh == nkh) {
      sh = 0;
      if (++sr < my_tiles) tile_origin(sr, sm0, sn0);
    }
  };

  // per-lane fragment offset inside a 16-row block (row lane & 15, k-chunk lane >> 4, swizzled)
  const int fofs = (lane & 15) * 64 + (((lane >> 4) ^ gpp::kh_swz(lane & 15)) << 4);
  const char* abase = smem + (wm * TM) * 64 + fofs;
  const char* bbase = smem + Gm::A_BYTES + (wn * TN) * 64 + fofs;

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto wait_ahead = [&](int n) __attribute__((always_inline)) {  // <= n staged k-halves still in flight
    if (n >= 3 && AHEAD >= 4) wait_vmcnt<3 * Gm::G>();
    else if (n >= 2) wait_vmcnt<2 * Gm::G>();
    else if (n == 1) wait_vmcnt<Gm::G>();
    else wait_vmcnt<0>();
  };
  // prologue: k-halves 0 .. AHEAD-1 in flight; k-half 0 landed everywhere before the first reads
  for (int q = 0; q < AHEAD && q < P; ++q) stage_next(q);
  wait_ahead(min(P, AHEAD) - 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

  int cr = 0, ch = 0;  // compute cursor: k-half ch of my tile cr
  int cm0 = 0, cn0 = 0;
  if (P > 0) tile_origin(0, cm0, cn0);
  for (int ph = 0; ph < P; ++ph) {
    const int so = (ph % RING) * Gm::SLOT;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(abase + so + i * 1024);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bbase + so + j * 1024);
    if (ph + AHEAD < P) stage_next(ph + AHEAD);
    // k-half ph + 1 must have landed before the NEXT phase's reads: the k-halves staged after it
    // (ph + 2 .. ph + AHEAD) may stay in flight
    wait_ahead(min(P - 1, ph + AHEAD) - (ph + 1));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if constexpr (epi_dt(EPI)) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);
        else acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (++ch == nkh) {  // tile done: write it back, start the next one
      gpp::epilogue_chunks<RM, RN, EPI, 0, 0>(p, acc, cm0 + wm * TM, cn0 + wn * TN, lane, cr * G + order);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ch = 0;
      if (++cr < my_tiles) tile_origin(cr, cm0, cn0);
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the groups
}

template <int BN, int WM, int EPI, int RING = 4>
inline int launch_pp(const GemmParams& p, hipStream_t s, int max_wg = 0) {
  const int tiles = ((p.M + 255) / 256) * ((p.N + BN - 1) / BN);
  int wg = max_wg > 0 ? max_wg : device_cus();
  if (tiles < wg) wg = tiles;
  hipLaunchKernelGGL((gemm_pp_kernel<BN, WM, EPI, RING>), dim3(wg), dim3(gpp::THREADS), 0, s, p, tiles);
  return (int)hipGetLastError();
}

// Two workgroups per CU: 256 threads (4 waves, 2 x 2), a 256 x BN tile per workgroup, a 3-slot k-half ring
// with ONE barrier per k-half; co-resident workgroups (not wave groups) overlap each other's epilogues.
template <int BN, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_d2_kernel(const GemmParams p) {
  using Gm = gpp::Geo<BN>;
  constexpr int TM = 128, TN = BN / 2, RM = TM / 16, RN = TN / 16;
  constexpr int GA = 256 / 16 / 4, GB = BN / 16 / 4, G = GA + GB;
  __shared__ __attribute__((aligned(1024))) char smem[3 * Gm::SLOT];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b);
  const uint32_t lds0 = lds_addr(smem);
  int bid, split;
  grid_tile(bid, split);
  int tm, tn;
  tile_raster<256>(p, bid, (p.N + BN - 1) / BN, tm, tn);
  const int m0 = tm * 256, n0 = tn * BN;
  const int nkh = p.K >> 5;
  auto stage = [&](int q) __attribute__((always_inline)) {
    const uint32_t slot = lds0 + (uint32_t)((q % 3) * Gm::SLOT);
    gpp::stage<256, 4>(A, p.lda, p.M, m0, q * 32, slot, wid, lane);
    gpp::stage<BN, 4>(B, p.ldb, p.N, n0, q * 32, slot + Gm::A_BYTES, wid, lane);
  };
  const int fofs = (lane & 15) * 64 + (((lane >> 4) ^ gpp::kh_swz(lane & 15)) << 4);
  const char* abase = smem + (wm * TM) * 64 + fofs;
  const char* bbase = smem + Gm::A_BYTES + (wn * TN) * 64 + fofs;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage(0);
  if (nkh > 1) stage(1);
  for (int ph = 0; ph < nkh; ++ph) {
    if (ph + 1 < nkh) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // k-half ph visible; every wave is done with slot (ph + 2) % 3
    if (ph + 2 < nkh) stage(ph + 2);
    const int so = (ph % 3) * Gm::SLOT;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(abase + so + i * 1024);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bbase + so + j * 1024);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if constexpr (epi_dt(EPI)) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);
        else acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
  }
  gpp::epilogue_chunks<RM, RN, EPI, 0, 0>(p, acc, m0 + wm * TM, n0 + wn * TN, lane, bid);
}

template <int BN, int EPI>
inline int launch_d2(const GemmParams& p, hipStream_t s) {
  const int tiles = ((p.M + 255) / 256) * ((p.N + BN - 1) / BN);
  hipLaunchKernelGGL((gemm_d2_kernel<BN, EPI>), dim3(tiles), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

// 128 x 128 tile, 4 waves of 64 x 64, four workgroups per CU (the production tile's occupancy), with a
// 2-slot k-half ring: ONE barrier per k-half, and k-half p + 1 streams in while the workgroup computes p
// (the single-stage kernel exposes each K-tile's load to the workgroup and relies on its co-resident
// neighbours to cover it).
template <int EPI>
__global__ __launch_bounds__(256, 4) void gemm_kh_kernel(const GemmParams p) {
  constexpr int BM = 128, BN = 128, A_BYTES = BM * 64, SLOT = (BM + BN) * 64;
  constexpr int TM = 64, TN = 64, RM = 4, RN = 4;
  __shared__ __attribute__((aligned(1024))) char smem[2 * SLOT];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b);
  const uint32_t lds0 = lds_addr(smem);
  int bid, split;
  grid_tile(bid, split);
  int tm, tn;
  tile_raster<BM>(p, bid, (p.N + BN - 1) / BN, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkh = p.K >> 5;
  auto stage = [&](int q) __attribute__((always_inline)) {
    const uint32_t slot = lds0 + (uint32_t)((q & 1) * SLOT);
    gpp::stage<BM, 4>(A, p.lda, p.M, m0, q * 32, slot, wid, lane);
    gpp::stage<BN, 4>(B, p.ldb, p.N, n0, q * 32, slot + A_BYTES, wid, lane);
  };
  const int fofs = (lane & 15) * 64 + (((lane >> 4) ^ gpp::kh_swz(lane & 15)) << 4);
  const char* abase = smem + (wm * TM) * 64 + fofs;
  const char* bbase = smem + A_BYTES + (wn * TN) * 64 + fofs;
  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage(0);
  for (int ph = 0; ph < nkh; ++ph) {
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // k-half ph visible; every wave is done with the other slot
    if (ph + 1 < nkh) stage(ph + 1);
    const int so = (ph & 1) * SLOT;
    bf16x8 af[RM], bfr[RN];
#pragma unroll
    for (int i = 0; i < RM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(abase + so + i * 1024);
#pragma unroll
    for (int j = 0; j < RN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(bbase + so + j * 1024);
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        if constexpr (epi_dt(EPI)) acc[i][j] = mfma16x16x32(bfr[j], af[i], acc[i][j]);
        else acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
  }
  gpp::epilogue_chunks<RM, RN, EPI, 0, 0>(p, acc, m0 + wm * TM, n0 + wn * TN, lane, bid);
}

template <int EPI>
inline int launch_kh(const GemmParams& p, hipStream_t s) {
  const int tiles = ((p.M + 127) / 128) * ((p.N + 127) / 128);
  hipLaunchKernelGGL((gemm_kh_kernel<EPI>), dim3(tiles), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ddl
