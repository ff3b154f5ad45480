// 256x256 ping-pong MFMA GEMM for gfx950 (plain KC / RC operands, K % 64 == 0).
//
// Structure (one 512-thread workgroup per CU, 2 waves per SIMD):
//   * 8 waves = 2 groups of 4 (wr = 0 / 1).  Group 1 runs one barrier behind group 0, so on
//     every SIMD one wave issues MFMAs while its partner issues LDS reads and LDS-DMA
//     staging — the matrix pipe stays fed without a register-hungry software pipeline.
//   * A K-tile (64 deep) is processed in 4 phases, one 128x128 quadrant of the 256x256 tile
//     per phase, quadrant order (0,0) (0,1) (1,1) (1,0) so each phase reloads only one of the
//     two fragment sets: per wave 64x32 outputs x K=64 = 16 v_mfma_f32_16x16x32_bf16 per phase.
//   * Operands are staged global -> LDS with global_load_lds_dwordx4 (LDS-DMA, no VGPR round
//     trip) in 16-KB half-tiles (128 rows x 64 k), one half-tile per phase, into an 8-slot ring
//     (2 K-tiles, 128 KB).  Each slot is refilled (for the tile two ahead) one phase after its
//     last read, so loads have 4-7 phases of latency cover; one counted s_waitcnt vmcnt(6) per
//     K-tile retires the next tile with three half-tiles still in flight.  Swizzles are applied
//     to the GLOBAL source address (LDS-DMA writes lane-linearly) and undone by the reads.
//   * KC operands (K-contiguous rows) are read with ds_read_b128; RC operands (row-contiguous,
//     i.e. the transposed operand of dgrad / wgrad) with ds_read_b64_tr_b16.
// Epilogue: the shared gemm_epilogue (bias / GELU / dropout / residual / ReLU / BN statistics,
// fp32 store or split-K atomics), called once per quadrant.
#pragma once
#include "ddl_gemm_kernel.h"

namespace ddl {
namespace g256 {

constexpr int THREADS = 512;
constexpr int HALF = 128 * 64 * 2;  // bytes of one half-tile slot
typedef __attribute__((address_space(3))) void lds_t;

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4); }
__device__ __forceinline__ int rc_sw(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 1; }
__device__ __forceinline__ int rc_off(int k, int col) {
  return k * 256 + (((col >> 3) ^ rc_sw(k)) << 4) + (col & 7) * 2;
}

// Stage rows [r0, r0 + 128) x k [k0, k0 + 64) of an operand into one 16-KB slot (2 LDS-DMA per lane).
template <int MODE>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ ptr, long ld, int rows, int r0, int k0, char* slot,
                                      int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = i * 8 + wid;  // 1-KB block of the slot written by this wave-instruction
    const bf16_t* src;
    if constexpr (MODE == OP_KC) {  // block = 8 rows x 128 B
      const int row = blk * 8 + (lane >> 3);
      const int ch = (lane & 7) ^ ((row >> 1) & 7);
      const int gr = min(r0 + row, rows - 1);  // rows past the end: any valid row (outputs discarded)
      src = ptr + (long)gr * ld + k0 + ch * 8;
    } else {  // RC: block = 4 k-rows x 256 B (128 columns)
      const int k = blk * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ rc_sw(k);
      const int gc = min(r0 + ch * 8, rows - 8);
      src = ptr + (long)(k0 + k) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_t*)(slot + blk * 1024), 16, 0, 0);
  }
}

// MFMA fragment of 16 operand rows starting at local row r (k = 32kk + 8(lane>>4) + j)
template <int MODE>
__device__ __forceinline__ bf16x8 frag(const char* slot, int r, int kk, int lane) {
  if constexpr (MODE == OP_KC) {
    return *reinterpret_cast<const bf16x8*>(slot + kc_off(r + (lane & 15), 4 * kk + (lane >> 4)));
  } else {
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int k1 = kk * 32 + 8 * g + q;
    const int col = r + 4 * pp;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(slot + rc_off(k1, col)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(slot + rc_off(k1 + 4, col)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

}  // namespace g256

template <int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(g256::THREADS, 1) void gemm256_kernel(const GemmParams p) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[8 * HALF];  // ring: [tile parity][A0, A1, B0, B1]

  const int tiles_n = (p.N + 255) >> 8;
  int bid, split;
  grid_tile(bid, split);
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * 256, n0 = tn * 256;
  const int kbeg = split * p.k_split;
  const int nk = (min(p.K, kbeg + p.k_split) - kbeg) >> 6;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const bf16_t* A = reinterpret_cast<const bf16_t*>(p.a);
  const bf16_t* B = reinterpret_cast<const bf16_t*>(p.b);

  auto slot = [&](int par, int h) -> char* { return smem + (par * 4 + h) * HALF; };
  auto stg = [&](int t, int h) {
    const int k0 = kbeg + t * 64;
    if (h < 2) stage<AMODE>(A, p.lda, p.M, m0 + h * 128, k0, slot(t & 1, h), wid, lane);
    else stage<BMODE>(B, p.ldb, p.N, n0 + (h - 2) * 128, k0, slot(t & 1, h), wid, lane);
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ar[4][2], br[2][2];

  // prologue: tile 0 complete + tile 1's A0, B1, A1 (its B0 is staged in phase 1 of tile 0)
  if (nk > 0) {
    stg(0, 0);
    stg(0, 2);
    stg(0, 3);
    stg(0, 1);
  }
  if (nk > 1) {
    stg(1, 0);
    stg(1, 3);
    stg(1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

  const int ra = wr * 64;  // this wave's first row inside an A half
  const int rb = wc * 32;  // this wave's first column inside a B half

#define DDL_G256_LOAD_A(par, h)                                                  \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                                  \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) ar[i][kk] =               \
          frag<AMODE>(slot(par, h), ra + 16 * i, kk, lane);
#define DDL_G256_LOAD_B(par, h)                                                  \
  _Pragma("unroll") for (int j = 0; j < 2; ++j)                                  \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) br[j][kk] =               \
          frag<BMODE>(slot(par, h), rb + 16 * j, kk, lane);
  // Fragment reads are retired (lgkmcnt 0) BEFORE the phase's first barrier, so a slot can be
  // restaged one phase after its last read even by the other (staggered) wave group.
#define DDL_G256_MMA(QM, QN)                                                                     \
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                             \
  __builtin_amdgcn_sched_barrier(0);                                                             \
  __builtin_amdgcn_s_barrier();                                                                  \
  __builtin_amdgcn_sched_barrier(0);                                                             \
  __builtin_amdgcn_s_setprio(1);                                                                 \
  _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) _Pragma("unroll") for (int i = 0; i < 4; ++i) \
      _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                            \
    if constexpr (epi_dt(EPI))                                                                   \
      acc[QM][QN][i][j] = mfma16x16x32(br[j][kk], ar[i][kk], acc[QM][QN][i][j]);                 \
    else                                                                                         \
      acc[QM][QN][i][j] = mfma16x16x32(ar[i][kk], br[j][kk], acc[QM][QN][i][j]);                 \
  }                                                                                              \
  __builtin_amdgcn_s_setprio(0);                                                                 \
  __builtin_amdgcn_sched_barrier(0);                                                             \
  __builtin_amdgcn_s_barrier();

  // Slot schedule: each half of the current buffer is restaged (for tile t+2, same parity) one
  // phase after its last read; B0 of tile t+1 goes in phase 1.  One counted vmcnt per K-tile
  // (phase 4) retires tile t+1 while tile t+2's three newest halves stay in flight.
  for (int t = 0; t < nk; ++t) {
    const int par = t & 1;
    const bool s1 = t + 1 < nk, s2 = t + 2 < nk;
    // phase 1: quadrant (0,0) — reads A0, B0
    DDL_G256_LOAD_A(par, 0)
    DDL_G256_LOAD_B(par, 2)
    if (s1) stg(t + 1, 2);
    DDL_G256_MMA(0, 0)
    // phase 2: quadrant (0,1) — reads B1; A0 is free
    DDL_G256_LOAD_B(par, 3)
    if (s2) stg(t + 2, 0);
    DDL_G256_MMA(0, 1)
    // phase 3: quadrant (1,1) — reads A1; B1 is free
    DDL_G256_LOAD_A(par, 1)
    if (s2) stg(t + 2, 3);
    DDL_G256_MMA(1, 1)
    // phase 4: quadrant (1,0) — reads B0; A1 is free; retire tile t+1
    DDL_G256_LOAD_B(par, 2)
    if (s2) {
      stg(t + 2, 1);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    DDL_G256_MMA(1, 0)
  }
#undef DDL_G256_LOAD_A
#undef DDL_G256_LOAD_B
#undef DDL_G256_MMA
  if (wr == 0) __builtin_amdgcn_s_barrier();  // re-align the groups

  const long coff = (long)split * p.split_stride;
  gemm_epilogue<4, 2, EPI>(p, acc[0][0], m0 + ra, n0 + rb, lane, bid, -1, coff);
  gemm_epilogue<4, 2, EPI>(p, acc[0][1], m0 + ra, n0 + 128 + rb, lane, bid, -1, coff);
  gemm_epilogue<4, 2, EPI>(p, acc[1][0], m0 + 128 + ra, n0 + rb, lane, bid, -1, coff);
  gemm_epilogue<4, 2, EPI>(p, acc[1][1], m0 + 128 + ra, n0 + 128 + rb, lane, bid, -1, coff);
}

template <int AMODE, int BMODE, int EPI>
inline int launch_g256(const GemmParams& p, hipStream_t s) {
  const int tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int splits = (p.K + p.k_split - 1) / p.k_split;
  hipLaunchKernelGGL((gemm256_kernel<AMODE, BMODE, EPI>), dim3(tiles, splits), dim3(g256::THREADS), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace ddl
