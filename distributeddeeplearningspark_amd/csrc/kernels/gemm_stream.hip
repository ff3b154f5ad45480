// Streaming "skinny-K" GEMM for gfx950: C[M][N] (bf16) = A[M][K] * B(N, K)^T with K in {64, 128, 256}.
//
// Target: the ResNet 1x1 convolutions (and their data-gradients) at large batch, e.g.
// M = 802,816 pixels x N = 256 x K = 64.  Those GEMMs are pure HBM streams — ~6 FLOP per byte —
// and the general 128x128 tile kernel loses on three counts: the weight tile is re-staged for
// every output tile, the MFMA-layout stores write 32-B row segments, and the fused BN statistics
// become one same-address atomic per column per tile.  This kernel is built for the stream:
//
//   * Weight-stationary: each wave keeps its WN x K slice of B in VGPRs for the whole kernel
//     (<= 64 VGPRs), loaded once; the workgroup (4 waves) covers a panel of NB = 4*WN columns.
//   * Persistent over 64-row tiles of A: the A tiles stream global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, swizzle applied to the source address) through an NBUF-deep
//     ring; a counted `s_waitcnt vmcnt` retires one tile while NBUF-2 stay in flight (loads,
//     stores and LDS-DMA retire in issue order, so the count includes the stores in between).
//   * Epilogue through LDS: alpha / bias / residual / ReLU are applied in the MFMA layout, the
//     bf16 tile is staged in LDS (XOR-swizzled, conflict-free) and written back as whole rows,
//     16 B per lane.  BN statistics (sum, sum of squares of the stored bf16 values) accumulate in
//     registers across all tiles of the workgroup and leave as ONE atomic per column per
//     workgroup at the end.
//
// Two 80-KB-or-smaller workgroups per CU.  B is K-contiguous ([N][K], a forward 1x1 conv / Linear
// weight) or row-contiguous ([K][N], the data-gradient of one), loaded once either way.
#include "ddl_gemm_kernel.h"

namespace ddl {
namespace gst {

constexpr int THREADS = 256;
constexpr int BM = 64;
constexpr int LDS_BUDGET = 80 * 1024;
typedef __attribute__((address_space(3))) void lds_t;

template <int WN, int K>
struct Cfg {
  static constexpr int NB = 4 * WN;                 // panel width
  static constexpr int RN = WN / 16;                // 16-column MFMA blocks per wave
  static constexpr int KS = K / 32;                 // MFMA k-steps
  static constexpr int CPR = K / 8;                 // 16-B chunks per A row
  static constexpr int TILE = BM * K * 2;           // bytes of one A tile
  static constexpr int D = TILE / 1024 / 4;         // LDS-DMA instructions per wave per tile
  static constexpr int OCPR = NB / 8;               // 16-B chunks per staged output row
  static constexpr int STAGE = BM * NB * 2;         // staged output tile
  static constexpr int RPP = THREADS / OCPR;        // output rows per read-out pass
  static constexpr int S = BM / RPP;                // 16-B stores per thread per tile
  static constexpr int NBUF_FIT = (LDS_BUDGET - STAGE) / TILE;
  static constexpr int NBUF = NBUF_FIT > 4 ? 4 : NBUF_FIT;
  static constexpr int LDS = NBUF * TILE + STAGE;
  static_assert(NBUF >= 2, "A ring needs two buffers");
  static_assert(D >= 1 && OCPR >= 8 && RPP >= 1 && BM % RPP == 0, "shape");
  static_assert((NBUF - 1) * (D + S) <= 63, "vmcnt range");
  static_assert(4 * 2 * OCPR * 8 * 4 <= STAGE, "stats reduction fits in the staging buffer");
};

// XOR swizzle of the 16-B chunk index of row r (rows of `cpr` chunks) so that 16 consecutive rows
// read / written at the same logical chunk hit 16 distinct 16-B bank groups.
template <int CPR>
__device__ __forceinline__ int sw(int r) {
  if constexpr (CPR == 8) return (r >> 1) & 7;
  else return r & 15;
}

// s_waitcnt vmcnt(N) as a real instruction (not inline asm), so the compiler's own wait
// insertion sees it and does not add a vmcnt(0) of its own (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]
// | lgkmcnt[11:8] | vmcnt_hi[15:14]; expcnt / lgkmcnt left at "don't wait").
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

template <class CF>
__device__ __forceinline__ void wait_tile(int younger_store_tiles) {
  constexpr int base = (CF::NBUF - 1) * CF::D;
  switch (younger_store_tiles) {
    case 0: wait_vm<base>(); break;
    case 1: wait_vm<base + CF::S>(); break;
    case 2: wait_vm<base + 2 * CF::S>(); break;
    default: wait_vm<base + 3 * CF::S>(); break;
  }
}

// Stage A rows [m0, m0 + BM) into one ring slot: LDS unit u (16 B) = row u / CPR, physical chunk
// u % CPR, which holds logical chunk (u % CPR) ^ sw(row).  Rows past M re-read row M - 1.
// The LDS-DMA is issued from inline asm: the compiler then does not know about the pending LDS
// writes and does not drain vmcnt(0) before every later LDS access — the ring's ordering is the
// kernel's own counted vmcnt + barrier (and compiler-placed waits for other loads can only be
// stricter than needed, never weaker, since they ignore these extra VMEM operations).
template <class CF>
__device__ __forceinline__ void stage_a(const bf16_t* __restrict__ A, long lda, int M, int m0, char* slot, int w,
                                        int lane) {
#pragma unroll
  for (int i = 0; i < CF::D; ++i) {
    const int blk = i * 4 + w;
    const int u = blk * 64 + lane;
    const int r = u / CF::CPR, cp = u % CF::CPR;
    const int c = cp ^ sw<CF::CPR>(r);
    const int gr = min(m0 + r, M - 1);
    const bf16_t* src = A + (long)gr * lda + c * 8;
    const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t) reinterpret_cast<uintptr_t>((lds_t*)(slot + blk * 1024)));
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(dst) : "memory", "m0");
  }
}

}  // namespace gst

// Side-operand loads of the residual / fused-BN-reduce epilogues (the residual rows, their ReLU mask, the BN
// input x and its mask byte) as inline asm: like the LDS-DMA ring they are invisible to the compiler's
// vmcnt model, so the only waits on them are the kernel's own counted ones.  Compiler-visible loads made
// the compiler wait for them with a count that ignores the (invisible) ring DMAs issued after them, i.e.
// it also drained the prefetch of the next A tile before every epilogue.
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
__device__ __forceinline__ u32x4_t ald128(const void* p) {
  u32x4_t v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ u32x2_t ald64(const void* p) {
  u32x2_t v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ald32(const void* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ald16(const void* p) {
  unsigned v;
  asm volatile("global_load_ushort %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ald8(const void* p) {
  unsigned v;
  asm volatile("global_load_ubyte %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
// ASM: the counted asm form; otherwise plain loads the compiler waits for itself (kept for A/B)
template <bool ASM> __device__ __forceinline__ u32x4_t sld128(const void* p) {
  if constexpr (ASM) return ald128(p);
  return *reinterpret_cast<const u32x4_t*>(p);
}
template <bool ASM> __device__ __forceinline__ u32x2_t sld64(const void* p) {
  if constexpr (ASM) return ald64(p);
  return *reinterpret_cast<const u32x2_t*>(p);
}
template <bool ASM> __device__ __forceinline__ unsigned sld32(const void* p) {
  if constexpr (ASM) return ald32(p);
  return *reinterpret_cast<const uint32_t*>(p);
}
template <bool ASM> __device__ __forceinline__ unsigned sld16(const void* p) {
  if constexpr (ASM) return ald16(p);
  return *reinterpret_cast<const uint16_t*>(p);
}
template <bool ASM> __device__ __forceinline__ unsigned sld8(const void* p) {
  if constexpr (ASM) return ald8(p);
  return *reinterpret_cast<const uint8_t*>(p);
}


// BNR: 0 off; 1 the ReLU mask of the BN-backward reduce from GemmParams::bnr_mask (bits, or all ones);
// 2 recomputed from the BN input as x * bnr_scale + bnr_shift > 0 (a BN without residual: mode 2)
template <int WN, int K, int BMODE, bool RES, int BNR = 0>
__global__ __launch_bounds__(gst::THREADS, 2) void gemm_stream_kernel(const GemmParams p) {
  using namespace gst;
  using CF = Cfg<WN, K>;
  // side-operand loads as counted asm (see sld128) on every ring: on the two-slot K = 256 rings it keeps the
  // refill DMA in flight through the epilogue (ResNet-50 +0.9 %); on the deeper rings it measured equal to
  // compiler-tracked loads end to end (profiles/r6/stream_side_loads/)
  constexpr bool kAsmSide = true;
  // the ring and the output staging tile are separate objects: with one array the compiler cannot
  // tell the staging writes from the in-flight LDS-DMA and drains vmcnt(0) before them
  __shared__ __attribute__((aligned(16))) char smem[CF::LDS];  // [ring NBUF x TILE | staging tile]
  char* const stg = smem + CF::NBUF * CF::TILE;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n0 = blockIdx.y * CF::NB;
  const int mt = (p.M + BM - 1) / BM;
  const int nloc = ((int)blockIdx.x < mt) ? (mt - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(p.a);

  // B slice in registers: bfr[rn][ks][j] = B(n0 + WN*w + 16rn + (lane&15), 32ks + 8(lane>>4) + j)
  bf16x8 bfr[CF::RN][CF::KS];
  {
    const bf16_t* __restrict__ B = reinterpret_cast<const bf16_t*>(p.b);
#pragma unroll
    for (int rn = 0; rn < CF::RN; ++rn)
#pragma unroll
      for (int ks = 0; ks < CF::KS; ++ks) {
        const int n = n0 + WN * w + 16 * rn + (lane & 15);
        const int k = 32 * ks + 8 * (lane >> 4);
        if constexpr (BMODE == OP_KC) {
          bfr[rn][ks] = *reinterpret_cast<const bf16x8*>(B + (long)n * p.ldb + k);
        } else {
          s16x8 v;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = (short)B[(long)(k + j) * p.ldb + n];
          bfr[rn][ks] = __builtin_bit_cast(bf16x8, v);
        }
      }
  }
  float bias_r[CF::RN][4];
#pragma unroll
  for (int rn = 0; rn < CF::RN; ++rn) {  // one 16-B load per 4 columns (N % panel == 0: always in range)
    const float4 bv = p.bias ? *reinterpret_cast<const float4*>(p.bias + n0 + WN * w + 16 * rn + 4 * (lane >> 4))
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    bias_r[rn][0] = bv.x;
    bias_r[rn][1] = bv.y;
    bias_r[rn][2] = bv.z;
    bias_r[rn][3] = bv.w;
  }
  wait_vm<0>();  // B fragments and bias in registers before the LDS-DMA ring starts
  auto tile_m0 = [&](int i) { return min((int)blockIdx.x + i * (int)gridDim.x, mt - 1) * BM; };

#pragma unroll
  for (int s = 0; s < CF::NBUF - 1; ++s) stage_a<CF>(A, p.lda, p.M, tile_m0(s), smem + s * CF::TILE, w, lane);

  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  const int oc = threadIdx.x % CF::OCPR, orow = threadIdx.x / CF::OCPR;
  // BNR: batch mean of the 8 columns this thread reads out (loaded once)
  float bmu[8];
  float bsc[BNR == 2 ? 8 : 1], bsh[BNR == 2 ? 8 : 1];
  if constexpr (BNR != 0) {
    const float4 a = *reinterpret_cast<const float4*>(p.bnr_mean + n0 + oc * 8);
    const float4 b = *reinterpret_cast<const float4*>(p.bnr_mean + n0 + oc * 8 + 4);
    bmu[0] = a.x; bmu[1] = a.y; bmu[2] = a.z; bmu[3] = a.w;
    bmu[4] = b.x; bmu[5] = b.y; bmu[6] = b.z; bmu[7] = b.w;
  }
  if constexpr (BNR == 2) {
    const float4 a0 = *reinterpret_cast<const float4*>(p.bnr_scale + n0 + oc * 8);
    const float4 a1 = *reinterpret_cast<const float4*>(p.bnr_scale + n0 + oc * 8 + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(p.bnr_shift + n0 + oc * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(p.bnr_shift + n0 + oc * 8 + 4);
    bsc[0] = a0.x; bsc[1] = a0.y; bsc[2] = a0.z; bsc[3] = a0.w; bsc[4] = a1.x; bsc[5] = a1.y; bsc[6] = a1.z; bsc[7] = a1.w;
    bsh[0] = b0.x; bsh[1] = b0.y; bsh[2] = b0.z; bsh[3] = b0.w; bsh[4] = b1.x; bsh[5] = b1.y; bsh[6] = b1.z; bsh[7] = b1.w;
  }
  bf16_t* __restrict__ Cout = reinterpret_cast<bf16_t*>(p.c);

  for (int i = 0; i < nloc; ++i) {
    // refill the slot consumed in iteration i - 1 (its reads finished before that iteration's
    // staging barrier) with the tile NBUF - 1 iterations ahead
    const int m0 = tile_m0(i);
    // residual rows of this tile, issued ahead of the refill so their wait can be counted past it
    // side operands (counted asm loads, see sld128): issued ahead of the refill, so the DMA of the tile
    // NBUF - 1 ahead is the youngest VMEM work when the epilogue waits for them (the ring stays in flight)
    u32x2_t rres[BM / 16][CF::RN];
    // residual ReLU mask (p.resid_mask): the 16 * RN columns this lane's row touches are 2 * RN
    // consecutive mask bytes — one 2/4/8-byte load per row block (from the residual itself when there is
    // no mask: always issued, so the counted wait holds); rodd rows (stride-2 subgrid) add nothing
    unsigned rmk32[BM / 16];
    u32x2_t rmk64[CF::RN == 4 ? BM / 16 : 1];
    unsigned rodd_bits = 0u;
    const bool has_mask = p.resid_mask != nullptr;
    if constexpr (RES) {
#pragma unroll
      for (int mb = 0; mb < BM / 16; ++mb) {
        const int m = min(m0 + 16 * mb + (lane & 15), p.M - 1);
        long rrow = m;  // stride-2 residual subgrid (GemmParams::rsub_h): odd rows add nothing
        if (p.rsub_h) {
          int rn_, ri_, rj_;
          pix_decompose((uint32_t)m, p.rsub_h, p.rsub_w, rn_, ri_, rj_);
          const bool rodd = (ri_ | rj_) & 1;
          rodd_bits |= (rodd ? 1u : 0u) << mb;
          rrow = rodd ? 0L : ((long)rn_ * ((p.rsub_h + 1) >> 1) + (ri_ >> 1)) * ((p.rsub_w + 1) >> 1) + (rj_ >> 1);
        }
        const long row = rrow * p.ldr + n0 + WN * w;
#pragma unroll
        for (int rn = 0; rn < CF::RN; ++rn)
          rres[mb][rn] = sld64<kAsmSide>(reinterpret_cast<const bf16_t*>(p.resid) + row + 16 * rn + 4 * (lane >> 4));
        const void* mp = has_mask ? (const void*)(p.resid_mask + (row >> 3)) : p.resid;
        if constexpr (CF::RN == 1) rmk32[mb] = sld16<kAsmSide>(mp);
        else if constexpr (CF::RN == 2) rmk32[mb] = sld32<kAsmSide>(mp);
        else rmk64[mb] = sld64<kAsmSide>(mp);
      }
    }
    // BNR: the BN input x and its ReLU-mask byte at this thread's read-out vectors
    u32x4_t bx[BNR ? CF::S : 1];
    unsigned bm8[BNR == 1 ? CF::S : 1];
    if constexpr (BNR) {
#pragma unroll
      for (int ps = 0; ps < CF::S; ++ps) {
        const int m = min(m0 + orow + ps * CF::RPP, p.M - 1);
        const long idx = (long)m * p.ldc + n0 + oc * 8;
        bx[ps] = sld128<kAsmSide>(reinterpret_cast<const bf16_t*>(p.bnr_x) + idx);
        if constexpr (BNR == 1)
          bm8[ps] = sld8<kAsmSide>(p.bnr_mask ? (const void*)(p.bnr_mask + (idx >> 3)) : (const void*)p.bnr_x);
      }
    }
    const int ahead = i + CF::NBUF - 1;
    stage_a<CF>(A, p.lda, p.M, tile_m0(ahead), smem + (ahead % CF::NBUF) * CF::TILE, w, lane);
    wait_tile<CF>(min(i, CF::NBUF - 1));
    __builtin_amdgcn_s_barrier();  // tile i visible to every wave; previous read-out finished

    const char* abuf = smem + (i % CF::NBUF) * CF::TILE;
    f32x4 acc[BM / 16][CF::RN];
#pragma unroll
    for (int mb = 0; mb < BM / 16; ++mb)
#pragma unroll
      for (int rn = 0; rn < CF::RN; ++rn) acc[mb][rn] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < CF::KS; ++ks)
#pragma unroll
      for (int mb = 0; mb < BM / 16; ++mb) {
        const int r = 16 * mb + (lane & 15);
        const int c = 4 * ks + (lane >> 4);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abuf + r * (K * 2) + ((c ^ sw<CF::CPR>(r)) << 4));
#pragma unroll
        for (int rn = 0; rn < CF::RN; ++rn) acc[mb][rn] = mfma16x16x32(bfr[rn][ks], a, acc[mb][rn]);
      }

    // counted waits (asm side loads): the residual before the epilogue math, with the BN-reduce loads (issued
    // after it) and the refill DMA (the youngest) still in flight; the BN-reduce loads before the read-out.
    // The empty asm redefines each loaded register after its wait, so no use is scheduled above it.
    constexpr int kBnrLoads = BNR == 1 ? 2 * CF::S : (BNR == 2 ? CF::S : 0);
    if constexpr (kAsmSide && RES) {
      wait_vm<CF::D + kBnrLoads>();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mb = 0; mb < BM / 16; ++mb) {
#pragma unroll
        for (int rn = 0; rn < CF::RN; ++rn) asm volatile("" : "+v"(rres[mb][rn]));
        if constexpr (CF::RN == 4) asm volatile("" : "+v"(rmk64[mb]));
        else asm volatile("" : "+v"(rmk32[mb]));
      }
    }
    // epilogue math in the MFMA layout: acc[mb][rn][e] = C[m0 + 16mb + (lane&15)][n0 + WN*w + 16rn + 4(lane>>4) + e]
#pragma unroll
    for (int mb = 0; mb < BM / 16; ++mb) {
      const int r = 16 * mb + (lane & 15);
#pragma unroll
      for (int rn = 0; rn < CF::RN; ++rn) {
        const int nl = WN * w + 16 * rn + 4 * (lane >> 4);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaf(acc[mb][rn][e], p.alpha, bias_r[rn][e]);
        if constexpr (RES) {
          const u32x2_t rv = rres[mb][rn];
          uint64_t mraw;
          if constexpr (CF::RN == 4) mraw = ((uint64_t)rmk64[mb].y << 32) | rmk64[mb].x;
          else mraw = rmk32[mb];
          const uint64_t rm = ((rodd_bits >> mb) & 1u) ? 0ull : (has_mask ? mraw : ~0ull);
          const uint32_t mk = (uint32_t)(rm >> (16 * rn + 4 * (lane >> 4)));
          v[0] += (mk & 1u) ? __uint_as_float(rv.x << 16) : 0.f;
          v[1] += (mk & 2u) ? __uint_as_float(rv.x & 0xffff0000u) : 0.f;
          v[2] += (mk & 4u) ? __uint_as_float(rv.y << 16) : 0.f;
          v[3] += (mk & 8u) ? __uint_as_float(rv.y & 0xffff0000u) : 0.f;
        }
        if (p.relu == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        *reinterpret_cast<uint2*>(stg + r * (CF::NB * 2) + (((nl >> 3) ^ sw<CF::OCPR>(r)) << 4) + (nl & 7) * 2) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): staging writes done before the barrier
    __builtin_amdgcn_s_barrier();

    if constexpr (kAsmSide && BNR) {
      wait_vm<CF::D>();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ps = 0; ps < CF::S; ++ps) {
        asm volatile("" : "+v"(bx[ps]));
        if constexpr (BNR == 1) asm volatile("" : "+v"(bm8[ps]));
      }
    }
    // read-out: whole rows, 16 B per lane (each thread always owns the same 8 columns)
#pragma unroll
    for (int ps = 0; ps < CF::S; ++ps) {
      const int r = orow + ps * CF::RPP;
      const int m = m0 + r;
      const uint4 v = *reinterpret_cast<const uint4*>(stg + r * (CF::NB * 2) + ((oc ^ sw<CF::OCPR>(r)) << 4));
      if (m < p.M) {
        *reinterpret_cast<uint4*>(Cout + (long)m * p.ldc + n0 + oc * 8) = v;
        if constexpr (BNR) {  // BN-backward partial sums of the stored gradient (see GemmParams)
          const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
          const uint32_t xv[4] = {bx[ps].x, bx[ps].y, bx[ps].z, bx[ps].w};
          uint32_t bmk = 0xffu;
          if constexpr (BNR == 1) bmk = p.bnr_mask ? bm8[ps] : 0xffu;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int e = 2 * q + h;
              const float xe = __uint_as_float(h ? (xv[q] & 0xffff0000u) : (xv[q] << 16));
              bool keep;
              if constexpr (BNR == 2) keep = xe * bsc[e] + bsh[e] > 0.f;  // the forward's own fmaf: same bits
              else keep = (bmk >> e) & 1u;
              const float d = keep ? __uint_as_float(h ? (wv[q] & 0xffff0000u) : (wv[q] << 16)) : 0.f;
              s1[e] += d;
              s2[e] += d * (xe - bmu[e]);
            }
          }
        } else if (p.stats) {
          const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = __uint_as_float(wv[q] << 16), hi = __uint_as_float(wv[q] & 0xffff0000u);
            s1[2 * q] += lo;
            s2[2 * q] += lo * lo;
            s1[2 * q + 1] += hi;
            s2[2 * q + 1] += hi * hi;
          }
        }
      }
    }
  }
  wait_vm<0>();  // no LDS-DMA may outlive the workgroup (the ring prefetches past the last tile)

  if (p.stats) {
    // lanes of a wave with equal (lane % OCPR) own the same columns
#pragma unroll
    for (int o = CF::OCPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    __syncthreads();
    float* red = reinterpret_cast<float*>(stg);  // [wave][OCPR][16]
    if (lane < CF::OCPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(w * CF::OCPR + lane) * 16 + e] = s1[e];
        red[(w * CF::OCPR + lane) * 16 + 8 + e] = s2[e];
      }
    }
    __syncthreads();
    float* st = p.stats + (long)(blockIdx.x % kStatShards) * 2 * p.N;
    for (int t = threadIdx.x; t < CF::NB; t += THREADS) {
      const int ch = t >> 3, e = t & 7;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) {
        a += red[(ww * CF::OCPR + ch) * 16 + e];
        b += red[(ww * CF::OCPR + ch) * 16 + 8 + e];
      }
      atomicAdd(st + n0 + t, a);
      atomicAdd(st + p.N + n0 + t, b);
    }
  }
}

namespace {

int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <int WN, int K, int BMODE>
int launch_ws(const GemmParams& p, hipStream_t s) {
  using CF = gst::Cfg<WN, K>;
  // variants launch_gemm_stream never routes here are not instantiated (they would spill): a residual on the
  // 256-wide K = 128 panel, the fused BN-backward reduce on panels wider than 128 (64 at K = 256)
  constexpr bool kRes = !(WN == 64 && K == 128);
  constexpr bool kBnr = CF::NB <= (K >= 256 ? 64 : 128);
  const int panels = p.N / CF::NB;
  const int mt = (p.M + gst::BM - 1) / gst::BM;
  const int gx = std::max(1, std::min(mt, 2 * num_cus() / std::max(1, panels)));
  if (p.bnr_x && p.bnr_scale) {  // mode 2 (no residual: a BN + ReLU without a shortcut)
    if constexpr (kBnr) {
      if (p.resid) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, false, 2>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
    } else {
      return (int)hipErrorInvalidValue;
    }
  } else if (p.bnr_x) {
    if constexpr (kBnr && kRes) {
      if (p.resid)
        hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, true, 1>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
      else
        hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, false, 1>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
    } else if constexpr (kBnr) {
      if (p.resid) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, false, 1>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
    } else {
      return (int)hipErrorInvalidValue;
    }
  } else if (p.resid) {
    if constexpr (kRes)
      hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, true>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
    else
      return (int)hipErrorInvalidValue;
  } else {
    hipLaunchKernelGGL((gemm_stream_kernel<WN, K, BMODE, false>), dim3(gx, panels), dim3(gst::THREADS), 0, s, p);
  }
  return (int)hipGetLastError();
}

template <int WN, int BMODE>
int launch_k(const GemmParams& p, hipStream_t s) {
  switch (p.K) {
    case 64: return launch_ws<WN, 64, BMODE>(p, s);
    case 128: return launch_ws<WN, 128, BMODE>(p, s);
    default:
      if constexpr (WN <= 32) return launch_ws<WN, 256, BMODE>(p, s);
      return (int)hipErrorInvalidValue;
  }
}

template <int BMODE>
int launch_panel(const GemmParams& p, int nb, hipStream_t s) {
  switch (nb) {
    case 64: return launch_k<16, BMODE>(p, s);
    case 128: return launch_k<32, BMODE>(p, s);
    default: return launch_k<64, BMODE>(p, s);
  }
}

}  // namespace

// Panel width for (N, K), or 0 when the streaming kernel does not apply.
int gemm_stream_panel(int N, int K) {
  if (K != 64 && K != 128 && K != 256) return 0;
  const int max_nb = K == 256 ? 128 : 256;
  for (int nb = max_nb; nb >= 64; nb >>= 1)
    if (N % nb == 0 && (N == nb || nb == max_nb)) return nb;
  return 0;
}

int launch_gemm_stream(const GemmParams& p, int epi, hipStream_t s) {
  int nb = gemm_stream_panel(p.N, p.K);
  if (p.resid && p.K == 128 && nb == 256) nb = 128;  // 256-wide panel + residual prefetch would spill
  // the fused BN-backward reduction prefetches x and the mask per read-out vector: narrower panels keep
  // those variants spill-free (128 wide up to K = 128, 64 at K = 256; A is re-read once more per panel)
  if (p.bnr_x && nb > (p.K >= 256 ? 64 : 128)) nb = p.K >= 256 ? 64 : 128;
  const bool ok = nb && epi == EPI_BF16 && p.a_mode == OP_KC && (p.b_mode == OP_KC || p.b_mode == OP_RC) &&
                  !p.om.enabled && !p.aux && !p.drop_thresh && (p.relu == ACT_NONE || p.relu == ACT_RELU) &&
                  p.beta == 0.f && p.k_split >= p.K && p.lda % 8 == 0 && p.ldc % 8 == 0 &&
                  (p.b_mode == OP_RC || p.ldb % 8 == 0) && (!p.resid || p.ldr % 4 == 0) &&
                  ((uintptr_t)p.a % 16 == 0) && ((uintptr_t)p.c % 16 == 0) &&
                  (p.b_mode == OP_RC || (uintptr_t)p.b % 16 == 0) && (!p.resid || (uintptr_t)p.resid % 8 == 0) &&
                  (!p.bnr_x || (p.stats && (uintptr_t)p.bnr_x % 16 == 0 && (uintptr_t)p.bnr_mean % 16 == 0)) &&
                  (!p.bnr_scale || (p.bnr_shift && !p.resid && (uintptr_t)p.bnr_scale % 16 == 0 &&
                                    (uintptr_t)p.bnr_shift % 16 == 0));
  if (!ok) return (int)hipErrorInvalidValue;
  return p.b_mode == OP_KC ? launch_panel<OP_KC>(p, nb, s) : launch_panel<OP_RC>(p, nb, s);
}

}  // namespace ddl
