// MFMA (v_mfma_f32_16x16x32_bf16) implicit-GEMM kernel template for gfx950.
//
// Block: 256 threads = 4 waves arranged 2(M) x 2(N); block tile BM x BN x 64.
// Operands are staged global -> VGPR -> LDS (double-buffered, one barrier per
// K-tile; the next tile's global loads are issued before the current tile's
// MFMAs so HBM latency hides under them).  LDS images:
//   KC image [R][64]  128-B rows, 16-B chunk XOR-swizzled by (row>>1)&7,
//                     fragments read with ds_read_b128 (conflict-free per 16-lane group)
//   RC image [64][R]  R*2-B rows, chunk XOR-swizzled by a 3-bit (R=128) / 2-bit (R=64)
//                     function of k, fragments read with ds_read_b64_tr_b16 (hardware
//                     transpose) so K-strided operands need no data reshuffle.
// Grid: 1-D over (M-tiles x N-tiles) with the XCD-aware bijective remap, y = split-K.
#pragma once
#include "ddl_common.h"
#include "ddl_gemm.h"
#include <stdlib.h>

namespace ddl {

constexpr int BK = 64;
constexpr int NTHREADS = 256;
// Minimum resident blocks per CU the LDS-DMA kernel is compiled for.  4 caps the bf16-output
// kernels at 128 VGPRs (the 128x128 conv kernel otherwise takes 134 -> 3 blocks/CU): one more
// block per CU to hide the single-stage DMA latency is worth +6 % on ResNet-50.  The fp32
// weight-gradient kernels keep 2 (at 128 VGPRs their RC fragments spill).
#ifndef DDL_WGRAD_MIN_BLOCKS
#define DDL_WGRAD_MIN_BLOCKS 2
#endif
#ifndef DDL_DMA_BF16_MIN_BLOCKS
#define DDL_DMA_BF16_MIN_BLOCKS 4  // resident workgroups per CU the bf16-output kernels' registers are capped for
#endif
// 128x128 bf16-output kernels with a row-contiguous (transpose-read) A operand, or a row-contiguous B with the
// lite / BN-reduce epilogue, need more than 128 VGPRs (they spilled 8-13 scratch instructions, some inside the
// main loop): 3 blocks per CU for those.  None of them is on the ResNet-50 / BERT-base / VGG-16 paths.
template <int BM, int BN, int AMODE, int BMODE, int EPI>
constexpr int dma_min_blocks() {
  if constexpr (EPI == EPI_F32 || EPI == EPI_F32_ATOMIC) return DDL_WGRAD_MIN_BLOCKS;
  if constexpr (BM * BN == 128 * 128 && (AMODE == OP_RC || (BMODE == OP_RC && EPI != EPI_BF16)))
    return DDL_DMA_BF16_MIN_BLOCKS < 3 ? DDL_DMA_BF16_MIN_BLOCKS : 3;
  return DDL_DMA_BF16_MIN_BLOCKS;
}

// Simple, exact division helper (used where the divisor is a power of two or tiny loops are fine)
__device__ __forceinline__ void pix_decompose(uint32_t p, uint32_t ho, uint32_t wo, int& n, int& i, int& j) {
  const uint32_t hw = ho * wo;
  n = (int)(p / hw);
  const uint32_t r = p - (uint32_t)n * hw;
  i = (int)(r / wo);
  j = (int)(r - (uint32_t)i * wo);
}

template <int R>
__device__ __forceinline__ int rc_swz(int k) {
  if constexpr (R == 128) return (k & 3) | (((k >> 3) & 1) << 2);
  else return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
}

__device__ __forceinline__ uint4 ldg16(const void* p) { return *reinterpret_cast<const uint4*>(p); }

// The gathering operand modes look tap offsets up in the kernel-argument tap table.  gfx950 has no
// scalar byte loads, so g.dh[t] / g.dw[t] compile to dependent VECTOR byte loads from the kernarg
// segment (per lane for KC_GATHER8, per K-tile even for a block-uniform t) whose s_waitcnt vmcnt
// also drains every LDS-DMA in flight: each K-tile paid a kernarg round trip before its DMAs could
// issue, and a deeper LDS-DMA ring was drained at every refill.  Gathering kernels therefore copy the
// table once into the first bytes of their LDS (ds_read: counted by lgkmcnt, not vmcnt):
// entry t = (dw[t] << 16) | (dh[t] & 0xffff).
template <int AMODE, int BMODE = OP_KC>
constexpr int tap_table_bytes() {
  return (AMODE == OP_KC_GATHER8 || AMODE == OP_KC_GATHER || BMODE == OP_RC_GATHER || BMODE == OP_RC_GATHER8)
             ? 4 * kMaxTaps
             : 0;
}
__device__ __forceinline__ int tap_dh(int e) { return (int)(short)(e & 0xffff); }
__device__ __forceinline__ int tap_dw(int e) { return e >> 16; }

__device__ __forceinline__ void load_tap_table(int* tab, const ConvGeom& g) {
  if ((int)threadIdx.x < g.ntaps) tab[threadIdx.x] = ((int)g.dw[threadIdx.x] << 16) | ((int)g.dh[threadIdx.x] & 0xffff);
  __syncthreads();
}


// Source selection of a staged vector: the LDS-DMA path (SWZ) substitutes the zero page for an
// out-of-range vector right here (a select, no branch around the address arithmetic and no second
// null test in dma()); the register path keeps nullptr (= load zeros).
template <bool SWZ>
__device__ __forceinline__ const bf16_t* vsrc(bool ok, const bf16_t* p) {
  if constexpr (SWZ) return ok ? p : reinterpret_cast<const bf16_t*>(ddl_zero_page);
  else return ok ? p : nullptr;
}

// ----------------------------------------------------------------------------------------
// Operand loaders. R = tile extent along the operand's row dimension (BM for A, BN for B).
// ----------------------------------------------------------------------------------------
template <int R, int MODE>
struct Operand {
  static constexpr bool KC = (MODE == OP_KC || MODE == OP_KC_GATHER || MODE == OP_KC_GATHER8);
  static constexpr int V = R / 32;  // 16-B vectors per thread per K-tile (R*64*2/16/256)
  uint4 reg[V];
  // per-thread precomputed state
  const bf16_t* ptr;
  long ld;
  int rows, r0, K;
  // gather state (KC_GATHER): per vector row
  int pixbase[V];  // n*hi*wi
  int hbase[V], wbase[V];
  bool rvalid[V];
  // KC gathers, LDS-DMA order: the element offset of the vector's output pixel at tap (0, 0),
  // channel chunk included — a K-tile adds the block-uniform tap offset (dh*wi + dw)*c + c0.
  // Gathered tensors hold < 2^31 elements (host check), so the offsets are 32-bit.
  int pofs[(MODE == OP_KC_GATHER || MODE == OP_KC_GATHER8) ? V : 1];
  // gather state (RC_GATHER / RC_GATHER8): the output pixel k = k0 + krow of vector v, kept as
  // (n, i, j) and advanced by BK per staged K-tile (the K-tiles are staged strictly in order), so
  // the main loop does no integer division (two runtime divisions per vector per K-tile made the
  // gathered weight-gradient kernels VALU-bound on address arithmetic)
  static constexpr bool RCG = (MODE == OP_RC_GATHER || MODE == OP_RC_GATHER8);
  int qn[RCG ? V : 1], qi[RCG ? V : 1], qj[RCG ? V : 1];
  int tap8[MODE == OP_RC_GATHER8 ? V : 1], ch8[MODE == OP_RC_GATHER8 ? V : 1];
  int dh8[MODE == OP_RC_GATHER8 ? V : 1], dw8[MODE == OP_RC_GATHER8 ? V : 1];  // that tap's offsets
  int dhb, dwb;  // RC_GATHER: the block's tap offsets (t = r0 / tap_c is fixed per block)
  // plain KC / RC modes, LDS-DMA (swizzled) order: each staged vector's element offset without the
  // K-tile term, its k offset inside the tile, and whether its row is in range — precomputed so a
  // K-tile's DMA addresses cost an add and a compare per vector instead of a 64-bit multiply, the
  // swizzle and a branch (the BERT weight-gradient loop issued 7 VALU per MFMA on address math)
  static constexpr bool PLAIN = (MODE == OP_KC || MODE == OP_RC);
  long boff[PLAIN ? V : 1];
  int kofs[PLAIN ? V : 1];
  bool rok[PLAIN ? V : 1];
  int di, dj;
  const DDL_LDS int* tt = nullptr;  // gather modes: the LDS copy of the tap table (load_tap_table)

  __device__ __forceinline__ void init(const void* p, long ld_, int rows_, int r0_, int K_, const ConvGeom& g,
                                       int k0 = 0) {
    ptr = reinterpret_cast<const bf16_t*>(p);
    ld = ld_;
    rows = rows_;
    r0 = r0_;
    K = K_;
    if constexpr (PLAIN) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        if constexpr (MODE == OP_KC) {
          const int row = idx >> 3;
          const int kc = (idx & 7) ^ ((row >> 1) & 7);
          const int r = r0 + row;
          kofs[v] = kc * 8;
          boff[v] = (long)r * ld + kc * 8;
          rok[v] = r < rows;
        } else {
          const int krow = idx / (R / 8);
          const int rc = (idx % (R / 8)) ^ (rc_swz<R>(krow) << 1);
          const int r = r0 + rc * 8;
          kofs[v] = krow;
          boff[v] = (long)krow * ld + r;
          rok[v] = r < rows;
        }
      }
    }
    if constexpr (RCG) {
      di = BK / g.wo;
      dj = BK - di * g.wo;
      if constexpr (MODE == OP_RC_GATHER) {
        const int e = tt[r0 / g.tap_c];
        dhb = tap_dh(e);
        dwb = tap_dw(e);
      }
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int krow = idx / (R / 8);
        const int k = k0 + krow;
        pix_decompose((uint32_t)(k < K ? k : 0), g.ho, g.wo, qn[v], qi[v], qj[v]);
        if constexpr (MODE == OP_RC_GATHER8) {
          // the (tap, channel) of this thread's 8 columns does not depend on k (SWZ or not: both
          // column permutations are functions of krow only, fixed per thread)
          const int rc = (idx % (R / 8)) ^ (rc_swz<R>(krow) << 1);
          const int r = r0 + rc * 8;
          tap8[v] = r < rows ? r / g.tap_c : 0;
          ch8[v] = r - tap8[v] * g.tap_c;
          dh8[v] = tap_dh(tt[tap8[v]]);
          dw8[v] = tap_dw(tt[tap8[v]]);
        }
      }
    }
    if constexpr (MODE == OP_KC_GATHER || MODE == OP_KC_GATHER8) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int row = idx >> 3;
        const int m = r0 + row;
        rvalid[v] = m < rows;
        int n, i, j;
        pix_decompose((uint32_t)(rvalid[v] ? m : 0), g.ho, g.wo, n, i, j);
        pixbase[v] = n * g.hi * g.wi;
        hbase[v] = i * g.sh;
        wbase[v] = j * g.sw;
        const int kc = (idx & 7) ^ ((row >> 1) & 7);  // the swizzled chunk the DMA path stages
        pofs[v] = (pixbase[v] + hbase[v] * g.wi + wbase[v]) * g.c + (MODE == OP_KC_GATHER ? kc * 8 : 0);
      }
    }
  }

  // Source of 16-B vector v of the K-tile at k0 (vsrc: zero page / nullptr).  SWZ: vector v is LDS unit
  // threadIdx.x + 256 v of the SWIZZLED image (the LDS-DMA writes lane-linearly, so the swizzle
  // moves to the source); !SWZ: vector v is the unswizzled (row, chunk) the register path stores.
  template <bool SWZ>
  __device__ __forceinline__ const bf16_t* addr(int v, int k0, const ConvGeom& g, int kdiv, long tap_stride) const {
    const int idx = threadIdx.x + v * NTHREADS;
    if constexpr (KC) {
      const int row = idx >> 3;
      const int kc = SWZ ? ((idx & 7) ^ ((row >> 1) & 7)) : (idx & 7);
      if constexpr (MODE == OP_KC) {
        if constexpr (SWZ) {
          return vsrc<true>(rok[v] && k0 + kofs[v] < K, ptr + boff[v] + k0);
        } else {
          const int r = r0 + row, k = k0 + kc * 8;
          return (r < rows && k < K) ? ptr + (long)r * ld + k : nullptr;
        }
      } else if constexpr (MODE == OP_KC_GATHER) {
        const int t = k0 / g.tap_c;  // block-uniform: tap_c % 64 == 0
        const int c0 = k0 - t * g.tap_c;
        const int e = tt[t];
        const int dh = tap_dh(e), dw = tap_dw(e);
        const int ih = hbase[v] + dh, iw = wbase[v] + dw;
        const bool ok = rvalid[v] && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        if constexpr (SWZ) return vsrc<true>(ok, ptr + (pofs[v] + (dh * g.wi + dw) * g.c + c0));
        else return vsrc<false>(ok, ptr + ((long)(pixbase[v] + ih * g.wi + iw)) * g.c + c0 + kc * 8);
      } else {  // OP_KC_GATHER8
        const int k = k0 + kc * 8;
        bool ok = rvalid[v] && k < K;
        const int t = ok ? (g.tap_shift >= 0 ? k >> g.tap_shift : k / g.tap_c) : 0;
        const int c = k - t * g.tap_c;
        const int e = tt[t];
        const int dh = tap_dh(e), dw = tap_dw(e);
        const int ih = hbase[v] + dh, iw = wbase[v] + dw;
        ok = ok && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        if constexpr (SWZ) return vsrc<true>(ok, ptr + (pofs[v] + (dh * g.wi + dw) * g.c + c));
        else return vsrc<false>(ok, ptr + ((long)(pixbase[v] + ih * g.wi + iw)) * g.c + c);
      }
    } else {
      const int krow = idx / (R / 8);
      const int rc = SWZ ? ((idx % (R / 8)) ^ (rc_swz<R>(krow) << 1)) : (idx % (R / 8));
      const int k = k0 + krow;
      if constexpr (MODE == OP_RC) {
        if constexpr (SWZ) {
          return vsrc<true>(rok[v] && k0 + kofs[v] < K, ptr + boff[v] + (long)k0 * ld);
        } else {
          const int r = r0 + rc * 8;
          return (r < rows && k < K) ? ptr + (long)k * ld + r : nullptr;
        }
      } else if constexpr (MODE == OP_RC_GATHER8) {
        // (rc is the SWZ-permuted column chunk; the (tap, channel) of it was fixed in init for the
        // swizzled order; the register path (SWZ = false) recomputes it)
        int c = ch8[v], dhv = dh8[v], dwv = dw8[v];
        bool ok = k < K;
        if constexpr (!SWZ) {
          const int r = r0 + rc * 8;
          ok = ok && r < rows;
          const int t = r < rows ? r / g.tap_c : 0;
          c = r - t * g.tap_c;
          dhv = tap_dh(tt[t]);
          dwv = tap_dw(tt[t]);
        } else {
          ok = ok && r0 + rc * 8 < rows;
        }
        const int ih = qi[v] * g.sh + dhv, iw = qj[v] * g.sw + dwv;
        ok = ok && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        return vsrc<SWZ>(ok, ptr + (((qn[v] * g.hi + ih) * g.wi + iw) * g.c + c));  // < 2^31: 32-bit
      } else if constexpr (MODE == OP_RC_GATHER) {
        const int t = r0 / g.tap_c;  // block-uniform: tap_c % R == 0
        const int c0 = r0 - t * g.tap_c;
        const int ih = qi[v] * g.sh + dhb, iw = qj[v] * g.sw + dwb;
        const bool ok = k < K && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        return vsrc<SWZ>(ok, ptr + (((qn[v] * g.hi + ih) * g.wi + iw) * g.c + c0 + rc * 8));  // 32-bit
      } else {  // OP_RC_TAPS: k = tap*kdiv + co ; addr = ptr + co*ld + wt[tap]*tap_stride + r
        const int t = k0 / kdiv;  // block-uniform: kdiv % 64 == 0
        const int co0 = k0 - t * kdiv;
        const int r = r0 + rc * 8;
        return vsrc<SWZ>(r < rows && k < K, ptr + (long)g.wt[t] * tap_stride + (long)(co0 + krow) * ld + r);
      }
    }
  }

  // RC gather modes: move the per-vector pixel state to the next K-tile (k += BK)
  __device__ __forceinline__ void advance(const ConvGeom& g) {
    if constexpr (RCG) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        qj[v] += dj;
        qi[v] += di;
        if (qj[v] >= g.wo) {
          qj[v] -= g.wo;
          qi[v] += 1;
        }
        while (qi[v] >= g.ho) {
          qi[v] -= g.ho;
          qn[v] += 1;
        }
      }
    }
  }

  __device__ __forceinline__ void load(int k0, const ConvGeom& g, int kdiv, long tap_stride) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const bf16_t* src = addr<false>(v, k0, g, kdiv, tap_stride);
      reg[v] = src ? ldg16(src) : make_uint4(0, 0, 0, 0);
    }
    advance(g);
  }

  // LDS-DMA of the K-tile at k0 into a (swizzled) LDS image: V wave-instructions of 1 KB each
  __device__ __forceinline__ void dma(char* lds, int k0, const ConvGeom& g, int kdiv, long tap_stride, int wid) {
    // the wave-uniform LDS destination once per call (the generic -> LDS cast carries a null check
    // and two readfirstlanes), then scalar offsets per vector
    const uint32_t base = lds_addr(lds) + (uint32_t)__builtin_amdgcn_readfirstlane(wid) * 1024u;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      dma16(addr<true>(v, k0, g, kdiv, tap_stride), base + (uint32_t)(v * NTHREADS * 16));
    }
    advance(g);
  }

  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int idx = threadIdx.x + v * NTHREADS;
      int byte;
      if constexpr (KC) {
        const int row = idx >> 3, kc = idx & 7;
        byte = row * 128 + ((kc ^ ((row >> 1) & 7)) << 4);
      } else {
        const int krow = idx / (R / 8), rc = idx % (R / 8);
        byte = krow * (R * 2) + ((rc ^ (rc_swz<R>(krow) << 1)) << 4);
      }
      *reinterpret_cast<uint4*>(lds + byte) = reg[v];
    }
  }

  // fragment for MFMA 16x16x32: rows wr0 + 16*rep + (lane&15), k = kk*32 + 8*(lane>>4) + j
  __device__ __forceinline__ bf16x8 frag(const char* lds, int kk, int rep, int wr0, int lane) const {
    if constexpr (KC) {
      const int row = wr0 + 16 * rep + (lane & 15);
      const int chunk = kk * 4 + (lane >> 4);
      const int byte = row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
      return *reinterpret_cast<const bf16x8*>(lds + byte);
    } else {
      const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
      const int k1 = kk * 32 + 8 * g + q;
      const int col = wr0 + 16 * rep + 4 * p;
      const int b1 = k1 * (R * 2) + ((((col >> 3) ^ (rc_swz<R>(k1) << 1))) << 4) + (col & 7) * 2;
      const int k2 = k1 + 4;
      const int b2 = k2 * (R * 2) + ((((col >> 3) ^ (rc_swz<R>(k2) << 1))) << 4) + (col & 7) * 2;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(lds + b1));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(lds + b2));
      s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      return __builtin_bit_cast(bf16x8, r);
    }
  }
};

// bf16-output epilogues take D^T fragments (a lane owns 4 consecutive columns of one row)
constexpr bool epi_dt(int epi) {
  return epi == EPI_BF16 || epi == EPI_BF16_LITE || epi == EPI_BF16_BNR;
}

// Per-column statistics of a wave's D^T fragments (lane: row lane & 15 of 16, columns nb + 16 j + 4 (lane >> 4)
// + e) summed over the 16 rows and added to st[0][n] / st[N][n] (s1 / s2).  A butterfly reduce-scatter:
// at each of the four xor levels a lane keeps one half of its values and trades the other half with its
// partner (NV/2 + NV/4 + NV/8 + NV/16 shuffles instead of 4 NV), leaving every lane NV/16 DIFFERENT column
// totals — so the adds go out as NV/16 whole-wave atomic instructions (64 lanes each) instead of NV/2
// instructions with 4 lanes active: the atomic issue rate (~50 ns per wave-instruction per CU) was the
// epilogue's bottleneck (a BN-reducing epilogue made a short GEMM 39 -> 71 us).
template <int H, int NV>
__device__ __forceinline__ void bfly_level(float (&v)[NV], const int mrow) {
  constexpr int M = (H * 16) / NV;  // xor mask of this level: 8, 4, 2, 1
  const bool up = (mrow & M) != 0;
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const float send = up ? v[i] : v[i + H];
    const float keep = up ? v[i + H] : v[i];
    v[i] = keep + __shfl_xor(send, M, 64);
  }
}
template <int RN>
__device__ __forceinline__ void col_stats_atomics(const float (&s1)[RN][4], const float (&s2)[RN][4], float* st,
                                                  const int N, const int nb, const int lane) {
  constexpr int RP = RN < 4 ? 4 : RN;  // column groups padded so every lane ends with >= 2 values
  constexpr int NV = 8 * RP;
  float v[NV];
#pragma unroll
  for (int j = 0; j < RP; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[4 * j + e] = j < RN ? s1[j < RN ? j : 0][e] : 0.f;
      v[NV / 2 + 4 * j + e] = j < RN ? s2[j < RN ? j : 0][e] : 0.f;
    }
  const int mrow = lane & 15;
  bfly_level<NV / 2, NV>(v, mrow);
  bfly_level<NV / 4, NV>(v, mrow);
  bfly_level<NV / 8, NV>(v, mrow);
  bfly_level<NV / 16, NV>(v, mrow);
  constexpr int PL = NV / 16;  // lane mrow now holds original values PL * mrow .. PL * mrow + PL - 1
#pragma unroll
  for (int q = 0; q < PL; ++q) {
    const int idx = PL * mrow + q;
    const int stt = idx / (NV / 2), rem = idx - stt * (NV / 2), j = rem >> 2, e = rem & 3;
    const int n = nb + 16 * j + 4 * (lane >> 4) + e;
    if (j < RN && n < N) atomicAdd(st + (long)stt * N + n, v[q]);
  }
}

// Paired D^T fragments (j, j + 1) of one row <-> 16-B memory accesses.  In the D^T layout lane group
// g = lane >> 4 holds columns 4g .. 4g + 3 of each fragment (8 B); v_permlane16_swap (odd 16-lane rows of
// its first operand <-> even rows of its second, an involution) regroups a pair so that group g holds the
// 8 consecutive columns 16 (g & 1) + 8 (g >> 1) .. + 7 of the 32: one 16-B access per lane instead of two
// 8-B ones.  `base` points at the pair's first column (16-B aligned).
__device__ __forceinline__ int pair_col(const int lane) { return 16 * ((lane >> 4) & 1) + 8 * (lane >> 5); }
__device__ __forceinline__ void pair_store(bf16_t* base, const uint2 a, const uint2 b, const int lane) {
  const auto sx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto sy = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  *reinterpret_cast<uint4*>(base + pair_col(lane)) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
}
__device__ __forceinline__ void pair_load(const bf16_t* base, uint2& a, uint2& b, const int lane) {
  const uint4 v = *reinterpret_cast<const uint4*>(base + pair_col(lane));
  const auto sx = __builtin_amdgcn_permlane16_swap(v.x, v.z, false, false);
  const auto sy = __builtin_amdgcn_permlane16_swap(v.y, v.w, false, false);
  a = make_uint2(sx[0], sy[0]);
  b = make_uint2(sx[1], sy[1]);
}
__device__ __forceinline__ void unpack4(const uint2 v, float (&f)[4]) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

// EPI_BF16_BNR: bf16 store of alpha*acc (+ the residual: optional ReLU bit mask / stride-2 subgrid, as the
// full epilogue adds it) + the BatchNorm-backward partial sums of the stored gradient (GemmParams::bnr_*),
// accumulated like the forward statistics (16-lane shuffle, one atomic per column and shard).  Output rows
// may scatter through the OutMap (a strided data-gradient's parity class): x, the mask and the store then
// use the destination row.  Column-outer so that only one column group's mean / scale / shift is live.
template <int RM, int RN>
__device__ __forceinline__ void gemm_epilogue_bnr(const GemmParams& p, f32x4 (&acc)[RM][RN], const int mb,
                                                  const int nb, const int lane, const int bid, const int mlim) {
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  const bf16_t* X = reinterpret_cast<const bf16_t*>(p.bnr_x);
  float* st = p.stats + (long)(bid % kStatShards) * 2 * p.N;
  float s1[RN][4], s2[RN][4];
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s1[j][e] = s2[j][e] = 0.f;
  // per-row destination and residual row offsets, once per row (the loops below are column-outer; the
  // OutMap / stride-2 subgrid decompositions are two integer divisions each)
  long rowoff[RM], resoff[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = mb + 16 * i + mrow;
    if (p.om.enabled) {
      int nn, ii, jj;
      pix_decompose((uint32_t)m, p.om.gh, p.om.gw, nn, ii, jj);
      rowoff[i] = ((long)(nn * p.om.hy + ii * p.om.so + p.om.oh) * p.om.wy + jj * p.om.so + p.om.ow) * p.ldc;
    } else {
      rowoff[i] = (long)m * p.ldc;
    }
    resoff[i] = -1;
    if (p.resid) {
      long rrow = m;
      if (p.rsub_h) {
        int rn_, ri_, rj_;
        pix_decompose((uint32_t)m, p.rsub_h, p.rsub_w, rn_, ri_, rj_);
        rrow = ((ri_ | rj_) & 1) ? -1L
                                 : ((long)rn_ * ((p.rsub_h + 1) >> 1) + (ri_ >> 1)) * ((p.rsub_w + 1) >> 1) + (rj_ >> 1);
      }
      resoff[i] = rrow < 0 ? -1L : rrow * p.ldr;
    }
  }
  // Fragment pairs whose 32 columns are in range could go through 16-B loads / stores (pair_load /
  // pair_store), but the extra live registers spill in the 128-VGPR 128x128 kernel (0 -> 92 B scratch,
  // ResNet-50 BNR GEMMs 7.80 -> 8.65 ms per 5 steps, profiles/r5/ab_epilogue_kernels.txt): off.
  constexpr bool wide = false;
#pragma unroll
  for (int jp = 0; jp < RN; jp += 2) {
    if (wide && jp + 1 < RN && nb + 16 * jp + 32 <= p.N) {  // wave-uniform
      const int j = jp;
      float mu[2][4], sc[2][4], sh[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int n = nb + 16 * (j + h) + ncol;
        const float4 a = *reinterpret_cast<const float4*>(p.bnr_mean + n);
        mu[h][0] = a.x; mu[h][1] = a.y; mu[h][2] = a.z; mu[h][3] = a.w;
        if (p.bnr_scale) {
          const float4 b = *reinterpret_cast<const float4*>(p.bnr_scale + n);
          const float4 c = *reinterpret_cast<const float4*>(p.bnr_shift + n);
          sc[h][0] = b.x; sc[h][1] = b.y; sc[h][2] = b.z; sc[h][3] = b.w;
          sh[h][0] = c.x; sh[h][1] = c.y; sh[h][2] = c.z; sh[h][3] = c.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) sc[h][e] = sh[h][e] = 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int m = mb + 16 * i + mrow;
        if (m >= mlim) continue;  // (partner lanes of the swaps share m)
        const long off0 = rowoff[i] + nb + 16 * j;  // the pair's first column
        uint2 xv[2], rr[2] = {make_uint2(0, 0), make_uint2(0, 0)};
        pair_load(X + off0, xv[0], xv[1], lane);
        if (p.resid && resoff[i] >= 0)
          pair_load(reinterpret_cast<const bf16_t*>(p.resid) + resoff[i] + nb + 16 * j, rr[0], rr[1], lane);
        uint2 ov[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = nb + 16 * (j + h) + ncol;
          const long off = rowoff[i] + n;
          uint32_t mbits = 0xfu;
          if (p.bnr_mask) mbits = (uint32_t)p.bnr_mask[off >> 3] >> (off & 7);
          float rv[4], x[4];
          unpack4(rr[h], rv);
          unpack4(xv[h], x);
          if (p.resid && p.resid_mask && resoff[i] >= 0) {
            const long bit = (long)m * p.ldr + n;
            const uint32_t rb = (uint32_t)p.resid_mask[bit >> 3] >> (bit & 7);
#pragma unroll
            for (int e = 0; e < 4; ++e) rv[e] = ((rb >> e) & 1u) ? rv[e] : 0.f;
          }
          bf16_t o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = f2bf(__fmul_rn(acc[i][j + h][e], p.alpha) + rv[e]);
            bool keep = (mbits >> e) & 1u;
            if (p.bnr_scale) keep = (x[e] * sc[h][e] + sh[h][e]) > 0.f;
            const float d = keep ? bf2f(o[e]) : 0.f;
            s1[j + h][e] += d;
            s2[j + h][e] += d * (x[e] - mu[h][e]);
          }
          ov[h] = make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
        }
        pair_store(reinterpret_cast<bf16_t*>(p.c) + off0, ov[0], ov[1], lane);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2 && jp + h < RN; ++h) {
        const int j = jp + h;
        const int n = nb + 16 * j + ncol;  // host check: N % 4 == 0, so n < N covers n .. n+3
        const bool nok = n < p.N;
        float mu[4] = {0.f, 0.f, 0.f, 0.f}, sc[4] = {0.f, 0.f, 0.f, 0.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
        if (nok) {
          const float4 a = *reinterpret_cast<const float4*>(p.bnr_mean + n);
          mu[0] = a.x; mu[1] = a.y; mu[2] = a.z; mu[3] = a.w;
          if (p.bnr_scale) {
            const float4 b = *reinterpret_cast<const float4*>(p.bnr_scale + n);
            const float4 c = *reinterpret_cast<const float4*>(p.bnr_shift + n);
            sc[0] = b.x; sc[1] = b.y; sc[2] = b.z; sc[3] = b.w;
            sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w;
          }
        }
    #pragma unroll
        for (int i = 0; i < RM; ++i) {
          const int m = mb + 16 * i + mrow;
          if (!nok || m >= mlim) continue;
          const long off = rowoff[i] + n;
          const uint2 xv = *reinterpret_cast<const uint2*>(X + off);
          uint32_t mbits = 0xfu;
          if (p.bnr_mask) mbits = (uint32_t)p.bnr_mask[off >> 3] >> (off & 7);
          float rv[4] = {0.f, 0.f, 0.f, 0.f};
          if (p.resid) {
            if (resoff[i] >= 0) {
              const uint2 r2 = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(p.resid) + resoff[i] + n);
              rv[0] = __uint_as_float(r2.x << 16);
              rv[1] = __uint_as_float(r2.x & 0xffff0000u);
              rv[2] = __uint_as_float(r2.y << 16);
              rv[3] = __uint_as_float(r2.y & 0xffff0000u);
              if (p.resid_mask) {
                const long bit = (long)m * p.ldr + n;
                const uint32_t rb = (uint32_t)p.resid_mask[bit >> 3] >> (bit & 7);
    #pragma unroll
                for (int e = 0; e < 4; ++e) rv[e] = ((rb >> e) & 1u) ? rv[e] : 0.f;
              }
            }
          }
          float x[4];
          x[0] = __uint_as_float(xv.x << 16);
          x[1] = __uint_as_float(xv.x & 0xffff0000u);
          x[2] = __uint_as_float(xv.y << 16);
          x[3] = __uint_as_float(xv.y & 0xffff0000u);
          bf16_t o[4];
    #pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = f2bf(__fmul_rn(acc[i][j][e], p.alpha) + rv[e]);  // (no fma contraction: the full epilogue's rounding)
            bool keep = (mbits >> e) & 1u;
            if (p.bnr_scale) keep = (x[e] * sc[e] + sh[e]) > 0.f;
            const float d = keep ? bf2f(o[e]) : 0.f;
            s1[j][e] += d;
            s2[j][e] += d * (x[e] - mu[e]);
          }
          *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(p.c) + off) =
              make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
        }
      }
    }
  }
  col_stats_atomics<RN>(s1, s2, st, p.N, nb, lane);
}

// WIDE: the LITE epilogue's paired 16-B stores (off for the gathered-A LDS-DMA kernels: their address state
// leaves no registers for the pair, 0 -> 24 B scratch and +0.03 ms/step on ResNet-50)
template <int RM, int RN, int EPI, bool WIDE = true>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, f32x4 (&acc)[RM][RN], const int mb, const int nb,
                                              const int lane, const int bid, int mend = -1, long coff = 0,
                                              long boff = 0) {
  const int mlim = mend < 0 ? p.M : mend;
  if constexpr (EPI == EPI_BF16_BNR) {
    gemm_epilogue_bnr<RM, RN>(p, acc, mb, nb, lane, bid, mlim);
    return;
  }
  // ---------------------------------- epilogue ----------------------------------
  constexpr bool BF = EPI == EPI_BF16 || EPI == EPI_BF16_LITE;
  constexpr bool LITE = EPI == EPI_BF16_LITE;
  if constexpr (!BF) {
    // fp32 (weight-gradient) epilogue, D orientation: acc[i][j][e] = C[m0+wm0+16i+4(lane>>4)+e][n0+wn0+16j+(lane&15)]
    // -> each atomic wave-instruction covers 4 rows x 64 contiguous bytes.
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = nb + 16 * j + (lane & 15);
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = mb + 16 * i + 4 * (lane >> 4) + e;
          if (m >= mlim) continue;
          float* c = reinterpret_cast<float*>(p.c) + coff + (long)m * p.ldc + n;
          const float v = acc[i][j][e] * p.alpha;
          if constexpr (EPI == EPI_F32) *c = (p.beta != 0.f) ? v + p.beta * *c : v;
          else atomicAdd(c, v);
        }
      }
    }
    return;
  }
  // acc[i][j][e] = C[m = m0+wm0+16i+(lane&15)][n = n0+wn0+16j+4*(lane>>4)+e]: each lane owns
  // 4 consecutive columns of one row -> 8-B (bf16x4) / 16-B (f32x4) vector stores.
  const int mrow = lane & 15;
  const int ncol = 4 * (lane >> 4);
  float s1[RN][4], s2[RN][4];
#pragma unroll
  for (int j = 0; j < RN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) s1[j][e] = s2[j][e] = 0.f;
  const bool vec_ok = (p.ldc % 4) == 0 && (LITE || !p.resid || (p.ldr % 4) == 0);
  // bf16 outputs: fragment pairs (j, j + 1) whose 32 columns are all in range leave as ONE 16-B store per
  // lane (8 consecutive columns) after a v_permlane16_swap: the epilogue's store tail is bound by store
  // INSTRUCTIONS issued (the same bytes in half the instructions)
  // (the full epilogue keeps 8-B stores: its GELU / residual / dropout values leave no registers for the pair
  // in the 128-VGPR 128x128 kernel — 8 -> 36 B scratch, BERT-base -1.2 % — profiles/r5/ab_epilogue_kernels.txt)
  const bool wide_ok = WIDE && LITE && (p.ldc % 8) == 0 && (reinterpret_cast<uintptr_t>(p.c) & 15) == 0;
  // bias of this lane's columns, loaded once: inside the row loop the compiler must re-load it
  // after every output store (p.bias may alias p.c), 4 * RM * RN dependent loads per lane
  // (one 16-B load per fragment column group where the 4 columns are in range: n % 4 == 0 and the
  // bias is a 16-B aligned fp32 vector — host check)
  float bias_r[RN][4];
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int n = nb + 16 * j + ncol;
    if (p.bias && n + 3 < p.N) {
      const float4 bv = *reinterpret_cast<const float4*>(p.bias + boff + n);
      bias_r[j][0] = bv.x;
      bias_r[j][1] = bv.y;
      bias_r[j][2] = bv.z;
      bias_r[j][3] = bv.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) bias_r[j][e] = (p.bias && n + e < p.N) ? p.bias[boff + n + e] : 0.f;
    }
  }
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const int m = mb + 16 * i + mrow;
    if (m >= mlim) continue;
    uint2 pk[RN];  // this row's packed bf16x4 per fragment (BF), stored after the column loop
    long rowoff;
    int nn = 0, ii = 0, jj = 0;
    if (!LITE && p.om.enabled) {
      pix_decompose((uint32_t)m, p.om.gh, p.om.gw, nn, ii, jj);
      rowoff = ((long)(nn * p.om.hy + ii * p.om.so + p.om.oh) * p.om.wy + jj * p.om.so + p.om.ow) * p.ldc;
    } else {
      rowoff = (long)m * p.ldc;
    }
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      const int n = nb + 16 * j + ncol;
      if (n >= p.N) continue;
      const bool full = vec_ok && (n + 3 < p.N);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * p.alpha;
      if constexpr (BF) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bias_r[j][e];
        if (!LITE && p.relu >= ACT_GELU) {  // transformer FFN: GELU fwd (saving the pre-activation) or its gradient
          bf16_t* ax = reinterpret_cast<bf16_t*>(p.aux) + (long)m * p.ldc + n;
          if (p.relu == ACT_GELU) {
            bf16_t pa[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              pa[e] = f2bf(v[e]);
              v[e] = gelu_f(bf2f(pa[e]));
            }
            if (full)
              *reinterpret_cast<uint2*>(ax) = make_uint2((uint32_t)pa[0] | ((uint32_t)pa[1] << 16),
                                                         (uint32_t)pa[2] | ((uint32_t)pa[3] << 16));
            else
              for (int e = 0; e < 4; ++e)
                if (n + e < p.N) ax[e] = pa[e];
          } else {  // one 8-B load of the 4 pre-activations (not four 2-B loads)
            float pre[4];
            if (full) {
              const uint2 av = *reinterpret_cast<const uint2*>(ax);
              pre[0] = __uint_as_float(av.x << 16);
              pre[1] = __uint_as_float(av.x & 0xffff0000u);
              pre[2] = __uint_as_float(av.y << 16);
              pre[3] = __uint_as_float(av.y & 0xffff0000u);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) pre[e] = (n + e < p.N) ? bf2f(ax[e]) : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= (n + e < p.N) ? gelu_grad_f(pre[e]) : 0.f;
          }
        }
        if (!LITE && p.drop_thresh) {
          const unsigned long long base = (unsigned long long)m * (unsigned long long)p.N + (unsigned long long)n;
          const uint32_t kb = drop_bits4(p.drop_seed, base, p.drop_thresh);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = ((kb >> e) & 1u) ? v[e] * p.drop_scale : 0.f;
        }
        long rrow = m;  // residual row of output row m (stride-2 subgrid: -1 = nothing to add)
        if (!LITE && p.resid && p.rsub_h) {
          int rn_, ri_, rj_;
          pix_decompose((uint32_t)m, p.rsub_h, p.rsub_w, rn_, ri_, rj_);
          rrow = ((ri_ | rj_) & 1) ? -1L
                                   : ((long)rn_ * ((p.rsub_h + 1) >> 1) + (ri_ >> 1)) * ((p.rsub_w + 1) >> 1) + (rj_ >> 1);
        }
        if (!LITE && p.resid && rrow >= 0) {
          const bf16_t* r = reinterpret_cast<const bf16_t*>(p.resid) + rrow * p.ldr + n;
          float rv4[4];
          if (full) {
            const uint2 rv = *reinterpret_cast<const uint2*>(r);
            rv4[0] = __uint_as_float(rv.x << 16);
            rv4[1] = __uint_as_float(rv.x & 0xffff0000u);
            rv4[2] = __uint_as_float(rv.y << 16);
            rv4[3] = __uint_as_float(rv.y & 0xffff0000u);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) rv4[e] = (n + e < p.N) ? bf2f(r[e]) : 0.f;
          }
          if (p.resid_mask) {  // bits n .. n+3 of the row's mask (n % 4 == 0: one byte)
            const long bit = (long)m * p.ldr + n;
            const uint32_t mb = (uint32_t)p.resid_mask[bit >> 3] >> (bit & 7);
#pragma unroll
            for (int e = 0; e < 4; ++e) rv4[e] = ((mb >> e) & 1u) ? rv4[e] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += rv4[e];
        }
        if (p.relu == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        bf16_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = f2bf(v[e]);
          const float rr = (n + e < p.N) ? bf2f(o[e]) : 0.f;
          s1[j][e] += rr;
          s2[j][e] += rr * rr;
        }
        bf16_t* c = reinterpret_cast<bf16_t*>(p.c) + coff + rowoff + n;
        pk[j] = make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
        if (wide_ok && (j & 1) == 0 && j + 1 < RN && nb + 16 * j + 32 <= p.N) {
          // stored with fragment j + 1 below
        } else if (wide_ok && (j & 1) == 1 && nb + 16 * j + 16 <= p.N) {
          // pair (j - 1, j), wave-uniform condition (pair_store)
          pair_store(reinterpret_cast<bf16_t*>(p.c) + coff + rowoff + nb + 16 * (j - 1), pk[j - 1], pk[j], lane);
        } else if (full) {
          *reinterpret_cast<uint2*>(c) = pk[j];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) c[e] = o[e];
        }
      } else if constexpr (EPI == EPI_F32) {
        float* c = reinterpret_cast<float*>(p.c) + coff + rowoff + n;
        if (full && p.beta == 0.f) {
          *reinterpret_cast<float4*>(c) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < p.N) c[e] = (p.beta != 0.f) ? v[e] + p.beta * c[e] : v[e];
        }
      } else {
        float* c = reinterpret_cast<float*>(p.c) + coff + rowoff + n;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < p.N) atomicAdd(c + e, v[e]);
      }
    }
    if constexpr (EPI == EPI_BF16) {  // (LITE: no output map)
      if (p.om.enabled && p.om.zero_siblings) {  // this class is the only one with taps: zero the rest
        bf16_t* cb = reinterpret_cast<bf16_t*>(p.c);
        for (int a = 0; a < p.om.so; ++a) {
          const int hy = ii * p.om.so + a;
          if (hy >= p.om.hy) break;
          for (int b = 0; b < p.om.so; ++b) {
            const int wy = jj * p.om.so + b;
            if (wy >= p.om.wy || (a == p.om.oh && b == p.om.ow)) continue;
            bf16_t* z = cb + ((long)(nn * p.om.hy + hy) * p.om.wy + wy) * p.ldc;
#pragma unroll
            for (int j = 0; j < RN; ++j) {
              const int n = nb + 16 * j + ncol;
              if (n + 3 < p.N && vec_ok) *reinterpret_cast<uint2*>(z + n) = make_uint2(0, 0);
              else
                for (int e = 0; e < 4; ++e)
                  if (n + e < p.N) z[n + e] = 0;
            }
          }
        }
      }
    }
  }
  if constexpr (BF) {
    if (p.stats)  // reduce over the 16 rows held by lanes sharing (lane>>4), whole-wave atomics
      col_stats_atomics<RN>(s1, s2, p.stats + (long)(bid % kStatShards) * 2 * p.N, p.N, nb, lane);
  }
}

// Output tile of logical block bid: row-major over the tiles, or (GemmParams::group_m > 1) groups of
// group_m M-tiles walked M-fastest across all N-tiles, so the tiles resident together on one XCD share
// fewer A rows and B columns in its L2.
template <int BM>
__device__ __forceinline__ void tile_raster(const GemmParams& p, int bid, int tiles_n, int& tm, int& tn) {
  if (p.group_m > 1) {
    const int tiles_m = (p.M + BM - 1) / BM;
    const int per = p.group_m * tiles_n;
    const int grp = bid / per, first = grp * p.group_m;
    const int gm = min(tiles_m - first, p.group_m);
    const int r = bid - grp * per;
    tm = first + r % gm;
    tn = r / gm;
  } else {
    tm = bid / tiles_n;
    tn = bid - tm * tiles_n;
  }
}

// The K-tiles are staged with global_load_lds (Operand::dma: no VGPR round trip, no VALU pack, the LDS
// swizzle moved to the source address; padding and out-of-range vectors read ddl_zero_page).
// ST = 1: one LDS stage per block (32 KB at 128x128, so 4 blocks share a CU and each block's load
// latency hides under the others' MFMAs); ST = 3: a 3-slot ring with one barrier per K-tile (the plain
// fp32 weight gradients at 2 workgroups per CU, too few for co-resident blocks alone to hide the DMA).
template <int BM, int BN, int AMODE, int BMODE, int EPI, int ST>
__global__ __launch_bounds__(NTHREADS, (dma_min_blocks<BM, BN, AMODE, BMODE, EPI>())) void gemm_dma_kernel(const GemmParams p) {
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int VA = BM / 32, VB = BN / 32;  // DMA wave-instructions per operand per K-tile
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  constexpr int TAPB = tap_table_bytes<AMODE, BMODE>();
  char* smem = smem_raw + TAPB;

  const int tiles_n = (p.N + BN - 1) / BN;
  int bid, split;
  grid_tile(bid, split);
  int tm, tn;
  tile_raster<BM>(p, bid, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const long zi = blockIdx.z;  // replica of a batched launch (GemmParams::zcount) / parity class (zcls), else 0
  int kz = p.K, tap0 = 0;
  long bz = zi * p.zb, cz = zi * p.zc;
  // parity class zi of a strided data-gradient (GemmParams::zcls; only the gathered bf16 conv instantiation: the
  // extra live values cost the plain 128x128 full-epilogue kernels 16 B/lane of VGPR spills)
  if (AMODE == OP_KC_GATHER && BMODE == OP_KC && EPI == EPI_BF16 && p.zcls) {
    tap0 = p.cls_tap0[zi];
    kz = p.cls_nt[zi] * p.g.tap_c;
    bz = (long)tap0 * p.g.tap_c;
    cz = p.cls_coff[zi];
  }
  const int kbeg = split * p.k_split;
  const int kend = min(kz, kbeg + p.k_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * WTM, wn0 = (wid & 1) * WTN;

  Operand<BM, AMODE> A;
  Operand<BN, BMODE> B;
  if constexpr (TAPB > 0) {
    load_tap_table(reinterpret_cast<int*>(smem_raw), p.g);
    A.tt = (const DDL_LDS int*)(smem_raw) + tap0;
    B.tt = (const DDL_LDS int*)(smem_raw);
  }
  A.init(reinterpret_cast<const bf16_t*>(p.a) + zi * p.za, p.lda, p.M, m0, kz, p.g, kbeg);
  B.init(reinterpret_cast<const bf16_t*>(p.b) + bz, p.ldb, p.N, n0, kz, p.g, kbeg);
  const long zc = (long)split * p.split_stride + cz, zb = zi * p.zbias;
  static_assert(ST == 1 || ST == 3, "stages: 1 or a 3-slot ring");
  auto bfrag = [&](const char* lb, int kk, int j) { return B.frag(lb, kk, j, wn0, lane); };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int buf) { return smem + buf * (A_BYTES + B_BYTES); };
  if constexpr (ST >= 3) {
    // ST-slot ring, ONE barrier per K-tile: ST-1 tiles are issued ahead.  At iteration t the wave
    // waits (counted vmcnt) for its tile-t DMAs only, the barrier then publishes tile t to every
    // wave AND proves every wave has finished reading slot (t-1) % ST (its tile t-1 fragments
    // were consumed by iteration t-1's MFMAs), so that slot is refilled with tile t+ST-1 right
    // after the barrier and loads stay in flight across ST-2 barriers.
    constexpr int PER = VA + VB;
#pragma unroll
    for (int s = 0; s < ST - 1; ++s)
      if (s < nk) {
        A.dma(stage(s), kbeg + s * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
        B.dma(stage(s) + A_BYTES, kbeg + s * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
      }
    int slot = 0;
    for (int t = 0; t < nk; ++t) {
      const int ahead = min(ST - 2, nk - 1 - t);  // tiles issued after tile t still allowed in flight
      if (ahead >= 2) wait_vmcnt<2 * PER>();
      else if (ahead == 1) wait_vmcnt<PER>();
      else wait_vmcnt<0>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + ST - 1 < nk) {
        char* nx = stage(slot == 0 ? ST - 1 : slot - 1);
        A.dma(nx, kbeg + (t + ST - 1) * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
        B.dma(nx + A_BYTES, kbeg + (t + ST - 1) * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
      }
      const char* la = stage(slot);
      const char* lb = la + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < BK / 32; ++kk) {
        bf16x8 af[RM], bf[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = A.frag(la, kk, i, wm0, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) bf[j] = bfrag(lb, kk, j);
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            if constexpr (epi_dt(EPI))
              acc[i][j] = mfma16x16x32(bf[j], af[i], acc[i][j]);
            else
              acc[i][j] = mfma16x16x32(af[i], bf[j], acc[i][j]);
          }
      }
      slot = slot + 1 == ST ? 0 : slot + 1;
    }
    gemm_epilogue<RM, RN, EPI, (AMODE == OP_KC || AMODE == OP_RC)>(p, acc, m0 + wm0, n0 + wn0, lane, bid, -1, zc, zb);
    return;
  }
  if (nk > 0) {
    A.dma(stage(0), kbeg, p.g, p.b_kdiv, p.b_tap_stride, wid);
    B.dma(stage(0) + A_BYTES, kbeg, p.g, p.b_kdiv, p.b_tap_stride, wid);
  }
  for (int t = 0; t < nk; ++t) {
    const char* la = stage(0);
    const char* lb = la + A_BYTES;
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // every wave's tile-t DMAs have landed
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[RM], bf[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = A.frag(la, kk, i, wm0, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[j] = bfrag(lb, kk, j);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          if constexpr (epi_dt(EPI))
            acc[i][j] = mfma16x16x32(bf[j], af[i], acc[i][j]);
          else
            acc[i][j] = mfma16x16x32(af[i], bf[j], acc[i][j]);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading this stage
    if (t + 1 < nk) {
      A.dma(smem, kbeg + (t + 1) * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
      B.dma(smem + A_BYTES, kbeg + (t + 1) * BK, p.g, p.b_kdiv, p.b_tap_stride, wid);
    }
  }

  gemm_epilogue<RM, RN, EPI, (AMODE == OP_KC || AMODE == OP_RC)>(p, acc, m0 + wm0, n0 + wn0, lane, bid, -1, zc, zb);
}

inline int device_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

template <int BM, int BN, int AMODE, int BMODE, int EPI>
inline int launch_tile(const GemmParams& p, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int splits = (p.K + p.k_split - 1) / p.k_split;
  const dim3 grid(tiles, splits > 0 ? splits : 1, p.zcount > 1 ? p.zcount : 1);
  constexpr int TAPB = tap_table_bytes<AMODE, BMODE>();
  if constexpr (AMODE == OP_RC && BMODE == OP_RC && BM * BN < 128 * 128 && (EPI == EPI_F32 || EPI == EPI_F32_ATOMIC)) {
    // the 3-slot ring for plain (1x1 / Linear) weight gradients on 64x128 / 128x64 tiles (72 KB: 2 workgroups
    // per CU), measured 10-25 % faster on the ResNet-50 1x1 layers; only when the grid is one round at 2
    // workgroups per CU and there is more than one K-tile (BERT's longer weight-gradient grids run 4
    // single-stage workgroups per CU; 128x128 tiles would drop to 1 workgroup per CU with the ring)
    if (p.k_split > BK && (long)grid.x * grid.y <= 2L * device_cus()) {
      constexpr int lds = 3 * (BM + BN) * BK * 2 + TAPB;
      static bool attr = [] {  // dynamic LDS above 64 KB must be allowed explicitly
        return lds <= 65536 ||
               hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_dma_kernel<BM, BN, AMODE, BMODE, EPI, 3>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds) == hipSuccess;
      }();
      (void)attr;
      hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, AMODE, BMODE, EPI, 3>), grid, dim3(NTHREADS), lds, s, p);
      return (int)hipGetLastError();
    }
  }
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, AMODE, BMODE, EPI, 1>), grid, dim3(NTHREADS), (BM + BN) * BK * 2 + TAPB,
                     s, p);
  return (int)hipGetLastError();
}

// The bf16 epilogue features a call uses beyond bias / ReLU / statistics.
inline bool needs_full_epilogue(const GemmParams& p) {
  return p.om.enabled || p.resid || p.aux || p.drop_thresh || p.relu > ACT_RELU;
}

template <int AMODE, int BMODE, int EPI>
inline int launch_modes(const GemmParams& p, int tile, hipStream_t s) {
  switch (tile) {
    case 0: return launch_tile<128, 128, AMODE, BMODE, EPI>(p, s);
    case 1: return launch_tile<128, 64, AMODE, BMODE, EPI>(p, s);
    case 2: return launch_tile<64, 128, AMODE, BMODE, EPI>(p, s);
    default: return launch_tile<64, 64, AMODE, BMODE, EPI>(p, s);
  }
}

}  // namespace ddl
