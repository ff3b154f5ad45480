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

namespace ddl {

constexpr int BK = 64;
constexpr int NTHREADS = 256;

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

// ----------------------------------------------------------------------------------------
// Operand loaders. R = tile extent along the operand's row dimension (BM for A, BN for B).
// ----------------------------------------------------------------------------------------
template <int R, int MODE>
struct Operand {
  static constexpr bool KC = (MODE == OP_KC || MODE == OP_KC_GATHER);
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

  __device__ __forceinline__ void init(const void* p, long ld_, int rows_, int r0_, int K_, const ConvGeom& g) {
    ptr = reinterpret_cast<const bf16_t*>(p);
    ld = ld_;
    rows = rows_;
    r0 = r0_;
    K = K_;
    if constexpr (MODE == OP_KC_GATHER) {
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
      }
    }
  }

  __device__ __forceinline__ void load(int k0, const ConvGeom& g, int kdiv, long tap_stride) {
    if constexpr (MODE == OP_KC) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int row = idx >> 3, kc = idx & 7;
        const int r = r0 + row, k = k0 + kc * 8;
        reg[v] = (r < rows && k < K) ? ldg16(ptr + (long)r * ld + k) : make_uint4(0, 0, 0, 0);
      }
    } else if constexpr (MODE == OP_RC) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int krow = idx / (R / 8), rc = idx % (R / 8);
        const int r = r0 + rc * 8, k = k0 + krow;
        reg[v] = (r < rows && k < K) ? ldg16(ptr + (long)k * ld + r) : make_uint4(0, 0, 0, 0);
      }
    } else if constexpr (MODE == OP_KC_GATHER) {
      const int t = k0 / g.tap_c;  // block-uniform: tap_c % 64 == 0
      const int c0 = k0 - t * g.tap_c;
      const int dh = g.dh[t], dw = g.dw[t];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int kc = idx & 7;
        const int ih = hbase[v] + dh, iw = wbase[v] + dw;
        const bool ok = rvalid[v] && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        reg[v] = ok ? ldg16(ptr + ((long)(pixbase[v] + ih * g.wi + iw)) * g.c + c0 + kc * 8) : make_uint4(0, 0, 0, 0);
      }
    } else if constexpr (MODE == OP_RC_GATHER) {
      const int t = r0 / g.tap_c;  // block-uniform: tap_c % R == 0
      const int c0 = r0 - t * g.tap_c;
      const int dh = g.dh[t], dw = g.dw[t];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int krow = idx / (R / 8), rc = idx % (R / 8);
        const int k = k0 + krow;
        int n, i, j;
        pix_decompose((uint32_t)(k < K ? k : 0), g.ho, g.wo, n, i, j);
        const int ih = i * g.sh + dh, iw = j * g.sw + dw;
        const bool ok = k < K && (unsigned)ih < (unsigned)g.hi && (unsigned)iw < (unsigned)g.wi;
        reg[v] = ok ? ldg16(ptr + ((long)((n * g.hi + ih) * g.wi + iw)) * g.c + c0 + rc * 8) : make_uint4(0, 0, 0, 0);
      }
    } else {  // OP_RC_TAPS: k = tap*kdiv + co ; addr = ptr + co*ld + wt[tap]*tap_stride + r
      const int t = k0 / kdiv;  // block-uniform: kdiv % 64 == 0
      const int co0 = k0 - t * kdiv;
      const bf16_t* base = ptr + (long)g.wt[t] * tap_stride;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const int idx = threadIdx.x + v * NTHREADS;
        const int krow = idx / (R / 8), rc = idx % (R / 8);
        const int r = r0 + rc * 8, k = k0 + krow;
        reg[v] = (r < rows && k < K) ? ldg16(base + (long)(co0 + krow) * ld + r) : make_uint4(0, 0, 0, 0);
      }
    }
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

template <int BM, int BN, int AMODE, int BMODE, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_bf16_kernel(const GemmParams p) {
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int RM = WTM / 16, RN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* lds_a0 = smem;
  char* lds_a1 = smem + A_BYTES;
  char* lds_b0 = smem + 2 * A_BYTES;
  char* lds_b1 = smem + 2 * A_BYTES + B_BYTES;

  const int tiles_n = (p.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * p.k_split;
  const int kend = min(p.K, kbeg + p.k_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm0 = (wid >> 1) * WTM, wn0 = (wid & 1) * WTN;

  Operand<BM, AMODE> A;
  Operand<BN, BMODE> B;
  A.init(p.a, p.lda, p.M, m0, p.K, p.g);
  B.init(p.b, p.ldb, p.N, n0, p.K, p.g);

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    A.load(kbeg, p.g, p.b_kdiv, p.b_tap_stride);
    B.load(kbeg, p.g, p.b_kdiv, p.b_tap_stride);
    A.store(lds_a0);
    B.store(lds_b0);
    __syncthreads();
  }
  for (int t = 0; t < nk; ++t) {
    const bool odd = t & 1;
    const char* la = odd ? lds_a1 : lds_a0;
    const char* lb = odd ? lds_b1 : lds_b0;
    const bool more = t + 1 < nk;
    if (more) {
      A.load(kbeg + (t + 1) * BK, p.g, p.b_kdiv, p.b_tap_stride);
      B.load(kbeg + (t + 1) * BK, p.g, p.b_kdiv, p.b_tap_stride);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[RM], bf[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = A.frag(la, kk, i, wm0, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j) bf[j] = B.frag(lb, kk, j, wn0, lane);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = mfma16x16x32(af[i], bf[j], acc[i][j]);
    }
    if (more) {
      A.store(odd ? lds_a0 : lds_a1);
      B.store(odd ? lds_b0 : lds_b1);
    }
    __syncthreads();
  }

  // ---------------------------------- epilogue ----------------------------------
  const int col_l = lane & 15;
  const int row_l = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int n = n0 + wn0 + 16 * j + col_l;
    const bool nok = n < p.N;
    const float bias = (EPI == EPI_BF16 && p.bias && nok) ? p.bias[n] : 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm0 + 16 * i + row_l + e;
        if (m >= p.M || !nok) continue;
        float v = acc[i][j][e] * p.alpha;
        long off;
        if (p.om.enabled) {
          int nn, ii, jj;
          pix_decompose((uint32_t)m, p.om.gh, p.om.gw, nn, ii, jj);
          off = ((long)(nn * p.om.hy + ii * p.om.so + p.om.oh) * p.om.wy + jj * p.om.so + p.om.ow) * p.ldc + n;
        } else {
          off = (long)m * p.ldc + n;
        }
        if constexpr (EPI == EPI_BF16) {
          v += bias;
          if (p.resid) v += bf2f(reinterpret_cast<const bf16_t*>(p.resid)[(long)m * p.ldr + n]);
          if (p.relu) v = fmaxf(v, 0.f);
          const bf16_t o = f2bf(v);
          reinterpret_cast<bf16_t*>(p.c)[off] = o;
          const float r = bf2f(o);
          s1 += r;
          s2 += r * r;
        } else if constexpr (EPI == EPI_F32) {
          float* c = reinterpret_cast<float*>(p.c);
          c[off] = (p.beta != 0.f) ? v + p.beta * c[off] : v;
        } else {
          atomicAdd(reinterpret_cast<float*>(p.c) + off, v);
        }
      }
    }
    if constexpr (EPI == EPI_BF16) {
      if (p.stats) {  // reduce over the 4 row-groups of the wave (lanes l, l^16, l^32, l^48)
        s1 += __shfl_xor(s1, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (lane < 16 && nok) {
          float* st = p.stats + (long)(bid % kStatShards) * 2 * p.N;
          atomicAdd(st + n, s1);
          atomicAdd(st + p.N + n, s2);
        }
      }
    }
  }
}

template <int BM, int BN, int AMODE, int BMODE, int EPI>
inline int launch_tile(const GemmParams& p, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const int splits = (p.K + p.k_split - 1) / p.k_split;
  const size_t lds = 2 * (BM + BN) * BK * 2;
  hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, AMODE, BMODE, EPI>), dim3(tiles, splits > 0 ? splits : 1), dim3(NTHREADS),
                     lds, s, p);
  return (int)hipGetLastError();
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
