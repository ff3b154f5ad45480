// NHWC pooling: max-pool with a byte-sized argmax (window index) so the backward is a
// gather (each input pixel collects from the <= ceil(k/s)^2 windows that cover it; no
// atomics), and global average pooling.  8 channels (16 B) per lane.
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {

__device__ __forceinline__ void unpack8p(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8p(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}

// KH_/KW_/SH_/SW_: compile-time window and stride (0 = the runtime value): with constants the loops
// unroll and the window loads issue together instead of one dependent load per loop trip
// (stem-pool backward 242 -> 212 us, 2x2 / 2 backward 17.2 -> 12.1 us; scripts/bench_pool.py).
// AFF: the input is a pre-BatchNorm tensor; relu(x * scale[c] + shift[c]) is applied to every loaded
// element (the ResNet stem: its BN-apply sweep — a full write and re-read of the largest activation —
// folds into the pool; padding windows are skipped, never compared, so no padded value is transformed).
template <int KH_, int KW_, int SH_, int SW_, bool AFF = false>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const uint4* __restrict__ x, uint4* __restrict__ y,
                                                           uint2* __restrict__ am, int N, int H, int W, int CV, int Ho,
                                                           int Wo, int kh_, int kw_, int sh_, int sw_, int ph, int pw,
                                                           const float* __restrict__ asc = nullptr,
                                                           const float* __restrict__ ash = nullptr) {
  const int kh = KH_ ? KH_ : kh_, kw = KW_ ? KW_ : kw_, sh = SH_ ? SH_ : sh_, sw = SW_ ? SW_ : sw_;
  // 32-bit index math (the launcher guarantees total < 2^31): 64-bit divisions cost ~10x more
  const uint32_t total = (uint32_t)N * Ho * Wo * CV;
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t q = v / (uint32_t)CV, cv = v - q * (uint32_t)CV;
    const uint32_t q2 = q / (uint32_t)Wo, ow = q - q2 * (uint32_t)Wo;
    const int oh = (int)(q2 % (uint32_t)Ho);
    const int n = (int)(q2 / (uint32_t)Ho);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      best[i] = -INFINITY;
      arg[i] = 0;
    }
    float sc[8], sf[8];
    if constexpr (AFF) {
      const float4 a0 = reinterpret_cast<const float4*>(asc)[2 * cv], a1 = reinterpret_cast<const float4*>(asc)[2 * cv + 1];
      const float4 b0 = reinterpret_cast<const float4*>(ash)[2 * cv], b1 = reinterpret_cast<const float4*>(ash)[2 * cv + 1];
      sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
      sf[0] = b0.x; sf[1] = b0.y; sf[2] = b0.z; sf[3] = b0.w; sf[4] = b1.x; sf[5] = b1.y; sf[6] = b1.z; sf[7] = b1.w;
    }
#pragma unroll
    for (int r = 0; r < kh; ++r) {
      const int ih = oh * sh - ph + r;
      if ((unsigned)ih >= (unsigned)H) continue;
#pragma unroll
      for (int s = 0; s < kw; ++s) {
        const int iw = (int)ow * sw - pw + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        float f[8];
        unpack8p(x[(((uint32_t)n * H + ih) * W + iw) * (uint32_t)CV + cv], f);  // < 2^31 (launcher)
        if constexpr (AFF) {
#pragma unroll
          for (int i = 0; i < 8; ++i) f[i] = fmaxf(f[i] * sc[i] + sf[i], 0.f);
        }
        const uint8_t idx = (uint8_t)(r * kw + s);
#pragma unroll
        for (int i = 0; i < 8; ++i)
          if (f[i] > best[i]) {
            best[i] = f[i];
            arg[i] = idx;
          }
      }
    }
    y[v] = pack8p(best);
    uint2 a;
    a.x = (uint32_t)arg[0] | ((uint32_t)arg[1] << 8) | ((uint32_t)arg[2] << 16) | ((uint32_t)arg[3] << 24);
    a.y = (uint32_t)arg[4] | ((uint32_t)arg[5] << 8) | ((uint32_t)arg[6] << 16) | ((uint32_t)arg[7] << 24);
    am[v] = a;
  }
}

// one vector per lane (the grid-stride cap of 8,192 workgroups cost the BN sweeps 2-3 %: bn.hip bn_grid_cap)
static unsigned pgrid(long n) {
  long g = (n + 255) / 256;
  if (g > (1L << 24)) g = 1L << 24;
  return (unsigned)(g > 0 ? g : 1);
}

int maxpool_fwd(const void* x, void* y, uint8_t* argmax, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw,
                int sh, int sw, int ph, int pw, hipStream_t s, const float* scale, const float* shift) {
  const long total = (long)N * Ho * Wo * (C / 8);
  if (total >= (1L << 31) || (long)N * H * W * (C / 8) >= (1L << 31)) return (int)hipErrorInvalidValue;
  if (scale) {  // fused BN + ReLU on load (the VGG block tails' 2x2 / 2 unrolled, else the generic window loop)
    if (!shift || kh > 16 || kw > 16) return (int)hipErrorInvalidValue;
    if (kh == 2 && kw == 2 && sh == 2 && sw == 2)
      hipLaunchKernelGGL((maxpool_fwd_kernel<2, 2, 2, 2, true>), dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)x,
                         (uint4*)y, (uint2*)argmax, N, H, W, C / 8, Ho, Wo, kh, kw, sh, sw, ph, pw, scale, shift);
    else
      hipLaunchKernelGGL((maxpool_fwd_kernel<0, 0, 0, 0, true>), dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)x,
                         (uint4*)y, (uint2*)argmax, N, H, W, C / 8, Ho, Wo, kh, kw, sh, sw, ph, pw, scale, shift);
    return (int)hipGetLastError();
  }
#define DDL_POOL_FWD(A, B, C_, D)                                                                          \
  hipLaunchKernelGGL((maxpool_fwd_kernel<A, B, C_, D>), dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)x, \
                     (uint4*)y, (uint2*)argmax, N, H, W, C / 8, Ho, Wo, kh, kw, sh, sw, ph, pw)
  // the unrolled 3x3 / 2 forward measured slower than the loop (156.7 vs 140.8 us at the stem shape):
  // only the 2x2 / 2 pools take the unrolled form
  if (kh == 2 && kw == 2 && sh == 2 && sw == 2) DDL_POOL_FWD(2, 2, 2, 2);
  else if (kh <= 16 && kw <= 16) DDL_POOL_FWD(0, 0, 0, 0);
  else return (int)hipErrorInvalidValue;
#undef DDL_POOL_FWD
  return (int)hipGetLastError();
}

template <int KH_, int KW_, int SH_, int SW_>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint4* __restrict__ dy, const uint2* __restrict__ am,
                                                           uint4* __restrict__ dx, int N, int H, int W, int CV, int Ho,
                                                           int Wo, int kh_, int kw_, int sh_, int sw_, int ph, int pw) {
  const int kh = KH_ ? KH_ : kh_, kw = KW_ ? KW_ : kw_, sh = SH_ ? SH_ : sh_, sw = SW_ ? SW_ : sw_;
  // at most MH x MW windows cover a pixel: all of their (argmax, dy) pairs load before any compare
  constexpr int MH = KH_ ? (KH_ + SH_ - 1) / SH_ : 16, MW = KW_ ? (KW_ + SW_ - 1) / SW_ : 16;
  const uint32_t total = (uint32_t)N * H * W * CV;  // < 2^31 (launcher): 32-bit index math
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t q = v / (uint32_t)CV, cv = v - q * (uint32_t)CV;
    const uint32_t q2 = q / (uint32_t)W;
    const int w = (int)(q - q2 * (uint32_t)W);
    const int h = (int)(q2 % (uint32_t)H);
    const int n = (int)(q2 / (uint32_t)H);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    // windows covering h: oh*sh - ph <= h <= oh*sh - ph + kh - 1
    int oh0 = h + ph - kh + 1;
    oh0 = oh0 <= 0 ? 0 : (oh0 + sh - 1) / sh;
    const int oh1 = min(Ho - 1, (h + ph) / sh);
    int ow0 = w + pw - kw + 1;
    ow0 = ow0 <= 0 ? 0 : (ow0 + sw - 1) / sw;
    const int ow1 = min(Wo - 1, (w + pw) / sw);
#pragma unroll
    for (int i = 0; i < MH; ++i) {
      const int oh = oh0 + i;
      if (oh > oh1) break;
#pragma unroll
      for (int j = 0; j < MW; ++j) {
        const int ow = ow0 + j;
        if (ow > ow1) break;
        const int idx = (h + ph - oh * sh) * kw + (w + pw - ow * sw);
        const uint32_t o = (((uint32_t)n * Ho + oh) * Wo + ow) * (uint32_t)CV + cv;
        const uint2 a = am[o];
        float g[8];
        unpack8p(dy[o], g);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t word = e < 4 ? a.x : a.y;
          const int ai = (word >> ((e & 3) * 8)) & 0xff;
          if (ai == idx) acc[e] += g[e];
        }
      }
    }
    dx[v] = pack8p(acc);
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool): one lane per 2x2 block of input pixels.  The block's
// pixels are covered by the same <= 2x2 windows (rows 2i, 2i+1 by windows i, i+1), so their four
// (argmax, dy) pairs are loaded once for four outputs instead of once per covered pixel (9 loads
// per block before).
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2p1_kernel(const uint4* __restrict__ dy,
                                                                  const uint2* __restrict__ am, uint4* __restrict__ dx,
                                                                  int N, int H, int W, int CV, int Ho, int Wo) {
  const int HB = (H + 1) >> 1, WB = (W + 1) >> 1;
  const uint32_t total = (uint32_t)N * HB * WB * CV;  // < 2^31 (launcher)
  for (uint32_t v = blockIdx.x * 256u + threadIdx.x; v < total; v += gridDim.x * 256u) {
    const uint32_t q = v / (uint32_t)CV, cv = v - q * (uint32_t)CV;
    const uint32_t q2 = q / (uint32_t)WB;
    const int bj = (int)(q - q2 * (uint32_t)WB);
    const int bi = (int)(q2 % (uint32_t)HB);
    const int n = (int)(q2 / (uint32_t)HB);
    uint2 a[2][2];
    float g[2][2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int oh = bi + i, ow = bj + j;
        if (oh < Ho && ow < Wo) {
          const uint32_t o = (((uint32_t)n * Ho + oh) * Wo + ow) * (uint32_t)CV + cv;
          a[i][j] = am[o];
          unpack8p(dy[o], g[i][j]);
        } else {
          a[i][j] = make_uint2(0xffffffffu, 0xffffffffu);  // no window index matches 0xff
#pragma unroll
          for (int e = 0; e < 8; ++e) g[i][j][e] = 0.f;
        }
      }
#pragma unroll
    for (int pa = 0; pa < 2; ++pa)
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        const int h = 2 * bi + pa, w = 2 * bj + pb;
        if (h >= H || w >= W) continue;
        float acc[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int dr = h + 1 - 2 * (bi + i), dc = w + 1 - 2 * (bj + j);  // position inside window
            if (dr < 0 || dr > 2 || dc < 0 || dc > 2) continue;  // compile-time after unrolling
            const uint32_t idx = (uint32_t)(dr * 3 + dc);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t word = e < 4 ? a[i][j].x : a[i][j].y;
              if (((word >> ((e & 3) * 8)) & 0xffu) == idx) acc[e] += g[i][j][e];
            }
          }
        dx[(((uint32_t)n * H + h) * W + w) * (uint32_t)CV + cv] = pack8p(acc);
      }
  }
}

int maxpool_bwd(const void* dy, const uint8_t* argmax, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh,
                int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  const long total = (long)N * H * W * (C / 8);
  if (total >= (1L << 31)) return (int)hipErrorInvalidValue;
#define DDL_POOL_BWD(A, B, C_, D)                                                                              \
  hipLaunchKernelGGL((maxpool_bwd_kernel<A, B, C_, D>), dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)dy,  \
                     (const uint2*)argmax, (uint4*)dx, N, H, W, C / 8, Ho, Wo, kh, kw, sh, sw, ph, pw)
  if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1) {
    const long blocks = (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
    hipLaunchKernelGGL(maxpool_bwd_k3s2p1_kernel, dim3(pgrid(blocks)), dim3(256), 0, s, (const uint4*)dy,
                       (const uint2*)argmax, (uint4*)dx, N, H, W, C / 8, Ho, Wo);
  } else if (kh == 3 && kw == 3 && sh == 2 && sw == 2) DDL_POOL_BWD(3, 3, 2, 2);
  else if (kh == 2 && kw == 2 && sh == 2 && sw == 2) DDL_POOL_BWD(2, 2, 2, 2);
  else if (kh <= 16 && kw <= 16 && sh >= 1 && sw >= 1) DDL_POOL_BWD(0, 0, 0, 0);
  else return (int)hipErrorInvalidValue;
#undef DDL_POOL_BWD
  return (int)hipGetLastError();
}

__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int N,
                                                           int HW, int CV) {
  const long total = (long)N * CV;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const int cv = (int)(v % CV);
    const long n = v / CV;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    // unrolled: eight independent 16-B loads in flight per lane (the rolled loop waited on each of the 49
    // pixels of ResNet-50's 7x7 map in turn: 27 us for 51 MB)
#pragma unroll 8
    for (int p = 0; p < HW; ++p) {
      float f[8];
      unpack8p(x[(n * HW + p) * CV + cv], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv;
    y[v] = pack8p(acc);
  }
}

int avgpool_global_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  const long total = (long)N * (C / 8);
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)x, (uint4*)y, N, HW, C / 8);
  return (int)hipGetLastError();
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const uint4* __restrict__ dy, uint4* __restrict__ dx, int N,
                                                           int HW, int CV) {
  const long total = (long)N * HW * CV;
  const float inv = 1.f / (float)HW;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const int cv = (int)(v % CV);
    const long n = v / ((long)CV * HW);
    float f[8];
    unpack8p(dy[n * CV + cv], f);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] *= inv;
    dx[v] = pack8p(f);
  }
}

int avgpool_global_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  const long total = (long)N * HW * (C / 8);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(pgrid(total)), dim3(256), 0, s, (const uint4*)dy, (uint4*)dx, N, HW,
                     C / 8);
  return (int)hipGetLastError();
}

}  // namespace ddl
