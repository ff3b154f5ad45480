// Batch normalisation for NHWC activations viewed as [M = N*H*W, C] (C % 8 == 0).
// Training-mode statistics are accumulated per channel with sharded fp32 atomics
// (kBnShards copies, so 1000+ workgroups do not serialise on one cache line), then a
// per-channel finalize turns them into scale/shift.  The apply pass fuses the residual
// add and ReLU of a ResNet block; the backward pass fuses the ReLU mask and writes the
// masked gradient for the residual branch in the same sweep.
// All sweeps move 16 B per lane (8 bf16) — these kernels are HBM-bound by design.
#include "ddl_common.h"
#include "ddl_ops.h"
#include <stdlib.h>

namespace ddl {

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
}

struct ColGeom {  // thread -> (row-lane, column-vector) mapping for column reductions
  int CV, CT, RT, ct, rt, cv;
  bool active;
  __device__ __forceinline__ ColGeom(int C) {
    CV = C >> 3;
    CT = CV < 256 ? CV : 256;
    RT = 256 / CT;
    ct = threadIdx.x % CT;
    rt = threadIdx.x / CT;
    cv = blockIdx.y * CT + ct;
    active = rt < RT && cv < CV;
  }
};

// Block reduction of 16 per-thread partials over the RT row-lanes (LDS tree), then ONE
// plain store per value into partial row blockIdx.x of ws[S][2][C] (no atomics: the
// per-channel finalize sums the S partial rows).
__device__ __forceinline__ void col_reduce_store(float (&acc)[16], const ColGeom& g, float* ws, int C) {
  __shared__ float red[256 * 17];
  if (g.RT > 1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[threadIdx.x * 17 + i] = acc[i];
    __syncthreads();
    for (int n = g.RT; n > 1;) {  // pairwise tree, any RT
      const int half = (n + 1) >> 1;
      const bool take = g.rt < n - half;
      n = half;
      if (take) {
        const int t = (g.rt + half) * g.CT + g.ct;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += red[t * 17 + i];
#pragma unroll
        for (int i = 0; i < 16; ++i) red[threadIdx.x * 17 + i] = acc[i];
      }
      __syncthreads();
    }
  }
  if (g.rt == 0 && g.cv < g.CV) {
    float* dst = ws + (long)blockIdx.x * 2 * C + g.cv * 8;
    *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(dst + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
    *reinterpret_cast<float4*>(dst + C) = make_float4(acc[8], acc[9], acc[10], acc[11]);
    *reinterpret_cast<float4*>(dst + C + 4) = make_float4(acc[12], acc[13], acc[14], acc[15]);
  }
}

__global__ __launch_bounds__(256) void bn_stats_kernel(const uint4* __restrict__ x, float* ws, long M, int C) {
  ColGeom g(C);
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (g.active) {
    const long step = (long)gridDim.x * g.RT;
    long r = (long)blockIdx.x * g.RT + g.rt;
    for (; r + 3 * step < M; r += 4 * step) {  // 4 independent 16-B loads in flight
      uint4 u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) u[q] = x[(r + q * step) * g.CV + g.cv];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float f[8];
        unpack8(u[q], f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] += f[i];
          acc[8 + i] += f[i] * f[i];
        }
      }
    }
    for (; r < M; r += step) {
      float f[8];
      unpack8(x[r * g.CV + g.cv], f);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] += f[i];
        acc[8 + i] += f[i] * f[i];
      }
    }
  }
  col_reduce_store(acc, g, ws, C);
}

// Split-K bf16 finalize: y = bf16(ws + bias) (ReLU) and ws = 0, plus per-column statistics of the ROUNDED
// output (slab form, splits > 0: ws holds `splits` partial slabs `slab_stride` floats apart, summed in
// split order and left as they are — the GEMM overwrites them next time)
// output accumulated into the [kStatShards][2][C] workspace of the GEMM epilogue (shard =
// block % kStatShards).  Convolutions whose output tiles cannot fill the chip (VGG / ResNet layers
// at 2x2-4x4 spatial) run their K loop split over workgroups into an fp32 workspace; this pass
// completes them with the epilogue the un-split GEMM would have applied.
// brows > 0: replica-batched rows — row r adds bias + (r / brows) * zbias (each replica's own bias)
__global__ __launch_bounds__(256) void splitk_finalize_kernel(float4* __restrict__ ws, uint4* __restrict__ y,
                                                              const float* __restrict__ bias, float* stats, long M,
                                                              int C, int relu, int splits, long slab_stride,
                                                              long brows, long zbias) {
  ColGeom g(C);
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (g.active) {
    float b[8];
    const float4 b0 = bias ? reinterpret_cast<const float4*>(bias)[2 * g.cv] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b1 = bias ? reinterpret_cast<const float4*>(bias)[2 * g.cv + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w;
    b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
    const long step = (long)gridDim.x * g.RT;
    for (long r = (long)blockIdx.x * g.RT + g.rt; r < M; r += step) {
      const long idx = r * g.CV + g.cv;
      if (brows > 0 && bias) {
        const float4* bz = reinterpret_cast<const float4*>(bias + (r / brows) * zbias);
        const float4 c0 = bz[2 * g.cv], c1 = bz[2 * g.cv + 1];
        b[0] = c0.x; b[1] = c0.y; b[2] = c0.z; b[3] = c0.w;
        b[4] = c1.x; b[5] = c1.y; b[6] = c1.z; b[7] = c1.w;
      }
      float4 u = ws[2 * idx], v = ws[2 * idx + 1];
      if (splits > 0) {
        const long st4 = slab_stride >> 2;
        for (int sp = 1; sp < splits; ++sp) {
          const float4 a = ws[sp * st4 + 2 * idx], c = ws[sp * st4 + 2 * idx + 1];
          u.x += a.x; u.y += a.y; u.z += a.z; u.w += a.w;
          v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
        }
      } else {
        // leave the workspace zeroed for the next split-K accumulation (no fill launch per call)
        ws[2 * idx] = make_float4(0.f, 0.f, 0.f, 0.f);
        ws[2 * idx + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      float f[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f[i] += b[i];
        if (relu) f[i] = fmaxf(f[i], 0.f);
      }
      const uint4 o = pack8(f);
      y[idx] = o;
      if (stats) {
        float q[8];
        unpack8(o, q);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] += q[i];
          acc[8 + i] += q[i] * q[i];
        }
      }
    }
  }
  if (!stats) return;
  __shared__ float red[256 * 17];
  if (g.RT > 1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[threadIdx.x * 17 + i] = acc[i];
    __syncthreads();
    if (g.rt == 0 && g.active)
      for (int t = 1; t < g.RT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += red[(t * g.CT + g.ct) * 17 + i];
  }
  if (g.rt == 0 && g.active) {
    float* st = stats + (long)(blockIdx.x % kBnShards) * 2 * C + g.cv * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      atomicAdd(st + i, acc[i]);
      atomicAdd(st + C + i, acc[8 + i]);
    }
  }
}

int splitk_finalize(float* ws, void* y, const float* bias, float* stats, long M, int C, int relu, int splits,
                    long slab_stride, hipStream_t s, long brows, long zbias) {
  if (brows > 0 && (stats || zbias % 4)) return (int)hipErrorInvalidValue;
  const int CV = C >> 3, CT = CV < 256 ? CV : 256, RT = 256 / CT;
  const int gy = (CV + CT - 1) / CT;
  long gx = (M + 4 * RT - 1) / (4 * RT);  // >= 4 rows per lane
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(splitk_finalize_kernel, dim3((unsigned)(gx > 0 ? gx : 1), (unsigned)gy), dim3(256), 0, s,
                     (float4*)ws, (uint4*)y, bias, stats, M, C, relu, splits, slab_stride, brows, zbias);
  return (int)hipGetLastError();
}

// partial rows (= grid.x) of a column reduction: >= 16 rows per lane, <= kMaxPartials rows
static dim3 col_grid(long M, int C) {
  const int CV = C >> 3, CT = CV < 256 ? CV : 256, RT = 256 / CT;
  const int gy = (CV + CT - 1) / CT;
  long gx = M / (16L * RT);
  if (gx > kMaxPartials) gx = kMaxPartials;
  if (gx < 1) gx = 1;
  return dim3((unsigned)gx, (unsigned)gy);
}

int bn_partial_rows(long M, int C) { return (int)col_grid(M, C).x; }

int bn_stats(const void* x, float* ws, long M, int C, hipStream_t s) {
  hipLaunchKernelGGL(bn_stats_kernel, col_grid(M, C), dim3(256), 0, s, (const uint4*)x, ws, M, C);
  return (int)hipGetLastError();
}

// Sum of the S partial rows of ws[S][2][C] for 64 channels per block: NL = blockDim / 64
// row-lanes per channel (4 for the 32 shard rows of the fused statistics, 16 for the up to 512
// partial rows of a reduce sweep — one lane per 32 rows instead of 128 keeps the per-layer
// finalize near the launch floor), 4 independent accumulators each, then an LDS combine.
// Returns true in the lane that owns channel c (row-lane 0).
__device__ __forceinline__ bool sum_partials(const float* ws, int S, int C, int& c, double& s1, double& s2) {
  const int NL = blockDim.x >> 6;
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  c = blockIdx.x * 64 + cl;
  double a1 = 0.0, a2 = 0.0;
  if (c < C) {
    float p1[4] = {0.f, 0.f, 0.f, 0.f}, p2[4] = {0.f, 0.f, 0.f, 0.f};
    int k = sl;
    for (; k + 3 * NL < S; k += 4 * NL) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        p1[u] += ws[(long)(k + NL * u) * 2 * C + c];
        p2[u] += ws[(long)(k + NL * u) * 2 * C + C + c];
      }
    }
    for (; k < S; k += NL) {
      p1[0] += ws[(long)k * 2 * C + c];
      p2[0] += ws[(long)k * 2 * C + C + c];
    }
    a1 = (double)p1[0] + p1[1] + p1[2] + p1[3];
    a2 = (double)p2[0] + p2[1] + p2[2] + p2[3];
  }
  __shared__ double red[2][1024];
  red[0][threadIdx.x] = a1;
  red[1][threadIdx.x] = a2;
  __syncthreads();
  if (sl != 0 || c >= C) return false;
  s1 = 0.0;
  s2 = 0.0;
  for (int l = 0; l < NL; ++l) {
    s1 += red[0][cl + 64 * l];
    s2 += red[1][cl + 64 * l];
  }
  return true;
}

// threads of a finalize block: 16 row-lanes for long partial-row lists, 8 for the 32 shard rows (each lane's
// four rows loaded in one round: the kernel is a chain of memory latencies)
static int finalize_threads(int S) { return S > 64 ? 1024 : 512; }

__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* ws, int S, long M, int C, const float* gamma,
                                                          const float* beta, float eps, float momentum, float* rmean,
                                                          float* rvar, float* smean, float* sinv, float* scale,
                                                          float* shift) {
  // the per-channel parameters are loaded first, so their latency overlaps the partial-sum loads (the kernel is
  // a chain of dependent memory latencies: ~5 us per BN, 53 of them per ResNet-50 step)
  const int c0 = blockIdx.x * 64 + (threadIdx.x & 63);
  const bool own = (threadIdx.x >> 6) == 0 && c0 < C;
  const float g = own && gamma ? gamma[c0] : 1.f;
  const float b = own && beta ? beta[c0] : 0.f;
  const float rm = own && rmean ? rmean[c0] : 0.f;
  const float rv = own && rvar ? rvar[c0] : 0.f;
  int c;
  double s1, s2;
  if (!sum_partials(ws, S, C, c, s1, s2)) return;
  const double mean = s1 / (double)M;
  double var = s2 / (double)M - mean * mean;
  if (var < 0) var = 0;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  if (smean) smean[c] = (float)mean;
  if (sinv) sinv[c] = inv;
  scale[c] = g * inv;
  shift[c] = b - (float)mean * g * inv;
  if (rmean) rmean[c] = (1.f - momentum) * rm + momentum * (float)mean;
  if (rvar) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rvar[c] = (1.f - momentum) * rv + momentum * (float)unb;
  }
}

int bn_finalize(const float* ws, int S, long M, int C, const float* gamma, const float* beta, float eps,
                float momentum, float* running_mean, float* running_var, float* save_mean, float* save_invstd,
                float* scale, float* shift, hipStream_t s) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(finalize_threads(S)), 0, s, ws, S, M, C, gamma, beta, eps,
                     momentum, running_mean, running_var, save_mean, save_invstd, scale, shift);
  return (int)hipGetLastError();
}

__device__ __forceinline__ void load8f(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
  f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// ReLU bit mask of a BN with a residual add: one byte per 16-B vector, bit i = channel 8 v + i
// positive, so the backward sweeps load each lane's byte with its data vectors (a byte load in flight
// with them, instead of the dependent scalar loads of a ballot-word layout: bn_bwd_reduce mode 3
// ran at 4.3 TB/s vs 5.5 for mode 2).  The store packs 4 lanes' bytes into one dword (the lanes
// of a wave hold consecutive vectors when CT * RT == 256); otherwise one byte per lane.
__device__ __forceinline__ void store_mask_bits(uint8_t* __restrict__ mask, long idx, uint32_t bits, bool packed) {
  if (packed) {
    // DPP row_shl:n (lane i reads lane i + n inside its 16-lane row): VALU moves, no LDS crossbar
    const int b = (int)(bits & 0xffu);
    const uint32_t w = (uint32_t)b | ((uint32_t)__builtin_amdgcn_update_dpp(0, b, 0x101, 0xf, 0xf, false) << 8) |
                       ((uint32_t)__builtin_amdgcn_update_dpp(0, b, 0x102, 0xf, 0xf, false) << 16) |
                       ((uint32_t)__builtin_amdgcn_update_dpp(0, b, 0x103, 0xf, 0xf, false) << 24);
    if ((threadIdx.x & 3) == 0) *reinterpret_cast<uint32_t*>(mask + idx) = w;
  } else {
    mask[idx] = (uint8_t)bits;
  }
}

// Streaming sweeps use the column-fixed mapping of ColGeom: a lane keeps ONE 8-channel
// vector (per-channel parameters live in registers, no per-element index division) and
// walks rows; R rows are in flight per lane (all R loads issued before the first use).
// bf16x8 store of the streaming sweeps; NT: nontemporal (streaming cache policy: the output is not
// kept in L2 / Infinity Cache ahead of the reads of the sweep)
template <bool NT>
__device__ __forceinline__ void store16(uint4* __restrict__ p, const uint4 v) {
  if constexpr (NT) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
  } else {
    *p = v;
  }
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void bn_apply_kernel(const uint4* __restrict__ x, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, const uint4* __restrict__ res,
                                                        uint4* __restrict__ y, uint8_t* __restrict__ mask, long M,
                                                        int C, int relu, const float* __restrict__ res_scale,
                                                        const float* __restrict__ res_shift) {
  ColGeom g(C);
  if (!g.active) return;
  float sc[8], sh[8], rsc[8], rsh[8];
  load8f(scale + g.cv * 8, sc);
  load8f(shift + g.cv * 8, sh);
  // dual apply: the residual is itself a pre-BN tensor (ResNet downsample shortcut), normalised
  // here instead of in a separate apply sweep that would write and re-read it
  const bool rbn = res_scale != nullptr;
  if (rbn) {
    load8f(res_scale + g.cv * 8, rsc);
    load8f(res_shift + g.cv * 8, rsh);
  }
  const long step = (long)gridDim.x * g.RT;
  for (long r = (long)blockIdx.x * g.RT + g.rt; r < M; r += R * step) {
    long ix[R];
    uint4 xv[R], rv[R];
#pragma unroll
    for (int h = 0; h < R; ++h) {
      const bool ok = r + h * step < M;  // row h of this lane exists (row 0 always does)
      ix[h] = (ok ? r + h * step : r) * g.CV + g.cv;
      xv[h] = x[ix[h]];
      if (res) rv[h] = res[ix[h]];
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
      if (h > 0 && r + h * step >= M) break;
      float f[8], q[8];
      unpack8(xv[h], f);
      if (res) unpack8(rv[h], q);
      uint32_t bits = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float o = f[i] * sc[i] + sh[i];
        if (res) o += rbn ? q[i] * rsc[i] + rsh[i] : q[i];
        bits |= (o > 0.f ? 1u : 0u) << i;
        if (relu) o = fmaxf(o, 0.f);
        f[i] = o;
      }
      store16<NT>(y + ix[h], pack8(f));
      if (mask) store_mask_bits(mask, ix[h], bits, g.CT * g.RT == 256);
    }
  }
}

// workgroup cap of a streaming sweep: effectively none — one workgroup per 2 x RT rows,
// every lane's loads issued at once and never a second grid-stride trip.  The former 4,096-workgroup cap
// (grid-stride loops) measured slower at every value: ResNet-50 11,914-11,928 (4,096) -> 12,018-12,049 (8,192)
// -> 12,106-12,144 (16,384) -> 12,166-12,195 (32,768) -> 12,203-12,217 img/s (65,536 = uncapped at ResNet-50's
// shapes), interleaved (profiles/r4/fuse_bn/ab_bn_grid.txt)
static long bn_grid_cap() { return 1L << 24; }

static dim3 stream_grid(long M, int C, int rows = 2) {
  const int CV = C >> 3, CT = CV < 256 ? CV : 256, RT = 256 / CT;
  const int gy = (CV + CT - 1) / CT;
  long gx = (M + rows * RT - 1) / (rows * RT);
  const long cap = bn_grid_cap() / gy > 1 ? bn_grid_cap() / gy : 1;
  if (gx > cap) gx = cap;
  return dim3((unsigned)(gx > 0 ? gx : 1), (unsigned)gy);
}

// 2 rows in flight per lane of the apply / dx sweeps (4 measured within noise or slower:
// profiles/r4/ab_bn_rows_stem_partials.txt) and nontemporal output stores (plain stores: ResNet-50
// 11,703 / 11,688 vs 11,785 / 11,805 img/s interleaved, profiles/r3/bn_sweeps/ab_bnnt.jsonl)
constexpr int kBnRows = 2;

int bn_apply(const void* x, const float* scale, const float* shift, const void* resid, void* y, void* mask, long M,
             int C, int relu, hipStream_t s, const float* res_scale, const float* res_shift) {
  const int rows = kBnRows;
  auto k = bn_apply_kernel<kBnRows, true>;
  hipLaunchKernelGGL(k, stream_grid(M, C, rows), dim3(256), 0, s, (const uint4*)x, scale, shift, (const uint4*)resid,
                     (uint4*)y, (uint8_t*)mask, M, C, relu, res_scale, res_shift);
  return (int)hipGetLastError();
}

// ReLU mask of the backward: mode 1 reads the forward output y (> 0); mode 2 recomputes
// x*scale+shift > 0 from the BN input already in registers (no extra tensor read: the
// forward computed the same fmaf on the same values); mode 3 reads the bit mask the forward
// apply stored (one byte per 8 channels: 1/16 of the bytes of y) — for BNs with a residual
// add, whose output cannot be recomputed from x alone.
// mode 3's mask byte of vector idx (loaded by the caller with its data vectors)
__device__ __forceinline__ uint32_t mask_byte(const uint4* __restrict__ y, long idx, int mode) {
  return mode == 3 ? (uint32_t)reinterpret_cast<const uint8_t*>(y)[idx] : 0u;
}
__device__ __forceinline__ void relu_mask(float* d, const float* xv, const uint4* __restrict__ y, long idx,
                                          const float* sc, const float* sh, int mode, uint32_t mb = 0) {
  if (mode == 3) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = ((mb >> i) & 1u) ? d[i] : 0.f;
  } else if (mode == 1) {
    float yv[8];
    unpack8(y[idx], yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
  } else if (mode == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = (xv[i] * sc[i] + sh[i]) > 0.f ? d[i] : 0.f;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                             const uint4* __restrict__ y, const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean, float* ws, long M, int C,
                                                             int mode) {
  ColGeom g(C);
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  if (g.active) {
    float mu[8], sc[8], sh[8];
    load8f(mean + g.cv * 8, mu);  // 16-B loads: 24 dependent 4-B loads per lane before the sweep otherwise
    if (mode == 2) {
      load8f(scale + g.cv * 8, sc);
      load8f(shift + g.cv * 8, sh);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) sc[i] = sh[i] = 0.f;
    }
    const long step = (long)gridDim.x * g.RT;
    long r = (long)blockIdx.x * g.RT + g.rt;
    for (; r + 3 * step < M; r += 4 * step) {  // four rows of dy and x in flight per lane
      long ix[4];
      uint4 dd[4], xx[4];
      uint32_t mb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ix[q] = (r + q * step) * g.CV + g.cv;
        dd[q] = dy[ix[q]];
        xx[q] = x[ix[q]];
        mb[q] = mask_byte(y, ix[q], mode);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float d[8], xv[8];
        unpack8(dd[q], d);
        unpack8(xx[q], xv);
        relu_mask(d, xv, y, ix[q], sc, sh, mode, mb[q]);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] += d[i];
          acc[8 + i] += d[i] * (xv[i] - mu[i]);
        }
      }
    }
    for (; r < M; r += step) {
      const long idx = r * g.CV + g.cv;
      float d[8], xv[8];
      unpack8(dy[idx], d);
      unpack8(x[idx], xv);
      relu_mask(d, xv, y, idx, sc, sh, mode, mask_byte(y, idx, mode));
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] += d[i];
        acc[8 + i] += d[i] * (xv[i] - mu[i]);
      }
    }
  }
  col_reduce_store(acc, g, ws, C);
}

int bn_bwd_reduce(const void* dy, const void* x, const void* y, const float* scale, const float* shift,
                  const float* mean, float* ws, long M, int C, int mode, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, col_grid(M, C), dim3(256), 0, s, (const uint4*)dy, (const uint4*)x,
                     (const uint4*)y, scale, shift, mean, ws, M, C, mode);
  return (int)hipGetLastError();
}

// coef[c] = A, coef[C+c] = B, coef[2C+c] = K with dx = A*dy' + B*x + K
//   (= gamma*invstd * (dy' - mean(dy') - xhat * mean(dy'*xhat)))
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* ws, int S, long M, int C,
                                                              const float* gamma, const float* mean,
                                                              const float* invstd, float* dgamma, float* dbeta,
                                                              float* coef) {
  // per-channel operands loaded before the partial sums (latency overlap, as in bn_finalize_kernel)
  const int c0 = blockIdx.x * 64 + (threadIdx.x & 63);
  const bool own = (threadIdx.x >> 6) == 0 && c0 < C;
  const float inv = own ? invstd[c0] : 0.f;
  const float mu = own ? mean[c0] : 0.f;
  const float g = own && gamma ? gamma[c0] : 1.f;
  const float db0 = own && dbeta ? dbeta[c0] : 0.f;
  const float dg0 = own && dgamma ? dgamma[c0] : 0.f;
  int c;
  double d1, d2;
  if (!sum_partials(ws, S, C, c, d1, d2)) return;
  float s1 = (float)d1, s2 = (float)d2;
  s2 *= inv;  // sum dy' * xhat
  if (dbeta) dbeta[c] = db0 + s1;
  if (dgamma) dgamma[c] = dg0 + s2;
  const float A = g * inv;
  const float m1 = s1 / (float)M, m2 = s2 / (float)M;
  coef[c] = A;
  coef[C + c] = -A * m2 * inv;
  coef[2 * C + c] = -A * m1 + A * m2 * inv * mu;
}

int bn_bwd_finalize(const float* ws, int S, long M, int C, const float* gamma, const float* mean, const float* invstd,
                    float* dgamma, float* dbeta, float* coef, hipStream_t s) {
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(finalize_threads(S)), 0, s, ws, S, M, C, gamma,
                     mean, invstd,
                     dgamma, dbeta, coef);
  return (int)hipGetLastError();
}

// RED: the same sweep also produces the backward partial sums of a SECOND BatchNorm that consumes the
// masked gradient d (the ResNet downsample BN, whose input gradient is the block output's masked
// gradient): row blockIdx.x of ws2[S][2][C] gets sum d and sum d * (x2 - mean2) — that BN's reduce sweep
// (a read of d and x2) and the write of d itself (dres) are then not needed.  Grid = col_grid (S rows).
template <int R, bool NT, bool RED>
__global__ __launch_bounds__(256) void bn_bwd_dx_kernel(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                         const uint4* __restrict__ y, const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const float* __restrict__ coef, uint4* __restrict__ dx,
                                                         uint4* __restrict__ dres, long M, int C, int mode,
                                                         const uint4* __restrict__ x2, const float* __restrict__ mean2,
                                                         float* ws2) {
  ColGeom g(C);
  float acc[RED ? 16 : 1];
  float mu2[RED ? 8 : 1];
  if constexpr (RED) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (g.active) load8f(mean2 + g.cv * 8, mu2);
  }
  if (g.active) {  // (inactive threads still join the RED block's LDS tree below)
  const int c = g.cv * 8;
  float A[8], B[8], K[8], sc[8], sh[8];
  load8f(coef + c, A);
  load8f(coef + C + c, B);
  load8f(coef + 2 * C + c, K);
  if (mode == 2) {
    load8f(scale + c, sc);
    load8f(shift + c, sh);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) sc[i] = sh[i] = 0.f;
  }
  const long step = (long)gridDim.x * g.RT;
  for (long r = (long)blockIdx.x * g.RT + g.rt; r < M; r += R * step) {
    long ix[R];
    uint4 dv[R], xv[R], x2v[RED ? R : 1];
    uint32_t mb[R];
#pragma unroll
    for (int h = 0; h < R; ++h) {
      const bool ok = r + h * step < M;
      ix[h] = (ok ? r + h * step : r) * g.CV + g.cv;
      dv[h] = dy[ix[h]];
      xv[h] = x[ix[h]];
      if constexpr (RED) x2v[h] = x2[ix[h]];
      mb[h] = mask_byte(y, ix[h], mode);
    }
#pragma unroll
    for (int h = 0; h < R; ++h) {
      if (h > 0 && r + h * step >= M) break;
      float d[8], xf[8], o[8];
      unpack8(dv[h], d);
      unpack8(xv[h], xf);
      relu_mask(d, xf, y, ix[h], sc, sh, mode, mb[h]);
      if (dres) store16<NT>(dres + ix[h], pack8(d));
      if constexpr (RED) {
        float x2f[8];
        unpack8(x2v[h], x2f);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          acc[i] += d[i];
          acc[8 + i] += d[i] * (x2f[i] - mu2[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = A[i] * d[i] + B[i] * xf[i] + K[i];
      store16<NT>(dx + ix[h], pack8(o));
    }
  }
  }  // g.active
  if constexpr (RED) col_reduce_store(acc, g, ws2, C);
}

int bn_bwd_dx(const void* dy, const void* x, const void* y, const float* scale, const float* shift, const float* coef,
              void* dx, void* dres, long M, int C, int mode, hipStream_t s, const void* x2, const float* mean2,
              float* ws2) {
  const int rows = kBnRows;
  if (x2) {  // fused second-BN reduce: partial row per block, so the reduction's grid (S = bn_partial_rows)
    auto k = bn_bwd_dx_kernel<kBnRows, true, true>;
    hipLaunchKernelGGL(k, col_grid(M, C), dim3(256), 0, s, (const uint4*)dy, (const uint4*)x, (const uint4*)y, scale,
                       shift, coef, (uint4*)dx, (uint4*)dres, M, C, mode, (const uint4*)x2, mean2, ws2);
    return (int)hipGetLastError();
  }
  auto k = bn_bwd_dx_kernel<kBnRows, true, false>;
  hipLaunchKernelGGL(k, stream_grid(M, C, rows), dim3(256), 0, s, (const uint4*)dy, (const uint4*)x, (const uint4*)y,
                     scale, shift, coef, (uint4*)dx, (uint4*)dres, M, C, mode, (const uint4*)nullptr,
                     (const float*)nullptr, (float*)nullptr);
  return (int)hipGetLastError();
}

}  // namespace ddl

namespace ddl {

// ResNet stem backward through its fused 3x3 / stride-2 / pad-1 max pool (the pool applied the BN affine +
// ReLU on load, _StemPoolFn): the BN's output gradient d is the pool's gather of the pooled gradient dy over
// the (<= 2 x 2) windows whose argmax byte names the pixel — recomputed here from dy and the argmax in both
// passes instead of being written out (411 MB at batch 256) and read back twice:
//   DX = false: backward partial sums sum d' and sum d' (x - mean) (d' = d under the ReLU mask recomputed
//               from x: mode 2) into partial row blockIdx.x of ws[S][2][C] — the reduce sweep;
//   DX = true : dx = A d' + B x + K with the finalize's coefficients — the dx sweep.
// A thread owns a 2 x 2 pixel block of one 8-channel vector (the four pooled outputs that can cover it are
// loaded once); the ColGeom mapping keeps that vector fixed per thread for the column reduction.
// PK = 2: the same for a 2 x 2 / stride-2 pool (VGG block tails, ops/fused_blocks.py:_ConvBNPoolFn), whose
// window (bi, bj) is exactly the thread's pixel block.
template <bool DX, int PK>
__global__ __launch_bounds__(256) void pool3s2_bn_bwd_kernel(const uint4* __restrict__ dy, const uint2* __restrict__ am,
                                                              const uint4* __restrict__ x, const float* __restrict__ scale,
                                                              const float* __restrict__ shift, const float* __restrict__ mean,
                                                              const float* __restrict__ coef, float* ws,
                                                              uint4* __restrict__ dx, int N, int H, int W, int Ho, int Wo,
                                                              int C) {
  ColGeom g(C);
  float acc[DX ? 1 : 16];
  if constexpr (!DX) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  }
  if (g.active) {
    const int CV = g.CV, cv = g.cv, c = cv * 8;
    float sc[8], sh[8], p0[8], p1[8], p2[8];
    load8f(scale + c, sc);
    load8f(shift + c, sh);
    if constexpr (DX) {
      load8f(coef + c, p0);
      load8f(coef + C + c, p1);
      load8f(coef + 2 * C + c, p2);
    } else {
      load8f(mean + c, p0);
    }
    const int HB = (H + 1) >> 1, WB = (W + 1) >> 1;
    const uint32_t nq = (uint32_t)N * HB * WB;  // < 2^31 / CV (launcher)
    for (uint32_t q = blockIdx.x * (uint32_t)g.RT + g.rt; q < nq; q += gridDim.x * (uint32_t)g.RT) {
      const uint32_t q2 = q / (uint32_t)WB;
      const int bj = (int)(q - q2 * (uint32_t)WB);
      const int bi = (int)(q2 % (uint32_t)HB);
      const int n = (int)(q2 / (uint32_t)HB);
      constexpr int NW = PK == 3 ? 2 : 1;  // pooled windows that can cover a pixel of the block, per axis
      uint2 a[2][2];
      uint4 gv[2][2], xv[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int oh = bi + i, ow = bj + j;
          if (i < NW && j < NW && oh < Ho && ow < Wo) {
            const uint32_t o = (((uint32_t)n * Ho + oh) * Wo + ow) * (uint32_t)CV + cv;
            a[i][j] = am[o];
            gv[i][j] = dy[o];
          } else {
            a[i][j] = make_uint2(0xffffffffu, 0xffffffffu);  // no window index matches 0xff
            gv[i][j] = make_uint4(0, 0, 0, 0);
          }
          const int h = 2 * bi + i, w = 2 * bj + j;  // pixel (pa, pb) = (i, j) of the block
          xv[i][j] = (h < H && w < W) ? x[(((uint32_t)n * H + h) * W + w) * (uint32_t)CV + cv] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
      for (int pa = 0; pa < 2; ++pa)
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
          const int h = 2 * bi + pa, w = 2 * bj + pb;
          if (h >= H || w >= W) continue;
          float d[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = 0.f;
#pragma unroll
          for (int i = 0; i < NW; ++i)
#pragma unroll
            for (int j = 0; j < NW; ++j) {
              // position inside window (bi + i, bj + j): 3x3 / 2 / pad 1 windows start one row / column before
              // the block, 2x2 / 2 windows at it
              const int dr = PK == 3 ? h + 1 - 2 * (bi + i) : pa, dc = PK == 3 ? w + 1 - 2 * (bj + j) : pb;
              if (dr < 0 || dr >= PK || dc < 0 || dc >= PK) continue;  // compile-time after unrolling
              const uint32_t idx = (uint32_t)(dr * PK + dc);
              float gf[8];
              unpack8(gv[i][j], gf);
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const uint32_t word = e < 4 ? a[i][j].x : a[i][j].y;
                if (((word >> ((e & 3) * 8)) & 0xffu) == idx) d[e] += gf[e];
              }
            }
          float xf[8];
          unpack8(xv[pa][pb], xf);
          // d is the bf16 value the separate pool backward would have stored (at most two windows add)
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = (xf[e] * sc[e] + sh[e]) > 0.f ? bf2f(f2bf(d[e])) : 0.f;
          if constexpr (DX) {
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = p0[e] * d[e] + p1[e] * xf[e] + p2[e];
            dx[(((uint32_t)n * H + h) * W + w) * (uint32_t)CV + cv] = pack8(o);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              acc[e] += d[e];
              acc[8 + e] += d[e] * (xf[e] - p0[e]);
            }
          }
        }
    }
  }
  if constexpr (!DX) col_reduce_store(acc, g, ws, C);
}

bool pool3s2_bn_bwd_ok(int N, int H, int W, int C, int Ho, int Wo, int k) {
  const bool shape = k == 3 ? (Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1) : (k == 2 && Ho == H / 2 && Wo == W / 2);
  return shape && C % 8 == 0 && C / 8 <= 256 &&
         (long)N * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8) < (1L << 31) && (long)N * H * W * (C / 8) < (1L << 31);
}

int pool3s2_bn_bwd(const void* dy, const uint8_t* am, const void* x, const float* scale, const float* shift,
                   const float* mean, const float* coef, float* ws, int S, void* dx, int N, int H, int W, int C, int Ho,
                   int Wo, hipStream_t s, int k) {
  if (!pool3s2_bn_bwd_ok(N, H, W, C, Ho, Wo, k)) return (int)hipErrorInvalidValue;
  const int CV = C / 8, CT = CV, RT = 256 / CT;
  const long nq = (long)N * ((H + 1) / 2) * ((W + 1) / 2);
  if (dx) {
    const long gx = (nq + RT - 1) / RT;  // one 2 x 2 block per lane, no grid-stride trips (see bn_grid_cap)
    if (k == 3)
      hipLaunchKernelGGL((pool3s2_bn_bwd_kernel<true, 3>), dim3((unsigned)gx), dim3(256), 0, s, (const uint4*)dy,
                         (const uint2*)am, (const uint4*)x, scale, shift, mean, coef, ws, (uint4*)dx, N, H, W, Ho, Wo, C);
    else
      hipLaunchKernelGGL((pool3s2_bn_bwd_kernel<true, 2>), dim3((unsigned)gx), dim3(256), 0, s, (const uint4*)dy,
                         (const uint2*)am, (const uint4*)x, scale, shift, mean, coef, ws, (uint4*)dx, N, H, W, Ho, Wo, C);
  } else {  // one partial row per block: S blocks (the caller's workspace rows; more than a reduce sweep's 512:
            // each thread's 2 x 2 gather is latency-bound, so the sweep needs the extra waves in flight)
    if (S < 1) return (int)hipErrorInvalidValue;
    if (k == 3)
      hipLaunchKernelGGL((pool3s2_bn_bwd_kernel<false, 3>), dim3((unsigned)S), dim3(256), 0, s, (const uint4*)dy,
                         (const uint2*)am, (const uint4*)x, scale, shift, mean, coef, ws, (uint4*)nullptr, N, H, W, Ho,
                         Wo, C);
    else
      hipLaunchKernelGGL((pool3s2_bn_bwd_kernel<false, 2>), dim3((unsigned)S), dim3(256), 0, s, (const uint4*)dy,
                         (const uint2*)am, (const uint4*)x, scale, shift, mean, coef, ws, (uint4*)nullptr, N, H, W, Ho,
                         Wo, C);
  }
  (void)CT;
  return (int)hipGetLastError();
}

}  // namespace ddl
