// Data-movement kernels: casts, ReLU backward, adds, bias gradients, im2col for the
// convolutions whose channel count does not fit the implicit-GEMM gather (C % 64 != 0,
// e.g. the 3-channel stem and the MNIST CNN), and the fused ingest normaliser
// (uint8 NHWC images -> bf16, channel padded) that runs right after the H2D copy.
#include "ddl_common.h"
#include "ddl_ops.h"
#include <stdlib.h>

namespace ddl {

// deterministic-reduction switch (ddl_ops.h); read by the launchers on the host, never by a kernel
static int g_deterministic = 0;
void set_deterministic(int on) { g_deterministic = on ? 1 : 0; }
int deterministic() { return g_deterministic; }

// one element group per lane (a former cap of 8,192 workgroups cost the sweeps 2-3 %: bn.hip bn_grid_cap)
static long misc_grid_cap() { return 1L << 24; }
static unsigned mgrid(long n) {
  long g = (n + 255) / 256;
  if (g > misc_grid_cap()) g = misc_grid_cap();
  return (unsigned)(g > 0 ? g : 1);
}

#define GRID_LOOP(i, n) for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < (n); i += (long)gridDim.x * 256)

__global__ void cast_f32_bf16_kernel(const float4* x, uint2* y, long n4) {
  GRID_LOOP(i, n4) {
    const float4 v = x[i];
    y[i] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
}
__global__ void cast_f32_bf16_tail(const float* x, bf16_t* y, long start, long n) {
  const long i = start + threadIdx.x;
  if (i < n) y[i] = f2bf(x[i]);
}

int cast_f32_bf16(const float* x, void* y, long n, hipStream_t s) {
  const long n4 = n / 4;
  if (n4) hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(mgrid(n4)), dim3(256), 0, s, (const float4*)x, (uint2*)y, n4);
  if (n % 4) hipLaunchKernelGGL(cast_f32_bf16_tail, dim3(1), dim3(4), 0, s, x, (bf16_t*)y, n4 * 4, n);
  return (int)hipGetLastError();
}

__global__ void cast_bf16_f32_kernel(const bf16_t* x, float* y, long n) {
  GRID_LOOP(i, n) y[i] = bf2f(x[i]);
}

int cast_bf16_f32(const void* x, float* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(mgrid(n)), dim3(256), 0, s, (const bf16_t*)x, y, n);
  return (int)hipGetLastError();
}

// y[i] = bf16( sum_r x[r][i] ) with an fp32 accumulator: the local reduction step of the bf16-wire
// gradient all-reduce (parallel/ddp.py: all-to-all of bf16 chunks -> this sum -> all-gather), so the
// sum over ranks is rounded to bf16 once instead of after every ring hop.  8 columns per lane
// (n % 8 == 0, 16-B aligned rows: host check).
__global__ __launch_bounds__(256) void sum_rows_bf16_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, int R,
                                                            long n8) {
  GRID_LOOP(i, n8) {
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < R; ++r) {
      const uint4 v = x[(long)r * n8 + i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[2 * q] += __uint_as_float(w[q] << 16);
        a[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
      }
    }
    y[i] = make_uint4(pack_bf16x2(a[0], a[1]), pack_bf16x2(a[2], a[3]), pack_bf16x2(a[4], a[5]),
                      pack_bf16x2(a[6], a[7]));
  }
}

int sum_rows_bf16(const void* x, void* y, int R, long n, hipStream_t s) {
  const long n8 = n / 8;
  hipLaunchKernelGGL(sum_rows_bf16_kernel, dim3(mgrid(n8)), dim3(256), 0, s, (const uint4*)x, (uint4*)y, R, n8);
  return (int)hipGetLastError();
}

// x *= s_dev[0] in place (bf16): an upstream gradient that lives on the device (a loss node's
// incoming gradient), applied without reading it back to the host
__global__ __launch_bounds__(256) void scale_bf16_dev_kernel(uint4* __restrict__ x, long n8, const float* __restrict__ sd) {
  const float sc = sd[0];
  GRID_LOOP(i, n8) {
    const uint4 v = x[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pack_bf16x2(__uint_as_float(w[q] << 16) * sc, __uint_as_float(w[q] & 0xffff0000u) * sc);
    x[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

int scale_bf16_dev(void* x, long n, const float* s_dev, hipStream_t s) {
  hipLaunchKernelGGL(scale_bf16_dev_kernel, dim3(mgrid(n / 8)), dim3(256), 0, s, (uint4*)x, n / 8, s_dev);
  return (int)hipGetLastError();
}

__global__ void relu_bwd_kernel(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long n) {
  GRID_LOOP(i, n) dx[i] = bf2f(y[i]) > 0.f ? dy[i] : (bf16_t)0;
}

int relu_bwd(const void* dy, const void* y, void* dx, long n, hipStream_t s) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(mgrid(n)), dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)y,
                     (bf16_t*)dx, n);
  return (int)hipGetLastError();
}

__global__ void add_bf16_kernel(const bf16_t* a, const bf16_t* b, bf16_t* y, long n) {
  GRID_LOOP(i, n) y[i] = f2bf(bf2f(a[i]) + bf2f(b[i]));
}

int add_bf16(const void* a, const void* b, void* y, long n, hipStream_t s) {
  hipLaunchKernelGGL(add_bf16_kernel, dim3(mgrid(n)), dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)y,
                     n);
  return (int)hipGetLastError();
}

// out[r][k] = k < K ? x[r * ldx + k] : 0 for r < R, k < Kp: a zero-padded [R][Kp] copy of a row-strided
// [R][K] view (the 16-B-vector width of the GEMM operands; params.py keeps weights padded, this pads
// activations that arrive unpadded).  One lane per output pair of columns.
__global__ __launch_bounds__(256) void pad_cols_bf16_kernel(const bf16_t* __restrict__ x, long ldx,
                                                            bf16_t* __restrict__ out, long R, int K, int Kp) {
  const int kh = Kp >> 1;
  GRID_LOOP(i, R * kh) {
    const long r = i / kh;
    const int k = (int)(i - r * kh) * 2;
    const bf16_t* xr = x + r * ldx;
    const unsigned lo = k < K ? (unsigned)xr[k] : 0u;
    const unsigned hi = k + 1 < K ? (unsigned)xr[k + 1] : 0u;
    reinterpret_cast<unsigned*>(out)[i] = lo | (hi << 16);
  }
}

// Several buffers zeroed by ONE launch (a training step's statistics workspaces and gradient arena):
// 16-B vector stores over the concatenated ranges, each range's < 16-B tail by the first workgroup.
__global__ __launch_bounds__(256) void zero_ranges_kernel(const ZeroRanges r) {
  GRID_LOOP(i, r.pre[r.count]) {
    int k = 0;
    while (k + 1 < r.count && i >= r.pre[k + 1]) ++k;
    reinterpret_cast<uint4*>(r.p[k])[i - r.pre[k]] = make_uint4(0u, 0u, 0u, 0u);
  }
  if (blockIdx.x == 0 && (int)threadIdx.x < r.count * 3) {
    const int k = threadIdx.x / 3, w = threadIdx.x % 3;
    if (w < r.tail_words[k])
      reinterpret_cast<uint32_t*>(r.p[k])[(r.pre[k + 1] - r.pre[k]) * 4 + w] = 0u;
  }
}

int zero_ranges(const ZeroRanges& r, hipStream_t s) {
  if (r.count <= 0 || r.count > kMaxZeroRanges) return r.count == 0 ? 0 : (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(zero_ranges_kernel, dim3(mgrid(r.pre[r.count] > 0 ? r.pre[r.count] : 1)), dim3(256), 0, s, r);
  return (int)hipGetLastError();
}

// Table-driven re-layout of a small weight: out[i] = idx[i] >= 0 ? src[idx[i]] : 0 (bf16), and its
// adjoint for the gradient, dst[idx[i]] += src[i] (fp32; idx injective, so no atomics) — the ResNet stem's
// space-to-depth filter (ops/fused_blocks.py) without the torch pad / permute / add kernels.
__global__ void gather_bf16_kernel(const bf16_t* __restrict__ src, const int* __restrict__ idx, bf16_t* __restrict__ out, long n) {
  GRID_LOOP(i, n) {
    const int j = idx[i];
    out[i] = j >= 0 ? src[j] : (bf16_t)0;
  }
}
__global__ void scatter_add_f32_kernel(const float* __restrict__ src, const int* __restrict__ idx, float* __restrict__ dst, long n) {
  GRID_LOOP(i, n) {
    const int j = idx[i];
    if (j >= 0) dst[j] += src[i];
  }
}
int gather_bf16(const void* src, const int* idx, void* out, long n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gather_bf16_kernel, dim3(mgrid(n)), dim3(256), 0, s, (const bf16_t*)src, idx, (bf16_t*)out, n);
  return (int)hipGetLastError();
}
int scatter_add_f32(const float* src, const int* idx, float* dst, long n, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scatter_add_f32_kernel, dim3(mgrid(n)), dim3(256), 0, s, src, idx, dst, n);
  return (int)hipGetLastError();
}

int pad_cols_bf16(const void* x, long ldx, void* out, long R, int K, int Kp, hipStream_t s) {
  if (Kp % 2 || K > Kp || ldx < K) return (int)hipErrorInvalidValue;
  if (R <= 0) return 0;
  hipLaunchKernelGGL(pad_cols_bf16_kernel, dim3(mgrid(R * (Kp / 2))), dim3(256), 0, s, (const bf16_t*)x, ldx,
                     (bf16_t*)out, R, K, Kp);
  return (int)hipGetLastError();
}

// db[n] += sum_m dy[m][n]; grid (col blocks, row splits) with one atomic per column per block
__global__ void bias_grad_kernel(const bf16_t* dy, float* db, long M, int N) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float acc = 0.f;
  for (long m = blockIdx.y; m < M; m += gridDim.y) acc += bf2f(dy[m * N + n]);
  atomicAdd(db + n, acc);
}

// Vector form for N % 8 == 0 and 16-byte aligned rows: a block covers 256 columns as 32 lanes of
// 8 bf16 (one 16-byte load each) x 8 row-lanes, reduces the row-lanes through LDS and issues one
// atomic per column per block.  The scalar form above moved 2 bytes per lane per load.
// pout != nullptr (deterministic mode): each workgroup stores its column totals to pout[blockIdx.y][n]
// instead of adding them into db; colsum_partials then sums the rows in index order, one writer per column
// ry != nullptr: the ReLU backward is fused in: dy is masked by ry > 0, the masked rows are stored to rdx
// and summed (a Dense / Conv2D with a fused ReLU: one sweep instead of relu_bwd + bias_grad)
// blockIdx.z = replica z of a batched launch: rows z*M.. of dy / ry / rdx, db + z * zdb
__global__ __launch_bounds__(256) void bias_grad_vec_kernel(const bf16_t* dy, float* db, long M, int N, float* pout,
                                                            const bf16_t* __restrict__ ry = nullptr,
                                                            bf16_t* __restrict__ rdx = nullptr, long zdb = 0) {
  __shared__ float part[8][257];
  if (blockIdx.z) {
    const long zr = (long)blockIdx.z * M * N;
    dy += zr;
    db += (long)blockIdx.z * zdb;
    if (ry) {
      ry += zr;
      rdx += zr;
    }
  }
  const int cg = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n0 = blockIdx.x * 256 + cg * 8;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (n0 < N && !ry) {
    // plain column sums: four rows' 16-B loads in flight per lane before their adds (one dependent load per
    // row was latency-bound: 22 us for BERT's 16384 x 2304 QKV gradient, 3.4 TB/s)
    const long step = (long)gridDim.y * 8;
    long m = (long)blockIdx.y * 8 + rl;
    for (; m + 3 * step < M; m += 4 * step) {
      uint4 q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) q[r] = *reinterpret_cast<const uint4*>(dy + (m + r * step) * N + n0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned u[4] = {q[r].x, q[r].y, q[r].z, q[r].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          acc[2 * k] += __uint_as_float(u[k] << 16);
          acc[2 * k + 1] += __uint_as_float(u[k] & 0xffff0000u);
        }
      }
    }
    for (; m < M; m += step) {
      const uint4 q = *reinterpret_cast<const uint4*>(dy + m * N + n0);
      const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(u[k] << 16);
        acc[2 * k + 1] += __uint_as_float(u[k] & 0xffff0000u);
      }
    }
  } else if (n0 < N) {
    for (long m = (long)blockIdx.y * 8 + rl; m < M; m += (long)gridDim.y * 8) {
      uint4 q = *reinterpret_cast<const uint4*>(dy + m * N + n0);
      if (ry) {
        const uint4 yv = *reinterpret_cast<const uint4*>(ry + m * N + n0);
        // bf16 > 0: sign bit clear and any other bit set, per 16-bit half
        auto msk = [](unsigned d, unsigned y) {
          const unsigned lo = ((y & 0x8000u) == 0 && (y & 0x7fffu) != 0) ? 0xffffu : 0u;
          const unsigned hi = ((y & 0x80000000u) == 0 && (y & 0x7fff0000u) != 0) ? 0xffff0000u : 0u;
          return d & (lo | hi);
        };
        q = make_uint4(msk(q.x, yv.x), msk(q.y, yv.y), msk(q.z, yv.z), msk(q.w, yv.w));
        *reinterpret_cast<uint4*>(rdx + m * N + n0) = q;
      }
      const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(u[k] << 16);
        acc[2 * k + 1] += __uint_as_float(u[k] & 0xffff0000u);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) part[rl][cg * 8 + k] = acc[k];
  __syncthreads();
  const int c = threadIdx.x, n = blockIdx.x * 256 + c;
  if (n < N) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) t += part[r][c];
    if (pout) pout[(long)blockIdx.y * N + n] = t;
    else atomicAdd(db + n, t);
  }
}

// c[m][n] = beta * c[m][n] + sum_s ws[s][m][n] (slabs [splits][M][N], contiguous), summed in split order by
// ONE lane per element: the reduce of split-K partial slabs (GemmParams::split_stride).  float4 per lane
// when N and ldc are multiples of 4.
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ ws, int splits, float* __restrict__ c,
                                                          long M, int N, long ldc, float beta, int vec) {
  const long slab = M * (long)N;
  if (vec) {
    const long n4 = slab >> 2;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
      float4 a = reinterpret_cast<const float4*>(ws)[i];
      int sp = 1;
      // four slab loads in flight per step (a dependent load-add chain per slab was latency-bound: 33 us
      // for the 8 x 9.4 MB of a BERT FFN weight gradient); the adds keep split order (same bits)
      for (; sp + 3 < splits; sp += 4) {
        float4 b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = reinterpret_cast<const float4*>(ws + (sp + q) * slab)[i];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          a.x += b[q].x; a.y += b[q].y; a.z += b[q].z; a.w += b[q].w;
        }
      }
      for (; sp < splits; ++sp) {
        const float4 b = reinterpret_cast<const float4*>(ws + sp * slab)[i];
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
      const long e = i << 2, m = e / N, n = e - m * N;
      float4* cp = reinterpret_cast<float4*>(c + m * ldc + n);
      if (beta != 0.f) {
        const float4 o = *cp;
        a.x += beta * o.x; a.y += beta * o.y; a.z += beta * o.z; a.w += beta * o.w;
      }
      *cp = a;
    }
  } else {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < slab; i += (long)gridDim.x * 256) {
      float a = ws[i];
      for (int sp = 1; sp < splits; ++sp) a += ws[sp * slab + i];
      const long m = i / N, n = i - m * N;
      float* cp = c + m * ldc + n;
      *cp = (beta != 0.f) ? a + beta * *cp : a;
    }
  }
}

int slab_reduce(const float* ws, int splits, float* c, long M, int N, long ldc, float beta, hipStream_t s) {
  if (splits < 1 || M <= 0 || N <= 0) return (int)hipErrorInvalidValue;
  const int vec = (N % 4 == 0 && ldc % 4 == 0 && ((uintptr_t)c & 15) == 0 && ((uintptr_t)ws & 15) == 0) ? 1 : 0;
  long work = vec ? (M * N) >> 2 : M * N;
  long blocks = (work + 255) / 256;
  if (blocks > misc_grid_cap()) blocks = misc_grid_cap();
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256), 0, s, ws, splits, c, M, N,
                     ldc, beta, vec);
  return (int)hipGetLastError();
}

int bias_grad_rows(long M) {
  long ys = M / 64;
  if (ys < 1) ys = 1;
  if (ys > 256) ys = 256;
  return (int)ys;
}

int bias_grad(const void* dy, float* db, long M, int N, int accumulate, hipStream_t s, float* det_ws, const void* ry,
              void* rdx, int zcount, long zdb) {
  if (zcount > 1) {  // replica-batched: the vector kernel, accumulate, non-deterministic form only
    if (!accumulate || det_ws || deterministic() || N % 8 || (reinterpret_cast<uintptr_t>(dy) & 15) || zdb % 4)
      return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(bias_grad_vec_kernel, dim3((N + 255) / 256, (unsigned)bias_grad_rows(M), (unsigned)zcount),
                       dim3(256), 0, s, (const bf16_t*)dy, db, M, N, (float*)nullptr, (const bf16_t*)ry, (bf16_t*)rdx,
                       zdb);
    return (int)hipGetLastError();
  }
  if (!accumulate) hipMemsetAsync(db, 0, sizeof(float) * N, s);
  long ys = bias_grad_rows(M);
  const bool vec = N % 8 == 0 && (reinterpret_cast<uintptr_t>(dy) & 15) == 0;
  if (ry && (!vec || (reinterpret_cast<uintptr_t>(ry) & 15) || (reinterpret_cast<uintptr_t>(rdx) & 15)))
    return (int)hipErrorInvalidValue;  // the fused ReLU form is the vector kernel only
  const bf16_t* ryb = reinterpret_cast<const bf16_t*>(ry);
  bf16_t* rdxb = reinterpret_cast<bf16_t*>(rdx);
  if (deterministic()) {
    if (vec && det_ws) {  // per-workgroup partial rows, then an in-order column sum (one writer per column)
      hipLaunchKernelGGL(bias_grad_vec_kernel, dim3((N + 255) / 256, (unsigned)ys), dim3(256), 0, s,
                         (const bf16_t*)dy, db, M, N, det_ws, ryb, rdxb);
      const int e = (int)hipGetLastError();
      return e ? e : colsum_partials(det_ws, (int)ys, N, db, 1, s);
    }
    ys = 1;  // no workspace: one workgroup per column block, a single writer per column
  }
  if (vec) {
    hipLaunchKernelGGL(bias_grad_vec_kernel, dim3((N + 255) / 256, (unsigned)ys), dim3(256), 0, s,
                       (const bf16_t*)dy, db, M, N, (float*)nullptr, ryb, rdxb);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(bias_grad_kernel, dim3((N + 255) / 256, (unsigned)ys), dim3(256), 0, s, (const bf16_t*)dy, db, M,
                     N);
  return (int)hipGetLastError();
}

// im2col with a tap table: col[m][t*C + c] = x[n][i*sh + dh[t]][j*sw + dw[t]][c], zero padded to kpad columns
struct Taps {
  int dh[64];
  int dw[64];
};

__global__ void im2col_kernel(const bf16_t* x, bf16_t* col, int N, int H, int W, int C, int Ho, int Wo, int sh, int sw,
                              int T, Taps taps, int kpad) {
  const long total = (long)N * Ho * Wo * kpad;
  GRID_LOOP(idx, total) {
    const int kk = (int)(idx % kpad);
    const long m = idx / kpad;
    bf16_t v = 0;
    if (kk < T * C) {
      const int t = kk / C, c = kk - t * C;
      const int j = (int)(m % Wo);
      const long q = m / Wo;
      const int i = (int)(q % Ho);
      const int n = (int)(q / Ho);
      const int ih = i * sh + taps.dh[t], iw = j * sw + taps.dw[t];
      if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) v = x[(((long)n * H + ih) * W + iw) * C + c];
    }
    col[idx] = v;
  }
}

int im2col(const void* x, void* col, int n, int hi, int wi, int c, int ho, int wo, int sh, int sw, int ntaps,
           const int* dh, const int* dw, int kpad, hipStream_t s) {
  if (ntaps > 64) return (int)hipErrorInvalidValue;
  Taps t;
  for (int i = 0; i < ntaps; ++i) {
    t.dh[i] = dh[i];
    t.dw[i] = dw[i];
  }
  const long total = (long)n * ho * wo * kpad;
  hipLaunchKernelGGL(im2col_kernel, dim3(mgrid(total)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)col, n, hi, wi, c,
                     ho, wo, sh, sw, ntaps, t, kpad);
  return (int)hipGetLastError();
}

__global__ void normalize_u8_kernel(const uint8_t* x, bf16_t* y, long npix, int C, int CP, const float* mean,
                                    const float* invstd) {
  GRID_LOOP(idx, npix * CP) {
    const int c = (int)(idx % CP);
    const long p = idx / CP;
    y[idx] = c < C ? f2bf(((float)x[p * C + c] - mean[c]) * invstd[c]) : (bf16_t)0;
  }
}

// RGB images (C = CP = 3): one lane per 4 pixels = 12 input bytes (three dword loads) and 24 output
// bytes (three 8-B stores), per-channel constants in registers, 32-bit indices.  The per-element
// kernel above (64-bit index division, byte loads, 2-B stores) moved the ResNet-50 input at 1.7 TB/s.
__global__ __launch_bounds__(256) void normalize_u8_rgb_kernel(const uint32_t* __restrict__ x, uint2* __restrict__ y,
                                                               uint32_t ngroups, const float* __restrict__ mean,
                                                               const float* __restrict__ invstd) {
  const float m0 = mean[0], m1 = mean[1], m2 = mean[2];
  const float i0 = invstd[0], i1 = invstd[1], i2 = invstd[2];
  for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < ngroups; g += gridDim.x * 256u) {
    const uint32_t w[3] = {x[3 * g], x[3 * g + 1], x[3 * g + 2]};
    float f[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      const float v = (float)((w[e >> 2] >> ((e & 3) * 8)) & 0xffu);
      const int c = e % 3;  // compile-time after unrolling
      f[e] = (v - (c == 0 ? m0 : (c == 1 ? m1 : m2))) * (c == 0 ? i0 : (c == 1 ? i1 : i2));
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
      y[3 * g + q] = make_uint2(pack_bf16x2(f[4 * q], f[4 * q + 1]), pack_bf16x2(f[4 * q + 2], f[4 * q + 3]));
  }
}

int normalize_u8(const uint8_t* x, void* y, long npix, int c, int cpad, const float* mean, const float* invstd,
                 hipStream_t s) {
  if (c == 3 && cpad == 3 && npix % 4 == 0 && npix * 3 < (1L << 31) && ((uintptr_t)x % 4) == 0 &&
      ((uintptr_t)y % 8) == 0) {
    const long ng = npix / 4;
    hipLaunchKernelGGL(normalize_u8_rgb_kernel, dim3(mgrid(ng)), dim3(256), 0, s, reinterpret_cast<const uint32_t*>(x),
                       reinterpret_cast<uint2*>(y), (uint32_t)ng, mean, invstd);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(normalize_u8_kernel, dim3(mgrid(npix * cpad)), dim3(256), 0, s, x, (bf16_t*)y, npix, c, cpad,
                     mean, invstd);
  return (int)hipGetLastError();
}

// Space-to-depth (block 2) with zero padding for the ResNet stem: x [N][H][W][C] (C <= 4) ->
// y [N][Ho][Wo][16], y[n][I][J][(2a + b) * C + ch] = x[n][2I + a - pad][2J + b - pad][ch] (0 outside),
// channels 4C..15 zero.  A 7x7 stride-2 conv on x equals a 4x4 stride-1 conv on y, with 12 of 16
// channels used instead of 3 of 8 after the 16-B channel padding (see ops/conv.py stem path).
// CC: the channel count as a compile-time constant (3: the RGB stem, every source load of a pixel block issued
// back to back), 0 = the runtime C
template <int CC>
__global__ void s2d_pad_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int H, int W, int C_,
                               int Ho, int Wo, int pad) {
  const int C = CC ? CC : C_;
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (long)N * Ho * Wo) return;
  const int J = (int)(pix % Wo);
  const long t = pix / Wo;
  const int I = (int)(t % Ho);
  const int n = (int)(t / Ho);
  uint16_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = 0;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int r = 2 * I + a - pad, c = 2 * J + b - pad;
      if ((unsigned)r < (unsigned)H && (unsigned)c < (unsigned)W) {
        const bf16_t* src = x + (((long)n * H + r) * W + c) * C;
#pragma unroll
        for (int ch = 0; ch < (CC ? CC : 4); ++ch)
          if (CC || ch < C) v[(2 * a + b) * C + ch] = src[ch];
      }
    }
  uint4* dst = reinterpret_cast<uint4*>(y + pix * 16);
  dst[0] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
  dst[1] = make_uint4(v[8] | (v[9] << 16), v[10] | (v[11] << 16), v[12] | (v[13] << 16), v[14] | (v[15] << 16));
}

int s2d_pad(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int pad, hipStream_t s) {
  const long n = (long)N * Ho * Wo;
  if (C > 4) return (int)hipErrorInvalidValue;
  if (C == 3)
    hipLaunchKernelGGL(s2d_pad_kernel<3>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const bf16_t*>(x), reinterpret_cast<bf16_t*>(y), N, H, W, C, Ho, Wo, pad);
  else
    hipLaunchKernelGGL(s2d_pad_kernel<0>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const bf16_t*>(x), reinterpret_cast<bf16_t*>(y), N, H, W, C, Ho, Wo, pad);
  return (int)hipGetLastError();
}

}  // namespace ddl

namespace ddl {

// y[c][r] = x[r][c] for a bf16 [R][C] matrix (row stride ldx), y contiguous [C][R].  One 64x64
// tile per 256-thread block, staged through LDS: 16-B global reads along x's rows, 16-B global
// writes along y's rows (the transposed weight copy read by the BERT-size Linear data-gradients).
// Requires R % 8 == 0, C % 8 == 0, ldx % 8 == 0 (checked by the launcher).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                             int R, int C, long ldx) {
  __shared__ bf16_t t[64][64 + 2];  // +2: odd 32-bit word stride, column reads spread over banks
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int v = 0; v < 2; ++v) {  // 64 rows x 8 vectors of 8
    const int idx = threadIdx.x + v * 256, rr = idx >> 3, cv = (idx & 7) * 8;
    uint4 d = make_uint4(0, 0, 0, 0);
    if (r0 + rr < R && c0 + cv < C) d = *reinterpret_cast<const uint4*>(x + (long)(r0 + rr) * ldx + c0 + cv);
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&d);
#pragma unroll
    for (int i = 0; i < 8; ++i) t[rr][cv + i] = e[i];
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < 2; ++v) {  // 64 output rows (x columns) x 8 vectors of 8
    const int idx = threadIdx.x + v * 256, cc = idx >> 3, rv = (idx & 7) * 8;
    if (c0 + cc >= C || r0 + rv >= R) continue;
    uint4 d;
    bf16_t* e = reinterpret_cast<bf16_t*>(&d);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = t[rv + i][cc];
    *reinterpret_cast<uint4*>(y + (long)(c0 + cc) * R + r0 + rv) = d;
  }
}

int transpose_bf16(const void* x, void* y, int R, int C, long ldx, hipStream_t s) {
  if (R % 8 || C % 8 || ldx % 8) return (int)hipErrorInvalidValue;
  const dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, R, C, ldx);
  return (int)hipGetLastError();
}

}  // namespace ddl
