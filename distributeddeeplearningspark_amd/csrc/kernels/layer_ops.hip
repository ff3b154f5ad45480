// Element-wise / small-window kernels of the Keras layer set that the flagship models do not
// fuse elsewhere: standalone Activation, softmax, Dropout, AveragePooling2D, and the fp32
// column sum for the bias gradient of fp32 Dense layers.  bf16 and fp32 tensors
// (template on the storage type, fp32 math).
//
// Activation codes (ddl_ops.h ActCode): derivatives are taken from the forward OUTPUT y
// (tanh 1-y^2, sigmoid y(1-y), hard_sigmoid 0.2 on (0,1), relu y>0, elu y+1 below 0,
// selu, softplus 1-e^-y), except GELU which needs its input x.
// Dropout keeps element i iff drop_keep(seed, i, t8) (ddl_common.h): the backward
// regenerates the mask instead of storing it.
#include "ddl_common.h"
#include "ddl_act.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

template <class T> __device__ __forceinline__ float ldf(const T* p, long i);
template <> __device__ __forceinline__ float ldf<float>(const float* p, long i) { return p[i]; }
template <> __device__ __forceinline__ float ldf<bf16_t>(const bf16_t* p, long i) { return bf2f(p[i]); }
template <class T> __device__ __forceinline__ void stf(T* p, long i, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stf<bf16_t>(bf16_t* p, long i, float v) { p[i] = f2bf(v); }

template <class T>
__global__ void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long n, int code) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) stf(y, i, act_f(code, ldf(x, i)));
}

template <class T>
__global__ void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ ref, T* __restrict__ dx, long n,
                               int code) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    stf(dx, i, ldf(dy, i) * act_d(code, ldf(ref, i)));
}

// one wave per row of length N (softmax over the last axis)
template <class T>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long R, int N) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const T* xr = x + row * N;
  float mx = -INFINITY;
  for (int j = lane; j < N; j += 64) mx = fmaxf(mx, ldf(xr, j));
  mx = warp_max(mx);
  float s = 0.f;
  for (int j = lane; j < N; j += 64) s += __expf(ldf(xr, j) - mx);
  s = warp_sum(s);
  const float inv = 1.f / s;
  for (int j = lane; j < N; j += 64) stf(y + row * N, j, __expf(ldf(xr, j) - mx) * inv);
}

template <class T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dx, long R, int N) {
  const long row = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= R) return;
  const long o = row * N;
  float d = 0.f;
  for (int j = lane; j < N; j += 64) d += ldf(dy + o, j) * ldf(y + o, j);
  d = warp_sum(d);
  for (int j = lane; j < N; j += 64) stf(dx + o, j, ldf(y + o, j) * (ldf(dy + o, j) - d));
}

// dstep (nullable): a device step counter (fp32, whole numbers) mixed into the seed, so a hipGraph replaying the
// step draws a fresh mask every replay (models/step.py ticks it once per step); the backward reads the same value
template <class T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, unsigned long long seed,
                               uint32_t thresh, float scale, const float* __restrict__ dstep) {
  if (dstep) seed += (unsigned long long)(*dstep) * 0x9E3779B97F4A7C15ull;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    stf(y, i, drop_keep(seed, (unsigned long long)i, thresh) ? ldf(x, i) * scale : 0.f);
}

// NHWC average pooling, padding excluded from the count (Keras / TF 'same' semantics)
template <class T>
__global__ void avgpool2d_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int Ho,
                                     int Wo, int kh, int kw, int sh, int sw, int ph, int pw) {
  const long total = (long)N * Ho * Wo * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long r = i / C;
    const int wo = (int)(r % Wo);
    r /= Wo;
    const int ho = (int)(r % Ho);
    const int n = (int)(r / Ho);
    const int h0 = max(ho * sh - ph, 0), h1 = min(ho * sh - ph + kh, H);
    const int w0 = max(wo * sw - pw, 0), w1 = min(wo * sw - pw + kw, W);
    float s = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) s += ldf(x, (((long)n * H + h) * W + w) * C + c);
    const int cnt = max((h1 - h0) * (w1 - w0), 1);
    stf(y, i, s / (float)cnt);
  }
}

template <class T>
__global__ void avgpool2d_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                     int Wo, int kh, int kw, int sh, int sw, int ph, int pw) {
  const long total = (long)N * H * W * C;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int c = (int)(i % C);
    long r = i / C;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    // outputs whose window [o*s - p, o*s - p + k) contains h
    const int ho0 = max((h + ph - kh + sh) / sh, 0), ho1 = min((h + ph) / sh, Ho - 1);
    const int wo0 = max((w + pw - kw + sw) / sw, 0), wo1 = min((w + pw) / sw, Wo - 1);
    float s = 0.f;
    for (int ho = ho0; ho <= ho1; ++ho) {
      const int h0 = max(ho * sh - ph, 0), h1 = min(ho * sh - ph + kh, H);
      if (h < h0 || h >= h1) continue;
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int w0 = max(wo * sw - pw, 0), w1 = min(wo * sw - pw + kw, W);
        if (w < w0 || w >= w1) continue;
        s += ldf(dy, (((long)n * Ho + ho) * Wo + wo) * C + c) / (float)max((h1 - h0) * (w1 - w0), 1);
      }
    }
    stf(dx, i, s);
  }
}

// db[n] += sum_m dy[m][n] (fp32): 64 columns x 4 row-lanes per workgroup, 256 rows per chunk
__global__ __launch_bounds__(256) void colsum_f32_kernel(const float* __restrict__ dy, float* __restrict__ db, long M,
                                                         int N, long chunk) {
  __shared__ float part[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const long r0 = (long)blockIdx.y * chunk;
  const long r1 = min(M, r0 + chunk);
  float s = 0.f;
  if (col < N)
    for (long r = r0 + rl; r < r1; r += 4) s += dy[r * N + col];
  part[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && col < N) atomicAdd(db + col, part[0][threadIdx.x] + part[1][threadIdx.x] + part[2][threadIdx.x] +
                                                  part[3][threadIdx.x]);
}

// Keras Embedding: out[t][:] = table[ids[t]][:]; one wave per token row
template <class T>
__global__ __launch_bounds__(256) void embedding_gather_kernel(const int64_t* __restrict__ ids,
                                                               const T* __restrict__ table, T* __restrict__ out,
                                                               long n, int D, long V, int* __restrict__ bad) {
  const long t = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  const long id = ids[t];
  const bool ok = id >= 0 && id < V;
  if (!ok && lane == 0) atomicOr(bad, 1);
  for (int d = lane; d < D; d += 64) out[t * D + d] = ok ? table[id * D + d] : T(0);
}

// gw[ids[t]][:] += dy[t][:] (fp32 atomics: Keras vocabularies are small, rows rarely collide)
template <class T>
__global__ __launch_bounds__(256) void embedding_scatter_kernel(const int64_t* __restrict__ ids,
                                                                const T* __restrict__ dy, float* __restrict__ gw,
                                                                long n, int D, long V) {
  const long t = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= n) return;
  const long id = ids[t];
  if (id < 0 || id >= V) return;
  for (int d = lane; d < D; d += 64) atomicAdd(gw + id * D + d, ldf(dy, t * D + d));
}

// Conv data-gradient filters: out[ci][t][co] = w[co][taps[t]][ci] (bf16) — the flipped filter
// of a stride-1 dgrad (taps reversed) and the K-contiguous per-class filters of a strided dgrad,
// in ONE pass (replaces flip + permute-copy / index_select + permute-copy: 2-3 ATen launches per
// conv per step).  32x32 (co, ci) tiles through LDS so both the read (ci) and the write (co) are
// contiguous; blockIdx.z = output tap.
// blockIdx.z = replica * nt + tap (replica batching: filters every zw, outputs every zo elements)
__global__ __launch_bounds__(256) void filter_taps_transpose_kernel(const bf16_t* __restrict__ w,
                                                                    bf16_t* __restrict__ out, int Co, int T,
                                                                    int Ci, int nt, FilterTaps taps, long zw, long zo) {
  __shared__ bf16_t tile[32][33];
  const int zr = blockIdx.z / nt, t = blockIdx.z - zr * nt, src_t = taps.t[t];
  w += zr * zw;
  out += zr * zo;
  const int co0 = blockIdx.y * 32, ci0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int co = co0 + i, ci = ci0 + tx;
    tile[i][tx] = (co < Co && ci < Ci) ? w[((long)co * T + src_t) * Ci + ci] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int ci = ci0 + i, co = co0 + tx;
    if (ci < Ci && co < Co) out[((long)ci * nt + t) * Co + co] = tile[tx][i];
  }
}

// Every weight-derived filter of a training step in ONE launch (ops/derived.py): job j transposes
// src [Co][T][Ci] into dst [Ci][nt][Co] over the taps taps[0..nt) (a flipped stride-1 dgrad filter, a strided
// dgrad class filter, or — T = nt = 1 — a plain [N][K] -> [K][N] weight transpose for a Linear dgrad).  The
// blocks of all jobs form one grid; a block finds its job in the (device-resident, per-model) table.
// jobs with Co, Ci in 64-multiples (BERT weights, every ResNet-50 filter but the stem's): 64x64 tiles of one tap
// moved as 16-B vectors both ways (the 2-B element tiles ran ~330 us for BERT-base's 85 M parameters per step)
__device__ __forceinline__ bool taps_job_vec(int Co, int Ci, int T, int nt) {
  (void)T;
  (void)nt;
  return Co % 64 == 0 && Ci % 64 == 0;  // any tap count: one 64 x 64 tile of one tap per block
}

__global__ __launch_bounds__(256) void taps_batch_kernel(const TapsJob* __restrict__ jobs, int njobs) {
  __shared__ bf16_t tile[32][33];
  __shared__ __attribute__((aligned(16))) bf16_t vt[64][72];
  const int blk = blockIdx.x;
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].blk0 <= blk) ++j;
  const TapsJob& jb = jobs[j];
  const int Co = jb.Co, Ci = jb.Ci, T = jb.T, nt = jb.nt;
  if (taps_job_vec(Co, Ci, T, nt)) {
    const int nbi = Ci >> 6, nbo = Co >> 6;
    const int local = blk - jb.blk0;
    const int t = local / (nbi * nbo), rem = local - t * nbi * nbo;
    const int co0 = (rem / nbi) * 64, ci0 = (rem % nbi) * 64;
    const int src_t = jb.taps[t];
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // 64 rows (co) x 8 vectors (ci) of source tap src_t
      const int idx = threadIdx.x + 256 * i, r = idx >> 3, cv = idx & 7;
      *reinterpret_cast<uint4*>(&vt[r][cv * 8]) =
          *reinterpret_cast<const uint4*>(jb.src + ((long)(co0 + r) * T + src_t) * Ci + ci0 + cv * 8);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // 64 rows (ci) x 8 vectors (co)
      const int idx = threadIdx.x + 256 * i, r = idx >> 3, cv = idx & 7;
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = (uint32_t)vt[cv * 8 + 2 * k][r] | ((uint32_t)vt[cv * 8 + 2 * k + 1][r] << 16);
      *reinterpret_cast<uint4*>(jb.dst + ((long)(ci0 + r) * nt + t) * Co + co0 + cv * 8) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return;
  }
  const int nbi = (Ci + 31) >> 5, nbo = (Co + 31) >> 5;
  const int local = blk - jb.blk0;
  const int t = local / (nbi * nbo), rem = local - t * nbi * nbo;
  const int co0 = (rem / nbi) * 32, ci0 = (rem % nbi) * 32;
  const int src_t = jb.taps[t];
  const bf16_t* w = jb.src;
  bf16_t* out = jb.dst;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int co = co0 + i, ci = ci0 + tx;
    tile[i][tx] = (co < Co && ci < Ci) ? w[((long)co * T + src_t) * Ci + ci] : (bf16_t)0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int ci = ci0 + i, co = co0 + tx;
    if (ci < Ci && co < Co) out[((long)ci * nt + t) * Co + co] = tile[tx][i];
  }
}

// y[C][R] = x[R][C] (fp32) through a padded 32x32 LDS tile
__global__ __launch_bounds__(256) void transpose_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int R,
                                                            int C) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8)
    if (r0 + i < R && c0 + tx < C) t[i][tx] = x[(long)(r0 + i) * C + c0 + tx];
  __syncthreads();
  for (int i = ty; i < 32; i += 8)
    if (c0 + i < C && r0 + tx < R) y[(long)(c0 + i) * R + r0 + tx] = t[tx][i];
}

inline int blocks_for(long n) { return (int)std::min<long>((n + 255) / 256, 8192); }

}  // namespace

int act_fwd(const void* x, void* y, long n, int code, int bf16, hipStream_t s) {
  if (n <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(act_fwd_kernel<bf16_t>, dim3(blocks_for(n)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n,
                       code);
  else
    hipLaunchKernelGGL(act_fwd_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, code);
  return (int)hipGetLastError();
}

int act_bwd(const void* dy, const void* ref, void* dx, long n, int code, int bf16, hipStream_t s) {
  if (n <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(act_bwd_kernel<bf16_t>, dim3(blocks_for(n)), dim3(256), 0, s, (const bf16_t*)dy,
                       (const bf16_t*)ref, (bf16_t*)dx, n, code);
  else
    hipLaunchKernelGGL(act_bwd_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, s, (const float*)dy, (const float*)ref,
                       (float*)dx, n, code);
  return (int)hipGetLastError();
}

int softmax_rows_fwd(const void* x, void* y, long R, int N, int bf16, hipStream_t s) {
  if (R <= 0) return 0;
  const dim3 grid((unsigned)((R + 3) / 4));
  if (bf16)
    hipLaunchKernelGGL(softmax_fwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, R, N);
  else
    hipLaunchKernelGGL(softmax_fwd_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (float*)y, R, N);
  return (int)hipGetLastError();
}

int softmax_rows_bwd(const void* dy, const void* y, void* dx, long R, int N, int bf16, hipStream_t s) {
  if (R <= 0) return 0;
  const dim3 grid((unsigned)((R + 3) / 4));
  if (bf16)
    hipLaunchKernelGGL(softmax_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)dy, (const bf16_t*)y,
                       (bf16_t*)dx, R, N);
  else
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)dy, (const float*)y, (float*)dx,
                       R, N);
  return (int)hipGetLastError();
}

int dropout_apply(const void* x, void* y, long n, unsigned long long seed, uint32_t thresh, float scale, int bf16,
                  hipStream_t s, const float* dstep) {
  if (n <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, dim3(blocks_for(n)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n,
                       seed, thresh, scale, dstep);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, s, (const float*)x, (float*)y, n, seed,
                       thresh, scale, dstep);
  return (int)hipGetLastError();
}

int avgpool2d_fwd(const void* x, void* y, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                  int ph, int pw, int bf16, hipStream_t s) {
  const long n = (long)N * Ho * Wo * C;
  if (n <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(avgpool2d_fwd_kernel<bf16_t>, dim3(blocks_for(n)), dim3(256), 0, s, (const bf16_t*)x,
                       (bf16_t*)y, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else
    hipLaunchKernelGGL(avgpool2d_fwd_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, s, (const float*)x, (float*)y, N,
                       H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  return (int)hipGetLastError();
}

int avgpool2d_bwd(const void* dy, void* dx, int N, int H, int W, int C, int Ho, int Wo, int kh, int kw, int sh, int sw,
                  int ph, int pw, int bf16, hipStream_t s) {
  const long n = (long)N * H * W * C;
  if (n <= 0) return 0;
  if (bf16)
    hipLaunchKernelGGL(avgpool2d_bwd_kernel<bf16_t>, dim3(blocks_for(n)), dim3(256), 0, s, (const bf16_t*)dy,
                       (bf16_t*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  else
    hipLaunchKernelGGL(avgpool2d_bwd_kernel<float>, dim3(blocks_for(n)), dim3(256), 0, s, (const float*)dy,
                       (float*)dx, N, H, W, C, Ho, Wo, kh, kw, sh, sw, ph, pw);
  return (int)hipGetLastError();
}

int filter_taps_transpose(const void* w, void* out, int Co, int T, int Ci, const FilterTaps& taps, int nt,
                          hipStream_t s, int zcount, long zw, long zo) {
  if (nt <= 0 || nt > kMaxFilterTaps || Co <= 0 || Ci <= 0 || zcount < 1) return (int)hipErrorInvalidValue;
  const dim3 grid((Ci + 31) / 32, (Co + 31) / 32, nt * zcount);
  hipLaunchKernelGGL(filter_taps_transpose_kernel, grid, dim3(256), 0, s, (const bf16_t*)w, (bf16_t*)out, Co, T, Ci,
                     nt, taps, zw, zo);
  return (int)hipGetLastError();
}

int taps_batch(const TapsJob* jobs, int njobs, int blocks, hipStream_t s) {
  if (njobs < 1 || blocks < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(taps_batch_kernel, dim3(blocks), dim3(256), 0, s, jobs, njobs);
  return (int)hipGetLastError();
}

int taps_job_blocks(int Co, int Ci, int nt, int T) {
  if (Co % 64 == 0 && Ci % 64 == 0) return (Ci / 64) * (Co / 64) * nt;  // = taps_job_vec
  return ((Ci + 31) / 32) * ((Co + 31) / 32) * nt;
}

int transpose_f32(const float* x, float* y, int R, int C, hipStream_t s) {
  if (R <= 0 || C <= 0) return 0;
  hipLaunchKernelGGL(transpose_f32_kernel, dim3((C + 31) / 32, (R + 31) / 32), dim3(256), 0, s, x, y, R, C);
  return (int)hipGetLastError();
}

int embedding_gather(const int64_t* ids, const void* table, void* out, long n, int D, long V, int* bad, int bf16,
                     hipStream_t s) {
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 3) / 4));
  if (bf16)
    hipLaunchKernelGGL(embedding_gather_kernel<bf16_t>, grid, dim3(256), 0, s, ids, (const bf16_t*)table, (bf16_t*)out,
                       n, D, V, bad);
  else
    hipLaunchKernelGGL(embedding_gather_kernel<float>, grid, dim3(256), 0, s, ids, (const float*)table, (float*)out, n,
                       D, V, bad);
  return (int)hipGetLastError();
}

int embedding_scatter(const int64_t* ids, const void* dy, float* gw, long n, int D, long V, int bf16, hipStream_t s) {
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 3) / 4));
  if (bf16)
    hipLaunchKernelGGL(embedding_scatter_kernel<bf16_t>, grid, dim3(256), 0, s, ids, (const bf16_t*)dy, gw, n, D, V);
  else
    hipLaunchKernelGGL(embedding_scatter_kernel<float>, grid, dim3(256), 0, s, ids, (const float*)dy, gw, n, D, V);
  return (int)hipGetLastError();
}

int colsum_f32(const float* dy, float* db, long M, int N, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const long chunk = deterministic() ? M : 256;  // deterministic: one writer per column
  const dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + chunk - 1) / chunk));
  hipLaunchKernelGGL(colsum_f32_kernel, grid, dim3(256), 0, s, dy, db, M, N, chunk);
  return (int)hipGetLastError();
}

}  // namespace ddl
