// Fused softmax + cross-entropy forward AND backward in one sweep per row:
// a 256-thread block per row computes an online (max, sum-exp) over the row, then
// writes the per-row loss and dlogits = (softmax - target) * grad_scale.
// Targets are class indices (with label smoothing / ignore_index) or probability rows
// (Keras categorical_crossentropy with one-hot label vectors).
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {

__device__ __forceinline__ void xent_unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(w[e] << 16);
    f[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 xent_pack8(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

template <bool BF16>
__device__ __forceinline__ float ld_logit(const void* p, long i) {
  if constexpr (BF16) return bf2f(reinterpret_cast<const bf16_t*>(p)[i]);
  else return reinterpret_cast<const float*>(p)[i];
}

// One workgroup per row (grid B): wide rows (the MLM decoder's 30,522 classes).
template <bool BF16>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const void* __restrict__ logits,
                                                            const int64_t* __restrict__ labels,
                                                            const float* __restrict__ tprob, float* loss_rows,
                                                            void* dlogits, int K, long ld, float gscale, float smooth,
                                                            int ignore_index, const float* __restrict__ gscale_dev) {
  const int b = blockIdx.x;
  if (gscale_dev) gscale *= gscale_dev[0];  // device-resident factor (e.g. 1 / #valid labels: no host sync)
  __shared__ float sm[2][4];
  const long base = (long)b * ld;  // row stride ld >= K (padded vocabularies); tprob rows are dense [B][K]
  // vec: bf16 logits with 16-B aligned rows and class labels (the MLM decoder: 30,522-wide rows):
  // both passes read 8 logits per lane per 16-B load (2-B loads before) and the gradient row is
  // written as 16-B vectors; the last K % 8 columns take the scalar loop
  const bool vec = BF16 && tprob == nullptr && (ld % 8) == 0 && ((uintptr_t)logits % 16) == 0 &&
                   (dlogits == nullptr || ((uintptr_t)dlogits % 16) == 0);
  const int KV = vec ? K / 8 : 0;
  // pass 1: online max / sum-exp
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < KV; v += 256) {
    float f[8];
    xent_unpack8(reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(logits) + base)[v], f);
    float mv = f[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) mv = fmaxf(mv, f[e]);
    const float nm = fmaxf(m, mv);
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += __expf(f[e] - nm);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + acc;
    m = nm;
  }
  for (int k = KV * 8 + threadIdx.x; k < K; k += 256) {
    const float x = ld_logit<BF16>(logits, base + k);
    if (x > m) {
      s = s * __expf(m - x) + 1.f;
      m = x;
    } else {
      s += __expf(x - m);
    }
  }
  // wave reduce (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    sm[0][wid] = m;
    sm[1][wid] = s;
  }
  __syncthreads();
  float M = sm[0][0];
  for (int w = 1; w < 4; ++w) M = fmaxf(M, sm[0][w]);
  float S = 0.f;
  for (int w = 0; w < 4; ++w) S += sm[1][w] * __expf(sm[0][w] - M);
  const float lse = M + __logf(S);
  const int64_t lab = labels ? labels[b] : -1;
  const bool ignored = labels && lab == (int64_t)ignore_index;
  // pass 2: loss terms and gradient
  float lpart = 0.f;
  const float off = smooth / (float)K;
  for (int v = threadIdx.x; v < KV; v += 256) {
    float f[8], g[8];
    xent_unpack8(reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(logits) + base)[v], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = v * 8 + e;
      const float t = ignored ? 0.f : (k == lab ? 1.f - smooth : 0.f) + off;
      lpart += t * (lse - f[e]);
      g[e] = ignored ? 0.f : (__expf(f[e] - lse) - t) * gscale;
    }
    if (dlogits) reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(dlogits) + base)[v] = xent_pack8(g);
  }
  for (int k = KV * 8 + threadIdx.x; k < K; k += 256) {
    const float x = ld_logit<BF16>(logits, base + k);
    const float p = __expf(x - lse);
    float t;
    if (tprob) t = tprob[(long)b * K + k];
    else t = (k == lab ? 1.f - smooth : 0.f) + off;
    if (ignored) t = 0.f;
    lpart += t * (lse - x);
    const float g = ignored ? 0.f : (p - t) * gscale;
    if (dlogits) {
      if constexpr (BF16) reinterpret_cast<bf16_t*>(dlogits)[base + k] = f2bf(g);
      else reinterpret_cast<float*>(dlogits)[base + k] = g;
    }
  }
  if (dlogits)  // zero the padding columns so padded GEMMs can consume dlogits directly
    for (long k = K + threadIdx.x; k < ld; k += 256) {
      if constexpr (BF16) reinterpret_cast<bf16_t*>(dlogits)[base + k] = 0;
      else reinterpret_cast<float*>(dlogits)[base + k] = 0.f;
    }
  lpart = warp_sum(lpart);
  __syncthreads();
  if (lane == 0) sm[0][wid] = lpart;
  __syncthreads();
  if (threadIdx.x == 0) loss_rows[b] = sm[0][0] + sm[0][1] + sm[0][2] + sm[0][3];
}

// Small batches (loss_out != nullptr): ONE workgroup of 16 waves, a wave per row (lanes over the classes),
// wave-level reductions only, then the batch loss reduced through LDS.  The block-per-row kernel above
// spends two block barriers per row; the MNIST head (16 x 10) ran 24 us on it as one workgroup.
template <bool BF16>
__global__ __launch_bounds__(1024) void softmax_xent_small_kernel(const void* __restrict__ logits,
                                                                   const int64_t* __restrict__ labels,
                                                                   const float* __restrict__ tprob, float* loss_rows,
                                                                   void* dlogits, int K, long ld, float gscale,
                                                                   float smooth, int ignore_index,
                                                                   const float* __restrict__ gscale_dev, int B,
                                                                   float* __restrict__ loss_out, float out_scale,
                                                                   int zrows) {
  // zrows > 0 (replica batching): rows [z * zrows, (z + 1) * zrows) belong to replica z, whose loss goes
  // to loss_out[z] (B / zrows <= 64 replicas)
  if (gscale_dev) gscale *= gscale_dev[0];
  __shared__ float part[16];
  __shared__ float rep[64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (zrows > 0 && threadIdx.x < 64) rep[threadIdx.x] = 0.f;
  if (zrows > 0) __syncthreads();
  float total = 0.f;
  const float off = smooth / (float)K;
  for (int b = wid; b < B; b += 16) {
    const long base = (long)b * ld;
    float m = -INFINITY;
    for (int k = lane; k < K; k += 64) m = fmaxf(m, ld_logit<BF16>(logits, base + k));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += __expf(ld_logit<BF16>(logits, base + k) - m);
    se = warp_sum(se);
    const float lse = m + __logf(se);
    const int64_t lab = labels ? labels[b] : -1;
    const bool ignored = labels && lab == (int64_t)ignore_index;
    float lpart = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float x = ld_logit<BF16>(logits, base + k);
      float t = tprob ? tprob[(long)b * K + k] : (k == lab ? 1.f - smooth : 0.f) + off;
      if (ignored) t = 0.f;
      lpart += t * (lse - x);
      const float gv = ignored ? 0.f : (__expf(x - lse) - t) * gscale;
      if (dlogits) {
        if constexpr (BF16) reinterpret_cast<bf16_t*>(dlogits)[base + k] = f2bf(gv);
        else reinterpret_cast<float*>(dlogits)[base + k] = gv;
      }
    }
    if (dlogits)  // zero padding columns (padded GEMMs read dlogits as is)
      for (long k = K + lane; k < ld; k += 64) {
        if constexpr (BF16) reinterpret_cast<bf16_t*>(dlogits)[base + k] = 0;
        else reinterpret_cast<float*>(dlogits)[base + k] = 0.f;
      }
    lpart = warp_sum(lpart);
    if (lane == 0) {
      if (loss_rows) loss_rows[b] = lpart;
      if (zrows > 0) atomicAdd(&rep[b / zrows], lpart);
      total += lpart;
    }
  }
  if (zrows > 0) {
    __syncthreads();
    const int nz = (B + zrows - 1) / zrows;
    if (threadIdx.x < nz) loss_out[threadIdx.x] = rep[threadIdx.x] * out_scale * (gscale_dev ? gscale_dev[0] : 1.f);
    return;
  }
  if (lane == 0) part[wid] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += part[w];
    loss_out[0] = t * out_scale * (gscale_dev ? gscale_dev[0] : 1.f);
  }
}

int softmax_xent(const void* logits, int logits_bf16, const int64_t* labels, const float* target_probs,
                 float* loss_rows, void* dlogits, int B, int K, long ld, float grad_scale, float label_smoothing,
                 int ignore_index, hipStream_t s, const float* grad_scale_dev, float* loss_out, float out_scale,
                 int zrows) {
  if (B <= 0) return 0;
  if (zrows > 0 && (!loss_out || (B + zrows - 1) / zrows > 64)) return (int)hipErrorInvalidValue;
  if (loss_out) {  // small batch: one workgroup, a wave per row, the reduced loss written in place
    if (logits_bf16)
      hipLaunchKernelGGL(softmax_xent_small_kernel<true>, dim3(1), dim3(1024), 0, s, logits, labels, target_probs,
                         loss_rows, dlogits, K, ld, grad_scale, label_smoothing, ignore_index, grad_scale_dev, B,
                         loss_out, out_scale, zrows);
    else
      hipLaunchKernelGGL(softmax_xent_small_kernel<false>, dim3(1), dim3(1024), 0, s, logits, labels, target_probs,
                         loss_rows, dlogits, K, ld, grad_scale, label_smoothing, ignore_index, grad_scale_dev, B,
                         loss_out, out_scale, zrows);
    return (int)hipGetLastError();
  }
  if (!loss_rows) return (int)hipErrorInvalidValue;
  if (logits_bf16)
    hipLaunchKernelGGL(softmax_xent_kernel<true>, dim3(B), dim3(256), 0, s, logits, labels, target_probs, loss_rows,
                       dlogits, K, ld, grad_scale, label_smoothing, ignore_index, grad_scale_dev);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<false>, dim3(B), dim3(256), 0, s, logits, labels, target_probs, loss_rows,
                       dlogits, K, ld, grad_scale, label_smoothing, ignore_index, grad_scale_dev);
  return (int)hipGetLastError();
}

// inv[0] = 1 / max(1, #labels != ignore_index): the masked-LM loss normaliser computed on the device,
// so a batch without a host-side num_masked costs no device -> host sync
__global__ __launch_bounds__(1024) void label_count_inv_kernel(const int64_t* __restrict__ labels, long n, int ignore,
                                                               float* __restrict__ inv) {
  __shared__ float part[16];
  float c = 0.f;
  for (long i = threadIdx.x; i < n; i += 1024) c += labels[i] != (int64_t)ignore ? 1.f : 0.f;
  c = warp_sum(c);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += part[w];
    inv[0] = 1.f / fmaxf(t, 1.f);
  }
}

int label_count_inv(const int64_t* labels, long n, int ignore_index, float* inv, hipStream_t s) {
  hipLaunchKernelGGL(label_count_inv_kernel, dim3(1), dim3(1024), 0, s, labels, n, ignore_index, inv);
  return (int)hipGetLastError();
}

// out[0] = scale * sum(rows) with scale = host factor * (dev ? dev[0] : 1): the per-row losses of the
// fused softmax-xent reduced to the scalar loss in one launch (no ATen reduce + divide)
__global__ __launch_bounds__(1024) void rows_sum_scaled_kernel(const float* __restrict__ rows, long n, float scale,
                                                               const float* __restrict__ dev, float* __restrict__ out) {
  __shared__ float part[16];
  float a = 0.f;
  for (long i = threadIdx.x; i < n; i += 1024) a += rows[i];
  a = warp_sum(a);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += part[w];
    out[0] = t * scale * (dev ? dev[0] : 1.f);
  }
}

int rows_sum_scaled(const float* rows, long n, float scale, const float* dev, float* out, hipStream_t s) {
  hipLaunchKernelGGL(rows_sum_scaled_kernel, dim3(1), dim3(1024), 0, s, rows, n, scale, dev, out);
  return (int)hipGetLastError();
}

// Keras categorical cross-entropy on PROBABILITIES (a model whose softmax output is not fused into the loss,
// or any probability head): loss_rows[b] = -sum_k y[b][k] log(clip(p[b][k], eps, 1 - eps)) and, in the same
// sweep, dp[b][k] = -scale * y[b][k] / p[b][k] inside the clip range (0 outside: the clip's gradient).
// y is the one-hot row of labels[b] (sparse form; ignore_index rows contribute nothing) or target[b][k].
// One wave per row, lanes over the classes.
__global__ __launch_bounds__(256) void prob_xent_kernel(const float* __restrict__ p, const int64_t* __restrict__ labels,
                                                        const float* __restrict__ target, float* __restrict__ loss_rows,
                                                        float* __restrict__ dp, int B, int K, float eps, float scale,
                                                        int ignore_index) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* pr = p + (long)b * K;
  float* dr = dp + (long)b * K;
  const long lab = labels ? labels[b] : -1;
  const bool skip = labels && (lab == ignore_index || lab < 0 || lab >= K);
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float y = labels ? ((!skip && k == lab) ? 1.f : 0.f) : target[(long)b * K + k];
    const float pv = pr[k];
    const float pc = fminf(fmaxf(pv, eps), 1.f - eps);
    acc -= y * __logf(pc);
    dr[k] = (pv > eps && pv < 1.f - eps) ? -scale * y / pv : 0.f;
  }
  acc = warp_sum(acc);
  if (lane == 0) loss_rows[b] = acc;
}

int prob_xent(const float* p, const int64_t* labels, const float* target, float* loss_rows, float* dp, int B, int K,
              float eps, float scale, int ignore_index, hipStream_t s) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(prob_xent_kernel, dim3((B + 3) / 4), dim3(256), 0, s, p, labels, target, loss_rows, dp, B, K, eps,
                     scale, ignore_index);
  return (int)hipGetLastError();
}

// Mean squared error (Keras 'mean_squared_error') forward AND backward in one sweep:
// loss[0] = mean((p - t)^2), grad = 2 (p - t) / n.  One 1024-thread workgroup (regression
// heads are small: the reference's Dense(1) over a batch of 32).
__global__ __launch_bounds__(1024) void mse_kernel(const float* __restrict__ p, const float* __restrict__ t, long n,
                                                   float* __restrict__ loss, float* __restrict__ grad) {
  __shared__ float part[16];
  const float inv = 1.f / (float)n;
  float acc = 0.f;
  for (long i = threadIdx.x; i < n; i += 1024) {
    const float d = p[i] - t[i];
    acc += d * d;
    grad[i] = 2.f * d * inv;
  }
  acc = warp_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int w = 0; w < 16; ++w) s += part[w];
    loss[0] = s * inv;
  }
}

int mse_fwd_bwd(const float* pred, const float* target, long n, float* loss, float* grad, hipStream_t s) {
  hipLaunchKernelGGL(mse_kernel, dim3(1), dim3(1024), 0, s, pred, target, n, loss, grad);
  return (int)hipGetLastError();
}

}  // namespace ddl
