// Optimizer steps over the flat fp32 parameter arena: ONE launch updates every
// parameter of the model (the arena makes "multi-tensor apply" a plain 1-D sweep),
// and the same sweep writes the bf16 compute copy, so no separate cast pass exists.
// float4 per lane; grad_scale folds the data-parallel 1/world averaging (or loss-scale)
// into the update instead of a separate pass over the gradients.
#include "ddl_common.h"
#include "ddl_ops.h"
#include <stdlib.h>

namespace ddl {

// one float4 per lane, no grid-stride trips (a 4,096-workgroup cap cost the sweeps 2-3 %: bn.hip bn_grid_cap)
static unsigned ogrid(long n4) {
  long g = (n4 + 255) / 256;
  if (g > (1L << 24)) g = 1L << 24;
  return (unsigned)(g > 0 ? g : 1);
}

__device__ __forceinline__ void store_bf16x4(void* w16, long i4, const float4& w) {
  uint2 o;
  o.x = pack_bf16x2(w.x, w.y);
  o.y = pack_bf16x2(w.z, w.w);
  reinterpret_cast<uint2*>(w16)[i4] = o;
}

#define DDL_FLAT_FOR(i, n) for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < ((n) >> 2); i += (long)gridDim.x * 256)

// ------------------------------ SGD (+momentum, nesterov, weight decay) ------------------------------
__global__ __launch_bounds__(256) void sgd_kernel(float4* w, const float4* g, float4* mom, void* w16, long n, float lr,
                                                   float mu, float damp, float wd, int nesterov, float gs) {
  DDL_FLAT_FOR(i, n) {
    float4 p = w[i], d = g[i];
    float* pp = &p.x;
    float* dd = &d.x;
    float4 b = mom ? mom[i] : make_float4(0, 0, 0, 0);
    float* bb = &b.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = dd[k] * gs + wd * pp[k];
      if (mom) {
        bb[k] = mu * bb[k] + (1.f - damp) * gg;
        gg = nesterov ? gg + mu * bb[k] : bb[k];
      }
      pp[k] -= lr * gg;
    }
    w[i] = p;
    if (mom) mom[i] = b;
    if (w16) store_bf16x4(w16, i, p);
  }
}

int sgd_step(float* w, const float* g, float* mom, void* w16, long n, float lr, float momentum, float dampening,
             float wd, int nesterov, float gscale, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(sgd_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, (float4*)w, (const float4*)g,
                     momentum != 0.f ? (float4*)mom : nullptr, w16, n, lr, momentum, dampening, wd, nesterov, gscale);
  return (int)hipGetLastError();
}

// ------------------------------ Adam / AdamW ------------------------------
// mode bit0: decoupled weight decay (AdamW); bit1: Keras epsilon placement
//   PyTorch: w -= lr * (m/bc1) / (sqrt(v/bc2) + eps)
//   Keras 2: w -= lr * sqrt(bc2)/bc1 * m / (sqrt(v) + eps)
// bit2 (kAdamTick): this launch also advances the device step counter: every workgroup uses t + 1 and the
//   last workgroup to finish (tick_ctr, an atomicInc that wraps back to 0) stores it — every other
//   workgroup has read the counter by then, so no separate step_tick launch precedes the update.
// bit3 (kAdamZeroGrad): the gradients are zeroed as they are consumed (the next step's zero_grad fill is
//   skipped: models/optimizers.py captured_update(zero_grads=True)).
constexpr int kAdamTick = 4, kAdamZeroGrad = 8;
__global__ __launch_bounds__(256) void adam_kernel(float4* w, const float4* g, float4* m, float4* v, void* w16, long n,
                                                    float lr, float b1, float b2, float eps, float wd, int mode,
                                                    float bc1, float bc2, float gs, float* tstep,
                                                    unsigned* __restrict__ tick_ctr) {
  float t = 0.f;
  if (tstep) {  // graph-replayed step: bias corrections from the device step counter
    t = *tstep + ((mode & kAdamTick) ? 1.f : 0.f);
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  const bool zg = mode & kAdamZeroGrad;
  const float sbc2 = sqrtf(bc2);
  auto upd = [&](float4& p, const float4& d, float4& mm, float4& vv) {
    float *pp = &p.x, *m_ = &mm.x, *v_ = &vv.x;
    const float* dd = &d.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = dd[k] * gs;
      if (mode & 1) pp[k] *= (1.f - lr * wd);
      else gg += wd * pp[k];
      m_[k] = b1 * m_[k] + (1.f - b1) * gg;
      v_[k] = b2 * v_[k] + (1.f - b2) * gg * gg;
      if (mode & 2) pp[k] -= lr * (sbc2 / bc1) * m_[k] / (sqrtf(v_[k]) + eps);
      else pp[k] -= lr * (m_[k] / bc1) / (sqrtf(v_[k]) / sbc2 + eps);
    }
  };
  // two float4 slots per lane per trip, all eight loads issued before any store: twice the
  // bytes in flight per wave for this 30-byte/parameter stream (HBM-bound)
  const long n4 = n >> 2, stride = (long)gridDim.x * 256;
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const long j = i + stride;
    float4 p0 = w[i], d0 = g[i], m0 = m[i], v0 = v[i];
    float4 p1 = w[j], d1 = g[j], m1 = m[j], v1 = v[j];
    upd(p0, d0, m0, v0);
    upd(p1, d1, m1, v1);
    w[i] = p0; m[i] = m0; v[i] = v0;
    w[j] = p1; m[j] = m1; v[j] = v1;
    if (w16) { store_bf16x4(w16, i, p0); store_bf16x4(w16, j, p1); }
    if (zg) { const_cast<float4*>(g)[i] = make_float4(0, 0, 0, 0); const_cast<float4*>(g)[j] = make_float4(0, 0, 0, 0); }
  }
  if (i < n4) {
    float4 p0 = w[i], d0 = g[i], m0 = m[i], v0 = v[i];
    upd(p0, d0, m0, v0);
    w[i] = p0; m[i] = m0; v[i] = v0;
    if (w16) store_bf16x4(w16, i, p0);
    if (zg) const_cast<float4*>(g)[i] = make_float4(0, 0, 0, 0);
  }
  if ((mode & kAdamTick) && tstep) {
    // no fence: every workgroup consumed its read of *tstep (the bias corrections) before this point, and
    // a device-scope fence per workgroup (an L2 write-back) cost the sweep 5x (8 -> 48 us per MNIST step)
    __syncthreads();
    if (threadIdx.x == 0 && atomicInc(tick_ctr, gridDim.x - 1) == gridDim.x - 1) *tstep = t;  // last workgroup
  }
}

int adam_step(float* w, const float* g, float* m, float* v, void* w16, long n, float lr, float b1, float b2, float eps,
              float wd, int adamw, float bc1, float bc2, float gscale, float* tstep, hipStream_t s, unsigned* tick_ctr) {
  if (n % 4) return (int)hipErrorInvalidValue;
  if ((adamw & kAdamTick) && (!tstep || !tick_ctr)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adam_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, (float4*)w, (const float4*)g, (float4*)m,
                     (float4*)v, w16, n, lr, b1, b2, eps, wd, adamw, bc1, bc2, gscale, tstep, tick_ctr);
  return (int)hipGetLastError();
}

// Device-resident optimizer step counter (t += 1), so a captured hipGraph that is
// replayed every step still sees the right Adam bias corrections.
__global__ void step_tick_kernel(float* t) { *t += 1.f; }

int step_tick(float* t, hipStream_t s) {
  hipLaunchKernelGGL(step_tick_kernel, dim3(1), dim3(1), 0, s, t);
  return (int)hipGetLastError();
}

// ------------------------------ Adagrad (Keras 2 semantics) ------------------------------
__global__ __launch_bounds__(256) void adagrad_kernel(float4* w, const float4* g, float4* acc, void* w16, long n,
                                                       float lr, float eps, float wd, float gs) {
  DDL_FLAT_FOR(i, n) {
    float4 p = w[i], d = g[i], a = acc[i];
    float *pp = &p.x, *dd = &d.x, *aa = &a.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gg = dd[k] * gs + wd * pp[k];
      aa[k] += gg * gg;
      pp[k] -= lr * gg / (sqrtf(aa[k]) + eps);
    }
    w[i] = p;
    acc[i] = a;
    if (w16) store_bf16x4(w16, i, p);
  }
}

int adagrad_step(float* w, const float* g, float* acc, void* w16, long n, float lr, float eps, float wd, float gscale,
                 hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(adagrad_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, (float4*)w, (const float4*)g, (float4*)acc,
                     w16, n, lr, eps, wd, gscale);
  return (int)hipGetLastError();
}

// ------------------------------ RMSprop (Keras 2 semantics) ------------------------------
__global__ __launch_bounds__(256) void rmsprop_kernel(float4* w, const float4* g, float4* acc, void* w16, long n,
                                                       float lr, float rho, float eps, float wd, float gs) {
  DDL_FLAT_FOR(i, n) {
    float4 p = w[i], d = g[i], a = acc[i];
    float *pp = &p.x, *dd = &d.x, *aa = &a.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gg = dd[k] * gs + wd * pp[k];
      aa[k] = rho * aa[k] + (1.f - rho) * gg * gg;
      pp[k] -= lr * gg / (sqrtf(aa[k]) + eps);
    }
    w[i] = p;
    acc[i] = a;
    if (w16) store_bf16x4(w16, i, p);
  }
}

int rmsprop_step(float* w, const float* g, float* acc, void* w16, long n, float lr, float rho, float eps, float wd,
                 float gscale, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsprop_kernel, dim3(ogrid(n / 4)), dim3(256), 0, s, (float4*)w, (const float4*)g, (float4*)acc,
                     w16, n, lr, rho, eps, wd, gscale);
  return (int)hipGetLastError();
}

// ------------------------------ sum of squares ------------------------------
__global__ __launch_bounds__(256) void sumsq_kernel(const float4* x, long n4, float* out) {
  float acc = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float4 v = x[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = warp_sum(acc);
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, sm[0] + sm[1] + sm[2] + sm[3]);
}

int sumsq_f32(const float* x, long n, float* out, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  const unsigned blocks = deterministic() ? 1u : (ogrid(n / 4) > 1024 ? 1024 : ogrid(n / 4));
  hipLaunchKernelGGL(sumsq_kernel, dim3(blocks), dim3(256), 0, s, (const float4*)x, n / 4, out);
  return (int)hipGetLastError();
}


// ------------------------------ dist-keras commit rounds (ADAG / DynSGD / DOWNPOUR / EASGD) ------------------------------
// The reference's commit arithmetic (residual = (W - W_pulled) / window, PS center += residual, pull;
// ddl_mnist_aztk.py:216-219 via distkeras' ADAGWorker) as two flat sweeps around the exchange:
//   commit_delta:  X = scale * (W - center); elastic (EASGD family): W -= X        (before the exchange)
//   commit_apply:  center += sum_j X_j over the exchanged buffers; W = center      (after it)
// X_j are either the all-reduced buffer (one pointer) or the peer replicas' buffers of workers
// co-located on this GPU, mapped through IPC handles (parallel/colocated.py): the reduction over
// workers is then this one kernel reading the peers' HBM directly, with no host staging.
__global__ __launch_bounds__(256) void commit_delta_kernel(float4* __restrict__ W, const float4* __restrict__ center,
                                                           float4* __restrict__ X, void* w16, long n, float scale,
                                                           int elastic) {
  DDL_FLAT_FOR(i, n) {
    float4 w = W[i];
    const float4 c = center[i];
    const float4 x = make_float4(scale * (w.x - c.x), scale * (w.y - c.y), scale * (w.z - c.z), scale * (w.w - c.w));
    X[i] = x;
    if (elastic) {
      w = make_float4(w.x - x.x, w.y - x.y, w.z - x.z, w.w - x.w);
      W[i] = w;
      if (w16) store_bf16x4(w16, i, w);
    }
  }
}

int commit_delta(float* W, const float* center, float* X, void* w16, long n, float scale, int elastic, hipStream_t s) {
  hipLaunchKernelGGL(commit_delta_kernel, dim3(ogrid(n >> 2)), dim3(256), 0, s, (float4*)W, (const float4*)center,
                     (float4*)X, w16, n, scale, elastic);
  return (int)hipGetLastError();
}

__global__ __launch_bounds__(256) void commit_apply_kernel(CommitPtrs xs, int nx, float4* __restrict__ center,
                                                           float4* __restrict__ W, void* w16, long n) {
  DDL_FLAT_FOR(i, n) {
    float4 c = center[i];
    for (int j = 0; j < nx; ++j) {
      const float4 x = reinterpret_cast<const float4*>(xs.p[j])[i];
      c.x += x.x;
      c.y += x.y;
      c.z += x.z;
      c.w += x.w;
    }
    center[i] = c;
    if (W) {
      W[i] = c;
      if (w16) store_bf16x4(w16, i, c);
    }
  }
}

int commit_apply(const CommitPtrs& xs, int nx, float* center, float* W, void* w16, long n, hipStream_t s) {
  hipLaunchKernelGGL(commit_apply_kernel, dim3(ogrid(n >> 2)), dim3(256), 0, s, xs, nx, (float4*)center, (float4*)W,
                     w16, n);
  return (int)hipGetLastError();
}

}  // namespace ddl
