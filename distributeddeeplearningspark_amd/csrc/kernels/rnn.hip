// Persistent recurrent kernels (Keras-2 GRU reset_after=False and LSTM; tanh + hard_sigmoid),
// fp32 like the reference's Keras models (GRU(128) / LSTM(128) over 25 steps).
//
// The input projection x W + b of ALL time steps is one GEMM done before the kernel; the
// kernel then owns BB batch rows for the whole sequence: h (and c) stay in LDS across the
// T steps, every step reads U (fp32, L2/L1-resident) column-per-thread (coalesced) and the
// hidden state as an LDS broadcast.  Post-activation gates, the hidden / cell sequences
// are saved for the backward.
// Backward (BPTT) runs the same persistent structure in reverse time, propagating dh (and dc)
// with U^T columns per thread; it emits the pre-activation gate gradients of every step so
// that dW, dU, db and dx are plain GEMMs / reductions afterwards.
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

constexpr int BB = 4;  // batch rows per workgroup

__device__ __forceinline__ float hsig(float x) { return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f); }
__device__ __forceinline__ float hsig_d(float y) { return (y > 0.f && y < 1.f) ? 0.2f : 0.f; }

// ----------------------------------------------------------------------------- forward
template <int CELL>  // 0 = GRU (gates z, r, h), 1 = LSTM (gates i, f, c, o)
__global__ __launch_bounds__(512) void rnn_fwd_kernel(const float* __restrict__ xw, const float* __restrict__ U,
                                                      float* __restrict__ hs, float* __restrict__ cs,
                                                      float* __restrict__ gates, float* __restrict__ y, int B, int T,
                                                      int H, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  extern __shared__ float sm[];
  const int GH = G * H;
  float* h = sm;              // [BB][H]
  float* c = h + BB * H;      // [BB][H]   (LSTM) / r*h (GRU)
  float* gb = c + BB * H;     // [BB][GH]  gate values of the current step
  const int b0 = blockIdx.x * BB;
  const int nb = min(BB, B - b0);
  for (int i = threadIdx.x; i < BB * H; i += blockDim.x) h[i] = c[i] = 0.f;
  for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
    const int r = i / H, k = i - r * H;
    hs[((long)(b0 + r) * (T + 1)) * H + k] = 0.f;
    if (CELL == 1) cs[((long)(b0 + r) * (T + 1)) * H + k] = 0.f;
  }
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    // gate pre-activations x W + h U (GRU: only z, r here; the candidate needs r * h first)
    const int jend = CELL == 0 ? 2 * H : GH;
    for (int j = threadIdx.x; j < jend; j += blockDim.x) {
      float acc[BB];
#pragma unroll
      for (int r = 0; r < BB; ++r) acc[r] = r < nb ? xw[((long)(b0 + r) * T + t) * GH + j] : 0.f;
      for (int k = 0; k < H; ++k) {
        const float u = U[(long)k * GH + j];
#pragma unroll
        for (int r = 0; r < BB; ++r) acc[r] += h[r * H + k] * u;
      }
      const bool is_tanh = CELL == 1 && j >= 2 * H && j < 3 * H;
#pragma unroll
      for (int r = 0; r < BB; ++r) gb[r * GH + j] = is_tanh ? tanhf(acc[r]) : hsig(acc[r]);
    }
    __syncthreads();
    if (CELL == 0) {
      for (int i = threadIdx.x; i < BB * H; i += blockDim.x) {
        const int r = i / H, k = i - r * H;
        c[i] = gb[r * GH + H + k] * h[i];  // r * h
      }
      __syncthreads();
      for (int j = 2 * H + threadIdx.x; j < GH; j += blockDim.x) {
        float acc[BB];
#pragma unroll
        for (int r = 0; r < BB; ++r) acc[r] = r < nb ? xw[((long)(b0 + r) * T + t) * GH + j] : 0.f;
        for (int k = 0; k < H; ++k) {
          const float u = U[(long)k * GH + j];
#pragma unroll
          for (int r = 0; r < BB; ++r) acc[r] += c[r * H + k] * u;
        }
#pragma unroll
        for (int r = 0; r < BB; ++r) gb[r * GH + j] = tanhf(acc[r]);
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
      const int r = i / H, k = i - r * H;
      const float* g = gb + r * GH;
      float hn;
      if (CELL == 0) {
        const float z = g[k], hh = g[2 * H + k];
        hn = z * h[i] + (1.f - z) * hh;
      } else {
        const float cn = g[H + k] * c[i] + g[k] * g[2 * H + k];
        c[i] = cn;
        hn = g[3 * H + k] * tanhf(cn);
        cs[((long)(b0 + r) * (T + 1) + t + 1) * H + k] = cn;
      }
      h[i] = hn;
      hs[((long)(b0 + r) * (T + 1) + t + 1) * H + k] = hn;
      if (rs) y[((long)(b0 + r) * T + t) * H + k] = hn;
      else if (t == T - 1) y[(long)(b0 + r) * H + k] = hn;
    }
    for (int i = threadIdx.x; i < nb * GH; i += blockDim.x) {
      const int r = i / GH, j = i - r * GH;
      gates[((long)(b0 + r) * T + t) * GH + j] = gb[r * GH + j];
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------- backward
// UT = U^T [GH][H]; dgates [B][T][GH] = d(pre-activation)
template <int CELL>
__global__ __launch_bounds__(512) void rnn_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ UT,
                                                      const float* __restrict__ hs, const float* __restrict__ cs,
                                                      const float* __restrict__ gates, float* __restrict__ dgates,
                                                      int B, int T, int H, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  extern __shared__ float sm[];
  const int GH = G * H;
  float* dh = sm;            // [BB][H] running dh (into h_t)
  float* aux = dh + BB * H;  // [BB][H] GRU: dh*z direct part; LSTM: running dc
  float* dp = aux + BB * H;  // [BB][GH] pre-activation gradients of the step
  const int b0 = blockIdx.x * BB;
  const int nb = min(BB, B - b0);
  for (int i = threadIdx.x; i < BB * H; i += blockDim.x) dh[i] = aux[i] = 0.f;
  for (int i = threadIdx.x; i < BB * GH; i += blockDim.x) dp[i] = 0.f;
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
      const int r = i / H, k = i - r * H;
      const long row = (long)(b0 + r);
      float d = dh[i];
      if (rs) d += dy[(row * T + t) * H + k];
      else if (t == T - 1) d += dy[row * H + k];
      const float* g = gates + (row * T + t) * GH;
      const float hp = hs[(row * (T + 1) + t) * H + k];
      float* p = dp + r * GH;
      if (CELL == 0) {
        const float z = g[k], hh = g[2 * H + k];
        p[k] = d * (hp - hh) * hsig_d(z);
        p[2 * H + k] = d * (1.f - z) * (1.f - hh * hh);
        aux[i] = d * z;
      } else {
        const float gi = g[k], gf = g[H + k], gg = g[2 * H + k], go = g[3 * H + k];
        const float cn = cs[(row * (T + 1) + t + 1) * H + k], cp = cs[(row * (T + 1) + t) * H + k];
        const float tc = tanhf(cn);
        const float dc = aux[i] + d * go * (1.f - tc * tc);
        p[k] = dc * gg * hsig_d(gi);
        p[H + k] = dc * cp * hsig_d(gf);
        p[2 * H + k] = dc * gi * (1.f - gg * gg);
        p[3 * H + k] = d * tc * hsig_d(go);
        aux[i] = dc * gf;
      }
    }
    __syncthreads();
    if (CELL == 0) {  // d(r*h) = dp_h Uh^T -> dr, and the r-path contribution to dh_{t-1}
      for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
        const int r = i / H, k = i - r * H;
        const long row = (long)(b0 + r);
        const float* p = dp + r * GH;
        float drh = 0.f;
        for (int j = 0; j < H; ++j) drh += p[2 * H + j] * UT[(long)(2 * H + j) * H + k];
        const float hp = hs[(row * (T + 1) + t) * H + k];
        const float rg = gates[(row * T + t) * GH + H + k];
        dp[r * GH + H + k] = drh * hp * hsig_d(rg);
        aux[i] += drh * rg;
      }
      __syncthreads();
    }
    // dh_{t-1} = direct + dp[:, gates feeding from h] U^T
    const int jend = CELL == 0 ? 2 * H : GH;
    for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
      const int r = i / H, k = i - r * H;
      const float* p = dp + r * GH;
      float s = CELL == 0 ? aux[i] : 0.f;
      for (int j = 0; j < jend; ++j) s += p[j] * UT[(long)j * H + k];
      dh[i] = s;
    }
    for (int i = threadIdx.x; i < nb * GH; i += blockDim.x) {
      const int r = i / GH, j = i - r * GH;
      dgates[((long)(b0 + r) * T + t) * GH + j] = dp[r * GH + j];
    }
    __syncthreads();
  }
}

}  // namespace

int rnn_fwd(int cell, const float* xw, const float* U, float* hs, float* cs, float* gates, float* y, int B, int T,
            int H, int rs, hipStream_t s) {
  const int G = cell == 0 ? 3 : 4;
  const size_t lds = sizeof(float) * (2 * BB * H + BB * G * H);
  const int threads = std::min(512, ((G * H + 63) / 64) * 64);
  const dim3 grid((B + BB - 1) / BB);
  if (cell == 0)
    hipLaunchKernelGGL(rnn_fwd_kernel<0>, grid, dim3(threads), lds, s, xw, U, hs, cs, gates, y, B, T, H, rs);
  else
    hipLaunchKernelGGL(rnn_fwd_kernel<1>, grid, dim3(threads), lds, s, xw, U, hs, cs, gates, y, B, T, H, rs);
  return (int)hipGetLastError();
}

int rnn_bwd(int cell, const float* dy, const float* UT, const float* hs, const float* cs, const float* gates,
            float* dgates, int B, int T, int H, int rs, hipStream_t s) {
  const int G = cell == 0 ? 3 : 4;
  const size_t lds = sizeof(float) * (2 * BB * H + BB * G * H);
  const int threads = std::min(512, ((G * H + 63) / 64) * 64);
  const dim3 grid((B + BB - 1) / BB);
  if (cell == 0)
    hipLaunchKernelGGL(rnn_bwd_kernel<0>, grid, dim3(threads), lds, s, dy, UT, hs, cs, gates, dgates, B, T, H, rs);
  else
    hipLaunchKernelGGL(rnn_bwd_kernel<1>, grid, dim3(threads), lds, s, dy, UT, hs, cs, gates, dgates, B, T, H, rs);
  return (int)hipGetLastError();
}

}  // namespace ddl
