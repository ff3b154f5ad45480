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


// =============================================================================================
// Register-resident fast path (H = 64 / 128, the reference's GRU(128) / LSTM(128)).
//
// The generic kernels above stream U from L2 on every step (latency-bound: ~3 ms per GRU step
// at B=32).  Here each workgroup pins the WHOLE recurrent matrix in VGPRs for the sequence:
//  forward : thread (j, kh) holds U[kh*64 .. kh*64+63][j]  (KS = H/64 lane-adjacent k-splits,
//            reduced with one xor-shuffle), so NT = G*H*KS threads (768 GRU / 1024 LSTM);
//  backward: thread (k, js) holds U[k][js*64 .. js*64+63]  (row chunk, contiguous loads),
//            JSP = pow2(G*H/64) lane-adjacent chunks reduced with xor-shuffles.
// h / (r*h) / gate-gradient rows live in LDS with 64-float chunks padded to 68 floats, so the
// lanes of a wave that read different chunks hit different banks.  Per step the only global
// traffic is the x W + b row (prefetched at the top of the step) and the saved activations.
// =============================================================================================
constexpr int CH = 64;       // k / j chunk held in registers
constexpr int CP = CH + 4;   // padded LDS chunk stride (floats)

__device__ __forceinline__ int cpos(int col) { return (col / CH) * CP + (col % CH); }

template <int CELL, int H>
constexpr int fwd_threads() { return (CELL == 0 ? 3 : 4) * H * (H / 64); }
template <int CELL, int H>
constexpr int bwd_threads() { return H * (((CELL == 0 ? 3 : 4) * H / 64) <= 4 ? 4 : 8); }

template <int CELL, int H, int BB_>
__global__ __launch_bounds__((fwd_threads<CELL, H>())) void rnn_fwd_reg_kernel(const float* __restrict__ xw, const float* __restrict__ U,
                                                           float* __restrict__ hs, float* __restrict__ cs,
                                                           float* __restrict__ gates, float* __restrict__ y, int B,
                                                           int T, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int GH = G * H;
  constexpr int KS = H / CH;
  constexpr int HC = KS * CP;  // padded row length of h / c
  __shared__ __attribute__((aligned(16))) float h[BB_][HC];
  __shared__ __attribute__((aligned(16))) float c[BB_][HC];  // LSTM cell state / GRU r*h
  __shared__ float gb[BB_][GH];
  const int tid = threadIdx.x;
  const int j = tid / KS, kh = tid % KS;
  const int b0 = blockIdx.x * BB_;
  const int nb = min(BB_, B - b0);
  float u[CH];
#pragma unroll
  for (int i = 0; i < CH; ++i) u[i] = U[(long)(kh * CH + i) * GH + j];
  for (int i = tid; i < BB_ * HC; i += blockDim.x) (&h[0][0])[i] = (&c[0][0])[i] = 0.f;
  for (int i = tid; i < nb * H; i += blockDim.x) {
    const int r = i / H, k = i - r * H;
    hs[((long)(b0 + r) * (T + 1)) * H + k] = 0.f;
    if (CELL == 1) cs[((long)(b0 + r) * (T + 1)) * H + k] = 0.f;
  }
  __syncthreads();
  auto contract = [&](float (*src)[HC], float* acc) {
#pragma unroll
    for (int r = 0; r < BB_; ++r) acc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < CH; i += 4) {
#pragma unroll
      for (int r = 0; r < BB_; ++r) {
        const float4 v = *reinterpret_cast<const float4*>(&src[r][kh * CP + i]);
        acc[r] += v.x * u[i] + v.y * u[i + 1] + v.z * u[i + 2] + v.w * u[i + 3];
      }
    }
    if (KS == 2) {
#pragma unroll
      for (int r = 0; r < BB_; ++r) acc[r] += __shfl_xor(acc[r], 1, 64);
    }
  };
  for (int t = 0; t < T; ++t) {
    float xv[BB_];
#pragma unroll
    for (int r = 0; r < BB_; ++r) xv[r] = (kh == 0 && r < nb) ? xw[((long)(b0 + r) * T + t) * GH + j] : 0.f;
    float acc[BB_];
    if (CELL == 1 || j < 2 * H) {  // wave-uniform: 2H columns span whole waves
      contract(h, acc);
      if (kh == 0) {
        const bool is_tanh = CELL == 1 && j >= 2 * H && j < 3 * H;
#pragma unroll
        for (int r = 0; r < BB_; ++r) gb[r][j] = is_tanh ? tanhf(acc[r] + xv[r]) : hsig(acc[r] + xv[r]);
      }
    }
    __syncthreads();
    if (CELL == 0) {
      for (int i = tid; i < BB_ * H; i += blockDim.x) {
        const int r = i / H, k = i - r * H;
        c[r][cpos(k)] = gb[r][H + k] * h[r][cpos(k)];
      }
      __syncthreads();
      if (j >= 2 * H) {
        contract(c, acc);
        if (kh == 0) {
#pragma unroll
          for (int r = 0; r < BB_; ++r) gb[r][j] = tanhf(acc[r] + xv[r]);
        }
      }
      __syncthreads();
    }
    for (int i = tid; i < nb * H; i += blockDim.x) {
      const int r = i / H, k = i - r * H;
      const long row = b0 + r;
      float hn;
      if (CELL == 0) {
        const float z = gb[r][k], hh = gb[r][2 * H + k];
        hn = z * h[r][cpos(k)] + (1.f - z) * hh;
      } else {
        const float cn = gb[r][H + k] * c[r][cpos(k)] + gb[r][k] * gb[r][2 * H + k];
        c[r][cpos(k)] = cn;
        hn = gb[r][3 * H + k] * tanhf(cn);
        cs[(row * (T + 1) + t + 1) * H + k] = cn;
      }
      h[r][cpos(k)] = hn;
      hs[(row * (T + 1) + t + 1) * H + k] = hn;
      if (rs) y[(row * T + t) * H + k] = hn;
      else if (t == T - 1) y[row * H + k] = hn;
    }
    for (int i = tid; i < nb * GH; i += blockDim.x) {
      const int r = i / GH, jj = i - r * GH;
      gates[((long)(b0 + r) * T + t) * GH + jj] = gb[r][jj];
    }
    __syncthreads();
  }
}

template <int CELL, int H, int BB_>
__global__ __launch_bounds__((bwd_threads<CELL, H>())) void rnn_bwd_reg_kernel(const float* __restrict__ dy, const float* __restrict__ U,
                                                           const float* __restrict__ hs, const float* __restrict__ cs,
                                                           const float* __restrict__ gates,
                                                           float* __restrict__ dgates, int B, int T, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int GH = G * H;
  constexpr int JS = GH / CH;                            // column chunks
  constexpr int JSP = JS <= 4 ? 4 : 8;                   // lanes per k (power of two)
  constexpr int ZR = CELL == 0 ? 2 * H / CH : JS;        // chunks feeding dh directly
  __shared__ __attribute__((aligned(16))) float p[BB_][JS * CP];  // pre-activation gradients
  __shared__ float dh[BB_][H];
  __shared__ float aux[BB_][H];  // GRU: d*z direct part; LSTM: running dc
  const int tid = threadIdx.x;
  const int k = tid / JSP, js = tid % JSP;
  const bool active = js < JS;
  const int b0 = blockIdx.x * BB_;
  const int nb = min(BB_, B - b0);
  float u[CH];
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(&U[(long)k * GH + min(js, JS - 1) * CH + i]);  // idle lanes: never used
    u[i] = v.x; u[i + 1] = v.y; u[i + 2] = v.z; u[i + 3] = v.w;
  }
  for (int i = tid; i < BB_ * H; i += blockDim.x) (&dh[0][0])[i] = (&aux[0][0])[i] = 0.f;
  for (int i = tid; i < BB_ * JS * CP; i += blockDim.x) (&p[0][0])[i] = 0.f;
  __syncthreads();
  auto contract = [&](bool use, float* acc) {
#pragma unroll
    for (int r = 0; r < BB_; ++r) acc[r] = 0.f;
    // every lane computes (no divergence inside the unrolled dot); lanes whose chunk is not
    // part of this contraction drop their partial before the shuffle reduction
    const int jc = min(js, JS - 1);
#pragma unroll
    for (int i = 0; i < CH; i += 4) {
#pragma unroll
      for (int r = 0; r < BB_; ++r) {
        const float4 v = *reinterpret_cast<const float4*>(&p[r][jc * CP + i]);
        acc[r] += v.x * u[i] + v.y * u[i + 1] + v.z * u[i + 2] + v.w * u[i + 3];
      }
      if ((i & 15) == 12) __builtin_amdgcn_sched_barrier(0);  // bound the LDS loads in flight
    }
#pragma unroll
    for (int r = 0; r < BB_; ++r) {
      acc[r] = use ? acc[r] : 0.f;
#pragma unroll
      for (int o = 1; o < JSP; o <<= 1) acc[r] += __shfl_xor(acc[r], o, 64);
    }
  };
  for (int t = T - 1; t >= 0; --t) {
    for (int i = tid; i < nb * H; i += blockDim.x) {
      const int r = i / H, kk = i - r * H;
      const long row = b0 + r;
      float d = dh[r][kk];
      if (rs) d += dy[(row * T + t) * H + kk];
      else if (t == T - 1) d += dy[row * H + kk];
      const float* g = gates + (row * T + t) * GH;
      float* pr = p[r];
      if (CELL == 0) {
        const float hp = hs[(row * (T + 1) + t) * H + kk];
        const float z = g[kk], hh = g[2 * H + kk];
        pr[cpos(kk)] = d * (hp - hh) * hsig_d(z);
        pr[cpos(2 * H + kk)] = d * (1.f - z) * (1.f - hh * hh);
        aux[r][kk] = d * z;
      } else {
        const float gi = g[kk], gf = g[H + kk], gg = g[2 * H + kk], go = g[3 * H + kk];
        const float cn = cs[(row * (T + 1) + t + 1) * H + kk], cp = cs[(row * (T + 1) + t) * H + kk];
        const float tc = tanhf(cn);
        const float dc = aux[r][kk] + d * go * (1.f - tc * tc);
        pr[cpos(kk)] = dc * gg * hsig_d(gi);
        pr[cpos(H + kk)] = dc * cp * hsig_d(gf);
        pr[cpos(2 * H + kk)] = dc * gi * (1.f - gg * gg);
        pr[cpos(3 * H + kk)] = d * tc * hsig_d(go);
        aux[r][kk] = dc * gf;
      }
    }
    __syncthreads();
    // GRU: phase 0 = d(r*h) = dp_h Uh^T -> dr and the r-path part of dh_{t-1}; phase 1 = dh_{t-1}.
    // One call site for the contraction (keeps a single register-resident copy of U).
#pragma unroll 1
    for (int ph = CELL == 0 ? 0 : 1; ph < 2; ++ph) {
      float acc[BB_];
      contract(active && (ph == 0 ? js >= ZR : js < ZR), acc);
      if (js == 0) {
        if (ph == 0) {
          for (int r = 0; r < nb; ++r) {
            const long row = b0 + r;
            const float hp = hs[(row * (T + 1) + t) * H + k];
            const float rg = gates[(row * T + t) * GH + H + k];
            p[r][cpos(H + k)] = acc[r] * hp * hsig_d(rg);
            aux[r][k] += acc[r] * rg;
          }
        } else {
#pragma unroll
          for (int r = 0; r < BB_; ++r) dh[r][k] = (CELL == 0 ? aux[r][k] : 0.f) + acc[r];
        }
      }
      if (ph == 0) __syncthreads();
    }
    for (int i = tid; i < nb * GH; i += blockDim.x) {
      const int r = i / GH, jj = i - r * GH;
      dgates[((long)(b0 + r) * T + t) * GH + jj] = p[r][cpos(jj)];
    }
    __syncthreads();
  }
}

template <int CELL, int H, int BB_>
int launch_fwd_reg(const float* xw, const float* U, float* hs, float* cs, float* gates, float* y, int B, int T, int rs,
                   hipStream_t s) {
  constexpr int G = CELL == 0 ? 3 : 4;
  const dim3 grid((B + BB_ - 1) / BB_);
  hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BB_>), grid, dim3(G * H * (H / CH)), 0, s, xw, U, hs, cs, gates, y,
                     B, T, rs);
  return (int)hipGetLastError();
}

template <int CELL, int H, int BB_>
int launch_bwd_reg(const float* dy, const float* U, const float* hs, const float* cs, const float* gates,
                   float* dgates, int B, int T, int rs, hipStream_t s) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int JS = G * H / CH;
  constexpr int JSP = JS <= 4 ? 4 : 8;
  const dim3 grid((B + BB_ - 1) / BB_);
  hipLaunchKernelGGL((rnn_bwd_reg_kernel<CELL, H, BB_>), grid, dim3(H * JSP), 0, s, dy, U, hs, cs, gates, dgates, B,
                     T, rs);
  return (int)hipGetLastError();
}

}  // namespace

int rnn_fwd(int cell, const float* xw, const float* U, float* hs, float* cs, float* gates, float* y, int B, int T,
            int H, int rs, hipStream_t s) {
  if (H == 128)
    return cell == 0 ? launch_fwd_reg<0, 128, 4>(xw, U, hs, cs, gates, y, B, T, rs, s)
                     : launch_fwd_reg<1, 128, 4>(xw, U, hs, cs, gates, y, B, T, rs, s);
  if (H == 64)
    return cell == 0 ? launch_fwd_reg<0, 64, 2>(xw, U, hs, cs, gates, y, B, T, rs, s)
                     : launch_fwd_reg<1, 64, 2>(xw, U, hs, cs, gates, y, B, T, rs, s);
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

bool rnn_bwd_uses_ut(int H) { return H != 128 && H != 64; }

int rnn_bwd(int cell, const float* dy, const float* U, const float* UT, const float* hs, const float* cs,
            const float* gates, float* dgates, int B, int T, int H, int rs, hipStream_t s) {
  if (H == 128)
    return cell == 0 ? launch_bwd_reg<0, 128, 2>(dy, U, hs, cs, gates, dgates, B, T, rs, s)
                     : launch_bwd_reg<1, 128, 4>(dy, U, hs, cs, gates, dgates, B, T, rs, s);
  if (H == 64)
    return cell == 0 ? launch_bwd_reg<0, 64, 2>(dy, U, hs, cs, gates, dgates, B, T, rs, s)
                     : launch_bwd_reg<1, 64, 2>(dy, U, hs, cs, gates, dgates, B, T, rs, s);
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
