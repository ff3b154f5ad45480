// Persistent recurrent kernels (Keras-2 GRU reset_after=False, LSTM and SimpleRNN), fp32 like the
// reference's Keras models (GRU(128) / LSTM(128) over 25 steps).  The generic
// kernels take the activation / recurrent activation as ActCodes (ddl_act.h); the
// register-resident fast path below serves the Keras defaults (tanh + hard_sigmoid).
//
// The input projection x W + b of ALL time steps is one GEMM done before the kernel; the
// kernel then owns BB batch rows for the whole sequence: h (and c) stay in LDS across the
// T steps, every step reads U (fp32, L2/L1-resident) column-per-thread (coalesced) and the
// hidden state as an LDS broadcast.  Post-activation gates, the hidden / cell sequences
// are saved for the backward.
// Backward (BPTT) runs the same persistent structure in reverse time, propagating dh (and dc)
// with U^T columns per thread; it emits the pre-activation gate gradients of every step so
// that dW, dU, db and dx are plain GEMMs / reductions afterwards.
#include "ddl_act.h"

namespace ddl {
namespace {

constexpr int BB = 4;  // batch rows per workgroup

__device__ __forceinline__ float hsig(float x) { return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f); }
__device__ __forceinline__ float hsig_d(float y) { return (y > 0.f && y < 1.f) ? 0.2f : 0.f; }

// ----------------------------------------------------------------------------- forward
template <int CELL>  // 0 = GRU (gates z, r, h), 1 = LSTM (gates i, f, c, o), 2 = SimpleRNN (h)
__global__ __launch_bounds__(512) void rnn_fwd_kernel(const float* __restrict__ xw, const float* __restrict__ U,
                                                      float* __restrict__ hs, float* __restrict__ cs,
                                                      float* __restrict__ gates, float* __restrict__ y, int B, int T,
                                                      int H, int rs, int act, int ract) {
  constexpr int G = CELL == 0 ? 3 : (CELL == 1 ? 4 : 1);
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
      // LSTM candidate and SimpleRNN use the activation, every other gate the recurrent one
      const bool main_act = CELL == 2 || (CELL == 1 && j >= 2 * H && j < 3 * H);
#pragma unroll
      for (int r = 0; r < BB; ++r) gb[r * GH + j] = act_f(main_act ? act : ract, acc[r]);
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
        for (int r = 0; r < BB; ++r) gb[r * GH + j] = act_f(act, acc[r]);
      }
      __syncthreads();
    }
    for (int i = threadIdx.x; i < nb * H; i += blockDim.x) {
      const int r = i / H, k = i - r * H;
      const float* g = gb + r * GH;
      float hn;
      if (CELL == 2) {
        hn = g[k];
      } else if (CELL == 0) {
        const float z = g[k], hh = g[2 * H + k];
        hn = z * h[i] + (1.f - z) * hh;
      } else {
        const float cn = g[H + k] * c[i] + g[k] * g[2 * H + k];
        c[i] = cn;
        hn = g[3 * H + k] * act_f(act, cn);
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
                                                      int B, int T, int H, int rs, int act, int ract) {
  constexpr int G = CELL == 0 ? 3 : (CELL == 1 ? 4 : 1);
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
      if (CELL == 2) {
        p[k] = d * act_d(act, g[k]);
      } else if (CELL == 0) {
        const float z = g[k], hh = g[2 * H + k];
        p[k] = d * (hp - hh) * act_d(ract, z);
        p[2 * H + k] = d * (1.f - z) * act_d(act, hh);
        aux[i] = d * z;
      } else {
        const float gi = g[k], gf = g[H + k], gg = g[2 * H + k], go = g[3 * H + k];
        const float cn = cs[(row * (T + 1) + t + 1) * H + k], cp = cs[(row * (T + 1) + t) * H + k];
        const float tc = act_f(act, cn);
        const float dc = aux[i] + d * go * act_d(act, tc);
        p[k] = dc * gg * act_d(ract, gi);
        p[H + k] = dc * cp * act_d(ract, gf);
        p[2 * H + k] = dc * gi * act_d(act, gg);
        p[3 * H + k] = d * tc * act_d(ract, go);
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
        dp[r * GH + H + k] = drh * hp * act_d(ract, rg);
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
// lanes of a wave that read different chunks hit different banks.
// Every per-step global input is prefetched one step ahead into registers (its latency hides
// behind the current step's contractions); the input projection x W + b is computed in-kernel
// for narrow inputs (I <= 8: the reference's 25x1 load series), so a step is a pure chain of
// LDS contractions and barriers.  Element-wise phases map one (row, unit) element per thread.
// =============================================================================================
constexpr int CH = 64;       // k / j chunk held in registers
constexpr int CP = CH + 4;   // padded LDS chunk stride (floats)
constexpr int IMAX = 8;      // widest input fused into the kernels
constexpr int RNN_BB_FWD = 1, RNN_BB_BWD = 1;  // default rows per workgroup (H = 128), measured

__device__ __forceinline__ int cpos(int col) { return (col / CH) * CP + (col % CH); }

// lane ^ 1 / lane ^ 2 / ... partner value by DPP (VALU) instead of ds_bpermute (an LDS round trip
// on the recurrence's critical path): quad_perm within 4 lanes, row_ror / row_mirror patterns beyond
template <int O>
__device__ __forceinline__ float xor_lane(float v) {
  const int iv = __builtin_bit_cast(int, v);
  if constexpr (O == 1) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(iv, 0xB1, 0xf, 0xf, false));
  else if constexpr (O == 2) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(iv, 0x4E, 0xf, 0xf, false));
  else return __shfl_xor(v, O, 64);
}
// partner-quad value inside each 8-lane group (row_half_mirror): lane i reads lane 7 - i, i.e. a lane
// of the OTHER quad — equal to lane ^ 4 whenever the values are uniform within quads, as they are
// after the xor 1 / xor 2 steps of a sum reduction
__device__ __forceinline__ float other_quad(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xf, 0xf, false));
}

// The waitcnt pass treats the values loaded before a loop as possibly still in flight inside it and
// then waits, in every iteration, for whatever vector loads are outstanding at their first use (the
// next step's prefetch).  One real s_waitcnt vmcnt(0) before the loop (a builtin the pass models,
// unlike an asm string) retires them once.  gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15.
__device__ __forceinline__ void retire_vm_loads() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int CELL, int H>
constexpr int fwd_threads() { return (CELL == 0 ? 3 : 4) * H * (H / 64); }
template <int CELL, int H>
constexpr int bwd_threads() { return H * (((CELL == 0 ? 3 : 4) * H / 64) <= 4 ? 4 : 8); }

template <int CELL, int H, int BB_, bool FUSE>
__global__ __launch_bounds__((fwd_threads<CELL, H>())) void rnn_fwd_reg_kernel(
    const float* __restrict__ xw, const float* __restrict__ x, const float* __restrict__ W,
    const float* __restrict__ bias, int I, const float* __restrict__ U, float* __restrict__ hs,
    float* __restrict__ cs, float* __restrict__ gates, float* __restrict__ y, int B, int T, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int GH = G * H;
  constexpr int KS = H / CH;
  constexpr int HC = KS * CP;  // padded row length of h / c
  constexpr int NT = fwd_threads<CELL, H>();  // == blockDim.x (the launcher's block size)
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
  float wv[IMAX], bv = 0.f;  // input-projection column j (fused path); wv[i] = 0 past the input width
#pragma unroll
  for (int i = 0; i < IMAX; ++i) wv[i] = (FUSE && i < I) ? W[(long)i * GH + j] : 0.f;
  if (FUSE && bias) bv = bias[j];
  // Step t's inputs are fetched one step ahead and contracted only when used, so their latency hides
  // behind a whole step.  The x row address is workgroup-uniform: an opaque zero offset keeps the loads
  // on the vector path (a scalar load is counted by lgkmcnt, which every LDS barrier drains), and the
  // loads are unconditional at clamped indices (a runtime-guarded load per element makes the compiler
  // branch and wait per element); padded inputs meet wv = 0.
  int zoff;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zoff));
  auto fetch_x = [&](int t, float (&xr)[BB_][IMAX]) {
    const int tc = min(max(t, 0), T - 1);
#pragma unroll
    for (int r = 0; r < BB_; ++r) {
      const long bt = (long)(b0 + min(r, nb - 1)) * T + tc;
      if constexpr (!FUSE) {
        xr[r][0] = xw[bt * GH + j];
      } else {
#pragma unroll
        for (int i = 0; i < IMAX; ++i) xr[r][i] = x[bt * I + min(i, I - 1) + zoff];
      }
    }
  };
  auto proj = [&](const float (&xr)[BB_][IMAX], float* xv) {
#pragma unroll
    for (int r = 0; r < BB_; ++r) {
      if constexpr (!FUSE) {
        xv[r] = xr[r][0];
      } else {
        float a = bv;
#pragma unroll
        for (int i = 0; i < IMAX; ++i) a += xr[r][i] * wv[i];
        xv[r] = a;
      }
    }
  };
  for (int i = tid; i < BB_ * HC; i += NT) (&h[0][0])[i] = (&c[0][0])[i] = 0.f;
  // element owned in the state-update phase
  const int er = tid / H, ek = tid - er * H;
  const bool eown = er < nb;
  const long erow = b0 + er;
  if (eown) {
    hs[(erow * (T + 1)) * H + ek] = 0.f;
    if (CELL == 1) cs[(erow * (T + 1)) * H + ek] = 0.f;
  }
  float xr[BB_][IMAX], xv[BB_];
  fetch_x(0, xr);
  proj(xr, xv);
  retire_vm_loads();
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
      for (int r = 0; r < BB_; ++r) acc[r] += xor_lane<1>(acc[r]);
    }
  };
  for (int t = 0; t < T; ++t) {
    fetch_x(t + 1, xr);  // the next step's inputs (consumed at the end of this step)
    float acc[BB_];
    if (CELL == 1 || j < 2 * H) {  // wave-uniform: 2H columns span whole waves
      contract(h, acc);
      if (kh == 0) {
        const bool is_tanh = CELL == 1 && j >= 2 * H && j < 3 * H;
#pragma unroll
        for (int r = 0; r < BB_; ++r) gb[r][j] = is_tanh ? tanhf(acc[r] + xv[r]) : hsig(acc[r] + xv[r]);
      }
    }
    lds_barrier();
    if (CELL == 0) {
      for (int i = tid; i < BB_ * H; i += NT) {
        const int r = i / H, k = i - r * H;
        c[r][cpos(k)] = gb[r][H + k] * h[r][cpos(k)];
      }
      lds_barrier();
      if (j >= 2 * H) {
        contract(c, acc);
        if (kh == 0) {
#pragma unroll
          for (int r = 0; r < BB_; ++r) gb[r][j] = tanhf(acc[r] + xv[r]);
        }
      }
      lds_barrier();
    }
    // next step's projection before this step's stores: its wait then covers the loads issued at the
    // top of the step and the PREVIOUS step's stores (a whole step old), never the stores below
    float xnext[BB_];
    proj(xr, xnext);
#pragma unroll
    for (int r = 0; r < BB_; ++r) asm volatile("" ::"v"(xnext[r]) : "memory");  // computed here, not sunk past the stores
    if (eown) {
      float hn;
      if (CELL == 0) {
        const float z = gb[er][ek], hh = gb[er][2 * H + ek];
        hn = z * h[er][cpos(ek)] + (1.f - z) * hh;
      } else {
        const float cn = gb[er][H + ek] * c[er][cpos(ek)] + gb[er][ek] * gb[er][2 * H + ek];
        c[er][cpos(ek)] = cn;
        hn = gb[er][3 * H + ek] * tanhf(cn);
        cs[(erow * (T + 1) + t + 1) * H + ek] = cn;
      }
      h[er][cpos(ek)] = hn;
      hs[(erow * (T + 1) + t + 1) * H + ek] = hn;
      if (rs) y[(erow * T + t) * H + ek] = hn;
      else if (t == T - 1) y[erow * H + ek] = hn;
    }
    for (int i = tid; i < nb * GH; i += NT) {
      const int r = i / GH, jj = i - r * GH;
      gates[((long)(b0 + r) * T + t) * GH + jj] = gb[r][jj];
    }
#pragma unroll
    for (int r = 0; r < BB_; ++r) xv[r] = xnext[r];
    lds_barrier();
  }
}

template <int CELL, int H, int BB_>
__global__ __launch_bounds__((bwd_threads<CELL, H>())) void rnn_bwd_reg_kernel(
    const float* __restrict__ dy, const float* __restrict__ U, const float* __restrict__ hs,
    const float* __restrict__ cs, const float* __restrict__ gates, float* __restrict__ dgates, int B, int T, int rs) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int GH = G * H;
  constexpr int JS = GH / CH;                            // column chunks
  constexpr int JSP = JS <= 4 ? 4 : 8;                   // lanes per k (power of two)
  constexpr int ZR = CELL == 0 ? 2 * H / CH : JS;        // chunks feeding dh directly
  constexpr int NT = bwd_threads<CELL, H>();            // == blockDim.x
  __shared__ __attribute__((aligned(16))) float p[BB_][JS * CP];  // pre-activation gradients
  __shared__ float dh[BB_][H];
  __shared__ float aux[BB_][H];  // GRU: d*z direct part; LSTM: running dc
  __shared__ float hpl[BB_][H];  // GRU: h_{t-1} and r of the step, staged for the dr phase
  __shared__ float rgl[BB_][H];
  const int tid = threadIdx.x;
  const int k = tid / JSP, js = tid % JSP;
  const bool active = js < JS;
  const int b0 = blockIdx.x * BB_;
  const int nb = min(BB_, B - b0);
  float u[CH];
#pragma unroll
  for (int i = 0; i < CH; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(&U[(long)k * GH + min(js, JS - 1) * CH + i]);  // idle: unused
    u[i] = v.x; u[i + 1] = v.y; u[i + 2] = v.z; u[i + 3] = v.w;
  }
  for (int i = tid; i < BB_ * H; i += NT) (&dh[0][0])[i] = (&aux[0][0])[i] = 0.f;
  for (int i = tid; i < BB_ * JS * CP; i += NT) (&p[0][0])[i] = 0.f;
  // element owned in the element-wise phase, and its prefetched inputs
  const int er = tid / H, ek = tid - er * H;
  const bool eown = er < nb;
  const long erow = b0 + er;
  struct In { float d, g0, g1, g2, g3, hp, cn, cp; };
  auto load_in = [&](int t, In& v) {
    if (!eown || t < 0) return;
    v.d = rs ? dy[(erow * T + t) * H + ek] : (t == T - 1 ? dy[erow * H + ek] : 0.f);
    const float* g = gates + (erow * T + t) * GH;
    v.g0 = g[ek]; v.g1 = g[H + ek]; v.g2 = g[2 * H + ek];
    if (CELL == 1) {
      v.g3 = g[3 * H + ek];
      v.cn = cs[(erow * (T + 1) + t + 1) * H + ek];
      v.cp = cs[(erow * (T + 1) + t) * H + ek];
    } else {
      v.hp = hs[(erow * (T + 1) + t) * H + ek];
    }
  };
  In cur{}, nxt{};
  load_in(T - 1, cur);
  retire_vm_loads();
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
      acc[r] += xor_lane<1>(acc[r]);
      acc[r] += xor_lane<2>(acc[r]);
      if constexpr (JSP == 8) acc[r] += other_quad(acc[r]);
    }
  };
  for (int t = T - 1; t >= 0; --t) {
    load_in(t - 1, nxt);  // prefetch the previous step's saved activations
    if (eown) {
      const float d = dh[er][ek] + cur.d;
      float* pr = p[er];
      if (CELL == 0) {
        const float z = cur.g0, hh = cur.g2;
        pr[cpos(ek)] = d * (cur.hp - hh) * hsig_d(z);
        pr[cpos(2 * H + ek)] = d * (1.f - z) * (1.f - hh * hh);
        aux[er][ek] = d * z;
        hpl[er][ek] = cur.hp;
        rgl[er][ek] = cur.g1;
      } else {
        const float gi = cur.g0, gf = cur.g1, gg = cur.g2, go = cur.g3;
        const float tc = tanhf(cur.cn);
        const float dc = aux[er][ek] + d * go * (1.f - tc * tc);
        pr[cpos(ek)] = dc * gg * hsig_d(gi);
        pr[cpos(H + ek)] = dc * cur.cp * hsig_d(gf);
        pr[cpos(2 * H + ek)] = dc * gi * (1.f - gg * gg);
        pr[cpos(3 * H + ek)] = d * tc * hsig_d(go);
        aux[er][ek] = dc * gf;
      }
    }
    lds_barrier();
    // GRU: phase 0 = d(r*h) = dp_h Uh^T -> dr and the r-path part of dh_{t-1}; phase 1 = dh_{t-1}.
    // One call site for the contraction (keeps a single register-resident copy of U).
#pragma unroll 1
    for (int ph = CELL == 0 ? 0 : 1; ph < 2; ++ph) {
      float acc[BB_];
      contract(active && (ph == 0 ? js >= ZR : js < ZR), acc);
      if (js == 0) {
        if (ph == 0) {
#pragma unroll
          for (int r = 0; r < BB_; ++r) {
            const float rg = rgl[r][k];
            p[r][cpos(H + k)] = acc[r] * hpl[r][k] * hsig_d(rg);
            aux[r][k] += acc[r] * rg;
          }
        } else {
#pragma unroll
          for (int r = 0; r < BB_; ++r) dh[r][k] = (CELL == 0 ? aux[r][k] : 0.f) + acc[r];
        }
      }
      if (ph == 0) lds_barrier();
    }
    for (int i = tid; i < nb * GH; i += NT) {
      const int r = i / GH, jj = i - r * GH;
      dgates[((long)(b0 + r) * T + t) * GH + jj] = p[r][cpos(jj)];
    }
    cur = nxt;
    lds_barrier();
  }
}

// Parameter gradients of a recurrent layer in ONE launch, accumulated (fp32 atomics) straight
// into the gradient arena:  rows m < H      : gU[m][j] += sum_bt A(bt,m,j) dg[bt][j]
//                           rows H <= m < H+I: gW[m-H][j] += sum_bt x[bt][m-H] dg[bt][j]
//                           row m = H+I      : gb[j] += sum_bt dg[bt][j]
// with A = h_{t-1}[m] (GRU candidate columns: r[m] * h_{t-1}[m]).  Tile 64(m) x 64(j) over a
// chunk of PG_BT (b,t) rows staged in LDS; 256 threads x 4x4 outputs.
constexpr int PG_BT = 128;

template <int CELL>
__global__ __launch_bounds__(256) void rnn_param_grad_kernel(const float* __restrict__ dg, const float* __restrict__ hs,
                                                             const float* __restrict__ gates,
                                                             const float* __restrict__ x, float* __restrict__ gU,
                                                             float* __restrict__ gW, float* __restrict__ gb, int B,
                                                             int T, int H, int I) {
  constexpr int G = CELL == 0 ? 3 : (CELL == 1 ? 4 : 1);
  const int GH = G * H;
  const int M = H + I + (gb ? 1 : 0);
  const long BT = (long)B * T;
  const int m0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  const long bt0 = (long)blockIdx.z * PG_BT;
  const int nbt = (int)min((long)PG_BT, BT - bt0);
  __shared__ float As[PG_BT][64 + 1];
  __shared__ float Ds[PG_BT][64 + 1];
  const bool cand = CELL == 0 && j0 >= 2 * H;  // 2H is a multiple of 64
  // fill: thread owns column c and rows q = q0, q0+4, ...; (b, t) advance incrementally
  // (a runtime-T division per element would dominate the kernel)
  const int c = threadIdx.x & 63, q0 = threadIdx.x >> 6;
  long b = (bt0 + q0) / T, t = (bt0 + q0) - b * T;
  for (int q = q0; q < nbt; q += 4, t += 4) {
    while (t >= T) { t -= T; ++b; }
    const long bt = bt0 + q;
    const int m = m0 + c;
    float a = 0.f;
    if (m < H) {
      a = hs[(b * (T + 1) + t) * H + m];
      if (cand) a *= gates[bt * GH + H + m];
    } else if (m < H + I) {
      a = x[bt * I + (m - H)];
    } else if (m < M) {
      a = 1.f;
    }
    As[q][c] = a;
    const int jj = j0 + c;
    Ds[q][c] = jj < GH ? dg[bt * GH + jj] : 0.f;
  }
  __syncthreads();
  const int tm = (threadIdx.x / 16) * 4, tj = (threadIdx.x % 16) * 4;
  float acc[4][4] = {};
  for (int q = 0; q < nbt; ++q) {
    float a[4], d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = As[q][tm + i]; d[i] = Ds[q][tj + i]; }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int l = 0; l < 4; ++l) acc[i][l] += a[i] * d[l];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm + i;
    if (m >= M) continue;
    float* dst = m < H ? gU + (long)m * GH : (m < H + I ? gW + (long)(m - H) * GH : gb);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int jj = j0 + tj + l;
      if (jj < GH) atomicAdd(dst + jj, acc[i][l]);
    }
  }
}

template <int CELL, int H, int BB_>
int launch_fwd_reg(const float* xw, const float* x, const float* W, const float* b, int I, const float* U, float* hs,
                   float* cs, float* gates, float* y, int B, int T, int rs, hipStream_t s) {
  constexpr int G = CELL == 0 ? 3 : 4;
  static_assert(BB_ * H <= fwd_threads<CELL, H>(), "one state element per thread");
  if (!xw && (I < 1 || I > IMAX)) return (int)hipErrorInvalidValue;
  const dim3 grid((B + BB_ - 1) / BB_);
  if (xw)
    hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BB_, false>), grid, dim3(G * H * (H / CH)), 0, s, xw, x, W, b, I,
                       U, hs, cs, gates, y, B, T, rs);
  else
    hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BB_, true>), grid, dim3(G * H * (H / CH)), 0, s, xw, x, W, b, I,
                       U, hs, cs, gates, y, B, T, rs);
  return (int)hipGetLastError();
}

template <int CELL, int H, int BB_>
int launch_bwd_reg(const float* dy, const float* U, const float* hs, const float* cs, const float* gates,
                   float* dgates, int B, int T, int rs, hipStream_t s) {
  static_assert(BB_ * H <= bwd_threads<CELL, H>(), "one state element per thread");
  const dim3 grid((B + BB_ - 1) / BB_);
  hipLaunchKernelGGL((rnn_bwd_reg_kernel<CELL, H, BB_>), grid, dim3(bwd_threads<CELL, H>()), 0, s, dy, U, hs, cs,
                     gates, dgates, B, T, rs);
  return (int)hipGetLastError();
}

}  // namespace

bool rnn_fast_path(int H) { return H == 128 || H == 64; }
bool rnn_fuses_input(int H, int I) { return rnn_fast_path(H) && I <= IMAX; }
bool rnn_reg_path(int cell, int H, int act, int ract) {
  return (cell == 0 || cell == 1) && rnn_fast_path(H) && act == ACT_C_TANH && ract == ACT_C_HARD_SIGMOID;
}

// batch rows per workgroup of the register-resident kernels: fewer rows = more CUs busy and
// less VALU work per step (the recurrence is latency-bound); DDL_RNN_BB overrides (1/2/4)
static int rnn_rows_per_wg(int dflt) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DDL_RNN_BB");
    v = e ? atoi(e) : 0;
    if (v != 1 && v != 2 && v != 4) v = 0;
  }
  return v ? v : dflt;
}

int rnn_fwd(int cell, const float* xw, const float* x, const float* W, const float* b, int I, const float* U,
            float* hs, float* cs, float* gates, float* y, int B, int T, int H, int rs, int act, int ract,
            hipStream_t s) {
  const bool reg = rnn_reg_path(cell, H, act, ract);
  if (reg && H == 128) {
    const int bb = rnn_rows_per_wg(RNN_BB_FWD);
#define DDL_RNN_FWD(BBV)                                                                                    \
  return cell == 0 ? launch_fwd_reg<0, 128, BBV>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s)           \
                   : launch_fwd_reg<1, 128, BBV>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s)
    if (bb == 1) DDL_RNN_FWD(1);
    if (bb == 2) DDL_RNN_FWD(2);
    DDL_RNN_FWD(4);
#undef DDL_RNN_FWD
  }
  if (reg && H == 64)
    return cell == 0 ? launch_fwd_reg<0, 64, 2>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s)
                     : launch_fwd_reg<1, 64, 2>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s);
  if (!xw) return (int)hipErrorInvalidValue;  // generic kernels need the projection precomputed
  const int G = cell == 0 ? 3 : (cell == 1 ? 4 : 1);
  const size_t lds = sizeof(float) * (2 * BB * H + BB * G * H);
  const int threads = std::min(512, ((G * H + 63) / 64) * 64);
  const dim3 grid((B + BB - 1) / BB);
  if (cell == 0)
    hipLaunchKernelGGL(rnn_fwd_kernel<0>, grid, dim3(threads), lds, s, xw, U, hs, cs, gates, y, B, T, H, rs, act, ract);
  else if (cell == 1)
    hipLaunchKernelGGL(rnn_fwd_kernel<1>, grid, dim3(threads), lds, s, xw, U, hs, cs, gates, y, B, T, H, rs, act, ract);
  else
    hipLaunchKernelGGL(rnn_fwd_kernel<2>, grid, dim3(threads), lds, s, xw, U, hs, cs, gates, y, B, T, H, rs, act, ract);
  return (int)hipGetLastError();
}

bool rnn_bwd_uses_ut(int H) { return !rnn_fast_path(H); }

int rnn_param_grad(int cell, const float* dg, const float* hs, const float* gates, const float* x, float* gU,
                   float* gW, float* gb, int B, int T, int H, int I, hipStream_t s) {
  const int G = cell == 0 ? 3 : (cell == 1 ? 4 : 1);
  if (cell == 0 && (2 * H) % 64) return (int)hipErrorInvalidValue;  // candidate columns start on a tile
  const int M = H + I + (gb ? 1 : 0);
  const long BT = (long)B * T;
  const dim3 grid((M + 63) / 64, (G * H + 63) / 64, (unsigned)((BT + PG_BT - 1) / PG_BT));
  if (cell == 0)
    hipLaunchKernelGGL(rnn_param_grad_kernel<0>, grid, dim3(256), 0, s, dg, hs, gates, x, gU, gW, gb, B, T, H, I);
  else if (cell == 1)
    hipLaunchKernelGGL(rnn_param_grad_kernel<1>, grid, dim3(256), 0, s, dg, hs, gates, x, gU, gW, gb, B, T, H, I);
  else
    hipLaunchKernelGGL(rnn_param_grad_kernel<2>, grid, dim3(256), 0, s, dg, hs, gates, x, gU, gW, gb, B, T, H, I);
  return (int)hipGetLastError();
}

int rnn_bwd(int cell, const float* dy, const float* U, const float* UT, const float* hs, const float* cs,
            const float* gates, float* dgates, int B, int T, int H, int rs, int act, int ract, hipStream_t s) {
  const bool reg = rnn_reg_path(cell, H, act, ract);
  if (reg && H == 128) {
    const int bb = rnn_rows_per_wg(RNN_BB_BWD);
#define DDL_RNN_BWD(BBV)                                                                                    \
  return cell == 0 ? launch_bwd_reg<0, 128, BBV>(dy, U, hs, cs, gates, dgates, B, T, rs, s)                   \
                   : launch_bwd_reg<1, 128, BBV>(dy, U, hs, cs, gates, dgates, B, T, rs, s)
    if (bb == 1) DDL_RNN_BWD(1);
    if (bb == 4) DDL_RNN_BWD(4);
    DDL_RNN_BWD(2);
#undef DDL_RNN_BWD
  }
  if (reg && H == 64)
    return cell == 0 ? launch_bwd_reg<0, 64, 2>(dy, U, hs, cs, gates, dgates, B, T, rs, s)
                     : launch_bwd_reg<1, 64, 2>(dy, U, hs, cs, gates, dgates, B, T, rs, s);
  const int G = cell == 0 ? 3 : (cell == 1 ? 4 : 1);
  const size_t lds = sizeof(float) * (2 * BB * H + BB * G * H);
  const int threads = std::min(512, ((G * H + 63) / 64) * 64);
  const dim3 grid((B + BB - 1) / BB);
  if (cell == 0)
    hipLaunchKernelGGL(rnn_bwd_kernel<0>, grid, dim3(threads), lds, s, dy, UT, hs, cs, gates, dgates, B, T, H, rs, act,
                       ract);
  else if (cell == 1)
    hipLaunchKernelGGL(rnn_bwd_kernel<1>, grid, dim3(threads), lds, s, dy, UT, hs, cs, gates, dgates, B, T, H, rs, act,
                       ract);
  else
    hipLaunchKernelGGL(rnn_bwd_kernel<2>, grid, dim3(threads), lds, s, dy, UT, hs, cs, gates, dgates, B, T, H, rs, act,
                       ract);
  return (int)hipGetLastError();
}

}  // namespace ddl
