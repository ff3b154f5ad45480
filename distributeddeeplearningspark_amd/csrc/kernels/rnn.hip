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

// REP: replica-batched (RnnRep): the workgroup's replica is b0 / rp.B; W / U / bias come from its table
// entries and x from its resident shard at mini-batch (*rp.ctr % rp.nbr[r]) — outputs stay global-row indexed.
template <int CELL, int H, int BB_, bool FUSE, bool REP = false>
__global__ __launch_bounds__((fwd_threads<CELL, H>())) void rnn_fwd_reg_kernel(
    const float* __restrict__ xw, const float* __restrict__ x, const float* __restrict__ W,
    const float* __restrict__ bias, int I, const float* __restrict__ U, float* __restrict__ hs,
    float* __restrict__ cs, float* __restrict__ gates, float* __restrict__ y, int B, int T, int rs, const RnnRep rp) {
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
  long xrow0 = b0;  // input row of the workgroup's first batch row
  if constexpr (REP) {
    const int r = b0 / rp.B;
    U = rp.U[r];
    W = rp.W[r];
    bias = rp.b[r];
    x = rp.x[r];
    xrow0 = (long)(*rp.ctr % rp.nbr[r]) * rp.B + (b0 - r * rp.B);
  }
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
      const long bt = (xrow0 + min(r, nb - 1)) * T + tc;
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

template <int CELL, int H, int BB_, bool REP = false>
__global__ __launch_bounds__((bwd_threads<CELL, H>())) void rnn_bwd_reg_kernel(
    const float* __restrict__ dy, const float* __restrict__ U, const float* __restrict__ hs,
    const float* __restrict__ cs, const float* __restrict__ gates, float* __restrict__ dgates, int B, int T, int rs,
    const RnnRep rp) {
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
  if constexpr (REP) U = rp.U[b0 / rp.B];
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
  const RnnRep none{};
  if (xw)
    hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BB_, false>), grid, dim3(G * H * (H / CH)), 0, s, xw, x, W, b, I,
                       U, hs, cs, gates, y, B, T, rs, none);
  else
    hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BB_, true>), grid, dim3(G * H * (H / CH)), 0, s, xw, x, W, b, I,
                       U, hs, cs, gates, y, B, T, rs, none);
  return (int)hipGetLastError();
}

template <int CELL, int H, int BB_>
int launch_bwd_reg(const float* dy, const float* U, const float* hs, const float* cs, const float* gates,
                   float* dgates, int B, int T, int rs, hipStream_t s) {
  static_assert(BB_ * H <= bwd_threads<CELL, H>(), "one state element per thread");
  const dim3 grid((B + BB_ - 1) / BB_);
  const RnnRep none{};
  hipLaunchKernelGGL((rnn_bwd_reg_kernel<CELL, H, BB_>), grid, dim3(bwd_threads<CELL, H>()), 0, s, dy, U, hs, cs,
                     gates, dgates, B, T, rs, none);
  return (int)hipGetLastError();
}

}  // namespace

bool rnn_fast_path(int H) { return H == 128 || H == 64; }
bool rnn_fuses_input(int H, int I) { return rnn_fast_path(H) && I <= IMAX; }
bool rnn_reg_path(int cell, int H, int act, int ract) {
  return (cell == 0 || cell == 1) && rnn_fast_path(H) && act == ACT_C_TANH && ract == ACT_C_HARD_SIGMOID;
}


int rnn_fwd(int cell, const float* xw, const float* x, const float* W, const float* b, int I, const float* U,
            float* hs, float* cs, float* gates, float* y, int B, int T, int H, int rs, int act, int ract,
            hipStream_t s) {
  const bool reg = rnn_reg_path(cell, H, act, ract);
  if (reg && H == 128)  // one batch row per workgroup: more CUs busy, less VALU per step (latency-bound)
    return cell == 0 ? launch_fwd_reg<0, 128, RNN_BB_FWD>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s)
                     : launch_fwd_reg<1, 128, RNN_BB_FWD>(xw, x, W, b, I, U, hs, cs, gates, y, B, T, rs, s);
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
  if (reg && H == 128)
    return cell == 0 ? launch_bwd_reg<0, 128, RNN_BB_BWD>(dy, U, hs, cs, gates, dgates, B, T, rs, s)
                     : launch_bwd_reg<1, 128, RNN_BB_BWD>(dy, U, hs, cs, gates, dgates, B, T, rs, s);
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

// =============================================================================================
// Replica-batched training step (RnnRep / OptRep, ddl_ops.h; parallel/replica_batch.py).
// The reference runs its dist-keras workers as separate Keras models, num_processes per executor
// (ddl_nyiso_aztk.py:51-55, 206-218); on one MI355X the R co-located replicas of RNN(H) -> Dense(K)
// with an MSE loss are ONE launch per phase: the recurrences of all R x B batch rows run side by side
// (each workgroup reads its replica's U / W from the pointer table), the Dense head + loss + its
// backward is one workgroup per replica, and the parameter gradients and optimizer sweep take the
// replica from blockIdx.z / blockIdx.y.  Gradients are written (not accumulated), so no step zeroes them.
// =============================================================================================
namespace {

constexpr int kRepMaxB = 64, kRepMaxK = 8;

// One workgroup per replica: y = h Wd^T + bd, loss = mean (y - t)^2 over B K (Keras / ops.loss.mse),
// dy = 2 (y - t) / (B K); gWd = dy^T h, gbd = colsum dy, dh = dy Wd; history[ctr] = loss; Adam tick.
template <int H>
__global__ __launch_bounds__(256) void dense_mse_rep_kernel(const float* __restrict__ hlast, float* __restrict__ dh,
                                                            const RnnRep rp, const OptRep op) {
  const int r = blockIdx.x, B = rp.B, K = rp.K, tid = threadIdx.x;
  __shared__ float hsm[kRepMaxB][H + 1];
  __shared__ float dys[kRepMaxB][kRepMaxK];
  __shared__ float red[256];
  const float* hb = hlast + (long)r * B * H;
  for (int i = tid; i < B * H; i += 256) hsm[i / H][i % H] = hb[i];
  const int ctr = *rp.ctr;
  const bool live = ctr < rp.steps[r];  // ragged shards: an exhausted replica computes but does not step
  const float* tgt = rp.y[r] + (long)(ctr % rp.nbr[r]) * B * K;
  const float* Wd = rp.Wd[r];
  const float* bd = rp.bd[r];
  __syncthreads();
  const float sc = 2.f / (float)(B * K);
  float se = 0.f;
  for (int q = tid; q < B * K; q += 256) {
    const int b = q / K, o = q - b * K;
    float a = bd ? bd[o] : 0.f;
    const float* w = Wd + (long)o * H;
#pragma unroll 8
    for (int i = 0; i < H; ++i) a += hsm[b][i] * w[i];
    const float e = a - tgt[q];
    se += e * e;
    dys[b][o] = sc * e;
  }
  red[tid] = se;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) {
    rp.live[r] = live ? 1 : 0;  // read by the optimizer sweep of this step
    if (live) {
      rp.hist[r][ctr] = red[0] / (float)(B * K);
      if (op.t[r]) op.t[r][0] += 1.f;  // Adam's device step counter (read by the optimizer sweep below)
    }
  }
  // gWd[o][i] = sum_b dy[b][o] h[b][i];  gbd[o] = sum_b dy[b][o]
  for (int q = tid; q < K * H; q += 256) {
    const int o = q / H, i = q - o * H;
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += dys[b][o] * hsm[b][i];
    rp.gWd[r][q] = a;
  }
  if (rp.gbd[r] && tid < K) {
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += dys[b][tid];
    rp.gbd[r][tid] = a;
  }
  // dh[b][i] = sum_o dy[b][o] Wd[o][i]  (the recurrent backward's dy at the last step)
  float* dhb = dh + (long)r * B * H;
  for (int q = tid; q < B * H; q += 256) {
    const int b = q / H, i = q - b * H;
    float a = 0.f;
    for (int o = 0; o < K; ++o) a += dys[b][o] * Wd[(long)o * H + i];
    dhb[q] = a;
  }
}

// Recurrent parameter gradients: rows m < H gU, H <= m < H + I gW, m = H + I gb (as rnn_param_grad).
// blockIdx.z = replica * S + slice: a workgroup sums PG_BT-row chunks [slice, slice + S, ...) of its
// replica's B T rows.  S = 1 (deterministic mode): one writer per output, plain stores in row order;
// S > 1: fp32 atomics into gradients the optimizer sweep of the previous step left zeroed.
template <int CELL>
__global__ __launch_bounds__(256) void rnn_param_grad_rep_kernel(const float* __restrict__ dg, const float* __restrict__ hs,
                                                                 const float* __restrict__ gates, const RnnRep rp,
                                                                 int T, int H, int I, int S) {
  constexpr int G = CELL == 0 ? 3 : (CELL == 1 ? 4 : 1);
  const int GH = G * H, r = blockIdx.z / S, slice = blockIdx.z - r * S, B = rp.B;
  const bool has_b = rp.gb[r] != nullptr;
  const int M = H + I + (has_b ? 1 : 0);
  const long BT = (long)B * T, row0 = (long)r * B;  // global batch row of the replica's row 0
  const long xrow0 = (long)(*rp.ctr % rp.nbr[r]) * B;  // shard row of its mini-batch
  const float* x = rp.x[r];
  const int m0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  __shared__ float As[PG_BT][64 + 1];
  __shared__ float Ds[PG_BT][64 + 1];
  const bool cand = CELL == 0 && j0 >= 2 * H;
  const int c = threadIdx.x & 63, q0 = threadIdx.x >> 6;
  const int tm = (threadIdx.x / 16) * 4, tj = (threadIdx.x % 16) * 4;
  float acc[4][4] = {};
  for (long bt0 = (long)slice * PG_BT; bt0 < BT; bt0 += (long)S * PG_BT) {
    const int nbt = (int)min((long)PG_BT, BT - bt0);
    long b = (bt0 + q0) / T, t = (bt0 + q0) - b * T;
    for (int q = q0; q < nbt; q += 4, t += 4) {
      while (t >= T) { t -= T; ++b; }
      const long gbt = (row0 + b) * T + t;  // global (row, step)
      const int m = m0 + c;
      float a = 0.f;
      if (m < H) {
        a = hs[((row0 + b) * (T + 1) + t) * H + m];
        if (cand) a *= gates[gbt * GH + H + m];
      } else if (m < H + I) {
        a = x[((xrow0 + b) * T + t) * I + (m - H)];
      } else if (m < M) {
        a = 1.f;
      }
      As[q][c] = a;
      const int jj = j0 + c;
      Ds[q][c] = jj < GH ? dg[gbt * GH + jj] : 0.f;
    }
    __syncthreads();
    for (int q = 0; q < nbt; ++q) {
      float a[4], d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] = As[q][tm + i]; d[i] = Ds[q][tj + i]; }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int l = 0; l < 4; ++l) acc[i][l] += a[i] * d[l];
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + tm + i;
    if (m >= M) continue;
    float* dst = m < H ? rp.gU[r] + (long)m * GH : (m < H + I ? rp.gW[r] + (long)(m - H) * GH : rp.gb[r]);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      const int jj = j0 + tj + l;
      if (jj < GH) {
        if (S == 1) dst[jj] = acc[i][l];
        else atomicAdd(dst + jj, acc[i][l]);
      }
    }
  }
}

// Optimizer sweep over the R replica arenas (blockIdx.y = replica), Keras semantics as the per-replica
// kernels (optim.hip): OPT 0 SGD (+momentum p1), 1 Adagrad, 2 Adam (b1 = p1, b2 = p2, amode as adam_step).
// zero_g: leave the gradients zeroed for the next step's atomic parameter-gradient slices.  Block (0, 0)
// advances the shared step counter (no block of this kernel reads it: the live flags come from the head kernel).
// A dead replica (ragged shard exhausted) keeps its parameters and state; its gradients are still zeroed.
template <int OPT>
__global__ __launch_bounds__(256) void opt_rep_kernel(const OptRep op, long n4, float lr, float p1, float p2, float eps,
                                                      float wd, int amode, int* ctr, const int* __restrict__ live,
                                                      int zero_g) {
  const int r = blockIdx.y;
  if (!live[r]) {
    if (zero_g) {
      float4* g = const_cast<float4*>(reinterpret_cast<const float4*>(op.g[r]));
      for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256)
        g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *ctr += 1;
    return;
  }
  float4* w = reinterpret_cast<float4*>(op.w[r]);
  float4* g = const_cast<float4*>(reinterpret_cast<const float4*>(op.g[r]));
  float4* s1 = reinterpret_cast<float4*>(op.s1[r]);
  float4* s2 = reinterpret_cast<float4*>(op.s2[r]);
  float bc1 = 1.f, bc2 = 1.f;
  if constexpr (OPT == 2) {
    const float t = op.t[r][0];
    bc1 = 1.f - powf(p1, t);
    bc2 = 1.f - powf(p2, t);
  }
  const float sbc2 = sqrtf(bc2);
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float4 p = w[i], d = g[i];
    float4 a = s1 ? s1[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 v = (OPT == 2) ? s2[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float *pp = &p.x, *dd = &d.x, *aa = &a.x, *vv = &v.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if constexpr (OPT == 0) {
        float gg = dd[k] + wd * pp[k];
        if (s1) {
          aa[k] = p1 * aa[k] + gg;
          gg = aa[k];
        }
        pp[k] -= lr * gg;
      } else if constexpr (OPT == 1) {
        const float gg = dd[k] + wd * pp[k];
        aa[k] += gg * gg;
        pp[k] -= lr * gg / (sqrtf(aa[k]) + eps);
      } else {
        float gg = dd[k];
        if (amode & 1) pp[k] *= (1.f - lr * wd);
        else gg += wd * pp[k];
        aa[k] = p1 * aa[k] + (1.f - p1) * gg;
        vv[k] = p2 * vv[k] + (1.f - p2) * gg * gg;
        if (amode & 2) pp[k] -= lr * (sbc2 / bc1) * aa[k] / (sqrtf(vv[k]) + eps);
        else pp[k] -= lr * (aa[k] / bc1) / (sqrtf(vv[k]) / sbc2 + eps);
      }
    }
    w[i] = p;
    if (s1) s1[i] = a;
    if constexpr (OPT == 2) s2[i] = v;
    if (zero_g) g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *ctr += 1;
}

template <int CELL, int H>
int rep_step(const RnnRep& rp, int R, int T, int I, float* hs, float* cs, float* gates, float* hlast, float* dh,
             float* dgates, const OptRep& op, long n, int opt, float lr, float p1, float p2, float eps, float wd,
             int amode, hipStream_t s) {
  constexpr int G = CELL == 0 ? 3 : 4;
  constexpr int BBF = H == 128 ? RNN_BB_FWD : 2, BBB = H == 128 ? RNN_BB_BWD : 2;
  const int RB = R * rp.B;
  hipLaunchKernelGGL((rnn_fwd_reg_kernel<CELL, H, BBF, true, true>), dim3((RB + BBF - 1) / BBF),
                     dim3(fwd_threads<CELL, H>()), 0, s, (const float*)nullptr, (const float*)nullptr,
                     (const float*)nullptr, (const float*)nullptr, I, (const float*)nullptr, hs, cs, gates, hlast, RB,
                     T, 0, rp);
  hipLaunchKernelGGL((dense_mse_rep_kernel<H>), dim3(R), dim3(256), 0, s, hlast, dh, rp, op);
  hipLaunchKernelGGL((rnn_bwd_reg_kernel<CELL, H, BBB, true>), dim3((RB + BBB - 1) / BBB), dim3(bwd_threads<CELL, H>()),
                     0, s, dh, (const float*)nullptr, hs, cs, gates, dgates, RB, T, 0, rp);
  const int M = H + I + 1;
  // row slices of the parameter gradients (atomics); deterministic mode: one ordered writer per output
  const int S = deterministic() ? 1 : (int)std::max<long>(1, ((long)rp.B * T + PG_BT - 1) / PG_BT);
  hipLaunchKernelGGL((rnn_param_grad_rep_kernel<CELL>), dim3((M + 63) / 64, (G * H + 63) / 64, R * S), dim3(256), 0,
                     s, dgates, hs, gates, rp, T, H, I, S);
  const long n4 = n / 4;
  const dim3 og((unsigned)std::min<long>((n4 + 255) / 256, 1024), R);
  const int zg = S > 1;
  if (opt == 0)
    hipLaunchKernelGGL(opt_rep_kernel<0>, og, dim3(256), 0, s, op, n4, lr, p1, p2, eps, wd, amode, rp.ctr, rp.live,
                       zg);
  else if (opt == 1)
    hipLaunchKernelGGL(opt_rep_kernel<1>, og, dim3(256), 0, s, op, n4, lr, p1, p2, eps, wd, amode, rp.ctr, rp.live,
                       zg);
  else
    hipLaunchKernelGGL(opt_rep_kernel<2>, og, dim3(256), 0, s, op, n4, lr, p1, p2, eps, wd, amode, rp.ctr, rp.live,
                       zg);
  return (int)hipGetLastError();
}

}  // namespace

bool rnn_replica_ok(int cell, int H, int I, int K, int B) {
  return (cell == 0 || cell == 1) && (H == 128 || (H == 64 && B % 2 == 0)) && I >= 1 && I <= IMAX && K >= 1 &&
         K <= kRepMaxK && B >= 1 && B <= kRepMaxB;
}

int rnn_replica_step(int cell, const RnnRep& rp, int R, int T, int H, int I, float* hs, float* cs, float* gates,
                     float* hlast, float* dh, float* dgates, const OptRep& op, long n, int opt, float lr, float p1,
                     float p2, float eps, float wd, int amode, hipStream_t s) {
  if (!rnn_replica_ok(cell, H, I, rp.K, rp.B) || R < 1 || R > kMaxRnnRep || n % 4 || opt < 0 || opt > 2 || !rp.live)
    return (int)hipErrorInvalidValue;
  for (int r = 0; r < R; ++r)
    if (rp.nbr[r] < 1) return (int)hipErrorInvalidValue;
  if (cell == 0)
    return H == 128 ? rep_step<0, 128>(rp, R, T, I, hs, cs, gates, hlast, dh, dgates, op, n, opt, lr, p1, p2, eps, wd, amode, s)
                    : rep_step<0, 64>(rp, R, T, I, hs, cs, gates, hlast, dh, dgates, op, n, opt, lr, p1, p2, eps, wd, amode, s);
  return H == 128 ? rep_step<1, 128>(rp, R, T, I, hs, cs, gates, hlast, dh, dgates, op, n, opt, lr, p1, p2, eps, wd, amode, s)
                  : rep_step<1, 64>(rp, R, T, I, hs, cs, gates, hlast, dh, dgates, op, n, opt, lr, p1, p2, eps, wd, amode, s);
}

}  // namespace ddl
