// fp32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32: exact fp32, a k-ordered fmaf chain).
//
// The reference's Keras models are fp32 (the NYISO GRU/LSTM regressors and their Dense(1)
// heads); their GEMMs are tiny and latency-bound (B*T = 800 rows, K <= 512), so
// this kernel favours a short critical path over peak rate: one 64x64 output tile per
// 256-thread workgroup, K staged through LDS 16 deep, each wave a 32x32 quadrant (2x2
// accumulators of 16x16, 4 independent MFMA chains cover the 40-cycle dependent latency).
//
//   C[m][n] = alpha * sum_k A(m,k) B(k,n) + beta * C[m][n] (+ bias[n]) (relu)
//   A(m,k) = a[m*sam + k*sak],  B(k,n) = b[k*sbk + n*sbn]
//
// Arbitrary element strides make every transpose combination of the forward / data-gradient /
// weight-gradient contractions one kernel (no transposed copies); the loads are coalesced
// along whichever of the two strides is 1.
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

constexpr int F_BM = 64, F_BN = 64, F_BK = 16;

__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ a, long sam, long sak,
                                                       const float* __restrict__ b, long sbk, long sbn,
                                                       float* __restrict__ c, long ldc, int M, int N, int K,
                                                       float alpha, float beta, const float* __restrict__ bias,
                                                       int relu) {
  __shared__ float As[F_BK][F_BM + 4];
  __shared__ float Bs[F_BK][F_BN + 4];
  const int tiles_n = (N + F_BN - 1) / F_BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / tiles_n) * F_BM, n0 = (bid % tiles_n) * F_BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  const bool a_kfast = sak == 1;  // block-uniform
  const bool b_nfast = sbn == 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < K; k0 += F_BK) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int e = threadIdx.x + v * 256;
      int mm, kk;
      if (a_kfast) { mm = e / F_BK; kk = e % F_BK; } else { kk = e / F_BM; mm = e % F_BM; }
      const int gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < K) ? a[(long)gm * sam + (long)gk * sak] : 0.f;
      int nn;
      if (b_nfast) { kk = e / F_BN; nn = e % F_BN; } else { nn = e / F_BK; kk = e % F_BK; }
      const int gn = n0 + nn, gk2 = k0 + kk;
      Bs[kk][nn] = (gn < N && gk2 < K) ? b[(long)gk2 * sbk + (long)gn * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kq = 0; kq < F_BK / 4; ++kq) {
      const int kr = kq * 4 + (lane >> 4);
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[kr][wm + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kr][wn + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // D layout: acc[i][j][e] = C[wm + 16i + 4(lane>>4) + e][wn + 16j + (lane&15)]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn + 16 * j + (lane & 15);
      if (n >= N) continue;
      const float bn = bias ? bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + e;
        if (m >= M) continue;
        float* dst = c + (long)m * ldc + n;
        float v = alpha * acc[i][j][e] + bn;
        if (beta != 0.f) v += beta * *dst;
        if (relu) v = fmaxf(v, 0.f);
        *dst = v;
      }
    }
}

}  // namespace

int gemm_f32(const float* a, long sam, long sak, const float* b, long sbk, long sbn, float* c, long ldc, int M, int N,
             int K, float alpha, float beta, const float* bias, int relu, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const int tiles = ((M + F_BM - 1) / F_BM) * ((N + F_BN - 1) / F_BN);
  hipLaunchKernelGGL(gemm_f32_kernel, dim3(tiles), dim3(256), 0, s, a, sam, sak, b, sbk, sbn, c, ldc, M, N, K, alpha,
                     beta, bias, relu);
  return (int)hipGetLastError();
}

}  // namespace ddl
