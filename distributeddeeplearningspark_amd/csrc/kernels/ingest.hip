// Device ETL kernels for the dist-keras column transformers (SURVEY §2.4 "device ingest
// kernels"): the column is copied to HBM once and transformed there, fp64 like the host
// DataFrame engine so results are bit-compatible with the vectorised numpy path.
//   minmax   y = (x - o_min) * scale + n_min              (MinMaxTransformer, any direction)
//   one_hot  y[i][k] = (label[i] == k)                     (OneHotTransformer)
//   argmax   idx[i] = argmax_k x[i][k]  (first maximum)     (LabelIndexTransformer)
#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

__global__ __launch_bounds__(256) void minmax_kernel(const double* __restrict__ x, double* __restrict__ y, long n,
                                                     double o_min, double scale, double n_min) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) y[i] = (x[i] - o_min) * scale + n_min;
}

__global__ __launch_bounds__(256) void one_hot_kernel(const int64_t* __restrict__ lab, double* __restrict__ y, long n,
                                                      int K, int* __restrict__ bad) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n * K; e += (long)gridDim.x * 256) {
    const long i = e / K;
    const int k = (int)(e - i * K);
    const int64_t l = lab[i];
    if (k == 0 && (l < 0 || l >= K)) atomicOr(bad, 1);
    y[e] = (l == k) ? 1.0 : 0.0;
  }
}

// one wave per row; ties resolve to the lowest index (numpy semantics)
__global__ __launch_bounds__(256) void argmax_kernel(const double* __restrict__ x, long rows, int K, long ld,
                                                     int64_t* __restrict__ out) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  double best = -INFINITY;
  int bi = K;
  for (int k = lane; k < K; k += 64) {
    const double v = x[r * ld + k];
    if (v > best || (v == best && k < bi) || (bi == K && v != v)) {
      best = v;
      bi = k;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) out[r] = bi >= K ? 0 : bi;
}

inline unsigned grid_for(long n) { return (unsigned)std::max(1L, std::min((n + 255) / 256, 4096L)); }

}  // namespace

int etl_minmax(const double* x, double* y, long n, double o_min, double scale, double n_min, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(minmax_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, y, n, o_min, scale, n_min);
  return (int)hipGetLastError();
}

int etl_one_hot(const int64_t* labels, double* y, long n, int K, int* bad, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(one_hot_kernel, dim3(grid_for(n * K)), dim3(256), 0, s, labels, y, n, K, bad);
  return (int)hipGetLastError();
}

int etl_argmax(const double* x, long rows, int K, long ld, int64_t* out, hipStream_t s) {
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(argmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, x, rows, K, ld, out);
  return (int)hipGetLastError();
}

}  // namespace ddl
