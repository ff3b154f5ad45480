// Standalone GEMM lab (no torch): times kernel variants of the framework's MFMA GEMM family on random
// bf16 operands, interleaved in one process, and checks each against the production 128x128 kernel
// (the same per-element MFMA K order, so outputs are expected to match bit for bit).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ../../distributeddeeplearningspark_amd/csrc/include \
//         lab.hip -o lab
//   ./lab M N K [bias] [rounds]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ddl_gemm256.h"
#include "ddl_gemm_kernel.h"
#include "gemm_variants.h"

using namespace ddl;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void init_bf16(bf16_t* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 15;
    x *= 0x2c1b3c6du;
    x ^= x >> 12;
    x *= 0x297a2d39u;
    x ^= x >> 15;
    const float f = (float)(x & 0xffffff) / 8388608.f - 1.f;  // uniform [-1, 1)
    p[i] = f2bf(f);
  }
}
__global__ void init_f32(float* p, long n, uint32_t seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 0x85ebca6bu ^ seed;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    p[i] = (float)(x & 0xffff) / 65536.f - 0.5f;
  }
}

struct Variant {
  std::string name;
  int (*fn)(const GemmParams&, hipStream_t);
};

template <int BN, int WM, int EPI>
int run_pp(const GemmParams& p, hipStream_t s) { return launch_pp<BN, WM, EPI>(p, s); }
template <int BN, int WM, int EPI, int RING>
int run_ppr(const GemmParams& p, hipStream_t s) { return launch_pp<BN, WM, EPI, RING>(p, s); }
template <int BN, int WM, int EPI>
int run_pp1(const GemmParams& p, hipStream_t s) { return launch_pp<BN, WM, EPI>(p, s, 1 << 30); }
template <int BN, int EPI>
int run_d2(const GemmParams& p, hipStream_t s) { return launch_d2<BN, EPI>(p, s); }
template <int EPI>
int run_kh(const GemmParams& p, hipStream_t s) { return launch_kh<EPI>(p, s); }
template <int EPI>
int run_t128(const GemmParams& p, hipStream_t s) { return launch_tile<128, 128, OP_KC, OP_KC, EPI>(p, s); }
template <int EPI>
int run_g256(const GemmParams& p, hipStream_t s) { return launch_g256<OP_KC, OP_KC, EPI>(p, s); }

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: lab M N K [epi: lite|bias|gelu|resid] [rounds]\n");
    return 2;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]);
  const std::string epi = argc > 4 ? argv[4] : "lite";
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const int iters = 20;
  bf16_t *A, *B, *R, *AUX;
  float* bias;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&R, (size_t)M * N * 2));
  CK(hipMalloc(&AUX, (size_t)M * N * 2));
  CK(hipMalloc(&bias, (size_t)N * 4));
  init_bf16<<<1024, 256>>>(A, (long)M * K, 1u);
  init_bf16<<<1024, 256>>>(B, (long)N * K, 2u);
  init_bf16<<<1024, 256>>>(R, (long)M * N, 3u);
  init_f32<<<64, 256>>>(bias, N, 4u);
  CK(hipDeviceSynchronize());

  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.a = A;
  p.lda = K;
  p.b = B;
  p.ldb = K;
  p.ldc = N;
  p.M = M;
  p.N = N;
  p.K = K;
  p.k_split = K;
  p.a_mode = OP_KC;
  p.b_mode = OP_KC;
  p.alpha = 1.f;
  p.group_m = 8;
  std::vector<Variant> vs;
  if (epi == "lite" || epi == "bias") {
    if (epi == "bias") p.bias = bias;
    vs = {{"t128", run_t128<EPI_BF16_LITE>},
          {"g256", run_g256<EPI_BF16_LITE>},
          {"pp256", run_pp<256, 2, EPI_BF16_LITE>},
          {"kh128", run_kh<EPI_BF16_LITE>},
          {"d2_128", run_d2<128, EPI_BF16_LITE>}};
  } else {
    p.bias = bias;
    if (epi == "gelu") {
      p.relu = ACT_GELU;
      p.aux = AUX;
    } else {
      p.resid = R;
      p.ldr = N;
    }
    vs = {{"t128", run_t128<EPI_BF16>},
          {"g256", run_g256<EPI_BF16>},
          {"pp256", run_pp<256, 2, EPI_BF16>},
          {"kh128", run_kh<EPI_BF16>},
          {"d2_128", run_d2<128, EPI_BF16>}};
  }
  const size_t cb = (size_t)M * N * 2;
  std::vector<bf16_t*> outs(vs.size());
  for (auto& o : outs) CK(hipMalloc(&o, cb));
  // correctness vs t128 (variant 0)
  std::vector<uint16_t> ref(M * (size_t)N), got(M * (size_t)N);
  for (size_t v = 0; v < vs.size(); ++v) {
    CK(hipMemset(outs[v], 0xff, cb));
    GemmParams q = p;
    q.c = outs[v];
    CK((hipError_t)vs[v].fn(q, 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(v == 0 ? ref.data() : got.data(), outs[v], cb, hipMemcpyDeviceToHost));
    if (v == 0) continue;
    size_t bad = 0, first = (size_t)-1;
    double maxd = 0;
    for (size_t i = 0; i < ref.size(); ++i) {
      if (ref[i] != got[i]) {
        uint32_t a = (uint32_t)ref[i] << 16, b = (uint32_t)got[i] << 16;
        float fa, fb;
        memcpy(&fa, &a, 4);
        memcpy(&fb, &b, 4);
        const double d = std::fabs((double)fa - fb) / (std::fabs((double)fa) + 1e-2);
        if (!(d <= 0.02)) {
          if (first == (size_t)-1) first = i;
          ++bad;
        }
        maxd = std::max(maxd, std::isfinite(d) ? d : 1e9);
      }
    }
    printf("check %-14s bad=%zu maxrel=%.3g first_bad=(%ld,%ld)\n", vs[v].name.c_str(), bad, maxd,
           first == (size_t)-1 ? -1L : (long)(first / N), first == (size_t)-1 ? -1L : (long)(first % N));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v < vs.size(); ++v) {
      GemmParams q = p;
      q.c = outs[v];
      vs[v].fn(q, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) vs[v].fn(q, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / iters);
    }
  }
  const double flop = 2.0 * M * N * (double)K;
  printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"epi\": \"%s\"", M, N, K, epi.c_str());
  for (size_t v = 0; v < vs.size(); ++v) {
    auto t = ms[v];
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    printf(", \"%s\": [%.4f, %.1f]", vs[v].name.c_str(), med, flop / med / 1e9);
  }
  printf("}\n");
  return 0;
}
