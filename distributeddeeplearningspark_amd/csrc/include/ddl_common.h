// Common device helpers for the CDNA4 (gfx950) kernels of the framework.
// Wave64, MFMA 16x16x32 bf16, LDS helpers.  No CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace ddl {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef uint16_t bf16_t;  // raw storage type for bf16 on the host/kernels boundary

#define DDL_LDS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even f32 -> bf16 (NaN kept NaN via the compiler's cvt)
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based dropout with uint8 thresholds: element `idx` of a call with seed `seed` is kept iff
// byte (idx & 3) of drop_hash4(seed + idx / 4) >= t8, and the kept values are scaled by 256 / (256 - t8)
// (the rate is quantised to 1/256: drop_t8 in ddl_ops.h).  Stateless, so backward passes regenerate
// the mask instead of storing it.  One hash serves four consecutive elements: the 64-bit counter is
// folded with a 24-bit multiply, premixed by one 32-bit multiply and finished with 24-bit multiplies
// (v_mul_u32_u24, full rate) — the previous per-element hash spent three quarter-rate v_mul_lo_u32
// on every element of the dropout-carrying LayerNorm / GEMM epilogues.
// Mirrored bit for bit by ops/transformer.py:drop_hash_ref.
__device__ __forceinline__ uint32_t drop_hash4(uint64_t q) {
  uint32_t x = ((uint32_t)q ^ __umul24((uint32_t)(q >> 32), 0x9E3779u)) * 0x9E3779B1u;
  x ^= x >> 16;
  x = __umul24(x, 0x7feb35u);
  x ^= x >> 15;
  x = __umul24(x, 0x846ca7u);
  return x ^ (x >> 16);
}
__device__ __forceinline__ bool drop_byte_keep(uint32_t h, uint32_t j, uint32_t t8) {
  return ((h >> (8u * (j & 3u))) & 0xffu) >= t8;
}
__device__ __forceinline__ bool drop_keep(uint64_t seed, uint64_t idx, uint32_t t8) {
  return drop_byte_keep(drop_hash4(seed + (idx >> 2)), (uint32_t)idx, t8);
}
// keep bits (bit e) of the 4 / 8 consecutive elements base, base + 1, ...: 1 / 2 hashes when base is
// 4-aligned, one more otherwise
__device__ __forceinline__ uint32_t drop_bits4(uint64_t seed, uint64_t base, uint32_t t8) {
  const uint64_t q = seed + (base >> 2);
  const uint32_t off = (uint32_t)base & 3u;
  const uint32_t h0 = drop_hash4(q), h1 = off ? drop_hash4(q + 1) : 0u;
  uint32_t bits = 0u;
#pragma unroll
  for (uint32_t e = 0; e < 4; ++e) {
    const uint32_t j = off + e;
    bits |= (drop_byte_keep(j < 4 ? h0 : h1, j, t8) ? 1u : 0u) << e;
  }
  return bits;
}
__device__ __forceinline__ uint32_t drop_bits8(uint64_t seed, uint64_t base, uint32_t t8) {
  const uint64_t q = seed + (base >> 2);
  const uint32_t off = (uint32_t)base & 3u;
  const uint32_t h0 = drop_hash4(q), h1 = drop_hash4(q + 1), h2 = off ? drop_hash4(q + 2) : 0u;
  uint32_t bits = 0u;
#pragma unroll
  for (uint32_t e = 0; e < 8; ++e) {
    const uint32_t j = off + e;
    bits |= (drop_byte_keep(j < 4 ? h0 : (j < 8 ? h1 : h2), j, t8) ? 1u : 0u) << e;
  }
  return bits;
}

// erf-form GELU and its derivative (BERT "gelu"; not the tanh approximation)
// erf without exp or branches (Abramowitz & Stegun 7.1.28, |error| <= 3e-7, far below bf16's
// 2^-9): 1 - (1 + a1 x + ... + a6 x^6)^-16 — 6 FMAs, 4 squarings and one v_rcp_f32.  In the GELU
// GEMM epilogues it replaced the library erff: BERT FFN1 forward 0.145 -> 0.131 ms, its GELU
// data-gradient 0.189 -> 0.144 ms (with the 8-B pre-activation load), BERT-base 671K -> 696K tok/s
__device__ __forceinline__ float erf_fast(float x) {
  const float a = fabsf(x);
  float p = fmaf(4.30638e-5f, a, 2.765672e-4f);
  p = fmaf(p, a, 1.520143e-4f);
  p = fmaf(p, a, 9.2705272e-3f);
  p = fmaf(p, a, 4.22820123e-2f);
  p = fmaf(p, a, 7.05230784e-2f);
  p = fmaf(p, a, 1.f);
  p *= p;
  p *= p;
  p *= p;
  p *= p;
  return copysignf(1.f - __builtin_amdgcn_rcpf(p), x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erf_fast(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// XCD-aware bijective remap of a 1-D block id (MI355X: 8 XCDs, blocks dealt round-robin).
// Blocks that share an XCD (bid % 8 equal) receive a contiguous range of logical tiles.
// 64 zero bytes: the source of LDS-DMA lanes whose element lies outside the operand
// (padding taps, rows / k past the end) — the DMA cannot write a constant.
static __device__ __attribute__((aligned(64))) uint4 ddl_zero_page[4];

// 16-B LDS-DMA (global_load_lds_dwordx4): lane i's 16 bytes land at lds_wave + 16 i, where
// lds_wave is the wave-uniform LDS byte address.  Issued from inline asm so the compiler does not
// see a pending LDS write (it would drain vmcnt(0) before every later LDS access); the kernel
// orders the ring itself with explicit s_waitcnt vmcnt + barriers.
__device__ __forceinline__ void dma16(const void* src, uint32_t lds_wave) {
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(lds_wave) : "memory", "m0");
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (uint32_t) reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p));
}
// s_waitcnt vmcnt(N) (gfx9 encoding), visible to the compiler's wait-insertion pass
// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup-scope fence + s_barrier,
// and the fence makes every wave drain its outstanding GLOBAL loads and stores (s_waitcnt vmcnt(0))
// first: in a latency-bound loop that streams results to HBM each iteration (the recurrent kernels)
// that is a full store round trip per barrier.  Here only the LDS / scalar queue is waited for; the
// "memory" clobber keeps the compiler from moving memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x0F70);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, idx = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Block -> (output tile, K split).  The remap runs over the WHOLE 2-D grid, split-major, so the
// output tiles of one K split are contiguous in the XCD-local order: they share the XCD's L2 and
// are resident at about the same time, and the K-slice both operands read for that split is
// fetched from HBM once per XCD instead of once per tile (the weight-gradient GEMMs have 5-9
// N-tiles per split; measured 976 MB fetched for a 206 MB problem with the 1-D remap).
__device__ __forceinline__ void grid_tile(int& tile, int& split) {
  const int tiles = gridDim.x;
  const int lin = xcd_remap(blockIdx.y * tiles + blockIdx.x, tiles * gridDim.y);
  split = lin / tiles;
  tile = lin - split * tiles;
}

}  // namespace ddl
