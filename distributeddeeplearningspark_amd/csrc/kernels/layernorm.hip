// LayerNorm forward/backward, BERT embeddings forward/backward, partial-row column sums.
//
// Rows are processed one wave per row with 16-B vectors (lane owns vectors lane, lane+64, ...
// of the row), statistics in fp32 registers, two-pass (mean, then centred variance).
// Backward: dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma, and the
// parameter gradients are accumulated per lane across the rows a wave visits, then
// written as one partial row per wave (no atomics); colsum_partials finishes them.
// The residual-branch dropout mask (same hash and element index as the producing GEMM's
// epilogue) is regenerated here so the masked gradient leaves in the same pass.
#include <algorithm>

#include <cstdlib>

#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(w[e] << 16);
    f[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8f(const float* f) {
  return make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]),
                    pack_bf16x2(f[6], f[7]));
}

// One wave per row, grid-stride over rows; gamma / beta of the lane's columns live in registers
// (loading them per element per row cost 4x the bytes of the row itself through L1).
// PF: the next row's vectors are loaded before this row's two reductions (one row in flight under
// the math of the current one; without it each row paid the full load latency serially).
template <int VPL, bool PF>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean, float* __restrict__ rstd, long M, int H,
                                                     float eps, uint32_t thresh, float dscale,
                                                     unsigned long long seed) {
  const int lane = threadIdx.x & 63;
  const int nv = H >> 3;
  float gm[VPL][8], bt[VPL][8];
#pragma unroll
  for (int u = 0; u < VPL; ++u) {  // 16-B loads (gamma / beta rows are 32-B aligned: H % 8 == 0)
    const int c = lane + 64 * u;
    const bool ok = c < nv;
    const float4 g0 = (gamma && ok) ? reinterpret_cast<const float4*>(gamma)[2 * c] : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 g1 = (gamma && ok) ? reinterpret_cast<const float4*>(gamma)[2 * c + 1] : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 b0 = (beta && ok) ? reinterpret_cast<const float4*>(beta)[2 * c] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 b1 = (beta && ok) ? reinterpret_cast<const float4*>(beta)[2 * c + 1] : make_float4(0.f, 0.f, 0.f, 0.f);
    gm[u][0] = g0.x; gm[u][1] = g0.y; gm[u][2] = g0.z; gm[u][3] = g0.w;
    gm[u][4] = g1.x; gm[u][5] = g1.y; gm[u][6] = g1.z; gm[u][7] = g1.w;
    bt[u][0] = b0.x; bt[u][1] = b0.y; bt[u][2] = b0.z; bt[u][3] = b0.w;
    bt[u][4] = b1.x; bt[u][5] = b1.y; bt[u][6] = b1.z; bt[u][7] = b1.w;
  }
  const long rstep = (long)gridDim.x * 4;
  long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  uint4 nx[VPL];
  auto fetch = [&](long r) {
#pragma unroll
    for (int u = 0; u < VPL; ++u)
      if (lane + 64 * u < nv) nx[u] = *reinterpret_cast<const uint4*>(x + r * H + (lane + 64 * u) * 8);
  };
  if (PF && row < M) fetch(row);
  for (; row < M; row += rstep) {
    uint4 cur[VPL];
    if (PF) {
#pragma unroll
      for (int u = 0; u < VPL; ++u) cur[u] = nx[u];
      if (row + rstep < M) fetch(row + rstep);
    } else {
      fetch(row);
#pragma unroll
      for (int u = 0; u < VPL; ++u) cur[u] = nx[u];
    }
    float v[VPL][8];
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const int c = lane + 64 * u;
      if (c < nv) {
        unpack8(cur[u], v[u]);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[u][e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
      }
    }
    const float mu = warp_sum(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int u = 0; u < VPL; ++u)
      if (lane + 64 * u < nv)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[u][e] - mu;
          q += d * d;
        }
    const float rs = rsqrtf(warp_sum(q) / (float)H + eps);
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const int c = lane + 64 * u;
      if (c < nv) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[u][e] - mu) * rs * gm[u][e] + bt[u][e];
        if (thresh) {  // output dropout (BERT embeddings), element index row*H + n
          const uint32_t kb = drop_bits8(seed, (unsigned long long)row * (unsigned long long)H + c * 8, thresh);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = ((kb >> e) & 1u) ? o[e] * dscale : 0.f;
        }
        *reinterpret_cast<uint4*>(y + row * H + c * 8) = pack8f(o);
      }
    }
    if (lane == 0) {
      mean[row] = mu;
      rstd[row] = rs;
    }
  }
}

// BR: the 4 waves of a workgroup sum their parameter-gradient partials through LDS and write ONE partial row
// per workgroup (H <= 1024): twice the waves of the per-wave form at the same partial-row count (so the same
// column-sum cost), 4 rows per wave instead of 8 — the sweep was latency-bound at 2 waves per SIMD.
template <int VPL, bool PF, bool BR = false>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                                     bf16_t* __restrict__ dxd, uint32_t thresh, float dscale,
                                                     unsigned long long seed, float* __restrict__ ws, long M, int H,
                                                     uint32_t in_thresh, float in_scale, unsigned long long in_seed,
                                                     int parts) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int nv = H >> 3;
  float dg[VPL][8], db[VPL][8], dd[VPL][8], gmv[VPL][8];
#pragma unroll
  for (int u = 0; u < VPL; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      dg[u][e] = db[u][e] = dd[u][e] = 0.f;
    }
#pragma unroll
  for (int u = 0; u < VPL; ++u) {  // hoisted out of the rows; 16-B loads (gamma is 16-B aligned: host check)
    const int c = lane + 64 * u;
    const bool ok = gamma && c < nv;
    const float4 g0 = ok ? reinterpret_cast<const float4*>(gamma)[2 * c] : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 g1 = ok ? reinterpret_cast<const float4*>(gamma)[2 * c + 1] : make_float4(1.f, 1.f, 1.f, 1.f);
    gmv[u][0] = g0.x; gmv[u][1] = g0.y; gmv[u][2] = g0.z; gmv[u][3] = g0.w;
    gmv[u][4] = g1.x; gmv[u][5] = g1.y; gmv[u][6] = g1.z; gmv[u][7] = g1.w;
  }
  // PF: the next row's dy / x vectors and statistics are loaded before this row's math (VPL <= 2 only:
  // the prefetched row costs 16 VGPRs per VPL and the VPL = 8 instantiation spilled)
  uint4 ndy[VPL], nx[VPL];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long r) {
#pragma unroll
    for (int u = 0; u < VPL; ++u)
      if (lane + 64 * u < nv) {
        ndy[u] = *reinterpret_cast<const uint4*>(dy + r * H + (lane + 64 * u) * 8);
        nx[u] = *reinterpret_cast<const uint4*>(x + r * H + (lane + 64 * u) * 8);
      }
    nmu = mean[r];
    nrs = rstd[r];
  };
  if (PF && wave < M) fetch(wave);
  for (long row = wave; row < M; row += nwaves) {
    uint4 cdy[VPL], cx[VPL];
    if (PF) {
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        cdy[u] = ndy[u];
        cx[u] = nx[u];
      }
    } else {  // loads stay inside the vector loop below (the VPL = 8 instantiation is at the VGPR limit)
      nmu = mean[row];
      nrs = rstd[row];
    }
    const float mu = nmu, rs = nrs;
    if (PF && row + nwaves < M) fetch(row + nwaves);
    float gy[VPL][8], xh[VPL][8];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const int c = lane + 64 * u;
      if (c < nv) {
        float d[8], xv[8];
        unpack8(PF ? cdy[u] : *reinterpret_cast<const uint4*>(dy + row * H + c * 8), d);
        unpack8(PF ? cx[u] : *reinterpret_cast<const uint4*>(x + row * H + c * 8), xv);
        if (in_thresh) {  // dy arrives through the forward's output dropout
          const unsigned long long base = (unsigned long long)row * (unsigned long long)H + c * 8;
          const uint32_t kb = drop_bits8(in_seed, base, in_thresh);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = ((kb >> e) & 1u) ? d[e] * in_scale : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xhat = (xv[e] - mu) * rs;
          const float gm = gmv[u][e];
          dg[u][e] += d[e] * xhat;
          db[u][e] += d[e];
          xh[u][e] = xhat;
          gy[u][e] = d[e] * gm;
          a += gy[u][e];
          b += gy[u][e] * xhat;
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xh[u][e] = gy[u][e] = 0.f;
      }
    }
    a = warp_sum(a) / (float)H;
    b = warp_sum(b) / (float)H;
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const int c = lane + 64 * u;
      if (c < nv) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rs * (gy[u][e] - a - xh[u][e] * b);
        uint4 packed = pack8f(o);
        *reinterpret_cast<uint4*>(dx + row * H + c * 8) = packed;
        if (dxd) {
          const unsigned long long base = (unsigned long long)row * (unsigned long long)H + c * 8;
          const uint32_t kb = drop_bits8(seed, base, thresh);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = ((kb >> e) & 1u) ? o[e] * dscale : 0.f;
          packed = pack8f(o);
          *reinterpret_cast<uint4*>(dxd + row * H + c * 8) = packed;
        }
        if (parts == 3) {  // column sums of the stored gradient (dx_drop, else dx): the sublayer's bias grad
          float r[8];
          unpack8(packed, r);
#pragma unroll
          for (int e = 0; e < 8; ++e) dd[u][e] += r[e];
        }
      }
    }
  }
  if constexpr (BR) {
  if (ws) {
    // block reduce: waves 1..3 park [dbias | dgamma | dbeta] in LDS, wave 0 adds them and writes the row
    __shared__ float red[3][3 * 8 * 64 * VPL];
    const int w = threadIdx.x >> 6;
    constexpr int CW = 8 * 64 * VPL;  // columns of one part held by a wave (>= H)
    if (w > 0) {
      float* r = red[w - 1];
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        const int c = lane + 64 * u;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          r[c * 8 + e] = dd[u][e];
          r[CW + c * 8 + e] = dg[u][e];
          r[2 * CW + c * 8 + e] = db[u][e];
        }
      }
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const float* r = red[q];
#pragma unroll
        for (int u = 0; u < VPL; ++u) {
          const int c = lane + 64 * u;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            dd[u][e] += r[c * 8 + e];
            dg[u][e] += r[CW + c * 8 + e];
            db[u][e] += r[2 * CW + c * 8 + e];
          }
        }
      }
    } else {
      return;
    }
  }
  }
  if (ws) {
    // parts == 2: [dgamma | dbeta]; parts == 3: [dbias | dgamma | dbeta] (the arena order of a
    // sublayer's output bias followed by the LayerNorm's gamma and beta)
    float* wb = ws + (long)(BR ? blockIdx.x : wave) * parts * H;
    float* w0 = parts == 3 ? wb + H : wb;
    if (parts == 3) {
#pragma unroll
      for (int u = 0; u < VPL; ++u) {
        const int c = lane + 64 * u;
        if (c < nv) {
          *reinterpret_cast<float4*>(wb + c * 8) = make_float4(dd[u][0], dd[u][1], dd[u][2], dd[u][3]);
          *reinterpret_cast<float4*>(wb + c * 8 + 4) = make_float4(dd[u][4], dd[u][5], dd[u][6], dd[u][7]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
      const int c = lane + 64 * u;
      if (c < nv) {
        *reinterpret_cast<float4*>(w0 + c * 8) = make_float4(dg[u][0], dg[u][1], dg[u][2], dg[u][3]);
        *reinterpret_cast<float4*>(w0 + c * 8 + 4) = make_float4(dg[u][4], dg[u][5], dg[u][6], dg[u][7]);
        *reinterpret_cast<float4*>(w0 + H + c * 8) = make_float4(db[u][0], db[u][1], db[u][2], db[u][3]);
        *reinterpret_cast<float4*>(w0 + H + c * 8 + 4) = make_float4(db[u][4], db[u][5], db[u][6], db[u][7]);
      }
    }
  }
}

// 8-byte-vector form for H = 256 NQ (NQ = 1..4; BERT-base H = 768: NQ = 3): one wave per row, each lane owns NQ
// 4-column quads (64 lanes x 8 B = one contiguous 512-B segment per load instruction), so every lane is busy —
// the 16-B form leaves a third of the lanes without their second vector at H = 768 — and the per-lane
// parameter-gradient partials are 3 x 4 NQ registers (the 16-B form holds 3 x 16).  The next row's dy / x /
// statistics are loaded before this row's math.  Partial rows: one per workgroup (LDS block reduce), the layout
// of ln_bwd_kernel's BR form, so colsum_partials finishes both.
__device__ __forceinline__ void unpack4(const uint2& u, float* f) {
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ uint2 pack4f(const float* f) {
  return make_uint2(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]));
}

template <int NQ>
__global__ __launch_bounds__(256) void ln_bwd_q_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                       const float* __restrict__ mean, const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma, bf16_t* __restrict__ dx,
                                                       bf16_t* __restrict__ dxd, uint32_t thresh, float dscale,
                                                       unsigned long long seed, float* __restrict__ ws, long M, int H,
                                                       uint32_t in_thresh, float in_scale, unsigned long long in_seed,
                                                       int parts) {
  const int lane = threadIdx.x & 63;
  const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long nwaves = (long)gridDim.x * 4;
  float dg[NQ][4], db[NQ][4], dd[NQ][4], gmv[NQ][4];
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int c = lane + 64 * u;  // quad index: columns 4c .. 4c + 3
    const float4 g = gamma ? reinterpret_cast<const float4*>(gamma)[c] : make_float4(1.f, 1.f, 1.f, 1.f);
    gmv[u][0] = g.x; gmv[u][1] = g.y; gmv[u][2] = g.z; gmv[u][3] = g.w;
#pragma unroll
    for (int e = 0; e < 4; ++e) dg[u][e] = db[u][e] = dd[u][e] = 0.f;
  }
  uint2 ndy[NQ], nx[NQ];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](long r) {
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      ndy[u] = *reinterpret_cast<const uint2*>(dy + r * H + (lane + 64 * u) * 4);
      nx[u] = *reinterpret_cast<const uint2*>(x + r * H + (lane + 64 * u) * 4);
    }
    nmu = mean[r];
    nrs = rstd[r];
  };
  if (wave < M) fetch(wave);
  for (long row = wave; row < M; row += nwaves) {
    uint2 cdy[NQ], cx[NQ];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      cdy[u] = ndy[u];
      cx[u] = nx[u];
    }
    const float mu = nmu, rs = nrs;
    if (row + nwaves < M) fetch(row + nwaves);
    float gy[NQ][4], xh[NQ][4];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int c = lane + 64 * u;
      float d[4], xv[4];
      unpack4(cdy[u], d);
      unpack4(cx[u], xv);
      if (in_thresh) {  // dy arrives through the forward's output dropout
        const uint32_t kb = drop_bits4(in_seed, (unsigned long long)row * (unsigned long long)H + c * 4, in_thresh);
#pragma unroll
        for (int e = 0; e < 4; ++e) d[e] = ((kb >> e) & 1u) ? d[e] * in_scale : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xhat = (xv[e] - mu) * rs;
        dg[u][e] += d[e] * xhat;
        db[u][e] += d[e];
        xh[u][e] = xhat;
        gy[u][e] = d[e] * gmv[u][e];
        a += gy[u][e];
        b += gy[u][e] * xhat;
      }
    }
    a = warp_sum(a) / (float)H;
    b = warp_sum(b) / (float)H;
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int c = lane + 64 * u;
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rs * (gy[u][e] - a - xh[u][e] * b);
      uint2 packed = pack4f(o);
      *reinterpret_cast<uint2*>(dx + row * H + c * 4) = packed;
      if (dxd) {
        const uint32_t kb = drop_bits4(seed, (unsigned long long)row * (unsigned long long)H + c * 4, thresh);
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = ((kb >> e) & 1u) ? o[e] * dscale : 0.f;
        packed = pack4f(o);
        *reinterpret_cast<uint2*>(dxd + row * H + c * 4) = packed;
      }
      if (parts == 3) {  // column sums of the stored gradient (dx_drop, else dx): the sublayer's bias grad
        float r[4];
        unpack4(packed, r);
#pragma unroll
        for (int e = 0; e < 4; ++e) dd[u][e] += r[e];
      }
    }
  }
  if (!ws) return;
  constexpr int CW = 4 * 64 * NQ;  // = H
  __shared__ float red[3][3 * CW];
  const int w = threadIdx.x >> 6;
  if (w > 0) {
    float* r = red[w - 1];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int c = lane + 64 * u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r[c * 4 + e] = dd[u][e];
        r[CW + c * 4 + e] = dg[u][e];
        r[2 * CW + c * 4 + e] = db[u][e];
      }
    }
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float* r = red[q];
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int c = lane + 64 * u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        dd[u][e] += r[c * 4 + e];
        dg[u][e] += r[CW + c * 4 + e];
        db[u][e] += r[2 * CW + c * 4 + e];
      }
    }
  }
  float* wb = ws + (long)blockIdx.x * parts * H;
  float* w0 = parts == 3 ? wb + H : wb;
#pragma unroll
  for (int u = 0; u < NQ; ++u) {
    const int c = lane + 64 * u;
    if (parts == 3) *reinterpret_cast<float4*>(wb + c * 4) = make_float4(dd[u][0], dd[u][1], dd[u][2], dd[u][3]);
    *reinterpret_cast<float4*>(w0 + c * 4) = make_float4(dg[u][0], dg[u][1], dg[u][2], dg[u][3]);
    *reinterpret_cast<float4*>(w0 + H + c * 4) = make_float4(db[u][0], db[u][1], db[u][2], db[u][3]);
  }
}

// out[n] += sum_p ws[p][n]; block = 64 columns x 16 row-lanes over a chunk of kColsumRows rows,
// grid.y = row chunks (one fp32 atomic per column per block; out zeroed by the launcher when
// not accumulating)
constexpr int kColsumRows = 128;
__global__ __launch_bounds__(1024) void colsum_kernel(const float* __restrict__ ws, int P, int N, long ld,
                                                      float* __restrict__ out, int chunk) {
  __shared__ float red[16][65];
  const int n = blockIdx.x * 64 + threadIdx.x;
  const int p0 = blockIdx.y * chunk, p1 = min(P, p0 + chunk);
  float s = 0.f;
  if (n < N)
    for (int p = p0 + threadIdx.y; p < p1; p += 16) s += ws[(long)p * ld + n];
  red[threadIdx.y][threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.y == 0 && n < N) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += red[r][threadIdx.x];
    atomicAdd(out + n, t);
  }
}

// 16-B form (N, ld % 4 == 0): a workgroup = 64 column quads (256 columns) x 4 row-lanes over a chunk of 32 rows;
// every lane keeps four row loads in flight (the 4-B form issued one dependent load per row: 7.4 us for BERT's
// 1024 x 2304 LayerNorm partial rows, 1.3 TB/s).  One fp32 atomic per column per workgroup.
constexpr int kColsumVecRows = 32;
__global__ __launch_bounds__(256) void colsum_vec_kernel(const float* __restrict__ ws, int P, int N, long ld,
                                                         float* __restrict__ out) {
  __shared__ float4 red[4][64];
  const int q = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + q * 4;
  const int p0 = blockIdx.y * kColsumVecRows, p1 = min(P, p0 + kColsumVecRows);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    int p = p0 + rl;
    for (; p + 12 < p1; p += 16) {
      float4 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = *reinterpret_cast<const float4*>(ws + (long)(p + 4 * r) * ld + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a.x += v[r].x; a.y += v[r].y; a.z += v[r].z; a.w += v[r].w;
      }
    }
    for (; p < p1; p += 4) {
      const float4 v = *reinterpret_cast<const float4*>(ws + (long)p * ld + n);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[rl][q] = a;
  __syncthreads();
  if (rl == 0 && n < N) {
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      a.x += red[r][q].x; a.y += red[r][q].y; a.z += red[r][q].z; a.w += red[r][q].w;
    }
    atomicAdd(out + n, a.x);
    atomicAdd(out + n + 1, a.y);
    atomicAdd(out + n + 2, a.z);
    atomicAdd(out + n + 3, a.w);
  }
}

// deterministic mode: 16 columns x 64 row-lanes per workgroup (4x the workgroups of colsum_kernel's
// one-chunk form, a quarter of the serial loop), rows summed in a fixed order, one writer per column
__global__ __launch_bounds__(1024) void colsum_det_kernel(const float* __restrict__ ws, int P, int N, long ld,
                                                          float* __restrict__ out) {
  __shared__ float red[64][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int n = blockIdx.x * 16 + tx;
  float s = 0.f;
  if (n < N)
    for (int p = ty; p < P; p += 64) s += ws[(long)p * ld + n];
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && n < N) {
    float t = 0.f;
    for (int r = 0; r < 64; ++r) t += red[r][tx];
    out[n] += t;
  }
}

__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ types,
                                                        const bf16_t* __restrict__ word, const bf16_t* __restrict__ pos,
                                                        const bf16_t* __restrict__ typ, bf16_t* __restrict__ out,
                                                        long T, int S, int H) {
  const int nv = H >> 3;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long t = gid / nv;
  if (t >= T) return;
  const int c = (int)(gid - t * nv) * 8;
  float a[8], b[8], d[8];
  unpack8(*reinterpret_cast<const uint4*>(word + ids[t] * H + c), a);
  unpack8(*reinterpret_cast<const uint4*>(pos + (t % S) * H + c), b);
  unpack8(*reinterpret_cast<const uint4*>(typ + (types ? types[t] : 0) * H + c), d);
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] += b[e] + d[e];
  *reinterpret_cast<uint4*>(out + t * H + c) = pack8f(a);
}

__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ ids,
                                                        const int64_t* __restrict__ types,
                                                        const bf16_t* __restrict__ ds, float* __restrict__ gword,
                                                        float* __restrict__ gpos, float* __restrict__ wsT, int ntypes,
                                                        long T, int S, int H) {
  // one wave per token (strided); lane owns columns 8*(lane + 64u)..+7
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int nv = H >> 3;
  float acc[2][4][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[a][u][e] = 0.f;
  // four of the wave's tokens per trip: their row loads are issued together, then accumulated in token
  // order (the same sums as one token at a time)
  constexpr int TU = 4;
  for (long t0 = wave; t0 < T; t0 += (long)TU * nwaves) {
    uint4 raw[TU][4];
    long id[TU];
    int ty[TU];
#pragma unroll
    for (int j = 0; j < TU; ++j) {
      const long t = t0 + (long)j * nwaves;
      const bool ok = t < T;
      id[j] = ok ? ids[t] : 0;
      ty[j] = ok && types ? (int)types[t] : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = lane + 64 * u;
        if (ok && c < nv) raw[j][u] = *reinterpret_cast<const uint4*>(ds + t * H + c * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < TU; ++j) {
      const long t = t0 + (long)j * nwaves;
      if (t >= T) break;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = lane + 64 * u;
        if (c < nv) {
          float d[8];
          unpack8(raw[j][u], d);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            if (gword) atomicAdd(gword + id[j] * H + c * 8 + e, d[e]);
            if (gpos) atomicAdd(gpos + (t % S) * H + c * 8 + e, d[e]);
            if (ty[j] == 0) acc[0][u][e] += d[e];
            else acc[1][u][e] += d[e];
          }
        }
      }
    }
  }
  if (wsT) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      if (a >= ntypes) break;
      float* w0 = wsT + ((long)wave * ntypes + a) * H;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = lane + 64 * u;
        if (c < nv)
#pragma unroll
          for (int e = 0; e < 8; ++e) w0[c * 8 + e] = acc[a][u][e];
      }
    }
  }
}

// word-embedding gradient from tokens sorted by id: wave w sums the rows of sorted positions
// [32w, 32w + 32), flushing one partial sum per run of equal ids.  A run that lies entirely
// inside the chunk has a single writer (plain read-modify-write); a run crossing a chunk edge
// (a frequent id such as [MASK]) is flushed with fp32 atomics, one per chunk.
constexpr int kEmbChunk = 32;
__global__ __launch_bounds__(256) void embed_word_grad_kernel(const int64_t* __restrict__ sorted_ids,
                                                             const int64_t* __restrict__ perm,
                                                             const bf16_t* __restrict__ ds, float* __restrict__ gword,
                                                             long T, int H) {
  const long c0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * kEmbChunk;
  const int lane = threadIdx.x & 63;
  if (c0 >= T) return;
  const long c1 = min(T, c0 + kEmbChunk);
  const bool head_shared = c0 > 0 && sorted_ids[c0 - 1] == sorted_ids[c0];
  const bool tail_shared = c1 < T && sorted_ids[c1] == sorted_ids[c1 - 1];
  for (int c = lane * 8; c < H; c += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    long run_start = c0;
    int64_t id = sorted_ids[c0];
    for (long j = c0; j < c1; ++j) {
      float d[8];
      unpack8(*reinterpret_cast<const uint4*>(ds + perm[j] * H + c), d);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += d[e];
      const bool last = j + 1 == c1 || sorted_ids[j + 1] != id;
      if (last) {
        float* g = gword + id * H + c;
        const bool shared = (run_start == c0 && head_shared) || (j + 1 == c1 && tail_shared);
        if (shared) {
#pragma unroll
          for (int e = 0; e < 8; ++e) atomicAdd(g + e, acc[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] += acc[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = 0.f;
        if (j + 1 < c1) {
          run_start = j + 1;
          id = sorted_ids[j + 1];
        }
      }
    }
  }
}

// Deterministic word-embedding gradient over the (stable) sorted ids, two passes with a fixed partition:
// pass 1 — one wave per 64-position chunk of the sorted array sums each same-id segment of its chunk in
// position order; a run that starts and ends inside the chunk is written to gword by that wave (its
// only writer), a run crossing a chunk boundary leaves its segment sums in `part` (the chunk's first
// segment when it continues a run, its last segment when it starts one);
// pass 2 — the wave of the chunk where a crossing run starts adds its segments chunk by chunk, in order,
// and writes the row once.  No atomics, the same bits on every run, and a frequent id ([MASK]: 15 % of
// the tokens) costs its owner one row add per chunk instead of a serial walk over all its tokens.
constexpr int kDetChunk = 64;
__device__ __forceinline__ void emb_seg_sum(const int64_t* perm, const bf16_t* ds, int H, long j0, long j1, int c,
                                            float (&acc)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (long j = j0; j < j1; ++j) {
    float d[8];
    unpack8(*reinterpret_cast<const uint4*>(ds + perm[j] * H + c), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += d[e];
  }
}

__global__ __launch_bounds__(256) void embed_word_grad_det_kernel(const int64_t* __restrict__ sorted_ids,
                                                                 const int64_t* __restrict__ perm,
                                                                 const bf16_t* __restrict__ ds,
                                                                 float* __restrict__ gword, float* __restrict__ part,
                                                                 long T, int H, long V) {
  const long ch = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long c0 = ch * kDetChunk;
  const int lane = threadIdx.x & 63;
  if (c0 >= T) return;
  const long c1 = min(T, c0 + kDetChunk);
  float* first = part + (2 * ch) * (long)H;  // segment continuing a run from the previous chunk
  float* last = first + H;                   // segment starting a run that continues into the next chunk
  long j0 = c0;
  while (j0 < c1) {
    const int64_t id = sorted_ids[j0];
    long j1 = j0 + 1;
    while (j1 < c1 && sorted_ids[j1] == id) ++j1;
    const bool starts = j0 == 0 || sorted_ids[j0 - 1] != id;
    const bool ends = j1 == T || sorted_ids[j1] != id;
    if ((uint64_t)id < (uint64_t)V) {
      for (int c = lane * 8; c < H; c += 512) {
        float acc[8];
        emb_seg_sum(perm, ds, H, j0, j1, c, acc);
        float* dst = starts && ends ? gword + id * H + c : (starts ? last + c : first + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = starts && ends ? dst[e] + acc[e] : acc[e];
      }
    }
    j0 = j1;
  }
}

__global__ __launch_bounds__(256) void embed_word_grad_det_join_kernel(const int64_t* __restrict__ sorted_ids,
                                                                      float* __restrict__ gword,
                                                                      const float* __restrict__ part, long T, int H,
                                                                      long V) {
  const long ch = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const long c0 = ch * kDetChunk;
  const int lane = threadIdx.x & 63;
  if (c0 >= T) return;
  const long e = min(T, c0 + kDetChunk) - 1;  // the chunk's last position
  const int64_t id = sorted_ids[e];
  if (e + 1 >= T || sorted_ids[e + 1] != id) return;  // its last run ends inside the chunk
  long s = e;
  while (s > c0 && sorted_ids[s - 1] == id) --s;
  if (s == c0 && c0 > 0 && sorted_ids[c0 - 1] == id) return;  // the run started in an earlier chunk
  if ((uint64_t)id >= (uint64_t)V) return;
  const long nch = (T + kDetChunk - 1) / kDetChunk;
  for (int c = lane * 8; c < H; c += 512) {
    float acc[8];
    const float* l = part + (2 * ch + 1) * (long)H + c;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = l[k];
    for (long q = ch + 1; q < nch; ++q) {  // the continuing segments, chunk by chunk
      const float* f = part + (2 * q) * (long)H + c;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += f[k];
      const long qe = min(T, (q + 1) * kDetChunk);
      if (qe >= T || sorted_ids[qe] != id) break;  // the run ends in chunk q
    }
    float* g = gword + id * H + c;
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] += acc[k];
  }
}

// word-embedding gradient without a sort: gword[ids[t]][h] += ds[t][h] as no-return fp32 atomics
// (executed at the memory side, ~1.3 TB/s of added bytes on MI355X: 16384 x 768 tokens x columns in
// ~40 us, vs ~105 us for the sorted one-writer walk, which also needed a radix sort of the ids).
// Lane i of a wave adds columns 2i, 2i+1 of one token row per step (one 4-B load of a bf16 pair).
__global__ __launch_bounds__(256) void embed_word_grad_atomic_kernel(const int64_t* __restrict__ ids,
                                                                    const uint32_t* __restrict__ ds,
                                                                    float* __restrict__ gword, long T, int H,
                                                                    long V) {
  const int HP = H >> 1;  // bf16 pairs per row
  const long n = T * HP;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long t = i / HP;
    const int c = (int)(i - t * HP) * 2;
    const int64_t id = ids[t];
    if ((uint64_t)id >= (uint64_t)V) continue;  // an out-of-vocabulary id adds nothing (never a wild write)
    const uint32_t w = ds[i];
    float* g = gword + id * H + c;
    atomicAdd(g, __uint_as_float(w << 16));
    atomicAdd(g + 1, __uint_as_float(w & 0xffff0000u));
  }
}

// position-embedding gradient: gpos[s][h] += sum_b ds[b*S + s][h]  (column sums, no atomics)
__global__ __launch_bounds__(256) void embed_pos_grad_kernel(const bf16_t* __restrict__ ds, float* __restrict__ gpos,
                                                            int B, int S, int H) {
  const long col = (long)blockIdx.x * 256 + threadIdx.x;  // over S*H/2 bf16 pairs
  if (col * 2 >= (long)S * H) return;
  float a = 0.f, b = 0.f;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(ds) + col;
  const long stride = (long)S * H / 2;
  // 8 rows' loads in flight per lane, then summed in row order (the same sums as one row at a time)
  int r = 0;
  for (; r + 8 <= B; r += 8) {
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = p[(r + k) * stride];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a += __uint_as_float(w[k] << 16);
      b += __uint_as_float(w[k] & 0xffff0000u);
    }
  }
  for (; r < B; ++r) {
    const uint32_t w = p[r * stride];
    a += __uint_as_float(w << 16);
    b += __uint_as_float(w & 0xffff0000u);
  }
  gpos[col * 2] += a;
  gpos[col * 2 + 1] += b;
}

// BERT MLM head input: the hidden rows of the masked positions.  Row r = b P + i of out is row b S + pos[b][i] of
// h (positions outside [0, S) give a zero row), computed in-kernel from the [B][P] positions (no arange / add /
// index_select launches).  One wave per row, 16-B vectors.
__global__ __launch_bounds__(256) void mlm_gather_kernel(const bf16_t* __restrict__ h, const int64_t* __restrict__ pos,
                                                         bf16_t* __restrict__ out, int B, int S, int P, int H) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= (long)B * P) return;
  const long b = r / P;
  const int64_t q = pos[r];
  const bool ok = q >= 0 && q < S;
  const uint4* src = reinterpret_cast<const uint4*>(h + (b * S + (ok ? q : 0)) * (long)H);
  uint4* dst = reinterpret_cast<uint4*>(out + r * (long)H);
  for (int v = lane; v < (H >> 3); v += 64) dst[v] = ok ? src[v] : make_uint4(0u, 0u, 0u, 0u);
}

// Its backward: dh[t] = sum of dout[b P + i] over the i with pos[b][i] == t - b S (b = t / S), in increasing i
// (duplicated padding positions sum in a fixed order: deterministic, no atomics), zero elsewhere — ONE pass that
// writes every row of dh (no zero fill + index_add).  One wave per row t: the wave ballots its sequence's P
// positions 64 at a time.
__global__ __launch_bounds__(256) void mlm_scatter_kernel(const bf16_t* __restrict__ dout,
                                                          const int64_t* __restrict__ pos, bf16_t* __restrict__ dh,
                                                          int B, int S, int P, int H) {
  const int lane = threadIdx.x & 63;
  const long t = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= (long)B * S) return;
  const long b = t / S;
  const int64_t q = t - b * S;
  const int nv = H >> 3;
  constexpr int VMAX = 4;  // H <= 2048
  float acc[VMAX][8];
#pragma unroll
  for (int u = 0; u < VMAX; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[u][e] = 0.f;
  for (int i0 = 0; i0 < P; i0 += 64) {
    const int i = i0 + lane;
    unsigned long long m = __ballot(i < P && pos[b * P + i] == q);
    while (m) {
      const int k = __ffsll((long long)m) - 1;
      m &= m - 1;
      const uint4* src = reinterpret_cast<const uint4*>(dout + (b * P + i0 + k) * (long)H);
#pragma unroll
      for (int u = 0; u < VMAX; ++u) {
        const int v = lane + 64 * u;
        if (v < nv) {
          float f[8];
          unpack8(src[v], f);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[u][e] += f[e];
        }
      }
    }
  }
  uint4* dst = reinterpret_cast<uint4*>(dh + t * (long)H);
#pragma unroll
  for (int u = 0; u < VMAX; ++u) {
    const int v = lane + 64 * u;
    if (v < nv) dst[v] = pack8f(acc[u]);
  }
}

constexpr int kLnBwdBlocks = 512;  // 2 waves/SIMD: LN bwd 48 -> 37 us per BERT call (256: 1 wave/SIMD, latency-bound)

}  // namespace

int mlm_gather(const void* h, const int64_t* pos, void* out, int B, int S, int P, int H, hipStream_t s) {
  if (H % 8 || H > 2048) return (int)hipErrorInvalidValue;
  const long rows = (long)B * P;
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(mlm_gather_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s,
                     reinterpret_cast<const bf16_t*>(h), pos, reinterpret_cast<bf16_t*>(out), B, S, P, H);
  return (int)hipGetLastError();
}

int mlm_scatter(const void* dout, const int64_t* pos, void* dh, int B, int S, int P, int H, hipStream_t s) {
  if (H % 8 || H > 2048) return (int)hipErrorInvalidValue;
  const long rows = (long)B * S;
  if (rows <= 0) return 0;
  hipLaunchKernelGGL(mlm_scatter_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s,
                     reinterpret_cast<const bf16_t*>(dout), pos, reinterpret_cast<bf16_t*>(dh), B, S, P, H);
  return (int)hipGetLastError();
}

int layernorm_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, long M,
                  int H, float eps, float drop_p, unsigned long long seed, hipStream_t s) {
  if (M <= 0) return 0;
  const uint32_t th = drop_t8(drop_p);
  const float ds = drop_scale8(th);
  const int nv = H / 8;
  // grid-stride: gamma / beta loaded once per wave
  const dim3 grid((unsigned)std::min<long>((M + 3) / 4, 2048L));
  auto X = reinterpret_cast<const bf16_t*>(x);
  auto Y = reinterpret_cast<bf16_t*>(y);
  if (nv <= 64) hipLaunchKernelGGL((ln_fwd_kernel<1, true>), grid, dim3(256), 0, s, X, gamma, beta, Y, mean, rstd, M, H, eps, th, ds, seed);
  else if (nv <= 128) hipLaunchKernelGGL((ln_fwd_kernel<2, true>), grid, dim3(256), 0, s, X, gamma, beta, Y, mean, rstd, M, H, eps, th, ds, seed);
  else if (nv <= 256) hipLaunchKernelGGL((ln_fwd_kernel<4, true>), grid, dim3(256), 0, s, X, gamma, beta, Y, mean, rstd, M, H, eps, th, ds, seed);
  else hipLaunchKernelGGL((ln_fwd_kernel<8, false>), grid, dim3(256), 0, s, X, gamma, beta, Y, mean, rstd, M, H, eps, th, ds, seed);
  return (int)hipGetLastError();
}

constexpr int kLnBwdBlocksBR = 1024;  // block-reduced form: 4,096 waves (4 per SIMD), one partial row per workgroup

// partial rows [P][parts][H] layernorm_bwd writes for M rows of width H
int ln_bwd_rows(long M, int H) {
  // H = 768 (ln_bwd_q_kernel, 148 VGPRs: 3 waves per SIMD): one round of 768 workgroups — LN backward + its column
  // sum 27.1 -> 24.9 us per BERT call vs 1,024 (512: 24.8, 1,536: 28.4; profiles/r6/ln_blocks.txt)
  if (H / 8 == 96) return (int)std::max<long>(1, std::min<long>(768L, (M + 3) / 4));
  if (H / 8 <= 128) return (int)std::max<long>(1, std::min<long>((long)kLnBwdBlocksBR, (M + 3) / 4));
  return ln_partial_rows(M);
}

int ln_partial_rows(long M) {
  // workgroups of the row-per-wave backward sweeps (4 waves each); also sizes embed_bwd's grid and its
  // token-type partial-row workspace, which share this partial-row count
  const long blocks = std::min<long>((long)kLnBwdBlocks, (M + 3) / 4);
  return (int)std::max<long>(1, blocks) * 4;
}

int layernorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const float* gamma, void* dx,
                  void* dx_drop, float drop_p, unsigned long long seed, float* ws, int P, long M, int H,
                  float in_drop_p, unsigned long long in_seed, int parts, hipStream_t s) {
  if (M <= 0) return 0;
  const uint32_t ith = drop_t8(in_drop_p);
  const float iscale = drop_scale8(ith);
  const int nv = H / 8;
  if (P != ln_bwd_rows(M, H)) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)(nv <= 128 ? P : P / 4));
  const uint32_t thresh = drop_t8(drop_p);
  const float dscale = drop_scale8(thresh);
  auto DY = reinterpret_cast<const bf16_t*>(dy);
  auto X = reinterpret_cast<const bf16_t*>(x);
  auto DX = reinterpret_cast<bf16_t*>(dx);
  auto DD = reinterpret_cast<bf16_t*>(dx_drop);
  // BERT-base: 8-B vectors, three per lane, every lane busy (ln_bwd_q_kernel): 30.3 -> 21.1 us per call,
  // BERT-base 900-902K -> 916-919K tok/s (profiles/r6/ab_ln_bwd.txt)
  if (nv == 96)
    hipLaunchKernelGGL((ln_bwd_q_kernel<3>), grid, dim3(256), 0, s, DY, X, mean, rstd, gamma, DX, DD, thresh, dscale, seed, ws, M, H, ith, iscale, in_seed, parts);
  else if (nv <= 64) hipLaunchKernelGGL((ln_bwd_kernel<1, true, true>), grid, dim3(256), 0, s, DY, X, mean, rstd, gamma, DX, DD, thresh, dscale, seed, ws, M, H, ith, iscale, in_seed, parts);
  else if (nv <= 128) hipLaunchKernelGGL((ln_bwd_kernel<2, true, true>), grid, dim3(256), 0, s, DY, X, mean, rstd, gamma, DX, DD, thresh, dscale, seed, ws, M, H, ith, iscale, in_seed, parts);
  else if (nv <= 256) hipLaunchKernelGGL((ln_bwd_kernel<4, false>), grid, dim3(256), 0, s, DY, X, mean, rstd, gamma, DX, DD, thresh, dscale, seed, ws, M, H, ith, iscale, in_seed, parts);
  else hipLaunchKernelGGL((ln_bwd_kernel<8, false>), grid, dim3(256), 0, s, DY, X, mean, rstd, gamma, DX, DD, thresh, dscale, seed, ws, M, H, ith, iscale, in_seed, parts);
  return (int)hipGetLastError();
}

int colsum_partials(const float* ws, int P, int N, float* out, int accumulate, hipStream_t s, long ld) {
  if (N <= 0) return 0;
  if (!accumulate) {
    const hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)N, s);
    if (e != hipSuccess) return (int)e;
  }
  // deterministic mode: one writer per column, partial rows summed in a fixed order
  if (deterministic()) {
    hipLaunchKernelGGL(colsum_det_kernel, dim3((N + 15) / 16), dim3(1024), 0, s, ws, P, N, ld > 0 ? ld : (long)N, out);
    return (int)hipGetLastError();
  }
  const long ldv = ld > 0 ? ld : (long)N;
  if (N % 4 == 0 && ldv % 4 == 0 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0) {
    hipLaunchKernelGGL(colsum_vec_kernel, dim3((N + 255) / 256, (P + kColsumVecRows - 1) / kColsumVecRows), dim3(256), 0,
                       s, ws, P, N, ldv, out);
    return (int)hipGetLastError();
  }
  const int chunk = kColsumRows;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64, (P + chunk - 1) / chunk), dim3(64, 16), 0, s, ws, P, N,
                     ld > 0 ? ld : (long)N, out, chunk);
  return (int)hipGetLastError();
}

int embed_fwd(const int64_t* ids, const int64_t* types, const void* word, const void* pos, const void* type,
              void* out, long T, int S, int H, hipStream_t s) {
  if (T <= 0) return 0;
  const long n = T * (H / 8);
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ids, types,
                     reinterpret_cast<const bf16_t*>(word), reinterpret_cast<const bf16_t*>(pos),
                     reinterpret_cast<const bf16_t*>(type), reinterpret_cast<bf16_t*>(out), T, S, H);
  return (int)hipGetLastError();
}

int embed_word_grad(const int64_t* sorted_ids, const int64_t* perm, const void* ds, float* gword, long T, int H,
                    hipStream_t s) {
  if (T <= 0) return 0;
  const long waves = (T + kEmbChunk - 1) / kEmbChunk;
  hipLaunchKernelGGL(embed_word_grad_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, sorted_ids, perm,
                     reinterpret_cast<const bf16_t*>(ds), gword, T, H);
  return (int)hipGetLastError();
}

int embed_word_grad_det(const int64_t* sorted_ids, const int64_t* perm, const void* ds, float* gword, long T, int H,
                        long V, float* part, hipStream_t s) {
  if (T <= 0) return 0;
  if (H % 8) return (int)hipErrorInvalidValue;
  const long waves = (T + kDetChunk - 1) / kDetChunk;
  hipLaunchKernelGGL(embed_word_grad_det_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, sorted_ids, perm,
                     reinterpret_cast<const bf16_t*>(ds), gword, part, T, H, V);
  hipLaunchKernelGGL(embed_word_grad_det_join_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, sorted_ids,
                     gword, part, T, H, V);
  return (int)hipGetLastError();
}
long embed_word_grad_det_ws(long T, int H) { return 2 * ((T + kDetChunk - 1) / kDetChunk) * (long)H; }

int embed_word_grad_atomic(const int64_t* ids, const void* ds, float* gword, long T, int H, long V, hipStream_t s) {
  if (T <= 0) return 0;
  const long n = T * (H / 2);
  const long blocks = std::min<long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(embed_word_grad_atomic_kernel, dim3((unsigned)blocks), dim3(256), 0, s, ids,
                     reinterpret_cast<const uint32_t*>(ds), gword, T, H, V);
  return (int)hipGetLastError();
}

int embed_pos_grad(const void* ds, float* gpos, int B, int S, int H, hipStream_t s) {
  const long n = (long)S * H / 2;
  hipLaunchKernelGGL(embed_pos_grad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const bf16_t*>(ds), gpos, B, S, H);
  return (int)hipGetLastError();
}

int embed_bwd(const int64_t* ids, const int64_t* types, const void* ds, float* gword, float* gpos, float* wsT, int P,
              int ntypes, long T, int S, int H, hipStream_t s) {
  if (T <= 0) return 0;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((unsigned)(P / 4)), dim3(256), 0, s, ids, types,
                     reinterpret_cast<const bf16_t*>(ds), gword, gpos, wsT, ntypes, T, S, H);
  return (int)hipGetLastError();
}

}  // namespace ddl
