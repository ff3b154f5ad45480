// Fused multi-head attention (forward + backward) for gfx950, head dim 64.
//
// Layout: the QKV projection output is consumed in place, [tokens, ld] row-major with
// head h of Q/K/V at columns q_off/k_off/v_off + 64h (BERT: ld = 3*768); the context
// output is [tokens, ldo] with head h at columns 64h — i.e. directly the input of the
// output projection.  No transposes, no materialised score matrix.
//
// Every product runs on v_mfma_f32_16x16x32_bf16.  The trick that keeps the softmax
// in registers: scores are computed TRANSPOSED, S^T = K Q^T, so that one lane owns one
// query (column lane&15 of the D fragment) across 4 keys per 16x16 tile.  Row
// statistics (max, sum) are then in-lane + two xor-shuffles, and P^T is already laid out
// as the B operand of O^T = V^T P^T once the 32 keys of an MFMA k-step are enumerated in
// the order the lane holds them (keys 4g..4g+3 and 16+4g..16+4g+3 of the step).  The V^T
// A-operand is produced in that same key order by ds_read_b64_tr_b16 (hardware transpose
// reads) from a row-major, XOR-swizzled 64x64 LDS tile.  The backward uses the same two
// fragment readers:
//   attn_bwd_dkdv : a workgroup owns 128 keys (32 per wave), streams 64-query tiles of
//                   Q/dO through LDS: S = Q K^T, dP = dO V^T, dV += P^T dO, dK += dS^T Q;
//   attn_bwd_dq   : a workgroup owns 128 queries, streams K/V tiles: dQ += dS K.
// (Two kernels instead of atomics on dQ: deterministic, no fp32 scratch.)  dQ runs first and
// also computes D = rowsum(dO * O) for its queries (it holds their dO already) into the
// scratch dvec that dK/dV reads — no separate elementwise pass over O and dO.
// Softmax uses base-2 exponentials with scale*log2(e) folded in; the forward saves the
// base-2 log-sum-exp per query.  Dropout on the attention probabilities is a stateless
// hash of (seed, b, h, i, j), regenerated in the backward.  Key padding: lens[b] valid
// keys (nullable -> all valid).
#include <stdlib.h>

#include <type_traits>

#include "ddl_common.h"
#include "ddl_ops.h"

namespace ddl {
namespace {

constexpr int HD = 64;            // head dim
constexpr int TQ = 64;            // rows of a streamed LDS tile
constexpr int TILE_BYTES = TQ * HD * 2;
constexpr int THREADS = 256;      // 4 waves, each owns 32 rows (queries or keys)
constexpr int BLOCK_ROWS = 128;

__device__ __forceinline__ int tile_byte(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }

// LDS-DMA of a 64x64 bf16 tile (rows r0.. of `base`, row stride ld) into the swizzled image:
// wave w's two 1-KB instructions fill linear 16-B slots v*256 + 64w + lane, i.e. tile row
// slot>>3, physical chunk slot&7 -> the lane fetches logical chunk (slot&7) ^ ((row>>1)&7).
// Rows at or past nrows read the zero page.  No staging registers; the caller waits
// vmcnt(0) + barrier before the tile is read.
__device__ __forceinline__ void dma_tile(const bf16_t* base, long ld, int r0, int nrows, char* lds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t lb = lds_addr(lds) + (uint32_t)__builtin_amdgcn_readfirstlane(w) * 1024u;
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    const int idx = v * THREADS + w * 64 + lane;
    const int row = idx >> 3, ch = (idx & 7) ^ ((row >> 1) & 7);
    const void* src = (r0 + row < nrows) ? (const void*)(base + (long)(r0 + row) * ld + ch * 8)
                                         : (const void*)ddl_zero_page;
    dma16(src, lb + (uint32_t)(v * THREADS * 16));
  }
}

// 8 consecutive elements of tile row `row` at columns 32kk + 8g (fragment whose k runs along the row)
__device__ __forceinline__ bf16x8 frag_row(const char* lds, int row, int kk, int g) {
  return *reinterpret_cast<const bf16x8*>(lds + tile_byte(row, 4 * kk + g));
}

// fragment whose k runs DOWN the tile: lane (g, li) gets column cb+li of rows ra..ra+3 (slots 0-3)
// and rb..rb+3 (slots 4-7); ra/rb are uniform per 16-lane group.
__device__ __forceinline__ bf16x8 frag_col(const char* lds, int ra, int rb, int cb, int lane) {
  const int li = lane & 15, q = li >> 2, pp = li & 3;
  const int col = cb + 4 * pp;
  const int ch = col >> 3, within = (col & 7) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(lds + tile_byte(ra + q, ch) + within));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DDL_LDS s16x4*)(lds + tile_byte(rb + q, ch) + within));
  const s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

__device__ __forceinline__ bf16x8 ldg_frag(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// Attention-probability dropout, rate quantised to 1/256 (uint8 thresholds): key j of query row r
// is kept iff byte (j & 3) of hash24(row_key(r) + j / 4) is >= t8, and the kept probabilities are
// scaled by 256 / (256 - t8).  One 32-bit hash serves four consecutive keys, and hash24 mixes with
// 24-bit multiplies (v_mul_u32_u24, full rate) where a 32-bit mix costs two quarter-rate
// v_mul_lo_u32; the per-row key keeps the full 32-bit mix (computed once per row).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t row_key(unsigned long long seed, int bh, int S, int i) {
  return mix32((uint32_t)seed ^ mix32((uint32_t)(bh * S + i) + (uint32_t)(seed >> 32)));
}
__device__ __forceinline__ uint32_t hash24(uint32_t x) {
  x ^= x >> 16;
  x = __umul24(x, 0x7feb35u);
  x ^= x >> 15;
  x = __umul24(x, 0x846ca7u);
  return x ^ (x >> 16);
}
__device__ __forceinline__ bool keep_byte(uint32_t h, int e, uint32_t t8) { return ((h >> (8 * e)) & 0xffu) >= t8; }
// value of lane (lane & ~3) + E within each quad of lanes (DPP quad_perm [E,E,E,E])
template <int E>
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, E * 0x55, 0xf, 0xf, false);
}
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Block -> (query/key block, head, sequence).  With xcd_remap the linear block id goes through the
// XCD-aware bijection first, so the S / 128 blocks of one (b, h) — which all stream the same K / V (or
// Q / dO) tiles — are dealt to ONE XCD and share its L2; in grid order they land on S / 128 different XCDs.
__device__ __forceinline__ void attn_block(const AttnParams& p, int& xb, int& h, int& b) {
  if (p.xcd_remap) {
    const int nx = gridDim.x, ny = gridDim.y;
    const int lin = xcd_remap(blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), nx * ny * gridDim.z);
    xb = lin % nx;
    const int t = lin / nx;
    h = t % ny;
    b = t / ny;
  } else {
    xb = blockIdx.x;
    h = blockIdx.y;
    b = blockIdx.z;
  }
}

// ================================================================ forward
// Lazy rescaling: the running maximum m that a row's exponentials are taken against only moves when
// a tile's scores exceed it by more than TAU (log2 units), so P = exp2(s*scale - m) <= 2^TAU (bf16
// keeps its relative precision; O and l accumulate in fp32).  The common tile therefore needs no
// cross-lane maximum (each lane tests its own 16 scores of the row against m) and no rescale of O
// (64 packed multiplies per tile beside the MFMAs); the wave-uniform branch into the rescale is
// taken on the first tile and rarely after.  Full tiles and the last partial tile (key padding) are
// separate instantiations of the tile body, dropout is a template parameter: no branches inside it.
constexpr float TAU = 8.f;

template <int MINB, bool DROP>
__global__ __launch_bounds__(THREADS, MINB) void attn_fwd_kernel(const AttnParams p) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][TILE_BYTES];
  int xb, h, b;
  attn_block(p, xb, h, b);
  const int S = p.S;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const long tok0 = (long)b * S;
  const bf16_t* Q = p.qkv + tok0 * p.ld + p.q_off + h * HD;
  const bf16_t* K = p.qkv + tok0 * p.ld + p.k_off + h * HD;
  const bf16_t* V = p.qkv + tok0 * p.ld + p.v_off + h * HD;
  const int len = p.lens ? min(max(p.lens[b], 0), S) : S;
  const int q0 = xb * BLOCK_ROWS + w * 32;
  const int bh = b * p.H + h;
  const float sl = p.scale_log2;

  bf16x8 qf[2][2];
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[it][kk] = ldg_frag(Q + (long)(q0 + 16 * it + li) * p.ld + 32 * kk + 8 * g);

  f32x4 o[4][2];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int it = 0; it < 2; ++it) o[dt][it] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  uint32_t hk[2] = {0u, 0u};  // dropout: row key + the lane's key group (keys 4g..4g+3 of every 16)
  if constexpr (DROP) {
#pragma unroll
    for (int it = 0; it < 2; ++it) hk[it] = row_key(p.drop_seed, bh, S, q0 + 16 * it + li) + (uint32_t)g;
  }
  const uint32_t t8 = p.drop_t8;

  // one 64-key tile: S^T[j = kb + 16jt + 4g + e][i = 16it + li] for all four 16-key groups jt, then
  // P^T and O^T[d][i] += sum_j V^T[d][j] P^T[j][i] per 32-key MFMA step kk (jt = 2kk, 2kk + 1)
  auto tile = [&](const char* kl, const char* vl, const int kb, auto masked) {
    constexpr bool MASK = decltype(masked)::value;
    f32x4 s[4][2];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const bf16x8 k0 = frag_row(kl, 16 * jt + li, 0, g), k1 = frag_row(kl, 16 * jt + li, 1, g);
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
        a = mfma16x16x32(k0, qf[it][0], a);
        s[jt][it] = mfma16x16x32(k1, qf[it][1], a);
      }
    }
    if constexpr (MASK) {
#pragma unroll
      for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (kb + 16 * jt + 4 * g + e >= len) s[jt][it][e] = -INFINITY;
    }
    float lmx[2];
    bool need = false;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      float mx = s[0][it][0];
#pragma unroll
      for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, s[jt][it][e]);
      lmx[it] = mx;
      need = need || (mx * sl > m[it] + TAU);
    }
    if (__any(need)) {  // wave-uniform: move the maximum of every row of the wave, rescale O and l
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        float mx = lmx[it];
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mn = fmaxf(m[it], mx * sl);
        const float alpha = m[it] == -INFINITY ? 0.f : fexp2(m[it] - mn);
        m[it] = mn;
        l[it] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt][it] *= alpha;
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        float rs = 0.f;
#pragma unroll
        for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = fexp2(fmaf(s[2 * kk + j2][it][e], sl, -m[it]));
            s[2 * kk + j2][it][e] = pv;
            rs += pv;
          }
        l[it] += rs;  // the softmax denominator sums the probabilities before dropout
      }
      if constexpr (DROP) {
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int j2 = 0; j2 < 2; ++j2) {
            const uint32_t hh = hash24(hk[it] + (uint32_t)((kb >> 2) + 8 * kk + 4 * j2));
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (!keep_byte(hh, e, t8)) s[2 * kk + j2][it][e] = 0.f;
          }
      }
      const bf16x8 pb0 = pack8(s[2 * kk][0], s[2 * kk + 1][0]);
      const bf16x8 pb1 = pack8(s[2 * kk][1], s[2 * kk + 1][1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 va = frag_col(vl, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * dt, lane);
        o[dt][0] = mfma16x16x32(va, pb0, o[dt][0]);
        o[dt][1] = mfma16x16x32(va, pb1, o[dt][1]);
      }
    }
  };

  const int nkt = (len + TQ - 1) / TQ, nfull = len / TQ;
  if (nkt > 0) {
    dma_tile(K, p.ld, 0, len, lds[0][0]);
    dma_tile(V, p.ld, 0, len, lds[0][1]);
  }
  wait_vmcnt<0>();
  __syncthreads();
  // full tiles in one loop (one instantiation: no register copies at the back edge), then the
  // partial tile of a padded sequence
  for (int t = 0; t < nfull; ++t) {
    if (t + 1 < nkt) {
      dma_tile(K, p.ld, (t + 1) * TQ, len, lds[(t + 1) & 1][0]);
      dma_tile(V, p.ld, (t + 1) * TQ, len, lds[(t + 1) & 1][1]);
    }
    tile(lds[t & 1][0], lds[t & 1][1], t * TQ, std::false_type{});
    wait_vmcnt<0>();
    __syncthreads();
  }
  if (nfull < nkt) tile(lds[nfull & 1][0], lds[nfull & 1][1], nfull * TQ, std::true_type{});
  const float num = DROP ? p.drop_scale : 1.f;  // the dropout scale folds into the normalisation
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    float lt = l[it];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const float inv = lt > 0.f ? num / lt : 0.f;
    const int i = q0 + 16 * it + li;
    bf16_t* orow = p.o + (tok0 + i) * p.ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f32x4 v = o[dt][it] * inv;
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
    if (g == 0) p.lse[(long)bh * S + i] = lt > 0.f ? m[it] + __log2f(lt) : INFINITY;
  }
}

// ================================================================ backward: dK, dV
// MINB = resident blocks per CU the register allocation is capped for: 1 (no spills) or 2 (twice the
// waves to hide latency); picked at launch by DDL_ATTN_DKDV_OCC (default 2).  Dropout is a template
// parameter; key padding is a second instantiation of the q-tile loop, chosen per workgroup (only
// workgroups whose 128 keys straddle the padding pay for the mask).  A lane holds P[i][j] for four
// consecutive queries i of one key j, and the dropout bytes of a (query, 4-key group) come from one
// hash: lane r of each quad hashes query row r, the quad shares the four hashes by DPP broadcast.
template <int MINB, bool DROP>
__global__ __launch_bounds__(THREADS, MINB) void attn_bwd_dkdv_kernel(const AttnParams p) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][TILE_BYTES];  // [buf][Q, dO]
  __shared__ __attribute__((aligned(16))) float s_lse[2][TQ];
  __shared__ __attribute__((aligned(16))) float s_d[2][TQ];
  __shared__ __attribute__((aligned(16))) uint32_t s_rk[2][TQ];
  int xb, h, b;
  attn_block(p, xb, h, b);
  const int S = p.S;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const long tok0 = (long)b * S;
  const int bh = b * p.H + h;
  const bf16_t* Q = p.qkv + tok0 * p.ld + p.q_off + h * HD;
  const bf16_t* K = p.qkv + tok0 * p.ld + p.k_off + h * HD;
  const bf16_t* V = p.qkv + tok0 * p.ld + p.v_off + h * HD;
  const bf16_t* dO = p.dout + tok0 * p.lddo + h * HD;
  const float* lse = p.lse + (long)bh * S;
  const float* dv = p.dvec + (long)bh * S;
  const int len = p.lens ? min(max(p.lens[b], 0), S) : S;
  const int k0 = xb * BLOCK_ROWS + w * 32;
  bf16_t* dK = p.dqkv + tok0 * p.lddqkv + p.k_off + h * HD;
  bf16_t* dV = p.dqkv + tok0 * p.lddqkv + p.v_off + h * HD;
  const float sl = p.scale_log2, dsc = p.drop_scale;
  const uint32_t t8 = p.drop_t8;

  // K / V fragments as the B operand of S = Q K^T and dP = dO V^T: [d][j = 16jt + li]
  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[jt][kk] = ldg_frag(K + (long)(k0 + 16 * jt + li) * p.ld + 32 * kk + 8 * g);
      vf[jt][kk] = ldg_frag(V + (long)(k0 + 16 * jt + li) * p.ld + 32 * kk + 8 * g);
    }
  // D layout accumulators: [j = 16jt + 4g + e][d = 16dt + li]
  f32x4 adv[2][4], adk[2][4];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) adv[jt][dt] = adk[jt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool any_key = xb * BLOCK_ROWS < len;  // block-uniform
  const int nqt = any_key ? S / TQ : 0;
  float r_lse = 0.f, r_d = 0.f;
  uint32_t r_rk = 0u;
  if (nqt > 0) {
    dma_tile(Q, p.ld, 0, S, lds[0][0]);
    dma_tile(dO, p.lddo, 0, S, lds[0][1]);
    if (threadIdx.x < TQ) {
      s_lse[0][threadIdx.x] = lse[threadIdx.x];
      s_d[0][threadIdx.x] = dv[threadIdx.x];
      if constexpr (DROP) s_rk[0][threadIdx.x] = row_key(p.drop_seed, bh, S, threadIdx.x);
    }
  }
  wait_vmcnt<0>();
  __syncthreads();

  auto qloop = [&](auto masked) {
    constexpr bool MASK = decltype(masked)::value;
    bool jok[2];  // key padding (MASK only): this lane's key of group jt is valid
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) jok[jt] = k0 + 16 * jt + li < len;
    for (int t = 0; t < nqt; ++t) {
      const int buf = t & 1;
      const char* ql = lds[buf][0];
      const char* dl = lds[buf][1];
      const bool more = t + 1 < nqt;
      if (more) {
        dma_tile(Q, p.ld, (t + 1) * TQ, S, lds[buf ^ 1][0]);
        dma_tile(dO, p.lddo, (t + 1) * TQ, S, lds[buf ^ 1][1]);
        if (threadIdx.x < TQ) {
          r_lse = lse[(t + 1) * TQ + threadIdx.x];
          r_d = dv[(t + 1) * TQ + threadIdx.x];
          if constexpr (DROP) r_rk = row_key(p.drop_seed, bh, S, (t + 1) * TQ + threadIdx.x);
        }
      }
      // The 64-query tile is processed as two 32-query halves: S / dP of one half (16 fp32 per
      // lane each) are consumed by the dV / dK MFMAs before the next half is formed.
#pragma unroll
      for (int kq = 0; kq < 2; ++kq) {
        // S, dP: [i = 32kq + 16i2 + 4g + e][j = 16jt + li]
        f32x4 s[2][2], dp[2][2];
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
          const int it = 2 * kq + i2;
          const bf16x8 q0f = frag_row(ql, 16 * it + li, 0, g), q1f = frag_row(ql, 16 * it + li, 1, g);
          const bf16x8 d0f = frag_row(dl, 16 * it + li, 0, g), d1f = frag_row(dl, 16 * it + li, 1, g);
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) {
            f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, c = f32x4{0.f, 0.f, 0.f, 0.f};
            a = mfma16x16x32(q0f, kf[jt][0], a);
            s[i2][jt] = mfma16x16x32(q1f, kf[jt][1], a);
            c = mfma16x16x32(d0f, vf[jt][0], c);
            dp[i2][jt] = mfma16x16x32(d1f, vf[jt][1], c);
          }
        }
        // P, dS (dropout-scaled P kept in s[] for dV); the lane's 4 query rows of a 16-row group
        // are consecutive, so their lse / D are one 16-B LDS read each
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
          const int il0 = 16 * (2 * kq + i2) + 4 * g;
          const f32x4 lq4 = *reinterpret_cast<const f32x4*>(&s_lse[buf][il0]);
          const f32x4 dq4 = *reinterpret_cast<const f32x4*>(&s_d[buf][il0]);
          uint32_t hq[2][4];  // [jt][e]: dropout hash of (query il0 + e, key group of j)
          if constexpr (DROP) {
            const uint32_t rkr = s_rk[buf][il0 + (li & 3)];
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) {
              const uint32_t hm = hash24(rkr + (uint32_t)((k0 + 16 * jt + li) >> 2));
              hq[jt][0] = quad_bcast<0>(hm);
              hq[jt][1] = quad_bcast<1>(hm);
              hq[jt][2] = quad_bcast<2>(hm);
              hq[jt][3] = quad_bcast<3>(hm);
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) {
              float pv = fexp2(fmaf(s[i2][jt][e], sl, -lq4[e]));
              if constexpr (MASK) pv = jok[jt] ? pv : 0.f;
              float dpv = dp[i2][jt][e], pd = pv;
              if constexpr (DROP) {
                const bool keep = keep_byte(hq[jt][e], li & 3, t8);
                dpv = keep ? dpv * dsc : 0.f;
                pd = keep ? pv * dsc : 0.f;
              }
              dp[i2][jt][e] = pv * (dpv - dq4[e]);  // dS
              s[i2][jt][e] = pd;                    // dropped P (for dV)
            }
          }
        }
        // dV[j][d] += sum_i Pd[i][j] dO[i][d] ; dK[j][d] += sum_i dS[i][j] Q[i][d]
        bf16x8 pa[2], sa[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          pa[jt] = pack8(s[0][jt], s[1][jt]);
          sa[jt] = pack8(dp[0][jt], dp[1][jt]);
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8 db = frag_col(dl, 32 * kq + 4 * g, 32 * kq + 16 + 4 * g, 16 * dt, lane);
          const bf16x8 qb2 = frag_col(ql, 32 * kq + 4 * g, 32 * kq + 16 + 4 * g, 16 * dt, lane);
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) {
            adv[jt][dt] = mfma16x16x32(pa[jt], db, adv[jt][dt]);
            adk[jt][dt] = mfma16x16x32(sa[jt], qb2, adk[jt][dt]);
          }
        }
      }
      if (more) {
        if (threadIdx.x < TQ) {
          s_lse[buf ^ 1][threadIdx.x] = r_lse;
          s_d[buf ^ 1][threadIdx.x] = r_d;
          if constexpr (DROP) s_rk[buf ^ 1][threadIdx.x] = r_rk;
        }
      }
      wait_vmcnt<0>();
      __syncthreads();
    }
  };
  if ((xb + 1) * BLOCK_ROWS <= len) qloop(std::false_type{});
  else qloop(std::true_type{});
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long j = k0 + 16 * jt + 4 * g + e;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dK[j * p.lddqkv + 16 * dt + li] = f2bf(adk[jt][dt][e] * p.scale);
        dV[j * p.lddqkv + 16 * dt + li] = f2bf(adv[jt][dt][e]);
      }
    }
}

// ================================================================ backward: dQ
template <int MINB, bool DROP>
__global__ __launch_bounds__(THREADS, MINB) void attn_bwd_dq_kernel(const AttnParams p) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][TILE_BYTES];  // [buf][K, V]
  int xb, h, b;
  attn_block(p, xb, h, b);
  const int S = p.S;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const long tok0 = (long)b * S;
  const int bh = b * p.H + h;
  const bf16_t* Q = p.qkv + tok0 * p.ld + p.q_off + h * HD;
  const bf16_t* K = p.qkv + tok0 * p.ld + p.k_off + h * HD;
  const bf16_t* V = p.qkv + tok0 * p.ld + p.v_off + h * HD;
  const bf16_t* dO = p.dout + tok0 * p.lddo + h * HD;
  const int len = p.lens ? min(max(p.lens[b], 0), S) : S;
  const int q0 = xb * BLOCK_ROWS + w * 32;
  bf16_t* dQ = p.dqkv + tok0 * p.lddqkv + p.q_off + h * HD;
  const float sl = p.scale_log2, dsc = p.drop_scale;
  const uint32_t t8 = p.drop_t8;

  bf16x8 qf[2][2], df[2][2];
  float lq[2], dq[2];
  uint32_t hk[2] = {0u, 0u};  // dropout: row key + the lane's key group
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = q0 + 16 * it + li;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[it][kk] = ldg_frag(Q + (long)i * p.ld + 32 * kk + 8 * g);
      df[it][kk] = ldg_frag(dO + (long)i * p.lddo + 32 * kk + 8 * g);
    }
    lq[it] = p.lse[(long)bh * S + i];
    if constexpr (DROP) hk[it] = row_key(p.drop_seed, bh, S, i) + (uint32_t)g;
  }
  // D_i = rowsum(dO * O): this block owns queries q0.., so it computes their D from the dO
  // fragments it already holds (the four g-lanes of a row cover its 64 columns) and publishes it
  // for the dK/dV kernel, which runs after this one — no separate pass over O and dO
  const bf16_t* O = p.o + tok0 * p.ldo + h * HD;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int i = q0 + 16 * it + li;
    float part = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 of = ldg_frag(O + (long)i * p.ldo + 32 * kk + 8 * g);
#pragma unroll
      for (int e = 0; e < 8; ++e) part = fmaf((float)of[e], (float)df[it][kk][e], part);
    }
    part += __shfl_xor(part, 16, 64);
    part += __shfl_xor(part, 32, 64);
    dq[it] = part;
    if (g == 0) p.dvec[(long)bh * S + i] = part;
  }
  f32x4 acc[2][4];  // dQ[i = 16it + 4g + e][d = 16dt + li]
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[it][dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one 64-key tile as two 32-key halves (S^T / dP^T of one half live at a time)
  auto tile = [&](const char* kl, const char* vl, const int kb, auto masked) {
    constexpr bool MASK = decltype(masked)::value;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      // S^T, dP^T: [j = kb + 32kk + 16j2 + 4g + e][i = 16it + li]
      f32x4 s[2][2], dp[2][2];
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2) {
        const int jt = 2 * kk + j2;
        const bf16x8 k0f = frag_row(kl, 16 * jt + li, 0, g), k1f = frag_row(kl, 16 * jt + li, 1, g);
        const bf16x8 v0f = frag_row(vl, 16 * jt + li, 0, g), v1f = frag_row(vl, 16 * jt + li, 1, g);
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f}, c = f32x4{0.f, 0.f, 0.f, 0.f};
          a = mfma16x16x32(k0f, qf[it][0], a);
          s[j2][it] = mfma16x16x32(k1f, qf[it][1], a);
          c = mfma16x16x32(v0f, df[it][0], c);
          dp[j2][it] = mfma16x16x32(v1f, df[it][1], c);
        }
      }
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          uint32_t hh = 0u;
          if constexpr (DROP) hh = hash24(hk[it] + (uint32_t)((kb >> 2) + 8 * kk + 4 * j2));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float pv = fexp2(fmaf(s[j2][it][e], sl, -lq[it]));
            if constexpr (MASK) {
              if (kb + 32 * kk + 16 * j2 + 4 * g + e >= len) pv = 0.f;
            }
            float dpv = dp[j2][it][e];
            if constexpr (DROP) dpv = keep_byte(hh, e, t8) ? dpv * dsc : 0.f;
            s[j2][it][e] = pv * (dpv - dq[it]);  // dS^T
          }
        }
      // dQ[i][d] += sum_j dS[i][j] K[j][d]
      const bf16x8 a0 = pack8(s[0][0], s[1][0]);
      const bf16x8 a1 = pack8(s[0][1], s[1][1]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 kb2 = frag_col(kl, 32 * kk + 4 * g, 32 * kk + 16 + 4 * g, 16 * dt, lane);
        acc[0][dt] = mfma16x16x32(a0, kb2, acc[0][dt]);
        acc[1][dt] = mfma16x16x32(a1, kb2, acc[1][dt]);
      }
    }
  };

  const int nkt = (len + TQ - 1) / TQ, nfull = len / TQ;
  if (nkt > 0) {
    dma_tile(K, p.ld, 0, len, lds[0][0]);
    dma_tile(V, p.ld, 0, len, lds[0][1]);
  }
  wait_vmcnt<0>();
  __syncthreads();
  // full tiles in one loop (one instantiation: no register copies at the back edge), then the
  // partial tile of a padded sequence
  for (int t = 0; t < nfull; ++t) {
    if (t + 1 < nkt) {
      dma_tile(K, p.ld, (t + 1) * TQ, len, lds[(t + 1) & 1][0]);
      dma_tile(V, p.ld, (t + 1) * TQ, len, lds[(t + 1) & 1][1]);
    }
    tile(lds[t & 1][0], lds[t & 1][1], t * TQ, std::false_type{});
    wait_vmcnt<0>();
    __syncthreads();
  }
  if (nfull < nkt) tile(lds[nfull & 1][0], lds[nfull & 1][1], nfull * TQ, std::true_type{});
#pragma unroll
  for (int it = 0; it < 2; ++it)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long i = q0 + 16 * it + 4 * g + e;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dQ[i * p.lddqkv + 16 * dt + li] = f2bf(acc[it][dt][e] * p.scale);
    }
}

}  // namespace

// XCD-aware block remap (attn_block): the S / 128 blocks of one sequence-head share an XCD's L2
static int attn_xcd() { return 1; }

#define DDL_ATTN_LAUNCH(KERNEL, grid, MINB, drop, s, p)                                   \
  do {                                                                                   \
    if (drop) hipLaunchKernelGGL((KERNEL<MINB, true>), grid, dim3(THREADS), 0, s, p);    \
    else hipLaunchKernelGGL((KERNEL<MINB, false>), grid, dim3(THREADS), 0, s, p);        \
  } while (0)

int attn_fwd(const AttnParams& p_in, hipStream_t s) {
  if (p_in.B <= 0) return 0;
  AttnParams p = p_in;
  p.xcd_remap = attn_xcd();
  const dim3 grid(p.S / BLOCK_ROWS, p.H, p.B);
  const bool drop = p.drop_t8 != 0;
  DDL_ATTN_LAUNCH(attn_fwd_kernel, grid, 2, drop, s, p);  // 2 workgroups per CU (measured vs 3 / 4)
  return (int)hipGetLastError();
}

int attn_bwd(const AttnParams& p_in, hipStream_t s) {
  if (p_in.B <= 0) return 0;
  AttnParams p = p_in;
  p.xcd_remap = attn_xcd();
  const dim3 grid(p.S / BLOCK_ROWS, p.H, p.B);
  const bool drop = p.drop_t8 != 0;
  // dQ first: it computes D = rowsum(dO * O) for its queries and writes p.dvec, which dK/dV reads
  DDL_ATTN_LAUNCH(attn_bwd_dq_kernel, grid, 2, drop, s, p);
  DDL_ATTN_LAUNCH(attn_bwd_dkdv_kernel, grid, 2, drop, s, p);
  return (int)hipGetLastError();
}

}  // namespace ddl
