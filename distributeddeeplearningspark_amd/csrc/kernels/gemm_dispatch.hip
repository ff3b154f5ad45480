// Host-side dispatch of the implicit-GEMM kernel family.
#include "ddl_gemm.h"
#include <hip/hip_runtime.h>
#include <stdlib.h>
namespace ddl {
int launch_gemm_plain_akc(const GemmParams& p, int epi, int tile, hipStream_t s);
int launch_gemm_plain_arc(const GemmParams& p, int epi, int tile, hipStream_t s);
int launch_gemm_conv(const GemmParams& p, int epi, int tile, hipStream_t s);
int launch_gemm256(const GemmParams& p, int epi, hipStream_t s);
int launch_gemm_stream(const GemmParams& p, int epi, hipStream_t s);
int launch_conv3x3(const GemmParams& p, int epi, hipStream_t s);

int launch_gemm_bf16(const GemmParams& p_in, int epi, int tile, void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (p_in.M <= 0 || p_in.N <= 0) return 0;
  // grouped tile raster (GemmParams::group_m): 8 measured +1-2 % on BERT-base (835K vs 817-824K tok/s),
  // ResNet-50 neutral; 128-tile GEMM 8192^3 810 -> 1089 TF/s (profiles/r3/ab/gemm_group_m.jsonl); 16 worse
  GemmParams p = p_in;
  p.group_m = 8;
  if (p.bnr_x && tile != kTileStream &&  // fused BN-backward reduce on the other kernels: EPI_BF16_BNR
      (tile == kTile256 || epi != EPI_BF16 || p.om.zero_siblings ||
       (p.resid && (p.ldr % 4 || (uintptr_t)p.resid % 8)) || p.aux || p.drop_thresh || p.bias || p.relu || p.N % 4 || p.ldc % 8 ||
       !(p.a_mode == OP_KC || p.a_mode == OP_KC_GATHER) || (p.a_mode == OP_KC_GATHER && p.b_mode != OP_KC)))
    return (int)hipErrorInvalidValue;
  if (p.bnr_scale && tile == kTileStream && p.resid) return (int)hipErrorInvalidValue;  // streaming: mode 2 w/o residual
  const bool plain = (p.a_mode == OP_KC || p.a_mode == OP_RC) && (p.b_mode == OP_KC || p.b_mode == OP_RC);
  if (tile == kTile256) {  // 256x256 ping-pong kernel: plain operands, K and k_split % 64
    if (!plain || p.K % 64 || p.k_split % 64 || p.om.enabled) return (int)hipErrorInvalidValue;
    return launch_gemm256(p, epi, s);
  }
  if (tile == kTileStream) return launch_gemm_stream(p, epi, s);  // validates its own preconditions
  if (tile == kTileConv3) return launch_conv3x3(p, epi, s);       // validates its own preconditions
  if (plain) return p.a_mode == OP_KC ? launch_gemm_plain_akc(p, epi, tile, s) : launch_gemm_plain_arc(p, epi, tile, s);
  return launch_gemm_conv(p, epi, tile, s);
}
}  // namespace ddl
