// Implicit-GEMM convolution instantiations (NHWC): forward, data-gradient, weight-gradient.
#include "ddl_gemm_kernel.h"
namespace ddl {
int launch_gemm_conv(const GemmParams& p, int epi, int tile, hipStream_t s) {
  if (p.a_mode == OP_KC_GATHER && p.b_mode == OP_KC && epi == EPI_F32_ATOMIC)  // split-K small-grid forward
    return launch_modes<OP_KC_GATHER, OP_KC, EPI_F32_ATOMIC>(p, tile, s);
  if (p.a_mode == OP_KC_GATHER && p.b_mode == OP_KC && epi == EPI_F32)  // ... into partial slabs
    return launch_modes<OP_KC_GATHER, OP_KC, EPI_F32>(p, tile, s);
  if (p.a_mode == OP_KC_GATHER && p.b_mode == OP_KC && p.bnr_x)  // stride-1 dgrad as a forward conv + BN reduce
    return launch_modes<OP_KC_GATHER, OP_KC, EPI_BF16_BNR>(p, tile, s);
  if (p.a_mode == OP_KC_GATHER && p.b_mode == OP_KC)
    return needs_full_epilogue(p) ? launch_modes<OP_KC_GATHER, OP_KC, EPI_BF16>(p, tile, s)
                                  : launch_modes<OP_KC_GATHER, OP_KC, EPI_BF16_LITE>(p, tile, s);
  if (p.a_mode == OP_KC_GATHER && p.b_mode == OP_RC_TAPS) return launch_modes<OP_KC_GATHER, OP_RC_TAPS, EPI_BF16>(p, tile, s);
  if (p.a_mode == OP_RC && p.b_mode == OP_RC_GATHER) {
    if (epi == EPI_F32) return launch_modes<OP_RC, OP_RC_GATHER, EPI_F32>(p, tile, s);
    return launch_modes<OP_RC, OP_RC_GATHER, EPI_F32_ATOMIC>(p, tile, s);
  }
  // small channel counts (stem with channels padded to 8, MNIST CNN): per-vector tap lookup
  if (p.a_mode == OP_KC_GATHER8 && p.b_mode == OP_KC)
    return needs_full_epilogue(p) ? launch_modes<OP_KC_GATHER8, OP_KC, EPI_BF16>(p, tile, s)
                                  : launch_modes<OP_KC_GATHER8, OP_KC, EPI_BF16_LITE>(p, tile, s);
  if (p.a_mode == OP_RC && p.b_mode == OP_RC_GATHER8) {
    if (epi == EPI_F32) return launch_modes<OP_RC, OP_RC_GATHER8, EPI_F32>(p, tile, s);
    return launch_modes<OP_RC, OP_RC_GATHER8, EPI_F32_ATOMIC>(p, tile, s);
  }
  return (int)hipErrorInvalidValue;
}
}  // namespace ddl
