// Plain GEMM instantiations with a K-contiguous A operand (NT / NN).
#include "ddl_gemm_kernel.h"
namespace ddl {
int launch_gemm_plain_akc(const GemmParams& p, int epi, int tile, hipStream_t s) {
  if (p.bnr_x && epi == EPI_BF16)  // data-gradient + fused BN-backward reduce (dispatch checked the epilogue)
    return p.b_mode == OP_KC ? launch_modes<OP_KC, OP_KC, EPI_BF16_BNR>(p, tile, s)
                             : launch_modes<OP_KC, OP_RC, EPI_BF16_BNR>(p, tile, s);
  if (p.b_mode == OP_KC) {
    if (epi == EPI_BF16)
      return !needs_full_epilogue(p) ? launch_modes<OP_KC, OP_KC, EPI_BF16_LITE>(p, tile, s)
                                     : launch_modes<OP_KC, OP_KC, EPI_BF16>(p, tile, s);
    if (epi == EPI_F32) return launch_modes<OP_KC, OP_KC, EPI_F32>(p, tile, s);
    return launch_modes<OP_KC, OP_KC, EPI_F32_ATOMIC>(p, tile, s);
  }
  if (epi == EPI_BF16)
    return !needs_full_epilogue(p) ? launch_modes<OP_KC, OP_RC, EPI_BF16_LITE>(p, tile, s)
                                   : launch_modes<OP_KC, OP_RC, EPI_BF16>(p, tile, s);
  if (epi == EPI_F32) return launch_modes<OP_KC, OP_RC, EPI_F32>(p, tile, s);
  return launch_modes<OP_KC, OP_RC, EPI_F32_ATOMIC>(p, tile, s);
}
}  // namespace ddl
