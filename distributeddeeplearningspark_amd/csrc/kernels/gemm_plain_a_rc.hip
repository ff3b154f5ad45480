// Plain GEMM instantiations with a row-contiguous (K-strided) A operand (TN / TT).
#include "ddl_gemm_kernel.h"
namespace ddl {
int launch_gemm_plain_arc(const GemmParams& p, int epi, int tile, hipStream_t s) {
  if (p.b_mode == OP_KC) {
    if (epi == EPI_BF16) return launch_modes<OP_RC, OP_KC, EPI_BF16>(p, tile, s);
    if (epi == EPI_F32) return launch_modes<OP_RC, OP_KC, EPI_F32>(p, tile, s);
    return launch_modes<OP_RC, OP_KC, EPI_F32_ATOMIC>(p, tile, s);
  }
  if (epi == EPI_BF16) return launch_modes<OP_RC, OP_RC, EPI_BF16>(p, tile, s);
  if (epi == EPI_F32) return launch_modes<OP_RC, OP_RC, EPI_F32>(p, tile, s);
  return launch_modes<OP_RC, OP_RC, EPI_F32_ATOMIC>(p, tile, s);
}
}  // namespace ddl
