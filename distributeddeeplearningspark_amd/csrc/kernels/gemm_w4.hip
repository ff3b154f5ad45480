// Instantiations of the four-wave 256x256 / 256x128 GEMM (ddl_gemm_w4.h): plain KC / RC operands.
#include "ddl_gemm_w4.h"
namespace ddl {
template <int BN, int AM, int BM>
static int launch_epi(const GemmParams& p, int epi, hipStream_t s) {
  if (epi == EPI_BF16)  // slim epilogue, or the LDS-staged row epilogue for residual / GELU / dropout
    return !needs_full_epilogue(p) ? launch_w4<BN, AM, BM, EPI_BF16_LITE>(p, s) : launch_w4<BN, AM, BM, EPI_BF16_ROW>(p, s);
  if (epi == EPI_F32) return launch_w4<BN, AM, BM, EPI_F32>(p, s);
  return launch_w4<BN, AM, BM, EPI_F32_ATOMIC>(p, s);
}
template <int BN>
static int launch_modes(const GemmParams& p, int epi, hipStream_t s) {
  if (p.a_mode == OP_KC)
    return p.b_mode == OP_KC ? launch_epi<BN, OP_KC, OP_KC>(p, epi, s) : launch_epi<BN, OP_KC, OP_RC>(p, epi, s);
  return p.b_mode == OP_KC ? launch_epi<BN, OP_RC, OP_KC>(p, epi, s) : launch_epi<BN, OP_RC, OP_RC>(p, epi, s);
}
int launch_gemm_w4(const GemmParams& p, int epi, int tile, hipStream_t s) {
  return tile == kTileW4 ? launch_modes<256>(p, epi, s) : launch_modes<128>(p, epi, s);
}
}  // namespace ddl
