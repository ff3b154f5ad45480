// Instantiations of the 256x256 ping-pong GEMM (ddl_gemm256.h): plain KC / RC operands.
#include "ddl_gemm256.h"
namespace ddl {
template <int AM, int BM>
static int launch_epi(const GemmParams& p, int epi, hipStream_t s) {
  if (epi == EPI_BF16)  // the slim epilogue when no residual / GELU / dropout / output map is used (code size)
    return !needs_full_epilogue(p) ? launch_g256<AM, BM, EPI_BF16_LITE>(p, s) : launch_g256<AM, BM, EPI_BF16>(p, s);
  if (epi == EPI_F32) return launch_g256<AM, BM, EPI_F32>(p, s);
  return launch_g256<AM, BM, EPI_F32_ATOMIC>(p, s);
}
int launch_gemm256(const GemmParams& p, int epi, hipStream_t s) {
  if (p.a_mode == OP_KC) return p.b_mode == OP_KC ? launch_epi<OP_KC, OP_KC>(p, epi, s) : launch_epi<OP_KC, OP_RC>(p, epi, s);
  return p.b_mode == OP_KC ? launch_epi<OP_RC, OP_KC>(p, epi, s) : launch_epi<OP_RC, OP_RC>(p, epi, s);
}
}  // namespace ddl
