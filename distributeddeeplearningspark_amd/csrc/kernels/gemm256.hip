// Instantiations of the 256x256 ping-pong GEMM (ddl_gemm256.h): plain KC / RC operands.
#include "ddl_gemm256.h"
namespace ddl {
template <int AM, int BM>
static int launch_epi(const GemmParams& p, int epi, hipStream_t s, bool ps) {
  if (epi == EPI_BF16)  // the slim epilogue when no residual / GELU / dropout / output map is used (code size)
    return !needs_full_epilogue(p) ? launch_g256<AM, BM, EPI_BF16_LITE>(p, s, ps)
                                   : (row_epilogue() ? launch_g256<AM, BM, EPI_BF16_ROW>(p, s, ps)
                                                     : launch_g256<AM, BM, EPI_BF16>(p, s, ps));
  if (epi == EPI_F32) return launch_g256<AM, BM, EPI_F32>(p, s, ps);
  return launch_g256<AM, BM, EPI_F32_ATOMIC>(p, s, ps);
}
int launch_gemm256(const GemmParams& p, int epi, hipStream_t s, bool persist) {
  if (p.a_mode == OP_KC) return p.b_mode == OP_KC ? launch_epi<OP_KC, OP_KC>(p, epi, s, persist) : launch_epi<OP_KC, OP_RC>(p, epi, s, persist);
  return p.b_mode == OP_KC ? launch_epi<OP_RC, OP_KC>(p, epi, s, persist) : launch_epi<OP_RC, OP_RC>(p, epi, s, persist);
}
}  // namespace ddl
