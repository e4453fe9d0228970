// Instantiations of the implicit-GEMM kernel for the WGRAD view (gemm_kernel.h).
#include "gemm16_select.h"

namespace tmrg {
int launch_gemm_wgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (use16(a, MODE_WGRAD))
    return a.prec == TMR_MATH_F32 ? launch_gemm16<MODE_WGRAD, 1>(a, splits, st)
                                  : launch_gemm16<MODE_WGRAD, 0>(a, splits, st);
  return launch_gemm_t<MODE_WGRAD>(a, al, splits, st);
}
}  // namespace tmrg
