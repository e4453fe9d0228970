// Instantiations of the implicit-GEMM kernel for the DGRAD view (gemm_kernel.h).
#include "gemm16_select.h"

namespace tmrg {
int launch_gemm_dgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (use16(a, MODE_DGRAD))
    return a.prec == TMR_MATH_F32 ? launch_gemm16<MODE_DGRAD, 1>(a, splits, st)
                                  : launch_gemm16<MODE_DGRAD, 0>(a, splits, st);
  return launch_gemm_t<MODE_DGRAD>(a, al, splits, st);
}

// the stride-parity classes of one strided dgrad in one launch; -1: not eligible, launch them
// one by one
int launch_gemm_dgrad_par(const GemmArgs* as, int n, hipStream_t st) {
  if (n < 1) return -1;
  return as[0].prec == TMR_MATH_F32 ? launch_gemm16_par<1>(as, n, st) : launch_gemm16_par<0>(as, n, st);
}
}  // namespace tmrg
