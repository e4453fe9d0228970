// Instantiations of the implicit-GEMM kernel for the DGRAD view (gemm_kernel.h).
#include "gemm16_kernel.h"

namespace tmrg {
int launch_gemm_dgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (use16(a, MODE_DGRAD)) return launch_gemm16_t<MODE_DGRAD>(a, splits, st);
  return launch_gemm_t<MODE_DGRAD>(a, al, splits, st);
}
}  // namespace tmrg
