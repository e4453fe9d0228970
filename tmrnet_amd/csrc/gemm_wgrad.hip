// Instantiations of the implicit-GEMM kernel for the WGRAD view (gemm_kernel.h).
#include "gemm16_kernel.h"

namespace tmrg {
int launch_gemm_wgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (use16(a, MODE_WGRAD)) return launch_gemm16_t<MODE_WGRAD>(a, splits, st);
  return launch_gemm_t<MODE_WGRAD>(a, al, splits, st);
}
}  // namespace tmrg
