// Instantiations of the implicit-GEMM kernel for the WGRAD view (gemm_kernel.h).
#include "gemm_kernel.h"

namespace tmrg {
int launch_gemm_wgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  return launch_gemm_t<MODE_WGRAD>(a, al, splits, st);
}
}  // namespace tmrg
