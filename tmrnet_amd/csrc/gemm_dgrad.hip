// Instantiations of the implicit-GEMM kernel for the DGRAD view (gemm_kernel.h).
#include "gemm_kernel.h"

namespace tmrg {
int launch_gemm_dgrad(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  return launch_gemm_t<MODE_DGRAD>(a, al, splits, st);
}
}  // namespace tmrg
