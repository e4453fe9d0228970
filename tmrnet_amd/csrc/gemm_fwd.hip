// Instantiations of the implicit-GEMM kernel for the FWD view (gemm_kernel.h).
#include "gemm16_kernel.h"

namespace tmrg {
int launch_gemm_fwd(const GemmArgs& a, bool al, int splits, hipStream_t st) {
  if (use16(a, MODE_FWD)) return launch_gemm16_t<MODE_FWD>(a, splits, st);
  return launch_gemm_t<MODE_FWD>(a, al, splits, st);
}
}  // namespace tmrg
