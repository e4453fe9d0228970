// LDS-DMA engine (gemm16_kernel.h), DGRAD view, bf16 form: one view x precision per translation unit.
#include "gemm16_kernel.h"

namespace tmrg {
template int launch_gemm16<MODE_DGRAD, 0>(const GemmArgs& a, int splits, hipStream_t st);
}  // namespace tmrg
