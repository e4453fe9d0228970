// LDS-DMA engine (gemm16_kernel.h), DGRAD view, f32 form: one view x precision per translation unit.
#include "gemm16_kernel.h"

namespace tmrg {
template int launch_gemm16<MODE_DGRAD, 1>(const GemmArgs& a, int splits, hipStream_t st);
}  // namespace tmrg
