// LDS-DMA engine (gemm16_kernel.h), the stride-parity classes of a strided DGRAD in one launch,
// f32 form: a translation unit of its own (compiles beside the per-view units).
#include "gemm16_kernel.h"

namespace tmrg {
template int launch_gemm16_par<1>(const GemmArgs* as, int n, hipStream_t st);
}  // namespace tmrg
