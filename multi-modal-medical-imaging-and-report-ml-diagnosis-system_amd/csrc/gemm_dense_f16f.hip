// Dense GEMM instantiations: compute f16, output float (gemm_dense.h).
#include "gemm_dense.h"

namespace mmdx {
MMDX_GEMM_TU_DEF(f16f, f16, float)
MMDX_GEMM_TU_DEF_WB(f16f, f16, float)
}  // namespace mmdx
