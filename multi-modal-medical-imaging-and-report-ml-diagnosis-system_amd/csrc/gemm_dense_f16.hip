// Dense GEMM instantiations: compute f16, output f16 (gemm_dense.h).
#include "gemm_dense.h"

namespace mmdx {
MMDX_GEMM_TU_DEF(f16, f16, f16)
MMDX_GEMM_TU_DEF_WB(f16, f16, f16)
}  // namespace mmdx
