// Dense GEMM instantiations: compute bf16, output float (gemm_dense.h).
#include "gemm_dense.h"

namespace mmdx {
MMDX_GEMM_TU_DEF(bf16f, bf16, float)
MMDX_GEMM_TU_DEF_WB(bf16f, bf16, float)
}  // namespace mmdx
