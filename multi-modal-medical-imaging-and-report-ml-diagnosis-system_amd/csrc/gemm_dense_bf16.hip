// Dense GEMM instantiations: compute bf16, output bf16 (gemm_dense.h).
#include "gemm_dense.h"

namespace mmdx {
MMDX_GEMM_TU_DEF(bf16, bf16, bf16)
MMDX_GEMM_TU_DEF_WB(bf16, bf16, bf16)
}  // namespace mmdx
