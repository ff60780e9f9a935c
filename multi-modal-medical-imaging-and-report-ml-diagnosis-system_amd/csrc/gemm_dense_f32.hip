// Dense GEMM instantiations: compute float, output float (gemm_dense.h); the fused weight +
// bias gradient is 16-bit only (mmdx_gemm_bias_grad takes the GEMM + column-sum path for fp32).
#include "gemm_dense.h"

namespace mmdx {
MMDX_GEMM_TU_DEF(f32, float, float)
int gemm_wgrad_bias_f32(const SplitPlan&, int, int, int, const void*, long, const void*, long,
                        void*, long, float*, void*, hipStream_t) {
  mmdx_set_error("gemm bias grad: the fused form is 16-bit only");
  return -22;
}
}  // namespace mmdx
