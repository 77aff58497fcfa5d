// TN-layout instantiations of the GEMM kernels (one translation unit per operand layout, so the
// template-heavy kernel family compiles in parallel).
#include "gemm_kernels.h"

namespace dllm {

hipError_t dispatch_tn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  return dispatch_epi<L_TN>(path, epi, a, in_dt, out_dt, s);
}

hipError_t dispatch_tn_opt(int path, int epi, const GemmArgs& a, int in_dt, hipStream_t s) {
  if (epi == EPI_SGD) return dispatch_opt<EPI_SGD>(path, a, in_dt, s);
  if (epi == EPI_SGDS) return dispatch_opt<EPI_SGDS>(path, a, in_dt, s);
  if (epi == EPI_ADAMS) return dispatch_opt<EPI_ADAMS>(path, a, in_dt, s);
  return dispatch_opt<EPI_ADAM>(path, a, in_dt, s);
}

hipError_t dispatch_tn_pair(int epi, const GemmArgs& a0, const GemmArgs& a1, int out_dt, hipStream_t s) {
  return dispatch_pair<L_TN, BT_M>(epi, a0, a1, out_dt, s);
}

// transposed plain store (operand-order experiments, tests): gemm_kernels.h dispatch_x
hipError_t dispatch_tn_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s) { return dispatch_x<L_TN>(epi, a, out_dt, s); }

}  // namespace dllm
