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
  switch (epi) {
    case EPI_STORE:
      return out_dt == DT_F32 ? launch_pair<EPI_STORE, float>(a0, a1, s) : launch_pair<EPI_STORE, uint16_t>(a0, a1, s);
    case EPI_SGD: return launch_pair<EPI_SGD, float>(a0, a1, s);
    case EPI_SGDS: return launch_pair<EPI_SGDS, float>(a0, a1, s);
    case EPI_ADAM: return launch_pair<EPI_ADAM, float>(a0, a1, s);
    case EPI_ADAMS: return launch_pair<EPI_ADAMS, float>(a0, a1, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dllm
