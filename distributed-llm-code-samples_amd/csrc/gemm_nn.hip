// NN-layout instantiations of the GEMM kernels (one translation unit per operand layout, so the
// template-heavy kernel family compiles in parallel).
#include "gemm_kernels.h"

namespace dllm {

hipError_t dispatch_nn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  return dispatch_epi<L_NN>(path, epi, a, in_dt, out_dt, s);
}

// the transposed-activation TP layout's weight gradients (M = F/tp on 224-row tiles): grouped pair / single fused update
hipError_t dispatch_nn_pair(int epi, const GemmArgs& a0, const GemmArgs& a1, int out_dt, hipStream_t s) {
  return dispatch_pair<L_NN, 224>(epi, a0, a1, out_dt, s);
}
hipError_t dispatch_nn_opt(int epi, const GemmArgs& a, hipStream_t s) {
  switch (epi) {
    case EPI_SGD: return launch_m224<L_NN, EPI_SGD>(a, DT_F32, s);
    case EPI_SGDS: return launch_m224<L_NN, EPI_SGDS>(a, DT_F32, s);
    case EPI_ADAM: return launch_m224<L_NN, EPI_ADAM>(a, DT_F32, s);
    case EPI_ADAMS: return launch_m224<L_NN, EPI_ADAMS>(a, DT_F32, s);
    default: return hipErrorInvalidValue;
  }
}

// the NN weight-gradient layout's launches (gemm_kernels.h dispatch_x)
hipError_t dispatch_nn_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s) { return dispatch_x<L_NN>(epi, a, out_dt, s); }

}  // namespace dllm
