// TN-layout instantiations of the GEMM kernels (one translation unit per operand layout, so the
// template-heavy kernel family compiles in parallel).
#include "gemm_kernels.h"

namespace dllm {

hipError_t dispatch_tn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  return dispatch_epi<L_TN>(path, epi, a, in_dt, out_dt, s);
}

hipError_t dispatch_tn_opt(int path, int epi, const GemmArgs& a, int in_dt, hipStream_t s) {
  return epi == EPI_SGD ? dispatch_opt<EPI_SGD>(path, a, in_dt, s) : dispatch_opt<EPI_ADAM>(path, a, in_dt, s);
}

// ablation launcher (performance investigation only): TN layout, bf16 out, square problems
hipError_t launch_tn_ablation(int abl, const GemmArgs& a, int nb, hipStream_t s) {
#define DLLM_ABL(X) \
  case X: hipLaunchKernelGGL((gemm_bf16_8ph<L_TN, EPI_STORE, uint16_t, true, X>), dim3(nb), dim3(512), 0, s, a); break;
  switch (abl) {
    DLLM_ABL(0) DLLM_ABL(3) DLLM_ABL(12) DLLM_ABL(15) DLLM_ABL(1) DLLM_ABL(4) DLLM_ABL(5) DLLM_ABL(10)
    default: return hipErrorInvalidValue;
  }
#undef DLLM_ABL
  return hipGetLastError();
}

}  // namespace dllm
