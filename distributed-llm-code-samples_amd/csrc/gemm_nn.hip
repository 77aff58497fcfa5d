// NN-layout instantiations of the GEMM kernels (one translation unit per operand layout, so the
// template-heavy kernel family compiles in parallel).
#include "gemm_kernels.h"

namespace dllm {

hipError_t dispatch_nn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  return dispatch_epi<L_NN>(path, epi, a, in_dt, out_dt, s);
}

}  // namespace dllm
