// NT-layout instantiations of the GEMM kernels (one translation unit per operand layout, so the
// template-heavy kernel family compiles in parallel).
#include "gemm_kernels.h"

namespace dllm {

hipError_t dispatch_nt(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  return dispatch_epi<L_NT>(path, epi, a, in_dt, out_dt, s);
}

// the NN weight-gradient layout's launches (gemm_kernels.h dispatch_x)
hipError_t dispatch_nt_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s) { return dispatch_x<L_NT>(epi, a, out_dt, s); }

}  // namespace dllm
