// CU occupier (performance investigation only, not part of the library): `nblocks` one-wave workgroups
// holding 96 KiB of LDS each (so no GEMM block can share the CU) spin for `usec` microseconds on the
// 100-MHz s_memrealtime clock -- a stand-in for RCCL channel workgroups occupying CUs while a collective
// overlaps the GEMMs.  Built on demand by experiments/interference.py into experiments/_occupy.so.
#include <hip/hip_runtime.h>
#include <cstdint>

// see dllm_occupy_cus
__global__ __launch_bounds__(64) void occupy_kernel(long ticks) {
  __shared__ char hold[96 * 1024];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 1023) hold[ticks & 1023] = 0;  // keeps the LDS allocation
}

extern "C" {

// Interference probe (performance investigation only): `nblocks` single-wave workgroups, each holding
// 96 KiB of LDS (at most one per CU, and no 128-KiB GEMM block can share the CU), spin for `usec`
// microseconds on the 100-MHz s_memrealtime clock -- a stand-in for RCCL channel workgroups occupying
// CUs while a collective overlaps the GEMMs (scripts/interference.py).
int dllm_occupy_cus(int nblocks, int usec, void* stream) {
  if (nblocks <= 0 || usec <= 0) return -1;
  hipLaunchKernelGGL(occupy_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, (long)usec * 100);
  return (int)hipGetLastError();
}

}  // extern "C"
