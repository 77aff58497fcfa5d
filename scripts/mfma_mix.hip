// Microbenchmark: what a one-wave-per-SIMD GEMM pays for each non-MFMA instruction it interleaves between MFMAs.
//
// Question (round 5): hipBLASLt's MT256x256x64 kernel runs 4 waves (one per SIMD, 128x128 register tile each) at
// 0.86 MFMA busy; our two 4-wave prototypes (experiments/gemm_w4*.hip) staged operands with LDS-DMA and ran 8-20 %
// under the two-waves-per-SIMD 8-phase kernel.  If an LDS-DMA piece costs the issuing wave ~60 cycles of MFMA issue
// (MI355X_MICROARCH.md constants table), a single wave cannot hide its 16 pieces per K-tile; register staging
// (global_load_dwordx4 -> ds_write_b128) might interleave for less.  Each variant runs ITERS iterations of
// 8 independent v_mfma_f32_16x16x32_bf16 (operands in registers) with a fixed mix of other instructions placed
// between them, one workgroup of 4 waves per CU on every CU; it reports cycles per iteration (s_memtime around the loop,
// median over waves) and the MFMA pipe's share (8 x 16 cycles / cycles).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/mfma_mix.hip -o /tmp/mfma_mix && /tmp/mfma_mix
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(4))) int i32x4;   // 8 bf16 per lane (bit patterns only)
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int ITERS = 2048;

#define MF(i) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b))
#define GLDS() \
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + lane * 8), \
                                   (__attribute__((address_space(3))) void*)(lds + wid * 4096), 16, 0, 0)
#define GLOAD(r) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(src + lane * 8))
#define DSW(r) asm volatile("ds_write_b128 %0, %1" ::"v"(wofs), "v"(r))
#define DSR(r) asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(rofs))

template <int V>
__global__ __launch_bounds__(256) void mix(const unsigned short* __restrict__ gsrc, unsigned long long* out) {
  __shared__ __attribute__((aligned(16))) char lds_[65536];
  char* lds = lds_;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned short* src = gsrc + (blockIdx.x % 64) * 4096;   // L2-resident
  const unsigned wofs = (unsigned)(uintptr_t)(lds + 16384 + wid * 4096 + lane * 16);
  const unsigned rofs = (unsigned)(uintptr_t)(lds + 32768 + wid * 4096 + lane * 16);
  i32x4 a, b;
  for (int i = 0; i < 4; ++i) {
    a[i] = 0x3c003c00 + lane + i;   // bf16 pairs near 0.0078
    b[i] = 0x3b803b80 + lane - i;
  }
  f32x4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 r0 = {0, 0, 0, 0}, r1 = r0, r2 = r0, r3 = r0;
  __syncthreads();
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < ITERS; ++it) {
    MF(0);
    if constexpr (V == 1 || V == 2 || V == 9) GLDS();
    if constexpr (V == 3 || V == 4 || V == 8) GLOAD(r0);
    if constexpr (V == 5 || V == 6) DSW(r0);
    if constexpr (V == 7 || V == 8 || V == 9) DSR(r2);
    MF(1);
    if constexpr (V == 7) DSR(r3);
    MF(2);
    if constexpr (V == 2) GLDS();
    if constexpr (V == 4) GLOAD(r1);
    if constexpr (V == 6 || V == 8) DSW(r1);
    MF(3);
    if constexpr (V == 7 || V == 8 || V == 9) DSR(r3);
    MF(4);
    if constexpr (V == 7) DSR(r2);
    MF(5);
    MF(6);
    MF(7);
    // bounded queues: the loads / stores of this iteration must be back before the next one reuses their registers
    if constexpr (V >= 1) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(2)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][3];
  s += r0[0] + r1[1] + r2[2] + r3[3];
  // one value per wave, stored by every lane (vector stores); s keeps the MFMAs and loads live
  out[(blockIdx.x * 4 + wid) * 64 + lane] = (t1 - t0) + (s == 12345.f ? 1 : 0);
}

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  unsigned short* src;
  unsigned long long* out;
  hipMalloc(&src, 64 * 4096 * 2 + 4096);
  hipMemset(src, 0, 64 * 4096 * 2 + 4096);
  hipMalloc(&out, (size_t)ncu * 4 * 64 * 8);
  const char* names[] = {"8 MFMA only", "+1 glds", "+2 glds", "+1 global_load_dwordx4", "+2 global_load_dwordx4",
                         "+1 ds_write_b128", "+2 ds_write_b128", "+4 ds_read_b128",
                         "W4 register staging: +1 gload +1 ds_write +2 ds_read",
                         "W4 LDS-DMA staging: +1 glds +2 ds_read"};
  auto run = [&](auto kern, int v) {
    std::vector<double> med;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(kern, dim3(ncu), dim3(256), 0, 0, src, out);
      hipDeviceSynchronize();
      std::vector<unsigned long long> h((size_t)ncu * 4 * 64);
      hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
      std::vector<double> w;
      for (int i = 0; i < ncu * 4; ++i) w.push_back((double)h[(size_t)i * 64] / ITERS);
      std::sort(w.begin(), w.end());
      med.push_back(w[w.size() / 2]);
    }
    std::sort(med.begin(), med.end());
    const double c = med[med.size() / 2];
    printf("V%d %-40s %7.1f cycles / 8 MFMA  (MFMA pipe share %.3f, extra %.1f cycles)\n", v, names[v], c, 128.0 / c,
           c - 128.0);
  };
  for (int pass = 0; pass < 2; ++pass) {   // pass 0 warms the clock
    if (pass == 1) printf("one workgroup of 4 waves per CU on %d CUs, %d iterations\n", ncu, ITERS);
    auto go = [&](auto k, int v) { if (pass == 1) run(k, v); else { hipLaunchKernelGGL(k, dim3(ncu), dim3(256), 0, 0, src, out); hipDeviceSynchronize(); } };
    go(mix<0>, 0); go(mix<1>, 1); go(mix<2>, 2); go(mix<3>, 3); go(mix<4>, 4);
    go(mix<5>, 5); go(mix<6>, 6); go(mix<7>, 7); go(mix<8>, 8); go(mix<9>, 9);
  }
  hipFree(src);
  hipFree(out);
  return 0;
}
