// Prototype: 256x256x64 bf16 GEMM with 4 waves (one per SIMD), 128x128 output per wave.
//
// Hypothesis under test (performance investigation, not yet wired into dllm_gemm): with a 128x128
// register tile per wave (64 accumulators of 16x16, 256 AGPR/VGPRs) each wave reads 0.25 fragments per
// MFMA from LDS instead of the 8-phase kernel's 0.375, cutting LDS read energy by a third; on this
// power-limited chip (MI355X_MICROARCH.md "DVFS give-back") fewer bytes per MFMA can buy clock.  The
// cost: one wave per SIMD, so LDS latency must be covered inside the wave (fragments for substep s+1
// are read while substep s's 64 MFMAs run) and the LDS-DMA issue cost is paid by the computing wave.
//
// Layout NT (A[M][K], B[N][K], both K-contiguous), bf16 out.  LDS: A stages at [0, 64K), B at
// [64K, 128K) so every fragment read is a per-lane base + 16-bit immediate.
#include <utility>

#include "common.h"

namespace dllm {
namespace w4 {

constexpr int BM = 256, BN = 256, BK = 64;

__device__ __forceinline__ void glds16(const uint16_t* src, DLLM_LDS char* dst) {
  __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)src, (DLLM_LDS void*)dst, 16, 0, 0);
}
template <int OFF>
__device__ __forceinline__ void rd(bf16x8_t& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
#define W4_LDS_WAIT()                                    \
  do {                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);                   \
  } while (0)
#define W4_BARRIER()                       \
  do {                                     \
    asm volatile("" ::: "memory");         \
    __builtin_amdgcn_s_barrier();          \
    asm volatile("" ::: "memory");         \
  } while (0)

struct Args {
  const void* A;
  const void* B;
  void* C;
  long lda, ldb, ldc;
  int M, N, K, group_m;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 32768];
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int width = p.group_m * tiles_n;
  const int first_m = (bid / width) * p.group_m;
  const int gsz = min(tiles_m - first_m, p.group_m);
  const int tm = first_m + (bid % width) % gsz;
  const int tn = (bid % width) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const uint16_t* Ag = (const uint16_t*)p.A + (long)m0 * p.lda;
  const uint16_t* Bg = (const uint16_t*)p.B + (long)n0 * p.ldb;
  // LDS: 2 stages x {A, B} of [256 rows][64 k] (128-B rows, 16-B chunk c of row r at c ^ ((r>>1)&7));
  // A stages at [0, 64K), B stages at [64K, 128K).  LDS-DMA: 32 pieces of 1 KiB (8 rows) per operand
  // and stage; this wave issues q = wid + 4*i, i < 8.
  constexpr int ST = 32768;
  int aoff[8], boff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = wid + 4 * i;
    const int row = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    aoff[i] = row * (int)p.lda + c * 8;
    boff[i] = row * (int)p.ldb + c * 8;
  }
  const int nk = p.K / BK;
  auto stage = [&](int kt, int buf) {
    const int koff = min(kt, nk - 1) * BK;
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(Ag + koff + aoff[i], lds + buf * ST + (wid + 4 * i) * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i) glds16(Bg + koff + boff[i], lds + 2 * ST + buf * ST + (wid + 4 * i) * 1024);
  };

  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int g = lane >> 4, i15 = lane & 15, fkc = (i15 >> 1) & 7;
  uint32_t ab[2], bb[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    ab[s] = lds_base + (wr * 128 + i15) * 128 + (((4 * s + g) ^ fkc) << 4);
    bb[s] = lds_base + 2 * ST + (wc * 128 + i15) * 128 + (((4 * s + g) ^ fkc) << 4);
  }

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
#define W4_MF(I, FA, FB)                                                                      \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"                                      \
               : "+a"(acc[(I) >> 3][(I)&7]) : "v"(FB[(I)&7]), "v"(FA[(I) >> 3]))
#define W4_RD(J, NA, NB, RS, RBUF)                                                            \
  [&] {                                                                                       \
    if constexpr ((J) < 8) rd<(RBUF)*ST + ((J)&7) * 2048>(NA[(J)&7], ab[RS]);                 \
    else rd<(RBUF)*ST + ((J)&7) * 2048>(NB[(J)&7], bb[RS]);                                   \
  }()
  // One substep = 64 MFMAs (k 32) on (FA, FB) with the next substep's 16 fragment reads (k-half RS of
  // buffer RBUF into NA/NB) one per RD_EVERY MFMAs and, when STG, K-tile skt's 16 LDS-DMA pieces into
  // buffer SBUF one per 4 MFMAs.  MFMAs are inline asm with the accumulator tied ("+a"): program order
  // is issue order and the 64 accumulators stay in fixed AGPRs.
  auto substep = [&](auto& FA, auto& FB, auto& NA, auto& NB, auto rs_c, auto rbuf_c, auto stg_c, int skt,
                     auto sbuf_c) {
    constexpr int RS = decltype(rs_c)::value, RBUF = decltype(rbuf_c)::value;
    constexpr bool STG = decltype(stg_c)::value;
    constexpr int SBUF = decltype(sbuf_c)::value;
    const int koff = min(skt, nk - 1) * BK;
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (
          [&] {
            W4_MF(I, FA, FB);
            if constexpr (I % 3 == 2 && I / 3 < 16) W4_RD(I / 3, NA, NB, RS, RBUF);
            if constexpr (STG && I % 4 == 0) {
              constexpr int q = I / 4;  // 0..15: A pieces 0..7, B pieces 0..7
              if constexpr (q < 8) glds16(Ag + koff + aoff[q], lds + SBUF * ST + (wid + 4 * q) * 1024);
              else glds16(Bg + koff + boff[q - 8], lds + 2 * ST + SBUF * ST + (wid + 4 * (q - 8)) * 1024);
            }
          }(),
          ...);
    }(std::make_integer_sequence<int, 64>{});
  };
  using F0 = std::integral_constant<int, 0>;
  using F1 = std::integral_constant<int, 1>;
  using NoStg = std::integral_constant<bool, false>;
  using Stg = std::integral_constant<bool, true>;

  // prologue: K-tiles 0 and 1 in flight, wait for 0, read its substep-0 fragments
  stage(0, 0);
  stage(1, 1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  W4_BARRIER();
  [&]<int... J>(std::integer_sequence<int, J...>) { (W4_RD(J, fa0, fb0, 0, 0), ...); }(std::make_integer_sequence<int, 16>{});
  W4_LDS_WAIT();

  // Two K-tiles per iteration.  Before a K-tile's second substep (which reads the NEXT tile's first
  // fragments): vmcnt(0) = this wave's LDS-DMA pieces of the next tile landed; the barrier makes all
  // pieces visible and retires every wave's reads of the buffer about to be restaged.
  for (int kt = 0; kt < nk; kt += 2) {
    substep(fa0, fb0, fa1, fb1, F1{}, F0{}, NoStg{}, 0, F0{});        // (kt, s0); read (kt, s1)
    W4_LDS_WAIT();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W4_BARRIER();
    substep(fa1, fb1, fa0, fb0, F0{}, F1{}, Stg{}, kt + 2, F0{});     // (kt, s1); read (kt+1, s0); DMA kt+2
    W4_LDS_WAIT();
    substep(fa0, fb0, fa1, fb1, F1{}, F1{}, NoStg{}, 0, F0{});        // (kt+1, s0); read (kt+1, s1)
    W4_LDS_WAIT();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    W4_BARRIER();
    substep(fa1, fb1, fa0, fb0, F0{}, F0{}, Stg{}, kt + 3, F1{});     // (kt+1, s1); read (kt+2, s0); DMA kt+3
    W4_LDS_WAIT();
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
#undef W4_MF
#undef W4_RD

  // epilogue: bf16, paired 16-B stores (nt = 2j, 2j+1 form one 32-column strip)
  const int pc = 16 * ((lane >> 4) & 1) + 8 * (lane >> 5);
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    const int m = m0 + wr * 128 + mt * 16 + i15;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t a = acc[mt][2 * j], b = acc[mt][2 * j + 1];
      const uint2 pa = {(uint32_t)f2bf(a[0]) | ((uint32_t)f2bf(a[1]) << 16), (uint32_t)f2bf(a[2]) | ((uint32_t)f2bf(a[3]) << 16)};
      const uint2 pb = {(uint32_t)f2bf(b[0]) | ((uint32_t)f2bf(b[1]) << 16), (uint32_t)f2bf(b[2]) | ((uint32_t)f2bf(b[3]) << 16)};
      const auto x = __builtin_amdgcn_permlane16_swap(pa.x, pb.x, false, false);
      const auto y = __builtin_amdgcn_permlane16_swap(pa.y, pb.y, false, false);
      *(uint4*)((uint16_t*)p.C + (long)m * p.ldc + n0 + wc * 128 + j * 32 + pc) = uint4{x[0], y[0], x[1], y[1]};
    }
  }
}

}  // namespace w4
}  // namespace dllm

extern "C" int dllm_gemm_w4_proto(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N,
                                  int K, int group_m, void* stream) {
  using namespace dllm::w4;
  if (M % BM || N % BN || K % (2 * BK) || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if ((long)M * lda >= (1L << 31) || (long)N * ldb >= (1L << 31)) return -1;  // 32-bit piece offsets
  Args a{A, B, C, lda, ldb, ldc, M, N, K, group_m > 0 ? group_m : 4};
  hipLaunchKernelGGL(gemm_nt_w4, dim3((M / BM) * (N / BN)), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
