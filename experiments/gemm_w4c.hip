// 4-wave 256x256x64 bf16 GEMM (NT, bf16 store): one wave per SIMD, a 128x128 register tile per wave.
//
// Why (round 5): hipBLASLt's kernel for the FFN's long-K NT store (y = a·W2ᵀ, train_ffns.py:41-42 / :57) is
// MT256x256x64 on 4 waves (solution metadata: waveNum 4, workGroup [32, 8, 1], DepthU 64), i.e. this tile shape,
// and holds 0.86 MFMA busy where the two-waves-per-SIMD 8-phase kernel holds 0.81: a 128x128 register tile reads a
// third fewer LDS bytes per MFMA and no partner wave shares the SIMD.  A microbenchmark of one wave per SIMD
// (scripts/mfma_mix.hip, profiles/r5/mfma_mix_r5.txt) prices what such a wave pays per instruction interleaved
// between MFMAs: ds_read_b128 ~2 cycles, LDS-DMA piece ~10, ds_write_b128 ~22 -- so operands are staged by LDS-DMA
// (global_load_lds) and the schedule exposes neither a DMA nor an LDS read:
//
//   LDS: 2 K-tile buffers x {A, B} of [256 rows][64 k] (128-B rows, 16-B chunk ^ (row>>1)&7) = 128 KiB.
//   Fragments: two register sets, F0 = k 0..31 and F1 = k 32..63 of a K-tile (8 A + 8 B ds_read_b128 each).
//   K-tile kt in buffer b = kt % 2, F0(kt) already in registers:
//     substep A: 64 MFMAs on F0(kt); reads F1(kt) from b.
//                end: lgkmcnt(0); vmcnt(0) retires this wave's DMA of K-tile kt+1 (issued a whole K-tile ago);
//                s_barrier (the only one per K-tile): K-tile kt+1 visible, and every wave is done reading b.
//     substep B: first the 16 DMA pieces of K-tile kt+2 into b (one per MFMA), then 64 MFMAs on F1(kt); reads
//                F0(kt+1) from b ^ 1.
//   So a DMA has two substeps (~2k cycles) to land, and each substep's MFMAs have their operands in registers.
// MFMAs are inline asm with the accumulators tied in AGPRs ("+a"), so program order is issue order and the 256
// accumulator registers never move; fragment reads are inline asm too (hipcc would otherwise drain the DMA queue
// with vmcnt(0) before every read).  The accumulation order per output element is the 8-phase kernel's (K-tiles in
// order, k 0..31 then 32..63 of each, one 16x16x32 MFMA per 32-deep step), so the outputs are bitwise equal.
#include <utility>

#include "common.h"

namespace dllm {
namespace w4 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int ST = 32768;  // one operand's K-tile stage (256 rows x 128 B)

struct Args {
  const void* A;
  const void* B;
  void* C;
  long lda, ldb, ldc;
  int M, N, K, group_m;
};

__device__ __forceinline__ void glds16(const uint16_t* src, DLLM_LDS char* dst) {
  __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)src, (DLLM_LDS void*)dst, 16, 0, 0);
}
template <int OFF>
__device__ __forceinline__ void rd(bf16x8_t& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}

// ABL (timing ablations only, wrong results): 1 no vmcnt wait, 2 no vmcnt wait and no barrier, 3 no LDS-DMA,
// 4 no LDS-DMA and no barrier, 5 no fragment reads.  DSP: DMA placement in substep B -- 0 one piece per MFMA at the
// head, 1 one per 4 MFMAs over the whole substep, 2 one per 2 MFMAs over its first half
template <int ABL, int DSP = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * ST];
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int tiles_m = p.M / BM, tiles_n = p.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int width = p.group_m * tiles_n;
  const int first_m = (bid / width) * p.group_m;
  const int gsz = min(tiles_m - first_m, p.group_m);
  const int m0 = (first_m + (bid % width) % gsz) * BM;
  const int n0 = ((bid % width) / gsz) * BN;

  const uint16_t* Ag = (const uint16_t*)p.A + (long)m0 * p.lda;
  const uint16_t* Bg = (const uint16_t*)p.B + (long)n0 * p.ldb;
  // LDS-DMA: 32 pieces of 1 KiB (8 rows) per operand and stage; this wave issues pieces q = wid + 4 i, i < 8.
  // Per-lane 32-bit byte offsets from the panel base (swizzle applied on the source: the DMA writes lane-linearly).
  uint32_t aoff[8], boff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int row = 8 * (wid + 4 * i) + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    aoff[i] = (uint32_t)(((long)row * p.lda + c * 8) * 2);
    boff[i] = (uint32_t)(((long)row * p.ldb + c * 8) * 2);
  }
  const int nk = p.K / BK;
  // piece j (0..15: A pieces 0..7, then B) of K-tile kt into buffer buf
  auto dma = [&](int kt, int buf, int j) {
    const long koff = (long)kt * BK * 2;  // bytes
    if (j < 8)
      glds16((const uint16_t*)((const char*)Ag + koff + aoff[j]), lds + buf * ST + (wid + 4 * j) * 1024);
    else
      glds16((const uint16_t*)((const char*)Bg + koff + boff[j - 8]), lds + 2 * ST + buf * ST + (wid + 4 * (j - 8)) * 1024);
  };

  // fragment bases: A rows wr*128 + mt*16 + (lane&15), B rows wc*128 + nt*16 + (lane&15); k-substep s: chunks 4s + g
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

#define W4_MF(I, FA, FB) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[(I) >> 3][(I)&7]) : "v"(FB[(I)&7]), "v"(FA[(I) >> 3]))
  // read the 16 fragments of k-substep S of buffer BUF into (NA, NB), fragment J = A tiles 0..7 then B tiles 0..7
#define W4_RD(J, NA, NB, S, BUF)                                                                  \
  do {                                                                                            \
    if constexpr ((J) < 8) rd<(BUF)*ST + ((J)&7) * 2048>(NA[(J)&7], ab[S]);                        \
    else rd<(BUF)*ST + ((J)&7) * 2048>(NB[(J)&7], bb[S]);                                          \
  } while (0)

  // substep: 64 MFMAs on (FA, FB); with RD the next fragments (k-substep RS of buffer RBUF) are read one per 4 MFMAs;
  // with DMA the 16 pieces of K-tile dkt go to buffer DBUF, one per MFMA at the head of the substep
  auto substep = [&](auto& FA, auto& FB, auto& NA, auto& NB, auto rs_c, auto rbuf_c, auto rd_c, auto dma_c, int dkt,
                     auto dbuf_c) {
    constexpr int RS = decltype(rs_c)::value, RBUF = decltype(rbuf_c)::value, DBUF = decltype(dbuf_c)::value;
    constexpr bool RD = decltype(rd_c)::value, DMA = decltype(dma_c)::value;
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (
          [&] {
            W4_MF(I, FA, FB);
            constexpr bool dma_here = DSP == 0 ? I < 16 : DSP == 1 ? I % 4 == 0 : (I < 32 && I % 2 == 0);
            constexpr int dj = DSP == 0 ? I : DSP == 1 ? I / 4 : I / 2;
            if constexpr (DMA && dma_here && ABL != 3 && ABL != 4) dma(dkt, DBUF, dj);
            if constexpr (RD && I % 4 == 2 && ABL != 5) W4_RD(I / 4, NA, NB, RS, RBUF);
          }(),
          ...);
    }(std::make_integer_sequence<int, 64>{});
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using T = std::integral_constant<bool, true>;
  using Fb = std::integral_constant<bool, false>;
#define W4_LDS_WAIT()                                    \
  do {                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_sched_barrier(0);                   \
  } while (0)
#define W4_BARRIER()                       \
  do {                                     \
    asm volatile("" ::: "memory");         \
    if constexpr (ABL != 2 && ABL != 4) __builtin_amdgcn_s_barrier(); \
    asm volatile("" ::: "memory");         \
  } while (0)
#define W4_VMWAIT()                                                         \
  do {                                                                      \
    if constexpr (ABL == 0 || ABL == 5) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
  } while (0)

  // prologue: K-tiles 0 and 1 in flight; retire K-tile 0 (16 younger pieces), read F0(0)
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(0, 0, j);
#pragma unroll
  for (int j = 0; j < 16; ++j) dma(min(1, nk - 1), 1, j);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  W4_BARRIER();
  [&]<int... J>(std::integer_sequence<int, J...>) {
    ([&] { W4_RD(J, fa0, fb0, 0, 0); }(), ...);
  }(std::make_integer_sequence<int, 16>{});
  W4_LDS_WAIT();

  // two K-tiles per iteration (static buffer indices); nk is even (host check).  The last iteration's DMAs (K-tiles
  // nk, nk+1, clamped to nk-1) and its final fragment reads land in buffers nobody reads again: every iteration runs
  // the same code (one instantiation per substep keeps the 256 accumulators in fixed AGPRs).
  for (int kt = 0; kt < nk; kt += 2) {
    const int k2 = min(kt + 2, nk - 1), k3 = min(kt + 3, nk - 1);
    // ---- K-tile kt, buffer 0 ----
    substep(fa0, fb0, fa1, fb1, I1{}, I0{}, T{}, Fb{}, 0, I0{});          // A: MFMA F0(kt); read F1(kt)
    W4_LDS_WAIT();
    W4_VMWAIT();                                                          // K-tile kt+1 landed (this wave's pieces)
    W4_BARRIER();
    substep(fa1, fb1, fa0, fb0, I0{}, I1{}, T{}, T{}, k2, I0{});          // B: DMA kt+2 -> buf 0; read F0(kt+1)
    W4_LDS_WAIT();
    // ---- K-tile kt+1, buffer 1 ----
    substep(fa0, fb0, fa1, fb1, I1{}, I1{}, T{}, Fb{}, 0, I0{});          // A: MFMA F0(kt+1); read F1(kt+1)
    W4_LDS_WAIT();
    W4_VMWAIT();                                                          // K-tile kt+2 landed
    W4_BARRIER();
    substep(fa1, fb1, fa0, fb0, I0{}, I0{}, T{}, T{}, k3, I1{});          // B: DMA kt+3 -> buf 1; read F0(kt+2)
    W4_LDS_WAIT();
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
#undef W4_MF
#undef W4_RD

  // epilogue: bf16, paired 16-B stores (nt = 2j, 2j+1 form one 32-column strip, exchanged with the lane 16 away)
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

// C = A[M][K] · B[N][K]ᵀ in bf16 (plain store) on the 4-wave kernel; returns -1 for shapes it does not take.
extern "C" int dllm_gemm_w4(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                            int group_m, void* stream, int ablate) {
  using namespace dllm::w4;
  if (M <= 0 || N <= 0 || M % BM || N % BN || K % (2 * BK) || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return -1;
  if ((long)(BM - 1) * lda * 2 + (long)K * 2 >= (1L << 32) || (long)(BN - 1) * ldb * 2 + (long)K * 2 >= (1L << 32))
    return -1;  // 32-bit per-lane DMA offsets from the panel base
  Args a{A, B, C, lda, ldb, ldc, M, N, K, group_m > 0 ? group_m : 4};
  const dim3 grid((M / BM) * (N / BN));
  switch (ablate) {
    case 1: hipLaunchKernelGGL(gemm_nt_w4<1>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 2: hipLaunchKernelGGL(gemm_nt_w4<2>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 3: hipLaunchKernelGGL(gemm_nt_w4<3>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 4: hipLaunchKernelGGL(gemm_nt_w4<4>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 5: hipLaunchKernelGGL(gemm_nt_w4<5>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 10: hipLaunchKernelGGL((gemm_nt_w4<0, 1>), grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 11: hipLaunchKernelGGL((gemm_nt_w4<0, 2>), grid, dim3(256), 0, (hipStream_t)stream, a); break;
    case 12: hipLaunchKernelGGL((gemm_nt_w4<2, 1>), grid, dim3(256), 0, (hipStream_t)stream, a); break;
    default: hipLaunchKernelGGL(gemm_nt_w4<0>, grid, dim3(256), 0, (hipStream_t)stream, a); break;
  }
  return (int)hipGetLastError();
}
