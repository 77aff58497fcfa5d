// Prototype (round 2): 256x256 bf16 GEMM, 4 waves (one per SIMD, 128x128 accumulators each in AGPRs), K-tiles
// of 32 in a 4-stage LDS-DMA ring (4 x 32 KiB), DMA issued THREE K-tiles ahead.
//
// Why: the flagship GEMMs run power-limited (1.84-2.13 GHz under load, profiles/r2/pmc_l2_clock_r2.txt), so
// energy per MFMA sets the throughput.  A 128x128 register tile per wave reads 0.25 fragments per MFMA from LDS
// (the 8-wave 8-phase kernel: 0.375).  The round-1 4-wave prototype (experiments/gemm_w4_proto.hip) matched the
// 8-phase kernel at 8192^3 but lost on the FFN's long-K shapes: with two 64-deep stages its DMA had ~1 substep
// (1024 cycles) of lead.  Here the DMA lead is 3 K-tiles (3 x 64 MFMAs x 16 cycles = 3072 cycles), one barrier per
// K-tile (4 waves), every MFMA / fragment read / DMA hand-placed (inline-asm MFMAs on tied AGPR accumulators).
//
// Layout NT (A[M][K], B[N][K], both K-contiguous), bf16 out.  LDS per stage: A [256 rows][32 k] then B, 64-B rows,
// 16-B chunk c of row r stored at c ^ ((r >> 2) & 3) (conflict-free ds_read_b128 of 16 rows x 4 chunks).
// Standalone: experiments/bench_w4b.py builds it into experiments/_w4b.so.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
#define DLLM_LDS __attribute__((address_space(3)))
#define DLLM_GLB __attribute__((address_space(1)))

namespace w4b {

#ifndef W4B_NST
#define W4B_NST 4
#endif
#ifndef W4B_RD_EVERY
#define W4B_RD_EVERY 2  // one fragment read per this many MFMAs, from the K-tile's first MFMA on
#endif
constexpr int BM = 256, BN = 256, BK = 32, NST = W4B_NST;
constexpr int OPB = BM * BK * 2;  // 16 KiB per operand per stage
constexpr int STB = 2 * OPB;      // 32 KiB per stage

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int xcd = bid % nx, q = nwg / nx, r = nwg % nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / nx;
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ void glds16(const uint16_t* src, DLLM_LDS char* dst) {
  __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)src, (DLLM_LDS void*)dst, 16, 0, 0);
}
template <int OFF>
__device__ __forceinline__ void rd(bf16x8_t& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
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

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_nt_w4b(Args p) {
  __shared__ __attribute__((aligned(16))) char smem[NST * STB];
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
  // LDS-DMA: an operand stage is 16 pieces of 1 KiB (16 rows x 64 B, lane-linear); wave w issues pieces
  // w, w+4, w+8, w+12 of A and of B.  Lane j of piece q: row 16q + j/4, stored chunk j%4 <- logical chunk
  // (j%4) ^ ((row>>2)&3).  Byte offsets (32-bit) from the K-tile's panel base.
  uint32_t aoff[4], boff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid + 4 * i, row = 16 * q + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);
    aoff[i] = (uint32_t)((row * p.lda + c * 8) * 2);
    boff[i] = (uint32_t)((row * p.ldb + c * 8) * 2);
  }
  const int nk = p.K / BK;
  auto dma = [&](int kt, int buf, int i) {  // piece i (0..3 A, 4..7 B) of K-tile kt (clamped) into buf
    const int koff = min(kt, nk - 1) * BK * 2;
    if (i < 4)
      glds16((const uint16_t*)((const char*)Ag + koff + aoff[i]), lds + buf * STB + (wid + 4 * i) * 1024);
    else
      glds16((const uint16_t*)((const char*)Bg + koff + boff[i - 4]), lds + buf * STB + OPB + (wid + 4 * (i - 4)) * 1024);
  };
  // fragment read addresses: lane reads row r0 + (lane&15), logical chunk lane>>4 (k 8c .. 8c+7)
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int g = lane >> 4, i15 = lane & 15;
  // row r = base + i15 (base multiple of 16): stored chunk g ^ ((i15 >> 2) & 3)
  const uint32_t frag = (uint32_t)(i15 * 64 + ((g ^ ((i15 >> 2) & 3)) << 4));
  const uint32_t abase = lds_base + (wr * 128) * 64 + frag;
  const uint32_t bbase = lds_base + OPB + (wc * 128) * 64 + frag;

  f32x4_t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa0[8], fb0[8], fa1[8], fb1[8];
#define W4_MF(I, FA, FB)                                                                      \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"                                      \
               : "+a"(acc[(I) >> 3][(I)&7]) : "v"(FB[(I)&7]), "v"(FA[(I) >> 3]))
  // one K-tile: 64 MFMAs on (FA, FB); the next K-tile's 16 fragment reads (buffer RB) one per 4 MFMAs; the
  // 8 DMA pieces of K-tile dkt (buffer DB) one per 8 MFMAs
  auto ktile = [&](auto& FA, auto& FB, auto& NA, auto& NB, int rb, int dkt, int db) {
    const uint32_t ra = abase + rb * STB, rbb = bbase + rb * STB;
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (
          [&] {
            W4_MF(I, FA, FB);
            if constexpr (I % W4B_RD_EVERY == W4B_RD_EVERY - 1 && I / W4B_RD_EVERY < 16) {
              constexpr int J = I / W4B_RD_EVERY;  // 0..15
              if constexpr (J < 8) rd<J * 1024>(NA[J], ra);
              else rd<(J - 8) * 1024>(NB[J - 8], rbb);
            }
            if constexpr (I % 8 == 3) dma(dkt, db, I / 8);
          }(),
          ...);
    }(std::make_integer_sequence<int, 64>{});
  };

  // prologue: K-tiles 0 .. NST-2 in flight; wait for 0; read its fragments
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
#pragma unroll
    for (int i = 0; i < 8; ++i) dma(s, s, i);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NST - 2)) : "memory");
  W4_BARRIER();
  [&]<int... J>(std::integer_sequence<int, J...>) {
    ((J < 8 ? rd<(J & 7) * 1024>(fa0[J & 7], abase) : rd<(J & 7) * 1024>(fb0[J & 7], bbase)), ...);
  }(std::make_integer_sequence<int, 16>{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // steady state, two K-tiles per iteration (register double buffer): before K-tile kt, this wave's DMA of
  // K-tile kt+1 has landed (vmcnt(8): only kt+2's 8 pieces younger) and the barrier makes every wave's pieces
  // visible and retires all reads of buffer (kt+3)%4 (K-tile kt-1, read during kt-2).
  for (int kt = 0; kt < nk; kt += 2) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NST - 3)) : "memory");
    W4_BARRIER();
    ktile(fa0, fb0, fa1, fb1, (kt + 1) % NST, kt + NST - 1, (kt + NST - 1) % NST);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * (NST - 3)) : "memory");
    W4_BARRIER();
    ktile(fa1, fb1, fa0, fb0, (kt + 2) % NST, kt + NST, (kt + NST) % NST);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
#undef W4_MF

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

}  // namespace w4b

extern "C" int dllm_gemm_w4b(const void* A, long lda, const void* B, long ldb, void* C, long ldc, int M, int N, int K,
                             int group_m, void* stream) {
  using namespace w4b;
  if (M % BM || N % BN || K % (2 * BK) || K < NST * BK || lda % 8 || ldb % 8 || ldc % 8) return -1;
  if ((long)BM * lda * 2 >= (1L << 31) || (long)BN * ldb * 2 >= (1L << 31)) return -1;  // 32-bit piece offsets
  if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return -1;
  Args a{A, B, C, lda, ldb, ldc, M, N, K, group_m > 0 ? group_m : 4};
  hipLaunchKernelGGL(gemm_nt_w4b, dim3((M / BM) * (N / BN)), dim3(256), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
