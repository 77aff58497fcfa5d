#pragma once
// MFMA GEMMs for the FFN hot path on gfx950 (MI355X): kernels and launch templates.
//
// Included by the per-layout translation units (gemm_nt.hip, gemm_nn.hip, gemm_tn.hip), which instantiate
// the kernels of one operand layout each and compile in parallel, and by gemm.hip (the C ABI).
//
// Replaces the reference's ATen GEMMs + elementwise ops (train_ffns.py:41-52, K1-K8 in SURVEY §2.4):
//   fwd   h  = x  · W1ᵀ  (NT)  -> epilogue act (ReLU/SiLU/GELU) [+ store h]        K1+K2
//         y  = a  · W2ᵀ  (NT)                                                        K3
//   dgrad da = dy · W2   (NN)  -> epilogue · act'(h)                                  K5+K6
//         dx = da · W1   (NN)                                                        K8
//   wgrad dW = dyᵀ· a    (TN)  -> fp32 (or bf16) out, optional beta-accumulate       K4, K7
//
// Layouts (all row-major storage):  NT: A[M][K], B[N][K]   NN: A[M][K], B[K][N]   TN: A[K][M], B[K][N]
//
// Kernel families:
//  * gemm_bf16_256: 256x256x64 tile, 512 threads (8 waves as 2(M) x 4(N), 128x64 per wave),
//    mfma_f32_16x16x32_bf16, both operands staged HBM->LDS by LDS-DMA (global_load_lds_dwordx4,
//    16 B/lane) into a 2-stage ring (128 KiB LDS, 1 block/CU).  K-contiguous operand tiles are
//    [256 rows][64 k] with the 16-B chunk index XOR-swizzled by (row>>1)&7, read by ds_read_b128
//    conflict-free; MN-contiguous operand tiles are [64 k][256 mn] with 32-B units XOR-swizzled by
//    (k&3)|((k>>3)&1)<<2, read transposed by ds_read_b64_tr_b16 conflict-free.  The swizzle is applied
//    on the per-lane global SOURCE address (the LDS image of an LDS-DMA is lane-linear, guide rule 21).
//    Operands are swapped in the MFMA (B-fragment first) so each lane ends with 4 consecutive output
//    columns -> 8-B (bf16) / 16-B (fp32) epilogue stores.  XCD-aware bijective block remap + grouped
//    raster so blocks sharing operand panels run on one XCD's L2.
//  * gemm_f32_128: exact-fp32 parity path (mfma_f32_16x16x4f32), 128x128x16 tile, register-staged.
//  * gemm_generic: any shape / any dtype, bounds-checked FMA kernel (tests, odd TP shards).
#include <algorithm>
#include <type_traits>

// MFMA-cluster wave priority of the 8-phase kernel (build-time experiment knob): 0 = s_setprio(1) around every
// MFMA cluster (default), 1 = static prio 1 for waves 4-7 only, 2 = none
#ifndef DLLM_PRIO_MODE
#define DLLM_PRIO_MODE 0
#endif
// fp32 path: the 256x256x32 LDS-DMA kernel where shapes allow (1), or always the 128x128 kernel (0)
#ifndef DLLM_ADAM_PIPE
#define DLLM_ADAM_PIPE 1  // fused-AdamW epilogue: row groups per batch, the next batch's master / moment loads issued
                          // before this batch's stores (0 = sequential batches; profiles/r2/epilogue_pipe_experiment_r2.log)
#endif
#ifndef DLLM_BPRE
#define DLLM_BPRE 1  // 8-phase kernel: each K-tile's B-half 0 read one phase early (balanced read segments)
#endif
#ifndef DLLM_EPI_PF
#define DLLM_EPI_PF 0  // 1: 8-phase kernels prefetch the epilogue's load operands (fused-optimizer master / moment planes,
                       // ReLU dgrad mask, SwiGLU dgrad pre-activations) by counted LDS-DMA in every main-loop iteration.
                       // Bitwise equal, spill-free -- and slower: the main loop pays more than the epilogue saves
                       // (fused-SGD weight gradient 855 vs 770 us, step 36.2 vs 34.5 ms; profiles/r6/epilogue_prefetch_r6.txt)
#endif
#ifndef DLLM_EPI_PF_LEAD
#define DLLM_EPI_PF_LEAD 8  // at least this many main-loop iterations (2 K-tiles each) of lead for the first prefetch
#endif
#ifndef DLLM_EPI_SKIP
#define DLLM_EPI_SKIP 0  // diagnostic only: the 8-phase kernels skip their epilogue (wrong results; prices it)
#endif
#ifndef DLLM_F32_256
#define DLLM_F32_256 1
#endif
// transposed-map fused AdamW (EPI_ADAMS_T): persistent blocks (1) or one tile per block (0, as the other AdamW epilogues)
#ifndef DLLM_ADAMS_T_PERS
#define DLLM_ADAMS_T_PERS 0
#endif

#include "common.h"

namespace dllm {

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const void* aux;   // EPI_DACT/EPI_DGLU: pre-activation (h) input
  void* aux_out;     // EPI_ACT/EPI_GLU: pre-activation store (nullable)
  long lda, ldb, ldc, ldaux;
  int M, N, K;
  float alpha, beta;
  int act;
  int group_m;
  // fused optimizer epilogues
  float lr, b1, b2, eps, wd, bc1, bc2;
  float* opt_m;
  float* opt_v;
  // split-K: ksplit > 1 -> the main kernel writes fp32 partials C + split*M*ldc (C = workspace)
  int ksplit;
  // tiles per block of a persistent 8-phase kernel (PERS instantiations only; set by grid_8ph)
  int tpb;
  // per-call launch policy (no process-wide kernel state: concurrent GEMMs on different streams may differ)
  int variant;   // bf16 main loop: 0 auto, 1 2-stage, 2 8-phase, 3 8-phase staggered, 4 4-phase staggered
  int tpb_req;   // requested tiles per persistent block (<= 1: one block per tile)
  int min_bpc;   // minimum blocks per CU of a persistent grid (2 when collectives overlap the GEMMs)
  float* ws;     // split-K fp32 partial workspace (caller-owned, ksplit * M * N floats)
  // ReLU activation-gradient bitmask (nullable; 8-phase kernels, bf16 out, compile-time ReLU): EPI_ACT writes
  // bit (act(h) != 0) per output element, EPI_DACT reads it instead of aux.  Tile-native layout: 8 KiB per
  // 256x256 tile (tile = tm * tiles_n + tn), 16 B per thread -- the same element->lane map in both GEMMs.
  void* mask;
  // gemm_bf16_pp: initial delay (x 64 clocks) of the odd workgroup slot of each CU, so the two co-resident blocks
  // start out of phase (experiment knob, DLLM_PP_SKEW; 0 = none)
  int skew;
};

// ----------------------------------------------------------------------------------------------
// epilogue helpers (shared by all kernel families)
// ----------------------------------------------------------------------------------------------
template <typename T> struct Vec4;
template <> struct Vec4<uint16_t> {
  static __device__ __forceinline__ f32x4_t load(const void* base, long idx) {
    uint2 u = *(const uint2*)((const uint16_t*)base + idx);
    f32x4_t r;
    r[0] = bf2f(u.x & 0xffff); r[1] = bf2f(u.x >> 16);
    r[2] = bf2f(u.y & 0xffff); r[3] = bf2f(u.y >> 16);
    return r;
  }
  static __device__ __forceinline__ void store(void* base, long idx, f32x4_t v) {
    uint2 u;
    u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *(uint2*)((uint16_t*)base + idx) = u;
  }
};
template <> struct Vec4<float> {
  static __device__ __forceinline__ f32x4_t load(const void* base, long idx) {
    return *(const f32x4_t*)((const float*)base + idx);
  }
  static __device__ __forceinline__ void store(void* base, long idx, f32x4_t v) {
    *(f32x4_t*)((float*)base + idx) = v;
  }
};

template <typename T> __device__ __forceinline__ float ld1(const void* b, long i);
template <> __device__ __forceinline__ float ld1<uint16_t>(const void* b, long i) {
  return bf2f(((const uint16_t*)b)[i]);
}
template <> __device__ __forceinline__ float ld1<float>(const void* b, long i) {
  return ((const float*)b)[i];
}
template <typename T> __device__ __forceinline__ void st1(void* b, long i, float v);
template <> __device__ __forceinline__ void st1<uint16_t>(void* b, long i, float v) {
  ((uint16_t*)b)[i] = f2bf(v);
}
template <> __device__ __forceinline__ void st1<float>(void* b, long i, float v) {
  ((float*)b)[i] = v;
}

// Apply the epilogue to 4 consecutive output columns (m, n..n+3) held by one lane.
// For EPI_GLU / EPI_DGLU the column index n is in the "interleaved" space: 16-column blocks alternate
// between the gate (W1, even blocks) and the up projection (W3, odd blocks); a lane's 4 columns and
// the matching 4 columns 16 further lie in the SAME lane of the neighbouring n-tile, so the pairs are
// combined by the caller (see epi_glu_pair).
template <int ACT> __device__ __forceinline__ float actf(int rt, float x) { return act_fwd(ACT < 0 ? rt : ACT, x); }
template <int ACT> __device__ __forceinline__ float actg(int rt, float x) { return act_grad(ACT < 0 ? rt : ACT, x); }

template <int EPI, typename OutT, int ACT = -1>
__device__ __forceinline__ void epi4(const GemmArgs& p, int m, int n, f32x4_t v) {
  const long ci = (long)m * p.ldc + n;
  if constexpr (EPI == EPI_STORE) {
    v *= p.alpha;
    if (p.beta != 0.f) v += p.beta * Vec4<OutT>::load(p.C, ci);
    Vec4<OutT>::store(p.C, ci, v);
  } else if constexpr (EPI == EPI_ACT) {
    if (p.aux_out) Vec4<OutT>::store(p.aux_out, (long)m * p.ldaux + n, v);
    f32x4_t a;
    for (int r = 0; r < 4; ++r) a[r] = actf<ACT>(p.act, v[r]);
    Vec4<OutT>::store(p.C, ci, a);
  } else if constexpr (EPI == EPI_DACT) {
    f32x4_t h = Vec4<OutT>::load(p.aux, (long)m * p.ldaux + n);
    for (int r = 0; r < 4; ++r) v[r] *= actg<ACT>(p.act, h[r]);
    Vec4<OutT>::store(p.C, ci, v);
  } else if constexpr (EPI == EPI_SGD) {
    f32x4_t w = Vec4<float>::load(p.C, ci);
    for (int r = 0; r < 4; ++r) w[r] = __fadd_rn(w[r], __fmul_rn(-p.lr, __fmul_rn(p.alpha, v[r])));
    Vec4<float>::store(p.C, ci, w);
    if (p.aux_out) Vec4<uint16_t>::store(p.aux_out, (long)m * p.ldaux + n, w);
  } else if constexpr (EPI == EPI_SGDS) {
    uint2* hp = (uint2*)((uint16_t*)p.aux_out + (long)m * p.ldaux + n);
    uint2* lp = (uint2*)((uint16_t*)p.C + ci);
    uint2 h = *hp, l = *lp;
    float w[4];
    split_join2(h.x, l.x, w[0], w[1]);
    split_join2(h.y, l.y, w[2], w[3]);
    for (int r = 0; r < 4; ++r) w[r] = __fadd_rn(w[r], __fmul_rn(-p.lr, __fmul_rn(p.alpha, v[r])));
    split_part2(w[0], w[1], h.x, l.x);
    split_part2(w[2], w[3], h.y, l.y);
    *hp = h;
    *lp = l;
  } else if constexpr (EPI == EPI_ADAMS) {
    uint2* hp = (uint2*)((uint16_t*)p.aux_out + (long)m * p.ldaux + n);
    uint2* lp = (uint2*)((uint16_t*)p.C + ci);
    uint2 h = *hp, l = *lp;
    f32x4_t mm = Vec4<float>::load(p.opt_m, ci), vv = Vec4<float>::load(p.opt_v, ci);
    float w[4];
    split_join2(h.x, l.x, w[0], w[1]);
    split_join2(h.y, l.y, w[2], w[3]);
    for (int r = 0; r < 4; ++r) {
      float m1 = mm[r], v1 = vv[r];
      adamw1(w[r], m1, v1, p.alpha * v[r], p.lr, p.b1, p.b2, p.eps, p.wd, p.bc1, p.bc2);
      mm[r] = m1;
      vv[r] = v1;
    }
    split_part2(w[0], w[1], h.x, l.x);
    split_part2(w[2], w[3], h.y, l.y);
    *hp = h;
    *lp = l;
    Vec4<float>::store(p.opt_m, ci, mm);
    Vec4<float>::store(p.opt_v, ci, vv);
  } else if constexpr (EPI == EPI_ADAM) {
    f32x4_t w = Vec4<float>::load(p.C, ci);
    f32x4_t mm = Vec4<float>::load(p.opt_m, ci);
    f32x4_t vv = Vec4<float>::load(p.opt_v, ci);
    for (int r = 0; r < 4; ++r) {
      const float g = p.alpha * v[r];
      mm[r] = p.b1 * mm[r] + (1.f - p.b1) * g;
      vv[r] = p.b2 * vv[r] + (1.f - p.b2) * g * g;
      const float mh = mm[r] / p.bc1, vh = vv[r] / p.bc2;
      w[r] = w[r] - p.lr * (mh / (sqrtf(vh) + p.eps) + p.wd * w[r]);
    }
    Vec4<float>::store(p.C, ci, w);
    Vec4<float>::store(p.opt_m, ci, mm);
    Vec4<float>::store(p.opt_v, ci, vv);
    if (p.aux_out) Vec4<uint16_t>::store(p.aux_out, (long)m * p.ldaux + n, w);
  }
}

// Gated (SwiGLU-style) pair epilogues.  g = acc of the gate column block, u = acc of the up block.
// Output of EPI_GLU has N/2 columns (de-interleaved): a = act(g) * u.  aux_out keeps interleaved
// [g|u] pre-activations (N columns) for the backward.
// EPI_DGLU: acc = da (N/2 de-interleaved columns, the GEMM runs with N/2), aux = interleaved [g|u];
// output C is interleaved [dg|du] with N = 2*(GEMM N) columns.
template <typename OutT, int ACT = -1>
__device__ __forceinline__ void epi_glu_pair(const GemmArgs& p, int m, int nc_out, int ng, int nu,
                                             f32x4_t g, f32x4_t u) {
  if (p.aux_out) {
    Vec4<OutT>::store(p.aux_out, (long)m * p.ldaux + ng, g);
    Vec4<OutT>::store(p.aux_out, (long)m * p.ldaux + nu, u);
  }
  f32x4_t a;
  for (int r = 0; r < 4; ++r) a[r] = actf<ACT>(p.act, g[r]) * u[r];
  Vec4<OutT>::store(p.C, (long)m * p.ldc + nc_out, a);
}
template <typename OutT, int ACT = -1>
__device__ __forceinline__ void epi_dglu(const GemmArgs& p, int m, int n_da, f32x4_t da) {
  // n_da indexes the de-interleaved F axis; interleaved column of the gate = (n/16)*32 + n%16
  const int blk = n_da >> 4, off = n_da & 15;
  const int ng = blk * 32 + off, nu = ng + 16;
  f32x4_t g = Vec4<OutT>::load(p.aux, (long)m * p.ldaux + ng);
  f32x4_t u = Vec4<OutT>::load(p.aux, (long)m * p.ldaux + nu);
  f32x4_t dg, du;
  for (int r = 0; r < 4; ++r) {
    du[r] = da[r] * actf<ACT>(p.act, g[r]);
    dg[r] = da[r] * u[r] * actg<ACT>(p.act, g[r]);
  }
  Vec4<OutT>::store(p.C, (long)m * p.ldc + ng, dg);
  Vec4<OutT>::store(p.C, (long)m * p.ldc + nu, du);
}

// ----------------------------------------------------------------------------------------------
// Batched epilogue of the 256x256 8-phase kernel.
//
// The per-element helpers above are fine for the elementwise split-K reduction, but inside the GEMM
// they serialise: hipcc cannot prove that a store to C (or aux_out) does not alias the NEXT group's
// load of C / aux, so every 4-column group became load -> s_waitcnt vmcnt(0) -> math -> store, i.e.
// 32 exposed HBM round trips per tile (measured: +105 us on a 1.1-TFLOP fused-SGD wgrad, +110 us on
// the act'-masked dgrad).  Here each wave issues all loads of a batch of row groups first (batch size
// chosen to keep <= 64 extra VGPRs live next to the 128 accumulators), then the math and stores, so a
// tile pays 1-8 round trips.  Optional side outputs (aux_out) are written under ONE uniform branch per
// batch.  ACT >= 0 selects the activation at compile time (no per-element switch: the runtime-switch
// build of the act epilogue was ~14k instructions, larger than the instruction cache).
// ----------------------------------------------------------------------------------------------

template <typename T> struct Raw4;
template <> struct Raw4<uint16_t> {
  using type = uint2;
  static __device__ __forceinline__ type load(const void* b, long i) { return *(const uint2*)((const uint16_t*)b + i); }
  static __device__ __forceinline__ f32x4_t cvt(type u) {
    return f32x4_t{bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16)};
  }
};
template <> struct Raw4<float> {
  using type = f32x4_t;
  static __device__ __forceinline__ type load(const void* b, long i) { return *(const f32x4_t*)((const float*)b + i); }
  static __device__ __forceinline__ f32x4_t cvt(type u) { return u; }
};

// row groups per batch for `cost` extra VGPRs per row group (<= 64 extra live VGPRs)
constexpr int epi_batch(int cost) {
  return cost == 0 ? 16 : (64 / cost >= 16 ? 16 : 64 / cost >= 8 ? 8 : 64 / cost >= 4 ? 4 : 64 / cost >= 2 ? 2 : 1);
}

// Paired 16-B bf16 access (guide T21 pattern, with v_permlane16_swap): a lane's 4 columns of the
// nt = 0 fragment (a) and of the nt = 1 fragment (b) of one row are exchanged with the lane 16 away so
// that lanes 16g..16g+15 hold 8 contiguous columns at pair_col(lane) = 16*(g&1) + 8*(g>>1) of the
// 32-column wave strip.  One dwordx4 store replaces two dwordx2 (the epilogue store tail is
// issue-bound); loads use the same map and the inverse (identical) exchange.
__device__ __forceinline__ int pair_col(int lane) { return 16 * ((lane >> 4) & 1) + 8 * (lane >> 5); }
__device__ __forceinline__ uint2 pk_bf16(f32x4_t v) {
  return uint2{(uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16), (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)};
}
__device__ __forceinline__ uint4 pair_swap(uint2 a, uint2 b) {
  const auto x = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
  const auto y = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
  return uint4{x[0], y[0], x[1], y[1]};
}
__device__ __forceinline__ void st_pair_bf16(void* base, long idx, f32x4_t a, f32x4_t b) {
  *(uint4*)((uint16_t*)base + idx) = pair_swap(pk_bf16(a), pk_bf16(b));
}
__device__ __forceinline__ void unpair_bf16(uint4 v, f32x4_t& a, f32x4_t& b) {
  const uint4 u = pair_swap(uint2{v.x, v.y}, uint2{v.z, v.w});
  a = Raw4<uint16_t>::cvt(uint2{u.x, u.y});
  b = Raw4<uint16_t>::cvt(uint2{u.z, u.w});
}

// 4x4 transpose across the lanes of a quad (lanes 4j .. 4j+3, element e = column): lane 4j + i returns column i,
// i.e. element e = the input element i of lane 4j + e.  Two xor exchanges (DPP quad_perm, no LDS): off-diagonal 2x2
// blocks between lanes i, i^2, then single elements between lanes i, i^1.  EXEC must be full (the epilogues are).
template <int CTRL> __device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ f32x4_t quad_transpose(f32x4_t v, int lane) {
  constexpr int XOR2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // quad_perm [2, 3, 0, 1]
  constexpr int XOR1 = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // quad_perm [1, 0, 3, 2]
  const bool hi = lane & 2, lo = lane & 1;
  const float d0 = dpp_f<XOR2>(v[0]), d1 = dpp_f<XOR2>(v[1]), d2 = dpp_f<XOR2>(v[2]), d3 = dpp_f<XOR2>(v[3]);
  const f32x4_t t{hi ? d2 : v[0], hi ? d3 : v[1], hi ? v[2] : d0, hi ? v[3] : d1};
  const float u0 = dpp_f<XOR1>(t[0]), u1 = dpp_f<XOR1>(t[1]), u2 = dpp_f<XOR1>(t[2]), u3 = dpp_f<XOR1>(t[3]);
  return f32x4_t{lo ? u1 : t[0], lo ? t[1] : u0, lo ? u3 : t[2], lo ? t[3] : u2};
}
// Pairs two quad-transposed fragments 16 rows apart (x: rows 4j..4j+3 of the first, y: of the second, packed bf16)
// across lanes 4 apart (DPP row_shl:4 / row_shr:4 inside each 16-lane row): lanes with j = (lane>>2)&3 even return the
// first fragment's rows 4j .. 4j+7, odd ones the second fragment's rows 4(j-1) .. 4(j-1)+7 -- 8 consecutive rows each.
__device__ __forceinline__ uint4 tpair_bf16(uint2 x, uint2 y, int lane) {
  const uint32_t x0 = __builtin_amdgcn_update_dpp(0, (int)x.x, 0x104, 0xf, 0xf, false);  // row_shl:4: lane + 4
  const uint32_t x1 = __builtin_amdgcn_update_dpp(0, (int)x.y, 0x104, 0xf, 0xf, false);
  const uint32_t y0 = __builtin_amdgcn_update_dpp(0, (int)y.x, 0x114, 0xf, 0xf, false);  // row_shr:4: lane - 4
  const uint32_t y1 = __builtin_amdgcn_update_dpp(0, (int)y.y, 0x114, 0xf, 0xf, false);
  return (lane & 4) ? uint4{y0, y1, y.x, y.y} : uint4{x.x, x.y, x0, x1};
}

// acc[QM][QN][mt][nt]: lane holds C[m0 + QM*128 + wr*64 + mt*16 + (lane&15)][n0 + QN*QNS + wc*32 + nt*16 + 4*(lane>>4) + 0..3]
// row group rg = QM*8 + QN*4 + mt (16 per wave), 2 column groups (nt) each.  QNS = quadrant width: 128 for the
// 256x256 tile (8 waves, wc 0..3), 64 for the 256x128 tile of gemm_bf16_pp (4 waves, wc 0..1).
// BM = 224 (gemm_8ph_body): the second row half has 3 row fragments per wave, at rows 128 + wr*48 + mt*16; row
// groups with QM = 1, mt = 3 do not exist (DLLM_OK).
// RBCAP caps the epilogue's row-group batch (the persistent fp32-master SGD kernel: its 8-group batch of master
// planes on top of the main loop's live state needed 3 scratch dwords; utils/kernel_resources.py)
template <int EPI, typename OutT, int ACT, int QNS = 128, int BM = 256, int RBCAP = 16>
__device__ __forceinline__ void epilogue_256(const GemmArgs& p, f32x4_t (&acc)[2][2][4][2], int m0, int n0,
                                             int wr, int wc, int lane, void* Cp) {
  static_assert(BM == 256 || (QNS == 128 && EPI != EPI_GLU && EPI != EPI_DGLU), "224-row tiles: no gated epilogues");
  static_assert(!(epi_tout(EPI) || EPI == EPI_STORE_DT) || (BM == 256 && QNS == 128), "transposed outputs: 256x256");
  if constexpr (ACT < 0 && (EPI == EPI_ACT || EPI == EPI_DACT || EPI == EPI_GLU || EPI == EPI_DGLU)) {
    // Runtime activation (the fallback / non-default-variant kernels): branch once per tile into a compile-time body.
    // A per-element switch inside the unrolled row-group loops made hipcc keep the accumulators in a 512-B scratch
    // array indexed at run time (every runtime-activation DGLU kernel spilled 528 B; utils/kernel_resources.py).
    switch (p.act) {
      case ACT_RELU: epilogue_256<EPI, OutT, ACT_RELU, QNS, BM, RBCAP>(p, acc, m0, n0, wr, wc, lane, Cp); return;
      case ACT_SILU: epilogue_256<EPI, OutT, ACT_SILU, QNS, BM, RBCAP>(p, acc, m0, n0, wr, wc, lane, Cp); return;
      case ACT_GELU: epilogue_256<EPI, OutT, ACT_GELU, QNS, BM, RBCAP>(p, acc, m0, n0, wr, wc, lane, Cp); return;
      default: epilogue_256<EPI, OutT, ACT_NONE, QNS, BM, RBCAP>(p, acc, m0, n0, wr, wc, lane, Cp); return;
    }
  }
  constexpr int NWC = QNS / 32;       // waves per tile row
  constexpr int TW = 2 * QNS;         // tile width
  constexpr int MASK_WAVES = 2 * NWC; // waves per tile: the ReLU mask holds 16 B per lane and wave
  constexpr bool BF = std::is_same<OutT, uint16_t>::value;
  using R = Raw4<OutT>;
  using RT = typename std::conditional<BF, uint4, f32x4_t>::type;  // bf16: one paired 16-B load per row group
  using RF = Raw4<float>;
  constexpr int WR = BF ? 4 : 8;  // VGPRs per row group and loaded operand
  // (the beta != 0 store path is off the FFN hot path: small batches keep the persistent kernel's
  // in-loop epilogue within the register budget)
  constexpr int COST = EPI == EPI_DACT ? WR : EPI == EPI_DGLU ? 8 * (BF ? 2 : 4)
                     : EPI == EPI_STORE || EPI == EPI_STORE_T || EPI == EPI_STORE_DT ? 4 * WR
                     : EPI == EPI_SGD || EPI == EPI_SGDS || EPI == EPI_SGDS_T ? 8
                     : EPI == EPI_ADAM || EPI == EPI_ADAMS || EPI == EPI_ADAMS_T ? 24 : 0;
  constexpr int RB = epi_batch(COST) < RBCAP ? epi_batch(COST) : RBCAP;
  const int pc = pair_col(lane);
#define DLLM_M(rg) (m0 + ((rg) >> 3) * 128 + wr * ((BM != 256 && ((rg) >> 3)) ? 48 : 64) + ((rg) & 3) * 16 + (lane & 15))
#define DLLM_OK(rg) (BM == 256 || ((rg) >> 3) == 0 || ((rg) & 3) != 3)
#define DLLM_NB(rg) (n0 + (((rg) >> 2) & 1) * QNS + wc * 32)
#define DLLM_N(rg, nt) (DLLM_NB(rg) + (nt) * 16 + 4 * (lane >> 4))
#define DLLM_ACC(rg, nt) acc[(rg) >> 3][((rg) >> 2) & 1][(rg) & 3][nt]
  // Transposed outputs (epi_tout: MFMA operands swapped in the main loop): lane holds
  // C[m0 + QM*128 + wr*64 + mt*16 + 4*(lane>>4) + e][n0 + QN*QNS + wc*32 + nt*16 + (lane&15)], written to Cᵀ [N][M].
  // Row group rg = (QM, QN, nt, p) is output row n = ...(lane&15) and pairs fragments mt = 2p, 2p+1 (32 consecutive
  // m), exactly as the normal layout pairs nt = 0, 1 -- so the paired 16-B accesses below serve both.
  constexpr bool TRO = epi_tout(EPI);
  auto row_of = [&](int rg) -> int {
    if constexpr (TRO) return n0 + ((rg >> 2) & 1) * QNS + wc * 32 + ((rg >> 1) & 1) * 16 + (lane & 15);
    else return DLLM_M(rg);
  };
  auto colb_of = [&](int rg) -> int {
    if constexpr (TRO) return m0 + (rg >> 3) * 128 + wr * 64 + (rg & 1) * 32;
    else return DLLM_NB(rg);
  };
  auto acc_of = [&](int rg, int h) -> f32x4_t {
    if constexpr (TRO) return acc[rg >> 3][(rg >> 2) & 1][2 * (rg & 1) + h][(rg >> 1) & 1];
    else return DLLM_ACC(rg, h);
  };
  // store the row group's two fragments (already epilogue-transformed) to a [*, ld] OutT matrix
  auto store_rg = [&](void* base, long ld, int m, int nb, f32x4_t a, f32x4_t b) {
    if constexpr (BF) {
      st_pair_bf16(base, (long)m * ld + nb + pc, a, b);
    } else {
      Vec4<float>::store(base, (long)m * ld + nb + 4 * (lane >> 4), a);
      Vec4<float>::store(base, (long)m * ld + nb + 16 + 4 * (lane >> 4), b);
    }
  };
  // load the row group's two fragments (raw) / decode them
  auto load_rg = [&](const void* base, long ld, int m, int nb, RT (&dst)[2]) {
    if constexpr (BF) {
      dst[0] = *(const uint4*)((const uint16_t*)base + (long)m * ld + nb + pc);
    } else {
      dst[0] = RF::load(base, (long)m * ld + nb + 4 * (lane >> 4));
      dst[1] = RF::load(base, (long)m * ld + nb + 16 + 4 * (lane >> 4));
    }
  };
  auto decode_rg = [&](const RT (&src)[2], f32x4_t& a, f32x4_t& b) {
    if constexpr (BF) unpair_bf16(src[0], a, b);
    else { a = src[0]; b = src[1]; }
  };
  if constexpr (EPI == EPI_STORE_T) {
#pragma unroll
    for (int rg = 0; rg < 16; ++rg)
      store_rg(Cp, p.ldc, row_of(rg), colb_of(rg), acc_of(rg, 0) * p.alpha, acc_of(rg, 1) * p.alpha);
  } else if constexpr (EPI == EPI_STORE_DT) {
    // C as EPI_STORE, then Cᵀ [N][M] into aux_out: per fragment a quad transpose gives lane 4j + i the 4 rows
    // m = mb + 4j .. 4j+3 of column n = nb + nt*16 + 4*(lane>>4) + i -> one 8-B store into row n of Cᵀ
    static_assert(BF, "transposed copy: bf16 output");
    // C as EPI_STORE; then Cᵀ [N][M] into aux_out.  Per fragment a quad transpose gives lane 4j + i the 4 rows
    // m = 4j .. 4j+3 (of the fragment's 16) of column n = nb + nt*16 + 4*(lane>>4) + i; the fragments of row groups
    // rg, rg+1 (rows 16 apart) are then paired across lanes 4 apart (tpair_bf16), so each lane stores 8 consecutive
    // m -- one 16-B store per lane covering 16 rows of Cᵀ x 64 contiguous bytes, the shape of the paired row store
    const int j4 = (lane >> 2) & 3;
    const int mq = 16 * (j4 & 1) + 4 * (j4 & 2) - (lane & 15);  // DLLM_M(rg) + mq = the lane's first row
    const int nq = 4 * (lane >> 4) + (lane & 3);
#pragma unroll
    for (int rg = 0; rg < 16; rg += 2) {
      const f32x4_t a00 = DLLM_ACC(rg, 0) * p.alpha, a01 = DLLM_ACC(rg, 1) * p.alpha;
      const f32x4_t a10 = DLLM_ACC(rg + 1, 0) * p.alpha, a11 = DLLM_ACC(rg + 1, 1) * p.alpha;
      store_rg(Cp, p.ldc, DLLM_M(rg), DLLM_NB(rg), a00, a01);
      store_rg(Cp, p.ldc, DLLM_M(rg + 1), DLLM_NB(rg + 1), a10, a11);
      uint16_t* tb = (uint16_t*)p.aux_out + (long)(DLLM_NB(rg) + nq) * p.ldaux + DLLM_M(rg) + mq;
      *(uint4*)tb = tpair_bf16(pk_bf16(quad_transpose(a00, lane)), pk_bf16(quad_transpose(a10, lane)), lane);
      *(uint4*)(tb + 16 * p.ldaux) =
          tpair_bf16(pk_bf16(quad_transpose(a01, lane)), pk_bf16(quad_transpose(a11, lane)), lane);
    }
  } else if constexpr (EPI == EPI_STORE) {
    if (p.beta == 0.f) {
#pragma unroll
      for (int rg = 0; rg < 16; ++rg)
        if (DLLM_OK(rg))
          store_rg(Cp, p.ldc, DLLM_M(rg), DLLM_NB(rg), DLLM_ACC(rg, 0) * p.alpha, DLLM_ACC(rg, 1) * p.alpha);
    } else {
#pragma unroll
      for (int b0 = 0; b0 < 16; b0 += RB) {
        RT L[RB][2];
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (DLLM_OK(b0 + r)) load_rg(Cp, p.ldc, DLLM_M(b0 + r), DLLM_NB(b0 + r), L[r]);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          if (!DLLM_OK(b0 + r)) continue;
          f32x4_t c0, c1;
          decode_rg(L[r], c0, c1);
          store_rg(Cp, p.ldc, DLLM_M(b0 + r), DLLM_NB(b0 + r), DLLM_ACC(b0 + r, 0) * p.alpha + p.beta * c0,
                   DLLM_ACC(b0 + r, 1) * p.alpha + p.beta * c1);
        }
      }
    }
  } else if constexpr (EPI == EPI_ACT) {
    if (p.aux_out) {
#pragma unroll
      for (int rg = 0; rg < 16; ++rg)
        if (DLLM_OK(rg)) store_rg(p.aux_out, p.ldaux, DLLM_M(rg), DLLM_NB(rg), DLLM_ACC(rg, 0), DLLM_ACC(rg, 1));
    }
    if constexpr (ACT == ACT_RELU && BF) {
      // optional mask: bit rg*8 + nt*4 + e of this thread's 128 = (stored bf16 activation != 0), i.e. exactly
      // the act'(h) the unmasked dgrad derives from the stored activation; one dword per 4 row groups
      const bool mk = p.mask != nullptr;
      const long tile = (long)(m0 / BM) * (p.N / TW) + n0 / TW;  // BM x TW tiles
      uint32_t* mw = (uint32_t*)p.mask + (tile * (MASK_WAVES * 64) + (wr * NWC + wc) * 64 + lane) * 4;
      uint32_t w = 0u;
#pragma unroll
      for (int rg = 0; rg < 16; ++rg) {
        if (!DLLM_OK(rg)) {  // 224-row tile: no such row group; still flush its mask word
          if (mk && (rg & 3) == 3) {
            mw[rg >> 2] = w;
            w = 0u;
          }
          continue;
        }
        f32x4_t a = DLLM_ACC(rg, 0), b = DLLM_ACC(rg, 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = actf<ACT>(p.act, a[e]);
          b[e] = actf<ACT>(p.act, b[e]);
        }
        const uint2 ua = pk_bf16(a), ub = pk_bf16(b);
        *(uint4*)((uint16_t*)Cp + (long)DLLM_M(rg) * p.ldc + DLLM_NB(rg) + pc) = pair_swap(ua, ub);
        if (mk) {
          const uint32_t bits = ((ua.x & 0xffffu) != 0u) | (((ua.x >> 16) != 0u) << 1) |
                                (((ua.y & 0xffffu) != 0u) << 2) | (((ua.y >> 16) != 0u) << 3) |
                                (((ub.x & 0xffffu) != 0u) << 4) | (((ub.x >> 16) != 0u) << 5) |
                                (((ub.y & 0xffffu) != 0u) << 6) | (((ub.y >> 16) != 0u) << 7);
          w |= bits << ((rg & 3) * 8);
          if ((rg & 3) == 3) {
            mw[rg >> 2] = w;
            w = 0u;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      if (!DLLM_OK(rg)) continue;
      f32x4_t a = DLLM_ACC(rg, 0), b = DLLM_ACC(rg, 1);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[e] = actf<ACT>(p.act, a[e]);
        b[e] = actf<ACT>(p.act, b[e]);
      }
      store_rg(Cp, p.ldc, DLLM_M(rg), DLLM_NB(rg), a, b);
    }
  } else if constexpr (EPI == EPI_DACT) {
    if constexpr (ACT == ACT_RELU && BF) {
      if (p.mask) {
        const long tile = (long)(m0 / BM) * (p.N / TW) + n0 / TW;  // BM x TW tiles
        const uint4 mv = ((const uint4*)p.mask)[tile * (MASK_WAVES * 64) + (wr * NWC + wc) * 64 + lane];
        const uint32_t w[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
        for (int rg = 0; rg < 16; ++rg) {
          if (!DLLM_OK(rg)) continue;
          const uint32_t bits = w[rg >> 2] >> ((rg & 3) * 8);
          f32x4_t a = DLLM_ACC(rg, 0), b = DLLM_ACC(rg, 1);
#pragma unroll
          for (int e = 0; e < 4; ++e) {  // multiply (not select): same -0 / NaN as the unmasked path
            a[e] *= ((bits >> e) & 1u) ? 1.f : 0.f;
            b[e] *= ((bits >> (4 + e)) & 1u) ? 1.f : 0.f;
          }
          store_rg(Cp, p.ldc, DLLM_M(rg), DLLM_NB(rg), a, b);
        }
        return;
      }
    }
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      RT H[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r)
        if (DLLM_OK(b0 + r)) load_rg(p.aux, p.ldaux, DLLM_M(b0 + r), DLLM_NB(b0 + r), H[r]);
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!DLLM_OK(b0 + r)) continue;
        f32x4_t h0, h1;
        decode_rg(H[r], h0, h1);
        f32x4_t a = DLLM_ACC(b0 + r, 0), b = DLLM_ACC(b0 + r, 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] *= actg<ACT>(p.act, h0[e]);
          b[e] *= actg<ACT>(p.act, h1[e]);
        }
        store_rg(Cp, p.ldc, DLLM_M(b0 + r), DLLM_NB(b0 + r), a, b);
      }
    }
  } else if constexpr (EPI == EPI_GLU) {
    // gate / up 16-column blocks alternate: nt = 0 gate, nt = 1 up (same lane)
    if (p.aux_out) {
#pragma unroll
      for (int rg = 0; rg < 16; ++rg)
        store_rg(p.aux_out, p.ldaux, DLLM_M(rg), DLLM_NB(rg), DLLM_ACC(rg, 0), DLLM_ACC(rg, 1));
    }
#pragma unroll
    for (int rg = 0; rg < 16; ++rg) {
      const int nb = DLLM_N(rg, 0);
      const f32x4_t g = DLLM_ACC(rg, 0), u = DLLM_ACC(rg, 1);
      f32x4_t a;
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] = actf<ACT>(p.act, g[e]) * u[e];
      Vec4<OutT>::store(Cp, (long)DLLM_M(rg) * p.ldc + (nb >> 5) * 16 + (nb & 15), a);
    }
  } else if constexpr (EPI == EPI_DGLU && BF) {
    // acc = da over the de-interleaved F axis; aux / C interleaved [g|u] 16-column blocks.  A 32-column
    // interleaved strip [g (16) | u (16)] has exactly the paired-access shape (nt = 0 columns -> g, nt = 1
    // columns -> u), so each row group is 2 paired 16-B loads + 2 paired 16-B stores per lane (16 rows x
    // 64 B per instruction) instead of 4 + 4 scattered 8-B accesses.
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      uint4 P[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          P[r][nt] = *(const uint4*)((const uint16_t*)p.aux + (long)DLLM_M(b0 + r) * p.ldaux + 2 * DLLM_NB(b0 + r) +
                                     32 * nt + pc);
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          f32x4_t g, u, dg, du;
          unpair_bf16(P[r][nt], g, u);
          const f32x4_t da = DLLM_ACC(b0 + r, nt);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            du[e] = da[e] * actf<ACT>(p.act, g[e]);
            dg[e] = da[e] * u[e] * actg<ACT>(p.act, g[e]);
          }
          st_pair_bf16(Cp, (long)DLLM_M(b0 + r) * p.ldc + 2 * DLLM_NB(b0 + r) + 32 * nt + pc, dg, du);
        }
    }
  } else if constexpr (EPI == EPI_DGLU) {
    // acc = da over the de-interleaved F axis; aux / C interleaved [g|u] 16-column blocks
    using RD = typename R::type;
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      RD G[RB][2], U[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int nd = DLLM_N(b0 + r, nt), ng = (nd >> 4) * 32 + (nd & 15);
          const long base = (long)DLLM_M(b0 + r) * p.ldaux + ng;
          G[r][nt] = R::load(p.aux, base);
          U[r][nt] = R::load(p.aux, base + 16);
        }
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const int nd = DLLM_N(b0 + r, nt), ng = (nd >> 4) * 32 + (nd & 15);
          const f32x4_t da = DLLM_ACC(b0 + r, nt), g = R::cvt(G[r][nt]), u = R::cvt(U[r][nt]);
          f32x4_t dg, du;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            du[e] = da[e] * actf<ACT>(p.act, g[e]);
            dg[e] = da[e] * u[e] * actg<ACT>(p.act, g[e]);
          }
          const long base = (long)DLLM_M(b0 + r) * p.ldc + ng;
          Vec4<OutT>::store(Cp, base, dg);
          Vec4<OutT>::store(Cp, base + 16, du);
        }
    }
  } else if constexpr (EPI == EPI_SGD) {
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      f32x4_t W[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          if (DLLM_OK(b0 + r)) W[r][nt] = RF::load(Cp, (long)DLLM_M(b0 + r) * p.ldc + DLLM_N(b0 + r, nt));
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          if (!DLLM_OK(b0 + r)) continue;
          const f32x4_t g = DLLM_ACC(b0 + r, nt);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            W[r][nt][e] = __fadd_rn(W[r][nt][e], __fmul_rn(-p.lr, __fmul_rn(p.alpha, g[e])));
          Vec4<float>::store(Cp, (long)DLLM_M(b0 + r) * p.ldc + DLLM_N(b0 + r, nt), W[r][nt]);
        }
      if (p.aux_out) {
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (DLLM_OK(b0 + r))
            st_pair_bf16(p.aux_out, (long)DLLM_M(b0 + r) * p.ldaux + DLLM_NB(b0 + r) + pc, W[r][0], W[r][1]);
      }
    }
  } else if constexpr (EPI == EPI_SGDS || EPI == EPI_SGDS_T) {
    // split master: hi plane = the bf16 working copy (aux_out), lo plane = the 16-bit residual (Cp), both in the
    // paired 16-B layout: per row group one 16-B load and one 16-B store per plane (4 B read + 4 B written per
    // parameter; the fp32 master form moves 4 B + 6 B in 5 accesses).  EPI_SGDS_T: the same on the transposed map
    // (row_of / colb_of / acc_of)
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      uint4 H[RB], Lw[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!DLLM_OK(b0 + r)) continue;
        H[r] = *(const uint4*)((const uint16_t*)p.aux_out + (long)row_of(b0 + r) * p.ldaux + colb_of(b0 + r) + pc);
        Lw[r] = *(const uint4*)((const uint16_t*)Cp + (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + pc);
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!DLLM_OK(b0 + r)) continue;
        // after the exchange: words 0-1 hold the nt = 0 fragment's 4 columns, words 2-3 the nt = 1 fragment's
        const uint4 h = pair_swap(uint2{H[r].x, H[r].y}, uint2{H[r].z, H[r].w});
        const uint4 l = pair_swap(uint2{Lw[r].x, Lw[r].y}, uint2{Lw[r].z, Lw[r].w});
        const f32x4_t g0 = acc_of(b0 + r, 0), g1 = acc_of(b0 + r, 1);
        uint32_t hw[4] = {h.x, h.y, h.z, h.w}, lw[4] = {l.x, l.y, l.z, l.w};
        const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float f0, f1;
          split_join2(hw[j], lw[j], f0, f1);
          f0 = __fadd_rn(f0, __fmul_rn(-p.lr, __fmul_rn(p.alpha, gg[2 * j])));
          f1 = __fadd_rn(f1, __fmul_rn(-p.lr, __fmul_rn(p.alpha, gg[2 * j + 1])));
          split_part2(f0, f1, hw[j], lw[j]);
        }
        *(uint4*)((uint16_t*)p.aux_out + (long)row_of(b0 + r) * p.ldaux + colb_of(b0 + r) + pc) =
            pair_swap(uint2{hw[0], hw[1]}, uint2{hw[2], hw[3]});
        *(uint4*)((uint16_t*)Cp + (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + pc) =
            pair_swap(uint2{lw[0], lw[1]}, uint2{lw[2], lw[3]});
      }
    }
  } else if constexpr (EPI == EPI_ADAMS || EPI == EPI_ADAMS_T) {
    // split master + fp32 moments: per row group one paired 16-B access per plane and two 16-B moment accesses per
    // fragment (24 B per parameter instead of 26 B).  EPI_ADAMS_T: the transposed map (row_of / colb_of / acc_of)
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      uint4 H[RB], Lw[RB];
      f32x4_t Mm[RB][2], Vv[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!DLLM_OK(b0 + r)) continue;
        H[r] = *(const uint4*)((const uint16_t*)p.aux_out + (long)row_of(b0 + r) * p.ldaux + colb_of(b0 + r) + pc);
        Lw[r] = *(const uint4*)((const uint16_t*)Cp + (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + pc);
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const long ci = (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + nt * 16 + 4 * (lane >> 4);
          Mm[r][nt] = RF::load(p.opt_m, ci);
          Vv[r][nt] = RF::load(p.opt_v, ci);
        }
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        if (!DLLM_OK(b0 + r)) continue;
        const uint4 h = pair_swap(uint2{H[r].x, H[r].y}, uint2{H[r].z, H[r].w});
        const uint4 l = pair_swap(uint2{Lw[r].x, Lw[r].y}, uint2{Lw[r].z, Lw[r].w});
        uint32_t hw[4] = {h.x, h.y, h.z, h.w}, lw[4] = {l.x, l.y, l.z, l.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int nt = j >> 1, e = 2 * (j & 1);
          const f32x4_t gg = acc_of(b0 + r, nt);
          float f0, f1;
          split_join2(hw[j], lw[j], f0, f1);
          float m0 = Mm[r][nt][e], v0 = Vv[r][nt][e], m1 = Mm[r][nt][e + 1], v1 = Vv[r][nt][e + 1];
          adamw1(f0, m0, v0, p.alpha * gg[e], p.lr, p.b1, p.b2, p.eps, p.wd, p.bc1, p.bc2);
          adamw1(f1, m1, v1, p.alpha * gg[e + 1], p.lr, p.b1, p.b2, p.eps, p.wd, p.bc1, p.bc2);
          Mm[r][nt][e] = m0;
          Vv[r][nt][e] = v0;
          Mm[r][nt][e + 1] = m1;
          Vv[r][nt][e + 1] = v1;
          split_part2(f0, f1, hw[j], lw[j]);
        }
        *(uint4*)((uint16_t*)p.aux_out + (long)row_of(b0 + r) * p.ldaux + colb_of(b0 + r) + pc) =
            pair_swap(uint2{hw[0], hw[1]}, uint2{hw[2], hw[3]});
        *(uint4*)((uint16_t*)Cp + (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + pc) =
            pair_swap(uint2{lw[0], lw[1]}, uint2{lw[2], lw[3]});
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const long ci = (long)row_of(b0 + r) * p.ldc + colb_of(b0 + r) + nt * 16 + 4 * (lane >> 4);
          Vec4<float>::store(p.opt_m, ci, Mm[r][nt]);
          Vec4<float>::store(p.opt_v, ci, Vv[r][nt]);
        }
      }
    }
  } else if constexpr (EPI == EPI_ADAM && DLLM_ADAM_PIPE) {
    // software-pipelined: batch b+1's master / moment loads are in flight while batch b is updated and stored, so a
    // wait for batch b's loads never also waits for the previous batch's stores (loads and stores share vmcnt)
    constexpr int SB = DLLM_ADAM_PIPE;
    f32x4_t W[2][SB][2], Mm[2][SB][2], Vv[2][SB][2];
    auto ld = [&](int b, int s) {
#pragma unroll
      for (int r = 0; r < SB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          if (!DLLM_OK(b * SB + r)) continue;
          const long ci = (long)DLLM_M(b * SB + r) * p.ldc + DLLM_N(b * SB + r, nt);
          W[s][r][nt] = RF::load(Cp, ci);
          Mm[s][r][nt] = RF::load(p.opt_m, ci);
          Vv[s][r][nt] = RF::load(p.opt_v, ci);
        }
    };
    ld(0, 0);
#pragma unroll
    for (int b = 0; b < 16 / SB; ++b) {
      if (b + 1 < 16 / SB) ld(b + 1, (b + 1) & 1);
      const int s = b & 1;
#pragma unroll
      for (int r = 0; r < SB; ++r) {
        if (!DLLM_OK(b * SB + r)) continue;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const f32x4_t gg = DLLM_ACC(b * SB + r, nt);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float g = p.alpha * gg[e];
            Mm[s][r][nt][e] = p.b1 * Mm[s][r][nt][e] + (1.f - p.b1) * g;
            Vv[s][r][nt][e] = p.b2 * Vv[s][r][nt][e] + (1.f - p.b2) * g * g;
            const float mh = Mm[s][r][nt][e] / p.bc1, vh = Vv[s][r][nt][e] / p.bc2;
            W[s][r][nt][e] = W[s][r][nt][e] - p.lr * (mh / (sqrtf(vh) + p.eps) + p.wd * W[s][r][nt][e]);
          }
          const long ci = (long)DLLM_M(b * SB + r) * p.ldc + DLLM_N(b * SB + r, nt);
          Vec4<float>::store(Cp, ci, W[s][r][nt]);
          Vec4<float>::store(p.opt_m, ci, Mm[s][r][nt]);
          Vec4<float>::store(p.opt_v, ci, Vv[s][r][nt]);
        }
        if (p.aux_out)
          st_pair_bf16(p.aux_out, (long)DLLM_M(b * SB + r) * p.ldaux + DLLM_NB(b * SB + r) + pc, W[s][r][0],
                       W[s][r][1]);
      }
    }
  } else if constexpr (EPI == EPI_ADAM) {
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RB) {
      f32x4_t W[RB][2], Mm[RB][2], Vv[RB][2];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          if (!DLLM_OK(b0 + r)) continue;
          const long ci = (long)DLLM_M(b0 + r) * p.ldc + DLLM_N(b0 + r, nt);
          W[r][nt] = RF::load(Cp, ci);
          Mm[r][nt] = RF::load(p.opt_m, ci);
          Vv[r][nt] = RF::load(p.opt_v, ci);
        }
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          if (!DLLM_OK(b0 + r)) continue;
          const f32x4_t gg = DLLM_ACC(b0 + r, nt);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float g = p.alpha * gg[e];
            Mm[r][nt][e] = p.b1 * Mm[r][nt][e] + (1.f - p.b1) * g;
            Vv[r][nt][e] = p.b2 * Vv[r][nt][e] + (1.f - p.b2) * g * g;
            const float mh = Mm[r][nt][e] / p.bc1, vh = Vv[r][nt][e] / p.bc2;
            W[r][nt][e] = W[r][nt][e] - p.lr * (mh / (sqrtf(vh) + p.eps) + p.wd * W[r][nt][e]);
          }
          const long ci = (long)DLLM_M(b0 + r) * p.ldc + DLLM_N(b0 + r, nt);
          Vec4<float>::store(Cp, ci, W[r][nt]);
          Vec4<float>::store(p.opt_m, ci, Mm[r][nt]);
          Vec4<float>::store(p.opt_v, ci, Vv[r][nt]);
        }
      if (p.aux_out) {
#pragma unroll
        for (int r = 0; r < RB; ++r)
          if (DLLM_OK(b0 + r))
            st_pair_bf16(p.aux_out, (long)DLLM_M(b0 + r) * p.ldaux + DLLM_NB(b0 + r) + pc, W[r][0], W[r][1]);
      }
    }
  }
#undef DLLM_M
#undef DLLM_OK
#undef DLLM_NB
#undef DLLM_N
#undef DLLM_ACC
}

// ----------------------------------------------------------------------------------------------
// bf16 256x256x64 MFMA kernel
// ----------------------------------------------------------------------------------------------
constexpr int BT_M = 256, BT_N = 256, BT_K = 64;
constexpr int BT_TILE_BYTES = BT_M * BT_K * 2;  // 32 KiB per operand per stage

__device__ __forceinline__ void glds16(const uint16_t* src, DLLM_LDS char* dst) {
  __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)src, (DLLM_LDS void*)dst, 16, 0, 0);
}

// per-lane element offsets (relative to the tile origin) of the 4 LDS-DMA pieces a wave issues
// for one operand tile.  Piece q (= i*8 + wave) fills LDS bytes [q*1024, q*1024+1024).
__device__ __forceinline__ void kc_offsets(long ld, int wid, int lane, long off[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 8 + wid;
    const int row = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    off[i] = (long)row * ld + c * 8;
  }
}
__device__ __forceinline__ int mc_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
__device__ __forceinline__ void mc_offsets(long ld, int wid, int lane, long off[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = i * 8 + wid;
    const int krow = 2 * q + (lane >> 5);
    const int u = (lane & 31) >> 1, h = lane & 1;
    off[i] = (long)krow * ld + ((u ^ mc_swz(krow)) * 16) + h * 8;
  }
}

// fragment of a K-contiguous tile: row `row`, 16-B chunk `chunk` (k = 8*chunk .. +7)
__device__ __forceinline__ bf16x8_t read_kc(const DLLM_LDS char* tile, int row, int chunk) {
  return *(const DLLM_LDS bf16x8_t*)(tile + row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}
// fragment of an MN-contiguous tile for the 16x16x32 operand map: lane holds op[mn0 + (lane&15)][k]
// for k = kbase + 0..7 (kbase = 32*s + 8*(lane>>4)); two ds_read_b64_tr_b16 of 4 k-rows each.
__device__ __forceinline__ bf16x8_t read_mc(const DLLM_LDS char* tile, int mn0, int kbase, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = kbase + q, k1 = kbase + 4 + q;
  const int u = mn0 >> 4;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (DLLM_LDS s16x4_t*)(tile + k0 * 512 + ((u ^ mc_swz(k0)) << 5) + 8 * p));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (DLLM_LDS s16x4_t*)(tile + k1 * 512 + ((u ^ mc_swz(k1)) << 5) + 8 * p));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

template <int LAYOUT, int EPI, typename OutT>
__global__ __launch_bounds__(512, 2) void gemm_bf16_256(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * BT_TILE_BYTES];  // [stage][A,B]
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_m = p.M / BT_M, tiles_n = p.N / BT_N;

  // tile schedule: XCD remap then grouped raster (group_m tile-rows per group)
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int width = p.group_m * tiles_n;
  const int first_m = (bid / width) * p.group_m;
  const int gsz = min(tiles_m - first_m, p.group_m);
  const int tm = first_m + (bid % width) % gsz;
  const int tn = (bid % width) / gsz;
  const int m0 = tm * BT_M, n0 = tn * BT_N;

  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  const uint16_t* Ag = (const uint16_t*)p.A + (A_KC ? (long)m0 * p.lda : (long)m0);
  const uint16_t* Bg = (const uint16_t*)p.B + (B_KC ? (long)n0 * p.ldb : (long)n0);
  long aoff[4], boff[4];
  if constexpr (A_KC) kc_offsets(p.lda, wid, lane, aoff); else mc_offsets(p.lda, wid, lane, aoff);
  if constexpr (B_KC) kc_offsets(p.ldb, wid, lane, boff); else mc_offsets(p.ldb, wid, lane, boff);
  const long a_step = A_KC ? BT_K : (long)BT_K * p.lda;
  const long b_step = B_KC ? BT_K : (long)BT_K * p.ldb;
  const int nk = p.K / BT_K;

  auto stage = [&](int kt, int buf) {
    DLLM_LDS char* As = lds + buf * 2 * BT_TILE_BYTES;
    DLLM_LDS char* Bs = As + BT_TILE_BYTES;
    const uint16_t* a = Ag + kt * a_step;
    const uint16_t* b = Bg + kt * b_step;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(a + aoff[i], As + (i * 8 + wid) * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(b + boff[i], Bs + (i * 8 + wid) * 1024);
  };

  const int wr = wid >> 2, wc = wid & 3;
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const DLLM_LDS char* As = lds + (kt & 1) * 2 * BT_TILE_BYTES;
    const DLLM_LDS char* Bs = As + BT_TILE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t af[8], bfg[4];
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int r0 = wr * 128 + mt * 16;
        if constexpr (A_KC) af[mt] = read_kc(As, r0 + (lane & 15), 4 * s + (lane >> 4));
        else af[mt] = read_mc(As, r0, 32 * s + 8 * (lane >> 4), lane);
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int c0 = wc * 64 + nt * 16;
        if constexpr (B_KC) bfg[nt] = read_kc(Bs, c0 + (lane & 15), 4 * s + (lane >> 4));
        else bfg[nt] = read_mc(Bs, c0, 32 * s + 8 * (lane >> 4), lane);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfg[nt], af[mt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: lane holds C[m0 + wr*128 + mt*16 + (lane&15)][n0 + wc*64 + nt*16 + 4*(lane>>4) + r]
  auto epilogue = [&](auto act_c) {
    constexpr int A = decltype(act_c)::value;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      const int m = m0 + wr * 128 + mt * 16 + (lane & 15);
      if constexpr (EPI == EPI_GLU) {
        // gate / up blocks alternate every 16 columns: nt even = gate, nt odd = up (same lane)
#pragma unroll
        for (int nt = 0; nt < 4; nt += 2) {
          const int ng = n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
          const int nc_out = (ng >> 5) * 16 + (ng & 15);
          epi_glu_pair<OutT, A>(p, m, nc_out, ng, ng + 16, acc[mt][nt], acc[mt][nt + 1]);
        }
      } else if constexpr (EPI == EPI_DGLU) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          epi_dglu<OutT, A>(p, m, n0 + wc * 64 + nt * 16 + 4 * (lane >> 4), acc[mt][nt]);
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          epi4<EPI, OutT, A>(p, m, n0 + wc * 64 + nt * 16 + 4 * (lane >> 4), acc[mt][nt]);
      }
    }
  };
  // activation epilogues: one branch per tile into a compile-time activation (a per-element switch kept the
  // accumulators in scratch, utils/kernel_resources.py)
  if constexpr (EPI == EPI_ACT || EPI == EPI_DACT || EPI == EPI_GLU || EPI == EPI_DGLU) {
    switch (p.act) {
      case ACT_RELU: epilogue(std::integral_constant<int, ACT_RELU>{}); break;
      case ACT_SILU: epilogue(std::integral_constant<int, ACT_SILU>{}); break;
      case ACT_GELU: epilogue(std::integral_constant<int, ACT_GELU>{}); break;
      default: epilogue(std::integral_constant<int, ACT_NONE>{}); break;
    }
  } else {
    epilogue(std::integral_constant<int, -1>{});
  }
}

// ----------------------------------------------------------------------------------------------
// bf16 256x256x64 MFMA kernel, 8-phase software pipeline (K % 128 == 0)
//
// LDS = 2 K-tile buffers x {A, B} x 2 half-tiles (16 KiB each: K-contiguous [128 rows][64 k], or
// MN-contiguous [64 k][128 mn]) = 128 KiB.  One loop iteration = 2 K-tiles = 8 phases; in phase P
// (buffer P/4, q = P%4) ALL waves compute block quadrant (QM,QN) = (0,0),(0,1),(1,1),(1,0)[q] — each
// wave a 64x32 piece of it (8 waves = 2(M) x 4(N)), 16 MFMAs = 4x2 tiles x K 64.
//   LDS reads : q0: A-half0 + B-half0, q1: B-half1, q2: A-half1, q3: none (B-half0 kept in registers)
//   LDS-DMA   : one half-tile per phase, restaged >= 1 phase after its last read:
//               P0 A1(odd,2i+1) P1 A0(even,2i+2) P2 B0(even) P3 B1(even) P4 A1(even)
//               P5 A0(odd,2i+3) P6 B0(odd) P7 B1(odd)
//   waits     : s_waitcnt vmcnt(6) (3 half-tiles left in flight) at P3 (retires the odd buffer, read in
//               P4..P6) and P7 (retires the even buffer, read in P0..P2 of the next iteration);
//               lgkmcnt(0) BEFORE the phase's first barrier, so a 1-phase restage distance is WAR-safe
//               even with the optional one-interval stagger of waves 4-7 (the SIMD partners of waves
//               0-3), which makes each SIMD alternate an MFMA segment with its partner's LDS segment.
// Out-of-range prefetches of the last iteration are clamped to the last K-tile and land in slots that
// are never read again, so every phase issues the same loads and the counted waits stay static.
// ----------------------------------------------------------------------------------------------
constexpr int HT = 16384;  // half-tile bytes

// Per-lane BYTE offsets (32-bit) of the 8-phase kernel's LDS-DMA pieces: with a uniform 64-bit panel base
// they select the SGPR-base + 32-bit VGPR-offset addressing form (no per-stage 64-bit VALU adds, half the
// VGPRs a 64-bit offset pair costs).
__device__ __forceinline__ void kc_half_offsets(long ld, int wid, int lane, uint32_t off[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wid + 8 * i;  // piece 0..15: rows 8q..8q+7
    const int row = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    off[i] = (uint32_t)(((long)row * ld + c * 8) * 2);
  }
}
__device__ __forceinline__ void mc_half_offsets(long ld, int wid, int lane, uint32_t off[2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = wid + 8 * i;  // piece 0..15: k rows 4q..4q+3 of 256 B
    const int krow = 4 * q + (lane >> 4);
    const int u = (lane & 15) >> 1, h = lane & 1;
    off[i] = (uint32_t)(((long)krow * ld + ((u ^ mc_swz(krow)) * 16) + h * 8) * 2);
  }
}
// MN-contiguous half-tile fragment: rows of 256 B, 8 units of 32 B, unit XOR mc_swz(k) (3 bits)
__device__ __forceinline__ bf16x8_t read_mc_half(const DLLM_LDS char* tile, int mn0, int kbase, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const int k0 = kbase + q, k1 = kbase + 4 + q;
  const int u = mn0 >> 4;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (DLLM_LDS s16x4_t*)(tile + k0 * 256 + ((u ^ mc_swz(k0)) << 5) + 8 * p));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (DLLM_LDS s16x4_t*)(tile + k1 * 256 + ((u ^ mc_swz(k1)) << 5) + 8 * p));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

#define DLLM_BARRIER()                      \
  do {                                      \
    asm volatile("" ::: "memory");          \
    __builtin_amdgcn_s_barrier();           \
    asm volatile("" ::: "memory");          \
  } while (0)

// Fragment reads of the 8-phase kernel are inline asm: hipcc cannot prove that a ds_read does not
// alias an in-flight LDS-DMA (global_load_lds) write and would drain the whole prefetch pipeline with
// s_waitcnt vmcnt(0) before every phase's reads.  RAW/WAR ordering against the DMA is instead carried
// by the counted vmcnt + barrier schedule below, and each phase ends its reads with an explicit
// lgkmcnt(0) + sched_barrier(0) before any MFMA consumes them (cdna_hip_programming.md §5.4 rule 18,
// §5.7 item 1 form (iii)).  Addresses are per-lane base VGPRs + compile-time offset immediates.
template <int OFF>
__device__ __forceinline__ void lds_b128(bf16x8_t& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
template <int OFF>
__device__ __forceinline__ void lds_tr16(s16x4_t& d, uint32_t addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
__device__ __forceinline__ bf16x8_t cat_tr(s16x4_t lo, s16x4_t hi) {
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}
// A fresh copy of the kernel arguments, loaded (s_load from the kernarg segment) at the call site.  hipcc
// does not rematerialise kernarg loads, so arguments used only by a persistent kernel's per-tile epilogue
// would otherwise stay live in SGPRs across the main loop (and spill).  The empty asm makes the pointer
// opaque so the loads cannot be hoisted.
// ``which`` selects the argument block of a grouped launch (gemm_bf16_8ph_pair: two GemmArgs back to back).
__device__ __forceinline__ GemmArgs reload_args(int which = 0) {
  typedef const __attribute__((address_space(4))) uint32_t* KargWords;
  KargWords pa = (KargWords)__builtin_amdgcn_kernarg_segment_ptr() + which * (int)(sizeof(GemmArgs) / 4);
  asm volatile("" : "+s"(pa));
  struct Words { uint32_t w[sizeof(GemmArgs) / 4]; } r;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(GemmArgs) / 4); ++i) r.w[i] = pa[i];
  return __builtin_bit_cast(GemmArgs, r);
}

#define DLLM_LDS_WAIT()                                   \
  do {                                                    \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    \
    __builtin_amdgcn_sched_barrier(0);                    \
  } while (0)

// Epilogue-operand prefetch (DLLM_EPI_PF): 16-B LDS-DMA pieces per wave and tile that touch exactly the bytes the
// tile's epilogue will load, so those loads hit L2 / MALL instead of paying a chip-wide HBM read burst at the tile
// boundary.  The split-master optimizers read hi + lo (2 per row group; AdamW also m and v: 4 more), the ReLU dgrad its
// 16-B mask, the SwiGLU dgrad two 16-B pre-activation pieces per row group.  0: no prefetch.
template <int EPI, typename OutT, int ACT>
constexpr int epi_pf_ops() {
  if constexpr (!DLLM_EPI_PF || !DLLM_BPRE) return 0;
  else if constexpr (EPI == EPI_SGDS || EPI == EPI_SGDS_T) return 32;
  else if constexpr (EPI == EPI_ADAMS || EPI == EPI_ADAMS_T) return 96;
  else if constexpr (EPI == EPI_DACT && ACT == ACT_RELU && std::is_same<OutT, uint16_t>::value) return 1;
  else if constexpr (EPI == EPI_DGLU && ACT >= 0 && std::is_same<OutT, uint16_t>::value) return 32;
  else return 0;
}

// ACT >= 0: activation of the ACT/DACT/GLU/DGLU epilogues fixed at compile time (-1: runtime p.act)
// NPH = 8: the 8-phase schedule below (one quadrant = 16 MFMAs per wave per barrier interval).
// NPH = 4: half-tile phases (two quadrants = 32 MFMAs per interval, two half-tiles restaged per phase):
// halves the barrier count per MFMA (see the NPH == 4 loop).
// GRP: one block of a grouped launch (gemm_bf16_8ph_pair): ``p`` is argument block ``which`` of the kernel, ``slot0``
// the block's tile in that problem (already XCD-remapped over the whole grid); one tile per block.
// BM = 224: 224-row tiles (A half-tiles of 128 + 96 rows; each wave row 64 + 48 rows, i.e. 4 + 3 row fragments), for
// GEMMs whose M is a multiple of 224 but not of 256 -- the MP (TP8) shard's F/8 = 1792 = 8 x 224 rows, which a 256-row
// tile grid fills only 7/8 of (224 tiles on 256 CUs).  K-contiguous A only (NT / NN), one tile per block.
template <int LAYOUT, int EPI, typename OutT, bool STAGGER, int ACT, int NPH, bool PERS, bool GRP, int BM = BT_M>
__device__ __forceinline__ void gemm_8ph_body(const GemmArgs& p, const int which, const int slot0) {
  static_assert(BM == BT_M || (BM == 224 && LAYOUT != L_TN && NPH == 8 && !PERS), "224-row tiles: K-contiguous A, 8 phases");
  constexpr int MT1 = BM == BT_M ? 4 : 3;  // row fragments per wave in the second A half
  // slot(op, hh, buf) = ((op*2 + hh)*2 + buf) * 16 KiB: A in [0, 64K), B in [64K, 128K), so every
  // fragment read is base + a 16-bit immediate
  // epilogue-operand prefetch: ops per wave per tile (BM = 256 tiles of the 8-phase loop only); their LDS-DMA writes
  // land in an 8 KiB sink nobody reads (1 KiB per wave)
  constexpr int PF_OPS = (NPH == 8 && BM == BT_M && !GRP) ? epi_pf_ops<EPI, OutT, ACT>() : 0;
  __shared__ __attribute__((aligned(16))) char smem[8 * HT + (PF_OPS ? 8192 : 0)];
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = p.M / BM, tiles_n = p.N / BT_N;
  const int ntiles = tiles_m * tiles_n;
  const int total = ntiles * p.ksplit;  // tile slots (split-K slices count as tiles)
  // Persistent blocks (PERS, NPH == 8, p.tpb > 1): block b runs slots b, b + G, b + 2G, ... (G = gridDim.x,
  // a multiple of the 8 XCDs, so every slot of a block maps to the block's own XCD under the remap).  Slot ->
  // tile goes through the XCD remap over ALL slots: the same tile placement and order as one block per tile.
  // A separate instantiation, so the one-tile-per-block kernels carry none of its state.
  const bool pers = PERS && !GRP && NPH == 8 && p.tpb > 1;
  int slot = slot0;
  // Per-slot helpers take the argument block explicitly: inside the slot loop they are called with a fresh
  // reload_args() copy, so the epilogue's arguments are loaded where they are used instead of being kept
  // live in SGPRs across the whole main loop.
  auto tile_of = [&](const GemmArgs& q, int s, int& sp, int& tm0, int& tn0) {
    const int tm_ = q.M / BM, tn_ = q.N / BT_N, nt = tm_ * tn_;
    const int bid0 = GRP ? s : xcd_remap(s, pers ? nt * q.ksplit : (int)gridDim.x);
    sp = bid0 / nt;  // split-K slice (0 when ksplit == 1)
    const int bid = bid0 % nt;
    const int width = q.group_m * tn_;
    const int first_m = (bid / width) * q.group_m;
    const int gsz = min(tm_ - first_m, q.group_m);
    tm0 = (first_m + (bid % width) % gsz) * BM;
    tn0 = ((bid % width) / gsz) * BT_N;
  };
  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  constexpr bool A_RKC = A_KC;  // fragment reads follow the operand image: ds_read_b128 / ds_read_b64_tr_b16
  constexpr bool B_RKC = B_KC;
  uint32_t aoff[2], boff[2];
  if constexpr (A_KC) kc_half_offsets(p.lda, wid, lane, aoff); else mc_half_offsets(p.lda, wid, lane, aoff);
  // BM = 224: the second A half has 96 rows; the DMA pieces of rows 96..127 re-load row 95 (slots never read), so
  // every wave still issues the same loads and the counted waits stay static
  uint32_t aoff1[2] = {aoff[0], aoff[1]};
  if constexpr (BM != BT_M) {
    const int row = 8 * (wid + 8) + (lane >> 3);  // piece wid + 8 (the only ones that can pass row 95)
    if (row >= BM - 128) {
      const int r = BM - 128 - 1, c = (lane & 7) ^ ((r >> 1) & 7);
      aoff1[1] = (uint32_t)(((long)r * p.lda + c * 8) * 2);
    }
  }
  if constexpr (B_KC) kc_half_offsets(p.ldb, wid, lane, boff); else mc_half_offsets(p.ldb, wid, lane, boff);
  const long a_kstep = A_KC ? BT_K : (long)BT_K * p.lda;
  const long b_kstep = B_KC ? BT_K : (long)BT_K * p.ldb;
  const long a_hstep = A_KC ? 128L * p.lda : 128L;
  const long b_hstep = B_KC ? 128L * p.ldb : 128L;
  const int nk = p.K / BT_K / p.ksplit;  // even (host guarantees (K/64) % (2*ksplit) == 0)
  // K-tile 0 of a slot's A / B panels
  auto a_base = [&](const GemmArgs& q, int s) {
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    return (const uint16_t*)q.A + (A_KC ? (long)tm0 * q.lda : (long)tm0) + (long)sp * nk * a_kstep;
  };
  auto b_base = [&](const GemmArgs& q, int s) {
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    return (const uint16_t*)q.B + (B_KC ? (long)tn0 * q.ldb : (long)tn0) + (long)sp * nk * b_kstep;
  };
  // epilogue of a slot; split-K slices write fp32 partial planes C + split*M*ldc
  auto slot_epilogue = [&](int s, f32x4_t (&ac)[2][2][4][2]) {
    const GemmArgs q = reload_args(which);
#if DLLM_EPI_SKIP
    // diagnostic build (scripts/bench_epilogue_cost.py): no epilogue -- the accumulators stay live through a branch
    // the host never takes (beta is 0 or 1 on every launch), so the main loop is unchanged and the results are wrong
    if (q.beta != 12345.f) return;
#endif
    int sp, tm0, tn0;
    tile_of(q, s, sp, tm0, tn0);
    void* out = q.C;
    if constexpr (EPI == EPI_STORE)
      if (q.ksplit > 1) out = (char*)q.C + (long)sp * q.M * q.ldc * sizeof(OutT);
    epilogue_256<EPI, OutT, ACT, 128, BM, (PERS && EPI == EPI_SGD) ? 2 : 16>(q, ac, tm0, tn0, wr, wc, lane, out);
  };
  // next slot of this block (>= total: none)
  int next_slot = total;
  auto begin_tile = [&]() { next_slot = pers ? slot + (int)gridDim.x : total; };
  begin_tile();

  // stage half hh of the K-tile at `src` (K-tile base of operand op) into buffer buf
  auto stage_at = [&](int op, int hh, const uint16_t* src, int buf) {
    DLLM_LDS char* dst = lds + ((op * 2 + hh) * 2 + buf) * HT;
    src += op == 0 ? hh * a_hstep : hh * b_hstep;
    const uint32_t* off = op == 0 ? (hh == 1 ? aoff1 : aoff) : boff;
    glds16((const uint16_t*)((const char*)src + off[0]), dst + wid * 1024);
    glds16((const uint16_t*)((const char*)src + off[1]), dst + (wid + 8) * 1024);
  };
  // 8-phase loop: running prefetch pointers at K-tile 2*it + 2 of the current slot; in the final iteration
  // they move to the NEXT slot's K-tile 0, so the last iteration's prefetches (K-tiles "nk", "nk+1") are
  // exactly the next slot's prologue -- the pipeline runs on across tiles without a drain and the epilogue
  // overlaps those loads.  Without a next slot they re-load this slot's K-tiles nk-2, nk-1 into buffers
  // that are never read again, so every phase issues the same loads.
  const uint16_t* Apf = a_base(p, slot);
  const uint16_t* Bpf = b_base(p, slot);
  // one-tile kernels (NPH == 4, 2-stage-compatible paths): K-tile kt of the block's only slot, clamped
  auto stage = [&](int op, int hh, int kt, int buf) {
    kt = min(kt, nk - 1);
    stage_at(op, hh, op == 0 ? Apf + kt * a_kstep : Bpf + kt * b_kstep, buf);
  };

  // ---- epilogue-operand prefetch (PF_OPS > 0) ----
  // Op j of a tile is issued in P1 (j even) / P5 (j odd) of main-loop iteration it0 + j / 2, after that phase's
  // stage and MFMA cluster, where it0 = nk/2 - max(ceil(PF_OPS / 2), DLLM_EPI_PF_LEAD): the last ops land a few phases before the
  // epilogue, the first ones at most the lead ahead (they must stay resident in L2 / MALL meanwhile).  Each op makes
  // the next two counted waits one deeper (P2 / P3 after a P1 op, P6 / P7 after a P5 op), so they still retire
  // exactly the staged half-tile they did before; the op itself is waited for only by later waits (vmcnt retires in
  // issue order on gfx950, loads and stores alike -- hipcc's own waitcnt model for this target).
  int pf_m0 = 0, pf_n0 = 0;   // tile origin of the slot being computed
  auto pf_begin = [&](const GemmArgs& q) {
    if constexpr (PF_OPS > 0) {
      int sp_;
      tile_of(q, slot, sp_, pf_m0, pf_n0);
      pf_m0 = __builtin_amdgcn_readfirstlane(pf_m0);
      pf_n0 = __builtin_amdgcn_readfirstlane(pf_n0);
    }
  };
  constexpr int PF_W = PF_OPS == 0 ? 0 : ((PF_OPS + 1) / 2 > DLLM_EPI_PF_LEAD ? (PF_OPS + 1) / 2 : DLLM_EPI_PF_LEAD);
  // issue op j (uniform) of the current slot's epilogue operands: the same 16-B per-lane pieces epilogue_256 loads
  auto pf_issue = [&](int j) {
    if constexpr (PF_OPS > 0) {
      const GemmArgs q = reload_args(which);   // loaded here: no argument stays live in SGPRs across the main loop
      DLLM_LDS char* sink = lds + 8 * HT + wid * 1024;
      // the lane id through an opaque copy: hipcc would otherwise hoist the per-lane address terms out of the main
      // loop and keep them live in VGPRs across it (the persistent kernels are at their 256-register budget)
      int ln = threadIdx.x & 63;
      asm volatile("" : "+v"(ln));
      const int pc = pair_col(ln);
      const void* base;
      uint32_t voff;   // byte offset from the plane's base (every plane < 4 GiB)
      if constexpr (EPI == EPI_DACT) {
        const uint32_t tile = (uint32_t)(pf_m0 / BM) * (uint32_t)(q.N / BT_N) + pf_n0 / BT_N;
        base = q.mask ? q.mask : q.aux;   // no mask (the bf16 pre-activation path): touch aux, 16x larger, instead
        voff = (tile * (8 * 64) + (wr * 4 + wc) * 64 + ln) * 16u;
      } else if constexpr (EPI == EPI_DGLU) {
        const int rg = j >> 1, nt = j & 1;
        const int row = pf_m0 + (rg >> 3) * 128 + wr * 64 + (rg & 3) * 16 + (ln & 15);
        const int colb = pf_n0 + ((rg >> 2) & 1) * 128 + wc * 32;
        base = q.aux;
        voff = ((uint32_t)row * (uint32_t)q.ldaux + 2 * colb + 32 * nt + pc) * 2u;
      } else {
        constexpr int PER = (EPI == EPI_SGDS || EPI == EPI_SGDS_T) ? 2 : 6;
        const int rg = j / PER, k = j - rg * PER;
        int row, colb;
        if constexpr (epi_tout(EPI)) {
          row = pf_n0 + ((rg >> 2) & 1) * 128 + wc * 32 + ((rg >> 1) & 1) * 16 + (ln & 15);
          colb = pf_m0 + (rg >> 3) * 128 + wr * 64 + (rg & 1) * 32;
        } else {
          row = pf_m0 + (rg >> 3) * 128 + wr * 64 + (rg & 3) * 16 + (ln & 15);
          colb = pf_n0 + ((rg >> 2) & 1) * 128 + wc * 32;
        }
        if (k == 0) {
          base = q.aux_out;
          voff = ((uint32_t)row * (uint32_t)q.ldaux + colb + pc) * 2u;
        } else if (k == 1) {
          base = q.C;
          voff = ((uint32_t)row * (uint32_t)q.ldc + colb + pc) * 2u;
        } else {
          base = k < 4 ? q.opt_m : q.opt_v;
          voff = ((uint32_t)row * (uint32_t)q.ldc + colb + ((k - 2) & 1) * 16 + 4 * (ln >> 4)) * 4u;
        }
      }
      // uniform 64-bit base + 32-bit per-lane offset: the SGPR-base / VGPR-offset addressing form of the stages
      glds16((const uint16_t*)((const char*)base + voff), sink);
    }
  };
  // P1 (h = 0) / P5 (h = 1) of iteration it: every iteration issues one op, so the counted waits stay static and the
  // main loop has no branch (a branch there cost 16 VGPRs and made the persistent kernels spill): outside the window the
  // op index is clamped to the window's first / last op (a re-touch of lines that are, or will be, prefetched anyway)
  auto pf_at = [&](int it, int h) {
    if constexpr (PF_OPS > 0) {
      int j = 2 * (it - (nk / 2 - PF_W)) + h;
      // opaque to hipcc: it would otherwise split the main loop at the window start into specialised copies
      asm volatile("" : "+s"(j));
      j = j < 0 ? 0 : (j >= PF_OPS ? PF_OPS - 1 : j);
      pf_issue(j);
    }
  };

  // ---- per-lane fragment base addresses (LDS byte addresses) ----
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int g = lane >> 4, i15 = lane & 15;
  // K-contiguous image (128-B rows, chunk ^= (row>>1)&7): base for k-substep s; rows R + mt*16 + i15
  const int fkc = (i15 >> 1) & 7;
  // MN-contiguous image (256-B rows, unit ^= (k&3)|((k>>3)&1)<<2): per tile t
  const int q = i15 >> 2, pp = i15 & 3, swz = q | ((g & 1) << 2);
  uint32_t abase[4], bbase[2], abase1[2];
  if constexpr (A_RKC) {
    abase[0] = lds_base + (wr * 64 + i15) * 128 + (((0 + g) ^ fkc) << 4);
    abase[1] = lds_base + (wr * 64 + i15) * 128 + (((4 + g) ^ fkc) << 4);
    // second A half of a 224-row tile: wave row wr reads rows wr*48 + mt*16 (the chunk swizzle depends on row bits
    // 1-3 only, which 48*wr does not touch)
    abase1[0] = abase[0] - (BM == BT_M ? 0 : wr * 16 * 128);
    abase1[1] = abase[1] - (BM == BT_M ? 0 : wr * 16 * 128);
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
      abase[t] = lds_base + (8 * g + q) * 256 + (((4 * wr + t) ^ swz) << 5) + 8 * pp;
  }
  if constexpr (B_RKC) {
    bbase[0] = lds_base + 4 * HT + (wc * 32 + i15) * 128 + (((0 + g) ^ fkc) << 4);
    bbase[1] = lds_base + 4 * HT + (wc * 32 + i15) * 128 + (((4 + g) ^ fkc) << 4);
  } else {
#pragma unroll
    for (int t = 0; t < 2; ++t)
      bbase[t] = lds_base + 4 * HT + (8 * g + q) * 256 + (((2 * wc + t) ^ swz) << 5) + 8 * pp;
  }

  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  bf16x8_t fa[4][2], fb0[2][2], fb1[2][2];  // [tile][k-substep]
  // transposed-read halves: issued in the read segment, combined after the phase's single lgkmcnt(0)
  s16x4_t ta_lo[4][2], ta_hi[4][2], tb_lo[2][2], tb_hi[2][2], tc_lo[2][2], tc_hi[2][2];

  // A half hh of buffer buf -> fa ; B half hh of buffer buf -> fb   (issue only)
  auto read_a = [&](auto hh_c, auto buf_c) {
    constexpr int SO = (hh_c.value * 2 + buf_c.value) * HT;
    if constexpr (A_RKC && BM != BT_M && hh_c.value == 1) {
      lds_b128<SO + 0 * 2048>(fa[0][0], abase1[0]); lds_b128<SO + 1 * 2048>(fa[1][0], abase1[0]);
      lds_b128<SO + 2 * 2048>(fa[2][0], abase1[0]);
      lds_b128<SO + 0 * 2048>(fa[0][1], abase1[1]); lds_b128<SO + 1 * 2048>(fa[1][1], abase1[1]);
      lds_b128<SO + 2 * 2048>(fa[2][1], abase1[1]);
    } else if constexpr (A_RKC) {
      lds_b128<SO + 0 * 2048>(fa[0][0], abase[0]); lds_b128<SO + 1 * 2048>(fa[1][0], abase[0]);
      lds_b128<SO + 2 * 2048>(fa[2][0], abase[0]); lds_b128<SO + 3 * 2048>(fa[3][0], abase[0]);
      lds_b128<SO + 0 * 2048>(fa[0][1], abase[1]); lds_b128<SO + 1 * 2048>(fa[1][1], abase[1]);
      lds_b128<SO + 2 * 2048>(fa[2][1], abase[1]); lds_b128<SO + 3 * 2048>(fa[3][1], abase[1]);
    } else {
#define DLLM_TRA(t, s)                                              \
  lds_tr16<SO + (s) * 8192>(ta_lo[t][s], abase[t]);                 \
  lds_tr16<SO + (s) * 8192 + 1024>(ta_hi[t][s], abase[t]);
      DLLM_TRA(0, 0) DLLM_TRA(1, 0) DLLM_TRA(2, 0) DLLM_TRA(3, 0)
      DLLM_TRA(0, 1) DLLM_TRA(1, 1) DLLM_TRA(2, 1) DLLM_TRA(3, 1)
#undef DLLM_TRA
    }
  };
  auto fin_a = [&]() {  // after the phase's lgkmcnt(0)
    if constexpr (!A_RKC) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) fa[t][s2] = cat_tr(ta_lo[t][s2], ta_hi[t][s2]);
    }
  };
  auto read_b = [&](auto hh_c, auto buf_c, bf16x8_t (&fb)[2][2]) {
    constexpr int SO = (hh_c.value * 2 + buf_c.value) * HT;
    if constexpr (B_RKC) {
      lds_b128<SO + 0 * 2048>(fb[0][0], bbase[0]); lds_b128<SO + 1 * 2048>(fb[1][0], bbase[0]);
      lds_b128<SO + 0 * 2048>(fb[0][1], bbase[1]); lds_b128<SO + 1 * 2048>(fb[1][1], bbase[1]);
    } else {
#define DLLM_TRB(t, s)                                              \
  lds_tr16<SO + (s) * 8192>(tb_lo[t][s], bbase[t]);                 \
  lds_tr16<SO + (s) * 8192 + 1024>(tb_hi[t][s], bbase[t]);
      DLLM_TRB(0, 0) DLLM_TRB(1, 0) DLLM_TRB(0, 1) DLLM_TRB(1, 1)
#undef DLLM_TRB
    }
  };
  auto fin_b = [&](bf16x8_t (&fb)[2][2]) {
    if constexpr (!B_RKC) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) fb[t][s2] = cat_tr(tb_lo[t][s2], tb_hi[t][s2]);
    }
  };  // second B half in the same phase (NPH == 4): its own transposed-read temporaries
  auto read_b2 = [&](auto hh_c, auto buf_c, bf16x8_t (&fb)[2][2]) {
    constexpr int SO = (hh_c.value * 2 + buf_c.value) * HT;
    if constexpr (B_RKC) {
      lds_b128<SO + 0 * 2048>(fb[0][0], bbase[0]); lds_b128<SO + 1 * 2048>(fb[1][0], bbase[0]);
      lds_b128<SO + 0 * 2048>(fb[0][1], bbase[1]); lds_b128<SO + 1 * 2048>(fb[1][1], bbase[1]);
    } else {
#define DLLM_TRC(t, s)                                              \
  lds_tr16<SO + (s) * 8192>(tc_lo[t][s], bbase[t]);                 \
  lds_tr16<SO + (s) * 8192 + 1024>(tc_hi[t][s], bbase[t]);
      DLLM_TRC(0, 0) DLLM_TRC(1, 0) DLLM_TRC(0, 1) DLLM_TRC(1, 1)
#undef DLLM_TRC
    }
  };  auto fin_b2 = [&](bf16x8_t (&fb)[2][2]) {
    if constexpr (!B_RKC) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) fb[t][s2] = cat_tr(tc_lo[t][s2], tc_hi[t][s2]);
    }
  };
  // qm_c: the quadrant's A half (second half of a 224-row tile: MT1 row fragments)
  auto mfma_quad = [&](f32x4_t (&c)[4][2], const bf16x8_t (&fb)[2][2], auto qm_c) {
    constexpr int NMT = qm_c.value == 1 ? MT1 : 4;
#if DLLM_PRIO_MODE == 0
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int mt = 0; mt < NMT; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          if constexpr (epi_tout(EPI))  // transposed output: lane ends with 4 consecutive rows of one column
            c[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][s2], fb[nt][s2], c[mt][nt], 0, 0, 0);
          else
            c[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nt][s2], fa[mt][s2], c[mt][nt], 0, 0, 0);
        }
#if DLLM_PRIO_MODE == 0
    __builtin_amdgcn_s_setprio(0);
#endif
  };
#if DLLM_PRIO_MODE == 1
  // static priority for the younger (second-dispatched) half, set once (MI355X_MICROARCH.md, two waves per SIMD
  // item 4) instead of raising every wave's priority around each MFMA cluster
  if (wr == 1) __builtin_amdgcn_s_setprio(1);
#endif
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  if constexpr (NPH == 4) {
    // Half-tile phases: P0 (tile te: quadrants (0,0),(0,1); reads A0 B0 B1), P1 (te: (1,1),(1,0); reads
    // A1), P2 / P3 the same on tile to.  Two half-tiles restaged per phase, each >= 1 phase after its
    // last read (lgkmcnt(0) before the reading phase's first barrier):
    //   P0 B1o A1o (tile to)   P1 A0e B0e (te+2)   P2 B1e A1e (te+2)   P3 A0o B0o (to+2)
    // vmcnt before each phase's first barrier retires exactly what the next phase reads:
    //   P0 -> A1e: 8 pieces younger (A0o B0o B1o A1o)   P1 -> A0o B0o B1o: 6 younger
    //   P2 -> A1o: 8 younger                             P3 -> A0e' B0e' B1e': 6 younger
    stage(0, 0, 0, 0); stage(1, 0, 0, 0); stage(1, 1, 0, 0); stage(0, 1, 0, 0);
    stage(0, 0, 1, 1); stage(1, 0, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    DLLM_BARRIER();
    if constexpr (STAGGER) {
      if (wr == 1) DLLM_BARRIER();
    }
    for (int it = 0; it < nk / 2; ++it) {
      const int te = 2 * it, to = 2 * it + 1;
#define DLLM_PHASE_END4(N)                                            \
  asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory");               \
  DLLM_LDS_WAIT();                                                    \
  DLLM_BARRIER();
      read_a(I0{}, I0{}); read_b(I0{}, I0{}, fb0); read_b2(I1{}, I0{}, fb1);
      stage(1, 1, to, 1); stage(0, 1, to, 1);            // P0: B1 A1 odd
      DLLM_PHASE_END4(8)
      fin_a(); fin_b(fb0); fin_b2(fb1);
      mfma_quad(acc[0][0], fb0, I0{}); mfma_quad(acc[0][1], fb1, I0{});
      DLLM_BARRIER();
      read_a(I1{}, I0{});
      stage(0, 0, te + 2, 0); stage(1, 0, te + 2, 0);    // P1: A0 B0 even
      DLLM_PHASE_END4(6)
      fin_a();
      mfma_quad(acc[1][1], fb1, I1{}); mfma_quad(acc[1][0], fb0, I1{});
      DLLM_BARRIER();
      read_a(I0{}, I1{}); read_b(I0{}, I1{}, fb0); read_b2(I1{}, I1{}, fb1);
      stage(1, 1, te + 2, 0); stage(0, 1, te + 2, 0);    // P2: B1 A1 even
      DLLM_PHASE_END4(8)
      fin_a(); fin_b(fb0); fin_b2(fb1);
      mfma_quad(acc[0][0], fb0, I0{}); mfma_quad(acc[0][1], fb1, I0{});
      DLLM_BARRIER();
      read_a(I1{}, I1{});
      stage(0, 0, to + 2, 1); stage(1, 0, to + 2, 1);    // P3: A0 B0 odd
      DLLM_PHASE_END4(6)
      fin_a();
      mfma_quad(acc[1][1], fb1, I1{}); mfma_quad(acc[1][0], fb0, I1{});
      DLLM_BARRIER();
#undef DLLM_PHASE_END4
    }
  } else {
  // prologue: tile 0 -> even buffer (4 half-tiles), tile 1 -> odd (A0, B0, B1; A1 comes at P0)
  stage(0, 0, 0, 0); stage(1, 0, 0, 0); stage(1, 1, 0, 0); stage(0, 1, 0, 0);
  stage(0, 0, 1, 1); stage(1, 0, 1, 1); stage(1, 1, 1, 1);
  Apf += 2 * a_kstep;
  Bpf += 2 * b_kstep;
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  DLLM_BARRIER();
#if DLLM_BPRE
  // B-half 0 of K-tile 0 ahead of the loop (the loop reads every K-tile's B0 one phase before its q0, see below)
  read_b(I0{}, I0{}, fb0);
  DLLM_LDS_WAIT();
  fin_b(fb0);
#endif
  if constexpr (STAGGER) {
    if (wr == 1) DLLM_BARRIER();
  }
  pf_begin(p);

  for (;;) {  // slots of this block (one pass unless persistent)
  for (int it = 0; it < nk / 2; ++it) {
#define DLLM_PHASE_END(VMWAIT)                                      \
  if (VMWAIT) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");       \
  DLLM_LDS_WAIT();                                                   \
  DLLM_BARRIER();
#if DLLM_BPRE
    // Balanced fragment reads (round 5).  The fragment-read segment of phase P overlaps the SIMD partner's MFMA
    // segment; the round-4 order read A0 + B0 (12 of the K-tile's 24 fragments) before q0 and nothing before q3.
    // Here each K-tile's B-half 0 is read one phase early, in the previous quadrant q3 (into whichever B register set
    // q2 has finished with: fb0 / fb1 alternate per K-tile), so the segments carry 8 / 4 / 8 / 4 fragments: +0.2 to
    // +3.1 % per FFN GEMM (profiles/r5/gemm_bpre_ab_r5.txt).  The MFMA sequence is unchanged (bitwise the same results).
    // That read needs the next buffer's B0 retired one phase earlier: vmcnt(8) at P2 / P6 (after the stage, 4
    // half-tiles left in flight) retires the B0 staged at P6 / P2 before, read at P3 / P7.
#define DLLM_PHASE_END8()                                           \
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                   \
  DLLM_LDS_WAIT();                                                   \
  DLLM_BARRIER();
    // with epilogue-operand prefetch the P2 / P6 and P3 / P7 waits are one deeper: the op issued in P1 / P5 is
    // younger than the staged half-tile they retire
#define DLLM_PHASE_END8_PF()                                        \
  if constexpr (PF_OPS > 0) asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); \
  else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");              \
  DLLM_LDS_WAIT();                                                   \
  DLLM_BARRIER();
#define DLLM_PHASE_END6_PF()                                        \
  if constexpr (PF_OPS > 0) asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); \
  else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");              \
  DLLM_LDS_WAIT();                                                   \
  DLLM_BARRIER();
    // ---- even buffer (K-tile 2it); its B0 is in fb0 ----
    read_a(I0{}, I0{});
    stage_at(0, 1, Apf - a_kstep, 1);          // P0: A1 odd (K-tile 2it+1)
    if (it == nk / 2 - 1) {
      if (next_slot < total) {
        const GemmArgs q = reload_args(which);
        Apf = a_base(q, next_slot);
        Bpf = b_base(q, next_slot);
      } else {
        Apf -= 2 * a_kstep;
        Bpf -= 2 * b_kstep;
      }
    }
    DLLM_PHASE_END(false)
    fin_a();
    mfma_quad(acc[0][0], fb0, I0{});
    DLLM_BARRIER();
    read_b(I1{}, I0{}, fb1);
    stage_at(0, 0, Apf, 0);                    // P1: A0 even (K-tile 2it+2)
    DLLM_PHASE_END(false)
    fin_b(fb1);
    mfma_quad(acc[0][1], fb1, I0{});
    // an epilogue-operand prefetch op: after P1's stage and before P2's (the same wait accounting as right after the
    // stage), here where the A fragments are dead until P2's reads (register pressure)
    pf_at(it, 0);
    DLLM_BARRIER();
    read_a(I1{}, I0{});
    stage_at(1, 0, Bpf, 0);                    // P2: B0 even
    DLLM_PHASE_END8_PF()
    fin_a();
    mfma_quad(acc[1][1], fb1, I1{});
    DLLM_BARRIER();
    read_b(I0{}, I1{}, fb1);                   // odd buffer's B0 (retired at P2) -> fb1 (free after q2)
    stage_at(1, 1, Bpf, 0);                    // P3: B1 even
    DLLM_PHASE_END6_PF()
    fin_b(fb1);
    mfma_quad(acc[1][0], fb0, I1{});
    DLLM_BARRIER();
    // ---- odd buffer (K-tile 2it+1); its B0 is in fb1 ----
    read_a(I0{}, I1{});
    stage_at(0, 1, Apf, 0);                    // P4: A1 even
    DLLM_PHASE_END(false)
    fin_a();
    mfma_quad(acc[0][0], fb1, I0{});
    DLLM_BARRIER();
    read_b(I1{}, I1{}, fb0);
    stage_at(0, 0, Apf + a_kstep, 1);          // P5: A0 odd (K-tile 2it+3)
    DLLM_PHASE_END(false)
    fin_b(fb0);
    mfma_quad(acc[0][1], fb0, I0{});
    pf_at(it, 1);                              // (see P1)
    DLLM_BARRIER();
    read_a(I1{}, I1{});
    stage_at(1, 0, Bpf + b_kstep, 1);          // P6: B0 odd
    DLLM_PHASE_END8_PF()
    fin_a();
    mfma_quad(acc[1][1], fb0, I1{});
    DLLM_BARRIER();
    read_b(I0{}, I0{}, fb0);                   // next even B0 (K-tile 2it+2, or the next slot's K-tile 0) -> fb0
    stage_at(1, 1, Bpf + b_kstep, 1);          // P7: B1 odd
    DLLM_PHASE_END6_PF()
    fin_b(fb0);
    mfma_quad(acc[1][0], fb1, I1{});
    DLLM_BARRIER();
#undef DLLM_PHASE_END8
#undef DLLM_PHASE_END8_PF
#undef DLLM_PHASE_END6_PF
#else
    // ---- even buffer (K-tile 2it) ----
    read_a(I0{}, I0{}); read_b(I0{}, I0{}, fb0);
    stage_at(0, 1, Apf - a_kstep, 1);          // P0: A1 odd (K-tile 2it+1)
    if (it == nk / 2 - 1) {
      // last iteration: the remaining prefetches are the next slot's K-tiles 0/1 (or harmless re-loads)
      if (next_slot < total) {
        const GemmArgs q = reload_args(which);
        Apf = a_base(q, next_slot);
        Bpf = b_base(q, next_slot);
      } else {
        Apf -= 2 * a_kstep;
        Bpf -= 2 * b_kstep;
      }
    }
    DLLM_PHASE_END(false)
    fin_a(); fin_b(fb0);
    mfma_quad(acc[0][0], fb0, I0{});
    DLLM_BARRIER();
    read_b(I1{}, I0{}, fb1);
    stage_at(0, 0, Apf, 0);                    // P1: A0 even (K-tile 2it+2)
    DLLM_PHASE_END(false)
    fin_b(fb1);
    mfma_quad(acc[0][1], fb1, I0{});
    DLLM_BARRIER();
    read_a(I1{}, I0{});
    stage_at(1, 0, Bpf, 0);                    // P2: B0 even
    DLLM_PHASE_END(false)
    fin_a();
    mfma_quad(acc[1][1], fb1, I1{});
    DLLM_BARRIER();
    stage_at(1, 1, Bpf, 0);                    // P3: B1 even
    DLLM_PHASE_END(true)
    mfma_quad(acc[1][0], fb0, I1{});
    DLLM_BARRIER();
    // ---- odd buffer (K-tile 2it+1) ----
    read_a(I0{}, I1{}); read_b(I0{}, I1{}, fb0);
    stage_at(0, 1, Apf, 0);                    // P4: A1 even
    DLLM_PHASE_END(false)
    fin_a(); fin_b(fb0);
    mfma_quad(acc[0][0], fb0, I0{});
    DLLM_BARRIER();
    read_b(I1{}, I1{}, fb1);
    stage_at(0, 0, Apf + a_kstep, 1);          // P5: A0 odd (K-tile 2it+3)
    DLLM_PHASE_END(false)
    fin_b(fb1);
    mfma_quad(acc[0][1], fb1, I0{});
    DLLM_BARRIER();
    read_a(I1{}, I1{});
    stage_at(1, 0, Bpf + b_kstep, 1);          // P6: B0 odd
    DLLM_PHASE_END(false)
    fin_a();
    mfma_quad(acc[1][1], fb1, I1{});
    DLLM_BARRIER();
    stage_at(1, 1, Bpf + b_kstep, 1);          // P7: B1 odd
    DLLM_PHASE_END(true)
    mfma_quad(acc[1][0], fb0, I1{});
    DLLM_BARRIER();
#endif
    Apf += 2 * a_kstep;
    Bpf += 2 * b_kstep;
#undef DLLM_PHASE_END
  }
  if (next_slot >= total) break;
  // Persistent: the next slot's K-tiles 0/1 are landed (even buffer) or in flight (odd half-tiles) and
  // Apf/Bpf already point at its K-tile 2; this slot's epilogue runs meanwhile.  It touches no LDS and
  // has no barrier, so the (staggered) barrier sequence continues unchanged into the next slot's P0; its
  // memory operations are older than the next slot's P0-P3 stages and are retired by P3's counted wait.
  slot_epilogue(slot, acc);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  slot = next_slot;
  begin_tile();
  if constexpr (PF_OPS > 0) pf_begin(reload_args(which));
  }  // slots
  }  // NPH == 8
  if constexpr (STAGGER) {
    if (wr == 0) DLLM_BARRIER();
  }
  // drain the tail prefetches before the block can release its LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  slot_epilogue(slot, acc);
}

template <int LAYOUT, int EPI, typename OutT, bool STAGGER, int ACT = -1, int NPH = 8, bool PERS = false>
__global__ __launch_bounds__(512, 2) void gemm_bf16_8ph(GemmArgs p) {
  gemm_8ph_body<LAYOUT, EPI, OutT, STAGGER, ACT, NPH, PERS, false>(p, 0, blockIdx.x);
}

// Two GEMMs of one layout, epilogue and K in ONE launch, one 256x256 tile per block (grid = tiles(p0) + tiles(p1)
// <= CUs).  For weight-gradient pairs whose own grids leave the chip part-empty -- the MP (TP8) shard's dW2 [D, F/8]
// and dW1 [F/8, D], 112 tiles each at F = 14336 -- instead of split-K slices and a reduction pass per GEMM.  The
// remapped block ids are split [0, tiles(p0)) | [tiles(p0), ...), so each problem's tiles fill whole XCDs of their own
// (no operand panel is shared across the two problems) and keep the grouped raster inside the problem.
template <int LAYOUT, int EPI, typename OutT, int BM = BT_M>
__global__ __launch_bounds__(512, 2) void gemm_bf16_8ph_pair(GemmArgs p0, GemmArgs p1) {
  const int nt0 = (p0.M / BM) * (p0.N / BT_N);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int which = bid >= nt0 ? 1 : 0;  // one inlined body over the selected argument block (code size)
  gemm_8ph_body<LAYOUT, EPI, OutT, true, -1, 8, false, true, BM>(which ? p1 : p0, which, bid - which * nt0);
}

// 224-row tiles (see gemm_8ph_body): one tile per block, staggered 8-phase main loop
template <int LAYOUT, int EPI, typename OutT, int ACT = -1>
__global__ __launch_bounds__(512, 2) void gemm_bf16_8ph_m224(GemmArgs p) {
  gemm_8ph_body<LAYOUT, EPI, OutT, true, ACT, 8, false, false, 224>(p, 0, blockIdx.x);
}

// ----------------------------------------------------------------------------------------------
// fp32 128x128x16 MFMA kernel (exact fp32: v_mfma_f32_16x16x4_f32 is a k-ordered fmaf chain)
// ----------------------------------------------------------------------------------------------
constexpr int FT = 128, FK = 16, FLD = FT + 4;

template <int LAYOUT, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f32_128(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * FK * FLD];
  float* As = smem;            // [k][m]
  float* Bs = smem + FK * FLD; // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_m = p.M / FT, tiles_n = p.N / FT;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int width = p.group_m * tiles_n;
  const int first_m = (bid / width) * p.group_m;
  const int gsz = min(tiles_m - first_m, p.group_m);
  const int tm = first_m + (bid % width) % gsz, tn = (bid % width) / gsz;
  const int m0 = tm * FT, n0 = tn * FT;
  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  const float* A = (const float*)p.A;
  const float* B = (const float*)p.B;

  f32x4_t ra[2], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int f = tid + 256 * j;
      if constexpr (A_KC) ra[j] = *(const f32x4_t*)(A + (long)(m0 + (f >> 2)) * p.lda + k0 + (f & 3) * 4);
      else ra[j] = *(const f32x4_t*)(A + (long)(k0 + (f >> 5)) * p.lda + m0 + (f & 31) * 4);
      if constexpr (B_KC) rb[j] = *(const f32x4_t*)(B + (long)(n0 + (f >> 2)) * p.ldb + k0 + (f & 3) * 4);
      else rb[j] = *(const f32x4_t*)(B + (long)(k0 + (f >> 5)) * p.ldb + n0 + (f & 31) * 4);
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int f = tid + 256 * j;
      if constexpr (A_KC) {
        const int row = f >> 2, kq = (f & 3) * 4;
        for (int e = 0; e < 4; ++e) As[(kq + e) * FLD + row] = ra[j][e];
      } else {
        *(f32x4_t*)(As + (f >> 5) * FLD + (f & 31) * 4) = ra[j];
      }
      if constexpr (B_KC) {
        const int row = f >> 2, kq = (f & 3) * 4;
        for (int e = 0; e < 4; ++e) Bs[(kq + e) * FLD + row] = rb[j][e];
      } else {
        *(f32x4_t*)(Bs + (f >> 5) * FLD + (f & 31) * 4) = rb[j];
      }
    }
  };

  const int wr = wid >> 1, wc = wid & 1;  // 2x2 waves, 64x64 each
  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / FK;
  gload(0);
  sstore();
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload((kt + 1) * FK);
#pragma unroll
    for (int ks = 0; ks < FK; ks += 4) {
      const int k = ks + (lane >> 4);
      float av[4], bv[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) av[mt] = As[k * FLD + wr * 64 + mt * 16 + (lane & 15)];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) bv[nt] = Bs[k * FLD + wc * 64 + nt * 16 + (lane & 15)];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[nt], av[mt], acc[mt][nt], 0, 0, 0);
    }
    __syncthreads();
    if (kt + 1 < nk) {
      sstore();
      __syncthreads();
    }
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = m0 + wr * 64 + mt * 16 + (lane & 15);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int n = n0 + wc * 64 + nt * 16 + 4 * (lane >> 4);
      if constexpr (EPI == EPI_GLU) {
        if ((nt & 1) == 0) {
          const int nc_out = (n >> 5) * 16 + (n & 15);
          epi_glu_pair<float>(p, m, nc_out, n, n + 16, acc[mt][nt], acc[mt][nt + 1]);
        }
      } else if constexpr (EPI == EPI_DGLU) {
        epi_dglu<float>(p, m, n, acc[mt][nt]);
      } else {
        epi4<EPI, float>(p, m, n, acc[mt][nt]);
      }
    }
  }
}

// ----------------------------------------------------------------------------------------------
// fp32 256x256x32 MFMA kernel (reference-precision path: exact-fp32 v_mfma_f32_16x16x4_f32)
//
// The fp32 MFMA is 4x slower per FLOP than bf16 (157 TF peak), so each 16x16x4 MFMA is 32 cycles and the LDS
// traffic per MFMA is small; what caps an fp32 GEMM is feeding the MFMA pipe without gaps: here 8 waves (2M x 4N,
// 2 per SIMD), a 256x256 block tile (half the operand bytes per FLOP of a 128x128 tile), K-tiles of 32 (128-B
// rows: every LDS-DMA touches whole cache lines), a 2-stage LDS ring (128 KiB) filled by LDS-DMA
// (global_load_lds_dwordx4) one K-tile ahead, and ONE barrier per K-tile (256 MFMAs = 8192 cycles per wave
// between barriers, far longer than the DMA latency it hides).
//
// K permutation: an MFMA consumes k = kk (lane group l/16) of its 4; at step s (0..7) lane group g supplies
// k = 8g + s for BOTH operands, so a K-contiguous fragment is two ds_read_b128 (A[row][8g .. 8g+7]) serving all
// 8 steps.  (Exact products; the fp32 sums run in a different order than a k-sequential chain -- like any
// blocked BLAS.)  Each K-tile is consumed in two halves (steps 0-3, 4-7) to keep the fragment registers at 48.
// LDS images (conflict-free):  K-contiguous [256 rows][32 k] (128-B rows), 16-B chunk ^= f2_swz(row);
//                              MN-contiguous [32 k][256 mn] (1 KiB rows), mn ^= ((k >> 3) & 3) << 4.
// The per-wave tile follows the 8-phase bf16 kernel's quadrant map, so its batched epilogues (act, dact,
// glu, dglu, sgd, adam, store) are reused as is.
// ----------------------------------------------------------------------------------------------
constexpr int F2_T = 256, F2_K = 32, F2_HALF = F2_T * F2_K * 4, F2_STAGE = 2 * F2_HALF;  // 64 KiB per stage

template <int LAYOUT, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_f32_256(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * F2_STAGE];
  DLLM_LDS char* lds = (DLLM_LDS char*)smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int tiles_m = p.M / F2_T, tiles_n = p.N / F2_T;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int width = p.group_m * tiles_n;
  const int first_m = (bid / width) * p.group_m;
  const int gsz = min(tiles_m - first_m, p.group_m);
  const int m0 = (first_m + (bid % width) % gsz) * F2_T, n0 = ((bid % width) / gsz) * F2_T;
  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  const float* A = (const float*)p.A + (A_KC ? (long)m0 * p.lda : (long)m0);
  const float* B = (const float*)p.B + (B_KC ? (long)n0 * p.ldb : (long)n0);
  const long a_kstep = A_KC ? F2_K : (long)F2_K * p.lda;
  const long b_kstep = B_KC ? F2_K : (long)F2_K * p.ldb;
  // LDS-DMA: the 32 KiB operand tile is 32 pieces of 1 KiB (64 lanes x 16 B, lane-linear); wave w fills pieces
  // w, w+8, w+16, w+24.  Per-lane 32-bit byte offsets of the source (the swizzle is applied on the source).
  uint32_t aoff[4], boff[4];
  // K-contiguous image: 16-B chunk c of row r sits at chunk position c ^ f2_swz(r).  The fragment reads take
  // chunk 2g + h in lane group g (lanes 16g .. 16g+15, rows r0 + (lane & 15)); ds_read_b128 serves lanes in four
  // 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, +32) that mix rows 0-3/12-15 of one g with rows 4-11
  // of g +- 1, i.e. chunk positions that differ by XOR 2: f2_swz keeps each group on 16 distinct 16-B slots of
  // the 256-B bank row.  (The bf16 kernel's (r >> 1) & 7 is conflict-free for its XOR-1 pairing but 2-way here:
  // SQ_LDS_BANK_CONFLICT was ~8 % of the fp32 kernel's cycles, hipBLASLt's 0.)
  auto f2_swz = [](int row) { return ((row >> 1) & 7) ^ (((row >> 2) & 1) << 2); };
  auto kc_off = [&](long ld, uint32_t (&o)[4]) {  // piece q = rows 8q .. 8q+7 (128 B each)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = wid + 8 * i, row = 8 * q + (lane >> 3);
      o[i] = (uint32_t)(((long)row * ld + 4 * ((lane & 7) ^ f2_swz(row))) * 4);
    }
  };
  auto mc_off = [&](long ld, uint32_t (&o)[4]) {  // piece q = k row q (1 KiB)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = wid + 8 * i;
      o[i] = (uint32_t)(((long)k * ld + ((4 * lane) ^ (((k >> 3) & 3) << 4))) * 4);
    }
  };
  if constexpr (A_KC) kc_off(p.lda, aoff); else mc_off(p.lda, aoff);
  if constexpr (B_KC) kc_off(p.ldb, boff); else mc_off(p.ldb, boff);
  auto stage = [&](int kt, int buf) {
    DLLM_LDS char* As = lds + buf * F2_STAGE;
    DLLM_LDS char* Bs = As + F2_HALF;
    const char* a = (const char*)(A + kt * a_kstep);
    const char* b = (const char*)(B + kt * b_kstep);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)(a + aoff[i]), (DLLM_LDS void*)(As + (wid + 8 * i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const DLLM_GLB void*)(b + boff[i]), (DLLM_LDS void*)(Bs + (wid + 8 * i) * 1024),
                                       16, 0, 0);
  };
  // fragment byte offsets.  Row tiles of the wave: r = QM*128 + wr*64 + mt*16 -> index QM*4 + mt; column tiles
  // c = QN*128 + wc*32 + nt*16 -> QN*2 + nt (the bf16 8-phase kernel's quadrant map).
  const int g = lane >> 4, i15 = lane & 15;
  auto kc_addr = [&](int r0, int h) {  // ds_read_b128: [row][k 8g + 4h .. +3]
    const int row = r0 + i15;
    return (uint32_t)(row * 128 + (((2 * g + h) ^ f2_swz(row)) << 4));
  };
  auto mc_addr = [&](int c0, int k) {  // ds_read_b32: [k][mn]
    return (uint32_t)(k * 1024 + (((c0 + i15) ^ (g << 4)) << 2));
  };
  f32x4_t acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / F2_K;
  stage(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed; the barrier publishes it to every wave and retires every wave's reads of the other
    // buffer (iteration kt - 1) before it is restaged with K-tile kt + 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) stage(kt + 1, (kt + 1) & 1);
    const DLLM_LDS char* As = lds + (kt & 1) * F2_STAGE;
    const DLLM_LDS char* Bs = As + F2_HALF;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float af[8][4], bf[4][4];  // [row tile][step], [col tile][step]
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const int r0 = (t >> 2) * 128 + wr * 64 + (t & 3) * 16;
        if constexpr (A_KC) {
          const f32x4_t v = *(const DLLM_LDS f32x4_t*)(As + kc_addr(r0, h));
          af[t][0] = v[0]; af[t][1] = v[1]; af[t][2] = v[2]; af[t][3] = v[3];
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) af[t][s2] = *(const DLLM_LDS float*)(As + mc_addr(r0, 8 * g + 4 * h + s2));
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c0 = (t >> 1) * 128 + wc * 32 + (t & 1) * 16;
        if constexpr (B_KC) {
          const f32x4_t v = *(const DLLM_LDS f32x4_t*)(Bs + kc_addr(c0, h));
          bf[t][0] = v[0]; bf[t][1] = v[1]; bf[t][2] = v[2]; bf[t][3] = v[3];
        } else {
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) bf[t][s2] = *(const DLLM_LDS float*)(Bs + mc_addr(c0, 8 * g + 4 * h + s2));
        }
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
          for (int u = 0; u < 4; ++u)
            acc[t >> 2][u >> 1][t & 3][u & 1] =
                __builtin_amdgcn_mfma_f32_16x16x4f32(bf[u][s2], af[t][s2], acc[t >> 2][u >> 1][t & 3][u & 1], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  epilogue_256<EPI, float, -1>(p, acc, m0, n0, wr, wc, lane, p.C);
}

// ----------------------------------------------------------------------------------------------
// generic bounds-checked kernel: any M/N/K, bf16 or fp32 inputs, fp32 FMA accumulation.
// 64x64 tile, 256 threads, 4x4 outputs per thread.
// ----------------------------------------------------------------------------------------------
template <int LAYOUT, int EPI, typename InT, typename OutT>
__global__ __launch_bounds__(256) void gemm_generic(GemmArgs p) {
  constexpr int T = 64, KT = 16;
  __shared__ float As[KT][T + 1];
  __shared__ float Bs[KT][T + 1];
  const int tid = threadIdx.x;
  const int m0 = blockIdx.y * T, n0 = blockIdx.x * T;
  constexpr bool A_KC = (LAYOUT != L_TN);
  constexpr bool B_KC = (LAYOUT == L_NT);
  const int ty = tid >> 4, tx = tid & 15;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < p.K; k0 += KT) {
    for (int e = tid; e < T * KT; e += 256) {
      const int mm = e / KT, kk = e % KT;
      const int gm = m0 + mm, gn = n0 + mm, gk = k0 + kk;
      float av = 0.f, bv = 0.f;
      if (gm < p.M && gk < p.K)
        av = ld1<InT>(p.A, A_KC ? (long)gm * p.lda + gk : (long)gk * p.lda + gm);
      if (gn < p.N && gk < p.K)
        bv = ld1<InT>(p.B, B_KC ? (long)gn * p.ldb + gk : (long)gk * p.ldb + gn);
      As[kk][mm] = av;
      Bs[kk][mm] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      float a[4], b[4];
      for (int i = 0; i < 4; ++i) a[i] = As[kk][ty * 4 + i];
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx * 4 + j];
      for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= p.M) continue;
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n >= p.N) continue;
      float v = acc[i][j];
      if constexpr (EPI == EPI_STORE) {
        v *= p.alpha;
        if (p.beta != 0.f) v += p.beta * ld1<OutT>(p.C, (long)m * p.ldc + n);
        st1<OutT>(p.C, (long)m * p.ldc + n, v);
      } else if constexpr (EPI == EPI_ACT) {
        if (p.aux_out) st1<OutT>(p.aux_out, (long)m * p.ldaux + n, v);
        st1<OutT>(p.C, (long)m * p.ldc + n, act_fwd(p.act, v));
      } else if constexpr (EPI == EPI_DACT) {
        v *= act_grad(p.act, ld1<OutT>(p.aux, (long)m * p.ldaux + n));
        st1<OutT>(p.C, (long)m * p.ldc + n, v);
      } else if constexpr (EPI == EPI_GLU) {
        // acc column n is interleaved; the partner lives in another thread -> store pre-acts only,
        // activation applied by glu_combine (host issues it) -- generic path is not perf-critical
        st1<OutT>(p.aux_out, (long)m * p.ldaux + n, v);
      } else if constexpr (EPI == EPI_DGLU) {
        const int blk = n >> 4, off = n & 15;
        const int ng = blk * 32 + off, nu = ng + 16;
        const float g = ld1<OutT>(p.aux, (long)m * p.ldaux + ng);
        const float u = ld1<OutT>(p.aux, (long)m * p.ldaux + nu);
        st1<OutT>(p.C, (long)m * p.ldc + nu, v * act_fwd(p.act, g));
        st1<OutT>(p.C, (long)m * p.ldc + ng, v * u * act_grad(p.act, g));
      } else if constexpr (EPI == EPI_SGD) {
        const long ci = (long)m * p.ldc + n;
        float* W = (float*)p.C;
        const float w = __fadd_rn(W[ci], __fmul_rn(-p.lr, __fmul_rn(p.alpha, v)));
        W[ci] = w;
        if (p.aux_out) st1<uint16_t>(p.aux_out, (long)m * p.ldaux + n, w);
      } else if constexpr (EPI == EPI_SGDS) {
        uint16_t* hp = (uint16_t*)p.aux_out + (long)m * p.ldaux + n;
        uint16_t* lp = (uint16_t*)p.C + (long)m * p.ldc + n;
        const float w = __fadd_rn(split_join(*hp, *lp), __fmul_rn(-p.lr, __fmul_rn(p.alpha, v)));
        split_part(w, *hp, *lp);
      } else if constexpr (EPI == EPI_ADAMS) {
        const long ci = (long)m * p.ldc + n;
        uint16_t* hp = (uint16_t*)p.aux_out + (long)m * p.ldaux + n;
        uint16_t* lp = (uint16_t*)p.C + ci;
        float w = split_join(*hp, *lp), mm = p.opt_m[ci], vv = p.opt_v[ci];
        adamw1(w, mm, vv, p.alpha * v, p.lr, p.b1, p.b2, p.eps, p.wd, p.bc1, p.bc2);
        split_part(w, *hp, *lp);
        p.opt_m[ci] = mm;
        p.opt_v[ci] = vv;
      } else if constexpr (EPI == EPI_ADAM) {
        const long ci = (long)m * p.ldc + n;
        float* W = (float*)p.C;
        const float g = p.alpha * v;
        const float mm = p.b1 * p.opt_m[ci] + (1.f - p.b1) * g;
        const float vv = p.b2 * p.opt_v[ci] + (1.f - p.b2) * g * g;
        const float w = W[ci] - p.lr * ((mm / p.bc1) / (sqrtf(vv / p.bc2) + p.eps) + p.wd * W[ci]);
        W[ci] = w;
        p.opt_m[ci] = mm;
        p.opt_v[ci] = vv;
        if (p.aux_out) st1<uint16_t>(p.aux_out, (long)m * p.ldaux + n, w);
      }
    }
  }
}

// a = act(g) * u from interleaved pre-activations (generic-path companion of EPI_GLU)
template <typename T>
__global__ void glu_combine(const T* h, long ldh, T* out, long ldo, int M, int Fh, int act) {
  const long total = (long)M * Fh;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = i / Fh, n = i % Fh;
    const int ng = (n >> 4) * 32 + (n & 15);
    const float g = ld1<T>(h, (long)m * ldh + ng), u = ld1<T>(h, (long)m * ldh + ng + 16);
    st1<T>(out, (long)m * ldo + n, act_fwd(act, g) * u);
  }
}

// ----------------------------------------------------------------------------------------------
// split-K reduction: sum the fp32 partials ws[0..S) and apply the real epilogue (any EPI / OutT)
// ----------------------------------------------------------------------------------------------
template <int EPI, typename OutT>
__global__ __launch_bounds__(256) void splitk_reduce(GemmArgs p, const float* ws, int S) {
  const long n4 = p.N / 4;
  const long total = (long)p.M * n4;
  const long plane = (long)p.M * p.N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i % n4) * 4;
    if constexpr (EPI == EPI_GLU) {
      if ((n & 31) >= 16) continue;  // the gate block's thread handles the pair (n, n+16)
      f32x4_t g = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < S; ++s) {
        g += *(const f32x4_t*)(ws + s * plane + (long)m * p.N + n);
        u += *(const f32x4_t*)(ws + s * plane + (long)m * p.N + n + 16);
      }
      epi_glu_pair<OutT>(p, m, (n >> 5) * 16 + (n & 15), n, n + 16, g, u);
    } else {
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < S; ++s) v += *(const f32x4_t*)(ws + s * plane + (long)m * p.N + n);
      if constexpr (EPI == EPI_DGLU) epi_dglu<OutT>(p, m, n, v);
      else epi4<EPI, OutT>(p, m, n, v);
    }
  }
}

#include "gemm_pp.h"

constexpr int MAX_DEV = 64;
inline int g_num_cu[MAX_DEV] = {};

static int num_cu() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEV) return 0;
  if (g_num_cu[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = -1;
    g_num_cu[dev] = n;
  }
  return g_num_cu[dev];
}

// grid of a persistent 8-phase launch over nb tile slots; sets a.tpb (1: launch the one-tile kernel instead).
// Persistent grids are a multiple of the 8 XCDs (every slot of a block maps to the block's own XCD).
// Tiles per block t <= tpb_req, and <= ceil(nb / (ncu * min_bpc)) (blocks enough to leave CUs to collectives: the grid
// then has ~min_bpc blocks per CU -- nb / t rounded, so e.g. 1000 tiles at min_bpc 2 run as 504 blocks of <= 2
// tiles, 1.97 per CU; "min_bpc" bounds tiles per block, it is not a strict floor on blocks per CU), chosen
// to minimise the makespan in tile-times, ceil(blocks / ncu) * ceil(nb / blocks) (one block per CU: 128 KiB
// LDS); ties go to fewer blocks.  E.g. 1792 tiles on 256 CUs: 256 blocks x 7 tiles = 7 tile-times, where a
// fixed 4 per block (448 blocks in two rounds) takes 8.
static int grid_8ph(GemmArgs& a, int nb) {
  a.tpb = 1;
  const int ncu = num_cu();
  if (a.tpb_req <= 1 || ncu <= 0) return nb;
  const int per = ncu * std::max(1, a.min_bpc);
  const int tmax = std::min(a.tpb_req, (nb + per - 1) / per);
  auto makespan = [&](long g) { return ((g + ncu - 1) / ncu) * ((nb + g - 1) / g); };
  int best_g = nb;
  long best = makespan(nb);
  for (int t = 2; t <= tmax; ++t) {
    const int g = ((nb + t - 1) / t + 7) / 8 * 8;
    if (g >= nb) continue;
    const long m = makespan(g);
    if (m < best || (m == best && g < best_g)) {
      best = m;
      best_g = g;
    }
  }
  if (best_g >= nb) return nb;
  a.tpb = (nb + best_g - 1) / best_g;
  return best_g;
}

// grid of a persistent 256x128 (gemm_bf16_pp) launch over nb tile slots: two blocks per CU (80 KiB LDS each), so the
// makespan in tile-times is ceil(blocks / (2 ncu)) * ceil(nb / blocks); at least max(2, min_bpc) blocks per CU.  Sets
// a.tpb (1: one block per tile).  A slot needs >= 2 K-tiles for the cross-slot prefetch (K-tiles nk, nk+1 = the next
// slot's 0, 1).
static int grid_pp(GemmArgs& a, int nb, int nk) {
  a.tpb = 1;
  const int ncu = num_cu();
  if (a.tpb_req <= 1 || ncu <= 0 || nk < 2) return nb;
  const long cap = 2L * ncu;
  const int per = ncu * std::max(2, a.min_bpc);
  const int tmax = std::min(a.tpb_req, (nb + per - 1) / per);
  auto makespan = [&](long g) { return ((g + cap - 1) / cap) * ((nb + g - 1) / g); };
  int best_g = nb;
  long best = makespan(nb);
  for (int t = 2; t <= tmax; ++t) {
    const int g = ((nb + t - 1) / t + 7) / 8 * 8;
    if (g >= nb) continue;
    const long m = makespan(g);
    if (m < best || (m == best && g < best_g)) {
      best = m;
      best_g = g;
    }
  }
  if (best_g >= nb) return nb;
  a.tpb = (nb + best_g - 1) / best_g;
  return best_g;
}

// gemm_bf16_pp launch: persistent where the 8-phase family is (persistent_kernel), else one block per tile
template <int L, int E, typename OutT, int ACT>
constexpr bool persistent_kernel();
template <int L, int E, typename OutT, int ACT>
static void launch_pp_act(const GemmArgs& a0, hipStream_t s) {
  const int nb0 = (a0.M / BT_M) * (a0.N / PP_BN) * a0.ksplit;
  if constexpr (persistent_kernel<L, E, OutT, ACT>()) {
    GemmArgs a = a0;
    const int nb = grid_pp(a, nb0, a0.K / BT_K / a0.ksplit);
    if (a.tpb > 1) {
      hipLaunchKernelGGL((gemm_bf16_pp<L, E, OutT, ACT, true>), dim3(nb), dim3(256), 0, s, a);
      return;
    }
  }
  GemmArgs a = a0;
  a.tpb = 1;
  hipLaunchKernelGGL((gemm_bf16_pp<L, E, OutT, ACT>), dim3(nb0), dim3(256), 0, s, a);
}
template <int L, int E, typename OutT, int NPH>
static void launch_8ph_stagger(const GemmArgs& a, int nb, hipStream_t s);
template <int L, int E, typename OutT>
static void launch_pp(const GemmArgs& a, hipStream_t s) {
  // every bf16 activation epilogue (NT / NN) on a compile-time activation: the runtime-activation pp kernels kept
  // their accumulators in scratch (utils/kernel_resources.py)
  constexpr bool actepi = L != L_TN && (E == EPI_ACT || E == EPI_GLU || E == EPI_DACT || E == EPI_DGLU);
  if constexpr (actepi && !std::is_same<OutT, uint16_t>::value) {
    // fp32-output activation epilogues (the bf16x6 fp32 path) stay on the 8-phase kernel: the runtime-activation pp
    // kernels kept their accumulators in scratch
    launch_8ph_stagger<L, E, OutT, 8>(a, (a.M / BT_M) * (a.N / BT_N), s);
    return;
  } else if constexpr (actepi) {
    switch (a.act) {
      case ACT_RELU: launch_pp_act<L, E, OutT, ACT_RELU>(a, s); return;
      case ACT_SILU: launch_pp_act<L, E, OutT, ACT_SILU>(a, s); return;
      case ACT_GELU: launch_pp_act<L, E, OutT, ACT_GELU>(a, s); return;
      default: return;   // unreachable: dllm_gemm rejects other activations (no runtime-activation bf16 kernel)
    }
  } else {
    launch_pp_act<L, E, OutT, -1>(a, s);
  }
}

// main kernel writes partials into the workspace, then the reduction applies the epilogue
template <int L, int E>
static hipError_t launch_splitk(const GemmArgs& a, int out_dt, float* ws, hipStream_t s) {
  GemmArgs w = a;
  w.C = ws;
  w.ldc = a.N;
  w.alpha = 1.f;
  w.beta = 0.f;
  const int nb = (a.M / BT_M) * (a.N / BT_N) * a.ksplit;
  w.tpb = 1;
  if (a.variant == 5) launch_pp<L, EPI_STORE, float>(w, s);
  else if (a.variant == 4) hipLaunchKernelGGL((gemm_bf16_8ph<L, EPI_STORE, float, true, -1, 4>), dim3(nb), dim3(512), 0, s, w);
  else hipLaunchKernelGGL((gemm_bf16_8ph<L, EPI_STORE, float, true>), dim3(nb), dim3(512), 0, s, w);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  long n4 = (long)a.M * (a.N / 4);
  int g = (int)std::min<long>((n4 + 255) / 256, 4096);
  if (out_dt == DT_F32) hipLaunchKernelGGL((splitk_reduce<E, float>), dim3(g), dim3(256), 0, s, a, ws, a.ksplit);
  else hipLaunchKernelGGL((splitk_reduce<E, uint16_t>), dim3(g), dim3(256), 0, s, a, ws, a.ksplit);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------------------------

// staggered 8-phase launch; the FFN's own activation epilogues (NT act/glu forward, NN dact/dglu
// dgrad, bf16 out) get a compile-time activation, everything else the runtime switch
// Persistent instantiations exist where they measured faster end to end (profiles/persistent_blocks_r1.log):
// the ReLU FFN's GEMMs -- bf16 forward / dgrad with a compile-time ReLU epilogue or a plain store -- and the
// weight-gradient GEMMs (stored gradients, fused SGD).  Gated (GLU/DGLU), SiLU/GELU and fused-AdamW epilogues
// stay one tile per block: their heavier in-loop epilogues measured 2 % slower persistent.
template <int L, int E, typename OutT, int ACT>
constexpr bool persistent_kernel() {
  constexpr bool bf = std::is_same<OutT, uint16_t>::value;
  if constexpr (E == EPI_ADAMS_T) return DLLM_ADAMS_T_PERS;   // fused AdamW: one tile per block (see above)
  if constexpr (E == EPI_STORE_DT || E == EPI_STORE_T || E == EPI_SGDS_T) return true;
  if constexpr (L == L_NN && E == EPI_SGDS) return true;   // the NN weight-gradient layout (dispatch_x)
  // gated (SwiGLU) stacks: the GLU forward / DGLU dgrad with a compile-time activation (round 3)
  // NT dgrad with the ReLU mask: W2 stored as W2ᵀ (the nn_w2t weight-gradient mode, parallel/engine.py)
  if constexpr (L == L_NT)
    return bf && ((E == EPI_ACT && ACT == ACT_RELU) || E == EPI_STORE || (E == EPI_GLU && ACT >= 0) ||
                  (E == EPI_DACT && ACT == ACT_RELU) || (E == EPI_DGLU && ACT >= 0));
  if constexpr (L == L_NN) return bf && ((E == EPI_DACT && ACT == ACT_RELU) || E == EPI_STORE || (E == EPI_DGLU && ACT >= 0));
  return E == EPI_STORE || E == EPI_SGD || E == EPI_SGDS;
}

// The NN weight-gradient layout's GEMMs (round 5; 8-phase 256x256 tiles, K % 128 == 0, no split-K): NN fused SGD on
// a split master (dW2 = dyᵀ·a with dyᵀ [D, T] K-contiguous), NN with a transposed output (dW1ᵀ = xᵀ·da into W1
// [F, D]: EPI_SGDS_T / EPI_STORE_T), and plain stores that also write a transposed copy (EPI_STORE_DT, NT y or NN dx).
template <int L>
static hipError_t dispatch_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s) {
  const int nb = (a.M / BT_M) * (a.N / BT_N);
  const bool f32 = out_dt == DT_F32;
  switch (epi) {
    case EPI_STORE_DT:
      if (f32) return hipErrorInvalidValue;
      launch_8ph_act<L, EPI_STORE_DT, uint16_t, -1, 8>(a, nb, s);
      break;
    case EPI_STORE_T:   // any layout (the NT / TN instantiations serve operand-order experiments and tests)
      if (f32) launch_8ph_act<L, EPI_STORE_T, float, -1, 8>(a, nb, s);
      else launch_8ph_act<L, EPI_STORE_T, uint16_t, -1, 8>(a, nb, s);
      break;
    case EPI_SGDS_T:
    case EPI_SGDS:
    case EPI_ADAMS_T:
    case EPI_ADAMS:
      if constexpr (L == L_NN) {
        if (epi == EPI_SGDS) launch_8ph_act<L, EPI_SGDS, float, -1, 8>(a, nb, s);
        else if (epi == EPI_SGDS_T) launch_8ph_act<L, EPI_SGDS_T, float, -1, 8>(a, nb, s);
        else if (epi == EPI_ADAMS) launch_8ph_act<L, EPI_ADAMS, float, -1, 8>(a, nb, s);
        else launch_8ph_act<L, EPI_ADAMS_T, float, -1, 8>(a, nb, s);
        break;
      } else if constexpr (L == L_TN) {   // W2 stored transposed with TN weight gradients (--w2_storage transposed)
        if (epi == EPI_SGDS_T) launch_8ph_act<L, EPI_SGDS_T, float, -1, 8>(a, nb, s);
        else if (epi == EPI_ADAMS_T) launch_8ph_act<L, EPI_ADAMS_T, float, -1, 8>(a, nb, s);
        else return hipErrorInvalidValue;
        break;
      } else {
        return hipErrorInvalidValue;
      }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int L, int E, typename OutT, int ACT, int NPH>
static void launch_8ph_act(const GemmArgs& a0, int nb0, hipStream_t s) {
  if constexpr (NPH == 8 && persistent_kernel<L, E, OutT, ACT>()) {
    GemmArgs a = a0;
    const int nb = grid_8ph(a, nb0);
    if (a.tpb > 1) {
      hipLaunchKernelGGL((gemm_bf16_8ph<L, E, OutT, true, ACT, NPH, true>), dim3(nb), dim3(512), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_bf16_8ph<L, E, OutT, true, ACT, NPH>), dim3(nb0), dim3(512), 0, s, a0);
}

template <int L, int E, typename OutT, int NPH>
static void launch_8ph_stagger(const GemmArgs& a, int nb, hipStream_t s) {
  constexpr bool fwd = L == L_NT && (E == EPI_ACT || E == EPI_GLU);
  constexpr bool bwd = (L == L_NN && (E == EPI_DACT || E == EPI_DGLU)) ||
                       (L == L_NT && (E == EPI_DACT || E == EPI_DGLU) && NPH == 8);
  if constexpr ((fwd || bwd) && std::is_same<OutT, uint16_t>::value) {
    switch (a.act) {
      case ACT_RELU: launch_8ph_act<L, E, OutT, ACT_RELU, NPH>(a, nb, s); return;
      case ACT_SILU: launch_8ph_act<L, E, OutT, ACT_SILU, NPH>(a, nb, s); return;
      case ACT_GELU: launch_8ph_act<L, E, OutT, ACT_GELU, NPH>(a, nb, s); return;
      default: return;   // unreachable: dllm_gemm rejects other activations (no runtime-activation bf16 kernel)
    }
  } else {
    launch_8ph_act<L, E, OutT, -1, NPH>(a, nb, s);
  }
}

template <int L, int E>
static hipError_t launch_bf16(const GemmArgs& a, int out_dt, hipStream_t s) {
  if (a.ksplit > 1) return launch_splitk<L, E>(a, out_dt, a.ws, s);
  const int nb = (a.M / BT_M) * (a.N / BT_N);
  int v = a.variant;
  if (v == 0) v = (a.K % (2 * BT_K) == 0) ? 3 : 1;
  if (v >= 2 && a.K % (2 * BT_K) != 0) v = 1;
  const bool f32 = out_dt == DT_F32;
  if (a.variant == 5) {  // 256x128 tiles, two blocks per CU (gemm_pp.h)
    if (f32) launch_pp<L, E, float>(a, s);
    else launch_pp<L, E, uint16_t>(a, s);
    return hipGetLastError();
  }
  if (v == 1) {
    if (f32) hipLaunchKernelGGL((gemm_bf16_256<L, E, float>), dim3(nb), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((gemm_bf16_256<L, E, uint16_t>), dim3(nb), dim3(512), 0, s, a);
  } else if (v == 2) {
    if (f32) hipLaunchKernelGGL((gemm_bf16_8ph<L, E, float, false>), dim3(nb), dim3(512), 0, s, a);
    else hipLaunchKernelGGL((gemm_bf16_8ph<L, E, uint16_t, false>), dim3(nb), dim3(512), 0, s, a);
  } else if (v == 4) {
    if (f32) launch_8ph_stagger<L, E, float, 4>(a, nb, s);
    else launch_8ph_stagger<L, E, uint16_t, 4>(a, nb, s);
  } else {
    if (f32) launch_8ph_stagger<L, E, float, 8>(a, nb, s);
    else launch_8ph_stagger<L, E, uint16_t, 8>(a, nb, s);
  }
  return hipGetLastError();
}
template <int L, int E>
static hipError_t launch_f32(const GemmArgs& a, hipStream_t s) {
  if (DLLM_F32_256 && a.M % F2_T == 0 && a.N % F2_T == 0 && a.K % F2_K == 0) {
    hipLaunchKernelGGL((gemm_f32_256<L, E>), dim3((a.M / F2_T) * (a.N / F2_T)), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  const int nb = (a.M / FT) * (a.N / FT);
  hipLaunchKernelGGL((gemm_f32_128<L, E>), dim3(nb), dim3(256), 0, s, a);
  return hipGetLastError();
}
template <int L, int E>
static hipError_t launch_generic(const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
  dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
  if (in_dt == DT_BF16 && out_dt == DT_BF16)
    hipLaunchKernelGGL((gemm_generic<L, E, uint16_t, uint16_t>), grid, dim3(256), 0, s, a);
  else if (in_dt == DT_BF16)
    hipLaunchKernelGGL((gemm_generic<L, E, uint16_t, float>), grid, dim3(256), 0, s, a);
  else if (out_dt == DT_BF16)
    hipLaunchKernelGGL((gemm_generic<L, E, float, uint16_t>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gemm_generic<L, E, float, float>), grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int L>
static hipError_t dispatch_epi(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s) {
#define DLLM_EPI_CASE(E)                                            \
  case E:                                                           \
    if (path == 0) return launch_bf16<L, E>(a, out_dt, s);          \
    if (path == 1) return launch_f32<L, E>(a, s);                   \
    if (path == 3) return launch_m224<L, E>(a, out_dt, s);          \
    return launch_generic<L, E>(a, in_dt, out_dt, s);
  if constexpr (L == L_TN) {   // weight gradients: store (fused optimizers: dispatch_opt); no activation epilogues
    switch (epi) {
      DLLM_EPI_CASE(EPI_STORE)
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (epi) {
      DLLM_EPI_CASE(EPI_STORE)
      DLLM_EPI_CASE(EPI_ACT)
      DLLM_EPI_CASE(EPI_DACT)
      DLLM_EPI_CASE(EPI_GLU)
      DLLM_EPI_CASE(EPI_DGLU)
      default: return hipErrorInvalidValue;
    }
  }
#undef DLLM_EPI_CASE
}

// weight-gradient GEMMs with a fused optimizer epilogue: TN layout, fp32 master output only
template <int E>
static hipError_t dispatch_opt(int path, const GemmArgs& a, int in_dt, hipStream_t s) {
  if (path == 0 && a.ksplit > 1) return launch_splitk<L_TN, E>(a, DT_F32, a.ws, s);
  if (path == 0) {
    const int nb = (a.M / BT_M) * (a.N / BT_N);
    if (a.variant == 5)
      launch_pp<L_TN, E, float>(a, s);
    else if (a.K % (2 * BT_K) == 0 && a.variant == 4)
      hipLaunchKernelGGL((gemm_bf16_8ph<L_TN, E, float, true, -1, 4>), dim3(nb), dim3(512), 0, s, a);
    else if (a.K % (2 * BT_K) == 0 && a.variant != 1)
      launch_8ph_act<L_TN, E, float, -1, 8>(a, nb, s);
    else
      hipLaunchKernelGGL((gemm_bf16_256<L_TN, E, float>), dim3(nb), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  dim3 grid((a.N + 63) / 64, (a.M + 63) / 64);
  if constexpr (E == EPI_SGDS || E == EPI_ADAMS) {  // split masters exist only next to a bf16 working copy
    if (path == 1 || in_dt != DT_BF16) return hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm_generic<L_TN, E, uint16_t, float>), grid, dim3(256), 0, s, a);
  } else {
    if (path == 1) return launch_f32<L_TN, E>(a, s);
    if (in_dt == DT_BF16) hipLaunchKernelGGL((gemm_generic<L_TN, E, uint16_t, float>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((gemm_generic<L_TN, E, float, float>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}


// grouped weight-gradient pair (gemm_bf16_8ph_pair): one tile per block, any wgrad epilogue.  TN (256-row tiles) or NN
// with 224-row tiles (the transposed-activation TP layout, models/ffn.py: dW2ᵀ = aᵀ·dy and dW1 = daᵀ·x, M = F/tp)
template <int L, int E, typename OutT, int BM>
static hipError_t launch_pair(const GemmArgs& a0, const GemmArgs& a1, hipStream_t s) {
  const int nb = (a0.M / BM) * (a0.N / BT_N) + (a1.M / BM) * (a1.N / BT_N);
  hipLaunchKernelGGL((gemm_bf16_8ph_pair<L, E, OutT, BM>), dim3(nb), dim3(512), 0, s, a0, a1);
  return hipGetLastError();
}
template <int L, int BM>
static hipError_t dispatch_pair(int epi, const GemmArgs& a0, const GemmArgs& a1, int out_dt, hipStream_t s) {
  switch (epi) {
    case EPI_STORE:
      return out_dt == DT_F32 ? launch_pair<L, EPI_STORE, float, BM>(a0, a1, s)
                              : launch_pair<L, EPI_STORE, uint16_t, BM>(a0, a1, s);
    case EPI_SGD: return launch_pair<L, EPI_SGD, float, BM>(a0, a1, s);
    case EPI_SGDS: return launch_pair<L, EPI_SGDS, float, BM>(a0, a1, s);
    case EPI_ADAM: return launch_pair<L, EPI_ADAM, float, BM>(a0, a1, s);
    case EPI_ADAMS: return launch_pair<L, EPI_ADAMS, float, BM>(a0, a1, s);
    default: return hipErrorInvalidValue;
  }
}

// single GEMM on 224-row tiles (path 3): NT / NN, the FFN's forward / dgrad activation epilogues with a compile-time
// ReLU (others: runtime activation), plain stores and the fused optimizers
template <int L, int E>
static hipError_t launch_m224(const GemmArgs& a, int out_dt, hipStream_t s) {
  if constexpr (L == L_TN || E == EPI_GLU || E == EPI_DGLU) {
    return hipErrorInvalidValue;
  } else {
    const int nb = (a.M / 224) * (a.N / BT_N);
    constexpr bool opt = E == EPI_SGD || E == EPI_SGDS || E == EPI_ADAM || E == EPI_ADAMS;
    if constexpr (opt) {
      hipLaunchKernelGGL((gemm_bf16_8ph_m224<L, E, float>), dim3(nb), dim3(512), 0, s, a);
    } else {
      if (out_dt == DT_F32)
        hipLaunchKernelGGL((gemm_bf16_8ph_m224<L, E, float>), dim3(nb), dim3(512), 0, s, a);
      else if ((E == EPI_ACT || E == EPI_DACT) && a.act == ACT_RELU)
        hipLaunchKernelGGL((gemm_bf16_8ph_m224<L, E, uint16_t, ACT_RELU>), dim3(nb), dim3(512), 0, s, a);
      else
        hipLaunchKernelGGL((gemm_bf16_8ph_m224<L, E, uint16_t>), dim3(nb), dim3(512), 0, s, a);
    }
    return hipGetLastError();
  }
}

// per-layout entry points (one translation unit each)
hipError_t dispatch_nt(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s);
hipError_t dispatch_nn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s);
hipError_t dispatch_tn(int path, int epi, const GemmArgs& a, int in_dt, int out_dt, hipStream_t s);
hipError_t dispatch_tn_opt(int path, int epi, const GemmArgs& a, int in_dt, hipStream_t s);
hipError_t dispatch_tn_pair(int epi, const GemmArgs& a0, const GemmArgs& a1, int out_dt, hipStream_t s);
hipError_t dispatch_nn_pair(int epi, const GemmArgs& a0, const GemmArgs& a1, int out_dt, hipStream_t s);
hipError_t dispatch_nn_opt(int epi, const GemmArgs& a, hipStream_t s);
hipError_t dispatch_nt_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s);
hipError_t dispatch_nn_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s);
hipError_t dispatch_tn_x(int epi, const GemmArgs& a, int out_dt, hipStream_t s);

}  // namespace dllm
