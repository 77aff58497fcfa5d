// Shared device/host helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
// Written directly for CDNA4: 64-lane waves, MFMA, LDS-DMA (global_load_lds), no CUDA shims.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dllm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

#define DLLM_LDS __attribute__((address_space(3)))
#define DLLM_GLB __attribute__((address_space(1)))

// ---- dtype / enum codes shared with the Python side (ops/_native.py) ----
enum DType : int { DT_BF16 = 0, DT_F32 = 1 };
enum Layout : int { L_NT = 0, L_NN = 1, L_TN = 2 };
// Epilogues fused into the GEMM (reference ops they replace: train_ffns.py:42,45,48,51).
//   EPI_STORE : C = alpha*acc (+ beta*C)                       plain linear fwd / dgrad / wgrad
//   EPI_ACT   : C = act(acc); aux_out = acc (pre-activation)  linear + activation fwd (K1+K2)
//   EPI_DACT  : C = acc * act'(aux)                            dgrad + activation bwd mask (K5+K6)
//   EPI_GLU   : gated: acc tiles of W1/W3 interleaved by 16 rows; C = act(h1)*h3; aux_out = [h1|h3]
//   EPI_DGLU  : gated bwd: C(16-col interleaved [dh1|dh3]) from acc = da and aux = interleaved [h1|h3]
//   EPI_SGD   : weight-gradient GEMM fused with the SGD update: C (fp32 master) += -lr*alpha*acc,
//               aux_out (bf16 working copy, nullable) = bf16(C)   (train_ffns.py:114,172 fused)
//   EPI_ADAM  : same with AdamW (moments m/v share C's layout)
//   EPI_SGDS  : EPI_SGD on a split master (below): C = the 16-bit residual plane, aux_out = the bf16 working copy
//               (required); reads 4 B and writes 4 B per parameter instead of reading 4 B and writing 6 B
//   EPI_ADAMS : EPI_ADAM on a split master (the moments stay fp32)
// Transposed outputs (round 5, the NN weight-gradient layout; 8-phase 256x256 kernels only):
//   EPI_SGDS_T : EPI_SGDS of Cᵀ: the GEMM's [M, N] result updates a split master stored [N, M] (C / aux_out ld'd
//                as N rows of M), e.g. dW1ᵀ = xᵀ·da into W1 [F, D]; the MFMA operands are swapped so each lane
//                holds 4 consecutive M (paired 16-B accesses as EPI_SGDS)
//   EPI_STORE_T : EPI_STORE of Cᵀ (beta = 0), same operand order
//   EPI_STORE_DT: EPI_STORE (beta = 0, bf16) plus a transposed copy Cᵀ [N, M] into aux_out (ldaux), e.g. a layer's
//                 output y and its yᵀ for the next layer's NN weight gradient
//   EPI_ADAMS_T : EPI_ADAMS of Cᵀ (moments in the master's transposed layout)
enum Epi : int { EPI_STORE = 0, EPI_ACT = 1, EPI_DACT = 2, EPI_GLU = 3, EPI_DGLU = 4, EPI_SGD = 5, EPI_ADAM = 6,
                 EPI_SGDS = 7, EPI_ADAMS = 8, EPI_SGDS_T = 9, EPI_STORE_T = 10, EPI_STORE_DT = 11, EPI_ADAMS_T = 12 };
__host__ __device__ constexpr bool epi_tout(int e) { return e == EPI_SGDS_T || e == EPI_STORE_T || e == EPI_ADAMS_T; }
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SILU = 2, ACT_GELU = 3 };

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ uint16_t f2bf(float f) {
  // plain cast -> v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// Split fp32 master weights.  The fp32 master w is stored as two 16-bit planes: hi = its bf16 working copy (the
// GEMM operand), rounded half away from zero, and lo = the signed residual, so that
//   bits(w) = (hi << 16) + sext(lo)      (mod 2^32; lossless for every bit pattern)
// with t = bits(w) + 0x8000: hi = t >> 16, lo = (t & 0xffff) ^ 0x8000.  The master stays exactly the fp32 value
// the unsplit update computes; only the working copy's rounding differs from RNE, on exact ties.  (A NaN with
// payload bits >= 0xffff8000 keeps its master bits but gets hi = +0.)  Word forms: two elements per 32-bit word,
// element 0 in bits 0-15.
__device__ __forceinline__ void split_join2(uint32_t wh, uint32_t wl, float& f0, float& f1) {
  f0 = __uint_as_float((wh << 16) + (uint32_t)((int32_t)(wl << 16) >> 16));
  f1 = __uint_as_float((wh & 0xffff0000u) + (uint32_t)((int32_t)wl >> 16));
}
__device__ __forceinline__ void split_part2(float f0, float f1, uint32_t& wh, uint32_t& wl) {
  const uint32_t t0 = __float_as_uint(f0) + 0x8000u, t1 = __float_as_uint(f1) + 0x8000u;
  wh = (t0 >> 16) | (t1 & 0xffff0000u);
  wl = ((t0 ^ 0x8000u) & 0xffffu) | ((t1 ^ 0x8000u) << 16);
}
__device__ __forceinline__ float split_join(uint16_t h, uint16_t l) {
  return __uint_as_float(((uint32_t)h << 16) + (uint32_t)(int32_t)(int16_t)l);
}
__device__ __forceinline__ void split_part(float f, uint16_t& h, uint16_t& l) {
  const uint32_t t = __float_as_uint(f) + 0x8000u;
  h = (uint16_t)(t >> 16);
  l = (uint16_t)((t ^ 0x8000u) & 0xffffu);
}

// the AdamW update of one parameter (shared by every AdamW epilogue / kernel)
__device__ __forceinline__ void adamw1(float& w, float& m, float& v, float g, float lr, float b1, float b2, float eps,
                                       float wd, float bc1, float bc2) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  const float mh = m / bc1, vh = v / bc2;
  w = w - lr * (mh / (sqrtf(vh) + eps) + wd * w);
}

__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_SILU: return x / (1.f + __expf(-x));
    case ACT_GELU: {  // tanh approximation (torch gelu(approximate='tanh'))
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float u = k0 * (x + k1 * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    default: return x;
  }
}
// derivative d act / d x evaluated at pre-activation x
__device__ __forceinline__ float act_grad(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case ACT_SILU: {
      float s = 1.f / (1.f + __expf(-x));
      return s * (1.f + x * (1.f - s));
    }
    case ACT_GELU: {
      const float k0 = 0.7978845608028654f, k1 = 0.044715f;
      float x2 = x * x;
      float u = k0 * (x + k1 * x2 * x);
      float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x2);
    }
    default: return 1.f;
  }
}

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5, T1): blocks that the
// dispatcher deals round-robin to the 8 XCDs get contiguous ranges of logical ids, so tiles that
// share operand panels run on one XCD and hit its private L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  int xcd = bid % nx, q = nwg / nx, r = nwg % nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / nx;
}

}  // namespace dllm
