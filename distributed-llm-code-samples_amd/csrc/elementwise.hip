// Memory-bound kernels: device mock-data RNG, fused optimizers over flat buffers, casts.
//
// * dllm_rng_normal   : Philox4x32-10 + Box-Muller, writes N(0,1)*scale as fp32 (32-bit uniforms) or bf16 (16-bit
//                       uniforms, 8 normals per Philox call), 16-B stores.
//                       Replaces the reference's per-step CPU torch.randn (mock_data, train_ffns.py:144-151;
//                       ≈430 ms/step on the host at T=8192,D=4096) for throughput mode.
// * dllm_rng_normal_bf16_t : the bf16 draw of a [R, C] tensor and its transpose in one pass (NN-layout inputs).
// * dllm_sgd_step     : master -= lr*g (fp32 master, fp32/bf16 grad), refreshes the bf16 working copy.
//                       Replaces param.add_(-LR*grad) (train_ffns.py:172,259,312) / p-LR*g (:114).
// * dllm_adam_step    : fused AdamW (north-star optimizer), same flat-buffer contract.
// * dllm_cast         : fp32 <-> bf16.
// * dllm_split3       : exact three-way bf16 split of an fp32 GEMM operand (the fp32-accurate bf16x6 GEMM).
// All kernels: grid-stride, 4 elements per lane per iteration (16-B fp32 / 8-B bf16 accesses),
// grid capped at 256 CUs x 8 blocks (cdna_hip_programming.md Guideline 11).
#include <algorithm>

#include "common.h"

namespace dllm {

// rounds of the mock-data Philox (build-time: 10 = Random123's default Philox4x32-10)
#ifndef DLLM_PHILOX_ROUNDS
#define DLLM_PHILOX_ROUNDS 10
#endif
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint2 k) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < DLLM_PHILOX_ROUNDS; ++r) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of separate mul_lo / mul_hi
    const uint64_t p0 = (uint64_t)M0 * c.x, p1 = (uint64_t)M1 * c.z;
    const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
    const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += W0;
    k.y += W1;
  }
  return c;
}

// Box-Muller on the hardware transcendentals: v_log_f32 is log2 (so -2 ln u1 = -2 ln2 * log2 u1), v_sqrt_f32, and
// v_sin_f32 / v_cos_f32 take their argument in revolutions -- u2 in [0, 1) is already one, so no 2*pi scaling and no
// range reduction (the libm-style __sincosf path reduced the argument first).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float u1 = ((float)a + 1.0f) * 2.3283064365386963e-10f;  // (0, 1]
  const float u2 = (float)b * 2.3283064365386963e-10f;           // [0, 1) revolutions
  const float r = __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(u2);
  z1 = r * __builtin_amdgcn_sinf(u2);
}

// bf16 outputs carry 8 mantissa bits, so each 32-bit Philox word is split into two 16-bit uniforms: one Philox call
// feeds 4 Box-Muller pairs (8 normals, one 16-B store) instead of 2 -- half the 64-bit multiplies per output.  The
// uniforms are made exactly from the bits: 1 + a/2^16 = as_float(0x3f800000 | a << 7), so u1 = 2 - that in (0, 1],
// u2 = that - 1 in [0, 1).  A 16-bit u1 cuts the radius at sqrt(-2 ln 2^-16) = 4.71 sigma (P(|z| > 4.71) = 2.5e-6).
__device__ __forceinline__ void box_muller16(uint32_t a, uint32_t b, float s, float& z0, float& z1) {
  const float u1 = 2.0f - __builtin_bit_cast(float, 0x3f800000u | (a << 7));
  const float u2 = __builtin_bit_cast(float, 0x3f800000u | (b << 7)) - 1.0f;
  const float r = s * __builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1));
  z0 = r * __builtin_amdgcn_cosf(u2);
  z1 = r * __builtin_amdgcn_sinf(u2);
}

__global__ __launch_bounds__(256) void rng_normal_bf16_kernel(uint16_t* out, long n, uint64_t seed, uint64_t offset,
                                                              float scale, const unsigned long long* seed_dev) {
  if (seed_dev) seed = *seed_dev;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const long n8 = (n + 7) / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const uint4 ctr = make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)offset, (uint32_t)(offset >> 32));
    const uint4 r = philox4x32_10(ctr, key);
    float z[8];
    // pairs (lo16, hi16) of each word, words in order: outputs 8i..8i+7
    box_muller16(r.x & 0xffffu, r.x >> 16, scale, z[0], z[1]);
    box_muller16(r.y & 0xffffu, r.y >> 16, scale, z[2], z[3]);
    box_muller16(r.z & 0xffffu, r.z >> 16, scale, z[4], z[5]);
    box_muller16(r.w & 0xffffu, r.w >> 16, scale, z[6], z[7]);
    const long base = i * 8;
    if (base + 8 <= n) {
      uint4 u;
      u.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
      u.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
      u.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
      u.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
      *(uint4*)(out + base) = u;
    } else {
      for (int j = 0; j < 8 && base + j < n; ++j) out[base + j] = f2bf(z[j]);
    }
  }
}

// Two bf16 draws of equal size in one launch (the step's x and dy; blockIdx.y picks the tensor), each bitwise the
// rng_normal_bf16_kernel draw with its own stream offset and scale.  32-bit element-group indices (n / 8 < 2^31, checked
// by the host) and the partial last group outside the loop: the flat kernel's 64-bit index arithmetic and per-group
// bounds test are a tenth of its instructions, and the draw is ALU-bound.
__global__ __launch_bounds__(256) void rng_normal_bf16_pair_kernel(uint16_t* out0, uint16_t* out1, long n,
                                                                   uint64_t seed, uint64_t off0, uint64_t off1,
                                                                   float scale0, float scale1,
                                                                   const unsigned long long* seed_dev) {
  if (seed_dev) seed = *seed_dev;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const bool second = blockIdx.y != 0;
  uint16_t* out = second ? out1 : out0;
  const uint64_t offset = second ? off1 : off0;
  const float scale = second ? scale1 : scale0;
  const uint32_t full = (uint32_t)(n / 8), stride = gridDim.x * blockDim.x;
  auto draw8 = [&](uint32_t i, float (&z)[8]) {
    const uint4 r = philox4x32_10(make_uint4(i, 0u, (uint32_t)offset, (uint32_t)(offset >> 32)), key);
    box_muller16(r.x & 0xffffu, r.x >> 16, scale, z[0], z[1]);
    box_muller16(r.y & 0xffffu, r.y >> 16, scale, z[2], z[3]);
    box_muller16(r.z & 0xffffu, r.z >> 16, scale, z[4], z[5]);
    box_muller16(r.w & 0xffffu, r.w >> 16, scale, z[6], z[7]);
  };
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < full; i += stride) {
    float z[8];
    draw8(i, z);
    uint4 u;
    u.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
    u.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
    u.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
    u.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
    *(uint4*)(out + 8 * (long)i) = u;
  }
  if ((long)full * 8 < n && blockIdx.x == 0 && threadIdx.x == 0) {
    float z[8];
    draw8(full, z);
    for (long j = 0; (long)full * 8 + j < n; ++j) out[(long)full * 8 + j] = f2bf(z[j]);
  }
}

// rng_normal_bf16_kernel's values for a [R, C] row-major tensor (C % 64 == 0, R % 64 == 0), written both as ``out``
// [R, C] and as its transpose ``out_t`` [C, R]: the NN weight-gradient layout's xᵀ / dyᵀ of the step's inputs come
// out of the draw instead of a separate transpose (a 64x64 tile per block: two Philox calls per lane, the 16-B row
// stores, then the LDS gather and 16-B column stores of transpose_bf16_kernel).  Philox counter of the 8 elements at
// (r, c..c+7) is (r*C + c)/8, as in the flat kernel, so both outputs are bitwise the flat draw + transpose.
__global__ __launch_bounds__(256) void rng_normal_bf16_t_kernel(uint16_t* __restrict__ out, long C,
                                                                uint16_t* __restrict__ out_t, long R, uint64_t seed,
                                                                uint64_t offset, float scale,
                                                                const unsigned long long* seed_dev) {
  __shared__ uint32_t sh[64 * 33];
  if (seed_dev) seed = *seed_dev;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const int t = threadIdx.x;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = t / 8 + 32 * k, ch = t % 8;
    const long e = (r0 + row) * C + c0 + 8 * ch, i = e / 8;
    const uint4 ctr = make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)offset, (uint32_t)(offset >> 32));
    const uint4 r = philox4x32_10(ctr, key);
    float z[8];
    box_muller16(r.x & 0xffffu, r.x >> 16, scale, z[0], z[1]);
    box_muller16(r.y & 0xffffu, r.y >> 16, scale, z[2], z[3]);
    box_muller16(r.z & 0xffffu, r.z >> 16, scale, z[4], z[5]);
    box_muller16(r.w & 0xffffu, r.w >> 16, scale, z[6], z[7]);
    uint4 u;
    u.x = (uint32_t)f2bf(z[0]) | ((uint32_t)f2bf(z[1]) << 16);
    u.y = (uint32_t)f2bf(z[2]) | ((uint32_t)f2bf(z[3]) << 16);
    u.z = (uint32_t)f2bf(z[4]) | ((uint32_t)f2bf(z[5]) << 16);
    u.w = (uint32_t)f2bf(z[6]) | ((uint32_t)f2bf(z[7]) << 16);
    *(uint4*)(out + e) = u;
    uint32_t* w = sh + row * 33 + 4 * ch;
    w[0] = u.x; w[1] = u.y; w[2] = u.z; w[3] = u.w;
  }
  __syncthreads();
  const uint16_t* h = (const uint16_t*)sh;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = t / 8 + 32 * k, rc = t % 8;
    uint32_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      q[j] = (uint32_t)h[(8 * rc + 2 * j) * 66 + c] | ((uint32_t)h[(8 * rc + 2 * j + 1) * 66 + c] << 16);
    *(uint4*)(out_t + (c0 + c) * R + r0 + 8 * rc) = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

__global__ __launch_bounds__(256) void rng_normal_f32_kernel(float* out, long n, uint64_t seed, uint64_t offset,
                                                             float scale, const unsigned long long* seed_dev) {
  // seed_dev (nullable): read the key from device memory so a captured graph can replay with new seeds
  if (seed_dev) seed = *seed_dev;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const long n4 = (n + 3) / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const uint4 ctr = make_uint4((uint32_t)i, (uint32_t)(i >> 32), (uint32_t)offset, (uint32_t)(offset >> 32));
    const uint4 r = philox4x32_10(ctr, key);
    float z0, z1, z2, z3;
    box_muller(r.x, r.y, z0, z1);
    box_muller(r.z, r.w, z2, z3);
    f32x4_t v = {z0, z1, z2, z3};
    v *= scale;
    const long base = i * 4;
    if (base + 4 <= n) {
      *(f32x4_t*)(out + base) = v;
    } else {
      for (int j = 0; j < 4 && base + j < n; ++j) out[base + j] = v[j];
    }
  }
}

__device__ __forceinline__ f32x4_t load_grad4(const void* g, int dt, long i) {
  if (dt == DT_F32) return *(const f32x4_t*)((const float*)g + i);
  const uint2 u = *(const uint2*)((const uint16_t*)g + i);
  return f32x4_t{bf2f(u.x & 0xffff), bf2f(u.x >> 16), bf2f(u.y & 0xffff), bf2f(u.y >> 16)};
}
__device__ __forceinline__ void store_bf16x4(uint16_t* p, long i, f32x4_t v) {
  uint2 u;
  u.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  u.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *(uint2*)(p + i) = u;
}

// n must be a multiple of 4 (flat buffers are padded on the host side)
__global__ __launch_bounds__(256) void sgd_kernel(float* master, const void* grad, int gdt, uint16_t* copy,
                                                  long n, float lr, float gscale) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4_t p = *(f32x4_t*)(master + 4 * i);
    const f32x4_t g = load_grad4(grad, gdt, 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = __fadd_rn(p[j], __fmul_rn(-lr, __fmul_rn(gscale, g[j])));
    *(f32x4_t*)(master + 4 * i) = p;
    if (copy) store_bf16x4(copy, 4 * i, p);
  }
}

// SGD on a split master (common.h split_join2 / split_part2): lo = the 16-bit residual plane, hi = the bf16 working
// copy; the same fp32 update as sgd_kernel, 4 B read + 4 B written per parameter (plus the gradient)
__global__ __launch_bounds__(256) void sgd_split_kernel(uint16_t* lo, uint16_t* hi, const void* grad, int gdt, long n,
                                                        float lr, float gscale) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    uint2 h = *(const uint2*)(hi + 4 * i), l = *(const uint2*)(lo + 4 * i);
    const f32x4_t g = load_grad4(grad, gdt, 4 * i);
    float w[4];
    split_join2(h.x, l.x, w[0], w[1]);
    split_join2(h.y, l.y, w[2], w[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = __fadd_rn(w[j], __fmul_rn(-lr, __fmul_rn(gscale, g[j])));
    split_part2(w[0], w[1], h.x, l.x);
    split_part2(w[2], w[3], h.y, l.y);
    *(uint2*)(hi + 4 * i) = h;
    *(uint2*)(lo + 4 * i) = l;
  }
}

// AdamW on a split master (moments fp32): the same update as adam_kernel, 4 B of master read + 4 B written
__global__ __launch_bounds__(256) void adam_split_kernel(uint16_t* lo, uint16_t* hi, const void* grad, int gdt,
                                                         float* m, float* v, long n, float lr, float b1, float b2,
                                                         float eps, float wd, float bc1, float bc2, float gscale) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    uint2 h = *(const uint2*)(hi + 4 * i), l = *(const uint2*)(lo + 4 * i);
    f32x4_t mm = *(f32x4_t*)(m + 4 * i);
    f32x4_t vv = *(f32x4_t*)(v + 4 * i);
    const f32x4_t g = load_grad4(grad, gdt, 4 * i) * gscale;
    float w[4];
    split_join2(h.x, l.x, w[0], w[1]);
    split_join2(h.y, l.y, w[2], w[3]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float m1 = mm[j], v1 = vv[j];
      adamw1(w[j], m1, v1, g[j], lr, b1, b2, eps, wd, bc1, bc2);
      mm[j] = m1;
      vv[j] = v1;
    }
    split_part2(w[0], w[1], h.x, l.x);
    split_part2(w[2], w[3], h.y, l.y);
    *(uint2*)(hi + 4 * i) = h;
    *(uint2*)(lo + 4 * i) = l;
    *(f32x4_t*)(m + 4 * i) = mm;
    *(f32x4_t*)(v + 4 * i) = vv;
  }
}

// split master <-> fp32 (checkpoints, parameter export / import)
__global__ __launch_bounds__(256) void split_join_kernel(const uint16_t* hi, const uint16_t* lo, float* out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = split_join(hi[i], lo[i]);
}
__global__ __launch_bounds__(256) void split_part_kernel(const float* in, uint16_t* hi, uint16_t* lo, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    split_part(in[i], hi[i], lo[i]);
}

__global__ __launch_bounds__(256) void adam_kernel(float* master, const void* grad, int gdt, float* m, float* v,
                                                   uint16_t* copy, long n, float lr, float b1, float b2, float eps,
                                                   float wd, float bc1, float bc2, float gscale) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4_t p = *(f32x4_t*)(master + 4 * i);
    f32x4_t mm = *(f32x4_t*)(m + 4 * i);
    f32x4_t vv = *(f32x4_t*)(v + 4 * i);
    const f32x4_t g = load_grad4(grad, gdt, 4 * i) * gscale;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      mm[j] = b1 * mm[j] + (1.f - b1) * g[j];
      vv[j] = b2 * vv[j] + (1.f - b2) * g[j] * g[j];
      const float mh = mm[j] / bc1, vh = vv[j] / bc2;
      p[j] = p[j] - lr * (mh / (sqrtf(vh) + eps) + wd * p[j]);
    }
    *(f32x4_t*)(master + 4 * i) = p;
    *(f32x4_t*)(m + 4 * i) = mm;
    *(f32x4_t*)(v + 4 * i) = vv;
    if (copy) store_bf16x4(copy, 4 * i, p);
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(const float* in, uint16_t* out, long n) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    store_bf16x4(out, 4 * i, *(const f32x4_t*)(in + 4 * i));
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = f2bf(in[i]);
}
__global__ __launch_bounds__(256) void cast_bf16_f32_kernel(const uint16_t* in, float* out, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = bf2f(in[i]);
}

// Streaming SGD for a side stream that shares the GPU with compute-bound GEMMs: few workgroups
// (max_blocks, e.g. 1/8 of the CUs), 512 threads, each thread keeping UNR f32x4 of master + grad in
// flight so a handful of CUs still pull HBM bandwidth (~50 GB/s per CU at ~2 us latency).
template <int UNR>
__global__ __launch_bounds__(512) void sgd_stream_kernel(float* master, const void* grad, int gdt, uint16_t* copy,
                                                         long n, float lr, float gscale) {
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i + (UNR - 1) * stride < n4; i += UNR * stride) {
    f32x4_t p[UNR], g[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      p[u] = *(f32x4_t*)(master + 4 * (i + u * stride));
      g[u] = load_grad4(grad, gdt, 4 * (i + u * stride));
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int j = 0; j < 4; ++j) p[u][j] = __fadd_rn(p[u][j], __fmul_rn(-lr, __fmul_rn(gscale, g[u][j])));
      *(f32x4_t*)(master + 4 * (i + u * stride)) = p[u];
      if (copy) store_bf16x4(copy, 4 * (i + u * stride), p[u]);
    }
  }
  for (; i < n4; i += stride) {
    f32x4_t p = *(f32x4_t*)(master + 4 * i);
    const f32x4_t g = load_grad4(grad, gdt, 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) p[j] = __fadd_rn(p[j], __fmul_rn(-lr, __fmul_rn(gscale, g[j])));
    *(f32x4_t*)(master + 4 * i) = p;
    if (copy) store_bf16x4(copy, 4 * i, p);
  }
}

// Three-way bf16 split of an fp32 GEMM operand (the fp32-accurate "bf16x6" GEMM, ops/gemm.py).
// x = x0 + x1 + x2 exactly for finite normal x: x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1), each
// difference exact in fp32 (24 = 8 + 8 + 8 mantissa bits, RNE giving each part a spare bit).  The GEMM then runs
// on the bf16 MFMA kernels with K' = 6K: plane p of A' times plane p of B' is one partial product x_i * y_j; the
// six with i + j <= 2 are kept (the dropped ones are < 2^-24 relative), the smallest accumulated first:
//   A' planes (a0, a1, a2, a0, a1, a0)  x  B' planes (b2, b1, b0, b1, b0, b0).
// Products of bf16 values are exact in fp32 and the MFMA accumulates in fp32, so the result carries fp32 GEMM
// accuracy at bf16 matrix-core rate (2.5 PF / 6 products > the 157 TF fp32 MFMA peak).
// rows_form 0: src [R, C] with K = C  -> dst [R, 6C],  dst[r, p*C + c]
// rows_form 1: src [R, C] with K = R  -> dst [6R, C],  dst[p*R + r, c]
// 8 elements per lane: two 16-B loads, six 16-B stores (C % 8 == 0, 16-B aligned rows).
__device__ __forceinline__ void split3(float x, uint16_t& h0, uint16_t& h1, uint16_t& h2) {
  h0 = f2bf(x);
  if (!__builtin_isfinite(bf2f(h0))) {
    if (!__builtin_isfinite(x)) {  // inf / nan: carried in x0 alone (no nan from inf - inf)
      h1 = 0;
      h2 = 0;
      return;
    }
    h0 = (uint16_t)(__float_as_uint(x) >> 16);  // finite x above the bf16 range: truncate instead of rounding up
  }
  const float x0 = bf2f(h0);
  const float r1 = x - x0;
  h1 = f2bf(r1);
  h2 = f2bf(r1 - bf2f(h1));
}

__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ src, long lds, long R, long C,
                                                     uint16_t* __restrict__ dst, int role, int rows_form) {
  const long c8 = C / 8, n8 = R * c8;
  // plane -> which part of x it carries, per role (A: 0,1,2,0,1,0; B: 2,1,0,1,0,0)
  const int codeA = 0 | (1 << 2) | (2 << 4) | (0 << 6) | (1 << 8) | (0 << 10);
  const int codeB = 2 | (1 << 2) | (0 << 4) | (1 << 6) | (0 << 8) | (0 << 10);
  const int code = role == 0 ? codeA : codeB;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long r = i / c8, c = (i - r * c8) * 8;
    const f32x4_t v0 = *(const f32x4_t*)(src + r * lds + c);
    const f32x4_t v1 = *(const f32x4_t*)(src + r * lds + c + 4);
    uint16_t h[3][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      split3(v0[j], h[0][j], h[1][j], h[2][j]);
      split3(v1[j], h[0][j + 4], h[1][j + 4], h[2][j + 4]);
    }
    uint4 w[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      w[q] = make_uint4((uint32_t)h[q][0] | ((uint32_t)h[q][1] << 16), (uint32_t)h[q][2] | ((uint32_t)h[q][3] << 16),
                        (uint32_t)h[q][4] | ((uint32_t)h[q][5] << 16), (uint32_t)h[q][6] | ((uint32_t)h[q][7] << 16));
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      const int q = (code >> (2 * p)) & 3;
      const long off = rows_form ? ((long)p * R + r) * C + c : r * 6 * C + (long)p * C + c;
      *(uint4*)(dst + off) = w[q];
    }
  }
}

// Stand-in for a collective kernel's CU footprint (scripts/bench_occupancy.py): `blocks` workgroups of `threads`
// lanes that stay resident for `ticks` of the 100 MHz s_memrealtime clock (bounded by the host at 100 ms), doing
// only register arithmetic.  Like an RCCL channel's workgroup, a resident wave takes SIMD slots a 256-VGPR GEMM
// block needs, so the GEMM block of that CU cannot start until it leaves.
__global__ void occupy_kernel(long ticks, float* sink) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  float acc = (float)threadIdx.x;
  while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) acc = acc * 0.999f + 1.f;
  if (acc == -1.f) sink[threadIdx.x] = acc;  // never true; keeps the loop
}

// Hardware-queue probe: one wave spins ``ticks`` of the 100 MHz realtime counter, then lane 0 records [start, end]
// (vector stores).  Two of these on two streams tell whether the streams share a hardware queue: a queue runs its
// dispatches in order, so the second one's start lands after the first one's end only when they share it.
__global__ void stamp_kernel(unsigned long long* out, long ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint64_t t = t0;
  while ((long)(t - t0) < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (out != nullptr && threadIdx.x == 0) {
    out[0] = t0;
    out[1] = t;
  }
}

// bf16 transpose dst[C][R] = src[R][C] through LDS, 64x64 tiles, 256 threads: 16-B row-chunk loads, the tile kept
// as 66-element LDS rows (a column gather then spreads over 32 banks), 8-row gathers packed into 16-B stores.  The
// NN weight-gradient layout's transposed copies of the step's input x (layer 0) and dL/dy (top layer): every other
// layer's copy comes out of the producing GEMM's epilogue (EPI_STORE_DT).
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const uint16_t* __restrict__ src, long lds,
                                                             uint16_t* __restrict__ dst, long ldd) {
  __shared__ uint32_t sh[64 * 33];
  const int t = threadIdx.x;
  const long r0 = (long)blockIdx.y * 64, c0 = (long)blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int row = t / 8 + 32 * k, ch = t % 8;
    const uint4 v = *(const uint4*)(src + (r0 + row) * lds + c0 + 8 * ch);
    uint32_t* w = sh + row * 33 + 4 * ch;
    w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
  }
  __syncthreads();
  const uint16_t* h = (const uint16_t*)sh;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = t / 8 + 32 * k, rc = t % 8;
    uint32_t q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      q[j] = (uint32_t)h[(8 * rc + 2 * j) * 66 + c] | ((uint32_t)h[(8 * rc + 2 * j + 1) * 66 + c] << 16);
    *(uint4*)(dst + (c0 + c) * ldd + r0 + 8 * rc) = make_uint4(q[0], q[1], q[2], q[3]);
  }
}

static inline int grid_for(long n4) {
  long g = (n4 + 255) / 256;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace dllm

using namespace dllm;

extern "C" {

static int rng_launch(void* out, int dtype, long n, unsigned long long seed, unsigned long long offset, float scale,
                      const unsigned long long* seed_dev, void* stream) {
  if (n <= 0) return 0;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(rng_normal_bf16_kernel, dim3(grid_for((n + 7) / 8)), dim3(256), 0, (hipStream_t)stream,
                       (uint16_t*)out, n, (uint64_t)seed, (uint64_t)offset, scale, seed_dev);
  else
    hipLaunchKernelGGL(rng_normal_f32_kernel, dim3(grid_for((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                       (float*)out, n, (uint64_t)seed, (uint64_t)offset, scale, seed_dev);
  return (int)hipGetLastError();
}

int dllm_rng_normal(void* out, int dtype, long n, unsigned long long seed, unsigned long long offset, float scale,
                    void* stream) {
  return rng_launch(out, dtype, n, seed, offset, scale, nullptr, stream);
}

// bf16 [R, C] draw (the same values as dllm_rng_normal) plus its transpose [C, R]; R, C multiples of 64, 16-B
// aligned bases.  seed_dev (nullable) as in dllm_rng_normal_devseed.
int dllm_rng_normal_bf16_t(void* out, void* out_t, long R, long C, unsigned long long seed,
                           const unsigned long long* seed_dev, unsigned long long offset, float scale, void* stream) {
  if (R <= 0 || C <= 0 || R % 64 || C % 64 || R / 64 > 65535 || ((uintptr_t)out | (uintptr_t)out_t) % 16) return -1;
  hipLaunchKernelGGL(rng_normal_bf16_t_kernel, dim3(C / 64, R / 64), dim3(256), 0, (hipStream_t)stream,
                     (uint16_t*)out, C, (uint16_t*)out_t, R, (uint64_t)seed, (uint64_t)offset, scale, seed_dev);
  return (int)hipGetLastError();
}

// two bf16 tensors of n elements each, in one launch (bitwise two dllm_rng_normal calls); n / 8 < 2^31
int dllm_rng_normal_bf16_pair(void* out0, void* out1, long n, unsigned long long seed,
                              const unsigned long long* seed_dev, unsigned long long off0, unsigned long long off1,
                              float scale0, float scale1, void* stream) {
  if (n <= 0 || n / 8 >= (1L << 31) || ((uintptr_t)out0 | (uintptr_t)out1) % 16) return -1;
  hipLaunchKernelGGL(rng_normal_bf16_pair_kernel, dim3(grid_for((n + 7) / 8), 2), dim3(256), 0, (hipStream_t)stream,
                     (uint16_t*)out0, (uint16_t*)out1, n, (uint64_t)seed, (uint64_t)off0, (uint64_t)off1, scale0,
                     scale1, seed_dev);
  return (int)hipGetLastError();
}

// graph-capturable variant: the seed is read from device memory at execution time
int dllm_rng_normal_devseed(void* out, int dtype, long n, const unsigned long long* seed_dev,
                            unsigned long long offset, float scale, void* stream) {
  return rng_launch(out, dtype, n, 0, offset, scale, seed_dev, stream);
}

int dllm_sgd_step(float* master, const void* grad, int grad_dtype, void* copy_bf16, long n, float lr, float gscale,
                  void* stream) {
  if (n % 4) return -1;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, master, grad, grad_dtype,
                     (uint16_t*)copy_bf16, n, lr, gscale);
  return (int)hipGetLastError();
}

// same update as dllm_sgd_step, bitwise, on at most max_blocks workgroups (side-stream optimizer)
int dllm_sgd_step_stream(float* master, const void* grad, int grad_dtype, void* copy_bf16, long n, float lr,
                         float gscale, int max_blocks, void* stream) {
  if (n % 4 || max_blocks <= 0) return -1;
  const long n4 = n / 4;
  const int g = (int)std::min<long>(max_blocks, std::max<long>(1, (n4 + 511) / 512));
  hipLaunchKernelGGL(sgd_stream_kernel<8>, dim3(g), dim3(512), 0, (hipStream_t)stream, master, grad, grad_dtype,
                     (uint16_t*)copy_bf16, n, lr, gscale);
  return (int)hipGetLastError();
}

int dllm_sgd_split_step(void* lo, void* hi, const void* grad, int grad_dtype, long n, float lr, float gscale,
                        void* stream) {
  if (n % 4 || ((uintptr_t)lo | (uintptr_t)hi) % 8) return -1;
  hipLaunchKernelGGL(sgd_split_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, (uint16_t*)lo,
                     (uint16_t*)hi, grad, grad_dtype, n, lr, gscale);
  return (int)hipGetLastError();
}

int dllm_adam_split_step(void* lo, void* hi, const void* grad, int grad_dtype, float* m, float* v, long n, float lr,
                         float b1, float b2, float eps, float wd, int step, float gscale, void* stream) {
  if (n % 4 || step < 1 || ((uintptr_t)lo | (uintptr_t)hi) % 8) return -1;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  hipLaunchKernelGGL(adam_split_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, (uint16_t*)lo,
                     (uint16_t*)hi, grad, grad_dtype, m, v, n, lr, b1, b2, eps, wd, bc1, bc2, gscale);
  return (int)hipGetLastError();
}

// mode 0: out_f32 = join(hi, lo);  mode 1: (hi, lo) = split(in_f32)
int dllm_split_master(void* hi, void* lo, void* f32, long n, int mode, void* stream) {
  if (n <= 0) return 0;
  const int g = grid_for((n + 3) / 4);
  if (mode == 0)
    hipLaunchKernelGGL(split_join_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)hi,
                       (const uint16_t*)lo, (float*)f32, n);
  else
    hipLaunchKernelGGL(split_part_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, (const float*)f32,
                       (uint16_t*)hi, (uint16_t*)lo, n);
  return (int)hipGetLastError();
}

int dllm_adam_step(float* master, const void* grad, int grad_dtype, float* m, float* v, void* copy_bf16, long n,
                   float lr, float b1, float b2, float eps, float wd, int step, float gscale, void* stream) {
  if (n % 4 || step < 1) return -1;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_for(n / 4)), dim3(256), 0, (hipStream_t)stream, master, grad,
                     grad_dtype, m, v, (uint16_t*)copy_bf16, n, lr, b1, b2, eps, wd, bc1, bc2, gscale);
  return (int)hipGetLastError();
}

int dllm_cast(const void* in, int in_dtype, void* out, int out_dtype, long n, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (in_dtype == DT_F32 && out_dtype == DT_BF16)
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, s, (const float*)in,
                       (uint16_t*)out, n);
  else if (in_dtype == DT_BF16 && out_dtype == DT_F32)
    hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), 0, s, (const uint16_t*)in,
                       (float*)out, n);
  else
    return -1;
  return (int)hipGetLastError();
}

// bf16x6 operand split (see split3_kernel); role 0 = A (left operand), 1 = B
int dllm_split3(const float* src, long lds, long R, long C, void* dst, int role, int rows_form, void* stream) {
  if (R <= 0 || C <= 0 || C % 8 || lds % 4 || (uintptr_t)src % 16 || (uintptr_t)dst % 16) return -1;
  const long n8 = R * (C / 8);
  int g = (int)std::min<long>((n8 + 255) / 256, 2048);
  hipLaunchKernelGGL(split3_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, src, lds, R, C, (uint16_t*)dst,
                     role, rows_form);
  return (int)hipGetLastError();
}

// dst [C, R] = src [R, C]ᵀ, bf16; R, C multiples of 64, 16-B aligned bases and row strides
int dllm_transpose_bf16(const void* src, long lds, void* dst, long ldd, long R, long C, void* stream) {
  if (R <= 0 || C <= 0 || R % 64 || C % 64 || lds % 8 || ldd % 8 || lds < C || ldd < R || (uintptr_t)src % 16 ||
      (uintptr_t)dst % 16 || R / 64 > 65535)
    return -1;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3(C / 64, R / 64), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)src, lds, (uint16_t*)dst, ldd);
  return (int)hipGetLastError();
}

int dllm_occupy(int blocks, int threads, float us, float* sink, void* stream) {
  if (blocks <= 0 || threads <= 0 || threads > 1024 || us < 0.f || us > 1e5f) return -1;
  hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(threads), 0, (hipStream_t)stream, (long)(us * 100.f), sink);
  return (int)hipGetLastError();
}

// 1: ``probe`` runs on the hardware queue of ``base`` (its stamp starts after base's spin ends), 0: a queue of its
// own, < 0: error.  Both streams are synchronised.
int dllm_queue_shared(void* base, void* probe, int spin_us) {
  static unsigned long long* buf = nullptr;
  if (!buf && hipMalloc(&buf, 64) != hipSuccess) return -2;
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)base, buf, (long)spin_us * 100);
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)probe, buf + 2, 0L);
  if (hipGetLastError() != hipSuccess) return -3;
  if (hipStreamSynchronize((hipStream_t)base) != hipSuccess || hipStreamSynchronize((hipStream_t)probe) != hipSuccess)
    return -4;
  unsigned long long h[4];
  if (hipMemcpy(h, buf, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return -5;
  return h[2] >= h[1] ? 1 : 0;
}

// Reserve ``base``'s hardware queue for it.  HIP gives a process GPU_MAX_HW_QUEUES queues per priority and puts each
// new stream on the least-used one, so any stream created later (torch's pool, which ProcessGroupNCCL / RCCL and the
// engine's side streams draw from) can land on the compute stream's queue and serialise with it
// (profiles/r3/hw_queue_collision_trace_r3.txt).  Here ``candidates`` non-blocking streams are created and used one by
// one; those that landed on base's queue are kept for the process (blockers: they raise that queue's use count) and
// the others destroyed, so later streams fill the other queues first.  Returns the number of blockers (< 0: error).
int dllm_queue_reserve(void* base, int candidates, int spin_us) {
  static hipStream_t blockers[512];
  static int nblock = 0;
  if (candidates <= 0 || candidates > 512) return -1;
  hipStream_t cand[512];
  int made = 0, err = 0;
  for (int i = 0; i < candidates && !err; ++i) {
    if (hipStreamCreateWithFlags(&cand[i], hipStreamNonBlocking) != hipSuccess) break;
    made = i + 1;
    // first use of a stream acquires its queue: do that before the timed probe, so a slow queue creation is not
    // mistaken for sharing
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, cand[i], (unsigned long long*)nullptr, -1L);
    if (hipStreamSynchronize(cand[i]) != hipSuccess) {
      err = -6;
      break;
    }
    // majority of 3 probes (one can read "shared" when the candidate's dispatch is merely late; a wrongly kept
    // blocker would raise a non-compute queue's use count and steer later streams onto the compute queue)
    int votes = 0;
    for (int t = 0; t < 3 && !err; ++t) {
      const int sh = dllm_queue_shared(base, (void*)cand[i], spin_us);
      if (sh < 0) err = sh;
      else votes += sh;
    }
    if (!err && votes >= 2 && nblock < 512) {
      blockers[nblock++] = cand[i];
      cand[i] = nullptr;
    }
  }
  for (int i = 0; i < made; ++i)  // every non-blocker candidate, on success and on error alike
    if (cand[i]) (void)hipStreamDestroy(cand[i]);
  return err ? err : nblock;
}

int dllm_abi_version() { return 13; }

}  // extern "C"
