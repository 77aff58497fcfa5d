// Custom two-shot all-reduce over xGMI peer memory ("car") for tensor-parallel activations.
//
// the reference all-reduces the TP partial outputs (y, dx: [T, D], 64 MiB in
// bf16) synchronously through one NCCL ring.  xGMI on MI355X is point-to-point (7 links per GPU), so a
// ring moves each byte over one link at a time.  Here every rank maps every peer's registration buffer
// (hipIpcGetMemHandle / hipIpcOpenMemHandle, handles exchanged through the job's store) and:
//
//   1. copy-in   : my input -> my IN region                                   (local HBM)
//   2. barrier   : system-scope release/acquire flags, one 64-B slot per (owner, sender)
//   3. rs-push   : rank r sums chunk r of every peer's IN region (n-1 remote reads, all links at once)
//                  and writes the sum into chunk r of every peer's OUT region (n-1 remote writes)
//   4. barrier
//   5. copy-out  : my OUT region -> my input tensor
//
// Zero-copy form (round 3, dllm_car_all_reduce_arena): the engine allocates the TP-exchanged activations (layer
// outputs, input gradients) inside one "arena" laid out identically on every rank and mapped by every peer.  The
// producing GEMM writes its partial straight into the arena, rank r sums chunk r of every peer's range IN PLACE and
// writes the sum back into every peer's range, and the consumer reads the arena tensor itself: no copy-in, no
// copy-out, no IN/OUT staging (release fences on every XCD -> barrier -> reduce-scatter + push -> barrier ->
// acquire fences).
//
// i.e. a reduce-scatter and an all-gather in one pass each direction, both spread over all links.
// Bulk-data visibility across devices relies on the kernel boundaries (HIP dispatches carry system-scope
// acquire/release fences); the barrier kernels add explicit system-scope fences and atomics.  Every
// spin is bounded (s_memrealtime, 100 MHz) and reports a timeout through a device error word instead
// of hanging the GPU.
#include <string.h>

#include <algorithm>

#include "common.h"

namespace dllm {
namespace car {

constexpr int MAXR = 8;
constexpr long SIG_BYTES = MAXR * 64;

struct Ptrs {
  char* p[MAXR];
};

struct State {
  int rank = 0, n = 1, dev = 0;
  long cap = 0;         // bytes per region (IN and OUT)
  char* buf = nullptr;  // [IN cap | OUT cap | signals SIG_BYTES]
  Ptrs peers{};         // peer bases (self included); opened IPC mappings for others
  bool opened[MAXR] = {};
  unsigned epoch = 0;
  int* err = nullptr;   // device error word (1 = barrier timeout)
  // zero-copy arena (dllm_car_attach_arena): a caller-owned allocation laid out identically on every rank; the
  // all-reduce runs in place on a byte range of it (no copy-in / copy-out)
  char* arena = nullptr;
  long arena_bytes = 0;
  Ptrs peer_arena{};
  char* arena_map[MAXR] = {};  // opened IPC bases (closed at destroy)
};

__device__ __forceinline__ void fence_release_sys() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); }
__device__ __forceinline__ void fence_acquire_sys() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); }

// one lane per workgroup issues the system-scope cache maintenance (the whole L2 of its XCD)
__device__ __forceinline__ void block_acquire() {
  if (threadIdx.x == 0) fence_acquire_sys();
  __syncthreads();
}
__device__ __forceinline__ void block_release() {
  __syncthreads();
  if (threadIdx.x == 0) fence_release_sys();
}

// err != nullptr (the copy-out): a barrier of this all-reduce timed out, so the OUT region may hold a partial
// or stale sum -- the result is poisoned with NaN (all-ones words) instead, so a stalled peer can never turn
// into silently wrong activations, and the host raises at its next check (CustomAllReduce.check).
__global__ void copy_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src, long n16, const int* err) {
  block_acquire();
  const bool bad = err != nullptr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  const uint4 nan = uint4{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x)
    dst[i] = bad ? nan : src[i];
  block_release();
}

// thread t < n: publish `epoch` into peer t's slot for me, then wait for peer t's `epoch` in my slot.
// Peers are at most one barrier ahead, so "slot >= epoch" (wrap-safe) is the arrival test.
__global__ void barrier_kernel(Ptrs peers, int rank, int n, long sig_off, unsigned epoch, long max_ticks,
                               int* err) {
  const int t = threadIdx.x;
  fence_release_sys();
  // after a timeout the epochs of the ranks no longer line up: every later barrier fails fast (no spin)
  // until the state is recreated, and every later result is poisoned by the copy-out
  const bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (t < n && !failed) {
    unsigned* slot = (unsigned*)(peers.p[t] + sig_off + rank * 64);
    __hip_atomic_store(slot, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* mine = (unsigned*)(peers.p[rank] + sig_off + t * 64);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if ((long)(__builtin_amdgcn_s_memrealtime() - t0) > max_ticks) {
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  fence_acquire_sys();
}

template <typename T> struct V8;
template <> struct V8<uint16_t> {  // 8 bf16 per 16 B
  static constexpr int E = 8;
  static __device__ __forceinline__ void add(float (&acc)[8], uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += bf2f(w[i] & 0xffff);
      acc[2 * i + 1] += bf2f(w[i] >> 16);
    }
  }
  static __device__ __forceinline__ uint4 pack(const float (&acc)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(acc[2 * i]) | ((uint32_t)f2bf(acc[2 * i + 1]) << 16);
    return uint4{w[0], w[1], w[2], w[3]};
  }
};
template <> struct V8<float> {  // 4 fp32 per 16 B (acc[4..7] unused)
  static constexpr int E = 4;
  static __device__ __forceinline__ void add(float (&acc)[8], uint4 v) {
    acc[0] += __uint_as_float(v.x); acc[1] += __uint_as_float(v.y);
    acc[2] += __uint_as_float(v.z); acc[3] += __uint_as_float(v.w);
  }
  static __device__ __forceinline__ uint4 pack(const float (&acc)[8]) {
    return uint4{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])};
  }
};

// chunk r (16-B vectors [v0, v1)) of the sum: read IN of every peer, write OUT of every peer.
// Peers are summed in rank order 0..n-1 on every rank, so every rank holds bitwise the same result.
template <typename T>
__global__ __launch_bounds__(256) void rs_push_kernel(Ptrs peers, int n, long out_off, long v0, long v1) {
  block_acquire();
  for (long v = v0 + blockIdx.x * (long)blockDim.x + threadIdx.x; v < v1; v += (long)gridDim.x * blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 in[MAXR];
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) in[p] = ((const uint4*)peers.p[p])[v];
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) V8<T>::add(acc, in[p]);
    const uint4 r = V8<T>::pack(acc);
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) ((uint4*)(peers.p[p] + out_off))[v] = r;
  }
  block_release();
}

// In-place variant over the zero-copy arena: rank r reads chunk r of every peer's range, sums in rank order and
// writes the sum back into chunk r of every peer's range.  Only rank r touches chunk r (of any peer) in this
// phase, so reading and overwriting the same addresses is race-free; the second barrier publishes the result.
template <typename T>
__global__ __launch_bounds__(256) void rs_inplace_kernel(Ptrs peers, int n, long off, long v0, long v1) {
  block_acquire();
  for (long v = v0 + blockIdx.x * (long)blockDim.x + threadIdx.x; v < v1; v += (long)gridDim.x * blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 in[MAXR];
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) in[p] = ((const uint4*)(peers.p[p] + off))[v];
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) V8<T>::add(acc, in[p]);
    const uint4 r = V8<T>::pack(acc);
#pragma unroll
    for (int p = 0; p < MAXR; ++p)
      if (p < n) ((uint4*)(peers.p[p] + off))[v] = r;
  }
  block_release();
}

// Device-wide cache maintenance around the in-place exchange, one fence per workgroup on a grid that covers every
// XCD: `fence_kernel(.., release)` writes back the producing GEMM's dirty L2 lines before peers read the range
// (every XCD's L2, not just the barrier kernel's); the acquire form, after the second barrier, drops stale lines of
// the range that peers have just rewritten, and poisons the range with NaN if a barrier timed out (a stalled peer
// never turns into a silently partial sum).
__global__ __launch_bounds__(64) void fence_kernel(uint4* __restrict__ data, long n16, const int* err, int release) {
  if (release) {
    block_release();
    return;
  }
  block_acquire();
  if (err != nullptr && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
    const uint4 nan = uint4{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) data[i] = nan;
    block_release();
  }
}

}  // namespace car
}  // namespace dllm

using namespace dllm::car;

extern "C" {

// Allocate this rank's registration buffer (IN and OUT regions of `cap_bytes` each + signal slots).
int dllm_car_create(int rank, int nranks, long cap_bytes, int device, void** out) {
  if (nranks < 1 || nranks > MAXR || rank < 0 || rank >= nranks || cap_bytes <= 0 || cap_bytes % 16) return -1;
  if (hipSetDevice(device) != hipSuccess) return -2;
  State* s = new State();
  s->rank = rank;
  s->n = nranks;
  s->dev = device;
  s->cap = cap_bytes;
  hipError_t e = hipMalloc(&s->buf, 2 * cap_bytes + SIG_BYTES);
  if (e == hipSuccess) e = hipMemset(s->buf + 2 * cap_bytes, 0, SIG_BYTES);
  if (e == hipSuccess) e = hipMalloc(&s->err, sizeof(int));
  if (e == hipSuccess) e = hipMemset(s->err, 0, sizeof(int));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    delete s;
    return (int)e;
  }
  s->peers.p[rank] = s->buf;
  *out = s;
  return 0;
}

int dllm_car_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

int dllm_car_get_handle(void* st, char* out, int nbytes) {
  State* s = (State*)st;
  if (nbytes < (int)sizeof(hipIpcMemHandle_t)) return -1;
  hipIpcMemHandle_t h;
  const hipError_t e = hipIpcGetMemHandle(&h, s->buf);
  if (e != hipSuccess) return (int)e;
  memcpy(out, &h, sizeof(h));
  return 0;
}

// handles: nranks consecutive hipIpcMemHandle_t (own entry ignored)
int dllm_car_open(void* st, const char* handles) {
  State* s = (State*)st;
  for (int p = 0; p < s->n; ++p) {
    if (p == s->rank) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, handles + p * sizeof(hipIpcMemHandle_t), sizeof(h));
    void* ptr = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    s->peers.p[p] = (char*)ptr;
    s->opened[p] = true;
  }
  return 0;
}

// testing without IPC: several ranks' states in one process share their buffers directly
int dllm_car_set_peer(void* st, int peer, void* peer_state) {
  State* s = (State*)st;
  if (peer < 0 || peer >= s->n) return -1;
  s->peers.p[peer] = ((State*)peer_state)->buf;
  return 0;
}

void* dllm_car_buffer(void* st) { return ((State*)st)->buf; }

// In-place sum all-reduce of `nbytes` at `data` (bf16: dtype 0, fp32: 1) on `stream`.
int dllm_car_all_reduce(void* st, void* data, long nbytes, int dtype, double timeout_s, void* stream) {
  State* s = (State*)st;
  if (nbytes <= 0 || nbytes % 16 || nbytes > s->cap || (dtype != 0 && dtype != 1)) return -1;
  hipStream_t q = (hipStream_t)stream;
  const long n16 = nbytes / 16;
  const long ticks = (long)(timeout_s * 1e8);
  const long sig_off = 2 * s->cap;
  const int cgrid = (int)std::min<long>((n16 + 255) / 256, 1024);
  hipLaunchKernelGGL(copy_kernel, dim3(cgrid), dim3(256), 0, q, (uint4*)s->buf, (const uint4*)data, n16,
                     (const int*)nullptr);
  if (s->n > 1) {
    hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, q, s->peers, s->rank, s->n, sig_off, ++s->epoch, ticks,
                       s->err);
    const long per = (n16 + s->n - 1) / s->n;
    const long v0 = std::min(n16, per * s->rank), v1 = std::min(n16, v0 + per);
    if (v1 > v0) {
      const int g = (int)std::min<long>((v1 - v0 + 255) / 256, 512);
      if (dtype == 0)
        hipLaunchKernelGGL(rs_push_kernel<uint16_t>, dim3(g), dim3(256), 0, q, s->peers, s->n, s->cap, v0, v1);
      else
        hipLaunchKernelGGL(rs_push_kernel<float>, dim3(g), dim3(256), 0, q, s->peers, s->n, s->cap, v0, v1);
    }
    hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, q, s->peers, s->rank, s->n, sig_off, ++s->epoch, ticks,
                       s->err);
    hipLaunchKernelGGL(copy_kernel, dim3(cgrid), dim3(256), 0, q, (uint4*)data, (const uint4*)(s->buf + s->cap), n16,
                       (const int*)s->err);
  } else {
    hipLaunchKernelGGL(copy_kernel, dim3(cgrid), dim3(256), 0, q, (uint4*)data, (const uint4*)s->buf, n16,
                       (const int*)nullptr);
  }
  return (int)hipGetLastError();
}

// ---- zero-copy arena ----------------------------------------------------------------------------------------
// IPC handle of the allocation holding `ptr` (its base) + the byte offset of `ptr` inside it: works for a
// caching-allocator sub-block as well as a whole allocation
int dllm_car_arena_handle(void* ptr, char* out, int nbytes, long* offset) {
  if (nbytes < (int)sizeof(hipIpcMemHandle_t)) return -1;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hipError_t e = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr);
  if (e != hipSuccess) return (int)e;
  hipIpcMemHandle_t h;
  e = hipIpcGetMemHandle(&h, (void*)base);
  if (e != hipSuccess) return (int)e;
  memcpy(out, &h, sizeof(h));
  *offset = (long)((char*)ptr - (char*)base);
  return 0;
}

// attach this rank's arena and map every peer's (handles: n consecutive hipIpcMemHandle_t, offsets: n longs; own
// entries ignored).  handles == nullptr: peers are set with dllm_car_set_peer_arena (single-process testing).
int dllm_car_attach_arena(void* st, void* arena, long bytes, const char* handles, const long* offsets) {
  State* s = (State*)st;
  if (!arena || bytes <= 0 || ((uintptr_t)arena % 16)) return -1;
  s->arena = (char*)arena;
  s->arena_bytes = bytes;
  s->peer_arena.p[s->rank] = s->arena;
  if (handles == nullptr) return 0;
  for (int p = 0; p < s->n; ++p) {
    if (p == s->rank) continue;
    hipIpcMemHandle_t h;
    memcpy(&h, handles + p * sizeof(hipIpcMemHandle_t), sizeof(h));
    void* base = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    s->arena_map[p] = (char*)base;
    s->peer_arena.p[p] = (char*)base + offsets[p];
  }
  return 0;
}

int dllm_car_set_peer_arena(void* st, int peer, void* peer_arena) {
  State* s = (State*)st;
  if (peer < 0 || peer >= s->n) return -1;
  s->peer_arena.p[peer] = (char*)peer_arena;
  return 0;
}

// In-place sum all-reduce of arena bytes [off, off + nbytes) on every rank (same offsets everywhere): no copies.
// release fences -> barrier -> in-place reduce-scatter + push -> barrier -> acquire fences (+ NaN poison on timeout)
int dllm_car_all_reduce_arena(void* st, long off, long nbytes, int dtype, double timeout_s, void* stream) {
  State* s = (State*)st;
  if (!s->arena || off < 0 || nbytes <= 0 || nbytes % 16 || off % 16 || off + nbytes > s->arena_bytes ||
      (dtype != 0 && dtype != 1))
    return -1;
  hipStream_t q = (hipStream_t)stream;
  const long n16 = nbytes / 16;
  const long ticks = (long)(timeout_s * 1e8);
  const long sig_off = 2 * s->cap;
  if (s->n == 1) return 0;  // a one-rank sum is the input
  const int fgrid = 512;    // >= 2 workgroups per CU: every XCD's L2 gets its fence
  hipLaunchKernelGGL(fence_kernel, dim3(fgrid), dim3(64), 0, q, (uint4*)nullptr, 0L, (const int*)nullptr, 1);
  hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, q, s->peers, s->rank, s->n, sig_off, ++s->epoch, ticks,
                     s->err);
  const long per = (n16 + s->n - 1) / s->n;
  const long v0 = std::min(n16, per * s->rank), v1 = std::min(n16, v0 + per);
  if (v1 > v0) {
    const int g = (int)std::min<long>((v1 - v0 + 255) / 256, 1024);
    if (dtype == 0)
      hipLaunchKernelGGL(rs_inplace_kernel<uint16_t>, dim3(g), dim3(256), 0, q, s->peer_arena, s->n, off, v0, v1);
    else
      hipLaunchKernelGGL(rs_inplace_kernel<float>, dim3(g), dim3(256), 0, q, s->peer_arena, s->n, off, v0, v1);
  }
  hipLaunchKernelGGL(barrier_kernel, dim3(1), dim3(64), 0, q, s->peers, s->rank, s->n, sig_off, ++s->epoch, ticks,
                     s->err);
  hipLaunchKernelGGL(fence_kernel, dim3(fgrid), dim3(64), 0, q, (uint4*)(s->arena + off), n16, (const int*)s->err, 0);
  return (int)hipGetLastError();
}

// 0 = ok, 1 = a barrier timed out (read after synchronising the stream); sticky until destroy
int dllm_car_error(void* st) {
  State* s = (State*)st;
  int h = 0;
  if (hipMemcpy(&h, s->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -2;
  return h;
}

int dllm_car_destroy(void* st) {
  State* s = (State*)st;
  if (!s) return 0;
  (void)hipDeviceSynchronize();
  for (int p = 0; p < s->n; ++p) {
    if (s->opened[p]) (void)hipIpcCloseMemHandle(s->peers.p[p]);
    if (s->arena_map[p]) (void)hipIpcCloseMemHandle(s->arena_map[p]);
  }
  (void)hipFree(s->buf);
  (void)hipFree(s->err);
  delete s;
  return 0;
}

}  // extern "C"
