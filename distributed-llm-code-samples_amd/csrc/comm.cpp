// Native RCCL communicator layer (one communicator + one HIP stream per communication role).
//
// The reference drives NCCL through torch.distributed ProcessGroupNCCL with a single process group, so
// its FSDP reduce-scatter serialises behind the prefetch all-gather on one internal stream
// (train_ffns.py:14, :252).  This layer is the MI355X-native replacement sketched in
// RCCL communicators created from a uniqueId exchanged through the job's store
// (ncclCommInitRank), split for 2-D meshes (ncclCommSplit), collectives enqueued on explicit
// hipStream_t's, and hipEvent_t edges between the compute stream and each role's stream.  Everything is
// zero-copy on caller-owned device buffers (flat gradient / parameter buffers).
//
// It binds to torch's bundled librccl.so (same SONAME librccl.so.1 as ROCm's), loaded after torch, so
// it shares the single HIP runtime of the process.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

namespace {
inline ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case 0: return ncclBfloat16;
    case 1: return ncclFloat32;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    case 4: return ncclInt64;
    default: return ncclNumTypes;
  }
}
inline int rc(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }
}  // namespace

extern "C" {

int dllm_nccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

int dllm_nccl_unique_id(char* out, int nbytes) {
  if (nbytes < (int)sizeof(ncclUniqueId)) return -1;
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return rc(r);
  memcpy(out, id.internal, sizeof(ncclUniqueId));
  return 0;
}

int dllm_nccl_unique_id_bytes() { return (int)sizeof(ncclUniqueId); }

// returns 0 and writes the communicator handle, or an error code
int dllm_nccl_comm_init(int nranks, int rank, const char* id_bytes, int device, void** comm_out) {
  if (hipSetDevice(device) != hipSuccess) return -2;
  ncclUniqueId id;
  memcpy(id.internal, id_bytes, sizeof(ncclUniqueId));
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
  *comm_out = (void*)c;
  return rc(r);
}

int dllm_nccl_comm_split(void* comm, int color, int key, void** comm_out) {
  ncclComm_t c = nullptr;
  const ncclResult_t r = ncclCommSplit((ncclComm_t)comm, color, key, &c, nullptr);
  *comm_out = (void*)c;
  return rc(r);
}

int dllm_nccl_comm_destroy(void* comm) { return comm ? rc(ncclCommDestroy((ncclComm_t)comm)) : 0; }
int dllm_nccl_comm_abort(void* comm) { return comm ? rc(ncclCommAbort((ncclComm_t)comm)) : 0; }

int dllm_nccl_comm_async_error(void* comm) {
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)comm, &e);
  return r != ncclSuccess ? rc(r) : rc(e);
}

int dllm_nccl_all_reduce(void* comm, const void* in, void* out, long count, int dtype, void* stream) {
  return rc(ncclAllReduce(in, out, (size_t)count, to_nccl(dtype), ncclSum, (ncclComm_t)comm, (hipStream_t)stream));
}

// out holds nranks * count_per_rank elements; in-place when in == out + rank*count_per_rank
int dllm_nccl_all_gather(void* comm, const void* in, void* out, long count_per_rank, int dtype, void* stream) {
  return rc(ncclAllGather(in, out, (size_t)count_per_rank, to_nccl(dtype), (ncclComm_t)comm, (hipStream_t)stream));
}

// in holds nranks * count_per_rank elements
int dllm_nccl_reduce_scatter(void* comm, const void* in, void* out, long count_per_rank, int dtype, void* stream) {
  return rc(ncclReduceScatter(in, out, (size_t)count_per_rank, to_nccl(dtype), ncclSum, (ncclComm_t)comm,
                              (hipStream_t)stream));
}

int dllm_nccl_group_start() { return rc(ncclGroupStart()); }
int dllm_nccl_group_end() { return rc(ncclGroupEnd()); }

const char* dllm_nccl_error_string(int code) {
  if (code >= 1000) return ncclGetErrorString((ncclResult_t)(code - 1000));
  return "dllm comm error";
}

// ---- streams and events (role streams + cross-stream edges) ----
int dllm_stream_create(int priority, void** out) {
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority);
  *out = (void*)s;
  return (int)e;
}
int dllm_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }
int dllm_event_create(void** out) {
  hipEvent_t ev = nullptr;
  const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  *out = (void*)ev;
  return (int)e;
}
int dllm_event_destroy(void* ev) { return (int)hipEventDestroy((hipEvent_t)ev); }
int dllm_event_record(void* ev, void* stream) { return (int)hipEventRecord((hipEvent_t)ev, (hipStream_t)stream); }
int dllm_stream_wait_event(void* stream, void* ev) {
  return (int)hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0);
}
// 1 = complete, 0 = pending, <0 error
int dllm_event_query(void* ev) {
  const hipError_t e = hipEventQuery((hipEvent_t)ev);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return -(int)e;
}
int dllm_event_synchronize(void* ev) { return (int)hipEventSynchronize((hipEvent_t)ev); }

}  // extern "C"
