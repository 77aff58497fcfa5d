// Single-process, multi-device RCCL collective self-test: the native counterpart of the reference's
// test_nccl.py (torch.cuda.nccl all_gather / all_reduce / reduce_scatter of 128 fp32 per GPU checked
// against host expectations, test_nccl.py:9-38).
//
// One communicator per visible device from ncclCommInitAll, one explicit hipStream_t per device, the
// per-device calls fused with ncclGroupStart/End.  Exit code 0 = all checks passed.
//
//   dllm_rccl_selftest [ndev] [count]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCHECK(x)                                                                         \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 2;                                                                             \
    }                                                                                       \
  } while (0)
#define NCCLCHECK(x)                                                                        \
  do {                                                                                      \
    ncclResult_t r_ = (x);                                                                  \
    if (r_ != ncclSuccess) {                                                                \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      return 3;                                                                             \
    }                                                                                       \
  } while (0)

static float val(int rank, long i) { return (float)(rank + 1) * 0.5f + (float)(i % 97); }

int main(int argc, char** argv) {
  int avail = 0;
  HIPCHECK(hipGetDeviceCount(&avail));
  int ndev = argc > 1 ? std::atoi(argv[1]) : avail;
  const long N = argc > 2 ? std::atol(argv[2]) : 128;
  if (ndev <= 0 || ndev > avail) {
    std::fprintf(stderr, "need 1..%d devices, asked %d\n", avail, ndev);
    return 4;
  }
  int ver = 0;
  ncclGetVersion(&ver);
  std::printf("RCCL %d, %d device(s), %ld fp32 per rank\n", ver, ndev, N);

  std::vector<int> devs(ndev);
  for (int d = 0; d < ndev; ++d) devs[d] = d;
  std::vector<ncclComm_t> comms(ndev);
  NCCLCHECK(ncclCommInitAll(comms.data(), ndev, devs.data()));

  std::vector<hipStream_t> streams(ndev);
  std::vector<float*> in(ndev), out(ndev), rs_in(ndev), rs_out(ndev);
  for (int d = 0; d < ndev; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamCreateWithFlags(&streams[d], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&in[d], N * sizeof(float)));
    HIPCHECK(hipMalloc(&out[d], N * ndev * sizeof(float)));
    HIPCHECK(hipMalloc(&rs_in[d], N * ndev * sizeof(float)));
    HIPCHECK(hipMalloc(&rs_out[d], N * sizeof(float)));
    std::vector<float> h(N * ndev);
    for (long i = 0; i < N; ++i) h[i] = val(d, i);
    HIPCHECK(hipMemcpy(in[d], h.data(), N * sizeof(float), hipMemcpyHostToDevice));
    for (long i = 0; i < N * ndev; ++i) h[i] = val(d, i) * 0.25f;
    HIPCHECK(hipMemcpy(rs_in[d], h.data(), N * ndev * sizeof(float), hipMemcpyHostToDevice));
  }
  auto sync_all = [&]() -> int {
    for (int d = 0; d < ndev; ++d) {
      HIPCHECK(hipSetDevice(d));
      HIPCHECK(hipStreamSynchronize(streams[d]));
    }
    return 0;
  };
  int bad = 0;
  std::vector<float> h(N * ndev);

  // all-gather: every device ends with cat(inputs)   (test_nccl.py:9-19)
  NCCLCHECK(ncclGroupStart());
  for (int d = 0; d < ndev; ++d) NCCLCHECK(ncclAllGather(in[d], out[d], N, ncclFloat32, comms[d], streams[d]));
  NCCLCHECK(ncclGroupEnd());
  if (sync_all()) return 2;
  for (int d = 0; d < ndev; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMemcpy(h.data(), out[d], N * ndev * sizeof(float), hipMemcpyDeviceToHost));
    for (int r = 0; r < ndev; ++r)
      for (long i = 0; i < N; ++i) bad += h[r * N + i] != val(r, i);
  }
  std::printf("all_gather %s\n", bad ? "FAIL" : "ok");
  int total = bad;

  // all-reduce (in place): elementwise sum   (test_nccl.py:22-27)
  bad = 0;
  NCCLCHECK(ncclGroupStart());
  for (int d = 0; d < ndev; ++d) NCCLCHECK(ncclAllReduce(in[d], in[d], N, ncclFloat32, ncclSum, comms[d], streams[d]));
  NCCLCHECK(ncclGroupEnd());
  if (sync_all()) return 2;
  for (int d = 0; d < ndev; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMemcpy(h.data(), in[d], N * sizeof(float), hipMemcpyDeviceToHost));
    for (long i = 0; i < N; ++i) {
      float e = 0.f;
      for (int r = 0; r < ndev; ++r) e += val(r, i);
      bad += std::fabs(h[i] - e) > 1e-5f * std::fabs(e);
    }
  }
  std::printf("all_reduce %s\n", bad ? "FAIL" : "ok");
  total += bad;

  // reduce-scatter: chunk r of the sum lands on device r   (test_nccl.py:29-38)
  bad = 0;
  NCCLCHECK(ncclGroupStart());
  for (int d = 0; d < ndev; ++d)
    NCCLCHECK(ncclReduceScatter(rs_in[d], rs_out[d], N, ncclFloat32, ncclSum, comms[d], streams[d]));
  NCCLCHECK(ncclGroupEnd());
  if (sync_all()) return 2;
  for (int d = 0; d < ndev; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMemcpy(h.data(), rs_out[d], N * sizeof(float), hipMemcpyDeviceToHost));
    for (long i = 0; i < N; ++i) {
      float e = 0.f;
      for (int r = 0; r < ndev; ++r) e += val(r, d * N + i) * 0.25f;
      bad += std::fabs(h[i] - e) > 1e-5f * std::fabs(e);
    }
  }
  std::printf("reduce_scatter %s\n", bad ? "FAIL" : "ok");
  total += bad;

  for (int d = 0; d < ndev; ++d) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipFree(in[d]));
    HIPCHECK(hipFree(out[d]));
    HIPCHECK(hipFree(rs_in[d]));
    HIPCHECK(hipFree(rs_out[d]));
    HIPCHECK(hipStreamDestroy(streams[d]));
    ncclCommDestroy(comms[d]);
  }
  std::printf("%s\n", total ? "FAILED" : "PASSED");
  return total ? 1 : 0;
}
