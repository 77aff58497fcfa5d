// C ABI of the GEMM library (ctypes, ops/gemm.py): argument checks, kernel-family selection, dispatch to
// the per-layout translation units.  Kernels and launch templates: gemm_kernels.h.
#include <cmath>
#include <cstdint>
#include <cstdlib>

#include "gemm_kernels.h"

using namespace dllm;

// --gemm_variant pp workgroup-slot skew (experiment knob): read once when the library loads, not per launch
static int pp_skew() {
  static const int skew = [] {
    const char* sk = getenv("DLLM_PP_SKEW");
    return sk ? atoi(sk) : 0;
  }();
  return skew;
}

// 224-row tiles instead of 256-row ones for an M x N output: M = 224k, and the 224-row grid fills the device's CUs
// strictly better (fraction of the last wave of tiles in use); mirrored by ops/gemm.py use_m224
static bool use_m224(int M, int N) {
  if (M % 224 != 0 || N % BT_N != 0) return false;
  if (M % BT_M != 0) return true;
  const long ncu = num_cu() > 0 ? num_cu() : 256;
  auto fill = [&](int bm) {
    const long t = (long)(M / bm) * (N / BT_N);
    return (double)t / (double)(((t + ncu - 1) / ncu) * ncu);
  };
  return fill(224) > fill(BT_M);
}

extern "C" {

// Returns 0 on success, a hipError_t otherwise, or -1 for a bad argument.
// force_path: -1 auto, 0 bf16-256 tile kernel, 1 fp32-128 kernel, 2 generic kernel, 3 bf16 224-row tiles.
int dllm_gemm(int in_dtype, int out_dtype, int layout, int epi, int act, const void* A, long lda,
              const void* B, long ldb, void* C, long ldc, const void* aux, void* aux_out, long ldaux,
              int M, int N, int K, float alpha, float beta, int group_m, int force_path, void* stream,
              float lr, float b1, float b2, float eps, float wd, int step, float* opt_m, float* opt_v,
              int ksplit, float* workspace, void* mask, int variant, int tpb, int min_bpc) {
  if (M <= 0 || N <= 0 || K <= 0) return -1;
  if (layout < 0 || layout > 2) return -1;
  if ((epi == EPI_GLU || epi == EPI_DGLU) && (N % 32) != 0) return -1;
  GemmArgs a;
  a.A = A; a.B = B; a.C = C; a.aux = aux; a.aux_out = aux_out;
  a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldaux = ldaux;
  a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.act = act;
  a.group_m = group_m > 0 ? group_m : 4;
  a.lr = lr; a.b1 = b1; a.b2 = b2; a.eps = eps; a.wd = wd; a.opt_m = opt_m; a.opt_v = opt_v;
  a.bc1 = 1.f; a.bc2 = 1.f;
  a.ksplit = 1;
  a.tpb = 1;
  a.mask = nullptr;
  a.variant = variant < 0 || variant > 5 ? 0 : variant;
  a.tpb_req = tpb;
  a.min_bpc = min_bpc < 1 ? 1 : min_bpc;
  a.ws = nullptr;
  a.skew = pp_skew();
  // the LDS-DMA loads and 16-B / paired epilogue accesses of the MFMA paths need 16-B aligned bases
  const bool aligned_ptr = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && ((uintptr_t)C % 16 == 0) &&
                           ((uintptr_t)aux % 16 == 0) && ((uintptr_t)aux_out % 16 == 0) &&
                           ((uintptr_t)opt_m % 16 == 0) && ((uintptr_t)opt_v % 16 == 0);
  const bool opt_epi = (epi == EPI_SGD || epi == EPI_ADAM || epi == EPI_SGDS || epi == EPI_ADAMS || epi == EPI_SGDS_T ||
                        epi == EPI_ADAMS_T);
  const bool split_epi = (epi == EPI_SGDS || epi == EPI_ADAMS || epi == EPI_SGDS_T || epi == EPI_ADAMS_T);
  if (opt_epi && layout == L_NT) return -1;
  // activation epilogues: relu / silu / gelu (the bf16 kernels are instantiated per activation only), in the NT / NN
  // layouts (TN runs the weight gradients: store or a fused optimizer)
  if ((epi == EPI_ACT || epi == EPI_DACT || epi == EPI_GLU || epi == EPI_DGLU) &&
      ((act != ACT_RELU && act != ACT_SILU && act != ACT_GELU) || layout == L_TN))
    return -1;
  if ((epi == EPI_SGD || epi == EPI_ADAM) && out_dtype != DT_F32) return -1;
  // split master: C = the 16-bit residual plane, aux_out = the bf16 working copy (paired 16-B rows: ld % 8 == 0)
  if (split_epi && (out_dtype != DT_BF16 || in_dtype != DT_BF16 || aux_out == nullptr)) return -1;
  if (epi == EPI_ADAM || epi == EPI_ADAMS || epi == EPI_ADAMS_T) {
    if (step < 1 || !opt_m || !opt_v) return -1;
    a.bc1 = 1.f - powf(b1, (float)step);
    a.bc2 = 1.f - powf(b2, (float)step);
  }
  int path = 2;
  const bool aligned_lds = aligned_ptr && (lda % 8 == 0) && (ldb % 8 == 0) && (ldc % 4 == 0) && (ldaux % 4 == 0) &&
                           (!split_epi || (ldc % 8 == 0 && ldaux % 8 == 0));
  if (in_dtype == DT_BF16 && M % BT_M == 0 && N % BT_N == 0 && K % BT_K == 0 && aligned_lds) path = 0;
  if (in_dtype == DT_F32 && out_dtype == DT_F32 && M % FT == 0 && N % FT == 0 && K % FK == 0 && aligned_lds) path = 1;
  // 224-row tiles where they fill the CUs better than 256-row tiles (the MP / TP8 shard's F/8 = 1792 rows: 8 x 224
  // = 256 tiles per 32 column tiles vs 7 x 256 = 224), K-contiguous A, 8-phase K step
  if (in_dtype == DT_BF16 && use_m224(M, N) && K % (2 * BT_K) == 0 && aligned_lds && layout != L_TN &&
      epi != EPI_GLU && epi != EPI_DGLU && ksplit <= 1 && variant != 5)
    path = 3;
  if (force_path >= 0) {
    if (force_path == 0 && path != 0) return -1;
    if (force_path == 1 && path != 1) return -1;
    if (force_path == 3 && path != 3) return -1;
    path = force_path;
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  // The NN weight-gradient layout (transposed outputs, transposed copies, NN fused SGD on 256-row tiles):
  // 8-phase 256x256 persistent kernels only (gemm_kernels.h dispatch_x)
  const bool xepi = epi == EPI_SGDS_T || epi == EPI_STORE_T || epi == EPI_STORE_DT || epi == EPI_ADAMS_T;
  if (xepi || ((epi == EPI_SGDS || epi == EPI_ADAMS) && layout == L_NN && path == 0)) {
    if (path != 0 || K % (2 * BT_K) != 0 || ksplit > 1 || mask != nullptr || beta != 0.f || ldc % 8 != 0 ||
        (a.variant != 0 && a.variant != 3))
      return -1;
    if (epi == EPI_STORE_DT && (aux_out == nullptr || out_dtype != DT_BF16 || ldaux % 8 != 0 || layout == L_TN))
      return -1;
    if (opt_epi && !(layout == L_NN || (layout == L_TN && epi_tout(epi)))) return -1;
    e = layout == L_NN ? dispatch_nn_x(epi, a, out_dtype, s)
        : layout == L_NT ? dispatch_nt_x(epi, a, out_dtype, s) : dispatch_tn_x(epi, a, out_dtype, s);
    return (int)e;
  }
  if (opt_epi && layout == L_NN && path != 3) return -1;  // NN fused optimizers otherwise: 224-row tiles only
  if (path == 2 && epi == EPI_GLU && aux_out == nullptr) return -1;
  if (ksplit > 1) {
    // split-K only on the bf16 8-phase path (each slice an even number of 64-deep K-tiles); a request
    // that cannot be honoured (other kernel family / forced 2-stage variant) runs unsplit
    if (workspace == nullptr) return -1;
    if (path == 0 && (K / BT_K) % (2 * ksplit) == 0 && a.variant != 1) {
      a.ksplit = ksplit;
      a.ws = workspace;
    }
  }
  if (mask != nullptr) {
    // the bitmask lives in the 8-phase kernels' tile-native layout: both GEMMs of a pair must run them
    if ((epi != EPI_ACT && epi != EPI_DACT) || act != ACT_RELU || in_dtype != DT_BF16 || out_dtype != DT_BF16 ||
        (path != 0 && path != 3) || a.ksplit != 1 || (K % (2 * BT_K) != 0 && a.variant != 5) || a.variant == 1)
      return -2;
    a.mask = mask;
  }
  if (opt_epi) {
    e = (layout == L_NN && path == 3) ? dispatch_nn_opt(epi, a, s) : dispatch_tn_opt(path, epi, a, in_dtype, s);
    return (int)e;
  }
  switch (layout) {
    case L_NT: e = dispatch_nt(path, epi, a, in_dtype, out_dtype, s); break;
    case L_NN: e = dispatch_nn(path, epi, a, in_dtype, out_dtype, s); break;
    default: e = dispatch_tn(path, epi, a, in_dtype, out_dtype, s); break;
  }
  if (e != hipSuccess) return (int)e;
  if (path == 2 && epi == EPI_GLU) {
    const int Fh = N / 2;
    if (in_dtype == DT_BF16 && out_dtype == DT_BF16)
      hipLaunchKernelGGL(glu_combine<uint16_t>, dim3(1024), dim3(256), 0, s, (const uint16_t*)aux_out, ldaux,
                         (uint16_t*)C, ldc, M, Fh, act);
    else
      hipLaunchKernelGGL(glu_combine<float>, dim3(1024), dim3(256), 0, s, (const float*)aux_out, ldaux,
                         (float*)C, ldc, M, Fh, act);
    e = hipGetLastError();
  }
  return (int)e;
}

// Two weight-gradient GEMMs of one layout, epilogue and K in a single grouped launch, one tile per block
// (gemm_bf16_8ph_pair): TN on 256x256 tiles, or NN on 224x256 tiles (the transposed-activation TP layout).  Per-problem
// arrays of 2: A, lda, B, ldb, C, ldc, aux_out, ldaux, opt_m, opt_v, M, N.  Returns -1 when the pair does not fit the
// grouped kernel (the caller then runs two dllm_gemm calls): bf16 operands, both shapes tiled, K % 128 == 0, 16-B
// aligned, and tiles(0) + tiles(1) <= the device's CUs.
int dllm_gemm_pair(int layout, int out_dtype, int epi, const void* const* A, const long* lda, const void* const* B,
                   const long* ldb, void* const* C, const long* ldc, void* const* aux_out, const long* ldaux,
                   float* const* opt_m, float* const* opt_v, const int* M, const int* N, int K, float alpha,
                   float lr, float b1, float b2, float eps, float wd, int step, void* stream) {
  if (K <= 0 || K % (2 * BT_K) != 0) return -1;
  if (layout != L_TN && layout != L_NN) return -1;
  // TN: 256-row tiles; NN: 224-row tiles (the transposed-activation TP layout's dW2ᵀ / dW1, M = F/tp)
  const int bm = layout == L_TN ? BT_M : 224;
  if (epi != EPI_STORE && epi != EPI_SGD && epi != EPI_SGDS && epi != EPI_ADAM && epi != EPI_ADAMS) return -1;
  const bool split_epi = (epi == EPI_SGDS || epi == EPI_ADAMS);
  if ((epi == EPI_SGD || epi == EPI_ADAM) && out_dtype != DT_F32) return -1;
  if (split_epi && out_dtype != DT_BF16) return -1;
  GemmArgs a[2];
  int tiles = 0;
  for (int i = 0; i < 2; ++i) {
    if (M[i] <= 0 || N[i] <= 0 || M[i] % bm || N[i] % BT_N) return -1;
    if (split_epi && aux_out[i] == nullptr) return -1;
    if ((epi == EPI_ADAM || epi == EPI_ADAMS) && (step < 1 || !opt_m[i] || !opt_v[i])) return -1;
    const bool al = ((uintptr_t)A[i] % 16 == 0) && ((uintptr_t)B[i] % 16 == 0) && ((uintptr_t)C[i] % 16 == 0) &&
                    ((uintptr_t)aux_out[i] % 16 == 0) && ((uintptr_t)opt_m[i] % 16 == 0) &&
                    ((uintptr_t)opt_v[i] % 16 == 0) && lda[i] % 8 == 0 && ldb[i] % 8 == 0 && ldc[i] % 4 == 0 &&
                    ldaux[i] % 4 == 0 && (!split_epi || (ldc[i] % 8 == 0 && ldaux[i] % 8 == 0));
    if (!al) return -1;
    GemmArgs& g = a[i];
    g = GemmArgs{};
    g.A = A[i]; g.B = B[i]; g.C = C[i]; g.aux = nullptr; g.aux_out = aux_out[i];
    g.lda = lda[i]; g.ldb = ldb[i]; g.ldc = ldc[i]; g.ldaux = ldaux[i];
    g.M = M[i]; g.N = N[i]; g.K = K; g.alpha = alpha; g.beta = 0.f; g.act = ACT_NONE; g.group_m = 4;
    g.lr = lr; g.b1 = b1; g.b2 = b2; g.eps = eps; g.wd = wd; g.opt_m = opt_m[i]; g.opt_v = opt_v[i];
    g.bc1 = 1.f; g.bc2 = 1.f;
    if (epi == EPI_ADAM || epi == EPI_ADAMS || epi == EPI_ADAMS_T) {
      g.bc1 = 1.f - powf(b1, (float)step);
      g.bc2 = 1.f - powf(b2, (float)step);
    }
    g.ksplit = 1; g.tpb = 1; g.variant = 3; g.tpb_req = 1; g.min_bpc = 1; g.ws = nullptr; g.mask = nullptr;
    g.skew = 0;
    tiles += (M[i] / bm) * (N[i] / BT_N);
  }
  const int ncu = num_cu();
  if (ncu <= 0 || tiles > ncu) return -1;
  return (int)(layout == L_TN ? dispatch_tn_pair(epi, a[0], a[1], out_dtype, (hipStream_t)stream)
                              : dispatch_nn_pair(epi, a[0], a[1], out_dtype, (hipStream_t)stream));
}

// which kernel family dllm_gemm would pick (for tests / profiling labels; 224-row tiles need a K-contiguous A too)
int dllm_gemm_path(int in_dtype, int out_dtype, int M, int N, int K, long lda, long ldb, long ldc) {
  const bool al = (lda % 8 == 0) && (ldb % 8 == 0) && (ldc % 4 == 0);  // (bases: checked per call)
  if (in_dtype == DT_BF16 && use_m224(M, N) && K % (2 * BT_K) == 0 && al) return 3;
  if (in_dtype == DT_BF16 && M % BT_M == 0 && N % BT_N == 0 && K % BT_K == 0 && al) return 0;
  if (in_dtype == DT_F32 && out_dtype == DT_F32 && M % FT == 0 && N % FT == 0 && K % FK == 0 && al) return 1;
  return 2;
}

}  // extern "C"
