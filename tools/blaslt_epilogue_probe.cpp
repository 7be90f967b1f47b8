// Probe: does hipBLASLt on this GPU run the BERT FFN with fused epilogues, and how fast?
//   fwd  : Y = GELU(X W1^T + b1) with the pre-activation Z as the aux output (GELU_AUX_BIAS)
//   bwd  : dZ = (dY2 W2) * GELU'(Z) with the bias gradient (DGELU_BGRAD)
// against the plain GEMMs (EPILOGUE_DEFAULT).  BERT-base FFN shapes at 8 episodes of 10-way 5-shot Q=5:
// T = 102400 tokens, H = 768, I = 3072.  Prints heuristic status and the mean time of 20 runs.
// Build: hipcc --offload-arch=gfx950 -O2 tools/blaslt_epilogue_probe.cpp -lhipblaslt -o variants/blaslt_probe
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    auto e = (x);                                                               \
    if ((int)e != 0) {                                                          \
      std::printf("FAIL %s -> %d (line %d)\n", #x, (int)e, __LINE__);           \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

static int run(hipblasLtHandle_t h, const char* name, hipblasLtEpilogue_t epi, int64_t m, int64_t n, int64_t k,
               hipblasOperation_t ta, int64_t lda, hipblasOperation_t tb, int64_t ldb, const void* A, const void* B,
               void* D, void* bias, hipDataType bias_t, void* aux, void* ws, size_t wsb, hipStream_t st) {
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (bias) {
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    int32_t bt = bias_t;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (aux) {
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
    int64_t ld = m;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    int32_t at = HIP_R_16BF;   // bf16 pre-activation
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at)));
  }
  hipblasLtMatrixLayout_t la, lb, ld;
  const int64_t ar = ta == HIPBLAS_OP_N ? m : k, ac = ta == HIPBLAS_OP_N ? k : m;
  const int64_t br = tb == HIPBLAS_OP_N ? k : n, bc = tb == HIPBLAS_OP_N ? n : k;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ar, ac, lda));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, br, bc, ldb));
  CK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, m, n, m));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t w = wsb;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w, sizeof(w)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int got = 0;
  auto hs = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, ld, ld, pref, 8, res, &got);
  std::printf("%-28s heuristic status %d, %d algos\n", name, (int)hs, got);
  if (hs != HIPBLAS_STATUS_SUCCESS || got == 0) return 0;
  const float alpha = 1.f, beta = 0.f;
  float best = 1e30f;
  for (int a = 0; a < got && a < 4; ++a) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto r = hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[a].algo, ws, wsb, st);
    if (r != HIPBLAS_STATUS_SUCCESS) {
      std::printf("  algo %d: matmul status %d\n", a, (int)r);
      continue;
    }
    hipEventRecord(e0, st);
    for (int i = 0; i < 20; ++i) hipblasLtMatmul(h, desc, &alpha, A, la, B, lb, &beta, D, ld, D, ld, &res[a].algo, ws, wsb, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const float us = ms * 1000.f / 20.f;
    std::printf("  algo %d: %.1f us  (%.0f TFLOP/s)\n", a, us, 2.0 * m * n * k / (us * 1e-6) / 1e12);
    if (us < best) best = us;
  }
  std::printf("  best %.1f us\n", best);
  return 0;
}

int main() {
  const int64_t T = 102400, H = 768, I = 3072;
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  void *X, *W1, *Y, *Z, *b1, *dY2, *W2, *dZ, *db, *ws;
  const size_t wsb = 64ull << 20;
  CK(hipMalloc(&X, T * H * 2));
  CK(hipMalloc(&W1, I * H * 2));
  CK(hipMalloc(&Y, T * I * 2));
  CK(hipMalloc(&Z, T * I * 2));
  CK(hipMalloc(&b1, I * 4));
  CK(hipMalloc(&dY2, T * H * 2));
  CK(hipMalloc(&W2, H * I * 2));
  CK(hipMalloc(&dZ, T * I * 2));
  CK(hipMalloc(&db, I * 4));
  CK(hipMalloc(&ws, wsb));
  hipMemset(X, 0, T * H * 2);
  hipMemset(W1, 0, I * H * 2);
  hipMemset(b1, 0, I * 4);
  hipMemset(dY2, 0, T * H * 2);
  hipMemset(W2, 0, H * I * 2);
  hipMemset(Z, 0, T * I * 2);
  // column-major view: D[I x T] = op(A) [I x H] * op(B) [H x T]; A = W1 row-major [I, H] = col-major [H x I] (T op)
  run(h, "fwd plain", HIPBLASLT_EPILOGUE_DEFAULT, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H, W1, X, Y, nullptr,
      HIP_R_32F, nullptr, ws, wsb, st);
  run(h, "fwd bias", HIPBLASLT_EPILOGUE_BIAS, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H, W1, X, Y, b1, HIP_R_32F,
      nullptr, ws, wsb, st);
  run(h, "fwd GELU_AUX_BIAS (f32 bias)", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H,
      W1, X, Y, b1, HIP_R_32F, Z, ws, wsb, st);
  run(h, "fwd GELU_AUX_BIAS (bf16 bias)", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N,
      H, W1, X, Y, b1, HIP_R_16BF, Z, ws, wsb, st);
  run(h, "fwd GELU", HIPBLASLT_EPILOGUE_GELU, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H, W1, X, Y, nullptr, HIP_R_32F,
      nullptr, ws, wsb, st);
  run(h, "fwd GELU_BIAS (f32 bias)", HIPBLASLT_EPILOGUE_GELU_BIAS, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H, W1, X,
      Y, b1, HIP_R_32F, nullptr, ws, wsb, st);
  run(h, "fwd GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX, I, T, H, HIPBLAS_OP_T, H, HIPBLAS_OP_N, H, W1, X, Y, nullptr,
      HIP_R_32F, Z, ws, wsb, st);
  // bwd: dH[I x T] = W2^T-ish: W2 row-major [H, I] = col-major [I x H] (N op), dY2 row-major [T, H] = col-major [H x T]
  run(h, "bwd plain", HIPBLASLT_EPILOGUE_DEFAULT, I, T, H, HIPBLAS_OP_N, I, HIPBLAS_OP_N, H, W2, dY2, dZ, nullptr,
      HIP_R_32F, nullptr, ws, wsb, st);
  run(h, "bwd DGELU", HIPBLASLT_EPILOGUE_DGELU, I, T, H, HIPBLAS_OP_N, I, HIPBLAS_OP_N, H, W2, dY2, dZ, nullptr,
      HIP_R_32F, Z, ws, wsb, st);
  run(h, "bwd DGELU_BGRAD (f32 db)", HIPBLASLT_EPILOGUE_DGELU_BGRAD, I, T, H, HIPBLAS_OP_N, I, HIPBLAS_OP_N, H, W2,
      dY2, dZ, db, HIP_R_32F, Z, ws, wsb, st);
  std::printf("done\n");
  return 0;
}
