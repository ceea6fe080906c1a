// Probe which hipBLASLt epilogues have algorithms for bf16 GEMMs on this GPU.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>
#include <cstdio>

int probe(hipblasLtHandle_t h, hipblasLtEpilogue_t epi, bool aux, hipDataType bias_t, bool set_aux_t, int m, int n,
          int k, hipblasOperation_t ta, hipblasOperation_t tb) {
  hipblasLtMatmulDesc_t op;
  hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
  void* dummy = (void*)0x1000;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dummy, sizeof(dummy));
  int32_t bt = bias_t;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  if (aux) {
    int64_t ld = m;
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &dummy, sizeof(dummy));
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
    if (set_aux_t) {
      int32_t at = HIP_R_16BF;
      hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
    }
  }
  hipblasLtMatrixLayout_t a, b, c;
  int ar = ta == HIPBLAS_OP_N ? m : k, ac = ta == HIPBLAS_OP_N ? k : m;
  int br = tb == HIPBLAS_OP_N ? k : n, bc = tb == HIPBLAS_OP_N ? n : k;
  hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, ar, ac, ar);
  hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, br, bc, br);
  hipblasLtMatrixLayoutCreate(&c, HIP_R_16BF, m, n, m);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = 64ull << 20;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[4];
  int found = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, op, a, b, c, c, pref, 4, res, &found);
  return st == HIPBLAS_STATUS_SUCCESS ? found : -(int)st;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);  // partial results survive a timeout
  hipblasLtHandle_t h;
  hipblasLtCreate(&h);
  if (argc > 1) {
    // bias-gradient epilogues on the WEIGHT-gradient GEMM of a Linear:
    // dW^T[K_in, N_out] = X^T[K_in, M] . dY[M, N_out] (column-major view of
    // row-major dW), db = sum_M dY = reduction of B over the GEMM's K
    struct E { const char* n; hipblasLtEpilogue_t e; };
    E es[] = {{"BGRADA", HIPBLASLT_EPILOGUE_BGRADA}, {"BGRADB", HIPBLASLT_EPILOGUE_BGRADB}};
    int shapes[][3] = {{1600, 6400, 8192}, {6400, 1600, 8192}, {1600, 4800, 8192}, {1600, 1600, 8192},
                       {4096, 4096, 4096}};
    for (auto& e : es)
      for (auto& sh : shapes)
        for (int bt = 0; bt < 2; ++bt)
          for (int ta = 0; ta < 2; ++ta)
            for (int tb = 0; tb < 2; ++tb) {
              int f = probe(h, e.e, false, bt ? HIP_R_32F : HIP_R_16BF, false, sh[0], sh[1], sh[2],
                            ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb ? HIPBLAS_OP_T : HIPBLAS_OP_N);
              printf("%-7s m=%d n=%d k=%d bias=%s transA=%d transB=%d -> %d\n", e.n, sh[0], sh[1], sh[2],
                     bt ? "f32" : "bf16", ta, tb, f);
            }
    return 0;
  }
  struct E { const char* n; hipblasLtEpilogue_t e; bool aux; };
  E es[] = {{"BIAS", HIPBLASLT_EPILOGUE_BIAS, false}, {"GELU", HIPBLASLT_EPILOGUE_GELU, false},
            {"GELU_BIAS", HIPBLASLT_EPILOGUE_GELU_BIAS, false}, {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX, true},
            {"GELU_AUX_BIAS", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS, true}, {"DGELU", HIPBLASLT_EPILOGUE_DGELU, true},
            {"DGELU_BGRAD", HIPBLASLT_EPILOGUE_DGELU_BGRAD, true}};
  for (auto& e : es)
    for (int bt = 0; bt < 2; ++bt)
      for (int sat = 0; sat < 2; ++sat)
        for (int t = 0; t < 2; ++t) {
          hipblasOperation_t ta = t ? HIPBLAS_OP_T : HIPBLAS_OP_N;
          int f = probe(h, e.e, e.aux, bt ? HIP_R_32F : HIP_R_16BF, sat, 6400, 8192, 1600, ta, HIPBLAS_OP_N);
          printf("%-14s bias=%s auxtype=%d transA=%d -> %d\n", e.n, bt ? "f32" : "bf16", sat, t, f);
        }
  return 0;
}
