// GEMMs with fused epilogues through hipBLASLt (library GEMM + its epilogue
// stage, so no separate elementwise pass over the activation gradient):
//
//  * dw_gemm_dgelu_bgrad     dh = (dy W2) * gelu'(pre), db = sum_rows dh
//      (HIPBLASLT_EPILOGUE_DGELU_BGRAD on the c_proj dgrad GEMM)
//  * dw_gemm_dgelu           dh = (dy W2) * gelu'(pre)   (HIPBLASLT_EPILOGUE_DGELU)
//  * dw_gemm_wgrad_bgradb    dW (+)= dy^T x, db = sum_rows dy  (HIPBLASLT_EPILOGUE_BGRADB)
//
// Probed on gfx950 / ROCm 7.2 (scripts/probe/epi_probe.cpp,
// profiles/r2/hipblaslt_epilogue_probe.txt): GELU_AUX(_BIAS) has no bf16
// algorithm, DGELU has one for non-transposed A, DGELU_BGRAD only for some
// shapes -- so the forward keeps the bias epilogue + a GELU pass and the
// backward tries BGRAD, then DGELU, per shape.
//
// Row-major tensors are handed to the column-major library as their
// transposes: out^T[N, M] = W[N, K] . x^T[K, M].  One handle + 64 MiB
// workspace per device, heuristics cached per (kind, shape).  When the
// library has no algorithm for a combination the call returns
// DW_EPI_UNSUPPORTED and the caller keeps its unfused path.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

#define DW_EPI_UNSUPPORTED (-100)

namespace {

struct Dev {
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  size_t ws_bytes = 64ull << 20;
};

std::mutex g_mu;
std::map<int, Dev> g_dev;
// (kind, M, N, K) -> algo (or "none")
std::map<std::tuple<int, int, int, int>, std::pair<bool, hipblasLtMatmulAlgo_t>> g_algo;

Dev* dev_state() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return nullptr;
  auto it = g_dev.find(d);
  if (it != g_dev.end()) return &it->second;
  Dev s;
  if (hipblasLtCreate(&s.h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
  if (hipMalloc(&s.ws, s.ws_bytes) != hipSuccess) {
    hipblasLtDestroy(s.h);
    return nullptr;
  }
  return &(g_dev[d] = s);
}

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  ~Plan() {
    if (op) hipblasLtMatmulDescDestroy(op);
    if (a) hipblasLtMatrixLayoutDestroy(a);
    if (b) hipblasLtMatrixLayoutDestroy(b);
    if (c) hipblasLtMatrixLayoutDestroy(c);
  }
};

#define CK(x)                                  \
  do {                                         \
    if ((x) != HIPBLAS_STATUS_SUCCESS) return -1; \
  } while (0)

// D[m, n] (col-major, ld m) = op(A) op(B) (+ D when beta = 1) with the given epilogue
int run(int kind, hipblasOperation_t ta, hipblasOperation_t tb, int m, int n, int k, const void* A, int lda,
        const void* B, int ldb, void* D, hipblasLtEpilogue_t epi, const void* bias, hipDataType bias_type,
        const void* aux, int64_t aux_ld, hipStream_t stream, float beta = 0.f) {
  std::lock_guard<std::mutex> lk(g_mu);
  Dev* dv = dev_state();
  if (!dv) return -1;
  Plan p;
  CK(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (bias) {
    CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)));
    int32_t bt = (int32_t)bias_type;
    CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (aux) {
    CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux)));
    CK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &aux_ld, sizeof(aux_ld)));
  }
  const int ar = ta == HIPBLAS_OP_N ? m : k, ac = ta == HIPBLAS_OP_N ? k : m;
  const int br = tb == HIPBLAS_OP_N ? k : n, bc = tb == HIPBLAS_OP_N ? n : k;
  CK(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ar, ac, lda));
  CK(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, br, bc, ldb));
  CK(hipblasLtMatrixLayoutCreate(&p.c, HIP_R_16BF, m, n, m));

  auto key = std::make_tuple(kind, m, n, k);
  auto it = g_algo.find(key);
  if (it == g_algo.end()) {
    hipblasLtMatmulPreference_t pref;
    CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t wsb = dv->ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[1];
    int found = 0;
    hipblasStatus_t st =
        hipblasLtMatmulAlgoGetHeuristic(dv->h, p.op, p.a, p.b, p.c, p.c, pref, 1, res, &found);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || found == 0) {
      g_algo[key] = {false, {}};
      return DW_EPI_UNSUPPORTED;
    }
    it = g_algo.emplace(key, std::make_pair(true, res[0].algo)).first;
  }
  if (!it->second.first) return DW_EPI_UNSUPPORTED;
  const float alpha = 1.f;
  CK(hipblasLtMatmul(dv->h, p.op, &alpha, A, p.a, B, p.b, &beta, D, p.c, D, p.c, &it->second.second, dv->ws,
                     dv->ws_bytes, stream));
  return 0;
}

}  // namespace

// dy [M, N2], w2 [N2, N1] (c_proj weight), pre [M, N1] -> dh [M, N1] bf16,
// dbias [N1] fp32 (written, not accumulated)
extern "C" int dw_gemm_dgelu_bgrad(const void* dy, const void* w2, const void* pre, void* dh, void* dbias, int M,
                                   int N1, int N2, void* stream) {
  return run(1, HIPBLAS_OP_N, HIPBLAS_OP_N, N1, M, N2, w2, N1, dy, N2, dh, HIPBLASLT_EPILOGUE_DGELU_BGRAD, dbias,
             HIP_R_32F, pre, N1, (hipStream_t)stream);
}

// dy [M, N2], w2 [N2, N1], pre [M, N1] -> dh [M, N1] bf16
extern "C" int dw_gemm_dgelu(const void* dy, const void* w2, const void* pre, void* dh, int M, int N1, int N2,
                             void* stream) {
  return run(2, HIPBLAS_OP_N, HIPBLAS_OP_N, N1, M, N2, w2, N1, dy, N2, dh, HIPBLASLT_EPILOGUE_DGELU, nullptr,
             HIP_R_16BF, pre, N1, (hipStream_t)stream);
}

// Weight gradient of a Linear with its bias gradient in the epilogue:
// dW [N, K] (+)= dy^T x, db [N] fp32 = sum over the M rows of dy
// (HIPBLASLT_EPILOGUE_BGRADB: the reduction of B over the GEMM's k).  In the
// library's column-major view dW^T [K, N] = x^T [K, M] . (dy^T [N, M])^T, i.e.
// transA = N, transB = T -- the one combination the gfx950 probe finds
// algorithms for (profiles/r4/hipblaslt_bgrad_probe.txt).  accumulate: beta 1
// on dW (direct flat-gradient storage); db is always written.
extern "C" int dw_gemm_wgrad_bgradb(const void* x, const void* dy, void* dw, void* db, int M, int K, int N,
                                    int accumulate, void* stream) {
  return run(3, HIPBLAS_OP_N, HIPBLAS_OP_T, K, N, M, x, K, dy, N, dw, HIPBLASLT_EPILOGUE_BGRADB, db, HIP_R_32F,
             nullptr, 0, (hipStream_t)stream, accumulate ? 1.f : 0.f);
}
