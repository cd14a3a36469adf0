// Which hipBLASLt epilogues have gfx950 bf16 kernels?  Asks the heuristic for
// each (epilogue, aux dtype set or not, bias dtype) at the MLP's shapes and
// prints how many algorithms it returns.  Built against torch's libhipblaslt.
#include <hipblaslt/hipblaslt.h>
#include <cstdio>
#include <cstdint>

static int try_one(hipblasLtHandle_t h, int epi, int transA, int64_t m, int64_t n, int64_t k,
                   int set_aux, int bias_type, int d_type) {
  hipblasLtMatmulDesc_t op;
  hipblasLtMatmulDescCreate(&op, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  int32_t ta = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
  uint32_t e = epi;
  hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  if (bias_type >= 0) hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_type, sizeof(bias_type));
  if (set_aux) {
    int64_t ld = m;
    hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
    int32_t at = HIP_R_16BF;
    if (set_aux == 2) hipblasLtMatmulDescSetAttribute(op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at, sizeof(at));
  }
  hipblasLtMatrixLayout_t a, b, c, d;
  hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, transA ? k : m, transA ? m : k, transA ? k : m);
  hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, k, n, k);
  hipblasLtMatrixLayoutCreate(&c, (hipDataType)d_type, m, n, m);
  hipblasLtMatrixLayoutCreate(&d, (hipDataType)d_type, m, n, m);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  uint64_t ws = 32u << 20;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws));
  hipblasLtMatmulHeuristicResult_t res[8];
  int nr = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, op, a, b, c, d, pref, 8, res, &nr);
  return st == HIPBLAS_STATUS_SUCCESS ? nr : -(int)st;
}

int main() {
  hipblasLtHandle_t h;
  hipblasLtCreate(&h);
  struct { const char* name; int epi; } epis[] = {
      {"DEFAULT", HIPBLASLT_EPILOGUE_DEFAULT}, {"BIAS", HIPBLASLT_EPILOGUE_BIAS},
      {"GELU", HIPBLASLT_EPILOGUE_GELU}, {"GELU_BIAS", HIPBLASLT_EPILOGUE_GELU_BIAS},
      {"GELU_AUX", HIPBLASLT_EPILOGUE_GELU_AUX}, {"GELU_AUX_BIAS", HIPBLASLT_EPILOGUE_GELU_AUX_BIAS},
      {"DGELU", HIPBLASLT_EPILOGUE_DGELU}, {"DGELU_BGRAD", HIPBLASLT_EPILOGUE_DGELU_BGRAD},
      {"BGRADB", HIPBLASLT_EPILOGUE_BGRADB}};
  const int64_t T = 262144;
  for (auto& E : epis)
    for (int transA = 0; transA < 2; ++transA)
      for (int set_aux = 0; set_aux < 3; ++set_aux)
        for (int bt : {-1, (int)HIP_R_16BF, (int)HIP_R_32F}) {
          int m = transA ? 3072 : 3072, k = transA ? 768 : 768;
          int nr = try_one(h, E.epi, transA, m, T, k, set_aux, bt, HIP_R_16BF);
          printf("%-14s transA=%d aux=%d bias_t=%3d -> %d\n", E.name, transA, set_aux, bt, nr);
        }
  return 0;
}
