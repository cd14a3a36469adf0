// hipBLASLt GEMMs with fused GELU epilogues for the transformer MLP (SURVEY
// K-M10): the library GEMMs the MLP already runs on, with the elementwise work
// moved into the GEMM epilogue so the [T, ffn] activation tensors cross HBM
// fewer times.
//
//   forward :  z = x W1^T + b1 (aux, bf16),  h = gelu(z)          GELU_AUX_BIAS
//   backward:  dz = (dy W2) * gelu'(z),  db1 = colsum(dz) (fp32)   DGELU_BGRAD
//
// Separate elementwise kernels would read z back and write h (forward), and
// write dh then read dh + z and write dz (backward).
//
// Row-major tensors are handed to the column-major library as their transposes:
// Y[T,N] = X[T,K] W[N,K]^T  <=>  Y^T (N x T, ld N) = op_T(W: K x N, ld K) * X^T (K x T, ld K).
// Descriptors and the heuristic's first algorithm are cached per shape; the
// per-call pointers (bias, aux) are re-set on the cached descriptor.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace dpa {
namespace {

#define DPA_LT_CHECK(expr)                                                                        \
  do {                                                                                            \
    hipblasStatus_t st_ = (expr);                                                                 \
    TORCH_CHECK(st_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed (", (int)st_, ")"); \
  } while (0)

constexpr size_t kWorkspace = 32u << 20;

enum Kind : int { FWD_GELU_AUX = 0, BWD_DGELU_BGRAD = 1, BWD_DGELU = 2 };

struct Plan {
  hipblasLtMatmulDesc_t op = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  bool ok = false;
};

struct State {
  hipblasLtHandle_t handle = nullptr;
  std::map<std::tuple<int, int64_t, int64_t, int64_t, int>, Plan> plans;
  std::mutex mu;
};

State& state() {
  static State s;
  return s;
}

hipblasLtHandle_t handle() {
  State& s = state();
  if (!s.handle) DPA_LT_CHECK(hipblasLtCreate(&s.handle));
  return s.handle;
}

// D (m x n col-major, ld m) = op(A) * B; A stored (transA ? k x m : m x k), B stored k x n.
Plan make_plan(int kind, int64_t m, int64_t n, int64_t k, bool transA, int64_t lda, int64_t ldb,
               bool has_bias) {
  Plan p;
  DPA_LT_CHECK(hipblasLtMatmulDescCreate(&p.op, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const int32_t ta = transA ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = HIPBLAS_OP_N;
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  uint32_t epi;
  int32_t bias_type;
  if (kind == FWD_GELU_AUX) {
    epi = has_bias ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_GELU_AUX;
    bias_type = HIP_R_16BF;
  } else {
    epi = kind == BWD_DGELU_BGRAD ? HIPBLASLT_EPILOGUE_DGELU_BGRAD : HIPBLASLT_EPILOGUE_DGELU;
    bias_type = HIP_R_32F;
  }
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (has_bias || kind == BWD_DGELU_BGRAD)
    DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE,
                                                 &bias_type, sizeof(bias_type)));
  const int64_t ld_aux = m;
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld_aux,
                                               sizeof(ld_aux)));
  const int32_t aux_type = HIP_R_16BF;
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE,
                                               &aux_type, sizeof(aux_type)));
  DPA_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, transA ? k : m, transA ? m : k, lda));
  DPA_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, k, n, ldb));
  DPA_LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, m, n, m));

  hipblasLtMatmulPreference_t pref;
  DPA_LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t ws = kWorkspace;
  DPA_LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES,
                                                     &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[4];
  int n_res = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(handle(), p.op, p.a, p.b, p.d, p.d, pref, 4,
                                                       res, &n_res);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st == HIPBLAS_STATUS_SUCCESS && n_res > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS) {
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    p.ok = true;
  }
  return p;
}

Plan& get_plan(int kind, int64_t m, int64_t n, int64_t k, bool transA, int64_t lda, int64_t ldb,
               bool has_bias) {
  State& s = state();
  std::lock_guard<std::mutex> g(s.mu);
  const auto key = std::make_tuple(kind * 2 + (int)has_bias, m, n, k, (int)transA);
  auto it = s.plans.find(key);
  if (it == s.plans.end())
    it = s.plans.emplace(key, make_plan(kind, m, n, k, transA, lda, ldb, has_bias)).first;
  return it->second;
}

void run(Plan& p, const void* A, const void* B, void* D, const void* bias, const void* aux,
         hipStream_t stream) {
  // the bias / aux pointers live in the (cached) descriptor: re-set per call
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                               sizeof(bias)));
  DPA_LT_CHECK(hipblasLtMatmulDescSetAttribute(p.op, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux,
                                               sizeof(aux)));
  at::DataPtr ws;
  void* wsp = nullptr;
  if (p.ws > 0) {
    ws = c10::hip::HIPCachingAllocator::get()->allocate(p.ws);
    wsp = ws.get();
  }
  const float alpha = 1.f, beta = 0.f;
  DPA_LT_CHECK(hipblasLtMatmul(handle(), p.op, &alpha, A, p.a, B, p.b, &beta, D, p.d, D, p.d, &p.algo,
                               wsp, p.ws, stream));
}

void check_bf16_2d(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.is_contiguous(),
              name, " must be a contiguous 2-D bf16 HIP tensor");
}

// [h, z] with z = x W^T + b and h = gelu(z); [] if the library has no kernel for it.
std::vector<at::Tensor> lt_linear_gelu(const at::Tensor& x, const at::Tensor& W,
                                       const c10::optional<at::Tensor>& b) {
  check_bf16_2d(x, "x");
  check_bf16_2d(W, "W");
  const int64_t T = x.size(0), K = x.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K, "W shape");
  const bool hb = b.has_value() && b->defined();
  if (hb) TORCH_CHECK(b->is_cuda() && b->scalar_type() == at::kBFloat16 && b->numel() == N, "bias");
  Plan& p = get_plan(FWD_GELU_AUX, N, T, K, true, K, K, hb);
  if (!p.ok) return {};
  auto h = at::empty({T, N}, x.options());
  auto z = at::empty({T, N}, x.options());
  run(p, W.data_ptr(), x.data_ptr(), h.data_ptr(), hb ? b->data_ptr() : nullptr, z.data_ptr(),
      c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  return {h, z};
}

// [dz(, db)] with dz = (dy W) * gelu'(z) and db = colsum(dz) in fp32 (if want_db).
std::vector<at::Tensor> lt_dgrad_dgelu(const at::Tensor& dy, const at::Tensor& W, const at::Tensor& z,
                                       bool want_db) {
  check_bf16_2d(dy, "dy");
  check_bf16_2d(W, "W");
  check_bf16_2d(z, "z");
  const int64_t T = dy.size(0), N = dy.size(1), F = W.size(1);
  TORCH_CHECK(W.size(0) == N && z.size(0) == T && z.size(1) == F, "shapes");
  // dZ^T (F x T) = W-as-stored (F x N, ld F) * dY^T (N x T, ld N)
  Plan& p = get_plan(want_db ? BWD_DGELU_BGRAD : BWD_DGELU, F, T, N, false, F, N, false);
  if (!p.ok) return {};
  auto dz = at::empty({T, F}, dy.options());
  at::Tensor db;
  if (want_db) db = at::empty({F}, dy.options().dtype(at::kFloat));
  run(p, W.data_ptr(), dy.data_ptr(), dz.data_ptr(), want_db ? db.data_ptr() : nullptr, z.data_ptr(),
      c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream());
  if (want_db) return {dz, db};
  return {dz};
}

}  // namespace

void register_blaslt(pybind11::module& m) {
  m.def("lt_linear_gelu", &lt_linear_gelu,
        "hipBLASLt GELU_AUX_BIAS: [gelu(x W^T + b), x W^T + b]; [] if unsupported");
  m.def("lt_dgrad_dgelu", &lt_dgrad_dgelu,
        "hipBLASLt DGELU(_BGRAD): [(dy W) * gelu'(z), colsum fp32]; [] if unsupported");
}

}  // namespace dpa
