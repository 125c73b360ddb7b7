// hipBLASLt epilogue support probe (tools/lt_probe.py): how many gfx950 kernels this library build
// (torch's bundled hipBLASLt) offers per epilogue / transpose / bias type / aux type. Used to
// decide whether the transformer MLP's elementwise passes could ride on GEMM epilogues: this build
// has no GELU_AUX(_BIAS) and no DGELU_BGRAD, and its DGELU kernels made the GPT-2 step 20 % slower
// than GEMM + the fused bias_gelu_bwd pass (profiles/round5_lt_mlp_ab.txt), so none is used.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>

namespace {
using torch::Tensor;

#define LT_CHECK(expr)                                                                          \
  do {                                                                                          \
    const hipblasStatus_t s_ = (expr);                                                          \
    TORCH_CHECK(s_ == HIPBLAS_STATUS_SUCCESS, "hipBLASLt: ", #expr, " failed with status ", \
                static_cast<int>(s_));                                                          \
  } while (0)

hipblasLtHandle_t handle() {
  static std::mutex mu;
  static std::map<int, hipblasLtHandle_t> handles;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  auto it = handles.find(dev);
  if (it != handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  LT_CHECK(hipblasLtCreate(&h));
  handles[dev] = h;
  return h;
}

constexpr size_t kWorkspace = size_t{32} << 20;

// Number of heuristic algorithms hipBLASLt offers for one configuration (support probe: which
// epilogue / bias type / aux type / transpose combinations this library build has kernels for).
int lt_probe(int64_t epi, int64_t m, int64_t n, int64_t k, bool ta, bool tb, int64_t bias_type,
             int64_t aux_type, bool set_ptrs) {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
  LT_CHECK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  const hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  const hipblasLtEpilogue_t e = static_cast<hipblasLtEpilogue_t>(epi);
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (bias_type >= 0) {
    const hipDataType bt = static_cast<hipDataType>(bias_type);
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  if (aux_type >= 0) {
    const hipDataType at_ = static_cast<hipDataType>(aux_type);
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &at_, sizeof(at_)));
    const int64_t ld_aux = m;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld_aux, sizeof(ld_aux)));
  }
  void* dummy = reinterpret_cast<void*>(uintptr_t{4096});
  if (set_ptrs) {
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dummy, sizeof(dummy)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &dummy, sizeof(dummy)));
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&la, HIP_R_16BF, ta ? k : m, ta ? m : k, ta ? k : m));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_16BF, tb ? n : k, tb ? k : n, tb ? n : k));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&ld, HIP_R_16BF, m, n, m));
  hipblasLtMatmulPreference_t pref = nullptr;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t ws = kWorkspace;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int found = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(handle(), desc, la, lb, ld, ld, pref, 8, res, &found);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(la);
  hipblasLtMatrixLayoutDestroy(lb);
  hipblasLtMatrixLayoutDestroy(ld);
  hipblasLtMatmulDescDestroy(desc);
  return st == HIPBLAS_STATUS_SUCCESS ? found : -static_cast<int>(st);
}

}  // namespace

void register_lt_ops(pybind11::module& m) {
  m.def("lt_probe", &lt_probe);
}
