// Bindings for the large-tile MFMA GEMM (gemm.hip).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>

#include "gemm_api.h"

namespace {
using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// a [..., K] (rows contiguous in K, any uniform row stride), b [N, K] -> (rows, lda)
int64_t rows_of(const Tensor& a, int64_t K, const char* what) {
  TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && a.dim() >= 2 && a.size(-1) == K &&
                  a.stride(-1) == 1,
              what, ": bf16 GPU tensor [..., K] with unit stride along K required");
  TORCH_CHECK(a.is_contiguous(), what, ": contiguous activations required");
  return a.numel() / K;
}

void check_shapes(int64_t M, int64_t N, int64_t K) {
  TORCH_CHECK(N % 256 == 0 && K % 64 == 0 && M >= 1, "gemm_nt: N % 256 == 0 and K % 64 == 0 required");
  // buffer-descriptor byte offsets are 32-bit with 2^31 as the out-of-range marker
  TORCH_CHECK(M * K < (int64_t{1} << 30) && N * K < (int64_t{1} << 30) && M < (int64_t{1} << 31),
              "gemm_nt: operands too large for 32-bit byte offsets");
}

Tensor f32_bias(const OptT& bias, int64_t N) {
  if (!bias.has_value() || !bias->defined()) return Tensor();
  TORCH_CHECK(bias->numel() == N && bias->is_cuda(), "gemm_nt: bias must be a GPU tensor of N elements");
  return bias->to(at::kFloat).contiguous();
}

// c = a @ b.T (+ bias): the projection of nn.Linear with weight b [N, K].
Tensor gemm_nt(const Tensor& a, const Tensor& b, const OptT& bias) {
  const c10::DeviceGuard dg(a.device());
  TORCH_CHECK(b.is_cuda() && b.scalar_type() == at::kBFloat16 && b.dim() == 2 && b.is_contiguous(),
              "gemm_nt: contiguous bf16 weight [N, K] required");
  const int64_t N = b.size(0), K = b.size(1);
  const int64_t M = rows_of(a, K, "gemm_nt");
  check_shapes(M, N, K);
  std::vector<int64_t> shape(a.sizes().begin(), a.sizes().end());
  shape.back() = N;
  Tensor c = torch::empty(shape, a.options());
  const Tensor bf = f32_bias(bias, N);
  dca::gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), static_cast<int>(M), static_cast<int>(N),
               static_cast<int>(K), static_cast<int>(K), static_cast<int>(K), static_cast<int>(N),
               dca::kGemmStore, bf.defined() ? bf.data_ptr<float>() : nullptr, nullptr, nullptr, stream());
  return c;
}

// GPT-2 MLP backward through the output projection and the GELU:
//   dz = (dy @ w2) * gelu'(z + bias), w2t = w2.T contiguous [F, E] (K = E), z [..., F]
// plus the fc-bias gradient's per-row-block column sums of dz, partial [blocks, F].
std::vector<Tensor> gemm_nt_dgelu(const Tensor& dy, const Tensor& w2t, const Tensor& z_in, const Tensor& bias) {
  const c10::DeviceGuard dg(dy.device());
  TORCH_CHECK(w2t.is_cuda() && w2t.scalar_type() == at::kBFloat16 && w2t.dim() == 2 && w2t.is_contiguous(),
              "gemm_nt_dgelu: contiguous bf16 [F, E] weight required");
  const int64_t F = w2t.size(0), E = w2t.size(1);
  const int64_t M = rows_of(dy, E, "gemm_nt_dgelu");
  const Tensor z = z_in.contiguous();
  TORCH_CHECK(z.scalar_type() == at::kBFloat16 && z.size(-1) == F && z.numel() / F == M,
              "gemm_nt_dgelu: z must be bf16 [..., F] with dy's rows");
  check_shapes(M, F, E);
  TORCH_CHECK(M * F < (int64_t{1} << 31), "gemm_nt_dgelu: output too large");
  const Tensor bf = f32_bias(bias, F);
  TORCH_CHECK(bf.defined(), "gemm_nt_dgelu: bias required");
  std::vector<int64_t> shape(z.sizes().begin(), z.sizes().end());
  Tensor dz = torch::empty(shape, z.options());
  Tensor partial = torch::empty({dca::gemm_nt_row_blocks(static_cast<int>(M)), F}, dy.options().dtype(at::kFloat));
  dca::gemm_nt(dy.data_ptr(), w2t.data_ptr(), dz.data_ptr(), static_cast<int>(M), static_cast<int>(F),
               static_cast<int>(E), static_cast<int>(E), static_cast<int>(E), static_cast<int>(F),
               dca::kGemmDGelu, bf.data_ptr<float>(), z.data_ptr(), partial.data_ptr<float>(), stream());
  return {dz, partial};
}

}  // namespace

void register_gemm_ops(pybind11::module& m) {
  m.def("gemm_nt", &gemm_nt, pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("bias") = pybind11::none());
  m.def("gemm_nt_dgelu", &gemm_nt_dgelu, pybind11::arg("dy"), pybind11::arg("w2t"), pybind11::arg("z"),
        pybind11::arg("bias"));
}
