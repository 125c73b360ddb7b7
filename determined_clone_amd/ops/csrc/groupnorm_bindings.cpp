// Bindings for the NHWC GroupNorm(+SiLU) kernels (groupnorm.hip).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>

namespace dca {
enum class GnDtype : int { kF32 = 0, kBF16 = 1 };
int gn_chunks(int N, int64_t HW, int C);
void groupnorm_forward(GnDtype dt, const void* x, void* y, const float* gamma, const float* beta,
                       int N, int64_t HW, int C, int G, float eps, bool act, float* partial,
                       float* scale, float* shift, float* xa, float* xb, float* mean, float* rstd,
                       hipStream_t st);
void groupnorm_backward(GnDtype dt, const void* dy, const void* x, void* dx, const float* gamma,
                        const float* scale, const float* shift, const float* xa, const float* xb,
                        const float* mean, const float* rstd, int N, int64_t HW, int C, int G,
                        bool act, float* partial, float* ab, float* coef, float* dgamma,
                        float* dbeta, bool accumulate, hipStream_t st);
}  // namespace dca

namespace {
using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

dca::GnDtype gdt(const Tensor& t) {
  if (t.scalar_type() == at::kBFloat16) return dca::GnDtype::kBF16;
  TORCH_CHECK(t.scalar_type() == at::kFloat, "groupnorm: bf16 or fp32 activations required");
  return dca::GnDtype::kF32;
}

// [N, C, H, W] channels_last (or [N, HW, C] contiguous) -> (N, HW, C)
void dims(const Tensor& x, int& N, int64_t& HW, int& C) {
  TORCH_CHECK(x.is_cuda(), "groupnorm: GPU tensor required");
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "groupnorm: channels_last input required");
    N = static_cast<int>(x.size(0)); C = static_cast<int>(x.size(1)); HW = x.size(2) * x.size(3);
  } else {
    TORCH_CHECK(x.dim() == 3 && x.is_contiguous(), "groupnorm: [N, HW, C] contiguous input required");
    N = static_cast<int>(x.size(0)); HW = x.size(1); C = static_cast<int>(x.size(2));
  }
}

const float* fptr(const OptT& t, int64_t n) {
  if (!(t.has_value() && t->defined())) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == n,
              "groupnorm: affine parameters must be contiguous fp32 of C elements");
  return t->data_ptr<float>();
}

// returns y, scale, shift, xa, xb, mean, rstd  (the last six are saved for the backward)
std::vector<Tensor> gn_fwd(const Tensor& x, const OptT& gamma, const OptT& beta, int64_t G,
                           double eps, bool act) {
  int N, C;
  int64_t HW;
  dims(x, N, HW, C);
  TORCH_CHECK(C % 8 == 0 && G > 0 && C % G == 0, "groupnorm: C must be a multiple of 8 and of G");
  const c10::DeviceGuard g(x.device());
  auto fo = x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous);
  Tensor y = torch::empty_like(x);
  const int chunks = dca::gn_chunks(N, HW, C);
  Tensor partial = torch::empty({static_cast<int64_t>(N) * chunks * 2 * C}, fo);
  Tensor scale = torch::empty({N, C}, fo), shift = torch::empty({N, C}, fo);
  Tensor xa = torch::empty({N, C}, fo), xb = torch::empty({N, C}, fo);
  Tensor mean = torch::empty({N, G}, fo), rstd = torch::empty({N, G}, fo);
  dca::groupnorm_forward(gdt(x), x.data_ptr(), y.data_ptr(), fptr(gamma, C), fptr(beta, C), N, HW, C,
                         static_cast<int>(G), static_cast<float>(eps), act, partial.data_ptr<float>(),
                         scale.data_ptr<float>(), shift.data_ptr<float>(), xa.data_ptr<float>(),
                         xb.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), stream());
  return {y, scale, shift, xa, xb, mean, rstd};
}

// returns dx, dgamma, dbeta (dgamma/dbeta undefined when accumulated into *_acc or not needed)
std::vector<Tensor> gn_bwd(const Tensor& dy_in, const Tensor& x, const OptT& gamma,
                           const Tensor& scale, const Tensor& shift, const Tensor& xa,
                           const Tensor& xb, const Tensor& mean, const Tensor& rstd, int64_t G,
                           bool act, bool need_param_grads, const OptT& dgamma_acc,
                           const OptT& dbeta_acc) {
  int N, C;
  int64_t HW;
  dims(x, N, HW, C);
  const c10::DeviceGuard g(x.device());
  Tensor dy = x.dim() == 4 ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "groupnorm: dy dtype must match x");
  auto fo = x.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous);
  Tensor dx = torch::empty_like(x);
  const int chunks = dca::gn_chunks(N, HW, C);
  Tensor partial = torch::empty({static_cast<int64_t>(N) * chunks * 2 * C}, fo);
  Tensor ab = torch::empty({N, 2, C}, fo), coef = torch::empty({N, 3, C}, fo);
  Tensor dgamma, dbeta;
  float *pg = nullptr, *pb = nullptr;
  bool acc = false;
  const bool has_acc = dgamma_acc.has_value() && dgamma_acc->defined() && dbeta_acc.has_value() && dbeta_acc->defined();
  if (need_param_grads && has_acc) {
    for (const Tensor* t : {&*dgamma_acc, &*dbeta_acc})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C,
                  "groupnorm: grad accumulation targets must be contiguous fp32");
    pg = dgamma_acc->data_ptr<float>();
    pb = dbeta_acc->data_ptr<float>();
    acc = true;
  } else if (need_param_grads) {
    dgamma = torch::empty({C}, fo);
    dbeta = torch::empty({C}, fo);
    pg = dgamma.data_ptr<float>();
    pb = dbeta.data_ptr<float>();
  }
  dca::groupnorm_backward(gdt(x), dy.data_ptr(), x.data_ptr(), dx.data_ptr(), fptr(gamma, C),
                          scale.data_ptr<float>(), shift.data_ptr<float>(), xa.data_ptr<float>(),
                          xb.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), N, HW,
                          C, static_cast<int>(G), act, partial.data_ptr<float>(), ab.data_ptr<float>(),
                          coef.data_ptr<float>(), pg, pb, acc, stream());
  return {dx, dgamma, dbeta};
}
}  // namespace

void register_groupnorm_ops(pybind11::module& m) {
  m.def("gn_fwd", &gn_fwd);
  m.def("gn_bwd", &gn_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("gamma"),
        pybind11::arg("scale"), pybind11::arg("shift"), pybind11::arg("xa"), pybind11::arg("xb"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("groups"), pybind11::arg("act"),
        pybind11::arg("need_param_grads"), pybind11::arg("dgamma_acc") = pybind11::none(),
        pybind11::arg("dbeta_acc") = pybind11::none());
}
