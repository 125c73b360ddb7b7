// Bindings for the implicit-GEMM convolution family (conv_igemm.hip).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>

#include "conv_api.h"

namespace {
using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

// NHWC activation [N, C, H, W] (channels_last) viewed as a row-major [N*H*W][C] matrix.
int64_t nhwc_rows(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4, what,
              ": bf16 4-D GPU tensor required");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what, ": channels_last layout required");
  TORCH_CHECK(t.size(1) % 64 == 0, what, ": channels must be a multiple of 64");
  const int64_t M = t.size(0) * t.size(2) * t.size(3);
  TORCH_CHECK(M < (int64_t{1} << 31), what, ": too many rows");
  return M;
}

Tensor nhwc_empty(const Tensor& like, int64_t c) {
  return torch::empty({like.size(0), c, like.size(2), like.size(3)},
                      like.options().memory_format(at::MemoryFormat::ChannelsLast));
}

// ---------------------------------------------------------------- k x k implicit GEMM
void check_nhwc(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4, what,
              ": bf16 4-D GPU tensor required");
  TORCH_CHECK(t.is_contiguous(at::MemoryFormat::ChannelsLast), what, ": channels_last layout required");
  TORCH_CHECK(t.size(1) % 64 == 0, what, ": channels must be a multiple of 64");
  // byte offsets of the buffer loads are 32-bit with 2^31 as the out-of-range marker
  TORCH_CHECK(t.numel() < (int64_t{1} << 30), what, ": tensor too large for 32-bit byte offsets");
}

dca::ConvGeom geom(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(1) == x.size(1),
              "conv_igemm: weight must be bf16 [K, C, R, S] matching the input channels");
  TORCH_CHECK(w.is_contiguous(at::MemoryFormat::ChannelsLast), "conv_igemm: weight must be channels_last");
  TORCH_CHECK(w.size(0) % 64 == 0, "conv_igemm: output channels must be a multiple of 64");
  TORCH_CHECK(stride >= 1 && pad >= 0, "conv_igemm: bad stride / padding");
  dca::ConvGeom g;
  g.N = static_cast<int>(x.size(0));
  g.C = static_cast<int>(x.size(1));
  g.H = static_cast<int>(x.size(2));
  g.W = static_cast<int>(x.size(3));
  g.K = static_cast<int>(w.size(0));
  g.R = static_cast<int>(w.size(2));
  g.S = static_cast<int>(w.size(3));
  g.stride = static_cast<int>(stride);
  g.pad = static_cast<int>(pad);
  g.P = static_cast<int>((g.H + 2 * pad - g.R) / stride + 1);
  g.Q = static_cast<int>((g.W + 2 * pad - g.S) / stride + 1);
  TORCH_CHECK(g.P > 0 && g.Q > 0, "conv_igemm: empty output");
  const int64_t M = static_cast<int64_t>(g.N) * g.P * g.Q;
  TORCH_CHECK(M * g.K < (int64_t{1} << 31), "conv_igemm: output too large for 32-bit offsets");
  g.M = static_cast<int>(M);
  return g;
}

// y = conv2d(x, w, stride, pad) (no bias); with `stats` also the [blocks, 2, K] BatchNorm partial
// statistics of y.
std::vector<Tensor> conv_igemm_fwd(const Tensor& x, const Tensor& w, int64_t stride, int64_t pad,
                                   bool stats) {
  const c10::DeviceGuard dg(x.device());
  check_nhwc(x, "conv_igemm_fwd");
  const dca::ConvGeom g = geom(x, w, stride, pad);
  Tensor y = torch::empty({g.N, g.K, g.P, g.Q}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor partial;
  if (stats) partial = torch::empty({dca::conv_igemm_row_blocks(g), 2, g.K}, x.options().dtype(at::kFloat));
  dca::conv_igemm_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(),
                      stats ? partial.data_ptr<float>() : nullptr, g, stream());
  return {y, partial};
}

// dx of a stride-1 convolution: the forward kernel on dy with the flipped, transposed weight.
Tensor conv_igemm_dgrad(const Tensor& dy_in, const Tensor& w, int64_t pad) {
  const Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const c10::DeviceGuard dg(dy.device());
  check_nhwc(dy, "conv_igemm_dgrad");
  TORCH_CHECK(w.dim() == 4 && w.size(0) == dy.size(1) && w.size(1) % 64 == 0 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.scalar_type() == at::kBFloat16,
              "conv_igemm_dgrad: weight must be bf16 channels_last [K, C, R, S], C a multiple of 64");
  const int64_t K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3);
  TORCH_CHECK(R == S && pad <= R - 1, "conv_igemm_dgrad: square kernels, padding < kernel");
  // [C, K, R, S] channels_last == physical [C][R][S][K]
  Tensor wt = torch::empty({C, K, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  dca::conv_flip_transpose(w.data_ptr(), wt.data_ptr(), static_cast<int>(K), static_cast<int>(C),
                           static_cast<int>(R * S), stream());
  const dca::ConvGeom g = geom(dy, wt, 1, R - 1 - pad);
  Tensor dx = torch::empty({g.N, g.K, g.P, g.Q}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  dca::conv_igemm_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), nullptr, g, stream());
  return dx;
}

// Weight gradient of y = conv2d(x, w, stride, pad) given dy; with `acc` (the parameter's
// persistent .grad view, fp32 or bf16, [K, C, R, S] channels_last) it is added in place and
// returned.
Tensor conv_igemm_wgrad(const Tensor& dy_in, const Tensor& x, const Tensor& w, int64_t stride,
                        int64_t pad, const OptT& acc) {
  const Tensor dy = dy_in.contiguous(at::MemoryFormat::ChannelsLast);
  const c10::DeviceGuard dg(dy.device());
  check_nhwc(x, "conv_igemm_wgrad");
  check_nhwc(dy, "conv_igemm_wgrad");
  const dca::ConvGeom g = geom(x, w, stride, pad);
  TORCH_CHECK(dy.size(0) == g.N && dy.size(1) == g.K && dy.size(2) == g.P && dy.size(3) == g.Q,
              "conv_igemm_wgrad: dy shape does not match the convolution output");
  TORCH_CHECK(g.M < (1 << 24), "conv_igemm_wgrad: at most 2^24 output pixels");
  Tensor ws = torch::empty({dca::conv_igemm_wgrad_ws_floats(g)}, dy.options().dtype(at::kFloat));
  Tensor out;
  bool accumulate = false, kcrs = false;
  if (acc.has_value() && acc->defined()) {
    out = *acc;
    kcrs = out.is_contiguous() && !out.is_contiguous(at::MemoryFormat::ChannelsLast);
    TORCH_CHECK(out.device() == dy.device() && out.sizes() == w.sizes() &&
                    (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16) &&
                    (kcrs || out.is_contiguous(at::MemoryFormat::ChannelsLast)),
                "conv_igemm_wgrad: accumulation target must be a dense fp32/bf16 tensor shaped like w");
    accumulate = true;
  } else {
    out = torch::empty(w.sizes(), w.options().memory_format(at::MemoryFormat::ChannelsLast));
  }
  dca::conv_igemm_wgrad(dy.data_ptr(), x.data_ptr(), ws.data_ptr<float>(), out.data_ptr(),
                        out.scalar_type() == at::kFloat, accumulate, kcrs, g, stream());
  return out;
}

}  // namespace

// dx (channels_last [N, C, H, W]) += small (channels_last [N, C, Ho, Wo]) at the stride-s
// positions, in place.
void strided_accumulate(Tensor& dx, const Tensor& small, int64_t s) {
  const c10::DeviceGuard dg(dx.device());
  TORCH_CHECK(dx.is_cuda() && dx.scalar_type() == at::kBFloat16 && small.scalar_type() == at::kBFloat16 &&
                  dx.dim() == 4 && small.dim() == 4, "strided_accumulate: bf16 4-D GPU tensors");
  TORCH_CHECK(dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  small.is_contiguous(at::MemoryFormat::ChannelsLast), "strided_accumulate: channels_last");
  const int64_t N = dx.size(0), C = dx.size(1), H = dx.size(2), W = dx.size(3);
  const int64_t Ho = small.size(2), Wo = small.size(3);
  TORCH_CHECK(s >= 1 && small.size(0) == N && small.size(1) == C && C % 8 == 0 &&
                  (Ho - 1) * s < H && (Wo - 1) * s < W, "strided_accumulate: shape mismatch");
  TORCH_CHECK(N * H * W * C < (int64_t{1} << 40), "strided_accumulate: too large");
  dca::strided_accumulate(dx.data_ptr(), small.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                          static_cast<int>(W), static_cast<int>(C), static_cast<int>(Ho),
                          static_cast<int>(Wo), static_cast<int>(s), stream());
}

// [N, 3, H, W] channels_last bf16 image -> [N, 12, (H+6)/2, (W+6)/2] channels_last (ops/conv.py
// _s2d_input: the space-to-depth form of the 7x7/2 padding-3 stem convolution).
Tensor stem_s2d(const Tensor& x) {
  constexpr int64_t co = 12;
  const c10::DeviceGuard dg(x.device());
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3,
              "stem_s2d: bf16 [N, 3, H, W] GPU tensor required");
  TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "stem_s2d: channels_last layout required");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0, "stem_s2d: even H and W required");
  TORCH_CHECK(N * (H + 6) * (W + 6) * 4 < (int64_t{1} << 40), "stem_s2d: too large");
  Tensor xs = torch::empty({N, co, (H + 6) / 2, (W + 6) / 2},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  if (xs.numel() == 0) return xs;
  dca::stem_s2d(x.data_ptr(), xs.data_ptr(), static_cast<int>(N), static_cast<int>(H),
                static_cast<int>(W), stream());
  return xs;
}

void register_conv_ops(pybind11::module& m) {
  m.def("stem_s2d", &stem_s2d, pybind11::arg("x"));
  m.def("strided_accumulate", &strided_accumulate, pybind11::arg("dx"), pybind11::arg("small"),
        pybind11::arg("stride"));
  m.def("conv_igemm_wgrad", &conv_igemm_wgrad, pybind11::arg("dy"), pybind11::arg("x"),
        pybind11::arg("w"), pybind11::arg("stride"), pybind11::arg("pad"),
        pybind11::arg("acc") = pybind11::none());
  m.def("conv_igemm_fwd", &conv_igemm_fwd, pybind11::arg("x"), pybind11::arg("w"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("stats"));
  m.def("conv_igemm_dgrad", &conv_igemm_dgrad, pybind11::arg("dy"), pybind11::arg("w"),
        pybind11::arg("pad"));
}
