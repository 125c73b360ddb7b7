// Python bindings of the determined_clone_amd HIP kernels (`determined_clone_amd.ops._C`).
// Tensor checks live here; the .hip translation units only see raw pointers and a hipStream_t so
// they compile without the torch headers.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>

namespace dca {
enum class BnDtype : int { kF32 = 0, kBF16 = 1, kF16 = 2 };
enum class OptDtype : int { kF32 = 0, kBF16 = 1, kF16 = 2, kNone = 3 };

int64_t bn_workspace_floats(int64_t M, int C);
void bn_forward_train(BnDtype dt, const void* x, const void* res, void* y, int64_t M, int C,
                      const float* gamma, const float* beta, float* running_mean,
                      float* running_var, float momentum, float eps, bool relu, float* save_mean,
                      float* save_invstd, int64_t* num_batches, uint8_t* mask, float* workspace,
                      const float* given_partials, int given_blocks, hipStream_t st);
void bn_forward_affine(BnDtype dt, const void* x, const void* res, void* y, int64_t M, int C,
                       const float* scale, const float* shift, bool relu, hipStream_t st);
void bn_relu_pool_forward(BnDtype dt, const void* x, void* y, uint8_t* idx, int N, int H, int W,
                          int C, const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, float* save_mean,
                          float* save_invstd, int64_t* num_batches, float* workspace,
                          const float* affine_scale, const float* affine_shift, hipStream_t st,
                          const float* given_partials = nullptr, int given_blocks = 0);
void bn_relu_pool_backward(BnDtype dt, const void* dyp, const uint8_t* idx, const void* x, int N,
                           int H, int W, int C, const float* gamma, const float* save_mean,
                           const float* save_invstd, void* dx, float* dgamma, float* dbeta,
                           float* workspace, hipStream_t st);
void bn_backward_train(BnDtype dt, const void* dy, const void* dy2, const uint8_t* mask, const void* x,
                       int64_t M, int C, const float* gamma, const float* save_mean, const float* save_invstd,
                       bool relu, void* dx, void* dres, float* dgamma, float* dbeta,
                       bool accumulate_dw, float* workspace, hipStream_t st,
                       const float* given_partials, int given_blocks);

void bn_forward_train_dual(BnDtype dt, const void* x, const void* x2, void* y, int64_t M, int C,
                           const float* gamma, const float* beta, float* running_mean,
                           float* running_var, const float* gamma2, const float* beta2,
                           float* running_mean2, float* running_var2, float momentum, float eps,
                           bool relu, float* save_mean, float* save_invstd, float* save_mean2,
                           float* save_invstd2, int64_t* num_batches, int64_t* num_batches2,
                           uint8_t* mask, float* workspace, float* workspace2,
                           const float* given_partials, int given_blocks,
                           const float* given_partials2, int given_blocks2, hipStream_t st);
void bn_backward_train_dual(BnDtype dt, const void* dy, const void* dy2, const uint8_t* mask,
                            const void* x, const void* x2, int64_t M, int C, const float* gamma,
                            const float* save_mean, const float* save_invstd,
                            const float* gamma2, const float* save_mean2,
                            const float* save_invstd2, bool relu, void* dx, void* dx2,
                            float* dgamma, float* dbeta, float* dgamma2, float* dbeta2,
                            bool accumulate_dw, float* workspace, float* workspace2,
                            hipStream_t st);

void spatial_mean_backward(BnDtype dt, const void* g, void* dx, int N, int HW, int C,
                           hipStream_t st);

int sumsq_partial_blocks(int64_t n);
void sumsq_partial(OptDtype g, const void* grad, int64_t n, float* partial, int blocks,
                   hipStream_t st);
void norm_finalize(const float* partial, int nparts, const float* loss_scale, float extra_scale,
                   float max_norm, float* out, hipStream_t st);
void sgd_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* mom,
              int64_t n, float lr, float momentum, float dampening, float wd, bool nesterov,
              bool first_step, float gscale, const float* dev_scale, const float* dyn, hipStream_t st);
void adam_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* m,
               float* v, int64_t n, float lr, float beta1, float beta2, float eps, float wd,
               bool adamw, float bc1, float bc2, float gscale, const float* dev_scale, const float* dyn,
               hipStream_t st);
void lamb_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* m,
               float* v, float* ubuf, const int64_t* cstart, const int* clen, const int* cseg,
               int nchunks, const int* seg_chunk_begin, int nseg, float* part_w, float* part_u,
               float* ratio, float lr, float beta1, float beta2, float eps, float wd, float bc1,
               float bc2, float gscale, const float* dev_scale, hipStream_t st);
void scaler_update(float* state, const float* dev_scale, float growth, float backoff, int interval,
                   hipStream_t st);
void scale_inplace(OptDtype dt, void* x, int64_t n, float s, const float* dev_scale,
                   hipStream_t st);
}  // namespace dca

namespace {

using torch::Tensor;
using OptT = c10::optional<Tensor>;

// PyTorch-ROCm exposes GPUs as device type "cuda"; its HIP stream/guard wrappers masquerade.
hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")

dca::BnDtype bn_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return dca::BnDtype::kBF16;
    case at::kHalf: return dca::BnDtype::kF16;
    case at::kFloat: return dca::BnDtype::kF32;
    default: TORCH_CHECK(false, "batchnorm: unsupported dtype ", t.scalar_type());
  }
}

dca::OptDtype opt_dtype(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return dca::OptDtype::kBF16;
    case at::kHalf: return dca::OptDtype::kF16;
    case at::kFloat: return dca::OptDtype::kF32;
    default: TORCH_CHECK(false, "optimizer: unsupported dtype ", t.scalar_type());
  }
}

template <typename T>
T* ptr_or_null(const OptT& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}
const void* vptr_or_null(const OptT& t) {
  return t.has_value() && t->defined() ? t->data_ptr() : nullptr;
}

// Rows x channels view of an NHWC (channels_last) 4-D tensor or a contiguous [.., C] tensor.
std::pair<int64_t, int> rows_channels(const Tensor& x) {
  int C = x.dim() >= 2 ? static_cast<int>(x.size(1)) : static_cast<int>(x.size(0));
  if (x.dim() == 4) {
    TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "batchnorm: 4-D input must be channels_last contiguous");
  } else {
    TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "batchnorm: input must be NHWC 4-D or [N, C]");
  }
  TORCH_CHECK(C % 8 == 0, "batchnorm: channels must be a multiple of 8, got ", C);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(M * C / 8 < (int64_t(1) << 31), "batchnorm: tensor too large for one launch");
  return {M, C};
}

static void check_partials(const OptT& p, int64_t C, const Tensor& x) {
  if (p.has_value() && p->defined())
    TORCH_CHECK(p->scalar_type() == at::kFloat && p->is_contiguous() && p->dim() == 3 &&
                    p->size(1) == 2 && p->size(2) == C && p->device() == x.device(),
                "batchnorm: partial statistics must be contiguous fp32 [blocks, 2, C]");
}

static bool has(const OptT& t) { return t.has_value() && t->defined(); }

std::vector<Tensor> bn_fwd_train(const Tensor& x, const OptT& residual, const OptT& weight,
                                 const OptT& bias, const OptT& running_mean,
                                 const OptT& running_var, const OptT& num_batches, double momentum,
                                 double eps, bool relu, const OptT& partials) {
  CHECK_DEV(x);
  const c10::DeviceGuard guard(x.device());
  auto [M, C] = rows_channels(x);
  if (residual.has_value()) {
    // same element order as x (NHWC / row-major contiguity), not identical strides: size-1 dims
    // (e.g. 1x1 spatial maps) may carry any stride in a channels_last-contiguous tensor
    const bool same_layout = x.dim() == 4
                                 ? residual->is_contiguous(at::MemoryFormat::ChannelsLast)
                                 : residual->is_contiguous();
    TORCH_CHECK(residual->sizes() == x.sizes() && same_layout &&
                    residual->scalar_type() == x.scalar_type(),
                "batchnorm: residual must match input shape/layout/dtype");
  }
  auto fopt = x.options().dtype(at::kFloat);
  Tensor y = torch::empty_like(x);
  Tensor save_mean = torch::empty({C}, fopt), save_invstd = torch::empty({C}, fopt);
  const bool given = partials.has_value() && partials->defined();
  if (given) {
    TORCH_CHECK(partials->scalar_type() == at::kFloat && partials->is_contiguous() &&
                    partials->dim() == 3 && partials->size(1) == 2 && partials->size(2) == C &&
                    partials->device() == x.device(),
                "batchnorm: partial statistics must be contiguous fp32 [blocks, 2, C]");
  }
  Tensor ws = torch::empty({given ? 2 * C : dca::bn_workspace_floats(M, C)}, fopt);
  Tensor mask = relu ? torch::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  dca::bn_forward_train(bn_dtype(x), x.data_ptr(), vptr_or_null(residual), y.data_ptr(), M, C,
                        ptr_or_null<float>(weight), ptr_or_null<float>(bias),
                        ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var),
                        static_cast<float>(momentum), static_cast<float>(eps), relu,
                        save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                        ptr_or_null<int64_t>(num_batches),
                        relu ? mask.data_ptr<uint8_t>() : nullptr, ws.data_ptr<float>(),
                        given ? partials->data_ptr<float>() : nullptr,
                        given ? static_cast<int>(partials->size(0)) : 0, cur_stream());
  return {y, save_mean, save_invstd, mask};
}

Tensor bn_fwd_affine(const Tensor& x, const OptT& residual, const Tensor& scale,
                     const Tensor& shift, bool relu) {
  CHECK_DEV(x);
  CHECK_F32(scale);
  CHECK_F32(shift);
  const c10::DeviceGuard guard(x.device());
  auto [M, C] = rows_channels(x);
  Tensor sc = scale.contiguous(), sh = shift.contiguous();
  Tensor y = torch::empty_like(x);
  dca::bn_forward_affine(bn_dtype(x), x.data_ptr(), vptr_or_null(residual), y.data_ptr(), M, C,
                         sc.data_ptr<float>(), sh.data_ptr<float>(), relu, cur_stream());
  return y;
}

std::vector<Tensor> bn_bwd_train(const Tensor& dy_in, const Tensor& x, const OptT& mask,
                                 const OptT& weight, const Tensor& save_mean,
                                 const Tensor& save_invstd, bool relu, bool need_dres,
                                 bool need_dweight, const OptT& dy2_in, const OptT& dweight_acc,
                                 const OptT& dbias_acc, const OptT& partials) {
  CHECK_DEV(x);
  const c10::DeviceGuard guard(x.device());
  auto [M, C] = rows_channels(x);
  Tensor dy = dy_in.dim() == 4 ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "batchnorm bwd: grad dtype mismatch");
  // optional second upstream gradient (the residual branch of the consumer), summed in-kernel
  Tensor dy2;
  if (dy2_in.has_value() && dy2_in->defined()) {
    dy2 = dy2_in->dim() == 4 ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast) : dy2_in->contiguous();
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == x.scalar_type(), "batchnorm bwd: dy2 mismatch");
  }
  TORCH_CHECK(!relu || (mask.has_value() && mask->defined() && mask->numel() == M * C / 8),
              "batchnorm bwd: relu needs the forward's ReLU bitmask");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dx = torch::empty_like(x);
  Tensor dres = need_dres ? torch::empty_like(x) : Tensor();
  // dweight_acc / dbias_acc: accumulate the parameter gradients in place (into .grad) instead
  // of returning fresh tensors.
  const bool acc = need_dweight && dweight_acc.has_value() && dweight_acc->defined() &&
                   dbias_acc.has_value() && dbias_acc->defined();
  if (acc) {
    for (const Tensor* t : {&*dweight_acc, &*dbias_acc})
      TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == C &&
                  t->device() == x.device(), "batchnorm bwd: accumulation target must be fp32 [C]");
  }
  Tensor dgamma = acc ? *dweight_acc : need_dweight ? torch::empty({C}, fopt) : Tensor();
  Tensor dbeta = acc ? *dbias_acc : need_dweight ? torch::empty({C}, fopt) : Tensor();
  // partials: the statistics pass already done by the producer of dy (a data-gradient epilogue)
  const bool given = has(partials);
  check_partials(partials, C, x);
  TORCH_CHECK(!given || !dy2.defined(), "batchnorm bwd: given partials exclude a second gradient");
  Tensor ws = torch::empty({dca::bn_workspace_floats(M, C)}, fopt);
  dca::bn_backward_train(bn_dtype(x), dy.data_ptr(), dy2.defined() ? dy2.data_ptr() : nullptr,
                         relu ? mask->data_ptr<uint8_t>() : nullptr, x.data_ptr(),
                         M, C, ptr_or_null<float>(weight), save_mean.data_ptr<float>(),
                         save_invstd.data_ptr<float>(), relu, dx.data_ptr(),
                         need_dres ? dres.data_ptr() : nullptr,
                         need_dweight ? dgamma.data_ptr<float>() : nullptr,
                         need_dweight ? dbeta.data_ptr<float>() : nullptr, acc,
                         ws.data_ptr<float>(), cur_stream(),
                         given ? partials->data_ptr<float>() : nullptr,
                         given ? static_cast<int>(partials->size(0)) : 0);
  if (acc) return {dx, Tensor(), Tensor(), dres};
  return {dx, dgamma, dbeta, dres};
}

// act(bn(x) + bn2(x2)) training forward (downsampling block: main branch + projection shortcut).
// Returns (y, mean, invstd, mask, mean2, invstd2).
std::vector<Tensor> bn_fwd_train_dual(const Tensor& x, const OptT& weight, const OptT& bias,
                                      const OptT& running_mean, const OptT& running_var,
                                      const OptT& num_batches, const Tensor& x2,
                                      const OptT& weight2, const OptT& bias2,
                                      const OptT& running_mean2, const OptT& running_var2,
                                      const OptT& num_batches2, double momentum, double eps,
                                      bool relu, const OptT& partials, const OptT& partials2) {
  CHECK_DEV(x);
  CHECK_DEV(x2);
  const c10::DeviceGuard guard(x.device());
  auto [M, C] = rows_channels(x);
  const bool same_layout = x.dim() == 4 ? x2.is_contiguous(at::MemoryFormat::ChannelsLast) : x2.is_contiguous();
  TORCH_CHECK(x2.sizes() == x.sizes() && same_layout && x2.scalar_type() == x.scalar_type(),
              "batchnorm dual: second input must match the first's shape/layout/dtype");
  check_partials(partials, C, x);
  check_partials(partials2, C, x);
  auto fopt = x.options().dtype(at::kFloat);
  Tensor y = torch::empty_like(x);
  Tensor m1 = torch::empty({C}, fopt), i1 = torch::empty({C}, fopt);
  Tensor m2 = torch::empty({C}, fopt), i2 = torch::empty({C}, fopt);
  Tensor ws = torch::empty({has(partials) ? 2 * C : dca::bn_workspace_floats(M, C)}, fopt);
  Tensor ws2 = torch::empty({has(partials2) ? 2 * C : dca::bn_workspace_floats(M, C)}, fopt);
  Tensor mask = relu ? torch::empty({M * C / 8}, x.options().dtype(at::kByte)) : Tensor();
  dca::bn_forward_train_dual(
      bn_dtype(x), x.data_ptr(), x2.data_ptr(), y.data_ptr(), M, C, ptr_or_null<float>(weight),
      ptr_or_null<float>(bias), ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var),
      ptr_or_null<float>(weight2), ptr_or_null<float>(bias2), ptr_or_null<float>(running_mean2),
      ptr_or_null<float>(running_var2), static_cast<float>(momentum), static_cast<float>(eps), relu,
      m1.data_ptr<float>(), i1.data_ptr<float>(), m2.data_ptr<float>(), i2.data_ptr<float>(),
      ptr_or_null<int64_t>(num_batches), ptr_or_null<int64_t>(num_batches2),
      relu ? mask.data_ptr<uint8_t>() : nullptr, ws.data_ptr<float>(), ws2.data_ptr<float>(),
      has(partials) ? partials->data_ptr<float>() : nullptr,
      has(partials) ? static_cast<int>(partials->size(0)) : 0,
      has(partials2) ? partials2->data_ptr<float>() : nullptr,
      has(partials2) ? static_cast<int>(partials2->size(0)) : 0, cur_stream());
  return {y, m1, i1, mask, m2, i2};
}

// Backward of bn_fwd_train_dual. Returns (dx, dx2, dgamma, dbeta, dgamma2, dbeta2); the four
// parameter gradients are accumulated into the given .grad targets instead when all four are
// passed (then returned undefined).
std::vector<Tensor> bn_bwd_train_dual(const Tensor& dy_in, const Tensor& x, const OptT& mask,
                                      const OptT& weight, const Tensor& mean, const Tensor& invstd,
                                      const Tensor& x2, const OptT& weight2, const Tensor& mean2,
                                      const Tensor& invstd2, bool relu, bool need_dweight,
                                      const OptT& dy2_in, const std::vector<Tensor>& acc) {
  CHECK_DEV(x);
  const c10::DeviceGuard guard(x.device());
  auto [M, C] = rows_channels(x);
  Tensor dy = dy_in.dim() == 4 ? dy_in.contiguous(at::MemoryFormat::ChannelsLast) : dy_in.contiguous();
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && x2.sizes() == x.sizes() &&
                  x2.scalar_type() == x.scalar_type(), "batchnorm dual bwd: shape/dtype mismatch");
  Tensor dy2;
  if (has(dy2_in)) {
    dy2 = dy2_in->dim() == 4 ? dy2_in->contiguous(at::MemoryFormat::ChannelsLast) : dy2_in->contiguous();
    TORCH_CHECK(dy2.sizes() == x.sizes() && dy2.scalar_type() == x.scalar_type(), "batchnorm dual bwd: dy2 mismatch");
  }
  TORCH_CHECK(!relu || (has(mask) && mask->numel() == M * C / 8),
              "batchnorm dual bwd: relu needs the forward's ReLU bitmask");
  const bool accumulate = need_dweight && acc.size() == 4;
  if (accumulate)
    for (const Tensor& t : acc)
      TORCH_CHECK(t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == C &&
                  t.device() == x.device(), "batchnorm dual bwd: accumulation target must be fp32 [C]");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dx = torch::empty_like(x), dx2 = torch::empty_like(x);
  std::vector<Tensor> dw(4);
  for (int i = 0; i < 4; ++i)
    dw[i] = accumulate ? acc[i] : need_dweight ? torch::empty({C}, fopt) : Tensor();
  Tensor ws = torch::empty({dca::bn_workspace_floats(M, C)}, fopt);
  Tensor ws2 = torch::empty({dca::bn_workspace_floats(M, C)}, fopt);
  auto p = [&](int i) { return need_dweight ? dw[i].data_ptr<float>() : nullptr; };
  dca::bn_backward_train_dual(bn_dtype(x), dy.data_ptr(), dy2.defined() ? dy2.data_ptr() : nullptr,
                              relu ? mask->data_ptr<uint8_t>() : nullptr, x.data_ptr(), x2.data_ptr(),
                              M, C, ptr_or_null<float>(weight), mean.data_ptr<float>(),
                              invstd.data_ptr<float>(), ptr_or_null<float>(weight2),
                              mean2.data_ptr<float>(), invstd2.data_ptr<float>(), relu,
                              dx.data_ptr(), dx2.data_ptr(), p(0), p(1), p(2), p(3), accumulate,
                              ws.data_ptr<float>(), ws2.data_ptr<float>(), cur_stream());
  if (accumulate) return {dx, dx2, Tensor(), Tensor(), Tensor(), Tensor()};
  return {dx, dx2, dw[0], dw[1], dw[2], dw[3]};
}

// Stem fusion: act(bn(x)) -> max_pool2d(3, 2, 1) without materialising the pre-pool tensor.
// x: NHWC (channels_last) [N, C, H, W]. Returns (y_pool, save_mean, save_invstd, idx).
std::vector<Tensor> bn_pool_fwd_train(const Tensor& x, const OptT& weight, const OptT& bias,
                                      const OptT& running_mean, const OptT& running_var,
                                      const OptT& num_batches, double momentum, double eps,
                                      const OptT& partials) {
  CHECK_DEV(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "bn_pool: channels_last [N, C%8==0, H, W] input required");
  const c10::DeviceGuard guard(x.device());
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto fopt = x.options().dtype(at::kFloat);
  Tensor y = torch::empty({N, C, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  Tensor idx = torch::empty({static_cast<int64_t>(N) * Ho * Wo * C}, x.options().dtype(at::kByte));
  Tensor save_mean = torch::empty({C}, fopt), save_invstd = torch::empty({C}, fopt);
  Tensor ws = torch::empty({dca::bn_workspace_floats(static_cast<int64_t>(N) * H * W, C)}, fopt);
  // partials: (sum, sum^2) per block already reduced by x's producer (the stem conv epilogue)
  const bool given = partials.has_value() && partials->defined();
  check_partials(partials, C, x);
  dca::bn_relu_pool_forward(bn_dtype(x), x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), N, H, W, C,
                            ptr_or_null<float>(weight), ptr_or_null<float>(bias),
                            ptr_or_null<float>(running_mean), ptr_or_null<float>(running_var),
                            static_cast<float>(momentum), static_cast<float>(eps),
                            save_mean.data_ptr<float>(), save_invstd.data_ptr<float>(),
                            ptr_or_null<int64_t>(num_batches), ws.data_ptr<float>(), nullptr, nullptr,
                            cur_stream(), given ? partials->data_ptr<float>() : nullptr,
                            given ? static_cast<int>(partials->size(0)) : 0);
  return {y, save_mean, save_invstd, idx};
}

Tensor bn_pool_fwd_affine(const Tensor& x, const Tensor& scale, const Tensor& shift) {
  CHECK_DEV(x);
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0,
              "bn_pool: channels_last [N, C%8==0, H, W] input required");
  const c10::DeviceGuard guard(x.device());
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  Tensor sc = scale.contiguous(), sh = shift.contiguous();
  Tensor y = torch::empty({N, C, (H - 1) / 2 + 1, (W - 1) / 2 + 1},
                          x.options().memory_format(at::MemoryFormat::ChannelsLast));
  dca::bn_relu_pool_forward(bn_dtype(x), x.data_ptr(), y.data_ptr(), nullptr, N, H, W, C, nullptr,
                            nullptr, nullptr, nullptr, 0.f, 0.f, nullptr, nullptr, nullptr, nullptr,
                            sc.data_ptr<float>(), sh.data_ptr<float>(), cur_stream());
  return y;
}

std::vector<Tensor> bn_pool_bwd(const Tensor& dyp_in, const Tensor& x, const Tensor& idx,
                                const OptT& weight, const Tensor& save_mean,
                                const Tensor& save_invstd, bool need_dweight) {
  const c10::DeviceGuard guard(x.device());
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  Tensor dyp = dyp_in.contiguous(at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(dyp.scalar_type() == x.scalar_type(), "bn_pool bwd: grad dtype mismatch");
  auto fopt = x.options().dtype(at::kFloat);
  Tensor dx = torch::empty_like(x);
  Tensor dgamma = need_dweight ? torch::empty({C}, fopt) : Tensor();
  Tensor dbeta = need_dweight ? torch::empty({C}, fopt) : Tensor();
  Tensor ws = torch::empty({dca::bn_workspace_floats(static_cast<int64_t>(N) * H * W, C)}, fopt);
  dca::bn_relu_pool_backward(bn_dtype(x), dyp.data_ptr(), idx.data_ptr<uint8_t>(), x.data_ptr(), N, H, W,
                             C, ptr_or_null<float>(weight), save_mean.data_ptr<float>(),
                             save_invstd.data_ptr<float>(), dx.data_ptr(),
                             need_dweight ? dgamma.data_ptr<float>() : nullptr,
                             need_dweight ? dbeta.data_ptr<float>() : nullptr, ws.data_ptr<float>(),
                             cur_stream());
  return {dx, dgamma, dbeta};
}

// Backward of the global average pool of an NHWC tensor: g [N, C] -> dx [N, C, H, W]
// (channels_last), every spatial position g / (H*W).
Tensor spatial_mean_bwd(const Tensor& g_in, int64_t H, int64_t W) {
  CHECK_DEV(g_in);
  const c10::DeviceGuard guard(g_in.device());
  Tensor g = g_in.contiguous();
  TORCH_CHECK(g.dim() == 2 && g.size(1) % 8 == 0, "spatial_mean_bwd: grad must be [N, C], C % 8 == 0");
  const int64_t N = g.size(0), C = g.size(1);
  TORCH_CHECK(N * H * W * C / 8 < (int64_t(1) << 31), "spatial_mean_bwd: tensor too large");
  Tensor dx = torch::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  dca::spatial_mean_backward(bn_dtype(g), g.data_ptr(), dx.data_ptr(), static_cast<int>(N),
                             static_cast<int>(H * W), static_cast<int>(C), cur_stream());
  return dx;
}

// Global gradient norm over one flat buffer: returns a 3-float device tensor
// [grad multiplier, found_inf, norm] (see optim.hip norm_finalize_kernel).
Tensor grad_norm_scale(const std::vector<Tensor>& grads, const OptT& loss_scale, double extra_scale,
                       double max_norm) {
  TORCH_CHECK(!grads.empty(), "grad_norm_scale: no gradients");
  const c10::DeviceGuard guard(grads[0].device());
  auto fopt = grads[0].options().dtype(at::kFloat);
  std::vector<int> blocks;
  int total = 0;
  for (auto& g : grads) {
    CHECK_DEV(g);
    TORCH_CHECK(g.is_contiguous(), "grad_norm_scale: flat gradient buffers must be contiguous");
    blocks.push_back(dca::sumsq_partial_blocks(g.numel()));
    total += blocks.back();
  }
  Tensor partial = torch::empty({total}, fopt);
  Tensor out = torch::empty({3}, fopt);
  int off = 0;
  for (size_t i = 0; i < grads.size(); ++i) {
    dca::sumsq_partial(opt_dtype(grads[i]), grads[i].data_ptr(), grads[i].numel(),
                       partial.data_ptr<float>() + off, blocks[i], cur_stream());
    off += blocks[i];
  }
  dca::norm_finalize(partial.data_ptr<float>(), total, ptr_or_null<float>(loss_scale),
                     static_cast<float>(extra_scale), static_cast<float>(max_norm),
                     out.data_ptr<float>(), cur_stream());
  return out;
}

// ZeRO path: per-rank sum-of-squares partials over the owned gradient shard (the caller sums them,
// all-reduces the scalar and then calls norm_finalize on it).
Tensor sumsq_partials(const std::vector<Tensor>& grads) {
  TORCH_CHECK(!grads.empty(), "sumsq_partials: no gradients");
  const c10::DeviceGuard guard(grads[0].device());
  std::vector<int> blocks;
  int total = 0;
  for (auto& g : grads) {
    CHECK_DEV(g);
    TORCH_CHECK(g.is_contiguous(), "sumsq_partials: contiguous gradient slices required");
    blocks.push_back(dca::sumsq_partial_blocks(g.numel()));
    total += blocks.back();
  }
  Tensor partial = torch::empty({total}, grads[0].options().dtype(at::kFloat));
  int off = 0;
  for (size_t i = 0; i < grads.size(); ++i) {
    dca::sumsq_partial(opt_dtype(grads[i]), grads[i].data_ptr(), grads[i].numel(),
                       partial.data_ptr<float>() + off, blocks[i], cur_stream());
    off += blocks[i];
  }
  return partial;
}

Tensor norm_finalize_t(const Tensor& partial, const OptT& loss_scale, double extra_scale,
                       double max_norm) {
  CHECK_DEV(partial);
  CHECK_F32(partial);
  TORCH_CHECK(partial.is_contiguous(), "norm_finalize: contiguous partials required");
  const c10::DeviceGuard guard(partial.device());
  Tensor out = torch::empty({3}, partial.options());
  dca::norm_finalize(partial.data_ptr<float>(), static_cast<int>(partial.numel()),
                     ptr_or_null<float>(loss_scale), static_cast<float>(extra_scale),
                     static_cast<float>(max_norm), out.data_ptr<float>(), cur_stream());
  return out;
}

void check_flat(const Tensor& master, const Tensor& grad, const OptT& model) {
  CHECK_DEV(master);
  CHECK_F32(master);
  TORCH_CHECK(master.is_contiguous() && grad.is_contiguous(), "flat buffers must be contiguous");
  TORCH_CHECK(grad.numel() == master.numel(), "grad/master size mismatch");
  if (model.has_value() && model->defined())
    TORCH_CHECK(model->numel() == master.numel() && model->is_contiguous(), "model buffer mismatch");
}

// Optional device-resident step hyper-parameters read by the optimizer kernels instead of their
// scalar arguments (a HIP graph replays the launch with the values current at replay time).
void check_dyn(const OptT& dyn, int64_t n) {
  if (dyn.has_value() && dyn->defined())
    TORCH_CHECK(dyn->is_cuda() && dyn->scalar_type() == at::kFloat && dyn->is_contiguous() &&
                    dyn->numel() >= n,
                "optimizer hyper-parameter buffer must be a contiguous fp32 GPU tensor of >= ", n);
}

void sgd(const Tensor& master, const OptT& model, const Tensor& grad, const OptT& mom, double lr,
         double momentum, double dampening, double wd, bool nesterov, bool first_step,
         double gscale, const OptT& dev_scale, const OptT& dyn) {
  check_flat(master, grad, model);
  const c10::DeviceGuard guard(master.device());
  check_dyn(dyn, 2);
  TORCH_CHECK(momentum == 0.0 || (mom.has_value() && mom->numel() == master.numel()),
              "sgd: momentum buffer required");
  dca::sgd_step(opt_dtype(grad),
                model.has_value() && model->defined() ? opt_dtype(*model) : dca::OptDtype::kNone,
                master.data_ptr<float>(), model.has_value() && model->defined() ? model->data_ptr() : nullptr,
                grad.data_ptr(), ptr_or_null<float>(mom), master.numel(), static_cast<float>(lr),
                static_cast<float>(momentum), static_cast<float>(dampening), static_cast<float>(wd),
                nesterov, first_step, static_cast<float>(gscale), ptr_or_null<float>(dev_scale),
                ptr_or_null<float>(dyn), cur_stream());
}

void adam(const Tensor& master, const OptT& model, const Tensor& grad, const Tensor& m,
          const Tensor& v, double lr, double beta1, double beta2, double eps, double wd, bool adamw,
          int64_t step, double gscale, const OptT& dev_scale, const OptT& dyn) {
  check_flat(master, grad, model);
  const c10::DeviceGuard guard(master.device());
  check_dyn(dyn, 3);
  const double bc1 = 1.0 - std::pow(beta1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(beta2, static_cast<double>(step));
  dca::adam_step(opt_dtype(grad),
                 model.has_value() && model->defined() ? opt_dtype(*model) : dca::OptDtype::kNone,
                 master.data_ptr<float>(), model.has_value() && model->defined() ? model->data_ptr() : nullptr,
                 grad.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(), master.numel(),
                 static_cast<float>(lr), static_cast<float>(beta1), static_cast<float>(beta2),
                 static_cast<float>(eps), static_cast<float>(wd), adamw, static_cast<float>(bc1),
                 static_cast<float>(bc2), static_cast<float>(gscale), ptr_or_null<float>(dev_scale),
                 ptr_or_null<float>(dyn), cur_stream());
}

// chunks: int64 [3][nchunks] = (start, len, seg) on device; seg_begin: int32 [nseg+1] on device.
void lamb(const Tensor& master, const OptT& model, const Tensor& grad, const Tensor& m,
          const Tensor& v, const Tensor& ubuf, const Tensor& cstart, const Tensor& clen,
          const Tensor& cseg, const Tensor& seg_begin, double lr, double beta1, double beta2,
          double eps, double wd, int64_t step, double gscale, const OptT& dev_scale) {
  check_flat(master, grad, model);
  const c10::DeviceGuard guard(master.device());
  const int nchunks = static_cast<int>(cstart.numel());
  const int nseg = static_cast<int>(seg_begin.numel()) - 1;
  auto fopt = master.options();
  Tensor pw = torch::empty({nchunks}, fopt), pu = torch::empty({nchunks}, fopt);
  Tensor ratio = torch::empty({nseg}, fopt);
  const double bc1 = 1.0 - std::pow(beta1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(beta2, static_cast<double>(step));
  dca::lamb_step(opt_dtype(grad),
                 model.has_value() && model->defined() ? opt_dtype(*model) : dca::OptDtype::kNone,
                 master.data_ptr<float>(), model.has_value() && model->defined() ? model->data_ptr() : nullptr,
                 grad.data_ptr(), m.data_ptr<float>(), v.data_ptr<float>(), ubuf.data_ptr<float>(),
                 cstart.data_ptr<int64_t>(), clen.data_ptr<int>(), cseg.data_ptr<int>(), nchunks,
                 seg_begin.data_ptr<int>(), nseg, pw.data_ptr<float>(), pu.data_ptr<float>(),
                 ratio.data_ptr<float>(), static_cast<float>(lr), static_cast<float>(beta1),
                 static_cast<float>(beta2), static_cast<float>(eps), static_cast<float>(wd),
                 static_cast<float>(bc1), static_cast<float>(bc2), static_cast<float>(gscale),
                 ptr_or_null<float>(dev_scale), cur_stream());
}

void amp_scaler_update(const Tensor& state, const Tensor& dev_scale, double growth, double backoff,
                       int64_t interval) {
  CHECK_DEV(state);
  const c10::DeviceGuard guard(state.device());
  dca::scaler_update(state.data_ptr<float>(), dev_scale.data_ptr<float>(),
                     static_cast<float>(growth), static_cast<float>(backoff),
                     static_cast<int>(interval), cur_stream());
}

void scale_(const Tensor& x, double s, const OptT& dev_scale) {
  CHECK_DEV(x);
  TORCH_CHECK(x.is_contiguous(), "scale_: contiguous buffer required");
  const c10::DeviceGuard guard(x.device());
  dca::scale_inplace(opt_dtype(x), x.data_ptr(), x.numel(), static_cast<float>(s),
                     ptr_or_null<float>(dev_scale), cur_stream());
}

}  // namespace

// Extra kernel families register themselves from their own translation units.
void register_transformer_ops(pybind11::module& m);
void register_conv_ops(pybind11::module& m);
void register_groupnorm_ops(pybind11::module& m);
void register_lt_ops(pybind11::module& m);

extern "C" const char dca_source_hash[];  // ops/build.py: sha256 of the csrc/ tree

PYBIND11_MODULE(_C, m) {
  m.doc() = "determined_clone_amd MI355X (gfx950) HIP kernels";
  m.attr("source_hash") = pybind11::str(static_cast<const char*>(dca_source_hash));
  m.def("bn_fwd_train", &bn_fwd_train, pybind11::arg("x"), pybind11::arg("residual"),
        pybind11::arg("weight"), pybind11::arg("bias"), pybind11::arg("running_mean"),
        pybind11::arg("running_var"), pybind11::arg("num_batches"), pybind11::arg("momentum"),
        pybind11::arg("eps"), pybind11::arg("relu"), pybind11::arg("partials") = pybind11::none());
  m.def("bn_fwd_affine", &bn_fwd_affine);
  m.def("bn_fwd_train_dual", &bn_fwd_train_dual);
  m.def("bn_bwd_train_dual", &bn_bwd_train_dual);
  m.def("bn_bwd_train", &bn_bwd_train, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("mask"),
        pybind11::arg("weight"), pybind11::arg("save_mean"), pybind11::arg("save_invstd"),
        pybind11::arg("relu"), pybind11::arg("need_dres"), pybind11::arg("need_dweight"),
        pybind11::arg("dy2") = pybind11::none(), pybind11::arg("dweight_acc") = pybind11::none(),
        pybind11::arg("dbias_acc") = pybind11::none(), pybind11::arg("partials") = pybind11::none());
  m.def("bn_pool_fwd_train", &bn_pool_fwd_train, pybind11::arg("x"), pybind11::arg("weight"),
        pybind11::arg("bias"), pybind11::arg("running_mean"), pybind11::arg("running_var"),
        pybind11::arg("num_batches"), pybind11::arg("momentum"), pybind11::arg("eps"),
        pybind11::arg("partials") = pybind11::none());
  m.def("bn_pool_fwd_affine", &bn_pool_fwd_affine);
  m.def("bn_pool_bwd", &bn_pool_bwd);
  m.def("spatial_mean_bwd", &spatial_mean_bwd);
  m.def("grad_norm_scale", &grad_norm_scale);
  m.def("sumsq_partials", &sumsq_partials);
  m.def("norm_finalize", &norm_finalize_t);
  m.def("sgd", &sgd, pybind11::arg("master"), pybind11::arg("model"), pybind11::arg("grad"),
        pybind11::arg("mom"), pybind11::arg("lr"), pybind11::arg("momentum"),
        pybind11::arg("dampening"), pybind11::arg("wd"), pybind11::arg("nesterov"),
        pybind11::arg("first_step"), pybind11::arg("gscale"), pybind11::arg("dev_scale"),
        pybind11::arg("dyn") = pybind11::none());
  m.def("adam", &adam, pybind11::arg("master"), pybind11::arg("model"), pybind11::arg("grad"),
        pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("lr"), pybind11::arg("beta1"),
        pybind11::arg("beta2"), pybind11::arg("eps"), pybind11::arg("wd"), pybind11::arg("adamw"),
        pybind11::arg("step"), pybind11::arg("gscale"), pybind11::arg("dev_scale"),
        pybind11::arg("dyn") = pybind11::none());
  m.def("lamb", &lamb);
  m.def("amp_scaler_update", &amp_scaler_update);
  m.def("scale_", &scale_);
  register_transformer_ops(m);
  register_conv_ops(m);
  register_groupnorm_ops(m);
  register_lt_ops(m);
}
