// Bindings for the transformer kernel family (transformer.hip, attention.hip).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <c10/core/DeviceGuard.h>

#include <hip/hip_runtime.h>

#include "transformer_api.h"


namespace {
using torch::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

dca::TDtype tdt(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kBFloat16: return dca::TDtype::kBF16;
    case at::kHalf: return dca::TDtype::kF16;
    case at::kFloat: return dca::TDtype::kF32;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
}
const void* vp(const OptT& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }
const float* fp(const OptT& t) {
  if (!(t.has_value() && t->defined())) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_contiguous(), "params must be contiguous fp32");
  return t->data_ptr<float>();
}

std::vector<Tensor> ln_fwd(const Tensor& x, const OptT& res, const OptT& gamma, const OptT& beta,
                           double eps, bool want_sum) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "ln_fwd: contiguous GPU input required");
  const c10::DeviceGuard g(x.device());
  const int D = static_cast<int>(x.size(-1));
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "ln_fwd: D must be a multiple of 8 and <= 8192");
  const int64_t rows = x.numel() / D;
  if (res.has_value()) TORCH_CHECK(res->sizes() == x.sizes() && res->is_contiguous(), "residual shape");
  Tensor y = torch::empty_like(x);
  Tensor sum = (res.has_value() && want_sum) ? torch::empty_like(x) : Tensor();
  auto fo = x.options().dtype(at::kFloat);
  Tensor mean = torch::empty({rows}, fo), rstd = torch::empty({rows}, fo);
  dca::layernorm_fwd(tdt(x), x.data_ptr(), vp(res), sum.defined() ? sum.data_ptr() : nullptr,
                     y.data_ptr(), fp(gamma), fp(beta), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), rows, D, static_cast<float>(eps), stream());
  return {y, sum, mean, rstd};
}

// Where a column reduction lands: accumulate into a parameter's .grad (fp32 or bf16, contiguous,
// `n` elements) or -- when `acc` is absent -- a fresh fp32 tensor returned to autograd.
bool want_acc(const OptT& acc) { return acc.has_value() && acc->defined(); }
void check_acc(const Tensor& t, int64_t n, const Tensor& like, const char* what) {
  TORCH_CHECK(t.is_contiguous() && t.numel() == n && t.device() == like.device() &&
                  (t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16),
              what, ": accumulation target must be a contiguous fp32/bf16 tensor of ", n, " elements");
}

std::vector<Tensor> ln_bwd(const Tensor& dy_in, const Tensor& x, const OptT& gamma,
                           const Tensor& mean, const Tensor& rstd, const OptT& dsum,
                           bool need_param_grads, const OptT& dgamma_acc, const OptT& dbeta_acc,
                           const OptT& colsum_acc) {
  const c10::DeviceGuard g(x.device());
  Tensor dy = dy_in.contiguous();
  const int D = static_cast<int>(x.size(-1));
  const int64_t rows = x.numel() / D;
  Tensor dx = torch::empty_like(x);
  auto fo = x.options().dtype(at::kFloat);
  // colsum_acc (+)= dx.sum(rows): the bias gradient of the linear layer that produced the
  // residual input, reduced in this pass (partial grows a third [D] row per block)
  const bool colsum = want_acc(colsum_acc);
  dca::ColumnOut cs;
  if (colsum) {
    check_acc(*colsum_acc, D, x, "ln_bwd colsum");
    cs = {colsum_acc->data_ptr(), nullptr, D, colsum_acc->scalar_type() == at::kBFloat16, true};
  }
  Tensor partial = torch::empty({dca::ln_bwd_partial_floats(rows, D, colsum)}, fo);
  const bool acc = need_param_grads && want_acc(dgamma_acc) && want_acc(dbeta_acc);
  Tensor dgb;
  dca::ColumnOut out;
  if (acc) {
    check_acc(*dgamma_acc, D, x, "ln_bwd");
    check_acc(*dbeta_acc, D, x, "ln_bwd");
    TORCH_CHECK(dgamma_acc->scalar_type() == dbeta_acc->scalar_type(), "ln_bwd: gamma/beta grad dtypes differ");
    out = {dgamma_acc->data_ptr(), dbeta_acc->data_ptr(), D,
           dgamma_acc->scalar_type() == at::kBFloat16, true};
  } else if (need_param_grads) {
    dgb = torch::empty({2, D}, fo);
    out = {dgb.data_ptr(), nullptr, 2 * static_cast<int64_t>(D), false, false};
  }
  Tensor ds = dsum.has_value() && dsum->defined() ? dsum->contiguous() : Tensor();
  dca::layernorm_bwd(tdt(x), dy.data_ptr(), x.data_ptr(), fp(gamma), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), ds.defined() ? ds.data_ptr() : nullptr, dx.data_ptr(),
                     partial.data_ptr<float>(), need_param_grads ? &out : nullptr, rows, D, stream(),
                     colsum ? &cs : nullptr);
  if (!need_param_grads || acc) return {dx, Tensor(), Tensor()};
  return {dx, dgb[0], dgb[1]};
}

// bias: fp32 or bf16 [N] (read directly -- no cast kernel for bf16 models).
std::pair<const void*, bool> bias_arg(const OptT& bias, int64_t N) {
  if (!bias.has_value() || !bias->defined()) return {nullptr, false};
  TORCH_CHECK(bias->is_contiguous() && bias->numel() == N &&
                  (bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16),
              "bias_gelu: bias must be a contiguous fp32/bf16 [N] tensor");
  return {bias->data_ptr(), bias->scalar_type() == at::kBFloat16};
}

Tensor bias_gelu(const Tensor& x, const OptT& bias) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "bias_gelu: contiguous GPU input required");
  const c10::DeviceGuard g(x.device());
  const int N = static_cast<int>(x.size(-1));
  TORCH_CHECK(N % 8 == 0, "bias_gelu: last dim must be a multiple of 8");
  Tensor y = torch::empty_like(x);
  auto [bp, bbf] = bias_arg(bias, N);
  dca::bias_gelu_fwd(tdt(x), x.data_ptr(), bp, bbf, y.data_ptr(), x.numel() / N, N, stream());
  return y;
}

std::vector<Tensor> bias_gelu_bwd(const Tensor& dy_in, const Tensor& x, const OptT& bias,
                                  bool need_db, const OptT& dbias_acc) {
  const c10::DeviceGuard g(x.device());
  Tensor dy = dy_in.contiguous();
  const int N = static_cast<int>(x.size(-1));
  const int64_t rows = x.numel() / N;
  Tensor dx = torch::empty_like(x);
  auto [bp, bbf] = bias_arg(bias, N);
  const bool want_db = need_db && bp != nullptr;
  const bool acc = want_db && want_acc(dbias_acc);
  auto fo = x.options().dtype(at::kFloat);
  Tensor partial = want_db ? torch::empty({static_cast<int64_t>(dca::bias_gelu_bwd_row_blocks(rows)) * N}, fo) : Tensor();
  Tensor db;
  dca::ColumnOut out;
  if (acc) {
    check_acc(*dbias_acc, N, x, "bias_gelu_bwd");
    out = {dbias_acc->data_ptr(), nullptr, N, dbias_acc->scalar_type() == at::kBFloat16, true};
  } else if (want_db) {
    db = torch::empty({N}, fo);
    out = {db.data_ptr(), nullptr, N, false, false};
  }
  dca::bias_gelu_bwd(tdt(x), dy.data_ptr(), x.data_ptr(), bp, bbf, dx.data_ptr(),
                     want_db ? partial.data_ptr<float>() : nullptr, want_db ? &out : nullptr, rows,
                     N, stream());
  return {dx, db};
}

// Bias gradient of a linear layer: sum of dy [.., N] over all leading dims. Accumulates into
// `acc` (the bias .grad) when given and returns an undefined tensor; else returns fp32 [N].
Tensor bias_grad(const Tensor& dy_in, const OptT& acc) {
  const c10::DeviceGuard g(dy_in.device());
  Tensor dy = dy_in.contiguous();
  const int N = static_cast<int>(dy.size(-1));
  TORCH_CHECK(N % 8 == 0, "bias_grad: last dim must be a multiple of 8");
  const int64_t rows = dy.numel() / N;
  auto fo = dy.options().dtype(at::kFloat);
  Tensor partial = torch::empty({static_cast<int64_t>(dca::row_sum_blocks(rows, N)) * N}, fo);
  Tensor db;
  dca::ColumnOut out;
  if (want_acc(acc)) {
    check_acc(*acc, N, dy, "bias_grad");
    out = {acc->data_ptr(), nullptr, N, acc->scalar_type() == at::kBFloat16, true};
  } else {
    db = torch::empty({N}, fo);
    out = {db.data_ptr(), nullptr, N, false, false};
  }
  dca::row_sum(tdt(dy), dy.data_ptr(), partial.data_ptr<float>(), out, rows, N, stream());
  return db;
}

// acc (+)= part.sum(0) for part fp32 [splits, *acc.shape]; acc bf16/fp32 contiguous.
void splitk_accumulate(const Tensor& part, Tensor& acc, bool accumulate) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous(),
              "splitk_accumulate: part must be a contiguous fp32 GPU tensor");
  TORCH_CHECK(acc.is_contiguous() && (acc.scalar_type() == at::kBFloat16 || acc.scalar_type() == at::kFloat),
              "splitk_accumulate: acc must be contiguous bf16/fp32");
  TORCH_CHECK(part.dim() >= 1 && part.numel() == part.size(0) * acc.numel(),
              "splitk_accumulate: part must be [splits, *acc.shape]");
  TORCH_CHECK(acc.numel() % 8 == 0, "splitk_accumulate: numel must be a multiple of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(acc.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(part.data_ptr()) % 16 == 0,
              "splitk_accumulate: 16-byte aligned buffers required");
  const c10::DeviceGuard g(acc.device());
  dca::splitk_accumulate(acc.scalar_type() == at::kBFloat16, part.data_ptr<float>(), acc.data_ptr(),
                         acc.numel(), static_cast<int>(part.size(0)), accumulate, stream());
}

Tensor rope_apply(const Tensor& x, const Tensor& cosT, const Tensor& sinT, int64_t H, int64_t S,
                  int64_t rot, bool backward) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "rope: contiguous GPU input [B, S, H, D] required");
  const c10::DeviceGuard g(x.device());
  const int D = static_cast<int>(x.size(-1));
  TORCH_CHECK(rot % 2 == 0 && rot <= D, "rope: rot_dim must be even and <= head dim");
  Tensor y = torch::empty_like(x);
  dca::rope(tdt(x), x.data_ptr(), y.data_ptr(), cosT.data_ptr<float>(), sinT.data_ptr<float>(),
            x.numel() / D, static_cast<int>(H), static_cast<int>(S), D, static_cast<int>(rot),
            backward, stream());
  return y;
}

// q/k/v/o are [B, S, H, D] tensors (any strides with the last dim contiguous). The kernels take
// (batch, head, seq) strides, so both [B,S,H,D] and [B,H,S,D] layouts (and slices of a fused QKV
// projection) work without copies.
struct AttnStrides {
  int64_t v[3];
};
AttnStrides bshd_strides(const Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 4, "attention: ", name, " must be [B, S, H, D]");
  TORCH_CHECK(t.stride(3) == 1, "attention: ", name, " last dim must be contiguous");
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, "attention: ", name, " must be bf16");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && t.stride(1) % 8 == 0 &&
                  t.stride(2) % 8 == 0 && t.stride(0) % 8 == 0,
              "attention: ", name, " must be 16-byte aligned per row");
  return {{t.stride(0), t.stride(2), t.stride(1)}};
}

// K / V (and, in the backward, Q / dO) tiles load through buffer descriptors with 32-bit byte
// offsets (attention.hip KVPrefetch): one (batch, head) slice must span < 2 GiB
void check_range(const Tensor& t, const char* name) {
  TORCH_CHECK((t.size(1) + 256) * t.stride(1) * 2 < (int64_t(1) << 31),
              "attention: a (batch, head) slice of ", name, " must span < 2 GiB (sequence x row stride)");
}

// kv_len: optional int32 [B] valid key count per batch row (right padding, e.g. an HF
// attention_mask); keys at or past it get zero weight and zero dK/dV
const int* kvlen_ptr(const OptT& kv_len, int B) {
  if (!kv_len.has_value()) return nullptr;
  const Tensor& t = *kv_len;
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() == B,
              "attention: kv_len must be a contiguous int32 GPU tensor [B]");
  return t.data_ptr<int>();
}

std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, double scale,
                             bool causal, const OptT& kv_len) {
  TORCH_CHECK(q.is_cuda(), "attention: GPU tensors required");
  const c10::DeviceGuard g(q.device());
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int Sk = k.size(1);
  TORCH_CHECK(D == 64 || D == 128, "attention: head dim must be 64 or 128");
  const int Hkv = k.size(2);  // grouped-query attention: H % Hkv == 0 query heads per K/V head
  TORCH_CHECK(k.size(0) == B && Hkv > 0 && H % Hkv == 0 && k.size(3) == D && v.sizes() == k.sizes(),
              "attention: k/v shape mismatch (K/V heads must divide the query heads)");
  TORCH_CHECK(!causal || Sq == Sk, "attention: causal requires Sq == Sk");
  auto qs = bshd_strides(q, "q"), ks = bshd_strides(k, "k"), vs = bshd_strides(v, "v");
  check_range(k, "k");
  check_range(v, "v");
  Tensor o = torch::empty({B, Sq, H, D}, q.options());
  Tensor lse = torch::empty({B, H, Sq}, q.options().dtype(at::kFloat));
  auto os = bshd_strides(o, "o");
  dca::attention_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                     B, H, Sq, Sk, D, qs.v, ks.v, vs.v, os.v, static_cast<float>(scale), causal,
                     kvlen_ptr(kv_len, B), H / Hkv, stream());
  return {o, lse};
}

std::vector<Tensor> attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v,
                             const Tensor& o, const Tensor& lse, double scale, bool causal,
                             const OptT& dq_out, const OptT& dk_out, const OptT& dv_out,
                             const OptT& kv_len) {
  const c10::DeviceGuard g(q.device());
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), D = q.size(3);
  const int Sk = k.size(1);
  const int Hkv = k.size(2);
  TORCH_CHECK(Hkv > 0 && H % Hkv == 0 && v.sizes() == k.sizes(), "attention: k/v heads must divide q heads");
  Tensor dO = dout.stride(3) == 1 ? dout : dout.contiguous();
  auto qs = bshd_strides(q, "q"), ks = bshd_strides(k, "k"), vs = bshd_strides(v, "v");
  auto os = bshd_strides(o, "o"), dos = bshd_strides(dO, "dout");
  for (const Tensor* t : std::initializer_list<const Tensor*>{&q, &k, &v, &dO}) check_range(*t, "q/k/v/dout");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == static_cast<int64_t>(B) * H * Sq, "attention: lse");
  // optional preallocated outputs (e.g. views into one packed dQKV buffer)
  Tensor dq = dq_out.has_value() ? *dq_out : torch::empty({B, Sq, H, D}, q.options());
  Tensor dk = dk_out.has_value() ? *dk_out : torch::empty({B, Sk, Hkv, D}, q.options());
  Tensor dv = dv_out.has_value() ? *dv_out : torch::empty({B, Sk, Hkv, D}, q.options());
  TORCH_CHECK(dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes(),
              "attention: gradient output shape mismatch");
  auto fo = q.options().dtype(at::kFloat);
  Tensor delta = torch::empty({B, H, Sq}, fo);
  auto dqs = bshd_strides(dq, "dq"), dks = bshd_strides(dk, "dk"), dvs = bshd_strides(dv, "dv");
  dca::attention_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dO.data_ptr(),
                     lse.data_ptr<float>(), delta.data_ptr<float>(), nullptr,
                     dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B, H, Sq, Sk, D, qs.v, ks.v, vs.v,
                     os.v, dos.v, dqs.v, dks.v, dvs.v, static_cast<float>(scale), causal,
                     kvlen_ptr(kv_len, B), H / Hkv, stream());
  return {dq, dk, dv};
}
// logits [N, V] contiguous, target [N] int64 -> (lse [N], per-row loss [N])
std::vector<Tensor> ce_fwd(const Tensor& logits, const Tensor& target, int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "ce_fwd: [N, V] GPU logits");
  TORCH_CHECK(target.scalar_type() == at::kLong && target.is_contiguous() && target.numel() == logits.size(0),
              "ce_fwd: int64 targets [N]");
  const int V = static_cast<int>(logits.size(1));
  TORCH_CHECK(V % 8 == 0, "ce_fwd: vocab must be a multiple of 8 (pad it)");
  const c10::DeviceGuard g(logits.device());
  auto fo = logits.options().dtype(at::kFloat);
  Tensor lse = torch::empty({logits.size(0)}, fo), loss = torch::empty({logits.size(0)}, fo);
  dca::cross_entropy_fwd(tdt(logits), logits.data_ptr(), target.data_ptr<int64_t>(),
                         lse.data_ptr<float>(), loss.data_ptr<float>(), logits.size(0), V,
                         ignore_index, stream());
  return {lse, loss};
}

// gscale = [grad_output, n_valid] (fp32, device)
Tensor ce_bwd(const Tensor& logits, const Tensor& target, const Tensor& lse, const Tensor& gscale,
              int64_t ignore_index) {
  const c10::DeviceGuard g(logits.device());
  TORCH_CHECK(gscale.scalar_type() == at::kFloat && gscale.numel() == 2 && gscale.is_contiguous(), "ce_bwd: gscale");
  Tensor d = torch::empty_like(logits);
  dca::cross_entropy_bwd(tdt(logits), logits.data_ptr(), target.data_ptr<int64_t>(),
                         lse.data_ptr<float>(), gscale.data_ptr<float>(), d.data_ptr(),
                         logits.size(0), static_cast<int>(logits.size(1)), ignore_index, stream());
  return d;
}
}  // namespace

void register_transformer_ops(pybind11::module& m) {
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("gamma"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("dsum"),
        pybind11::arg("need_param_grads"), pybind11::arg("dgamma_acc") = pybind11::none(),
        pybind11::arg("dbeta_acc") = pybind11::none(), pybind11::arg("colsum_acc") = pybind11::none());
  m.def("bias_grad", &bias_grad, pybind11::arg("dy"), pybind11::arg("acc") = pybind11::none());
  m.def("bias_gelu", &bias_gelu);
  m.def("splitk_accumulate", &splitk_accumulate, pybind11::arg("part"), pybind11::arg("acc"),
        pybind11::arg("accumulate") = true);
  m.def("bias_gelu_bwd", &bias_gelu_bwd, pybind11::arg("dy"), pybind11::arg("x"),
        pybind11::arg("bias"), pybind11::arg("need_db") = true,
        pybind11::arg("dbias_acc") = pybind11::none());
  m.def("rope", &rope_apply);
  m.def("attn_fwd", &attn_fwd, pybind11::arg("q"), pybind11::arg("k"), pybind11::arg("v"),
        pybind11::arg("scale"), pybind11::arg("causal"), pybind11::arg("kv_len") = pybind11::none());
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("attn_bwd", &attn_bwd, pybind11::arg("dout"), pybind11::arg("q"), pybind11::arg("k"),
        pybind11::arg("v"), pybind11::arg("o"), pybind11::arg("lse"), pybind11::arg("scale"),
        pybind11::arg("causal"), pybind11::arg("dq_out") = pybind11::none(),
        pybind11::arg("dk_out") = pybind11::none(), pybind11::arg("dv_out") = pybind11::none(),
        pybind11::arg("kv_len") = pybind11::none());
}
