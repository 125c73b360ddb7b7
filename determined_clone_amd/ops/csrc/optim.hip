// Flat-buffer fused optimizers, gradient-norm clipping and AMP loss-scale kernels for MI355X.
//
// Parity targets in the reference: `PyTorchTrialContext.step_optimizer(clip_grads=...)`
// (harness/determined/pytorch/_pytorch_context.py:827-925), native/apex AMP loss scaling
// (_pytorch_context.py:515-700) and the fused Adam/LAMB the DeepSpeedTrial path gets from DeepSpeed.
//
// MI355X-first design: parameters, gradients and optimizer state live in FLAT per-dtype buffers
// (parallel/flat.py), so one optimizer step is ONE grid-stride streaming pass at HBM rate instead
// of a per-tensor loop, DDP buckets are plain slices of the gradient buffer, and ZeRO shards are
// contiguous ranges. Everything that would force a host sync in the reference (GradScaler's inf
// check, clip coefficient) stays on the device:
//   sumsq_partial -> norm_finalize   : global grad L2 norm, found_inf, combined grad multiplier
//   sgd/adam kernels                 : read that multiplier + found_inf flag (skip step on inf)
//   scaler_update                    : dynamic loss-scale growth/backoff on the device
// LAMB needs per-tensor norms: a chunk table (chunk -> segment) drives seg_sumsq/lamb kernels.
#include "common.h"

namespace dca {

enum class OptDtype : int { kF32 = 0, kBF16 = 1, kF16 = 2, kNone = 3 };

namespace {

constexpr int kBlock = 256;

template <typename T> struct V4;
template <> struct V4<F32> {
  __device__ __forceinline__ static float4 load(const void* p, int64_t i) {
    return reinterpret_cast<const float4*>(p)[i];
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, float4 v) {
    reinterpret_cast<float4*>(p)[i] = v;
  }
  __device__ __forceinline__ static float load1(const void* p, int64_t i) {
    return reinterpret_cast<const float*>(p)[i];
  }
  __device__ __forceinline__ static void store1(void* p, int64_t i, float v) {
    reinterpret_cast<float*>(p)[i] = v;
  }
};
template <> struct V4<BF16> {
  __device__ __forceinline__ static float4 load(const void* p, int64_t i) {
    uint2 q = reinterpret_cast<const uint2*>(p)[i];
    return make_float4(bf16_lo(q.x), bf16_hi(q.x), bf16_lo(q.y), bf16_hi(q.y));
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, float4 v) {
    reinterpret_cast<uint2*>(p)[i] = make_uint2(pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w));
  }
  __device__ __forceinline__ static float load1(const void* p, int64_t i) {
    return __uint_as_float(static_cast<uint32_t>(reinterpret_cast<const uint16_t*>(p)[i]) << 16);
  }
  __device__ __forceinline__ static void store1(void* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(f2bf_bits(v));
  }
};
template <> struct V4<F16> {
  __device__ __forceinline__ static float4 load(const void* p, int64_t i) {
    uint2 q = reinterpret_cast<const uint2*>(p)[i];
    return make_float4(h2f(q.x & 0xffff), h2f(q.x >> 16), h2f(q.y & 0xffff), h2f(q.y >> 16));
  }
  __device__ __forceinline__ static void store(void* p, int64_t i, float4 v) {
    reinterpret_cast<uint2*>(p)[i] =
        make_uint2(f2h(v.x) | (static_cast<uint32_t>(f2h(v.y)) << 16),
                   f2h(v.z) | (static_cast<uint32_t>(f2h(v.w)) << 16));
  }
  __device__ __forceinline__ static float load1(const void* p, int64_t i) {
    return h2f(reinterpret_cast<const uint16_t*>(p)[i]);
  }
  __device__ __forceinline__ static void store1(void* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = f2h(v);
  }
};

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }

// ------------------------------------------------------------------ global sum of squares
template <typename G>
__global__ __launch_bounds__(kBlock) void sumsq_partial_kernel(const void* __restrict__ g,
                                                               int64_t n, float* __restrict__ partial) {
  __shared__ float scratch[kBlock / 64];
  float acc = 0.f;
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = V4<G>::load(g, i);
    acc = fmaf(v.x, v.x, acc); acc = fmaf(v.y, v.y, acc);
    acc = fmaf(v.z, v.z, acc); acc = fmaf(v.w, v.w, acc);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float v = V4<G>::load1(g, i);
      acc = fmaf(v, v, acc);
    }
  acc = block_sum(acc, scratch);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// out[0] = grad multiplier (inv_loss_scale * extra_scale * clip_coef), out[1] = found_inf (0/1),
// out[2] = unscaled global grad norm (after extra_scale, before clipping).
__global__ __launch_bounds__(kBlock) void norm_finalize_kernel(
    const float* __restrict__ partial, int nparts, const float* __restrict__ loss_scale,
    float extra_scale, float max_norm, float* __restrict__ out) {
  __shared__ double red[kBlock];
  double s = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double tot = red[0];
    const bool inf = !isfinite(tot);
    const float inv_ls = loss_scale ? 1.f / loss_scale[0] : 1.f;
    const float mult = inv_ls * extra_scale;
    const float norm = static_cast<float>(sqrt(tot)) * mult;
    float coef = 1.f;
    if (max_norm > 0.f && isfinite(norm)) {
      const float c = max_norm / (norm + 1e-6f);
      coef = c < 1.f ? c : 1.f;
    }
    out[0] = mult * coef;
    out[1] = inf ? 1.f : 0.f;
    out[2] = inf ? __builtin_inff() : norm;
  }
}

// ------------------------------------------------------------------ SGD (momentum, nesterov)
// master (fp32) is updated in place; `model` (optional, dtype P) receives the low-precision copy.
template <typename G, typename P>
__global__ __launch_bounds__(kBlock) void sgd_kernel(
    float* __restrict__ master, void* __restrict__ model, const void* __restrict__ grad,
    float* __restrict__ mom, int64_t n, float lr, float momentum, float dampening, float wd,
    bool nesterov, bool first_step, float gscale, const float* __restrict__ dev_scale,
    const float* __restrict__ dyn) {
  if (dev_scale && dev_scale[1] != 0.f) return;  // found_inf: skip the step
  // Device-resident step hyper-parameters (HIP-graph replay: refreshed before each launch).
  if (dyn) { lr = dyn[0]; first_step = dyn[1] != 0.f; }
  const float gs = gscale * (dev_scale ? dev_scale[0] : 1.f);
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  auto upd = [&](float w, float g, float& b) -> float {
    g = fmaf(g, gs, wd * w);
    if (momentum != 0.f) {
      b = first_step ? g : fmaf(momentum, b, (1.f - dampening) * g);
      g = nesterov ? fmaf(momentum, b, g) : b;
    }
    return fmaf(-lr, g, w);
  };
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 w = V4<F32>::load(master, i);
    float4 g = V4<G>::load(grad, i);
    float4 b = momentum != 0.f ? V4<F32>::load(mom, i) : f4(0.f);
    w.x = upd(w.x, g.x, b.x); w.y = upd(w.y, g.y, b.y);
    w.z = upd(w.z, g.z, b.z); w.w = upd(w.w, g.w, b.w);
    V4<F32>::store(master, i, w);
    if (momentum != 0.f) V4<F32>::store(mom, i, b);
    if (model) V4<P>::store(model, i, w);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float b = momentum != 0.f ? mom[i] : 0.f;
      float w = upd(master[i], V4<G>::load1(grad, i), b);
      master[i] = w;
      if (momentum != 0.f) mom[i] = b;
      if (model) V4<P>::store1(model, i, w);
    }
}

// ------------------------------------------------------------------ Adam / AdamW
template <typename G, typename P>
__global__ __launch_bounds__(kBlock) void adam_kernel(
    float* __restrict__ master, void* __restrict__ model, const void* __restrict__ grad,
    float* __restrict__ m, float* __restrict__ v, int64_t n, float lr, float beta1, float beta2,
    float eps, float wd, bool adamw, float bc1, float bc2, float gscale,
    const float* __restrict__ dev_scale, const float* __restrict__ dyn) {
  if (dev_scale && dev_scale[1] != 0.f) return;
  if (dyn) { lr = dyn[0]; bc1 = dyn[1]; bc2 = dyn[2]; }
  const float gs = gscale * (dev_scale ? dev_scale[0] : 1.f);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  auto upd = [&](float w, float g, float& mm, float& vv) -> float {
    g *= gs;
    if (adamw) w = w * (1.f - lr * wd);
    else g = fmaf(wd, w, g);
    mm = fmaf(beta1, mm, (1.f - beta1) * g);
    vv = fmaf(beta2, vv, (1.f - beta2) * g * g);
    const float denom = sqrtf(vv) * inv_sqrt_bc2 + eps;
    return w - step_size * mm / denom;
  };
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 w = V4<F32>::load(master, i), g = V4<G>::load(grad, i);
    float4 a = V4<F32>::load(m, i), b = V4<F32>::load(v, i);
    w.x = upd(w.x, g.x, a.x, b.x); w.y = upd(w.y, g.y, a.y, b.y);
    w.z = upd(w.z, g.z, a.z, b.z); w.w = upd(w.w, g.w, a.w, b.w);
    V4<F32>::store(master, i, w); V4<F32>::store(m, i, a); V4<F32>::store(v, i, b);
    if (model) V4<P>::store(model, i, w);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
      float a = m[i], b = v[i];
      float w = upd(master[i], V4<G>::load1(grad, i), a, b);
      master[i] = w; m[i] = a; v[i] = b;
      if (model) V4<P>::store1(model, i, w);
    }
}

// ------------------------------------------------------------------ LAMB (chunk table)
// Chunk c covers [start[c], start[c]+len[c]) of the flat buffers and belongs to segment seg[c].
// Stage 1: m,v update and the raw update u (incl. decoupled weight decay) written into `ubuf`
//          (fp32, may alias nothing), plus per-chunk partial ||w||^2 and ||u||^2.
template <typename G>
__global__ __launch_bounds__(kBlock) void lamb_stage1_kernel(
    const float* __restrict__ master, const void* __restrict__ grad, float* __restrict__ m,
    float* __restrict__ v, float* __restrict__ ubuf, const int64_t* __restrict__ cstart,
    const int* __restrict__ clen, float beta1, float beta2, float eps, float wd, float bc1,
    float bc2, float gscale, const float* __restrict__ dev_scale, float* __restrict__ part_w,
    float* __restrict__ part_u) {
  __shared__ float scratch[kBlock / 64];
  if (dev_scale && dev_scale[1] != 0.f) {
    if (threadIdx.x == 0) { part_w[blockIdx.x] = 0.f; part_u[blockIdx.x] = 0.f; }
    return;
  }
  const float gs = gscale * (dev_scale ? dev_scale[0] : 1.f);
  const int64_t s0 = cstart[blockIdx.x];
  const int len = clen[blockIdx.x];
  float aw = 0.f, au = 0.f;
  for (int j = threadIdx.x; j < len; j += blockDim.x) {
    const int64_t i = s0 + j;
    const float w = master[i];
    const float g = V4<G>::load1(grad, i) * gs;
    const float mm = fmaf(beta1, m[i], (1.f - beta1) * g);
    const float vv = fmaf(beta2, v[i], (1.f - beta2) * g * g);
    m[i] = mm; v[i] = vv;
    const float u = (mm / bc1) / (sqrtf(vv / bc2) + eps) + wd * w;
    ubuf[i] = u;
    aw = fmaf(w, w, aw);
    au = fmaf(u, u, au);
  }
  aw = block_sum(aw, scratch);
  au = block_sum(au, scratch);
  if (threadIdx.x == 0) { part_w[blockIdx.x] = aw; part_u[blockIdx.x] = au; }
}

// Per-segment trust ratio from the chunk partials (chunks of a segment are consecutive).
__global__ void lamb_ratio_kernel(const float* __restrict__ part_w, const float* __restrict__ part_u,
                                  const int* __restrict__ seg_chunk_begin, int nseg,
                                  float* __restrict__ ratio) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  double w = 0.0, u = 0.0;
  for (int c = seg_chunk_begin[s]; c < seg_chunk_begin[s + 1]; ++c) { w += part_w[c]; u += part_u[c]; }
  const double wn = sqrt(w), un = sqrt(u);
  ratio[s] = (wn > 0.0 && un > 0.0) ? static_cast<float>(wn / un) : 1.f;
}

template <typename P>
__global__ __launch_bounds__(kBlock) void lamb_stage2_kernel(
    float* __restrict__ master, void* __restrict__ model, const float* __restrict__ ubuf,
    const int64_t* __restrict__ cstart, const int* __restrict__ clen, const int* __restrict__ cseg,
    const float* __restrict__ ratio, float lr, const float* __restrict__ dev_scale) {
  if (dev_scale && dev_scale[1] != 0.f) return;
  const int64_t s0 = cstart[blockIdx.x];
  const int len = clen[blockIdx.x];
  const float r = lr * ratio[cseg[blockIdx.x]];
  for (int j = threadIdx.x; j < len; j += blockDim.x) {
    const int64_t i = s0 + j;
    const float w = fmaf(-r, ubuf[i], master[i]);
    master[i] = w;
    if (model) V4<P>::store1(model, i, w);
  }
}

// ------------------------------------------------------------------ AMP loss scale update
// state: [0] scale, [1] growth_tracker (as float). found_inf read from `dev_scale[1]`.
__global__ void scaler_update_kernel(float* __restrict__ state, const float* __restrict__ dev_scale,
                                     float growth, float backoff, int interval) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (dev_scale[1] != 0.f) {
    state[0] *= backoff;
    state[1] = 0.f;
  } else {
    state[1] += 1.f;
    if (state[1] >= static_cast<float>(interval)) {
      const float ns = state[0] * growth;
      if (isfinite(ns)) state[0] = ns;
      state[1] = 0.f;
    }
  }
}

// y = x * s (in place allowed) over a flat buffer, s read from device dev_scale[0] * host scale.
template <typename G>
__global__ __launch_bounds__(kBlock) void scale_kernel(void* __restrict__ x, int64_t n, float s,
                                                       const float* __restrict__ dev_scale) {
  const float k = s * (dev_scale ? dev_scale[0] : 1.f);
  const int64_t n4 = n / 4;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = V4<G>::load(x, i);
    v.x *= k; v.y *= k; v.z *= k; v.w *= k;
    V4<G>::store(x, i, v);
  }
  if (blockIdx.x == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) V4<G>::store1(x, i, V4<G>::load1(x, i) * k);
}

}  // namespace

int sumsq_partial_blocks(int64_t n) { return stream_grid((n + 3) / 4, kBlock); }

void sumsq_partial(OptDtype g, const void* grad, int64_t n, float* partial, int blocks,
                   hipStream_t st) {
  switch (g) {
    case OptDtype::kBF16: hipLaunchKernelGGL(sumsq_partial_kernel<BF16>, dim3(blocks), dim3(kBlock), 0, st, grad, n, partial); break;
    case OptDtype::kF16: hipLaunchKernelGGL(sumsq_partial_kernel<F16>, dim3(blocks), dim3(kBlock), 0, st, grad, n, partial); break;
    default: hipLaunchKernelGGL(sumsq_partial_kernel<F32>, dim3(blocks), dim3(kBlock), 0, st, grad, n, partial); break;
  }
}

void norm_finalize(const float* partial, int nparts, const float* loss_scale, float extra_scale,
                   float max_norm, float* out, hipStream_t st) {
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(kBlock), 0, st, partial, nparts,
                     loss_scale, extra_scale, max_norm, out);
}

#define DCA_DISPATCH_GP(G, P, KERNEL, GRID, ...)                                                \
  do {                                                                                          \
    dim3 _g(GRID), _b(kBlock);                                                                  \
    auto _launch = [&](auto gtag, auto ptag) {                                                  \
      using GT = decltype(gtag);                                                                \
      using PT = decltype(ptag);                                                                \
      hipLaunchKernelGGL((KERNEL<GT, PT>), _g, _b, 0, st, __VA_ARGS__);                         \
    };                                                                                          \
    auto _p = [&](auto gtag) {                                                                  \
      switch (P) {                                                                              \
        case OptDtype::kBF16: _launch(gtag, BF16{}); break;                                     \
        case OptDtype::kF16: _launch(gtag, F16{}); break;                                       \
        default: _launch(gtag, F32{}); break;                                                   \
      }                                                                                         \
    };                                                                                          \
    switch (G) {                                                                                \
      case OptDtype::kBF16: _p(BF16{}); break;                                                  \
      case OptDtype::kF16: _p(F16{}); break;                                                    \
      default: _p(F32{}); break;                                                                \
    }                                                                                           \
  } while (0)

void sgd_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* mom,
              int64_t n, float lr, float momentum, float dampening, float wd, bool nesterov,
              bool first_step, float gscale, const float* dev_scale, const float* dyn,
              hipStream_t st) {
  const int grid = stream_grid((n + 3) / 4, kBlock);
  DCA_DISPATCH_GP(gdt, pdt, sgd_kernel, grid, master, model, grad, mom, n, lr, momentum,
                  dampening, wd, nesterov, first_step, gscale, dev_scale, dyn);
}

void adam_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* m,
               float* v, int64_t n, float lr, float beta1, float beta2, float eps, float wd,
               bool adamw, float bc1, float bc2, float gscale, const float* dev_scale,
               const float* dyn, hipStream_t st) {
  const int grid = stream_grid((n + 3) / 4, kBlock);
  DCA_DISPATCH_GP(gdt, pdt, adam_kernel, grid, master, model, grad, m, v, n, lr, beta1, beta2,
                  eps, wd, adamw, bc1, bc2, gscale, dev_scale, dyn);
}

void lamb_step(OptDtype gdt, OptDtype pdt, float* master, void* model, const void* grad, float* m,
               float* v, float* ubuf, const int64_t* cstart, const int* clen, const int* cseg,
               int nchunks, const int* seg_chunk_begin, int nseg, float* part_w, float* part_u,
               float* ratio, float lr, float beta1, float beta2, float eps, float wd, float bc1,
               float bc2, float gscale, const float* dev_scale, hipStream_t st) {
  switch (gdt) {
    case OptDtype::kBF16: hipLaunchKernelGGL(lamb_stage1_kernel<BF16>, dim3(nchunks), dim3(kBlock), 0, st, master, grad, m, v, ubuf, cstart, clen, beta1, beta2, eps, wd, bc1, bc2, gscale, dev_scale, part_w, part_u); break;
    case OptDtype::kF16: hipLaunchKernelGGL(lamb_stage1_kernel<F16>, dim3(nchunks), dim3(kBlock), 0, st, master, grad, m, v, ubuf, cstart, clen, beta1, beta2, eps, wd, bc1, bc2, gscale, dev_scale, part_w, part_u); break;
    default: hipLaunchKernelGGL(lamb_stage1_kernel<F32>, dim3(nchunks), dim3(kBlock), 0, st, master, grad, m, v, ubuf, cstart, clen, beta1, beta2, eps, wd, bc1, bc2, gscale, dev_scale, part_w, part_u); break;
  }
  hipLaunchKernelGGL(lamb_ratio_kernel, dim3((nseg + 255) / 256), dim3(256), 0, st, part_w, part_u,
                     seg_chunk_begin, nseg, ratio);
  switch (pdt) {
    case OptDtype::kBF16: hipLaunchKernelGGL(lamb_stage2_kernel<BF16>, dim3(nchunks), dim3(kBlock), 0, st, master, model, ubuf, cstart, clen, cseg, ratio, lr, dev_scale); break;
    case OptDtype::kF16: hipLaunchKernelGGL(lamb_stage2_kernel<F16>, dim3(nchunks), dim3(kBlock), 0, st, master, model, ubuf, cstart, clen, cseg, ratio, lr, dev_scale); break;
    default: hipLaunchKernelGGL(lamb_stage2_kernel<F32>, dim3(nchunks), dim3(kBlock), 0, st, master, model, ubuf, cstart, clen, cseg, ratio, lr, dev_scale); break;
  }
}

void scaler_update(float* state, const float* dev_scale, float growth, float backoff, int interval,
                   hipStream_t st) {
  hipLaunchKernelGGL(scaler_update_kernel, dim3(1), dim3(64), 0, st, state, dev_scale, growth,
                     backoff, interval);
}

void scale_inplace(OptDtype dt, void* x, int64_t n, float s, const float* dev_scale, hipStream_t st) {
  const int grid = stream_grid((n + 3) / 4, kBlock);
  switch (dt) {
    case OptDtype::kBF16: hipLaunchKernelGGL(scale_kernel<BF16>, dim3(grid), dim3(kBlock), 0, st, x, n, s, dev_scale); break;
    case OptDtype::kF16: hipLaunchKernelGGL(scale_kernel<F16>, dim3(grid), dim3(kBlock), 0, st, x, n, s, dev_scale); break;
    default: hipLaunchKernelGGL(scale_kernel<F32>, dim3(grid), dim3(kBlock), 0, st, x, n, s, dev_scale); break;
  }
}

}  // namespace dca
