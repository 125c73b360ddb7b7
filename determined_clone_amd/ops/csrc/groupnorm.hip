// Fused NHWC GroupNorm (+ SiLU) forward/backward for MI355X -- the normalisation of every
// ResNet block and spatial transformer in the latent-diffusion family (models/diffusion.py).
//
// Reference: the diffusion example runs diffusers' UNet/VAE, i.e. torch.nn.GroupNorm followed by
// F.silu (examples/diffusion/textual_inversion_stable_diffusion/detsd). On channels_last bf16
// activations PyTorch's GroupNorm transposes to NCHW and back (two full copies), runs its
// moments + apply kernels, and SiLU is another pass; here the whole thing is 3 launches / 2 passes
// over x forward and 4 launches / 2 passes backward, in the NHWC layout the convolutions use.
//
// x is [N][HW][C] (C % 8 == 0), G groups of Cg = C / G consecutive channels.
//   gn_reduce<FWD>   : per-(n, chunk) partial (sum x, sum x^2) per channel          (reads x)
//   gn_finalize_fwd  : per sample: channel sums -> group mean / rstd (fp64) -> per-(n, c)
//                      scale/shift for the apply and (rstd, -mean*rstd) for the backward
//   gn_apply_fwd     : y = act(x * scale[n,c] + shift[n,c])                     (reads x, writes y)
//   gn_reduce<BWD>   : dz = dy * act'(z) (z recomputed from x), partial (sum dz, sum dz*xhat)
//   gn_finalize_bwd  : per sample: group terms -> dx = k1[n,c]*dz + k2[n,c]*x + k3[n,c]
//   gn_param_grad    : dgamma[c] = sum_n sum dz*xhat, dbeta[c] = sum_n sum dz (into .grad)
//   gn_apply_bwd     : dx
// Every lane moves 8 channels (16 B of bf16); TPR lanes cover a row's channel group, chunks of
// contiguous rows per workgroup; reductions are deterministic (no float atomics).
#include <cstdio>
#include <type_traits>
#include "common.h"

namespace dca {

enum class GnDtype : int { kF32 = 0, kBF16 = 1 };

namespace {

constexpr int kBlock = 256;

struct GnGeom {
  int tpr, rpi, cgroups, chunks;
};

// TPR = largest power of two <= 32 dividing C/8, so channel groups are exact (C = 320 -> 8
// lanes x 5 groups, 640 -> 16 x 5, 1280 -> 32 x 5); chunks per sample sized for ~2048 blocks.
inline GnGeom gn_geom(int N, int64_t HW, int C) {
  const int c8 = C / 8;
  int tpr = 32;
  while (tpr > 1 && c8 % tpr) tpr >>= 1;
  GnGeom g;
  g.tpr = tpr;
  g.rpi = kBlock / tpr;
  g.cgroups = c8 / tpr;
  int64_t want = 2048 / (static_cast<int64_t>(N) * g.cgroups);
  int64_t max_chunks = (HW + g.rpi * 2 - 1) / (g.rpi * 2);  // >= 2 row iterations per block
  if (want > max_chunks) want = max_chunks;
  if (want < 1) want = 1;
  g.chunks = static_cast<int>(want);
  return g;
}

__device__ __forceinline__ void chunk_range(int64_t HW, int rpi, int bx, int nb, int64_t& b, int64_t& e) {
  int64_t per = (HW + nb - 1) / nb;
  per = (per + rpi - 1) / rpi * rpi;
  b = static_cast<int64_t>(bx) * per;
  e = b + per;
  if (b > HW) b = HW;
  if (e > HW) e = HW;
}

__device__ __forceinline__ float silu_grad(float z) {
  const float s = 1.f / (1.f + __expf(-z));
  return s * (1.f + z * (1.f - s));
}

template <typename T>
__device__ __forceinline__ void ld(const void* p, int64_t off, float (&v)[8]) {
  Vec8<T>::load(reinterpret_cast<const char*>(p) + off * Vec8<T>::bytes, v);
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// grid (chunks, N, cgroups). partial: [N][chunks][2][C].
template <typename T, bool BWD, bool ACT>
__global__ __launch_bounds__(kBlock) void gn_reduce_kernel(
    const void* __restrict__ x, const void* __restrict__ dy, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ xa, const float* __restrict__ xb,
    int64_t HW, int C, int tpr, int rpi, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [rpi][tpr*16]
  const int tid = threadIdx.x, lc = tid % tpr, r0 = tid / tpr;
  const int n = blockIdx.y;
  const int c = (blockIdx.z * tpr + lc) * 8;
  int64_t b, e;
  chunk_range(HW, rpi, blockIdx.x, gridDim.x, b, e);
  const int64_t base = static_cast<int64_t>(n) * HW * C;
  float s[8], q[8], sc[8], sh[8], a[8], bb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  if (BWD) {
    const int64_t pc = static_cast<int64_t>(n) * C + c;
    ld8f(scale + pc, sc); ld8f(shift + pc, sh); ld8f(xa + pc, a); ld8f(xb + pc, bb);
  }
  for (int64_t r = b + r0; r < e; r += rpi) {
    const int64_t off = base + r * C + c;
    float xv[8];
    ld<T>(x, off, xv);
    if (!BWD) {
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += xv[k]; q[k] = fmaf(xv[k], xv[k], q[k]); }
    } else {
      float g[8];
      ld<T>(dy, off, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float dz = g[k];
        if (ACT) dz *= silu_grad(fmaf(xv[k], sc[k], sh[k]));
        s[k] += dz;
        q[k] = fmaf(dz, fmaf(xv[k], a[k], bb[k]), q[k]);
      }
    }
  }
  const int width = tpr * 16;
  float* mine = lds + r0 * width + lc * 16;
#pragma unroll
  for (int k = 0; k < 8; ++k) { mine[k] = s[k]; mine[8 + k] = q[k]; }
  __syncthreads();
  for (int o = tid; o < width; o += kBlock) {
    float acc = 0.f;
    for (int r = 0; r < rpi; ++r) acc += lds[r * width + o];
    const int ch = (blockIdx.z * tpr + o / 16) * 8 + (o % 16 & 7);
    const int which = (o % 16) >> 3;
    partial[((static_cast<int64_t>(n) * gridDim.x + blockIdx.x) * 2 + which) * C + ch] = acc;
  }
}

// One block per sample: channel sums in LDS, then group statistics, then per-channel outputs.
__global__ __launch_bounds__(kBlock) void gn_finalize_fwd_kernel(
    const float* __restrict__ partial, int chunks, int C, int G, int64_t HW,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
    float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ xa,
    float* __restrict__ xb, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  extern __shared__ double dl[];  // [2][C] channel sums, then [2][G] group stats
  const int n = blockIdx.x, Cg = C / G;
  double* cs = dl;
  double* gs = dl + 2 * C;
  for (int c = threadIdx.x; c < C; c += kBlock) {
    double a = 0.0, q = 0.0;
    for (int k = 0; k < chunks; ++k) {
      const float* p = partial + ((static_cast<int64_t>(n) * chunks + k) * 2) * C;
      a += p[c];
      q += p[C + c];
    }
    cs[c] = a;
    cs[C + c] = q;
  }
  __syncthreads();
  const double M = static_cast<double>(HW) * Cg;
  for (int g = threadIdx.x; g < G; g += kBlock) {
    double a = 0.0, q = 0.0;
    for (int j = 0; j < Cg; ++j) { a += cs[g * Cg + j]; q += cs[C + g * Cg + j]; }
    const double mu = a / M;
    double var = q / M - mu * mu;
    if (var < 0.0) var = 0.0;
    gs[g] = mu;
    gs[G + g] = 1.0 / sqrt(var + static_cast<double>(eps));
    mean_out[n * G + g] = static_cast<float>(mu);
    rstd_out[n * G + g] = static_cast<float>(gs[G + g]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    const int g = c / Cg;
    const float mu = static_cast<float>(gs[g]), rs = static_cast<float>(gs[G + g]);
    const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
    const int64_t i = static_cast<int64_t>(n) * C + c;
    scale[i] = rs * ga;
    shift[i] = be - mu * rs * ga;
    xa[i] = rs;
    xb[i] = -mu * rs;
  }
}

template <typename T, bool ACT>
__global__ __launch_bounds__(kBlock) void gn_apply_fwd_kernel(
    const void* __restrict__ x, void* __restrict__ y, const float* __restrict__ scale,
    const float* __restrict__ shift, int64_t HW, int C, int tpr, int rpi) {
  const int tid = threadIdx.x, lc = tid % tpr, r0 = tid / tpr;
  const int n = blockIdx.y;
  const int c = (blockIdx.z * tpr + lc) * 8;
  int64_t b, e;
  chunk_range(HW, rpi, blockIdx.x, gridDim.x, b, e);
  const int64_t base = static_cast<int64_t>(n) * HW * C;
  float sc[8], sh[8];
  ld8f(scale + static_cast<int64_t>(n) * C + c, sc);
  ld8f(shift + static_cast<int64_t>(n) * C + c, sh);
  int64_t r = b + r0;
  for (; r + rpi < e; r += 2 * rpi) {  // two rows in flight per lane
    const int64_t o0 = base + r * C + c, o1 = o0 + static_cast<int64_t>(rpi) * C;
    float v0[8], v1[8];
    ld<T>(x, o0, v0);
    ld<T>(x, o1, v1);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v0[k] = fmaf(v0[k], sc[k], sh[k]);
      v1[k] = fmaf(v1[k], sc[k], sh[k]);
      if (ACT) {
        v0[k] = v0[k] / (1.f + __expf(-v0[k]));
        v1[k] = v1[k] / (1.f + __expf(-v1[k]));
      }
    }
    Vec8<T>::store(reinterpret_cast<char*>(y) + o0 * Vec8<T>::bytes, v0);
    Vec8<T>::store(reinterpret_cast<char*>(y) + o1 * Vec8<T>::bytes, v1);
  }
  for (; r < e; r += rpi) {
    const int64_t o = base + r * C + c;
    float v[8];
    ld<T>(x, o, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      v[k] = fmaf(v[k], sc[k], sh[k]);
      if (ACT) v[k] = v[k] / (1.f + __expf(-v[k]));
    }
    Vec8<T>::store(reinterpret_cast<char*>(y) + o * Vec8<T>::bytes, v);
  }
}

// One block per sample. ab: [N][2][C] (sum dz, sum dz*xhat); coef: [N][3][C].
__global__ __launch_bounds__(kBlock) void gn_finalize_bwd_kernel(
    const float* __restrict__ partial, int chunks, int C, int G, int64_t HW,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ ab, float* __restrict__ coef) {
  extern __shared__ float fl[];  // [2][C] + [2][G]
  const int n = blockIdx.x, Cg = C / G;
  float* cs = fl;
  float* gs = fl + 2 * C;
  for (int c = threadIdx.x; c < C; c += kBlock) {
    float a = 0.f, q = 0.f;
    for (int k = 0; k < chunks; ++k) {
      const float* p = partial + ((static_cast<int64_t>(n) * chunks + k) * 2) * C;
      a += p[c];
      q += p[C + c];
    }
    cs[c] = a;
    cs[C + c] = q;
    ab[(static_cast<int64_t>(n) * 2) * C + c] = a;
    ab[(static_cast<int64_t>(n) * 2 + 1) * C + c] = q;
  }
  __syncthreads();
  const float invM = 1.f / (static_cast<float>(HW) * Cg);
  for (int g = threadIdx.x; g < G; g += kBlock) {
    float a = 0.f, q = 0.f;
    for (int j = 0; j < Cg; ++j) {
      const int c = g * Cg + j;
      const float ga = gamma ? gamma[c] : 1.f;
      a += ga * cs[c];
      q += ga * cs[C + c];
    }
    gs[g] = a * invM;      // mean over the group of gamma * dz
    gs[G + g] = q * invM;  // mean of gamma * dz * xhat
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kBlock) {
    const int g = c / Cg;
    const float mu = mean[n * G + g], rs = rstd[n * G + g];
    const float ga = gamma ? gamma[c] : 1.f;
    const float mg = gs[g], mgx = gs[G + g];
    float* o = coef + static_cast<int64_t>(n) * 3 * C;
    o[c] = rs * ga;                               // * dz
    o[C + c] = -rs * rs * mgx;                    // * x
    o[2 * C + c] = -rs * mg + mu * rs * rs * mgx;  // constant
  }
}

__global__ __launch_bounds__(kBlock) void gn_param_grad_kernel(
    const float* __restrict__ ab, int N, int C, float* __restrict__ dgamma, float* __restrict__ dbeta,
    bool accumulate) {
  const int c = blockIdx.x * kBlock + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, q = 0.f;
  for (int n = 0; n < N; ++n) {
    a += ab[(static_cast<int64_t>(n) * 2) * C + c];
    q += ab[(static_cast<int64_t>(n) * 2 + 1) * C + c];
  }
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + q : q;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + a : a;
}

template <typename T, bool ACT>
__global__ __launch_bounds__(kBlock) void gn_apply_bwd_kernel(
    const void* __restrict__ x, const void* __restrict__ dy, void* __restrict__ dx,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ coef,
    int64_t HW, int C, int tpr, int rpi) {
  const int tid = threadIdx.x, lc = tid % tpr, r0 = tid / tpr;
  const int n = blockIdx.y;
  const int c = (blockIdx.z * tpr + lc) * 8;
  int64_t b, e;
  chunk_range(HW, rpi, blockIdx.x, gridDim.x, b, e);
  const int64_t base = static_cast<int64_t>(n) * HW * C;
  float sc[8], sh[8], k1[8], k2[8], k3[8];
  const int64_t pc = static_cast<int64_t>(n) * C + c;
  if (ACT) { ld8f(scale + pc, sc); ld8f(shift + pc, sh); }
  const float* co = coef + static_cast<int64_t>(n) * 3 * C + c;
  ld8f(co, k1); ld8f(co + C, k2); ld8f(co + 2 * C, k3);
  for (int64_t r = b + r0; r < e; r += rpi) {
    const int64_t o = base + r * C + c;
    float xv[8], g[8], out[8];
    ld<T>(x, o, xv);
    ld<T>(dy, o, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float dz = g[k];
      if (ACT) dz *= silu_grad(fmaf(xv[k], sc[k], sh[k]));
      out[k] = fmaf(k1[k], dz, fmaf(k2[k], xv[k], k3[k]));
    }
    Vec8<T>::store(reinterpret_cast<char*>(dx) + o * Vec8<T>::bytes, out);
  }
}

template <typename T>
void fwd_impl(const void* x, void* y, const float* gamma, const float* beta, int N, int64_t HW,
              int C, int G, float eps, bool act, float* partial, float* scale, float* shift,
              float* xa, float* xb, float* mean, float* rstd, hipStream_t st) {
  const GnGeom g = gn_geom(N, HW, C);
  dim3 grid(g.chunks, N, g.cgroups);
  const size_t lds = static_cast<size_t>(g.rpi) * g.tpr * 16 * sizeof(float);
  hipLaunchKernelGGL((gn_reduce_kernel<T, false, false>), grid, dim3(kBlock), lds, st, x, nullptr,
                     nullptr, nullptr, nullptr, nullptr, HW, C, g.tpr, g.rpi, partial);
  hipLaunchKernelGGL(gn_finalize_fwd_kernel, dim3(N), dim3(kBlock), (2 * C + 2 * G) * sizeof(double), st,
                     partial, g.chunks, C, G, HW, gamma, beta, eps, scale, shift, xa, xb, mean, rstd);
  if (act)
    hipLaunchKernelGGL((gn_apply_fwd_kernel<T, true>), grid, dim3(kBlock), 0, st, x, y, scale, shift, HW, C, g.tpr, g.rpi);
  else
    hipLaunchKernelGGL((gn_apply_fwd_kernel<T, false>), grid, dim3(kBlock), 0, st, x, y, scale, shift, HW, C, g.tpr, g.rpi);
}

template <typename T>
void bwd_impl(const void* dy, const void* x, void* dx, const float* gamma, const float* scale,
              const float* shift, const float* xa, const float* xb, const float* mean,
              const float* rstd, int N, int64_t HW, int C, int G, bool act, float* partial,
              float* ab, float* coef, float* dgamma, float* dbeta, bool accumulate, hipStream_t st) {
  const GnGeom g = gn_geom(N, HW, C);
  dim3 grid(g.chunks, N, g.cgroups);
  const size_t lds = static_cast<size_t>(g.rpi) * g.tpr * 16 * sizeof(float);
  if (act)
    hipLaunchKernelGGL((gn_reduce_kernel<T, true, true>), grid, dim3(kBlock), lds, st, x, dy, scale,
                       shift, xa, xb, HW, C, g.tpr, g.rpi, partial);
  else
    hipLaunchKernelGGL((gn_reduce_kernel<T, true, false>), grid, dim3(kBlock), lds, st, x, dy, scale,
                       shift, xa, xb, HW, C, g.tpr, g.rpi, partial);
  hipLaunchKernelGGL(gn_finalize_bwd_kernel, dim3(N), dim3(kBlock), (2 * C + 2 * G) * sizeof(float), st,
                     partial, g.chunks, C, G, HW, gamma, mean, rstd, ab, coef);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(gn_param_grad_kernel, dim3((C + kBlock - 1) / kBlock), dim3(kBlock), 0, st, ab,
                       N, C, dgamma, dbeta, accumulate);
  if (act)
    hipLaunchKernelGGL((gn_apply_bwd_kernel<T, true>), grid, dim3(kBlock), 0, st, x, dy, dx, scale, shift, coef, HW, C, g.tpr, g.rpi);
  else
    hipLaunchKernelGGL((gn_apply_bwd_kernel<T, false>), grid, dim3(kBlock), 0, st, x, dy, dx, scale, shift, coef, HW, C, g.tpr, g.rpi);
}

}  // namespace

int gn_chunks(int N, int64_t HW, int C) { return gn_geom(N, HW, C).chunks; }

void groupnorm_forward(GnDtype dt, const void* x, void* y, const float* gamma, const float* beta,
                       int N, int64_t HW, int C, int G, float eps, bool act, float* partial,
                       float* scale, float* shift, float* xa, float* xb, float* mean, float* rstd,
                       hipStream_t st) {
  if (dt == GnDtype::kBF16)
    fwd_impl<BF16>(x, y, gamma, beta, N, HW, C, G, eps, act, partial, scale, shift, xa, xb, mean, rstd, st);
  else
    fwd_impl<F32>(x, y, gamma, beta, N, HW, C, G, eps, act, partial, scale, shift, xa, xb, mean, rstd, st);
}

void groupnorm_backward(GnDtype dt, const void* dy, const void* x, void* dx, const float* gamma,
                        const float* scale, const float* shift, const float* xa, const float* xb,
                        const float* mean, const float* rstd, int N, int64_t HW, int C, int G,
                        bool act, float* partial, float* ab, float* coef, float* dgamma,
                        float* dbeta, bool accumulate, hipStream_t st) {
  if (dt == GnDtype::kBF16)
    bwd_impl<BF16>(dy, x, dx, gamma, scale, shift, xa, xb, mean, rstd, N, HW, C, G, act, partial,
                   ab, coef, dgamma, dbeta, accumulate, st);
  else
    bwd_impl<F32>(dy, x, dx, gamma, scale, shift, xa, xb, mean, rstd, N, HW, C, G, act, partial,
                  ab, coef, dgamma, dbeta, accumulate, st);
}

}  // namespace dca
