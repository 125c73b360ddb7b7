// Fused NHWC BatchNorm (+ residual add) (+ ReLU) forward/backward for MI355X.
//
// Replaces the reference's cuDNN BatchNorm + separate add/ReLU kernels in the ResNet-50 trial
// (reference: torchvision resnet50 driven by harness/determined/pytorch/_pytorch_trial.py).
// Activations are channels_last, i.e. a row-major [M = N*H*W][C] matrix, C % 8 == 0.
//
// Training forward = 3 launches, 2 passes over x:
//   bn_reduce<FWD>   : per-block partial (sum x, sum x^2) per channel          (reads x)
//   bn_finalize_fwd  : channel-parallel combine of partials in fp64, running stats update,
//                      per-channel scale/shift, num_batches_tracked += 1
//   bn_apply_fwd     : y = act(x*scale + shift [+ res])                        (reads x[,res], writes y)
// Training backward = 3 launches, 2 passes:
//   bn_reduce<BWD>   : partial (sum dy', sum dy'*(x-mean)), dy' = relu ? dy*mask : dy
// The forward stores the ReLU decision as a 1-bit-per-element mask (1/16 of the bf16 output), so
// the backward never re-reads y.
//   bn_finalize_bwd  : dgamma, dbeta and the affine form dx = k1*dy' + k2*x + k3
//   bn_apply_bwd     : dx (and d_residual = dy' when the residual add was fused)
// Every lane moves 8 channels (16 B of bf16) per access; reductions are deterministic.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include "common.h"

namespace dca {

enum class BnDtype : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

namespace {

constexpr int kBlock = 256;

// Row-tile geometry shared by every pass over a [M rows][C channels] channels_last tensor:
// TPR threads cover one row (8 channels = 16 B of bf16 each), RPI = rows per block iteration,
// channel groups on grid.y when C/8 > 256. Each workgroup owns ONE contiguous run of rows (a
// multiple of RPI), so its loads stream through a contiguous region, every thread keeps the same
// 8 channels for the whole kernel (per-channel parameters are loaded once, no per-vector modulo),
// and U rows per thread are loaded before any of them is used (U x 16 B in flight per lane).
struct RowGeom {
  int tpr, rpi, cgroups;
};
// At most 32 threads (256 channels, 512 B of bf16) per row: wide tensors are split over grid.y
// channel groups, which multiplies the workgroups of the reduce passes without growing their
// [blocks][2][C] partials.
inline int max_tpr() { return 32; }
inline RowGeom row_geom(int C) {
  int c8 = C / 8;
  RowGeom g;
  const int cap = max_tpr();
  g.tpr = c8 < cap ? c8 : cap;
  // tpr must divide 256 for the row mapping; fall back to the largest divisor <= c8.
  while (kBlock % g.tpr != 0) --g.tpr;
  g.rpi = kBlock / g.tpr;
  g.cgroups = (c8 + g.tpr - 1) / g.tpr;
  return g;
}
using ReduceGeom = RowGeom;
inline ReduceGeom reduce_geom(int C) { return row_geom(C); }

// Apply-pass block -> (channel group, row chunk). With more channel groups than one (C > 8 * tpr)
// the launcher may use a flat grid (gridDim.y == 1) whose FASTEST index is the channel group, so
// the blocks that share a row range -- together covering whole rows -- run together and each row's
// bytes are streamed at once, instead of one channel slice of every row per pass over the tensor
// (blockIdx.y slowest): C 1024-2048 apply 3.8-4.4 -> 5.2 TB/s (profiles/round4_bn_apply_flat_grid_ab.txt).
struct BlkMap {
  int cg, bx, nb;
};
__device__ __forceinline__ BlkMap apply_block_map(int C, int tpr) {
  if (gridDim.y > 1) return {static_cast<int>(blockIdx.y), static_cast<int>(blockIdx.x), static_cast<int>(gridDim.x)};
  const int ncg = (C / 8 + tpr - 1) / tpr;
  return {static_cast<int>(blockIdx.x) % ncg, static_cast<int>(blockIdx.x) / ncg,
          static_cast<int>(gridDim.x) / ncg};
}

struct RowRange {
  int64_t begin, end;
};
// Rows of chunk `bx` out of `nb` equal contiguous chunks (each a multiple of rpi).
__device__ __forceinline__ RowRange chunk_rows(int64_t M, int rpi, int bx, int nb) {
  int64_t per = (M + nb - 1) / nb;
  per = (per + rpi - 1) / rpi * rpi;
  int64_t b = static_cast<int64_t>(bx) * per;
  int64_t e = b + per;
  if (b > M) b = M;
  if (e > M) e = M;
  return {b, e};
}

template <typename T>
__device__ __forceinline__ void st8(void* base, int64_t elem_off, const float (&v)[8]) {
  Vec8<T>::store(reinterpret_cast<char*>(base) + elem_off * Vec8<T>::bytes, v);
}

// Statistics pass. FWD: per-chunk (sum x, sum x^2); BWD: (sum dy', sum dy'*(x-mean)) with
// dy' = (dy [+ dy2]) masked by the forward's ReLU bit. Chunks are visited in DESCENDING order:
// the tensors' producer (a convolution, or the previous pass) wrote/read them ascending, so the
// rows it touched last are still in the 256 MB Infinity Cache when the first chunks run here;
// the apply pass then walks ascending and starts on the rows this pass read last.
// DUAL (backward only): a second BatchNorm input x2 whose output was ADDED before the ReLU
// (relu(bn(x) + bn2(x2)), the projection shortcut of a downsampling block) shares the masked
// upstream gradient dy'; the pass also reduces sum dy'*(x2-mean2) into partial2 (whose first
// statistic, sum dy', is the same as partial's).
template <typename T, bool BWD, int U, bool NT = false, bool DUAL = false>
__global__ __launch_bounds__(kBlock) void bn_reduce_kernel(
    const void* __restrict__ x, const void* __restrict__ dy, const void* __restrict__ dy2,
    const uint8_t* __restrict__ mask, const float* __restrict__ mean, int64_t M, int C, int tpr,
    int rpi, bool relu, float* __restrict__ partial, const void* __restrict__ x2,
    const float* __restrict__ mean2, float* __restrict__ partial2) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [rpi][tpr*(DUAL ? 24 : 16)]
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const int c = (blockIdx.y * tpr + lc) * 8;
  const bool active = c < C;
  const int bx = static_cast<int>(gridDim.x) - 1 - static_cast<int>(blockIdx.x);
  const RowRange rr = chunk_rows(M, rpi, bx, gridDim.x);
  float s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  float mu[8], mu2[8], q2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) q2[k] = 0.f;
  if (BWD && active) {
#pragma unroll
    for (int k = 0; k < 8; ++k) mu[k] = mean[c + k];
    if (DUAL) {
#pragma unroll
      for (int k = 0; k < 8; ++k) mu2[k] = mean2[c + k];
    }
  }
  if (active) {
    int64_t r = rr.begin + r0;
    for (; r + (U - 1) * rpi < rr.end; r += U * rpi) {
      Raw8<T> rx[U], rg[U], rg2[U], rx2[U];
      uint32_t mk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t off = (r + u * rpi) * C + c;
        rx[u] = NT ? ld8nt<T>(x, off) : ld8<T>(x, off);
        if (BWD) {
          rg[u] = NT ? ld8nt<T>(dy, off) : ld8<T>(dy, off);
          if (dy2) rg2[u] = NT ? ld8nt<T>(dy2, off) : ld8<T>(dy2, off);
          if (DUAL) rx2[u] = NT ? ld8nt<T>(x2, off) : ld8<T>(x2, off);
          mk[u] = relu ? mask[off >> 3] : 0xffu;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float xv[8];
        unpack8<T>(rx[u], xv);
        if (!BWD) {
#pragma unroll
          for (int k = 0; k < 8; ++k) { s[k] += xv[k]; q[k] = fmaf(xv[k], xv[k], q[k]); }
        } else {
          float g[8];
          unpack8<T>(rg[u], g);
          if (dy2) {
            float g2[8];
            unpack8<T>(rg2[u], g2);
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] += g2[k];
          }
          float x2v[8];
          if (DUAL) unpack8<T>(rx2[u], x2v);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float gk = ((mk[u] >> k) & 1u) ? g[k] : 0.f;
            s[k] += gk;
            q[k] = fmaf(gk, xv[k] - mu[k], q[k]);
            if (DUAL) q2[k] = fmaf(gk, x2v[k] - mu2[k], q2[k]);
          }
        }
      }
    }
    for (; r < rr.end; r += rpi) {
      const int64_t off = r * C + c;
      float xv[8];
      unpack8<T>(ld8<T>(x, off), xv);
      if (!BWD) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { s[k] += xv[k]; q[k] = fmaf(xv[k], xv[k], q[k]); }
      } else {
        float g[8];
        unpack8<T>(ld8<T>(dy, off), g);
        if (dy2) {
          float g2[8];
          unpack8<T>(ld8<T>(dy2, off), g2);
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] += g2[k];
        }
        if (relu) {
          const uint32_t m = mask[off >> 3];  // one ReLU bit per element, 8 channels per byte
#pragma unroll
          for (int k = 0; k < 8; ++k) g[k] = ((m >> k) & 1u) ? g[k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) { s[k] += g[k]; q[k] = fmaf(g[k], xv[k] - mu[k], q[k]); }
        if (DUAL) {
          float x2v[8];
          unpack8<T>(ld8<T>(x2, off), x2v);
#pragma unroll
          for (int k = 0; k < 8; ++k) q2[k] = fmaf(g[k], x2v[k] - mu2[k], q2[k]);
        }
      }
    }
  }
  // Combine the rpi row-groups that share channels through LDS: per lane 8 channels x
  // (sum, sum2 [, dual sum2]).
  constexpr int W = DUAL ? 24 : 16;
  const int width = tpr * W;
  float* mine = lds + r0 * width + lc * W;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mine[k] = s[k];
    mine[8 + k] = q[k];
    if (DUAL) mine[16 + k] = q2[k];
  }
  __syncthreads();
  for (int o = tid; o < width; o += kBlock) {
    float acc = 0.f;
    for (int r = 0; r < rpi; ++r) acc += lds[r * width + o];
    const int lco = o / W, k = o % W, stat = k >> 3;
    const int ch = (blockIdx.y * tpr + lco) * 8 + (k & 7);
    if (ch >= C) continue;
    const int64_t b2 = static_cast<int64_t>(bx) * 2;
    if (stat < 2) partial[(b2 + stat) * C + ch] = acc;
    if (DUAL && stat == 0) partial2[b2 * C + ch] = acc;
    if (DUAL && stat == 2) partial2[(b2 + 1) * C + ch] = acc;
  }
}

// Channel-parallel combine of the per-block partials: block = 256 threads = 8 channels x 32
// slices of the partial list, fp64 accumulation.
__device__ __forceinline__ void combine_partials(const float* __restrict__ partial, int B, int C,
                                                 double* red, double& s_out, double& q_out,
                                                 int& ch_out) {
  const int tid = threadIdx.x;
  const int cl = tid & 7, sl = tid >> 3;
  const int ch = blockIdx.x * 8 + cl;
  double s = 0.0, q = 0.0;
  if (ch < C) {
    // 4 independent partial rows in flight per thread (latency-bound otherwise)
    float fs[4] = {0.f, 0.f, 0.f, 0.f}, fq[4] = {0.f, 0.f, 0.f, 0.f};
    double ds[4] = {0.0, 0.0, 0.0, 0.0}, dq[4] = {0.0, 0.0, 0.0, 0.0};
    int b = sl;
    for (; b + 96 < B; b += 128) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        fs[u] = partial[(static_cast<int64_t>(b + 32 * u) * 2) * C + ch];
        fq[u] = partial[(static_cast<int64_t>(b + 32 * u) * 2 + 1) * C + ch];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { ds[u] += fs[u]; dq[u] += fq[u]; }
    }
    for (; b < B; b += 32) {
      ds[0] += partial[(static_cast<int64_t>(b) * 2) * C + ch];
      dq[0] += partial[(static_cast<int64_t>(b) * 2 + 1) * C + ch];
    }
    s = (ds[0] + ds[1]) + (ds[2] + ds[3]);
    q = (dq[0] + dq[1]) + (dq[2] + dq[3]);
  }
  red[tid] = s;
  red[256 + tid] = q;
  __syncthreads();
  if (sl == 0) {
    for (int j = 1; j < 32; ++j) { s += red[j * 8 + cl]; q += red[256 + j * 8 + cl]; }
  }
  s_out = s; q_out = q; ch_out = ch;
}

__global__ __launch_bounds__(kBlock) void bn_finalize_fwd_kernel(
    const float* __restrict__ partial, int B, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ running_mean,
    float* __restrict__ running_var, float momentum, float eps, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, float* __restrict__ scale, float* __restrict__ shift,
    int64_t* __restrict__ num_batches) {
  __shared__ double red[512];
  double s, q;
  int ch;
  combine_partials(partial, B, C, red, s, q, ch);
  if ((threadIdx.x >> 3) == 0 && ch < C) {
    const double mean = s / static_cast<double>(M);
    double var = q / static_cast<double>(M) - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = static_cast<float>(1.0 / sqrt(var + static_cast<double>(eps)));
    const float g = gamma ? gamma[ch] : 1.f, bt = beta ? beta[ch] : 0.f;
    save_mean[ch] = static_cast<float>(mean);
    save_invstd[ch] = invstd;
    scale[ch] = g * invstd;
    shift[ch] = bt - static_cast<float>(mean) * g * invstd;
    if (running_mean) {
      const double unbiased = M > 1 ? var * static_cast<double>(M) / static_cast<double>(M - 1) : var;
      running_mean[ch] = (1.f - momentum) * running_mean[ch] + momentum * static_cast<float>(mean);
      running_var[ch] = (1.f - momentum) * running_var[ch] + momentum * static_cast<float>(unbiased);
    }
  }
  if (num_batches && blockIdx.x == 0 && threadIdx.x == 0) *num_batches += 1;
}

__global__ __launch_bounds__(kBlock) void bn_finalize_bwd_kernel(
    const float* __restrict__ partial, int B, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ invstd, float* __restrict__ dgamma,
    float* __restrict__ dbeta, bool accumulate, float* __restrict__ coef /* [3][C] */) {
  __shared__ double red[512];
  double s, q;
  int ch;
  combine_partials(partial, B, C, red, s, q, ch);
  if ((threadIdx.x >> 3) == 0 && ch < C) {
    const float is = invstd[ch];
    const float g = gamma ? gamma[ch] : 1.f;
    const float sdy = static_cast<float>(s);
    const float sdyx = static_cast<float>(q);  // sum dy' * (x - mean)
    // accumulate: dgamma/dbeta are the parameters' .grad (flat-buffer views) -- add in place so
    // autograd never runs a separate AccumulateGrad add for them.
    if (dgamma) dgamma[ch] = accumulate ? dgamma[ch] + sdyx * is : sdyx * is;
    if (dbeta) dbeta[ch] = accumulate ? dbeta[ch] + sdy : sdy;
    const float invM = 1.f / static_cast<float>(M);
    const float k1 = g * is;
    const float k2 = -k1 * is * is * sdyx * invM;
    const float k3 = -k1 * sdy * invM - k2 * mean[ch];
    coef[ch] = k1;
    coef[C + ch] = k2;
    coef[2 * C + ch] = k3;
  }
}

// y = act(x*scale + shift [+ res]) (+ ReLU bitmask), row-tile mapping, U rows in flight per lane.
// Bit k of mask byte (row*C + c)/8 is the ReLU decision of channel c+k.
// res2_scale / res2_shift (optional): the residual is itself normalised in this pass,
// res -> res*res2_scale + res2_shift (a projection shortcut's BatchNorm, never materialised).
template <typename T, int U>
__global__ __launch_bounds__(kBlock) void bn_apply_fwd_kernel(
    const void* __restrict__ x, const void* __restrict__ res, void* __restrict__ y,
    const float* __restrict__ scale, const float* __restrict__ shift, int64_t M, int C, int tpr,
    int rpi, bool relu, uint8_t* __restrict__ mask, const float* __restrict__ res2_scale,
    const float* __restrict__ res2_shift) {
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const BlkMap bm = apply_block_map(C, tpr);
  const int c = (bm.cg * tpr + lc) * 8;
  if (c >= C) return;
  const RowRange rr = chunk_rows(M, rpi, bm.bx, bm.nb);
  float a[8], b[8];
  {
    const float4 a0 = *reinterpret_cast<const float4*>(scale + c);
    const float4 a1 = *reinterpret_cast<const float4*>(scale + c + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(shift + c);
    const float4 b1 = *reinterpret_cast<const float4*>(shift + c + 4);
    a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w; a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
    b[0] = b0.x; b[1] = b0.y; b[2] = b0.z; b[3] = b0.w; b[4] = b1.x; b[5] = b1.y; b[6] = b1.z; b[7] = b1.w;
  }
  float a2[8], b2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a2[k] = res2_scale ? res2_scale[c + k] : 1.f;
    b2[k] = res2_shift ? res2_shift[c + k] : 0.f;
  }
  auto finish = [&](int64_t off, float (&o)[8]) {
    if (relu) {
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        bits |= (o[k] > 0.f ? 1u : 0u) << k;
        o[k] = fmaxf(o[k], 0.f);
      }
      if (mask) mask[off >> 3] = static_cast<uint8_t>(bits);
    }
    st8<T>(y, off, o);
  };
  int64_t r = rr.begin + r0;
  for (; r + (U - 1) * rpi < rr.end; r += U * rpi) {
    Raw8<T> rx[U], rres[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * rpi) * C + c;
      rx[u] = ld8<T>(x, off);
      if (res) rres[u] = ld8<T>(res, off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * rpi) * C + c;
      float xv[8], o[8];
      unpack8<T>(rx[u], xv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(xv[k], a[k], b[k]);
      if (res) {
        float rv[8];
        unpack8<T>(rres[u], rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] += fmaf(rv[k], a2[k], b2[k]);
      }
      finish(off, o);
    }
  }
  for (; r < rr.end; r += rpi) {
    const int64_t off = r * C + c;
    float xv[8], o[8];
    unpack8<T>(ld8<T>(x, off), xv);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(xv[k], a[k], b[k]);
    if (res) {
      float rv[8];
      unpack8<T>(ld8<T>(res, off), rv);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] += fmaf(rv[k], a2[k], b2[k]);
    }
    finish(off, o);
  }
}

// dx = k1*dy' + k2*x + k3 with dy' = (dy [+ dy2]) masked by the ReLU bit; dres = dy' when the
// forward fused a residual add. Row-tile mapping, coefficients held in registers.
// DUAL: also dx2 = k1b*dy' + k2b*x2 + k3b for the second BatchNorm input that was added before
// the ReLU (coef2 = its [3][C] coefficients); dres is not written then (dy' is consumed here).
template <typename T, int U, bool DUAL = false>
__global__ __launch_bounds__(kBlock) void bn_apply_bwd_kernel(
    const void* __restrict__ dy, const void* __restrict__ dy2, const uint8_t* __restrict__ mask,
    const void* __restrict__ x, const float* __restrict__ coef, void* __restrict__ dx,
    void* __restrict__ dres, int64_t M, int C, int tpr, int rpi, bool relu,
    const void* __restrict__ x2, const float* __restrict__ coef2, void* __restrict__ dx2) {
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const BlkMap bm = apply_block_map(C, tpr);
  const int c = (bm.cg * tpr + lc) * 8;
  if (c >= C) return;
  const RowRange rr = chunk_rows(M, rpi, bm.bx, bm.nb);
  float k1[8], k2[8], k3[8], j1[8], j2[8], j3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { k1[k] = coef[c + k]; k2[k] = coef[C + c + k]; k3[k] = coef[2 * C + c + k]; }
  if (DUAL) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { j1[k] = coef2[c + k]; j2[k] = coef2[C + c + k]; j3[k] = coef2[2 * C + c + k]; }
  }
  auto body = [&](int64_t off, float (&g)[8], const float (&xv)[8], const float (&x2v)[8], uint32_t m) {
    if (relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = ((m >> k) & 1u) ? g[k] : 0.f;
    }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(k1[k], g[k], fmaf(k2[k], xv[k], k3[k]));
    st8<T>(dx, off, o);
    if (DUAL) {
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(j1[k], g[k], fmaf(j2[k], x2v[k], j3[k]));
      st8<T>(dx2, off, o);
    } else if (dres) {
      st8<T>(dres, off, g);
    }
  };
  int64_t r = rr.begin + r0;
  for (; r + (U - 1) * rpi < rr.end; r += U * rpi) {
    Raw8<T> rg[U], rg2[U], rx[U], rx2[U];
    uint32_t mk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * rpi) * C + c;
      rg[u] = ld8<T>(dy, off);
      if (dy2) rg2[u] = ld8<T>(dy2, off);
      rx[u] = ld8<T>(x, off);
      if (DUAL) rx2[u] = ld8<T>(x2, off);
      mk[u] = relu ? mask[off >> 3] : 0xffu;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * rpi) * C + c;
      float g[8], xv[8], x2v[8];
      unpack8<T>(rg[u], g);
      if (dy2) {
        float g2[8];
        unpack8<T>(rg2[u], g2);
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] += g2[k];
      }
      unpack8<T>(rx[u], xv);
      if (DUAL) unpack8<T>(rx2[u], x2v);
      body(off, g, xv, x2v, mk[u]);
    }
  }
  for (; r < rr.end; r += rpi) {
    const int64_t off = r * C + c;
    float g[8], xv[8], x2v[8];
    unpack8<T>(ld8<T>(dy, off), g);
    if (dy2) {
      float g2[8];
      unpack8<T>(ld8<T>(dy2, off), g2);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += g2[k];
    }
    unpack8<T>(ld8<T>(x, off), xv);
    if (DUAL) unpack8<T>(ld8<T>(x2, off), x2v);
    body(off, g, xv, x2v, relu ? mask[off >> 3] : 0xffu);
  }
}

constexpr int kUReduceFwd = 8;  // rows in flight per lane: 8 x 16 B (x)
constexpr int kUReduceBwd = 4;  // 4 x (16 B dy + 16 B x [+ 16 B dy2] + 1 B mask)
constexpr int kUApply = 4;

struct ReduceTuning {
  int64_t elems_per_block, min_blocks, max_blocks, cap_floats;
};
inline const ReduceTuning& reduce_tuning() {
  static const ReduceTuning t{32768, 256, 2048, int64_t(1) << 18};
  return t;
}

inline int reduce_blocks(int64_t M, int C, const ReduceGeom& g) {
  // ~elems_per_block elements per workgroup, clamped to [min_blocks, max_blocks] in x (x cgroups
  // in y); the per-block partials (B x 2 x C floats, re-read by the finalize pass) are capped at
  // 2^18 floats per statistic, and every block gets at least one row-iteration.
  const ReduceTuning& t = reduce_tuning();
  int64_t total = M * static_cast<int64_t>(C);
  int64_t b = (total + t.elems_per_block - 1) / t.elems_per_block;
  if (b < t.min_blocks) b = t.min_blocks;
  if (b > t.max_blocks) b = t.max_blocks;
  const int64_t cap = std::max<int64_t>(64, t.cap_floats / C);
  if (b > cap) b = cap;
  int64_t rows_iter = (M + g.rpi - 1) / g.rpi;
  if (b > rows_iter) b = rows_iter;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

// Apply-pass geometry. Large tensors (>= 32M elements) run as an almost one-shot grid: 2 rows
// in flight per lane and no workgroup cap (each workgroup does 2 unrolled iterations), which
// streams at 5.4-5.7 TB/s on the bs-1024 ResNet-50 shapes against 4.9-5.3 for the old 8-per-CU
// grid with 4 rows per lane (tools/bench_bn.py, profiles/round4_bn_apply_oneshot_ab.txt; the
// one-shot copy ceiling of this box is 6.16 TB/s, profiles/round4_hbm_streaming_ceilings.txt);
// smaller tensors keep 4 rows per lane and the 2048-workgroup cap.
struct ApplyTuning {
  int u, max_blocks;
};
inline ApplyTuning apply_tuning(int64_t elems) {
  if (elems >= (int64_t{1} << 25)) return {2, 1 << 30};
  return {kUApply, 2048};
}

// Workgroups (in x) for the apply passes, each with >= 2 unrolled iterations.
inline int apply_blocks(int64_t M, const RowGeom& g, const ApplyTuning& t) {
  int64_t b = (M + static_cast<int64_t>(g.rpi) * t.u * 2 - 1) / (static_cast<int64_t>(g.rpi) * t.u * 2);
  if (b > t.max_blocks) b = t.max_blocks;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

inline dim3 apply_grid(int64_t M, const RowGeom& g, const ApplyTuning& t) {
  const int bx = apply_blocks(M, g, t);
  if (g.cgroups > 1 && static_cast<int64_t>(bx) * g.cgroups < (int64_t{1} << 31))
    return dim3(bx * g.cgroups, 1);  // see apply_block_map
  return dim3(bx, g.cgroups);
}

// Reduce-pass variant: the statistics passes stream with NONTEMPORAL loads by default (-3% on
// the bs-1024 ResNet-50 BN shapes, fwd+bwd 32.3 -> 31.4 ms per step in tools/bench_bn.py,
// profiles/round4_bn_reduce_nt_ab.txt).

template <typename T>
void launch_reduce(bool bwd, const void* x, const void* dy, const void* dy2, const uint8_t* y,
                   const float* mean,
                   int64_t M, int C, bool relu, float* partial, int B, const ReduceGeom& g,
                   hipStream_t st, const void* x2 = nullptr, const float* mean2 = nullptr,
                   float* partial2 = nullptr) {
  dim3 grid(B, g.cgroups);
  const bool dual = bwd && x2 != nullptr;
  size_t lds = static_cast<size_t>(g.rpi) * g.tpr * (dual ? 24 : 16) * sizeof(float);
#define DCA_RED(BW, UU, DU)                                                                       \
  hipLaunchKernelGGL((bn_reduce_kernel<T, BW, UU, true, DU>), grid, dim3(kBlock), lds, st, x, dy, dy2, \
                     y, mean, M, C, g.tpr, g.rpi, relu, partial, x2, mean2, partial2)
  if (dual) DCA_RED(true, kUReduceBwd, true);
  else if (bwd) DCA_RED(true, kUReduceBwd, false);
  else DCA_RED(false, kUReduceFwd, false);
#undef DCA_RED
}

template <typename T>
void launch_apply_fwd(const void* x, const void* res, void* y, const float* scale,
                      const float* shift, int64_t M, int C, bool relu, uint8_t* mask,
                      hipStream_t st, const float* res_scale = nullptr,
                      const float* res_shift = nullptr) {
  const RowGeom g = row_geom(C);
  const ApplyTuning t = apply_tuning(M * C);
  const dim3 grid = apply_grid(M, g, t);
  switch (t.u) {
    case 2: hipLaunchKernelGGL((bn_apply_fwd_kernel<T, 2>), grid, dim3(kBlock), 0, st, x, res, y, scale, shift, M, C, g.tpr, g.rpi, relu, mask, res_scale, res_shift); break;
    case 8: hipLaunchKernelGGL((bn_apply_fwd_kernel<T, 8>), grid, dim3(kBlock), 0, st, x, res, y, scale, shift, M, C, g.tpr, g.rpi, relu, mask, res_scale, res_shift); break;
    default: hipLaunchKernelGGL((bn_apply_fwd_kernel<T, kUApply>), grid, dim3(kBlock), 0, st, x, res, y, scale, shift, M, C, g.tpr, g.rpi, relu, mask, res_scale, res_shift); break;
  }
}

template <typename T>
void launch_apply_bwd(const void* dy, const void* dy2, const uint8_t* mask, const void* x,
                      const float* coef, void* dx, void* dres, int64_t M, int C, bool relu,
                      hipStream_t st, const void* x2 = nullptr, const float* coef2 = nullptr,
                      void* dx2 = nullptr) {
  const RowGeom g = row_geom(C);
  const ApplyTuning t = apply_tuning(M * C);
  const dim3 grid = apply_grid(M, g, t);
  if (x2 != nullptr) {  // dual: fixed 2 rows in flight (three 16-B loads + two stores per row)
    hipLaunchKernelGGL((bn_apply_bwd_kernel<T, 2, true>), grid, dim3(kBlock), 0, st, dy, dy2, mask, x, coef, dx, dres, M, C, g.tpr, g.rpi, relu, x2, coef2, dx2);
    return;
  }
  switch (t.u) {
    case 2: hipLaunchKernelGGL((bn_apply_bwd_kernel<T, 2>), grid, dim3(kBlock), 0, st, dy, dy2, mask, x, coef, dx, dres, M, C, g.tpr, g.rpi, relu, x2, coef2, dx2); break;
    case 8: hipLaunchKernelGGL((bn_apply_bwd_kernel<T, 8>), grid, dim3(kBlock), 0, st, dy, dy2, mask, x, coef, dx, dres, M, C, g.tpr, g.rpi, relu, x2, coef2, dx2); break;
    default: hipLaunchKernelGGL((bn_apply_bwd_kernel<T, kUApply>), grid, dim3(kBlock), 0, st, dy, dy2, mask, x, coef, dx, dres, M, C, g.tpr, g.rpi, relu, x2, coef2, dx2); break;
  }
}

// ------------------------------------------------------------------ stem: BN + ReLU + MaxPool(3,2,1)
// ResNet stem fusion: the pre-pool activation (N x 112 x 112 x 64 for ImageNet -- the largest
// tensor of the network) is never written. Forward writes the pooled output and one byte per
// pooled element: window slot (0..8) of the max | 0x10 if the max is > 0 (i.e. the ReLU passed).
// Backward re-derives the pre-pool gradient on the fly by GATHER (each input position is covered
// by at most 2x2 pooling windows) inside the BN-backward reduce/apply passes, instead of a zero-fill
// + scatter max-pool backward followed by a full-size BN backward read.
struct PoolGeom {
  int H, W, Ho, Wo;
};

// Forward in quad form: one thread per 2x2 block of pooled outputs (ho = 2hq + a, wo = 2wq + b)
// and 8 channels. Their windows cover input rows 4hq-1 .. 4hq+3 and columns 4wq-1 .. 4wq+3: 25 loads
// for 4 outputs instead of 36, each input vector applied to every window that contains it. Visiting
// the 5x5 inputs row-major gives every window its taps in (kh, kw) order, so "first maximum wins"
// is unchanged.
template <typename T>
__global__ __launch_bounds__(kBlock) void bn_relu_pool_fwd_quad_kernel(
    const void* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
    void* __restrict__ y, uint8_t* __restrict__ idx, int64_t nthr, int C, PoolGeom g) {
  const int c8 = C / 8;
  const int Hq = (g.Ho + 1) / 2, Wq = (g.Wo + 1) / 2;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < nthr;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(t % c8) * 8;
    const int64_t o = t / c8;  // (n, hq, wq)
    const int wq = static_cast<int>(o % Wq);
    const int hq = static_cast<int>((o / Wq) % Hq);
    const int64_t n = o / (static_cast<int64_t>(Wq) * Hq);
    float a8[8], b8[8], best[4][8];
    uint32_t slot[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { a8[k] = scale[c + k]; b8[k] = shift[c + k]; }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) { best[q][k] = 0.f; slot[q][k] = 0xff; }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int h = 4 * hq - 1 + i;
      if (h < 0 || h >= g.H) continue;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const int w = 4 * wq - 1 + j;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        Vec8<T>::load(reinterpret_cast<const char*>(x) + (((n * g.H + h) * g.W + w) * C + c) * Vec8<T>::bytes, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaxf(fmaf(v[k], a8[k], b8[k]), 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kh = i - 2 * (q >> 1), kw = j - 2 * (q & 1);
          if (kh < 0 || kh > 2 || kw < 0 || kw > 2) continue;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (slot[q][k] == 0xff || v[k] > best[q][k]) { best[q][k] = v[k]; slot[q][k] = kh * 3 + kw; }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ho = 2 * hq + (q >> 1), wo = 2 * wq + (q & 1);
      if (ho >= g.Ho || wo >= g.Wo) continue;
      const int64_t ot = ((n * g.Ho + ho) * g.Wo + wo) * c8 + c / 8;  // output vector index
      Vec8<T>::store(reinterpret_cast<char*>(y) + ot * 8 * Vec8<T>::bytes, best[q]);
      if (idx) {
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) lo |= ((slot[q][k] | (best[q][k] > 0.f ? 0x10u : 0u)) & 0xffu) << (8 * k);
#pragma unroll
        for (int k = 0; k < 4; ++k) hi |= ((slot[q][4 + k] | (best[q][4 + k] > 0.f ? 0x10u : 0u)) & 0xffu) << (8 * k);
        *reinterpret_cast<uint2*>(idx + ot * 8) = make_uint2(lo, hi);
      }
    }
  }
}

// BN-backward statistics and apply passes of the stem (BN + ReLU + max-pool), in quad form: one
// thread per 2x2 block of pre-pool positions (rows 2hb, 2hb+1, columns 2wb, 2wb+1) and 8 channels. Such a block is covered by exactly the pooled windows
// (hb + a, wb + b), a, b in {0, 1} (3x3 / stride 2 / padding 1), so the thread loads those 4
// (gradient, slot byte) pairs ONCE for its 4 positions -- the per-position gather loaded them 4
// times (9 loads per position -> 3): 0.95 -> 0.45 ms and 1.10 -> 0.75 ms for the bs-1024 stem (with the prefetch below),
// +0.6 % on the ResNet-50 step (profiles/round5_stem_pool_bwd_quad_ab.txt).
// The loads of one quad (issued one quad ahead of their use: the passes are latency-bound at 4
// waves per SIMD, so the next quad's 12 loads stay in flight while this one is computed).
template <typename T>
struct QuadLoads {
  Raw8<T> x[4], dy[4];
  uint2 ib[4];
};

// quad q -> (n, hb, wb); Q = N * Hb * Wb < 2^31 (host check)
__device__ __forceinline__ void pool_quad(int64_t q, int Hb, int Wb, int64_t& n, int& hb, int& wb) {
  const uint32_t qu = static_cast<uint32_t>(q);
  const uint32_t nh = qu / static_cast<uint32_t>(Wb);
  wb = static_cast<int>(qu - nh * static_cast<uint32_t>(Wb));
  const uint32_t nn = nh / static_cast<uint32_t>(Hb);
  hb = static_cast<int>(nh - nn * static_cast<uint32_t>(Hb));
  n = nn;
}

template <typename T>
__device__ __forceinline__ void load_quad(const void* __restrict__ x, const void* __restrict__ dyp,
                                          const uint8_t* __restrict__ idx, int64_t n, int hb, int wb,
                                          int c, int C, const PoolGeom& g, QuadLoads<T>& L) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int h = 2 * hb + (p >> 1), w = 2 * wb + (p & 1);
    if (h < g.H && w < g.W) L.x[p] = ld8<T>(x, ((n * g.H + h) * g.W + w) * C + c);
    const int ho = hb + (p >> 1), wo = wb + (p & 1);
    L.ib[p] = make_uint2(0, 0);  // no window -> no slot matches
    if (ho < g.Ho && wo < g.Wo) {
      const int64_t off = ((n * g.Ho + ho) * g.Wo + wo) * C + c;
      L.ib[p] = *reinterpret_cast<const uint2*>(idx + off);
      L.dy[p] = ld8<T>(dyp, off);
    }
  }
}

// Pre-pool gradient of quad position p = (dh, dw), i.e. (2hb + dh, 2wb + dw): that position is
// tap (kh, kw) = (dh + 1 - 2a, dw + 1 - 2b) of pooled window (hb + a, wb + b); it receives the
// window's gradient when the window's slot byte names the tap with the ReLU bit set.
template <typename T, int P>
__device__ __forceinline__ void quad_grad(const QuadLoads<T>& L, float (&gp)[8]) {
  constexpr int dh = P >> 1, dw = P & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) gp[k] = 0.f;
#pragma unroll
  for (int ab = 0; ab < 4; ++ab) {
    const int kh = dh + 1 - 2 * (ab >> 1), kw = dw + 1 - 2 * (ab & 1);
    if (kh < 0 || kh > 2 || kw < 0 || kw > 2) continue;
    const uint32_t want = static_cast<uint32_t>(kh * 3 + kw) | 0x10u;
    float d[8];
    unpack8<T>(L.dy[ab], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t byte = ((k < 4 ? L.ib[ab].x : L.ib[ab].y) >> (8 * (k & 3))) & 0xffu;
      if (byte == want) gp[k] += d[k];
    }
  }
}

// the 4 positions of a quad, unrolled with compile-time P
template <typename F>
__device__ __forceinline__ void for_quad(F&& f) {
  f(std::integral_constant<int, 0>{});
  f(std::integral_constant<int, 1>{});
  f(std::integral_constant<int, 2>{});
  f(std::integral_constant<int, 3>{});
}

template <typename T>
__global__ __launch_bounds__(kBlock) void bn_pool_reduce_bwd_quad_kernel(
    const void* __restrict__ x, const void* __restrict__ dyp, const uint8_t* __restrict__ idx,
    const float* __restrict__ mean, int64_t Qn, int C, int tpr, int rpi, PoolGeom g,
    float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const int c = (blockIdx.y * tpr + lc) * 8;
  const bool active = c < C;
  const int bx = static_cast<int>(gridDim.x) - 1 - static_cast<int>(blockIdx.x);
  const RowRange rr = chunk_rows(Qn, rpi, bx, gridDim.x);
  const int Hb = (g.H + 1) / 2, Wb = (g.W + 1) / 2;
  float s[8], q[8], mu[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; mu[k] = active ? mean[c + k] : 0.f; }
  if (active && rr.begin + r0 < rr.end) {
    int64_t n;
    int hb, wb;
    pool_quad(rr.begin + r0, Hb, Wb, n, hb, wb);
    QuadLoads<T> nxt;
    load_quad<T>(x, dyp, idx, n, hb, wb, c, C, g, nxt);
    for (int64_t r = rr.begin + r0; r < rr.end; r += rpi) {
      const QuadLoads<T> cur = nxt;
      const int chb = hb, cwb = wb;
      if (r + rpi < rr.end) {
        pool_quad(r + rpi, Hb, Wb, n, hb, wb);
        load_quad<T>(x, dyp, idx, n, hb, wb, c, C, g, nxt);
      }
      for_quad([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        if (2 * chb + (p >> 1) < g.H && 2 * cwb + (p & 1) < g.W) {
          float gp[8], xv[8];
          quad_grad<T, p>(cur, gp);
          unpack8<T>(cur.x[p], xv);
#pragma unroll
          for (int k = 0; k < 8; ++k) { s[k] += gp[k]; q[k] = fmaf(gp[k], xv[k] - mu[k], q[k]); }
        }
      });
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
    const int lco = o / 16, k = o % 16;
    const int ch = (blockIdx.y * tpr + lco) * 8 + (k & 7);
    if (ch < C) partial[(static_cast<int64_t>(bx) * 2 + (k >> 3)) * C + ch] = acc;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void bn_pool_apply_bwd_quad_kernel(
    const void* __restrict__ x, const void* __restrict__ dyp, const uint8_t* __restrict__ idx,
    const float* __restrict__ coef, void* __restrict__ dx, int64_t Qn, int C, int tpr, int rpi,
    PoolGeom g) {
  const int tid = threadIdx.x;
  const int lc = tid % tpr, r0 = tid / tpr;
  const BlkMap bm = apply_block_map(C, tpr);
  const int c = (bm.cg * tpr + lc) * 8;
  if (c >= C) return;
  const RowRange rr = chunk_rows(Qn, rpi, bm.bx, bm.nb);
  if (rr.begin + r0 >= rr.end) return;
  const int Hb = (g.H + 1) / 2, Wb = (g.W + 1) / 2;
  float k1[8], k2[8], k3[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { k1[k] = coef[c + k]; k2[k] = coef[C + c + k]; k3[k] = coef[2 * C + c + k]; }
  int64_t n;
  int hb, wb;
  pool_quad(rr.begin + r0, Hb, Wb, n, hb, wb);
  QuadLoads<T> nxt;
  load_quad<T>(x, dyp, idx, n, hb, wb, c, C, g, nxt);
  for (int64_t r = rr.begin + r0; r < rr.end; r += rpi) {
    const QuadLoads<T> cur = nxt;
    const int64_t cn = n;
    const int chb = hb, cwb = wb;
    if (r + rpi < rr.end) {
      pool_quad(r + rpi, Hb, Wb, n, hb, wb);
      load_quad<T>(x, dyp, idx, n, hb, wb, c, C, g, nxt);
    }
    for_quad([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      const int h = 2 * chb + (p >> 1), w = 2 * cwb + (p & 1);
      if (h < g.H && w < g.W) {
        float gp[8], xv[8], o[8];
        quad_grad<T, p>(cur, gp);
        unpack8<T>(cur.x[p], xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf(k1[k], gp[k], fmaf(k2[k], xv[k], k3[k]));
        st8<T>(dx, ((cn * g.H + h) * g.W + w) * C + c, o);
      }
    });
  }
}

// Backward of a global average pool over an NHWC tensor: dx[n, hw, c] = g[n, c] * inv_hw,
// written at streaming bandwidth (16 B per lane) instead of an expand + divide.
template <typename T>
__global__ __launch_bounds__(kBlock) void spatial_mean_bwd_kernel(const void* __restrict__ g,
                                                                 void* __restrict__ dx, int64_t nvec,
                                                                 int c8, int hw, float inv_hw) {
  const uint32_t stride = gridDim.x * blockDim.x, n = static_cast<uint32_t>(nvec);
  for (uint32_t v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += stride) {
    const uint32_t row = v / static_cast<uint32_t>(c8);
    const uint32_t cv = v - row * static_cast<uint32_t>(c8);
    const uint32_t img = row / static_cast<uint32_t>(hw);
    float gv[8];
    unpack8<T>(ld8<T>(g, (static_cast<int64_t>(img) * c8 + cv) * 8), gv);
#pragma unroll
    for (int k = 0; k < 8; ++k) gv[k] *= inv_hw;
    st8<T>(dx, static_cast<int64_t>(v) * 8, gv);
  }
}

}  // namespace

// Workspace floats needed by bn_forward_train / bn_backward_train for (M, C).
int64_t bn_workspace_floats(int64_t M, int C) {
  ReduceGeom g = reduce_geom(C);
  int B = reduce_blocks(M, C, g);
  return static_cast<int64_t>(B) * 2 * C + 4 * static_cast<int64_t>(C);
}

// Per-channel (scale, shift) of a training-mode forward: statistics pass over x (unless the
// producer already reduced them into given_partials, e.g. a convolution epilogue in the same
// [B][2][C] layout), then the fp64 finalize (running stats, saved mean / invstd). Returns the
// scale pointer inside workspace; shift = scale + C.
static float* forward_affine_from_stats(BnDtype dt, const void* x, int64_t M, int C,
                                        const float* gamma, const float* beta,
                                        float* running_mean, float* running_var, float momentum,
                                        float eps, float* save_mean, float* save_invstd,
                                        int64_t* num_batches, float* workspace,
                                        const float* given_partials, int given_blocks,
                                        hipStream_t st) {
  const float* partial = given_partials;
  int B = given_blocks;
  float* scale = workspace;
  if (given_partials == nullptr) {
    ReduceGeom g = reduce_geom(C);
    B = reduce_blocks(M, C, g);
    float* part = workspace;
    scale = workspace + static_cast<int64_t>(B) * 2 * C;
    switch (dt) {
      case BnDtype::kBF16: launch_reduce<BF16>(false, x, nullptr, nullptr, nullptr, nullptr, M, C, false, part, B, g, st); break;
      case BnDtype::kF16: launch_reduce<F16>(false, x, nullptr, nullptr, nullptr, nullptr, M, C, false, part, B, g, st); break;
      default: launch_reduce<F32>(false, x, nullptr, nullptr, nullptr, nullptr, M, C, false, part, B, g, st); break;
    }
    partial = part;
  }
  float* shift = scale + C;
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3((C + 7) / 8), dim3(kBlock), 0, st, partial, B,
                     C, M, gamma, beta, running_mean, running_var, momentum, eps, save_mean,
                     save_invstd, scale, shift, num_batches);
  return scale;
}

void bn_forward_train(BnDtype dt, const void* x, const void* res, void* y, int64_t M, int C,
                      const float* gamma, const float* beta, float* running_mean,
                      float* running_var, float momentum, float eps, bool relu, float* save_mean,
                      float* save_invstd, int64_t* num_batches, uint8_t* mask, float* workspace,
                      const float* given_partials, int given_blocks, hipStream_t st) {
  const float* scale = forward_affine_from_stats(dt, x, M, C, gamma, beta, running_mean, running_var,
                                                 momentum, eps, save_mean, save_invstd, num_batches,
                                                 workspace, given_partials, given_blocks, st);
  const float* shift = scale + C;
  switch (dt) {
    case BnDtype::kBF16: launch_apply_fwd<BF16>(x, res, y, scale, shift, M, C, relu, mask, st); break;
    case BnDtype::kF16: launch_apply_fwd<F16>(x, res, y, scale, shift, M, C, relu, mask, st); break;
    default: launch_apply_fwd<F32>(x, res, y, scale, shift, M, C, relu, mask, st); break;
  }
}

// act(bn(x) + bn2(x2)): a downsampling ResNet block's main-branch BatchNorm and its projection
// shortcut's BatchNorm in ONE apply pass -- the shortcut's normalised tensor is never written
// (both statistics are finalised first; x2 is read once, inside the apply).
void bn_forward_train_dual(BnDtype dt, const void* x, const void* x2, void* y, int64_t M, int C,
                           const float* gamma, const float* beta, float* running_mean,
                           float* running_var, const float* gamma2, const float* beta2,
                           float* running_mean2, float* running_var2, float momentum, float eps,
                           bool relu, float* save_mean, float* save_invstd, float* save_mean2,
                           float* save_invstd2, int64_t* num_batches, int64_t* num_batches2,
                           uint8_t* mask, float* workspace, float* workspace2,
                           const float* given_partials, int given_blocks,
                           const float* given_partials2, int given_blocks2, hipStream_t st) {
  const float* scale = forward_affine_from_stats(dt, x, M, C, gamma, beta, running_mean, running_var,
                                                 momentum, eps, save_mean, save_invstd, num_batches,
                                                 workspace, given_partials, given_blocks, st);
  const float* scale2 = forward_affine_from_stats(dt, x2, M, C, gamma2, beta2, running_mean2,
                                                  running_var2, momentum, eps, save_mean2,
                                                  save_invstd2, num_batches2, workspace2,
                                                  given_partials2, given_blocks2, st);
  switch (dt) {
    case BnDtype::kBF16: launch_apply_fwd<BF16>(x, x2, y, scale, scale + C, M, C, relu, mask, st, scale2, scale2 + C); break;
    case BnDtype::kF16: launch_apply_fwd<F16>(x, x2, y, scale, scale + C, M, C, relu, mask, st, scale2, scale2 + C); break;
    default: launch_apply_fwd<F32>(x, x2, y, scale, scale + C, M, C, relu, mask, st, scale2, scale2 + C); break;
  }
}

// Inference-mode forward with precomputed per-channel scale/shift (fp32, [C] each).
void bn_forward_affine(BnDtype dt, const void* x, const void* res, void* y, int64_t M, int C,
                       const float* scale, const float* shift, bool relu, hipStream_t st) {
  uint8_t* mask = nullptr;
  switch (dt) {
    case BnDtype::kBF16: launch_apply_fwd<BF16>(x, res, y, scale, shift, M, C, relu, mask, st); break;
    case BnDtype::kF16: launch_apply_fwd<F16>(x, res, y, scale, shift, M, C, relu, mask, st); break;
    default: launch_apply_fwd<F32>(x, res, y, scale, shift, M, C, relu, mask, st); break;
  }
}

void bn_backward_train(BnDtype dt, const void* dy, const void* dy2, const uint8_t* y, const void* x,
                       int64_t M, int C,
                       const float* gamma, const float* save_mean, const float* save_invstd,
                       bool relu, void* dx, void* dres, float* dgamma, float* dbeta,
                       bool accumulate_dw, float* workspace, hipStream_t st,
                       const float* given_partials, int given_blocks) {
  ReduceGeom g = reduce_geom(C);
  int B = reduce_blocks(M, C, g);
  float* partial = workspace;
  float* coef = workspace + static_cast<int64_t>(B) * 2 * C;  // [3][C]
  if (given_partials != nullptr) {  // statistics reduced by dy's producer (conv dgrad epilogue)
    B = given_blocks;
    coef = workspace;
  } else {
    switch (dt) {
      case BnDtype::kBF16: launch_reduce<BF16>(true, x, dy, dy2, y, save_mean, M, C, relu, partial, B, g, st); break;
      case BnDtype::kF16: launch_reduce<F16>(true, x, dy, dy2, y, save_mean, M, C, relu, partial, B, g, st); break;
      default: launch_reduce<F32>(true, x, dy, dy2, y, save_mean, M, C, relu, partial, B, g, st); break;
    }
  }
  const float* stats = given_partials != nullptr ? given_partials : partial;
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 7) / 8), dim3(kBlock), 0, st, stats, B,
                     C, M, gamma, save_mean, save_invstd, dgamma, dbeta, accumulate_dw, coef);
  switch (dt) {
    case BnDtype::kBF16: launch_apply_bwd<BF16>(dy, dy2, y, x, coef, dx, dres, M, C, relu, st); break;
    case BnDtype::kF16: launch_apply_bwd<F16>(dy, dy2, y, x, coef, dx, dres, M, C, relu, st); break;
    default: launch_apply_bwd<F32>(dy, dy2, y, x, coef, dx, dres, M, C, relu, st); break;
  }
}

// Backward of act(bn(x) + bn2(x2)): one statistics pass (the masked upstream gradient dy' is
// shared; sum dy' * (x - mean) and sum dy' * (x2 - mean2) reduced together), two finalizes, one
// apply pass writing dx and dx2 -- instead of two reduce + two apply passes and the dres tensor.
void bn_backward_train_dual(BnDtype dt, const void* dy, const void* dy2, const uint8_t* mask,
                            const void* x, const void* x2, int64_t M, int C, const float* gamma,
                            const float* save_mean, const float* save_invstd,
                            const float* gamma2, const float* save_mean2,
                            const float* save_invstd2, bool relu, void* dx, void* dx2,
                            float* dgamma, float* dbeta, float* dgamma2, float* dbeta2,
                            bool accumulate_dw, float* workspace, float* workspace2,
                            hipStream_t st) {
  ReduceGeom g = reduce_geom(C);
  int B = reduce_blocks(M, C, g);
  float* partial = workspace;
  float* coef = workspace + static_cast<int64_t>(B) * 2 * C;
  float* partial2 = workspace2;
  float* coef2 = workspace2 + static_cast<int64_t>(B) * 2 * C;
  switch (dt) {
    case BnDtype::kBF16: launch_reduce<BF16>(true, x, dy, dy2, mask, save_mean, M, C, relu, partial, B, g, st, x2, save_mean2, partial2); break;
    case BnDtype::kF16: launch_reduce<F16>(true, x, dy, dy2, mask, save_mean, M, C, relu, partial, B, g, st, x2, save_mean2, partial2); break;
    default: launch_reduce<F32>(true, x, dy, dy2, mask, save_mean, M, C, relu, partial, B, g, st, x2, save_mean2, partial2); break;
  }
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 7) / 8), dim3(kBlock), 0, st, partial, B,
                     C, M, gamma, save_mean, save_invstd, dgamma, dbeta, accumulate_dw, coef);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 7) / 8), dim3(kBlock), 0, st, partial2, B,
                     C, M, gamma2, save_mean2, save_invstd2, dgamma2, dbeta2, accumulate_dw, coef2);
  switch (dt) {
    case BnDtype::kBF16: launch_apply_bwd<BF16>(dy, dy2, mask, x, coef, dx, nullptr, M, C, relu, st, x2, coef2, dx2); break;
    case BnDtype::kF16: launch_apply_bwd<F16>(dy, dy2, mask, x, coef, dx, nullptr, M, C, relu, st, x2, coef2, dx2); break;
    default: launch_apply_bwd<F32>(dy, dy2, mask, x, coef, dx, nullptr, M, C, relu, st, x2, coef2, dx2); break;
  }
}

void bn_relu_pool_forward(BnDtype dt, const void* x, void* y, uint8_t* idx, int N, int H, int W,
                          int C, const float* gamma, const float* beta, float* running_mean,
                          float* running_var, float momentum, float eps, float* save_mean,
                          float* save_invstd, int64_t* num_batches, float* workspace,
                          const float* affine_scale, const float* affine_shift, hipStream_t st,
                          const float* given_partials, int given_blocks) {
  const PoolGeom g{H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t M = static_cast<int64_t>(N) * H * W;
  const float* scale = affine_scale;
  const float* shift = affine_shift;
  if (scale == nullptr) {  // training: batch statistics (reduced here unless the conv epilogue did)
    scale = forward_affine_from_stats(dt, x, M, C, gamma, beta, running_mean, running_var, momentum,
                                      eps, save_mean, save_invstd, num_batches, workspace,
                                      given_partials, given_blocks, st);
    shift = scale + C;
  }
  {
    const int64_t nthr = static_cast<int64_t>(N) * ((g.Ho + 1) / 2) * ((g.Wo + 1) / 2) * (C / 8);
    const int qgrid = stream_grid(nthr, kBlock);
    switch (dt) {
      case BnDtype::kBF16: hipLaunchKernelGGL(bn_relu_pool_fwd_quad_kernel<BF16>, dim3(qgrid), dim3(kBlock), 0, st, x, scale, shift, y, idx, nthr, C, g); break;
      case BnDtype::kF16: hipLaunchKernelGGL(bn_relu_pool_fwd_quad_kernel<F16>, dim3(qgrid), dim3(kBlock), 0, st, x, scale, shift, y, idx, nthr, C, g); break;
      default: hipLaunchKernelGGL(bn_relu_pool_fwd_quad_kernel<F32>, dim3(qgrid), dim3(kBlock), 0, st, x, scale, shift, y, idx, nthr, C, g); break;
    }
  }
}

void bn_relu_pool_backward(BnDtype dt, const void* dyp, const uint8_t* idx, const void* x, int N,
                           int H, int W, int C, const float* gamma, const float* save_mean,
                           const float* save_invstd, void* dx, float* dgamma, float* dbeta,
                           float* workspace, hipStream_t st) {
  const PoolGeom g{H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t M = static_cast<int64_t>(N) * H * W;
  ReduceGeom rg = reduce_geom(C);
  int B = reduce_blocks(M, C, rg);
  float* partial = workspace;
  float* coef = workspace + static_cast<int64_t>(B) * 2 * C;
  size_t lds = static_cast<size_t>(rg.rpi) * rg.tpr * 16 * sizeof(float);
  const int64_t Qn = static_cast<int64_t>(N) * ((H + 1) / 2) * ((W + 1) / 2);
  const int64_t qiters = (Qn + rg.rpi - 1) / rg.rpi;
  if (B > qiters) B = static_cast<int>(qiters);
  dim3 grid(B, rg.cgroups);
  switch (dt) {
    case BnDtype::kBF16: hipLaunchKernelGGL(bn_pool_reduce_bwd_quad_kernel<BF16>, grid, dim3(kBlock), lds, st, x, dyp, idx, save_mean, Qn, C, rg.tpr, rg.rpi, g, partial); break;
    case BnDtype::kF16: hipLaunchKernelGGL(bn_pool_reduce_bwd_quad_kernel<F16>, grid, dim3(kBlock), lds, st, x, dyp, idx, save_mean, Qn, C, rg.tpr, rg.rpi, g, partial); break;
    default: hipLaunchKernelGGL(bn_pool_reduce_bwd_quad_kernel<F32>, grid, dim3(kBlock), lds, st, x, dyp, idx, save_mean, Qn, C, rg.tpr, rg.rpi, g, partial); break;
  }
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3((C + 7) / 8), dim3(kBlock), 0, st, partial, B,
                     C, M, gamma, save_mean, save_invstd, dgamma, dbeta, false, coef);
  dim3 ag(apply_blocks(Qn, rg, ApplyTuning{1, 2048}), rg.cgroups);
  switch (dt) {
    case BnDtype::kBF16: hipLaunchKernelGGL(bn_pool_apply_bwd_quad_kernel<BF16>, ag, dim3(kBlock), 0, st, x, dyp, idx, coef, dx, Qn, C, rg.tpr, rg.rpi, g); break;
    case BnDtype::kF16: hipLaunchKernelGGL(bn_pool_apply_bwd_quad_kernel<F16>, ag, dim3(kBlock), 0, st, x, dyp, idx, coef, dx, Qn, C, rg.tpr, rg.rpi, g); break;
    default: hipLaunchKernelGGL(bn_pool_apply_bwd_quad_kernel<F32>, ag, dim3(kBlock), 0, st, x, dyp, idx, coef, dx, Qn, C, rg.tpr, rg.rpi, g); break;
  }
}

void spatial_mean_backward(BnDtype dt, const void* g, void* dx, int N, int HW, int C,
                           hipStream_t st) {
  const int64_t nvec = static_cast<int64_t>(N) * HW * C / 8;
  const int grid = stream_grid(nvec, kBlock);
  const float inv = 1.f / static_cast<float>(HW);
  switch (dt) {
    case BnDtype::kBF16: hipLaunchKernelGGL(spatial_mean_bwd_kernel<BF16>, dim3(grid), dim3(kBlock), 0, st, g, dx, nvec, C / 8, HW, inv); break;
    case BnDtype::kF16: hipLaunchKernelGGL(spatial_mean_bwd_kernel<F16>, dim3(grid), dim3(kBlock), 0, st, g, dx, nvec, C / 8, HW, inv); break;
    default: hipLaunchKernelGGL(spatial_mean_bwd_kernel<F32>, dim3(grid), dim3(kBlock), 0, st, g, dx, nvec, C / 8, HW, inv); break;
  }
}

}  // namespace dca
