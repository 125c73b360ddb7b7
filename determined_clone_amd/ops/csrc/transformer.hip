// Transformer-block memory-bound kernels for MI355X: fused residual-add + LayerNorm (fwd/bwd),
// fused bias + GELU(tanh) (fwd/bwd), rotary position embedding (fwd/bwd).
//
// Used by the GPT-2 / GPT-NeoX DeepSpeedTrial (reference: examples/deepspeed/gpt_neox, which
// relies on DeepSpeed/apex CUDA kernels for these ops).
//
// Layout: activations are row-major [rows][D] bf16/fp32, D % 8 == 0. One wave64 owns a row (LN) so
// row statistics are pure in-register wave reductions (no LDS, no __syncthreads); every lane moves
// 16 B per access. Parameter gradients (dgamma/dbeta/dbias) are reduced deterministically:
// each block accumulates its rows in registers, writes one partial row, and a column-reduce kernel
// sums the partials.
#include "common.h"
#include "transformer_api.h"

#include <cstdlib>
#include <type_traits>

namespace dca {


namespace {

constexpr int kWaves = 4;             // rows (LN) handled concurrently per block
constexpr int kBlock = kWaves * 64;
constexpr int kLnColsumMaxD = 2048;    // LN backward reduces dx's column sums in-pass up to this width

// 8 consecutive fp32 affine parameters (gamma or beta) from c, or `fill` when absent / out of range.
__device__ __forceinline__ void load_affine8(const float* __restrict__ p, int c, bool ok, float fill,
                                             float (&out)[8]) {
  if (p && ok) {
    const float4 a = *reinterpret_cast<const float4*>(p + c);
    const float4 b = *reinterpret_cast<const float4*>(p + c + 4);
    out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
    out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = fill;
  }
}

template <typename T, int NV>
__global__ __launch_bounds__(kBlock) void ln_fwd_kernel(
    const void* __restrict__ x, const void* __restrict__ res, void* __restrict__ sum_out,
    void* __restrict__ y, const float* __restrict__ gamma, const float* __restrict__ beta,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nvec = D / 8;
  // gamma / beta: two 16-B loads per 8 columns, once per wave (not 16 scalar loads per row)
  float gv[NV][8], bv[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (lane + i * 64) * 8;
    load_affine8(gamma, c, c < D, 1.f, gv[i]);
    load_affine8(beta, c, c < D, 0.f, bv[i]);
  }
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid; row < rows;
       row += static_cast<int64_t>(gridDim.x) * kWaves) {
    const int64_t base = row * D;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        Vec8<T>::load(reinterpret_cast<const char*>(x) + (base + vi * 8) * Vec8<T>::bytes, v[i]);
        if (res) {
          float r[8];
          Vec8<T>::load(reinterpret_cast<const char*>(res) + (base + vi * 8) * Vec8<T>::bytes, r);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[i][k] += r[k];
          if (sum_out) Vec8<T>::store(reinterpret_cast<char*>(sum_out) + (base + vi * 8) * Vec8<T>::bytes, v[i]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[i][k];
      }
    }
    const float mean = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (lane + i * 64 < nvec) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = v[i][k] - mean;
          q = fmaf(d, d, q);
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        const int c = vi * 8;
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf((v[i][k] - mean) * rstd, gv[i][k], bv[i][k]);
        Vec8<T>::store(reinterpret_cast<char*>(y) + (base + c) * Vec8<T>::bytes, o);
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) [+ dres passthrough handled by caller]
// Per-block partial dgamma/dbeta: partial[blockIdx.x][2][D] (fp32).
// COLSUM: also the per-block column sums of dx itself (partial[blockIdx.x][3][D], third row): in a
// pre-LN transformer the residual branch that fed this LayerNorm ends in a linear layer whose
// output gradient IS dx, so its bias gradient comes out of this pass (no separate reduction).
template <typename T, int NV, bool COLSUM = false>
__global__ __launch_bounds__(kBlock) void ln_bwd_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const void* __restrict__ dsum, void* __restrict__ dx, float* __restrict__ partial,
    int64_t rows, int D) {
  constexpr int NP = COLSUM ? 3 : 2;  // partial rows per block
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nvec = D / 8;
  float dg[NV][8], db[NV][8], gam[NV][8], cs[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) { dg[i][k] = 0.f; db[i][k] = 0.f; cs[i][k] = 0.f; }
    const int c = (lane + i * 64) * 8;
    load_affine8(gamma, c, c < D, 1.f, gam[i]);
  }
  // One row per wave per iteration, with the NEXT row's x / dy / dsum / mean / rstd loads issued
  // before this row's math and wave reduction: two rows of loads in flight per wave, so the kernel
  // keeps HBM busy even when a concurrent side-stream GEMM leaves it few waves per CU.
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kWaves;
  Raw8<T> nx[NV] = {}, ng[NV] = {}, nr[NV] = {};  // zero: lanes past D and nr without dsum
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int64_t row) {
    const int64_t base = row * D;
    nmu = mean_in[row];
    nrs = rstd_in[row];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        nx[i] = ld8<T>(x, base + vi * 8);
        ng[i] = ld8<T>(dy, base + vi * 8);
        if (dsum) nr[i] = ld8<T>(dsum, base + vi * 8);
      }
    }
  };
  int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid;
  if (row < rows) fetch(row);
  for (; row < rows; row += stride) {
    const int64_t base = row * D;
    const float mean = nmu, rstd = nrs;
    Raw8<T> cx[NV], cg[NV], cr[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      cx[i] = nx[i];
      cg[i] = ng[i];
      cr[i] = nr[i];
    }
    if (row + stride < rows) fetch(row + stride);
    float xh[NV][8], g[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        float xv[8];
        unpack8<T>(cx[i], xv);
        unpack8<T>(cg[i], g[i]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xh[i][k] = (xv[k] - mean) * rstd;
          dg[i][k] = fmaf(g[i][k], xh[i][k], dg[i][k]);
          db[i][k] += g[i][k];
          const float gg = g[i][k] * gam[i][k];
          g[i][k] = gg;
          s1 += gg;
          s2 = fmaf(gg, xh[i][k], s2);
        }
      }
    }
    const float m1 = wave_sum(s1) / D, m2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        const int c = vi * 8;
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = rstd * (g[i][k] - m1 - xh[i][k] * m2);
        if (dsum) {
          float r[8];
          unpack8<T>(cr[i], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        if (COLSUM) {
#pragma unroll
          for (int k = 0; k < 8; ++k) cs[i][k] += o[k];
        }
        Vec8<T>::store(reinterpret_cast<char*>(dx) + (base + c) * Vec8<T>::bytes, o);
      }
    }
  }
  // block-level combine of the kWaves waves' column partials through LDS
  // cross-wave reduction, one partial row at a time through a [kWaves][D] LDS buffer (<= 128 KB
  // at D = 8192)
  extern __shared__ __attribute__((aligned(16))) float lds[];
#pragma unroll
  for (int which = 0; which < NP; ++which) {
    if (which) __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec)
#pragma unroll
        for (int k = 0; k < 8; ++k)
          lds[wid * D + vi * 8 + k] = which == 0 ? dg[i][k] : which == 1 ? db[i][k] : cs[i][k];
    }
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += kBlock) {
      float a = 0.f;
      for (int w = 0; w < kWaves; ++w) a += lds[w * D + col];
      partial[(static_cast<int64_t>(blockIdx.x) * NP + which) * D + col] = a;
    }
  }
}

// Row-group LayerNorm backward for D <= 2048 (the transformer widths). A row is covered by a group
// of W = ceil(D / 512) waves -- 8 columns per lane, one 16-B nontemporal load per tensor -- so a
// lane keeps only 8 columns of dgamma / dbeta (/ dx column sum) accumulators and gamma: ~1/2 the
// registers of the one-row-per-wave kernel above, hence twice the waves per CU to keep HBM busy.
// A 512-thread block runs G = 8 / W groups; each group takes R rows per step, all their loads
// issued before the first use. The per-row sums (g.gamma, g.gamma.xhat) cross the W waves of a
// group through a double-buffered LDS slot (one barrier per step; none when W == 1), and at the
// end the G groups' column partials combine through LDS into ONE partial row set per block
// (partial[blockIdx.x][NP][D]), so the partial traffic stays ~1-2 % of the pass.
constexpr int kLnRgThreads = 512;
template <typename T, int W, int R, bool COLSUM>
__global__ __launch_bounds__(kLnRgThreads) void ln_bwd_rg_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const void* __restrict__ dsum, void* __restrict__ dx, float* __restrict__ partial,
    int64_t rows, int D) {
  constexpr int G = 8 / W;
  constexpr int NP = COLSUM ? 3 : 2;
  __shared__ float red[2][G][R][W][2];
  __shared__ __attribute__((aligned(16))) float comb[G][W * 512];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar row math
  const int grp = wid / W, wg = wid % W;
  const int cl = (wg * 64 + lane) * 8;  // first of this lane's 8 columns
  const bool ok = cl < D;
  const int clc = ok ? cl : 0;          // loads stay in bounds; !ok lanes never store
  float gam[8], dg[8], db[8], cs[8];
  load_affine8(gamma, cl, ok, 1.f, gam);
#pragma unroll
  for (int k = 0; k < 8; ++k) { dg[k] = 0.f; db[k] = 0.f; cs[k] = 0.f; }
  int par = 0;
  // block-uniform trip count (every wave reaches every barrier); rows past the end load the last
  // row again and are masked out of the sums and stores
  for (int64_t b0 = static_cast<int64_t>(blockIdx.x) * G * R; b0 < rows;
       b0 += static_cast<int64_t>(gridDim.x) * G * R) {
    const int64_t r0 = b0 + static_cast<int64_t>(grp) * R;
    Raw8<T> rx[R], rg[R], rr[R];
    float mu[R], rs[R], s1[R], s2[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t row = r0 + j < rows ? r0 + j : rows - 1;
      mu[j] = mean_in[row];
      rs[j] = rstd_in[row];
      rx[j] = ld8nt<T>(x, row * D + clc);
      rg[j] = ld8nt<T>(dy, row * D + clc);
      rr[j] = {};
      if (dsum) rr[j] = ld8nt<T>(dsum, row * D + clc);
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      float xv[8], g[8];
      unpack8<T>(rx[j], xv);
      unpack8<T>(rg[j], g);
      const float live = (r0 + j < rows && ok) ? 1.f : 0.f;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float gk = g[k] * live;
        const float xh = (xv[k] - mu[j]) * rs[j];
        dg[k] = fmaf(gk, xh, dg[k]);
        db[k] += gk;
        const float gg = gk * gam[k];
        a += gg;
        b = fmaf(gg, xh, b);
      }
      s1[j] = wave_sum_dpp(a);
      s2[j] = wave_sum_dpp(b);
    }
    if constexpr (W > 1) {
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < R; ++j) {
          red[par][grp][j][wg][0] = s1[j];
          red[par][grp][j][wg][1] = s2[j];
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < R; ++j) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          a += red[par][grp][j][w][0];
          b += red[par][grp][j][w][1];
        }
        s1[j] = a;
        s2[j] = b;
      }
      par ^= 1;
    }
    const float inv_d = 1.f / static_cast<float>(D);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int64_t row = r0 + j;
      if (row < rows && ok) {
        float xv[8], g[8], o[8];
        unpack8<T>(rx[j], xv);
        unpack8<T>(rg[j], g);
        const float m1 = s1[j] * inv_d, m2 = s2[j] * inv_d;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = (xv[k] - mu[j]) * rs[j];
          o[k] = rs[j] * (g[k] * gam[k] - m1 - xh * m2);
        }
        if (dsum) {
          float r[8];
          unpack8<T>(rr[j], r);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] += r[k];
        }
        if (COLSUM) {
#pragma unroll
          for (int k = 0; k < 8; ++k) cs[k] += o[k];
        }
        Vec8<T>::store(reinterpret_cast<char*>(dx) + (row * D + cl) * Vec8<T>::bytes, o);
      }
    }
  }
  // the G groups' column partials -> one partial row per quantity
#pragma unroll
  for (int which = 0; which < NP; ++which) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k)
      comb[grp][cl + k] = which == 0 ? dg[k] : which == 1 ? db[k] : cs[k];  // cl < W * 512
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += kLnRgThreads) {
      float a = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < G; ++g2) a += comb[g2][col];
      partial[(static_cast<int64_t>(blockIdx.x) * NP + which) * D + col] = a;
    }
  }
}

// out[j] = sum_b partial[b][j] for j < ncols (fp32). Block = 16 waves x 64 columns: lane -> column
// (coalesced 256-B rows), wave -> every 16th partial row with 4 independent loads in flight, then an
// LDS tree over the 16 waves. Deterministic (fixed order).
constexpr int kColWaves = 16;
__device__ __forceinline__ void column_store(const ColumnOut& o, int64_t j, float v) {
  char* base = static_cast<char*>(j < o.split ? o.p0 : o.p1);
  const int64_t k = j < o.split ? j : j - o.split;
  if (o.bf16) {
    uint16_t* q = reinterpret_cast<uint16_t*>(base) + k;
    if (o.accumulate) v += __uint_as_float(static_cast<uint32_t>(*q) << 16);
    *q = static_cast<uint16_t>(f2bf_bits(v));
  } else {
    float* q = reinterpret_cast<float*>(base) + k;
    *q = o.accumulate ? *q + v : v;
  }
}

// Columns j >= n0 land in out2 (at j - n0): one launch reduces several quantities whose partial
// rows sit side by side (LayerNorm backward: dgamma | dbeta | dx column sums).
__global__ __launch_bounds__(kColWaves * 64) void column_reduce_kernel(const float* __restrict__ partial,
                                                                      int nparts, int64_t ncols,
                                                                      ColumnOut out, int64_t pstride,
                                                                      ColumnOut out2, int64_t n0) {
  __shared__ float red[kColWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t j = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (j < ncols) {
    int b = w;
    for (; b + 3 * kColWaves < nparts; b += 4 * kColWaves) {
      a0 += partial[static_cast<int64_t>(b) * pstride + j];
      a1 += partial[static_cast<int64_t>(b + kColWaves) * pstride + j];
      a2 += partial[static_cast<int64_t>(b + 2 * kColWaves) * pstride + j];
      a3 += partial[static_cast<int64_t>(b + 3 * kColWaves) * pstride + j];
    }
    for (; b < nparts; b += kColWaves) a0 += partial[static_cast<int64_t>(b) * pstride + j];
  }
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  for (int s = kColWaves / 2; s > 0; s >>= 1) {
    if (w < s) red[w][lane] += red[w + s][lane];
    __syncthreads();
  }
  if (w == 0 && j < ncols) {
    if (j < n0) column_store(out, j, red[0][lane]);
    else column_store(out2, j - n0, red[0][lane]);
  }
}

// Per-block column partial sums of dy [rows][N] (bias gradient of a linear layer). Block = 4 waves;
// a wave's 64 lanes cover 512 consecutive columns (8 per lane, one 16-B load per row) and the 4
// waves take interleaved rows, so every lane is busy whatever N is (the previous 2048-column block
// left half the block idle at N = 1024). Rows stride by gridDim.y * 4 with 4 independent loads in
// flight; the waves combine through LDS and the block writes one partial row (grid.y partial rows,
// summed by column_reduce_kernel).
constexpr int kRsWaves = 4;
constexpr int kRsCols = 512;
template <typename T>
__global__ __launch_bounds__(kRsWaves * 64) void row_sum_kernel(const void* __restrict__ dy,
                                                                float* __restrict__ partial,
                                                                int64_t rows, int N) {
  __shared__ __attribute__((aligned(16))) float red[kRsWaves][kRsCols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * kRsCols + lane * 8;
  const bool ok = c < N;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (ok) {
    const int64_t step = static_cast<int64_t>(gridDim.y) * kRsWaves;
    int64_t r = static_cast<int64_t>(blockIdx.y) * kRsWaves + w;
    for (; r + 3 * step < rows; r += 4 * step) {
      float g[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        Vec8<T>::load(reinterpret_cast<const char*>(dy) + ((r + u * step) * N + c) * Vec8<T>::bytes, g[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += g[u][k];
    }
    for (; r < rows; r += step) {
      float g[8];
      Vec8<T>::load(reinterpret_cast<const char*>(dy) + (r * N + c) * Vec8<T>::bytes, g);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += g[k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[w][lane * 8 + k] = acc[k];
  __syncthreads();
  // 256 threads x 2 columns each: sum the 4 waves' rows in fixed order
  for (int j = threadIdx.x; j < kRsCols; j += kRsWaves * 64) {
    const int col = blockIdx.x * kRsCols + j;
    if (col < N)
      partial[static_cast<int64_t>(blockIdx.y) * N + col] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
  }
}

// acc[i] (+)= sum_s part[s][i] for the split-K weight gradients of ops/transformer.py: the
// per-slice fp32 GEMM outputs are summed in a fixed order and added into the parameter's
// persistent .grad view (bf16 or fp32) in one pass -- replaces a torch reduce over the slices plus
// a mixed-dtype add (two kernels, ~95 us per GPT-2-medium weight at 32k tokens).
template <typename A>
__global__ __launch_bounds__(256) void splitk_accumulate_kernel(const float* __restrict__ part,
                                                                void* __restrict__ acc, int64_t n,
                                                                int splits, bool accumulate) {
  const int64_t nv = n / 8;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < nv;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    float s[8];
    Vec8<F32>::load(part + i * 8, s);
    for (int p = 1; p < splits; ++p) {
      float t[8];
      Vec8<F32>::load(part + static_cast<int64_t>(p) * n + i * 8, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += t[k];
    }
    char* dst = reinterpret_cast<char*>(acc) + i * 8 * Vec8<A>::bytes;
    if (accumulate) {
      float a[8];
      Vec8<A>::load(dst, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) s[k] += a[k];
    }
    Vec8<A>::store(dst, s);
  }
}

// 8 bias values starting at column c, fp32 or bf16 storage (nullptr -> zeros).
__device__ __forceinline__ void load_bias8(const void* bias, bool bf16, int c, float (&b)[8]) {
  if (!bias) {
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = 0.f;
  } else if (bf16) {
    Vec8<BF16>::load(static_cast<const char*>(bias) + static_cast<int64_t>(c) * 2, b);
  } else {
    Vec8<F32>::load(static_cast<const char*>(bias) + static_cast<int64_t>(c) * 4, b);
  }
}

// ------------------------------------------------------------------ bias + GELU(tanh)
// 0.5 (1 + tanh(u)) = sigmoid(2u): one v_exp_f32 + one v_rcp_f32 instead of libm tanhf.
// s = 1 / (1 + 2^(-2u log2 e)); u -> -inf gives 2^+inf = inf -> s = 0, u -> +inf gives s = 1.
__device__ __forceinline__ float sigmoid2u(float u) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
}
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * fmaf(k1 * x * x, x, x);
  return x * sigmoid2u(u);
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  // d/dx [x s(u)] = s + x s (1 - s) * 2 u',  u' = k0 (1 + 3 k1 x^2)
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * fmaf(k1 * x2, x, x);
  const float s = sigmoid2u(u);
  return fmaf(x * s * (1.f - s), 2.f * k0 * fmaf(3.f * k1, x2, 1.f), s);
}

template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const void* __restrict__ x,
                                                            const void* __restrict__ bias,
                                                            bool bias_bf16,
                                                            void* __restrict__ y, int64_t rows,
                                                            int N) {
  const int n8 = N / 8;
  const int64_t total = rows * n8;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; v < total;
       v += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int c = static_cast<int>(v % n8) * 8;
    float a[8];
    Vec8<T>::load(reinterpret_cast<const char*>(x) + v * 8 * Vec8<T>::bytes, a);
    float b[8];
    load_bias8(bias, bias_bf16, c, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = gelu_tanh(a[k] + b[k]);
    Vec8<T>::store(reinterpret_cast<char*>(y) + v * 8 * Vec8<T>::bytes, a);
  }
}

// Block = 256 threads covering 2048 columns (8 per thread) x a slab of rows; dbias partials
// [gridDim.y][N] reduced by column_reduce_kernel.
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(
    const void* __restrict__ dy, const void* __restrict__ x, const void* __restrict__ bias,
    bool bias_bf16, void* __restrict__ dx, float* __restrict__ partial, int64_t rows, int N) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= N) return;
  float bsum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float b[8];
  load_bias8(bias, bias_bf16, c, b);
  const int64_t step = gridDim.y;
  int64_t r = blockIdx.y;
  // 4 rows per iteration: 8 independent 16-B loads in flight per lane (this grid is only
  // ~2 blocks per CU, so memory-level parallelism has to come from inside the thread)
  for (; r + 3 * step < rows; r += 4 * step) {
    float g[4][8], a[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      // streamed once: nontemporal loads (profiles/round4_hbm_streaming_ceilings.txt)
      const int64_t e = (r + u * step) * N + c;
      unpack8<T>(ld8nt<T>(dy, e), g[u]);
      unpack8<T>(ld8nt<T>(x, e), a[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[u][k] *= gelu_tanh_grad(a[u][k] + b[k]);
        bsum[k] += g[u][k];
      }
      Vec8<T>::store(reinterpret_cast<char*>(dx) + ((r + u * step) * N + c) * Vec8<T>::bytes, g[u]);
    }
  }
  for (; r < rows; r += step) {
    const int64_t off = (r * N + c) * Vec8<T>::bytes;
    float g[8], a[8];
    Vec8<T>::load(reinterpret_cast<const char*>(dy) + off, g);
    Vec8<T>::load(reinterpret_cast<const char*>(x) + off, a);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      g[k] *= gelu_tanh_grad(a[k] + b[k]);
      bsum[k] += g[k];
    }
    Vec8<T>::store(reinterpret_cast<char*>(dx) + off, g);
  }
  if (partial)
#pragma unroll
    for (int k = 0; k < 8; ++k) partial[static_cast<int64_t>(blockIdx.y) * N + c + k] = bsum[k];
}

// ------------------------------------------------------------------ rotary embedding
// x: [rows = B*S*H][D] (head-major inner layout [.., S, H, D] flattened so row -> position
// pos = (row / H) % S). Rotates the first rot_dim features as pairs (i, i + rot_dim/2)
// (GPT-NeoX "rotate_half" convention); cos/sin tables [S][rot_dim/2] fp32. backward = forward
// with -sin.
template <typename T>
__global__ __launch_bounds__(256) void rope_kernel(const void* __restrict__ x, void* __restrict__ y,
                                                   const float* __restrict__ cosT,
                                                   const float* __restrict__ sinT, int64_t rows,
                                                   int H, int S, int D, int rot, float sign) {
  const int half = rot / 2;
  const int per_row = D / 2;  // threads per row: each handles one (i, i+half) pair or 2 passthrough
  const int64_t total = rows * per_row;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t row = t / per_row;
    const int i = static_cast<int>(t % per_row);
    const int pos = static_cast<int>((row / H) % S);
    if (i < half) {
      const float cs = cosT[pos * half + i], sn = sinT[pos * half + i] * sign;
      const float a = Elem<T>::get(x, row * D + i), b = Elem<T>::get(x, row * D + i + half);
      Elem<T>::put(y, row * D + i, a * cs - b * sn);
      Elem<T>::put(y, row * D + i + half, b * cs + a * sn);
    } else {
      // pass-through features beyond rot_dim: two per thread
      const int j = rot + 2 * (i - half);
      if (j < D) {
        Elem<T>::put(y, row * D + j, Elem<T>::get(x, row * D + j));
        if (j + 1 < D) Elem<T>::put(y, row * D + j + 1, Elem<T>::get(x, row * D + j + 1));
      }
    }
  }
}

template <int NV>
struct NVTag {
  static constexpr int value = NV;
};

template <typename T, typename F>
void dispatch_nv(int D, F&& f) {
  const int nv = (D / 8 + 63) / 64;
  if (nv <= 1) f(NVTag<1>{});
  else if (nv <= 2) f(NVTag<2>{});
  else if (nv <= 4) f(NVTag<4>{});
  else if (nv <= 8) f(NVTag<8>{});
  else f(NVTag<16>{});
}

template <typename F>
void dispatch_t(TDtype dt, F&& f) {
  switch (dt) {
    case TDtype::kBF16: f(BF16{}); break;
    case TDtype::kF16: f(F16{}); break;
    default: f(F32{}); break;
  }
}

inline int ln_grid(int64_t rows) {
  int64_t g = (rows + kWaves - 1) / kWaves;
  return static_cast<int>(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

}  // namespace

int ln_bwd_blocks(int64_t rows) {
  // 512-4096 blocks measure within 15% of each other at GPT-2-medium rows (2.7-3.1 TB/s,
  // tools/bench_tx_bwd.py)
  constexpr int cap = 1024;
  int64_t g = (rows + kWaves - 1) / kWaves;
  return static_cast<int>(g < cap ? (g < 1 ? 1 : g) : cap);
}

void splitk_accumulate(bool acc_bf16, const float* part, void* acc, int64_t n, int splits,
                       bool accumulate, hipStream_t st) {
  const int grid = stream_grid(n / 8, 256);
  if (acc_bf16)
    hipLaunchKernelGGL(splitk_accumulate_kernel<BF16>, dim3(grid), dim3(256), 0, st, part, acc, n,
                       splits, accumulate);
  else
    hipLaunchKernelGGL(splitk_accumulate_kernel<F32>, dim3(grid), dim3(256), 0, st, part, acc, n,
                       splits, accumulate);
}

void layernorm_fwd(TDtype dt, const void* x, const void* res, void* sum_out, void* y,
                   const float* gamma, const float* beta, float* mean, float* rstd, int64_t rows,
                   int D, float eps, hipStream_t st) {
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    dispatch_nv<T>(D, [&](auto nvt) {
      constexpr int NV = decltype(nvt)::value;
      hipLaunchKernelGGL((ln_fwd_kernel<T, NV>), dim3(ln_grid(rows)), dim3(kBlock), 0, st, x, res,
                         sum_out, y, gamma, beta, mean, rstd, rows, D, eps);
    });
  });
}

// Row-group kernel launch shape (D <= kLnColsumMaxD): W waves per row, R rows per group step.
int ln_rg_waves(int D) { return D <= 512 ? 1 : D <= 1024 ? 2 : 4; }
// 2 rows per group step (4 measured slower: profiles/round5_ln_bwd_row_group_sweep.txt)
int ln_rg_rows() { return 2; }
int ln_rg_blocks(int64_t rows, int D) {
  // fills every CU with two 8-wave blocks
  constexpr int cap = 512;
  const int64_t per = static_cast<int64_t>(8 / ln_rg_waves(D)) * ln_rg_rows();
  const int64_t g = (rows + per - 1) / per;
  return static_cast<int>(g < cap ? (g < 1 ? 1 : g) : cap);
}
bool ln_rg_path(int D) { return D <= kLnColsumMaxD; }

int64_t ln_bwd_partial_floats(int64_t rows, int D, bool colsum) {
  const int blocks = ln_rg_path(D) ? ln_rg_blocks(rows, D) : ln_bwd_blocks(rows);
  const int64_t n = static_cast<int64_t>(blocks) * (colsum && D <= kLnColsumMaxD ? 3 : 2) * D;
  const int64_t r = colsum && D > kLnColsumMaxD ? static_cast<int64_t>(row_sum_blocks(rows, D)) * D : 0;
  return n > r ? n : r;
}

void layernorm_bwd(TDtype dt, const void* dy, const void* x, const float* gamma, const float* mean,
                   const float* rstd, const void* dsum, void* dx, float* partial,
                   const ColumnOut* dgamma_dbeta, int64_t rows, int D, hipStream_t st,
                   const ColumnOut* dx_colsum) {
  const bool rg = ln_rg_path(D);
  const int blocks = rg ? ln_rg_blocks(rows, D) : ln_bwd_blocks(rows);
  const bool fused_colsum = dx_colsum && D <= kLnColsumMaxD;
  const int np = fused_colsum ? 3 : 2;
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    if (rg) {
      const int W = ln_rg_waves(D), R = ln_rg_rows();
      auto go = [&](auto wt, auto rt) {
        constexpr int Wc = decltype(wt)::value, Rc = decltype(rt)::value;
        if (fused_colsum)
          hipLaunchKernelGGL((ln_bwd_rg_kernel<T, Wc, Rc, true>), dim3(blocks), dim3(kLnRgThreads), 0, st,
                             dy, x, gamma, mean, rstd, dsum, dx, partial, rows, D);
        else
          hipLaunchKernelGGL((ln_bwd_rg_kernel<T, Wc, Rc, false>), dim3(blocks), dim3(kLnRgThreads), 0, st,
                             dy, x, gamma, mean, rstd, dsum, dx, partial, rows, D);
      };
      auto by_rows = [&](auto wt) {
        if (R == 4) go(wt, NVTag<4>{}); else go(wt, NVTag<2>{});
      };
      if (W == 1) by_rows(NVTag<1>{});
      else if (W == 2) by_rows(NVTag<2>{});
      else by_rows(NVTag<4>{});
      return;
    }
    dispatch_nv<T>(D, [&](auto nvt) {
      constexpr int NV = decltype(nvt)::value;
      const size_t lds = static_cast<size_t>(kWaves) * D * sizeof(float);
      if constexpr (NV <= 4) {  // D <= 2048: the extra accumulators fit in registers
        if (fused_colsum) {
          hipLaunchKernelGGL((ln_bwd_kernel<T, NV, true>), dim3(blocks), dim3(kBlock), lds, st, dy, x,
                             gamma, mean, rstd, dsum, dx, partial, rows, D);
          return;
        }
      }
      hipLaunchKernelGGL((ln_bwd_kernel<T, NV, false>), dim3(blocks), dim3(kBlock), lds, st, dy, x, gamma,
                         mean, rstd, dsum, dx, partial, rows, D);
    });
  });
  const int64_t pstride = static_cast<int64_t>(np) * D;
  if (dgamma_dbeta || fused_colsum) {
    // one launch: dgamma | dbeta (2D columns) and the dx column sums (D more) when fused
    const int64_t n0 = dgamma_dbeta ? 2 * static_cast<int64_t>(D) : 0;
    const int64_t ncols = n0 + (fused_colsum ? D : 0);
    const float* src = dgamma_dbeta ? partial : partial + 2 * D;
    hipLaunchKernelGGL(column_reduce_kernel, dim3((ncols + 63) / 64), dim3(kColWaves * 64), 0, st,
                       src, blocks, ncols, dgamma_dbeta ? *dgamma_dbeta : ColumnOut{}, pstride,
                       fused_colsum ? *dx_colsum : ColumnOut{}, n0);
  }
  if (dx_colsum && !fused_colsum)  // wide rows: a separate column reduction of dx (see ln_bwd_partial_floats)
    row_sum(dt, dx, partial, *dx_colsum, rows, D, st);
}

void bias_gelu_fwd(TDtype dt, const void* x, const void* bias, bool bias_bf16, void* y,
                   int64_t rows, int N, hipStream_t st) {
  const int grid = stream_grid(rows * N / 8, 256);
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bias_gelu_fwd_kernel<T>, dim3(grid), dim3(256), 0, st, x, bias, bias_bf16, y,
                       rows, N);
  });
}

int bias_gelu_bwd_row_blocks(int64_t rows) {
  // row slabs (grid.y; profiles/round5_bias_gelu_bwd_sweep_and_ln_rg_ab.txt)
  constexpr int cap = 256;
  return static_cast<int>(rows < cap ? (rows < 1 ? 1 : rows) : cap);
}

void bias_gelu_bwd(TDtype dt, const void* dy, const void* x, const void* bias, bool bias_bf16,
                   void* dx, float* partial, const ColumnOut* dbias, int64_t rows, int N,
                   hipStream_t st) {
  const int rb = bias_gelu_bwd_row_blocks(rows);
  dim3 grid((N / 8 + 255) / 256, rb);
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(bias_gelu_bwd_kernel<T>, grid, dim3(256), 0, st, dy, x, bias, bias_bf16, dx,
                       dbias ? partial : nullptr, rows, N);
  });
  if (dbias)
    hipLaunchKernelGGL(column_reduce_kernel, dim3((N + 63) / 64), dim3(kColWaves * 64), 0, st,
                       partial, rb, static_cast<int64_t>(N), *dbias, static_cast<int64_t>(N), ColumnOut{},
                       static_cast<int64_t>(N));
}

int row_sum_blocks(int64_t rows, int N) {
  // ~4096 waves over the whole chip (16 per CU): grid.y row slabs of >= 16 rows per wave
  const int cb = (N + kRsCols - 1) / kRsCols;
  int64_t b = 1024 / cb;
  const int64_t cap = (rows + 16 * kRsWaves - 1) / (16 * kRsWaves);
  if (b > cap) b = cap;
  return static_cast<int>(b < 1 ? 1 : b);
}

void row_sum(TDtype dt, const void* dy, float* partial, const ColumnOut& out, int64_t rows, int N,
             hipStream_t st) {
  const int rb = row_sum_blocks(rows, N);
  dim3 grid((N + kRsCols - 1) / kRsCols, rb);
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(row_sum_kernel<T>, grid, dim3(kRsWaves * 64), 0, st, dy, partial, rows, N);
  });
  hipLaunchKernelGGL(column_reduce_kernel, dim3((N + 63) / 64), dim3(kColWaves * 64), 0, st,
                     partial, rb, static_cast<int64_t>(N), out, static_cast<int64_t>(N), ColumnOut{},
                     static_cast<int64_t>(N));
}

void rope(TDtype dt, const void* x, void* y, const float* cosT, const float* sinT, int64_t rows,
          int H, int S, int D, int rot, bool backward, hipStream_t st) {
  const int grid = stream_grid(rows * (D / 2), 256);
  dispatch_t(dt, [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(rope_kernel<T>, dim3(grid), dim3(256), 0, st, x, y, cosT, sinT, rows, H, S, D,
                       rot, backward ? -1.f : 1.f);
  });
}

// ------------------------------------------------------------------ fused softmax cross-entropy
// logits [rows][V] (bf16/f16/f32) -> per-row lse (fp32) and loss = lse - logit[target]
// (0 for ignore_index rows) in ONE read of the logits (online max/sum per thread, then a
// wave/LDS combine). Backward recomputes softmax from the saved lse:
// dlogits = (exp(x - lse) - onehot) * grad / n_valid, with grad and n_valid read from device
// memory (no host sync). Replaces the reference GPT trial's fp32 upcast + log_softmax + nll.
template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const void* __restrict__ logits,
                                                     const int64_t* __restrict__ target,
                                                     float* __restrict__ lse_out,
                                                     float* __restrict__ loss_out, int V,
                                                     int64_t ignore_index) {
  __shared__ float sm[8], ss[8];
  const int64_t row = blockIdx.x;
  const char* base = reinterpret_cast<const char*>(logits) + row * V * Vec8<T>::bytes;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += blockDim.x * 8) {
    float v[8];
    Vec8<T>::load(base + static_cast<int64_t>(c) * Vec8<T>::bytes, v);
    float mx = v[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) mx = fmaxf(mx, v[k]);
    const float nm = fmaxf(m, mx);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += __expf(v[k] - nm);
    m = nm;
    s = acc;
  }
  // combine (m, s) across the wave, then across waves
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64), os = __shfl_xor(s, off, 64);
    const float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < static_cast<int>(blockDim.x >> 6); ++i) {
      const float nm = fmaxf(M, sm[i]);
      S = S * __expf(M - nm) + ss[i] * __expf(sm[i] - nm);
      M = nm;
    }
    const float l = M + __logf(S);
    lse_out[row] = l;
    const int64_t t = target[row];
    float loss = 0.f;
    if (t != ignore_index && t >= 0 && t < V) loss = l - Elem<T>::get(logits, row * V + t);
    loss_out[row] = loss;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const void* __restrict__ logits,
                                                     const int64_t* __restrict__ target,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ gscale,
                                                     void* __restrict__ dlogits, int V,
                                                     int64_t ignore_index) {
  const int64_t row = blockIdx.x;
  const int64_t t = target[row];
  const bool valid = t != ignore_index;
  // gscale = [grad_output, n_valid]
  const float g = valid ? gscale[0] / fmaxf(gscale[1], 1.f) : 0.f;
  const float l = lse[row];
  const int64_t off = row * V;
  for (int c = threadIdx.x * 8; c < V; c += blockDim.x * 8) {
    float v[8];
    Vec8<T>::load(reinterpret_cast<const char*>(logits) + (off + c) * Vec8<T>::bytes, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (__expf(v[k] - l) - ((c + k) == t ? 1.f : 0.f)) * g;
    Vec8<T>::store(reinterpret_cast<char*>(dlogits) + (off + c) * Vec8<T>::bytes, v);
  }
}

void cross_entropy_fwd(TDtype dt, const void* logits, const int64_t* target, float* lse,
                       float* loss, int64_t rows, int V, int64_t ignore_index, hipStream_t st) {
  dispatch_t(dt, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(ce_fwd_kernel<T>, dim3(rows), dim3(256), 0, st, logits, target, lse, loss, V,
                       ignore_index);
  });
}

void cross_entropy_bwd(TDtype dt, const void* logits, const int64_t* target, const float* lse,
                       const float* gscale, void* dlogits, int64_t rows, int V,
                       int64_t ignore_index, hipStream_t st) {
  dispatch_t(dt, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(ce_bwd_kernel<T>, dim3(rows), dim3(256), 0, st, logits, target, lse, gscale,
                       dlogits, V, ignore_index);
  });
}

}  // namespace dca
