// Pointwise (1x1, stride 1) NHWC convolutions of the ResNet-50 bottleneck as MFMA GEMMs, with the
// following BatchNorm's statistics fused into the forward epilogue.
//
// The reference trains torchvision's resnet50 through cuDNN (examples/deepspeed_autotune/
// torchvision, harness/determined/pytorch/_pytorch_trial.py). In NHWC a 1x1 convolution IS a GEMM
// over rows m = (n, h, w):
//   forward   Y[m][co]  = sum_ci X[m][ci]  * W[co][ci]
//   dgrad     dX[m][ci] = sum_co dY[m][co] * W[co][ci]
//   wgrad     dW[co][ci] = sum_m dY[m][co] * X[m][ci]
//
// gemm_rowk_kernel (forward and dgrad): both operands are "k-contiguous rows" (X / dY rows, W / W^T
// rows), staged in LDS with a 144-B row stride (conflict-free ds_read_b128 fragment reads for
// v_mfma_f32_32x32x16_bf16). The MFMA computes the TRANSPOSED tile (rows = output channels, cols =
// m) so each lane's accumulator registers hold 4 consecutive channels of one output row: the
// epilogue packs them into 8-B LDS writes, then streams the tile out with 16-B coalesced stores
// and -- in the forward -- accumulates per-channel (sum, sum^2) of the bf16-rounded outputs into
// the partial-statistics layout of batchnorm.hip, so the BatchNorm that consumes Y skips its own
// statistics pass over HBM. Tiles are dealt XCD-contiguously (all n-tiles of an m-tile run on one
// XCD, sharing X rows in its L2).
//
// wgrad_kernel: the reduction runs over m (millions of rows), so the grid is output tiles x splits
// of m; both operands are m-major in memory and arrive as MFMA fragments through transposed LDS
// reads (ds_read_b64_tr_b16). Per-split fp32 tiles go to a workspace and wgrad_reduce_kernel sums
// them deterministically into the weight gradient (optionally accumulating into the parameter's
// persistent .grad view, ops/_grad.py).
//
// Measured against MIOpen (tools/bench_pointwise.py, profiles/r8_pointwise_conv_study.txt): these
// kernels win the layer3/4 weight gradients but lose forward/dgrad (single LDS stage with two
// barriers per 64-k step, 3 waves/SIMD), so the model path is opt-in (ops/conv.py, DCA_CONV1X1=1).
#include <cstdlib>

#include "common.h"

namespace dca {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kThreads = 256;
constexpr int kBK = 64;       // k elements per LDS stage (gemm_rowk)
constexpr int kRS = kBK + 8;  // LDS row stride in elements: 144 B -> 16 rows hit 16 distinct 16-B slots

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// The hardware deals workgroup ids round-robin over the 8 XCDs; give each XCD a contiguous range of
// tile ids instead (identity when the grid is not a multiple of 8).
__device__ __forceinline__ int xcd_swizzle(int id, int G) {
  if ((G & 7) != 0) return id;
  return (id & 7) * (G >> 3) + (id >> 3);
}

// ------------------------------------------------------------------ forward / dgrad GEMM
// Y[m][n0:n0+BN] = X[m][:] . B[n][:]^T for the BM rows of one tile; B is [N][K] (k contiguous).
template <int BM, int BN, bool STATS>
__global__ __launch_bounds__(kThreads) void gemm_rowk_kernel(
    const uint16_t* __restrict__ X, const uint16_t* __restrict__ B, uint16_t* __restrict__ Y,
    float* __restrict__ partial, int M, int N, int K) {
  constexpr int TN = BN / 2, TM = BM / 2;  // wave tile (2 x 2 waves)
  constexpr int FN = TN / 32, FM = TM / 32;
  constexpr int XCH = BM * kBK / 8 / kThreads;  // 16-B chunks per thread per stage
  constexpr int BCH = BN * kBK / 8 / kThreads;
  static_assert(XCH >= 1 && BCH >= 1, "tile too small for the block");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  uint16_t* Xs = lds;             // [BM][kRS]
  uint16_t* Bs = lds + BM * kRS;  // [BN][kRS]

  const int NT = N / BN;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int mt = t / NT, nt = t - mt * NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wn = w & 1, wm = w >> 1;
  const int r = lane & 31, h = lane >> 5;

  uint4 xr[XCH], br[BCH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int c = tid + i * kThreads, row = c >> 3, kc = (c & 7) * 8;
      xr[i] = make_uint4(0, 0, 0, 0);
      if (m0 + row < M)
        xr[i] = *reinterpret_cast<const uint4*>(X + static_cast<int64_t>(m0 + row) * K + k0 + kc);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kThreads, row = c >> 3, kc = (c & 7) * 8;
      br[i] = *reinterpret_cast<const uint4*>(B + static_cast<int64_t>(n0 + row) * K + k0 + kc);
    }
  };

  f32x16 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = zero16();

  gload(0);
  const int KT = K / kBK;
  for (int kt = 0; kt < KT; ++kt) {
    __syncthreads();  // the previous stage's fragment reads are done
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int c = tid + i * kThreads;
      *reinterpret_cast<uint4*>(Xs + (c >> 3) * kRS + (c & 7) * 8) = xr[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kThreads;
      *reinterpret_cast<uint4*>(Bs + (c >> 3) * kRS + (c & 7) * 8) = br[i];
    }
    __syncthreads();
    if (kt + 1 < KT) gload((kt + 1) * kBK);  // next stage's HBM reads overlap this stage's MFMAs
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ++ks) {
      bf16x8 a[FN], b[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(Bs + (wn * TN + i * 32 + r) * kRS + ks * 16 + 8 * h);
#pragma unroll
      for (int j = 0; j < FM; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(Xs + (wm * TM + j * 32 + r) * kRS + ks * 16 + 8 * h);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }

  // Epilogue: stage the bf16 tile as [BM][BN] rows in LDS, then coalesced 16-B stores.
  constexpr int CS = BN + 8;
  uint16_t* Cs = lds;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = wm * TM + j * 32 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = wn * TN + i * 32 + 8 * g + 4 * h;
        uint2 pk;
        pk.x = pack_bf16x2(acc[i][j][4 * g + 0], acc[i][j][4 * g + 1]);
        pk.y = pack_bf16x2(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
        *reinterpret_cast<uint2*>(Cs + m * CS + n) = pk;
      }
    }
  __syncthreads();
  constexpr int CPR = BN / 8;           // 16-B chunks per output row
  constexpr int RPP = kThreads / CPR;   // rows per pass
  const int cc = tid % CPR, rr = tid / CPR;
  float s[8], q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
  for (int row = rr; row < BM; row += RPP) {
    if (m0 + row >= M) break;
    const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * CS + cc * 8);
    *reinterpret_cast<uint4*>(Y + static_cast<int64_t>(m0 + row) * N + n0 + cc * 8) = v;
    if (STATS) {
      const float f[8] = {bf16_lo(v.x), bf16_hi(v.x), bf16_lo(v.y), bf16_hi(v.y),
                          bf16_lo(v.z), bf16_hi(v.z), bf16_lo(v.w), bf16_hi(v.w)};
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += f[k]; q[k] = fmaf(f[k], f[k], q[k]); }
    }
  }
  if (STATS) {
    // partial[mt][0][n] = sum, partial[mt][1][n] = sum of squares (batchnorm.hip layout)
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [RPP][CPR * 16]
    constexpr int width = CPR * 16;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[rr * width + cc * 16 + k] = s[k];
      red[rr * width + cc * 16 + 8 + k] = q[k];
    }
    __syncthreads();
    for (int o = tid; o < width; o += kThreads) {
      float a = 0.f;
      for (int j = 0; j < RPP; ++j) a += red[j * width + o];
      const int ch = n0 + (o >> 4) * 8 + (o & 7);
      partial[(static_cast<int64_t>(mt) * 2 + ((o >> 3) & 1)) * N + ch] = a;
    }
  }
}

// ------------------------------------------------------------------ weight gradient (split over m)
constexpr int kBKM = 64;  // m rows per LDS stage

template <int BCO, int BCI>
__global__ __launch_bounds__(kThreads) void wgrad_kernel(
    const uint16_t* __restrict__ dY, const uint16_t* __restrict__ X, float* __restrict__ ws,
    int M, int Cout, int Cin, int rows_per_split) {
  // Row strides = 32 (mod 128) elements: the 4 rows a transposed read touches per half-wave land
  // in 4 distinct 64-B bank groups.
  constexpr int RA = BCO + 32, RB = BCI + 32;
  constexpr int TA = BCO / 2, TB = BCI / 2;
  constexpr int FA = TA / 32, FB = TB / 32;
  constexpr int ACH = kBKM * BCO / 8 / kThreads, BCH = kBKM * BCI / 8 / kThreads;
  constexpr int ACPR = BCO / 8, BCPR = BCI / 8;
  __shared__ __attribute__((aligned(16))) uint16_t As[kBKM * RA];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[kBKM * RB];

  const int tiles_ci = Cin / BCI;
  const int tile = blockIdx.x;
  const int co0 = (tile / tiles_ci) * BCO, ci0 = (tile % tiles_ci) * BCI;
  const int split = blockIdx.y;
  const int mb = split * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wa = w & 1, wb = w >> 1;
  const int r = lane & 31, h = lane >> 5;
  const int tr_row = (r & 15) >> 2;
  const int tr_col = 16 * (r >> 4) + 4 * (r & 3);

  uint4 ar[ACH], brg[BCH];
  auto gload = [&](int m) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kThreads, row = c / ACPR, col = (c % ACPR) * 8;
      ar[i] = make_uint4(0, 0, 0, 0);
      if (m + row < me)
        ar[i] = *reinterpret_cast<const uint4*>(dY + static_cast<int64_t>(m + row) * Cout + co0 + col);
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kThreads, row = c / BCPR, col = (c % BCPR) * 8;
      brg[i] = make_uint4(0, 0, 0, 0);
      if (m + row < me)
        brg[i] = *reinterpret_cast<const uint4*>(X + static_cast<int64_t>(m + row) * Cin + ci0 + col);
    }
  };

  f32x16 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) acc[i][j] = zero16();

  if (mb < me) gload(mb);
  for (int m = mb; m < me; m += kBKM) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + i * kThreads;
      *reinterpret_cast<uint4*>(As + (c / ACPR) * RA + (c % ACPR) * 8) = ar[i];
    }
#pragma unroll
    for (int i = 0; i < BCH; ++i) {
      const int c = tid + i * kThreads;
      *reinterpret_cast<uint4*>(Bs + (c / BCPR) * RB + (c % BCPR) * 8) = brg[i];
    }
    __syncthreads();
    if (m + kBKM < me) gload(m + kBKM);
#pragma unroll
    for (int s2 = 0; s2 < kBKM / 16; ++s2) {
      // both operands use the same k permutation (rows 16*s2 + 4h + q and +8), so the MFMA's
      // k sum is over the same 16 rows of m for A and B.
      bf16x8 a[FA], b[FB];
#pragma unroll
      for (int i = 0; i < FA; ++i) {
        const uint16_t* base = As + (16 * s2 + 4 * h + tr_row) * RA + wa * TA + i * 32 + tr_col;
        a[i] = cat8(tr_read(base), tr_read(base + 8 * RA));
      }
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const uint16_t* base = Bs + (16 * s2 + 4 * h + tr_row) * RB + wb * TB + j * 32 + tr_col;
        b[j] = cat8(tr_read(base), tr_read(base + 8 * RB));
      }
#pragma unroll
      for (int i = 0; i < FA; ++i)
#pragma unroll
        for (int j = 0; j < FB; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
  }
  // fp32 partial tile -> ws[split][co][ci]
  float* out = ws + static_cast<int64_t>(split) * Cout * Cin;
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int ci = ci0 + wb * TB + j * 32 + r;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int co = co0 + wa * TA + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        out[static_cast<int64_t>(co) * Cin + ci] = acc[i][j][reg];
      }
    }
}

// dW (+)= sum over splits; 8 elements per thread.
template <typename OUT>
__global__ __launch_bounds__(kThreads) void wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                int splits, int64_t n,
                                                                void* __restrict__ dw,
                                                                bool accumulate) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (v * 8 >= n) return;
  float a[8];
  for (int k = 0; k < 8; ++k) a[k] = 0.f;
  for (int s = 0; s < splits; ++s) {
    float p[8];
    Vec8<F32>::load(ws + s * n + v * 8, p);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += p[k];
  }
  char* dst = reinterpret_cast<char*>(dw) + v * 8 * Vec8<OUT>::bytes;
  if (accumulate) {
    float o[8];
    Vec8<OUT>::load(dst, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += o[k];
  }
  Vec8<OUT>::store(dst, a);
}

// W [R][C] -> Wt [C][R], bf16, 64x64 tiles through LDS.
__global__ __launch_bounds__(kThreads) void transpose_kernel(const uint16_t* __restrict__ in,
                                                             uint16_t* __restrict__ out, int R,
                                                             int C) {
  __shared__ uint16_t tile[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += kThreads) {
    const int rr = i / 64, cc = i % 64;
    if (r0 + rr < R && c0 + cc < C) tile[rr][cc] = in[static_cast<int64_t>(r0 + rr) * C + c0 + cc];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += kThreads) {
    const int cc = i / 64, rr = i % 64;
    if (r0 + rr < R && c0 + cc < C) out[static_cast<int64_t>(c0 + cc) * R + r0 + rr] = tile[rr][cc];
  }
}

struct GemmCfg {
  int bm, bn;
};

GemmCfg gemm_cfg(int64_t M, int N) {
  static const int force_bm = [] {
    const char* e = std::getenv("DCA_PW_BM");  // tuning sweeps only
    return e ? std::atoi(e) : 0;
  }();
  const int bn = N == 64 ? 64 : 128;
  if (force_bm == 64 || force_bm == 128 || force_bm == 256) return {force_bm, bn};
  const int64_t tiles256 = (M + 255) / 256 * (N / bn);
  return {tiles256 >= 512 ? 256 : 128, bn};
}

template <int BM, int BN, bool STATS>
void launch_gemm(const void* x, const void* b, void* y, float* partial, int64_t M, int N, int K,
                 hipStream_t st) {
  constexpr size_t stage = static_cast<size_t>(BM + BN) * kRS * 2;
  constexpr size_t epi = static_cast<size_t>(BM) * (BN + 8) * 2;
  constexpr size_t lds = stage > epi ? stage : epi;
  const int grid = static_cast<int>((M + BM - 1) / BM * (N / BN));
  hipLaunchKernelGGL((gemm_rowk_kernel<BM, BN, STATS>), dim3(grid), dim3(kThreads), lds, st,
                     static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(b),
                     static_cast<uint16_t*>(y), partial, static_cast<int>(M), N, K);
}

template <bool STATS>
void gemm_dispatch(const void* x, const void* b, void* y, float* partial, int64_t M, int N, int K,
                   hipStream_t st) {
  const GemmCfg c = gemm_cfg(M, N);
  if (c.bn == 64) {
    if (c.bm == 256) launch_gemm<256, 64, STATS>(x, b, y, partial, M, N, K, st);
    else if (c.bm == 128) launch_gemm<128, 64, STATS>(x, b, y, partial, M, N, K, st);
    else launch_gemm<64, 64, STATS>(x, b, y, partial, M, N, K, st);
  } else {
    if (c.bm == 256) launch_gemm<256, 128, STATS>(x, b, y, partial, M, N, K, st);
    else if (c.bm == 128) launch_gemm<128, 128, STATS>(x, b, y, partial, M, N, K, st);
    else launch_gemm<64, 128, STATS>(x, b, y, partial, M, N, K, st);
  }
}

struct WgradCfg {
  int bco, bci, splits, rows_per_split;
};

WgradCfg wgrad_cfg(int64_t M, int Cout, int Cin) {
  WgradCfg c;
  c.bco = Cout >= 128 ? 128 : 64;
  c.bci = Cin >= 128 ? 128 : 64;
  const int tiles = (Cout / c.bco) * (Cin / c.bci);
  static const int target = [] {
    const char* e = std::getenv("DCA_PW_WG_BLOCKS");  // tuning sweeps only
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 1024;
  }();
  // ~target workgroups, at least 4 stages of m per split
  int64_t s = (target + tiles - 1) / tiles;
  const int64_t max_s = (M + 4 * kBKM - 1) / (4 * kBKM);
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  int64_t rps = (M + s - 1) / s;
  rps = (rps + kBKM - 1) / kBKM * kBKM;
  c.rows_per_split = static_cast<int>(rps);
  c.splits = static_cast<int>((M + rps - 1) / rps);
  return c;
}

}  // namespace

// ------------------------------------------------------------------ host API
int conv1x1_fwd_row_blocks(int64_t M, int N) {
  const GemmCfg c = gemm_cfg(M, N);
  return static_cast<int>((M + c.bm - 1) / c.bm);
}

void conv1x1_fwd(const void* x, const void* w, void* y, float* partial, int64_t M, int Cin,
                 int Cout, hipStream_t st) {
  if (partial) gemm_dispatch<true>(x, w, y, partial, M, Cout, Cin, st);
  else gemm_dispatch<false>(x, w, y, nullptr, M, Cout, Cin, st);
}

void conv1x1_dgrad(const void* dy, const void* w, void* wt, void* dx, int64_t M, int Cin, int Cout,
                   hipStream_t st) {
  hipLaunchKernelGGL(transpose_kernel, dim3((Cin + 63) / 64, (Cout + 63) / 64), dim3(kThreads), 0,
                     st, static_cast<const uint16_t*>(w), static_cast<uint16_t*>(wt), Cout, Cin);
  gemm_dispatch<false>(dy, wt, dx, nullptr, M, Cin, Cout, st);
}

int64_t conv1x1_wgrad_ws_floats(int64_t M, int Cin, int Cout) {
  const WgradCfg c = wgrad_cfg(M, Cout, Cin);
  return static_cast<int64_t>(c.splits) * Cout * Cin;
}

void conv1x1_wgrad(const void* dy, const void* x, float* ws, void* dw, bool dw_f32,
                   bool accumulate, int64_t M, int Cin, int Cout, hipStream_t st) {
  const WgradCfg c = wgrad_cfg(M, Cout, Cin);
  const dim3 grid((Cout / c.bco) * (Cin / c.bci), c.splits);
  const auto* a = static_cast<const uint16_t*>(dy);
  const auto* b = static_cast<const uint16_t*>(x);
  const int m = static_cast<int>(M);
  if (c.bco == 128 && c.bci == 128)
    hipLaunchKernelGGL((wgrad_kernel<128, 128>), grid, dim3(kThreads), 0, st, a, b, ws, m, Cout, Cin, c.rows_per_split);
  else if (c.bco == 128)
    hipLaunchKernelGGL((wgrad_kernel<128, 64>), grid, dim3(kThreads), 0, st, a, b, ws, m, Cout, Cin, c.rows_per_split);
  else if (c.bci == 128)
    hipLaunchKernelGGL((wgrad_kernel<64, 128>), grid, dim3(kThreads), 0, st, a, b, ws, m, Cout, Cin, c.rows_per_split);
  else
    hipLaunchKernelGGL((wgrad_kernel<64, 64>), grid, dim3(kThreads), 0, st, a, b, ws, m, Cout, Cin, c.rows_per_split);
  const int64_t n = static_cast<int64_t>(Cout) * Cin;
  const int rg = static_cast<int>((n / 8 + kThreads - 1) / kThreads);
  if (dw_f32)
    hipLaunchKernelGGL(wgrad_reduce_kernel<F32>, dim3(rg), dim3(kThreads), 0, st, ws, c.splits, n, dw, accumulate);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<BF16>, dim3(rg), dim3(kThreads), 0, st, ws, c.splits, n, dw, accumulate);
}

}  // namespace dca
