// k x k NHWC convolutions of the ResNet-50 bottleneck (3x3, stride 1 or 2, padding 1) as implicit
// GEMMs on gfx950 MFMA, with the following BatchNorm's statistics fused into the forward epilogue.
//
// The reference trains torchvision's resnet50 through cuDNN (examples/deepspeed_autotune/
// torchvision, harness/determined/pytorch/_pytorch_trial.py); on MI355X MIOpen's NHWC solvers run
// the 3x3 convolutions at 360-900 TFLOP/s (profiles/round3_conv3x3_miopen_bs1024.txt, 28% of the
// bs-1024 step). GEMM view, NHWC activations and [K][R][S][C] (channels_last) weights:
//   y[m = (n, p, q)][k] = sum_{(r, s, c)} x[n][p*str + r - pad][q*str + s - pad][c] * w[k][r][s][c]
// i.e. M = N*P*Q output pixels, Ngemm = K, Kgemm = R*S*C, visited as R*S*C/64 stages of one tap and
// 64 channels. The stride-1 data gradient is the same kernel on dy with the flipped, transposed
// weight w'[c][r][s][k] = w[k][R-1-r][S-1-s][c] and padding R-1-pad.
//
// Kernel structure (cdna_hip_programming.md §5: 2-phase glds pipeline):
//  * 256 threads = 4 waves in a WM x WN grid; block tile BM pixels x BN channels; LDS holds two
//    stages of [BM rows][64] (pixels) + [BN rows][64] (weights), 128-B rows;
//  * every stage is loaded by global_load_lds_dwordx4 (16 B per lane, 8 rows per wave
//    instruction, no VGPR staging); the im2col gather is the per-lane SOURCE address: a padding
//    tap reads a 16-B block of zeros in device memory, so the LDS image stays lane-linear;
//  * rows are XOR-swizzled in 16-B chunks by (row >> 1) & 7 -- applied to the source chunk a lane
//    fetches and to the ds_read_b128 fragment address (guide rule 21: both sides or neither), which
//    makes the 16-lane groups of the MFMA fragment reads conflict-free on 128-B rows;
//  * v_mfma_f32_32x32x16_bf16 computes the TRANSPOSED tile (rows = output channels, cols = pixels)
//    so every lane holds 4 consecutive channels of one pixel: the epilogue packs 8-B LDS writes,
//    streams the tile out with 16-B coalesced stores and -- forward -- reduces per-channel
//    (sum, sum^2) of the bf16-rounded outputs into batchnorm.hip's partial-statistics layout;
//  * one barrier per stage: issue the NEXT stage's loads, compute the current one, then
//    vmcnt(0) + barrier (the "minimum 2-phase" loop of guide T3/T4);
//  * tiles are dealt XCD-contiguously (neighbouring pixel tiles share input rows in an XCD's L2).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "conv_api.h"

namespace dca {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int kBK = 64;  // k elements (channels of one tap) per stage

// 16-B block of zeros that padding taps read (static device memory is zero-initialised).
__device__ __attribute__((aligned(64))) uint16_t g_zero_block[32];

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* src, void* lds_dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds_dst), 16, 0, 0);
}

__device__ __forceinline__ int xcd_swizzle(int id, int G) {
  // bijective for any G: block ids that share an XCD (id % 8) get one contiguous range of tiles
  const int q = G >> 3, r = G & 7, xcd = id & 7, k = id >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Workgroup barrier that does not drain the vector-memory counter; the empty asm keeps the
// compiler from moving LDS accesses across it.
__device__ __forceinline__ void barrier_raw() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// buffer_load_dwordx4 ... lds: a 16-B piece per lane straight into LDS (wave-uniform LDS base +
// lane * 16). The buffer descriptor's range check returns zeros for an offset past num_records:
// padding taps and rows past M pass kOOB instead of branching to a zero block.
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t soff,
                                       void* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      rsrc, (__attribute__((address_space(3))) void*)(lds_dst), 16, voff, soff, 0, 0);
}

// Epilogue modes (EPI):
//   kEpiNone  -- store y;
//   kEpiStats -- also reduce (sum y, sum y^2) of the bf16 outputs -- the following BatchNorm's
//                statistics -- into partial[mt][2][K] (batchnorm.hip's layout). (The backward form,
//                BatchNorm backward statistics in the data-gradient epilogue, measured -0.4 % on the
//                step and was removed: profiles/round5_dgrad_bn_stats_epilogue_ab.txt.)
constexpr int kEpiNone = 0, kEpiStats = 1;
template <int BM, int BN, int WM, int WN, int NSTAGE, int EPI>
__global__ __launch_bounds__(kThreads, 2) void conv_fwd_kernel(
    const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, uint16_t* __restrict__ y,
    float* __restrict__ partial, ConvGeom g) {
  constexpr bool STATS = EPI == kEpiStats;
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN / WN;  // wave tile: pixels x channels
  constexpr int FM = TM / 32, FN = TN / 32;
  static_assert(FM >= 1 && FN >= 1, "wave tile below one 32x32 MFMA tile");
  constexpr int A_INS = BM / 32;  // buffer-lds loads per wave per stage (8 rows x 128 B each)
  constexpr int B_INS = BN / 32;
  constexpr int STAGE = (BM + BN) * kBK;  // elements per LDS stage
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int NT = g.K / BN;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int mt = t / NT, nt = t - mt * NT;
  const int m0 = mt * BM, n0 = nt * BN;
  const int PQ = g.P * g.Q;
  const int CT = g.C / kBK;
  const int KT = g.R * g.S * CT;

  // num_records in bytes (< 2^31 by the host checks, so kOOB is always out of range)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(x), 0, static_cast<int>(static_cast<uint32_t>(g.N * g.H * g.W) * g.C * 2u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(w), 0, static_cast<int>(static_cast<uint32_t>(g.K * g.R * g.S * g.C) * 2u),
      0x00020000);

  // ---- per-lane gather state: for each A load, the output pixel's input origin
  uint32_t a_vo[A_INS];  // byte offset of x[n][ih0][iw0][chunk*8] (wraps for pad rows; never used then)
  int a_ih[A_INS], a_iw[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int j = wv + 4 * i;
    const int row = 8 * j + (lane >> 3);
    const int m = m0 + row;
    const int chunk = (lane & 7) ^ swz(row);
    if (m < g.M) {
      const int n = m / PQ, rem = m - n * PQ, p = rem / g.Q, q = rem - p * g.Q;
      a_ih[i] = p * g.stride - g.pad;
      a_iw[i] = q * g.stride - g.pad;
      a_vo[i] = static_cast<uint32_t>((((n * g.H + a_ih[i]) * g.W + a_iw[i]) * g.C + chunk * 8) * 2);
    } else {
      a_ih[i] = -(1 << 20);  // never valid
      a_iw[i] = 0;
      a_vo[i] = kOOB;
    }
  }
  const int RSC = g.R * g.S * g.C;
  uint32_t b_vo[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int j = wv + 4 * i;
    const int row = 8 * j + (lane >> 3);
    b_vo[i] = static_cast<uint32_t>(((n0 + row) * RSC + ((lane & 7) ^ swz(row)) * 8) * 2);
  }

  // the stage to load next, as loop-carried (tap r, s; channel chunk cc) counters -- no divisions
  int ld_r = 0, ld_s = 0, ld_cc = 0;
  auto stage = [&](int buf) {
    const uint32_t tap_b = static_cast<uint32_t>(((ld_r * g.W + ld_s) * g.C + ld_cc * kBK) * 2);
    uint16_t* As = lds + buf * STAGE;
    uint16_t* Bs = As + BM * kBK;
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      const int j = wv + 4 * i;
      const bool ok = static_cast<unsigned>(a_ih[i] + ld_r) < static_cast<unsigned>(g.H) &&
                      static_cast<unsigned>(a_iw[i] + ld_s) < static_cast<unsigned>(g.W);
      blds16(xr, ok ? a_vo[i] + tap_b : kOOB, 0, As + j * 8 * kBK);
    }
    const uint32_t wk = static_cast<uint32_t>(((ld_r * g.S + ld_s) * g.C + ld_cc * kBK) * 2);
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int j = wv + 4 * i;
      blds16(wr, b_vo[i], wk, Bs + j * 8 * kBK);
    }
    if (++ld_cc == CT) {
      ld_cc = 0;
      if (++ld_s == g.S) {
        ld_s = 0;
        ++ld_r;
      }
    }
  };

  const int wm = wv % WM, wn = wv / WM;
  const int r32 = lane & 31, h = lane >> 5;

  f32x16 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // fragment addresses (element offsets inside a stage) for k-substep ks
  auto frag = [&](const uint16_t* base, int row, int ks) {
    return *reinterpret_cast<const bf16x8*>(base + row * kBK + (((2 * ks + h) ^ swz(row)) << 3));
  };

  // NSTAGE-deep LDS ring: stages kt+1 .. kt+NSTAGE-1 are in flight while stage kt is computed.
  // Every wave issues LPS loads per stage, so "stage kt+1 landed" is vmcnt(LPS * (stages issued
  // after it)); raw s_barrier (not __syncthreads, which would drain vmcnt to 0) publishes it.
  constexpr int LPS = A_INS + B_INS;
#pragma unroll
  for (int p = 0; p < NSTAGE - 1; ++p)
    if (p < KT) stage(p);
  if constexpr (NSTAGE == 3) {
    if (KT > 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
  } else {
    wait_vmcnt<0>();
  }
  barrier_raw();
  int buf = 0;
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NSTAGE - 1 < KT) {
      int nb = buf + NSTAGE - 1;
      if (nb >= NSTAGE) nb -= NSTAGE;
      stage(nb);
    }
    const uint16_t* As = lds + buf * STAGE;
    const uint16_t* Bs = As + BM * kBK;
    // fragments of substep ks+1 are read while the MFMAs of ks run
    bf16x8 a0[FN], b0[FM], a1[FN], b1[FM];
#pragma unroll
    for (int i = 0; i < FN; ++i) a0[i] = frag(Bs, wn * TN + i * 32 + r32, 0);
#pragma unroll
    for (int j = 0; j < FM; ++j) b0[j] = frag(As, wm * TM + j * 32 + r32, 0);
#pragma unroll
    for (int ks = 0; ks < kBK / 16; ks += 2) {
#pragma unroll
      for (int i = 0; i < FN; ++i) a1[i] = frag(Bs, wn * TN + i * 32 + r32, ks + 1);
#pragma unroll
      for (int j = 0; j < FM; ++j) b1[j] = frag(As, wm * TM + j * 32 + r32, ks + 1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma32(a0[i], b0[j], acc[i][j]);
      if (ks + 2 < kBK / 16) {
#pragma unroll
        for (int i = 0; i < FN; ++i) a0[i] = frag(Bs, wn * TN + i * 32 + r32, ks + 2);
#pragma unroll
        for (int j = 0; j < FM; ++j) b0[j] = frag(As, wm * TM + j * 32 + r32, ks + 2);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = mfma32(a1[i], b1[j], acc[i][j]);
    }
    // stage kt+1 must have landed; later stages may stay in flight
    if constexpr (NSTAGE == 3) {
      if (kt + 2 < KT) wait_vmcnt<LPS>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    barrier_raw();
    buf = buf + 1 == NSTAGE ? 0 : buf + 1;
  }

  // ---- epilogue: bf16 tile -> LDS [BM][BN + 8] -> 16-B coalesced stores (+ BN statistics)
  constexpr int CS = BN + 8;
  uint16_t* Cs = lds;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = wm * TM + j * 32 + r32;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const int n = wn * TN + i * 32 + 8 * q4 + 4 * h;
        uint2 pk;
        pk.x = pack_bf16x2(acc[i][j][4 * q4 + 0], acc[i][j][4 * q4 + 1]);
        pk.y = pack_bf16x2(acc[i][j][4 * q4 + 2], acc[i][j][4 * q4 + 3]);
        *reinterpret_cast<uint2*>(Cs + m * CS + n) = pk;
      }
    }
  __syncthreads();
  constexpr int CPR = BN / 8;          // 16-B chunks per output row
  constexpr int RPP = kThreads / CPR;  // rows per pass
  const int cc = tid % CPR, rr = tid / CPR;
  float s8[8], q8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s8[k] = 0.f;
    q8[k] = 0.f;
  }
  for (int row = rr; row < BM; row += RPP) {
    if (m0 + row >= g.M) break;
    const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * CS + cc * 8);
    const int64_t off = static_cast<int64_t>(m0 + row) * g.K + n0 + cc * 8;
    *reinterpret_cast<uint4*>(y + off) = v;
    if constexpr (STATS) {
      const float f[8] = {bf16_lo(v.x), bf16_hi(v.x), bf16_lo(v.y), bf16_hi(v.y),
                          bf16_lo(v.z), bf16_hi(v.z), bf16_lo(v.w), bf16_hi(v.w)};
#pragma unroll
      for (int k = 0; k < 8; ++k) { s8[k] += f[k]; q8[k] = fmaf(f[k], f[k], q8[k]); }
    }
  }
  if constexpr (EPI != kEpiNone) {
    // partial[mt][0][k] = sum, partial[mt][1][k] = sum of squares (batchnorm.hip layout)
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);  // [RPP][CPR * 16]
    constexpr int width = CPR * 16;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[rr * width + cc * 16 + k] = s8[k];
      red[rr * width + cc * 16 + 8 + k] = q8[k];
    }
    __syncthreads();
    for (int o = tid; o < width; o += kThreads) {
      float a = 0.f;
      for (int j = 0; j < RPP; ++j) a += red[j * width + o];
      const int ch = n0 + (o >> 4) * 8 + (o & 7);
      partial[(static_cast<int64_t>(mt) * 2 + ((o >> 3) & 1)) * g.K + ch] = a;
    }
  }
}

// w [K][R][S][C] -> wt [C][R][S][K] with the taps flipped (the stride-1 data-gradient weight).
__global__ __launch_bounds__(kThreads) void flip_transpose_kernel(const uint16_t* __restrict__ w,
                                                                  uint16_t* __restrict__ wt, int K,
                                                                  int C, int RS) {
  __shared__ uint16_t tile[64][65];
  const int tap = blockIdx.z;
  const int k0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += kThreads) {
    const int kk = i / 64, c = i % 64;
    if (k0 + kk < K && c0 + c < C)
      tile[kk][c] = w[(static_cast<int64_t>(k0 + kk) * RS + tap) * C + c0 + c];
  }
  __syncthreads();
  const int ftap = RS - 1 - tap;
  for (int i = threadIdx.x; i < 64 * 64; i += kThreads) {
    const int c = i / 64, kk = i % 64;
    if (k0 + kk < K && c0 + c < C)
      wt[(static_cast<int64_t>(c0 + c) * RS + ftap) * K + k0 + kk] = tile[kk][c];
  }
}

// ------------------------------------------------------------------ weight gradient
// dW[k][r][s][c] = sum_m dy[m][k] * x[n][p*str + r - pad][q*str + s - pad][c]: a GEMM with the
// 10^4..10^6 output pixels as its reduction. Grid = (k tile, tap, c tile) x pixel splits; each
// workgroup streams 64-pixel stages of dy [64][BKO] and of the tap-shifted x [64][BC] (zero rows
// for padding / past the split) into LDS by global_load_lds, and both MFMA operands come out of
// those m-major images through ds_read_b64_tr_b16 (guide T10): lane (r, h) of a 32x32x16 fragment
// takes column r of rows 16ks + 8h + 0..7 with two transposed reads, the same rows for dy and x
// so the k sums match. 16-B chunks are XOR-swizzled by row (f = (row & 3) << 2 on 256-B rows,
// ((row >> 1) & 1) << 2 on 128-B rows) so the 4 rows x 64 B of a 32-lane transposed read hit 64
// distinct banks. fp32 split tiles go to a workspace; wgrad_reduce_kernel sums them in a fixed
// order (deterministic) into dW, optionally accumulating into the parameter's .grad view.
template <int ROWB>
__device__ __forceinline__ int wswz(int row) {
  if constexpr (ROWB == 256) return (row & 3) << 2;
  return ((row >> 1) & 1) << 2;
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ s16x4 tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

__device__ __forceinline__ bf16x8 cat8(s16x4 a, s16x4 b) {
  const s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// floor(a / d) for 0 <= a < 2^24 via the float reciprocal, corrected to exact.
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
  int q = static_cast<int>(static_cast<float>(a) * inv);
  q += (q + 1) * d <= a;
  q -= q * d > a;
  return q;
}

constexpr int kWM = 64;  // pixels per stage

template <int BKO, int BC>
__global__ __launch_bounds__(kThreads, 2) void conv_wgrad_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, float* __restrict__ ws,
    ConvGeom g, int rows_per_split, float inv_pq, float inv_q) {
  constexpr int TA = BKO / 2, TB = BC / 2;  // wave tile (2 x 2 waves)
  constexpr int FA = TA / 32, FB = TB / 32;
  constexpr int RA = BKO * 2, RB = BC * 2;          // LDS row bytes
  constexpr int LA = RA / 16, LB = RB / 16;          // lanes per row in a glds instruction
  constexpr int IA = kWM * BKO * 2 / 1024 / 4;       // glds per wave per stage
  constexpr int IB = kWM * BC * 2 / 1024 / 4;
  constexpr int STAGE = kWM * (BKO + BC);            // elements
  static_assert(IA >= 1 && IB >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int CT = g.C / BC, RS = g.R * g.S;
  int t = blockIdx.x;
  const int ct = t % CT;
  t /= CT;
  const int tap = t % RS;
  const int kt = t / RS;
  const int k0 = kt * BKO, c0 = ct * BC;
  const int r = tap / g.S, s = tap - r * g.S;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(g.M, mb + rows_per_split);
  const int PQ = g.P * g.Q;

  // buffer loads into LDS with hardware out-of-range zeros (see conv_fwd_kernel); the x rows of
  // each lane advance 64 pixels per stage, so their (n, p, q) are carried, not divided for
  const __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(dy), 0, static_cast<int>(static_cast<uint32_t>(g.M) * g.K * 2u), 0x00020000);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(x), 0, static_cast<int>(static_cast<uint32_t>(g.N * g.H * g.W) * g.C * 2u),
      0x00020000);
  // Loader state, all carried incrementally (round 6: the per-stage address math -- three 32-bit
  // multiplies, a 64-bit multiply-add and a data-dependent carry loop per x row -- was ~150 VALU
  // per 16 MFMAs in the ISA, more than the matrix work):
  //  * dy rows: byte offset of (row m, channel k0 + chunk) advanced by kWM * K * 2 per stage;
  //  * x rows: the output pixel's (p, q), its input coordinates (ih, iw) at this workgroup's tap and
  //    the byte offset of x[n][ih][iw][c0 + chunk], advanced by kWM pixels per stage with at most one
  //    q-wrap and one p-wrap (kWM % Q < Q and (kWM / Q) % P + 1 <= P); the offset may leave the
  //    tensor while the tap is a padding tap (unsigned wrap-around), it is only used when valid.
  uint32_t dy_vo[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int j = wv + 4 * i;
    const int row = j * (64 / LA) + lane / LA;
    const int chunk = (lane % LA) ^ wswz<RA>(row);
    dy_vo[i] = (static_cast<uint32_t>(mb + row) * g.K + static_cast<uint32_t>(k0 + chunk * 8)) * 2u;
  }
  const uint32_t dy_step = static_cast<uint32_t>(kWM) * g.K * 2u;
  const int C2 = g.C * 2;
  const int st = g.stride;
  int xq[IB], xp[IB], xih[IB], xiw[IB];
  uint32_t xvo[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int j = wv + 4 * i;
    const int row = j * (64 / LB) + lane / LB;
    const int m = mb + row;
    const int n = fdiv(m, PQ, inv_pq);
    const int rem = m - n * PQ;
    xp[i] = fdiv(rem, g.Q, inv_q);
    xq[i] = rem - xp[i] * g.Q;
    xih[i] = xp[i] * st - g.pad + r;
    xiw[i] = xq[i] * st - g.pad + s;
    xvo[i] = static_cast<uint32_t>((n * g.H + xih[i]) * g.W + xiw[i]) * static_cast<uint32_t>(C2) +
             static_cast<uint32_t>((c0 + ((lane % LB) ^ wswz<RB>(row)) * 8) * 2);
  }
  // per-stage deltas (uniform): kWM pixels = dn images + dp rows + dq columns
  const int dq = kWM % g.Q, dp = (kWM / g.Q) % g.P, dn = kWM / PQ;
  const uint32_t a_q = static_cast<uint32_t>(st * C2), a_p = static_cast<uint32_t>(st * g.W * C2),
                 a_n = static_cast<uint32_t>(g.H * g.W * C2);
  const uint32_t d_step = dn * a_n + dp * a_p + dq * a_q;
  const uint32_t d_qwrap = a_p - static_cast<uint32_t>(g.Q) * a_q;  // q -= Q, p += 1
  const uint32_t d_pwrap = a_n - static_cast<uint32_t>(g.P) * a_p;  // p -= P, n += 1

  auto stage = [&](int m_base, int buf) {
    uint16_t* As = lds + buf * STAGE;
    uint16_t* Bs = As + kWM * BKO;
    const int lim = me - m_base;  // rows of this stage inside the split
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int j = wv + 4 * i;                  // instruction index within the tile
      const int row = j * (64 / LA) + lane / LA;
      blds16(dyr, row < lim ? dy_vo[i] : kOOB, 0, As + j * 512);
      dy_vo[i] += dy_step;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int j = wv + 4 * i;
      const int row = j * (64 / LB) + lane / LB;
      const bool ok = row < lim && static_cast<unsigned>(xih[i]) < static_cast<unsigned>(g.H) &&
                      static_cast<unsigned>(xiw[i]) < static_cast<unsigned>(g.W);
      blds16(xr, ok ? xvo[i] : kOOB, 0, Bs + j * 512);
      // advance this row by kWM pixels
      int q = xq[i] + dq, p = xp[i] + dp;
      int ih = xih[i] + dp * st, iw = xiw[i] + dq * st;
      uint32_t vo = xvo[i] + d_step;
      if (q >= g.Q) { q -= g.Q; iw -= g.Q * st; ++p; ih += st; vo += d_qwrap; }
      if (p >= g.P) { p -= g.P; ih -= g.P * st; vo += d_pwrap; }
      xq[i] = q; xp[i] = p; xih[i] = ih; xiw[i] = iw; xvo[i] = vo;
    }
  };

  const int wa = wv & 1, wb = wv >> 1;
  // transposed read: lane 4q + p of a 16-lane group addresses row q, columns 4p .. 4p+3
  const int h = lane >> 5, gq = (lane >> 2) & 3, gp = lane & 3, half16 = (lane >> 4) & 1;

  f32x16 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int nst = (me - mb + kWM - 1) / kWM;
  if (nst > 0) stage(mb, 0);
  wait_vmcnt<0>();
  barrier_raw();
  for (int it = 0; it < nst; ++it) {
    const int buf = it & 1;
    if (it + 1 < nst) stage(mb + (it + 1) * kWM, buf ^ 1);
    const uint16_t* As = lds + buf * STAGE;
    const uint16_t* Bs = As + kWM * BKO;
#pragma unroll
    for (int ks = 0; ks < kWM / 16; ++ks) {
      const int row0 = 16 * ks + 8 * h + gq;  // + 4 for the second read
      bf16x8 a[FA], b[FB];
#pragma unroll
      for (int i = 0; i < FA; ++i) {
        const int col = wa * TA + i * 32 + half16 * 16 + 4 * gp;
        const int ch = col >> 3, off = col & 7;
        const uint16_t* p0 = As + row0 * BKO + (((ch ^ wswz<RA>(row0)) << 3) | off);
        const uint16_t* p1 = As + (row0 + 4) * BKO + (((ch ^ wswz<RA>(row0 + 4)) << 3) | off);
        a[i] = cat8(tr_read(p0), tr_read(p1));
      }
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int col = wb * TB + j * 32 + half16 * 16 + 4 * gp;
        const int ch = col >> 3, off = col & 7;
        const uint16_t* p0 = Bs + row0 * BC + (((ch ^ wswz<RB>(row0)) << 3) | off);
        const uint16_t* p1 = Bs + (row0 + 4) * BC + (((ch ^ wswz<RB>(row0 + 4)) << 3) | off);
        b[j] = cat8(tr_read(p0), tr_read(p1));
      }
#pragma unroll
      for (int i = 0; i < FA; ++i)
#pragma unroll
        for (int j = 0; j < FB; ++j) acc[i][j] = mfma32(a[i], b[j], acc[i][j]);
    }
    wait_vmcnt<0>();
    barrier_raw();
  }
  // fp32 split tile -> ws[split][k][tap][c] (the weight's own [K][R][S][C] order)
  float* out = ws + static_cast<int64_t>(blockIdx.y) * g.K * RS * g.C;
  const int cl = lane & 31;
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int c = c0 + wb * TB + j * 32 + cl;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int k = k0 + wa * TA + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        out[(static_cast<int64_t>(k) * RS + tap) * g.C + c] = acc[i][j][reg];
      }
    }
}

// dW (+)= sum over splits in a fixed order; 8 elements per thread. The workspace is in the
// weight's [K][R][S][C] order; `kcrs` writes dW in [K][C][R][S] order instead (a contiguous NCHW
// .grad view of a channels_last parameter).
template <typename OUT>
__global__ __launch_bounds__(kThreads) void wgrad_reduce_kernel(const float* __restrict__ ws,
                                                                int splits, int64_t n,
                                                                void* __restrict__ dw,
                                                                bool accumulate, bool kcrs, int RS,
                                                                int C) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (v * 8 >= n) return;
  float a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = 0.f;
  for (int sp = 0; sp < splits; ++sp) {
    float p[8];
    Vec8<F32>::load(ws + sp * n + v * 8, p);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += p[k];
  }
  if (!kcrs || RS == 1) {
    char* dst = reinterpret_cast<char*>(dw) + v * 8 * Vec8<OUT>::bytes;
    if (accumulate) {
      float o[8];
      Vec8<OUT>::load(dst, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) a[k] += o[k];
    }
    Vec8<OUT>::store(dst, a);
    return;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t e = v * 8 + k;  // [K][RS][C]
    const int64_t c = e % C, rest = e / C;
    const int64_t tap = rest % RS, kk = rest / RS;
    const int64_t d = (kk * C + c) * RS + tap;
    float o = accumulate ? Elem<OUT>::get(dw, d) : 0.f;
    Elem<OUT>::put(dw, d, a[k] + o);
  }
}

struct WgCfg {
  int bko, bc, splits, rows_per_split;
};

WgCfg wgrad_cfg(const ConvGeom& g) {
  constexpr int target = 1024;  // workgroups to aim for (tiles x pixel splits)
  WgCfg c;
  c.bko = g.K % 128 == 0 ? 128 : 64;
  c.bc = g.C % 128 == 0 ? 128 : 64;
  const int tiles = (g.K / c.bko) * g.R * g.S * (g.C / c.bc);
  int64_t sp = (target + tiles - 1) / tiles;
  const int64_t max_sp = (g.M + 8 * kWM - 1) / (8 * kWM);  // >= 8 stages per split
  if (sp > max_sp) sp = max_sp;
  if (sp < 1) sp = 1;
  int64_t rps = (g.M + sp - 1) / sp;
  rps = (rps + kWM - 1) / kWM * kWM;
  c.rows_per_split = static_cast<int>(rps);
  c.splits = static_cast<int>((g.M + rps - 1) / rps);
  return c;
}

template <int BKO, int BC>
void launch_wgrad(const void* dy, const void* x, float* ws, const ConvGeom& g, const WgCfg& c,
                  hipStream_t st) {
  constexpr size_t lds = static_cast<size_t>(kWM) * (BKO + BC) * 2 * 2;
  const dim3 grid((g.K / BKO) * g.R * g.S * (g.C / BC), c.splits);
  auto kern = conv_wgrad_kernel<BKO, BC>;
  static const bool attr = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, grid, dim3(kThreads), lds, st, static_cast<const uint16_t*>(dy),
                     static_cast<const uint16_t*>(x), ws, g, c.rows_per_split,
                     1.0f / static_cast<float>(g.P * g.Q), 1.0f / static_cast<float>(g.Q));
}

struct Cfg {
  int bm, bn;
};

Cfg pick(const ConvGeom& g) {
  Cfg c;
  c.bn = g.K % 128 == 0 ? 128 : 64;
  // 256 x 64 (80 KB of stages) and 128 x 128 (64 KB) both keep two workgroups per CU; 256 x 128
  // (96 KB) would keep one and measured 10-20% slower (profiles/round4_igemm_v2_stages.txt)
  c.bm = c.bn == 64 ? 256 : 128;
  return c;
}

// LDS ring depth 2: two workgroups per CU fit for tiles up to 80 KB of stages, which measured
// faster than a 3-deep ring at one workgroup per CU (profiles/round4_igemm_v2_stages.txt).
template <int BM, int BN, int EPI>
void launch_fwd(const void* x, const void* w, void* y, float* partial, const ConvGeom& g,
                hipStream_t st) {
  constexpr int NSTAGE = 2;
  constexpr int WM = BN >= 128 ? 2 : 4, WN = 4 / WM;
  constexpr size_t stage = static_cast<size_t>(BM + BN) * kBK * 2 * NSTAGE;
  constexpr size_t epi = static_cast<size_t>(BM) * (BN + 8) * 2;
  constexpr size_t lds = stage > epi ? stage : epi;
  const int grid = static_cast<int>((static_cast<int64_t>(g.M) + BM - 1) / BM * (g.K / BN));
  auto kern = conv_fwd_kernel<BM, BN, WM, WN, NSTAGE, EPI>;
  static const bool attr = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, st,
                     static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w),
                     static_cast<uint16_t*>(y), partial, g);
}

template <int EPI>
void fwd_dispatch(const void* x, const void* w, void* y, float* partial, const ConvGeom& g,
                  hipStream_t st) {
  const Cfg c = pick(g);
  if (c.bn == 128) launch_fwd<128, 128, EPI>(x, w, y, partial, g, st);
  else launch_fwd<256, 64, EPI>(x, w, y, partial, g, st);
}

}  // namespace

// ------------------------------------------------------------------ host API
int conv_igemm_row_blocks(const ConvGeom& g) {
  const Cfg c = pick(g);
  return static_cast<int>((static_cast<int64_t>(g.M) + c.bm - 1) / c.bm);
}

void conv_igemm_fwd(const void* x, const void* w, void* y, float* partial, const ConvGeom& g,
                    hipStream_t st) {
  if (partial) fwd_dispatch<kEpiStats>(x, w, y, partial, g, st);
  else fwd_dispatch<kEpiNone>(x, w, y, nullptr, g, st);
}

int64_t conv_igemm_wgrad_ws_floats(const ConvGeom& g) {
  const WgCfg c = wgrad_cfg(g);
  return static_cast<int64_t>(c.splits) * g.K * g.R * g.S * g.C;
}

void conv_igemm_wgrad(const void* dy, const void* x, float* ws, void* dw, bool dw_f32,
                      bool accumulate, bool dw_kcrs, const ConvGeom& g, hipStream_t st) {
  const WgCfg c = wgrad_cfg(g);
  if (c.bko == 128 && c.bc == 128) launch_wgrad<128, 128>(dy, x, ws, g, c, st);
  else if (c.bko == 128) launch_wgrad<128, 64>(dy, x, ws, g, c, st);
  else if (c.bc == 128) launch_wgrad<64, 128>(dy, x, ws, g, c, st);
  else launch_wgrad<64, 64>(dy, x, ws, g, c, st);
  const int64_t n = static_cast<int64_t>(g.K) * g.R * g.S * g.C;
  const int rg = static_cast<int>((n / 8 + kThreads - 1) / kThreads);
  const int RS = g.R * g.S;
  if (dw_f32)
    hipLaunchKernelGGL(wgrad_reduce_kernel<F32>, dim3(rg), dim3(kThreads), 0, st, ws, c.splits, n, dw,
                       accumulate, dw_kcrs, RS, g.C);
  else
    hipLaunchKernelGGL(wgrad_reduce_kernel<BF16>, dim3(rg), dim3(kThreads), 0, st, ws, c.splits, n, dw,
                       accumulate, dw_kcrs, RS, g.C);
}

// dx[n][s*i][s*j][:] += small[n][i][j][:] (NHWC bf16): the projection shortcut's data gradient of
// a stride-s downsampling block added in place at the strided positions of conv1's data gradient.
// One lane per 16 B (8 channels), fp32 add, grid-stride; ATen's generic strided add ran this at
// 1.1-2.5 TB/s (64-bit index arithmetic per element, 2-byte accesses; round-4 step breakdown).
__global__ __launch_bounds__(256) void strided_accumulate_kernel(uint16_t* __restrict__ dx,
                                                                 const uint16_t* __restrict__ small,
                                                                 int64_t n_vec, int c8, int Wo, int Ho,
                                                                 int W, int H, int s) {
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n_vec;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int cv = static_cast<int>(t % c8);
    const int64_t pix = t / c8;  // (n, i, j) of the small tensor
    const int j = static_cast<int>(pix % Wo);
    const int64_t ni = pix / Wo;
    const int i = static_cast<int>(ni % Ho);
    const int64_t n = ni / Ho;
    const int64_t dpix = (n * H + static_cast<int64_t>(s) * i) * W + static_cast<int64_t>(s) * j;
    uint4* dp = reinterpret_cast<uint4*>(dx + (dpix * c8 + cv) * 8);
    const uint4 a = *dp;
    const uint4 b = *reinterpret_cast<const uint4*>(small + t * 8);
    auto add2 = [](uint32_t x, uint32_t y) {
      const float lo = __uint_as_float(x << 16) + __uint_as_float(y << 16);
      const float hi = __uint_as_float(x & 0xffff0000u) + __uint_as_float(y & 0xffff0000u);
      return pack_bf16x2(lo, hi);
    };
    *dp = make_uint4(add2(a.x, b.x), add2(a.y, b.y), add2(a.z, b.z), add2(a.w, b.w));
  }
}

void strided_accumulate(void* dx, const void* small, int N, int H, int W, int C, int Ho, int Wo,
                        int s, hipStream_t st) {
  const int c8 = C / 8;
  const int64_t n_vec = static_cast<int64_t>(N) * Ho * Wo * c8;
  const int64_t blocks = std::min<int64_t>((n_vec + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(strided_accumulate_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     static_cast<uint16_t*>(dx), static_cast<const uint16_t*>(small), n_vec, c8, Wo,
                     Ho, W, H, s);
}

// Space-to-depth of the 3-channel stem image with its 3-pixel zero padding in the same pass:
// x [N][H][W][3] (NHWC bf16) -> xs [N][(H+6)/2][(W+6)/2][12], channel (dy, dx, c) of output pixel
// (i, j) = x[2i+dy-3][2j+dx-3][c] or 0 outside the image. Replaces ATen's pad (fill + copy) and
// the strided reshape copy (423 us of the ResNet-50 bs-1024 step, profiles/round5_stem_conv_kernel_ab.txt).
// Row kernel: a block owns output rows 2b and 2b+1 (n * Ho + i numbering); each half-block brings
// its row's two input rows (contiguous, 6W bytes each) into LDS with 16-byte nontemporal loads,
// then the block writes its 2 * Wo * 24 contiguous output bytes as 16-byte stores (8 channels a
// lane, 16-byte aligned: 48 * Wo * b). Needs 6W % 16 == 0 (W % 8 == 0); other widths take the
// per-pixel kernel below. Dynamic LDS: 4 input rows, 24W bytes.
constexpr int kS2dMaxW = 2048;
template <int CO>
__global__ __launch_bounds__(256) void stem_s2d_rows_kernel(const uint16_t* __restrict__ x,
                                                            uint16_t* __restrict__ xs, int rows_out,
                                                            int Wo, int Ho, int W, int H) {
  extern __shared__ uint4 tile[];  // [half][dy][W * 3 / 8]
  const int h = threadIdx.x >> 7, lt = threadIdx.x & 127;
  const int g0 = blockIdx.x * 2;
  const int row_vec = W * 3 / 8;  // 16-byte vectors per input row
  if (g0 + h < rows_out) {
    const int g = g0 + h, n = g / Ho, i = g - n * Ho;
    for (int idx = lt; idx < 2 * row_vec; idx += 128) {
      const int dy = idx >= row_vec, v = idx - dy * row_vec;
      const int r = 2 * i + dy - 3;
      tile[(2 * h + dy) * row_vec + v] =
          (r >= 0 && r < H) ? ldnt16(x + (static_cast<int64_t>(n) * H + r) * W * 3 + v * 8)
                            : make_uint4(0, 0, 0, 0);
    }
  }
  __syncthreads();
  const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
  const int row_el = Wo * CO;                               // bf16 per output row
  const int n_el = (g0 + 1 < rows_out ? 2 : 1) * row_el;    // this block's output elements
  uint4* out = reinterpret_cast<uint4*>(xs + static_cast<int64_t>(g0) * row_el);
  for (int k = threadIdx.x; k * 8 < n_el; k += 256) {
    int e = 8 * k;
    int rr = e >= row_el;
    int rem = e - rr * row_el;
    int j = rem / CO, ch = rem - CO * j;
    uint32_t v[8];
#pragma unroll
    for (int e8 = 0; e8 < 8; ++e8) {
      const int dy = ch >= 6, dx = (ch - 6 * dy) >= 3, c = ch - 6 * dy - 3 * dx;
      const int col = 2 * j + dx - 3;
      v[e8] = (ch < 12 && rr < 2 && col >= 0 && col < W) ? t16[(2 * rr + dy) * row_vec * 8 + col * 3 + c] : 0u;
      if (++ch == CO) {  // next output pixel (row_el is a multiple of CO: rows wrap on pixels)
        ch = 0;
        if (++j == Wo) { j = 0; ++rr; }
      }
    }
    if (8 * k + 8 <= n_el) {
      out[k] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
    } else {  // odd row count and odd Wo: the last block's run ends inside a 16-byte chunk
      uint16_t* o16 = reinterpret_cast<uint16_t*>(out + k);
#pragma unroll
      for (int e8 = 0; e8 < 8; ++e8)
        if (e8 < n_el - 8 * k) o16[e8] = static_cast<uint16_t>(v[e8]);
    }
  }
}

// Per-pixel fallback for widths the row kernel does not take: one lane per output pixel.
template <int CO>
__global__ __launch_bounds__(256) void stem_s2d_kernel(const uint16_t* __restrict__ x,
                                                       uint16_t* __restrict__ xs, int64_t n_pix,
                                                       int Wo, int Ho, int W, int H) {
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n_pix;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int j = static_cast<int>(t % Wo);
    const int64_t ni = t / Wo;
    const int i = static_cast<int>(ni % Ho);
    const int64_t n = ni / Ho;
    uint16_t v[CO];
#pragma unroll
    for (int e = 12; e < CO; ++e) v[e] = 0;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const int r = 2 * i + dy - 3;
      const bool row_ok = r >= 0 && r < H;
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int c0 = 2 * j + dx - 3;
        const bool ok = row_ok && c0 >= 0 && c0 < W;
        const uint16_t* src = x + ((n * H + r) * W + c0) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) v[(dy * 2 + dx) * 3 + c] = ok ? __builtin_nontemporal_load(src + c) : 0;
      }
    }
    uint2* dst = reinterpret_cast<uint2*>(xs + t * CO);
#pragma unroll
    for (int q = 0; q < CO / 4; ++q)
      dst[q] = make_uint2(v[4 * q] | (static_cast<uint32_t>(v[4 * q + 1]) << 16),
                          v[4 * q + 2] | (static_cast<uint32_t>(v[4 * q + 3]) << 16));
  }
}

template <int CO>
void stem_s2d_launch(const void* x, void* xs, int N, int H, int W, hipStream_t st) {
  const int Ho = (H + 6) / 2, Wo = (W + 6) / 2;
  const int64_t rows_out = static_cast<int64_t>(N) * Ho;
  if (W % 8 == 0 && W <= kS2dMaxW && rows_out < (int64_t{1} << 31)) {
    hipLaunchKernelGGL(stem_s2d_rows_kernel<CO>, dim3(static_cast<unsigned>((rows_out + 1) / 2)), dim3(256),
                       static_cast<size_t>(24) * W, st, static_cast<const uint16_t*>(x), static_cast<uint16_t*>(xs),
                       static_cast<int>(rows_out), Wo, Ho, W, H);
    return;
  }
  const int64_t n_pix = rows_out * Wo;
  const int64_t blocks = std::min<int64_t>((n_pix + 255) / 256, 256 * 64);
  hipLaunchKernelGGL(stem_s2d_kernel<CO>, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     static_cast<const uint16_t*>(x), static_cast<uint16_t*>(xs), n_pix, Wo, Ho, W, H);
}

void stem_s2d(const void* x, void* xs, int N, int H, int W, hipStream_t st) {
  stem_s2d_launch<12>(x, xs, N, H, W, st);
}

void conv_flip_transpose(const void* w, void* wt, int K, int C, int RS, hipStream_t st) {
  hipLaunchKernelGGL(flip_transpose_kernel, dim3((C + 63) / 64, (K + 63) / 64, RS), dim3(kThreads),
                     0, st, static_cast<const uint16_t*>(w), static_cast<uint16_t*>(wt), K, C, RS);
}

}  // namespace dca
