// Large-tile MFMA GEMM for transformer projections on gfx950:
//   C[M][N] = A[M][K] . B[N][K]^T
// with both operands K-contiguous -- activations [tokens][features] and nn.Linear weights
// [out][in] -- bf16 in, fp32 accumulate, bf16 out through a fused epilogue (bias, or the GELU
// backward of a transformer MLP with its bias-gradient column sums).
//
// Structure (the 256x256 phased schedule of cdna_hip_programming.md §5, derived for this kernel):
//  * one workgroup = 8 waves (2 along M x 4 along N) = one 256 x 256 output tile, one workgroup per
//    CU; a wave owns 128 x 64 outputs = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (128 accumulator
//    registers);
//  * K in 64-deep tiles through a 2-buffer LDS ring (2 x 64 KB) filled by buffer_load ... lds
//    (LDS-DMA, 16 B per lane, no VGPR round trip). Rows are 128 B with the 16-B chunks XOR-swizzled
//    by (row >> 1) & 7 -- applied to the DMA's SOURCE address, since the DMA writes LDS linearly --
//    so the 16 rows of a ds_read_b128 fragment read land on 16 distinct bank groups;
//  * a K-tile is 4 phases, one 64 x 32 output quadrant (16 MFMAs) each, ordered (0,0) (0,1) (1,1)
//    (1,0) so fragments are reused across phases: A rows are read in phases 1 and 3, B columns in
//    phases 1 and 2, phase 4 reads nothing;
//  * the next K-tile streams in during phases 1 (A) and 2 (B) into the other buffer -- whose last
//    reads retired at least two barriers earlier -- and is waited for (vmcnt(0)) only before phase
//    4's first barrier, 2-3 phases (~1000-1500 cycles) after issue;
//  * every phase is [fragment reads, DMA issue, lgkmcnt(0)] barrier [MFMA cluster at s_setprio 1]
//    barrier, and the wave group holding rows 128-255 runs ONE barrier behind the other: on each SIMD
//    (one wave of each group) one wave issues its MFMA cluster while the other reads fragments,
//    issues DMA or waits (ping-pong). The RAW / WAR orders above hold for both groups at that offset
//    (see the comment on the main loop).
// Reference role: the projections of the GPT-2 / GPT-NeoX DeepSpeedTrial
// (examples/deepspeed/gpt_neox), which the reference runs through cuBLAS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "gemm_api.h"

namespace dca {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 256, kBN = 256, kBK = 64;
constexpr int kThreads = 512;
constexpr int kStage = (kBM + kBN) * kBK;  // bf16 elements of one K-tile (A rows, then B rows)
constexpr int kCS = kBN + 8;               // epilogue C-tile row stride (elements)
constexpr int kLdsBytes = 2 * kStage * 2 > kBM * kCS * 2 ? 2 * kStage * 2 : kBM * kCS * 2;
constexpr uint32_t kOOB = 0x80000000u;     // a buffer offset past every operand: loads zeros

__device__ __forceinline__ int xcd_swizzle(int id, int G) {
  // bijective: block ids that share an XCD (id % 8) get one contiguous range of tiles
  const int q = G >> 3, r = G & 7, xcd = id & 7, k = id >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 16 B per lane into LDS at (wave-uniform) byte address lds + 16 * lane. Inline asm: with the
// builtin hipcc assumes later ds_reads may alias the in-flight DMA and drains vmcnt in front of
// them, which would serialise the next K-tile's loads with this one's MFMAs. The loop waits for
// these loads itself. M0 is saved and restored inside the statement.
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t soff,
                                       uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(rsrc), "s"(soff)
      : "memory");
}

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// value of lane ^ 1 (DPP quad_perm [1, 0, 3, 2]: a VALU move, no LDS round trip)
__device__ __forceinline__ float swap_pair(float x) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));
}

// GELU(tanh) derivative, the formula of transformer.hip's gelu_tanh_grad (so the fused and the
// separate MLP backward agree): d/dx [x s(u)] = s + x s (1 - s) 2 u', s = sigmoid(2u).
__device__ __forceinline__ float gelu_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float x2 = x * x;
  const float u = k0 * fmaf(k1 * x2, x, x);
  const float s = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
  return fmaf(x * s * (1.f - s), 2.f * k0 * fmaf(3.f * k1, x2, 1.f), s);
}

template <int EPI, bool STAGGER>
__global__ __launch_bounds__(kThreads, 1) void gemm_nt_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C, int M,
    int N, int K, int lda, int ldb, int ldc, const float* __restrict__ bias,
    const uint16_t* __restrict__ z, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;  // wave rows wr*128 .., columns wc*64 ..
  const int NT = N / kBN;
  const int t = xcd_swizzle(blockIdx.x, gridDim.x);
  const int mt = t / NT, nt = t - mt * NT;
  const int m0 = mt * kBM, n0 = nt * kBN;
  const int KT = K / kBK;

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(A), 0, static_cast<int>((static_cast<uint32_t>(M - 1) * lda + K) * 2u),
      0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(B), 0, static_cast<int>((static_cast<uint32_t>(N - 1) * ldb + K) * 2u),
      0x00020000);
  // this lane's DMA pieces: wave w moves rows (4w + s) * 8 + lane / 8 of the A and B tiles, 16-B
  // position lane % 8 = source chunk (lane % 8) ^ swz(row)
  uint32_t avo[4], bvo[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int row = (4 * w + s) * 8 + (lane >> 3);
    const uint32_t c8 = static_cast<uint32_t>(((lane & 7) ^ ((row >> 1) & 7)) * 8);
    avo[s] = m0 + row < M ? (static_cast<uint32_t>(m0 + row) * lda + c8) * 2u : kOOB;
    bvo[s] = (static_cast<uint32_t>(n0 + row) * ldb + c8) * 2u;
  }
  const uint32_t lds0 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)(lds)));
  auto stage_a = [&](int buf, int kt) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      glds16(ar, avo[s], static_cast<uint32_t>(kt * kBK * 2),
             lds0 + static_cast<uint32_t>((buf * kStage + (4 * w + s) * 512) * 2));
  };
  auto stage_b = [&](int buf, int kt) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      glds16(br, bvo[s], static_cast<uint32_t>(kt * kBK * 2),
             lds0 + static_cast<uint32_t>((buf * kStage + kBM * kBK + (4 * w + s) * 512) * 2));
  };

  // fragment element offsets inside a 16-row block: row lane & 15, chunk 4 ks + lane / 16 (the row's
  // swizzle depends on lane & 15 only, as blocks start at multiples of 16)
  int fo[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
    fo[ks] = (lane & 15) * kBK + (((4 * ks + (lane >> 4)) ^ ((lane >> 1) & 7)) << 3);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[4][2], b0[2][2], b1[2][2];

  auto load_a = [&](const uint16_t* As, int mh) {
#pragma unroll
    for (int ri = 0; ri < 4; ++ri)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        a[ri][ks] = *reinterpret_cast<const bf16x8*>(As + (wr * 128 + mh * 64 + ri * 16) * kBK + fo[ks]);
  };
  auto load_b = [&](const uint16_t* Bs, int nh, bf16x8 (&b)[2][2]) {
#pragma unroll
    for (int cj = 0; cj < 2; ++cj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        b[cj][ks] = *reinterpret_cast<const bf16x8*>(Bs + (wc * 64 + nh * 32 + cj * 16) * kBK + fo[ks]);
  };
  auto quad = [&](int mh, int nh, const bf16x8 (&b)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri)
#pragma unroll
        for (int cj = 0; cj < 2; ++cj)
          acc[mh * 4 + ri][nh * 2 + cj] = mfma16(a[ri][ks], b[cj][ks], acc[mh * 4 + ri][nh * 2 + cj]);
    __builtin_amdgcn_s_setprio(0);
  };

  // Main loop. Barrier numbering (prologue barrier = 0): group 0 (wr = 0) meets barriers
  // 8kt + 2p - 1 / 8kt + 2p around its phase-p MFMA cluster of K-tile kt, group 1 one later.
  //  RAW: each wave drains its DMA (vmcnt(0)) before its phase-4 first barrier (8kt + 7 / 8kt + 8);
  //   the next tile's first reads follow barrier 8kt + 8 (group 0) / 8kt + 9 (group 1).
  //  WAR: a buffer's last reads (phase 3 of tile kt - 1, retired by lgkmcnt(0) before barrier
  //   8kt - 3 / 8kt - 2) precede its restaging (tile kt + 1, phases 1-2, after barrier 8kt / 8kt + 1).
  stage_a(0, 0);
  stage_b(0, 0);
  wait_vm0();
  barrier();
  if (STAGGER && wr == 1) barrier();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    const uint16_t* As = lds + cur * kStage;
    const uint16_t* Bs = As + kBM * kBK;
    const bool pre = kt + 1 < KT;
    // phase 1: quadrant (0, 0); next tile's A
    load_a(As, 0);
    load_b(Bs, 0, b0);
    if (pre) stage_a(cur ^ 1, kt + 1);
    wait_lgkm0();
    barrier();
    quad(0, 0, b0);
    barrier();
    // phase 2: quadrant (0, 1); next tile's B
    load_b(Bs, 1, b1);
    if (pre) stage_b(cur ^ 1, kt + 1);
    wait_lgkm0();
    barrier();
    quad(0, 1, b1);
    barrier();
    // phase 3: quadrant (1, 1)
    load_a(As, 1);
    wait_lgkm0();
    barrier();
    quad(1, 1, b1);
    barrier();
    // phase 4: quadrant (1, 0) from registers; the next tile has landed (this wave's part)
    wait_vm0();
    barrier();
    quad(1, 0, b0);
    barrier();
  }
  if (STAGGER && wr == 0) barrier();
  __syncthreads();

  // ---- epilogue: accumulators (+ bias) -> bf16 C tile in LDS -> 16-B row-contiguous stores.
  // A lane holds rows R..R+3 of one column; lanes 2c / 2c+1 swap halves so each writes 4-byte column
  // pairs (rows R, R+2 from the even lane, R+1, R+3 from the odd one).
  uint16_t* Cs = lds;
  const bool odd = lane & 1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wc * 64 + j * 16 + (lane & 15);
    const float bj = (EPI == kGemmStore && bias != nullptr) ? bias[n0 + col] : 0.f;
    const int ce = col & ~1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int R = wr * 128 + i * 16 + (lane >> 4) * 4;
      const f32x4 v = acc[i][j];
      const float v0 = v[0] + bj, v1 = v[1] + bj, v2 = v[2] + bj, v3 = v[3] + bj;
      const float r0 = swap_pair(odd ? v0 : v1), r1 = swap_pair(odd ? v2 : v3);
      if (!odd) {
        *reinterpret_cast<uint32_t*>(Cs + R * kCS + ce) = pack_bf16x2(v0, r0);
        *reinterpret_cast<uint32_t*>(Cs + (R + 2) * kCS + ce) = pack_bf16x2(v2, r1);
      } else {
        *reinterpret_cast<uint32_t*>(Cs + (R + 1) * kCS + ce) = pack_bf16x2(r0, v1);
        *reinterpret_cast<uint32_t*>(Cs + (R + 3) * kCS + ce) = pack_bf16x2(r1, v3);
      }
    }
  }
  __syncthreads();
  const int cc = tid & 31, rr = tid >> 5;  // 16-B chunk of a row, first row of this thread
  float s8[8], eb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s8[k] = 0.f;
    eb[k] = (EPI == kGemmDGelu && bias != nullptr) ? bias[n0 + cc * 8 + k] : 0.f;
  }
  for (int row = rr; row < kBM; row += kThreads / 32) {
    if (m0 + row >= M) break;
    const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * kCS + cc * 8);
    const int64_t off = static_cast<int64_t>(m0 + row) * ldc + n0 + cc * 8;
    if constexpr (EPI == kGemmDGelu) {
      const uint4 zv = *reinterpret_cast<const uint4*>(z + off);
      const float dh[8] = {bf16_lo(v.x), bf16_hi(v.x), bf16_lo(v.y), bf16_hi(v.y),
                           bf16_lo(v.z), bf16_hi(v.z), bf16_lo(v.w), bf16_hi(v.w)};
      const float zf[8] = {bf16_lo(zv.x), bf16_hi(zv.x), bf16_lo(zv.y), bf16_hi(zv.y),
                           bf16_lo(zv.z), bf16_hi(zv.z), bf16_lo(zv.w), bf16_hi(zv.w)};
      float dz[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dz[k] = dh[k] * gelu_grad(zf[k] + eb[k]);
        s8[k] += dz[k];
      }
      *reinterpret_cast<uint4*>(C + off) = make_uint4(pack_bf16x2(dz[0], dz[1]), pack_bf16x2(dz[2], dz[3]),
                                                      pack_bf16x2(dz[4], dz[5]), pack_bf16x2(dz[6], dz[7]));
    } else {
      *reinterpret_cast<uint4*>(C + off) = v;
    }
  }
  if constexpr (EPI == kGemmDGelu) {
    // column sums of dZ over this row block: [16 row groups][256 columns] through LDS
    __syncthreads();
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int k = 0; k < 8; ++k) red[rr * kBN + cc * 8 + k] = s8[k];
    __syncthreads();
    if (tid < kBN) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < kThreads / 32; ++g) s += red[g * kBN + tid];
      partial[static_cast<int64_t>(mt) * N + n0 + tid] = s;
    }
  }
}

template <int EPI>
void launch(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
            const float* bias, const void* z, float* partial, hipStream_t st) {
  auto kern = gemm_nt_kernel<EPI, true>;
  static const bool attr = [&] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    return true;
  }();
  (void)attr;
  const int grid = gemm_nt_row_blocks(M) * (N / kBN);
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), kLdsBytes, st, static_cast<const uint16_t*>(A),
                     static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M, N, K, lda, ldb, ldc,
                     bias, static_cast<const uint16_t*>(z), partial);
}

}  // namespace

int gemm_nt_row_blocks(int M) { return (M + kBM - 1) / kBM; }

void gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
             int epi, const float* bias, const void* z, float* partial, hipStream_t st) {
  if (epi == kGemmDGelu) launch<kGemmDGelu>(A, B, C, M, N, K, lda, ldb, ldc, bias, z, partial, st);
  else launch<kGemmStore>(A, B, C, M, N, K, lda, ldb, ldc, bias, z, partial, st);
}

}  // namespace dca
