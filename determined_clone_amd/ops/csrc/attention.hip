// Flash attention (forward + backward) on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16), bf16 in/out,
// fp32 softmax statistics, causal or full, head dim 64 / 128.
//
// Replaces the fused softmax/attention CUDA kernels the reference's GPT-NeoX DeepSpeedTrial gets
// from DeepSpeed/apex (examples/deepspeed/gpt_neox). Inputs are strided [B, S, H, D] or
// [B, H, S, D] views (last dim contiguous), so the model can pass slices of its fused QKV
// projection without copies.
//
// Forward, one workgroup = 4 wave64 = 64 query rows of one (batch, head):
//   Q fragments live in VGPRs for the whole kernel; per 64-key tile K is staged row-major and V
//   transposed into LDS (padded rows, 16-B ds_read_b128 fragment reads), S = Q K^T (16x16x32
//   MFMA), online softmax in the exp2 domain with 16-lane shuffle row reductions, P goes through a
//   per-wave LDS tile to become the A operand of O += P V. Writes O and the row log-sum-exp.
// Backward (FlashAttention-2 ordering), one workgroup = 64 keys; dK/dV accumulate in VGPRs while
//   the workgroup sweeps the query tiles; recomputed P^T = exp2(S^T - LSE), dP^T = V dO^T,
//   dS^T = P^T (dP^T - rowsum(dO*O)); dQ partials are added into an fp32 buffer with float atomics.
#include "common.h"

namespace dca {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 64;   // query rows per forward block / keys per backward block
constexpr int kPad = 8;     // LDS row padding (elements) to break power-of-two bank strides

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 load8(const uint16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

__device__ __forceinline__ bf16x8 zero8() {
  uint4 z = make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, z);
}

__device__ __forceinline__ uint16_t to_bf16(float f) { return static_cast<uint16_t>(f2bf_bits(f)); }
__device__ __forceinline__ float from_bf16(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

struct Strides {
  int64_t b, h, s;  // element strides; d stride is 1
};

// Stage a [64 rows][D] tile (rows r0.., clamped to n_rows, zero-filled beyond) into LDS,
// row-major (dst[r][d], row stride D + kPad) and/or transposed (dstT[d][r], row stride 64 + kPad).
template <int D>
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ src, Strides st, int r0,
                                           int n_rows, uint16_t* dst, uint16_t* dstT) {
  constexpr int chunks_per_row = D / 8;
  constexpr int total = kTile * chunks_per_row;
  for (int c = threadIdx.x; c < total; c += blockDim.x) {
    const int r = c / chunks_per_row;
    const int d0 = (c % chunks_per_row) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < n_rows) v = *reinterpret_cast<const uint4*>(src + static_cast<int64_t>(r0 + r) * st.s + d0);
    if (dst) *reinterpret_cast<uint4*>(dst + r * (D + kPad) + d0) = v;
    if (dstT) {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int i = 0; i < 8; ++i) dstT[(d0 + i) * (kTile + kPad) + r] = e[i];
    }
  }
}

// ------------------------------------------------------------------------------------ forward
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void attn_fwd_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    uint16_t* __restrict__ o, float* __restrict__ lse, int Sq, int Sk, int H, Strides qs,
    Strides ks, Strides vs, Strides os, float scale_log2) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;                                 // [64][D + pad]
  uint16_t* Vt = Ks + kTile * (D + kPad);              // [D][64 + pad]
  uint16_t* Ps = Vt + D * (kTile + kPad);              // [4][16][64 + pad]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int q_blk = blockIdx.x * kTile;
  const int q0 = q_blk + w * 16;
  const uint16_t* qb = q + b * qs.b + h * qs.h;
  const uint16_t* kb = k + b * ks.b + h * ks.h;
  const uint16_t* vb = v + b * vs.b + h * vs.h;
  uint16_t* ob = o + b * os.b + h * os.h;
  uint16_t* Pw = Ps + w * 16 * (kTile + kPad);

  bf16x8 qa[D / 32];
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const int row = q0 + lr;
    qa[s] = row < Sq ? load8(qb + static_cast<int64_t>(row) * qs.s + 32 * s + 8 * lg) : zero8();
  }
  f32x4 oacc[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) oacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = -INFINITY; l[i] = 0.f; }

  const int k_end = CAUSAL ? min(Sk, q_blk + kTile) : Sk;
  for (int kt = 0; kt < k_end; kt += kTile) {
    __syncthreads();
    stage_tile<D>(kb, ks, kt, Sk, Ks, nullptr);
    stage_tile<D>(vb, vs, kt, Sk, nullptr, Vt);
    __syncthreads();
    f32x4 sacc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s)
        acc = mfma(qa[s], load8(Ks + (16 * n + lr) * (D + kPad) + 32 * s + 8 * lg), acc);
      sacc[n] = acc;
    }
    float mx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = q0 + lg * 4 + i;
      float t = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int key = kt + 16 * n + lr;
        float sv = sacc[n][i] * scale_log2;
        if (key >= Sk || (CAUSAL && key > row)) sv = -INFINITY;
        sacc[n][i] = sv;
        t = fmaxf(t, sv);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) t = fmaxf(t, __shfl_xor(t, off, 64));
      mx[i] = t;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mnew = fmaxf(m[i], mx[i]);
      const float mref = mnew == -INFINITY ? 0.f : mnew;
      const float alpha = exp2f(m[i] - mref);
      float rs = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(sacc[n][i] - mref);
        sacc[n][i] = p;
        rs += p;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l[i] = l[i] * alpha + rs;
      m[i] = mnew;
#pragma unroll
      for (int n = 0; n < D / 16; ++n) oacc[n][i] *= alpha;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) Pw[(lg * 4 + i) * (kTile + kPad) + 16 * n + lr] = to_bf16(sacc[n][i]);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pa = load8(Pw + lr * (kTile + kPad) + 32 * s + 8 * lg);
#pragma unroll
      for (int n = 0; n < D / 16; ++n)
        oacc[n] = mfma(pa, load8(Vt + (16 * n + lr) * (kTile + kPad) + 32 * s + 8 * lg), oacc[n]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = q0 + lg * 4 + i;
    if (row >= Sq) continue;
    const float inv = l[i] > 0.f ? 1.f / l[i] : 0.f;
#pragma unroll
    for (int n = 0; n < D / 16; ++n)
      ob[static_cast<int64_t>(row) * os.s + 16 * n + lr] = to_bf16(oacc[n][i] * inv);
    if (lr == 0)
      lse[(static_cast<int64_t>(b) * H + h) * Sq + row] = l[i] > 0.f ? m[i] + log2f(l[i]) : INFINITY;
  }
}

// delta[b,h,q] = sum_d dO * O  (one wave per row)
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(const uint16_t* __restrict__ o,
                                                         const uint16_t* __restrict__ dO,
                                                         float* __restrict__ delta, int B, int H,
                                                         int Sq, Strides os, Strides ds) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= static_cast<int64_t>(B) * H * Sq) return;
  const int s = static_cast<int>(row % Sq);
  const int h = static_cast<int>((row / Sq) % H);
  const int b = static_cast<int>(row / (static_cast<int64_t>(Sq) * H));
  const uint16_t* op = o + b * os.b + h * os.h + static_cast<int64_t>(s) * os.s;
  const uint16_t* dp = dO + b * ds.b + h * ds.h + static_cast<int64_t>(s) * ds.s;
  float acc = 0.f;
  for (int d = lane; d < D; d += 64) acc = fmaf(from_bf16(op[d]), from_bf16(dp[d]), acc);
  acc = wave_sum(acc);
  if (lane == 0) delta[row] = acc;
}

// ------------------------------------------------------------------------------------ backward
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256) void attn_bwd_kernel(
    const uint16_t* __restrict__ q, const uint16_t* __restrict__ k, const uint16_t* __restrict__ v,
    const uint16_t* __restrict__ dO, const float* __restrict__ lse, const float* __restrict__ delta,
    float* __restrict__ dq_acc, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, int Sq,
    int Sk, int H, Strides qs, Strides ks, Strides vs, Strides dos, Strides dks, Strides dvs,
    float scale_log2, float scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  constexpr int RS = D + kPad;      // row-major tile stride
  constexpr int TS = kTile + kPad;  // transposed tile stride
  uint16_t* Qs = smem;              // [64 q][D]
  uint16_t* Qt = Qs + kTile * RS;   // [D][64 q]
  uint16_t* dOs = Qt + D * TS;      // [64 q][D]
  uint16_t* dOt = dOs + kTile * RS; // [D][64 q]
  uint16_t* Kt = dOt + D * TS;      // [D][64 keys]
  uint16_t* Pw_all = Kt + D * TS;   // [4][16 keys][64 q]   P^T
  uint16_t* Sw_all = Pw_all + 4 * 16 * TS;  // [4][16 keys][64 q]  dS^T
  uint16_t* dSq = Sw_all + 4 * 16 * TS;     // [64 q][64 keys]    dS
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int kb0 = blockIdx.x * kTile;
  const int key0 = kb0 + w * 16;
  const uint16_t* qb = q + b * qs.b + h * qs.h;
  const uint16_t* kb = k + b * ks.b + h * ks.h;
  const uint16_t* vb = v + b * vs.b + h * vs.h;
  const uint16_t* dob = dO + b * dos.b + h * dos.h;
  const float* lseb = lse + (static_cast<int64_t>(b) * H + h) * Sq;
  const float* delb = delta + (static_cast<int64_t>(b) * H + h) * Sq;
  float* dqb = dq_acc + (static_cast<int64_t>(b) * H + h) * Sq * D;
  uint16_t* Pw = Pw_all + w * 16 * TS;
  uint16_t* Sw = Sw_all + w * 16 * TS;

  bf16x8 ka[D / 32], va[D / 32];
#pragma unroll
  for (int s = 0; s < D / 32; ++s) {
    const int key = key0 + lr;
    ka[s] = key < Sk ? load8(kb + static_cast<int64_t>(key) * ks.s + 32 * s + 8 * lg) : zero8();
    va[s] = key < Sk ? load8(vb + static_cast<int64_t>(key) * vs.s + 32 * s + 8 * lg) : zero8();
  }
  stage_tile<D>(kb, ks, kb0, Sk, nullptr, Kt);
  f32x4 dkacc[D / 16], dvacc[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) {
    dkacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    dvacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int q_start = CAUSAL ? (kb0 / kTile) * kTile : 0;
  for (int qt = q_start; qt < Sq; qt += kTile) {
    __syncthreads();
    stage_tile<D>(qb, qs, qt, Sq, Qs, Qt);
    stage_tile<D>(dob, dos, qt, Sq, dOs, dOt);
    __syncthreads();
    f32x4 pt[4], dpt[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f}, c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < D / 32; ++s) {
        a = mfma(ka[s], load8(Qs + (16 * n + lr) * RS + 32 * s + 8 * lg), a);
        c = mfma(va[s], load8(dOs + (16 * n + lr) * RS + 32 * s + 8 * lg), c);
      }
      pt[n] = a;
      dpt[n] = c;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int qi = qt + 16 * n + lr;
      const float lq = qi < Sq ? lseb[qi] : INFINITY;
      const float dl = qi < Sq ? delb[qi] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = key0 + lg * 4 + i;
        float p = exp2f(pt[n][i] * scale_log2 - lq);
        if (qi >= Sq || key >= Sk || (CAUSAL && key > qi)) p = 0.f;
        const float ds = p * (dpt[n][i] - dl) * scale;
        Pw[(lg * 4 + i) * TS + 16 * n + lr] = to_bf16(p);
        const uint16_t dsb = to_bf16(ds);
        Sw[(lg * 4 + i) * TS + 16 * n + lr] = dsb;
        dSq[(16 * n + lr) * TS + w * 16 + lg * 4 + i] = dsb;
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 pa = load8(Pw + lr * TS + 32 * s + 8 * lg);
      const bf16x8 sa = load8(Sw + lr * TS + 32 * s + 8 * lg);
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        dvacc[n] = mfma(pa, load8(dOt + (16 * n + lr) * TS + 32 * s + 8 * lg), dvacc[n]);
        dkacc[n] = mfma(sa, load8(Qt + (16 * n + lr) * TS + 32 * s + 8 * lg), dkacc[n]);
      }
    }
    // dQ rows 16w.. of this query tile: dS[q][keys 0..63] . K[keys][D]
    f32x4 dqacc[D / 16];
#pragma unroll
    for (int n = 0; n < D / 16; ++n) dqacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 a = load8(dSq + (16 * w + lr) * TS + 32 * s + 8 * lg);
#pragma unroll
      for (int n = 0; n < D / 16; ++n)
        dqacc[n] = mfma(a, load8(Kt + (16 * n + lr) * TS + 32 * s + 8 * lg), dqacc[n]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qi = qt + 16 * w + lg * 4 + i;
      if (qi >= Sq) continue;
#pragma unroll
      for (int n = 0; n < D / 16; ++n)
        atomicAdd(dqb + static_cast<int64_t>(qi) * D + 16 * n + lr, dqacc[n][i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int key = key0 + lg * 4 + i;
    if (key >= Sk) continue;
#pragma unroll
    for (int n = 0; n < D / 16; ++n) {
      dk[b * dks.b + h * dks.h + static_cast<int64_t>(key) * dks.s + 16 * n + lr] = to_bf16(dkacc[n][i]);
      dv[b * dvs.b + h * dvs.h + static_cast<int64_t>(key) * dvs.s + 16 * n + lr] = to_bf16(dvacc[n][i]);
    }
  }
}

// dq (strided bf16) <- dq_acc (contiguous fp32 [B, H, S, D])
__global__ __launch_bounds__(256) void attn_dq_convert_kernel(const float* __restrict__ acc,
                                                              uint16_t* __restrict__ dq, int B,
                                                              int H, int Sq, int D, Strides st) {
  const int64_t total = static_cast<int64_t>(B) * H * Sq * D;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int d = static_cast<int>(i % D);
    const int s = static_cast<int>((i / D) % Sq);
    const int h = static_cast<int>((i / (static_cast<int64_t>(D) * Sq)) % H);
    const int b = static_cast<int>(i / (static_cast<int64_t>(D) * Sq * H));
    dq[b * st.b + h * st.h + static_cast<int64_t>(s) * st.s + d] = to_bf16(acc[i]);
  }
}

size_t fwd_lds(int D) { return (static_cast<size_t>(kTile) * (D + kPad) + D * (kTile + kPad) + 4 * 16 * (kTile + kPad)) * 2; }
size_t bwd_lds(int D) {
  return (2 * static_cast<size_t>(kTile) * (D + kPad) + 3 * static_cast<size_t>(D) * (kTile + kPad) +
          2 * 4 * 16 * (kTile + kPad) + kTile * (kTile + kPad)) * 2;
}

template <int D, bool C>
void launch_fwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, uint16_t* o, float* lse,
                int B, int H, int Sq, int Sk, Strides qs, Strides ks, Strides vs, Strides os,
                float scale_log2, hipStream_t st) {
  dim3 grid((Sq + kTile - 1) / kTile, H, B);
  const size_t lds = fwd_lds(D);
  hipFuncSetAttribute(reinterpret_cast<const void*>(attn_fwd_kernel<D, C>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  hipLaunchKernelGGL((attn_fwd_kernel<D, C>), grid, dim3(256), lds, st, q, k, v, o, lse, Sq, Sk, H,
                     qs, ks, vs, os, scale_log2);
}

template <int D, bool C>
void launch_bwd(const uint16_t* q, const uint16_t* k, const uint16_t* v, const uint16_t* o,
                const uint16_t* dO, const float* lse, float* delta, float* dq_acc, uint16_t* dq,
                uint16_t* dk, uint16_t* dv, int B, int H, int Sq, int Sk, Strides qs, Strides ks,
                Strides vs, Strides os, Strides dos, Strides dqs, Strides dks, Strides dvs,
                float scale_log2, float scale, hipStream_t st) {
  const int64_t rows = static_cast<int64_t>(B) * H * Sq;
  hipLaunchKernelGGL(attn_delta_kernel<D>, dim3((rows + 3) / 4), dim3(256), 0, st, o, dO, delta, B,
                     H, Sq, os, dos);
  hipMemsetAsync(dq_acc, 0, rows * D * sizeof(float), st);
  dim3 grid((Sk + kTile - 1) / kTile, H, B);
  const size_t lds = bwd_lds(D);
  hipFuncSetAttribute(reinterpret_cast<const void*>(attn_bwd_kernel<D, C>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  hipLaunchKernelGGL((attn_bwd_kernel<D, C>), grid, dim3(256), lds, st, q, k, v, dO, lse, delta,
                     dq_acc, dk, dv, Sq, Sk, H, qs, ks, vs, dos, dks, dvs, scale_log2, scale);
  hipLaunchKernelGGL(attn_dq_convert_kernel, dim3(stream_grid(rows * D, 256)), dim3(256), 0, st,
                     dq_acc, dq, B, H, Sq, D, dqs);
}

}  // namespace

void attention_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H,
                   int Sq, int Sk, int D, const int64_t* qs, const int64_t* ks, const int64_t* vs,
                   const int64_t* os, float scale, bool causal, hipStream_t st) {
  const float sl2 = scale * 1.4426950408889634f;
  Strides a{qs[0], qs[1], qs[2]}, bb{ks[0], ks[1], ks[2]}, c{vs[0], vs[1], vs[2]}, d{os[0], os[1], os[2]};
  auto Q = static_cast<const uint16_t*>(q);
  auto K = static_cast<const uint16_t*>(k);
  auto V = static_cast<const uint16_t*>(v);
  auto O = static_cast<uint16_t*>(o);
  if (D == 64) {
    if (causal) launch_fwd<64, true>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, st);
    else launch_fwd<64, false>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, st);
  } else {
    if (causal) launch_fwd<128, true>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, st);
    else launch_fwd<128, false>(Q, K, V, O, lse, B, H, Sq, Sk, a, bb, c, d, sl2, st);
  }
}

void attention_bwd(const void* q, const void* k, const void* v, const void* o, const void* dO,
                   const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                   int B, int H, int Sq, int Sk, int D, const int64_t* st_q, const int64_t* st_k,
                   const int64_t* st_v, const int64_t* st_o, const int64_t* st_do,
                   const int64_t* st_dq, const int64_t* st_dk, const int64_t* st_dv, float scale,
                   bool causal, hipStream_t stream) {
  const float sl2 = scale * 1.4426950408889634f;
  auto S = [](const int64_t* p) { return Strides{p[0], p[1], p[2]}; };
  auto c16 = [](const void* p) { return static_cast<const uint16_t*>(p); };
  auto m16 = [](void* p) { return static_cast<uint16_t*>(p); };
  if (D == 64) {
    if (causal) launch_bwd<64, true>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, dq_acc, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, stream);
    else launch_bwd<64, false>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, dq_acc, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, stream);
  } else {
    if (causal) launch_bwd<128, true>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, dq_acc, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, stream);
    else launch_bwd<128, false>(c16(q), c16(k), c16(v), c16(o), c16(dO), lse, delta, dq_acc, m16(dq), m16(dk), m16(dv), B, H, Sq, Sk, S(st_q), S(st_k), S(st_v), S(st_o), S(st_do), S(st_dq), S(st_dk), S(st_dv), sl2, scale, stream);
  }
}

}  // namespace dca
