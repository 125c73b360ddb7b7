// Shared device helpers for the determined_clone_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this directory:
//  * wave64: lane = threadIdx.x & 63, block sizes are multiples of 64;
//  * memory-bound kernels move 16 bytes per lane per access (8 x bf16 / 4 x fp32), never scalar
//    bf16 (cdna_hip_programming.md Guideline 13);
//  * reductions are deterministic: per-block partials -> a second, channel-parallel pass
//    (no float atomics, so results are bitwise reproducible run to run).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dca {

constexpr int kWave = 64;

// ---------------------------------------------------------------- bf16 / fp16 bit helpers
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// fp32 -> bf16 round-to-nearest-even (NaN stays NaN) with gfx950's v_cvt_pk_bf16_f32: one VALU
// instruction per PAIR instead of the ~6-instruction integer rounding sequence per value (that
// sequence was a third of the attention kernels' VALU stream).
typedef __bf16 dca_bf16x2 __attribute__((ext_vector_type(2)));
typedef float dca_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const dca_f32x2 f = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, dca_bf16x2));
}
__device__ __forceinline__ uint32_t f2bf_bits(float f) { return pack_bf16x2(f, 0.f) & 0xffffu; }

__device__ __forceinline__ float h2f(uint32_t bits) {
  const uint16_t h = static_cast<uint16_t>(bits);
  _Float16 f;
  __builtin_memcpy(&f, &h, 2);
  return static_cast<float>(f);
}
__device__ __forceinline__ uint16_t f2h(float f) {
  const _Float16 h = static_cast<_Float16>(f);
  uint16_t u;
  __builtin_memcpy(&u, &h, 2);
  return u;
}

// ---------------------------------------------------------------- 8-element vector I/O
// Type tags: element storage for the templated kernels.
struct BF16 { using raw = uint16_t; };
struct F16 { using raw = uint16_t; };
struct F32 { using raw = float; };

template <typename T> struct Vec8;

template <> struct Vec8<BF16> {
  __device__ __forceinline__ static void load(const void* p, float (&v)[8]) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    v[0] = bf16_lo(q.x); v[1] = bf16_hi(q.x); v[2] = bf16_lo(q.y); v[3] = bf16_hi(q.y);
    v[4] = bf16_lo(q.z); v[5] = bf16_hi(q.z); v[6] = bf16_lo(q.w); v[7] = bf16_hi(q.w);
  }
  __device__ __forceinline__ static void store(void* p, const float (&v)[8]) {
    uint4 q;
    q.x = pack_bf16x2(v[0], v[1]); q.y = pack_bf16x2(v[2], v[3]);
    q.z = pack_bf16x2(v[4], v[5]); q.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = q;
  }
  static constexpr int bytes = 2;
};

template <> struct Vec8<F16> {
  __device__ __forceinline__ static void load(const void* p, float (&v)[8]) {
    uint4 q = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = h2f(static_cast<uint16_t>(w[i] & 0xffffu));
      v[2 * i + 1] = h2f(static_cast<uint16_t>(w[i] >> 16));
    }
  }
  __device__ __forceinline__ static void store(void* p, const float (&v)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = static_cast<uint32_t>(f2h(v[2 * i])) | (static_cast<uint32_t>(f2h(v[2 * i + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  static constexpr int bytes = 2;
};

template <> struct Vec8<F32> {
  __device__ __forceinline__ static void load(const void* p, float (&v)[8]) {
    const float4* q = reinterpret_cast<const float4*>(p);
    float4 a = q[0], b = q[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ static void store(void* p, const float (&v)[8]) {
    float4* q = reinterpret_cast<float4*>(p);
    q[0] = make_float4(v[0], v[1], v[2], v[3]);
    q[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  static constexpr int bytes = 4;
};

// Scalar element access (for gather-style kernels; bulk paths use Vec8).
template <typename T> struct Elem;
template <> struct Elem<BF16> {
  __device__ __forceinline__ static float get(const void* p, int64_t i) {
    return __uint_as_float(static_cast<uint32_t>(reinterpret_cast<const uint16_t*>(p)[i]) << 16);
  }
  __device__ __forceinline__ static void put(void* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = static_cast<uint16_t>(f2bf_bits(v));
  }
};
template <> struct Elem<F16> {
  __device__ __forceinline__ static float get(const void* p, int64_t i) {
    return h2f(reinterpret_cast<const uint16_t*>(p)[i]);
  }
  __device__ __forceinline__ static void put(void* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = f2h(v);
  }
};
template <> struct Elem<F32> {
  __device__ __forceinline__ static float get(const void* p, int64_t i) {
    return reinterpret_cast<const float*>(p)[i];
  }
  __device__ __forceinline__ static void put(void* p, int64_t i, float v) {
    reinterpret_cast<float*>(p)[i] = v;
  }
};

// ---------------------------------------------------------------- reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
// Wave-wide sum on the VALU, no LDS round trips: DPP quad / half-row / row mirrors give every lane
// its 16-lane row sum, then the gfx950 permlane16 / permlane32 half swaps add the other rows
// (r[0] + r[1] of a swap of v with itself = v + the partner lane's v).
template <int kCtrl>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), kCtrl, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]: + lane ^ 1
  v += dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]: + lane ^ 2
  v += dpp_f32<0x141>(v);  // row_half_mirror: + the other quad of the 8-lane half row
  v += dpp_f32<0x140>(v);  // row_mirror: + the other half row
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `scratch` needs blockDim.x/64 floats. Result valid in
// every thread.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// Memory-bound grid size: enough workgroups to fill 256 CUs several times, grid-stride the rest.
inline int stream_grid(int64_t work_items, int block) {
  int64_t g = (work_items + block - 1) / block;
  if (g > 256 * 8) g = 256 * 8;
  if (g < 1) g = 1;
  return static_cast<int>(g);
}

// Raw 8-element vectors: loads are issued into these (no conversion in between), so the U loads
// of an unrolled iteration are all in flight before the first use; unpacked afterwards.
template <typename T> struct Raw8;
template <> struct Raw8<BF16> { uint4 q; };
template <> struct Raw8<F16> { uint4 q; };
template <> struct Raw8<F32> { float4 a, b; };

template <typename T>
__device__ __forceinline__ Raw8<T> ld8(const void* base, int64_t elem_off) {
  Raw8<T> r;
  if constexpr (std::is_same<T, F32>::value) {
    const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + elem_off);
    r.a = p[0];
    r.b = p[1];
  } else {
    r.q = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(base) + elem_off);
  }
  return r;
}
// Nontemporal variant (streamed once: one-shot reads measured 6.9 TB/s with nt against 6.0
// without, profiles/round4_hbm_streaming_ceilings.txt).
typedef unsigned int dca_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt16(const void* p) {
  const dca_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const dca_u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <typename T>
__device__ __forceinline__ Raw8<T> ld8nt(const void* base, int64_t elem_off) {
  Raw8<T> r;
  if constexpr (std::is_same<T, F32>::value) {
    const float* p = reinterpret_cast<const float*>(base) + elem_off;
    const uint4 a = ldnt16(p), b = ldnt16(p + 4);
    r.a = make_float4(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z), __uint_as_float(a.w));
    r.b = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), __uint_as_float(b.w));
  } else {
    r.q = ldnt16(reinterpret_cast<const uint16_t*>(base) + elem_off);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void unpack8(const Raw8<T>& r, float (&v)[8]) {
  if constexpr (std::is_same<T, F32>::value) {
    v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w;
    v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  } else if constexpr (std::is_same<T, BF16>::value) {
    v[0] = bf16_lo(r.q.x); v[1] = bf16_hi(r.q.x); v[2] = bf16_lo(r.q.y); v[3] = bf16_hi(r.q.y);
    v[4] = bf16_lo(r.q.z); v[5] = bf16_hi(r.q.z); v[6] = bf16_lo(r.q.w); v[7] = bf16_hi(r.q.w);
  } else {
    const uint32_t w[4] = {r.q.x, r.q.y, r.q.z, r.q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = h2f(w[i] & 0xffffu);
      v[2 * i + 1] = h2f(w[i] >> 16);
    }
  }
}

}  // namespace dca
