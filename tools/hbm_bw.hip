// HBM streaming ceilings on MI355X for the memory-bound kernels (BatchNorm, optimizers): read-only,
// write-only, copy (1R1W) and the BN-backward shape (2R1W) with several issue strategies, so the
// "roofline" the fused BN kernels are measured against is the best streaming kernel we can write,
// not torch's copy_ (profiles/round2_hbm_copy_roofline.txt: 5.1 TB/s).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_bw tools/hbm_bw.hip
// Run:   tools/bin/hbm_bw [MiB per buffer, default 1024]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// One-shot grid: each thread moves U 16-B vectors, U loads issued before any store.
// Block b covers [b*256*U, (b+1)*256*U) vectors, lane-contiguous within each of the U slices.
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_oneshot(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n) {
  const long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    v[u] = i < n ? ld<NTL>(in + i) : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    if (i < n) st<NTS>(out + i, v[u]);
  }
}

// Persistent grid-stride: grid = CUs x k blocks, U vectors per thread per iteration.
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_stride(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n) {
  const long stride = static_cast<long>(gridDim.x) * 256 * U;
  for (long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x; base < n; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * 256;
      v[u] = i < n ? ld<NTL>(in + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = base + u * 256;
      if (i < n) st<NTS>(out + i, v[u]);
    }
  }
}

// Read-only: xor-reduce, one store per block.
template <int U, bool NTL>
__global__ __launch_bounds__(256) void read_oneshot(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n) {
  const long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    if (i < n) acc ^= ld<NTL>(in + i);
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[blockIdx.x] = acc;  // keeps loads live
}

template <int U, bool NTS>
__global__ __launch_bounds__(256) void fill_oneshot(u32x4* __restrict__ out, long n) {
  const long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    if (i < n) st<NTS>(out + i, u32x4{1u, 2u, 3u, static_cast<unsigned>(i)});
  }
}

// BN-backward shape: out = a + b (2 reads, 1 write)
template <int U, bool NTS>
__global__ __launch_bounds__(256) void add2_oneshot(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                    u32x4* __restrict__ out, long n) {
  const long base = static_cast<long>(blockIdx.x) * 256 * U + threadIdx.x;
  u32x4 va[U], vb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    va[u] = i < n ? a[i] : u32x4{0, 0, 0, 0};
    vb[u] = i < n ? b[i] : u32x4{0, 0, 0, 0};
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    if (i < n) st<NTS>(out + i, va[u] + vb[u]);
  }
}

template <typename F>
static float time_ms(F f, int reps = 15) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const long mib = argc > 1 ? std::atol(argv[1]) : 1024;
  const long bytes = mib << 20;
  const long n = bytes / 16;
  u32x4 *a, *b, *c;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  CK(hipMemset(c, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto rep = [&](const char* name, float ms, double moved) {
    std::printf("{\"kernel\": \"%s\", \"MiB\": %ld, \"ms\": %.4f, \"TBps\": %.3f}\n", name, mib, ms,
                moved / (ms * 1e-3) / 1e12);
    std::fflush(stdout);
  };
#define ONESHOT_COPY(U, NTL, NTS)                                                                 \
  rep("copy_oneshot U=" #U " ntl=" #NTL " nts=" #NTS,                                            \
      time_ms([&] {                                                                               \
        const long g = (n + 256L * U - 1) / (256L * U);                                           \
        hipLaunchKernelGGL((copy_oneshot<U, NTL, NTS>), dim3(g), dim3(256), 0, 0, a, c, n);       \
      }),                                                                                         \
      2.0 * bytes)
  ONESHOT_COPY(1, false, false);
  ONESHOT_COPY(2, false, false);
  ONESHOT_COPY(4, false, false);
  ONESHOT_COPY(8, false, false);
  ONESHOT_COPY(4, true, false);
  ONESHOT_COPY(4, false, true);
  ONESHOT_COPY(4, true, true);
  ONESHOT_COPY(8, true, true);
#define STRIDE_COPY(U, K, NTL, NTS)                                                               \
  rep("copy_stride U=" #U " blocks/CU=" #K " ntl=" #NTL " nts=" #NTS,                             \
      time_ms([&] {                                                                               \
        hipLaunchKernelGGL((copy_stride<U, NTL, NTS>), dim3(cus * K), dim3(256), 0, 0, a, c, n);  \
      }),                                                                                         \
      2.0 * bytes)
  STRIDE_COPY(4, 4, false, false);
  STRIDE_COPY(4, 8, false, false);
  STRIDE_COPY(8, 4, false, false);
  STRIDE_COPY(4, 8, true, true);
  STRIDE_COPY(2, 16, false, false);
#define READ(U, NTL)                                                                              \
  rep("read_oneshot U=" #U " ntl=" #NTL,                                                         \
      time_ms([&] {                                                                               \
        const long g = (n + 256L * U - 1) / (256L * U);                                           \
        hipLaunchKernelGGL((read_oneshot<U, NTL>), dim3(g), dim3(256), 0, 0, a, c, n);            \
      }),                                                                                         \
      1.0 * bytes)
  READ(1, false);
  READ(4, false);
  READ(8, false);
  READ(8, true);
  READ(16, false);
#define FILL(U, NTS)                                                                              \
  rep("fill_oneshot U=" #U " nts=" #NTS,                                                         \
      time_ms([&] {                                                                               \
        const long g = (n + 256L * U - 1) / (256L * U);                                           \
        hipLaunchKernelGGL((fill_oneshot<U, NTS>), dim3(g), dim3(256), 0, 0, c, n);               \
      }),                                                                                         \
      1.0 * bytes)
  FILL(1, false);
  FILL(4, false);
  FILL(4, true);
#define ADD2(U, NTS)                                                                              \
  rep("add2_oneshot U=" #U " nts=" #NTS,                                                         \
      time_ms([&] {                                                                               \
        const long g = (n + 256L * U - 1) / (256L * U);                                           \
        hipLaunchKernelGGL((add2_oneshot<U, NTS>), dim3(g), dim3(256), 0, 0, a, b, c, n);         \
      }),                                                                                         \
      3.0 * bytes)
  ADD2(1, false);
  ADD2(2, false);
  ADD2(4, false);
  ADD2(4, true);
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  return 0;
}
