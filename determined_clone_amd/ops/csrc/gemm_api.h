// Host API of the large-tile MFMA GEMM (gemm.hip), shared by the kernel's translation unit and the
// PyTorch bindings (gemm_bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dca {
// Epilogues of gemm_nt.
enum GemmEpi : int {
  kGemmStore = 0,  // C = A B^T (+ bias[n] when bias != nullptr)
  kGemmDGelu = 1,  // C = (A B^T) * gelu_tanh'(z + bias), partial[row block][n] = column sums of C
};
// 256-row blocks of a gemm_nt launch = first dimension of its kGemmDGelu partial sums.
int gemm_nt_row_blocks(int M);
// C[M][N] (bf16, row stride ldc) = A[M][K] . B[N][K]^T, A / B bf16 with unit stride along K and row
// strides lda / ldb. N % 256 == 0, K % 64 == 0; the byte offsets of A and B must fit 31 bits.
// bias: fp32 [N] or nullptr; z: bf16 [M][ldc] (kGemmDGelu); partial: fp32 [row blocks][N].
void gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
             int epi, const float* bias, const void* z, float* partial, hipStream_t st);
}  // namespace dca
