// Host API of the pointwise-convolution family (conv1x1.hip), shared by the kernels' translation
// unit and the PyTorch bindings (conv_bindings.cpp). Activations are NHWC bf16 viewed as
// [M = N*H*W][C] row-major matrices; weights are bf16 [Cout][Cin]. Channel counts are multiples of
// 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dca {
// Number of row blocks of the forward GEMM = first dimension of its BatchNorm partial-statistics
// output ([blocks][2][Cout] fp32: per-block sum and sum of squares of the bf16 outputs).
int conv1x1_fwd_row_blocks(int64_t M, int Cout);
void conv1x1_fwd(const void* x, const void* w, void* y, float* partial, int64_t M, int Cin,
                 int Cout, hipStream_t st);
// wt: Cin*Cout bf16 scratch for the transposed weight.
void conv1x1_dgrad(const void* dy, const void* w, void* wt, void* dx, int64_t M, int Cin, int Cout,
                   hipStream_t st);
int64_t conv1x1_wgrad_ws_floats(int64_t M, int Cin, int Cout);
void conv1x1_wgrad(const void* dy, const void* x, float* ws, void* dw, bool dw_f32,
                   bool accumulate, int64_t M, int Cin, int Cout, hipStream_t st);

// ---- k x k implicit-GEMM convolutions (conv_igemm.hip). x [N][H][W][C], w [K][R][S][C],
// y [N][P][Q][K], all bf16; C and K multiples of 64; N*H*W*C and N*P*Q*K below 2^31.
struct ConvGeom {
  int N, H, W, C, K, P, Q, R, S, stride, pad, M;  // M = N*P*Q
};
// Row blocks of the forward = first dimension of its [blocks][2][K] BatchNorm partial statistics.
int conv_igemm_row_blocks(const ConvGeom& g);
void conv_igemm_fwd(const void* x, const void* w, void* y, float* partial, const ConvGeom& g,
                    hipStream_t st);
// Weight gradient dW (bf16 or fp32; accumulate adds into it) from dy [M][K] and x, stored
// [K][R][S][C] (channels_last) or, with dw_kcrs, [K][C][R][S]; ws: conv_igemm_wgrad_ws_floats(g)
// fp32 scratch.
int64_t conv_igemm_wgrad_ws_floats(const ConvGeom& g);
void conv_igemm_wgrad(const void* dy, const void* x, float* ws, void* dw, bool dw_f32,
                      bool accumulate, bool dw_kcrs, const ConvGeom& g, hipStream_t st);
// w [K][RS][C] -> wt [C][RS][K] with the taps reversed (stride-1 data-gradient weight).
void conv_flip_transpose(const void* w, void* wt, int K, int C, int RS, hipStream_t st);
// dx [N][H][W][C] += small [N][Ho][Wo][C] at rows s*i, columns s*j (bf16, C a multiple of 8).
void strided_accumulate(void* dx, const void* small, int N, int H, int W, int C, int Ho, int Wo,
                        int s, hipStream_t st);
}  // namespace dca
