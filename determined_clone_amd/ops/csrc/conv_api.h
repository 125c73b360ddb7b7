// Host API of the implicit-GEMM convolution family (conv_igemm.hip), shared by the kernels'
// translation unit and the PyTorch bindings (conv_bindings.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dca {
// ---- k x k implicit-GEMM convolutions (conv_igemm.hip). x [N][H][W][C], w [K][R][S][C],
// y [N][P][Q][K], all bf16; C and K multiples of 64; N*H*W*C and N*P*Q*K below 2^31.
struct ConvGeom {
  int N, H, W, C, K, P, Q, R, S, stride, pad, M;  // M = N*P*Q
};
// Row blocks of the forward = first dimension of its [blocks][2][K] BatchNorm partial statistics.
int conv_igemm_row_blocks(const ConvGeom& g);
// partial (optional): [row blocks][2][K] fp32 (sum y, sum y^2) of the bf16 output.
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
// ResNet stem space-to-depth with zero padding 3: x [N][H][W][3] -> [N][(H+6)/2][(W+6)/2][12] bf16.
void stem_s2d(const void* x, void* xs, int N, int H, int W, hipStream_t st);
// dx [N][H][W][C] += small [N][Ho][Wo][C] at rows s*i, columns s*j (bf16, C a multiple of 8).
void strided_accumulate(void* dx, const void* small, int N, int H, int W, int C, int Ho, int Wo,
                        int s, hipStream_t st);
}  // namespace dca
