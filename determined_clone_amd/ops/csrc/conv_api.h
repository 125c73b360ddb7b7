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
// With bn_x / bn_mask / bn_mean (data gradient of a convolution whose input was relu(bn(bn_x)),
// y laid out like bn_x): partial receives that BatchNorm's BACKWARD statistics instead,
// (sum g*m, sum g*m*(bn_x - bn_mean)) of the bf16 output g masked by the ReLU bits m.
void conv_igemm_fwd(const void* x, const void* w, void* y, float* partial, const ConvGeom& g,
                    hipStream_t st, const void* bn_x = nullptr, const uint8_t* bn_mask = nullptr,
                    const float* bn_mean = nullptr);
// Weight gradient dW (bf16 or fp32; accumulate adds into it) from dy [M][K] and x, stored
// [K][R][S][C] (channels_last) or, with dw_kcrs, [K][C][R][S]; ws: conv_igemm_wgrad_ws_floats(g)
// fp32 scratch.
int64_t conv_igemm_wgrad_ws_floats(const ConvGeom& g);
void conv_igemm_wgrad(const void* dy, const void* x, float* ws, void* dw, bool dw_f32,
                      bool accumulate, bool dw_kcrs, const ConvGeom& g, hipStream_t st);
// w [K][RS][C] -> wt [C][RS][K] with the taps reversed (stride-1 data-gradient weight).
void conv_flip_transpose(const void* w, void* wt, int K, int C, int RS, hipStream_t st);
// ResNet stem space-to-depth with zero padding 3: x [N][H][W][3] -> [N][(H+6)/2][(W+6)/2][co] bf16
// (co = 12, or 16 with 4 zero channels for stem_conv_fwd).
void stem_s2d(const void* x, void* xs, int N, int H, int W, int co, hipStream_t st);
// Stem 4x4/1 convolution on the 16-channel S2D tensor: xs [N][Hs][Ws][16], w16 [64][4][4][16] ->
// y [N][Hs-3][Ws-3][64] bf16 + BatchNorm partial statistics [stem_conv_blocks()][2][64] fp32.
// Requires Ws - 3 >= 64 and Ws <= 256.
int stem_conv_blocks(int N, int Hs, int Ws);
// Stem weight gradient on the 12-channel S2D tensor: dy [N][Hs-3][Ws-3][64], xs [N][Hs][Ws][12] bf16
// -> per-block fp32 partials ws [stem_wgrad_blocks(N)][64][4 (di)][4 (dj)][12] (summed by the
// caller). Requires Ws - 3 <= 128.
int stem_wgrad_blocks(int N);
void stem_wgrad(const void* dy, const void* xs, float* ws, int N, int Hs, int Ws, hipStream_t st);
void stem_conv_fwd(const void* xs, const void* w16, void* y, float* partial, int N, int Hs, int Ws,
                   hipStream_t st);
// dx [N][H][W][C] += small [N][Ho][Wo][C] at rows s*i, columns s*j (bf16, C a multiple of 8).
void strided_accumulate(void* dx, const void* small, int N, int H, int W, int C, int Ho, int Wo,
                        int s, hipStream_t st);
}  // namespace dca
