// Host API of the transformer kernel family (transformer.hip, attention.hip), shared by the
// kernels' translation units and the PyTorch bindings.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dca {
enum class TDtype : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

// Destination of a column reduction (bias / LayerNorm-affine gradients): column j < split goes to
// p0[j], the rest to p1[j - split]; fp32 or bf16 elements. accumulate = add to the existing value
// -- used to write parameter gradients straight into their persistent .grad views (flat ZeRO/DDP
// buffers), which removes autograd's separate AccumulateGrad kernels.
struct ColumnOut {
  void* p0 = nullptr;
  void* p1 = nullptr;
  int64_t split = 0;
  bool bf16 = false;
  bool accumulate = false;
};
int ln_bwd_blocks(int64_t rows);
void layernorm_fwd(TDtype dt, const void* x, const void* res, void* sum_out, void* y,
                   const float* gamma, const float* beta, float* mean, float* rstd, int64_t rows,
                   int D, float eps, hipStream_t st);
// floats of `partial` layernorm_bwd needs
int64_t ln_bwd_partial_floats(int64_t rows, int D, bool colsum);
// dx_colsum (optional): column sums of dx (the bias gradient of the linear layer whose output fed
// the LayerNorm as its residual); partial then holds [blocks][3][D].
void layernorm_bwd(TDtype dt, const void* dy, const void* x, const float* gamma, const float* mean,
                   const float* rstd, const void* dsum, void* dx, float* partial,
                   const ColumnOut* dgamma_dbeta, int64_t rows, int D, hipStream_t st,
                   const ColumnOut* dx_colsum = nullptr);
void bias_gelu_fwd(TDtype dt, const void* x, const void* bias, bool bias_bf16, void* y,
                   int64_t rows, int N, hipStream_t st);
int bias_gelu_bwd_row_blocks(int64_t rows);
void bias_gelu_bwd(TDtype dt, const void* dy, const void* x, const void* bias, bool bias_bf16,
                   void* dx, float* partial, const ColumnOut* dbias, int64_t rows, int N,
                   hipStream_t st);
// Bias gradient of a linear layer: out[j] (+)= sum_r dy[r][j], dy [rows][N] (N % 8 == 0).
int row_sum_blocks(int64_t rows, int N);
// acc[i] (+)= sum_s part[s][i], part fp32 [splits][n], acc bf16 or fp32 [n] (n % 8 == 0).
void splitk_accumulate(bool acc_bf16, const float* part, void* acc, int64_t n, int splits,
                       bool accumulate, hipStream_t st);
void row_sum(TDtype dt, const void* dy, float* partial, const ColumnOut& out, int64_t rows, int N,
             hipStream_t st);
void rope(TDtype dt, const void* x, void* y, const float* cosT, const float* sinT, int64_t rows,
          int H, int S, int D, int rot, bool backward, hipStream_t st);
void attention_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H,
                   int Sq, int Sk, int D, const int64_t* qs, const int64_t* ks, const int64_t* vs,
                   const int64_t* os, float scale, bool causal, const int* kvlen, int G,
                   hipStream_t st);
void attention_bwd(const void* q, const void* k, const void* v, const void* o, const void* dO,
                   const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                   int B, int H, int Sq, int Sk, int D, const int64_t* st_q, const int64_t* st_k,
                   const int64_t* st_v, const int64_t* st_o, const int64_t* st_do,
                   const int64_t* st_dq, const int64_t* st_dk, const int64_t* st_dv, float scale,
                   bool causal, const int* kvlen, int G, hipStream_t stream);
void cross_entropy_fwd(TDtype dt, const void* logits, const int64_t* target, float* lse,
                       float* loss, int64_t rows, int V, int64_t ignore_index, hipStream_t st);
void cross_entropy_bwd(TDtype dt, const void* logits, const int64_t* target, const float* lse,
                       const float* gscale, void* dlogits, int64_t rows, int V,
                       int64_t ignore_index, hipStream_t st);
}  // namespace dca
