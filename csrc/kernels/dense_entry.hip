// Production entry points of the dense / 1x1-conv GEMMs: straight to the native MFMA
// kernels of igemm.hip.  (The bench-only twin library swaps this file for
// csrc/bench/blaslt.hip, which adds a timed per-shape hipBLASLt selection for A/B runs;
// this library links no vendor GEMM library at all.)
#include "common.h"

extern "C" int mlc_gemm_bf16_ex_native(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int lda, int ldb,
                                       int ldc, int ta, int tb, const float* bias, int act, bf16* preact,
                                       const bf16* addend, const bf16* dact, float* ws, long ws_floats,
                                       hipStream_t st);
extern "C" int mlc_conv_wgrad_native(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C, int Co,
                                      int KH, int KW, int stride, int pad, int dil, int Ho, int Wo, int splits,
                                      int accumulate, float* ws, long ws_floats, const float* in_sc,
                                      const float* in_sh, hipStream_t st);
extern "C" int mlc_linear_wgrad_bias_native(const bf16* A, const bf16* B, float* C, float* dbias, int M, int N,
                                            int K, int lda, int ldb, int ldc, int splits, float* ws, long ws_floats,
                                            hipStream_t st);

MLC_EXPORT int mlc_gemm_bf16_ex(const bf16* A, const bf16* B, bf16* C, int M, int N, int K, int lda, int ldb,
                                int ldc, int ta, int tb, const float* bias, int act, bf16* preact,
                                const bf16* addend, const bf16* dact, float* ws, long ws_floats,
                                hipStream_t st) {
  return mlc_gemm_bf16_ex_native(A, B, C, M, N, K, lda, ldb, ldc, ta, tb, bias, act, preact, addend, dact, ws,
                                 ws_floats, st);
}

MLC_EXPORT int mlc_linear_wgrad_bias(const bf16* A, const bf16* B, float* C, float* dbias, int M, int N, int K,
                                     int lda, int ldb, int ldc, int splits, float* ws, long ws_floats,
                                     hipStream_t st) {
  return mlc_linear_wgrad_bias_native(A, B, C, dbias, M, N, K, lda, ldb, ldc, splits, ws, ws_floats, st);
}

MLC_EXPORT int mlc_conv_wgrad(const bf16* dy, const bf16* x, float* dw, int N, int H, int W, int C, int Co, int KH,
                              int KW, int stride, int pad, int dil, int Ho, int Wo, int splits, int accumulate,
                              float* ws, long ws_floats, const float* in_sc, const float* in_sh, hipStream_t st) {
  return mlc_conv_wgrad_native(dy, x, dw, N, H, W, C, Co, KH, KW, stride, pad, dil, Ho, Wo, splits, accumulate, ws,
                               ws_floats, in_sc, in_sh, st);
}

// The library selection does not exist in this build: the mode reads 0 and any request to
// turn it on is refused (-1); no cached choices.
MLC_EXPORT int mlc_blaslt_mode(int m) { return m > 0 ? -1 : 0; }
MLC_EXPORT int mlc_blaslt_choices(int* out, int cap) { return 0; }
