// bf16 GEMM on the gfx950 matrix cores for Dense layers (keras.layers.Dense under mixed_bfloat16;
// the ResNet-50 classifier of BASELINE configs 4/5).  f32 accumulation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

// M, N, K multiples of 8 (16-byte operand loads); N multiple of 4 (output stores).
bool gemm_bf16_supported(int M, int N, int K);

// C[m][n] = alpha * sum_k A[m][k] B[k][n] (+ bias[n]):
//   ta = 0: A[m][k] = a[m*lda + k], ta = 1: A[m][k] = a[k*lda + m]
//   tb = 0: B[k][n] = b[n*ldb + k], tb = 1: B[k][n] = b[k*ldb + n]
// into c32 (f32, += when accumulate) or c16 (bf16) with row stride ldc.
void gemm_bf16(int ta, int tb, const void* a, long long lda, const void* b, long long ldb, int M, int N, int K,
               float* c32, void* c16, long long ldc, const float* bias, float alpha, bool accumulate, hipStream_t s);

// Global average pooling of NHWC bf16: y[n][c] = mean over the HW pixels (f32 accumulation, bf16 out);
// backward: dx[n][p][c] = dy[n][c] / HW.  C % 8 == 0.
void gap_fwd_bf16(const void* x, void* y, int N, int HW, int C, hipStream_t s);
void gap_bwd_bf16(const void* dy, void* dx, int N, int HW, int C, hipStream_t s);

// Sparse softmax cross-entropy on f32 logits [N][K] with int64 labels: loss[n] = logsumexp(z[n]) -
// z[n][label] (0 for a label outside [0, K)); backward dz = (softmax(z) - onehot) * g[n].
void softmax_xent_fwd(const float* z, const long long* labels, int N, int K, float* loss, float* lse, hipStream_t s);
// Fused loss head of the generic engine: loss_out[0] = sum of the rows' sparse softmax cross-entropy / gn,
// dz = (softmax - onehot) / gn, and the loss / accuracy metric accumulators (f64, any may be null)
// advanced by (sum of losses, N) / (correct top-1, N); one workgroup, rows summed in a fixed order.
// rows_ws: null for a one-workgroup head (small N*K), else [2N] f32 scratch of the two-kernel form
void xent_head(const float* z, const long long* labels, int N, int K, double gn, float* loss_out, float* dz,
               double* lt_total, double* lt_count, double* acc_total, double* acc_count, float* rows_ws,
               hipStream_t s);
void softmax_xent_bwd(const float* z, const long long* labels, int N, int K, const float* g, float* dz,
                      hipStream_t s);

}  // namespace tdl
