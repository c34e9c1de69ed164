// bf16-operand MFMA GEMM (fp32 accumulate) with the learner's fused
// epilogues (gemm_bf16.hip): the bf16 learner's torso-FC / LSTM input
// projection / their gradients.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {

// v = acc [+ bias[n]] [* (mask[m, n] > 0)] [relu] [+= C[m, n] (fp32 C only)]
// -> C[m, n] as fp32 or bf16 (c_bf16).  aug_c0 > 0: also writes C[m, aug_c0
// .. ldc) = [clip(reward[m], -1, 1), one_hot(action[m]), 0...] (the core-input
// columns next to the torso FC, experiment.py:191-198).
struct GemmBf16Epilogue {
  void* C;
  int ldc;
  int c_bf16;
  const float* bias;
  const uint16_t* mask;  // bf16 [M, ldm] (the ReLU derivative source)
  int ldm;
  int relu;
  int accumulate;
  float* colsum;  // ones_row: [N] += column sums of op(B) over K
  const float* aug_reward;
  const int64_t* aug_action;
  int aug_c0;
};

int gemm_bf16_splits(int M, int N, int K, int ones_row);
int64_t gemm_bf16_part_floats(int M, int N, int K, int ones_row, int splits);

// C[M, N] (+)= op(A) op(B) over bf16 A / B: op(A)[m, k] = ta ? A[k*lda + m] :
// A[m*lda + k], op(B)[k, n] = tb ? B[n*ldb + k] : B[k*ldb + n].  lda, ldb
// multiples of 8 (16-B rows) and 16-B aligned bases; K a multiple of 8 where
// it is an operand's contiguous index (!ta or tb).  false = nothing launched.
bool gemm_bf16_launch(const uint16_t* A, const uint16_t* B, int M, int N, int K,
                      int lda, int ldb, bool ta, bool tb, bool ones_row, int splits,
                      float* part, const GemmBf16Epilogue& ep, hipStream_t stream);

}  // namespace sa
