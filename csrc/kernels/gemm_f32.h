// Exact-fp32 MFMA GEMM with the learner's fused epilogues (gemm_f32.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace sa {

// v = acc [+ bias[n]] [* (mask[m, n] > 0)] [relu] [+= C[m, n]] -> C[m, n]
// aug_c0 > 0: also writes C[m, aug_c0 ..ldc) = [clip(reward[m], -1, 1),
// one_hot(action[m]), 0...] (the core-input columns next to the torso FC).
struct GemmEpilogue {
  float* C;
  int ldc;
  const float* bias;
  const float* mask;
  int ldm;
  int relu;
  int accumulate;
  float* colsum;  // ones_row: [N] += column sums of op(B) over K
  const float* aug_reward;
  const int64_t* aug_action;
  int aug_c0;
};

// K splits the launch would use (grid.z) and the partial-slab workspace they
// need (floats; 0 when no split).
int gemm_f32_splits(int M, int N, int K, int ones_row);
int64_t gemm_f32_part_floats(int M, int N, int K, int ones_row, int splits);

// C[M, N] (+)= op(A) op(B): op(A)[m, k] = ta ? A[k*lda + m] : A[m*lda + k],
// op(B)[k, n] = tb ? B[n*ldb + k] : B[k*ldb + n].  lda, ldb, K multiples of
// 4 and 16-B aligned bases (false otherwise, nothing launched).
bool gemm_f32_launch(const float* A, const float* B, int M, int N, int K, int lda,
                     int ldb, bool ta, bool tb, bool ones_row, int splits, float* part,
                     const GemmEpilogue& ep, hipStream_t stream);

}  // namespace sa
