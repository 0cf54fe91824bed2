// ResNet bottleneck conv1 (1x1, K = 4p -> N = p, no residual) from whole activation
// rows staged in LDS (conv1x1_rows.hip).
#pragma once

#include "common.h"

namespace wsp {

// out[m][n] = relu(bias[n] + sum_k x[m][k] * W[n][k]) * scale[n] + shift[n], fp32
// rows m < M (leading dimensions ldx = K, ldo = N).  w = [K/16 k-steps][hi, lo][N/32
// column tiles][64 lanes][8] bf16 in MFMA B-fragment order (the conv3x3_img layout with
// one tap), k ascending: the same products in the same order as conv_gemm_x3 (bit-identical).
struct Conv1x1Args {
  const float* x;
  float* out;
  int M;
  const void* w;
  const float* bias;
  const float* scale;
  const float* shift;
  int relu = 1;
};
bool conv1x1_rows_supported(int K, int N);
void launch_conv1x1_rows(const Conv1x1Args& p, int K, int N, hipStream_t s);

}  // namespace wsp
