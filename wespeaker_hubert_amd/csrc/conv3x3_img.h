// Small-channel stride-1 3x3 conv of the ResNet bottleneck blocks from an LDS
// image of the input patch (conv3x3_img.hip).
#pragma once

#include "common.h"

namespace wsp {

// out[b][f][t][n] = relu(bias[n] + sum_{df,dt,c} x[b][f+df][t+dt][c] * W[n][c][df][dt] (+ res)) * scale + shift
// (zero padding 1, stride 1; scale / shift optional as in conv_gemm_x3), NHWC fp32,
// C = in = out channels.  w = [9C/16 k-steps][hi, lo][C/32 column tiles][64 lanes][8] bf16
// in MFMA B-fragment order, k = (kf * 3 + kt) * C + c (conv_gemm_x3's 2-D k order,
// so the two kernels add the same products in the same order: bit-identical).
struct Conv3x3Args {
  const float* x;
  float* out;
  int B, F, T;
  const void* w;
  const float* bias;
  const float* scale;
  const float* shift;
  const float* res = nullptr;  // optional residual [B][F][T][C], added before the ReLU (basic blocks)
  int relu = 1;                // 0: no activation (SimAM-ResNet conv2, whose BN output feeds SimAM)
  int variant = 0;             // C = 128 tile: 3 = 2 x 32 positions (two blocks per CU), else 4 x 32
};
bool conv3x3_img_supported(int C);
void launch_conv3x3_img(const Conv3x3Args& p, int C, hipStream_t s);

}  // namespace wsp
