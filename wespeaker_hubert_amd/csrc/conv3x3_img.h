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

// Bottleneck tail in one launch (resnet.py:101-107, stride 1):
//   y2  = relu(conv2_3x3(y1) + b2)                 (bn2 folded; never leaves the CU)
//   out = relu(conv3_1x1(y2) + b3 + res)           (bn3 folded; res = x or the shortcut)
// y1 [B][F][T][C], res / out [B][F][T][4C], NHWC fp32, C = planes in {32, 64, 128}.
// w2 = conv3x3_img's fragment image of conv2.  w3 = [C/16 k-steps][hi, lo][4C/32 column
// tiles][64 lanes][8] bf16 B fragments of conv3 whose lane l, element e holds
// W3[n][16 ks + (e & 3) + 8 (e >> 2) + 4 (l >> 5)]: the k order in which conv2's
// transposed accumulators hold y2's channels, so they feed conv3 as its A operand
// straight from registers (Model::Impl::pack_frag_acc).
struct BottleneckTailArgs {
  const float* y1;
  const float* res;
  float* out;
  int B, F, T;
  const void* w2;
  const float* b2;
  const void* w3;
  const float* b3;
  // optional: the NEXT block's conv1 (1x1, 4C -> C, bn1 folded, ReLU) on `out` while it is on
  // chip: w1n = pack_frag B fragments [4C/16][hi, lo][C/32][64][8], y1n [B][F][T][C]
  const void* w1n = nullptr;
  const float* b1n = nullptr;
  float* y1n = nullptr;
  // the next conv1's output channels: C, or 2C at a stage transition (the next stage's first
  // block: 4C -> 2C, y1n [B][F][T][2C]; 32 / 64 planes); 0 = C
  int c1n = 0;
  // optional (32 planes, with w1n): the block's projection shortcut computed inside conv3 from its
  // input x [B][F][T][C] (C -> 4C; w3 then holds KS3 more k-steps, natural k order, and b3 = b3 +
  // b_sc); res must be null
  const float* xsc = nullptr;
};
bool bottleneck_tail_supported(int C);
void launch_bottleneck_tail(const BottleneckTailArgs& p, int C, hipStream_t s);

}  // namespace wsp
