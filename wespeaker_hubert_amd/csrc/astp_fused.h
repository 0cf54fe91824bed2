// Fused attentive-statistics pooling head (astp_fused.hip).
#pragma once

#include "common.h"

namespace wsp {

// ASTP second projection + softmax-over-frames statistics in one launch
// (pooling_layers.py:133-144): per utterance b and channel c
//   e[t][c]  = bias2[c] + sum_k att[t][k] * W2[c][k]          (linear2, K = 128)
//   alpha    = softmax_t(e[:, c]);  mu = sum_t alpha x[t][c]
//   sd       = sqrt(max(sum_t alpha x[t][c]^2 - mu^2, var_floor))
//   out[b] = [mu (C) | sd (C)]
// e is never written: the logits stay in the MFMA accumulators (bf16x3).
// att: [rows][128] fp32 (tanh(linear1) output), x: [rows][ldx] fp32, rows of
// utterance b = [seg[b], seg[b+1]) or [b*T, (b+1)*T).  w2 = [8][2][C/32][64][8]
// bf16 (hi, lo) in MFMA B-fragment order (k-step, plane, column tile, lane).
struct AstpArgs {
  const float* att;
  const float* x;
  int ldx, B, T, C;
  const int* seg;
  const void* w2;
  const float* bias2;
  float var_floor;
  float* out;
};
bool astp_fused_supported(int C, int K);  // K = 128, C % 256 == 0
void launch_astp_fused(const AstpArgs& p, hipStream_t s);

}  // namespace wsp
