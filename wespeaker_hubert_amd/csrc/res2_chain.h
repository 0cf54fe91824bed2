// Fused Res2Net chain launcher (res2_chain.hip).
#pragma once

#include "common.h"

namespace wsp {

// Res2Net k3 chain of one SE_Res2Block in one launch (res2_chain.hip,
// ecapa_tdnn.py:64-78): x = conv1 output [M][ldx] (chunk i = columns [i*w, (i+1)*w)),
// out[:, i*w ..] = sp_i for i < 7.  w = scale width (64 or 128), dilation 1..4.
// w_packed = [7][3w/16][2][w/32][64][8] bf16 (hi, lo) in MFMA B-fragment order;
// bias / scale / shift = [7][w] (conv bias, eval-BN affine).
struct Res2Args {
  const float* x;
  float* out;
  int ldx, ldo, M, T, dil, rout;
  const int* seg;
  int nseg;
  const void* w;
  const float* bias;
  const float* scale;
  const float* shift;
  int variant;  // 0 / 2 / 3: 128-row windows (halo recompute); 4: strips (w = 128, else as 3)
};
bool res2_chain_supported(int w, int dil);
int res2_chain_rout(int dil, int variant, int M);  // output rows per block
void launch_res2_chain(const Res2Args& p, int w, hipStream_t s);

}  // namespace wsp
