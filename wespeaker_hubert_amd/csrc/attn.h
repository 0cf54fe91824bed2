// HuBERT self-attention with K / V staged once per key block in LDS (attn.hip).
#pragma once

#include "common.h"

namespace wsp {

// softmax(Q K^T / sqrt(dh)) V per (utterance, head); qkv [rows][ldq] = [q | k | v]
// (H*dh each), out [rows][ldo]; seg (device [B+1] row offsets) for ragged batches.
// pipe = 1: the persistent pipelined kernel (default), 0: one block per (utterance, head)
void launch_attn(const float* qkv, int ldq, float* out, int ldo, int B, int T, int H, int dh, hipStream_t s,
                 const int* seg = nullptr, int pipe = 1);

}  // namespace wsp
