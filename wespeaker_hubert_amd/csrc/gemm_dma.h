// LDS-DMA staged bf16x3 GEMM variants (conv_gemm_dma.hip) beyond the default
// launch_conv_gemm_dma (variant 0 = 256 x 128 / 8 waves / 3 stages):
//   2 = 256 x 256 block, 8 waves of 64 x 128, 2 stages (N % 256 == 0; supports the
//       fused SE column sums with 256 block rows, as conv_gemm_x3 variant 5)
// Measured on MI355X (ECAPA c1024, B = 256): slower than conv_gemm_x3 variant 5
// (C x C conv 4.79 vs 4.45 ms/step; a 16-wave 64 x 64 form spilled ~490 VGPRs
// at the 128-register cap and ran 4.93 ms) -- kept as a selectable variant.
#pragma once

#include "kernels.h"

namespace wsp {

bool conv_gemm_dma_v_supported(const ConvGemmArgs& p, int variant);
void launch_conv_gemm_dma_v(const ConvGemmArgs& p, const void* whi, const void* wlo, int variant, hipStream_t s);

}  // namespace wsp
