// Implicit-GEMM conv1d on gfx950 bf16 MFMA with a 3-term split ("bf16x3"):
//   a = a_hi + a_lo,  a_hi = bf16(a), a_lo = bf16(a - a_hi)   (same for w)
//   a*w ~= a_hi*w_hi + a_hi*w_lo + a_lo*w_hi   (fp32 accumulation in the MFMA)
// The dropped a_lo*w_lo term and the split remainders are ~2^-17 relative,
// i.e. products are accurate to ~1e-5 relative with fp32 accumulation —
// fp32-class results (measured on the c1024 golden fixture: max |d emb|
// 3.5e-6) at 3 bf16 MFMAs per K=16 step = 5.3x the f32-MFMA rate.
//
// Same operator and epilogue contract as conv_gemm.hip (ConvGemmArgs), used
// for the reference's Conv1d layers (ecapa_tdnn.py:85-106, :29-78, :203,
// pooling_layers.py:105-117).
//
// Tiling: NW waves (4 or 8), block BM x BN x BK=32, each wave TM x TN tiles
// of 32x32 (v_mfma_f32_32x32x16_bf16).  The default (variant 5) uses, where
// N % 256 == 0, a 256 x 256 block of 8 waves with 64 x 128 per wave (12 fragment
// reads per 24 MFMAs instead of 8 per 12) and ONE register staging set — its
// 128 accumulators leave no room for a second.  A (fp32 activations) is split into
// hi/lo bf16 while staging; W is pre-split on the host.  LDS rows are
// 32 bf16 + 8 pad (80 B): the 16-byte fragment reads (row = lane&31,
// k = 16 s + 8 (lane>>5)) hit 16 distinct slots per ds_read_b128 group.
#include "conv_gemm_x3_impl.h"

namespace wsp {

int conv_gemm_x3_block_rows(const ConvGemmArgs& p, int variant) {
  if (p.N % 64 != 0 || (p.gcols && p.gcols % 64 != 0)) return 128;
  if (p.gcols || p.N % 128 != 0) return 128;
  return variant == 3 ? 128 : 256;
}

namespace {
__global__ __launch_bounds__(256) void colsum_mean_kernel(const double* __restrict__ part, int bm, int T, int N,
                                                          float* __restrict__ out, int ldo) {
  const int b = blockIdx.y;
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const long r0 = (long)b * T, r1 = r0 + T;  // utterance rows
  double v = 0.0;
  for (long mt = r0 / bm; mt * bm < r1; ++mt) {
    const int slot = (mt * bm) / T == b ? 0 : 1;  // the block starts in utterance b, or in b-1
    v += part[((size_t)mt * 2 + slot) * N + n];
  }
  out[(long)b * ldo + n] = (float)(v / (double)T);
}
}  // namespace

void launch_colsum_mean(const double* part, int block_rows, int T, int B, int N, float* out, int ldo,
                        hipStream_t s) {
  WSP_CHECK(block_rows > 0 && T >= block_rows && B > 0 && N > 0, "colsum_mean: bad shape");
  hipLaunchKernelGGL(colsum_mean_kernel, dim3((N + 255) / 256, B), dim3(256), 0, s, part, block_rows, T, N, out,
                     ldo);
  WSP_HIP(hipGetLastError());
}

void launch_conv_gemm_x3(const ConvGemmArgs& args, const void* whi, const void* wlo, int variant,
                         hipStream_t s) {
  const ConvGemmArgs p = normalized(args);
  check_conv_args(p, "conv_gemm_x3");
  if (p.colsum) {
    const int bm = conv_gemm_x3_block_rows(p, variant);
    WSP_CHECK(!p.seg && !p.row_bias && !p.conv2d && p.T >= bm,
              "conv_gemm_x3: column sums need a uniform batch with T >= block rows and no row bias");
  }
  WSP_CHECK(p.Kp % 64 == 0, "conv_gemm_x3: packed K must be a multiple of 64");
  WSP_CHECK(variant >= 3 && variant <= 7, "conv_gemm_x3: tile family must be 3, 4, 5, 6 or 7");
  const __bf16* h = static_cast<const __bf16*>(whi);
  const __bf16* l = static_cast<const __bf16*>(wlo);
  x3::TileFn f;
  WSP_CHECK(!p.lnmode || (variant == 7 && x3::g256_supported(p)),
            "conv_gemm_x3: the LayerNorm fold runs on tile family 7 only");
  WSP_CHECK(!p.sc2d || (variant == 7 && x3::g256_supported(p)),
            "conv_gemm_x3: conv3 + shortcut runs on tile family 7 only (N % 256 == 0, 16-B aligned operands)");
  if (variant == 7 && x3::g256_supported(p)) {
    // variant 7 (r4): the 256 x 256 16x16x32 tile with every operand staged by LDS-DMA and the
    // fp32 A split at fragment time (conv_gemm_x3_t6.hip); bit-identical to 6, which serves
    // the operands it does not take (2-D, added operand, grouped, N % 256 != 0)
    x3::t_g256(p, h, l, s);
    return;
  }
  if (variant == 7) variant = 6;
  if (p.N % 64 != 0 || (p.gcols && p.gcols % 64 != 0)) {
    f = x3::t_4x1_1x1;  // 128 x 32, 4 waves
  } else if (p.gcols) {
    // grouped (HuBERT pos_conv: 16 groups x 64 padded columns, K = 48 x 128): 256-row
    // blocks halve the per-row re-reads of the group's 1.5 MB weight slice
    f = variant >= 5 ? x3::t_8x1_1x2_sw : x3::t_4x1_1x2;  // blocks stay inside one group
  } else if (p.N % 128 != 0) {
    f = x3::t_4x1_1x2;  // 128 x 64, 4 waves
  } else if (variant == 3) {
    f = x3::t_2x2_2x2_sw;  // 128 x 128, 4 waves, swizzled rows: 2 blocks / CU
  } else if (variant == 4) {
    f = x3::t_4x2_2x2_sw;  // 256 x 128, 8 waves, swizzled rows
  } else if (p.N % 256 == 0) {
    // variant 5: 256 x 256 (8 waves 4 x 2, 64 x 128 per wave) wherever N allows it: in-model
    // C x C -10 %, conv_cat -15 %, HuBERT fc1 -18 %, fc2 -20 %, CNN -12 % vs 256 x 128 (with
    // the per-tile residual epilogue and the A&S GELU; the libm erff made fc1's epilogue lose).
    // variant 6: the same tile on v_mfma_f32_16x16x32_bf16 (MI355X holds a higher clock on that
    // shape; ECAPA default, C2 +0.8-1.2 %; HuBERT measured neutral: fc2 / CNN faster, QKV /
    // out_proj slower)
    f = variant == 6 ? x3::t_4x2_2x4_mf16 : x3::t_4x2_2x4_sw1;
  } else {
    f = x3::t_4x2_2x2_sw;  // variant 5 with N % 256 != 0
  }
  f(p, h, l, s);
}

}  // namespace wsp
