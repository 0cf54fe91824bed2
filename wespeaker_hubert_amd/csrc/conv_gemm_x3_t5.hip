// conv_gemm_x3 tile family instantiations (see conv_gemm_x3_impl.h).
#include "conv_gemm_x3_impl.h"

namespace wsp {
namespace x3 {

void t_4x2_2x4_mf16(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  if (p.conv2d || p.amode == kAAdd) {  // not instantiated on 16x16 (nothing launches them there)
    t_4x2_2x4_sw1(p, h, l, s);
    return;
  }
  launch_x3_tile<4, 2, 2, 4, true, 1, 16>(p, h, l, s);
}

}  // namespace x3
}  // namespace wsp
