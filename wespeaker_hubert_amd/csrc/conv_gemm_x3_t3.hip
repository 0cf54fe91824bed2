// conv_gemm_x3 tile family instantiations (see conv_gemm_x3_impl.h).
#include "conv_gemm_x3_impl.h"

namespace wsp {
namespace x3 {

void t_4x2_2x2_sw(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  launch_x3_tile<4, 2, 2, 2, true>(p, h, l, s);
}

}  // namespace x3
}  // namespace wsp
