// Implicit-GEMM conv1d on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// Replaces the nn.Conv1d calls of the reference ECAPA-TDNN
// (wespeaker/models/ecapa_tdnn.py:85-106 Conv1dReluBn, :29-78 Res2Conv1dReluBn,
// :203 self.conv, pooling_layers.py:105-117 ASTP linear1/linear2), fused with
// the bias / ReLU / eval-BatchNorm / tanh epilogues that follow them.
//
// Precision: exact fp32 products and fp32 accumulation (the f32-input MFMA is
// a k-ordered fmaf chain, cdna_hip_programming.md §3), so the result differs
// from PyTorch's CPU conv only by summation order.
//
// Tiling (256 threads = 4 waves, one 32x32 MFMA tile grid per wave):
//   block BM x BN x BK=32, waves WM x WN, each wave TM x TN tiles of 32x32.
//   LDS: A tile [BM][36] and B tile [BN][36] (k contiguous, +4 pad), double
//   buffered; a lane reads 4 consecutive k of one row with ds_read_b128 and
//   feeds 4 MFMA steps: MFMA step s of half h (lane>>5) contracts k = 16h + s,
//   the same permutation on both operands (conflict-free: row stride 9 slots).
//   Global->LDS staging is register-staged float4 (128-B row segments),
//   issued before the MFMA block and written after it (cdna guide T14).
#include "gemm_common.h"

namespace wsp {

namespace {

constexpr int BK = 32;
constexpr int LDK = BK + 4;

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI>
__global__ __launch_bounds__(256, 2) void conv_gemm_f32(const ConvGemmArgs p) {
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int AR = BM / 32;  // float4 A loads per thread per k-tile
  constexpr int BR = BN / 32;  // float4 B loads per thread per k-tile
  static_assert(WM * WN == 4, "4 waves");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* As = smem;                  // [2][BM][LDK]
  float* Bs = smem + 2 * BM * LDK;   // [2][BN][LDK]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntiles = p.N / BN;
  const int mtiles = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, ntiles * mtiles);
  const int mt = wg / ntiles;
  const int nt = wg - mt * ntiles;
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // ---- staging geometry: thread loads rows (tid>>3) + 32 i, k-chunk (tid&7)
  const int srow = tid >> 3;
  const int c4 = (tid & 7) * 4;
  ALoader<AR, AMODE, UNI> al;
  al.init(p, m0, srow, 32, c4);
  if (p.gcols) al.a0 += (n0 / p.gcols) * p.gcin;  // grouped conv: this block's input channels
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  int woff[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) woff[i] = ((n0 + srow + 32 * i) * p.Kp + c4) * 4;

  f32x4 ra[AR], rb[BR];

  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = bload4(rw, woff[i] + k0 * 4);
    al.load(k0, ra);
  };

  auto store_tile = [&](int buf) {
    float* a = As + buf * BM * LDK;
    float* b = Bs + buf * BN * LDK;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      *reinterpret_cast<f32x4*>(a + (srow + 32 * i) * LDK + c4) = ra[i];
#pragma unroll
    for (int i = 0; i < BR; ++i)
      *reinterpret_cast<f32x4*>(b + (srow + 32 * i) * LDK + c4) = rb[i];
  };

  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = p.Kp / BK;
  load_tile(0);
  store_tile(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile((kt + 1) * BK);
    const float* a = As + cur * BM * LDK + (wm * TM * 32 + r32) * LDK + h * 16;
    const float* b = Bs + cur * BN * LDK + (wn * TN * 32 + r32) * LDK + h * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const f32x4*>(a + i * 32 * LDK + q * 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) bf[j] = *reinterpret_cast<const f32x4*>(b + j * 32 * LDK + q * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  gemm_epilogue<TM, TN>(p, acc, m0, n0, wm, wn, lane);
}

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI>
void launch_k(const ConvGemmArgs& p, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const size_t lds = (size_t)2 * (BM + BN) * LDK * sizeof(float);
  hipLaunchKernelGGL((conv_gemm_f32<WM, WN, TM, TN, AMODE, UNI>), dim3(nwg), dim3(256), lds, s, p);
  WSP_HIP(hipGetLastError());
}

template <int WM, int WN, int TM, int TN>
void launch_tile(const ConvGemmArgs& p, hipStream_t s) {
  const bool uni = uniform_ktiles(p);
  if (p.amode == kAAdd) {
    if (uni) launch_k<WM, WN, TM, TN, kAAdd, true>(p, s);
    else launch_k<WM, WN, TM, TN, kAAdd, false>(p, s);
  } else {
    if (uni) launch_k<WM, WN, TM, TN, kACat, true>(p, s);
    else launch_k<WM, WN, TM, TN, kACat, false>(p, s);
  }
}

}  // namespace

int conv_gemm_tile_for(int N) { return (N % 128 == 0) ? 0 : 1; }

void launch_conv_gemm(const ConvGemmArgs& args, hipStream_t s) {
  const ConvGemmArgs p = normalized(args);
  check_conv_args(p, "conv_gemm");
  WSP_CHECK(!p.colsum, "conv_gemm: column sums are a bf16x3-kernel epilogue");
  WSP_CHECK(!p.conv2d && p.N % 64 == 0, "conv_gemm (f32): 1-D convs with N % 64 == 0 only");
  WSP_CHECK(!p.gcols || p.gcols % 64 == 0, "conv_gemm (f32): grouped columns must be a multiple of 64");
  if (conv_gemm_tile_for(p.N) == 0 && !p.gcols)
    launch_tile<2, 2, 2, 2>(p, s);
  else
    launch_tile<4, 1, 1, 2>(p, s);
}

}  // namespace wsp
