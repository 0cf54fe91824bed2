// Implicit-GEMM conv1d, bf16x3 split MFMA, LDS-DMA staged (gfx950).
//
// Same operator / epilogue contract as conv_gemm_x3.hip (ConvGemmArgs, kACat
// operands): the reference's Conv1d layers (ecapa_tdnn.py:85-106 / :203,
// pooling_layers.py:105-117).  Differences from the register-staged kernel:
//   * global -> LDS with buffer_load ... lds (LDS-DMA, 16 B per lane): no VGPR
//     staging, no VALU/ds_write store pass; a 3-stage LDS ring keeps two
//     k-tiles in flight behind the one being multiplied (counted vmcnt, raw
//     s_barrier — cdna_hip_programming.md §5 "Pipelining across barriers");
//   * A stays fp32 in LDS and is split into bf16 hi/lo at fragment-read time;
//     W arrives as pre-split bf16 hi/lo images;
//   * LDS images are lane-linear per DMA instruction; the XOR swizzle lives on
//     the per-lane SOURCE chunk (A: chunk ^ ((row>>1)&7), W: chunk ^ ((row>>2)&3))
//     and on the fragment read, making every ds_read_b128 conflict-free;
//   * out-of-range buffer offsets (conv padding, tail tiles) load zeros.
// Block 256 x 128 x 32, 8 waves (4 x 2), each 2 x 2 tiles of 32x32x16 MFMA.
#include "gemm_common.h"
#include "gemm_dma.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BK = 32;

// s_waitcnt vmcnt(N) needs a literal
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ void split8(const f32x4& x0, const f32x4& x1, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h0 = (__bf16)x0[e];
    const __bf16 h1 = (__bf16)x1[e];
    hi[e] = h0;
    hi[4 + e] = h1;
    lo[e] = (__bf16)(x0[e] - (float)h0);
    lo[4 + e] = (__bf16)(x1[e] - (float)h1);
  }
}

// WM x WN waves of TM x TN 32x32 tiles, NST-stage LDS ring (NST - 1 tiles in
// flight behind the one being multiplied).
template <int WM, int WN, int TM, int TN, int NST, bool UNI, int ROLE>
__global__ __launch_bounds__(WM* WN * 64, WM* WN / 4) void conv_gemm_x3d(const ConvGemmArgs p,
                                                                          const __bf16* __restrict__ whi,
                                                                          const __bf16* __restrict__ wlo) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int A_BYTES = BM * BK * 4;   // fp32 rows of 128 B
  constexpr int B_IMG = BN * BK * 2;     // bf16 rows of 64 B
  constexpr int STAGE = A_BYTES + 2 * B_IMG;
  constexpr int A_INS = BM / 8 / NW;     // 1-KB A DMA instructions per wave per tile
  constexpr int B_INS = BN / 16 / NW;    // per image
  static_assert(A_INS >= 1 && B_INS >= 1, "tile/wave mismatch");
  constexpr int OPS = A_INS + 2 * B_INS; // DMA ops per wave per tile

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = p.N / BN;
  const int mtiles = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, ntiles * mtiles);
  const int mt = wg / ntiles;
  const int nt = wg - mt * ntiles;
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // ---- A DMA geometry: instruction i of this wave covers tile rows
  // (wave*A_INS + i)*8 .. +7; lane -> row (lane>>3), physical chunk (lane&7)
  // holding logical chunk pc ^ ((row>>1)&7).
  int a_m[A_INS], a_t[A_INS], a_lc[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int row = (wave * A_INS + i) * 8 + (lane >> 3);
    const int m = m0 + row;
    a_m[i] = m;
    a_t[i] = (m < p.M) ? (m % p.T) : -0x40000000;
    a_lc[i] = ((lane & 7) ^ ((row >> 1) & 7)) * 4;  // logical float offset in the k-tile
  }
  // ---- W DMA geometry: instruction covers 16 rows of 64 B; lane -> row
  // (lane>>2), physical chunk (lane&3) holding logical chunk pc ^ ((row>>2)&3).
  int b_off[B_INS];
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    const int row = (wave * B_INS + i) * 16 + (lane >> 2);
    b_off[i] = ((n0 + row) * p.Kp + ((lane & 3) ^ ((row >> 2) & 3)) * 8) * 2;
  }
  const __amdgpu_buffer_rsrc_t rwhi = make_rsrc(whi);
  const __amdgpu_buffer_rsrc_t rwlo = make_rsrc(wlo);
  const float* a0 = p.a[0];
  const float* a1 = p.a[1];
  const float* a2 = p.a[2];
  int tj = 0, tc = 0;  // UNI: tap / channel of the next tile to issue

  auto issue = [&](int k0, int stage, bool live) {
    unsigned char* st = smem + stage * STAGE;
    if constexpr (UNI) {
      const int off = tj * p.dil - p.pad;
      const float* base = a0;
      int ld = p.lda[0], cl = tc;
      if (tc >= p.cseg[2]) {
        base = a2;
        ld = p.lda[2];
        cl = tc - p.cseg[2];
      } else if (tc >= p.cseg[1]) {
        base = a1;
        ld = p.lda[1];
        cl = tc - p.cseg[1];
      }
      const __amdgpu_buffer_rsrc_t ra = make_rsrc(base);
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int tt = a_t[i] + off;
        const bool ok = live && tt >= 0 && tt < p.T;
        dma16(ra, st + (wave * A_INS + i) * 1024, ok ? ((a_m[i] + off) * ld + cl + a_lc[i]) * 4 : kOOB);
      }
      tc += BK;
      if (tc >= p.cin) {
        tc -= p.cin;
        ++tj;
      }
    } else {
      const __amdgpu_buffer_rsrc_t ra = make_rsrc(a0);
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int k = k0 + a_lc[i];
        const bool kin = live && k < p.K;
        const int j = kin ? k / p.cin : 0;
        const int c = k - j * p.cin;
        const int off = j * p.dil - p.pad;
        const int tt = a_t[i] + off;
        const bool ok = kin && tt >= 0 && tt < p.T;
        dma16(ra, st + (wave * A_INS + i) * 1024, ok ? ((a_m[i] + off) * p.lda[0] + c) * 4 : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < B_INS; ++i) {
      const int o = live ? b_off[i] + k0 * 2 : kOOB;
      dma16(rwhi, st + A_BYTES + (wave * B_INS + i) * 1024, o);
      dma16(rwlo, st + A_BYTES + B_IMG + (wave * B_INS + i) * 1024, o);
    }
  };

  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  // fragment read offsets (bytes, within a stage)
  int a_rd[TM][2][2], b_rd[TN][2];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = (wm * TM + i) * 32 + r32;
    const int sw = (row >> 1) & 7;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int q = 0; q < 2; ++q) a_rd[i][s][q] = row * 128 + (((4 * s + 2 * h + q) ^ sw) * 16);
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int row = (wn * TN + j) * 32 + r32;
    const int sw = (row >> 2) & 3;
#pragma unroll
    for (int s = 0; s < 2; ++s) b_rd[j][s] = A_BYTES + row * 64 + (((2 * s + h) ^ sw) * 16);
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = p.Kp / BK;
#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0) issue(s0 * BK, s0, s0 < nk);

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed (this wave's part); the barrier publishes every wave's
    // part and retires all reads of the stage the next issue overwrites.
    wait_vmcnt<OPS * (NST - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue((kt + NST - 1) * BK, (kt + NST - 1) % NST, kt + NST - 1 < nk);
    const unsigned char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(st + b_rd[j][s]);
        bl[j] = *reinterpret_cast<const bf16x8*>(st + b_rd[j][s] + B_IMG);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + a_rd[i][s][0]);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + a_rd[i][s][1]);
        split8(x0, x1, ah[i], al[i]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  }
  // drain the (dummy) DMA still in flight before the LDS is reused / released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the fused column sums reuse the LDS

  gemm_epilogue<TM, TN, WM, WN>(p, acc, m0, n0, wm, wn, lane, smem);
}

template <int WM, int WN, int TM, int TN, int NST, bool UNI, int ROLE>
void launch_d(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int STAGE = BM * BK * 4 + 2 * BN * BK * 2;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  hipLaunchKernelGGL((conv_gemm_x3d<WM, WN, TM, TN, NST, UNI, ROLE>), dim3(nwg), dim3(WM * WN * 64),
                     (size_t)NST * STAGE, s, p, whi, wlo);
  WSP_HIP(hipGetLastError());
}

template <int WM, int WN, int TM, int TN, int NST>
void launch_dv(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  if (!uniform_ktiles(p))
    launch_d<WM, WN, TM, TN, NST, false, 0>(p, h, l, s);
  else if (p.role == 1)
    launch_d<WM, WN, TM, TN, NST, true, 1>(p, h, l, s);
  else
    launch_d<WM, WN, TM, TN, NST, true, 0>(p, h, l, s);
}

}  // namespace

bool conv_gemm_dma_supported(const ConvGemmArgs& p) {
  return !p.colsum && !p.conv2d && p.amode == kACat && p.N % 128 == 0 && (uniform_ktiles(p) || p.cseg[1] == p.cin) &&
         p.stride <= 1 && (p.Ti == 0 || p.Ti == p.T) && !p.gcols && !p.seg;
}

bool conv_gemm_dma_v_supported(const ConvGemmArgs& p, int variant) {
  if (variant == 0) return conv_gemm_dma_supported(p);
  return !p.conv2d && p.amode == kACat && p.N % 256 == 0 && (uniform_ktiles(p) || p.cseg[1] == p.cin) &&
         p.stride <= 1 && (p.Ti == 0 || p.Ti == p.T) && !p.gcols && !p.seg;
}

void launch_conv_gemm_dma_v(const ConvGemmArgs& args, const void* whi, const void* wlo, int variant, hipStream_t s) {
  const ConvGemmArgs p = normalized(args);
  check_conv_args(p, "conv_gemm_dma");
  WSP_CHECK(conv_gemm_dma_v_supported(p, variant), "conv_gemm_dma: unsupported operand layout");
  if (p.colsum) WSP_CHECK(!p.row_bias && p.T >= 256, "conv_gemm_dma: column sums need T >= 256 and no row bias");
  const __bf16* h = static_cast<const __bf16*>(whi);
  const __bf16* l = static_cast<const __bf16*>(wlo);
  switch (variant) {
    case 0: launch_dv<4, 2, 2, 2, 3>(p, h, l, s); break;   // 256 x 128, 8 waves, 3 stages
    case 2: launch_dv<4, 2, 2, 4, 2>(p, h, l, s); break;   // 256 x 256, 8 waves of 64 x 128, 2 stages
    default: throw InvalidArg{"conv_gemm_dma: unknown variant"};
  }
}

void launch_conv_gemm_dma(const ConvGemmArgs& args, const void* whi, const void* wlo, hipStream_t s) {
  launch_conv_gemm_dma_v(args, whi, wlo, 0, s);
}

}  // namespace wsp
