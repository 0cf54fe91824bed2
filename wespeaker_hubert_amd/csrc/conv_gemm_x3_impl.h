// bf16x3 implicit-GEMM conv kernel template (conv_gemm_x3.hip explains the
// scheme) and its tile launchers.  Each tile family is instantiated in its own
// translation unit (conv_gemm_x3_t*.hip) so the families compile in parallel;
// conv_gemm_x3.hip dispatches between them.
#pragma once

#include <type_traits>

#include "gemm_common.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;

// LDS row layout of one 32-wide k-tile row (bf16): padded 80-B rows, or
// unpadded 64-B rows with the 16-B chunk XOR-swizzled by (row >> 2) & 3 —
// both conflict-free for the fragment reads (row = lane & 31, chunk = 2s + h);
// the swizzled form is 20 % smaller (two 128 x 128 blocks fit a CU).
// MF = 16 (v_mfma_f32_16x16x32_bf16 fragments: row = lane & 15, chunk = lane >> 4) swizzles
// by the {0, 2, 3, 1} map of (row >> 2) & 3, which keeps each ds_read_b128 lane group on 16
// distinct 16-B slots of the bank row (tools/mf16_bench.hip).
template <bool SWZ, int MF = 32>
struct Lds {
  static constexpr int ROWB = SWZ ? 64 : 80;
  static constexpr int SKEW = SWZ ? 0 : 64;  // lo W image offset (padded rows: 16-bank skew)
  __device__ __forceinline__ static int off(int row, int byte) {
    static_assert(MF == 32 || SWZ, "16x16 fragments need the swizzled rows");
    if constexpr (SWZ && MF == 16)
      return row * 64 + ((((byte >> 4) ^ (0x1320 >> (4 * ((row >> 2) & 3)))) & 3) << 4) + (byte & 15);
    else if constexpr (SWZ) return row * 64 + ((((byte >> 4) ^ (row >> 2)) & 3) << 4) + (byte & 15);
    else return row * 80 + byte;
  }
};

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI, int ROLE, bool C2D = false, bool SWZ = false,
          int NSET = 2, int MF = 32>
__global__ __launch_bounds__(WM* WN * 64, 2) void conv_gemm_x3(const ConvGemmArgs p,
                                                               const __bf16* __restrict__ whi,
                                                               const __bf16* __restrict__ wlo) {
  using L = Lds<SWZ, MF>;
  static_assert(MF == 32 || NSET == 1, "16x16 MFMA: one-staging-set wide tiles only");
  constexpr int ROWB = L::ROWB;
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int AR = BM * 8 / NT;       // float4 A loads per thread per k-tile
  constexpr int BR = BN * 8 / NT;       // 16-byte W loads per thread per k-tile (hi + lo)
  constexpr int ROWS_A = NT / 8;        // A rows covered per pass
  constexpr int A_BYTES = BM * ROWB;    // one bf16 image (hi or lo) of the A tile
  constexpr int B_BYTES = BN * ROWB;
  constexpr int B_LO = B_BYTES + L::SKEW;
  constexpr int STAGE = 2 * A_BYTES + B_LO + B_BYTES;
  static_assert(AR >= 1 && BR >= 1, "tile too small for the thread count");
  static_assert(BN * 4 % 64 == 0, "a W image must be a whole number of wave loads");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

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

  // ---- A staging geometry
  const int srow = tid >> 3;
  const int c4 = (tid & 7) * 4;
  std::conditional_t<C2D, ALoader2D<AR>, ALoader<AR, AMODE, UNI>> al;
  al.init(p, m0, srow, ROWS_A, c4);
  if (p.gcols) al.a0 += (n0 / p.gcols) * p.gcin;  // grouped conv: this block's input channels
  // ---- W staging geometry: 16-B chunk id q = tid + NT*i over both images
  // (BN*4 chunks each; image = q / (BN*4) is wave-uniform), row = (q % (BN*4)) >> 2
  const __amdgpu_buffer_rsrc_t rwhi = make_rsrc(whi);
  const __amdgpu_buffer_rsrc_t rwlo = make_rsrc(wlo);
  int boff[BR], bls[BR];
  bool bimg[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int q = tid + NT * i;
    const int img = __builtin_amdgcn_readfirstlane(q / (BN * 4));  // wave-uniform (BN*4 % 64 == 0)
    const int qq = q - img * BN * 4;
    const int row = qq >> 2, part = qq & 3;
    bimg[i] = img != 0;
    boff[i] = ((n0 + row) * p.Kp + part * 8) * 2;
    bls[i] = L::off(row, part * 16) + (img ? B_LO : 0);
  }

  // Two register sets: tile k+1 is converted and written to LDS while tile k
  // is multiplied, and tile k+2 is in flight (loads get a whole k-step of
  // MFMA time to land before anyone waits on them).
  f32x4 ra0[AR], ra1[AR];  // (ra1 / rb1 unused with NSET == 1)
  bf16x8 rb0[BR], rb1[BR];

  auto load_tile = [&](f32x4 (&ra)[AR], bf16x8 (&rb)[BR], int k0, bool live) {
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int o = live ? boff[i] + k0 * 2 : kOOB;
      rb[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(bimg[i] ? rwlo : rwhi, o, 0, 0));
    }
    al.load(k0, ra, live);
  };

  auto store_tile = [&](const f32x4 (&ra)[AR], const bf16x8 (&rb)[BR], int buf) {
    unsigned char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = ra[i][e];
        const __bf16 hh = (__bf16)x;
        hi[e] = hh;
        lo[e] = (__bf16)(x - (float)hh);
      }
      const int off = L::off(srow + ROWS_A * i, c4 * 2);
      *reinterpret_cast<bf16x4*>(st + off) = hi;
      *reinterpret_cast<bf16x4*>(st + A_BYTES + off) = lo;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) *reinterpret_cast<bf16x8*>(st + 2 * A_BYTES + bls[i]) = rb[i];
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

  auto mma_step = [&](int buf, int s) {
    const unsigned char* st = smem + buf * STAGE;
    const unsigned char* a_hi = st + L::off(wm * TM * 32 + r32, h * 16 + s * 32);
    const unsigned char* a_lo = a_hi + A_BYTES;
    const unsigned char* b_hi = st + 2 * A_BYTES + L::off(wn * TN * 32 + r32, h * 16 + s * 32);
    const unsigned char* b_lo = b_hi + B_LO;
    bf16x8 ah[TM], al_[TM], bh[TN], bl[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      ah[i] = *reinterpret_cast<const bf16x8*>(a_hi + i * 32 * ROWB);
      al_[i] = *reinterpret_cast<const bf16x8*>(a_lo + i * 32 * ROWB);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(b_hi + j * 32 * ROWB);
      bl[j] = *reinterpret_cast<const bf16x8*>(b_lo + j * 32 * ROWB);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al_[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
  };

  const int nk = p.Kp / BK;
  if constexpr (MF == 16) {
    // 16x16x32: one MFMA spans the whole 32-deep k-tile.  The wave tile is 2 TM x 2 TN blocks
    // of 16 x 16; sub-step s of a k-tile runs the quarters (ih, jh) = (0, 0), (0, 1) (s = 0)
    // and (1, 1), (1, 0) (s = 1) — a snake, so each quarter re-reads only the fragments it does
    // not share with the previous one and 6 TM + 6 TN... fragment registers stay live
    const int r16 = lane & 15, qk = lane >> 4;
    f32x4 acc16[2 * TM][2 * TN];
#pragma unroll
    for (int i = 0; i < 2 * TM; ++i)
#pragma unroll
      for (int j = 0; j < 2 * TN; ++j) acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fah[TM], fal[TM], fbh[TN], fbl[TN];
    auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int o = L::off(wm * TM * 32 + (ih * TM + i) * 16 + r16, qk * 16);
        fah[i] = *reinterpret_cast<const bf16x8*>(st + o);
        fal[i] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + o);
      }
    };
    auto rdB = [&](const unsigned char* st, int jh) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int o = L::off(wn * TN * 32 + (jh * TN + j) * 16 + r16, qk * 16);
        fbh[j] = *reinterpret_cast<const bf16x8*>(st + 2 * A_BYTES + o);
        fbl[j] = *reinterpret_cast<const bf16x8*>(st + 2 * A_BYTES + B_LO + o);
      }
    };
    auto mm = [&](int ih, int jh) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x4& c = acc16[ih * TM + i][jh * TN + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fal[i], fbh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fah[i], fbl[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fah[i], fbh[j], c, 0, 0, 0);
        }
    };
    load_tile(ra0, rb0, 0, true);
    store_tile(ra0, rb0, 0);
    load_tile(ra0, rb0, BK, true);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      const unsigned char* st = smem + buf * STAGE;
      rdA(st, 0);
      rdB(st, 0);
      mm(0, 0);
      rdB(st, 1);
      mm(0, 1);
      store_tile(ra0, rb0, buf ^ 1);  // past-the-end tiles are zeros nobody reads
      load_tile(ra0, rb0, (kt + 2) * BK, kt + 2 < nk);
      rdA(st, 1);
      mm(1, 1);
      rdB(st, 0);
      mm(1, 0);
      __syncthreads();
    }
    gemm_epilogue16<2 * TM, 2 * TN, WM, WN>(p, acc16, m0, n0, wm, wn, lane, smem);
    return;
  } else if constexpr (NSET == 1) {
    // One register set (wide wave tiles: the accumulators leave no room for a
    // second): tile k+1, loaded during step k-1, is written to the free buffer
    // between step k's two sub-steps, and tile k+2 is issued right after it.
    load_tile(ra0, rb0, 0, true);
    store_tile(ra0, rb0, 0);
    load_tile(ra0, rb0, BK, true);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      mma_step(buf, 0);
      store_tile(ra0, rb0, buf ^ 1);  // past-the-end tiles are zeros nobody reads
      load_tile(ra0, rb0, (kt + 2) * BK, kt + 2 < nk);
      mma_step(buf, 1);
      __syncthreads();
    }
    gemm_epilogue<TM, TN, WM, WN>(p, acc, m0, n0, wm, wn, lane, smem);
    return;
  }
  load_tile(ra0, rb0, 0, true);
  load_tile(ra1, rb1, BK, true);
  store_tile(ra0, rb0, 0);
  __syncthreads();

  if constexpr (ROLE == 2) {
    // residual convs (short K, the epilogue's residual read is a large part of a
    // block): the last two k-tiles have no successors to load, so the residual
    // loads go out in their place and land while those k-tiles multiply
    for (int kt = 0; kt < nk - 2; kt += 2) {
      load_tile(ra0, rb0, (kt + 2) * BK, true);
      mma_step(0, 0);
      store_tile(ra1, rb1, 1);
      mma_step(0, 1);
      __syncthreads();
      load_tile(ra1, rb1, (kt + 3) * BK, true);
      mma_step(1, 0);
      store_tile(ra0, rb0, 0);
      mma_step(1, 1);
      __syncthreads();
    }
    float rv[TM][TN][16];
    load_residual_tiles<TM, TN>(p, rv, m0, n0, wm, wn, lane);
    mma_step(0, 0);
    store_tile(ra1, rb1, 1);
    mma_step(0, 1);
    __syncthreads();
    mma_step(1, 0);
    mma_step(1, 1);
    gemm_epilogue_res_pre<TM, TN>(p, acc, m0, n0, wm, wn, lane, rv);
    return;
  }

  // nk is even (Kp % 64 == 0, checked on the host).  Loads and stores are
  // unconditional (past-the-end tiles load zeros into a buffer nobody reads),
  // so the waitcnt pass sees one straight-line stream: the wait before
  // store_tile(R) only covers R's loads, issued one k-step earlier.
  for (int kt = 0; kt < nk; kt += 2) {
    // even step: compute buffer 0 (tile kt); R1 = tile kt+1 -> buffer 1
    load_tile(ra0, rb0, (kt + 2) * BK, kt + 2 < nk);
    mma_step(0, 0);
    store_tile(ra1, rb1, 1);
    mma_step(0, 1);
    __syncthreads();
    // odd step: compute buffer 1 (tile kt+1); R0 = tile kt+2 -> buffer 0
    load_tile(ra1, rb1, (kt + 3) * BK, kt + 3 < nk);
    mma_step(1, 0);
    store_tile(ra0, rb0, 0);
    mma_step(1, 1);
    __syncthreads();
  }

  gemm_epilogue<TM, TN, WM, WN>(p, acc, m0, n0, wm, wn, lane, smem);
}

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI, int ROLE, bool C2D, bool SWZ, int NSET, int MF = 32>
void launch_x3_k(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int ROWB = Lds<SWZ>::ROWB;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const size_t lds = (size_t)2 * (2 * BM * ROWB + 2 * BN * ROWB + Lds<SWZ>::SKEW);
  hipLaunchKernelGGL((conv_gemm_x3<WM, WN, TM, TN, AMODE, UNI, ROLE, C2D, SWZ, NSET, MF>), dim3(nwg), dim3(NT), lds,
                     s, p, whi, wlo);
  WSP_HIP(hipGetLastError());
}

template <int WM, int WN, int TM, int TN, bool SWZ = false, int NSET = 2, int MF = 32>
void launch_x3_tile(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  // the 16x16 form serves 1-D convs with one A operand (ECAPA, HuBERT): its 2-D and added-operand
  // kernels are not instantiated (t_4x2_2x4_mf16 routes those GEMMs to the 32x32 form)
  if constexpr (MF == 32) {
    if (p.conv2d) {
      launch_x3_k<WM, WN, TM, TN, kACat, true, 0, true, SWZ, NSET, MF>(p, whi, wlo, s);
      return;
    }
  }
  const bool uni = uniform_ktiles(p);
  if (MF == 32 && p.amode == kAAdd) {
    if constexpr (MF == 32) {
      if (uni)
        launch_x3_k<WM, WN, TM, TN, kAAdd, true, 0, false, SWZ, NSET, MF>(p, whi, wlo, s);
      else
        launch_x3_k<WM, WN, TM, TN, kAAdd, false, 0, false, SWZ, NSET, MF>(p, whi, wlo, s);
    }
  } else if (!uni) {
    launch_x3_k<WM, WN, TM, TN, kACat, false, 0, false, SWZ, NSET, MF>(p, whi, wlo, s);
  } else if (p.role == 1) {
    launch_x3_k<WM, WN, TM, TN, kACat, true, 1, false, SWZ, NSET, MF>(p, whi, wlo, s);
  } else if constexpr (NSET == 2 && TM * TN <= 4) {
    // residual convs: the residual is loaded ahead of the last two k-tiles (ROLE 2)
    if (p.res && p.role == 2)
      launch_x3_k<WM, WN, TM, TN, kACat, true, 2, false, SWZ, NSET>(p, whi, wlo, s);
    else
      launch_x3_k<WM, WN, TM, TN, kACat, true, 0, false, SWZ, NSET>(p, whi, wlo, s);
  } else {
    launch_x3_k<WM, WN, TM, TN, kACat, true, 0, false, SWZ, NSET, MF>(p, whi, wlo, s);
  }
}

}  // namespace

namespace x3 {
using TileFn = void (*)(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);
void t_4x1_1x1(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);      // 128 x 32
void t_4x1_1x2(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);      // 128 x 64
void t_8x1_1x2_sw(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);   // 256 x 64 swizzled
void t_2x2_2x2_sw(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);   // 128 x 128 swizzled (v3)
void t_4x2_2x2_sw(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);   // 256 x 128 swizzled (v4)
void t_4x2_2x4_sw1(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);  // 256 x 256, one set (v5)
void t_4x2_2x4_mf16(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);  // v5 on 16x16x32 (v6)
bool g256_supported(const ConvGemmArgs&);                                              // v7 operands
void t_g256(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t);         // v6 by LDS-DMA (v7)
}  // namespace x3

}  // namespace wsp
