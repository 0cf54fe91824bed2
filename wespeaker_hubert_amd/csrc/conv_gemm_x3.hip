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
template <bool SWZ>
struct Lds {
  static constexpr int ROWB = SWZ ? 64 : 80;
  static constexpr int SKEW = SWZ ? 0 : 64;  // lo W image offset (padded rows: 16-bank skew)
  __device__ __forceinline__ static int off(int row, int byte) {
    if constexpr (SWZ) return row * 64 + ((((byte >> 4) ^ (row >> 2)) & 3) << 4) + (byte & 15);
    else return row * 80 + byte;
  }
};

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI, int ROLE, bool C2D = false, bool SWZ = false,
          int NSET = 2>
__global__ __launch_bounds__(WM* WN * 64, 2) void conv_gemm_x3(const ConvGemmArgs p,
                                                               const __bf16* __restrict__ whi,
                                                               const __bf16* __restrict__ wlo) {
  using L = Lds<SWZ>;
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
  if constexpr (NSET == 1) {
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

template <int WM, int WN, int TM, int TN, int AMODE, bool UNI, int ROLE, bool C2D, bool SWZ, int NSET>
void launch_x3_k(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  constexpr int ROWB = Lds<SWZ>::ROWB;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const size_t lds = (size_t)2 * (2 * BM * ROWB + 2 * BN * ROWB + Lds<SWZ>::SKEW);
  hipLaunchKernelGGL((conv_gemm_x3<WM, WN, TM, TN, AMODE, UNI, ROLE, C2D, SWZ, NSET>), dim3(nwg), dim3(NT), lds, s,
                     p, whi, wlo);
  WSP_HIP(hipGetLastError());
}

template <int WM, int WN, int TM, int TN, bool SWZ = false, int NSET = 2>
void launch_x3_tile(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  if (p.conv2d) {
    launch_x3_k<WM, WN, TM, TN, kACat, true, 0, true, SWZ, NSET>(p, whi, wlo, s);
    return;
  }
  const bool uni = uniform_ktiles(p);
  if (p.amode == kAAdd) {
    if (uni)
      launch_x3_k<WM, WN, TM, TN, kAAdd, true, 0, false, SWZ, NSET>(p, whi, wlo, s);
    else
      launch_x3_k<WM, WN, TM, TN, kAAdd, false, 0, false, SWZ, NSET>(p, whi, wlo, s);
  } else if (!uni) {
    launch_x3_k<WM, WN, TM, TN, kACat, false, 0, false, SWZ, NSET>(p, whi, wlo, s);
  } else if (p.role == 1) {
    launch_x3_k<WM, WN, TM, TN, kACat, true, 1, false, SWZ, NSET>(p, whi, wlo, s);
  } else {
    launch_x3_k<WM, WN, TM, TN, kACat, true, 0, false, SWZ, NSET>(p, whi, wlo, s);
  }
}

}  // namespace

int conv_gemm_x3_block_rows(const ConvGemmArgs& p, int variant) {
  if (p.N % 64 != 0 || (p.gcols && p.gcols % 64 != 0)) return 128;
  if (p.gcols || p.N % 128 != 0) return 128;
  return (variant == 1 || variant == 4 || variant == 5 || variant == 6) ? 256 : 128;
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
    WSP_CHECK(!p.seg && !p.row_bias && !p.conv2d && p.T >= bm && (variant == 1 || variant == 3 || variant == 4 ||
                                                                  variant == 5 || variant == 6 || variant == 0),
              "conv_gemm_x3: column sums need a uniform batch with T >= block rows and no row bias");
  }
  WSP_CHECK(p.Kp % 64 == 0, "conv_gemm_x3: packed K must be a multiple of 64");
  const __bf16* h = static_cast<const __bf16*>(whi);
  const __bf16* l = static_cast<const __bf16*>(wlo);
  if (p.N % 64 != 0 || (p.gcols && p.gcols % 64 != 0)) {
    launch_x3_tile<4, 1, 1, 1>(p, h, l, s);  // 128 x 32, 4 waves
  } else if (p.gcols) {
    // grouped (HuBERT pos_conv: 16 groups x 64 padded columns, K = 48 x 128): 256-row
    // blocks halve the per-row re-reads of the group's 1.5 MB weight slice
    if (variant == 5) launch_x3_tile<8, 1, 1, 2, true>(p, h, l, s);
    else launch_x3_tile<4, 1, 1, 2>(p, h, l, s);  // blocks stay inside one group
  } else if (p.N % 128 != 0) {
    launch_x3_tile<4, 1, 1, 2>(p, h, l, s);  // 128 x 64, 4 waves
  } else if (variant == 1) {
    launch_x3_tile<4, 2, 2, 2>(p, h, l, s);  // 256 x 128, 8 waves
  } else if (variant == 3) {
    launch_x3_tile<2, 2, 2, 2, true>(p, h, l, s);  // 128 x 128, 4 waves, swizzled rows: 2 blocks / CU
  } else if (variant == 4) {
    launch_x3_tile<4, 2, 2, 2, true>(p, h, l, s);  // 256 x 128, 8 waves, swizzled rows
  } else if (variant == 5) {
    // 256 x 256 (8 waves 4 x 2, 64 x 128 per wave) wherever N allows it: in-model C x C
    // -10 %, conv_cat -15 %, HuBERT fc1 -18 %, fc2 -20 %, CNN -12 % vs 256 x 128 (with the
    // per-tile residual epilogue and the A&S GELU; the libm erff made fc1's epilogue lose)
    if (p.N % 256 == 0 && !p.gcols)
      launch_x3_tile<4, 2, 2, 4, true, 1>(p, h, l, s);
    else
      launch_x3_tile<4, 2, 2, 2, true>(p, h, l, s);  // variant 4
  } else if (variant == 6) {
    // experiments slot (now the same tiles as 5; a 16-wave 64 x 64 form of the wide tile
    // caps registers at 128 and spilled ~300 B per lane in the k-loop)
    if (p.N % 256 == 0 && !p.gcols)
      launch_x3_tile<4, 2, 2, 4, true, 1>(p, h, l, s);
    else
      launch_x3_tile<4, 2, 2, 2, true>(p, h, l, s);
  } else {
    launch_x3_tile<2, 2, 2, 2>(p, h, l, s);  // 128 x 128, 4 waves
  }
}

}  // namespace wsp
