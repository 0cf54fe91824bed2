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
// of 32x32 (v_mfma_f32_32x32x16_bf16).  A (fp32 activations) is split into
// hi/lo bf16 while staging; W is pre-split on the host.  LDS rows are
// 32 bf16 + 8 pad (80 B): the 16-byte fragment reads (row = lane&31,
// k = 16 s + 8 (lane>>5)) hit 16 distinct slots per ds_read_b128 group.
#include "kernels.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
constexpr int ROWB = 80;  // bytes per LDS row (32 bf16 + 8 pad)

template <int WM, int WN, int TM, int TN, int AMODE>
__global__ __launch_bounds__(WM* WN * 64, 2) void conv_gemm_x3(const ConvGemmArgs p,
                                                               const __bf16* __restrict__ whi,
                                                               const __bf16* __restrict__ wlo) {
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int AR = BM * 8 / NT;       // float4 A loads per thread per k-tile
  constexpr int BR = BN * 8 / NT;       // 16-byte W loads per thread per k-tile
  constexpr int ROWS_A = NT / 8;        // A rows covered per pass
  constexpr int A_BYTES = BM * ROWB;    // one bf16 image (hi or lo) of the A tile
  constexpr int B_BYTES = BN * ROWB;
  constexpr int STAGE = 2 * A_BYTES + 2 * B_BYTES;
  static_assert(AR >= 1 && BR >= 1, "tile too small for the thread count");

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
  int a_m[AR], a_t[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + srow + ROWS_A * i;
    a_m[i] = m;
    a_t[i] = (m < p.M) ? (m % p.T) : -0x40000000;
  }
  // ---- W staging geometry: chunk = (row, part); parts 0-3 hi, 4-7 lo
  const int bpart = tid & 7;
  const __bf16* bsrc[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int row = (tid + NT * i) >> 3;
    bsrc[i] = ((bpart < 4) ? whi : wlo) + (size_t)(n0 + row) * p.Kp + (bpart & 3) * 8;
  }

  f32x4 ra[AR];
  bf16x8 rb[BR];

  auto load_tile = [&](int k0) {
    const int k = k0 + c4;
    int j = 0, c = 0;
    const bool kin = k < p.K;
    if (kin) {
      j = k / p.cin;
      c = k - j * p.cin;
    }
    const int off = j * p.dil - p.pad;
    int seg = 0, cl = c;
    if (AMODE == kACat) {
      seg = (c >= p.cseg[1]) + (c >= p.cseg[2]);
      cl = c - p.cseg[seg];
    }
    const float* base = (seg == 0) ? p.a[0] : ((seg == 1) ? p.a[1] : p.a[2]);
    const int ld = (seg == 0) ? p.lda[0] : ((seg == 1) ? p.lda[1] : p.lda[2]);
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int tt = a_t[i] + off;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (kin && tt >= 0 && tt < p.T) {
        const long row = (long)a_m[i] + off;
        if (AMODE == kACat) {
          v = *reinterpret_cast<const f32x4*>(base + row * ld + cl);
        } else {
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(p.a[0] + row * p.lda[0] + c);
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(p.a[1] + row * p.lda[1] + c);
          v = x0 + x1;
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = *reinterpret_cast<const bf16x8*>(bsrc[i] + k0);
  };

  auto store_tile = [&](int buf) {
    unsigned char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = ra[i][e];
        const __bf16 h = (__bf16)x;
        hi[e] = h;
        lo[e] = (__bf16)(x - (float)h);
      }
      const int off = (srow + ROWS_A * i) * ROWB + c4 * 2;
      *reinterpret_cast<bf16x4*>(st + off) = hi;
      *reinterpret_cast<bf16x4*>(st + A_BYTES + off) = lo;
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = (tid + NT * i) >> 3;
      const int off = 2 * A_BYTES + ((bpart < 4) ? 0 : B_BYTES) + row * ROWB + (bpart & 3) * 16;
      *reinterpret_cast<bf16x8*>(st + off) = rb[i];
    }
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
    const unsigned char* st = smem + cur * STAGE;
    const unsigned char* a_hi = st + (wm * TM * 32 + r32) * ROWB + h * 16;
    const unsigned char* a_lo = a_hi + A_BYTES;
    const unsigned char* b_hi = st + 2 * A_BYTES + (wn * TN * 32 + r32) * ROWB + h * 16;
    const unsigned char* b_lo = b_hi + B_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        ah[i] = *reinterpret_cast<const bf16x8*>(a_hi + i * 32 * ROWB + s * 32);
        al[i] = *reinterpret_cast<const bf16x8*>(a_lo + i * 32 * ROWB + s * 32);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(b_hi + j * 32 * ROWB + s * 32);
        bl[j] = *reinterpret_cast<const bf16x8*>(b_lo + j * 32 * ROWB + s * 32);
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
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue (gfx950 32x32 C/D map: col = lane&31, row = (r&3)+8(r>>2)+4h)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + (wn * TN + j) * 32 + r32;
    const float bv = p.bias ? p.bias[col] : 0.f;
    const float sc = p.scale ? p.scale[col] : 1.f;
    const float sh = p.scale ? p.shift[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rbase = m0 + (wm * TM + i) * 32 + 4 * h;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < p.M) {
          float y = acc[i][j][r] + bv;
          if (p.row_bias) y += p.row_bias[(size_t)(row / p.T) * p.N + col];
          if (p.res) y += p.res[(size_t)row * p.ldres + col];
          if (p.act == kActRelu) y = fmaxf(y, 0.f);
          else if (p.act == kActTanh) y = tanhf(y);
          if (p.scale) y = y * sc + sh;
          p.out[(size_t)row * p.ldo + col] = y;
        }
      }
    }
  }
}

template <int WM, int WN, int TM, int TN>
void launch_x3_tile(const ConvGemmArgs& p, const __bf16* whi, const __bf16* wlo, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = WM * WN * 64;
  const int nwg = ((p.M + BM - 1) / BM) * (p.N / BN);
  const size_t lds = (size_t)2 * (2 * BM * ROWB + 2 * BN * ROWB);
  if (p.amode == kAAdd)
    hipLaunchKernelGGL((conv_gemm_x3<WM, WN, TM, TN, kAAdd>), dim3(nwg), dim3(NT), lds, s, p, whi, wlo);
  else
    hipLaunchKernelGGL((conv_gemm_x3<WM, WN, TM, TN, kACat>), dim3(nwg), dim3(NT), lds, s, p, whi, wlo);
  WSP_HIP(hipGetLastError());
}

}  // namespace

void launch_conv_gemm_x3(const ConvGemmArgs& p, const void* whi, const void* wlo, int variant,
                         hipStream_t s) {
  WSP_CHECK(p.M > 0 && p.N > 0 && p.K > 0 && p.T > 0, "conv_gemm_x3: empty shape");
  WSP_CHECK(p.cin % 4 == 0, "conv_gemm_x3: cin must be a multiple of 4");
  WSP_CHECK(p.Kp % BK == 0 && p.Kp >= p.K, "conv_gemm_x3: bad packed K");
  WSP_CHECK(p.N % 64 == 0, "conv_gemm_x3: N must be a multiple of 64");
  for (int i = 0; i < 3; ++i) WSP_CHECK(p.lda[i] % 4 == 0, "conv_gemm_x3: lda must be a multiple of 4");
  if (p.amode == kACat) {
    WSP_CHECK(p.cseg[0] == 0 && p.cseg[3] == p.cin, "conv_gemm_x3: bad channel segments");
    for (int i = 1; i < 3; ++i) WSP_CHECK(p.cseg[i] % 4 == 0, "conv_gemm_x3: segment not float4 aligned");
  }
  const __bf16* h = static_cast<const __bf16*>(whi);
  const __bf16* l = static_cast<const __bf16*>(wlo);
  if (p.N % 128 != 0) {
    launch_x3_tile<4, 1, 1, 2>(p, h, l, s);  // 128 x 64, 4 waves
  } else if (variant == 1) {
    launch_x3_tile<4, 2, 2, 2>(p, h, l, s);  // 256 x 128, 8 waves
  } else {
    launch_x3_tile<2, 2, 2, 2>(p, h, l, s);  // 128 x 128, 4 waves
  }
}

}  // namespace wsp
