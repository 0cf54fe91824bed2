// conv_gemm_x3 tile family 7: the 256 x 256 bf16x3 tile on 16x16x32 MFMAs with EVERY operand
// staged by LDS-DMA (buffer_load ... lds, 16 B per lane) and the fp32 A split into bf16 hi / lo
// when its fragments are read (r4; x3_variant 7).
//
// Family 6 (conv_gemm_x3<..., MF = 16>) stages A through one register set: fp32 loads, the
// hi / lo split and ds_write passes sit between the MFMA sub-steps of every k-tile, and its
// 128 accumulators leave no room for a second set (the staging costs ~20 % of
// the loop).  Here nothing passes through registers on the way to LDS: per k-tile and lane,
// four 16-B DMAs of A rows (fp32, 128-B LDS rows) and four of W (bf16 hi / lo images, 64-B
// rows) land in the free half of a two-stage ring while the other half multiplies; a k-tile
// ends with one vmcnt(0) + barrier and the next DMAs are issued right behind it.  The split
// moves to the fragment reads (8 floats -> bf16x8 hi + lo per 16x16x32 A fragment), where its
// VALU issues beside the MFMAs.  Same products, same MFMA order, same epilogue as family 6:
// bit-identical results.  The k-loop alone (timing build without epilogue) runs 0.56-0.58 ms on
// the C x C shape against 0.64-0.66 with plain stores and 0.69-0.72 for family 6 with the bias +
// ReLU epilogue (tools/g7_check.hip); in the model (C2, r4) conv_cat 2.72-2.78 -> 2.69-2.70 ms,
// C2 +0.9 %.  The epilogue (the 0.5 GB C write at one block per CU, nothing overlapping it) is
// ~15-25 % of a block at K <= 1024; a persistent form fetching the next tile's first k-tiles
// behind it measured no faster (profiles/r4e_gemm_family7_experiments.txt).
//
// LDS per stage (64 KB; two stages = 128 KB, one block of 8 waves per CU):
//   A [256 rows][32 k] fp32, 16-B chunk c of row r at slot c ^ ((r >> 1) & 5) — the two
//     ds_read_b128 of a 16x16x32 fragment (rows lane & 15, chunks 2 (lane >> 4) + {0, 1}) hit
//     16 distinct 16-B slots in every lane group (found by exhaustive search over r mod 16);
//   W hi, W lo [256 columns][32 k] bf16, family 6's {0, 2, 3, 1} row swizzle.
// A DMA lane writes LDS base + 16 lane (lane-linear), so the swizzle is applied to the SOURCE
// chunk it fetches (cdna_hip_programming.md §5.4 rule 21).
// Supported operands: 1-D convs with one or three concatenated A segments on 32-aligned k-tiles
// (taps / dilation / padding / stride / ragged batches as ALoader), no added operand, no
// grouped columns, N % 256 == 0, and an epilogue without SE column sums or residual —
// launch_conv_gemm_x3 routes everything else to family 6.
#include "conv_gemm_x3_impl.h"

namespace wsp {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
constexpr int kGA = 256 * 128, kGW = 256 * 64, kGStage = kGA + 2 * kGW;

__device__ __forceinline__ int g_aslot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 5)) << 4); }

__device__ __forceinline__ void g_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// DENSE: 1x1 row-local GEMMs (taps 1, no padding, stride 1: A row = output row, also in ragged
// batches) keep one register per A row; the conv form keeps ALoader's (row, frame, length) triple.
template <bool DENSE>
__global__ __launch_bounds__(512, 1) void conv_gemm_g(const ConvGemmArgs p, const __bf16* __restrict__ whi,
                                                      const __bf16* __restrict__ wlo) {
  using L = Lds<true, 16>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int ntiles = p.N / 256;
  const int mtiles = (p.M + 255) / 256;
  const int wg = xcd_remap(blockIdx.x, ntiles * mtiles);
  const int mt = wg / ntiles;
  const int nt = wg - mt * ntiles;
  const int m0 = mt * 256;
  const int n0 = nt * 256;

  // ---- A rows of this lane: DMA i (0..3) of wave w fills LDS rows (4 w + i) * 8 .. + 7, lane
  // l row + (l >> 3), slot l & 7 <- source chunk (l & 7) ^ swizzle(row) (ALoader's row logic)
  // row = 32 w + 8 i + (l >> 3): swizzle(row) = (row >> 1) & 5 = ((l >> 4) & 1) | ((i & 1) << 2)
  const int ac0 = 4 * ((lane & 7) ^ ((lane >> 4) & 1)), ac1 = ac0 ^ 16;
  int a_r[4], a_t[DENSE ? 1 : 4], a_l[DENSE ? 1 : 4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (4 * wave + i) * 8 + (lane >> 3);
    if constexpr (DENSE) {
      a_r[i] = m < p.M ? m : -1;
    } else if (p.seg) {
      const int mm = m < p.M ? m : p.M - 1;
      const int b = seg_of(p.seg, p.nseg, mm);
      const int t = (mm - p.seg[b]) * p.stride;
      const int* is = p.iseg ? p.iseg : p.seg;
      a_r[i] = is[b] + t;
      a_t[i] = (m < p.M) ? t : -0x40000000;
      a_l[i] = is[b + 1] - is[b];
    } else {
      const int b = m / p.T;
      const int t = (m - b * p.T) * p.stride;
      a_r[i] = b * p.Ti + t;
      a_t[i] = (m < p.M) ? t : -0x40000000;  // rows >= M fail the t-range test
      a_l[i] = p.Ti;
    }
  }
  // ---- W: DMA i (0..1) of wave w fills columns (2 w + i) * 16 .. + 15 of the hi and lo images
  int woff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * wave + i) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);
    woff[i] = ((n0 + row) * p.Kp + 8 * c) * 2;
  }
  const __amdgpu_buffer_rsrc_t rwh = make_rsrc(whi);
  const __amdgpu_buffer_rsrc_t rwl = make_rsrc(wlo);
  const int nk = p.Kp / BK;  // >= 2 (Kp % 64 == 0)
  int jt = 0, ct = 0;  // tap and channel of the next k-tile to fetch (k-tiles are fetched in order)
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * kGStage;
    const int off = jt * p.dil - p.pad;
    const float* base = p.a[0];
    int ld = p.lda[0], cl = ct;
    if (ct >= p.cseg[2]) {
      base = p.a[2];
      ld = p.lda[2];
      cl = ct - p.cseg[2];
    } else if (ct >= p.cseg[1]) {
      base = p.a[1];
      ld = p.lda[1];
      cl = ct - p.cseg[1];
    }
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (DENSE) {
        g_dma(ra, st + (4 * wave + i) * 1024, a_r[i] >= 0 ? (a_r[i] * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      } else {
        const int tt = a_t[i] + off;
        const bool ok = tt >= 0 && tt < a_l[i];
        g_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + off) * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = woff[i] + kt * 64;
      g_dma(rwh, st + kGA + (2 * wave + i) * 1024, o);
      g_dma(rwl, st + kGA + kGW + (2 * wave + i) * 1024, o);
    }
    ct += 32;
    if (ct >= p.cin) {
      ct -= p.cin;
      ++jt;
    }
  };

  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 x 128
  const int r16 = lane & 15, qk = lane >> 4;
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[2], al[2], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st, int ih) {  // fp32 rows -> bf16 hi / lo fragments
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 64 + (ih * 2 + i) * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + g_aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + g_aslot(r, 2 * qk + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[i][e] = h0;
        ah[i][4 + e] = h1;
        al[i][e] = (__bf16)(x0[e] - (float)h0);
        al[i][4 + e] = (__bf16)(x1[e] - (float)h1);
      }
    }
  };
  auto rdB = [&](const unsigned char* st, int jh) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = L::off(wn * 128 + (jh * 4 + j) * 16 + r16, qk * 16);
      bh[j] = *reinterpret_cast<const bf16x8*>(st + kGA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + kGA + kGW + o);
    }
  };
  auto mm = [&](int ih, int jh) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[ih * 2 + i][jh * 4 + j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
      }
  };

  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed (8 DMAs per k-tile and lane)
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const unsigned char* st = smem + buf * kGStage;
    // family 6's snake over the four 2 x 4 quarters of the 64 x 128 wave tile
    rdA(st, 0);
    rdB(st, 0);
    mm(0, 0);
    rdB(st, 1);
    mm(0, 1);
    rdA(st, 1);
    mm(1, 1);
    rdB(st, 0);
    mm(1, 0);
    // tile kt + 1 (issued a k-tile ago) has landed and every wave is done reading this half
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) dma(kt + 2, buf);
  }
  // no DMA is in flight and every wave is past the last reads: the epilogue may use LDS
  gemm_epilogue16<4, 8, 4, 2>(p, acc, m0, n0, wm, wn, lane, smem);
}

}  // namespace

namespace x3 {

bool g256_supported(const ConvGemmArgs& p) {
  // SE column-sum and residual epilogues measured no faster here than on family 6 (r4, in model:
  // the epilogue, ~15-25 % of a 256 x 256 block at K <= 1024, is the same code) and stay there
  return !p.colsum && !p.res && p.N % 256 == 0 && !p.conv2d && !p.gcols && p.amode == kACat && uniform_ktiles(p);
}

void t_g256(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  if (p.taps == 1 && p.pad == 0 && p.stride == 1)
    hipLaunchKernelGGL(conv_gemm_g<true>, dim3(nwg), dim3(512), 2 * kGStage, s, p, h, l);
  else
    hipLaunchKernelGGL(conv_gemm_g<false>, dim3(nwg), dim3(512), 2 * kGStage, s, p, h, l);
  WSP_HIP(hipGetLastError());
}

}  // namespace x3
}  // namespace wsp
