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
// VALU issues beside the MFMAs.  Same products, same MFMA order, same per-element epilogue
// arithmetic as family 6: bit-identical results.  The epilogue (the 256 KB C tile leaving one
// block per CU with nothing overlapping it, ~15-25 % of a block at K <= 1024) goes through LDS
// and leaves as whole 512-B row pieces in 16-B stores (g_epilogue_rows; the SE column sums
// re-read the staged outputs in family 6's summation order — bit-identical f64 partials — in
// two column passes of 64 (g_epilogue_cs, a kernel instance of its own) so that no sum stays
// live across passes).  C x C conv: bias + ReLU + BN 0.69-0.70 -> 0.64-0.65 ms, + SE column
// sums 0.78-0.80 -> 0.71-0.73 (tools/g7_check); C2 +5.2 %, C4 +3.2-3.6 % against family 6.  A transposed
// accumulator map storing 16 B per lane straight from registers (16 rows x 64 B per store) was
// slower in the model, and a persistent form fetching the next tile's first k-tiles behind the
// epilogue measured no faster (profiles/r4e_gemm_family7_experiments.txt).  r5: a ping-pong k-loop
// (the SIMD partners one barrier apart; READ / MFMA segments; 2- and 4-phase forms, the split in the
// READ segment or in the wave's own MFMA shadows) was bit-identical and never faster — the fp32 A
// split's VALU is the loop's largest overhead wherever it is placed
// (profiles/r5a_gemm_pp_experiments.txt, r5a_gemm_check.txt).
//
// LDS per stage (64 KB; two stages = 128 KB, one block of 8 waves per CU):
//   A [256 rows][32 k] fp32, 16-B chunk c of row r at slot c ^ ((r >> 1) & 5) — the two
//     ds_read_b128 of a 16x16x32 fragment (rows lane & 15, chunks 2 (lane >> 4) + {0, 1}) hit
//     16 distinct 16-B slots in every lane group (found by exhaustive search over r mod 16);
//   W hi, W lo [256 columns][32 k] bf16, family 6's {0, 2, 3, 1} row swizzle.
// A DMA lane writes LDS base + 16 lane (lane-linear), so the swizzle is applied to the SOURCE
// chunk it fetches (cdna_hip_programming.md §5.4 rule 21).
// Supported operands: 1-D convs with one or three concatenated A segments on 32-aligned k-tiles,
// or one segment on k-tiles straddling taps (taps / dilation / padding / stride / ragged batches
// as ALoader), no added operand, no grouped columns, N % 256 == 0, 16-B aligned epilogue operands —
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

// A modes (AM): 1 = dense, 1x1 row-local GEMMs (taps 1, no padding, stride 1: A row = output row,
// also in ragged batches) keep one register per A row; 0 = convs on uniform k-tiles (one tap and
// one concat segment per k-tile) keep ALoader's (row, frame, length) triple; 2 = k-tiles that
// straddle taps (cin % 32 != 0: ECAPA layer1, cin 80) decode tap and channel per lane and 16-B
// chunk (ALoader's non-uniform path; one A segment, zeros past K).
// Epilogue through LDS: each wave parks its raw 64 x 128 accumulators, 32 rows at a time, in a
// private [32][132] fp32 block (padded rows: the 16 column lanes x rows 4q + r of a
// ds_write_b32 hit distinct banks), then walks them back row-major — lane l owns columns
// 4 (l & 31) .. + 3 and rows 2u + (l >> 5) — so every epilogue operand (bias / BN / row bias /
// residual) is one 16-B load and every output leaves in a 16-B store that, with its 31
// neighbours, writes a whole 512-B row piece (4 full 128-B lines per row instead of 64-B pieces
// of 4 rows per dword store).  Same per-element arithmetic and order as gemm_epilogue_store16.
constexpr int kGEpiLd = 132;
constexpr int kGEpiBytes = 8 * 32 * kGEpiLd * 4;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// LayerNorm fold (ConvGemmArgs::lnmode): mean and 1 / sqrt(var + eps) of row `row` from its
// ln_parts (mean, M2) partials of 128 columns, combined in order (Chan et al.'s pairwise update;
// every consumer of the row computes the same values).
// Each lane computes one row (the wave's 64 rows); the epilogue fetches them by lane shuffle.
constexpr int kLnMaxParts = 8;
__device__ __forceinline__ void g_ln_row(const ConvGemmArgs& p, int row, float& mu, float& rstd) {
  const float* s = p.ln_in + (size_t)row * p.ln_parts * 2;
  float m = s[0], m2 = s[1];
#pragma unroll
  for (int k = 1; k < kLnMaxParts; ++k) {
    if (k < p.ln_parts) {  // merge part k (128 values) into the first k parts (128 k values)
      const float d = s[2 * k] - m;
      m += d * (1.f / (float)(k + 1));
      m2 += s[2 * k + 1] + d * d * (128.f * (float)k / (float)(k + 1));
    }
  }
  mu = m;
  rstd = 1.f / sqrtf(m2 / (128.f * (float)p.ln_parts) + p.ln_eps);
}

// (mean, M2) of the 128 values the 32 lanes of a half-wave hold (4 each) for R rows at once ->
// lane 16 of the half (lanes 16 / 48): pairwise merges of equal counts, symmetric in the two
// partners up to the last step (same result on both); the R rows' merge chains interleave
template <int R>
__device__ __forceinline__ void g_ln_pieces(float (&m)[R], float (&m2)[R]) {
  float n = 4.f;
  auto merge = [&](int i, float mo, float m2o) {
    const float d = mo - m[i];
    m[i] = 0.5f * (m[i] + mo);
    m2[i] = (m2[i] + m2o) + d * d * (0.5f * n);
  };
#define WSP_DPP(v, ctrl) __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false))
  // the first four steps inside rows of 16 lanes: quad xor 1, xor 2, then half-row / row mirrors
  // (partners already hold equal values, so a mirror is the xor 4 / 8 exchange); then xor 16
#pragma unroll
  for (int i = 0; i < R; ++i) merge(i, WSP_DPP(m[i], 0xB1), WSP_DPP(m2[i], 0xB1));
  n *= 2.f;
#pragma unroll
  for (int i = 0; i < R; ++i) merge(i, WSP_DPP(m[i], 0x4E), WSP_DPP(m2[i], 0x4E));
  n *= 2.f;
#pragma unroll
  for (int i = 0; i < R; ++i) merge(i, WSP_DPP(m[i], 0x141), WSP_DPP(m2[i], 0x141));
  n *= 2.f;
#pragma unroll
  for (int i = 0; i < R; ++i) merge(i, WSP_DPP(m[i], 0x140), WSP_DPP(m2[i], 0x140));
  n *= 2.f;
#undef WSP_DPP
  // rows 1 / 3 of 16 lanes take row 0's / 2's value (row_bcast:15): lanes 16 and 48 end with the
  // half-wave's statistics (the other rows keep their own)
#define WSP_BC15(v) \
  __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x142, 0xA, 0xF, false))
#pragma unroll
  for (int i = 0; i < R; ++i) merge(i, WSP_BC15(m[i]), WSP_BC15(m2[i]));
#undef WSP_BC15
}

template <int ACT, bool RB, bool RES, int LNM = 0>
__device__ __forceinline__ void g_epilogue_rows(const ConvGemmArgs& p, f32x4 (&acc)[4][8], int m0, int n0, int wm,
                                                int wn, int wave, int lane, unsigned char* smem, float lmu = 0.f,
                                                float lrs = 1.f) {
  float* stg = reinterpret_cast<float*>(smem) + wave * 32 * kGEpiLd;
  const int c16 = lane & 15, q = lane >> 4;
  const int cl = 4 * (lane & 31);  // this lane's 4 columns within the wave's 128
  const int col = n0 + wn * 128 + cl;
  const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 sc = p.scale ? *reinterpret_cast<const f32x4*>(p.scale + col) : f32x4{1.f, 1.f, 1.f, 1.f};
  const f32x4 sh = p.scale ? *reinterpret_cast<const f32x4*>(p.shift + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 lcs{0.f, 0.f, 0.f, 0.f}, lg{1.f, 1.f, 1.f, 1.f}, lb{0.f, 0.f, 0.f, 0.f};
  if constexpr ((LNM & 2) != 0) lcs = *reinterpret_cast<const f32x4*>(p.ln_cs + col);
  if constexpr ((LNM & 4) != 0) {
    lg = *reinterpret_cast<const f32x4*>(p.ln_g + col);
    lb = *reinterpret_cast<const f32x4*>(p.ln_b + col);
  }
  const int lparts = p.N / 128, lpart = (n0 + wn * 128) / 128;  // lmu / lrs: row m0 + wm * 64 + lane
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? p.res : p.out);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    float pm[(LNM & 1) ? 16 : 1], pm2[(LNM & 1) ? 16 : 1];  // LayerNorm pieces of the half's 16 rows
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(i2 * 16 + 4 * q + r) * kGEpiLd + j * 16 + c16] = acc[2 * h + i2][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private block: in-order LDS, no barrier
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int rl = 2 * u + (lane >> 5);
      const int row = m0 + wm * 64 + h * 32 + rl;
      const bool ok = row < p.M;
      const f32x4 x = *reinterpret_cast<const f32x4*>(stg + rl * kGEpiLd + cl);
      f32x4 rv{0.f, 0.f, 0.f, 0.f}, rb{0.f, 0.f, 0.f, 0.f};
      if constexpr (RES) rv = bload4(rres, ok ? (row * p.ldres + col) * 4 : kOOB);
      if constexpr (RB) {
        const int rowc = ok ? row : p.M - 1;
        const int ub = p.seg ? seg_of(p.seg, p.nseg, rowc) : rowc / p.T;
        rb = *reinterpret_cast<const f32x4*>(p.row_bias + (size_t)ub * p.N + col);
      }
      float mu = 0.f, rstd = 1.f;
      if constexpr ((LNM & 6) != 0) {  // row rl of this half: lane h * 32 + rl holds its statistics
        auto rd = [](float v, int l) {
          return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
        };
        mu = lane < 32 ? rd(lmu, h * 32 + 2 * u) : rd(lmu, h * 32 + 2 * u + 1);
        rstd = lane < 32 ? rd(lrs, h * 32 + 2 * u) : rd(lrs, h * 32 + 2 * u + 1);
      }
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v;
        if constexpr ((LNM & 2) != 0) v = (x[e] - mu * lcs[e]) * rstd + bv[e];
        else v = x[e] + bv[e];
        if constexpr ((LNM & 4) != 0) v += (rv[e] - mu) * rstd * lg[e] + lb[e];
        else if constexpr (RES) v += rv[e];
        if constexpr (RB) v += rb[e];
        if constexpr (ACT == kActRelu) v = fmaxf(v, 0.f);
        else if constexpr (ACT == kActTanh) v = tanhf(v);
        else if constexpr (ACT == kActGelu) v = gelu_as(v);
        y[e] = v * sc[e] + sh[e];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), ro, ok ? (row * p.ldo + col) * 4 : kOOB, 0,
                                             0);
      if constexpr ((LNM & 1) != 0) {  // this lane's 4 values of the row: (mean, M2)
        pm[u] = ((y[0] + y[1]) + (y[2] + y[3])) * 0.25f;
        float q2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) q2 += (y[e] - pm[u]) * (y[e] - pm[u]);
        pm2[u] = q2;
      }
    }
    if constexpr ((LNM & 1) != 0) {  // merge the half-wave's 32 lanes per row; lanes 16 / 48 store
      g_ln_pieces<16>(pm, pm2);
      if ((lane & 31) == 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int row = m0 + wm * 64 + h * 32 + 2 * u + (lane >> 5);
          if (row < p.M) *reinterpret_cast<float2*>(p.ln_out + ((size_t)row * lparts + lpart) * 2) = float2{pm[u], pm2[u]};
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next half overwrites
  }
}

// The SE-column-sum epilogue (CSK instances) in two column passes of 64: each wave stages its
// 64 rows x 64 columns ([64][68] fp32), writes them out row-major (16 lanes x 16 B = 256 B per
// row piece) and re-reads the staged outputs for the column sums of those 4 column tiles, so
// no column sum stays live across passes (the one-pass form spilled ~130 registers).  Sums in
// family 6's order: per lane rows 16 i + 4 q + r (i, then r), lanes l ^ 16, l ^ 32, then waves.
constexpr int kGCsLd = 68;
constexpr int kGCsBytes = 8 * 64 * kGCsLd * 4;
template <int ACT>
__device__ __forceinline__ void g_epilogue_cs(const ConvGemmArgs& p, f32x4 (&acc)[4][8], int m0, int n0, int wm,
                                              int wn, int wave, int lane, unsigned char* smem) {
  float* stg = reinterpret_cast<float*>(smem) + wave * 64 * kGCsLd;
  const int c16 = lane & 15, q = lane >> 4;
  const int cl = 4 * c16;  // this lane's 4 columns within the pass's 64
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  // rows of this lane's sums relative to the block: side 0 below nb, side 1 from nb to mb
  const int nb = min((m0 / p.T + 1) * p.T, p.M) - m0, mb = p.M - m0;
  unsigned side0 = 0, side1 = 0;  // bit 4 i + r
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rr = wm * 64 + (k >> 2) * 16 + 4 * q + (k & 3);
    side0 |= (rr < nb ? 1u : 0u) << k;
    side1 |= (rr >= nb && rr < mb ? 1u : 0u) << k;
  }
  double rs[8][2];
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
#pragma unroll
        for (int r = 0; r < 4; ++r) stg[(16 * i + 4 * q + r) * kGCsLd + 16 * jj + c16] = acc[i][4 * pp + jj][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private block: in-order LDS, no barrier
    const int col = n0 + wn * 128 + 64 * pp + cl;
    const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 sc = p.scale ? *reinterpret_cast<const f32x4*>(p.scale + col) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 sh = p.scale ? *reinterpret_cast<const f32x4*>(p.shift + col) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int rl = 4 * u + q;
      const int row = m0 + wm * 64 + rl;
      float* sp = stg + rl * kGCsLd + cl;
      const f32x4 x = *reinterpret_cast<const f32x4*>(sp);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = x[e] + bv[e];
        if constexpr (ACT == kActRelu) v = fmaxf(v, 0.f);
        else if constexpr (ACT == kActTanh) v = tanhf(v);
        else if constexpr (ACT == kActGelu) v = gelu_as(v);
        y[e] = v * sc[e] + sh[e];
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), ro,
                                             row < p.M ? (row * p.ldo + col) * 4 : kOOB, 0, 0);
      *reinterpret_cast<f32x4*>(sp) = y;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      double c0 = 0.0, c1 = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const double yd = (double)stg[((k >> 2) * 16 + 4 * q + (k & 3)) * kGCsLd + 16 * jj + c16];
        c0 += (side0 >> k) & 1 ? yd : 0.0;
        c1 += (side1 >> k) & 1 ? yd : 0.0;
      }
      double v0 = c0 + __shfl_xor(c0, 16);
      v0 += __shfl_xor(v0, 32);
      double v1 = c1 + __shfl_xor(c1, 16);
      v1 += __shfl_xor(v1, 32);
      rs[4 * pp + jj][0] = v0;
      rs[4 * pp + jj][1] = v1;
      __builtin_amdgcn_sched_barrier(0);  // one column tile's 16 reads at a time
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass overwrites
  }
  __syncthreads();  // the reduction buffer overlaps other waves' staging blocks
  constexpr int BN = 256;
  double* red = reinterpret_cast<double*>(smem);  // [4 wm][2][BN], as gemm_colsum_reduce16
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) red[(wm * 2 + u) * BN + (wn * 8 + j) * 16 + lane] = rs[j][u];
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < 2 * BN) {
    const int u = tid / BN, c = tid - u * BN;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + u) * BN + c];
    p.colsum[((size_t)(m0 / 256) * 2 + u) * p.N + n0 + c] = v;
  }
}

// XP: development experiments (tools/gemm_check built with -DWSP_G7_XP; the library instantiates
// XP = 0 only): 1 = timing-only, the A fragments bit-reinterpreted instead of split (no split
// VALU; wrong results); 2 = the next tile's DMA pieces interleaved into the quarters; 3 = timing-
// only, no DMA and no barrier inside the k-loop (every k-tile re-reads the two staged tiles: the
// LDS -> split -> MFMA loop alone); 4 = 3 without the split (LDS -> MFMA alone)
template <int AM, bool CSK, int LNM = 0, int XP = 0>
__global__ __launch_bounds__(512, 1) void conv_gemm_g(const ConvGemmArgs p, const __bf16* __restrict__ whi,
                                                      const __bf16* __restrict__ wlo) {
  using L = Lds<true, 16>;
  // AM 3: AM 1 whose A segment 1 is the projection shortcut's 2-D strided input (ConvGemmArgs::sc2d)
  constexpr bool DENSE = AM == 1 || AM == 3;
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
  int a_r[4], a_t[DENSE ? 1 : 4], a_l[DENSE ? 1 : 4], a_s[AM == 3 ? 4 : 1];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (4 * wave + i) * 8 + (lane >> 3);
    if constexpr (DENSE) {
      a_r[i] = m < p.M ? m : -1;
      if constexpr (AM == 3) {  // shortcut input row of output (b, fo, to)
        const int fto = p.Fo * p.To;
        const int b = m / fto, fo = (m - b * fto) / p.To, to = m - b * fto - fo * p.To;
        a_s[i] = m < p.M ? (b * p.Fi + fo * p.stride) * p.Ti + to * p.stride : -1;
      }
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
  auto dma = [&](int kt, int buf, int part = 3) {  // part bit 0: A pieces, bit 1: W pieces
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
      if (!(part & 1)) break;
      if constexpr (DENSE) {
        const int ar = AM == 3 && ct >= p.cseg[1] ? a_s[i] : a_r[i];
        g_dma(ra, st + (4 * wave + i) * 1024, ar >= 0 ? (ar * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      } else if constexpr (AM == 2) {
        const int k = kt * BK + (i & 1 ? ac1 : ac0);
        const int tap = k / p.cin;
        const int offk = tap * p.dil - p.pad;
        const int tt = a_t[i] + offk;
        const bool ok = k < p.K && tt >= 0 && tt < a_l[i];
        g_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + offk) * ld + k - tap * p.cin) * 4 : kOOB);
      } else {
        const int tt = a_t[i] + off;
        const bool ok = tt >= 0 && tt < a_l[i];
        g_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + off) * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (!(part & 2)) break;
      const int o = woff[i] + kt * 64;
      g_dma(rwh, st + kGA + (2 * wave + i) * 1024, o);
      g_dma(rwl, st + kGA + kGW + (2 * wave + i) * 1024, o);
    }
    if (!(part & 2)) return;  // the tap / channel cursor advances with the W half (issued last)
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
      if constexpr (XP == 1 || XP == 4) {
        ah[i] = __builtin_bit_cast(bf16x8, x0);
        al[i] = __builtin_bit_cast(bf16x8, x1);
        continue;
      }
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

  // LayerNorm fold: this lane's row statistics, loaded ahead of the first DMAs (their latency hides
  // behind tile 0's) and held through the k-loop (2 registers)
  float lmu = 0.f, lrs = 1.f;
  if constexpr ((LNM & 6) != 0) g_ln_row(p, min(m0 + wm * 64 + lane, p.M - 1), lmu, lrs);
  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 landed (8 DMAs per k-tile and lane)
  __builtin_amdgcn_s_barrier();
  // (XP 2 keeps this prologue: tile 1 is in flight, iteration 0 issues nothing, iteration kt >= 1
  // issues tile kt + 1 into the buffer tile kt - 1 left)
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const unsigned char* st = smem + buf * kGStage;
    if constexpr (XP == 2) {
      // the next tile's pieces go out between this tile's quarters (the other buffer is free:
      // every wave passed the barrier that ended tile kt - 1's reads of it)
      rdA(st, 0);
      rdB(st, 0);
      mm(0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (kt >= 1 && kt + 1 < nk) dma(kt + 1, buf ^ 1, 1);
      __builtin_amdgcn_sched_barrier(0);
      rdB(st, 1);
      mm(0, 1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt >= 1 && kt + 1 < nk) dma(kt + 1, buf ^ 1, 2);
      __builtin_amdgcn_sched_barrier(0);
      rdA(st, 1);
      mm(1, 1);
      rdB(st, 0);
      mm(1, 0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
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
    if constexpr (XP >= 3) {  // timing-only: the staged tiles are re-read, nothing is waited for
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      continue;
    }
    // tile kt + 1 (issued a k-tile ago) has landed and every wave is done reading this half
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) dma(kt + 2, buf);
  }
  // no DMA is in flight and every wave is past the last reads: the epilogue may use LDS
#define WSP_GEPI(RB, RES)                                                                                   \
  switch (p.act) {                                                                                         \
    case kActRelu: g_epilogue_rows<kActRelu, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    case kActTanh: g_epilogue_rows<kActTanh, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    case kActGelu: g_epilogue_rows<kActGelu, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    default: g_epilogue_rows<kActNone, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;          \
  }
  if constexpr (LNM != 0) {  // HuBERT LayerNorm fold instances (own kernels: the others keep their code)
    if constexpr ((LNM & 5) != 0)
      g_epilogue_rows<kActNone, false, true, LNM>(p, acc, m0, n0, wm, wn, wave, lane, smem, lmu, lrs);
    else if (p.act == kActGelu)
      g_epilogue_rows<kActGelu, false, false, LNM>(p, acc, m0, n0, wm, wn, wave, lane, smem, lmu, lrs);
    else
      g_epilogue_rows<kActNone, false, false, LNM>(p, acc, m0, n0, wm, wn, wave, lane, smem, lmu, lrs);
  } else if constexpr (CSK) {  // SE column sums: own kernel instance (its epilogue's registers stay out of the others)
    switch (p.act) {
      case kActRelu: g_epilogue_cs<kActRelu>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      case kActTanh: g_epilogue_cs<kActTanh>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      case kActGelu: g_epilogue_cs<kActGelu>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      default: g_epilogue_cs<kActNone>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
    }
  } else if (p.res) {
    WSP_GEPI(false, true)
  } else if (p.row_bias) {
    WSP_GEPI(true, false)
  } else {
    WSP_GEPI(false, false)
  }
#undef WSP_GEPI
}

#ifdef WSP_G7_XP
// ---------------------------------------------------------------------------------------------
// Tile family 10 (r6): family 7's 256 x 256 tile, waves and epilogue, with W's fragments loaded
// by each wave straight from L2 into registers (16 B per lane: the [N][Kp] hi / lo images already
// hold a 16x16x32 B fragment's 8 k of one column contiguously) and only A staged through LDS, in a
// 4-deep ring of 32 KB stages (family 7: A + W in a 2-deep ring of 64 KB).  Per k-tile a wave
// reads 8 A fragments from LDS (family 7: 24 fragment reads), issues 4 A DMA pieces (family 7: 8
// pieces) and 16 B loads, and the barrier that ends k-tile t waits for tile t + 1's A, issued three
// k-tiles earlier (family 7: one).  Quarters run (0,0) (1,0) (1,1) (0,1) so each B half is dead for
// half a k-tile before the next tile's copy of it is loaded into the same registers.  Every VMEM
// op is issued whether or not its tile exists (kOOB offsets past the end: zeros, still counted), so
// the counted vmcnt waits are exact.  Same products, per-accumulator MFMA order and epilogue as
// families 6 / 7: bit-identical — and 1.5-1.7x slower (profiles/r6d_gemm_family10.txt): the four
// waves of a column half each fetch the same W fragments, so a 64-k tile moves 160 KB through the
// CU's vector-memory address path (family 7: 128 KB per two 32-k tiles, each byte once), which at
// ~64 B/clk outlasts the tile's MFMA issue.  Development build only (tools/gemm_check, WSP_G7_XP).
constexpr int kBStages = 4;
template <int AM, bool CSK>
__global__ __launch_bounds__(512, 1) void conv_gemm_gb(const ConvGemmArgs p, const __bf16* __restrict__ whi,
                                                       const __bf16* __restrict__ wlo) {
  constexpr bool DENSE = AM == 1;
  static_assert(AM == 0 || AM == 1, "family 10: uniform k-tiles only");
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

  // ---- A rows of this lane (family 7's mapping)
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
      a_t[i] = (m < p.M) ? t : -0x40000000;
      a_l[i] = p.Ti;
    }
  }
  const int nk = p.Kp / BK;
  int jt = 0, ct = 0;  // tap and channel of the next A k-tile to fetch (fetched in order)
  auto dma_a = [&](int kt) {  // kt >= nk: the same pieces at kOOB (zeros into a stage nobody reads)
    unsigned char* st = smem + (kt & (kBStages - 1)) * kGA;
    const bool live = kt < nk;
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
        g_dma(ra, st + (4 * wave + i) * 1024,
              live && a_r[i] >= 0 ? (a_r[i] * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      } else {
        const int tt = a_t[i] + off;
        const bool ok = live && tt >= 0 && tt < a_l[i];
        g_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + off) * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      }
    }
    ct += 32;
    if (ct >= p.cin) {
      ct -= p.cin;
      ++jt;
    }
  };

  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 x 128
  const int r16 = lane & 15, qk = lane >> 4;
  // B fragment (jh, j) of k-tile kt: column n0 + wn 128 + (4 jh + j) 16 + r16, k 32 kt + 8 qk .. + 7
  const __amdgpu_buffer_rsrc_t rwh = make_rsrc(whi);
  const __amdgpu_buffer_rsrc_t rwl = make_rsrc(wlo);
  const int bcol0 = ((n0 + wn * 128 + r16) * p.Kp + 8 * qk) * 2;
  const int bjstep = 16 * p.Kp * 2;
  bf16x8 bh[2][4], bl[2][4];
  auto load_b = [&](int kt, int jh) {
    const bool live = kt < nk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = live ? bcol0 + (4 * jh + j) * bjstep + kt * 64 : kOOB;
      bh[jh][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rwh, o, 0, 0));
      bl[jh][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rwl, o, 0, 0));
    }
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[2][2], al[2][2];
  auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 64 + (ih * 2 + i) * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + g_aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + g_aslot(r, 2 * qk + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[ih][i][e] = h0;
        ah[ih][i][4 + e] = h1;
        al[ih][i][e] = (__bf16)(x0[e] - (float)h0);
        al[ih][i][4 + e] = (__bf16)(x1[e] - (float)h1);
      }
    }
  };
  auto mm = [&](int ih, int jh) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[ih * 2 + i][jh * 4 + j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[ih][i], bh[jh][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ih][i], bl[jh][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[ih][i], bh[jh][j], c, 0, 0, 0);
      }
  };

  // prologue: A tiles 0..3 and both B halves of tile 0, all waited for
  dma_a(0);
  dma_a(1);
  dma_a(2);
  dma_a(3);
  load_b(0, 0);
  load_b(0, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // Per k-tile t, VMEM issue order: B half 0 of t + 1 (8), B half 1 of t + 1 (8), and after the
  // barrier A of t + 4 (4).  Waits: B half 0 of t has B half 1 of t and A of t + 3 behind it (12);
  // B half 1 of t has A of t + 3 and B half 0 of t + 1 behind it (12); A of t + 1 (issued after
  // the barrier of t - 3) has 3 x 16 B loads and 2 x 4 A pieces behind it at the barrier of t (56).
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = smem + (kt & (kBStages - 1)) * kGA;
    // (the B registers' loads are register dependencies: hipcc places their vmcnt waits itself;
    // only the LDS-DMA data below needs a counted wait)
    rdA(st, 0);
    mm(0, 0);
    rdA(st, 1);  // its reads and split interleave with quarter (0,0)'s MFMAs
    mm(1, 0);
    __builtin_amdgcn_sched_barrier(0);
    load_b(kt + 1, 0);
    __builtin_amdgcn_sched_barrier(0);
    mm(1, 1);
    mm(0, 1);
    __builtin_amdgcn_sched_barrier(0);
    load_b(kt + 1, 1);
    // A of kt + 1 has landed and every wave is done reading this stage
    asm volatile("s_waitcnt vmcnt(56) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma_a(kt + 4);
  }
  // every DMA (including the zero pieces past the end) has landed and every wave is past its
  // last LDS read before the epilogue reuses LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
#define WSP_GBEPI(RB, RES)                                                                                  \
  switch (p.act) {                                                                                         \
    case kActRelu: g_epilogue_rows<kActRelu, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    case kActTanh: g_epilogue_rows<kActTanh, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    case kActGelu: g_epilogue_rows<kActGelu, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;    \
    default: g_epilogue_rows<kActNone, RB, RES>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;          \
  }
  if constexpr (CSK) {
    switch (p.act) {
      case kActRelu: g_epilogue_cs<kActRelu>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      case kActTanh: g_epilogue_cs<kActTanh>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      case kActGelu: g_epilogue_cs<kActGelu>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
      default: g_epilogue_cs<kActNone>(p, acc, m0, n0, wm, wn, wave, lane, smem); break;
    }
  } else if (p.res) {
    WSP_GBEPI(false, true)
  } else if (p.row_bias) {
    WSP_GBEPI(true, false)
  } else {
    WSP_GBEPI(false, false)
  }
#undef WSP_GBEPI
}
#endif  // WSP_G7_XP

}  // namespace

namespace x3 {

bool g256_supported(const ConvGemmArgs& p) {
  auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool aligned = a16(p.out) && p.ldo % 4 == 0 && a16(p.bias) && a16(p.scale) && a16(p.shift) &&
                       a16(p.row_bias) && a16(p.res) && (!p.res || p.ldres % 4 == 0);
  // non-uniform k-tiles (AM 2): one A segment only, as ALoader's per-lane path
  return aligned && p.N % 256 == 0 && !p.conv2d && !p.gcols && p.amode == kACat &&
         (uniform_ktiles(p) || (p.cseg[1] >= p.cin && !p.colsum)) &&
         (!p.sc2d || (uniform_ktiles(p) && !p.colsum && !p.lnmode && !p.row_bias));
}

void t_g256(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  constexpr int lds0 = 2 * kGStage > kGEpiBytes ? 2 * kGStage : kGEpiBytes;
  constexpr int lds = lds0 > kGCsBytes ? lds0 : kGCsBytes;
  // AM 1 reads A row m for output row m: only when ALoader's row map is the identity (no separate
  // input offsets, and uniform batches with Ti == T); ragged iseg / Ti != T 1x1 GEMMs take AM 0.
  const bool dense = p.taps == 1 && p.pad == 0 && p.stride == 1 && !p.iseg && (p.seg || p.Ti == p.T);
  const int am = !uniform_ktiles(p) ? 2 : dense ? 1 : 0;
  if (p.sc2d) {  // conv3 + projection shortcut (check_conv_args / g256_supported: dense, uniform k-tiles)
    hipLaunchKernelGGL((conv_gemm_g<3, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
    WSP_HIP(hipGetLastError());
    return;
  }
  if (p.lnmode) {
    // LayerNorm fold: 1 = emit (out_proj / fc2 on the residual), 2 = fold (qkv / fc1), 4 = residual
    // normalised on the fly, 5 = both (fc2 / out_proj under the full fold)
    WSP_CHECK(am == 1 && !p.colsum && !p.row_bias && !p.scale && p.N % 128 == 0 &&
                  ((p.lnmode & 1) == 0 || (p.ln_out && p.res && p.act == kActNone)) &&
                  ((p.lnmode & 6) == 0 || (p.ln_in && p.ln_parts >= 1 && p.ln_parts <= kLnMaxParts)) && ((p.lnmode & 2) == 0 || (p.ln_cs && !p.res)) &&
                  ((p.lnmode & 4) == 0 || (p.ln_g && p.ln_b && p.res && p.act == kActNone)),
              "conv_gemm_x3: LayerNorm fold needs a dense 1x1 GEMM and its operands");
    switch (p.lnmode) {
      case 1: hipLaunchKernelGGL((conv_gemm_g<1, false, 1>), dim3(nwg), dim3(512), lds, s, p, h, l); break;
      case 2: hipLaunchKernelGGL((conv_gemm_g<1, false, 2>), dim3(nwg), dim3(512), lds, s, p, h, l); break;
      case 4: hipLaunchKernelGGL((conv_gemm_g<1, false, 4>), dim3(nwg), dim3(512), lds, s, p, h, l); break;
      case 5: hipLaunchKernelGGL((conv_gemm_g<1, false, 5>), dim3(nwg), dim3(512), lds, s, p, h, l); break;
      default: WSP_CHECK(false, "conv_gemm_x3: lnmode must be 1, 2, 4 or 5");
    }
    WSP_HIP(hipGetLastError());
    return;
  }
  if (p.colsum && am == 1)
    hipLaunchKernelGGL((conv_gemm_g<1, true>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else if (p.colsum && am == 0)
    hipLaunchKernelGGL((conv_gemm_g<0, true>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else if (am == 1)
    hipLaunchKernelGGL((conv_gemm_g<1, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else if (am == 0)
    hipLaunchKernelGGL((conv_gemm_g<0, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else
    hipLaunchKernelGGL((conv_gemm_g<2, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
  WSP_HIP(hipGetLastError());
}

#ifdef WSP_G7_XP
// family 10 (development build): the operands family 7 takes on uniform k-tiles (no LayerNorm fold)
bool gb256_supported(const ConvGemmArgs& p) {
  return g256_supported(p) && uniform_ktiles(p) && !p.lnmode && p.Kp % BK == 0;
}

void t_gb256(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  WSP_CHECK(gb256_supported(p), "conv_gemm_x3 family 10: unsupported operands");
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  constexpr int lds0 = kBStages * kGA > kGEpiBytes ? kBStages * kGA : kGEpiBytes;
  constexpr int lds = lds0 > kGCsBytes ? lds0 : kGCsBytes;
  const bool dense = p.taps == 1 && p.pad == 0 && p.stride == 1 && !p.iseg && (p.seg || p.Ti == p.T);
  if (p.colsum && dense)
    hipLaunchKernelGGL((conv_gemm_gb<1, true>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else if (p.colsum)
    hipLaunchKernelGGL((conv_gemm_gb<0, true>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else if (dense)
    hipLaunchKernelGGL((conv_gemm_gb<1, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else
    hipLaunchKernelGGL((conv_gemm_gb<0, false>), dim3(nwg), dim3(512), lds, s, p, h, l);
  WSP_HIP(hipGetLastError());
}

// development entry (tools/gemm_check): plain family 7 operand forms (no LayerNorm fold)
void t_g256_xp(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s, int xp) {
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  constexpr int lds0 = 2 * kGStage > kGEpiBytes ? 2 * kGStage : kGEpiBytes;
  constexpr int lds = lds0 > kGCsBytes ? lds0 : kGCsBytes;
  const bool dense = p.taps == 1 && p.pad == 0 && p.stride == 1 && !p.iseg && (p.seg || p.Ti == p.T);
  const int am = !uniform_ktiles(p) ? 2 : dense ? 1 : 0;
  WSP_CHECK(am != 2 && !p.lnmode, "t_g256_xp: AM 0 / 1 only");
#define WSP_XPL(AMv, CS, XPv) hipLaunchKernelGGL((conv_gemm_g<AMv, CS, 0, XPv>), dim3(nwg), dim3(512), lds, s, p, h, l)
  if (xp == 1) {
    if (p.colsum) { if (am == 1) WSP_XPL(1, true, 1); else WSP_XPL(0, true, 1); }
    else { if (am == 1) WSP_XPL(1, false, 1); else WSP_XPL(0, false, 1); }
  } else if (xp == 3) {
    WSP_CHECK(am == 1 && !p.colsum, "t_g256_xp 3: dense, no column sums");
    WSP_XPL(1, false, 3);
  } else if (xp == 4) {
    WSP_CHECK(am == 1 && !p.colsum, "t_g256_xp 4: dense, no column sums");
    WSP_XPL(1, false, 4);
  } else {
    if (p.colsum) { if (am == 1) WSP_XPL(1, true, 2); else WSP_XPL(0, true, 2); }
    else { if (am == 1) WSP_XPL(1, false, 2); else WSP_XPL(0, false, 2); }
  }
#undef WSP_XPL
  WSP_HIP(hipGetLastError());
}
#endif

}  // namespace x3
}  // namespace wsp
