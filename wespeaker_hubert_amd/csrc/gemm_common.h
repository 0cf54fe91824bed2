// Shared A-operand staging for the implicit-GEMM conv kernels.
//
// A(row, k) with k = tap*cin + c reads channels-last activations at frame
// t + tap*dil - pad of the same utterance (zero outside [0, T)).  When every
// 32-wide k-tile lies inside one tap and one concat segment (cin and the
// segment boundaries multiples of 32 — every layer except ECAPA layer1), the
// tap / segment / base pointer are wave-uniform scalars advanced
// incrementally per k-tile; otherwise (layer1: cin = 80) each lane decodes its
// own k (single segment only).
#pragma once

#include <algorithm>

#include "kernels.h"

namespace wsp {

// Buffer (SRSRC) loads: 32-bit byte offsets, and an out-of-range offset
// returns zeros — the conv's zero padding without exec-mask branches.
constexpr int kOOB = 0x7FFFFFF0;

// The base must be wave-uniform; readfirstlane makes that provable so hipcc
// keeps the descriptor in SGPRs (no waterfall loop, cdna guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, kOOB, 0x00020000);
}

__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

template <int AR, int AMODE, bool UNI>
struct ALoader {
  const float* a0;
  const float* a1;
  const float* a2;
  int ld0, ld1, ld2, cs1, cs2;
  int cin, dil, pad, Ti, K;
  int c4;
  int a_r[AR], a_t[AR], a_l[AR];  // input row / frame of tap 0 (before dil/pad), utterance frames
  int j, c;  // UNI: tap and channel of the current k-tile start

  __device__ __forceinline__ void init(const ConvGemmArgs& p, int m0, int srow, int rows_step,
                                       int c4_) {
    a0 = p.a[0];
    a1 = p.a[1];
    a2 = p.a[2];
    ld0 = p.lda[0];
    ld1 = p.lda[1];
    ld2 = p.lda[2];
    cs1 = p.cseg[1];
    cs2 = p.cseg[2];
    cin = p.cin;
    dil = p.dil;
    pad = p.pad;
    Ti = p.Ti;
    K = p.K;
    c4 = c4_;
    j = 0;
    c = 0;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + srow + rows_step * i;
      if (p.seg) {  // segmented batch: output row m = frame t of utterance seg_of(m)
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
        a_t[i] = (m < p.M) ? t : -0x40000000;  // invalid rows fail the t-range test
        a_l[i] = p.Ti;
      }
    }
  }

  // Loads the k-tile starting at k0; UNI requires calls with k0 = 0, 32, 64, ...
  // `live` = false issues the same loads with out-of-range offsets (zeros):
  // pipelines past the last tile keep a branch-free, exactly counted stream.
  __device__ __forceinline__ void load(int k0, f32x4 (&ra)[AR], bool live = true) {
    if constexpr (UNI) {
      const int off = j * dil - pad;
      const float* base = a0;
      int ld = ld0, cl = c;
      if (AMODE == kACat) {
        if (c >= cs2) {
          base = a2;
          ld = ld2;
          cl = c - cs2;
        } else if (c >= cs1) {
          base = a1;
          ld = ld1;
          cl = c - cs1;
        }
      }
      const __amdgpu_buffer_rsrc_t r0 = make_rsrc(base);
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a1);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int tt = a_t[i] + off;
        const bool ok = live && tt >= 0 && tt < a_l[i];
        const int row = a_r[i] + off;
        ra[i] = bload4(r0, ok ? (row * ld + cl + c4) * 4 : kOOB);
        if (AMODE == kAAdd) ra[i] += bload4(r1, ok ? (row * ld1 + c + c4) * 4 : kOOB);
      }
      c += 32;
      if (c >= cin) {
        c -= cin;
        ++j;
      }
    } else {
      const int k = k0 + c4;
      const bool kin = k < K;
      const int jj = kin ? k / cin : 0;
      const int cc = k - jj * cin;
      const int off = jj * dil - pad;
      const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a0);
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a1);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int tt = a_t[i] + off;
        const bool ok = live && kin && tt >= 0 && tt < a_l[i];
        const int row = a_r[i] + off;
        ra[i] = bload4(r0, ok ? (row * ld0 + cc) * 4 : kOOB);
        if (AMODE == kAAdd) ra[i] += bload4(r1, ok ? (row * ld1 + cc) * 4 : kOOB);
      }
    }
  }
};

// 2-D NHWC variant (ResNet): rows are output positions (b, fo, to); one
// segment, cin % 32 == 0 (uniform k-tiles).
template <int AR>
struct ALoader2D {
  const float* a0;
  int ld, cin, Fi, Ti, kw, T0;
  int c4;
  int rb[AR], fi0[AR], ti0[AR];
  int j, c;

  __device__ __forceinline__ void init(const ConvGemmArgs& p, int m0, int srow, int rows_step,
                                       int c4_) {
    a0 = p.a[0];
    ld = p.lda[0];
    cin = p.cin;
    Fi = p.Fi;
    Ti = p.Ti;
    kw = p.kw;
    c4 = c4_;
    j = 0;
    c = 0;
    const int plane = p.Fo * p.To;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + srow + rows_step * i;
      const int b = m / plane;
      const int rem = m - b * plane;
      const int fo = rem / p.To;
      const int to = rem - fo * p.To;
      rb[i] = b * p.Fi * p.Ti;
      fi0[i] = (m < p.M) ? fo * p.stride - p.pad : -0x40000000;
      ti0[i] = to * p.stride - p.pad;
    }
  }

  __device__ __forceinline__ void load(int /*k0*/, f32x4 (&ra)[AR], bool live = true) {
    const int kf = j / kw;
    const int kt = j - kf * kw;
    const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a0);
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int fi = fi0[i] + kf;
      const int ti = ti0[i] + kt;
      const bool ok = live && fi >= 0 && fi < Fi && ti >= 0 && ti < Ti;
      const int row = rb[i] + fi * Ti + ti;
      ra[i] = bload4(r0, ok ? (row * ld + c + c4) * 4 : kOOB);
    }
    c += 32;
    if (c >= cin) {
      c -= cin;
      ++j;
    }
  }
};

// Shared GEMM epilogue for a wave's TM x TN tiles of 32x32 accumulators
// (gfx950 32x32 C/D map: col = lane&31, row = (r&3) + 8(r>>2) + 4(lane>>5)).
//   y = act(acc + bias[n] + row_bias[utt(row)][n] + res[row][n]) * scale[n] + shift[n]
// Branch-free per element: the launch-uniform choices (activation, per-utterance
// bias) select one of eight straight-line store loops up front — per-element
// uniform branches made the epilogue ~18 % of a K=1024 block (in-kernel
// s_memtime stamps) — and a row's byte offset is the tile's base plus a
// compile-time row step times 4*ldo (no per-element multiply).  Rows >= M get
// out-of-range buffer offsets: loads return 0, stores are dropped.
// Residual rows of a wave's tiles in the accumulator layout (row (r&3) + 8(r>>2) + 4h
// of tile i, column lane&31 of tile j): one b32 load per register.
template <int TM, int TN>
__device__ __forceinline__ void load_residual_tiles(const ConvGemmArgs& p, float (&rv)[TM][TN][16], int m0, int n0,
                                                    int wm, int wn, int lane) {
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(p.res);
  const int ldr4 = p.ldres * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row0 = m0 + (wm * TM + i) * 32 + 4 * h;
      const int lim = p.M - row0;
      const int rbase = row0 * ldr4 + (n0 + (wn * TN + j) * 32 + r32) * 4;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2);
        rv[i][j][r] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rres, rr < lim ? rbase + rr * ldr4 : kOOB, 0, 0));
      }
    }
}

// PRE: the residual was loaded by the caller (rext, load_residual_tiles) ahead of
// the last k-steps, so its latency overlaps them.
template <int TM, int TN, int ACT, bool RB, bool CS = false, bool RES = false, bool PRE = false>
__device__ __forceinline__ void gemm_epilogue_store(const ConvGemmArgs& p, f32x16 (&acc)[TM][TN], int m0, int n0,
                                                    int wm, int wn, int lane, double (*cs)[2] = nullptr,
                                                    const float (*rext)[TN][16] = nullptr) {
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const int ldo4 = p.ldo * 4;
  // RES: the residual is read per 32-row tile right where it is added (the 16 loads
  // of a tile are independent and issue together) — no residual register file next
  // to the accumulators, which wide wave tiles cannot afford
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? p.res : p.out);
  const int ldr4 = p.ldres * 4;
  // narrow wave tiles (<= 4 tiles) can afford every residual load up front: one
  // round trip per wave instead of one per tile (HBM-bound ResNet conv3: -4 %)
  constexpr bool RPRE = RES && !PRE && TM * TN <= 4;
  float rpre[RPRE ? TM : 1][RPRE ? TN : 1][16];
  if constexpr (RPRE) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row0 = m0 + (wm * TM + i) * 32 + 4 * h;
        const int lim = p.M - row0;
        const int rbase = row0 * ldr4 + (n0 + (wn * TN + j) * 32 + r32) * 4;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2);
          rpre[i][j][r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rres, rr < lim ? rbase + rr * ldr4 : kOOB, 0, 0));
        }
      }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + (wn * TN + j) * 32 + r32;
    const float bv = p.bias ? p.bias[col] : 0.f;
    const float sc = p.scale ? p.scale[col] : 1.f;
    const float sh = p.scale ? p.shift[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row0 = m0 + (wm * TM + i) * 32 + 4 * h;
      const int lim = p.M - row0;  // rows row0 + rr with rr < lim exist
      const int base = row0 * ldo4 + col * 4;
      // CS: the 32-row tile lies wholly in the block's first utterance (0), wholly
      // in the next one (1), or straddles the boundary / the end of M (2)
      int mode = 2;
      if constexpr (CS) {
        const int t0 = m0 + (wm * TM + i) * 32;
        const int next = (m0 / p.T + 1) * p.T;
        if (t0 + 32 <= p.M) mode = t0 + 32 <= next ? 0 : (t0 >= next ? 1 : 2);
      }
      float rv[16];
      if constexpr (PRE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) rv[r] = rext[i][j][r];
      } else if constexpr (RPRE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) rv[r] = rpre[i][j][r];
      } else if constexpr (RES && !PRE) {
        const int rbase = row0 * ldr4 + col * 4;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2);
          rv[r] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rres, rr < lim ? rbase + rr * ldr4 : kOOB, 0, 0));
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2);
        float y = acc[i][j][r] + bv;
        if constexpr (RES) y += rv[r];
        if constexpr (RB) {
          const int row = row0 + rr;
          const int rowc = row < p.M ? row : p.M - 1;
          const int ub = p.seg ? seg_of(p.seg, p.nseg, rowc) : rowc / p.T;
          y += p.row_bias[(size_t)ub * p.N + col];
        }
        if constexpr (ACT == kActRelu) y = fmaxf(y, 0.f);
        else if constexpr (ACT == kActTanh) y = tanhf(y);
        else if constexpr (ACT == kActGelu) y = gelu_as(y);
        y = y * sc + sh;
        const int off = rr < lim ? base + rr * ldo4 : kOOB;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, off, 0, 0);
        if constexpr (CS) {  // rows < next: block's first utterance; next <= rows < M: the next one
          const double yd = (double)y;
          if (mode == 0) {
            cs[j][0] += yd;
          } else if (mode == 1) {
            cs[j][1] += yd;
          } else {
            const int row = row0 + rr;
            const int next = (m0 / p.T + 1) * p.T;
            cs[j][0] += (row < next && row < p.M) ? yd : 0.0;
            cs[j][1] += (row >= next && row < p.M) ? yd : 0.0;
          }
        }
      }
    }
  }
}

// Block-level reduction of the per-lane column sums into the f64 partials
// p.colsum[((m0 / BM) * 2 + slot) * N + n] — lanes l and l+32 (same column) by
// a shuffle, the WM waves of a column through LDS in wave order (fixed order:
// deterministic).  All threads of the block call it (it holds a barrier); smem
// must be free (after the k-loop's last barrier).
template <int TN, int WM, int WN, int BM>
__device__ __forceinline__ void gemm_colsum_reduce(const ConvGemmArgs& p, double (*cs)[2], int m0, int n0, int wm,
                                                   int wn, int lane, unsigned char* smem) {
  constexpr int BN = WN * TN * 32;
  double* red = reinterpret_cast<double*>(smem);  // [WM][2][BN]
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const double v = cs[j][u] + __shfl_xor(cs[j][u], 32);
      if (lane < 32) red[(wm * 2 + u) * BN + (wn * TN + j) * 32 + lane] = v;
    }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < 2 * BN) {
    const int u = tid / BN, c = tid - u * BN;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < WM; ++w) v += red[(w * 2 + u) * BN + c];
    p.colsum[((size_t)(m0 / BM) * 2 + u) * p.N + n0 + c] = v;
  }
}

template <int TM, int TN, int WM = 0, int WN = 0>
__device__ __forceinline__ void gemm_epilogue(const ConvGemmArgs& p, f32x16 (&acc)[TM][TN], int m0, int n0,
                                              int wm, int wn, int lane, unsigned char* smem = nullptr) {
  if constexpr (WM > 0) {
    if (p.colsum) {  // fused per-utterance column sums (host: uniform batch, T >= BM, no row bias)
      double cs[TN][2];
#pragma unroll
      for (int j = 0; j < TN; ++j) cs[j][0] = cs[j][1] = 0.0;
      switch (p.act) {
        case kActRelu: gemm_epilogue_store<TM, TN, kActRelu, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
        case kActTanh: gemm_epilogue_store<TM, TN, kActTanh, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
        case kActGelu: gemm_epilogue_store<TM, TN, kActGelu, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
        default: gemm_epilogue_store<TM, TN, kActNone, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
      }
      gemm_colsum_reduce<TN, WM, WN, WM * TM * 32>(p, cs, m0, n0, wm, wn, lane, smem);
      return;
    }
  }
  if (p.res) {  // residual convs: no row bias / column sums (checked on the host)
    switch (p.act) {
      case kActRelu: gemm_epilogue_store<TM, TN, kActRelu, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store<TM, TN, kActTanh, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store<TM, TN, kActGelu, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store<TM, TN, kActNone, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
    }
    return;
  }
  if (p.row_bias) {
    switch (p.act) {
      case kActRelu: gemm_epilogue_store<TM, TN, kActRelu, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store<TM, TN, kActTanh, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store<TM, TN, kActGelu, true>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store<TM, TN, kActNone, true>(p, acc, m0, n0, wm, wn, lane); break;
    }
  } else {
    switch (p.act) {
      case kActRelu: gemm_epilogue_store<TM, TN, kActRelu, false>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store<TM, TN, kActTanh, false>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store<TM, TN, kActGelu, false>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store<TM, TN, kActNone, false>(p, acc, m0, n0, wm, wn, lane); break;
    }
  }
}

// Residual epilogue with the residual already in registers (see gemm_epilogue_store).
template <int TM, int TN>
__device__ __forceinline__ void gemm_epilogue_res_pre(const ConvGemmArgs& p, f32x16 (&acc)[TM][TN], int m0, int n0,
                                                      int wm, int wn, int lane, const float (&rv)[TM][TN][16]) {
  switch (p.act) {
    case kActRelu: gemm_epilogue_store<TM, TN, kActRelu, false, false, true, true>(p, acc, m0, n0, wm, wn, lane, nullptr, rv); break;
    case kActTanh: gemm_epilogue_store<TM, TN, kActTanh, false, false, true, true>(p, acc, m0, n0, wm, wn, lane, nullptr, rv); break;
    case kActGelu: gemm_epilogue_store<TM, TN, kActGelu, false, false, true, true>(p, acc, m0, n0, wm, wn, lane, nullptr, rv); break;
    default: gemm_epilogue_store<TM, TN, kActNone, false, false, true, true>(p, acc, m0, n0, wm, wn, lane, nullptr, rv); break;
  }
}

// The same epilogue for 16x16 accumulator tiles (v_mfma_f32_16x16x32_bf16 C/D map: col =
// lane & 15, row = 4 (lane >> 4) + r, r = 0..3): a wave's TM x TN tiles of 16 x 16.  The
// residual is read per tile (4 loads) right where it is added.
template <int TM, int TN, int ACT, bool RB, bool CS = false, bool RES = false>
__device__ __forceinline__ void gemm_epilogue_store16(const ConvGemmArgs& p, f32x4 (&acc)[TM][TN], int m0, int n0,
                                                      int wm, int wn, int lane, double (*cs)[2] = nullptr) {
  const int c16 = lane & 15;
  const int q = lane >> 4;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const int ldo4 = p.ldo * 4;
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? p.res : p.out);
  const int ldr4 = p.ldres * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + (wn * TN + j) * 16 + c16;
    const float bv = p.bias ? p.bias[col] : 0.f;
    const float sc = p.scale ? p.scale[col] : 1.f;
    const float sh = p.scale ? p.shift[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int t0 = m0 + (wm * TM + i) * 16;  // the tile's first row
      const int row0 = t0 + 4 * q;
      const int lim = p.M - row0;  // rows row0 + r with r < lim exist
      const int base = row0 * ldo4 + col * 4;
      int mode = 2;  // CS: as gemm_epilogue_store, per 16-row tile
      if constexpr (CS) {
        const int next = (m0 / p.T + 1) * p.T;
        if (t0 + 16 <= p.M) mode = t0 + 16 <= next ? 0 : (t0 >= next ? 1 : 2);
      }
      float rv[4];
      if constexpr (RES) {
        const int rbase = row0 * ldr4 + col * 4;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          rv[r] = __builtin_bit_cast(float,
                                     __builtin_amdgcn_raw_buffer_load_b32(rres, r < lim ? rbase + r * ldr4 : kOOB, 0, 0));
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float y = acc[i][j][r] + bv;
        if constexpr (RES) y += rv[r];
        if constexpr (RB) {
          const int row = row0 + r;
          const int rowc = row < p.M ? row : p.M - 1;
          const int ub = p.seg ? seg_of(p.seg, p.nseg, rowc) : rowc / p.T;
          y += p.row_bias[(size_t)ub * p.N + col];
        }
        if constexpr (ACT == kActRelu) y = fmaxf(y, 0.f);
        else if constexpr (ACT == kActTanh) y = tanhf(y);
        else if constexpr (ACT == kActGelu) y = gelu_as(y);
        y = y * sc + sh;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, r < lim ? base + r * ldo4 : kOOB, 0,
                                              0);
        if constexpr (CS) {
          const double yd = (double)y;
          if (mode == 0) {
            cs[j][0] += yd;
          } else if (mode == 1) {
            cs[j][1] += yd;
          } else {
            const int row = row0 + r;
            const int next = (m0 / p.T + 1) * p.T;
            cs[j][0] += (row < next && row < p.M) ? yd : 0.0;
            cs[j][1] += (row >= next && row < p.M) ? yd : 0.0;
          }
        }
      }
    }
  }
}

// gemm_colsum_reduce for the 16x16 map: lanes l, l ^ 16, l ^ 32, l ^ 48 share a column.
template <int TN, int WM, int WN, int BM>
__device__ __forceinline__ void gemm_colsum_reduce16(const ConvGemmArgs& p, double (*cs)[2], int m0, int n0, int wm,
                                                     int wn, int lane, unsigned char* smem) {
  constexpr int BN = WN * TN * 16;
  double* red = reinterpret_cast<double*>(smem);  // [WM][2][BN]
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      double v = cs[j][u] + __shfl_xor(cs[j][u], 16);
      v += __shfl_xor(v, 32);
      if (lane < 16) red[(wm * 2 + u) * BN + (wn * TN + j) * 16 + lane] = v;
    }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < 2 * BN) {
    const int u = tid / BN, c = tid - u * BN;
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < WM; ++w) v += red[(w * 2 + u) * BN + c];
    p.colsum[((size_t)(m0 / BM) * 2 + u) * p.N + n0 + c] = v;
  }
}

template <int TM, int TN, int WM, int WN>
__device__ __forceinline__ void gemm_epilogue16(const ConvGemmArgs& p, f32x4 (&acc)[TM][TN], int m0, int n0, int wm,
                                                int wn, int lane, unsigned char* smem) {
  if (p.colsum) {
    double cs[TN][2];
#pragma unroll
    for (int j = 0; j < TN; ++j) cs[j][0] = cs[j][1] = 0.0;
    switch (p.act) {
      case kActRelu: gemm_epilogue_store16<TM, TN, kActRelu, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
      case kActTanh: gemm_epilogue_store16<TM, TN, kActTanh, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
      case kActGelu: gemm_epilogue_store16<TM, TN, kActGelu, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
      default: gemm_epilogue_store16<TM, TN, kActNone, false, true>(p, acc, m0, n0, wm, wn, lane, cs); break;
    }
    gemm_colsum_reduce16<TN, WM, WN, WM * TM * 16>(p, cs, m0, n0, wm, wn, lane, smem);
    return;
  }
  if (p.res) {
    switch (p.act) {
      case kActRelu: gemm_epilogue_store16<TM, TN, kActRelu, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store16<TM, TN, kActTanh, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store16<TM, TN, kActGelu, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store16<TM, TN, kActNone, false, false, true>(p, acc, m0, n0, wm, wn, lane); break;
    }
    return;
  }
  if (p.row_bias) {
    switch (p.act) {
      case kActRelu: gemm_epilogue_store16<TM, TN, kActRelu, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store16<TM, TN, kActTanh, true>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store16<TM, TN, kActGelu, true>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store16<TM, TN, kActNone, true>(p, acc, m0, n0, wm, wn, lane); break;
    }
  } else {
    switch (p.act) {
      case kActRelu: gemm_epilogue_store16<TM, TN, kActRelu, false>(p, acc, m0, n0, wm, wn, lane); break;
      case kActTanh: gemm_epilogue_store16<TM, TN, kActTanh, false>(p, acc, m0, n0, wm, wn, lane); break;
      case kActGelu: gemm_epilogue_store16<TM, TN, kActGelu, false>(p, acc, m0, n0, wm, wn, lane); break;
      default: gemm_epilogue_store16<TM, TN, kActNone, false>(p, acc, m0, n0, wm, wn, lane); break;
    }
  }
}

// True when every 32-wide k-tile of the operand stays in one tap and segment.
inline bool uniform_ktiles(const ConvGemmArgs& p) {
  if (p.cin % 32 != 0) return false;
  if (p.amode == kACat && (p.cseg[1] % 32 != 0 || p.cseg[2] % 32 != 0)) return false;
  return true;
}

inline void check_conv_args(const ConvGemmArgs& p, const char* who) {
  const std::string w(who);
  // buffer-load byte offsets are 32-bit: every operand must stay below 2 GiB
  // input rows: 1-D strided convs read (M / T) * Ti rows; 2-D reads B*Fi*Ti
  const long long in_rows = (p.conv2d || p.sc2d) ? std::max<long long>(p.M, (long long)(p.M / (p.Fo * p.To)) * p.Fi * p.Ti)
                            : p.seg ? (long long)std::max(p.M, p.Ti)
                                     : std::max<long long>(p.M, (long long)((p.M + p.T - 1) / p.T) * p.Ti);
  for (int i = 0; i < 3; ++i)
    WSP_CHECK(in_rows * p.lda[i] * 4 < (long long)kOOB, w + ": operand exceeds 2 GiB (split the batch)");
  WSP_CHECK((long long)p.M * p.ldo * 4 < (long long)kOOB, w + ": output exceeds 2 GiB (split the batch)");
  if (p.res) WSP_CHECK((long long)p.M * p.ldres * 4 < (long long)kOOB, w + ": residual exceeds 2 GiB");
  WSP_CHECK((long long)p.N * p.Kp * 4 < (long long)kOOB, w + ": weights exceed 2 GiB");
  WSP_CHECK(p.M > 0 && p.N > 0 && p.K > 0 && p.T > 0, w + ": empty shape");
  WSP_CHECK(p.cin % 4 == 0, w + ": cin must be a multiple of 4");
  WSP_CHECK(p.K == p.cin * p.taps, w + ": K != cin * taps");
  WSP_CHECK(p.Kp % 32 == 0 && p.Kp >= p.K, w + ": bad packed K");
  WSP_CHECK(p.N % 32 == 0, w + ": N must be a multiple of 32");
  if (p.conv2d) {
    WSP_CHECK(p.amode == kACat && p.cseg[1] == p.cin && p.cin % 32 == 0,
              w + ": 2-D conv needs one segment with cin % 32 == 0");
    WSP_CHECK(p.M == p.T * p.Fo * p.To || p.T > 0, w + ": bad 2-D shape");
    WSP_CHECK(p.taps % p.kw == 0 && p.stride >= 1, w + ": bad 2-D taps/stride");
  }
  for (int i = 0; i < 3; ++i) WSP_CHECK(p.lda[i] % 4 == 0, w + ": lda must be a multiple of 4");
  if (p.sc2d)
    WSP_CHECK(!p.conv2d && !p.seg && p.taps == 1 && p.pad == 0 && p.amode == kACat && p.cseg[1] % 32 == 0 &&
                  p.cseg[2] == p.cin && p.stride >= 1 && p.Fo >= 1 && p.To >= 1 && p.M % (p.Fo * p.To) == 0 &&
                  (p.Fo - 1) * p.stride < p.Fi && (p.To - 1) * p.stride < p.Ti,
              w + ": conv3 + shortcut needs a dense 1x1 segment and a 2-D strided segment");
  if (!p.conv2d) WSP_CHECK(p.stride >= 1 && p.Ti >= 1, w + ": call normalized() first");
  if (p.seg) WSP_CHECK(!p.conv2d && p.nseg >= 1 && (p.iseg || p.stride == 1), w + ": segmented batch needs a 1-D conv (input offsets when strided)");
  WSP_CHECK(!p.res || (!p.row_bias && !p.colsum), w + ": a residual epilogue has no row bias / column sums");
  if (p.gcols) {
    WSP_CHECK(p.amode == kACat && p.cseg[1] == p.cin && !p.conv2d, w + ": grouped conv needs one 1-D segment");
    WSP_CHECK(p.N % p.gcols == 0 && p.gcols % 32 == 0 && p.gcin % 4 == 0, w + ": bad grouped-conv columns");
    WSP_CHECK(p.res == nullptr, w + ": grouped conv has no residual epilogue");
  }
  if (p.amode == kACat) {
    WSP_CHECK(p.cseg[0] == 0 && p.cseg[3] == p.cin && p.cseg[1] <= p.cseg[2] &&
                  p.cseg[2] <= p.cseg[3],
              w + ": bad channel segments");
    for (int i = 1; i < 3; ++i) WSP_CHECK(p.cseg[i] % 4 == 0, w + ": segment not float4 aligned");
    if (!uniform_ktiles(p))
      WSP_CHECK(p.cseg[1] == p.cin, w + ": multi-segment A needs 32-aligned segments");
  }
}

}  // namespace wsp
