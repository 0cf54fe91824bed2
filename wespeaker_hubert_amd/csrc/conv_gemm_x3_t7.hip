// conv_gemm_x3 tile family 7, persistent form (r5, option gemm_persist): one block per CU walks its
// tiles, and the next tile's first two k-tiles are fetched while the current tile's epilogue runs.
//
// Family 7 (conv_gemm_x3_t6.hip) holds one block per CU, so every tile pays its epilogue (256 KB of
// outputs staged through LDS and stored) and its first k-tiles' DMA latency with no MFMA work on the
// CU.  Here, when a tile's k-loop ends, the next tile's k-tiles 0 and 1 go out by LDS-DMA into the
// two stages BEFORE the epilogue, which stages its rows 8 at a time in the 32 KB above the stages
// (128 + 32 KB = the whole LDS); the next tile starts after a full drain (vmcnt(0): stores and
// loads share the counter, so a counted wait past the stores would not be safe).  Tiles are
// visited in family 7's XCD-remapped order (the grid is a multiple of 8 blocks, so a block's tiles
// stay on its XCD).  Same k order, MFMA order and per-element epilogue arithmetic as family 7:
// bit-identical.  Operands: family 7's, without the SE column sums or the LayerNorm fold.
#include "conv_gemm_x3_impl.h"

namespace wsp {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPA = 256 * 128, kPW = 256 * 64, kPStage = kPA + 2 * kPW;
constexpr int kPEpiLd = 128;
constexpr int kPEpiOff = 2 * kPStage;                   // staging above both stages
constexpr int kPLds = kPEpiOff + 8 * 8 * kPEpiLd * 4;   // 163,840 B: all of the LDS

__device__ __forceinline__ int p_aslot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 5)) << 4); }

__device__ __forceinline__ void p_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// family 7's g_epilogue_rows in 8-row passes (rows 8 h .. + 7 of acc block i: the lanes with
// q >> 1 == h hold them, rows 4 (q & 1) + r), so the staging fits above the two stages
template <int ACT, bool RB, bool RES>
__device__ __forceinline__ void p_epilogue(const ConvGemmArgs& p, f32x4 (&acc)[4][8], int m0, int n0, int wm, int wn,
                                           int wave, int lane, unsigned char* smem) {
  float* stg = reinterpret_cast<float*>(smem + kPEpiOff) + wave * 8 * kPEpiLd;
  const int c16 = lane & 15, q = lane >> 4;
  const int cl = 4 * (lane & 31);
  const int col = n0 + wn * 128 + cl;
  const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 sc = p.scale ? *reinterpret_cast<const f32x4*>(p.scale + col) : f32x4{1.f, 1.f, 1.f, 1.f};
  const f32x4 sh = p.scale ? *reinterpret_cast<const f32x4*>(p.shift + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? p.res : p.out);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if ((q >> 1) == h) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) stg[(4 * (q & 1) + r) * kPEpiLd + j * 16 + c16] = acc[i][j][r];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private block: in-order LDS, no barrier
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int rl = 2 * u + (lane >> 5);
        const int row = m0 + wm * 64 + i * 16 + h * 8 + rl;
        const bool ok = row < p.M;
        const f32x4 x = *reinterpret_cast<const f32x4*>(stg + rl * kPEpiLd + cl);
        f32x4 rv{0.f, 0.f, 0.f, 0.f}, rb{0.f, 0.f, 0.f, 0.f};
        if constexpr (RES) rv = bload4(rres, ok ? (row * p.ldres + col) * 4 : kOOB);
        if constexpr (RB) {
          const int rowc = ok ? row : p.M - 1;
          const int ub = p.seg ? seg_of(p.seg, p.nseg, rowc) : rowc / p.T;
          rb = *reinterpret_cast<const f32x4*>(p.row_bias + (size_t)ub * p.N + col);
        }
        f32x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = x[e] + bv[e];
          if constexpr (RES) v += rv[e];
          if constexpr (RB) v += rb[e];
          if constexpr (ACT == kActRelu) v = fmaxf(v, 0.f);
          else if constexpr (ACT == kActTanh) v = tanhf(v);
          else if constexpr (ACT == kActGelu) v = gelu_as(v);
          y[e] = v * sc[e] + sh[e];
        }
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), ro, ok ? (row * p.ldo + col) * 4 : kOOB,
                                               0, 0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass overwrites
    }
}

template <int AM>
__global__ __launch_bounds__(512, 1) void conv_gemm_gp(const ConvGemmArgs p, const __bf16* __restrict__ whi,
                                                       const __bf16* __restrict__ wlo) {
  using L = Lds<true, 16>;
  constexpr bool DENSE = AM == 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int ntiles = p.N / 256;
  const int nwg = ntiles * ((p.M + 255) / 256);
  const int ac0 = 4 * ((lane & 7) ^ ((lane >> 4) & 1)), ac1 = ac0 ^ 16;
  const __amdgpu_buffer_rsrc_t rwh = make_rsrc(whi);
  const __amdgpu_buffer_rsrc_t rwl = make_rsrc(wlo);
  const int nk = p.Kp / BK;  // >= 2 (Kp % 64 == 0)

  // per-tile A / W geometry (family 7's DMA pieces)
  int m0 = 0, n0 = 0;
  int a_r[4], a_t[DENSE ? 1 : 4], a_l[DENSE ? 1 : 4], woff[2];
  int jt = 0, ct = 0;  // tap and channel of the next k-tile to fetch
  auto setup = [&](int v) {
    const int wg = xcd_remap(v, nwg);
    const int mt = wg / ntiles;
    m0 = mt * 256;
    n0 = (wg - mt * ntiles) * 256;
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
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = (2 * wave + i) * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((0x1320 >> (4 * ((row >> 2) & 3))) & 3);
      woff[i] = ((n0 + row) * p.Kp + 8 * c) * 2;
    }
    jt = 0;
    ct = 0;
  };
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * kPStage;
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
        p_dma(ra, st + (4 * wave + i) * 1024, a_r[i] >= 0 ? (a_r[i] * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      } else {
        const int tt = a_t[i] + off;
        const bool ok = tt >= 0 && tt < a_l[i];
        p_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + off) * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = woff[i] + kt * 64;
      p_dma(rwh, st + kPA + (2 * wave + i) * 1024, o);
      p_dma(rwl, st + kPA + kPW + (2 * wave + i) * 1024, o);
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
  bf16x8 ah[2], al[2], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 64 + (ih * 2 + i) * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + p_aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + p_aslot(r, 2 * qk + 1));
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
      bh[j] = *reinterpret_cast<const bf16x8*>(st + kPA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + kPA + kPW + o);
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

  int v = blockIdx.x;  // virtual block id of the current tile (family 7's blockIdx)
  if (v >= nwg) return;  // block-uniform
  setup(v);
  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0's k-tile 0 landed (8 DMAs per k-tile and lane)
  __builtin_amdgcn_s_barrier();
  while (true) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      const unsigned char* st = smem + buf * kPStage;
      rdA(st, 0);
      rdB(st, 0);
      mm(0, 0);
      rdB(st, 1);
      mm(0, 1);
      rdA(st, 1);
      mm(1, 1);
      rdB(st, 0);
      mm(1, 0);
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) dma(kt + 2, buf);
    }
    // every wave is past the last reads and no DMA is in flight: the next tile's k-tiles 0 and 1 go
    // into the stages ahead of this tile's epilogue (which stages above them)
    const int m0c = m0, n0c = n0;
    const int vn = v + gridDim.x;
    const bool more = vn < nwg;  // block-uniform
    if (more) {
      setup(vn);
      dma(0, 0);
      dma(1, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#define WSP_PEPI(RB, RES)                                                                                  \
  switch (p.act) {                                                                                        \
    case kActRelu: p_epilogue<kActRelu, RB, RES>(p, acc, m0c, n0c, wm, wn, wave, lane, smem); break;      \
    case kActTanh: p_epilogue<kActTanh, RB, RES>(p, acc, m0c, n0c, wm, wn, wave, lane, smem); break;      \
    case kActGelu: p_epilogue<kActGelu, RB, RES>(p, acc, m0c, n0c, wm, wn, wave, lane, smem); break;      \
    default: p_epilogue<kActNone, RB, RES>(p, acc, m0c, n0c, wm, wn, wave, lane, smem); break;            \
  }
    if (p.res) {
      WSP_PEPI(false, true)
    } else if (p.row_bias) {
      WSP_PEPI(true, false)
    } else {
      WSP_PEPI(false, false)
    }
#undef WSP_PEPI
    if (!more) break;
    // the next tile's k-tiles 0 / 1 have landed (full drain, see the header) in every wave
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    v = vn;
  }
}

}  // namespace

namespace x3 {

bool gp256_supported(const ConvGemmArgs& p) {
  return g256_supported(p) && !p.colsum && !p.lnmode && uniform_ktiles(p);
}

void t_gp256(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  // one block per CU; a multiple of 8 keeps every block's tiles on its XCD (xcd_remap)
  const int grid = std::min(nwg, std::max(8, device_cu_count() / 8 * 8));
  const bool dense = p.taps == 1 && p.pad == 0 && p.stride == 1 && !p.iseg && (p.seg || p.Ti == p.T);
  if (dense)
    hipLaunchKernelGGL((conv_gemm_gp<1>), dim3(grid), dim3(512), kPLds, s, p, h, l);
  else
    hipLaunchKernelGGL((conv_gemm_gp<0>), dim3(grid), dim3(512), kPLds, s, p, h, l);
  WSP_HIP(hipGetLastError());
}

}  // namespace x3
}  // namespace wsp
