// conv_gemm_x3 tile family 9 (r5, x3_variant 9): family 7's 256 x 256 bf16x3 tile with every
// operand staged by LDS-DMA, on 8 waves of 32 rows x 256 columns instead of 4 x 2 waves of
// 64 x 128.
//
// In family 7 each A element is split into bf16 hi / lo by both column waves that read it; the
// split (~3 VALU per float, a wave64 VALU op issuing over 4 cycles) is the k-loop's largest
// overhead.  Here a wave owns whole rows: every A fragment is split once, for 16 B fragments, at
// the price of 1.5x the B fragment reads per MFMA (36 ds_read_b128 per 96 MFMAs against 24).
// (A 16-wave form of 64 x 64 wave tiles — four waves per SIMD for latency hiding, but twice the
// split work — was bit-identical and 2-55 % slower on every in-model shape.)  Same LDS stage
// layout, DMA pieces and k order as family 7, the same MFMA order per accumulator and the same
// epilogue arithmetic: bit-identical to families 6 / 7.  The epilogue stages each wave's rows 16
// at a time in a private [16][260] fp32 block and stores whole 1-KB row pieces in 16-B stores.
#include "conv_gemm_x3_impl.h"

namespace wsp {
namespace {

typedef __attribute__((address_space(3))) void lds_void;
constexpr int kQA = 256 * 128, kQW = 256 * 64, kQStage = kQA + 2 * kQW;
constexpr int kQEpiLd = 260;
constexpr int kQEpiBytes = 8 * 16 * kQEpiLd * 4;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int q_aslot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 5)) << 4); }

__device__ __forceinline__ void q_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

template <int ACT, bool RB, bool RES>
__device__ __forceinline__ void q_epilogue(const ConvGemmArgs& p, f32x4 (&acc)[2][16], int m0, int n0, int wave,
                                           int lane, unsigned char* smem) {
  float* stg = reinterpret_cast<float*>(smem) + wave * 16 * kQEpiLd;
  const int c16 = lane & 15, q = lane >> 4;
  const int cl = 4 * lane;  // this lane's 4 columns of the 256
  const int col = n0 + cl;
  const f32x4 bv = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 sc = p.scale ? *reinterpret_cast<const f32x4*>(p.scale + col) : f32x4{1.f, 1.f, 1.f, 1.f};
  const f32x4 sh = p.scale ? *reinterpret_cast<const f32x4*>(p.shift + col) : f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const __amdgpu_buffer_rsrc_t rres = make_rsrc(RES ? p.res : p.out);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) stg[(4 * q + r) * kQEpiLd + j * 16 + c16] = acc[i][j][r];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private block: in-order LDS, no barrier
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int row = m0 + wave * 32 + i * 16 + u;
      const bool ok = row < p.M;
      const f32x4 x = *reinterpret_cast<const f32x4*>(stg + u * kQEpiLd + cl);
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
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, y), ro, ok ? (row * p.ldo + col) * 4 : kOOB, 0,
                                             0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next pass overwrites
  }
}

template <int AM>
__global__ __launch_bounds__(512, 1) void conv_gemm_q(const ConvGemmArgs p, const __bf16* __restrict__ whi,
                                                       const __bf16* __restrict__ wlo) {
  using L = Lds<true, 16>;
  constexpr bool DENSE = AM == 1;
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

  // ---- A rows: DMA i (0..3) of wave w fills LDS rows (4 w + i) * 8 .. + 7 (family 7's pieces)
  const int ac0 = 4 * ((lane & 7) ^ ((lane >> 4) & 1)), ac1 = ac0 ^ 16;
  int a_r[DENSE ? 1 : 4], a_t[DENSE ? 1 : 4], a_l[DENSE ? 1 : 4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (4 * wave + i) * 8 + (lane >> 3);
    if constexpr (DENSE) {
      (void)m;
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
  int jt = 0, ct = 0;        // tap and channel of the next k-tile to fetch (k-tiles are fetched in order)
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * kQStage;
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
      if constexpr (DENSE) {  // the row is recomputed here (2 VALU) rather than held through the loop
        const int m = m0 + (4 * wave + i) * 8 + (lane >> 3);
        q_dma(ra, st + (4 * wave + i) * 1024, m < p.M ? (m * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      } else {
        const int tt = a_t[i] + off;
        const bool ok = tt >= 0 && tt < a_l[i];
        q_dma(ra, st + (4 * wave + i) * 1024, ok ? ((a_r[i] + off) * ld + cl + (i & 1 ? ac1 : ac0)) * 4 : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = woff[i] + kt * 64;
      q_dma(rwh, st + kQA + (2 * wave + i) * 1024, o);
      q_dma(rwl, st + kQA + kQW + (2 * wave + i) * 1024, o);
    }
    ct += 32;
    if (ct >= p.cin) {
      ct -= p.cin;
      ++jt;
    }
  };

  const int r16 = lane & 15, qk = lane >> 4;  // wave w: rows 32 w .. + 31, all 256 columns
  f32x4 acc[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[2], al[2], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st) {  // fp32 rows -> bf16 hi / lo fragments, once per k-tile
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wave * 32 + i * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + q_aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + q_aslot(r, 2 * qk + 1));
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
  auto rdB = [&](const unsigned char* st, int jq) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = L::off((jq * 4 + j) * 16 + r16, qk * 16);
      bh[j] = *reinterpret_cast<const bf16x8*>(st + kQA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + kQA + kQW + o);
    }
  };
  auto mm = [&](int jq) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[i][jq * 4 + j];
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
    const unsigned char* st = smem + buf * kQStage;
    rdA(st);
#pragma unroll
    for (int jq = 0; jq < 4; ++jq) {
      rdB(st, jq);
      mm(jq);
    }
    // tile kt + 1 (issued a k-tile ago) has landed and every wave is done reading this half
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) dma(kt + 2, buf);
  }
  // no DMA is in flight and every wave is past the last reads: the epilogue may use LDS
#define WSP_QEPI(RB, RES)                                                                                \
  switch (p.act) {                                                                                      \
    case kActRelu: q_epilogue<kActRelu, RB, RES>(p, acc, m0, n0, wave, lane, smem); break;      \
    case kActTanh: q_epilogue<kActTanh, RB, RES>(p, acc, m0, n0, wave, lane, smem); break;      \
    case kActGelu: q_epilogue<kActGelu, RB, RES>(p, acc, m0, n0, wave, lane, smem); break;      \
    default: q_epilogue<kActNone, RB, RES>(p, acc, m0, n0, wave, lane, smem); break;            \
  }
  if (p.res) {
    WSP_QEPI(false, true)
  } else if (p.row_bias) {
    WSP_QEPI(true, false)
  } else {
    WSP_QEPI(false, false)
  }
#undef WSP_QEPI
}

}  // namespace

namespace x3 {

bool q256_supported(const ConvGemmArgs& p) { return g256_supported(p) && !p.colsum && !p.lnmode && uniform_ktiles(p); }

void t_q256(const ConvGemmArgs& p, const __bf16* h, const __bf16* l, hipStream_t s) {
  const int nwg = ((p.M + 255) / 256) * (p.N / 256);
  constexpr int lds = 2 * kQStage > kQEpiBytes ? 2 * kQStage : kQEpiBytes;
  const bool dense = p.taps == 1 && p.pad == 0 && p.stride == 1 && !p.iseg && (p.seg || p.Ti == p.T);
  if (dense)
    hipLaunchKernelGGL((conv_gemm_q<1>), dim3(nwg), dim3(512), lds, s, p, h, l);
  else
    hipLaunchKernelGGL((conv_gemm_q<0>), dim3(nwg), dim3(512), lds, s, p, h, l);
  WSP_HIP(hipGetLastError());
}

}  // namespace x3
}  // namespace wsp
