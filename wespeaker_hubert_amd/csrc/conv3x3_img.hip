// Stride-1 3x3 conv with C = 32 / 64 / 128 channels (the ResNet bottleneck conv2 of
// stages 1-3, resnet.py:72-107, and the basic-block convs of ResNet18/34,
// resnet.py:44-69, with the residual in the epilogue, and the SimAM-ResNet
// basic-block convs, samresnet.py:20-60) on bf16x3 MFMA from an LDS image of the
// input patch.
//
// The implicit GEMM (conv_gemm_x3 with ALoader2D) stages, for every 32-wide
// k-tile, the tile's rows of ONE tap from global memory: each input position is
// fetched nine times (once per tap, mostly L2 hits) and split into bf16 hi / lo
// nine times, and with N = C = 32 / 64 the MFMA work per staged byte is small
// (135-205 TFLOP/s).  Here a block owns an FB x TB tile of output
// positions of one utterance and stages the (FB + 2) x (TB + 2) input patch once,
// already split into bf16 hi / lo planes (rows = patch positions, 16-B chunks
// XOR-swizzled by row so the fragment reads are conflict-free); every tap is a
// row offset into that image.  W arrives in MFMA B-fragment order straight from
// L1 / L2, two k-steps ahead in registers (the res2_chain.hip scheme), so the
// k-loop has no barrier.  k order, MFMA order and epilogue are conv_gemm_x3's:
// the results are bit-identical to the implicit GEMM.
// C = 128 (102 KB image of a 4 x 32 tile, one block per CU): each wave owns one
// 32-position time run and all 128 channels (4 column tiles), or with WN = 2 half
// of them (8 waves; option conv3x3_img 3).  r2: ResNet293 stage-3 3x3 21.2 ->
// 18.4 ms/step (one stream), C3 1 260 -> 1 280 emb/s, ResNet34 10 740 -> 11 030.
#include "conv3x3_img.h"
#include "gemm_common.h"

// Development stamps: tools/tail_check.cpp defines WSP_TAIL_STAMP(k) to record s_memtime at
// tail2_kernel's phase boundaries; in the library it expands to nothing.
#ifndef WSP_TAIL_STAMP
#define WSP_TAIL_STAMP(k)
#endif

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int C, int FB, int TB, int WN = 1, int NWO = 0>
struct Img {
  static constexpr int PT = TB + 2;
  static constexpr int IR = (FB + 2) * PT;  // patch positions
  static constexpr int RB = 2 * C;          // bytes per image row and plane
  static constexpr int PLANE = IR * RB;
  static constexpr int LDS = 2 * PLANE;
  // waves: 32 positions (one time run) x C / WN channels each (NWO: a kernel's own wave count)
  static constexpr int NW = NWO ? NWO : FB * TB / 32 * WN;
  static constexpr int NT = NW * 64;
  static constexpr int CT = C / 32;         // 32-channel column tiles
  static constexpr int TN = CT / WN;        // column tiles per wave
  static constexpr int KC = C / 16;         // k-steps per tap
  static constexpr int KS = 9 * KC;         // k-steps
  static constexpr int C4 = C / 4;
  static constexpr int NQ = (IR * C4 + NT - 1) / NT;  // float4 staging loads per thread
  static_assert(TB % 32 == 0 && KS % 2 == 0, "conv3x3_img tile");
  // 16-B chunk ch of row r at slot ch ^ sw(r): the 16 rows of a ds_read_b128 lane
  // group (16 distinct rows mod 16) hit 16 distinct slots of the 256-B bank row
  __device__ __forceinline__ static int sw(int r) {
    return C == 32 ? ((r >> 2) & 3) : C == 64 ? ((r >> 1) & 7) : (r & 15);
  }
  __device__ __forceinline__ static int addr(int r, int ch) { return r * RB + ((ch ^ sw(r)) << 4); }
};

// The (f0 - 1 .. f0 + FB, t0 - 1 .. t0 + TB) input patch of utterance-relative
// descriptor rx -> bf16 hi / lo image planes, zeros outside the utterance.
template <typename G>
__device__ __forceinline__ void stage_patch(__amdgpu_buffer_rsrc_t rx, int F, int T, int f0, int t0, int tid,
                                            unsigned char* xhi, unsigned char* xlo) {
  constexpr int C = G::RB / 2, PT = G::PT;
  f32x4 v[G::NQ];
#pragma unroll
  for (int i = 0; i < G::NQ; ++i) {
    const int q = tid + i * G::NT;
    const int ir = q / G::C4;
    const int c = (q - ir * G::C4) * 4;
    const int pf = ir / PT;
    const int f = f0 - 1 + pf, t = t0 - 1 + (ir - pf * PT);
    // unsigned range tests joined by & (not &&): compare + select, no exec-mask branches
    const bool ok = (q < G::IR * G::C4) & ((unsigned)f < (unsigned)F) & ((unsigned)t < (unsigned)T);
    v[i] = bload4(rx, ok ? (int)((((unsigned)f * T + t) * C + c) * 4) : kOOB);
  }
#pragma unroll
  for (int i = 0; i < G::NQ; ++i) {
    const int q = tid + i * G::NT;
    if (q < G::IR * G::C4) {
      const int ir = q / G::C4;
      const int c = (q - ir * G::C4) * 4;
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 hh = (__bf16)v[i][e];
        hi[e] = hh;
        lo[e] = (__bf16)(v[i][e] - (float)hh);
      }
      const int a = G::addr(ir, c >> 3) + (c & 7) * 2;
      *reinterpret_cast<bf16x4*>(xhi + a) = hi;
      *reinterpret_cast<bf16x4*>(xlo + a) = lo;
    }
  }
}

template <int C, int FB, int TB, int WN, int MINB, bool RES, bool RELU>
__global__ __launch_bounds__(FB* TB * 2 * WN, MINB) void conv3x3_img_kernel(const Conv3x3Args p) {
  using G = Img<C, FB, TB, WN>;
  constexpr int TN = G::TN, PT = G::PT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int ntf = (p.F + FB - 1) / FB, ntt = (p.T + TB - 1) / TB;
  const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo rows) on one XCD
  const int b = id / (ntf * ntt);
  const int rem = id - b * (ntf * ntt);
  const int tf = rem / ntt;
  const int f0 = tf * FB, t0 = (rem - tf * ntt) * TB;
  const size_t ubase = (size_t)b * p.F * p.T * C;  // utterance b's first element
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x + ubase);

  // ---- input patch (f0 - 1 .. f0 + FB, t0 - 1 .. t0 + TB) -> image, zeros outside
  stage_patch<G>(rx, p.F, p.T, f0, t0, tid, xhi, xlo);

  // this lane's output position: patch-local (lf, lt); tap (kf, kt) reads image row
  // (lf + kf) * PT + lt + kt
  const int pr = wave / WN, wn = wave - pr * WN;  // position run, column group
  const int lf = pr / (TB / 32);
  const int lt0 = (pr % (TB / 32)) * 32;
  const int row0 = lf * PT + lt0 + r32;

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  auto wload = [&](int g, bf16x8 (&bh)[TN], bf16x8 (&bl)[TN]) {
    const bool ok = g < G::KS;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = ((g * 2 * G::CT + wn * TN + j) * 64 + lane) * 16;
      bh[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o : kOOB, 0, 0));
      bl[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o + G::CT * 1024 : kOOB, 0, 0));
    }
  };
  auto read_a = [&](int g, bf16x8& ah, bf16x8& al) {
    const int tap = g / G::KC, cb = g - tap * G::KC;
    const int kf = tap / 3, kt = tap - kf * 3;
    const int a = G::addr(row0 + kf * PT + kt, 2 * cb + h);
    ah = *reinterpret_cast<const bf16x8*>(xhi + a);
    al = *reinterpret_cast<const bf16x8*>(xlo + a);
  };
  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  auto mma = [&](const bf16x8& ah, const bf16x8& al, const bf16x8 (&bh)[TN], const bf16x8 (&bl)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[j], acc[j], 0, 0, 0);
    }
  };

  bf16x8 b0h[TN], b0l[TN], b1h[TN], b1l[TN], a0h, a0l, a1h, a1l;
  wload(0, b0h, b0l);
  wload(1, b1h, b1l);
  __syncthreads();  // image complete
  read_a(0, a0h, a0l);
#pragma unroll 1
  for (int g = 0; g < G::KS; g += 2) {
    // scheduling fences: the next k-step's fragment reads go out before this k-step's
    // MFMAs and each ring slot's reload right behind them (hipcc otherwise sinks the
    // loads to the end of the loop body and waits on the reads right after issuing them)
    read_a(g + 1, a1h, a1l);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0h, a0l, b0h, b0l);
    wload(g + 2, b0h, b0l);
    __builtin_amdgcn_sched_barrier(0);
    if (g + 2 < G::KS) read_a(g + 2, a0h, a0l);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1h, a1l, b1h, b1l);
    wload(g + 3, b1h, b1l);
    __builtin_amdgcn_sched_barrier(0);
  }

  // ---- epilogue (conv_gemm_x3's: y = act(acc + bias (+ res)) * scale + shift)
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out + ubase);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc((RES ? p.res : p.out) + ubase);
  const int f = f0 + lf;
  const int tw = t0 + lt0 + 4 * h;  // time of register 0
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = (wn * TN + j) * 32 + r32;
    const float bv = p.bias ? p.bias[col] : 0.f;
    const float sc = p.scale ? p.scale[col] : 1.f;
    const float sh = p.scale ? p.shift[col] : 0.f;
    float rv[16];
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = tw + (r & 3) + 8 * (r >> 2);
        rv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rr, f < p.F && t < p.T ? ((f * p.T + t) * C + col) * 4 : kOOB, 0, 0));
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = tw + (r & 3) + 8 * (r >> 2);
      float y = acc[j][r] + bv;
      if constexpr (RES) y += rv[r];
      if constexpr (RELU) y = fmaxf(y, 0.f);
      y = y * sc + sh;
      const bool ok = f < p.F && t < p.T;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro,
                                            ok ? ((f * p.T + t) * C + col) * 4 : kOOB, 0, 0);
    }
  }
}

// Bottleneck tail (resnet.py:101-107, stride 1) in one launch:
//   y2 = relu(conv2_3x3(y1) + b2),  out = relu(conv3_1x1(y2) + b3 + res)
// Phase 1 is conv3x3_img's k-loop with the MFMA operands swapped (A = the W2
// fragments, B = the image rows), so the accumulators hold y2 TRANSPOSED: lane l
// = position l & 31 of the wave's run, register r of channel tile j = channel
// 32 j + (r & 3) + 8 (r >> 2) + 4 (l >> 5).  That is an MFMA A-operand layout (row =
// lane & 31, eight k slots per lane half) with the k slots permuted: after bias +
// ReLU and the hi / lo split the registers ARE conv3's A fragments, and the
// permutation is absorbed by packing W3's k in the same order (pack_frag_acc).
// WN = 2 (C = 128): two waves share a 32-position run, each computing half of
// conv2's channels (8 waves: two per SIMD); they swap their y2 fragments through
// LDS (8 KB per wave, the image's space once conv2 is done) and each runs conv3 for
// half of the 4C output columns over all C input channels.
// Phase 2 runs conv3 over the wave's output columns in chunks of NC column tiles
// (W3 fragments from L1 / L2 two k-steps ahead, the chunk's residual loaded before
// its k-loop), then b3 + residual, ReLU, store.  y2 never exists in memory: per
// position the HBM traffic is y1 (halo re-reads mostly L2 hits) + res + out instead
// of conv2's y1 + y2 and conv3's y2 + res + out.
template <int C, int FB, int TB, int WN, int MINB, int NC, int P1, int PM>
__global__ __launch_bounds__(FB* TB * 2 * WN, MINB) void bottleneck_tail_kernel(const BottleneckTailArgs p) {
  using G = Img<C, FB, TB, WN>;
  constexpr int TN = G::TN, PT = G::PT;
  constexpr int C4 = 4 * C, NT3 = C4 / 32, KS3 = C / 16;
  constexpr int NTW = NT3 / WN, NCH = NTW / NC;  // conv3 column tiles per wave, chunks
  static_assert(NTW % NC == 0 && KS3 % 2 == 0, "bottleneck_tail chunks");
  static_assert(WN == 1 || G::IR * G::RB * 2 >= G::NW / WN * KS3 * 2048, "y2 exchange must fit the image");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int ntf = (p.F + FB - 1) / FB, ntt = (p.T + TB - 1) / TB;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int b = id / (ntf * ntt);
  const int rem = id - b * (ntf * ntt);
  const int tf = rem / ntt;
  const int f0 = tf * FB, t0 = (rem - tf * ntt) * TB;
  const size_t plane = (size_t)p.F * p.T;
  stage_patch<G>(make_rsrc(p.y1 + (size_t)b * plane * C), p.F, p.T, f0, t0, tid, xhi, xlo);

  const int pr = wave / WN, wn = wave - pr * WN;  // phase-2 position run, column half
  const int lf = pr / (TB / 32);
  const int lt0 = (pr % (TB / 32)) * 32;

  // ---- phase 1: conv2, transposed accumulators.  PM = 1: the wave's own position run
  // and its phase-2 channel half (TN tiles).  PM = 2: two position runs x TNP channel
  // tiles per wave, so each W2 fragment fetched feeds two MFMA triples (half the vector
  // memory instructions per MFMA; the y2 tiles are then regrouped through LDS).
  constexpr int NR = FB * TB / 32;                              // position runs
  constexpr int TNP = PM == 1 ? TN : G::CT * NR / (PM * G::NW);  // phase-1 channel tiles per wave
  constexpr int NCG = G::CT / TNP;                              // phase-1 channel groups
  static_assert(PM == 1 || (PM == 2 && NR % 2 == 0 && TNP >= 1 && (NR / PM) * NCG == G::NW),
                "bottleneck_tail: phase-1 wave layout");
  const int pg = wave / NCG, cg = wave - pg * NCG;  // PM = 1: pg = pr, cg = wn
  int prow[PM];
#pragma unroll
  for (int i = 0; i < PM; ++i) {
    const int run = pg * PM + i;
    prow[i] = (run / (TB / 32)) * PT + (run % (TB / 32)) * 32 + r32;
  }
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w2);
  auto wload = [&](int g, bf16x8 (&bh)[TNP], bf16x8 (&bl)[TNP]) {
    const bool ok = g < G::KS;
#pragma unroll
    for (int j = 0; j < TNP; ++j) {
      const int o = ((g * 2 * G::CT + cg * TNP + j) * 64 + lane) * 16;
      bh[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o : kOOB, 0, 0));
      bl[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o + G::CT * 1024 : kOOB, 0, 0));
    }
  };
  auto read_b = [&](int g, bf16x8 (&xh)[PM], bf16x8 (&xl)[PM]) {
    const int tap = g / G::KC, cb = g - tap * G::KC;
    const int kf = tap / 3, kt = tap - kf * 3;
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const int a = G::addr(prow[i] + kf * PT + kt, 2 * cb + h);
      xh[i] = *reinterpret_cast<const bf16x8*>(xhi + a);
      xl[i] = *reinterpret_cast<const bf16x8*>(xlo + a);
    }
  };
  f32x16 acc[PM][TNP];
#pragma unroll
  for (int i = 0; i < PM; ++i)
#pragma unroll
    for (int j = 0; j < TNP; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto mma_t = [&](const bf16x8 (&xh)[PM], const bf16x8 (&xl)[PM], const bf16x8 (&bh)[TNP],
                   const bf16x8 (&bl)[TNP]) {
#pragma unroll
    for (int i = 0; i < PM; ++i)
#pragma unroll
      for (int j = 0; j < TNP; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[j], xl[i], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl[j], xh[i], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh[j], xh[i], acc[i][j], 0, 0, 0);
      }
  };
  {
    // W2 fragments of k-step g in ring slot g % P1 (P1 k-steps in flight: phase 1's live
    // registers are few, so the ring can be deeper than the phase 2 rings)
    static_assert(P1 % 2 == 0 && G::KS % P1 == 0, "bottleneck_tail: W2 prefetch depth");
    bf16x8 wh[P1][TNP], wl[P1][TNP], xh[2][PM], xl[2][PM];
#pragma unroll
    for (int d = 0; d < P1; ++d) wload(d, wh[d], wl[d]);
    __syncthreads();  // image complete
    read_b(0, xh[0], xl[0]);
#pragma unroll 1
    for (int g = 0; g < G::KS; g += P1) {
#pragma unroll
      for (int u = 0; u < P1; ++u) {
        // fences as in conv3x3_img_kernel: reads one k-step ahead, reloads behind their MFMAs
        if (u + 1 < P1 || g + P1 < G::KS) read_b(g + u + 1, xh[(u + 1) & 1], xl[(u + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mma_t(xh[u & 1], xl[u & 1], wh[u], wl[u]);
        wload(g + u + P1, wh[u], wl[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- phase 2 operands: W3 fragments g = chunk * KS3 + ks of this wave's columns,
  // the first two issued before the y2 conversion
  const __amdgpu_buffer_rsrc_t rw3 = make_rsrc(p.w3);
  auto w3load = [&](int g, bf16x8 (&bh)[NC], bf16x8 (&bl)[NC]) {
    const bool ok = g < NCH * KS3;
    const int ch = g / KS3, ks = g - ch * KS3;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int o = ((ks * 2 * NT3 + wn * NTW + ch * NC + j) * 64 + lane) * 16;
      bh[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw3, ok ? o : kOOB, 0, 0));
      bl[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw3, ok ? o + NT3 * 1024 : kOOB, 0, 0));
    }
  };
  // slot q of the y2 fragments (below) holds conv3 k-step ksof(q): the wave's own k-steps
  // first, then (WN = 2) the partner's
  // (PM = 2: every slot comes back from LDS in k order)
  auto ksof = [&](int q) {
    return WN == 1 || PM == 2 ? q : (q < 2 * TN ? wn * 2 * TN + q : (1 - wn) * 2 * TN + q - 2 * TN);
  };
  bf16x8 c0h[NC], c0l[NC], c1h[NC], c1l[NC];
  w3load(ksof(0), c0h, c0l);
  w3load(ksof(1), c1h, c1l);

  // ---- y2 = relu(acc + b2) -> conv3's A fragments (k-step 2 jj + s = registers 8 s .. 8 s + 7
  // of channel tile jj)
  bf16x8 yh[KS3], yl[KS3];
  if constexpr (PM == 1) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ch = 32 * (wn * TN + j) + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float y = fmaxf(acc[0][j][r] + p.b2[ch], 0.f);
        const __bf16 hh = (__bf16)y;
        // own k-steps sit at [0, 2 TN) of yh / yl; the partner's (WN = 2) at [2 TN, 4 TN)
        yh[2 * j + (r >> 3)][r & 7] = hh;
        yl[2 * j + (r >> 3)][r & 7] = (__bf16)(y - (float)hh);
      }
    if constexpr (WN == 2) {
      // swap halves with the partner wave through LDS: [run][k-step][plane][64 lanes] x 16 B
      __syncthreads();  // every wave is done reading the image
#pragma unroll
      for (int q = 0; q < 2 * TN; ++q) {
        const int o = ((pr * KS3 + ksof(q)) * 2) * 1024 + lane * 16;
        *reinterpret_cast<bf16x8*>(smem + o) = yh[q];
        *reinterpret_cast<bf16x8*>(smem + o + 1024) = yl[q];
      }
      __syncthreads();
#pragma unroll
      for (int q = 2 * TN; q < KS3; ++q) {
        const int o = ((pr * KS3 + ksof(q)) * 2) * 1024 + lane * 16;
        yh[q] = *reinterpret_cast<const bf16x8*>(smem + o);
        yl[q] = *reinterpret_cast<const bf16x8*>(smem + o + 1024);
      }
    }
  } else {
    // every wave's (run, k-step) fragments -> LDS [run][k-step][plane][64 lanes] x 16 B;
    // each wave then takes its phase-2 run's KS3 k-steps in order
    static_assert(NR * KS3 * 2048 <= G::LDS, "bottleneck_tail: y2 regrouping must fit the image");
    __syncthreads();  // every wave is done reading the image
#pragma unroll
    for (int i = 0; i < PM; ++i)
#pragma unroll
      for (int j = 0; j < TNP; ++j)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 vh, vl;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int r = 8 * s2 + e;
            const int ch = 32 * (cg * TNP + j) + (r & 3) + 8 * (r >> 2) + 4 * h;
            const float y = fmaxf(acc[i][j][r] + p.b2[ch], 0.f);
            const __bf16 hh = (__bf16)y;
            vh[e] = hh;
            vl[e] = (__bf16)(y - (float)hh);
          }
          const int o = (((pg * PM + i) * KS3 + 2 * (cg * TNP + j) + s2) * 2) * 1024 + lane * 16;
          *reinterpret_cast<bf16x8*>(smem + o) = vh;
          *reinterpret_cast<bf16x8*>(smem + o + 1024) = vl;
        }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KS3; ++q) {
      const int o = ((pr * KS3 + q) * 2) * 1024 + lane * 16;
      yh[q] = *reinterpret_cast<const bf16x8*>(smem + o);
      yl[q] = *reinterpret_cast<const bf16x8*>(smem + o + 1024);
    }
  }

  // ---- phase 2: conv3 over NCH chunks of NC column tiles
  const size_t obase = (size_t)b * plane * C4;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out + obase);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.res + obase);
  const int f = f0 + lf;
  const int tw = t0 + lt0 + 4 * h;  // time of register 0
  auto roff = [&](int col, int r) {
    const int t = tw + (r & 3) + 8 * (r >> 2);
    return f < p.F && t < p.T ? ((f * p.T + t) * C4 + col) * 4 : kOOB;
  };
#pragma unroll 1
  for (int chunk = 0; chunk < NCH; ++chunk) {
    const int cb = (wn * NTW + chunk * NC) * 32 + r32;  // column of tile 0
    float rv[NC][16];
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        rv[j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, roff(cb + 32 * j, r), 0, 0));
    f32x16 a3[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) a3[j][r] = 0.f;
    // slots in k order: k-step ks lives in slot q with ksof(q) == ks; summing in slot order
    // is the same sum (the fp32 accumulation order differs from k order only by whole k-steps)
#pragma unroll
    for (int q = 0; q < KS3; q += 2) {
      // W3 fragments were loaded for k-steps ksof(q), ksof(q + 1) (consecutive: own / partner
      // halves are each 2 TN consecutive k-steps and 2 TN is even)
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yl[q], c0h[j], a3[j], 0, 0, 0);
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yh[q], c0l[j], a3[j], 0, 0, 0);
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yh[q], c0h[j], a3[j], 0, 0, 0);
      }
      {
        const int qn = q + 2 < KS3 ? q + 2 : 0;
        w3load((q + 2 < KS3 ? chunk : chunk + 1) * KS3 + ksof(qn), c0h, c0l);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yl[q + 1], c1h[j], a3[j], 0, 0, 0);
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yh[q + 1], c1l[j], a3[j], 0, 0, 0);
        a3[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(yh[q + 1], c1h[j], a3[j], 0, 0, 0);
      }
      {
        const int qn = q + 3 < KS3 ? q + 3 : 1;
        w3load((q + 3 < KS3 ? chunk : chunk + 1) * KS3 + ksof(qn), c1h, c1l);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue: y = relu(acc + b3 + res), conv3x3_img's store pattern over 4C channels
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int col = cb + 32 * j;
      const float bv = p.b3[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float y = fmaxf(a3[j][r] + bv + rv[j][r], 0.f);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, roff(col, r), 0, 0);
      }
    }
  }
}

// Bottleneck tail with the next conv1 fused, every wave on TWO position runs in both phases
// (option res_tail 1, default, r3; 32 / 64 / 128 planes).  The first fused form (the r3
// bottleneck_tail_kernel with FUSE1, since removed) fetched, per chunk and wave, W3 / W1
// fragments that fed one 32-position run (for 64 planes also conv2's W2); here each of the 4
// waves runs conv2, conv3 and the next conv1 for a PAIR of runs and 1 / GW of the columns, so
// every weight fragment fetched from L2 feeds two MFMA triples.  128 planes: a 2 x 32 tile (one
// run pair, GW = 4 column groups); 64 planes: 4 x 32 (two run pairs, GW = 2); 32 planes: 8 x 32
// (four run pairs, GW = 1).  y2 stays in LDS as MFMA A fragments ([run][k-step][hi, lo][64
// lanes] x 16 B, 32 KB) read per k-step.  Chunk c = conv3 column tiles GW c .. GW c + GW - 1
// (wave (pair, g): tile GW c + g) = the next conv1's k-steps 2 GW c .. 2 GW c + 2 GW - 1; its
// LDS buffer holds those channels for every run.  Issue order keeps HBM latency off the
// critical path: chunk c + 1's residual (and bias) goes out right behind chunk c's last W1 fetch
// (chunk 0's at the start of conv2's last W2 ring group, conv2's bias with the patch), so the
// first wait covering it comes RD3 + RD1 k-steps later (the first form issued the residual at
// the chunk start and waited on it 2 k-steps later, and its epilogue's bias load drained every
// prefetch).  RD3 / RD1: W3 / W1 ring depths.  (Holding the outputs in registers to store them
// later as well spilled; an in-place variant through the accumulators was miscompiled: one
// element stored 16 times.)  Against the first form: C3 ResNet293 1 622 -> 1 732 emb/s
// (interleaved model-level A/B).

// dynamic LDS of tail2_kernel: the patch image, later y2 fragments + the chunk buffer
// FB: position runs (frequency rows) per block — 2 / 4 / 8 for 128 / 64 / 32 planes, or 1 for
// 128 planes (r6: one run per block, 51 KB, three blocks per CU)
template <int C>
constexpr int tail2_fb() { return C == 128 ? 2 : C == 64 ? 4 : 8; }
template <int C, int FB = tail2_fb<C>()>
constexpr int tail2_lds() {
  constexpr int RW = FB >= 2 ? 2 : 1, GW = 4 * RW / FB;
  constexpr int cbp = FB * 32 * GW * 64, need = FB * (C / 16) * 2048 + cbp + 64 + cbp;
  return Img<C, FB, 32>::LDS > need ? Img<C, FB, 32>::LDS : need;
}

// R1: the next conv1's output channels in units of C (2 at a stage transition: wave g computes
// conv1 output tiles g and g + GW).  SCX: the block's projection shortcut (C -> 4C, its input x
// of C channels at the output positions: a stage's stride-1 first block) as KS3 more conv3
// k-steps with x's fragments in registers, instead of a residual read (BottleneckTailArgs::xsc)
template <int C, int P1, int RD3, int RD1, int FB = tail2_fb<C>(), int MINB = 2, int R1 = 1, bool SCX = false>
__global__ __launch_bounds__(256, MINB) void tail2_kernel(const BottleneckTailArgs p) {
  constexpr int TB = 32;
  using G = Img<C, FB, TB, 1, 4>;  // patch image staged by the 4 waves
  constexpr int PT = G::PT, CT = G::CT, KS = G::KS;
  // runs; runs per wave (a pair, or the block's one run); column groups per wave's runs
  constexpr int NR = FB, RW = NR >= 2 ? 2 : 1, GW = 4 * RW / NR;
  constexpr int C4 = 4 * C, NT3 = C4 / 32, KS3 = C / 16, NT1 = R1 * C / 32, C1N = R1 * C;
  constexpr int KT3 = SCX ? 2 * KS3 : KS3;  // conv3 k-steps: y2, then (SCX) the shortcut's x
  constexpr int NCHK = NT3 / GW, KB = 2 * GW;    // chunks of GW tiles; conv1 k-steps per chunk
  constexpr int Y2B = NR * KS3 * 2048;           // y2 fragments of every run
  constexpr int CBR = GW * 64, CBP = NR * 32 * CBR;  // chunk buffer: NR x 32 rows x GW x 32 bf16 per plane
  constexpr int CBLO = CBP + 64;                 // lo plane 64 B off: paired hi / lo stores, distinct banks
  static_assert(G::NT == 256 && CT == GW && NT1 == R1 * GW && KS % P1 == 0 && P1 % 2 == 0, "tail2: wave layout");
  static_assert(KS3 % RD3 == 0 && KT3 % RD3 == 0 && RD1 >= 1 && RD1 + 1 <= KB, "tail2: ring depths");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;
  unsigned char* y2s = smem;
  unsigned char* cbhi = smem + Y2B;
  unsigned char* cblo = cbhi + CBLO;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int pp = w / GW, g = w - pp * GW;  // run group (runs RW pp .. RW pp + RW - 1), column group
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int ntf = (p.F + FB - 1) / FB, ntt = (p.T + TB - 1) / TB;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int b = id / (ntf * ntt);
  const int rem = id - b * (ntf * ntt);
  const int tf = rem / ntt;
  const int f0 = tf * FB, t0 = (rem - tf * ntt) * TB;
  const size_t plane = (size_t)p.F * p.T;
  WSP_TAIL_STAMP(0);
  // conv2 bias of this lane's y2 registers, fetched before the patch (waited on with it, not
  // in the y2 conversion, where the wait would also cover chunk 0's residual)
  float b2v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) b2v[r] = p.b2[32 * g + (r & 3) + 8 * (r >> 2) + 4 * h];
  stage_patch<G>(make_rsrc(p.y1 + (size_t)b * plane * C), p.F, p.T, f0, t0, tid, xhi, xlo);

  // residual of chunk c, this wave's runs (run 2 pp + i = frequency row f0 + 2 pp + i) and tile
  const size_t obase = (size_t)b * plane * C4;
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out + obase);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.res + obase);
  const int tw = t0 + 4 * h;  // time of register 0
  const int fw = f0 + RW * pp;  // frequency row of the wave's first run
  // register r holds time tw + tro(r): inside the utterance iff tro(r) < T - tw.  Run i's limit
  // folds its frequency-row test (and a dead load's) into that one compare, so every offset is a
  // compare + select: the nested conditional form compiled to exec-mask branches (and predicate
  // spills to VGPR lanes) around each of the 32 residual loads inside conv1's MFMA stream
  auto tro = [](int r) { return (r & 3) + 8 * (r >> 2); };
  auto rlim = [&](int i, bool live) { return live && fw + i < p.F ? p.T - tw : 0; };
  auto roff = [&](int i, int col, int r, int lim) {
    const unsigned o = (((unsigned)(fw + i) * p.T + tw + tro(r)) * C4 + col) * 4;
    return tro(r) < lim ? (int)o : kOOB;
  };
  float rv[RW][16], b3v;
  const __amdgpu_buffer_rsrc_t rb3 = make_rsrc(p.b3);
  auto rload = [&](int c, bool live) {  // !live: the same loads, out of range (branch-free count)
    const int col = (GW * c + g) * 32 + r32;
    b3v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb3, live ? col * 4 : kOOB, 0, 0));
    if constexpr (!SCX) {
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int lim = rlim(i, live);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          rv[i][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, roff(i, col, r, lim), 0, 0));
      }
    }
  };

  // ---- phase 1: conv2 for the wave's two runs, channel tile g; transposed accumulators
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w2);
  auto wload = [&](int kg, bf16x8& bh, bf16x8& bl) {
    const int o = ((kg * 2 * CT + g) * 64 + lane) * 16;
    bh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, o, 0, 0));
    bl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, o + CT * 1024, 0, 0));
  };
  auto read_b = [&](int kg, bf16x8 (&xh)[RW], bf16x8 (&xl)[RW]) {
    const int tap = kg / G::KC, cb = kg - tap * G::KC;
    const int kf = tap / 3, kt = tap - kf * 3;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int a = G::addr((RW * pp + i) * PT + r32 + kf * PT + kt, 2 * cb + h);
      xh[i] = *reinterpret_cast<const bf16x8*>(xhi + a);
      xl[i] = *reinterpret_cast<const bf16x8*>(xlo + a);
    }
  };
  f32x16 acc[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  auto mma_t = [&](const bf16x8 (&xh)[RW], const bf16x8 (&xl)[RW], const bf16x8& bh, const bf16x8& bl) {
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, xl[i], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bl, xh[i], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bh, xh[i], acc[i], 0, 0, 0);
    }
  };
  {
    bf16x8 wh[P1], wl[P1], xh[2][RW], xl[2][RW];
#pragma unroll
    for (int d = 0; d < P1; ++d) wload(d, wh[d], wl[d]);
    __syncthreads();  // image complete
    WSP_TAIL_STAMP(1);
    read_b(0, xh[0], xl[0]);
#pragma unroll 1
    for (int kg = 0; kg < KS - P1; kg += P1) {
#pragma unroll
      for (int u = 0; u < P1; ++u) {
        read_b(kg + u + 1, xh[(u + 1) & 1], xl[(u + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mma_t(xh[u & 1], xl[u & 1], wh[u], wl[u]);
        wload(kg + u + P1, wh[u], wl[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // last ring group: no reloads; chunk 0's residual goes out in their place
    rload(0, true);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < P1; ++u) {
      if (u + 1 < P1) read_b(KS - P1 + u + 1, xh[(u + 1) & 1], xl[(u + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      mma_t(xh[u & 1], xl[u & 1], wh[u], wl[u]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  WSP_TAIL_STAMP(2);
  // ---- phase 2 weights: W3 B fragments [ks][hi, lo][NT3][64][8] (pack_frag_acc k order),
  // W1' [ks][hi, lo][NT1][64][8]
  const __amdgpu_buffer_rsrc_t rw3 = make_rsrc(p.w3);
  const __amdgpu_buffer_rsrc_t rw1 = make_rsrc(p.w1n);
  auto w3load = [&](int c, int ks, bf16x8& bh, bf16x8& bl) {  // c == NCHK: past the end (zeros)
    const int o = ((ks * 2 * NT3 + GW * c + g) * 64 + lane) * 16;
    bh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw3, c < NCHK ? o : kOOB, 0, 0));
    bl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw3, c < NCHK ? o + NT3 * 1024 : kOOB, 0, 0));
  };
  auto w1load = [&](int ks, int j, bf16x8& bh, bf16x8& bl) {  // conv1 output tile g + GW j
    const int o = ((ks * 2 * NT1 + g + GW * j) * 64 + lane) * 16;
    bh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw1, o, 0, 0));
    bl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw1, o + NT1 * 1024, 0, 0));
  };
  // W3 / W1 rings (slot j = k-step j mod RD3 / RD1); chunk 0's first RD3 W3 k-steps go out
  // before the y2 conversion
  bf16x8 ch_[RD3], cl_[RD3], uh_[RD1][R1], ul_[RD1][R1];
#pragma unroll
  for (int j = 0; j < RD3; ++j) w3load(0, j, ch_[j], cl_[j]);
  // SCX: the shortcut input's A fragments, natural k order (lane: position t0 + r32 of run i,
  // channels 16 ks + 8 h .. + 7), split into bf16 hi / lo once for every chunk
  bf16x8 xsh[SCX ? KS3 : 1][RW], xsl[SCX ? KS3 : 1][RW];
  if constexpr (SCX) {
    const __amdgpu_buffer_rsrc_t rxs = make_rsrc(p.xsc + (size_t)b * plane * C);
#pragma unroll
    for (int ks = 0; ks < KS3; ++ks)
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const bool ok = fw + i < p.F && t0 + r32 < p.T;
        const unsigned o = (((unsigned)(fw + i) * p.T + t0 + r32) * C + 16 * ks + 8 * h) * 4;
        const f32x4 v0 = bload4(rxs, ok ? (int)o : kOOB), v1 = bload4(rxs, ok ? (int)(o + 16) : kOOB);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __bf16 h0 = (__bf16)v0[e], h1 = (__bf16)v1[e];
          xsh[ks][i][e] = h0;
          xsh[ks][i][4 + e] = h1;
          xsl[ks][i][e] = (__bf16)(v0[e] - (float)h0);
          xsl[ks][i][4 + e] = (__bf16)(v1[e] - (float)h1);
        }
      }
  }

  // ---- y2 = relu(acc + b2) -> LDS fragments [run][k-step][hi, lo][lane] (k-step 2 g + s2 =
  // registers 8 s2 .. 8 s2 + 7 of channel tile g)
  __syncthreads();  // every wave is done reading the image
#pragma unroll
  for (int i = 0; i < RW; ++i)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 vh, vl;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int r = 8 * s2 + e;
        const float y = fmaxf(acc[i][r] + b2v[r], 0.f);
        const __bf16 hh = (__bf16)y;
        vh[e] = hh;
        vl[e] = (__bf16)(y - (float)hh);
      }
      const int o = (((RW * pp + i) * KS3 + 2 * g + s2) * 2) * 1024 + lane * 16;
      *reinterpret_cast<bf16x8*>(y2s + o) = vh;
      *reinterpret_cast<bf16x8*>(y2s + o + 1024) = vl;
    }
  // GW = 1 (32 planes): a wave reads back only the y2 / chunk-buffer rows of its own runs, so
  // ordering its own LDS accesses replaces the workgroup barriers
  auto sync = [] {
    if constexpr (GW > 1) {
      __syncthreads();
    } else {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  };
  sync();
  WSP_TAIL_STAMP(3);

  auto read_y2 = [&](int ks, bf16x8 (&ah)[RW], bf16x8 (&al)[RW]) {
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int o = (((RW * pp + i) * KS3 + ks) * 2) * 1024 + lane * 16;
      ah[i] = *reinterpret_cast<const bf16x8*>(y2s + o);
      al[i] = *reinterpret_cast<const bf16x8*>(y2s + o + 1024);
    }
  };
  // 16-B chunks XOR-swizzled by row as Img's (256-B rows: row & 15; 128-B: (row >> 1) & 7; 64-B:
  // (row >> 2) & 3)
  auto cbaddr = [](int row, int c16) {
    return row * CBR + ((c16 ^ (CBR == 256 ? row & 15 : CBR == 128 ? (row >> 1) & 7 : (row >> 2) & 3)) << 4);
  };
  auto read_cb = [&](int kk, bf16x8 (&ah)[RW], bf16x8 (&al)[RW]) {
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      const int a = cbaddr((RW * pp + i) * 32 + r32, 2 * kk + h);
      ah[i] = *reinterpret_cast<const bf16x8*>(cbhi + a);
      al[i] = *reinterpret_cast<const bf16x8*>(cblo + a);
    }
  };
  auto mma2 = [](f32x16 (&d)[RW], const bf16x8 (&ah)[RW], const bf16x8 (&al)[RW], const bf16x8& bh,
                 const bf16x8& bl) {
#pragma unroll
    for (int i = 0; i < RW; ++i) {
      d[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, d[i], 0, 0, 0);
      d[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh, d[i], 0, 0, 0);
    }
  };

  f32x16 acc1[R1][RW], a3[RW];
#pragma unroll
  for (int j = 0; j < R1; ++j)
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[j][i][r] = 0.f;
#pragma unroll 1
  for (int c = 0; c < NCHK; ++c) {
#pragma unroll
    for (int j = 0; j < RD1; ++j)  // land during the chunk's conv3
#pragma unroll
      for (int u = 0; u < R1; ++u) w1load(KB * c + j, u, uh_[j][u], ul_[j][u]);
    // conv3, column tile GW c + g, the wave's two runs
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) a3[i][r] = 0.f;
    bf16x8 ah[2][RW], al[2][RW];
    read_y2(0, ah[0], al[0]);
#pragma unroll
    for (int q = 0; q < KT3; ++q) {
      if (q + 1 < KS3) read_y2(q + 1, ah[(q + 1) & 1], al[(q + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (q < KS3)
        mma2(a3, ah[q & 1], al[q & 1], ch_[q % RD3], cl_[q % RD3]);
      else
        mma2(a3, xsh[q < KS3 ? 0 : q - KS3], xsl[q < KS3 ? 0 : q - KS3], ch_[q % RD3], cl_[q % RD3]);
      if (q + RD3 < KT3) w3load(c, q + RD3, ch_[q % RD3], cl_[q % RD3]);
      else w3load(c + 1, q + RD3 - KT3, ch_[q % RD3], cl_[q % RD3]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c == 1) WSP_TAIL_STAMP(8);
    if (c > 0) sync();  // every wave is done reading chunk c - 1 from the buffer
    if (c == 1) WSP_TAIL_STAMP(9);
    // epilogue: out = relu(a3 + b3 + res) -> HBM and as bf16 hi / lo rows of the chunk buffer.
    // The first wait covering these stores is the one on the W1 fetch that conv1's k-step 0
    // issues after them, RD1 k-steps later (stores count in vmcnt like loads)
    {
      const int col = (GW * c + g) * 32 + r32;
      const bool odd = lane & 1;
      const int cbsel = odd ? CBLO : 0, ksh = odd ? 16 : 0;  // plane; this lane's own half in the word
      const int cc = g * 32 + (r32 & ~1);
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int lim = rlim(i, true);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float y = SCX ? fmaxf(a3[i][r] + b3v, 0.f) : fmaxf(a3[i][r] + b3v + rv[i][r], 0.f);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, roff(i, col, r, lim), 0, 0);
          // lanes l, l ^ 1 hold columns c, c ^ 1: the even lane stores both hi halves, the odd
          // lane both lo halves — one 4-B store per lane at a lane-parity plane offset, the word
          // assembled by shifts (an if / else on the parity compiled to two half-masked stores
          // and exec-mask branches per element)
          const __bf16 hh = (__bf16)y;
          const __bf16 ll = (__bf16)(y - (float)hh);
          const unsigned hb = __builtin_bit_cast(unsigned short, hh);
          const unsigned lb = __builtin_bit_cast(unsigned short, ll);
          const unsigned send = odd ? hb : lb;
          const unsigned recv = (unsigned)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);
          const int row = (RW * pp + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int a = cbaddr(row, cc >> 3) + (cc & 7) * 2;
          *reinterpret_cast<unsigned*>(cbhi + cbsel + a) = ((odd ? lb : hb) << ksh) | (recv << (16 - ksh));
        }
      }
    }
    if (c == 1) WSP_TAIL_STAMP(10);
    sync();  // the chunk's GW x 32 channels of every run are in LDS
    if (c == 1) WSP_TAIL_STAMP(11);
    // next conv1: k-steps KB c .. KB c + KB - 1, output tile g, the wave's two runs
    read_cb(0, ah[0], al[0]);
#pragma unroll
    for (int kk = 0; kk < KB; ++kk) {
      if (kk + 1 < KB) read_cb(kk + 1, ah[(kk + 1) & 1], al[(kk + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < R1; ++u) mma2(acc1[u], ah[kk & 1], al[kk & 1], uh_[kk % RD1][u], ul_[kk % RD1][u]);
#pragma unroll
      for (int u = 0; u < R1; ++u)
        if (kk + RD1 < KB) w1load(KB * c + kk + RD1, u, uh_[kk % RD1][u], ul_[kk % RD1][u]);
      if (kk + RD1 + 1 == KB) rload(c + 1, c + 1 < NCHK);  // right behind the chunk's last W1 fetch
      __builtin_amdgcn_sched_barrier(0);
    }
    WSP_TAIL_STAMP(4 + c);
  }
  // y1' = relu(acc1 + b1') -> y1n [B][F][T][C1N], output tiles g + GW j
  {
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y1n + (size_t)b * plane * C1N);
#pragma unroll
    for (int u = 0; u < R1; ++u) {
      const int col = (g + GW * u) * 32 + r32;
      const float bv = p.b1n[col];
#pragma unroll
      for (int i = 0; i < RW; ++i) {
        const int lim = rlim(i, true);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float y = fmaxf(acc1[u][i][r] + bv, 0.f);
          const unsigned o = (((unsigned)(fw + i) * p.T + tw + tro(r)) * C1N + col) * 4;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ry, tro(r) < lim ? (int)o : kOOB, 0, 0);
        }
      }
    }
  }
  WSP_TAIL_STAMP(15);
}

template <int C, int FB, int TB, int MINB, int WN = 1>
void launch_k(const Conv3x3Args& p, hipStream_t s) {
  using G = Img<C, FB, TB, WN>;
  const int nblk = p.B * ((p.F + FB - 1) / FB) * ((p.T + TB - 1) / TB);
  if (p.res)
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, true, true>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
  else if (p.relu)
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, false, true>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
  else
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, false, false>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
}

}  // namespace

bool conv3x3_img_supported(int C) { return C == 32 || C == 64 || C == 128; }

void launch_conv3x3_img(const Conv3x3Args& p, int C, hipStream_t s) {
  WSP_CHECK(conv3x3_img_supported(C), "conv3x3_img: channels must be 32, 64 or 128");
  WSP_CHECK(p.B > 0 && p.F > 0 && p.T > 0 && p.x && p.out && p.w, "conv3x3_img: bad arguments");
  WSP_CHECK(p.relu || !p.res, "conv3x3_img: a residual comes with the ReLU");
  // buffer offsets are per utterance (descriptors based at its first element)
  WSP_CHECK((long long)p.F * p.T * C * 4 < (long long)kOOB, "conv3x3_img: utterance exceeds 2 GiB");
  if (C == 32)
    launch_k<32, 4, 64, 3>(p, s);  // 256 positions, 8 waves, 50 KB image: 3 blocks / CU
  else if (C == 64)
    launch_k<64, 4, 32, 3>(p, s);  // 128 positions, 4 waves x 2 column tiles, 51 KB image
  else if (p.variant == 3)
    launch_k<128, 4, 32, 1, 2>(p, s);  // 128 positions, 8 waves x 2 column tiles, 102 KB image
  else
    launch_k<128, 4, 32, 1>(p, s);  // 128 positions, 4 waves x 4 column tiles, 102 KB image
  WSP_HIP(hipGetLastError());
}

namespace {
template <int C, int FB, int TB, int WN, int MINB, int NC, int PM = 1>
void launch_tail_k(const BottleneckTailArgs& p, hipStream_t s) {
  using G = Img<C, FB, TB, WN>;
  // W2 k-steps in flight in phase 1: 4 where the register budget (MINB) leaves room
  constexpr int P1 = G::KS % 4 == 0 && MINB <= 2 ? 4 : 2;
  const int nblk = p.B * ((p.F + FB - 1) / FB) * ((p.T + TB - 1) / TB);
  hipLaunchKernelGGL((bottleneck_tail_kernel<C, FB, TB, WN, MINB, NC, P1, PM>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
}

template <int C, int P1, int RD3, int RD1, int FB = tail2_fb<C>(), int MINB = 2, int R1 = 1, bool SCX = false>
void launch_tail2(const BottleneckTailArgs& p, hipStream_t s) {
  const int nblk = p.B * ((p.F + FB - 1) / FB) * ((p.T + 31) / 32);
  hipLaunchKernelGGL((tail2_kernel<C, P1, RD3, RD1, FB, MINB, R1, SCX>), dim3(nblk), dim3(256), (tail2_lds<C, FB>()),
                     s, p);
}
}  // namespace

bool bottleneck_tail_supported(int C) { return C == 32 || C == 64 || C == 128; }

void launch_bottleneck_tail(const BottleneckTailArgs& p, int C, hipStream_t s) {
  WSP_CHECK(bottleneck_tail_supported(C), "bottleneck_tail: planes must be 32, 64 or 128");
  WSP_CHECK(p.B > 0 && p.F > 0 && p.T > 0 && p.y1 && (p.res || p.xsc) && p.out && p.w2 && p.w3 && p.b2 && p.b3,
            "bottleneck_tail: bad arguments");
  WSP_CHECK(p.out != p.res && p.out != p.y1, "bottleneck_tail: out must not alias its inputs");
  // buffer offsets are per utterance (descriptors based at its first element)
  WSP_CHECK((long long)p.F * p.T * 4 * C * 4 < (long long)kOOB, "bottleneck_tail: utterance exceeds 2 GiB");
  WSP_CHECK(!p.w1n || (p.b1n && p.y1n && p.y1n != p.out && p.y1n != p.y1 && p.y1n != p.res),
            "bottleneck_tail: next conv1 needs bias and a separate output");
  WSP_CHECK(p.c1n == 0 || p.c1n == C || (p.c1n == 2 * C && p.w1n && C <= 64),
            "bottleneck_tail: the next conv1 is C -> C, or C -> 2C with 32 / 64 planes");
  WSP_CHECK(!p.xsc || (C == 32 && p.w1n && !p.res && (p.c1n == 0 || p.c1n == C) && p.xsc != p.out),
            "bottleneck_tail: the in-tail shortcut needs 32 planes, the fused next conv1 and no residual");
  if (p.w1n) {  // with the next block's conv1: every wave on two position runs (tail2_kernel)
    // <C, W2 ring depth, W3 ring, W1 ring>; 128 planes with an 8-deep W2 ring: 0.323 -> 0.314 ms
    // per launch (tools/tail_check, B = 64, interleaved rounds); deeper W2 / W1 rings for 32 / 64
    // planes measured within 0.5 %
    const bool wide = p.c1n == 2 * C;  // stage transition: the next conv1 is 4C -> 2C
    if (p.xsc)  // the stage's stride-1 first block with its shortcut inside conv3 (32 planes)
      launch_tail2<32, 2, 2, 1, tail2_fb<32>(), 2, 1, true>(p, s);
    else if (C == 32 && wide)
      launch_tail2<32, 2, 2, 1, tail2_fb<32>(), 2, 2>(p, s);
    else if (C == 32)
      launch_tail2<32, 2, 2, 1>(p, s);  // 8 x 32 positions, 4 waves, 64 KB: 2 blocks / CU
    else if (C == 64 && wide)
      launch_tail2<64, 4, 4, 2, tail2_fb<64>(), 2, 2>(p, s);
    else if (C == 64)
      launch_tail2<64, 4, 4, 2>(p, s);  // 4 x 32 positions, 64 KB
    else
      launch_tail2<128, 8, 4, 4>(p, s);  // 2 x 32 positions, 68 KB
  } else if (C == 32) {  // <C, FB, TB, WN, MINB, NC[, PM]>
    launch_tail_k<32, 4, 64, 1, 4, 1>(p, s);  // 256 positions, 8 waves, 50 KB image: 2 blocks / CU
  } else if (C == 64) {  // (a 2 x 32 tile: C3 -1.3 %)
    launch_tail_k<64, 4, 32, 1, 3, 2>(p, s);  // 128 positions, 4 waves, 51 KB image: 3 blocks / CU
  } else {
    launch_tail_k<128, 4, 32, 2, 2, 2, 2>(p, s);  // 128 positions, 8 waves (2 per position run), 102 KB image
  }
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
