// Res2Net dilated-k3 chain of one SE_Res2Block in ONE launch (bf16x3 MFMA).
//
// Reference: Res2Conv1dReluBn.forward, ecapa_tdnn.py:64-78 —
//   spx = split(x, w);  for i < 7: sp = spx[i] if i == 0 else sp + spx[i]
//                                  sp = BN_i(ReLU(Conv1d_i(sp)))   (k3, dilation d, pad d)
//   out = cat(sp_0 .. sp_6, spx[7])
// The 7 convs form a serial chain whose every step reads the previous step's
// output: run as 7 GEMM launches, each step round-trips HBM (read sp + spx[i],
// write sp).  Here a block owns `rout` output rows and keeps the chain on chip:
//   * a window of R = 128 frame rows (the owned rows plus a 6d halo on each
//     side) is the GEMM's M; step i is valid on window rows [i*d, kR - i*d)
//     (the conv's +-d taps lose d rows per side per step), so after 7 steps the
//     owned rows [6d, kR - 6d) are exact — halo recomputation instead of a
//     cross-block exchange;
//   * the conv input X_i = sp_{i-1} + spx[i] lives in LDS as bf16 hi / lo planes
//     (x = hi + lo, the bf16x3 split of conv_gemm_x3.hip), rows XOR-swizzled by
//     16-B chunk so the A-fragment ds_read_b128s are conflict-free; the k3 taps
//     are row offsets into that image, and a tap that leaves its utterance reads
//     a zero row (the reference's zero padding, per utterance of a ragged batch);
//   * the step's epilogue (bias, ReLU, BN) stores the owned rows of sp_i to
//     out[:, i*w ..] and writes X_{i+1} = sp_i + spx[i+1] (fp32 add, then split)
//     back into the image;
//   * W_i is host-packed in MFMA B-fragment order, so each wave reads its
//     fragments straight from global memory (1 KB contiguous per instruction,
//     L1/L2-resident, two k-steps ahead in registers): the X image is the only
//     LDS operand, constant during a step, and the k-loop has no barrier;
//   * 128-row windows (70 KB of LDS) run two blocks per CU, so one block's
//     epilogue (addend loads, stores, image update) overlaps the other's MFMA
//     loop.  Default: 8 waves of 64 rows x 32 channels (res2_variant 3; C2
//     1.63 -> 1.45 ms/step over 4 waves of 64 x 64).  Measured and dropped (r3):
//     256-row windows (half the halo rows, one block per CU: 1.57 ms/step even
//     with 4 W k-steps in flight).  Ablations of variant 3 (ms per launch, 0.486):
//     no W reloads 0.416, no addend loads 0.422, no sp stores 0.446 — no single
//     term dominates; the rest is the per-step barriers and image rewrite.
// HBM traffic per row: spx[0..6] read once (+ halo re-reads, mostly L2 hits of
// the neighbouring block) and sp_0..6 written once.
#include <algorithm>
#include <type_traits>

#include "gemm_common.h"
#include "res2_chain.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kPad = 4;  // image rows beyond each window edge (max dilation)

template <int W, int R, int WNv, int NWv = R / 32>
struct Geo {
  static constexpr int IR = R + 2 * kPad;          // image rows; row IR is the zero row
  static constexpr int RB = 2 * W;                 // bytes per image row and plane
  static constexpr int PLANE = (IR + 1) * RB;      // + the zero row
  static constexpr int KS = 3 * W / 16;            // 16-deep MFMA k-steps per conv (K = 3W)
  static constexpr int KC = W / 16;                // k-steps per tap
  static constexpr int WST = 64 * W;               // one k-step of W: W cols x 16 k x (hi, lo) bf16
  static constexpr int NW = NWv;                   // waves: R / 32 (4 for R = 128, 8 for 256), or 8 at R = 128
  static constexpr int WN = WNv, WM = NW / WN, TM = R / 32 / WM, TN = W / 32 / WN;
  static_assert(TN >= 1 && TM >= 1, "res2 wave layout");
  static constexpr int NT = NW * 64;
  static constexpr int LDS = 2 * PLANE;
  // 16-B chunk swizzle: the 16 rows of a ds_read_b128 lane group land on 16
  // distinct chunk slots of the 256-B bank row
  __device__ __forceinline__ static int sw(int ir) { return W == 128 ? (ir & 15) : ((ir >> 1) & 7); }
  __device__ __forceinline__ static int addr(int ir, int ch) {
    return ir * RB + (((ch >> 3) ^ sw(ir)) << 4) + (ch & 7) * 2;
  }
};

__device__ __forceinline__ unsigned short bf_bits(__bf16 x) { return __builtin_bit_cast(unsigned short, x); }

template <int W, int R, int WNv, int NWv, int PD>
__global__ __launch_bounds__(NWv * 64, R == 128 ? NWv / 2 : 1) void res2_chain_kernel(const Res2Args p) {
  using G = Geo<W, R, WNv, NWv>;
  constexpr int TM = G::TM, TN = G::TN, NT = G::NT, IR = G::IR;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / G::WN;
  const int wn = wave - wm * G::WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int d = p.dil;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring windows share an XCD L2 (halo rows)
  const int own0 = blk * p.rout;
  const int own1 = min(own0 + p.rout, p.M);
  const int wr0 = own0 - 6 * d;  // window row 0

  // ---- zero row + X_0 = spx[0] on image rows [0, IR) (window rows -kPad .. R + kPad)
  if (tid < G::RB / 4) {
    reinterpret_cast<unsigned*>(xhi + IR * G::RB)[tid] = 0u;
    reinterpret_cast<unsigned*>(xlo + IR * G::RB)[tid] = 0u;
  }
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x);
  constexpr int C4 = W / 4;
  for (int q = tid; q < IR * C4; q += NT) {
    const int ir = q / C4;
    const int c = (q - ir * C4) * 4;
    const int m = wr0 + ir - kPad;
    const f32x4 v = bload4(rx, (m >= 0 && m < p.M) ? (m * p.ldx + c) * 4 : kOOB);
    bf16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const __bf16 hh = (__bf16)v[e];
      hi[e] = hh;
      lo[e] = (__bf16)(v[e] - (float)hh);
    }
    const int a = G::addr(ir, c);
    *reinterpret_cast<bf16x4*>(xhi + a) = hi;
    *reinterpret_cast<bf16x4*>(xlo + a) = lo;
  }

  // ---- A-fragment rows: this lane's window row per tile, per tap (or the zero row)
  int arow[TM][3], asw[TM][3];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = (wm * TM + i) * 32 + r32;
    const int m = wr0 + r;
    int t = -1, L = 0;
    if (m >= 0 && m < p.M) {
      if (p.seg) {
        const int u = seg_of(p.seg, p.nseg, m);
        t = m - p.seg[u];
        L = p.seg[u + 1] - p.seg[u];
      } else {
        const int u = m / p.T;
        t = m - u * p.T;
        L = p.T;
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int off = (j - 1) * d;
      const bool ok = t >= 0 && t + off >= 0 && t + off < L;
      const int ir = ok ? r + off + kPad : IR;
      arow[i][j] = ir * G::RB;
      asw[i][j] = G::sw(ir);
    }
  }

  // ---- W fragments from global: k-step g, plane pl, column tile ct at
  // ((g * 2 + pl) * (W / 32) + ct) * 1 KB + lane * 16
  constexpr int kTotal = 7 * G::KS;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  const int wlane = (wn * TN * 64 + lane) * 16;
  auto wload = [&](int g, bf16x8 (&bh)[TN], bf16x8 (&bl)[TN]) {
    const bool ok = g < kTotal;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = (g * 2 * (W / 32) + j) * 1024 + wlane;
      bh[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o : kOOB, 0, 0));
      bl[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o + (W / 32) * 1024 : kOOB, 0, 0));
    }
  };
  // W fragments of k-step k in ring slot k % PD (PD k-steps in flight)
  static_assert(PD % 2 == 0 && G::KS % PD == 0, "res2 W prefetch depth");
  bf16x8 wbh[PD][TN], wbl[PD][TN];
#pragma unroll
  for (int d = 0; d < PD; ++d) wload(d, wbh[d], wbl[d]);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rout = make_rsrc(p.out);
  f32x16 acc[TM][TN];
  // A fragments of k-step t of the current conv (tap t / KC, channel block t % KC)
  auto read_a = [&](int t, bf16x8 (&ah)[TM], bf16x8 (&al)[TM]) {
    const int tap = t / G::KC, q = (t % G::KC) * 2 + h;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ar = tap == 0 ? arow[i][0] : tap == 1 ? arow[i][1] : arow[i][2];
      const int as = tap == 0 ? asw[i][0] : tap == 1 ? asw[i][1] : asw[i][2];
      const int a = ar + ((q ^ as) << 4);
      ah[i] = *reinterpret_cast<const bf16x8*>(xhi + a);
      al[i] = *reinterpret_cast<const bf16x8*>(xlo + a);
    }
  };
  // one 16-deep k-step g on the fragments in (ah, al) and (bh, bl); the W
  // fragments are then reloaded with k-step g + PD
  auto mma = [&](int g, const bf16x8 (&ah)[TM], const bf16x8 (&al)[TM], bf16x8 (&bh)[TN], bf16x8 (&bl)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    wload(g + PD, bh, bl);
  };
  bf16x8 ah2[2][TM], al2[2][TM];

#pragma unroll 1
  for (int step = 0; step < 7; ++step) {
    const int gb = step * G::KS;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // k-steps in groups of PD: A fragments alternate between two register sets —
    // k-step t+1's are read from LDS while k-step t's MFMAs run (the image only
    // changes between steps) — and W comes from the ring
    read_a(0, ah2[0], al2[0]);
#pragma unroll 1
    for (int t = 0; t < G::KS - PD; t += PD) {
#pragma unroll
      for (int u = 0; u < PD; ++u) {
        read_a(t + u + 1, ah2[(u + 1) & 1], al2[(u + 1) & 1]);
        mma(gb + t + u, ah2[u & 1], al2[u & 1], wbh[u], wbl[u]);
      }
    }
    // the next conv's addend spx[step + 1] (accumulator layout: row per register,
    // col = lane & 31), issued PD k-steps before the epilogue.  Row offsets are
    // laundered per step (asm) so hipcc rebuilds them here instead of hoisting 64
    // per-element addresses out of the step loop into registers.
    int ldx4 = p.ldx * 4, ldo4 = p.ldo * 4, mw = wr0 + wm * TM * 32 + 4 * h;
    asm volatile("" : "+s"(ldx4), "+s"(ldo4), "+v"(mw));
    float nx[TM][TN][16];
    if (step < 6) {
      const __amdgpu_buffer_rsrc_t rxs = make_rsrc(p.x);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m0 = mw + i * 32;  // row of register 0
        const int lo = -m0, hi = p.M - m0;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int base = (m0 * p.ldx + (step + 1) * W + (wn * TN + j) * 32 + r32) * 4;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = (r & 3) + 8 * (r >> 2);
            nx[i][j][r] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rxs, (rr >= lo && rr < hi) ? base + rr * ldx4 : kOOB, 0, 0));
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      if (u + 1 < PD) read_a(G::KS - PD + u + 1, ah2[(u + 1) & 1], al2[(u + 1) & 1]);
      mma(gb + G::KS - PD + u, ah2[u & 1], al2[u & 1], wbh[u], wbl[u]);
    }
    __syncthreads();  // every wave is done reading X_step

    // ---- epilogue: sp = BN(ReLU(acc + b)); owned rows -> out; X_{step+1} -> LDS
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = (wn * TN + j) * 32 + r32;
      const float bv = p.bias[step * W + col];
      const float sc = p.scale[step * W + col];
      const float sh = p.shift[step * W + col];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m0 = mw + i * 32;
        const int olo = own0 - m0, ohi = own1 - m0;
        const int base = (m0 * p.ldo + step * W + col) * 4;
        const int irb = m0 - wr0 + kPad;  // image row of register 0
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = (r & 3) + 8 * (r >> 2);
          const float y = fmaxf(acc[i][j][r] + bv, 0.f) * sc + sh;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), rout,
                                                (rr >= olo && rr < ohi) ? base + rr * ldo4 : kOOB, 0, 0);
          if (step < 6) {
            const float x = y + nx[i][j][r];
            const __bf16 hh = (__bf16)x;
            const __bf16 ll = (__bf16)(x - (float)hh);
            // lanes l, l^1 hold channels col, col^1 of this row: the even lane
            // writes both hi halves, the odd lane both lo halves (one 4-B store each)
            const unsigned send = (lane & 1) ? bf_bits(hh) : bf_bits(ll);
            const unsigned recv = (unsigned)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);
            const int a = G::addr(irb + rr, col & ~1);
            if (lane & 1)
              *reinterpret_cast<unsigned*>(xlo + a) = recv | ((unsigned)bf_bits(ll) << 16);
            else
              *reinterpret_cast<unsigned*>(xhi + a) = (unsigned)bf_bits(hh) | (recv << 16);
          }
        }
      }
    }
    __syncthreads();  // X_{step+1} visible
  }
}


// ---- variant 4: halo-free strips (skewed chunk pipeline), W = 128 ----------
// A block owns a strip of `rout` consecutive frame rows (about M / (2 x CUs):
// one round of two blocks per CU) and walks it in chunks of kSR = 96 rows.  In
// chunk c, conv i computes the rows [r0 + c*kSR - i*d, ... + kSR): each conv lags
// the previous one by d rows, so the rows it needs of X_i = sp_{i-1} + spx[i]
// are the kSR rows conv i-1 has just produced plus 2d rows from the previous
// chunk (kept in LDS: the last 2d image rows of X_i are saved as the image is
// overwritten, and copied back in front of the next chunk's X_i).  The chain's
// receptive field costs 6d warm-up rows at the start of a strip and 6d drain rows
// at its end — 12d per ~250-row strip instead of 12d per 128-row window — and one
// round of blocks instead of 3-4 rounds of windows.  Same operands, k order and
// epilogue as the other variants, so the owned rows are bit-identical.
constexpr int kSR = 96;                            // output rows per chunk (3 tiles of 32)
constexpr int kSIR = kSR + 2 * kPad;               // image rows: 2d history + kSR new
constexpr int kSRB = 256;                          // bytes per image row and plane (128 bf16)
// + the zero row; + 64 B so the lo plane sits 16 banks after the hi plane (the epilogue's
// paired hi / lo 4-B stores of one row then hit distinct banks)
constexpr int kSPlane = (kSIR + 1) * kSRB + 64;
constexpr int kSHistRows = 2 * kPad;               // history rows per slot
constexpr int kSLds = 2 * kSPlane + 6 * kSHistRows * 2 * kSRB;  // image + 6 history slots (X_1..X_6)
static_assert(kSR % 16 == 0, "history rows keep their swizzle only if kSR % 16 == 0");
static_assert(2 * kSLds <= 160 * 1024, "two strip blocks per CU");

__device__ __forceinline__ int s_off(int ir, int ch) { return ((((ch >> 3) ^ (ir & 15)) << 4)) + (ch & 7) * 2; }

template <int PD>
__global__ __launch_bounds__(256, 2) void res2_strip_kernel(const Res2Args p) {
  constexpr int W = 128, KS = 3 * W / 16, KC = W / 16, TM = 3, kTotal = 7 * KS;
  static_assert(KS % PD == 0 && PD % 2 == 0, "res2 strip W prefetch depth");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + kSPlane;
  unsigned char* hist = smem + 2 * kSPlane;  // [slot 6][row 2kPad][plane 2][kSRB]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wn = tid >> 6;  // 4 waves, 32 output channels each
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int d = p.dil;
  const int M = p.M;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring strips share an XCD L2
  const int own0 = blk * p.rout;
  const int own1 = min(own0 + p.rout, M);
  const int r0 = own0 - 6 * d;  // chunk 0's first conv-0 output row
  const int nch = (own1 - own0 + 12 * d + kSR - 1) / kSR;

  // ---- zero row, zeroed history, X_0 of chunk 0: image row ir = frame row r0 - d + ir
  if (tid < kSRB / 4) {
    reinterpret_cast<unsigned*>(xhi + kSIR * kSRB)[tid] = 0u;
    reinterpret_cast<unsigned*>(xlo + kSIR * kSRB)[tid] = 0u;
  }
  for (int q = tid; q < 6 * kSHistRows * 2 * kSRB / 16; q += 256)
    reinterpret_cast<u32x4*>(hist)[q] = u32x4{0u, 0u, 0u, 0u};
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x);
  auto put4 = [&](int ir, int c, const f32x4& v) {
    bf16x4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const __bf16 hh = (__bf16)v[e];
      hi[e] = hh;
      lo[e] = (__bf16)(v[e] - (float)hh);
    }
    const int a = ir * kSRB + s_off(ir, c);
    *reinterpret_cast<bf16x4*>(xhi + a) = hi;
    *reinterpret_cast<bf16x4*>(xlo + a) = lo;
  };
  for (int q = tid; q < (kSR + 2 * d) * (W / 4); q += 256) {
    const int ir = q / (W / 4);
    const int c = (q - ir * (W / 4)) * 4;
    const int m = r0 - d + ir;
    put4(ir, c, bload4(rx, (m >= 0 && m < M) ? (m * p.ldx + c) * 4 : kOOB));
  }

  // ---- W fragments from global: k-step g (0 .. 7*KS-1, wrapping across chunks),
  // plane pl, column tile wn at ((g * 2 + pl) * (W / 32) + wn) * 1 KB + lane * 16
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  const int wlane = (wn * 64 + lane) * 16;
  auto wload = [&](int g, bf16x8& bh, bf16x8& bl) {
    const int o = g * 2 * (W / 32) * 1024 + wlane;
    bh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, o, 0, 0));
    bl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, o + (W / 32) * 1024, 0, 0));
  };
  bf16x8 wbh[PD], wbl[PD];
#pragma unroll
  for (int u = 0; u < PD; ++u) wload(u, wbh[u], wbl[u]);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rout = make_rsrc(p.out);
  const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias);
  const __amdgpu_buffer_rsrc_t rscale = make_rsrc(p.scale);
  const __amdgpu_buffer_rsrc_t rshift = make_rsrc(p.shift);
  f32x16 acc[TM];
  // A-fragment row of tile i for tap j: image row i*32 + r32 + j*d when bit j of
  // vm[i] says the tap stays inside the row's utterance, else the zero row (computed,
  // not looked up: a tap-indexed array would live in scratch)
  int vm[TM];
  int dq = d;
  // NA = active tiles (the last chunk of a strip may need fewer than TM)
  auto read_a = [&](auto na, int t, bf16x8 (&ah)[TM], bf16x8 (&al)[TM]) {
    constexpr int NA = decltype(na)::value;
    const int tap = t / KC, q = (t % KC) * 2 + h;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int ir = ((vm[i] >> tap) & 1) ? i * 32 + r32 + tap * dq : kSIR;
      const int a = ir * kSRB + ((q ^ (ir & 15)) << 4);
      ah[i] = *reinterpret_cast<const bf16x8*>(xhi + a);
      al[i] = *reinterpret_cast<const bf16x8*>(xlo + a);
    }
    __builtin_amdgcn_sched_barrier(0);  // k-step t's fragment reads go out before k-step t-1's MFMAs
  };
  // one 16-deep k-step g; its ring slot then reloads k-step g + PD (mod 7*KS: the
  // next chunk's conv 0 follows conv 6)
  auto mma = [&](auto na, int g, const bf16x8 (&ah)[TM], const bf16x8 (&al)[TM], bf16x8& bh, bf16x8& bl) {
    constexpr int NA = decltype(na)::value;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh, acc[i], 0, 0, 0);
    }
    const int gn = g + PD;
    wload(gn >= kTotal ? gn - kTotal : gn, bh, bl);
    // keep the slot's reload right behind its MFMAs (hipcc otherwise sinks the whole
    // group's loads to the end of the unrolled group: the ring would hide nothing)
    __builtin_amdgcn_sched_barrier(0);
  };
  bf16x8 ah2[2][TM], al2[2][TM];
  const int col = wn * 32 + r32;

  // one conv of one chunk on its NA active 32-row tiles
  auto conv_step = [&](auto na, int c, int step, bool more) {
    constexpr int NA = decltype(na)::value;
        const int base = r0 + c * kSR - step * d;  // frame row of this conv's output row 0
        // per step: keeps hipcc from hoisting the 48 d-dependent image addresses of the
        // epilogue (and the fragment rows) out of the loops into spilled registers
        dq = d;
        asm volatile("" : "+s"(dq));
        // A-fragment rows of this lane per tile and tap: image row lr + j*d, or the zero
        // row when the tap leaves the row's utterance (or the row is outside the batch)
  #pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int lr = i * 32 + r32;
          const int m = base + lr;
          int t = -1, L = 0;
          if (m >= 0 && m < M) {
            if (p.seg) {
              const int u = seg_of(p.seg, p.nseg, m);
              t = m - p.seg[u];
              L = p.seg[u + 1] - p.seg[u];
            } else {
              const int u = m / p.T;
              t = m - u * p.T;
              L = p.T;
            }
          }
          int v = 0;
  #pragma unroll
          for (int j = 0; j < 3; ++j) {
            const int tt = t + (j - 1) * d;
            v |= (t >= 0 && tt >= 0 && tt < L) ? 1 << j : 0;
          }
          vm[i] = v;
        }
  #pragma unroll
        for (int i = 0; i < NA; ++i)
  #pragma unroll
          for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
        const int gb = step * KS;
        // this conv's epilogue constants, fetched now (they land during the k-loop)
        const float bv = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rbias, (step * W + col) * 4, 0, 0));
        const float sc = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rscale, (step * W + col) * 4, 0, 0));
        const float sh = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rshift, (step * W + col) * 4, 0, 0));
        read_a(na, 0, ah2[0], al2[0]);
  #pragma unroll 1
        for (int t = 0; t < KS - PD; t += PD) {
  #pragma unroll
          for (int u = 0; u < PD; ++u) {
            read_a(na, t + u + 1, ah2[(u + 1) & 1], al2[(u + 1) & 1]);
            mma(na, gb + t + u, ah2[u & 1], al2[u & 1], wbh[u], wbl[u]);
          }
        }
        // next image rows' addend, issued PD k-steps before the epilogue: spx[step + 1]
        // on this conv's rows, or (after conv 6) spx[0] on the next chunk's new rows
        const bool wimg = step < 6 || more;
        int ldx4 = p.ldx * 4, ldo4 = p.ldo * 4;
        int abase = step < 6 ? base : r0 + (c + 1) * kSR + d;
        asm volatile("" : "+s"(ldx4), "+s"(ldo4), "+s"(abase));
        const int acol = step < 6 ? (step + 1) * W : 0;
        float nx[TM][16];
        f32x4 xh = {0.f, 0.f, 0.f, 0.f};
        if (wimg) {
  #pragma unroll
          for (int i = 0; i < NA; ++i) {
            const int m0 = abase + i * 32 + 4 * h;  // row of register 0
            const int lo = -m0, hi = M - m0;
            const int b0 = (m0 * p.ldx + acol + col) * 4;
            if (abase + i * 32 >= 0 && abase + i * 32 + 32 <= M) {  // wave-uniform: every row in range
  #pragma unroll
              for (int r = 0; r < 16; ++r)  // row step in the scalar offset: no per-register VALU
                nx[i][r] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rx, b0, ((r & 3) + 8 * (r >> 2)) * ldx4, 0));
            } else {
  #pragma unroll
              for (int r = 0; r < 16; ++r) {
                const int rr = (r & 3) + 8 * (r >> 2);
                nx[i][r] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rx, (rr >= lo && rr < hi) ? b0 + rr * ldx4 : kOOB, 0, 0));
              }
            }
          }
          if (step == 6 && tid < 2 * d * (W / 4)) {  // the next chunk's X_0 history rows
            const int k = tid / (W / 4), c4 = (tid - k * (W / 4)) * 4;
            const int m = r0 + (c + 1) * kSR - d + k;
            xh = bload4(rx, (m >= 0 && m < M) ? (m * p.ldx + c4) * 4 : kOOB);
          }
        }
  #pragma unroll
        for (int u = 0; u < PD; ++u) {
          if (u + 1 < PD) read_a(na, KS - PD + u + 1, ah2[(u + 1) & 1], al2[(u + 1) & 1]);
          mma(na, gb + KS - PD + u, ah2[u & 1], al2[u & 1], wbh[u], wbl[u]);
        }
        __syncthreads();  // every wave is done reading X_step

        // ---- epilogue: sp = BN(ReLU(acc + b)); owned rows -> out; X_{step+1} (or the
        // next chunk's X_0) -> image rows [2d, 2d + kSR); X_step's last 2d rows -> history
        const int cp = col & ~1;
        unsigned char* hslot = hist + (step - 1) * (kSHistRows * 2 * kSRB);  // X_step's slot (step >= 1)
        // image byte offsets (within a plane; the lo plane is kSPlane above the hi one): tile 0's
        // registers 0..3 are image rows ib .. ib + 3; register r + 4 is 8 rows down, which flips bit
        // 3 of the row's XOR swizzle ((a ^ 128) + 8 rows); r + 8 and tile i + 1 are 16 and 32 rows
        // down, same swizzle — 4 computed offsets per lane and conv instead of one per register
        const bool odd = lane & 1;
        const int ib = 2 * dq + 4 * h;
        int a4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a4[k] = (ib + k) * kSRB + s_off(ib + k, cp);
        unsigned char* img = xhi + (odd ? kSPlane : 0);
        // MODE 0: stores only (the strip's last conv 6); 1: X_{step+1} = sp + spx[step+1];
        // 2: the next chunk's X_0 = spx[0].  FULL: every row of the chunk is owned (no
        // per-row bounds).  Uniform choices hoisted out of the 48-register loop.
        auto epi = [&](auto mode_, auto full_) {
          constexpr int MODE = decltype(mode_)::value;
          constexpr bool FULL = decltype(full_)::value;
#pragma unroll
          for (int i = 0; i < NA; ++i) {
            const int lr0 = i * 32 + 4 * h;
            const int m0 = base + lr0;
            const int olo = own0 - m0, ohi = own1 - m0;
            const int b0 = (m0 * p.ldo + step * W + col) * 4;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rr = (r & 3) + 8 * (r >> 2);
              const float y = fmaxf(acc[i][r] + bv, 0.f) * sc + sh;
              if constexpr (FULL)  // every row owned: the row step rides in the scalar offset
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), rout, b0, rr * ldo4, 0);
              else
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), rout,
                                                      rr >= olo && rr < ohi ? b0 + rr * ldo4 : kOOB, 0, 0);
              if constexpr (MODE != 0) {
                const float x = MODE == 1 ? y + nx[i][r] : nx[i][r];
                const __bf16 hh = (__bf16)x;
                const __bf16 ll = (__bf16)(x - (float)hh);
                // lanes l, l^1 hold channels col, col^1 of this row: the even lane writes
                // both hi halves, the odd lane both lo halves (one 4-B store each)
                const unsigned send = odd ? bf_bits(hh) : bf_bits(ll);
                const unsigned recv = (unsigned)__builtin_amdgcn_mov_dpp((int)send, 0xB1, 0xF, 0xF, false);
                const int ir = ib + 32 * i + rr;
                const int a = ((r >> 2) & 1 ? (a4[r & 3] ^ 128) + 8 * kSRB : a4[r & 3]) + ((r >> 3) * 16 + 32 * i) * kSRB;
                unsigned* dst = reinterpret_cast<unsigned*>(img + a);
                if (NA == TM && i == TM - 1 && ir >= kSR) {  // X_step's rows [kSR, kSR + 2d): save before overwriting
                  if (step >= 1)
                    *reinterpret_cast<unsigned*>(hslot + ((ir - kSR) * 2 + (lane & 1)) * kSRB + (a - ir * kSRB)) = *dst;
                }
                *dst = odd ? (recv | ((unsigned)bf_bits(ll) << 16)) : ((unsigned)bf_bits(hh) | (recv << 16));
              }
            }
          }
        };
        const bool full = base >= own0 && base + NA * 32 <= own1;
        if (!wimg) epi(std::integral_constant<int, 0>{}, std::false_type{});
        else if (step == 6) epi(std::integral_constant<int, 2>{}, std::false_type{});
        else if (full) epi(std::integral_constant<int, 1>{}, std::true_type{});
        else epi(std::integral_constant<int, 1>{}, std::false_type{});
        // image rows [0, 2d): X_{step+1}'s history from the previous chunk (slot step),
        // or the next chunk's X_0 rows fetched above
        if (step < 6) {
          if (tid < 2 * d * 32) {  // 16-B pieces: row k, plane pl, piece e
            const int k = tid >> 5, pl = (tid >> 4) & 1, e = tid & 15;
            const u32x4 v = reinterpret_cast<const u32x4*>(hist + step * (kSHistRows * 2 * kSRB) + (k * 2 + pl) * kSRB)[e];
            reinterpret_cast<u32x4*>((pl ? xlo : xhi) + k * kSRB)[e] = v;
          }
        } else if (more && tid < 2 * d * (W / 4)) {
          const int k = tid / (W / 4), c4 = (tid - k * (W / 4)) * 4;
          put4(k, c4, xh);
        }
  };

  // the last chunk needs only the rows up to the strip's end (+ the 6d drain rows
  // of conv 6): its inactive tiles are skipped (their image rows are never read)
  const int last_tiles = (own1 - own0 + 12 * d - (nch - 1) * kSR + 31) / 32;
#pragma unroll 1
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    const int nt = more ? TM : last_tiles;
#pragma unroll 1
    for (int step = 0; step < 7; ++step) {
      if (nt >= 3) conv_step(std::integral_constant<int, 3>{}, c, step, more);
      else if (nt == 2) conv_step(std::integral_constant<int, 2>{}, c, step, more);
      else conv_step(std::integral_constant<int, 1>{}, c, step, more);
      __syncthreads();  // the next conv's image is complete
    }
  }
}

}  // namespace

bool res2_chain_supported(int w, int dil) { return (w == 64 || w == 128) && dil >= 1 && dil <= kPad; }

static int res2_rows(int) { return 128; }

template <int W, int R, int WN, int NW = R / 32, int PD = 2>
void launch_res2_k(const Res2Args& p, int nblk, hipStream_t s) {
  hipLaunchKernelGGL((res2_chain_kernel<W, R, WN, NW, PD>), dim3(nblk), dim3(Geo<W, R, WN, NW>::NT),
                     (Geo<W, R, WN, NW>::LDS), s, p);
}

template <int W>
void launch_res2_w(const Res2Args& p, int nblk, hipStream_t s) {
  if (W == 128 && p.variant == 4) {
    hipLaunchKernelGGL(res2_strip_kernel<4>, dim3(nblk), dim3(256), kSLds, s, p);
  } else if (p.variant == 3) {
    if constexpr (W == 128) launch_res2_k<W, 128, 4, 8>(p, nblk, s);  // 8 waves of 64 rows x 32 channels
    else launch_res2_k<W, 128, 2, 8>(p, nblk, s);
  } else if (p.variant == 2) {
    if constexpr (W == 128) launch_res2_k<W, 128, 4, 4, 4>(p, nblk, s);  // 1 x 4 waves: 128 rows x 32 channels, 4 W k-steps in flight
    else launch_res2_k<W, 128, 2>(p, nblk, s);
  } else {
    launch_res2_k<W, 128, 2>(p, nblk, s);
  }
}

void launch_res2_chain(const Res2Args& p, int w, hipStream_t s) {
  WSP_CHECK(res2_chain_supported(w, p.dil), "res2_chain: width must be 64 or 128 and dilation 1..4");
  WSP_CHECK(p.M > 0 && (p.seg || p.T > 0), "res2_chain: empty shape");
  WSP_CHECK(p.rout == res2_chain_rout(p.dil, p.variant, p.M), "res2_chain: rout must be res2_chain_rout(dil, variant, M)");
  WSP_CHECK((long long)p.M * p.ldx * 4 < (long long)kOOB && (long long)p.M * p.ldo * 4 < (long long)kOOB,
            "res2_chain: operand exceeds 2 GiB (split the batch)");
  WSP_CHECK(p.ldx >= 8 * w && p.ldo >= 7 * w && p.ldx % 4 == 0, "res2_chain: bad leading dimensions");
  const int nblk = (p.M + p.rout - 1) / p.rout;
  if (w == 128)
    launch_res2_w<128>(p, nblk, s);
  else
    launch_res2_w<64>(p, nblk, s);
  WSP_HIP(hipGetLastError());
}

// Strips (variant 4, W = 128): one round of two blocks per CU over the batch's rows,
// at least 64 rows per strip (the 12d warm-up / drain rows are per strip).
int res2_chain_rout(int dil, int variant, int M) {
  if (variant == 4) return std::max(64, ceil_div(M, 2 * device_cu_count()));
  return res2_rows(variant) - 12 * dil;
}

}  // namespace wsp
