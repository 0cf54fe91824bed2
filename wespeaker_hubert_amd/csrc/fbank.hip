// Batched Kaldi log-mel fbank + fused CMN on gfx950.
//
// Restates torchaudio.compliance.kaldi.fbank as the reference calls it
// (wespeaker/cli/speaker.py:89-104, wespeaker/dataset/processor.py:472-502;
// native restatement runtime/core/frontend/fbank.h:138-198): snip-edges
// framing 400/160, DC removal, pre-emphasis 0.97 (replicate pad), symmetric
// Hamming window, zero pad to 512, real FFT, |X|^2, 80 triangular mel
// filters (Nyquist weight 0), log(max(e, FLT_EPSILON)); then optional CMN
// (speaker.py:102-103 / dataset_utils.py:19-26).
//
// Precision: everything from the DC mean to the mel energies runs in float64
// (the mel filter weights are torchaudio's float32 values); the log is logf of
// the energy rounded to float32 (the output is float32: ~1 output ulp against
// the f64 log's 0.5, at 15 % fewer instructions per frame).  The reference's
// own path is float32 (torchaudio's fp32 rfft), which deviates from exact
// arithmetic by ~1e-4 on low-energy bins; this kernel sits ~1e-6 from the
// float64 oracle, i.e. it is never less accurate than the fp32 reference it
// replaces.  f64 costs little here: the whole fbank is ~12 kflop per frame,
// latency-bound.
//
// Layout: one workgroup (16 waves) = one utterance; wave w takes frames
// w, w+16, ... and loads the samples of its next frame while it transforms
// the current one.  Each wave owns a 256-entry complex f64 LDS buffer: the
// 512-point real FFT is a 256-point complex FFT of z[n] = y[2n] + i y[2n+1]
// (radix-4 Stockham, 4 in-place stages, one butterfly per lane; a wave's LDS
// ops execute in order, so a stage's reads of all lanes precede its writes
// and no workgroup barrier is needed) followed by the even/odd split.  The
// per-utterance mel-column sums for CMN accumulate in registers (f64), are
// combined across waves in a fixed order (deterministic, batch-independent)
// and the block then subtracts the mean from its own (L2-hot) output: one
// launch, no second pass over HBM.  Output is channels-last (B, T, 80).
#include <cfloat>
#include <cmath>

#include "fbank_mel_table.h"
#include "kernels.h"

namespace wsp {

namespace {

constexpr int kFL = 400, kFS = 160, kNB = 80;
constexpr int kWaves = 16, kThreads = kWaves * 64;

// table layout (doubles): window[400] | cos256 | sin256 | cos512 | sin512 |
//   start[80] | len[80] | off[80] | w[<=1024]
// w is stored lane-interleaved and zero-padded to a fixed length per lane
// group: bins 0..63 as w0[i][64] (i < kMelLen0), bins 64..79 as w1[i][16]
// (i < kMelLen1).  Every lane of a group then runs the same unrolled loop,
// the weight reads are lane-contiguous (no bank conflicts), and the padded
// terms add w = 0 exactly (e + 0*p == e for the finite, non-negative sums),
// so the sums equal the sparse form's bit for bit.
constexpr int kTabWin = 0, kTabC256 = 400, kTabS256 = 656, kTabC512 = 912, kTabS512 = 1168,
              kTabStart = 1424, kTabLen = 1504, kTabOff = 1584, kTabW = 1664;
// tw: per-lane twiddles of FFT stages 1..3 as (cos, sin) pairs, [stage][r-1][lane]:
// lane-contiguous 16-B reads (the c256/s256 gathers at stride 4..12 doubles
// conflicted 2-4 ways); same values as c256[m]/s256[m]
constexpr int kTabTw = kTabW + 1024;
constexpr int kTabSize = kTabTw + 3 * 3 * 64 * 2;
constexpr int kMelLen0 = 10, kMelLen1 = 16;
constexpr int kTabW1 = kTabW + kMelLen0 * 64;
static_assert(kTabW1 + kMelLen1 * 16 <= kTabSize, "fbank interleaved mel table");
static_assert(kTabSize == kFbankTableDoubles, "fbank table size");

// Bank swizzle of a wave's 256-entry complex buffer (16-B entries, 16 slots per
// 256-B row): odd rows XOR the low 4 index bits by 13.  ds_write_b128 serves
// 8 contiguous lanes per cycle: the radix-4 Stockham writes of the first two
// stages (index 4j + m, and 16 (j >> 2) + (j & 3) + 4m) put those 8 lanes on an
// even and an odd row with equal low bits, which the XOR (13 differs from 0 in
// both bit pairs) separates.  ds_read_b128 serves the lane groups {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31} (+32): for a contiguous read, row 2r's entries
// {0-3, 12-15} and row 2r+1's {4-11} stay disjoint under XOR 13 (it maps
// {4-11} onto itself), so contiguous reads and writes stay conflict-free.
__device__ __forceinline__ int zsw(int i) { return i ^ (((i >> 4) & 1) * 13); }

// 64-bit DPP move (both halves with one control; lanes the masks leave out get 0)
#define WSP_DPP64(v, ctrl, rmask)                                                                               \
  __longlong_as_double(                                                                                         \
      (long long)(((unsigned long long)(unsigned)__builtin_amdgcn_update_dpp(                                   \
                       0, (int)(unsigned)((unsigned long long)__double_as_longlong(v) >> 32), ctrl, rmask, 0xF, \
                       false)                                                                                   \
                   << 32) |                                                                                     \
                  (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)__double_as_longlong(v), ctrl, rmask,  \
                                                        0xF, false)))

// Sum over the wave, uniform result: DPP pairs / quads / half-rows / rows, then
// row_bcast15 / row_bcast31 into lane 63 (VALU latency instead of six
// ds_bpermute round trips); fixed order, so deterministic and batch-independent.
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += WSP_DPP64(v, 0xB1, 0xF);   // quad_perm [1,0,3,2]
  v += WSP_DPP64(v, 0x4E, 0xF);   // quad_perm [2,3,0,1]
  v += WSP_DPP64(v, 0x141, 0xF);  // row_half_mirror
  v += WSP_DPP64(v, 0x140, 0xF);  // row_mirror: every lane holds its row's sum
  v += WSP_DPP64(v, 0x142, 0xA);  // row_bcast15: rows 1, 3 += rows 0, 2
  v += WSP_DPP64(v, 0x143, 0xC);  // row_bcast31: rows 2, 3 += lane 31 (rows 0 + 1)
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)u, 63);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Orders this wave's LDS accesses (a compiler scheduling fence; the hardware
// keeps one wave's LDS instructions in order).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// lane l receives v of lane l-1 (DPP wave_shr:1); lane 0 receives `first`
__device__ __forceinline__ double wave_shr1(double v, double first) {
  const unsigned long long u = __double_as_longlong(v), f = __double_as_longlong(first);
  const int lo = __builtin_amdgcn_update_dpp((int)(unsigned)f, (int)(unsigned)u, 0x138, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(unsigned)(f >> 32), (int)(unsigned)(u >> 32), 0x138, 0xF,
                                             0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

__device__ __forceinline__ double readlane63(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)u, 63);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int kDtype>
__device__ __forceinline__ double load_sample(const void* __restrict__ wav, long i) {
  if (kDtype == 1) return (double)reinterpret_cast<const short*>(wav)[i];
  return (double)reinterpret_cast<const float*>(wav)[i];
}

}  // namespace

template <int kDtype>
__global__ __launch_bounds__(kThreads) void fbank_cmn_kernel(const void* __restrict__ wav, int N_, int ld,
                                                             float scale, float* __restrict__ feats, int T_,
                                                             int cmn, const double* __restrict__ tab,
                                                             const int* __restrict__ wseg,
                                                             const int* __restrict__ fseg) {
  __shared__ double s_tab[kTabSize];
  __shared__ double2 s_buf[kWaves][256];
  __shared__ double s_part[kWaves][kNB];
  __shared__ double s_mean[kNB];

  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // uniform batch: utterance b = samples [b*ld, b*ld + N_), frames [b*T_, (b+1)*T_);
  // segmented batch: samples [wseg[b], wseg[b+1]), frames [fseg[b], fseg[b+1])
  const long wbase = wseg ? (long)wseg[b] : (long)b * ld;
  const long fbase = fseg ? (long)fseg[b] : (long)b * T_;
  const int T = fseg ? fseg[b + 1] - fseg[b] : T_;
  (void)N_;
  if (T <= 0) return;  // block-uniform

  for (int i = tid; i < kTabSize; i += kThreads) s_tab[i] = tab[i];
  __syncthreads();

  const double* win = s_tab + kTabWin;
  const double2* tw = reinterpret_cast<const double2*>(s_tab + kTabTw);
  const double* c512 = s_tab + kTabC512;
  const double* s512 = s_tab + kTabS512;
  double2* buf = s_buf[wave];
  double* pw = reinterpret_cast<double*>(buf);
  const double dscale = (double)scale;

  // mel bins of this lane: bin0 = lane, bin1 = lane + 64 (< 80)
  const int bin1 = lane + 64;
  const bool has1 = bin1 < kNB;
  const int st0 = (int)s_tab[kTabStart + lane];
  const int st1 = has1 ? (int)s_tab[kTabStart + bin1] : 0;
  double csum0 = 0.0, csum1 = 0.0;

  // raw samples of the wave's next frame, loaded one frame ahead so their
  // latency hides behind the current frame's FFT (PCM16 and f32 values are
  // exact in f32)
  float ne[4], no[4];
  auto fetch = [&](int t) {
    const long x0 = wbase + (long)t * kFS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      ne[q] = no[q] = 0.f;
      if (n < kFL / 2) {
        ne[q] = (float)load_sample<kDtype>(wav, x0 + 2 * n);
        no[q] = (float)load_sample<kDtype>(wav, x0 + 2 * n + 1);
      }
    }
  };
  if (wave < T) fetch(wave);

  for (int t = wave; t < T; t += kWaves) {
    // 1. samples of z[n] = y[2n] + i y[2n+1], n = lane + 64q (n < 200 carries data)
    double xe[4], xo[4], xp[4];
    double sum = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      xe[q] = (double)ne[q] * dscale;
      xo[q] = (double)no[q] * dscale;
      if (n < kFL / 2) sum += xe[q] + xo[q];
    }
    if (t + kWaves < T) fetch(t + kWaves);
    // y[2n-1] is the odd sample of element n-1: lane-1's xo (wave_shr:1), or
    // lane 63's xo of the previous q; n = 0 replicates y[0] (pre-emphasis pad)
#pragma unroll
    for (int q = 0; q < 4; ++q) xp[q] = wave_shr1(xo[q], q > 0 ? readlane63(xo[q - 1]) : xe[0]);
    // 2. DC removal, pre-emphasis, window (f64; exact sums for PCM16 input)
    const double mean = wave_sum_f64(sum) * (1.0 / kFL);
    // z[n] for n = lane + 64q stays in registers: it is exactly what the first
    // Stockham stage's butterfly of this lane reads (a[r] = z[lane + 64 r])
    double2 zin[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      double2 z = make_double2(0.0, 0.0);
      if (n < kFL / 2) {
        const double de = xe[q] - mean, dd = xo[q] - mean, dp = xp[q] - mean;
        z.x = (de - 0.97 * dp) * win[2 * n];
        z.y = (dd - 0.97 * de) * win[2 * n + 1];
      }
      zin[q] = z;
    }
    // 3. 256-point complex FFT, radix-4 Stockham, in place; the last stage's
    // outputs j + 64 m are also kept in registers (zl: the split's own-lane reads)
    double2 zl[4];
#pragma unroll
    for (int ns = 1; ns < 256; ns *= 4) {
      const int j = lane;
      const int k = j & (ns - 1);
      double2 a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = ns == 1 ? zin[r] : buf[zsw(j + 64 * r)];
      if (ns > 1) {
        const int stage = ns == 4 ? 0 : ns == 16 ? 1 : 2;
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const double2 cs = tw[(stage * 3 + r - 1) * 64 + j];
          const double c = cs.x, s = cs.y;
          // a *= exp(-i 2 pi m / 256) = c - i s
          const double re = a[r].x * c + a[r].y * s;
          const double im = a[r].y * c - a[r].x * s;
          a[r] = make_double2(re, im);
        }
      }
      const double2 s02 = make_double2(a[0].x + a[2].x, a[0].y + a[2].y);
      const double2 d02 = make_double2(a[0].x - a[2].x, a[0].y - a[2].y);
      const double2 s13 = make_double2(a[1].x + a[3].x, a[1].y + a[3].y);
      const double2 d13 = make_double2(a[1].x - a[3].x, a[1].y - a[3].y);
      wave_lds_fence();
      // -i * d13 = (d13.y, -d13.x)
      const int d = (j / ns) * ns * 4 + k;
      const double2 o0 = make_double2(s02.x + s13.x, s02.y + s13.y);
      const double2 o1 = make_double2(d02.x + d13.y, d02.y - d13.x);
      const double2 o2 = make_double2(s02.x - s13.x, s02.y - s13.y);
      const double2 o3 = make_double2(d02.x - d13.y, d02.y + d13.x);
      buf[zsw(d)] = o0;
      buf[zsw(d + ns)] = o1;
      buf[zsw(d + 2 * ns)] = o2;
      buf[zsw(d + 3 * ns)] = o3;
      if (ns == 64) {  // d = j: outputs j, j + 64, j + 128, j + 192
        zl[0] = o0;
        zl[1] = o1;
        zl[2] = o2;
        zl[3] = o3;
      }
      wave_lds_fence();
    }
    // 4. even/odd split -> X[k], power |X[k]|^2 for k = 0..255 (Nyquist weight is 0)
    double pk[4];
    {
      double2 z[4], zc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = lane + 64 * q;
        z[q] = zl[q];
        zc[q] = buf[zsw((256 - k) & 255)];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = lane + 64 * q;
        // Xe = (Z + conj(Zc))/2 ; Xo = -i (Z - conj(Zc))/2
        const double er = 0.5 * (z[q].x + zc[q].x), ei = 0.5 * (z[q].y - zc[q].y);
        const double dr = 0.5 * (z[q].x - zc[q].x), di = 0.5 * (z[q].y + zc[q].y);
        const double or_ = di, oi = -dr;
        const double c = c512[k], s = s512[k];  // W^k = c - i s
        const double xr = er + (or_ * c + oi * s);
        const double xi = ei + (oi * c - or_ * s);
        pk[q] = xr * xr + xi * xi;
      }
    }
    wave_lds_fence();
#pragma unroll
    for (int q = 0; q < 4; ++q) pw[lane + 64 * q] = pk[q];
    wave_lds_fence();
    // 5. mel filter bank + log (lane -> bins lane, lane + 64)
    float* frow = feats + (fbase + t) * kNB;
    {
      double e = 0.0;
#pragma unroll
      for (int i = 0; i < kMelLen0; ++i) e += s_tab[kTabW + i * 64 + lane] * pw[st0 + i];
      const float v = logf((float)fmax(e, (double)FLT_EPSILON));
      frow[lane] = v;
      csum0 += (double)v;
    }
    if (has1) {
      double e = 0.0;
#pragma unroll
      for (int i = 0; i < kMelLen1; ++i) e += s_tab[kTabW1 + i * 16 + (lane & 15)] * pw[st1 + i];
      const float v = logf((float)fmax(e, (double)FLT_EPSILON));
      frow[bin1] = v;
      csum1 += (double)v;
    }
    wave_lds_fence();  // the next frame overwrites buf
  }
  if (!cmn) return;  // block-uniform

  // CMN: per-utterance column means, combined over waves in a fixed order
  s_part[wave][lane] = csum0;  // waves without frames contribute zero
  if (has1) s_part[wave][bin1] = csum1;
  __syncthreads();
  if (tid < kNB) {
    double s = 0.0;
    for (int w = 0; w < kWaves; ++w) s += s_part[w][tid];
    s_mean[tid] = s / (double)T;
  }
  __syncthreads();
  float* f = feats + fbase * kNB;
  const long total = (long)T * kNB;
  for (long e = tid; e < total; e += kThreads) f[e] = (float)((double)f[e] - s_mean[e % kNB]);
}

// Host-side tables: f64 window / twiddles; the mel filters are torchaudio's
// float32 get_mel_banks values with a correctly rounded log
// (fbank_mel_table.h, made by tools/gen_fbank_mel_table.py), stored as doubles.
void fbank_tables(double* tab) {
  for (int i = 0; i < kTabSize; ++i) tab[i] = 0.0;
  const double kPi = 3.14159265358979323846;
  for (int n = 0; n < kFL; ++n) tab[kTabWin + n] = 0.54 - 0.46 * std::cos(2.0 * kPi * n / (kFL - 1));
  for (int m = 0; m < 256; ++m) {
    tab[kTabC256 + m] = std::cos(2.0 * kPi * m / 256.0);
    tab[kTabS256 + m] = std::sin(2.0 * kPi * m / 256.0);
    tab[kTabC512 + m] = std::cos(2.0 * kPi * m / 512.0);
    tab[kTabS512 + m] = std::sin(2.0 * kPi * m / 512.0);
  }
  for (int st = 0, ns = 4; st < 3; ++st, ns *= 4)
    for (int r = 1; r < 4; ++r)
      for (int j = 0; j < 64; ++j) {
        const int m = r * (j & (ns - 1)) * (64 / ns);
        tab[kTabTw + ((st * 3 + r - 1) * 64 + j) * 2] = tab[kTabC256 + m];
        tab[kTabTw + ((st * 3 + r - 1) * 64 + j) * 2 + 1] = tab[kTabS256 + m];
      }
  // mel filters: torchaudio get_mel_banks in float32 (generated table),
  // stored lane-interleaved and zero-padded (see kMelLen0 / kMelLen1)
  int o = 0;
  for (int b = 0; b < kNB; ++b) {
    const int len = b < 64 ? kMelLen0 : kMelLen1;
    WSP_CHECK(kMelLen[b] <= len && kMelStart[b] + len <= 256, "fbank: mel table overflow");
    tab[kTabStart + b] = kMelStart[b];
    tab[kTabLen + b] = kMelLen[b];
    tab[kTabOff + b] = o;
    for (int i = 0; i < kMelLen[b]; ++i, ++o)
      tab[b < 64 ? kTabW + i * 64 + b : kTabW1 + i * 16 + (b - 64)] = (double)kMelW[o];
  }
  WSP_CHECK(o == kMelWeights, "fbank: mel table size");
}

void launch_fbank(const void* wav, int dtype, int B, int N, int ld, float scale, float* feats,
                  int T, int cmn, const double* tables, hipStream_t s, const int* wseg, const int* fseg) {
  if (B == 0 || T == 0) return;
  WSP_CHECK((wseg == nullptr) == (fseg == nullptr), "fbank: sample and frame segments go together");
  if (dtype == 1)
    hipLaunchKernelGGL(fbank_cmn_kernel<1>, dim3(B), dim3(kThreads), 0, s, wav, N, ld, scale, feats, T, cmn,
                       tables, wseg, fseg);
  else
    hipLaunchKernelGGL(fbank_cmn_kernel<0>, dim3(B), dim3(kThreads), 0, s, wav, N, ld, scale, feats, T, cmn,
                       tables, wseg, fseg);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
