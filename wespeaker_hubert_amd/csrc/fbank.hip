// Batched Kaldi log-mel fbank + fused CMN on gfx950.
//
// Restates torchaudio.compliance.kaldi.fbank as the reference calls it
// (wespeaker/cli/speaker.py:89-104, wespeaker/dataset/processor.py:472-502;
// native restatement runtime/core/frontend/fbank.h:138-198): snip-edges
// framing, DC removal, pre-emphasis 0.97 (replicate pad), the symmetric
// window of `window_type` (hamming / hanning / povey / rectangular / blackman,
// kaldi.py _feature_window_function), zero pad to the next power of two,
// real FFT, |X|^2, triangular mel filters (Nyquist weight 0),
// log(max(e, FLT_EPSILON)); then optional CMN (speaker.py:102-103 /
// dataset_utils.py:19-26).  Configurations: any num_mel_bins in 4..128 and
// any rate / frame length whose frame pads to 256 or 512 samples (8 kHz and
// 16 kHz at the recipes' 25 / 10 ms: examples/sre/v2,v3/conf/resnet.yaml use
// 40 / 64 bins at 8 kHz, voxceleb 80 at 16 kHz).
//
// Precision: everything from the DC mean to the mel energies runs in float64
// (the mel filter weights are torchaudio's float32 values, computed on the host
// by fbank_mel_banks below); the log is logf of the energy rounded to float32
// (the output is float32: ~1 output ulp against the f64 log's 0.5, at 15 %
// fewer instructions per frame).  The reference's own path is float32
// (torchaudio's fp32 rfft), which deviates from exact arithmetic by ~1e-4 on
// low-energy bins; this kernel sits ~1e-6 from the float64 oracle, i.e. it is
// never less accurate than the fp32 reference it replaces.  f64 costs little
// here: the whole fbank is ~12 kflop per frame, latency-bound.
//
// Layout: one workgroup (16 waves) = one utterance; wave w takes frames
// w, w+16, ... and loads the samples of its next frame while it transforms
// the current one.  Each wave owns a 256-entry complex f64 LDS buffer: a
// 512-point real FFT is a 256-point complex FFT of z[n] = y[2n] + i y[2n+1]
// (radix-4 Stockham, 4 in-place stages, one butterfly per lane; a wave's LDS
// ops execute in order, so a stage's reads of all lanes precede its writes
// and no workgroup barrier is needed) followed by the even/odd split; a
// 256-point real FFT (8 kHz) is the same 256-point complex FFT of z[n] = y[n]
// (the imaginary half idle: a non-headline configuration, one code path).  The
// per-utterance mel-column sums for CMN accumulate in registers (f64), are
// combined across waves in a fixed order (deterministic, batch-independent)
// and the block then subtracts the mean from its own (L2-hot) output: one
// launch, no second pass over HBM.  Output is channels-last (B, T, bins).
//
// The 80-bin 16 kHz 25 / 10 ms hamming configuration (every voxceleb recipe,
// the bench) is its own instance with the geometry and the padded filter
// lengths as compile-time constants (fully unrolled mel loops); the others
// read them from the plan.
#include <algorithm>
#include <cfloat>
#include <cmath>

#include "../../include/wespeaker_amd.h"
#include "kernels.h"

namespace wsp {

namespace {

constexpr int kWaves = 16, kThreads = kWaves * 64;

// table layout (doubles): window[512] | cos512[256] | sin512[256] |
//   tw[3][3][64][2] | start[128] | w0[len0][64] | w1[len1][W1S]
// tw: per-lane twiddles of FFT stages 1..3 as (cos, sin) pairs, [stage][r-1][lane]:
// lane-contiguous 16-B reads.  The mel filters are stored lane-interleaved and
// zero-padded to a fixed length per lane group: bins 0..63 as w0[i][64]
// (i < len0), bins 64.. as w1[i][W1S] (i < len1; W1S = 16 for the 80-bin
// instance, 64 otherwise).  Every lane of a group then runs the same loop,
// the weight reads are lane-contiguous (no bank conflicts), and the padded
// terms add w = 0 exactly (e + 0*p == e for the finite, non-negative sums),
// so the sums equal the sparse form's bit for bit.  start[b] is chosen so that
// start[b] + len <= padded / 2 (filters near Nyquist are shifted left and
// front-padded with zeros).
constexpr int kTabWin = 0, kTabC512 = 512, kTabS512 = 768, kTabTw = 1024, kTabStart = 2176, kTabW = 2304;
constexpr int kMaxBins = 128;
constexpr int kMaxMelRows = 96;  // len0 + len1 of a generic plan
constexpr int kTabMax = kTabW + kMaxMelRows * 64;
// the headline instance
constexpr int kFixFL = 400, kFixFS = 160, kFixNB = 80, kFixMel0 = 10, kFixMel1 = 16;
constexpr int kTabFixed = kTabW + kFixMel0 * 64 + kFixMel1 * 16;

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

// runtime geometry of a generic plan (ignored by the fixed instance)
struct FbankGeom {
  int fl, fs, nb, len0, len1, tab_doubles;
};

}  // namespace

// kN: padded FFT size (512: complex 256-point FFT of even / odd samples + split;
// 256: complex 256-point FFT of the real frame).  kFixed: the headline geometry.
template <int kDtype, int kN, bool kFixed>
__global__ __launch_bounds__(kThreads) void fbank_cmn_kernel(const void* __restrict__ wav, int ld, float scale,
                                                             float* __restrict__ feats, int T_, int cmn,
                                                             const double* __restrict__ tab,
                                                             const int* __restrict__ wseg,
                                                             const int* __restrict__ fseg, FbankGeom g) {
  static_assert(kN == 512 || kN == 256, "fbank: padded size");
  static_assert(!kFixed || kN == 512, "fbank: fixed instance is 512-point");
  constexpr int kNB = kFixed ? kFixNB : kMaxBins;
  constexpr int kTabN = kFixed ? kTabFixed : kTabMax;
  constexpr int kW1S = kFixed ? 16 : 64;
  __shared__ double s_tab[kTabN];
  __shared__ double2 s_buf[kWaves][256];
  __shared__ double s_part[kWaves][kNB];
  __shared__ double s_mean[kNB];

  const int fl = kFixed ? kFixFL : g.fl;
  const int fs = kFixed ? kFixFS : g.fs;
  const int nb = kFixed ? kFixNB : g.nb;
  const int len0 = kFixed ? kFixMel0 : g.len0;
  const int len1 = kFixed ? kFixMel1 : g.len1;
  const int ntab = kFixed ? kTabFixed : g.tab_doubles;

  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // uniform batch: utterance b = samples [b*ld, ...), frames [b*T_, (b+1)*T_);
  // segmented batch: samples [wseg[b], wseg[b+1]), frames [fseg[b], fseg[b+1])
  const long wbase = wseg ? (long)wseg[b] : (long)b * ld;
  const long fbase = fseg ? (long)fseg[b] : (long)b * T_;
  const int T = fseg ? fseg[b + 1] - fseg[b] : T_;
  if (T <= 0) return;  // block-uniform

  for (int i = tid; i < ntab; i += kThreads) s_tab[i] = tab[i];
  __syncthreads();

  const double* win = s_tab + kTabWin;
  const double2* tw = reinterpret_cast<const double2*>(s_tab + kTabTw);
  const double* c512 = s_tab + kTabC512;
  const double* s512 = s_tab + kTabS512;
  const double* w0 = s_tab + kTabW;
  const double* w1 = w0 + len0 * 64;
  double2* buf = s_buf[wave];
  double* pw = reinterpret_cast<double*>(buf);
  const double dscale = (double)scale;

  // mel bins of this lane: bin0 = lane (< nb), bin1 = lane + 64 (< nb)
  const int bin1 = lane + 64;
  const bool has0 = kFixed || lane < nb;
  const bool has1 = bin1 < nb;
  const int st0 = has0 ? (int)s_tab[kTabStart + lane] : 0;
  const int st1 = has1 ? (int)s_tab[kTabStart + bin1] : 0;
  double csum0 = 0.0, csum1 = 0.0;

  // raw samples of the wave's next frame, loaded one frame ahead so their
  // latency hides behind the current frame's FFT (PCM16 and f32 values are
  // exact in f32).  kN = 512: ne / no = y[2n] / y[2n+1]; kN = 256: ne = y[n].
  float ne[4], no[4];
  auto fetch = [&](int t) {
    const long x0 = wbase + (long)t * fs;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      ne[q] = no[q] = 0.f;
      if (kN == 512) {
        if (2 * n < fl) ne[q] = (float)load_sample<kDtype>(wav, x0 + 2 * n);
        if (2 * n + 1 < fl) no[q] = (float)load_sample<kDtype>(wav, x0 + 2 * n + 1);
      } else if (n < fl) {
        ne[q] = (float)load_sample<kDtype>(wav, x0 + n);
      }
    }
  };
  if (wave < T) fetch(wave);

  for (int t = wave; t < T; t += kWaves) {
    // 1. samples (n = lane + 64q); out-of-frame entries are 0
    double xe[4], xo[4], xp[4];
    double sum = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      xe[q] = (double)ne[q] * dscale;
      xo[q] = (double)no[q] * dscale;
      if (kN == 512) {
        if (2 * n < fl) sum += xe[q] + xo[q];
      } else if (n < fl) {
        sum += xe[q];
      }
    }
    if (t + kWaves < T) fetch(t + kWaves);
    // the previous sample: kN = 512: y[2n-1] is the odd sample of element n-1
    // (lane-1's xo, wave_shr:1, or lane 63's xo of the previous q); kN = 256:
    // y[n-1] likewise from xe; n = 0 replicates y[0] (pre-emphasis pad)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const double* src = kN == 512 ? xo : xe;
      xp[q] = wave_shr1(src[q], q > 0 ? readlane63(src[q - 1]) : xe[0]);
    }
    // 2. DC removal, pre-emphasis, window (f64; exact sums for PCM16 input)
    const double mean = wave_sum_f64(sum) * (1.0 / fl);
    // z[n] for n = lane + 64q stays in registers: it is exactly what the first
    // Stockham stage's butterfly of this lane reads (a[r] = z[lane + 64 r])
    double2 zin[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = lane + 64 * q;
      double2 z = make_double2(0.0, 0.0);
      if (kN == 512) {
        const double de = xe[q] - mean, dd = xo[q] - mean, dp = xp[q] - mean;
        if (2 * n < fl) z.x = (de - 0.97 * dp) * win[2 * n];
        if (2 * n + 1 < fl) z.y = (dd - 0.97 * de) * win[2 * n + 1];
      } else if (n < fl) {
        const double de = xe[q] - mean, dp = xp[q] - mean;
        z.x = (de - 0.97 * dp) * win[n];
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
      if (kN == 512 || ns < 64) {  // kN = 256 reads only its own-lane last-stage outputs
        buf[zsw(d)] = o0;
        buf[zsw(d + ns)] = o1;
        buf[zsw(d + 2 * ns)] = o2;
        buf[zsw(d + 3 * ns)] = o3;
      }
      if (ns == 64) {  // d = j: outputs j, j + 64, j + 128, j + 192
        zl[0] = o0;
        zl[1] = o1;
        zl[2] = o2;
        zl[3] = o3;
      }
      wave_lds_fence();
    }
    // 4. power |X[k]|^2 for k = lane + 64 q (the Nyquist weight is 0).  kN = 512:
    // even / odd split of Z -> X[k], k = 0..255; kN = 256: X = Z, k = 0..127 used
    double pk[4];
    if (kN == 512) {
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
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) pk[q] = zl[q].x * zl[q].x + zl[q].y * zl[q].y;
    }
    wave_lds_fence();
#pragma unroll
    for (int q = 0; q < 4; ++q) pw[lane + 64 * q] = pk[q];
    wave_lds_fence();
    // 5. mel filter bank + log (lane -> bins lane, lane + 64)
    float* frow = feats + (fbase + t) * nb;
    if (has0) {
      double e = 0.0;
      if (kFixed) {
#pragma unroll
        for (int i = 0; i < kFixMel0; ++i) e += w0[i * 64 + lane] * pw[st0 + i];
      } else {
        for (int i = 0; i < len0; ++i) e += w0[i * 64 + lane] * pw[st0 + i];
      }
      const float v = logf((float)fmax(e, (double)FLT_EPSILON));
      frow[lane] = v;
      csum0 += (double)v;
    }
    if (has1) {
      double e = 0.0;
      if (kFixed) {
#pragma unroll
        for (int i = 0; i < kFixMel1; ++i) e += w1[i * kW1S + (lane & (kW1S - 1))] * pw[st1 + i];
      } else {
        for (int i = 0; i < len1; ++i) e += w1[i * kW1S + (lane & (kW1S - 1))] * pw[st1 + i];
      }
      const float v = logf((float)fmax(e, (double)FLT_EPSILON));
      frow[bin1] = v;
      csum1 += (double)v;
    }
    wave_lds_fence();  // the next frame overwrites buf
  }
  if (!cmn) return;  // block-uniform

  // CMN: per-utterance column means, combined over waves in a fixed order
  if (has0) s_part[wave][lane] = csum0;  // waves without frames contribute zero
  if (has1) s_part[wave][bin1] = csum1;
  __syncthreads();
  if (tid < nb) {
    double s = 0.0;
    for (int w = 0; w < kWaves; ++w) s += s_part[w][tid];
    s_mean[tid] = s / (double)T;
  }
  __syncthreads();
  float* f = feats + fbase * nb;
  const long total = (long)T * nb;
  for (long e = tid; e < total; e += kThreads) f[e] = (float)((double)f[e] - s_mean[e % nb]);
}

// ------------------------------------------------------------------ host ---

void fbank_config_resolve(FbankConfig& c) {
  WSP_CHECK(c.num_bins > 3 && c.num_bins <= kMaxBins, "fbank: num_mel_bins must be in 4..128");
  WSP_CHECK(c.sample_rate > 0, "fbank: bad sample rate");
  WSP_CHECK(c.window >= WSP_WINDOW_HAMMING && c.window <= WSP_WINDOW_BLACKMAN, "fbank: unknown window type");
  // kaldi.py _get_waveform_and_window_properties: int(sr * ms * MILLISECONDS_TO_SECONDS)
  c.frame_len = (int)((double)c.sample_rate * c.frame_length_ms * 0.001);
  c.frame_shift = (int)((double)c.sample_rate * c.frame_shift_ms * 0.001);
  WSP_CHECK(c.frame_len >= 2 && c.frame_shift >= 1, "fbank: frame length / shift too small");
  int p = 1;
  while (p < c.frame_len) p <<= 1;  // round_to_power_of_two
  c.padded = p;
  WSP_CHECK(p == 256 || p == 512,
            "fbank: the frame must pad to 256 or 512 samples (e.g. 25 ms at 8 or 16 kHz)");
  const double nyq = 0.5 * c.sample_rate;
  const double hi = c.high_freq <= 0.0 ? c.high_freq + nyq : c.high_freq;
  WSP_CHECK(c.low_freq >= 0.0 && c.low_freq < nyq && hi > 0.0 && hi <= nyq && c.low_freq < hi,
            "fbank: bad low / high frequency");
}

// torchaudio.compliance.kaldi.get_mel_banks (published kaldi.py, no VTLN) in its
// arithmetic: python-double mel_low / delta scalars rounded to float32, then
// float32 tensor ops in kaldi.py's order; mel_scale's float32 log taken
// correctly rounded (torch's CPU float32 log is SLEEF-u10 and host-dependent).
// No FMA contraction: each float op rounds as torch's elementwise kernels do.
void fbank_mel_banks(const FbankConfig& c, std::vector<float>& w) {
#pragma clang fp contract(off)
  const int nfft = c.padded / 2;
  const double nyq = 0.5 * c.sample_rate;
  const double high = c.high_freq <= 0.0 ? c.high_freq + nyq : c.high_freq;
  const double fft_bin_width = (double)c.sample_rate / c.padded;
  const double mel_low = 1127.0 * std::log(1.0 + c.low_freq / 700.0);
  const double mel_high = 1127.0 * std::log(1.0 + high / 700.0);
  const float delta = (float)((mel_high - mel_low) / (c.num_bins + 1));
  const float lowf = (float)mel_low;
  std::vector<float> mel(nfft);
  for (int i = 0; i < nfft; ++i) {
    const float prod = (float)fft_bin_width * (float)i;
    const float x = 1.0f + prod / 700.0f;
    const float lg = (float)std::log((double)x);
    mel[i] = 1127.0f * lg;
  }
  w.assign((size_t)c.num_bins * (nfft + 1), 0.f);
  for (int b = 0; b < c.num_bins; ++b) {
    const float bf = (float)b;
    const float l_ = bf * delta;
    const float c1 = bf + 1.0f;
    const float c_ = c1 * delta;
    const float r1 = bf + 2.0f;
    const float r_ = r1 * delta;
    const float left = lowf + l_, center = lowf + c_, right = lowf + r_;
    for (int i = 0; i < nfft; ++i) {
      const float upn = mel[i] - left, upd = center - left;
      const float dnn = right - mel[i], dnd = right - center;
      const float up = upn / upd, down = dnn / dnd;
      const float v = std::fmax(0.f, std::fmin(up, down));
      w[(size_t)b * (nfft + 1) + i] = v;
    }
  }
}

void fbank_plan(const FbankConfig& cin, FbankPlan& p) {
  p.cfg = cin;
  FbankConfig& c = p.cfg;
  fbank_config_resolve(c);
  p.fixed = c.num_bins == kFixNB && c.frame_len == kFixFL && c.frame_shift == kFixFS && c.padded == 512 &&
            c.window == WSP_WINDOW_HAMMING && c.low_freq == 20.0 && c.high_freq == 0.0 && c.sample_rate == 16000;
  const int nb = c.num_bins, half = c.padded / 2;
  // sparse mel filters: first / last nonzero weight per bin
  std::vector<float> w;
  fbank_mel_banks(c, w);
  std::vector<int> lo(nb, 0), len(nb, 0);
  for (int b = 0; b < nb; ++b) {
    int first = -1, last = -1;
    for (int i = 0; i < half; ++i)
      if (w[(size_t)b * (half + 1) + i] > 0.f) {
        if (first < 0) first = i;
        last = i;
      }
    lo[b] = first < 0 ? 0 : first;
    len[b] = first < 0 ? 0 : last - first + 1;
  }
  int l0 = 0, l1 = 0;
  for (int b = 0; b < nb; ++b) (b < 64 ? l0 : l1) = std::max(b < 64 ? l0 : l1, len[b]);
  if (p.fixed) {
    WSP_CHECK(l0 <= kFixMel0 && l1 <= kFixMel1, "fbank: headline mel filters wider than the fixed instance");
    l0 = kFixMel0;
    l1 = kFixMel1;
  }
  WSP_CHECK(l0 + l1 <= kMaxMelRows, "fbank: mel filters too wide (num_mel_bins too small for this FFT size)");
  WSP_CHECK(l0 <= half && l1 <= half, "fbank: mel filter longer than the spectrum");
  p.len0 = l0;
  p.len1 = l1;
  const int w1s = p.fixed ? 16 : 64;
  const int ntab = kTabW + l0 * 64 + l1 * w1s;
  p.host_tab.assign(ntab, 0.0);
  double* tab = p.host_tab.data();
  // window (kaldi.py _feature_window_function, symmetric, in f64)
  const double kPi = 3.14159265358979323846;
  const int L = c.frame_len;
  for (int n = 0; n < L; ++n) {
    const double a = 2.0 * kPi * n / (L - 1);
    double v = 1.0;
    switch (c.window) {
      case WSP_WINDOW_HAMMING: v = 0.54 - 0.46 * std::cos(a); break;
      case WSP_WINDOW_HANNING: v = 0.5 - 0.5 * std::cos(a); break;
      case WSP_WINDOW_POVEY: v = std::pow(0.5 - 0.5 * std::cos(a), 0.85); break;
      case WSP_WINDOW_RECTANGULAR: v = 1.0; break;
      case WSP_WINDOW_BLACKMAN: v = 0.42 - 0.5 * std::cos(a) + 0.08 * std::cos(2.0 * a); break;
    }
    tab[kTabWin + n] = v;
  }
  for (int m = 0; m < 256; ++m) {
    tab[kTabC512 + m] = std::cos(2.0 * kPi * m / 512.0);
    tab[kTabS512 + m] = std::sin(2.0 * kPi * m / 512.0);
  }
  for (int st = 0, ns = 4; st < 3; ++st, ns *= 4)
    for (int r = 1; r < 4; ++r)
      for (int j = 0; j < 64; ++j) {
        const int m = r * (j & (ns - 1)) * (64 / ns);
        tab[kTabTw + ((st * 3 + r - 1) * 64 + j) * 2] = std::cos(2.0 * kPi * m / 256.0);
        tab[kTabTw + ((st * 3 + r - 1) * 64 + j) * 2 + 1] = std::sin(2.0 * kPi * m / 256.0);
      }
  // mel filters, lane-interleaved and zero-padded; a filter whose padded span
  // would pass the spectrum end starts earlier (front zeros)
  for (int b = 0; b < nb; ++b) {
    const int glen = b < 64 ? l0 : l1;
    const int st = std::min(lo[b], half - glen);
    tab[kTabStart + b] = st;
    for (int i = 0; i < len[b]; ++i) {
      const int slot = lo[b] - st + i;
      const double v = (double)w[(size_t)b * (half + 1) + lo[b] + i];
      if (b < 64)
        tab[kTabW + slot * 64 + b] = v;
      else
        tab[kTabW + l0 * 64 + slot * w1s + (b - 64)] = v;
    }
  }
}

void launch_fbank(const void* wav, int dtype, int B, int N, int ld, float scale, float* feats, int T, int cmn,
                  const FbankPlan& p, hipStream_t s, const int* wseg, const int* fseg) {
  (void)N;
  if (B == 0 || T == 0) return;
  WSP_CHECK((wseg == nullptr) == (fseg == nullptr), "fbank: sample and frame segments go together");
  WSP_CHECK(p.tab != nullptr, "fbank: plan has no device table");
  const FbankGeom g{p.cfg.frame_len, p.cfg.frame_shift, p.cfg.num_bins, p.len0, p.len1, (int)p.host_tab.size()};
  WSP_CHECK(g.tab_doubles <= kTabMax, "fbank: table too large");
#define WSP_FBANK_LAUNCH(DT, NN, FX)                                                                             \
  hipLaunchKernelGGL((fbank_cmn_kernel<DT, NN, FX>), dim3(B), dim3(kThreads), 0, s, wav, ld, scale, feats, T, cmn, \
                     p.tab, wseg, fseg, g)
  if (p.fixed) {
    if (dtype == 1)
      WSP_FBANK_LAUNCH(1, 512, true);
    else
      WSP_FBANK_LAUNCH(0, 512, true);
  } else if (p.cfg.padded == 512) {
    if (dtype == 1)
      WSP_FBANK_LAUNCH(1, 512, false);
    else
      WSP_FBANK_LAUNCH(0, 512, false);
  } else {
    if (dtype == 1)
      WSP_FBANK_LAUNCH(1, 256, false);
    else
      WSP_FBANK_LAUNCH(0, 256, false);
  }
#undef WSP_FBANK_LAUNCH
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
