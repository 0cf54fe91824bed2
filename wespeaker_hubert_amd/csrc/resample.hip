// Band-limited sinc (Hann window) resampling — the torchaudio.transforms.Resample
// the reference applies before fbank (wespeaker/cli/speaker.py:155-157,
// wespeaker/dataset/processor.py:242-260).  Algorithm restated in
// oracle/resample_ref.py (torchaudio's published default: sinc_interp_hann,
// lowpass_filter_width 6, rolloff 0.99):
//   y[n*new + j] = sum_k kern[j][k] * x[n*orig + k - width]
// The [new][2*width + orig] f32 kernel is built once per rate pair on the host
// (f64 arithmetic, like torchaudio) with each phase's nonzero tap band, so an
// output sample costs ~2*lpw*orig/base taps (the clamped taps are exactly 0).
// One thread per output sample, fp32 accumulation (torch conv1d is fp32);
// neighbouring outputs share input samples through L1.  HBM-bound.
#include <algorithm>
#include <cmath>
#include <numeric>
#include <vector>

#include "kernels.h"

namespace wsp {

namespace {
__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ x, int N, long ldx,
                                                       const float* __restrict__ kern, const int2* __restrict__ band,
                                                       int L, int orig, int nw, int width, float* __restrict__ y,
                                                       long ldy, int Nout) {
  const int o = blockIdx.x * 256 + threadIdx.x;
  if (o >= Nout) return;
  const int b = blockIdx.y;
  const int n = o / nw;
  const int j = o - n * nw;
  const int2 bd = band[j];
  const float* xb = x + (long)b * ldx;
  const float* kr = kern + (long)j * L;
  const int s0 = n * orig - width;
  float acc = 0.f;
  for (int k = bd.x; k < bd.y; ++k) {
    const int s = s0 + k;
    if ((unsigned)s < (unsigned)N) acc = fmaf(kr[k], xb[s], acc);
  }
  y[(long)b * ldy + o] = acc;
}
}  // namespace

void resample_plan(int orig_freq, int new_freq, int lowpass_filter_width, double rolloff, ResamplePlan& p) {
  WSP_CHECK(orig_freq > 0 && new_freq > 0, "resample: rates must be positive");
  WSP_CHECK(lowpass_filter_width > 0, "resample: lowpass_filter_width must be positive");
  WSP_CHECK(rolloff > 0.0 && rolloff <= 1.0, "resample: rolloff must be in (0, 1]");
  const int g = std::gcd(orig_freq, new_freq);
  p.orig = orig_freq / g;
  p.nw = new_freq / g;
  p.identity = orig_freq == new_freq;
  const double base = std::min(p.orig, p.nw) * rolloff;
  p.width = (int)std::ceil(lowpass_filter_width * (double)p.orig / base);
  p.L = 2 * p.width + p.orig;
  WSP_CHECK((long long)p.nw * p.L <= (1LL << 26), "resample: rate pair too large (reduce the rates' ratio)");
  p.kern.assign((size_t)p.nw * p.L, 0.f);
  p.band.assign((size_t)p.nw * 2, 0);
  const double pi = 3.14159265358979323846;
  for (int j = 0; j < p.nw; ++j) {
    int lo = p.L, hi = 0;
    for (int k = 0; k < p.L; ++k) {
      double t = ((double)(k - p.width) / p.orig - (double)j / p.nw) * base;
      t = std::max(-(double)lowpass_filter_width, std::min((double)lowpass_filter_width, t));
      const double c = std::cos(t * pi / lowpass_filter_width / 2);
      const double w = c * c;
      const double tp = t * pi;
      const double s = tp == 0.0 ? 1.0 : std::sin(tp) / tp;
      const float v = (float)(s * w * (base / p.orig));
      p.kern[(size_t)j * p.L + k] = v;
      if (v != 0.f) {
        lo = std::min(lo, k);
        hi = k + 1;
      }
    }
    p.band[2 * j] = lo < hi ? lo : 0;
    p.band[2 * j + 1] = lo < hi ? hi : 0;
  }
}

long long resample_out_len(const ResamplePlan& p, long long n) {
  if (p.identity) return n;
  return (p.nw * n + p.orig - 1) / p.orig;
}

void launch_resample(const ResamplePlan& p, const float* d_kern, const int* d_band, const float* x, int B, int N,
                     long ldx, float* y, long ldy, hipStream_t s) {
  WSP_CHECK(B >= 0 && N >= 0 && ldx >= N, "resample: bad input shape");
  const long long nout = resample_out_len(p, N);
  WSP_CHECK(nout < (1LL << 31), "resample: output too long");
  WSP_CHECK(ldy >= nout, "resample: ldy < output length");
  if (B == 0 || N == 0) return;
  if (p.identity) {
    WSP_HIP(hipMemcpy2DAsync(y, ldy * sizeof(float), x, ldx * sizeof(float), (size_t)N * sizeof(float), B,
                             hipMemcpyDeviceToDevice, s));
    return;
  }
  const dim3 grid((unsigned)((nout + 255) / 256), B);
  hipLaunchKernelGGL(resample_kernel, grid, dim3(256), 0, s, x, N, ldx, d_kern,
                     reinterpret_cast<const int2*>(d_band), p.L, p.orig, p.nw, p.width, y, ldy, (int)nout);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
