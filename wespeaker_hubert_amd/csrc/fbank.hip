// Batched Kaldi log-mel fbank + CMN on gfx950.
//
// Restates torchaudio.compliance.kaldi.fbank as the reference calls it
// (wespeaker/cli/speaker.py:89-104, wespeaker/dataset/processor.py:472-502;
// native restatement runtime/core/frontend/fbank.h:138-198): snip-edges
// framing 400/160, DC removal, pre-emphasis 0.97 (replicate pad), symmetric
// Hamming window, zero pad to 512, real FFT, |X|^2, 80 triangular mel
// filters (Nyquist weight 0), log(max(e, FLT_EPSILON)); then optional CMN
// (speaker.py:102-103 / dataset_utils.py:19-26).
//
// Layout: one workgroup (4 waves) = 16 consecutive frames of one utterance.
// The 2 800 overlapping samples are staged once in LDS (coalesced), each wave
// takes 4 frames.  The 512-point real FFT is a 256-point complex FFT of
// z[n] = y[2n] + i y[2n+1] (radix-4 Stockham, 4 stages, one butterfly per
// lane, LDS ping-pong) followed by the even/odd split; the power spectrum and
// the sparse mel filter bank are evaluated from LDS.  Output is channels-last
// (B, T, 80) = exactly the reference's feature layout.
#include <cfloat>
#include <cmath>

#include "kernels.h"

namespace wsp {

namespace {

constexpr int kFL = 400, kFS = 160, kNB = 80, kFPB = 16;
constexpr int kSeg = (kFPB - 1) * kFS + kFL;  // 2800 samples per workgroup

}  // namespace

// tables layout (floats): window[400] | cos256 | sin256 | cos512 | sin512 |
//   start[80] | len[80] | off[80] (ints stored as int32 bit patterns) | w[...]
constexpr int kTabWin = 0, kTabC256 = 400, kTabS256 = 656, kTabC512 = 912, kTabS512 = 1168,
              kTabStart = 1424, kTabLen = 1504, kTabOff = 1584, kTabW = 1664;
constexpr int kTabSize = kTabW + 1024;

__global__ __launch_bounds__(256) void fbank_kernel(const void* __restrict__ wav, int dtype, int N_,
                                                    int ld, float scale, float* __restrict__ feats,
                                                    int T_, const float* __restrict__ tab,
                                                    const int* __restrict__ wseg,
                                                    const int* __restrict__ fseg) {
  __shared__ __attribute__((aligned(16))) float s_tab[kTabSize];
  __shared__ float s_x[kSeg];
  __shared__ __attribute__((aligned(16))) float2 s_buf[4][2][256];

  const int b = blockIdx.x;
  const int t0 = blockIdx.y * kFPB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // uniform batch: utterance b = samples [b*ld, b*ld + N_), frames [b*T_, (b+1)*T_);
  // segmented batch: samples [wseg[b], wseg[b+1]), frames [fseg[b], fseg[b+1])
  const long wbase = wseg ? (long)wseg[b] : (long)b * ld;
  const int N = wseg ? wseg[b + 1] - wseg[b] : N_;
  const long fbase = fseg ? (long)fseg[b] : (long)b * T_;
  const int T = fseg ? fseg[b + 1] - fseg[b] : T_;
  if (t0 >= T) return;  // block-uniform: past this utterance's frames

  for (int i = tid; i < kTabSize; i += 256) s_tab[i] = tab[i];
  const long start = (long)t0 * kFS;
  const int avail = (int)min((long)kSeg, (long)N - start);
  for (int i = tid; i < kSeg; i += 256) {
    float v = 0.f;
    if (i < avail) {
      if (dtype == 1)
        v = (float)reinterpret_cast<const short*>(wav)[wbase + start + i];
      else
        v = reinterpret_cast<const float*>(wav)[wbase + start + i];
    }
    s_x[i] = v * scale;
  }
  __syncthreads();

  const float* win = s_tab + kTabWin;
  const float* c256 = s_tab + kTabC256;
  const float* s256 = s_tab + kTabS256;
  const float* c512 = s_tab + kTabC512;
  const float* s512 = s_tab + kTabS512;
  const int* bstart = reinterpret_cast<const int*>(s_tab + kTabStart);
  const int* blen = reinterpret_cast<const int*>(s_tab + kTabLen);
  const int* boff = reinterpret_cast<const int*>(s_tab + kTabOff);
  const float* bw = s_tab + kTabW;
  float2* buf0 = s_buf[wave][0];
  float2* buf1 = s_buf[wave][1];
  float* real0 = reinterpret_cast<float*>(buf0);

  // Uniform control flow: every wave runs 4 frame slots (barriers below are
  // workgroup-wide); slots past T compute on zeros and store nothing.
  for (int slot = 0; slot < kFPB / 4; ++slot) {
    const int f = wave + 4 * slot;
    const int t = t0 + f;
    const float* x = s_x + f * kFS;
    // 1. DC offset (mean over the 400-sample frame)
    float sum = 0.f;
    for (int i = lane; i < kFL; i += 64) sum += x[i];
    const float mean = wave_sum(sum) * (1.0f / kFL);
    // 2. pre-emphasis on the DC-removed frame, then the window; zero pad
    for (int i = lane; i < 512; i += 64) {
      float y = 0.f;
      if (i < kFL) {
        const float xd = x[i] - mean;
        const float xp = (i == 0) ? xd : (x[i - 1] - mean);
        y = (xd - 0.97f * xp) * win[i];
      }
      real0[i] = y;
    }
    __syncthreads();
    // 3. 256-point complex FFT, radix-4 Stockham (4 stages)
    float2* in = buf0;
    float2* out = buf1;
#pragma unroll
    for (int ns = 1; ns < 256; ns *= 4) {
      const int j = lane;
      const int k = j & (ns - 1);
      float2 a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = in[j + 64 * r];
      if (ns > 1) {
#pragma unroll
        for (int r = 1; r < 4; ++r) {
          const int m = r * k * (64 / ns);
          const float c = c256[m], s = s256[m];
          // a *= exp(-i 2 pi m / 256) = c - i s
          const float re = a[r].x * c + a[r].y * s;
          const float im = a[r].y * c - a[r].x * s;
          a[r] = make_float2(re, im);
        }
      }
      const float2 s02 = make_float2(a[0].x + a[2].x, a[0].y + a[2].y);
      const float2 d02 = make_float2(a[0].x - a[2].x, a[0].y - a[2].y);
      const float2 s13 = make_float2(a[1].x + a[3].x, a[1].y + a[3].y);
      const float2 d13 = make_float2(a[1].x - a[3].x, a[1].y - a[3].y);
      // -i * d13 = (d13.y, -d13.x)
      const int d = (j / ns) * ns * 4 + k;
      out[d] = make_float2(s02.x + s13.x, s02.y + s13.y);
      out[d + ns] = make_float2(d02.x + d13.y, d02.y - d13.x);
      out[d + 2 * ns] = make_float2(s02.x - s13.x, s02.y - s13.y);
      out[d + 3 * ns] = make_float2(d02.x - d13.y, d02.y + d13.x);
      __syncthreads();
      float2* tmp = in;
      in = out;
      out = tmp;
    }
    // after 4 stages the spectrum Z is back in buf0 (in == buf0)
    // 4. even/odd split -> X[k], power |X[k]|^2 for k = 0..255 (into buf1)
    float* pw = reinterpret_cast<float*>(buf1);
    float pk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = lane + 64 * q;
      const float2 z = in[k];
      const float2 zc = in[(256 - k) & 255];  // conj taken below
      // Xe = (Z + conj(Zc))/2 ; Xo = -i (Z - conj(Zc))/2
      const float er = 0.5f * (z.x + zc.x), ei = 0.5f * (z.y - zc.y);
      const float dr = 0.5f * (z.x - zc.x), di = 0.5f * (z.y + zc.y);
      const float or_ = di, oi = -dr;
      const float c = c512[k], s = s512[k];  // W^k = c - i s
      const float xr = er + (or_ * c + oi * s);
      const float xi = ei + (oi * c - or_ * s);
      pk[q] = xr * xr + xi * xi;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) pw[lane + 64 * q] = pk[q];
    __syncthreads();
    // 5. mel filter bank + log
    if (t < T) {
      for (int bin = lane; bin < kNB; bin += 64) {
        const int s0 = bstart[bin], n = blen[bin], o = boff[bin];
        float e = 0.f;
        for (int i = 0; i < n; ++i) e += bw[o + i] * pw[s0 + i];
        e = fmaxf(e, FLT_EPSILON);
        feats[(fbase + t) * kNB + bin] = logf(e);
      }
    }
    __syncthreads();
  }
}

// CMN: subtract the per-utterance mean over frames.  One workgroup per
// utterance; 80 columns x 3 frame groups.
__global__ __launch_bounds__(256) void cmn_kernel(float* __restrict__ feats, int T_,
                                                  const int* __restrict__ fseg) {
  __shared__ float part[3][kNB];
  __shared__ float mean[kNB];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = fseg ? fseg[b + 1] - fseg[b] : T_;
  float* f = feats + (fseg ? (long)fseg[b] : (long)b * T_) * kNB;
  const int c = tid % kNB, g = tid / kNB;
  if (g < 3) {
    float s = 0.f;
    for (int t = g; t < T; t += 3) s += f[t * kNB + c];
    part[g][c] = s;
  }
  __syncthreads();
  if (tid < kNB) mean[tid] = (part[0][tid] + part[1][tid] + part[2][tid]) / (float)T;
  __syncthreads();
  if (g < 3)
    for (int t = g; t < T; t += 3) f[t * kNB + c] -= mean[c];
}

// Host-side tables, mirroring torchaudio's float32 get_mel_banks /
// hamming_window(periodic=False) arithmetic (kaldi.py).
void fbank_tables(float* tab) {
  for (int i = 0; i < kTabSize; ++i) tab[i] = 0.f;
  const double kPi = 3.14159265358979323846;
  for (int n = 0; n < kFL; ++n) tab[kTabWin + n] = (float)(0.54 - 0.46 * std::cos(2.0 * kPi * n / (kFL - 1)));
  for (int m = 0; m < 256; ++m) {
    tab[kTabC256 + m] = (float)std::cos(2.0 * kPi * m / 256.0);
    tab[kTabS256 + m] = (float)std::sin(2.0 * kPi * m / 256.0);
    tab[kTabC512 + m] = (float)std::cos(2.0 * kPi * m / 512.0);
    tab[kTabS512 + m] = (float)std::sin(2.0 * kPi * m / 512.0);
  }
  const double mel_low = 1127.0 * std::log(1.0 + 20.0 / 700.0);
  const double mel_high = 1127.0 * std::log(1.0 + 8000.0 / 700.0);
  const float delta = (float)((mel_high - mel_low) / (kNB + 1));
  int* start = reinterpret_cast<int*>(tab + kTabStart);
  int* len = reinterpret_cast<int*>(tab + kTabLen);
  int* off = reinterpret_cast<int*>(tab + kTabOff);
  int o = 0;
  for (int b = 0; b < kNB; ++b) {
    const float left = (float)b * delta + (float)mel_low;
    const float center = ((float)b + 1.0f) * delta + (float)mel_low;
    const float right = ((float)b + 2.0f) * delta + (float)mel_low;
    int first = -1, last = -1;
    float w[256];
    for (int i = 0; i < 256; ++i) {
      const float freq = 31.25f * (float)i;
      const float mel = 1127.0f * logf(1.0f + freq / 700.0f);
      const float up = (mel - left) / (center - left);
      const float down = (right - mel) / (right - center);
      w[i] = fmaxf(0.f, fminf(up, down));
      if (w[i] > 0.f) {
        if (first < 0) first = i;
        last = i;
      }
    }
    if (first < 0) first = last = 0;
    start[b] = first;
    len[b] = last - first + 1;
    off[b] = o;
    for (int i = first; i <= last; ++i) tab[kTabW + o++] = w[i];
  }
}

void launch_fbank(const void* wav, int dtype, int B, int N, int ld, float scale, float* feats,
                  int T, int cmn, const float* tables, hipStream_t s, const int* wseg, const int* fseg) {
  if (B == 0 || T == 0) return;
  WSP_CHECK((wseg == nullptr) == (fseg == nullptr), "fbank: sample and frame segments go together");
  dim3 grid(B, (T + kFPB - 1) / kFPB);  // T = frames of the longest utterance when segmented
  hipLaunchKernelGGL(fbank_kernel, grid, dim3(256), 0, s, wav, dtype, N, ld, scale, feats, T,
                     tables, wseg, fseg);
  WSP_HIP(hipGetLastError());
  if (cmn) {
    hipLaunchKernelGGL(cmn_kernel, dim3(B), dim3(256), 0, s, feats, T, fseg);
    WSP_HIP(hipGetLastError());
  }
}

}  // namespace wsp
