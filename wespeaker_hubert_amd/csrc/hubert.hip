// HuBERT-base front-end kernels (s3prl `hubert` upstream as wrapped by
// wespeaker/frontend/s3prl.py:23-93; fairseq HuBERT semantics, restated in
// oracle/hubert_ref.py).  The dense contractions (conv1..6, projections, FFN,
// pos_conv) run on the implicit-GEMM MFMA kernels and self-attention on attn.hip;
// this file holds the rest:
//
//   conv0 + GroupNorm(512, 512) + GELU : waveform -> [B][T0][512]
//       (1 input channel, k10 s5: 10 MACs per output — VALU; the GroupNorm
//        statistics come from 65 f64 moments of the waveform, not from a pass over y)
//   layernorm  : rows of D in {512, 768}, optional (remapped) residual add,
//                optional s3prl Featurizer accumulation + length match
//   cmn_rows   : per-utterance mean removal over frames (dataset_utils.py:19-26)
#include <cfloat>

#include "kernels.h"

namespace wsp {

namespace {

// GELU: gelu_as (common.h, A&S 7.1.26 erf, |err| <= 2e-7) — conv0 evaluates one per output
__device__ __forceinline__ float gelu_erf(float x) { return gelu_as(x); }

// ---------------------------------------------------------------- conv0 ---
constexpr int kC0 = 512, kK0 = 10, kS0 = 5, kTC = 128;

// GroupNorm(512, 512) normalises every channel over the utterance's frames.  Its
// statistics need no pass over conv0's output: y_t[c] = sum_k w[c][k] x[5t + k], so
//   sum_t y_t[c]   = sum_k w[c][k] S_k,            S_k  = sum_t x[5t + k]
//   sum_t y_t[c]^2 = sum_jk w[c][j] w[c][k] R_jk,   R_jk = sum_t x[5t + j] x[5t + k]
// — 10 + 55 moments of the (strided) waveform per utterance (conv0_moments_kernel,
// f64), combined with each channel's weights where they are used (conv0_kernel).
// The former statistics pass recomputed conv0 for all 512 channels of every frame
// (0.8 ms of C4's 65 ms step); the moments read the waveform once.
constexpr int kNM = kK0 + kK0 * (kK0 + 1) / 2;  // 65 moments per utterance
constexpr int kMT = 1024;                        // frames per moments block

__global__ __launch_bounds__(256) void conv0_moments_kernel(const float* __restrict__ wav, int N_, int ldw, int T0_,
                                                            double* __restrict__ mom, const int* __restrict__ wseg,
                                                            const int* __restrict__ oseg) {
  __shared__ float xs[kMT * kS0 + kK0];
  __shared__ double red[4][kNM];
  const int b = blockIdx.y, t0 = blockIdx.x * kMT, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = wseg ? wseg[b + 1] - wseg[b] : N_;
  const int T0 = oseg ? oseg[b + 1] - oseg[b] : T0_;
  double* part = mom + ((size_t)b * gridDim.x + blockIdx.x) * kNM;  // this block's partial moments
  if (t0 >= T0) {  // block-uniform: past this utterance (ragged batch); its partials are zero
    if (tid < kNM) part[tid] = 0.0;
    return;
  }
  const float* x = wav + (wseg ? (size_t)wseg[b] : (size_t)b * ldw);
  for (int i = tid; i < kMT * kS0 + kK0; i += 256) {
    const int n = t0 * kS0 + i;
    xs[i] = n < N ? x[n] : 0.f;
  }
  __syncthreads();
  double m[kNM];
#pragma unroll
  for (int i = 0; i < kNM; ++i) m[i] = 0.0;
  const int nt = min(kMT, T0 - t0);
  for (int t = tid; t < nt; t += 256) {
    double v[kK0];
#pragma unroll
    for (int k = 0; k < kK0; ++k) v[k] = (double)xs[t * kS0 + k];
    int q = kK0;
#pragma unroll
    for (int j = 0; j < kK0; ++j) {
      m[j] += v[j];
#pragma unroll
      for (int k = j; k < kK0; ++k, ++q) m[q] = fma(v[j], v[k], m[q]);
    }
  }
  // fixed-order reduction: lanes (butterfly), waves (LDS), then one partial per moment and
  // block, summed in block order by conv0_kernel (deterministic: no atomics)
#pragma unroll
  for (int i = 0; i < kNM; ++i) {
    double v = m[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave][i] = v;
  }
  __syncthreads();
  if (tid < kNM) part[tid] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
}

// out = GELU(GroupNorm(y)).  One thread per channel, one block per (128-frame chunk,
// utterance); the waveform chunk is staged in LDS and read as a broadcast.
// Segmented batch (wseg / oseg non-null): utterance b = samples [wseg[b], wseg[b+1])
// -> output rows [oseg[b], oseg[b+1]); GroupNorm statistics per utterance as before.
__global__ __launch_bounds__(kC0) void conv0_kernel(const float* __restrict__ wav, int N_, int ldw, int T0_,
                                                    const float* __restrict__ w, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, const double* __restrict__ mom,
                                                    int nmb, float* __restrict__ out, const int* __restrict__ wseg,
                                                    const int* __restrict__ oseg) {
  __shared__ float xs[kTC * kS0 + kK0];
  __shared__ double ms[kNM];
  const int b = blockIdx.y, t0 = blockIdx.x * kTC, c = threadIdx.x;
  const int N = wseg ? wseg[b + 1] - wseg[b] : N_;
  const int T0 = oseg ? oseg[b + 1] - oseg[b] : T0_;
  if (t0 >= T0) return;  // block-uniform: past this utterance
  const float* x = wav + (wseg ? (size_t)wseg[b] : (size_t)b * ldw);
  const size_t obase = oseg ? (size_t)oseg[b] : (size_t)b * T0_;
  for (int i = c; i < kTC * kS0 + kK0; i += kC0) {
    const int n = t0 * kS0 + i;
    xs[i] = n < N ? x[n] : 0.f;
  }
  // the utterance's waveform moments: its moments blocks' partials summed in block order
  if (c < kNM) {
    const double* pm = mom + (size_t)b * nmb * kNM + c;
    double a = 0.0;
    for (int i = 0; i < (T0 + kMT - 1) / kMT; ++i) a += pm[(size_t)i * kNM];
    ms[c] = a;
  }
  float wr[kK0];
#pragma unroll
  for (int k = 0; k < kK0; ++k) wr[k] = w[c * kK0 + k];
  __syncthreads();
  // this channel's first and second moments from the utterance's waveform moments (f64;
  // var = E[y^2] - mean^2 is exact enough in f64 for fp32 outputs)
  float scale, shift;
  {
    const double* mo = ms;
    double s0 = 0.0, s1 = 0.0;
    int q = kK0;
#pragma unroll
    for (int j = 0; j < kK0; ++j) {
      const double wj = (double)wr[j];
      s0 = fma(wj, mo[j], s0);
#pragma unroll
      for (int k = j; k < kK0; ++k) s1 = fma((k == j ? 1.0 : 2.0) * wj * (double)wr[k], mo[q++], s1);
    }
    const double mean = s0 / T0;
    const double var = fmax(s1 / T0 - mean * mean, 0.0);
    const float rstd = (float)(1.0 / sqrt(var + 1e-5));
    scale = rstd * gamma[c];
    shift = beta[c] - (float)mean * scale;
  }
  __syncthreads();
  const int nt = min(kTC, T0 - t0);
  for (int t = 0; t < nt; ++t) {
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < kK0; ++k) y = fmaf(wr[k], xs[t * kS0 + k], y);
    out[(obase + t0 + t) * kC0 + c] = gelu_erf(fmaf(y, scale, shift));
  }
}

// ------------------------------------------------------------ layernorm ---
// One wave per row, 16-B accesses: lane owns channels 4*lane + 256*i (i < V4).
// The remapped residual (pos_conv's 64-wide group padding) keeps 4-aligned
// channel runs inside one group (gin % 4 == 0), so it is read as float4 too.
template <int V4>
__global__ __launch_bounds__(256) void layernorm_kernel(const LayerNormArgs p) {
  constexpr int D = V4 * 256;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  f32x4 v[V4];
  const float* x = p.x + (size_t)row * p.ldx;
#pragma unroll
  for (int i = 0; i < V4; ++i) v[i] = *reinterpret_cast<const f32x4*>(x + 4 * lane + 256 * i);
  if (p.add) {
    const float* a = p.add + (size_t)row * p.ldadd;
#pragma unroll
    for (int i = 0; i < V4; ++i) {
      const int c = 4 * lane + 256 * i;
      const int g = c / p.gin;
      v[i] += *reinterpret_cast<const f32x4*>(a + g * p.gout + (c - g * p.gin));
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < V4; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  const float mean = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[i][e] -= mean;
      q = fmaf(v[i][e], v[i][e], q);
    }
  const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / D) + p.eps);
  float* o = p.out + (size_t)row * p.ldo;
#pragma unroll
  for (int i = 0; i < V4; ++i) {
    const int c = 4 * lane + 256 * i;
    const f32x4 g = *reinterpret_cast<const f32x4*>(p.gamma + c);
    const f32x4 b = *reinterpret_cast<const f32x4*>(p.beta + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[i][e] = v[i][e] * rstd * g[e] + b[e];
    *reinterpret_cast<f32x4*>(o + c) = v[i];
  }
  if (p.feat) {
    // s3prl Featurizer: feat += w_l * h_l; length match replicates the last
    // frame up to Tout (and trims frames >= Tout).  Segmented: per utterance.
    int b, t, T, Tout;
    size_t fbase;
    if (p.seg) {
      b = seg_of(p.seg, p.nseg, row);
      t = row - p.seg[b];
      T = p.seg[b + 1] - p.seg[b];
      Tout = p.fseg[b + 1] - p.fseg[b];
      fbase = p.fseg[b];
    } else {
      b = row / p.T;
      t = row - b * p.T;
      T = p.T;
      Tout = p.Tout;
      fbase = (size_t)b * p.Tout;
    }
    const int t_end = (t == T - 1) ? Tout : min(t + 1, Tout);
    for (int tt = t; tt < t_end; ++tt) {
      float* f = p.feat + (fbase + tt) * D;
#pragma unroll
      for (int i = 0; i < V4; ++i) {
        f32x4* fp = reinterpret_cast<f32x4*>(f + 4 * lane + 256 * i);
        if (p.feat_init) {
          *fp = p.feat_w * v[i];
        } else {
          f32x4 acc = *fp;
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = fmaf(p.feat_w, v[i][e], acc[e]);
          *fp = acc;
        }
      }
    }
  }
}

// ------------------------------------------------------------- cmn_rows ---
// Block = (64 channels, utterance); 4 row groups of 64 lanes: coalesced
// 256-B row segments, partial sums combined through LDS.  mode bit 0: mean
// removal; bit 1: division by sqrt(unbiased variance + 1e-7) (apply_cmvn's
// norm_var, dataset_utils.py:24-25), the variance taken about the mean of the
// values as they are after bit 0 (torch.var centres itself).
__device__ __forceinline__ double cmn_block_sum(double s, double (*part)[64]) {
  part[threadIdx.x >> 6][threadIdx.x & 63] = s;
  __syncthreads();
  const int l = threadIdx.x & 63;
  const double r = part[0][l] + part[1][l] + part[2][l] + part[3][l];
  __syncthreads();  // part is reused by the next reduction
  return r;
}

__global__ __launch_bounds__(256) void cmn_rows_kernel(float* __restrict__ x, int T_, int D,
                                                       const int* __restrict__ seg, int mode) {
  // f64 partial sums in a fixed order (torch's float32 mean is cascade-summed,
  // i.e. ~exact; a plain f32 running sum drifts ~1e-5 at a few hundred frames)
  __shared__ double part[4][64];
  const int b = blockIdx.y, c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  float* p = x + (seg ? (size_t)seg[b] : (size_t)b * T_) * D + c;
  if (mode & 1) {
    double s = 0.0;
    if (c < D)
      for (int t = g; t < T; t += 4) s += (double)p[(size_t)t * D];
    const double mean = cmn_block_sum(s, part) / (double)T;
    if (c < D)
      for (int t = g; t < T; t += 4) p[(size_t)t * D] = (float)((double)p[(size_t)t * D] - mean);
  }
  if (mode & 2) {
    double s = 0.0;
    if (c < D)
      for (int t = g; t < T; t += 4) s += (double)p[(size_t)t * D];
    const double m = cmn_block_sum(s, part) / (double)T;
    double q = 0.0;
    if (c < D)
      for (int t = g; t < T; t += 4) {
        const double d = (double)p[(size_t)t * D] - m;
        q += d * d;
      }
    const double var = cmn_block_sum(q, part) / (double)(T - 1);  // T = 1: 0 / 0 = NaN, as torch.var
    const double inv = 1.0 / sqrt(var + 1e-7);
    if (c < D)
      for (int t = g; t < T; t += 4) p[(size_t)t * D] = (float)((double)p[(size_t)t * D] * inv);
  }
}

}  // namespace

void launch_hubert_conv0(const float* wav, int B, int N, int ldw, int T0, const float* w, const float* gamma,
                         const float* beta, double* stats, float* out, hipStream_t s, const int* wseg,
                         const int* oseg) {
  WSP_CHECK((wseg == nullptr) == (oseg == nullptr), "hubert conv0: sample and row segments go together");
  if (!wseg) {
    WSP_CHECK(B > 0 && T0 == (N - kK0) / kS0 + 1 && T0 > 0, "hubert conv0: bad frame count");
    WSP_CHECK(ldw >= N, "hubert conv0: ldw < N");
  }
  WSP_CHECK(B > 0 && T0 > 0, "hubert conv0: empty batch");  // segmented: T0 = longest utterance's frames
  // stats: hubert_conv0_stats_doubles(B, T0) partial moments, one set per (utterance, moments block)
  const int nmb = (T0 + kMT - 1) / kMT;
  hipLaunchKernelGGL(conv0_moments_kernel, dim3(nmb, B), dim3(256), 0, s, wav, N, ldw, T0, stats, wseg, oseg);
  hipLaunchKernelGGL(conv0_kernel, dim3((T0 + kTC - 1) / kTC, B), dim3(kC0), 0, s, wav, N, ldw, T0, w, gamma, beta,
                     stats, nmb, out, wseg, oseg);
  WSP_HIP(hipGetLastError());
}

size_t hubert_conv0_stats_doubles(int B, int T0) { return (size_t)B * ((T0 + kMT - 1) / kMT) * kNM; }

void launch_layernorm(const LayerNormArgs& p, hipStream_t s) {
  WSP_CHECK(p.M > 0 && (p.D == 512 || p.D == 768), "layernorm: D must be 512 or 768");
  WSP_CHECK(!p.add || (p.gin > 0 && p.gout >= p.gin && p.gin % 4 == 0 && p.gout % 4 == 0 && p.ldadd % 4 == 0),
            "layernorm: bad add remap");
  WSP_CHECK(p.ldx % 4 == 0 && p.ldo % 4 == 0, "layernorm: rows must be 16-B aligned");
  WSP_CHECK(!p.feat || p.seg || (p.T > 0 && p.Tout > 0 && p.M % p.T == 0), "layernorm: bad featurizer shape");
  WSP_CHECK(!p.seg || (p.fseg && p.nseg > 0), "layernorm: segmented featurizer needs output offsets");
  const dim3 grid((p.M + 3) / 4);
  if (p.D == 512)
    hipLaunchKernelGGL(layernorm_kernel<2>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(layernorm_kernel<3>, grid, dim3(256), 0, s, p);
  WSP_HIP(hipGetLastError());
}

void launch_cmn_rows(float* x, int B, int T, int D, hipStream_t s, const int* seg) {
  WSP_CHECK(B > 0 && (T > 0 || seg) && D > 0, "cmn: bad shape");
  hipLaunchKernelGGL(cmn_rows_kernel, dim3((D + 63) / 64, B), dim3(256), 0, s, x, T, D, seg, 1);
  WSP_HIP(hipGetLastError());
}

void launch_cmvn_rows(float* x, int B, int T, int D, int norm_mean, int norm_var, hipStream_t s, const int* seg) {
  WSP_CHECK(B > 0 && (T > 0 || seg) && D > 0, "cmvn: bad shape");
  const int mode = (norm_mean ? 1 : 0) | (norm_var ? 2 : 0);
  if (!mode) return;
  hipLaunchKernelGGL(cmn_rows_kernel, dim3((D + 63) / 64, B), dim3(256), 0, s, x, T, D, seg, mode);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
