// Scoring back end on gfx950: L2 normalisation, cosine trials, AS-Norm
// cohort statistics (exact top-n via an in-workgroup radix select), and
// grouped embedding sums (mean vector / per-speaker cohort means).
//
// Reference: bin/score.py:25-72, bin/score_norm.py:26-36 (get_mean_std),
// tools/vector_mean.py:24-53.  The reference sorts every row of the
// N_eval x N_cohort score matrix (np.sort) and keeps top_n; here the k-th
// largest score is found by a 4-pass 8-bit radix select over order-preserving
// integer keys, then mean/std of the top_n multiset are accumulated in f64.
#include "kernels.h"

namespace wsp {

namespace {

__global__ __launch_bounds__(256) void l2_normalize_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ sub,
                                                           float* __restrict__ y, int D) {
  __shared__ double part[4];
  const int r = blockIdx.x, tid = threadIdx.x;
  double s = 0.0;
  for (int d = tid; d < D; d += 256) {
    const float v = x[(long)r * D + d] - (sub ? sub[d] : 0.f);
    s += (double)v * v;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) part[tid >> 6] = s;
  __syncthreads();
  const double nrm = sqrt(part[0] + part[1] + part[2] + part[3]);
  const float inv = (float)(1.0 / nrm);
  for (int d = tid; d < D; d += 256) {
    const float v = x[(long)r * D + d] - (sub ? sub[d] : 0.f);
    y[(long)r * D + d] = v * inv;
  }
}

__global__ __launch_bounds__(256) void cosine_pairs_kernel(const float* __restrict__ E, int D,
                                                           const int32_t* __restrict__ ia,
                                                           const int32_t* __restrict__ ib, int P,
                                                           double* __restrict__ score) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= P) return;
  const float* a = E + (long)ia[p] * D;
  const float* b = E + (long)ib[p] * D;
  double ab = 0.0, aa = 0.0, bb = 0.0;
  for (int d = lane; d < D; d += 64) {
    const double x = a[d], y = b[d];
    ab += x * y;
    aa += x * x;
    bb += y * y;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ab += __shfl_xor(ab, o, 64);
    aa += __shfl_xor(aa, o, 64);
    bb += __shfl_xor(bb, o, 64);
  }
  if (lane == 0) score[p] = ab / (sqrt(aa) * sqrt(bb));
}

__device__ __forceinline__ unsigned fkey(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// One workgroup per row of S [Ne][lds]; first Nc entries valid.
__global__ __launch_bounds__(256) void topn_stats_kernel(const float* __restrict__ S, long lds,
                                                         int Nc, int top_n, double* __restrict__ mu,
                                                         double* __restrict__ sd) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_kk;
  __shared__ double red[2][4];
  const int r = blockIdx.x, tid = threadIdx.x;
  const float* row = S + (long)r * lds;
  unsigned prefix = 0, mask = 0, kk = (unsigned)top_n;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int i = tid; i < Nc; i += 256) {
      const unsigned k = fkey(row[i]);
      if ((k & mask) == prefix) atomicAdd(&hist[(k >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned above = 0;
      int d = 255;
      for (; d > 0; --d) {
        if (above + hist[d] >= kk) break;
        above += hist[d];
      }
      s_prefix = prefix | ((unsigned)d << shift);
      s_kk = kk - above;
    }
    __syncthreads();
    prefix = s_prefix;
    kk = s_kk;
    mask |= 0xFFu << shift;
    __syncthreads();
  }
  // prefix = key of the top_n-th largest score; (top_n - kk) scores are strictly greater.
  const float v = fkey_inv(prefix);
  const unsigned n_gt = (unsigned)top_n - kk;
  double s = 0.0;
  for (int i = tid; i < Nc; i += 256) {
    const float x = row[i];
    if (fkey(x) > prefix) s += x;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((tid & 63) == 0) red[0][tid >> 6] = s;
  __syncthreads();
  const double tot = red[0][0] + red[0][1] + red[0][2] + red[0][3] + (double)(top_n - n_gt) * v;
  const double mean = tot / top_n;
  double q = 0.0;
  for (int i = tid; i < Nc; i += 256) {
    const float x = row[i];
    if (fkey(x) > prefix) {
      const double d = x - mean;
      q += d * d;
    }
  }
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  if ((tid & 63) == 0) red[1][tid >> 6] = q;
  __syncthreads();
  if (tid == 0) {
    const double dv = v - mean;
    const double var = (red[1][0] + red[1][1] + red[1][2] + red[1][3] + (double)(top_n - n_gt) * dv * dv) / top_n;
    mu[r] = mean;
    sd[r] = sqrt(var);
  }
}

__global__ void pad_rows_kernel(const float* __restrict__ src, int R, int D, float* __restrict__ dst,
                                int Rp, int Dp) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= (long)Rp * Dp) return;
  const int r = (int)(i / Dp), d = (int)(i - (long)r * Dp);
  dst[i] = (r < R && d < D) ? src[(long)r * D + d] : 0.f;
}

__global__ __launch_bounds__(256) void row_accum_kernel(const float* __restrict__ x,
                                                        const int32_t* __restrict__ group, int D,
                                                        double* __restrict__ acc,
                                                        double* __restrict__ cnt) {
  const int r = blockIdx.x;
  const int g = group[r];
  for (int d = threadIdx.x; d < D; d += 256) atomicAdd(&acc[(long)g * D + d], (double)x[(long)r * D + d]);
  if (threadIdx.x == 0) atomicAdd(&cnt[g], 1.0);
}

}  // namespace

void launch_l2_normalize(const float* x, const float* sub, float* y, int R, int D, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(l2_normalize_kernel, dim3(R), dim3(256), 0, s, x, sub, y, D);
  WSP_HIP(hipGetLastError());
}

void launch_cosine_pairs(const float* E, int D, const int32_t* ia, const int32_t* ib, int P,
                         double* score, hipStream_t s) {
  if (P == 0) return;
  hipLaunchKernelGGL(cosine_pairs_kernel, dim3(ceil_div(P, 4)), dim3(256), 0, s, E, D, ia, ib, P,
                     score);
  WSP_HIP(hipGetLastError());
}

static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

void asnorm_layout(int Ne, int Nc, int D, int* Ncp, int* Dp, size_t* bytes) {
  *Ncp = round_up(Nc, 128);
  *Dp = round_up(D, 32);
  *bytes = ((size_t)(*Ncp) * (*Dp) + (size_t)Ne * (*Ncp)) * sizeof(float) + 256;
}

void launch_asnorm_stats(const float* E, int Ne, const float* C, int Nc, int D, int top_n,
                         double* mu, double* sd, float* ws, hipStream_t s) {
  WSP_CHECK(top_n >= 1 && top_n <= Nc, "asnorm: need 1 <= top_n <= Nc");
  WSP_CHECK(D % 4 == 0, "asnorm: D must be a multiple of 4");
  int Ncp, Dp;
  size_t bytes;
  asnorm_layout(Ne, Nc, D, &Ncp, &Dp, &bytes);
  float* Cp = ws;
  float* S = ws + (size_t)Ncp * Dp;
  const long n = (long)Ncp * Dp;
  hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, C, Nc, D,
                     Cp, Ncp, Dp);
  WSP_HIP(hipGetLastError());
  ConvGemmArgs g{};
  g.a[0] = g.a[1] = g.a[2] = E;
  g.lda[0] = g.lda[1] = g.lda[2] = D;
  g.cseg[0] = 0;
  g.cseg[1] = g.cseg[2] = g.cseg[3] = D;
  g.cin = D;
  g.taps = 1;
  g.dil = 1;
  g.pad = 0;
  g.M = Ne;
  g.T = Ne;
  g.N = Ncp;
  g.w = Cp;
  g.K = D;
  g.Kp = Dp;
  g.out = S;
  g.ldo = Ncp;
  g.act = kActNone;
  g.amode = kACat;
  launch_conv_gemm(g, s);
  hipLaunchKernelGGL(topn_stats_kernel, dim3(Ne), dim3(256), 0, s, S, (long)Ncp, Nc, top_n, mu, sd);
  WSP_HIP(hipGetLastError());
}

void launch_row_mean_accum(const float* x, const int32_t* group, int R, int D, double* acc,
                           double* cnt, hipStream_t s) {
  if (R == 0) return;
  hipLaunchKernelGGL(row_accum_kernel, dim3(R), dim3(256), 0, s, x, group, D, acc, cnt);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
