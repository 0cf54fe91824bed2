// SimAM-ResNet helpers (wespeaker/models/samresnet.py): the parameter-free
// SimAM attention of every SimAMBasicBlock and the (B,C,F,T) -> (B,C*F,T)
// regrouping in front of ASP pooling.  All HBM-bound.
//
//   SimAM(X) = X * sigmoid((X - mean)^2 / (4 (v + 1e-4)) + 0.5),
//   mean / v over the F*T positions of each (utterance, channel), v with the
//   n - 1 divisor (samresnet.py:64-69); the block output is
//   relu(SimAM(bn2(conv2(.))) + shortcut)  (samresnet.py:56-62).
#include "kernels.h"

namespace wsp {

namespace {
// Partial first / second moments: block (b, chunk) sums rows
// [chunk*rows_per, min(rows, (chunk+1)*rows_per)) of utterance b in f64.
// A thread owns 4 channels (16-B loads); tpr = C/4 threads per row, 256/tpr
// rows per pass.  part[b][chunk][2][C].
__global__ __launch_bounds__(256) void simam_moments_kernel(const float* __restrict__ z, int rows, int C,
                                                            int rows_per, double* __restrict__ part) {
  __shared__ double red[2][256 * 4];
  const int b = blockIdx.x, chunk = blockIdx.y, nchunk = gridDim.y;
  const int tpr = C >> 2, rp = 256 / tpr;
  const int tid = threadIdx.x, cg = tid % tpr, r0 = tid / tpr;
  const int lo = chunk * rows_per, hi = min(rows, lo + rows_per);
  const float* zb = z + (long)b * rows * C + cg * 4;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  int r = lo + r0;
  for (; r + rp < hi; r += 2 * rp) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(zb + (long)r * C);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(zb + (long)(r + rp) * C);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double a = v0[e], c = v1[e];
      s1[e] += a + c;
      s2[e] += a * a + c * c;
    }
  }
  if (r < hi) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(zb + (long)r * C);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double a = v0[e];
      s1[e] += a;
      s2[e] += a * a;
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    red[0][r0 * C + cg * 4 + e] = s1[e];
    red[1][r0 * C + cg * 4 + e] = s2[e];
  }
  __syncthreads();
  double* out = part + ((long)b * nchunk + chunk) * 2 * C;
  for (int c = tid; c < C; c += 256) {
    double a = 0.0, q = 0.0;
    for (int k = 0; k < rp; ++k) {  // fixed order: deterministic
      a += red[0][k * C + c];
      q += red[1][k * C + c];
    }
    out[c] = a;
    out[C + c] = q;
  }
}

// coef[b][c] = mean, coef[b][C + c] = 1 / (4 (var_{n-1} + lambda)); chunks summed in order.
__global__ __launch_bounds__(256) void simam_coef_kernel(const double* __restrict__ part, int nchunk, int rows,
                                                         int C, float* __restrict__ coef) {
  const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
  if (c >= C) return;
  double s1 = 0.0, s2 = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const double* p = part + ((long)b * nchunk + k) * 2 * C;
    s1 += p[c];
    s2 += p[C + c];
  }
  const double n = (double)rows;
  const double mean = s1 / n;
  const double var = fmax(s2 - s1 * mean, 0.0) / (n - 1.0);
  coef[(long)b * 2 * C + c] = (float)mean;
  coef[(long)b * 2 * C + C + c] = (float)(1.0 / (4.0 * ((double)(float)var + 1e-4)));
}

// out = relu(z * sigmoid((z - mean)^2 * k + 0.5) + res), [B][rows][C] f32x4-wise.
__global__ __launch_bounds__(256) void simam_apply_kernel(const f32x4* __restrict__ z, const float* __restrict__ coef,
                                                          const f32x4* __restrict__ res, f32x4* __restrict__ out,
                                                          long n4, long per_utt4, int C4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long b = i / per_utt4;
    const int c4 = (int)(i % C4);
    const f32x4 m = *reinterpret_cast<const f32x4*>(coef + b * 8 * C4 + c4 * 4);
    const f32x4 k = *reinterpret_cast<const f32x4*>(coef + b * 8 * C4 + 4 * C4 + c4 * 4);
    const f32x4 v = z[i], r = res[i];
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = v[e] - m[e];
      const float ei = d * d * k[e] + 0.5f;
      const float g = 1.f / (1.f + expf(-ei));
      y[e] = fmaxf(fmaf(v[e], g, r[e]), 0.f);
    }
    out[i] = y;
  }
}

// [B][F][T][C] -> [B][T][F][C] (16-B granules)
__global__ __launch_bounds__(256) void nhwc_to_tfc_kernel(const f32x4* __restrict__ in, f32x4* __restrict__ out, int F,
                                                          int T, int C4, long n4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const int c4 = (int)(i % C4);
    long q = i / C4;
    const int f = (int)(q % F);
    q /= F;
    const int t = (int)(q % T);
    const long b = q / T;
    out[i] = in[((b * F + f) * T + t) * C4 + c4];
  }
}

int grid_for(long n4) { return (int)std::min<long>((n4 + 255) / 256, 256L * 16); }
}  // namespace

int simam_chunks(int B, int rows) {
  int nchunk = std::max(1, ceil_div(2048, std::max(B, 1)));
  nchunk = std::min(nchunk, std::max(1, rows / 64));
  return nchunk;
}

void launch_simam(const float* z, const float* res, float* out, int B, int rows, int C, double* part, float* coef,
                  hipStream_t s) {
  WSP_CHECK(C % 4 == 0 && C <= 1024 && 256 % (C / 4) == 0, "simam: C must be 4 * a divisor of 256");
  WSP_CHECK(rows >= 2, "simam: need >= 2 positions per channel");
  if (B == 0) return;
  const int nchunk = simam_chunks(B, rows);
  const int rows_per = ceil_div(rows, nchunk);
  hipLaunchKernelGGL(simam_moments_kernel, dim3(B, nchunk), dim3(256), 0, s, z, rows, C, rows_per, part);
  WSP_HIP(hipGetLastError());
  hipLaunchKernelGGL(simam_coef_kernel, dim3(B, ceil_div(C, 256)), dim3(256), 0, s, part, nchunk, rows, C, coef);
  WSP_HIP(hipGetLastError());
  const long n4 = (long)B * rows * C / 4;
  hipLaunchKernelGGL(simam_apply_kernel, dim3(grid_for(n4)), dim3(256), 0, s, reinterpret_cast<const f32x4*>(z), coef,
                     reinterpret_cast<const f32x4*>(res), reinterpret_cast<f32x4*>(out), n4, (long)rows * C / 4,
                     C / 4);
  WSP_HIP(hipGetLastError());
}

void launch_nhwc_to_tfc(const float* in, float* out, int B, int F, int T, int C, hipStream_t s) {
  WSP_CHECK(C % 4 == 0, "nhwc_to_tfc: C % 4");
  const long n4 = (long)B * F * T * C / 4;
  if (n4 == 0) return;
  hipLaunchKernelGGL(nhwc_to_tfc_kernel, dim3(grid_for(n4)), dim3(256), 0, s, reinterpret_cast<const f32x4*>(in),
                     reinterpret_cast<f32x4*>(out), F, T, C / 4, n4);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
