// Bandwidth-bound kernels around the MFMA convolutions: frame statistics,
// SE gating, residual, attentive-statistics pooling, small row-batched
// linears (SE FCs, GLOB context bias, BN-folded embedding head).
#include "kernels.h"

namespace wsp {

// ----------------------------------------------------------- small linear ---
// out[r][n] = post(act(bias[n] + sum_k in[r][k] * wt[k][n])).  One workgroup =
// kRB rows x 256 outputs; the kRB input rows are staged through LDS in 256-wide
// k chunks, the weight column is read coalesced (wt is k-major).
namespace {
constexpr int kRB = 8;
constexpr int kKC = 256;

__global__ __launch_bounds__(256) void small_linear_kernel(const SmallLinearArgs p) {
  __shared__ float s_in[kRB][kKC];
  const int tid = threadIdx.x;
  const int n = blockIdx.y * 256 + tid;
  const int r0 = blockIdx.x * kRB;
  float acc[kRB];
#pragma unroll
  for (int r = 0; r < kRB; ++r) acc[r] = 0.f;
  for (int k0 = 0; k0 < p.K; k0 += kKC) {
    const int kc = min(kKC, p.K - k0);
    for (int i = tid; i < kRB * kKC; i += 256) {
      const int r = i / kKC, k = i - r * kKC;
      s_in[r][k] = (r0 + r < p.R && k < kc) ? p.in[(long)(r0 + r) * p.ldin + k0 + k] : 0.f;
    }
    __syncthreads();
    if (n < p.N) {
      const float* w = p.wt + (long)k0 * p.N + n;
      int k = 0;
      for (; k + 4 <= kc; k += 4) {
        const float w0 = w[(long)k * p.N], w1 = w[(long)(k + 1) * p.N];
        const float w2 = w[(long)(k + 2) * p.N], w3 = w[(long)(k + 3) * p.N];
#pragma unroll
        for (int r = 0; r < kRB; ++r) {
          float a = acc[r];
          a = fmaf(s_in[r][k], w0, a);
          a = fmaf(s_in[r][k + 1], w1, a);
          a = fmaf(s_in[r][k + 2], w2, a);
          a = fmaf(s_in[r][k + 3], w3, a);
          acc[r] = a;
        }
      }
      for (; k < kc; ++k) {
        const float w0 = w[(long)k * p.N];
#pragma unroll
        for (int r = 0; r < kRB; ++r) acc[r] = fmaf(s_in[r][k], w0, acc[r]);
      }
    }
    __syncthreads();
  }
  if (n < p.N) {
    const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < kRB; ++r) {
      if (r0 + r >= p.R) break;
      float y = acc[r] + bv;
      if (p.act == 1) y = fmaxf(y, 0.f);
      else if (p.act == 2) y = tanhf(y);
      else if (p.act == 3) y = 1.f / (1.f + expf(-y));
      p.out[(long)(r0 + r) * p.ldo + n] = y;
    }
  }
}
}  // namespace

void launch_small_linear(const SmallLinearArgs& p, hipStream_t s) {
  if (p.R == 0) return;
  dim3 grid(ceil_div(p.R, kRB), ceil_div(p.N, 256));
  hipLaunchKernelGGL(small_linear_kernel, grid, dim3(256), 0, s, p);
  WSP_HIP(hipGetLastError());
}

// ------------------------------------------------------------ frame stats ---
// One workgroup = one utterance x 64 channels; 4 waves split the frames.
// Two passes (mean, then centred sum of squares) for an accurate unbiased
// variance (torch.var default, pooling_layers.py:81,131).
namespace {
__global__ __launch_bounds__(256) void frame_stats_kernel(const float* __restrict__ x, int ldx,
                                                          int T, int C, float* __restrict__ out,
                                                          int ldo, int with_std, int std_off) {
  __shared__ float part[4][64];
  __shared__ float s_mean[64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y * 64 + lane;
  const bool ok = c < C;
  const float* xb = x + (long)b * T * ldx + c;
  float s = 0.f;
  if (ok)
    for (int t = wave; t < T; t += 4) s += xb[(long)t * ldx];
  part[wave][lane] = s;
  __syncthreads();
  if (wave == 0) {
    const float m = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)T;
    s_mean[lane] = m;
    if (ok) out[(long)b * ldo + c] = m;
  }
  __syncthreads();
  if (!with_std) return;
  const float m = s_mean[lane];
  float q = 0.f;
  if (ok)
    for (int t = wave; t < T; t += 4) {
      const float d = xb[(long)t * ldx] - m;
      q = fmaf(d, d, q);
    }
  __syncthreads();
  part[wave][lane] = q;
  __syncthreads();
  if (wave == 0 && ok) {
    const float v = (part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane]) / (float)(T - 1);
    out[(long)b * ldo + std_off + c] = sqrtf(v + 1e-7f);
  }
}
}  // namespace

void launch_frame_stats(const float* x, int ldx, int B, int T, int C, float* out, int ldo,
                        int with_std, int std_off, hipStream_t s) {
  if (B == 0) return;
  dim3 grid(B, ceil_div(C, 64));
  hipLaunchKernelGGL(frame_stats_kernel, grid, dim3(256), 0, s, x, ldx, T, C, out, ldo, with_std,
                     std_off);
  WSP_HIP(hipGetLastError());
}

// --------------------------------------------------------- residual scale ---
namespace {
__global__ __launch_bounds__(256) void residual_scale_kernel(const f32x4* __restrict__ x,
                                                             const f32x4* __restrict__ h,
                                                             const float* __restrict__ g,
                                                             f32x4* __restrict__ out, long n4,
                                                             int T, int C4) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long row = i / C4;
    const int c4 = (int)(i - row * C4);
    const int b = (int)(row / T);
    const f32x4 gv = *reinterpret_cast<const f32x4*>(g + ((long)b * C4 + c4) * 4);
    out[i] = x[i] + h[i] * gv;
  }
}
}  // namespace

void launch_residual_scale(const float* x, const float* h, const float* g, float* out, int B,
                           int T, int C, hipStream_t s) {
  WSP_CHECK(C % 4 == 0, "residual_scale: C % 4");
  const long n4 = (long)B * T * C / 4;
  if (n4 == 0) return;
  const int grid = (int)std::min<long>(ceil_div((int)std::min<long>(n4, 1L << 30), 256), 256 * 16);
  hipLaunchKernelGGL(residual_scale_kernel, dim3(grid), dim3(256), 0, s,
                     reinterpret_cast<const f32x4*>(x), reinterpret_cast<const f32x4*>(h), g,
                     reinterpret_cast<f32x4*>(out), n4, T, C / 4);
  WSP_HIP(hipGetLastError());
}

// -------------------------------------------------------------- ASTP pool ---
// Online (max-rescaled) softmax over frames fused with the alpha-weighted
// first and second moments: one read of logits and features, no alpha tensor.
namespace {
__global__ __launch_bounds__(256) void astp_pool_kernel(const float* __restrict__ e,
                                                        const float* __restrict__ x, int T, int C,
                                                        float* __restrict__ out) {
  __shared__ float sm[4][4][64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y * 64 + lane;
  const bool ok = c < C;
  float mx = -INFINITY, se = 0.f, a1 = 0.f, a2 = 0.f;
  if (ok) {
    const long base = (long)b * T * C + c;
    for (int t = wave; t < T; t += 4) {
      const float ev = e[base + (long)t * C];
      const float xv = x[base + (long)t * C];
      if (ev > mx) {
        const float sc = expf(mx - ev);  // 0 on the first frame (mx = -inf)
        se = se * sc + 1.f;
        a1 = a1 * sc + xv;
        a2 = a2 * sc + xv * xv;
        mx = ev;
      } else {
        const float pe = expf(ev - mx);
        se += pe;
        a1 = fmaf(pe, xv, a1);
        a2 = fmaf(pe * xv, xv, a2);
      }
    }
  }
  sm[wave][0][lane] = mx;
  sm[wave][1][lane] = se;
  sm[wave][2][lane] = a1;
  sm[wave][3][lane] = a2;
  __syncthreads();
  if (wave == 0 && ok) {
    float M = sm[0][0][lane];
    for (int w = 1; w < 4; ++w) M = fmaxf(M, sm[w][0][lane]);
    float S = 0.f, A1 = 0.f, A2 = 0.f;
    for (int w = 0; w < 4; ++w) {
      const float m = sm[w][0][lane];
      const float f = (m == -INFINITY) ? 0.f : expf(m - M);
      S += sm[w][1][lane] * f;
      A1 += sm[w][2][lane] * f;
      A2 += sm[w][3][lane] * f;
    }
    const float mean = A1 / S;
    const float var = A2 / S - mean * mean;
    out[(long)b * 2 * C + c] = mean;
    out[(long)b * 2 * C + C + c] = sqrtf(fmaxf(var, 1e-7f));
  }
}
}  // namespace

void launch_astp_pool(const float* e, const float* x, int B, int T, int C, float* out,
                      hipStream_t s) {
  if (B == 0) return;
  dim3 grid(B, ceil_div(C, 64));
  hipLaunchKernelGGL(astp_pool_kernel, grid, dim3(256), 0, s, e, x, T, C, out);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
