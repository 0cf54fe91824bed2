// Bandwidth-bound kernels around the MFMA convolutions: frame statistics,
// SE gating, residual, attentive-statistics pooling, small row-batched
// linears (SE FCs, GLOB context bias, BN-folded embedding head).
#include "kernels.h"

namespace wsp {

// ----------------------------------------------------------- small linear ---
// out[r][n] = act(bias[n] + sum_k in[r][k] * wt[k][n]) for the row-batched
// GEMVs (SE FCs, GLOB context bias, BN-folded embedding heads): R = batch rows,
// K up to ~20k (ResNet293's 20480-wide TSTP statistics).  One workgroup = kRB
// rows x 64 outputs (lane = output, coalesced k-major weight reads); its kSW
// waves split K (short per-wave dependency chains: latency, not bandwidth, bounds
// these) and reduce through LDS in a fixed order.  Input rows are wave-uniform.
namespace {
constexpr int kRB = 4;
constexpr int kSW = 16;

__global__ __launch_bounds__(64 * kSW) void small_linear_kernel(const SmallLinearArgs p) {
  __shared__ float part[kSW][kRB][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n = blockIdx.y * 64 + lane;
  const int r0 = blockIdx.x * kRB;
  const int kq = (p.K + kSW - 1) / kSW;
  const int k0 = wave * kq, k1 = min(p.K, k0 + kq);
  float acc[kRB];
#pragma unroll
  for (int r = 0; r < kRB; ++r) acc[r] = 0.f;
  const float* in[kRB];
#pragma unroll
  for (int r = 0; r < kRB; ++r) in[r] = p.in + (long)min(r0 + r, p.R - 1) * p.ldin;
  if (n < p.N) {
    const float* w = p.wt + n;
    int k = k0;
    for (; k + 4 <= k1; k += 4) {
      const float w0 = w[(long)k * p.N], w1 = w[(long)(k + 1) * p.N];
      const float w2 = w[(long)(k + 2) * p.N], w3 = w[(long)(k + 3) * p.N];
#pragma unroll
      for (int r = 0; r < kRB; ++r) {
        float a = acc[r];
        a = fmaf(in[r][k], w0, a);
        a = fmaf(in[r][k + 1], w1, a);
        a = fmaf(in[r][k + 2], w2, a);
        a = fmaf(in[r][k + 3], w3, a);
        acc[r] = a;
      }
    }
    for (; k < k1; ++k) {
      const float w0 = w[(long)k * p.N];
#pragma unroll
      for (int r = 0; r < kRB; ++r) acc[r] = fmaf(in[r][k], w0, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kRB; ++r) part[wave][r][lane] = acc[r];
  __syncthreads();
  if (wave < kRB && n < p.N) {  // wave r finishes row r
    const int r = wave;
    if (r0 + r >= p.R) return;
    float y = 0.f;
#pragma unroll
    for (int w = 0; w < kSW; ++w) y += part[w][r][lane];
    y += p.bias ? p.bias[n] : 0.f;
    if (p.act == 1) y = fmaxf(y, 0.f);
    else if (p.act == 2) y = tanhf(y);
    else if (p.act == 3) y = 1.f / (1.f + expf(-y));
    p.out[(long)(r0 + r) * p.ldo + n] = y;
  }
}

// Split-K form for long K (r5; the ResNet / SimAM heads, K = F/8 x 2 x C = 10-20k): block
// (row block of 16, 64 columns, k slice) -> partial sums part[slice][row][col]; the 16 waves split
// the slice and reduce through LDS in wave order.  The one-pass kernel above ran 64 blocks, each
// row block re-reading the whole weight matrix (C3: 0.29 ms per head launch).
constexpr int kSKR = 16;  // rows per split-K block
__global__ __launch_bounds__(64 * kSW) void small_linear_splitk_kernel(const SmallLinearArgs p, int kslice) {
  __shared__ float part[kSW][kSKR][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int n = blockIdx.y * 64 + lane;
  const int r0 = blockIdx.x * kSKR;
  const int ks = blockIdx.z;
  const int kb = ks * kslice, ke = min(p.K, kb + kslice);
  const int kq = (ke - kb + kSW - 1) / kSW;
  const int k0 = kb + wave * kq, k1 = min(ke, k0 + kq);
  float acc[kSKR];
#pragma unroll
  for (int r = 0; r < kSKR; ++r) acc[r] = 0.f;
  if (n < p.N) {
    const float* w = p.wt + n;
    for (int k = k0; k < k1; ++k) {
      const float wk = w[(long)k * p.N];
#pragma unroll
      for (int r = 0; r < kSKR; ++r) acc[r] = fmaf(p.in[(long)min(r0 + r, p.R - 1) * p.ldin + k], wk, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < kSKR; ++r) part[wave][r][lane] = acc[r];
  __syncthreads();
  // waves 0 .. kSKR - 1: wave r sums row r over the 16 waves in order
  if (wave < kSKR && n < p.N && r0 + wave < p.R) {
    float y = 0.f;
#pragma unroll
    for (int w = 0; w < kSW; ++w) y += part[w][wave][lane];
    p.scratch[((size_t)ks * p.R + r0 + wave) * p.N + n] = y;
  }
}

__global__ __launch_bounds__(256) void small_linear_reduce_kernel(const SmallLinearArgs p, int nks) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= p.R * p.N) return;
  const int r = i / p.N, n = i - r * p.N;
  float y = 0.f;
  for (int ks = 0; ks < nks; ++ks) y += p.scratch[(size_t)ks * p.R * p.N + i];
  y += p.bias ? p.bias[n] : 0.f;
  if (p.act == 1) y = fmaxf(y, 0.f);
  else if (p.act == 2) y = tanhf(y);
  else if (p.act == 3) y = 1.f / (1.f + expf(-y));
  p.out[(long)r * p.ldo + n] = y;
}
}  // namespace

size_t small_linear_scratch_floats(int R, int N, int K) {
  if (K < 4096) return 0;
  const int kslice = std::max(256, (ceil_div(K, 32) + 63) / 64 * 64);
  return (size_t)ceil_div(K, kslice) * R * N;
}

void launch_small_linear(const SmallLinearArgs& p, hipStream_t s) {
  if (p.R == 0) return;
  const int rb = ceil_div(p.R, kSKR), nb = ceil_div(p.N, 64);
  // 32 k slices (of >= 256): the slicing depends on K alone, so every row sums its products in
  // the same order whatever the batch (rows of a batch equal their batch-of-one results)
  if (p.scratch && p.K >= 4096) {
    const int kslice = std::max(256, (ceil_div(p.K, 32) + 63) / 64 * 64);
    const int nks = ceil_div(p.K, kslice);
    // a caller offering scratch must offer enough (small_linear_scratch_floats): falling back to
    // the one-pass kernel would sum in another order, and a batch would no longer equal its
    // batch-of-one rows
    WSP_CHECK((size_t)nks * p.R * p.N <= p.scratch_floats, "small_linear: split-K scratch too small");
    hipLaunchKernelGGL(small_linear_splitk_kernel, dim3(rb, nb, nks), dim3(64 * kSW), 0, s, p, kslice);
    WSP_HIP(hipGetLastError());
    hipLaunchKernelGGL(small_linear_reduce_kernel, dim3(ceil_div(p.R * p.N, 256)), dim3(256), 0, s, p, nks);
    WSP_HIP(hipGetLastError());
    return;
  }
  dim3 grid(ceil_div(p.R, kRB), ceil_div(p.N, 64));
  hipLaunchKernelGGL(small_linear_kernel, grid, dim3(64 * kSW), 0, s, p);
  WSP_HIP(hipGetLastError());
}

// ------------------------------------------------------------ frame stats ---
// One workgroup = one utterance x 64 channels; 4 waves split the frames.
// Two passes (mean, then centred sum of squares) for an accurate unbiased
// variance (torch.var default, pooling_layers.py:81,131).
namespace {
__global__ __launch_bounds__(256) void frame_stats_kernel(const float* __restrict__ x, int ldx,
                                                          int T_, int C, float* __restrict__ out,
                                                          int ldo, int with_std, int std_off,
                                                          const int* __restrict__ seg) {
  __shared__ float part[4][64];
  __shared__ float s_mean[64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y * 64 + lane;
  const bool ok = c < C;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  const float* xb = x + (seg ? (long)seg[b] : (long)b * T_) * ldx + c;
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

// Vector form (C, ldx multiples of 4): a lane owns 4 channels (16-B loads), a
// wave every 4th frame, 4 frames in flight per lane.  Sums in f64: the mean is
// then (up to rounding ties) the correctly rounded one whatever the summation
// order, so it matches the fused conv3-epilogue SE sums (colsum partials) and a
// utterance gets the same statistics in any batch.
__global__ __launch_bounds__(256) void frame_stats4_kernel(const float* __restrict__ x, int ldx, int T_,
                                                           int C, float* __restrict__ out, int ldo,
                                                           int with_std, int std_off,
                                                           const int* __restrict__ seg) {
  __shared__ double part[4][4][64];
  __shared__ float s_mean[4][64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = (blockIdx.y * 64 + lane) * 4;
  const bool ok = c < C;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  const float* xb = x + (seg ? (long)seg[b] : (long)b * T_) * ldx + (ok ? c : 0);
  auto row = [&](int t) { return *reinterpret_cast<const f32x4*>(xb + (long)t * ldx); };
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  int t = wave;
  if (ok) {
    for (; t + 12 < T; t += 16) {
      const f32x4 r0 = row(t), r1 = row(t + 4), r2 = row(t + 8), r3 = row(t + 12);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += ((double)r0[e] + (double)r1[e]) + ((double)r2[e] + (double)r3[e]);
    }
    for (; t < T; t += 4) {
      const f32x4 r0 = row(t);
#pragma unroll
      for (int e = 0; e < 4; ++e) a[e] += (double)r0[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) part[wave][e][lane] = a[e];
  __syncthreads();
  if (wave == 0) {
    f32x4 m;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      m[e] = (float)((part[0][e][lane] + part[1][e][lane] + part[2][e][lane] + part[3][e][lane]) / (double)T);
      s_mean[e][lane] = m[e];
    }
    if (ok) *reinterpret_cast<f32x4*>(out + (long)b * ldo + c) = m;
  }
  __syncthreads();
  if (!with_std) return;
  double q[4] = {0.0, 0.0, 0.0, 0.0};
  float m[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) m[e] = s_mean[e][lane];
  if (ok)
    for (t = wave; t < T; t += 4) {
      const f32x4 r0 = row(t);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double d = (double)(r0[e] - m[e]);
        q[e] += d * d;
      }
    }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < 4; ++e) part[wave][e][lane] = q[e];
  __syncthreads();
  if (wave == 0 && ok) {
    f32x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const double v = (part[0][e][lane] + part[1][e][lane] + part[2][e][lane] + part[3][e][lane]) / (double)(T - 1);
      r[e] = sqrtf((float)v + 1e-7f);
    }
    float* o = out + (long)b * ldo + std_off + c;
    if (((ldo | std_off) & 3) == 0) *reinterpret_cast<f32x4*>(o) = r;
    else for (int e = 0; e < 4; ++e) o[e] = r[e];
  }
}
}  // namespace

void launch_frame_stats(const float* x, int ldx, int B, int T, int C, float* out, int ldo,
                        int with_std, int std_off, hipStream_t s, const int* seg) {
  if (B == 0) return;
  const bool vec = C % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  if (vec) {
    dim3 grid(B, ceil_div(C, 256));
    hipLaunchKernelGGL(frame_stats4_kernel, grid, dim3(256), 0, s, x, ldx, T, C, out, ldo, with_std, std_off,
                       seg);
  } else {
    dim3 grid(B, ceil_div(C, 64));
    hipLaunchKernelGGL(frame_stats_kernel, grid, dim3(256), 0, s, x, ldx, T, C, out, ldo, with_std,
                       std_off, seg);
  }
  WSP_HIP(hipGetLastError());
}

// --------------------------------------------------------- residual scale ---
// out = x + h * g[utt]: HBM-bound (2 reads + 1 write per element).  A thread owns
// one 4-channel column for a run of rows (no per-element 64-bit index division:
// the utterance is decoded once per row), four rows in flight per step.
namespace {
constexpr int kRSRows = 64;  // rows per workgroup

// HX = false: out = h * g (no residual operand)
template <bool HX>
__global__ __launch_bounds__(256) void residual_scale_kernel(const f32x4* __restrict__ x,
                                                             const f32x4* __restrict__ h,
                                                             const float* __restrict__ g,
                                                             f32x4* __restrict__ out, int M, int T, int C4,
                                                             const int* __restrict__ seg, int nseg) {
  const int tpr = min(C4, 256);             // threads per row
  const int rpp = 256 / tpr;                // rows per pass
  const int sub = threadIdx.x / tpr;
  const int r0 = blockIdx.x * kRSRows;
  const int r1 = min(M, r0 + kRSRows);
  for (int c4 = threadIdx.x % tpr; c4 < C4; c4 += tpr) {
    int r = r0 + sub;
    // 8 rows per pass: 16 float4 loads in flight per thread
    for (; r + 7 * rpp < r1; r += 8 * rpp) {
      f32x4 xv[8], hv[8], gv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const long i = (long)(r + u * rpp) * C4 + c4;
        xv[u] = HX ? __builtin_nontemporal_load(x + i) : f32x4{0.f, 0.f, 0.f, 0.f};
        hv[u] = __builtin_nontemporal_load(h + i);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int row = r + u * rpp;
        const int b = seg ? seg_of(seg, nseg, row) : row / T;
        gv[u] = *reinterpret_cast<const f32x4*>(g + ((long)b * C4 + c4) * 4);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) out[(long)(r + u * rpp) * C4 + c4] = HX ? xv[u] + hv[u] * gv[u] : hv[u] * gv[u];
    }
    for (; r < r1; r += rpp) {
      const int b = seg ? seg_of(seg, nseg, r) : r / T;
      const long i = (long)r * C4 + c4;
      const f32x4 gv = *reinterpret_cast<const f32x4*>(g + ((long)b * C4 + c4) * 4);
      out[i] = HX ? x[i] + h[i] * gv : h[i] * gv;
    }
  }
}
}  // namespace

void launch_residual_scale(const float* x, const float* h, const float* g, float* out, int B,
                           int T, int C, hipStream_t s, const int* seg, int M) {
  WSP_CHECK(C % 4 == 0, "residual_scale: C % 4");
  const int C4 = C / 4;
  WSP_CHECK(C4 % 256 == 0 || 256 % C4 == 0, "residual_scale: C/4 must divide or be a multiple of 256");
  const int rows = seg ? M : B * T;
  if (rows == 0) return;
  const dim3 grid(ceil_div(rows, kRSRows));
  const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
  const f32x4* h4 = reinterpret_cast<const f32x4*>(h);
  f32x4* o4 = reinterpret_cast<f32x4*>(out);
  if (x)
    hipLaunchKernelGGL(residual_scale_kernel<true>, grid, dim3(256), 0, s, x4, h4, g, o4, rows, T, C4, seg, B);
  else
    hipLaunchKernelGGL(residual_scale_kernel<false>, grid, dim3(256), 0, s, x4, h4, g, o4, rows, T, C4, seg, B);
  WSP_HIP(hipGetLastError());
}

// -------------------------------------------------------------- ASTP pool ---
// Online (max-rescaled) softmax over frames fused with the alpha-weighted
// first and second moments: one read of logits and features, no alpha tensor.
namespace {
__global__ __launch_bounds__(256) void astp_pool_kernel(const float* __restrict__ e,
                                                        const float* __restrict__ x, int T_, int C,
                                                        float* __restrict__ out, const int* __restrict__ seg,
                                                        float floor_) {
  __shared__ float sm[4][4][64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = blockIdx.y * 64 + lane;
  const bool ok = c < C;
  float mx = -INFINITY, se = 0.f, a1 = 0.f, a2 = 0.f;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  if (ok) {
    const long base = (seg ? (long)seg[b] : (long)b * T_) * C + c;
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
    out[(long)b * 2 * C + C + c] = sqrtf(fmaxf(var, floor_));
  }
}

// Vector form (C % 4 == 0): 4 channels per lane (16-B loads of e and x), two
// frames per step with their loads issued first, branch-free online softmax
// (running max m, rescale exp(m - m') — two exps per element instead of a
// per-lane branch).
__global__ __launch_bounds__(256) void astp_pool4_kernel(const float* __restrict__ e,
                                                         const float* __restrict__ x, int T_, int C,
                                                         float* __restrict__ out, const int* __restrict__ seg,
                                                         float floor_) {
  __shared__ f32x4 sm[4][4][64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = (blockIdx.y * 64 + lane) * 4;
  const bool ok = c < C;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 mx = {-INFINITY, -INFINITY, -INFINITY, -INFINITY}, se = z, a1 = z, a2 = z;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  auto step = [&](const f32x4& ev, const f32x4& xv) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float m1 = fmaxf(mx[k], ev[k]);
      const float sc = __expf(mx[k] - m1);  // 0 on the first frame (mx = -inf)
      const float pe = __expf(ev[k] - m1);
      se[k] = fmaf(se[k], sc, pe);
      a1[k] = fmaf(a1[k], sc, pe * xv[k]);
      a2[k] = fmaf(a2[k], sc, pe * xv[k] * xv[k]);
      mx[k] = m1;
    }
  };
  if (ok) {
    const long base = (seg ? (long)seg[b] : (long)b * T_) * C + c;
    auto ld = [&](const float* p, int t) { return *reinterpret_cast<const f32x4*>(p + base + (long)t * C); };
    int t = wave;
    for (; t + 4 < T; t += 8) {
      const f32x4 e0 = ld(e, t), x0 = ld(x, t), e1 = ld(e, t + 4), x1 = ld(x, t + 4);
      step(e0, x0);
      step(e1, x1);
    }
    if (t < T) step(ld(e, t), ld(x, t));
  }
  sm[wave][0][lane] = mx;
  sm[wave][1][lane] = se;
  sm[wave][2][lane] = a1;
  sm[wave][3][lane] = a2;
  __syncthreads();
  if (wave == 0 && ok) {
    f32x4 mean, sd;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float M = sm[0][0][lane][k];
      for (int w = 1; w < 4; ++w) M = fmaxf(M, sm[w][0][lane][k]);
      float S = 0.f, A1 = 0.f, A2 = 0.f;
      for (int w = 0; w < 4; ++w) {
        const float m = sm[w][0][lane][k];
        const float f = (m == -INFINITY) ? 0.f : __expf(m - M);
        S += sm[w][1][lane][k] * f;
        A1 += sm[w][2][lane][k] * f;
        A2 += sm[w][3][lane][k] * f;
      }
      mean[k] = A1 / S;
      sd[k] = sqrtf(fmaxf(A2 / S - mean[k] * mean[k], floor_));
    }
    *reinterpret_cast<f32x4*>(out + (long)b * 2 * C + c) = mean;
    *reinterpret_cast<f32x4*>(out + (long)b * 2 * C + C + c) = sd;
  }
}
}  // namespace

void launch_astp_pool(const float* e, const float* x, int B, int T, int C, float* out,
                      hipStream_t s, const int* seg, float var_floor) {
  if (B == 0) return;
  const bool vec = C % 4 == 0 && ((reinterpret_cast<uintptr_t>(e) | reinterpret_cast<uintptr_t>(x) |
                                   reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (vec) {
    dim3 grid(B, ceil_div(C, 256));
    hipLaunchKernelGGL(astp_pool4_kernel, grid, dim3(256), 0, s, e, x, T, C, out, seg, var_floor);
  } else {
    dim3 grid(B, ceil_div(C, 64));
    hipLaunchKernelGGL(astp_pool_kernel, grid, dim3(256), 0, s, e, x, T, C, out, seg, var_floor);
  }
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp

namespace wsp {

// ------------------------------------------------------------ ResNet stem ---
// conv1 of the r-vector ResNet (resnet.py:130-136,174-176): 1 -> C0 channels,
// 3x3, pad 1, BN folded into (w, bias), ReLU.  Input = the reference's (B,T,F)
// features read as the (B,1,F,T) image; output NHWC [B][F][T][C0].
namespace {
template <int C0>
__global__ __launch_bounds__(256) void resnet_stem_kernel(const float* __restrict__ feats, int T, int F,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, long total) {
  __shared__ float s_w[C0 * 9];
  __shared__ float s_b[C0];
  for (int i = threadIdx.x; i < C0 * 9; i += 256) s_w[i] = w[i];
  for (int i = threadIdx.x; i < C0; i += 256) s_b[i] = bias[i];
  __syncthreads();
  const long idx = blockIdx.x * 256L + threadIdx.x;
  if (idx >= total) return;
  const int t = (int)(idx % T);
  const long bf = idx / T;
  const int f = (int)(bf % F);
  const int b = (int)(bf / F);
  float x[9];
#pragma unroll
  for (int kf = 0; kf < 3; ++kf)
#pragma unroll
    for (int kt = 0; kt < 3; ++kt) {
      const int ff = f + kf - 1, tt = t + kt - 1;
      x[kf * 3 + kt] = (ff >= 0 && ff < F && tt >= 0 && tt < T) ? feats[((long)b * T + tt) * F + ff] : 0.f;
    }
  f32x4* o = reinterpret_cast<f32x4*>(out + idx * C0);
#pragma unroll
  for (int c4 = 0; c4 < C0 / 4; ++c4) {
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c4 * 4 + e;
      float a = s_b[c];
#pragma unroll
      for (int q = 0; q < 9; ++q) a = fmaf(x[q], s_w[c * 9 + q], a);
      v[e] = fmaxf(a, 0.f);
    }
    o[c4] = v;
  }
}
}  // namespace

void launch_resnet_stem(const float* feats, int B, int T, int F, int C0, const float* w, const float* bias,
                        float* out, hipStream_t s) {
  WSP_CHECK(C0 == 32 || C0 == 64, "resnet stem: m_channels must be 32 or 64");
  const long total = (long)B * F * T;
  if (total == 0) return;
  const unsigned grid = (unsigned)((total + 255) / 256);
  if (C0 == 32)
    hipLaunchKernelGGL(resnet_stem_kernel<32>, dim3(grid), dim3(256), 0, s, feats, T, F, w, bias, out, total);
  else
    hipLaunchKernelGGL(resnet_stem_kernel<64>, dim3(grid), dim3(256), 0, s, feats, T, F, w, bias, out, total);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
