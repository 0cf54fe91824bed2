// HuBERT-base front-end kernels (s3prl `hubert` upstream as wrapped by
// wespeaker/frontend/s3prl.py:23-93; fairseq HuBERT semantics, restated in
// oracle/hubert_ref.py).  The dense contractions (conv1..6, projections, FFN,
// pos_conv) run on the implicit-GEMM MFMA kernels; this file holds the rest:
//
//   conv0 + GroupNorm(512, 512) + GELU : waveform -> [B][T0][512]
//       (1 input channel, k10 s5: 10 MACs per output — VALU, recomputed per
//        pass instead of round-tripping 33 MB/utt of pre-norm activations)
//   layernorm  : rows of D in {512, 768}, optional (remapped) residual add,
//                optional s3prl Featurizer accumulation + length match
//   mha        : softmax(QK^T/8) V per (utterance, head), online softmax over
//                64-key blocks staged in LDS (T = 249 frames for 5 s)
//   cmn_rows   : per-utterance mean removal over frames (dataset_utils.py:19-26)
#include <cfloat>

#include "kernels.h"

namespace wsp {

namespace {

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// ---------------------------------------------------------------- conv0 ---
constexpr int kC0 = 512, kK0 = 10, kS0 = 5, kTC = 128;

// PASS 0: stats[0][b][c] += sum_t y;  PASS 1: stats[1][b][c] += sum_t (y - mean)^2;
// PASS 2: out = GELU(GroupNorm(y)).  One thread per channel, one block per
// (128-frame chunk, utterance); the waveform chunk is staged in LDS and read
// as a broadcast.
template <int PASS>
__global__ __launch_bounds__(kC0) void conv0_kernel(const float* __restrict__ wav, int N, int ldw, int T0,
                                                    const float* __restrict__ w, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, double* __restrict__ stats,
                                                    float* __restrict__ out, int B) {
  __shared__ float seg[kTC * kS0 + kK0];
  const int b = blockIdx.y, t0 = blockIdx.x * kTC, c = threadIdx.x;
  const float* x = wav + (size_t)b * ldw;
  for (int i = c; i < kTC * kS0 + kK0; i += kC0) {
    const int n = t0 * kS0 + i;
    seg[i] = n < N ? x[n] : 0.f;
  }
  float wr[kK0];
#pragma unroll
  for (int k = 0; k < kK0; ++k) wr[k] = w[c * kK0 + k];
  __syncthreads();
  const int nt = min(kTC, T0 - t0);
  double* s0 = stats + (size_t)b * kC0 + c;
  double* s1 = stats + (size_t)(B + b) * kC0 + c;
  float mean = 0.f, scale = 1.f, shift = 0.f;
  if (PASS >= 1) mean = (float)(*s0 / T0);
  if (PASS == 2) {
    const float rstd = (float)(1.0 / sqrt(*s1 / T0 + 1e-5));
    scale = rstd * gamma[c];
    shift = beta[c] - mean * scale;
  }
  float acc = 0.f;
  for (int t = 0; t < nt; ++t) {
    float y = 0.f;
#pragma unroll
    for (int k = 0; k < kK0; ++k) y = fmaf(wr[k], seg[t * kS0 + k], y);
    if (PASS == 0) {
      acc += y;
    } else if (PASS == 1) {
      const float d = y - mean;
      acc = fmaf(d, d, acc);
    } else {
      out[((size_t)b * T0 + t0 + t) * kC0 + c] = gelu_erf(fmaf(y, scale, shift));
    }
  }
  if (PASS == 0) atomicAdd(s0, (double)acc);
  if (PASS == 1) atomicAdd(s1, (double)acc);
}

// ------------------------------------------------------------ layernorm ---
template <int VPL>
__global__ __launch_bounds__(256) void layernorm_kernel(const LayerNormArgs p) {
  constexpr int D = VPL * 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= p.M) return;
  float v[VPL];
  const float* x = p.x + (size_t)row * p.ldx;
#pragma unroll
  for (int i = 0; i < VPL; ++i) v[i] = x[lane + 64 * i];
  if (p.add) {
    const float* a = p.add + (size_t)row * p.ldadd;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const int g = c / p.gin;
      v[i] += a[g * p.gout + (c - g * p.gin)];
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += v[i];
  const float mean = wave_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    v[i] -= mean;
    q = fmaf(v[i], v[i], q);
  }
  const float rstd = 1.f / sqrtf(wave_sum(q) * (1.f / D) + p.eps);
  float* o = p.out + (size_t)row * p.ldo;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    v[i] = v[i] * rstd * p.gamma[c] + p.beta[c];
    o[c] = v[i];
  }
  if (p.feat) {
    // s3prl Featurizer: feat += w_l * h_l; length match replicates the last
    // frame up to Tout (and trims frames >= Tout).
    const int b = row / p.T, t = row - b * p.T;
    const int t_end = (t == p.T - 1) ? p.Tout : min(t + 1, p.Tout);
    for (int tt = t; tt < t_end; ++tt) {
      float* f = p.feat + ((size_t)b * p.Tout + tt) * D;
#pragma unroll
      for (int i = 0; i < VPL; ++i) {
        const int c = lane + 64 * i;
        f[c] = p.feat_init ? p.feat_w * v[i] : fmaf(p.feat_w, v[i], f[c]);
      }
    }
  }
}

// ------------------------------------------------------------------ mha ---
// One block = (64 queries, head, utterance); thread (q = tid/4, sub = tid%4)
// scores keys 4j+sub of each 64-key block and owns output dims 16 sub..+15.
constexpr int kDH = 64, kQB = 64, kKB = 64, kLD = kDH + 4;

__global__ __launch_bounds__(256) void mha_kernel(const float* __restrict__ qkv, int ldq, float* __restrict__ out,
                                                  int ldo, int T, int D, float scale) {
  __shared__ __attribute__((aligned(16))) float Ks[kKB * kLD];
  __shared__ __attribute__((aligned(16))) float Vs[kKB * kLD];
  __shared__ __attribute__((aligned(16))) float Ps[kQB * kLD];
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * kQB;
  const int tid = threadIdx.x, qi = tid >> 2, sub = tid & 3;
  const int tq = q0 + qi;
  const float* base = qkv + (size_t)b * T * ldq;
  float q[kDH];
  {
    const float* qr = base + (size_t)min(tq, T - 1) * ldq + h * kDH;
#pragma unroll
    for (int d = 0; d < kDH; d += 4) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(qr + d);
      q[d] = v[0] * scale;
      q[d + 1] = v[1] * scale;
      q[d + 2] = v[2] * scale;
      q[d + 3] = v[3] * scale;
    }
  }
  float m = -FLT_MAX, l = 0.f, o[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) o[i] = 0.f;

  for (int k0 = 0; k0 < T; k0 += kKB) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = tid + 256 * i;
      const int r = f >> 4, c4 = (f & 15) * 4;
      const int tk = k0 + r;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (tk < T) {
        kv = *reinterpret_cast<const f32x4*>(base + (size_t)tk * ldq + D + h * kDH + c4);
        vv = *reinterpret_cast<const f32x4*>(base + (size_t)tk * ldq + 2 * D + h * kDH + c4);
      }
      *reinterpret_cast<f32x4*>(Ks + r * kLD + c4) = kv;
      *reinterpret_cast<f32x4*>(Vs + r * kLD + c4) = vv;
    }
    __syncthreads();
    float s[16];
    float bm = -FLT_MAX;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int kr = 4 * j + sub;
      const float* kp = Ks + kr * kLD;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int d = 0; d < kDH; d += 8) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(kp + d);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(kp + d + 4);
        a0 = fmaf(q[d], x0[0], a0);
        a0 = fmaf(q[d + 1], x0[1], a0);
        a0 = fmaf(q[d + 2], x0[2], a0);
        a0 = fmaf(q[d + 3], x0[3], a0);
        a1 = fmaf(q[d + 4], x1[0], a1);
        a1 = fmaf(q[d + 5], x1[1], a1);
        a1 = fmaf(q[d + 6], x1[2], a1);
        a1 = fmaf(q[d + 7], x1[3], a1);
      }
      s[j] = (k0 + kr < T) ? a0 + a1 : -FLT_MAX;
      bm = fmaxf(bm, s[j]);
    }
    bm = fmaxf(bm, __shfl_xor(bm, 1, 64));
    bm = fmaxf(bm, __shfl_xor(bm, 2, 64));
    const float mn = fmaxf(m, bm);
    const float corr = expf(m - mn);
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const float pj = (k0 + 4 * j + sub < T) ? expf(s[j] - mn) : 0.f;
      ls += pj;
      Ps[qi * kLD + 4 * j + sub] = pj;
    }
    ls += __shfl_xor(ls, 1, 64);
    ls += __shfl_xor(ls, 2, 64);
    l = l * corr + ls;
    m = mn;
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] *= corr;
    __syncthreads();
    const int kn = min(kKB, T - k0);
    for (int kk = 0; kk < kn; ++kk) {
      const float pv = Ps[qi * kLD + kk];
      const float* vp = Vs + kk * kLD + sub * 16;
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(vp + i);
        o[i] = fmaf(pv, v[0], o[i]);
        o[i + 1] = fmaf(pv, v[1], o[i + 1]);
        o[i + 2] = fmaf(pv, v[2], o[i + 2]);
        o[i + 3] = fmaf(pv, v[3], o[i + 3]);
      }
    }
  }
  if (tq < T) {
    const float inv = 1.f / l;
    float* op = out + ((size_t)b * T + tq) * ldo + h * kDH + sub * 16;
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      const f32x4 v = {o[i] * inv, o[i + 1] * inv, o[i + 2] * inv, o[i + 3] * inv};
      *reinterpret_cast<f32x4*>(op + i) = v;
    }
  }
}

// ------------------------------------------------------------- cmn_rows ---
__global__ __launch_bounds__(256) void cmn_rows_kernel(float* __restrict__ x, int T, int D) {
  const int b = blockIdx.y, c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  float* p = x + (size_t)b * T * D + c;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += p[(size_t)t * D];
  const float mean = s / (float)T;
  for (int t = 0; t < T; ++t) p[(size_t)t * D] -= mean;
}

}  // namespace

void launch_hubert_conv0(const float* wav, int B, int N, int ldw, int T0, const float* w, const float* gamma,
                         const float* beta, double* stats, float* out, hipStream_t s) {
  WSP_CHECK(B > 0 && T0 == (N - kK0) / kS0 + 1 && T0 > 0, "hubert conv0: bad frame count");
  WSP_CHECK(ldw >= N, "hubert conv0: ldw < N");
  WSP_HIP(hipMemsetAsync(stats, 0, sizeof(double) * 2 * B * kC0, s));
  const dim3 grid((T0 + kTC - 1) / kTC, B);
  hipLaunchKernelGGL(conv0_kernel<0>, grid, dim3(kC0), 0, s, wav, N, ldw, T0, w, gamma, beta, stats, out, B);
  hipLaunchKernelGGL(conv0_kernel<1>, grid, dim3(kC0), 0, s, wav, N, ldw, T0, w, gamma, beta, stats, out, B);
  hipLaunchKernelGGL(conv0_kernel<2>, grid, dim3(kC0), 0, s, wav, N, ldw, T0, w, gamma, beta, stats, out, B);
  WSP_HIP(hipGetLastError());
}

void launch_layernorm(const LayerNormArgs& p, hipStream_t s) {
  WSP_CHECK(p.M > 0 && (p.D == 512 || p.D == 768), "layernorm: D must be 512 or 768");
  WSP_CHECK(!p.add || (p.gin > 0 && p.gout >= p.gin), "layernorm: bad add remap");
  WSP_CHECK(!p.feat || (p.T > 0 && p.Tout > 0 && p.M % p.T == 0), "layernorm: bad featurizer shape");
  const dim3 grid((p.M + 3) / 4);
  if (p.D == 512)
    hipLaunchKernelGGL(layernorm_kernel<8>, grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL(layernorm_kernel<12>, grid, dim3(256), 0, s, p);
  WSP_HIP(hipGetLastError());
}

void launch_mha(const float* qkv, int ldq, float* out, int ldo, int B, int T, int H, int dh, hipStream_t s) {
  WSP_CHECK(dh == kDH, "mha: head dim must be 64");
  WSP_CHECK(B > 0 && T > 0 && H > 0 && ldq >= 3 * H * dh && ldq % 4 == 0 && ldo % 4 == 0, "mha: bad shape");
  const dim3 grid((T + kQB - 1) / kQB, H, B);
  hipLaunchKernelGGL(mha_kernel, grid, dim3(256), 0, s, qkv, ldq, out, ldo, T, H * dh, 1.f / sqrtf((float)dh));
  WSP_HIP(hipGetLastError());
}

void launch_cmn_rows(float* x, int B, int T, int D, hipStream_t s) {
  WSP_CHECK(B > 0 && T > 0 && D > 0, "cmn: bad shape");
  hipLaunchKernelGGL(cmn_rows_kernel, dim3((D + 255) / 256, B), dim3(256), 0, s, x, T, D);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
