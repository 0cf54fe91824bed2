// Development experiment (not part of the product): the product's conv_gemm_x3 family 7
// kernel (conv_gemm_x3_t6.hip, included) against family 6 (conv_gemm_x3_t5.hip, included)
// and the tools/gemm_g3.hip prototype, on the same operands, interleaved rounds.
//   g7_check [M N K reps act]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <random>
#include <vector>
#include "../wespeaker_hubert_amd/csrc/conv_gemm_x3_t5.hip"
#include "../wespeaker_hubert_amd/csrc/conv_gemm_x3_t6.hip"
namespace wsp { namespace x3 {
void t_4x2_2x4_sw1(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t) { std::abort(); }
} }
using namespace wsp;
namespace {
// Variant G: every operand by LDS-DMA (buffer_load ... lds, 16 B per lane), A staged as the
// fp32 it is (no register staging set, no ds_write pass) and split into bf16 hi / lo when
// its fragments are read.  LDS per stage: A [256][32] fp32 (128-B rows, 16-B chunk c of row
// r at slot c ^ ((r >> 1) & 5): conflict-free 2 x ds_read_b128 per 16x16x32 fragment) +
// W hi / lo [256][32] bf16 (64-B rows, the {0,2,3,1} swizzle).  Two stages: tile k + 1 lands
// while tile k multiplies; one vmcnt(0) + barrier per k-tile.
constexpr int BM = 256, BN = 256, BK_ = 32, GA = BM * 128, GW = BN * 64, GSTAGE = GA + 2 * GW;  // 64 KB
__device__ __forceinline__ int aslot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 5)) << 4); }

template <int PRE>
__global__ __launch_bounds__(512, 1) void gemm_g(const float* __restrict__ A, const __bf16* __restrict__ whi,
                                                const __bf16* __restrict__ wlo, float* __restrict__ out, int M,
                                                int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = N / BN;
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr8 = nwg & 7;
  const int wg = ((xcd < rr8) ? xcd * (qq + 1) : rr8 * (qq + 1) + (xcd - rr8) * qq) + (bid >> 3);
  const int mt = wg / ntn, nt = wg - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A), rwh = make_rsrc(whi), rwl = make_rsrc(wlo);
  // DMA geometry.  A: wave-instruction i (0..3) of wave w fills rows (4 w + i) * 8 .. + 7, lane l
  // row + (l >> 3), slot l & 7 <- global chunk (l & 7) ^ swz(row).  W: instruction i (0..1) of
  // wave w fills rows (2 w + i) * 16 .. + 15 of hi and of lo, lane l row + (l >> 2), slot l & 3.
  int aoff[4], woff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (4 * wave + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 5);
    const int m = m0 + row;
    aoff[i] = m < M ? (m * K + 4 * c) * 4 : kOOB;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * wave + i) * 16 + (lane >> 2);
    const int q = (row >> 2) & 3;
    const int c = ((lane & 3) ^ ((0x1320 >> (4 * q)) & 3));
    woff[i] = ((n0 + row) * K + 8 * c) * 2;
  }
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * GSTAGE;
    const bool live = kt * BK_ < K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(st + (4 * wave + i) * 1024),
                                               16, live && aoff[i] != kOOB ? aoff[i] + kt * BK_ * 4 : kOOB, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = live ? woff[i] + kt * BK_ * 2 : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwh, (lds_void*)(st + GA + (2 * wave + i) * 1024), 16, o, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwl, (lds_void*)(st + GA + GW + (2 * wave + i) * 1024), 16, o, 0, 0,
                                               0);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, qk = lane >> 4;
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[2], al[2], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 64 + (ih * 2 + i) * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[i][e] = h0;
        ah[i][4 + e] = h1;
        al[i][e] = (__bf16)(x0[e] - (float)h0);
        al[i][4 + e] = (__bf16)(x1[e] - (float)h1);
      }
    }
  };
  auto rdB = [&](const unsigned char* st, int jh) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = Lds<true, 16>::off(wn * 128 + (jh * 4 + j) * 16 + r16, qk * 16);
      bh[j] = *reinterpret_cast<const bf16x8*>(st + GA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + GA + GW + o);
    }
  };
  auto mm = [&](int ih, int jh) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[ih * 2 + i][jh * 4 + j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
      }
  };
  const int nk = K / BK_;
  if constexpr (PRE == 1) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 (8 DMAs per tile per lane)
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const unsigned char* st = smem + buf * GSTAGE;
    rdA(st, 0);
    rdB(st, 0);
    mm(0, 0);
    rdB(st, 1);
    mm(0, 1);
    rdA(st, 1);
    mm(1, 1);
    rdB(st, 0);
    mm(1, 0);
    // tile kt + 1 (issued one k-tile ago) has landed; every wave is done with this buffer
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma(kt + 2, buf);  // past-the-end tiles: out-of-range DMAs (zeros nobody reads)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + qk * 4 + r;
        const int col = n0 + wn * 128 + j * 16 + r16;
        if (row < M) out[(size_t)row * N + col] = acc[i][j][r];
      }
}



}  // namespace
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); std::exit(1); } } while (0)
static uint16_t f2bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); u += 0x7FFFu + ((u >> 16) & 1u); return (uint16_t)(u >> 16); }
static float bf2f(uint16_t b) { const uint32_t u = (uint32_t)b << 16; float f; std::memcpy(&f, &u, 4); return f; }
int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 127488, N = argc > 2 ? std::atoi(argv[2]) : 1024;
  const int K = argc > 3 ? std::atoi(argv[3]) : 1024, reps = argc > 4 ? std::atoi(argv[4]) : 10;
  const int act = argc > 5 ? std::atoi(argv[5]) : kActNone;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> ua(-1.f, 1.f), uw(-0.05f, 0.05f);
  std::vector<float> a((size_t)M * K), w((size_t)N * K), bias(N);
  for (auto& x : a) x = std::fmax(ua(rng), 0.f);
  for (auto& x : w) x = uw(rng);
  for (auto& x : bias) x = uw(rng);
  std::vector<uint16_t> hi(w.size()), lo(w.size());
  for (size_t i = 0; i < w.size(); ++i) { hi[i] = f2bf(w[i]); lo[i] = f2bf(w[i] - bf2f(hi[i])); }
  float *da, *db, *o[3];
  void *dh, *dl;
  CK(hipMalloc(&da, a.size() * 4)); CK(hipMalloc(&db, N * 4));
  for (int i = 0; i < 3; ++i) CK(hipMalloc(&o[i], (size_t)M * N * 4));
  CK(hipMalloc(&dh, hi.size() * 2)); CK(hipMalloc(&dl, lo.size() * 2));
  CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dh, hi.data(), hi.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
  ConvGemmArgs g{};
  g.a[0] = g.a[1] = g.a[2] = da; g.lda[0] = g.lda[1] = g.lda[2] = K;
  g.cseg[1] = g.cseg[2] = g.cseg[3] = K; g.cin = K; g.taps = 1; g.dil = 1; g.pad = 0;
  g.M = M; g.T = M; g.N = N; g.K = K; g.Kp = K; g.ldo = N; g.act = act; g.bias = act == kActNone ? nullptr : db;
  // mode 1: + BN scale / shift; 2: + residual; 3: + per-utterance row bias; 4: + SE column sums
  const int mode = argc > 6 ? std::atoi(argv[6]) : 0;
  float *dsc = nullptr, *dsh = nullptr;
  float* dres = nullptr;
  if (mode >= 1) {
    std::vector<float> sc(N, 0.9f), sh(N, 0.01f);
    CK(hipMalloc(&dsc, N * 4)); CK(hipMalloc(&dsh, N * 4));
    CK(hipMemcpy(dsc, sc.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsh, sh.data(), N * 4, hipMemcpyHostToDevice));
    g.scale = dsc; g.shift = dsh;
  }
  if (mode == 2) {  // residual epilogue (HuBERT out_proj / fc2)
    std::vector<float> res((size_t)M * N);
    for (auto& x : res) x = ua(rng);
    CK(hipMalloc(&dres, res.size() * 4));
    CK(hipMemcpy(dres, res.data(), res.size() * 4, hipMemcpyHostToDevice));
    g.res = dres; g.ldres = N;
  }
  double* dcs[3] = {nullptr, nullptr, nullptr};
  const size_t ncs = (size_t)((M + 255) / 256) * 2 * N;
  if (mode == 4) {  // SE column sums (the SE-Res2Block conv3 epilogue: ReLU, BN, f64 column sums)
    for (int v = 0; v < 3; ++v) CK(hipMalloc(&dcs[v], ncs * 8));
    g.T = 498;
  }
  if (mode == 3) {  // row bias per utterance of 498 rows (ECAPA conv_cat / ASTP linear1 form)
    g.T = 498;
    std::vector<float> rb((size_t)((M + 497) / 498) * N);
    for (auto& x : rb) x = uw(rng);
    CK(hipMalloc(&dres, rb.size() * 4));
    CK(hipMemcpy(dres, rb.data(), rb.size() * 4, hipMemcpyHostToDevice));
    g.row_bias = dres;
  }
  g = normalized(g);
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[3] = {"family6", "family7", "proto_G"};
  auto run = [&](int v) {
    ConvGemmArgs q = g; q.out = o[v]; q.colsum = dcs[v];
    if (v == 0) x3::t_4x2_2x4_mf16(q, (const __bf16*)dh, (const __bf16*)dl, s);
    else if (v == 1) x3::t_g256(q, (const __bf16*)dh, (const __bf16*)dl, s);
    else hipLaunchKernelGGL(gemm_g<0>, dim3(((M + 255) / 256) * (N / 256)), dim3(512), 2 * GSTAGE, s, da, (const __bf16*)dh, (const __bf16*)dl, o[2], M, N, K);
  };
  for (int round = 0; round < 4; ++round)
    for (int v = 0; v < 3; ++v) {
      run(v); CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) run(v);
      CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
      float ms = 0; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      std::printf("round %d %-8s M=%d N=%d K=%d act=%d %8.4f ms %7.1f TF\n", round, names[v], M, N, K, act, ms, 2.0 * M * N * K / (ms * 1e-3) / 1e12);
      std::fflush(stdout);
    }
  std::vector<float> r0((size_t)M * N), r1((size_t)M * N), r2((size_t)M * N);
  CK(hipMemcpy(r0.data(), o[0], r0.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1.data(), o[1], r1.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), o[2], r2.size() * 4, hipMemcpyDeviceToHost));
  double d01 = 0, d02 = 0;
  for (size_t i = 0; i < r0.size(); ++i) { d01 = std::fmax(d01, std::fabs(r0[i] - r1[i])); d02 = std::fmax(d02, std::fabs(r0[i] - r2[i])); }
  std::printf("max |f6 - f7| = %.3g  max |f6 - proto| = %.3g (proto has no epilogue: equal only at act 0)\n", d01, d02);
  if (dcs[0]) {
    std::vector<double> c0(ncs), c1(ncs);
    CK(hipMemcpy(c0.data(), dcs[0], ncs * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(c1.data(), dcs[1], ncs * 8, hipMemcpyDeviceToHost));
    size_t ndiff = 0;
    for (size_t i = 0; i < ncs; ++i) ndiff += c0[i] != c1[i];
    std::printf("column sums: %zu of %zu differ (f6 vs f7)\n", ndiff, ncs);
  }
  return 0;
}
