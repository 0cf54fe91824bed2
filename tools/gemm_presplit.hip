// Development experiment (not part of the product): a bf16x3 GEMM whose A
// operand arrives pre-split as bf16 hi / lo planes (as a producer epilogue
// could write it), so both operands stream global -> LDS by LDS-DMA with no
// VALU split, against the shipped conv_gemm_x3 (fp32 A split while staging).
//   gemm_presplit [M N K reps]
// Both kernels see the same operands (host split = device split, RNE), so the
// outputs must agree bit for bit.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../wespeaker_hubert_amd/csrc/gemm_common.h"

using namespace wsp;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 256 x 256 block, 8 waves (4 x 2) of 64 x 128, BK-deep stages of four bf16
// images (A hi, A lo, W hi, W lo), NST-stage ring.  BK = 32: 64-B rows, chunk
// swizzle ^ ((row >> 2) & 3); BK = 16: 32-B rows, ^ ((row >> 3) & 1).
template <int BK, int NST>
__global__ __launch_bounds__(512, 2) void presplit_gemm(const ConvGemmArgs p, const __bf16* __restrict__ ahi,
                                                        const __bf16* __restrict__ alo, const __bf16* __restrict__ whi,
                                                        const __bf16* __restrict__ wlo) {
  constexpr int WM = 4, WN = 2, TM = 2, TN = 4, BM = 256, BN = 256;
  constexpr int ROWB = BK * 2;                 // bytes per image row
  constexpr int IMG = BM * ROWB;               // one image
  constexpr int STAGE = 4 * IMG;
  constexpr int RPI = 1024 / ROWB;             // rows per 1-KB DMA instruction
  constexpr int CPR = ROWB / 16;               // 16-B chunks per row
  constexpr int INS = BM / RPI / 8;            // DMA instructions per wave per image
  constexpr int OPS = 4 * INS;                 // per wave per stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto swz = [](int row) { return BK == 32 ? ((row >> 2) & 3) : ((row >> 3) & 1); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntiles = p.N / BN, mtiles = (p.M + BM - 1) / BM;
  const int wg = xcd_remap(blockIdx.x, ntiles * mtiles);
  const int mt = wg / ntiles, nt = wg - mt * ntiles;
  const int m0 = mt * BM, n0 = nt * BN;
  int a_off[INS], b_off[INS];
#pragma unroll
  for (int i = 0; i < INS; ++i) {
    const int row = (wave * INS + i) * RPI + lane / CPR;
    const int lc = (lane % CPR) ^ swz(row);
    a_off[i] = (m0 + row < p.M) ? ((m0 + row) * p.K + lc * 8) * 2 : kOOB;
    b_off[i] = ((n0 + row) * p.Kp + lc * 8) * 2;
  }
  const __amdgpu_buffer_rsrc_t rah = make_rsrc(ahi), ral = make_rsrc(alo), rwh = make_rsrc(whi), rwl = make_rsrc(wlo);
  auto issue = [&](int k0, int stage, bool live) {
    unsigned char* st = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < INS; ++i) {
      const int dst = (wave * INS + i) * 1024;
      const int ao = (live && a_off[i] != kOOB) ? a_off[i] + k0 * 2 : kOOB;
      const int bo = live ? b_off[i] + k0 * 2 : kOOB;
      dma16(rah, st + dst, ao);
      dma16(ral, st + IMG + dst, ao);
      dma16(rwh, st + 2 * IMG + dst, bo);
      dma16(rwl, st + 3 * IMG + dst, bo);
    }
  };
  const int wm = wave / WN, wn = wave - wm * WN, r32 = lane & 31, h = lane >> 5;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = p.Kp / BK;
#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0) issue(s0 * BK, s0, s0 < nk);
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<OPS * (NST - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    issue((kt + NST - 1) * BK, (kt + NST - 1) % NST, kt + NST - 1 < nk);
    const unsigned char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = (wm * TM + i) * 32 + r32;
        const int o = row * ROWB + (((2 * s + h) ^ swz(row)) << 4);
        ah[i] = *reinterpret_cast<const bf16x8*>(st + o);
        al[i] = *reinterpret_cast<const bf16x8*>(st + IMG + o);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = (wn * TN + j) * 32 + r32;
        const int o = row * ROWB + (((2 * s + h) ^ swz(row)) << 4);
        bh[j] = *reinterpret_cast<const bf16x8*>(st + 2 * IMG + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(st + 3 * IMG + o);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  gemm_epilogue_store<TM, TN, kActRelu, false>(p, acc, m0, n0, wm, wn, lane);
}

static uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t b) {
  const uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 127488, N = argc > 2 ? std::atoi(argv[2]) : 1024;
  const int K = argc > 3 ? std::atoi(argv[3]) : 1024, reps = argc > 4 ? std::atoi(argv[4]) : 20;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> ua(-1.f, 1.f), uw(-0.05f, 0.05f);
  std::vector<float> a((size_t)M * K), w((size_t)N * K), bias(N);
  for (auto& x : a) x = std::fmax(ua(rng), 0.f);  // post-ReLU activations
  for (auto& x : w) x = uw(rng);
  for (auto& x : bias) x = uw(rng);
  auto split = [](const std::vector<float>& v, std::vector<uint16_t>& hi, std::vector<uint16_t>& lo) {
    hi.resize(v.size());
    lo.resize(v.size());
    for (size_t i = 0; i < v.size(); ++i) {
      hi[i] = f2bf(v[i]);
      lo[i] = f2bf(v[i] - bf2f(hi[i]));
    }
  };
  std::vector<uint16_t> ah, al, wh, wl;
  split(a, ah, al);
  split(w, wh, wl);
  float *da, *db, *o1, *o2;
  void *dah, *dal, *dwh, *dwl;
  CK(hipMalloc(&da, a.size() * 4));
  CK(hipMalloc(&db, N * 4));
  CK(hipMalloc(&o1, (size_t)M * N * 4));
  CK(hipMalloc(&o2, (size_t)M * N * 4));
  CK(hipMalloc(&dah, ah.size() * 2));
  CK(hipMalloc(&dal, al.size() * 2));
  CK(hipMalloc(&dwh, wh.size() * 2));
  CK(hipMalloc(&dwl, wl.size() * 2));
  CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dah, ah.data(), ah.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dal, al.data(), al.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwh, wh.data(), wh.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dwl, wl.data(), wl.size() * 2, hipMemcpyHostToDevice));
  ConvGemmArgs g{};
  g.a[0] = g.a[1] = g.a[2] = da;
  g.lda[0] = g.lda[1] = g.lda[2] = K;
  g.cseg[1] = g.cseg[2] = g.cseg[3] = K;
  g.cin = K;
  g.taps = 1;
  g.dil = 1;
  g.M = M;
  g.T = 498;
  g.N = N;
  g.K = K;
  g.Kp = K;
  g.bias = db;
  g.act = kActRelu;
  g.ldo = N;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<float> r1((size_t)M * N), r2((size_t)M * N);
  auto timeit = [&](const char* name, auto&& launch, float* out, bool ref) {
    launch();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    CK(hipMemcpy((ref ? r1 : r2).data(), out, r1.size() * 4, hipMemcpyDeviceToHost));
    double diff = 0;
    if (!ref)
      for (size_t i = 0; i < r1.size(); ++i) diff = std::fmax(diff, std::fabs(r1[i] - r2[i]));
    std::printf("M=%d N=%d K=%d  %-22s %8.4f ms  %7.1f TF  maxdiff %.3g\n", M, N, K, name, ms,
                2.0 * M * N * K / (ms * 1e-3) / 1e12, diff);
    std::fflush(stdout);
  };
  const int nwg = ((M + 255) / 256) * (N / 256);
  for (int round = 0; round < 2; ++round) {
    ConvGemmArgs q = g;
    q.out = o1;
    timeit("conv_gemm_x3 v5", [&] { launch_conv_gemm_x3(q, dwh, dwl, 5, s); }, o1, true);
    ConvGemmArgs q2 = g;
    q2.out = o2;
    timeit("presplit BK32 NST2", [&] {
      hipLaunchKernelGGL((presplit_gemm<32, 2>), dim3(nwg), dim3(512), 2 * 4 * 256 * 64, s, q2,
                         (const __bf16*)dah, (const __bf16*)dal, (const __bf16*)dwh, (const __bf16*)dwl);
    }, o2, false);
    timeit("presplit BK16 NST4", [&] {
      hipLaunchKernelGGL((presplit_gemm<16, 4>), dim3(nwg), dim3(512), 4 * 4 * 256 * 32, s, q2,
                         (const __bf16*)dah, (const __bf16*)dal, (const __bf16*)dwh, (const __bf16*)dwl);
    }, o2, false);
  }
  return 0;
}
