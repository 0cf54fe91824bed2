// GEMM microbenchmark for the implicit-GEMM conv kernels (development tool,
// not part of the product).  Plain GEMM shapes (taps = 1) or 1-D convs:
//   gemm_bench M N K [taps [reps]] ...   (K = cin * taps)
// For every kernel variant: average launch time over `reps` launches with HIP
// events, algorithmic TFLOP/s (2*M*N*K), and max |diff| against variant 4
// (r4: families 6 and 7 in interleaved rounds).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../wespeaker_hubert_amd/csrc/kernels.h"

using namespace wsp;

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
#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

int main(int argc, char** argv) {
  std::vector<int> shapes;
  for (int i = 1; i < argc; ++i) shapes.push_back(std::atoi(argv[i]));
  if (shapes.empty()) shapes = {127488, 1024, 1024, 1, 20};
  for (size_t si = 0; si + 4 < shapes.size() + 1; si += 5) {
    const int M = shapes[si], N = shapes[si + 1], K = shapes[si + 2], taps = shapes[si + 3], reps = shapes[si + 4];
    const int cin = K / taps, Kp = (K + 63) / 64 * 64, T = 498;
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> ua(-1.f, 1.f), uw(-0.05f, 0.05f);
    std::vector<float> a((size_t)M * cin), w((size_t)N * Kp, 0.f), bias(N);
    const bool relu_a = std::getenv("GB_RELU_A") != nullptr;  // post-ReLU activations: half zeros
    for (auto& x : a) x = relu_a ? std::fmax(ua(rng), 0.f) : ua(rng);
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k) w[(size_t)n * Kp + k] = uw(rng);
    for (auto& x : bias) x = uw(rng);
    std::vector<uint16_t> hi(w.size()), lo(w.size());
    for (size_t i = 0; i < w.size(); ++i) {
      hi[i] = f2bf(w[i]);
      lo[i] = f2bf(w[i] - bf2f(hi[i]));
    }
    float *da, *dw, *db, *dout, *dref;
    void *dhi, *dlo;
    CK(hipMalloc(&da, a.size() * 4));
    CK(hipMalloc(&dw, w.size() * 4));
    CK(hipMalloc(&db, N * 4));
    CK(hipMalloc(&dout, (size_t)M * N * 4));
    CK(hipMalloc(&dref, (size_t)M * N * 4));
    CK(hipMalloc(&dhi, hi.size() * 2));
    CK(hipMalloc(&dlo, lo.size() * 2));
    CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bias.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dhi, hi.data(), hi.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dlo, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
    ConvGemmArgs g{};
    g.a[0] = g.a[1] = g.a[2] = da;
    g.lda[0] = g.lda[1] = g.lda[2] = cin;
    g.cseg[1] = g.cseg[2] = g.cseg[3] = cin;
    g.cin = cin;
    g.taps = taps;
    g.dil = 1;
    g.pad = taps / 2;
    g.M = M;
    g.T = T;
    g.N = N;
    g.w = dw;
    g.K = K;
    g.Kp = Kp;
    g.bias = db;
    g.ldo = N;
    g.act = std::getenv("GB_ACT") ? std::atoi(std::getenv("GB_ACT")) : kActRelu;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
      const char* name;
      int kind;
    } vars[] = {{"x3_256swz", 4}, {"x3_256mf16", 6}, {"x3_256dma", 7}, {"x3_256mf16", 6}, {"x3_256dma", 7},
                {"x3_256mf16", 6}, {"x3_256dma", 7}};
    std::vector<float> ref((size_t)M * N), out((size_t)M * N);
    for (auto& v : vars) {
      ConvGemmArgs q = g;
      q.out = v.kind == 4 ? dref : dout;
      auto launch = [&] {
        if (v.kind < 0) launch_conv_gemm(q, s);
        else launch_conv_gemm_x3(q, dhi, dlo, v.kind, s);
      };
      try {
        launch();
      } catch (...) {
        std::printf("  %-12s unsupported\n", v.name);
        continue;
      }
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) launch();
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      double diff = 0;
      if (v.kind == 4) {
        CK(hipMemcpy(ref.data(), dref, ref.size() * 4, hipMemcpyDeviceToHost));
      } else {
        CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < out.size(); ++i) diff = std::fmax(diff, std::fabs(out[i] - ref[i]));
      }
      std::printf("M=%d N=%d K=%d taps=%d  %-12s %8.4f ms  %7.1f TF  maxdiff %.3g\n", M, N, K, taps, v.name, ms,
                  2.0 * M * N * K / (ms * 1e-3) / 1e12, diff);
      std::fflush(stdout);
    }
    hipFree(da); hipFree(dw); hipFree(db); hipFree(dout); hipFree(dref); hipFree(dhi); hipFree(dlo);
    hipStreamDestroy(s);
  }
  return 0;
}
