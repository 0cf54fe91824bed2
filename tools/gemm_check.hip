// Development check + microbenchmark (not part of the product): the product's bf16x3 GEMM tile
// families 6 (conv_gemm_x3_t5.hip, register-staged) and 7 (conv_gemm_x3_t6.hip, LDS-DMA) on the
// operand shapes the models launch, plus the operand forms only tests reach (ragged row bias,
// 1x1 with Ti != T).  Family 7 must equal family 6 bit for bit (outputs and SE column sums); then
// interleaved timing rounds.  (r5's family 8, a ping-pong k-loop, and family 9, family 7 on 16 waves
// of 64 x 64 or 8 waves of 32 x 256, and a persistent family 7, were measured with this tool and
// pruned: profiles/r5a_gemm_check.txt, r5m_gemm_family9.txt, r5p_gemm_persistent.txt; a staggered
// start of every other CU's first block, r5ac_gemm_stagger_experiment.txt.)
//   gemm_check [case|all] [reps] [variants, e.g. 67]
// r6 experiment variants: 8 = family 7 with the A split replaced by a bit reinterpretation
// (timing only: no split VALU, same LDS / DMA traffic; its outputs differ), 9 = family 7 with the
// next tile's DMA pieces interleaved into the k-tile's quarters (bit-identical); 10 = family 7's
// LDS -> split -> MFMA loop alone (no DMA, no barrier in the k-loop; timing only); 11 = 10 without
// the split (LDS -> MFMA alone; timing only); 'c' (12) = family 10 (W fragments from L2 into
// registers, A alone through a 4-deep LDS ring; bit-identical to 6 / 7).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>
#define WSP_G7_XP 1
#include "../wespeaker_hubert_amd/csrc/conv_gemm_x3_t5.hip"
#include "../wespeaker_hubert_amd/csrc/conv_gemm_x3_t6.hip"
namespace wsp { namespace x3 {
void t_4x2_2x4_sw1(const ConvGemmArgs&, const __bf16*, const __bf16*, hipStream_t) { std::abort(); }
} }
using namespace wsp;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

namespace {
__device__ inline unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
// uniform [lo, hi), optionally max(., 0) (post-ReLU activations)
__global__ void fill_kernel(float* x, size_t n, unsigned seed, float lo, float hi, int relu) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float u = (hash32((unsigned)i * 2654435761U ^ seed) >> 8) * (1.f / 16777216.f);
    const float v = lo + (hi - lo) * u;
    x[i] = relu ? fmaxf(v, 0.f) : v;
  }
}
// W [N][Kp] (zero past K) -> bf16 hi / lo images
__global__ void split_kernel(const float* w, __bf16* hi, __bf16* lo, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const __bf16 h = (__bf16)w[i];
    hi[i] = h;
    lo[i] = (__bf16)(w[i] - (float)h);
  }
}
__global__ void zero_pad_kernel(float* w, int N, int K, int Kp) {
  const int n = blockIdx.x, k = K + threadIdx.x;
  if (k < Kp) w[(size_t)n * Kp + k] = 0.f;
}
__global__ void diff_kernel(const unsigned* a, const unsigned* b, size_t n, unsigned long long* cnt) {
  unsigned long long c = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += a[i] != b[i];
  if (c) atomicAdd(cnt, c);
}

float* dfill(size_t n, unsigned seed, float lo, float hi, int relu) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, p, n, seed, lo, hi, relu);
  return p;
}
unsigned long long ndiff(const void* a, const void* b, size_t words) {
  unsigned long long* d;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(diff_kernel, dim3(2048), dim3(256), 0, 0, (const unsigned*)a, (const unsigned*)b, words, d);
  unsigned long long h = 0;
  CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  return h;
}

struct Case {
  std::string name;
  ConvGemmArgs g{};
  double flops = 0;
  std::vector<void*> bufs;
  __bf16 *whi = nullptr, *wlo = nullptr;
  size_t out_words = 0, cs_words = 0;
};

// uniform batch of B utterances, T output rows each (Ti input rows), 1-D conv over cin channels
Case make(const std::string& name, int B, int T, int Ti, int stride, int cin, int taps, int dil, int pad, int N,
          int act, bool bn, bool colsum, bool res, bool row_bias, int nseg_cat, const std::vector<int>* seglens) {
  Case c;
  c.name = name;
  ConvGemmArgs& g = c.g;
  int M;
  std::vector<int> seg;
  if (seglens) {
    seg.push_back(0);
    for (int l : *seglens) seg.push_back(seg.back() + l);
    M = seg.back();
    B = (int)seglens->size();
    Ti = T = *std::max_element(seglens->begin(), seglens->end());
  } else {
    M = B * T;
  }
  const int K = cin * taps, Kp = (K + 63) / 64 * 64;
  const long in_rows = seglens ? M : (long)B * Ti;
  float* a = dfill((size_t)in_rows * cin, 11, -1.f, 1.f, 1);
  c.bufs.push_back(a);
  for (int i = 0; i < 3; ++i) { g.a[i] = a; g.lda[i] = cin; }
  g.cseg[0] = 0;
  g.cseg[1] = g.cseg[2] = g.cseg[3] = cin;
  if (nseg_cat == 3) {  // ECAPA conv_cat: cat(out2, out3, out4) as three row-major buffers
    const int cs = cin / 3;
    for (int i = 0; i < 3; ++i) {
      float* ai = dfill((size_t)in_rows * cs, 20 + i, -1.f, 1.f, 1);
      c.bufs.push_back(ai);
      g.a[i] = ai;
      g.lda[i] = cs;
    }
    g.cseg[1] = cs; g.cseg[2] = 2 * cs;
  }
  g.cin = cin; g.taps = taps; g.dil = dil; g.pad = pad;
  g.M = M; g.T = T; g.N = N; g.K = K; g.Kp = Kp; g.Ti = Ti; g.stride = stride;
  g.act = act; g.amode = kACat; g.ldo = N;
  float* w = dfill((size_t)N * Kp, 5, -0.05f, 0.05f, 0);
  hipLaunchKernelGGL(zero_pad_kernel, dim3(N), dim3(64), 0, 0, w, N, K, Kp);
  CK(hipMalloc(&c.whi, (size_t)N * Kp * 2));
  CK(hipMalloc(&c.wlo, (size_t)N * Kp * 2));
  hipLaunchKernelGGL(split_kernel, dim3(2048), dim3(256), 0, 0, w, c.whi, c.wlo, (size_t)N * Kp);
  c.bufs.push_back(w);
  float* bias = dfill(N, 6, -0.05f, 0.05f, 0);
  c.bufs.push_back(bias);
  g.bias = bias;
  if (bn) {
    g.scale = dfill(N, 7, 0.5f, 1.5f, 0);
    g.shift = dfill(N, 8, -0.1f, 0.1f, 0);
  }
  if (res) {
    g.res = dfill((size_t)M * N, 9, -1.f, 1.f, 0);
    g.ldres = N;
  }
  if (row_bias) g.row_bias = dfill((size_t)B * N, 10, -0.05f, 0.05f, 0);
  if (seglens) {
    int* ds;
    CK(hipMalloc(&ds, seg.size() * 4));
    CK(hipMemcpy(ds, seg.data(), seg.size() * 4, hipMemcpyHostToDevice));
    g.seg = ds;
    g.nseg = B;
  }
  c.out_words = (size_t)M * N;
  if (colsum) c.cs_words = (size_t)((M + 255) / 256) * 2 * N * 2;  // doubles as words
  c.flops = 2.0 * M * N * K;
  g = normalized(g);
  check_conv_args(g, name.c_str());
  return c;
}

void run(const Case& c, int v, float* out, double* cs, hipStream_t s) {
  ConvGemmArgs q = c.g;
  q.out = out;
  q.colsum = cs;
  if (v == 6) x3::t_4x2_2x4_mf16(q, c.whi, c.wlo, s);
  else if (v == 12) x3::t_gb256(q, c.whi, c.wlo, s);  // family 10 ('c')
  else if (v >= 8) x3::t_g256_xp(q, c.whi, c.wlo, s, v == 8 ? 1 : v == 9 ? 2 : v - 7);  // r6 experiments
  else {
    if (!x3::g256_supported(q)) { std::fprintf(stderr, "%s: family %d does not take these operands\n", c.name.c_str(), v); std::exit(2); }
    x3::t_g256(q, c.whi, c.wlo, s);
  }
}
}  // namespace

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "all";
  const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
  const std::string vs = argc > 3 ? argv[3] : "67";
  std::vector<int> vars;
  for (char ch : vs) vars.push_back(ch >= 'a' ? ch - 'a' + 10 : ch - '0');  // 'a' = 10, 'b' = 11
  const std::vector<int> ragged = {300, 257, 511, 123, 800, 6};
  std::vector<Case> cases;
  auto want = [&](const char* n) { return which == "all" || which == n; };
  // ECAPA c1024, B = 256 x 498 frames (C2)
  if (want("cxc_se")) cases.push_back(make("cxc_se", 256, 498, 498, 1, 1024, 1, 1, 0, 1024, kActRelu, true, true, false, false, 1, nullptr));
  if (want("cxc_bn")) cases.push_back(make("cxc_bn", 256, 498, 498, 1, 1024, 1, 1, 0, 1024, kActRelu, true, false, false, false, 1, nullptr));
  if (want("conv_cat")) cases.push_back(make("conv_cat", 256, 498, 498, 1, 3072, 1, 1, 0, 1536, kActRelu, false, false, false, false, 3, nullptr));
  if (want("layer1")) cases.push_back(make("layer1", 256, 498, 498, 1, 80, 5, 1, 2, 1024, kActRelu, true, false, false, false, 1, nullptr));
  // HuBERT-base, B = 256 x 5 s (C4): FFN at 249 frames, CNN conv1 (k3 s2) on 51-utterance chunks
  if (want("fc1")) cases.push_back(make("fc1", 256, 249, 249, 1, 768, 1, 1, 0, 3072, kActGelu, false, false, false, false, 1, nullptr));
  if (want("fc2")) cases.push_back(make("fc2", 256, 249, 249, 1, 3072, 1, 1, 0, 768, kActNone, false, false, true, false, 1, nullptr));
  if (want("qkv")) cases.push_back(make("qkv", 256, 249, 249, 1, 768, 1, 1, 0, 2304, kActNone, false, false, false, false, 1, nullptr));
  if (want("out_proj")) cases.push_back(make("out_proj", 256, 249, 249, 1, 768, 1, 1, 0, 768, kActNone, false, false, true, false, 1, nullptr));
  if (want("cnn_c1")) cases.push_back(make("cnn_c1", 51, 7999, 15999, 2, 512, 3, 1, 0, 512, kActGelu, false, false, false, false, 1, nullptr));
  // operand forms no shipped model sends to families 7 / 8
  if (want("rb_ragged")) cases.push_back(make("rb_ragged", 0, 0, 0, 1, 512, 1, 1, 0, 512, kActRelu, true, false, false, true, 1, &ragged));
  if (want("tiT_1x1")) cases.push_back(make("tiT_1x1", 9, 300, 310, 1, 256, 1, 1, 0, 256, kActRelu, false, false, false, false, 1, nullptr));
  if (want("k3_ragged")) cases.push_back(make("k3_ragged", 0, 0, 0, 1, 256, 3, 2, 2, 256, kActRelu, true, false, false, false, 1, &ragged));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad = 0;
  for (const Case& c : cases) {
    std::vector<float*> out(13, nullptr);
    std::vector<double*> cs(13, nullptr);
    std::vector<int> vv;  // family 10 takes uniform-k-tile operands only (gb256_supported)
    for (int v : vars)
      if (v != 12 || x3::gb256_supported(c.g)) vv.push_back(v);
      else std::printf("%-10s family 12 skipped: operands family 10 does not take\n", c.name.c_str());
    for (int v : vv) {
      CK(hipMalloc(&out[v], c.out_words * 4));
      CK(hipMemset(out[v], 0xff, c.out_words * 4));
      if (c.cs_words) CK(hipMalloc(&cs[v], c.cs_words * 4));
      run(c, v, out[v], cs[v], s);
    }
    CK(hipStreamSynchronize(s));
    for (int v : vv) {
      if (v == vv[0]) continue;
      const unsigned long long d = ndiff(out[vv[0]], out[v], c.out_words);
      const unsigned long long dc = c.cs_words ? ndiff(cs[vv[0]], cs[v], c.cs_words) : 0;
      std::printf("%-10s family %d vs %d: %llu of %zu outputs differ, %llu column-sum words differ\n", c.name.c_str(), v,
                  vv[0], d, c.out_words, dc);
      bad += (d != 0 || dc != 0) && v != 8 && v != 10 && v != 11;  // variants 8, 10, 11 are timing-only
    }
    for (int round = 0; round < 3; ++round)
      for (int v : vv) {
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < reps; ++r) run(c, v, out[v], cs[v], s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        std::printf("round %d %-10s family %d M=%d N=%d K=%d %8.4f ms %7.1f TF (x3 issue %7.1f)\n", round, c.name.c_str(),
                    v, c.g.M, c.g.N, c.g.K, ms, c.flops / (ms * 1e-3) / 1e12, 3 * c.flops / (ms * 1e-3) / 1e12);
        std::fflush(stdout);
      }
    for (int v : vv) {
      CK(hipFree(out[v]));
      if (cs[v]) CK(hipFree(cs[v]));
    }
  }
  std::printf(bad ? "MISMATCH in %d comparisons\n" : "all families bit-identical\n", bad);
  return bad ? 1 : 0;
}
