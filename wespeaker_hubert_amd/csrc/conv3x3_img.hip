// Stride-1 3x3 conv with C = 32 / 64 / 128 channels (the ResNet bottleneck conv2 of
// stages 1-3, resnet.py:72-107, and the basic-block convs of ResNet18/34,
// resnet.py:44-69, with the residual in the epilogue, and the SimAM-ResNet
// basic-block convs, samresnet.py:20-60) on bf16x3 MFMA from an LDS image of the
// input patch.
//
// The implicit GEMM (conv_gemm_x3 with ALoader2D) stages, for every 32-wide
// k-tile, the tile's rows of ONE tap from global memory: each input position is
// fetched nine times (once per tap, mostly L2 hits) and split into bf16 hi / lo
// nine times, and with N = C = 32 / 64 the MFMA work per staged byte is small
// (135-205 TFLOP/s).  Here a block owns an FB x TB tile of output
// positions of one utterance and stages the (FB + 2) x (TB + 2) input patch once,
// already split into bf16 hi / lo planes (rows = patch positions, 16-B chunks
// XOR-swizzled by row so the fragment reads are conflict-free); every tap is a
// row offset into that image.  W arrives in MFMA B-fragment order straight from
// L1 / L2, two k-steps ahead in registers (the res2_chain.hip scheme), so the
// k-loop has no barrier.  k order, MFMA order and epilogue are conv_gemm_x3's:
// the results are bit-identical to the implicit GEMM.
// C = 128 (102 KB image of a 4 x 32 tile, one block per CU): each wave owns one
// 32-position time run and all 128 channels (4 column tiles), or with WN = 2 half
// of them (8 waves; option conv3x3_img 3).  r2: ResNet293 stage-3 3x3 21.2 ->
// 18.4 ms/step (one stream), C3 1 260 -> 1 280 emb/s, ResNet34 10 740 -> 11 030.
#include "conv3x3_img.h"
#include "gemm_common.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int C, int FB, int TB, int WN = 1>
struct Img {
  static constexpr int PT = TB + 2;
  static constexpr int IR = (FB + 2) * PT;  // patch positions
  static constexpr int RB = 2 * C;          // bytes per image row and plane
  static constexpr int PLANE = IR * RB;
  static constexpr int LDS = 2 * PLANE;
  static constexpr int NW = FB * TB / 32 * WN;  // waves: 32 positions (one time run) x C / WN channels each
  static constexpr int NT = NW * 64;
  static constexpr int CT = C / 32;         // 32-channel column tiles
  static constexpr int TN = CT / WN;        // column tiles per wave
  static constexpr int KC = C / 16;         // k-steps per tap
  static constexpr int KS = 9 * KC;         // k-steps
  static constexpr int C4 = C / 4;
  static constexpr int NQ = (IR * C4 + NT - 1) / NT;  // float4 staging loads per thread
  static_assert(TB % 32 == 0 && KS % 2 == 0, "conv3x3_img tile");
  // 16-B chunk ch of row r at slot ch ^ sw(r): the 16 rows of a ds_read_b128 lane
  // group (16 distinct rows mod 16) hit 16 distinct slots of the 256-B bank row
  __device__ __forceinline__ static int sw(int r) {
    return C == 32 ? ((r >> 2) & 3) : C == 64 ? ((r >> 1) & 7) : (r & 15);
  }
  __device__ __forceinline__ static int addr(int r, int ch) { return r * RB + ((ch ^ sw(r)) << 4); }
};

template <int C, int FB, int TB, int WN, int MINB, bool RES, bool RELU>
__global__ __launch_bounds__(FB* TB * 2 * WN, MINB) void conv3x3_img_kernel(const Conv3x3Args p) {
  using G = Img<C, FB, TB, WN>;
  constexpr int TN = G::TN, PT = G::PT;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int ntf = (p.F + FB - 1) / FB, ntt = (p.T + TB - 1) / TB;
  const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles (shared halo rows) on one XCD
  const int b = id / (ntf * ntt);
  const int rem = id - b * (ntf * ntt);
  const int tf = rem / ntt;
  const int f0 = tf * FB, t0 = (rem - tf * ntt) * TB;
  const size_t ubase = (size_t)b * p.F * p.T * C;  // utterance b's first element
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x + ubase);

  // ---- input patch (f0 - 1 .. f0 + FB, t0 - 1 .. t0 + TB) -> image, zeros outside
  {
    f32x4 v[G::NQ];
#pragma unroll
    for (int i = 0; i < G::NQ; ++i) {
      const int q = tid + i * G::NT;
      const int ir = q / G::C4;
      const int c = (q - ir * G::C4) * 4;
      const int pf = ir / PT;
      const int f = f0 - 1 + pf, t = t0 - 1 + (ir - pf * PT);
      const bool ok = q < G::IR * G::C4 && f >= 0 && f < p.F && t >= 0 && t < p.T;
      v[i] = bload4(rx, ok ? ((f * p.T + t) * C + c) * 4 : kOOB);
    }
#pragma unroll
    for (int i = 0; i < G::NQ; ++i) {
      const int q = tid + i * G::NT;
      if (q < G::IR * G::C4) {
        const int ir = q / G::C4;
        const int c = (q - ir * G::C4) * 4;
        bf16x4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const __bf16 hh = (__bf16)v[i][e];
          hi[e] = hh;
          lo[e] = (__bf16)(v[i][e] - (float)hh);
        }
        const int a = G::addr(ir, c >> 3) + (c & 7) * 2;
        *reinterpret_cast<bf16x4*>(xhi + a) = hi;
        *reinterpret_cast<bf16x4*>(xlo + a) = lo;
      }
    }
  }

  // this lane's output position: patch-local (lf, lt); tap (kf, kt) reads image row
  // (lf + kf) * PT + lt + kt
  const int pr = wave / WN, wn = wave - pr * WN;  // position run, column group
  const int lf = pr / (TB / 32);
  const int lt0 = (pr % (TB / 32)) * 32;
  const int row0 = lf * PT + lt0 + r32;

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  auto wload = [&](int g, bf16x8 (&bh)[TN], bf16x8 (&bl)[TN]) {
    const bool ok = g < G::KS;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int o = ((g * 2 * G::CT + wn * TN + j) * 64 + lane) * 16;
      bh[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o : kOOB, 0, 0));
      bl[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o + G::CT * 1024 : kOOB, 0, 0));
    }
  };
  auto read_a = [&](int g, bf16x8& ah, bf16x8& al) {
    const int tap = g / G::KC, cb = g - tap * G::KC;
    const int kf = tap / 3, kt = tap - kf * 3;
    const int a = G::addr(row0 + kf * PT + kt, 2 * cb + h);
    ah = *reinterpret_cast<const bf16x8*>(xhi + a);
    al = *reinterpret_cast<const bf16x8*>(xlo + a);
  };
  f32x16 acc[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  auto mma = [&](const bf16x8& ah, const bf16x8& al, const bf16x8 (&bh)[TN], const bf16x8 (&bl)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[j], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[j], acc[j], 0, 0, 0);
    }
  };

  bf16x8 b0h[TN], b0l[TN], b1h[TN], b1l[TN], a0h, a0l, a1h, a1l;
  wload(0, b0h, b0l);
  wload(1, b1h, b1l);
  __syncthreads();  // image complete
  read_a(0, a0h, a0l);
#pragma unroll 1
  for (int g = 0; g < G::KS; g += 2) {
    read_a(g + 1, a1h, a1l);
    mma(a0h, a0l, b0h, b0l);
    wload(g + 2, b0h, b0l);
    if (g + 2 < G::KS) read_a(g + 2, a0h, a0l);
    mma(a1h, a1l, b1h, b1l);
    wload(g + 3, b1h, b1l);
  }

  // ---- epilogue (conv_gemm_x3's: y = act(acc + bias (+ res)) * scale + shift)
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out + ubase);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc((RES ? p.res : p.out) + ubase);
  const int f = f0 + lf;
  const int tw = t0 + lt0 + 4 * h;  // time of register 0
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = (wn * TN + j) * 32 + r32;
    const float bv = p.bias ? p.bias[col] : 0.f;
    const float sc = p.scale ? p.scale[col] : 1.f;
    const float sh = p.scale ? p.shift[col] : 0.f;
    float rv[16];
    if constexpr (RES) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = tw + (r & 3) + 8 * (r >> 2);
        rv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                              rr, f < p.F && t < p.T ? ((f * p.T + t) * C + col) * 4 : kOOB, 0, 0));
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = tw + (r & 3) + 8 * (r >> 2);
      float y = acc[j][r] + bv;
      if constexpr (RES) y += rv[r];
      if constexpr (RELU) y = fmaxf(y, 0.f);
      y = y * sc + sh;
      const bool ok = f < p.F && t < p.T;
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro,
                                            ok ? ((f * p.T + t) * C + col) * 4 : kOOB, 0, 0);
    }
  }
}

template <int C, int FB, int TB, int MINB, int WN = 1>
void launch_k(const Conv3x3Args& p, hipStream_t s) {
  using G = Img<C, FB, TB, WN>;
  const int nblk = p.B * ((p.F + FB - 1) / FB) * ((p.T + TB - 1) / TB);
  if (p.res)
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, true, true>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
  else if (p.relu)
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, false, true>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
  else
    hipLaunchKernelGGL((conv3x3_img_kernel<C, FB, TB, WN, MINB, false, false>), dim3(nblk), dim3(G::NT), G::LDS, s, p);
}

}  // namespace

bool conv3x3_img_supported(int C) { return C == 32 || C == 64 || C == 128; }

void launch_conv3x3_img(const Conv3x3Args& p, int C, hipStream_t s) {
  WSP_CHECK(conv3x3_img_supported(C), "conv3x3_img: channels must be 32, 64 or 128");
  WSP_CHECK(p.B > 0 && p.F > 0 && p.T > 0 && p.x && p.out && p.w, "conv3x3_img: bad arguments");
  WSP_CHECK(p.relu || !p.res, "conv3x3_img: a residual comes with the ReLU");
  // buffer offsets are per utterance (descriptors based at its first element)
  WSP_CHECK((long long)p.F * p.T * C * 4 < (long long)kOOB, "conv3x3_img: utterance exceeds 2 GiB");
  if (C == 32)
    launch_k<32, 4, 64, 3>(p, s);  // 256 positions, 8 waves, 50 KB image: 3 blocks / CU
  else if (C == 64)
    launch_k<64, 4, 32, 3>(p, s);  // 128 positions, 4 waves x 2 column tiles, 51 KB image
  else if (p.variant == 3)
    launch_k<128, 4, 32, 1, 2>(p, s);  // 128 positions, 8 waves x 2 column tiles, 102 KB image
  else
    launch_k<128, 4, 32, 1>(p, s);  // 128 positions, 4 waves x 4 column tiles, 102 KB image
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
