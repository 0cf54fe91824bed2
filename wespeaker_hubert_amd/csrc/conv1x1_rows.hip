// 1x1 conv K -> N (K = 128 / 256 / 512, N = 32 ... 128) from whole activation rows in
// LDS: the ResNet bottleneck conv1 (resnet.py:95-99) on bf16x3 MFMA.
//
// conv_gemm_x3 stages 32-channel k-tiles: every k-step of a block fetches a 128-B
// piece of each of its rows, so at any moment the GPU reads 128-B pieces spread
// over rows K * 4 bytes apart; the measured stream rate falls with the row length
// (1x1 convs at 0.5 / 1 / 2 / 4 KB rows: 5.3 / 4.5 / 3.8 / 2.5 TB/s).
// Here a block owns R = 16384 / K rows, reads them whole (consecutive threads take
// consecutive 16-B pieces of a row: contiguous streams of R * K * 4 bytes), splits
// them once into bf16 hi / lo planes in LDS (64 KB, two blocks per CU, 16-B chunks
// XOR-swizzled by row: conflict-free fragment reads) and runs all K/16 k-steps from
// LDS with W in MFMA B-fragment order from L1 / L2 two k-steps ahead (the
// conv3x3_img scheme) — no barrier in the k-loop.  Each wave owns one 32-row run
// and one 32-column tile.  k order, MFMA order and epilogue are conv_gemm_x3's:
// bit-identical results.
#include "conv1x1_rows.h"
#include "gemm_common.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

template <int K, int N>
struct Rows {
  static constexpr int R = 16384 / K;      // rows per block (64 KB of bf16 hi / lo)
  static constexpr int RB = 2 * K;         // bytes per row and plane
  static constexpr int PLANE = R * RB;
  static constexpr int LDS = 2 * PLANE;
  static constexpr int CT = N / 32;        // column tiles = waves per row run
  static constexpr int NW = R / 32 * CT;
  static constexpr int NT = NW * 64;
  static constexpr int KS = K / 16;
  static constexpr int K4 = K / 4;
  static constexpr int NQ = R * K4 / NT;   // float4 staging loads per thread
  static_assert(K >= 128 && R % 32 == 0 && R * K4 % NT == 0 && KS % 2 == 0, "conv1x1_rows shape");
  // 16-B chunk ch of row r at slot ch ^ (r & 15): the 16 rows of a ds_read_b128
  // lane group hit 16 distinct slots (K / 8 >= 16 chunks per row)
  __device__ __forceinline__ static int addr(int r, int ch) { return r * RB + ((ch ^ (r & 15)) << 4); }
};

template <int K, int N>
__global__ __launch_bounds__(16384 / K / 32 * (N / 32) * 64, 2) void conv1x1_rows_kernel(const Conv1x1Args p) {
  using G = Rows<K, N>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* xhi = smem;
  unsigned char* xlo = smem + G::PLANE;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int m0 = blockIdx.x * G::R;
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x);

  // ---- rows m0 .. m0 + R: one contiguous stream, split into hi / lo planes
  {
    f32x4 v[G::NQ];
#pragma unroll
    for (int i = 0; i < G::NQ; ++i) {
      const int q = tid + i * G::NT;
      const int r = q / G::K4;
      const int c = (q - r * G::K4) * 4;
      v[i] = bload4(rx, m0 + r < p.M ? ((m0 + r) * K + c) * 4 : kOOB);
    }
#pragma unroll
    for (int i = 0; i < G::NQ; ++i) {
      const int q = tid + i * G::NT;
      const int r = q / G::K4;
      const int c = (q - r * G::K4) * 4;
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 hh = (__bf16)v[i][e];
        hi[e] = hh;
        lo[e] = (__bf16)(v[i][e] - (float)hh);
      }
      const int a = G::addr(r, c >> 3) + (c & 7) * 2;
      *reinterpret_cast<bf16x4*>(xhi + a) = hi;
      *reinterpret_cast<bf16x4*>(xlo + a) = lo;
    }
  }

  const int run = wave / G::CT, ct = wave - run * G::CT;  // 32-row run, column tile
  const int row = run * 32 + r32;

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w);
  auto wload = [&](int g, bf16x8& bh, bf16x8& bl) {
    const int o = ((g * 2 * G::CT + ct) * 64 + lane) * 16;
    const bool ok = g < G::KS;
    bh = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o : kOOB, 0, 0));
    bl = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, ok ? o + G::CT * 1024 : kOOB, 0, 0));
  };
  auto read_a = [&](int g, bf16x8& ah, bf16x8& al) {
    const int a = G::addr(row, 2 * g + h);
    ah = *reinterpret_cast<const bf16x8*>(xhi + a);
    al = *reinterpret_cast<const bf16x8*>(xlo + a);
  };
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  auto mma = [&](const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  };

  bf16x8 b0h, b0l, b1h, b1l, a0h, a0l, a1h, a1l;
  wload(0, b0h, b0l);
  wload(1, b1h, b1l);
  __syncthreads();  // rows complete
  read_a(0, a0h, a0l);
#pragma unroll 4
  for (int g = 0; g < G::KS; g += 2) {
    read_a(g + 1, a1h, a1l);
    mma(a0h, a0l, b0h, b0l);
    wload(g + 2, b0h, b0l);
    if (g + 2 < G::KS) read_a(g + 2, a0h, a0l);
    mma(a1h, a1l, b1h, b1l);
    wload(g + 3, b1h, b1l);
  }

  // ---- epilogue (conv_gemm_x3's: y = act(acc + bias) * scale + shift)
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
  const int col = ct * 32 + r32;
  const float bv = p.bias ? p.bias[col] : 0.f;
  const float sc = p.scale ? p.scale[col] : 1.f;
  const float sh = p.scale ? p.shift[col] : 0.f;
  const int rw0 = m0 + run * 32 + 4 * h;  // row of register 0
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = rw0 + (r & 3) + 8 * (r >> 2);
    float y = acc[r] + bv;
    if (p.relu) y = fmaxf(y, 0.f);
    y = y * sc + sh;
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro, m < p.M ? (m * N + col) * 4 : kOOB,
                                          0, 0);
  }
}

template <int K, int N>
void launch_k(const Conv1x1Args& p, hipStream_t s) {
  using G = Rows<K, N>;
  hipLaunchKernelGGL((conv1x1_rows_kernel<K, N>), dim3((p.M + G::R - 1) / G::R), dim3(G::NT), G::LDS, s, p);
}

}  // namespace

bool conv1x1_rows_supported(int K, int N) {
  return (K == 128 && (N == 32 || N == 64)) || (K == 256 && (N == 64 || N == 128)) || (K == 512 && N == 128);
}

void launch_conv1x1_rows(const Conv1x1Args& p, int K, int N, hipStream_t s) {
  WSP_CHECK(conv1x1_rows_supported(K, N), "conv1x1_rows: unsupported K / N");
  WSP_CHECK(p.M > 0 && p.x && p.out && p.w, "conv1x1_rows: bad arguments");
  WSP_CHECK((long long)p.M * K * 4 < (long long)kOOB && (long long)p.M * N * 4 < (long long)kOOB,
            "conv1x1_rows: operand exceeds 2 GiB (split the batch)");
  if (K == 128 && N == 32)
    launch_k<128, 32>(p, s);
  else if (K == 128)
    launch_k<128, 64>(p, s);
  else if (K == 256 && N == 64)
    launch_k<256, 64>(p, s);
  else if (K == 256)
    launch_k<256, 128>(p, s);
  else
    launch_k<512, 128>(p, s);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
