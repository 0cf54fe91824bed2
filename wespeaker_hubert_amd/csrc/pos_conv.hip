// HuBERT positional convolution as a direct grouped conv (r5): out = GELU(conv(x) + bias) with
// Conv1d(768, 768, k = 128, padding 64, groups 16) under weight_norm(dim = 2), SamePad dropping
// the last output frame (s3prl / fairseq ConvPositionalEmbedding; oracle/hubert_ref.py:45-70,
// SURVEY.md §8 row (a) "HuBERT encoder").  bf16x3 products (hi*hi + hi*lo + lo*hi, fp32
// accumulation) as conv_gemm_x3.
//
// The grouped implicit GEMM (conv_gemm_x3's gcols path) pads every group's 48 output columns to
// 64 (a quarter of its MFMAs multiply zeros), re-stages the same input rows for each of the 128
// taps, and splits fp32 A into hi / lo on every k-tile.  Here one block owns 256 output frames of
// one utterance and one group:
//   * the input patch — frames t0 - 64 .. t0 + 319 (zeros outside the utterance) x the group's 48
//     channels — is split into bf16 hi / lo ONCE and stays in LDS (2 x 36 KB, 96-B rows).  The
//     packed k index is tap * 48 + c, so output row r at k reads patch byte 96 r + 2 k: the A
//     fragment of a 16x16x32 step is one ds_read_b128 at a linear offset, and the 96-B rows
//     put every ds_read_b128 lane group on 16 distinct 16-B slots (exhaustive check over all
//     k-steps and both lane-group shapes, profiles/r5c_pos_conv.txt);
//   * W (the group's 48 output rows x 6144 k, bf16 hi / lo from the padded grouped pack, rows
//     g * 64 + n) streams through a 3-stage LDS-DMA ring of 128-k stages (24 KB each, family 6's
//     {0, 2, 3, 1} row swizzle applied to the DMA source chunk; one barrier per 72 MFMAs a wave);
//   * 8 waves x 32 rows x 48 columns: 2 x 3 accumulators, 18 MFMAs per 32-k step, no VALU in
//     the loop.
// Blocks are ordered group-major behind the XCD remap, so the blocks resident on one XCD share
// one or two groups' 1.2 MB weight slices in its L2.
#include "gemm_common.h"

namespace wsp {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int kCin = 48, kTaps = 128, kPad = 64, kK = kCin * kTaps;  // 6144
constexpr int kRows = 256;                                          // output frames per block
constexpr int kPatch = kRows + kTaps;                               // 384 input frames
constexpr int kPlane = kPatch * kCin * 2;                           // one bf16 plane, 36,864 B
constexpr int kWRows = 48;
constexpr int kWStep = kWRows * 64;                                 // [48 rows][32 k] bf16: 3 KB
constexpr int kKS = 4;                                              // 32-k steps per stage
constexpr int kStage = 2 * kKS * kWStep;                            // [plane][k-step][48][64 B]
constexpr int kNStage = 3;
constexpr int kStages = kK / (32 * kKS);                            // 48
constexpr int kPieces = 6 * kKS / 8;                                // 1-KB DMA pieces per wave and stage
constexpr int kLdsBytes = 2 * kPlane + kNStage * kStage;            // 147,456

struct PosConvArgs {
  const float* x;
  int ldx;
  const int* seg;  // [B+1] frame offsets
  int B, nwin, M;
  const __bf16* whi;
  const __bf16* wlo;
  int ldw;   // elements per W row (packed K)
  int gout;  // W rows / bias entries / output columns per group (64: the padded grouped pack)
  const float* bias;
  float* out;
  int ldo;
};

// 16-B chunk c of W row `row` sits at slot c ^ f(row) (Lds<true, 16>::off)
__device__ __forceinline__ int w_swz(int row) { return (0x1320 >> (4 * ((row >> 2) & 3))) & 3; }

__global__ __launch_bounds__(512, 1) void pos_conv_kernel(const PosConvArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int per_g = p.B * p.nwin;
  const int g = tile / per_g;
  const int rem = tile - g * per_g;
  const int u = rem / p.nwin;
  const int t0 = (rem - u * p.nwin) * kRows;
  const int r0 = p.seg[u], T = p.seg[u + 1] - r0;
  if (t0 >= T) return;  // block-uniform, before any barrier

  unsigned char* phi = smem;
  unsigned char* plo = smem + kPlane;
  unsigned char* ring = smem + 2 * kPlane;

  // ---- W DMAs: piece d (0 .. 6 kKS - 1) = plane d / (3 kKS), k-step (d / 3) % kKS, rows
  // 16 (d % 3) .. + 15; wave w issues pieces w, w + 8, ...
  static_assert(6 * kKS % 8 == 0, "whole DMA pieces per wave");
  const __amdgpu_buffer_rsrc_t rwh = make_rsrc(p.whi);
  const __amdgpu_buffer_rsrc_t rwl = make_rsrc(p.wlo);
  int woff[kPieces], wdst[kPieces];
  bool wlo_[kPieces];
#pragma unroll
  for (int i = 0; i < kPieces; ++i) {
    const int d = wave + 8 * i;
    const int plane = d / (3 * kKS), ks = (d / 3) % kKS, rg = d % 3;
    const int row = 16 * rg + (lane >> 2);
    woff[i] = ((g * p.gout + row) * p.ldw + 32 * ks + 8 * ((lane & 3) ^ w_swz(row))) * 2;
    wdst[i] = plane * kKS * kWStep + ks * kWStep + rg * 1024;
    wlo_[i] = plane == 1;
  }
  auto dma = [&](int st) {
    unsigned char* dst = ring + (st % kNStage) * kStage;
#pragma unroll
    for (int i = 0; i < kPieces; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(wlo_[i] ? rwl : rwh, (lds_void*)(dst + wdst[i]), 16,
                                               woff[i] + st * 64 * kKS, 0, 0, 0);
  };
  dma(0);
  dma(1);

  // ---- the input patch: 384 frames x 48 channels, split into hi / lo once
  {
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x);
#pragma unroll
    for (int j = 0; j < kPatch * 12 / 512; ++j) {
      const int q = tid + 512 * j;
      const int row = q / 12, c4 = q - row * 12;
      const int t = t0 - kPad + row;
      const bool ok = t >= 0 && t < T;
      const f32x4 v = bload4(rx, ok ? ((r0 + t) * p.ldx + g * kCin + 4 * c4) * 4 : kOOB);
      bf16x4 h, l;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        h[e] = (__bf16)v[e];
        l[e] = (__bf16)(v[e] - (float)h[e]);
      }
      *reinterpret_cast<bf16x4*>(phi + row * 96 + 8 * c4) = h;
      *reinterpret_cast<bf16x4*>(plo + row * 96 + 8 * c4) = l;
    }
  }

  const int r16 = lane & 15, qk = lane >> 4;
  const int aoff = (wave * 32 + r16) * 96 + 16 * qk;  // + 1536 i + 2 k0 (k0 = the step's first k)
  int boff[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int row = 16 * j + r16;
    boff[j] = row * 64 + ((qk ^ w_swz(row)) << 4);
  }
  f32x4 acc[2][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int st = 0; st < kStages; ++st) {
    // this wave's pieces of stage st have landed (stage st + 1's may still fly), and every wave is
    // done with stage st - 1, whose ring slot the DMA below refills
    // (raw s_barrier: __syncthreads' release fence would wait for stage st + 1 too)
    static_assert(kPieces == 3, "the counted wait below");
    if (st + 1 < kStages) {
      asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    if (st + 2 < kStages) dma(st + 2);
    const unsigned char* w = ring + (st % kNStage) * kStage;
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) {
      const int ka = aoff + 64 * (kKS * st + ks);
      bf16x8 ah[2], al[2], bh[3], bl[3];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = *reinterpret_cast<const bf16x8*>(phi + ka + 1536 * i);
        al[i] = *reinterpret_cast<const bf16x8*>(plo + ka + 1536 * i);
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        bh[j] = *reinterpret_cast<const bf16x8*>(w + ks * kWStep + boff[j]);
        bl[j] = *reinterpret_cast<const bf16x8*>(w + kKS * kWStep + ks * kWStep + boff[j]);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          f32x4& c = acc[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
        }
    }
  }

  // ---- epilogue: lane holds rows 16 i + 4 qk + r, column 16 j + r16 of the wave's 32 x 48
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(p.out);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = g * p.gout + 16 * j + r16;
    const float bv = p.bias[col];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + wave * 32 + 16 * i + 4 * qk + r;
        const float y = gelu_as(acc[i][j][r] + bv);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y), ro,
                                              t < T ? ((r0 + t) * p.ldo + col) * 4 : kOOB, 0, 0);
      }
  }
}

}  // namespace

void launch_hubert_pos_conv(const float* x, int ldx, const int* seg, int B, int maxT, int M, const void* whi,
                            const void* wlo, int ldw, int gout, const float* bias, float* out, int ldo,
                            hipStream_t s) {
  WSP_CHECK(B > 0 && maxT > 0 && M > 0, "pos_conv: empty batch");
  WSP_CHECK(ldw >= kK && ldw % 8 == 0 && gout >= kWRows && ldx >= 16 * kCin && ldx % 4 == 0 && ldo >= 16 * gout,
            "pos_conv: bad strides");
  WSP_CHECK((reinterpret_cast<uintptr_t>(x) & 15) == 0, "pos_conv: x must be 16-byte aligned");
  WSP_CHECK((long long)M * ldx * 4 < (long long)kOOB && (long long)M * ldo * 4 < (long long)kOOB &&
                (long long)16 * gout * ldw * 2 < (long long)kOOB,
            "pos_conv: operand exceeds 2 GiB (split the batch)");
  PosConvArgs a{x, ldx, seg, B, (maxT + kRows - 1) / kRows, M,
                static_cast<const __bf16*>(whi), static_cast<const __bf16*>(wlo), ldw, gout, bias, out, ldo};
  const long long nwg = 16LL * B * a.nwin;
  WSP_CHECK(nwg < (1LL << 31), "pos_conv: grid too large");
  hipLaunchKernelGGL(pos_conv_kernel, dim3((unsigned)nwg), dim3(512), kLdsBytes, s, a);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
