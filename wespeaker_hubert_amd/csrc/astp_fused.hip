// ASTP pooling head fused: linear2 (K = 128) on bf16x3 MFMA + online softmax
// over frames + attentive mean / std (pooling_layers.py:133-144).
//
// Unfused, the head writes the [rows][C] logit matrix (0.78 GB at B = 256 x
// 498 frames, C = 1536) and the pooling kernel reads it back together with x:
// ~2.3 GB of HBM traffic.  Here a block owns one utterance and 256 channels
// (8 waves x 32); each chunk's logits come out of three MFMAs per k-step
// (a = hi + lo split of the tanh(linear1) rows) and the accumulators feed the
// running softmax statistics (max, sum e, sum e x, sum e x^2) directly — x is
// read once, the logits never leave registers.  (r2 history: a 128-channel /
// 4-wave block with W2 in LDS, and a 256-channel block with W2 in LDS and a
// two-chunk ring, were 0.465 / 0.35 ms per C2 step against this kernel's 0.31.)
#include "astp_fused.h"
#include "gemm_common.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kK = 128;  // attention bottleneck width (pooling_layers.py:107-117)

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

constexpr int kCB2 = 256;                 // channels per block
constexpr int kChunkBytes = 32 * kK * 4;  // one 32-frame att chunk: 16 KB

// A block owns one utterance and 256 channels (8 waves x 32).  The 32-frame
// chunk of att rows (16 KB) is fetched ONCE per block by LDS-DMA (each wave
// issues two 1-KB pieces) instead of every wave loading the same A fragments from
// L2 right before it multiplies them; att rows are 512 B in LDS with 16-B chunk c
// stored at slot c ^ (row & 15), so the ds_read_b128 fragment reads (row =
// lane & 31) are conflict-free.  Each wave's W2 fragments (its 32 channels:
// 8 k-steps x hi / lo) are held in VGPRs, so
// LDS holds only a 3-slot att ring (48 KB) and chunks are issued TWO ahead: one
// barrier per chunk — [wait for chunk c] barrier [issue chunk c + 2 into the slot
// chunk c - 1 used] [multiply chunk c] — and x in three register sets.
constexpr int kLds3 = 3 * kChunkBytes;

__global__ __launch_bounds__(512, 1) void astp_fused3_kernel(const AstpArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char ring[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int nct = p.C / kCB2;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int b = id / nct;
  const int ct = id - b * nct;
  const int r0 = p.seg ? p.seg[b] : b * p.T;
  const int T = p.seg ? p.seg[b + 1] - r0 : p.T;
  const int col = ct * kCB2 + wave * 32 + r32;
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.att + (size_t)r0 * kK);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x + (size_t)r0 * p.ldx);

  auto dma_chunk = [&](int t0, int slot) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = 2 * wave + j;
      const int row = 2 * piece + h;
      const int c = r32 ^ (row & 15);
      const int t = t0 + row;
      dma16(ra, ring + slot * kChunkBytes + piece * 1024, t < T ? (t * kK + c * 4) * 4 : kOOB);
    }
  };
  auto load_x = [&](int t0, float (&xv)[16]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      xv[r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            rx, t < T ? (t * p.ldx + col) * 4 : kOOB, 0, 0));
    }
  };
  // this wave's W2 fragments: (k-step, plane) piece i of column tile ct * 8 + wave
  bf16x8 wf[16];
  {
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w2);
    const int ntile = p.C / 32;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      wf[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                             rw, ((i * ntile + ct * (kCB2 / 32) + wave) * 64 + lane) * 16, 0, 0));
  }
  const float bias = p.bias2[col];

  float m = -INFINITY, s = 0.f, a1 = 0.f, a2 = 0.f;
  auto consume = [&](int t0, int slot, const float (&xv)[16]) {
    const unsigned char* ab = ring + slot * kChunkBytes + r32 * 512;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int c0 = 4 * ks + 2 * h;
      const f32x4 v0 = *reinterpret_cast<const f32x4*>(ab + ((c0 ^ (r32 & 15)) << 4));
      const f32x4 v1 = *reinterpret_cast<const f32x4*>(ab + (((c0 + 1) ^ (r32 & 15)) << 4));
      bf16x8 ah, al;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = e < 4 ? v0[e] : v1[e - 4];
        const __bf16 hh = (__bf16)v;
        ah[e] = hh;
        al[e] = (__bf16)(v - (float)hh);
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, wf[2 * ks], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wf[2 * ks + 1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wf[2 * ks], acc, 0, 0, 0);
    }
    float ev[16], mc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      ev[r] = t < T ? acc[r] + bias : -INFINITY;
      mc = fmaxf(mc, ev[r]);
    }
    if (mc != -INFINITY) {
      const float m1 = fmaxf(m, mc);
      const float sc = __expf(m - m1);
      s *= sc;
      a1 *= sc;
      a2 *= sc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pe = __expf(ev[r] - m1);
        s += pe;
        a1 = fmaf(pe, xv[r], a1);
        a2 = fmaf(pe * xv[r], xv[r], a2);
      }
      m = m1;
    }
  };

  float xa[16], xb[16], xc[16];
  const int nch = (T + 31) / 32;
  dma_chunk(0, 0);
  load_x(0, xa);
  if (nch > 1) {
    dma_chunk(32, 1);
    load_x(32, xb);
  }
  // chunk c: its operations were issued two chunks earlier; at most chunk c+1's
  // 18 (2 DMA + 16 x) may still be in flight when it is consumed
  auto step = [&](int c, int slot, const float (&xcur)[16], float (&xnext2)[16]) {
    if (c + 1 < nch)
      asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 2 < nch) {
      dma_chunk((c + 2) * 32, slot == 0 ? 2 : slot - 1);
      load_x((c + 2) * 32, xnext2);
    }
    consume(c * 32, slot, xcur);
  };
  for (int c = 0; c < nch; c += 3) {
    step(c, 0, xa, xc);
    if (c + 1 >= nch) break;
    step(c + 1, 1, xb, xa);
    if (c + 2 >= nch) break;
    step(c + 2, 2, xc, xb);
  }
  const float mo = __shfl_xor(m, 32), so = __shfl_xor(s, 32), a1o = __shfl_xor(a1, 32), a2o = __shfl_xor(a2, 32);
  const float M = fmaxf(m, mo);
  const float f0 = m == -INFINITY ? 0.f : __expf(m - M);
  const float f1 = mo == -INFINITY ? 0.f : __expf(mo - M);
  const float S = s * f0 + so * f1;
  const float A1 = a1 * f0 + a1o * f1;
  const float A2 = a2 * f0 + a2o * f1;
  if (h == 0) {
    const float mean = A1 / S;
    p.out[(size_t)b * 2 * p.C + col] = mean;
    p.out[(size_t)b * 2 * p.C + p.C + col] = sqrtf(fmaxf(A2 / S - mean * mean, p.var_floor));
  }
}

}  // namespace

bool astp_fused_supported(int C, int K) { return K == kK && C > 0 && C % kCB2 == 0; }

void launch_astp_fused(const AstpArgs& p, hipStream_t s) {
  WSP_CHECK(astp_fused_supported(p.C, kK) && p.B > 0 && (p.seg || p.T > 0), "astp_fused: bad shape");
  // buffer offsets are per utterance (the descriptors are based at its first row)
  WSP_CHECK(p.seg || (long long)p.T * p.ldx * 4 < (long long)kOOB, "astp_fused: utterance exceeds 2 GiB");
  hipLaunchKernelGGL(astp_fused3_kernel, dim3(p.B * (p.C / kCB2)), dim3(512), kLds3, s, p);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
