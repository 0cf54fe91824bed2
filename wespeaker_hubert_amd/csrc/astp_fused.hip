// ASTP pooling head fused: linear2 (K = 128) on bf16x3 MFMA + online softmax
// over frames + attentive mean / std (pooling_layers.py:133-144).
//
// Unfused, the head writes the [rows][C] logit matrix (0.78 GB at B = 256 x
// 498 frames, C = 1536) and the pooling kernel reads it back together with x:
// ~2.3 GB of HBM traffic.  Here a block owns one utterance and 128 channels
// (4 waves x 32): the block's W2 B-fragments (8 k-steps x hi / lo, 64 KB) sit in
// LDS for the whole utterance, x loads run a 32-frame chunk ahead, each
// chunk's logits come out of
// three MFMAs per k-step (a = hi + lo split of the tanh(linear1) rows), and the
// accumulators feed the running softmax statistics (max, sum e, sum e x,
// sum e x^2) directly — x is read once, the logits never leave registers.
// Variants 2 / 3 (below; 3 is the default) widen the block to 256 channels and
// share each att chunk through an LDS-DMA ring.
#include "astp_fused.h"
#include "gemm_common.h"

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kK = 128;  // attention bottleneck width (pooling_layers.py:107-117)

__global__ __launch_bounds__(256, 2) void astp_fused_kernel(const AstpArgs p) {
  // W2 B-fragments of the block's 128 channels: [k-step][plane][4 column tiles][64 lanes] x 16 B
  __shared__ __attribute__((aligned(16))) unsigned char wsm[8 * 2 * 4 * 1024];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int r32 = lane & 31;
  const int h = lane >> 5;
  const int nct = p.C / 128;
  const int id = xcd_remap(blockIdx.x, gridDim.x);  // an utterance's channel tiles share an XCD L2 (att rows)
  const int b = id / nct;
  const int ct = id - b * nct;
  const int r0 = p.seg ? p.seg[b] : b * p.T;
  const int T = p.seg ? p.seg[b + 1] - r0 : p.T;
  const int col = ct * 128 + wave * 32 + r32;
  {
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w2);
    const int ntile = p.C / 32;
#pragma unroll
    for (int i = 0; i < 16; ++i) {  // 16 x 4 KB pieces: (k-step, plane) x this block's 4 column tiles
      const int o = ((i * ntile + ct * 4) * 64) * 16 + tid * 16;
      *reinterpret_cast<f32x4*>(wsm + i * 4096 + tid * 16) =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, o, 0, 0));
    }
  }
  const float bias = p.bias2[col];
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.att + (size_t)r0 * kK);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(p.x + (size_t)r0 * p.ldx);

  // chunk loads: A fragments (frame t0 + (lane & 31), k = 16 ks + 8 h .. + 7; att rows
  // are L2-resident, shared by the utterance's channel tiles) and x in the
  // accumulator layout (frame t0 + (r & 3) + 8 (r >> 2) + 4 h, channel col; streamed
  // once from HBM, so issued a chunk ahead)
  auto load_a = [&](int t0, f32x4 (&av)[16]) {
    const int arow = t0 + r32;
    const bool ain = arow < T;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int o = (arow * kK + 16 * ks + 8 * h) * 4;
      av[2 * ks] = bload4(ra, ain ? o : kOOB);
      av[2 * ks + 1] = bload4(ra, ain ? o + 16 : kOOB);
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

  float m = -INFINITY, s = 0.f, a1 = 0.f, a2 = 0.f;
  auto consume = [&](int t0, const f32x4 (&av)[16], const float (&xv)[16]) {
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      bf16x8 ah, al;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = e < 4 ? av[2 * ks][e] : av[2 * ks + 1][e - 4];
        const __bf16 hh = (__bf16)v;
        ah[e] = hh;
        al[e] = (__bf16)(v - (float)hh);
      }
      const bf16x8 wh = *reinterpret_cast<const bf16x8*>(wsm + (ks * 2) * 4096 + wave * 1024 + lane * 16);
      const bf16x8 wl = *reinterpret_cast<const bf16x8*>(wsm + (ks * 2 + 1) * 4096 + wave * 1024 + lane * 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, wh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wh, acc, 0, 0, 0);
    }
    // online softmax over this lane's 16 frames of the chunk
    float ev[16], mc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int t = t0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      ev[r] = t < T ? acc[r] + bias : -INFINITY;
      mc = fmaxf(mc, ev[r]);
    }
    if (mc != -INFINITY) {
      const float m1 = fmaxf(m, mc);
      const float sc = __expf(m - m1);  // 0 while m = -inf
      s *= sc;
      a1 *= sc;
      a2 *= sc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float pe = __expf(ev[r] - m1);  // 0 for frames past the utterance
        s += pe;
        a1 = fmaf(pe, xv[r], a1);
        a2 = fmaf(pe * xv[r], xv[r], a2);
      }
      m = m1;
    }
  };

  // x one chunk ahead of the MFMAs
  f32x4 av[16];
  float xv0[16], xv1[16];
  load_x(0, xv0);
  __syncthreads();  // W2 fragments in LDS
  for (int t0 = 0; t0 < T; t0 += 64) {
    load_x(t0 + 32, xv1);
    load_a(t0, av);
    consume(t0, av, xv0);
    if (t0 + 32 >= T) break;
    load_x(t0 + 64, xv0);
    load_a(t0 + 32, av);
    consume(t0 + 32, av, xv1);
  }
  // lanes l and l ^ 32 hold the same channel: merge their statistics
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

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// Variant 2: a block owns one utterance and 256 channels (8 waves x 32).  The
// 32-frame chunk of att rows (16 KB) is fetched ONCE per block by LDS-DMA into
// a two-chunk ring (each wave issues two 1-KB pieces), one chunk ahead of the
// MFMAs, instead of every wave loading the same A fragments from L2 right before
// it multiplies them.  att rows are 512 B in LDS with 16-B chunk c stored at slot
// c ^ (row & 15): the ds_read_b128 fragment reads (row = lane & 31) are
// conflict-free.  W2 fragments (256 channels: 128 KB) + the ring fill the 160 KB.
constexpr int kCB2 = 256;
constexpr int kW2Bytes = 8 * 2 * (kCB2 / 32) * 1024;  // 128 KB
constexpr int kChunkBytes = 32 * kK * 4;                // 16 KB
constexpr int kLds2 = kW2Bytes + 2 * kChunkBytes;       // 160 KB

__global__ __launch_bounds__(512, 1) void astp_fused2_kernel(const AstpArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* wsm = smem;
  unsigned char* ring = smem + kW2Bytes;
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

  // att chunk t0 -> ring slot: wave w issues rows 4w .. 4w + 3 (two 1-KB pieces)
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
  // W2 fragments of the block's 256 channels: 16 (k-step, plane) pieces of 8 KB
  {
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.w2);
    const int ntile = p.C / 32;
#pragma unroll 4
    for (int i = 0; i < 16; ++i) {
      const int o = ((i * ntile + ct * (kCB2 / 32)) * 64) * 16 + tid * 16;
      *reinterpret_cast<f32x4*>(wsm + i * 8192 + tid * 16) =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rw, o, 0, 0));
    }
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
      const bf16x8 wh = *reinterpret_cast<const bf16x8*>(wsm + (ks * 2) * 8192 + wave * 1024 + lane * 16);
      const bf16x8 wl = *reinterpret_cast<const bf16x8*>(wsm + (ks * 2 + 1) * 8192 + wave * 1024 + lane * 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, wh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, wh, acc, 0, 0, 0);
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

  // chunk c: [barrier: slot (c+1)&1 free] issue chunk c+1 (att DMA + x loads);
  // wait until chunk c's DMA and x loads have landed (only chunk c+1's 2 + 16
  // operations may still be in flight); [barrier: chunk c's att visible]; multiply
  float xv0[16], xv1[16];
  dma_chunk(0, 0);
  load_x(0, xv0);
  for (int t0 = 0; t0 < T; t0 += 64) {
    __syncthreads();
    const bool n1 = t0 + 32 < T;
    if (n1) {
      dma_chunk(t0 + 32, 1);
      load_x(t0 + 32, xv1);
      asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    consume(t0, 0, xv0);
    if (!n1) break;
    __syncthreads();
    const bool n2 = t0 + 64 < T;
    if (n2) {
      dma_chunk(t0 + 64, 0);
      load_x(t0 + 64, xv0);
      asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    consume(t0 + 32, 1, xv1);
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

// Variant 3: variant 2's block (one utterance x 256 channels, 8 waves) with each
// wave's W2 fragments (its 32 channels: 8 k-steps x hi / lo) held in VGPRs, so
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

bool astp_fused_supported(int C, int K, int variant) {
  return K == kK && C > 0 && C % (variant >= 2 ? kCB2 : 128) == 0;
}

void launch_astp_fused(const AstpArgs& p, hipStream_t s) {
  WSP_CHECK(astp_fused_supported(p.C, kK, p.variant) && p.B > 0 && (p.seg || p.T > 0), "astp_fused: bad shape");
  // buffer offsets are per utterance (the descriptors are based at its first row)
  WSP_CHECK(p.seg || (long long)p.T * p.ldx * 4 < (long long)kOOB, "astp_fused: utterance exceeds 2 GiB");
  if (p.variant == 3) {
    hipLaunchKernelGGL(astp_fused3_kernel, dim3(p.B * (p.C / kCB2)), dim3(512), kLds3, s, p);
    WSP_HIP(hipGetLastError());
    return;
  }
  if (p.variant == 2) {
    hipLaunchKernelGGL(astp_fused2_kernel, dim3(p.B * (p.C / kCB2)), dim3(512), kLds2, s, p);
    WSP_HIP(hipGetLastError());
    return;
  }
  const int nblk = p.B * (p.C / 128);
  hipLaunchKernelGGL(astp_fused_kernel, dim3(nblk), dim3(256), 0, s, p);
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
