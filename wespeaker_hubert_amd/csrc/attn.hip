// HuBERT self-attention, softmax(Q K^T / 8) V per (utterance, head), on bf16x3
// MFMA with K and V resident in LDS (fairseq MultiheadAttention as used by the
// s3prl hubert upstream; restated in oracle/hubert_ref.py).
//
// A block owns 256 queries (8 waves x 32) of one (utterance, head) and walks
// the keys in blocks of 256: each key block is staged ONCE into LDS already
// split into bf16 hi / lo planes — K as [key][64 d] (128-B rows, 16-B chunks
// XOR-swizzled by (key >> 1) & 7: conflict-free A-fragment reads) and V^T as
// [64 d][keys] (520-B rows: conflict-free 8-B reads) — so the per-chunk loop
// has no global loads, no VALU split of K / V and no barrier.  Per 32-key chunk
// each wave computes S^T = K_c Q^T (queries on the lanes), an online softmax per
// lane column, then O^T += V_c^T P with P taken from the S^T accumulators
// (k order 16 s + 8 (j >> 2) + 4 h + (j & 3), cdna_hip_programming.md §3).
// For 5 s utterances (249 frames) one block per (utterance, head) stages the
// whole K / V once; the previous kernel (hubert.hip mha_kernel) streamed 32-key
// chunks through a register / LDS ring with a barrier and an exposed global
// load per chunk.
#include "attn.h"
#include "gemm_common.h"

#include <algorithm>
#include <cfloat>

namespace wsp {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kDh = 64;                 // head dim
constexpr int kKB = 256;                // keys per staged block
constexpr int kQB = 256;                // queries per workgroup (8 waves x 32)
constexpr int kVRow = 520;              // V^T row stride in bytes (260 bf16: 2-dword bank shift per row)
constexpr int kKPlane = kKB * kDh * 2;  // 32 KB per K plane
constexpr int kVPlane = kDh * kVRow;    // 33 KB per V^T plane
constexpr int kLds = 2 * kKPlane + 2 * kVPlane;

__device__ __forceinline__ int k_addr(int key, int chunk) {  // byte offset of a 16-B chunk of K row `key`
  return key * 128 + ((chunk ^ ((key >> 1) & 7)) << 4);
}

__device__ __forceinline__ void split8(const f32x4 a, const f32x4 b, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h0 = (__bf16)a[e], h1 = (__bf16)b[e];
    hi[e] = h0;
    hi[e + 4] = h1;
    lo[e] = (__bf16)(a[e] - (float)h0);
    lo[e + 4] = (__bf16)(b[e] - (float)h1);
  }
}

__device__ __forceinline__ f32x16 mma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

__global__ __launch_bounds__(512, 2) void attn_kernel(const float* __restrict__ qkv, int ldq, float* __restrict__ out,
                                                      int ldo, int T_, int D, float scale, const int* __restrict__ seg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* kh_s = smem;
  unsigned char* kl_s = smem + kKPlane;
  unsigned char* vh_s = smem + 2 * kKPlane;
  unsigned char* vl_s = vh_s + kVPlane;

  const int b = blockIdx.z, head = blockIdx.y;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const size_t rbase = seg ? (size_t)seg[b] : (size_t)b * T_;
  const int T = seg ? seg[b + 1] - seg[b] : T_;
  const int q0 = blockIdx.x * kQB;
  if (q0 >= T) return;  // block-uniform (segmented: grid sized by the longest utterance)
  const float* base = qkv + rbase * ldq;
  const int q = q0 + wave * 32 + r;
  const bool wave_live = q0 + wave * 32 < T;  // wave-uniform

  // Q^T fragments (B operand of S^T = K Q^T): lane = query r, d = 16 s + 8 hh + e;
  // pre-scaled by 1/sqrt(dh) = 1/8 (exact in binary)
  bf16x8 qh[4], ql[4];
  {
    const float* qr = base + (size_t)min(q, T - 1) * ldq + head * kDh + 8 * hh;
    const float sc = q < T ? scale : 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
      split8(*reinterpret_cast<const f32x4*>(qr + 16 * s) * sc, *reinterpret_cast<const f32x4*>(qr + 16 * s + 4) * sc,
             qh[s], ql[s]);
  }

  f32x16 o[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[t][e] = 0.f;
  float m = -FLT_MAX, l = 0.f;

  for (int k0 = 0; k0 < T; k0 += kKB) {
    const int nk = min(kKB, T - k0);
    if (k0 > 0) __syncthreads();  // the previous key block is no longer read
    // ---- stage keys [k0, k0 + 256): K and V rows as hi / lo bf16 (zeros past T); all
    // 16 loads of a thread are issued before the first conversion
    constexpr int kPer = kKB * (kDh / 4) / 512;  // float4 pieces of K (and of V) per thread
    f32x4 kv[kPer], vv[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int f = tid + 512 * i, key = f >> 4, d4 = (f & 15) * 4;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const float* row = base + (size_t)(k0 + min(key, nk - 1)) * ldq + head * kDh + d4;
      kv[i] = key < nk ? *reinterpret_cast<const f32x4*>(row + D) : z;
      vv[i] = key < nk ? *reinterpret_cast<const f32x4*>(row + 2 * D) : z;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int f = tid + 512 * i, key = f >> 4, d4 = (f & 15) * 4;
      bf16x4 h4, l4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)kv[i][e];
        h4[e] = h0;
        l4[e] = (__bf16)(kv[i][e] - (float)h0);
      }
      const int ka = k_addr(key, d4 >> 3) + (d4 & 7) * 2;
      *reinterpret_cast<bf16x4*>(kh_s + ka) = h4;
      *reinterpret_cast<bf16x4*>(kl_s + ka) = l4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)vv[i][e];
        const int va = (d4 + e) * kVRow + key * 2;
        *reinterpret_cast<__bf16*>(vh_s + va) = h0;
        *reinterpret_cast<__bf16*>(vl_s + va) = (__bf16)(vv[i][e] - (float)h0);
      }
    }
    __syncthreads();
    if (!wave_live) continue;  // wave-uniform; the barriers above are outside this branch

    const int nch = (nk + 31) / 32;
    for (int c = 0; c < nch; ++c) {
      // S^T (32 keys x 32 queries)
      f32x16 st;
#pragma unroll
      for (int e = 0; e < 16; ++e) st[e] = 0.f;
      const int key = c * 32 + r;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ka = k_addr(key, 2 * s + hh);
        st = mma3(*reinterpret_cast<const bf16x8*>(kh_s + ka), *reinterpret_cast<const bf16x8*>(kl_s + ka), qh[s],
                  ql[s], st);
      }
      // online softmax over the keys of this lane's query column
      float cmax = -FLT_MAX;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kk = c * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        if (kk >= nk) st[e] = -FLT_MAX;
        cmax = fmaxf(cmax, st[e]);
      }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      const float mn = fmaxf(m, cmax);
      const float corr = __expf(m - mn);
      float ls = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kk = c * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
        const float pe = kk < nk ? __expf(st[e] - mn) : 0.f;
        st[e] = pe;
        ls += pe;
      }
      l = l * corr + ls;
      m = mn;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[t][e] *= corr;
      // O^T (64 d x 32 queries) += V_c^T P; V^T row d = 32 t + r, keys c*32 + 16 s + 4 hh + {0..3, 8..11}
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 ph, pl;
        const f32x4 p0 = {st[8 * s], st[8 * s + 1], st[8 * s + 2], st[8 * s + 3]};
        const f32x4 p1 = {st[8 * s + 4], st[8 * s + 5], st[8 * s + 6], st[8 * s + 7]};
        split8(p0, p1, ph, pl);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int va = (32 * t + r) * kVRow + (c * 32 + 16 * s + 4 * hh) * 2;
          const bf16x4 a0 = *reinterpret_cast<const bf16x4*>(vh_s + va);
          const bf16x4 a1 = *reinterpret_cast<const bf16x4*>(vh_s + va + 16);
          const bf16x4 b0 = *reinterpret_cast<const bf16x4*>(vl_s + va);
          const bf16x4 b1 = *reinterpret_cast<const bf16x4*>(vl_s + va + 16);
          const bf16x8 vh = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
          const bf16x8 vl = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
          o[t] = mma3(vh, vl, ph, pl, o[t]);
        }
      }
    }
  }
  if (!wave_live) return;
  const float inv = 1.f / (l + __shfl_xor(l, 32, 64));
  if (q < T) {
    float* op = out + (rbase + q) * ldo + head * kDh + 4 * hh;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = {o[t][4 * g] * inv, o[t][4 * g + 1] * inv, o[t][4 * g + 2] * inv, o[t][4 * g + 3] * inv};
        *reinterpret_cast<f32x4*>(op + 32 * t + 8 * g) = v;
      }
  }
}

// ---------------------------------------------------------------------------
// Pipelined form (default, r3): a persistent block walks its (utterance, head,
// 256-query block) items and each item's keys in halves of 128; while it multiplies
// one half out of LDS, the next half's K / V rows (the next item's first half at an
// item's end) are already in flight to registers, then written into the other of two
// LDS buffers — so the staging that the one-block-per-CU kernel above exposes per
// (utterance, head) overlaps the MFMAs.  Same chunk order; r5: the softmax in the log2 domain
// with a lazily raised maximum (equal up to fp32 rounding; h_attn -8 %, VALU-bound chunk loop).
constexpr int kKH = 128;                            // keys per staged half
constexpr int kVRowH = 264;                         // V^T row stride: 128 keys + 8 B (2-dword bank shift per row)
constexpr int kKPlaneH = kKH * kDh * 2;             // 16 KB per K plane
constexpr int kVPlaneH = kDh * kVRowH;              // 16.5 KB per V^T plane
constexpr int kBufH = 2 * kKPlaneH + 2 * kVPlaneH;  // one staged half
constexpr int kLdsPipe = 2 * kBufH;                 // two buffers: 130 KB
constexpr int kPerH = kKH * (kDh / 4) / 512;        // float4 pieces of K (and of V) per thread and half

__device__ __forceinline__ int k_addr_h(int key, int chunk) { return key * 128 + ((chunk ^ ((key >> 1) & 7)) << 4); }

__global__ __launch_bounds__(512, 2) void attn_pipe_kernel(const float* __restrict__ qkv, int ldq,
                                                           float* __restrict__ out, int ldo, int T_, int D, int H,
                                                           int nqb, int nitems, float scale,
                                                           const int* __restrict__ seg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;

  // item = (utterance b, head, query block qb); halves of 128 keys
  auto item_T = [&](int it) {
    const int b = it / (H * nqb);
    return seg ? seg[b + 1] - seg[b] : T_;
  };
  auto item_halves = [&](int it) {  // 0: no queries of this utterance in the query block
    const int T = item_T(it);
    const int qb = it % nqb;
    return qb * 256 < T ? (T + kKH - 1) / kKH : 0;
  };
  auto next = [&](int& it, int& hf) {  // advance (it, hf); it >= nitems when done
    if (++hf < item_halves(it)) return;
    hf = 0;
    for (it += gridDim.x; it < nitems && item_halves(it) == 0; it += gridDim.x) {
    }
  };
  auto base_of = [&](int it) {
    const int b = it / (H * nqb);
    return qkv + (seg ? (size_t)seg[b] : (size_t)b * T_) * ldq;
  };

  f32x4 kv[kPerH], vv[kPerH];
  auto load_half = [&](int it, int hf) {
    const int T = item_T(it);
    const int head = (it / nqb) % H;
    const int k0 = hf * kKH, nk = min(kKH, T - k0);
    const float* base = base_of(it);
#pragma unroll
    for (int i = 0; i < kPerH; ++i) {
      const int f = tid + 512 * i, key = f >> 4, d4 = (f & 15) * 4;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const float* row = base + (size_t)(k0 + min(key, nk - 1)) * ldq + head * kDh + d4;
      kv[i] = key < nk ? *reinterpret_cast<const f32x4*>(row + D) : z;
      vv[i] = key < nk ? *reinterpret_cast<const f32x4*>(row + 2 * D) : z;
    }
  };
  auto write_half = [&](unsigned char* buf) {
    unsigned char* kh_s = buf;
    unsigned char* kl_s = buf + kKPlaneH;
    unsigned char* vh_s = buf + 2 * kKPlaneH;
    unsigned char* vl_s = vh_s + kVPlaneH;
#pragma unroll
    for (int i = 0; i < kPerH; ++i) {
      const int f = tid + 512 * i, key = f >> 4, d4 = (f & 15) * 4;
      bf16x4 h4, l4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)kv[i][e];
        h4[e] = h0;
        l4[e] = (__bf16)(kv[i][e] - (float)h0);
      }
      const int ka = k_addr_h(key, d4 >> 3) + (d4 & 7) * 2;
      *reinterpret_cast<bf16x4*>(kh_s + ka) = h4;
      *reinterpret_cast<bf16x4*>(kl_s + ka) = l4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)vv[i][e];
        const int va = (d4 + e) * kVRowH + key * 2;
        *reinterpret_cast<__bf16*>(vh_s + va) = h0;
        *reinterpret_cast<__bf16*>(vl_s + va) = (__bf16)(vv[i][e] - (float)h0);
      }
    }
  };

  int it = blockIdx.x, hf = 0;
  while (it < nitems && item_halves(it) == 0) it += gridDim.x;
  if (it >= nitems) return;  // block-uniform
  load_half(it, hf);

  bf16x8 qh[4], ql[4];
  f32x16 o[2];
  float m = -FLT_MAX, l = 0.f;
  int buf = 0;
  while (true) {
    unsigned char* cur = smem + buf * kBufH;
    write_half(cur);
    __syncthreads();  // the half is in LDS; the other buffer's readers are one barrier behind
    const int T = item_T(it);
    const int head = (it / nqb) % H;
    const int q0 = (it % nqb) * 256;
    const int q = q0 + wave * 32 + r;
    const bool wave_live = q0 + wave * 32 < T;  // wave-uniform
    const float* base = base_of(it);
    if (hf == 0 && wave_live) {
      // Q^T fragments (B operand of S^T = K Q^T), pre-scaled by log2(e) / sqrt(dh): the scores
      // come out in the log2 domain, so the softmax takes one v_exp_f32 per score (r5); issued
      // before the next half's loads, so waiting for them does not wait for those
      const float* qr = base + (size_t)min(q, T - 1) * ldq + head * kDh + 8 * hh;
      const float sc = q < T ? scale * 1.4426950408889634f : 0.f;
#pragma unroll
      for (int s = 0; s < 4; ++s)
        split8(*reinterpret_cast<const f32x4*>(qr + 16 * s) * sc, *reinterpret_cast<const f32x4*>(qr + 16 * s + 4) * sc,
               qh[s], ql[s]);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[t][e] = 0.f;
      m = -FLT_MAX;
      l = 0.f;
    }
    int nit = it, nhf = hf;
    next(nit, nhf);
    if (nit < nitems) load_half(nit, nhf);  // lands while this half is multiplied

    const int k0 = hf * kKH, nk = min(kKH, T - k0);
    if (wave_live) {
      const unsigned char* kh_s = cur;
      const unsigned char* kl_s = cur + kKPlaneH;
      const unsigned char* vh_s = cur + 2 * kKPlaneH;
      const unsigned char* vl_s = vh_s + kVPlaneH;
      const int nch = (nk + 31) / 32;
      for (int c = 0; c < nch; ++c) {
        f32x16 st;
#pragma unroll
        for (int e = 0; e < 16; ++e) st[e] = 0.f;
        const int key = c * 32 + r;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int ka = k_addr_h(key, 2 * s + hh);
          st = mma3(*reinterpret_cast<const bf16x8*>(kh_s + ka), *reinterpret_cast<const bf16x8*>(kl_s + ka), qh[s],
                    ql[s], st);
        }
        // online softmax in the log2 domain with a lazy maximum (r5): the running max m moves
        // only when a score exceeds it by more than 8 (p <= 2^8 then; l <= 2^8 x keys), so the
        // 32-register rescale of O runs on the few chunks that raise the max, not on every
        // chunk; masks only in the utterance's last, partial chunk
        const bool part = c * 32 + 32 > nk;  // wave-uniform
        float cmax = -FLT_MAX;
        if (part) {
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const int kk = c * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh;
            if (kk >= nk) st[e] = -FLT_MAX;
          }
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) cmax = fmaxf(cmax, st[e]);
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
        if (__any(cmax > m + 8.f)) {  // wave-uniform
          const float mn = cmax > m + 8.f ? cmax : m;
          const float corr = __builtin_amdgcn_exp2f(m - mn);
          l *= corr;
          m = mn;
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[t][e] *= corr;
        }
        float ls = 0.f;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const float pe = __builtin_amdgcn_exp2f(st[e] - m);  // masked scores: exp2(-huge) = 0
          st[e] = pe;
          ls += pe;
        }
        l += ls;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 ph, pl;
          const f32x4 p0 = {st[8 * s], st[8 * s + 1], st[8 * s + 2], st[8 * s + 3]};
          const f32x4 p1 = {st[8 * s + 4], st[8 * s + 5], st[8 * s + 6], st[8 * s + 7]};
          split8(p0, p1, ph, pl);
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int va = (32 * t + r) * kVRowH + (c * 32 + 16 * s + 4 * hh) * 2;
            const bf16x4 a0 = *reinterpret_cast<const bf16x4*>(vh_s + va);
            const bf16x4 a1 = *reinterpret_cast<const bf16x4*>(vh_s + va + 16);
            const bf16x4 b0 = *reinterpret_cast<const bf16x4*>(vl_s + va);
            const bf16x4 b1 = *reinterpret_cast<const bf16x4*>(vl_s + va + 16);
            const bf16x8 vh = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            const bf16x8 vl = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
            o[t] = mma3(vh, vl, ph, pl, o[t]);
          }
        }
      }
      if (hf + 1 == (T + kKH - 1) / kKH) {  // the item's last half: normalise and store
        const float inv = 1.f / (l + __shfl_xor(l, 32, 64));
        if (q < T) {
          const size_t rbase = seg ? (size_t)seg[it / (H * nqb)] : (size_t)(it / (H * nqb)) * T_;
          float* op = out + (rbase + q) * ldo + head * kDh + 4 * hh;
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const f32x4 v = {o[t][4 * g] * inv, o[t][4 * g + 1] * inv, o[t][4 * g + 2] * inv,
                               o[t][4 * g + 3] * inv};
              *reinterpret_cast<f32x4*>(op + 32 * t + 8 * g) = v;
            }
        }
      }
    }
    if (nit >= nitems) break;  // block-uniform
    it = nit;
    hf = nhf;
    buf ^= 1;
  }
}

}  // namespace

void launch_attn(const float* qkv, int ldq, float* out, int ldo, int B, int T, int H, int dh, hipStream_t s,
                 const int* seg, int pipe) {
  WSP_CHECK(dh == kDh, "attn: head dim must be 64");
  WSP_CHECK(B > 0 && T > 0 && H > 0 && ldq >= 3 * H * dh && ldq % 4 == 0 && ldo % 4 == 0, "attn: bad shape");
  if (pipe) {
    const int ncu = device_cu_count();
    const int nqb = (T + kQB - 1) / kQB;  // segmented: T = longest utterance
    const int nitems = B * H * nqb;
    hipLaunchKernelGGL(attn_pipe_kernel, dim3(std::min(nitems, ncu)), dim3(512), kLdsPipe, s, qkv, ldq, out, ldo, T,
                       H * dh, H, nqb, nitems, 1.f / sqrtf((float)dh), seg);
  } else {
    const dim3 grid((T + kQB - 1) / kQB, H, B);  // segmented: T = longest utterance
    hipLaunchKernelGGL(attn_kernel, grid, dim3(512), kLds, s, qkv, ldq, out, ldo, T, H * dh, 1.f / sqrtf((float)dh),
                       seg);
  }
  WSP_HIP(hipGetLastError());
}

}  // namespace wsp
