// Shared A-operand staging for the implicit-GEMM conv kernels.
//
// A(row, k) with k = tap*cin + c reads channels-last activations at frame
// t + tap*dil - pad of the same utterance (zero outside [0, T)).  When every
// 32-wide k-tile lies inside one tap and one concat segment (cin and the
// segment boundaries multiples of 32 — every layer except ECAPA layer1), the
// tap / segment / base pointer are wave-uniform scalars advanced
// incrementally per k-tile; otherwise (layer1: cin = 80) each lane decodes its
// own k (single segment only).
#pragma once

#include "kernels.h"

namespace wsp {

// Buffer (SRSRC) loads: 32-bit byte offsets, and an out-of-range offset
// returns zeros — the conv's zero padding without exec-mask branches.
constexpr int kOOB = 0x7FFFFFF0;

// The base must be wave-uniform; readfirstlane makes that provable so hipcc
// keeps the descriptor in SGPRs (no waterfall loop, cdna guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, kOOB, 0x00020000);
}

__device__ __forceinline__ f32x4 bload4(__amdgpu_buffer_rsrc_t r, int voff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0));
}

template <int AR, int AMODE, bool UNI>
struct ALoader {
  const float* a0;
  const float* a1;
  const float* a2;
  int ld0, ld1, ld2, cs1, cs2;
  int cin, dil, pad, T, K;
  int c4;
  int a_m[AR], a_t[AR];
  int j, c;  // UNI: tap and channel of the current k-tile start

  __device__ __forceinline__ void init(const ConvGemmArgs& p, int m0, int srow, int rows_step,
                                       int c4_) {
    a0 = p.a[0];
    a1 = p.a[1];
    a2 = p.a[2];
    ld0 = p.lda[0];
    ld1 = p.lda[1];
    ld2 = p.lda[2];
    cs1 = p.cseg[1];
    cs2 = p.cseg[2];
    cin = p.cin;
    dil = p.dil;
    pad = p.pad;
    T = p.T;
    K = p.K;
    c4 = c4_;
    j = 0;
    c = 0;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + srow + rows_step * i;
      a_m[i] = m;
      a_t[i] = (m < p.M) ? (m % p.T) : -0x40000000;  // invalid rows fail the t-range test
    }
  }

  // Loads the k-tile starting at k0; UNI requires calls with k0 = 0, 32, 64, ...
  // `live` = false issues the same loads with out-of-range offsets (zeros):
  // pipelines past the last tile keep a branch-free, exactly counted stream.
  __device__ __forceinline__ void load(int k0, f32x4 (&ra)[AR], bool live = true) {
    if constexpr (UNI) {
      const int off = j * dil - pad;
      const float* base = a0;
      int ld = ld0, cl = c;
      if (AMODE == kACat) {
        if (c >= cs2) {
          base = a2;
          ld = ld2;
          cl = c - cs2;
        } else if (c >= cs1) {
          base = a1;
          ld = ld1;
          cl = c - cs1;
        }
      }
      const __amdgpu_buffer_rsrc_t r0 = make_rsrc(base);
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a1);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int tt = a_t[i] + off;
        const bool ok = live && tt >= 0 && tt < T;
        const int row = a_m[i] + off;
        ra[i] = bload4(r0, ok ? (row * ld + cl + c4) * 4 : kOOB);
        if (AMODE == kAAdd) ra[i] += bload4(r1, ok ? (row * ld1 + c + c4) * 4 : kOOB);
      }
      c += 32;
      if (c >= cin) {
        c -= cin;
        ++j;
      }
    } else {
      const int k = k0 + c4;
      const bool kin = k < K;
      const int jj = kin ? k / cin : 0;
      const int cc = k - jj * cin;
      const int off = jj * dil - pad;
      const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a0);
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a1);
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int tt = a_t[i] + off;
        const bool ok = live && kin && tt >= 0 && tt < T;
        const int row = a_m[i] + off;
        ra[i] = bload4(r0, ok ? (row * ld0 + cc) * 4 : kOOB);
        if (AMODE == kAAdd) ra[i] += bload4(r1, ok ? (row * ld1 + cc) * 4 : kOOB);
      }
    }
  }
};

// True when every 32-wide k-tile of the operand stays in one tap and segment.
inline bool uniform_ktiles(const ConvGemmArgs& p) {
  if (p.cin % 32 != 0) return false;
  if (p.amode == kACat && (p.cseg[1] % 32 != 0 || p.cseg[2] % 32 != 0)) return false;
  return true;
}

inline void check_conv_args(const ConvGemmArgs& p, const char* who) {
  const std::string w(who);
  // buffer-load byte offsets are 32-bit: every operand must stay below 2 GiB
  for (int i = 0; i < 3; ++i)
    WSP_CHECK((long long)p.M * p.lda[i] * 4 < (long long)kOOB, w + ": operand exceeds 2 GiB (split the batch)");
  WSP_CHECK((long long)p.N * p.Kp * 4 < (long long)kOOB, w + ": weights exceed 2 GiB");
  WSP_CHECK(p.M > 0 && p.N > 0 && p.K > 0 && p.T > 0, w + ": empty shape");
  WSP_CHECK(p.cin % 4 == 0, w + ": cin must be a multiple of 4");
  WSP_CHECK(p.K == p.cin * p.taps, w + ": K != cin * taps");
  WSP_CHECK(p.Kp % 32 == 0 && p.Kp >= p.K, w + ": bad packed K");
  WSP_CHECK(p.N % 64 == 0, w + ": N must be a multiple of 64");
  for (int i = 0; i < 3; ++i) WSP_CHECK(p.lda[i] % 4 == 0, w + ": lda must be a multiple of 4");
  if (p.amode == kACat) {
    WSP_CHECK(p.cseg[0] == 0 && p.cseg[3] == p.cin && p.cseg[1] <= p.cseg[2] &&
                  p.cseg[2] <= p.cseg[3],
              w + ": bad channel segments");
    for (int i = 1; i < 3; ++i) WSP_CHECK(p.cseg[i] % 4 == 0, w + ": segment not float4 aligned");
    if (!uniform_ktiles(p))
      WSP_CHECK(p.cseg[1] == p.cin, w + ": multi-segment A needs 32-aligned segments");
  }
}

}  // namespace wsp
