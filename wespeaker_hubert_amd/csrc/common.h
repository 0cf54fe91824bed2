// Shared helpers for the gfx950 kernels and the C-ABI runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>

namespace wsp {

void set_error(const std::string& msg);
const std::string& get_error();

struct HipError {
  hipError_t err;
  std::string where;
};

#define WSP_HIP(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) throw ::wsp::HipError{_e, std::string(#expr)};     \
  } while (0)

struct InvalidArg {
  std::string msg;
};

#define WSP_CHECK(cond, msg)                                                 \
  do {                                                                       \
    if (!(cond)) throw ::wsp::InvalidArg{std::string(msg)};                  \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 / T1): blocks
// b and b+8 share an XCD under round-robin dispatch, so give each XCD a
// contiguous range of logical tile ids.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + (bid >> 3);
}

// GELU (exact erf form, fairseq / torch default) with erf from Abramowitz & Stegun
// 7.1.26 (|error| <= 1.5e-7, ~2.5 fp32 ulp near 1): one exp, one reciprocal and five
// FMAs instead of the libm erff's branchy rational approximations — the GELU epilogue
// of a 256-column wave tile evaluates 128 of them per lane.
__device__ __forceinline__ float gelu_as(float y) {
  const float x = fabsf(y) * 0.70710678118654752f;
  const float t = __frcp_rn(fmaf(0.3275911f, x, 1.f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  const float e = 1.f - q * t * __expf(-x * x);  // erf(|y| / sqrt 2)
  return 0.5f * y * (1.f + copysignf(e, y));
}

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

// CU count of the CURRENT device, cached per device id (launch geometry of the
// persistent / strip kernels).  Concurrent first calls from several host threads
// store the same value, so a relaxed atomic per device is enough.
inline int device_cu_count() {
  static std::atomic<int> cache[64];
  int dev = 0;
  WSP_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) {
    int n = 0;
    WSP_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return n > 0 ? n : 256;
  }
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    WSP_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    if (n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

// Utterance of row m in a segmented (ragged) batch: seg[b] <= m < seg[b+1],
// seg = int32 [nseg+1] row offsets (binary search; seg is tiny and cache-hot).
__device__ __forceinline__ int seg_of(const int* __restrict__ seg, int nseg, int m) {
  int lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (seg[mid] <= m) lo = mid;
    else hi = mid;
  }
  return lo;
}

}  // namespace wsp
