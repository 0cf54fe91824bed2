// Development experiment (not part of the product; r4: variant G, every operand by LDS-DMA): the bf16x3 256 x 256 GEMM
// k-loop of conv_gemm_x3 (variant 5: 8 waves of 64 x 128, BK = 32, one register
// staging set, fp32 A split while staging) on v_mfma_f32_32x32x16_bf16 against
// the same loop on v_mfma_f32_16x16x32_bf16 (MI355X_MICROARCH.md "DVFS give-back"
// item 7: the 16x16 shape holds a higher clock under MFMA load).  Dense A [M][K]
// fp32, W [N][K] as bf16 hi / lo images, plain fp32 stores in each kernel's own
// accumulator layout; both outputs are checked against each other.
//   mf16_bench [M N K reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kOOB = 0x7FFFFFF0;
constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int ROWB = 64, IMG = BM * ROWB, STAGE = 4 * IMG;  // A hi, A lo, W hi, W lo

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  const unsigned long long a = reinterpret_cast<unsigned long long>(base);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, kOOB, 0x00020000);
}

// 16-B chunk swizzle of a 64-B k-tile row: MF = 32 reads rows lane & 31 at chunk
// 2s + h; MF = 16 reads rows lane & 15 at chunk lane >> 4 (the {0,2,3,1} map keeps
// every ds_read_b128 lane group on 16 distinct 16-B slots of the bank row)
template <int MF>
__device__ __forceinline__ int loff(int row, int byte) {
  const int q = (row >> 2) & 3;
  const int f = MF == 32 ? q : ((0x1320 >> (4 * q)) & 3);  // MF 16 / 17 share the layout
  return row * ROWB + ((((byte >> 4) ^ f) & 3) << 4) + (byte & 15);
}

template <int MF>
__global__ __launch_bounds__(NT, 1) void gemm_kernel(const float* __restrict__ A, const __bf16* __restrict__ whi,
                                                     const __bf16* __restrict__ wlo, float* __restrict__ out, int M,
                                                     int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = N / BN;
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr8 = nwg & 7;
  const int wg = ((xcd < rr8) ? xcd * (qq + 1) : rr8 * (qq + 1) + (xcd - rr8) * qq) + (bid >> 3);
  const int mt = wg / ntn, nt = wg - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A), rwh = rsrc(whi), rwl = rsrc(wlo);
  // staging: A 4 float4 per thread (rows srow + 64 i, k c4..c4+3); W 4 x 16 B
  const int srow = tid >> 3, c4 = (tid & 7) * 4;
  int aoff[4], boff[4], bls[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + srow + 64 * i;
    aoff[i] = m < M ? (m * K + c4) * 4 : kOOB;
    const int q = tid + NT * i, img = i >= 2, qr = q - img * 1024;
    const int row = qr >> 2, part = qr & 3;
    boff[i] = ((n0 + row) * K + part * 8) * 2;
    bls[i] = loff<MF>(row, part * 16) + (img ? IMG : 0);
  }
  f32x4 ra_[4];
  bf16x8 rb_[4];
  auto load_tile = [&](int k0, bool live) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int o = live ? boff[i] + k0 * 2 : kOOB;
      rb_[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(i >= 2 ? rwl : rwh, o, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = (live && aoff[i] != kOOB) ? aoff[i] + k0 * 4 : kOOB;
      ra_[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, 0));
    }
  };
  auto store_tile = [&](int buf) {
    unsigned char* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h = (__bf16)ra_[i][e];
        hi[e] = h;
        lo[e] = (__bf16)(ra_[i][e] - (float)h);
      }
      const int off = loff<MF>(srow + 64 * i, c4 * 2);
      *reinterpret_cast<bf16x4*>(st + off) = hi;
      *reinterpret_cast<bf16x4*>(st + IMG + off) = lo;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<bf16x8*>(st + 2 * IMG + bls[i]) = rb_[i];
  };
  const int wm = wave >> 1, wn = wave & 1;  // 4 x 2 waves of 64 x 128
  if constexpr (MF == 32) {
    const int r32 = lane & 31, h = lane >> 5;
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto mma_step = [&](int buf, int s) {
      const unsigned char* st = smem + buf * STAGE;
      bf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = loff<32>(wm * 64 + i * 32 + r32, h * 16 + s * 32);
        ah[i] = *reinterpret_cast<const bf16x8*>(st + o);
        al[i] = *reinterpret_cast<const bf16x8*>(st + IMG + o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = loff<32>(wn * 128 + j * 32 + r32, h * 16 + s * 32);
        bh[j] = *reinterpret_cast<const bf16x8*>(st + 2 * IMG + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(st + 3 * IMG + o);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    };
    const int nk = K / BK;
    load_tile(0, true);
    store_tile(0);
    load_tile(BK, true);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      mma_step(buf, 0);
      store_tile(buf ^ 1);
      load_tile((kt + 2) * BK, kt + 2 < nk);
      mma_step(buf, 1);
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const int col = n0 + wn * 128 + j * 32 + r32;
          if (row < M) out[(size_t)row * N + col] = acc[i][j][r];
        }
  } else {
    // 16x16x32: lane l holds A[row l & 15][k 8 (l >> 4) .. +7]; quarter steps of
    // 2 row blocks x 4 column blocks keep 48 fragment registers live, as MF = 32
    const int r16 = lane & 15, qk = lane >> 4;
    f32x4 acc[4][8];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mma_q = [&](int buf, int ih, int jh) {
      const unsigned char* st = smem + buf * STAGE;
      bf16x8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = loff<16>(wm * 64 + (ih * 2 + i) * 16 + r16, qk * 16);
        ah[i] = *reinterpret_cast<const bf16x8*>(st + o);
        al[i] = *reinterpret_cast<const bf16x8*>(st + IMG + o);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = loff<16>(wn * 128 + (jh * 4 + j) * 16 + r16, qk * 16);
        bh[j] = *reinterpret_cast<const bf16x8*>(st + 2 * IMG + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(st + 3 * IMG + o);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4& c = acc[ih * 2 + i][jh * 4 + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
        }
    };
    // MF 17: snake order (0,0) (0,1) (1,1) (1,0), each quarter re-reading only the fragments it
    // does not share with the previous one (32 instead of 48 ds_read_b128 per k-tile)
    bf16x8 ah[2], al[2], bh[4], bl[4];
    auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int o = loff<16>(wm * 64 + (ih * 2 + i) * 16 + r16, qk * 16);
        ah[i] = *reinterpret_cast<const bf16x8*>(st + o);
        al[i] = *reinterpret_cast<const bf16x8*>(st + IMG + o);
      }
    };
    auto rdB = [&](const unsigned char* st, int jh) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = loff<16>(wn * 128 + (jh * 4 + j) * 16 + r16, qk * 16);
        bh[j] = *reinterpret_cast<const bf16x8*>(st + 2 * IMG + o);
        bl[j] = *reinterpret_cast<const bf16x8*>(st + 3 * IMG + o);
      }
    };
    auto mm = [&](int ih, int jh) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4& c = acc[ih * 2 + i][jh * 4 + j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
        }
    };
    const int nk = K / BK;
    load_tile(0, true);
    store_tile(0);
    load_tile(BK, true);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if constexpr (MF == 17) {
        const unsigned char* st = smem + buf * STAGE;
        rdA(st, 0);
        rdB(st, 0);
        mm(0, 0);
        rdB(st, 1);
        mm(0, 1);
        store_tile(buf ^ 1);
        load_tile((kt + 2) * BK, kt + 2 < nk);
        rdA(st, 1);
        mm(1, 1);
        rdB(st, 0);
        mm(1, 0);
      } else {
        mma_q(buf, 0, 0);
        mma_q(buf, 0, 1);
        store_tile(buf ^ 1);
        load_tile((kt + 2) * BK, kt + 2 < nk);
        mma_q(buf, 1, 0);
        mma_q(buf, 1, 1);
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * 64 + i * 16 + qk * 4 + r;
          const int col = n0 + wn * 128 + j * 16 + r16;
          if (row < M) out[(size_t)row * N + col] = acc[i][j][r];
        }
  }
}


// ---------------------------------------------------------------------------------------
// Variant G: every operand by LDS-DMA (buffer_load ... lds, 16 B per lane), A staged as the
// fp32 it is (no register staging set, no ds_write pass) and split into bf16 hi / lo when
// its fragments are read.  LDS per stage: A [256][32] fp32 (128-B rows, 16-B chunk c of row
// r at slot c ^ ((r >> 1) & 5): conflict-free 2 x ds_read_b128 per 16x16x32 fragment) +
// W hi / lo [256][32] bf16 (64-B rows, the {0,2,3,1} swizzle).  Two stages: tile k + 1 lands
// while tile k multiplies; one vmcnt(0) + barrier per k-tile.
typedef __attribute__((address_space(3))) void lds_void;
constexpr int GA = BM * 128, GW = BN * 64, GSTAGE = GA + 2 * GW;  // 64 KB
__device__ __forceinline__ int aslot(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 5)) << 4); }

template <int PRE>
__global__ __launch_bounds__(NT, 1) void gemm_g(const float* __restrict__ A, const __bf16* __restrict__ whi,
                                                const __bf16* __restrict__ wlo, float* __restrict__ out, int M,
                                                int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = N / BN;
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr8 = nwg & 7;
  const int wg = ((xcd < rr8) ? xcd * (qq + 1) : rr8 * (qq + 1) + (xcd - rr8) * qq) + (bid >> 3);
  const int mt = wg / ntn, nt = wg - mt * ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A), rwh = rsrc(whi), rwl = rsrc(wlo);
  // DMA geometry.  A: wave-instruction i (0..3) of wave w fills rows (4 w + i) * 8 .. + 7, lane l
  // row + (l >> 3), slot l & 7 <- global chunk (l & 7) ^ swz(row).  W: instruction i (0..1) of
  // wave w fills rows (2 w + i) * 16 .. + 15 of hi and of lo, lane l row + (l >> 2), slot l & 3.
  int aoff[4], woff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (4 * wave + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 5);
    const int m = m0 + row;
    aoff[i] = m < M ? (m * K + 4 * c) * 4 : kOOB;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (2 * wave + i) * 16 + (lane >> 2);
    const int q = (row >> 2) & 3;
    const int c = ((lane & 3) ^ ((0x1320 >> (4 * q)) & 3));
    woff[i] = ((n0 + row) * K + 8 * c) * 2;
  }
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * GSTAGE;
    const bool live = kt * BK < K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(st + (4 * wave + i) * 1024),
                                               16, live && aoff[i] != kOOB ? aoff[i] + kt * BK * 4 : kOOB, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int o = live ? woff[i] + kt * BK * 2 : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwh, (lds_void*)(st + GA + (2 * wave + i) * 1024), 16, o, 0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rwl, (lds_void*)(st + GA + GW + (2 * wave + i) * 1024), 16, o, 0, 0,
                                               0);
    }
  };
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, qk = lane >> 4;
  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[2], al[2], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st, int ih) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 64 + (ih * 2 + i) * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[i][e] = h0;
        ah[i][4 + e] = h1;
        al[i][e] = (__bf16)(x0[e] - (float)h0);
        al[i][4 + e] = (__bf16)(x1[e] - (float)h1);
      }
    }
  };
  auto rdB = [&](const unsigned char* st, int jh) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = loff<16>(wn * 128 + (jh * 4 + j) * 16 + r16, qk * 16);
      bh[j] = *reinterpret_cast<const bf16x8*>(st + GA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + GA + GW + o);
    }
  };
  auto mm = [&](int ih, int jh) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[ih * 2 + i][jh * 4 + j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
      }
  };
  const int nk = K / BK;
  if constexpr (PRE == 1) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  dma(0, 0);
  dma(1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 (8 DMAs per tile per lane)
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const unsigned char* st = smem + buf * GSTAGE;
    rdA(st, 0);
    rdB(st, 0);
    mm(0, 0);
    rdB(st, 1);
    mm(0, 1);
    rdA(st, 1);
    mm(1, 1);
    rdB(st, 0);
    mm(1, 0);
    // tile kt + 1 (issued one k-tile ago) has landed; every wave is done with this buffer
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma(kt + 2, buf);  // past-the-end tiles: out-of-range DMAs (zeros nobody reads)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + qk * 4 + r;
        const int col = n0 + wn * 128 + j * 16 + r16;
        if (row < M) out[(size_t)row * N + col] = acc[i][j][r];
      }
}


// Variant G3: 256 x 128 block (8 waves of 64 x 64), the same LDS-DMA staging, THREE stages
// (48 KB each): tiles k + 1 and k + 2 are in flight while tile k multiplies.
constexpr int G3N = 128, G3W = G3N * 64, G3STAGE = GA + 2 * G3W;  // 48 KB
__global__ __launch_bounds__(NT, 1) void gemm_g3(const float* __restrict__ A, const __bf16* __restrict__ whi,
                                                 const __bf16* __restrict__ wlo, float* __restrict__ out, int M,
                                                 int N, int K) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = N / G3N;
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr8 = nwg & 7;
  const int wg = ((xcd < rr8) ? xcd * (qq + 1) : rr8 * (qq + 1) + (xcd - rr8) * qq) + (bid >> 3);
  const int mt = wg / ntn, nt = wg - mt * ntn;
  const int m0 = mt * BM, n0 = nt * G3N;
  const __amdgpu_buffer_rsrc_t ra = rsrc(A), rwh = rsrc(whi), rwl = rsrc(wlo);
  int aoff[4], woff;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (4 * wave + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 5);
    const int m = m0 + row;
    aoff[i] = m < M ? (m * K + 4 * c) * 4 : kOOB;
  }
  {
    const int row = wave * 16 + (lane >> 2);
    const int q = (row >> 2) & 3;
    const int c = ((lane & 3) ^ ((0x1320 >> (4 * q)) & 3));
    woff = ((n0 + row) * K + 8 * c) * 2;
  }
  auto dma = [&](int kt, int buf) {
    unsigned char* st = smem + buf * G3STAGE;
    const bool live = kt * BK < K;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(st + (4 * wave + i) * 1024),
                                               16, live && aoff[i] != kOOB ? aoff[i] + kt * BK * 4 : kOOB, 0, 0, 0);
    const int o = live ? woff + kt * BK * 2 : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rwh, (lds_void*)(st + GA + wave * 1024), 16, o, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rwl, (lds_void*)(st + GA + G3W + wave * 1024), 16, o, 0, 0, 0);
  };
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, qk = lane >> 4;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ah[4], al[4], bh[4], bl[4];
  auto rdA = [&](const unsigned char* st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + i * 16 + r16;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk));
      const f32x4 x1 = *reinterpret_cast<const f32x4*>(st + aslot(r, 2 * qk + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const __bf16 h0 = (__bf16)x0[e], h1 = (__bf16)x1[e];
        ah[i][e] = h0;
        ah[i][4 + e] = h1;
        al[i][e] = (__bf16)(x0[e] - (float)h0);
        al[i][4 + e] = (__bf16)(x1[e] - (float)h1);
      }
    }
  };
  auto rdB = [&](const unsigned char* st) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = loff<16>(wn * 64 + j * 16 + r16, qk * 16);
      bh[j] = *reinterpret_cast<const bf16x8*>(st + GA + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(st + GA + G3W + o);
    }
  };
  const int nk = K / BK;
  dma(0, 0);
  dma(1, 1);
  dma(2, 2);
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // tile 0 (6 DMAs per tile per lane)
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt % 3;
    const unsigned char* st = smem + buf * G3STAGE;
    rdB(st);
    rdA(st);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        f32x4& c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], c, 0, 0, 0);
      }
    // tile kt + 1 has landed (kt + 2 may still be in flight); every wave is done with buf
    asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    dma(kt + 3, buf);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + qk * 4 + r;
        const int col = n0 + wn * 64 + j * 16 + r16;
        if (row < M) out[(size_t)row * N + col] = acc[i][j][r];
      }
}

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

int main(int argc, char** argv) {
  const int M = argc > 1 ? std::atoi(argv[1]) : 127488, N = argc > 2 ? std::atoi(argv[2]) : 1024;
  const int K = argc > 3 ? std::atoi(argv[3]) : 1024, reps = argc > 4 ? std::atoi(argv[4]) : 20;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> ua(-1.f, 1.f), uw(-0.05f, 0.05f);
  std::vector<float> a((size_t)M * K), w((size_t)N * K);
  for (auto& x : a) x = std::fmax(ua(rng), 0.f);  // post-ReLU activations
  for (auto& x : w) x = uw(rng);
  std::vector<uint16_t> hi(w.size()), lo(w.size());
  for (size_t i = 0; i < w.size(); ++i) {
    hi[i] = f2bf(w[i]);
    lo[i] = f2bf(w[i] - bf2f(hi[i]));
  }
  float *da, *o1, *o2, *o3;
  void *dh, *dl;
  CK(hipMalloc(&da, a.size() * 4));
  CK(hipMalloc(&o1, (size_t)M * N * 4));
  CK(hipMalloc(&o2, (size_t)M * N * 4));
  CK(hipMalloc(&o3, (size_t)M * N * 4));
  CK(hipMalloc(&dh, hi.size() * 2));
  CK(hipMalloc(&dl, lo.size() * 2));
  CK(hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dh, hi.data(), hi.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int nwg = ((M + BM - 1) / BM) * (N / BN);
  auto run = [&](int mf, float* o) {
    if (mf == 32)
      hipLaunchKernelGGL(gemm_kernel<32>, dim3(nwg), dim3(NT), 2 * STAGE, s, da, (const __bf16*)dh,
                         (const __bf16*)dl, o, M, N, K);
    else if (mf == 98)
      hipLaunchKernelGGL(gemm_g3, dim3(((M + BM - 1) / BM) * (N / G3N)), dim3(NT), 3 * G3STAGE, s, da,
                         (const __bf16*)dh, (const __bf16*)dl, o, M, N, K);
    else if (mf == 99)
      hipLaunchKernelGGL(gemm_g<0>, dim3(nwg), dim3(NT), 2 * GSTAGE, s, da, (const __bf16*)dh, (const __bf16*)dl, o, M,
                         N, K);
    else if (mf == 97)
      hipLaunchKernelGGL(gemm_g<1>, dim3(nwg), dim3(NT), 2 * GSTAGE, s, da, (const __bf16*)dh, (const __bf16*)dl, o, M,
                         N, K);
    else if (mf == 17)
      hipLaunchKernelGGL(gemm_kernel<17>, dim3(nwg), dim3(NT), 2 * STAGE, s, da, (const __bf16*)dh,
                         (const __bf16*)dl, o, M, N, K);
    else
      hipLaunchKernelGGL(gemm_kernel<16>, dim3(nwg), dim3(NT), 2 * STAGE, s, da, (const __bf16*)dh,
                         (const __bf16*)dl, o, M, N, K);
  };
  // interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)
  for (int round = 0; round < 4; ++round) {
    for (int mf : {17, 99, 97}) {
      float* o = mf == 17 ? o1 : (mf == 99 ? o2 : o3);
      run(mf, o);
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) run(mf, o);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      std::printf("round %d MF%-2d M=%d N=%d K=%d  %8.4f ms  %7.1f TF algorithmic\n", round, mf, M, N, K, ms,
                  2.0 * M * N * K / (ms * 1e-3) / 1e12);
      std::fflush(stdout);
    }
  }
  std::vector<float> r1((size_t)M * N), r2((size_t)M * N);
  CK(hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost));
  double md = 0, mx = 0;
  for (size_t i = 0; i < r1.size(); ++i) {
    md = std::fmax(md, std::fabs(r1[i] - r2[i]));
    mx = std::fmax(mx, std::fabs(r1[i]));
  }
  // exact check of a few rows against a host f64 product
  double he = 0;
  for (int m : {0, 1, M / 2, M - 1})
    for (int n = 0; n < N; n += 37) {
      double acc = 0;
      for (int k = 0; k < K; ++k) acc += (double)a[(size_t)m * K + k] * w[(size_t)n * K + k];
      he = std::fmax(he, std::fabs(acc - r2[(size_t)m * N + n]));
    }
  std::printf("max |MF17 - G| = %.3g (max |y| %.3g); max |G - f64 host| = %.3g\n", md, mx, he);
  std::vector<float> r3((size_t)M * N);
  CK(hipMemcpy(r3.data(), o3, r3.size() * 4, hipMemcpyDeviceToHost));
  double md3 = 0;
  for (size_t i = 0; i < r1.size(); ++i) md3 = std::fmax(md3, std::fabs(r1[i] - r3[i]));
  std::printf("max |MF17 - G(prio)| = %.3g\n", md3);
  return 0;
}
