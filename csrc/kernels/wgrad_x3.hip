// dgraph_amd — fp32 weight gradient C = [A1[a1(m)] | A2[m]]^T G, summed over m, as bf16x3
// split-product MFMAs (gfx950). Same contract as wgrad_f32.hip (per-block partial slabs,
// fixed-order reduce, fresh_from accumulation across calls); only the products differ.
//
// Every fp32 operand value is split exactly into bf16 hi + mid + lo (gemm_x3.hip) while it
// is staged into LDS, and each 32-deep reduction stage runs SIX 16x16x32 bf16 MFMAs per
// output tile (a_lo g_hi, a_hi g_lo, a_mid g_mid, a_mid g_hi, a_hi g_mid, a_hi g_hi; the
// dropped terms total <= 2^-24 |a g|) instead of eight 16x16x4 f32 ones at twice the cycles.
// The reduction index m is the MFMA's k: both operands are staged TRANSPOSED, [3][K][32] and
// [3][N][32] bf16 (m contiguous), so a lane's 8-deep fragment is one 16-B LDS read. Staging
// slot t covers two consecutive m rows of one 4-column chunk (one b32 write of the pair per
// column and part; consecutive threads take consecutive m pairs: conflict-free writes).
// One LDS buffer (96 KB at K = N = 256), two barriers per stage, next stage's global loads in
// flight during the MFMAs.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int kWRows = 32;
constexpr int kWThr = 512;

template <int K, int N>
struct WXCfg {
  static constexpr int NTK = K / 16, NTN = N / 16;
  // 256 x 256: 8 waves along K (2 x 16 tiles each: fewer cached A fragments, no spills)
  static constexpr bool TWO = (NTN % 2 == 0) && (NTK % 4 == 0) && !(K == 256 && N == 256);
  static constexpr int WN = TWO ? 2 : 1;
  static constexpr int WM = TWO ? 4 : 8;
  static constexpr int TM = NTK / WM, TN = NTN / WN;
  static constexpr int A_PART = K * kWRows, G_PART = N * kWRows;  // bf16 per part
  static constexpr size_t BYTES = 3 * (A_PART + G_PART) * 2;
  // staging pair-slots: (K/4 column chunks) x (16 m pairs)
  static constexpr int A_SL = (K / 4) * 16 / kWThr;  // per thread
  static_assert(TM >= 1 && TM * WM == NTK && TN * WN == NTN, "wgrad tiling");
  static_assert(A_SL >= 1 && A_SL * kWThr == (K / 4) * 16, "K slots");
  static_assert(BYTES <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ uint32_t rne_hi_w(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u & 0xFFFF0000u;
}
__device__ __forceinline__ void split1(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = rne_hi_w(x);
  const float r1 = x - __uint_as_float(h);
  m = rne_hi_w(r1);
  l = __float_as_uint(r1 - __uint_as_float(m));
}
__device__ __forceinline__ uint32_t pk(uint32_t e0, uint32_t e1) {
  return __builtin_amdgcn_perm(e1, e0, 0x07060302u);
}
__device__ __forceinline__ f32x4 mfw(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

template <int K, int N>
__global__ __launch_bounds__(kWThr, 1) void wgrad_x3_kernel(
    const float* __restrict__ A1, int64_t lda1, int K1, const float* __restrict__ A2,
    int64_t lda2, const int64_t* __restrict__ a1_rows, const float* __restrict__ G,
    int64_t ldg, int64_t M, int64_t rows_per_block, float* __restrict__ partials,
    int fresh_from) {
  using C = WXCfg<K, N>;
  constexpr int TM = C::TM, TN = C::TN, WN = C::WN;
  constexpr int NGS = (N / 4) * 16;  // G pair-slots in a stage
  constexpr int G_SL = (NGS + kWThr - 1) / kWThr;
  extern __shared__ __attribute__((aligned(16))) uint16_t wl[];
  uint16_t* sa = wl;                     // [3][K][32]
  uint16_t* sg = wl + 3 * C::A_PART;     // [3][N][32]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15;
  const int lh = lane >> 4;
  const int64_t m_begin = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  int64_t m_end = m_begin + rows_per_block;
  m_end = m_end < M ? m_end : M;
  const int64_t nst = m_end > m_begin ? (m_end - m_begin + kWRows - 1) / kWRows : 0;

  // pair-slot v of this thread: m pair p = slot % 16 (rows 2p, 2p+1), column chunk slot / 16
  f32x4 ra[C::A_SL][2];
  f32x4 rg[G_SL][2];
  int64_t ix[C::A_SL][2];
  auto row_of = [&](int64_t s, int rr) {
    const int64_t m = m_begin + s * kWRows + rr;
    return m < m_end ? m : m_begin;
  };
  auto load_idx = [&](int64_t s) {
#pragma unroll
    for (int v = 0; v < C::A_SL; ++v) {
      const int slot = tid + kWThr * v;
      const int p = slot % 16, c = (slot / 16) * 4;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int64_t mm = row_of(s, 2 * p + h);
        ix[v][h] = (a1_rows && c < K1) ? a1_rows[mm] : mm;
      }
    }
  };
  auto load_data = [&](int64_t s) {
#pragma unroll
    for (int v = 0; v < C::A_SL; ++v) {
      const int slot = tid + kWThr * v;
      const int c = (slot / 16) * 4;
      const bool first = c < K1;
      const float* base = first ? A1 : A2;
      const int64_t ld = first ? lda1 : lda2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        ra[v][h] = *reinterpret_cast<const f32x4*>(base + ix[v][h] * ld + (first ? c : c - K1));
    }
#pragma unroll
    for (int v = 0; v < G_SL; ++v) {
      int slot = tid + kWThr * v;
      slot = slot < NGS ? slot : NGS - 1;
      const int p = slot % 16, c = (slot / 16) * 4;
#pragma unroll
      for (int h = 0; h < 2; ++h)
        rg[v][h] = *reinterpret_cast<const f32x4*>(G + row_of(s, 2 * p + h) * ldg + c);
    }
  };
  auto store_stage = [&](int64_t s) {
#pragma unroll
    for (int v = 0; v < C::A_SL; ++v) {
      const int slot = tid + kWThr * v;
      const int p = slot % 16, c = (slot / 16) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split1(ra[v][0][i], h0, m0, l0);
        split1(ra[v][1][i], h1, m1, l1);
        uint32_t* q = reinterpret_cast<uint32_t*>(sa + (c + i) * kWRows + 2 * p);
        q[0] = pk(h0, h1);
        q[C::A_PART / 2] = pk(m0, m1);
        q[C::A_PART] = pk(l0, l1);
      }
    }
#pragma unroll
    for (int v = 0; v < G_SL; ++v) {
      int slot = tid + kWThr * v;
      slot = slot < NGS ? slot : NGS - 1;  // surplus slots rewrite the last pair (same values)
      const int p = slot % 16, c = (slot / 16) * 4;
      // rows past the block's range contribute zero (zeroing one operand suffices)
      const bool ok0 = m_begin + s * kWRows + 2 * p < m_end;
      const bool ok1 = m_begin + s * kWRows + 2 * p + 1 < m_end;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split1(ok0 ? rg[v][0][i] : 0.f, h0, m0, l0);
        split1(ok1 ? rg[v][1][i] : 0.f, h1, m1, l1);
        uint32_t* q = reinterpret_cast<uint32_t*>(sg + (c + i) * kWRows + 2 * p);
        q[0] = pk(h0, h1);
        q[C::G_PART / 2] = pk(m0, m1);
        q[C::G_PART] = pk(l0, l1);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kw = wm * TM * 16, nw = wn * TN * 16;
  if (nst > 0) {
    load_idx(0);
    load_data(0);
    load_idx(nst > 1 ? 1 : 0);
    for (int64_t s = 0; s < nst; ++s) {
      __syncthreads();  // every wave is done reading the previous stage
      store_stage(s);
      const int64_t sn = s + 1 < nst ? s + 1 : s;
      load_data(sn);  // in flight during this stage's MFMAs
      load_idx(s + 2 < nst ? s + 2 : sn);
      __syncthreads();
      uint4 ah[TM], am[TM], al[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int off = (kw + a * 16 + li) * kWRows + lh * 8;
        ah[a] = *reinterpret_cast<const uint4*>(sa + off);
        am[a] = *reinterpret_cast<const uint4*>(sa + C::A_PART + off);
        al[a] = *reinterpret_cast<const uint4*>(sa + 2 * C::A_PART + off);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int off = (nw + b * 16 + li) * kWRows + lh * 8;
        const uint4 gh = *reinterpret_cast<const uint4*>(sg + off);
        const uint4 gm = *reinterpret_cast<const uint4*>(sg + C::G_PART + off);
        const uint4 gl = *reinterpret_cast<const uint4*>(sg + 2 * C::G_PART + off);
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          f32x4 c = acc[a][b];
          c = mfw(al[a], gh, c);
          c = mfw(ah[a], gl, c);
          c = mfw(am[a], gm, c);
          c = mfw(am[a], gh, c);
          c = mfw(ah[a], gm, c);
          acc[a][b] = mfw(ah[a], gh, c);
        }
      }
    }
  }
  float* slab = partials + static_cast<int64_t>(blockIdx.x) * K * N;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = kw + a * 16 + 4 * lh + r;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        float* p = slab + k * N + nw + b * 16 + li;
        *p = static_cast<int>(blockIdx.x) < fresh_from ? *p + acc[a][b][r] : acc[a][b][r];
      }
    }
}

template <int K, int N>
hipError_t launch_wx3(const float* A1, int64_t lda1, int K1, const float* A2, int64_t lda2,
                      const int64_t* a1_rows, const float* G, int64_t ldg, int64_t M,
                      float* partials, int P, int fresh_from, hipStream_t st) {
  using C = WXCfg<K, N>;
  auto kern = &wgrad_x3_kernel<K, N>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(C::BYTES));
    attr = true;
  }
  int64_t rpb = (M + P - 1) / P;
  rpb = (rpb + kWRows - 1) / kWRows * kWRows;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(P)), dim3(kWThr), C::BYTES, st, A1, lda1,
                     K1, A2, lda2, a1_rows, G, ldg, M, rpb, partials, fresh_from);
  return hipGetLastError();
}

}  // namespace

bool wgrad_x3_supported(int64_t K, int64_t N) {
  return (K == 128 || K == 256) && (N == 128 || N == 192 || N == 256);
}

hipError_t wgrad_x3(const float* A1, int64_t lda1, int64_t K1, const float* A2, int64_t lda2,
                    int64_t K2, const int64_t* a1_rows, const float* G, int64_t ldg, int64_t M,
                    int64_t N, float* partials, int P, int fresh_from, hipStream_t st) {
  const int64_t K = K1 + (A2 ? K2 : 0);
  if (!wgrad_x3_supported(K, N) || P <= 0 || M < 0) return hipErrorInvalidValue;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (K1 % 4 || !al(A1) || lda1 % 4 || !al(G) || ldg % 4) return hipErrorInvalidValue;
  if (A2 && K2 > 0 && (!al(A2) || lda2 % 4)) return hipErrorInvalidValue;
  const int k1 = static_cast<int>(K1);
#define DG_WX(K_, N_)                                                                    \
  if (K == K_ && N == N_)                                                                \
    return launch_wx3<K_, N_>(A1, lda1, k1, A2, lda2, a1_rows, G, ldg, M, partials, P,  \
                              fresh_from, st);
  DG_WX(256, 256) DG_WX(256, 192) DG_WX(256, 128)
  DG_WX(128, 256) DG_WX(128, 192) DG_WX(128, 128)
#undef DG_WX
  return hipErrorInvalidValue;
}

}  // namespace dgraph
