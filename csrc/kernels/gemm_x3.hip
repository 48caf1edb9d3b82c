// dgraph_amd — fp32 dual GEMM for the GraphSAGE combine as bf16x3 split-product MFMAs (gfx950).
//
//   out[o(i), :] = epi( A1[a(i), 0:K1] @ B1[K1, N] (+ A2[i, 0:K2] @ B2[K2, N]) )   (gemm_f32.hip)
//
// gfx950 has no xf32: the exact-f32 MFMA (v_mfma_f32_16x16x4_f32) runs at the f32 VECTOR
// rate, 1/16 of bf16 MFMA. Every fp32 value x is exactly hi + mid + lo with hi = rne_bf16(x),
// mid = rne_bf16(x - hi), lo = x - hi - mid (<= 8 significant bits, exact in bf16; x normal).
// The product a*b is the sum of the nine part products; the six kept here
//   a_lo b_hi, a_hi b_lo, a_mid b_mid, a_mid b_hi, a_hi b_mid, a_hi b_hi   (smallest first)
// are exact in fp32 and accumulate in fp32; the three dropped ones total <= 2^-24 |a b|, i.e.
// below one fp32 rounding of the product. Measured against fp64: max error 3.6-4.4e-7 of
// sum|a b| vs 4.5-5.3e-7 for the exact-f32 MFMA (profiles/r03/gemm_bf16x3_vs_f32_probe.log):
// fp32-accurate results, 6 x 16 cycles of MFMA per 32-deep stage instead of 8 x 32.
//
// Operand preparation:
//   * B (the weights, small): split ONCE per call on the host side into bf16 parts stored
//     [3][N][K] (k contiguous, so a lane's 8-deep B fragment is one 16-B LDS read);
//   * A (the tall activation operand): read as fp32 and split once per stage while staging
//     into LDS as [3][BM][32] bf16 (every element is split by exactly one thread).
// Tile: BM = 128 rows x all N columns, 512 threads = 8 waves as 2 (rows) x 4 (columns), each
// wave 64 rows x N/4 columns = 4 x N/64 16x16 tiles; K in 32-deep stages through two LDS
// buffers (register-staged global loads issued one stage ahead, one barrier per stage);
// persistent grid (one block per CU) walking 128-row tiles with next-tile prefetch.
// Epilogue identical to gemm_f32 (row scale, bias, cin, gate, ReLU, row-mapped store).
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

constexpr int kXBM = 128;
constexpr int kXBK = 32;
constexpr int kXThr = 512;

template <int N>
struct XCfg {
  static constexpr int WM = 2, WN = 4;
  static constexpr int TM = kXBM / (16 * WM);  // 4
  static constexpr int TN = N / (16 * WN);     // N / 64
  static constexpr int A_PART = kXBM * kXBK;   // bf16 elements per A part
  static constexpr int B_PART = N * kXBK;      // bf16 elements per B part
  static constexpr int STAGE_B16 = 3 * (A_PART + B_PART);
  static constexpr size_t BYTES = 2 * STAGE_B16 * 2;
  static constexpr int A_V4 = kXBM * kXBK / 4 / kXThr;                 // fp32 float4 / thread = 2
  static constexpr int B_U4 = (3 * B_PART / 8 + kXThr - 1) / kXThr;    // 16-B chunks / thread
  static_assert(TN >= 1 && TN * 16 * WN == N, "N must be a multiple of 64");
  static_assert(BYTES <= 160 * 1024, "LDS budget");
};

__device__ __forceinline__ uint32_t rne_hi_bits(float x) {
  uint32_t u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return u & 0xFFFF0000u;
}
__device__ __forceinline__ uint32_t pack2(uint32_t e0, uint32_t e1) {
  return __builtin_amdgcn_perm(e1, e0, 0x07060302u);  // [e0.hi16 | e1.hi16 << 16]
}
// 4 fp32 -> 3 x 4 bf16 (hi, mid, lo), each as 2 packed words
__device__ __forceinline__ void split4(const f32x4& f, uint2& H, uint2& M, uint2& L) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float x = f[k];
    h[k] = rne_hi_bits(x);
    const float r1 = x - __uint_as_float(h[k]);
    m[k] = rne_hi_bits(r1);
    l[k] = __float_as_uint(r1 - __uint_as_float(m[k]));
  }
  H = uint2{pack2(h[0], h[1]), pack2(h[2], h[3])};
  M = uint2{pack2(m[0], m[1]), pack2(m[2], m[3])};
  L = uint2{pack2(l[0], l[1]), pack2(l[2], l[3])};
}
__device__ __forceinline__ f32x4 mfma3(const uint4& a, const uint4& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

template <int N, bool HAS_A2, bool RELU, bool HAS_BIAS, bool HAS_CIN, bool HAS_GATE>
__global__ __launch_bounds__(kXThr, 1) void gemm_x3_kernel(
    const float* __restrict__ A1, int64_t lda1, int K1, const uint16_t* __restrict__ B1p,
    const float* __restrict__ A2, int64_t lda2, int K2, const uint16_t* __restrict__ B2p,
    const int64_t* __restrict__ a_rows, const float* __restrict__ bias, const float* cin,
    int64_t ldc, float beta, const float* __restrict__ gate, int64_t ldg,
    const int64_t* __restrict__ o_rows, const float* __restrict__ row_scale, float* out,
    int64_t ldo, int64_t M) {
  using C = XCfg<N>;
  constexpr int TM = C::TM, TN = C::TN, WN = C::WN;
  extern __shared__ __attribute__((aligned(16))) uint16_t xl[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15;
  const int lh = lane >> 4;
  const int K = K1 + K2;
  const int nst = K / kXBK;
  const int64_t ntiles = (M + kXBM - 1) / kXBM;
  int64_t tile = blockIdx.x;
  if (tile >= ntiles) return;  // block-uniform

  // A stage slots: float4 q = tid + kXThr * u -> row q / 8, k chunk q % 8 (4 k each)
  int32_t a_src_row[C::A_V4];
  int32_t nx_src_row[C::A_V4];
  int64_t ld_tile = tile;
  auto rows_of = [&](int64_t t, int32_t* a1) {
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = tid + kXThr * u;
      int64_t r = t * kXBM + q / 8;
      r = r < M ? r : M - 1;
      a1[u] = static_cast<int32_t>(a_rows ? a_rows[r] : r);
    }
  };
  rows_of(tile, a_src_row);
  f32x4 ra[C::A_V4];
  uint4 rb[C::B_U4];
  auto load_stage = [&](int s) {
    const int k0 = s * kXBK;
    const bool first = !HAS_A2 || k0 < K1;
    const float* Ab = first ? A1 : A2;
    const int64_t lda = first ? lda1 : lda2;
    const int ka = first ? k0 : k0 - K1;
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = tid + kXThr * u;
      int64_t r2 = ld_tile * kXBM + q / 8;
      r2 = r2 < M ? r2 : M - 1;
      const int64_t ar = first ? static_cast<int64_t>(a_src_row[u]) : r2;
      ra[u] = *reinterpret_cast<const f32x4*>(Ab + ar * lda + ka + (q % 8) * 4);
    }
    // B parts: [3][N][Kx] bf16 (k contiguous); this stage's [3][N][32] slice as 16-B chunks
    const uint16_t* Bp = first ? B1p : B2p;
    const int Kx = first ? K1 : K2;
#pragma unroll
    for (int u = 0; u < C::B_U4; ++u) {
      int q = tid + kXThr * u;
      q = q < 3 * C::B_PART / 8 ? q : 3 * C::B_PART / 8 - 1;  // unconditional (clamped)
      const int pn = q / 4, c = q % 4;                        // (part, n) row, 8-k chunk
      const int part = pn / N, n = pn % N;
      rb[u] = *reinterpret_cast<const uint4*>(Bp + (static_cast<int64_t>(part) * N + n) * Kx +
                                              ka + c * 8);
    }
  };
  auto store_stage = [&](int buf) {
    uint16_t* sa = xl + buf * C::STAGE_B16;  // [3][BM][32]
    uint16_t* sb = sa + 3 * C::A_PART;       // [3][N][32]
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = tid + kXThr * u;
      const int r = q / 8, c = q % 8;
      uint2 h, m, l;
      split4(ra[u], h, m, l);
      const int off = r * kXBK + c * 4;
      *reinterpret_cast<uint2*>(sa + off) = h;
      *reinterpret_cast<uint2*>(sa + C::A_PART + off) = m;
      *reinterpret_cast<uint2*>(sa + 2 * C::A_PART + off) = l;
    }
#pragma unroll
    for (int u = 0; u < C::B_U4; ++u) {
      int q = tid + kXThr * u;
      q = q < 3 * C::B_PART / 8 ? q : 3 * C::B_PART / 8 - 1;
      *reinterpret_cast<uint4*>(sb + q * 8) = rb[u];  // [part][n][32]: chunk q at 8 q
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_stage(0);
  store_stage(0);
  __syncthreads();
  const int arow_w = wm * TM * 16;
  const int bcol_w = wn * TN * 16;
  int g = 0;
  while (true) {
    const int64_t next = tile + gridDim.x;
    const bool has_next = next < ntiles;
    rows_of(has_next ? next : tile, nx_src_row);
    for (int s = 0; s < nst; ++s, ++g) {
      const int buf = g & 1;
      const bool last = s + 1 == nst;
      const bool switch_tile = last && has_next;
#pragma unroll
      for (int u = 0; u < C::A_V4; ++u) a_src_row[u] = switch_tile ? nx_src_row[u] : a_src_row[u];
      ld_tile = switch_tile ? next : ld_tile;
      load_stage(last ? 0 : s + 1);
      __builtin_amdgcn_sched_barrier(0);
      const uint16_t* sa = xl + buf * C::STAGE_B16;
      const uint16_t* sb = sa + 3 * C::A_PART;
      // A fragments: row (arow_w + 16 a + li), k = 8 lh .. 8 lh + 7 of each part
      uint4 ah[TM], am[TM], al[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int off = (arow_w + a * 16 + li) * kXBK + lh * 8;
        ah[a] = *reinterpret_cast<const uint4*>(sa + off);
        am[a] = *reinterpret_cast<const uint4*>(sa + C::A_PART + off);
        al[a] = *reinterpret_cast<const uint4*>(sa + 2 * C::A_PART + off);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int off = (bcol_w + b * 16 + li) * kXBK + lh * 8;
        const uint4 bh = *reinterpret_cast<const uint4*>(sb + off);
        const uint4 bm = *reinterpret_cast<const uint4*>(sb + C::B_PART + off);
        const uint4 bl = *reinterpret_cast<const uint4*>(sb + 2 * C::B_PART + off);
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          f32x4 c = acc[a][b];
          c = mfma3(al[a], bh, c);
          c = mfma3(ah[a], bl, c);
          c = mfma3(am[a], bm, c);
          c = mfma3(am[a], bh, c);
          c = mfma3(ah[a], bm, c);
          acc[a][b] = mfma3(ah[a], bh, c);
        }
      }
      store_stage(buf ^ 1);
      __syncthreads();
    }
    // epilogue: tile (a, b) register r of lane l is (row 4 (l >> 4) + r, column l & 15)
    const int64_t row0 = tile * kXBM;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = row0 + arow_w + a * 16 + 4 * lh + r;
        if (i < M) {
          const int64_t orow = o_rows ? o_rows[i] : i;
          const float rsc = row_scale ? row_scale[i] : 1.f;
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int n = bcol_w + b * 16 + li;
            float v = acc[a][b][r] * rsc;
            if constexpr (HAS_BIAS) v += bias[n];
            if constexpr (HAS_CIN) v = fmaf(beta, cin[orow * ldc + n], v);
            if constexpr (HAS_GATE) v = gate[orow * ldg + n] > 0.f ? v : 0.f;
            if constexpr (RELU) v = v > 0.f ? v : 0.f;
            out[orow * ldo + n] = v;
          }
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b][r] = 0.f;
      }
    }
    if (!has_next) break;
    tile = next;
  }
}

template <int N, bool HAS_A2, bool RELU, bool HAS_BIAS, bool HAS_CIN, bool HAS_GATE>
hipError_t launch_x3(const float* A1, int64_t lda1, int K1, const uint16_t* B1p,
                     const float* A2, int64_t lda2, int K2, const uint16_t* B2p,
                     const int64_t* a_rows, const float* bias, const float* cin, int64_t ldc,
                     float beta, const float* gate, int64_t ldg, const int64_t* o_rows,
                     const float* rsc, float* out, int64_t ldo, int64_t M, hipStream_t st) {
  auto kern = &gemm_x3_kernel<N, HAS_A2, RELU, HAS_BIAS, HAS_CIN, HAS_GATE>;
  constexpr size_t lds = XCfg<N>::BYTES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr = true;
  }
  static int num_cus = 0;
  if (num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess || num_cus <= 0)
      num_cus = 256;
  }
  const int64_t ntiles = (M + kXBM - 1) / kXBM;
  const int64_t blocks = ntiles < num_cus ? ntiles : num_cus;
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(kXThr), lds, st, A1, lda1,
                     K1, B1p, A2, lda2, K2, B2p, a_rows, bias, cin, ldc, beta, gate, ldg,
                     o_rows, rsc, out, ldo, M);
  return hipGetLastError();
}

template <int N, bool HAS_A2, bool RELU>
hipError_t x3_flags(const float* A1, int64_t lda1, int K1, const uint16_t* B1p, const float* A2,
                    int64_t lda2, int K2, const uint16_t* B2p, const int64_t* a_rows,
                    const float* bias, const float* cin, int64_t ldc, float beta,
                    const float* gate, int64_t ldg, const int64_t* o_rows, const float* rsc,
                    float* out, int64_t ldo, int64_t M, hipStream_t st) {
#define DG_X3(HB_, HC_, HG_)                                                                   \
  return launch_x3<N, HAS_A2, RELU, HB_, HC_, HG_>(A1, lda1, K1, B1p, A2, lda2, K2, B2p,       \
                                                   a_rows, bias, cin, ldc, beta, gate, ldg,    \
                                                   o_rows, rsc, out, ldo, M, st);
  const bool hb = bias != nullptr, hc = cin != nullptr, hg = gate != nullptr;
  if (hb && !hc && !hg) { DG_X3(true, false, false) }
  if (!hb && !hc && !hg) { DG_X3(false, false, false) }
  if (!hb && hc && !hg) { DG_X3(false, true, false) }
  if (!hb && hc && hg) { DG_X3(false, true, true) }
  if (!hb && !hc && hg) { DG_X3(false, false, true) }
  if (hb && hc && !hg) { DG_X3(true, true, false) }
  if (hb && !hc && hg) { DG_X3(true, false, true) }
  DG_X3(true, true, true)
#undef DG_X3
}

template <int N>
hipError_t x3_n(const float* A1, int64_t lda1, int K1, const uint16_t* B1p, const float* A2,
                int64_t lda2, int K2, const uint16_t* B2p, const int64_t* a_rows,
                const float* bias, const float* cin, int64_t ldc, float beta, const float* gate,
                int64_t ldg, const int64_t* o_rows, const float* rsc, bool relu, float* out,
                int64_t ldo, int64_t M, hipStream_t st) {
#define DG_XN(A2_, R_)                                                                        \
  return x3_flags<N, A2_, R_>(A1, lda1, K1, B1p, A2, lda2, K2, B2p, a_rows, bias, cin, ldc,   \
                              beta, gate, ldg, o_rows, rsc, out, ldo, M, st);
  const bool two = A2 != nullptr && K2 > 0;
  if (two) {
    if (relu) { DG_XN(true, true) }
    DG_XN(true, false)
  }
  if (relu) { DG_XN(false, true) }
  DG_XN(false, false)
#undef DG_XN
}

inline bool al16x(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool gemm_x3_supported(int64_t N, int64_t K1, int64_t K2) {
  return (N == 64 || N == 128 || N == 192 || N == 256) && K1 > 0 && K1 % kXBK == 0 &&
         K2 >= 0 && K2 % kXBK == 0;
}

hipError_t gemm_x3(const float* A1, int64_t lda1, int64_t K1, const uint16_t* B1p,
                   const float* A2, int64_t lda2, int64_t K2, const uint16_t* B2p,
                   const int64_t* a_rows, const float* bias, const float* cin, int64_t ldc,
                   float beta, const float* gate, int64_t ldg, const int64_t* o_rows,
                   const float* row_scale, bool relu, float* out, int64_t ldo, int64_t M,
                   int64_t N, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!gemm_x3_supported(N, K1, A2 ? K2 : 0)) return hipErrorInvalidValue;
  if (!al16x(A1) || lda1 % 4 || !al16x(B1p)) return hipErrorInvalidValue;
  if (A2 && K2 > 0 && (!al16x(A2) || lda2 % 4 || !al16x(B2p))) return hipErrorInvalidValue;
  const int k1 = static_cast<int>(K1), k2 = A2 ? static_cast<int>(K2) : 0;
  switch (N) {
    case 256: return x3_n<256>(A1, lda1, k1, B1p, A2, lda2, k2, B2p, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    case 192: return x3_n<192>(A1, lda1, k1, B1p, A2, lda2, k2, B2p, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    case 128: return x3_n<128>(A1, lda1, k1, B1p, A2, lda2, k2, B2p, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
    default: return x3_n<64>(A1, lda1, k1, B1p, A2, lda2, k2, B2p, a_rows, bias, cin, ldc, beta, gate, ldg, o_rows, row_scale, relu, out, ldo, M, st);
  }
}

}  // namespace dgraph
