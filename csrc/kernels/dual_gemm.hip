// dgraph_amd — fused tall-skinny "dual GEMM" on MFMA for the GraphSAGE layer combine.
//
//   out[M, N] = epi( A1[M, K1] @ B1[K1, N]  (+ A2[M, K2] @ B2[K2, N])  (+ bias[N])  (+ Cin) )
//   epi: optional ReLU that also writes a 1-bit keep mask, or an input keep mask (the
//        ReLU derivative of the previous layer applied to a gradient).
//
// SAGE forward  y  = relu(h Ws + (A h) Wn + b)          -> one kernel, mask written
// SAGE backward dh = mask_prev * (g Ws^T + u Wn^T)        -> one kernel, mask applied
// The library path is mm + addmm + a bias/ReLU/mask kernel: the [M, N] output crosses HBM
// five times (write, read + write, read + write); here once.
//
// Shapes: M ~ 1e8 rows (vertices), N = 32 * NT in {128, 192, 256}, K1/K2 in {128, 192,
// 256} (bf16 in, fp32 accumulate). Design (measured, benchmarks/native/):
//   * persistent blocks of 8 wave64s, one per CU; a block owns one column half of the
//     output and keeps that half of B^T resident in LDS (<= 133 KB) for the whole run, so
//     the k loop has no barrier and no B traffic (re-staging B per tile through LDS with a
//     barrier per k-stage ran at ~2.2 TB/s);
//   * a wave owns 32 rows x N/2 columns: NT/2 accumulators of v_mfma_f32_32x32x16_bf16;
//     its A fragments stream from HBM straight into VGPRs (16 B per lane per k-step) in a
//     ring PD k-chunks deep that runs across tile boundaries;
//   * the two column halves of a row tile run on blocks b and b + 8 (same XCD) so the
//     second read of an A row can hit that XCD's L2;
//   * epilogue per 32x32 tile through a private LDS tile -> 16-B row-segment stores.
// Mask layout ("tile32"): for each 32-row block rb and 32-column tile t, 16 uint64 words
// word[(rb * NT + t) * 16 + r] whose bit l is the keep bit of accumulator register r of
// lane l, i.e. of element (row 32 rb + (r & 3) + 8 (r >> 2) + 4 (l >> 5), col 32 t + (l & 31)).
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int kRowsPerBlock = 256;  // 8 waves x 32 rows (one column half per block)
constexpr int kThreads = 512;
constexpr int kBK = 32;             // k per A chunk (2 MFMA k-steps of 16)
#ifndef DG_PD
#define DG_PD 8                     // A prefetch ring depth (chunks) for long k loops
#endif

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

template <int NC>
constexpr int ring_depth() {
  // a divisor of NC (static ring slots) leaving >= 2 groups in the rolled k loop (a single
  // fully unrolled group lets the compiler hoist every LDS read and spill)
  return (NC % DG_PD == 0 && NC >= 2 * DG_PD) ? DG_PD
         : (NC % 4 == 0 && NC >= 8)           ? 4
         : (NC % 3 == 0 && NC >= 6)           ? 3
                                              : 2;
}

// Persistent blocks, one per CU. Block b owns column half h = (b / 8) % 2 of the output
// and keeps that half of B^T ([N/2][K1 + K2], 133 KB) resident in LDS for the whole run:
// the k loop has no barrier and no B traffic. The two halves of a row tile are computed by
// blocks b and b + 8, which the dispatcher places on the same XCD, so the second reader of
// an A row hits that XCD's L2. Each wave owns 32 rows x N/2 columns; the A ring runs
// straight across tile boundaries (HBM latency paid once per block).
template <int NT, int NC1, int NC2>
__global__ __launch_bounds__(kThreads, 1) void dual_gemm_kernel(
    const uint16_t* __restrict__ A1, int64_t lda1, const uint16_t* __restrict__ B1t,
    const uint16_t* __restrict__ A2, int64_t lda2, const uint16_t* __restrict__ B2t,
    const float* __restrict__ bias, const uint16_t* __restrict__ cin, int64_t ldc,
    uint16_t* __restrict__ out, int64_t ldo, uint64_t* __restrict__ mask_out,
    const uint64_t* __restrict__ mask_in, int64_t M, int relu) {
  constexpr int K1 = NC1 * kBK, K2 = NC2 * kBK;
  constexpr int KT = K1 + K2;
  constexpr int NC = NC1 + NC2;
  constexpr int PD = ring_depth<NC>();
  constexpr int NTW = NT / 2;         // 32-column tiles per wave = per block (column half)
  constexpr int NH = NTW * 32;        // columns per block
  constexpr int kBRow = KT + 8;       // staged B^T row (bf16): +16 B pad, conflict-free
  constexpr int kSB = NH * kBRow;     // resident B half
  constexpr int kEW = 40;             // epilogue tile row (32 + 8 pad)
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* const sB = smem;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int khalf = 8 * (lane >> 5);
  const int64_t ntiles = (M + kRowsPerBlock - 1) / kRowsPerBlock;
  // block -> (column half, tile stream); streams are shared by the XCD-paired blocks
  const int G = gridDim.x;            // multiple of 16
  const int b = blockIdx.x;
  const int half = (b >> 3) & 1;
  const int stream = (b & 7) | ((b >> 4) << 3);
  const int nstreams = G >> 1;
  const int col0 = half * NH;

  // ---- resident B half: rows col0 .. col0 + NH of B1t | B2t, 16-B pieces
  constexpr int PPR = KT / 8;
  for (int p = tid; p < NH * PPR; p += kThreads) {
    const int n = p / PPR, q = p % PPR;
    const int k = q * 8;
    const uint16_t* src = k < K1 ? B1t + static_cast<int64_t>(col0 + n) * K1 + k
                                 : B2t + static_cast<int64_t>(col0 + n) * K2 + (k - K1);
    *reinterpret_cast<uint4*>(&sB[n * kBRow + k]) = *reinterpret_cast<const uint4*>(src);
  }
  __syncthreads();

  int64_t tile = stream;
  if (tile >= ntiles) return;
  auto lane_row = [&](int64_t t) -> int64_t {
    const int64_t r = t * kRowsPerBlock + wave * 32 + (lane & 31);
    return r < M ? r : M - 1;  // rows past M are computed and discarded
  };
#define DG_A_SRC(pa1, pa2, c, s)                                                            \
  ((c) < NC1 ? (pa1) + (c) * kBK + 16 * (s) : (pa2) + ((c) - NC1) * kBK + 16 * (s))
  int64_t arow = lane_row(tile);
  const uint16_t* pa1 = A1 + arow * lda1 + khalf;
  const uint16_t* pa2 = NC2 ? A2 + arow * lda2 + khalf : pa1;
  uint4 a0[PD], a1[PD];
#pragma unroll
  for (int c = 0; c < PD; ++c) {
    a0[c] = *reinterpret_cast<const uint4*>(DG_A_SRC(pa1, pa2, c, 0));
    a1[c] = *reinterpret_cast<const uint4*>(DG_A_SRC(pa1, pa2, c, 1));
  }
  uint16_t* sE = smem + kSB + wave * (32 * kEW);
  const int col_l = lane & 31;
  const int rsub = 4 * (lane >> 5);
  const uint16_t* sbl = &sB[col_l * kBRow + khalf];  // this lane's B^T row base (tile 0)

  for (; tile < ntiles; tile += nstreams) {
    const int64_t next = tile + nstreams;
    const bool has_next = next < ntiles;
    const int64_t narow = has_next ? lane_row(next) : arow;
    const uint16_t* na1 = A1 + narow * lda1 + khalf;
    const uint16_t* na2 = NC2 ? A2 + narow * lda2 + khalf : na1;
    f32x16 acc[NTW];
#pragma unroll
    for (int t = 0; t < NTW; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    // k loop: a rolled loop over groups of PD chunks (bounds the compiler's hoisting of
    // LDS fragment reads, which otherwise spilled), unrolled inside so ring slots are static
#pragma unroll 1
    for (int cb = 0; cb < NC; cb += PD) {
#pragma unroll
      for (int j = 0; j < PD; ++j) {
        const int c = cb + j;
        const bf16x8 fa0 = as_bf16x8(a0[j]);
        const bf16x8 fa1 = as_bf16x8(a1[j]);
#pragma unroll
        for (int t = 0; t < NTW; ++t) {
          const uint16_t* rowp = sbl + t * 32 * kBRow + c * kBK;
          const uint4 bv0 = *reinterpret_cast<const uint4*>(rowp);
          const uint4 bv1 = *reinterpret_cast<const uint4*>(rowp + 16);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa0, as_bf16x8(bv0), acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa1, as_bf16x8(bv1), acc[t], 0, 0, 0);
        }
        // refill the consumed slot: chunk c + PD of this tile or of the next one
        const int cn = c + PD;
        const uint16_t* src = nullptr;
        if (cn < NC) {
          src = cn < NC1 ? pa1 + cn * kBK : pa2 + (cn - NC1) * kBK;
        } else if (has_next) {
          const int cm = cn - NC;
          src = cm < NC1 ? na1 + cm * kBK : na2 + (cm - NC1) * kBK;
        }
        if (src) {
          a0[j] = *reinterpret_cast<const uint4*>(src);
          a1[j] = *reinterpret_cast<const uint4*>(src + 16);
        }
      }
    }

    // ---- epilogue per 32x32 tile: registers -> (bias, cin, mask, ReLU) -> private LDS
    // tile -> 64-B row segments -> 16-B global stores (the lane owns a column of 16 rows in
    // the MFMA C layout; both 64-B halves of a 128-B line leave the same wave back to back)
    const int64_t row0 = tile * kRowsPerBlock + wave * 32;
    const int64_t rb = row0 >> 5;  // 32-row block index
#pragma unroll
    for (int u = 0; u < NTW; ++u) {
      const int t = half * NTW + u;  // global 32-column tile
      const int col = t * 32 + col_l;
      const float bv = bias ? bias[col] : 0.f;
      uint64_t keep_in = 0;
      if (mask_in && lane < 16) keep_in = mask_in[(rb * NT + t) * 16 + lane];
      uint64_t my_word = 0;
      if (cin) {
        // stage the tile's cin rows through the LDS tile with coalesced 16-B loads (per-
        // element 2-byte loads in the C layout ran this kernel 3x slower)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rr = (lane >> 2) + 16 * q;
          const int64_t row = row0 + rr;
          uint4 v = make_uint4(0, 0, 0, 0);
          if (row < M) v = *reinterpret_cast<const uint4*>(cin + row * ldc + t * 32 + (lane & 3) * 8);
          *reinterpret_cast<uint4*>(&sE[rr * kEW + (lane & 3) * 8]) = v;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = (r & 3) + 8 * (r >> 2) + rsub;
        const int64_t row = row0 + rr;
        float v = acc[u][r] + bv;
        if (cin) v += bf16_to_f32(sE[rr * kEW + col_l]);
        if (mask_in) {
          const uint64_t w =
              (static_cast<uint64_t>(__shfl(static_cast<int>(keep_in), r, 64)) & 0xffffffffull) |
              (static_cast<uint64_t>(__shfl(static_cast<int>(keep_in >> 32), r, 64)) << 32);
          if (!((w >> lane) & 1ull)) v = 0.f;
        }
        if (relu) {
          const bool k = v > 0.f && row < M;
          const uint64_t bal = __ballot(k);
          if (lane == r) my_word = bal;
          v = k ? v : 0.f;
        }
        sE[rr * kEW + col_l] = f32_to_bf16(v);
      }
      if (relu && mask_out && lane < 16) mask_out[(rb * NT + t) * 16 + lane] = my_word;
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS tile is written
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int rr = (lane >> 2) + 16 * q;  // 4 lanes x 16 B per 64-B row segment
        const int64_t row = row0 + rr;
        if (row < M) {
          const uint4 v = *reinterpret_cast<const uint4*>(&sE[rr * kEW + (lane & 3) * 8]);
          *reinterpret_cast<uint4*>(out + row * ldo + t * 32 + (lane & 3) * 8) = v;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();  // read back before the next tile overwrites it
    }
    arow = narow;
    pa1 = na1;
    pa2 = na2;
  }
#undef DG_A_SRC
}

template <int NT, int NC1, int NC2>
constexpr size_t lds_bytes() {
  return (static_cast<size_t>(NT / 2) * 32 * ((NC1 + NC2) * kBK + 8) +
          static_cast<size_t>(kThreads / 64) * 32 * 40) * sizeof(uint16_t);
}

template <int NT, int NC1, int NC2>
hipError_t launch(const void* A1, int64_t lda1, const void* B1t, const void* A2, int64_t lda2,
                  const void* B2t, const float* bias, const void* cin, int64_t ldc, void* out,
                  int64_t ldo, uint64_t* mask_out, const uint64_t* mask_in, int64_t M,
                  bool relu, hipStream_t st) {
  const int64_t tiles = (M + kRowsPerBlock - 1) / kRowsPerBlock;
  static int num_cus = 0;
  if (num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess
        || num_cus <= 0)
      num_cus = 256;
  }
  // persistent: one block per CU, a multiple of 16 (XCD pairs of column halves); at most
  // two blocks per row tile
  int64_t blocks = (num_cus / 16) * 16;
  const int64_t need = (tiles * 2 + 15) / 16 * 16;
  if (blocks > need) blocks = need;
  if (blocks < 16) blocks = 16;
  constexpr size_t lds = lds_bytes<NT, NC1, NC2>();
  static_assert(lds <= 160 * 1024, "resident B half must fit in LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&dual_gemm_kernel<NT, NC1, NC2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr_set = true;
  }
  hipLaunchKernelGGL((dual_gemm_kernel<NT, NC1, NC2>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kThreads), lds, st, static_cast<const uint16_t*>(A1), lda1,
                     static_cast<const uint16_t*>(B1t), static_cast<const uint16_t*>(A2), lda2,
                     static_cast<const uint16_t*>(B2t), bias,
                     static_cast<const uint16_t*>(cin), ldc, static_cast<uint16_t*>(out), ldo,
                     mask_out, mask_in, M, relu ? 1 : 0);
  return hipGetLastError();
}

template <int NT, int NC1>
hipError_t by_nc2(int nc2, const void* A1, int64_t lda1, const void* B1t, const void* A2,
                  int64_t lda2, const void* B2t, const float* bias, const void* cin,
                  int64_t ldc, void* out, int64_t ldo, uint64_t* mo, const uint64_t* mi,
                  int64_t M, bool relu, hipStream_t st) {
  switch (nc2) {
    case 0: return launch<NT, NC1, 0>(A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 4: return launch<NT, NC1, 4>(A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 6: return launch<NT, NC1, 6>(A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 8: return launch<NT, NC1, 8>(A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    default: return hipErrorInvalidValue;
  }
}

template <int NT>
hipError_t by_nc1(int nc1, int nc2, const void* A1, int64_t lda1, const void* B1t,
                  const void* A2, int64_t lda2, const void* B2t, const float* bias,
                  const void* cin, int64_t ldc, void* out, int64_t ldo, uint64_t* mo,
                  const uint64_t* mi, int64_t M, bool relu, hipStream_t st) {
  switch (nc1) {
    case 4: return by_nc2<NT, 4>(nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 6: return by_nc2<NT, 6>(nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    case 8: return by_nc2<NT, 8>(nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mo, mi, M, relu, st);
    default: return hipErrorInvalidValue;
  }
}

int g_dual_gemm_variant = 2;

}  // namespace

void set_dual_gemm_variant(int variant) {
  g_dual_gemm_variant = (variant == 1 || variant == 2) ? variant : 2;
}
int get_dual_gemm_variant() { return g_dual_gemm_variant; }

bool dual_gemm_supported(int64_t N, int64_t K1, int64_t K2) {
  auto okk = [](int64_t k) { return k == 128 || k == 192 || k == 256; };
  return (N == 128 || N == 192 || N == 256) && okk(K1) && (K2 == 0 || okk(K2));
}

hipError_t dual_gemm(const void* A1, int64_t lda1, const void* B1t, int64_t K1, const void* A2,
                     int64_t lda2, const void* B2t, int64_t K2, const float* bias,
                     const void* cin, int64_t ldc, void* out, int64_t ldo, int64_t M, int64_t N,
                     uint64_t* mask_out, const uint64_t* mask_in, bool relu, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if (!dual_gemm_supported(N, K1, K2)) return hipErrorInvalidValue;
  if (g_dual_gemm_variant == 2 && dual_gemm_bs_supported(N, K1, K2))
    return dual_gemm_bs(A1, lda1, B1t, K1, A2, lda2, B2t, K2, bias, cin, ldc, out, ldo, M, N,
                        mask_out, mask_in, relu, st);
  const int nc1 = static_cast<int>(K1 / kBK), nc2 = static_cast<int>(K2 / kBK);
  switch (N) {
    case 128: return by_nc1<4>(nc1, nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
    case 192: return by_nc1<6>(nc1, nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
    default: return by_nc1<8>(nc1, nc2, A1, lda1, B1t, A2, lda2, B2t, bias, cin, ldc, out, ldo, mask_out, mask_in, M, relu, st);
  }
}

}  // namespace dgraph
