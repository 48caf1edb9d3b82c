// dgraph_amd — fp32 MFMA weight gradient for tall operands (gfx950, v_mfma_f32_16x16x4_f32).
//
//   C[K1 + K2, N] = [A1[a1(m), 0:K1] | A2[m, 0:K2]]^T  @  G[m, 0:N]     summed over m < M
//
// The GraphSAGE weight gradients x^T g and agg^T g reduce over 10^7 - 10^8 vertex rows
// into a 256 x 256 output: a library GEMM gets only (K/tile) x (N/tile) output tiles, i.e.
// a handful of workgroups for 256 CUs. Here the REDUCTION is split into U units of
// contiguous rows; a persistent grid of at most one block per CU pulls units from a work
// counter (a block whose CU is held by another stream's kernel — RCCL's during a halo
// exchange — starts late and finds the units taken), accumulates the whole [K, N] product of
// a unit in MFMA accumulators (8 waves x TM x TN 16x16 tiles) and writes (or adds to) the
// UNIT's fp32 partial slab partials[u]. wgrad_f32_reduce sums the slabs in unit order —
// deterministic whichever block ran a unit, for a fixed sequence of calls, which can
// accumulate over row chunks of one step before the reduce.
// Data flow per 32-row stage: A and G rows -> registers (issued one stage ahead) -> padded
// LDS [32][K+4] / [32][N+4]; MFMA step j uses rows 8h + j (lane group h = lane >> 4) of both
// (the k-slot permutation of gemm_f32.hip, here over the reduced row index). Stage rows with
// bit 3 set sit 16 floats further (srow): the two 16-lane halves of every ds_read_b32 read
// rows 8 apart, which a (K+4)-float pitch alone maps to the same banks (2-way conflict).
#include "../common.h"
#include "kernels.h"
#include "lds_dma.h"

namespace dgraph {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 32;  // rows per stage
constexpr int kThr = 512;

template <int K, int N>
struct WCfg {
  static constexpr int NTK = K / 16, NTN = N / 16;
  static constexpr bool TWO = (NTN % 2 == 0) && (NTK % 4 == 0);
  static constexpr int WN = TWO ? 2 : 1;
  static constexpr int WM = TWO ? 4 : 8;
  static constexpr int TM = NTK / WM, TN = NTN / WN;
  static constexpr int AP = K + 16, GP = N + 16;  // LDS row pitches (floats; srow shift)
  static constexpr int A_FL = kRows * AP, G_FL = kRows * GP;
  static constexpr int STAGE = A_FL + G_FL;
  static constexpr size_t BYTES = 2 * STAGE * sizeof(float);
  static constexpr int A_V4 = (kRows * K / 4 + kThr - 1) / kThr;
  static constexpr int G_V4 = (kRows * N / 4 + kThr - 1) / kThr;
  static_assert(TM >= 1 && TM * WM == NTK && TN * WN == NTN, "wgrad tiling");
};

template <int P>
__device__ __forceinline__ int srow(int r) { return r * P + ((r >> 3) & 1) * 16; }

template <int K, int N>
__device__ __forceinline__ void wgrad_f32_body(
    const float* __restrict__ A1, int64_t lda1, int K1, const float* __restrict__ A2,
    int64_t lda2, const int64_t* __restrict__ a1_rows, const float* __restrict__ G,
    int64_t ldg, int64_t M, int64_t rows_per_unit, int units, float* __restrict__ partials,
    int fresh_from, int* __restrict__ unit_ctr, float* __restrict__ col_partials) {
  using C = WCfg<K, N>;
  constexpr int TM = C::TM, TN = C::TN, WN = C::WN;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ int s_unit;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int li = lane & 15;
  const int lh = lane >> 4;
  // unit_ctr == nullptr: static schedule (block b runs units b, b + grid, ...)
  for (int it = 0;; ++it) {
  int unit;
  if (unit_ctr != nullptr) {
    __syncthreads();  // the previous unit's LDS reads and s_unit reads are done
    if (tid == 0) s_unit = atomicAdd(unit_ctr, 1);
    __syncthreads();
    unit = s_unit;
  } else {
    if (it > 0) __syncthreads();  // the previous unit's LDS reads are done
    unit = static_cast<int>(blockIdx.x) + it * static_cast<int>(gridDim.x);
  }
  if (unit >= units) return;  // block-uniform
  const int64_t m_begin = static_cast<int64_t>(unit) * rows_per_unit;
  int64_t m_end = m_begin + rows_per_unit;
  m_end = m_end < M ? m_end : M;
  const int64_t nst = m_end > m_begin ? (m_end - m_begin + kRows - 1) / kRows : 0;

  f32x4 ra[C::A_V4];
  f32x4 rg[C::G_V4];
  int64_t ix[C::A_V4];  // A rows (through a1_rows for A1 slots) of the next stage to load
  // slot u of this thread: stage row rr(u), column c(u) (surplus slots clamped to the
  // stage's last float4: every load and store is unconditional — a load under a branch
  // gets sunk next to its use by the compiler, exposing its latency)
  auto slot = [&](int u, int W) {
    int q = tid + kThr * u;
    return q < kRows * W / 4 ? q : kRows * W / 4 - 1;
  };
  auto row_of = [&](int64_t s, int rr) {
    const int64_t m = m_begin + s * kRows + rr;
    return m < m_end ? m : m_begin;  // a valid row (its G row is zeroed at the store)
  };
  // the indices of stage s's A1 rows: loaded one stage before their data
  auto load_idx = [&](int64_t s) {
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = slot(u, K);
      const int64_t mm = row_of(s, q / (K / 4));
      ix[u] = (a1_rows && (q % (K / 4)) * 4 < K1) ? a1_rows[mm] : mm;
    }
  };
  auto load_data = [&](int64_t s) {
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = slot(u, K);
      const int c = (q % (K / 4)) * 4;
      const bool first = c < K1;
      const float* base = first ? A1 : A2;
      const int64_t ld = first ? lda1 : lda2;
      ra[u] = *reinterpret_cast<const f32x4*>(base + ix[u] * ld + (first ? c : c - K1));
    }
#pragma unroll
    for (int u = 0; u < C::G_V4; ++u) {
      const int q = slot(u, N);
      rg[u] = *reinterpret_cast<const f32x4*>(G + row_of(s, q / (N / 4)) * ldg +
                                              (q % (N / 4)) * 4);
    }
  };
  auto store_stage = [&](int buf, int64_t s) {
    float* sa = lds + buf * C::STAGE;
    float* sg = sa + C::A_FL;
#pragma unroll
    for (int u = 0; u < C::A_V4; ++u) {
      const int q = slot(u, K);  // surplus: same value, same place
      const int rr = q / (K / 4), c = (q % (K / 4)) * 4;
      *reinterpret_cast<f32x4*>(sa + srow<C::AP>(rr) + c) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < C::G_V4; ++u) {
      const int q = slot(u, N);
      const int rr = q / (N / 4), c = (q % (N / 4)) * 4;
      // rows past the block's range contribute zero (zeroing one operand suffices)
      const bool ok = m_begin + s * kRows + rr < m_end;
      *reinterpret_cast<f32x4*>(sg + srow<C::GP>(rr) + c) =
          ok ? rg[u] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kw = wm * TM * 16, nw = wn * TN * 16;
  float csum = 0.f;
  if (nst > 0) {
    load_idx(0);
    load_data(0);
    store_stage(0, 0);
    load_idx(nst > 1 ? 1 : 0);
    __syncthreads();
    for (int64_t s = 0; s < nst; ++s) {
      const int buf = static_cast<int>(s & 1);
      // unconditional (the last stage re-reads itself into a buffer never read again);
      // then the indices of the stage after
      const int64_t sn = s + 1 < nst ? s + 1 : s;
      load_data(sn);
      load_idx(s + 2 < nst ? s + 2 : sn);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of this stage's MFMAs
      const float* sa = lds + buf * C::STAGE;
      const float* sg = sa + C::A_FL;
      // operand fragments double-buffered across MFMA steps (reads of step j+1 are in
      // flight during step j's MFMAs); rows 8 lh + j, j < 8, share srow's shift
      if (col_partials != nullptr && tid < N) {
        // the bias gradient's column sums ride along: column tid of this stage's G rows,
        // added in row order (rows past the unit were stored as zeros)
#pragma unroll 8
        for (int rr = 0; rr < kRows; ++rr) csum += sg[srow<C::GP>(rr) + tid];
      }
      const float* saw = sa + srow<C::AP>(8 * lh) + kw + li;
      const float* sgw = sg + srow<C::GP>(8 * lh) + nw + li;
      float av[2][TM], gv[2][TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) av[0][a] = saw[a * 16];
#pragma unroll
      for (int b = 0; b < TN; ++b) gv[0][b] = sgw[b * 16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (j + 1 < 8) {
#pragma unroll
          for (int a = 0; a < TM; ++a) av[(j + 1) & 1][a] = saw[(j + 1) * C::AP + a * 16];
#pragma unroll
          for (int b = 0; b < TN; ++b) gv[(j + 1) & 1][b] = sgw[(j + 1) * C::GP + b * 16];
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j & 1][a], gv[j & 1][b],
                                                             acc[a][b], 0, 0, 0);
      }
      store_stage(buf ^ 1, sn);
      __syncthreads();
    }
  }
  // register r of tile (a, b), lane l: C[kw + 16a + 4(l>>4) + r][nw + 16b + (l&15)]
  float* slab = partials + static_cast<int64_t>(unit) * K * N;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = kw + a * 16 + 4 * lh + r;
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        float* p = slab + k * N + nw + b * 16 + li;
        // slabs below fresh_from hold this step's earlier calls: accumulate; the rest are
        // written fresh (a call may use fewer blocks than an earlier one)
        *p = unit < fresh_from ? *p + acc[a][b][r] : acc[a][b][r];
      }
    }
  if (col_partials != nullptr && tid < N) {
    float* p = col_partials + static_cast<int64_t>(unit) * N + tid;
    *p = unit < fresh_from ? *p + csum : csum;
  }
  }  // units
}

template <int K, int N>
__global__ __launch_bounds__(kThr, 1) void wgrad_f32_kernel(
    const float* __restrict__ A1, int64_t lda1, int K1, const float* __restrict__ A2,
    int64_t lda2, const int64_t* __restrict__ a1_rows, const float* __restrict__ G,
    int64_t ldg, int64_t M, int64_t rows_per_unit, int units, float* __restrict__ partials,
    int fresh_from, int* __restrict__ unit_ctr, float* __restrict__ col_partials) {
  wgrad_f32_body<K, N>(A1, lda1, K1, A2, lda2, a1_rows, G, ldg, M, rows_per_unit, units,
                       partials, fresh_from, unit_ctr, col_partials);
  work_counter_release(unit_ctr);
}

// out[i] = sum of the P slabs' element i, added in slab order (deterministic). Each lane
// keeps 16 slab loads in flight ahead of the (ordered) adds: a 128 x 128 product over 256
// slabs is only 64 blocks, and one dependent load per add made the reduce latency-bound
// (63 us per call, a third of a GraphCast weight gradient: profiles/r04).
__global__ __launch_bounds__(64) void wgrad_reduce_kernel(const float* __restrict__ partials,
                                                          int P, int64_t KN,
                                                          float* __restrict__ out) {
  constexpr int D = 16;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= KN) return;
  const float* p = partials + i;
  float s = 0.f;
  int b = 0;
  for (; b + D <= P; b += D) {
    float v[D];
#pragma unroll
    for (int j = 0; j < D; ++j) v[j] = p[static_cast<int64_t>(b + j) * KN];
#pragma unroll
    for (int j = 0; j < D; ++j) s += v[j];
  }
  for (; b < P; ++b) s += p[static_cast<int64_t>(b) * KN];
  out[i] = s;
}

template <int K, int N>
hipError_t launch_wgrad(const float* A1, int64_t lda1, int K1, const float* A2, int64_t lda2,
                        const int64_t* a1_rows, const float* G, int64_t ldg, int64_t M,
                        float* partials, int P, int fresh_from, float* col_partials,
                        hipStream_t st) {
  using C = WCfg<K, N>;
  auto kern = &wgrad_f32_kernel<K, N>;
  static_assert(C::BYTES <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              static_cast<int>(C::BYTES));
    attr = true;
  }
  // P units (slabs) of whole 32-row stages, run by at most one block per CU
  int64_t rpu = (M + P - 1) / P;
  rpu = (rpu + kRows - 1) / kRows * kRows;
  static int num_cus = 0;
  if (num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess || num_cus <= 0)
      num_cus = 256;
  }
  const int blocks = P < num_cus ? P : num_cus;
  int* ctr = nullptr;
  if (g_f32_dynamic) {
    // no free slot (more than the captured-launch budget recorded into graphs, or more
    // streams than slots): the static tile schedule of the same kernel (ctr == nullptr),
    // identical results, instead of failing the launch
    ctr = work_counter(st);
  }
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(kThr), C::BYTES, st, A1,
                     lda1, K1, A2, lda2, a1_rows, G, ldg, M, rpu, P, partials, fresh_from, ctr,
                     col_partials);
  return hipGetLastError();
}

inline bool al16w(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool wgrad_f32_supported(int64_t K, int64_t N) {
  return (K == 128 || K == 256) && (N == 128 || N == 176 || N == 192 || N == 256);
}

hipError_t wgrad_f32(const float* A1, int64_t lda1, int64_t K1, const float* A2, int64_t lda2,
                     int64_t K2, const int64_t* a1_rows, const float* G, int64_t ldg,
                     int64_t M, int64_t N, float* partials, int P, int fresh_from,
                     float* col_partials, hipStream_t st) {
  const int64_t K = K1 + (A2 ? K2 : 0);
  if (!wgrad_f32_supported(K, N) || P <= 0) return hipErrorInvalidValue;
  if (K1 % 4 || !al16w(A1) || lda1 % 4 || !al16w(G) || ldg % 4) return hipErrorInvalidValue;
  if (A2 && K2 > 0 && (!al16w(A2) || lda2 % 4)) return hipErrorInvalidValue;
  if (M < 0) return hipErrorInvalidValue;
  const int k1 = static_cast<int>(K1);
#define DG_WG(K_, N_)                                                                      \
  if (K == K_ && N == N_)                                                                  \
    return launch_wgrad<K_, N_>(A1, lda1, k1, A2, lda2, a1_rows, G, ldg, M, partials, P,  \
                                fresh_from, col_partials, st);
  DG_WG(256, 256) DG_WG(256, 176) DG_WG(256, 192) DG_WG(256, 128)
  DG_WG(128, 256) DG_WG(128, 176) DG_WG(128, 192) DG_WG(128, 128)
#undef DG_WG
  return hipErrorInvalidValue;
}

hipError_t wgrad_f32_reduce(const float* partials, int P, int64_t KN, float* out,
                            hipStream_t st) {
  if (KN <= 0) return hipSuccess;
  const int64_t blocks = (KN + 63) / 64;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>(blocks)), dim3(64), 0, st,
                     partials, P, KN, out);
  return hipGetLastError();
}

}  // namespace dgraph
