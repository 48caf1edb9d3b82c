// dgraph_amd — indexed row movement for gfx950 (K-new-1; replaces K4/K5/K7/K8).
//
// The reference's Optimized_Masked_Scatter_Gather_Kernel (local_data_kernels.cuh:353-406)
// broadcast one row's indices with a 32-lane __shfl_sync; on a 64-lane wavefront that
// packs two rows into one wave and hands lanes 32-63 the wrong indices. Here a row is
// owned by an explicit lane group of LPR lanes (LPR divides 64), G = 64/LPR rows per
// wave per step, each lane moving up to 16 B per access. The reference's ReLU baked
// into its plain scatter (K5, :247) is not reproduced.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

// U rows per lane group in flight: all U index pairs, then all U row loads, then the
// stores. One row per iteration left each wave with a single index->load->store chain
// (~2 latencies per 4 rows): the halo pack of the streamed exchange (10^8 rows x 64
// columns) ran at ~2 TB/s, bound by that chain, not by HBM.
template <typename T, typename IdxT, int VEC, int LPR, bool ACC, int U>
__global__ __launch_bounds__(256) void copy_rows_kernel(
    const T* __restrict__ x, int64_t ldx, const IdxT* __restrict__ src_idx,
    const IdxT* __restrict__ dst_idx, T* __restrict__ out, int64_t ldo, int64_t n, int F) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t base = wave * G * U; base < n; base += nwaves * G * U) {
    int64_t s[U], d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + u * G + g;
      const bool in = i < n;
      s[u] = !in ? -1 : src_idx ? static_cast<int64_t>(src_idx[i]) : i;
      d[u] = !in ? -1 : dst_idx ? static_cast<int64_t>(dst_idx[i]) : i;
    }
    for (int f = l * VEC; f < F; f += LPR * VEC) {
      float v[U][VEC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (d[u] >= 0 && s[u] >= 0) {
          load_vec_f32<T, VEC>(x + s[u] * ldx + f, v[u]);
        } else {
#pragma unroll
          for (int k = 0; k < VEC; ++k) v[u][k] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (d[u] < 0) continue;
        T* o = out + d[u] * ldo + f;
        if constexpr (ACC) {
          // fp32 output only (checked on the host): global_atomic_add_f32, no CAS loop.
#pragma unroll
          for (int k = 0; k < VEC; ++k) unsafeAtomicAdd(reinterpret_cast<float*>(o) + k, v[u][k]);
        } else {
          store_vec_f32<T, VEC>(o, v[u]);
        }
      }
    }
  }
}

template <typename T, int VEC, int LPR>
__global__ __launch_bounds__(256) void masked_gather_kernel(
    const T* __restrict__ x, int64_t ldx, const int64_t* __restrict__ idx,
    const int64_t* __restrict__ mask, int64_t value, T* __restrict__ out, int64_t ldo,
    int64_t n, int F) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t base = wave * G; base < n; base += nwaves * G) {
    const int64_t i = base + g;
    if (i >= n || mask[i] != value) continue;
    const int64_t s = idx[i];
    for (int f = l * VEC; f < F; f += LPR * VEC) {
      float v[VEC];
      load_vec_f32<T, VEC>(x + s * ldx + f, v);
      store_vec_f32<T, VEC>(out + i * ldo + f, v);
    }
  }
}

inline bool aligned(const void* p, int bytes) {
  return (reinterpret_cast<uintptr_t>(p) % bytes) == 0;
}

template <int VEC>
inline int pick_lpr(int F) {
  const int lanes = (F + VEC - 1) / VEC;
  if (lanes <= 4) return 4;
  if (lanes <= 8) return 8;
  if (lanes <= 16) return 16;
  if (lanes <= 32) return 32;
  return 64;
}

template <typename T, typename IdxT, int VEC, bool ACC>
hipError_t copy_launch(const T* x, int64_t ldx, const IdxT* si, const IdxT* di, T* out,
                       int64_t ldo, int64_t n, int F, hipStream_t st) {
  const int lpr = pick_lpr<VEC>(F);
  constexpr int U = 4;
  const int64_t rows_per_block = 4 * (kWave / lpr) * U;
  dim3 grid(static_cast<unsigned>(cap_blocks((n + rows_per_block - 1) / rows_per_block, 256 * 32)));
  dim3 block(256);
  switch (lpr) {
#define DG_CASE(L)                                                                           \
  case L:                                                                                    \
    hipLaunchKernelGGL((copy_rows_kernel<T, IdxT, VEC, L, ACC, U>), grid, block, 0, st, x, ldx, \
                       si, di, out, ldo, n, F);                                              \
    break;
    DG_CASE(4) DG_CASE(8) DG_CASE(16) DG_CASE(32) DG_CASE(64)
#undef DG_CASE
  }
  return hipGetLastError();
}

template <typename T, typename IdxT>
hipError_t copy_dispatch(const T* x, int64_t ldx, const IdxT* si, const IdxT* di, T* out,
                         int64_t ldo, int64_t n, int F, bool acc, hipStream_t st) {
  constexpr int kMaxVec = 16 / sizeof(T);
  auto ok = [&](int v) {
    return F % v == 0 && ldx % v == 0 && ldo % v == 0 && aligned(x, v * sizeof(T)) &&
           aligned(out, v * sizeof(T));
  };
  if (acc) {
    if constexpr (sizeof(T) == 4) {
      if (ok(4)) return copy_launch<T, IdxT, 4, true>(x, ldx, si, di, out, ldo, n, F, st);
      return copy_launch<T, IdxT, 1, true>(x, ldx, si, di, out, ldo, n, F, st);
    } else {
      return hipErrorInvalidValue;
    }
  }
  if (ok(kMaxVec)) return copy_launch<T, IdxT, kMaxVec, false>(x, ldx, si, di, out, ldo, n, F, st);
  if (ok(2)) return copy_launch<T, IdxT, 2, false>(x, ldx, si, di, out, ldo, n, F, st);
  return copy_launch<T, IdxT, 1, false>(x, ldx, si, di, out, ldo, n, F, st);
}

}  // namespace

hipError_t copy_rows(DType dt, IType it, const void* x, int64_t ldx, const void* src_idx,
                     const void* dst_idx, void* out, int64_t ldo, int64_t n, int F,
                     bool accumulate, hipStream_t stream) {
  if (n <= 0 || F <= 0) return hipSuccess;
#define DG_ARGS(T, I)                                                                     \
  static_cast<const T*>(x), ldx, static_cast<const I*>(src_idx),                          \
      static_cast<const I*>(dst_idx), static_cast<T*>(out), ldo, n, F, accumulate, stream
  if (dt == DType::F32) {
    if (it == IType::I32) return copy_dispatch<float, int32_t>(DG_ARGS(float, int32_t));
    return copy_dispatch<float, int64_t>(DG_ARGS(float, int64_t));
  }
  if (it == IType::I32) return copy_dispatch<uint16_t, int32_t>(DG_ARGS(uint16_t, int32_t));
  return copy_dispatch<uint16_t, int64_t>(DG_ARGS(uint16_t, int64_t));
#undef DG_ARGS
}

hipError_t masked_gather_rows(DType dt, const void* x, int64_t ldx, const int64_t* idx,
                              const int64_t* mask, int64_t value, void* out, int64_t ldo,
                              int64_t n, int F, hipStream_t st) {
  if (n <= 0 || F <= 0) return hipSuccess;
  dim3 block(256);
  dim3 grid(static_cast<unsigned>(cap_blocks((n + 3) / 4, 256 * 32)));
  // Row-per-16-lanes is enough for the legacy masked paths (small F in practice).
  if (dt == DType::F32) {
    hipLaunchKernelGGL((masked_gather_kernel<float, 1, 16>), grid, block, 0, st,
                       static_cast<const float*>(x), ldx, idx, mask, value,
                       static_cast<float*>(out), ldo, n, F);
  } else {
    hipLaunchKernelGGL((masked_gather_kernel<uint16_t, 1, 16>), grid, block, 0, st,
                       static_cast<const uint16_t*>(x), ldx, idx, mask, value,
                       static_cast<uint16_t*>(out), ldo, n, F);
  }
  return hipGetLastError();
}

}  // namespace dgraph
