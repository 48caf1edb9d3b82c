// dgraph_amd — fused bias + activation for the MLP layers of GraphCast (MeshGraphMLP:
// Linear, SiLU, ..., experiments/GraphCast/layers.py:24-75) and any linear + pointwise act.
//
//   forward : y = act(z + b)                      (z: the bias-free GEMM output, kept)
//   backward: dz = dy * act'(z + b),  db = sum_rows dz    (ONE pass over dy and z)
//
// PyTorch runs the forward as an addmm with a bias epilogue plus a SiLU pass, and the
// backward as silu_backward (read dy, z; write dz) followed by a column reduction (read dz
// again) for the bias gradient; here the reduction rides the backward pass. Column sums are
// per-block partials combined through LDS in a fixed order, then summed over blocks in a
// fixed order by the caller: deterministic. Layout: thread t owns VEC consecutive columns
// of row group t / TPR (TPR = F / VEC threads per row), blocks own contiguous row ranges.
// ACT: 0 identity, 1 SiLU, 2 ReLU.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <int ACT>
__device__ __forceinline__ float act_f(float t) {
  if constexpr (ACT == 1) return t / (1.f + __expf(-t));
  if constexpr (ACT == 2) return t > 0.f ? t : 0.f;
  return t;
}

template <int ACT>
__device__ __forceinline__ float act_grad(float t) {
  if constexpr (ACT == 1) {
    const float s = 1.f / (1.f + __expf(-t));
    return s * (1.f + t * (1.f - s));
  }
  if constexpr (ACT == 2) return t > 0.f ? 1.f : 0.f;
  return 1.f;
}

template <typename T, int VEC, int ACT>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const T* __restrict__ z, int64_t ldz,
                                                           const float* __restrict__ b,
                                                           T* __restrict__ y, int64_t ldy,
                                                           int64_t M, int F) {
  const int tpr = F / VEC;
  const int rpi = blockDim.x / tpr;
  const int t = threadIdx.x;
  const int rg = t / tpr;
  if (rg >= rpi) return;
  const int cc = (t % tpr) * VEC;
  float bv[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) bv[i] = b ? b[cc + i] : 0.f;
  const int64_t step = static_cast<int64_t>(gridDim.x) * rpi;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * rpi + rg; r < M; r += step) {
    float v[VEC];
    load_vec_f32<T, VEC>(z + r * ldz + cc, v);
#pragma unroll
    for (int i = 0; i < VEC; ++i) v[i] = act_f<ACT>(v[i] + bv[i]);
    store_vec_f32<T, VEC>(y + r * ldy + cc, v);
  }
}

template <typename T, int VEC, int ACT>
__global__ __launch_bounds__(256) void bias_act_bwd_kernel(
    const T* __restrict__ dy, int64_t lddy, const T* __restrict__ z, int64_t ldz,
    const float* __restrict__ b, T* __restrict__ dz, int64_t lddz, int64_t M, int F,
    int64_t rows_per_block, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tpr = F / VEC;
  const int rpi = blockDim.x / tpr;
  const int t = threadIdx.x;
  const int rg = t / tpr;
  const int cc = (t % tpr) * VEC;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  if (rg < rpi) {
    float bv[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) bv[i] = b ? b[cc + i] : 0.f;
    for (int64_t r = r0 + rg; r < r1; r += rpi) {
      float g[VEC], v[VEC];
      load_vec_f32<T, VEC>(dy + r * lddy + cc, g);
      load_vec_f32<T, VEC>(z + r * ldz + cc, v);
#pragma unroll
      for (int i = 0; i < VEC; ++i) v[i] = g[i] * act_grad<ACT>(v[i] + bv[i]);
      store_vec_f32<T, VEC>(dz + r * lddz + cc, v);
      // the bias gradient sums the STORED (rounded) dz, as a separate reduction would
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] += Elem<T>::to_f32(Elem<T>::from_f32(v[i]));
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) smem[rg * F + cc + i] = acc[i];
  }
  __syncthreads();
  for (int c = t; c < F; c += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < rpi; ++k) s += smem[k * F + c];
    partial[static_cast<int64_t>(blockIdx.x) * F + c] = s;
  }
}

template <typename T, int VEC>
hipError_t fwd_vec(int act, const T* z, int64_t ldz, const float* b, T* y, int64_t ldy,
                   int64_t M, int F, hipStream_t st) {
  const int rpi = 256 / (F / VEC);
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((M + rpi - 1) / rpi, 256 * 8)));
  if (act == 1)
    hipLaunchKernelGGL((bias_act_fwd_kernel<T, VEC, 1>), grid, block, 0, st, z, ldz, b, y, ldy, M, F);
  else if (act == 2)
    hipLaunchKernelGGL((bias_act_fwd_kernel<T, VEC, 2>), grid, block, 0, st, z, ldz, b, y, ldy, M, F);
  else
    hipLaunchKernelGGL((bias_act_fwd_kernel<T, VEC, 0>), grid, block, 0, st, z, ldz, b, y, ldy, M, F);
  return hipGetLastError();
}

template <typename T, int VEC>
hipError_t bwd_vec(int act, const T* dy, int64_t lddy, const T* z, int64_t ldz, const float* b,
                   T* dz, int64_t lddz, int64_t M, int F, float* partial, int nblocks,
                   hipStream_t st) {
  const int rpi = 256 / (F / VEC);
  const size_t lds = static_cast<size_t>(rpi) * F * sizeof(float);
  const int64_t rpb = (M + nblocks - 1) / nblocks;
  dim3 block(256), grid(nblocks);
#define DG_BA(A_)                                                                          \
  hipLaunchKernelGGL((bias_act_bwd_kernel<T, VEC, A_>), grid, block, lds, st, dy, lddy, z, \
                     ldz, b, dz, lddz, M, F, rpb, partial);
  if (act == 1) { DG_BA(1) } else if (act == 2) { DG_BA(2) } else { DG_BA(0) }
#undef DG_BA
  return hipGetLastError();
}

inline bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

hipError_t bias_act_fwd(DType dt, int act, const void* z, int64_t ldz, const float* b, void* y,
                        int64_t ldy, int64_t M, int F, hipStream_t st) {
  if (M <= 0 || F <= 0) return hipSuccess;
  if (act < 0 || act > 2) return hipErrorInvalidValue;
  if (dt == DType::F32) {
    auto zp = static_cast<const float*>(z);
    auto yp = static_cast<float*>(y);
    if (F % 4 == 0 && ldz % 4 == 0 && ldy % 4 == 0 && F / 4 <= 256 && a16(z) && a16(y))
      return fwd_vec<float, 4>(act, zp, ldz, b, yp, ldy, M, F, st);
    if (F > 256) return hipErrorInvalidValue;
    return fwd_vec<float, 1>(act, zp, ldz, b, yp, ldy, M, F, st);
  }
  auto zp = static_cast<const uint16_t*>(z);
  auto yp = static_cast<uint16_t*>(y);
  if (F % 8 == 0 && ldz % 8 == 0 && ldy % 8 == 0 && F / 8 <= 256 && a16(z) && a16(y))
    return fwd_vec<uint16_t, 8>(act, zp, ldz, b, yp, ldy, M, F, st);
  if (F > 256) return hipErrorInvalidValue;
  return fwd_vec<uint16_t, 1>(act, zp, ldz, b, yp, ldy, M, F, st);
}

hipError_t bias_act_bwd(DType dt, int act, const void* dy, int64_t lddy, const void* z,
                        int64_t ldz, const float* b, void* dz, int64_t lddz, int64_t M, int F,
                        float* partial, int nblocks, hipStream_t st) {
  if (M <= 0 || F <= 0) return hipSuccess;
  if (act < 0 || act > 2 || nblocks <= 0) return hipErrorInvalidValue;
  if (dt == DType::F32) {
    auto g = static_cast<const float*>(dy);
    auto zp = static_cast<const float*>(z);
    auto o = static_cast<float*>(dz);
    if (F % 4 == 0 && lddy % 4 == 0 && ldz % 4 == 0 && lddz % 4 == 0 && F / 4 <= 256 &&
        a16(dy) && a16(z) && a16(dz))
      return bwd_vec<float, 4>(act, g, lddy, zp, ldz, b, o, lddz, M, F, partial, nblocks, st);
    if (F > 256) return hipErrorInvalidValue;
    return bwd_vec<float, 1>(act, g, lddy, zp, ldz, b, o, lddz, M, F, partial, nblocks, st);
  }
  auto g = static_cast<const uint16_t*>(dy);
  auto zp = static_cast<const uint16_t*>(z);
  auto o = static_cast<uint16_t*>(dz);
  if (F % 8 == 0 && lddy % 8 == 0 && ldz % 8 == 0 && lddz % 8 == 0 && F / 8 <= 256 &&
      a16(dy) && a16(z) && a16(dz))
    return bwd_vec<uint16_t, 8>(act, g, lddy, zp, ldz, b, o, lddz, M, F, partial, nblocks, st);
  if (F > 256) return hipErrorInvalidValue;
  return bwd_vec<uint16_t, 1>(act, g, lddy, zp, ldz, b, o, lddz, M, F, partial, nblocks, st);
}

}  // namespace dgraph
