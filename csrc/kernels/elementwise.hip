// dgraph_amd — fused elementwise epilogues and reductions for gfx950 (memory-bound).
//
//  bias_relu_pack : y = relu(y + bias) in place + a 1-bit keep mask. The mask lets the
//                   owning layer drop its activation (F/8 bytes per row instead of 2F),
//                   which is what fits a 111M x 256 bf16 model in 288 GB.
//  relu_mask_bwd  : g = keep ? g : 0 in place.
//  col_sum_partial: per-block fp32 column sums of [L, F] (bias gradients; torch's dim-0
//                   reduction ran at ~1/5 of HBM bandwidth on these shapes, profiles/).
//
// Mask layout (private to these kernels): the tensor is cut into 512-element chunks; a
// wavefront owns a chunk, lane l holds elements [8l, 8l+8) as one 16-B bf16 load (the
// whole wave-instruction is 1 KiB contiguous), and the chunk's mask is 8 x 64-bit
// ballots: bit l of word j = keep(element 8l + j). Mask and data accesses are therefore
// perfectly coalesced, with no cross-lane packing beyond one ballot per element slot.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void bias_relu_pack_kernel(
    T* __restrict__ y, const float* __restrict__ bias, uint64_t* __restrict__ bits,
    int64_t numel, int F, bool relu) {
  constexpr int VEC = 8;  // elements per lane (16 B bf16, 32 B fp32)
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (numel + 511) / 512;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t ch = wave; ch < nchunks; ch += nwaves) {
    const int64_t e0 = ch * 512 + lane * VEC;
    const bool valid = e0 < numel;  // numel % 8 == 0 (host check)
    float x[VEC];
    if (valid) {
      if constexpr (sizeof(T) == 2) {
        load_vec_f32<T, 8>(y + e0, x);
      } else {
        float a[4], b[4];
        load_vec_f32<T, 4>(y + e0, a);
        load_vec_f32<T, 4>(y + e0 + 4, b);
#pragma unroll
        for (int i = 0; i < 4; ++i) { x[i] = a[i]; x[i + 4] = b[i]; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < VEC; ++i) x[i] = 0.f;
    }
    const int c0 = static_cast<int>(e0 % F);  // F % 8 == 0: one row per lane slot
    uint64_t my_word = 0;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float t = x[j] + ((bias && valid) ? bias[c0 + j] : 0.f);
      bool keep = t > 0.f;
      if (relu) t = keep ? t : 0.f;
      x[j] = t;
      const uint64_t b = __ballot(valid && keep);
      if (lane == j) my_word = b;
    }
    if (valid) {
      if constexpr (sizeof(T) == 2) {
        store_vec_f32<T, 8>(y + e0, x);
      } else {
        float a[4] = {x[0], x[1], x[2], x[3]}, b[4] = {x[4], x[5], x[6], x[7]};
        store_vec_f32<T, 4>(y + e0, a);
        store_vec_f32<T, 4>(y + e0 + 4, b);
      }
    }
    if (bits && relu && lane < VEC) bits[ch * 8 + lane] = my_word;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void relu_mask_bwd_kernel(
    T* __restrict__ g, const uint64_t* __restrict__ bits, int64_t numel) {
  constexpr int VEC = 8;
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (numel + 511) / 512;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t ch = wave; ch < nchunks; ch += nwaves) {
    const int64_t e0 = ch * 512 + lane * VEC;
    // lane j < 8 loads word j; broadcast through shuffles (64-bit: two halves)
    uint64_t w = lane < VEC ? bits[ch * 8 + lane] : 0;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const uint32_t lo = __shfl(static_cast<uint32_t>(w), j, 64);
      const uint32_t hi = __shfl(static_cast<uint32_t>(w >> 32), j, 64);
      const uint32_t bit = lane < 32 ? (lo >> lane) & 1u : (hi >> (lane - 32)) & 1u;
      m |= bit << j;
    }
    if (e0 >= numel || m == 0xFFu) continue;
    if constexpr (sizeof(T) == 2) {
      float x[8];
      load_vec_f32<T, 8>(g + e0, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = ((m >> j) & 1u) ? x[j] : 0.f;
      store_vec_f32<T, 8>(g + e0, x);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (!((m >> j) & 1u)) g[e0 + j] = 0.f;
    }
  }
}

// Column sums: block b owns rows [b*rows_per_block, ...). Thread t owns VEC consecutive
// columns of row-group t / TPR; partial sums are combined through LDS in a fixed order
// (deterministic) and written to partial[b, :].
template <typename T, int VEC>
__global__ __launch_bounds__(256) void col_sum_partial_kernel(
    const T* __restrict__ g, int64_t ld, int64_t L, int F, int64_t rows_per_block,
    float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tpr = F / VEC;           // threads per row
  const int rpi = blockDim.x / tpr;  // rows per iteration
  const int t = threadIdx.x;
  const int rg = t / tpr;
  const int cc = (t % tpr) * VEC;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < L ? r0 + rows_per_block : L;
  float acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
  if (rg < rpi) {
    for (int64_t r = r0 + rg; r < r1; r += rpi) {
      float x[VEC];
      load_vec_f32<T, VEC>(g + r * ld + cc, x);
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] += x[i];
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

}  // namespace

hipError_t bias_relu_pack(DType dt, void* y, const float* bias, uint32_t* bits, int64_t numel,
                          int F, bool relu, hipStream_t st) {
  if (numel <= 0) return hipSuccess;
  if (numel % 8 != 0 || F % 8 != 0) return hipErrorInvalidValue;
  const int64_t nchunks = (numel + 511) / 512;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nchunks + 3) / 4, 256 * 16)));
  auto* b64 = reinterpret_cast<uint64_t*>(bits);
  if (dt == DType::F32)
    hipLaunchKernelGGL(bias_relu_pack_kernel<float>, grid, block, 0, st,
                       static_cast<float*>(y), bias, b64, numel, F, relu);
  else
    hipLaunchKernelGGL(bias_relu_pack_kernel<uint16_t>, grid, block, 0, st,
                       static_cast<uint16_t*>(y), bias, b64, numel, F, relu);
  return hipGetLastError();
}

hipError_t relu_mask_bwd(DType dt, void* g, const uint32_t* bits, int64_t numel,
                         hipStream_t st) {
  if (numel <= 0) return hipSuccess;
  if (numel % 8 != 0) return hipErrorInvalidValue;
  const int64_t nchunks = (numel + 511) / 512;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nchunks + 3) / 4, 256 * 16)));
  const auto* b64 = reinterpret_cast<const uint64_t*>(bits);
  if (dt == DType::F32)
    hipLaunchKernelGGL(relu_mask_bwd_kernel<float>, grid, block, 0, st,
                       static_cast<float*>(g), b64, numel);
  else
    hipLaunchKernelGGL(relu_mask_bwd_kernel<uint16_t>, grid, block, 0, st,
                       static_cast<uint16_t*>(g), b64, numel);
  return hipGetLastError();
}

hipError_t col_sum_partial(DType dt, const void* g, int64_t ld, int64_t L, int F,
                           float* partial, int nblocks, hipStream_t st) {
  if (L <= 0 || F <= 0) return hipSuccess;
  const int vec = dt == DType::F32 ? 4 : 8;
  if (F % vec != 0 || F / vec > 256 || ld % vec != 0) return hipErrorInvalidValue;
  const int64_t rpb = (L + nblocks - 1) / nblocks;
  const int tpr = F / vec;
  const int rpi = 256 / tpr;
  const size_t lds = static_cast<size_t>(rpi) * F * sizeof(float);
  dim3 block(256), grid(nblocks);
  if (dt == DType::F32)
    hipLaunchKernelGGL((col_sum_partial_kernel<float, 4>), grid, block, lds, st,
                       static_cast<const float*>(g), ld, L, F, rpb, partial);
  else
    hipLaunchKernelGGL((col_sum_partial_kernel<uint16_t, 8>), grid, block, lds, st,
                       static_cast<const uint16_t*>(g), ld, L, F, rpb, partial);
  return hipGetLastError();
}

}  // namespace dgraph
