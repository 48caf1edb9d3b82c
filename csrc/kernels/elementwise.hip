// dgraph_amd — fused elementwise epilogues for gfx950 (memory-bound, 16-B vectorised).
//
//  bias_relu_pack : y = relu(y + bias) in place, and a 1-bit-per-element keep mask
//                   (bits[i/32] bit i%32). The mask (F/8 bytes per row instead of 2F)
//                   is all that a ReLU backward needs, which lets the owning layer free
//                   its activation early (288 GB budget at 111M x 256 activations).
//  relu_mask_bwd  : g = bit ? g : 0 in place.
// Each lane owns 32 consecutive elements (one mask word): 4 x 16-B loads for bf16.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void bias_relu_pack_kernel(
    T* __restrict__ y, const float* __restrict__ bias, uint32_t* __restrict__ bits,
    int64_t nwords, int F, bool relu) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NV = 32 / VEC;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; w < nwords;
       w += stride) {
    T* p = y + w * 32;
    const int c0 = static_cast<int>((w * 32) % F);
    uint32_t m = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float x[VEC];
      load_vec_f32<T, VEC>(p + v * VEC, x);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        const int e = v * VEC + i;
        float t = x[i] + (bias ? bias[c0 + e] : 0.f);
        if (relu) {
          const bool keep = t > 0.f;
          m |= (keep ? 1u : 0u) << e;
          t = keep ? t : 0.f;
        }
        x[i] = t;
      }
      store_vec_f32<T, VEC>(p + v * VEC, x);
    }
    if (bits) bits[w] = m;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void relu_mask_bwd_kernel(T* __restrict__ g,
                                                            const uint32_t* __restrict__ bits,
                                                            int64_t nwords) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NV = 32 / VEC;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; w < nwords;
       w += stride) {
    const uint32_t m = bits[w];
    T* p = g + w * 32;
    if (m == 0xFFFFFFFFu) continue;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      float x[VEC];
      load_vec_f32<T, VEC>(p + v * VEC, x);
#pragma unroll
      for (int i = 0; i < VEC; ++i) x[i] = ((m >> (v * VEC + i)) & 1u) ? x[i] : 0.f;
      store_vec_f32<T, VEC>(p + v * VEC, x);
    }
  }
}

}  // namespace

hipError_t bias_relu_pack(DType dt, void* y, const float* bias, uint32_t* bits, int64_t numel,
                          int F, bool relu, hipStream_t st) {
  if (numel <= 0) return hipSuccess;
  if (numel % 32 != 0 || F % 32 != 0) return hipErrorInvalidValue;
  const int64_t nwords = numel / 32;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nwords + 255) / 256, 256 * 16)));
  if (dt == DType::F32)
    hipLaunchKernelGGL(bias_relu_pack_kernel<float>, grid, block, 0, st,
                       static_cast<float*>(y), bias, bits, nwords, F, relu);
  else
    hipLaunchKernelGGL(bias_relu_pack_kernel<uint16_t>, grid, block, 0, st,
                       static_cast<uint16_t*>(y), bias, bits, nwords, F, relu);
  return hipGetLastError();
}

hipError_t relu_mask_bwd(DType dt, void* g, const uint32_t* bits, int64_t numel,
                         hipStream_t st) {
  if (numel <= 0) return hipSuccess;
  if (numel % 32 != 0) return hipErrorInvalidValue;
  const int64_t nwords = numel / 32;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nwords + 255) / 256, 256 * 16)));
  if (dt == DType::F32)
    hipLaunchKernelGGL(relu_mask_bwd_kernel<float>, grid, block, 0, st,
                       static_cast<float*>(g), bits, nwords);
  else
    hipLaunchKernelGGL(relu_mask_bwd_kernel<uint16_t>, grid, block, 0, st,
                       static_cast<uint16_t*>(g), bits, nwords);
  return hipGetLastError();
}

}  // namespace dgraph
