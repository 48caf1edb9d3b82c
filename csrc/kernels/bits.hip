// dgraph_amd — 1-bit ReLU keep masks of selected rows (gfx950).
//
// The memory-lean fp32 executor (models/sage_fused.py) frees a hidden activation right after
// the forward, but the backward needs its ReLU derivative on the gradient-support rows. It
// keeps exactly that: one bit per element of the selected rows (32 x smaller than the fp32
// rows; ~1 GB for 3.3e7 x 256 at the papers100M shape).
//   row_keep_bits:   bits[i][w] bit j = (h[rows[i]][32 w + j] > 0)
//   apply_keep_bits: g[i][f] = bit(i, f) ? g[i][f] : 0   (in place)
// One thread per 32-column word; 8 x 16-B loads per thread.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

__global__ __launch_bounds__(256) void row_keep_bits_kernel(const float* __restrict__ h,
                                                            int64_t ldh,
                                                            const int64_t* __restrict__ rows,
                                                            int64_t n, int words,
                                                            uint32_t* __restrict__ bits) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n * words) return;
  const int64_t i = t / words;
  const int w = static_cast<int>(t % words);
  const int64_t r = rows ? rows[i] : i;
  const float4* p = reinterpret_cast<const float4*>(h + r * ldh + 32 * w);
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 v = p[q];
    m |= (v.x > 0.f ? 1u : 0u) << (4 * q);
    m |= (v.y > 0.f ? 1u : 0u) << (4 * q + 1);
    m |= (v.z > 0.f ? 1u : 0u) << (4 * q + 2);
    m |= (v.w > 0.f ? 1u : 0u) << (4 * q + 3);
  }
  bits[t] = m;
}

__global__ __launch_bounds__(256) void apply_keep_bits_kernel(float* __restrict__ g,
                                                              int64_t ldg,
                                                              const uint32_t* __restrict__ bits,
                                                              int64_t n, int words) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n * words) return;
  const int64_t i = t / words;
  const int w = static_cast<int>(t % words);
  const uint32_t m = bits[t];
  float4* p = reinterpret_cast<float4*>(g + i * ldg + 32 * w);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float4 v = p[q];
    v.x = (m >> (4 * q)) & 1u ? v.x : 0.f;
    v.y = (m >> (4 * q + 1)) & 1u ? v.y : 0.f;
    v.z = (m >> (4 * q + 2)) & 1u ? v.z : 0.f;
    v.w = (m >> (4 * q + 3)) & 1u ? v.w : 0.f;
    p[q] = v;
  }
}

}  // namespace

hipError_t row_keep_bits(const float* h, int64_t ldh, const int64_t* rows, int64_t n, int F,
                         uint32_t* bits, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (F % 32 != 0 || ldh % 4 != 0 || (reinterpret_cast<uintptr_t>(h) & 15)) return hipErrorInvalidValue;
  const int words = F / 32;
  const int64_t blocks = (n * words + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_keep_bits_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     h, ldh, rows, n, words, bits);
  return hipGetLastError();
}

hipError_t apply_keep_bits(float* g, int64_t ldg, const uint32_t* bits, int64_t n, int F,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (F % 32 != 0 || ldg % 4 != 0 || (reinterpret_cast<uintptr_t>(g) & 15)) return hipErrorInvalidValue;
  const int words = F / 32;
  const int64_t blocks = (n * words + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(apply_keep_bits_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     st, g, ldg, bits, n, words);
  return hipGetLastError();
}

}  // namespace dgraph
