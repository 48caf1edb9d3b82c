// dgraph_amd — 1-bit ReLU keep masks of selected rows (gfx950).
//
// The memory-lean fp32 executor (models/sage_fused.py) frees a hidden activation right after
// the forward, but the backward needs its ReLU derivative on the gradient-support rows. It
// keeps exactly that: one bit per element of the selected rows (32 x smaller than the fp32
// rows; ~1 GB for 3.3e7 x 256 at the papers100M shape).
//   row_keep_bits:   bits[i][w] bit j = (h[rows[i]][32 w + j] > 0)
//   apply_keep_bits: g[i][f] = bit(i, f) ? g[i][f] : 0   (in place)
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

// Lane per 16-B float4 of a row (a wave reads 1 KB contiguously); 8 consecutive lanes hold
// one 32-bit word (F % 32 == 0, so words never straddle rows or waves). (Was one thread per
// word with 8 x 16-B loads 128 B apart: 2.9-3.5 TB/s, profiles/r04/prof_w1_step_kernels.txt.)
__global__ __launch_bounds__(256) void row_keep_bits_kernel(const float* __restrict__ h,
                                                            int64_t ldh,
                                                            const int64_t* __restrict__ rows,
                                                            int64_t n, int F,
                                                            uint32_t* __restrict__ bits) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int V = F / 4;
  const bool in = t < n * V;
  const int64_t i = in ? t / V : 0;
  const int f = static_cast<int>(t - i * V);
  uint32_t nib = 0;
  if (in) {
    const int64_t r = rows ? rows[i] : i;
    const float4 v = *reinterpret_cast<const float4*>(h + r * ldh + 4 * f);
    nib = (v.x > 0.f ? 1u : 0u) | (v.y > 0.f ? 2u : 0u) | (v.z > 0.f ? 4u : 0u) |
          (v.w > 0.f ? 8u : 0u);
  }
  uint32_t m = nib << (4 * (f & 7));
  m |= __shfl_xor(m, 1, kWave);
  m |= __shfl_xor(m, 2, kWave);
  m |= __shfl_xor(m, 4, kWave);
  if (in && (f & 7) == 0) bits[i * (V / 8) + f / 8] = m;
}

__global__ __launch_bounds__(256) void apply_keep_bits_kernel(float* __restrict__ g,
                                                              int64_t ldg,
                                                              const uint32_t* __restrict__ bits,
                                                              int64_t n, int F,
                                                              const int64_t* __restrict__ rows) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int V = F / 4;
  if (t >= n * V) return;
  const int64_t k = t / V;
  const int f = static_cast<int>(t - k * V);
  const int64_t i = rows ? rows[k] : k;  // (rows: a subset of g's rows, bits indexed alike)
  const uint32_t m = bits[i * (V / 8) + f / 8] >> (4 * (f & 7));
  float4* p = reinterpret_cast<float4*>(g + i * ldg + 4 * f);
  float4 v = *p;
  v.x = (m & 1u) ? v.x : 0.f;
  v.y = (m & 2u) ? v.y : 0.f;
  v.z = (m & 4u) ? v.z : 0.f;
  v.w = (m & 8u) ? v.w : 0.f;
  *p = v;
}

}  // namespace

hipError_t row_keep_bits(const float* h, int64_t ldh, const int64_t* rows, int64_t n, int F,
                         uint32_t* bits, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (F % 32 != 0 || ldh % 4 != 0 || (reinterpret_cast<uintptr_t>(h) & 15)) return hipErrorInvalidValue;
  const int64_t blocks = (n * (F / 4) + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(row_keep_bits_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     h, ldh, rows, n, F, bits);
  return hipGetLastError();
}

hipError_t apply_keep_bits(float* g, int64_t ldg, const uint32_t* bits, int64_t n, int F,
                           hipStream_t st, const int64_t* rows) {
  if (n <= 0) return hipSuccess;
  if (F % 32 != 0 || ldg % 4 != 0 || (reinterpret_cast<uintptr_t>(g) & 15)) return hipErrorInvalidValue;
  const int64_t blocks = (n * (F / 4) + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(apply_keep_bits_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     st, g, ldg, bits, n, F, rows);
  return hipGetLastError();
}

}  // namespace dgraph
