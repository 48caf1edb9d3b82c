// dgraph_amd — edge softmax over CSR segments for gfx950 (K-new-3).
//
// Replaces the exp -> scatter-sum -> gather -> divide chain of the reference's
// CommAwareGAT (RGAT.py:147-165,191-202), which also skipped the max subtraction
// (RGAT.py:154). One wavefront owns one destination segment; lanes are split into
// LPE = pow2(H) lanes per edge (one per head) and EPW = 64/LPE edges per step.
// Three passes (max, sum, normalise) re-read the segment from L1/L2.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <int LPE>
__global__ __launch_bounds__(256) void edge_softmax_fwd_kernel(
    const int64_t* __restrict__ rowptr, const float* __restrict__ s, float* __restrict__ alpha,
    int64_t nrows, int H) {
  constexpr int EPW = kWave / LPE;
  const int lane = threadIdx.x & (kWave - 1);
  const int eg = lane / LPE;
  const int h = lane % LPE;
  const bool hv = h < H;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t b = rowptr[r], e = rowptr[r + 1];
    float m = -INFINITY;
    for (int64_t j = b + eg; j < e; j += EPW)
      if (hv) m = fmaxf(m, s[j * H + h]);
#pragma unroll
    for (int off = LPE; off < kWave; off <<= 1) m = fmaxf(m, __shfl_xor(m, off, kWave));
    float sum = 0.f;
    for (int64_t j = b + eg; j < e; j += EPW)
      if (hv) sum += __expf(s[j * H + h] - m);
#pragma unroll
    for (int off = LPE; off < kWave; off <<= 1) sum += __shfl_xor(sum, off, kWave);
    const float inv = sum > 0.f ? 1.f / sum : 0.f;
    for (int64_t j = b + eg; j < e; j += EPW)
      if (hv) alpha[j * H + h] = __expf(s[j * H + h] - m) * inv;
  }
}

template <int LPE>
__global__ __launch_bounds__(256) void edge_softmax_bwd_kernel(
    const int64_t* __restrict__ rowptr, const float* __restrict__ alpha,
    const float* __restrict__ g, float* __restrict__ ds, int64_t nrows, int H) {
  constexpr int EPW = kWave / LPE;
  const int lane = threadIdx.x & (kWave - 1);
  const int eg = lane / LPE;
  const int h = lane % LPE;
  const bool hv = h < H;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t b = rowptr[r], e = rowptr[r + 1];
    float dot = 0.f;
    for (int64_t j = b + eg; j < e; j += EPW)
      if (hv) dot = fmaf(alpha[j * H + h], g[j * H + h], dot);
#pragma unroll
    for (int off = LPE; off < kWave; off <<= 1) dot += __shfl_xor(dot, off, kWave);
    for (int64_t j = b + eg; j < e; j += EPW)
      if (hv) {
        const float a = alpha[j * H + h];
        ds[j * H + h] = a * (g[j * H + h] - dot);
      }
  }
}

inline int lpe_for(int H) {
  int l = 1;
  while (l < H) l <<= 1;
  return l;
}

}  // namespace

#define DG_SOFTMAX_SWITCH(KERNEL, ...)                                                 \
  switch (lpe_for(H)) {                                                                \
    case 1: hipLaunchKernelGGL((KERNEL<1>), grid, block, 0, st, __VA_ARGS__); break;   \
    case 2: hipLaunchKernelGGL((KERNEL<2>), grid, block, 0, st, __VA_ARGS__); break;   \
    case 4: hipLaunchKernelGGL((KERNEL<4>), grid, block, 0, st, __VA_ARGS__); break;   \
    case 8: hipLaunchKernelGGL((KERNEL<8>), grid, block, 0, st, __VA_ARGS__); break;   \
    case 16: hipLaunchKernelGGL((KERNEL<16>), grid, block, 0, st, __VA_ARGS__); break; \
    case 32: hipLaunchKernelGGL((KERNEL<32>), grid, block, 0, st, __VA_ARGS__); break; \
    case 64: hipLaunchKernelGGL((KERNEL<64>), grid, block, 0, st, __VA_ARGS__); break; \
    default: return hipErrorInvalidValue;                                              \
  }

hipError_t edge_softmax_fwd(const int64_t* rowptr, const float* s, float* alpha,
                            int64_t nrows, int H, hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  if (H < 1 || H > 64) return hipErrorInvalidValue;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nrows + 3) / 4, 256 * 32)));
  DG_SOFTMAX_SWITCH(edge_softmax_fwd_kernel, rowptr, s, alpha, nrows, H)
  return hipGetLastError();
}

hipError_t edge_softmax_bwd(const int64_t* rowptr, const float* alpha, const float* g,
                            float* ds, int64_t nrows, int H, hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  if (H < 1 || H > 64) return hipErrorInvalidValue;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nrows + 3) / 4, 256 * 32)));
  DG_SOFTMAX_SWITCH(edge_softmax_bwd_kernel, rowptr, alpha, g, ds, nrows, H)
  return hipGetLastError();
}

}  // namespace dgraph
