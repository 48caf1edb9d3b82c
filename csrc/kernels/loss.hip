// dgraph_amd — fused softmax cross-entropy and argmax hits of selected logit rows (gfx950).
//
// The full-graph step computes logits for every vertex in row chunks and needs, per chunk,
// the loss rows' cross-entropy and its gradient, and the validation/test rows' argmax hits
// (experiments/OGB/main.py:140-184 does the same on a dense [V, C] logit matrix with
// torch ops). One wave per row, C <= 256 logits (4 per lane), wave64 butterfly reductions:
//   xent_rows:   row_loss[i] = logsumexp(z_r) - z_r[y_i]
//                dz[i, c]    = (softmax(z_r)_c - [c == y_i]) * scale   (c < C; 0 up to dz_width)
//   argmax_hits: hit[i] = (first argmax of z_r == y_i)        (r = rows[i])
// Per-row outputs (no atomics): the caller sums them once per step in a fixed order.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__global__ __launch_bounds__(256) void xent_rows_kernel(
    const float* __restrict__ z, int64_t ldz, int C, const int64_t* __restrict__ rows,
    const int64_t* __restrict__ y, int64_t n, float scale, float* __restrict__ dz,
    int64_t ldd, int dz_width, float* __restrict__ row_loss) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (i >= n) return;  // wave-uniform
  const float* zr = z + rows[i] * ldz;
  const int yi = static_cast<int>(y[i]);
  float v[4];
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    v[q] = c < C ? zr[c] : -INFINITY;
    m = fmaxf(m, v[q]);
  }
  m = wave_max(m);
  float se = 0.f, zy = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    const float e = c < C ? __expf(v[q] - m) : 0.f;
    v[q] = e;
    se += e;
    zy += c == yi ? zr[c] : 0.f;
  }
  se = wave_sum(se);
  zy = wave_sum(zy);
  const float inv = 1.f / se;
  float* dr = dz + i * ldd;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    if (c < dz_width) dr[c] = c < C ? (v[q] * inv - (c == yi ? 1.f : 0.f)) * scale : 0.f;
  }
  if (lane == 0) row_loss[i] = (m + __logf(se)) - zy;
}

__global__ __launch_bounds__(256) void argmax_hits_kernel(
    const float* __restrict__ z, int64_t ldz, int C, const int64_t* __restrict__ rows,
    const int64_t* __restrict__ y, int64_t n, uint8_t* __restrict__ hit) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (i >= n) return;
  const float* zr = z + rows[i] * ldz;
  float best = -INFINITY;
  int bi = 0x7fffffff;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = lane + 64 * q;
    if (c < C) {
      const float v = zr[c];
      if (v > best || (v == best && c < bi)) {
        best = v;
        bi = c;
      }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ob = __shfl_xor(best, off, kWave);
    const int oi = __shfl_xor(bi, off, kWave);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  if (lane == 0) hit[i] = bi == static_cast<int>(y[i]) ? 1 : 0;
}

}  // namespace

hipError_t xent_rows(const float* z, int64_t ldz, int C, const int64_t* rows, const int64_t* y,
                     int64_t n, float scale, float* dz, int64_t ldd, int dz_width,
                     float* row_loss, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (C <= 0 || C > 256 || dz_width > 256 || dz_width < C) return hipErrorInvalidValue;
  const int64_t blocks = (n + 3) / 4;
  hipLaunchKernelGGL(xent_rows_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, z,
                     ldz, C, rows, y, n, scale, dz, ldd, dz_width, row_loss);
  return hipGetLastError();
}

hipError_t argmax_hits(const float* z, int64_t ldz, int C, const int64_t* rows,
                       const int64_t* y, int64_t n, uint8_t* hit, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (C <= 0 || C > 256) return hipErrorInvalidValue;
  const int64_t blocks = (n + 3) / 4;
  hipLaunchKernelGGL(argmax_hits_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     z, ldz, C, rows, y, n, hit);
  return hipGetLastError();
}

}  // namespace dgraph
