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

// One 512-element chunk per wave-iteration step; CH chunks are loaded before any is
// processed so each wave keeps CH x 1 KiB of loads in flight (a single chunk per
// iteration left the kernel latency-bound at ~2.2 TB/s, profiles/).
template <typename T, int CH>
__global__ __launch_bounds__(256) void bias_relu_pack_kernel(
    T* __restrict__ y, const float* __restrict__ bias, uint64_t* __restrict__ bits,
    int64_t numel, int F, bool relu) {
  constexpr int VEC = 8;  // elements per lane (16 B bf16, 32 B fp32)
  // the bias is staged once per block in LDS (the per-element global bias loads made the
  // first version VMEM-issue bound: 8 loads per 16 B of data)
  extern __shared__ __attribute__((aligned(16))) float sbias[];
  if (bias)
    for (int c = threadIdx.x; c < F; c += blockDim.x) sbias[c] = bias[c];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (numel + 511) / 512;
  const int64_t wave =
      __builtin_amdgcn_readfirstlane((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t ch0 = wave * CH; ch0 < nchunks; ch0 += nwaves * CH) {
    float x[CH][VEC];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t e0 = (ch0 + c) * 512 + lane * VEC;
      if (e0 < numel) {  // numel % 8 == 0 (host check)
        if constexpr (sizeof(T) == 2) {
          load_vec_f32<T, 8>(y + e0, x[c]);
        } else {
          float a[4], b[4];
          load_vec_f32<T, 4>(y + e0, a);
          load_vec_f32<T, 4>(y + e0 + 4, b);
#pragma unroll
          for (int i = 0; i < 4; ++i) { x[c][i] = a[i]; x[c][i + 4] = b[i]; }
        }
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) x[c][i] = 0.f;
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t ch = ch0 + c;
      if (ch >= nchunks) break;  // wave-uniform
      const int64_t e0 = ch * 512 + lane * VEC;
      const bool valid = e0 < numel;
      // column of this lane's first element: one 64-bit modulo per chunk (scalar), then
      // 32-bit math per lane; F % 8 == 0 keeps a lane's 8 elements in one row
      const int cbase = static_cast<int>((ch * 512) % F);
      const int c0 = (cbase + lane * VEC) % F;
      uint64_t my_word = 0;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float t = x[c][j] + (bias ? sbias[c0 + j] : 0.f);
        const bool keep = t > 0.f;
        if (relu) t = keep ? t : 0.f;
        x[c][j] = t;
        const uint64_t b = __ballot(valid && keep);
        if (lane == j) my_word = b;
      }
      if (valid) {
        if constexpr (sizeof(T) == 2) {
          store_vec_f32<T, 8>(y + e0, x[c]);
        } else {
          float a[4] = {x[c][0], x[c][1], x[c][2], x[c][3]};
          float b[4] = {x[c][4], x[c][5], x[c][6], x[c][7]};
          store_vec_f32<T, 4>(y + e0, a);
          store_vec_f32<T, 4>(y + e0 + 4, b);
        }
      }
      if (bits && relu && lane < VEC) bits[ch * 8 + lane] = my_word;
    }
  }
}

template <typename T, int CH>
__global__ __launch_bounds__(256) void relu_mask_bwd_kernel(
    T* __restrict__ g, const uint64_t* __restrict__ bits, int64_t numel) {
  constexpr int VEC = 8;
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (numel + 511) / 512;
  const int64_t wave =
      __builtin_amdgcn_readfirstlane((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t ch0 = wave * CH; ch0 < nchunks; ch0 += nwaves * CH) {
    T v[CH][VEC];
#pragma unroll
    for (int c = 0; c < CH; ++c) {  // issue every data load of the group first
      const int64_t e0 = (ch0 + c) * 512 + lane * VEC;
      if (e0 < numel) {
#pragma unroll
        for (int k = 0; k < VEC * static_cast<int>(sizeof(T)) / 16; ++k)
          reinterpret_cast<uint4*>(v[c])[k] = reinterpret_cast<const uint4*>(g + e0)[k];
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t ch = ch0 + c;
      if (ch >= nchunks) break;  // wave-uniform
      const int64_t e0 = ch * 512 + lane * VEC;
      // the chunk's 8 mask words are wave-uniform: scalar loads (s_load), then each lane
      // extracts its bit of word j with one 64-bit shift
      const uint64_t* wp = bits + ch * 8;
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < VEC; ++j) m |= static_cast<uint32_t>((wp[j] >> lane) & 1u) << j;
      if (e0 >= numel || m == 0xFFu) continue;
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (!((m >> j) & 1u)) v[c][j] = T(0);
#pragma unroll
      for (int k = 0; k < VEC * static_cast<int>(sizeof(T)) / 16; ++k)
        reinterpret_cast<uint4*>(g + e0)[k] = reinterpret_cast<const uint4*>(v[c])[k];
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
  constexpr int CH = 4;
  dim3 block(256),
      grid(static_cast<unsigned>(cap_blocks((nchunks + 4 * CH - 1) / (4 * CH), 256 * 8)));
  auto* b64 = reinterpret_cast<uint64_t*>(bits);
  const size_t lds = bias ? static_cast<size_t>(F) * sizeof(float) : 0;
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  if (dt == DType::F32)
    hipLaunchKernelGGL((bias_relu_pack_kernel<float, CH>), grid, block, lds, st,
                       static_cast<float*>(y), bias, b64, numel, F, relu);
  else
    hipLaunchKernelGGL((bias_relu_pack_kernel<uint16_t, CH>), grid, block, lds, st,
                       static_cast<uint16_t*>(y), bias, b64, numel, F, relu);
  return hipGetLastError();
}

hipError_t relu_mask_bwd(DType dt, void* g, const uint32_t* bits, int64_t numel,
                         hipStream_t st) {
  if (numel <= 0) return hipSuccess;
  if (numel % 8 != 0) return hipErrorInvalidValue;
  const int64_t nchunks = (numel + 511) / 512;
  constexpr int CH = 4;
  dim3 block(256),
      grid(static_cast<unsigned>(cap_blocks((nchunks + 4 * CH - 1) / (4 * CH), 256 * 8)));
  const auto* b64 = reinterpret_cast<const uint64_t*>(bits);
  if (dt == DType::F32)
    hipLaunchKernelGGL((relu_mask_bwd_kernel<float, CH>), grid, block, 0, st,
                       static_cast<float*>(g), b64, numel);
  else
    hipLaunchKernelGGL((relu_mask_bwd_kernel<uint16_t, CH>), grid, block, 0, st,
                       static_cast<uint16_t*>(g), b64, numel);
  return hipGetLastError();
}

hipError_t col_sum_partial(DType dt, const void* g, int64_t ld, int64_t L, int F,
                           float* partial, int nblocks, hipStream_t st) {
  if (L <= 0 || F <= 0) return hipSuccess;
  int vec = dt == DType::F32 ? 4 : 8;
  if (F % vec != 0 || ld % vec != 0) vec = 1;  // scalar lanes for odd widths (e.g. 73)
  if (F / vec > 256) return hipErrorInvalidValue;
  const int64_t rpb = (L + nblocks - 1) / nblocks;
  const int tpr = F / vec;
  const int rpi = 256 / tpr;
  const size_t lds = static_cast<size_t>(rpi) * F * sizeof(float);
  dim3 block(256), grid(nblocks);
  if (dt == DType::F32) {
    auto gp = static_cast<const float*>(g);
    if (vec == 4)
      hipLaunchKernelGGL((col_sum_partial_kernel<float, 4>), grid, block, lds, st, gp, ld, L,
                         F, rpb, partial);
    else
      hipLaunchKernelGGL((col_sum_partial_kernel<float, 1>), grid, block, lds, st, gp, ld, L,
                         F, rpb, partial);
  } else {
    auto gp = static_cast<const uint16_t*>(g);
    if (vec == 8)
      hipLaunchKernelGGL((col_sum_partial_kernel<uint16_t, 8>), grid, block, lds, st, gp, ld,
                         L, F, rpb, partial);
    else
      hipLaunchKernelGGL((col_sum_partial_kernel<uint16_t, 1>), grid, block, lds, st, gp, ld,
                         L, F, rpb, partial);
  }
  return hipGetLastError();
}

}  // namespace dgraph

// ---------------------------------------------------------------------------
// row_scale_cols: out[r, j] = x[r, c0 + j] * s[r] for j < w (bf16 or fp32 data, fp32 s).
// The pre-scale pass of the transposed mean aggregation (dist_graph._spmm_col_scaled):
// torch's broadcast mul on a strided [1.1e8, 128] column slice split into 32 sub-launches
// per call (int32 indexing) and ran at ~1/3 of HBM bandwidth (profiles/). Here a lane owns
// one 16-B vector of a row, a wave covers 64 * VEC / w rows, and every wave keeps CH
// vectors in flight before it stores.
// ---------------------------------------------------------------------------
namespace dgraph {
namespace {

template <typename T, int CH>
__global__ __launch_bounds__(256) void row_scale_cols_kernel(
    const T* __restrict__ x, int64_t ldx, const float* __restrict__ s, T* __restrict__ out,
    int64_t ldo, int64_t L, int w) {
  constexpr int VEC = 16 / sizeof(T);
  const int vpr = w / VEC;  // vectors per row (w % VEC == 0, host check)
  const int64_t nvec = L * vpr;
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t nthreads = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v0 = tid; v0 < nvec; v0 += nthreads * CH) {
    float val[CH][VEC];
    float sc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t v = v0 + c * nthreads;
      if (v < nvec) {
        const int64_t r = v / vpr;
        const int j = static_cast<int>(v - r * vpr) * VEC;
        load_vec_f32<T, VEC>(x + r * ldx + j, val[c]);
        sc[c] = s[r];
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int64_t v = v0 + c * nthreads;
      if (v < nvec) {
        const int64_t r = v / vpr;
        const int j = static_cast<int>(v - r * vpr) * VEC;
#pragma unroll
        for (int i = 0; i < VEC; ++i) val[c][i] *= sc[c];
        store_vec_f32<T, VEC>(out + r * ldo + j, val[c]);
      }
    }
  }
}

// Same pass, plus the fp32 column sums of the UNSCALED x (the SAGE bias gradient of the
// layer whose output gradient is being pre-scaled for the transposed mean aggregation):
// the bias gradient then costs no pass of its own over x. Block b owns rows
// [b * rows_per_block, ...) (col_sum_partial's layout: fixed partition, fixed-order LDS
// reduction, deterministic); each thread keeps UR rows' vectors in flight.
template <int UR>
__global__ __launch_bounds__(256) void row_scale_colsum_kernel(
    const uint16_t* __restrict__ x, int64_t ldx, const float* __restrict__ s,
    uint16_t* __restrict__ out, int64_t ldo, int64_t L, int w, int64_t rows_per_block,
    float* __restrict__ partial, int64_t ldp) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int VEC = 8;
  const int tpr = w / VEC;           // threads per row (w <= 256)
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
    for (int64_t rb = r0 + rg; rb < r1; rb += static_cast<int64_t>(rpi) * UR) {
      float v[UR][VEC];
      float sc[UR];
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int64_t r = rb + static_cast<int64_t>(u) * rpi;
        if (r < r1) {
          load_vec_f32<uint16_t, VEC>(x + r * ldx + cc, v[u]);
          sc[u] = s[r];
        }
      }
#pragma unroll
      for (int u = 0; u < UR; ++u) {
        const int64_t r = rb + static_cast<int64_t>(u) * rpi;
        if (r < r1) {
#pragma unroll
          for (int i = 0; i < VEC; ++i) {
            acc[i] += v[u][i];
            v[u][i] *= sc[u];
          }
          store_vec_f32<uint16_t, VEC>(out + r * ldo + cc, v[u]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) smem[rg * w + cc + i] = acc[i];
  }
  __syncthreads();
  for (int c = t; c < w; c += blockDim.x) {
    float sum = 0.f;
    for (int k = 0; k < rpi; ++k) sum += smem[k * w + c];
    partial[static_cast<int64_t>(blockIdx.x) * ldp + c] = sum;
  }
}

}  // namespace

hipError_t row_scale_colsum(const void* x, int64_t ldx, const float* s, void* out,
                            int64_t ldo, int64_t L, int w, float* partial, int64_t ldp,
                            int nblocks, hipStream_t st) {
  if (L <= 0 || w <= 0) return hipSuccess;
  if (w % 8 != 0 || w > 256 || ldx % 8 != 0 || ldo % 8 != 0) return hipErrorInvalidValue;
  const int64_t rpb = (L + nblocks - 1) / nblocks;
  const int rpi = 256 / (w / 8);
  const size_t lds = static_cast<size_t>(rpi) * w * sizeof(float);
  hipLaunchKernelGGL((row_scale_colsum_kernel<4>), dim3(nblocks), dim3(256), lds, st,
                     static_cast<const uint16_t*>(x), ldx, s, static_cast<uint16_t*>(out),
                     ldo, L, w, rpb, partial, ldp);
  return hipGetLastError();
}

hipError_t row_scale_cols(DType dt, const void* x, int64_t ldx, const float* s, void* out,
                          int64_t ldo, int64_t L, int w, hipStream_t st) {
  if (L == 0 || w == 0) return hipSuccess;
  const int vec = dt == DType::BF16 ? 8 : 4;
  const int64_t nvec = L * (w / vec);
  const int64_t blocks = cap_blocks((nvec + 255) / 256, 256 * 32);
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
  if (dt == DType::BF16) {
    hipLaunchKernelGGL((row_scale_cols_kernel<uint16_t, 4>), grid, block, 0, st,
                       static_cast<const uint16_t*>(x), ldx, s, static_cast<uint16_t*>(out),
                       ldo, L, w);
  } else {
    hipLaunchKernelGGL((row_scale_cols_kernel<float, 4>), grid, block, 0, st,
                       static_cast<const float*>(x), ldx, s, static_cast<float*>(out), ldo, L,
                       w);
  }
  return hipGetLastError();
}

}  // namespace dgraph
