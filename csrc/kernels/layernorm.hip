// dgraph_amd — row LayerNorm for tall-skinny activations (GraphCast MLP epilogues).
//
// PyTorch's generic LayerNorm launches one block per row and reduces dgamma/dbeta with a
// separate two-stage kernel; at the GraphCast shapes (3.1 M x 128 edge rows) that ran at
// ~0.9 ms per forward and ~1.4 ms per backward (profiles/graphcast_1gpu_kernel_stats.txt).
// Here:
//   * LPR lanes own one row (F / LPR / VEC chunks per lane, values kept in VGPRs), so a
//     wave normalises 64 / LPR rows at once with 16-B loads; mean and variance are two
//     xor-shuffle reductions inside the lane group (exact two-pass, no E[x^2] - mean^2);
//   * forward optionally adds a residual (y = LN(x) * g + b + r, the GraphCast block
//     ``mlp(x) + x``) and stores per-row mean / rstd (fp32) for backward;
//   * backward recomputes x_hat, writes dx, and accumulates dgamma / dbeta per lane in
//     registers across the rows a wave visits; waves of a block combine through LDS in a
//     fixed order into one fp32 partial row per block (deterministic), summed on the host
//     side over <= 1024 blocks.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <typename T, int VEC, int LPR, int CH, bool RES>
__global__ __launch_bounds__(256) void layer_norm_fwd_kernel(
    const T* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    const T* __restrict__ res, T* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, int64_t N, int F, float eps) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & 63;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const float invF = 1.f / static_cast<float>(F);
  // a lane owns the same columns in every row: gamma / beta live in registers for the
  // whole grid-stride loop (per-row per-element loads made the kernel issue-bound)
  float ga[CH][VEC], be[CH][VEC];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int f = (c * LPR + l) * VEC;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const bool in = gamma != nullptr && f + i < F;
      ga[c][i] = in ? gamma[f + i] : 1.f;
      be[c][i] = in ? beta[f + i] : 0.f;
    }
  }
  for (int64_t base = wave * G; base < N; base += nwaves * G) {
    const int64_t r = base + g;
    const bool valid = r < N;
    float v[CH][VEC];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (valid && f < F) {
        load_vec_f32<T, VEC>(x + r * F + f, v[c]);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) v[c][i] = 0.f;
      }
#pragma unroll
      for (int i = 0; i < VEC; ++i) s += v[c][i];
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) s += __shfl_xor(s, off, kWave);
    const float mu = s * invF;
    float q = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (f < F) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float d = v[c][i] - mu;
          q += d * d;
        }
      }
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) q += __shfl_xor(q, off, kWave);
    const float rs = rsqrtf(q * invF + eps);
    if (!valid) continue;
    if (l == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rs;
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (f >= F) continue;
      float o[VEC], rr[VEC];
      if constexpr (RES) load_vec_f32<T, VEC>(res + r * F + f, rr);
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        float t = (v[c][i] - mu) * rs * ga[c][i] + be[c][i];
        if constexpr (RES) t += rr[i];
        o[i] = t;
      }
      store_vec_f32<T, VEC>(y + r * F + f, o);
    }
  }
}

template <typename T, int VEC, int LPR, int CH>
__global__ __launch_bounds__(256) void layer_norm_bwd_kernel(
    const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma, T* __restrict__ dx,
    float* __restrict__ partial, int64_t N, int F) {
  constexpr int G = kWave / LPR;
  extern __shared__ float sred[];  // [waves][2][F]
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const int g = lane / LPR, l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const float invF = 1.f / static_cast<float>(F);
  float dg[CH][VEC], db[CH][VEC], ga[CH][VEC];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int f = (c * LPR + l) * VEC;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      dg[c][i] = db[c][i] = 0.f;
      ga[c][i] = (gamma != nullptr && f + i < F) ? gamma[f + i] : 1.f;
    }
  }
  for (int64_t base = wave * G; base < N; base += nwaves * G) {
    const int64_t r = base + g;
    const bool valid = r < N;
    const float mu = valid ? mean[r] : 0.f;
    const float rs = valid ? rstd[r] : 0.f;
    float xh[CH][VEC], gy[CH][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (valid && f < F) {
        float xv[VEC];
        load_vec_f32<T, VEC>(x + r * F + f, xv);
        load_vec_f32<T, VEC>(dy + r * F + f, gy[c]);
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          xh[c][i] = (xv[i] - mu) * rs;
          dg[c][i] += gy[c][i] * xh[c][i];
          db[c][i] += gy[c][i];
          const float d = gy[c][i] * ga[c][i];
          gy[c][i] = d;  // now dxhat
          s1 += d;
          s2 += d * xh[c][i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) xh[c][i] = gy[c][i] = 0.f;
      }
    }
#pragma unroll
    for (int off = 1; off < LPR; off <<= 1) {
      s1 += __shfl_xor(s1, off, kWave);
      s2 += __shfl_xor(s2, off, kWave);
    }
    if (!valid) continue;
    const float m1 = s1 * invF, m2 = s2 * invF;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (f >= F) continue;
      float o[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) o[i] = rs * (gy[c][i] - m1 - xh[c][i] * m2);
      store_vec_f32<T, VEC>(dx + r * F + f, o);
    }
  }
  // combine the G row groups of the wave (xor over the group bits), then the waves
#pragma unroll
  for (int off = LPR; off < kWave; off <<= 1)
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        dg[c][i] += __shfl_xor(dg[c][i], off, kWave);
        db[c][i] += __shfl_xor(db[c][i], off, kWave);
      }
  if (g == 0) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int f = (c * LPR + l) * VEC;
      if (f >= F) continue;
#pragma unroll
      for (int i = 0; i < VEC; ++i) {
        sred[(w * 2) * F + f + i] = dg[c][i];
        sred[(w * 2 + 1) * F + f + i] = db[c][i];
      }
    }
  }
  __syncthreads();
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < nw; ++k) {
      a += sred[(k * 2) * F + f];
      b += sred[(k * 2 + 1) * F + f];
    }
    partial[(static_cast<int64_t>(blockIdx.x) * 2) * F + f] = a;
    partial[(static_cast<int64_t>(blockIdx.x) * 2 + 1) * F + f] = b;
  }
}

template <typename T>
struct LNCfg {
  int vec, lpr, ch;
};

template <typename T>
LNCfg<T> ln_cfg(int F) {
  constexpr int V = 16 / sizeof(T);
  const int vec = (F % V == 0) ? V : 1;
  const int per = (F + vec - 1) / vec;  // vector slots per row
  int lpr = per <= 4 ? 4 : per <= 8 ? 8 : per <= 16 ? 16 : per <= 32 ? 32 : 64;
  int ch = (per + lpr - 1) / lpr;
  ch = ch <= 1 ? 1 : ch <= 2 ? 2 : ch <= 4 ? 4 : 8;
  return {vec, lpr, ch};
}

#define DG_LN_SWITCH(VEC_, BODY)                                            \
  switch (c.lpr * 16 + c.ch) {                                              \
    case 4 * 16 + 1: { constexpr int L_ = 4, C_ = 1; BODY; } break;         \
    case 8 * 16 + 1: { constexpr int L_ = 8, C_ = 1; BODY; } break;         \
    case 16 * 16 + 1: { constexpr int L_ = 16, C_ = 1; BODY; } break;       \
    case 32 * 16 + 1: { constexpr int L_ = 32, C_ = 1; BODY; } break;       \
    case 64 * 16 + 1: { constexpr int L_ = 64, C_ = 1; BODY; } break;       \
    case 64 * 16 + 2: { constexpr int L_ = 64, C_ = 2; BODY; } break;       \
    case 64 * 16 + 4: { constexpr int L_ = 64, C_ = 4; BODY; } break;       \
    default: { constexpr int L_ = 64, C_ = 8; BODY; } break;                \
  }

template <typename T>
hipError_t ln_fwd(const void* x, const float* gamma, const float* beta, const void* res,
                  void* y, float* mean, float* rstd, int64_t N, int F, float eps,
                  hipStream_t st) {
  const auto c = ln_cfg<T>(F);
  const int64_t G = kWave / c.lpr;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((N + 4 * G - 1) / (4 * G), 256 * 32)));
  auto xp = static_cast<const T*>(x);
  auto rp = static_cast<const T*>(res);
  auto yp = static_cast<T*>(y);
  if (c.vec == 16 / static_cast<int>(sizeof(T))) {
    constexpr int V_ = 16 / sizeof(T);
    if (res) {
      DG_LN_SWITCH(V_, hipLaunchKernelGGL((layer_norm_fwd_kernel<T, V_, L_, C_, true>), grid,
                                          block, 0, st, xp, gamma, beta, rp, yp, mean, rstd, N,
                                          F, eps))
    } else {
      DG_LN_SWITCH(V_, hipLaunchKernelGGL((layer_norm_fwd_kernel<T, V_, L_, C_, false>), grid,
                                          block, 0, st, xp, gamma, beta, rp, yp, mean, rstd, N,
                                          F, eps))
    }
  } else {
    if (res) {
      DG_LN_SWITCH(1, hipLaunchKernelGGL((layer_norm_fwd_kernel<T, 1, L_, C_, true>), grid,
                                         block, 0, st, xp, gamma, beta, rp, yp, mean, rstd, N,
                                         F, eps))
    } else {
      DG_LN_SWITCH(1, hipLaunchKernelGGL((layer_norm_fwd_kernel<T, 1, L_, C_, false>), grid,
                                         block, 0, st, xp, gamma, beta, rp, yp, mean, rstd, N,
                                         F, eps))
    }
  }
  return hipGetLastError();
}

template <typename T>
hipError_t ln_bwd(const void* dy, const void* x, const float* mean, const float* rstd,
                  const float* gamma, void* dx, float* partial, int nblocks, int64_t N, int F,
                  hipStream_t st) {
  const auto c = ln_cfg<T>(F);
  dim3 block(256), grid(static_cast<unsigned>(nblocks));
  const size_t lds = static_cast<size_t>(256 / 64) * 2 * F * sizeof(float);
  auto dyp = static_cast<const T*>(dy);
  auto xp = static_cast<const T*>(x);
  auto dxp = static_cast<T*>(dx);
  if (c.vec == 16 / static_cast<int>(sizeof(T))) {
    constexpr int V_ = 16 / sizeof(T);
    DG_LN_SWITCH(V_, hipLaunchKernelGGL((layer_norm_bwd_kernel<T, V_, L_, C_>), grid, block,
                                        lds, st, dyp, xp, mean, rstd, gamma, dxp, partial, N,
                                        F))
  } else {
    DG_LN_SWITCH(1, hipLaunchKernelGGL((layer_norm_bwd_kernel<T, 1, L_, C_>), grid, block, lds,
                                       st, dyp, xp, mean, rstd, gamma, dxp, partial, N, F))
  }
  return hipGetLastError();
}

}  // namespace

hipError_t layer_norm_fwd(DType dt, const void* x, const float* gamma, const float* beta,
                          const void* res, void* y, float* mean, float* rstd, int64_t N, int F,
                          float eps, hipStream_t st) {
  if (N <= 0 || F <= 0) return hipSuccess;
  if (dt == DType::F32) return ln_fwd<float>(x, gamma, beta, res, y, mean, rstd, N, F, eps, st);
  return ln_fwd<uint16_t>(x, gamma, beta, res, y, mean, rstd, N, F, eps, st);
}

hipError_t layer_norm_bwd(DType dt, const void* dy, const void* x, const float* mean,
                          const float* rstd, const float* gamma, void* dx, float* partial,
                          int nblocks, int64_t N, int F, hipStream_t st) {
  if (N <= 0 || F <= 0) return hipSuccess;
  if (dt == DType::F32)
    return ln_bwd<float>(dy, x, mean, rstd, gamma, dx, partial, nblocks, N, F, st);
  return ln_bwd<uint16_t>(dy, x, mean, rstd, gamma, dx, partial, nblocks, N, F, st);
}

}  // namespace dgraph
