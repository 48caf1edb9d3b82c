// dgraph_amd — synchronised BatchNorm over vertex rows (K-new-7), gfx950.
//
// Replaces the reference's DistributedBatchNorm1D math (experiments/OGB-LSC/
// distributed_layers.py:22-207: torch reductions in fp32 on full-size temporaries, four
// all-reduces, D8 defects). Four launches per layer, none of which materialises an fp32
// copy of the [N, F] activations (at N ~ 15M, F = 256 each fp32 temporary is 15.6 GB,
// and their malloc/free churn dominated a step):
//
//   bn_reduce mode 0 (statistics):  P[b] = ( sum (x - shift), sum (x - shift)^2 )
//   bn_reduce mode 1 (backward):    P[b] = ( sum dy', sum dy' * xhat )
//                                    dy' = dy * [y > 0] when the ReLU is fused
//   bn_finalize: out[k][f] = sum_b P[b][k][f] in a fixed order, in fp64 (deterministic)
//   bn_apply mode 0 (forward):      y  = drop(act((x - mean) * rstd * g + b))
//   bn_apply mode 1 (backward):     dx = (dy' - c1 - xhat * c2) * rstd * g
//
// Fused dropout (drop_thresh > 0): element (r, c) is kept iff hash(seed, r * F + c) >=
// drop_thresh (= p * 2^32), kept values scaled by 1/(1-p). The mask is a pure function of
// (seed, index), so the backward kernels regenerate it (dy' = dy * keep / (1-p) first):
// no mask tensor, no separate dropout / masked-scale passes over [N, F].
//
// Mapping: a row of F elements is covered by LPR lanes with VEC-element (16-byte) vectors;
// a wave holds 64/LPR rows, a block 4 waves; blocks stride over row groups (grid.x) and
// column tiles of LPR*VEC (grid.y). Per-column parameters live in registers. The
// statistics are shifted by a per-column reference value (the first row) so the
// single-pass sum/sum-of-squares does not cancel when |mean| >> std.
#include <type_traits>

#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

struct BNArgs {
  const void* x;
  int64_t ldx;
  const void* dy;
  int64_t ldy;
  void* out;
  int64_t ldo;
  int64_t N;
  int F;
  const float* mean;  // or shift (stats)
  const float* rstd;
  const float* gamma;
  const float* beta;
  const float* c1;
  const float* c2;
  float* partial;  // [gridDim.x][2][F]
  bool relu;
  uint32_t drop_thresh;  // 0: no dropout
  float keep_scale;
  uint32_t seed_lo, seed_hi;
};

// counter-based keep decision (murmur3 fmix32 of the element index mixed with the seed)
__device__ __forceinline__ bool dropout_keep(const BNArgs& a, int64_t idx) {
  uint32_t h = static_cast<uint32_t>(idx) ^ a.seed_lo;
  h ^= (static_cast<uint32_t>(static_cast<uint64_t>(idx) >> 32) + a.seed_hi) * 0x9E3779B1u;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h >= a.drop_thresh;
}

template <int VEC>
__device__ __forceinline__ void load_param(const float* p, int col, float (&o)[VEC],
                                           float dflt) {
#pragma unroll
  for (int i = 0; i < VEC; ++i) o[i] = p ? p[col + i] : dflt;
}

// MODE 0: stats reduce, 1: backward reduce, 2: forward apply, 3: backward apply
template <typename T, int VEC, int LPR, int MODE>
__global__ __launch_bounds__(256) void bn_kernel(BNArgs a) {
  constexpr int RPW = kWave / LPR;  // rows per wave
  constexpr int RB = 4 * RPW;       // rows per block iteration
  constexpr int CT = LPR * VEC;     // columns per tile
  const int tid = threadIdx.x;
  const int wave = tid / kWave, lane = tid % kWave;
  const int sub = lane / LPR, cl = lane % LPR;
  const int col = blockIdx.y * CT + cl * VEC;
  const bool active = col < a.F;
  const int c = active ? col : 0;

  float mean[VEC], rstd[VEC], g[VEC], b[VEC], c1[VEC], c2[VEC];
  load_param<VEC>(a.mean, c, mean, 0.f);
  if constexpr (MODE != 0) {
    load_param<VEC>(a.rstd, c, rstd, 1.f);
    load_param<VEC>(a.gamma, c, g, 1.f);
    load_param<VEC>(a.beta, c, b, 0.f);
  }
  if constexpr (MODE == 3) {
    load_param<VEC>(a.c1, c, c1, 0.f);
    load_param<VEC>(a.c2, c, c2, 0.f);
  }
  float acc0[VEC], acc1[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc0[i] = acc1[i] = 0.f;

  const T* X = static_cast<const T*>(a.x);
  const T* DY = static_cast<const T*>(a.dy);
  T* O = static_cast<T*>(a.out);
  const int64_t stride = static_cast<int64_t>(gridDim.x) * RB;
  if (active) {
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * RB + wave * RPW + sub; r < a.N;
         r += stride) {
      float x[VEC];
      load_vec_f32<T, VEC>(X + r * a.ldx + col, x);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float d = x[i] - mean[i];
          acc0[i] += d;
          acc1[i] = fmaf(d, d, acc1[i]);
        }
      } else if constexpr (MODE == 2) {
        float y[VEC];
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          float v = fmaf((x[i] - mean[i]) * rstd[i], g[i], b[i]);
          y[i] = a.relu ? fmaxf(v, 0.f) : v;
        }
        if (a.drop_thresh) {
#pragma unroll
          for (int i = 0; i < VEC; ++i)
            y[i] = dropout_keep(a, r * a.F + col + i) ? y[i] * a.keep_scale : 0.f;
        }
        store_vec_f32<T, VEC>(O + r * a.ldo + col, y);
      } else {
        float d[VEC];
        load_vec_f32<T, VEC>(DY + r * a.ldy + col, d);
        if (a.drop_thresh) {
#pragma unroll
          for (int i = 0; i < VEC; ++i)
            d[i] = dropout_keep(a, r * a.F + col + i) ? d[i] * a.keep_scale : 0.f;
        }
#pragma unroll
        for (int i = 0; i < VEC; ++i) {
          const float xh = (x[i] - mean[i]) * rstd[i];
          if (a.relu && fmaf(xh, g[i], b[i]) <= 0.f) d[i] = 0.f;
          if constexpr (MODE == 1) {
            acc0[i] += d[i];
            acc1[i] = fmaf(d[i], xh, acc1[i]);
          } else {
            d[i] = (d[i] - c1[i] - xh * c2[i]) * rstd[i] * g[i];
          }
        }
        if constexpr (MODE == 3) store_vec_f32<T, VEC>(O + r * a.ldo + col, d);
      }
    }
  }
  if constexpr (MODE == 0 || MODE == 1) {
    // fixed-order reduction of the RB row slots of the block through LDS
    __shared__ float s0[RB][CT];
    __shared__ float s1[RB][CT];
    const int slot = wave * RPW + sub;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      s0[slot][cl * VEC + i] = acc0[i];
      s1[slot][cl * VEC + i] = acc1[i];
    }
    __syncthreads();
    float* P = a.partial + static_cast<int64_t>(blockIdx.x) * 2 * a.F;
    for (int t = tid; t < CT; t += 256) {
      const int f = blockIdx.y * CT + t;
      if (f >= a.F) continue;
      float u = 0.f, v = 0.f;
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        u += s0[k][t];
        v += s1[k][t];
      }
      P[f] = u;
      P[a.F + f] = v;
    }
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ P, int nb, int F,
                                   double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // over 2F
  if (i >= 2 * F) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += static_cast<double>(P[static_cast<int64_t>(b) * 2 * F + i]);
  out[i] = s;
}

inline bool aligned_to(const void* p, int bytes) {
  return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0;
}

template <typename T, int VEC, int MODE>
hipError_t launch_lpr(const BNArgs& a, int64_t gx_fixed, hipStream_t st) {
  const int lanes = (a.F + VEC - 1) / VEC;
  auto go = [&](auto lpr_tag) -> hipError_t {
    constexpr int LPR = decltype(lpr_tag)::value;
    constexpr int RB = 4 * (kWave / LPR);
    constexpr int CT = LPR * VEC;
    // reductions launch exactly gx_fixed blocks (one partial row each); the apply
    // kernels take enough row groups to fill the chip
    int64_t gx = gx_fixed > 0 ? gx_fixed : cap_blocks((a.N + RB - 1) / RB, 256 * 16);
    dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>((a.F + CT - 1) / CT));
    hipLaunchKernelGGL((bn_kernel<T, VEC, LPR, MODE>), grid, dim3(256), 0, st, a);
    return hipGetLastError();
  };
  if (lanes <= 8) return go(std::integral_constant<int, 8>{});
  if (lanes <= 16) return go(std::integral_constant<int, 16>{});
  if (lanes <= 32) return go(std::integral_constant<int, 32>{});
  return go(std::integral_constant<int, 64>{});
}

template <typename T, int MODE>
hipError_t launch_any(const BNArgs& a, int64_t gx_fixed, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const bool vec_ok = a.F % V == 0 && a.ldx % V == 0 && aligned_to(a.x, 16) &&
                      (a.dy == nullptr || (a.ldy % V == 0 && aligned_to(a.dy, 16))) &&
                      (a.out == nullptr || (a.ldo % V == 0 && aligned_to(a.out, 16)));
  if (vec_ok) return launch_lpr<T, V, MODE>(a, gx_fixed, st);
  return launch_lpr<T, 1, MODE>(a, gx_fixed, st);
}

template <int MODE>
hipError_t dispatch(DType dt, const BNArgs& a, int64_t gx_fixed, hipStream_t st) {
  if (dt == DType::F32) return launch_any<float, MODE>(a, gx_fixed, st);
  return launch_any<uint16_t, MODE>(a, gx_fixed, st);
}

}  // namespace

int bn_reduce_blocks(int64_t N) {
  // ~1024 row-group blocks: enough to fill 256 CUs; partials stay small (1024 x 2F fp32)
  int64_t b = (N + 31) / 32;
  return static_cast<int>(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

// dropout parameters of a fused BN pass: keep probability 1 - p, 64-bit seed
static void set_dropout(BNArgs& a, float p, uint64_t seed) {
  if (p > 0.f && p < 1.f) {
    const double t = static_cast<double>(p) * 4294967296.0;
    a.drop_thresh = t >= 4294967295.0 ? 4294967295u : static_cast<uint32_t>(t < 1.0 ? 1.0 : t);
    a.keep_scale = 1.f / (1.f - p);
  } else {
    a.drop_thresh = 0;
    a.keep_scale = 1.f;
  }
  a.seed_lo = static_cast<uint32_t>(seed);
  a.seed_hi = static_cast<uint32_t>(seed >> 32);
}

hipError_t bn_reduce(DType dt, int mode, const void* x, int64_t ldx, const void* dy,
                     int64_t ldy, int64_t N, int F, const float* shift_or_mean,
                     const float* rstd, const float* gamma, const float* beta, bool relu,
                     float* partial, int nblocks, double* out, hipStream_t st, float drop_p,
                     uint64_t seed) {
  if (F <= 0) return hipSuccess;
  BNArgs a{x, ldx, dy, ldy, nullptr, 0, N < 0 ? 0 : N, F, shift_or_mean, rstd, gamma, beta,
           nullptr, nullptr, partial, relu, 0, 1.f, 0, 0};
  if (mode == 1) set_dropout(a, drop_p, seed);
  hipError_t e = mode == 0 ? dispatch<0>(dt, a, nblocks, st) : dispatch<1>(dt, a, nblocks, st);
  if (e != hipSuccess) return e;
  const int n2 = 2 * F;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((n2 + 255) / 256), dim3(256), 0, st, partial,
                     nblocks, F, out);
  return hipGetLastError();
}

hipError_t bn_apply(DType dt, int mode, const void* x, int64_t ldx, const void* dy,
                    int64_t ldy, void* out, int64_t ldo, int64_t N, int F, const float* mean,
                    const float* rstd, const float* gamma, const float* beta, const float* c1,
                    const float* c2, bool relu, hipStream_t st, float drop_p, uint64_t seed) {
  if (N <= 0 || F <= 0) return hipSuccess;
  BNArgs a{x, ldx, dy, ldy, out, ldo, N, F, mean, rstd, gamma, beta, c1, c2, nullptr, relu,
           0, 1.f, 0, 0};
  set_dropout(a, drop_p, seed);
  return mode == 0 ? dispatch<2>(dt, a, 0, st) : dispatch<3>(dt, a, 0, st);
}

}  // namespace dgraph
