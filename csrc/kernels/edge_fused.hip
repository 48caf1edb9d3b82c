// dgraph_amd — fused edge-MLP kernels (K-new-6).
//
// The reference materialises per-edge concatenations and runs a GEMM on them:
//   GCN    m_ij = ReLU(W [x_i || x_j] + b),  out_i = sum_j m_ij         (GCN.py:43-65)
//   GraphCast / RGAT edge MLPs  act(W [e_ij || x_src || x_dst] + b)      (layers.py:205-215)
// The first Linear of such an MLP distributes over the concatenation:
//   W [x_i || x_j] + b = P[i] + Q[j]   with  P = x W_i^T + b,  Q = x W_j^T
// so the E x 2F concat and the E-row GEMM become two V-row GEMMs (MFMA, hipBLASLt) plus
// the gather-bound kernels below, which never write per-edge intermediates for GCN:
//
//   pair_relu_agg   (CSR by destination row i)
//       out[i] = sum_{j in N(i)} relu(P[i] + Q[j])                      (forward)
//   pair_relu_cnt   (same CSR)
//       dP[i]  = g[i] * #{j in N(i) : P[i] + Q[j] > 0}                 (backward, dP)
//   pair_relu_tgrad (transposed CSR: row j, neighbours i)
//       dQ[j]  = sum_{i : j in N(i)} g[i] * [P[i] + Q[j] > 0]          (backward, dQ)
//   gather_add_act  (edge-parallel, for MLPs with more layers)
//       h[e]   = act(Y[e] + P[src[e]] + Q[dst[e]])  act in {none, relu, silu, leaky 0.2}
//   gather_add_act_bwd
//       d[e]   = g[e] * act'(Y[e] + P[src[e]] + Q[dst[e]])  (pre-activation recomputed)
//
// Layout: one wavefront per CSR row (LPR lanes x VEC features per lane group, 64/LPR
// neighbours in flight per step, 4x unrolled); fp32 accumulation; bf16 or fp32 storage;
// deterministic (fixed neighbour order, xor-butterfly combine, no atomics).
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

enum PairMode : int { kAgg = 0, kCnt = 1, kTGrad = 2 };

template <typename T, typename IdxT, int VEC, int LPR, int MODE>
__global__ __launch_bounds__(256) void pair_relu_kernel(
    const int64_t* __restrict__ rowptr, const IdxT* __restrict__ col,
    const T* __restrict__ rowterm, int64_t ldr,   // P (agg/cnt) or Q (tgrad), by row
    const T* __restrict__ gat, int64_t ldg,       // Q (agg/cnt) or P (tgrad), gathered
    const T* __restrict__ gat2, int64_t ldg2,     // g (tgrad), gathered
    const T* __restrict__ rowmul, int64_t ldm,    // g (cnt), by row
    T* __restrict__ out, int64_t ldo, int64_t nrows, int F) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t s = rowptr[r];
    const int64_t e = rowptr[r + 1];
    for (int fc = 0; fc < F; fc += LPR * VEC) {
      const int f = fc + l * VEC;
      const bool active = f < F;
      float a[VEC], acc[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
      if (active) load_vec_f32<T, VEC>(rowterm + r * ldr + f, a);
      int64_t j = s + g;
      for (; j + 3 * G < e; j += 4 * G) {
        int64_t c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = static_cast<int64_t>(col[j + u * G]);
        if (active) {
          float v[4][VEC];
#pragma unroll
          for (int u = 0; u < 4; ++u) load_vec_f32<T, VEC>(gat + c[u] * ldg + f, v[u]);
          if constexpr (MODE == kTGrad) {
            float w[4][VEC];
#pragma unroll
            for (int u = 0; u < 4; ++u) load_vec_f32<T, VEC>(gat2 + c[u] * ldg2 + f, w[u]);
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int i = 0; i < VEC; ++i) acc[i] += (a[i] + v[u][i] > 0.f) ? w[u][i] : 0.f;
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int i = 0; i < VEC; ++i) {
                const float p = a[i] + v[u][i];
                if constexpr (MODE == kAgg) acc[i] += fmaxf(p, 0.f);
                else acc[i] += (p > 0.f) ? 1.f : 0.f;
              }
          }
        }
      }
      for (; j < e; j += G) {
        const int64_t c0 = static_cast<int64_t>(col[j]);
        if (active) {
          float v[VEC];
          load_vec_f32<T, VEC>(gat + c0 * ldg + f, v);
          if constexpr (MODE == kTGrad) {
            float w[VEC];
            load_vec_f32<T, VEC>(gat2 + c0 * ldg2 + f, w);
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[i] += (a[i] + v[i] > 0.f) ? w[i] : 0.f;
          } else {
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
              const float p = a[i] + v[i];
              if constexpr (MODE == kAgg) acc[i] += fmaxf(p, 0.f);
              else acc[i] += (p > 0.f) ? 1.f : 0.f;
            }
          }
        }
      }
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += __shfl_xor(acc[i], off, kWave);
      if (g == 0 && active) {
        if constexpr (MODE == kCnt) {
          float m[VEC];
          load_vec_f32<T, VEC>(rowmul + r * ldm + f, m);
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] *= m[i];
        }
        store_vec_f32<T, VEC>(out + r * ldo + f, acc);
      }
    }
  }
}

__device__ __forceinline__ float act_fwd(float x, int act) {
  if (act == 1) return fmaxf(x, 0.f);
  if (act == 3) return x > 0.f ? x : 0.2f * x;
  if (act == 2) return x / (1.f + __expf(-x));
  return x;
}
__device__ __forceinline__ float act_grad(float x, int act) {
  if (act == 1) return x > 0.f ? 1.f : 0.f;
  if (act == 3) return x > 0.f ? 1.f : 0.2f;
  if (act == 2) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
  return 1.f;
}

// BWD == false: out[e] = act(Y[e] + P[src[e]] + Q[dst[e]])
// BWD == true : out[e] = gin[e] * act'(Y[e] + P[src[e]] + Q[dst[e]])
template <typename T, int VEC, int LPR, bool BWD>
__global__ __launch_bounds__(256) void gather_add_act_kernel(
    const T* __restrict__ Y, int64_t ldy, const T* __restrict__ P, int64_t ldp,
    const int64_t* __restrict__ src, const T* __restrict__ Q, int64_t ldq,
    const int64_t* __restrict__ dst, const T* __restrict__ gin, int64_t ldgi,
    T* __restrict__ out, int64_t ldo, int64_t E, int F, int act) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  for (int64_t base = wave * G; base < E; base += nwaves * G) {
    const int64_t e = base + g;
    if (e >= E) continue;
    const int64_t sp = P ? src[e] : 0;
    const int64_t dq = Q ? dst[e] : 0;
    for (int f = l * VEC; f < F; f += LPR * VEC) {
      float acc[VEC], t[VEC];
      if (Y) {
        load_vec_f32<T, VEC>(Y + e * ldy + f, acc);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
      }
      if (P) {
        load_vec_f32<T, VEC>(P + sp * ldp + f, t);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += t[i];
      }
      if (Q) {
        load_vec_f32<T, VEC>(Q + dq * ldq + f, t);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += t[i];
      }
      if constexpr (BWD) {
        load_vec_f32<T, VEC>(gin + e * ldgi + f, t);
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = t[i] * act_grad(acc[i], act);
      } else {
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] = act_fwd(acc[i], act);
      }
      store_vec_f32<T, VEC>(out + e * ldo + f, acc);
    }
  }
}

inline int lanes_for(int F, int vec) {
  const int need = (F + vec - 1) / vec;
  return need <= 4 ? 4 : need <= 8 ? 8 : need <= 16 ? 16 : need <= 32 ? 32 : 64;
}

template <typename T>
int pick_vec(int F, std::initializer_list<int64_t> lds, std::initializer_list<const void*> ptrs) {
  constexpr int V = 16 / sizeof(T);
  bool ok = F % V == 0;
  for (auto ld : lds) ok = ok && (ld % V == 0);
  for (auto p : ptrs) ok = ok && (reinterpret_cast<uintptr_t>(p) % 16 == 0);
  return ok ? V : 1;
}

template <typename T, typename IdxT, int MODE>
hipError_t launch_pair(const int64_t* rowptr, const IdxT* col, const T* R, int64_t ldr,
                       const T* X, int64_t ldx, const T* X2, int64_t ldx2, const T* M,
                       int64_t ldm, T* out, int64_t ldo, int64_t nrows, int F, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const int vec = pick_vec<T>(F, {ldr, ldx, ldx2 ? ldx2 : V, ldm ? ldm : V, ldo},
                              {R, X, X2 ? X2 : out, M ? M : out, out});
  const int lpr = lanes_for(F, vec);
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((nrows + 3) / 4, 256 * 64)));
#define DG_PAIR(VV, L)                                                                    \
  hipLaunchKernelGGL((pair_relu_kernel<T, IdxT, VV, L, MODE>), grid, block, 0, st, rowptr, \
                     col, R, ldr, X, ldx, X2, ldx2, M, ldm, out, ldo, nrows, F)
#define DG_PAIR_L(VV)                 \
  switch (lpr) {                      \
    case 4: DG_PAIR(VV, 4); break;    \
    case 8: DG_PAIR(VV, 8); break;    \
    case 16: DG_PAIR(VV, 16); break;  \
    case 32: DG_PAIR(VV, 32); break;  \
    default: DG_PAIR(VV, 64); break;  \
  }
  if (vec == V) { DG_PAIR_L(V) } else { DG_PAIR_L(1) }
#undef DG_PAIR_L
#undef DG_PAIR
  return hipGetLastError();
}

template <typename T, bool BWD>
hipError_t launch_gaa(const T* Y, int64_t ldy, const T* P, int64_t ldp, const int64_t* src,
                      const T* Q, int64_t ldq, const int64_t* dst, const T* gin, int64_t ldgi,
                      T* out, int64_t ldo, int64_t E, int F, int act, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const int vec = pick_vec<T>(F, {Y ? ldy : V, P ? ldp : V, Q ? ldq : V, gin ? ldgi : V, ldo},
                              {Y ? Y : out, P ? P : out, Q ? Q : out, gin ? gin : out, out});
  const int lpr = lanes_for(F, vec);
  const int64_t G = kWave / lpr;
  dim3 block(256), grid(static_cast<unsigned>(cap_blocks((E + 4 * G - 1) / (4 * G), 256 * 64)));
#define DG_GAA(VV, L)                                                                       \
  hipLaunchKernelGGL((gather_add_act_kernel<T, VV, L, BWD>), grid, block, 0, st, Y, ldy, P, \
                     ldp, src, Q, ldq, dst, gin, ldgi, out, ldo, E, F, act)
#define DG_GAA_L(VV)                 \
  switch (lpr) {                     \
    case 4: DG_GAA(VV, 4); break;    \
    case 8: DG_GAA(VV, 8); break;    \
    case 16: DG_GAA(VV, 16); break;  \
    case 32: DG_GAA(VV, 32); break;  \
    default: DG_GAA(VV, 64); break;  \
  }
  if (vec == V) { DG_GAA_L(V) } else { DG_GAA_L(1) }
#undef DG_GAA_L
#undef DG_GAA
  return hipGetLastError();
}

template <typename T>
hipError_t pair_dispatch(IType it, int mode, const int64_t* rowptr, const void* col,
                         const void* R, int64_t ldr, const void* X, int64_t ldx, const void* X2,
                         int64_t ldx2, const void* M, int64_t ldm, void* out, int64_t ldo,
                         int64_t nrows, int F, hipStream_t st) {
  auto r = static_cast<const T*>(R);
  auto x = static_cast<const T*>(X);
  auto x2 = static_cast<const T*>(X2);
  auto m = static_cast<const T*>(M);
  auto o = static_cast<T*>(out);
#define DG_PD(IDX)                                                                           \
  switch (mode) {                                                                            \
    case kAgg:                                                                               \
      return launch_pair<T, IDX, kAgg>(rowptr, static_cast<const IDX*>(col), r, ldr, x, ldx, \
                                       x2, ldx2, m, ldm, o, ldo, nrows, F, st);             \
    case kCnt:                                                                               \
      return launch_pair<T, IDX, kCnt>(rowptr, static_cast<const IDX*>(col), r, ldr, x, ldx, \
                                       x2, ldx2, m, ldm, o, ldo, nrows, F, st);             \
    default:                                                                                 \
      return launch_pair<T, IDX, kTGrad>(rowptr, static_cast<const IDX*>(col), r, ldr, x,    \
                                         ldx, x2, ldx2, m, ldm, o, ldo, nrows, F, st);      \
  }
  if (it == IType::I32) { DG_PD(int32_t) } else { DG_PD(int64_t) }
#undef DG_PD
}

}  // namespace

hipError_t pair_relu(DType dt, IType it, int mode, const int64_t* rowptr, const void* col,
                     const void* rowterm, int64_t ldr, const void* gat, int64_t ldg,
                     const void* gat2, int64_t ldg2, const void* rowmul, int64_t ldm, void* out,
                     int64_t ldo, int64_t nrows, int F, hipStream_t st) {
  if (nrows <= 0 || F <= 0) return hipSuccess;
  if (dt == DType::F32)
    return pair_dispatch<float>(it, mode, rowptr, col, rowterm, ldr, gat, ldg, gat2, ldg2,
                                rowmul, ldm, out, ldo, nrows, F, st);
  return pair_dispatch<uint16_t>(it, mode, rowptr, col, rowterm, ldr, gat, ldg, gat2, ldg2,
                                 rowmul, ldm, out, ldo, nrows, F, st);
}

hipError_t gather_add_act(DType dt, bool bwd, const void* Y, int64_t ldy, const void* P,
                          int64_t ldp, const int64_t* src, const void* Q, int64_t ldq,
                          const int64_t* dst, const void* gin, int64_t ldgi, void* out,
                          int64_t ldo, int64_t E, int F, int act, hipStream_t st) {
  if (E <= 0 || F <= 0) return hipSuccess;
#define DG_G(T)                                                                               \
  {                                                                                           \
    auto y = static_cast<const T*>(Y);                                                        \
    auto p = static_cast<const T*>(P);                                                        \
    auto q = static_cast<const T*>(Q);                                                        \
    auto gi = static_cast<const T*>(gin);                                                     \
    auto o = static_cast<T*>(out);                                                            \
    return bwd ? launch_gaa<T, true>(y, ldy, p, ldp, src, q, ldq, dst, gi, ldgi, o, ldo, E, F, \
                                     act, st)                                                 \
               : launch_gaa<T, false>(y, ldy, p, ldp, src, q, ldq, dst, gi, ldgi, o, ldo, E,  \
                                      F, act, st);                                            \
  }
  if (dt == DType::F32) DG_G(float)
  DG_G(uint16_t)
#undef DG_G
}

}  // namespace dgraph
