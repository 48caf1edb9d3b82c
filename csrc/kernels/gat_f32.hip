// dgraph_amd — fused fp32 graph-attention aggregation for gfx950 (the RGAT relation layer).
//
// The reference computes a relation's attention with per-EDGE tensors: gather h_i and h_j
// into [E, C] buffers, concatenate to [E, 2C], a linear layer, exp, a scatter-sum for the
// denominator, a gather back to the edges, a divide, a multiply and a scatter-sum
// (experiments/OGB-LSC/RGAT.py:108-206) — ~8 passes over E x C memory, no max subtraction.
// Here one relation is three row-parallel kernels and no per-edge feature tensor:
//
//   e_ij  = leaky_relu(sd[i, k] + ss[j, k])          (per head k; sd/ss: the two halves
//   alpha = softmax_j(e_ij)                            of the attention vector applied to
//   out_i += sum_j alpha_ij z_j[head k columns]        h_i / h_j, computed by the GEMMs)
//
// * gat_fwd: per destination row, a lane-parallel pass over the row's edges for the per-head
//   max and sum (reads 4 * HH bytes of ss per edge), then the gather pass of the SpMM with the
//   weights computed on the fly; writes the row's (max, sum) per head — alpha is never
//   stored.
// * gat_bwd_dst: per destination row, with g = dL/dout_i resident in registers: gathers z_j,
//   ga = <g^k, z_j^k> (head-segmented lane reduction), and accumulates
//   c = sum alpha ga, A = sum lambda alpha ga, B = sum lambda alpha  (lambda = leaky-ReLU
//   slope of the edge). dL/dsd_i = A - c B; c is kept for the source side.
// * gat_bwd_src: per SOURCE row over the transposed pattern, with z_j resident: gathers g_i,
//   recomputes alpha and ga, and accumulates dz_j = sum alpha g_i (the transposed SpMM)
//   and dss_j = sum lambda alpha (ga - c_i); adds dss_j * a_src (ss_j = z_j . a_src) to dz_j.
//
// Two sources (x for columns < nsplit, x2 for columns >= nsplit: local rows and received halo
// rows) as in spmm_f32.hip, so a rank's own transformed rows and its halo rows are never
// concatenated. Layout: one LPR-lane group per row (LPR = C / 4, 16-B fp32 vectors), the HH
// heads as contiguous lane blocks of LH = LPR / HH lanes. Fixed summation orders, no atomics:
// bitwise deterministic.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

constexpr int kU = 8;  // edges in flight per lane in the gather loops

struct GatArgs {
  const int64_t* rowptr;
  const void* col;
  int64_t nrows;
  int C;            // feature width (= 4 * LPR)
  float slope;      // leaky-ReLU negative slope
  int64_t lds;      // row stride (floats) of every per-head score / statistics array:
                    // heads for whole-row calls; the caller's heads for a one-head column
                    // pass over a slice of wider rows
  // operands
  const float* x;   // rows gathered (z for fwd / bwd_dst, g for bwd_src)
  int64_t ldx;
  const float* x2;  // second source (columns >= nsplit) or nullptr
  int64_t ldx2;
  int64_t nsplit;
  const float* ss;  // [*, HH] source scores (two sources like x: ss2 past nsplit)
  const float* ss2;
  const float* sd;  // [nrows or cols, HH] destination scores
  // fwd
  float* out;       // [nrows, C] (beta: add to it)
  int64_t ldo;
  float beta;
  float* stat_m;    // [nrows, HH]
  float* stat_l;
  // bwd_dst
  const float* g;   // [nrows, C] dL/dout rows
  int64_t ldg;
  float* c_out;     // [nrows, HH]
  float* gsd_out;   // [nrows, HH]
  // bwd_src (rows = sources; x = g of the destinations, z = this row's own features)
  const float* z;
  int64_t ldz;
  const float* ss_row;  // [nrows, HH] the source rows' own scores
  const float* m_dst;   // [dst rows, HH] statistics of the destinations
  const float* l_dst;
  const float* c_dst;
  const float* a_src;   // [C] attention vector (source half), flat over heads
  float* gz;            // [nrows, C]
  int64_t ldgz;
  float* gss;           // [nrows, HH] (nullable)
};

template <typename IdxT>
__device__ __forceinline__ int64_t load_col(const GatArgs& a, int64_t pos) {
  return static_cast<int64_t>(static_cast<const IdxT*>(a.col)[pos]);
}

__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }

// sum over the LH lanes of one head (contiguous, aligned lane blocks)
template <int LH>
__device__ __forceinline__ float head_sum(float v) {
#pragma unroll
  for (int off = LH / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// reduce over the LPR lanes of a row group
template <int LPR>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int off = LPR / 2; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = LPR / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
template <int LPR>
__device__ __forceinline__ int group_imax(int v) {
#pragma unroll
  for (int off = LPR; off < kWave; off <<= 1) {
    const int o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

// ------------------------------------------------------------------------------------ fwd
template <typename IdxT, int LPR, int HH>
__global__ __launch_bounds__(256) void gat_fwd_kernel(GatArgs a) {
  constexpr int G = kWave / LPR;
  constexpr int LH = LPR / HH;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, l = lane % LPR, hk = l / LH;
  const int f = 4 * l;
  const int64_t ngroups = (a.nrows + G - 1) / G;
  const int64_t q0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t qstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const uint32_t ns = static_cast<uint32_t>(a.nsplit);
  auto ssp = [&](int64_t c) -> const float* {
    return (a.ss2 && c >= ns) ? a.ss2 + (c - ns) * a.lds : a.ss + c * a.lds;
  };
  auto xrow = [&](int64_t c) -> const float* {
    return (a.x2 && c >= ns) ? a.x2 + (c - ns) * a.ldx2 + f : a.x + c * a.ldx + f;
  };
  for (int64_t q = q0; q < ngroups; q += qstep) {
    const int64_t r = q * G + g;
    const bool has_row = r < a.nrows;
    const int64_t s = has_row ? a.rowptr[r] : 0;
    const int deg = has_row ? static_cast<int>(a.rowptr[r + 1] - s) : 0;
    const int maxdeg = group_imax<LPR>(deg);
    float sd[HH];
#pragma unroll
    for (int k = 0; k < HH; ++k) sd[k] = has_row ? a.sd[r * a.lds + k] : 0.f;
    // pass A: per-head max, then sum of exp, lane-parallel over the row's edges
    float m[HH], lsum[HH];
#pragma unroll
    for (int k = 0; k < HH; ++k) m[k] = -INFINITY;
    for (int t = l; t < deg; t += LPR) {
      const float* sp = ssp(load_col<IdxT>(a, s + t));
#pragma unroll
      for (int k = 0; k < HH; ++k) m[k] = fmaxf(m[k], lrelu(sd[k] + sp[k], a.slope));
    }
#pragma unroll
    for (int k = 0; k < HH; ++k) {
      m[k] = group_max<LPR>(m[k]);
      lsum[k] = 0.f;
    }
    for (int t = l; t < deg; t += LPR) {
      const float* sp = ssp(load_col<IdxT>(a, s + t));
#pragma unroll
      for (int k = 0; k < HH; ++k) lsum[k] += __expf(lrelu(sd[k] + sp[k], a.slope) - m[k]);
    }
    float my_m = 0.f, my_inv = 0.f, my_sd = 0.f;
#pragma unroll
    for (int k = 0; k < HH; ++k) {
      lsum[k] = group_sum<LPR>(lsum[k]);
      if (k == hk) {
        my_m = m[k];
        my_inv = lsum[k] > 0.f ? 1.f / lsum[k] : 0.f;
        my_sd = sd[k];
      }
    }
    // pass B: the weighted gather (edges sequential, kU rows in flight)
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k0 = 0; k0 < maxdeg; k0 += LPR) {
      const int kk = k0 + l;
      const int64_t my_c = kk < deg ? load_col<IdxT>(a, s + kk) : 0;
      for (int j0 = 0; j0 < LPR && k0 + j0 < maxdeg; j0 += kU) {
        float4 v[kU];
        float w[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = j0 + u;
          const int64_t c = __shfl(my_c, g * LPR + (j < LPR ? j : 0), kWave);
          const bool ok = j < LPR && k0 + j < deg;
          v[u] = *reinterpret_cast<const float4*>(xrow(ok ? c : 0));
          const float e = lrelu(my_sd + ssp(ok ? c : 0)[hk], a.slope);
          w[u] = ok ? __expf(e - my_m) * my_inv : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          acc.x = fmaf(w[u], v[u].x, acc.x);
          acc.y = fmaf(w[u], v[u].y, acc.y);
          acc.z = fmaf(w[u], v[u].z, acc.z);
          acc.w = fmaf(w[u], v[u].w, acc.w);
        }
      }
    }
    if (!has_row) continue;
    float* o = a.out + r * a.ldo + f;
    if (a.beta != 0.f) {
      const float4 old = *reinterpret_cast<const float4*>(o);
      acc.x = fmaf(a.beta, old.x, acc.x);
      acc.y = fmaf(a.beta, old.y, acc.y);
      acc.z = fmaf(a.beta, old.z, acc.z);
      acc.w = fmaf(a.beta, old.w, acc.w);
    }
    *reinterpret_cast<float4*>(o) = acc;
    if (l % LH == 0) {
      a.stat_m[r * a.lds + hk] = my_m;
      a.stat_l[r * a.lds + hk] = my_inv;  // 1 / sum (0 for an isolated row)
    }
  }
}

// -------------------------------------------------------------------------------- bwd dst
template <typename IdxT, int LPR, int HH>
__global__ __launch_bounds__(256) void gat_bwd_dst_kernel(GatArgs a) {
  constexpr int G = kWave / LPR;
  constexpr int LH = LPR / HH;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, l = lane % LPR, hk = l / LH;
  const int f = 4 * l;
  const int64_t ngroups = (a.nrows + G - 1) / G;
  const int64_t q0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t qstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const uint32_t ns = static_cast<uint32_t>(a.nsplit);
  auto ssp = [&](int64_t c) -> const float* {
    return (a.ss2 && c >= ns) ? a.ss2 + (c - ns) * a.lds : a.ss + c * a.lds;
  };
  auto xrow = [&](int64_t c) -> const float* {
    return (a.x2 && c >= ns) ? a.x2 + (c - ns) * a.ldx2 + f : a.x + c * a.ldx + f;
  };
  for (int64_t q = q0; q < ngroups; q += qstep) {
    const int64_t r = q * G + g;
    const bool has_row = r < a.nrows;
    const int64_t rr = has_row ? r : 0;
    const int64_t s = has_row ? a.rowptr[r] : 0;
    const int deg = has_row ? static_cast<int>(a.rowptr[r + 1] - s) : 0;
    const int maxdeg = group_imax<LPR>(deg);
    const float4 gv = *reinterpret_cast<const float4*>(a.g + rr * a.ldg + f);
    const float my_sd = a.sd[rr * a.lds + hk];
    const float my_m = a.stat_m[rr * a.lds + hk];
    const float my_inv = a.stat_l[rr * a.lds + hk];
    float cacc = 0.f, aacc = 0.f, bacc = 0.f;
    for (int k0 = 0; k0 < maxdeg; k0 += LPR) {
      const int kk = k0 + l;
      const int64_t my_c = kk < deg ? load_col<IdxT>(a, s + kk) : 0;
      for (int j0 = 0; j0 < LPR && k0 + j0 < maxdeg; j0 += kU) {
        float4 v[kU];
        float e[kU];
        bool ok[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = j0 + u;
          const int64_t c = __shfl(my_c, g * LPR + (j < LPR ? j : 0), kWave);
          ok[u] = j < LPR && k0 + j < deg;
          v[u] = *reinterpret_cast<const float4*>(xrow(ok[u] ? c : 0));
          e[u] = my_sd + ssp(ok[u] ? c : 0)[hk];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          float p = gv.x * v[u].x;
          p = fmaf(gv.y, v[u].y, p);
          p = fmaf(gv.z, v[u].z, p);
          p = fmaf(gv.w, v[u].w, p);
          p = head_sum<LH>(p);
          const float lam = e[u] > 0.f ? 1.f : a.slope;
          const float al = ok[u] ? __expf(lrelu(e[u], a.slope) - my_m) * my_inv : 0.f;
          cacc = fmaf(al, p, cacc);
          aacc = fmaf(lam * al, p, aacc);
          bacc = fmaf(lam, al, bacc);
        }
      }
    }
    if (has_row && l % LH == 0) {
      a.c_out[r * a.lds + hk] = cacc;
      a.gsd_out[r * a.lds + hk] = aacc - cacc * bacc;
    }
  }
}

// -------------------------------------------------------------------------------- bwd src
template <typename IdxT, int LPR, int HH>
__global__ __launch_bounds__(256) void gat_bwd_src_kernel(GatArgs a) {
  constexpr int G = kWave / LPR;
  constexpr int LH = LPR / HH;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR, l = lane % LPR, hk = l / LH;
  const int f = 4 * l;
  const int64_t ngroups = (a.nrows + G - 1) / G;
  const int64_t q0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t qstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const float4 av = *reinterpret_cast<const float4*>(a.a_src + f);
  for (int64_t q = q0; q < ngroups; q += qstep) {
    const int64_t r = q * G + g;
    const bool has_row = r < a.nrows;
    const int64_t rr = has_row ? r : 0;
    const int64_t s = has_row ? a.rowptr[r] : 0;
    const int deg = has_row ? static_cast<int>(a.rowptr[r + 1] - s) : 0;
    const int maxdeg = group_imax<LPR>(deg);
    const float4 zv = *reinterpret_cast<const float4*>(a.z + rr * a.ldz + f);
    const float my_ss = a.ss_row[rr * a.lds + hk];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    float gss = 0.f;
    for (int k0 = 0; k0 < maxdeg; k0 += LPR) {
      const int kk = k0 + l;
      const int64_t my_i = kk < deg ? load_col<IdxT>(a, s + kk) : 0;
      for (int j0 = 0; j0 < LPR && k0 + j0 < maxdeg; j0 += kU) {
        float4 v[kU];
        float e[kU], m[kU], il[kU], c[kU];
        bool ok[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = j0 + u;
          const int64_t i = __shfl(my_i, g * LPR + (j < LPR ? j : 0), kWave);
          ok[u] = j < LPR && k0 + j < deg;
          const int64_t ii = ok[u] ? i : 0;
          v[u] = *reinterpret_cast<const float4*>(a.x + ii * a.ldx + f);
          e[u] = a.sd[ii * a.lds + hk] + my_ss;
          m[u] = a.m_dst[ii * a.lds + hk];
          il[u] = a.l_dst[ii * a.lds + hk];
          c[u] = a.c_dst[ii * a.lds + hk];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          float p = v[u].x * zv.x;
          p = fmaf(v[u].y, zv.y, p);
          p = fmaf(v[u].z, zv.z, p);
          p = fmaf(v[u].w, zv.w, p);
          p = head_sum<LH>(p);
          const float lam = e[u] > 0.f ? 1.f : a.slope;
          const float al = ok[u] ? __expf(lrelu(e[u], a.slope) - m[u]) * il[u] : 0.f;
          acc.x = fmaf(al, v[u].x, acc.x);
          acc.y = fmaf(al, v[u].y, acc.y);
          acc.z = fmaf(al, v[u].z, acc.z);
          acc.w = fmaf(al, v[u].w, acc.w);
          gss = fmaf(lam * al, p - c[u], gss);
        }
      }
    }
    if (!has_row) continue;
    // ss_j = z_j . a_src (per head): its gradient flows back into z_j
    acc.x = fmaf(gss, av.x, acc.x);
    acc.y = fmaf(gss, av.y, acc.y);
    acc.z = fmaf(gss, av.z, acc.z);
    acc.w = fmaf(gss, av.w, acc.w);
    *reinterpret_cast<float4*>(a.gz + r * a.ldgz + f) = acc;
    if (a.gss && l % LH == 0) a.gss[r * a.lds + hk] = gss;
  }
}

template <int KIND, typename IdxT, int LPR, int HH>
void launch_one(const GatArgs& a, int64_t blocks, hipStream_t st) {
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
  if constexpr (KIND == 0)
    hipLaunchKernelGGL((gat_fwd_kernel<IdxT, LPR, HH>), grid, block, 0, st, a);
  else if constexpr (KIND == 1)
    hipLaunchKernelGGL((gat_bwd_dst_kernel<IdxT, LPR, HH>), grid, block, 0, st, a);
  else
    hipLaunchKernelGGL((gat_bwd_src_kernel<IdxT, LPR, HH>), grid, block, 0, st, a);
}

template <int KIND, typename IdxT>
hipError_t launch_kind(const GatArgs& a, int heads, hipStream_t st) {
  const int LPR = a.C / 4;
  const int64_t G = kWave / LPR;
  const int64_t ngroups = (a.nrows + G - 1) / G;
  int64_t blocks = (ngroups + 3) / 4;  // one row group per wave, in order
  if (blocks < 1) blocks = 1;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
#define DG_GAT(L_, H_)                                   \
  if (LPR == L_ && heads == H_) {                        \
    launch_one<KIND, IdxT, L_, H_>(a, blocks, st);       \
    return hipGetLastError();                            \
  }
  DG_GAT(16, 1) DG_GAT(16, 2) DG_GAT(16, 4) DG_GAT(16, 8)
  DG_GAT(32, 1) DG_GAT(32, 2) DG_GAT(32, 4) DG_GAT(32, 8)
  DG_GAT(64, 1) DG_GAT(64, 2) DG_GAT(64, 4) DG_GAT(64, 8)
#undef DG_GAT
  return hipErrorInvalidValue;
}

template <int KIND>
hipError_t launch(const GatArgs& a, IType it, int heads, hipStream_t st) {
  if (a.nrows <= 0) return hipSuccess;
  if (a.C != 64 && a.C != 128 && a.C != 256) return hipErrorInvalidValue;
  return it == IType::I32 ? launch_kind<KIND, int32_t>(a, heads, st)
                          : launch_kind<KIND, int64_t>(a, heads, st);
}

}  // namespace

bool gat_f32_shape_ok(int C, int heads) {
  if (C != 64 && C != 128 && C != 256) return false;
  if (heads != 1 && heads != 2 && heads != 4 && heads != 8) return false;
  return (C / 4) / heads >= 2;  // at least two lanes per head
}

hipError_t gat_fwd_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows, int C,
                       int heads, int64_t lds, float slope, const float* x, int64_t ldx, const float* x2,
                       int64_t ldx2, int64_t nsplit, const float* ss, const float* ss2,
                       const float* sd, float* out, int64_t ldo, float beta, float* stat_m,
                       float* stat_l, hipStream_t st) {
  GatArgs a{};
  a.rowptr = rowptr;
  a.col = col;
  a.nrows = nrows;
  a.C = C;
  a.lds = lds;
  a.slope = slope;
  a.x = x;
  a.ldx = ldx;
  a.x2 = x2;
  a.ldx2 = ldx2;
  a.nsplit = nsplit;
  a.ss = ss;
  a.ss2 = ss2;
  a.sd = sd;
  a.out = out;
  a.ldo = ldo;
  a.beta = beta;
  a.stat_m = stat_m;
  a.stat_l = stat_l;
  return launch<0>(a, it, heads, st);
}

hipError_t gat_bwd_dst_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows,
                           int C, int heads, int64_t lds, float slope, const float* x, int64_t ldx,
                           const float* x2, int64_t ldx2, int64_t nsplit, const float* ss,
                           const float* ss2, const float* sd, const float* stat_m,
                           const float* stat_l, const float* g, int64_t ldg, float* c_out,
                           float* gsd_out, hipStream_t st) {
  GatArgs a{};
  a.rowptr = rowptr;
  a.col = col;
  a.nrows = nrows;
  a.C = C;
  a.lds = lds;
  a.slope = slope;
  a.x = x;
  a.ldx = ldx;
  a.x2 = x2;
  a.ldx2 = ldx2;
  a.nsplit = nsplit;
  a.ss = ss;
  a.ss2 = ss2;
  a.sd = sd;
  a.stat_m = const_cast<float*>(stat_m);
  a.stat_l = const_cast<float*>(stat_l);
  a.g = g;
  a.ldg = ldg;
  a.c_out = c_out;
  a.gsd_out = gsd_out;
  return launch<1>(a, it, heads, st);
}

hipError_t gat_bwd_src_f32(IType it, const int64_t* rowptr, const void* col, int64_t nrows,
                           int C, int heads, int64_t lds, float slope, const float* g, int64_t ldg,
                           const float* z, int64_t ldz, const float* ss_row, const float* sd,
                           const float* m_dst, const float* l_dst, const float* c_dst,
                           const float* a_src, float* gz, int64_t ldgz, float* gss,
                           hipStream_t st) {
  GatArgs a{};
  a.rowptr = rowptr;
  a.col = col;
  a.nrows = nrows;
  a.C = C;
  a.lds = lds;
  a.slope = slope;
  a.x = g;
  a.ldx = ldg;
  a.z = z;
  a.ldz = ldz;
  a.ss_row = ss_row;
  a.sd = sd;
  a.m_dst = m_dst;
  a.l_dst = l_dst;
  a.c_dst = c_dst;
  a.a_src = a_src;
  a.gz = gz;
  a.ldgz = ldgz;
  a.gss = gss;
  return launch<2>(a, it, heads, st);
}

}  // namespace dgraph
