// dgraph_amd — CSR SpMM / segment-sum aggregation for gfx950 (K-new-2).
//
// Replaces the reference's scatter_add-based aggregation (GCN.py:57-65,
// _torch_func_impl.py:222-227, RankLocalOps.py:148-206 with its atomic float4 path)
// by a destination-sorted, atomic-free segment reduction:
//   * one wavefront (64 lanes) owns an output row; the wave is split into
//     G = 64/LPR lane groups, each group streams every G-th neighbour row with
//     VEC-wide (up to 16 B) loads, so a wave keeps 4*G neighbour rows in flight;
//   * accumulation is fp32 in VGPRs, the G partial sums are combined with
//     cross-lane xor shuffles (fixed order => bitwise deterministic);
//   * the result is written once with a row scale (mean = 1/deg) and optional
//     beta*out accumulate (used to add the halo part after the interior part).
// The kernel is HBM/Infinity-Cache bandwidth bound (random row gathers), so the
// target is bytes/s, not FLOP/s (see profiles/).
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

template <typename T, typename IdxT, int VEC, int LPR>
__global__ __launch_bounds__(256) void spmm_csr_kernel(
    const int64_t* __restrict__ rowptr, const IdxT* __restrict__ col,
    const float* __restrict__ ew, int heads, int head_dim,
    const float* __restrict__ col_scale, const float* __restrict__ row_scale,
    const T* __restrict__ x, int64_t ldx, T* __restrict__ out, int64_t ldo,
    int64_t nrows, int F, float beta) {
  constexpr int G = kWave / LPR;  // lane groups per wave = neighbour rows per step
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
      const int h = (heads > 1) ? (f / head_dim) : 0;
      float acc[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = 0.f;

      int64_t j = s + g;
      // Main loop: 4 neighbour rows per lane group in flight.
      for (; j + 3 * G < e; j += 4 * G) {
        int64_t c[4];
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) c[u] = static_cast<int64_t>(col[j + u * G]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float wu = ew ? ew[(j + u * G) * heads + h] : 1.f;
          if (col_scale) wu *= col_scale[c[u]];
          w[u] = wu;
        }
        if (active) {
          float v[4][VEC];
#pragma unroll
          for (int u = 0; u < 4; ++u) load_vec_f32<T, VEC>(x + c[u] * ldx + f, v[u]);
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < VEC; ++i) acc[i] = fmaf(w[u], v[u][i], acc[i]);
        }
      }
      for (; j < e; j += G) {
        const int64_t c0 = static_cast<int64_t>(col[j]);
        float w0 = ew ? ew[j * heads + h] : 1.f;
        if (col_scale) w0 *= col_scale[c0];
        if (active) {
          float v[VEC];
          load_vec_f32<T, VEC>(x + c0 * ldx + f, v);
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] = fmaf(w0, v[i], acc[i]);
        }
      }
      // Combine the G lane groups (xor butterfly over the group index bits).
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += __shfl_xor(acc[i], off, kWave);

      if (g == 0 && active) {
        const float rs = row_scale ? row_scale[r] : 1.f;
        T* o = out + r * ldo + f;
        if (beta != 0.f) {
          float old[VEC];
          load_vec_f32<T, VEC>(o, old);
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] = fmaf(acc[i], rs, beta * old[i]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] *= rs;
        }
        store_vec_f32<T, VEC>(o, acc);
      }
    }
  }
}

// v2: the wave loads up to 64 (col, weight) pairs of its row with ONE coalesced load
// (lane j <- slot base+j) and broadcasts them to the lane groups with ds_bpermute
// shuffles, so the neighbour-row loads no longer wait on a per-group dependent index
// load; U neighbour rows per lane group in flight. Optional XCD-aware row mapping: the
// rows are cut into 8 contiguous chunks, chunk x served by the blocks that share XCD x
// (blockIdx % 8), so each XCD's L2 sees one contiguous row window (speed only).
template <typename T, typename IdxT, int VEC, int LPR, int U, bool XCD>
__global__ __launch_bounds__(256) void spmm_csr_v2_kernel(
    const int64_t* __restrict__ rowptr, const IdxT* __restrict__ col,
    const float* __restrict__ ew, int heads, int head_dim,
    const float* __restrict__ col_scale, const float* __restrict__ row_scale,
    const T* __restrict__ x, int64_t ldx, T* __restrict__ out, int64_t ldo,
    int64_t nrows, int F, float beta) {
  constexpr int G = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int wpb = blockDim.x >> 6;
  int64_t r0, rstep, rend;
  if constexpr (XCD) {
    const int nx = 8;
    const int64_t bx = blockIdx.x % nx;
    const int64_t bpx = gridDim.x / nx;  // host guarantees gridDim.x % 8 == 0
    const int64_t chunk = (nrows + nx - 1) / nx;
    const int64_t lo = bx * chunk;
    rend = lo + chunk < nrows ? lo + chunk : nrows;
    r0 = lo + (blockIdx.x / nx) * wpb + (threadIdx.x >> 6);
    rstep = bpx * wpb;
  } else {
    r0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    rstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    rend = nrows;
  }
  const bool multi_head = heads > 1;
  for (int64_t r = r0; r < rend; r += rstep) {
    const int64_t s = rowptr[r];
    const int64_t e = rowptr[r + 1];
    for (int fc = 0; fc < F; fc += LPR * VEC) {
      const int f = fc + l * VEC;
      const bool active = f < F;
      const int h = multi_head ? (f / head_dim) : 0;
      float acc[VEC];
#pragma unroll
      for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
      for (int64_t base = s; base < e; base += kWave) {
        const int n = (e - base) < kWave ? static_cast<int>(e - base) : kWave;
        // cooperative index/weight load: lane j owns slot base + j
        IdxT my_c = 0;
        float my_w = 1.f;
        if (lane < n) {
          my_c = col[base + lane];
          if (col_scale) my_w = col_scale[my_c];
        }
        using R = typename RawVec<VEC * sizeof(T)>::type;
        // wave-uniform trip count: every lane stays active through the shuffles
        // (ds_bpermute cannot read a lane that has left the loop)
        for (int k0 = 0; k0 < n; k0 += G * U) {
          R v[U];  // raw (packed bf16) rows: half the VGPRs of an fp32 staging copy
          float w[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int kk = k0 + g + u * G;
            const int src = kk < n ? kk : 0;
            const int64_t c = static_cast<int64_t>(__shfl(my_c, src, kWave));
            // unconditional load (padding slots re-read slot 0 with weight 0; lanes past
            // F read column 0): a per-slot "load or zero" select makes hipcc branch
            // around each load and drain vmcnt per slot (guide §5 trap (c))
            v[u] = *reinterpret_cast<const R*>(x + c * ldx + (active ? f : 0));
          }
          // weights after the row loads are issued: the col_scale gather (a dependent
          // load of my_c) then overlaps the row gathers instead of gating them
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int kk = k0 + g + u * G;
            const int src = kk < n ? kk : 0;
            float wu = __shfl(my_w, src, kWave);
            if (ew) wu *= ew[(base + src) * heads + h];
            w[u] = kk < n ? wu : 0.f;
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const T* e = reinterpret_cast<const T*>(&v[u]);
            const bool ok = k0 + g + u * G < n;  // select, not a branch (inf*0 safe)
#pragma unroll
            for (int i = 0; i < VEC; ++i) {
              const float t = fmaf(w[u], Elem<T>::to_f32(e[i]), acc[i]);
              acc[i] = ok ? t : acc[i];
            }
          }
        }
      }
#pragma unroll
      for (int off = LPR; off < kWave; off <<= 1)
#pragma unroll
        for (int i = 0; i < VEC; ++i) acc[i] += __shfl_xor(acc[i], off, kWave);
      if (g == 0 && active) {
        const float rs = row_scale ? row_scale[r] : 1.f;
        T* o = out + r * ldo + f;
        if (beta != 0.f) {
          float old[VEC];
          load_vec_f32<T, VEC>(o, old);
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] = fmaf(acc[i], rs, beta * old[i]);
        } else {
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] *= rs;
        }
        store_vec_f32<T, VEC>(o, acc);
      }
    }
  }
}

int g_spmm_variant = 2;  // 1 = per-group index loads, 2 = cooperative + shuffles
// 0 = grid-stride, 1 = XCD-chunked grid-stride, 2 = XCD-chunked in-order (default),
// 3 = in-order without chunking. The in-order mappings keep the resident waves on a
// narrow advancing row window, so the neighbour rows they gather (which cluster near the
// row ids on locality-ordered graphs) are reused from the Infinity Cache: papers100M-
// shaped graph, F=256: 313 ms (1) -> 211 ms (2) (benchmarks/bench_spmm.py).
int g_spmm_xcd = 2;
int g_spmm_pass_cols = 128;  // bf16 rows wider than this run as column passes

template <typename T, typename IdxT, int VEC>
hipError_t launch_lpr(const int64_t* rowptr, const IdxT* col, const float* ew, int heads,
                      int head_dim, const float* cs, const float* rs, const T* x, int64_t ldx,
                      T* out, int64_t ldo, int64_t nrows, int F, float beta, hipStream_t st) {
  const int lanes_needed = (F + VEC - 1) / VEC;
  int64_t blocks = cap_blocks((nrows + 3) / 4, 256 * 32);
  if (g_spmm_xcd == 3) blocks = (nrows + 3) / 4;  // in-order, one row per wave, no chunking
  const bool xcd = (g_spmm_xcd == 1 || g_spmm_xcd == 2) && blocks >= 64;
  if (xcd) blocks = (blocks / 8) * 8;
  if (xcd && g_spmm_xcd == 2) {
    // in-order mapping: enough blocks that every wave owns ONE row of its XCD's chunk,
    // so each XCD's resident waves sweep a narrow, advancing row window (in dispatch
    // order) instead of a grid-stride spread over the whole chunk
    const int64_t chunk = (nrows + 7) / 8;
    blocks = 8 * ((chunk + 3) / 4);
  }
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
  if (g_spmm_variant == 2) {
    // U rows in flight per lane group: ~16 neighbour rows per wave
#define DG_V2(LPR_, U_)                                                                    \
  if (xcd)                                                                                 \
    hipLaunchKernelGGL((spmm_csr_v2_kernel<T, IdxT, VEC, LPR_, U_, true>), grid, block, 0, \
                       st, rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,     \
                       nrows, F, beta);                                                    \
  else                                                                                     \
    hipLaunchKernelGGL((spmm_csr_v2_kernel<T, IdxT, VEC, LPR_, U_, false>), grid, block,   \
                       0, st, rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,  \
                       nrows, F, beta);                                                    \
  return hipGetLastError();
    if (lanes_needed <= 4) { DG_V2(4, 2) }
    if (lanes_needed <= 8) { DG_V2(8, 2) }
    if (lanes_needed <= 16) { DG_V2(16, 4) }
    if (lanes_needed <= 32) { DG_V2(32, 8) }
    DG_V2(64, 8)
#undef DG_V2
  }
#define DG_SPMM_CASE(LPR_)                                                               \
  hipLaunchKernelGGL((spmm_csr_kernel<T, IdxT, VEC, LPR_>), grid, block, 0, st, rowptr, \
                     col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo, nrows, F, beta); \
  return hipGetLastError();
  if (lanes_needed <= 4) { DG_SPMM_CASE(4) }
  if (lanes_needed <= 8) { DG_SPMM_CASE(8) }
  if (lanes_needed <= 16) { DG_SPMM_CASE(16) }
  if (lanes_needed <= 32) { DG_SPMM_CASE(32) }
  DG_SPMM_CASE(64)
#undef DG_SPMM_CASE
}

inline bool aligned(const void* p, int bytes) {
  return (reinterpret_cast<uintptr_t>(p) % bytes) == 0;
}

template <typename T, typename IdxT>
hipError_t launch_vec(const int64_t* rowptr, const IdxT* col, const float* ew, int heads,
                      int head_dim, const float* cs, const float* rs, const T* x, int64_t ldx,
                      T* out, int64_t ldo, int64_t nrows, int F, float beta, hipStream_t st) {
  // Widest vector that divides the row, both leading dimensions, the head
  // size and both base pointers.
  constexpr int kMaxVec = 16 / sizeof(T);
  auto ok = [&](int v) {
    return F % v == 0 && ldx % v == 0 && ldo % v == 0 && (heads <= 1 || head_dim % v == 0) &&
           aligned(x, v * sizeof(T)) && aligned(out, v * sizeof(T));
  };
  if (ok(kMaxVec))
    return launch_lpr<T, IdxT, kMaxVec>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out,
                                        ldo, nrows, F, beta, st);
  if (ok(4))
    return launch_lpr<T, IdxT, 4>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,
                                  nrows, F, beta, st);
  return launch_lpr<T, IdxT, 1>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,
                                nrows, F, beta, st);
}

}  // namespace

void set_spmm_config(int variant, int xcd, int pass_cols) {
  if (variant == 1 || variant == 2) g_spmm_variant = variant;
  if (xcd >= 0 && xcd <= 3) g_spmm_xcd = xcd;
  if (pass_cols >= 0) g_spmm_pass_cols = pass_cols;
}

hipError_t spmm_csr(DType dt, IType it, const int64_t* rowptr, const void* col,
                    const float* ew, int heads, int head_dim, const float* col_scale,
                    const float* row_scale, const void* x, int64_t ldx, void* out,
                    int64_t ldo, int64_t nrows, int F, float beta, hipStream_t stream) {
  if (nrows <= 0 || F <= 0) return hipSuccess;
  if (heads < 1) heads = 1;
  if (head_dim < 1) head_dim = F;
#define DG_ARGS(T, I)                                                                   \
  rowptr, static_cast<const I*>(col), ew, heads, head_dim, col_scale, row_scale,        \
      static_cast<const T*>(x), ldx, static_cast<T*>(out), ldo, nrows, F, beta, stream
  if (dt == DType::F32) {
    if (it == IType::I32) return launch_vec<float, int32_t>(DG_ARGS(float, int32_t));
    return launch_vec<float, int64_t>(DG_ARGS(float, int64_t));
  }
  const int pc = g_spmm_pass_cols;
  if (heads == 1 && pc > 0 && F > pc && F % pc == 0) {
    // column passes of 256-B rows: a pass's gathered window (rows near the front times
    // 256 B) stays cache-resident where a full 512-B row window does not (-11% at F=256)
    for (int c0 = 0; c0 < F; c0 += pc) {
      const auto* xp = static_cast<const uint16_t*>(x) + c0;
      auto* op = static_cast<uint16_t*>(out) + c0;
      hipError_t err = it == IType::I32
          ? launch_vec<uint16_t, int32_t>(rowptr, static_cast<const int32_t*>(col), ew, 1, pc,
                                          col_scale, row_scale, xp, ldx, op, ldo, nrows, pc,
                                          beta, stream)
          : launch_vec<uint16_t, int64_t>(rowptr, static_cast<const int64_t*>(col), ew, 1, pc,
                                          col_scale, row_scale, xp, ldx, op, ldo, nrows, pc,
                                          beta, stream);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  if (it == IType::I32) return launch_vec<uint16_t, int32_t>(DG_ARGS(uint16_t, int32_t));
  return launch_vec<uint16_t, int64_t>(DG_ARGS(uint16_t, int64_t));
#undef DG_ARGS
}

}  // namespace dgraph
