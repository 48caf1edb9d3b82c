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
    int64_t nrows, int F, float beta, int64_t cap,
    const int64_t* __restrict__ row_map) {
  constexpr int G = kWave / LPR;  // lane groups per wave = neighbour rows per step
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;

  for (int64_t r = wave; r < nrows; r += nwaves) {
    const int64_t s = rowptr[r];
    const int64_t e1 = rowptr[r + 1];
    const int64_t e = (cap > 0 && e1 - s > cap) ? s + cap : e1;
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
        const int64_t orow = row_map ? row_map[r] : r;  // compacted CSR: output row
        const float rs = row_scale ? row_scale[orow] : 1.f;
        T* o = out + orow * ldo + f;
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
    int64_t nrows, int F, float beta, int64_t cap,
    const int64_t* __restrict__ row_map) {
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
    const int64_t e1 = rowptr[r + 1];
    const int64_t e = (cap > 0 && e1 - s > cap) ? s + cap : e1;
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
        const int64_t orow = row_map ? row_map[r] : r;  // compacted CSR: output row
        const float rs = row_scale ? row_scale[orow] : 1.f;
        T* o = out + orow * ldo + f;
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

// v3 (tried, removed): the v2 data flow with packed-fp32 accumulate and no per-element
// padding select. Same time as v2 (76.7 vs 76.9 ms at F=128): v2 is not VALU bound, it
// pays a fixed ~40 ms per pass for its one-row-per-wave structure (see v4).
typedef float f32x2 __attribute__((ext_vector_type(2)));

// v4 (bf16 rows, one head): ROW-GROUP kernel. v2/v3 give a whole wave to one row and
// split its ~30 neighbours over the lane groups, so every row pays a cross-group
// butterfly, a dependent rowptr -> col -> row chain and its own wave launch: ~40 ms of
// fixed cost per pass over the papers100M CSR, whatever the width. That fixed cost is
// what makes narrow passes (whose neighbour windows fit the 4 MiB per-XCD L2) lose.
// v4 gives each LPR-lane group its OWN row (G = 64/LPR consecutive rows per wave):
//   * no cross-lane reduction at all; one 16-B store per lane writes G rows at once;
//   * each lane loads one column id of its group's row per chunk of LPR neighbours, and
//     the next chunk's ids are prefetched while the current chunk's rows are in flight;
//   * neighbour c of row g is broadcast in-group with one ds_bpermute, its 16-B slice is
//     unpacked and added with packed fp32 math (v_pk_fma_f32, 1.5 VALU per element);
//   * trip count = the largest degree of the G rows (wave-uniform); slots past a row's
//     degree read row 0 with weight 0 (no branches around loads).
//   * weights (edge weights and/or a column scale, compile-time WMODE bits) are loaded
//     branch-free one chunk ahead, after the current chunk's row loads are issued: a
//     runtime "if (col_scale)" made hipcc drain vmcnt at the chunk top (weighted passes
//     ran 54 % slower than unweighted ones).
// A global load hipcc cannot move (it sinks a plain prefetch load down to its first use)
// and does not track: the caller waits with an explicit s_waitcnt before the use.
// Extra untracked loads only make hipcc's own vmcnt waits conservative (in-order count).
__device__ __forceinline__ int32_t load_nosink(const int32_t* p) {
  int32_t v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}
__device__ __forceinline__ int64_t load_nosink(const int64_t* p) {
  int64_t v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p));
  return v;
}

// (second bound: at least 6 waves per SIMD for <= 64-column passes; unbounded, the
// weighted LPR-8 variant took 118 VGPRs = 4 waves and ran 55 % slower than unweighted;
// wider weighted variants would spill under the bound)
template <typename IdxT, int LPR, int WMODE, bool XCD>
__global__ __launch_bounds__(256, (LPR <= 8 ? 6 : 1)) void spmm_bf16_rowgroup_kernel(
    const int64_t* __restrict__ rowptr, const IdxT* __restrict__ col,
    const float* __restrict__ ew, const float* __restrict__ col_scale,
    const float* __restrict__ row_scale, const uint16_t* __restrict__ x, int64_t ldx,
    uint16_t* __restrict__ out, int64_t ldo, int64_t nrows, int F, float beta, int cap,
    const int64_t* __restrict__ row_map) {
  constexpr int VEC = 8;
  constexpr int G = kWave / LPR;
  constexpr int U = LPR < 8 ? LPR : 8;  // neighbour rows in flight per lane per batch
  constexpr bool HAS_EW = (WMODE & 1) != 0;
  constexpr bool HAS_CS = (WMODE & 2) != 0;
  constexpr bool WEIGHTED = WMODE != 0;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int wpb = blockDim.x >> 6;
  const int64_t ngroups = (nrows + G - 1) / G;
  int64_t q0, qstep, qend;
  if constexpr (XCD) {
    const int nx = 8;
    const int64_t bx = blockIdx.x % nx;
    const int64_t chunk = (ngroups + nx - 1) / nx;
    const int64_t lo = bx * chunk;
    qend = lo + chunk < ngroups ? lo + chunk : ngroups;
    q0 = lo + (blockIdx.x / nx) * wpb + (threadIdx.x >> 6);
    qstep = (gridDim.x / nx) * wpb;
  } else {
    q0 = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    qstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
    qend = ngroups;
  }
  const uint32_t ldx32 = static_cast<uint32_t>(ldx);
  const int f = l * VEC;  // launcher guarantees F <= LPR * VEC
  const bool active = f < F;
  const uint16_t* xf = x + (active ? f : 0);
  for (int64_t q = q0; q < qend; q += qstep) {
    const int64_t r = q * G + g;
    const bool has_row = r < nrows;
    const int64_t s = has_row ? rowptr[r] : 0;
    const int64_t deg1 = has_row ? rowptr[r + 1] - s : 0;
    // hub rows (degree > cap) aggregate their first cap entries here; the rest is summed
    // by spmm_hub_partials / spmm_hub_reduce (hub-row splitting)
    const int deg = static_cast<int>(deg1 > cap ? cap : deg1);
    int maxdeg = deg;
#pragma unroll
    for (int off = LPR; off < kWave; off <<= 1) {
      const int o = __shfl_xor(maxdeg, off, kWave);
      maxdeg = o > maxdeg ? o : maxdeg;
    }
    f32x2 acc[VEC / 2];
#pragma unroll
    for (int i = 0; i < VEC / 2; ++i) acc[i] = f32x2{0.f, 0.f};
    // slot k of this group's row: its column id and weight (0 for padding slots, whose
    // id is col[0], a valid row). Branch-free loads at clamped addresses (the CSR has
    // >= 1 entry whenever maxdeg > 0); no select on the loaded id, so nothing waits for
    // a prefetch before its first use.
    auto load_c = [&](int k) -> IdxT { return col[k < deg ? s + k : 0]; };
    auto load_w = [&](IdxT c, int k) -> float {
      float w = k < deg ? 1.f : 0.f;
      if constexpr (HAS_EW) w *= ew[k < deg ? s + k : 0];
      if constexpr (HAS_CS) w *= col_scale[c];
      return w;
    };
    IdxT my_c = IdxT(0);
    float my_w = 0.f;
    if (maxdeg > 0) {
      my_c = load_c(l);
      if constexpr (WEIGHTED) my_w = load_w(my_c, l);
    }
    for (int k0 = 0; k0 < maxdeg; k0 += LPR) {
      const int kn = k0 + LPR + l;
      IdxT nx_c;
      // the previous chunk's asm prefetch of my_c is invisible to hipcc's waitcnt pass:
      // wait for it here (tied to my_c so no use moves above). By now that chunk's row
      // loads have been consumed, so this waits on nothing else.
      if constexpr (!WEIGHTED) asm volatile("s_waitcnt vmcnt(0)" : "+v"(my_c));
#pragma unroll
      for (int j0 = 0; j0 < LPR; j0 += U) {
        if (j0 > 0 && k0 + j0 >= maxdeg) break;  // wave-uniform: no all-padding batch
        uint4 v[U];
        uint32_t c[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          c[u] = static_cast<uint32_t>(__shfl(static_cast<int>(my_c), g * LPR + j0 + u, kWave));
        // next chunk's ids in flight during this chunk, issued after this batch's id
        // shuffles (issued first, hipcc waited for it before the shuffles) and
        // unconditionally (past the last chunk it re-reads col[0]; under a branch hipcc
        // waited for it at the join)
        // (an asm load: a plain load is sunk by LLVM to its use at the next chunk top,
        // where the wave then waits for it; a volatile one waits at once)
        // Weighted passes read the ids again in this chunk (the next weights), so there
        // a plain load stays put.
        if (j0 == 0) {
          if constexpr (WEIGHTED) nx_c = load_c(kn);
          else nx_c = load_nosink(col + (kn < deg ? s + kn : 0));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = *reinterpret_cast<const uint4*>(xf + static_cast<uint64_t>(c[u]) * ldx32);
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (WEIGHTED) {
            w[u] = __shfl(my_w, g * LPR + j0 + u, kWave);  // 0 past the degree
          } else {
            w[u] = (k0 + j0 + u < deg) ? 1.f : 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t d[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
          const f32x2 ww{w[u], w[u]};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const f32x2 t{__uint_as_float(d[i] << 16), __uint_as_float(d[i] & 0xffff0000u)};
            acc[i] = __builtin_elementwise_fma(t, ww, acc[i]);
          }
        }
      }
      if constexpr (WEIGHTED) my_w = load_w(nx_c, kn);
      my_c = nx_c;
    }
    if (has_row && active) {
      const int64_t orow = row_map ? row_map[r] : r;  // compacted CSR: output row
      const float rs = row_scale ? row_scale[orow] : 1.f;
      uint16_t* o = out + orow * ldo + f;
      float res[VEC];
      if (beta != 0.f) {
        float old[VEC];
        load_vec_f32<uint16_t, VEC>(o, old);
#pragma unroll
        for (int i = 0; i < VEC / 2; ++i) {
          res[2 * i] = fmaf(acc[i].x, rs, beta * old[2 * i]);
          res[2 * i + 1] = fmaf(acc[i].y, rs, beta * old[2 * i + 1]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < VEC / 2; ++i) {
          res[2 * i] = acc[i].x * rs;
          res[2 * i + 1] = acc[i].y * rs;
        }
      }
      store_vec_f32<uint16_t, VEC>(o, res);
    }
  }
}

template <typename IdxT>
hipError_t launch_rowgroup(const int64_t* rowptr, const IdxT* col, const float* ew,
                           const float* cs, const float* rs, const uint16_t* x, int64_t ldx,
                           uint16_t* out, int64_t ldo, int64_t nrows, int F, float beta,
                           bool xcd_mode, int64_t cap, const int64_t* row_map,
                           hipStream_t st) {
  const int icap = (cap > 0 && cap < (int64_t(1) << 30)) ? static_cast<int>(cap) : (1 << 30);
  // one pass covers LPR * 8 columns; the caller splits wider rows into passes
  const int lanes = (F + 7) / 8;
  const int LPR = lanes <= 4 ? 4 : lanes <= 8 ? 8 : lanes <= 16 ? 16 : lanes <= 32 ? 32 : 64;
  const int64_t G = kWave / LPR;
  const int64_t ngroups = (nrows + G - 1) / G;
  int64_t blocks = (ngroups + 3) / 4;
  bool xcd = xcd_mode && blocks >= 64;
  if (xcd) blocks = 8 * (((ngroups + 7) / 8 + 3) / 4);  // in-order: one group per wave
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const int wmode = (ew != nullptr ? 1 : 0) | (cs != nullptr ? 2 : 0);
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
#define DG_RG_W(LPR_, W_)                                                                    \
  if (LPR == LPR_ && wmode == W_) {                                                          \
    if (xcd)                                                                                 \
      hipLaunchKernelGGL((spmm_bf16_rowgroup_kernel<IdxT, LPR_, W_, true>), grid, block, 0,  \
                         st, rowptr, col, ew, cs, rs, x, ldx, out, ldo, nrows, F, beta,      \
                         icap, row_map);                                                     \
    else                                                                                     \
      hipLaunchKernelGGL((spmm_bf16_rowgroup_kernel<IdxT, LPR_, W_, false>), grid, block, 0, \
                         st, rowptr, col, ew, cs, rs, x, ldx, out, ldo, nrows, F, beta,      \
                         icap, row_map);                                                     \
    return hipGetLastError();                                                                \
  }
#define DG_RG(LPR_) DG_RG_W(LPR_, 0) DG_RG_W(LPR_, 1) DG_RG_W(LPR_, 2) DG_RG_W(LPR_, 3)
  DG_RG(4)
  DG_RG(8)
  DG_RG(16)
  DG_RG(32)
  DG_RG(64)
#undef DG_RG_W
#undef DG_RG
  return hipErrorInvalidValue;
}

// 1 = per-group index loads, 2 = cooperative + shuffles (fp32 and unaligned bf16 rows),
// 4 = row groups (bf16, 16-B aligned rows: the default). papers100M-shaped CSR, window
// 16384, bf16: F=128 95.3 ms (v2, xcd 2, 128-col passes) -> 64.2 ms (v4, xcd 0, 64-col
// passes); F=256 190.8 -> 129.1 ms (benchmarks/bench_spmm.py). With row groups the plain
// in-order grid (all XCDs on one advancing row band) beats XCD-chunking by 2-7 %.
// Unweighted passes cost the same per column at 64 and 128 columns; weighted (column
// scale) ones are cheaper at 128 (80 vs 2 x 50 ms per 128 columns), hence 128.
constexpr int kSpmmDefaultVariant = 4;
constexpr int kSpmmDefaultXcd = 0;
constexpr int kSpmmDefaultPassCols = 128;
int g_spmm_variant = kSpmmDefaultVariant;
// 0 = grid-stride, 1 = XCD-chunked grid-stride, 2 = XCD-chunked in-order (default),
// 3 = in-order without chunking. The in-order mappings keep the resident waves on a
// narrow advancing row window, so the neighbour rows they gather (which cluster near the
// row ids on locality-ordered graphs) are reused from the Infinity Cache: papers100M-
// shaped graph, F=256: 313 ms (1) -> 211 ms (2) (benchmarks/bench_spmm.py).
int g_spmm_xcd = kSpmmDefaultXcd;
int g_spmm_pass_cols = kSpmmDefaultPassCols;  // bf16 rows wider than this run as passes

template <typename T, typename IdxT, int VEC>
hipError_t launch_lpr(const int64_t* rowptr, const IdxT* col, const float* ew, int heads,
                      int head_dim, const float* cs, const float* rs, const T* x, int64_t ldx,
                      T* out, int64_t ldo, int64_t nrows, int F, float beta, int64_t cap,
                      const int64_t* row_map, hipStream_t st) {
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
  if (g_spmm_variant >= 2) {
    // U rows in flight per lane group: ~16 neighbour rows per wave
#define DG_V2(LPR_, U_)                                                                    \
  if (xcd)                                                                                 \
    hipLaunchKernelGGL((spmm_csr_v2_kernel<T, IdxT, VEC, LPR_, U_, true>), grid, block, 0, \
                       st, rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,     \
                       nrows, F, beta, cap, row_map);                                      \
  else                                                                                     \
    hipLaunchKernelGGL((spmm_csr_v2_kernel<T, IdxT, VEC, LPR_, U_, false>), grid, block,   \
                       0, st, rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,  \
                       nrows, F, beta, cap, row_map);                                      \
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
                     col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo, nrows, F, beta,  \
                     cap, row_map);                                                       \
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
                      T* out, int64_t ldo, int64_t nrows, int F, float beta, int64_t cap,
                      const int64_t* row_map, hipStream_t st) {
  // Widest vector that divides the row, both leading dimensions, the head
  // size and both base pointers.
  constexpr int kMaxVec = 16 / sizeof(T);
  auto ok = [&](int v) {
    return F % v == 0 && ldx % v == 0 && ldo % v == 0 && (heads <= 1 || head_dim % v == 0) &&
           aligned(x, v * sizeof(T)) && aligned(out, v * sizeof(T));
  };
  if (ok(kMaxVec))
    return launch_lpr<T, IdxT, kMaxVec>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out,
                                        ldo, nrows, F, beta, cap, row_map, st);
  if (ok(4))
    return launch_lpr<T, IdxT, 4>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,
                                  nrows, F, beta, cap, row_map, st);
  return launch_lpr<T, IdxT, 1>(rowptr, col, ew, heads, head_dim, cs, rs, x, ldx, out, ldo,
                                nrows, F, beta, cap, row_map, st);
}

}  // namespace

// ---------------------------------------------------------------------------
// Hub-row splitting. A power-law graph has rows whose degree is 10^3-10^5 x the mean
// (the structureless papers100M-shaped graph: ~150K at the top hub). In the row-group
// kernel such a row keeps its whole wave (and the G-1 rows sharing it) iterating long
// after the rest of the grid is done. Rows are therefore capped at `cap` entries in the
// main pass, and the tails are cut into segments of <= cap entries that run as
// independent waves (fp32 partial sums), then added to their rows in a fixed order.
template <typename T, typename IdxT, int VEC>
__global__ __launch_bounds__(256) void hub_partials_kernel(
    const int64_t* __restrict__ seg_beg, const int64_t* __restrict__ seg_end,
    const IdxT* __restrict__ col, const float* __restrict__ ew,
    const float* __restrict__ col_scale, const T* __restrict__ x, int64_t ldx,
    float* __restrict__ part, int64_t nseg, int F) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t w = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (w >= nseg) return;  // wave-uniform
  const int64_t s = seg_beg[w], e = seg_end[w];
  for (int fc = 0; fc < F; fc += kWave * VEC) {
    const int f = fc + lane * VEC;
    const bool active = f < F;
    float acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.f;
    for (int64_t base = s; base < e; base += kWave) {
      const int n = (e - base) < kWave ? static_cast<int>(e - base) : kWave;
      IdxT my_c = IdxT(0);
      float my_w = 0.f;
      if (lane < n) {
        my_c = col[base + lane];
        my_w = ew ? ew[base + lane] : 1.f;
        if (col_scale) my_w *= col_scale[my_c];
      }
      for (int u0 = 0; u0 < n; u0 += 4) {  // n is wave-uniform: shuffles see every lane
        float v[4][VEC];
        float wu[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int src = u0 + k < n ? u0 + k : 0;
          const int64_t c = static_cast<int64_t>(__shfl(my_c, src, kWave));
          wu[k] = u0 + k < n ? __shfl(my_w, src, kWave) : 0.f;
          load_vec_f32<T, VEC>(x + c * ldx + (active ? f : 0), v[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] = fmaf(wu[k], v[k][i], acc[i]);
      }
    }
    if (active) {
      float* o = part + w * F + f;
#pragma unroll
      for (int i = 0; i < VEC; ++i) o[i] = acc[i];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void hub_reduce_kernel(
    const float* __restrict__ part, const int64_t* __restrict__ hub_seg_ptr,
    const int64_t* __restrict__ hub_rows, const float* __restrict__ row_scale,
    T* __restrict__ out, int64_t ldo, int64_t nhub, int F) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t h = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (h >= nhub) return;
  const int64_t r = hub_rows[h];
  const int64_t p0 = hub_seg_ptr[h], p1 = hub_seg_ptr[h + 1];
  const float rs = row_scale ? row_scale[r] : 1.f;
  for (int f = lane; f < F; f += kWave) {
    float acc = 0.f;
    for (int64_t i = p0; i < p1; ++i) acc += part[i * F + f];  // segment order
    T* o = out + r * ldo + f;
    *o = Elem<T>::from_f32(fmaf(rs, acc, Elem<T>::to_f32(*o)));
  }
}

hipError_t spmm_hub_partials(DType dt, IType it, const int64_t* seg_beg,
                             const int64_t* seg_end, const void* col, const float* ew,
                             const float* col_scale, const void* x, int64_t ldx,
                             float* partials, int64_t nseg, int F, hipStream_t stream) {
  if (nseg <= 0 || F <= 0) return hipSuccess;
  const int64_t blocks = (nseg + 3) / 4;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
  // widest vector that divides the row width and the row stride and matches the base
  // pointer's alignment (an output-width aggregate can be 47 or 153 columns wide: a
  // fixed 4-wide bf16 vector would read past the row and write past the partial row)
  const int esz = dt == DType::BF16 ? 2 : 4;
  auto vec_ok = [&](int v) {
    return F % v == 0 && ldx % v == 0 && aligned(x, v * esz);
  };
  const int vec = dt == DType::BF16 ? (vec_ok(4) ? 4 : vec_ok(2) ? 2 : 1)
                                    : (vec_ok(2) ? 2 : 1);
#define DG_HP(T_, I_, V_)                                                                   \
  hipLaunchKernelGGL((hub_partials_kernel<T_, I_, V_>), grid, block, 0, stream, seg_beg,  \
                     seg_end, static_cast<const I_*>(col), ew, col_scale,                  \
                     static_cast<const T_*>(x), ldx, partials, nseg, F);                   \
  return hipGetLastError();
#define DG_HP_V(T_, I_)                      \
  if (vec == 4) { DG_HP(T_, I_, 4) }         \
  if (vec == 2) { DG_HP(T_, I_, 2) }         \
  DG_HP(T_, I_, 1)
  if (dt == DType::BF16) {
    if (it == IType::I32) { DG_HP_V(uint16_t, int32_t) }
    DG_HP_V(uint16_t, int64_t)
  }
  if (vec == 2) {
    if (it == IType::I32) { DG_HP(float, int32_t, 2) }
    DG_HP(float, int64_t, 2)
  }
  if (it == IType::I32) { DG_HP(float, int32_t, 1) }
  DG_HP(float, int64_t, 1)
#undef DG_HP_V
#undef DG_HP
}

hipError_t spmm_hub_reduce(DType dt, const float* partials, const int64_t* hub_seg_ptr,
                           const int64_t* hub_rows, const float* row_scale, void* out,
                           int64_t ldo, int64_t nhub, int F, hipStream_t stream) {
  if (nhub <= 0 || F <= 0) return hipSuccess;
  const int64_t blocks = (nhub + 3) / 4;
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
  if (dt == DType::BF16)
    hipLaunchKernelGGL((hub_reduce_kernel<uint16_t>), grid, block, 0, stream, partials,
                       hub_seg_ptr, hub_rows, row_scale, static_cast<uint16_t*>(out), ldo,
                       nhub, F);
  else
    hipLaunchKernelGGL((hub_reduce_kernel<float>), grid, block, 0, stream, partials,
                       hub_seg_ptr, hub_rows, row_scale, static_cast<float*>(out), ldo, nhub,
                       F);
  return hipGetLastError();
}

bool g_spmm_f32_rowgroup = true;

void set_spmm_f32_config(int rowgroup, int pass_cols) {
  if (rowgroup >= 0) g_spmm_f32_rowgroup = rowgroup != 0;
  if (pass_cols >= 0) set_spmm_f32_pass_cols(pass_cols);
}

void set_spmm_config(int variant, int xcd, int pass_cols) {
  if (variant < 0) {  // restore the defaults
    g_spmm_variant = kSpmmDefaultVariant;
    g_spmm_xcd = kSpmmDefaultXcd;
    g_spmm_pass_cols = kSpmmDefaultPassCols;
    return;
  }
  if (variant == 1 || variant == 2 || variant == 4) g_spmm_variant = variant;
  if (xcd >= 0 && xcd <= 3) g_spmm_xcd = xcd;
  if (pass_cols >= 0) g_spmm_pass_cols = pass_cols;
}

hipError_t spmm_csr(DType dt, IType it, const int64_t* rowptr, const void* col,
                    const float* ew, int heads, int head_dim, const float* col_scale,
                    const float* row_scale, const void* x, int64_t ldx, void* out,
                    int64_t ldo, int64_t nrows, int F, float beta, hipStream_t stream,
                    int64_t cap, const int64_t* row_map) {
  if (nrows <= 0 || F <= 0) return hipSuccess;
  if (heads < 1) heads = 1;
  if (head_dim < 1) head_dim = F;
#define DG_ARGS(T, I)                                                                   \
  rowptr, static_cast<const I*>(col), ew, heads, head_dim, col_scale, row_scale,        \
      static_cast<const T*>(x), ldx, static_cast<T*>(out), ldo, nrows, F, beta, cap, row_map, stream
  if (dt == DType::F32) {
    // fp32 row-group kernel (spmm_f32.hip) for one head and 16-B aligned rows
    if (g_spmm_f32_rowgroup && heads <= 1 && spmm_f32_rowgroup_ok(F, ldx, ldo, x, out))
      return spmm_f32_rowgroup(it, rowptr, col, ew, col_scale, row_scale, nullptr, nullptr,
                               static_cast<const float*>(x), ldx, static_cast<float*>(out),
                               ldo, nrows, F, beta, cap, row_map, stream);
    if (it == IType::I32) return launch_vec<float, int32_t>(DG_ARGS(float, int32_t));
    return launch_vec<float, int64_t>(DG_ARGS(float, int64_t));
  }
  if (g_spmm_variant == 4 && heads <= 1 && F % 8 == 0 && ldx % 8 == 0 && ldo % 8 == 0 &&
      aligned(x, 16) && aligned(out, 16) && ldx < (int64_t(1) << 31)) {
    int pc = g_spmm_pass_cols > 0 ? g_spmm_pass_cols : 512;
    pc = pc > 512 ? 512 : (pc < 8 ? 8 : pc - pc % 8);
    const bool xcd = g_spmm_xcd == 1 || g_spmm_xcd == 2;
    for (int c0 = 0; c0 < F; c0 += pc) {
      const int w = F - c0 < pc ? F - c0 : pc;
      const auto* xp = static_cast<const uint16_t*>(x) + c0;
      auto* op = static_cast<uint16_t*>(out) + c0;
      hipError_t err = it == IType::I32
          ? launch_rowgroup<int32_t>(rowptr, static_cast<const int32_t*>(col), ew, col_scale,
                                     row_scale, xp, ldx, op, ldo, nrows, w, beta, xcd, cap,
                                     row_map, stream)
          : launch_rowgroup<int64_t>(rowptr, static_cast<const int64_t*>(col), ew, col_scale,
                                     row_scale, xp, ldx, op, ldo, nrows, w, beta, xcd, cap,
                                     row_map, stream);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
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
                                          beta, cap, row_map, stream)
          : launch_vec<uint16_t, int64_t>(rowptr, static_cast<const int64_t*>(col), ew, 1, pc,
                                          col_scale, row_scale, xp, ldx, op, ldo, nrows, pc,
                                          beta, cap, row_map, stream);
      if (err != hipSuccess) return err;
    }
    return hipSuccess;
  }
  if (it == IType::I32) return launch_vec<uint16_t, int32_t>(DG_ARGS(uint16_t, int32_t));
  return launch_vec<uint16_t, int64_t>(DG_ARGS(uint16_t, int64_t));
#undef DG_ARGS
}

}  // namespace dgraph
