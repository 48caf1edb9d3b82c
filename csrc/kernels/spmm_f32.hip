// dgraph_amd — fp32 row-group CSR SpMM for gfx950 (K-new-2 at the reference's precision).
//
// The reference is fp32-only (DGraph/distributed/csrc/torch_local_kernels.cu:43-46); its
// aggregation was scatter_add + float atomics. This is the fp32 instantiation of the
// row-group design of spmm.hip (v4), not a widened bf16 kernel:
//   * each LPR-lane group of a wave owns ONE output row (G = 64/LPR rows per wave): no
//     cross-lane reduction, one 16-B store per lane per row;
//   * lane l of a group covers columns [4l, 4l+4) (16-B fp32 vector); a pass covers
//     4*LPR columns, wider rows run as column passes (the launcher slices them);
//   * per chunk of LPR neighbours every lane loads ONE column id (coalesced), the ids are
//     broadcast in-group with ds_bpermute and U neighbour rows are in flight per lane;
//   * weights (edge weights / column scale, compile-time WMODE) are loaded one chunk ahead;
//   * trip count = the largest degree of the G rows (wave-uniform); slots past a row's
//     degree read a valid row with weight 0 (no branches around loads).
// Two extensions used by the memory-lean full-graph executor (models/sage_fused.py):
//   * row_ids (runtime, nullable): group row i aggregates CSR row row_ids[i] (an input row
//     list, e.g. the gradient-support rows) and writes output row i (or row_map[i]);
//   * col_map (compile-time CMAP): column c reads x row col_map[c]; entries with
//     col_map[c] < 0 are skipped (x is a row-compacted operand, e.g. a gradient that is
//     nonzero only on the support rows and is stored only there).
//   * rowend (runtime, nullable): row r's entries are [rowptr[rr], rowend[rr]) instead of
//     [rowptr[rr], rowptr[rr + 1]) — one part of a row whose entries are stored in two runs
//     (a vertex-partitioned rank's unified adjacency: interior columns, then halo columns);
//   * two sources (compile-time TWO): column c < nsplit reads x row c, column c >= nsplit
//     reads x2 row c - nsplit (the received halo rows) — interior and halo of a row in ONE
//     pass when the halo is resident, instead of an interior pass plus a beta=1 halo pass.
//     With a col_map the split applies to the mapped index (a support-row gradient and the
//     received support rows of the halo, one map over local + halo columns).
// Accumulation fp32 with packed FMAs in a fixed order per row: bitwise deterministic.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// Batches of 8 neighbour rows per lane (98 VGPRs, 4 waves per SIMD). Measured against one
// batch of all LPR rows (all loads of a chunk before its FMAs: -3 %) and against forcing 6 or
// 8 waves per SIMD (fewer registers, fewer loads in flight: -28 % / -38 %),
// profiles/r04/spmm_f32_variants_ab.log.
template <typename IdxT, int LPR, int WMODE, bool CMAP, bool TWO, bool KB = false>
__global__ __launch_bounds__(256) void spmm_f32_rowgroup_kernel(SpmmF32Args a) {
  constexpr int VEC = 4;
  constexpr int G = kWave / LPR;
  constexpr int U = LPR < 8 ? LPR : 8;  // neighbour rows in flight per lane per batch
  constexpr bool HAS_EW = (WMODE & 1) != 0;
  constexpr bool HAS_CS = (WMODE & 2) != 0;
  const IdxT* __restrict__ col = static_cast<const IdxT*>(a.col);
  const int64_t* __restrict__ rowptr = a.rowptr;
  const int lane = threadIdx.x & (kWave - 1);
  const int g = lane / LPR;
  const int l = lane % LPR;
  const int wv = threadIdx.x >> 6;  // wave of the block (its row of the compaction table)
  __shared__ uint8_t inv[CMAP ? 4 * 64 : 1];
  const int64_t nrows = a.nrows;
  const int F = a.F;
  const int64_t ngroups = (nrows + G - 1) / G;
  // XCD-contiguous rows: blocks are dealt round-robin over the 8 XCDs (b and b + 8 share
  // one, MI355X_MICROARCH.md "Workgroup dispatch"), so in-order blocks would give every
  // XCD's L2 every 8th row group and each neighbour row of a local window would be fetched
  // into all 8 L2s. Remapped, the XCD of blocks b = 8k + x walks the contiguous block range
  // [x * nb/8, (x + 1) * nb/8) in order: a row's in-window uses all hit one L2. Only for
  // the unpersisted grid (one row group per wave); the tail past a multiple of 8 keeps its
  // place. Placement is for speed only: any mapping is correct (a bijection).
  int64_t blk = blockIdx.x;
  if (a.xcd_remap) {
    const int64_t full = static_cast<int64_t>(gridDim.x) & ~int64_t(7);
    if (blk < full) blk = (blk & 7) * (full >> 3) + (blk >> 3);
  }
  const int64_t q0 = (blk * blockDim.x + threadIdx.x) >> 6;
  const int64_t qstep = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  const int f = l * VEC;  // launcher guarantees F <= LPR * VEC
  const bool active = f < F;
  const float* xf = a.x + (active ? f : 0);
  const float* x2f = TWO ? a.x2 + (active ? f : 0) : nullptr;
  const uint64_t ldx = static_cast<uint64_t>(a.ldx);
  const uint64_t ldx2 = static_cast<uint64_t>(a.ldx2);
  const uint32_t ns = static_cast<uint32_t>(a.nsplit);
  const int cap = a.cap;
  // the row of x (or x2) that column id c reads
  auto row_ptr = [&](uint32_t c) -> const float* {
    if constexpr (TWO) {
      return c < ns ? xf + static_cast<uint64_t>(c) * ldx
                    : x2f + static_cast<uint64_t>(c - ns) * ldx2;
    } else {
      return xf + static_cast<uint64_t>(c) * ldx;
    }
  };
  for (int64_t q = q0; q < ngroups; q += qstep) {
    const int64_t r = q * G + g;
    const bool has_row = r < nrows;
    const int64_t rr = has_row ? (a.row_ids ? a.row_ids[r] : r) : 0;
    const int64_t s = has_row ? rowptr[rr] : 0;
    const int64_t deg1 = has_row ? (a.rowend ? a.rowend[rr] : rowptr[rr + 1]) - s : 0;
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
    // slot k of this group's row -> (row of x to read, weight); padding slots read row 0
    // of x (column id 0: valid for x, col_map and col_scale whatever part of a row the
    // call covers; an entry of the column array may be a halo column) with weight 0
    auto load_c = [&](int k) -> int64_t {
      // unconditional load (entry 0 for padding slots: a load under a branch is waited for
      // at the join), its value replaced by column 0 for padding
      const IdxT c = col[k < deg ? s + k : 0];
      return k < deg ? static_cast<int64_t>(c) : int64_t(0);
    };
    auto load_w = [&](int64_t& c, int k) -> float {
      float w = k < deg ? 1.f : 0.f;
      if constexpr (CMAP) {
        const int32_t m = a.col_map[c];
        w = m >= 0 ? w : 0.f;
        c = m >= 0 ? m : 0;
      }
      if constexpr (HAS_EW) w *= a.ew[k < deg ? s + k : 0];
      if constexpr (HAS_CS) w *= a.col_scale[c];
      return w;
    };
    int64_t my_c = 0;
    float my_w = 0.f;
    if (maxdeg > 0) {
      my_c = load_c(l);
      my_w = load_w(my_c, l);
    }
    for (int k0 = 0; k0 < maxdeg; k0 += LPR) {
      const int kn = k0 + LPR + l;
      int64_t nx_c = 0;
      if constexpr (CMAP) {
        // column-mapped operand (e.g. a gradient stored only on the support rows): most
        // entries map to -1. Compact this chunk's mapped entries to the front of the group
        // (ballot + rank, the inverse permutation through a 64-byte LDS table per wave) and
        // gather only those: the trip count is the largest mapped count among the wave's
        // groups, not LPR. Summation order = entry order (deterministic, same as uncompacted)
        const bool valid = my_w != 0.f;
        const uint64_t bal = __ballot(valid);
        const uint64_t gm = LPR == 64 ? bal : (bal >> (g * LPR)) & ((1ull << (LPR & 63)) - 1);
        const int cnt = __popcll(gm);
        int mc = cnt;
#pragma unroll
        for (int off = LPR; off < kWave; off <<= 1) {
          const int o = __shfl_xor(mc, off, kWave);
          mc = o > mc ? o : mc;
        }
        const int rank = __popcll(gm & ((1ull << l) - 1));
        if (valid) inv[wv * kWave + g * LPR + rank] = static_cast<uint8_t>(l);
        nx_c = load_c(kn);
        for (int j0 = 0; j0 < mc; j0 += U) {
          uint4 v[U];
          uint32_t c[U];
          float w[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int j = j0 + u;
            const int src = j < cnt ? static_cast<int>(inv[wv * kWave + g * LPR + j]) : 0;
            c[u] = static_cast<uint32_t>(__shfl(static_cast<int>(my_c), g * LPR + src, kWave));
            const float ww = __shfl(my_w, g * LPR + src, kWave);
            w[u] = j < cnt ? ww : 0.f;
          }
#pragma unroll
          for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(row_ptr(c[u]));
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const f32x2 ww{w[u], w[u]};
            const f32x2 t0{__uint_as_float(v[u].x), __uint_as_float(v[u].y)};
            const f32x2 t1{__uint_as_float(v[u].z), __uint_as_float(v[u].w)};
            acc[0] = __builtin_elementwise_fma(t0, ww, acc[0]);
            acc[1] = __builtin_elementwise_fma(t1, ww, acc[1]);
          }
        }
        my_w = load_w(nx_c, kn);
        my_c = nx_c;
        continue;
      }
#pragma unroll
      for (int j0 = 0; j0 < LPR; j0 += U) {
        if (j0 > 0 && k0 + j0 >= maxdeg) break;  // wave-uniform: no all-padding batch
        uint4 v[U];
        uint32_t c[U];
        float w[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          c[u] = static_cast<uint32_t>(
              __shfl(static_cast<int>(my_c), g * LPR + j0 + u, kWave));
        // next chunk's ids in flight during this chunk (issued after this batch's
        // shuffles, unconditionally: past the end it re-reads entry 0)
        if (j0 == 0) nx_c = load_c(kn);
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const uint4*>(row_ptr(c[u]));
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = __shfl(my_w, g * LPR + j0 + u, kWave);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const f32x2 ww{w[u], w[u]};
          const f32x2 t0{__uint_as_float(v[u].x), __uint_as_float(v[u].y)};
          const f32x2 t1{__uint_as_float(v[u].z), __uint_as_float(v[u].w)};
          acc[0] = __builtin_elementwise_fma(t0, ww, acc[0]);
          acc[1] = __builtin_elementwise_fma(t1, ww, acc[1]);
        }
      }
      my_w = load_w(nx_c, kn);
      my_c = nx_c;
    }
    if (has_row && active) {
      const int64_t orow = a.row_map ? a.row_map[r] : r;
      const float rs = a.row_scale ? a.row_scale[orow] : 1.f;
      float* o = a.out + orow * a.ldo + f;
      const float beta = a.beta;
      float4 res;
      if (beta != 0.f) {
        const float4 old = *reinterpret_cast<const float4*>(o);
        res.x = fmaf(acc[0].x, rs, beta * old.x);
        res.y = fmaf(acc[0].y, rs, beta * old.y);
        res.z = fmaf(acc[1].x, rs, beta * old.z);
        res.w = fmaf(acc[1].y, rs, beta * old.w);
      } else {
        res.x = acc[0].x * rs;
        res.y = acc[0].y * rs;
        res.z = acc[1].x * rs;
        res.w = acc[1].y * rs;
      }
      if (a.self_add) {  // + the row's own term, stored row-compacted (row-uniform branch)
        const int32_t m = a.self_map[a.self_row0 + orow];
        if (m >= 0) {
          const float4 sv = *reinterpret_cast<const float4*>(a.self_add + m * a.ld_self + f);
          res.x += sv.x;
          res.y += sv.y;
          res.z += sv.z;
          res.w += sv.w;
        }
      }
      if (a.gate) {  // ReLU derivative from a stored activation (row-uniform branch)
        const float4 gv = *reinterpret_cast<const float4*>(a.gate + orow * a.ldgate + f);
        res.x = gv.x > 0.f ? res.x : 0.f;
        res.y = gv.y > 0.f ? res.y : 0.f;
        res.z = gv.z > 0.f ? res.z : 0.f;
        res.w = gv.w > 0.f ? res.w : 0.f;
      }
      // the same from a 1-bit mask (4 columns never straddle a word); compile-time, so the
      // variants without it keep their register count (the 64-column pass: 94 VGPRs, 5
      // waves per SIMD; a runtime branch here cost a wave)
      if constexpr (KB) {
        const int c = a.bits_col0 + f;
        const uint32_t w = a.keep_bits[orow * a.ld_bits + (c >> 5)] >> (c & 31);
        res.x = (w & 1u) ? res.x : 0.f;
        res.y = (w & 2u) ? res.y : 0.f;
        res.z = (w & 4u) ? res.z : 0.f;
        res.w = (w & 8u) ? res.w : 0.f;
      }
      *reinterpret_cast<float4*>(o) = res;
    }
  }
}

// grid cap (0 = one row group per wave, the whole graph in one launch): the kernel is
// grid-strided, so a capped grid is a persistent one that leaves room on every CU for a
// kernel of another stream (set_spmm_f32_grid)
int g_f32_grid_cap = 0;
int g_f32_xcd = 0;  // measured: no gain (PERFORMANCE.md, round 5)

template <typename IdxT>
hipError_t launch_f32_rg(const SpmmF32Args& a, hipStream_t st) {
  const int lanes = (a.F + 3) / 4;
  const int LPR = lanes <= 8 ? 8 : lanes <= 16 ? 16 : lanes <= 32 ? 32 : 64;
  const int64_t G = kWave / LPR;
  const int64_t ngroups = (a.nrows + G - 1) / G;
  int64_t blocks = (ngroups + 3) / 4;  // in order: one row group per wave
  SpmmF32Args ka = a;
  ka.xcd_remap = g_f32_xcd ? 1 : 0;
  if (g_f32_grid_cap > 0 && blocks > g_f32_grid_cap) {
    blocks = g_f32_grid_cap;
    ka.xcd_remap = 0;  // persistent grid-stride: blocks stay interleaved
  }
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const int wmode = (a.ew != nullptr ? 1 : 0) | (a.col_scale != nullptr ? 2 : 0);
  const bool cmap = a.col_map != nullptr;
  const bool two = a.x2 != nullptr;
  const bool kb = a.keep_bits != nullptr;
  if (two && wmode != 0) return hipErrorInvalidValue;  // not instantiated
  if (kb && (two || cmap || wmode != 0)) return hipErrorInvalidValue;  // not instantiated
  if (kb) {
#define DG_F32_KB(LPR_)                                                                      \
    if (LPR == LPR_) {                                                                       \
      hipLaunchKernelGGL((spmm_f32_rowgroup_kernel<IdxT, LPR_, 0, false, false, true>), grid, \
                         block, 0, st, ka);                                                  \
      return hipGetLastError();                                                              \
    }
    dim3 grid(static_cast<unsigned>(blocks)), block(256);
    DG_F32_KB(8) DG_F32_KB(16) DG_F32_KB(32) DG_F32_KB(64)
#undef DG_F32_KB
    return hipErrorInvalidValue;
  }
  dim3 grid(static_cast<unsigned>(blocks)), block(256);
#define DG_F32_K(LPR_, W_, C_, T_)                                                          \
  if (LPR == LPR_ && wmode == W_ && cmap == C_ && two == T_) {                              \
    hipLaunchKernelGGL((spmm_f32_rowgroup_kernel<IdxT, LPR_, W_, C_, T_>), grid, block, 0, \
                       st, ka);                                                             \
    return hipGetLastError();                                                               \
  }
#define DG_F32(LPR_)                                                                        \
  DG_F32_K(LPR_, 0, false, false) DG_F32_K(LPR_, 1, false, false)                           \
  DG_F32_K(LPR_, 2, false, false) DG_F32_K(LPR_, 3, false, false)                           \
  DG_F32_K(LPR_, 0, true, false) DG_F32_K(LPR_, 1, true, false)                             \
  DG_F32_K(LPR_, 2, true, false) DG_F32_K(LPR_, 3, true, false)                             \
  DG_F32_K(LPR_, 0, false, true) DG_F32_K(LPR_, 0, true, true)
  DG_F32(8)
  DG_F32(16)
  DG_F32(32)
  DG_F32(64)
#undef DG_F32_K
#undef DG_F32
  return hipErrorInvalidValue;
}

// fp32 rows wider than this run as column passes (each pass gathers a narrower window,
// which the per-XCD L2 / Infinity Cache holds longer). A/B: benchmarks/bench_spmm.py
int g_f32_pass_cols = 64;

}  // namespace

void set_spmm_f32_pass_cols(int cols) { g_f32_pass_cols = cols > 0 ? cols : 64; }

void set_spmm_f32_grid(int blocks) { g_f32_grid_cap = blocks > 0 ? blocks : 0; }

void set_spmm_f32_xcd(int on) { g_f32_xcd = on ? 1 : 0; }

bool spmm_f32_rowgroup_ok(int F, int64_t ldx, int64_t ldo, const void* x, const void* out) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) % 16) == 0; };
  return F % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && al(x) && al(out) &&
         ldx < (int64_t(1) << 40);
}

hipError_t spmm_f32_run(const SpmmF32Args& args, hipStream_t st) {
  if (args.nrows <= 0 || args.F <= 0) return hipSuccess;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (args.self_add && (!args.self_map || !al(args.self_add) || args.ld_self % 4))
    return hipErrorInvalidValue;
  if (args.gate && (!al(args.gate) || args.ldgate % 4)) return hipErrorInvalidValue;
  if (!spmm_f32_rowgroup_ok(args.F, args.ldx, args.ldo, args.x, args.out))
    return hipErrorInvalidValue;
  if (args.x2 && (!al(args.x2) || args.ldx2 % 4 || args.nsplit < 0 ||
                  args.nsplit >= (int64_t(1) << 32)))
    return hipErrorInvalidValue;
  SpmmF32Args a = args;
  a.cap = (args.cap > 0 && args.cap < (int64_t(1) << 30)) ? args.cap : (1 << 30);
  int pc = args.pass_cols > 0 ? args.pass_cols : g_f32_pass_cols;
  pc = pc > 256 ? 256 : (pc < 16 ? 16 : pc - pc % 4);
  for (int c0 = 0; c0 < args.F; c0 += pc) {
    SpmmF32Args p = a;
    p.F = args.F - c0 < pc ? args.F - c0 : pc;
    p.x = args.x + c0;
    p.x2 = args.x2 ? args.x2 + c0 : nullptr;
    p.out = args.out + c0;
    p.gate = args.gate ? args.gate + c0 : nullptr;
    p.self_add = args.self_add ? args.self_add + c0 : nullptr;
    p.bits_col0 = args.bits_col0 + c0;
    const hipError_t err = args.it == IType::I32 ? launch_f32_rg<int32_t>(p, st)
                                                 : launch_f32_rg<int64_t>(p, st);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

hipError_t spmm_f32_rowgroup(IType it, const int64_t* rowptr, const void* col,
                             const float* ew, const float* col_scale, const float* row_scale,
                             const int32_t* col_map, const int64_t* row_ids, const float* x,
                             int64_t ldx, float* out, int64_t ldo, int64_t nrows, int F,
                             float beta, int64_t cap, const int64_t* row_map,
                             hipStream_t st, const float* gate, int64_t ldgate,
                             const float* self_add, int64_t ld_self, const int32_t* self_map,
                             int64_t self_row0) {
  SpmmF32Args a{};
  a.rowptr = rowptr;
  a.col = col;
  a.it = it;
  a.ew = ew;
  a.col_scale = col_scale;
  a.row_scale = row_scale;
  a.col_map = col_map;
  a.row_ids = row_ids;
  a.row_map = row_map;
  a.x = x;
  a.ldx = ldx;
  a.out = out;
  a.ldo = ldo;
  a.nrows = nrows;
  a.F = F;
  a.beta = beta;
  a.cap = cap;
  a.gate = gate;
  a.ldgate = ldgate;
  a.self_add = self_add;
  a.ld_self = ld_self;
  a.self_map = self_map;
  a.self_row0 = self_row0;
  return spmm_f32_run(a, st);
}

}  // namespace dgraph
