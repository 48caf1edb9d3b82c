// dgraph_amd — fused fp32 GraphSAGE hidden layer: aggregation AND combine in one kernel.
//
//   out[r, :] = relu( X[r, :] @ Ws + (inv_deg[r] * sum_{c in N(r)} X[c, :]) @ Wn + b )
//
// Why: the aggregation is a memory-bound gather (13 TB/s effective from the Infinity Cache)
// and the combine a compute-bound exact-f32 MFMA GEMM; as two kernels on two streams they
// do NOT overlap — the GEMM's blocks take every SIMD's registers, so no gather wave can sit
// next to them (benchmarks/bench_overlap_f32.py, profiles/r03/overlap_probe*.log). Here one
// persistent block per CU owns BOTH roles, so they are co-resident by construction:
//   * waves 0-3 (MFMA role): the combine of 128-row tile t — [X_t | AGG_t] @ [Ws; Wn] with
//     v_mfma_f32_16x16x4_f32 (exact f32), one wave per SIMD (32 rows x 256 columns each),
//     K staged in 32-deep steps through two LDS buffers (the lean tile of gemm_f32.hip);
//   * waves 4-7 (gather role): the aggregate rows of the block's NEXT tile into a per-block
//     global ring of two 128-row slots (L2-resident), one row per wave at a time, 16-B
//     vector loads, up to 32 neighbour rows in flight per lane.
// The roles synchronise through LDS counters only (the MFMA waves' per-stage barrier is a
// 4-wave counter barrier, not __syncthreads): "ready" (tiles gathered) and "consumed"
// (tiles whose aggregate the MFMA role has read), so the gather of tile t+1 runs while
// tile t's MFMAs run, on the same CU. Every spin is bounded (a stuck peer sets *err and the
// waits give up, so the grid always drains). Deterministic: fixed summation order per row,
// fixed MFMA k order.
#include "../common.h"
#include "kernels.h"

namespace dgraph {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSM = 128;   // rows per tile
constexpr int kSK = 32;    // K per stage
constexpr int kSN = 256;   // output width (hidden)
constexpr int kSBP = kSN + 16;
constexpr int kSA = kSM * kSK;            // A stage floats
constexpr int kSB = kSK * kSBP;           // B stage floats
constexpr int kSStage = kSA + kSB;
constexpr int kSpinMax = 1 << 24;

__device__ __forceinline__ int sa_chunk(int r, int c) {
  constexpr uint32_t kSwz = 0x32765410u;
  return c ^ static_cast<int>((kSwz >> (4 * ((r >> 1) & 7))) & 7u);
}
__device__ __forceinline__ int sb_row(int k) { return k * kSBP + ((k >> 3) & 1) * 16; }

__device__ __forceinline__ int lds_load(int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// wait until *p >= target (bounded); every lane of the wave waits. agent_acq: the data the
// signal publishes is in GLOBAL memory (the aggregate ring), which this CU's vector L1 may
// still hold from the slot's previous use: acquire at agent scope, which invalidates the L1
// (a workgroup-scope acquire leaves it, and stale ring lines were read at full scale)
template <bool AGENT_ACQ = false>
__device__ __forceinline__ void wait_ge(int* p, int target, int* err) {
  int spins = 0;
  while (lds_load(p) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > kSpinMax) {
      if ((threadIdx.x & 63) == 0) atomicExch(err, 1);
      break;
    }
  }
  if constexpr (AGENT_ACQ)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  else
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void signal_add(int* p) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(p, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int F>
__global__ __launch_bounds__(512, 1) void sage_fwd_f32_kernel(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, const float* __restrict__ inv_deg,
    const float* __restrict__ Ws, const float* __restrict__ Wn, const float* __restrict__ bias,
    float* __restrict__ out, int64_t ldo, int64_t M, float* __restrict__ ring, int* err) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  // [1] consumed (tiles whose aggregate the MFMA role has read), [2] MFMA-wave barrier,
  // [4 + w] tiles gathered by gather wave w: one counter PER gather wave — a single shared
  // count is ambiguous when the waves drift apart (a wave one tile ahead makes the total
  // look like a complete tile; the full-scale check caught exactly that)
  int* ctr = reinterpret_cast<int*>(lds + 2 * kSStage);
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int64_t ntiles = (M + kSM - 1) / kSM;
  if (tid < 8) ctr[tid] = 0;
  __syncthreads();  // the only block-wide barrier: before the roles split
  if (static_cast<int64_t>(blockIdx.x) >= ntiles) return;
  float* slot0 = ring + static_cast<int64_t>(blockIdx.x) * 2 * kSM * F;

  if (wave >= 4) {
    // ------------------------------------------------------------------ gather role
    constexpr int LPR = F / 4;         // lanes per row (64 for F=256, 32 for F=128)
    constexpr int G = 64 / LPR;        // rows per wave at a time
    constexpr int U = 32;              // neighbour rows in flight per lane per batch
    const int gw = wave - 4;
    const int g = lane / LPR, l = lane % LPR;
    int i = 0;
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x, ++i) {
      wait_ge(&ctr[1], i - 1, err);  // slot i%2 was last read by tile i-2
      float* slot = slot0 + (i & 1) * kSM * F;
      const int64_t r0 = t * kSM;
      // software-pipelined over this wave's rows: the next row's bounds and its first chunk
      // of column ids are loaded while the current row's neighbour rows are in flight (the
      // index loads would otherwise add two dependent latencies per row)
      const float* xf = X + 4 * l;
      auto bounds = [&](int q0, int64_t& sb, int& db) {
        const int64_t rq = r0 + q0 + g;
        const bool h = q0 < kSM && rq < M;
        sb = h ? rowptr[rq] : 0;
        db = h ? static_cast<int>(rowptr[rq + 1] - sb) : 0;
      };
      int64_t s;
      int deg;
      bounds(gw * G, s, deg);
      int c_first = col[l < deg ? s + l : (deg > 0 ? s : 0)];
      for (int rr0 = gw * G; rr0 < kSM; rr0 += 4 * G) {
        const int rr = rr0 + g;
        const int64_t r = r0 + rr;
        const bool has = r < M;
        int64_t sn;
        int degn;
        bounds(rr0 + 4 * G, sn, degn);  // next row (in flight during this row's gathers)
        const float sc = has ? inv_deg[r] : 0.f;
        int maxdeg = deg;
#pragma unroll
        for (int off = LPR; off < 64; off <<= 1) {
          const int o = __shfl_xor(maxdeg, off, 64);
          maxdeg = o > maxdeg ? o : maxdeg;
        }
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
        int c_next_first = 0;
        for (int k0 = 0; k0 < maxdeg || k0 == 0; k0 += LPR) {
          const int kk = k0 + l;
          const int my_c = k0 == 0 ? c_first : col[kk < deg ? s + kk : (deg > 0 ? s : 0)];
          const float my_w = kk < deg ? 1.f : 0.f;
          const int cnt = maxdeg - k0 < LPR ? maxdeg - k0 : LPR;
          for (int j0 = 0; j0 < cnt; j0 += U) {
            f32x4 v[U];
            float w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int j = j0 + u < LPR ? j0 + u : LPR - 1;
              const int c = __shfl(my_c, g * LPR + j, 64);
              w[u] = j0 + u < cnt ? __shfl(my_w, g * LPR + j, 64) : 0.f;
              v[u] = *reinterpret_cast<const f32x4*>(xf + static_cast<int64_t>(c) * ldx);
            }
            if (k0 == 0 && j0 == 0)  // the next row's first ids, behind this batch's loads
              c_next_first = col[l < degn ? sn + l : (degn > 0 ? sn : 0)];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              a0 = fmaf(v[u][0], w[u], a0);
              a1 = fmaf(v[u][1], w[u], a1);
              a2 = fmaf(v[u][2], w[u], a2);
              a3 = fmaf(v[u][3], w[u], a3);
            }
          }
          if (k0 == 0 && cnt <= 0)  // empty row pair: still fetch the next row's ids
            c_next_first = col[l < degn ? sn + l : (degn > 0 ? sn : 0)];
          if (maxdeg == 0) break;
        }
        *reinterpret_cast<f32x4*>(slot + rr * F + 4 * l) = f32x4{a0 * sc, a1 * sc, a2 * sc, a3 * sc};
        s = sn;
        deg = degn;
        c_first = c_next_first;
      }
      signal_add(&ctr[4 + gw]);  // this wave's rows of tile i are in the ring
    }
    return;
  }

  // -------------------------------------------------------------------- MFMA role
  constexpr int TM = 2, TN = 16;
  constexpr int nst = 2 * F / kSK;
  constexpr int nst1 = F / kSK;   // stages of the self part (X rows)
  const int li = lane & 15, lh = lane >> 4;
  const int arow_w = wave * TM * 16;
  int bar = 0;
  auto group_bar = [&]() {
    bar += 4;
    signal_add(&ctr[2]);
    wait_ge(&ctr[2], bar, err);
  };
  int64_t tile = blockIdx.x;
  int i = 0;
  int64_t ld_tile = tile;
  int ld_i = 0;
  f32x4 ra[4];  // A stage: 128 x 32 floats = 1024 float4 / 256 threads
  f32x4 rb[8];  // B stage: 32 x 256 floats = 2048 float4 / 256 threads
  auto load_stage = [&](int s) {
    const bool self_part = s < nst1;
    const int ka = (self_part ? s : s - nst1) * kSK;
    const float* slot = slot0 + (ld_i & 1) * kSM * F;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u;
      const int rr = q / 8, c4 = (q % 8) * 4;
      int64_t r = ld_tile * kSM + rr;
      r = r < M ? r : M - 1;
      const float* p = self_part ? X + r * ldx + ka + c4 : slot + rr * F + ka + c4;
      ra[u] = *reinterpret_cast<const f32x4*>(p);
    }
    const float* B = self_part ? Ws : Wn;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = tid + 256 * u;
      const int kr = q / (kSN / 4), c4 = (q % (kSN / 4)) * 4;
      rb[u] = *reinterpret_cast<const f32x4*>(B + static_cast<int64_t>(ka + kr) * kSN + c4);
    }
  };
  auto store_stage = [&](int buf) {
    float* sa = lds + buf * kSStage;
    float* sb = sa + kSA;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int q = tid + 256 * u;
      const int r = q / 8;
      *reinterpret_cast<f32x4*>(sa + r * kSK + sa_chunk(r, q % 8) * 4) = ra[u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int q = tid + 256 * u;
      const int kr = q / (kSN / 4), c4 = (q % (kSN / 4)) * 4;
      *reinterpret_cast<f32x4*>(sb + sb_row(kr) + c4) = rb[u];
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  load_stage(0);
  store_stage(0);
  group_bar();
  int gstage = 0;
  while (true) {
    const int64_t next = tile + gridDim.x;
    const bool has_next = next < ntiles;
    for (int s = 0; s < nst; ++s, ++gstage) {
      const int buf = gstage & 1;
      const bool last = s + 1 == nst;
      if (s + 1 == nst1) {  // this tile's aggregate: every gather wave's rows
#pragma unroll
        for (int w = 0; w < 4; ++w) wait_ge<true>(&ctr[4 + w], i + 1, err);
      }
      if (last && has_next) {
        ld_tile = next;
        ld_i = i + 1;
      }
      load_stage(last ? 0 : s + 1);
      __builtin_amdgcn_sched_barrier(0);
      const float* sa = lds + buf * kSStage;
      const float* sb = sa + kSA;
      f32x4 af[TM][2];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int r = arow_w + a * 16 + li;
        const float* p = sa + r * kSK;
        af[a][0] = *reinterpret_cast<const f32x4*>(p + sa_chunk(r, 2 * lh) * 4);
        af[a][1] = *reinterpret_cast<const f32x4*>(p + sa_chunk(r, 2 * lh + 1) * 4);
      }
      const float* sbw = sb + sb_row(8 * lh) + li;
      float bf[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = sbw[b * 16];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float av0 = af[0][j >> 2][j & 3];
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[0][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av0, bf[b], acc[0][b], 0, 0, 0);
        const float av1 = af[1][j >> 2][j & 3];
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[1][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av1, bf[b], acc[1][b], 0, 0, 0);
          if (j + 1 < 8) bf[b] = sbw[(j + 1) * kSBP + b * 16];
        }
      }
      store_stage(buf ^ 1);
      group_bar();
      // the last aggregate stage of this tile is in LDS: its ring slot may be reused
      if (s + 2 == nst && wave == 0) signal_add(&ctr[1]);
    }
    const int64_t row0 = tile * kSM;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t rw = row0 + arow_w + a * 16 + 4 * lh + r;
        if (rw < M) {
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const int n = b * 16 + li;
            float v = acc[a][b][r] + bias[n];
            out[rw * ldo + n] = v > 0.f ? v : 0.f;
          }
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b][r] = 0.f;
      }
    }
    if (!has_next) break;
    tile = next;
    ++i;
  }
}

}  // namespace

hipError_t sage_fwd_f32(const float* X, int64_t ldx, int F, const int64_t* rowptr,
                        const int32_t* col, const float* inv_deg, const float* Ws,
                        const float* Wn, const float* bias, float* out, int64_t ldo, int64_t M,
                        float* ring, int64_t ring_floats, int* err, hipStream_t st) {
  if (M <= 0) return hipSuccess;
  if ((F != 128 && F != 256) || ldx % 4 || ldo % 4) return hipErrorInvalidValue;
  static int num_cus = 0;
  if (num_cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) !=
            hipSuccess || num_cus <= 0)
      num_cus = 256;
  }
  const int64_t ntiles = (M + kSM - 1) / kSM;
  const int64_t blocks = ntiles < num_cus ? ntiles : num_cus;
  if (ring_floats < blocks * 2 * kSM * F) return hipErrorInvalidValue;
  constexpr size_t lds = 2 * kSStage * sizeof(float) + 64;
  static bool attr[2] = {false, false};
  const int fi = F == 256 ? 1 : 0;
  auto kern = F == 256 ? &sage_fwd_f32_kernel<256> : &sage_fwd_f32_kernel<128>;
  if (!attr[fi]) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    attr[fi] = true;
  }
  hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(blocks)), dim3(512), lds, st, X, ldx,
                     rowptr, col, inv_deg, Ws, Wn, bias, out, ldo, M, ring, err);
  return hipGetLastError();
}

}  // namespace dgraph
